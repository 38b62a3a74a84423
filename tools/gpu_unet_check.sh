#!/bin/bash
# U-Net parity tests then the cfg5 bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_unet.py > gpurun_out/u_tests.log 2>&1
rc=$?
grep -E "^\[|PASSED|FAILED|Error" gpurun_out/u_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/ub_cfg5.json 2> gpurun_out/ub_cfg5.err || { tail -30 gpurun_out/ub_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ub_cfg5.json'));print(d['ms_per_step'],d['value'],d['roofline'],d['cpu_baseline']);print(json.dumps(d['kernels']))"
