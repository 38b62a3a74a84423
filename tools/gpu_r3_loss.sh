#!/bin/bash
# Loss-touching GPU tests (+ the cell variants), then the default bench and a kernel trace.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 400 --timeout-method thread -s"
timeout -k 10 900 $T tests/test_gpu_fullsize.py "tests/test_gpu_parity.py" tests/test_gpu_unet.py -k "warping or golden or fused_adam or wide_vs_oracle or unet or reproducible or variants or cfg2_train" > gpurun_out/t_loss.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_loss.log | cut -c1-160 | tail -70
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || { tail -30 gpurun_out/bench_l.err; exit 4; }
cat gpurun_out/bench_l.json
exit $rc
