#!/bin/bash
# C = 32 weight gradients at two blocks per CU: parity at C = 32, bench A/B against k_wgrad_bf<32>;
# host phases of the eager loop; the U-Net line with its CPU baseline.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 400 --timeout-method thread -s"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "wide or C32" > gpurun_out/t_c32.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|grad rel-L2 worst" gpurun_out/t_c32.log | cut -c1-250 | tail -20
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for v in libsnnflow libsnnflow_wg32old; do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$v.so timeout -k 10 300 python bench.py --channels 32 --no-cpu-baseline > gpurun_out/c32_$v.json 2> gpurun_out/c32_$v.err || { tail -20 gpurun_out/c32_$v.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/c32_$v.json'));print('$v', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'wgrad' in k})"
done
timeout -k 10 200 python tools/host_phases.py 30 > gpurun_out/host_phases.txt 2>&1 || { tail -20 gpurun_out/host_phases.txt; exit 3; }
cat gpurun_out/host_phases.txt
timeout -k 10 500 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 > gpurun_out/unet_cpu.json 2> gpurun_out/unet_cpu.err || { tail -20 gpurun_out/unet_cpu.err; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/unet_cpu.json'));print('unet', d['ms_per_step'], d['cpu_baseline'])"
exit $rc
