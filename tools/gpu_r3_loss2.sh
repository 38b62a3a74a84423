#!/bin/bash
# Deterministic splat: loss tests + cfg5-shape U-Net test, then bench A/B (fixed-point vs fp32 splat).
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 400 --timeout-method thread -s"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_unet.py -k "warping or reproducible or cfg5 or fused_adam or liffirenet_c8" > gpurun_out/t_loss2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|cfg5 shapes\]" gpurun_out/t_loss2.log | cut -c1-300 | tail -40
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
for v in libsnnflow libsnnflow_splatf libsnnflow; do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { tail -30 gpurun_out/bench_$v.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'iwe' in k})"
done
exit $rc
