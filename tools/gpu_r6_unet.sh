#!/bin/bash
# U-Net: parity tests, then the cfg5 bench line (3 steps) under each $AB setting.
set -u
O=gpurun_out/r6unet
mkdir -p $O
if [ "${NOTEST:-0}" != 1 ]; then
timeout -k 10 700 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  ${K:+-k "$K"} > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/tests.log | tail -5
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
fi
for E in ${AB:-X=0}; do
  env $E timeout -k 10 400 python bench.py --no-cpu-baseline --model SpikingRecEVFlowNet --steps 3 --warmup 2 > $O/unet.json 2> $O/unet.err || { tail -20 $O/unet.err; exit 5; }
  python -c "import json;d=json.load(open('$O/unet.json'));print('$E unet', d['ms_per_step'], {k:(v['avg_us'],v.get('issued_frac')) for k,v in list(d['kernels'].items())[:8]})"
done
