#!/bin/bash
# fused head weight gradient (ABI 40): the whole GPU suite, then cfg2 / C = 32 lines with SNNFLOW_FUSE_HEAD 1 / 0.
set -u
O=gpurun_out/r6c9
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread ${K:+-k "$K"} > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -40; exit $rc; fi
for a in "" "--channels 32"; do
for E in SNNFLOW_FUSE_HEAD=1 SNNFLOW_FUSE_HEAD=0 SNNFLOW_FUSE_HEAD=1 SNNFLOW_FUSE_HEAD=0; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline $a --steps 30 > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 5; }
  python -c "import json;d=json.load(open('$O/l.json'));print('$a $E', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'slot' in k or 'wgrad' in k or 'slab' in k})"
done
done
