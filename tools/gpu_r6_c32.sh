#!/bin/bash
# C = 32 checks: parity tests at C = 32 / 16, then an env A/B of the C = 32 bench line.
set -u
O=gpurun_out/r6c32
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${K:-bit_planes or cfg2-C32 or wide or clip_adam}" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED|grad rel-L2 worst|bit planes" $O/tests.log | tail -12
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
for i in 1 2; do
  for E in ${AB:-X=0}; do
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --channels 32 > $O/c32.json 2> $O/c32.err || { tail -20 $O/c32.err; exit 5; }
    python -c "import json;d=json.load(open('$O/c32.json'));print('$E c32', d['ms_per_step'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:9]})"
  done
done
