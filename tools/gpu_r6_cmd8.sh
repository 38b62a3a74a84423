#!/bin/bash
# C = 32 head weight gradient k_wgrad<2, 32, false, SPLIT>: SPLIT 2 (default) vs 1; C = 32 oracle tests.
set -u
O=gpurun_out/r6c8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "C32" > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 3; }
grep -E "passed|failed" $O/tests.log | tail -2
for E in SNNFLOW_WG_HEAD_SP2=1 SNNFLOW_WG_HEAD_SP2=0 SNNFLOW_WG_HEAD_SP2=1 SNNFLOW_WG_HEAD_SP2=0; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --channels 32 --steps 20 --warmup 3 > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 5; }
  python -c "import json;d=json.load(open('$O/l.json'));print('$E', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'wgrad' in k})"
done
