#!/bin/bash
# two-team k_wgrad_b32: C = 32 parity (oracle + bits on/off bit identity), then the C = 32 line with the diag split.
set -u
O=gpurun_out/r6c7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "C32" > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 3; }
grep -E "passed|failed" $O/tests.log | tail -2
for D in ${DIAGS:-0 1 2 3}; do
  SNNFLOW_WG_DIAG=$D timeout -k 10 300 python bench.py --no-cpu-baseline --channels 32 --steps 10 --warmup 3 > $O/d$D.json 2> $O/d$D.err || { tail -20 $O/d$D.err; exit 5; }
  python -c "import json;d=json.load(open('$O/d$D.json'));print('diag $D', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'wgrad' in k or 'slot' in k})"
done
