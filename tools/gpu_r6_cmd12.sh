#!/bin/bash
set -u
O=gpurun_out/r6c12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-slab_reduce or fused_head or cfg2_train_step or pingpong}" > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 3; }
grep -E "passed|failed" $O/tests.log | tail -2
for a in "" "--channels 32" "" "--channels 32"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a --steps 30 > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 5; }
  python -c "import json;d=json.load(open('$O/l.json'));print('$a', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'slab' in k or 'adam' in k})"
done
