#!/bin/bash
# Quick: selected GPU tests (-k $K), then cfg2 x2, C = 32 and the per-window (eager) loop lines.
set -u
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${K:-skips_bit_identical or test_cfg2_train_step_vs_oracle and cfg2-sequence or pingpong or forward_sequence_matches or per_step or chain or defer}" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|^FAILED" $O/tests.log | tail -4
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
for a in "" "" "--channels 32" "--per-step" "--per-step --no-graph"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 5; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$a', d['ms_per_step'], {k:v['avg_us'] for k,v in list(d.get('kernels',{}).items())[:8]})"
done
