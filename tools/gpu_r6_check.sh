#!/bin/bash
# closing check of the committed tree: every GPU test, smoke, the default bench line
set -u
O=gpurun_out/r6check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
