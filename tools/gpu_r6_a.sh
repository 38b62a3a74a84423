#!/bin/bash
# Round 6: selected GPU tests (-k $1) then the cfg2 and C = 32 bench lines.
set -u
O=gpurun_out/r6a
mkdir -p $O
K=${1:-bit_planes or skips_bit_identical}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|^\[" $O/tests.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
[ "${NOBENCH:-0}" = 1 ] && exit 0
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.err || { tail -20 $O/cfg2.err; exit 4; }
python -c "import json;d=json.load(open('$O/cfg2.json'));print('cfg2', d['ms_per_step'], d['roofline']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --no-cpu-baseline --channels 32 > $O/c32.json 2> $O/c32.err || { tail -20 $O/c32.err; exit 5; }
python -c "import json;d=json.load(open('$O/c32.json'));print('c32', d['ms_per_step'], d['roofline']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
