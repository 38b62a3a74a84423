#!/bin/bash
# Round-6 validation: every GPU test with -s (flip counts, |dAEE|, worst gradients printed), smoke,
# the default bench line, and the C = 32 / U-Net lines.  LINES selects the extra lines.
set -u
O=gpurun_out/r6full${TAG:-}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread ${K:+-k "$K"} > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_us'], (d.get('cpu_baseline') or {}).get('value')); print({k:v['avg_us'] for k,v in d['kernels'].items()})"
for l in ${LINES:-c32 unet}; do
  case $l in
    c32) a="--channels 32" ;;
    unet) a="--model SpikingRecEVFlowNet --steps 3 --warmup 2" ;;
    cfg3) a="--res 256 --batch 4" ;;
    perstep) a="--per-step" ;;
    eager) a="--per-step --no-graph" ;;
    eval) a="--eval" ;;
  esac
  timeout -k 10 400 python bench.py --no-cpu-baseline $a > $O/line_$l.json 2> $O/line_$l.err || { echo "$l failed"; tail -10 $O/line_$l.err; exit 5; }
  python -c "import json;d=json.load(open('$O/line_$l.json'));print('$l', d['ms_per_step'], d['value'], (d.get('roofline') or {}).get('frac'), {k:v['avg_us'] for k,v in list(d.get('kernels',{}).items())[:10]})"
done
