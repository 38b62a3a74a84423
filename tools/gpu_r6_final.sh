#!/bin/bash
# Round-6 final evidence, part 1: every GPU test with -s (flip counts, |dAEE|, worst gradients printed),
# smoke, the default bench line (cpu_baseline included), a rocprofv3 kernel trace + stats of the bench.
set -u
O=gpurun_out/r6final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_us'], (d.get('cpu_baseline') or {}).get('value')); print({k:v['avg_us'] for k,v in d['kernels'].items()})"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/kstats.py $R/$O/prof/run_kernel_stats.csv 14
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -16 $R/$O/step_breakdown.txt
