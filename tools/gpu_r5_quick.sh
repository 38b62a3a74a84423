#!/bin/bash
# Quick check after a kernel change: the GPU tests matching $1 (pytest -k; all if empty), the default
# bench line, a rocprofv3 kernel trace of a short bench run (step breakdown + per-task-kind slot times).
set -u
O=gpurun_out/quick${QTAG:-}
mkdir -p $O
K=${1:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_us']); print({k:v['avg_us'] for k,v in d['kernels'].items()})"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -18 $R/$O/step_breakdown.txt
python3 $R/tools/slot_attrib.py $R/$O/prof/run_kernel_trace.csv bwd | python3 -c "import json,sys;d=json.load(sys.stdin);print('bwd', d['quantities']['duration_us']['per_task'], d['quantities']['duration_us']['pass_total'])"
python3 $R/tools/slot_attrib.py $R/$O/prof/run_kernel_trace.csv fwd | python3 -c "import json,sys;d=json.load(sys.stdin);print('fwd', d['quantities']['duration_us']['per_task'], d['quantities']['duration_us']['pass_total'])"
