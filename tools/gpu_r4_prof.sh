#!/bin/bash
# Round-4: rocprofv3 kernel trace + stats of the default bench line, one step's breakdown
set -u -o pipefail
mkdir -p gpurun_out/r4
O=gpurun_out/r4
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -30 $R/$O/step_breakdown.txt
