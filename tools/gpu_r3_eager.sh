#!/bin/bash
# Eager per-window loop: host-cost attribution, and a kernel trace (GPU busy vs span per step).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/eager_micro.py > gpurun_out/eager_micro.txt 2>&1 || { tail -20 gpurun_out/eager_micro.txt; exit 3; }
cat gpurun_out/eager_micro.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_eager -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --per-step --no-graph --steps 5 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_eager.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_eager.err || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_eager.err; exit 5; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_eager -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_step.py $f -2 | head -30
