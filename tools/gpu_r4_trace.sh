#!/bin/bash
# Round-4: phase stamps of the 4-task slot launches (fwd pipeline, legacy bwd) + rocprofv3 kernel stats
# of the default bench line.
set -u -o pipefail
mkdir -p gpurun_out/r4
O=gpurun_out/r4
SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace_slot.so timeout -k 10 200 python tools/ktrace_slot.py > $O/ktrace_slot.json 2> $O/ktrace_slot.err || { tail -20 $O/ktrace_slot.err; exit 3; }
cat $O/ktrace_slot.json | head -80
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -30 $R/$O/step_breakdown.txt
