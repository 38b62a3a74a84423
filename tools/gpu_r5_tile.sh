#!/bin/bash
# The one-tile backward body (SNNFLOW_BWD_TILE=1): its unit parity tests, the whole GPU suite with it
# on, an A/B of the bench line, and a kernel trace with per-task attribution.
set -u
O=gpurun_out/tile${QTAG:-}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pipe_tests.log 2>&1
rc=$?; grep -E "^\[bwd|passed|failed" $O/pipe_tests.log | tail -14
[ $rc -ne 0 ] && { grep -E "^E " $O/pipe_tests.log | head -20; exit $rc; }
SNNFLOW_BWD_TILE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests_tile.log 2>&1
rc=$?; tail -2 $O/gpu_tests_tile.log
[ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/gpu_tests_tile.log | head -20; exit $rc; }
ABTAG=_tile ENVS="tile:SNNFLOW_BWD_TILE=1" bash tools/gpu_envab.sh || exit 4
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SNNFLOW_BWD_TILE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -8 $R/$O/step_breakdown.txt
python3 $R/tools/slot_attrib.py $R/$O/prof/run_kernel_trace.csv bwd | python3 -c "import json,sys;d=json.load(sys.stdin);print('bwd', d['quantities']['duration_us']['per_task'], d['quantities']['duration_us']['pass_total'])"
cd $R
if [ -f snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace_slot.so ]; then
  SNNFLOW_BWD_TILE=1 SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace_slot.so timeout -k 10 300 python tools/ktrace_slot.py > $O/ktrace.json 2> $O/ktrace.err || { echo "ktrace failed"; tail -5 $O/ktrace.err; exit 6; }
  python3 -c "
import json;d=json.load(open('$O/ktrace.json'))
for dr,v in d['kinds'].items():
  print(dr, v['launch_span_us'], v['resident_blocks_per_us'])
  for k,x in v.items():
    if isinstance(x,dict): print(' ',k,x['blocks'],x['start_us_p10_50_90_100'],x['end_us_p10_50_90_100'],x['block_us_med_p90'],x['phases_med_p90_us'])
"
fi
