#!/bin/bash
# Round 3 full check: every GPU test, smoke, the default bench line, the persistent-forward window
# timing, and a rocprofv3 kernel trace of the bench.  Stops on any GPU fault.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread -s > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc -> stop"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
timeout -k 10 200 python tools/seq_time.py > gpurun_out/seq_time.txt 2>&1 || { echo "seq_time failed"; tail -20 gpurun_out/seq_time.txt; exit 6; }
cat gpurun_out/seq_time.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.err; exit 5; }
cat $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json
exit $rc
