#!/bin/bash
# Selected GPU tests with their printed measurements: tools/gpu_tests_sel.sh <log name> <pytest args...>
set -u
mkdir -p gpurun_out
log=gpurun_out/$1; shift
timeout -k 10 1000 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > $log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|Error" $log | tail -40
exit $rc
