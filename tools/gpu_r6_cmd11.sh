#!/bin/bash
set -u
O=gpurun_out/r6c11
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-fused_head}" > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 3; }
grep -E "fuse_head|passed|failed" $O/tests.log | tail -8
