#!/bin/bash
# Persistent forward: its parity tests, the full-size sequence tests, then the bench.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -x tests/test_gpu_parity.py::test_persistent_forward_matches_slots > gpurun_out/t_d.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Error|assert" gpurun_out/t_d.log | head -30
if [ $rc -ne 0 ]; then tail -30 gpurun_out/t_d.log; exit $rc; fi
SNNFLOW_SEQ=1 timeout -k 10 600 $T "tests/test_gpu_parity.py::test_forward_sequence_matches_per_step_full_size" "tests/test_gpu_fullsize.py::test_cfg2_train_step_vs_oracle" tests/test_gpu_unet.py::test_unet_cfg5_shapes_vs_oracle -s > gpurun_out/t_d2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|cfg5 shapes\]" gpurun_out/t_d2.log | cut -c1-600 | head -30
if [ $rc -gt 1 ]; then exit $rc; fi
SNNFLOW_SEQ=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err || { tail -30 gpurun_out/bench_d.err; exit 4; }
cat gpurun_out/bench_d.json
SNNFLOW_SEQ=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_d0.json 2> gpurun_out/bench_d0.err || { tail -30 gpurun_out/bench_d0.err; exit 4; }
cat gpurun_out/bench_d0.json
exit $rc
