#!/bin/bash
# Round 3 iteration: the GPU tests touched this round + the wavefront (sequence) parity tests, then
# the default bench line.  Stops on any GPU fault.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 1000 $T tests/test_gpu_fullsize.py tests/test_gpu_unet.py::test_unet_cfg5_shapes_vs_oracle \
  "tests/test_gpu_parity.py::test_replaced_parameters_after_forward" "tests/test_gpu_parity.py::test_convlayer_wide_unet_preds_vs_torch" \
  "tests/test_gpu_parity.py::test_engine_gradients_wide_vs_oracle" "tests/test_gpu_parity.py::test_subtract_reset_cell_vs_oracle" \
  "tests/test_gpu_parity.py::test_forward_sequence_matches_per_step" "tests/test_gpu_parity.py::test_forward_sequence_matches_per_step_full_size" \
  "tests/test_gpu_parity.py::test_forward_sequence_input_and_state_grads" "tests/test_gpu_parity.py::test_forward_sequence_chained_without_detach" \
  "tests/test_gpu_parity.py::test_forward_sequence_vs_golden" "tests/test_gpu_parity.py::test_training_steps_fused_adam_vs_oracle" \
  -s > gpurun_out/t_b.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/t_b.log | tail -60
if [ $rc -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { echo "bench failed"; tail -30 gpurun_out/bench_b.err; exit 4; }
cat gpurun_out/bench_b.json
exit $rc
