#!/bin/bash
# Round 3: the new / changed GPU tests, then a plain `bench.py --gpus 2` (ranks sharing the GPU over
# gloo) and the default bench line.  Stops on any GPU fault.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 600 --timeout-method thread"
timeout -k 10 900 $T --deselect "tests/test_gpu_fullsize.py::test_cfg2_train_step_vs_oracle[cfg2-sequence]" --deselect "tests/test_gpu_fullsize.py::test_cfg2_train_step_vs_oracle[cfg2-per_step]" tests/test_gpu_fullsize.py tests/test_gpu_unet.py::test_unet_cfg5_shapes_vs_oracle \
  "tests/test_gpu_parity.py::test_replaced_parameters_after_forward" "tests/test_gpu_parity.py::test_convlayer_wide_unet_preds_vs_torch" \
  "tests/test_gpu_parity.py::test_engine_gradients_wide_vs_oracle" "tests/test_gpu_parity.py::test_subtract_reset_cell_vs_oracle" \
  -s > gpurun_out/t_new.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|flips|grad rel|AEE|flow rel|loss ours|dp-check|cfg5" gpurun_out/t_new.log | tail -80
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; fi
if [ $rc -gt 1 ]; then exit $rc; fi
exit $rc
SNNFLOW_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_gpus2.json 2> gpurun_out/bench_gpus2.err || { echo "gpus2 bench failed"; tail -30 gpurun_out/bench_gpus2.err; exit 4; }
cat gpurun_out/bench_gpus2.json
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
exit $rc
