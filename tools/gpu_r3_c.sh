#!/bin/bash
# U-Net cfg5-shape test (fp64 oracle) + backward/forward slot phase trace.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 500 --timeout-method thread -s \
  tests/test_gpu_unet.py::test_unet_cfg5_shapes_vs_oracle > gpurun_out/t_c.log 2>&1
rc=$?
grep -E "PASSED|FAILED|cfg5 shapes|Error" gpurun_out/t_c.log | cut -c1-1500
if [ $rc -gt 1 ]; then exit $rc; fi
SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace_slot.so timeout -k 10 200 python tools/ktrace_slot.py > gpurun_out/ktrace_r3_fused.json 2> gpurun_out/ktrace.err || { tail -20 gpurun_out/ktrace.err; exit 5; }
cat gpurun_out/ktrace_r3_fused.json
exit $rc
