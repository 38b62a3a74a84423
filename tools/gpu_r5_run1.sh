#!/bin/bash
# round-5 first GPU call: validation (tools/gpu_r5.sh), then the LDS-swizzle A/B.
bash tools/gpu_r5.sh && LIBS="noswz:snn_event-based_optical_flow_amd/snnflow/libsnnflow_noswz.so" bash tools/gpu_r5_ab.sh
