#!/bin/bash
# Round-5 validation + profiles: tools/gpu_r5.sh (GPU tests, smoke, bench, kernel trace, SQ pass attributed
# per slot-task kind), the traffic / SQ counter passes (tools/pmc.sh), the matrix-core passes at C = 8
# and C = 32 (tools/pmc_mfma.sh), and the other bench lines (tools/gpu_r5_lines.sh).
set -u
R5TAG=_final bash tools/gpu_r5.sh || exit $?
PMC_KEY=C8_R128_B8 bash tools/pmc.sh > gpurun_out/pmc_summary.txt 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_summary.txt; exit 7; }
tail -25 gpurun_out/pmc_summary.txt
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
WL="c8 c32" bash tools/pmc_mfma.sh > gpurun_out/pmc_mfma_summary.txt 2>&1 || { echo "pmc_mfma failed"; tail -5 gpurun_out/pmc_mfma_summary.txt; exit 8; }
LINES="${LINES:-cfg3 perstep eager}" bash tools/gpu_r5_lines.sh || exit 9
