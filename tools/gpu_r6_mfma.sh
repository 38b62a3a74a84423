#!/bin/bash
# Round-6 matrix-core passes (C = 8, C = 32, U-Net cfg5; tools/pmc_mfma.sh) -> gpurun_out/pmc_mfma*.
set -u
WL="${WL:-c8 c32 unet}" bash tools/pmc_mfma.sh > gpurun_out/pmc_mfma_summary.txt 2>&1 || { echo "pmc_mfma failed"; tail -8 gpurun_out/pmc_mfma_summary.txt; exit 8; }
tail -30 gpurun_out/pmc_mfma_summary.txt
ls gpurun_out/pmc_mfma | head
