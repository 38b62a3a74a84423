#!/bin/bash
# U-Net parity + per-shape line for the 3-part fragment read-ahead in k_unet_conv_dma, then counter
# passes over the C = 32 LIFFireNet step (k_wgrad_b32, the slots).
set -u
R=$GRAFT_REPO_ROOT
O=gpurun_out/r6c5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > $O/unet_tests.log 2>&1 || { tail -30 $O/unet_tests.log; exit 3; }
tail -2 $O/unet_tests.log
PAT='conv|dgrad|wgrad' TAG=5 timeout -k 10 500 bash tools/gpu_r6_unet_ab.sh || exit 4
cd /tmp && export TMPDIR=/tmp
P=$R/$O/pmc32
mkdir -p $P
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $ctrs -d $P/p$i -o run --output-format csv -- python3 $R/tools/prof_step.py 32 128 8 10 2 > $P/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $P/p$i.log; exit 1; }
done
python3 $R/tools/pmc_sum.py $P 'wgrad|slot|slab' | tee $R/$O/pmc32_summary.txt
