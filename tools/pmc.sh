#!/bin/bash
# rocprofv3 counter passes (each pass its own run; no tracing domains combined with --pmc).
set -u
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py ${PMC_ARGS:-} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
ls -R $OUT | head -30
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py $OUT ${PMC_KEY:-C8_R128_B8} $GRAFT_REPO_ROOT/gpurun_out/pmc_counters.json
