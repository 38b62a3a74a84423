#!/bin/bash
# Matrix-core utilisation passes: one rocprofv3 --pmc run per (workload, pass),
# counters only (no trace domains).  Workloads: cfg2 C=8 wavefront, C=32 128^2 per-step, U-Net cfg5.
# The counter names are checked against rocprofv3's list for this agent first; missing ones are dropped.
set -u
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_mfma
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "list failed"; tail -5 $OUT/avail.txt; exit 1; }
pick() {
  local r=""
  for c in "$@"; do grep -qw "$c" $OUT/avail.txt && r="$r $c"; done
  echo $r
}
P1=$(pick SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_WAVE_CYCLES SQ_WAVES)
P2=$(pick GRBM_GUI_ACTIVE GRBM_COUNT)
echo "pass1: $P1" | tee $OUT/passes.txt
echo "pass2: $P2" | tee -a $OUT/passes.txt
run() {  # name, args...
  local name=$1; shift
  local i=0
  for ctrs in "$P1" "$P2"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $ctrs -d $OUT/$name/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py "$@" > $OUT/$name.p$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 $OUT/$name.p$i.log; exit 1; }
  done
}
for w in ${WL:-c8 c32 unet}; do
  case $w in
    c8) run c8 8 128 8 10 2 || exit 1 ;;
    c32) run c32 32 128 8 10 2 || exit 1 ;;
    unet) run unet unet 256 16 20 32 1 || exit 1 ;;
  esac
done
python3 $GRAFT_REPO_ROOT/tools/pmc_mfma.py $OUT
