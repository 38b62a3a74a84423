#!/bin/bash
# U-Net elementwise kernels per dispatch: a kernel trace (grid sizes, durations) and separate
# FETCH_SIZE / WRITE_SIZE passes over a short cfg5-shape train step (256^2, B=16, 2 windows).
set -u
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/unet_ew
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py unet 256 16 2 32 1 > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -5 $OUT/kt.log; exit 1; }
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py unet 256 16 2 32 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
