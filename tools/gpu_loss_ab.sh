#!/bin/bash
# Loss-kernel check and A/B: the loss parity tests, then rocprofv3 kernel stats of the bench
# workload (tools/prof_step.py) for the default library and the splat-split variants
# (make -C csrc variant_loss V=split2 D=-DSNNFLOW_SPLAT_SPLIT=2), then FETCH/WRITE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/loss
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "warping or iwe or cfg2_train_step or forward_sequence_matches" tests/ > gpurun_out/loss/tests.txt 2>&1 || { tail -30 gpurun_out/loss/tests.txt; exit 3; }
tail -3 gpurun_out/loss/tests.txt
export TMPDIR=/tmp
for v in ${VARIANTS:-""}; do
  unset SNNFLOW_LIB; [ -n "$v" ] && export SNNFLOW_LIB=$GRAFT_REPO_ROOT/snn_event-based_optical_flow_amd/snnflow/libsnnflow_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/loss/ks_${v:-base} -o run --output-format csv -- python3 tools/prof_step.py > gpurun_out/loss/ks_${v:-base}.log 2>&1 || exit 3
  f=$(find gpurun_out/loss/ks_${v:-base} -name "*kernel_stats.csv" | head -1)
  echo "== ${v:-base}"; grep -i iwe $f | cut -d, -f1-4
done
unset SNNFLOW_LIB
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/loss/pmc_$ctr -o run --output-format csv -- python3 tools/prof_step.py > gpurun_out/loss/pmc_$ctr.log 2>&1 || exit 3
done
echo done
