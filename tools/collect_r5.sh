#!/bin/bash
# Copy the judged outputs of tools/gpu_r5_final.sh (+ tools/gpu_r5_lines.sh) from gpurun_out/ into profiles/r05/final/.
set -eu
D=profiles/r05/final
mkdir -p $D
for f in gpu_tests.log smoke.log bench.json step_breakdown.txt attrib_time_bwd.json attrib_time_fwd.json attrib_sq_bwd.json attrib_sq_fwd.json; do
  cp gpurun_out/r5_final/$f $D/
done
cp gpurun_out/r5_final/prof/run_kernel_stats.csv $D/kernel_stats.csv
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
cp gpurun_out/pmc_counters.json $D/pmc_counters.json
cp gpurun_out/pmc_summary.txt $D/pmc.txt
cp gpurun_out/pmc_mfma/pmc_mfma.json $D/pmc_mfma.json
for l in gpurun_out/lines/line_*.json; do cp $l $D/; done
for p in gpurun_out/lines/prof_*/run_kernel_stats.csv; do n=$(basename $(dirname $p)); cp $p $D/kernel_stats_${n#prof_}.csv; done
ls $D
