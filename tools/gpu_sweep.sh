#!/bin/bash
# Bench sweep over the BASELINE.json configurations that fit one GPU (no CPU baseline) plus
# the rocprofv3 PMC traffic passes of the default workload.  Stops at the first failure.
set -u
mkdir -p gpurun_out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/sweep_$n.json 2> gpurun_out/sweep_$n.err \
    || { echo "bench $n failed"; tail -20 gpurun_out/sweep_$n.err; exit 4; }
  cut -c1-400 gpurun_out/sweep_$n.json
}
run c8_r128_b8
run c32_r128_b8 --channels 32
run c8_r256_b4 --res 256 --batch 4
run c32_r256_b4 --res 256 --batch 4 --channels 32
[ "${SKIP_PMC:-0}" = "1" ] && exit 0
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc.log; exit 5; }
tail -30 gpurun_out/pmc.log
