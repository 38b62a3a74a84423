#!/bin/bash
# Round-4: rocprofv3 kernel stats of the --eval bench line
set -u -o pipefail
mkdir -p gpurun_out/r4e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4e/prof -o run --output-format csv -- python3 $R/bench.py --eval --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r4e/bench.json 2> $R/gpurun_out/r4e/bench.err || { tail -5 $R/gpurun_out/r4e/bench.err; exit 3; }
python3 $R/tools/kstats.py $R/gpurun_out/r4e/prof/run_kernel_stats.csv 20
