#!/bin/bash
# rocprofv3 kernel trace of a short bench run; prints mean duration per kernel name.
#   bash tools/prof_kernels.sh <tag> [bench args]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_$tag.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_$tag.err || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_$tag.err; exit 5; }
python3 - $GRAFT_REPO_ROOT/gpurun_out/prof_$tag/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    print(f'{float(r["AverageNs"])/1000:9.2f} us x{r["Calls"]:>5}  {n[:90]}')
PY
