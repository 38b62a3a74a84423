#!/bin/bash
# Loss kernel times (rocprofv3 --stats of a short bench run) per library build: LIBS="name:path ..."
# (the default build is "base").  Only builds whose every kernel writes what its readers read.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lossprobe
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for spec in base:default ${LIBS:-}; do
  n=${spec%%:*}; path=${spec#*:}
  if [ "$path" = default ]; then unset SNNFLOW_LIB; else export SNNFLOW_LIB=$R/$path; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -10 $O/$n.err; exit 4; }
  echo "== $n"; python3 $R/tools/kstats.py $O/$n/run_kernel_stats.csv 14 | grep iwe
done
