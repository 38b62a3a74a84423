#!/bin/bash
# A/B of environment settings on the default bench line (alternating runs).
#   ENVS="name:VAR=val[,VAR2=val] ..." (a "base" run with nothing set comes first in every round)
set -u
O=gpurun_out/envab${ABTAG:-}
mkdir -p $O
run() {  # name, env assignments (comma separated)
  local n=$1 e=$2
  env $(echo $e | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -20 $O/bench_$n.err; return 4; }
  python -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n', d['ms_per_step'], d['value'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:6]})"
}
for rep in 1 2; do
  run base_$rep "SNNFLOW_NONE=1" || exit 4
  for spec in ${ENVS:-}; do run ${spec%%:*}_$rep ${spec#*:} || exit 4; done
done
