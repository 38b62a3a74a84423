#!/bin/bash
# A/B of two library builds on the default bench (no CPU baseline): alternating runs.
#   LIB_B=<path to .so> bash tools/gpu_ab.sh [bench args]
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export SNNFLOW_LIB=$LIB_B; else unset SNNFLOW_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { tail -20 gpurun_out/ab_$v$i.err; exit 4; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$i.json'));print('$v', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:8]})"
  done
done
