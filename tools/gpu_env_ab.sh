#!/bin/bash
# A/B of an environment setting on the default bench (no CPU baseline), alternating runs.
#   ENV_B="NAME=value" bash tools/gpu_env_ab.sh [bench args]
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then envset="$ENV_B"; else envset=""; fi
    env $envset timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/eab_$v$i.json 2> gpurun_out/eab_$v$i.err || { tail -20 gpurun_out/eab_$v$i.err; exit 4; }
    python -c "import json;d=json.load(open('gpurun_out/eab_$v$i.json'));print('$v', d['value'], d['ms_per_step'])"
  done
done
