#!/bin/bash
# Environment A/B on one box: tools/gpu_envab.sh "<bench args>" "VAR=a" "VAR=b" [reps]
# alternates the bench line under each environment setting; prints ms_per_step and the kernel averages.
set -u
ARGS=$1; A=$2; B=$3; N=${4:-2}
O=gpurun_out/envab
mkdir -p $O
for i in $(seq $N); do
  for E in "$A" "$B"; do
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > $O/run.json 2> $O/run.err || { tail -20 $O/run.err; exit 4; }
    python -c "import json;d=json.load(open('$O/run.json'));print('$E', d['ms_per_step'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:6]})"
  done
done
