#!/bin/bash
# cfg2 bench under the forward tile-pipeline knobs (SNNFLOW_PIPE_FWD tiles per block, SNNFLOW_PIPE_ORDER), alternated.
set -u
O=gpurun_out/r6knobs
mkdir -p $O
for rep in 1 2; do
for E in "SNNFLOW_PIPE_FWD=2" "SNNFLOW_PIPE_FWD=3" "SNNFLOW_PIPE_FWD=4" "SNNFLOW_PIPE_ORDER=0" "SNNFLOW_PIPE_ORDER=2"; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 5; }
  python -c "import json;d=json.load(open('$O/l.json'));print('$E', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'slot' in k})"
done
done
