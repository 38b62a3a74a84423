#!/bin/bash
# Round 4: dynamic tile hand-out of the forward tile pipeline -- tests, then bench A/B
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pipe or forward_sequence or fullsize" > gpurun_out/t_dyn.log 2>&1 || { tail -30 gpurun_out/t_dyn.log; exit 3; }
tail -2 gpurun_out/t_dyn.log
for rep in 1 2; do
for v in "2 1 150" "2 0 150" "2 1 100" "2 1 200" "3 1 150" "1 1 150"; do set -- $v
  SNNFLOW_PIPE_FWD=$1 SNNFLOW_PIPE_DYN=$2 SNNFLOW_PIPE_RECW=$3 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/d_$1_$2_$3.json 2>/dev/null || exit 4
  python -c "import json;d=json.load(open('gpurun_out/d_$1_$2_$3.json'));print('tpb $1 dyn $2 recw $3', round(d['ms_per_step'],4), 'ms', {k:v['avg_us'] for k,v in list(d.get('kernels',{}).items())[:2]})"
done; done
