#!/bin/bash
# Like tools/gpu_variants.sh for a given channel count: bash tools/gpu_variants_c.sh C name1 ...
set -o pipefail
mkdir -p gpurun_out
C=$1; shift
for v in base "$@"; do
  if [ $v = base ]; then unset SNNFLOW_LIB; else export SNNFLOW_LIB=$PWD/snn_event-based_optical_flow_amd/snnflow/libsnnflow_$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --channels $C > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "$v failed"; tail -5 gpurun_out/var_$v.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('$v', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:7]})"
done
