#!/bin/bash
# Default bench under several library builds (make -C csrc variant V=<name> ...): prints the
# per-kernel times of each.   bash tools/gpu_variants.sh name1 name2 ...   (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
for v in base "$@"; do
  if [ $v = base ]; then unset SNNFLOW_LIB; else export SNNFLOW_LIB=$PWD/snn_event-based_optical_flow_amd/snnflow/libsnnflow_$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "$v failed"; tail -5 gpurun_out/var_$v.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('$v', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:6]})"
done
