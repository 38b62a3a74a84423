#!/bin/bash
# A/B of variant builds of the library (SNNFLOW_LIB), C = 32 line by default: $VARS = library suffixes ("" = default).
set -u
O=gpurun_out/r6libab
mkdir -p $O
L=$GRAFT_REPO_ROOT/snn_event-based_optical_flow_amd/snnflow
for rep in 1 2; do
for v in ${VARS:-_ _u2 _u4}; do
  lib=$L/libsnnflow${v#_}.so; [ "$v" != "_" ] && lib=$L/libsnnflow$v.so; [ "$v" = "_" ] && lib=$L/libsnnflow.so
  SNNFLOW_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline ${ARGS:---channels 32} --steps 20 > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 5; }
  python -c "import json;d=json.load(open('$O/l.json'));print('$v', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'wgrad' in k or 'slot' in k})"
done
done
