#!/bin/bash
# Round-4: bench A/B over library variants: LIBS="libsnnflow libsnnflow_x" BENCH_ARGS="..."
set -u -o pipefail
mkdir -p gpurun_out/libab
for rep in 1 2; do
  for l in ${LIBS}; do
    SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$l.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/libab/${l}_$rep.json 2> gpurun_out/libab/${l}_$rep.err || { tail -20 gpurun_out/libab/${l}_$rep.err; exit 4; }
    python -c "import json;d=json.load(open('gpurun_out/libab/${l}_$rep.json'));print('$l', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],4), 'ms', {k:v['avg_us'] for k,v in list(d.get('kernels',{}).items())[:4]})"
  done
done
