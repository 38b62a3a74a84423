#!/bin/bash
# k_wgrad_b32 time split (ran against a diagnostic build, not kept, that compiled k_wgrad_b32<DIAG> variants selected by SNNFLOW_WG_DIAG):
# DIAG 0 normal, 1 no MFMA phase, 2 no G loads, 3 neither (C = 32 line, per-layer wgrad times).
set -u
O=gpurun_out/r6c6
mkdir -p $O
for D in 0 1 2 3; do
  SNNFLOW_WG_DIAG=$D timeout -k 10 300 python bench.py --no-cpu-baseline --channels 32 --steps 10 --warmup 3 > $O/d$D.json 2> $O/d$D.err || { tail -20 $O/d$D.err; exit 5; }
  python -c "import json;d=json.load(open('$O/d$D.json'));print('diag $D', d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items() if 'wgrad' in k or 'slot' in k})"
done
