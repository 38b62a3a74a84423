#!/bin/bash
# U-Net cfg5 A/B: for each env setting in $AB the line (3 steps) with per-GEMM-shape kernel names;
# prints ms/step and the per-shape totals (ms per step) of the kernels matching $PAT.
set -u
O=gpurun_out/r6unetab${TAG:-}
mkdir -p $O
i=0
for E in ${AB:-X=0}; do
  i=$((i+1))
  env SNNFLOW_UNET_SHAPES=1 $E timeout -k 10 400 python bench.py --no-cpu-baseline --model SpikingRecEVFlowNet --steps 3 --warmup 2 > $O/u$i.json 2> $O/u$i.err || { tail -20 $O/u$i.err; exit 5; }
  python - $O/u$i.json "$E" "${PAT:-conv|dgrad|wgrad}" <<'PY'
import json, re, sys
d = json.load(open(sys.argv[1])); pat = re.compile(sys.argv[3])
ks = sorted(d['kernels'].items(), key=lambda kv: -kv[1]['avg_us'] * kv[1]['launches'])
tot = {}
for k, v in ks:
    fam = k.split('[')[0]
    tot[fam] = tot.get(fam, 0) + v['avg_us'] * v['launches'] / 1000
print(sys.argv[2], 'ms/step', d['ms_per_step'], {k: round(v, 2) for k, v in tot.items() if v > 1})
for k, v in ks[:40]:
    if pat.search(k):
        print(f"   {k:48s} n={v['launches']:4d} avg={v['avg_us']:8.2f} ms={v['avg_us']*v['launches']/1000:6.2f} tf={v.get('tflops')}")
PY
done
