#!/bin/bash
# U-Net cfg5 line with per-GEMM-shape kernel names (SNNFLOW_UNET_SHAPES=1), sorted by total time.
set -u
O=gpurun_out/r6shapes${TAG:-}
mkdir -p $O
SNNFLOW_UNET_SHAPES=1 timeout -k 10 400 python bench.py --no-cpu-baseline --model SpikingRecEVFlowNet --steps 3 --warmup 2 > $O/unet.json 2> $O/unet.err || { tail -20 $O/unet.err; exit 5; }
python - <<PY
import json
d=json.load(open('$O/unet.json'))
print('unet', d['ms_per_step'])
ks=sorted(d['kernels'].items(), key=lambda kv: -kv[1]['avg_us']*kv[1]['launches'])
for k,v in ks[:45]:
    print(f"{k:60s} n={v['launches']:4d} avg={v['avg_us']:8.2f} tot_ms/step={v['avg_us']*v['launches']/1000/3:7.2f} tf={v.get('tflops')} iss={v.get('issued_frac')}")
PY
