#!/bin/bash
# U-Net: tests, then cfg5 line A/B (NSTAGE 2 default / 3).
set -u
mkdir -p gpurun_out
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_unet.py tests/test_gpu_parity.py -k "unet or convlif or variants" > gpurun_out/t_unet3.log 2>&1
rc=$?
tail -2 gpurun_out/t_unet3.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/t_unet3.log | head -20; exit $rc; fi
for v in libsnnflow; do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$v.so SNNFLOW_UNET_SHAPES=1 timeout -k 10 400 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/unet3_$v.json 2> gpurun_out/unet3_$v.err || { tail -20 gpurun_out/unet3_$v.err; exit 4; }
  python -c "
import json;d=json.load(open('gpurun_out/unet3_$v.json'));k=d['kernels']
cls={}
for n,v in k.items():
    c=n.split('[')[0]; cls[c]=cls.get(c,0)+v['avg_us']*v['launches']/1e3
print('$v', d['ms_per_step'], ' '.join('%s %.1f' % (c, t) for c, t in sorted(cls.items(), key=lambda x: -x[1])[:8]))"
done
