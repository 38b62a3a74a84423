#!/bin/bash
# U-Net forward convs through LDS-DMA: every U-Net / ConvLIF GPU test, then the cfg5 line A/B
# (DMA 3 stages / 2 stages / the register-staged kernel).
set -u
mkdir -p gpurun_out
T="python -u -m pytest -v -p no:cacheprovider --timeout 400 --timeout-method thread -s"
timeout -k 10 700 $T tests/test_gpu_unet.py tests/test_gpu_parity.py -k "unet or convlif or variants" > gpurun_out/t_unet.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|cfg5 shapes\] max" gpurun_out/t_unet.log | cut -c1-250 | tail -30
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
for v in libsnnflow libsnnflow_unetns2 libsnnflow_unetold; do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$v.so SNNFLOW_UNET_SHAPES=1 timeout -k 10 400 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/unet_$v.json 2> gpurun_out/unet_$v.err || { tail -20 gpurun_out/unet_$v.err; exit 4; }
  python -c "
import json;d=json.load(open('gpurun_out/unet_$v.json'));k=d['kernels']
conv=sum(v['avg_us']*v['launches'] for n,v in k.items() if n.startswith('unet_conv'))/1e3/d['steps']
print('$v', d['ms_per_step'], 'conv ms/step %.1f' % conv)"
done
exit $rc
