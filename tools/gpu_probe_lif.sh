#!/bin/bash
set -u
mkdir -p gpurun_out
for v in libsnnflow libsnnflow_probe_noatomic; do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$v.so timeout -k 10 400 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/probe_$v.json 2> gpurun_out/probe_$v.err || { tail -20 gpurun_out/probe_$v.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/probe_$v.json'));k=d['kernels'];print('$v', d['ms_per_step'], k['unet_lif_bwd'])"
done
