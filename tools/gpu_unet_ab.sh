#!/bin/bash
# U-Net kernel A/B: the U-Net parity tests, then the cfg5 bench line per-shape with the
# tap-fused weight gradient on and off (SNNFLOW_UNET_WROWS).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/unet
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_unet.py > gpurun_out/unet/tests.txt 2>&1 || { tail -30 gpurun_out/unet/tests.txt; exit 3; }
tail -2 gpurun_out/unet/tests.txt
fi
for w in ${WROWS:-1 0}; do
  SNNFLOW_UNET_WROWS=$w SNNFLOW_UNET_SHAPES=1 timeout -k 10 300 python bench.py --model SpikingRecEVFlowNet --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/unet/b_w$w.json 2> gpurun_out/unet/b_w$w.err || { tail -5 gpurun_out/unet/b_w$w.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/unet/b_w$w.json'));print('wrows=$w', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'])"
done
