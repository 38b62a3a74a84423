#!/bin/bash
# U-Net backward elementwise work: tests, the cfg5 line, the per-dispatch lif_bwd trace, and the
# torch ops (fills / copies) of one eager step.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_unet.py tests/test_gpu_parity.py -k "unet or convlif or variants or pack or dec_in" > gpurun_out/t_unet5.log 2>&1
rc=$?
tail -2 gpurun_out/t_unet5.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/t_unet5.log | head -20; exit $rc; fi
timeout -k 10 400 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/unet5.json 2> gpurun_out/unet5.err || { tail -20 gpurun_out/unet5.err; exit 4; }
python -c "
import json;d=json.load(open('gpurun_out/unet5.json'));k=d['kernels']
print('unet', d['ms_per_step'], ' '.join('%s %.1f' % (n, v['avg_us']*v['launches']/1e3) for n, v in sorted(k.items(), key=lambda x: -x[1]['avg_us']*x[1]['launches'])[:10]))"
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/unet_ew5
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py unet 256 16 2 32 1 > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -5 $OUT/kt.log; exit 6; }
echo done
