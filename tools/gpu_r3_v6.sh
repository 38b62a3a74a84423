#!/bin/bash
# Every GPU test, the default line, the cfg5 line and a cfg5 kernel trace (U-Net elementwise kernels,
# deterministic loss backward).
set -u
mkdir -p gpurun_out/v6
O=gpurun_out/v6
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print('cfg2', d['ms_per_step'], d['value'], d['roofline'].get('frac'))"
timeout -k 10 600 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > $O/unet.json 2> $O/unet.err || { echo "unet failed"; tail -20 $O/unet.err; exit 8; }
python -c "
import json;d=json.load(open('$O/unet.json'));k=d['kernels']
print('unet', d['ms_per_step'], ' '.join('%s %.1f' % (n, v['avg_us']*v['launches']/1e3) for n, v in sorted(k.items(), key=lambda x: -x[1]['avg_us']*x[1]['launches'])[:12]))"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_step.py unet 256 16 2 32 1 > $R/$O/kt.log 2>&1 || { echo "trace failed"; tail -5 $R/$O/kt.log; exit 6; }
echo done
