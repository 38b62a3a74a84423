#!/bin/bash
# Conflict-free LDS swizzle for the U-Net conv kernels: U-Net / ConvLIF tests, the cfg5 line, and the
# LDS counters of one pass.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_unet.py tests/test_gpu_parity.py -k "unet or convlif or variants" > gpurun_out/t_unet2.log 2>&1
rc=$?
tail -2 gpurun_out/t_unet2.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/t_unet2.log | head -20; exit $rc; fi
SNNFLOW_UNET_SHAPES=1 timeout -k 10 400 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/unet_swz.json 2> gpurun_out/unet_swz.err || { tail -20 gpurun_out/unet_swz.err; exit 4; }
python -c "
import json;d=json.load(open('gpurun_out/unet_swz.json'));k=d['kernels']
conv=sum(v['avg_us']*v['launches'] for n,v in k.items() if n.startswith('unet_conv'))/1e3
dg=sum(v['avg_us']*v['launches'] for n,v in k.items() if n.startswith('unet_dgrad'))/1e3
print('unet', d['ms_per_step'], 'conv ms %.1f dgrad ms %.1f' % (conv, dg))"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY -d $GRAFT_REPO_ROOT/gpurun_out/pmc_swz -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py unet 256 16 2 32 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc_swz.log 2>&1 || { echo "pmc failed"; exit 5; }
python3 - $GRAFT_REPO_ROOT/gpurun_out/pmc_swz <<'PY'
import collections, csv, glob, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"k_\w+(<[^>]*>)?", r["Kernel_Name"])
        k = m.group(0) if m else r["Kernel_Name"][:40]
        if "conv" in k:
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, cs in sorted(acc.items()):
    print(k, "conflict cycles per LDS inst %.2f" % (cs["SQ_LDS_BANK_CONFLICT"] / max(cs["SQ_INSTS_LDS"], 1)),
          "wait/wave %.2f" % (cs["SQ_WAIT_ANY"] / max(cs["SQ_WAVE_CYCLES"], 1)))
PY
