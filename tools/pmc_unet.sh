#!/bin/bash
# Counter passes over a short cfg5-shape U-Net train step (256^2, B=16, 2 windows): per kernel
# template, the SQ wait / LDS / VMEM picture, matrix-core busy, L2 and HBM traffic.  One rocprofv3
# run per pass, counters only.
set -u
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_unet
mkdir -p $OUT
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
            "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py unet 256 16 2 32 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import collections, csv, glob, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        m = re.search(r"k_\w+(<[^>]*>)?", n)
        k = m.group(0) if m else n[:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, cs in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    out = []
    for c, v in sorted(cs.items()):
        nd = max(len(disp[(k, c)]), 1)
        out.append(f"{c}={v / nd:.4g}")
    print(k, "n=%d" % max(len(disp[(k, c)]) for c in cs), " ".join(out))
PY
