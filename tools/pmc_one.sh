#!/bin/bash
# One rocprofv3 counter pass over tools/prof_step.py; per-kernel-class averages of each counter.
#   bash tools/pmc_one.sh <tag> "<counters>"   (<= 8 SQ_ counters; no trace domains with --pmc)
set -u
tag=$1; ctrs=$2
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_step.py > $OUT.log 2>&1 || { echo "pass failed"; tail -5 $OUT.log; exit 1; }
python3 - $OUT <<'PY'
import collections, csv, glob, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        m = re.search(r"k_\w+(<[^>]*>)?", n)
        k = m.group(0) if m else n[:40]
        key = (r["Dispatch_Id"], r["Counter_Name"])
        acc[k][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
for k, cs in sorted(acc.items()):
    out = []
    for c, vals in sorted(cs.items()):
        per = collections.defaultdict(float)
        for d, v in vals:
            per[d] += v
        out.append(f"{c}={sum(per.values()) / len(per):.0f}")
    print(k, " ".join(out))
PY
