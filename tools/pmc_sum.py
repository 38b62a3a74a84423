"""Per-kernel-template averages of rocprofv3 --pmc counter CSVs under a directory (one line per kernel)."""
import collections
import csv
import glob
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        m = re.search(r"k_\w+(<[^>]*>)?", n)
        k = m.group(0) if m else n[:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
for k, cs in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if pat and not pat.search(k):
        continue
    out = []
    for c, v in sorted(cs.items()):
        nd = max(len(disp[(k, c)]), 1)
        out.append(f"{c}={v / nd:.4g}")
    print(k, "n=%d" % max(len(disp[(k, c)]) for c in cs), " ".join(out))
