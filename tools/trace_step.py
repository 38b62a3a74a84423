"""Per-step breakdown of a rocprofv3 kernel trace: kernels between consecutive
slab_reduce launches (one train step), duration and preceding gap per kernel name."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "slab_reduce" in r["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
seg = rows[idx[which - 1] + 1:idx[which] + 1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
d, g = collections.defaultdict(list), collections.defaultdict(float)
prev = None
for r in seg:
    m = re.search(r"k_\w+(<[^>]*>)?|multi_tensor_apply_kernel|copyBuffer\w*|CatArray\w*|fillBuffer\w*|reduce_kernel|"
                  r"lpnorm\w*|elementwise_kernel\w*", r["Kernel_Name"])
    k = m.group(0) if m else r["Kernel_Name"][:50]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    d[k].append((e - s) / 1e3)
    if prev is not None:
        g[k] += (s - prev) / 1e3
    prev = e
busy = sum(sum(v) for v in d.values())
print(f"step span {(t1 - t0) / 1e3:.1f} us, kernels {len(seg)}, busy {busy:.1f} us")
print(f"{'total_us':>9} {'gap_us':>8} {'n':>4}  kernel")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v):9.1f} {g[k]:8.1f} {len(v):4d}  {k}")
