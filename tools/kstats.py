"""Summary of a rocprofv3 run_kernel_stats.csv: kernel (short name), calls, average and total us."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"].replace("(anonymous namespace)::", "")
    m = re.match(r"(void )?([\w:]+(<[^(]*>)?)", n)
    out.append((m.group(2)[:60] if m else n[:60], int(r["Calls"]), float(r["AverageNs"]) / 1e3,
                float(r["TotalDurationNs"]) / 1e3))
for name, calls, avg, tot in sorted(out, key=lambda x: -x[3])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{tot:10.1f} us  {calls:6d} x {avg:8.2f} us  {name}")
