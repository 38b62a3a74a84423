#!/bin/bash
# A/B of two library builds on the loss: bitwise dL/dflow comparison + kernel-trace stats of each.
#   bash tools/gpu_lossbits.sh   (expects snnflow/libsnnflow_old.so next to libsnnflow.so)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then export SNNFLOW_LIB=$R/snn_event-based_optical_flow_amd/snnflow/libsnnflow_old.so; else unset SNNFLOW_LIB; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $R/tools/loss_bits.py $O/$v.npz > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  tail -1 $O/$v.log
done
unset SNNFLOW_LIB
python3 - <<PY
import numpy as np, glob, csv
a, b = np.load("$O/old.npz"), np.load("$O/new.npz")
for k in ("loss", "g"):
    x, y = a[k], b[k]
    print(k, "bit-identical" if x.tobytes() == y.tobytes() else f"DIFFER max {np.abs(x - y).max()}")
for v in ("old", "new"):
    f = glob.glob(f"$O/{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "iwe" in r["Name"]:
            print(v, r["Name"].split("(")[0][-28:], r["Calls"], f'{float(r["AverageNs"]) / 1000:.2f} us')
PY
