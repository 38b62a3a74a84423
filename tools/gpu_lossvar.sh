#!/bin/bash
# Loss A/B over library variants: bitwise dL/dflow vs the default library + kernel-trace stats of each.
#   VARS="b256_n128 b512_n512" bash tools/gpu_lossvar.sh   (snnflow/libsnnflow_<var>.so next to libsnnflow.so)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base ${VARS}; do
  if [ $v = base ]; then unset SNNFLOW_LIB; else export SNNFLOW_LIB=$R/snn_event-based_optical_flow_amd/snnflow/libsnnflow_$v.so; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $R/tools/loss_bits.py $O/$v.npz > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
done
unset SNNFLOW_LIB
python3 - <<PY
import numpy as np, glob, csv, re
base = np.load("$O/base.npz")
for v in ["base"] + "${VARS}".split():
    x = np.load(f"$O/{v}.npz")
    same = all(x[k].tobytes() == base[k].tobytes() for k in ("loss", "g"))
    f = glob.glob(f"$O/{v}/**/*kernel_stats.csv", recursive=True)[0]
    t = {re.search(r"(k_iwe_\w+)", r["Name"]).group(1): float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f)) if "k_iwe" in r["Name"]}
    print(v, "bit-identical" if same else "DIFFERS", " ".join(f"{k} {t[k]:.2f}" for k in sorted(t)), f"sum {sum(t.values()):.2f} us")
PY
