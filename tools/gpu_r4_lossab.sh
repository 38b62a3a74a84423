#!/bin/bash
# Round-4: kernel times of the loss kernels per library variant (rocprofv3 --stats of a short bench)
set -u -o pipefail
mkdir -p gpurun_out/lossab
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-base}; do
  lib=$R/snn_event-based_optical_flow_amd/snnflow/libsnnflow.so
  [ "$v" != base ] && lib=$R/snn_event-based_optical_flow_amd/snnflow/libsnnflow_$v.so
  SNNFLOW_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lossab/$v -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $R/gpurun_out/lossab/$v.json 2> $R/gpurun_out/lossab/$v.err || { echo "$v failed"; tail -5 $R/gpurun_out/lossab/$v.err; exit 3; }
  python3 - "$R/gpurun_out/lossab/$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("iwe", "clip_adam", "aee", "wgrad<2", "prep_weights", "slab_reduce")):
        out.append((n.split("(")[0].replace("(anonymous namespace)::", "")[:40], round(float(r["AverageNs"]) / 1e3, 2)))
print(sys.argv[2], out)
PY
done
