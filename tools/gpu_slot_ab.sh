#!/bin/bash
# Multi-tile slot kernels: GPU suite with multi-tile blocks forced, then the default bench line
# per (library variant, tiles per block).  Variants: make -C csrc variant V=<v> D=...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/slot
if [ -z "${SKIP_TESTS:-}" ]; then
SNNFLOW_SLOT_TPB=${TEST_TPB:-3} timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/slot/tests.txt 2>&1 || { tail -40 gpurun_out/slot/tests.txt; exit 3; }
tail -2 gpurun_out/slot/tests.txt
fi
DEF="base:1 base:2 base:4 bw6:1 bw6:2 pf0:2"
for cfg in ${CFGS:-$DEF}; do
  v=${cfg%%:*}; t=${cfg##*:}
  unset SNNFLOW_LIB; [ "$v" != base ] && export SNNFLOW_LIB=$GRAFT_REPO_ROOT/snn_event-based_optical_flow_amd/snnflow/libsnnflow_$v.so
  SNNFLOW_SLOT_TPB=$t timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/slot/b_${v}_$t.json 2>gpurun_out/slot/b_${v}_$t.err || { tail -5 gpurun_out/slot/b_${v}_$t.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/slot/b_${v}_$t.json'));print('$v tpb=$t', d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
done
