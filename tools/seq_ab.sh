#!/bin/bash
# Persistent-forward visibility A/B: diagnostics with each library variant.
set -u
L=snn_event-based_optical_flow_amd/snnflow
for v in libsnnflow libsnnflow_plain libsnnflow_fence libsnnflow_plainfence; do
  echo "== $v"
  SNNFLOW_LIB=$L/$v.so timeout -k 10 120 python tools/seq_diag.py 2>/dev/null | grep -E "t=0: state|t=2: state|sync" || exit 3
done
