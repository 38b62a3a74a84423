#!/bin/bash
set -u
L=snn_event-based_optical_flow_amd/snnflow
for v in libsnnflow libsnnflow_sleep8 libsnnflow_pollat libsnnflow_pollat8; do
  echo "== $v"
  SNNFLOW_LIB=$L/$v.so timeout -k 10 120 python tools/seq_time.py 2>/dev/null || exit 3
done
