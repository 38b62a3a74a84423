#!/bin/bash
# Timing attribution: tools/kprobe.py against the shipped library and each probe build.
set -u
mkdir -p gpurun_out
for L in $(cd snn_event-based_optical_flow_amd/snnflow && ls libsnnflow*.so); do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$L timeout -k 10 120 python tools/kprobe.py >> gpurun_out/kprobe.jsonl 2>> gpurun_out/kprobe.err || { echo "kprobe $L failed rc=$?"; tail -20 gpurun_out/kprobe.err; exit 1; }
done
cat gpurun_out/kprobe.jsonl
