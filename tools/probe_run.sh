#!/bin/bash
# Timing attribution: tools/kprobe.py against the shipped library and each probe build.
set -u
mkdir -p gpurun_out
for L in libsnnflow.so libsnnflow_probe1.so libsnnflow_probe2.so libsnnflow_probe4.so libsnnflow_probe8.so libsnnflow_probe16.so libsnnflow_probe3.so libsnnflow_probe15.so; do
  SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/$L timeout -k 10 120 python tools/kprobe.py >> gpurun_out/kprobe.jsonl 2>> gpurun_out/kprobe.err || { echo "kprobe $L failed rc=$?"; tail -20 gpurun_out/kprobe.err; exit 1; }
done
cat gpurun_out/kprobe.jsonl
