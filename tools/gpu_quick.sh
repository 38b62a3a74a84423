#!/bin/bash
# Parity tests + short benches (no CPU baseline) at C=8 and C=32.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for C in ${QUICK_CHANNELS:-8 32}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --channels $C > gpurun_out/b$C.json 2> gpurun_out/b$C.err || { tail -20 gpurun_out/b$C.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/b$C.json'));print($C, d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
