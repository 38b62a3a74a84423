#!/bin/bash
# Eager host path: parity tests that touch the engine's caches, then the host attribution and the
# eager / per-step bench lines.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py -k "replaced or state_api or subtract or detach or golden or fused_adam or norm" > gpurun_out/t_eager2.log 2>&1
rc=$?
tail -3 gpurun_out/t_eager2.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/t_eager2.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/eager_micro.py > gpurun_out/eager_micro3.txt 2>&1 || { tail -20 gpurun_out/eager_micro3.txt; exit 3; }
tail -12 gpurun_out/eager_micro3.txt
timeout -k 10 300 python bench.py --per-step --no-graph --no-cpu-baseline > gpurun_out/line_eager2.json 2> gpurun_out/line_eager2.err || { tail -20 gpurun_out/line_eager2.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/line_eager2.json'));print('eager', d['ms_per_step'], d['value'])"
