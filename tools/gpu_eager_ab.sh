#!/bin/bash
# A/B of the eager drop-in loop: tools/host_profile.py's loop vs bench.py --per-step --no-graph.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python tools/host_profile.py 50 --noprof > gpurun_out/hp_$i.txt 2>&1 || exit 3
  grep "eager" gpurun_out/hp_$i.txt
  timeout -k 10 200 python bench.py --no-cpu-baseline --per-step --no-graph --steps 50 --warmup 10 > gpurun_out/be_$i.json 2>/dev/null || exit 3
  python -c "import json;d=json.load(open('gpurun_out/be_$i.json'));print('bench eager', d['ms_per_step'])"
done
