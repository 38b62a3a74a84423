#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_profile.py 10 > gpurun_out/host_prof.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --per-step --no-graph > gpurun_out/b_eager.json 2> gpurun_out/b_eager.err
rc=$?
head -3 gpurun_out/host_prof.txt
python -c "import json;d=json.load(open('gpurun_out/b_eager.json'));print('b_eager',d['ms_per_step'],d['value'])"
exit $rc
