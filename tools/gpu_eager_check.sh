#!/bin/bash
# Eager drop-in loop vs graph lines + the parity tests the host-path changes touch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "golden or sequence or cell or state or hooks or tebn or full" \
  > gpurun_out/eager_tests.txt 2>&1 || { tail -30 gpurun_out/eager_tests.txt; exit 3; }
tail -2 gpurun_out/eager_tests.txt
timeout -k 10 200 python tools/host_profile.py 10 > gpurun_out/host_prof.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --per-step > gpurun_out/b_perstep.json 2> gpurun_out/b_perstep.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --per-step --no-graph > gpurun_out/b_eager.json 2> gpurun_out/b_eager.err
rc=$?
head -3 gpurun_out/host_prof.txt
for f in b_perstep b_eager; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['ms_per_step'],d['value'],d['roofline']['frac'])"; done
exit $rc
