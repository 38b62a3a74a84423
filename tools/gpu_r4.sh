#!/bin/bash
# Round-4 GPU iteration: the whole -m gpu suite, then bench A/B over the tile-pipeline settings
#   PIPES="0:0 2:0" bash tools/gpu_r4.sh        (fwd:bwd tiles per block; 0 = one tile per block)
set -u -o pipefail
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${KSEL:+-k "$KSEL"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -25 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && { echo "pytest rc=$rc -> stop"; exit $rc; }
fi
for rep in 1 2; do
  for pv in ${PIPES:-0:0 2:0}; do
    f=${pv%%:*}; b=${pv##*:}
    SNNFLOW_PIPE_FWD=$f SNNFLOW_PIPE_BWD=$b timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${f}_${b}_$rep.json 2> gpurun_out/ab_${f}_${b}_$rep.err || { tail -20 gpurun_out/ab_${f}_${b}_$rep.err; exit 4; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${f}_${b}_$rep.json'));print('pipe $pv', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],4), 'ms', {k:v['avg_us'] for k,v in list(d.get('kernels',{}).items())[:6]})"
  done
done
