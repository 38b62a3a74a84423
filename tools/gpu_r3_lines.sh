#!/bin/bash
# The secondary bench lines: C = 32, cfg3, the eager per-window loop, the per-step graph, cfg5 U-Net
# (with its CPU baseline).  Each bench in its own time limit; stops at the first failure.
set -u
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 420 python bench.py "$@" > gpurun_out/line_$tag.json 2> gpurun_out/line_$tag.err || { echo "$tag failed"; tail -20 gpurun_out/line_$tag.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/line_$tag.json'));print('$tag', d['ms_per_step'], d['value'], d['roofline'].get('kernel'), d['roofline'].get('frac'), {k:(v['avg_us'],v['launches']) for k,v in list(d.get('kernels',{}).items())[:8]})"
}
run c32 --channels 32 --no-cpu-baseline
run cfg3 --res 256 --batch 4 --no-cpu-baseline
run eager --per-step --no-graph --no-cpu-baseline
run perstep --per-step --no-cpu-baseline
run unet --model SpikingRecEVFlowNet --steps 3 --warmup 1
