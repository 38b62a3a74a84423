#!/bin/bash
# The other bench lines with a rocprofv3 kernel trace each: C = 32 (README width), the U-Net (cfg5),
# cfg3 and the per-window loops.  LINES="c32 unet cfg3 perstep eager" selects.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lines
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 $R/bench.py --no-cpu-baseline "$@" > $O/line_$n.json 2> $O/line_$n.err || { echo "$n failed"; tail -10 $O/line_$n.err; return 4; }
  python3 -c "import json;d=json.load(open('$O/line_$n.json'));print('$n', d['ms_per_step'], d['value'], (d.get('roofline') or {}).get('frac'))"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 2 "$@" > $O/prof_$n.json 2> $O/prof_$n.err || { echo "$n rocprof failed"; tail -10 $O/prof_$n.err; return 5; }
  python3 $R/tools/kstats.py $O/prof_$n/run_kernel_stats.csv 12
}
for l in ${LINES:-c32 unet}; do
  case $l in
    c32) run c32 --channels 32 || exit 4 ;;
    unet) run unet --model SpikingRecEVFlowNet --steps 3 --warmup 2 || exit 4 ;;
    cfg3) run cfg3 --res 256 --batch 4 || exit 4 ;;
    perstep) run perstep --per-step || exit 4 ;;
    eager) run eager --per-step --no-graph || exit 4 ;;
  esac
done
