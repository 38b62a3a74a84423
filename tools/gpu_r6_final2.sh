#!/bin/bash
# Round-6 final evidence, part 2: the other bench lines with a kernel trace each (tools/gpu_r5_lines.sh:
# C = 32, U-Net cfg5, cfg3, the per-window loops), the eval line, and the HBM-traffic / SQ counter passes
# over the cfg2 workload (tools/pmc.sh -> profiles/pmc_traffic.json, copied to gpurun_out).
set -u
LINES="${LINES:-c32 unet cfg3 perstep eager}" bash tools/gpu_r5_lines.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --eval > gpurun_out/lines/line_eval.json 2> gpurun_out/lines/line_eval.err || { echo "eval failed"; tail -10 gpurun_out/lines/line_eval.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/lines/line_eval.json'));print('eval', d['ms_per_step'], d['value'], (d.get('roofline') or {}).get('frac'))"
PMC_KEY=C8_R128_B8 bash tools/pmc.sh > gpurun_out/pmc_summary.txt 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_summary.txt; exit 7; }
tail -12 gpurun_out/pmc_summary.txt
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
