#!/bin/bash
# Round-4 validation: every GPU test, smoke, the default bench line (with its CPU baseline), the eval
# line, the rocprofv3 kernel trace + stats, the PMC passes (SQ + traffic), and the secondary lines.
# Stops at the first failure of a GPU step.
set -u
O=gpurun_out/final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread -s > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 4; }
cat $O/bench.json
timeout -k 10 400 python bench.py --eval > $O/bench_eval.json 2> $O/bench_eval.err || { echo "eval bench failed"; tail -30 $O/bench_eval.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench_eval.json'));print('eval', d['ms_per_step'], d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['configs0'])"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -16 $R/$O/step_breakdown.txt
cd $R
bash tools/pmc.sh > $O/pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.txt; exit 6; }
tail -25 $O/pmc.txt
python3 tools/pmc_traffic.py gpurun_out/pmc C8_R128_B8 $O/pmc_counters.json > /dev/null
for spec in "c32:--channels 32" "cfg3:--res 256 --batch 4" "eager:--per-step --no-graph" "perstep:--per-step"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 400 python bench.py $args --no-cpu-baseline > $O/line_$tag.json 2> $O/line_$tag.err || { echo "$tag failed"; tail -20 $O/line_$tag.err; exit 7; }
  python -c "import json;d=json.load(open('$O/line_$tag.json'));print('$tag', d['ms_per_step'], d['value'], d['roofline'].get('kernel'), d['roofline'].get('frac'))"
done
timeout -k 10 600 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 --no-cpu-baseline > $O/line_unet.json 2> $O/line_unet.err || { echo "unet failed"; tail -20 $O/line_unet.err; exit 8; }
python -c "import json;d=json.load(open('$O/line_unet.json'));print('unet', d['ms_per_step'], d['value'], d['roofline'].get('frac'))"
