#!/bin/bash
# Round-5 GPU run: every GPU test (or those matching $1), smoke, the default bench line, a rocprofv3
# kernel trace of the bench (step breakdown + per-task-kind attribution of the slot launches), and one
# SQ counter pass over the eager bench workload attributed per task kind (tools/slot_attrib.py).
# Stops at the first failing GPU step.
set -u
O=gpurun_out/r5${R5TAG:-}
mkdir -p $O
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread -s ${K:+-k "$K"} > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['avg_us'], (d.get('cpu_baseline') or {}).get('value')); print({k:v['avg_us'] for k,v in d['kernels'].items()})"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 5; }
python3 $R/tools/trace_step.py $R/$O/prof/run_kernel_trace.csv -2 > $R/$O/step_breakdown.txt && head -16 $R/$O/step_breakdown.txt
python3 $R/tools/slot_attrib.py $R/$O/prof/run_kernel_trace.csv bwd > $R/$O/attrib_time_bwd.json
python3 $R/tools/slot_attrib.py $R/$O/prof/run_kernel_trace.csv fwd > $R/$O/attrib_time_fwd.json
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $R/$O/pmc1 -o run --output-format csv -- python3 $R/tools/prof_step.py > $R/$O/pmc1.log 2>&1 || { echo "pmc failed"; tail -5 $R/$O/pmc1.log; exit 6; }
F=$(ls $R/$O/pmc1/*counter_collection.csv $R/$O/pmc1/*/*counter_collection.csv 2>/dev/null | head -1)
python3 $R/tools/slot_attrib.py $F bwd > $R/$O/attrib_sq_bwd.json
python3 $R/tools/slot_attrib.py $F fwd > $R/$O/attrib_sq_fwd.json
python3 -c "
import json
for f in ['attrib_time_bwd','attrib_time_fwd','attrib_sq_bwd','attrib_sq_fwd']:
    d=json.load(open('$R/$O/'+f+'.json'))
    for q,v in d['quantities'].items(): print(f, q, v['per_task'], 'total', v['pass_total'], 'res', v['fit_rel_residual'])
"
