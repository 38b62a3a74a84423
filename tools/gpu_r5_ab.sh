#!/bin/bash
# A/B of library builds on the default bench line (alternating runs) plus one SQ counter pass each,
# attributed per slot-task kind (tools/slot_attrib.py).  LIBS="name:path ..." (the default build is "base").
set -u
O=gpurun_out/ab${ABTAG:-}
mkdir -p $O
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for spec in base:default ${LIBS:-}; do
    n=${spec%%:*}; path=${spec#*:}
    if [ "$path" = default ]; then unset SNNFLOW_LIB; else export SNNFLOW_LIB=$R/$path; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "bench $n failed"; tail -20 $O/bench_${n}_$rep.err; exit 4; }
    python -c "import json;d=json.load(open('$O/bench_${n}_$rep.json'));print('$n', d['ms_per_step'], d['value'], d['roofline']['avg_us'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:9]})"
  done
done
cd /tmp && export TMPDIR=/tmp
for spec in base:default ${LIBS:-}; do
  n=${spec%%:*}; path=${spec#*:}
  if [ "$path" = default ]; then unset SNNFLOW_LIB; else export SNNFLOW_LIB=$R/$path; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $R/$O/pmc_$n -o run --output-format csv -- python3 $R/tools/prof_step.py > $R/$O/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $R/$O/pmc_$n.log; exit 6; }
  F=$(ls $R/$O/pmc_$n/*counter_collection.csv $R/$O/pmc_$n/*/*counter_collection.csv 2>/dev/null | head -1)
  python3 $R/tools/slot_attrib.py $F bwd > $R/$O/attrib_${n}_bwd.json
  python3 -c "
import json
d=json.load(open('$R/$O/attrib_${n}_bwd.json'))
for q,v in d['quantities'].items(): print('$n', q, v['per_task'], 'total', v['pass_total'])
"
done
