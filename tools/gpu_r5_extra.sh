#!/bin/bash
# Extra round-5 lines: the evaluation pass, C = 16, and the U-Net matrix-core pass.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/extra
mkdir -p $O
timeout -k 10 300 python3 $R/bench.py --eval > $O/bench_eval.json 2> $O/bench_eval.err || { echo "eval failed"; tail -5 $O/bench_eval.err; exit 4; }
python3 -c "import json;d=json.load(open('$O/bench_eval.json'));print('eval', d['ms_per_step'], d['value'], (d.get('roofline') or {}).get('frac'))"
timeout -k 10 300 python3 $R/bench.py --channels 16 --no-cpu-baseline > $O/line_c16.json 2> $O/line_c16.err || { echo "c16 failed"; tail -5 $O/line_c16.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/line_c16.json'));print('c16', d['ms_per_step'], d['value'], (d.get('roofline') or {}).get('frac'))"
WL="unet" bash $R/tools/pmc_mfma.sh > $O/pmc_mfma_unet.txt 2>&1 || { echo "unet mfma failed"; tail -5 $O/pmc_mfma_unet.txt; exit 6; }
cp $R/gpurun_out/pmc_mfma/pmc_mfma.json $O/pmc_mfma_unet.json
python3 -c "
import json
d=json.load(open('$O/pmc_mfma_unet.json'))
for wl,ks in d['kernels'].items():
  print(wl, {k: v.get('mfma_busy_frac') for k,v in ks.items() if v.get('mfma_busy_frac')})
"
