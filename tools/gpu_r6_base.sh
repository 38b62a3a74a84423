#!/bin/bash
# Round-6 baseline lines on this round's boxes: cfg2 (default), C = 32.
set -u
O=gpurun_out/r6base
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.err || { tail -20 $O/cfg2.err; exit 4; }
python -c "import json;d=json.load(open('$O/cfg2.json'));print('cfg2', d['ms_per_step'], d['roofline']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --no-cpu-baseline --channels 32 > $O/c32.json 2> $O/c32.err || { tail -20 $O/c32.err; exit 5; }
python -c "import json;d=json.load(open('$O/c32.json'));print('c32', d['ms_per_step'], d['roofline']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
