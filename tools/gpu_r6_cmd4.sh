# Host profile of the eager per-window loop (cProfile of the timed loop) and a kernel trace of the C = 32 line.
set -u
O=gpurun_out/r6c4
mkdir -p $O
for i in 1 2; do
SNNFLOW_BENCH_PROFILE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --per-step --no-graph --steps 40 --warmup 5 > $O/eager$i.json 2> $O/eager_prof$i.txt || { tail -20 $O/eager_prof$i.txt; exit 4; }
python -c "import json;d=json.load(open('$O/eager$i.json'));print('eager', d['ms_per_step'])"
done
head -60 $O/eager_prof2.txt | cut -c1-200
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_c32 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --channels 32 --steps 5 --warmup 3 > $R/$O/c32.json 2> $R/$O/c32.err || { tail -20 $R/$O/c32.err; exit 5; }
python3 $R/tools/kstats.py $R/$O/prof_c32/run_kernel_stats.csv 20
