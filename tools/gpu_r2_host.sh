mkdir -p gpurun_out
timeout -k 10 200 python tools/host_profile.py 10 > gpurun_out/host_prof.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_default.json 2> gpurun_out/b_default.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --per-step > gpurun_out/b_perstep.json 2> gpurun_out/b_perstep.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --per-step --no-graph > gpurun_out/b_eager.json 2> gpurun_out/b_eager.err
rc=$?
head -3 gpurun_out/host_prof.txt
for f in b_default b_perstep b_eager; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['ms_per_step'],d['value'],d['roofline']['frac'])"; done
exit $rc
