mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model SpikingRecEVFlowNet --res 128 --batch 4 --T 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ub_small.json 2> gpurun_out/ub_small.err || { tail -30 gpurun_out/ub_small.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ub_small.json'));print(d['ms_per_step'],d['value'],d['roofline']);print(json.dumps(d['kernels']))"
timeout -k 10 600 python bench.py --model SpikingRecEVFlowNet --steps 3 --warmup 1 > gpurun_out/ub_cfg5.json 2> gpurun_out/ub_cfg5.err || { tail -30 gpurun_out/ub_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ub_cfg5.json'));print(d['ms_per_step'],d['value'],d['roofline'],d['cpu_baseline']);print(json.dumps(d['kernels']))"
