#!/bin/bash
# Capacity-capped slot schedule: the sequence parity tests, then bench A/B over SNNFLOW_SLOT_CAP.
set -u
mkdir -p gpurun_out
T="python -u -m pytest -q -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sequence or cfg2_train or wide or golden or persistent" > gpurun_out/t_cap.log 2>&1
rc=$?
tail -3 gpurun_out/t_cap.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " gpurun_out/t_cap.log | head -20; exit $rc; fi
for cap in 3 0 3 0; do
  SNNFLOW_SLOT_CAP=$cap timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/cap_$cap.json 2> gpurun_out/cap_$cap.err || { tail -20 gpurun_out/cap_$cap.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/cap_$cap.json'));print('cap $cap', d['ms_per_step'], {k:(v['avg_us'],v['launches']) for k,v in list(d['kernels'].items())[:2]})"
done
for cap in 3 0; do
  SNNFLOW_SLOT_CAP=$cap timeout -k 10 300 python bench.py --channels 32 --no-cpu-baseline > gpurun_out/cap32_$cap.json 2> gpurun_out/cap32_$cap.err || { tail -20 gpurun_out/cap32_$cap.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/cap32_$cap.json'));print('C32 cap $cap', d['ms_per_step'], {k:(v['avg_us'],v['launches']) for k,v in list(d['kernels'].items())[:2]})"
done
