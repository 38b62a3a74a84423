set -o pipefail
SNNFLOW_PIPE_FWD=2 KTRACE_PIPE=1 SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace_slot.so timeout -k 10 200 python tools/ktrace_slot.py > gpurun_out/ktrace_pipe2.json 2>&1 || exit 3
for v in "0 1" "2 0" "2 1" "2 2" "4 1" "4 0" "8 0"; do set -- $v
  SNNFLOW_PIPE_FWD=$1 SNNFLOW_PIPE_ORDER=$2 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/o_$1_$2.json 2>/dev/null || exit 4
  python -c "import json;d=json.load(open('gpurun_out/o_$1_$2.json'));print('tpb $1 order $2', round(d['ms_per_step'],4), 'ms', {k:v['avg_us'] for k,v in list(d.get('kernels',{}).items())[:2]})"
done
