set -u
ABTAG=_ps BENCH_ARGS="--per-step" ENVS="tile:SNNFLOW_BWD_TILE=1" bash tools/gpu_envab.sh || exit 4
ABTAG=_psng BENCH_ARGS="--per-step --no-graph" ENVS="tile:SNNFLOW_BWD_TILE=1" bash tools/gpu_envab.sh || exit 4
ABTAG=_r256 BENCH_ARGS="--res 256 --steps 10" ENVS="tile:SNNFLOW_BWD_TILE=1" bash tools/gpu_envab.sh || exit 4
