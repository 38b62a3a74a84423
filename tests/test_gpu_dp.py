"""The N>1 bench step path on the GPU (per resident batch a forward + backward graph, the SUM
all-reduce of that graph's flat gradient buffer, and its update graph, bench.py step()), rehearsed with 2 fresh ranks sharing the box's
one GPU over gloo (SNNFLOW_SHARE_GPU=1).  bench.py --dp-check replays one step exactly as timed
and checks that the all-reduced gradient is the sum of the two ranks' own gradients (each rank
draws its own synthetic stream, so they differ) and that after clip + Adam both ranks hold the
same parameters.  The RCCL (nccl backend) path is the same code with another backend string: it is
rehearsed here at world size 1 (bench.py --force-dist: the one-rank SUM all-reduce over RCCL between
the two graphs), and runs at 8 ranks only in the driver's scaling bench.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("extra", [[], ["--no-graph"]])
def test_dp_step_two_ranks_shared_gpu(extra):
    env = dict(os.environ, SNNFLOW_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    port = 29611 + len(extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--dist-backend", "gloo",
           "--dp-check", "--batch", "2", "--pool", "2"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:]
    res = json.loads(lines[-1])["dp_check"]
    print("\n[dp-check]", res)
    assert res["world"] == 2
    assert res["ranks_local_grads_differ_by"] > 0  # the ranks really saw different batches
    assert res["allreduce_rel_err"] < 1e-6
    assert res["param_max_diff_after_update"] == 0.0


def test_bench_gpus_flag_launches_its_ranks():
    """`python bench.py --gpus 2` with no launcher and no WORLD_SIZE: bench.py starts the two ranks
    itself (children through torch.distributed.run; the ranks share the box's one GPU over gloo
    here) and the step path runs with world == 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SNNFLOW_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--no-cpu-baseline", "--dp-check", "--batch", "2", "--pool", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:]
    res = json.loads(lines[-1])["dp_check"]
    print("\n[dp-check via --gpus]", res)
    assert res["world"] == 2
    assert res["allreduce_rel_err"] < 1e-6
    assert res["param_max_diff_after_update"] == 0.0


def test_bench_two_ranks_timed_line():
    """The timed N = 2 path end to end (gloo rehearsal on the shared GPU, 3 resident batches, so 6
    graph pairs with the state ping-pong): one JSON line with n_gpus 2 and a positive rate."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SNNFLOW_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--batch", "2", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:]
    res = json.loads(lines[-1])
    print("\n[N=2 timed]", res["value"], res["ms_per_step"])
    assert res["n_gpus"] == 2 and res["value"] > 0 and res["config"]["parallelism"] == "dp2"


def test_rccl_world_size_one_dp_check():
    """The real RCCL code path once on the box: bench.py --force-dist runs the N>1
    step path -- process group on the `nccl` backend (= RCCL), batch 1's forward + backward graph, the
    SUM all-reduce of that graph's flat gradient buffer, its update graph -- at world size 1 under
    torch.distributed.run.  The all-reduced buffer must equal the local gradient exactly (a one-rank SUM),
    which also proves the collective is ordered after the graph that wrote the buffer."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SNNFLOW_SHARE_GPU")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29631", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--force-dist", "--dp-check",
           "--pool", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])["dp_check"]
    print("\n[rccl world 1 dp-check]", res)
    assert res["world"] == 1 and res["backend"] == "nccl"
    assert res["grad_numel"] > 0
    assert res["allreduce_rel_err"] == 0.0
    assert res["param_max_diff_after_update"] == 0.0


def test_rccl_world_size_one_timed_line():
    """The timed N>1 step path at world size 1 over RCCL (no launcher: bench.py forms a one-rank group on
    127.0.0.1 itself): one JSON line whose config names the nccl collective."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "SNNFLOW_SHARE_GPU")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cpu-baseline",
           "--force-dist"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:]
    res = json.loads(lines[-1])
    print("\n[rccl world 1 timed]", res["value"], res["ms_per_step"], res["config"]["collective"])
    assert res["n_gpus"] == 1 and res["value"] > 0 and res["config"]["collective"] == "nccl"
