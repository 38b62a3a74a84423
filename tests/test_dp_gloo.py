"""Data-parallel path on CPU: world_size-2 gloo process group.

Covers the sharding helpers, the flat-buffer detection used for the engine's
gradient layout, the single-bucket SUM all-reduce (flat and packed paths) and the
clip helper against torch.nn.utils.clip_grad_norm_.  The GPU ranks run the same
code over RCCL (bench.py under torch.distributed.run)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from snnflow import dp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _params(rank, flat_layout):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(8, 2, 3, 3)), torch.nn.Parameter(torch.randn(8)),
          torch.nn.Parameter(torch.randn(2, 8, 1, 1))]
    g = torch.Generator().manual_seed(100 + rank)
    vals = [torch.randn(p.shape, generator=g) for p in ps]
    if flat_layout:
        flat = torch.cat([v.reshape(-1) for v in vals])
        off = 0
        for p in ps:
            p.grad = flat[off:off + p.numel()].view(p.shape)
            off += p.numel()
    else:
        for p, v in zip(ps, vals):
            p.grad = v.clone()
    return ps, vals


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        for flat_layout in (True, False):
            ps, _ = _params(rank, flat_layout)
            assert (dp.flat_grad_buffer(ps) is not None) == flat_layout
            dp.GradAllReduce(ps)()
            expect = [sum(_params(r, False)[1][i] for r in range(world)) for i in range(len(ps))]
            out[flat_layout] = max(float((p.grad - e).abs().max()) for p, e in zip(ps, expect))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in res:
        assert out[True] < 1e-6 and out[False] < 1e-6, (rank, out)


def test_shard_slots_partition():
    slots = [list(dp.shard_slots(64, r, 8)) for r in range(8)]
    assert sum(slots, []) == list(range(64))
    assert all(len(s) == 8 for s in slots)
    with pytest.raises(ValueError):
        dp.shard_slots(10, 0, 4)
    assert len({dp.stream_seed(1, r) for r in range(8)}) == 8


def test_flat_buffer_detection_any_order_rejects_gaps_and_overlaps():
    """The engine's flat buffer follows its own parameter order, not the module's
    registration order: any order that tiles one range exactly is accepted."""
    flat = torch.arange(10.0)
    a, b = torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(4))
    a.grad, b.grad = flat[0:4], flat[4:8]
    f = dp.flat_grad_buffer([a, b])
    assert f is not None and f.numel() == 8 and f.data_ptr() == flat.data_ptr()
    assert dp.flat_grad_buffer([b, a]) is not None
    b.grad = flat[5:9]   # gap
    assert dp.flat_grad_buffer([a, b]) is None
    b.grad = flat[3:7]   # overlap
    assert dp.flat_grad_buffer([a, b]) is None
    b.grad = torch.zeros(4)  # other storage
    assert dp.flat_grad_buffer([a, b]) is None


@pytest.mark.parametrize("flat_layout", [True, False])
def test_clip_matches_torch(flat_layout):
    ps, _ = _params(0, flat_layout)
    ref, _ = _params(0, False)
    for p in ps + ref:
        p.grad.mul_(3.0)
    n1 = dp.clip_grad_norm_(ps, 1.0)
    n2 = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    assert abs(float(n1) - float(n2)) <= 1e-5 * float(n2)
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.grad, r.grad, rtol=1e-5, atol=1e-7)


def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_backend_resolution():
    """`bench.py --gpus N` without --dist-backend runs RCCL ("nccl") when a GPU is visible, gloo on a
    CPU-only host or when ranks share one GPU (SNNFLOW_SHARE_GPU=1); an explicit choice wins."""
    b = _bench()
    assert b.resolve_backend(None, 8, False) == "nccl"
    assert b.resolve_backend(None, 1, False) == "nccl"
    assert b.resolve_backend(None, 0, False) == "gloo"
    assert b.resolve_backend(None, 1, True) == "gloo"
    assert b.resolve_backend("gloo", 8, False) == "gloo"
    assert b.resolve_backend("nccl", 1, True) == "nccl"


def test_bench_gpus_flag_spawns_ranks(monkeypatch):
    """A plain `bench.py --gpus 2` (no WORLD_SIZE) starts its two ranks itself as children through
    torch.distributed.run on 127.0.0.1 with the same arguments, and exits with their exit code;
    the parent does no GPU work (the launch is intercepted here before any rank would start)."""
    import subprocess
    import sys as _sys
    b = _bench()
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(_sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        b.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "2"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def _bn_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Conv2d(2, 4, 3), torch.nn.BatchNorm2d(4), torch.nn.BatchNorm2d(4))
        model.train()
        torch.manual_seed(10 + rank)  # rank-local batches: rank-local running statistics
        for _ in range(3 + rank):
            model(torch.randn(2, 2, 8, 8))
        before = [b.clone() for b in dp.bn_buffers(model)]
        dp.broadcast_bn_stats(model, src=0)
        after = [b.clone() for b in dp.bn_buffers(model)]
        q.put((rank, [b.tolist() for b in before], [b.tolist() for b in after]))
    finally:
        dist.destroy_process_group()


def test_broadcast_bn_stats_gloo_world2():
    """dp.broadcast_bn_stats: after the broadcast every rank holds rank 0's running mean / var and
    num_batches_tracked (which differed before: rank-local batches and step counts)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bn_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (b, a)) for r, b, a in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] != res[1][0]  # rank-local before
    assert res[1][1] == res[0][0] and res[0][1] == res[0][0]  # rank 0's everywhere after
