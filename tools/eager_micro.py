"""Host-cost attribution of the eager per-window path (one model() call per window, train_flow.py:
231-279): per-call host time of its building blocks, and forward-only / backward-only loops, each
timed with the GPU kept busy (host issue time) and with a sync after every call (host + GPU).

    python tools/eager_micro.py"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

import snnflow  # noqa: E402
from snnflow import _lib  # noqa: E402
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def per_call(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    return 1e6 * host, 1e6 * wall


def main():
    dev = torch.device("cuda:0")
    B, R, T = 8, 128, 10
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=8)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    x = wins[0]["event_cnt"]
    rows = []
    rows.append(("torch.empty 1 MB", per_call(lambda: torch.empty(262144, device=dev))))
    rows.append(("stream_ptr", per_call(lambda: _lib.stream_ptr(dev))))
    rows.append(("ctypes abi_version", per_call(lambda: _lib.lib.snnflow_abi_version())))
    io = _lib.FireNetFwdIo()
    rows.append(("FireNetFwdIo() + 12 fields", per_call(lambda: [setattr(io, "x", 1) for _ in range(12)])))

    class Nop(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *a):
            return a[1].view_as(a[1])

        @staticmethod
        def backward(ctx, g):
            return (None,) * 10
    st = [torch.zeros(2, B, 8, R, R, device=dev, requires_grad=True) for _ in range(7)]
    rows.append(("autograd.Function.apply, 10 inputs", per_call(lambda: Nop.apply(None, x, *st, x))))

    def fwd_only():
        with torch.no_grad():
            model(None, x)
    rows.append(("model() no_grad", per_call(fwd_only, 100)))
    model.detach_states()

    def fwd_grad():
        model(None, x)
        model.detach_states()
    rows.append(("model() + detach_states", per_call(fwd_grad, 100)))

    def fwd_bwd():
        out = model(None, x)
        out["flow"][0].sum().backward()
        model.detach_states()
    rows.append(("model() + flow.sum().backward() (1 step chain)", per_call(fwd_bwd, 100)))
    for name, (h, w) in rows:
        print(f"{name:48s} host {h:8.1f} us   host+GPU {w:8.1f} us")

    # time inside the C-ABI calls of a whole eager train step (the rest is Python / autograd / torch)
    import collections
    acc = collections.defaultdict(float)
    cnt = collections.Counter()
    orig = _lib.call

    def timed(name, fn, *args, work=None):
        t0 = time.perf_counter()
        orig(name, fn, *args, work=work)
        acc[name.split("[")[0]] += time.perf_counter() - t0
        cnt[name.split("[")[0]] += 1
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4, fused=True)
    import snnflow.dp as sdp

    def step():
        lf.reset()
        outs = [model(w["event_voxel"], w["event_cnt"]) for w in wins]
        for w, out in zip(wins, outs):
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        lf().backward()
        sdp.clip_grad_norm_(list(model.parameters()), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        model.detach_states()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    _lib.call = timed
    import snnflow.engine as E
    E._lib.call = timed
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    _lib.call = orig
    print(f"eager step host {1e3 * host:.3f} ms; inside C-ABI calls per step:")
    tot = 0.0
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        tot += v
        print(f"  {k:24s} {1e6 * v / n:8.1f} us  ({cnt[k] / n:.0f} calls, {1e6 * v / cnt[k]:.1f} us each)")
    print(f"  total C-ABI {1e6 * tot / n:.1f} us of {1e6 * host:.1f} us")


if __name__ == "__main__":
    main()
