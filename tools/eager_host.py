"""Host time per phase of the eager per-window train step (bench.py --per-step --no-graph): the
FireNetStep forward / backward bodies (the backward runs on autograd's device thread, which cProfile of
the main thread does not see), the loss calls, the optimizer, timed with perf_counter wrappers.

    python tools/eager_host.py [steps]"""
import collections
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

import snnflow  # noqa: E402
from snnflow import engine, loss as loss_mod  # noqa: E402
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402

ACC = collections.defaultdict(float)
CNT = collections.defaultdict(int)


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[name] += time.perf_counter() - t0
            CNT[name] += 1
    return w


def main(steps=20, C=8, R=128, B=8, T=10):
    engine.FireNetStep.forward = staticmethod(timed("step.forward", engine.FireNetStep.forward))
    engine.FireNetStep.backward = staticmethod(timed("step.backward", engine.FireNetStep.backward))
    engine._chain_backward_batched = timed("chain_backward_batched", engine._chain_backward_batched)
    engine.FireNetEngine.flush_weight_grads = timed("flush_weight_grads", engine.FireNetEngine.flush_weight_grads)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    params = list(model.parameters())
    opt = snnflow.ClipAdam(params, lr=2e-4, max_norm=1.0)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    phases = collections.defaultdict(float)

    def step():
        t = time.perf_counter
        t0 = t()
        opt.zero_grad(set_to_none=True)
        lf.reset()
        t1 = t()
        outs = [model(w["event_voxel"], w["event_cnt"]) for w in wins]
        t2 = t()
        for w, o in zip(wins, outs):
            lf.event_flow_association(o["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = lf()
        t3 = t()
        loss.backward()
        t4 = t()
        opt.step()
        t5 = t()
        model.detach_states()
        t6 = t()
        for k, a, b in (("zero+reset", t0, t1), ("forward x T", t1, t2), ("loss fwd", t2, t3), ("backward", t3, t4),
                        ("clip+adam", t4, t5), ("detach", t5, t6)):
            phases[k] += b - a

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    ACC.clear(); CNT.clear(); phases.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"eager step {1000 * dt / steps:.3f} ms (host phases, per step, us):")
    for k, v in phases.items():
        print(f"  {k:14s} {1e6 * v / steps:8.1f}")
    for k, v in ACC.items():
        print(f"  [{k}] {1e6 * v / CNT[k]:.1f} us per call, {CNT[k] // steps} calls per step")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
