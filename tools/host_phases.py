"""Host time per phase of the eager drop-in train step (train_flow.py:231-279): the T model() calls,
the loss association + value, backward, clip, Adam -- wall-clock on the host without synchronising
(the GPU runs behind; when the host is the bound these add up to the step).

    python tools/host_phases.py [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

import snnflow  # noqa: E402
import snnflow.dp  # noqa: E402,F401
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def main(steps=30, C=8, R=128, B=8, T=10):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4, fused=True)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    ph = {k: 0.0 for k in ("forward", "assoc", "loss", "backward", "clip", "adam", "detach")}

    def step(acc):
        tt = time.perf_counter
        t0 = tt()
        lf.reset()
        outs = [model(w["event_voxel"], w["event_cnt"]) for w in wins]
        t1 = tt()
        for w, out in zip(wins, outs):
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        t2 = tt()
        loss = lf()
        t3 = tt()
        loss.backward()
        t4 = tt()
        snnflow.dp.clip_grad_norm_(list(model.parameters()), 1.0)
        t5 = tt()
        opt.step()
        opt.zero_grad(set_to_none=True)
        t6 = tt()
        model.detach_states()
        t7 = tt()
        if acc:
            for k, a, b in (("forward", t0, t1), ("assoc", t1, t2), ("loss", t2, t3), ("backward", t3, t4),
                            ("clip", t4, t5), ("adam", t5, t6), ("detach", t6, t7)):
                ph[k] += b - a

    for _ in range(5):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    host = (time.perf_counter() - t0) / steps
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    print(f"eager per-step: wall {1e3 * wall:.3f} ms/step, host issue {1e3 * host:.3f} ms/step")
    for k, v in ph.items():
        print(f"  {k:9s} {1e3 * v / steps:7.3f} ms")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
