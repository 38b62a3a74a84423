"""Host-side cost of the eager drop-in loop: T model() calls per train step (train_flow.py:231-279,
no HIP graph), timed per step and profiled with cProfile (top entries by cumulative time).

    python tools/host_profile.py [steps] [--seq]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

import snnflow  # noqa: E402
import snnflow.dp  # noqa: E402,F401
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def main(steps=10, seq=False, C=8, R=128, B=8, T=10):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4, fused=True)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]

    def step():
        lf.reset()
        if seq:
            outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        else:
            outs = [model(w["event_voxel"], w["event_cnt"]) for w in wins]
        for w, out in zip(wins, outs):
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        lf().backward()
        snnflow.dp.clip_grad_norm_(list(model.parameters()), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        model.detach_states()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"eager {'sequence' if seq else 'per-step'}: {1e3 * dt:.3f} ms/step, {B * T * 1000 / dt / 1e6:.2f} M events/s")
    if "--noprof" in sys.argv:
        return
    # the backward Functions run on autograd's device thread: profile with it run inline
    torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    torch.autograd.set_multithreading_enabled(True)
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(35)
    st.sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(int(args[0]) if args else 10, "--seq" in sys.argv)
