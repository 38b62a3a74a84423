"""cProfile of the eager per-window loop's main-thread host work (model() calls, the loss calls, the
optimizer; the backward body runs on autograd's device thread and is not seen here -- see
eager_host.py).  Prints the top functions by total (self) time per step.

    python tools/eager_prof.py [steps] [top]"""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

import snnflow  # noqa: E402
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def main(steps=20, top=45, C=8, R=128, B=8, T=10):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = snnflow.ClipAdam(list(model.parameters()), lr=2e-4, max_norm=1.0)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]

    def step():
        opt.zero_grad(set_to_none=True)
        lf.reset()
        outs = [model(w["event_voxel"], w["event_cnt"]) for w in wins]
        for w, o in zip(wins, outs):
            lf.event_flow_association(o["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = lf()
        loss.backward()
        opt.step()
        model.detach_states()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    rows = []
    for (fn, line, name), (cc, nc, tt, ct, _) in st.stats.items():
        rows.append((tt, ct, nc, f"{os.path.basename(fn)}:{line}:{name}"))
    rows.sort(reverse=True)
    print(f"per step ({steps} steps, cProfile on): self us, cumulative us, calls per step, function")
    for tt, ct, nc, n in rows[:top]:
        print(f"{1e6 * tt / steps:9.1f} {1e6 * ct / steps:9.1f} {nc / steps:7.1f}  {n}")
    print("\nby cumulative:")
    rows.sort(key=lambda r: -r[1])
    for tt, ct, nc, n in rows[:top]:
        print(f"{1e6 * tt / steps:9.1f} {1e6 * ct / steps:9.1f} {nc / steps:7.1f}  {n}")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
