"""Which torch ops of a cfg5-shape U-Net train step launch device work outside the HIP library
(fills, copies, elementwise): one eager steady-state step (256^2, B=16, 2 windows) under a
TorchDispatchMode that records each such op with its bytes and the snnflow call site."""
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import snnflow  # noqa: E402
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.defaultdict(lambda: [0, 0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        if name in ("empty", "empty_strided", "as_strided", "view", "_unsafe_view", "detach", "t", "permute",
                    "select", "slice", "unsqueeze", "squeeze", "expand", "alias", "set_", "_reshape_alias",
                    "transpose", "split", "unbind", "lift_fresh"):
            return out
        o = out[0] if isinstance(out, (tuple, list)) and out else out
        nb = o.numel() * o.element_size() if isinstance(o, torch.Tensor) else 0
        site = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack()
                if "snnflow" in f.filename or "unet_ops" in f.filename][-3:]
        r = self.rows[(name, " <- ".join(reversed(site)))]
        r[0] += 1
        r[1] += nb
        return out


def main(R=256, B=16, T=2, base=32):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.SpikingRecEVFlowNet(train_snn_model_kwargs("SpikingRecEVFlowNet", base_num_channels=base)).to(dev)
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]

    def step():
        lf.reset()
        for w in wins:
            out = model(w["event_voxel"], w["event_cnt"])
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        lf().backward()
        opt.step()
        opt.zero_grad()
        model.detach_states()

    step()
    torch.cuda.synchronize()
    log = Log()
    with log:
        step()
    torch.cuda.synchronize()
    rows = sorted(log.rows.items(), key=lambda kv: -kv[1][1])
    print(f"{'MB':>9} {'n':>4}  op  call site   (one steady-state step, T={T})")
    for (name, site), (n, nb) in rows[:60]:
        print(f"{nb / 1e6:9.2f} {n:4d}  {name}  {site}")


if __name__ == "__main__":
    main()
