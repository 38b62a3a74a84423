"""Debug: per-parameter gradient differences between the backward tile pipeline and the one-tile bodies."""
import copy
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import snnflow  # noqa: E402
from oracle import lif_ref  # noqa: E402
from snnflow import _lib  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def main(tb=int(os.environ.get("TB", "2")), T=int(os.environ.get("T", "5")), B=8, H=32, W=32):
    dev = torch.device("cuda:0")
    torch.manual_seed(21)
    kw = lif_ref.make_unet_kwargs(base_num_channels=8)
    ma = snnflow.LIFFireNet(dict(kw)).to(dev).train()
    mb = copy.deepcopy(ma)
    if os.environ.get("FUSE") == "0":
        ma.engine.fuse_wgrad = mb.engine.fuse_wgrad = False
    gen = torch.Generator(device=dev).manual_seed(22)
    wins = [make_window(B, 500, H, W, gen, dev) for _ in range(T)]
    for m, bwd in ((ma, tb), (mb, 0)):
        _lib.lib.snnflow_set_pipe(0, bwd)
        outs = m.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        loss = sum(((o["flow"][0] * (t + 1)) ** 2).sum() for t, o in enumerate(outs))
        loss.backward()
        torch.cuda.synchronize()
    print(f"TB={tb} T={T} CAP={os.environ.get('SNNFLOW_SLOT_CAP', '0')} FUSE={os.environ.get('FUSE', '1')}")
    for (n, a), (_, b) in zip(ma.named_parameters(), mb.named_parameters()):
        if "lif.beta" in n or "bn.bias" in n:
            continue
        print(f"{n:28s} {rel(a.grad.cpu().numpy(), b.grad.cpu().numpy()):.3e}  |ref| {float(b.grad.norm()):.3e}")


if __name__ == "__main__":
    main()
