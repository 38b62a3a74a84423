"""Debug helper: compare the HIP event-warping intermediates with the oracle."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import snnflow  # noqa: E402
from oracle import iwe_ref  # noqa: E402
from snnflow.loss import EventWarpingFn  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def main(H=40, W=56, B=3, N=500, T=4):
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(3)
    cfg = {"loader": {"resolution": [H, W]}, "loss": {"flow_regul_weight": 0.01, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    ew = snnflow.EventWarping(cfg, dev)
    ref = iwe_ref.EventWarpingRef([H, W], weight=0.01)
    for t in range(T):
        w = make_window(B, N, H, W, gen, dev)
        f = ((torch.rand(B, 2, H, W, generator=gen, device=dev) - 0.5) * 0.1).requires_grad_(True)
        ew.event_flow_association([f], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        ref.event_flow_association([f.detach().cpu()], w["event_list"].cpu(), w["event_list_pol_mask"].cpu(),
                                   w["event_mask"].cpu())
    loss = ew()
    node = loss.grad_fn
    images = node.saved_tensors[4].view(2, 4, B, H * W).cpu()
    persample = node.saved_tensors[5].view(2, B, 4).cpu()
    smooth = node.saved_tensors[6].cpu()
    events = torch.cat(ref.events, 1)
    flow_ev = torch.cat(ref.flows_ev, 1)
    pol4 = torch.cat([torch.cat(ref.pols, 1)] * 4, 1)
    ts4 = torch.cat([events[:, :, 0:1]] * 4, 1)
    for d, (tref, tsw) in enumerate(((T, ts4), (0, T - ts4))):
        idx, wt = iwe_ref.get_interpolation_t(events, flow_ev, tref, [H, W], max(H, W))
        imgs = [iwe_ref.interpolate_t(idx, wt, [H, W], pol4[:, :, 0:1]),
                iwe_ref.interpolate_t(idx, wt, [H, W], pol4[:, :, 1:2]),
                iwe_ref.interpolate_t(idx, wt * tsw, [H, W], pol4[:, :, 0:1]),
                iwe_ref.interpolate_t(idx, wt * tsw, [H, W], pol4[:, :, 1:2])]
        for k in range(4):
            r = imgs[k].reshape(B, H * W)
            o = images[d, k]
            print(f"dir {d} img {k}: max|diff| {float((r - o).abs().max()):.3e}  sum ref {float(r.sum()):.4f} ours {float(o.sum()):.4f}")
    print("persample", persample)
    print("smooth", smooth)
    print("loss ours", loss.item(), "oracle", ref().item())


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
