"""Loss forward + backward at cfg2 shapes on fixed inputs: writes the loss and dL/dflow to an .npz
(compare two library builds bit for bit: SNNFLOW_LIB=<other .so> python tools/loss_bits.py out.npz)
and prints the backward's average time over repeated calls (HIP events).

    python tools/loss_bits.py OUT.npz [R] [B] [T]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import snnflow  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def main(out, R=128, B=8, T=10):
    dev = torch.device("cuda:0")
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    torch.manual_seed(3)
    flows = [(0.2 * torch.tanh(torch.randn(B, 2, R, R, device=dev))).requires_grad_() for _ in range(T)]

    def run():
        lf.reset()
        for w, f in zip(wins, flows):
            lf.event_flow_association([f], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = lf()
        g = torch.autograd.grad(loss, flows)
        return loss, g

    loss, g = run()
    np.savez(out, loss=loss.detach().cpu().numpy(), g=torch.stack(g).cpu().numpy())
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    a.record()
    for _ in range(n):
        run()
    b.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('SNNFLOW_LIB', 'libsnnflow.so')}: loss {loss.item():.9g}, "
          f"loss fwd+bwd {1000 * a.elapsed_time(b) / n:.1f} us per call (host included)")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:5]))
