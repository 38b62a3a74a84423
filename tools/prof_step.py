"""A few eager LIFFireNet train steps of the bench workload (for rocprofv3 --pmc passes)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

import snnflow  # noqa: E402
from snnflow.parser import train_snn_model_kwargs  # noqa: E402
from snnflow.synthetic import make_window  # noqa: E402


def main(C=8, R=128, B=8, T=10, steps=3):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    for _ in range(steps):
        lf.reset()
        if os.environ.get("SNNFLOW_PER_STEP") == "1":
            outs = [model(w["event_voxel"], w["event_cnt"]) for w in wins]
        else:  # as bench.py: wavefront launches
            outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        for w, out in zip(wins, outs):
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        lf().backward()
        opt.step()
        opt.zero_grad()
        model.detach_states()
    # evaluation passes (model.eval() under no_grad: the fused eval_slot launches at C = 8)
    model.eval()
    with torch.no_grad():
        for _ in range(2):
            model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
    torch.cuda.synchronize()


def main_unet(R=256, B=16, T=20, base=32, steps=2):
    """SpikingRecEVFlowNet (cfg5) eager train steps, the bench's unet mode without the graph."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.SpikingRecEVFlowNet(train_snn_model_kwargs("SpikingRecEVFlowNet", base_num_channels=base)).to(dev)
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    for _ in range(steps):
        lf.reset()
        for w in wins:
            out = model(w["event_voxel"], w["event_cnt"])
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        lf().backward()
        opt.step()
        opt.zero_grad()
        model.detach_states()
    torch.cuda.synchronize()


if __name__ == "__main__":
    if sys.argv[1:2] == ["unet"]:
        main_unet(*[int(a) for a in sys.argv[2:]])
    else:
        main(*[int(a) for a in sys.argv[1:]])
