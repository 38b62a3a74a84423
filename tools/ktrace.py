"""Phase timeline of the C x C layer kernels from a SNNFLOW_TRACE build (`make -C csrc trace`).

    SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace.so python tools/ktrace.py [C R B]

Runs eager train steps of the bench workload; thread 0 of every block of the last launch
of each traced kernel kind left 100 MHz wall-clock stamps at its phase boundaries.  Prints,
per kind, the dispatch spread of block starts and the median / p90 of every phase, all
in microseconds relative to the earliest block start of that launch.  Timing only."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402

KINDS = {0: ("conv_fwd", ["prologue", "lif_halo", "conv", "store+sums"]),
         1: ("conv_fwd_rec", ["prologue", "lif_halo", "conv", "store+sums"]),
         2: ("layer_bwd", ["prologue", "bn_bwd_halo", "dgrad", "lif_bwd+store", "sums"]),
         3: ("layer_bwd_rec", ["prologue", "bn_bwd_halo", "dgrad", "lif_bwd+store", "sums"])}


def main(C=8, R=128, B=8):
    import snnflow
    from snnflow import _lib
    from snnflow.parser import train_snn_model_kwargs
    from snnflow.synthetic import make_window

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=C)).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    lf = snnflow.EventWarping(cfg, dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(10)]
    for _ in range(3):
        lf.reset()
        for w in wins:
            out = model(w["event_voxel"], w["event_cnt"])
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        model.zero_grad(set_to_none=True)
        lf().backward()
        model.detach_states()
    torch.cuda.synchronize()
    buf = np.zeros((4, 4096, 16), dtype=np.uint64)
    fn = _lib.lib.snnflow_trace_copy
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    nblk = _lib.lib.snnflow_conv_blocks(B, R, R)
    res = {}
    for k, (name, phases) in KINDS.items():
        t = buf[k, :nblk, :len(phases) + 1].astype(np.int64)
        if (t == 0).any():
            continue
        t0 = t[:, 0].min()
        rel = (t - t0) * 0.01  # 100 MHz -> us
        d = np.diff(rel, axis=1)
        res[name] = {
            "start_spread_us": [round(float(np.percentile(rel[:, 0], q)), 2) for q in (50, 90, 100)],
            "end_us": [round(float(np.percentile(rel[:, -1], q)), 2) for q in (50, 90, 100)],
            "phases_med_p90_us": {p: [round(float(np.median(d[:, i])), 2), round(float(np.percentile(d[:, i], 90)), 2)]
                                  for i, p in enumerate(phases)},
        }
    print(json.dumps({"C": C, "R": R, "B": B, "blocks": nblk, "kinds": res}, indent=1))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
