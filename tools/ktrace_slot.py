"""Phase timeline of a 4-task wavefront launch (forward and backward slot kernels) from the
`make -C csrc trace_slot` build (thread 0 of every block stamps 100 MHz wall-clock times at its
phase boundaries; only launches of >= 1700 blocks stamp, i.e. the 4-task launches of cfg2).

    SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_trace_slot.so python tools/ktrace_slot.py

Prints per block kind: block count, start spread, end spread, median / p90 of every phase and of
the whole block, in microseconds relative to the earliest block start of the launch (all kinds of
one direction share the launch).  Timing only."""
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
         2: ("layer_bwd", ["prologue", "bn_bwd_halo", "dgrad", "lif_bwd+store", "sums", "fused_wgrad"]),
         3: ("layer_bwd_rec", ["prologue", "bn_bwd_halo", "dgrad", "lif_bwd+store", "sums", "fused_wgrad"])}


# the forward tile pipeline (fwd_lif8_pipe, 2 tiles per block) stamps per tile; whether it runs
# follows the library's default / SNNFLOW_PIPE_FWD (0 = one tile per block)
if os.environ.get("SNNFLOW_PIPE_FWD", "2") != "0":
    _P = ["gather", "coef", "frag+zero", "wait0", "lif0", "conv0", "wait1", "lif1", "conv1"]
    KINDS[0] = ("pipe_fwd", _P)
    KINDS[1] = ("pipe_fwd_rec", _P)


def residency(rows, t0, step_us=1.0):
    """Blocks resident (started, not finished) at each step_us of the launch, over the traced kinds."""
    st = np.concatenate([(t[:, 0] - t0) * 0.01 for t, _ in rows.values()])
    en = np.concatenate([(t[:, -1] - t0) * 0.01 for t, _ in rows.values()])
    grid = np.arange(0.0, float(en.max()) + step_us, step_us)
    return [int(((st <= x) & (en > x)).sum()) for x in grid]


def main(C=8, R=128, B=8, T=10):
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
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    for _ in range(3):
        lf.reset()
        outs = model.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        for w, out in zip(wins, outs):
            lf.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        model.zero_grad(set_to_none=True)
        lf().backward()
        model.detach_states()
    torch.cuda.synchronize()
    buf = np.zeros((4, 4096, 16), dtype=np.uint64)
    fn = _lib.lib.snnflow_trace_copy
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    res = {}
    for direction, kinds in (("fwd", (0, 1)), ("bwd", (2, 3))):
        rows = {}
        for k in kinds:
            name, phases = KINDS[k]
            t = buf[k, :, :len(phases) + 1].astype(np.int64)
            ok = (t > 0).all(axis=1)
            if ok.any():
                rows[name] = (t[ok], phases)
        if not rows:
            continue
        t0 = min(t[:, 0].min() for t, _ in rows.values())
        t1 = max(t[:, -1].max() for t, _ in rows.values())
        out = {"launch_span_us": round(float(t1 - t0) * 0.01, 2), "resident_blocks_per_us": residency(rows, t0)}
        for name, (t, phases) in rows.items():
            rel = (t - t0) * 0.01
            d = np.diff(rel, axis=1)
            tot = rel[:, -1] - rel[:, 0]
            out[name] = {
                "blocks": int(t.shape[0]),
                "start_us_p10_50_90_100": [round(float(np.percentile(rel[:, 0], q)), 2) for q in (10, 50, 90, 100)],
                "end_us_p10_50_90_100": [round(float(np.percentile(rel[:, -1], q)), 2) for q in (10, 50, 90, 100)],
                "block_us_med_p90": [round(float(np.median(tot)), 2), round(float(np.percentile(tot, 90)), 2)],
                "phases_med_p90_us": {p: [round(float(np.median(d[:, i])), 2), round(float(np.percentile(d[:, i], 90)), 2)]
                                      for i, p in enumerate(phases)},
            }
        res[direction] = out
    print(json.dumps({"C": C, "R": R, "B": B, "T": T, "launch": "last 4-task wavefront launch", "kinds": res},
                     indent=1))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
