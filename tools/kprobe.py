"""Per-kernel-class timing of one eager train step, for a given libsnnflow build.

    SNNFLOW_LIB=snn_event-based_optical_flow_amd/snnflow/libsnnflow_probe3.so python tools/kprobe.py

Prints one JSON line {lib, kernels: {class: avg_us}}.  Used with the SNNFLOW_PROBE
variants (csrc/Makefile `probe` target) to attribute kernel time to stages; the
numbers of a probe build are timings only (its results are wrong by design)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "snn_event-based_optical_flow_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    import snnflow
    from snnflow import _lib
    from snnflow.synthetic import make_window

    C, R, B, T, N = 8, 128, 8, 10, 1000
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    from snnflow.parser import train_snn_model_kwargs
    kw = train_snn_model_kwargs(base_num_channels=C)
    model = snnflow.LIFFireNet(kw).to(dev).train()
    cfg = {"loader": {"resolution": [R, R]}, "loss": {"flow_regul_weight": 0.001, "overwrite_intermediate": False},
           "model": {"mask_output": True}}
    loss_fn = snnflow.EventWarping(cfg, dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, N, R, R, gen, dev) for _ in range(T)]
    rec = {i for i, (_, r) in enumerate(model.layer_spec) if r}

    def step():
        loss_fn.reset()
        for w in wins:
            out = model(w["event_voxel"], w["event_cnt"])
            loss_fn.event_flow_association(out["flow"], w["event_list"], w["event_list_pol_mask"], w["event_mask"])
        loss = loss_fn()
        model.zero_grad(set_to_none=True)
        loss.backward()
        model.detach_states()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    agg = {}
    for _ in range(3):
        _lib.TIMER = _lib.KernelTimer()
        torch.cuda._sleep(100_000_000)  # host runs ahead: events bracket kernels only
        step()
        for name, v in _lib.TIMER.summary().items():
            k = bench.classify(name, rec)
            n, tot = agg.get(k, (0, 0.0))
            agg[k] = (n + v["launches"], tot + v["total_ms"])
        _lib.TIMER = None
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH),
                      "kernels": {k: round(1000 * t / n, 2) for k, (n, t) in sorted(agg.items())}}))


if __name__ == "__main__":
    main()
