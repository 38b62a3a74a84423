"""Diagnostics of the persistent forward (snnflow_fwd_seq) against the slot launches: XCC ids of a
512-thread grid, then per (step, layer) the largest state difference of one window."""
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402


def main():
    import snnflow
    from oracle import lif_ref
    from snnflow import _lib
    from snnflow.synthetic import make_window

    dev = torch.device("cuda:0")
    out = torch.zeros(64, dtype=torch.int32, device=dev)
    _lib.lib.snnflow_debug_xcc(out.data_ptr(), 64, _lib.stream_ptr(dev))
    print("xcc ids of blocks 0..63:", out.cpu().tolist())
    B, H, W, T = 8, 32, 32, 3
    torch.manual_seed(21)
    ma = snnflow.LIFFireNet(lif_ref.make_unet_kwargs(base_num_channels=8)).to(dev).train()
    mb = copy.deepcopy(ma)
    gen = torch.Generator(device=dev).manual_seed(22)
    wins = [make_window(B, 500, H, W, gen, dev) for _ in range(T)]
    sts = {}
    for tag, m, flag in (("seq", ma, "1"), ("slots", mb, "0")):
        os.environ["SNNFLOW_SEQ"] = flag
        m.engine.capture_states = True
        with torch.no_grad():
            m.forward_sequence([w["event_voxel"] for w in wins], [w["event_cnt"] for w in wins])
        torch.cuda.synchronize()
        sts[tag] = [[s.detach().cpu() for s in st] for st in m.engine.seq_states]
        ys, stats, facc = m.engine.seq_debug
        sts[tag + "_dbg"] = (ys.cpu(), stats.cpu(), facc.cpu())
        if flag == "1":
            print("sync words:", m.engine.last_seq_work[:64].view(torch.int32).cpu().tolist()[:16])
    ya, sa, fa = sts["seq_dbg"]
    yb, sb, fb = sts["slots_dbg"]
    for t in range(T):
        print(f"t={t}: ys max|d| per layer", [f"{float((ya[t, l] - yb[t, l]).abs().max()):.2e}" for l in range(ya.shape[1])])
        print(f"      stats max|d|", [f"{float((sa[t, l] - sb[t, l]).abs().max()):.2e}" for l in range(sa.shape[1])])
        print(f"      facc sum seq/slots", [f"{float(fa[t, l].sum()):.4e}/{float(fb[t, l].sum()):.4e}" for l in range(2)])
        print(f"      ys[0] per image", [f"{float((ya[t, 0, i] - yb[t, 0, i]).abs().max()):.1e}" for i in range(ya.shape[2])])
    for t in range(T):
        row = []
        for l in range(len(sts["seq"][t])):
            a, b = sts["seq"][t][l], sts["slots"][t][l]
            row.append(f"{float((a - b).abs().max()):.2e}")
        print(f"t={t}: state max|d| per layer", row)
        # per image of the last layer
        a, b = sts["seq"][t][-1], sts["slots"][t][-1]
        print("   per image:", [f"{float((a[:, i] - b[:, i]).abs().max()):.1e}" for i in range(B)])


if __name__ == "__main__":
    main()
