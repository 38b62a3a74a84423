"""Forward-window timing: forward_sequence of the bench window (cfg2) with the persistent dataflow
kernel (SNNFLOW_SEQ=1) and the wavefront slot launches (0); ms per window, no autograd."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "snn_event-based_optical_flow_amd")]
import torch  # noqa: E402


def main():
    import snnflow
    from snnflow.parser import train_snn_model_kwargs
    from snnflow.synthetic import make_window

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, R, T = 8, 128, 10
    model = snnflow.LIFFireNet(train_snn_model_kwargs(base_num_channels=8)).to(dev).train()
    gen = torch.Generator(device=dev).manual_seed(1)
    wins = [make_window(B, 1000, R, R, gen, dev) for _ in range(T)]
    xs = [w["event_cnt"] for w in wins]
    for flag in ("0", "1", "0", "1"):
        os.environ["SNNFLOW_SEQ"] = flag
        with torch.no_grad():
            for _ in range(3):
                model.forward_sequence(xs, xs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 20
            for _ in range(n):
                model.forward_sequence(xs, xs)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        err = None
        if flag == "1":
            w = model.engine.last_seq_work[:128]
            err = int(w.view(torch.int32)[8].item())
            st = w[40:72].view(torch.int64).tolist()
            print(f"  last launch: blocks {st[2]}, items {st[3]}, mean per block: wait {st[0] / max(st[2], 1) / 100:.1f} us, "
                  f"items {st[1] / max(st[2], 1) / 100:.1f} us; per item {st[1] / max(st[3], 1) / 100:.2f} us")
        print(f"SNNFLOW_SEQ={flag}: {ms:.3f} ms per forward window" + (f" (timeout flag {err})" if err is not None else ""))


if __name__ == "__main__":
    main()
