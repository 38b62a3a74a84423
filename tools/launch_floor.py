"""Per-kernel floor of a dependent chain under hipGraph replay: N tiny kernels (one-element
add_) captured in one graph, replayed; host wall time / N.  Also a chain of N snnflow
prep_weights launches (our smallest C-ABI kernel)."""
import json
import time

import torch


def main(N=200, reps=20):
    x = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N):
            x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    big = torch.zeros(8 * 128 * 128 * 8, device="cuda")
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        for _ in range(N):
            big.add_(1.0)
    g2.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g2.replay()
    torch.cuda.synchronize()
    dt2 = (time.perf_counter() - t0) / reps
    print(json.dumps({"tiny_us_per_kernel": round(1e6 * dt / N, 2),
                      "4MB_add_us_per_kernel": round(1e6 * dt2 / N, 2), "N": N}))


if __name__ == "__main__":
    main()
