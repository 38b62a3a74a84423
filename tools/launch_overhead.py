"""Per-kernel fixed cost of back-to-back dependent launches in a HIP graph on this GPU.

Captures N launches of (a) a 1-element add, (b) a 4 MiB copy, (c) a 16 MiB copy into one
torch.cuda graph, replays it and prints the average time per launch.  Used to size the
launch-count budget of the fused time step."""
import json
import time

import torch


def per_launch(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / (reps * n)


def main():
    x = torch.zeros(1, device="cuda")
    a4, b4 = torch.zeros(1 << 20, device="cuda"), torch.zeros(1 << 20, device="cuda")
    a16, b16 = torch.zeros(1 << 22, device="cuda"), torch.zeros(1 << 22, device="cuda")
    out = {
        "tiny_add_us": per_launch(lambda: x.add_(1.0)),
        "copy_4MiB_us": per_launch(lambda: b4.copy_(a4)),
        "copy_16MiB_us": per_launch(lambda: b16.copy_(a16)),
    }
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()


def branches():
    """Do independent branches of a captured graph (two streams, fork/join) run
    concurrently?  Two chains of n dependent 4 MiB copies, serial vs forked."""
    n = 100
    bufs = [torch.zeros(1 << 20, device="cuda") for _ in range(4)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def chain(a, b):
        for _ in range(n // 2):
            b.copy_(a)
            a.copy_(b)

    def serial():
        chain(bufs[0], bufs[1])
        chain(bufs[2], bufs[3])

    def forked():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            chain(bufs[0], bufs[1])
        with torch.cuda.stream(s2):
            chain(bufs[2], bufs[3])
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    res = {}
    for name, fn in (("serial", serial), ("forked", forked)):
        g = torch.cuda.CUDAGraph()
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        res[name + "_graph_us_per_pair"] = round(1e6 * (time.perf_counter() - t0) / (20 * n), 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        res[name + "_eager_us_per_pair"] = round(1e6 * (time.perf_counter() - t0) / (20 * n), 2)
    print(json.dumps(res))


if __name__ == "__main__" and True:
    branches()
