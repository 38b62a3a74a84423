"""Does a HIP graph captured from two forked streams run its independent branches concurrently?
Two device sleeps on two streams inside one graph: replay time ~1x a sleep => concurrent, ~2x => serial.
Also the same eagerly (no graph)."""
import time

import torch

dev = torch.device("cuda", 0)
N = 20_000_000  # ~ cycles of one sleep
main = torch.cuda.current_stream(dev)


def branches():
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s1.wait_stream(torch.cuda.current_stream(dev))
    s2.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s1):
        torch.cuda._sleep(N)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(N)
    torch.cuda.current_stream(dev).wait_stream(s1)
    torch.cuda.current_stream(dev).wait_stream(s2)


def timed(fn, reps=5):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps * 1e3


timed(lambda: torch.cuda._sleep(N))  # warm-up
timed(branches)
one = timed(lambda: torch.cuda._sleep(N))
eager = timed(branches)
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream(dev)
side.wait_stream(main)
with torch.cuda.stream(side):
    branches()
torch.cuda.synchronize(dev)
with torch.cuda.graph(g):
    branches()
graph = timed(g.replay)
print(f"one sleep {one:.3f} ms; two streams eager {eager:.3f} ms; two-branch graph {graph:.3f} ms "
      f"-> graph branches {'concurrent' if graph < 1.5 * one else 'serialised'}")
