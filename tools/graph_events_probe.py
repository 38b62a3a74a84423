"""Graph capture of a wavefront of tasks on 4 side streams ordered by per-task events (the pattern of
engine._SlotStreams), with device sleeps as tasks.  argv[1]: 'events' (record per task, wait_event on
the readers), 'waitstream' (reader waits on the whole writer stream), 'keep' (events kept alive)."""
import sys

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "events"
dev = torch.device("cuda", 0)
ss = [torch.cuda.Stream(dev) for _ in range(4)]
KEEP = []


def wave(T=4, K=8):
    main = torch.cuda.current_stream(dev)
    for st in ss:
        st.wait_stream(main)
    done = {}
    stream = lambda k: ss[(k // 2) % 4]
    for d in range(K + 2 * (T - 1)):
        for k in range(K):
            if (d - k) % 2 or not 0 <= (d - k) // 2 < T:
                continue
            t = (d - k) // 2
            st = stream(k)
            for dk, dt in ((k - 1, t), (k, t - 1), (k + 1, t - 1)):
                if 0 <= dk < K and dt >= 0 and stream(dk) is not st:
                    if mode == "waitstream":
                        st.wait_stream(stream(dk))
                    else:
                        st.wait_event(done[(dk, dt)])
            with torch.cuda.stream(st):
                torch.cuda._sleep(1000)
            # "needed": record only the events some task on another stream will wait for
            readers = [(k + 1, t), (k, t + 1), (k - 1, t + 1)]
            if mode != "needed" or any(0 <= rk < K and rt < T and stream(rk) is not st for rk, rt in readers):
                ev = torch.cuda.Event()
                ev.record(st)
                done[(k, t)] = ev
                if mode in ("keep", "needed"):
                    KEEP.append(ev)
    for st in ss:
        main.wait_stream(st)


side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    wave()
torch.cuda.synchronize(dev)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    wave()
g.replay()
torch.cuda.synchronize(dev)
print(mode, "ok")
