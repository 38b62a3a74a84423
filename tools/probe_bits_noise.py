import sys, os, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo/snn_event-based_optical_flow_amd")
import test_gpu_fullsize as T
from snnflow.synthetic import make_window
dev = torch.device("cuda:0")
C, B, H = 32, 8, 128
gen = torch.Generator(device=dev).manual_seed(1)
wins = [make_window(B, 1000, H, H, gen, dev) for _ in range(10)]
runs = {"f1": T._window_run(dev, wins, C, True, bits=False), "f2": T._window_run(dev, wins, C, True, bits=False),
        "b1": T._window_run(dev, wins, C, False, bits=True), "b2": T._window_run(dev, wins, C, False, bits=True),
        "fs": T._window_run(dev, wins, C, False, bits=False)}
names = [n for n, _ in T._new_model(C).named_parameters()]
def cmp(a, b):
    out = []
    for n, x, y in zip(names, runs[a][2], runs[b][2]):
        d = float((x - y).abs().max() / x.abs().max().clamp_min(1e-30))
        if d > 0: out.append((n, d))
    return out
for a, b in [("f1", "f2"), ("b1", "b2"), ("f1", "b1"), ("f1", "fs"), ("fs", "b1")]:
    print(a, b, cmp(a, b)[:8])
