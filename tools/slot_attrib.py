"""Per-task-kind attribution of the C = 8 wavefront slot launches from per-dispatch rocprofv3 data.

    python tools/slot_attrib.py <counter_collection.csv | kernel_trace.csv> [fwd|bwd] [T] > out.json

Every slot launch of a LIFFireNet window holds a known mix of layer-steps (task (k, t) in launch
k + 2t, engine.wavefront_slots), so a per-dispatch quantity -- a PMC counter, or the duration from a
kernel trace -- regressed on the launch's task mix (non-negative least squares) gives each task kind's
marginal share: which layer-step kind carries the LDS bank conflicts, the VALU instructions or the
time.  Dispatches of one pass are taken in order, 2(T-1)+L+1 per pass (LIFFireNet: L = 7 cells, the
recurrent ones G1 = 1 and G2 = 4).

Task kinds, backward (launch d: j + 2 tau = d, j = 0 top, j >= 1 layer L - j, step t = T-1-tau):
  top (pred + LIF backward of layer 6), ff (LIF-fed feed-forward layer with its fused weight
  gradient), rec (recurrent layer, t >= 1: packed dW_ff | dW_rec), rec0 (recurrent layer at t = 0:
  no s_prev), head (layer 0: one block).
Forward (launch d: k + 2t = d): head (conv of the event counts), ff (LIF of layer k-1 + conv k),
rec (the same + the recurrent conv), top (LIF of layer 6 + pred).
"""
import collections
import csv
import json
import sys

import numpy as np
from scipy.optimize import nnls

L, REC = 7, (1, 4)


def mix(direction, T):
    K = L + 1
    kinds = ["top", "ff", "rec", "rec0", "head"] if direction == "bwd" else ["head", "ff", "rec", "top"]
    rows = []
    for d in range(K + 2 * (T - 1)):
        v = dict.fromkeys(kinds, 0)
        for k in range(K):
            if (d - k) % 2 or not 0 <= (d - k) // 2 < T:
                continue
            s = (d - k) // 2
            if direction == "bwd":
                j, t = k, T - 1 - s
                if j == 0:
                    v["top"] += 1
                elif L - j == 0:
                    v["head"] += 1
                elif L - j in REC:
                    v["rec" if t >= 1 else "rec0"] += 1
                else:
                    v["ff"] += 1
            else:
                if k == 0:
                    v["head"] += 1
                elif k == L:
                    v["top"] += 1
                else:
                    v["rec" if k in REC else "ff"] += 1
        rows.append([v[x] for x in kinds])
    return kinds, np.array(rows, dtype=np.float64)


def dispatch_values(path, kname):
    """{quantity: [value per dispatch in dispatch order]} of the kernels whose name contains kname."""
    per = collections.defaultdict(dict)
    with open(path) as f:
        rows = list(csv.DictReader(f))
    if rows and "Counter_Name" in rows[0]:
        for r in rows:
            if kname in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"])
                per[r["Counter_Name"]][d] = per[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
    else:
        for r in rows:
            if kname in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"])
                per["duration_us"][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    return {q: [v[d] for d in sorted(v)] for q, v in per.items()}


def main():
    path = sys.argv[1]
    direction = sys.argv[2] if len(sys.argv) > 2 else "bwd"
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    kinds, A1 = mix(direction, T)
    n = A1.shape[0]
    vals = {}
    for kname in (f"k_{direction}_slot<8>(", f"k_{direction}_slot_t8(", f"k_{direction}_slot_p8("):
        vals = dispatch_values(path, kname)  # (the C = 8 slot kernel the run launched)
        if vals:
            break
    out = {"direction": direction, "T": T, "launches_per_pass": n, "kinds": kinds,
           "tasks_per_launch": A1.tolist(), "quantities": {}}
    for q, v in vals.items():
        m = len(v) // n * n
        if m == 0:
            continue
        y = np.array(v[len(v) - m:])  # whole passes at the end (warm)
        A = np.tile(A1, (m // n, 1))
        A = np.hstack([A, np.ones((m, 1))])  # + a per-launch constant
        coef, res = nnls(A, y)
        mean = y.reshape(-1, n).mean(0)
        out["quantities"][q] = {"per_task": dict(zip(kinds + ["launch"], [round(float(c), 2) for c in coef])),
                                "per_launch_mean": [round(float(x), 1) for x in mean],
                                "pass_total": round(float(mean.sum()), 1),
                                "fit_rel_residual": round(float(res / max(np.linalg.norm(y), 1e-30)), 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
