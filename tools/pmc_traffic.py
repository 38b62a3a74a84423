"""HBM traffic per launch from rocprofv3 --pmc passes (tools/pmc.sh) -> profiles/pmc_traffic.json.

    python tools/pmc_traffic.py gpurun_out/pmc [C8_R128_B8]

Bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KB as reported x 1024): on gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads and WRITE_SIZE is
exact for 16-B stores (MI355X_MICROARCH.md §HBM).  Averaged per kernel class (the
classes bench.py reports), each counter from its own pass.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_class(name):
    m = re.search(r"k_(conv_fwd|layer_bwd)<(\d+), (\d+), (true|false), (true|false)(, \d+)?>", name)
    if m:
        kind, cin, rec = m.group(1), int(m.group(2)), m.group(5) == "true"
        lif_in = m.group(4) == "true"
        if not lif_in and not rec:
            return f"{kind}[0]" if kind == "conv_fwd" else "layer_bwd_head"
        return f"{kind}_rec" if rec else kind
    m = re.search(r"k_(lif_fwd|lif_bwd)<", name)
    if m:
        return m.group(1)
    m = re.search(r"k_(\w+)", name)
    return m.group(1) if m else None


def per_kernel(counter_csv, counter):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(counter_csv) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            vals[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = collections.defaultdict(list)
    for kname, disp in vals.items():
        k = kernel_class(kname)
        if k:
            out[k] += list(disp.values())
    return {k: sum(v) / len(v) for k, v in out.items()}


def find(root, counter):
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            head = f.read(1 << 16)
        if counter in head:
            return path
    return None


def all_counters(root):
    """Per-kernel-class averages of every counter found under root (one dict per class)."""
    out = collections.defaultdict(dict)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        names = set()
        with open(path) as f:
            for r in csv.DictReader(f):
                names.add(r["Counter_Name"])
        for n in names:
            for k, v in per_kernel(path, n).items():
                out[k][n] = round(v, 1)
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "pmc")
    key = sys.argv[2] if len(sys.argv) > 2 else "C8_R128_B8"
    fetch = per_kernel(find(root, "FETCH_SIZE"), "FETCH_SIZE")
    write = per_kernel(find(root, "WRITE_SIZE"), "WRITE_SIZE")
    res = {k: int(round(1024 * (2 * fetch[k] + write.get(k, 0.0)))) for k in fetch}
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    d = {}
    if os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
    d[key] = res
    d["_note"] = ("HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE from separate rocprofv3 --pmc passes "
                  "(tools/pmc.sh, tools/pmc_traffic.py); eager tools/prof_step.py steps")
    with open(path, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 3:  # full per-class counter summary for profiles/
        with open(sys.argv[3], "w") as f:
            json.dump({"note": "rocprofv3 --pmc per-dispatch averages per kernel class (tools/pmc.sh passes); "
                               "FETCH_SIZE/WRITE_SIZE in KB as reported", "workload": key,
                       "kernels": all_counters(root)}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
