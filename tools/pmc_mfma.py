"""Matrix-core utilisation per kernel class from tools/pmc_mfma.sh -> <dir>/pmc_mfma.json (kept as profiles/r02/pmc_mfma.json).

    python tools/pmc_mfma.py gpurun_out/pmc_mfma

mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (SIMD-cycles of the dispatch), the SIMD-cycles being
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) x 256 CUs x 4 SIMDs; the two counters come from
separate passes over the same eager steps, averaged per dispatch of the class.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import REPO, all_counters  # noqa: E402

SIMDS = 256 * 4


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "pmc_mfma")
    res = {}
    for wl in ("c8", "c32", "unet"):
        d = os.path.join(root, wl)
        if not os.path.isdir(d):
            continue
        ks = all_counters(d)
        rows = {}
        for k, c in sorted(ks.items()):
            busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("GRBM_GUI_ACTIVE")
            row = dict(c)
            if busy is not None and gui:
                row["mfma_busy_frac"] = round(busy / (gui / 8 * SIMDS), 4)
            rows[k] = row
        res[wl] = rows
    out = {"note": "rocprofv3 --pmc (tools/pmc_mfma.sh), per-dispatch averages per kernel class; mfma_busy_frac = "
                   "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
           "workloads": {"c8": "LIFFireNet C=8 128^2 B=8 T=10 wavefront (eager)",
                         "c32": "LIFFireNet C=32 128^2 B=8 T=10 wavefront (eager)",
                         "unet": "SpikingRecEVFlowNet base 32, 256^2 B=16 T=20 (eager)"},
           "kernels": res}
    path = os.path.join(root, "pmc_mfma.json")  # copied to profiles/r02/
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for wl, rows in res.items():
        for k, r in rows.items():
            if r.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                print(wl, k, r.get("mfma_busy_frac"))


if __name__ == "__main__":
    main()
