"""FETCH_SIZE calibration for the lean kernel's access shape (per-lane 16-B loads in 64-B
windows, one document per lane): its loads-only ablation (kernel mode 15,
ajx_scan_lean<true, 1>; scripts/prof_modes.py) reads every document's aligned 16-B blocks
exactly once, so exact bytes / FETCH_SIZE is the factor for this shape (MI355X_MICROARCH.md
calibrates only wide coalesced streams, at 2). Merged into pmc_traffic.json as
"calibration"; scripts/pmc_traffic.py applies it.

  python scripts/fetch_calibration.py <fetch_dir> <workload> <n> [out.json] [kernel]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import workloads  # noqa: E402
from pmc_traffic import per_launch  # noqa: E402


def main():
    d, wl, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else "pmc_traffic.json"
    kernel = sys.argv[5] if len(sys.argv) > 5 else "ajx_scan_lean<true, 1>"
    # the documents bench.py builds for this workload (rank 0)
    w = workloads.make(wl, n=n, seed=workloads.DEFAULT_SEEDS.get(wl, 0), unique=4096 if wl == "c5" else 16384,
                       uniquify=True)
    mis = (w.offs & np.uint64(15)).astype(np.int64)  # (the device arena is 256-B aligned)
    exact = int((((w.lens.astype(np.int64) + mis + 15) // 16) * 16).sum())
    fb, nl = per_launch(d, "FETCH_SIZE", kernel)
    res = {"workload": wl, "n": n, "exact_bytes_per_launch": exact, "fetch_bytes_per_launch_raw": fb,
           "launches": nl, "factor": exact / fb if fb else None,
           "kernel": kernel, "note": "loads-only ablation: exact aligned 16-B block bytes / FETCH_SIZE"}
    try:
        with open(out) as f:
            allw = json.load(f)
    except (OSError, ValueError):
        allw = {}
    allw["calibration"] = res
    with open(out, "w") as f:
        json.dump(allw, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
