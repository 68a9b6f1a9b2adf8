"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into HBM bytes per
launch of the dominant kernel, merged per workload into pmc_traffic.json at the repo root
(read by bench.py for roofline.traffic; a copy goes to profiles/<round>/).

  python scripts/pmc_traffic.py <fetch_dir> <write_dir> <workload> <n> [out.json] [kernel]

FETCH_SIZE / WRITE_SIZE are reported in KiB. MI355X_MICROARCH.md (HBM/rocprofv3 section):
FETCH_SIZE counts exactly half the bytes of a wide coalesced streaming read on gfx950;
other access widths are uncalibrated. The dominant kernel reads each document with
per-lane 16-byte loads (one document per lane): scripts/fetch_calibration.py measures the
factor for that shape (exact bytes of the loads-only ablation / its FETCH_SIZE), and
`hbm_bytes_per_launch` = FETCH_SIZE x factor + WRITE_SIZE (raw values kept beside it).
"""
import csv
import glob
import json
import statistics
import sys


def per_launch(d, counter, kernel_sub, names=None):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]) * 1024.0)
                if names is not None:
                    names.add(r["Kernel_Name"])
    return statistics.median(vals) if vals else None, len(vals)


def source_commit():
    """The commit the counters were taken on: $AJX_COMMIT (set by the GPU scripts from the
    checkout the box ran), else git's HEAD here."""
    import os
    import subprocess

    c = os.environ.get("AJX_COMMIT")
    if c:
        return c
    try:
        return subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                              check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None


def main():
    fetch_dir, write_dir, workload, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else "pmc_traffic.json"
    kernel = sys.argv[6] if len(sys.argv) > 6 else "ajx_scan_fused"
    names = set()
    fb, nf = per_launch(fetch_dir, "FETCH_SIZE", kernel, names)
    wb, nw = per_launch(write_dir, "WRITE_SIZE", kernel, names)
    try:
        with open(out) as f:
            allw = json.load(f)
        if "workload" in allw:  # (an older single-workload file)
            allw = {allw["workload"]: allw}
    except (OSError, ValueError):
        allw = {}
    # the factor scripts/fetch_calibration.py measured for this access shape (else raw)
    k = (allw.get("calibration") or {}).get("factor")
    res = {
        "workload": workload,
        "n": n,
        "kernel": kernel,
        "kernel_names": sorted(names),
        "commit": source_commit(),
        "fetch_bytes_per_launch_raw": fb,
        "fetch_calibration": k,
        "write_bytes_per_launch": wb,
        "launches": [nf, nw],
        "hbm_bytes_per_launch": (fb or 0) * (k or 1.0) + (wb or 0),
        "note": ("FETCH_SIZE x calibration (loads-only ablation, same shape) + WRITE_SIZE" if k else
                 "FETCH_SIZE+WRITE_SIZE raw (uncalibrated)") + ", KiB*1024, median over launches",
    }
    allw[workload] = res
    with open(out, "w") as f:
        json.dump(allw, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
