"""Median per-dispatch value of each counter, per kernel, from rocprofv3 counter CSVs:
python scripts/pmc_summary.py gpurun_out/pmcm_*"""
import collections
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"].split("(")[0][:60], r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
        print("==", f)
        for (k, c), v in sorted(per.items()):
            if max(v.values()) > 0:
                print(f"  {k:60s} {c:14s} n={len(v):3d} median={statistics.median(v.values()):.4g}")
