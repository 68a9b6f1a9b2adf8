"""Print kernel ms / roofline fraction / parity counters of gpurun_out/<dir>/bench_*.log."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/quick"
for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
    for ln in open(f):
        if ln.startswith("{"):
            r = json.loads(ln)
            print(os.path.basename(f), "step %.3f ms  kernel %.3f ms  frac %.4f  undecided %s  exact %s" % (
                r["ms_per_step"], r["roofline"]["kernel_ms"], r["roofline"]["frac"], r.get("undecided"),
                r.get("exact_path_requests")))
