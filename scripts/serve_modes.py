"""Profiling: the c4 serving leg (64 producers, 50 and 20 µs windows) under the batcher's
wake / sync / zero-copy modes (authjx_debug_batcher_modes), with the per-stage means of
authjx_debug_batcher_profile, results checked against one batch evaluation.
Usage: python scripts/serve_modes.py [wake,sync,zcopy ...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import runtime, workloads  # noqa: E402


def main():
    ctx = runtime.Context(0)
    n = int(os.environ.get("SERVE_N", "65536"))
    w = workloads.make("c4", n=n)
    rss = [ctx.compile_expression(e) for e in w.sets]
    tri, _, _ = ctx.eval_host_arena(rss, w.arena, w.offs, w.lens, set_of_req=w.set_of_req)
    modes = [tuple(int(x) for x in m.split(",")) for m in (sys.argv[1:] or ["0,0,0", "1,0,0", "0,1,0", "0,0,1", "1,1,1"])]
    for m in modes:
        cfgs = os.environ.get("SERVE_CONFIGS", "64:50,64:20,256:200")
        for threads, window_us in [tuple(int(x) for x in c.split(":")) for c in cfgs.split(",")]:
            b = runtime.Batcher(ctx, max_batch=8192, window_us=window_us, modes=m)
            try:
                b.loadgen(rss, w.set_of_req[:4096], w.arena, w.offs[:4096], w.lens[:4096], threads=threads)
                p0 = b.profile()
                lat, stri, wall = b.loadgen(rss, w.set_of_req, w.arena, w.offs, w.lens, threads=threads)
                p1 = b.profile()
            finally:
                b.close()
            nb = max(p1["batches"] - p0["batches"], 1)
            nr = max(p1["requests"] - p0["requests"], 1)
            prof = {k: round((p1[k] * (p1["requests"] if k in ("wait_us", "resume_us") else p1["batches"])
                              - p0[k] * (p0["requests"] if k in ("wait_us", "resume_us") else p0["batches"]))
                             / (nr if k in ("wait_us", "resume_us") else nb), 1)
                    for k in ("wait_us", "resume_us", "eval_us", "wake_us", "pack_us", "launch_us", "sync_us")}
            us = np.sort(lat.astype(np.float64) / 1e3)
            eq = bool(np.array_equal(stri.reshape(n, -1)[:, 0], tri.reshape(n, -1)[:, 0].astype(np.uint8)))
            print(json.dumps({"modes": m, "producers": threads, "window_us": window_us, "p50_us": round(us[n // 2], 1),
                              "p99_us": round(us[int(n * 0.99)], 1), "decisions_per_s": round(n / (wall * 1e-9)),
                              "batches": nb, "req_per_batch": round(nr / nb, 1), "equal": eq, **prof}), flush=True)


if __name__ == "__main__":
    main()
