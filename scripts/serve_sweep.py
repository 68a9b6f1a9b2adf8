"""Profiling: the c4 serving leg (bench.py's) over batcher worker counts and windows, with
the results checked against one batch evaluation. Usage: python scripts/serve_sweep.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import runtime, workloads  # noqa: E402


def main():
    ctx = runtime.Context(0)
    n = 65536
    w = workloads.make("c4", n=n)
    rss = [ctx.compile_expression(e) for e in w.sets]
    tri, _, _ = ctx.eval_host_arena(rss, w.arena, w.offs, w.lens, set_of_req=w.set_of_req)
    for workers in [int(x) for x in os.environ.get("SWEEP_WORKERS", "2,3,4").split(",")]:
        for threads, window_us in ((64, 50), (64, 20), (256, 200)):
            b = runtime.Batcher(ctx, max_batch=8192, window_us=window_us, workers=workers)
            try:
                b.loadgen(rss, w.set_of_req[:4096], w.arena, w.offs[:4096], w.lens[:4096], threads=threads)
                b0 = b.stats()["batches"]
                lat, stri, wall = b.loadgen(rss, w.set_of_req, w.arena, w.offs, w.lens, threads=threads)
                st = b.stats()
            finally:
                b.close()
            us = np.sort(lat.astype(np.float64) / 1e3)
            print("workers %d producers %3d window %3d: p50 %7.1f p99 %7.1f us, %7.0f decisions/s, %5d batches, equal %s" % (
                workers, threads, window_us, us[n // 2], us[int(n * 0.99)], n / (wall * 1e-9), st["batches"] - b0,
                bool(np.array_equal(stri.reshape(n, -1)[:, 0], tri.reshape(n, -1)[:, 0].astype(np.uint8)))),
                flush=True)


if __name__ == "__main__":
    main()
