"""Profiling helper: blob sizes of the c4 rulesets and the share of waves the multi-tenant
kernel can run from LDS (its staging rule restated: the leading runs of each 256-request
workgroup while their blobs fit the staging region, at most 8 runs)."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import runtime, workloads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
region = int(sys.argv[2]) if len(sys.argv) > 2 else 8192 - 256
w = workloads.make("c4", n=n, unique=16384, uniquify=True)
ctx = runtime.Context(0)
L = runtime.load_library()
L.authjx_debug_blob_bytes.restype = C.c_uint32
L.authjx_debug_blob_bytes.argtypes = [C.c_void_p]
used = np.unique(w.set_of_req)
size = np.zeros(len(w.sets), dtype=np.int64)
for i in used:
    rs = ctx.compile_expression(w.sets[i])
    size[i] = L.authjx_debug_blob_bytes(rs._h)
s = w.set_of_req.astype(np.int64)
waves_lds = waves = 0
for g0 in range(0, n, 256):
    g = s[g0:g0 + 256]
    starts = np.r_[True, g[1:] != g[:-1]]
    ridx = np.cumsum(starts) - 1
    rs = g[starts][:8]
    off, nst = 0, 0
    for x in rs:
        if off + size[x] > region:
            break
        off += size[x]
        nst += 1
    for q in range(0, len(g), 64):
        waves += 1
        waves_lds += int((ridx[q:q + 64] < nst).all())
print(json.dumps({"n": n, "region": region, "rulesets": int(len(used)), "blob_bytes": {
    "mean": float(size[used].mean()), "p50": float(np.percentile(size[used], 50)),
    "p90": float(np.percentile(size[used], 90)), "max": int(size[used].max())},
    "waves": waves, "waves_lds_frac": waves_lds / waves}))
