"""Profiling helper: time stage A of the single-pass path in its ablation variants
(0 fused single pass (default), 1 stage-A loads only, 2 stage-A loads + classification, 3 stage A and B as two launches) on the c2 workload, interleaved
in one process (cdna_hip_programming.md §5.4 rule 24). Prints one JSON line."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import runtime, workloads  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
w = workloads.make(wl, n=n)
ctx = runtime.Context(0)
rs = ctx.compile_expression(w.expr)
L = runtime.load_library()
L.authjx_debug_ablate.argtypes = [C.c_void_p, C.c_int]
arena = torch.from_numpy(w.arena).to(dev)
offs = torch.from_numpy(w.offs.view(np.int64)).to(dev)
lens = torch.from_numpy(w.lens.view(np.int32)).to(dev)
R = w.n_patterns
tri = torch.empty(n, dtype=torch.uint8, device=dev)
err = torch.empty(n, dtype=torch.int32, device=dev)
bm = torch.empty((n, (R + 63) // 64), dtype=torch.int64, device=dev)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
res = {0: [], 1: [], 2: [], 3: []}
outs = {}
for rep in range(6):
    for mode in (0, 1, 2, 3):
        L.authjx_debug_ablate(ctx._h, mode)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        ctx.eval_device([rs], arena, offs, lens, tri, err, bm, stream=stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        if rep:
            res[mode].append(a.elapsed_time(b))
        if mode in (0, 3) and rep == 1:
            outs[mode] = (tri.cpu().numpy().copy(), bm.cpu().numpy().copy())
bytes_ = int(w.lens.astype(np.int64).sum())
out = {m: {"ms": float(np.median(v)), "GBps": bytes_ / (np.median(v) * 1e-3) / 1e9} for m, v in res.items() if v}
same = bool(np.array_equal(outs[0][0], outs[3][0]) and np.array_equal(outs[0][1], outs[3][1]))
print(json.dumps({"workload": wl, "n": n, "doc_bytes": bytes_, "modes": out, "fused_equals_split": same}))
