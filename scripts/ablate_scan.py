"""Profiling helper: time the fast-path variants interleaved in one process
(cdna_hip_programming.md §5.4 rule 24) and print one JSON line. Modes (authjx_debug_ablate):
0 single-pass kernel (default), 5 line engine, 11 line engine loads + ring writes only,
12 + classification, 1/2 single-pass loads / + classification, 3 stage A / stage B split;
100 + m: mode m without the length-bucketed request order; 200 + m: with it also for
multi-tenant batches."""
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
if w.auth_config is not None:  # c5: the phase's forest ruleset
    cfg = w.auth_config
    rss = [ctx.compile_forest([cfg.conditions] + [e for c in cfg.authorization for e in (c.conditions, c.rules)])]
else:
    rss = [ctx.compile_expression(e) for e in w.sets]
sor = torch.from_numpy(w.set_of_req.view(np.int32)).to(dev) if w.set_of_req is not None else None
L = runtime.load_library()
L.authjx_debug_ablate.argtypes = [C.c_void_p, C.c_int]
L.authjx_debug_len_sort.argtypes = [C.c_void_p, C.c_int]
L.authjx_debug_tenant_stage.argtypes = [C.c_void_p, C.c_int]
arena = torch.from_numpy(w.arena).to(dev)
offs = torch.from_numpy(w.offs.view(np.int64)).to(dev)
lens = torch.from_numpy(w.lens.view(np.int32)).to(dev)
R = max(r.n_patterns for r in rss)
tri = torch.empty(n * rss[0].n_trees, dtype=torch.uint8, device=dev)
err = torch.empty(n * rss[0].n_trees, dtype=torch.int32, device=dev)
bm = torch.empty((n, (R + 63) // 64), dtype=torch.int64, device=dev)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
MODES = [int(m) for m in (sys.argv[3].split(',') if len(sys.argv) > 3 else ['0', '5', '11', '12'])]
res = {m: [] for m in MODES}
outs = {}
for rep in range(6):
    for mode in MODES:
        L.authjx_debug_ablate(ctx._h, mode % 100)
        L.authjx_debug_len_sort(ctx._h, 2 if 200 <= mode < 300 else 0 if 100 <= mode < 200 else 1)
        L.authjx_debug_tenant_stage(ctx._h, 0 if 300 <= mode < 400 else 1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        ctx.eval_device(rss, arena, offs, lens, tri, err, bm, set_of_req=sor, stream=stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        if rep:
            res[mode].append(a.elapsed_time(b))
        if rep == 1 and mode == 0:
            exact0 = ctx.last_exact_count()
        if rep == 1 and mode % 100 in (0, 5):
            outs[mode] = (tri.cpu().numpy().copy(), bm.cpu().numpy().copy())
bytes_ = int(w.lens.astype(np.int64).sum())
out = {m: {"ms": float(np.median(v)), "GBps": bytes_ / (np.median(v) * 1e-3) / 1e9} for m, v in res.items() if v}
ref = outs[MODES[0]]
same = all(bool(np.array_equal(ref[0], o[0]) and np.array_equal(ref[1], o[1])) for o in outs.values())
print(json.dumps({"workload": wl, "n": n, "doc_bytes": bytes_, "exact_requests_mode0": exact0, "modes": out, "outputs_equal_across_modes": same}))
