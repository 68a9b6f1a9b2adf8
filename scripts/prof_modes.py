"""Time several kernel modes of the one-ruleset path in one process (one workload build):

  python scripts/prof_modes.py --workload c2 --modes 0,15,16,17,18 --reps 5

Modes (ajx_api.cpp / ajx_kernels.hip): 0 the product path; 15..18 the lean kernel's stage-A
ablations (15 loads + ring stores, 16 + classification, 17 + walk without eager patterns,
18 full stage A), no stage B. Under `rocprofv3 --pmc ...` each mode's kernel instance has
its own name (ajx_scan_lean<true, ABL>), so one counter pass covers every mode.
Prints one JSON line per mode: mean HIP-event ms per launch on the eval stream.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--modes", default="0,15,16,17,18")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None, help="AUTHJX_LIB: a variant build of libauthjx.so")
    ap.add_argument("--alias", type=int, default=0,
                    help="request i reads document i %% K (the batch's bytes then fit the caches: "
                         "the kernel without its HBM traffic)")
    a = ap.parse_args()
    if a.lib:
        os.environ["AUTHJX_LIB"] = a.lib
    import torch

    from authorino_amd import runtime, workloads

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    unique = 4096 if a.workload == "c5" else 16384
    w = workloads.make(a.workload, n=a.n, unique=unique, uniquify=True)
    if a.alias:
        k = a.alias
        end = int(w.offs[k - 1]) + int(w.lens[k - 1])
        w.arena = w.arena[:end + 64].copy()
        w.offs = w.offs[np.arange(w.n) % k].copy()
        w.lens = w.lens[np.arange(w.n) % k].copy()
    ctx = runtime.Context(0)
    rss = [ctx.compile_expression(e) for e in w.sets]
    arena = torch.from_numpy(w.arena).to(dev)
    offs = torch.from_numpy(w.offs.view(np.int64)).to(dev)
    lens = torch.from_numpy(w.lens.view(np.int32)).to(dev)
    sor = torch.from_numpy(w.set_of_req.view(np.int32)).to(dev) if w.set_of_req is not None else None
    R = int(max(len(e.flatten()[0]) for e in w.sets))
    tri = torch.empty(w.n, dtype=torch.uint8, device=dev)
    err = torch.empty(w.n, dtype=torch.int32, device=dev)
    bm = torch.empty((w.n, (R + 63) // 64), dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ref = None
    for m in [int(x) for x in a.modes.split(",")]:
        ctx.set_kernel_mode(m)
        ctx.eval_device(rss, arena, offs, lens, tri, err, bm, set_of_req=sor, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record(stream)
            ctx.eval_device(rss, arena, offs, lens, tri, err, bm, set_of_req=sor, stream=stream.cuda_stream)
            e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
        line = {"workload": a.workload, "n": w.n, "mode": m, "ms": round(ms, 4), "alias": a.alias,
                "bytes": int(w.lens.astype(np.int64).sum())}
        if m == 0:
            ref = tri.cpu().numpy().copy()
            line["allowed"] = int((ref == runtime.T).sum())
        elif ref is not None and m in (41, 52):
            line["equal_to_mode0"] = bool(np.array_equal(tri.cpu().numpy(), ref))
        print(json.dumps(line), flush=True)
    ctx.set_kernel_mode(0)


if __name__ == "__main__":
    main()
