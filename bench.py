"""bench.py — headline benchmark (BASELINE.json metric) for the pattern-matching hot path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4] [--n N_REQUESTS]

A step = one pass of the hot path (ajx kernels behind authjx_eval_batch_device) over one
batch of N synthetic Authorization-JSON documents already resident in HBM. N=1 runs the
config BASELINE.json's metric is quoted on that fits one GPU (configs[1], "c2": 1M
requests x 16 eq/neq/incl patterns). Multi-GPU: one process per GPU
(torch.distributed.run), each rank evaluates its own shard (weak scaling, no data-path
collective); the timed region is bracketed by barrier + synchronize, the max over ranks
is reported. Rank 0 prints one JSON line. c4 (multi-tenant: 10k AuthConfigs, per-request
set ids from the host index) defaults to 2M requests per GPU (16M over 8 GPUs).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--n", type=int, default=None, help="requests per GPU per step (c2/c3 1M, c4 2M)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def cpu_baseline(w, rpr, target_s, gpu_tri, gpu_bm):
    """Oracle (C restatement, oracle/) on a bounded sample of the same workload; also the
    parity check of the GPU results on that sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    rss = [pyoracle.Ruleset.from_expression(e) for e in w.sets]
    sor = w.set_of_req
    pilot = min(w.n, 16384)

    def run(k):
        return pyoracle.eval_batch(rss, w.arena, w.offs[:k], w.lens[:k], nthreads=threads,
                                   set_of_req=None if sor is None else sor[:k])

    t0 = time.perf_counter()
    run(pilot)
    dt = max(time.perf_counter() - t0, 1e-6)
    # the whole batch when it fits the time budget (repeated passes up to ~target_s), else
    # a prefix of it
    sample = int(min(w.n, max(pilot, pilot * target_s / dt)))
    reps = max(1, int(target_s / (dt * sample / pilot)))
    t0 = time.perf_counter()
    for _ in range(reps):
        tri, err, bm = run(sample)
    dt = time.perf_counter() - t0
    mism = int((tri != gpu_tri[:sample]).sum()) + int((bm != gpu_bm[:sample, :bm.shape[1]]).any(axis=1).sum())
    return {
        "value": reps * int(rpr[:sample].sum()) / dt,
        "unit": "request×rule evals/s",
        "decisions_per_s": reps * sample / dt,
        "cores": threads,
        "kind": "port",
        "sample": f"first {sample} of the {w.n} synthetic docs x {reps} passes, same ruleset, oracle/ C "
                  f"restatement (gjson re-scan per pattern like the reference), {threads} host threads, {dt:.1f}s",
    }, {"sample": sample, "mismatches": mism}


def phase_cpu_baseline(w, exprs, target_s, gpu_tri):
    """c5: the oracle evaluates every tree of the phase (re-scanning the document per
    pattern, like the reference) on a bounded prefix; parity of the per-tree results."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    rss = [pyoracle.Ruleset.from_expression(e) for e in exprs]
    R = sum(len(e.flatten()[0]) for e in exprs)
    k = min(w.n, 4096)
    t0 = time.perf_counter()
    outs = [pyoracle.eval_batch([r], w.arena, w.offs[:k], w.lens[:k], nthreads=threads)[0] for r in rss]
    dt = time.perf_counter() - t0
    if dt < target_s:
        k = int(min(w.n, k * target_s / max(dt, 1e-6)))
        t0 = time.perf_counter()
        outs = [pyoracle.eval_batch([r], w.arena, w.offs[:k], w.lens[:k], nthreads=threads)[0] for r in rss]
        dt = time.perf_counter() - t0
    got = np.stack(outs, axis=1)
    mism = int((got != gpu_tri[:k]).any(axis=1).sum())
    return {"value": k * R / dt, "unit": "request×rule evals/s", "decisions_per_s": k / dt, "cores": threads,
            "kind": "port", "sample": f"first {k} of the {w.n} docs, every tree of the phase, oracle/ C restatement, "
                                      f"{threads} host threads, {dt:.1f}s"}, {"sample": k, "mismatches": mism}


def timed_steps(step, steps, warmup, dist, torch, dev, stream=None):
    """W untimed steps, then exactly K timed steps bracketed by barrier + synchronize on
    both sides; returns (wall seconds, mean per-step event ms on `stream`), each the max
    over ranks. With dev=None (CPU tests, gloo) the synchronize / events are skipped."""
    gpu = dev is not None

    def sync():
        if gpu:
            torch.cuda.synchronize(dev)

    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)] if gpu else []
    t0 = time.perf_counter()
    for k in range(steps):
        if gpu:
            ev[k][0].record(stream)
        step()
        if gpu:
            ev[k][1].record(stream)
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if gpu else 0.0
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev if gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from authorino_amd import runtime, workloads

    w = workloads.make(args.workload, n=args.n, seed=1000 + rank)
    ctx = runtime.Context(local)
    phase = w.auth_config is not None  # c5: the whole authorization phase per request
    if phase:
        # one forest ruleset: top-level when, each evaluator's when and rules, and last the
        # response-header selectors as a root-less tree; one scan per document captures
        # them all, and authjx_select_from_eval_device reads the selectors' spans from it
        from authorino_amd.response import ResponseSelectors

        cfg = w.auth_config
        exprs = [cfg.conditions] + [e for c in cfg.authorization for e in (c.conditions, c.rules)]
        sel = ResponseSelectors(cfg.response, ctx)
        rss = [ctx.compile_forest(exprs, extra_selectors=sel.paths)]
        R = rss[0].n_patterns  # (bitmap width: phase patterns + the selectors' entries)
        r_phase = R - len(sel.paths)
        rpr = np.full(w.n, r_phase, dtype=np.int64)
    else:
        rpr = w.patterns_per_request()  # R of each request's rule set
        R = int(max(len(e.flatten()[0]) for e in w.sets))
        rss = [ctx.compile_expression(e) for e in w.sets]

    arena = torch.from_numpy(w.arena).to(dev)
    offs = torch.from_numpy(w.offs.view(np.int64)).to(dev)
    lens = torch.from_numpy(w.lens.view(np.int32)).to(dev)
    sor = torch.from_numpy(w.set_of_req.view(np.int32)).to(dev) if w.set_of_req is not None else None
    words = (R + 63) // 64
    nt = rss[0].n_trees
    tri = torch.empty(w.n * nt, dtype=torch.uint8, device=dev)
    err = torch.empty(w.n * nt, dtype=torch.int32, device=dev)
    bm = torch.empty((w.n, words), dtype=torch.int64, device=dev)
    spans = torch.empty((w.n, len(sel.paths), 3), dtype=torch.int32, device=dev) if phase else None
    # a dedicated (non-null) stream: the kernel and the timing events share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream

    def step():
        ctx.eval_device(rss, arena, offs, lens, tri, err, bm, set_of_req=sor, stream=sp)
        if phase:
            ctx.select_from_eval_device(rss[0], r_phase, arena, offs, lens, spans, stream=sp)

    elapsed, kern_ms = timed_steps(step, args.steps, args.warmup, dist, torch, dev, stream)

    total_req = w.n * args.steps * world
    value = int(rpr.sum()) * args.steps * world / elapsed  # shards are equal-sized (weak scaling)
    # doc read once + pattern bitmap + one result byte per tree (+ 12-B spans of the response
    # selectors for c5; its selector tree's result byte is not counted)
    nt_out = nt - 1 if phase else nt
    algo_bytes = int(w.lens.astype(np.int64).sum()) + int(((rpr + 7) // 8 + nt_out).sum())
    if phase:
        algo_bytes += w.n * len(sel.paths) * 12
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.pmc_json) as f:
            pmc = json.load(f)
        if pmc.get("workload") == args.workload and pmc.get("n") == w.n:
            traffic = pmc.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    cpu, parity = None, None
    extra = {}
    if phase:
        # the phase decision from the per-tree results (auth_pipeline.go:454-457, :287-322)
        t = tri.cpu().numpy().reshape(w.n, nt)[:, :nt_out]  # (the last tree: response selectors)
        skipped = t[:, 0] != runtime.T
        ok = np.ones(w.n, dtype=bool)
        for k in range(len(cfg.authorization)):
            ok &= (t[:, 1 + 2 * k] != runtime.T) | (t[:, 2 + 2 * k] == runtime.T)
        extra = {"phase": {"trees": nt_out, "skipped": int(skipped.sum()), "allowed": int((skipped | ok).sum()),
                           "response_selectors": len(sel.paths)}}
        if rank == 0 and world == 1 and not args.no_cpu:
            cpu, parity = phase_cpu_baseline(w, exprs, args.cpu_seconds, t)
    elif rank == 0 and world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(w, rpr, args.cpu_seconds, tri.cpu().numpy(), bm.cpu().numpy().view(np.uint64))
    undecided = int((tri == runtime.UNDECIDED).sum().item())
    exact_path = ctx.last_exact_count()  # requests the single-pass kernel handed to the exact scan

    if rank == 0:
        line = {
            "metric": "request×rule evals/sec (+ allow/deny decisions/sec, % HBM roofline)",
            "value": value,
            "unit": "request×rule evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "decisions_per_s": total_req / elapsed,
            "config": {
                "workload": args.workload,
                "description": w.description,
                "requests_per_gpu": w.n,
                "patterns": int(rpr.max()) if w.set_of_req is None else float(rpr.mean()),
                "selectors": rss[0].n_selectors if len(rss) == 1 else float(np.mean([r.n_selectors for r in rss])),
                "auth_configs": len(rss),
                "trees_per_request": nt_out,
                "doc_bytes_mean": float(w.lens.mean()),
                "parallelism": f"dp{world} (independent request shards, no collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "kernel_ms": kern_ms,
                "algorithmic_bytes_per_launch": algo_bytes,
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "undecided": undecided,
            **extra,
            "exact_path_requests": exact_path,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
