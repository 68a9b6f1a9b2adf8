"""bench.py — headline benchmark (BASELINE.json metric) for the pattern-matching hot path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5] [--requests N]

A step = one pass of the hot path (ajx kernels behind authjx_eval_batch_device) over one
batch of N synthetic Authorization-JSON documents already resident in HBM. N=1 runs the
config BASELINE.json's metric is quoted on that fits one GPU (configs[1], "c2": 1M
requests x 16 eq/neq/incl patterns). Multi-GPU: one process per GPU, each rank
evaluating its own shard (weak scaling, no data-path collective); `--gpus N` started
without a torch.distributed.run environment re-launches itself under
torch.distributed.run (before touching any GPU) with N ranks. The timed region is
bracketed by barrier + synchronize, the max over ranks is reported, rank 0 prints one
JSON line. c4 (10k AuthConfigs, per-request set ids from the host index) and c5 (full
phase, 4 KiB documents) default to 2M requests per GPU (16M over 8 GPUs).
`--dry-run` runs the same distributed driver on the CPU (gloo) with a stand-in step, for
the CPU tests of the N>1 path.
"""
import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--requests", "--n", dest="n", type=int, default=None,
                    help="requests per GPU per step (c2/c3 1M, c4/c5 2M)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--no-serve", action="store_true", help="skip the micro-batcher serving leg (c4)")
    ap.add_argument("--unique", type=int, default=None,
                    help="distinct document templates (default 16384 for c2/c3/c4, 4096 for c5)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo test of the distributed driver: no GPU, a stand-in step")
    ap.add_argument("--kernel-mode", type=int, default=0,
                    help="0 the single-pass kernel (default), 20 the lane kernel; others: profiling ablations")
    ap.add_argument("--gather-decisions", action="store_true",
                    help="N>1: all-gather every rank's decision bitmap inside each step (SURVEY.md §8e, optional)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "pmc_traffic.json"))
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(args) -> None:
    """`--gpus N` (N > 1) outside a torch.distributed.run environment: start N ranks as a
    child torch.distributed.run and exit with its status. Runs before anything touches
    the GPU (the child is a separate process, never an exec)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    # (`--n` would be an ambiguous abbreviation of torch.distributed.run's own options)
    cmd += ["--requests" if a == "--n" else a for a in sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def host_threads() -> int:
    """Host threads the CPU baseline uses: every core this process may run on, capped by
    OMP_NUM_THREADS (the GPU box sets it to its per-GPU CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def host_cores() -> dict:
    """The host's core count beside the threads the baseline used: the north star asks for
    the reference timed with GOMAXPROCS = host cores; the GPU box gives a process its
    per-GPU share (OMP_NUM_THREADS), which the baseline stays within."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return {"host_cores": os.cpu_count(), "affinity_cores": aff,
            "threads_cap": int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None}


def cpu_baseline(w, rpr, target_s, gpu_tri, gpu_bm):
    """Oracle (C restatement, oracle/) on a bounded sample of the same workload; also the
    parity check of the GPU results on that sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    threads = host_threads()
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
        **host_cores(),
        "kind": "port",
        "sample": f"first {sample} of the {w.n} synthetic docs x {reps} passes, same ruleset, oracle/ C "
                  f"restatement (gjson re-scan per pattern like the reference, each pattern evaluated once), "
                  f"{threads} host threads, {dt:.1f}s",
    }, {"sample": sample, "mismatches": mism}


def phase_cpu_baseline(w, exprs, target_s, gpu_tri):
    """c5: the oracle evaluates every tree of the phase (re-scanning the document per
    pattern, like the reference) on a bounded prefix; parity of the per-tree results."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    threads = host_threads()
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
            **host_cores(), "kind": "port", "sample": f"first {k} of the {w.n} docs, every tree of the phase, oracle/ C restatement, "
                                      f"{threads} host threads, {dt:.1f}s"}, {"sample": k, "mismatches": mism}


def decision_bitmap(torch, tri, T, weights):
    """One bit per (request, tree) result that is T, LSB first (entry k at bit k % 8 of byte
    k // 8): the decision bitmap a front-end reads. tri: u8 results, length a multiple of 8."""
    return ((tri == T).view(-1, 8).to(torch.uint8) * weights).sum(dim=1, dtype=torch.uint8)


class DecisionGather:
    """The optional exchange of SURVEY.md §8e: every rank's decision bitmap all-gathered
    into one (world × bytes) buffer on every rank, with one all_gather_into_tensor (RCCL
    over xGMI on the GPU, gloo in the CPU tests) per step. Off by default: the shards are
    independent and the bench value needs no collective."""

    def __init__(self, torch, dist, world, rank, n_entries, T, dev):
        if n_entries % 8:
            raise ValueError("decision gather: results per rank must be a multiple of 8")
        self.torch, self.dist, self.world, self.rank, self.T = torch, dist, world, rank, T
        self.weights = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=dev)
        self.out = torch.empty(world * (n_entries // 8), dtype=torch.uint8, device=dev)
        self.popcount = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.int64, device=dev)

    def __call__(self, tri):
        self.local = decision_bitmap(self.torch, tri, self.T, self.weights)
        self.dist.all_gather_into_tensor(self.out, self.local)

    def report(self, dev=None) -> dict:
        """Checks every rank's slice of the gathered buffer against that rank's own bitmap
        (a MIN over ranks of the per-rank check)."""
        nb = self.local.numel()
        ok = bool(self.torch.equal(self.out[self.rank * nb:(self.rank + 1) * nb], self.local))
        t = self.torch.tensor([1 if ok else 0], dtype=self.torch.int32, device=self.out.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return {"ranks": self.world, "bytes_per_rank": nb, "bytes_gathered": int(self.out.numel()),
                "allowed_bits": int(self.popcount[self.out.long()].sum()), "slices_equal_to_local": bool(int(t[0]))}


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


def c1_cpu_ns_per_op(reps: int = 200000) -> dict:
    """BASELINE configs[0]: one ~700-byte document, All(eq, incl,
    matches), the oracle on ONE host thread, ns per Matches call (the analogue of the
    reference's BenchmarkJSONPatternMatchingAuthz, pkg/evaluators/authorization/json_test.go:275-303)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from authorino_amd import workloads

    w = workloads.make("c1")
    rs = pyoracle.Ruleset.from_expression(w.expr)
    offs = np.zeros(reps, dtype=np.uint64)  # the same document, reps times
    lens = np.full(reps, int(w.lens[0]), dtype=np.uint32)
    pyoracle.eval_batch([rs], w.arena, offs[:1000], lens[:1000], nthreads=1)
    t0 = time.perf_counter()
    tri, _, _ = pyoracle.eval_batch([rs], w.arena, offs, lens, nthreads=1)
    dt = time.perf_counter() - t0
    return {"ns_per_op": dt / reps * 1e9, "patterns": 3, "doc_bytes": int(w.lens[0]), "threads": 1,
            "result": int(tri[0]), "kind": "port",
            "note": "oracle/ C restatement (gjson re-scan per pattern, DFA regex), not the Go binary; "
                    "the published Go figure is 1.797 us/op for 2 eq patterns on a Xeon 8370C core"}


def parallelism(world, gather) -> str:
    if gather:
        return f"dp{world} (independent request shards; all-gather of decision bitmaps per step)"
    return f"dp{world} (independent request shards, no collective)"


def dry_main(args, world, rank, dist, torch) -> None:
    """The distributed driver without a GPU (gloo): same sharding, seeds, barriers, timing
    and JSON line; the step is a stand-in (a checksum over the rank's shard)."""
    from authorino_amd import workloads

    seed = workloads.DEFAULT_SEEDS.get(args.workload, 0) + 7919 * rank
    w = workloads.make(args.workload, n=args.n or 256, seed=seed, unique=args.unique or 64, uniquify=True)
    acc = [0]
    gather = None
    if args.gather_decisions and dist:
        # stand-in results: one byte per request from its length (T = 1)
        tri = torch.from_numpy((w.lens % 3).astype(np.uint8))
        gather = DecisionGather(torch, dist, world, rank, tri.numel(), 1, "cpu")

    def step():
        acc[0] += int(w.arena.sum(dtype=np.uint64)) + int(w.lens.sum())
        if gather:
            gather(tri)

    elapsed, _ = timed_steps(step, args.steps, args.warmup, dist, torch, None)
    gathered = gather.report() if gather else None
    shard = {"rank": rank, "seed": seed, "n": w.n, "first_doc_sha": __import__("hashlib").sha1(w.doc(0)).hexdigest()}
    shards = [None] * world
    if dist:
        dist.all_gather_object(shards, shard)
    else:
        shards = [shard]
    if rank == 0:
        print(json.dumps({"metric": "request×rule evals/sec (dry run: stand-in step, no GPU)", "value": None,
                          "unit": "request×rule evals/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "synthetic", "dry_run": True, "shards": shards, "decision_gather": gathered,
                          "config": {"workload": args.workload, "requests_per_gpu": w.n,
                                     "parallelism": parallelism(world, gather)}}),
              flush=True)


def main():
    args = parse()
    relaunch(args)  # --gpus N without torch.distributed.run: N child ranks, then exit
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != max(1, args.gpus) and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist

            dist.init_process_group("gloo")
        dry_main(args, world, rank, dist, torch)
        if dist:
            dist.destroy_process_group()
        return
    # RCCL for N > 1 ranks, and for one rank started by torch.distributed.run with
    # --gather-decisions (the single-GPU rehearsal of the N-rank path)
    if world > 1 or (args.gather_decisions and "WORLD_SIZE" in os.environ):
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from authorino_amd import runtime, workloads

    # SURVEY.md §8d seeds; rank k > 0 draws its own shard from seed + 7919 k
    seed = workloads.DEFAULT_SEEDS.get(args.workload, 0) + 7919 * rank
    unique = args.unique or (4096 if args.workload == "c5" else 16384)
    w = workloads.make(args.workload, n=args.n, seed=seed, unique=unique, uniquify=True)
    ctx = runtime.Context(local)
    if args.kernel_mode:
        ctx.set_kernel_mode(args.kernel_mode)
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

    gather = DecisionGather(torch, dist, world, rank, tri.numel(), runtime.T, dev) \
        if args.gather_decisions and dist else None

    def step():
        ctx.eval_device(rss, arena, offs, lens, tri, err, bm, set_of_req=sor, stream=sp)
        if phase:
            ctx.select_from_eval_device(rss[0], r_phase, arena, offs, lens, spans, stream=sp)
        if gather:
            gather(tri)  # (on `stream`, the current stream: inside the timed step)

    extra = {}
    elapsed, kern_ms = timed_steps(step, args.steps, args.warmup, dist, torch, dev, stream)
    if gather:
        extra["decision_gather"] = gather.report()

    total_req = w.n * args.steps * world
    value = int(rpr.sum()) * args.steps * world / elapsed  # shards are equal-sized (weak scaling)
    # doc read once + pattern bitmap + one result byte per tree (+ 12-B spans of the response
    # selectors for c5; its selector tree's result byte is not counted)
    nt_out = nt - 1 if phase else nt
    algo_bytes = int(w.lens.astype(np.int64).sum()) + int(((rpr + 7) // 8 + nt_out).sum())
    if phase:
        algo_bytes += w.n * len(sel.paths) * 12
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    traffic, traffic_note, traffic_src = None, None, None
    try:
        with open(args.pmc_json) as f:
            pmc = json.load(f).get(args.workload, {})
        # (measured by scripts/pmc_traffic.py on the same workload, size and kernel)
        # (the kernel the counters were taken on: the lean kernel for one ruleset, the
        # tenant kernel for a multi-tenant batch, the token scanner on kernel mode 40)
        kname = ("ajx_scan_fused_tenant" if w.set_of_req is not None else
                 "ajx_scan_fused" if args.kernel_mode == 40 else "ajx_scan_lean")
        if pmc.get("n") == w.n and args.kernel_mode in (0, 40) and kname in pmc.get("kernel", "") and \
                (kname != "ajx_scan_fused" or "tenant" not in pmc.get("kernel", "")):
            traffic = pmc.get("hbm_bytes_per_launch")
            traffic_note = pmc.get("note")
            traffic_src = {"file": os.path.relpath(args.pmc_json, ROOT), "kernel": pmc.get("kernel_names") or
                           pmc.get("kernel"), "commit": pmc.get("commit")}
    except (OSError, ValueError):
        pass

    cpu, parity, c1, pcie = None, None, None, None
    tri_h = tri.cpu().numpy()
    if phase:
        # the phase decision from the per-tree results (auth_pipeline.go:454-457, :287-322)
        t = tri_h.reshape(w.n, nt)[:, :nt_out]  # (the last tree: response selectors)
        skipped = t[:, 0] != runtime.T
        ok = np.ones(w.n, dtype=bool)
        for k in range(len(cfg.authorization)):
            ok &= (t[:, 1 + 2 * k] != runtime.T) | (t[:, 2 + 2 * k] == runtime.T)
        extra = {"phase": {"trees": nt_out, "skipped": int(skipped.sum()), "allowed": int((skipped | ok).sum()),
                           "response_selectors": len(sel.paths)}}
        if rank == 0 and world == 1 and not args.no_cpu:
            cpu, parity = phase_cpu_baseline(w, exprs, args.cpu_seconds, t)
    elif rank == 0 and world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(w, rpr, args.cpu_seconds, tri_h, bm.cpu().numpy().view(np.uint64))
    if rank == 0 and world == 1 and not args.no_cpu:
        c1 = c1_cpu_ns_per_op()
    if rank == 0 and world == 1 and not args.no_pcie and not phase:
        # authjx_eval_batch from host buffers: H2D copy of the arena + kernels + D2H of the
        # results, synchronous (never the bench value)
        torch.cuda.synchronize(dev)
        ctx.eval_host_arena(rss, w.arena, w.offs, w.lens, set_of_req=w.set_of_req)
        t0 = time.perf_counter()
        ctx.eval_host_arena(rss, w.arena, w.offs, w.lens, set_of_req=w.set_of_req)
        dt = time.perf_counter() - t0
        pcie = {"value": int(rpr.sum()) / dt, "unit": "request×rule evals/s", "ms_per_batch": dt * 1e3,
                "decisions_per_s": w.n / dt,
                "note": "authjx_eval_batch from pageable host buffers (H2D arena copy + kernels + D2H), one GPU"}
    if rank == 0 and world == 1 and not args.no_cpu and w.hosts is not None:
        # c4's AuthConfig selection on the host: the native batched index
        # lookup (authjx_index_lookup_batch) of every request's host, all host threads; not
        # in the timed GPU step, as in the reference (pkg/service/auth.go:270-289)
        from authorino_amd import index as hix

        nat = hix.NativeIndex()
        for key, sid in workloads.c4_index_entries():
            nat.set(key, sid)
        ha, ho, hl = hix.pack_hosts(w.hosts)
        nth = host_threads()
        got = nat.lookup_batch(ha, ho, hl, n_threads=nth)
        t0 = time.perf_counter()
        nat.lookup_batch(ha, ho, hl, n_threads=nth)
        dt = time.perf_counter() - t0
        extra["host_lookup"] = {"requests": w.n, "ms": dt * 1e3, "hosts_per_s": w.n / dt, "threads": nth,
                                "equal_to_restatement": bool(np.array_equal(got, w.set_of_req.astype(np.int32)))}
    undecided = int((tri_h == runtime.UNDECIDED).sum())
    exact_path = ctx.last_exact_count()  # requests the single-pass kernel handed to the exact scan
    if rank == 0 and world == 1 and not args.no_serve and w.set_of_req is not None and nt == 1:
        # the serving path (never the headline value): 64 native producer threads push a
        # sample of the batch through the micro-batcher one blocking request at a time, as
        # serving goroutines would (main.go:69,451; pkg/service/auth_pipeline.go:150-164)
        extra["serving"] = []
        # (64 producers: the VERDICT's case; 256: a loaded server, within the box's task cap;
        # the window trades latency for batch size; batches up to the stream threshold take
        # the streaming kernel, one request per wave)
        for threads, window_us in ((64, 200), (64, 50), (64, 20), (256, 200)):
            ns = min(w.n, 1 << 18)
            b = runtime.Batcher(ctx, max_batch=8192, window_us=window_us)
            try:
                b.loadgen(rss, w.set_of_req[:4096], w.arena, w.offs[:4096], w.lens[:4096], threads=threads)  # (warm up)
                b0 = b.stats()["batches"]
                lat, stri, wall = b.loadgen(rss, w.set_of_req[:ns], w.arena, w.offs[:ns], w.lens[:ns], threads=threads)
                st = b.stats()
            finally:
                b.close()
            us = np.sort(lat.astype(np.float64) / 1e3)
            extra["serving"].append({
                "producer_threads": threads, "requests": int(ns), "decisions_per_s": ns / (wall * 1e-9),
                "latency_us": {"p50": float(us[ns // 2]), "p99": float(us[int(ns * 0.99)]), "max": float(us[-1])},
                "batches": st["batches"] - b0, "max_batch_seen": st["max_batch_seen"], "max_batch": 8192,
                "window_us": window_us, "workers": 2,
                "equal_to_batch_results": bool(np.array_equal(stri, tri_h[:ns].astype(np.uint8))),
                "note": "authjx_batcher_eval per request, blocking, from pageable host memory (the batch packed into pinned staging that the kernel reads over PCIe and writes its results to: no copies)"})

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
                "unique_templates": unique,
                "seed_rank0": workloads.DEFAULT_SEEDS.get(args.workload, 0),
                "patterns": int(rpr.max()) if w.set_of_req is None else float(rpr.mean()),
                "selectors": rss[0].n_selectors if len(rss) == 1 else float(np.mean([r.n_selectors for r in rss])),
                "auth_configs": len(rss),
                "trees_per_request": nt_out,
                "doc_bytes_mean": float(w.lens.mean()),
                "parallelism": parallelism(world, gather),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_note": traffic_note,
                "traffic_source": traffic_src,  # (the PMC file's kernel instance and commit)
                "kernel_ms": kern_ms,
                **({"note": "kernel_ms is the whole step's event time, decision all-gather included"}
                   if gather else {}),
                "algorithmic_bytes_per_launch": algo_bytes,
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "c1_cpu": c1,
            "pcie_inclusive": pcie,
            "undecided": undecided,
            **extra,
            "exact_path_requests": exact_path,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
