"""GPU: the micro-batcher's serving path (ajx_api.cpp authjx_batcher::evaluate): one staging
copy per batch (documents, offsets, lengths, ruleset indices, blob pointers), results
written by the kernel into mapped pinned memory, and the streaming kernel's counters left
zero by its last wave. Batches of many rulesets, invalid and mutated documents (the exact
path inside the kernel) and, on the same batcher, batches that take the other kernels
(stream threshold 0) in between: every result equal to the oracle's (oracle/, the CPU
restatement) on the same requests, so that a bug shared by the serving path and the batch
kernels can not pass unnoticed."""
import numpy as np
import pytest

import fuzz_util as FU
import pyoracle as O

pytestmark = pytest.mark.gpu


def _pack(docs):
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return np.frombuffer(b"".join(docs) + b"\0" * 64, dtype=np.uint8), offs, lens


def test_batcher_mixed_rulesets_and_kernels():
    from authorino_amd import runtime
    from test_stream_scan import INVALID

    ctx = runtime.Context(0)
    try:
        rng = np.random.default_rng(95)
        sets, specs = [], []
        while len(sets) < 6:
            pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
            nodes, root = FU.chain(len(pats))
            sets.append(ctx.compile(pats, nodes, root))
            specs.append((pats, nodes, root))
        docs = list(INVALID) + [FU.rand_doc(rng, ws=False) for _ in range(700)]
        docs += [FU.mutate(rng, FU.rand_doc(rng, ws=False)) for _ in range(300)]
        arena, offs, lens = _pack(docs)
        sor = rng.integers(0, len(sets), len(docs)).astype(np.uint32)
        want, _, _ = O.eval_batch([O.Ruleset(p, n, r) for p, n, r in specs], arena, offs, lens, set_of_req=sor,
                                  nthreads=8)
        b = runtime.Batcher(ctx, max_batch=512, window_us=100)
        try:
            for n_max in (4096, 0, 4096, 4096):  # (stream, lean / tenant, stream again)
                ctx.set_stream_max(n_max)
                _, got, _ = b.loadgen(sets, sor, arena, offs, lens, threads=48)
                bad = np.nonzero(got != want.astype(np.uint8))[0]
                assert bad.size == 0, (n_max, bad[:10], got[bad[:10]], want[bad[:10]])
        finally:
            ctx.set_stream_max(4096)
            b.close()
    finally:
        ctx.close()


def test_batcher_forest_results_per_tree():
    """A forest ruleset (c5's phase: one result per tree): every tree's result and error
    index comes back through the mapped buffer, from concurrent callers."""
    from concurrent.futures import ThreadPoolExecutor

    from authorino_amd import runtime, workloads

    ctx = runtime.Context(0)
    try:
        w = workloads.make("c5", n=160)
        exprs = [w.auth_config.conditions] + [e for c in w.auth_config.authorization for e in (c.conditions, c.rules)]
        forest = ctx.compile_forest(exprs)
        # the oracle, one tree at a time (a forest's result k is tree k's Matches)
        outs = [O.eval_batch([O.Ruleset.from_expression(e)], w.arena, w.offs, w.lens, nthreads=8) for e in exprs]
        tri = np.stack([o[0] for o in outs], axis=1)
        # (forest numbering: tree k's pattern j is forest.offsets[k] + j)
        err = np.stack([np.where(o[1] >= 0, o[1] + forest.offsets[k], -1) for k, o in enumerate(outs)], axis=1)
        docs = [bytes(w.arena[int(o):int(o) + int(n)]) for o, n in zip(w.offs, w.lens)]
        b = runtime.Batcher(ctx, max_batch=64, window_us=200)
        try:
            with ThreadPoolExecutor(16) as ex:
                got = list(ex.map(lambda d: b.eval(forest, d), docs))
        finally:
            b.close()
        for r, (t, e) in enumerate(got):
            assert list(t) == [int(x) for x in tri[r]], (r, t, tri[r])
            assert list(e) == [int(x) for x in err[r]], (r, e, err[r])
    finally:
        ctx.close()
