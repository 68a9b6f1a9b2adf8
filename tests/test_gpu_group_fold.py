"""GPU parity of the two-level bitmap fold (kFlagGroupFold, ajx_fast.h group_fold) against
the oracle, through the C-ABI: c3's All(Any x4, All x4) and random All / Any rulesets over
lone patterns and groups of the other kind (patterns that are T, F, E or undecided on
random documents), on small batches (the streaming kernel) and on batches the lean kernel
takes. Reference: pkg/jsonexp/expressions.go:59-154 (And / Or / All / Any)."""
import numpy as np
import pytest

import fuzz_util as FU
import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from authorino_amd import runtime

    c = runtime.Context(0)
    yield c


def _pack(docs):
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    if len(docs):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return np.frombuffer(b"".join(docs) + b"\0" * 64, dtype=np.uint8), offs, lens


def _same(ctx, expr, arena, offs, lens):
    pats, nodes, root = expr.flatten()
    spec = [(p.selector, int(p.operator), p.value) for p in pats]
    rs = ctx.compile(spec, nodes, root)
    tri, err, bm = ctx.eval_host_arena([rs], arena, offs, lens)
    otri, oerr, obm = O.eval_batch([O.Ruleset(spec, nodes, root)], arena, offs, lens, nthreads=8)
    bad = np.nonzero((tri != otri) | (err != oerr) | (bm[:, :obm.shape[1]] != obm).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], tri[bad[:10]], otri[bad[:10]], err[bad[:10]], oerr[bad[:10]])
    return otri


@pytest.mark.parametrize("n", [1, 64, 700, 20000])
def test_c3_group_fold(ctx, n):
    from authorino_amd import workloads

    w = workloads.make("c3", n=n, unique=min(n, 4096))
    otri = _same(ctx, w.expr, w.arena, w.offs, w.lens)
    if n >= 700:
        assert 0 < int((otri == 1).sum()) < n  # (both outcomes occur)


def _random_group_expr(rng):
    from authorino_amd import jsonexp as J

    outer = J.All if rng.random() < 0.5 else J.Any
    inner = J.Any if outer is J.All else J.All
    kids = [None if rng.random() < 0.5 else int(rng.integers(2, 7)) for _ in range(int(rng.integers(2, 7)))]
    if all(k is None for k in kids):
        kids[0] = 3
    npat = sum(1 if k is None else k for k in kids)
    ps = [J.Pattern(s, J.Operator(op), v) for s, op, v in FU.rand_patterns(rng, npat)]
    args, i = [], 0
    for k in kids:
        if k is None:
            args.append(ps[i])
            i += 1
        else:
            args.append(inner(*ps[i:i + k]))
            i += k
    return outer(*args)


@pytest.mark.parametrize("seed", [0, 1])
def test_random_group_folds(ctx, seed):
    rng = np.random.default_rng(4100 + seed)
    for _ in range(12):
        expr = _random_group_expr(rng)
        for n in (48, 9000):
            docs = [FU.rand_doc(rng, ws=bool(rng.random() < 0.2)) for _ in range(min(n, 600))]
            docs = [docs[i % len(docs)] for i in range(n)]
            arena, offs, lens = _pack(docs)
            _same(ctx, expr, arena, offs, lens)


@pytest.mark.parametrize("seed", [0, 1])
def test_random_forest_tree_folds(ctx, seed):
    """Forests of flat and two-level trees (TreeFold: each tree folds off its own bits of the
    128-bit bitmaps, bases on both sides of bit 64) and one three-level tree (interpreted):
    every tree's result and error index against the oracle of that tree alone."""
    from authorino_amd import jsonexp as J

    rng = np.random.default_rng(4300 + seed)
    for _ in range(4):
        exprs, total = [], 0
        while total < 80:  # (at most 35 patterns a tree: 115 in all, then 4 more)
            e = _random_group_expr(rng)
            exprs.append(e)
            total += len(e.flatten()[0])
        p4 = [J.Pattern(s, J.Operator(op), v) for s, op, v in FU.rand_patterns(rng, 4)]
        exprs.insert(int(rng.integers(0, len(exprs) + 1)), J.All(J.Any(J.All(p4[0], p4[1]), p4[2]), p4[3]))
        assert sum(len(e.flatten()[0]) for e in exprs) <= 128
        forest = ctx.compile_forest(exprs)
        docs = [FU.rand_doc(rng, ws=bool(rng.random() < 0.2)) for _ in range(500)]
        docs = [docs[i % len(docs)] for i in range(6000)]
        arena, offs, lens = _pack(docs)
        ftri, ferr, _ = ctx.eval_host_arena([forest], arena, offs, lens)
        for k, e in enumerate(exprs):
            pats, nodes, root = e.flatten()
            spec = [(p.selector, int(p.operator), p.value) for p in pats]
            otri, oerr, _ = O.eval_batch([O.Ruleset(spec, nodes, root)], arena, offs, lens, nthreads=8)
            off = forest.offsets[k]
            assert np.array_equal(ftri[:, k], otri), k
            assert np.array_equal(ferr[:, k], np.where(oerr >= 0, oerr + off, -1)), k
