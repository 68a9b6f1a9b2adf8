"""GPU parity of the streaming kernel (authorino_amd/csrc/ajx_stream.h, ajx_scan_stream /
ajx_stream_finish) against the oracle, through the C-ABI: the bench workloads at 32
requests per wave (kernel mode 52), small batches at 1..N requests per wave (the default
path for batches up to the stream threshold), a multi-tenant small batch (one request per
wave under its own ruleset), mutated and invalid documents (handed to the exact scan:
results still the oracle's), and the host emulation's decisions on the same inputs
(tests/test_stream_scan.py) as a cross-check of which requests the stream proves."""
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
    c.set_kernel_mode(0)
    c.set_stream_max(4096)


def _pack(docs):
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    if len(docs):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return np.frombuffer(b"".join(docs) + b"\0" * 64, dtype=np.uint8), offs, lens


def _flat(expr):
    pats, nodes, root = expr.flatten()
    return [(p.selector, int(p.operator), p.value) for p in pats], nodes, root


def _same(ctx, specs, arena, offs, lens, set_of_req=None):
    sets = [ctx.compile(p, n, r) for p, n, r in specs]
    tri, err, bm = ctx.eval_host_arena(sets, arena, offs, lens, set_of_req=set_of_req)
    otri, oerr, obm = O.eval_batch([O.Ruleset(p, n, r) for p, n, r in specs], arena, offs, lens,
                                   set_of_req=set_of_req, nthreads=8)
    bad = np.nonzero((tri != otri) | (err != oerr) | (bm[:, :obm.shape[1]] != obm).any(axis=1))[0]
    assert bad.size == 0, (bad[:10], tri[bad[:10]], otri[bad[:10]], err[bad[:10]], oerr[bad[:10]])
    return tri


@pytest.mark.parametrize("wl,n", [("c2", 20000), ("c5", 3000)])
def test_stream_workloads_on_device(ctx, wl, n):
    """The bench documents through the streaming kernel at 32 requests per wave: every
    request equal to the oracle, none handed to the exact scan."""
    from authorino_amd import workloads

    w = workloads.make(wl, n=n)
    exprs = [w.expr] if wl == "c2" else [w.auth_config.conditions] + [
        e for c in w.auth_config.authorization for e in (c.conditions, c.rules)]
    ctx.set_kernel_mode(52)
    try:
        for e in exprs:
            _same(ctx, [_flat(e)], w.arena, w.offs, w.lens)
            assert ctx.last_exact_count() == 0
    finally:
        ctx.set_kernel_mode(0)


@pytest.mark.parametrize("n", [1, 2, 31, 64, 700, 4096])
def test_stream_small_batches(ctx, n):
    """The default path for small batches (requests per wave by batch size)."""
    from authorino_amd import workloads

    w = workloads.make("c2", n=n, unique=min(n, 256))
    _same(ctx, [_flat(w.expr)], w.arena, w.offs, w.lens)
    assert ctx.last_exact_count() == 0


def test_stream_multi_tenant_small_batch(ctx):
    """A small multi-tenant batch: one request per wave, each under its own ruleset."""
    rng = np.random.default_rng(91)
    specs = []
    while len(specs) < 12:  # (array indices included: stage B's exact Get)
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        specs.append((pats, nodes, root))
    docs = [FU.rand_doc(rng, ws=False) for _ in range(600)]
    sor = np.sort(rng.integers(0, len(specs), len(docs))).astype(np.uint32)
    _same(ctx, specs, *_pack(docs), set_of_req=sor)


def test_stream_c4_small_multi_tenant_batches(ctx):
    """c4's AuthConfigs (array-index selectors among them) in small multi-tenant batches,
    as the micro-batcher sends them: one request per wave, equal to the oracle."""
    from authorino_amd import workloads

    w = workloads.make("c4", n=3000)
    specs = [_flat(e) for e in w.exprs]
    used = sorted(set(int(x) for x in w.set_of_req[:3000]))
    remap = {u: i for i, u in enumerate(used)}
    sor = np.array([remap[int(x)] for x in w.set_of_req[:3000]], dtype=np.uint32)
    for lo in range(0, 3000, 1000):
        hi = lo + 1000
        sub = sorted(set(sor[lo:hi].tolist()))
        m = {u: i for i, u in enumerate(sub)}
        _same(ctx, [specs[used[u]] for u in sub], w.arena, w.offs[lo:hi], w.lens[lo:hi],
              set_of_req=np.array([m[int(x)] for x in sor[lo:hi]], dtype=np.uint32))


def test_stream_mutated_and_invalid_documents(ctx):
    """Truncated / flipped / whitespace documents and the host tests' invalid list: what the
    stream does not prove goes to the exact scan, and every result is the oracle's."""
    from test_stream_scan import INVALID

    rng = np.random.default_rng(92)
    pats = [("a", 1, "1"), ("b", 2, "v"), ("a.b", 1, "2"), ("a.a.a", 3, "x")]
    nodes, root = FU.chain(len(pats))
    docs = list(INVALID) * 3 + [FU.mutate(rng, FU.rand_doc(rng, ws=False)) for _ in range(500)]
    for n_max in (4096, 0):  # (the stream, then the lean kernel, on the same batch)
        ctx.set_stream_max(n_max)
        _same(ctx, [(pats, nodes, root)], *_pack(docs))
    ctx.set_stream_max(4096)


def test_stream_counters_across_launches(ctx):
    """The small-batch instance clears its counters for the next launch on the stream (no
    fill) and publishes the exact-path count apart: repeated batches, and batches of the
    other kernels in between, all equal to the oracle with the same exact-path count."""
    from test_stream_scan import INVALID

    rng = np.random.default_rng(93)
    pats = [("a", 1, "1"), ("b", 2, "v"), ("a.b", 1, "2")]
    nodes, root = FU.chain(len(pats))
    docs = list(INVALID) * 2 + [FU.mutate(rng, FU.rand_doc(rng, ws=False)) for _ in range(300)]
    counts = []
    for n_max in (4096, 4096, 0, 4096, 4096):  # (stream, stream, lean, stream, stream)
        ctx.set_stream_max(n_max)
        _same(ctx, [(pats, nodes, root)], *_pack(docs))
        counts.append(ctx.last_exact_count())
    ctx.set_stream_max(4096)
    stream_counts = [c for c, m in zip(counts, (1, 1, 0, 1, 1)) if m]
    assert stream_counts[0] > 0 and len(set(stream_counts)) == 1, counts


def _dense_docs(rng, n):
    """Documents whose 32-byte blocks hold many opens and keys: nested arrays and objects
    with one-letter keys (`[[[[[[[[[[1]]]]]]]]]]`, `{"a":{"b":{"c":...`), so a block has
    more than 8 opens (the capture loop's open ordinals: round 4's out-of-range
    `oids >> (8 * no)` for no >= 8) and runs of short keys."""
    out = []
    for _ in range(n):
        k = int(rng.integers(6, 20))
        arr = "[" * k + str(int(rng.integers(0, 9))) + "]" * k
        keys = "abcdefghij"
        obj = "".join('{"%s":' % keys[j % 10] for j in range(k)) + '"v"' + "}" * k
        flat = "{" + ",".join('"%s":%d' % (keys[j], j) for j in range(10)) + "}"
        parts = [('"x"', arr), ('"y"', obj), ('"z"', flat)]
        rng.shuffle(parts)
        out.append(("{" + ",".join("%s:%s" % p for p in parts) + "}").encode())
    return out


@pytest.mark.parametrize("n", [1, 64, 2000])
def test_stream_dense_blocks(ctx, n):
    """Regression for round 4's launch failures on one-request batches: blocks with more
    than 8 opens / many keys, selectors into them (array indices, deep keys), at 1, 64 and
    2000 requests per batch; every result the oracle's."""
    rng = np.random.default_rng(94 + n)
    pats = [("x.0.0.0", 1, "[[[1]]]"), ("y.a.b.c", 3, "v"), ("z.j", 1, "9"), ("z.a", 2, "0"),
            ("y.a.b.c.d.e.f.g", 1, "v"), ("x.0.0.0.0.0.0.0.0", 1, "3")]
    nodes, root = FU.chain(len(pats))
    _same(ctx, [(pats, nodes, root)], *_pack(_dense_docs(rng, n)))


def test_stream_slow_path_batch_latency(ctx):
    """a 4096-request small batch whose documents all leave the stream (nesting
    deeper than it tracks, documents over one step) goes through the grid-stride stage-B
    launch, not one wave's list: results equal to the oracle, and the batch takes well under
    the time one wave's serial walk of the list would."""
    import time

    deep = b'{"a":' + b'{"b":' * 20 + b'"v"' + b"}" * 20 + b',"c":"' + b"p" * 2100 + b'","d":"w"}'
    docs = [deep] * 4096
    pats = [("d", 1, "w"), ("c", 2, "x"), ("a.b.b", 3, "v")]
    nodes, root = FU.chain(len(pats))
    arena, offs, lens = _pack(docs)
    rs = ctx.compile(pats, nodes, root)
    ctx.eval_host_arena([rs], arena, offs, lens)  # (warm up)
    t0 = time.perf_counter()
    tri, _, _ = ctx.eval_host_arena([rs], arena, offs, lens)
    dt = time.perf_counter() - t0
    otri, _, _ = O.eval_batch([O.Ruleset(pats, nodes, root)], arena, offs, lens, nthreads=8)
    assert np.array_equal(tri, otri)
    # (one wave walking 4096 exact scans serially took seconds; the grid-stride launch takes
    # milliseconds. The bound is generous so that load on the shared box can not fail it.)
    assert dt < 0.5, dt
