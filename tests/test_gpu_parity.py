"""GPU parity tests: the HIP path (through the C-ABI) against the oracle.

Bit-exact: per-request tri-state, per-pattern T bitmap and the deciding error pattern.
"""
import numpy as np
import pytest

import pyoracle as O
from kat_util import build, flat, load_kats

pytestmark = pytest.mark.gpu

KATS = load_kats()


@pytest.fixture(scope="module")
def ctx():
    from authorino_amd import runtime

    return runtime.Context(0)


def _oracle(w_expr, arena, offs, lens, set_of_req=None, sets=None):
    if sets is None:
        pats, nodes, root = flat(w_expr)
        sets = [O.Ruleset(pats, nodes, root)]
    return O.eval_batch(sets, arena, offs, lens, set_of_req=set_of_req, nthreads=8)


def test_reference_kats_via_jsonexp_api():
    """The jsonexp mirror (Expression.matches) on the reference's own vectors."""
    for case in KATS:
        expr = build(case["tree"])
        ok, err = expr.matches(case["doc"])
        if case["expect"] == "T":
            assert ok and err is None, case
        elif case["expect"] == "F":
            assert not ok and err is None, case
        else:
            assert not ok and err is not None and case["error_contains"] in str(err), case


def test_reference_kats_one_batch(ctx):
    """All KATs in one multi-ruleset batch (set_of_req)."""
    sets, osets, docs = [], [], []
    for case in KATS:
        pats, nodes, root = flat(build(case["tree"]))
        sets.append(ctx.compile(pats, nodes, root))
        osets.append(O.Ruleset(pats, nodes, root))
        docs.append(case["doc"].encode())
    sor = np.arange(len(KATS), dtype=np.uint32)
    tri, err, bm = ctx.eval_host(sets, docs, set_of_req=sor)
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(docs), dtype=np.uint8)
    otri, oerr, obm = O.eval_batch(osets, arena, offs, lens, set_of_req=sor)
    assert np.array_equal(tri, otri)
    assert np.array_equal(err, oerr)
    assert np.array_equal(bm, obm)


@pytest.mark.parametrize("workload,n", [("c2", 50000), ("c3", 30000), ("c1", 1)])
def test_workload_parity(ctx, workload, n):
    from authorino_amd import workloads as W

    w = W.make(workload, n=n)
    rs = ctx.compile_expression(w.expr)
    tri, err, bm = ctx.eval_host_arena([rs], w.arena, w.offs, w.lens)
    otri, oerr, obm = _oracle(w.expr, w.arena, w.offs, w.lens)
    assert np.array_equal(tri, otri)
    assert np.array_equal(err, oerr)
    assert np.array_equal(bm, obm)
    assert (tri == 3).sum() == 0


@pytest.mark.parametrize("spread", ["narrow", "wide"])
def test_outputs_gathered_to_request_order(ctx, spread):
    """In length order the lean kernel writes its outputs in work-item order and
    ajx_unpermute gathers them back by each request's work-item (pos_of from the length
    sort), before the exact scan writes the requests it was handed: lengths in a 200-byte
    band (the sort keeps the identity order) and over the whole c2 range, one request in 16
    re-spaced so that it takes the exact scan, a 3-word bitmap stride; then the same batch
    without the error and bitmap outputs."""
    import torch

    from authorino_amd import workloads as W

    w = W.make("c2", n=12000)
    idx = np.arange(w.n)
    if spread == "narrow":
        idx = np.nonzero((w.lens >= 900) & (w.lens < 1100))[0][:6000]
    assert idx.size >= 4096
    docs = [bytes(w.arena[w.offs[i]:w.offs[i] + w.lens[i]]) for i in idx]
    docs = [d.replace(b'":', b'": ', 3) if j % 16 == 5 else d for j, d in enumerate(docs)]
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(docs) + b"\0" * 64, dtype=np.uint8)
    rs = ctx.compile_expression(w.expr)
    tri, err, bm = ctx.eval_host_arena([rs], arena, offs, lens, bitmap_words=3)
    otri, oerr, obm = _oracle(w.expr, arena, offs, lens)
    assert ctx.last_exact_count() >= len(docs) // 16
    assert np.array_equal(tri, otri)
    assert np.array_equal(err, oerr)
    assert np.array_equal(bm[:, :1], obm) and not bm[:, 1:].any()
    dev = torch.device("cuda", 0)
    t_tri = torch.full((len(docs),), 7, dtype=torch.uint8, device=dev)
    ctx.eval_device([rs], torch.from_numpy(arena).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev),
                    torch.from_numpy(lens.view(np.int32)).to(dev), t_tri)
    torch.cuda.synchronize()
    assert np.array_equal(t_tri.cpu().numpy(), otri)


def test_full_size_c2_properties(ctx):
    """BASELINE config c2 at full size (1M requests): bit-exact on a strided sample plus
    size-independent properties (decision == AND of the 16 pattern bits for an All of
    eq/neq/incl patterns; every pattern's T-rate near its design rate)."""
    import torch

    from authorino_amd import workloads as W

    w = W.make("c2", n=1 << 20)
    rs = ctx.compile_expression(w.expr)
    dev = torch.device("cuda", 0)
    arena = torch.from_numpy(w.arena).to(dev)
    offs = torch.from_numpy(w.offs.view(np.int64)).to(dev)
    lens = torch.from_numpy(w.lens.view(np.int32)).to(dev)
    tri = torch.empty(w.n, dtype=torch.uint8, device=dev)
    err = torch.empty(w.n, dtype=torch.int32, device=dev)
    bm = torch.empty((w.n, 1), dtype=torch.int64, device=dev)
    ctx.eval_device([rs], arena, offs, lens, tri, err, bm)
    torch.cuda.synchronize()
    tri = tri.cpu().numpy()
    bits = bm.cpu().numpy().view(np.uint64)[:, 0]
    allow = bits == np.uint64((1 << 16) - 1)
    assert np.array_equal(tri == 1, allow)
    assert set(np.unique(tri)) <= {0, 1}
    rates = [((bits >> np.uint64(p)) & np.uint64(1)).mean() for p in range(16)]
    assert min(rates) > 0.9
    idx = np.arange(0, w.n, 97)
    sub_offs, sub_lens = w.offs[idx], w.lens[idx]
    otri, _, obm = _oracle(w.expr, w.arena, sub_offs, sub_lens)
    assert np.array_equal(tri[idx], otri)
    assert np.array_equal(bits[idx], obm[:, 0])


def _mutations(rng, docs, k):
    """Malformed / edge-case variants: truncation, byte flips, structural deletions."""
    out = []
    for _ in range(k):
        d = bytearray(docs[int(rng.integers(0, len(docs)))])
        m = int(rng.integers(0, 5))
        if m == 0 and len(d) > 2:
            d = d[: int(rng.integers(0, len(d)))]
        elif m == 1 and len(d):
            for _ in range(int(rng.integers(1, 4))):
                d[int(rng.integers(0, len(d)))] = int(rng.choice(list(b'{}[]":,\\ 0a-eu')))
        elif m == 2 and len(d) > 4:
            i = int(rng.integers(0, len(d) - 1))
            del d[i:i + int(rng.integers(1, 4))]
        elif m == 3:
            d = bytearray(b"  \n" + bytes(d) + b" trailing")
        else:
            d = bytearray(bytes(d).replace(b'"', b'\\"', 1))
        out.append(bytes(d))
    return out


def test_malformed_and_edge_documents(ctx):
    """Exact on arbitrary bytes: empty docs, truncated docs, flipped structural bytes."""
    from authorino_amd import workloads as W

    w = W.make("c3", n=400, seed=11)
    base = [w.doc(i) for i in range(w.n)]
    rng = np.random.default_rng(5)
    docs = _mutations(rng, base, 4000) + [b"", b"{", b"[", b"{}", b"[]", b"null", b'"x"', b"{]", b"[}"]
    rs = ctx.compile_expression(w.expr)
    tri, err, bm = ctx.eval_host([rs], docs)
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
    otri, oerr, obm = _oracle(w.expr, arena, offs, lens)
    # every document decided, malformed ones included (no hex / '_' numbers here)
    assert (tri == 3).sum() == 0
    assert np.array_equal(tri, otri)
    assert np.array_equal(err, oerr)
    assert np.array_equal(bm, obm)


def test_fast_and_exact_scan_kernels_agree(ctx):
    """The single-pass kernel and the exact per-selector scan kernel give identical
    outputs on the same batch (c3, 64 patterns incl. 8 regexes)."""
    from authorino_amd import workloads as W

    w = W.make("c3", n=20000, seed=21)
    rs = ctx.compile_expression(w.expr)
    tri, err, bm = ctx.eval_host_arena([rs], w.arena, w.offs, w.lens)
    assert ctx.last_exact_count() == 0  # every synthetic doc took the single-pass path
    ctx.set_exact_scan(True)
    try:
        tri2, err2, bm2 = ctx.eval_host_arena([rs], w.arena, w.offs, w.lens)
    finally:
        ctx.set_exact_scan(False)
    assert np.array_equal(tri, tri2)
    assert np.array_equal(err, err2)
    assert np.array_equal(bm, bm2)


def test_random_documents_and_selectors(ctx):
    """Random JSON (escapes, arrays, duplicate keys, numbers, malformed bytes) and random
    selector sets: GPU == oracle, per pattern and per tree."""
    import fuzz_util as FU

    rng = np.random.default_rng(77)
    checked = 0
    for _ in range(40):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 10)))
        nodes = [(0, -1, -1, i) for i in range(len(pats))]
        root = -1
        for i in reversed(range(len(pats))):
            nodes.append((2 if rng.random() < 0.3 else 1, i, root, -1))
            root = len(nodes) - 1
        ors = O.Ruleset(pats, nodes, root)
        docs = []
        for _ in range(200):
            d = FU.rand_doc(rng)
            docs.append(FU.mutate(rng, d) if rng.random() < 0.3 else d)
        if any(ors.pattern(p, docs[0]) == O.UNSUPPORTED for p in range(len(pats))):
            continue
        rs = ctx.compile(pats, nodes, root)
        tri, err, bm = ctx.eval_host([rs], docs)
        lens = np.array([len(d) for d in docs], dtype=np.uint32)
        offs = np.zeros(len(docs), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1])
        arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
        otri, oerr, obm = O.eval_batch([ors], arena, offs, lens)
        # 16-17-digit floats, subnormals and range ends among the numbers (fuzz_util.NUMS):
        # all decided by the exact scan
        assert (tri == 3).sum() == 0
        assert np.array_equal(tri, otri)
        assert np.array_equal(err, oerr)
        assert np.array_equal(bm, obm)
        checked += len(docs)
    assert checked > 5000


def test_regex_spans_every_alignment(ctx):
    """`matches` over spans read by 16-byte blocks (dfa_match_span): strings of 0..70 bytes
    at every alignment of the document, ASCII and with 2-byte UTF-8 sequences at random
    places (block boundaries among them), through the lean kernel (a 5000-request batch)
    and the streaming kernel (300 requests); equal to the oracle."""
    import json

    rng = np.random.default_rng(41)
    pats = [("v", 5, r"^[a-z]{3,40}$"), ("v", 5, "\u00e9"), ("v", 5, "x$"), ("v", 5, r"^(ab)+c?$"),
            ("v", 5, r"(?i)A.*X"), ("w", 1, "z")]
    nodes = [(0, -1, -1, i) for i in range(len(pats))]
    root = -1
    for i in reversed(range(len(pats))):
        nodes.append((2, i, root, -1))
        root = len(nodes) - 1
    docs = []
    for j in range(5000):
        n = int(rng.integers(0, 71))
        if j % 7 == 0:
            t = "ab" * (n // 2) + ("c" if n % 2 else "")
        else:
            t = "".join(rng.choice(list("abcxAX"), size=n))
        if j % 3 == 0 and n:
            k = int(rng.integers(0, n))
            t = t[:k] + rng.choice(["\u00e9", "\u00df"]) + t[k + 1:]
        pad = "p" * int(rng.integers(0, 16))
        docs.append(json.dumps({"pad": pad, "v": t, "w": "z"}, ensure_ascii=False, separators=(",", ":")).encode())
    rs = ctx.compile(pats, nodes, root)
    ors = O.Ruleset(pats, nodes, root)
    for sub in (docs, docs[:300]):
        lens = np.array([len(d) for d in sub], dtype=np.uint32)
        offs = np.zeros(len(sub), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1])
        arena = np.frombuffer(b"".join(sub) + b"\0" * 64, dtype=np.uint8)
        tri, err, bm = ctx.eval_host_arena([rs], arena, offs, lens)
        otri, oerr, obm = O.eval_batch([ors], arena, offs, lens)
        assert np.array_equal(tri, otri)
        assert np.array_equal(err, oerr)
        assert np.array_equal(bm, obm)


def test_pipeline_batch_on_device():
    """The batched `when` + authorization phase (authorino_amd.pipeline) on the device
    against the same phase evaluated with the oracle (tests/test_pipeline_host.py)."""
    from test_pipeline_host import OracleCtx, _doc

    from authorino_amd import jsonexp as J
    from authorino_amd import pipeline as P

    rng = np.random.default_rng(8)
    subs, groups = ["alice", "bob", "carol"], ["users", "admins", "devs"]
    cfgs = []
    for k in range(8):
        rules = J.Any(J.Pattern("auth.identity.sub", J.EqualOperator, str(rng.choice(subs))),
                      J.Pattern("auth.identity.groups", J.IncludesOperator, str(rng.choice(groups))))
        cond = None if k % 3 == 0 else J.All(
            J.Pattern("context.request.http.path", J.RegexOperator, "^/" + str(rng.choice(["api", "op", "a"]))))
        cfgs.append(P.AuthorizationConfig(f"c{k}", rules=rules, conditions=cond, priority=k % 3))
    cfgs.append(P.AuthorizationConfig("bad", rules=J.All(J.Pattern("x", J.RegexOperator, "(")), priority=3))
    cfg = P.AuthConfig(conditions=J.All(J.Pattern("context.request.http.path", J.NotEqualOperator, "/x")),
                       authorization=cfgs)
    docs = [_doc(str(rng.choice(["/operation", "/api/v1", "/admin", "/x"])), str(rng.choice(subs)),
                 list(rng.choice(groups, size=2, replace=False))) for _ in range(2000)]
    got = P.AuthPipelineBatch(cfg).evaluate(docs)
    want = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate(docs)
    for g, w in zip(got, want):
        assert (g.code, g.message, g.skipped, g.denied_by, g.authorization) == \
               (w.code, w.message, w.skipped, w.denied_by, w.authorization)


def test_multi_tenant_c4(ctx):
    """C4: 10k AuthConfigs compiled to device tables, per-request set ids from the host
    index, one batch bucketed by AuthConfig, against the oracle on the same selection."""
    from authorino_amd import workloads

    w = workloads.make("c4", n=60000, seed=41)
    sets = [ctx.compile_expression(e) for e in w.exprs]
    assert all(st == 0 for s in sets for st in s.status)
    tri, err, bm = ctx.eval_host_arena(sets, w.arena, w.offs, w.lens, set_of_req=w.set_of_req)
    osets = [O.Ruleset.from_expression(e) for e in w.exprs]
    otri, oerr, obm = _oracle(None, w.arena, w.offs, w.lens, set_of_req=w.set_of_req, sets=osets)
    assert (tri == 3).sum() == 0
    assert np.array_equal(tri, otri)
    assert np.array_equal(err, oerr)
    assert np.array_equal(bm, obm)
    assert 0 < (tri == 1).sum() < w.n


def test_multi_tenant_runs_staged(ctx):
    """The multi-tenant kernel's run staging: requests of 600 AuthConfigs in runs of ~100
    (2-4 runs per workgroup, one or two staged in LDS, the rest from global memory), and
    an unsorted copy of the same batch (a run per request), against the oracle."""
    from authorino_amd import workloads

    w = workloads.make("c4", n=60000, seed=43)
    sid = (w.set_of_req.astype(np.int64) % 600)
    order = np.argsort(sid, kind="stable")
    used = np.unique(sid)
    sets = [ctx.compile_expression(w.exprs[i]) for i in used]
    osets = [O.Ruleset.from_expression(w.exprs[i]) for i in used]
    remap = np.searchsorted(used, sid).astype(np.uint32)
    for perm in (order, np.random.default_rng(3).permutation(w.n)):
        offs, lens, sor = w.offs[perm], w.lens[perm], remap[perm]
        tri, err, bm = ctx.eval_host_arena(sets, w.arena, offs, lens, set_of_req=sor)
        otri, oerr, obm = _oracle(None, w.arena, offs, lens, set_of_req=sor, sets=osets)
        assert (tri == 3).sum() == 0
        assert np.array_equal(tri, otri)
        assert np.array_equal(err, oerr)
        assert np.array_equal(bm, obm)


def test_select_values_match_oracle(ctx):
    """authjx_select_batch (gjson.Get spans for response selectors)
    against the oracle's Get on random documents (escapes, numbers, containers, missing
    paths), on the reference's json_test.go document and on C5 documents."""
    from authorino_amd import workloads
    from test_response_host import DOC, _rand_doc

    rng = np.random.default_rng(12)
    docs, paths = [DOC], ["auth.identity.username", "auth.identity.address", "auth.identity.roles",
                          "auth.identity.exp", r"auth.identity.github\.com", "auth.identity.email_verified", "nope"]
    cases = [(DOC, p) for p in paths]
    for _ in range(400):
        d, ps = _rand_doc(rng)
        cases += [(d, p) for p in ps]
    w = workloads.make("c5", n=256, seed=52)
    sel5 = ["auth.identity.sub", "auth.identity.exp", "auth.identity.realm_access.roles", "auth.metadata.tenant",
            "auth.identity.resource_access.talker-api.roles", "context.request.http.host", "auth.identity.acr"]
    cases += [(w.doc(i), p) for i in range(w.n) for p in sel5]
    # one selector ruleset per distinct path; one request per (doc, path)
    uniq = sorted({p for _, p in cases})
    sets = {p: ctx.compile([(p, 1, "")], [], -1) for p in uniq}
    order = [sets[p] for p in uniq]
    sid = {p: i for i, p in enumerate(uniq)}
    sor = np.array([sid[p] for _, p in cases], dtype=np.uint32)
    blobs = [d for d, _ in cases]
    lens = np.array([len(b) for b in blobs], dtype=np.uint32)
    offs = np.zeros(len(blobs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    got = ctx.select_host_arena(order, arena, offs, lens, set_of_req=sor)
    for k, (d, p) in enumerate(cases):
        t, st, ln = O.gjson_span(d, p)
        g = got[k, 0]
        assert (int(g[2]) & 0xFF, int(g[0]), int(g[1])) == (t, st, ln), (d[:200], p)
    # one ruleset of all C5 response paths (LDS-staged single-pass scan, length-ordered)
    w = workloads.make("c5", n=8192, seed=55)
    rs = ctx.compile([(p, 1, "") for p in sel5], [], -1)
    got = ctx.select_host_arena([rs], w.arena, w.offs, w.lens)
    ctx.set_exact_scan(True)
    exact = ctx.select_host_arena([rs], w.arena, w.offs, w.lens)
    ctx.set_exact_scan(False)
    assert np.array_equal(got[:, :, :2], exact[:, :, :2]) and np.array_equal(got[:, :, 2] & 0xFF, exact[:, :, 2] & 0xFF)
    for i in range(0, w.n, 97):
        for j, p in enumerate(sel5):
            t, st, ln = O.gjson_span(w.doc(i), p)
            assert (int(got[i, j, 2]) & 0xFF, int(got[i, j, 0]), int(got[i, j, 1])) == (t, st, ln)


def test_c5_full_phase_on_device(ctx):
    """C5: `when` gates + 4 authz configs + response headers on the device against the
    same phase through the oracle (headers compared byte for byte)."""
    from test_pipeline_host import OracleCtx

    from authorino_amd import pipeline as P
    from authorino_amd import workloads

    w = workloads.make("c5", n=3000, seed=53)
    docs = [w.doc(i) for i in range(w.n)]
    got = P.AuthPipelineBatch(w.auth_config, ctx=ctx).evaluate(docs)
    want = P.AuthPipelineBatch(w.auth_config, ctx=OracleCtx()).evaluate(docs)
    n_ok = 0
    for g, o in zip(got, want):
        assert (g.code, g.message, g.skipped, g.denied_by, g.authorization, g.headers, g.metadata) == \
               (o.code, o.message, o.skipped, o.denied_by, o.authorization, o.headers, o.metadata)
        n_ok += bool(g.headers)
    assert 0 < n_ok < w.n


def test_denywith_and_cache_on_device(ctx):
    """denyWith (auth_pipeline.go:581-608) and evaluator-cache keys (authorization.go:56-76)
    resolved by the device select kernel on C5 documents, against the same phase through
    the oracle: status, message, body and headers of every denied request byte for byte,
    and the cache-granted objects (tests/test_denywith_cache_host.py has the host cases)."""
    import dataclasses

    from test_pipeline_host import OracleCtx

    from authorino_amd import cache as CA
    from authorino_amd import pipeline as P
    from authorino_amd import workloads
    from authorino_amd.response import JSONValue

    w = workloads.make("c5", n=3000, seed=57)
    docs = [w.doc(i) for i in range(w.n)]

    def config():
        clk = lambda: 1000.0  # noqa: E731
        authz = list(w.auth_config.authorization)
        authz[0] = dataclasses.replace(authz[0], cache=CA.EvaluatorCache(
            JSONValue(pattern="{auth.metadata.tenant}:{auth.identity.sub}"), 60, clock=clk))
        authz[-1] = dataclasses.replace(authz[-1], cache=CA.EvaluatorCache(
            JSONValue(pattern="auth.metadata.tenant"), 60, clock=clk))
        dw = P.DenyWithValues(
            code=302,
            message=JSONValue(pattern="denied {auth.identity.sub} on {context.request.http.path}"),
            body=JSONValue(pattern="auth.identity.realm_access.roles"),
            headers=[("Location", JSONValue(pattern="https://login/?to=https://{context.request.http.host}"
                                                    "{context.request.http.path}")),
                     ("X-Exp", JSONValue(pattern="auth.identity.exp")),
                     ("X-Static", JSONValue(static="s"))])
        return dataclasses.replace(w.auth_config, authorization=authz, unauthorized=dw)

    got = P.AuthPipelineBatch(config(), ctx=ctx).evaluate(docs)
    want = P.AuthPipelineBatch(config(), ctx=OracleCtx()).evaluate(docs)
    n_denied = 0
    for g, o in zip(got, want):
        assert (g.code, g.status, g.message, g.body, g.deny_headers, g.undecided, g.authorization, g.headers) == \
               (o.code, o.status, o.message, o.body, o.deny_headers, o.undecided, o.authorization, o.headers)
        n_denied += g.code == P.CODE_PERMISSION_DENIED
    assert 0 < n_denied < w.n


def test_forest_matches_single_rulesets(ctx):
    """authjx_compile_forest: every tree of the C5 phase (+ c2's rules and a tree with a
    static regex error) in one ruleset, one scan per document; per-tree results, error
    indices (forest numbering) and pattern bits equal the trees compiled one by one, which
    the oracle pins."""
    from authorino_amd import jsonexp as J
    from authorino_amd import workloads

    w = workloads.make("c5", n=20000, seed=54)
    cfg = w.auth_config
    exprs = [cfg.conditions] + [e for c in cfg.authorization for e in (c.conditions, c.rules)]
    exprs += [workloads.c2_expression(), J.Any(J.Pattern("auth.identity.sub", J.EqualOperator, "user-0042"),
                                               J.Pattern("context.request.http.path", J.RegexOperator, "(["))]
    forest = ctx.compile_forest(exprs)
    assert forest.n_trees == len(exprs)
    ftri, ferr, fbm = ctx.eval_host_arena([forest], w.arena, w.offs, w.lens)
    assert ftri.shape == (w.n, len(exprs))
    bits = np.unpackbits(fbm.view(np.uint8), axis=1, bitorder="little")
    for k, e in enumerate(exprs):
        rs = ctx.compile_expression(e)
        tri, err, bm = ctx.eval_host_arena([rs], w.arena, w.offs, w.lens)
        off = forest.offsets[k]
        assert np.array_equal(ftri[:, k], tri), k
        assert np.array_equal(ferr[:, k], np.where(err >= 0, err + off, -1)), k
        tb = np.unpackbits(bm.view(np.uint8), axis=1, bitorder="little")[:, :rs.n_patterns]
        assert np.array_equal(bits[:, off:off + rs.n_patterns], tb), k
        if k < 3 or k == len(exprs) - 1:
            otri, oerr, _ = _oracle(e, w.arena, w.offs, w.lens)
            assert np.array_equal(tri, otri) and np.array_equal(err, oerr), k
    assert (ftri[:, -1] == 2).any()  # the static error decides some requests


def test_select_from_eval_matches_select_batch(ctx):
    """C5 response selectors compiled as the forest's last tree: their spans read from the
    evaluation's capture rows equal authjx_select_batch_device's (its own scan), including
    requests the single-pass kernel hands to the exact path; the phase trees' results do
    not change; rows of another evaluation are refused."""
    import torch

    from authorino_amd import runtime, workloads
    from authorino_amd.response import ResponseSelectors

    w = workloads.make("c5", n=8192, seed=57)
    cfg = w.auth_config
    exprs = [cfg.conditions] + [e for c in cfg.authorization for e in (c.conditions, c.rules)]
    sel = ResponseSelectors(cfg.response, ctx)
    plain = ctx.compile_forest(exprs)
    fused = ctx.compile_forest(exprs, extra_selectors=sel.paths)
    k = len(sel.paths)
    assert fused.n_patterns == plain.n_patterns + k and fused.n_trees == plain.n_trees + 1
    arena = w.arena.copy()
    cut = np.arange(0, w.n, 97)
    arena[(w.offs[cut] + w.lens[cut] - 1).astype(np.int64)] = ord(" ")  # truncated: exact path
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(arena).to(dev)
    Of = torch.from_numpy(w.offs.view(np.int64)).to(dev)
    Ln = torch.from_numpy(w.lens.view(np.int32)).to(dev)

    def run(rs):
        tri = torch.empty(w.n * rs.n_trees, dtype=torch.uint8, device=dev)
        bm = torch.empty((w.n, (rs.n_patterns + 63) // 64), dtype=torch.int64, device=dev)
        ctx.eval_device([rs], A, Of, Ln, tri, None, bm)
        return tri

    tri_f = run(fused)
    got = torch.empty((w.n, k, 3), dtype=torch.int32, device=dev)
    ctx.select_from_eval_device(fused, fused.n_patterns - k, A, Of, Ln, got)
    torch.cuda.synchronize()
    assert ctx.last_exact_count() >= len(cut)
    want = torch.empty((w.n, k, 3), dtype=torch.int32, device=dev)
    ctx.select_device([sel.ruleset], A, Of, Ln, want)
    tri_p = run(plain)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want.cpu().numpy())
    tf = tri_f.cpu().numpy().reshape(w.n, fused.n_trees)
    assert np.array_equal(tf[:, :plain.n_trees], tri_p.cpu().numpy().reshape(w.n, plain.n_trees))
    assert (tf[:, -1] == runtime.T).all()
    with pytest.raises(runtime.AuthjxError):  # the rows are the plain forest's now
        ctx.select_from_eval_device(fused, fused.n_patterns - k, A, Of, Ln, got)


@pytest.mark.parametrize("mode", [0])
def test_kernels_match_oracle(ctx, mode):
    """The single-pass kernel on the c2 / c3 workloads, random and malformed documents (and
    c4's multi-tenant kernel): the same outputs as the oracle."""
    import fuzz_util as FU
    from authorino_amd import workloads as W

    ctx.set_kernel_mode(mode)
    try:
        for workload, n in (("c2", 50000), ("c3", 20000)):
            w = W.make(workload, n=n, seed=31)
            rs = ctx.compile_expression(w.expr)
            tri, err, bm = ctx.eval_host_arena([rs], w.arena, w.offs, w.lens)
            assert ctx.last_exact_count() == 0  # every synthetic document stayed on the fast path
            otri, oerr, obm = _oracle(w.expr, w.arena, w.offs, w.lens)
            assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)
        if True:
            w = W.make("c4", n=30000, seed=32)
            rss = [ctx.compile_expression(e) for e in w.exprs]
            tri, err, bm = ctx.eval_host_arena(rss, w.arena, w.offs, w.lens, set_of_req=w.set_of_req)
            osets = [O.Ruleset.from_expression(e) for e in w.exprs]
            otri, oerr, obm = _oracle(None, w.arena, w.offs, w.lens, set_of_req=w.set_of_req, sets=osets)
            assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)
        rng = np.random.default_rng(78)
        for _ in range(20):
            pats = FU.rand_patterns(rng, int(rng.integers(1, 10)))
            nodes, root = FU.chain(len(pats))
            ors = O.Ruleset(pats, nodes, root)
            docs = [FU.mutate(rng, d) if rng.random() < 0.3 else d for d in
                    (FU.rand_doc(rng, ws=False) for _ in range(300))]
            if any(ors.pattern(p, docs[0]) == O.UNSUPPORTED for p in range(len(pats))):
                continue
            rs = ctx.compile(pats, nodes, root)
            tri, err, bm = ctx.eval_host([rs], docs)
            lens = np.array([len(d) for d in docs], dtype=np.uint32)
            offs = np.zeros(len(docs), dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1])
            arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
            otri, oerr, obm = O.eval_batch([ors], arena, offs, lens)
            assert (tri == 3).sum() == 0
            assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)
    finally:
        ctx.set_kernel_mode(0)


def test_hard_numbers_on_device(ctx):
    """Go-marshalled float64 values (16-17 significant digits), subnormals, the 1e21
    boundary and the float64 ends as selected values: the single-pass kernel hands those
    requests to the exact scan, which decides them (ajx_float.h); every result equals the
    oracle and none is UNDECIDED."""
    rng = np.random.default_rng(91)
    pats = [("geo.lat", 1, "37.77492950000001"), ("geo.lon", 2, "-122.4194155"), ("score", 1, "0.30000000000000004"),
            ("big", 1, "1000000000000000000000"), ("tiny", 1, "0.000001"), ("v", 4, "^-?[0-9]+\\.[0-9]{15,}$")]
    nodes = [(0, -1, -1, i) for i in range(len(pats))]
    root = -1
    for i in reversed(range(len(pats))):
        nodes.append((2 if i % 2 else 1, i, root, -1))
        root = len(nodes) - 1
    ors = O.Ruleset(pats, nodes, root)
    rs = ctx.compile(pats, nodes, root)
    docs = []
    for _ in range(3000):
        f = float(rng.standard_normal() * 10.0 ** int(rng.integers(-12, 12)))
        g = float(np.frombuffer(rng.integers(0, 2**63, dtype=np.int64).tobytes(), dtype=np.float64)[0])
        if not np.isfinite(g):
            g = 1.5
        vals = {"geo": {"lat": repr(37.77492950000001 if rng.random() < 0.5 else f), "lon": repr(-122.41941550000001)},
                "score": repr(0.1 + 0.2 if rng.random() < 0.5 else f), "big": ["1e21", "9.999999999999999e20",
                                                                            "1.7976931348623157e308"][int(rng.integers(0, 3))],
                "tiny": ["1e-6", "1e-7", "4.9406564584124654e-324", "2.2250738585072014e-308"][int(rng.integers(0, 4))],
                "v": repr(g)}
        doc = ('{"geo":{"lat":%s,"lon":%s},"score":%s,"big":%s,"tiny":%s,"v":%s}'
               % (vals["geo"]["lat"], vals["geo"]["lon"], vals["score"], vals["big"], vals["tiny"], vals["v"]))
        docs.append(doc.encode())
    tri, err, bm = ctx.eval_host([rs], docs)
    assert ctx.last_exact_count() > 0  # hard numbers went through the exact scan
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
    otri, oerr, obm = O.eval_batch([ors], arena, offs, lens)
    assert (tri == 3).sum() == 0
    assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)
    assert len(set(tri.tolist())) > 1


def test_micro_batcher_concurrent_producers():
    """8 producer threads x 10^4 requests through three micro-batchers: two on one
    context (two streams, so two workspaces of that context run concurrently) and one on
    a second context; mixed AuthConfigs (c4's rulesets): every result equals the oracle;
    the batchers formed multi-request batches."""
    import threading

    from authorino_amd import runtime
    from authorino_amd import workloads as W

    w = W.make("c4", n=4000, seed=41)
    ctxs = [runtime.Context(0), runtime.Context(0)]
    used = [int(x) for x in np.unique(w.set_of_req)]
    sets = [{k: c.compile_expression(w.exprs[k]) for k in used} for c in ctxs]
    osets = [O.Ruleset(*flat(w.exprs[k])) for k in used]
    remap = np.zeros(int(w.set_of_req.max()) + 1, dtype=np.uint32)
    remap[used] = np.arange(len(used), dtype=np.uint32)
    otri, oerr, _ = O.eval_batch(osets, w.arena, w.offs, w.lens, set_of_req=remap[w.set_of_req], nthreads=8)
    batchers = [runtime.Batcher(ctxs[k], max_batch=2048, window_us=300) for k in (0, 0, 1)]
    bad = []

    def producer(t):
        b = batchers[t % 3]
        cs = sets[0 if t % 3 < 2 else 1]
        rng = np.random.default_rng(1000 + t)
        for _ in range(10000):
            i = int(rng.integers(0, w.n))
            tri, err = b.eval(cs[int(w.set_of_req[i])], w.doc(i))
            if tri[0] != otri[i] or err[0] != oerr[i]:
                bad.append((t, i, tri, err, int(otri[i]), int(oerr[i])))

    ts = [threading.Thread(target=producer, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    stats = [b.stats() for b in batchers]
    for b in batchers:
        b.close()
    assert not bad, bad[:5]
    assert sum(s["requests"] for s in stats) == 80000
    assert all(s["max_batch_seen"] > 1 for s in stats)


def test_pipeline_sets_aside_undecided_requests():
    """A request whose selected value is a hex number literal (never valid JSON; gjson
    still reads it as a number) is left undecided by the device: the pipeline marks that
    request only (AuthResult.undecided) and decides the others of the batch."""
    from authorino_amd import jsonexp, pipeline

    rules = jsonexp.Pattern("a", jsonexp.Operator.EqualOperator, "0")
    cfg = pipeline.AuthConfig(authorization=[pipeline.AuthorizationConfig("r", rules=rules)])
    p = pipeline.AuthPipelineBatch(cfg)
    res = p.evaluate([b'{"a":0x10}', b'{"a":0}', b'{"a":1}'])
    assert res[0].undecided and res[0].code == pipeline.CODE_UNKNOWN
    assert not res[1].undecided and res[1].code == pipeline.CODE_OK
    assert not res[2].undecided and res[2].code == pipeline.CODE_PERMISSION_DENIED


def test_count_selectors_on_device(ctx):
    """`#` selectors through the C-ABI — element counts and "#." lists: pattern results
    and selected values (AUTHJX_VALUE_COUNT; lists are not selectable) against the
    oracle (tests/test_count_selector.py)."""
    import fuzz_util as FU
    from test_count_selector import rand_count_patterns

    rng = np.random.default_rng(1300)
    checked = 0
    for _ in range(25):
        pats = rand_count_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        ors = O.Ruleset(pats, nodes, root)
        docs = [FU.rand_doc(rng) for _ in range(300)]
        if any(ors.pattern(p, docs[0]) == O.UNSUPPORTED for p in range(len(pats))):
            continue
        rs = ctx.compile(pats, nodes, root)
        tri, err, bm = ctx.eval_host([rs], docs)
        lens = np.array([len(d) for d in docs], dtype=np.uint32)
        offs = np.zeros(len(docs), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1])
        arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
        otri, oerr, obm = O.eval_batch([ors], arena, offs, lens)
        assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)
        vals = ctx.select_host_arena([rs], arena, offs, lens)
        for r in range(0, len(docs), 7):
            for p, (sel, _, _) in enumerate(pats):
                st, ln, t = (int(x) for x in vals[r][p])
                ot, _, os_ = O.gjson_get(docs[r], sel.encode())
                if t == 255:  # a "#." list: a built text, not selectable (AUTHJX_JSON_UNSUPPORTED)
                    assert (sel.startswith("#.") or ".#." in sel) and ot == O.T_JSON, sel
                    continue
                if t >> 8 == 2:
                    assert ot == O.T_NUMBER and os_ == str(st).encode(), (sel, docs[r])
                else:
                    assert (t & 0xFF) == ot, (sel, docs[r])
        checked += len(docs)
    assert checked > 3000
