"""GPU tests of SURVEY.md §8 f2 on the device: selectors with the reference's gjson
modifiers and "#." lists as VALUES — response headers, denyWith and evaluator-cache keys
(pkg/json/json.go:41-53, :96-151, :161-264; pkg/evaluators/authorization.go:56-66;
pkg/service/auth_pipeline.go:581-608). The select kernel's TEXT instance builds each
such value (authjx_select_text_batch[_device]) into the request's text slot; the bytes
and types are compared with the oracle's gjson.Get with the same modifiers."""
import collections
import json
import random

import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from authorino_amd import runtime

    return runtime.Context(0)


def _pack(blobs):
    lens = np.array([len(b) for b in blobs], dtype=np.uint32)
    offs = np.zeros(len(blobs), dtype=np.uint64)
    if len(blobs):
        offs[1:] = np.cumsum(lens[:-1])
    return np.frombuffer(b"".join(blobs) + b"\0", dtype=np.uint8), offs, lens


def _check(vals, text, k, j, d, want):
    st, ln, tt = (int(x) for x in vals[k, j])
    src = text[k].tobytes() if (tt >> 8) & 4 else d
    t, raw = want
    assert (tt & 0xFF, src[st:st + ln]) == (t, raw), (d[:200], k, j)
    return ln if (tt >> 8) & 4 else 0


def _check_request(vals, text, k, d, wants, stride, counts):
    """Request k's values in slot order: each equals the oracle's, or is UNDECIDED (255)
    for the one reason the select kernel has on these inputs — its built text does not
    fit what is left of the request's text slot (`stride` bytes). counts: tallies."""
    used = 0
    for j, want in enumerate(wants):
        if want is None:  # (the oracle restates @case / @strip for ASCII text only:
            counts["skipped"] += 1  # tests/test_unicode_case.py pins the Unicode tables)
            continue
        if (int(vals[k, j, 2]) & 0xFF) == 255:
            assert used + len(want[1]) > stride, ("undecided without a reason", d[:200], k, j, want)
            counts["undecided: text slot full"] += 1
            continue
        used += _check(vals, text, k, j, d, want)
        counts["checked"] += 1


def test_modifier_chains_as_values_match_oracle(ctx):
    """Random documents under random modifier chains (tests/test_modifiers.py's
    generator), several chains per ruleset, one request per document: every decided value
    equals the oracle's Result (type + raw text); undecided only where the oracle is."""
    from test_modifiers import _chain, _doc

    rng = random.Random(77)
    sels = []
    while len(sels) < 48:
        s = _chain(rng)
        try:
            O.gjson_get_mods(b"{}", s)
        except ValueError:
            continue
        sels.append(s)
    groups = [sels[i:i + 6] for i in range(0, len(sels), 6)]
    sets = [ctx.compile([(s, 1, "") for s in g], [], -1) for g in groups]
    assert all(st == 0 for rs in sets for st in rs.status)
    docs = [_doc(rng) for _ in range(2000)]
    sor = np.array([i % len(sets) for i in range(len(docs))], dtype=np.uint32)
    arena, offs, lens = _pack(docs)
    vals, text = ctx.select_text_host_arena(sets, arena, offs, lens, set_of_req=sor, text_stride=4096)
    checked = und = 0
    for k, d in enumerate(docs):
        for j, s in enumerate(groups[sor[k]]):
            want = O.gjson_get_mods(d, s)
            if want is None:  # (the oracle restates @case / @strip for ASCII text only:
                continue      # tests/test_unicode_case.py pins the Unicode tables)
            if (int(vals[k, j, 2]) & 0xFF) == 255:  # (rare number forms, special casing)
                und += 1
                continue
            _check(vals, text, k, j, d, want)
            checked += 1
    assert checked > 8000 and und <= checked // 5, (checked, und)


def test_lists_and_device_buffers(ctx):
    """"#." lists (built text) next to plain spans and counts through the device entry
    point on HBM-resident tensors; a text slot too small for a list leaves that value
    unresolved (255) and the plain values intact."""
    import torch

    rng = np.random.default_rng(5)
    docs = []
    for i in range(3000):
        arr = [{"k": int(x)} if x % 3 else {"j": "y"} for x in rng.integers(0, 50, int(rng.integers(0, 12)))]
        docs.append(json.dumps({"a": arr, "s": "v%d" % i, "n": {"m": [{"k": "é"}, {"k": [1, 2]}]}},
                               separators=(",", ":"), ensure_ascii=False).encode())
    paths = ["a.#.k", "s", "a.#", "n.m.#.k", "s|@case:upper", "missing.#.k"]
    rs = ctx.compile([(p, 1, "") for p in paths], [], -1)
    arena, offs, lens = _pack(docs)
    dev = torch.device("cuda:0")
    A = torch.from_numpy(arena.copy()).to(dev)
    Of = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    Ln = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
    for stride in (1024, 16):
        out = torch.zeros((len(docs), len(paths), 3), dtype=torch.int32, device=dev)
        text = torch.zeros((len(docs), stride), dtype=torch.uint8, device=dev)
        ctx.select_text_device([rs], A, Of, Ln, out, text)
        torch.cuda.synchronize()
        vals = out.cpu().numpy().view(np.uint32)
        tx = text.cpu().numpy()
        for k, d in enumerate(docs):
            used = 0
            for j, p in enumerate(paths):
                t, raw, string = O.gjson_get(d, p) if "@" not in p else (*O.gjson_get_mods(d, p), None)
                st, ln, tt = (int(x) for x in vals[k, j])
                if (tt >> 8) == 2:  # an element count (AUTHJX_VALUE_COUNT)
                    assert t == 2 and string == str(st).encode()
                    continue
                built = "#." in p or "@" in p
                if built and raw and used + len(raw) > stride:
                    assert (tt & 0xFF) == 255, (stride, k, p)
                    continue
                _check(vals, tx, k, j, d, (t, raw))
                if built and raw:
                    used += len(raw)


def test_reference_templates_on_device(ctx):
    """ReplaceJSONPlaceholders' cases with modifiers (json_test.go:165-169, :180-187)
    through ResponseSelectors on the device."""
    from authorino_amd import response as R
    from test_response_host import DOC

    cases = [("Username: {auth.identity.username.@case:upper}", "Username: JOHN"),
             ('Domain: {auth.identity.email.@extract:{"sep":"@","pos":1}}', "Domain: test"),
             (r'Github username: {auth.identity.github\.com|@extract:{"sep":"/","pos":3}|@case:upper}',
              "Github username: JOHN"),
             (r'\{"msg":"I can build a JSON with dynamic values","username":"{auth.identity.github\.com|'
              r'@extract:{"sep":"/","pos":3}|@case:upper}"\}',
              '{"msg":"I can build a JSON with dynamic values","username":"JOHN"}'),
             ("Username: {auth.identity.username}", "Username: john")]
    cfgs = [R.ResponseConfig("r%d" % i, plain=R.JSONValue(pattern=t)) for i, (t, _) in enumerate(cases)]
    s = R.ResponseSelectors(cfgs, ctx)
    arena = np.frombuffer(DOC + b"\0", dtype=np.uint8)
    sel = s.resolve([DOC], arena, np.zeros(1, np.uint64), np.array([len(DOC)], np.uint32))
    assert [s.call(c, DOC, sel[0]) for c in cfgs] == [w for _, w in cases]


def test_denywith_and_cache_keys_with_modifiers_on_device(ctx):
    """The same denyWith / cache-key configuration as
    tests/test_denywith_cache_host.py::test_modifier_value_selectors_resolve_to_built_text,
    through the kernels: identical results to the oracle stand-in."""
    from authorino_amd import cache as CA
    from authorino_amd import jsonexp as J
    from authorino_amd import pipeline as P
    from authorino_amd.response import JSONValue
    from test_denywith_cache_host import _deny_all, _req
    from test_pipeline_host import OracleCtx

    def cfg():
        dw = P.DenyWithValues(message=JSONValue(pattern="auth.identity.tenant.@case:upper"),
                              body=JSONValue(pattern='{auth.identity.sub|@extract:{"sep":"i","pos":0}}-'
                                                     '{auth.identity.roles.#.x}'),
                              headers=[("X-Roles", JSONValue(pattern="auth.identity.roles|@case:upper"))])
        return P.AuthConfig(authorization=[_deny_all()], unauthorized=dw)

    docs = [_req(sub="s%d" % i, tenant="t%d" % (i % 7), roles=("r%d" % i, "x")) for i in range(300)]
    docs.append(_req(sub="bob", tenant="zeta").replace(b'"zeta"', '"straße"'.encode()))  # (SpecialCasing)
    got = P.AuthPipelineBatch(cfg(), ctx=ctx).evaluate(docs)
    want = P.AuthPipelineBatch(cfg(), ctx=OracleCtx()).evaluate(docs[:-1])
    key = lambda r: (r.code, r.undecided, r.message, r.body, r.deny_headers, r.status)  # noqa: E731
    assert [key(r) for r in got[:-1]] == [key(r) for r in want]
    assert got[0].message == "T0"
    # (the oracle restates @case for ASCII only; Go's strings.ToUpper keeps ß: simple mapping)
    assert not got[-1].undecided and got[-1].message == "STRAßE", key(got[-1])
    cache_cfg = lambda: P.AuthorizationConfig(  # noqa: E731
        "c", rules=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice")),
        cache=CA.EvaluatorCache(JSONValue(pattern="{auth.identity.tenant|@case:lower}/{auth.identity.sub}"), 60))
    c = cache_cfg()
    res = P.AuthPipelineBatch(P.AuthConfig(authorization=[c]), ctx=ctx).evaluate([_req(tenant="ACME")])
    assert res[0].code == P.CODE_OK and c.cache.get("acme/alice") is True


def test_fromstr_and_tails_on_device(ctx):
    """gjson's @fromstr and a path after a modifier (validating-webhook.md:156,
    json_test.go:247-257) through the kernels: selected values (type + raw) and pattern
    results (eq / neq / incl against values from the documents, T bitmap and tri-state)
    equal the oracle's on AdmissionReview-shaped, malformed and scalar bodies."""
    from authorino_amd import runtime
    from test_fromstr import PATHS, _fromstr_doc, _jwt_doc

    rng = random.Random(99)
    docs = [_fromstr_doc(rng) for _ in range(3000)] + [_jwt_doc()]
    arena, offs, lens = _pack(docs)
    rs = ctx.compile([(p, 1, "") for p in PATHS], [], -1)
    assert rs.status == [0] * len(PATHS)
    vals, text = ctx.select_text_host_arena([rs], arena, offs, lens, text_stride=8192)
    counts = collections.Counter()
    for k, d in enumerate(docs):
        _check_request(vals, text, k, d, [O.gjson_get_mods(d, p) for p in PATHS], 8192, counts)
    print(dict(counts))
    assert counts["checked"] > 25000, counts
    jwt = 'access_token.@extract:{"pos":1}|@extract:{"sep":".","pos":1}|@base64:decode|@fromstr'
    pats = [(PATHS[1], 1, "authorino"), (PATHS[1], 2, "authorino"), (PATHS[3], 1, "AdmissionReview"),
            (PATHS[2], 3, "AdmissionReview"), (PATHS[0], 1, ""), (PATHS[7], 1, "5"), (PATHS[9], 1, "v"),
            (PATHS[4], 1, "DEFAULT"), (jwt + ".exp", 1, "1685557675"), (jwt + ".aud", 3,
                                                                          "https://kubernetes.default.svc.cluster.local")]
    nodes = [(0, -1, -1, i) for i in range(len(pats))]
    root = -1
    for i in reversed(range(len(pats))):
        nodes.append((2, i, root, -1))  # (an Or chain: every pattern is evaluated)
        root = len(nodes) - 1
    dev = ctx.compile(pats, nodes, root)
    orc = O.Ruleset(pats, nodes, root)
    tri, _, bm = ctx.eval_host_arena([dev], arena, offs, lens)
    otri, _, obm = O.eval_batch([orc], arena, offs, lens, nthreads=8)
    # (every request decided by both, identically: the host build of the same code decides
    # all of them, tests/test_fromstr.py)
    print({"undecided": int((tri == runtime.UNDECIDED).sum()), "oracle undecided": int((otri == runtime.UNDECIDED).sum())})
    assert np.array_equal(tri, otri) and np.array_equal(bm, obm)
    assert (bm[-1, 0] >> 8) & 1 and (bm[-1, 0] >> 9) & 1  # (the JWT claims)


def test_unicode_case_and_strip_on_device(ctx):
    """@case / @strip on non-ASCII and invalid UTF-8 text through the kernels (the Unicode
    tables of ajx_unicode.h in device memory) against tests/test_unicode_case.py's Go
    restatement; SpecialCasing / unassigned code points UNDECIDED (255)."""
    from test_unicode_case import _raw_string

    rng = random.Random(6200)
    raws = [_raw_string(rng) for _ in range(3000)]
    docs = [b'{"s":' + r + b',"n":1}' for r in raws]
    rs = ctx.compile([(p, 1, "") for p in UNICODE_PATHS], [], -1)
    arena, offs, lens = _pack(docs)
    vals, text = ctx.select_text_host_arena([rs], arena, offs, lens, text_stride=2048)
    counts = check_unicode_values(vals, text, raws)
    print(dict(counts))
    assert counts["decided"] > 5000 and counts["undecided: SpecialCasing or unassigned"] > 100, counts


UNICODE_PATHS = ["s.@case:upper", "s|@case:lower", "s.@strip"]


def check_unicode_values(vals, text, raws):
    """Values of UNICODE_PATHS on documents {"s":raw,"n":1}: each equals the Go
    restatement's (tests/test_unicode_case.py) byte for byte, or is UNDECIDED exactly where
    that restatement declines (SpecialCasing, code points unassigned in its tables)."""
    from test_unicode_case import Undecided, go_case, go_strip

    fns = [lambda r: go_case(r, True), lambda r: go_case(r, False), go_strip]
    counts = collections.Counter()
    for k, raw in enumerate(raws):
        doc = b'{"s":' + raw + b',"n":1}'
        for j, f in enumerate(fns):
            try:
                want = f(raw)
            except Undecided:
                assert (int(vals[k, j, 2]) & 0xFF) == 255, (UNICODE_PATHS[j], raw)
                counts["undecided: SpecialCasing or unassigned"] += 1
                continue
            st, ln, tt = (int(x) for x in vals[k, j])
            assert (tt & 0xFF) == 3, (UNICODE_PATHS[j], raw, vals[k, j])
            got = (text[k].tobytes() if (tt >> 8) & 4 else doc)[st:st + ln]
            assert got == want, (UNICODE_PATHS[j], raw, got, want)
            counts["decided"] += 1
    return counts
