"""GPU: the UNDECIDED fraction on a realistic selector mix (tests/undecided_mix.py: the
selectors of the reference's user guides on Authorization-JSON documents) through the
kernels, one multi-tenant batch: 0 on ASCII documents and 0 with non-ASCII user names (é,
ß: Go's simple case mapping keeps ß, ajx_unicode.h); every request the oracle decides
equal to it, and the ones it leaves undecided (it restates @case for ASCII only) equal to
tests/test_unicode_case.py's Go restatement. Rulesets with a
by-design-unsupported form are skipped by the other random GPU tests; here they are
counted: every such pattern is one of undecided_mix.BY_DESIGN_UNSUPPORTED's forms."""
import random

import numpy as np
import pytest

import pyoracle as O
import undecided_mix as M

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from authorino_amd import runtime

    return runtime.Context(0)


def _batch(ctx, non_ascii, full=False):
    from authorino_amd import runtime

    rng = random.Random(31 + non_ascii)
    docs = [M.make_doc(rng, non_ascii=non_ascii) for _ in range(4000)]
    specs = M.make_rulesets(rng, docs[:200], k=24)
    if non_ascii:  # (not in the docs' mix: a case mapping of the user name)
        specs.append(([("auth.identity.username.@case:upper", 1, "JOHN1")], [(0, -1, -1, 0)], 0))
    dev = [ctx.compile(p, n, r) for p, n, r in specs]
    assert all(st == 0 for d in dev for st in d.status)
    orc = [O.Ruleset(p, n, r) for p, n, r in specs]
    sor = np.array(sorted(rng.randrange(len(specs)) for _ in docs), dtype=np.uint32)
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
    tri, err, bm = ctx.eval_host_arena(dev, arena, offs, lens, set_of_req=sor)
    otri, oerr, obm = O.eval_batch(orc, arena, offs, lens, set_of_req=sor, nthreads=8)
    und = tri == runtime.UNDECIDED
    ok = ~und & (otri != runtime.UNDECIDED)
    assert np.array_equal(tri[ok], otri[ok]) and np.array_equal(err[ok], oerr[ok])
    return (docs, specs, sor, und, tri, otri) if full else (docs, specs, sor, und)


def test_no_undecided_on_ascii_documents(ctx):
    _, _, _, und = _batch(ctx, False)
    assert und.sum() == 0


def test_no_undecided_under_unicode_case_mapping(ctx):
    import json

    from authorino_amd import runtime
    from test_unicode_case import go_case

    docs, specs, sor, und, tri, otri = _batch(ctx, True, full=True)
    assert und.sum() == 0, np.nonzero(und)[0][:10]
    checked = 0
    for i in np.nonzero(otri == runtime.UNDECIDED)[0].tolist():
        pats = specs[sor[i]][0]
        assert pats == [("auth.identity.username.@case:upper", 1, "JOHN1")], (pats, docs[i][:200])
        user = json.loads(docs[i])["auth"]["identity"]["username"]
        assert go_case(user.encode(), True) != b"JOHN1"  # (a name with é / ß: never equal)
        assert tri[i] == 0, (user, tri[i])
        checked += 1
    print({"requests": len(docs), "undecided": int(und.sum()), "non-ASCII @case checked against Go": checked})
    assert checked > 0


def test_by_design_unsupported_forms(ctx):
    for s in M.BY_DESIGN_UNSUPPORTED:
        assert ctx.compile([(s, 1, "x")], [(0, -1, -1, 0)], 0).status == [2], s
