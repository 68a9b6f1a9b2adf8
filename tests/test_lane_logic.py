"""CPU differential tests of the lane kernel's scanner (authorino_amd/csrc/ajx_lane.h, host
build with the kernel's window staging, tests/native/lane_host.cpp) against the oracle: per-pattern tri-states and the fold on the BASELINE workload documents (every one
must take the lane path), random compact documents, long values across windows and
malformed / non-compact documents (which must either match the oracle or be handed to
the exact scan)."""
import json

import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O


def _check(rs, wr, pats, d, mis=0, fill=0x41):
    ot = [rs.pattern(p, d) for p in range(len(pats))]
    if O.UNSUPPORTED in ot:
        return None
    t, _, res, _ = wr.eval(d, mis=mis, fill=fill)
    if t == -2:
        return None
    if t >= 0 and 3 not in res:
        assert res == ot, (pats, d, mis)
        assert t == rs.matches(d)[0], (pats, d, mis)
        return True
    return False


@pytest.mark.parametrize("workload", ["c1", "c2", "c3", "c5"])
def test_lane_workload_documents(workload):
    from authorino_amd import workloads as W

    w = W.make(workload, n=120 if workload != "c5" else 40, seed=12)
    pats, nodes, root = w.expr.flatten()
    pl = [(p.selector, int(p.operator), p.value) for p in pats]
    rs = O.Ruleset(pl, nodes, root)
    wr = H.LaneRuleset(pl, nodes, root)
    assert wr.ok
    for i in range(w.n):
        d = w.doc(i)
        t, _, res, _ = wr.eval(d, mis=int(w.offs[i]) % 16)
        assert t >= 0, (workload, i, d[:200])
        assert res == [rs.pattern(p, d) for p in range(len(pl))], (workload, i)
        assert t == rs.matches(d)[0]


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_lane_random_compact_documents(seed):
    rng = np.random.default_rng(500 + seed)
    n_lane = n_all = 0
    for _ in range(25):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 7)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        wr = H.LaneRuleset(pats, nodes, root)
        for _ in range(12):
            d = FU.rand_doc(rng, ws=False)
            r = _check(rs, wr, pats, d, mis=int(rng.integers(0, 16)))
            if r is None:
                continue
            n_all += 1
            n_lane += bool(r)
    assert n_all > 100 and n_lane > 0.5 * n_all, (n_lane, n_all)


@pytest.mark.parametrize("seed", [0, 1])
def test_lane_long_values_across_chunks(seed):
    rng = np.random.default_rng(600 + seed)
    n_lane = n_all = 0
    for _ in range(30):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        wr = H.LaneRuleset(pats, nodes, root)
        for _ in range(6):
            d = FU.long_doc(rng, pats)
            d = d[:1] + b'"pad":"' + b"x" * int(rng.integers(0, 2100)) + b'",' + d[1:] if len(d) > 2 else d
            r = _check(rs, wr, pats, d, mis=int(rng.integers(0, 16)))
            if r is None:
                continue
            n_all += 1
            n_lane += bool(r)
    assert n_all > 60 and n_lane > 0.4 * n_all, (n_lane, n_all)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lane_malformed_documents(seed):
    """Mutated documents: the lane path either equals the oracle or hands over."""
    rng = np.random.default_rng(700 + seed)
    for _ in range(20):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        wr = H.LaneRuleset(pats, nodes, root)
        for _ in range(15):
            d = FU.mutate(rng, FU.rand_doc(rng, ws=False))
            _check(rs, wr, pats, d, mis=int(rng.integers(0, 16)), fill=int(rng.choice([0x41, 0x22, 0x7D, 0x2C])))


def test_lane_edge_documents():
    pats = [("a", 1, "1"), ("a.b", 1, "x"), ("c.0", 1, "y"), ("d", 3, "z")]
    nodes, root = FU.chain(len(pats))
    rs = O.Ruleset(pats, nodes, root)
    wr = H.LaneRuleset(pats, nodes, root)
    docs = [b"", b"{", b"[", b"{}", b"[]", b"null", b'"x"', b"{]", b"[}", b'{"a":1}', b'{"a":1,}', b'{"a" :1}',
            b'{"a":1}x', b'{"a":1}}', b'{"a":"k":1}', b'{"a","b":1}', b'["a":1]', b'{"a":1 ,"b":2}',
            b'{"a":tru}', b'{"a":true1}', b'{"a":nul}', b'{"a":-}', b'{"c":["y",1]}', b'{"d":["z"]}',
            b'{"a":{"b":"x"},"a":1}', b'{"a":1,"a":{"b":"x"}}', b'{"a\\u0062":1}', b'{"a":"x\\"y"}',
            b'{"\\u0061":"1"}', b'[{"a":1}]', b'{"a":[1,2,{"b":"x"}]}', b'{"c":{"0":"y"}}', b'{"a":1}\n']
    for d in docs:
        r = _check(rs, wr, pats, d)
        assert r is not None
