"""CPU differential tests of the event scanner (authorino_amd/csrc/ajx_events.h, stage A
of the default single-pass kernel; host build in tests/native/host_eval.cpp) against the
oracle and against the token scanner (ajx_fast.h): per-pattern tri-states, the fold and
the capture rows, on random compact documents, malformed bytes, values straddling the
64-byte windows and the BASELINE workload documents (every one must stay on the
single-pass path)."""
import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O


def _check(rs, hr, pats, d, mis):
    """Event path vs the oracle; returns True when the event path decided the request."""
    ot = [rs.pattern(p, d) for p in range(len(pats))]
    if O.UNSUPPORTED in ot:
        return None
    te, _, eres, _ = H.eval_ev(hr, d, mis=mis)
    if te == -2:
        return None
    if te >= 0 and 3 not in eres:
        assert eres == ot, (pats, d, mis)
        assert te == rs.matches(d)[0], (pats, d, mis)
        return True
    return False


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_events_random_compact_documents(seed):
    rng = np.random.default_rng(700 + seed)
    n_ev = n_all = 0
    for _ in range(120):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(15):
            d = FU.rand_doc(rng, ws=False)
            r = _check(rs, hr, pats, d, int(rng.integers(0, 16)))
            if r is None:
                continue
            n_all += 1
            n_ev += bool(r)
    assert n_all > 1000 and n_ev > 0.4 * n_all, (n_ev, n_all)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_events_malformed_documents(seed):
    """Mutated documents: decided ones match the oracle, the rest go to the exact scan."""
    rng = np.random.default_rng(800 + seed)
    n_all = 0
    for _ in range(100):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(20):
            d = FU.mutate(rng, FU.rand_doc(rng, ws=False))
            if _check(rs, hr, pats, d, int(rng.integers(0, 16))) is not None:
                n_all += 1
    assert n_all > 1000


@pytest.mark.parametrize("seed", [0, 1])
def test_events_long_values_across_windows(seed):
    rng = np.random.default_rng(900 + seed)
    n_ev = n_all = 0
    for _ in range(60):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(10):
            r = _check(rs, hr, pats, FU.long_doc(rng, pats), int(rng.integers(0, 16)))
            if r is None:
                continue
            n_all += 1
            n_ev += bool(r)
    assert n_all > 200 and n_ev > 0.5 * n_all, (n_ev, n_all)


@pytest.mark.parametrize("seed", [0, 1])
def test_events_capture_rows_match_token_scanner(seed):
    """Where both scanners decide a request, their capture rows are identical (spans,
    types, escape flags): the response selectors read them (authjx_select_from_eval)."""
    rng = np.random.default_rng(950 + seed)
    n = 0
    for _ in range(80):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        nodes, root = FU.chain(len(pats))
        hr = H.HostRuleset(pats, nodes, root)
        n_sel = len({p[0] for p in pats})
        for _ in range(10):
            d = FU.rand_doc(rng, ws=False) if rng.random() < 0.7 else FU.long_doc(rng, pats)
            mis = int(rng.integers(0, 16))
            te, _, eres, erow = H.eval_ev(hr, d, mis=mis, n_sel=n_sel)
            tf, _, fres, frow = H.eval_ev(hr, d, mis=mis, n_sel=n_sel, token_scanner=True)
            assert (te >= 0) == (tf >= 0), (pats, d)  # compact documents: the same requests decided
            if te >= 0:
                assert eres == fres and te == tf, (pats, d)
                found = erow[0]
                assert found == frow[0], (pats, d)
                for s in range(n_sel):
                    if (found >> s) & 1:
                        assert erow[1 + s] == frow[1 + s], (pats, d, s)
                n += 1
    assert n > 300


@pytest.mark.parametrize("workload", ["c1", "c2", "c3", "c5"])
def test_events_workload_documents(workload):
    from authorino_amd import workloads as W

    w = W.make(workload, n=200 if workload != "c5" else 40, seed=12)
    exprs = [w.expr] if w.auth_config is None else [e for c in w.auth_config.authorization for e in (c.conditions, c.rules)]
    for expr in exprs:
        pats, nodes, root = expr.flatten()
        pl = [(p.selector, int(p.operator), p.value) for p in pats]
        rs = O.Ruleset(pl, nodes, root)
        hr = H.HostRuleset(pl, nodes, root)
        for i in range(w.n):
            d = bytes(w.arena[w.offs[i]:w.offs[i] + w.lens[i]])
            te, _, eres, _ = H.eval_ev(hr, d, mis=int(w.offs[i]) % 16)
            assert te >= 0, (workload, i)
            assert eres == [rs.pattern(p, d) for p in range(len(pl))], (workload, i)
            assert te == rs.matches(d)[0]
