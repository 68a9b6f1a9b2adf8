"""CPU differential fuzz: oracle vs the kernels' per-document logic (host build):
the exact scan (gj_get) and the single-pass path (fast_eval) on random documents,
random selector sets (escaped keys, array indices, duplicates) and malformed bytes."""
import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O


def _chain(n):
    nodes = [(0, -1, -1, i) for i in range(n)]
    root = -1
    for i in reversed(range(n)):
        nodes.append((1, i, root, -1))
        root = len(nodes) - 1
    return nodes, root


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_fuzz_scan_and_fast_match_oracle(seed):
    rng = np.random.default_rng(seed)
    n_fast = 0
    for _ in range(120):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(15):
            d = FU.rand_doc(rng)
            if rng.random() < 0.4:
                d = FU.mutate(rng, d)
            ot = [rs.pattern(p, d) for p in range(len(pats))]
            if O.UNSUPPORTED in ot:
                continue
            t_or, _ = rs.matches(d)
            ts, _, sres = hr.eval(d)
            if 3 not in sres:
                assert sres == ot, (pats, d)
                assert ts == t_or, (pats, d)
            tf, _, fres = H.eval_fast(hr, d, mis=int(rng.integers(0, 16)))
            if tf >= 0 and 3 not in fres:
                n_fast += 1
                assert fres == ot, (pats, d)
                assert tf == t_or, (pats, d)
    assert n_fast > 300


@pytest.mark.parametrize("seed", [10, 11])
def test_fuzz_fast_whitespace_runs(seed):
    """Single-pass path on valid documents with long whitespace runs between tokens."""
    rng = np.random.default_rng(seed)
    n_fast = 0
    for _ in range(150):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(8):
            d = FU.rand_doc_ws(rng)
            ot = [rs.pattern(p, d) for p in range(len(pats))]
            if O.UNSUPPORTED in ot:
                continue
            tf, _, fres = H.eval_fast(hr, d, mis=int(rng.integers(0, 16)))
            if tf >= 0 and 3 not in fres:
                n_fast += 1
                assert fres == ot, (pats, d)
    assert n_fast > 300


@pytest.mark.parametrize("seed", [0, 1])
def test_fast_long_values_across_windows(seed):
    """Long keys / values / arrays placed at random offsets so that tokens, key tails and
    scalars straddle the single-pass scanner's 64-byte windows."""
    rng = np.random.default_rng(300 + seed)
    n_fast = n_all = 0
    for _ in range(60):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(10):
            d = FU.long_doc(rng, pats)
            ot = [rs.pattern(p, d) for p in range(len(pats))]
            if O.UNSUPPORTED in ot:
                continue
            t_or, _ = rs.matches(d)
            tf, _, fres = H.eval_fast(hr, d, mis=int(rng.integers(0, 16)))
            if tf == -2:
                continue
            n_all += 1
            if tf >= 0 and 3 not in fres:
                n_fast += 1
                assert fres == ot, (pats, d)
                assert tf == t_or, (pats, d)
    assert n_all > 200 and n_fast > 0.4 * n_all, (n_fast, n_all)


@pytest.mark.parametrize("workload", ["c1", "c2", "c3"])
def test_fast_workload_documents(workload):
    from authorino_amd import workloads as W

    w = W.make(workload, n=300, seed=12)
    pats, nodes, root = w.expr.flatten()
    pl = [(p.selector, int(p.operator), p.value) for p in pats]
    rs = O.Ruleset(pl, nodes, root)
    hr = H.HostRuleset(pl, nodes, root)
    for i in range(w.n):
        d = bytes(w.arena[w.offs[i]:w.offs[i] + w.lens[i]])
        tf, _, fres = H.eval_fast(hr, d, mis=int(w.offs[i]) % 16)
        assert tf >= 0, (workload, i)
        assert fres == [rs.pattern(p, d) for p in range(len(pl))]
        assert tf == rs.matches(d)[0]
