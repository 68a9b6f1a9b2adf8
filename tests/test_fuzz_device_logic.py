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
