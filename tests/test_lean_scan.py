"""CPU tests of the lean single-pass scan (authorino_amd/csrc/ajx_lean.h) on its host
build: the byte-class LUT + transpose against plain compares, and the scan + stage B
against the oracle (and its capture rows against the token scanner's) on the workloads'
documents, random documents, mutated bytes and selector sets with indices / duplicates."""
import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O


def _ref_classes(b: bytes):
    out = [0] * 8
    for k, x in enumerate(b):
        cls = [x == 0x22, x == 0x5C, x in (0x7B, 0x5B), x in (0x7D, 0x5D), x == 0x3A, x == 0x2C,
               x in (0x20, 0x21, 0x28, 0x29), x < 0x20]
        for c in range(8):
            if cls[c]:
                out[c] |= 1 << k
    return out


def test_byte_classes_match_plain_compares():
    rng = np.random.default_rng(5)
    alphabet = np.frombuffer(b'"\\{}[]:, !()\x00\x1f\x7fa0zZ\x80\xff', dtype=np.uint8)
    for _ in range(400):
        if rng.random() < 0.5:
            b = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        else:
            b = bytes(rng.choice(alphabet, 32))
        assert H.lean_classes(b) == _ref_classes(b), b
    for v in range(256):  # every byte value in every position
        b = bytes([v]) * 32
        assert H.lean_classes(b) == _ref_classes(b)


def _chain(n):
    nodes = [(0, -1, -1, i) for i in range(n)]
    root = -1
    for i in reversed(range(n)):
        nodes.append((1, i, root, -1))
        root = len(nodes) - 1
    return nodes, root


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5])
def test_lean_fuzz_matches_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    n_lean = 0
    for _ in range(120):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(15):
            d = FU.rand_doc(rng, ws=False) if rng.random() < 0.7 else FU.rand_doc(rng)
            if rng.random() < 0.4:
                d = FU.mutate(rng, d)
            ot = [rs.pattern(p, d) for p in range(len(pats))]
            if O.UNSUPPORTED in ot:
                continue
            t_or, _ = rs.matches(d)
            tl, _, lres, _ = H.eval_lean(hr, d, mis=int(rng.integers(0, 16)))
            if tl >= 0 and 3 not in lres:
                n_lean += 1
                assert lres == ot, (pats, d)
                assert tl == t_or, (pats, d)
    assert n_lean > 300


@pytest.mark.parametrize("workload", ["c1", "c2", "c3", "c5"])
def test_lean_decides_workload_documents(workload):
    """Every synthetic document (compact Go JSON) is proved by the lean scan, with the
    oracle's results and the token scanner's capture rows."""
    from authorino_amd import workloads as W

    w = W.make(workload, n=300, seed=17)
    hr = H.HostRuleset.from_expression(w.expr)
    rs = O.Ruleset.from_expression(w.expr)
    n_sel = len({p.selector for p in w.expr.flatten()[0]})
    for i in range(w.n):
        d = w.doc(i)
        for mis in (0, 7):
            tl, el, lres, lrow = H.eval_lean(hr, d, mis=mis, n_sel=n_sel)
            assert tl >= 0, (i, d)
            tt, et, tres, trow = H.eval_tok(hr, d, mis=mis, n_sel=n_sel)
            assert tt >= 0
            assert lrow == trow, (i, d)
            assert lres == tres and tl == tt and el == et
            t_or, _ = rs.matches(d)
            assert tl == t_or
