"""CPU tests of the row kernel (authorino_amd/csrc/ajx_row.h) on its 64-lane host
emulation (ajx_wave.h), against the oracle: documents it keeps must give the oracle's
results bit for bit (and the token scanner's capture rows), documents it can not prove
must be handed to the exact scan (-1), never guessed."""
import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O


def _rulesets(pats):
    nodes, root = FU.chain(len(pats))
    return O.Ruleset(pats, nodes, root), H.HostRuleset(pats, nodes, root)


def _check(rs, hr, d, mis=0, **kw):
    """(tri from the row kernel or -1/-2, oracle pattern results); asserts parity when kept."""
    n = hr.n
    ot = [rs.pattern(p, d) for p in range(n)]
    t, _, res = H.eval_row(hr, d, mis=mis, **kw)
    if t >= 0 and O.UNSUPPORTED not in ot:
        assert res == ot, (d, res, ot)
        assert t == rs.matches(d)[0], d
    return t, ot


@pytest.mark.parametrize("workload", ["c1", "c2", "c3", "c5"])
def test_row_kernel_workload_documents(workload):
    """Every benchmark document stays on the row path and equals the oracle."""
    from authorino_amd import workloads as W

    w = W.make(workload, n=120, seed=21)
    pats, nodes, root = w.expr.flatten()
    pl = [(p.selector, int(p.operator), p.value) for p in pats]
    rs, hr = O.Ruleset(pl, nodes, root), H.HostRuleset(pl, nodes, root)
    for i in range(w.n):
        d = bytes(w.arena[w.offs[i]:w.offs[i] + w.lens[i]])
        t, _, res = H.eval_row(hr, d, mis=int(w.offs[i]) % 16)
        assert t >= 0, (workload, i)
        assert res == [rs.pattern(p, d) for p in range(len(pl))]
        assert t == rs.matches(d)[0]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_row_kernel_fuzz_matches_oracle(seed):
    """Random selectors (escaped keys, indices, duplicates) over random, long and mutated
    documents at random misalignments: kept documents equal the oracle."""
    rng = np.random.default_rng(700 + seed)
    kept = total = 0
    for _ in range(120):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        rs, hr = _rulesets(pats)
        for _ in range(10):
            k = rng.random()
            d = FU.rand_doc(rng, ws=False) if k < 0.55 else FU.long_doc(rng, pats) if k < 0.85 else FU.rand_doc(rng)
            if rng.random() < 0.25:
                d = FU.mutate(rng, d)
            t, ot = _check(rs, hr, d, mis=int(rng.integers(0, 16)))
            if t == -2:
                continue
            total += 1
            kept += t >= 0
    assert total > 800 and kept > 0.35 * total, (kept, total)


def test_row_capture_rows_equal_token_scanner():
    """The row kernel's capture rows (spans, types, escape flags, found bits) equal the
    token scanner's on documents both keep; four documents per wavefront."""
    from authorino_amd import workloads as W

    rng = np.random.default_rng(5)
    for workload in ["c2", "c3", "c5"]:
        w = W.make(workload, n=40, seed=3)
        pats, nodes, root = w.expr.flatten()
        pl = [(p.selector, int(p.operator), p.value) for p in pats]
        hr = H.HostRuleset(pl, nodes, root)
        ns = len({p.selector for p in pats})
        for i0 in range(0, w.n, 4):
            docs = [bytes(w.arena[w.offs[i]:w.offs[i] + w.lens[i]]) for i in range(i0, min(w.n, i0 + 4))]
            mis = [int(rng.integers(0, 16)) for _ in docs]
            rc, rows = H.scan_rows(hr, docs, mis, ns)
            assert rc == len(docs)
            for d, m, row in zip(docs, mis, rows):
                t = H.eval_tok(hr, d, mis=m, n_sel=ns)
                assert t[0] >= 0
                tok = t[3]
                assert row[0] == tok[0], (workload, d)
                for s in range(ns):  # (records of selectors not found are not defined)
                    if (row[0] >> s) & 1:
                        assert row[1 + s] == tok[1 + s], (workload, d, s)


def test_row_kernel_four_documents_independent():
    """Four documents of different shapes in one wavefront give the same rows as each alone."""
    rng = np.random.default_rng(9)
    for _ in range(40):
        pats = FU.rand_patterns(rng, 5)
        _, hr = _rulesets(pats)
        ns = len({p[0] for p in pats})  # (selectors are deduplicated)
        docs = [FU.long_doc(rng, pats) if rng.random() < 0.5 else FU.rand_doc(rng, ws=False) for _ in range(4)]
        mis = [int(rng.integers(0, 16)) for _ in docs]
        _, rows4 = H.scan_rows(hr, docs, mis, ns)
        for k in range(4):
            _, rows1 = H.scan_rows(hr, [docs[k]], [mis[k]], ns)
            assert rows1[0] == rows4[k]


def _one(sel, op, val):
    return _rulesets([(sel, op, val)])


def test_row_kernel_backslash_runs_across_lanes():
    """Backslash runs of every length ending at every byte of a 16-byte lane and of a
    256-byte step: escapes and string ends carried lane to lane and step to step."""
    rs, hr = _one("k.z", 1, "v")
    for pad in range(0, 40):
        for run in range(1, 6):
            s = "p" * pad + "\\\\" * run + '\\"' + "q"
            d = ('{"a":"%s","k":{"z":"v"}}' % s).encode()
            for mis in (0, 7, 15):
                t, ot = _check(rs, hr, d, mis=mis)
                assert t == 1, (pad, run, mis)
    # across the 256-byte step
    for pad in range(230, 262):
        d = ('{"a":"%s\\\\\\"x","k":{"z":"v"}}' % ("p" * pad)).encode()
        t, _ = _check(rs, hr, d)
        assert t == 1


def test_row_kernel_whole_lane_of_backslashes_goes_exact():
    rs, hr = _one("k", 1, "v")
    d = ('{"a":"%s","k":"v"}' % ("\\\\" * 20)).encode()  # 40 backslashes: whole 16-B lanes
    t, _ = _check(rs, hr, d)
    assert t == -1
    assert rs.matches(d)[0] == 1


def test_row_kernel_duplicate_keys_first_complete_match():
    """gjson descends into every matching key: a.b is found in the second "a"."""
    rs, hr = _one("a.b", 1, "2")
    d = b'{"a":{"x":1},"a":{"b":2},"a":{"b":3}}'
    t, _ = _check(rs, hr, d)
    assert t == 1
    rs, hr = _one("a", 1, "1")
    t, _ = _check(rs, hr, b'{"a":1,"a":2}')
    assert t == 1


def test_row_kernel_hands_over_what_it_can_not_prove():
    cases = [
        ("a", b'{"a": 1}'),                        # whitespace outside strings
        ("a", b'{"a":1,}'),                        # not JSON
        ("a", b' {"a":1}'),                        # the root not at byte 0
        ("a", b'{"a":1'),                          # the root never closes
        ("a", b'{"\\u0061":1}'),                   # an escaped key on a selector path
        ("a.0.b", b'{"a":[{"b":1}]}'),             # a container inside an indexed array
        ("a", b'{"a":tru}'),                       # a scalar that is no JSON value
        ("a", b'{"x":' + b'[' * 40 + b']' * 40 + b',"a":1}'),  # deeper than the level stack
    ]
    for sel, d in cases:
        rs, hr = _one(sel, 1, "1")
        t, _ = _check(rs, hr, d)
        assert t == -1, (sel, d)


def test_row_kernel_keys_sharing_their_tail():
    """Dictionary keys with the same length and last 8 bytes (the probe goes on past a
    prefix mismatch)."""
    pats = [("a-long-key-name.x", 1, "1"), ("b-long-key-name.x", 1, "2"), ("c-long-key-name", 1, "3")]
    rs, hr = _rulesets(pats)
    d = b'{"c-long-key-name":3,"b-long-key-name":{"x":2},"a-long-key-name":{"x":1}}'
    t, _ = _check(rs, hr, d)
    assert t == 1


def test_row_kernel_index_selectors():
    pats = [("g.0", 1, "a"), ("g.2", 1, "c"), ("g.5", 1, ""), ("h.1", 1, "2.5"), ("0", 1, "x")]
    rs, hr = _rulesets(pats)
    for d in [b'{"g":["a","b","c"],"h":[1,2.5]}', b'{"g":[],"h":[1]}', b'{"g":"abc","h":{"1":2.5}}',
              b'{"g":["a",{"x":1},"c"],"h":[1,2.5]}']:
        t, _ = _check(rs, hr, d)
    rs, hr = _one("0", 1, "x")
    t, _ = _check(rs, hr, b'["x",1]')
    assert t == 1


def test_row_kernel_limits():
    rs, hr = _one("a", 1, "1")
    d = b'{' + b','.join(b'"k%d":%d' % (i, i) for i in range(40)) + b',"a":1}'
    assert _check(rs, hr, d)[0] == 1
    assert _check(rs, hr, d, maxe=32)[0] == -1       # more events than the row holds
    assert _check(rs, hr, d, maxb=256)[0] == -1      # longer than the row buffer


@pytest.mark.parametrize("seed", [77, 78])
def test_row_kernel_random_trees_match_oracle(seed):
    """Random And/Or trees over random selectors, documents with whitespace and mutations
    (the GPU suite's test_random_documents_and_selectors, per document): tri-state, error
    pattern and per-pattern results equal the oracle wherever the row kernel decides —
    Null values included (Array() of Null is empty: excl true, incl false)."""
    rng = np.random.default_rng(seed)
    kept = 0
    for _ in range(50):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 10)))
        nodes = [(0, -1, -1, i) for i in range(len(pats))]
        root = -1
        for i in reversed(range(len(pats))):
            nodes.append((2 if rng.random() < 0.3 else 1, i, root, -1))
            root = len(nodes) - 1
        ors, hr = O.Ruleset(pats, nodes, root), H.HostRuleset(pats, nodes, root)
        for _ in range(60):
            d = FU.rand_doc(rng)
            d = FU.mutate(rng, d) if rng.random() < 0.3 else d
            ot = [ors.pattern(p, d) for p in range(len(pats))]
            if O.UNSUPPORTED in ot:
                continue
            t, e, res = H.eval_row(hr, d, mis=int(rng.integers(0, 16)))
            if t < 0:
                continue
            kept += 1
            assert (t, e) == ors.matches(d), (pats, nodes, root, d)
            assert res == ot, (pats, d)
    assert kept > 600


def test_row_kernel_incl_excl_on_null_and_scalars():
    pats = [("n", 3, ""), ("n", 4, ""), ("s", 3, "x"), ("s", 4, "x"), ("o", 3, '{"a":1}'), ("m", 4, "")]
    rs, hr = _rulesets(pats)
    for d in [b'{"n":null,"s":"x","o":{"a":1}}', b'{"n":[null],"s":["y","x"],"o":[{"a":1}]}', b'{"s":1}']:
        _check(rs, hr, d)
