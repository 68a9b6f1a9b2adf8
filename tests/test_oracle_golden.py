"""CPU tests: the oracle against the reference's own known-answer vectors, and the
kernels' per-document logic (host build, tests/native) against the oracle."""
import numpy as np
import pytest

import _hosttest as H
import pyoracle as O
from kat_util import build, flat, load_kats

KATS = load_kats()
EXPECT = {"F": O.F, "T": O.T, "E": O.E}


@pytest.mark.parametrize("case", KATS, ids=[c["source"] for c in KATS])
def test_oracle_reference_kats(case):
    expr = build(case["tree"])
    if expr is None:
        pytest.skip("nil expression")
    pats, nodes, root = flat(expr)
    rs = O.Ruleset(pats, nodes, root)
    t, ep = rs.matches(case["doc"])
    assert t == EXPECT[case["expect"]], case
    if case["expect"] == "E":
        assert case["error_contains"] in rs.error(ep)


@pytest.mark.parametrize("case", KATS, ids=[c["source"] for c in KATS])
def test_device_logic_reference_kats(case):
    expr = build(case["tree"])
    pats, nodes, root = flat(expr)
    hr = H.HostRuleset(pats, nodes, root)
    t, ep, _ = hr.eval(case["doc"])
    assert t == EXPECT[case["expect"]], case
    if case["expect"] == "E":
        assert ep >= 0


def test_gjson_string_cases():
    doc = ('{"a":{"b\\\\.c":1,"x.y":"esc\\u00e9\\ud83d\\ude00","q":"a\\"b"},'
           '"n":[1.50,1e3,-0.0,1e400,0.1,-12,007,12345678901234567890],"t":true,"f":false,"z":null,'
           '"o":{"k":[1, {"z":2}]}}')
    expect = {
        "a.x\\.y": "escé\U0001F600".encode(), "a.q": b'a"b', "n.0": b"1.5", "n.1": b"1000", "n.2": b"-0",
        "n.3": b"+Inf", "n.4": b"0.1", "n.5": b"-12", "n.6": b"007", "n.7": b"12345678901234567890",
        "t": b"true", "f": b"false", "z": b"", "missing": b"", "o.k": b'[1, {"z":2}]', "o.k.1.z": b"2",
        "o.k.1": b'{"z":2}',
    }
    for path, want in expect.items():
        assert O.gjson_get(doc, path)[2] == want, path
        assert H.string(doc, path) == want, path


def test_go_float_formatting():
    cases = {"1.50": "1.5", "1e3": "1000", "-0.0": "-0", "1e400": "+Inf", "-1e400": "-Inf", "0.1": "0.1",
             "1e-7": "0.0000001", "123.456e2": "12345.6", "NaN": "NaN", "inf": "+Inf", "-Infinity": "-Inf",
             "1.2.3": "0", "-": "0", "+5": "5", ".5": "0.5", "5.": "5", "1e": "0", "0x1p3": "8",
             "1_000.5": "1000.5", "1__0": "0", "100000000000000000000000": "100000000000000000000000",
             "1e23": "100000000000000000000000", "9007199254740993": "9007199254740992",
             "0.30000000000000004": "0.30000000000000004", "1.7976931348623157e308": None}
    for raw, want in cases.items():
        rc, v = O.parse_float(raw)
        got = O.format_float(v).decode()
        if want is not None:
            assert got == want, (raw, got)


def _corpus_eval(workload, n):
    from authorino_amd import workloads as W
    w = W.make(workload, n=n)
    pats, nodes, root = flat(w.expr)
    rs = O.Ruleset(pats, nodes, root)
    tri, err, bm = O.eval_batch([rs], w.arena, w.offs, w.lens, nthreads=4)
    hr = H.HostRuleset(pats, nodes, root)
    for i in range(w.n):
        t, e, res = hr.eval(w.doc(i))
        assert t == tri[i], i
        bits = sum(1 << p for p, v in enumerate(res) if v == 1)
        assert bits == sum(int(bm[i][k]) << (64 * k) for k in range(bm.shape[1])), i
    return tri


@pytest.mark.parametrize("workload", ["c2", "c3"])
def test_device_logic_matches_oracle_on_workloads(workload):
    tri = _corpus_eval(workload, 1500)
    assert 0.05 < (tri == O.T).mean() < 0.95  # the workload exercises both decisions
