"""CPU differential fuzz of the line engine (authorino_amd/csrc/ajx_lines.h, host build)
against the oracle: per-pattern tri-states and the fold, on random compact documents,
mutated (malformed) documents, long values that straddle the two-line ring, every
in-line offset of the document start, and the BASELINE workload documents."""
import json

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


def _check(rs, hr, pats, d, mis, fill=0x41):
    ot = [rs.pattern(p, d) for p in range(len(pats))]
    if O.UNSUPPORTED in ot:
        return None
    t_or, _ = rs.matches(d)
    tl, _, lres = H.eval_lines(hr, d, mis=mis, fill=fill)
    if tl == -2:
        return None
    if tl >= 0 and 3 not in lres:
        assert lres == ot, (pats, d, mis)
        assert tl == t_or, (pats, d, mis)
        return True
    return False


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5])
def test_lines_random_compact_documents(seed):
    rng = np.random.default_rng(100 + seed)
    n_fast = n_all = 0
    for _ in range(120):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 8)))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(12):
            d = FU.rand_doc(rng, ws=False)
            if rng.random() < 0.3:
                d = FU.mutate(rng, d)
            r = _check(rs, hr, pats, d, int(rng.integers(0, 128)), int(rng.choice([0x41, 0x22, 0x5C, 0x20, 0x7B])))
            if r is not None:
                n_all += 1
                n_fast += int(r)
    assert n_all > 500
    assert n_fast > 0.35 * n_all, (n_fast, n_all)  # escaped keys on selector paths go exact


def _long_doc(rng, pats):
    """A compact document whose selector values are long strings / arrays, placed after
    padding so that they straddle line boundaries."""
    parts = []
    for k in range(int(rng.integers(1, 6))):
        parts.append('"pad%d":"%s"' % (k, "p" * int(rng.integers(0, 300))))
    for sel, op, val in pats:
        keys = sel.split(".")
        if any(not k or "\\" in k or '"' in k for k in keys):
            continue
        v = rng.random()
        if v < 0.3:
            inner = json.dumps(val) if rng.random() < 0.5 else '"%s"' % ("L" * int(rng.integers(100, 300)))
        elif v < 0.6:
            inner = "[" + ",".join('"%s"' % ("e" * int(rng.integers(0, 150))) for _ in range(int(rng.integers(0, 6)))) + "]"
        elif v < 0.8:
            inner = "[" + ",".join(['{"k":"%s"}' % ("o" * int(rng.integers(0, 90))), "12", "true", "null", json.dumps(val)]) + "]"
        else:
            inner = str(int(rng.integers(-10**12, 10**12)))
        for k in reversed(keys):
            inner = "{%s:%s}" % (json.dumps(k, ensure_ascii=False), inner)
        parts.append(inner[1:-1])
    rng.shuffle(parts)
    return ("{" + ",".join(parts) + "}").encode()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lines_long_values_and_ring(seed):
    rng = np.random.default_rng(200 + seed)
    n_fast = n_all = 0
    for _ in range(60):
        pats = [(s, op, v) for s, op, v in FU.rand_patterns(rng, int(rng.integers(1, 6)))]
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(10):
            d = _long_doc(rng, pats)
            r = _check(rs, hr, pats, d, int(rng.integers(0, 128)))
            if r is not None:
                n_all += 1
                n_fast += int(r)
    assert n_all > 200
    assert n_fast > 0.4 * n_all, (n_fast, n_all)  # values longer than the ring go exact


@pytest.mark.parametrize("workload", ["c1", "c2", "c3"])
def test_lines_workload_documents(workload):
    from authorino_amd import workloads as W

    w = W.make(workload, n=300, seed=11)
    pats, nodes, root = w.expr.flatten()
    pl = [(p.selector, int(p.operator), p.value) for p in pats]
    rs = O.Ruleset(pl, nodes, root)
    hr = H.HostRuleset(pl, nodes, root)
    rng = np.random.default_rng(5)
    for i in range(w.n):
        d = bytes(w.arena[w.offs[i]:w.offs[i] + w.lens[i]])
        r = _check(rs, hr, pl, d, int(rng.integers(0, 128)))
        assert r is True, (workload, i)


def test_lines_number_and_escape_values():
    """Numbers whose String() the line engine takes from the raw text (integers and
    canonical fixed-notation floats) and escaped strings it unescapes, against the
    oracle's strconv / unescape restatement; every other form goes to the exact scan."""
    rng = np.random.default_rng(77)
    nums = []
    for _ in range(400):
        k = rng.integers(0, 6)
        if k == 0:
            nums.append(str(int(rng.integers(-10**6, 10**6))))
        elif k == 1:
            nums.append("%.*f" % (int(rng.integers(0, 8)), rng.normal() * 10 ** int(rng.integers(-6, 10))))
        elif k == 2:
            nums.append(repr(float(rng.normal())))
        elif k == 3:
            nums.append("0." + "0" * int(rng.integers(0, 20)) + str(int(rng.integers(1, 10**int(rng.integers(1, 17))))))
        elif k == 4:
            nums.append(str(rng.choice(["0.5", "-0.5", "10.25", "0.0", "1.0", "007.5", "1e5", "1.5e-3", "-", "-0",
                                        "123456789012345.5", "12345678901234.5", "0.1000", "9007199254740993.0"])))
        else:
            nums.append("%d.%d" % (rng.integers(0, 1000), rng.integers(0, 1000)))
    strs = ["a\\u003cb\\u003e", "x\\\\y", "q\\\"t", "tab\\tx", "\\u00e9", "\\u2028", "\\ud83d\\ude00", "p\\/q",
            "\\u0026amp", "bad\\x", "\\u00zz"]
    n_fast = 0
    for i in range(len(nums)):
        num = nums[i]
        st = strs[i % len(strs)]
        lit_num = num if rng.random() < 0.5 else num.rstrip("0")
        lit_str = json_unescape_guess(st)
        pats = [("n", 1, lit_num), ("n", 2, "0.5"), ("s", 1, lit_str), ("s", 5, "^a<b>$|é|\\\\y|/q"),
                ("arr", 3, lit_str), ("arr", 4, lit_num)]
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        d = ('{"n":%s,"s":"%s","arr":[%s,"%s",1]}' % (num, st, num, st)).encode()
        r = _check(rs, hr, pats, d, int(rng.integers(0, 128)))
        n_fast += int(bool(r))
    assert n_fast > 100, n_fast


def json_unescape_guess(s):
    try:
        return json.loads('"' + s + '"')
    except ValueError:
        return s
