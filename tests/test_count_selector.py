"""gjson `#` (array element count) selectors: `groups.#`, `a.0.#`, `#` on a root array —
gjson v1.14.0 parseArray answers Number(element count) at the array's ']' (Raw =
strconv.Itoa); on an object the part is the key "#". `#.key` lists and `#(...)` queries
stay AUTHJX_PAT_UNSUPPORTED. No reference test covers `#` (parity unpinned: the cases
below follow gjson's documented semantics, e.g. its README's `friends.#` -> 3); the
device exact scan (host build, tests/native) is checked against the oracle
restatement (oracle/gjson_ref.c), and tests/test_gpu_parity.py checks the GPU."""
import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O

KATS = [  # (document, path, Result.String(), found)
    ('{"friends":[{"first":"Dale"},{"first":"Roger"},{"first":"Jane"}]}', "friends.#", b"3", True),
    ('{"a":[]}', "a.#", b"0", True),
    ('{"a":[1,[2,3],{"x":4},"s",null]}', "a.#", b"5", True),
    ('{"a":[[1],[1,2]]}', "a.1.#", b"2", True),
    ('[1,2,3,4]', "#", b"4", True),
    ('{"a":{"#":"key"}}', "a.#", b"key", True),  # object context: the key "#"
    ('{"a":"x"}', "a.#", b"", False),
    ('{"a":[1,2]}', "b.#", b"", False),
    ('{"a" : [ 1 , 2 ] }', "a.#", b"2", True),
]


@pytest.mark.parametrize("doc,path,want,found", KATS)
def test_count_kats_oracle_and_exact_scan(doc, path, want, found):
    t, _, s = O.gjson_get(doc.encode(), path.encode())
    assert (t != O.T_NULL) == found and s == want
    assert H.string(doc, path) == want


def test_count_queries_and_lists_unsupported():
    for path in ["a.#.b", "a.#(b==1)", "a.#[b==1]", "#.x"]:
        with pytest.raises(ValueError):
            O.gjson_get(b'{"a":[]}', path.encode())
        hr = H.HostRuleset([(path, 1, "1")], [(0, -1, -1, 0)], 0)
        assert hr.status[0] != 0  # AUTHJX_PAT_UNSUPPORTED


def rand_count_patterns(rng, k):
    pats = []
    for _ in range(k):
        sel = FU.rand_selector(rng)
        if rng.random() < 0.6:
            sel = "#" if rng.random() < 0.1 else sel + ".#"
        op = int(rng.choice([1, 2, 3, 4, 5]))
        val = str(int(rng.integers(0, 6))) if op != 5 else ["^[0-9]$", "^0$", "[2-4]"][int(rng.integers(0, 3))]
        pats.append((sel, op, val))
    return pats


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_count_patterns_exact_scan_vs_oracle(seed):
    rng = np.random.default_rng(1200 + seed)
    n = 0
    for _ in range(60):
        pats = rand_count_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        for _ in range(20):
            d = FU.rand_doc(rng)
            ot = [rs.pattern(p, d) for p in range(len(pats))]
            if O.UNSUPPORTED in ot:
                continue
            t, _, res = hr.eval(d)
            assert res == ot, (pats, d)
            assert t == rs.matches(d)[0]
            n += 1
    assert n > 1000
