"""gjson `#` selectors: `groups.#` / `a.0.#` / `#` (array element count — gjson v1.14.0
parseArray answers Number(count) at the array's ']', Raw = strconv.Itoa) and `friends.#.first`
lists (parseArray's alog: the JSON array of Get(element, "first").Raw over the elements
where it exists); on an object the part is the key "#". `#(...)` / `#[...]` queries and
a '#' form inside a list's key path stay AUTHJX_PAT_UNSUPPORTED. No reference test covers `#` (parity unpinned: the cases
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
    ('{"friends":[{"first":"Dale"},{"first":"Roger"},{"last":"x"},3,"s",{"first":{"a":1}}]}', "friends.#.first",
     b'["Dale","Roger",{"a":1}]', True),
    ('{"a":[]}', "a.#.b", b"[]", True),
    ('{"a":{"#":{"b":7}}}', "a.#.b", b"7", True),  # object context: key "#", then b
    ('{"a":[{"b":{"c":1}},{"b":{"c":2}}]}', "a.#.b.c", b"[1,2]", True),
    ('{"a":[ {"b":"x\\"y"} , {"b":null} ]}', "a.#.b", b'["x\\"y",null]', True),
    ('[{"x":1},{"x":2}]', "#.x", b"[1,2]", True),
    ('{"a":"s"}', "a.#.b", b"", False),
]


@pytest.mark.parametrize("doc,path,want,found", KATS)
def test_count_kats_oracle_and_exact_scan(doc, path, want, found):
    t, _, s = O.gjson_get(doc.encode(), path.encode())
    assert (t != O.T_NULL) == found and s == want
    assert H.string(doc, path) == want


def test_count_queries_and_nested_lists_unsupported():
    for path in ["a.#(b==1)", "a.#[b==1]", "a.#.b.#", "a.#.#.c"]:
        with pytest.raises(ValueError):
            O.gjson_get(b'{"a":[]}', path.encode())
        hr = H.HostRuleset([(path, 1, "1")], [(0, -1, -1, 0)], 0)
        assert hr.status[0] != 0  # AUTHJX_PAT_UNSUPPORTED


def rand_count_patterns(rng, k):
    pats = []
    for _ in range(k):
        sel = FU.rand_selector(rng)
        r = rng.random()
        if r < 0.4:
            sel = "#" if rng.random() < 0.1 else sel + ".#"
        elif r < 0.7:  # a list: the key path after it from the random keys
            sel = sel + ".#." + FU.rand_selector(rng)
        op = int(rng.choice([1, 2, 3, 4, 5]))
        val = (str(int(rng.integers(0, 6))) if rng.random() < 0.6 else
               ["[]", '["x"]', "v3", "[1]", "true", '["hello"]'][int(rng.integers(0, 6))])
        if op == 5:
            val = ["^[0-9]$", "^0$", "[2-4]", "^\\[\\]$", "v"][int(rng.integers(0, 5))]
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
