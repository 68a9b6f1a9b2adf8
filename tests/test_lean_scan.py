"""CPU tests of the lean single-pass scan (authorino_amd/csrc/ajx_lean.h) on its host
build: the byte-class LUT + transpose against plain compares, and the scan + stage B
against the oracle (and its capture rows against the token scanner's) on the workloads'
documents, random documents, mutated bytes and selector sets with indices / duplicates."""
import json

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


@pytest.fixture(params=[True, False], ids=["keep_rows", "needed_rows"])
def keep(request):
    """Both capture-row modes of the lean scan: rows a caller reads (the records of its
    selectors, kEagerKeep, as well) and only what stage B needs (values decided in the scan
    leave no record)."""
    H.lean_keep(request.param)
    yield request.param
    H.lean_keep(True)


@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5])
def test_lean_fuzz_matches_oracle(seed, keep):
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
def test_lean_decides_workload_documents(workload, keep):
    """Every synthetic document (compact Go JSON) is proved by the lean scan, with the
    oracle's results and the token scanner's capture rows."""
    from authorino_amd import workloads as W

    w = W.make(workload, n=300, seed=17)
    # kept rows: the forest with a root-less tree of every selector (what a caller of
    # authjx_select_from_eval_device compiles): every record is written
    hr = H.HostRuleset.with_selector_tree(w.expr) if keep else H.HostRuleset.from_expression(w.expr)
    rs = O.Ruleset.from_expression(w.expr)
    np_ = len(w.expr.flatten()[0])
    n_sel = len({p.selector for p in w.expr.flatten()[0]})
    for i in range(w.n):
        d = w.doc(i)
        for mis in (0, 7):
            tl, el, lres, lrow = H.eval_lean(hr, d, mis=mis, n_sel=n_sel)
            assert tl >= 0, (i, d)
            tt, et, tres, trow = H.eval_tok(hr, d, mis=mis, n_sel=n_sel)
            assert tt >= 0
            if keep:
                assert lrow == trow, (i, d)
            assert lres == tres and tl == tt and el == et
            assert lres[:np_] == [rs.pattern(p, d) for p in range(np_)]
            if not keep:
                t_or, _ = rs.matches(d)
                assert tl == t_or


def _tree(rng, depth, keys):
    r = rng.random()
    if depth <= 0 or r < 0.35:
        k = rng.integers(0, 4)
        if k == 0:
            return ("s", "".join(rng.choice(list("abcxyz/\\\"é -"), int(rng.integers(0, 90)))))
        if k == 1:
            return ("n", str(int(rng.integers(-10**9, 10**9))))
        if k == 2:
            return ("l", ["true", "false", "null"][rng.integers(0, 3)])
        return ("s", "v%d" % rng.integers(0, 20))
    n = int(rng.integers(0, 7))
    if r < 0.75:
        return ("o", [(keys[rng.integers(0, len(keys))], _tree(rng, depth - 1, keys)) for _ in range(n)])
    return ("a", [_tree(rng, depth - 1, keys) for _ in range(n)])


def _paths(v, prefix, out):
    t, x = v
    if t == "o":
        for k, c in x:
            p = prefix + [FU.esc_key(k)]
            out.append(p)
            _paths(c, p, out)
    elif t == "a":
        for i, c in enumerate(x):
            p = prefix + [str(i)]
            out.append(p)
            _paths(c, p, out)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_lean_deep_trees_selectors_from_the_document(seed):
    """Compact documents of 1-6 KiB (keys of 1..40 bytes, strings up to 90 bytes, squashed
    containers spanning sub-windows), selectors taken from the document's own paths
    (array indices included), every misalignment: the oracle's results, and the token
    scanner's capture rows."""
    rng = np.random.default_rng(300 + seed)
    keys = ["k", "ab", "x.y", "0", "name", "a-much-longer-key-name", "key-with-sixteen", "nine-byte",
            "a b", "the-key-name-that-goes-past-thirty-bytes", "é", "ab-tail-", "zz-tail-"]
    decided = decided_tok = total = 0
    for _ in range(60):
        v = ("o", [(keys[rng.integers(0, len(keys))], _tree(rng, 5, keys)) for _ in range(int(rng.integers(2, 9)))])
        d = FU.dump(v, rng, False).encode()
        paths = []
        _paths(v, [], paths)
        if not paths:
            continue
        pats = []
        for _ in range(int(rng.integers(1, 9))):
            p = paths[int(rng.integers(0, len(paths)))]
            pats.append((".".join(p), [1, 2, 3, 4][rng.integers(0, 4)], ["v3", "", "true", "x"][rng.integers(0, 4)]))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        ot = [rs.pattern(p, d) for p in range(len(pats))]
        if O.UNSUPPORTED in ot:
            continue
        # (with a root-less tree of every selector: rows a caller reads, every record kept)
        sels = list(dict.fromkeys(p[0] for p in pats))
        hr = H.HostRuleset.forest([(pats, nodes, root), ([(x, 1, "") for x in sels], [], -1)])
        n_sel = len(sels)
        for mis in (0, int(rng.integers(1, 16))):
            total += 1
            tl, _, lres, lrow = H.eval_lean(hr, d, mis=mis, n_sel=n_sel)
            tt, _, tres, trow = H.eval_tok(hr, d, mis=mis, n_sel=n_sel)
            decided_tok += tt >= 0
            if tl >= 0:
                decided += 1
                assert lres[:len(pats)] == ot, (pats, d)
                if tt >= 0:
                    assert lrow == trow, (pats, d, mis)
    # (selectors into containers nested in indexed arrays, deep index chains: the exact
    # scan, by design, for both scanners)
    assert decided >= decided_tok and decided >= 0.1 * total, (decided, decided_tok, total)


@pytest.mark.parametrize("seed", [0, 1])
def test_lean_long_values(seed):
    """Selector values that are long strings / arrays after long padding (they straddle
    sub-windows and 64-byte windows)."""
    rng = np.random.default_rng(400 + seed)
    n = 0
    for _ in range(150):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        d = FU.long_doc(rng, pats)
        ot = [rs.pattern(p, d) for p in range(len(pats))]
        if O.UNSUPPORTED in ot:
            continue
        hr = H.HostRuleset(pats, nodes, root)
        tl, _, lres, _ = H.eval_lean(hr, d, mis=int(rng.integers(0, 16)))
        if tl >= 0 and 3 not in lres:
            n += 1
            assert lres == ot, (pats, d)
    assert n > 80


def test_eager_patterns_decided_in_the_scan(keep):
    """c2's eq / neq patterns with literals of <= 16 bytes are decided while the scan
    captures (EagerSel): strings by their contents, `true` by the literal's String(). Left
    to stage B: the 35-byte iss literal, the incl patterns on arrays (squashed, one pass in
    stage B) and missing keys (Null). Same results, with or without the decided values'
    capture records."""
    from authorino_amd import workloads as W

    w = W.make("c2", n=100, seed=23)
    hr = H.HostRuleset.from_expression(w.expr)
    rs = O.Ruleset.from_expression(w.expr)
    for i in range(w.n):
        d = w.doc(i)
        t, _, res, _ = H.eval_lean(hr, d, mis=i % 16)
        assert t >= 0 and res == [rs.pattern(p, d) for p in range(16)]
        dm, tm = H.lean_last_dec()
        assert bin(dm).count("1") >= 10, hex(dm)  # (x-blocked: mostly missing)
        assert not (dm >> 4) & 1  # the iss pattern
        assert not (dm >> 12) & 0xF  # the incl patterns on the groups / roles arrays
        assert (dm >> 6) & 1  # email_verified (a literal)
        for p in range(16):
            if (dm >> p) & 1:
                assert ((tm >> p) & 1) == (res[p] == 1)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_eager_arrays_and_strings(seed, keep):
    """incl / excl over arrays of strings (escaped elements, numbers, nested containers,
    empty arrays, more than two patterns per selector), eq / neq on strings of 0..20 bytes."""
    rng = np.random.default_rng(500 + seed)
    words = ["", "a", "users", "reader", "admins", "x" * 16, "y" * 17, "é", "a\"b", "v3"]
    for _ in range(200):
        def elem():
            r = rng.random()
            if r < 0.7:
                return json.dumps(words[rng.integers(0, len(words))])
            if r < 0.8:
                return "12"
            if r < 0.9:
                return "[\"users\"]"
            return "true"
        arrs = {k: "[" + ",".join(elem() for _ in range(int(rng.integers(0, 5)))) + "]" for k in ("g", "r")}
        strs = {k: json.dumps(words[rng.integers(0, len(words))]) for k in ("s", "t")}
        vals = {**arrs, **strs}
        d = ("{" + ",".join('"%s":%s' % (k, v) for k, v in vals.items()) + "}").encode()
        pats = []
        for _ in range(int(rng.integers(1, 7))):
            sel = ["g", "r", "s", "t"][rng.integers(0, 4)]
            op = [1, 2, 3, 4][rng.integers(0, 4)]
            pats.append((sel, op, words[rng.integers(0, len(words))]))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        ot = [rs.pattern(p, d) for p in range(len(pats))]
        t, _, res, _ = H.eval_lean(hr, d, mis=int(rng.integers(0, 16)))
        if t >= 0 and 3 not in res:
            assert res == ot, (pats, d)


@pytest.mark.parametrize("klen", [17, 24, 31, 40])
def test_lean_colliding_long_keys(klen):
    """keys of 17..40 bytes that share their length, parent and last 8 bytes (one
    key-table signature, so the head decides), padded so that each key straddles sub-window
    and 64-byte window boundaries, at every misalignment; heads past the ring's 32 bytes
    before the sub-window are read from the document. The oracle's results."""
    tail = "tail-key"
    heads = ["a" * (klen - 8), "b" * (klen - 8), "a" * (klen - 9) + "b", "b" + "a" * (klen - 9)]
    keys = [h + tail for h in heads]
    pats = [(keys[0], 1, "v0"), (keys[3], 2, "v3"), ("o." + keys[2], 1, "v2")]
    nodes, root = _chain(len(pats))
    rs = O.Ruleset(pats, nodes, root)
    hr = H.HostRuleset(pats, nodes, root)
    n = 0
    for pad in range(0, 70):
        order = [1, 2, 0, 3] if pad % 2 else [3, 0, 2, 1]
        members = ['"p":"%s"' % ("x" * pad)]
        members += ['"%s":"v%d"' % (keys[j], j) for j in order]
        members.append('"o":{%s}' % ",".join('"%s":"v%d"' % (keys[j], j) for j in (1, 2, 3)))
        d = ("{" + ",".join(members) + "}").encode()
        ot = [rs.pattern(p, d) for p in range(len(pats))]
        t_or, _ = rs.matches(d)
        for mis in range(16):
            tl, _, lres, _ = H.eval_lean(hr, d, mis=mis)
            assert tl >= 0, (pad, mis)
            n += 1
            assert lres == ot and tl == t_or, (klen, pad, mis, d)
    assert n == 70 * 16


@pytest.mark.parametrize("seed", [0, 1])
def test_stage_b_arrays_from_the_ring(seed):
    """Stage B's incl / excl walk of an array copied into the lane's ring (incl_hits_ring):
    arrays of unescaped strings of 0..17 bytes whose aligned blocks number 7..9 around the
    ring's eight (every misalignment), with an escaped, numeric, nested or trailing-comma
    element now and then (the memory walk decides those); the oracle's results."""
    rng = np.random.default_rng(900 + seed)
    words = ["", "a", "users", "reader", "x" * 8, "y" * 9, "z" * 15, "w" * 16, "v" * 17]
    n = 0
    for _ in range(60):
        elems = []
        target = int(rng.integers(90, 135))
        while len("[" + ",".join(elems) + "]") < target:
            elems.append(json.dumps(words[rng.integers(0, len(words))]))
        r = rng.random()
        if r < 0.1:
            elems.insert(int(rng.integers(0, len(elems) + 1)), '"a\\"b"')
        elif r < 0.2:
            elems.insert(int(rng.integers(0, len(elems) + 1)), "12")
        elif r < 0.25:
            elems.insert(int(rng.integers(0, len(elems) + 1)), '["users"]')
        arr = "[" + ",".join(elems) + "]"
        d = ('{"s":"%s","g":%s,"t":"x"}' % ("p" * int(rng.integers(0, 40)), arr)).encode()
        pats = [("g", int(rng.integers(3, 5)), words[rng.integers(0, len(words))]) for _ in range(3)]
        pats.append(("g", 3, json.loads(elems[-1]) if elems[-1].startswith('"') else "12"))
        nodes, root = _chain(len(pats))
        rs = O.Ruleset(pats, nodes, root)
        hr = H.HostRuleset(pats, nodes, root)
        ot = [rs.pattern(p, d) for p in range(len(pats))]
        t_or, _ = rs.matches(d)
        for mis in range(16):
            t, _, res, _ = H.eval_lean(hr, d, mis=mis)
            if t >= 0 and 3 not in res:
                n += 1
                assert res == ot and t == t_or, (pats, d, mis)
    assert n >= 60 * 16 * 0.8


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_flat_fold_agrees_with_the_code_interpreter(seed):
    """Rulesets of one flat All / Any over patterns 0..n-1 (kFlagFlatFold: the kernels read
    the fold off the bitmaps) on random documents: the host harness computes both folds and
    returns no tri-state when they differ; the oracle's results. c2's ruleset is one."""
    import ctypes as C

    from authorino_amd import jsonexp as J
    from authorino_amd import workloads as W

    L = H.lib()
    L.ht_flat_folds.restype = C.c_uint64
    before = L.ht_flat_folds()
    rng = np.random.default_rng(700 + seed)
    n = 0
    for _ in range(60):
        pats = FU.rand_patterns(rng, int(rng.integers(1, 12)))
        expr = (J.All if rng.random() < 0.5 else J.Any)(*[J.Pattern(s, J.Operator(op), v) for s, op, v in pats])
        hr = H.HostRuleset.from_expression(expr)
        rs = O.Ruleset.from_expression(expr)
        for _ in range(10):
            d = FU.rand_doc(rng, ws=False)
            t_or, _ = rs.matches(d)
            tl, _, _, _ = H.eval_lean(hr, d, mis=int(rng.integers(0, 16)))
            if tl >= 0:
                n += 1
                assert tl == t_or, (pats, d)
    w = W.make("c2", n=50, seed=3)
    hr = H.HostRuleset.from_expression(w.expr)
    rs = O.Ruleset.from_expression(w.expr)
    for i in range(w.n):
        tl, _, _, _ = H.eval_lean(hr, w.doc(i), mis=i & 15)
        assert tl == rs.matches(w.doc(i))[0]
    assert L.ht_flat_folds() - before >= w.n + n // 2  # (one-pattern trees compile without a group)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_group_fold_agrees_with_the_code_interpreter(seed):
    """Rulesets of one All / Any over lone patterns and groups of the other kind
    (kFlagGroupFold: the kernels read the fold off the bitmaps, one step per group): the
    harness's group_fold against the code interpreter on random T / U / static-E bitmaps
    (E and U at every position, groups first, last, adjacent, of one to eight patterns), and
    on random documents against the oracle. c3's ruleset is one."""
    import ctypes as C

    from authorino_amd import jsonexp as J
    from authorino_amd import workloads as W

    L = H.lib()
    L.ht_group_folds.restype = C.c_uint64
    L.ht_group_fold_check.restype = C.c_int64
    L.ht_group_fold_check.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
    before = L.ht_group_folds()
    rng = np.random.default_rng(800 + seed)
    n = n_group = 0
    for it in range(60):
        outer = J.All if rng.random() < 0.5 else J.Any
        inner = J.Any if outer is J.All else J.All
        kids = []
        for _ in range(int(rng.integers(1, 7))):
            if rng.random() < 0.5:
                kids.append(None)
            else:
                kids.append(int(rng.integers(2, 9)))
        if all(k is None for k in kids):
            kids[int(rng.integers(0, len(kids)))] = int(rng.integers(2, 9))
        npat = sum(1 if k is None else k for k in kids)
        pats = FU.rand_patterns(rng, npat)
        ps = [J.Pattern(s, J.Operator(op), v) for s, op, v in pats]
        args, i = [], 0
        for k in kids:
            if k is None:
                args.append(ps[i])
                i += 1
            else:
                args.append(inner(*ps[i:i + k]))
                i += k
        expr = outer(*args)
        hr = H.HostRuleset.from_expression(expr)
        bad = L.ht_group_fold_check(hr._h, it + 1000 * seed, 4000)
        if bad < 0:
            continue  # (the compiler merged or reordered it: not a group fold)
        n_group += 1
        assert bad == 0, (kids, pats)
        rs = O.Ruleset.from_expression(expr)
        for _ in range(6):
            d = FU.rand_doc(rng, ws=False)
            t_or, _ = rs.matches(d)
            tl, _, _, _ = H.eval_lean(hr, d, mis=int(rng.integers(0, 16)))
            if tl >= 0:
                n += 1
                assert tl == t_or, (kids, pats, d)
    assert n_group >= 40
    w = W.make("c3", n=50, seed=3)
    hr = H.HostRuleset.from_expression(w.expr)
    assert L.ht_group_fold_check(hr._h, 7 + seed, 20000) == 0
    rs = O.Ruleset.from_expression(w.expr)
    for i in range(w.n):
        tl, _, _, _ = H.eval_lean(hr, w.doc(i), mis=i & 15)
        assert tl == rs.matches(w.doc(i))[0]
    assert L.ht_group_folds() - before >= w.n + n // 2


@pytest.mark.parametrize("seed", [0, 1])
def test_forest_tree_folds_agree_with_the_code_interpreter(seed):
    """Forest rulesets (one fold program per tree, patterns concatenated by tree): trees of
    one flat or two-level All / Any carry a TreeFold and fold off their own bits of the
    128-bit bitmaps (bases across the 64-bit word boundary); tree_fold against the code
    interpreter on random T / U / static-E bitmaps. c5's forest is one."""
    import ctypes as C

    from authorino_amd import jsonexp as J
    from authorino_amd import workloads as W

    L = H.lib()
    L.ht_tree_fold_check.restype = C.c_int64
    L.ht_tree_fold_check.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32]
    rng = np.random.default_rng(950 + seed)
    checked = 0
    for it in range(25):
        trees, total = [], 0
        while total < 110:
            outer = J.All if rng.random() < 0.5 else J.Any
            inner = J.Any if outer is J.All else J.All
            kids = [None if rng.random() < 0.5 else int(rng.integers(2, 6)) for _ in range(int(rng.integers(1, 6)))]
            npat = sum(1 if k is None else k for k in kids)
            ps = [J.Pattern(s, J.Operator(op), v) for s, op, v in FU.rand_patterns(rng, npat)]
            args, i = [], 0
            for k in kids:
                if k is None:
                    args.append(ps[i])
                    i += 1
                else:
                    args.append(inner(*ps[i:i + k]))
                    i += k
            e = outer(*args) if len(args) > 1 or rng.random() < 0.5 else args[0]
            if rng.random() < 0.15:  # a third level: interpreted
                e = inner(e, outer(*ps[:2])) if npat >= 2 else e
            trees.append(e.flatten())
            total += npat
        if sum(len(p) for p, _, _ in trees) > 128:
            trees = trees[:-1]
        hr = H.HostRuleset.forest([([(p.selector, int(p.operator), p.value) for p in pats], nodes, root)
                                   for pats, nodes, root in trees])
        bad = L.ht_tree_fold_check(hr._h, it + 100 * seed, 3000)
        if bad >= 0:
            checked += 1
            assert bad == 0, it
    assert checked >= 20
    w = W.make("c5", n=16)
    ac = w.auth_config
    ex = [ac.conditions] + [e for c in ac.authorization for e in (c.conditions, c.rules)]
    hr = H.HostRuleset.forest([([(p.selector, int(p.operator), p.value) for p in pats], nodes, root)
                               for pats, nodes, root in (e.flatten() for e in ex)])
    assert L.ht_tree_fold_check(hr._h, 5 + seed, 20000) == 0
