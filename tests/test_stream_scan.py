"""CPU tests of the streaming kernel's code (authorino_amd/csrc/ajx_stream.h) on its host
build: every wave is run on 64 host threads (ajx_wave.h's emulation of ballots, lane
shifts and scans), and its decisions are compared bit for bit with the oracle (tri-state,
error index, pattern bitmap) wherever it does not hand a request to the exact scan.

Inputs: the bench workloads' documents (all proved, none handed over), random compact
documents with random selectors, mutated documents (soundness: a document the stream
proves must give the oracle's answer), documents at every byte alignment and across step
boundaries, and hand-written invalid documents the stream must not prove."""
import json

import numpy as np
import pytest

import _hosttest as H
import fuzz_util as FU
import pyoracle as O


def _pack(docs):
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    if len(docs):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(docs), dtype=np.uint8).copy() if docs else np.zeros(0, np.uint8)
    return arena, offs, lens


def _check(pats, nodes, root, arena, offs, lens, allow_slow=True, mode=0, stage_b=None, per=0):
    """The stream's answers (in-stream fold or stage B) equal the oracle's wherever the
    exact scan is not needed; returns the mask of requests handed to the exact scan (None:
    the ruleset has no stream tables). stage_b: None any, False none may need stage B."""
    hr = H.HostRuleset(pats, nodes, root)
    assert hr.rc == 0, hr.error
    res = H.eval_stream(hr, arena, offs, lens, mode=mode, per=per)
    if res is None:
        return None
    tri, err, bm, slow = res
    if stage_b is False:
        assert not (slow == 2).any(), np.nonzero(slow == 2)[0]
    slow = (slow == 1).astype(np.uint8)
    rs = O.Ruleset(pats, nodes, root)
    otri, oerr, obm = O.eval_batch([rs], arena, offs, lens)
    ok = slow == 0
    np.testing.assert_array_equal(tri[ok], otri[ok])
    np.testing.assert_array_equal(err[ok], oerr[ok])
    np.testing.assert_array_equal(bm[ok, :obm.shape[1]], obm[ok])
    if not allow_slow:
        assert not slow.any(), np.nonzero(slow)[0]
    return slow.astype(bool)


def _flat(expr):
    pats, nodes, root = expr.flatten()
    return [(p.selector, int(p.operator), p.value) for p in pats], nodes, root


@pytest.mark.parametrize("wl,n", [("c2", 256), ("c5", 96), ("c4", 200)])
def test_stream_workloads_match_oracle(wl, n):
    """The bench documents: every one proved (no exact-scan hand-over), bit-exact; c4's
    rulesets include array-index selectors (`groups.0`: stage B's exact Get)."""
    from authorino_amd import workloads

    w = workloads.make(wl, n=n, unique=n)
    exprs = ([w.expr] if wl == "c2" else w.exprs[:40] if wl == "c4" else [w.auth_config.conditions] + [
        e for c in w.auth_config.authorization for e in (c.conditions, c.rules)])
    for e in exprs:
        slow = _check(*_flat(e), w.arena, w.offs, w.lens, allow_slow=False)
        assert slow is not None


@pytest.mark.parametrize("per", [1, 3, 17])
def test_stream_fewer_requests_per_wave(per):
    """The latency configuration: 1..31 requests per wave (small batches spread over more
    waves) gives the same answers."""
    from authorino_amd import workloads

    w = workloads.make("c2", n=40, unique=40)
    assert _check(*_flat(w.expr), w.arena, w.offs, w.lens, allow_slow=False, per=per) is not None


def test_stream_every_alignment_and_step_boundary():
    """The same documents at all 32 byte alignments of the arena and with long fillers
    that put keys, values and containers across lane and step boundaries."""
    from authorino_amd import workloads

    w = workloads.make("c2", n=48, unique=48)
    rng = np.random.default_rng(7)
    docs = []
    for i in range(w.n):
        d = w.doc(i)
        if i % 3 == 0:  # a filler key of 1..2100 bytes in front: everything after it shifts
            pad = '"zz%d":"%s",' % (i, "q" * int(rng.integers(1, 2100)))
            d = d[:1] + pad.encode() + d[1:]
        docs.append(d)
    for shift in range(0, 32, 3):
        a, o, ln = _pack([b"x" * shift] + docs)
        slow = _check(*_flat(w.expr), a, o[1:], ln[1:], allow_slow=False)
        assert slow is not None


def _stream_patterns(rng, k):
    return FU.rand_patterns(rng, k)  # (array indices: stage B's exact Get)


@pytest.mark.parametrize("per", [1, 4])
def test_stream_small_batch_stage_b_in_lds(per):
    """Small batches: spans that fit one step run stage B on the ring's copy of each document
    (the kernel's LAT instance), array-index selectors included (exact Get on the copy)."""
    rng = np.random.default_rng(600 + per)
    for _ in range(4):
        pats = _stream_patterns(rng, int(rng.integers(1, 7)))
        nodes, root = FU.chain(len(pats))
        docs = [FU.rand_doc(rng, ws=False) for _ in range(48)]
        _check(pats, nodes, root, *_pack(docs), per=per)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_stream_random_documents(seed):
    """Random compact documents and selectors: bit-exact where decided (light and full
    stage B), and with the full stage B compact valid documents are mostly decided."""
    rng = np.random.default_rng(400 + seed)
    decided = total = 0
    for _ in range(6):
        pats = _stream_patterns(rng, int(rng.integers(1, 7)))
        nodes, root = FU.chain(len(pats))
        docs = [FU.rand_doc(rng, ws=False) for _ in range(64)]
        a, o, ln = _pack(docs)
        if _check(pats, nodes, root, a, o, ln) is None:
            continue
        slow = _check(pats, nodes, root, a, o, ln, mode=0)
        decided += int((~slow).sum())
        total += len(docs)
    assert total == 0 or decided >= total // 2


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_stream_mutated_documents_are_sound(seed):
    """Truncated, byte-flipped, whitespace-padded documents: whatever the stream decides
    equals the oracle (which restates gjson on any input)."""
    rng = np.random.default_rng(500 + seed)
    for _ in range(6):
        pats = _stream_patterns(rng, int(rng.integers(1, 6)))
        nodes, root = FU.chain(len(pats))
        docs = [FU.mutate(rng, FU.rand_doc(rng, ws=False)) for _ in range(64)]
        _check(pats, nodes, root, *_pack(docs))


INVALID = [
    b'{"a","b":"v"}', b'{"a":1,"b"}', b'{"a":1,2}', b'["a":1]', b'{"a"}', b'{{}}', b'{"a":{},{}}',
    b'{"a":"b":"v"}', b'{"a":[1}', b'{"a":[1]]}', b'{"b":{"a":1]}', b'{"a":1}}', b'{"a":1', b'{"a" :1}',
    b' {"a":1}', b'{"a":tru}', b'{"a":1,}', b'{,"a":1}', b'{"a":(1)}', b'{"a":[1,{"b":2]]}', b'{"a\\u0062":1}',
    b'{"a":"x"' + b'"y"}', b'{"a":1}' + b'{"b":2', b'[{"a":1},"b":2]', b'{"a":x}',
    b'{"a":1\x01}',
    b'{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":{"a":1}}}}}}}}}}}}}}}}}',
]


def test_stream_invalid_documents_go_to_the_exact_scan():
    """Documents the stream must not prove (object alternation, kinds, depth, escapes in
    keys, whitespace, inexact literals, ...) are handed over — or, where the problem lies
    after the root's close, decided like the oracle."""
    pats = [("a", 1, "1"), ("b", 2, "v"), ("a.b", 1, "2"), ("a.a.a", 3, "x")]
    nodes, root = FU.chain(len(pats))
    docs = INVALID * 3
    slow = _check(pats, nodes, root, *_pack(docs))
    assert slow is not None
    after_root = {b'{"a":1}' + b'{"b":2', b'{"a":1}}'}
    for d, s in zip(docs, slow):
        if d not in after_root:
            assert s, d


def test_stream_keys_with_escapes_and_long_values():
    """A key that needs unescaping, keys and values longer than a lane or a step, strings
    with escaped quotes and backslashes right at lane boundaries."""
    rng = np.random.default_rng(11)
    pats = [("k", 1, "v"), ("long-key-name-%s" % ("x" * 40), 1, "w"), ("s", 2, 'a"b'), ("t.u", 3, "e")]
    nodes, root = FU.chain(len(pats))
    docs = []
    for i in range(128):
        pad = "p" * int(rng.integers(0, 90))
        val = "\\\\" * int(rng.integers(0, 4)) + '\\"' * int(rng.integers(0, 3)) + "q" * int(rng.integers(0, 40))
        parts = ['"pad":"%s"' % pad, '"s":"%s"' % val, '"k":"%s"' % ("v" if i % 2 else "w" * (i % 37)),
                 '"long-key-name-%s":"w"' % ("x" * 40), '"t":{"u":["e","f%s"]}' % ("g" * (i % 50))]
        if i % 5 == 0:
            parts.append('"k\\u0020":"v"')
        rng.shuffle(parts)
        docs.append(("{" + ",".join(parts) + "}").encode())
    assert _check(pats, nodes, root, *_pack(docs)) is not None
    slow = _check(pats, nodes, root, *_pack(docs), mode=0)
    assert not slow[[i for i in range(128) if i % 5]].any()


def test_stream_empty_and_tiny_documents():
    pats = [("a", 1, "1"), ("b", 4, "x")]
    nodes, root = FU.chain(len(pats))
    docs = [b"", b"{}", b"[]", b'{"a":1}', b"1", b'"a"', b"{", b'{"a":1}' * 2, b'{"a":[]}', b'{"b":["x"]}',
            b'{"a":[1,2\x01]}', b'{"b":[1\x01,"x"]}', b'{"b":"x\x01"}']
    _check(pats, nodes, root, *_pack(docs))


@pytest.mark.parametrize("per", [1, 32])
def test_stream_dense_blocks(per):
    """Blocks with more than 8 opens and runs of one-letter keys (the capture loop's open /
    key ordinals; tests/test_gpu_stream.py runs the same documents on the device)."""
    from test_gpu_stream import _dense_docs

    rng = np.random.default_rng(95 + per)
    pats = [("x.0.0.0", 1, "[[[1]]]"), ("y.a.b.c", 3, "v"), ("z.j", 1, "9"), ("z.a", 2, "0"),
            ("y.a.b.c.d.e.f.g", 1, "v"), ("x.0.0.0.0.0.0.0.0", 1, "3")]
    nodes, root = FU.chain(len(pats))
    _check(pats, nodes, root, *_pack(_dense_docs(rng, 96)), per=per)
    # a document whose first block holds 9 opens, the 9th on a selector path, at every
    # misalignment (at 1 and 2 the block's byte 0 lies before the document: the mark that
    # sends it to the exact scan was lost there, and z.a missed)
    d = (b'{"x":[[[[[[[7]]]]]]],"z":{"a":0,"b":1,"c":2,"d":3,"e":4,"f":5,"g":6,"h":7,"i":8,"j":9},'
         b'"y":{"a":{"b":{"c":{"d":{"e":{"f":{"g":"v"}}}}}}}}')
    pats = [("z.a", 2, "0"), ("y.a.b.c", 3, "v")]
    nodes, root = FU.chain(len(pats))
    for mis in range(32):
        _check(pats, nodes, root, *_pack([b"x" * mis, d] if mis else [d]), per=per)
