"""Round-4 launch-failure analysis (profiling aid, not product code).

Runs the streaming kernel's host emulation (ajx_stream.h on ajx_wave.h's 64 host threads)
of a given checkout under AddressSanitizer + UBSan on the inputs of the failing round-4
tests: the reference KATs as one-request batches (test_reference_kats_via_jsonexp_api,
where `unspecified launch failure` was reported) and dense blocks (more than 8 opens / keys
in one 32-byte block, round 5's regression test), at every misalignment and 1, 2, 31 and
64 requests per wave. Reports what the sanitizers find; results are compared with the
oracle of the current tree.

  LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libstdc++.so.6)" \\
  ASAN_OPTIONS=detect_leaks=0 \\
    python scripts/r4_stream_san.py /tmp/r4pre      # a checkout built with -fsanitize
"""
import json
import os
import sys

import numpy as np

tree = sys.argv[1]
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "oracle"))
import pyoracle as O  # noqa: E402  (the current tree's oracle: the expected results)

sys.path.insert(0, os.path.join(tree, "tests"))
sys.path.insert(0, tree)
import _hosttest as H  # noqa: E402  (the checkout's host build)


def dense_docs(rng, n):
    out = []
    for _ in range(n):
        k = int(rng.integers(6, 20))
        arr = "[" * k + str(int(rng.integers(0, 9))) + "]" * k
        keys = "abcdefghij"
        obj = "".join('{"%s":' % keys[j % 10] for j in range(k)) + '"v"' + "}" * k
        flat = "{" + ",".join('"%s":%d' % (keys[j], j) for j in range(10)) + "}"
        parts = [('"x"', arr), ('"y"', obj), ('"z"', flat)]
        rng.shuffle(parts)
        out.append(("{" + ",".join("%s:%s" % p for p in parts) + "}").encode())
    return out


def chain(n):
    nodes = [(0, -1, -1, i) for i in range(n)]
    root = -1
    for i in reversed(range(n)):
        nodes.append((1, i, root, -1))
        root = len(nodes) - 1
    return nodes, root


def run(pats, nodes, root, docs, per_list, mis_list, tag):
    hr = H.HostRuleset(pats, nodes, root)
    ors = O.Ruleset(pats, nodes, root)
    bad = checked = 0
    for mis in mis_list:
        for per in per_list:
            parts = [b"\x7a" * mis]
            offs, lens, pos = [], [], mis
            for d in docs:
                offs.append(pos)
                lens.append(len(d))
                parts.append(d)
                pos += len(d)
            arena = np.frombuffer(b"".join(parts), dtype=np.uint8)
            offs = np.array(offs, np.uint64)
            lens = np.array(lens, np.uint32)
            r = H.eval_stream(hr, arena, offs, lens, per=per)
            if r is None:
                print(f"{tag}: no stream tables for this ruleset in this checkout", flush=True)
                return 0, 0
            tri, slow = r[0], r[3]
            otri, _, _ = O.eval_batch([ors], arena, offs, lens, nthreads=4)
            dec = slow != 1  # (slow == 1: handed to the exact scan, which the emulation does not run)
            checked += int(dec.sum())
            bad += int((tri[dec] != otri[dec]).sum())
    print(f"{tag}: {checked} requests decided by the stream, {bad} differ from the oracle", flush=True)
    return checked, bad


def main():
    sys.path.insert(0, os.path.join(HERE, "tests"))
    sys.path.insert(0, HERE)
    import kat_util as K  # (the current tree's KAT loader)

    n = 0
    for c in K.load_kats():
        e = K.build(c.get("tree"))
        if e is None:
            continue
        pats, nodes, root = K.flat(e)
        run(pats, nodes, root, [c["doc"].encode()], [1], range(16), f"kat {n}")
        n += 1
    rng = np.random.default_rng(94)
    pats = [("x.0.0.0", 1, "[[[1]]]"), ("y.a.b.c", 3, "v"), ("z.j", 1, "9"), ("z.a", 2, "0"),
            ("y.a.b.c.d.e.f.g", 1, "v"), ("x.0.0.0.0.0.0.0.0", 1, "3")]
    nodes, root = chain(len(pats))
    docs = dense_docs(rng, 64)
    run(pats, nodes, root, docs, [1, 2, 31, 32], range(16), "dense blocks")
    # (without the array-index selectors, which round 4's stream tables did not take)
    pats = [("y.a.b.c", 3, "v"), ("z.j", 1, "9"), ("z.a", 2, "0"), ("y.a.b", 1, "x"), ("x", 2, "[]")]
    nodes, root = chain(len(pats))
    run(pats, nodes, root, docs, [1, 2, 31, 32], range(16), "dense blocks, key selectors")
    print("done")


if __name__ == "__main__":
    main()
