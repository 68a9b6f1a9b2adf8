"""Model of the lean walk's wave cost (profiling aid, not product code).

The host build of ajx_lean.h traces every walker iteration of a document (sub-window,
token kind; AJX_LEAN_TRACE). Requests go to waves of 64 in the kernel's length order; a
wave runs each sub-window's token loop as long as its busiest lane, and an iteration costs
the union of the branches its lanes take. The model compares that with other schedules:

  lockstep   now: iteration j of sub-window s runs every kind that some lane's j-th token has
  typed      each step runs ONE kind (the most common among the lanes' next tokens); lanes
             whose next token is another kind wait
  window64   lockstep over 64-byte windows (two sub-windows per loop)

  python scripts/sim_walk_sched.py [--workload c2] [--n 8192]
"""
import argparse
import collections
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

KINDS = ["squash", "str_elem", "pend_val", "key_str", "key_cont", "key_scalar", "root", "elem_cont", "close",
         "scalar_elem"]
# rough per-kind cost in wave instructions (VALU + SALU) of the branch body
COST = [20, 90, 60, 140, 120, 110, 40, 100, 50, 90]
OVERHEAD = 30  # loop head: ctz, bit clear, dispatch tests
KIND_ITERS = collections.Counter()  # iterations in which some lane runs each kind
NKINDS = []


def traces(expr, docs):
    import _hosttest as H

    L = H.lib()
    L.ht_lean_trace.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    L.ht_lean_trace.restype = C.c_uint32
    hr = H.HostRuleset.from_expression(expr)
    buf = (C.c_uint32 * (1 << 16))()
    out = []
    for d in docs:
        L.ht_lean_trace(buf, 1 << 16)
        H.eval_lean(hr, d, mis=0)
        n = L.ht_lean_trace(None, 0)
        t = np.frombuffer(buf, dtype=np.uint32, count=n).copy()
        out.append((t >> 8, t & 0xFF))
    return out


def per_sub(tr, window=1):
    sub, kind = tr
    g = collections.defaultdict(list)
    for s, k in zip(sub.tolist(), kind.tolist()):
        g[s // window].append(k)
    return g


def wave_costs(wave, window=1):
    subs = [per_sub(t, window) for t in wave]
    keys = set()
    for g in subs:
        keys |= set(g)
    lock = typed = iters = tsteps = 0
    for s in sorted(keys):
        seqs = [g.get(s, []) for g in subs]
        m = max(len(q) for q in seqs)
        iters += m
        for j in range(m):
            present = {q[j] for q in seqs if j < len(q)}
            lock += OVERHEAD + sum(COST[k] for k in present)
            KIND_ITERS.update(present)
            NKINDS.append(len(present))
        heads = [0] * len(seqs)
        while True:
            c = collections.Counter(q[h] for q, h in zip(seqs, heads) if h < len(q))
            if not c:
                break
            k = c.most_common(1)[0][0]
            tsteps += 1
            typed += OVERHEAD + 12 + COST[k]
            for i, q in enumerate(seqs):
                if heads[i] < len(q) and q[heads[i]] == k:
                    heads[i] += 1
    return lock, typed, iters, tsteps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--n", type=int, default=4096)
    a = ap.parse_args()
    from authorino_amd import workloads

    w = workloads.make(a.workload, n=a.n, unique=a.n, uniquify=True)
    docs = [w.doc(i) for i in range(w.n)]
    order = np.argsort(-(w.lens.astype(np.int64) >> 3), kind="stable")  # the kernel's length classes
    trs = traces(w.expr, [docs[i] for i in order])
    kinds = collections.Counter()
    for _, k in trs:
        kinds.update(k.tolist())
    print("tokens per doc:", round(sum(kinds.values()) / len(trs), 1),
          {KINDS[k]: round(v / len(trs), 1) for k, v in sorted(kinds.items())})
    tot = collections.Counter()
    for b in range(0, len(trs) - 63, 64):
        wave = trs[b:b + 64]
        l1, t1, i1, s1 = wave_costs(wave, 1)
        l2, _, i2, _ = wave_costs(wave, 2)
        tot.update({"lock": l1, "typed": t1, "iters": i1, "typed_steps": s1, "win64": l2, "win64_iters": i2,
                    "waves": 1})
    nw = tot["waves"]
    print({k: round(v / nw, 1) for k, v in tot.items()})
    print("kinds per lockstep iteration:", round(float(np.mean(NKINDS)), 2),
          "iterations per wave running each kind:", {KINDS[k]: round(v / nw / 2, 1) for k, v in KIND_ITERS.items()})


if __name__ == "__main__":
    main()
