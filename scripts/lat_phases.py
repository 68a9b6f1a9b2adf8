"""Profiling: the streaming kernel's per-phase clock counts on small batches (kernel mode 53:
lane 0 of each one-request wave writes blob copy | stream | stage B over the request's
bitmap word, 21 bits each in units of 16 clocks). Usage: python scripts/lat_phases.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import runtime, workloads  # noqa: E402


def phases(bm, word=0):
    w = bm[:, word].astype(np.uint64)
    f = lambda k: ((w >> np.uint64(21 * k)) & np.uint64(0x1FFFFF)).astype(np.float64) * 16  # noqa: E731
    return f(0), f(1), f(2)


SUB = ("step: loads", "classify+grammar", "keys+stack", "captures", "step end", "B: arrays",
       "B: resolve", "B: tails", "B: patterns")


def sub_phases(label, bm):
    """the stream step's and (whole-wave) stage B's sub-phases (words 1..3)"""
    vals = []
    for word in (1, 2, 3):
        vals.extend(phases(bm, word))
    live = bm[:, 3] != 0
    if not live.any():
        print("  %s: no sub-phase clocks (no whole-wave stage B)" % label)
        return
    print("  %s sub-phases, clocks median over %d requests:" % (label, int(live.sum())))
    print("    " + ", ".join("%s %.0f" % (k, np.median(v[live])) for k, v in zip(SUB, vals)))


def main():
    ctx = runtime.Context(0)
    ctx.set_kernel_mode(53)
    w = workloads.make("c2", n=64, unique=64)
    rs = ctx.compile_expression(w.expr)
    for _ in range(3):
        _, _, bm = ctx.eval_host_arena([rs], w.arena, w.offs, w.lens, bitmap_words=4)
    a, b, c = phases(bm)
    print("c2 n=64 one ruleset: clocks median blob %.0f stream %.0f stageB %.0f (max %.0f %.0f %.0f)" % (
        np.median(a), np.median(b), np.median(c), a.max(), b.max(), c.max()))
    sub_phases("c2", bm)
    w4 = workloads.make("c4", n=65536)
    idx = np.arange(0, 65536, 1024)  # (64 requests of different AuthConfigs)
    sor = w4.set_of_req[idx]
    used = sorted(set(int(x) for x in sor))
    sets = [ctx.compile_expression(w4.exprs[u]) for u in used]
    m = {u: i for i, u in enumerate(used)}
    sor2 = np.array([m[int(x)] for x in sor], dtype=np.uint32)
    for _ in range(3):
        _, _, bm = ctx.eval_host_arena(sets, w4.arena, w4.offs[idx], w4.lens[idx], set_of_req=sor2, bitmap_words=4)
    a, b, c = phases(bm)
    print("c4 n=64 multi-tenant (%d rulesets): clocks median blob %.0f stream %.0f stageB %.0f (max %.0f %.0f %.0f)" % (
        len(used), np.median(a), np.median(b), np.median(c), a.max(), b.max(), c.max()))
    sub_phases("c4", bm)
    ctx.set_kernel_mode(0)


if __name__ == "__main__":
    main()
