"""Lane-balance model of the single-pass kernel's token loop (host-only, no GPU):
a wave runs each 64-byte window's token loop as long as its busiest lane. Prints the
iterations per wave and the lane efficiency for requests in arrival order and in the
length-bucketed order (8/32-byte classes), on tiled and on fully unique c2 documents.

  python scripts/sim_lane_balance.py [waves]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from authorino_amd import workloads as W  # noqa: E402


def tokens(d: bytes):
    """Token positions as the kernel iterates them: closing quotes, brackets, and ',' / ':'
    not taken together with the closing quote before them."""
    out, instr, esc, prev_close = [], False, False, -5
    for i, c in enumerate(d):
        if instr:
            if esc:
                esc = False
            elif c == 92:
                esc = True
            elif c == 34:
                instr = False
                out.append(i)
                prev_close = i
            continue
        if c == 34:
            instr = True
        elif c in b"{}[]":
            out.append(i)
        elif c in b",:" and prev_close != i - 1:
            out.append(i)
    return out


def run(arena, offs, lens, label):
    counts, cache = [], {}
    for r in range(len(lens)):
        d = arena[offs[r]:offs[r] + lens[r]].tobytes()
        mis = int(offs[r]) % 16
        if (d, mis) not in cache:
            c = np.zeros(64, int)
            for p in tokens(d):
                c[(p + mis) // 64] += 1
            cache[(d, mis)] = c
        counts.append(cache[(d, mis)])
    C = np.array(counts)
    rng = np.random.default_rng(0)
    orders = {"arrival": np.arange(len(lens))}
    for sh in (3, 5):
        orders[f"len/{1 << sh}B"] = np.lexsort((rng.random(len(lens)), -(lens.astype(np.int64) >> sh)))
    for name, p in orders.items():
        tx = tm = 0.0
        for g in range(0, len(lens) - 63, 64):
            blk = C[p[g:g + 64]]
            tx += blk.max(axis=0).sum()
            tm += blk.mean(axis=0).sum()
        w = len(lens) // 64
        print(f"{label:10s} {name:9s} iterations/wave {tx / w:6.1f}  tokens/doc {tm / w:6.1f}  efficiency {tm / tx:.3f}")


if __name__ == "__main__":
    waves = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    run(*W.make_docs(64 * waves, 2), "tiled")
    run(*W.make_docs(64 * waves, 3, unique=64 * waves), "unique")
