"""Profiling aid (not product code): scratch (spill) accesses inside loops of a kernel.
A scratch access in the walk or window loop waits on vmcnt behind the document's LDS-DMA
loads in flight (in-order), which exposes their latency; this counts them per loop.
  python scripts/isa_scratch_in_loops.py file.s KERNEL_SUBSTRING"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l))
en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur = "top"
c = collections.Counter()
for l in lines[st:en]:
    t = l.strip()
    if t.endswith(":") or t.startswith("; %bb") or t.startswith(".LBB"):
        m2 = re.search(r"Header=(BB\S+) Depth=(\d+)", t)
        m3 = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", t)
        lab = re.match(r"^(\.LBB\S+|; %bb\.\d+)", t)
        cur = (m2.group(1) + "/d" + m2.group(2)) if m2 else (
            (lab.group(1).lstrip(".").replace("; %bb.", "BB") + "/d" + m3.group(1)) if m3 and lab else "top")
        continue
    if t.startswith("scratch_"):
        c[cur] += 1
print(name, dict(c))
