"""Profiling aid (not product code): instructions of one kernel grouped by the innermost
loop (the compiler's `; in Loop: Header=... Depth=...` block comments).
  python scripts/isa_loopcount.py file.s KERNEL_SUBSTRING"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l))
en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur = "top"
cnt = collections.defaultdict(collections.Counter)
for l in lines[st:en]:
    t = l.strip()
    m = re.search(r"(in Loop|This (?:Inner )?Loop Header): (?:Header=)?(BB\S+)? ?Depth=(\d+)", t)
    if t.endswith(":") or t.startswith("; %bb") or t.startswith(".LBB"):
        m2 = re.search(r"Header=(BB\S+) Depth=(\d+)", t)
        m3 = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", t)
        lab = re.match(r"^(\.LBB\S+|; %bb\.\d+)", t)
        if m2:
            cur = "%s/d%s" % (m2.group(1), m2.group(2))
        elif m3 and lab:
            cur = "%s/d%s" % (lab.group(1).lstrip(".").replace("; %bb.", "BB2_"), m3.group(1))
        else:
            cur = "top"
        continue
    if t.startswith("; =>") and "Loop Header" in t:
        m3 = re.search(r"Depth=(\d+)", t)
        continue
    if not t or t.startswith((".", ";")):
        continue
    op = t.split()[0]
    k = "s" if op.startswith("s_") else "v" if op.startswith("v_") else "ds" if op.startswith("ds_") else "m"
    cnt[cur][k] += 1
for k, c in sorted(cnt.items(), key=lambda x: -sum(x[1].values()))[:25]:
    print("%-22s %6d %s" % (k, sum(c.values()), dict(c)))
