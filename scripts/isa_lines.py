"""Profiling aid (not product code): static instruction counts of one kernel by source
line (from a `hipcc -g -S` listing's .loc directives), optionally only inside the loops whose
header line lies in a given source range.
  python scripts/isa_lines.py file.s KERNEL_SUBSTRING FILE_NO [LINE_LO LINE_HI]"""
import collections
import re
import sys


def main():
    path, name, fno = sys.argv[1], sys.argv[2], int(sys.argv[3])
    lo, hi = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (0, 1 << 30)
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cur = (None, 0)
    cnt = collections.Counter()
    kinds = collections.defaultdict(collections.Counter)
    for l in lines[st:en]:
        t = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (int(m.group(1)), int(m.group(2)))
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if cur[0] == fno and lo <= cur[1] <= hi:
            cnt[cur[1]] += 1
            k = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_") else "m"
            kinds[cur[1]][k] += 1
    tot = sum(cnt.values())
    print("total", tot)
    for ln, c in sorted(cnt.items()):
        print(f"{ln:5d} {c:5d}  {dict(kinds[ln])}")


if __name__ == "__main__":
    main()
