"""Profiling aid (not product code): the loops of one kernel in a gfx950 .s file, with
their instruction counts by kind. A loop = the blocks from a label to the last branch back
to it.   python scripts/isa_loops.py file.s KERNEL_SUBSTRING"""
import re
import sys


def kernel_lines(path, name):
    out, on = [], False
    for ln in open(path):
        if not on and re.match(r"^_Z\S*%s\S*:\s*(;.*)?$" % re.escape(name), ln):
            on = True
            continue
        if on:
            if ln.startswith("\t.section") or re.match(r"^\.Lfunc_end", ln):
                break
            out.append(ln.rstrip("\n"))
    return out


def kind(ins):
    op = ins.split()[0]
    if op.startswith("s_waitcnt") or op in ("s_nop",):
        return "wait"
    if op.startswith("v_") :
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "flat_", "buffer_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    L = kernel_lines(path, name)
    items = []  # (label or None, instruction)
    for ln in L:
        t = ln.strip()
        if not t or t.startswith((";", ".")) and not re.match(r"^\.LBB", t):
            continue
        m = re.match(r"^(\.LBB\S+):", t)
        if m:
            items.append(("label", m.group(1)))
            continue
        items.append(("ins", t.split(";")[0].strip()))
    pos = {}
    for k, (ty, v) in enumerate(items):
        if ty == "label":
            pos[v] = k
    loops = {}
    for k, (ty, v) in enumerate(items):
        if ty == "ins" and v.startswith("s_cbranch") or (ty == "ins" and v.startswith("s_branch")):
            tgt = v.split()[-1]
            if tgt in pos and pos[tgt] < k:
                loops[tgt] = max(loops.get(tgt, 0), k)
    tot = {}
    for ty, v in items:
        if ty == "ins":
            tot[kind(v)] = tot.get(kind(v), 0) + 1
    print("kernel", name, "instructions", sum(tot.values()), tot)
    for tgt, end in sorted(loops.items(), key=lambda x: pos[x[0]]):
        c = {}
        for ty, v in items[pos[tgt]:end + 1]:
            if ty == "ins":
                c[kind(v)] = c.get(kind(v), 0) + 1
        print(f"loop {tgt:14s} lines {pos[tgt]:6d}-{end:6d} n={sum(c.values()):5d} {c}")


if __name__ == "__main__":
    main()
