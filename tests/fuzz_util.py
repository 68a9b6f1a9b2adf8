"""Random documents and selector sets for differential tests (oracle vs device logic)."""
import json

import numpy as np

KEYS = ["a", "b", "c", "ab", "x.y", "0", "1", "ké", "long-key-name", "", "a b", "q\"t", "s\\l", "n",
        "a-long-key-name", "b-long-key-name"]
STRS = ["", "x", "hello", "a\"b", "back\\slash", "t\tab", "é", "\U0001F600", "<&>", "1", "true", "null",
        "line\nbreak", " ", "-0", "GET", "/api/v1/orders/7"]
NUMS = ["0", "-0", "1", "-12", "007", "1.5", "1.50", "1e3", "1E-7", "-0.0", "123456789012345", "0.1", "2.5e10",
        "1e400", "12345678901234567890", "3.14159", "100",
        # 16-17 significant digits (Go's encoding/json shortest texts), subnormals, the
        # 1e21 'f'-layout boundary and the float64 ends: decided by the exact scan
        "0.30000000000000004", "37.77492950000001", "-122.41941550000001", "1.0000000000000002",
        "9.999999999999999e20", "1e21", "1.2345678901234567e-5", "4.9406564584124654e-324",
        "2.2250738585072014e-308", "1.7976931348623157e308", "-1.7976931348623157e308", "5e-324",
        "1.7976931348623159e308", "2.4703282292062328e-324", "1234567890123456.7"]


def rand_value(rng, depth):
    r = rng.random()
    if depth <= 0 or r < 0.45:
        k = rng.integers(0, 5)
        if k == 0:
            return ("s", STRS[rng.integers(0, len(STRS))])
        if k == 1:
            return ("n", NUMS[rng.integers(0, len(NUMS))])
        if k == 2:
            return ("l", ["true", "false", "null"][rng.integers(0, 3)])
        return ("s", "v%d" % rng.integers(0, 20))
    if r < 0.75:
        n = int(rng.integers(0, 5))
        return ("o", [(KEYS[rng.integers(0, len(KEYS))], rand_value(rng, depth - 1)) for _ in range(n)])
    n = int(rng.integers(0, 5))
    return ("a", [rand_value(rng, depth - 1) for _ in range(n)])


def dump(v, rng, ws=False):
    sp = (lambda: " " * int(rng.integers(0, 2))) if ws else (lambda: "")
    t, x = v
    if t == "s":
        s = json.dumps(x, ensure_ascii=bool(rng.integers(0, 2)))
        return s
    if t in ("n", "l"):
        return x
    if t == "o":
        return "{" + sp() + ",".join(sp() + json.dumps(k) + sp() + ":" + sp() + dump(val, rng, ws) for k, val in x) + sp() + "}"
    return "[" + sp() + ",".join(sp() + dump(val, rng, ws) for val in x) + sp() + "]"


def rand_doc(rng, ws=None):
    v = ("o", [(KEYS[rng.integers(0, len(KEYS))], rand_value(rng, 4)) for _ in range(int(rng.integers(1, 7)))])
    if rng.random() < 0.1:
        v = ("a", [rand_value(rng, 3) for _ in range(int(rng.integers(0, 4)))])
    return dump(v, rng, ws if ws is not None else bool(rng.random() < 0.3)).encode("utf-8")


def esc_key(k):
    return k.replace("\\", "\\\\").replace(".", "\\.")


def rand_selector(rng):
    n = int(rng.integers(1, 4))
    parts = []
    for _ in range(n):
        if rng.random() < 0.25:
            parts.append(str(int(rng.integers(0, 3))))
        else:
            parts.append(esc_key(KEYS[rng.integers(0, len(KEYS))]))
    return ".".join(parts)


def rand_patterns(rng, k):
    ops = [1, 2, 3, 4]
    out = []
    for _ in range(k):
        op = ops[rng.integers(0, len(ops))]
        if rng.random() < 0.5:
            val = STRS[rng.integers(0, len(STRS))]
        elif rng.random() < 0.5:
            val = NUMS[rng.integers(0, len(NUMS))]
        else:
            val = ["true", "false", "", "v3", "[]", "{}"][rng.integers(0, 6)]
        if rng.random() < 0.1:
            op = 5
            val = ["^v\\d+$", "(?i)HELLO", "^$", "\\d", "é", "^/api/v[0-9]+/", "[^a-z]", "true|false"][rng.integers(0, 8)]
        out.append((rand_selector(rng), op, val))
    return out


def mutate(rng, d: bytes) -> bytes:
    d = bytearray(d)
    m = int(rng.integers(0, 6))
    if m == 0 and len(d) > 1:
        d = d[: int(rng.integers(0, len(d)))]
    elif m == 1 and len(d):
        for _ in range(int(rng.integers(1, 3))):
            d[int(rng.integers(0, len(d)))] = int(rng.choice(list(b'{}[]":,\\ 0aeu\x01\xff(')))
    elif m == 2 and len(d) > 2:
        i = int(rng.integers(0, len(d) - 1))
        del d[i:i + int(rng.integers(1, 3))]
    elif m == 3:
        d = bytearray(b" \t" + bytes(d) + b" tail")
    elif m == 4 and len(d):
        i = int(rng.integers(0, len(d)))
        d[i:i] = bytes(rng.choice([b"\\", b'"', b"1", b"{", b"]", b"x"]))
    return bytes(d)


def _ws(rng):
    return "".join(str(rng.choice([" ", "\n", "\t", "\r"])) for _ in range(int(rng.integers(0, 3)) * int(rng.integers(0, 12))))


def dump_ws(v, rng):
    """Like dump() but with whitespace runs of 0..22 bytes around every token (scalars
    and keys whose bytes straddle 16-byte blocks, literals followed by long runs)."""
    t, x = v
    if t == "s":
        return json.dumps(x, ensure_ascii=bool(rng.integers(0, 2)))
    if t in ("n", "l"):
        return x
    w = lambda: _ws(rng)  # noqa: E731
    if t == "o":
        return "{" + w() + ",".join(w() + json.dumps(k) + w() + ":" + w() + dump_ws(val, rng) + w() for k, val in x) + w() + "}"
    return "[" + w() + ",".join(w() + dump_ws(val, rng) + w() for val in x) + w() + "]"


def rand_doc_ws(rng):
    v = ("o", [(KEYS[rng.integers(0, len(KEYS))], rand_value(rng, 4)) for _ in range(int(rng.integers(1, 7)))])
    return (_ws(rng) + dump_ws(v, rng) + _ws(rng)).encode("utf-8")


def chain(n):
    nodes = [(0, -1, -1, i) for i in range(n)]
    root = -1
    for i in reversed(range(n)):
        nodes.append((1, i, root, -1))
        root = len(nodes) - 1
    return nodes, root


def long_doc(rng, pats):
    """A compact document whose selector values are long strings / arrays, placed after
    padding so that they straddle line boundaries."""
    parts = []
    for k in range(int(rng.integers(1, 6))):
        parts.append('"pad%d":"%s"' % (k, "p" * int(rng.integers(0, 300))))
    for sel, op, val in pats:
        keys = sel.split(".")
        if any(not k or "\\" in k or '"' in k for k in keys):
            continue
        v = rng.random()
        if v < 0.3:
            inner = json.dumps(val) if rng.random() < 0.5 else '"%s"' % ("L" * int(rng.integers(100, 300)))
        elif v < 0.6:
            inner = "[" + ",".join('"%s"' % ("e" * int(rng.integers(0, 150))) for _ in range(int(rng.integers(0, 6)))) + "]"
        elif v < 0.8:
            inner = "[" + ",".join(['{"k":"%s"}' % ("o" * int(rng.integers(0, 90))), "12", "true", "null", json.dumps(val)]) + "]"
        else:
            inner = str(int(rng.integers(-10**12, 10**12)))
        for k in reversed(keys):
            inner = "{%s:%s}" % (json.dumps(k, ensure_ascii=False), inner)
        parts.append(inner[1:-1])
    rng.shuffle(parts)
    return ("{" + ",".join(parts) + "}").encode()
