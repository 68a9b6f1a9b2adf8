"""TEST-ONLY ctypes binding of tests/native/libajx_hosttest.so (host build of the kernels'
per-document logic, for CPU-side debugging against the oracle). Not product code."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_NATIVE = os.path.join(_HERE, "native")
_L = None


class _Pattern(C.Structure):
    _fields_ = [("selector", C.c_char_p), ("selector_len", C.c_uint32), ("op", C.c_int32),
                ("value", C.c_char_p), ("value_len", C.c_uint32)]


class _Node(C.Structure):
    _fields_ = [("kind", C.c_int32), ("left", C.c_int32), ("right", C.c_int32), ("pattern", C.c_int32)]


class _Tree(C.Structure):
    _fields_ = [("patterns", C.POINTER(_Pattern)), ("n_patterns", C.c_uint32),
                ("nodes", C.POINTER(_Node)), ("n_nodes", C.c_uint32), ("root", C.c_int32)]


def lib():
    global _L
    if _L is None:
        path = os.environ.get("AJX_HOSTTEST_LIB")  # (debugging: e.g. an ASan build of the same sources)
        if not path:
            subprocess.run(["make", "-s", "-C", _NATIVE], check=True)
            path = os.path.join(_NATIVE, "libajx_hosttest.so")
        L = C.CDLL(path)
        L.ht_compile.argtypes = [C.POINTER(_Tree), C.POINTER(C.c_int32), C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
        L.ht_compile.restype = C.c_void_p
        L.ht_free.argtypes = [C.c_void_p]
        L.ht_eval.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]
        L.ht_eval.restype = C.c_int
        L.ht_get.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ht_get.restype = C.c_int
        L.ht_string.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32]
        L.ht_select_value.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                      C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ht_select_value.restype = C.c_int
        L.ht_inject_truncate.argtypes = [C.c_int]
        L.ht_json_valid.argtypes = [C.c_char_p, C.c_uint32]
        L.ht_json_valid.restype = C.c_int
        L.ht_string.restype = C.c_int
        L.ht_regex.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
        L.ht_regex.restype = C.c_void_p
        L.ht_regex_free.argtypes = [C.c_void_p]
        L.ht_regex_states.argtypes = [C.c_void_p]
        L.ht_regex_states.restype = C.c_uint32
        L.ht_regex_match.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32]
        L.ht_regex_match.restype = C.c_int
        _L = L
    return _L


def _b(s):
    return s if isinstance(s, bytes) else s.encode("utf-8")


def make_tree(patterns, nodes, root):
    keep = []
    parr = (_Pattern * max(len(patterns), 1))()
    for i, (sel, op, val) in enumerate(patterns):
        sb, vb = _b(sel), _b(val)
        keep += [sb, vb]
        parr[i] = _Pattern(sb, len(sb), int(op), vb, len(vb))
    narr = (_Node * max(len(nodes), 1))()
    for i, nd in enumerate(nodes):
        narr[i] = _Node(*nd)
    keep += [parr, narr]
    t = _Tree(parr, len(patterns), narr, len(nodes), root)
    return t, keep


class HostRuleset:
    def __init__(self, patterns, nodes, root):
        self.n = len(patterns)
        t, self._keep = make_tree(patterns, nodes, root)
        st = (C.c_int32 * max(self.n, 1))()
        err = C.create_string_buffer(512)
        rc = C.c_int(0)
        self._h = lib().ht_compile(C.byref(t), st, err, 512, C.byref(rc))
        self.rc = rc.value
        self.status = list(st)[: self.n]
        self.error = err.value.decode()

    @classmethod
    def forest(cls, trees):
        """trees: [(patterns, nodes, root)] compiled as one forest ruleset (ht_compile_forest;
        root -1: a root-less tree, whose selectors' capture records the kernel keeps)."""
        self = cls.__new__(cls)
        built = [make_tree(*t) for t in trees]
        self._keep = [k for _, k in built]
        arr = (_Tree * len(trees))(*[t for t, _ in built])
        self._keep.append(arr)
        self.n = sum(len(t[0]) for t in trees)
        err = C.create_string_buffer(512)
        rc = C.c_int(0)
        L = lib()
        L.ht_compile_forest.argtypes = [C.POINTER(_Tree), C.c_uint32, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
        L.ht_compile_forest.restype = C.c_void_p
        self._h = L.ht_compile_forest(arr, len(trees), err, 512, C.byref(rc))
        self.rc = rc.value
        self.status = []
        self.error = err.value.decode()
        return self

    @classmethod
    def with_selector_tree(cls, expr):
        """expr's tree plus a root-less tree of an EQ "" pattern per selector (the response
        selectors' shape, runtime.Context.compile_forest(extra_selectors=...)): every
        selector's capture record is kept."""
        pats, nodes, root = expr.flatten()
        sels = list(dict.fromkeys(p.selector for p in pats))
        return cls.forest([([(p.selector, int(p.operator), p.value) for p in pats], nodes, root),
                           ([(s, 1, "") for s in sels], [], -1)])

    @classmethod
    def from_expression(cls, expr):
        pats, nodes, root = expr.flatten()
        return cls([(p.selector, int(p.operator), p.value) for p in pats], nodes, root)

    def eval(self, doc):
        d = _b(doc)
        res = (C.c_uint8 * max(self.n, 1))()
        err = C.c_int32(-1)
        t = lib().ht_eval(self._h, d, len(d), res, C.byref(err))
        return t, err.value, list(res)[: self.n]

    def select_value(self, p, doc, text, used):
        """select_value of pattern p's selector (the select kernel's TEXT instance): (rc,
        [start, len, type | esc << 8], used) with built text appended to `text` (bytearray)."""
        d = _b(doc)
        buf = (C.c_uint8 * len(text)).from_buffer(text)
        u = C.c_uint32(used)
        out = (C.c_uint32 * 3)()
        rc = lib().ht_select_value(self._h, p, d, len(d), buf, len(text), C.byref(u), out)
        return rc, list(out), u.value

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ht_free(self._h)


def get(doc, path):
    d, p = _b(doc), _b(path)
    s, e = C.c_uint32(), C.c_uint32()
    t = lib().ht_get(p, len(p), d, len(d), C.byref(s), C.byref(e))
    return t, d[s.value:e.value] if t >= 0 else b""


def string(doc, path):
    d, p = _b(doc), _b(path)
    buf = C.create_string_buffer(1 << 16)
    k = lib().ht_string(p, len(p), d, len(d), buf, 1 << 16)
    if k < 0:
        return k
    return buf.raw[:k]


class HostRegex:
    def __init__(self, pat):
        p = _b(pat)
        st = C.c_int()
        err = C.create_string_buffer(512)
        self._h = lib().ht_regex(p, len(p), C.byref(st), err, 512)
        self.status = st.value
        self.error = err.value.decode("utf-8", "replace")

    def match(self, s):
        s = _b(s)
        return bool(lib().ht_regex_match(self._h, s, len(s)))

    @property
    def states(self):
        return lib().ht_regex_states(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ht_regex_free(self._h)


def _fast_decl():
    L = lib()
    if not hasattr(L, "_fast_declared"):
        L.ht_eval_fast.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8),
                                   C.POINTER(C.c_int32)]
        L.ht_eval_fast.restype = C.c_int
        L.ht_eval_tok.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8),
                                  C.POINTER(C.c_int32), C.c_void_p]
        L.ht_eval_tok.restype = C.c_int
        L._fast_declared = True
    return L


def eval_fast(hr: "HostRuleset", doc, mis: int = 0):
    """Single-pass path on the host: (tri | -1 slow | -2 not eligible, err, res)."""
    L = _fast_decl()
    d = _b(doc)
    res = (C.c_uint8 * max(hr.n, 1))()
    err = C.c_int32(-1)
    t = L.ht_eval_fast(hr._h, d, len(d), mis, res, C.byref(err))
    return t, err.value, list(res)[: hr.n]


def eval_tok(hr: "HostRuleset", doc, mis: int = 0, n_sel: int = 0):
    """The token-scanner single-pass path on the host: (tri | -1 slow | -2 not eligible,
    err, res, capture row [found, records...] or None)."""
    L = _fast_decl()
    d = _b(doc)
    res = (C.c_uint8 * max(hr.n, 1))()
    err = C.c_int32(-1)
    row = (C.c_uint64 * (1 + max(n_sel, 64)))()
    t = L.ht_eval_tok(hr._h, d, len(d), mis, res, C.byref(err), C.cast(row, C.c_void_p))
    return t, err.value, list(res)[: hr.n], (list(row)[: 1 + n_sel] if t >= 0 else None)




def _lean_decl():
    L = lib()
    if not hasattr(L, "_lean_declared"):
        L.ht_eval_lean_row.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8),
                                       C.POINTER(C.c_int32), C.c_void_p]
        L.ht_eval_lean_row.restype = C.c_int
        L.ht_lean_classes.argtypes = [C.c_char_p, C.POINTER(C.c_uint32)]
        L.ht_lean_classes.restype = None
        L._lean_declared = True
    return L


def lean_keep(keep: bool) -> None:
    """keep False: the lean scan writes only the capture records stage B needs (the
    kernel's default when no caller reads the rows); True: also those of the selectors a
    caller reads back (a forest's root-less trees, kEagerKeep)."""
    L = lib()
    L.ht_lean_keep.argtypes = [C.c_int]
    L.ht_lean_keep(1 if keep else 0)


def eval_lean(hr: "HostRuleset", doc, mis: int = 0, n_sel: int = 0):
    """The lean single-pass scan (ajx_lean.h) + stage B on the host: (tri | -1 exact scan |
    -2 not eligible, err, res, capture row or None)."""
    L = _lean_decl()
    d = _b(doc)
    res = (C.c_uint8 * max(hr.n, 1))()
    err = C.c_int32(-1)
    row = (C.c_uint64 * (1 + max(n_sel, 64)))()
    t = L.ht_eval_lean_row(hr._h, d, len(d), mis, res, C.byref(err), C.cast(row, C.c_void_p))
    return t, err.value, list(res)[: hr.n], (list(row)[: 1 + n_sel] if t >= 0 else None)


def lean_classes(b32: bytes):
    """The lean scan's eight byte-class masks of 32 bytes (LUT + transpose)."""
    L = _lean_decl()
    out = (C.c_uint32 * 8)()
    L.ht_lean_classes(bytes(b32), out)
    return list(out)


def lean_last_dec():
    """(decided, true) pattern bits of the last eval_lean (eager patterns)."""
    L = _lean_decl()
    out = (C.c_uint64 * 2)()
    L.ht_lean_last_dec(out)
    return out[0], out[1]


def json_valid(text) -> int:
    """gjson Valid as the device restates it: 1 / 0, -1 undecided (nesting > 256)."""
    d = _b(text)
    return lib().ht_json_valid(d, len(d))


def eval_stream(hr, arena, offs, lens, mode=0, stride=2, dbg=None, per=0):
    """The streaming scan (ajx_stream.h) over a batch on the host emulation of the wave,
    then its stage B: (tri, err, bitmap, slow) — slow[r] = 1 where request r goes to the
    exact scan, 2 where stage B decided it; None when the ruleset has no stream tables.
    per: requests per wave (0: 32)."""
    L = lib()
    if not getattr(L, "_stream_decl", False):
        L.ht_eval_stream.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p, C.c_uint32]
        L.ht_eval_stream.restype = C.c_int
        L._stream_decl = True
    import numpy as np

    n = len(lens)
    a = np.concatenate([np.asarray(arena, dtype=np.uint8), np.zeros(64, np.uint8)])
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    tri = np.full(n, 0xEE, np.uint8)
    err = np.full(n, -7, np.int32)
    bm = np.zeros((n, stride), np.uint64)
    slow = np.zeros(n, np.uint8)
    rc = L.ht_eval_stream(hr._h, a.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, tri.ctypes.data,
                          err.ctypes.data, bm.ctypes.data, stride, slow.ctypes.data, mode,
                          None if dbg is None else dbg.ctypes.data, per)
    if rc < 0:
        return None
    return tri, err, bm, slow
