"""pyoracle — TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (liboracle.so).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
The product (authorino_amd / libauthjx.so) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

T_NULL, T_FALSE, T_NUMBER, T_STRING, T_TRUE, T_JSON = range(6)
F, T, E, UNSUPPORTED = 0, 1, 2, 3


class _Buf(C.Structure):
    _fields_ = [("p", C.c_void_p), ("n", C.c_size_t), ("cap", C.c_size_t)]


class _Result(C.Structure):
    _fields_ = [
        ("type", C.c_int),
        ("raw", C.c_void_p),
        ("raw_len", C.c_size_t),
        ("str", C.c_void_p),
        ("str_len", C.c_size_t),
        ("num", C.c_double),
        ("own", _Buf),
    ]


class _Pattern(C.Structure):
    _fields_ = [
        ("selector", C.c_char_p),
        ("selector_len", C.c_uint32),
        ("op", C.c_int32),
        ("value", C.c_char_p),
        ("value_len", C.c_uint32),
    ]


class _Node(C.Structure):
    _fields_ = [("kind", C.c_int32), ("left", C.c_int32), ("right", C.c_int32), ("pattern", C.c_int32)]


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.or_gjson_get.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(_Result)]
        L.or_gjson_get.restype = C.c_int
        L.or_gjson_get_mods.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(_Result),
                                        C.POINTER(_Buf)]
        L.or_gjson_get_mods.restype = C.c_int
        L.or_valid.argtypes = [C.c_char_p, C.c_size_t]
        L.or_valid.restype = C.c_int
        L.or_result_string.argtypes = [C.POINTER(_Result), C.POINTER(_Buf)]
        L.or_result_array_next.argtypes = [C.POINTER(_Result), C.POINTER(C.c_size_t), C.POINTER(_Result)]
        L.or_result_array_next.restype = C.c_int
        L.or_result_free.argtypes = [C.POINTER(_Result)]
        L.or_buf_free.argtypes = [C.POINTER(_Buf)]
        L.or_unescape.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(_Buf)]
        L.or_go_parse_float.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_double)]
        L.or_go_parse_float.restype = C.c_int
        L.or_go_format_float.argtypes = [C.c_double, C.POINTER(_Buf)]
        L.or_regex_compile.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
        L.or_regex_compile.restype = C.c_void_p
        L.or_regex_match.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        L.or_regex_match.restype = C.c_int
        L.or_regex_free.argtypes = [C.c_void_p]
        L.or_ruleset_new.argtypes = [C.POINTER(_Pattern), C.c_uint32, C.POINTER(_Node), C.c_uint32, C.c_int32]
        L.or_ruleset_new.restype = C.c_void_p
        L.or_ruleset_free.argtypes = [C.c_void_p]
        L.or_pattern_matches.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]
        L.or_pattern_matches.restype = C.c_int
        L.or_expression_matches.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_int32)]
        L.or_expression_matches.restype = C.c_int
        L.or_pattern_error.argtypes = [C.c_void_p, C.c_uint32]
        L.or_pattern_error.restype = C.c_char_p
        L.or_eval_batch.argtypes = [
            C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int,
        ]
        _LIB = L
    return _LIB


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else s.encode("utf-8")


def _buf_bytes(b: _Buf) -> bytes:
    return C.string_at(b.p, b.n) if b.n else b""


def gjson_get(doc, path) -> Tuple[int, bytes, bytes]:
    """-> (type, raw, String())"""
    L = lib()
    d, p = _b(doc), _b(path)
    r = _Result()
    rc = L.or_gjson_get(d, len(d), p, len(p), C.byref(r))
    if rc != 0:
        raise ValueError(f"oracle: unsupported selector {path!r}")
    b = _Buf()
    L.or_result_string(C.byref(r), C.byref(b))
    out = (r.type, C.string_at(r.raw, r.raw_len) if r.raw_len else b"", _buf_bytes(b))
    L.or_buf_free(C.byref(b))
    L.or_result_free(C.byref(r))
    return out


def gjson_string_mods(doc, path):
    """String() of gjson.Get(doc, path) for a path with the reference's modifiers
    (gjson_mods_ref.c); None when undecided (non-ASCII text under @case / @strip)."""
    L = lib()
    d, p = _b(doc), _b(path)
    r = _Result()
    text = _Buf()
    rc = L.or_gjson_get_mods(d, len(d), p, len(p), C.byref(r), C.byref(text))
    if rc == -1:
        L.or_buf_free(C.byref(text))
        raise ValueError(f"oracle: unsupported selector {path!r}")
    out = None
    if rc == 0:
        b = _Buf()
        L.or_result_string(C.byref(r), C.byref(b))
        out = _buf_bytes(b)
        L.or_buf_free(C.byref(b))
    L.or_result_free(C.byref(r))
    L.or_buf_free(C.byref(text))
    return out


def valid(text) -> bool:
    """gjson Valid (or_valid, the recursive restatement)."""
    d = _b(text)
    return lib().or_valid(d, len(d)) == 1


def gjson_get_mods(doc, path):
    """(type, raw) of gjson.Get(doc, path) with the path's modifiers (gjson_mods_ref.c);
    None when undecided (non-ASCII text under @case / @strip)."""
    L = lib()
    d, p = _b(doc), _b(path)
    r = _Result()
    text = _Buf()
    rc = L.or_gjson_get_mods(d, len(d), p, len(p), C.byref(r), C.byref(text))
    if rc == -1:
        L.or_buf_free(C.byref(text))
        raise ValueError(f"oracle: unsupported selector {path!r}")
    out = None
    if rc == 0:
        out = (r.type, C.string_at(r.raw, r.raw_len) if r.raw_len else b"")
    L.or_result_free(C.byref(r))
    L.or_buf_free(C.byref(text))
    return out


def gjson_span(doc, path) -> Tuple[int, int, int]:
    """-> (type, start, length): gjson.Get's Raw as a span of the document"""
    L = lib()
    d, p = _b(doc), _b(path)
    buf = C.create_string_buffer(d, len(d))
    r = _Result()
    rc = L.or_gjson_get(buf, len(d), p, len(p), C.byref(r))
    if rc != 0:
        raise ValueError(f"oracle: unsupported selector {path!r}")
    start = (r.raw - C.addressof(buf)) if r.raw_len else 0
    out = (r.type, start, r.raw_len)
    L.or_result_free(C.byref(r))
    return out


def gjson_array(doc, path) -> List[bytes]:
    L = lib()
    d, p = _b(doc), _b(path)
    r = _Result()
    L.or_gjson_get(d, len(d), p, len(p), C.byref(r))
    cur = C.c_size_t(0)
    it = _Result()
    out = []
    while L.or_result_array_next(C.byref(r), C.byref(cur), C.byref(it)):
        b = _Buf()
        L.or_result_string(C.byref(it), C.byref(b))
        out.append(_buf_bytes(b))
        L.or_buf_free(C.byref(b))
    L.or_result_free(C.byref(it))
    L.or_result_free(C.byref(r))
    return out


def parse_float(s) -> Tuple[int, float]:
    v = C.c_double()
    rc = lib().or_go_parse_float(_b(s), len(_b(s)), C.byref(v))
    return rc, v.value


def format_float(f: float) -> bytes:
    b = _Buf()
    lib().or_go_format_float(f, C.byref(b))
    out = _buf_bytes(b)
    lib().or_buf_free(C.byref(b))
    return out


class Regex:
    def __init__(self, pattern):
        p = _b(pattern)
        err = C.create_string_buffer(512)
        uns = C.c_int(0)
        self._h = lib().or_regex_compile(p, len(p), err, 512, C.byref(uns))
        self.error = err.value.decode("utf-8", "replace") if not self._h else None
        self.unsupported = bool(uns.value)

    def match(self, s) -> bool:
        s = _b(s)
        return bool(lib().or_regex_match(self._h, s, len(s)))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_regex_free(self._h)
            self._h = None


class Ruleset:
    """Oracle checker for one flattened expression tree (see authorino_amd.jsonexp)."""

    def __init__(self, patterns: Sequence[Tuple[str, int, str]], nodes: Sequence[Tuple[int, int, int, int]], root: int):
        self._keep = []
        n = len(patterns)
        parr = (_Pattern * max(n, 1))()
        for i, (sel, op, val) in enumerate(patterns):
            sb, vb = _b(sel), _b(val)
            self._keep += [sb, vb]
            parr[i] = _Pattern(sb, len(sb), int(op), vb, len(vb))
        narr = (_Node * max(len(nodes), 1))()
        for i, nd in enumerate(nodes):
            narr[i] = _Node(*nd)
        self._keep += [parr, narr]
        self.n_patterns = n
        self._h = lib().or_ruleset_new(parr, n, narr, len(nodes), root)

    @classmethod
    def from_expression(cls, expr) -> "Ruleset":
        pats, nodes, root = expr.flatten()
        return cls([(p.selector, int(p.operator), p.value) for p in pats], nodes, root)

    def pattern(self, i: int, doc) -> int:
        d = _b(doc)
        return lib().or_pattern_matches(self._h, i, d, len(d))

    def matches(self, doc) -> Tuple[int, int]:
        d = _b(doc)
        ep = C.c_int32(-1)
        t = lib().or_expression_matches(self._h, d, len(d), C.byref(ep))
        return t, ep.value

    def error(self, i: int) -> str:
        return lib().or_pattern_error(self._h, i).decode("utf-8", "replace")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_ruleset_free(self._h)
            self._h = None


def eval_batch(sets: Sequence[Ruleset], arena: np.ndarray, offs: np.ndarray, lens: np.ndarray,
               set_of_req: Optional[np.ndarray] = None, nthreads: int = 1, with_bitmap: bool = True):
    """-> (tristate u8[n], err_idx i32[n], bitmap u64[n, words])"""
    n = int(lens.shape[0])
    words = max(1, max((s.n_patterns + 63) // 64 for s in sets))
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    tri = np.zeros(n, dtype=np.uint8)
    err = np.zeros(n, dtype=np.int32)
    bm = np.zeros((n, words), dtype=np.uint64) if with_bitmap else None
    sarr = (C.c_void_p * len(sets))(*[s._h for s in sets])
    sor = None
    if set_of_req is not None:
        set_of_req = np.ascontiguousarray(set_of_req, dtype=np.uint32)
        sor = set_of_req.ctypes.data
    lib().or_eval_batch(sarr, sor, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                        tri.ctypes.data, err.ctypes.data, bm.ctypes.data if bm is not None else None,
                        words, nthreads)
    return tri, err, bm
