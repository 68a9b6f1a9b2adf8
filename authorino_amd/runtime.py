"""authorino_amd.runtime — binding of libauthjx.so (include/authjx.h) for Python callers.

PyTorch is only plumbing here: it allocates HBM buffers and supplies the stream; all
evaluation happens in the HIP kernels behind the C-ABI. There is no CPU fallback: if
the library or a GPU is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libauthjx.so")
# profiling only: AUTHJX_LIB points the binding at an ablation build of the same C-ABI
LIB_PATH = os.environ.get("AUTHJX_LIB", LIB_PATH)

OP_UNKNOWN, OP_EQ, OP_NEQ, OP_INCL, OP_EXCL, OP_MATCHES = range(6)
F, T, E, UNDECIDED = 0, 1, 2, 3
PAT_OK, PAT_STATIC_ERROR, PAT_UNSUPPORTED = 0, 1, 2


class AuthjxError(RuntimeError):
    pass


class _Pattern(C.Structure):
    _fields_ = [("selector", C.c_char_p), ("selector_len", C.c_uint32), ("op", C.c_int32),
                ("value", C.c_char_p), ("value_len", C.c_uint32)]


class _Node(C.Structure):
    _fields_ = [("kind", C.c_int32), ("left", C.c_int32), ("right", C.c_int32), ("pattern", C.c_int32)]


class _Tree(C.Structure):
    _fields_ = [("patterns", C.POINTER(_Pattern)), ("n_patterns", C.c_uint32),
                ("nodes", C.POINTER(_Node)), ("n_nodes", C.c_uint32), ("root", C.c_int32)]


_lib = None
_lib_lock = threading.Lock()

EXPORTS = [
    "authjx_init", "authjx_shutdown", "authjx_device_count", "authjx_compile", "authjx_free",
    "authjx_ruleset_patterns", "authjx_ruleset_selectors", "authjx_pattern_error",
    "authjx_eval_batch_device", "authjx_eval_batch", "authjx_last_kernel_ms", "authjx_set_exact_scan",
    "authjx_last_exact_count", "authjx_select_batch_device", "authjx_select_batch", "authjx_compile_forest",
    "authjx_select_from_eval_device", "authjx_select_text_batch_device", "authjx_select_text_batch",
    "authjx_release_stream",
    "authjx_ruleset_trees", "authjx_batcher_create", "authjx_batcher_destroy", "authjx_batcher_eval",
    "authjx_batcher_stats",
    "authjx_index_new", "authjx_index_free", "authjx_index_set", "authjx_index_delete_key", "authjx_index_get",
    "authjx_index_lookup_batch", "authjx_pack_json", "authjx_build_hash",
]


def _check_build_hash(L, path: str) -> None:
    """The binary must have been built from the sources next to it (when they are here)."""
    from . import build as _b

    if not os.path.isdir(_b.CSRC):
        return
    want = _b.source_hash()
    got = (L.authjx_build_hash() or b"").decode()
    if got != want:
        raise AuthjxError(f"{path} was built from other sources (hash {got}, sources {want}): "
                          "run __graft_entry__.build()")


def load_library(path: str = LIB_PATH):
    """Load libauthjx.so and declare its signatures (does not touch the GPU)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise AuthjxError(f"libauthjx.so not built at {path}: run __graft_entry__.build()")
        # One HIP runtime per process: torch ships its own libamdhip64.so.7. Loading torch
        # first makes libauthjx.so bind to that copy (same soname), so HBM buffers and
        # streams handed over from torch belong to the runtime that launches our kernels.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(path)
        L.authjx_build_hash.argtypes = []
        L.authjx_build_hash.restype = C.c_char_p
        # (a profiling build named by AUTHJX_LIB is a whole library of its own, possibly of
        # an earlier tree for an A/B run: only the in-tree library must match the sources)
        if not os.environ.get("AUTHJX_LIB"):
            _check_build_hash(L, path)
        L.authjx_init.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.authjx_init.restype = C.c_int
        L.authjx_shutdown.argtypes = [C.c_void_p]
        L.authjx_shutdown.restype = None
        L.authjx_device_count.argtypes = []
        L.authjx_device_count.restype = C.c_int
        L.authjx_compile.argtypes = [C.c_void_p, C.POINTER(_Tree), C.POINTER(C.c_void_p), C.POINTER(C.c_int32),
                                     C.c_char_p, C.c_size_t]
        L.authjx_compile.restype = C.c_int
        L.authjx_compile_forest.argtypes = [C.c_void_p, C.POINTER(_Tree), C.c_uint32, C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_int32), C.c_char_p, C.c_size_t]
        L.authjx_compile_forest.restype = C.c_int
        L.authjx_ruleset_trees.argtypes = [C.c_void_p]
        L.authjx_ruleset_trees.restype = C.c_uint32
        L.authjx_free.argtypes = [C.c_void_p]
        L.authjx_free.restype = None
        L.authjx_ruleset_patterns.argtypes = [C.c_void_p]
        L.authjx_ruleset_patterns.restype = C.c_uint32
        L.authjx_ruleset_selectors.argtypes = [C.c_void_p]
        L.authjx_ruleset_selectors.restype = C.c_uint32
        L.authjx_pattern_error.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]
        L.authjx_pattern_error.restype = C.c_size_t
        L.authjx_eval_batch_device.argtypes = [
            C.c_void_p, C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
            C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
        L.authjx_eval_batch_device.restype = C.c_int
        L.authjx_eval_batch.argtypes = [
            C.c_void_p, C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
            C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
        L.authjx_eval_batch.restype = C.c_int
        L.authjx_select_batch_device.argtypes = [
            C.c_void_p, C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
            C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
        L.authjx_select_batch_device.restype = C.c_int
        L.authjx_select_from_eval_device.argtypes = [
            C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
            C.c_uint32, C.c_void_p]
        L.authjx_select_from_eval_device.restype = C.c_int
        L.authjx_select_batch.argtypes = [
            C.c_void_p, C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
            C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
        L.authjx_select_batch.restype = C.c_int
        L.authjx_select_text_batch_device.argtypes = [
            C.c_void_p, C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
            C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
        L.authjx_select_text_batch_device.restype = C.c_int
        L.authjx_select_text_batch.argtypes = [
            C.c_void_p, C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
            C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
        L.authjx_select_text_batch.restype = C.c_int
        L.authjx_last_kernel_ms.argtypes = [C.c_void_p]
        L.authjx_last_kernel_ms.restype = C.c_float
        L.authjx_set_exact_scan.argtypes = [C.c_void_p, C.c_int]
        L.authjx_set_exact_scan.restype = C.c_int
        L.authjx_last_exact_count.argtypes = [C.c_void_p]
        L.authjx_last_exact_count.restype = C.c_int64
        L.authjx_batcher_create.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p)]
        L.authjx_batcher_create.restype = C.c_int
        L.authjx_batcher_destroy.argtypes = [C.c_void_p]
        L.authjx_batcher_destroy.restype = None
        L.authjx_batcher_eval.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t, C.c_uint64,
                                          C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]
        L.authjx_batcher_eval.restype = C.c_int
        L.authjx_batcher_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint64)] * 4
        L.authjx_batcher_stats.restype = C.c_int
        L.authjx_index_new.argtypes = [C.POINTER(C.c_void_p)]
        L.authjx_index_new.restype = C.c_int
        L.authjx_index_free.argtypes = [C.c_void_p]
        L.authjx_index_free.restype = None
        L.authjx_index_set.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int32, C.c_int]
        L.authjx_index_set.restype = C.c_int
        L.authjx_index_delete_key.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.c_int32]
        L.authjx_index_delete_key.restype = C.c_int
        L.authjx_index_get.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.POINTER(C.c_int32)]
        L.authjx_index_get.restype = C.c_int
        L.authjx_index_lookup_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                                C.c_void_p, C.c_uint32]
        L.authjx_index_lookup_batch.restype = C.c_int
        L.authjx_pack_json.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64,
                                       C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]
        L.authjx_pack_json.restype = C.c_int
        L.authjx_debug_last_error.argtypes = []
        L.authjx_debug_last_error.restype = C.c_char_p
        _lib = L
        return L


def _check(rc: int, what: str):
    if rc != 0:
        names = {-1: "EINVAL", -2: "ENOMEM", -3: "EDEVICE", -4: "ELIMIT", -5: "ETIMEDOUT", -6: "ECLOSED"}
        detail = ""
        if rc == -3 and _lib is not None:  # (the HIP error behind it, on this thread)
            detail = " (%s)" % _lib.authjx_debug_last_error().decode()
        raise AuthjxError(f"{what} failed: {names.get(rc, rc)}{detail}")


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else s.encode("utf-8")


class Context:
    """One device context (HIP stream + set table) per GPU."""

    def __init__(self, device: int = 0):
        L = load_library()
        if L.authjx_device_count() <= device:
            raise AuthjxError(f"no HIP device {device} (authjx_device_count={L.authjx_device_count()})")
        h = C.c_void_p()
        _check(L.authjx_init(device, C.byref(h)), "authjx_init")
        self._h = h
        self.device = device
        self._batchers = weakref.WeakSet()  # (authjx_shutdown destroys those still alive)

    def compile(self, patterns: Sequence[Tuple[str, int, str]], nodes: Sequence[Tuple[int, int, int, int]],
                root: int) -> "Ruleset":
        return Ruleset(self, patterns, nodes, root)

    def compile_expression(self, expr) -> "Ruleset":
        pats, nodes, root = expr.flatten()
        return Ruleset(self, [(p.selector, int(p.operator), p.value) for p in pats], nodes, root)

    def compile_forest(self, exprs, extra_selectors=None) -> "Ruleset":
        """Several expressions (None = nil) as one ruleset (authjx_compile_forest): one
        scan per document, one result per expression. extra_selectors: gjson paths added
        as a last, root-less tree of EQ "" patterns (its result is T), so that the same
        scan captures them for select_from_eval_device at pattern index
        n_patterns - len(extra_selectors)."""
        trees = []
        for e in exprs:
            if e is None:
                trees.append(([], [], -1))
            else:
                pats, nodes, root = e.flatten()
                trees.append(([(p.selector, int(p.operator), p.value) for p in pats], nodes, root))
        if extra_selectors:
            trees.append(([(p, 1, "") for p in extra_selectors], [], -1))
        return Ruleset(self, None, None, None, forest=trees)

    def eval_device(self, sets: Sequence["Ruleset"], arena, offs, lens, out_tri, out_err=None, out_bm=None,
                    set_of_req=None, stream=None) -> None:
        """Evaluate a batch resident in HBM (torch tensors on this device). Asynchronous."""
        n = int(lens.numel())
        words = int(out_bm.shape[1]) if out_bm is not None else 0
        sarr = (C.c_void_p * len(sets))(*[s._h.value for s in sets])
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        rc = load_library().authjx_eval_batch_device(
            self._h, sarr, len(sets), ptr(set_of_req), ptr(arena), ptr(offs), ptr(lens), n,
            ptr(out_tri), ptr(out_err), ptr(out_bm), words, C.c_void_p(stream) if stream else None)
        _check(rc, "authjx_eval_batch_device")

    def set_exact_scan(self, force: bool) -> None:
        """Route every request through the exact scan kernel (for cross-checks)."""
        _check(load_library().authjx_set_exact_scan(self._h, 1 if force else 0), "authjx_set_exact_scan")

    def set_kernel_mode(self, mode: int) -> None:
        """Select the kernel: 0 the default (the streaming kernel for small batches, the lean
        or multi-tenant kernel otherwise), 41 the lean kernel for every batch, 52 the
        streaming kernel for every one-ruleset batch; 50 / 51 and others are profiling
        ablations whose outputs are meaningless. Not part of authjx.h."""
        L = load_library()
        L.authjx_debug_ablate.argtypes = [C.c_void_p, C.c_int]
        _check(L.authjx_debug_ablate(self._h, int(mode)), "authjx_debug_ablate")

    def set_stream_max(self, n: int) -> None:
        """Batches of up to n requests take the streaming kernel (default 4096; 0 never).
        Profiling; not part of authjx.h."""
        L = load_library()
        L.authjx_debug_stream_max.argtypes = [C.c_void_p, C.c_uint32]
        _check(L.authjx_debug_stream_max(self._h, int(n)), "authjx_debug_stream_max")

    def last_exact_count(self) -> int:
        """Requests of the last batch the single-pass kernel handed to the exact scan."""
        return int(load_library().authjx_last_exact_count(self._h))

    def last_kernel_ms(self) -> float:
        return float(load_library().authjx_last_kernel_ms(self._h))

    def eval_host(self, sets: Sequence["Ruleset"], docs: Sequence[bytes], set_of_req=None, with_bitmap=True):
        """Evaluate host documents (copies to HBM and back); returns (tri, err, bitmap)."""
        docs = [_b(d) for d in docs]
        n = len(docs)
        lens = np.fromiter((len(d) for d in docs), dtype=np.uint32, count=n)
        offs = np.zeros(n, dtype=np.uint64)
        if n:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(docs) or b"\0", dtype=np.uint8)
        return self.eval_host_arena(sets, arena, offs, lens, set_of_req, with_bitmap)

    def eval_host_arena(self, sets, arena, offs, lens, set_of_req=None, with_bitmap=True, bitmap_words=0):
        n = int(lens.shape[0])
        words = max(1, bitmap_words, max((s.n_patterns + 63) // 64 for s in sets))
        nt = sets[0].n_trees
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        tri = np.zeros(max(n, 1) * nt, dtype=np.uint8)
        err = np.zeros(max(n, 1) * nt, dtype=np.int32)
        bm = np.zeros((max(n, 1), words), dtype=np.uint64) if with_bitmap else None
        sor = None
        if set_of_req is not None:
            set_of_req = np.ascontiguousarray(set_of_req, dtype=np.uint32)
            sor = C.c_void_p(set_of_req.ctypes.data)
        sarr = (C.c_void_p * len(sets))(*[s._h.value for s in sets])
        rc = load_library().authjx_eval_batch(
            self._h, sarr, len(sets), sor, C.c_void_p(arena.ctypes.data), int(arena.nbytes),
            C.c_void_p(offs.ctypes.data), C.c_void_p(lens.ctypes.data), n, C.c_void_p(tri.ctypes.data),
            C.c_void_p(err.ctypes.data), C.c_void_p(bm.ctypes.data) if bm is not None else None,
            words if bm is not None else 0)
        _check(rc, "authjx_eval_batch")
        if nt > 1:
            return tri.reshape(-1, nt)[:n], err.reshape(-1, nt)[:n], (bm[:n] if bm is not None else None)
        return tri[:n], err[:n], (bm[:n] if bm is not None else None)

    def select_device(self, sets, arena, offs, lens, out, set_of_req=None, stream=None) -> None:
        """authjx_select_batch_device on HBM-resident torch tensors; out: u32[n][stride][3].
        Asynchronous."""
        n = int(lens.numel())
        sarr = (C.c_void_p * len(sets))(*[s._h.value for s in sets])
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        rc = load_library().authjx_select_batch_device(
            self._h, sarr, len(sets), ptr(set_of_req), ptr(arena), ptr(offs), ptr(lens), n, ptr(out),
            int(out.shape[1]), C.c_void_p(stream) if stream else None)
        _check(rc, "authjx_select_batch_device")

    def select_from_eval_device(self, rs, first_pattern: int, arena, offs, lens, out, stream=None) -> None:
        """authjx_select_from_eval_device: the values of patterns [first_pattern,
        first_pattern + out.shape[1]) of `rs` from the capture rows of the last
        eval_device(rs, ...) over the same tensors (no second document scan). Asynchronous."""
        n = int(lens.numel())
        ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        rc = load_library().authjx_select_from_eval_device(
            self._h, rs._h, int(first_pattern), ptr(arena), ptr(offs), ptr(lens), n, ptr(out), int(out.shape[1]),
            C.c_void_p(stream) if stream else None)
        _check(rc, "authjx_select_from_eval_device")

    def select_text_device(self, sets, arena, offs, lens, out, text, set_of_req=None, stream=None) -> None:
        """authjx_select_text_batch_device: select_device plus modifier chains and "#." lists,
        whose values are built text in text[r] (u8[n][text_stride]). Asynchronous."""
        n = int(lens.numel())
        sarr = (C.c_void_p * len(sets))(*[s._h.value for s in sets])
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        rc = load_library().authjx_select_text_batch_device(
            self._h, sarr, len(sets), ptr(set_of_req), ptr(arena), ptr(offs), ptr(lens), n, ptr(out),
            int(out.shape[1]), ptr(text), int(text.shape[1]), C.c_void_p(stream) if stream else None)
        _check(rc, "authjx_select_text_batch_device")

    def select_text_host_arena(self, sets, arena, offs, lens, set_of_req=None, text_stride: int = 4096):
        """authjx_select_text_batch: (u32[n][stride][3] values, u8[n][text_stride] text
        slots); a value whose esc has VALUE_TEXT is [start, start + len) of its request's
        slot (a modifier chain's / "#." list's Result), else a span of the document."""
        n = int(lens.shape[0])
        stride = max(1, max(s.n_patterns for s in sets))
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        if arena.nbytes == 0:
            arena = np.zeros(1, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros((max(n, 1), stride, 3), dtype=np.uint32)
        text = np.zeros((max(n, 1), text_stride), dtype=np.uint8)
        sor = None
        if set_of_req is not None:
            set_of_req = np.ascontiguousarray(set_of_req, dtype=np.uint32)
            sor = C.c_void_p(set_of_req.ctypes.data)
        sarr = (C.c_void_p * len(sets))(*[s._h.value for s in sets])
        rc = load_library().authjx_select_text_batch(
            self._h, sarr, len(sets), sor, C.c_void_p(arena.ctypes.data), int(arena.nbytes),
            C.c_void_p(offs.ctypes.data), C.c_void_p(lens.ctypes.data), n, C.c_void_p(out.ctypes.data), stride,
            C.c_void_p(text.ctypes.data), text_stride)
        _check(rc, "authjx_select_text_batch")
        return out[:n], text[:n]

    def select_host_arena(self, sets, arena, offs, lens, set_of_req=None) -> np.ndarray:
        """gjson.Get of every pattern selector of each request's ruleset on the device
        (authjx_select_batch): u32[n][stride][3] = {start, len, type | esc << 8}."""
        n = int(lens.shape[0])
        stride = max(1, max(s.n_patterns for s in sets))
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        if arena.nbytes == 0:
            arena = np.zeros(1, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros((max(n, 1), stride, 3), dtype=np.uint32)
        sor = None
        if set_of_req is not None:
            set_of_req = np.ascontiguousarray(set_of_req, dtype=np.uint32)
            sor = C.c_void_p(set_of_req.ctypes.data)
        sarr = (C.c_void_p * len(sets))(*[s._h.value for s in sets])
        rc = load_library().authjx_select_batch(
            self._h, sarr, len(sets), sor, C.c_void_p(arena.ctypes.data), int(arena.nbytes),
            C.c_void_p(offs.ctypes.data), C.c_void_p(lens.ctypes.data), n, C.c_void_p(out.ctypes.data), stride)
        _check(rc, "authjx_select_batch")
        return out[:n]

    def release_stream(self, stream) -> None:
        """authjx_release_stream: free the workspace kept for a (short-lived) stream."""
        L = load_library()
        L.authjx_release_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.authjx_release_stream.restype = C.c_int
        _check(L.authjx_release_stream(self._h, C.c_void_p(stream)), "authjx_release_stream")

    def close(self):
        if getattr(self, "_h", None):
            for b in list(getattr(self, "_batchers", ())):
                b._h = None  # (destroyed by authjx_shutdown below)
            load_library().authjx_shutdown(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Ruleset:
    """A compiled jsonexp tree resident in HBM (authjx_compile / authjx_free)."""

    def __init__(self, ctx: Context, patterns, nodes, root, forest=None):
        L = load_library()
        self.ctx = ctx
        keep = []

        def tree_of(patterns, nodes, root):
            parr = (_Pattern * max(len(patterns), 1))()
            for i, (sel, op, val) in enumerate(patterns):
                sb, vb = _b(sel), _b(val)
                keep.extend([sb, vb])
                parr[i] = _Pattern(sb, len(sb), int(op), vb, len(vb))
            narr = (_Node * max(len(nodes), 1))()
            for i, nd in enumerate(nodes):
                narr[i] = _Node(*nd)
            keep.extend([parr, narr])
            return _Tree(parr, len(patterns), narr, len(nodes), root)

        trees = forest if forest is not None else [(patterns, nodes, root)]
        self.offsets = list(np.cumsum([0] + [len(t[0]) for t in trees])[:-1])  # first pattern of each tree
        self.n_patterns = sum(len(t[0]) for t in trees)
        st = (C.c_int32 * max(self.n_patterns, 1))()
        err = C.create_string_buffer(512)
        h = C.c_void_p()
        if forest is None:
            tree = tree_of(patterns, nodes, root)
            rc = L.authjx_compile(ctx._h, C.byref(tree), C.byref(h), st, err, 512)
        else:
            tarr = (_Tree * len(trees))(*[tree_of(*t) for t in trees])
            rc = L.authjx_compile_forest(ctx._h, tarr, len(trees), C.byref(h), st, err, 512)
        if rc != 0:
            raise AuthjxError(f"authjx_compile failed ({rc}): {err.value.decode(errors='replace')}")
        self._h = h
        self.status = list(st)[: self.n_patterns]
        self.n_selectors = int(L.authjx_ruleset_selectors(h))
        self.n_trees = int(L.authjx_ruleset_trees(h))

    def pattern_error(self, i: int) -> str:
        buf = C.create_string_buffer(1024)
        load_library().authjx_pattern_error(self._h, i, buf, 1024)
        return buf.value.decode("utf-8", "replace")

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                load_library().authjx_free(self._h)
            except Exception:
                pass
            self._h = None


# -------------------------------------------------------------------------------------
# jsonexp.Expression adapter
# -------------------------------------------------------------------------------------
_ctx_lock = threading.Lock()
_default_ctx: Dict[int, Context] = {}


def context(device: int = 0) -> Context:
    with _ctx_lock:
        if device not in _default_ctx:
            _default_ctx[device] = Context(device)
        return _default_ctx[device]


class MatchError(Exception):
    """The (false, err) result of Pattern.Matches: carries the Go error text."""


class CompiledExpression:
    def __init__(self, expr, device: int = 0):
        self.ctx = context(device)
        self.ruleset = self.ctx.compile_expression(expr)

    def _to_result(self, t: int, ep: int):
        if t == T:
            return True, None
        if t == F:
            return False, None
        if t == E:
            return False, MatchError(self.ruleset.pattern_error(ep))
        raise AuthjxError("device could not decide this document (AUTHJX_UNDECIDED)")

    def matches(self, json):
        tri, err, _ = self.ctx.eval_host([self.ruleset], [_b(json)], with_bitmap=False)
        return self._to_result(int(tri[0]), int(err[0]))

    def matches_batch(self, docs):
        tri, err, _ = self.ctx.eval_host([self.ruleset], [_b(d) for d in docs], with_bitmap=False)
        return [self._to_result(int(t), int(e)) for t, e in zip(tri, err)]


def expression_for(expr) -> CompiledExpression:
    c = getattr(expr, "_compiled", None)
    if c is None:
        c = CompiledExpression(expr)
        expr._compiled = c
    return c


class BatchTimeout(AuthjxError):
    """The request's deadline passed before its batch was evaluated (AUTHJX_ETIMEDOUT)."""


_batcher_knob_lock = threading.Lock()


class Batcher:
    """The micro-batcher (authjx_batcher_*): many threads call eval() with one request
    each; the native worker forms batches (size / window flush, deadlines, AuthConfig
    buckets) and evaluates each with one launch on its own stream. ctypes releases the
    GIL around the blocking call, so Python threads wait concurrently."""

    def __init__(self, ctx: "Context", max_batch: int = 4096, window_us: int = 200, queue_cap: int = 0,
                 workers: int = 0, modes=None):
        """workers: worker threads, each with its own stream (0: the library's default, 2;
        profiling knob, authjx_debug_batcher_workers, not part of authjx.h). modes: None, or
        (wake, sync, zero-copy) for authjx_debug_batcher_modes (profiling; the library's
        default modes, (0, 0, 1), are restored afterwards)."""
        L = load_library()
        h = C.c_void_p()
        # (the worker count and modes are process-wide knobs of the library that batcher
        # creation reads: set, create and restore under one lock, so that batchers created
        # at the same time in other threads keep what they asked for)
        with _batcher_knob_lock:
            prev = 0
            if workers:
                L.authjx_debug_batcher_workers.argtypes = [C.c_uint32]
                prev = L.authjx_debug_batcher_workers(0)  # (0: the current count, restored below)
                _check(L.authjx_debug_batcher_workers(int(workers)), "authjx_debug_batcher_workers")
            if modes is not None:
                L.authjx_debug_batcher_modes.argtypes = [C.c_uint32] * 3
                _check(L.authjx_debug_batcher_modes(*[int(m) for m in modes]), "authjx_debug_batcher_modes")
            try:
                _check(L.authjx_batcher_create(ctx._h, max_batch, window_us, queue_cap, C.byref(h)),
                       "authjx_batcher_create")
            finally:
                if workers and prev > 0:
                    L.authjx_debug_batcher_workers(prev)
                if modes is not None:
                    L.authjx_debug_batcher_modes(0, 0, 1)
        self.ctx = ctx
        self._h = h
        ctx._batchers.add(self)

    def eval(self, ruleset: "Ruleset", doc, timeout_s: float = 0.0):
        """(tri-states, error indices) of `ruleset`'s trees on one document."""
        d = _b(doc)
        nt = max(1, len(ruleset.offsets))
        tri = (C.c_uint8 * nt)()
        err = (C.c_int32 * nt)()
        rc = load_library().authjx_batcher_eval(self._h, ruleset._h, d, len(d), int(timeout_s * 1e6), tri, err)
        if rc == -5:
            raise BatchTimeout("authjx_batcher_eval: deadline passed")
        _check(rc, "authjx_batcher_eval")
        return list(tri), list(err)

    def loadgen(self, rulesets, set_of_req, arena, offs, lens, threads: int = 64):
        """Profiling: `threads` native producer threads push every request through this
        batcher one blocking call at a time (authjx_debug_loadgen). Returns (per-request
        latency ns, first result per request, wall ns)."""
        L = load_library()
        L.authjx_debug_loadgen.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        n = len(lens)
        sets = (C.c_void_p * len(rulesets))(*[r._h.value if isinstance(r._h, C.c_void_p) else r._h for r in rulesets])
        sor = np.ascontiguousarray(set_of_req, dtype=np.uint32)
        ar = np.ascontiguousarray(arena, dtype=np.uint8)
        of = np.ascontiguousarray(offs, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        lat = np.zeros(n, dtype=np.uint64)
        tri = np.zeros(n, dtype=np.uint8)
        wall = C.c_uint64()
        _check(L.authjx_debug_loadgen(self._h, sets, sor.ctypes.data, ar.ctypes.data, of.ctypes.data, ln.ctypes.data,
                                      n, threads, lat.ctypes.data, tri.ctypes.data, C.byref(wall)),
               "authjx_debug_loadgen")
        return lat, tri, wall.value

    def stats(self) -> Dict[str, int]:
        v = [C.c_uint64() for _ in range(4)]
        _check(load_library().authjx_batcher_stats(self._h, *[C.byref(x) for x in v]), "authjx_batcher_stats")
        return dict(zip(("batches", "requests", "expired", "max_batch_seen"), (x.value for x in v)))

    def profile(self) -> Dict[str, float]:
        """Profiling: mean µs per request (queue wait, caller resume) and per batch
        (evaluation, waking callers, packing, launch calls, device wait)."""
        L = load_library()
        L.authjx_debug_batcher_profile.argtypes = [C.c_void_p, C.c_void_p]
        v = np.zeros(9, dtype=np.uint64)
        _check(L.authjx_debug_batcher_profile(self._h, v.ctypes.data), "authjx_debug_batcher_profile")
        nb, nr = max(int(v[0]), 1), max(int(v[1]), 1)
        per_r = {"wait_us": v[2], "resume_us": v[5]}
        per_b = {"eval_us": v[3], "wake_us": v[4], "pack_us": v[6], "launch_us": v[7], "sync_us": v[8]}
        out = {"batches": int(v[0]), "requests": int(v[1])}
        out.update({k: round(int(x) / nr / 1e3, 2) for k, x in per_r.items()})
        out.update({k: round(int(x) / nb / 1e3, 2) for k, x in per_b.items()})
        return out

    def close(self):
        if getattr(self, "_h", None):
            load_library().authjx_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

