"""The Authorization JSON producer, batched.

pkg/service/auth_pipeline.go:542-616 (GetAuthorizationJSON / NewAuthorizationJSON) builds
each request's Authorization JSON with encoding/json — once per evaluator call, at least
twice per authorization evaluator. Here a micro-batch is produced once: each request's
values are walked into a tape (include/authjx.h AUTHJX_TAPE_*) and libauthjx.so's
authjx_pack_json encodes all of them with encoding/json's rules straight into the batch
arena (arena, offs, lens) that the device evaluation reads, on all host threads.

Values: dict = a Go struct (members in insertion order, omitempty applied by the
caller), GoMap (or `go_map(d)`) = a Go map (keys sorted by bytes by the packer), str,
float (float64), int (integer types), bool, None, list / tuple (slices), RawJSON (a
json.RawMessage, copied as is). `authorization_json` assembles the reference's document
shape: {"context", "request", "source", "destination", "auth": {...}} with the
well-known attribute structs (pkg/service/well_known_attributes.go:29-200).
"""
from __future__ import annotations

import ctypes as C
import struct
from typing import Iterable, List, Optional, Sequence

import numpy as np

TAPE_NULL, TAPE_TRUE, TAPE_FALSE, TAPE_F64, TAPE_I64, TAPE_STRING, TAPE_RAW, TAPE_ARRAY, TAPE_OBJECT, TAPE_MAP = \
    range(1, 11)


class GoMap(dict):
    """A Go map value: encoding/json writes its members sorted by key bytes."""


class RawJSON(bytes):
    """A json.RawMessage: pre-encoded JSON copied into the document as is."""


def go_map(d: dict) -> GoMap:
    return GoMap(d)


def tape(value) -> bytes:
    """One value as an AUTHJX_TAPE_* stream."""
    out = bytearray()
    _put(value, out)
    return bytes(out)


def _put_str(s: bytes, out: bytearray, tag: int):
    out.append(tag)
    out += struct.pack("<I", len(s))
    out += s


def _put(v, out: bytearray):
    if v is None:
        out.append(TAPE_NULL)
    elif v is True:
        out.append(TAPE_TRUE)
    elif v is False:
        out.append(TAPE_FALSE)
    elif isinstance(v, RawJSON):
        _put_str(bytes(v), out, TAPE_RAW)
    elif isinstance(v, str):
        _put_str(v.encode("utf-8", "surrogatepass"), out, TAPE_STRING)
    elif isinstance(v, bytes):
        _put_str(v, out, TAPE_STRING)  # (a Go string holding these bytes, valid UTF-8 or not)
    elif isinstance(v, float):
        out.append(TAPE_F64)
        out += struct.pack("<d", v)
    elif isinstance(v, int):
        out.append(TAPE_I64)
        out += struct.pack("<q", v)
    elif isinstance(v, dict):
        out.append(TAPE_MAP if isinstance(v, GoMap) else TAPE_OBJECT)
        out += struct.pack("<I", len(v))
        for k, x in v.items():
            kb = k.encode("utf-8", "surrogatepass")
            out += struct.pack("<I", len(kb))
            out += kb
            _put(x, out)
    elif isinstance(v, (list, tuple)):
        out.append(TAPE_ARRAY)
        out += struct.pack("<I", len(v))
        for x in v:
            _put(x, out)
    else:
        raise TypeError(f"no JSON encoding for {type(v).__name__}")


class PackError(ValueError):
    """authjx_pack_json refused a request (a malformed tape, a NaN / Inf float64)."""


def pack(values: Sequence, n_threads: int = 0, tapes: Optional[List[bytes]] = None):
    """Encode every request's value into one arena: (arena u8, offs u64, lens u32).
    `tapes` may be given ready (the walk a Go shim does from its own structs)."""
    from . import runtime

    L = runtime.load_library()
    if tapes is None:
        tapes = [tape(v) for v in values]
    n = len(tapes)
    tl = np.fromiter((len(t) for t in tapes), dtype=np.uint32, count=n)
    to = np.zeros(n, dtype=np.uint64)
    if n > 1:
        to[1:] = np.cumsum(tl[:-1], dtype=np.uint64)
    tbuf = np.frombuffer(b"".join(tapes) or b"\0", dtype=np.uint8)
    offs = np.zeros(max(n, 1), dtype=np.uint64)
    lens = np.zeros(max(n, 1), dtype=np.uint32)
    total = C.c_uint64(0)
    # sized from the tapes (every encoded byte comes from at most 6 tape bytes, + 8 per
    # value for the JSON punctuation); grown once when that is short
    cap = int(tl.sum()) * 6 + 64
    for _ in range(2):
        arena = np.empty(max(cap, 1), dtype=np.uint8)
        rc = L.authjx_pack_json(tbuf.ctypes.data, to.ctypes.data, tl.ctypes.data, n, arena.ctypes.data, cap,
                                offs.ctypes.data, lens.ctypes.data, C.byref(total), int(n_threads))
        if rc == -4 and total.value > cap:  # AUTHJX_ELIMIT
            cap = int(total.value)
            continue
        if rc != 0:
            bad = [int(i) for i in np.nonzero(offs[:n] == np.uint64(0xFFFFFFFFFFFFFFFF))[0][:5]]
            raise PackError(f"authjx_pack_json: {rc} (requests {bad})")
        return arena[: int(total.value)], offs[:n], lens[:n]
    raise PackError("authjx_pack_json: arena sizing")


def authorization_json(context: dict, request: Optional[dict] = None, source: Optional[dict] = None,
                       destination: Optional[dict] = None, identity=None, metadata: Optional[dict] = None,
                       authorization: Optional[dict] = None, response: Optional[dict] = None,
                       callbacks: Optional[dict] = None, top_metadata: Optional[dict] = None) -> dict:
    """The value GetAuthorizationJSON marshals (auth_pipeline.go:542-579, 610-616):
    context (the envoy AttributeContext), the well-known attributes (request, source,
    destination; metadata when set) and auth {identity, metadata, authorization,
    response, callbacks} with empty maps omitted."""
    doc = {"context": context}
    if top_metadata:
        doc["metadata"] = top_metadata
    doc["request"] = request if request is not None else {}
    doc["source"] = source if source is not None else {}
    doc["destination"] = destination if destination is not None else {}
    auth = {}
    if identity is not None:
        auth["identity"] = identity
    for name, m in (("metadata", metadata), ("authorization", authorization), ("response", response),
                    ("callbacks", callbacks)):
        if m:
            auth[name] = GoMap(m)
    doc["auth"] = auth
    return doc
