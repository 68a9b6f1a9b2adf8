"""Build libauthjx.so in-tree for gfx950 (hipcc). Used by __graft_entry__.build().

Each object is rebuilt when its source or a header it includes (transitively) changed.
The library carries the hash of the sources it was built from (authjx_build_hash);
runtime.load_library compares it with source_hash() so that a stale binary never runs.
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libauthjx.so")
INCLUDE_H = os.path.join(HERE, "..", "include", "authjx.h")
SOURCES = ["ajx_regex.cpp", "ajx_compiler.cpp", "ajx_api.cpp", "ajx_index.cpp", "ajx_producer.cpp", "ajx_kernels.hip", "ajx_lean.hip"]
ARCH = os.environ.get("AUTHJX_ARCH", "gfx950")
_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path: str, seen=None) -> set:
    """path and every quoted include it reaches (resolved next to the including file)."""
    seen = set() if seen is None else seen
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        text = f.read()
    for inc in _INC.findall(text):
        _deps(os.path.join(os.path.dirname(path), inc), seen)
    return seen


def source_hash() -> str:
    """sha256 over every source and header of the library (sorted by name)."""
    files = set()
    for src in SOURCES:
        files |= _deps(os.path.join(CSRC, src))
    files.add(os.path.normpath(INCLUDE_H))
    h = hashlib.sha256()
    for p in sorted(files):
        h.update(os.path.relpath(p, HERE).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:32]


def _obj(src: str) -> str:
    return os.path.join(CSRC, "build", src + ".o")


def _stale_obj(src: str) -> bool:
    obj = _obj(src)
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = _deps(os.path.join(CSRC, src)) | {os.path.normpath(__file__)}
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    digest = source_hash()
    stale = [s for s in SOURCES if force or _stale_obj(s)]
    # the hash is compiled into ajx_api.cpp: rebuilt whenever any source changed
    if stale and "ajx_api.cpp" not in stale:
        stale.append("ajx_api.cpp")
    # every stale object compiled at once (the kernel translation units take minutes each)
    procs = []
    for src in stale:
        obj = _obj(src)
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
               f'-DAJX_SRC_HASH="{digest}"', "-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), obj, cmd))
    failed = [cmd for p, _, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    for _, obj, _ in procs:
        os.replace(obj + ".tmp", obj)
    if stale or not os.path.exists(OUT):
        tmp = OUT + ".tmp"
        subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + [_obj(s) for s in SOURCES],
                       check=True)
        os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
