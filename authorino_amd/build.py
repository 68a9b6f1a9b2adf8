"""Build libauthjx.so in-tree for gfx950 (hipcc). Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libauthjx.so")
SOURCES = ["ajx_regex.cpp", "ajx_compiler.cpp", "ajx_api.cpp", "ajx_index.cpp", "ajx_producer.cpp", "ajx_kernels.hip"]
HEADERS = ["ajx_blob.h", "ajx_device.h", "ajx_float.h", "ajx_modifiers.h", "ajx_batcher.h", "ajx_fast.h", "ajx_events.h", "ajx_lane.h", "ajx_regex.h", "ajx_compiler.h", "ajx_kernels.h"]
ARCH = os.environ.get("AUTHJX_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "authjx.h"))
    deps.append(__file__)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, "build", src + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
               "-Wno-unused-function", "-c", os.path.join(CSRC, src), "-o", obj]
        if not src.endswith(".hip"):
            cmd[1:1] = ["-x", "hip"] if False else []
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = OUT + ".tmp"
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
