"""CPU tests: libauthjx.so loads and exports every entry point include/authjx.h declares;
the product path refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "authjx.h")).read()
    return sorted(set(re.findall(r"\b(authjx_[a-z_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared_functions()
    for required in ["authjx_init", "authjx_compile", "authjx_free", "authjx_eval_batch",
                     "authjx_eval_batch_device", "authjx_shutdown"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    from authorino_amd import build, runtime

    path = build.build()
    lib = ctypes.CDLL(path)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(runtime.EXPORTS) == set(declared_functions())


def test_jsonexp_flatten_shapes():
    from authorino_amd.jsonexp import All, And, Any, Or, Pattern

    p = Pattern("a", "eq", "1")
    pats, nodes, root = All(p, Any(p)).flatten()
    assert len(pats) == 2 and nodes[root][0] == 1
    pats, nodes, root = And().flatten()
    assert pats == [] and nodes == [(1, -1, -1, -1)] and root == 0
    pats, nodes, root = Or(None, p).flatten()
    assert nodes[root] == (2, -1, 1, -1)
