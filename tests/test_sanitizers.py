"""ASan + UBSan over the host code: the reconcile-time compiler (ajx_compiler.cpp), the
Go-RE2 -> DFA builder (ajx_regex.cpp, it parses CRD text), the selector parser and the
host builds of the device logic (exact scan, single-pass scan, lane scanner, number
canon), driven by random selectors / regexes / mutated documents
(tests/native/san_fuzz.cpp). Any sanitizer report aborts the binary; it also checks the
single-pass and lane paths against the exact path where they decide."""
import os
import subprocess

import pytest

_NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def san_bin():
    subprocess.run(["make", "-s", "-C", _NATIVE, "san"], check=True, timeout=600)
    return os.path.join(_NATIVE, "san_fuzz")


@pytest.mark.parametrize("seed", [1, 2])
def test_host_code_under_asan_ubsan(san_bin, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([san_bin, "4000", str(seed)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "mismatches 0" in r.stdout
