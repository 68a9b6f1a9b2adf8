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


@pytest.fixture(scope="module")
def chain_bins():
    subprocess.run(["make", "-s", "-C", _NATIVE, "san_chain", "tsan_driver"], check=True, timeout=600)
    return os.path.join(_NATIVE, "san_chain"), os.path.join(_NATIVE, "tsan_driver")


@pytest.mark.parametrize("seed", [1, 2])
def test_producer_and_index_under_asan_ubsan(chain_bins, seed):
    """authjx_pack_json on random and malformed tapes (truncated, flipped bytes, huge
    counts, NaN / Inf), arenas that are too small; the index under random Set /
    DeleteKey / Get and batched lookups (which must equal Get)."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([chain_bins[0], "300", str(seed)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and r.stdout.startswith("ok "), (r.stdout[-2000:], r.stderr[-4000:])


def test_batcher_and_index_under_tsan(chain_bins):
    """The micro-batcher (two workers, 16 producers, deadlines) and the index's reader /
    writer lock (4 lookup threads against a reconcile writer, which must not starve)
    under ThreadSanitizer: no report, every caller gets its own result."""
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([chain_bins[1], "16", "300"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, (r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("ok ") and "wrong 0" in r.stdout


def test_workspace_lifetime_under_tsan():
    """The C-ABI's per-stream workspaces (ajx_api.cpp) on a host stand-in of the HIP runtime
    (tests/native/hipstub): evaluations on short-lived streams released while other threads
    read authjx_last_exact_count / authjx_last_kernel_ms, a stream released while a call is
    still on it, host-buffer batches with rulesets compiled and freed, a micro-batcher
    created and destroyed — under ThreadSanitizer, no report. (The same driver on the
    round-3 code, which freed a released workspace under a waiting reader, reported
    use-after-free races.)"""
    subprocess.run(["make", "-s", "-C", _NATIVE, "tsan_api"], check=True, timeout=600)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(_NATIVE, "tsan_api"), "150"], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, (r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("ok ") and "errors 0" in r.stdout
