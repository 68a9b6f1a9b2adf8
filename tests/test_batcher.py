"""The micro-batcher's queue logic (authorino_amd/csrc/ajx_batcher.h) on the CPU, with a
stand-in evaluator (tests/native/batcher_host.cpp): concurrent producers each get their
own result, batches form by size and by window, batches are ordered by ruleset and never
mix result shapes, deadlines expire unevaluated requests (also while waiting for queue
room). Every test runs under each wake mode (one condition variable per caller; one
broadcast per batch; one futex word per caller; callers waking each other in a tree). The device-backed batcher is tested in test_gpu_parity.py."""
import ctypes as C
import os
import subprocess
import threading
import time

import numpy as np
import pytest

_NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
ETIMEDOUT = -5


@pytest.fixture(scope="module", params=[0, 1, 2, 3], ids=["wake-cv", "wake-broadcast", "wake-futex", "wake-tree"])
def lib(request):
    subprocess.run(["make", "-s", "-C", _NATIVE, "libajx_batchtest.so"], check=True)
    L = C.CDLL(os.path.join(_NATIVE, "libajx_batchtest.so"))
    L.hb_set_wake.argtypes = [C.c_uint32]
    L.hb_set_wake(request.param)
    L.wake_mode = request.param
    L.hb_create.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    L.hb_create.restype = C.c_void_p
    L.hb_eval.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint8, C.c_uint64, C.POINTER(C.c_uint8)]
    L.hb_eval.restype = C.c_int
    L.hb_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.hb_destroy.argtypes = [C.c_void_p]
    return L


def _stats(L, h):
    out = (C.c_uint64 * 6)()
    L.hb_stats(h, out)
    return dict(zip(("batches", "requests", "expired", "max_batch", "order_violations", "shape_violations"), out))


def _expect(rs, byte, k=0):
    return (byte ^ (rs & 0xFF) ^ k) & 0xFF


def test_concurrent_producers_get_their_own_results(lib):
    h = lib.hb_create(256, 500, 0, 200)
    errors = []

    def producer(seed):
        rng = np.random.default_rng(seed)
        out = (C.c_uint8 * 2)()
        for _ in range(1500):
            rs = int(rng.integers(1, 6))
            nt = 1 if rs != 5 else 2  # ruleset 5 has two trees (another result shape)
            b = int(rng.integers(0, 256))
            rc = lib.hb_eval(h, rs, nt, b, 0, out)
            if rc != 0 or any(out[k] != _expect(rs, b, k) for k in range(nt)):
                errors.append((rc, rs, b, list(out)))

    ts = [threading.Thread(target=producer, args=(s,)) for s in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    st = _stats(lib, h)
    lib.hb_destroy(h)
    assert not errors, errors[:5]
    assert st["requests"] == 8 * 1500
    assert st["batches"] < st["requests"] / 2 and st["max_batch"] > 2  # requests were batched
    assert st["order_violations"] == 0 and st["shape_violations"] == 0


def test_window_flushes_a_partial_batch(lib):
    h = lib.hb_create(10000, 2000, 0, 0)
    out = (C.c_uint8 * 1)()
    t0 = time.perf_counter()
    assert lib.hb_eval(h, 3, 1, 7, 0, out) == 0
    dt = time.perf_counter() - t0
    lib.hb_destroy(h)
    assert out[0] == _expect(3, 7)
    assert dt < 0.5  # one request, batch never fills: flushed by the 2 ms window


def test_deadlines_expire_unevaluated(lib):
    # 50 ms per batch of at most 4: with 32 concurrent callers and a 20 ms deadline most
    # requests are still queued when their deadline passes
    h = lib.hb_create(4, 1000, 0, 50000)
    rcs = [None] * 32
    outs = [(C.c_uint8 * 1)() for _ in range(32)]

    def call(i):
        rcs[i] = lib.hb_eval(h, 1 + i % 3, 1, i, 20000, outs[i])

    ts = [threading.Thread(target=call, args=(i,)) for i in range(32)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    st = _stats(lib, h)
    lib.hb_destroy(h)
    done = [i for i in range(32) if rcs[i] == 0]
    assert set(rcs) <= {0, ETIMEDOUT}
    assert rcs.count(ETIMEDOUT) >= 16 and len(done) >= 1
    assert st["expired"] == rcs.count(ETIMEDOUT)
    assert all(outs[i][0] == _expect(1 + i % 3, i) for i in done)


def test_queue_room_wait_honours_the_deadline(lib):
    # a queue of 2 behind a slow evaluator: producers that find it full give up at their
    # deadline without being queued
    h = lib.hb_create(1, 0, 2, 100000)
    rcs = []
    lock = threading.Lock()

    def call(i):
        out = (C.c_uint8 * 1)()
        rc = lib.hb_eval(h, 1, 1, i, 30000, out)
        with lock:
            rcs.append(rc)

    ts = [threading.Thread(target=call, args=(i,)) for i in range(12)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    lib.hb_destroy(h)
    assert rcs.count(ETIMEDOUT) >= 8 and rcs.count(0) >= 1


def test_two_workers_keep_each_requests_window(lib):
    """with two workers, a worker that wakes after the other one drained the queue
    waits for the NEW oldest request's window (it used to flush at the old deadline, sending
    small batches early). 16 closed-loop producers and a 3 ms window: batches stay full.
    (Not under the broadcast wake, a profiling mode: every batch wakes every waiting caller,
    so batch sizes depend on the host's load.)"""
    if lib.wake_mode == 1:
        pytest.skip("broadcast wake: batch sizes depend on host load")
    h = lib.hb_create(64, 3000, 0, 300)
    done = []

    def producer(seed):
        out = (C.c_uint8 * 1)()
        for i in range(40):
            assert lib.hb_eval(h, 1 + (seed % 3), 1, (seed + i) & 0xFF, 0, out) == 0
        done.append(seed)

    ts = [threading.Thread(target=producer, args=(s,)) for s in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    st = _stats(lib, h)
    lib.hb_destroy(h)
    assert len(done) == 16 and st["requests"] == 16 * 40
    print(st)
    assert st["requests"] / st["batches"] >= 12, st  # (mean batch size; 16 would be ideal)
