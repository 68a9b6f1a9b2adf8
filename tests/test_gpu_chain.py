"""The device chain around the kernels on the GPU, through the
C-ABI, against the oracle:
  f3  the Authorization-JSON producer (authjx_pack_json, pkg/service/auth_pipeline.go:
      542-616) packs request values straight into the arena the kernels read;
  f4  the batched host -> AuthConfig lookup (authjx_index_lookup_batch, pkg/index/
      index.go:153-174 + the ':port' retry of pkg/service/auth.go:270-289) gives the
      set_of_req of a multi-tenant (c4) batch."""
import json

import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from authorino_amd import runtime

    return runtime.Context(0)


def _device_eval(ctx, sets, arena, offs, lens, sor=None):
    import torch

    dev = torch.device("cuda", 0)
    A = torch.from_numpy(np.ascontiguousarray(arena)).to(dev)
    Of = torch.from_numpy(offs.view(np.int64)).to(dev)
    Ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    S = torch.from_numpy(sor.astype(np.int32)).to(dev) if sor is not None else None
    n = len(lens)
    words = (max(s.n_patterns for s in sets) + 63) // 64
    tri = torch.empty(n, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.int32, device=dev)
    bm = torch.empty((n, words), dtype=torch.int64, device=dev)
    ctx.eval_device(sets, A, Of, Ln, tri, err, bm, set_of_req=S)
    torch.cuda.synchronize()
    return tri.cpu().numpy(), err.cpu().numpy(), bm.cpu().numpy().view(np.uint64)


def test_producer_arena_on_device(ctx):
    """Request values (the c2 documents as Go structs / maps) encoded by authjx_pack_json
    into one arena: byte for byte the workload's documents, evaluated on the device from
    that arena equal to the oracle."""
    from authorino_amd import producer as P
    from authorino_amd import workloads as W

    w = W.make("c2", n=30000, seed=61)
    values = [json.loads(w.doc(i)) for i in range(w.n)]  # (dict order = Go field order)
    arena, offs, lens = P.pack(values)
    assert np.array_equal(lens, w.lens)
    assert all(bytes(arena[int(o):int(o) + int(n)]) == w.doc(i) for i, (o, n) in enumerate(zip(offs, lens)))
    rs = ctx.compile_expression(w.expr)
    tri, err, bm = _device_eval(ctx, [rs], arena, offs, lens)
    ors = O.Ruleset.from_expression(w.expr)
    otri, oerr, obm = O.eval_batch([ors], arena, offs, lens, nthreads=8)
    assert (tri == 3).sum() == 0
    assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)
    assert 0 < (tri == 1).sum() < w.n


def test_native_index_selects_c4_rulesets_on_device(ctx):
    """c4: every request's host resolved by the native batched lookup (all host threads)
    to a ruleset id — equal to the restatement's selection — and that set_of_req drives
    the multi-tenant kernel; results equal the oracle on the same selection."""
    from authorino_amd import index as hix
    from authorino_amd import workloads as W

    w = W.make("c4", n=60000, seed=62)
    nat = hix.NativeIndex()
    for key, sid in W.c4_index_entries():
        nat.set(key, sid)
    ha, ho, hl = hix.pack_hosts(w.hosts)
    sor = nat.lookup_batch(ha, ho, hl)
    assert (sor >= 0).all()
    assert np.array_equal(sor, w.set_of_req.astype(sor.dtype))
    sets = [ctx.compile_expression(e) for e in w.exprs]
    tri, err, bm = _device_eval(ctx, sets, w.arena, w.offs, w.lens, sor=sor.astype(np.uint32))
    osets = [O.Ruleset.from_expression(e) for e in w.exprs]
    otri, oerr, obm = O.eval_batch(osets, w.arena, w.offs, w.lens, set_of_req=sor.astype(np.uint32), nthreads=8)
    assert (tri == 3).sum() == 0
    assert np.array_equal(tri, otri) and np.array_equal(err, oerr) and np.array_equal(bm, obm)


def test_shutdown_destroys_live_batchers():
    """authjx_shutdown with a micro-batcher still alive on the context: the
    batcher is destroyed first (its queue drained, workers joined), no use after free."""
    from authorino_amd import runtime

    ctx = runtime.Context(0)
    rs = ctx.compile([("a", 1, "x")], [(0, -1, -1, 0)], 0)
    b = runtime.Batcher(ctx, max_batch=64, window_us=100)
    tri, _ = b.eval(rs, b'{"a":"x"}')
    assert int(tri[0]) == runtime.T
    ctx.close()
    assert b._h is None
    b.close()  # (a no-op now)


def test_release_stream_workspace():
    """authjx_release_stream (one workspace per stream handle, kept until
    shutdown): a short-lived stream's workspace is freed after its batch; evaluating on
    a new stream afterwards still gives the oracle's results."""
    import torch

    from authorino_amd import runtime

    ctx = runtime.Context(0)
    rs = ctx.compile([("a", 1, "x")], [(0, -1, -1, 0)], 0)
    docs = [b'{"a":"x"}', b'{"a":"y"}'] * 64
    arena = np.frombuffer(b"".join(docs) + b"\0", dtype=np.uint8)
    lens = np.array([len(d) for d in docs], dtype=np.uint32)
    offs = np.zeros(len(docs), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    dev = torch.device("cuda:0")
    A = torch.from_numpy(arena.copy()).to(dev)
    Of = torch.from_numpy(offs.view(np.int64).copy()).to(dev)
    Ln = torch.from_numpy(lens.view(np.int32).copy()).to(dev)
    for _ in range(3):
        s = torch.cuda.Stream()
        tri = torch.zeros(len(docs), dtype=torch.uint8, device=dev)
        ctx.eval_device([rs], A, Of, Ln, tri, stream=s.cuda_stream)
        s.synchronize()
        assert tri.cpu().numpy().tolist() == [runtime.T, runtime.F] * 64
        ctx.release_stream(s.cuda_stream)
    ctx.close()
