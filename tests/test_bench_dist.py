"""The N>1 path of bench.py on CPU (gloo, world_size 2): each rank times its own shard,
the timed region is bracketed by barriers and the reported time is the max over ranks;
shards are independent (different documents per rank, no data-path collective)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from authorino_amd import workloads

    w = workloads.make("c2", n=64, seed=workloads.DEFAULT_SEEDS["c2"] + 7919 * rank)  # the shard bench.py gives this rank
    delay = 0.02 * (rank + 1)
    calls = []

    def step():
        calls.append(1)
        time.sleep(delay)

    elapsed, _ = bench.timed_steps(step, 4, 2, dist, torch, None)
    with open(os.path.join(out, f"r{rank}.json"), "w") as f:
        json.dump({"elapsed": elapsed, "calls": len(calls), "first_doc": w.doc(0).decode()}, f)
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_timing_and_shards(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    r = [json.load(open(tmp_path / f"r{k}.json")) for k in range(world)]
    assert r[0]["calls"] == r[1]["calls"] == 6  # warmup + exactly K timed steps
    assert r[0]["elapsed"] == r[1]["elapsed"]  # max over ranks, reported identically
    assert r[0]["elapsed"] >= 4 * 0.04 * 0.95  # at least the slower rank's timed steps
    assert r[0]["first_doc"] != r[1]["first_doc"]  # independent shards


@pytest.mark.timeout(300)
def test_bench_gpus2_relaunches_two_ranks():
    """`bench.py --gpus 2` without a torch.distributed.run environment starts two ranks
    itself (torch.distributed.run child), each with its own shard; rank 0 prints one JSON
    line with n_gpus 2. --dry-run keeps the GPU out (gloo, stand-in step)."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--workload", "c2", "--n", "96", "--steps", "3", "--warmup", "1"],
                         capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1 and rec["scaling"] == "weak"
    shards = rec["shards"]
    assert [s["rank"] for s in shards] == [0, 1]
    assert shards[0]["seed"] != shards[1]["seed"]
    assert shards[0]["first_doc_sha"] != shards[1]["first_doc_sha"]  # independent shards
    assert all(s["n"] == 96 for s in shards)


@pytest.mark.timeout(300)
def test_bench_gather_decisions_two_ranks():
    """--gather-decisions (optional): each step all-gathers every rank's
    decision bitmap; every rank finds its own bitmap in its slice of the gathered buffer."""
    import subprocess

    import numpy as np

    sys.path.insert(0, ROOT)
    from authorino_amd import workloads

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--gather-decisions", "--workload", "c2", "--n", "96", "--steps", "2", "--warmup", "1"],
                         capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    g = rec["decision_gather"]
    assert g["ranks"] == 2 and g["bytes_per_rank"] == 12 and g["bytes_gathered"] == 24
    assert g["slices_equal_to_local"]
    # the stand-in results are lens % 3 (T = 1) on each rank's own shard
    want = 0
    for r in range(2):
        w = workloads.make("c2", n=96, seed=workloads.DEFAULT_SEEDS["c2"] + 7919 * r, unique=64, uniquify=True)
        want += int((w.lens % 3 == 1).sum())
    assert g["allowed_bits"] == want
    assert "all-gather" in rec["config"]["parallelism"]


def test_decision_bitmap_layout():
    sys.path.insert(0, ROOT)
    import bench

    tri = torch.tensor([1, 0, 1, 1, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1], dtype=torch.uint8)
    wts = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8)
    got = bench.decision_bitmap(torch, tri, 1, wts)
    assert got.tolist() == [0b00101101, 0b10000000]


@pytest.mark.gpu
def test_decision_bitmap_on_device():
    """The bitmap bench.py all-gathers, built by the same torch ops on the GPU."""
    sys.path.insert(0, ROOT)
    import bench

    g = torch.Generator().manual_seed(5)
    tri = torch.randint(0, 4, (4096,), generator=g, dtype=torch.uint8)
    wts = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8)
    want = bench.decision_bitmap(torch, tri, 1, wts)
    got = bench.decision_bitmap(torch, tri.cuda(), 1, wts.cuda()).cpu()
    assert torch.equal(got, want)
    assert int(want[0]) == sum(1 << k for k in range(8) if int(tri[k]) == 1)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_rccl_gather_one_rank_on_device():
    """The real multi-GPU driver at world size 1: bench.py under torch.distributed.run
    (a child process started before anything here touches the GPU), RCCL process group
    with device_id, the decision bitmap all-gathered on the bench stream inside the timed
    step; the JSON line, the gathered slice equal to the rank's own bitmap, and parity of
    the shard against the oracle sample."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--gather-decisions", "--steps", "2", "--warmup", "1", "--requests", "65536",
           "--cpu-seconds", "2", "--no-pcie"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=540, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = lines[0]
    g = rec["decision_gather"]
    assert g["ranks"] == 1 and g["slices_equal_to_local"]
    assert g["bytes_per_rank"] * 8 == rec["config"]["requests_per_gpu"] * rec["config"]["trees_per_request"]
    assert rec["parity"]["mismatches"] == 0 and rec["parity"]["sample"] > 0
    assert rec["undecided"] == 0
