"""The N>1 path of bench.py on CPU (gloo, world_size 2): each rank times its own shard,
the timed region is bracketed by barriers and the reported time is the max over ranks;
shards are independent (different documents per rank, no data-path collective)."""
import json
import os
import socket
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

    w = workloads.make("c2", n=64, seed=1000 + rank)  # the shard bench.py gives this rank
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
