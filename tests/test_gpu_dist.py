"""The multi-GPU driver on the single-GPU box: bench.py under torch.distributed.run at
world size 1 with the NCCL (RCCL) backend and --gather-decisions, so the process-group
init with device_id, the per-rank device selection and the in-step
all_gather_into_tensor of the decision bitmaps on the bench stream all run on the GPU
(the N-rank runs are the driver's). The child is started before this process
touches the GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_rccl_world1_gather_decisions():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--gather-decisions", "--steps", "2", "--warmup", "1", "--requests", "65536", "--no-pcie",
           "--cpu-seconds", "1"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    assert "all-gather" in d["config"]["parallelism"]
    g = d["decision_gather"]
    assert g["ranks"] == 1 and g["slices_equal_to_local"] is True
    assert g["bytes_gathered"] == g["bytes_per_rank"] == 65536 // 8
    # the shard's decisions against the oracle (the bench's CPU sample)
    assert d["parity"] is not None and d["parity"]["mismatches"] == 0, d["parity"]
    assert d["undecided"] == 0
