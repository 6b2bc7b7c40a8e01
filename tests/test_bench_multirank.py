"""bench.py with two ranks on the one GPU of a test box (the 8-GPU run is the driver's): the
launcher, the ensemble sharding, GroupedBroadcast's one-group-ahead scan stream and the product
library on every rank. Transport: gloo on host copies (BENCH_SAME_DEVICE=1 puts both ranks on
device 0, where RCCL cannot pair a device with itself); the RCCL path differs only in the
collective call (slam_ros_amd/dist.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("bcast_every", [3, 8])
def test_bench_two_ranks_one_gpu(bcast_every):
    env = dict(os.environ, BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "13", "--warmup", "3",
           "--preroll", "0", "--capacity", "256", "--instances", "2", "--no-cpu",
           "--dist-backend", "gloo", "--bcast-every", str(bcast_every)]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 prints one line
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 4
    assert r["all_lines_matched"] is True        # every instance of both ranks matched its 8 lines
    assert r["value"] > 0 and r["steps"] == 13
    assert f"broadcast of {bcast_every} scans" in r["config"]["parallelism"]
