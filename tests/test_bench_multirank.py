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

import numpy as np
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


@pytest.mark.gpu
@pytest.mark.parametrize("arith", ["exact", "bf16x6"])
def test_two_ranks_equal_one_rank(tmp_path, arith):
    """Every instance's final state (P, y, savedLineCount, pose) after bench.py's whole schedule on
    two ranks (two instances each) is bitwise the state a single-rank run of the same four global
    instances ends in: the sharding, the grouped broadcast of the scan stream and the per-rank
    contexts change nothing per instance (the arithmetic of an instance never depends on the
    others in its launch)."""
    common = ["--steps", "13", "--warmup", "3", "--preroll", "0", "--capacity", "256", "--no-cpu",
              "--arith", arith, "--flush-interval", "8" if arith == "exact" else "12"]
    env = dict(os.environ, BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1")
    two = tmp_path / "two"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--instances", "2", "--dist-backend", "gloo",
           "--bcast-every", "3", "--dump-state", str(two)] + common
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    one = tmp_path / "one"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--instances", "4",
           "--dump-state", str(one)] + common
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    for k in range(4):
        a, b = np.load(two / f"state_{k}.npz"), np.load(one / f"state_{k}.npz")
        for key in ("P", "y", "saved", "pose"):
            assert np.array_equal(a[key], b[key]), (arith, k, key)
        assert int(a["saved"]) == 246   # s = N − 10 kept: every line matched, no augmentation


@pytest.mark.gpu
def test_rccl_grouped_broadcast_world1(tmp_path):
    """GroupedBroadcast's device branch (dist.py: the payload rows copied on the stream, RCCL's
    in-place broadcast into the double-buffered receive area, work.wait() ordering the stream) on
    the nccl backend, forced at a world of one on the test box's single GPU (--force-collective):
    over several groups and a partial last one, every instance ends bitwise in the state of the
    same run fed straight from the payload (the stream ordering and the buffer reuse lose or
    reorder no scan). The multi-GPU curve is the driver's 8-GPU run."""
    common = ["--steps", "13", "--warmup", "3", "--preroll", "4", "--capacity", "256", "--instances", "4",
              "--no-cpu", "--arith", "f16x3", "--flush-interval", "6", "--bcast-every", "5"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    coll = tmp_path / "coll"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-collective",
                          "--dist-backend", "nccl", "--dump-state", str(coll)] + common,
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert "forced through the nccl collective" in r["config"]["parallelism"], r["config"]
    assert r["all_lines_matched"] is True
    plain = tmp_path / "plain"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dump-state", str(plain)] + common,
                         cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-3000:]
    for k in range(4):
        a, b = np.load(coll / f"state_{k}.npz"), np.load(plain / f"state_{k}.npz")
        for key in ("P", "y", "saved", "pose"):
            assert np.array_equal(a[key], b[key]), (k, key)
