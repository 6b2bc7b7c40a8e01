"""One instance row-sharded across two ranks on the product kernels:
two gloo ranks on the one GPU of the test box, each a context owning half of the landmarks
(ekf_shard_*), against a single context of the same library on the same scans. Exact arithmetic:
the owned rows of P (all columns), the robot block and strip columns of the owned landmarks, the
owned entries of the mean, the pose and every association are bit-identical (the phases run the
scan kernel's sequential-path expressions; the flush is the product wave kernel on the wave-tiles
that hold an owned row block, with the all-gathered operand rows)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from slam_ros_amd import scan_gen as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("prec,N,T,scans", [(1, 1024, 4, 9), (1, 1000, 6, 8), (0, 512, 4, 6)])
def test_two_rank_shard_equals_single_context(ekf_mod, tmp_path, prec, N, T, scans):
    w = G.make_world(N)
    st = G.initial_state(w)
    one = ekf_mod.Ensemble(N, 1, prec, max_lines=8, flush_interval=T)
    one.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
    ref_matches = []
    for step in range(1, scans + 1):
        enc, lines, nl = G.make_scan(w, step, instances=1)
        r = one.localize(enc, lines, nl)
        ref_matches.append(r[0]["match"][:nl[0]])
    P, y, saved, pose = one.download_state(0)
    one.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "rowshard_gpu_worker.py"), "--out", str(tmp_path), "--N", str(N),
           "--T", str(T), "--scans", str(scans), "--precision", str(prec)]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    covered = 0
    for r in range(2):
        d = np.load(tmp_path / f"rank{r}.npz")
        idx = d["rows"]
        covered += len(idx)
        assert [list(m) for m in d["matches"]] == [list(m) for m in ref_matches], r
        assert all(len(m) == 8 and min(m) >= 0 for m in ref_matches)   # the sharded form needs no augmentation
        np.testing.assert_array_equal(d["P_rows"], P[idx])            # owned rows, every column
        np.testing.assert_array_equal(d["P_robot"][:, :3], P[:3, :3])
        np.testing.assert_array_equal(d["P_robot"][:, idx], P[:3, idx])
        np.testing.assert_array_equal(d["y"][idx], y[idx])
        np.testing.assert_array_equal(d["y"][:3], y[:3])
        np.testing.assert_array_equal(d["pose"], pose)
        assert int(d["saved"]) == saved and int(d["status"]) == 0
    assert covered == 2 * N


def test_shard_refuses_augmentation(ekf_mod):
    """A scan with an unmatched line (a new landmark) is refused before anything is committed."""
    import torch.distributed as dist
    from slam_ros_amd import rowshard_gpu as R
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    N = 256
    w = G.make_world(N)
    st = G.initial_state(w)
    inst = R.ShardedInstance(N, 1, max_lines=8, flush_interval=4)
    inst.init_lowrank(st.diag, st.U, st.y, st.saved, st.pose)
    enc, lines, nl = G.make_scan(w, 1, instances=1)
    extra = G.random_lines(np.random.default_rng(2), 1)
    with pytest.raises(ekf_mod.EkfError):
        inst.localize(np.concatenate([lines[0, :7], extra]), enc[0])
    inst.close()
    dist.destroy_process_group()
