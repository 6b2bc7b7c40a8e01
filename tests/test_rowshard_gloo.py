"""§8f #4: one EKF instance with P row-sharded over ranks (tests/rowshard_protocol.py)
against the single-process CPU restatement (oracle/, fast mode). gloo, world_size 2 and 3: the
trajectory — matches, augmentation rows that land on either rank, the capacity reset — must be
bit-identical, association included (the sharded gating picks the first passing landmark over
all ranks with one all-reduce per line)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from slam_ros_amd import scan_gen as G

N = 40
SCANS = 22


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def scenario():
    """Scans of the synthetic world (re-observations) plus new lines every third scan; the map
    fills past N − 10 (reset) mid-trajectory."""
    w = G.make_world(N, active=N - 13)
    st = G.initial_state(w)
    rng = np.random.default_rng(3)
    scans = []
    for step in range(1, SCANS + 1):
        enc, lines, _ = G.make_scan(w, step, lines=6)
        extra = G.random_lines(rng, 2 if step % 3 == 0 else 0)
        scans.append((enc[0], np.concatenate([lines[0], extra])))
    return st, scans


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.rowshard_protocol import RowShardedRobot
    st, scans = scenario()
    rob = RowShardedRobot(N, dist)
    rob.set_state(st.dense_P(), st.y, st.saved, st.pose)
    log = []
    for enc, lines in scans:
        m = rob.localize(lines, enc)
        log.append((m, list(rob.pose), rob.saved, rob.status))
    P = rob.gather_P()
    if rank == 0:
        q.put((log, P, rob.y.copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_instance_matches_single_process(oracle_mod, world):
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    log, P, y = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    st, scans = scenario()
    ref = oracle_mod.OracleRobot(N, mode=oracle_mod.FAST)
    ref.set_state(st.dense_P(), st.y, st.saved, st.pose)
    resets = matched = added = 0
    prev_saved = st.saved
    for k, ((enc, lines), (m, pose, saved, status)) in enumerate(zip(scans, log)):
        mref = ref.localize(lines, enc)
        assert m == mref, (k, m, mref)
        assert list(pose) == list(ref.pose), (k, pose, ref.pose)
        assert saved == ref.savedLineCount, k
        matched += sum(1 for j in m if j >= 0)
        added += sum(1 for j in m if j < 0)
        resets += saved < prev_saved
        prev_saved = saved
    np.testing.assert_array_equal(P, ref.P_t0)
    np.testing.assert_array_equal(y, ref.y)
    assert resets >= 1 and matched >= 4 * SCANS and added >= 10


def test_row_ownership_partition():
    from slam_ros_amd.dist import shard
    for Ncap in (5, 40, 4096):
        for world in (1, 2, 3, 8):
            rows = []
            for r in range(world):
                a, c = shard(Ncap, world, r)
                rows += list(range(3 + 2 * a, 3 + 2 * (a + c)))
            assert rows == list(range(3, 3 + 2 * Ncap))
