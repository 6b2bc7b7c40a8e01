"""Rank process of tests/test_rowshard_gpu.py: one instance with its landmark block partitioned
over the ranks (slam_ros_amd/rowshard_gpu.py), every rank a partitioned context of the product
library (gloo group; on the test box every rank shares its one GPU). Writes its state (the robot
rows, mean, pose and its tiles' entries of P), the matches per scan, its landmark-block bytes and
the per-scan wall time to OUT/rank<r>.npz."""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf as E, rowshard_gpu as R, scan_gen as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--N", type=int, default=1024)
ap.add_argument("--T", type=int, default=4)
ap.add_argument("--scans", type=int, default=9)
ap.add_argument("--precision", type=int, default=E.PREC_F32)
ap.add_argument("--active", type=int, default=0, help="active landmarks (0: N - 10)")
ap.add_argument("--extra-every", type=int, default=0, help="two unmatched lines every k scans")
ap.add_argument("--backend", default="gloo")
ap.add_argument("--per-line", action="store_true", help="the per-line protocol only (no speculative run)")
ap.add_argument("--dup-every", type=int, default=0, help="line 1 repeats line 0 every k scans")
ap.add_argument("--wrong-guess", action="store_true", help="EKF_OPT_SPECULATE = 2: every line guesses landmark 0")
ap.add_argument("--native", action="store_true", help="the whole scan in one library call on its own RCCL communicator")
args = ap.parse_args()

dist.init_process_group(args.backend)
rank = dist.get_rank()
torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) if args.backend == "nccl" else 0)
w = G.make_world(args.N, active=args.active or args.N - 10)
st = G.initial_state(w)
inst = R.ShardedInstance(args.N, args.precision, max_lines=8, flush_interval=args.T, speculate=not args.per_line,
                         options={"speculate": 2} if args.wrong_guess else None, native=args.native)
inst.init_lowrank(st.diag, st.U, st.y, st.saved, st.pose)
matches, times = [], []
rng = np.random.default_rng(11)
for step in range(1, args.scans + 1):
    enc, lines, nl = G.make_scan(w, step, instances=1, lines=6 if args.extra_every else 8)
    ln = lines[0, :nl[0]]
    if args.extra_every and step % args.extra_every == 0:
        ln = np.concatenate([ln, G.random_lines(rng, 2)])
    if args.dup_every and step % args.dup_every == 0:
        ln = ln.copy()
        ln[1] = ln[0]
    dist.barrier()
    t0 = time.perf_counter()
    matches.append(inst.localize(ln, enc[0]) + [-2] * (8 - len(ln)))
    times.append(time.perf_counter() - t0)
P, y, saved, pose = inst.download_state()
np.savez(os.path.join(args.out, f"rank{rank}.npz"), P=P, y=y, saved=saved, pose=pose, matches=np.array(matches),
         tile_rows=np.array(inst.tile_rows), block_bytes=inst.landmark_block_bytes(), times=np.array(times),
         status=inst.status(), spec_runs=np.array(inst.spec_runs))
inst.close()
dist.barrier()
dist.destroy_process_group()
