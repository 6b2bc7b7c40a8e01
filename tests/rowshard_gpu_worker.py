"""Rank process of tests/test_rowshard_gpu.py: one instance row-sharded over the ranks of a gloo
group, every rank a context of the product library on the same GPU (slam_ros_amd/rowshard_gpu.py).
Writes its owned rows of the final state and the matches per scan to OUT/rank<r>.npz."""
import argparse
import os
import sys

import numpy as np
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
args = ap.parse_args()

dist.init_process_group("gloo")
rank = dist.get_rank()
w = G.make_world(args.N, active=args.active or args.N - 10)
st = G.initial_state(w)
inst = R.ShardedInstance(args.N, args.precision, max_lines=8, flush_interval=args.T)
inst.init_lowrank(st.diag, st.U, st.y, st.saved, st.pose)
matches = []
rng = np.random.default_rng(11)
for step in range(1, args.scans + 1):
    enc, lines, nl = G.make_scan(w, step, instances=1, lines=6 if args.extra_every else 8)
    ln = lines[0, :nl[0]]
    if args.extra_every and step % args.extra_every == 0:
        ln = np.concatenate([ln, G.random_lines(rng, 2)])
    matches.append(inst.localize(ln, enc[0]) + [-2] * (8 - len(ln)))
P, y, saved, pose = inst.download_state()
idx = inst.owned_index()
np.savez(os.path.join(args.out, f"rank{rank}.npz"), rows=idx, P_rows=P[idx], P_robot=P[:3, :], y=y,
         saved=saved, pose=pose, matches=np.array(matches), a=inst.a, b=inst.b, status=inst.status())
inst.close()
dist.barrier()
dist.destroy_process_group()
