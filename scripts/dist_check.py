"""Rehearsal of bench.py's grouped, one-group-ahead scan broadcast on one GPU (gloo or nccl):
every rank checks that the buffer it hands to each step holds exactly rank 0's payload row."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
from slam_ros_amd import dist as D

backend = sys.argv[1] if len(sys.argv) > 1 else "gloo"
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group(backend)
steps, per, B = 23, 1000, 4
expect = torch.arange(steps * per, dtype=torch.float64, device=dev).reshape(steps, per)
payload = expect.clone() if rank == 0 else torch.empty_like(expect)
recv = torch.empty((2, B, per), dtype=torch.float64, device=dev)
inflight = {}
def issue(gi):
    if gi * B >= steps:
        return
    buf = recv[gi & 1]
    cnt = min(B, steps - gi * B)
    if rank == 0:
        buf[:cnt].copy_(payload[gi * B: gi * B + cnt], non_blocking=True)
    inflight[gi] = D.broadcast_async(buf, dist, src=0)
issue(0)
bad = 0
for s in range(steps):
    gi, k = divmod(s, B)
    if k == 0:
        inflight.pop(gi).wait()
        issue(gi + 1)
    got = recv[gi & 1][k]
    bad += int(not torch.equal(got, expect[s]))
    torch.cuda._sleep(1000000)   # the consumer runs behind, as the EKF kernels do
torch.cuda.synchronize()
print(f"rank {rank} backend {backend}: {bad} bad steps of {steps}")
dist.destroy_process_group()
