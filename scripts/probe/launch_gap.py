"""Dependent back-to-back kernel launches on one stream: µs per launch for an empty-ish kernel and
for the association kernel's shape (one tiny kernel per step), to size the inter-kernel gap a
step pays. usage: python scripts/probe/launch_gap.py"""
import time

import torch

dev = torch.device("cuda", 0)
x = torch.zeros(256, device=dev)
s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    for n in (1000, 4000):
        for _ in range(50):
            x.add_(1.0)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            x.add_(1.0)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / n * 1e6
        print(f"torch add_ on 256 floats, {n} launches: {dt:.2f} us per launch (host-bound if > GPU)")
    # GPU-side: events around a block of launches queued while the GPU is held busy by a long op
    big = torch.randn(8192, 8192, device=dev)
    for n in (200, 1000):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        big @ big   # keeps the GPU busy while the small launches are queued
        e0.record()
        for _ in range(n):
            x.add_(1.0)
        e1.record()
        torch.cuda.synchronize(dev)
        print(f"GPU time per queued dependent launch ({n}): {e0.elapsed_time(e1) * 1e3 / n:.2f} us")
