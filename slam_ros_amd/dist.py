"""Ensemble sharding across ranks: one process per GPU, E_total independent EKF
instances split into contiguous slices, the scan stream sent once per step from the sensor rank.

The reference has a single Robot per node (slam_ros/main.cpp:98) fed by one scan topic
(main.cpp:37-56); the ensemble gives every instance the same scan with its own seeded
perturbation. The only data-path collective is the broadcast of each step's payload — all
instances' encoder poses and lines, ≈ E_total × (3 + 6L) doubles — from rank 0 over
RCCL/xGMI (backend "nccl" on ROCm; "gloo" in the CPU tests). The landmark covariances never move.

Payload layout of one step (float64): [encoder (E_total, 3) | lines (E_total, L, 6)], where a line
row is ekf_line {alpha, r, R00, R01, R10, R11} (include/slam_ekf.h).
"""
from __future__ import annotations

import numpy as np

LINE_FIELDS = 6


def shard(E_total: int, world: int, rank: int) -> tuple[int, int]:
    """(first instance, count) of `rank`: contiguous, sizes differing by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(E_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def payload_len(E_total: int, L: int) -> int:
    return E_total * 3 + E_total * L * LINE_FIELDS


def pack(encoder: np.ndarray, lines: np.ndarray) -> np.ndarray:
    """encoder (E_total, 3), lines (E_total, L, 6) → flat float64 payload."""
    E = encoder.shape[0]
    if lines.shape[0] != E or lines.shape[2] != LINE_FIELDS:
        raise ValueError("payload shapes")
    return np.concatenate([np.ascontiguousarray(encoder, dtype=np.float64).ravel(),
                           np.ascontiguousarray(lines, dtype=np.float64).ravel()])


def offsets(E_total: int, L: int, first: int) -> tuple[int, int]:
    """Element offsets (not bytes) of a slice's encoder rows and line rows inside a payload."""
    return first * 3, E_total * 3 + first * L * LINE_FIELDS


def unpack_slice(buf, E_total: int, L: int, first: int, count: int):
    """Views of one rank's encoder (count, 3) and lines (count, L, 6) inside a payload (numpy
    array or torch tensor; no copy)."""
    eo, lo = offsets(E_total, L, first)
    enc = buf[eo: eo + count * 3].reshape(count, 3)
    lines = buf[lo: lo + count * L * LINE_FIELDS].reshape(count, L, LINE_FIELDS)
    return enc, lines


def broadcast_step(buf, dist, src: int = 0) -> None:
    """The one exchange of a step: the sensor rank's payload to every rank (in place)."""
    dist.broadcast(buf, src=src)


def broadcast_async(buf, dist, src: int = 0):
    """Same for a group of steps, asynchronously; `.wait()` on the returned work orders the
    caller's current stream after it (NCCL/RCCL) or blocks until it is done (gloo)."""
    return dist.broadcast(buf, src=src, async_op=True)
