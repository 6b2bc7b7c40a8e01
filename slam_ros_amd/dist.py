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


class GroupedBroadcast:
    """The scan stream of bench.py's multi-rank run: rank `src` holds every step's payload
    (`payload`, shape (steps_total, per_step)); groups of B consecutive steps go out in one
    collective, issued one group ahead of the steps that consume them, into a double-buffered
    receive area. Step s reads row s % B of group s // B:

        gi, k = divmod(s, B)
        k == 0: wait for group gi (NCCL/RCCL: the current stream waits; gloo: blocks), then issue
                group gi + 1 into the other buffer (it overlaps group gi's steps)

    Buffer reuse is ordered by construction: group gi + 1 overwrites the buffer group gi − 1's
    steps read, and those were issued before it (stream order on the GPU; synchronous on CPU).
    `host_coll`: the collective runs on host copies (gloo rehearsal of GPU ranks). `force`: the
    collective path even for a world of one (the RCCL device branch on a one-GPU box)."""

    def __init__(self, payload, B: int, dist, rank: int, world: int, src: int = 0,
                 host_coll: bool = False, sync=None, force: bool = False):
        self.payload, self.B, self.dist = payload, max(1, int(B)), dist
        self.rank, self.world, self.src = rank, world, src
        self.coll = world > 1 or force
        self.steps_total = payload.shape[0]
        self.host_coll, self.sync = host_coll, sync
        self.recv = payload.new_empty((2, self.B, payload.shape[1])) if self.coll else None
        self.inflight = {}
        self.issued = []        # group indices in issue order (tests)

    class _Done:
        def wait(self):
            pass

    def issue(self, gi: int) -> None:
        if not self.coll or gi * self.B >= self.steps_total:
            return
        import torch
        B = self.B
        buf = self.recv[gi & 1]
        cnt = min(B, self.steps_total - gi * B)
        self.issued.append(gi)
        if self.host_coll:
            if self.sync:
                self.sync()     # the previous user of this buffer is done
            hb = (self.payload[gi * B: gi * B + cnt].cpu() if self.rank == self.src
                  else torch.empty((cnt, self.payload.shape[1]), dtype=self.payload.dtype))
            broadcast_step(hb, self.dist, src=self.src)
            buf[:cnt].copy_(hb[:cnt].to(buf.device))
            self.inflight[gi] = self._Done()
            return
        if self.rank == self.src:
            buf[:cnt].copy_(self.payload[gi * B: gi * B + cnt], non_blocking=True)
        self.inflight[gi] = broadcast_async(buf, self.dist, src=self.src)

    def start(self) -> None:
        self.issue(0)

    def step_buffer(self, s: int):
        """The payload row step s consumes (a view into the receive area for world > 1)."""
        if not self.coll:
            return self.payload[s]
        gi, k = divmod(s, self.B)
        if k == 0:
            self.inflight.pop(gi).wait()
            self.issue(gi + 1)
        return self.recv[gi & 1][k]
