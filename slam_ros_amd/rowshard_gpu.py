"""One EKF instance row-sharded across ranks on the product kernels.

Each rank holds a context (include/slam_ekf.h ekf_shard_*) that owns the landmarks [a, b) of the
instance: its association phases touch those landmarks only, and its deferred flush runs the
product wave kernel on the wave-tiles that hold an owned row block. Per scan (Robot::localize,
Robot.cpp:126-904, sequential association):

  ekf_shard_begin                  predict (Robot.cpp:130-286), the owned landmarks' scan state
  per line i (Robot.cpp:298-641):
    ekf_shard_gate                 first passing owned unmatched landmark
    all-reduce MIN                 the reference takes the first passing landmark in index order
    ekf_shard_package (owner)      S, S⁻¹, v, H row, K·S and K robot rows, the winner's V history
    broadcast from the owner
    ekf_shard_apply                gain rows of the owned landmarks (Robot.cpp:522-602), robot update
  ekf_shard_end                    commit (Robot.cpp:702-716), augmentation (Robot.cpp:776-866): each
                                   rank its columns of the new landmarks' rows, the new landmark's
                                   owner its strip columns and mean; the reset (Robot.cpp:893-904)
  all-gather of the operand rows   the step's U/V rows: the flush of a tile needs the rows of both
                                   its row and its column block (the n×2m exchange of rowshard.py),
  and of the new-landmark rows     and the new rows' columns of every rank
  ekf_shard_commit                 the step joins the flush schedule

The collectives go through torch.distributed (gloo: host-staged, as the tests run two ranks on one
GPU; on an 8-GPU node the same calls run over RCCL on device tensors).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import ekf as E

INT_MAX = 0x7FFFFFFF
LINE_FIELDS = 6   # struct ekf_line: alpha, r, R[4]
TILE = 32


def shard_range(N: int, world: int, rank: int, align: int = 16) -> tuple[int, int]:
    """Owned landmarks [a, b): contiguous, in multiples of `align` landmarks (one 32-row tile
    block), sizes differing by at most one multiple."""
    units = (N + align - 1) // align
    base, extra = divmod(units, world)
    first = rank * base + min(rank, extra)
    cnt = base + (1 if rank < extra else 0)
    return min(first * align, N), min((first + cnt) * align, N)


def operand_rows(nb: int, kmax: int, f64: bool) -> np.ndarray:
    """Row of every element of one instance's operand array (ekf_layout.h op_index_f32 / _f64)."""
    rows = np.repeat(np.arange(nb * TILE), kmax)
    ks = np.tile(np.arange(kmax), nb * TILE)
    rb = rows >> 5
    if f64:
        h = (rows >> 4) & 1
        kq = kmax // 4
        lane = (rows & 15) + 16 * (ks & 3)
        idx = (rb * 64 + lane) * (2 * kq) + h * kq + (ks >> 2)
    else:
        lane = (rows & 31) + 32 * (ks & 1)
        idx = (rb * 64 + lane) * (kmax // 2) + (ks >> 1)
    out = np.empty(nb * TILE * kmax, dtype=np.int64)
    out[idx] = rows
    return out


class ShardedInstance:
    """One instance over the ranks of the default process group (or `group`)."""

    def __init__(self, capacity: int, precision: int = E.PREC_F32, max_lines: int = 8,
                 flush_interval: int = 4, r_mode: int = E.R_INTENDED, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.N = capacity
        self.ranges = [shard_range(capacity, self.world, r) for r in range(self.world)]
        self.a, self.b = self.ranges[self.rank]
        self.ens = E.Ensemble(capacity, 1, precision, max_lines=max_lines, flush_interval=flush_interval,
                              r_mode=r_mode)
        self.lib = E.load_library()
        self.h = self.ens._h
        self.max_lines = max_lines
        self.f64 = precision == E.PREC_F64
        self._inited = False
        self.words = self.lib.ekf_shard_package_words(self.h)
        self.opb = self.lib.ekf_shard_operand_bytes(self.h)
        dt = np.float64 if self.f64 else np.float32
        nb = (2 * capacity + TILE - 1) // TILE
        kmax = ((2 * max_lines + 15) // 16) * 16
        rows = operand_rows(nb, kmax, self.f64)
        self.mask = [(rows >= 2 * a) & (rows < 2 * b) for a, b in self.ranges]
        self.dtype = dt
        # the patch buffer [max_lines][2][2N]: column c belongs to landmark c // 2
        self.pwords = self.lib.ekf_shard_patch_bytes(self.h) // 8
        cols = np.tile(np.arange(2 * capacity), self.pwords // (2 * capacity))
        self.pmask = [(cols >= 2 * a) & (cols < 2 * b) for a, b in self.ranges]

    # state: every rank starts from the same full state, then keeps its rows
    def init_lowrank(self, diag, U, y, saved, pose):
        self.ens.init_lowrank(0, diag, U, y, saved, pose)
        self._shard()

    def upload_state(self, P, y, saved, pose):
        self.ens.upload_state(0, P, y, saved, pose)
        self._shard()

    def _shard(self):
        if not self._inited:
            E._check(self.lib.ekf_shard_init(self.h, self.a, self.b), "ekf_shard_init")
            self._inited = True

    def owner(self, j: int) -> int:
        for r, (a, b) in enumerate(self.ranges):
            if a <= j < b:
                return r
        raise ValueError(j)

    def localize(self, lines, enc) -> list[int]:
        """Robot::localize on the sharded instance; returns the matched landmark per line."""
        lib, h = self.lib, self.h
        ln = np.ascontiguousarray(np.asarray(lines, dtype=np.float64).reshape(-1, LINE_FIELDS))
        L = ln.shape[0]
        enc = np.ascontiguousarray(np.asarray(enc, dtype=np.float64).reshape(3))
        E._check(lib.ekf_shard_begin(h, E._dp(enc), ln.ctypes.data_as(ctypes.c_void_p), L), "ekf_shard_begin")
        out, pkg = [], np.zeros(self.words)
        best = ctypes.c_int32()
        for i in range(L):
            E._check(lib.ekf_shard_gate(h, i, ctypes.byref(best)), "ekf_shard_gate")
            t = torch.tensor([best.value], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            j = int(t.item())
            j = -1 if j == INT_MAX else j
            if j >= 0:
                src = self.owner(j)
                if src == self.rank:
                    E._check(lib.ekf_shard_package(h, i, j, E._dp(pkg)), "ekf_shard_package")
                tp = torch.from_numpy(pkg)
                dist.broadcast(tp, src=src, group=self.group)
                pkg = tp.numpy()
            E._check(lib.ekf_shard_apply(h, i, j, E._dp(pkg)), "ekf_shard_apply")
            out.append(j)
        E._check(lib.ekf_shard_end(h), "ekf_shard_end")
        # the step's operand rows: every rank contributes its rows
        U = np.empty(self.opb // self.dtype().itemsize, dtype=self.dtype)
        V = np.empty_like(U)
        E._check(lib.ekf_shard_operands(h, U.ctypes.data_as(ctypes.c_void_p), V.ctypes.data_as(ctypes.c_void_p), 0),
                 "ekf_shard_operands")
        gu = [torch.empty(U.shape, dtype=torch.from_numpy(U).dtype) for _ in range(self.world)]
        gv = [torch.empty(V.shape, dtype=torch.from_numpy(V).dtype) for _ in range(self.world)]
        dist.all_gather(gu, torch.from_numpy(U), group=self.group)
        dist.all_gather(gv, torch.from_numpy(V), group=self.group)
        Uc, Vc = U.copy(), V.copy()
        for r in range(self.world):
            m = self.mask[r]
            Uc[m] = gu[r].numpy()[m]
            Vc[m] = gv[r].numpy()[m]
        E._check(lib.ekf_shard_operands(h, Uc.ctypes.data_as(ctypes.c_void_p), Vc.ctypes.data_as(ctypes.c_void_p), 1),
                 "ekf_shard_operands")
        if out.count(-1):   # new landmarks: their rows' columns from every rank
            pr = np.empty(self.pwords)
            E._check(lib.ekf_shard_patch(h, E._dp(pr), 0), "ekf_shard_patch")
            gp = [torch.empty(pr.shape, dtype=torch.float64) for _ in range(self.world)]
            dist.all_gather(gp, torch.from_numpy(pr), group=self.group)
            pc = pr.copy()
            for r in range(self.world):
                pc[self.pmask[r]] = gp[r].numpy()[self.pmask[r]]
            E._check(lib.ekf_shard_patch(h, E._dp(pc), 1), "ekf_shard_patch")
        E._check(lib.ekf_shard_commit(h), "ekf_shard_commit")
        return out

    def status(self) -> int:
        st = ctypes.c_int32()
        E._check(self.lib.ekf_shard_status(self.h, ctypes.byref(st)), "ekf_shard_status")
        return st.value

    def download_state(self):
        """(P, y, saved, pose) of this context: the owned rows / entries, the robot block and the pose
        are the instance's; the other rows are not maintained here."""
        return self.ens.download_state(0)

    def owned_index(self) -> np.ndarray:
        """State indices of the owned landmarks' rows (3 + 2a … 3 + 2b − 1)."""
        return np.arange(3 + 2 * self.a, 3 + 2 * self.b)

    def close(self):
        self.ens.close()
