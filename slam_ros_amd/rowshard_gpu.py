"""One EKF instance with its landmark block partitioned over ranks.

Each rank holds a partitioned context (include/slam_ekf.h ekf_shard_create): it stores the packed
tiles of its tile rows only — a contiguous slice of the packed block balanced by tile count, ≈1/world
of P — while everything of size O(n) (robot strip, mean, every landmark's scan state and diagonal
block, the downdate operand rows) is replicated and evolves identically on every rank. Per scan
(Robot::localize, Robot.cpp:126-904, the sequential association):

  ekf_shard_begin           predict (Robot.cpp:130-286); the rank's diagonal blocks into buf
  SUM buf                   every landmark's diagonal block (one [N][4] all-reduce per scan)
  per line i (Robot.cpp:298-641):
    ekf_shard_line          gate of every landmark — every rank finds the same first passing one —,
                            the winner's gain package, the rank's blocks of the winner's column
    SUM buf                 the winner's column (one [N][4] all-reduce per line)
    ekf_shard_apply         gain rows of every landmark (Robot.cpp:522-602), robot update
  ekf_shard_end             augmentation (Robot.cpp:776-866), the reset (Robot.cpp:893-904), commit;
                            the step joins the deferred flush, which rewrites the rank's tiles only

Every rank fills only the blocks its tiles hold and zeros elsewhere, so the sums are exact and every
rank ends up with the same values; the library's phases are asynchronous on the torch stream the
context is bound to, so a scan has no host round trip until ekf_shard_end. The buffer is a device
tensor: with the nccl backend (RCCL over xGMI on MI355X) the all-reduce runs on it directly; gloo
(the CPU rehearsal on one GPU) stages it through host memory.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import ekf as E

LINE_FIELDS = 6   # struct ekf_line: alpha, r, R[4]


class ShardedInstance:
    """One instance over the ranks of the default process group (or `group`)."""

    def __init__(self, capacity: int, precision: int = E.PREC_F32, max_lines: int = 8,
                 flush_interval: int = 4, r_mode: int = E.R_INTENDED, group=None, device: int | None = None,
                 speculate: bool = True, options: dict | None = None, native: bool = False):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.N = capacity
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        torch.cuda.set_device(dev)
        self.ens = E.Ensemble(capacity, 1, precision, max_lines=max_lines, flush_interval=flush_interval,
                              r_mode=r_mode, device=dev.index, shard=(self.rank, self.world), options=options or {})
        self.lib = E.load_library()
        self.h = self.ens.handle
        self.max_lines = max_lines
        # the library's phases and torch's work (the all-reduce, host staging) on one dedicated stream:
        # the exchange buffer's writes, the sum and the reads are ordered on one queue (torch's
        # default stream has handle 0, which the C-ABI reads as "the context's own stream"). The
        # caller's current stream is left alone: every torch operation here runs inside
        # `with torch.cuda.stream(self.stream)`.
        self.stream = torch.cuda.Stream(dev)
        self.ens.set_stream(self.stream.cuda_stream)
        self.words = int(self.lib.ekf_shard_buffer_words(self.h))
        self.speculate = speculate
        self.swords = int(self.lib.ekf_shard_spec_buffer_words(self.h))
        with torch.cuda.stream(self.stream):
            # + one word: the number of ranks whose phase failed, summed with every exchange. The
            # flag words stay zero while no phase fails (a sum of zeros), so they are written only
            # after a failure (self._dirty). The agreement pair [failure flag, stopping line] is the
            # columns' flag word and the word after it: the columns' sum leaves their flag in place
            # and ekf_shard_run writes its stopping line next to it, with no copy in between.
            self.buf = torch.zeros(self.words + 1, dtype=torch.float64, device=dev)
            self._cols = torch.zeros(self.swords + 2, dtype=torch.float64, device=dev)
            self.cols = self._cols[: self.swords + 1]
            self.agree = self._cols[self.swords:]
        self._dirty = False
        self.spec_runs = []   # per scan: the line the speculative run stopped at (L: all lines)
        self.host_coll = dist.get_backend(group) != "nccl"
        r0, r1 = ctypes.c_int32(), ctypes.c_int32()
        E._check(self.lib.ekf_shard_tiles(self.h, ctypes.byref(r0), ctypes.byref(r1)), "ekf_shard_tiles")
        self.tile_rows = (r0.value, r1.value)
        self._res = (E.EkfResult * 1)()
        # native: the whole scan in one library call (ekf_shard_localize) on the library's own RCCL
        # communicator; rank 0's id reaches the others through the process group (host objects)
        self.native = native
        if native:
            if not speculate:
                E._check(self.lib.ekf_set_option(self.h, E.OPT_SPECULATE, 0), "ekf_set_option")
            uid = (ctypes.c_ubyte * 128)()
            if self.rank == 0:
                E._check(self.lib.ekf_rccl_unique_id(uid), "ekf_rccl_unique_id")
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            uid = (ctypes.c_ubyte * 128).from_buffer_copy(box[0])
            E._check(self.lib.ekf_shard_attach_rccl(self.h, uid, self.rank, self.world), "ekf_shard_attach_rccl")

    def init_lowrank(self, diag, U, y, saved, pose):
        self.ens.init_lowrank(0, diag, U, y, saved, pose)

    def upload_state(self, P, y, saved, pose):
        self.ens.upload_state(0, P, y, saved, pose)

    def _sum(self, failed: bool, buf=None):
        """The exchange (on self.stream), carrying this rank's failure flag in the last word."""
        buf = self.buf if buf is None else buf
        if failed:
            buf[-1].fill_(1.0)
            self._dirty = True
        if self.host_coll:
            t = buf.cpu()
            dist.all_reduce(t, group=self.group)
            buf.copy_(t)
        else:
            dist.all_reduce(buf, group=self.group)

    def localize(self, lines, enc) -> list[int]:
        """Robot::localize on the partitioned instance; returns the matched landmark per line."""
        lib, h = self.lib, self.h
        ln = np.ascontiguousarray(np.asarray(lines, dtype=np.float64).reshape(-1, LINE_FIELDS))
        L = ln.shape[0]
        enc = np.ascontiguousarray(np.asarray(enc, dtype=np.float64).reshape(3))
        if self.native:
            E._check(lib.ekf_shard_localize(h, enc.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p),
                                            L, ctypes.byref(self._res)), "ekf_shard_localize")
            return self._finish()
        bp = ctypes.c_void_p(self.buf.data_ptr())
        # A phase that fails on one rank must not leave the others waiting in an exchange: every
        # rank runs the whole exchange sequence, a failed one without further library calls, and
        # the summed flag word of the last exchange tells every rank alike whether to abandon the
        # scan (ekf_shard_abort) and raise.
        err = None
        with torch.cuda.stream(self.stream):
            if self._dirty:   # (a failed scan left nonzero flag words)
                self.buf[-1].fill_(0.0)
                self.agree.fill_(0.0)
                self._dirty = False
            rc = lib.ekf_shard_begin(h, E._dp(enc), ln.ctypes.data_as(ctypes.c_void_p), L, bp)
            err = err or (rc and (rc, "ekf_shard_begin"))
            self._sum(bool(err))
            first, abandon = 0, False
            if self.speculate and L > 0:
                # one exchange of every guessed column, then the lines on cooperating workgroups up
                # to the first wrong guess (ekf_shard_run, stream-ordered; the replicated state
                # makes every rank stop at the same line). A small agreement exchange (max of the failure flag
                # and of the stopping line) keeps the ranks' exchange sequences equal even when
                # one rank's run fails.
                cp_ = ctypes.c_void_p(self.cols.data_ptr())
                if not err:
                    rc = lib.ekf_shard_speculate(h, bp, cp_)
                    err = rc and (rc, "ekf_shard_speculate")
                self._sum(bool(err), self.cols)
                # stream-ordered: the run writes its stopping line into agree[1]; agree[0] is the
                # columns' summed failure flag; one host read after the agreement
                if not err:
                    rc = lib.ekf_shard_run(h, cp_, ctypes.c_void_p(self.agree.data_ptr() + 8))
                    err = rc and (rc, "ekf_shard_run")
                if err:
                    self.agree[0].fill_(1.0)
                    self.agree[1].fill_(float(L))
                    self._dirty = True
                if self.host_coll:
                    t = self.agree.cpu()
                    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                    self.agree.copy_(t)
                else:
                    dist.all_reduce(self.agree, op=dist.ReduceOp.MAX, group=self.group)
                ag = self.agree.cpu()
                # (a stopping line past L: the run's workgroups timed out on some rank)
                abandon = bool(ag[0] > 0) or int(ag[1]) > L
                first = L if abandon else int(ag[1])
                if not abandon:
                    rc = lib.ekf_shard_resume(h, first)
                    err = err or (rc and (rc, "ekf_shard_resume"))
                self.spec_runs.append(first)
            for i in range(first, L):
                if not err:
                    rc = lib.ekf_shard_line(h, i, bp)
                    err = rc and (rc, "ekf_shard_line")
                self._sum(bool(err))
                if not err:
                    rc = lib.ekf_shard_apply(h, i, bp)
                    err = rc and (rc, "ekf_shard_apply")
            if first < L:
                # the last line's apply ran after its exchange: one more word, the MAX over the ranks
                # of the summed flags and of every rank's failure since, so that a rank whose apply
                # failed does not abandon the scan alone while its peers commit it
                fw = self.buf[self.words:self.words + 1]
                if err:
                    fw.fill_(1.0)
                    self._dirty = True
                if self.host_coll:
                    t = fw.cpu()
                    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                    fw.copy_(t)
                else:
                    dist.all_reduce(fw, op=dist.ReduceOp.MAX, group=self.group)
            if first < L or not (self.speculate and L > 0):
                # the last exchange was a per-line (or begin's) sum: its flag word
                failed = float(self.buf[self.words].item())
            else:
                # every line on the speculative run: the agreement carried every failure flag
                failed = float(ag[0]) if ag[0] > 0 else 0.0
        if abandon and failed == 0:
            failed = 1.0
        if failed > 0:
            self._dirty = True
            lib.ekf_shard_abort(h)
            rc, what = err if err else (0, "a peer rank's phase")
            raise E.EkfError(f"{what} failed on {int(failed)} of {self.world} ranks (rc {rc}); scan abandoned")
        E._check(lib.ekf_shard_end(h, ctypes.byref(self._res)), "ekf_shard_end")
        return self._finish()

    def _finish(self) -> list[int]:
        r = self._res[0]
        self.last = dict(matches=r.matches, new_landmarks=r.new_landmarks, saved=r.saved, reset=r.reset,
                         status=r.status, pose=np.array(r.pose[:]))
        return list(r.match[: r.nlines])

    def status(self) -> int:
        return self.last["status"]

    def download_state(self):
        """(P, y, saved, pose): the robot rows, mean, pose and savedLineCount of the instance, and the
        landmark-block entries of this rank's tiles (zero elsewhere: the ranks' blocks sum to P)."""
        return self.ens.download_state(0)

    def landmark_block_bytes(self) -> int:
        return self.ens.landmark_block_bytes()

    def close(self):
        self.ens.close()
