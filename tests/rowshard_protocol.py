"""TEST INFRASTRUCTURE (not product code; only tests/test_rowshard_gloo.py imports it). One EKF
instance row-sharded across ranks: the protocol for
N ≫ 4096, where a single landmark block outgrows what one GPU should rewrite per scan, as an
executable specification on host arrays. The product form is slam_ros_amd/rowshard_gpu.py over
the library's ekf_shard_* kernels.

Partition: rank r owns the landmarks [a_r, b_r) (contiguous, sizes differing by at most one,
`dist.shard`), i.e. the full rows 3+2a_r … 3+2b_r−1 of P (all n columns). Every rank keeps a
replica of the robot strip P[0:3, :] (3×n), the state vector y, the pose and savedLineCount;
they evolve identically on every rank because every input to them is either replicated or
exchanged. Per scan (Robot::localize, Robot.cpp:126-904):

  predict (Robot.cpp:130-258)   local: the strip (replicated) and the robot columns of the owned
                                rows (P_pre differs from P only in rows/columns 0..2)
  per line i (Robot.cpp:298)    local gating of the owned, not yet matched landmarks against the
                                current P (Robot.cpp:313-498: 5×5 sub-block = strip + the owned
                                2×2 diagonal block), then ONE all-reduce(min) of
                                (first passing landmark, first singular S) — the reference takes
                                the FIRST landmark in index order that passes the gate, so the
                                global winner is the minimum over ranks
  match j (Robot.cpp:500-641)   the owner of j broadcasts (S, S⁻¹, innovation) — 10 doubles;
                                every rank forms its rows of W = P_pre·Hᵀ (Robot.cpp:522) and
                                all-gathers W (n×2 fp64 — the sharded step's one real exchange);
                                then K = W·S⁻¹, K·S (replicated, n×2) and the downdate
                                P_pre −= (K·S)·Kᵀ (Robot.cpp:556-575) of the OWNED rows and the
                                strip, the state update y += K·v (Robot.cpp:579-602) replicated
  augmentation (Robot.cpp:776-866)  the new rows come from the strip (replicated): the owner of
                                landmark s stores rows l0, l0+1; every rank writes columns l0, l0+1
                                of its owned rows and of the strip
  reset (Robot.cpp:893-904)     local

Exchanges per scan: L all-reduces of two integers, m broadcasts of 10 doubles and m all-gathers
of n×2 doubles (≈1 MB at N = 4096, m = 8); the landmark rows never move.

This module is the protocol's executable specification on host arrays (float64 numpy, the
operation order of the CPU restatement's fast mode, oracle/ekf_oracle.c, so that the sharded run
is bit-identical to the single-process one: tests/test_rowshard_gloo.py, world_size 2 over
gloo). On MI355X ranks the owned rows live in HBM in the packed tile layout of one instance and
the local steps are the library's shard phases. It is not on the benchmark path
(the ensemble is).
"""
from __future__ import annotations

import math

import numpy as np

from slam_ros_amd.dist import shard

MAHALANOBIS = 0.4          # Robot.h:15
ENCODERNOISE = 0.024       # Robot.h:17
R_INTENDED, R_AS_WRITTEN = 0, 1


def normalize_radian(rad: float) -> float:
    """Robot.cpp:62-71 (one fold, if / else-if)."""
    if rad > math.pi:
        rad = rad - (2.0 * math.pi + math.floor(rad / (2.0 * math.pi)) * 2.0 * math.pi)
    elif rad < -math.pi:
        rad = rad + (2.0 * math.pi + math.floor(abs(rad) / (2.0 * math.pi)) * 2.0 * math.pi)
    return rad


def lu_invert2(S):
    """gsl_linalg_LU_decomp + LU_invert on 2×2 (Robot.cpp:443-457): (singular, S⁻¹); a singular
    U leaves S⁻¹ at zero (GSL_EDOM, output untouched)."""
    a0, a1, a2, a3 = S
    p0, p1 = 0, 1
    if abs(a2) > abs(a0):
        a0, a1, a2, a3 = a2, a3, a0, a1
        p0, p1 = 1, 0
    if a0 != 0.0:
        l = a2 / a0
        a2 = l
        a3 -= l * a1
    if a0 == 0.0 or a3 == 0.0:
        return True, [0.0, 0.0, 0.0, 0.0]
    out = [0.0] * 4
    for c in range(2):
        b0 = 1.0 if p0 == c else 0.0
        b1 = 1.0 if p1 == c else 0.0
        b1 = b1 - a2 * b0
        x1 = b1 / a3
        x0 = (b0 - a1 * x1) / a0
        out[c] = x0
        out[2 + c] = x1
    return False, out


def _mm_n2x22(A, B):
    """(n×2)·(2×2) as gslcblas NN (C = 0, then per k the rows with A[:, k] ≠ 0 accumulate)."""
    C = np.zeros((A.shape[0], 2))
    for k in range(2):
        nz = A[:, k] != 0.0
        for j in range(2):
            C[nz, j] += A[nz, k] * B[2 * k + j]
    return C


class RowShardedRobot:
    """`class Robot` (Robot.h:21-77) with its P row-sharded over the ranks of `dist` (an
    initialised torch.distributed group; gloo on CPU tensors here)."""

    def __init__(self, capacity: int, dist, x=0.0, y=0.0, theta=0.0, r_mode=R_INTENDED,
                 reset_margin=10):
        import torch
        self.torch, self.dist = torch, dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.N = capacity
        self.n = 3 + 2 * capacity
        self.r_mode, self.reset_margin = r_mode, reset_margin
        self.lm0, cnt = shard(capacity, self.world, self.rank)
        self.lm1 = self.lm0 + cnt
        self.r0, self.r1 = 3 + 2 * self.lm0, 3 + 2 * self.lm1
        self.maxrows = 2 * shard(capacity, self.world, 0)[1]
        n = self.n
        self.strip = np.zeros((3, n))               # P[0:3, :], replicated
        self.rows = np.zeros((self.r1 - self.r0, n))  # P[r0:r1, :], owned
        self.y = np.zeros(n)
        self.strip[0, 0] = self.strip[1, 1] = 0.05    # Robot::Robot, Robot.cpp:20-35
        self.pose = [x, y, theta]
        self.saved = 0
        self.status = 0

    # ---- state transfer -------------------------------------------------------------------
    def owner(self, landmark: int) -> int:
        for r in range(self.world):
            a, c = shard(self.N, self.world, r)
            if a <= landmark < a + c:
                return r
        raise ValueError(landmark)

    def set_state(self, P, y, saved, pose):
        self.strip[:] = P[:3]
        self.rows[:] = P[self.r0:self.r1]
        self.y[:] = y
        self.saved = int(saved)
        self.pose = [float(v) for v in pose]

    def gather_P(self):
        """Full n×n P on every rank (tests): strip + every rank's rows."""
        t = self.torch
        pad = t.zeros((self.maxrows, self.n), dtype=t.float64)
        pad[: self.rows.shape[0]] = t.from_numpy(self.rows)
        parts = [t.zeros_like(pad) for _ in range(self.world)]
        self.dist.all_gather(parts, pad)
        P = np.zeros((self.n, self.n))
        P[:3] = self.strip
        for r in range(self.world):
            a, c = shard(self.N, self.world, r)
            P[3 + 2 * a: 3 + 2 * (a + c)] = parts[r][: 2 * c].numpy()
        return P

    # ---- the exchanges ----------------------------------------------------------------------
    def _allreduce_min(self, vals):
        t = self.torch.tensor(vals, dtype=self.torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return [int(v) for v in t.tolist()]

    def _broadcast(self, vals, src):
        t = self.torch.tensor(vals if vals is not None else [0.0] * 10, dtype=self.torch.float64)
        self.dist.broadcast(t, src=src)
        return t.tolist()

    def _allgather_W(self, W_own):
        """W rows of every rank → the full n×2 W (rows 0..2 are computed everywhere)."""
        t = self.torch
        pad = t.zeros((self.maxrows, 2), dtype=t.float64)
        pad[: W_own.shape[0]] = t.from_numpy(W_own)
        parts = [t.zeros_like(pad) for _ in range(self.world)]
        self.dist.all_gather(parts, pad)
        W = np.zeros((self.n, 2))
        for r in range(self.world):
            a, c = shard(self.N, self.world, r)
            W[3 + 2 * a: 3 + 2 * (a + c)] = parts[r][: 2 * c].numpy()
        return W

    # ---- P_pre entries ----------------------------------------------------------------------
    def _p(self, i, j):
        if i < 3:
            return self.strip[i, j]
        return self.rows[i - self.r0, j]

    # ---- Robot::localize ----------------------------------------------------------------------
    def localize(self, lines, enc):
        """lines: (L, 6) {alpha, r, R00, R01, R10, R11}; enc: encoder pose. Returns the match
        list (Robot.cpp:126-904, the restatement's fast mode)."""
        n, N = self.n, self.N
        y = self.y
        strip, rows = self.strip, self.rows
        self.status = 0
        L = len(lines)
        # motion model (Robot.cpp:130-148)
        x_t0 = list(self.pose)
        u2 = x_t0[2] - enc[2]
        dX = x_t0[0] - enc[0]
        dY = x_t0[1] - enc[1]
        u0 = math.sqrt(dX * dX + dY * dY)
        x_pre = [x_t0[0] + u0 * math.cos(x_t0[2] + u2 / 2.0),
                 x_t0[1] + u0 * math.sin(x_t0[2] + u2 / 2.0), x_t0[2] + u2]
        c = u2 / 2.0 + x_t0[2]
        F3 = [1.0, 0.0, -u0 * math.sin(c), 0.0, 1.0, u0 * math.cos(c), 0.0, 0.0, 1.0]
        Fu3 = [math.cos(c), 0.0, -u0 * math.sin(c) / 2.0, math.sin(c), 1.0, u0 * math.cos(c) / 2.0,
               0.0, 0.0, 1.0]
        qs = (-1.0 / (1 + abs(u0)) + 1)
        Q = [ENCODERNOISE * qs, 0.0, 0.0, 0.0, 2 * ENCODERNOISE * qs, 0.0, 0.0, 0.0, ENCODERNOISE * qs]
        self._predict(F3, Fu3, Q)

        matches = 0
        matched = []
        extra = []
        match_out = [-1] * L
        for i in range(L):
            ln = lines[i]
            if self.r_mode == R_AS_WRITTEN:
                R = [0.0] * 4
                if i < 4:
                    R[i] = float(ln[5])
            else:
                R = [float(v) for v in ln[2:6]]
            s = self.saved
            if s == 0:
                extra.append(i)
                continue
            # local gating over the owned landmarks (first passing in index order)
            first_pass, first_sing = s, s
            winner = None
            for j in range(max(self.lm0, 0), min(self.lm1, s)):
                if j in matched:
                    continue
                ev = self._gate(j, ln, R, x_pre)
                if ev[0] and first_sing == s:
                    first_sing = j
                if ev[1]:
                    first_pass = j
                    winner = ev[2]
                    break
            jstar, jsing = self._allreduce_min([first_pass, first_sing])
            if jsing < s and jsing <= jstar:
                self.status |= 1
            if jstar >= s:
                extra.append(i)
                continue
            pkt = self._broadcast(winner if jstar == first_pass and winner is not None else None,
                                  self.owner(jstar))
            S, Sinv, z = pkt[0:4], pkt[4:8], pkt[8:10]
            matched.append(jstar)
            matches += 1
            match_out[i] = jstar
            self._update(jstar, S, Sinv, z, x_pre)
            x_pre = [y[0], y[1], y[2]]
        if L == 0 or matches == 0:
            y[0], y[1], y[2] = x_pre
            self.pose = [y[0], y[1], normalize_radian(y[2])]
        for i in extra:
            self._augment(lines[i])
        if self.saved > N - self.reset_margin:
            self.saved = 0
            y[3:] = 0.0
            strip[:, 3:] = 0.0
            rows[:] = 0.0
        return match_out

    def _predict(self, F3, Fu3, Q):
        """predict_fast (oracle/ekf_oracle.c): rows 0..2 for columns ≥ 3 and the owned rows'
        columns 0..2 by the 3×3 products, the 3×3 block F·P·Fᵀ + Fu·Q·Fuᵀ."""
        strip, rows = self.strip, self.rows
        P33 = strip[:, :3].copy()
        old = strip[:, 3:].copy()
        for a in range(3):
            s_ = 0.0 + F3[a * 3 + 0] * old[0]
            s_ = s_ + F3[a * 3 + 1] * old[1]
            strip[a, 3:] = s_ + F3[a * 3 + 2] * old[2]
        if rows.shape[0]:
            oc = rows[:, :3].copy()
            for a in range(3):
                s_ = 0.0 + oc[:, 0] * F3[a * 3 + 0]
                s_ = s_ + oc[:, 1] * F3[a * 3 + 1]
                rows[:, a] = s_ + oc[:, 2] * F3[a * 3 + 2]
        FP = [0.0] * 9
        FuQ = [0.0] * 9
        for a in range(3):
            for b in range(3):
                s_, t_ = 0.0, 0.0
                for k in range(3):
                    s_ += F3[a * 3 + k] * P33[k, b]
                    t_ += Fu3[a * 3 + k] * Q[k * 3 + b]
                FP[a * 3 + b] = s_
                FuQ[a * 3 + b] = t_
        for a in range(3):
            for b in range(3):
                s_, t_ = 0.0, 0.0
                for k in range(3):
                    s_ += FP[a * 3 + k] * F3[b * 3 + k]
                    t_ += FuQ[a * 3 + k] * Fu3[b * 3 + k]
                strip[a, b] = s_ + t_

    def _gate(self, j, ln, R, x_pre):
        """Robot.cpp:367-498 for landmark j (owned): (singular, passes, (S, S⁻¹, v))."""
        y = self.y
        l0, l1 = 3 + 2 * j, 4 + 2 * j
        ma, mr = y[l0], y[l1]
        h10, h11 = -math.cos(ma), -math.sin(ma)
        h1l = x_pre[0] * math.sin(ma) - x_pre[1] * math.cos(ma)
        idx = (0, 1, 2, l0, l1)
        hr0 = (0.0, 0.0, -1.0, 1.0, 0.0)
        hr1 = (h10, h11, 0.0, h1l, 1.0)
        hp0, hp1 = [0.0] * 5, [0.0] * 5
        for b in range(5):
            s0, s1 = 0.0, 0.0
            for a in range(5):
                p = self._p(idx[a], idx[b])
                s0 += hr0[a] * p
                s1 += hr1[a] * p
            hp0[b], hp1[b] = s0, s1
        S = [0.0] * 4
        for b in range(5):
            S[0] += hp0[b] * hr0[b]
            S[1] += hp0[b] * hr1[b]
            S[2] += hp1[b] * hr0[b]
            S[3] += hp1[b] * hr1[b]
        for e in range(4):
            S[e] += R[e]
        z = [float(ln[0]), float(ln[1])]
        h = [ma - x_pre[2], mr - (x_pre[0] * math.cos(ma) + x_pre[1] * math.sin(ma))]
        h[0] = normalize_radian(h[0])
        sing, Sinv = lu_invert2(S)
        z[0] -= h[0]
        z[1] -= h[1]
        if abs(z[0] - 2.0 * math.pi) < abs(z[0]):
            z[0] -= 2.0 * math.pi
        elif abs(z[0] + 2.0 * math.pi) < abs(z[0]):
            z[0] += 2.0 * math.pi
        # vᵀ S⁻¹ v as two gslcblas NN products (Robot.cpp:479-486)
        vS = [0.0, 0.0]
        for k in range(2):
            t = z[k]
            if t != 0.0:
                vS[0] += t * Sinv[k * 2 + 0]
                vS[1] += t * Sinv[k * 2 + 1]
        d2 = 0.0
        for k in range(2):
            t = vS[k]
            if t != 0.0:
                d2 += t * z[k]
        passes = not (math.sqrt(abs(d2)) > MAHALANOBIS)
        return sing, passes, S + Sinv + z

    def _update(self, j, S, Sinv, z, x_pre):
        """Robot.cpp:500-602 for the winner j: W rows (owned + strip), all-gather, K, K·S, the
        owned rows' and the strip's downdate, the replicated state update."""
        y, strip, rows = self.y, self.strip, self.rows
        l0, l1 = 3 + 2 * j, 4 + 2 * j
        ma = y[l0]
        h10, h11 = -math.cos(ma), -math.sin(ma)
        h1l = x_pre[0] * math.sin(ma) - x_pre[1] * math.cos(ma)
        W_own = np.zeros((rows.shape[0], 2))
        if rows.shape[0]:
            W_own[:, 0] = -1.0 * rows[:, 2] + 1.0 * rows[:, l0] + 0.0 * rows[:, l1]
            W_own[:, 1] = h10 * rows[:, 0] + h11 * rows[:, 1] + h1l * rows[:, l0] + 1.0 * rows[:, l1]
        W = self._allgather_W(W_own)
        W[:3, 0] = -1.0 * strip[:, 2] + 1.0 * strip[:, l0] + 0.0 * strip[:, l1]
        W[:3, 1] = h10 * strip[:, 0] + h11 * strip[:, 1] + h1l * strip[:, l0] + 1.0 * strip[:, l1]
        K = _mm_n2x22(W, Sinv)
        KS = _mm_n2x22(K, S)
        if rows.shape[0]:
            a0 = KS[self.r0:self.r1, 0:1]
            a1 = KS[self.r0:self.r1, 1:2]
            rows -= (0.0 + a0 * K[None, :, 0]) + a1 * K[None, :, 1]
        strip -= (0.0 + KS[:3, 0:1] * K[None, :, 0]) + KS[:3, 1:2] * K[None, :, 1]
        y[0], y[1], y[2] = x_pre
        y += (0.0 + K[:, 0] * z[0]) + K[:, 1] * z[1]
        y[2] = normalize_radian(y[2])
        self.pose = [y[0], y[1], y[2]]

    def _augment(self, ln):
        """Robot.cpp:776-866 for one extra line: the new rows from the strip."""
        y, strip, rows, n = self.y, self.strip, self.rows, self.n
        s = self.saved
        if 3 + 2 * s + 2 > n:
            self.status |= 2
            return
        alfa = float(ln[0])
        r = float(ln[1]) + (self.pose[0] * math.cos(alfa) + self.pose[1] * math.sin(alfa))
        alfa += self.pose[2]
        Gx = [0.0, 0.0, 1.0, math.cos(alfa), math.sin(alfa), 0.0]
        Gl = [1.0, 0.0, y[1] * math.cos(alfa) - y[0] * math.sin(alfa), 1.0]
        alfa = normalize_radian(alfa)
        y[3 + 2 * s] = alfa
        y[3 + 2 * s + 1] = r
        R = [float(v) for v in ln[2:6]]
        # Gx·P[0:3,0:3] (NN), ·Gxᵀ (NT), Gl·R (NN), ·Glᵀ (NT)
        GxPrr = [0.0] * 6
        for k in range(3):
            for i in range(2):
                t = Gx[i * 3 + k]
                if t != 0.0:
                    for jj in range(3):
                        GxPrr[i * 3 + jj] += t * strip[k, jj]
        Pll = [0.0] * 4
        for i in range(2):
            for jj in range(2):
                t = 0.0
                for k in range(3):
                    t += GxPrr[i * 3 + k] * Gx[jj * 3 + k]
                Pll[i * 2 + jj] += t
        GlR = [0.0] * 4
        for k in range(2):
            for i in range(2):
                t = Gl[i * 2 + k]
                if t != 0.0:
                    for jj in range(2):
                        GlR[i * 2 + jj] += t * R[k * 2 + jj]
        GlRGl = [0.0] * 4
        for i in range(2):
            for jj in range(2):
                t = 0.0
                for k in range(2):
                    t += GlR[i * 2 + k] * Gl[jj * 2 + k]
                GlRGl[i * 2 + jj] += t
        for q in range(4):
            Pll[q] += GlRGl[q]
        l0 = 3 + 2 * s
        # the new rows' entries left of the diagonal block: Gx·P[0:3, 0:l0] (NN, C zeroed)
        new = np.zeros((2, l0))
        for k in range(3):
            for i in range(2):
                t = Gx[i * 3 + k]
                if t != 0.0:
                    new[i] += t * strip[k, :l0]
        if self.r0 <= l0 < self.r1:
            rr = rows[l0 - self.r0: l0 - self.r0 + 2]
            rr[0, l0], rr[0, l0 + 1], rr[1, l0], rr[1, l0 + 1] = Pll
            rr[:, :l0] = new
        # the new columns: owned rows below l0, and the strip
        if rows.shape[0]:
            top = min(self.r1, l0)
            if top > self.r0:
                rows[: top - self.r0, l0] = new[0, self.r0:top]
                rows[: top - self.r0, l0 + 1] = new[1, self.r0:top]
        strip[:, l0] = new[0, :3]
        strip[:, l0 + 1] = new[1, :3]
        self.saved = s + 1
