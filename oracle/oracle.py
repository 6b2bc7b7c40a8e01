"""ctypes wrapper for the CPU restatement in ekf_oracle.c — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It is the parity checker for the HIP path (slam_ros_amd), never a fallback for it.

Mirrors the reference's `class Robot` (slam_ros/Robot.h:21-77): construct with a pose,
call `localize(lines, encoder)` (Robot.cpp:126-904), read `xPos/yPos/thetaPos`, `P_t0`, `y`.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libekf_oracle.so")
_lib = None

FAITHFUL, FAST = 0, 1
R_INTENDED, R_AS_WRITTEN = 0, 1


class OracleLine(ctypes.Structure):
    _fields_ = [("alpha", ctypes.c_double), ("r", ctypes.c_double), ("R", ctypes.c_double * 4)]


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        dp = ctypes.POINTER(ctypes.c_double)
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [i, d, d, d, i, i]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_localize.restype = i
        L.oracle_localize.argtypes = [vp, ctypes.c_void_p, i, dp, ctypes.POINTER(ctypes.c_int)]
        for name in ("oracle_n", "oracle_capacity", "oracle_saved", "oracle_status"):
            getattr(L, name).restype = i
            getattr(L, name).argtypes = [vp]
        L.oracle_pose.argtypes = [vp, dp]
        L.oracle_P.restype = dp
        L.oracle_P.argtypes = [vp]
        L.oracle_y.restype = dp
        L.oracle_y.argtypes = [vp]
        L.oracle_set_state.argtypes = [vp, dp, dp, i, dp]
        L.oracle_dgemm.argtypes = [i, i, i, i, i, d, dp, i, dp, i, d, dp, i]
        L.oracle_lu_invert2.restype = i
        L.oracle_lu_invert2.argtypes = [dp, dp]
        L.oracle_normalize_radian.restype = d
        L.oracle_normalize_radian.argtypes = [d]
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def lines_to_struct(lines) -> ctypes.Array:
    """lines: array-like (L, 6) = [alpha, r, R00, R01, R10, R11] per line."""
    arr = np.ascontiguousarray(np.asarray(lines, dtype=np.float64).reshape(-1, 6))
    out = (OracleLine * max(len(arr), 1))()
    for k, row in enumerate(arr):
        out[k].alpha = row[0]
        out[k].r = row[1]
        for q in range(4):
            out[k].R[q] = row[2 + q]
    return out, len(arr)


class OracleRobot:
    """CPU restatement of `Robot` (Robot.h:21-77) with runtime capacity N."""

    def __init__(self, capacity: int, x: float = 0.0, y: float = 0.0, theta: float = 0.0,
                 mode: int = FAST, r_mode: int = R_INTENDED):
        self._lib = lib()
        self._h = self._lib.oracle_create(int(capacity), x, y, theta, int(mode), int(r_mode))
        if not self._h:
            raise MemoryError("oracle_create failed")
        self.capacity = int(capacity)
        self.n = self._lib.oracle_n(self._h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.oracle_destroy(h)
            self._h = None

    def localize(self, lines, encoder) -> list:
        """Robot::localize(lines, rot, encoder) — returns per-line matched index or -1."""
        arr, L = lines_to_struct(lines)
        enc = np.ascontiguousarray(np.asarray(encoder, dtype=np.float64))
        match = (ctypes.c_int * max(L, 1))()
        self._lib.oracle_localize(self._h, ctypes.byref(arr), L, _dp(enc), match)
        return [match[k] for k in range(L)]

    @property
    def P_t0(self) -> np.ndarray:
        p = self._lib.oracle_P(self._h)
        return np.ctypeslib.as_array(p, shape=(self.n, self.n))

    @property
    def y(self) -> np.ndarray:
        return np.ctypeslib.as_array(self._lib.oracle_y(self._h), shape=(self.n,))

    @property
    def pose(self) -> np.ndarray:
        out = np.zeros(3)
        self._lib.oracle_pose(self._h, _dp(out))
        return out

    @property
    def xPos(self) -> float:
        return float(self.pose[0])

    @property
    def yPos(self) -> float:
        return float(self.pose[1])

    @property
    def thetaPos(self) -> float:
        return float(self.pose[2])

    @property
    def savedLineCount(self) -> int:
        return self._lib.oracle_saved(self._h)

    @property
    def status(self) -> int:
        return self._lib.oracle_status(self._h)

    def set_state(self, P=None, y=None, saved: int = 0, pose=None):
        Pc = None if P is None else np.ascontiguousarray(P, dtype=np.float64)
        yc = None if y is None else np.ascontiguousarray(y, dtype=np.float64)
        pc = None if pose is None else np.ascontiguousarray(pose, dtype=np.float64)
        nul = ctypes.POINTER(ctypes.c_double)()
        self._lib.oracle_set_state(self._h, nul if Pc is None else _dp(Pc),
                                   nul if yc is None else _dp(yc), int(saved),
                                   nul if pc is None else _dp(pc))


def dgemm(transA: bool, transB: bool, A: np.ndarray, B: np.ndarray, alpha=1.0, beta=0.0,
          C: np.ndarray | None = None) -> np.ndarray:
    A = np.ascontiguousarray(A, dtype=np.float64)
    B = np.ascontiguousarray(B, dtype=np.float64)
    M = A.shape[1] if transA else A.shape[0]
    K = A.shape[0] if transA else A.shape[1]
    N = B.shape[0] if transB else B.shape[1]
    C = np.zeros((M, N)) if C is None else np.ascontiguousarray(C, dtype=np.float64).copy()
    lib().oracle_dgemm(int(transA), int(transB), M, N, K, alpha, _dp(A), A.shape[1], _dp(B),
                       B.shape[1], beta, _dp(C), N)
    return C


def lu_invert2(S: np.ndarray):
    S = np.ascontiguousarray(S, dtype=np.float64).reshape(4)
    out = np.zeros(4)
    rc = lib().oracle_lu_invert2(_dp(S), _dp(out))
    return out.reshape(2, 2), rc


def normalize_radian(x: float) -> float:
    return lib().oracle_normalize_radian(float(x))
