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
_OMP_PATH = os.path.join(_HERE, "libekf_oracle_omp.so")   # same source, -fopenmp (B1 baseline)
_libs = {}

FAITHFUL, FAST = 0, 1
R_INTENDED, R_AS_WRITTEN = 0, 1


PRED_GATE, PRED_CANCEL, PRED_RANGE = 1, 2, 4   # oracle_pred_flags bits (ekf_oracle.h)


class OracleLine(ctypes.Structure):
    _fields_ = [("alpha", ctypes.c_double), ("r", ctypes.c_double), ("R", ctypes.c_double * 4)]


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(omp: bool = False):
    """The restatement (single-threaded), or its OpenMP build (bit-identical, all host cores;
    OMP_NUM_THREADS sets the team) with omp=True."""
    if omp not in _libs:
        path = _OMP_PATH if omp else _LIB_PATH
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
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
        L.oracle_threads.restype = i
        L.oracle_threads.argtypes = []
        L.oracle_gate_margin.restype = d
        L.oracle_gate_margin.argtypes = [vp]
        L.oracle_set_pred.argtypes = [vp, d, d]
        L.oracle_pred_flags.restype = i
        L.oracle_pred_flags.argtypes = [vp]
        _libs[omp] = L
    return _libs[omp]


def threads(omp: bool = True) -> int:
    return lib(omp).oracle_threads()


def host_cpus() -> dict:
    """What the CPU baseline may use on this host: logical CPUs, the affinity mask, the cgroup CPU
    quota and OMP_NUM_THREADS (the OpenMP build uses the latter; on the GPU pool it is set to the
    process's share of the host, which the pool also enforces)."""
    import os
    out = {"logical_cpus": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        out["affinity_cpus"] = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                out["cgroup_cpu_max"] = f.read().strip()
            break
        except OSError:
            continue
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    out["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return out


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
                 mode: int = FAST, r_mode: int = R_INTENDED, omp: bool = False):
        self._lib = lib(omp)
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

    @property
    def gate_margin(self) -> float:
        """min |sqrt(|d²|) − 0.4| over the candidates the last localize evaluated."""
        return float(self._lib.oracle_gate_margin(self._h))

    def set_prediction(self, eta: float, cancel: float = 16.0):
        """Test instrumentation: predict, from this restatement's own fp64 state, the decisions a
        stored state within relative precision eta cannot resolve (oracle_set_pred)."""
        self._lib.oracle_set_pred(self._h, float(eta), float(cancel))

    @property
    def pred_flags(self) -> int:
        """PRED_* bits of the last localize (0: every decision resolved at the set precision)."""
        return int(self._lib.oracle_pred_flags(self._h))

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


# ---- Robot::getEllipse (Robot.cpp:73-124) ---------------------------------------------------
# GSL is not vendored (system libgsl, version unpinned: slam_ros/CMakeLists.txt:43-51). This
# restates, in Python floats (IEEE double, one operation per statement), the published GSL
# algorithm the reference calls: gsl_eigen_nonsymmv (gsl/eigen/nonsymmv.c; default workspace
# parameters: Schur vectors on, no balancing) on the 2x2 block, gsl_eigen_nonsymmv_sort with
# GSL_EIGEN_SORT_ABS_ASC, then axii[i] = 2·sqrt(5.991·|Re λ_i|) and
# angle = atan2(Re z1, Re z2) of the eigenvector of the larger |λ| (Robot.cpp:100-112).
_DBL_EPS = 2.220446049250313e-16
_DBL_MIN = 2.2250738585072014e-308


def _gsl_sign(x):
    return 1.0 if x >= 0.0 else -1.0


def _gsl_hypot(x, y):
    xa, ya = abs(x), abs(y)
    mn, mx = (xa, ya) if xa < ya else (ya, xa)
    if mn == 0.0:
        return mx
    u = mn / mx
    return mx * float(np.sqrt(1.0 + u * u))


def _dnrm2(xs):
    # gslcblas source_nrm2_r.h: scaled sum of squares
    scale, ssq = 0.0, 1.0
    for x in xs:
        if x != 0.0:
            ax = abs(x)
            if scale < ax:
                ssq = 1.0 + ssq * (scale / ax) * (scale / ax)
                scale = ax
            else:
                ssq += (ax / scale) * (ax / scale)
    return scale * float(np.sqrt(ssq))


def _francis_standardize(a, b, c, d):
    """gsl/eigen/francis.c francis_schur_standardize (LAPACK dlanv2): Schur form of a 2x2 block
    [a b; c d] = Z [a' b'; c' d'] Zᵀ, Z = [[cs, -sn], [sn, cs]]."""
    sq = lambda v: float(np.sqrt(v))
    if c == 0.0:
        cs, sn = 1.0, 0.0
    elif b == 0.0:
        cs, sn = 0.0, 1.0
        a, d = d, a
        b, c = -c, 0.0
    elif (a - d) == 0.0 and _gsl_sign(b) != _gsl_sign(c):
        cs, sn = 1.0, 0.0
    else:
        tmp = a - d
        p = 0.5 * tmp
        bcmax = max(abs(b), abs(c))
        bcmis = min(abs(b), abs(c)) * _gsl_sign(b) * _gsl_sign(c)
        scale = max(abs(p), bcmax)
        z = (p / scale) * p + (bcmax / scale) * bcmis
        if z >= 4.0 * _DBL_EPS:
            z = p + _gsl_sign(p) * abs(sq(scale) * sq(z))
            a = d + z
            d -= (bcmax / z) * bcmis
            tau = _gsl_hypot(c, z)
            cs = z / tau
            sn = c / tau
            b -= c
            c = 0.0
        else:
            sigma = b + c
            tau = _gsl_hypot(sigma, tmp)
            cs = sq(0.5 * (1.0 + abs(sigma) / tau))
            sn = -(p / (tau * cs)) * _gsl_sign(sigma)
            aa, bb = a * cs + b * sn, -a * sn + b * cs
            cc, dd = c * cs + d * sn, -c * sn + d * cs
            a, b = aa * cs + cc * sn, bb * cs + dd * sn
            c, d = -aa * sn + cc * cs, -bb * sn + dd * cs
            tmp = 0.5 * (a + d)
            a = d = tmp
            if c != 0.0:
                if b != 0.0:
                    if _gsl_sign(b) == _gsl_sign(c):
                        sab, sac = sq(abs(b)), sq(abs(c))
                        p = _gsl_sign(c) * abs(sab * sac)
                        tau = 1.0 / sq(abs(b + c))
                        a, d = tmp + p, tmp - p
                        b -= c
                        c = 0.0
                        cs1, sn1 = sab * tau, sac * tau
                        tmp = cs * cs1 - sn * sn1
                        sn = cs * sn1 + sn * cs1
                        cs = tmp
                else:
                    b, c = -c, 0.0
                    cs, sn = -sn, cs
    return a, b, c, d, cs, sn


def gsl_ellipse(P22):
    """(ok, [axii0, axii1], angle) as float32 values, for P22 = (P00, P01, P10, P11)."""
    P00, P01, P10, P11 = (float(v) for v in np.asarray(P22, dtype=np.float64).reshape(4))
    if not all(np.isfinite([P00, P01, P10, P11])):
        return False, None, None
    a, b, c, d, cs, sn = _francis_standardize(P00, P01, P10, P11)
    if c != 0.0:
        return False, None, None      # complex pair (not from a symmetric covariance)
    # right eigenvectors of [a b; 0 d]: x = (1, 0) for a; x = (-b / (a - d), 1) for d
    # (gsl_schur_solve_equation, denominator floored at smin), v = Z x (gslcblas dgemv: y = Z[:,1]
    # then y += Z[:,0]·x0), max-norm scaling, then unit 2-norm (nonsymmv_normalize_eigenvectors)
    smin = max(_DBL_EPS * abs(d), _DBL_MIN * (2 / _DBL_EPS))
    den = a - d
    if abs(den) < smin:
        den = smin
    x0 = -b / den
    vecs = [[cs, sn], [-sn + x0 * cs, cs + x0 * sn]]
    for v in vecs:
        emax = max(abs(v[0]), abs(v[1]))
        if emax > 0.0:
            r = 1.0 / emax
            v[0] *= r
            v[1] *= r
        nr = _dnrm2(v)
        if nr > 0.0:
            s = 1.0 / nr
            v[0] *= s
            v[1] *= s
    lam = [a, d]
    order = [1, 0] if abs(lam[1]) < abs(lam[0]) else [0, 1]
    axii = [float(np.float32(2.0) * np.float32(np.sqrt(5.991 * abs(lam[i])))) for i in order]
    big = vecs[order[1]]
    angle = float(np.float32(np.arctan2(big[0], big[1])))
    return True, axii, angle
