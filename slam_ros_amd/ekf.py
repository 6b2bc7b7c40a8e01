"""Host-side mirror of the reference `class Robot` over the C-ABI of libslam_ekf.so.

`Robot` mirrors slam_ros/Robot.h:21-77 (constructor pose, `localize(lines, rot, encoder)`,
`getEllipse()`, `xPos/yPos/thetaPos`, `P_t0`, `lineIntervals`) and adds the two halves
`predict(encoder)` / `update(lines)`. `Ensemble` drives E independent
instances per call — the benchmark and multi-GPU path.

All arithmetic runs in the HIP kernels of libslam_ekf.so (gfx950). There is no CPU
fallback: if the library or a GPU is missing, constructing a context raises.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

from . import build as _build

EKF_MAX_LINES = 64
PREC_F64, PREC_F32, PREC_F16 = 0, 1, 2
R_INTENDED, R_AS_WRITTEN = 0, 1
ARITH_EXACT, ARITH_BF16X6, ARITH_F16X3 = 0, 1, 2   # fp32 flush arithmetic (slam_ekf.h EKF_ARITH_*)
ST_SINGULAR_S, ST_CAPACITY, ST_NONSYM, ST_SYNC_TIMEOUT, ST_RANGE, ST_PRECISION = 1, 2, 4, 8, 16, 32
EXP_AUTO = -1000
# per-context options (slam_ekf.h EKF_OPT_*, ekf_set_option)
OPT_SPECULATE, OPT_SPIN_LOG2, OPT_FLUSH_FORM, OPT_FLUSH_BLOCKS_PER_CU = 1, 2, 3, 4
OPT_MFMA_REPLAY, OPT_SCAN_STAMPS, OPT_TEST_DROP_WG, OPT_TEST_VERDICT_TIMEOUT = 5, 6, 7, 8
OPT_ACTIVE_FLUSH, OPT_SCAN_THREADS = 9, 10
OPTIONS = {"speculate": OPT_SPECULATE, "spin_log2": OPT_SPIN_LOG2, "flush_form": OPT_FLUSH_FORM,
           "flush_blocks_per_cu": OPT_FLUSH_BLOCKS_PER_CU, "mfma_replay": OPT_MFMA_REPLAY,
           "scan_stamps": OPT_SCAN_STAMPS, "test_drop_wg": OPT_TEST_DROP_WG,
           "test_verdict_timeout": OPT_TEST_VERDICT_TIMEOUT, "active_flush": OPT_ACTIVE_FLUSH,
           "scan_threads": OPT_SCAN_THREADS}

LIB_PATH = _build.LIB_PATH

# symbols declared by include/slam_ekf.h (checked by tests/test_abi.py)
EXPORTED = [
    "ekf_config_init", "ekf_strerror", "ekf_abi_version", "ekf_create", "ekf_destroy",
    "ekf_set_stream", "ekf_sync", "ekf_set_option", "ekf_get_option", "ekf_reset_instance", "ekf_localize", "ekf_localize_device",
    "ekf_predict", "ekf_update", "ekf_read_results", "ekf_upload_state", "ekf_download_state",
    "ekf_init_lowrank", "ekf_storage_exponent", "ekf_rescale", "ekf_get_pose_cov", "ekf_get_ellipse", "ekf_ellipse_of_block",
    "ekf_landmark_block_bytes",
    "ekf_state_dim", "ekf_profile_enable", "ekf_profile_read", "ekf_profile_flushes",
    "ekf_flush_kernel_name", "ekf_debug_scan_stamps", "ekf_debug_result_words",
    "ekf_shard_create", "ekf_shard_tiles", "ekf_shard_buffer_words", "ekf_shard_begin", "ekf_shard_line",
    "ekf_shard_apply", "ekf_shard_end", "ekf_shard_abort", "ekf_shard_spec_buffer_words",
    "ekf_shard_speculate", "ekf_shard_run", "ekf_shard_resume",
    "ekf_rccl_unique_id", "ekf_shard_attach_rccl", "ekf_shard_localize",
]


class EkfConfig(ctypes.Structure):
    _fields_ = [
        ("capacity", ctypes.c_int32), ("instances", ctypes.c_int32),
        ("precision", ctypes.c_int32), ("device", ctypes.c_int32),
        ("max_lines", ctypes.c_int32), ("r_mode", ctypes.c_int32),
        ("reset_margin", ctypes.c_int32), ("pipeline", ctypes.c_int32),
        ("flush_interval", ctypes.c_int32), ("arith", ctypes.c_int32),
        ("mahalanobis", ctypes.c_double), ("encoder_noise", ctypes.c_double),
    ]


class EkfLine(ctypes.Structure):
    _fields_ = [("alpha", ctypes.c_double), ("r", ctypes.c_double), ("R", ctypes.c_double * 4)]


class EkfResult(ctypes.Structure):
    _fields_ = [
        ("pose", ctypes.c_double * 3), ("matches", ctypes.c_int32),
        ("new_landmarks", ctypes.c_int32), ("saved", ctypes.c_int32),
        ("reset", ctypes.c_int32), ("status", ctypes.c_int32), ("nlines", ctypes.c_int32),
        ("match", ctypes.c_int32 * EKF_MAX_LINES),
    ]


class EkfError(RuntimeError):
    pass


_lib = None
loaded_path = None   # the file load_library() loaded


def load_library(path: str = ""):
    """Load libslam_ekf.so (never builds implicitly on a GPU box: fail loudly instead).
    SLAM_EKF_LIB selects another build of the same library (A/B experiments)."""
    global _lib, loaded_path
    if _lib is not None:
        return _lib
    path = path or os.environ.get("SLAM_EKF_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise EkfError(f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`"
                       " (HIP extension required; there is no CPU fallback)")
    L = ctypes.CDLL(path)
    loaded_path = path
    vp, i32, d, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_size_t
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int32)
    cp = ctypes.POINTER(vp)
    sig = {
        "ekf_config_init": (None, [ctypes.POINTER(EkfConfig)]),
        "ekf_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "ekf_abi_version": (ctypes.c_int, []),
        "ekf_create": (ctypes.c_int, [ctypes.POINTER(EkfConfig), cp]),
        "ekf_destroy": (ctypes.c_int, [vp]),
        "ekf_set_stream": (ctypes.c_int, [vp, vp]),
        "ekf_sync": (ctypes.c_int, [vp]),
        "ekf_set_option": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
        "ekf_get_option": (ctypes.c_int, [vp, ctypes.c_int, ip]),
        "ekf_reset_instance": (ctypes.c_int, [vp, ctypes.c_int, d, d, d]),
        "ekf_localize": (ctypes.c_int, [vp, dp, vp, ip, vp]),
        "ekf_localize_device": (ctypes.c_int, [vp, vp, vp, vp]),
        "ekf_predict": (ctypes.c_int, [vp, dp]),
        "ekf_update": (ctypes.c_int, [vp, vp, ip, vp]),
        "ekf_read_results": (ctypes.c_int, [vp, vp]),
        "ekf_upload_state": (ctypes.c_int, [vp, ctypes.c_int, dp, dp, ctypes.c_int, dp]),
        "ekf_download_state": (ctypes.c_int, [vp, ctypes.c_int, dp, dp, ip, dp]),
        "ekf_init_lowrank": (ctypes.c_int, [vp, ctypes.c_int, dp, dp, ctypes.c_int, dp,
                                            ctypes.c_int, dp]),
        "ekf_storage_exponent": (ctypes.c_int, [vp, ctypes.c_int]),
        "ekf_rescale": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
        "ekf_get_pose_cov": (ctypes.c_int, [vp, ctypes.c_int, dp]),
        "ekf_get_ellipse": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(ctypes.c_float)]),
        "ekf_ellipse_of_block": (ctypes.c_int, [dp, ctypes.POINTER(ctypes.c_float),
                                                ctypes.POINTER(ctypes.c_float)]),
        "ekf_landmark_block_bytes": (sz, [vp]),
        "ekf_state_dim": (ctypes.c_int, [vp]),
        "ekf_profile_enable": (ctypes.c_int, [vp, ctypes.c_int]),
        "ekf_profile_read": (ctypes.c_int, [vp, dp, dp, dp, ip]),
        "ekf_profile_flushes": (ctypes.c_int, [vp, ctypes.c_int, ip, ctypes.POINTER(ctypes.c_float)]),
        "ekf_flush_kernel_name": (ctypes.c_char_p, [vp, ctypes.c_int]),
        "ekf_debug_scan_stamps": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_ulonglong)]),
        "ekf_debug_result_words": (ctypes.c_int, [vp, ctypes.c_int, ip]),
        "ekf_shard_create": (ctypes.c_int, [ctypes.POINTER(EkfConfig), ctypes.c_int, ctypes.c_int, cp]),
        "ekf_shard_tiles": (ctypes.c_int, [vp, ip, ip]),
        "ekf_shard_buffer_words": (sz, [vp]),
        "ekf_shard_begin": (ctypes.c_int, [vp, dp, vp, ctypes.c_int, vp]),
        "ekf_shard_line": (ctypes.c_int, [vp, ctypes.c_int, vp]),
        "ekf_shard_apply": (ctypes.c_int, [vp, ctypes.c_int, vp]),
        "ekf_shard_end": (ctypes.c_int, [vp, vp]),
        "ekf_shard_abort": (ctypes.c_int, [vp]),
        "ekf_shard_spec_buffer_words": (sz, [vp]),
        "ekf_shard_speculate": (ctypes.c_int, [vp, vp, vp]),
        "ekf_shard_run": (ctypes.c_int, [vp, vp, vp]),
        "ekf_rccl_unique_id": (ctypes.c_int, [vp]),
        "ekf_shard_attach_rccl": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int]),
        "ekf_shard_localize": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, vp]),
        "ekf_shard_resume": (ctypes.c_int, [vp, ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str):
    if rc != 0:
        msg = load_library().ekf_strerror(rc).decode()
        raise EkfError(f"{what}: {msg} ({rc})")


def _dp(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def lines_array(lines, max_lines: int, instances: int = 1) -> np.ndarray:
    """(E, max_lines, 6) float64 array → contiguous ekf_line buffer (zero padded)."""
    arr = np.asarray(lines, dtype=np.float64)
    if arr.ndim == 2:
        arr = arr[None]
    out = np.zeros((instances, max_lines, 6))
    L = min(arr.shape[1], max_lines)
    out[: arr.shape[0], :L] = arr[:, :L, :6]
    return np.ascontiguousarray(out)


def ellipse_of_block(P22):
    """Robot::getEllipse arithmetic (Robot.cpp:73-124) on a given 2x2 block, host side of the
    library (no device): (ok, [axii0, axii1], angle)."""
    blk = np.ascontiguousarray(np.asarray(P22, dtype=np.float64).reshape(4))
    axii = (ctypes.c_float * 2)()
    ang = ctypes.c_float()
    rc = load_library().ekf_ellipse_of_block(_dp(blk), axii, ctypes.byref(ang))
    if rc < 0:
        _check(-rc, "ekf_ellipse_of_block")
    return rc == 1, [axii[0], axii[1]], ang.value


class Ensemble:
    """E independent EKF instances of capacity N on one GPU (one C-ABI context)."""

    def __init__(self, capacity: int, instances: int = 1, precision: int = PREC_F64,
                 max_lines: int = 20, device: int = -1, r_mode: int = R_INTENDED,
                 reset_margin: int = 10, mahalanobis: float = 0.4, encoder_noise: float = 0.024,
                 pipeline: bool = False, flush_interval: int = 1, arith: int = ARITH_EXACT,
                 options: dict | None = None, shard: tuple[int, int] | None = None):
        """shard = (rank, world): a partitioned instance (slam_ekf.h ekf_shard_create; instances = 1)
        storing its share of the landmark block only; rowshard_gpu.ShardedInstance drives it."""
        self._lib = load_library()
        cfg = EkfConfig()
        self._lib.ekf_config_init(ctypes.byref(cfg))
        cfg.capacity, cfg.instances, cfg.precision = capacity, instances, precision
        cfg.device, cfg.max_lines, cfg.r_mode = device, max_lines, r_mode
        cfg.reset_margin, cfg.mahalanobis, cfg.encoder_noise = reset_margin, mahalanobis, encoder_noise
        cfg.pipeline = 1 if pipeline else 0
        cfg.flush_interval = int(flush_interval)
        cfg.arith = int(arith)
        h = ctypes.c_void_p()
        if shard is None:
            _check(self._lib.ekf_create(ctypes.byref(cfg), ctypes.byref(h)), "ekf_create")
        else:
            _check(self._lib.ekf_shard_create(ctypes.byref(cfg), int(shard[0]), int(shard[1]), ctypes.byref(h)),
                   "ekf_shard_create")
        self._h = h
        self.capacity, self.instances, self.precision = capacity, instances, precision
        self.max_lines = max_lines
        self.arith = int(arith)
        self.n = self._lib.ekf_state_dim(h)
        self._res = (EkfResult * instances)()
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ekf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_handle: int | None):
        _check(self._lib.ekf_set_stream(self._h, ctypes.c_void_p(stream_handle or 0)), "ekf_set_stream")

    def sync(self):
        _check(self._lib.ekf_sync(self._h), "ekf_sync")

    def set_option(self, option, value: int):
        """ekf_set_option: option is an OPT_* number or an OPTIONS name (e.g. "speculate")."""
        opt = OPTIONS[option] if isinstance(option, str) else int(option)
        _check(self._lib.ekf_set_option(self._h, opt, int(value)), f"ekf_set_option({option}, {value})")

    def get_option(self, option) -> int:
        opt = OPTIONS[option] if isinstance(option, str) else int(option)
        v = ctypes.c_int32()
        _check(self._lib.ekf_get_option(self._h, opt, ctypes.byref(v)), f"ekf_get_option({option})")
        return v.value

    def reset(self, e: int = -1, x: float = 0.0, y: float = 0.0, theta: float = 0.0):
        _check(self._lib.ekf_reset_instance(self._h, e, x, y, theta), "ekf_reset_instance")

    def _results(self) -> list[dict]:
        out = []
        for r in self._res:
            out.append(dict(pose=np.array(r.pose[:]), matches=r.matches,
                            new_landmarks=r.new_landmarks, saved=r.saved, reset=r.reset,
                            status=r.status, match=list(r.match[: r.nlines])))
        return out

    def localize(self, encoder, lines, nlines=None) -> list[dict]:
        enc = np.ascontiguousarray(np.asarray(encoder, dtype=np.float64).reshape(self.instances, 3))
        la = lines_array(lines, self.max_lines, self.instances)
        if nlines is None:
            nl = np.array([min(np.asarray(lines).reshape(self.instances, -1, 6).shape[1],
                               self.max_lines)] * self.instances, dtype=np.int32)
        else:
            nl = np.ascontiguousarray(np.asarray(nlines, dtype=np.int32).reshape(self.instances))
        _check(self._lib.ekf_localize(self._h, _dp(enc), la.ctypes.data_as(ctypes.c_void_p),
                                      nl.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      ctypes.byref(self._res)), "ekf_localize")
        return self._results()

    def localize_device(self, d_enc: int, d_lines: int, d_nlines: int):
        """Inputs already in device memory (raw pointers); asynchronous on the context stream."""
        _check(self._lib.ekf_localize_device(self._h, ctypes.c_void_p(d_enc), ctypes.c_void_p(d_lines),
                                             ctypes.c_void_p(d_nlines)), "ekf_localize_device")

    def predict(self, encoder):
        enc = np.ascontiguousarray(np.asarray(encoder, dtype=np.float64).reshape(self.instances, 3))
        _check(self._lib.ekf_predict(self._h, _dp(enc)), "ekf_predict")

    def update(self, lines, nlines=None) -> list[dict]:
        la = lines_array(lines, self.max_lines, self.instances)
        if nlines is None:
            nl = np.array([min(np.asarray(lines).reshape(self.instances, -1, 6).shape[1],
                               self.max_lines)] * self.instances, dtype=np.int32)
        else:
            nl = np.ascontiguousarray(np.asarray(nlines, dtype=np.int32).reshape(self.instances))
        _check(self._lib.ekf_update(self._h, la.ctypes.data_as(ctypes.c_void_p),
                                    nl.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    ctypes.byref(self._res)), "ekf_update")
        return self._results()

    def read_results(self) -> list[dict]:
        _check(self._lib.ekf_read_results(self._h, ctypes.byref(self._res)), "ekf_read_results")
        return self._results()

    def upload_state(self, e: int, P=None, y=None, saved: int = 0, pose=None):
        Pc = None if P is None else np.ascontiguousarray(P, dtype=np.float64)
        yc = None if y is None else np.ascontiguousarray(y, dtype=np.float64)
        pc = None if pose is None else np.ascontiguousarray(pose, dtype=np.float64)
        _check(self._lib.ekf_upload_state(self._h, e, _dp(Pc), _dp(yc), int(saved), _dp(pc)),
               "ekf_upload_state")

    def init_lowrank(self, e: int, diag, U, y, saved: int, pose=(0.0, 0.0, 0.0)):
        dc = np.ascontiguousarray(diag, dtype=np.float64)
        Uc = np.ascontiguousarray(U, dtype=np.float64)
        yc = np.ascontiguousarray(y, dtype=np.float64)
        pc = np.ascontiguousarray(pose, dtype=np.float64)
        _check(self._lib.ekf_init_lowrank(self._h, e, _dp(dc), _dp(Uc), int(Uc.shape[1]), _dp(yc),
                                          int(saved), _dp(pc)), "ekf_init_lowrank")

    def download_state(self, e: int, with_P: bool = True):
        P = np.zeros((self.n, self.n)) if with_P else None
        y = np.zeros(self.n)
        saved = ctypes.c_int32()
        pose = np.zeros(3)
        _check(self._lib.ekf_download_state(self._h, e, _dp(P), _dp(y), ctypes.byref(saved), _dp(pose)),
               "ekf_download_state")
        return P, y, saved.value, pose

    def storage_exponent(self, e: int = 0) -> int:
        """fp16 storage: the landmark block holds fp16(2^exp·P); 0 for f32 / f64."""
        return int(self._lib.ekf_storage_exponent(self._h, e))

    def rescale(self, e: int = 0, exp: int = EXP_AUTO):
        """Re-choose (or set) instance e's fp16 storage exponent (after ST_RANGE)."""
        _check(self._lib.ekf_rescale(self._h, e, int(exp)), "ekf_rescale")

    def pose_cov(self, e: int = 0) -> np.ndarray:
        out = np.zeros(9)
        _check(self._lib.ekf_get_pose_cov(self._h, e, _dp(out)), "ekf_get_pose_cov")
        return out.reshape(3, 3)

    def ellipse(self, e: int = 0):
        axii = (ctypes.c_float * 2)()
        ang = ctypes.c_float()
        rc = self._lib.ekf_get_ellipse(self._h, e, axii, ctypes.byref(ang))
        if rc < 0:
            _check(-rc, "ekf_get_ellipse")
        return rc == 1, [axii[0], axii[1]], ang.value

    def profile_flushes(self) -> list[tuple[int, float]]:
        """(steps, ms) of every flush launch timed since the last profile() call."""
        n = self._lib.ekf_profile_flushes(self._h, 0, None, None)
        if n < 0:
            _check(-n, "ekf_profile_flushes")
        ns = (ctypes.c_int32 * max(n, 1))()
        ms = (ctypes.c_float * max(n, 1))()
        n = self._lib.ekf_profile_flushes(self._h, n, ns, ms)
        if n < 0:
            _check(-n, "ekf_profile_flushes")
        return [(ns[k], ms[k]) for k in range(n)]

    def flush_kernel_name(self, nsteps: int) -> str:
        return self._lib.ekf_flush_kernel_name(self._h, int(nsteps)).decode()

    def result_words(self, e: int = 0) -> list[int]:
        out = (ctypes.c_int32 * 16)()
        _check(self._lib.ekf_debug_result_words(self._h, e, out), "ekf_debug_result_words")
        return list(out)

    def scan_stamps(self) -> list[int]:
        out = (ctypes.c_ulonglong * 32)()
        _check(self._lib.ekf_debug_scan_stamps(self._h, out), "ekf_debug_scan_stamps")
        return list(out)

    def landmark_block_bytes(self) -> int:
        return int(self._lib.ekf_landmark_block_bytes(self._h))

    def profile(self, level: int = 2):
        """HIP-event timing: 0 off, 1 the flush only, 2 also every association kernel
        (True = 2)."""
        level = 2 if level is True else int(level)
        _check(self._lib.ekf_profile_enable(self._h, level), "ekf_profile_enable")

    def profile_read(self):
        s, dd, a = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        k = ctypes.c_int32()
        _check(self._lib.ekf_profile_read(self._h, ctypes.byref(s), ctypes.byref(dd), ctypes.byref(a),
                                          ctypes.byref(k)), "ekf_profile_read")
        return dict(scan_ms=s.value, downdate_ms=dd.value, augment_ms=a.value, launches=k.value)


class Robot:
    """Mirror of `class Robot` (Robot.h:21-77) for one EKF instance on the GPU.

    `localize(lines, rot=None, encoder=None)` follows Robot.cpp:126-904 with
    SIMULATIONOFF == true (Robot.h:18): the encoder pose drives the motion model and `rot` is
    ignored. `lines` is a sequence of (alfa, r, C_AR[4]) or objects with `.alfa`, `.r`,
    `.C_AR` and optional `.lineInterval` [(alfa, r), (alfa, r)] endpoints.
    """

    def __init__(self, x: float, y: float, theta: float, capacity: int = 100,
                 precision: int = PREC_F64, max_lines: int = 20, r_mode: int = R_INTENDED):
        self._ens = Ensemble(capacity, 1, precision, max_lines, r_mode=r_mode)
        self._ens.reset(0, x, y, theta)
        self.xPos, self.yPos, self.thetaPos = float(x), float(y), float(theta)
        self.lineIntervals: list[float] = []
        self.matchesNum = 0
        self.savedLineCount = 0
        self.last = None

    @staticmethod
    def _as_rows(lines):
        rows, intervals = [], []
        for ln in lines:
            if hasattr(ln, "alfa"):
                R = np.asarray(ln.C_AR, dtype=np.float64).reshape(4)
                rows.append([ln.alfa, ln.r, *R])
                intervals.append(getattr(ln, "lineInterval", None))
            else:
                a = np.asarray(ln, dtype=np.float64).reshape(-1)
                rows.append(list(a[:6]))
                intervals.append(None)
        return np.array(rows, dtype=np.float64).reshape(-1, 6), intervals

    def _store_intervals(self, res, intervals):
        # Robot.cpp:870-879: endpoints of every appended line, world frame, float32
        for i, m in enumerate(res["match"]):
            iv = intervals[i] if i < len(intervals) else None
            if m >= 0 or iv is None or len(iv) != 2:
                continue
            for (alfa_r, r_r) in (iv[0], iv[-1]):
                alpha = float(np.float32(alfa_r))
                a = alpha + self.thetaPos
                rr = r_r + self.xPos * math.cos(alpha) + self.yPos * math.sin(alpha)
                self.lineIntervals.append(float(np.float32(math.cos(a) * rr)))
                self.lineIntervals.append(float(np.float32(math.sin(a) * rr)))

    def _commit(self, res, intervals):
        self.xPos, self.yPos, self.thetaPos = (float(v) for v in res["pose"])
        self.matchesNum = res["matches"]
        self.savedLineCount = res["saved"]
        self.last = res
        self._store_intervals(res, intervals)

    def localize(self, lines, rot=None, encoder=None):
        if encoder is None:
            raise EkfError("encoder pose required (SIMULATIONOFF == true, Robot.cpp:140-145)")
        rows, intervals = self._as_rows(lines)
        res = self._ens.localize(np.asarray(encoder, dtype=np.float64)[None], rows[None],
                                 [len(rows)])[0]
        self._commit(res, intervals)

    def predict(self, encoder):
        self._ens.predict(np.asarray(encoder, dtype=np.float64)[None])

    def update(self, lines):
        rows, intervals = self._as_rows(lines)
        res = self._ens.update(rows[None], [len(rows)])[0]
        self._commit(res, intervals)

    def getEllipse(self):
        ok, axii, angle = self._ens.ellipse(0)
        return ok, axii, angle

    @property
    def P_t0(self) -> np.ndarray:
        return self._ens.download_state(0)[0]

    @property
    def y(self) -> np.ndarray:
        return self._ens.download_state(0, with_P=False)[1]

    def set_state(self, P, y, saved, pose):
        self._ens.upload_state(0, P, y, saved, pose)
        self.xPos, self.yPos, self.thetaPos = (float(v) for v in pose)
        self.savedLineCount = int(saved)
