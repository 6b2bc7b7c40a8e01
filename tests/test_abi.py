"""CPU checks of the drop-in boundary: the C-ABI library builds, loads and exports exactly the
entry points include/slam_ekf.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "slam_ekf.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(ekf_[a-z_0-9]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ("ekf_create", "ekf_localize", "ekf_predict", "ekf_update", "ekf_get_ellipse",
                 "ekf_download_state", "ekf_upload_state", "ekf_localize_device"):
        assert must in names


def test_library_exports_every_declared_symbol(ekf_mod):
    lib = ctypes.CDLL(ekf_mod.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(ekf_mod.EXPORTED) == declared_functions()


def test_library_is_gfx950_code_object(ekf_mod):
    """The device code embedded in the .so targets gfx950 (and only gfx950)."""
    data = open(ekf_mod.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in data


def test_cpu_only_calls(ekf_mod):
    lib = ekf_mod.load_library()
    assert lib.ekf_abi_version() == 3   # ABI 3: options instead of environment variables
    # no context: every option call is EKF_EINVAL before any HIP call
    v = ctypes.c_int32()
    assert lib.ekf_set_option(None, ekf_mod.OPT_SPECULATE, 1) == 1
    assert lib.ekf_get_option(None, ekf_mod.OPT_SPECULATE, ctypes.byref(v)) == 1
    assert lib.ekf_shard_abort(None) == 1
    assert lib.ekf_strerror(0) == b"ok"
    cfg = ekf_mod.EkfConfig()
    lib.ekf_config_init(ctypes.byref(cfg))
    # defaults are the reference's compile-time constants (Robot.h:13-17, Robot.cpp:893)
    assert cfg.capacity == 100 and cfg.reset_margin == 10
    assert cfg.mahalanobis == 0.4 and cfg.encoder_noise == 0.024
    h = ctypes.c_void_p()
    bad = ekf_mod.EkfConfig()
    lib.ekf_config_init(ctypes.byref(bad))
    bad.max_lines = 1000
    assert lib.ekf_create(ctypes.byref(bad), ctypes.byref(h)) == 1   # EKF_EINVAL before any HIP call
    # ekf_config.arith (the former reserved word): EXACT by default, unknown values rejected
    assert cfg.arith == ekf_mod.ARITH_EXACT == 0
    lib.ekf_config_init(ctypes.byref(bad))
    bad.arith = 7
    assert lib.ekf_create(ctypes.byref(bad), ctypes.byref(h)) == 1
    # EKF_ARITH_BF16X6 only where it can run (fp32, intended R, max_lines <= 8): EKF_EINVAL
    # otherwise, before any HIP call (no silent fallback to the exact arithmetic)
    for field, val in (("precision", ekf_mod.PREC_F64), ("r_mode", ekf_mod.R_AS_WRITTEN), ("max_lines", 9)):
        lib.ekf_config_init(ctypes.byref(bad))
        bad.precision, bad.max_lines, bad.arith = ekf_mod.PREC_F32, 8, ekf_mod.ARITH_BF16X6
        setattr(bad, field, val)
        assert lib.ekf_create(ctypes.byref(bad), ctypes.byref(h)) == 1, field


def test_library_reads_no_environment(ekf_mod):
    """The product library reads no environment variables (a stray EKF_TEST_DROP_WG
    made an instance time out on every scan): no getenv import in the shared object, and the
    former knobs are per-context options (slam_ekf.h EKF_OPT_*)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", ekf_mod.LIB_PATH], capture_output=True, text=True)
    assert out.returncode == 0
    assert not re.search(r"\b(secure_)?getenv\b", out.stdout), out.stdout
    src = open(HEADER).read()
    for name in ("EKF_OPT_SPECULATE", "EKF_OPT_SPIN_LOG2", "EKF_OPT_FLUSH_FORM", "EKF_OPT_FLUSH_BLOCKS_PER_CU",
                 "EKF_OPT_MFMA_REPLAY", "EKF_OPT_SCAN_STAMPS", "EKF_OPT_TEST_DROP_WG",
                 "EKF_OPT_TEST_VERDICT_TIMEOUT", "EKF_OPT_ACTIVE_FLUSH"):
        assert name in src
        assert getattr(ekf_mod, name[4:]) == int(re.search(name + r" = (\d+)", src).group(1))


def test_struct_layouts_match_header():
    # ekf_line is 6 doubles; ekf_result as declared
    from slam_ros_amd import ekf
    assert ctypes.sizeof(ekf.EkfLine) == 48
    assert ctypes.sizeof(ekf.EkfConfig) == 56
    assert ekf.EkfConfig.arith.offset == 36   # after the nine int32 fields, as in slam_ekf.h
    assert ctypes.sizeof(ekf.EkfResult) == 24 + 6 * 4 + 4 * ekf.EKF_MAX_LINES


def test_layout_header_bijective(tmp_path):
    """Host-compile ekf_layout.h and check the packed tile maps are bijections."""
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include "ekf_layout.h"
#include <cstdio>
#include <vector>
using namespace ekf;
int main() {
  for (int r = 0; r < 32; r++) for (int c = 0; c < 32; c++) {
    if (tile_off_f32(r, c) < 0 || tile_off_f32(r, c) >= 1024) return 1;
    if (tile_off_f64(r, c) < 0 || tile_off_f64(r, c) >= 1024) return 1;
  }
  std::vector<int> s32(1024, 0), s64(1024, 0);
  for (int r = 0; r < 32; r++) for (int c = 0; c < 32; c++) { s32[tile_off_f32(r,c)]++; s64[tile_off_f64(r,c)]++; }
  for (int k = 0; k < 1024; k++) if (s32[k] != 1 || s64[k] != 1) return 2;
  const int M = 200, nb = (M + 31) / 32;
  std::vector<int> hit((size_t)nb * (nb + 1) / 2 * 1024, 0);
  for (int i = 0; i < M; i++) for (int j = 0; j < M; j++) {
    if (ll_offset<float>(i, j, nb) != ll_offset<float>(j, i, nb) && (i >> 5) != (j >> 5)) return 3;
    hit[ll_offset<float>(i, j, nb)]++;
  }
  for (int i = 0; i < M; i++) for (int j = 0; j < M; j++) {
    int want = ((i >> 5) == (j >> 5)) ? 1 : 2;
    if (hit[ll_offset<float>(i, j, nb)] != want) return 4;
  }
  for (int bi = 0; bi < nb; bi++) for (int bj = bi; bj < nb; bj++)
    if (tile_index(bi, bj, nb) < 0 || tile_index(bi, bj, nb) >= (long)nb*(nb+1)/2) return 5;
  if (tile_index(nb - 1, nb - 1, nb) != (long)nb*(nb+1)/2 - 1) return 6;
  // operand maps stay inside their per-row-block slab
  const int kmax = 16;
  for (int row = 0; row < 64; row++) for (int k = 0; k < kmax; k++) {
    long a = op_index_f32(row, k, kmax), b = op_index_f64(row, k, kmax);
    if (a < (row >> 5) * 64L * (kmax / 2) || a >= ((row >> 5) + 1) * 64L * (kmax / 2)) return 7;
    if (b < (row >> 5) * 64L * (kmax / 2) || b >= ((row >> 5) + 1) * 64L * (kmax / 2)) return 8;
  }
  puts("ok");
  return 0;
}
''')
    exe = tmp_path / "t"
    inc = os.path.join(ROOT, "slam_ros_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{inc}", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.returncode


def test_commit_decision(tmp_path):
    """The association kernel's rollback bookkeeping (ekf_commit.h, host-compiled): a launch
    commits only if every workgroup's completion word carries this launch's epoch and no timeout
    bit; a stale word (a workgroup that never completed) or a timeout anywhere rolls it back; the
    other status bits are OR-ed; epochs wrap modulo 2^24."""
    src = tmp_path / "c.cpp"
    src.write_text(r"""
#include "ekf_commit.h"
#include <cstdio>
using namespace ekf;
int main() {
  const unsigned ep = 77;
  unsigned w[4] = {done_word(ep, 0), done_word(ep, EKF_ST_SINGULAR_S), done_word(ep, 0), done_word(ep, EKF_ST_RANGE)};
  int st = commit_status(w, 4, ep);
  if (st != (EKF_ST_SINGULAR_S | EKF_ST_RANGE)) return 1;                // commits, bits OR-ed
  w[2] = done_word(ep - 1, 0);                                          // stale: never completed
  st = commit_status(w, 4, ep);
  if (!(st & EKF_ST_SYNC_TIMEOUT) || !(st & EKF_ST_SINGULAR_S)) return 2;
  w[2] = done_word(ep, EKF_ST_SYNC_TIMEOUT);                            // timed out itself
  if (!(commit_status(w, 4, ep) & EKF_ST_SYNC_TIMEOUT)) return 3;
  if (commit_status(w, 1, ep) & EKF_ST_SYNC_TIMEOUT) return 4;          // G = 1: its own word only
  const unsigned big = (1u << 24) + 5;                                  // epoch tags wrap mod 2^24
  unsigned v[2] = {done_word(big, 0), done_word(5, 0)};
  if (commit_status(v, 2, big) != 0) return 5;
  if (done_word(ep, 0x1ff) & ~0xffffff00u & 0x100u) return 6;           // status confined to 8 bits
  if (commit_fold(0, 0u, 0u) != 0) return 7;                            // epoch 0 = a zeroed word: "arrived"
  puts("ok");
  return 0;
}
""")
    exe = tmp_path / "c"
    inc = os.path.join(ROOT, "slam_ros_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{inc}", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.returncode
