"""Host-side AddressSanitizer / UndefinedBehaviorSanitizer builds, CPU only.

* oracle/: the CPU restatement (both modes) on a seeded trajectory with map building, matches,
  an empty scan, capacity overflow and the reset (oracle/asan_driver.c, `make -C oracle sanitize`).
* host headers: line_extraction.hpp + ros_output.hpp (the config-1 ray-cast → extraction path,
  tests/cpp/config1_driver.cpp in `extract` mode) and robot_ekf.hpp's host code
  (tests/cpp/normalize_driver.cpp), compiled with -fsanitize=address,undefined.
GPU code is not sanitized (no GPU ASan on this pool); the library itself is not linked here
except by the config-1 driver, whose extract mode never creates a context.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
       "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    out = subprocess.run([os.path.join(ROOT, "oracle", "oracle_asan")], capture_output=True, text=True,
                         env=ENV, timeout=300)
    assert out.returncode == 0, (out.returncode, out.stdout[-2000:], out.stderr[-4000:])
    assert "runtime error" not in out.stderr and "ERROR: AddressSanitizer" not in out.stderr


def test_extraction_headers_under_asan_ubsan(tmp_path, ekf_mod):
    from tests.test_line_extraction import scenario, trajectory
    exe = tmp_path / "config1_asan"
    libdir = os.path.dirname(ekf_mod.LIB_PATH)
    subprocess.run(["g++", "-std=c++11", *SAN, f"-I{os.path.join(ROOT, 'include')}",
                    f"-I{os.path.join(ROOT, 'slam_ros_amd', 'host')}",
                    os.path.join(ROOT, "tests", "cpp", "config1_driver.cpp"), "-o", str(exe),
                    f"-L{libdir}", "-lslam_ekf", f"-Wl,-rpath,{libdir}"], check=True)
    poses = trajectory(4) + [(3.6, 2.6, 0.0), (-2.7, -1.7, 2.5), (1.5, 0.45, -1.0)]
    # the library's own GPU runtime is not what is checked here: leaks in it are not reported
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0")
    out = subprocess.run([str(exe), "extract", str(scenario(tmp_path, poses))], capture_output=True,
                         text=True, env=env, timeout=300)
    assert out.returncode == 0, (out.returncode, out.stderr[-4000:])
    assert out.stdout.count("pose") == len(poses)
    assert "runtime error" not in out.stderr


def test_robot_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "normalize_asan"
    subprocess.run(["g++", "-std=c++11", *SAN, f"-I{os.path.join(ROOT, 'include')}",
                    f"-I{os.path.join(ROOT, 'slam_ros_amd', 'host')}",
                    os.path.join(ROOT, "tests", "cpp", "normalize_driver.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "7", "-7", "1e300", "-1e300", "nan"], capture_output=True, text=True,
                         env=ENV, timeout=60)
    assert out.returncode == 0 and "runtime error" not in out.stderr, out.stderr
