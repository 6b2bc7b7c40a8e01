"""Build the in-tree gfx950 library libslam_ekf.so (hipcc, no torch extension machinery).

The library is the product path: slam_ros_amd/ekf.py loads it with ctypes and fails loudly if
it is missing. Built in-tree so the .so travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import socket
import subprocess
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libslam_ekf.so")
SOURCES = ["ekf_kernels.hip", "ekf_api.hip"]
HEADERS = ["ekf_kernels.h", "ekf_layout.h", "ekf_commit.h"]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libslam_ekf.so)")


def _file_sha(path: str) -> str:   # (bench.py's lib_sha)
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def _sha(paths: list[str]) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            for blk in iter(lambda: f.read(1 << 20), b""):
                h.update(blk)
    return h.hexdigest()[:16]


# Build provenance: the library carries a sidecar record of the sources it was
# compiled from (LIB_PATH + ".json": source_sha over the sources, headers and this file, lib_sha of
# the binary). build() reuses the library only when both hashes match — not by file times, which a
# copy of the tree does not keep reliably — and writes what it did to lib/last_build.json
# ("compiled" or "reused", host, time), which bench.py reports as build_mode.
RECORD = LIB_PATH + ".json"
LAST_BUILD = os.path.join(LIB_DIR, "last_build.json")


def _record() -> dict:
    try:
        with open(RECORD) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def last_build() -> dict:
    """The last build() on this copy of the tree, or {"mode": "prebuilt"} when build() never ran
    here (the library as shipped, with its own record)."""
    try:
        with open(LAST_BUILD) as f:
            return json.load(f)
    except (OSError, ValueError):
        rec = _record()
        return {"mode": "prebuilt", "source_sha": rec.get("source_sha"), "lib_sha": rec.get("lib_sha")}


# MFMA accumulators in VGPRs (not AGPRs): the fp16 flush rounds every accumulator after each
# step on the VALU, which cannot read AGPRs, so the AGPR form paid a read + write copy per
# element per step (fp16 flush 0.84 -> 0.72 ms at N=4096, T=8; fp32 unchanged or faster)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-mllvm", "-amdgpu-mfma-vgpr-form"]
# ekf_kernels.hip is compiled as nine units (EKF_TU: 1 association kernels, 2 the exact and fp64
# flushes, 3 the rest, 4 / 5 / 6 the split-fp16, 2 x 4 and split-bf16 flushes, 7 / 8 the association
# kernel on 128 / 64 landmarks per workgroup, 9 the split-fp16 quad flush), in parallel with ekf_api.hip: each unit instantiates
# only the kernels its launchers use
UNITS = [("ekf_kernels.hip", 4), ("ekf_kernels.hip", 2), ("ekf_kernels.hip", 1), ("ekf_kernels.hip", 7),
         ("ekf_kernels.hip", 8), ("ekf_kernels.hip", 5), ("ekf_kernels.hip", 6), ("ekf_kernels.hip", 3), ("ekf_kernels.hip", 9),
         ("ekf_api.hip", 0)]


def _compile_link(out: str, defines: list[str], verbose: bool = False, csrc: str = CSRC) -> None:
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    procs, objs = [], []
    for src, tu in UNITS:
        obj = os.path.join(objdir, f"{os.path.splitext(src)[0]}_{tu}.o")
        cmd = [hipcc(), f"--offload-arch={ARCH}", *FLAGS, *[f"-D{d}" for d in defines],
               *([f"-DEKF_TU={tu}"] if tu else []), "-c", os.path.join(csrc, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc (libslam_ekf units)")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    shutil.rmtree(objdir, ignore_errors=True)


def build_variant(out: str, defines: list[str], csrc: str = CSRC) -> str:
    """An A/B build with extra -D flags, or of a patched copy of csrc/ (scripts only; SLAM_EKF_LIB)."""
    _compile_link(out, defines, csrc=csrc)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "slam_ekf.h"))
    deps.append(os.path.abspath(__file__))   # compile flags live here
    src = _sha(deps)
    rec = _record()
    reuse = (not force and os.path.exists(LIB_PATH) and rec.get("source_sha") == src
             and rec.get("lib_sha") == _file_sha(LIB_PATH))
    if not reuse:
        os.makedirs(LIB_DIR, exist_ok=True)
        tmp = LIB_PATH + ".tmp"
        _compile_link(tmp, [], verbose)
        os.replace(tmp, LIB_PATH)
        rec = {"source_sha": src, "lib_sha": _file_sha(LIB_PATH), "built_on": socket.gethostname(),
               "built_at": time.strftime("%Y-%m-%dT%H:%M:%S")}
        with open(RECORD, "w") as f:
            json.dump(rec, f)
    last = {"mode": "reused" if reuse else "compiled", "source_sha": src, "lib_sha": rec["lib_sha"],
            "host": socket.gethostname(), "at": time.strftime("%Y-%m-%dT%H:%M:%S")}
    with open(LAST_BUILD, "w") as f:
        json.dump(last, f)
    print(f"libslam_ekf.so: {last['mode']} (source {src}, library {rec['lib_sha']})")
    return LIB_PATH


if __name__ == "__main__":
    print(build(force=True, verbose=True))
