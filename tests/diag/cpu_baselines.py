"""CPU baselines of SURVEY.md §8d / BASELINE.md §2 on the host it runs on (no GPU use):
  B0 "GSL path": the restatement in faithful mode (dense GSL-order loops: the n³ Fx·P·Fxᵀ
     predict, per-candidate dense H·P·Hᵀ, dense n² updates), 1 core (gslcblas is
     single-threaded, as is the reference). N = 4096 is timed once (one update: minutes).
  B1: fast mode (sparse predict/gating, dense O(n²) update per match), OpenMP build on the host
     threads OMP_NUM_THREADS allows (bit-identical results), and its 1-core build.
Same synthetic worlds and scans as bench.py (L = m = 8). Prints one JSON line per (mode, N).
usage: python tests/diag/cpu_baselines.py [B0|B1|all]"""
import json
import os
import platform
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402,F401

from oracle import oracle as O  # noqa: E402
from slam_ros_amd import scan_gen as G  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
budget = float(os.environ.get("CPU_SECONDS", "20"))
cpu = "unknown"
try:
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
except OSError:
    pass
print(json.dumps({"host_cpu": cpu, "logical_cpus": os.cpu_count(), "omp_threads": O.threads(True),
                  "python": platform.python_version()}), flush=True)
runs = []
if which in ("B0", "all"):
    runs.append((O.FAITHFUL, False, "B0 faithful (GSL-order dense)", (64, 256, 1024, 4096)))
if which in ("B1", "all"):
    runs.append((O.FAST, True, "B1 fast, OpenMP", (64, 256, 1024, 4096)))
    runs.append((O.FAST, False, "B1 fast, 1 core", (64, 256, 1024, 4096)))
for mode, omp, name, sizes in runs:
    for N in sizes:
        w = G.make_world(N)
        st = G.initial_state(w)
        ref = O.OracleRobot(N, mode=mode, omp=omp)
        ref.set_state(st.dense_P(), st.y, st.saved, st.pose)
        t = 0.0
        k = 0
        while (t < budget and k < 200) or k == 0:
            enc, lines, _ = G.make_scan(w, k + 1)
            t0 = time.perf_counter()
            m = ref.localize(lines[0], enc[0])
            t += time.perf_counter() - t0
            k += 1
            assert sum(1 for x in m if x >= 0) == 8, m
        print(json.dumps({"baseline": name, "N": N, "n": 3 + 2 * N, "updates": k, "seconds": round(t, 3),
                          "updates_per_s": k / t, "cores": O.threads(True) if omp else 1,
                          "host_cpu": cpu}), flush=True)
        del ref
