"""CPU baselines of SURVEY.md §8d on the host it runs on (no GPU use):
  B0 "GSL path": the restatement in faithful mode (dense GSL-order loops: the n³ Fx·P·Fxᵀ
     predict, per-candidate dense H·P·Hᵀ, dense n² updates), 1 core;
  B1: fast mode (sparse predict/gating, dense O(n²) update per match), 1 core.
Same synthetic worlds and scans as bench.py (L = m = 8). Prints one JSON line per (mode, N)."""
import json
import os
import platform
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
from slam_ros_amd import scan_gen as G  # noqa: E402

budget = float(os.environ.get("CPU_SECONDS", "20"))
cpu = "unknown"
try:
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
except OSError:
    pass
print(json.dumps({"host_cpu": cpu, "logical_cpus": os.cpu_count(), "python": platform.python_version()}), flush=True)
for mode, name, sizes in ((O.FAITHFUL, "B0 faithful (GSL-order dense)", (64, 256, 1024)),
                          (O.FAST, "B1 fast", (64, 256, 1024, 4096))):
    for N in sizes:
        w = G.make_world(N)
        st = G.initial_state(w)
        ref = O.OracleRobot(N, mode=mode)
        ref.set_state(st.dense_P(), st.y, st.saved, st.pose)
        t = 0.0
        k = 0
        while t < budget and k < 200:
            enc, lines, _ = G.make_scan(w, k + 1)
            t0 = time.perf_counter()
            m = ref.localize(lines[0], enc[0])
            t += time.perf_counter() - t0
            k += 1
            assert sum(1 for x in m if x >= 0) == 8, m
        print(json.dumps({"baseline": name, "N": N, "n": 3 + 2 * N, "updates": k, "seconds": round(t, 3),
                          "updates_per_s": k / t, "cores": 1}), flush=True)
        del ref
