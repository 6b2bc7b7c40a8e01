"""Time the drop-in on the path slam_ros/main.cpp calls: one Robot at the
reference's capacity (LINESIZE 100, n = 203), fp64, synchronous Robot::localize per scan through
slam_ros_amd/host/robot_ekf.hpp (tests/cpp/dropin_bench.cpp), P_t0 mirrored in full (kFull, the
default) or its pose block only (kPoseBlock); beside it the restatement's B0 (faithful GSL-order,
1 core) and B1 (fast, 1 core and the OpenMP team) on the same scans of the same host.
Bench world at N = 100: s = 90 landmarks, L = m = 8 matched lines per scan.
usage: python scripts/r06/dropin_bench.py OUT_DIR [warmup timed]"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

out_dir = sys.argv[1]
W, K = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (20, 200)
os.makedirs(out_dir, exist_ok=True)
N, L = 100, 8
world = G.make_world(N)
st = G.initial_state(world)
P0 = st.dense_P()
scans = [G.make_scan(world, s + 1, instances=1, lines=L) for s in range(W + K)]
scen = os.path.join(out_dir, "scenario.txt")
with open(scen, "w") as f:
    f.write(f"{len(scans)}\n")
    for enc, lines, nl in scans:
        f.write("%.17g %.17g %.17g %d\n" % (enc[0, 0], enc[0, 1], enc[0, 2], L))
        for ln in lines[0, :L]:
            f.write(" ".join("%.17g" % v for v in list(ln) + [0.0, 1.0, 0.1, 1.0]) + "\n")
state = os.path.join(out_dir, "state.bin")
np.concatenate([P0.ravel(), st.y, [float(st.saved)], st.pose]).astype(np.float64).tofile(state)
exe = os.path.join(out_dir, "dropin_bench")
libdir = os.path.dirname(ekf.LIB_PATH)
subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", f"-I{ROOT}/include", f"-I{ROOT}/slam_ros_amd/host",
                f"{ROOT}/tests/cpp/dropin_bench.cpp", "-o", exe, f"-L{libdir}", "-lslam_ekf",
                f"-Wl,-rpath,{libdir}"], check=True)
res = {"config": {"capacity": N, "n": 2 * N + 3, "active": int(st.saved), "lines": L, "precision": "f64",
                  "arith": "exact (the drop-in's)", "warmup": W, "timed": K,
                  "path": "BasicRobot<line, Float32MultiArray, 100>::localize (robot_ekf.hpp) -> ekf_localize"}}
if os.environ.get("DROPIN_GPU", "1") == "1":
    r = subprocess.run([exe, scen, state, str(W), str(K)], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(r.stdout, r.stderr, file=sys.stderr)
        sys.exit(r.returncode)
    res["gpu"] = json.loads(r.stdout)
# B0 / B1 on the same scans, this host
def cpu(mode, omp, count):
    ref = O.OracleRobot(N, mode=mode, omp=omp)
    ref.set_state(P0, st.y, st.saved, st.pose)
    t = []
    for enc, lines, nl in scans[:count]:
        t0 = time.perf_counter()
        ref.localize(lines[0, :L], enc[0])
        t.append((time.perf_counter() - t0) * 1e6)
    t = np.array(t[min(5, count // 4):])
    return {"median_us": float(np.median(t)), "mean_us": float(t.mean()), "calls": int(t.size),
            "threads": O.threads(omp)}
res["cpu"] = {"B0_faithful_1core": cpu(O.FAITHFUL, False, min(len(scans), 60)),
              "B1_fast_1core": cpu(O.FAST, False, len(scans)),
              "B1_fast_omp": cpu(O.FAST, True, len(scans)),
              "host_cpus": O.host_cpus()}
with open(os.path.join(out_dir, "dropin.json"), "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
