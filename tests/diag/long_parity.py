"""Long-horizon parity of the bench configuration (diagnostic, not a test): N = 4096, E = 8, L = 8,
fp32 storage, split-fp16 products, T = 20, the bench world, after `pre` untimed scans; then `scans`
scans with instances 0 and 7 checked against the restatement (oracle/, fast mode, fp64): y and the
pose re-synced to the GPU's after every scan (the per-scan contract), the whole state
at every flush-group end; association compared on every scan. A second restatement of instance 0
is never re-synced (the drift of a whole trajectory). One JSON line.

usage: python tests/diag/long_parity.py [pre] [scans] [T] [precision f32|f16|f64]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402
from oracle import oracle as O  # noqa: E402

N, E, L = 4096, 8, 8
CHECK = (0, 7)


def rel(a, b):
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


def main():
    pre = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    scans = int(sys.argv[2]) if len(sys.argv) > 2 else 240
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    precision = sys.argv[4] if len(sys.argv) > 4 else "f32"
    prec = {"f32": ekf.PREC_F32, "f16": ekf.PREC_F16, "f64": ekf.PREC_F64}[precision]
    arith = ekf.ARITH_EXACT if prec == ekf.PREC_F64 else ekf.ARITH_F16X3
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf.Ensemble(N, E, prec, max_lines=L, flush_interval=T, arith=arith)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    for s in range(1, pre + 1):
        enc, lines, nl = G.make_scan(w, s, instances=E, lines=L)
        ens.localize(enc, lines, nl)
    ens.sync()
    refs = {e: O.OracleRobot(N, mode=O.FAST, omp=True) for e in CHECK}
    for e in CHECK:
        refs[e].set_state(*ens.download_state(e))
    traj = O.OracleRobot(N, mode=O.FAST, omp=True)
    traj.set_state(*ens.download_state(0))
    y_scan, p_group, assoc_diff, status = [], [], 0, 0
    t0 = time.time()
    for k in range(scans):
        enc, lines, nl = G.make_scan(w, pre + 1 + k, instances=E, lines=L)
        res = ens.localize(enc, lines, nl)
        traj.localize(lines[0], enc[0])
        for e in CHECK:
            m = refs[e].localize(lines[e], enc[e])
            assoc_diff += int(res[e]["match"] != m)
            status |= int(res[e]["status"])
            _, yg, sg, pg = ens.download_state(e, with_P=False)
            y_scan.append(rel(yg, refs[e].y))
            refs[e].set_state(None, yg, sg, pg)
        if (k + 1) % T == 0 or k + 1 == scans:
            for e in CHECK:
                P, y, saved, pose = ens.download_state(e)
                p_group.append(rel(P, refs[e].P_t0))
                refs[e].set_state(P, y, saved, pose)
    P0, y0, _, _ = ens.download_state(0)
    out = {"config": f"N={N} E={E} L={L} {precision} storage {'exact' if arith == ekf.ARITH_EXACT else 'f16x3'} "
                     f"T={T}, bench world, pre-roll {pre}",
           "scans": scans, "groups": len(p_group) // len(CHECK), "instances_checked": list(CHECK),
           "assoc_differences": assoc_diff, "status_bits": status,
           "y_per_scan_max": max(y_scan), "y_per_scan_median": float(np.median(y_scan)),
           "P_per_group_max": max(p_group), "P_per_group_median": float(np.median(p_group)),
           "trajectory_never_resynced": {"P": rel(P0, traj.P_t0), "y": rel(y0, traj.y)},
           "wall_s": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)
    ens.close()


if __name__ == "__main__":
    main()
