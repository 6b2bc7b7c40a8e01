"""Speculative association diagnostics: per EKF_SPECULATE mode the phase stamps and the number
of fallbacks (stamp 15) over a few scans."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["EKF_SCAN_STAMPS"] = "1"
from slam_ros_amd import ekf, scan_gen as G
N = int(os.environ.get("N", 64)); E = int(os.environ.get("E", 1)); T = int(os.environ.get("T", 1))
w = G.make_world(N); st = G.initial_state(w)
for mode in (0, 1, 2):
    os.environ["EKF_SPECULATE"] = str(mode)
    ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, flush_interval=T)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    ms = []
    for s in range(1, 11):
        enc, lines, nl = G.make_scan(w, s, instances=E)
        r = ens.localize(enc, lines, nl)
        ms.append(r[0]["matches"])
    stp = ens.scan_stamps()
    n = stp[9] or 1
    print(mode, ms, json.dumps([round(v * 10e-3 / n, 2) for v in stp[:15]]), "fallbacks", stp[15])
    ens.close()
