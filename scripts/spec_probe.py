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
    us = [round(v * 10e-3 / n, 2) for v in stp[:15]]
    names = {0: "predict", 1: "diag", 2: "seq-gating|spec-ex1-xchg", 3: "seq-mbox|leader-eval", 4: "seq-exch|leader-gain", 6: "seq-gain/spec-verdict",
             5: "spec-guess", 10: "spec-resolve", 11: "spec-prefetch(wave0)", 12: "spec-records+stage", 13: "spec-leader",
             14: "spec-local", 7: "commit", 8: "total"}
    print(mode, ms, json.dumps({names[k]: us[k] for k in sorted(names) if us[k]}), "fallbacks", stp[15])
    ens.close()
