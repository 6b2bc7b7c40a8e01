"""Debug: determinism and T-independence of fp16 storage at N=1024 (E=3)."""
import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G
N, E = 1024, 3
prec = int(os.environ.get("PREC", "2"))
w = G.make_world(N, active=N - 10); st = G.initial_state(w)
def run(T, steps=24):
    a = ekf.Ensemble(N, E, prec, max_lines=8, flush_interval=T)
    for e in range(E): a.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    for step in range(1, steps + 1):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=8)
        r = a.localize(enc, ln, nl)
        if T == 8 and steps == 9: print("step", step, [x["matches"] for x in r], [x["new_landmarks"] for x in r])
    out = [a.download_state(e) for e in range(E)]
    a.close(); return out
def cmp(X, Y):
    return [int(np.argwhere(X[e][0] != Y[e][0]).shape[0]) for e in range(E)], [bool(np.array_equal(X[e][1], Y[e][1])) for e in range(E)]
os.environ["EKF_SPECULATE"] = os.environ.get("SPEC", "1")
for steps in (1, 2, 9):
    B1 = run(1, steps); B2 = run(1, steps); A1 = run(8, steps); A2 = run(8, steps)
    print("steps", steps, "T1 vs T1", cmp(B1, B2), "T8 vs T8", cmp(A1, A2), "T8 vs T1", cmp(A1, B1), flush=True)
