"""Phase breakdown of the association kernel (EKF_OPT_SCAN_STAMPS = 1), N=4096 f32, 8 instances."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G
N = int(os.environ.get("N", 4096)); E = 8
names = ["predict", "diag", "gating", "mailbox-write", "exchange", "unused",
         "gain-rows", "commit", "total"]
T = int(os.environ.get("T", 1)); PIPE = int(os.environ.get("PIPE", 0))
w = G.make_world(N); st = G.initial_state(w)
ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, pipeline=bool(PIPE), flush_interval=T,
                   options={"scan_stamps": 1})
for e in range(E):
    ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
for s in range(1, 11):
    enc, lines, nl = G.make_scan(w, s, instances=E)
    r = ens.localize(enc, lines, nl)
st_ = ens.scan_stamps()
launches = st_[9] or 1
print(T, PIPE, json.dumps({k: round(st_[i] * 10e-3 / launches, 2) for i, k in enumerate(names)}))  # µs per launch (per instance)
