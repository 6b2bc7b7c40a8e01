import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from slam_ros_amd import ekf, scan_gen as G
N = 64
w = G.make_world(N, active=N - 14); st = G.initial_state(w)
for pipe in (True, False):
    a = ekf.Ensemble(N, 2, 1, max_lines=8, pipeline=pipe)
    b = ekf.Ensemble(N, 2, 1, max_lines=8, pipeline=pipe)
    for ens in (a, b):
        for e in range(2):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(11)
    for step in range(1, 21):
        enc, lines, nl = G.make_scan(w, step, instances=2, lines=6)
        extra = G.random_lines(rng, 2)[None].repeat(2, axis=0) if step % 3 == 0 else np.zeros((2, 0, 6))
        ln = np.concatenate([lines, extra], axis=1)
        nl = np.full(2, ln.shape[1], dtype=np.int32)
        ra = a.localize(enc, ln, nl); rb = b.localize(enc, ln, nl)
        b.download_state(0, with_P=False)
        ca, cb = a.pose_cov(0), b.pose_cov(0)
        print(pipe, step, ra[0]["matches"], ra[0]["new_landmarks"], ra[0]["reset"], ra[0]["saved"],
              "dR33", float(np.abs(ca - cb).max()), "dpose", float(np.abs(ra[0]["pose"] - rb[0]["pose"]).max()))
