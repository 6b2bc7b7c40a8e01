"""Quad flush timing experiment: in-kernel clock of the split-fp16 quad flush (a build with
-DEKF_Q_CLOCK, run with SLAM_EKF_LIB): shader cycles over 100 MHz real-time ticks of each MFMA wave 0,
summed (EKF_OPT_SCAN_STAMPS = 1 provides the buffer; slots 28, 29), and the flush's HIP-event time.
usage: SLAM_EKF_LIB=... python scripts/r06/quad_clock.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

N, E, T = 4096, 8, 20
w = G.make_world(N)
st = G.initial_state(w)
ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, flush_interval=T, arith=ekf.ARITH_F16X3,
                   options={"scan_stamps": 1, "flush_form": int(os.environ.get("XP_FORM", "44"))})
for e in range(E):
    ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
t0 = time.time()
for s in range(1, T * 6 + 1):
    enc, lines, nl = G.make_scan(w, s, instances=E)
    ens.localize(enc, lines, nl)
ens.sync()
stp = ens.scan_stamps()
print(json.dumps({"lib": os.environ.get("SLAM_EKF_LIB"), "kernel": ens.flush_kernel_name(T),
                  "clock_ghz": stp[28] / stp[29] * 0.1 if stp[29] else None, "wall_s": time.time() - t0}))
