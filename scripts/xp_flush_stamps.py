"""Flush timing experiment (build with -DEKF_XP_FLUSH_STAMPS, SLAM_EKF_LIB): shader cycles per
wave-tile in the wave flush's boundary (entry, tile copy, next tiles issued), MFMA steps, and
tile stores, summed over waves (EKF_OPT_SCAN_STAMPS = 1 provides the buffer; instance 0's slots
24..27). usage: SLAM_EKF_LIB=... python scripts/xp_flush_stamps.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

N, E = 4096, 8
BF = os.environ.get("XP_ARITH", "exact") == "bf16x6"   # the split-bf16 form also stamps its clock
T = int(os.environ.get("XP_T", "12" if BF else "8"))
w = G.make_world(N)
st = G.initial_state(w)
ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, flush_interval=T,
                   arith=ekf.ARITH_BF16X6 if BF else ekf.ARITH_EXACT, options={"scan_stamps": 1})
for e in range(E):
    ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
for s in range(1, T * 6 + 1):
    enc, lines, nl = G.make_scan(w, s, instances=E)
    ens.localize(enc, lines, nl)
ens.sync()
stp = ens.scan_stamps()
n = stp[27] or 1
out = {"T": T, "arith": "bf16x6" if BF else "exact", "wave_tiles": stp[27], "cycles_per_wave_tile": {
    "boundary": stp[24] / n, "mfma_steps": stp[25] / n, "stores": stp[26] / n}}
if BF and stp[29]:   # in-kernel clock: shader cycles over 100 MHz real-time ticks, summed over waves
    out["clock_ghz"] = stp[28] / stp[29] * 0.1
    out["mfma_cycles_per_wave_tile"] = T * 24 * 32
print(json.dumps(out))
