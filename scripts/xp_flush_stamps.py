"""Flush timing experiment (git apply scripts/xp/flush_timing_probes.patch, then a build with
-DEKF_XP_FLUSH_STAMPS via slam_ros_amd.build.build_variant, run with SLAM_EKF_LIB): shader cycles per
wave-tile in the wave flush's boundary (entry, tile copy, next tiles issued), MFMA steps, and
tile stores, summed over waves (EKF_OPT_SCAN_STAMPS = 1 provides the buffer; instance 0's slots
24..27). usage: SLAM_EKF_LIB=... python scripts/xp_flush_stamps.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

N, E = 4096, 8
ARITH = os.environ.get("XP_ARITH", "exact")
BF = ARITH in ("bf16x6", "f16x3")   # the split forms also stamp their clock
T = int(os.environ.get("XP_T", "12" if BF else "8"))
w = G.make_world(N)
st = G.initial_state(w)
ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, flush_interval=T,
                   arith={"exact": ekf.ARITH_EXACT, "bf16x6": ekf.ARITH_BF16X6, "f16x3": ekf.ARITH_F16X3}[ARITH], options={"scan_stamps": 1})
for e in range(E):
    ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
for s in range(1, T * 6 + 1):
    enc, lines, nl = G.make_scan(w, s, instances=E)
    ens.localize(enc, lines, nl)
ens.sync()
stp = ens.scan_stamps()
n = stp[27] or 1
out = {"T": T, "arith": ARITH, "wave_tiles": stp[27], "cycles_per_wave_tile": {
    "boundary": stp[24] / n, "mfma_steps": stp[25] / n, "stores": stp[26] / n}}
if BF and stp[29]:   # in-kernel clock: shader cycles over 100 MHz real-time ticks, summed over waves
    out["clock_ghz"] = stp[28] / stp[29] * 0.1
    out["mfma_cycles_per_wave_tile"] = T * (12 if ARITH == "f16x3" else 24) * 32
print(json.dumps(out))
