"""Debug: test_deferred_flush_equals_drained[False-4-()-fp32] replicated step by step (contexts a
(T=4) and b (T=1, drained) alive together), printing instance 1's path codes and guesses."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G

N = 64
w = G.make_world(N, active=N - 14)
st = G.initial_state(w)
a = ekf.Ensemble(N, 2, 1, max_lines=8, pipeline=False, flush_interval=4)
b = ekf.Ensemble(N, 2, 1, max_lines=8)
for ens in (a, b):
    for e in range(2):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
rng = np.random.default_rng(11)
for step in range(1, 21):
    enc, lines, nl = G.make_scan(w, step, instances=2, lines=6)
    extra = G.random_lines(rng, 2)[None].repeat(2, axis=0) if step % 3 == 0 else np.zeros((2, 0, 6))
    ln = np.concatenate([lines, extra], axis=1)
    nl = np.full(2, ln.shape[1], dtype=np.int32)
    ra = a.localize(enc, ln, nl)
    wa = [a.result_words(e) for e in range(2)]
    rb = b.localize(enc, ln, nl)
    wb = [b.result_words(e) for e in range(2)]
    b.download_state(0, with_P=False)
    flag = "" if ra[1]["match"] == rb[1]["match"] and ra[0]["match"] == rb[0]["match"] else "  <== DIFF"
    print(step, "a:", [r["match"] for r in ra], [x[9] for x in wa], "b:", [r["match"] for r in rb], [x[9] for x in wb], flag, flush=True)
for e in range(2):
    Pa = a.download_state(e)[0]
    Pb = b.download_state(e)[0]
    print("final e", e, "max|Pa-Pb|", float(np.abs(Pa - Pb).max()))
