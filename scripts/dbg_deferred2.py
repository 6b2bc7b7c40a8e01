"""Debug: per step of the deferred scenario (N=64, E=2, fp32) the association path and guesses of
instance 1, deferred (T=4) vs drained (T=1), and the P difference at group ends."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G

def run(T, steps=17):
    N = 64
    w = G.make_world(N, active=N - 14)
    st = G.initial_state(w)
    ens = ekf.Ensemble(N, 2, 1, max_lines=8, flush_interval=T)
    for e in range(2):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(11)
    out = []
    for step in range(1, steps + 1):
        enc, lines, nl = G.make_scan(w, step, instances=2, lines=6)
        extra = G.random_lines(rng, 2)[None].repeat(2, axis=0) if step % 3 == 0 else np.zeros((2, 0, 6))
        ln = np.concatenate([lines, extra], axis=1)
        nl = np.full(2, ln.shape[1], dtype=np.int32)
        r = ens.localize(enc, ln, nl)
        words = ens.result_words(1)
        P = ens.download_state(1)[0] if (T == 1 or step % T == 0 or step >= 15) else None
        out.append((r[1]["match"], words, P))
    return out

a, b = run(4), run(1)
for k in range(len(a)):
    ma, wa, Pa = a[k]
    mb, wb, Pb = b[k]
    d = None if Pa is None else float(np.abs(Pa - Pb).max())
    print(k + 1, "T4", ma, "path", wa[9], "guess", wa[10:16], "| T1", mb, "path", wb[9], "guess", wb[10:16], "| Pdiff", d)
