"""Debug: the deferred-flush scenario of test_deferred_flush_equals_drained (N=64, E=2, fp32,
T=4) under EKF_SPECULATE=1 and 0; prints per-step associations of both instances and the
first step where deferred and drained disagree, plus the P difference after each step."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G

def run(spec, T, steps=20, prec=1):
    os.environ["EKF_SPECULATE"] = str(spec)
    N = 64
    w = G.make_world(N, active=N - 14)
    st = G.initial_state(w)
    ens = ekf.Ensemble(N, 2, prec, max_lines=8, flush_interval=T)
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
        if T == 1:
            ens.download_state(0, with_P=False)
        Ps = [ens.download_state(e)[0] for e in range(2)] if T == 1 or step % T == 0 else None
        out.append(([x["match"] for x in r], [x["status"] for x in r], Ps))
    ens.close()
    return out

res = {(s, T): run(s, T) for s in (1, 0) for T in (1, 4)}
for step in range(20):
    row = {k: v[step][0] for k, v in res.items()}
    same = len({str(x) for x in row.values()}) == 1
    print(step + 1, "same" if same else "DIFF", row if not same else row[(1, 1)], [v[step][1] for v in res.values()])
    for T in (4,):
        for s in (1, 0):
            Pa = res[(s, T)][step][2]
            if Pa is not None:
                Pb = res[(s, 1)][step][2]
                print("   P spec=%d T=%d vs T=1: maxdiff e0 %.3g e1 %.3g" % (s, T, np.abs(Pa[0] - Pb[0]).max(), np.abs(Pa[1] - Pb[1]).max()))
