"""Per-step divergence of the split-bf16 context (T) from the exact arithmetic drained per scan,
with and without the MFMA replay (EKF_MFREP), to locate a failing configuration."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import ekf, scan_gen as G

def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))

for (N, T, lines, xe) in [(256, 16, 6, 7), (256, 16, 6, 0), (80, 16, 7, 0), (256, 8, 6, 7), (1024, 12, 8, 0)]:
    for mf in ("1", "0"):
        os.environ["EKF_MFREP"] = mf
        E = 3
        w = G.make_world(N, active=N - 14 if xe else N - 10)
        st = G.initial_state(w)
        a = ekf.Ensemble(N, E, 1, max_lines=8, flush_interval=T, arith=ekf.ARITH_BF16X6)
        b = ekf.Ensemble(N, E, 1, max_lines=8)
        for ens in (a, b):
            for e in range(E):
                ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
        rng = np.random.default_rng(5)
        out = []
        for step in range(1, 3 * T + 2):
            enc, ln, nl = G.make_scan(w, step, instances=E, lines=lines)
            if xe and step % xe == 0:
                ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
                ln = np.concatenate([ln, ex], axis=1)
                nl = np.full(E, ln.shape[1], dtype=np.int32)
            ra = a.localize(enc, ln, nl)
            rb = b.localize(enc, ln, nl)
            out.append((step, float(np.abs(ra[0]["pose"] - rb[0]["pose"]).max()), ra[0]["matches"], ra[0]["reset"],
                        ra[0]["match"] == rb[0]["match"]))
        Pa = a.download_state(0)[0]; Pb = b.download_state(0)[0]
        print(f"N={N} T={T} L={lines} xe={xe} mf={mf}: P {rel(Pa, Pb):.2e}", flush=True)
        print("  pose per step:", " ".join(f"{s}:{r:.1e}{'' if ok else '!'}" for s, r, m, rs, ok in out), flush=True)
        a.close(); b.close()
