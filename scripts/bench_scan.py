"""Decompose the association kernel's cost: vary active landmarks s and lines L (N=4096 f32)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from slam_ros_amd import ekf, scan_gen as G

N = int(os.environ.get("N", 4096)); E = 8
out = []
for active, L in ((N - 10, 8), (N - 10, 4), (N - 10, 1), (N - 10, 0), (512, 8), (64, 8)):
    w = G.make_world(N, active=active); st = G.initial_state(w)
    ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, pipeline=bool(int(os.environ.get("PIPE", "0"))))
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    enc, lines, nl = G.make_scan(w, 1, instances=E, lines=8)
    nl[:] = L
    ens.localize(enc, lines, nl)
    ens.profile(True)
    for s in range(2, 12):
        enc, lines, nl = G.make_scan(w, s, instances=E, lines=8); nl[:] = L
        r = ens.localize(enc, lines, nl)
    p = ens.profile_read()
    p.update(active=active, L=L, matches=[x["matches"] for x in r])
    out.append(p); print(json.dumps(p), flush=True)
    ens.close()
