"""Round-5 diagnosis of SURVEY §8d's world on the CPU restatement only (oracle/, test infrastructure);
DESIGN.md §2.1. usage: PYTHONPATH=. python tests/diag/oracle_steady.py [args]"""
import numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import scan_gen as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
N=4096
w=G.make_world(N); st=G.initial_state(w, profile="survey")
P0=st.dense_P()
for e in range(8):
    r=O.OracleRobot(N, mode=O.FAST, omp=True)
    r.set_state(P0, st.y, st.saved, st.pose)
    for s in range(1,201):
        enc, lines, nl = G.make_scan(w, s, instances=8, profile="survey")
        r.localize(lines[e], enc[e])
    P=r.P_t0
    print(e, "pose", r.pose, "enc", enc[e], "Prob %.3e trP %.3e |y| %.3e saved %d"%(np.abs(P[:3,:3]).max(), np.trace(P), np.linalg.norm(r.y), r.savedLineCount), flush=True)
