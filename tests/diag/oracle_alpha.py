"""Round-5 diagnosis of SURVEY §8d's world on the CPU restatement only (oracle/, test infrastructure);
DESIGN.md §2.1. usage: PYTHONPATH=. python tests/diag/oracle_alpha.py [args]"""
import sys

import numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import scan_gen as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
N=4096
prof = None if sys.argv[1]=="bench" else "survey"
pre=int(sys.argv[2])
w=G.make_world(N); st=G.initial_state(w, profile=prof)
P0=st.dense_P()
def dtr(P, s):
    d=np.diag(P)[3:3+2*s]
    return d[0::2]+d[1::2]
for e in (0,7):
    r=O.OracleRobot(N, mode=O.FAST, omp=True)
    r.set_state(P0, st.y, st.saved, st.pose)
    out=[]
    for s in range(1,pre+49):
        enc, lines, nl = G.make_scan(w, s, instances=8, profile=prof)
        s0=r.savedLineCount
        tb=dtr(r.P_t0, s0) if s>pre else None
        m=r.localize(lines[e], enc[e])
        if s>pre:
            if r.savedLineCount>=s0 and s0>0 and not (r.savedLineCount==0):
                ta=dtr(r.P_t0, s0)
                a=np.max(tb/np.maximum(ta,1e-300))
            else: a=0
            out.append(a)
    print(e, " ".join("%.0e"%x for x in out), flush=True)
