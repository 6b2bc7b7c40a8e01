"""Round-5 diagnosis of SURVEY §8d's world on the CPU restatement only (oracle/, test infrastructure);
DESIGN.md §2.1. usage: PYTHONPATH=. python tests/diag/oracle_fp32store.py [args]"""
"""Intrinsic error of fp32 storage in the survey world: the fp64 restatement with its landmark block
re-rounded to fp32 after every scan vs the plain fp64 restatement, both re-synced at group ends."""
import sys
import time

import numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import scan_gen as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
N=4096; T=int(sys.argv[1]) if len(sys.argv)>1 else 16
w=G.make_world(N); st=G.initial_state(w, profile="survey")
P0=st.dense_P()
def r32(P):
    Q=P.copy(); Q[3:,3:]=P[3:,3:].astype(np.float32); return Q
def rel(a,b): return np.linalg.norm(a-b)/np.linalg.norm(b)
for e in (0,7):
    a=O.OracleRobot(N, mode=O.FAST, omp=True); b=O.OracleRobot(N, mode=O.FAST, omp=True)
    P=r32(P0); a.set_state(P, st.y, st.saved, st.pose); b.set_state(P, st.y, st.saved, st.pose)
    for s in range(1,49):
        enc, lines, nl = G.make_scan(w, s, instances=8, profile="survey")
        ma=a.localize(lines[e], enc[e]); mb=b.localize(lines[e], enc[e])
        Pb=r32(b.P_t0); b.set_state(Pb, b.y, b.savedLineCount, b.pose)
        if ma!=mb: print(f"e{e} scan {s}: association differs {ma} {mb}")
        if s%T==0:
            print(f"e{e} group end {s}: fp32-storage vs fp64: P {rel(b.P_t0,a.P_t0):.2e} y {rel(b.y,a.y):.2e}", flush=True)
            a.set_state(b.P_t0, b.y, b.savedLineCount, b.pose)
