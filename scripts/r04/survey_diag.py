"""SURVEY §8d world at the bench shape (N = 4096, E = 8, L = 8, split-fp16, T from argv): after a
preroll of scans, per scan the association path word (RES_DBG: 16 sequential, 64 exact pending
replay, 128 a pending reset; 1 fast guess, 2 collision-resolved, 4 unresolved, 8 verdict
failed, 32 a guessed winner failed, 256 a pending plane exponent other than the scan's) and the map size,
as a histogram per position in the flush group. usage: python scripts/r04/survey_diag.py [T] [preroll] [scans]"""
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pre = int(sys.argv[2]) if len(sys.argv) > 2 else 200
scans = int(sys.argv[3]) if len(sys.argv) > 3 else 60
N, E = 4096, 8
w = G.make_world(N)
st = G.initial_state(w, profile="survey")
ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, flush_interval=T, arith=ekf.ARITH_F16X3)
for e in range(E):
    ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
bits = Counter()
per_inst = {e: Counter() for e in range(E)}
flags = Counter()
words = Counter()
per_pos = {}
saved = []
for s in range(1, pre + scans + 1):
    enc, lines, nl = G.make_scan(w, s, instances=E, profile="survey")
    r = ens.localize(enc, lines, nl)
    if s <= pre:
        continue
    pos = (s - 1) % T
    for e in range(E):
        dw = int(ens.result_words(e)[9])
        words[dw] += 1
        if dw & 16:
            per_inst[e]["sequential"] += 1
        if r[e]["status"] & (ekf.ST_PRECISION | ekf.ST_RANGE):
            flags[e] += 1
        for b in (1, 2, 4, 8, 16, 32, 64, 128, 256):
            if dw & b:
                bits[b] += 1
                per_pos.setdefault(pos, Counter())[b] += 1
    saved.append([x["saved"] for x in r])
print(json.dumps({"T": T, "preroll": pre, "scans": scans, "instances": E, "bits": dict(bits), "words": dict(words),
                  "per_group_position": {k: dict(v) for k, v in sorted(per_pos.items())},
                  "saved_first": saved[0], "saved_last": saved[-1],
                  "sequential_per_instance": {e: c["sequential"] for e, c in per_inst.items()},
                  "flagged_scans_per_instance": dict(flags)}), flush=True)
ens.close()
