"""SURVEY §8d world at the bench shape (N = 4096, E = 8, L = 8, split-fp16, T from argv): after a
preroll, per instance-scan the association path (RES_DBG) and, for a restart after a failed verdict
(bit 8), the first violating line (bits 10..12; bit 512: lines before it kept) and, for a line < 5,
how the guess (RES_DBG + 1 + t) differs from the true match. The full record is
read with read_results (a synchronous call mirrors only ekf_result's words).
usage: python scripts/r06/restart_diag.py [T] [preroll] [scans] > out.json"""
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
first = Counter()
kind = Counter()   # at the first violating line t (t < 5): the guess against the true match
words = Counter()
per_inst = Counter()
matches = Counter()
n = 0
for s in range(1, pre + scans + 1):
    enc, lines, nl = G.make_scan(w, s, instances=E, profile="survey")
    ens.localize(enc, lines, nl)
    if s <= pre:
        continue
    res = ens.read_results()
    for e in range(E):
        dw = int(ens.result_words(e)[9])
        n += 1
        words[dw & 1023] += 1
        if dw & 8:
            t = (dw >> 10) & 7
            first[t] += 1
            if t < 5:
                words16 = ens.result_words(e)
                guess, true = int(words16[10 + t]), int(res[e]["match"][t])
                k = ("no_guess" if guess < 0 else "guess_failed_other_passed" if true < 0 or true > guess
                     else "smaller_landmark_passed" if true < guess else "guess_right_earlier_state_differs")
                kind[f"line{t}:{k}"] += 1
            per_inst[e] += 1
            matches[res[e]["matches"]] += 1
        if dw & 16 and not dw & 8:
            first["seq_no_verdict"] += 1
print(json.dumps({"T": T, "preroll": pre, "scans": scans, "instance_scans": n,
                  "restarts": sum(v for k, v in first.items() if k != "seq_no_verdict"),
                  "first_line": {str(k): v for k, v in sorted(first.items(), key=str)},
                  "restarts_per_instance": {str(k): v for k, v in sorted(per_inst.items())},
                  "violation_kind": dict(sorted(kind.items())),
                  "matches_of_restarted": {str(k): v for k, v in sorted(matches.items())},
                  "words": {str(k): v for k, v in words.most_common()}}, indent=1))
