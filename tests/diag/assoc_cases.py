"""Association-kernel cost in its bad cases (µs per scan, HIP events on every association kernel)
and how often the speculative path falls back, at the bench configuration (N = 4096, E = 8, fp32,
split-bf16 flush, T = 12):

  spec1   the default: speculative association, bench world (SURVEY §8d parameters tuned, scan_gen)
  spec0   speculate option 0: the sequential chain (one cross-workgroup exchange per line) every scan
  spec2   speculate option 2: every guess deliberately wrong — the full speculative path, its verdict
          fails, then the sequential restart (the worst case a wrong guess can cost)
  survey  SURVEY §8d literally (scan_gen profile "survey"), speculative
  surveyR the same with §8d's gate-margin rejection: a scan is redrawn while some candidate that
          instance 0's restatement evaluates has |sqrt(d²) − 0.4| < 1e-3

Per configuration: W warm-up scans, then K measured scans; reports the mean association-kernel time,
the fraction of (instance, scan) whose speculation failed its verdict or was unresolved (path code
bits 4/8, slam_ekf.h ekf_debug_result_words) or that ran the sequential path, matches per scan,
augmented landmarks and resets. usage: python tests/diag/assoc_cases.py [case ...] [--k K] [--n N]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("cases", nargs="*", default=["spec1", "spec0", "spec2", "survey", "surveyR"])
ap.add_argument("--k", type=int, default=48)
ap.add_argument("--w", type=int, default=12)
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--e", type=int, default=8)
ap.add_argument("--t", type=int, default=12)
args = ap.parse_args()

N, E, T = args.n, args.e, args.t
for case in args.cases:
    spec = {"spec0": "0", "spec2": "2"}.get(case, "1")
    profile = "survey" if case.startswith("survey") else None
    w = G.make_world(N)
    st = G.initial_state(w, profile=profile)
    ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=8, flush_interval=T, arith=ekf.ARITH_BF16X6,
                       options={"speculate": int(spec)})
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    ref = None
    if case == "surveyR":
        from oracle import oracle as O
        ref = O.OracleRobot(N, mode=O.FAST, omp=True)
        ref.set_state(*ens.download_state(0))
    stats = dict(scans=0, fallback=0, sequential=0, matches=0, added=0, resets=0, redraws=0, status=0)
    for s in range(1, args.w + args.k + 1):
        if s == args.w + 1:
            ens.sync()
            ens.profile(2)
        redraw = 0
        while True:
            enc, lines, nl = G.make_scan(w, s, instances=E, profile=profile, redraw=redraw)
            if ref is None:
                break
            probe = O.OracleRobot(N, mode=O.FAST, omp=True)
            P, y, sv, pose = ref.P_t0, ref.y, ref.savedLineCount, ref.pose
            probe.set_state(P, y, sv, pose)
            probe.localize(lines[0], enc[0])
            if probe.gate_margin >= 1e-3 or redraw >= 20:
                ref = probe
                break
            redraw += 1
        stats["redraws"] += redraw if s > args.w else 0
        res = ens.localize(enc, lines, nl)
        if s <= args.w:
            continue
        for e in range(E):
            code = ens.result_words(e)[9]
            stats["scans"] += 1
            stats["fallback"] += 1 if code & 12 else 0
            stats["sequential"] += 1 if code & 16 else 0
            stats["matches"] += res[e]["matches"]
            stats["added"] += res[e]["new_landmarks"]
            stats["resets"] += res[e]["reset"]
            stats["status"] |= res[e]["status"]
    prof = ens.profile_read()
    ens.profile(0)
    ens.close()
    sc = stats["scans"]
    print(json.dumps({"case": case, "N": N, "E": E, "T": T, "speculate": int(spec), "world": profile or "bench",
                      "scan_us": prof["scan_ms"] * 1e3, "flush_ms": prof["downdate_ms"],
                      "fallback_frac": stats["fallback"] / sc, "sequential_frac": stats["sequential"] / sc,
                      "matches_per_scan": stats["matches"] / sc, "new_landmarks_per_scan": stats["added"] / sc,
                      "resets": stats["resets"], "redraws": stats["redraws"], "status_or": stats["status"]}),
          flush=True)
