"""Association-kernel phase timers (EKF_OPT_SCAN_STAMPS = 1; thread 0 of workgroup 0 of each instance,
s_memrealtime, 100 MHz), µs per launch averaged over instances, at the bench's shapes
(f32, E = 8, L = m = 8; split-bf16 arithmetic, PROBE_ARITH=exact / f16x3 for the others).
usage: python scripts/assoc_probe.py [N:T ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slam_ros_amd import ekf, scan_gen as G  # noqa: E402

NAMES = {0: "predict+state", 1: "diag+ctl", 5: "guess", 2: "exchange1", 10: "resolve",
         12: "records+stage", 11: "staged_replay(w0)", 13: "replay_wave_total", 3: "rw_eval+publish",
         4: "rw_gain+robot", 16: "lw_gate", 17: "lw_wait_pkg", 18: "lw_gain+store", 19: "lw_robot",
         14: "landmark_total", 6: "verdict", 27: "commit:augment", 28: "commit:state", 24: "commit:operands", 25: "commit:planes", 26: "commit:collect",
         7: "commit:record", 8: "total", 15: "fallbacks"}
E = int(os.environ.get("PROBE_E", "8"))
cfgs = sys.argv[1:] or ["4096:8", "4096:1", "1024:8"]
for c in cfgs:
    N, T = (int(x) for x in c.split(":"))
    world = os.environ.get("PROBE_WORLD") or None   # "survey": SURVEY §8d's literal world
    w = G.make_world(N)
    st = G.initial_state(w, profile=world)
    arith = {"exact": ekf.ARITH_EXACT, "f16x3": ekf.ARITH_F16X3}.get(os.environ.get("PROBE_ARITH"), ekf.ARITH_BF16X6)
    prec = {"f64": ekf.PREC_F64, "f16": ekf.PREC_F16}.get(os.environ.get("PROBE_PREC"), ekf.PREC_F32)
    if prec == ekf.PREC_F64:
        arith = ekf.ARITH_EXACT
    ens = ekf.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=arith,
                       options={"scan_stamps": 1, **({"scan_threads": int(os.environ["PROBE_NT"])} if os.environ.get("PROBE_NT") else {})})
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    base = ens.scan_stamps()
    for s in range(1, 25):
        enc, lines, nl = G.make_scan(w, s, instances=E, profile=world)
        r = ens.localize(enc, lines, nl)
        if not os.environ.get("PROBE_NOASSERT") and not world:
            assert all(x["matches"] == 8 for x in r)
    stp = [a - b for a, b in zip(ens.scan_stamps(), base)]
    n = stp[9] or 1
    out = {v: round(stp[k] * 10e-3 / n, 2) for k, v in NAMES.items()}
    out["fallbacks"] = stp[15]
    out["after_records:rw_start"] = round(stp[29] * 10e-3 / n, 2)   # replay wave's chain starts
    out["after_records:rw_end"] = round(stp[30] * 10e-3 / n, 2)     # ... ends
    out["after_records:lw0_end"] = round(stp[31] * 10e-3 / n, 2)    # landmark wave 0 done
    out["gate_waves"] = stp[22]                  # (wave, line) gate evaluations, workgroup 0
    out["past_quick_filter"] = stp[20]           # ... with a lane past the quick certified filter
    out["past_f32_filter"] = stp[21]             # ... past the fp32 certified filter
    out["past_f64_filter"] = stp[23]             # ... and past the fp64 one (exact evaluation)
    an = {ekf.ARITH_EXACT: "exact", ekf.ARITH_BF16X6: "bf16x6", ekf.ARITH_F16X3: "f16x3"}[arith]
    print(json.dumps({"N": N, "T": T, "E": E, "arith": an, "precision": os.environ.get("PROBE_PREC", "f32"),
                      "world": world or "bench", "launches_x_instances": stp[9],
                      "us": out}), flush=True)
    ens.close()
