"""GPU parity at the configurations bench.py times, with no intermediate drains.

BASELINE config 4 per GPU: N = 4096 landmarks (n = 8195), E = 8 instances, L = m = 8 matched lines
per scan, the deferred flush schedule (T = 8: flush_f32_wave_kernel<float, 8> on every full group),
inputs resident in HBM through ekf_localize_device — exactly the bench's call sequence. 16 scans =
two full flush groups. The restatement (oracle/, fast mode; its OpenMP build, bit-identical) starts
from the GPU's own stored (rounded) start state for instances 0 and 7 and then runs the same 16
scans on its own — never re-synchronised — which is the sequential chain of Robot.cpp:298-641 per
scan that the deferral replaces.

Checked: the association of every scan (ekf_read_results after each scan only synchronises the
stream: no flush is added), status == 0 (no singular S, no capacity, no exchange timeout), and
after each group end the full P, y and pose of both instances.

Bound on P over k scans: the per-scan bar is 1e-6 (BASELINE.json north_star); rounding to the
storage precision enters once per scan and (I − K·H) does not amplify earlier errors, so after k
scans ‖ΔP‖_F/‖P‖_F ≤ k · (per-scan bar). A second restatement is re-synced to the GPU state at every
group end (the only points where the schedule materialises P), so each flush group runs from
identical inputs: that group error is held to the per-scan bar itself — fp32 1e-6, fp16 storage
(config 5) its re-stated 1e-3, fp64 storage 1e-10 — and the
trajectory to k times it (fp32 measured 3.1e-7 after 8 scans, 4.6e-7 after 16 at N = 4096;
1.06e-6 after 20 at N = 256). State vector: ‖Δy‖/‖y‖ ≤ 1e-8, and the pose
(y[0:3]) within the same absolute amount, 1e-8·‖y‖ (fp64: 1e-12). The measured values are
written to gpurun_out/bench_config_parity.json.
"""
import json
import os

import numpy as np
import pytest

from slam_ros_amd import dist as D, scan_gen as G

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, E, L = 4096, 8, 8
CHECK = (0, 7)
PER_SCAN = {0: 1e-10, 1: 1e-6, 2: 1e-3}


def rel(a, b):
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


def record(key, value):
    path = os.path.join(ROOT, "gpurun_out", "bench_config_parity.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[key] = value
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(data, f, indent=1, default=lambda o: o.item() if hasattr(o, "item") else str(o))
    os.replace(tmp, path)


def run_config(ekf_mod, oracle_mod, prec, T, scans, pipeline=False, arith=0, N=N):
    from tests.hipmem import DeviceArray
    world = G.make_world(N)
    st = G.initial_state(world)
    ens = ekf_mod.Ensemble(N, E, prec, max_lines=L, flush_interval=T, pipeline=pipeline, arith=arith)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    refs, grps = {}, {}
    for e in CHECK:
        P0, y0, s0, pose0 = ens.download_state(e)       # the GPU's rounded start state
        refs[e] = oracle_mod.OracleRobot(N, mode=oracle_mod.FAST, omp=True)
        refs[e].set_state(P0, y0, s0, pose0)
        grps[e] = oracle_mod.OracleRobot(N, mode=oracle_mod.FAST, omp=True)
        grps[e].set_state(P0, y0, s0, pose0)
        del P0
    host = np.stack([D.pack(*G.make_scan(world, s + 1, instances=E, lines=L)[:2]) for s in range(scans)])
    payload = DeviceArray(host)
    nlines = DeviceArray(np.full(E, L, dtype=np.int32))
    eo, lo = D.offsets(E, L, 0)
    out = {"P": [], "y": [], "pose": [], "P_group": [], "y_group": []}
    for s in range(scans):
        base = payload.address + s * host.shape[1] * 8
        ens.localize_device(base + eo * 8, base + lo * 8, nlines.address)
        res = ens.read_results()                        # stream sync only: no flush added
        for e in CHECK:
            ln_e, enc_e = host[s, lo + e * L * 6: lo + (e + 1) * L * 6].reshape(L, 6), host[s, e * 3: e * 3 + 3]
            m = refs[e].localize(ln_e, enc_e)
            assert grps[e].localize(ln_e, enc_e) == m
            assert res[e]["match"] == m, (prec, s, e, res[e]["match"], m)
            assert res[e]["matches"] == L
        assert all(r["status"] == 0 for r in res), [r["status"] for r in res]
        if (s + 1) % T == 0 or s + 1 == scans:         # a group end: the flush has run
            k = s + 1
            if k % T:
                ens.sync()                              # the partial last group (bench's ekf_sync)
            for e in CHECK:
                P, y, saved, pose = ens.download_state(e)
                rp, ry = rel(P, refs[e].P_t0), rel(y, refs[e].y)
                rg, ryg = rel(P, grps[e].P_t0), rel(y, grps[e].y)
                dp = float(np.abs(pose - refs[e].pose).max())
                grps[e].set_state(P, y, saved, pose)     # the next group from identical inputs
                del P
                out["P"].append(rp)
                out["y"].append(ry)
                out["pose"].append(dp)
                out["P_group"].append(rg)
                out["y_group"].append(ryg)
                bound = PER_SCAN[prec]
                # the group from identical inputs: the per-scan bar; the never re-synced trajectory:
                # k scans of it (module docstring); both recorded
                assert rg <= bound, (prec, k, e, rg, bound)
                assert ryg <= 1e-8, (prec, k, e, ryg)
                assert rp <= bound * k, (prec, k, e, rp, bound * k)
                assert ry <= 1e-8 * k, (prec, k, e, ry)
                assert dp <= (1e-12 if prec == 0 else 1e-8 * np.linalg.norm(refs[e].y)), (prec, k, e, dp)
    ens.close()
    payload.close()
    nlines.close()
    return out


def test_bench_config_fp32_t8(ekf_mod, oracle_mod):
    out = run_config(ekf_mod, oracle_mod, 1, 8, 16)
    record("f32_T8_N4096_E8", out)


def test_bench_config_fp32_t8_pipelined(ekf_mod, oracle_mod):
    """pipeline = 1 at G = 22 cooperating workgroups per instance: such a context runs the
    sequential schedule (slam_ekf.h ekf_config.pipeline), so the results are those of T = 8."""
    out = run_config(ekf_mod, oracle_mod, 1, 8, 16, pipeline=True)
    record("f32_T8_N4096_E8_pipelined", out)


def test_bench_config_fp16_t8(ekf_mod, oracle_mod):
    out = run_config(ekf_mod, oracle_mod, 2, 8, 16)
    record("f16_T8_N4096_E8", out)


def test_bench_config_fp64_t4(ekf_mod, oracle_mod):
    out = run_config(ekf_mod, oracle_mod, 0, 4, 8)
    record("f64_T4_N4096_E8", out)


def test_bench_config_fp32_t8_bf16x6(ekf_mod, oracle_mod):
    """EKF_ARITH_BF16X6 (the split-bf16 flush, flush_f32_wave_kernel<float, NS, true>) over the
    bench's exact step count: 20 scans = two groups of 8 and a partial group of 4 flushed by
    ekf_sync. The same per-scan bar (1e-6 on P, 1e-8 on y) against the fp64 restatement."""
    out = run_config(ekf_mod, oracle_mod, 1, 8, 20, arith=ekf_mod.ARITH_BF16X6)
    record("f32_T8_N4096_E8_bf16x6", out)


def test_bench_config_fp32_t8_bf16x6_pipelined(ekf_mod, oracle_mod):
    out = run_config(ekf_mod, oracle_mod, 1, 8, 16, pipeline=True, arith=ekf_mod.ARITH_BF16X6)
    record("f32_T8_N4096_E8_bf16x6_pipelined", out)


@pytest.mark.parametrize("n_cap", [256, 1024, 4096])
def test_bench_config_fp32_t12_bf16x6(ekf_mod, oracle_mod, n_cap):
    """bench.py's default schedule at every capacity BASELINE names (configs 2, 3 and 4's per-GPU
    slice): EKF_ARITH_BF16X6 at T = 12, E = 8, over the driver's 20 timed steps (a group of 12, then
    8 flushed by ekf_sync), no intermediate drains; up to 11 pending steps replayed on read by MFMA
    on the operand planes. Instances 0 and 7 against the restatement, never re-synchronised."""
    out = run_config(ekf_mod, oracle_mod, 1, 12, 20, arith=ekf_mod.ARITH_BF16X6, N=n_cap)
    record(f"f32_T12_N{n_cap}_E8_bf16x6", out)


@pytest.mark.parametrize("n_cap,prec,T", [(256, 1, 16), (1024, 1, 16), (4096, 1, 16), (4096, 1, 12), (4096, 2, 16),
                                          (1024, 1, 12), (4096, 1, 20), (4096, 1, 24), (1024, 1, 24)])
def test_bench_config_f16x3(ekf_mod, oracle_mod, n_cap, prec, T):
    """EKF_ARITH_F16X3 (operands split into hi + lo fp16 of 2^σ·V, three fp16 MFMA products, the
    MFMA replay on the same planes) at T = 12 to 24, E = 8 over 20 scans with no
    intermediate drains (a group of T, then the rest flushed by ekf_sync): the fp32 bar (1e-6 on P,
    1e-8 on y; fp16 storage its re-stated 1e-3) per group against the re-synced restatement, the
    trajectory to k times it, association identical."""
    out = run_config(ekf_mod, oracle_mod, prec, T, 20, arith=ekf_mod.ARITH_F16X3, N=n_cap)
    record(f"{'f32' if prec == 1 else 'f16'}_T{T}_N{n_cap}_E8_f16x3", out)


def test_bench_config_fp32_t16_bf16x6(ekf_mod, oracle_mod):
    out = run_config(ekf_mod, oracle_mod, 1, 16, 20, arith=ekf_mod.ARITH_BF16X6)
    record("f32_T16_N4096_E8_bf16x6", out)


def test_bench_config_fp16_t12_bf16x6(ekf_mod, oracle_mod):
    """fp16 storage (BASELINE config 5) with the split-bf16 flush (flush_f32_wave_kernel<_Float16,
    NS, true>: tiles scaled out of the storage exponent on load, rounded to fp16 once per group)
    and the MFMA replay of the pending steps, T = 12 over 20 scans: P within the re-stated 1e-3 at
    every group end, y within 1e-8, association identical."""
    out = run_config(ekf_mod, oracle_mod, 2, 12, 20, arith=ekf_mod.ARITH_BF16X6)
    record("f16_T12_N4096_E8_bf16x6", out)


def test_bench_config_fp16_t8_bf16x6(ekf_mod, oracle_mod):
    out = run_config(ekf_mod, oracle_mod, 2, 8, 20, arith=ekf_mod.ARITH_BF16X6)
    record("f16_T8_N4096_E8_bf16x6", out)


def run_survey(ekf_mod, oracle_mod, prec, T, scans, arith, N=N):
    """SURVEY §8d's literal world (scan_gen profile "survey": R = 9e-4, σ_z = 1e-2, P₀ 0.05 / 1e-3):
    most lines fail the 0.4 gate and become new landmarks, the map fills and resets. Per flush group
    from identical inputs (the restatement re-synced to the GPU state at every group end: a
    trajectory through a map reset is chaotic, SURVEY §8d's contract is per scan from identical
    inputs); association and status of every scan; how many scans took the sequential path."""
    from tests.hipmem import DeviceArray
    world = G.make_world(N)
    st = G.initial_state(world, profile="survey")
    ens = ekf_mod.Ensemble(N, E, prec, max_lines=L, flush_interval=T, arith=arith)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    refs = {}
    for e in CHECK:
        refs[e] = oracle_mod.OracleRobot(N, mode=oracle_mod.FAST, omp=True)
        refs[e].set_state(*ens.download_state(e))
        refs[e].set_prediction(PRED_ETA)
    host = np.stack([D.pack(*G.make_scan(world, s + 1, instances=E, lines=L, profile="survey")[:2])
                     for s in range(scans)])
    payload = DeviceArray(host)
    nlines = DeviceArray(np.full(E, L, dtype=np.int32))
    eo, lo = D.offsets(E, L, 0)
    out = {"P": [], "y": [], "sequential": 0, "scans": 0, "matches": 0, "added": 0, "resets": 0,
           "dpath": {}}   # association path words: 1 fast guess, 2 collision-resolved, 4 unresolved, 8 verdict failed, 16 sequential
    flagged = {e: False for e in CHECK}
    for s in range(scans):
        base = payload.address + s * host.shape[1] * 8
        ens.localize_device(base + eo * 8, base + lo * 8, nlines.address)
        res = ens.read_results()
        for e in range(E):
            dw = int(ens.result_words(e)[9])
            out["sequential"] += 1 if dw & 16 else 0
            out["dpath"][str(dw)] = out["dpath"].get(str(dw), 0) + 1
            out["scans"] += 1
            out["matches"] += res[e]["matches"]
            out["added"] += res[e]["new_landmarks"]
            out["resets"] += res[e]["reset"]
        flag_bits = ekf_mod.ST_PRECISION | ekf_mod.ST_RANGE
        for e in CHECK:
            m = refs[e].localize(host[s, lo + e * L * 6: lo + (e + 1) * L * 6].reshape(L, 6),
                                 host[s, e * 3: e * 3 + 3])
            if not flagged[e]:   # (identical inputs up to here: the library's flags vs the prediction)
                check_flags(ekf_mod, oracle_mod, res[e]["status"], refs[e].pred_flags, (prec, s, e))
            assert res[e]["match"] == m, (prec, s, e, res[e]["match"], m)
            assert res[e]["saved"] == refs[e].savedLineCount, (s, e)
        # (EKF_ST_PRECISION / EKF_ST_RANGE: the library's statement that the fp32 block no longer
        # resolves the fp64 reference there, DESIGN §2.1, each one checked against the restatement's
        # prediction above; such an instance-group's P is exempt below)
        assert all(r["status"] & ~(ekf_mod.ST_CAPACITY | flag_bits) == 0 for r in res), [r["status"] for r in res]
        for e in CHECK:
            flagged[e] |= bool(res[e]["status"] & flag_bits) or bool(refs[e].pred_flags)
        if (s + 1) % T == 0 or s + 1 == scans:
            for e in CHECK:
                P, y, saved, pose = ens.download_state(e)
                rp, ry = rel(P, refs[e].P_t0), rel(y, refs[e].y)
                out["P"].append(rp)
                out["y"].append(ry)
                if not flagged[e]:
                    assert rp <= PER_SCAN[prec], (prec, s, e, rp)
                    assert ry <= 1e-8, (prec, s, e, ry)
                flagged[e] = False
                refs[e].set_state(P, y, saved, pose)   # the next group from identical inputs
                del P
    ens.close()
    payload.close()
    nlines.close()
    return out


@pytest.mark.parametrize("arith", [1, 2])
def test_survey_world_association(ekf_mod, oracle_mod, arith):
    """SURVEY §8d literally at N = 4096, E = 8, T = 12, 24 scans: associations
    identical to the restatement on every scan, P per group within the fp32 bar, and the
    speculative association falls back to the sequential path on at most 10 % of the scans (eight
    guessed candidates per workgroup and line resolve every line's guess)."""
    out = run_survey(ekf_mod, oracle_mod, 1, 12, 24, arith)
    record(f"survey_f32_T12_N4096_E8_{'bf16x6' if arith == 1 else 'f16x3'}", out)
    assert out["added"] > 0
    assert out["sequential"] <= 0.10 * out["scans"], out


# The storage precision the library's flags assume for fp32 storage (gate_eta, ekf_kernels.hip):
# the restatement predicts from its own fp64 state which decisions a state that far from it cannot
# resolve (oracle_set_pred), with 3x the library's eta (the GPU and the restatement differ by up to
# the P bar, 2^-4 of eta, plus the library's fp32 square roots)
PRED_ETA = 3 * 2.0 ** -16


def check_flags(ekf_mod, oracle_mod, status, pred, where):
    """The library's EKF_ST_PRECISION / EKF_ST_RANGE on a scan must be ones the restatement
    predicts on the same inputs: a precision flag needs a predicted unresolved gate decision or
    cancellation, a range flag a predicted out-of-range variance (GPU flags ⊆ oracle flags)."""
    if status & ekf_mod.ST_PRECISION:
        assert pred & (oracle_mod.PRED_GATE | oracle_mod.PRED_CANCEL), ("unpredicted EKF_ST_PRECISION", where, pred)
    if status & ekf_mod.ST_RANGE:
        assert pred & oracle_mod.PRED_RANGE, ("unpredicted EKF_ST_RANGE", where, pred)


def run_survey_parity(ekf_mod, oracle_mod, arith, T, pre, scans, N=N, options=None):
    """SURVEY §8d's world through the bench's schedule (E = 8, no drains inside a group), the
    restatement re-synced to the GPU per scan for y and the pose (committed every scan, read
    without a drain) and per group for the whole state.

    Which instance-scans are exempt is the restatement's decision, not the library's: on its own
    fp64 state it predicts the decisions a stored state within the library's precision cannot
    resolve (a gate distance within eta of the gate, an update cancelling more than 4 bits, a
    variance past fp32's range: PRED_*). Every flag the library raises (EKF_ST_PRECISION,
    EKF_ST_RANGE) must be one the restatement predicts on the same inputs; every scan it does not
    predict is held to the bar — association identical, no flag, y per scan ≤ 1e-8 — and so is P
    at the end of every group with no predicted scan. After a predicted scan the rest of its group
    is exempt (the two states may then differ beyond the bar until the group end re-syncs them)."""
    world = G.make_world(N)
    st = G.initial_state(world, profile="survey")
    ens = ekf_mod.Ensemble(N, E, 1, max_lines=L, flush_interval=T, arith=arith, options=options or {})
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    for s in range(1, pre + 1):
        enc, lines, nl = G.make_scan(world, s, instances=E, lines=L, profile="survey")
        ens.localize(enc, lines, nl)
    refs = {}
    for e in CHECK:
        refs[e] = oracle_mod.OracleRobot(N, mode=oracle_mod.FAST, omp=True)
        refs[e].set_state(*ens.download_state(e))
        refs[e].set_prediction(PRED_ETA)
    tainted = {e: False for e in CHECK}
    out = {"y_scan": [], "P_group": [], "groups": 0, "groups_unchecked": 0, "instance_scans": 0,
           "assoc_checked": 0, "oracle_predicted": 0, "exempt_after_prediction": 0, "gpu_flagged": 0,
           "gpu_flagged_checked_against_prediction": 0}
    bad = ekf_mod.ST_PRECISION | ekf_mod.ST_RANGE
    for k in range(scans):
        enc, lines, nl = G.make_scan(world, pre + k + 1, instances=E, lines=L, profile="survey")
        res = ens.localize(enc, lines, nl)
        for e in CHECK:
            m = refs[e].localize(lines[e], enc[e])
            pred = refs[e].pred_flags
            gst = res[e]["status"]
            out["instance_scans"] += 1
            out["gpu_flagged"] += bool(gst & bad)
            assert gst & ~(bad | ekf_mod.ST_CAPACITY) == 0, (k, e, gst)
            _, yg, sg, pg = ens.download_state(e, with_P=False)
            if tainted[e]:
                out["exempt_after_prediction"] += 1
            else:
                # identical inputs (y and pose re-synced every scan, P at every group end)
                check_flags(ekf_mod, oracle_mod, gst, pred, (arith, T, pre, k, e))
                out["gpu_flagged_checked_against_prediction"] += bool(gst & bad)
                if pred:
                    out["oracle_predicted"] += 1
                    tainted[e] = True
                else:
                    assert res[e]["match"] == m, (arith, T, pre, k, e, res[e]["match"], m)
                    ry = rel(yg, refs[e].y)
                    out["y_scan"].append(ry)
                    out["assoc_checked"] += 1
                    assert ry <= 1e-8, (arith, T, pre, k, e, ry)
            refs[e].set_state(None, yg, sg, pg)
        if (k + 1) % T == 0 or k + 1 == scans:
            for e in CHECK:
                P, y, saved, pose = ens.download_state(e)
                out["groups"] += 1
                if tainted[e]:
                    out["groups_unchecked"] += 1
                else:
                    rp = rel(P, refs[e].P_t0)
                    out["P_group"].append(rp)
                    assert rp <= PER_SCAN[1], (arith, T, pre, k, e, rp)
                refs[e].set_state(P, y, saved, pose)
                tainted[e] = False
                del P
    ens.close()
    # every instance-scan is accounted for: checked, the restatement's prediction, or after one
    assert out["assoc_checked"] + out["oracle_predicted"] + out["exempt_after_prediction"] == out["instance_scans"], out
    return out


@pytest.mark.parametrize("arith,T,rep", [(2, 20, 1), (2, 24, 1), (2, 20, 2), (1, 16, 1), (0, 16, 1)])
def test_survey_world_parity_from_init(ekf_mod, oracle_mod, arith, T, rep):
    """VERDICT r04 Missing #1: the split arithmetics at the bench's T in SURVEY §8d's world, from
    the initial state over 48 scans (augmentation, the reset, the robot's heading starting to run
    away): every instance-group not flagged by the library meets the bar. rep: the on-read replay
    (EKF_OPT_MFMA_REPLAY: 1 the split products on the planes, 2 fp32 MFMA)."""
    out = run_survey_parity(ekf_mod, oracle_mod, arith, T, 0, 48, options={"mfma_replay": rep})
    record(f"survey_parity_init_a{arith}_T{T}_rep{rep}", out)
    # from the initial state the restatement predicts one unresolved scan per instance (scan 30:
    # instance 0's gate, instance 7's cancellation; CPU restatement alone): few predictions, each
    # exempting at most the rest of its flush group (T − 1 scans); everything else is checked
    assert out["oracle_predicted"] <= 0.05 * out["instance_scans"], out
    assert out["exempt_after_prediction"] <= out["oracle_predicted"] * (T - 1), out
    assert out["assoc_checked"] >= out["instance_scans"] - out["oracle_predicted"] * T, out


@pytest.mark.parametrize("arith,T,rep", [(2, 20, 1), (2, 20, 2), (0, 16, 1)])
def test_survey_world_parity_steady_state(ekf_mod, oracle_mod, arith, T, rep):
    """The same after a 200-scan pre-roll (the bench's): the reference's motion model has run away
    in every instance (poses 1e9-1e21 m, P up to 1e43). Instance 0 (P ≈ 1e30: every
    arithmetic, EXACT included, differs from the fp64 reference there) must be flagged; whatever
    is not flagged meets the bar (instance 7, P ≈ 1e16-1e19: the split-fp16 planes cannot carry its
    dynamic range, PLANE_SIGMA_EXACT takes its steps to the exact forms)."""
    out = run_survey_parity(ekf_mod, oracle_mod, arith, T, 200, 48, options={"mfma_replay": rep})
    record(f"survey_parity_steady_a{arith}_T{T}_rep{rep}", out)
    # (every library flag was checked against the restatement's prediction in run_survey_parity;
    # the run-away instances are the predicted ones)
    assert out["oracle_predicted"] > 0, out
