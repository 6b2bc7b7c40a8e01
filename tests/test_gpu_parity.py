"""GPU parity: the HIP path (through the C-ABI) against the CPU restatement (oracle/).

Tolerances (BASELINE.json north_star): per scan from identical inputs,
‖P − P_ref‖_F / ‖P_ref‖_F ≤ 1e-6 and ‖y − y_ref‖₂ / ‖y_ref‖₂ ≤ 1e-8, association identical
(fp16 storage: P ≤ 1e-3, see P_TOL).
fp64 storage is held to 1e-10 over whole trajectories.
"""
import math
import os

import numpy as np
import pytest

from slam_ros_amd import scan_gen as G

pytestmark = pytest.mark.gpu

# precision → per-scan relative Frobenius bound on P. fp16 storage (BASELINE config 5, tolerance
# re-stated): the block is rounded to fp16 (11-bit significand) after the scan, which alone is
# ≈3e-4 relative in Frobenius norm; the state vector and the association are still fp64 exact.
P_TOL = {0: 1e-10, 1: 1e-6, 2: 1e-3}
Y_TOL = 1e-8


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def is_bf_form(name):
    """A split-bf16 flush form: the 2 × 2 wave form's <.., true> (default) or the 2 × 4 kernel."""
    return name.startswith("flush_bf24_kernel") or name.endswith(", true>")


def make_pair(ekf, oracle, N, prec, state=None, r_mode=0, max_lines=16, mode=None,
              reset_margin=10):
    ens = ekf.Ensemble(N, 1, prec, max_lines=max_lines, r_mode=r_mode, reset_margin=reset_margin)
    ref = oracle.OracleRobot(N, mode=oracle.FAST if mode is None else mode, r_mode=r_mode)
    if state is not None:
        P0, y0, s0, pose0 = state
        ens.upload_state(0, P0, y0, s0, pose0)
        Pg, yg, sg, pg = ens.download_state(0)
        ref.set_state(Pg, yg, sg, pg)
    return ens, ref


def check_same(ens, ref, prec, res=None, mref=None, where=""):
    if res is not None:
        assert res["match"] == mref, (where, res["match"], mref)
    P, y, saved, pose = ens.download_state(0)
    assert saved == ref.savedLineCount, where
    rp = rel(P, ref.P_t0)
    ry = rel(y, ref.y)
    assert rp <= P_TOL[prec], (where, "P", rp)
    assert ry <= Y_TOL, (where, "y", ry)
    np.testing.assert_allclose(pose, ref.pose, rtol=0, atol=1e-9 if prec else 1e-12)
    return P, y, saved, pose


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("N", [5, 37, 64, 100])
def test_state_roundtrip(ekf_mod, prec, N):
    n = 3 + 2 * N
    rng = np.random.default_rng(N)
    A = rng.normal(size=(n, n))
    P = A @ A.T
    P = (P + P.T) / 2                           # exactly symmetric (packed storage)
    if prec == 2:
        P = P / (2 * n)                         # within the fp16 storage range (|P| < 64)
    y = rng.normal(size=n)
    ens = ekf_mod.Ensemble(N, 1, prec)
    ens.upload_state(0, P, y, N // 2, [1.0, 2.0, 0.3])
    Pg, yg, sg, pg = ens.download_state(0)
    assert sg == N // 2 and list(pg) == [1.0, 2.0, 0.3]
    np.testing.assert_array_equal(yg, y)
    if prec == 0:
        np.testing.assert_array_equal(Pg, P)
    else:
        np.testing.assert_array_equal(Pg[:3], P[:3])            # robot strip kept in fp64
        if prec == 1:
            want = P[3:, 3:].astype(np.float32)
        else:                                                   # fp16 scaled by 2^10
            want = (P[3:, 3:].astype(np.float32) * 1024).astype(np.float16).astype(np.float64) / 1024
        np.testing.assert_allclose(Pg[3:, 3:], want, rtol=0, atol=0)


@pytest.mark.parametrize("prec", [0, 1, 2])
def test_lowrank_init_equals_dense(ekf_mod, prec):
    N = 48
    w = G.make_world(N)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, 1, prec)
    a.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
    Pa = a.download_state(0)[0]
    ref = st.dense_P()
    tol = {0: 1e-14, 1: 1e-7, 2: 1e-3}[prec]
    assert rel(Pa, ref) <= tol


def test_ctor_state_matches_reference(ekf_mod, oracle_mod):
    ens = ekf_mod.Ensemble(12, 2, 0)
    ens.reset(1, 1.5, -2.0, 0.25)
    ref = oracle_mod.OracleRobot(12, 1.5, -2.0, 0.25)
    P, y, s, pose = ens.download_state(1)
    np.testing.assert_array_equal(P, ref.P_t0)
    np.testing.assert_array_equal(y, ref.y)
    assert s == 0 and list(pose) == [1.5, -2.0, 0.25]


@pytest.mark.parametrize("prec", [0, 1, 2])
def test_map_from_scratch(ekf_mod, oracle_mod, prec):
    """Robot(0,0,0) → first scan augments every line → later scans match and augment.
    fp64: one trajectory vs the faithful dense restatement. fp32: per scan from identical state."""
    N = 24
    rng = np.random.default_rng(1)
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, mode=oracle_mod.FAITHFUL)
    first = G.random_lines(rng, 5)
    res = ens.localize([0.01, 0.0, 0.0], first[None], [5])[0]
    m = ref.localize(first, [0.01, 0.0, 0.0])
    P, yg, s, pose = check_same(ens, ref, prec, res, m, "first")
    assert res["new_landmarks"] == 5 and res["saved"] == 5
    if prec:
        ref.set_state(P, yg, s, pose)   # next scan from the stored (rounded) state
    for step in range(15):
        y = ref.y
        lines = []
        for j in rng.choice(ref.savedLineCount, size=min(3, ref.savedLineCount), replace=False):
            a, rr = y[3 + 2 * j], y[4 + 2 * j]
            lines.append([G.wrap_pi(a - ref.thetaPos),
                          rr - (ref.xPos * math.cos(a) + ref.yPos * math.sin(a)), 1e-2, 0, 0, 1e-2])
        lines = np.array(lines + list(G.random_lines(rng, 1)))
        enc = [ref.xPos - 0.01, ref.yPos, ref.thetaPos + 0.001]
        res = ens.localize(enc, lines[None], [len(lines)])[0]
        m = ref.localize(lines, enc)
        P, yg, s, pose = check_same(ens, ref, prec, res, m, f"step {step}")
        if prec:
            ref.set_state(P, yg, s, pose)


def test_trajectory_fp64_with_reset(ekf_mod, oracle_mod):
    """25 scans at N=64 in fp64 incl. augmentation and the capacity reset (Robot.cpp:893-904)."""
    N = 64
    w = G.make_world(N, active=N - 13)
    st = G.initial_state(w)
    ens, ref = make_pair(ekf_mod, oracle_mod, N, 0, (st.dense_P(), st.y, st.saved, st.pose),
                         mode=oracle_mod.FAITHFUL)
    rng = np.random.default_rng(3)
    resets = 0
    for step in range(1, 26):
        enc, lines, _ = G.make_scan(w, step, lines=6)
        ln = np.concatenate([lines[0], G.random_lines(rng, 1)])
        res = ens.localize(enc, ln[None], [len(ln)])[0]
        m = ref.localize(ln, enc[0])
        check_same(ens, ref, 0, res, m, f"step {step}")
        resets += res["reset"]
    assert resets >= 1


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("pipeline,T,drain_at", [(True, 1, ()), (False, 4, ()), (True, 3, (7,)),
                                                 (False, 8, (5,)), (True, 8, ()), (False, 6, ()),
                                                 (False, 16, (5,)), (True, 16, ())])
def test_deferred_flush_equals_drained(ekf_mod, oracle_mod, prec, pipeline, T, drain_at):
    """Deferred covariance downdates — the landmark block rewritten once per T scans, the
    association kernels applying the pending steps on read, optionally overlapped with the
    next scans (pipeline) — give bit-identical state to one in-place flush per scan drained
    after every step; fp64 also vs the oracle. Covers matches, augmentation rows, the
    capacity reset inside a group and partial groups (a drain mid-group, the trajectory end)."""
    N = 64
    w = G.make_world(N, active=N - 14)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, 2, prec, max_lines=8, pipeline=pipeline, flush_interval=T)
    b = ekf_mod.Ensemble(N, 2, prec, max_lines=8)
    for ens in (a, b):
        for e in range(2):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(*b.download_state(0))
    rng = np.random.default_rng(11)
    resets = 0
    for step in range(1, 21):
        enc, lines, nl = G.make_scan(w, step, instances=2, lines=6)
        extra = G.random_lines(rng, 2)[None].repeat(2, axis=0) if step % 3 == 0 else np.zeros((2, 0, 6))
        ln = np.concatenate([lines, extra], axis=1)
        nl = np.full(2, ln.shape[1], dtype=np.int32)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        b.download_state(0, with_P=False)          # drains b after every step
        if step in drain_at:
            a.download_state(1, with_P=False)      # partial group flushed mid-trajectory
        m = ref.localize(ln[0], enc[0])
        assert ra[0]["match"] == rb[0]["match"] == m, (step, ra[0]["match"], m)
        assert ra[1]["match"] == rb[1]["match"], step
        resets += ra[0]["reset"]
    assert resets >= 1
    for e in range(2):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        bad = np.argwhere(Pa != Pb)
        assert bad.size == 0, (e, bad[:12].tolist(), rel(Pa, Pb))
        np.testing.assert_array_equal(ya, yb)
        np.testing.assert_array_equal(pa, pb)
        assert sa == sb
    if prec == 0:
        check_same(a, ref, 0, where="deferred fp64 trajectory")


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("N", [64, 256, 1024])
def test_per_scan_parity(ekf_mod, oracle_mod, prec, N):
    w = G.make_world(N)
    st = G.initial_state(w)
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, (st.dense_P(), st.y, st.saved, st.pose),
                         max_lines=8)
    for step in range(1, 4):
        enc, lines, nl = G.make_scan(w, step)
        res = ens.localize(enc, lines, nl)[0]
        m = ref.localize(lines[0], enc[0])
        assert res["matches"] == 8
        P, y, s, pose = check_same(ens, ref, prec, res, m, f"N={N} step {step}")
        ref.set_state(P, y, s, pose)


def test_n4096_fp32_scan(ekf_mod, oracle_mod):
    """Headline size (N=4096, n=8195): one fp32 scan from identical state vs the restatement."""
    N = 4096
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, 1, 1, max_lines=8)
    ens.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
    P0, y0, s0, pose0 = ens.download_state(0)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(P0, y0, s0, pose0)
    del P0
    enc, lines, nl = G.make_scan(w, 1)
    res = ens.localize(enc, lines, nl)[0]
    m = ref.localize(lines[0], enc[0])
    assert res["matches"] == 8
    check_same(ens, ref, 1, res, m, "N=4096")


@pytest.mark.parametrize("prec", [0, 1, 2])
def test_predict_then_update_equals_localize(ekf_mod, prec):
    N = 64
    w = G.make_world(N)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, 1, prec, max_lines=8)
    b = ekf_mod.Ensemble(N, 1, prec, max_lines=8)
    for e in (a, b):
        e.upload_state(0, st.dense_P(), st.y, st.saved, st.pose)
    for step in range(1, 4):
        enc, lines, nl = G.make_scan(w, step)
        ra = a.localize(enc, lines, nl)[0]
        b.predict(enc)
        rb = b.update(lines, nl)[0]
        assert ra["match"] == rb["match"]
        Pa, ya, _, pa = a.download_state(0)
        Pb, yb, _, pb = b.download_state(0)
        np.testing.assert_array_equal(Pa, Pb)
        np.testing.assert_array_equal(ya, yb)
        np.testing.assert_array_equal(pa, pb)


@pytest.mark.parametrize("prec,T", [(0, 1), (1, 4), (0, 8)])
def test_synchronous_result_mirror(ekf_mod, prec, T):
    """ekf_localize / ekf_update read their result from the pinned mirror the scan's lead writes (no
    copies; the call waits for the association kernel only) and ekf_get_pose_cov the mirrored robot
    block until the next launch: equal to the device copies (ekf_read_results, the state's top-left
    3 × 3), also after a state upload or an asynchronous launch invalidated the mirror."""
    N, E = 300, 3
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    for step in range(1, 2 * T + 3):
        enc, ln, nl = G.make_scan(w, step, instances=E)
        if step % 3 == 0:
            ens.predict(enc)
            res = ens.update(ln, nl)
        else:
            res = ens.localize(enc, ln, nl)
        p33 = [ens.pose_cov(e) for e in range(E)]   # (the mirror, before any other call)
        dev = ens.read_results()                      # the device copies and the host fold
        for e in range(E):
            np.testing.assert_array_equal(res[e]["pose"], dev[e]["pose"])
            assert ({k: v for k, v in res[e].items() if k != "pose"} ==
                    {k: v for k, v in dev[e].items() if k != "pose"}), (step, e)
            P, y, saved, pose = ens.download_state(e)
            np.testing.assert_array_equal(p33[e], P[:3, :3])
            np.testing.assert_array_equal(res[e]["pose"], pose)
            assert res[e]["saved"] == saved and res[e]["matches"] == 8
    # an upload changes the robot block without a scan: the mirror no longer serves it
    P, y, saved, pose = ens.download_state(1)
    P[:3, :3] *= 1.5
    ens.upload_state(1, P, y, saved, pose)
    np.testing.assert_array_equal(ens.pose_cov(1), P[:3, :3])
    ens.close()


@pytest.mark.parametrize("prec", [0, 1, 2])
def test_ensemble_instances_are_independent(ekf_mod, prec):
    N, E = 64, 3
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, E, prec, max_lines=8)
    singles = [ekf_mod.Ensemble(N, 1, prec, max_lines=8) for _ in range(E)]
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
        singles[e].init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
    for step in range(1, 4):
        enc, lines, nl = G.make_scan(w, step, instances=E)
        nl[1] = 5                                  # ragged line counts across instances
        rs = ens.localize(enc, lines, nl)
        for e in range(E):
            r1 = singles[e].localize(enc[e:e + 1], lines[e:e + 1], nl[e:e + 1])[0]
            assert rs[e]["match"] == r1["match"]
    for e in range(E):
        Pa, ya, _, _ = ens.download_state(e)
        Pb, yb, _, _ = singles[e].download_state(0)
        np.testing.assert_array_equal(Pa, Pb)
        np.testing.assert_array_equal(ya, yb)


def test_as_written_r_mode(ekf_mod, oracle_mod):
    """Robot.cpp:302-304 as written (zero-initialised stack): exact whenever the as-written R is
    symmetric. Lines 1 and 2 get a single OFF-diagonal R entry; if such a line matches, the
    reference's P turns non-symmetric and the GPU flags EKF_ST_NONSYM instead of pretending."""
    N = 40
    w = G.make_world(N, active=20)
    st = G.initial_state(w)
    state = (st.dense_P(), st.y, st.saved, st.pose)
    enc, lines, _ = G.make_scan(w, 1, lines=6, var_alpha=2e-4, var_r=3e-4)
    far = np.array([[0.123, 55.0, 1e-4, 0, 0, 1e-4], [-2.0, 40.0, 1e-4, 0, 0, 2e-4]])
    for L, ln in ((1, lines[0][:1]), (6, np.concatenate([lines[0][:1], far, lines[0][3:]]))):
        ens, ref = make_pair(ekf_mod, oracle_mod, N, 0, state, r_mode=1)
        res = ens.localize(enc, ln[None], [L])[0]
        m = ref.localize(ln, enc[0])
        check_same(ens, ref, 0, res, m, f"as_written L={L}")
        assert not res["status"] & ekf_mod.ST_NONSYM
    ens, ref = make_pair(ekf_mod, oracle_mod, N, 0, state, r_mode=1)
    res = ens.localize(enc, lines[:, :3], [3])[0]
    assert res["match"][1] >= 0 and res["status"] & ekf_mod.ST_NONSYM


@pytest.mark.parametrize("prec", [0, 1, 2])
def test_edge_cases(ekf_mod, oracle_mod, prec):
    N = 30
    w = G.make_world(N, active=12)
    st = G.initial_state(w)
    state = (st.dense_P(), st.y, st.saved, st.pose)
    # no lines: prediction committed (Robot.cpp:702-716)
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, state)
    res = ens.localize([0.05, -0.02, 0.3], np.zeros((1, 0, 6)), [0])[0]
    ref.localize(np.zeros((0, 6)), [0.05, -0.02, 0.3])
    assert res["matches"] == 0 and res["new_landmarks"] == 0
    check_same(ens, ref, prec, where="no lines")
    # every line rejected by the gate → all appended
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, state)
    far = np.array([[0.123, 55.0, 1e-4, 0, 0, 1e-4], [-2.0, 40.0, 1e-4, 0, 0, 2e-4]])
    res = ens.localize([0, 0, 0], far[None], [2])[0]
    m = ref.localize(far, [0, 0, 0])
    assert m == [-1, -1]
    check_same(ens, ref, prec, res, m, "gate reject")
    # capacity overflow: s = N - 1 with 3 unmatched lines and no reset margin
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, reset_margin=0,
                         state=None)
    ref = oracle_mod.OracleRobot(N)  # reset margin is fixed at 10 in the reference
    w2 = G.make_world(N, active=N - 1)
    st2 = G.initial_state(w2)
    ens.upload_state(0, st2.dense_P(), st2.y, st2.saved, st2.pose)
    lines = np.array([[0.1, 60.0, 1e-4, 0, 0, 1e-4], [0.2, 61.0, 1e-4, 0, 0, 1e-4],
                      [0.3, 62.0, 1e-4, 0, 0, 1e-4]])
    res = ens.localize([0, 0, 0], lines[None], [3])[0]
    assert res["saved"] == N and res["status"] & ekf_mod.ST_CAPACITY


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("theta", [7.0, -7.0, 13.0, 3.2, -3.5, 2 * np.pi])
def test_normalize_radian_quirk_on_gpu(ekf_mod, oracle_mod, prec, theta):
    """Robot.cpp:62-71's fold for |rad| >= 2π (if / else-if, no loop: 7 → −5.566, not 0.717) on the
    device: a pose heading past ±π (and past ±2π) goes through the no-match commit
    (Robot.cpp:702-716: pose = normalizeRadian(x_pre)), the innovation angles of the gate
    (Robot.cpp:347-349) and the post-update heading (Robot.cpp:596), against the restatement."""
    N = 30
    w = G.make_world(N, active=12)
    st = G.initial_state(w)
    y0 = st.y.copy()
    y0[2] = theta
    pose0 = np.array([st.pose[0], st.pose[1], theta])
    state = (st.dense_P(), y0, st.saved, pose0)
    # no lines: the prediction is committed through normalizeRadian
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, state)
    res = ens.localize([0.05, -0.02, 0.3], np.zeros((1, 0, 6)), [0])[0]
    ref.localize(np.zeros((0, 6)), [0.05, -0.02, 0.3])
    assert res["matches"] == 0
    check_same(ens, ref, prec, where=f"no lines, theta {theta}")
    # lines: gating angles and the updated heading, two scans in a row
    ens, ref = make_pair(ekf_mod, oracle_mod, N, prec, state)
    for step in (1, 2):
        enc, lines, nl = G.make_scan(w, step)
        res = ens.localize(enc, lines, nl)[0]
        m = ref.localize(lines[0][:nl[0]], enc[0])
        check_same(ens, ref, prec, res, m, f"lines, theta {theta}, scan {step}")


def test_ellipse_matches_eigen(ekf_mod):
    N = 8
    ens = ekf_mod.Ensemble(N, 1, 0)
    n = 3 + 2 * N
    P = np.eye(n) * 0.01
    P[:2, :2] = [[0.04, 0.012], [0.012, 0.01]]
    ens.upload_state(0, P, np.zeros(n), 0, [0, 0, 0])
    ok, axii, angle = ens.ellipse(0)
    lam, vec = np.linalg.eigh(P[:2, :2])
    assert ok
    np.testing.assert_allclose(axii, 2 * np.sqrt(5.991 * np.abs(lam)), rtol=1e-6)
    v = vec[:, 1]
    want = math.atan2(v[0], v[1])
    d = (angle - want) % math.pi
    assert min(d, math.pi - d) < 1e-5          # GSL eigenvector sign: parity modulo π


def test_large_capacity_multi_workgroup_exchange(ekf_mod, oracle_mod):
    """N=8192 (32 cooperating workgroups per instance, two instances per launch) with the
    benchmark's deferred flush: 4 scans vs the restatement, association identical."""
    N = 8192
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, 2, 1, max_lines=8, flush_interval=4)
    for e in range(2):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    P0, y0, s0, pose0 = ens.download_state(1)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(P0, y0, s0, pose0)
    del P0
    for step in range(1, 5):
        enc, lines, nl = G.make_scan(w, step, instances=2)
        res = ens.localize(enc, lines, nl)
        m = ref.localize(lines[1], enc[1])
        assert res[1]["match"] == m and res[1]["matches"] == 8, (step, res[1]["match"], m)
    P, y, s, pose = ens.download_state(1)
    assert rel(P, ref.P_t0) <= 1e-5 and rel(y, ref.y) <= 1e-8


@pytest.mark.parametrize("T", [1, 4])
def test_many_lines_per_scan(ekf_mod, oracle_mod, T):
    """max_lines = EKF_MAX_LINES (kmax = 128: the general flush path) with 40 lines per scan, most
    of them matches (rank-80 downdates), some new; per scan vs the restatement."""
    N = 512
    w = G.make_world(N, active=N - 40)   # room for the new landmarks below the reset threshold
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, 1, 1, max_lines=ekf_mod.EKF_MAX_LINES, flush_interval=T)
    ens.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(*ens.download_state(0))
    rng = np.random.default_rng(5)
    for step in range(1, 4):
        enc, lines, _ = G.make_scan(w, step, lines=36)
        ln = np.concatenate([lines[0], G.random_lines(rng, 4)])
        res = ens.localize(enc, ln[None], [len(ln)])[0]
        m = ref.localize(ln, enc[0])
        assert res["match"] == m, (step, res["match"], m)
        assert res["matches"] >= 30
    P, y, s, pose = ens.download_state(0)
    assert rel(P, ref.P_t0) <= 1e-5 and rel(y, ref.y) <= 1e-8


def _spec_scans(w, rng, steps, L=8):
    """Scans that stress the speculative association: ordinary scans, a landmark observed twice
    in one scan, lines that match nothing (appended), and a mix."""
    out = []
    for step in range(1, steps + 1):
        enc, lines, _ = G.make_scan(w, step, lines=L)
        ln = lines[0].copy()
        kind = step % 4
        if kind == 1:
            ln[3] = ln[1]                                   # the same landmark twice
        elif kind == 2:
            ln[5:] = G.random_lines(rng, L - 5)             # unmatched → new landmarks
        elif kind == 3:
            ln[[0, 6]] = ln[[6, 0]]
            ln[2, 1] += 0.02                                # near-miss observation
        out.append((enc, ln))
    return out


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("N,T", [(64, 4), (1024, 4), (4096, 4), (1024, 8), (4096, 8)])
def test_speculative_association_identical(ekf_mod, oracle_mod, monkeypatch, prec, N, T):
    """The speculative association (guessed winners, three exchanges per scan, exact local
    re-check) gives bit-identical state and results to the per-line sequential exchange, also
    when every guess is wrong (EKF_OPT_SPECULATE = 2: every scan falls back) and when only the
    later lines' guesses are (3: the restart keeps the lines before the first wrong one, from the
    speculative packages); association vs the restatement."""
    w = G.make_world(N, active=N - 30)
    st = G.initial_state(w)
    scans = _spec_scans(w, np.random.default_rng(3), 8)
    runs = {}
    for mode in (0, 1, 2, 3):
        ens = ekf_mod.Ensemble(N, 1, prec, max_lines=8, flush_interval=T,
                               options={"scan_stamps": 1, "speculate": mode})
        ens.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
        if mode == 1:
            ref = oracle_mod.OracleRobot(N)
            ref.set_state(*ens.download_state(0))
        results = []
        kept = 0   # restarts that kept the lines before the first wrong guess (RES_DBG bit 512)
        for enc, ln in scans:
            r = ens.localize(enc, ln[None], [len(ln)])[0]
            results.append((r["match"], r["matches"], r["new_landmarks"], r["status"]))
            ens.read_results()   # (the full record: a synchronous call mirrors only ekf_result's words)
            kept += 1 if int(ens.result_words(0)[9]) & 512 else 0
            if mode == 1:
                assert r["match"] == ref.localize(ln, enc[0]), r["match"]
        stamps = ens.scan_stamps()
        runs[mode] = (results, ens.download_state(0), stamps[15], kept)
        ens.close()
    assert runs[1][2] == 0, "speculation fell back on ordinary scans"
    assert runs[2][2] >= 4, "wrong guesses did not fall back"
    assert runs[3][2] >= 2 and runs[3][3] >= 1, "wrong late guesses did not keep the lines before them"
    for mode in (1, 2, 3):
        assert runs[mode][0] == runs[0][0], mode
        P, y, s, pose = runs[mode][1]
        P0, y0, s0, pose0 = runs[0][1]
        bad = np.argwhere(P != P0)
        assert bad.size == 0, (mode, bad[:8].tolist(), rel(P, P0))
        np.testing.assert_array_equal(y, y0)
        np.testing.assert_array_equal(pose, pose0)
        assert s == s0


@pytest.mark.parametrize("prec", [1, 2])
@pytest.mark.parametrize("arith", [0, 1])
def test_hot_scan_kernel_equals_generic(ekf_mod, monkeypatch, prec, arith):
    """The association kernel's HOT instantiation (symmetric fp32 operands, kmax 16: the product
    launch of every EKF_R_INTENDED fp32/fp16 context with max_lines <= 8) and the generic
    instrumented one (EKF_OPT_SCAN_STAMPS = 1, `scan_kernel<T, true, false>`) give bit-identical state
    and results — on the speculative path (with the early U/V operand stores after the fourth
    match) and when every guess is wrong (the restart after those stores), in both flush
    arithmetics (Robot.cpp:313-641)."""
    N, T = 1024, 8
    w = G.make_world(N, active=N - 30)
    st = G.initial_state(w)
    scans = _spec_scans(w, np.random.default_rng(5), 10)
    runs = {}
    for stamps in ("0", "1"):
        for spec in ("1", "2", "3"):
            ens = ekf_mod.Ensemble(N, 1, prec, max_lines=8, flush_interval=T, arith=arith,
                                   options={"scan_stamps": int(stamps), "speculate": int(spec)})
            ens.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
            results = []
            for enc, ln in scans:
                r = ens.localize(enc, ln[None], [len(ln)])[0]
                results.append((r["match"], r["matches"], r["new_landmarks"], r["status"]))
            runs[(stamps, spec)] = (results, ens.download_state(0))
            ens.close()
    for spec in ("1", "2", "3"):
        hot, gen = runs[("0", spec)], runs[("1", spec)]
        assert hot[0] == gen[0], spec
        P, y, s, pose = hot[1]
        P0, y0, s0, pose0 = gen[1]
        bad = np.argwhere(P != P0)
        assert bad.size == 0, (spec, bad[:8].tolist(), rel(P, P0))
        np.testing.assert_array_equal(y, y0)
        np.testing.assert_array_equal(pose, pose0)
        assert s == s0
    if arith == 0:   # exact arithmetic: the restart is the sequential chain, bit for bit
        assert runs[("0", "2")][0] == runs[("0", "1")][0]
        np.testing.assert_array_equal(runs[("0", "2")][1][0], runs[("0", "1")][1][0])


@pytest.mark.parametrize("prec,arith", [(1, 2), (2, 2), (1, 0), (1, 1), (2, 1)])
@pytest.mark.parametrize("N,T", [(256, 4), (1000, 8), (1024, 20), (2048, 12)])
def test_narrow_scan_workgroups_identical(ekf_mod, prec, arith, N, T):
    """EKF_OPT_SCAN_THREADS: the association kernel on 128 and 64 landmarks per workgroup (more
    workgroups per instance, a partial last one at N = 1000) gives bit-identical results and state
    to the 192-wide one, in every flush arithmetic, on the speculative path and when every guess is
    wrong (the sequential restart: one cross-workgroup exchange per line), three instances per
    launch."""
    if arith != 2 and T > 16:
        T = 16   # (EKF_ARITH_EXACT / BF16X6: T <= 16)
    E = 3
    w = G.make_world(N, active=N - 30)
    st = G.initial_state(w)
    scans = _spec_scans(w, np.random.default_rng(11), 2 * T + 3)
    runs = {}
    for nt in (192, 128, 64):
        for spec in (1, 2):
            ens = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=arith,
                                   options={"scan_threads": nt, "speculate": spec})
            for e in range(E):
                ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
            results = []
            for enc, ln in scans:
                lines = np.stack([ln] * E)
                r = ens.localize(np.repeat(enc, E, axis=0), lines, [len(ln)] * E)
                results.append([(x["match"], x["matches"], x["new_landmarks"], x["status"]) for x in r])
            runs[(nt, spec)] = (results, [ens.download_state(e) for e in range(E)])
            ens.close()
    for key, (res, states) in runs.items():
        ref_res, ref_states = runs[(192, key[1])]
        assert res == ref_res, key
        for e in range(E):
            P, y, s, pose = states[e]
            P0, y0, s0, pose0 = ref_states[e]
            bad = np.argwhere(P != P0)
            assert bad.size == 0, (key, e, bad[:8].tolist(), rel(P, P0))
            np.testing.assert_array_equal(y, y0)
            np.testing.assert_array_equal(pose, pose0)
            assert s == s0


@pytest.mark.parametrize("prec", [1, 2])
@pytest.mark.parametrize("N,T,lines,extra_every", [(80, 8, 6, 3), (80, 2, 8, 0), (64, 6, 6, 4),
                                                  (1024, 8, 8, 0), (1024, 4, 6, 5)])
def test_wave_flush_equals_drained(ekf_mod, monkeypatch, prec, N, T, lines, extra_every):
    """The barrier-free per-wave flush (2 × 2-tile wave-tiles, software-pipelined operand ring;
    forced with EKF_OPT_FLUSH_FORM = 8) gives bit-identical state to one in-place flush per scan:
    full groups in its pipelined loop (8 matches, or partial downdates predicated), groups with
    augmentation rows or the capacity reset in its general loop, odd tile counts (N = 80: 5 tile
    rows, a wave-tile column past the block) and several instances per XCD range."""
    E = 3
    w = G.make_world(N, active=N - 14 if extra_every else N - 10)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, options={"flush_form": 8})
    b = ekf_mod.Ensemble(N, E, prec, max_lines=8)
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(5)
    for step in range(1, 3 * T + 1):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=lines)
        if extra_every and step % extra_every == 0:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            ln = np.concatenate([ln, ex], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        b.download_state(0, with_P=False)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        bad = np.argwhere(Pa != Pb)
        assert bad.size == 0, (e, bad[:12].tolist(), rel(Pa, Pb))
        np.testing.assert_array_equal(ya, yb)
        assert sa == sb


@pytest.mark.parametrize("arith", [1, 2])
@pytest.mark.parametrize("N,T,lines,extra_every", [(80, 8, 6, 3), (80, 2, 8, 0), (64, 6, 6, 4),
                                                  (1024, 8, 8, 0), (1024, 4, 6, 5), (96, 3, 8, 0),
                                                  (1024, 12, 8, 0), (256, 16, 6, 7), (80, 16, 7, 0)])
def test_bf16x6_flush_close_to_exact(ekf_mod, oracle_mod, N, T, lines, extra_every, arith):
    """EKF_ARITH_BF16X6 (split-bf16 wave flush for plain groups of 2, 4, 6 or 8 steps; groups
    with augmentation rows or the reset, odd group sizes and the partial last group fall back to
    the fp32 forms): same associations as the exact arithmetic drained after every scan, and the
    state within the fp32 bar — P ≤ 1e-6 relative (BASELINE's bound), y ≤ 1e-8 — also against
    the fp64 restatement for instance 0."""
    E = 3
    # the trajectory stays clear of the capacity reset: after a reset the map is rebuilt from the
    # observations and the reference's own fp64 dynamics double any perturbation every scan
    # (measured with the restatement: 1e-16 → 6e-8 in 28 scans), so an uninterrupted trajectory
    # across it compares chaos, not arithmetic. Resets inside deferred groups are covered by
    # test_deferred_flush_equals_drained and the fp64 trajectories.
    active = N - 12 - 2 * ((3 * T + 1) // extra_every) if extra_every else N - 10
    w = G.make_world(N, active=active)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, 1, max_lines=8, flush_interval=T, arith=arith)
    b = ekf_mod.Ensemble(N, E, 1, max_lines=8)
    if T % 2 == 0:
        assert is_bf_form(a.flush_kernel_name(T)), a.flush_kernel_name(T)
    assert not is_bf_form(b.flush_kernel_name(8))
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(*b.download_state(0))
    rng = np.random.default_rng(5)
    for step in range(1, 3 * T + 2):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=lines)
        if extra_every and step % extra_every == 0:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            ln = np.concatenate([ln, ex], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        b.download_state(0, with_P=False)
        m = ref.localize(ln[0], enc[0])
        assert ra[0]["match"] == m, (step, ra[0]["match"], m)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
            assert ra[e]["status"] == 0, (step, e, ra[e]["status"])
            assert not ra[e]["reset"], (step, e)
    k = 3 * T + 1
    meas = {}
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        meas[e] = {"P_bf_vs_exact": rel(Pa, Pb), "y_bf_vs_exact": rel(ya, yb)}
        if e == 0:
            meas[e].update(P_bf_vs_fp64=rel(Pa, ref.P_t0), P_exact_vs_fp64=rel(Pb, ref.P_t0),
                           y_bf_vs_fp64=rel(ya, ref.y), y_exact_vs_fp64=rel(yb, ref.y))
        # k scans, never re-synchronised: the per-scan bars (1e-6 on P, 1e-8 on y) times k
        assert rel(Pa, Pb) <= k * 1e-6 and rel(ya, yb) <= k * 1e-8, (e, meas[e])
        assert sa == sb
        if e == 0:   # vs fp64: no further than the exact arithmetic's own distance plus the bars
            assert meas[0]["P_bf_vs_fp64"] <= meas[0]["P_exact_vs_fp64"] + k * 1e-6, meas[0]
            assert meas[0]["y_bf_vs_fp64"] <= meas[0]["y_exact_vs_fp64"] + k * 1e-8, meas[0]
    from tests.test_bench_config import record
    record(f"{'bf16x6' if arith == 1 else 'f16x3'}_vs_exact_N{N}_T{T}_L{lines}_x{extra_every}", meas)
    # kmax > 16 (max_lines 16) can never take the split-bf16 flush: rejected, no silent fallback
    with pytest.raises(ekf_mod.EkfError):
        ekf_mod.Ensemble(N, 1, 1, max_lines=16, flush_interval=8, arith=ekf_mod.ARITH_BF16X6)


@pytest.mark.parametrize("arith", [1, 2])
@pytest.mark.parametrize("N,T,extra_every", [(256, 8, 0), (256, 12, 5), (80, 16, 0), (1024, 6, 4)])
def test_bf16x6_fp16_storage(ekf_mod, oracle_mod, N, T, extra_every, arith):
    """fp16 storage with EKF_ARITH_BF16X6 (split-bf16 flush on the fp16 tiles, rounded once per
    group — the general path of groups with augmented rows and the on-read replay too; MFMA replay
    of plain pending steps, the VALU replay after augmented rows) against the
    fp64 restatement, never re-synchronised: association identical, P within the re-stated 1e-3
    (fp16 rounding ≈3e-4 per materialisation), y within 1e-8, at the end and after every drain."""
    E = 2
    active = N - 12 - 2 * ((3 * T + 1) // extra_every) if extra_every else N - 10
    w = G.make_world(N, active=active)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, 2, max_lines=8, flush_interval=T, arith=arith)
    assert a.flush_kernel_name(T if T % 2 == 0 else T - 1).startswith("flush_f32_wave_kernel<_Float16")
    for e in range(E):
        a.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(*a.download_state(0))
    rng = np.random.default_rng(11)
    for step in range(1, 3 * T + 2):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=6 if extra_every else 8)
        if extra_every and step % extra_every == 0:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            ln = np.concatenate([ln, ex], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        r = a.localize(enc, ln, nl)
        m = ref.localize(ln[0], enc[0])
        assert r[0]["match"] == m and r[0]["status"] == 0, (step, r[0], m)
    P, y, saved, pose = a.download_state(0)
    assert saved == ref.savedLineCount
    assert rel(P, ref.P_t0) <= 1e-3, rel(P, ref.P_t0)
    assert rel(y, ref.y) <= 1e-8, rel(y, ref.y)


@pytest.mark.parametrize("N,T,lines,extra_every", [(80, 4, 8, 0), (80, 4, 6, 3), (64, 3, 6, 2), (100, 2, 8, 0),
                                                   (96, 1, 5, 0), (2000, 4, 8, 0), (2000, 8, 8, 0),
                                                   (80, 8, 6, 3), (100, 6, 8, 0), (96, 5, 6, 2)])
def test_f64_wave_flush_equals_tile_kernel(ekf_mod, monkeypatch, N, T, lines, extra_every):
    """fp64 storage: the wave flush (1 × 2-tile wave-tiles, every k-step run over the −0·(+0)
    operand padding; default for groups of ≤ 8 steps, operand ring of 4 steps beyond four) gives
    bit-identical state to the per-tile
    downdate_f64_kernel (EKF_OPT_FLUSH_FORM = 2) flushed after every scan — fast loop, predicated
    partial downdates, and the general loop for groups with augmentation rows or the reset.
    N = 2000 gives every wave a dozen wave-tiles (the prefetch chain across wave-tiles)."""
    E = 3
    w = G.make_world(N, active=N - 14 if extra_every else N - 10)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, 0, max_lines=8, flush_interval=T)
    b = ekf_mod.Ensemble(N, E, 0, max_lines=8, options={"flush_form": 2})
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(9)
    for step in range(1, 3 * T + 2):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=lines)
        if extra_every and step % extra_every == 0:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            ln = np.concatenate([ln, ex], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        b.download_state(0, with_P=False)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
            assert ra[e]["status"] == 0
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        bad = np.argwhere(Pa != Pb)
        assert bad.size == 0, (e, bad[:12].tolist(), rel(Pa, Pb))
        np.testing.assert_array_equal(ya, yb)
        assert sa == sb


@pytest.mark.parametrize("arith", [1, 2])
def test_active_flush_pipelined_reset_and_upload(ekf_mod, arith):
    """pipeline = 1 at N <= 192 (one association workgroup: the flush double-buffers the block):
    a capacity reset inside a group followed by groups without matches, then an upload followed
    by a group without matches. A wave-tile skipped by the active-map flush would keep the output
    buffer's copy from two flushes earlier (the pre-reset covariance), so the double-buffered flush
    never skips: P, y and the matches equal the flush over every wave-tile bit for bit."""
    N, E, T = 160, 2, 4
    w = G.make_world(N, active=N - 14)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, 1, max_lines=8, flush_interval=T, arith=arith, pipeline=True)
    b = ekf_mod.Ensemble(N, E, 1, max_lines=8, flush_interval=T, arith=arith, pipeline=True,
                         options={"active_flush": 0})
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(5)
    empty = np.zeros(E, dtype=np.int32)
    resets = 0
    for step in range(1, 6 * T + 2):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=4)
        if step in (3, 4):     # new landmarks past N - 10: the capacity reset
            ln = np.concatenate([ln, G.random_lines(rng, 4)[None].repeat(E, axis=0)], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        elif 5 <= step < 5 + 3 * T:
            nl = empty         # groups without a match (the upload below lands inside them)
        if step == 5 + 2 * T:  # upload (drains), then a group without matches
            for ens in (a, b):
                P, y, s, pose = ens.download_state(0)
                ens.upload_state(1, P, y, s, pose)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
            assert ra[e]["status"] & ~ekf_mod.ST_CAPACITY == 0
            resets += ra[e]["reset"]
    assert resets > 0
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        bad = np.argwhere(Pa != Pb)
        assert bad.size == 0, (e, bad[:12].tolist(), rel(Pa, Pb))
        np.testing.assert_array_equal(ya, yb)
        assert sa == sb
    a.close()
    b.close()


@pytest.mark.parametrize("arith", [1, 2])
@pytest.mark.parametrize("N,active,T,extra_every", [(1024, 300, 12, 3), (4096, 1500, 20, 4), (512, 100, 8, 0),
                                                     (1024, 1014, 12, 0)])
def test_active_flush_equals_full_flush(ekf_mod, arith, N, active, T, extra_every):
    """A partly filled map: the split flush that skips the wave-tiles past every step's nonzero
    operand rows and new rows (EKF_OPT_ACTIVE_FLUSH = 1, default) leaves P, y and the matches
    equal to the flush over every wave-tile (0), with new landmarks appended inside the groups
    and groups of several lengths."""
    if arith == 1 and T > 16:
        pytest.skip("EKF_ARITH_BF16X6 takes flush_interval <= 16")
    E = 3
    w = G.make_world(N, active=active)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, 1, max_lines=8, flush_interval=T, arith=arith)
    b = ekf_mod.Ensemble(N, E, 1, max_lines=8, flush_interval=T, arith=arith, options={"active_flush": 0})
    assert a.get_option("active_flush") == 1 and b.get_option("active_flush") == 0
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(11)
    for step in range(1, 2 * T + 3):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=6 if extra_every else 8)
        if extra_every:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            if step % extra_every == 0:
                ln = np.concatenate([ln, ex], axis=1)
                nl = np.full(E, ln.shape[1], dtype=np.int32)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
            assert ra[e]["status"] == rb[e]["status"] == 0
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        bad = np.argwhere(Pa != Pb)
        assert bad.size == 0, (e, bad[:12].tolist(), rel(Pa, Pb))
        np.testing.assert_array_equal(ya, yb)
        assert sa == sb
    a.close()
    b.close()


@pytest.mark.parametrize("N,T,lines", [(2000, 4, 8), (4096, 4, 8), (100, 8, 8), (300, 6, 5), (4096, 8, 8),
                                        (1000, 8, 8), (520, 8, 3)])
def test_f64_mfma_replay_equals_per_element_replay(ekf_mod, N, T, lines):
    """fp64 storage, speculative association with pending steps: the owned blocks of the guessed
    columns and the diagonal blocks replayed by v_mfma_f64_16x16x4f64 (EKF_OPT_MFMA_REPLAY = 1,
    default; two tile rows per pass), and the winners' mutual blocks from their operand rows staged
    in LDS, give the same matches, P and y bit for bit as the per-element FMA replay (0). N = 100,
    300 and 520 leave lanes without a landmark in the last wave (and a lone last tile row of a
    pass); N = 4096 at T = 8 is the bench's fp64 shape (up to seven pending steps)."""
    E = 3
    w = G.make_world(N)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, 0, max_lines=8, flush_interval=T)
    b = ekf_mod.Ensemble(N, E, 0, max_lines=8, flush_interval=T, options={"mfma_replay": 0})
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    for step in range(1, 2 * T + 3):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=lines)
        ra = a.localize(enc, ln, nl)
        rb = b.localize(enc, ln, nl)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
            assert ra[e]["status"] == rb[e]["status"] == 0
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        bad = np.argwhere(Pa != Pb)
        assert bad.size == 0, (e, bad[:12].tolist(), rel(Pa, Pb))
        np.testing.assert_array_equal(ya, yb)
        np.testing.assert_array_equal(pa, pb)
    a.close()
    b.close()


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("spec", ["1", "0"])
def test_singular_status_counts_only_evaluated_candidates(ekf_mod, oracle_mod, monkeypatch, prec, spec):
    """GSL_EDOM (EKF_ST_SINGULAR_S) is raised only for candidates the reference evaluates: the
    unmatched landmarks up to the line's winner (Robot.cpp:313-498 stops at the first passing
    one). Landmark 1 has a zero covariance and the lines an exact R = 0, so its S is singular;
    observing landmark 0 never evaluates it, observing landmark 1 does (after landmark 0 fails).
    Speculative and sequential association paths."""
    N = 16
    n = 3 + 2 * N
    P = np.zeros((n, n))
    P[3:5, 3:5] = [[0.01, 0.0], [0.0, 0.02]]
    y = np.zeros(n)
    y[3:5] = (0.5, 2.0)
    y[5:7] = (1.2, 3.0)
    for target, want in ((0, 0), (1, 1)):
        ens = ekf_mod.Ensemble(N, 1, prec, max_lines=8, options={"speculate": int(spec)})
        ens.upload_state(0, P, y, 2, [0.0, 0.0, 0.0])
        ref = oracle_mod.OracleRobot(N)
        ref.set_state(*ens.download_state(0))
        line = np.array([[y[3 + 2 * target], y[4 + 2 * target], 0.0, 0.0, 0.0, 0.0]])
        res = ens.localize([0.0, 0.0, 0.0], line[None], [1])[0]
        m = ref.localize(line, [0.0, 0.0, 0.0])
        assert res["match"] == m == [target], (res["match"], m)
        assert ref.status & 1 == want
        assert res["status"] & ekf_mod.ST_SINGULAR_S == want, (target, res["status"])
        ens.close()


@pytest.mark.parametrize("arith", [1, 2])
@pytest.mark.parametrize("prec,N,T,extra_every", [(1, 1024, 12, 0), (1, 200, 8, 3), (2, 512, 10, 0), (1, 100, 16, 0),
                                                  (1, 1024, 20, 0)])
def test_bf16_2x4_flush_equals_2x2(ekf_mod, monkeypatch, prec, N, T, extra_every, arith):
    """The split-bf16 / split-fp16 flush on 2 × 4 wave-tiles (flush_bf24_kernel, EKF_OPT_FLUSH_FORM = 24)
    and on 2 × 2 wave-tiles (flush_f32_wave_kernel<.., true>, default) run the same MFMA sequence per element
    (same part products in the same order, bf16 MFMA deterministic): bit-identical state for plain
    groups, fp32 and fp16 storage, block sizes that are not multiples of the wave-tile. Groups with
    augmented rows: the 2 × 4 form runs every wave-tile on the general loop, the 2 × 2 form only
    those the new rows touch, so the two agree to the storage bar there."""
    E = 3
    active = N - 12 - 2 * ((3 * T + 1) // extra_every) if extra_every else N - 10
    w = G.make_world(N, active=active)
    st = G.initial_state(w)
    if arith == 1 and T > 16:
        pytest.skip("EKF_ARITH_BF16X6: flush_interval <= 16")
    a = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=arith, options={"flush_form": 24})
    b = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=arith)
    assert a.flush_kernel_name(T).startswith("flush_bf24_kernel"), a.flush_kernel_name(T)
    assert b.flush_kernel_name(T).endswith(", true>"), b.flush_kernel_name(T)
    assert a.flush_kernel_name(T).endswith(", true>") == (arith == 2), a.flush_kernel_name(T)
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(3)
    for step in range(1, 3 * T + 2):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=6 if extra_every else 8)
        if extra_every and step % extra_every == 0:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            ln = np.concatenate([ln, ex], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        ra, rb = a.localize(enc, ln, nl), b.localize(enc, ln, nl)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        assert sa == sb, e
        if extra_every:
            assert rel(Pa, Pb) <= (1e-6 if prec == 1 else 1e-3), (e, rel(Pa, Pb))
            assert rel(ya, yb) <= 1e-10, (e, rel(ya, yb))
        else:
            assert np.array_equal(Pa, Pb) and np.array_equal(ya, yb), e


@pytest.mark.parametrize("prec,N,T,extra_every,active", [(1, 1024, 20, 0, 0), (1, 1000, 12, 0, 0), (2, 512, 10, 0, 0),
                                                         (1, 200, 8, 3, 0), (1, 100, 16, 0, 0), (2, 2048, 24, 0, 0),
                                                         (1, 1024, 12, 3, 300), (2, 4096, 20, 4, 1500),
                                                         (1, 64, 6, 2, 0), (1, 256, 8, 2, 240), (2, 256, 14, 3, 240),
                                                         (1, 4096, 20, 0, 0)])
def test_f16_quad_flush_equals_2x2(ekf_mod, prec, N, T, extra_every, active):
    """The split-fp16 flush on groups of 2 × 2 wave-tiles whose operand planes loader waves move into
    an LDS ring by DMA (flush_f16q_kernel, EKF_OPT_FLUSH_FORM = 44) and the 2 × 2 wave form (default)
    run the same three products per accumulator and step in the same order on the same planes, and
    send the same wave-tiles (new rows, σ changes) through the general loop: equal state for plain
    groups, groups with augmented rows, fp32 and fp16 storage, partly filled maps (whole dead groups
    skipped; a dead wave-tile in a live group recomputed unchanged), block sizes that are not
    multiples of the group, step counts whose ring does not divide them (14, 6)."""
    E = 3
    if not active:
        active = N - 12 - 2 * ((3 * T + 1) // extra_every) if extra_every else N - 10
    w = G.make_world(N, active=active)
    st = G.initial_state(w)
    a = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=2, options={"flush_form": 44})
    b = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=2)
    assert a.flush_kernel_name(T).startswith("flush_f16q_kernel"), a.flush_kernel_name(T)
    assert b.flush_kernel_name(T).startswith("flush_f32_wave_kernel"), b.flush_kernel_name(T)
    for ens in (a, b):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    rng = np.random.default_rng(5)
    for step in range(1, 3 * T + 2):
        enc, ln, nl = G.make_scan(w, step, instances=E, lines=6 if extra_every else 8)
        if extra_every and step % extra_every == 0:
            ex = G.random_lines(rng, 2)[None].repeat(E, axis=0)
            ln = np.concatenate([ln, ex], axis=1)
            nl = np.full(E, ln.shape[1], dtype=np.int32)
        ra, rb = a.localize(enc, ln, nl), b.localize(enc, ln, nl)
        for e in range(E):
            assert ra[e]["match"] == rb[e]["match"], (step, e)
            assert ra[e]["status"] == rb[e]["status"], (step, e)
    for e in range(E):
        Pa, ya, sa, pa = a.download_state(e)
        Pb, yb, sb, pb = b.download_state(e)
        assert sa == sb, e
        assert np.array_equal(Pa, Pb) and np.array_equal(ya, yb), (e, rel(Pa, Pb))
    a.close()
    b.close()


def _gate_case(ekf_mod, oracle_mod, prec, p22, p2a, daa, delta):
    """One landmark at (alpha 0.3, r 2.0) seen from the pose (0, 0, 0) without motion (the encoder
    equals the pose: F = I, Q = 0, Robot.cpp:136-286), its angle variance p22 / daa / covariance
    p2a, and one line at Mahalanobis distance² = 0.16·(1 + delta) from it (v1 = 0, S01 = 0: d² =
    v0²/S00 with S00 = p22 − 2·p2a + daa + R00 from the STORED block). Returns (status, match,
    the restatement's match)."""
    N = 16
    n = 3 + 2 * N
    P = np.zeros((n, n))
    P[0, 0] = P[1, 1] = 1e-3
    P[2, 2] = p22
    P[3, 3] = daa
    P[4, 4] = 1e-3
    P[2, 3] = P[3, 2] = p2a
    for k in range(5, n):
        P[k, k] = 1e-3
    y = np.zeros(n)
    y[3], y[4] = 0.3, 2.0
    ens = ekf_mod.Ensemble(N, 1, prec, max_lines=8)
    ens.upload_state(0, P, y, 1, [0.0, 0.0, 0.0])
    Ps = ens.download_state(0)[0]
    R00 = 1e-3
    S00 = Ps[2, 2] - 2.0 * Ps[2, 3] + Ps[3, 3] + R00
    v0 = np.sqrt(0.16 * (1.0 + delta) * S00)
    line = np.array([[0.3 + v0, 2.0, R00, 0.0, 0.0, 1e-3]])
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(*ens.download_state(0))
    r = ens.localize(np.zeros((1, 3)), line[None], [1])[0]
    m = ref.localize(line, np.zeros(3))
    ens.close()
    return r["status"], r["match"][0], m[0]


@pytest.mark.parametrize("prec", [1, 2])
def test_gate_storage_precision_flag(ekf_mod, oracle_mod, prec):
    """EKF_ST_PRECISION from the gate (gate_eta): a distance within the stored state's
    precision of the 0.4 gate (Robot.cpp:489) is reported, both where S00 is the difference of
    terms 1e7 times larger (the robot and landmark angles correlated to 1 − 1e-7: a run-away
    filter) and, without cancellation, within 1e-7 of the threshold; a clear decision is not, and
    matches the restatement from the same stored state."""
    ST = ekf_mod.ST_PRECISION
    # cancellation: flagged on either side of the gate
    for delta in (0.05, -0.05):
        st, _, _ = _gate_case(ekf_mod, oracle_mod, prec, 1e4, 1e4 - 1e-3, 1e4, delta)
        assert st & ST, (prec, delta, st)
    # no cancellation, clear decisions: not flagged, the reference's decision
    for delta, want in ((0.05, -1), (-0.05, 0)):
        st, got, ref = _gate_case(ekf_mod, oracle_mod, prec, 1e-3, 0.0, 1e-3, delta)
        assert not (st & ST), (prec, delta, st)
        assert got == ref == want, (prec, delta, got, ref)
    if prec == 1:   # (fp16 storage: eta 2^-8 flags ±1 % already)
        st, _, _ = _gate_case(ekf_mod, oracle_mod, prec, 1e-3, 0.0, 1e-3, 1e-7)
        assert st & ST, st
