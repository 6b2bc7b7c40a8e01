"""Rollback on an exchange timeout (slam_ekf.h EKF_ST_SYNC_TIMEOUT).

The reference always commits a valid state (Robot.cpp:909-917: localize prints the GSL status and
returns). Here an instance spans G cooperating workgroups; if one of them never arrives, the
others give up after a bounded spin. The launch must then leave that instance exactly as it was
before the call — robot strip, mean, pose, savedLineCount and the landmark block, including across
the deferred flushes of later groups — while every other instance of the same launch proceeds.
The test hook EKF_OPT_TEST_DROP_WG = e + 1 makes the last workgroup of instance e never run (a
workgroup that is not co-resident), EKF_OPT_SPIN_LOG2 shortens the spin bound, and
EKF_OPT_TEST_VERDICT_TIMEOUT = e + 1 makes one non-lead workgroup's verdict poll time out while the
others complete (the race of two polls against the spin bound). The library reads no environment
variables: a stray EKF_TEST_DROP_WG in the environment changes nothing.
"""
import numpy as np
import pytest

from slam_ros_amd import scan_gen as G

pytestmark = pytest.mark.gpu


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.mark.parametrize("prec,T,spec", [(1, 4, "1"), (1, 1, "0"), (0, 3, "1"), (2, 4, "1")])
def test_timeout_rolls_back_the_instance(ekf_mod, oracle_mod, prec, T, spec, hook="test_drop_wg", arith=0, nt=0):
    N, E = 1024, 3   # G = 6 workgroups per instance (16 / 8 with 64 / 128 landmarks per workgroup)
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, E, prec, max_lines=8, flush_interval=T, arith=arith,
                           options={hook: 2, "spin_log2": 12, "speculate": int(spec), "scan_threads": nt})
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    before = ens.download_state(1)
    ref = oracle_mod.OracleRobot(N)
    ref.set_state(*ens.download_state(0))
    tol = {0: 1e-10, 1: 1e-6, 2: 3e-3}[prec]
    for step in range(1, 2 * T + 3):
        enc, lines, nl = G.make_scan(w, step, instances=E)
        res = ens.localize(enc, lines, nl)
        # the dropped instance: timed out, rolled back, nothing reported as matched
        assert res[1]["status"] & ekf_mod.ST_SYNC_TIMEOUT, (step, res[1])
        assert res[1]["matches"] == 0 and all(m == -1 for m in res[1]["match"]), res[1]
        assert res[1]["saved"] == st.saved and ens.result_words(1)[15] == 1
        np.testing.assert_array_equal(res[1]["pose"], before[3])
        # the other instances of the same launches proceed as the restatement does
        m = ref.localize(lines[0], enc[0])
        assert res[0]["match"] == m and res[0]["status"] == 0, (step, res[0])
        assert res[2]["status"] == 0 and res[2]["matches"] == 8, (step, res[2])
    after = ens.download_state(1)   # drains: every group's flush has run over the rolled-back steps
    np.testing.assert_array_equal(after[0], before[0])
    np.testing.assert_array_equal(after[1], before[1])
    assert after[2] == before[2]
    np.testing.assert_array_equal(after[3], before[3])
    P, y, saved, pose = ens.download_state(0)
    assert rel(P, ref.P_t0) <= tol * (2 * T + 2) and rel(y, ref.y) <= 1e-8 * (2 * T + 2)
    assert saved == ref.savedLineCount
    ens.close()


@pytest.mark.parametrize("prec,T", [(1, 4), (0, 3), (2, 4)])
def test_verdict_timeout_of_one_workgroup_rolls_back(ekf_mod, oracle_mod, prec, T):
    """One non-lead workgroup's speculative verdict poll times out while every other workgroup
    (the lead included) sees a passed verdict: that workgroup must not restart alone on the
    sequential path and the lead must not commit without its completion word: the
    instance's calls roll back, the other instances proceed."""
    test_timeout_rolls_back_the_instance(ekf_mod, oracle_mod, prec, T, "1", hook="test_verdict_timeout")


@pytest.mark.parametrize("prec,nt,hook", [(1, 64, "test_drop_wg"), (1, 128, "test_drop_wg"), (2, 64, "test_drop_wg"),
                                          (1, 64, "test_verdict_timeout")])
def test_timeout_rolls_back_narrow_workgroups(ekf_mod, oracle_mod, prec, nt, hook):
    """The same with the split-fp16 association kernel on 64 / 128 landmarks per workgroup
    (EKF_OPT_SCAN_THREADS): more workgroups per instance in the exchanges, the collection and the
    completion words (sized for the narrowest width)."""
    test_timeout_rolls_back_the_instance(ekf_mod, oracle_mod, prec, 4, "1", hook=hook, arith=2, nt=nt)


def test_environment_is_not_read(ekf_mod, monkeypatch):
    """The former environment knobs have no effect: a stray EKF_TEST_DROP_WG (which used to make
    an instance time out on every scan) leaves every call committing."""
    monkeypatch.setenv("EKF_TEST_DROP_WG", "0")
    monkeypatch.setenv("EKF_SPECULATE", "2")
    monkeypatch.setenv("EKF_SPIN_LOG2", "8")
    test_no_rollback_without_timeout(ekf_mod)


def test_no_rollback_without_timeout(ekf_mod):
    """A normal launch commits: the committed copy alternates, nothing is rolled back."""
    N, E = 1024, 2
    w = G.make_world(N)
    st = G.initial_state(w)
    ens = ekf_mod.Ensemble(N, E, 1, max_lines=8, flush_interval=2)
    assert ens.get_option("test_drop_wg") == 0 and ens.get_option("speculate") == 1
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    for step in range(1, 4):
        enc, lines, nl = G.make_scan(w, step, instances=E)
        res = ens.localize(enc, lines, nl)
        for e in range(E):
            assert res[e]["status"] == 0 and res[e]["matches"] == 8
            assert ens.result_words(e)[15] == 0
    ens.close()
