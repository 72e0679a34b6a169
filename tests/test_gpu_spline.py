"""configs[4] on the GPU (kb_sp_* C-ABI) against the CPU restatement (oracle/kb_oracle_spline.c).

Tolerances (FP64 throughout): cost rel 1e-12; normal-equation blocks rel 1e-10 of the block's scale; solve dx
rel 1e-8 (block cyclic reduction on the device vs band Cholesky on the CPU); full GN / LM runs: identical
iteration counts, state within 1e-6 (north_star bar on intrinsics / extrinsics).
"""
import numpy as np
import pytest

from kalibr_amd import capi, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def case():
    p = synth.make_spline_config(n_frames=40)
    return p, O.SplineOracle(p), capi.SplineSolver(p)


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def test_cost_parity(case):
    p, o, g = case
    for st in (p.state_init, p.state_truth):
        g.set_state(st)
        J = g.eval_cost()
        Jo = o.cost(st)
        assert abs(J - Jo) <= 1e-12 * Jo, (J, Jo)


def test_normal_equations_parity(case):
    p, o, g = case
    g.set_state(p.state_init)
    g.build()
    s = g.system()
    so = o.system(p.state_init, nthreads=4)
    assert abs(s["cost"] - so["cost"]) <= 1e-12 * so["cost"]
    for k in ("Hcc", "Hsc", "gc", "gs"):
        assert _rel(s[k], so[k]) < 1e-10, k
    assert _rel(s["Hband"], so["Hband"]) < 1e-10
    r = g.rhs()
    assert _rel(r, np.concatenate([so["gc"], so["gs"]])) < 1e-10


@pytest.mark.parametrize("lam", [0.0, 10.0])
def test_solve_parity(case, lam):
    p, o, g = case
    g.set_state(p.state_init)
    g.build()
    g.set_constant_conditioner(lam)
    ok, dx = g.solve()
    so = o.system(p.state_init, nthreads=4)
    ok_o, dx_o = o.solve(so, lam)
    assert ok and ok_o
    assert _rel(dx, dx_o) < 1e-8


def test_update_and_revert(case):
    p, o, g = case
    g.set_state(p.state_init)
    g.build()
    g.set_constant_conditioner(0.0)
    ok, dx = g.solve()
    assert ok
    dX = g.apply_update()
    st_o, dX_o = o.apply_update(p.state_init, dx)
    assert abs(dX - dX_o) <= 1e-15 * dX_o
    assert np.abs(g.get_state() - st_o).max() < 1e-12
    g.revert()
    assert np.array_equal(g.get_state(), p.state_init)
    # host-given dx takes the same update rules
    g.apply_update(dx)
    assert np.abs(g.get_state() - st_o).max() < 1e-12


@pytest.mark.parametrize("policy", ["gn", "lm"])
def test_optimize_parity(case, policy):
    p, o, g = case
    g.set_state(p.state_init)
    res = g.optimize(policy=policy, lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    st_o, res_o = o.optimize(p.state_init, policy=policy, lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3,
                             nthreads=4)
    assert res["iterations"] == res_o["iterations"] and res["failed_iterations"] == res_o["failed_iterations"]
    assert abs(res["J_final"] - res_o["J_final"]) <= 1e-9 * res_o["J_final"]
    assert np.abs(g.get_state() - st_o).max() < 1e-6


def test_full_size_gn_properties():
    """configs[4] at its full size (1200 frames, 2 cameras, 200 Hz IMU): the captured GN passes run, the cost
    falls to the noise level and the calibration is recovered."""
    p = synth.make_spline_config()
    g = capi.SplineSolver(p)
    g.set_state(p.state_init)
    J0 = g.eval_cost()
    g.run_gn(8)
    J = g.eval_cost()
    st = g.get_state()
    assert np.isfinite(J) and J < 1e-4 * J0
    expect = 2 * p.n_corners * p.meta["noise_px"] ** 2 + 6 * p.n_imu
    assert J < 1.2 * expect
    N = p.n_cams
    intr = (st - p.state_truth)[: N * synth.MAX_INTR].reshape(N, synth.MAX_INTR)
    assert np.abs(intr[:, :4]).max() < 0.5
    # deterministic: the same passes from the same state give the same bits
    g.set_state(p.state_init)
    g.run_gn(8)
    assert np.array_equal(g.get_state(), st)


# ---- BSplineMotionError (kb_sp_set_motion_error) against the oracle's restatement ----
W_MOTION = np.diag([4.0, 4.0, 4.0, 1.0, 1.0, 1.0]) + 0.1 * (np.ones((6, 6)) - np.eye(6))


@pytest.fixture(scope="module")
def motion_case():
    p = synth.make_spline_config(n_frames=40)
    g = capi.SplineSolver(p)
    g.set_motion_error(W_MOTION, 2)
    return p, O.SplineOracle(p, motion_W=W_MOTION, motion_order=2), g


def test_motion_error_cost_system_solve(motion_case):
    """Q is formed two independent ways -- the reference's moment matrices M^T D^T V D M on the device side's host
    (segmentQuadraticIntegral) and Gauss-Legendre quadrature of the basis products in the oracle -- which agree
    entry-wise to ~1e-15 relative; c^T Q c cancels against Q's ~1/dt^3 entries, so the cost bar is 1e-10."""
    p, o, g = motion_case
    for st in (p.state_init, p.state_truth):
        g.set_state(st)
        J, Jo = g.eval_cost(), o.cost(st)
        assert abs(J - Jo) <= 1e-10 * Jo, (J, Jo)
    g.set_state(p.state_init)
    g.build()
    s = g.system()
    so = o.system(p.state_init, nthreads=4)
    assert abs(s["cost"] - so["cost"]) <= 1e-10 * so["cost"]
    for k in ("Hcc", "Hsc", "gc", "gs", "Hband"):
        assert _rel(s[k], so[k]) < 1e-10, k
    for lam in (0.0, 10.0):
        g.set_constant_conditioner(lam)
        ok, dx = g.solve()
        ok_o, dx_o = o.solve(so, lam)
        assert ok and ok_o and _rel(dx, dx_o) < 1e-8


@pytest.mark.parametrize("policy", ["gn", "lm"])
def test_motion_error_optimize_parity(motion_case, policy):
    p, o, g = motion_case
    g.set_state(p.state_init)
    res = g.optimize(policy=policy, lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    st_o, res_o = o.optimize(p.state_init, policy=policy, lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3,
                             nthreads=4)
    assert res["iterations"] == res_o["iterations"] and res["failed_iterations"] == res_o["failed_iterations"]
    assert abs(res["J_final"] - res_o["J_final"]) <= 1e-9 * res_o["J_final"]
    assert np.abs(g.get_state() - st_o).max() < 1e-6


def test_motion_error_removed_restores_the_plain_system(motion_case):
    p, o, g = motion_case
    g.set_motion_error(None)
    g.set_state(p.state_init)
    o0 = O.SplineOracle(p)
    assert abs(g.eval_cost() - o0.cost(p.state_init)) <= 1e-12 * o0.cost(p.state_init)
    g.set_motion_error(W_MOTION, 2)


# ---- full-size configs[4] (1200 frames, 279 k corners, 12 k IMU samples) against the oracle ----
@pytest.fixture(scope="module")
def full_case():
    p = synth.make_spline_config()
    return p, O.SplineOracle(p), capi.SplineSolver(p)


def _full_threads():
    import os
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _compare_runs(res, st, res_o, st_o, lam_rtol=1e-12):
    """identical iteration counts and accept/revert sequence, per-pass J within 1e-9, state within 1e-6"""
    assert res["iterations"] == res_o["iterations"] and res["failed_iterations"] == res_o["failed_iterations"]
    tr, tro = res["trace"], res_o["trace"]
    assert tr.shape == tro.shape, (tr.shape, tro.shape)
    assert np.array_equal(tr[:, 3], tro[:, 3])  # accepted flags
    ok = np.isfinite(tro[:, 0])
    assert np.all(np.abs(tr[ok, 0] - tro[ok, 0]) <= 1e-9 * np.abs(tro[ok, 0]))
    assert np.allclose(tr[:, 1], tro[:, 1], rtol=lam_rtol, atol=0.0)  # lambda schedule
    assert abs(res["J_final"] - res_o["J_final"]) <= 1e-9 * res_o["J_final"]
    assert np.abs(st - st_o).max() < 1e-6


@pytest.mark.parametrize("policy", ["gn", "lm"])
def test_full_size_optimize_parity(full_case, policy):
    """configs[4] at full size: GN (maxIt 20) and Kalibr2-default LM (lambda0 10) against SplineOracle"""
    p, o, g = full_case
    g.set_motion_error(None)
    g.set_state(p.state_init)
    kw = dict(policy=policy, lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    res = g.optimize(**kw)
    st_o, res_o = o.optimize(p.state_init, nthreads=_full_threads(), **kw)
    _compare_runs(res, g.get_state(), res_o, st_o)


def test_full_size_motion_error_parity(full_case):
    """the BSplineMotionError variant at full size (GN, maxIt 20)"""
    p, _, g = full_case
    om = O.SplineOracle(p, motion_W=W_MOTION, motion_order=2)
    g.set_motion_error(W_MOTION, 2)
    try:
        g.set_state(p.state_init)
        kw = dict(policy="gn", lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
        res = g.optimize(**kw)
        st_o, res_o = om.optimize(p.state_init, nthreads=_full_threads(), **kw)
        _compare_runs(res, g.get_state(), res_o, st_o)
    finally:
        g.set_motion_error(None)


# ---- ErrorTermEuclidean priors on the spline position (kb_sp_set_position_priors) against the oracle ----
@pytest.fixture(scope="module")
def prior_case():
    p = synth.make_spline_config(n_frames=40)
    pri = synth.make_position_priors(p, 0, rate=50.0, seed=3)  # a 50 Hz position track, anisotropic covariances
    g = capi.SplineSolver(p)
    g.set_position_priors(*pri)
    return p, pri, O.SplineOracle(p, position_priors=pri), g


def test_position_prior_cost_system_solve(prior_case):
    """per-term restatement on both sides (e = p(t) - prior, H += w w^T (x) N^-1, rhs -= w (x) N^-1 e): cost 1e-12,
    blocks 1e-10, dx 1e-8"""
    p, pri, o, g = prior_case
    assert pri[0].size > 50
    for st in (p.state_init, p.state_truth):
        g.set_state(st)
        J, Jo = g.eval_cost(), o.cost(st)
        assert abs(J - Jo) <= 1e-12 * Jo, (J, Jo)
    g.set_state(p.state_init)
    g.build()
    s = g.system()
    so = o.system(p.state_init, nthreads=4)
    assert abs(s["cost"] - so["cost"]) <= 1e-12 * so["cost"]
    for k in ("Hcc", "Hsc", "gc", "gs", "Hband"):
        assert _rel(s[k], so[k]) < 1e-10, k
    assert _rel(g.rhs(), np.concatenate([so["gc"], so["gs"]])) < 1e-10
    for lam in (0.0, 10.0):
        g.set_constant_conditioner(lam)
        ok, dx = g.solve()
        ok_o, dx_o = o.solve(so, lam)
        assert ok and ok_o and _rel(dx, dx_o) < 1e-8


@pytest.mark.parametrize("policy", ["gn", "lm"])
def test_position_prior_optimize_parity(prior_case, policy):
    p, pri, o, g = prior_case
    g.set_state(p.state_init)
    kw = dict(policy=policy, lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    res = g.optimize(**kw)
    st_o, res_o = o.optimize(p.state_init, nthreads=4, **kw)
    # the LM schedule divides the cost decrease by the predicted one: with the priors' large weights (N = (2 mm)^2)
    # a 1e-13 cost difference moves lambda in its 1e-10th digit, so the schedule bar here is 1e-8
    _compare_runs(res, g.get_state(), res_o, st_o, lam_rtol=1e-8)


def test_position_prior_with_motion_error(prior_case):
    """priors and BSplineMotionError together (both coefficient-only terms share the node-cost path)"""
    p, pri, _, g = prior_case
    om = O.SplineOracle(p, motion_W=W_MOTION, motion_order=2, position_priors=pri)
    g.set_motion_error(W_MOTION, 2)
    try:
        g.set_state(p.state_init)
        assert abs(g.eval_cost() - om.cost(p.state_init)) <= 1e-10 * om.cost(p.state_init)
        res = g.optimize(policy="gn", lambda0=10.0, max_iterations=10, eps_x=1e-3, eps_j=1e-3)
        st_o, res_o = om.optimize(p.state_init, policy="gn", lambda0=10.0, max_iterations=10, eps_x=1e-3, eps_j=1e-3,
                                  nthreads=4)
        _compare_runs(res, g.get_state(), res_o, st_o)
    finally:
        g.set_motion_error(None)


def test_position_prior_removed_and_bad_input(prior_case):
    p, pri, _, g = prior_case
    g.set_position_priors()
    g.set_state(p.state_init)
    o0 = O.SplineOracle(p)
    assert abs(g.eval_cost() - o0.cost(p.state_init)) <= 1e-12 * o0.cost(p.state_init)
    with pytest.raises(capi.KbError):  # outside the spline's time range
        g.set_position_priors(pri[0] + 1e3, pri[1], pri[2])
    with pytest.raises(capi.KbError):  # not positive definite
        g.set_position_priors(pri[0], pri[1], -pri[2])
    # det > 0 and N00 > 0, but indefinite: diag(1, -1, -1) (the 2 x 2 leading minor is negative)
    indef = np.broadcast_to(np.diag([1.0, -1.0, -1.0]), pri[2].shape).copy()
    with pytest.raises(capi.KbError):
        g.set_position_priors(pri[0], pri[1], indef)
    # repeated calls replace the prior tables (no accumulation, same system)
    g.set_position_priors(*pri)
    J1 = g.eval_cost()
    for _ in range(3):
        g.set_position_priors(*pri)
    assert g.eval_cost() == J1


def test_deep_level_kernel_parity(case, monkeypatch):
    """KSP_DEEP=1 (the cyclic reduction's deep levels in one block, measured slower and kept opt-in): the same GN run
    as the per-level kernels with the C + 1 column back substitution (KSP_ZS=0: the same arithmetic in the same order,
    state and J bitwise) and as the oracle"""
    p, o, _ = case
    kw = dict(policy="gn", lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    monkeypatch.setenv("KSP_ZS", "0")
    g = capi.SplineSolver(p)
    g.set_state(p.state_init)
    res = g.optimize(**kw)
    st = g.get_state()
    monkeypatch.setenv("KSP_DEEP", "1")
    gd = capi.SplineSolver(p)
    gd.set_state(p.state_init)
    res_d = gd.optimize(**kw)
    assert res_d["iterations"] == res["iterations"] and res_d["J_final"] == res["J_final"]
    assert np.array_equal(gd.get_state(), st)
    st_o, res_o = o.optimize(p.state_init, nthreads=4, **kw)
    assert res_d["iterations"] == res_o["iterations"]
    assert abs(res_d["J_final"] - res_o["J_final"]) <= 1e-9 * res_o["J_final"]
    assert np.abs(gd.get_state() - st_o).max() < 1e-6


def test_one_column_back_substitution_matches_full(case, monkeypatch):
    """The default solve (Schur complement from the forward reduction, sum_i Z_R,i^T Z_R,i, and the back substitution
    with the one column [-dtheta | 1]) against the C + 1 column back substitution (KSP_ZS=0): the same dx to 1e-10
    at lambda 0 and 10, and the same GN run (iteration count, J to 1e-12, state to 1e-9)"""
    p, o, g = case
    monkeypatch.setenv("KSP_ZS", "0")
    gf = capi.SplineSolver(p)
    for sv in (g, gf):
        sv.set_state(p.state_init)
        sv.build()
    for lam in (0.0, 10.0):
        dxs = []
        for sv in (g, gf):
            sv.set_constant_conditioner(lam)
            ok, dx = sv.solve()
            assert ok
            dxs.append(dx)
        assert np.abs(dxs[0] - dxs[1]).max() <= 1e-10 * np.abs(dxs[1]).max(), lam
    kw = dict(policy="gn", lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    res = []
    for sv in (g, gf):
        sv.set_state(p.state_init)
        res.append((sv.optimize(**kw), sv.get_state()))
    assert res[0][0]["iterations"] == res[1][0]["iterations"]
    assert abs(res[0][0]["J_final"] - res[1][0]["J_final"]) <= 1e-12 * res[1][0]["J_final"]
    assert np.abs(res[0][1] - res[1][1]).max() < 1e-9
