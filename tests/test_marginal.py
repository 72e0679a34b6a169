"""CPU tests of the marginal (camera-block) truncated-SVD solver of aslam_incremental_calibration's
LinearSolver, restated in the oracle (oracle/kb_oracle.c kbo_marginal_solve / kbo_arrow_solve_ex).

Pinned by the reference's own test (incremental_calibration/test/LinearSolverTest.cpp:37-70,130-150): a random
dense 100 x 30 system b = A x is solved for every marginalisation index j = 1..29, with and without column scaling,
and the residual |b - A x_est| must vanish (tol 1e-9).  The SVD itself is checked against numpy's eigvalsh.
"""
import numpy as np
import pytest

from kalibr_amd import synth


def _schur(A, b, j):
    Al, Ar = A[:, :j], A[:, j:]
    H = Al.T @ Al
    K = np.linalg.solve(H, Al.T @ Ar)
    S = Ar.T @ Ar - (Al.T @ Ar).T @ K
    br = Ar.T @ b - K.T @ (Al.T @ b)
    return S, br, Ar


@pytest.mark.parametrize("scaling", [False, True])
def test_reference_linear_solver_random_dense(oracle_mod, scaling):
    """LinearSolverTest.cpp testLinearSolver 'standard case': evaluateSVDSPQRSolver over every split."""
    rng = np.random.default_rng(7)
    A = rng.uniform(-1, 1, (100, 30))
    x = rng.uniform(-1, 1, 30)
    b = A @ x
    for j in range(1, 30):
        S, br, Ar = _schur(A, b, j)
        opts = oracle_mod.marg_opts(100, column_scaling=scaling, eps_svd=oracle_mod.EPS)
        xr, info = oracle_mod.marginal_solve(S, br, np.sum(Ar * Ar, axis=0), opts)
        xl = np.linalg.lstsq(A[:, :j], b - Ar @ xr, rcond=None)[0]
        xe = np.concatenate([xl, xr])
        assert np.linalg.norm(b - A @ xe) < 1e-9
        assert info["rank"] == 30 - j


def test_rank_deficient_zero_column(oracle_mod):
    """LinearSolverTest.cpp 'rank-deficient case 1' (a zero column): the column-norm tolerance zeroes its scale,
    the SVD rank drops by one and the remaining system is still solved exactly."""
    rng = np.random.default_rng(8)
    A = rng.uniform(-1, 1, (100, 30))
    A[:, 25] = 0.0
    x = rng.uniform(-1, 1, 30)
    b = A @ x
    j = 20
    S, br, Ar = _schur(A, b, j)
    xr, info = oracle_mod.marginal_solve(S, br, np.sum(Ar * Ar, axis=0), oracle_mod.marg_opts(100, eps_svd=1e-6))
    assert info["rank"] == 9 and info["sv"][-1] == 0.0 and np.isinf(info["gap"])  # sv_rank = 0
    assert xr[25 - j] == 0.0
    xl = np.linalg.lstsq(A[:, :j], b - Ar @ xr, rcond=None)[0]
    assert np.linalg.norm(b - A @ np.concatenate([xl, xr])) < 1e-9


def test_singular_values_and_rank_rules(oracle_mod):
    """rankTol = sv_0 * epsSVD * n, estimateNumericalRank counts down from the back and never below 1, svGap
    = sv_(rank-1) / sv_rank (linalg.cpp:243-282); singular values against numpy."""
    rng = np.random.default_rng(9)
    n = 12
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    sv = np.array([10.0 ** (-k) for k in range(n)])
    S = Q @ np.diag(sv) @ Q.T
    x, info = oracle_mod.marginal_solve(S, np.ones(n), None, oracle_mod.marg_opts(50, column_scaling=False,
                                                                                 eps_svd=1e-6))
    assert np.allclose(info["sv"], sv, rtol=1e-9, atol=1e-15)
    assert info["tol"] == pytest.approx(sv[0] * 1e-6 * n)
    assert info["rank"] == 5  # sv_4 = 1e-4 > tol = 1.2e-5 >= sv_5 = 1e-5
    assert info["gap"] == pytest.approx(info["sv"][info["rank"] - 1] / info["sv"][info["rank"]])
    # the solve is the truncated pseudo-inverse
    V = info["V"][:, : info["rank"]]
    ref = V @ np.diag(1.0 / info["sv"][: info["rank"]]) @ V.T @ np.ones(n)
    assert np.abs(x - ref).max() <= 1e-9 * np.abs(ref).max()


def test_arrow_marginal_equals_cholesky_when_full_rank(oracle_mod):
    p = synth.make_config(2, n_frames=12, seed_offset=5)
    o = oracle_mod.Oracle(p)
    A = o.arrow(p.state_init)
    ok, dx = o.solve(A, 0.0)
    okm, dxm, info = o.solve_marginal(A)
    assert ok and okm and info["rank"] == p.cam_cols
    assert np.abs(dxm - dx).max() <= 1e-8 * np.abs(dx).max()


def test_gn_with_marginal_solver(oracle_mod):
    """Optimizer2 + GaussNewtonTrustRegionPolicy + LinearSolver, the IncrementalEstimator's optimizer
    (IncrementalEstimator.cpp:46-66; CalibrateCameras.cpp:258-272: maxIterations 20, epsSVD 1e-6, scaling)."""
    p = synth.make_config(1, n_frames=10)
    o = oracle_mod.Oracle(p)
    mo = oracle_mod.marg_opts(2 * p.n_corners)
    st, r = o.optimize(p.state_init, policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1e-3, marg=mo)
    st2, r2 = o.optimize(p.state_init, policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1e-3)
    assert r["iterations"] == r2["iterations"] and np.abs(st - st2).max() < 1e-6
    ai, si = r["analyze_info"], r["solve_info"]
    assert si["rank"] == ai["rank"] == p.cam_cols
    # analyzeMarginal: singular values of the unscaled Schur complement of the last built system
    assert ai["sv"][0] > 1e3 * si["sv"][0]  # unscaled (pixel^2 per unit) vs column-scaled (O(1))
    assert ai["log2sum"] == pytest.approx(np.sum(np.log2(ai["sv"][: ai["rank"]])))
