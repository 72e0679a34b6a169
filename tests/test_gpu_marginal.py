"""GPU parity of the marginal truncated-SVD solver (aslam_incremental_calibration LinearSolver, k_marg) against the
oracle's restatement (oracle/kb_oracle.c kbo_marginal_solve), through the C-ABI (kb_solve_marginal /
kb_analyze_marginal).

Tolerances (FP64; Jacobi rotations in a different association order than the oracle):
  rank, sweeps-independent quantities     exact
  singular values                          |sv_gpu - sv_oracle| <= 1e-11 sv_0
  dx                                       rel 1e-8 of max|dx|
  GN loop with the marginal solver         final state within 1e-6, same iteration count
"""
import numpy as np
import pytest

from kalibr_amd import synth

pytestmark = pytest.mark.gpu

PROBLEMS = {
    "c1": lambda: synth.make_config(1, n_frames=20),
    "c1_one_view": lambda: synth.make_config(1, n_frames=1),  # rank-deficient camera block
    "c2_small": lambda: synth.make_config(2, n_frames=40),
    "c3_small": lambda: synth.make_config(3, n_frames=30),
    "c4_small": lambda: synth.make_config(4, n_frames=24, p_view=0.7),  # C = 106
    "c6_small": lambda: synth.make_config(6, n_frames=30, p_view=0.8),
}


@pytest.fixture(scope="module")
def capi():
    from kalibr_amd import capi as K
    return K


@pytest.mark.parametrize("name", list(PROBLEMS))
def test_solve_marginal_matches_oracle(capi, oracle_mod, name):
    p = PROBLEMS[name]()
    o = oracle_mod.Oracle(p)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.build()
    ok, dx, info = g.solve_marginal()
    A = o.arrow(p.state_init)
    ok_o, dx_o, info_o = o.solve_marginal(A)
    assert ok and ok_o
    assert info["rank"] == info_o["rank"]
    assert np.abs(info["sv"] - info_o["sv"]).max() <= 1e-11 * info_o["sv"][0]
    assert info["tol"] == pytest.approx(info_o["tol"], rel=1e-12)
    assert np.abs(dx - dx_o).max() <= 1e-8 * np.abs(dx_o).max()
    # the singular vectors of the kept subspace agree up to sign: compare projectors
    r = info["rank"]
    P, Po = info["V"][:, :r] @ info["V"][:, :r].T, info_o["V"][:, :r] @ info_o["V"][:, :r].T
    assert np.abs(P - Po).max() < 1e-8
    # analyzeMarginal: unscaled SVD of the same system
    ai = g.analyze_marginal()
    _, ai_o = oracle_mod.marginal_solve(A["Hcc"] - o.schur_partial(A, 0.0, 0, p.n_frames)[1], np.zeros(p.cam_cols),
                                        None, oracle_mod.marg_opts(2 * p.n_corners, column_scaling=False))
    assert np.abs(ai["sv"] - ai_o["sv"]).max() <= 1e-11 * ai_o["sv"][0]


def test_one_view_is_rank_deficient(capi):
    p = PROBLEMS["c1_one_view"]()
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.build()
    ok, dx, info = g.solve_marginal()
    assert ok and info["rank"] < p.cam_cols and np.isfinite(dx).all()


def _gn_marginal_loop(g, max_iterations=20, eps_x=1e-3, eps_j=1e-3):
    """Optimizer2::optimize (Optimizer2.cpp:183-273) with GaussNewtonTrustRegionPolicy over the marginal solver,
    driven through the per-call C-ABI as the C++ host layer does."""
    J = g.eval_cost()
    p_J = J
    dX, dJ, it = eps_x + 1, eps_j + 1, 0
    info = None
    while it < max_iterations and dX > eps_x and abs(dJ) > eps_j:
        g.build()
        ok, dx, info = g.solve_marginal()
        assert ok
        dX = g.apply_update(dx)
        J = g.eval_cost()
        dJ = p_J - J
        p_J = J
        it += 1
    return it, J, info


@pytest.mark.parametrize("name", ["c1", "c2_small", "c6_small"])
def test_gn_marginal_loop_matches_oracle(capi, oracle_mod, name):
    p = PROBLEMS[name]()
    o = oracle_mod.Oracle(p)
    st_o, r_o = o.optimize(p.state_init, policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1e-3,
                           marg=oracle_mod.marg_opts(2 * p.n_corners))
    g = capi.Solver(p)
    g.set_state(p.state_init)
    it, J, info = _gn_marginal_loop(g)
    assert it == r_o["iterations"]
    assert abs(J - r_o["J_final"]) <= 1e-9 * r_o["J_final"]
    assert np.abs(g.get_state() - st_o).max() < 1e-6
    assert info["rank"] == r_o["solve_info"]["rank"]
    ai = g.analyze_marginal()
    assert np.abs(ai["sv"] - r_o["analyze_info"]["sv"]).max() <= 1e-9 * r_o["analyze_info"]["sv"][0]


@pytest.mark.parametrize("name", ["c1", "c2_small"])
def test_device_loop_with_fused_analyze(capi, oracle_mod, name):
    """kb_optimize_marginal (the estimator's device loop) against the oracle's GN + marginal loop, and its fused
    analyzeMarginal (kb_optimize_marginal_analyze) bitwise equal to the separate kb_analyze_marginal call."""
    p = PROBLEMS[name]()
    st_o, r_o = oracle_mod.Oracle(p).optimize(p.state_init, policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1e-3,
                                               marg=oracle_mod.marg_opts(2 * p.n_corners))
    out = []
    for fused in (True, False):
        g = capi.Solver(p)
        g.set_state(p.state_init)
        sol, info, ai = g.optimize_marginal(analyze=fused)
        if not fused:
            ai = g.analyze_marginal()
        out.append((sol, info, ai, g.get_state()))
        g.close()
    (s1, i1, a1, x1), (s2, i2, a2, x2) = out
    assert s1["iterations"] == s2["iterations"] == r_o["iterations"]
    assert np.array_equal(x1, x2)
    assert abs(s1["J_final"] - r_o["J_final"]) <= 1e-9 * r_o["J_final"]
    assert np.abs(x1 - st_o).max() < 1e-6
    assert i1["rank"] == r_o["solve_info"]["rank"]
    assert np.array_equal(a1["sv"], a2["sv"]) and np.array_equal(a1["V"], a2["V"]) and a1["rank"] == a2["rank"]
    assert np.abs(a1["sv"] - r_o["analyze_info"]["sv"]).max() <= 1e-9 * r_o["analyze_info"]["sv"][0]
