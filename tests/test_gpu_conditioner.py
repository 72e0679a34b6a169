"""LinearSystemSolver::setConditioner with a non-constant diagonal (LinearSystemSolver.cpp:98-102) on the device:
kb_set_conditioner's squares enter the frame blocks (k_schur) and the camera block (k_solve) of kb_solve; the
dx must solve (J^T J + diag(d^2)) dx = rhs, checked against a dense numpy solve of the arrow system."""
import numpy as np
import pytest

from kalibr_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    from kalibr_amd import capi as K
    return K


def _dense(blocks, d2):
    C, F = blocks["Hcc"].shape[0], blocks["Hff"].shape[0]
    n = C + 6 * F
    H = np.zeros((n, n))
    H[:C, :C] = blocks["Hcc"]
    for f in range(F):
        o = C + 6 * f
        H[o:o + 6, o:o + 6] = blocks["Hff"][f]
        H[o:o + 6, :C] = blocks["Hfc"][f]
        H[:C, o:o + 6] = blocks["Hfc"][f].T
    return H + np.diag(d2), np.concatenate([blocks["gc"], blocks["gf"].ravel()])


@pytest.mark.parametrize("cfg,frames", [(2, 30), (4, 16), (3, 12)])
def test_diagonal_conditioner_matches_dense_solve(capi, cfg, frames):
    p = synth.make_config(cfg, n_frames=frames, p_view=0.8)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.build()
    rng = np.random.default_rng(7)
    diag = rng.uniform(0.5, 20.0, size=g.ncols)
    g.set_conditioner(diag)
    ok, dx = g.solve()
    assert ok
    H, b = _dense(g.normal_blocks(), diag * diag)
    ref = np.linalg.solve(H, b)
    err = np.abs(dx - ref).max() / np.abs(ref).max()
    assert err < 1e-8, err
    # a constant conditioner afterwards is the constant path again
    g.set_constant_conditioner(10.0)
    ok, dx2 = g.solve()
    H2, _ = _dense(g.normal_blocks(), np.full(g.ncols, 100.0))
    assert ok and np.abs(dx2 - np.linalg.solve(H2, b)).max() / np.abs(dx2).max() < 1e-8
