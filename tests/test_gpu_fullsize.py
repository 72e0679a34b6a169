"""Full-size end-to-end parity: the device-resident optimizer (through the C-ABI) against the CPU oracle on the
BASELINE.json problems at their full sizes, with Kalibr2's optimizer settings.

  LM  : CalibrationTools.hpp:57-66 defaults (lambda0 = 10, epsX = 1e-3, epsJ = 1, maxIterations = 200)
  GN  : GaussNewtonTrustRegionPolicy, maxIterations = 20 (IncrementalEstimator's batch setting)

Bar (north_star: intrinsics / extrinsics within 1e-6 of the reference CPU path):
  identical iterations and failed_iterations, identical accept / revert trace,
  J_final within 1e-9 relative, intrinsics and baselines within 1e-6 absolute, every frame pose within 1e-6.

synth.make_config numbering is SURVEY.md's (1-based): make_config(2) = configs[1] (2-cam, 500 frames),
make_config(3) = configs[2] (2 omni-radtan + 2 EUCM, 1000 frames), make_config(4) = configs[3] (8-cam, 2000 frames).
"""
import time

import numpy as np
import pytest

from kalibr_amd import synth

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16
_cache = {}


def _problem(idx):
    if idx not in _cache:
        _cache[idx] = synth.make_config(idx)
    return _cache[idx]


def _intr_ext(p, st):
    """intrinsics (per camera, padded slots) and baselines: the calibration result Kalibr2 exports"""
    n_cam = p.n_cams
    off_frame = synth.state_size(n_cam, 0)
    return st[:off_frame]


# configs[2] runs LM only: its camera block (omni xi / EUCM alpha-beta against the focal lengths) is numerically
# rank-deficient at lambda = 0 (cond ~ 6e16, test_gpu_parity.py::test_solve), so undamped Gauss-Newton steps are
# linear-solver failures for any two solvers and the failure trajectory is not a reproducible quantity (measured:
# 20 failed iterations on both, different successful counts)
CASES = [(2, "lm"), (2, "gn"), (3, "lm"), (4, "lm"), (4, "gn")]


@pytest.mark.parametrize("idx,policy", CASES, ids=[f"configs[{i - 1}]-{p}" for i, p in CASES])
def test_full_size_optimize_parity(oracle_mod, idx, policy):
    from kalibr_amd import capi
    p = _problem(idx)
    kw = dict(lambda0=10.0, max_iterations=200, eps_x=1e-3, eps_j=1.0) if policy == "lm" else \
        dict(max_iterations=20, eps_x=1e-3, eps_j=1.0)
    o = oracle_mod.Oracle(p)
    t0 = time.time()
    st_o, r_o = o.optimize(p.state_init, policy=policy, nthreads=ORACLE_THREADS, **kw)
    t1 = time.time()
    g = capi.Solver(p)
    g.set_state(p.state_init)
    r_g = g.optimize(policy=policy, **kw)
    t2 = time.time()
    st_g = g.get_state()
    g.close()
    print(f"configs[{idx - 1}] {policy}: corners={p.n_corners} iterations gpu={r_g['iterations']} "
          f"oracle={r_o['iterations']} failed={r_g['failed_iterations']}/{r_o['failed_iterations']} "
          f"J_final={r_g['J_final']:.12g}/{r_o['J_final']:.12g} oracle {t1 - t0:.1f}s gpu {t2 - t1:.2f}s")
    assert r_g["iterations"] == r_o["iterations"]
    assert r_g["failed_iterations"] == r_o["failed_iterations"]
    assert r_g["linear_solver_failure"] == r_o["linear_solver_failure"]
    assert np.array_equal(r_g["trace"][:, 3], r_o["trace"][:, 3])  # same accept / revert decisions
    assert abs(r_g["J_final"] - r_o["J_final"]) <= 1e-9 * r_o["J_final"]
    d_cal = np.abs(_intr_ext(p, st_g) - _intr_ext(p, st_o)).max()
    d_all = np.abs(st_g - st_o).max()
    print(f"  max|intrinsics/baselines - oracle| = {d_cal:.3e}, max|state - oracle| = {d_all:.3e}")
    assert d_cal < 1e-6
    assert d_all < 1e-6
    # the run calibrated: the camera block moved toward the truth
    assert np.abs(_intr_ext(p, st_g) - _intr_ext(p, p.state_truth)).max() < \
        np.abs(_intr_ext(p, p.state_init) - _intr_ext(p, p.state_truth)).max()
