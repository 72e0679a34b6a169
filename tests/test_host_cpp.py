"""C++ host layer (kalibr_amd/host/kalibr_backend.*): the aslam_backend-style Optimizer2 / trust-region
policies / LinearSystemSolver mirror over the C-ABI.

CPU: the host Optimizer2 + LM / GN policy driving an oracle-backed LinearSystemSolver must reproduce the
oracle's own Optimizer2 restatement (kbo_optimize) exactly -- pins the host policy code
(Optimizer2.cpp:183-273, TrustRegionPolicy.cpp:29-57, LevenbergMarquardtTrustRegionPolicy.cpp:50-113).
GPU: the host-driven loop over GpuLinearSystemSolver (per-call C-ABI), the device-resident loop
(Optimizer2::optimizeOnDevice -> kb_optimize) and the oracle agree (same iteration counts, state within 1e-6).
"""
import json
import os
import subprocess

import pytest

from kalibr_amd import build as B
from kalibr_amd import synth

from .host_problem import write_problem

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def driver(tmp_path_factory, oracle_mod):
    if not os.path.exists(B.OUT):
        B.build()
    B.build_host()
    out = str(tmp_path_factory.mktemp("host") / "test_host")
    ob = os.path.join(ROOT, "oracle", "_build")
    cmd = ["g++", "-O2", "-std=c++17", "-o", out, os.path.join(ROOT, "tests", "cpp", "test_host.cpp"),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "kalibr_amd", "host"),
           "-I", os.path.join(ROOT, "oracle"),
           "-L", os.path.join(ROOT, "kalibr_amd"), "-lkalibr_backend", "-lkalibr_hip",
           "-L", ob, "-lkb_oracle", "-lpthread",
           "-Wl,-rpath," + os.path.join(ROOT, "kalibr_amd") + ":" + ob]
    subprocess.run(cmd, check=True)
    return out


def run(driver, tmp_path, mode, prob, policy, max_it):
    path = str(tmp_path / "p.bin")
    write_problem(path, prob)
    r = subprocess.run([driver, mode, path, policy, str(max_it)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("policy", ["lm", "gn"])
def test_host_optimizer_matches_oracle_loop(driver, tmp_path, policy):
    p = synth.make_config(1, n_frames=16)
    r = run(driver, tmp_path, "cpu", p, policy, 30)
    assert r["iterations"] == r["ref_iterations"] and r["failed"] == r["ref_failed"], r
    assert r["J_final"] == r["ref_J_final"], r
    assert r["cam_diff"] == 0.0 and r["frame_diff"] == 0.0, r


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,frames,policy", [(1, 20, "lm"), (2, 24, "lm"), (3, 12, "lm"), (2, 24, "gn")])
def test_host_gpu_loops_match_oracle(driver, tmp_path, cfg, frames, policy):
    p = synth.make_config(cfg, n_frames=frames)
    r = run(driver, tmp_path, "gpu", p, policy, 30)
    assert r["host_iterations"] == r["dev_iterations"] == r["ref_iterations"], r
    assert r["host_failed"] == r["dev_failed"] == r["ref_failed"], r
    assert r["trace_len"] >= r["dev_iterations"], r
    for k in ("host_vs_ref_cam", "dev_vs_ref_cam"):
        assert r[k] < 1e-6, r  # north_star tolerance on intrinsics / extrinsics
    for k in ("host_vs_ref_frame", "dev_vs_ref_frame", "host_vs_dev"):
        assert r[k] < 1e-6, r


def run_incr(driver, tmp_path, mode, prob, delta, max_it):
    path = str(tmp_path / "p.bin")
    write_problem(path, prob)
    r = subprocess.run([driver, mode, path, str(delta), str(max_it)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("cfg,frames,delta", [(1, 10, 0.2), (2, 8, 0.2), (2, 8, 5.0)])
def test_incremental_estimator_matches_oracle(driver, tmp_path, cfg, frames, delta):
    """IncrementalEstimator::addBatch (IncrementalEstimator.cpp:337-530): one batch per frame, GN over the
    marginal solver, information-gain / rank acceptance.  The host estimator over an oracle-backed marginal
    solver takes the same decisions as the addBatch rule over the oracle's own loop, bitwise."""
    p = synth.make_config(cfg, n_frames=frames)
    r = run_incr(driver, tmp_path, "incr-cpu", p, delta, 20)
    assert r["accepted"] == r["ref_accepted"] and r["rank"] == r["ref_rank"], r
    assert r["iters"] == r["ref_iters"], r
    assert r["accepted"][0] == 1, r  # the first batch always raises the rank
    if delta > 1.0:
        assert 0 in r["accepted"], r  # a large threshold rejects some batches
    assert r["gain_rel"] == 0.0 and r["cam_diff"] == 0.0 and r["frame_diff"] == 0.0, r


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,frames,delta", [(1, 10, 0.2), (2, 8, 5.0), (1, 120, 0.2), (2, 100, 0.2)])
def test_incremental_estimator_gpu_matches_oracle(driver, tmp_path, cfg, frames, delta):
    """The GPU estimator (GpuMarginalLinearSolver: every accepted batch appended to the device handle in place,
    kb_append_frames; a rejected one dropped, kb_drop_last_frames) takes the oracle-backed estimator's decisions:
    same accept / reject sequence, ranks and GN iteration counts, state within 1e-6 -- up to 120 batches."""
    p = synth.make_config(cfg, n_frames=frames)
    r = run_incr(driver, tmp_path, "incr-gpu", p, delta, 20)
    assert r["accepted"] == r["ref_accepted"] and r["rank"] == r["ref_rank"], r
    assert r["iters"] == r["ref_iters"], r
    assert r["gain_rel"] < 1e-6, r
    assert r["cam_diff"] < 1e-6 and r["frame_diff"] < 1e-6, r


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,frames,policy", [(1, 20, "lm"), (2, 24, "lm")])
def test_host_gpu_pcg_loop(driver, tmp_path, cfg, frames, policy):
    """Optimizer2 over GpuLinearSystemSolver with the block-Jacobi PCG solver: converged tightly it reproduces
    the oracle's (direct-solve) iteration sequence; at LinearSolverPCG's defaults (tol 1e-6) the inexact steps
    still drive LM to the same optimum region without a linear-solver failure."""
    p = synth.make_config(cfg, n_frames=frames)
    r = run(driver, tmp_path, "gpu-pcg", p, policy, 30)
    assert r["name"] == "kalibr_hip_block_jacobi_pcg", r
    assert r["tight_iterations"] == r["ref_iterations"] and r["tight_failed"] == r["ref_failed"], r
    assert r["tight_vs_ref_cam"] < 1e-6 and r["tight_vs_ref_frame"] < 1e-6, r
    assert r["default_lin_fail"] == 0 and r["default_J"] <= 1.05 * r["ref_J"], r


@pytest.mark.parametrize("cfg,frames,policy", [(2, 10, "lm"), (2, 10, "gn"), (3, 6, "lm"), (4, 5, "lm")])
def test_term_solver_over_oracle(driver, tmp_path, cfg, frames, policy):
    """initMatrixStructure(dvs, errors, useDiag) (LinearSystemSolver.hpp:28,73): the problem as DesignVariables and
    ReprojectionError terms in CreateBatchProblem order (CalibrationTools.hpp:460-521), DVs in insertion order,
    in the IncrementalEstimator's group order (target poses and landmarks first, the calibration group last,
    IncrementalEstimator.cpp:550-565) and shuffled.  Packing gives back the problem; every DV's block of dx / rhs in
    the caller's column order equals the canonical solve's; Optimizer2 through the terms ends at the canonical
    run's state -- bitwise when the frames keep their order (the inner solver sees the same canonical problem),
    to rounding when the shuffle reorders them (frame blocks summed in another order)."""
    p = synth.make_config(cfg, n_frames=frames, p_view=0.8)
    r = run(driver, tmp_path, "terms-cpu", p, policy, 20)
    assert r["pack_diff"] == 0.0 and r["cost_rel"] == 0.0, r
    assert r["dx_rel"] == 0.0 and r["rhs_rel"] == 0.0, r
    assert r["state_diff"] == 0.0, r  # caller order = canonical order: the same run bit for bit
    # frames-first caller order: the device run is the canonical one, but the LM policy's host-side rho sum runs in
    # the caller's column order (last-bit differences of lambda)
    assert r["perm_state_diff"] < 1e-10, r
    assert r["shuf_cost_rel"] < 1e-12 and r["shuf_rhs_rel"] < 1e-10 and r["shuf_dx_rel"] < 1e-7, r
    assert r["shuf_state_diff"] < 1e-8, r
    assert r["iterations"] == [r["ref_iterations"]] * 3, r
    assert r["frames_reordered"] > 0, r  # the shuffle exercised the frame permutation


@pytest.mark.gpu
def test_term_solver_over_gpu(driver, tmp_path):
    p = synth.make_config(4, n_frames=12, p_view=0.8)
    r = run(driver, tmp_path, "terms-gpu", p, "lm", 20)
    assert r["pack_diff"] == 0.0 and r["cost_rel"] == 0.0, r
    assert r["dx_rel"] == 0.0 and r["rhs_rel"] == 0.0, r
    assert r["state_diff"] == 0.0, r  # caller order = canonical order: the same run bit for bit
    # frames-first caller order: the device run is the canonical one, but the LM policy's host-side rho sum runs in
    # the caller's column order (last-bit differences of lambda)
    assert r["perm_state_diff"] < 1e-10, r
    assert r["shuf_cost_rel"] < 1e-12 and r["shuf_rhs_rel"] < 1e-10 and r["shuf_dx_rel"] < 1e-7, r
    assert r["shuf_state_diff"] < 1e-8, r
    assert r["iterations"] == [r["ref_iterations"]] * 3, r
