"""Sharded HIP path with several ranks on one GPU (kb_comm_init_local).

The frames of one problem are split over 2-3 handles of uneven size; the handles form an in-process group whose
collectives (all-reduce of the stage-1 camera-block rows, all-gather of the per-frame step rows and of the
cost / step statistics) are device copies summed in rank order instead of RCCL.  Everything else -- the F_max
padding of the step rows, the per-rank max|dx_f| columns (Wtot = Wp + nranks), the rank-order reductions in
k_post / k_red_gather -- is the code the multi-GPU run executes.  Each handle is driven from its own thread, as
each rank drives its own in a multi-process run.

Bar: the sharded run takes the same accept/revert decisions as the unsharded handle (identical iteration
counts and trace flags), J within 1e-12 and the state within 1e-9 (the column sums group the frames
differently, so the last bits may differ), and it matches the CPU oracle within the 1e-6 state bar of
test_gpu_parity.py.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from kalibr_amd import synth

pytestmark = pytest.mark.gpu

POSE = 7


@pytest.fixture(scope="module")
def capi():
    from kalibr_amd import capi as K
    return K


def _shards(capi, p, cuts):
    bounds = [0] + list(cuts) + [p.n_frames]
    subs = [p.frame_slice(a, b) for a, b in zip(bounds[:-1], bounds[1:])]
    solvers = [capi.Solver(s) for s in subs]
    capi.comm_init_local(solvers)
    for s, sub in zip(solvers, subs):
        s.set_state(sub.state_init)
    return solvers


def _run_all(solvers, fn):
    with ThreadPoolExecutor(max_workers=len(solvers)) as ex:
        futs = [ex.submit(fn, s) for s in solvers]
        return [f.result(timeout=300) for f in futs]


def _joined_state(p, states):
    so = p.n_cams * synth.MAX_INTR + POSE * (p.n_cams - 1)
    for s in states[1:]:  # every rank holds the same camera block
        assert np.array_equal(s[:so], states[0][:so])
    return np.concatenate([states[0][:so]] + [s[so:] for s in states])


CASES = {
    # C = 22: the 8 stage-1 rows are all-reduced and summed by k_solve
    "c2_2ranks": (lambda: synth.make_config(2, n_frames=12), [7]),
    # C = 106: stage-1 rows all-reduced, finished by k_colimg for the tiled camera solve; ragged views
    "c4_2ranks": (lambda: synth.make_config(4, n_frames=24, p_view=0.7), [13]),
    "c4_3ranks": (lambda: synth.make_config(4, n_frames=24, p_view=0.7), [5, 16]),
    "c3_2ranks": (lambda: synth.make_config(3, n_frames=20), [9]),
}


# undamped GN diverges on the 20-frame omni-radtan + EUCM rig (the oracle too: state ~1e10 after one step, so
# rounding decides the trajectory); that rig runs LM only
RUNS = [(n, "lm") for n in CASES] + [(n, "gn") for n in CASES if n != "c3_2ranks"]


@pytest.mark.parametrize("name,policy", RUNS)
def test_sharded_optimize_matches_unsharded(capi, oracle_mod, name, policy):
    mk, cuts = CASES[name]
    p = mk()
    kw = dict(policy=policy, lambda0=10.0, max_iterations=200 if policy == "lm" else 20, eps_x=1e-3, eps_j=1.0)
    ref = capi.Solver(p)
    ref.set_state(p.state_init)
    r0 = ref.optimize(**kw)
    s0 = ref.get_state()
    solvers = _shards(capi, p, cuts)
    res = _run_all(solvers, lambda s: s.optimize(**kw))
    st = _joined_state(p, [s.get_state() for s in solvers])
    st_o, r_o = oracle_mod.Oracle(p).optimize(p.state_init, **kw)
    print(f"{name} {policy}: J_final unsharded {r0['J_final']!r} sharded {[r['J_final'] for r in res]} oracle "
          f"{r_o['J_final']!r}; iterations {r0['iterations']} / {[r['iterations'] for r in res]} / {r_o['iterations']}; "
          f"max|unsharded - oracle| {np.abs(s0 - st_o).max():.3e} max|sharded - oracle| {np.abs(st - st_o).max():.3e}")
    for r in res:
        assert r["iterations"] == r0["iterations"] and r["failed_iterations"] == r0["failed_iterations"]
        assert np.array_equal(r["trace"][:, 3], r0["trace"][:, 3])  # accept / revert sequence
        assert abs(r["J_final"] - r0["J_final"]) <= 1e-12 * r0["J_final"]
        assert r["J_final"] == res[0]["J_final"]  # every rank holds the same reduced numbers
        # max|dx| (the eps_x test): every rank's frame-step maximum reaches the reduction (GN fused passes: one image
        # slot per rank)
        assert np.allclose(r["trace"][:, 2], r0["trace"][:, 2], rtol=1e-9, atol=0.0)
    d = float(np.abs(st - s0).max())
    assert d < 1e-9, d
    assert res[0]["iterations"] == r_o["iterations"]
    assert float(np.abs(st - st_o).max()) < 1e-6
    print(f"{name} {policy}: ranks={len(solvers)} iterations={r0['iterations']} max|sharded - unsharded|={d:.2e}")


@pytest.mark.parametrize("name", ["c2_2ranks", "c4_3ranks"])
def test_sharded_fixed_gn_passes_and_per_call_api(capi, name):
    """kb_run_gn_iterations (the bench loop: GN fused passes, per-rank max|dx_f| columns, the last step's
    back-substitution in finish_pass) and the per-call evaluateError / buildSystem / solveSystem surface."""
    mk, cuts = CASES[name]
    p = mk()
    ref = capi.Solver(p)
    ref.set_state(p.state_init)
    ref.run_gn(6)
    s0 = ref.get_state()
    solvers = _shards(capi, p, cuts)
    _run_all(solvers, lambda s: s.run_gn(6))
    st = _joined_state(p, [s.get_state() for s in solvers])
    assert float(np.abs(st - s0).max()) < 1e-9
    # per-call surface at the initial state: cost, camera-block solve
    for s, sub in zip(solvers, [p.frame_slice(a, b) for a, b in zip([0] + cuts, cuts + [p.n_frames])]):
        s.set_state(sub.state_init)
    ref.set_state(p.state_init)
    J = _run_all(solvers, lambda s: s.eval_cost())
    J0 = ref.eval_cost()
    assert all(j == J[0] for j in J) and abs(J[0] - J0) <= 1e-12 * J0

    def solve(s):
        s.build()
        s.set_constant_conditioner(10.0)
        return s.solve()

    out = _run_all(solvers, solve)
    ref.build()
    ref.set_constant_conditioner(10.0)
    ok0, dx0 = ref.solve()
    C = ref.C
    assert ok0 and all(o[0] for o in out)
    dxc = dx0[:C]
    for ok, dx in out:
        assert np.array_equal(dx[:C], out[0][1][:C])
        assert float(np.abs(dx[:C] - dxc).max()) <= 1e-8 * float(np.abs(dxc).max())
    dxf = np.concatenate([o[1][C:] for o in out])
    assert float(np.abs(dxf - dx0[C:]).max()) <= 1e-8 * float(np.abs(dx0).max())


@pytest.mark.parametrize("name", ["c2_2ranks", "c4_3ranks"])
def test_sharded_pcg_schur_matches_unsharded(capi, name):
    """KB_SOLVER_PCG_SCHUR on a sharded handle: every rank runs the same block-Jacobi PCG on the all-reduced camera
    Schur complement, so all ranks hold bitwise-identical camera steps, iteration counts and _residual; the frame
    steps are each rank's own back-substitution.  Bars: converged tightly, the unsharded handle's PCG-on-S step (the
    column sums group the frames differently, so the CG iterates differ in the last bits; at the reference tolerance CG
    amplifies that, so the defaults are checked for rank agreement and the _residual carry-over only)."""
    mk, cuts = CASES[name]
    p = mk()
    tight = dict(tolerance=1e-28, max_iterations=4000, absolute_tolerance=False)
    ref = capi.Solver(p)
    ref.set_state(p.state_init)
    ref.set_linear_solver("pcg_schur", **tight)
    ref.build()
    ref.set_constant_conditioner(10.0)
    ok0, dx0 = ref.solve()
    solvers = _shards(capi, p, cuts)

    def solve(s):
        s.build()
        s.set_constant_conditioner(10.0)
        s.set_linear_solver("pcg_schur", **tight)
        rt = s.solve()
        s.set_linear_solver("pcg_schur")  # LinearSolverPCG defaults (absolute tolerance), _residual reset
        r1 = s.solve()
        a = s.pcg_info()
        r2 = s.solve()  # absolute tolerance: d0 = max(tol dn0, the previous solve's _residual)
        return rt, r1, a, r2, s.pcg_info()

    out = _run_all(solvers, solve)
    C = ref.C
    assert ok0
    for (okt, dxt), (ok1, dx1), inf, (ok2, dx2), inf2 in out:
        assert okt and ok1 and ok2
        assert np.array_equal(dxt[:C], out[0][0][1][:C]) and np.array_equal(dx1[:C], out[0][1][1][:C])
        assert inf == out[0][2] and inf2 == out[0][4]  # every rank: the same PCG run
        assert float(np.abs(dxt[:C] - dx0[:C]).max()) <= 1e-8 * float(np.abs(dx0[:C]).max())
        assert inf2["d0"] >= inf["residual"] * (1 - 1e-12)  # LinearSolverPCG: d0 = max(tol dn, _residual)
    dxf = np.concatenate([o[0][1][C:] for o in out])
    assert float(np.abs(dxf - dx0[C:]).max()) <= 1e-8 * float(np.abs(dx0).max())


def test_local_group_rejects_bad_lists(capi):
    p = synth.make_config(2, n_frames=6)
    a = capi.Solver(p)
    with pytest.raises(capi.KbError):
        capi.comm_init_local([a, a])
    b = capi.Solver(synth.make_config(4, n_frames=6))
    with pytest.raises(capi.KbError):
        capi.comm_init_local([a, b])


def test_configs3_eight_shards_on_one_gpu(capi):
    """The driver's N=8 strong-scaling layout of the north-star problem (configs[3], 2000 frames -> 8 x 250), as 8
    in-process ranks on one GPU: fixed GN passes match the unsharded handle."""
    p = synth.make_config(4)
    ref = capi.Solver(p)
    ref.set_state(p.state_init)
    ref.run_gn(4)
    s0 = ref.get_state()
    ref.close()
    solvers = _shards(capi, p, [250 * r for r in range(1, 8)])
    _run_all(solvers, lambda s: s.run_gn(4))
    st = _joined_state(p, [s.get_state() for s in solvers])
    d = float(np.abs(st - s0).max())
    print(f"configs[3] 8 in-process shards: max|sharded - unsharded| after 4 GN passes = {d:.2e}")
    assert d < 1e-9


@pytest.mark.parametrize("policy", ["lm", "gn"])
def test_configs3_eight_shards_full_optimize_against_oracle(capi, oracle_mod, policy):
    """The N=8 layout (configs[3], 8 x 250 frames, in-process ranks) through a whole Optimizer2 run with Kalibr2's
    settings, against the CPU oracle on the unsharded problem: the same iteration counts and accept / revert trace,
    J within 1e-9, every intrinsic, baseline and frame pose within 1e-6 (north_star)"""
    p = synth.make_config(4)
    kw = dict(policy=policy, lambda0=10.0, max_iterations=200 if policy == "lm" else 20, eps_x=1e-3, eps_j=1.0)
    solvers = _shards(capi, p, [250 * r for r in range(1, 8)])
    res = _run_all(solvers, lambda s: s.optimize(**kw))
    st = _joined_state(p, [s.get_state() for s in solvers])
    for s in solvers:
        s.close()
    st_o, r_o = oracle_mod.Oracle(p).optimize(p.state_init, nthreads=16, **kw)
    print(f"configs[3] 8 shards {policy}: iterations {[r['iterations'] for r in res][0]} / oracle {r_o['iterations']}, "
          f"J {res[0]['J_final']!r} / {r_o['J_final']!r}, max|state - oracle| {np.abs(st - st_o).max():.3e}")
    for r in res:
        assert r["iterations"] == r_o["iterations"] and r["failed_iterations"] == r_o["failed_iterations"]
        assert np.array_equal(r["trace"][:, 3], r_o["trace"][:, 3])
        assert abs(r["J_final"] - r_o["J_final"]) <= 1e-9 * r_o["J_final"]
    assert float(np.abs(st - st_o).max()) < 1e-6


@pytest.mark.parametrize("name", ["c4_2ranks"])
def test_direct_allreduce_bitwise_equals_copies(capi, name, monkeypatch):
    """k_xar, the direct all-reduce of the sharded camera-block image (C > 64): the group's members read each other's
    partial images and sum them in rank order, as the in-process copies do -- bitwise-identical states and traces.
    With KB_DIRECT_AR=0 the group keeps the copies.  The direct path needs one member per device: on this one-GPU box
    the default keeps the copies, and KB_DIRECT_AR=force (tests only) lets a two-member group share the device."""
    mk, cuts = CASES[name]
    p = mk()
    out = {}
    monkeypatch.setenv("KB_DIRECT_AR", "1")  # the product rule: members on one device keep the copies
    for cc in ([13], [5, 16]):
        shared = _shards(capi, p, cc)
        assert not any(s.comm_direct() for s in shared)
        for s in shared:
            s.close()
    for mode in ("0", "force"):
        monkeypatch.setenv("KB_DIRECT_AR", mode)
        solvers = _shards(capi, p, cuts)
        assert all(s.comm_direct() == (mode == "force") for s in solvers)
        if mode == "force":  # three members on the one device keep the copies even when forced
            three = _shards(capi, p, [5, 16])
            assert not any(s.comm_direct() for s in three)
            for s in three:
                s.close()
        _run_all(solvers, lambda s: s.run_gn(6))
        gn = [s.get_state() for s in solvers]
        subs = [p.frame_slice(a, b) for a, b in zip([0] + cuts, cuts + [p.n_frames])]
        for s, sub in zip(solvers, subs):
            s.set_state(sub.state_init)
        res = _run_all(solvers, lambda s: s.optimize(policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1.0))
        out[mode] = (gn, [s.get_state() for s in solvers], res)
        for s in solvers:
            s.close()
    for a, b in zip(out["0"][0] + out["0"][1], out["force"][0] + out["force"][1]):
        assert np.array_equal(a, b)
    for r0, r1 in zip(out["0"][2], out["force"][2]):
        assert r0["iterations"] == r1["iterations"] and r0["J_final"] == r1["J_final"]
        assert np.array_equal(r0["trace"], r1["trace"])


def test_direct_allreduce_peer_drop_then_retry(capi, monkeypatch):
    """A rank whose peer stops taking part in the direct all-reduce: its k_xar gives up after the wait bound
    (KB_XAR_TIMEOUT_MS), ends the enqueued passes (ctrl done) and the call fails; at the next loop start the ranks
    agree to leave the direct path, and the retried optimize runs over the copies -- bitwise equal to a group that
    used the copies from the start."""
    mk, cuts = CASES["c4_2ranks"]
    p = mk()
    subs = [p.frame_slice(a, b) for a, b in zip([0] + cuts, cuts + [p.n_frames])]
    kw = dict(policy="gn", max_iterations=20, eps_x=1e-3, eps_j=1.0)
    monkeypatch.setenv("KB_DIRECT_AR", "0")
    ref = _shards(capi, p, cuts)
    r_ref = _run_all(ref, lambda s: s.optimize(**kw))
    st_ref = [s.get_state() for s in ref]
    for s in ref:
        s.close()
    monkeypatch.setenv("KB_DIRECT_AR", "force")
    monkeypatch.setenv("KB_XAR_TIMEOUT_MS", "300")
    solvers = _shards(capi, p, cuts)
    assert all(s.comm_direct() for s in solvers)

    def uneven(s):  # rank 1 stops after 2 passes: rank 0's third k_xar waits in vain
        try:
            s.run_gn(5 if s is solvers[0] else 2)
            return None
        except RuntimeError as e:
            return str(e)

    errs = _run_all(solvers, uneven)
    assert errs[0] is not None and "k_xar" in errs[0], errs
    assert errs[1] is None, errs
    assert all(s.comm_direct() for s in solvers)  # still installed: the agreement is at the next loop start
    for s, sub in zip(solvers, subs):
        s.set_state(sub.state_init)
    res = _run_all(solvers, lambda s: s.optimize(**kw))
    assert not any(s.comm_direct() for s in solvers)
    for a, b in zip(st_ref, [s.get_state() for s in solvers]):
        assert np.array_equal(a, b)
    for r0, r1 in zip(r_ref, res):
        assert r0["iterations"] == r1["iterations"] and r0["J_final"] == r1["J_final"]
    for s in solvers:
        s.close()


@pytest.mark.parametrize("name", ["c2_2ranks", "c4_3ranks"])
def test_sharded_reprojection_error_stats(capi, name):
    """kb_reprojection_error_stats on a sharded group: every rank returns the statistics over ALL ranks' terms (the
    per-camera sums all-reduced between the two passes), equal to the unsharded handle's to rounding"""
    mk, cuts = CASES[name]
    p = mk()
    ref = capi.Solver(p)
    ref.set_state(p.state_init)
    want = ref.reprojection_error_stats()
    solvers = _shards(capi, p, cuts)
    got = _run_all(solvers, lambda s: s.reprojection_error_stats())
    for g in got:
        assert np.array_equal(g[:, 0], want[:, 0])
        assert np.abs(g[:, 1:] - want[:, 1:]).max() <= 1e-12 * np.abs(want[:, 1:]).max()
    for s in solvers + [ref]:
        s.close()
