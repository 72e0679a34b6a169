"""Edge cases of the device path through the C-ABI: malformed inputs fail loudly with a message (host-side
validation before any kernel sees them, kb_upload_observations / kb_create), the CHOLMOD failure semantics of
kb_solve (ok = 0 on a non-positive-definite system, SparseCholeskyLinearSystemSolver.cpp:69-72), minimal views,
and full-size parity at the largest configuration (configs[3]: 8 cameras, 2000 frames, C = 106).
"""
import dataclasses

import numpy as np
import pytest

from kalibr_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    from kalibr_amd import capi as K
    return K


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-300, np.abs(np.asarray(b)).max()))


def _truncate_view(p, v, keep):
    """problem with view v cut to its first `keep` corners"""
    o = p.view_offset
    idx = np.concatenate([np.arange(o[u], o[u + 1] if u != v else o[u] + keep) for u in range(p.n_views)])
    counts = np.array([(o[u + 1] - o[u]) if u != v else keep for u in range(p.n_views)])
    return dataclasses.replace(p, corner_id=p.corner_id[idx].astype(np.int32), y=p.y[idx].copy(),
                               view_offset=np.concatenate([[0], np.cumsum(counts)]).astype(np.int32))


BAD_INPUTS = {
    "unsorted_views": (lambda p: dataclasses.replace(p, view_frame=p.view_frame[::-1].copy(),
                                                     view_cam=p.view_cam[::-1].copy()), "sorted by frame"),
    "duplicate_view": (lambda p: dataclasses.replace(p, view_cam=np.zeros_like(p.view_cam)), "two views"),
    "corner_out_of_range": (lambda p: dataclasses.replace(p, corner_id=np.where(
        np.arange(p.n_corners) == 5, 500, p.corner_id).astype(np.int32)), "corner_id out of range"),
    "offsets_mismatch": (lambda p: dataclasses.replace(p, view_offset=np.concatenate(
        [p.view_offset[:-1], [p.view_offset[-1] - 1]]).astype(np.int32)), "view_offsets"),
    "camera_out_of_range": (lambda p: dataclasses.replace(p, view_cam=np.where(
        np.arange(p.n_views) == p.n_views - 1, 7, p.view_cam).astype(np.int32)), "out of range"),
}


@pytest.mark.parametrize("name", list(BAD_INPUTS))
def test_malformed_observations_are_rejected(capi, name):
    p = synth.make_config(2, n_frames=6)
    mutate, msg = BAD_INPUTS[name]
    with pytest.raises(capi.KbError, match=msg):
        capi.Solver(mutate(p))


def test_layout_limits_are_rejected(capi):
    with pytest.raises(capi.KbError, match="n_cams"):
        capi.Solver(synth.make_problem([synth.PINHOLE_RADTAN] * 17, 2, seed=1))
    # 12 pinhole-radtan cameras: C = 12 * 8 + 66 = 162 > 111
    with pytest.raises(capi.KbError, match="C > 111"):
        capi.Solver(synth.make_problem([synth.PINHOLE_RADTAN] * 12, 2, seed=1))


def test_second_upload_is_rejected(capi):
    p = synth.make_config(1, n_frames=4)
    g = capi.Solver(p)
    y = np.ascontiguousarray(p.y)
    cid = np.ascontiguousarray(p.corner_id, dtype=np.uint16)
    vo = np.ascontiguousarray(p.view_offset, dtype=np.uint32)
    vf = np.ascontiguousarray(p.view_frame, dtype=np.uint32)
    vc = np.ascontiguousarray(p.view_cam, dtype=np.uint8)
    rc = capi.lib().kb_upload_observations(g.h, p.n_views, p.n_corners, capi._d(y), cid.ctypes.data, vo.ctypes.data,
                                           vf.ctypes.data, vc.ctypes.data)
    assert rc < 0 and b"already uploaded" in capi.lib().kb_last_error()


def test_degenerate_frame_is_not_positive_definite(capi, oracle_mod):
    """A frame whose only view has no seen corner: its 6 x 6 block is zero.  Without damping both CHOLMOD (the
    reference) and the Schur solve report failure; with the LM conditioner the system is solvable again."""
    p = _truncate_view(synth.make_config(1, n_frames=6), 3, 0)
    o = oracle_mod.Oracle(p)
    A = o.arrow(p.state_init)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.build()
    g.set_constant_conditioner(0.0)
    ok, _ = g.solve()
    ok_o, _ = o.solve(A, 0.0, dense=True)
    assert not ok and not ok_o
    g.set_constant_conditioner(10.0)
    ok, dx = g.solve()
    ok_o, dx_o = o.solve(A, 10.0)
    assert ok and ok_o and _rel(dx, dx_o) < 1e-8


def test_minimal_views(capi, oracle_mod):
    """Views of one corner next to full views: cost, blocks and the damped solve match the oracle."""
    p = synth.make_config(2, n_frames=8)
    for v in (1, 4, 9):
        p = _truncate_view(p, v, 1)
    o = oracle_mod.Oracle(p)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    J = g.eval_cost()
    assert abs(J - o.cost(p.state_init)) <= 1e-12 * J
    A = o.arrow(p.state_init)
    g.build()
    g.set_constant_conditioner(1.0)
    ok, dx = g.solve()
    ok_o, dx_o = o.solve(A, 1.0)
    assert ok and ok_o and _rel(dx, dx_o) < 1e-8


def test_full_size_rig8_parity(capi, oracle_mod):
    """configs[3] at full size on one GPU (1.9 M corners, C = 106: the blocked camera LDL^T): cost, rhs and the
    damped solve against the oracle."""
    p = synth.make_config(4)
    o = oracle_mod.Oracle(p)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    J = g.eval_cost()
    J_o = o.cost(p.state_init, nthreads=16)
    assert abs(J - J_o) <= 1e-11 * J_o
    g.build()
    A = o.arrow(p.state_init, nthreads=16)
    assert _rel(g.rhs(), A["rhs"]) < 1e-10
    g.set_constant_conditioner(10.0)
    ok, dx = g.solve()
    ok_o, dx_o = o.solve(A, 10.0, nthreads=16)
    assert ok and ok_o and _rel(dx, dx_o) < 1e-8


def test_stale_preparation_and_system_are_refused(capi):
    """kb_gn_launch refuses a preparation that a later call voided (state set, per-call solve, another loop), and the
    per-call system accessors (kb_rhs_jtj_rhs, kb_get_normal_blocks) refuse to read blocks a device-resident loop
    overwrote or skipped; a fresh kb_build makes them valid again."""
    p = synth.make_config(2, n_frames=16)
    g = capi.Solver(p)
    g.set_state(p.state_init)
    g.gn_prepare(3)
    g.set_state(p.state_init)  # voids the prepared loop start
    with pytest.raises(capi.KbError, match="not prepared"):
        g.gn_launch(3)
    g.gn_prepare(3)
    g.build()  # a per-call entry point voids it too
    with pytest.raises(capi.KbError, match="not prepared"):
        g.gn_launch(3)
    g.gn_prepare(3)
    g.gn_launch(3)  # prepared and untouched: runs
    with pytest.raises(capi.KbError, match="no intact system"):
        g.rhs_jtj_rhs()
    with pytest.raises(capi.KbError, match="no intact system"):
        g.normal_blocks()
    g.build()
    assert np.isfinite(g.rhs_jtj_rhs())
    g.optimize(policy="lm", max_iterations=3)
    with pytest.raises(capi.KbError, match="no intact system"):
        g.rhs_jtj_rhs()
