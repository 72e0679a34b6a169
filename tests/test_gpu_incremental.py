"""Frames appended to / dropped from an uploaded handle in place (kb_append_frames / kb_drop_last_frames: the device
side of IncrementalEstimator::addBatch, IncrementalEstimator.cpp:343-373, 517-527).

Bar: a handle grown frame by frame (across several capacity doublings, and across a change of the build kernel's
frames per block) holds exactly the problem a fresh handle of the same frames holds: the normal-equation blocks, the
cost and fixed GN passes are bitwise identical (same frames, same blocks, same reduction order), and so after dropping
frames and appending them again.
"""
import numpy as np
import pytest

from kalibr_amd import synth

pytestmark = pytest.mark.gpu

POSE = 7


@pytest.fixture(scope="module")
def capi():
    from kalibr_amd import capi as K
    return K


def _fresh(capi, p, f1):
    sub = p.frame_slice(0, f1)
    g = capi.Solver(sub)
    g.set_state(sub.state_init)
    return g, sub


def _same(a, b, name):
    a.build()
    b.build()
    A, B = a.normal_blocks(), b.normal_blocks()
    for k in ("Hff", "Hfc", "gf", "Hcc", "gc"):
        assert np.array_equal(A[k], B[k]), (name, k)
    assert A["cost"] == B["cost"], name
    assert np.array_equal(a.get_state(), b.get_state()), name


@pytest.mark.parametrize("cfg,nf,first,chunk,pv", [(2, 40, 3, 9, 1.0), (4, 300, 100, 90, 0.8)])
def test_append_and_drop_match_fresh_handles(capi, cfg, nf, first, chunk, pv):
    p = synth.make_config(cfg, n_frames=nf, p_view=pv)
    g, _ = _fresh(capi, p, first)
    f = first
    # one block of frames, then single frames (capacity doublings on the way)
    g.append_frames(p.frame_slice(f, f + chunk))
    f += chunk
    while f < nf - 5:
        g.append_frames(p.frame_slice(f, f + 1))
        f += 1
    ref, sub = _fresh(capi, p, f)
    assert g.S == ref.S and g.ncols == ref.ncols
    _same(g, ref, "grown")
    # GN passes from the same state: bitwise the same trajectory
    g.run_gn(3)
    ref.run_gn(3)
    assert np.array_equal(g.get_state(), ref.get_state())
    # drop the last 4 frames, restore the state of the smaller problem, compare; then append them again
    g.drop_last_frames(4)
    small, ssub = _fresh(capi, p, f - 4)
    g.set_state(ssub.state_init)
    _same(g, small, "dropped")
    g.append_frames(p.frame_slice(f - 4, nf))
    full, fsub = _fresh(capi, p, nf)
    g.set_state(fsub.state_init)
    _same(g, full, "re-appended")
    g.run_gn(2)
    full.run_gn(2)
    assert np.array_equal(g.get_state(), full.get_state())


def test_drop_on_fresh_handle_across_frames_per_block(capi):
    """a freshly created handle dropped across a change of the build's frames per block: configs[3]'s rig at 300 frames
    runs 150 build blocks of 2 frames, at 256 frames 256 blocks of one, so the handle needs more partial rows than it
    was created with (they are regrown) and matches a fresh 256-frame handle bitwise"""
    p = synth.make_config(4, n_frames=300)
    g, _ = _fresh(capi, p, 300)
    g.drop_last_frames(44)
    ref, sub = _fresh(capi, p, 256)
    g.set_state(sub.state_init)
    _same(g, ref, "dropped 300 -> 256")
    g.run_gn(2)
    ref.run_gn(2)
    assert np.array_equal(g.get_state(), ref.get_state())


def test_append_validation(capi):
    p = synth.make_config(2, n_frames=8)
    g, _ = _fresh(capi, p, 4)
    sub = p.frame_slice(4, 6)
    bad = synth.Problem(cam_model=sub.cam_model, target=sub.target, view_frame=sub.view_frame[::-1].copy(),
                        view_cam=sub.view_cam[::-1].copy(), view_offset=sub.view_offset, corner_id=sub.corner_id,
                        y=sub.y, state_truth=sub.state_truth, state_init=sub.state_init)
    with pytest.raises(capi.KbError, match="sorted by frame"):
        g.append_frames(bad)
    with pytest.raises(capi.KbError, match="at least one frame"):
        g.drop_last_frames(4)
    g.append_frames(sub)  # a rejected append left the handle usable
    assert g.ncols == p.frame_slice(0, 6).total_cols
