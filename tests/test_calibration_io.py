"""The data formats either side of the path, C++ host layer kalibr_amd/host/calibration_io.*:

* GridCalibrationTargetObservation records in synchronized sets -> buildRigProblem must rebuild the packed problem
  exactly (same views, corner ids in target order, keypoints): CalibrateMultiCameraRig's term creation
  (CalibrationTools.hpp:376-414, CameraCalibrator.hpp:203-265);
* AprilGrid corner geometry (GridCalibrationTargetAprilgrid.cpp:83-95) == the synthetic generator's;
* targetPoseGuess (CalibrationTools.hpp:315-355) incl. the reference's accumulate order T_t_cN * B_0 * ... * B_{N-1};
* the CameraInfo / TransformStamped / TFMessage YAML of kalibr_calibrate_cameras (CalibrateCameras.cpp:313-356,
  ROSToYAMLConverter.cpp:32-75, KalibrToROSConverter.cpp:15-55), parsed back and checked field by field.
No GPU: the driver only packs and writes files.
"""
import json
import os
import subprocess

import numpy as np
import pytest
import yaml

from kalibr_amd import synth
from tests.host_problem import write_problem
from tests.test_host_cpp import driver  # noqa: F401  (fixture: builds tests/cpp/test_host.cpp)

ROS_MODEL = {synth.PINHOLE_RADTAN: ("pinhole-radtan", "plumb_bob"), synth.OMNI_RADTAN: ("omni-radtan", "plumb_bob"),
             synth.EUCM: ("eucm-none", ""), synth.OMNI: ("omni-none", ""), synth.DS: ("ds-none", "double_sphere"),
             synth.PINHOLE_EQUI: ("pinhole-equi", "equidistant"), synth.PINHOLE_FOV: ("pinhole-fov", "fov")}
# index of fu in the intrinsics vector, and the d[] entries (CameraCalibrator::GetCameraInfoParams)
K_AT = {synth.PINHOLE_RADTAN: 0, synth.PINHOLE_EQUI: 0, synth.PINHOLE_FOV: 0, synth.OMNI_RADTAN: 1, synth.OMNI: 1,
        synth.EUCM: 2, synth.DS: 2}
D_IDX = {synth.PINHOLE_RADTAN: [4, 5, 6, 7], synth.PINHOLE_EQUI: [4, 5, 6, 7], synth.PINHOLE_FOV: [4],
         synth.OMNI_RADTAN: [0, 5, 6, 7, 8], synth.OMNI: [0], synth.EUCM: [0, 1], synth.DS: [0, 1]}


def run_io(driver, tmp_path, p):  # noqa: F811
    path = str(tmp_path / "p.bin")
    write_problem(path, p)
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([driver, "io", path, str(out), "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1]), out


CASES = {
    "stereo_ragged": lambda: synth.make_config(2, n_frames=40, p_view=0.5, seed_offset=7),
    "rig8": lambda: synth.make_config(4, n_frames=10, p_view=0.7),
    "omni_eucm": lambda: synth.make_config(3, n_frames=12, p_view=0.8),
    "ds_equi_fov_omni": lambda: synth.make_config(6, n_frames=10, p_view=0.8),
    "mono": lambda: synth.make_config(1, n_frames=8),
}


@pytest.mark.parametrize("name", list(CASES))
def test_observations_pack_into_the_same_problem(driver, tmp_path, name):  # noqa: F811
    p = CASES[name]()
    r, _ = run_io(driver, tmp_path, p)
    assert r["target_diff"] == 0.0, r
    assert r["same_views"] == 1 and r["same_corners"] == 1 and r["same_y"] == 1 and r["same_intr_base"] == 1, r
    assert r["n_frames"] == p.n_frames


@pytest.mark.parametrize("name", ["stereo_ragged", "rig8"])
def test_target_pose_guess_reference_order(driver, tmp_path, name):  # noqa: F811
    p = CASES[name]()
    r, _ = run_io(driver, tmp_path, p)
    N, st = p.n_cams, p.state_init
    offb = N * 10
    offf = offb + 7 * (N - 1)
    B = [synth.pose_to_T(st[offb + 7 * j: offb + 7 * j + 7]) for j in range(N - 1)]
    for f, g in enumerate(r["guess"]):
        counts = np.zeros(N, dtype=int)
        for v in np.nonzero(p.view_frame == f)[0]:
            counts[p.view_cam[v]] = p.view_offset[v + 1] - p.view_offset[v]
        m = int(np.argmax(counts))  # first maximum, as std::max_element
        chain = np.eye(4)
        for j in range(m):
            chain = B[j] @ chain
        T = synth.pose_to_T(st[offf + 7 * f: offf + 7 * f + 7]) @ synth.inv_T(chain)  # T_t_cm
        for j in range(m):
            T = T @ B[j]  # std::accumulate(baselines[0..m), T_t_cm, std::multiplies)
        G = synth.pose_to_T(np.asarray(g))
        assert np.abs(G - T).max() < 1e-12, (f, m)


@pytest.mark.parametrize("name", list(CASES))
def test_yaml_export(driver, tmp_path, name):  # noqa: F811
    p = CASES[name]()
    r, out = run_io(driver, tmp_path, p)
    N, st = p.n_cams, p.state_init
    assert r["n_files"] == N + (1 if N > 1 else 0)
    for i in range(N):
        m = int(p.cam_model[i])
        ci = yaml.safe_load((out / f"calibration_cam{i}.yaml").read_text())
        intr = st[10 * i: 10 * i + 10]
        k = K_AT[m]
        fx, fy, cx, cy = intr[k: k + 4]
        assert ci["header"]["frame_id"] == f"cam{i}" and ci["width"] == 1280 and ci["height"] == 1024
        assert ci["distortion_model"] == ROS_MODEL[m][1]
        assert ci["k"] == [fx, 0.0, cx, 0.0, fy, cy, 0.0, 0.0, 1.0]
        assert ci["p"] == [fx, 0.0, cx, 0.0, 0.0, fy, cy, 0.0, 0.0, 0.0, 1.0, 0.0]
        assert ci["r"] == [1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0]
        assert ci["d"] == [float(intr[j]) for j in D_IDX[m]]  # shortest round-trip decimals: exact
        assert ci["roi"]["do_rectify"] is False
    if N == 1:
        return
    offb = N * 10
    if N == 2:
        tfs = [yaml.safe_load((out / "transform_cam0_to_cam1.yaml").read_text())]
    else:
        tfs = yaml.safe_load((out / "camera_chain_transforms.yaml").read_text())["transforms"]
    assert len(tfs) == N - 1
    for j, tf in enumerate(tfs):
        b = st[offb + 7 * j: offb + 7 * j + 7]
        assert tf["header"]["frame_id"] == f"cam{j}" and tf["child_frame_id"] == f"cam{j + 1}"
        tr, ro = tf["transform"]["translation"], tf["transform"]["rotation"]
        assert [tr["x"], tr["y"], tr["z"]] == [float(x) for x in b[4:7]]
        q = np.array([ro["x"], ro["y"], ro["z"], ro["w"]])
        assert q[3] >= 0.0  # Transformation(T) re-derives q with r2quat's sign convention
        assert np.abs(synth.quat2r(q) - synth.quat2r(b[:4])).max() < 1e-14


def _run_init(driver, tmp_path, p):  # noqa: F811
    import copy
    q = copy.copy(p)
    q.state_init = p.state_truth  # the driver reads the truth as the problem state
    path = str(tmp_path / "init.bin")
    write_problem(path, q)
    W, H = p.resolution
    r = subprocess.run([driver, "init", path, str(W), str(H)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("models,noise,rot_tol,trans_tol", [
    ([synth.PINHOLE_RADTAN] * 2, 0.0, 1e-7, 1e-7),
    ([synth.PINHOLE_RADTAN] * 2, 0.3, 5e-3, 5e-3),
    ([synth.PINHOLE_EQUI, synth.PINHOLE_FOV], 0.0, 1e-6, 1e-6),
])
def test_estimate_transformation_recovers_pose(driver, tmp_path, models, noise, rot_tol, trans_tol):  # noqa: F811
    """PinholeProjection::estimateTransformation (PinholeProjection.hpp(impl):811-880) without OpenCV: back-projection
    through the model, planar DLT + LM in normalised coordinates; every view's T_t_c recovered from the synthetic
    keypoints with the true intrinsics (exactly without noise, to the noise level at 0.3 px)."""
    p = synth.make_problem(models, 30, seed=4242, noise_px=noise, resolution=(1280, 1024))
    r = _run_init(driver, tmp_path, p)
    assert r["estimated"] == r["views"] > 0, r
    assert r["max_rot"] < rot_tol and r["max_trans"] < trans_tol, r


def test_initialize_intrinsics_vanishing_points(driver, tmp_path):  # noqa: F811
    """PinholeProjection::initializeIntrinsics (:713-803): focal length from the vanishing points of circles fitted to
    the corner rows of complete views -- an approximate initialiser for strongly distorted (equidistant) lenses: within
    20 % of the true focal length; the image centre at ((cols - 1) / 2, (rows - 1) / 2); the fallback focal length
    when no view yields a guess."""
    p = synth.make_problem([synth.PINHOLE_EQUI], 40, seed=99, noise_px=0.0, resolution=(1280, 1024))
    r = _run_init(driver, tmp_path, p)
    ok, f0, _, cu, cv = r["init"][0][:5]
    fu = p.state_truth[0]
    assert ok == 1 and abs(f0 - fu) / fu < 0.2, (f0, fu)
    assert cu == (1280 - 1) / 2 and cv == (1024 - 1) / 2
    assert r["fallback_ok"] == 1 and r["fallback_f"] == 777.0


OMNI_EXACT = {synth.OMNI: [1.0, 450.0, 450.0, 639.5, 511.5], synth.EUCM: [0.5, 1.0, 225.0, 225.0, 639.5, 511.5],
              synth.DS: [0.0, 0.5, 225.0, 225.0, 639.5, 511.5]}


def test_omni_family_initializers_exact(driver, tmp_path):  # noqa: F811
    """OmniProjection::initializeIntrinsics (OmniProjection.hpp(impl):724-846) and the EUCM / DS initialisers built
    on it (ExtendedUnifiedProjection.hpp(impl):731-760, DoubleSphereProjection.hpp(impl):783-812).  Each row's image
    is exactly the conic the initialiser fits when the true camera is the xi = 1 unified model (EUCM alpha = 1/2,
    beta = 1; DS xi = 0, alpha = 1/2, all with the principal point at the image centre): noise-free keypoints give
    back the true intrinsics (EUCM / DS focal = gamma / 2).  estimateTransformation through each model's
    keypointToEuclidean recovers every view's pose."""
    models = [synth.OMNI, synth.EUCM, synth.DS]
    p = synth.make_problem(models, 24, seed=77, noise_px=0.0, resolution=(1280, 1024),
                           intrinsics=[OMNI_EXACT[m] for m in models])
    r = _run_init(driver, tmp_path, p)
    assert r["estimated"] == r["views"] > 0 and r["max_rot"] < 1e-6 and r["max_trans"] < 1e-6, r
    for i, m in enumerate(models):
        ok, *intr = r["init"][i]
        assert ok == 1, r
        np.testing.assert_allclose(intr, OMNI_EXACT[m], rtol=1e-6, atol=1e-9)
    # the omni fallback: the focal length is set, false returned (the reference's warning path)
    assert r["fallback_ok"] == 0 and r["fallback_f"] == 777.0


@pytest.mark.parametrize("model", [synth.OMNI_RADTAN, synth.EUCM, synth.DS])
def test_omni_family_initializers_approximate(driver, tmp_path, model):  # noqa: F811
    """The same initialisers on the default synthetic lenses (omni xi = 0.9 with radtan, EUCM alpha = 0.6 beta = 1.1,
    DS xi = -0.2 alpha = 0.6) and 0.3 px noise: the initial guess is an xi = 1 / alpha = 1/2 camera whose focal
    length matches the lens's near-axis focal length (omni 2 f / (1 + xi), EUCM f: within 15 %; DS f / (1 + xi): within
    20 %, its rows' curvature away from the axis pulls the fitted xi = 1 focal length down by ~16 %); the
    poses from estimateTransformation with the true intrinsics stay at the noise level."""
    p = synth.make_problem([model] * 2, 30, seed=5, noise_px=0.3, resolution=(1280, 1024))
    r = _run_init(driver, tmp_path, p)
    # 0.3 px at these wide lenses' ~240-450 px near-axis focal lengths: the single-view pose is good to ~1e-2
    assert r["estimated"] == r["views"] > 0 and r["max_rot"] < 2e-2 and r["max_trans"] < 2e-2, r
    t = p.state_truth[: synth.NINTR[model]]
    if model == synth.OMNI_RADTAN:
        f_eff, k = 2 * t[1] / (1 + t[0]), 1
    elif model == synth.EUCM:
        f_eff, k = t[2], 2
    else:
        f_eff, k = t[2] / (1 + t[0]), 2
    for i in range(2):
        ok, *intr = r["init"][i]
        assert ok == 1, r
        assert abs(intr[k] - f_eff) / f_eff < (0.2 if model == synth.DS else 0.15), (intr, f_eff)
        assert intr[k] == intr[k + 1] and intr[k + 2] == 639.5 and intr[k + 3] == 511.5
