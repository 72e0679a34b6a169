"""Deterministic synthetic AprilGrid calibration problems.

Generates the observation set that Kalibr2's CalibrateMultiCameraRig consumes
(kalibr2/include/kalibr2/CalibrationTools.hpp:376-428): one target pose per
synchronised frame, camera i observes p_ci = B_{i-1} ... B_0 T_f^-1 P.

Target geometry follows GridCalibrationTargetAprilgrid::createGridPoints
(aslam_cv/aslam_cameras_april/src/GridCalibrationTargetAprilgrid.cpp:83-95) with
the board of kalibr2_ros/calibration_config.yaml:1-6 (6x5 tags, 0.088 m,
spacing 0.2954) -> 120 corners.  Quaternions are JPL [x, y, z, w]
(Schweizer-Messer/sm_kinematics/src/quaternion_algebra.cpp).

The flat state layout and the column order are documented in DESIGN.md and in
include/kalibr_hip.h.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

MAX_INTR = 10
POSE = 7

PINHOLE_RADTAN = 0
OMNI_RADTAN = 1
EUCM = 2
OMNI = 3
DS = 4
PINHOLE_EQUI = 5
PINHOLE_FOV = 6
MODEL_NAMES = {PINHOLE_RADTAN: "pinhole-radtan", OMNI_RADTAN: "omni-radtan", EUCM: "eucm", OMNI: "omni",
               DS: "ds", PINHOLE_EQUI: "pinhole-equi", PINHOLE_FOV: "pinhole-fov"}
NINTR = {PINHOLE_RADTAN: 8, OMNI_RADTAN: 9, EUCM: 6, OMNI: 5, DS: 6, PINHOLE_EQUI: 8, PINHOLE_FOV: 5}


def aprilgrid_points(tag_rows=5, tag_cols=6, tag_size=0.088, tag_spacing=0.2954):
    rows, cols = 2 * tag_rows, 2 * tag_cols
    pts = np.zeros((rows * cols, 3))
    for r in range(rows):
        for c in range(cols):
            pts[r * cols + c, 0] = (c // 2) * (1 + tag_spacing) * tag_size + (c % 2) * tag_size
            pts[r * cols + c, 1] = (r // 2) * (1 + tag_spacing) * tag_size + (r % 2) * tag_size
    return pts


# ---- JPL quaternion helpers (restated from quaternion_algebra.cpp) ----

def quat2r(q):
    x, y, z, w = q
    return np.array([
        [x * x - y * y - z * z + w * w, 2 * x * y + 2 * z * w, 2 * x * z - 2 * y * w],
        [2 * x * y - 2 * z * w, -x * x + y * y - z * z + w * w, 2 * x * w + 2 * y * z],
        [2 * x * z + 2 * y * w, -2 * x * w + 2 * y * z, -x * x - y * y + z * z + w * w],
    ])


def r2quat(R):
    c1, c2, c3 = R[0, 0], R[1, 0], R[2, 0]
    c4, c5, c6 = R[0, 1], R[1, 1], R[2, 1]
    c7, c8, c9 = R[0, 2], R[1, 2], R[2, 2]
    dc = np.abs([1 + c1 - c5 - c9, 1 - c1 + c5 - c9, 1 - c1 - c5 + c9, 1 + c1 + c5 + c9])
    m = int(np.argmax(dc))
    q = np.zeros(4)
    if m == 0:
        q[0] = 0.5 * np.sqrt(dc[0]); c = 0.25 / q[0]
        q[1] = c * (c4 + c2); q[2] = c * (c7 + c3); q[3] = c * (c8 - c6)
    elif m == 1:
        q[1] = 0.5 * np.sqrt(dc[1]); c = 0.25 / q[1]
        q[0] = c * (c4 + c2); q[2] = c * (c6 + c8); q[3] = c * (c3 - c7)
    elif m == 2:
        q[2] = 0.5 * np.sqrt(dc[2]); c = 0.25 / q[2]
        q[0] = c * (c3 + c7); q[1] = c * (c6 + c8); q[3] = c * (c4 - c2)
    else:
        q[3] = 0.5 * np.sqrt(dc[3]); c = 0.25 / q[3]
        q[0] = c * (c8 - c6); q[1] = c * (c3 - c7); q[2] = c * (c4 - c2)
    if q[3] < 0:
        q = -q
    return q


def rotvec(a):
    """Standard (right-handed, active) rotation matrix exp([a]x)."""
    th = np.linalg.norm(a)
    if th < 1e-15:
        return np.eye(3)
    k = a / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def pose_from_Rt(R, t):
    return np.concatenate([r2quat(R), t])


def pose_to_T(pose):
    T = np.eye(4)
    T[:3, :3] = quat2r(pose[:4])
    T[:3, 3] = pose[4:7]
    return T


def inv_T(T):
    Ti = np.eye(4)
    Ti[:3, :3] = T[:3, :3].T
    Ti[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return Ti


# ---- projection (vectorised, used only to synthesise observations) ----

def project(model, intr, p):
    """p: (n,3) camera-frame points -> (n,2) keypoints, valid mask."""
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    if model == PINHOLE_RADTAN:
        fu, fv, cu, cv, k1, k2, p1, p2 = intr[:8]
        mx, my = x / z, y / z
        valid = z > 0
        dist = True
    elif model in (OMNI_RADTAN, OMNI):
        xi, fu, fv, cu, cv = intr[:5]
        d = np.sqrt(x * x + y * y + z * z)
        fovp = xi if xi <= 1 else 1 / xi
        valid = z > -(fovp * d)
        mx, my = x / (z + xi * d), y / (z + xi * d)
        dist = model == OMNI_RADTAN
        if dist:
            k1, k2, p1, p2 = intr[5:9]
    elif model == EUCM:
        al, be, fu, fv, cu, cv = intr[:6]
        d = np.sqrt(be * (x * x + y * y) + z * z)
        fovp = al / (1 - al) if al <= 0.5 else (1 - al) / al
        valid = z > -(fovp * d)
        n = al * d + (1 - al) * z
        mx, my = x / n, y / n
        dist = False
    elif model == DS:
        xi, al, fu, fv, cu, cv = intr[:6]
        r2 = x * x + y * y
        d1 = np.sqrt(r2 + z * z)
        t = al / (1 - al) if al <= 0.5 else (1 - al) / al
        fovp = (t + xi) / np.sqrt(2 * t * xi + xi * xi + 1)
        valid = z > -(fovp * d1)
        k = xi * d1 + z
        n = al * np.sqrt(r2 + k * k) + (1 - al) * k
        mx, my = x / n, y / n
        dist = False
    elif model in (PINHOLE_EQUI, PINHOLE_FOV):
        fu, fv, cu, cv = intr[:4]
        mx, my = x / z, y / z
        valid = z > 0
        r = np.sqrt(mx * mx + my * my)
        if model == PINHOLE_EQUI:
            k1, k2, k3, k4 = intr[4:8]
            th = np.arctan(r)
            t2 = th * th
            thd = th * (1 + t2 * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4))))
            sc = np.where(r > 1e-8, thd / np.maximum(r, 1e-300), 1.0)
        else:
            w = intr[4]
            tw = np.tan(w / 2)
            sc = np.where(r * r < 1e-5, 2 * tw / w, np.arctan(2 * tw * r) / (np.maximum(r, 1e-300) * w))
        mx, my = mx * sc, my * sc
        dist = False
    else:
        raise ValueError(model)
    if dist:
        mx2, my2, mxy = mx * mx, my * my, mx * my
        r2 = mx2 + my2
        rad = k1 * r2 + k2 * r2 * r2
        ux = mx + mx * rad + 2 * p1 * mxy + p2 * (r2 + 2 * mx2)
        uy = my + my * rad + 2 * p2 * mxy + p1 * (r2 + 2 * my2)
        mx, my = ux, uy
    return np.stack([fu * mx + cu, fv * my + cv], axis=1), valid


@dataclass
class Problem:
    """Observation set + state in the layout of include/kalibr_hip.h."""

    cam_model: np.ndarray  # int32 [N]
    target: np.ndarray  # float64 [K,3]
    view_frame: np.ndarray  # int32 [V]  (sorted by frame, then camera)
    view_cam: np.ndarray  # int32 [V]
    view_offset: np.ndarray  # int32 [V+1]
    corner_id: np.ndarray  # int32 [Nc]
    y: np.ndarray  # float64 [Nc,2]
    state_truth: np.ndarray
    state_init: np.ndarray
    resolution: tuple = (1280, 1024)
    name: str = ""
    meta: dict = field(default_factory=dict)

    @property
    def n_cams(self):
        return int(self.cam_model.shape[0])

    @property
    def n_frames(self):
        return int(self.view_frame.max()) + 1 if self.view_frame.size else 0

    @property
    def n_views(self):
        return int(self.view_frame.shape[0])

    @property
    def n_corners(self):
        return int(self.corner_id.shape[0])

    @property
    def cam_cols(self):
        return int(sum(NINTR[int(m)] for m in self.cam_model) + 6 * (self.n_cams - 1))

    @property
    def total_cols(self):
        return self.cam_cols + 6 * self.n_frames

    def frame_slice(self, f0, f1):
        """Sub-problem holding frames [f0, f1) (frames renumbered from 0), used for sharding."""
        vm = (self.view_frame >= f0) & (self.view_frame < f1)
        vidx = np.nonzero(vm)[0]
        offs = self.view_offset
        corners = np.concatenate([np.arange(offs[v], offs[v + 1]) for v in vidx]) if vidx.size else np.zeros(0, int)
        counts = offs[vidx + 1] - offs[vidx]
        N = self.n_cams
        so = N * MAX_INTR + POSE * (N - 1)

        def cut(st):
            return np.concatenate([st[:so], st[so + POSE * f0: so + POSE * f1]])

        return Problem(
            cam_model=self.cam_model.copy(), target=self.target.copy(),
            view_frame=(self.view_frame[vidx] - f0).astype(np.int32), view_cam=self.view_cam[vidx].copy(),
            view_offset=np.concatenate([[0], np.cumsum(counts)]).astype(np.int32),
            corner_id=self.corner_id[corners].astype(np.int32), y=self.y[corners].copy(),
            state_truth=cut(self.state_truth), state_init=cut(self.state_init),
            resolution=self.resolution, name=f"{self.name}[{f0}:{f1}]", meta=dict(self.meta))


def state_size(n_cams, n_frames):
    return n_cams * MAX_INTR + POSE * (n_cams - 1) + POSE * n_frames


def make_problem(models, n_frames, seed, p_view=1.0, noise_px=0.3, min_corners=12,
                 resolution=(1280, 1024), name="", init_noise=True, intrinsics=None):
    """Synthesise an N-camera x F-frame AprilGrid problem.  intrinsics: optional per-camera
    override of the default true intrinsics (a list with None for the defaults)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    W, H = resolution
    N = len(models)
    target = aprilgrid_points()
    tcen = target.mean(axis=0)
    intr_truth = np.zeros((N, MAX_INTR))
    for i, m in enumerate(models):
        if m == PINHOLE_RADTAN:
            intr_truth[i, :8] = [881.0, 881.0, 640.0, 512.0, -0.2, 0.13, 5e-4, 5e-4]
        elif m == OMNI_RADTAN:
            intr_truth[i, :9] = [0.9, 450.0, 450.0, 640.0, 512.0, -0.05, 0.01, 1e-4, 1e-4]
        elif m == OMNI:
            intr_truth[i, :5] = [0.9, 450.0, 450.0, 640.0, 512.0]
        elif m == EUCM:
            intr_truth[i, :6] = [0.6, 1.1, 450.0, 450.0, 640.0, 512.0]
        elif m == DS:
            intr_truth[i, :6] = [-0.2, 0.6, 400.0, 400.0, 640.0, 512.0]
        elif m == PINHOLE_EQUI:
            intr_truth[i, :8] = [600.0, 600.0, 640.0, 512.0, -0.01, 0.02, -0.01, 0.003]
        elif m == PINHOLE_FOV:
            intr_truth[i, :5] = [700.0, 700.0, 640.0, 512.0, 0.9]
        else:
            raise ValueError(m)
        if intrinsics is not None and intrinsics[i] is not None:
            intr_truth[i, :NINTR[m]] = intrinsics[i]
    # rig: camera i+1 sits 0.12 m along -x from camera i, +-3 deg, +-5 mm
    base_T = []
    cam_T_c0 = [np.eye(4)]  # T_{ci, c0}
    for j in range(N - 1):
        R = rotvec(np.deg2rad(rng.uniform(-3, 3, 3)))
        o = np.array([-0.12, 0.0, 0.0]) + rng.uniform(-0.005, 0.005, 3)
        T_ci_cj1 = np.eye(4)
        T_ci_cj1[:3, :3] = R
        T_ci_cj1[:3, 3] = o
        B = inv_T(T_ci_cj1)  # T_{c(j+1), c(j)}
        base_T.append(B)
        cam_T_c0.append(B @ cam_T_c0[-1])
    rig_centre = np.array([-0.12 * (N - 1) / 2.0, 0.0, 0.0])

    frames, views = [], []
    attempts = 0
    while len(frames) < n_frames:
        attempts += 1
        if attempts > 200 * n_frames + 1000:
            raise RuntimeError("could not synthesise enough visible frames")
        depth = rng.uniform(0.6, 1.5)
        tilt_axis = rng.normal(size=2)
        tilt_axis = np.array([tilt_axis[0], tilt_axis[1], 0.0]) / np.linalg.norm(tilt_axis)
        tilt = np.deg2rad(rng.uniform(0, 35))
        roll = np.deg2rad(rng.uniform(-180, 180))
        R = rotvec(tilt_axis * tilt) @ rotvec(np.array([0, 0, roll]))
        centre = rig_centre + np.array([rng.uniform(-0.15, 0.15), rng.uniform(-0.15, 0.15), depth])
        T_c0_t = np.eye(4)
        T_c0_t[:3, :3] = R
        T_c0_t[:3, 3] = centre - R @ tcen
        fviews = []
        for i in range(N):
            T = cam_T_c0[i] @ T_c0_t
            pc = (T[:3, :3] @ target.T).T + T[:3, 3]
            kp, valid = project(models[i], intr_truth[i], pc)
            ok = valid & (pc[:, 2] > 0.05) & (kp[:, 0] >= 5) & (kp[:, 0] <= W - 5) & (kp[:, 1] >= 5) & (kp[:, 1] <= H - 5)
            ids = np.nonzero(ok)[0]
            if ids.size < min_corners or rng.uniform() > p_view:
                continue
            meas = kp[ids] + rng.normal(0.0, noise_px, (ids.size, 2))
            fviews.append((i, ids, meas))
        if not fviews:
            continue
        frames.append(inv_T(T_c0_t))  # T_f: p_c0 = T_f^-1 P
        views.append(fviews)

    vf, vc, counts, cid, ys = [], [], [], [], []
    for f, fv in enumerate(views):
        for (i, ids, meas) in fv:
            vf.append(f)
            vc.append(i)
            counts.append(ids.size)
            cid.append(ids)
            ys.append(meas)
    st_truth = np.zeros(state_size(N, n_frames))
    st_truth[: N * MAX_INTR] = intr_truth.reshape(-1)
    so = N * MAX_INTR
    for j, B in enumerate(base_T):
        st_truth[so + POSE * j: so + POSE * (j + 1)] = pose_from_Rt(B[:3, :3], B[:3, 3])
    so += POSE * (N - 1)
    for f, T in enumerate(frames):
        st_truth[so + POSE * f: so + POSE * (f + 1)] = pose_from_Rt(T[:3, :3], T[:3, 3])

    st_init = st_truth.copy()
    if init_noise:
        for i, m in enumerate(models):
            base = i * MAX_INTR
            if m == PINHOLE_RADTAN:
                st_init[base + 0: base + 2] *= 1 + 0.02 * rng.normal(size=2)
                st_init[base + 2: base + 4] += 5.0 * rng.normal(size=2)
                st_init[base + 4: base + 8] = 0.0
            elif m in (OMNI_RADTAN, OMNI):
                st_init[base + 0] *= 1 + 0.02 * rng.normal()
                st_init[base + 1: base + 3] *= 1 + 0.02 * rng.normal(size=2)
                st_init[base + 3: base + 5] += 5.0 * rng.normal(size=2)
                if m == OMNI_RADTAN:
                    st_init[base + 5: base + 9] = 0.0
            elif m == DS:
                st_init[base + 0] += 0.02 * rng.normal()
                st_init[base + 1] *= 1 + 0.02 * rng.normal()
                st_init[base + 2: base + 4] *= 1 + 0.02 * rng.normal(size=2)
                st_init[base + 4: base + 6] += 5.0 * rng.normal(size=2)
            elif m in (PINHOLE_EQUI, PINHOLE_FOV):
                st_init[base + 0: base + 2] *= 1 + 0.02 * rng.normal(size=2)
                st_init[base + 2: base + 4] += 5.0 * rng.normal(size=2)
                if m == PINHOLE_EQUI:
                    st_init[base + 4: base + 8] = 0.0
                else:
                    st_init[base + 4] *= 1 + 0.05 * rng.normal()
            elif m == EUCM:
                st_init[base + 0: base + 2] *= 1 + 0.02 * rng.normal(size=2)
                st_init[base + 2: base + 4] *= 1 + 0.02 * rng.normal(size=2)
                st_init[base + 4: base + 6] += 5.0 * rng.normal(size=2)
        so = N * MAX_INTR
        for k in range(N - 1 + n_frames):
            o = so + POSE * k
            T = pose_to_T(st_truth[o: o + POSE])
            Rn = rotvec(np.deg2rad(1.0) * rng.normal(size=3) / np.sqrt(3)) @ T[:3, :3]
            tn = T[:3, 3] + 0.01 * rng.normal(size=3) / np.sqrt(3)
            st_init[o: o + POSE] = pose_from_Rt(Rn, tn)
    return Problem(
        cam_model=np.asarray(models, dtype=np.int32), target=target,
        view_frame=np.asarray(vf, dtype=np.int32), view_cam=np.asarray(vc, dtype=np.int32),
        view_offset=np.concatenate([[0], np.cumsum(counts)]).astype(np.int32),
        corner_id=np.concatenate(cid).astype(np.int32), y=np.concatenate(ys, axis=0).astype(np.float64),
        state_truth=st_truth, state_init=st_init, resolution=resolution, name=name,
        meta={"seed": seed, "p_view": p_view, "noise_px": noise_px})


# BASELINE.json configs; seeds PCG64(20261015 + config_index)
CONFIGS = {
    1: dict(models=[PINHOLE_RADTAN], n_frames=50, name="1x pinhole-radtan, 50-frame 6x5 AprilGrid"),
    2: dict(models=[PINHOLE_RADTAN] * 2, n_frames=500, name="2-cam stereo pinhole-radtan, 500 frames"),
    3: dict(models=[OMNI_RADTAN, OMNI_RADTAN, EUCM, EUCM], n_frames=1000, name="4-cam omni + EUCM mixed rig, 1000 frames"),
    4: dict(models=[PINHOLE_RADTAN] * 8, n_frames=2000, name="8-cam pinhole rig, 2000 frames"),
    # not a BASELINE.json config: the remaining Kalibr2 camera models (CameraModels.hpp:25-133) in one rig,
    # for parity tests only
    6: dict(models=[DS, PINHOLE_EQUI, PINHOLE_FOV, OMNI], n_frames=200,
            name="4-cam double-sphere + equidistant + FOV + omni rig, 200 frames (parity only)"),
}


def make_config(idx, p_view=1.0, n_frames=None, seed_offset=0, **kw):
    c = CONFIGS[idx]
    return make_problem(c["models"], n_frames or c["n_frames"], seed=20261015 + idx + seed_offset,
                        p_view=p_view, name=c["name"], **kw)


# ---------------------------------------------------------------------------------------------
# configs[4]: 2-cam + IMU continuous-time calibration on a B-spline pose trajectory.
# The rig (IMU body b) moves in front of the fixed target (world = target frame) along a cubic
# BSplinePose with a RotationVector rotation (bsplines/src/BSplinePose.cpp; RotationVector.cpp).
# Truth = the spline with the coefficients below; camera and IMU measurements are generated from it.
# ---------------------------------------------------------------------------------------------

def bspline_basis(order, knots, seg):
    """Basis matrix of valid segment `seg`: the M(k, i) recursion of BSpline.cpp:70-152."""
    def d0(k, i, j):
        den = knots[j + k - 1] - knots[j]
        return 0.0 if den <= 0 else (knots[i] - knots[j]) / den

    def d1(k, i, j):
        den = knots[j + k - 1] - knots[j]
        return 0.0 if den <= 0 else (knots[i + 1] - knots[i]) / den

    def M(k, i):
        if k == 1:
            return np.ones((1, 1))
        Mp = M(k - 1, i)
        M1 = np.vstack([Mp, np.zeros((1, k - 1))])
        M2 = np.vstack([np.zeros((1, k - 1)), Mp])
        A = np.zeros((k - 1, k))
        B = np.zeros((k - 1, k))
        for idx in range(k - 1):
            j = i - k + 2 + idx
            A[idx, idx], A[idx, idx + 1] = 1 - d0(k, i, j), d0(k, i, j)
            B[idx, idx], B[idx, idx + 1] = -d1(k, i, j), d1(k, i, j)
        return M1 @ A + M2 @ B

    return M(order, seg + order - 1)


def bspline_weights(order, knots, t, deriv):
    """(bidx, w[order]) of BSpline::evalDAndJacobian at t (BSpline.cpp:237-387)."""
    knots = np.asarray(knots)
    n = knots.size
    tmin, tmax = knots[order - 1], knots[n - order]
    if t < tmin or t > tmax + 1e-10:
        raise ValueError("time outside the spline interval")
    if abs(tmax - t) < 1e-10:
        t = tmax
    idx = n - order - 1 if t == tmax else int(np.searchsorted(knots, t, side="right")) - 1
    dt = knots[idx + 1] - knots[idx]
    u = 0.0 if dt <= 0 else (t - knots[idx]) / dt
    mult = 0.0 if dt <= 0 else 1.0 / dt ** deriv
    uv = np.zeros(order)
    uu = 1.0
    for i in range(deriv, order):
        dm = 1
        for q in range(deriv):
            dm *= i - q
        uv[i] = mult * uu * dm
        uu *= u
    bidx = idx - order + 1
    return bidx, bspline_basis(order, knots, bidx).T @ uv


def rv_to_C(a):
    """RotationVector::parametersToRotationMatrix (RotationVector.cpp:10-52) = standard exp(-[a]x)."""
    return rotvec(-np.asarray(a, dtype=float))


def rv_from_C(C):
    """RotationVector::rotationMatrixToParameters (RotationVector.cpp:54-78)."""
    tr = max(-1.0, min((C[0, 0] + C[1, 1] + C[2, 2] - 1.0) * 0.5, 1.0))
    a = np.arccos(tr)
    if abs(a) < 1e-14:
        return np.zeros(3)
    p = np.array([C[2, 1] - C[1, 2], C[0, 2] - C[2, 0], C[1, 0] - C[0, 1]])
    n2 = np.linalg.norm(p)
    if abs(n2) < 1e-14:
        return np.zeros(3)
    return (-a / n2) * p


def rv_S(a):
    """RotationVector::parametersToSMatrix (RotationVector.cpp:80-103)."""
    a = np.asarray(a, dtype=float)
    ang = np.linalg.norm(a)
    if ang < 1e-14:
        return np.eye(3)
    ax = a / ang
    c1 = -2.0 * np.sin(ang / 2) ** 2 / ang
    c2 = (ang - np.sin(ang)) / ang
    X = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + c1 * X + c2 * X @ X


@dataclass
class SplineProblem:
    order: int
    knots: np.ndarray
    cam_model: np.ndarray
    target: np.ndarray
    frame_time: np.ndarray
    view_frame: np.ndarray
    view_cam: np.ndarray
    view_offset: np.ndarray
    corner_id: np.ndarray
    y: np.ndarray
    imu_time: np.ndarray
    imu_gyro: np.ndarray
    imu_acc: np.ndarray
    sigma_gyro: float
    sigma_acc: float
    state_truth: np.ndarray
    state_init: np.ndarray
    name: str = ""
    meta: dict = field(default_factory=dict)

    @property
    def n_cams(self):
        return int(self.cam_model.size)

    @property
    def n_frames(self):
        return int(self.frame_time.size)

    @property
    def n_views(self):
        return int(self.view_frame.size)

    @property
    def n_corners(self):
        return int(self.corner_id.size)

    @property
    def n_imu(self):
        return int(self.imu_time.size)

    @property
    def n_coeffs(self):
        return int(self.knots.size - self.order)

    @property
    def cam_cols(self):
        return int(sum(NINTR[int(m)] for m in self.cam_model)) + 6 * (self.n_cams - 1) + 6 + 9

    @property
    def total_cols(self):
        return self.cam_cols + 6 * self.n_coeffs

    @property
    def off_coeff(self):
        return self.n_cams * MAX_INTR + POSE * (self.n_cams - 1) + POSE + 9


def spline_state_size(n_cams, n_coeffs):
    return n_cams * MAX_INTR + POSE * (n_cams - 1) + POSE + 9 + 6 * n_coeffs


def spline_eval(order, knots, coeffs, t, deriv):
    b, w = bspline_weights(order, knots, t, deriv)
    return w @ coeffs[b: b + order]


def make_spline_problem(models, n_frames, seed, cam_rate=20.0, imu_rate=200.0, knots_per_second=50.0,
                        order=4, noise_px=0.3, sigma_gyro=0.005, sigma_acc=0.05, min_corners=12,
                        resolution=(1280, 1024), name="", init_noise=True):
    """Synthesise configs[4]: an N-camera rig + IMU on a B-spline trajectory in front of the AprilGrid."""
    rng = np.random.Generator(np.random.PCG64(seed))
    W, H = resolution
    N = len(models)
    target = aprilgrid_points()
    tcen = target.mean(axis=0)
    base = make_problem(models, 1, seed, init_noise=False)  # camera truth (intrinsics, baselines)
    intr_truth = base.state_truth[: N * MAX_INTR].reshape(N, MAX_INTR)
    cam_T_c0 = [np.eye(4)]
    base_T = []
    for j in range(N - 1):
        o = N * MAX_INTR + POSE * j
        B = pose_to_T(base.state_truth[o: o + POSE])
        base_T.append(B)
        cam_T_c0.append(B @ cam_T_c0[-1])
    # IMU -> cam0
    T_c0_b = np.eye(4)
    T_c0_b[:3, :3] = rotvec(np.deg2rad(np.array([2.0, -3.0, 1.5])))
    T_c0_b[:3, 3] = [0.03, -0.02, 0.01]
    t0 = 0.0
    span = (n_frames - 1) / cam_rate  # frames at t0 .. t0 + span
    dtk = 1.0 / knots_per_second
    nseg = max(1, int(np.ceil(span / dtk - 1e-9)))
    n_knots = nseg + 2 * order - 1  # uniform knots, [t_min, t_max] = [t0, t0 + nseg dtk]
    knots = t0 + dtk * (np.arange(n_knots) - (order - 1))
    K = n_knots - order
    # smooth excitation (rotation about all axes, translation) of cam0 in the target frame
    ph = rng.uniform(0, 2 * np.pi, 6)
    fr = np.array([0.23, 0.31, 0.17, 0.13, 0.19, 0.11])
    amp_r = np.deg2rad(np.array([14.0, 12.0, 18.0]))
    rig_centre = np.array([-0.12 * (N - 1) / 2.0, 0.0, 0.0])

    def T_w_c0(t):
        R = rotvec(amp_r * np.sin(2 * np.pi * fr[:3] * t + ph[:3]))
        c = tcen - rig_centre + np.array([0.12 * np.sin(2 * np.pi * fr[3] * t + ph[3]),
                                          0.10 * np.sin(2 * np.pi * fr[4] * t + ph[4]),
                                          -1.0 + 0.2 * np.sin(2 * np.pi * fr[5] * t + ph[5])])
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = c
        return T

    # Greville abscissae -> coefficients [p | rotation vector] of T_w_b = T_w_c0 T_c0_b
    coeffs = np.zeros((K, 6))
    for k in range(K):
        tau = knots[k + 1: k + order].mean()
        Twb = T_w_c0(tau) @ T_c0_b
        coeffs[k, :3] = Twb[:3, 3]
        coeffs[k, 3:] = rv_from_C(Twb[:3, :3])
    frame_time = t0 + np.arange(n_frames) / cam_rate
    vf, vc, counts, cid, ys = [], [], [], [], []
    T_b_c0 = inv_T(T_c0_b)
    for f, t in enumerate(frame_time):
        v = spline_eval(order, knots, coeffs, t, 0)
        Twb = np.eye(4)
        Twb[:3, :3] = rv_to_C(v[3:])
        Twb[:3, 3] = v[:3]
        T_c0_w = inv_T(Twb @ T_b_c0)
        for i in range(N):
            T = cam_T_c0[i] @ T_c0_w
            pc = (T[:3, :3] @ target.T).T + T[:3, 3]
            kp, valid = project(models[i], intr_truth[i], pc)
            ok = valid & (pc[:, 2] > 0.05) & (kp[:, 0] >= 5) & (kp[:, 0] <= W - 5) & (kp[:, 1] >= 5) & (kp[:, 1] <= H - 5)
            ids = np.nonzero(ok)[0]
            if ids.size < min_corners:
                continue
            vf.append(f)
            vc.append(i)
            counts.append(ids.size)
            cid.append(ids)
            ys.append(kp[ids] + rng.normal(0.0, noise_px, (ids.size, 2)))
    g_w = 9.81 * np.array([0.08, -0.99, 0.06]) / np.linalg.norm([0.08, -0.99, 0.06])
    b_g = np.array([0.002, -0.001, 0.003])
    b_a = np.array([0.05, -0.03, 0.02])
    t_max = knots[n_knots - order]
    imu_time = t0 + np.arange(int(np.floor((t_max - t0) * imu_rate + 1e-9)) + 1) / imu_rate
    gyro = np.zeros((imu_time.size, 3))
    acc = np.zeros((imu_time.size, 3))
    for m, t in enumerate(imu_time):
        v0 = spline_eval(order, knots, coeffs, t, 0)
        v1 = spline_eval(order, knots, coeffs, t, 1)
        v2 = spline_eval(order, knots, coeffs, t, 2)
        Cwb = rv_to_C(v0[3:])
        om = -Cwb.T @ rv_S(v0[3:]) @ v1[3:]   # BSplinePose::angularVelocityBodyFrame
        fb = Cwb.T @ (v2[:3] - g_w)
        gyro[m] = om + b_g + rng.normal(0.0, sigma_gyro, 3)
        acc[m] = fb + b_a + rng.normal(0.0, sigma_acc, 3)
    st = np.zeros(spline_state_size(N, K))
    st[: N * MAX_INTR] = intr_truth.reshape(-1)
    so = N * MAX_INTR
    for j, B in enumerate(base_T):
        st[so + POSE * j: so + POSE * (j + 1)] = pose_from_Rt(B[:3, :3], B[:3, 3])
    so += POSE * (N - 1)
    st[so: so + POSE] = pose_from_Rt(T_c0_b[:3, :3], T_c0_b[:3, 3])
    so += POSE
    st[so: so + 3] = b_g
    st[so + 3: so + 6] = b_a
    st[so + 6: so + 9] = g_w
    so += 9
    st[so:] = coeffs.reshape(-1)
    st_init = st.copy()
    if init_noise:
        pinit = make_problem(models, 1, seed, init_noise=True)
        st_init[: N * MAX_INTR] = pinit.state_init[: N * MAX_INTR]
        so = N * MAX_INTR
        for k in range(N):  # baselines + T_c0_b: 1 deg / 1 cm
            o = so + POSE * k
            T = pose_to_T(st[o: o + POSE])
            Rn = rotvec(np.deg2rad(1.0) * rng.normal(size=3) / np.sqrt(3)) @ T[:3, :3]
            tn = T[:3, 3] + 0.01 * rng.normal(size=3) / np.sqrt(3)
            st_init[o: o + POSE] = pose_from_Rt(Rn, tn)
        so += POSE * N
        st_init[so: so + 6] = 0.0  # biases
        st_init[so + 6: so + 9] = rotvec(np.deg2rad(3.0) * rng.normal(size=3) / np.sqrt(3)) @ g_w
        so += 9
        c = st_init[so:].reshape(K, 6)
        c[:, :3] += 0.005 * rng.normal(size=(K, 3))
        c[:, 3:] += np.deg2rad(0.5) * rng.normal(size=(K, 3))
    return SplineProblem(
        order=order, knots=knots, cam_model=np.asarray(models, dtype=np.int32), target=target,
        frame_time=frame_time, view_frame=np.asarray(vf, dtype=np.int32), view_cam=np.asarray(vc, dtype=np.int32),
        view_offset=np.concatenate([[0], np.cumsum(counts)]).astype(np.int32),
        corner_id=np.concatenate(cid).astype(np.int32), y=np.concatenate(ys, axis=0).astype(np.float64),
        imu_time=imu_time, imu_gyro=gyro, imu_acc=acc, sigma_gyro=sigma_gyro, sigma_acc=sigma_acc,
        state_truth=st, state_init=st_init, name=name,
        meta={"seed": seed, "cam_rate": cam_rate, "imu_rate": imu_rate, "knots_per_second": knots_per_second,
              "noise_px": noise_px})


def make_spline_config(n_frames=None, seed_offset=0, **kw):
    """configs[4]: '2-cam + IMU continuous-time B-spline (aslam_splines) calibration, 1200 frames'."""
    return make_spline_problem([PINHOLE_RADTAN] * 2, n_frames or 1200, seed=20261015 + 5 + seed_offset,
                               name="2-cam + IMU continuous-time B-spline calibration, 1200 frames", **kw)


def make_position_priors(p, n, sigma=0.002, seed=7, rate=None, anisotropic=True):
    """ErrorTermEuclidean priors on the spline position (e.g. a motion-capture or GNSS track): n times spread over
    the spline's valid range (or every 1/rate s), priors = the true p(t) plus noise, covariances N (sigma^2 I, or a
    random SPD of that scale).  Returns (times [n], priors [n][3], N [n][3][3])."""
    rng = np.random.default_rng(seed)
    o, kn = p.order, p.knots
    t0, t1 = kn[o - 1], kn[kn.size - o]
    if rate:
        t = t0 + np.arange(int(np.floor((t1 - t0) * rate + 1e-9)) + 1) / rate
    else:
        t = np.sort(rng.uniform(t0, t1, n))
    c = p.state_truth[p.off_coeff:].reshape(-1, 6)
    pr = np.array([spline_eval(o, kn, c, tk, 0)[:3] for tk in t])
    N = np.zeros((t.size, 3, 3))
    for k in range(t.size):
        if anisotropic:
            A = rng.normal(size=(3, 3))
            Q, _ = np.linalg.qr(A)
            N[k] = sigma ** 2 * (Q @ np.diag(rng.uniform(0.5, 2.0, 3)) @ Q.T)
        else:
            N[k] = sigma ** 2 * np.eye(3)
        pr[k] += np.linalg.cholesky(N[k]) @ rng.normal(size=3)
    return t, pr, N
