"""ctypes wrapper of the CPU restatement (oracle/kb_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package kalibr_amd/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libkb_oracle.so")
_lib = None

dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int)


class _Problem(C.Structure):
    _fields_ = [("n_cams", C.c_int), ("n_frames", C.c_int), ("n_views", C.c_int), ("n_corners", C.c_int),
                ("n_target", C.c_int), ("cam_model", ip), ("target", dp), ("view_frame", ip), ("view_cam", ip),
                ("view_offset", ip), ("corner_id", ip), ("y", dp)]


class _Arrow(C.Structure):
    _fields_ = [("C", C.c_int), ("F", C.c_int), ("Hff", dp), ("Hfc", dp), ("Hcc", dp), ("gf", dp), ("gc", dp),
                ("cost", C.c_double)]


class _MargOpts(C.Structure):
    _fields_ = [("column_scaling", C.c_int), ("eps_norm", C.c_double), ("eps_svd", C.c_double),
                ("svd_tol", C.c_double), ("n_rows", C.c_double)]


class _MargInfo(C.Structure):
    _fields_ = [("sv", dp), ("V", dp), ("rank", C.c_int), ("sweeps", C.c_int), ("tol", C.c_double),
                ("gap", C.c_double), ("log2sum", C.c_double)]


class _Options(C.Structure):
    _fields_ = [("policy", C.c_int), ("lambda0", C.c_double), ("max_iterations", C.c_int), ("eps_x", C.c_double),
                ("eps_j", C.c_double), ("nthreads", C.c_int), ("marg", C.POINTER(_MargOpts)),
                ("solve_info", C.POINTER(_MargInfo)), ("analyze_info", C.POINTER(_MargInfo))]


EPS = float(np.finfo(float).eps)


def marg_opts(n_rows, column_scaling=True, eps_norm=EPS, eps_svd=1e-6, svd_tol=-1.0):
    """LinearSolverOptions as Kalibr2's CalibrateCameras sets them (CalibrateCameras.cpp:263-267): column scaling,
    epsSVD 1e-6, the rest default (LinearSolverOptions.cpp:30-38)."""
    return _MargOpts(int(column_scaling), eps_norm, eps_svd, svd_tol, float(n_rows))


class _InfoBuf:
    def __init__(self, Cc):
        self.sv = np.zeros(Cc)
        self.V = np.zeros((Cc, Cc))
        self.s = _MargInfo(_d(self.sv), _d(self.V), 0, 0, 0.0, 0.0, 0.0)

    def result(self):
        return dict(sv=self.sv.copy(), V=self.V.copy(), rank=self.s.rank, sweeps=self.s.sweeps, tol=self.s.tol,
                    gap=self.s.gap, log2sum=self.s.log2sum)


class _PcgOpts(C.Structure):
    _fields_ = [("tolerance", C.c_double), ("max_iterations", C.c_int), ("absolute_tolerance", C.c_int),
                ("prev_residual", C.c_double)]


class _PcgInfo(C.Structure):
    _fields_ = [("iterations", C.c_int), ("residual", C.c_double), ("d0", C.c_double)]


# projection / distortion DV sizes per camera model (CameraDesignVariable's projection and distortion DVs,
# CameraDesignVariable.hpp(impl):4-81; PinholeProjection.hpp:28, OmniProjection.hpp:26, ...)
_DV_SPLIT = {0: (4, 4), 1: (5, 4), 2: (6,), 3: (5,), 4: (6,), 5: (4, 4), 6: (4, 1)}


def pcg_camera_blocks(cam_model):
    """Design-variable blocks of the camera columns: per camera projection (+ distortion), then per baseline the
    rotation and translation DVs."""
    sizes = [s for m in cam_model for s in _DV_SPLIT[int(m)]]
    return sizes + [3, 3] * (len(cam_model) - 1)


class _Srv(C.Structure):
    _fields_ = [("J_start", C.c_double), ("J_final", C.c_double), ("dx_final", C.c_double), ("dj_final", C.c_double),
                ("iterations", C.c_int), ("failed_iterations", C.c_int), ("linear_solver_failure", C.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        L.kbo_eval_cost.restype = C.c_double
        L.kbo_term_dense.restype = C.c_double
        L.kbo_apply_update.restype = C.c_double
        L.kbo_time_gn.restype = C.c_double
        L.kbo_jt_create.restype = C.c_void_p
        L.kbo_jt_destroy.argtypes = [C.c_void_p]
        L.kbo_jt_build.argtypes = [C.c_void_p, dp, C.c_int, dp]
        L.kbo_jt_normal_arrow.argtypes = [C.c_void_p, C.c_int, C.POINTER(_Arrow)]
        L.kbo_jt_nnz.argtypes = [C.c_void_p]
        L.kbo_jt_nnz.restype = C.c_longlong
        L.kbo_arrow_solve.argtypes = [C.POINTER(_Arrow), C.c_double, C.c_int, dp]
        L.kbo_dense_solve.argtypes = [C.POINTER(_Arrow), C.c_double, dp]
        L.kbo_arrow_schur_partial.argtypes = [C.POINTER(_Arrow), C.c_double, C.c_int, C.c_int, dp, dp, ip]
        L.kbo_arrow_solve_ex.argtypes = [C.POINTER(_Arrow), C.c_double, C.c_int, dp, C.POINTER(_MargOpts),
                                         C.POINTER(_MargInfo)]
        L.kbo_marginal_solve.argtypes = [C.c_int, dp, dp, dp, C.POINTER(_MargOpts), dp, C.POINTER(_MargInfo)]
        L.kbo_sym_eig.argtypes = [C.c_int, dp, dp, dp]
        L.kbo_arrow_pcg.argtypes = [C.POINTER(_Arrow), C.c_double, C.c_int, ip, C.POINTER(_PcgOpts), dp,
                                    C.POINTER(_PcgInfo)]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(dp)


def _i(a):
    return a.ctypes.data_as(ip)


class Oracle:
    """Holds one problem (arrays kept alive) and exposes the restated reference path."""

    def __init__(self, prob):
        self.prob = prob
        self._keep = dict(
            cam_model=np.ascontiguousarray(prob.cam_model, dtype=np.int32),
            target=np.ascontiguousarray(prob.target, dtype=np.float64),
            view_frame=np.ascontiguousarray(prob.view_frame, dtype=np.int32),
            view_cam=np.ascontiguousarray(prob.view_cam, dtype=np.int32),
            view_offset=np.ascontiguousarray(prob.view_offset, dtype=np.int32),
            corner_id=np.ascontiguousarray(prob.corner_id, dtype=np.int32),
            y=np.ascontiguousarray(prob.y, dtype=np.float64))
        k = self._keep
        self.P = _Problem(prob.n_cams, prob.n_frames, prob.n_views, prob.n_corners, k["target"].shape[0],
                          _i(k["cam_model"]), _d(k["target"]), _i(k["view_frame"]), _i(k["view_cam"]),
                          _i(k["view_offset"]), _i(k["corner_id"]), _d(k["y"]))
        self.C = prob.cam_cols
        self.ncols = prob.total_cols

    # -- primitives --
    def cost(self, state, nthreads=1):
        st = np.ascontiguousarray(state, dtype=np.float64)
        return lib().kbo_eval_cost(C.byref(self.P), _d(st), nthreads)

    def reprojection_stats(self, state):
        """kbo_reprojection_stats: per camera [n, mean_u, mean_v, std_u, std_v, rmse] (CameraCalibrator.hpp:368-411)"""
        st = np.ascontiguousarray(state, dtype=np.float64)
        out = np.zeros((self.P.n_cams, 6))
        lib().kbo_reprojection_stats(C.byref(self.P), _d(st), _d(out))
        return out

    def term_dense(self, state, view, k):
        st = np.ascontiguousarray(state, dtype=np.float64)
        J = np.zeros((2, self.ncols))
        e = np.zeros(2)
        chi2 = lib().kbo_term_dense(C.byref(self.P), _d(st), view, k, _d(e), _d(J), self.ncols)
        return chi2, e, J

    def dense_jacobian(self, state):
        """Full J (2Nc x ncols) and e for small problems (test use)."""
        rows = []
        es = []
        for v in range(self.prob.n_views):
            nk = self.prob.view_offset[v + 1] - self.prob.view_offset[v]
            for k in range(nk):
                _, e, J = self.term_dense(state, v, k)
                rows.append(J)
                es.append(e)
        return np.concatenate(rows, axis=0), np.concatenate(es)

    def arrow(self, state, nthreads=1, via_ccs=True):
        """Normal-equation blocks (J^T J, rhs = -J^T e) in canonical order."""
        F, Cc = self.prob.n_frames, self.C
        out = dict(Hff=np.zeros((F, 6, 6)), Hfc=np.zeros((F, 6, Cc)), Hcc=np.zeros((Cc, Cc)), gf=np.zeros((F, 6)),
                   gc=np.zeros(Cc))
        A = _Arrow(Cc, F, _d(out["Hff"]), _d(out["Hfc"]), _d(out["Hcc"]), _d(out["gf"]), _d(out["gc"]), 0.0)
        st = np.ascontiguousarray(state, dtype=np.float64)
        rhs = np.zeros(self.ncols)
        jt = lib().kbo_jt_create(C.byref(self.P))
        lib().kbo_jt_build(jt, _d(st), nthreads, _d(rhs))
        lib().kbo_jt_normal_arrow(jt, nthreads, C.byref(A))
        out["nnz"] = lib().kbo_jt_nnz(jt)
        lib().kbo_jt_destroy(jt)
        out["cost"] = A.cost
        out["rhs"] = rhs
        out["_A"] = A
        return out

    def solve(self, arrow, conditioner=0.0, nthreads=1, dense=False):
        dx = np.zeros(self.ncols)
        if dense:
            ok = lib().kbo_dense_solve(C.byref(arrow["_A"]), conditioner, _d(dx))
        else:
            ok = lib().kbo_arrow_solve(C.byref(arrow["_A"]), conditioner, nthreads, _d(dx))
        return bool(ok), dx

    def solve_marginal(self, arrow, opts=None):
        """calibration::LinearSolver::solve on the arrow system: (ok, dx, info) with the scaled SVD of Omega."""
        opts = opts or marg_opts(2 * self.prob.n_corners)
        dx = np.zeros(self.ncols)
        buf = _InfoBuf(self.C)
        ok = lib().kbo_arrow_solve_ex(C.byref(arrow["_A"]), 0.0, 1, _d(dx), C.byref(opts), C.byref(buf.s))
        return bool(ok), dx, buf.result()

    def solve_pcg(self, arrow, conditioner=0.0, tolerance=1e-6, max_iterations=-1, absolute_tolerance=True,
                  prev_residual=-1.0):
        """sparse_block_matrix LinearSolverPCG::solve on the arrow system: (ok, dx, info)."""
        sizes = np.ascontiguousarray(pcg_camera_blocks(self.prob.cam_model), dtype=np.int32)
        dx = np.zeros(self.ncols)
        o = _PcgOpts(tolerance, max_iterations, int(absolute_tolerance), prev_residual)
        info = _PcgInfo()
        ok = lib().kbo_arrow_pcg(C.byref(arrow["_A"]), conditioner, sizes.size, _i(sizes), C.byref(o), _d(dx),
                                 C.byref(info))
        return bool(ok), dx, dict(iterations=info.iterations, residual=info.residual, d0=info.d0)

    def schur_partial(self, arrow, conditioner, f0, f1):
        S = np.zeros((self.C, self.C))
        b = np.zeros(self.C)
        ok = C.c_int(1)
        lib().kbo_arrow_schur_partial(C.byref(arrow["_A"]), conditioner, f0, f1, _d(S), _d(b), C.byref(ok))
        return bool(ok.value), S, b

    def apply_update(self, state, dx):
        st = np.array(state, dtype=np.float64, copy=True)
        dX = lib().kbo_apply_update(C.byref(self.P), _d(st), _d(np.ascontiguousarray(dx, dtype=np.float64)))
        return st, dX

    def optimize(self, state, policy="lm", lambda0=10.0, max_iterations=200, eps_x=1e-3, eps_j=1.0, nthreads=1,
                 trace_cap=1000, marg=None):
        """Optimizer2::optimize; marg (a marg_opts()) selects calibration::LinearSolver, then res["solve_info"] is
        the last solve's scaled SVD and res["analyze_info"] LinearSolver::analyzeMarginal's."""
        st = np.array(state, dtype=np.float64, copy=True)
        o = _Options(0 if policy == "lm" else 1, lambda0, max_iterations, eps_x, eps_j, nthreads)
        if marg is not None:
            si, ai = _InfoBuf(self.C), _InfoBuf(self.C)
            o.marg = C.pointer(marg)
            o.solve_info = C.pointer(si.s)
            o.analyze_info = C.pointer(ai.s)
        srv = _Srv()
        tr = np.zeros((trace_cap, 4))
        n = lib().kbo_optimize(C.byref(self.P), _d(st), C.byref(o), C.byref(srv), _d(tr), trace_cap)
        res = {f: getattr(srv, f) for f, _ in _Srv._fields_}
        res["trace"] = tr[:n].copy()
        if marg is not None:
            res["solve_info"] = si.result()
            res["analyze_info"] = ai.result()
        return st, res

    def time_gn(self, state, n_iter, nthreads):
        st = np.array(state, dtype=np.float64, copy=True)
        return lib().kbo_time_gn(C.byref(self.P), _d(st), n_iter, nthreads)


def sym_eig(A):
    """kbo_sym_eig: (w sorted by |w| descending, V with eigenvectors in columns, sweeps)."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    n = A.shape[0]
    w, V = np.zeros(n), np.zeros((n, n))
    sw = lib().kbo_sym_eig(n, _d(A), _d(w), _d(V))
    return w, V, sw


def marginal_solve(S, b, hdiag, opts):
    """kbo_marginal_solve on a reduced system: (x, info)."""
    Cc = S.shape[0]
    x = np.zeros(Cc)
    buf = _InfoBuf(Cc)
    hd = np.ascontiguousarray(hdiag if hdiag is not None else np.ones(Cc), dtype=np.float64)
    lib().kbo_marginal_solve(Cc, _d(np.ascontiguousarray(S, dtype=np.float64)),
                             _d(np.ascontiguousarray(b, dtype=np.float64)), _d(hd), C.byref(opts), _d(x),
                             C.byref(buf.s))
    return x, buf.result()


def axis_angle2quat(a):
    q = np.zeros(4)
    lib().kbo_axis_angle2quat(_d(np.ascontiguousarray(a, dtype=np.float64)), _d(q))
    return q


def quat2axis_angle(q):
    a = np.zeros(3)
    lib().kbo_quat2axis_angle(_d(np.ascontiguousarray(q, dtype=np.float64)), _d(a))
    return a


def update_quat(q, dq):
    out = np.zeros(4)
    lib().kbo_update_quat(_d(np.ascontiguousarray(q, dtype=np.float64)), _d(np.ascontiguousarray(dq, dtype=np.float64)),
                          _d(out))
    return out


def quat2r(q):
    R = np.zeros(9)
    lib().kbo_quat2r(_d(np.ascontiguousarray(q, dtype=np.float64)), _d(R))
    return R.reshape(3, 3)


def r2quat(R):
    q = np.zeros(4)
    lib().kbo_r2quat(_d(np.ascontiguousarray(R, dtype=np.float64).reshape(-1)), _d(q))
    return q


def project(model, intr, p):
    """returns (valid, y[2], Jp[2,3], Ji[2,MAX_INTR])."""
    y = np.zeros(2)
    Jp = np.zeros(6)
    Ji = np.zeros(20)
    ok = lib().kbo_project(int(model), _d(np.ascontiguousarray(intr, dtype=np.float64)),
                           _d(np.ascontiguousarray(p, dtype=np.float64)), _d(y), _d(Jp), _d(Ji))
    return bool(ok), y, Jp.reshape(2, 3), Ji.reshape(2, 10)


# ------------------------------------------------------------------------------------------------
# configs[4]: B-spline pose trajectory + IMU (oracle/kb_oracle_spline.c)
# ------------------------------------------------------------------------------------------------
class _SpProblem(C.Structure):
    _fields_ = [("order", C.c_int), ("n_knots", C.c_int), ("knots", dp), ("n_cams", C.c_int), ("n_target", C.c_int),
                ("cam_model", ip), ("target", dp), ("n_frames", C.c_int), ("frame_time", dp), ("n_views", C.c_int),
                ("n_corners", C.c_int), ("view_frame", ip), ("view_cam", ip), ("view_offset", ip),
                ("corner_id", ip), ("y", dp), ("n_imu", C.c_int), ("imu_time", dp), ("imu_gyro", dp),
                ("imu_acc", dp), ("sigma_gyro", C.c_double), ("sigma_acc", C.c_double), ("motion_W", dp),
                ("motion_order", C.c_int), ("n_pos", C.c_int), ("pos_time", dp), ("pos_prior", dp),
                ("pos_invR", dp)]


class _SpSystem(C.Structure):
    _fields_ = [("C", C.c_int), ("K", C.c_int), ("order", C.c_int), ("Hcc", dp), ("Hsc", dp), ("Hband", dp),
                ("gc", dp), ("gs", dp), ("cost", C.c_double)]


def _sp_lib():
    L = lib()
    if not getattr(L, "_sp_ready", False):
        for f in ("kbo_sp_eval_cost", "kbo_sp_reproj_dense", "kbo_sp_imu_dense", "kbo_sp_apply_update",
                  "kbo_sp_time_gn", "kbo_sp_motion_cost", "kbo_sp_pos_dense", "kbo_sp_pos_cost"):
            getattr(L, f).restype = C.c_double
        L.kbo_bspline_weights.argtypes = [C.c_int, dp, C.c_int, C.c_double, C.c_int, dp]
        L.kbo_bspline_basis.argtypes = [C.c_int, dp, C.c_int, dp]
        L._sp_ready = True
    return L


def bspline_weights(order, knots, t, deriv):
    kn = np.ascontiguousarray(knots, dtype=np.float64)
    w = np.zeros(order)
    b = _sp_lib().kbo_bspline_weights(order, _d(kn), kn.size, C.c_double(t), deriv, _d(w))
    return b, w


def rv_to_C(a):
    Cm = np.zeros(9)
    _sp_lib().kbo_rv_to_C(_d(np.ascontiguousarray(a, dtype=np.float64)), _d(Cm))
    return Cm.reshape(3, 3)


def rv_S(a):
    S = np.zeros(9)
    _sp_lib().kbo_rv_S(_d(np.ascontiguousarray(a, dtype=np.float64)), _d(S))
    return S.reshape(3, 3)


def rv_dSv(a, v):
    D = np.zeros(9)
    _sp_lib().kbo_rv_dSv(_d(np.ascontiguousarray(a, dtype=np.float64)), _d(np.ascontiguousarray(v, dtype=np.float64)),
                         _d(D))
    return D.reshape(3, 3)


class SplineOracle:
    """configs[4] restatement over one SplineProblem (kalibr_amd/synth.py)."""

    def __init__(self, prob, motion_W=None, motion_order=2, position_priors=None):
        """motion_W (6 x 6, optional): add a BSplineMotionError of that weight and derivative order.
        position_priors (optional): (times [n], priors [n][3], N [n][3][3] covariances) -- ErrorTermEuclidean terms
        on the spline position p(t_k) with invR = N^-1, as the reference's first constructor sets it."""
        self.prob = prob
        k = self._keep = dict(
            knots=np.ascontiguousarray(prob.knots, dtype=np.float64),
            cam_model=np.ascontiguousarray(prob.cam_model, dtype=np.int32),
            target=np.ascontiguousarray(prob.target, dtype=np.float64),
            frame_time=np.ascontiguousarray(prob.frame_time, dtype=np.float64),
            view_frame=np.ascontiguousarray(prob.view_frame, dtype=np.int32),
            view_cam=np.ascontiguousarray(prob.view_cam, dtype=np.int32),
            view_offset=np.ascontiguousarray(prob.view_offset, dtype=np.int32),
            corner_id=np.ascontiguousarray(prob.corner_id, dtype=np.int32),
            y=np.ascontiguousarray(prob.y, dtype=np.float64),
            imu_time=np.ascontiguousarray(prob.imu_time, dtype=np.float64),
            imu_gyro=np.ascontiguousarray(prob.imu_gyro, dtype=np.float64),
            imu_acc=np.ascontiguousarray(prob.imu_acc, dtype=np.float64))
        self.P = _SpProblem(prob.order, k["knots"].size, _d(k["knots"]), prob.n_cams, k["target"].shape[0],
                            _i(k["cam_model"]), _d(k["target"]), prob.n_frames, _d(k["frame_time"]), prob.n_views,
                            prob.n_corners, _i(k["view_frame"]), _i(k["view_cam"]), _i(k["view_offset"]),
                            _i(k["corner_id"]), _d(k["y"]), prob.n_imu, _d(k["imu_time"]), _d(k["imu_gyro"]),
                            _d(k["imu_acc"]), prob.sigma_gyro, prob.sigma_acc, None, int(motion_order))
        if motion_W is not None:
            k["motion_W"] = np.ascontiguousarray(motion_W, dtype=np.float64).reshape(6, 6)
            self.P.motion_W = _d(k["motion_W"])
        self.P.n_pos = 0
        if position_priors is not None:
            t, pr, N = position_priors
            k["pos_time"] = np.ascontiguousarray(t, dtype=np.float64).reshape(-1)
            k["pos_prior"] = np.ascontiguousarray(pr, dtype=np.float64).reshape(-1, 3)
            k["pos_invR"] = np.ascontiguousarray(np.linalg.inv(np.asarray(N, dtype=np.float64).reshape(-1, 3, 3)))
            self.P.n_pos = k["pos_time"].size
            self.P.pos_time, self.P.pos_prior, self.P.pos_invR = _d(k["pos_time"]), _d(k["pos_prior"]), _d(k["pos_invR"])
        L = _sp_lib()
        self.C = L.kbo_sp_cam_cols(C.byref(self.P))
        self.K = L.kbo_sp_num_coeffs(C.byref(self.P))
        self.ncols = L.kbo_sp_total_cols(C.byref(self.P))
        self.nstate = L.kbo_sp_state_size(C.byref(self.P))
        assert self.C == prob.cam_cols and self.K == prob.n_coeffs and self.nstate == prob.state_init.size

    def cost(self, state, nthreads=1):
        st = np.ascontiguousarray(state, dtype=np.float64)
        return _sp_lib().kbo_sp_eval_cost(C.byref(self.P), _d(st), nthreads)

    def reproj_dense(self, state, view, k):
        st = np.ascontiguousarray(state, dtype=np.float64)
        e, J = np.zeros(2), np.zeros((2, self.ncols))
        _sp_lib().kbo_sp_reproj_dense(C.byref(self.P), _d(st), view, k, _d(e), _d(J), self.ncols)
        return e, J

    def imu_dense(self, state, m):
        st = np.ascontiguousarray(state, dtype=np.float64)
        e, J = np.zeros(6), np.zeros((6, self.ncols))
        _sp_lib().kbo_sp_imu_dense(C.byref(self.P), _d(st), m, _d(e), _d(J), self.ncols)
        return e, J

    def system(self, state, nthreads=1):
        st = np.ascontiguousarray(state, dtype=np.float64)
        Cc, K, o = self.C, self.K, self.prob.order
        out = dict(Hcc=np.zeros((Cc, Cc)), Hsc=np.zeros((6 * K, Cc)), Hband=np.zeros((K, o, 6, 6)), gc=np.zeros(Cc),
                   gs=np.zeros(6 * K))
        A = _SpSystem(Cc, K, o, _d(out["Hcc"]), _d(out["Hsc"]), _d(out["Hband"]), _d(out["gc"]), _d(out["gs"]), 0.0)
        _sp_lib().kbo_sp_build(C.byref(self.P), _d(st), nthreads, C.byref(A))
        out["cost"] = A.cost
        out["_A"] = A
        return out

    def solve(self, sysd, lam=0.0, dense=False):
        dx = np.zeros(self.ncols)
        f = _sp_lib().kbo_sp_dense_solve if dense else _sp_lib().kbo_sp_solve
        ok = f(C.byref(sysd["_A"]), C.c_double(lam), _d(dx))
        return bool(ok), dx

    def apply_update(self, state, dx):
        st = np.array(state, dtype=np.float64, copy=True)
        dX = _sp_lib().kbo_sp_apply_update(C.byref(self.P), _d(st), _d(np.ascontiguousarray(dx, dtype=np.float64)))
        return st, dX

    def optimize(self, state, policy="gn", lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1.0, nthreads=1,
                 trace_cap=1000):
        st = np.array(state, dtype=np.float64, copy=True)
        o = _Options(0 if policy == "lm" else 1, lambda0, max_iterations, eps_x, eps_j, nthreads)
        srv = _Srv()
        tr = np.zeros((trace_cap, 4))
        n = _sp_lib().kbo_sp_optimize(C.byref(self.P), _d(st), C.byref(o), C.byref(srv), _d(tr), trace_cap)
        res = {f: getattr(srv, f) for f, _ in _Srv._fields_}
        res["trace"] = tr[:n].copy()
        return st, res

    def time_gn(self, state, n_iter, nthreads):
        st = np.array(state, dtype=np.float64, copy=True)
        return _sp_lib().kbo_sp_time_gn(C.byref(self.P), _d(st), n_iter, nthreads)

    def motion_band(self):
        """q[k][d] = int b_k^(m) b_(k+d)^(m) dt (None without a motion term)"""
        q = np.zeros((self.K, self.prob.order))
        return q if _sp_lib().kbo_sp_motion_band(C.byref(self.P), _d(q)) else None

    def pos_dense(self, state, k):
        """ErrorTermEuclidean prior k: e = p(t_k) - prior_k (unwhitened) and its Jacobian rows; returns (chi2, e, J)"""
        st = np.ascontiguousarray(state, dtype=np.float64)
        e, J = np.zeros(3), np.zeros((3, self.ncols))
        c = _sp_lib().kbo_sp_pos_dense(C.byref(self.P), _d(st), k, _d(e), _d(J), self.ncols)
        return c, e, J

    def pos_cost(self, state):
        st = np.ascontiguousarray(state, dtype=np.float64)
        return _sp_lib().kbo_sp_pos_cost(C.byref(self.P), _d(st))

    def motion_cost(self, state):
        st = np.ascontiguousarray(state, dtype=np.float64)
        return _sp_lib().kbo_sp_motion_cost(C.byref(self.P), _d(st))
