"""ctypes binding of the C-ABI in include/kalibr_hip.h (libkalibr_hip.so, built in-tree).

There is no CPU fallback: if the shared library or a HIP device is missing, every entry point
raises.  The library is loaded from this package directory so the GPU box loads the in-tree build.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KB_DIAG_LIB=1 selects the diagnostic build (libkalibr_hip_stamps.so: stop points, timelines) for the tools
LIB_PATH = os.path.join(_HERE, "libkalibr_hip_stamps.so" if os.environ.get("KB_DIAG_LIB") == "1" else "libkalibr_hip.so")
# KB_VARIANT_LIB=<name>: a measurement variant built by kalibr_amd/build.py build_variant (tools only)
if os.environ.get("KB_VARIANT_LIB"):
    LIB_PATH = os.path.join(_HERE, "libkalibr_hip_%s.so" % os.environ["KB_VARIANT_LIB"])
_lib = None

dp = C.POINTER(C.c_double)

# every symbol declared in include/kalibr_hip.h
EXPORTS = [
    "kb_create", "kb_destroy", "kb_last_error", "kb_upload_observations", "kb_set_state", "kb_set_state_flat",
    "kb_get_state_flat", "kb_state_size", "kb_num_cols", "kb_camera_cols", "kb_eval_cost", "kb_build",
    "kb_set_constant_conditioner", "kb_set_conditioner", "kb_solve", "kb_get_rhs", "kb_rhs_jtj_rhs", "kb_reprojection_error_stats", "kb_apply_update", "kb_revert", "kb_get_normal_blocks",
    "kb_optimize", "kb_get_trace", "kb_run_gn_iterations", "kb_gn_prepare", "kb_gn_launch", "kb_build_kernel_stats",
    "kb_build_kernel_name", "kb_comm_get_unique_id", "kb_gn_pass_times", "kb_append_frames", "kb_drop_last_frames", "kb_optimize_marginal", "kb_optimize_marginal_analyze",
    "kb_comm_init", "kb_comm_init_local", "kb_comm_direct", "kb_xar_export", "kb_xar_test", "kb_selftest_mfma", "kb_solve_marginal", "kb_analyze_marginal",
    # block-Jacobi PCG (LinearSolverPCG)
    "kb_set_linear_solver", "kb_pcg_init", "kb_get_pcg_info",
    # configs[4]: B-spline pose trajectory + IMU
    "kb_sp_create", "kb_sp_destroy", "kb_sp_upload", "kb_sp_state_size", "kb_sp_num_cols", "kb_sp_camera_cols",
    "kb_sp_set_state", "kb_sp_get_state", "kb_sp_eval_cost", "kb_sp_build", "kb_sp_set_constant_conditioner",
    "kb_sp_solve", "kb_sp_get_rhs", "kb_sp_apply_update", "kb_sp_revert", "kb_sp_get_system", "kb_sp_optimize",
    "kb_sp_get_trace", "kb_sp_run_gn_iterations", "kb_sp_kernel_stats", "kb_sp_assemble_stats", "kb_sp_set_motion_error",
    "kb_sp_set_position_priors",
]


class KbError(RuntimeError):
    pass


class SpLayout(C.Structure):
    _fields_ = [("n_cams", C.c_int32), ("n_target", C.c_int32), ("cam_model", C.POINTER(C.c_int32)),
                ("target_points", dp), ("order", C.c_int32), ("n_knots", C.c_int32), ("knots", dp),
                ("sigma_gyro", C.c_double), ("sigma_acc", C.c_double), ("device", C.c_int32)]


class Layout(C.Structure):
    _fields_ = [("n_cams", C.c_int32), ("n_frames", C.c_int32), ("n_target", C.c_int32),
                ("cam_model", C.POINTER(C.c_int32)), ("target_points", dp), ("device", C.c_int32)]


class OptimizerOptions(C.Structure):
    _fields_ = [("policy", C.c_int32), ("lambda_init", C.c_double), ("max_iterations", C.c_int32),
                ("convergence_dx", C.c_double), ("convergence_dj", C.c_double), ("sync_every", C.c_int32),
                ("use_graph", C.c_int32)]


class Solution(C.Structure):
    _fields_ = [("J_start", C.c_double), ("J_final", C.c_double), ("dx_final", C.c_double), ("dj_final", C.c_double),
                ("iterations", C.c_int32), ("failed_iterations", C.c_int32), ("linear_solver_failure", C.c_int32),
                ("passes", C.c_int32), ("graphed", C.c_int32)]


class MarginalOptions(C.Structure):
    _fields_ = [("column_scaling", C.c_int32), ("eps_norm", C.c_double), ("eps_svd", C.c_double),
                ("svd_tol", C.c_double)]


class MarginalInfo(C.Structure):
    _fields_ = [("rank", C.c_int32), ("sweeps", C.c_int32), ("tolerance", C.c_double), ("sv_gap", C.c_double),
                ("sv_log2_sum", C.c_double)]


class PcgOptions(C.Structure):
    _fields_ = [("tolerance", C.c_double), ("max_iterations", C.c_int32), ("absolute_tolerance", C.c_int32)]


class PcgInfo(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("residual", C.c_double), ("d0", C.c_double)]


SOLVER_SCHUR, SOLVER_PCG, SOLVER_PCG_SCHUR = 0, 1, 2

DBL_EPS = float(np.finfo(float).eps)


def marginal_options(column_scaling=True, eps_norm=DBL_EPS, eps_svd=1e-6, svd_tol=-1.0):
    """LinearSolverOptions as CalibrateCameras sets them (CalibrateCameras.cpp:263-267)."""
    return MarginalOptions(int(column_scaling), eps_norm, eps_svd, svd_tol)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise KbError(f"{LIB_PATH} missing: run __graft_entry__.build() (the HIP path has no fallback)")
        L = C.CDLL(LIB_PATH)
        L.kb_create.restype = C.c_void_p
        L.kb_create.argtypes = [C.POINTER(Layout)]
        L.kb_destroy.argtypes = [C.c_void_p]
        L.kb_last_error.restype = C.c_char_p
        for name in EXPORTS:
            fn = getattr(L, name)
            if name not in ("kb_create", "kb_destroy", "kb_last_error", "kb_sp_create", "kb_sp_destroy"):
                fn.restype = C.c_int
        L.kb_upload_observations.argtypes = [C.c_void_p, C.c_int32, C.c_int32, dp, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p]
        L.kb_set_state_flat.argtypes = [C.c_void_p, dp]
        L.kb_get_state_flat.argtypes = [C.c_void_p, dp]
        L.kb_set_state.argtypes = [C.c_void_p, dp, dp, dp, dp]
        for n in ("kb_state_size", "kb_num_cols", "kb_camera_cols", "kb_revert"):
            getattr(L, n).argtypes = [C.c_void_p]
        L.kb_eval_cost.argtypes = [C.c_void_p, dp]
        L.kb_build.argtypes = [C.c_void_p, C.c_int]
        L.kb_set_constant_conditioner.argtypes = [C.c_void_p, C.c_double]
        L.kb_set_conditioner.argtypes = [C.c_void_p, dp]
        L.kb_solve.argtypes = [C.c_void_p, dp, C.POINTER(C.c_int)]
        L.kb_get_rhs.argtypes = [C.c_void_p, dp]
        L.kb_rhs_jtj_rhs.argtypes = [C.c_void_p, dp]
        L.kb_reprojection_error_stats.argtypes = [C.c_void_p, dp]
        L.kb_apply_update.argtypes = [C.c_void_p, dp, dp]
        L.kb_get_normal_blocks.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp]
        L.kb_optimize.argtypes = [C.c_void_p, C.POINTER(OptimizerOptions), C.POINTER(Solution)]
        L.kb_get_trace.argtypes = [C.c_void_p, dp, C.c_int32]
        L.kb_run_gn_iterations.argtypes = [C.c_void_p, C.c_int32, dp]
        L.kb_gn_prepare.argtypes = [C.c_void_p, C.c_int32]
        L.kb_gn_launch.argtypes = [C.c_void_p, C.c_int32, dp]
        L.kb_build_kernel_name.argtypes = [C.c_void_p, C.c_char_p, C.c_int32]
        L.kb_build_kernel_stats.argtypes = [C.c_void_p, dp, dp, dp]
        L.kb_gn_pass_times.argtypes = [C.c_void_p, C.c_int32, dp, dp]
        L.kb_append_frames.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, dp, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, dp]
        L.kb_drop_last_frames.argtypes = [C.c_void_p, C.c_int32]
        L.kb_comm_get_unique_id.argtypes = [C.c_void_p]
        L.kb_comm_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]
        L.kb_comm_init_local.argtypes = [C.POINTER(C.c_void_p), C.c_int32]
        L.kb_comm_direct.argtypes = [C.c_void_p]
        L.kb_xar_export.argtypes = [C.c_void_p, C.c_void_p]
        L.kb_xar_test.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_int32)]
        L.kb_selftest_mfma.argtypes = [dp]
        L.kb_set_linear_solver.argtypes = [C.c_void_p, C.c_int32, C.POINTER(PcgOptions)]
        L.kb_pcg_init.argtypes = [C.c_void_p]
        L.kb_get_pcg_info.argtypes = [C.c_void_p, C.POINTER(PcgInfo)]
        L.kb_solve_marginal.argtypes = [C.c_void_p, C.POINTER(MarginalOptions), dp, C.POINTER(C.c_int),
                                        C.POINTER(MarginalInfo), dp, dp]
        L.kb_analyze_marginal.argtypes = [C.c_void_p, C.POINTER(MarginalOptions), C.POINTER(MarginalInfo), dp, dp]
        L.kb_sp_create.restype = C.c_void_p
        L.kb_sp_create.argtypes = [C.POINTER(SpLayout)]
        L.kb_sp_destroy.argtypes = [C.c_void_p]
        L.kb_sp_upload.argtypes = [C.c_void_p, C.c_int32, dp, C.c_int32, C.c_int32, dp, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_int32, dp, dp, dp]
        for n in ("kb_sp_state_size", "kb_sp_num_cols", "kb_sp_camera_cols", "kb_sp_build", "kb_sp_revert"):
            getattr(L, n).argtypes = [C.c_void_p]
        L.kb_sp_set_state.argtypes = [C.c_void_p, dp]
        L.kb_sp_get_state.argtypes = [C.c_void_p, dp]
        L.kb_sp_eval_cost.argtypes = [C.c_void_p, dp]
        L.kb_sp_set_constant_conditioner.argtypes = [C.c_void_p, C.c_double]
        L.kb_sp_solve.argtypes = [C.c_void_p, dp, C.POINTER(C.c_int)]
        L.kb_sp_get_rhs.argtypes = [C.c_void_p, dp]
        L.kb_sp_apply_update.argtypes = [C.c_void_p, dp, dp]
        L.kb_sp_get_system.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp]
        L.kb_sp_optimize.argtypes = [C.c_void_p, C.POINTER(OptimizerOptions), C.POINTER(Solution)]
        L.kb_sp_get_trace.argtypes = [C.c_void_p, dp, C.c_int32]
        L.kb_sp_run_gn_iterations.argtypes = [C.c_void_p, C.c_int32, dp]
        L.kb_sp_kernel_stats.argtypes = [C.c_void_p, C.c_int32, dp, dp]
        L.kb_sp_assemble_stats.argtypes = [C.c_void_p, C.c_int32, dp, dp]
        L.kb_sp_set_motion_error.argtypes = [C.c_void_p, dp, C.c_int32]
        L.kb_sp_set_position_priors.argtypes = [C.c_void_p, C.c_int32, dp, dp, dp]
        _lib = L
    return _lib


def _check(rc):
    if rc < 0:
        raise KbError(lib().kb_last_error().decode())
    return rc


def _d(a):
    return a.ctypes.data_as(dp)


def selftest_mfma():
    err = C.c_double(0.0)
    _check(lib().kb_selftest_mfma(C.byref(err)))
    return err.value


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    _check(lib().kb_comm_get_unique_id(buf))
    return buf.raw


class Solver:
    """One device handle = one LinearSystemSolver instance over a synthetic/real observation set."""

    def __init__(self, prob, device=0):
        self.prob = prob
        self._cm = np.ascontiguousarray(prob.cam_model, dtype=np.int32)
        self._tg = np.ascontiguousarray(prob.target, dtype=np.float64)
        lay = Layout(prob.n_cams, prob.n_frames, self._tg.shape[0], self._cm.ctypes.data_as(C.POINTER(C.c_int32)),
                     _d(self._tg), device)
        h = lib().kb_create(C.byref(lay))
        if not h:
            raise KbError(lib().kb_last_error().decode())
        self.h = C.c_void_p(h)
        y = np.ascontiguousarray(prob.y, dtype=np.float64)
        cid = np.ascontiguousarray(prob.corner_id, dtype=np.uint16)
        vo = np.ascontiguousarray(prob.view_offset, dtype=np.uint32)
        vf = np.ascontiguousarray(prob.view_frame, dtype=np.uint32)
        vc = np.ascontiguousarray(prob.view_cam, dtype=np.uint8)
        _check(lib().kb_upload_observations(self.h, prob.n_views, prob.n_corners, _d(y), cid.ctypes.data,
                                            vo.ctypes.data, vf.ctypes.data, vc.ctypes.data))
        self.S = lib().kb_state_size(self.h)
        self.ncols = lib().kb_num_cols(self.h)
        self.C = lib().kb_camera_cols(self.h)

    def close(self):
        if getattr(self, "h", None):
            lib().kb_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- LinearSystemSolver-like surface --
    def set_state(self, state):
        st = np.ascontiguousarray(state, dtype=np.float64)
        assert st.shape[0] == self.S
        _check(lib().kb_set_state_flat(self.h, _d(st)))

    def get_state(self):
        st = np.zeros(self.S)
        _check(lib().kb_get_state_flat(self.h, _d(st)))
        return st

    def eval_cost(self):
        J = C.c_double()
        _check(lib().kb_eval_cost(self.h, C.byref(J)))
        return J.value

    def build(self, use_mestimator=True):
        _check(lib().kb_build(self.h, int(use_mestimator)))

    def set_constant_conditioner(self, diag):
        _check(lib().kb_set_constant_conditioner(self.h, float(diag)))

    def set_conditioner(self, diag):
        """setConditioner: diag (canonical column order), squares added to the diagonal of kb_solve's system."""
        d = np.ascontiguousarray(diag, dtype=np.float64)
        assert d.shape == (self.ncols,)
        _check(lib().kb_set_conditioner(self.h, _d(d)))

    def solve(self):
        dx = np.zeros(self.ncols)
        ok = C.c_int(0)
        _check(lib().kb_solve(self.h, _d(dx), C.byref(ok)))
        return bool(ok.value), dx

    def set_linear_solver(self, kind="schur", tolerance=1e-6, max_iterations=-1, absolute_tolerance=True):
        """kind "schur" (direct, default), "pcg" (LinearSolverPCG: block-Jacobi PCG on the full system) or "pcg_schur"
        (the same PCG on the camera-block Schur complement, frames eliminated exactly) for solve()."""
        k = {"schur": SOLVER_SCHUR, "pcg": SOLVER_PCG, "pcg_schur": SOLVER_PCG_SCHUR}[kind]
        o = PcgOptions(float(tolerance), int(max_iterations), int(absolute_tolerance))
        _check(lib().kb_set_linear_solver(self.h, k, C.byref(o)))

    def pcg_init(self):
        _check(lib().kb_pcg_init(self.h))

    def pcg_info(self):
        i = PcgInfo()
        _check(lib().kb_get_pcg_info(self.h, C.byref(i)))
        return dict(iterations=i.iterations, residual=i.residual, d0=i.d0)

    def _minfo(self, inf, sv, V):
        return dict(rank=inf.rank, sweeps=inf.sweeps, tol=inf.tolerance, gap=inf.sv_gap, log2sum=inf.sv_log2_sum,
                    sv=sv, V=V)

    def solve_marginal(self, opts=None):
        """calibration::LinearSolver::solveSystem after build(): (ok, dx, info with the scaled SVD)."""
        opts = opts or marginal_options()
        dx = np.zeros(self.ncols)
        sv, V = np.zeros(self.C), np.zeros((self.C, self.C))
        ok = C.c_int(0)
        inf = MarginalInfo()
        _check(lib().kb_solve_marginal(self.h, C.byref(opts), _d(dx), C.byref(ok), C.byref(inf), _d(sv), _d(V)))
        return bool(ok.value), dx, self._minfo(inf, sv, V)

    def analyze_marginal(self, opts=None):
        """LinearSolver::analyzeMarginal: unscaled SVD of the last built system."""
        opts = opts or marginal_options()
        sv, V = np.zeros(self.C), np.zeros((self.C, self.C))
        inf = MarginalInfo()
        _check(lib().kb_analyze_marginal(self.h, C.byref(opts), C.byref(inf), _d(sv), _d(V)))
        return self._minfo(inf, sv, V)

    def rhs(self):
        r = np.zeros(self.ncols)
        _check(lib().kb_get_rhs(self.h, _d(r)))
        return r

    def rhs_jtj_rhs(self):
        """kb_rhs_jtj_rhs: rhs^T (J^T J) rhs of the last build"""
        v = C.c_double()
        _check(lib().kb_rhs_jtj_rhs(self.h, C.byref(v)))
        return v.value

    def reprojection_error_stats(self):
        """kb_reprojection_error_stats: per camera [n, mean_u, mean_v, std_u, std_v, rmse] of the current state
        (CameraCalibrator.hpp:368-411; rmse = |sum e| / sqrt(n) as the reference prints it)"""
        out = np.zeros((self.prob.n_cams, 6))
        _check(lib().kb_reprojection_error_stats(self.h, _d(out)))
        return out

    def apply_update(self, dx):
        dX = C.c_double()
        _check(lib().kb_apply_update(self.h, _d(np.ascontiguousarray(dx, dtype=np.float64)), C.byref(dX)))
        return dX.value

    def revert(self):
        _check(lib().kb_revert(self.h))

    def normal_blocks(self):
        Cc = self.C
        F = (self.ncols - Cc) // 6  # the handle's frames (kb_append_frames / kb_drop_last_frames change them)
        out = dict(Hff=np.zeros((F, 6, 6)), Hfc=np.zeros((F, 6, Cc)), gf=np.zeros((F, 6)), Hcc=np.zeros((Cc, Cc)),
                   gc=np.zeros(Cc), cost=np.zeros(1))
        _check(lib().kb_get_normal_blocks(self.h, _d(out["Hff"]), _d(out["Hfc"]), _d(out["gf"]), _d(out["Hcc"]),
                                          _d(out["gc"]), _d(out["cost"])))
        out["cost"] = float(out["cost"][0])
        return out

    # -- device-resident Optimizer2 --
    def optimize_marginal(self, max_iterations=20, eps_x=1e-3, eps_j=1e-3, opts=None, analyze=False, sync_every=2,
                          use_graph=False):
        """kb_optimize_marginal (the IncrementalEstimator's device loop: GN over the truncated-SVD camera solve);
        analyze: kb_optimize_marginal_analyze, the last build's analyzeMarginal in the same sync.  Returns
        (solution dict, marginal info of the last solve, analyze info or None)."""
        mo = opts or marginal_options()
        o = OptimizerOptions(1, 0.0, max_iterations, eps_x, eps_j, sync_every, int(use_graph))
        s = Solution()
        sv, V = np.zeros(self.C), np.zeros((self.C, self.C))
        inf = MarginalInfo()
        if analyze:
            asv, aV = np.zeros(self.C), np.zeros((self.C, self.C))
            ainf = MarginalInfo()
            _check(lib().kb_optimize_marginal_analyze(self.h, C.byref(o), C.byref(mo), C.byref(s), C.byref(inf),
                                                      _d(sv), _d(V), C.byref(ainf), _d(asv), _d(aV)))
            a = self._minfo(ainf, asv, aV)
        else:
            _check(lib().kb_optimize_marginal(self.h, C.byref(o), C.byref(mo), C.byref(s), C.byref(inf), _d(sv), _d(V)))
            a = None
        res = {f: getattr(s, f) for f, _ in Solution._fields_}
        return res, self._minfo(inf, sv, V), a

    def optimize(self, policy="lm", lambda0=10.0, max_iterations=200, eps_x=1e-3, eps_j=1.0, sync_every=4,
                 use_graph=True):
        o = OptimizerOptions(0 if policy == "lm" else 1, lambda0, max_iterations, eps_x, eps_j, sync_every,
                             int(use_graph))
        s = Solution()
        _check(lib().kb_optimize(self.h, C.byref(o), C.byref(s)))
        res = {f: getattr(s, f) for f, _ in Solution._fields_}
        cap = 2 * max_iterations + 2
        tr = np.zeros((cap, 4))
        n = _check(lib().kb_get_trace(self.h, _d(tr), cap))
        res["trace"] = tr[:n].copy()
        return res

    def run_gn(self, n_iter):
        sec = C.c_double()
        _check(lib().kb_run_gn_iterations(self.h, int(n_iter), C.byref(sec)))
        return sec.value

    def gn_prepare(self, n_iter):
        """loop start + every graph n_iter passes need, captured and uploaded (kb_gn_prepare); True if graphed"""
        return bool(_check(lib().kb_gn_prepare(self.h, int(n_iter))))

    def gn_launch(self, n_iter):
        """the n_iter prepared passes between two stream syncs; returns their wall seconds (kb_gn_launch)"""
        sec = C.c_double()
        _check(lib().kb_gn_launch(self.h, int(n_iter), C.byref(sec)))
        return sec.value

    def build_kernel_name(self):
        buf = C.create_string_buffer(32)
        _check(lib().kb_build_kernel_name(self.h, buf, 32))
        return buf.value.decode()

    def build_kernel_stats(self):
        ms, by, fl = C.c_double(), C.c_double(), C.c_double()
        _check(lib().kb_build_kernel_stats(self.h, C.byref(ms), C.byref(by), C.byref(fl)))
        return ms.value, by.value, fl.value

    def append_frames(self, sub, poses=None):
        """kb_append_frames: the frames of problem `sub` (same rig; its frames numbered from 0) appended in place;
        poses [n_frames][7] default to the frame poses of sub.state_init"""
        y = np.ascontiguousarray(sub.y, dtype=np.float64)
        cid = np.ascontiguousarray(sub.corner_id, dtype=np.uint16)
        vo = np.ascontiguousarray(sub.view_offset, dtype=np.uint32)
        vf = np.ascontiguousarray(sub.view_frame, dtype=np.uint32)
        vc = np.ascontiguousarray(sub.view_cam, dtype=np.uint8)
        so = sub.n_cams * 10 + 7 * (sub.n_cams - 1)  # KB_MAX_INTR = 10
        ps = np.ascontiguousarray(sub.state_init[so:] if poses is None else poses, dtype=np.float64)
        _check(lib().kb_append_frames(self.h, sub.n_frames, sub.n_views, sub.n_corners, _d(y), cid.ctypes.data,
                                      vo.ctypes.data, vf.ctypes.data, vc.ctypes.data, _d(ps)))
        self._resize()

    def drop_last_frames(self, n):
        _check(lib().kb_drop_last_frames(self.h, int(n)))
        self._resize()

    def _resize(self):
        self.S = lib().kb_state_size(self.h)
        self.ncols = lib().kb_num_cols(self.h)

    def gn_pass_times(self, n):
        """(pass_ms [n], build_ms [n]) of n GN passes from the current state, device-timed (kb_gn_pass_times)"""
        pm, bm = np.zeros(n), np.zeros(n)
        _check(lib().kb_gn_pass_times(self.h, int(n), _d(pm), _d(bm)))
        return pm, bm

    def comm_init(self, uid: bytes, nranks, rank):
        buf = C.create_string_buffer(uid, 128)
        _check(lib().kb_comm_init(self.h, buf, int(nranks), int(rank)))

    def xar_export(self):
        """kb_xar_export: this handle's exchange-region IPC handle (64 bytes)."""
        buf = C.create_string_buffer(64)
        _check(lib().kb_xar_export(self.h, buf))
        return buf.raw

    def xar_test(self, nranks, rank, handles: bytes):
        """kb_xar_test: the direct all-reduce's self-test exchange with the peers' exported regions."""
        ok = C.c_int32(0)
        buf = C.create_string_buffer(handles, len(handles))
        _check(lib().kb_xar_test(self.h, int(nranks), int(rank), buf, C.byref(ok)))
        return bool(ok.value)

    def comm_direct(self):
        """kb_comm_direct: the sharded image is all-reduced by k_xar (peers read over xGMI), not a collective."""
        return bool(lib().kb_comm_direct(self.h))


def comm_init_local(solvers):
    """kb_comm_init_local: the solvers (frame shards of one problem, in rank order) exchange in-process; drive each
    one from its own thread afterwards."""
    arr = (C.c_void_p * len(solvers))(*[s.h.value for s in solvers])
    _check(lib().kb_comm_init_local(arr, len(solvers)))


class SplineSolver:
    """One kb_sp handle: the configs[4] spline + IMU system on one MI355X (include/kalibr_hip.h kb_sp_*)."""

    def __init__(self, prob, device=0):
        self.prob = prob
        self._cm = np.ascontiguousarray(prob.cam_model, dtype=np.int32)
        self._tg = np.ascontiguousarray(prob.target, dtype=np.float64)
        self._kn = np.ascontiguousarray(prob.knots, dtype=np.float64)
        lay = SpLayout(prob.n_cams, self._tg.shape[0], self._cm.ctypes.data_as(C.POINTER(C.c_int32)), _d(self._tg),
                       prob.order, self._kn.size, _d(self._kn), prob.sigma_gyro, prob.sigma_acc, device)
        h = lib().kb_sp_create(C.byref(lay))
        if not h:
            raise KbError(lib().kb_last_error().decode())
        self.h = C.c_void_p(h)
        ft = np.ascontiguousarray(prob.frame_time, dtype=np.float64)
        y = np.ascontiguousarray(prob.y, dtype=np.float64)
        cid = np.ascontiguousarray(prob.corner_id, dtype=np.uint16)
        vo = np.ascontiguousarray(prob.view_offset, dtype=np.uint32)
        vf = np.ascontiguousarray(prob.view_frame, dtype=np.uint32)
        vc = np.ascontiguousarray(prob.view_cam, dtype=np.uint8)
        it = np.ascontiguousarray(prob.imu_time, dtype=np.float64)
        ig = np.ascontiguousarray(prob.imu_gyro, dtype=np.float64)
        ia = np.ascontiguousarray(prob.imu_acc, dtype=np.float64)
        _check(lib().kb_sp_upload(self.h, prob.n_frames, _d(ft), prob.n_views, prob.n_corners, _d(y), cid.ctypes.data,
                                  vo.ctypes.data, vf.ctypes.data, vc.ctypes.data, prob.n_imu, _d(it), _d(ig), _d(ia)))
        self.S = lib().kb_sp_state_size(self.h)
        self.ncols = lib().kb_sp_num_cols(self.h)
        self.C = lib().kb_sp_camera_cols(self.h)
        self.K = (self.ncols - self.C) // 6

    def close(self):
        if getattr(self, "h", None):
            lib().kb_sp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_motion_error(self, W, derivative_order=2):
        """BSplineMotionError on the pose spline (W 6 x 6 symmetric; None removes it)."""
        if W is None:
            _check(lib().kb_sp_set_motion_error(self.h, None, 0))
            return
        self._motion_W = np.ascontiguousarray(W, dtype=np.float64).reshape(6, 6)
        _check(lib().kb_sp_set_motion_error(self.h, _d(self._motion_W), int(derivative_order)))

    def set_position_priors(self, times=None, priors=None, N=None):
        """ErrorTermEuclidean priors on the spline position p(t_k) (times [n], priors [n][3], covariances N [n][3][3]);
        no arguments removes them."""
        if times is None:
            _check(lib().kb_sp_set_position_priors(self.h, 0, None, None, None))
            return
        self._pos = (np.ascontiguousarray(times, dtype=np.float64).reshape(-1),
                     np.ascontiguousarray(priors, dtype=np.float64).reshape(-1, 3),
                     np.ascontiguousarray(N, dtype=np.float64).reshape(-1, 3, 3))
        t, pr, n3 = self._pos
        _check(lib().kb_sp_set_position_priors(self.h, t.size, _d(t), _d(pr), _d(n3)))

    def set_state(self, state):
        st = np.ascontiguousarray(state, dtype=np.float64)
        assert st.shape[0] == self.S
        _check(lib().kb_sp_set_state(self.h, _d(st)))

    def get_state(self):
        st = np.zeros(self.S)
        _check(lib().kb_sp_get_state(self.h, _d(st)))
        return st

    def eval_cost(self):
        J = C.c_double()
        _check(lib().kb_sp_eval_cost(self.h, C.byref(J)))
        return J.value

    def build(self):
        _check(lib().kb_sp_build(self.h))

    def set_constant_conditioner(self, diag):
        _check(lib().kb_sp_set_constant_conditioner(self.h, float(diag)))

    def solve(self):
        dx = np.zeros(self.ncols)
        ok = C.c_int(0)
        _check(lib().kb_sp_solve(self.h, _d(dx), C.byref(ok)))
        return bool(ok.value), dx

    def rhs(self):
        r = np.zeros(self.ncols)
        _check(lib().kb_sp_get_rhs(self.h, _d(r)))
        return r

    def apply_update(self, dx=None):
        dX = C.c_double()
        _check(lib().kb_sp_apply_update(self.h, None if dx is None else _d(np.ascontiguousarray(dx, dtype=np.float64)),
                                        C.byref(dX)))
        return dX.value

    def revert(self):
        _check(lib().kb_sp_revert(self.h))

    def system(self):
        Cc, K = self.C, self.K
        out = dict(Hcc=np.zeros((Cc, Cc)), Hsc=np.zeros((6 * K, Cc)), Hband=np.zeros((K, 4, 6, 6)), gc=np.zeros(Cc),
                   gs=np.zeros(6 * K))
        cost = C.c_double()
        _check(lib().kb_sp_get_system(self.h, _d(out["Hcc"]), _d(out["Hsc"]), _d(out["Hband"]), _d(out["gc"]),
                                      _d(out["gs"]), C.byref(cost)))
        out["cost"] = cost.value
        return out

    def optimize(self, policy="gn", lambda0=10.0, max_iterations=20, eps_x=1e-3, eps_j=1.0):
        o = OptimizerOptions(0 if policy == "lm" else 1, lambda0, max_iterations, eps_x, eps_j, 1, 0)
        s = Solution()
        _check(lib().kb_sp_optimize(self.h, C.byref(o), C.byref(s)))
        res = {f: getattr(s, f) for f, _ in Solution._fields_}
        cap = 2 * max_iterations + 2
        tr = np.zeros((cap, 4))
        n = _check(lib().kb_sp_get_trace(self.h, _d(tr), cap))
        res["trace"] = tr[:n].copy()
        return res

    def run_gn(self, n_iter):
        sec = C.c_double()
        _check(lib().kb_sp_run_gn_iterations(self.h, int(n_iter), C.byref(sec)))
        return sec.value

    def kernel_stats(self, n=10):
        ms = np.zeros(6)
        fb = C.c_double()
        _check(lib().kb_sp_kernel_stats(self.h, int(n), _d(ms), C.byref(fb)))
        return dict(frames_ms=ms[0], assemble_ms=ms[1], reduction_ms=ms[2], camsolve_ms=ms[3], update_cost_ms=ms[4],
                    pass_ms=ms[5], frames_bytes=fb.value)

    def assemble_stats(self, n=10):
        """(ms per launch, algorithmic bytes per launch) of the node-assembly kernel k_sp_assemble"""
        ms, b = C.c_double(), C.c_double()
        _check(lib().kb_sp_assemble_stats(self.h, int(n), C.byref(ms), C.byref(b)))
        return ms.value, b.value
