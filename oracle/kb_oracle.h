/*
 * kb_oracle.h -- CPU restatement of the Kalibr2 / aslam_backend Gauss-Newton /
 * Levenberg-Marquardt hot path over camera ReprojectionError terms.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in kalibr_amd/ (the product) may link,
 * import or call this code; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, as the checker / CPU baseline.
 *
 * Pinning: the reference (Eigen/Boost/SuiteSparse C++) cannot be built in this
 * image.  The restatement is pinned by the reference's own
 * known-answer table (sm_kinematics/test/QuaternionTests.cpp:44-59), by its
 * finite-difference Jacobian harnesses (CameraGeometryTestHarness.hpp,
 * ErrorTermTestHarness.hpp) and by its structural identities
 * (H = J^T J, rhs = -J^T e: aslam_backend/test/TestOptimizer.cpp:101-120;
 * solver agreement: LinearSolverTests.cpp:18-63).  See tests/golden/.
 *
 * All citations are relative to /root/reference.
 */
#ifndef KB_ORACLE_H
#define KB_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define KBO_MAX_INTR 10   /* per-camera intrinsic slot stride in the state */
#define KBO_POSE 7        /* q (JPL x,y,z,w) + t */

/* camera models (kalibr2/include/kalibr2/CameraModels.hpp:25-133) */
enum {
  KBO_PINHOLE_RADTAN = 0, /* PinholeProjection<RadialTangentialDistortion>: fu fv cu cv | k1 k2 p1 p2 */
  KBO_OMNI_RADTAN = 1,    /* OmniProjection<RadialTangentialDistortion>: xi fu fv cu cv | k1 k2 p1 p2 */
  KBO_EUCM = 2,           /* ExtendedUnifiedProjection<NoDistortion>: alpha beta fu fv cu cv */
  KBO_OMNI = 3,           /* OmniProjection<NoDistortion>: xi fu fv cu cv */
  KBO_DS = 4,             /* DoubleSphereProjection<NoDistortion>: xi alpha fu fv cu cv */
  KBO_PINHOLE_EQUI = 5,   /* PinholeProjection<EquidistantDistortion>: fu fv cu cv | k1 k2 k3 k4 */
  KBO_PINHOLE_FOV = 6,    /* PinholeProjection<FovDistortion>: fu fv cu cv | w */
  KBO_NUM_MODELS = 7
};

typedef struct {
  int n_cams, n_frames, n_views, n_corners, n_target;
  const int* cam_model;   /* [n_cams] */
  const double* target;   /* [n_target][3] target-frame corner coordinates */
  const int* view_frame;  /* [n_views] */
  const int* view_cam;    /* [n_views] */
  const int* view_offset; /* [n_views+1] corner range of each view */
  const int* corner_id;   /* [n_corners] index into target */
  const double* y;        /* [n_corners][2] measured keypoints */
} kbo_problem;

/* Flat state layout (shared with the device path):
 *   intr  [n_cams][KBO_MAX_INTR]   (projection params then distortion params)
 *   base  [n_cams-1][7]            baseline B_j = T_{c(j+1), c(j)}  (q, t)
 *   frame [n_frames][7]            target pose DV T_f (p_c0 = T_f^-1 * P)
 * Canonical column order of dx / rhs / H:
 *   [intr cam0 | intr cam1 | ... | B_0 (dphi,dt) | ... | frame 0 (dphi,dt) | ...]
 * which is the DV insertion order of CalibrateMultiCameraRig
 * (kalibr2/include/kalibr2/CalibrationTools.hpp:376-428; Optimizer2.cpp:110-124). */
int kbo_model_nintr(int model);
int kbo_state_size(int n_cams, int n_frames);
int kbo_cam_cols(const kbo_problem* P);   /* C = sum nintr + 6 (N-1) */
int kbo_total_cols(const kbo_problem* P); /* C + 6F */

/* --- sm_kinematics restatements (known-answer tested) --- */
void kbo_axis_angle2quat(const double a[3], double q[4]);
void kbo_quat2axis_angle(const double q[4], double a[3]);
void kbo_update_quat(const double q[4], const double dq[3], double out[4]);
void kbo_quat2r(const double q[4], double R[9]);
void kbo_r2quat(const double R[9], double q[4]);

/* --- camera maths: keypoint, dy/dp (2x3), dy/dintrinsics (2 x nintr) --- */
int kbo_project(int model, const double* intr, const double p[3], double y[2], double Jp[6], double Ji[2 * KBO_MAX_INTR]);

/* --- one ReprojectionError term through the expression chain --- */
/* J out: dense row block 2 x total_cols (caller zeroes), e out: y - yhat. returns chi2. */
double kbo_term_dense(const kbo_problem* P, const double* state, int view, int k, double e[2], double* Jrow, int ncols);

/* --- cost (LinearSystemSolver::evaluateError) --- */
double kbo_eval_cost(const kbo_problem* P, const double* state, int nthreads);

/* --- CameraCalibrator::PrintReprojectionErrorStatistics (kalibr2/include/kalibr2/CameraCalibrator.hpp:368-411) ---
 * per camera: the terms flattened view by view in problem order, corners in order (per_view_reprojection_errors_,
 * CameraCalibrator.hpp:140-152), e = y - yhat; sum in order (std::accumulate), mean = sum / n, the sample standard
 * deviation of a second pass (N - 1; 0 for n < 2), "RMSE" = |sum| / sqrt(n).  out[n_cams][6] =
 * [n, mean_u, mean_v, std_u, std_v, rmse]; a camera without terms gets zeros (the reference prints and returns). */
void kbo_reprojection_stats(const kbo_problem* P, const double* state, double* out);

/* --- arrow normal equations --- */
typedef struct {
  int C, F;
  double* Hff; /* [F][36] */
  double* Hfc; /* [F][6*C] row-major 6 x C */
  double* Hcc; /* [C*C] */
  double* gf;  /* [F][6]  rhs = -J^T e */
  double* gc;  /* [C] */
  double cost;
} kbo_arrow;

/* CCS J^T (CompressedColumnJacobianTransposeBuilder restatement) */
typedef struct kbo_jt kbo_jt;
kbo_jt* kbo_jt_create(const kbo_problem* P);
void kbo_jt_destroy(kbo_jt* jt);
/* threaded per-term evaluation into J^T values + _e = -e (buildSystem) then rhs = J^T _e */
void kbo_jt_build(kbo_jt* jt, const double* state, int nthreads, double* rhs);
/* J^T J accumulated into the arrow blocks (what CHOLMOD's A A^T forms) */
void kbo_jt_normal_arrow(kbo_jt* jt, int nthreads, kbo_arrow* A);
long long kbo_jt_nnz(const kbo_jt* jt);

/* Build straight into arrow blocks (same numbers, no CCS) */
void kbo_build_arrow(const kbo_problem* P, const double* state, int nthreads, kbo_arrow* A);

/* Solve (J^T J + lambda^2 I) dx = rhs  (LinearSystemSolver.hpp:33-39: square of the conditioner).
 * Schur onto the camera block.  returns 1 on success, 0 on non-PD. */
int kbo_arrow_solve(const kbo_arrow* A, double conditioner, int nthreads, double* dx);
/* Dense reference solve on the full (small) system, for cross-checking the Schur path. */
int kbo_dense_solve(const kbo_arrow* A, double conditioner, double* dx);
/* Partial Schur quantities of a frame range (for sharding): S_part (C*C), b_part (C) */
void kbo_arrow_schur_partial(const kbo_arrow* A, double conditioner, int f0, int f1, double* S_part, double* b_part, int* ok);

/* --- aslam_incremental_calibration LinearSolver: marginal (camera-block) truncated-SVD solve --- */
#define KBO_JACOBI_MAX_SWEEPS 40
#define KBO_JACOBI_TOL 1.1102230246251565e-16 /* skip |a_pq| <= 2^-53 sqrt|a_pp a_qq| */
typedef struct kbo_marg_opts_s {
  int column_scaling; /* LinearSolverOptions::columnScaling */
  double eps_norm;    /* epsNorm (default DBL_EPSILON) */
  double eps_svd;     /* epsSVD (Kalibr2: 1e-6) */
  double svd_tol;     /* svdTol (-1: rankTol from epsSVD) */
  double n_rows;      /* rows of J (2 x corners): the column-norm tolerance sqrt(n_rows * epsNorm) */
} kbo_marg_opts;
typedef struct kbo_marg_info_s {
  double* sv;  /* [C] singular values, descending */
  double* V;   /* [C*C] row-major, right singular vector j in column j (may be NULL) */
  int rank, sweeps;
  double tol, gap, log2sum; /* svdTolerance, svGap, getSingularValuesLog2Sum */
} kbo_marg_info;
int kbo_sym_eig(int n, const double* A, double* w, double* V);
void kbo_marginal_solve(int C, const double* S, const double* b, const double* hdiag, const kbo_marg_opts* o,
                        double* x, kbo_marg_info* info);
int kbo_arrow_solve_ex(const kbo_arrow* A, double conditioner, int nthreads, double* dx, const kbo_marg_opts* marg,
                       kbo_marg_info* info);

/* --- sparse_block_matrix LinearSolverPCG (block-Jacobi preconditioned CG, linear_solver_pcg.hpp:58-130) --- */
typedef struct kbo_pcg_opts_s {
  double tolerance;       /* _tolerance (default 1e-6): stop when r^T M^-1 r <= tolerance * (r0^T M^-1 r0) */
  int max_iterations;     /* _maxIter (-1: number of rows) */
  int absolute_tolerance; /* _absoluteTolerance (default true): d0 = max(d0, previous _residual) */
  double prev_residual;   /* _residual of the previous solve (-1 after init()) */
} kbo_pcg_opts;
typedef struct kbo_pcg_info_s {
  int iterations;
  double residual; /* _residual = 0.5 r^T M^-1 r at exit */
  double d0;       /* the stopping threshold used */
} kbo_pcg_info;
/* (H + conditioner^2 I) dx = g by PCG with the diagonal design-variable blocks as preconditioner:
 * cam_block_size[n_cam_blocks] partitions the C camera columns; each frame contributes its rotation (3) and
 * translation (3) DV blocks.  Returns 1, or 0 on a singular block / non-positive curvature. */
int kbo_arrow_pcg(const kbo_arrow* A, double conditioner, int n_cam_blocks, const int* cam_block_size,
                  const kbo_pcg_opts* o, double* dx, kbo_pcg_info* info);

/* Optimizer2::applyStateUpdate / revert */
double kbo_apply_update(const kbo_problem* P, double* state, const double* dx);

/* Optimizer2::optimize with LM (LevenbergMarquardtTrustRegionPolicy) or GN */
typedef struct {
  int policy;      /* 0 = levenberg_marquardt, 1 = gauss_newton */
  double lambda0;  /* LM lambdaInit */
  int max_iterations;
  double eps_x, eps_j;
  int nthreads;
  /* calibration::LinearSolver in place of CHOLMOD when marg != NULL (IncrementalEstimator's optimizer);
   * solve_info (optional): the last solve's scaled SVD; analyze_info (optional): LinearSolver::analyzeMarginal
   * after the loop -- unscaled SVD of the last built system, rank kept from the last solve */
  const struct kbo_marg_opts_s* marg;
  struct kbo_marg_info_s* solve_info;
  struct kbo_marg_info_s* analyze_info;
} kbo_options;
typedef struct {
  double J_start, J_final, dx_final, dj_final;
  int iterations, failed_iterations, linear_solver_failure;
} kbo_srv;
/* trace (optional, may be NULL): per loop pass: [J_after, lambda, deltaX, accepted] */
int kbo_optimize(const kbo_problem* P, double* state, const kbo_options* o, kbo_srv* srv, double* trace, int trace_cap);

/* CPU baseline: time n_iter GN iterations (build + solve + update + cost), returns seconds. */
double kbo_time_gn(const kbo_problem* P, double* state, int n_iter, int nthreads);

/* ------------------------------------------------------------------------------------------------
 * configs[4]: continuous-time calibration on a B-spline pose trajectory (kb_oracle_spline.c).
 * Camera i at frame time t_f:  T_ci_w = B_{i-1} ... B_0 * T_c0_b * T_wb(t_f)^-1
 * IMU sample m at t_m:          gyro w_m = w_b(t_m) + b_g,  accel a_m = C_wb^T (p_ddot - g_w) + b_a
 * State:  intr [n_cams][KBO_MAX_INTR] | base [n_cams-1][7] | T_c0_b [7] | b_g [3] | b_a [3] | g_w [3] |
 *         coefficients [K][6] (BSplinePose curve value [p | rotation vector])
 * Columns: [intr | B_j (dphi, dt) | T_c0_b (dphi, dt) | b_g | b_a | g_w | coefficients 6K]
 * ------------------------------------------------------------------------------------------------ */
typedef struct {
  int order;             /* spline order (4 = cubic) */
  int n_knots;
  const double* knots;   /* non-decreasing */
  int n_cams, n_target;
  const int* cam_model;
  const double* target;
  int n_frames;
  const double* frame_time;
  int n_views, n_corners;
  const int* view_frame;  /* views sorted by frame */
  const int* view_cam;
  const int* view_offset;
  const int* corner_id;
  const double* y;
  int n_imu;
  const double* imu_time;
  const double* imu_gyro; /* [n_imu][3] */
  const double* imu_acc;  /* [n_imu][3] */
  double sigma_gyro, sigma_acc;
  /* optional BSplineMotionError (aslam_splines BSplineMotionError.hpp:29-160): cost c^T Q c with
   * Q = curveQuadraticIntegralSparse(W, order) (BSpline.cpp:1585-1622); NULL = no motion term */
  const double* motion_W; /* [6][6] symmetric */
  int motion_order;       /* errorTermOrder (BSplineMotionError default 2: acceleration) */
  /* optional ErrorTermEuclidean priors on the spline position (ErrorTermEuclidean.cpp:9-66 over
   * BSplinePoseDesignVariable::position(t_k), BSplinePoseDesignVariable.cpp:91-103 / BSplineExpressions.cpp:132-149):
   * e_k = p(t_k) - prior_k, chi^2_k = e_k^T invR_k e_k, J = w_j(t_k) [I_3 | 0] on coefficient bidx + j */
  int n_pos;
  const double* pos_time;  /* [n_pos] */
  const double* pos_prior; /* [n_pos][3] */
  const double* pos_invR;  /* [n_pos][3][3] symmetric (the reference's setInvR(N^-1)) */
} kbo_sp_problem;

typedef struct {
  int C, K, order;
  double* Hcc;   /* [C][C] */
  double* Hsc;   /* [6K][C] */
  double* Hband; /* [K][order][6][6]: block (k, k+d) */
  double* gc;    /* [C]  = -J_c^T e */
  double* gs;    /* [6K] */
  double cost;
} kbo_sp_system;

int kbo_bspline_num_coeffs(int order, int n_knots);
void kbo_bspline_basis(int order, const double* knots, int segment, double* M);
/* basis weights of derivative `deriv` at t (BSpline::evalDAndJacobian's B^T u); returns the first
 * coefficient index (bidx) or -1 outside [t_min, t_max] */
int kbo_bspline_weights(int order, const double* knots, int n_knots, double t, int deriv, double* w);
void kbo_rv_to_C(const double a[3], double Cm[9]);
void kbo_rv_S(const double a[3], double S[9]);
void kbo_rv_dSv(const double a[3], const double v[3], double D[9]);
int kbo_sp_state_size(const kbo_sp_problem* P);
int kbo_sp_num_coeffs(const kbo_sp_problem* P);
int kbo_sp_cam_cols(const kbo_sp_problem* P);
int kbo_sp_total_cols(const kbo_sp_problem* P);
double kbo_sp_reproj_dense(const kbo_sp_problem* P, const double* st, int v, int k, double e[2], double* J, int ncols);
double kbo_sp_imu_dense(const kbo_sp_problem* P, const double* st, int m, double e[6], double* J, int ncols);
/* ErrorTermEuclidean prior k: whitening-free residual e = p(t_k) - prior_k and its dense Jacobian rows [3][ncols];
 * returns e^T invR e (0 and e = 0 outside the spline's time range) */
double kbo_sp_pos_dense(const kbo_sp_problem* P, const double* st, int k, double e[3], double* J, int ncols);
double kbo_sp_pos_cost(const kbo_sp_problem* P, const double* st);
double kbo_sp_eval_cost(const kbo_sp_problem* P, const double* st, int nthreads);
int kbo_sp_system_alloc(const kbo_sp_problem* P, kbo_sp_system* A);
void kbo_sp_system_free(kbo_sp_system* A);
void kbo_sp_build(const kbo_sp_problem* P, const double* st, int nthreads, kbo_sp_system* A);
int kbo_sp_solve(const kbo_sp_system* A, double lambda, double* dx);
int kbo_sp_dense_solve(const kbo_sp_system* A, double lambda, double* dx);
double kbo_sp_apply_update(const kbo_sp_problem* P, double* st, const double* dx);
int kbo_sp_optimize(const kbo_sp_problem* P, double* st, const kbo_options* o, kbo_srv* srv, double* trace,
                    int trace_cap);
/* scalar band of the motion quadratic form: q[k][d] = int b_k^(m) b_(k+d)^(m) dt (d = 0..order-1), so that
 * Q_(k,k+d) = q[k][d] W; returns 0 if P has no motion term */
int kbo_sp_motion_band(const kbo_sp_problem* P, double* q);
double kbo_sp_motion_cost(const kbo_sp_problem* P, const double* st);
double kbo_sp_time_gn(const kbo_sp_problem* P, double* st, int n_iter, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
