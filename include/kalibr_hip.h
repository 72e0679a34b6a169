/*
 * kalibr_hip.h -- C-ABI of the MI355X-native batch calibration backend.
 *
 * Drop-in boundary for aslam_backend's LinearSystemSolver plugin surface
 * (aslam_optimizer/aslam_backend/include/aslam/backend/LinearSystemSolver.hpp:16-109,
 * paths relative to the reference repository) specialised to the
 * ReprojectionError<Geometry> terms Kalibr2 builds in CalibrateMultiCameraRig
 * (aslam_offline_calibration/kalibr2/include/kalibr2/CalibrationTools.hpp:376-428).
 *
 * Plain pointers and sizes only; every entry point returns an int status
 * (0 = OK, < 0 = error, message in kb_last_error()).  One handle per optimizer,
 * one HIP stream per handle, calls are not re-entrant (LinearSystemSolver is
 * single-threaded at the API level).
 *
 * State layout (flat doubles, also used by kb_set_state_flat / kb_get_state_flat):
 *   intr  [n_cams][KB_MAX_INTR]   projection params then distortion params
 *   base  [n_cams-1][7]           B_j = T_{c(j+1),c(j)}: JPL quaternion (x,y,z,w) + t
 *   frame [n_frames][7]           target pose DV T_f, p_c0 = T_f^-1 * P_target
 * Column order of dx / rhs (canonical): [intrinsics cam0..cam(N-1) | B_0..B_(N-2) | frame 0..F-1],
 * each pose block ordered (dphi[3], dt[3]) -- the DV insertion order of
 * CalibrateMultiCameraRig (q DV before t DV, CalibrationTools.hpp:32-45).
 */
#ifndef KALIBR_HIP_H
#define KALIBR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KB_MAX_INTR 10
#define KB_MAX_CAMS 16

/* camera models (kalibr2/include/kalibr2/CameraModels.hpp:25-133) */
enum kb_camera_model {
  KB_PINHOLE_RADTAN = 0, /* DistortedPinhole: fu fv cu cv | k1 k2 p1 p2 */
  KB_OMNI_RADTAN = 1,    /* DistortedOmni:    xi fu fv cu cv | k1 k2 p1 p2 */
  KB_EUCM = 2,           /* ExtendedUnified:  alpha beta fu fv cu cv */
  KB_OMNI = 3,           /* Omni:             xi fu fv cu cv */
  KB_DS = 4,             /* DoubleSphere:     xi alpha fu fv cu cv */
  KB_PINHOLE_EQUI = 5,   /* EquidistantPinhole: fu fv cu cv | k1 k2 k3 k4 */
  KB_PINHOLE_FOV = 6     /* FovPinhole:       fu fv cu cv | w */
};

typedef struct kb_handle kb_handle;

typedef struct kb_layout {
  int32_t n_cams;            /* N <= KB_MAX_CAMS */
  int32_t n_frames;          /* F (frames held by this handle / rank) */
  int32_t n_target;          /* target corners (120 for the 6x5 AprilGrid) */
  const int32_t* cam_model;  /* [n_cams] kb_camera_model */
  const double* target_points; /* [n_target][3] */
  int32_t device;            /* HIP device ordinal */
} kb_layout;

/* Replaces SparseCholeskyLinearSystemSolver construction
 * (aslam_backend/src/SparseCholeskyLinearSystemSolver.cpp:8-15). */
kb_handle* kb_create(const kb_layout* layout);
void kb_destroy(kb_handle* h);
const char* kb_last_error(void);

/* Replaces LinearSystemSolver::initMatrixStructure (LinearSystemSolver.cpp:117-138) for
 * ReprojectionError terms: one term per observed corner, grouped in views.
 * Views must be sorted by frame (then camera); one view per (frame, camera).
 *   y            [n_corners][2]  measured keypoints (invR = I, CalibrationTools.hpp:391-393)
 *   corner_id    [n_corners]     target corner index of each term
 *   view_offsets [n_views+1]     corner range of each view
 *   view_frame   [n_views], view_cam [n_views] */
int kb_upload_observations(kb_handle* h, int32_t n_views, int32_t n_corners, const double* y,
                           const uint16_t* corner_id, const uint32_t* view_offsets,
                           const uint32_t* view_frame, const uint8_t* view_cam);

/* Design-variable values (the device owns the state between calls). */
int kb_set_state(kb_handle* h, const double* poses_q, const double* poses_t, const double* baselines,
                 const double* intrinsics);
int kb_set_state_flat(kb_handle* h, const double* state);
int kb_get_state_flat(kb_handle* h, double* state);
int kb_state_size(const kb_handle* h);
int kb_num_cols(const kb_handle* h);     /* JCols = C + 6F */
int kb_camera_cols(const kb_handle* h);  /* C = sum(intrinsics) + 6(N-1) */

/* LinearSystemSolver::evaluateError (LinearSystemSolver.cpp:81-92): chi^2 = sum e^T invR e. */
int kb_eval_cost(kb_handle* h, double* J_out);
/* LinearSystemSolver::buildSystem (SparseCholeskyLinearSystemSolver.cpp:39-46): J, rhs = -J^T e,
 * assembled as the arrow normal equations (no explicit J).  use_mestimator must be 0 or 1
 * (Kalibr2 uses NoMEstimator, weight 1). */
int kb_build(kb_handle* h, int use_mestimator);
/* LinearSystemSolver::setConstantConditioner (LinearSystemSolver.cpp:111-114):
 * "the square of this value will be added to the diagonal" (LinearSystemSolver.hpp:33-39). */
int kb_set_constant_conditioner(kb_handle* h, double diag);
/* LinearSystemSolver::setConditioner (LinearSystemSolver.cpp:98-102): diag[ncols] in the canonical column order;
 * its squares are added to the diagonal of the system kb_solve solves (until kb_set_constant_conditioner).
 * The direct solver only; the device-resident loop conditions with the trust-region lambda as before. */
int kb_set_conditioner(kb_handle* h, const double* diag);
/* LinearSystemSolver::solveSystem (SparseCholeskyLinearSystemSolver.cpp:48-89):
 * solves (J^T J + diag^2 I) dx = rhs.  *ok = 0 on a non-positive-definite system
 * (CHOLMOD failure semantics, Cholmod(impl).hpp:287-328); dx_out untouched then. */
int kb_solve(kb_handle* h, double* dx_out, int* ok);
/* IncrementalEstimator::addBatch on the device (aslam_incremental_calibration IncrementalEstimator.cpp:343-373,
 * 517-527): the reference re-runs initMatrixStructure over the grown problem on every batch; here the new frames are
 * appended to the uploaded handle in place.  kb_append_frames adds n_frames frames (their views sorted by frame,
 * view_frame counted from 0 within the appended block, view_offsets local: [n_views + 1] from 0 to n_corners) and
 * writes their poses ([n_frames][7], q xyzw | t) into the current state; the other design variables keep their
 * device values.  Device buffers grow geometrically and only the new observations cross PCIe, so appending F frames
 * one at a time moves O(F) data in total (the reference's re-initialisation: O(F^2)).  kb_drop_last_frames removes the
 * last n_frames frames with their views and corners (a rejected batch; at least one frame stays).  Captured graphs
 * and a kb_gn_prepare'd loop are voided.  Unsharded handles. */
int kb_append_frames(kb_handle* h, int32_t n_frames, int32_t n_views, int32_t n_corners, const double* y,
                     const uint16_t* corner_id, const uint32_t* view_offsets, const uint32_t* view_frame,
                     const uint8_t* view_cam, const double* frame_poses);
int kb_drop_last_frames(kb_handle* h, int32_t n_frames);

/* Linear solver behind kb_solve ("direct or PCG by mode").
 *   KB_SOLVER_SCHUR  (default) frame-block Schur complement + dense camera-block LDL^T: the exact solve that
 *                    replaces CHOLMOD (SparseCholeskyLinearSystemSolver.cpp:48-89); parity mode.
 *   KB_SOLVER_PCG    block-Jacobi preconditioned conjugate gradients on the full arrow system, as
 *                    sparse_block_matrix's LinearSolverPCG::solve
 *                    (sparse_block_matrix/include/sparse_block_matrix/implementation/linear_solver_pcg.hpp:58-130):
 *                    preconditioner = inverses of the diagonal design-variable blocks; stops when
 *                    r^T M^-1 r <= tolerance * r0^T M^-1 r0 (absolute mode: or <= the previous solve's _residual).
 *                    The reference always returns true; here *ok = 0 on a singular DV block or non-positive
 *                    curvature d^T A d.  One-GPU handles only (a sharded handle returns an error).
 *   KB_SOLVER_PCG_SCHUR  the frame blocks eliminated exactly (as KB_SOLVER_SCHUR), then the same block-Jacobi
 *                    PCG (same options, stopping rule and _residual semantics) on the C x C camera-block Schur
 *                    complement instead of its LDL^T, the frames back-substituted from that camera step.  One
 *                    block, ~1 us per iteration; a different iterate sequence than KB_SOLVER_PCG's full-system CG.
 *                    Sharded handles are supported: every rank runs the same PCG on the all-reduced S, b, so all
 *                    ranks hold bitwise-identical camera steps, iteration counts and _residual; each rank then
 *                    back-substitutes its own frames.  _residual (and kb_get_pcg_info) are updated only by a
 *                    completed solve: a failed one (*ok = 0) leaves the previous values for the next d0.
 * kb_optimize always uses the direct solve (its passes are captured graphs); the per-call path
 * (kb_build / kb_solve / kb_apply_update, driven by the host Optimizer2) uses the selected solver. */
enum kb_linear_solver { KB_SOLVER_SCHUR = 0, KB_SOLVER_PCG = 1, KB_SOLVER_PCG_SCHUR = 2 };
typedef struct kb_pcg_options {
  double tolerance;           /* _tolerance (LinearSolverPCG default 1e-6) */
  int32_t max_iterations;     /* _maxIter (-1: number of rows, the default) */
  int32_t absolute_tolerance; /* _absoluteTolerance (default 1) */
} kb_pcg_options;
typedef struct kb_pcg_info {
  int32_t iterations; /* PCG iterations of the last solve */
  double residual;    /* _residual = 0.5 r^T M^-1 r at exit */
  double d0;          /* stopping threshold used */
} kb_pcg_info;
/* selects the solver (pcg may be NULL: defaults); resets the PCG state as LinearSolverPCG::init() does */
int kb_set_linear_solver(kb_handle* h, int32_t kind, const kb_pcg_options* pcg);
/* LinearSolverPCG::init() (linear_solver_pcg.h:53-59): _residual = -1 */
int kb_pcg_init(kb_handle* h);
int kb_get_pcg_info(kb_handle* h, kb_pcg_info* info);

/* LinearSystemSolver::rhs (LinearSystemSolver.hpp:47). */
int kb_get_rhs(kb_handle* h, double* rhs_out);
/* LinearSystemSolver::rhsJtJrhs (LinearSystemSolver.hpp:66-69): rhs^T (J^T J) rhs of the last kb_build (the reference
 * forms ||J rhs||^2, SparseCholeskyLinearSystemSolver.cpp:106-111; DogLeg / steepest descent), on the device from
 * the arrow blocks.  Unsharded handles.  Fails unless the last system came from kb_build: the device-resident
 * loops (kb_optimize, kb_gn_*, kb_build_kernel_stats) overwrite or skip the per-call blocks it reads. */
int kb_rhs_jtj_rhs(kb_handle* h, double* out);
/* CameraCalibrator::PrintReprojectionErrorStatistics (kalibr2/include/kalibr2/CameraCalibrator.hpp:368-411, called per
 * camera after the estimator by kalibr2_ros/src/CalibrateCameras.cpp:318) on the device, for every camera of the
 * handle at its current state: e = y - yhat of every term (ReprojectionError::getPredictedMeasurement), then
 * out[cam][6] = [n, mean_u, mean_v, std_u, std_v, rmse] with the sample standard deviation (N - 1; 0 when n < 2) of a
 * second pass about the mean, and the reference's "RMSE" = |sum e| / sqrt(n) (the norm of the error SUM, kept as the
 * reference prints it).  A camera without terms gets zeros.  Sharded handles sum over all ranks' frames. */
int kb_reprojection_error_stats(kb_handle* h, double* out);
/* Optimizer2::applyStateUpdate / revertLastStateUpdate (Optimizer2.cpp:290-318).
 * dx == NULL applies the device-resident dx of the last kb_solve. */
int kb_apply_update(kb_handle* h, const double* dx, double* deltaX_out);
int kb_revert(kb_handle* h);

/* aslam_incremental_calibration's LinearSolver (incremental_calibration/src/core/LinearSolver.cpp), the
 * linear solver of IncrementalEstimator's optimizer (IncrementalEstimator.cpp:46-66) and so of the CLI's final
 * calibration (CalibrateCameras.cpp:258-272).  Options: LinearSolverOptions (LinearSolverOptions.cpp:30-38). */
typedef struct kb_marginal_options {
  int32_t column_scaling; /* columnScaling (Kalibr2: 1) */
  double eps_norm;        /* epsNorm: column-norm tolerance sqrt(rows * epsNorm) (default DBL_EPSILON) */
  double eps_svd;         /* epsSVD: rankTol = sv_0 * epsSVD * C (Kalibr2: 1e-6) */
  double svd_tol;         /* svdTol: fixed tolerance, -1 = rankTol */
} kb_marginal_options;
typedef struct kb_marginal_info {
  int32_t rank;       /* getSVDRank (C - rank = getSVDRankDeficiency) */
  int32_t sweeps;     /* Jacobi sweeps used */
  double tolerance;   /* getSVDTolerance */
  double sv_gap;      /* getSvGap: sv[rank-1] / sv[rank], +inf at full rank */
  double sv_log2_sum; /* getSingularValuesLog2Sum over the first rank singular values */
} kb_marginal_info;
/* LinearSolver::solveSystem -> solve (LinearSolver.cpp:247-280, 299-466) after kb_build: the frame blocks are
 * eliminated (lambda = 0; the conditioner is ignored, as LinearSolver ignores it), the camera block Omega is
 * column-scaled and solved by truncated SVD, the frame steps back-substituted.  sv_out [C] (descending) and
 * V_out [C][C] (row-major, singular vector j in column j) are the scaled SVD (getSingularValues /
 * getMatrixV); either may be NULL.  *ok = 0 if a frame block is not positive definite.  C <= 112. */
int kb_solve_marginal(kb_handle* h, const kb_marginal_options* opts, double* dx_out, int* ok,
                      kb_marginal_info* info, double* sv_out, double* V_out);
/* LinearSolver::analyzeMarginal (LinearSolver.cpp:468-528): SVD of the unscaled Omega of the last kb_build.
 * info->rank / tolerance / sv_gap / sv_log2_sum are those of this SVD; the reference keeps the rank of the last
 * solve (the C++ host layer's MarginalLinearSolver does the same). */
int kb_analyze_marginal(kb_handle* h, const kb_marginal_options* opts, kb_marginal_info* info, double* sv_out,
                        double* V_out);

/* Normal-equation blocks of the last kb_build, for parity tests:
 * Hff [F][6][6], Hfc [F][6][C], gf [F][6], Hcc [C][C], gc [C], cost (chi^2 at build state).  Fails after a
 * device-resident loop until the next kb_build (as kb_rhs_jtj_rhs). */
int kb_get_normal_blocks(kb_handle* h, double* Hff, double* Hfc, double* gf, double* Hcc, double* gc,
                         double* cost);

/* Device-resident Optimizer2::optimize (Optimizer2.cpp:183-273) with the
 * LevenbergMarquardt (policy 0, LevenbergMarquardtTrustRegionPolicy.cpp:50-113) or
 * GaussNewton (policy 1, GaussNewtonTrustRegionPolicy.cpp:18-39) trust-region policy.
 * The whole loop (build, Schur solve, update, cost, policy) runs as one hipGraph per
 * iteration; the host synchronises only every `sync_every` iterations. */
typedef struct kb_optimizer_options {
  int32_t policy;          /* 0 = levenberg_marquardt, 1 = gauss_newton */
  double lambda_init;      /* LM lambdaInit (CalibrationTools.hpp:65: 10) */
  int32_t max_iterations;  /* Optimizer2Options::maxIterations */
  double convergence_dx;   /* convergenceDeltaX */
  double convergence_dj;   /* convergenceDeltaJ */
  int32_t sync_every;      /* host checks the done flag every n passes (0 = auto) */
  int32_t use_graph;       /* capture the iteration in a hipGraph (1) or launch eagerly (0) */
} kb_optimizer_options;

typedef struct kb_solution {
  double J_start, J_final, dx_final, dj_final; /* SolutionReturnValue (backend.hpp:11-24) */
  int32_t iterations, failed_iterations, linear_solver_failure;
  int32_t passes;
  int32_t graphed;         /* 1 if the passes ran as captured hipGraphs (RCCL calls included when sharded) */
} kb_solution;

int kb_optimize(kb_handle* h, const kb_optimizer_options* opts, kb_solution* out);

/* The IncrementalEstimator's optimisation device-resident (IncrementalEstimator.cpp:46-77, 373: Optimizer2 with the
 * GaussNewtonTrustRegionPolicy over calibration::LinearSolver): every pass builds with the frame blocks eliminated,
 * solves the camera block by the column-scaled truncated SVD of kb_solve_marginal, updates the design variables,
 * evaluates the cost and runs the policy (accept, convergence tests on convergence_dx / convergence_dj,
 * max_iterations) on the device; the passes run as captured graphs and the host polls the done flag every sync_every
 * passes.  opts->policy must be 1 (GN); opts->lambda_init is unused.  info / sv_out / V_out: the SVD of the last
 * solve (as kb_solve_marginal reports it; any may be NULL).  kb_analyze_marginal afterwards analyses the last
 * build, as analyzeMarginal after Optimizer2::optimize does.  Unsharded handles, C <= 112. */
int kb_optimize_marginal(kb_handle* h, const kb_optimizer_options* opts, const kb_marginal_options* mopts,
                         kb_solution* out, kb_marginal_info* info, double* sv_out, double* V_out);
/* kb_optimize_marginal followed by kb_analyze_marginal of the last build on the same stream, before the one host
 * sync that ends the loop (the IncrementalEstimator's optimize + analyzeMarginal pair, IncrementalEstimator.cpp:373,
 * 400): analyze_info / analyze_sv_out / analyze_V_out are what kb_analyze_marginal would return (any may be NULL). */
int kb_optimize_marginal_analyze(kb_handle* h, const kb_optimizer_options* opts, const kb_marginal_options* mopts,
                                 kb_solution* out, kb_marginal_info* info, double* sv_out, double* V_out,
                                 kb_marginal_info* analyze_info, double* analyze_sv_out, double* analyze_V_out);

/* Per-pass trace of the last kb_optimize: [J, lambda, deltaX, accepted] x n (returns count). */
int kb_get_trace(kb_handle* h, double* trace, int32_t cap);

/* Benchmark entry: run exactly n_iter Gauss-Newton passes of the device loop (convergence
 * tests disabled), no host sync inside; *seconds = wall time between stream syncs. */
int kb_run_gn_iterations(kb_handle* h, int32_t n_iter, double* seconds);
/* kb_run_gn_iterations in two calls, so that a multi-process run can put a host barrier between them:
 * kb_gn_prepare = the loop start (evaluateError on the current state, first prelude) + capture and upload of
 * every graph n_iter passes will launch, then a stream sync; kb_gn_launch = the n_iter passes and the last
 * pass's end between two stream syncs (*seconds = that wall time).  Same passes, same results.
 * kb_gn_prepare returns 1 when the passes will run as captured hipGraphs (RCCL calls included when sharded),
 * 0 when they run eagerly, < 0 on error.  Any call that changes the state, the control block or the graphs in
 * between (state setters, per-call entry points, kb_optimize, kb_comm_init, ...) voids the preparation:
 * kb_gn_launch then fails instead of running from a stale loop start. */
int kb_gn_prepare(kb_handle* h, int32_t n_iter);
int kb_gn_launch(kb_handle* h, int32_t n_iter, double* seconds);
/* Average device duration (ms) of the build kernel inside Gauss-Newton passes (runs 22 passes from the
 * current state, HIP events around each build launch on the handle's stream); algorithmic bytes per build launch and
 * the pass's algorithmic FP64 flops (projection + Jacobian, cost and local Hessian per corner, the
 * 6-D chain expansion per view, the Schur sums per frame; not the padded MFMA work the kernel executes).  The state,
 * camera chains and control block are restored afterwards. */
int kb_build_kernel_stats(kb_handle* h, double* avg_ms, double* bytes_per_launch, double* flops_per_launch);
/* Per-pass device timing of n Gauss-Newton passes from the current state (iteration 1 = the first pass after the
 * loop start): HIP events at every pass start and around every build kernel, captured in one graph with the passes,
 * on the handle's stream.  pass_ms [n] (pass r: from its start to the next pass's start), build_ms [n] (either may be
 * NULL).  A query: the state, camera chains and control block are restored afterwards.  Unsharded handles time the
 * graph; sharded ones run the passes eagerly. */
int kb_gn_pass_times(kb_handle* h, int32_t n, double* pass_ms, double* build_ms);
/* Name of the build kernel this handle launches ("k_buildp" or "k_build") into buf (NUL-terminated). */
int kb_build_kernel_name(kb_handle* h, char* buf, int32_t cap);

/* Multi-GPU (frame sharding): each rank's handle holds its own frames;
 * the camera-block [S | b] and the cost/step statistics are all-reduced over RCCL once
 * per pass.  unique_id is the 128-byte ncclUniqueId. */
int kb_comm_get_unique_id(void* unique_id_out128);
int kb_comm_init(kb_handle* h, const void* unique_id128, int32_t nranks, int32_t rank);
/* In-process group: n handles of this process (any devices, one device included) become ranks 0..n-1 of one
 * sharded problem and exchange through device copies instead of RCCL (sums in rank order).  Each handle must
 * then be driven from its own host thread: the collectives of a pass meet in a host barrier (60 s timeout ->
 * error).  Passes run eagerly, not graph-captured.  Used to test the sharded path with several ranks on one GPU. */
int kb_comm_init_local(kb_handle* const* handles, int32_t n);
/* Direct all-reduce of the sharded camera-block image (C > 64, GN fused passes; replaces the collective of
 * LinearSystemSolver.cpp:81-92's host sum): kb_comm_init / kb_comm_init_local map every rank's exchange region (IPC
 * handles all-gathered over the communicator; the members' buffers in-process), self-test one exchange, and from then
 * on k_xar sums the ranks' partial images in rank order on every rank, reading the peers over xGMI -- no RCCL
 * collective for it, bitwise-identical images on all ranks.  KB_DIRECT_AR=0, a failed mapping or a failed self-test
 * (agreed over all ranks) keep the collective.  Returns 1 when the handle uses the direct path. */
int kb_comm_direct(const kb_handle* h);
/* The IPC half of the direct all-reduce on its own (test hook: RCCL refuses several ranks on one device, so the
 * multi-process mapping is tested with processes sharing one GPU).  kb_xar_export writes this handle's exchange-region
 * IPC handle (64 bytes); kb_xar_test maps the peers' regions from handles64 [nranks][64] (own slot ignored) and runs
 * the self-test exchange with them: *ok = 1 when every rank's known values arrived in rank-order sums, 0 when not or
 * when a peer did not take part within 2 s.  The handle stays unsharded.  C > 64 only. */
int kb_xar_export(kb_handle* h, void* handle_out64);
int kb_xar_test(kb_handle* h, int32_t nranks, int32_t rank, const void* handles64, int32_t* ok);

/* Self test of the f64 MFMA fragment layout used by the build kernel (A = I, asymmetric B). */
int kb_selftest_mfma(double* max_err);

/* ------------------------------------------------------------------------------------------------
 * Continuous-time calibration (configs[4]): the rig (IMU body b) on a B-spline pose trajectory
 * T_wb(t) (bsplines::BSplinePose with a RotationVector rotation, BSplinePose.cpp:21-41,384-412;
 * one DesignVariableMappedVector<6> per coefficient, BSplinePoseDesignVariable.cpp:9-19).
 *   camera terms  ReprojectionError at frame time t_f through T_ci_w = B_{i-1}..B_0 T_c0_b T_wb(t_f)^-1
 *                 (BSplineTransformationExpressionNode, BSplineExpressions.cpp:23-45)
 *   IMU terms     (not in the reference -- defined in DESIGN.md 10):
 *                 gyro  w_m = w_b(t) + b_g,  w_b = -C^T S(theta) theta_dot (BSplinePose.cpp:207-219)
 *                 accel a_m = C^T (p_ddot(t) - g_w) + b_a                  (cf. BSplinePose.cpp:175-180)
 *                 whitened by 1/sigma_gyro, 1/sigma_acc.
 * State:   intr [N][KB_MAX_INTR] | base [N-1][7] | T_c0_b [7] | b_g [3] | b_a [3] | g_w [3] | coeff [K][6]
 * Columns: [intr | B_j (dphi, dt) | T_c0_b (dphi, dt) | b_g | b_a | g_w | coeff 0..K-1 (6 each)]
 * Knot vector: non-decreasing, n_knots = K + order; the device path supports order 4 (cubic).
 * The coefficient block is solved by block cyclic reduction on the device.
 * ------------------------------------------------------------------------------------------------ */
typedef struct kb_sp_handle kb_sp_handle;

typedef struct kb_sp_layout {
  int32_t n_cams;
  int32_t n_target;
  const int32_t* cam_model;     /* [n_cams] */
  const double* target_points;  /* [n_target][3] */
  int32_t order;                /* 4 */
  int32_t n_knots;
  const double* knots;          /* [n_knots] */
  double sigma_gyro, sigma_acc; /* IMU noise (whitening) */
  int32_t device;
} kb_sp_layout;

kb_sp_handle* kb_sp_create(const kb_sp_layout* layout);
void kb_sp_destroy(kb_sp_handle* h);
/* initMatrixStructure for the spline problem: frames (times, views sorted by frame) and IMU samples.
 * All times inside the spline interval [knots[order-1], knots[n_knots-order]]. */
int kb_sp_upload(kb_sp_handle* h, int32_t n_frames, const double* frame_time, int32_t n_views, int32_t n_corners,
                 const double* y, const uint16_t* corner_id, const uint32_t* view_offsets,
                 const uint32_t* view_frame, const uint8_t* view_cam, int32_t n_imu, const double* imu_time,
                 const double* imu_gyro, const double* imu_acc);
int kb_sp_state_size(const kb_sp_handle* h);
int kb_sp_num_cols(const kb_sp_handle* h);
int kb_sp_camera_cols(const kb_sp_handle* h);
int kb_sp_set_state(kb_sp_handle* h, const double* state);
int kb_sp_get_state(kb_sp_handle* h, double* state);
/* evaluateError / buildSystem / setConstantConditioner / solveSystem / rhs / applyStateUpdate /
 * revertLastStateUpdate of the spline system, same semantics as the kb_* rig entry points. */
int kb_sp_eval_cost(kb_sp_handle* h, double* J_out);
int kb_sp_build(kb_sp_handle* h);
int kb_sp_set_constant_conditioner(kb_sp_handle* h, double diag);
/* BSplineMotionError (aslam_splines/include/aslam/backend/implementation/BSplineMotionError.hpp:29-160) on the pose
 * spline: cost c^T Q c with Q = curveQuadraticIntegralSparse(W, derivative_order) (bsplines/src/BSpline.cpp:
 * 1585-1622), added to evaluateError; buildSystem adds Q to the coefficient band and -Q c to the rhs (the
 * reference's buildHessianImplementation).  W [6][6] symmetric (row-major); derivative_order >= order is reduced to
 * order - 1 as the reference does; W == NULL removes the term. */
int kb_sp_set_motion_error(kb_sp_handle* h, const double* W, int32_t derivative_order);
/* ErrorTermEuclidean priors on the spline position: n terms ErrorTermEuclidean(bsp.position(times[k]), priors[k],
 * N[k]) (aslam_backend_expressions ErrorTermEuclidean.cpp:10-23,50-66 over BSplinePoseDesignVariable::position,
 * BSplinePoseDesignVariable.cpp:91-103): e = p(t_k) - prior_k, chi^2 = e^T N_k^-1 e, Jacobian w_j(t_k) [I_3 | 0] on the
 * active coefficients.  times [n] inside the spline interval, priors [n][3], N [n][3][3] symmetric positive definite
 * covariances (the reference's first constructor); n == 0 removes the terms. */
int kb_sp_set_position_priors(kb_sp_handle* h, int32_t n, const double* times, const double* priors, const double* N);
int kb_sp_solve(kb_sp_handle* h, double* dx_out, int* ok);
int kb_sp_get_rhs(kb_sp_handle* h, double* rhs_out);
int kb_sp_apply_update(kb_sp_handle* h, const double* dx, double* deltaX_out);
int kb_sp_revert(kb_sp_handle* h);
/* Normal equations of the last kb_sp_build (parity tests): Hcc [C][C], Hsc [6K][C], Hband [K][order][6][6]
 * (block (k, k+d)), gc [C], gs [6K], cost. */
int kb_sp_get_system(kb_sp_handle* h, double* Hcc, double* Hsc, double* Hband, double* gc, double* gs,
                     double* cost);
/* Optimizer2::optimize over the spline system (LM policy 0 / GN policy 1), host-driven loop over the
 * device passes; trace as kb_get_trace. */
int kb_sp_optimize(kb_sp_handle* h, const kb_optimizer_options* opts, kb_solution* out);
int kb_sp_get_trace(kb_sp_handle* h, double* trace, int32_t cap);
/* Benchmark: exactly n_iter GN passes (build + solve + update + cost), captured in a hipGraph. */
int kb_sp_run_gn_iterations(kb_sp_handle* h, int32_t n_iter, double* seconds);
/* Per-kernel device time (ms, HIP events on the handle's stream) of one GN pass, averaged over n passes:
 * out[0] frames kernel, [1] assemble, [2] cyclic reduction (all levels), [3] Schur + camera solve,
 * [4] update + cost, [5] whole pass; bytes[0] algorithmic bytes of the frames kernel per launch. */
int kb_sp_kernel_stats(kb_sp_handle* h, int32_t n, double* ms_out6, double* frames_bytes);
/* Device time (ms, HIP events around each launch on the handle's stream, averaged over n launches inside built
 * passes) and algorithmic bytes per launch of the node-assembly kernel (the pass's largest single launch). */
int kb_sp_assemble_stats(kb_sp_handle* h, int32_t n, double* ms, double* bytes);

#ifdef __cplusplus
}
#endif
#endif
