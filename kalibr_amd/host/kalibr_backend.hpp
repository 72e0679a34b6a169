// kalibr_backend.hpp -- C++ host layer over the kalibr_hip C-ABI, mirroring the aslam_backend plugin surface
// that Kalibr2's batch calibration drives (paths relative to the reference repository):
//   LinearSystemSolver      aslam_optimizer/aslam_backend/include/aslam/backend/LinearSystemSolver.hpp:16-109
//   TrustRegionPolicy       aslam_optimizer/aslam_backend/include/aslam/backend/TrustRegionPolicy.hpp:13-57
//   LevenbergMarquardt...   aslam_optimizer/aslam_backend/src/LevenbergMarquardtTrustRegionPolicy.cpp:7-117
//   GaussNewton...          aslam_optimizer/aslam_backend/src/GaussNewtonTrustRegionPolicy.cpp:7-39
//   Optimizer2Options       aslam_optimizer/aslam_backend/include/aslam/backend/Optimizer2Options.hpp:9-42
//   Optimizer2::optimize    aslam_optimizer/aslam_backend/src/Optimizer2.cpp:183-273
//   SolutionReturnValue     aslam_optimizer/aslam_backend/include/aslam/backend/backend.hpp:11-24
//   MarginalLinearSolver    aslam_incremental_calibration/incremental_calibration/src/core/LinearSolver.cpp:113-528
//                           (calibration::LinearSolver; options LinearSolverOptions.cpp:30-38)
//   IncrementalEstimator    aslam_incremental_calibration/incremental_calibration/src/core/IncrementalEstimator.cpp
//                           :44-77, 337-530 (addBatch: GN optimize, marginal analysis, information-gain acceptance)
// Same names, argument meaning and error behaviour (contract violations and device errors throw
// LinearSystemSolver::Exception, a std::runtime_error; a numerically failed solve returns false).
// Deviations, all because the device owns the design variables:
//   * evaluateError is virtual (the GPU solver owns the cost pass);
//   * applyStateUpdate / revertLastStateUpdate go through the solver, which holds the device state;
//   * vectors are std::vector<double> instead of Eigen::VectorXd (Eigen is not a dependency here).
#pragma once

#include <cfloat>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <string>
#include <array>
#include <vector>

namespace kalibr_amd {
namespace backend {

// ---------------------------------------------------------------- problem description
// What CalibrateMultiCameraRig / CreateBatchProblem hand to the optimizer (CalibrationTools.hpp:376-521):
// the camera models, the target corners, one ReprojectionError term per observed corner grouped in
// (frame, camera) views, and the design-variable values (flat state, include/kalibr_hip.h).
struct CalibrationProblem {
  std::vector<int32_t> cam_model;    // kb_camera_model per camera
  std::vector<double> target;        // [n_target][3]
  std::vector<uint32_t> view_frame;  // [n_views], sorted by frame
  std::vector<uint8_t> view_cam;     // [n_views]
  std::vector<uint32_t> view_offset; // [n_views + 1]
  std::vector<uint16_t> corner_id;   // [n_corners]
  std::vector<double> y;             // [n_corners][2]
  std::vector<double> state;         // flat design-variable values
  int n_frames = 0;
  int n_cams() const { return (int)cam_model.size(); }
  int n_views() const { return (int)view_frame.size(); }
  int n_corners() const { return (int)corner_id.size(); }
  int n_target() const { return (int)target.size() / 3; }
};

struct SolutionReturnValue {  // backend.hpp:11-24
  double JStart = 0.0, JFinal = 0.0, dXFinal = 0.0, dJFinal = 0.0;
  int iterations = 0, failedIterations = 0;
  bool linearSolverFailure = false;
};

// ---------------------------------------------------------------- LinearSystemSolver
class LinearSystemSolver {
 public:
  struct Exception : std::runtime_error {
    explicit Exception(const std::string& m) : std::runtime_error(m) {}
  };
  virtual ~LinearSystemSolver() = default;

  /// chi^2 = sum_i e_i^T invR e_i of the current state (LinearSystemSolver.cpp:81-92)
  virtual double evaluateError(size_t nThreads, bool useMEstimator) = 0;
  /// build J and rhs = -J^T e at the current state
  virtual void buildSystem(size_t nThreads, bool useMEstimator) = 0;
  /// "The square of these values will be added to the diagonal of the Hessian matrix" (:33-35)
  virtual void setConditioner(const std::vector<double>& diag);
  virtual void setConstantConditioner(double diag);
  /// solve (J^T J + diag^2) dx = rhs; false on a numerically failed factorisation
  virtual bool solveSystem(std::vector<double>& outDx) = 0;
  virtual std::string name() const = 0;
  virtual const std::vector<double>& rhs() const { return _rhs; }
  virtual double rhsJtJrhs() = 0;
  /// design-variable update x <- x [+] dx, returns max|dx| (Optimizer2.cpp:290-310)
  virtual double applyStateUpdate(const std::vector<double>& dx) = 0;
  virtual void revertLastStateUpdate() = 0;

  size_t JRows() const { return _JRows; }
  size_t JCols() const { return _JCols; }

 protected:
  std::vector<double> _rhs;
  std::vector<double> _diagonalConditioner;
  size_t _JRows = 0, _JCols = 0;
};

/// A LinearSystemSolver that takes its terms as a packed CalibrationProblem in the canonical column order
/// [intrinsics | baselines | frames] (the GPU solver; the tests' oracle-backed solver).
class ProblemLinearSystemSolver : public LinearSystemSolver {
 public:
  virtual void initMatrixStructure(const CalibrationProblem& problem, bool useDiagonalConditioner) = 0;
  /// flat design-variable values (include/kalibr_hip.h layout)
  virtual std::vector<double> state() const = 0;
  /// CameraCalibrator::PrintReprojectionErrorStatistics (CameraCalibrator.hpp:368-411) of every camera at the current
  /// state: [n, mean_u, mean_v, std_u, std_v, rmse] (sample std; rmse = |sum e| / sqrt(n), as the reference prints it)
  virtual std::vector<std::array<double, 6>> reprojectionErrorStatistics() {
    throw Exception(name() + ": no reprojection-error statistics");
  }
};

// ---------------------------------------------------------------- design variables and error terms
/// aslam_backend::DesignVariable (DesignVariable.hpp) reduced to what the batch problem's terms read: the kind,
/// minimal dimension and activity, the block index / column base Optimizer2::initialize assigns
/// (Optimizer2.cpp:110-124), and the value.  Kinds: the camera's projection and distortion DVs
/// (CameraDesignVariable: e.g. 4 | 4 for pinhole-radtan, 6 | none for EUCM), RotationQuaternion (value: JPL
/// quaternion [x y z w], minimal dimension 3), EuclideanPoint (3), HomogeneousPoint (the target landmarks,
/// inactive in the batch problems, CalibrationTools.hpp:470-473).
struct DesignVariable {
  enum class Kind { Projection, Distortion, RotationQuaternion, EuclideanPoint, HomogeneousPoint };
  Kind kind = Kind::EuclideanPoint;
  int camera = -1;       // Projection / Distortion: the camera's index in the rig
  int cameraModel = -1;  // Projection: its kb_camera_model
  std::vector<double> value;
  bool active = true;
  int blockIndex = -1, columnBase = -1;
  bool isActive() const { return active; }
  int minimalDimensions() const;
};

/// One ReprojectionError term (ReprojectionError.hpp(impl):49-77) of the rig problem: the corner `cornerId` of the
/// target seen at `y` by camera `camera` through T_cam_w = B_{camera-1} .. B_0 T^-1, T = (targetRotation,
/// targetTranslation), B_j = (baselines[2j], baselines[2j + 1]) -- the chain CalibrateMultiCameraRig and
/// CreateBatchProblem build (CalibrationTools.hpp:401-410, 497-508); invR = I (corner uncertainty 1).
struct ReprojectionErrorTerm {
  int camera = 0;
  int cornerId = 0;
  double y[2] = {0.0, 0.0};
  DesignVariable* targetRotation = nullptr;
  DesignVariable* targetTranslation = nullptr;
  std::vector<DesignVariable*> baselines;  // rotation, translation of B_0 .. B_{camera-1}
  DesignVariable* projection = nullptr;
  DesignVariable* distortion = nullptr;  // null for models without a distortion DV (EUCM, omni, double sphere)
  int dimension() const { return 2; }
};

/// Optimizer2::initialize (Optimizer2.cpp:110-124): the active DVs in the given order get block index i and
/// column base = the sum of the preceding minimal dimensions.  Returns the active list.
std::vector<DesignVariable*> assignColumnBases(const std::vector<DesignVariable*>& dvs);

/// The terms packed for a ProblemLinearSystemSolver: the canonical problem (frames in the order of their rotation
/// DVs' column bases, views sorted by frame, terms of a view in the given order) and perm[k] = the caller's column
/// of canonical column k.
struct TermAssembly {
  CalibrationProblem problem;
  std::vector<int> perm;
  std::vector<DesignVariable*> projection, distortion;  // per camera (distortion may be null)
  std::vector<DesignVariable*> baseRotation, baseTranslation;  // per baseline
  std::vector<DesignVariable*> frameRotation, frameTranslation;  // per frame, canonical order
};

/// Walks the terms (which must form the rig structure above) and packs them; `target` = [n_target][3] corners.
/// Throws LinearSystemSolver::Exception on anything the device path cannot represent (an active DV no term
/// reads, a chain that is not B_{c-1}..B_0 T^-1, missing column bases).
TermAssembly assembleTerms(const std::vector<DesignVariable*>& dvs, const std::vector<ReprojectionErrorTerm*>& errors,
                           const std::vector<double>& target);

/// Design-variable values from a flat state (include/kalibr_hip.h layout) of the assembled problem.
void pullDesignVariables(const TermAssembly& a, const std::vector<double>& state);

/// LinearSystemSolver::initMatrixStructure(dvs, errors, useDiagonalConditioner) (LinearSystemSolver.hpp:28, 73)
/// in front of a ProblemLinearSystemSolver: the terms are packed once, and rhs, dx and the conditioner are
/// permuted between the caller's column order (the DVs' column bases) and the canonical one.
class TermLinearSystemSolver : public LinearSystemSolver {
 public:
  TermLinearSystemSolver(std::shared_ptr<ProblemLinearSystemSolver> inner, std::vector<double> target);
  void initMatrixStructure(const std::vector<DesignVariable*>& dvs, const std::vector<ReprojectionErrorTerm*>& errors,
                           bool useDiagonalConditioner);
  double evaluateError(size_t nThreads, bool useMEstimator) override;
  void buildSystem(size_t nThreads, bool useMEstimator) override;
  void setConditioner(const std::vector<double>& diag) override;
  void setConstantConditioner(double diag) override;
  bool solveSystem(std::vector<double>& outDx) override;
  std::string name() const override { return _inner->name(); }
  const std::vector<double>& rhs() const override;
  double rhsJtJrhs() override { return _inner->rhsJtJrhs(); }  // invariant under the column permutation
  double applyStateUpdate(const std::vector<double>& dx) override;
  void revertLastStateUpdate() override { _inner->revertLastStateUpdate(); }
  /// the solver's state into the design variables' values
  void pullDesignVariables() const;
  const TermAssembly& assembly() const { return _a; }
  ProblemLinearSystemSolver& inner() { return *_inner; }

 private:
  std::shared_ptr<ProblemLinearSystemSolver> _inner;
  std::vector<double> _target;
  TermAssembly _a;
  mutable std::vector<double> _rhs_caller;
};

// ---------------------------------------------------------------- GPU solver over the C-ABI
/// linearSolver: "schur" (frame-block Schur + camera-block LDL^T, the exact CHOLMOD replacement, default) or
/// "pcg" (sparse_block_matrix LinearSolverPCG: block-Jacobi PCG, linear_solver_pcg.hpp:58-130, with its
/// defaults tolerance 1e-6 / maxIter = rows / absoluteTolerance, linear_solver_pcg.h:39-47) or "pcg_schur" (the
/// same PCG on the camera-block Schur complement, the frame blocks eliminated exactly).
struct GpuOptions {
  int device = 0;
  std::string linearSolver = "schur";
  double pcgTolerance = 1e-6;
  int pcgMaxIterations = -1;
  bool pcgAbsoluteTolerance = true;
};

/// LinearSystemSolver whose build / solve / update / cost run on one MI355X (kalibr_hip.h).  The
/// per-call methods mirror the reference solver one call at a time; optimizeOnDevice() runs the whole
/// Optimizer2 loop device-resident (one captured graph per pass).
class GpuLinearSystemSolver : public ProblemLinearSystemSolver {
 public:
  explicit GpuLinearSystemSolver(const GpuOptions& o = GpuOptions());
  ~GpuLinearSystemSolver() override;
  GpuLinearSystemSolver(const GpuLinearSystemSolver&) = delete;
  GpuLinearSystemSolver& operator=(const GpuLinearSystemSolver&) = delete;

  /// LinearSystemSolver::initMatrixStructure (LinearSystemSolver.cpp:117-138): uploads the terms and state
  void initMatrixStructure(const CalibrationProblem& problem, bool useDiagonalConditioner) override;

  double evaluateError(size_t nThreads, bool useMEstimator) override;
  void buildSystem(size_t nThreads, bool useMEstimator) override;
  void setConstantConditioner(double diag) override;
  void setConditioner(const std::vector<double>& diag) override;
  bool solveSystem(std::vector<double>& outDx) override;
  std::string name() const override {
    return _opt.linearSolver == "pcg"         ? "kalibr_hip_block_jacobi_pcg"
           : _opt.linearSolver == "pcg_schur" ? "kalibr_hip_schur_block_jacobi_pcg"
                                              : "kalibr_hip_schur_cholesky";
  }
  const std::vector<double>& rhs() const override;
  double rhsJtJrhs() override;
  double applyStateUpdate(const std::vector<double>& dx) override;
  void revertLastStateUpdate() override;

  std::vector<double> state() const override;
  std::vector<std::array<double, 6>> reprojectionErrorStatistics() override;  // kb_reprojection_error_stats
  void setState(const std::vector<double>& s);
  size_t cameraCols() const { return _C; }
  void* handle() const { return _h; }
  /// PCG iterations of the last solveSystem (0 with the direct solver)
  int lastPcgIterations() const;
  /// the problem's frames from `firstFrame` on appended to the uploaded handle in place (kb_append_frames), the
  /// handle holding exactly frames [0, firstFrame) of `problem` before; then the whole state set from problem.state.
  /// Returns false (nothing changed) when the handle does not hold that prefix; initMatrixStructure then applies.
  bool appendFrames(const CalibrationProblem& problem, size_t firstFrame);
  /// the last n frames removed (kb_drop_last_frames), then the state set to `state` (the smaller problem's)
  void dropLastFrames(size_t n, const std::vector<double>& state);
  size_t framesHeld() const { return _F; }

 private:
  void check(int rc, const char* what) const;
  void* _h = nullptr;
  GpuOptions _opt;
  size_t _C = 0, _F = 0, _N = 0;
  double _conditioner = 0.0;
  bool _built = false;
  mutable bool _rhs_valid = false;
};

// ---------------------------------------------------------------- marginal (camera-block) solver
/// LinearSolverOptions (LinearSolverOptions.cpp:30-38); Kalibr2 sets columnScaling = true, epsSVD = 1e-6
/// (CalibrateCameras.cpp:263-267).  The QR part of the reference (epsQR, SPQR) is the frame-block
/// elimination here; its options have no counterpart.
struct LinearSolverOptions {
  bool columnScaling = false;
  double epsNorm = DBL_EPSILON;
  double epsSVD = DBL_EPSILON;
  double svdTol = -1.0;
  bool verbose = false;
};

/// The calibration::LinearSolver surface the IncrementalEstimator drives (LinearSolver.h:60-236): the
/// Schur complement onto the marginalized (camera) block solved by truncated SVD, plus the SVD statistics
/// of the last solve (scaled when columnScaling) and of analyzeMarginal (unscaled).
class MarginalLinearSystemSolver : public LinearSystemSolver {
 public:
  /// LinearSystemSolver::initMatrixStructure over a (re)assembled problem (IncrementalEstimator.cpp:593-596)
  virtual void initMatrixStructure(const CalibrationProblem& problem, bool useDiagonalConditioner) = 0;
  virtual std::vector<double> state() const = 0;
  /// LinearSolver::analyzeMarginal (LinearSolver.cpp:468-528): SVD of the unscaled marginal system of the
  /// last build.  As in the reference the rank is the one of the last solve.
  virtual void analyzeMarginal() = 0;
  /// in-place growth for the IncrementalEstimator (kb_append_frames): false if not supported or the solver does not
  /// hold frames [0, firstFrame) of `problem`, and then initMatrixStructure is called instead
  virtual bool appendFrames(const CalibrationProblem& /*problem*/, size_t /*firstFrame*/) { return false; }
  /// drop the last n frames and set `state` (a rejected batch); false if not supported
  virtual bool dropLastFrames(size_t /*n*/, const std::vector<double>& /*state*/) { return false; }
  /// Optimizer2::optimize with the GaussNewtonTrustRegionPolicy over this solver, run device-resident
  /// (kb_optimize_marginal); false if not supported (the host Optimizer2 runs instead).  Leaves the SVD statistics
  /// of the last solve, as solveSystem does.
  virtual bool optimizeDevice(const struct Optimizer2Options& /*o*/, struct SolutionReturnValue& /*out*/) { return false; }
  const LinearSolverOptions& getOptions() const { return _lopt; }
  std::ptrdiff_t getSVDRank() const { return _svdRank; }
  std::ptrdiff_t getSVDRankDeficiency() const { return _svdRank == -1 ? -1 : (std::ptrdiff_t)_sv.size() - _svdRank; }
  double getSVDTolerance() const { return _svdTolerance; }
  double getSvGap() const { return _svGap; }
  const std::vector<double>& getSingularValues() const { return _sv; }
  /// V [C][C] row-major, right singular vector j in column j
  const std::vector<double>& getMatrixV() const { return _V; }
  double getSingularValuesLog2Sum() const;  // LinearSolver.cpp:196-201
  std::vector<double> getNullSpace() const;  // [C][C - rank] (LinearSolver.cpp:166-171)
  std::vector<double> getRowSpace() const;   // [C][rank] (:173-178)
  std::vector<double> getCovariance() const; // [C][C] = V_r diag(1/sv_r) V_r^T (:180-187)

 protected:
  LinearSolverOptions _lopt;
  std::ptrdiff_t _svdRank = -1;
  double _svdTolerance = -1.0, _svGap = -1.0;
  std::vector<double> _sv, _V;
};

/// MarginalLinearSystemSolver on one MI355X: build / cost / update through GpuLinearSystemSolver, the
/// solve through kb_solve_marginal (k_marg: Jacobi SVD of the column-scaled Omega in LDS).
class GpuMarginalLinearSolver : public MarginalLinearSystemSolver {
 public:
  explicit GpuMarginalLinearSolver(const LinearSolverOptions& o = LinearSolverOptions(),
                                   const GpuOptions& g = GpuOptions());
  void initMatrixStructure(const CalibrationProblem& problem, bool useDiagonalConditioner) override;
  double evaluateError(size_t nThreads, bool useMEstimator) override { return _g.evaluateError(nThreads, useMEstimator); }
  void buildSystem(size_t nThreads, bool useMEstimator) override {
    _analyzed = false;
    _g.buildSystem(nThreads, useMEstimator);
  }
  void setConstantConditioner(double d) override { LinearSystemSolver::setConstantConditioner(d); }  // ignored (:247-280)
  bool solveSystem(std::vector<double>& outDx) override;
  std::string name() const override { return "kalibr_hip_marginal_svd"; }
  const std::vector<double>& rhs() const override { return _g.rhs(); }
  double rhsJtJrhs() override { return _g.rhsJtJrhs(); }
  double applyStateUpdate(const std::vector<double>& dx) override { return _g.applyStateUpdate(dx); }
  void revertLastStateUpdate() override { _g.revertLastStateUpdate(); }
  std::vector<double> state() const override { return _g.state(); }
  void analyzeMarginal() override;
  bool appendFrames(const CalibrationProblem& problem, size_t firstFrame) override;
  bool dropLastFrames(size_t n, const std::vector<double>& state) override;
  bool optimizeDevice(const Optimizer2Options& o, SolutionReturnValue& out) override;
  GpuLinearSystemSolver& gpu() { return _g; }
  /// false: optimizeDevice declines and the IncrementalEstimator drives the per-call host loop (parity / timing)
  bool deviceLoop = true;
  /// the device loop's launches: eager (default) or captured pass graphs, and the passes between host checks of the
  /// loop state (0: the library default).  The estimator appends frames every batch, which voids the graphs: over
  /// configs[1]'s 500 batches eager launches with a check every 2 passes take 0.35 s, recaptured graphs 0.61 s
  bool useGraph = false;
  int syncEvery = 2;
  /// the device loop also analyses the last build before its one host sync (kb_optimize_marginal_analyze); the next
  /// analyzeMarginal() then takes that result instead of a second call
  bool fuseAnalyze = true;

 private:
  GpuLinearSystemSolver _g;
  bool _analyzed = false;  // _asv / _aV / _ainfo hold analyzeMarginal's result for the current system
  std::vector<double> _asv, _aV;
  int _aRank = -1;
  double _aTol = 0.0, _aGap = 0.0;
};

// ---------------------------------------------------------------- trust-region policies
class TrustRegionPolicy {
 public:
  virtual ~TrustRegionPolicy() = default;
  /// called by the optimizer when an optimization is starting (TrustRegionPolicy.cpp:29-37)
  void optimizationStarting(double J);
  /// TrustRegionPolicy::solveSystem (TrustRegionPolicy.cpp:39-52): true if the solution was successful
  bool solveSystem(double J, bool previousIterationFailed, int nThreads, std::vector<double>& outDx);
  std::shared_ptr<LinearSystemSolver> getSolver() { return _solver; }
  virtual void setSolver(std::shared_ptr<LinearSystemSolver> solver) { _solver = std::move(solver); }
  virtual bool revertOnFailure() { return true; }
  virtual std::ostream& printState(std::ostream& out) const = 0;
  virtual std::string name() const = 0;
  virtual bool requiresAugmentedDiagonal() const = 0;

 protected:
  double get_dJ() const { return _p_J - _J; }
  bool isFirstIteration() const { return _isFirstIteration; }
  virtual void optimizationStartingImplementation(double J) = 0;
  virtual bool solveSystemImplementation(double J, bool previousIterationFailed, int nThreads,
                                         std::vector<double>& outDx) = 0;
  std::shared_ptr<LinearSystemSolver> _solver;

 private:
  double _J = 0.0, _p_J = 0.0, _last_successful_J = 0.0;
  bool _isFirstIteration = true;
};

class LevenbergMarquardtTrustRegionPolicy : public TrustRegionPolicy {
 public:
  LevenbergMarquardtTrustRegionPolicy() : _lambdaInit(1e-3) {}
  explicit LevenbergMarquardtTrustRegionPolicy(double lambdaInit) : _lambdaInit(lambdaInit) {}
  bool revertOnFailure() override { return true; }
  std::ostream& printState(std::ostream& out) const override;
  std::string name() const override { return "levenberg_marquardt"; }
  bool requiresAugmentedDiagonal() const override { return true; }
  double lambdaInit() const { return _lambdaInit; }
  double lambda() const { return _lambda; }

 protected:
  void optimizationStartingImplementation(double J) override;
  bool solveSystemImplementation(double J, bool previousIterationFailed, int nThreads,
                                 std::vector<double>& outDx) override;

 private:
  double getLmRho();
  std::vector<double> _dx;
  double _lambdaInit, _gammaInit = 3, _betaInit = 2, _muInit = 2;
  int _pInit = 3;
  double _lambda = 0, _gamma = 0, _beta = 0, _mu = 0;
  int _p = 0;
};

class GaussNewtonTrustRegionPolicy : public TrustRegionPolicy {
 public:
  bool revertOnFailure() override { return false; }
  std::ostream& printState(std::ostream& out) const override { return out << "GN"; }
  std::string name() const override { return "gauss_newton"; }
  bool requiresAugmentedDiagonal() const override { return false; }

 protected:
  void optimizationStartingImplementation(double) override {}
  bool solveSystemImplementation(double J, bool previousIterationFailed, int nThreads,
                                 std::vector<double>& outDx) override;
};

// ---------------------------------------------------------------- optimizer
struct Optimizer2Options {  // Optimizer2Options.hpp:9-42 (defaults kept)
  double convergenceDeltaJ = 1e-3;
  double convergenceDeltaX = 1e-3;
  int maxIterations = 20;
  bool verbose = false;
  int linearSolverMaximumFails = 0;
  int nThreads = 4;
  std::shared_ptr<LinearSystemSolver> linearSystemSolver;
  std::shared_ptr<TrustRegionPolicy> trustRegionPolicy;
};

class Optimizer2 {
 public:
  using Exception = LinearSystemSolver::Exception;
  explicit Optimizer2(const Optimizer2Options& options);
  /// host-driven loop, Optimizer2.cpp:183-273 statement by statement (any LinearSystemSolver)
  SolutionReturnValue optimize();
  /// the same loop device-resident (GpuLinearSystemSolver with an LM or GN policy): one captured graph per
  /// pass, the host only polls the done flag every `syncEvery` passes
  SolutionReturnValue optimizeOnDevice(int syncEvery = 0);
  const Optimizer2Options& options() const { return _options; }
  /// per-pass [J, lambda, deltaX, accepted] of the last optimizeOnDevice()
  const std::vector<double>& trace() const { return _trace; }

 private:
  Optimizer2Options _options;
  std::vector<double> _dx;
  std::vector<double> _trace;
};

// ---------------------------------------------------------------- incremental estimator
/// One batch = one synchronized set of views: a new target pose (frame) and its observations
/// (CreateBatchProblem, CalibrationTools.hpp:440-521; CalibrateCameras.cpp:302-307).
struct CalibrationBatch {
  std::vector<double> frame_pose;    // 7: initial T_t_c guess of the frame (q xyzw | t), state layout
  std::vector<uint8_t> view_cam;     // [n_views]
  std::vector<uint32_t> view_offset; // [n_views + 1]
  std::vector<uint16_t> corner_id;   // [n_corners]
  std::vector<double> y;             // [n_corners][2]
};

/// IncrementalEstimator (IncrementalEstimator.cpp:44-77, 337-530): adds batches one at a time, optimizes the
/// accumulated problem with Optimizer2 + GaussNewtonTrustRegionPolicy over the marginal linear solver, and
/// keeps a batch only if it raises the information of the camera block (0.5 * delta sum log2 sv >
/// infoGainDelta) or its SVD rank, on a valid solution.  A rejected batch is removed and the design
/// variables restored.  The calibration group (cameras + baselines) takes the role of _margGroupId.
struct IncrementalEstimatorOptions {  // IncrementalEstimator.h:83-95
  double infoGainDelta = 0.2;
  bool checkValidity = false;
  bool verbose = false;
};

class IncrementalEstimator {
 public:
  using Options = IncrementalEstimatorOptions;
  struct ReturnValue {  // IncrementalEstimator.h:97-142 (the QR fields have no counterpart)
    bool batchAccepted = false;
    double informationGain = 0.0;
    std::ptrdiff_t rankTheta = -1, rankThetaDeficiency = -1;
    double svdTolerance = 0.0;
    std::vector<double> singularValues, singularValuesScaled;
    std::vector<double> nobsBasis, obsBasis, sigma2Theta;  // unscaled (analyzeMarginal), row-major [C][.]
    size_t numIterations = 0;
    double JStart = 0.0, JFinal = 0.0, elapsedTime = 0.0;
  };

  /// `base` holds the cameras, the target and the initial calibration state (intrinsics + baselines) and no
  /// frames; `solver` is the marginal solver the optimizer uses (GpuMarginalLinearSolver on the device).
  IncrementalEstimator(const CalibrationProblem& base, std::shared_ptr<MarginalLinearSystemSolver> solver,
                       const Options& options = Options(), const Optimizer2Options& optimizerOptions = Optimizer2Options());
  ReturnValue addBatch(const CalibrationBatch& batch, bool force = false);
  /// the accumulated problem of the accepted batches with the current design-variable values
  const CalibrationProblem& getProblem() const { return _problem; }
  size_t getNumBatches() const { return (size_t)_problem.n_frames; }
  double getInformationGain() const { return _informationGain; }
  std::ptrdiff_t getRankTheta() const { return _rankTheta; }
  double getSvLog2Sum() const { return _svLog2Sum; }
  const Options& getOptions() const { return _options; }
  /// host seconds spent per phase over all addBatch calls: append / initMatrixStructure, optimize, state read-back,
  /// analyzeMarginal, the host bookkeeping, the drop of a rejected batch
  double profile[6] = {0, 0, 0, 0, 0, 0};

 private:
  void appendBatch(const CalibrationBatch& b);
  void removeLastBatch(size_t n_views, size_t n_corners);
  Options _options;
  Optimizer2Options _optOptions;
  std::shared_ptr<MarginalLinearSystemSolver> _solver;
  CalibrationProblem _problem;
  double _informationGain = 0.0, _svLog2Sum = 0.0, _svdTolerance = 0.0;
  std::ptrdiff_t _rankTheta = -1, _rankThetaDeficiency = -1;
  double _initialCost = 0.0, _finalCost = 0.0;
};

}  // namespace backend
}  // namespace kalibr_amd
