// kalibr_backend.cpp -- host layer over the kalibr_hip C-ABI (see kalibr_backend.hpp for the reference map).
#include "kalibr_backend.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <iostream>

#include "kalibr_hip.h"

namespace kalibr_amd {
namespace backend {

// ---------------------------------------------------------------- LinearSystemSolver defaults
void LinearSystemSolver::setConditioner(const std::vector<double>& diag) {
  if (diag.size() != _JCols)  // LinearSystemSolver.cpp:98-102
    throw Exception("The diagonal conditioner must have the same number of rows as the Hessian matrix");
  _diagonalConditioner = diag;
}

void LinearSystemSolver::setConstantConditioner(double diag) {
  _diagonalConditioner.assign(_JCols, diag);  // LinearSystemSolver.cpp:104-107
}

// ---------------------------------------------------------------- design variables and error terms
namespace {
using Kind = DesignVariable::Kind;

// projection | distortion DV sizes of a camera model (CameraDesignVariable)
void dv_split(int model, int* a, int* b) {
  switch (model) {
    case KB_OMNI_RADTAN: *a = 5, *b = 4; break;
    case KB_EUCM: *a = 6, *b = 0; break;
    case KB_OMNI: *a = 5, *b = 0; break;
    case KB_DS: *a = 6, *b = 0; break;
    case KB_PINHOLE_FOV: *a = 4, *b = 1; break;
    case KB_PINHOLE_RADTAN:
    case KB_PINHOLE_EQUI: *a = 4, *b = 4; break;
    default: throw LinearSystemSolver::Exception("unknown camera model");
  }
}

void need(bool c, const std::string& m) {
  if (!c) throw LinearSystemSolver::Exception("initMatrixStructure: " + m);
}
}  // namespace

int DesignVariable::minimalDimensions() const {
  switch (kind) {
    case Kind::Projection:
    case Kind::Distortion: return (int)value.size();
    case Kind::RotationQuaternion:
    case Kind::EuclideanPoint:
    case Kind::HomogeneousPoint: return 3;
  }
  return 0;
}

std::vector<DesignVariable*> assignColumnBases(const std::vector<DesignVariable*>& dvs) {
  std::vector<DesignVariable*> act;
  for (DesignVariable* dv : dvs)
    if (dv && dv->isActive()) act.push_back(dv);
  int columnBase = 0;
  for (size_t i = 0; i < act.size(); ++i) {
    act[i]->blockIndex = (int)i;
    act[i]->columnBase = columnBase;
    columnBase += act[i]->minimalDimensions();
  }
  return act;
}

TermAssembly assembleTerms(const std::vector<DesignVariable*>& dvs, const std::vector<ReprojectionErrorTerm*>& errors,
                           const std::vector<double>& target) {
  need(!errors.empty(), "no error terms");
  need(target.size() % 3 == 0 && !target.empty(), "target must be [n][3]");
  TermAssembly a;
  // the rig: cameras, baselines and frames the terms read
  int N = 0;
  for (const ReprojectionErrorTerm* e : errors) {
    need(e && e->projection && e->targetRotation && e->targetTranslation, "term without its design variables");
    need(e->camera >= 0 && e->camera < KB_MAX_CAMS, "camera index out of range");
    N = std::max(N, e->camera + 1);
  }
  a.projection.assign(N, nullptr);
  a.distortion.assign(N, nullptr);
  a.baseRotation.assign(std::max(N - 1, 0), nullptr);
  a.baseTranslation.assign(std::max(N - 1, 0), nullptr);
  std::vector<DesignVariable*> rots;  // frames, by first appearance
  for (const ReprojectionErrorTerm* e : errors) {
    const int c = e->camera;
    need(e->projection->kind == Kind::Projection && e->projection->camera == c, "projection DV of another camera");
    need(!a.projection[c] || a.projection[c] == e->projection, "two projection DVs for one camera");
    a.projection[c] = e->projection;
    need(!e->distortion || (e->distortion->kind == Kind::Distortion && e->distortion->camera == c),
         "distortion DV of another camera");
    need(!a.distortion[c] || a.distortion[c] == e->distortion, "two distortion DVs for one camera");
    a.distortion[c] = e->distortion;
    need(e->baselines.size() == 2 * (size_t)c, "pose chain is not B_{c-1} .. B_0 T^-1");
    for (int j = 0; j < c; ++j) {
      DesignVariable *r = e->baselines[2 * j], *t = e->baselines[2 * j + 1];
      need(r && t && r->kind == Kind::RotationQuaternion && t->kind == Kind::EuclideanPoint, "baseline DV kinds");
      need(!a.baseRotation[j] || (a.baseRotation[j] == r && a.baseTranslation[j] == t), "inconsistent baselines");
      a.baseRotation[j] = r;
      a.baseTranslation[j] = t;
    }
    need(e->targetRotation->kind == Kind::RotationQuaternion && e->targetTranslation->kind == Kind::EuclideanPoint,
         "target pose DV kinds");
    need(e->cornerId >= 0 && 3 * (size_t)e->cornerId < target.size(), "corner id outside the target");
    if (std::find(rots.begin(), rots.end(), e->targetRotation) == rots.end()) rots.push_back(e->targetRotation);
  }
  for (int c = 0; c < N; ++c) need(a.projection[c] != nullptr, "a camera without terms");
  for (int j = 0; j + 1 < N; ++j) need(a.baseRotation[j] != nullptr, "a baseline no term reads");
  // frames in the order of their rotation DVs' columns; every active DV must be one the terms read
  std::vector<DesignVariable*> act;
  for (DesignVariable* dv : dvs)
    if (dv && dv->isActive()) act.push_back(dv);
  std::sort(rots.begin(), rots.end(),
            [](const DesignVariable* x, const DesignVariable* y) { return x->columnBase < y->columnBase; });
  const int F = (int)rots.size();
  std::vector<int> frame_of_rot;  // by rots index
  a.frameRotation = rots;
  a.frameTranslation.assign(F, nullptr);
  for (const ReprojectionErrorTerm* e : errors) {
    const int f = (int)(std::lower_bound(rots.begin(), rots.end(), e->targetRotation,
                                         [](const DesignVariable* x, const DesignVariable* y) {
                                           return x->columnBase < y->columnBase;
                                         }) - rots.begin());
    need(!a.frameTranslation[f] || a.frameTranslation[f] == e->targetTranslation, "inconsistent target pose");
    a.frameTranslation[f] = e->targetTranslation;
  }
  // canonical columns -> caller columns
  CalibrationProblem& p = a.problem;
  p.n_frames = F;
  p.target = target;
  std::vector<const DesignVariable*> order;  // canonical DV sequence
  for (int c = 0; c < N; ++c) {
    int na = 0, nb = 0;
    dv_split(a.projection[c]->cameraModel, &na, &nb);
    need((int)a.projection[c]->value.size() == na, "projection DV size does not match the camera model");
    need(nb == 0 ? a.distortion[c] == nullptr : (a.distortion[c] && (int)a.distortion[c]->value.size() == nb),
         "distortion DV does not match the camera model");
    p.cam_model.push_back(a.projection[c]->cameraModel);
    order.push_back(a.projection[c]);
    if (a.distortion[c]) order.push_back(a.distortion[c]);
  }
  for (int j = 0; j + 1 < N; ++j) {
    order.push_back(a.baseRotation[j]);
    order.push_back(a.baseTranslation[j]);
  }
  for (int f = 0; f < F; ++f) {
    order.push_back(a.frameRotation[f]);
    order.push_back(a.frameTranslation[f]);
  }
  size_t ncols_caller = 0;
  for (const DesignVariable* dv : act) ncols_caller += dv->minimalDimensions();
  for (const DesignVariable* dv : order) {
    need(dv->isActive() && dv->columnBase >= 0, "a design variable the terms read is inactive or has no column base");
    for (int k = 0; k < dv->minimalDimensions(); ++k) a.perm.push_back(dv->columnBase + k);
  }
  need(a.perm.size() == ncols_caller, "active design variables that no term reads (the device solves [intrinsics | "
                                      "baselines | target poses] only)");
  {
    std::vector<char> seen(ncols_caller, 0);
    for (int q : a.perm) {
      need(q >= 0 && (size_t)q < ncols_caller && !seen[q], "overlapping column bases");
      seen[q] = 1;
    }
  }
  // views: the terms of (frame, camera) in their given order, views sorted by frame then camera
  std::vector<std::vector<std::vector<const ReprojectionErrorTerm*>>> vt(F, std::vector<std::vector<const ReprojectionErrorTerm*>>(N));
  for (const ReprojectionErrorTerm* e : errors) {
    const int f = (int)(std::find(rots.begin(), rots.end(), e->targetRotation) - rots.begin());
    vt[f][e->camera].push_back(e);
  }
  p.view_offset.push_back(0);
  for (int f = 0; f < F; ++f)
    for (int c = 0; c < N; ++c) {
      if (vt[f][c].empty()) continue;
      for (const ReprojectionErrorTerm* e : vt[f][c]) {
        p.corner_id.push_back((uint16_t)e->cornerId);
        p.y.push_back(e->y[0]);
        p.y.push_back(e->y[1]);
      }
      p.view_frame.push_back((uint32_t)f);
      p.view_cam.push_back((uint8_t)c);
      p.view_offset.push_back((uint32_t)p.corner_id.size());
    }
  // state from the DV values
  p.state.assign((size_t)N * KB_MAX_INTR + 7 * (size_t)(N - 1) + 7 * (size_t)F, 0.0);
  for (int c = 0; c < N; ++c) {
    const std::vector<double>& pv = a.projection[c]->value;
    std::copy(pv.begin(), pv.end(), p.state.begin() + (size_t)c * KB_MAX_INTR);
    if (a.distortion[c])
      std::copy(a.distortion[c]->value.begin(), a.distortion[c]->value.end(),
                p.state.begin() + (size_t)c * KB_MAX_INTR + pv.size());
  }
  auto put_pose = [&](size_t o, const DesignVariable* r, const DesignVariable* t) {
    need(r->value.size() == 4 && t->value.size() == 3, "pose DV values must be a quaternion and a point");
    std::copy(r->value.begin(), r->value.end(), p.state.begin() + o);
    std::copy(t->value.begin(), t->value.end(), p.state.begin() + o + 4);
  };
  const size_t ob = (size_t)N * KB_MAX_INTR, of = ob + 7 * (size_t)(N - 1);
  for (int j = 0; j + 1 < N; ++j) put_pose(ob + 7 * j, a.baseRotation[j], a.baseTranslation[j]);
  for (int f = 0; f < F; ++f) put_pose(of + 7 * f, a.frameRotation[f], a.frameTranslation[f]);
  return a;
}

void pullDesignVariables(const TermAssembly& a, const std::vector<double>& state) {
  const size_t N = a.projection.size(), F = a.frameRotation.size();
  if (state.size() != N * KB_MAX_INTR + 7 * (N - 1) + 7 * F)
    throw LinearSystemSolver::Exception("pullDesignVariables: state size mismatch");
  for (size_t c = 0; c < N; ++c) {
    std::vector<double>& pv = a.projection[c]->value;
    std::copy(state.begin() + c * KB_MAX_INTR, state.begin() + c * KB_MAX_INTR + pv.size(), pv.begin());
    if (a.distortion[c]) {
      std::vector<double>& dv = a.distortion[c]->value;
      const size_t o = c * KB_MAX_INTR + pv.size();
      std::copy(state.begin() + o, state.begin() + o + dv.size(), dv.begin());
    }
  }
  auto get_pose = [&](size_t o, DesignVariable* r, DesignVariable* t) {
    std::copy(state.begin() + o, state.begin() + o + 4, r->value.begin());
    std::copy(state.begin() + o + 4, state.begin() + o + 7, t->value.begin());
  };
  const size_t ob = N * KB_MAX_INTR, of = ob + 7 * (N - 1);
  for (size_t j = 0; j + 1 < N; ++j) get_pose(ob + 7 * j, a.baseRotation[j], a.baseTranslation[j]);
  for (size_t f = 0; f < F; ++f) get_pose(of + 7 * f, a.frameRotation[f], a.frameTranslation[f]);
}

TermLinearSystemSolver::TermLinearSystemSolver(std::shared_ptr<ProblemLinearSystemSolver> inner,
                                               std::vector<double> target)
    : _inner(std::move(inner)), _target(std::move(target)) {
  if (!_inner) throw Exception("TermLinearSystemSolver: null inner solver");
}

void TermLinearSystemSolver::initMatrixStructure(const std::vector<DesignVariable*>& dvs,
                                                 const std::vector<ReprojectionErrorTerm*>& errors,
                                                 bool useDiagonalConditioner) {
  _a = assembleTerms(dvs, errors, _target);
  _inner->initMatrixStructure(_a.problem, useDiagonalConditioner);
  _JRows = _inner->JRows();
  _JCols = _inner->JCols();
  if (_JCols != _a.perm.size()) throw Exception("initMatrixStructure: column count mismatch");
  _rhs.assign(_JCols, 0.0);
  _diagonalConditioner.assign(_JCols, 0.0);
}

double TermLinearSystemSolver::evaluateError(size_t nThreads, bool useMEstimator) {
  return _inner->evaluateError(nThreads, useMEstimator);
}

void TermLinearSystemSolver::buildSystem(size_t nThreads, bool useMEstimator) {
  _inner->buildSystem(nThreads, useMEstimator);
}

void TermLinearSystemSolver::setConditioner(const std::vector<double>& diag) {
  LinearSystemSolver::setConditioner(diag);
  std::vector<double> dc(_JCols);
  for (size_t k = 0; k < _JCols; ++k) dc[k] = diag[_a.perm[k]];
  _inner->setConditioner(dc);
}

void TermLinearSystemSolver::setConstantConditioner(double diag) {
  LinearSystemSolver::setConstantConditioner(diag);
  _inner->setConstantConditioner(diag);
}

bool TermLinearSystemSolver::solveSystem(std::vector<double>& outDx) {
  std::vector<double> dc;
  if (!_inner->solveSystem(dc)) return false;
  outDx.assign(_JCols, 0.0);
  for (size_t k = 0; k < _JCols; ++k) outDx[_a.perm[k]] = dc[k];
  return true;
}

const std::vector<double>& TermLinearSystemSolver::rhs() const {
  const std::vector<double>& rc = _inner->rhs();
  _rhs_caller.assign(_JCols, 0.0);
  for (size_t k = 0; k < _JCols && k < rc.size(); ++k) _rhs_caller[_a.perm[k]] = rc[k];
  return _rhs_caller;
}

double TermLinearSystemSolver::applyStateUpdate(const std::vector<double>& dx) {
  if (dx.size() != _JCols) throw Exception("applyStateUpdate: dx has the wrong size");
  std::vector<double> dc(_JCols);
  for (size_t k = 0; k < _JCols; ++k) dc[k] = dx[_a.perm[k]];
  return _inner->applyStateUpdate(dc);
}

void TermLinearSystemSolver::pullDesignVariables() const { backend::pullDesignVariables(_a, _inner->state()); }

// ---------------------------------------------------------------- GpuLinearSystemSolver
GpuLinearSystemSolver::GpuLinearSystemSolver(const GpuOptions& o) : _opt(o) {}

GpuLinearSystemSolver::~GpuLinearSystemSolver() {
  if (_h) kb_destroy(static_cast<kb_handle*>(_h));
}

void GpuLinearSystemSolver::check(int rc, const char* what) const {
  if (rc < 0) throw Exception(std::string(what) + ": " + kb_last_error());
}

void GpuLinearSystemSolver::initMatrixStructure(const CalibrationProblem& p, bool /*useDiagonalConditioner*/) {
  if (p.view_offset.size() != p.view_frame.size() + 1 || p.view_cam.size() != p.view_frame.size() ||
      p.y.size() != 2 * p.corner_id.size() || p.target.size() % 3 != 0)
    throw Exception("initMatrixStructure: inconsistent problem arrays");
  if (_h) {
    kb_destroy(static_cast<kb_handle*>(_h));
    _h = nullptr;
  }
  kb_layout L{};
  L.n_cams = p.n_cams();
  L.n_frames = p.n_frames;
  L.n_target = p.n_target();
  L.cam_model = p.cam_model.data();
  L.target_points = p.target.data();
  L.device = _opt.device;
  kb_handle* h = kb_create(&L);
  if (!h) throw Exception(std::string("kb_create: ") + kb_last_error());
  _h = h;
  check(kb_upload_observations(h, p.n_views(), p.n_corners(), p.y.data(), p.corner_id.data(), p.view_offset.data(),
                               p.view_frame.data(), p.view_cam.data()),
        "kb_upload_observations");
  if ((int)p.state.size() != kb_state_size(h)) throw Exception("initMatrixStructure: state size mismatch");
  check(kb_set_state_flat(h, p.state.data()), "kb_set_state_flat");
  if (_opt.linearSolver == "pcg" || _opt.linearSolver == "pcg_schur") {
    kb_pcg_options po{_opt.pcgTolerance, _opt.pcgMaxIterations, _opt.pcgAbsoluteTolerance ? 1 : 0};
    check(kb_set_linear_solver(h, _opt.linearSolver == "pcg" ? KB_SOLVER_PCG : KB_SOLVER_PCG_SCHUR, &po),
          "kb_set_linear_solver");
  } else if (_opt.linearSolver != "schur") {
    throw Exception("GpuLinearSystemSolver: unknown linearSolver " + _opt.linearSolver);
  }
  _JRows = 2 * (size_t)p.n_corners();
  _JCols = (size_t)kb_num_cols(h);
  _C = (size_t)kb_camera_cols(h);
  _F = (size_t)p.n_frames;
  _N = (size_t)p.n_cams();
  _rhs.assign(_JCols, 0.0);
  _diagonalConditioner.assign(_JCols, 0.0);
  _conditioner = 0.0;
  _built = false;
  _rhs_valid = false;
}

double GpuLinearSystemSolver::evaluateError(size_t, bool) {
  if (!_h) throw Exception("evaluateError: initMatrixStructure first");
  double J = 0.0;
  check(kb_eval_cost(static_cast<kb_handle*>(_h), &J), "kb_eval_cost");
  return J;
}

void GpuLinearSystemSolver::buildSystem(size_t, bool useMEstimator) {
  if (!_h) throw Exception("buildSystem: initMatrixStructure first");
  check(kb_build(static_cast<kb_handle*>(_h), useMEstimator ? 1 : 0), "kb_build");
  _built = true;
  _rhs_valid = false;
}

void GpuLinearSystemSolver::setConstantConditioner(double diag) {
  LinearSystemSolver::setConstantConditioner(diag);
  _conditioner = diag;
  if (_h) check(kb_set_constant_conditioner(static_cast<kb_handle*>(_h), diag), "kb_set_constant_conditioner");
}

void GpuLinearSystemSolver::setConditioner(const std::vector<double>& diag) {
  LinearSystemSolver::setConditioner(diag);
  bool constant = true;
  for (double v : diag) constant = constant && v == diag.front();
  if (constant) {  // the device's constant path (what the LM policies set, :86-88)
    setConstantConditioner(diag.empty() ? 0.0 : diag.front());
    return;
  }
  if (_h) check(kb_set_conditioner(static_cast<kb_handle*>(_h), diag.data()), "kb_set_conditioner");
}

bool GpuLinearSystemSolver::solveSystem(std::vector<double>& outDx) {
  if (!_built) throw Exception("solveSystem: buildSystem first");
  outDx.resize(_JCols);
  int ok = 0;
  check(kb_solve(static_cast<kb_handle*>(_h), outDx.data(), &ok), "kb_solve");
  return ok != 0;
}

const std::vector<double>& GpuLinearSystemSolver::rhs() const {
  if (!_rhs_valid && _h && _built) {
    auto* self = const_cast<GpuLinearSystemSolver*>(this);
    check(kb_get_rhs(static_cast<kb_handle*>(_h), self->_rhs.data()), "kb_get_rhs");
    _rhs_valid = true;
  }
  return _rhs;
}

double GpuLinearSystemSolver::rhsJtJrhs() {
  // rhs^T (J^T J) rhs of the last build, on the device from the arrow blocks (kb_rhs_jtj_rhs)
  if (!_built) throw Exception("rhsJtJrhs: buildSystem first");
  double s = 0.0;
  check(kb_rhs_jtj_rhs(static_cast<kb_handle*>(_h), &s), "kb_rhs_jtj_rhs");
  return s;
}

double GpuLinearSystemSolver::applyStateUpdate(const std::vector<double>& dx) {
  if (dx.size() != _JCols) throw Exception("applyStateUpdate: dx has the wrong size");
  double deltaX = 0.0;
  check(kb_apply_update(static_cast<kb_handle*>(_h), dx.data(), &deltaX), "kb_apply_update");
  return deltaX;
}

void GpuLinearSystemSolver::revertLastStateUpdate() { check(kb_revert(static_cast<kb_handle*>(_h)), "kb_revert"); }

int GpuLinearSystemSolver::lastPcgIterations() const {
  if (!_h || _opt.linearSolver != "pcg") return 0;
  kb_pcg_info info{};
  check(kb_get_pcg_info(static_cast<kb_handle*>(_h), &info), "kb_get_pcg_info");
  return info.iterations;
}

bool GpuLinearSystemSolver::appendFrames(const CalibrationProblem& p, size_t f0) {
  if (!_h || _F != f0 || (size_t)p.n_frames <= f0) return false;
  // the views of frames >= f0 (views are sorted by frame), renumbered from 0, offsets made local
  const size_t v0 = std::lower_bound(p.view_frame.begin(), p.view_frame.end(), (uint32_t)f0) - p.view_frame.begin();
  const size_t nv = p.view_frame.size() - v0, c0 = p.view_offset[v0], nc = p.corner_id.size() - c0;
  std::vector<uint32_t> vo(nv + 1), vf(nv);
  for (size_t v = 0; v <= nv; ++v) vo[v] = p.view_offset[v0 + v] - (uint32_t)c0;
  for (size_t v = 0; v < nv; ++v) vf[v] = p.view_frame[v0 + v] - (uint32_t)f0;
  const size_t nf = (size_t)p.n_frames - f0, so = p.state.size() - 7 * (size_t)p.n_frames;
  kb_handle* h = static_cast<kb_handle*>(_h);
  check(kb_append_frames(h, (int32_t)nf, (int32_t)nv, (int32_t)nc, p.y.data() + 2 * c0, p.corner_id.data() + c0,
                         vo.data(), vf.data(), p.view_cam.data() + v0, p.state.data() + so + 7 * f0),
        "kb_append_frames");
  if ((int)p.state.size() != kb_state_size(h)) throw Exception("appendFrames: state size mismatch");
  check(kb_set_state_flat(h, p.state.data()), "kb_set_state_flat");
  _F = (size_t)p.n_frames;
  _N = (size_t)p.n_cams();
  _JRows = 2 * (size_t)p.n_corners();
  _JCols = (size_t)kb_num_cols(h);
  _rhs.assign(_JCols, 0.0);
  _diagonalConditioner.assign(_JCols, 0.0);
  _built = false;
  _rhs_valid = false;
  return true;
}

void GpuLinearSystemSolver::dropLastFrames(size_t n, const std::vector<double>& st) {
  kb_handle* h = static_cast<kb_handle*>(_h);
  check(kb_drop_last_frames(h, (int32_t)n), "kb_drop_last_frames");
  _F -= n;
  if ((int)st.size() != kb_state_size(h)) throw Exception("dropLastFrames: state size mismatch");
  check(kb_set_state_flat(h, st.data()), "kb_set_state_flat");
  _JCols = (size_t)kb_num_cols(h);
  _rhs.assign(_JCols, 0.0);
  _diagonalConditioner.assign(_JCols, 0.0);
  _built = false;
  _rhs_valid = false;
}

std::vector<double> GpuLinearSystemSolver::state() const {
  std::vector<double> s((size_t)kb_state_size(static_cast<kb_handle*>(_h)));
  check(kb_get_state_flat(static_cast<kb_handle*>(_h), s.data()), "kb_get_state_flat");
  return s;
}

std::vector<std::array<double, 6>> GpuLinearSystemSolver::reprojectionErrorStatistics() {
  if (!_h) throw Exception("reprojectionErrorStatistics: initMatrixStructure first");
  kb_handle* h = static_cast<kb_handle*>(_h);
  std::vector<std::array<double, 6>> out(_N);
  check(kb_reprojection_error_stats(h, out[0].data()), "kb_reprojection_error_stats");
  return out;
}

void GpuLinearSystemSolver::setState(const std::vector<double>& s) {
  if ((int)s.size() != kb_state_size(static_cast<kb_handle*>(_h))) throw Exception("setState: size mismatch");
  check(kb_set_state_flat(static_cast<kb_handle*>(_h), s.data()), "kb_set_state_flat");
  _built = false;
}

// ---------------------------------------------------------------- TrustRegionPolicy (TrustRegionPolicy.cpp)
void TrustRegionPolicy::optimizationStarting(double J) {
  _J = J;
  _p_J = J;
  _last_successful_J = J;
  _isFirstIteration = true;
  optimizationStartingImplementation(J);
}

bool TrustRegionPolicy::solveSystem(double J, bool previousIterationFailed, int nThreads, std::vector<double>& outDx) {
  if (previousIterationFailed) {
    _J = J;
  } else {
    _p_J = _last_successful_J;
    _last_successful_J = J;
    _J = J;
  }
  const bool success = solveSystemImplementation(J, previousIterationFailed, nThreads, outDx);
  _isFirstIteration = false;
  return success;
}

// ---------------------------------------------------------------- LM (LevenbergMarquardtTrustRegionPolicy.cpp)
void LevenbergMarquardtTrustRegionPolicy::optimizationStartingImplementation(double) {
  _lambda = _lambdaInit;
  _gamma = _gammaInit;
  _beta = _betaInit;
  _p = _pInit;
  _mu = _muInit;
}

bool LevenbergMarquardtTrustRegionPolicy::solveSystemImplementation(double, bool previousIterationFailed, int nThreads,
                                                                    std::vector<double>& outDx) {
  if (!_solver) throw LinearSystemSolver::Exception("The solver is null");
  if (isFirstIteration()) {
    _solver->buildSystem(nThreads, true);
  } else {
    const double rho = getLmRho();
    if (previousIterationFailed) {  // the last step was a regression
      _mu *= 2;
      _lambda *= _mu;
    } else if (rho <= 0) {  // no rebuild, only a new conditioner
      _mu *= 10;
      _lambda *= _mu;
    } else {  // success: rebuild
      _solver->buildSystem(nThreads, true);
      if (_lambda > 1e-16) {
        const double u1 = 1 / _gamma;
        const double u2 = 1 - (_beta - 1) * std::pow((2 * rho - 1), _p);
        if (u1 > u2)
          _lambda *= u1;
        else
          _lambda *= u2;
        _mu = _beta;
      } else {
        _lambda = 1e-15;
      }
    }
  }
  _solver->setConstantConditioner(_lambda);
  const bool success = _solver->solveSystem(_dx);
  outDx = _dx;
  return success;
}

double LevenbergMarquardtTrustRegionPolicy::getLmRho() {
  const double d1 = get_dJ();
  // L(0) - L(h) = dx^T (lambda dx + rhs)   (:107-113: lambda, not lambda^2)
  const std::vector<double>& r = _solver->rhs();
  double d2 = 0.0;
  for (size_t i = 0; i < _dx.size(); ++i) d2 += _dx[i] * (_lambda * _dx[i] + r[i]);
  return d1 / d2;
}

std::ostream& LevenbergMarquardtTrustRegionPolicy::printState(std::ostream& out) const {
  return out << "LM - lambda:" << _lambda << " mu:" << _mu;
}

// ---------------------------------------------------------------- GN (GaussNewtonTrustRegionPolicy.cpp:18-24)
bool GaussNewtonTrustRegionPolicy::solveSystemImplementation(double, bool, int nThreads, std::vector<double>& outDx) {
  _solver->buildSystem(nThreads, true);
  return _solver->solveSystem(outDx);
}

// ---------------------------------------------------------------- Optimizer2 (Optimizer2.cpp:183-273)
Optimizer2::Optimizer2(const Optimizer2Options& options) : _options(options) {}

SolutionReturnValue Optimizer2::optimize() {
  auto solver = _options.linearSystemSolver;
  auto policy = _options.trustRegionPolicy;
  if (!solver) throw Exception("The solver is null");
  if (!policy) throw Exception("The trust region policy is null");
  SolutionReturnValue srv;
  double J = solver->evaluateError(_options.nThreads, true);
  double p_J = J;
  srv.JStart = p_J;
  double deltaX = _options.convergenceDeltaX + 1.0;
  double deltaJ = _options.convergenceDeltaJ + 1.0;
  bool previousIterationFailed = false;
  bool linearSolverFailure = false;
  policy->setSolver(solver);
  policy->optimizationStarting(J);
  while (srv.iterations < _options.maxIterations && srv.failedIterations < _options.maxIterations &&
         ((deltaX > _options.convergenceDeltaX && std::fabs(deltaJ) > _options.convergenceDeltaJ) ||
          linearSolverFailure)) {
    const bool solutionSuccess = policy->solveSystem(J, previousIterationFailed, _options.nThreads, _dx);
    if (!solutionSuccess) {
      if (_options.verbose) std::cout << "[WARNING] System solution failed\n";
      previousIterationFailed = true;
      linearSolverFailure = true;
      srv.failedIterations++;
    } else {
      deltaX = solver->applyStateUpdate(_dx);
      J = solver->evaluateError(_options.nThreads, true);
      deltaJ = p_J - J;
      if (policy->revertOnFailure()) {
        if (deltaJ < 0.0) {
          if (_options.verbose) std::cout << "Last step was a regression. Reverting\n";
          solver->revertLastStateUpdate();
          srv.failedIterations++;
          previousIterationFailed = true;
        } else {
          p_J = J;
          previousIterationFailed = false;
        }
      } else {
        p_J = J;
      }
      srv.iterations++;
      if (_options.verbose) {
        std::cout << "[" << srv.iterations << "]: J: " << J << ", dJ: " << deltaJ << ", deltaX: " << deltaX << ", ";
        policy->printState(std::cout);
        std::cout << std::endl;
      }
    }
  }
  srv.JFinal = p_J;
  srv.dXFinal = deltaX;
  srv.dJFinal = deltaJ;
  srv.linearSolverFailure = linearSolverFailure;
  return srv;
}

SolutionReturnValue Optimizer2::optimizeOnDevice(int syncEvery) {
  // the GPU solver itself, or behind the design-variable / error-term layer (the device runs the canonical problem;
  // the caller pulls the optimised values into its design variables)
  GpuLinearSystemSolver* gpu = dynamic_cast<GpuLinearSystemSolver*>(_options.linearSystemSolver.get());
  if (!gpu)
    if (auto* ts = dynamic_cast<TermLinearSystemSolver*>(_options.linearSystemSolver.get()))
      gpu = dynamic_cast<GpuLinearSystemSolver*>(&ts->inner());
  if (!gpu) throw Exception("optimizeOnDevice: the linear system solver is not a GpuLinearSystemSolver");
  auto policy = _options.trustRegionPolicy;
  if (!policy) throw Exception("The trust region policy is null");
  kb_optimizer_options o{};
  if (auto lm = std::dynamic_pointer_cast<LevenbergMarquardtTrustRegionPolicy>(policy)) {
    o.policy = 0;
    o.lambda_init = lm->lambdaInit();
  } else if (std::dynamic_pointer_cast<GaussNewtonTrustRegionPolicy>(policy)) {
    o.policy = 1;
  } else {
    throw Exception("optimizeOnDevice: only the LM and GN policies run device-resident");
  }
  o.max_iterations = _options.maxIterations;
  o.convergence_dx = _options.convergenceDeltaX;
  o.convergence_dj = _options.convergenceDeltaJ;
  o.sync_every = syncEvery;
  o.use_graph = 1;
  kb_solution s{};
  auto* h = static_cast<kb_handle*>(gpu->handle());
  if (kb_optimize(h, &o, &s) < 0) throw Exception(std::string("kb_optimize: ") + kb_last_error());
  const int cap = 2 * _options.maxIterations + 2;
  _trace.assign(4 * (size_t)cap, 0.0);
  const int n = kb_get_trace(h, _trace.data(), cap);
  if (n < 0) throw Exception(std::string("kb_get_trace: ") + kb_last_error());
  _trace.resize(4 * (size_t)n);
  SolutionReturnValue srv;
  srv.JStart = s.J_start;
  srv.JFinal = s.J_final;
  srv.dXFinal = s.dx_final;
  srv.dJFinal = s.dj_final;
  srv.iterations = s.iterations;
  srv.failedIterations = s.failed_iterations;
  srv.linearSolverFailure = s.linear_solver_failure != 0;
  return srv;
}

// ---------------------------------------------------------------- marginal solver (LinearSolver.cpp)
double MarginalLinearSystemSolver::getSingularValuesLog2Sum() const {
  if (_svdRank == -1) return 0.0;
  double s = 0.0;
  for (std::ptrdiff_t i = 0; i < _svdRank; ++i) s += std::log(_sv[(size_t)i]);
  return s / std::log(2);
}

std::vector<double> MarginalLinearSystemSolver::getNullSpace() const {
  const size_t C = _sv.size();
  if (_svdRank == -1 || (size_t)_svdRank > C) return {};
  const size_t r = (size_t)_svdRank, k = C - r;
  std::vector<double> out(C * k);
  for (size_t i = 0; i < C; ++i)
    for (size_t j = 0; j < k; ++j) out[i * k + j] = _V[i * C + r + j];
  return out;
}

std::vector<double> MarginalLinearSystemSolver::getRowSpace() const {
  const size_t C = _sv.size();
  if (_svdRank == -1 || (size_t)_svdRank > C) return {};
  const size_t r = (size_t)_svdRank;
  std::vector<double> out(C * r);
  for (size_t i = 0; i < C; ++i)
    for (size_t j = 0; j < r; ++j) out[i * r + j] = _V[i * C + j];
  return out;
}

std::vector<double> MarginalLinearSystemSolver::getCovariance() const {
  const size_t C = _sv.size();
  if (_svdRank == -1 || (size_t)_svdRank > C) return {};
  std::vector<double> out(C * C, 0.0);
  for (size_t k = 0; k < (size_t)_svdRank; ++k) {
    const double w = 1.0 / _sv[k];
    for (size_t i = 0; i < C; ++i)
      for (size_t j = 0; j < C; ++j) out[i * C + j] += _V[i * C + k] * w * _V[j * C + k];
  }
  return out;
}

GpuMarginalLinearSolver::GpuMarginalLinearSolver(const LinearSolverOptions& o, const GpuOptions& g) : _g(g) {
  _lopt = o;
}

void GpuMarginalLinearSolver::initMatrixStructure(const CalibrationProblem& p, bool useDiagonalConditioner) {
  _analyzed = false;  // a changed system voids the fused analyzeMarginal result
  _g.initMatrixStructure(p, useDiagonalConditioner);
  _JRows = _g.JRows();
  _JCols = _g.JCols();
  _diagonalConditioner.assign(_JCols, 0.0);
  _svdRank = -1;
  _svdTolerance = _svGap = -1.0;
  _sv.clear();
  _V.clear();
}

bool GpuMarginalLinearSolver::appendFrames(const CalibrationProblem& p, size_t firstFrame) {
  _analyzed = false;  // a changed system voids the fused analyzeMarginal result
  if (!_g.appendFrames(p, firstFrame)) return false;
  _JRows = _g.JRows();
  _JCols = _g.JCols();
  _diagonalConditioner.assign(_JCols, 0.0);
  _svdRank = -1;  // a new problem for the marginal statistics, as after initMatrixStructure
  _svdTolerance = _svGap = -1.0;
  _sv.clear();
  _V.clear();
  return true;
}

bool GpuMarginalLinearSolver::dropLastFrames(size_t n, const std::vector<double>& st) {
  _analyzed = false;  // a changed system voids the fused analyzeMarginal result
  _g.dropLastFrames(n, st);
  _JRows = _g.JRows();
  _JCols = _g.JCols();
  _diagonalConditioner.assign(_JCols, 0.0);
  return true;
}

static kb_marginal_options marg_opts(const LinearSolverOptions& o);

bool GpuMarginalLinearSolver::optimizeDevice(const Optimizer2Options& oo, SolutionReturnValue& srv) {
  if (!deviceLoop || !_g.handle() || _g.cameraCols() > 112) return false;
  kb_optimizer_options o{};
  o.policy = 1;  // GaussNewtonTrustRegionPolicy (IncrementalEstimator.cpp:66-71)
  o.max_iterations = oo.maxIterations;
  o.convergence_dx = oo.convergenceDeltaX;
  o.convergence_dj = oo.convergenceDeltaJ;
  o.sync_every = syncEvery;
  o.use_graph = useGraph ? 1 : 0;
  kb_marginal_options m = marg_opts(_lopt);
  kb_solution s{};
  kb_marginal_info inf{};
  const size_t C = _g.cameraCols();
  _sv.resize(C);
  _V.resize(C * C);
  _analyzed = false;
  if (fuseAnalyze) {
    kb_marginal_info ainf{};
    _asv.resize(C);
    _aV.resize(C * C);
    if (kb_optimize_marginal_analyze(static_cast<kb_handle*>(_g.handle()), &o, &m, &s, &inf, _sv.data(), _V.data(),
                                     &ainf, _asv.data(), _aV.data()) < 0)
      throw Exception(std::string("kb_optimize_marginal_analyze: ") + kb_last_error());
    _aRank = ainf.rank;
    _aTol = ainf.tolerance;
    _aGap = ainf.sv_gap;
    _analyzed = true;
  } else if (kb_optimize_marginal(static_cast<kb_handle*>(_g.handle()), &o, &m, &s, &inf, _sv.data(), _V.data()) < 0) {
    throw Exception(std::string("kb_optimize_marginal: ") + kb_last_error());
  }
  _svdRank = inf.rank;
  _svdTolerance = inf.tolerance;
  _svGap = inf.sv_gap;
  srv = SolutionReturnValue{};
  srv.JStart = s.J_start;
  srv.JFinal = s.J_final;
  srv.dXFinal = s.dx_final;
  srv.dJFinal = s.dj_final;
  srv.iterations = s.iterations;
  srv.failedIterations = s.failed_iterations;
  srv.linearSolverFailure = s.linear_solver_failure != 0;
  return true;
}

static kb_marginal_options marg_opts(const LinearSolverOptions& o) {
  kb_marginal_options m{};
  m.column_scaling = o.columnScaling ? 1 : 0;
  m.eps_norm = o.epsNorm;
  m.eps_svd = o.epsSVD;
  m.svd_tol = o.svdTol;
  return m;
}

bool GpuMarginalLinearSolver::solveSystem(std::vector<double>& outDx) {
  _analyzed = false;  // a changed system voids the fused analyzeMarginal result
  const size_t C = _g.cameraCols();
  std::vector<double> dx(_JCols);
  _sv.resize(C);
  _V.resize(C * C);
  kb_marginal_options m = marg_opts(_lopt);
  kb_marginal_info inf{};
  int ok = 0;
  const int rc = kb_solve_marginal(static_cast<kb_handle*>(_g.handle()), &m, dx.data(), &ok, &inf, _sv.data(),
                                   _V.data());
  if (rc < 0) throw Exception(std::string("kb_solve_marginal: ") + kb_last_error());
  _svdRank = inf.rank;
  _svdTolerance = inf.tolerance;
  _svGap = inf.sv_gap;
  if (ok) outDx = dx;
  return ok != 0;
}

void GpuMarginalLinearSolver::analyzeMarginal() {
  const size_t C = _g.cameraCols();
  kb_marginal_info inf{};
  if (_analyzed) {  // the device loop analysed the last build already (kb_optimize_marginal_analyze)
    _sv = _asv;
    _V = _aV;
    inf.rank = _aRank;
    inf.tolerance = _aTol;
    inf.sv_gap = _aGap;
    _analyzed = false;
  } else {
    _sv.resize(C);
    _V.resize(C * C);
    kb_marginal_options m = marg_opts(_lopt);
    if (kb_analyze_marginal(static_cast<kb_handle*>(_g.handle()), &m, &inf, _sv.data(), _V.data()) < 0)
      throw Exception(std::string("kb_analyze_marginal: ") + kb_last_error());
  }
  // rank, tolerance and gap stay those of the last solve when there was one (LinearSolver.cpp:518-524)
  if (_svdRank == -1) {
    _svdRank = inf.rank;
    _svdTolerance = inf.tolerance;
    _svGap = inf.sv_gap;
  }
}

// ---------------------------------------------------------------- IncrementalEstimator
IncrementalEstimator::IncrementalEstimator(const CalibrationProblem& base,
                                           std::shared_ptr<MarginalLinearSystemSolver> solver, const Options& options,
                                           const Optimizer2Options& optimizerOptions)
    : _options(options), _optOptions(optimizerOptions), _solver(std::move(solver)), _problem(base) {
  if (!_solver) throw LinearSystemSolver::Exception("IncrementalEstimator: the linear solver is null");
  if (base.n_frames != 0 || !base.view_frame.empty())
    throw LinearSystemSolver::Exception("IncrementalEstimator: the base problem must not hold frames");
  _problem.view_offset.assign(1, 0u);
  // IncrementalEstimator.cpp:66-71: the optimizer runs the GN policy over the marginal linear solver
  _optOptions.linearSystemSolver = _solver;
  _optOptions.trustRegionPolicy = std::make_shared<GaussNewtonTrustRegionPolicy>();
}

void IncrementalEstimator::appendBatch(const CalibrationBatch& b) {
  if (b.frame_pose.size() != 7 || b.view_offset.size() != b.view_cam.size() + 1 ||
      b.y.size() != 2 * b.corner_id.size() || (b.view_offset.empty() ? 0 : b.view_offset.back()) != b.corner_id.size())
    throw LinearSystemSolver::Exception("addBatch: inconsistent batch arrays");
  const uint32_t f = (uint32_t)_problem.n_frames, c0 = (uint32_t)_problem.corner_id.size();
  for (size_t v = 0; v < b.view_cam.size(); ++v) {
    if (b.view_cam[v] >= _problem.n_cams()) throw LinearSystemSolver::Exception("addBatch: camera index out of range");
    _problem.view_frame.push_back(f);
    _problem.view_cam.push_back(b.view_cam[v]);
    _problem.view_offset.push_back(c0 + b.view_offset[v + 1]);
  }
  _problem.corner_id.insert(_problem.corner_id.end(), b.corner_id.begin(), b.corner_id.end());
  _problem.y.insert(_problem.y.end(), b.y.begin(), b.y.end());
  _problem.state.insert(_problem.state.end(), b.frame_pose.begin(), b.frame_pose.end());
  _problem.n_frames++;
}

void IncrementalEstimator::removeLastBatch(size_t n_views, size_t n_corners) {
  _problem.view_frame.resize(_problem.view_frame.size() - n_views);
  _problem.view_cam.resize(_problem.view_cam.size() - n_views);
  _problem.view_offset.resize(_problem.view_offset.size() - n_views);
  _problem.corner_id.resize(_problem.corner_id.size() - n_corners);
  _problem.y.resize(_problem.y.size() - 2 * n_corners);
  _problem.state.resize(_problem.state.size() - 7);
  _problem.n_frames--;
}

IncrementalEstimator::ReturnValue IncrementalEstimator::addBatch(const CalibrationBatch& batch, bool force) {
  const auto t0 = std::chrono::steady_clock::now();
  // insert the new batch; save the design variables in case it is rejected (:343-351)
  const std::vector<double> saved = _problem.state;
  appendBatch(batch);
  auto lap = [&, tl = t0](int k) mutable {  // the per-phase host time (profile[])
    const auto tn = std::chrono::steady_clock::now();
    profile[k] += std::chrono::duration<double>(tn - tl).count();
    tl = tn;
  };
  // Optimizer2::initialize -> initMatrixStructure over the grown problem, then optimize (:373).  The reference
  // re-initialises the whole structure; a solver that holds the accepted frames appends the new one in place
  // (kb_append_frames: only the batch's observations are uploaded) instead
  if (!_solver->appendFrames(_problem, (size_t)_problem.n_frames - 1)) _solver->initMatrixStructure(_problem, false);
  lap(0);
  // the optimisation itself: device-resident when the solver runs it (kb_optimize_marginal), else the host loop
  SolutionReturnValue srv;
  if (!_solver->optimizeDevice(_optOptions, srv)) {
    Optimizer2 optimizer(_optOptions);
    srv = optimizer.optimize();
  }
  lap(1);
  ReturnValue ret;
  ret.numIterations = (size_t)srv.iterations;
  ret.JStart = srv.JStart;
  ret.JFinal = srv.JFinal;
  if (_solver->getOptions().columnScaling) ret.singularValuesScaled = _solver->getSingularValues();  // :384-397
  const std::vector<double> state = _solver->state();
  lap(2);
  // analyze the unscaled marginal system (:400)
  _solver->analyzeMarginal();
  lap(3);
  ret.rankTheta = _solver->getSVDRank();
  ret.rankThetaDeficiency = _solver->getSVDRankDeficiency();
  ret.svdTolerance = _solver->getSVDTolerance();
  ret.nobsBasis = _solver->getNullSpace();
  ret.obsBasis = _solver->getRowSpace();
  ret.sigma2Theta = _solver->getCovariance();
  ret.singularValues = _solver->getSingularValues();
  // validity (:419-422) and information gain (:425-426)
  bool solutionValid = true;
  if (_options.checkValidity && (srv.iterations == _optOptions.maxIterations || srv.JFinal >= srv.JStart))
    solutionValid = false;
  const double svLog2Sum = _solver->getSingularValuesLog2Sum();
  ret.informationGain = 0.5 * (svLog2Sum - _svLog2Sum);
  // keep the batch on an information gain or a rank increase of a valid solution, or when forced (:463-494)
  bool keep = false;
  if (((ret.informationGain > _options.infoGainDelta || ret.rankTheta > _rankTheta) && solutionValid) || force) {
    if (ret.rankTheta < _rankTheta && _options.verbose)
      std::cerr << "IncrementalEstimator::addBatch(): WARNING: RANK GOING DOWN!" << std::endl;
    keep = true;
    _informationGain = ret.informationGain;
    _svLog2Sum = svLog2Sum;
    _svdTolerance = ret.svdTolerance;
    _rankTheta = ret.rankTheta;
    _rankThetaDeficiency = ret.rankThetaDeficiency;
    _initialCost = srv.JStart;
    _finalCost = srv.JFinal;
    _problem.state = state;
  }
  ret.batchAccepted = keep;
  if (_options.verbose)
    std::cout << "[IncrementalEstimator::addBatch] Batch #" << _problem.n_frames << " information gain "
              << ret.informationGain << " rank " << ret.rankTheta << " cost " << ret.JStart << " -> " << ret.JFinal
              << (keep ? " ACCEPTED" : " REJECTED") << std::endl;
  if (!keep) {  // restore the design variables and drop the batch (:517-527)
    removeLastBatch(batch.view_cam.size(), batch.corner_id.size());
    _problem.state = saved;
    // the solver keeps the accepted frames with their restored values for the next append (a solver that cannot, or
    // a first batch rejected, leaves frames the problem does not hold: the next addBatch re-initialises)
    lap(4);
    if (_problem.n_frames > 0) _solver->dropLastFrames(1, saved);
    lap(5);
  }
  lap(4);
  ret.elapsedTime = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return ret;
}

}  // namespace backend
}  // namespace kalibr_amd
