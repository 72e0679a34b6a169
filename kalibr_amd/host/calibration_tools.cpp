// calibration_tools.cpp -- see calibration_tools.hpp.  Paths relative to the reference repository.
#include "calibration_tools.hpp"

#include <algorithm>
#include <cmath>
#include <iostream>
#include <limits>
#include <queue>
#include <stdexcept>

#include "kalibr_hip.h"

namespace kalibr_amd {
namespace tools {

using backend::DesignVariable;
using backend::ReprojectionErrorTerm;

namespace {
// projection | distortion DV sizes of a camera model (CameraDesignVariable; the shutter DV is inactive)
void dv_split(int32_t m, int* a, int* b) {
  switch (m) {
    case KB_OMNI_RADTAN: *a = 5, *b = 4; break;
    case KB_EUCM: *a = 6, *b = 0; break;
    case KB_OMNI: *a = 5, *b = 0; break;
    case KB_DS: *a = 6, *b = 0; break;
    case KB_PINHOLE_FOV: *a = 4, *b = 1; break;
    case KB_PINHOLE_RADTAN:
    case KB_PINHOLE_EQUI: *a = 4, *b = 4; break;
    default: throw std::runtime_error("calibration tools: unknown camera model");
  }
}

// sm::kinematics quaternion helpers (JPL, [x y z w]; quaternion_algebra.cpp)
std::array<double, 4> quat_normalized(std::array<double, 4> q) {
  const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (double& v : q) v /= n;
  return q;
}

// one stage's optimisation problem as design variables and ReprojectionError terms, in insertion order
struct StageProblem {
  struct Pose {
    DesignVariable* q = nullptr;
    DesignVariable* t = nullptr;
  };
  struct Intr {
    DesignVariable* proj = nullptr;
    DesignVariable* dist = nullptr;
  };
  std::vector<std::unique_ptr<DesignVariable>> store;
  std::vector<DesignVariable*> order;
  std::vector<std::unique_ptr<ReprojectionErrorTerm>> termStore;
  std::vector<ReprojectionErrorTerm*> terms;
  size_t views = 0;

  DesignVariable* add(DesignVariable::Kind k, std::vector<double> v, int cam = -1, int model = -1) {
    store.push_back(std::make_unique<DesignVariable>());
    DesignVariable* d = store.back().get();
    d->kind = k;
    d->value = std::move(v);
    d->camera = cam;
    d->cameraModel = model;
    order.push_back(d);
    return d;
  }
  // tools::AddPoseDesignVariable (CalibrationTools.hpp:32-45): a RotationQuaternion, then an EuclideanPoint
  Pose addPose(const Transformation& T) {
    Pose p;
    p.q = add(DesignVariable::Kind::RotationQuaternion, {T.q[0], T.q[1], T.q[2], T.q[3]});
    p.t = add(DesignVariable::Kind::EuclideanPoint, {T.t[0], T.t[1], T.t[2]});
    return p;
  }
  // CameraCalibrator::AddIntrinsicDesignVariables (CameraCalibrator.hpp:116-122): projection, distortion (the shutter
  // DV is inactive and takes no columns)
  Intr addIntrinsics(const CameraCalibrator& c, int cam) {
    int a = 0, b = 0;
    dv_split(c.model, &a, &b);
    Intr r;
    r.proj = add(DesignVariable::Kind::Projection,
                 std::vector<double>(c.intrinsics.begin(), c.intrinsics.begin() + a), cam, c.model);
    if (b)
      r.dist = add(DesignVariable::Kind::Distortion,
                   std::vector<double>(c.intrinsics.begin() + a, c.intrinsics.begin() + a + b), cam);
    return r;
  }
  // AddReprojectionErrorsForView (CameraCalibrator.hpp:238-265): one term per seen corner in target order, through
  // T_cam_w = chain[c-1] .. chain[0] T^-1
  void addView(int cam, const Intr& in, const GridObservation& obs, const Pose& target, const std::vector<Pose>& chain,
               size_t K) {
    if (obs.success.size() != K) throw std::runtime_error("calibration tools: observation size != target size");
    double y[2];
    bool any = false;
    for (size_t k = 0; k < K; ++k) {
      if (!obs.imagePoint(k, y)) continue;
      termStore.push_back(std::make_unique<ReprojectionErrorTerm>());
      ReprojectionErrorTerm* e = termStore.back().get();
      e->camera = cam;
      e->cornerId = (int)k;
      e->y[0] = y[0];
      e->y[1] = y[1];
      e->targetRotation = target.q;
      e->targetTranslation = target.t;
      for (int j = 0; j < cam; ++j) {
        e->baselines.push_back(chain.at((size_t)j).q);
        e->baselines.push_back(chain.at((size_t)j).t);
      }
      e->projection = in.proj;
      e->distortion = in.dist;
      terms.push_back(e);
      any = true;
    }
    views += any ? 1 : 0;
  }
  // pose DVs no term reads (a target pose or a baseline) are decoupled blocks of the reference's system (their LM step is
  // 0 and they change neither cost nor rho): they stay out of the device problem
  std::vector<DesignVariable*> usedOrder() const {
    std::vector<const DesignVariable*> read;
    for (const ReprojectionErrorTerm* e : terms) {
      read.push_back(e->targetRotation);
      read.push_back(e->targetTranslation);
      for (const DesignVariable* b : e->baselines) read.push_back(b);
    }
    std::sort(read.begin(), read.end());
    std::vector<DesignVariable*> out;
    for (DesignVariable* d : order) {
      const bool pose = d->kind == DesignVariable::Kind::RotationQuaternion || d->kind == DesignVariable::Kind::EuclideanPoint;
      if (!pose || std::binary_search(read.begin(), read.end(), d)) out.push_back(d);
    }
    return out;
  }
  size_t frames() const {
    std::vector<const DesignVariable*> r;
    for (const ReprojectionErrorTerm* e : terms) r.push_back(e->targetRotation);
    std::sort(r.begin(), r.end());
    return (size_t)(std::unique(r.begin(), r.end()) - r.begin());
  }
};

// Optimizer2 over the stage problem; the DV values hold the optimum afterwards
StageResult run_stage(StageProblem& sp, const AprilgridTarget& target, const StageOptions& so,
                      const backend::Optimizer2Options& opt0) {
  if (!so.solver) throw std::runtime_error("calibration tools: no solver factory");
  if (sp.terms.empty()) throw std::runtime_error("calibration tools: the stage problem has no error terms");
  auto ts = std::make_shared<backend::TermLinearSystemSolver>(so.solver(), target.points());
  const std::vector<DesignVariable*> dvs = backend::assignColumnBases(sp.usedOrder());
  ts->initMatrixStructure(dvs, sp.terms, true);
  backend::Optimizer2Options opt = opt0;
  opt.linearSystemSolver = ts;
  backend::Optimizer2 optimizer(opt);
  StageResult r;
  r.ret = so.deviceLoop ? optimizer.optimizeOnDevice() : optimizer.optimize();
  ts->pullDesignVariables();
  r.frames = sp.frames();
  r.views = sp.views;
  r.terms = sp.terms.size();
  return r;
}

void pull_intrinsics(CameraCalibrator& c, const StageProblem::Intr& in) {
  std::copy(in.proj->value.begin(), in.proj->value.end(), c.intrinsics.begin());
  if (in.dist) std::copy(in.dist->value.begin(), in.dist->value.end(), c.intrinsics.begin() + in.proj->value.size());
}

Transformation pose_value(const StageProblem::Pose& p) {
  Transformation T;
  std::copy(p.q->value.begin(), p.q->value.end(), T.q.begin());
  std::copy(p.t->value.begin(), p.t->value.end(), T.t.begin());
  return T;
}

void check_cam(const CameraCalibrator& c) {
  if (c.intrinsics.size() != KB_MAX_INTR) throw std::runtime_error("calibration tools: intrinsics must hold KB_MAX_INTR values");
  int a, b;
  dv_split(c.model, &a, &b);
}
}  // namespace

bool CameraCalibrator::estimateTransformation(const GridObservation& obs, const AprilgridTarget& target,
                                              Transformation& T) const {
  return io::estimateTransformation(obs, target, model, intrinsics.data(), T);
}

backend::Optimizer2Options defaultOptimizerOptions() {
  backend::Optimizer2Options o;
  o.nThreads = 4;
  o.convergenceDeltaX = 1e-3;
  o.convergenceDeltaJ = 1;
  o.maxIterations = 200;
  o.trustRegionPolicy = std::make_shared<backend::LevenbergMarquardtTrustRegionPolicy>(10);
  return o;
}

// ---------------------------------------------------------------- CalibrateSingleCamera (CalibrationTools.hpp:93-144)
bool calibrateSingleCamera(const std::vector<GridObservation>& observations, CameraCalibrator& cam,
                           const AprilgridTarget& target, std::optional<double> fallbackFocalLength,
                           const StageOptions& so, StageResult* out) {
  check_cam(cam);
  // initializeIntrinsics: the geometry takes whatever the initialiser set (its bool is shadowed and unused, :100)
  std::vector<double> init;
  io::initializeIntrinsics(observations, target, fallbackFocalLength, cam.model, init);
  if (!init.empty()) {
    std::fill(cam.intrinsics.begin(), cam.intrinsics.end(), 0.0);
    std::copy(init.begin(), init.end(), cam.intrinsics.begin());
  }
  StageProblem sp;
  const StageProblem::Intr in = sp.addIntrinsics(cam, 0);
  for (const GridObservation& obs : observations) {
    Transformation T_t_c;
    if (!cam.estimateTransformation(obs, target, T_t_c)) continue;  // SM_WARN and skip (:118-122)
    const StageProblem::Pose p = sp.addPose(T_t_c);
    sp.addView(0, in, obs, p, {}, target.size());
  }
  const StageResult r = run_stage(sp, target, so, defaultOptimizerOptions());
  pull_intrinsics(cam, in);
  if (out) *out = r;
  return !r.ret.linearSolverFailure;
}

// ---------------------------------------------------------------- sm::kinematics / math helpers
double median(std::vector<double> v) {  // BasicMathUtils.cpp:10-17
  if (v.empty()) throw std::runtime_error("Cannot compute median of an empty vector.");
  std::nth_element(v.begin(), v.begin() + (long)(v.size() / 2), v.end());
  return v.at(v.size() / 2);
}

std::array<double, 3> rotationMatrixToParameters(const std::array<double, 9>& C) {  // RotationVector.cpp:57-80
  const double tr = std::max(-1.0, std::min((C[0] + C[4] + C[8] - 1.0) * 0.5, 1.0));
  const double a = std::acos(tr);
  if (std::fabs(a) < 1e-14) return {0.0, 0.0, 0.0};
  std::array<double, 3> p{C[7] - C[5], C[2] - C[6], C[3] - C[1]};
  const double n2 = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  if (std::fabs(n2) < 1e-14) return {0.0, 0.0, 0.0};
  const double scale = -a / n2;
  for (double& v : p) v *= scale;
  return p;
}

std::array<double, 9> parametersToRotationMatrix(const std::array<double, 3>& p) {  // RotationVector.cpp:10-50
  const double angle = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  if (angle < 1e-14) return {1, 0, 0, 0, 1, 0, 0, 0, 1};
  const double ra = 1.0 / angle, ax = p[0] * ra, ay = p[1] * ra, az = p[2] * ra;
  const double sa = std::sin(angle), ca = std::cos(angle), ax2 = ax * ax, ay2 = ay * ay, az2 = az * az;
  return {ax2 + ca * (1.0 - ax2),      ax * ay - ca * ax * ay + sa * az, ax * az - ca * ax * az - sa * ay,
          ax * ay - ca * ax * ay - sa * az, ay2 + ca * (1.0 - ay2),      ay * az - ca * ay * az + sa * ax,
          ax * az - ca * ax * az + sa * ay, ay * az - ca * ay * az - sa * ax, az2 + ca * (1.0 - az2)};
}

Transformation inverse(const Transformation& T) {  // Transformation.cpp:83-87: (quatInv(q), quatRotate(quatInv(q), -t))
  Transformation out;
  out.q = quat_normalized({-T.q[0], -T.q[1], -T.q[2], T.q[3]});
  const std::array<double, 9> R = Transformation{out.q, {0, 0, 0}}.C();
  for (int r = 0; r < 3; ++r) out.t[r] = -(R[3 * r] * T.t[0] + R[3 * r + 1] * T.t[1] + R[3 * r + 2] * T.t[2]);
  return out;
}

// ---------------------------------------------------------------- CalibrateStereoPair (CalibrationTools.hpp:183-300)
namespace {
// the guess loop of :198-216 with the caller's T_L / T_H, which the reference reuses in the DV loop that follows
Transformation stereo_guess(const CameraCalibrator& L, const CameraCalibrator& H,
                            const std::vector<std::optional<GridObservation>>& obsL,
                            const std::vector<std::optional<GridObservation>>& obsH, const AprilgridTarget& target,
                            Transformation& T_L, Transformation& T_H) {
  if (obsL.size() != obsH.size())
    throw std::runtime_error("The number of observations for both cameras must be the same.");
  std::vector<Transformation> trs;
  for (size_t i = 0; i < obsL.size(); ++i) {
    if (!obsL[i] || !obsH[i]) continue;
    if (!L.estimateTransformation(*obsL[i], target, T_L)) continue;  // SM_ERROR and skip
    if (!H.estimateTransformation(*obsH[i], target, T_H)) continue;
    trs.push_back(inverse(T_H) * T_L);  // T_H^-1 T_L = T_cH_cL
  }
  std::vector<double> tx, ty, tz, rx, ry, rz;
  for (const Transformation& t : trs) {
    tx.push_back(t.t[0]);
    ty.push_back(t.t[1]);
    tz.push_back(t.t[2]);
    const std::array<double, 3> r = rotationMatrixToParameters(t.C());
    rx.push_back(r[0]);
    ry.push_back(r[1]);
    rz.push_back(r[2]);
  }
  const std::array<double, 3> mt{median(tx), median(ty), median(tz)};
  const std::array<double, 3> mr{median(rx), median(ry), median(rz)};
  // rt2Transform(C, t) -> Transformation(T): the quaternion by r2quat
  return Transformation::fromMatrix(parametersToRotationMatrix(mr), mt);
}
}  // namespace

Transformation stereoBaselineGuess(const CameraCalibrator& L, const CameraCalibrator& H,
                                   const std::vector<std::optional<GridObservation>>& obsL,
                                   const std::vector<std::optional<GridObservation>>& obsH,
                                   const AprilgridTarget& target) {
  Transformation T_L, T_H;
  return stereo_guess(L, H, obsL, obsH, target, T_L, T_H);
}

StageResult calibrateStereoPair(CameraCalibrator& L, CameraCalibrator& H,
                                const std::vector<std::optional<GridObservation>>& obsL,
                                const std::vector<std::optional<GridObservation>>& obsH, const AprilgridTarget& target,
                                const StageOptions& so, Transformation& T_H_L, Transformation* guess) {
  check_cam(L);
  check_cam(H);
  Transformation T_L, T_H;
  const Transformation B0 = stereo_guess(L, H, obsL, obsH, target, T_L, T_H);
  if (guess) *guess = B0;
  StageProblem sp;
  const StageProblem::Pose B = sp.addPose(B0);
  std::vector<StageProblem::Pose> P;  // target_pose_dvs
  const Transformation B0inv = inverse(B0);
  for (size_t i = 0; i < obsL.size(); ++i) {
    // the PnP results are not checked here (:245-247): a failed estimate leaves T_L / T_H as they were, possibly
    // from the guess loop.  Quirk kept: a set seen by camera H only takes T_L = T_H * T_H_L^-1 (:251-252), not
    // T_H * T_H_L.
    if (obsL[i]) {
      L.estimateTransformation(*obsL[i], target, T_L);
    } else if (obsH[i]) {
      H.estimateTransformation(*obsH[i], target, T_H);
      T_L = T_H * B0inv;
    } else {
      continue;
    }
    P.push_back(sp.addPose(T_L));
  }
  const StageProblem::Intr inL = sp.addIntrinsics(L, 0), inH = sp.addIntrinsics(H, 1);
  // the error terms index target_pose_dvs by the observation index (:274, :283) although the loop above appended one
  // DV per set seen by L or H only: a set seen by neither before the last set with a view makes that index run past
  // the vector (undefined behaviour in the reference), refused here
  auto pose_of = [&](size_t i) -> const StageProblem::Pose& {
    if (i >= P.size())
      throw std::runtime_error("calibrateStereoPair: a synchronized set seen by neither camera precedes a set with a "
                               "view (the reference indexes target_pose_dvs past its end, CalibrationTools.hpp:274,283)");
    return P[i];
  };
  for (size_t i = 0; i < obsL.size(); ++i)
    if (obsL[i]) sp.addView(0, inL, *obsL[i], pose_of(i), {}, target.size());
  for (size_t i = 0; i < obsH.size(); ++i)
    if (obsH[i]) sp.addView(1, inH, *obsH[i], pose_of(i), {B}, target.size());
  const StageResult r = run_stage(sp, target, so, defaultOptimizerOptions());
  // a linear solver failure is not raised: the reference constructs the std::runtime_error without throwing (:292-294)
  pull_intrinsics(L, inL);
  pull_intrinsics(H, inH);
  const Transformation Bv = pose_value(B);
  T_H_L = Transformation::fromMatrix(Bv.C(), Bv.t);  // Transformation(toTransformationMatrix()) (:297)
  return r;
}

// ---------------------------------------------------------------- getTargetPoseGuess (CalibrationTools.hpp:315-356)
Transformation getTargetPoseGuess(const std::vector<CameraCalibrator>& cams, const SyncedSet& set,
                                  const std::vector<Transformation>& baselineGuesses, const AprilgridTarget& target) {
  size_t best = 0;
  unsigned best_n = 0;
  std::vector<unsigned> idx;
  for (size_t i = 0; i < set.size(); ++i) {  // std::max_element: the first maximum
    const unsigned n = set[i] ? set[i]->getCornersIdx(idx) : 0u;
    if (n > best_n) best_n = n, best = i;
  }
  if (set.empty() || !set.at(best)) throw std::runtime_error("getTargetPoseGuess: no observation in the set (bad_optional_access)");
  if (best > baselineGuesses.size()) throw std::runtime_error("getTargetPoseGuess: too few baseline guesses");
  Transformation T;  // identity: a failed PnP is not checked (:350)
  cams.at(best).estimateTransformation(*set[best], target, T);
  for (size_t j = 0; j < best; ++j) T = T * baselineGuesses[j];  // std::accumulate(.., std::multiplies)
  return T;
}

// ---------------------------------------------------------------- CalibrateMultiCameraRig (CalibrationTools.hpp:376-428)
std::vector<Transformation> calibrateMultiCameraRig(std::vector<CameraCalibrator>& cams,
                                                    const std::vector<SyncedSet>& sets, const AprilgridTarget& target,
                                                    const std::vector<Transformation>& baselineGuesses,
                                                    const StageOptions& so, StageResult* out) {
  const size_t N = cams.size();
  if (N < 1 || baselineGuesses.size() != N - 1) throw std::runtime_error("calibrateMultiCameraRig: need N - 1 baselines");
  for (const auto& c : cams) check_cam(c);
  StageProblem sp;
  std::vector<StageProblem::Intr> in;
  for (size_t i = 0; i < N; ++i) in.push_back(sp.addIntrinsics(cams[i], (int)i));
  std::vector<StageProblem::Pose> B;
  for (const Transformation& t : baselineGuesses) B.push_back(sp.addPose(t));
  for (const SyncedSet& s : sets) {
    if (s.size() != N) throw std::runtime_error("calibrateMultiCameraRig: synchronized set size != number of cameras");
    const StageProblem::Pose P = sp.addPose(getTargetPoseGuess(cams, s, baselineGuesses, target));
    for (size_t i = 0; i < N; ++i)
      if (s[i]) sp.addView((int)i, in[i], *s[i], P, B, target.size());
  }
  const StageResult r = run_stage(sp, target, so, defaultOptimizerOptions());
  if (r.ret.linearSolverFailure) throw std::runtime_error("Linear solver failed during optimization.");
  for (size_t i = 0; i < N; ++i) pull_intrinsics(cams[i], in[i]);
  std::vector<Transformation> res;
  for (const auto& b : B) {
    const Transformation v = pose_value(b);
    res.push_back(Transformation::fromMatrix(v.C(), v.t));
  }
  if (out) *out = r;
  return res;
}

// ---------------------------------------------------------------- SynchronizedObservationView.cpp:35-90
std::vector<SyncedSet> synchronizeObservations(const std::vector<std::vector<GridObservation>>& src, double tol) {
  const size_t n = src.size();
  std::vector<size_t> it(n, 0);
  std::vector<SyncedSet> out;
  for (;;) {
    long pivot = -1;  // get_pivot_index: the oldest head, first index on ties (strict <)
    for (size_t i = 0; i < n; ++i) {
      if (it[i] == src[i].size()) continue;
      if (pivot < 0 || src[i][it[i]].time < src[(size_t)pivot][it[(size_t)pivot]].time) pivot = (long)i;
    }
    if (pivot < 0) break;
    const double w0 = src[(size_t)pivot][it[(size_t)pivot]].time, w1 = w0 + tol;
    SyncedSet s(n);
    for (size_t i = 0; i < n; ++i) {
      if (it[i] == src[i].size()) continue;
      const double t = src[i][it[i]].time;
      if (t >= w0 && t <= w1) s[i] = src[i][it[i]++];
    }
    out.push_back(std::move(s));
  }
  return out;
}

std::vector<std::optional<GridObservation>> observationsFromSource(const std::vector<SyncedSet>& sets, size_t source) {
  std::vector<std::optional<GridObservation>> o;
  for (const SyncedSet& s : sets) o.push_back(s.at(source));
  return o;
}

// ---------------------------------------------------------------- CameraGraph.cpp
CameraGraph buildCameraGraph(const std::vector<SyncedSet>& sets) {
  if (sets.empty()) throw std::runtime_error("buildCameraGraph: no synchronized sets");
  CameraGraph g;
  g.nodes = sets.at(0).size();
  for (const SyncedSet& s : sets)
    if (s.size() != g.nodes) throw std::runtime_error("All synced sets must have the same number of cameras");
  std::map<std::pair<size_t, size_t>, size_t> common;  // ComputeTotalCommonCorners (:44-78)
  std::vector<std::vector<unsigned>> idx(g.nodes);
  for (const SyncedSet& s : sets) {
    for (size_t i = 0; i < g.nodes; ++i) {
      idx[i].clear();
      if (s[i]) s[i]->getCornersIdx(idx[i]);
    }
    for (size_t i = 0; i < g.nodes; ++i)
      for (size_t j = i + 1; j < g.nodes; ++j) {
        std::vector<unsigned> c;
        std::set_intersection(idx[i].begin(), idx[i].end(), idx[j].begin(), idx[j].end(), std::back_inserter(c));
        common[{i, j}] += c.size();
      }
  }
  for (const auto& kv : common)
    if (kv.second > 0) g.edges[kv.first] = 1.0 / (double)kv.second;  // AddEdgesBetweenNodes(i, j, 1 / n) (:100-106)
  return g;
}

DijkstraResult dijkstra(const CameraGraph& g, size_t start) {
  const size_t n = g.nodes;
  if (start >= n) throw std::runtime_error("dijkstra: start node out of range");
  DijkstraResult r;
  r.distance.assign(n, std::numeric_limits<double>::infinity());
  r.previous.assign(n, -1);
  std::vector<char> done(n, 0);
  r.distance[start] = 0.0;
  r.previous[start] = (long)start;
  using Item = std::pair<double, size_t>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> q;  // (distance, index): lowest index on ties
  q.push({0.0, start});
  while (!q.empty()) {
    const auto [d, u] = q.top();
    q.pop();
    if (done[u]) continue;
    done[u] = 1;
    for (size_t v = 0; v < n; ++v) {
      if (v == u || done[v]) continue;
      const auto e = g.edges.find({std::min(u, v), std::max(u, v)});
      if (e == g.edges.end()) continue;
      const double nd = d + e->second;
      if (nd < r.distance[v]) {
        r.distance[v] = nd;
        r.previous[v] = (long)u;
        q.push({nd, v});
      }
    }
  }
  return r;
}

Transformation getTransform(const std::map<std::pair<size_t, size_t>, Transformation>& map, const DijkstraResult& r,
                            size_t left, size_t right) {
  if (r.size() < 2) throw std::runtime_error("Dijkstra result must contain at least two nodes to compute a transform.");
  const bool leftFurther = r.distance.at(left) > r.distance.at(right);
  const size_t start = leftFurther ? left : right, end = leftFurther ? right : left;
  std::vector<Transformation> trs;
  size_t cur = start;
  while (cur != end) {
    const long prev = r.previous.at(cur);
    if (prev < 0 || (size_t)prev == cur)
      throw std::runtime_error("getTransform: the nearer camera is not on the further camera's path to the search start "
                               "(the reference loops or leaves its map here, CameraGraph.cpp:151-156)");
    trs.push_back(map.at({cur, (size_t)prev}));
    cur = (size_t)prev;
  }
  Transformation T;  // std::accumulate(.., Transformation{}, std::multiplies): path order, as the reference
  for (const Transformation& t : trs) T = T * t;
  return leftFurther ? T : inverse(T);
}

// ---------------------------------------------------------------- CalibrateCameras.cpp:142-356
CalibrateCamerasResult calibrateCameras(const std::vector<int32_t>& models,
                                        const std::vector<std::vector<GridObservation>>& byCam,
                                        const AprilgridTarget& target, const CalibrateCamerasOptions& opt,
                                        const StageOptions& stages,
                                        std::shared_ptr<backend::MarginalLinearSystemSolver> estimatorSolver) {
  const size_t N = models.size();
  if (N < 2 || byCam.size() != N) throw std::runtime_error("calibrateCameras: at least two cameras, one list each");
  CalibrateCamerasResult res;
  std::vector<CameraCalibrator> cams(N);
  for (size_t i = 0; i < N; ++i) cams[i] = CameraCalibrator{models[i], std::vector<double>(KB_MAX_INTR, 0.0)};
  // initial intrinsics per camera (:142-153)
  res.single.resize(N);
  for (size_t c = 0; c < N; ++c) {
    const std::optional<double> fl = c < opt.focalLengths.size() ? opt.focalLengths[c] : std::nullopt;
    if (!calibrateSingleCamera(byCam[c], cams[c], target, fl, stages, &res.single[c]))
      throw std::runtime_error("Failed to calibrate intrinsics from observations for camera ID: " + std::to_string(c));
  }
  res.afterSingle = cams;
  // synchronized sets, camera graph, Dijkstra from camera 0 (:155-174)
  res.syncedSets = synchronizeObservations(byCam, opt.approxSyncTolerance);
  const CameraGraph graph = buildCameraGraph(res.syncedSets);
  res.graphSearch = dijkstra(graph, 0);
  // stereo calibration of every camera with its predecessor on the search tree (:176-194)
  for (size_t i = 1; i < N; ++i) {
    const long best = res.graphSearch.previousIndex(i);
    if (best < 0) throw std::runtime_error("calibrateCameras: camera " + std::to_string(i) + " shares no corners");
    Transformation tf;
    res.stereo.push_back(calibrateStereoPair(cams[i], cams[(size_t)best], observationsFromSource(res.syncedSets, i),
                                             observationsFromSource(res.syncedSets, (size_t)best), target, stages, tf));
    res.stereoPairs.push_back({i, (size_t)best});
    res.optimalBaselines[{i, (size_t)best}] = tf;
  }
  res.afterStereo = cams;
  // consecutive baselines (:196-226)
  auto& ob = res.optimalBaselines;
  for (size_t i = 0; i + 1 < N; ++i) {
    if (ob.count({i, i + 1})) continue;
    const auto inv = ob.find({i + 1, i});
    if (inv != ob.end()) {
      ob[{i, i + 1}] = inverse(inv->second);
      continue;
    }
    ob[{i, i + 1}] = getTransform(ob, res.graphSearch, i, i + 1);
  }
  for (size_t i = 0; i + 1 < N; ++i) res.baselineGuesses.push_back(ob.at({i, i + 1}));
  // full batch refinement (:228-230)
  res.rigBaselines = calibrateMultiCameraRig(cams, res.syncedSets, target, res.baselineGuesses, stages, &res.rig);
  res.afterRig = cams;
  // the incremental estimator over the synchronized sets (:234-311)
  backend::CalibrationProblem base;
  base.cam_model = models;
  base.target = target.points();
  base.state.assign(N * KB_MAX_INTR + 7 * (N - 1), 0.0);
  for (size_t i = 0; i < N; ++i) std::copy(cams[i].intrinsics.begin(), cams[i].intrinsics.end(), base.state.begin() + (long)(i * KB_MAX_INTR));
  for (size_t j = 0; j + 1 < N; ++j) {
    std::copy(res.rigBaselines[j].q.begin(), res.rigBaselines[j].q.end(), base.state.begin() + (long)(N * KB_MAX_INTR + 7 * j));
    std::copy(res.rigBaselines[j].t.begin(), res.rigBaselines[j].t.end(), base.state.begin() + (long)(N * KB_MAX_INTR + 7 * j + 4));
  }
  backend::IncrementalEstimator::Options eo;
  eo.infoGainDelta = opt.mutualInformationTolerance;
  eo.checkValidity = true;
  eo.verbose = opt.verbose;
  backend::Optimizer2Options oo;
  oo.maxIterations = (int)opt.estimatorMaxIterations;
  oo.nThreads = 16;
  oo.verbose = opt.verbose;
  backend::IncrementalEstimator est(base, estimatorSolver, eo, oo);
  std::vector<backend::CalibrationBatch> processed;  // every batch handed to addBatch (the statistics' terms)
  for (const SyncedSet& s : res.syncedSets) {
    if (opt.maxBatches && res.acceptedBatches >= *opt.maxBatches) break;
    // the guess uses the calibrators' live intrinsics (the estimator's DVs) and the rig stage's baselines, which
    // the reference passes by value (:293)
    std::vector<CameraCalibrator> now = cams;
    const std::vector<double>& st = est.getProblem().state;
    for (size_t i = 0; i < N; ++i)
      std::copy(st.begin() + (long)(i * KB_MAX_INTR), st.begin() + (long)((i + 1) * KB_MAX_INTR), now[i].intrinsics.begin());
    const Transformation T = getTargetPoseGuess(now, s, res.rigBaselines, target);
    backend::CalibrationBatch b;  // CreateBatchProblem (CalibrationTools.hpp:460-521)
    b.frame_pose = {T.q[0], T.q[1], T.q[2], T.q[3], T.t[0], T.t[1], T.t[2]};
    b.view_offset.push_back(0);
    for (size_t i = 0; i < N; ++i) {
      if (!s[i]) continue;
      const size_t before = b.corner_id.size();
      double y[2];
      for (size_t k = 0; k < target.size(); ++k)
        if (s[i]->imagePoint(k, y)) {
          b.corner_id.push_back((uint16_t)k);
          b.y.push_back(y[0]);
          b.y.push_back(y[1]);
        }
      if (b.corner_id.size() == before) continue;  // a view without seen corners adds no term
      b.view_cam.push_back((uint8_t)i);
      b.view_offset.push_back((uint32_t)b.corner_id.size());
    }
    const auto rv = est.addBatch(b);
    processed.push_back(b);
    res.processedBatches++;
    if (rv.numIterations > (size_t)oo.maxIterations) throw std::runtime_error("Optimizer reached max iterations. Something went wrong.");
    res.batchAccepted.push_back(rv.batchAccepted ? 1 : 0);
    res.batchIterations.push_back((long)rv.numIterations);
    res.batchRank.push_back((long)rv.rankTheta);
    if (rv.batchAccepted) res.acceptedBatches++;
  }
  res.finalState = est.getProblem().state;
  res.final = cams;
  for (size_t i = 0; i < N; ++i)
    std::copy(res.finalState.begin() + (long)(i * KB_MAX_INTR), res.finalState.begin() + (long)((i + 1) * KB_MAX_INTR),
              res.final[i].intrinsics.begin());
  for (size_t j = 0; j + 1 < N; ++j) {
    Transformation B;
    const double* p = res.finalState.data() + N * KB_MAX_INTR + 7 * j;
    std::copy(p, p + 4, B.q.begin());
    std::copy(p + 4, p + 7, B.t.begin());
    res.finalBaselines.push_back(Transformation::fromMatrix(B.C(), B.t));
  }
  // the final reprojection-error statistics (CalibrateCameras.cpp:316-318): one frame per processed batch, its views
  // in camera order and corners in target order (the order the reference's calibrators stored the terms)
  if (stages.solver && !processed.empty()) {
    backend::CalibrationProblem sp;
    sp.cam_model = models;
    sp.target = target.points();
    sp.state.assign(res.finalState.begin(), res.finalState.begin() + (long)(N * KB_MAX_INTR + 7 * (N - 1)));
    size_t kept = 0;
    const size_t so = N * KB_MAX_INTR + 7 * (N - 1);
    for (size_t bi = 0; bi < processed.size(); ++bi) {
      const backend::CalibrationBatch& b = processed[bi];
      for (size_t v = 0; v < b.view_cam.size(); ++v) {
        sp.view_frame.push_back((uint32_t)bi);
        sp.view_cam.push_back(b.view_cam[v]);
        sp.view_offset.push_back((uint32_t)sp.corner_id.size());
        for (uint32_t k = b.view_offset[v]; k < b.view_offset[v + 1]; ++k) {
          sp.corner_id.push_back(b.corner_id[k]);
          sp.y.push_back(b.y[2 * k]);
          sp.y.push_back(b.y[2 * k + 1]);
        }
      }
      if (res.batchAccepted[bi]) {  // the estimator's pose of the kept batch (its frames in acceptance order)
        sp.state.insert(sp.state.end(), res.finalState.begin() + (long)(so + 7 * kept),
                        res.finalState.begin() + (long)(so + 7 * kept + 7));
        ++kept;
      } else {
        sp.state.insert(sp.state.end(), b.frame_pose.begin(), b.frame_pose.end());
      }
    }
    sp.view_offset.push_back((uint32_t)sp.corner_id.size());
    sp.n_frames = (int)processed.size();
    auto sv = stages.solver();
    sv->initMatrixStructure(sp, false);
    res.reprojectionErrorStatistics = sv->reprojectionErrorStatistics();
  }
  return res;
}

}  // namespace tools
}  // namespace kalibr_amd
