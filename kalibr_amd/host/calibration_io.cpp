// calibration_io.cpp -- see calibration_io.hpp.  Paths relative to the reference repository.
#include "calibration_io.hpp"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <fstream>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "kalibr_hip.h"

namespace kalibr_amd {
namespace io {

// ---------------------------------------------------------------- sm::kinematics restatements
static std::array<double, 9> quat2r(const std::array<double, 4>& q) {  // quaternion_algebra.cpp:77-101 (JPL)
  return {q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3],
          2.0 * (q[0] * q[1] + q[2] * q[3]),
          2.0 * (q[0] * q[2] - q[1] * q[3]),
          2.0 * (q[0] * q[1] - q[2] * q[3]),
          -q[0] * q[0] + q[1] * q[1] - q[2] * q[2] + q[3] * q[3],
          2.0 * (q[0] * q[3] + q[1] * q[2]),
          2.0 * (q[0] * q[2] + q[1] * q[3]),
          2.0 * (q[1] * q[2] - q[0] * q[3]),
          -q[0] * q[0] - q[1] * q[1] + q[2] * q[2] + q[3] * q[3]};
}

static std::array<double, 4> r2quat(const std::array<double, 9>& R) {  // quaternion_algebra.cpp:16-75
  // column-major names of the reference: c1 = R(0,0), c2 = R(1,0), c3 = R(2,0), c4 = R(0,1), ...
  const double c1 = R[0], c2 = R[3], c3 = R[6], c4 = R[1], c5 = R[4], c6 = R[7], c7 = R[2], c8 = R[5], c9 = R[8];
  const double dg[4] = {std::fabs(1.0 + c1 - c5 - c9), std::fabs(1.0 - c1 + c5 - c9), std::fabs(1.0 - c1 - c5 + c9),
                        std::fabs(1.0 + c1 + c5 + c9)};
  const int k = (int)(std::max_element(dg, dg + 4) - dg);
  std::array<double, 4> q{};
  q[k] = 0.5 * std::sqrt(dg[k]);
  const double c = 0.25 / q[k];
  switch (k) {
    case 0: q[1] = c * (c4 + c2), q[2] = c * (c7 + c3), q[3] = c * (c8 - c6); break;
    case 1: q[0] = c * (c4 + c2), q[2] = c * (c6 + c8), q[3] = c * (c3 - c7); break;
    case 2: q[0] = c * (c3 + c7), q[1] = c * (c6 + c8), q[3] = c * (c4 - c2); break;
    default: q[0] = c * (c8 - c6), q[1] = c * (c3 - c7), q[2] = c * (c4 - c2); break;
  }
  if (q[3] < 0.0)
    for (double& v : q) v = -v;
  return q;
}

static std::array<double, 4> qplus(const std::array<double, 4>& q, const std::array<double, 4>& p) {
  // quaternion_algebra.cpp:136-149
  return {p[0] * q[3] + p[1] * q[2] - p[2] * q[1] + p[3] * q[0], p[2] * q[0] - p[0] * q[2] + p[1] * q[3] + p[3] * q[1],
          p[0] * q[1] - p[1] * q[0] + p[2] * q[3] + p[3] * q[2], p[3] * q[3] - p[1] * q[1] - p[2] * q[2] - p[0] * q[0]};
}

std::array<double, 9> Transformation::C() const { return quat2r(q); }

Transformation Transformation::operator*(const Transformation& rhs) const {
  Transformation out;
  out.q = qplus(q, rhs.q);
  // Transformation(q, t) normalises its quaternion (Transformation.cpp:31-35)
  const double qn = std::sqrt(out.q[0] * out.q[0] + out.q[1] * out.q[1] + out.q[2] * out.q[2] + out.q[3] * out.q[3]);
  for (double& v : out.q) v /= qn;
  const std::array<double, 9> R = C();
  for (int r = 0; r < 3; ++r) out.t[r] = R[3 * r] * rhs.t[0] + R[3 * r + 1] * rhs.t[1] + R[3 * r + 2] * rhs.t[2] + t[r];
  return out;
}

Transformation Transformation::fromMatrix(const std::array<double, 9>& C, const std::array<double, 3>& t) {
  Transformation out;
  out.q = r2quat(C);
  out.t = t;
  return out;
}

// ---------------------------------------------------------------- target and observations
std::vector<double> AprilgridTarget::points() const {
  std::vector<double> p(3 * size());
  for (size_t r = 0; r < rows(); ++r)
    for (size_t c = 0; c < cols(); ++c) {
      double* x = p.data() + 3 * (r * cols() + c);
      x[0] = (double)(int)(c / 2) * (1 + tagSpacing) * tagSize + (double)(c % 2) * tagSize;
      x[1] = (double)(int)(r / 2) * (1 + tagSpacing) * tagSize + (double)(r % 2) * tagSize;
      x[2] = 0.0;
    }
  return p;
}

bool GridObservation::imagePoint(size_t i, double out[2]) const {
  if (i >= success.size()) throw std::out_of_range("GridObservation::imagePoint: index out of range");
  out[0] = points[2 * i];
  out[1] = points[2 * i + 1];
  return success[i] != 0;
}

void GridObservation::updateImagePoint(size_t i, double u, double v) {
  if (i >= success.size()) throw std::out_of_range("GridObservation::updateImagePoint: index out of range");
  points[2 * i] = u;
  points[2 * i + 1] = v;
  success[i] = 1;
}

void GridObservation::removeImagePoint(size_t i) {
  if (i >= success.size()) throw std::out_of_range("GridObservation::removeImagePoint: index out of range");
  success[i] = 0;
}

unsigned GridObservation::getCornersIdx(std::vector<unsigned>& idx) const {
  idx.clear();
  for (size_t i = 0; i < success.size(); ++i)
    if (success[i]) idx.push_back((unsigned)i);
  return (unsigned)idx.size();
}

bool GridObservation::hasSuccessfulObservation() const {
  return std::any_of(success.begin(), success.end(), [](uint8_t s) { return s != 0; });
}

Transformation targetPoseGuess(const SyncedSet& set, const std::vector<Transformation>& baselineGuesses) {
  // n_corners per camera, 0 when absent; first maximum wins (std::max_element)
  size_t best = 0;
  unsigned best_n = 0;
  std::vector<unsigned> idx;
  for (size_t i = 0; i < set.size(); ++i) {
    const unsigned n = set[i] ? set[i]->getCornersIdx(idx) : 0u;
    if (n > best_n) best_n = n, best = i;
  }
  if (set.empty() || !set[best]) throw std::runtime_error("targetPoseGuess: no observation in the synchronized set");
  if (!set[best]->T_t_c) throw std::runtime_error("targetPoseGuess: observation without T_t_c (run the PnP first)");
  if (best > baselineGuesses.size()) throw std::runtime_error("targetPoseGuess: too few baseline guesses");
  Transformation T = *set[best]->T_t_c;
  for (size_t j = 0; j < best; ++j) T = T * baselineGuesses[j];  // std::accumulate(..., std::multiplies)
  return T;
}

backend::CalibrationProblem buildRigProblem(const std::vector<int32_t>& camModels, const std::vector<double>& intrinsics,
                                            const AprilgridTarget& target, const std::vector<SyncedSet>& sets,
                                            const std::vector<Transformation>& baselineGuesses) {
  const size_t N = camModels.size(), K = target.size();
  if (N < 1 || N > KB_MAX_CAMS) throw std::runtime_error("buildRigProblem: 1..KB_MAX_CAMS cameras");
  if (intrinsics.size() != N * KB_MAX_INTR) throw std::runtime_error("buildRigProblem: intrinsics size");
  if (baselineGuesses.size() != N - 1) throw std::runtime_error("buildRigProblem: need n_cams - 1 baselines");
  if (K > 65535) throw std::runtime_error("buildRigProblem: target too large for uint16 corner ids");
  backend::CalibrationProblem p;
  p.cam_model = camModels;
  p.target = target.points();
  p.n_frames = (int)sets.size();
  p.state.assign(N * KB_MAX_INTR + 7 * (N - 1) + 7 * sets.size(), 0.0);
  std::copy(intrinsics.begin(), intrinsics.end(), p.state.begin());
  for (size_t j = 0; j + 1 < N; ++j) {
    double* b = p.state.data() + N * KB_MAX_INTR + 7 * j;
    std::copy(baselineGuesses[j].q.begin(), baselineGuesses[j].q.end(), b);
    std::copy(baselineGuesses[j].t.begin(), baselineGuesses[j].t.end(), b + 4);
  }
  p.view_offset.push_back(0);
  for (size_t f = 0; f < sets.size(); ++f) {
    const SyncedSet& s = sets[f];
    if (s.size() != N) throw std::runtime_error("buildRigProblem: synchronized set size != n_cams");
    const Transformation T0 = targetPoseGuess(s, baselineGuesses);
    double* fp = p.state.data() + N * KB_MAX_INTR + 7 * (N - 1) + 7 * f;
    std::copy(T0.q.begin(), T0.q.end(), fp);
    std::copy(T0.t.begin(), T0.t.end(), fp + 4);
    for (size_t i = 0; i < N; ++i) {
      if (!s[i]) continue;
      const GridObservation& o = *s[i];
      if (o.success.size() != K || o.points.size() != 2 * K)
        throw std::runtime_error("buildRigProblem: observation size != target size");
      const size_t before = p.corner_id.size();
      double y[2];
      for (size_t k = 0; k < K; ++k)
        if (o.imagePoint(k, y)) {
          p.corner_id.push_back((uint16_t)k);
          p.y.push_back(y[0]);
          p.y.push_back(y[1]);
        }
      if (p.corner_id.size() == before) continue;  // a view without seen corners adds no term
      p.view_frame.push_back((uint32_t)f);
      p.view_cam.push_back((uint8_t)i);
      p.view_offset.push_back((uint32_t)p.corner_id.size());
    }
  }
  return p;
}

// ---------------------------------------------------------------- export
std::string kalibrModelName(int32_t m) {
  switch (m) {
    case KB_PINHOLE_RADTAN: return "pinhole-radtan";
    case KB_OMNI_RADTAN: return "omni-radtan";
    case KB_EUCM: return "eucm-none";
    case KB_OMNI: return "omni-none";
    case KB_DS: return "ds-none";
    case KB_PINHOLE_EQUI: return "pinhole-equi";
    case KB_PINHOLE_FOV: return "pinhole-fov";
    default: throw std::runtime_error("kalibrModelName: unknown camera model");
  }
}

std::string toRosDistortionModel(const std::string& m) {
  static const std::pair<const char*, const char*> table[] = {
      {"pinhole-radtan", "plumb_bob"}, {"pinhole-rs-radtan", "plumb_bob"}, {"pinhole-equi", "equidistant"},
      {"pinhole-rs-equi", "equidistant"}, {"pinhole-fov", "fov"}, {"omni-radtan", "plumb_bob"},
      {"omni-rs-radtan", "plumb_bob"}, {"omni-none", ""}, {"eucm-none", ""}, {"ds-none", "double_sphere"}};
  for (const auto& e : table)
    if (m == e.first) return e.second;
  return "unknown";
}

CameraInfoParams cameraInfoParams(int32_t m, const double* in) {
  // K from getCameraMatrix (fu, fv, cu, cv); d = model scalars (xi / alpha, beta) then the distortion parameters
  CameraInfoParams p;
  int k = 0;  // first of fu fv cu cv in the projection vector
  switch (m) {
    case KB_PINHOLE_RADTAN:
    case KB_PINHOLE_EQUI: k = 0, p.d = {in[4], in[5], in[6], in[7]}; break;
    case KB_PINHOLE_FOV: k = 0, p.d = {in[4]}; break;
    case KB_OMNI_RADTAN: k = 1, p.d = {in[0], in[5], in[6], in[7], in[8]}; break;
    case KB_OMNI: k = 1, p.d = {in[0]}; break;
    case KB_EUCM: k = 2, p.d = {in[0], in[1]}; break;  // alpha, beta
    case KB_DS: k = 2, p.d = {in[0], in[1]}; break;    // xi, alpha
    default: throw std::runtime_error("cameraInfoParams: unknown camera model");
  }
  p.fx = in[k];
  p.fy = in[k + 1];
  p.cx = in[k + 2];
  p.cy = in[k + 3];
  return p;
}

TransformStamped transformationToRos(const Transformation& T, const std::string& parent, const std::string& child) {
  TransformStamped tf;
  tf.frame_id = parent;
  tf.child_frame_id = child;
  tf.translation = T.t;
  tf.rotation = T.q;
  return tf;
}

// rosidl block-style scalars: shortest round-trip decimal for doubles, quoted strings
static std::string num(double v) {
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  std::string s(buf, r.ptr);
  if (std::isfinite(v) && s.find_first_of(".e") == std::string::npos) s += ".0";
  return s;
}

static std::string quoted(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

static void header_yaml(std::ostringstream& o, const std::string& ind, const std::string& frame_id) {
  o << ind << "header:\n" << ind << "  stamp:\n" << ind << "    sec: 0\n" << ind << "    nanosec: 0\n"
    << ind << "  frame_id: " << quoted(frame_id) << "\n";
}

static void seq_yaml(std::ostringstream& o, const char* name, const double* v, size_t n) {
  if (n == 0) {
    o << name << ": []\n";
    return;
  }
  o << name << ":\n";
  for (size_t i = 0; i < n; ++i) o << "- " << num(v[i]) << "\n";
}

std::string cameraInfoYaml(const CameraInfoParams& p, const std::string& kalibrModel, const std::string& frameId,
                           size_t width, size_t height) {
  double K[9] = {0}, R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, P[12] = {0};
  K[0] = p.fx, K[2] = p.cx, K[4] = p.fy, K[5] = p.cy, K[8] = 1.0;
  P[0] = p.fx, P[2] = p.cx, P[5] = p.fy, P[6] = p.cy, P[10] = 1.0;
  std::ostringstream o;
  header_yaml(o, "", frameId);
  o << "height: " << height << "\nwidth: " << width << "\n";
  o << "distortion_model: " << quoted(toRosDistortionModel(kalibrModel)) << "\n";
  seq_yaml(o, "d", p.d.data(), p.d.size());
  seq_yaml(o, "k", K, 9);
  seq_yaml(o, "r", R, 9);
  seq_yaml(o, "p", P, 12);
  o << "binning_x: 0\nbinning_y: 0\nroi:\n  x_offset: 0\n  y_offset: 0\n  height: 0\n  width: 0\n"
       "  do_rectify: false\n";
  return o.str();
}

static void tf_body(std::ostringstream& o, const std::string& ind, const TransformStamped& tf) {
  header_yaml(o, ind, tf.frame_id);
  o << ind << "child_frame_id: " << quoted(tf.child_frame_id) << "\n" << ind << "transform:\n";
  o << ind << "  translation:\n";
  const char* xyz[] = {"x", "y", "z", "w"};
  for (int i = 0; i < 3; ++i) o << ind << "    " << xyz[i] << ": " << num(tf.translation[i]) << "\n";
  o << ind << "  rotation:\n";
  for (int i = 0; i < 4; ++i) o << ind << "    " << xyz[i] << ": " << num(tf.rotation[i]) << "\n";
}

std::string transformStampedYaml(const TransformStamped& tf) {
  std::ostringstream o;
  tf_body(o, "", tf);
  return o.str();
}

std::string tfMessageYaml(const std::vector<TransformStamped>& tfs) {
  std::ostringstream o;
  if (tfs.empty()) return "transforms: []\n";
  o << "transforms:\n";
  for (const auto& tf : tfs) {
    o << "-\n";
    tf_body(o, "  ", tf);
  }
  return o.str();
}

static void write_file(const std::string& path, const std::string& text) {
  std::ofstream f(path);
  if (!f.is_open()) throw std::runtime_error("Failed to open file: " + path);
  f << text;
}

std::vector<std::string> exportCalibration(const std::string& dir, const std::vector<std::string>& names,
                                           const std::vector<int32_t>& models,
                                           const std::vector<std::pair<size_t, size_t>>& sizes,
                                           const std::vector<double>& state) {
  const size_t N = models.size();
  if (names.size() != N || sizes.size() != N || state.size() < N * KB_MAX_INTR + 7 * (N - 1))
    throw std::runtime_error("exportCalibration: inconsistent inputs");
  std::vector<std::string> out;
  for (size_t i = 0; i < N; ++i) {
    const std::string path = dir + "/calibration_" + names[i] + ".yaml";
    write_file(path, cameraInfoYaml(cameraInfoParams(models[i], state.data() + i * KB_MAX_INTR),
                                    kalibrModelName(models[i]), names[i], sizes[i].first, sizes[i].second));
    out.push_back(path);
  }
  if (N < 2) return out;
  // baselines through Transformation(T) of the DV's matrix (CalibrateCameras.cpp:329-334)
  std::vector<TransformStamped> tfs;
  for (size_t j = 0; j + 1 < N; ++j) {
    Transformation B;
    const double* b = state.data() + N * KB_MAX_INTR + 7 * j;
    std::copy(b, b + 4, B.q.begin());
    std::copy(b + 4, b + 7, B.t.begin());
    tfs.push_back(transformationToRos(Transformation::fromMatrix(B.C(), B.t), names[j], names[j + 1]));
  }
  if (tfs.size() == 1) {
    const std::string path = dir + "/transform_" + names[0] + "_to_" + names[1] + ".yaml";
    write_file(path, transformStampedYaml(tfs[0]));
    out.push_back(path);
  } else {
    const std::string path = dir + "/camera_chain_transforms.yaml";
    write_file(path, tfMessageYaml(tfs));
    out.push_back(path);
  }
  return out;
}

// ---------------------------------------------------------------- initialisers (PinholeProjection.hpp(impl))
namespace {
// modified least squares circle fit (PinholeProjection.hpp(impl):642-691)
void fit_circle(const std::vector<std::array<double, 2>>& pts, double& cx, double& cy, double& radius) {
  double sx = 0, sy = 0, sxx = 0, sxy = 0, syy = 0, sxxx = 0, sxxy = 0, sxyy = 0, syyy = 0;
  const int n = (int)pts.size();
  for (const auto& p : pts) {
    const double x = p[0], y = p[1];
    sx += x;
    sy += y;
    sxx += x * x;
    sxy += x * y;
    syy += y * y;
    sxxx += x * x * x;
    sxxy += x * x * y;
    sxyy += x * y * y;
    syyy += y * y * y;
  }
  const double A = n * sxx - sx * sx, B = n * sxy - sx * sy, C = n * syy - sy * sy;
  const double D = 0.5 * (n * sxyy - sx * syy + n * sxxx - sx * sxx);
  const double E = 0.5 * (n * sxxy - sy * sxx + n * syyy - sy * syy);
  cx = (D * C - B * E) / (A * C - B * B);
  cy = (A * E - B * D) / (A * C - B * B);
  double sr = 0.0;
  for (const auto& p : pts) sr += std::hypot(p[0] - cx, p[1] - cy);
  radius = sr / n;
}

// intersection points of two circles (:611-640)
std::vector<std::array<double, 2>> intersect_circles(double x1, double y1, double r1, double x2, double y2, double r2) {
  std::vector<std::array<double, 2>> out;
  const double d = std::hypot(x1 - x2, y1 - y2);
  if (d > r1 + r2 || d < std::fabs(r1 - r2)) return out;
  const double a = (r1 * r1 - r2 * r2 + d * d) / (2.0 * d), h = std::sqrt(r1 * r1 - a * a);
  const double x3 = x1 + a * (x2 - x1) / d, y3 = y1 + a * (y2 - y1) / d;
  if (h < 1e-10) {
    out.push_back({x3, y3});
    return out;
  }
  out.push_back({x3 + h * (y2 - y1) / d, y3 - h * (x2 - x1) / d});
  out.push_back({x3 - h * (y2 - y1) / d, y3 + h * (x2 - x1) / d});
  return out;
}

double median_of(std::vector<double> v) {  // medianOfVectorElements (:693-703)
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n % 2 == 0 ? (v[n / 2 - 1] + v[n / 2]) / 2 : v[n / 2];
}

int n_distortion(int32_t m) {
  switch (m) {
    case KB_PINHOLE_RADTAN:
    case KB_PINHOLE_EQUI: return 4;
    case KB_PINHOLE_FOV: return 1;
    default: return -1;  // not a PinholeProjection model
  }
}

// forward distortion of normalised coordinates (RadialTangential / Equidistant / Fov distort), Jacobian for radtan
void distort(int32_t m, const double* d, double& x, double& y, double* J) {
  if (m == KB_PINHOLE_RADTAN) {  // RadialTangentialDistortion.hpp(impl):20-60
    const double k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3];
    const double mx2 = x * x, my2 = y * y, mxy = x * y, rho2 = mx2 + my2, rad = k1 * rho2 + k2 * rho2 * rho2;
    if (J) {
      J[0] = 1 + rad + k1 * 2.0 * mx2 + k2 * rho2 * 4 * mx2 + 2.0 * p1 * y + 6 * p2 * x;
      J[1] = k1 * 2.0 * x * y + k2 * 4 * rho2 * x * y + p1 * 2.0 * x + 2.0 * p2 * y;
      J[2] = J[1];
      J[3] = 1 + rad + k1 * 2.0 * my2 + k2 * rho2 * 4 * my2 + 6 * p1 * y + 2.0 * p2 * x;
    }
    const double nx = x + x * rad + 2.0 * p1 * mxy + p2 * (rho2 + 2.0 * mx2);
    const double ny = y + y * rad + 2.0 * p2 * mxy + p1 * (rho2 + 2.0 * my2);
    x = nx;
    y = ny;
    return;
  }
  double s = 1.0;
  const double r = std::hypot(x, y);
  if (m == KB_PINHOLE_EQUI) {  // EquidistantDistortion.hpp(impl):31-80
    const double th = std::atan(r), t2 = th * th;
    const double thd = th * (1.0 + t2 * (d[0] + t2 * (d[1] + t2 * (d[2] + t2 * d[3]))));
    s = r > 1e-8 ? thd / r : 1.0;
  } else if (m == KB_PINHOLE_FOV) {  // FovDistortion.hpp(impl):19-60
    const double w = d[0];
    if (w * w < 1e-5) s = 1.0;
    else if (r * r < 1e-5) s = 2.0 * std::tan(0.5 * w) / w;
    else s = std::atan(2.0 * std::tan(0.5 * w) * r) / (r * w);
  }
  x *= s;
  y *= s;
}

// n x n symmetric: the eigenvector of the smallest eigenvalue (cyclic Jacobi)
template <int n>
std::array<double, n> smallest_eigvec(std::array<double, n * n> A) {
  std::array<double, n * n> V{};
  for (int i = 0; i < n; ++i) V[i * n + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int p = 0; p < n; ++p)
      for (int q = 0; q < n; ++q) (p == q ? tot : off) += A[p * n + q] * A[p * n + q];
    if (off <= 1e-30 * tot || off < 1e-300) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (std::fabs(apq) < 1e-300) continue;
        const double th = 0.5 * (A[q * n + q] - A[p * n + p]) / apq;
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
        for (int k = 0; k < n; ++k) {  // A <- J^T A J
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - sn * akq;
          A[k * n + q] = sn * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - sn * aqk;
          A[q * n + k] = sn * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - sn * vkq;
          V[k * n + q] = sn * vkp + c * vkq;
        }
      }
  }
  int m = 0;
  for (int i = 1; i < n; ++i)
    if (A[i * n + i] < A[m * n + m]) m = i;
  std::array<double, n> v{};
  for (int k = 0; k < n; ++k) v[k] = V[k * n + m];
  return v;
}

// rotation vector -> matrix (Rodrigues), row-major
std::array<double, 9> rodrigues(const double w[3]) {
  const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  std::array<double, 9> R{1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (th < 1e-300) return R;
  const double k[3] = {w[0] / th, w[1] / th, w[2] / th}, c = std::cos(th), s = std::sin(th), v = 1.0 - c;
  R = {c + k[0] * k[0] * v,        k[0] * k[1] * v - k[2] * s, k[0] * k[2] * v + k[1] * s,
       k[1] * k[0] * v + k[2] * s, c + k[1] * k[1] * v,        k[1] * k[2] * v - k[0] * s,
       k[2] * k[0] * v - k[1] * s, k[2] * k[1] * v + k[0] * s, c + k[2] * k[2] * v};
  return R;
}

std::array<double, 9> matmul3(const std::array<double, 9>& A, const std::array<double, 9>& B) {
  std::array<double, 9> C{};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 3; ++k) C[r * 3 + c] += A[r * 3 + k] * B[k * 3 + c];
  return C;
}
}  // namespace

namespace {
// normalised coordinates -> undistorted by Gauss-Newton on distort(ybar) = y: 5 steps for radtan (the reference's
// RadialTangentialDistortion::undistort loop, RadialTangentialDistortion.hpp(impl):68-98), up to 20 otherwise
void undistort(int32_t distModel, const double* d, double& x, double& y) {
  const double yu = x, yv = y;
  double bx = yu, by = yv;
  const int n = distModel == KB_PINHOLE_RADTAN ? 5 : 20;
  for (int i = 0; i < n; ++i) {
    double tx = bx, ty = by, F[4];
    if (distModel == KB_PINHOLE_RADTAN) {
      distort(distModel, d, tx, ty, F);
    } else {  // central differences of the forward map
      const double h = 1e-7;
      double a0 = bx + h, a1 = by, b0 = bx - h, b1 = by, c0 = bx, c1 = by + h, e0 = bx, e1 = by - h;
      distort(distModel, d, a0, a1, nullptr);
      distort(distModel, d, b0, b1, nullptr);
      distort(distModel, d, c0, c1, nullptr);
      distort(distModel, d, e0, e1, nullptr);
      F[0] = (a0 - b0) / (2 * h);
      F[2] = (a1 - b1) / (2 * h);
      F[1] = (c0 - e0) / (2 * h);
      F[3] = (c1 - e1) / (2 * h);
      distort(distModel, d, tx, ty, nullptr);
    }
    const double ex = yu - tx, ey = yv - ty;
    // du = (F^T F)^-1 F^T e = F^-1 e for a square F
    const double det = F[0] * F[3] - F[1] * F[2];
    bx += (F[3] * ex - F[1] * ey) / det;
    by += (-F[2] * ex + F[0] * ey) / det;
    if (ex * ex + ey * ey < 1e-15) break;
  }
  x = bx;
  y = by;
}

// OmniProjection::euclideanToKeypoint (OmniProjection.hpp(impl):76-114) without distortion (the initialiser's
// cleared distortion): false behind the fov limit or off the sensor (isValid: 0 <= u < ru, 0 <= v < rv)
bool omni_project(double xi, double fu, double fv, double cu, double cv, double ru, double rv, const double p[3],
                  double kp[2]) {
  const double d = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  const double fov = xi <= 1.0 ? xi : 1.0 / xi;  // updateTemporaries (:627-633)
  if (p[2] <= -(fov * d)) return false;
  const double rz = 1.0 / (p[2] + xi * d);
  kp[0] = fu * p[0] * rz + cu;
  kp[1] = fv * p[1] * rz + cv;
  return kp[0] >= 0 && kp[0] < ru && kp[1] >= 0 && kp[1] < rv;
}
}  // namespace

namespace {
// OmniProjection::initializeIntrinsics (OmniProjection.hpp(impl):724-846): xi = 1, the image centre, then per corner
// row of every view the conic through the centred points (u, v, 1/2, -(u^2 + v^2)/2) (cv::SVD::solveZ: the right
// singular vector of the smallest singular value), skipped when t < 0 or the line is radial (|n_xy| > 0.95); each
// candidate gamma = |c2 d / n_z| is scored by the mean reprojection error of the view under the pose
// estimateTransformation finds with it, and the lowest wins.  out = (gamma0, success); gamma0 = the fallback when
// no row scored (success false, as the reference returns).
bool omni_focal(const std::vector<GridObservation>& observations, const AprilgridTarget& target,
                std::optional<double> fallbackFocalLength, double& gamma0) {
  const double cu = (observations[0].imCols - 1.0) / 2.0, cv = (observations[0].imRows - 1.0) / 2.0;
  const double ru = (double)observations[0].imCols, rv = (double)observations[0].imRows;
  const size_t R = target.rows(), Cn = target.cols();
  const std::vector<double> P = target.points();
  constexpr size_t kMinCorners = 4;
  double minErr = std::numeric_limits<double>::max();
  bool success = false;
  gamma0 = 0.0;
  for (const GridObservation& obs : observations) {
    for (size_t r = 0; r < R; ++r) {
      std::array<double, 16> PtP{};
      size_t count = 0;
      for (size_t c = 0; c < Cn; ++c) {
        double kp[2];
        if (!obs.imagePoint(r * Cn + c, kp)) continue;
        const double u = kp[0] - cu, v = kp[1] - cv, row[4] = {u, v, 0.5, -0.5 * (u * u + v * v)};
        for (int a = 0; a < 4; ++a)
          for (int b = 0; b < 4; ++b) PtP[a * 4 + b] += row[a] * row[b];
        ++count;
      }
      if (count <= kMinCorners) continue;
      const std::array<double, 4> Cz = smallest_eigvec<4>(PtP);
      const double t = Cz[0] * Cz[0] + Cz[1] * Cz[1] + Cz[2] * Cz[3];
      if (t < 0) continue;
      const double d = std::sqrt(1.0 / t), nx = Cz[0] * d, ny = Cz[1] * d;
      if (std::hypot(nx, ny) > 0.95) continue;  // a radial line
      const double nz = std::sqrt(1.0 - nx * nx - ny * ny);
      const double gamma = std::fabs(Cz[2] * d / nz);
      const double trial[5] = {1.0, gamma, gamma, cu, cv};
      Transformation T_t_c;
      if (!estimateTransformation(obs, target, KB_OMNI, trial, T_t_c)) continue;
      // computeReprojectionError (:848-869): sum of |y - yhat| over the corners that project
      const std::array<double, 9> Rm = T_t_c.C();
      double err = 0.0;
      size_t n = 0;
      for (size_t i = 0; i < target.size(); ++i) {
        double y[2], yh[2], pc[3];
        if (!obs.imagePoint(i, y)) continue;
        const double dx = P[3 * i] - T_t_c.t[0], dy = P[3 * i + 1] - T_t_c.t[1], dz = P[3 * i + 2] - T_t_c.t[2];
        for (int a = 0; a < 3; ++a) pc[a] = Rm[a] * dx + Rm[3 + a] * dy + Rm[6 + a] * dz;  // C^T (P - t)
        if (!omni_project(1.0, gamma, gamma, cu, cv, ru, rv, pc, yh)) continue;
        err += std::hypot(y[0] - yh[0], y[1] - yh[1]);
        ++n;
      }
      if (n > kMinCorners && err / n < minErr) {
        minErr = err / n;
        gamma0 = gamma;
        success = true;
      }
    }
  }
  if (!success && fallbackFocalLength) gamma0 = *fallbackFocalLength;
  return success;
}
}  // namespace

bool initializeIntrinsics(const std::vector<GridObservation>& observations, const AprilgridTarget& target,
                          std::optional<double> fallbackFocalLength, int32_t camModel, std::vector<double>& intr) {
  if (observations.empty()) throw std::runtime_error("initializeIntrinsics: Need min. one observation");
  if (camModel == KB_OMNI_RADTAN || camModel == KB_OMNI || camModel == KB_EUCM || camModel == KB_DS) {
    double g = 0.0;
    const bool ok = omni_focal(observations, target, fallbackFocalLength, g);
    const double cu = (observations[0].imCols - 1.0) / 2.0, cv = (observations[0].imRows - 1.0) / 2.0;
    if (camModel == KB_OMNI_RADTAN || camModel == KB_OMNI) {
      // the omni model keeps the fallback focal length (set, but false returned) when no row scored
      if (!ok && !fallbackFocalLength) return false;
      intr.assign(camModel == KB_OMNI ? 5 : 9, 0.0);  // xi fu fv cu cv | distortion cleared
      intr[0] = 1.0;
      intr[1] = intr[2] = g;
      intr[3] = cu;
      intr[4] = cv;
      return ok;
    }
    if (!ok) return false;  // EUCM / DS take the omni result only on success (intr untouched)
    // ExtendedUnifiedProjection.hpp(impl):731-760: alpha = xi / 2, beta = 1, f = gamma / 2 (the same rays);
    // DoubleSphereProjection.hpp(impl):783-812: xi = 0 (the spheres coincide), alpha = 1/2, f = gamma / 2
    intr = camModel == KB_EUCM ? std::vector<double>{0.5, 1.0, 0.5 * g, 0.5 * g, cu, cv}
                               : std::vector<double>{0.0, 0.5, 0.5 * g, 0.5 * g, cu, cv};
    return true;
  }
  const int nd = n_distortion(camModel);
  if (nd < 0) throw std::runtime_error("initializeIntrinsics: unknown camera model");
  const double cu = (observations[0].imCols - 1.0) / 2.0, cv = (observations[0].imRows - 1.0) / 2.0;
  const size_t R = target.rows(), Cn = target.cols();
  std::vector<double> guesses;
  for (const GridObservation& obs : observations) {
    std::vector<std::array<double, 3>> circ(R);  // centre x, y, radius per corner row
    bool skip = false;
    for (size_t r = 0; r < R; ++r) {
      std::vector<std::array<double, 2>> pts;
      for (size_t c = 0; c < Cn; ++c) {
        double p[2];
        if (obs.imagePoint(r * Cn + c, p)) pts.push_back({p[0], p[1]});
        else skip = true;  // the view is not complete
      }
      if (!pts.empty()) fit_circle(pts, circ[r][0], circ[r][1], circ[r][2]);
    }
    if (skip) continue;
    for (size_t j = 0; j < R; ++j)
      for (size_t k = j + 1; k < std::min(Cn, R); ++k) {
        const auto ip = intersect_circles(circ[j][0], circ[j][1], circ[j][2], circ[k][0], circ[k][1], circ[k][2]);
        if (ip.size() < 2) continue;
        const double f = std::hypot(ip[0][0] - ip[1][0], ip[0][1] - ip[1][1]) / M_PI;
        if (std::isfinite(f)) guesses.push_back(f);
      }
  }
  if (guesses.empty()) {
    if (!fallbackFocalLength) return false;
    guesses.push_back(*fallbackFocalLength);
  }
  const double f0 = median_of(guesses);
  intr.assign(4 + nd, 0.0);
  intr[0] = f0;
  intr[1] = f0;
  intr[2] = cu;
  intr[3] = cv;
  return true;
}

bool keypointToEuclidean(int32_t camModel, const double* intr, size_t imCols, size_t imRows, const double kp[2],
                         double out[3]) {
  switch (camModel) {
    case KB_PINHOLE_RADTAN:
    case KB_PINHOLE_EQUI:
    case KB_PINHOLE_FOV: {  // PinholeProjection.hpp(impl):202-227
      double bx = (kp[0] - intr[2]) / intr[0], by = (kp[1] - intr[3]) / intr[1];
      undistort(camModel, intr + 4, bx, by);
      out[0] = bx;
      out[1] = by;
      out[2] = 1.0;
      return kp[0] >= 0.0 && kp[1] >= 0.0 && kp[0] < (double)imCols && kp[1] < (double)imRows;  // isValid
    }
    case KB_OMNI_RADTAN:
    case KB_OMNI: {  // OmniProjection.hpp(impl):230-262 (no isValid test of the keypoint)
      const double xi = intr[0];
      double mx = (kp[0] - intr[3]) / intr[1], my = (kp[1] - intr[4]) / intr[2];
      if (camModel == KB_OMNI_RADTAN) undistort(KB_PINHOLE_RADTAN, intr + 5, mx, my);
      const double r2 = mx * mx + my * my;
      if (!(xi <= 1.0 || r2 <= 1.0 / (xi * xi - 1))) return false;  // isUndistortedKeypointValid (:584-588)
      out[0] = mx;
      out[1] = my;
      out[2] = 1 - xi * (r2 + 1) / (xi + std::sqrt(1 + (1 - xi * xi) * r2));
      return true;
    }
    case KB_EUCM: {  // ExtendedUnifiedProjection.hpp(impl):248-283
      const double alpha = intr[0], beta = intr[1];
      const double mx = (kp[0] - intr[4]) / intr[2], my = (kp[1] - intr[5]) / intr[3], r2 = mx * mx + my * my;
      if (!(alpha <= 0.5 || r2 <= 1.0 / (beta * (2 * alpha - 1)))) return false;  // (:612-616, :655)
      const double gamma = 1 - alpha;
      const double k = (1 - alpha * alpha * beta * r2) / (alpha * std::sqrt(1 - (alpha - gamma) * beta * r2) + gamma);
      const double ninv = 1.0 / std::sqrt(r2 + k * k);
      out[0] = mx * ninv;
      out[1] = my * ninv;
      out[2] = k * ninv;
      return true;
    }
    case KB_DS: {  // DoubleSphereProjection.hpp(impl):271-307
      const double xi = intr[0], alpha = intr[1];
      const double mx = (kp[0] - intr[4]) / intr[2], my = (kp[1] - intr[5]) / intr[3], r2 = mx * mx + my * my;
      if (!(alpha <= 0.5 || r2 <= 1.0 / (2 * alpha - 1))) return false;  // (:660-664, :703)
      const double mz = (1 - alpha * alpha * r2) / (alpha * std::sqrt(1 - (2 * alpha - 1) * r2) + 1 - alpha);
      const double mz2 = mz * mz;
      const double k = (mz * xi + std::sqrt(mz2 + (1 - xi * xi) * r2)) / (mz2 + r2);
      out[0] = k * mx;
      out[1] = k * my;
      out[2] = k * mz - xi;
      return true;
    }
    default: throw std::runtime_error("keypointToEuclidean: unknown camera model");
  }
}

bool estimateTransformation(const GridObservation& obs, const AprilgridTarget& target, int32_t camModel,
                            const double* intr, Transformation& out_T_t_c) {
  const std::vector<double> P = target.points();
  std::vector<std::array<double, 2>> m;  // normalised image points
  std::vector<std::array<double, 3>> X;  // target points
  const double cos80 = std::cos(80.0 * M_PI / 180.0);
  for (size_t i = 0; i < target.size(); ++i) {
    double kp[2], b[3];
    if (!obs.imagePoint(i, kp)) continue;
    if (!keypointToEuclidean(camModel, intr, obs.imCols, obs.imRows, kp, b)) continue;
    if (b[2] / std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]) <= cos80) continue;
    m.push_back({b[0] / b[2], b[1] / b[2]});
    X.push_back({P[3 * i], P[3 * i + 1], P[3 * i + 2]});
  }
  if (m.size() < 4) return false;
  for (const auto& x : X)
    if (x[2] != 0.0) throw std::runtime_error("estimateTransformation: planar targets only");
  // normalised DLT of the homography (X, Y, 1) -> (x, y, 1)
  const size_t n = m.size();
  double mx = 0, my = 0, Mx = 0, My = 0;
  for (size_t i = 0; i < n; ++i) {
    mx += m[i][0];
    my += m[i][1];
    Mx += X[i][0];
    My += X[i][1];
  }
  mx /= n;
  my /= n;
  Mx /= n;
  My /= n;
  double sm = 0, sM = 0;
  for (size_t i = 0; i < n; ++i) {
    sm += std::hypot(m[i][0] - mx, m[i][1] - my);
    sM += std::hypot(X[i][0] - Mx, X[i][1] - My);
  }
  sm = std::sqrt(2.0) * n / sm;
  sM = std::sqrt(2.0) * n / sM;
  std::array<double, 81> AtA{};
  for (size_t i = 0; i < n; ++i) {
    const double X0 = (X[i][0] - Mx) * sM, Y0 = (X[i][1] - My) * sM;
    const double u = (m[i][0] - mx) * sm, v = (m[i][1] - my) * sm;
    const double r1[9] = {-X0, -Y0, -1, 0, 0, 0, u * X0, u * Y0, u};
    const double r2[9] = {0, 0, 0, -X0, -Y0, -1, v * X0, v * Y0, v};
    for (int a = 0; a < 9; ++a)
      for (int b = 0; b < 9; ++b) AtA[a * 9 + b] += r1[a] * r1[b] + r2[a] * r2[b];
  }
  const std::array<double, 9> hn = smallest_eigvec<9>(AtA);
  // denormalise: H = Tm^-1 Hn TM
  const std::array<double, 9> Tmi{1 / sm, 0, mx, 0, 1 / sm, my, 0, 0, 1}, TM{sM, 0, -sM * Mx, 0, sM, -sM * My, 0, 0, 1};
  std::array<double, 9> H = matmul3(Tmi, matmul3(hn, TM));
  // H ~ [r1 r2 t]
  const double n1 = std::sqrt(H[0] * H[0] + H[3] * H[3] + H[6] * H[6]), n2 = std::sqrt(H[1] * H[1] + H[4] * H[4] + H[7] * H[7]);
  double lam = 2.0 / (n1 + n2);
  if (H[8] * lam < 0) lam = -lam;  // target in front of the camera
  std::array<double, 9> Rm;
  double t[3];
  for (int r = 0; r < 3; ++r) {
    Rm[r * 3 + 0] = lam * H[r * 3 + 0];
    Rm[r * 3 + 1] = lam * H[r * 3 + 1];
    t[r] = lam * H[r * 3 + 2];
  }
  Rm[2] = Rm[3] * Rm[7] - Rm[6] * Rm[4];  // r3 = r1 x r2
  Rm[5] = Rm[6] * Rm[1] - Rm[0] * Rm[7];
  Rm[8] = Rm[0] * Rm[4] - Rm[3] * Rm[1];
  for (int it = 0; it < 30; ++it) {  // polar decomposition: R <- (R + R^-T) / 2
    std::array<double, 9> cof{Rm[4] * Rm[8] - Rm[5] * Rm[7], Rm[5] * Rm[6] - Rm[3] * Rm[8], Rm[3] * Rm[7] - Rm[4] * Rm[6],
                              Rm[2] * Rm[7] - Rm[1] * Rm[8], Rm[0] * Rm[8] - Rm[2] * Rm[6], Rm[1] * Rm[6] - Rm[0] * Rm[7],
                              Rm[1] * Rm[5] - Rm[2] * Rm[4], Rm[2] * Rm[3] - Rm[0] * Rm[5], Rm[0] * Rm[4] - Rm[1] * Rm[3]};
    const double det = Rm[0] * cof[0] + Rm[1] * cof[1] + Rm[2] * cof[2];
    for (int k = 0; k < 9; ++k) Rm[k] = 0.5 * (Rm[k] + cof[k] / det);  // R^-T = cof / det
  }
  // Levenberg-Marquardt on the normalised reprojection error, parameters (rotation-vector increment, t)
  auto residual = [&](const std::array<double, 9>& Rr, const double* tt, std::vector<double>& e) {
    e.resize(2 * n);
    double c = 0.0;
    for (size_t i = 0; i < n; ++i) {
      const double* x = X[i].data();
      const double p0 = Rr[0] * x[0] + Rr[1] * x[1] + Rr[2] * x[2] + tt[0];
      const double p1 = Rr[3] * x[0] + Rr[4] * x[1] + Rr[5] * x[2] + tt[1];
      const double p2 = Rr[6] * x[0] + Rr[7] * x[1] + Rr[8] * x[2] + tt[2];
      e[2 * i] = p0 / p2 - m[i][0];
      e[2 * i + 1] = p1 / p2 - m[i][1];
      c += e[2 * i] * e[2 * i] + e[2 * i + 1] * e[2 * i + 1];
    }
    return c;
  };
  std::vector<double> e, e2;
  double cost = residual(Rm, t, e), mu = 1e-3;
  for (int it = 0; it < 50; ++it) {
    double JtJ[36] = {0}, Jte[6] = {0};
    std::vector<double> J(2 * n * 6);
    const double h = 1e-7;
    for (int k = 0; k < 6; ++k) {  // forward differences of the 6 parameters
      double w[3] = {0, 0, 0}, tt[3] = {t[0], t[1], t[2]};
      if (k < 3) w[k] = h;
      else tt[k - 3] += h;
      const std::array<double, 9> Rk = matmul3(rodrigues(w), Rm);
      residual(Rk, tt, e2);
      for (size_t r = 0; r < 2 * n; ++r) J[r * 6 + k] = (e2[r] - e[r]) / h;
    }
    for (size_t r = 0; r < 2 * n; ++r)
      for (int a = 0; a < 6; ++a) {
        Jte[a] += J[r * 6 + a] * e[r];
        for (int b = 0; b < 6; ++b) JtJ[a * 6 + b] += J[r * 6 + a] * J[r * 6 + b];
      }
    bool improved = false;
    for (int tries = 0; tries < 10 && !improved; ++tries) {
      double A[36], bvec[6];
      for (int a = 0; a < 36; ++a) A[a] = JtJ[a];
      for (int a = 0; a < 6; ++a) {
        A[a * 6 + a] += mu * (1.0 + JtJ[a * 6 + a]);
        bvec[a] = -Jte[a];
      }
      for (int k = 0; k < 6; ++k) {  // Gaussian elimination with partial pivoting
        int piv = k;
        for (int r = k + 1; r < 6; ++r)
          if (std::fabs(A[r * 6 + k]) > std::fabs(A[piv * 6 + k])) piv = r;
        for (int c = 0; c < 6; ++c) std::swap(A[k * 6 + c], A[piv * 6 + c]);
        std::swap(bvec[k], bvec[piv]);
        for (int r = k + 1; r < 6; ++r) {
          const double fct = A[r * 6 + k] / A[k * 6 + k];
          for (int c = k; c < 6; ++c) A[r * 6 + c] -= fct * A[k * 6 + c];
          bvec[r] -= fct * bvec[k];
        }
      }
      double dlt[6];
      for (int k = 5; k >= 0; --k) {
        double sacc = bvec[k];
        for (int c = k + 1; c < 6; ++c) sacc -= A[k * 6 + c] * dlt[c];
        dlt[k] = sacc / A[k * 6 + k];
      }
      const std::array<double, 9> Rn = matmul3(rodrigues(dlt), Rm);
      const double tn[3] = {t[0] + dlt[3], t[1] + dlt[4], t[2] + dlt[5]};
      const double cn = residual(Rn, tn, e2);
      if (cn < cost) {
        Rm = Rn;
        t[0] = tn[0];
        t[1] = tn[1];
        t[2] = tn[2];
        const double rel = (cost - cn) / std::max(cost, 1e-300);
        cost = cn;
        e = e2;
        mu = std::max(mu * 0.3, 1e-12);
        improved = true;
        if (rel < 1e-14) it = 50;
      } else {
        mu *= 10.0;
      }
    }
    if (!improved) break;
  }
  // T_c_t = (R, t); out = T_t_c = T_c_t^-1
  std::array<double, 9> Rt{Rm[0], Rm[3], Rm[6], Rm[1], Rm[4], Rm[7], Rm[2], Rm[5], Rm[8]};
  const std::array<double, 3> ti{-(Rt[0] * t[0] + Rt[1] * t[1] + Rt[2] * t[2]), -(Rt[3] * t[0] + Rt[4] * t[1] + Rt[5] * t[2]),
                                 -(Rt[6] * t[0] + Rt[7] * t[1] + Rt[8] * t[2])};
  out_T_t_c = Transformation::fromMatrix(Rt, ti);
  return true;
}

}  // namespace io
}  // namespace kalibr_amd
