// calibration_io.hpp -- the data formats either side of the hot path:
//   in:  AprilGrid target geometry + GridCalibrationTargetObservation records grouped in synchronized sets,
//        packed into the device problem exactly as CalibrateMultiCameraRig creates its terms;
//   out: the calibration as ROS CameraInfo / TransformStamped / TFMessage YAML, as kalibr_calibrate_cameras
//        exports it.
// Paths are relative to the reference repository.  Target detection (AprilTags, OpenCV) is not rebuilt; the
// initialisers of every model (initializeIntrinsics, estimateTransformation) are, without OpenCV.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "kalibr_backend.hpp"

namespace kalibr_amd {
namespace io {

/// sm::kinematics::Transformation: JPL quaternion q = (x, y, z, w) of C_a_b and t_a_b_a
/// (Schweizer-Messer/sm_kinematics/src/Transformation.cpp).
struct Transformation {
  std::array<double, 4> q{0.0, 0.0, 0.0, 1.0};
  std::array<double, 3> t{0.0, 0.0, 0.0};
  /// operator* (Transformation.cpp:95-98): q = qplus(q_a, q_b) normalised, t = C(q_a) t_b + t_a
  Transformation operator*(const Transformation& rhs) const;
  /// the rotation matrix (quat2r, quaternion_algebra.cpp:77-101), row-major
  std::array<double, 9> C() const;
  /// Transformation(T) (Transformation.cpp:24-29): q = r2quat(C) (canonical sign, w >= 0)
  static Transformation fromMatrix(const std::array<double, 9>& C, const std::array<double, 3>& t);
};

/// GridCalibrationTargetAprilgrid geometry (aslam_cv/aslam_cameras_april/src/GridCalibrationTargetAprilgrid.cpp:
/// 29-32, 83-95): 2 tagRows x 2 tagCols corners, row-major index r * cols + c, z = 0.
struct AprilgridTarget {
  size_t tagRows = 5, tagCols = 6;  // kalibr2_ros/calibration_config.yaml:1-6 (6 x 5 tags)
  double tagSize = 0.088, tagSpacing = 0.2954;
  size_t rows() const { return 2 * tagRows; }
  size_t cols() const { return 2 * tagCols; }
  size_t size() const { return rows() * cols(); }
  std::vector<double> points() const;  // [size][3]
};

/// GridCalibrationTargetObservation (aslam_cv/aslam_cameras/include/aslam/cameras/
/// GridCalibrationTargetObservation.hpp:46-150): row-major image points of every target corner, a success
/// flag per corner, the image size and (once estimateTransformation ran) T_t_c.
struct GridObservation {
  std::vector<double> points;    // [target size][2]
  std::vector<uint8_t> success;  // [target size]
  size_t imRows = 0, imCols = 0;
  std::optional<Transformation> T_t_c;
  double time = 0.0;

  explicit GridObservation(size_t targetSize = 0) : points(2 * targetSize, 0.0), success(targetSize, 0) {}
  /// imagePoint(i, out): false if corner i was not seen
  bool imagePoint(size_t i, double out[2]) const;
  /// updateImagePoint(i, p): sets the point and marks it seen
  void updateImagePoint(size_t i, double u, double v);
  /// removeImagePoint(i)
  void removeImagePoint(size_t i);
  /// getCornersIdx: indices of the seen corners; returns their count
  unsigned getCornersIdx(std::vector<unsigned>& idx) const;
  bool hasSuccessfulObservation() const;
};

/// one synchronized set: an optional observation per camera (CalibrationTools.hpp:28)
using SyncedSet = std::vector<std::optional<GridObservation>>;

/// getTargetPoseGuess (CalibrationTools.hpp:315-355): T_t_c of the camera with the most corners, carried to
/// camera 0 as std::accumulate(baselines[0 .. max), T_t_cN, *) -- i.e. T_t_cN * B_0 * ... * B_{max-1}, the
/// reference's multiplication order.  Throws if that observation has no T_t_c.
Transformation targetPoseGuess(const SyncedSet& set, const std::vector<Transformation>& baselineGuesses);

/// CalibrateMultiCameraRig's problem (CalibrationTools.hpp:376-414): intrinsics DVs, baseline DVs, one target
/// pose DV per synchronized set (initialised by targetPoseGuess, stored as T_f = T_t_c0), one ReprojectionError
/// per seen corner of every present observation (CameraCalibrator.hpp:203-265 loops over the target corners in
/// index order).  intrinsics: [n_cams][KB_MAX_INTR] in the state layout of include/kalibr_hip.h.
backend::CalibrationProblem buildRigProblem(const std::vector<int32_t>& camModels,
                                            const std::vector<double>& intrinsics, const AprilgridTarget& target,
                                            const std::vector<SyncedSet>& sets,
                                            const std::vector<Transformation>& baselineGuesses);

// ---------------------------------------------------------------- initialisers (Pinhole / Omni / EUCM / DS)
/// PinholeProjection::initializeIntrinsics (aslam_cv/aslam_cameras/include/aslam/cameras/implementation/
/// PinholeProjection.hpp:713-803): image centre (cols - 1) / 2, (rows - 1) / 2; focal length = the median over the
/// complete views of |v1 - v2| / pi for the intersections v1, v2 of the circles fitted to pairs of corner rows
/// (Hughes et al., PAMI 2010; circle fit by modified least squares, Umbach & Jones 2000, :642-691); the fallback
/// when no guess is finite.  intr = [fu fv cu cv | distortion cleared to 0] (4 + nDistortion values).
/// Deviation: the reference pairs row j with rows j + 1 .. target.cols() - 1 and so reads past its row array when
/// cols > rows; here the pairs stop at the last row.  Returns false (the reference's SM_ERROR path) when neither a
/// guess nor a fallback exists.
/// Omni / omni-radtan (OmniProjection.hpp(impl):724-846): xi = 1, the image centre, the focal length gamma from the
/// conic fitted to each corner row (the row's image under xi = 1), scored by the view's mean reprojection error
/// under the pose estimateTransformation finds with it; intr = [1 gamma gamma cu cv | distortion 0].  With no
/// scored row: the fallback focal length is set and false returned (the reference's warning path), or false.
/// EUCM (ExtendedUnifiedProjection.hpp(impl):731-760) and DS (DoubleSphereProjection.hpp(impl):783-812) run the
/// omni initialiser and, on success only, map it onto the same rays: EUCM [alpha 1/2, beta 1, gamma/2, gamma/2,
/// cu, cv], DS [xi 0, alpha 1/2, gamma/2, gamma/2, cu, cv].
bool initializeIntrinsics(const std::vector<GridObservation>& observations, const AprilgridTarget& target,
                          std::optional<double> fallbackFocalLength, int32_t camModel, std::vector<double>& intr);

/// keypointToEuclidean of every model: pinhole (PinholeProjection.hpp(impl):202-227: normalised coordinates, the
/// distortion inverted by 5 Gauss-Newton steps for radtan (RadialTangentialDistortion.hpp(impl):68-98) and up to 20
/// for equidistant / FOV; false off the image, isValid); omni (OmniProjection.hpp(impl):230-262, radtan undistorted
/// first), EUCM (ExtendedUnifiedProjection.hpp(impl):248-283), DS (DoubleSphereProjection.hpp(impl):271-307): the
/// lifted ray, false where isUndistortedKeypointValid fails (the keypoint itself is not range-checked there).
bool keypointToEuclidean(int32_t camModel, const double* intr, size_t imCols, size_t imRows, const double kp[2],
                         double out[3]);

/// estimateTransformation (PinholeProjection.hpp(impl):811-880; OmniProjection.hpp(impl):871-958, EUCM and DS
/// alike): the seen corners back-projected (kept when the ray is within 80 degrees of the axis), then the pose of
/// the planar target from those points' x/z, y/z -- solvePnP with K = I there; here a normalised-DLT homography,
/// its decomposition into (R, t) and a Levenberg-Marquardt refinement of the normalised reprojection error.  out_T_t_c takes camera points to the target frame.  False
/// with fewer than 4 usable corners.
bool estimateTransformation(const GridObservation& obs, const AprilgridTarget& target, int32_t camModel,
                            const double* intr, Transformation& out_T_t_c);

// ---------------------------------------------------------------- export (kalibr2_ros)
/// CameraCalibratorBase::CameraInfoParams (kalibr2/include/kalibr2/CameraCalibrator.hpp:156-191)
struct CameraInfoParams {
  double fx = 0, fy = 0, cx = 0, cy = 0;
  std::vector<double> d;
};
CameraInfoParams cameraInfoParams(int32_t camModel, const double* intr);
/// Kalibr2 model name of a kb_camera_model ("pinhole-radtan", "omni-radtan", "eucm-none", "omni-none",
/// "ds-none", "pinhole-equi", "pinhole-fov"; kalibr2_ros Config.cpp model strings)
std::string kalibrModelName(int32_t camModel);
/// ToROSDistortionModel (KalibrToROSConverter.hpp:26-44, KalibrToROSConverter.cpp:5-13); "unknown" fallback
std::string toRosDistortionModel(const std::string& kalibrModel);

/// geometry_msgs TransformStamped as TransformationToROS fills it (KalibrToROSConverter.cpp:15-37)
struct TransformStamped {
  std::string frame_id, child_frame_id;
  std::array<double, 3> translation{};
  std::array<double, 4> rotation{};  // x, y, z, w = the JPL quaternion fields, as the reference copies them
};
TransformStamped transformationToRos(const Transformation& T, const std::string& parent, const std::string& child);

/// CalibratorToYAML (ROSToYAMLConverter.cpp:32-75): CameraInfo in rosidl block style
std::string cameraInfoYaml(const CameraInfoParams& p, const std::string& kalibrModel, const std::string& frameId,
                           size_t width, size_t height);
/// transformStampedToYAML / tfMessageToYAML (ROSToYAMLConverter.cpp:14-30)
std::string transformStampedYaml(const TransformStamped& tf);
std::string tfMessageYaml(const std::vector<TransformStamped>& tfs);

/// The export step of kalibr_calibrate_cameras (CalibrateCameras.cpp:313-356) from a solved flat state:
/// calibration_<camera>.yaml per camera, then transform_<cam0>_to_<cam1>.yaml (one baseline) or
/// camera_chain_transforms.yaml (several); each baseline re-read through Transformation(T) as the reference
/// does.  Returns the written paths.
std::vector<std::string> exportCalibration(const std::string& outputDir, const std::vector<std::string>& cameraNames,
                                           const std::vector<int32_t>& camModels,
                                           const std::vector<std::pair<size_t, size_t>>& imageSizes,
                                           const std::vector<double>& state);

}  // namespace io
}  // namespace kalibr_amd
