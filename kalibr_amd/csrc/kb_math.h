// kb_math.h -- device maths for the calibration hot path (gfx950, FP64).
//
// Restates, for the GPU, the per-term quantities of the reference:
//   quaternion algebra  Schweizer-Messer/sm_kinematics/src/quaternion_algebra.cpp:77-101,200-220,302-315
//   camera projections  aslam_cv/aslam_cameras/include/aslam/cameras/implementation/
//                        PinholeProjection.hpp:99-145,310-378; RadialTangentialDistortion.hpp:28-65,152-182;
//                        OmniProjection.hpp:117-183,383-445; ExtendedUnifiedProjection.hpp:131-198,399-457;
//                        DoubleSphereProjection.hpp:140-221,443-505; EquidistantDistortion.hpp:31-200,244-273;
//                        FovDistortion.hpp:19-83,130-168
// (paths relative to the reference repository).  Written once for the device; the CPU
// oracle under oracle/ is an independent restatement used only as the checker.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/kalibr_hip.h"

namespace kb {

// eps^(1/4) for doubles == 2^-13 exactly (quaternion_algebra.cpp:10-13)
constexpr double kEps4thRoot = 1.220703125e-4;

// 1/z of a projection: v_rcp_f64 + two Newton steps, within an ulp of the IEEE quotient (the division's scale /
// fixup sequence is ~10 dependent instructions on every corner's chain)
__device__ __forceinline__ double proj_recip(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

__device__ __forceinline__ void quat2r(const double* q, double* R) {
  R[0] = q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3];
  R[1] = q[0] * q[1] * 2.0 + q[2] * q[3] * 2.0;
  R[2] = q[0] * q[2] * 2.0 - q[1] * q[3] * 2.0;
  R[3] = q[0] * q[1] * 2.0 - q[2] * q[3] * 2.0;
  R[4] = -q[0] * q[0] + q[1] * q[1] - q[2] * q[2] + q[3] * q[3];
  R[5] = q[0] * q[3] * 2.0 + q[1] * q[2] * 2.0;
  R[6] = q[0] * q[2] * 2.0 + q[1] * q[3] * 2.0;
  R[7] = q[0] * q[3] * (-2.0) + q[1] * q[2] * 2.0;
  R[8] = -q[0] * q[0] - q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
}

// q <- axisAngle2quat(dq) (x) q  (JPL), translation additive: one pose DV update.
__device__ __forceinline__ void update_pose(const double* in, const double* d6, double* out) {
  const double a0 = d6[0], a1 = d6[1], a2 = d6[2];
  const double th = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
  double sh, ca;
  sincos(th * 0.5, &sh, &ca);  // one argument reduction for both
  const double na = (th < kEps4thRoot) ? 0.5 + (th * th) * (1.0 / 48.0) : sh / th;
  const double d0 = a0 * na, d1 = a1 * na, d2 = a2 * na;
  const double q0 = in[0], q1 = in[1], q2 = in[2], q3 = in[3];
  out[0] = q0 * ca + d0 * q3 - d1 * q2 + d2 * q1;
  out[1] = q1 * ca + d0 * q2 + d1 * q3 - d2 * q0;
  out[2] = q2 * ca - d0 * q1 + d1 * q0 + d2 * q3;
  out[3] = q3 * ca - d0 * q0 - d1 * q1 - d2 * q2;
  out[4] = in[4] + d6[3];
  out[5] = in[5] + d6[4];
  out[6] = in[6] + d6[5];
}

__device__ __forceinline__ int model_nintr(int m) {
  return (m == KB_PINHOLE_RADTAN || m == KB_PINHOLE_EQUI) ? 8 : m == KB_OMNI_RADTAN ? 9
         : (m == KB_EUCM || m == KB_DS)                   ? 6 : 5;
}

// Equidistant: y *= thetad / r, theta = atan r (scaling 1 for r <= 1e-8).  Jd = d(y')/dy (2x2, row-major),
// Jk = d(y')/dk (2x4, row-major), both evaluated at the undistorted y, as the reference does.
__device__ __forceinline__ void equi(const double* k, double& x, double& y, double* Jd, double* Jk) {
  const double r2 = x * x + y * y, r = sqrt(r2), th = atan(r), t2 = th * th;
  const double P = 1.0 + t2 * (k[0] + t2 * (k[1] + t2 * (k[2] + t2 * k[3])));
  const double thd = th * P;
  if (Jd) {
    const double dP = 1.0 + t2 * (3.0 * k[0] + t2 * (5.0 * k[1] + t2 * (7.0 * k[2] + t2 * 9.0 * k[3])));
    const double s = thd / r, g = (dP / (1.0 + r2) - s) / r2;
    Jd[0] = s + x * x * g;
    Jd[1] = x * y * g;
    Jd[2] = Jd[1];
    Jd[3] = s + y * y * g;
    const double a = th * t2 / r, b = a * t2, c = b * t2, e = c * t2;
    Jk[0] = x * a; Jk[1] = x * b; Jk[2] = x * c; Jk[3] = x * e;
    Jk[4] = y * a; Jk[5] = y * b; Jk[6] = y * c; Jk[7] = y * e;
  }
  const double sc = (r > 1e-8) ? thd / r : 1.0;
  x *= sc;
  y *= sc;
}

// FOV: y *= atan(2 tan(w/2) r) / (w r), with the reference's limits (w^2 < 1e-5: identity; r^2 < 1e-5: constant
// scale 2 tan(w/2)/w, constant w column (w - sin w)/(w^2 cos^2(w/2)) in both rows).  Jw = d(y')/dw (2).
__device__ __forceinline__ void fov(double w, double& x, double& y, double* Jd, double* Jw) {
  const double u = x, v = y, r2 = u * u + v * v, r = sqrt(r2);
  const double tw = tan(0.5 * w), tw2 = tw * tw;
  double s;
  if (w * w < 1e-5) {
    s = 1.0;
    if (Jd) { Jd[0] = 1.0; Jd[1] = 0.0; Jd[2] = 0.0; Jd[3] = 1.0; Jw[0] = 0.0; Jw[1] = 0.0; }
  } else if (r2 < 1e-5) {
    s = 2.0 * tw / w;
    if (Jd) {
      const double c = cos(0.5 * w);
      Jd[0] = s; Jd[1] = 0.0; Jd[2] = 0.0; Jd[3] = s;
      Jw[0] = Jw[1] = (w - sin(w)) / (w * w * c * c);
    }
  } else {
    const double den = 1.0 / (w * (1.0 + 4.0 * tw2 * r2));
    s = atan(2.0 * tw * r) / (r * w);
    if (Jd) {
      const double q = (2.0 * tw * den - s) / r2;
      Jd[0] = s + u * u * q;
      Jd[1] = u * v * q;
      Jd[2] = Jd[1];
      Jd[3] = s + v * v * q;
      const double ds = (1.0 + tw2) * den - s / w;
      Jw[0] = u * ds;
      Jw[1] = v * ds;
    }
  }
  x = u * s;
  y = v * s;
}

__device__ __forceinline__ void radtan(const double* d, double& x, double& y, double* Jd) {
  const double k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3];
  const double mx2 = x * x, my2 = y * y, mxy = x * y, rho2 = mx2 + my2;
  const double rad = k1 * rho2 + k2 * rho2 * rho2;
  Jd[0] = 1 + rad + k1 * 2.0 * mx2 + k2 * rho2 * 4 * mx2 + 2.0 * p1 * y + 6 * p2 * x;
  Jd[2] = k1 * 2.0 * x * y + k2 * 4 * rho2 * x * y + p1 * 2.0 * x + 2.0 * p2 * y;
  Jd[1] = Jd[2];
  Jd[3] = 1 + rad + k1 * 2.0 * my2 + k2 * rho2 * 4 * my2 + 6 * p1 * y + 2.0 * p2 * x;
  const double nx = x + x * rad + 2.0 * p1 * mxy + p2 * (rho2 + 2.0 * mx2);
  const double ny = y + y * rad + 2.0 * p2 * mxy + p1 * (rho2 + 2.0 * my2);
  x = nx;
  y = ny;
}

__device__ __forceinline__ void radtan_only(const double* d, double& x, double& y) {
  const double k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3];
  const double mx2 = x * x, my2 = y * y, mxy = x * y, rho2 = mx2 + my2;
  const double rad = k1 * rho2 + k2 * rho2 * rho2;
  const double nx = x + x * rad + 2.0 * p1 * mxy + p2 * (rho2 + 2.0 * mx2);
  const double ny = y + y * rad + 2.0 * p2 * mxy + p1 * (rho2 + 2.0 * my2);
  x = nx;
  y = ny;
}

// Camera-model sets: kernels are instantiated per set of models present in the rig, so a one-model rig
// compiles only its own projection (the all-models union costs the build kernel ~40 spilled VGPRs).
constexpr unsigned kMmAll = 0x7Fu;
#define KB_MM(m) ((MM >> (m)) & 1u)

// Keypoint only (cost pass).
template <unsigned MM = kMmAll>
__device__ __forceinline__ void project(int model, const double* in, double px, double py, double pz, double& u,
                                        double& v) {
  if (MM == (1u << KB_PINHOLE_RADTAN)) model = KB_PINHOLE_RADTAN;  // single-model sets: constant model
  else if (MM == (1u << KB_OMNI_RADTAN)) model = KB_OMNI_RADTAN;
  else if (MM == (1u << KB_EUCM)) model = KB_EUCM;
  else if (MM == (1u << KB_OMNI)) model = KB_OMNI;
  else if (MM == (1u << KB_DS)) model = KB_DS;
  else if (MM == (1u << KB_PINHOLE_EQUI)) model = KB_PINHOLE_EQUI;
  else if (MM == (1u << KB_PINHOLE_FOV)) model = KB_PINHOLE_FOV;
  if (KB_MM(KB_PINHOLE_RADTAN) && model == KB_PINHOLE_RADTAN) {
    const double rz = proj_recip(pz);
    double x = px * rz, y = py * rz;
    radtan_only(in + 4, x, y);
    u = in[0] * x + in[2];
    v = in[1] * y + in[3];
  } else if ((KB_MM(KB_OMNI_RADTAN) && model == KB_OMNI_RADTAN) || (KB_MM(KB_OMNI) && model == KB_OMNI)) {
    const double xi = in[0];
    const double d = sqrt(px * px + py * py + pz * pz);
    const double rz = 1.0 / (pz + xi * d);
    double x = px * rz, y = py * rz;
    if (KB_MM(KB_OMNI_RADTAN) && model == KB_OMNI_RADTAN) radtan_only(in + 5, x, y);
    u = in[1] * x + in[3];
    v = in[2] * y + in[4];
  } else if (KB_MM(KB_EUCM) && model == KB_EUCM) {
    const double al = in[0], be = in[1];
    const double d = sqrt(be * (px * px + py * py) + pz * pz);
    const double ninv = 1.0 / (al * d + (1 - al) * pz);
    u = in[2] * (px * ninv) + in[4];
    v = in[3] * (py * ninv) + in[5];
  } else if (KB_MM(KB_DS) && model == KB_DS) {
    const double xi = in[0], al = in[1], r2 = px * px + py * py;
    const double k = xi * sqrt(r2 + pz * pz) + pz;
    const double ninv = 1.0 / (al * sqrt(r2 + k * k) + (1 - al) * k);
    u = in[2] * (px * ninv) + in[4];
    v = in[3] * (py * ninv) + in[5];
  } else if (KB_MM(KB_PINHOLE_EQUI) || KB_MM(KB_PINHOLE_FOV)) {  // pinhole + equidistant / FOV
    const double rz = proj_recip(pz);
    double x = px * rz, y = py * rz;
    if (KB_MM(KB_PINHOLE_EQUI) && (!KB_MM(KB_PINHOLE_FOV) || model == KB_PINHOLE_EQUI))
      equi(in + 4, x, y, nullptr, nullptr);
    else
      fov(in[4], x, y, nullptr, nullptr);
    u = in[0] * x + in[2];
    v = in[1] * y + in[3];
  }
}

// Keypoint, dy/dp (2x3, row-major Jp[6]) and dy/dintrinsics (Ji[2][KB_MAX_INTR] row-major, only the
// first nintr columns written).  Mirrors the reference per model, including its quirks (EUCM alpha/beta
// rows both scaled by fu, ExtendedUnifiedProjection.hpp(impl):440-441).
template <unsigned MM = kMmAll>
__device__ __forceinline__ void project_jac(int model, const double* in, double px, double py, double pz, double& u,
                                            double& v, double* Jp, double* Ji) {
  if (MM == (1u << KB_PINHOLE_RADTAN)) model = KB_PINHOLE_RADTAN;
  else if (MM == (1u << KB_OMNI_RADTAN)) model = KB_OMNI_RADTAN;
  else if (MM == (1u << KB_EUCM)) model = KB_EUCM;
  else if (MM == (1u << KB_OMNI)) model = KB_OMNI;
  else if (MM == (1u << KB_DS)) model = KB_DS;
  else if (MM == (1u << KB_PINHOLE_EQUI)) model = KB_PINHOLE_EQUI;
  else if (MM == (1u << KB_PINHOLE_FOV)) model = KB_PINHOLE_FOV;
  if (KB_MM(KB_PINHOLE_RADTAN) && model == KB_PINHOLE_RADTAN) {
    const double fu = in[0], fv = in[1];
    const double rz = proj_recip(pz), rz2 = rz * rz;
    const double ux = px * rz, uy = py * rz;
    double x = ux, y = uy, Jd[4];
    radtan(in + 4, x, y, Jd);
    Jp[0] = fu * Jd[0] * rz;
    Jp[1] = fu * Jd[1] * rz;
    Jp[2] = -fu * (px * Jd[0] + py * Jd[1]) * rz2;
    Jp[3] = fv * Jd[2] * rz;
    Jp[4] = fv * Jd[3] * rz;
    Jp[5] = -fv * (px * Jd[2] + py * Jd[3]) * rz2;
    const double r2 = ux * ux + uy * uy, r4 = r2 * r2;
    Ji[0] = x; Ji[1] = 0.0; Ji[2] = 1.0; Ji[3] = 0.0;
    Ji[4] = ux * r2 * fu; Ji[5] = ux * r4 * fu; Ji[6] = 2.0 * ux * uy * fu; Ji[7] = (r2 + 2.0 * ux * ux) * fu;
    Ji[KB_MAX_INTR + 0] = 0.0; Ji[KB_MAX_INTR + 1] = y; Ji[KB_MAX_INTR + 2] = 0.0; Ji[KB_MAX_INTR + 3] = 1.0;
    Ji[KB_MAX_INTR + 4] = uy * r2 * fv; Ji[KB_MAX_INTR + 5] = uy * r4 * fv;
    Ji[KB_MAX_INTR + 6] = (r2 + 2.0 * uy * uy) * fv; Ji[KB_MAX_INTR + 7] = 2.0 * ux * uy * fv;
    u = fu * x + in[2];
    v = fv * y + in[3];
  } else if ((KB_MM(KB_OMNI_RADTAN) && model == KB_OMNI_RADTAN) || (KB_MM(KB_OMNI) && model == KB_OMNI)) {
    const double xi = in[0], fu = in[1], fv = in[2];
    const double d = sqrt(px * px + py * py + pz * pz);
    const double rz = 1.0 / (pz + xi * d);
    const double ux = px * rz, uy = py * rz;
    double J[6];
    double rzj = rz * rz / d;
    J[0] = rzj * (d * pz + xi * (py * py + pz * pz));
    J[3] = -rzj * xi * px * py;
    J[1] = J[3];
    J[4] = rzj * (d * pz + xi * (px * px + pz * pz));
    rzj = rzj * (-xi * pz - d);
    J[2] = px * rzj;
    J[5] = py * rzj;
    double x = ux, y = uy, Jd[4] = {1.0, 0.0, 0.0, 1.0};
    if (KB_MM(KB_OMNI_RADTAN) && model == KB_OMNI_RADTAN) radtan(in + 5, x, y, Jd);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      Jp[c] = fu * (J[c] * Jd[0] + J[3 + c] * Jd[1]);
      Jp[3 + c] = fv * (J[c] * Jd[2] + J[3 + c] * Jd[3]);
    }
    const double jx0 = -ux * d * rz, jx1 = -uy * d * rz;
    Ji[0] = fu * (Jd[0] * jx0 + Jd[1] * jx1);
    Ji[1] = x; Ji[2] = 0.0; Ji[3] = 1.0; Ji[4] = 0.0;
    Ji[KB_MAX_INTR + 0] = fv * (Jd[2] * jx0 + Jd[3] * jx1);
    Ji[KB_MAX_INTR + 1] = 0.0; Ji[KB_MAX_INTR + 2] = y; Ji[KB_MAX_INTR + 3] = 0.0; Ji[KB_MAX_INTR + 4] = 1.0;
    if (KB_MM(KB_OMNI_RADTAN) && model == KB_OMNI_RADTAN) {
      const double r2 = ux * ux + uy * uy, r4 = r2 * r2;
      Ji[5] = ux * r2 * fu; Ji[6] = ux * r4 * fu; Ji[7] = 2.0 * ux * uy * fu; Ji[8] = (r2 + 2.0 * ux * ux) * fu;
      Ji[KB_MAX_INTR + 5] = uy * r2 * fv; Ji[KB_MAX_INTR + 6] = uy * r4 * fv;
      Ji[KB_MAX_INTR + 7] = (r2 + 2.0 * uy * uy) * fv; Ji[KB_MAX_INTR + 8] = 2.0 * ux * uy * fv;
    }
    u = fu * x + in[3];
    v = fv * y + in[4];
  } else if (KB_MM(KB_EUCM) && model == KB_EUCM) {
    const double al = in[0], be = in[1], fu = in[2], fv = in[3];
    const double xx = px * px, yy = py * py, r2 = xx + yy;
    const double d = sqrt(be * r2 + pz * pz), d_inv = 1.0 / d;
    const double norm = al * d + (1 - al) * pz, ninv = 1.0 / norm;
    const double mx = px * ninv, my = py * ninv;
    const double denom = ninv * ninv * d_inv;
    const double mid = -(al * be * px * py) * denom;
    const double add = norm * d;
    const double addz = (al * pz + (1 - al) * d);
    Jp[0] = fu * (add - px * px * al * be) * denom;
    Jp[3] = fv * mid;
    Jp[1] = fu * mid;
    Jp[4] = fv * (add - py * py * al * be) * denom;
    Jp[2] = -fu * px * addz * denom;
    Jp[5] = -fv * py * addz * denom;
    const double ninv2 = ninv * ninv;
    const double tx = -fu * px * ninv2, ty = -fu * py * ninv2;
    const double t4 = d - pz, t5 = 0.5 * al * r2 * d_inv;
    Ji[0] = tx * t4; Ji[1] = tx * t5; Ji[2] = mx; Ji[3] = 0.0; Ji[4] = 1.0; Ji[5] = 0.0;
    Ji[KB_MAX_INTR + 0] = ty * t4; Ji[KB_MAX_INTR + 1] = ty * t5; Ji[KB_MAX_INTR + 2] = 0.0;
    Ji[KB_MAX_INTR + 3] = my; Ji[KB_MAX_INTR + 4] = 0.0; Ji[KB_MAX_INTR + 5] = 1.0;
    u = fu * mx + in[4];
    v = fv * my + in[5];
  } else if (KB_MM(KB_DS) && model == KB_DS) {
    const double xi = in[0], al = in[1], fu = in[2], fv = in[3];
    const double r2 = px * px + py * py, d1 = sqrt(r2 + pz * pz), d1_inv = 1.0 / d1;
    const double k = xi * d1 + pz, d2 = sqrt(r2 + k * k), d2_inv = 1.0 / d2;
    const double ninv = 1.0 / (al * d2 + (1 - al) * k), ninv2 = ninv * ninv;
    const double mx = px * ninv, my = py * ninv;
    const double tt2 = xi * pz * d1_inv + 1;
    const double dn = (xi * (1 - al) * d1_inv + al * (xi * k * d1_inv + 1) * d2_inv) * ninv2;
    const double t2 = ((1 - al) * tt2 + al * k * tt2 * d2_inv) * ninv2;
    Jp[0] = fu * (ninv - px * px * dn);
    Jp[1] = -fu * px * py * dn;
    Jp[2] = -fu * px * t2;
    Jp[3] = -fv * px * py * dn;
    Jp[4] = fv * (ninv - py * py * dn);
    Jp[5] = -fv * py * t2;
    const double t4 = (al - 1 - al * k * d2_inv) * d1 * ninv2, t5 = (k - d2) * ninv2;
    Ji[0] = fu * px * t4; Ji[1] = fu * px * t5; Ji[2] = mx; Ji[3] = 0.0; Ji[4] = 1.0; Ji[5] = 0.0;
    Ji[KB_MAX_INTR + 0] = fv * py * t4; Ji[KB_MAX_INTR + 1] = fv * py * t5; Ji[KB_MAX_INTR + 2] = 0.0;
    Ji[KB_MAX_INTR + 3] = my; Ji[KB_MAX_INTR + 4] = 0.0; Ji[KB_MAX_INTR + 5] = 1.0;
    u = fu * mx + in[4];
    v = fv * my + in[5];
  } else if (KB_MM(KB_PINHOLE_EQUI) || KB_MM(KB_PINHOLE_FOV)) {  // pinhole + equidistant (4) / FOV (1)
    const bool eq = KB_MM(KB_PINHOLE_EQUI) && (!KB_MM(KB_PINHOLE_FOV) || model == KB_PINHOLE_EQUI);
    const double fu = in[0], fv = in[1];
    const double rz = proj_recip(pz), rz2 = rz * rz;
    double x = px * rz, y = py * rz, Jd[4], Jk[8];
    if (eq)
      equi(in + 4, x, y, Jd, Jk);
    else
      fov(in[4], x, y, Jd, Jk);
    Jp[0] = fu * Jd[0] * rz;
    Jp[1] = fu * Jd[1] * rz;
    Jp[2] = -fu * (px * Jd[0] + py * Jd[1]) * rz2;
    Jp[3] = fv * Jd[2] * rz;
    Jp[4] = fv * Jd[3] * rz;
    Jp[5] = -fv * (px * Jd[2] + py * Jd[3]) * rz2;
    Ji[0] = x; Ji[1] = 0.0; Ji[2] = 1.0; Ji[3] = 0.0;
    Ji[KB_MAX_INTR + 0] = 0.0; Ji[KB_MAX_INTR + 1] = y; Ji[KB_MAX_INTR + 2] = 0.0; Ji[KB_MAX_INTR + 3] = 1.0;
    if (eq) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        Ji[4 + c] = Jk[c] * fu;
        Ji[KB_MAX_INTR + 4 + c] = Jk[4 + c] * fv;
      }
    } else {
      Ji[4] = Jk[0] * fu;
      Ji[KB_MAX_INTR + 4] = Jk[1] * fv;
    }
    u = fu * x + in[2];
    v = fv * y + in[3];
  }
}

}  // namespace kb
