/*
 * kb_oracle.c -- CPU restatement of the aslam_backend GN/LM iteration over
 * camera ReprojectionError terms (TEST INFRASTRUCTURE ONLY, see kb_oracle.h).
 *
 * Every function cites the reference file:line it restates (paths relative to
 * /root/reference).  Plain C99 + pthreads, row-major matrices.
 */
#define _GNU_SOURCE
#include "kb_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* small helpers                                                       */
/* ------------------------------------------------------------------ */

typedef struct {
  void (*fn)(void* ctx, int tid, int nthreads);
  void* ctx;
  int tid, n;
} kbo_job;

static void* kbo_job_run(void* a) {
  kbo_job* j = (kbo_job*)a;
  j->fn(j->ctx, j->tid, j->n);
  return NULL;
}

/* A fresh thread group per call, like LinearSystemSolver::setupThreadedJob
 * (aslam_optimizer/aslam_backend/src/LinearSystemSolver.cpp:50-78). */
static void kbo_parallel(int nthreads, void (*fn)(void*, int, int), void* ctx) {
  if (nthreads <= 1) {
    fn(ctx, 0, 1);
    return;
  }
  pthread_t th[256];
  kbo_job jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].fn = fn;
    jobs[t].ctx = ctx;
    jobs[t].tid = t;
    jobs[t].n = nthreads;
    pthread_create(&th[t], NULL, kbo_job_run, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

static void mat_mul(const double* A, const double* B, double* C, int m, int k, int n) {
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += A[i * k + l] * B[l * n + j];
      C[i * n + j] = s;
    }
}

/* crossMx (Schweizer-Messer/sm_kinematics/src/rotations.cpp:78-84) */
static void cross_mx(const double v[3], double M[9]) {
  M[0] = 0.0;   M[1] = -v[2]; M[2] = v[1];
  M[3] = v[2];  M[4] = 0.0;   M[5] = -v[0];
  M[6] = -v[1]; M[7] = v[0];  M[8] = 0.0;
}

/* boxMinus (sm_kinematics/src/transformations.cpp:45-53): 4x6 */
static void box_minus(const double p[4], double B[24]) {
  memset(B, 0, 24 * sizeof(double));
  B[0 * 6 + 0] = p[3]; B[0 * 6 + 4] = -p[2]; B[0 * 6 + 5] = p[1];
  B[1 * 6 + 1] = p[3]; B[1 * 6 + 3] = p[2];  B[1 * 6 + 5] = -p[0];
  B[2 * 6 + 2] = p[3]; B[2 * 6 + 3] = -p[1]; B[2 * 6 + 4] = p[0];
}

/* boxTimes (sm_kinematics/src/transformations.cpp:132-141): 6x6 of a 4x4 T */
static void box_times(const double T[16], double A[36]) {
  memset(A, 0, 36 * sizeof(double));
  double t[3] = {T[3], T[7], T[11]};
  double tx[9], C[9], txC[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) C[r * 3 + c] = T[r * 4 + c];
  cross_mx(t, tx);
  mat_mul(tx, C, txC, 3, 3, 3);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      A[r * 6 + c] = C[r * 3 + c];
      A[(r + 3) * 6 + c + 3] = C[r * 3 + c];
      A[r * 6 + c + 3] = -txC[r * 3 + c];
    }
}

/* ------------------------------------------------------------------ */
/* quaternion algebra (JPL, [x y z w])                                 */
/* ------------------------------------------------------------------ */

static int less_than_eps_4th_root(double x) {
  /* quaternion_algebra.cpp:10-13 */
  static double e4 = -1.0;
  if (e4 < 0.0) e4 = pow(DBL_EPSILON, 0.25);
  return x < e4;
}

/* quat2r (quaternion_algebra.cpp:77-101) */
void kbo_quat2r(const double q[4], double R[9]) {
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

/* r2quat (quaternion_algebra.cpp:16-75) */
void kbo_r2quat(const double R[9], double q[4]) {
  const double c1 = R[0], c2 = R[3], c3 = R[6], c4 = R[1], c5 = R[4], c6 = R[7], c7 = R[2], c8 = R[5], c9 = R[8];
  double dc[4] = {fabs(1.0 + c1 - c5 - c9), fabs(1.0 - c1 + c5 - c9), fabs(1.0 - c1 - c5 + c9), fabs(1.0 + c1 + c5 + c9)};
  int maxq = 0;
  double maxv = dc[0];
  for (int i = 1; i < 4; ++i)
    if (dc[i] > maxv) { maxq = i; maxv = dc[i]; }
  double c;
  if (maxq == 0) {
    q[0] = 0.5 * sqrt(dc[0]); c = 0.25 / q[0];
    q[1] = c * (c4 + c2); q[2] = c * (c7 + c3); q[3] = c * (c8 - c6);
  } else if (maxq == 1) {
    q[1] = 0.5 * sqrt(dc[1]); c = 0.25 / q[1];
    q[0] = c * (c4 + c2); q[2] = c * (c6 + c8); q[3] = c * (c3 - c7);
  } else if (maxq == 2) {
    q[2] = 0.5 * sqrt(dc[2]); c = 0.25 / q[2];
    q[0] = c * (c3 + c7); q[1] = c * (c6 + c8); q[3] = c * (c4 - c2);
  } else {
    q[3] = 0.5 * sqrt(dc[3]); c = 0.25 / q[3];
    q[0] = c * (c8 - c6); q[1] = c * (c3 - c7); q[2] = c * (c4 - c2);
  }
  if (q[3] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
}

/* axisAngle2quat (quaternion_algebra.cpp:200-220) */
void kbo_axis_angle2quat(const double a[3], double q[4]) {
  double theta = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  double na;
  if (less_than_eps_4th_root(theta)) {
    static const double one_over_48 = 1.0 / 48.0;
    na = 0.5 + (theta * theta) * one_over_48;
  } else {
    na = sin(theta * 0.5) / theta;
  }
  q[0] = a[0] * na;
  q[1] = a[1] * na;
  q[2] = a[2] * na;
  q[3] = cos(theta * 0.5);
}

/* quat2AxisAngle (quaternion_algebra.cpp:228-275) */
void kbo_quat2axis_angle(const double q[4], double a[3]) {
  double na = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]), eta = q[3], scale;
  if (fabs(eta) < na) {
    scale = acos(eta) / na;
  } else if (eta > 0) {
    scale = less_than_eps_4th_root(fabs(na)) ? 1.0 + na * na * (1.0 / 6.0) : asin(na) / na;
  } else {
    scale = (M_PI - asin(na)) / na;
  }
  for (int i = 0; i < 3; ++i) a[i] = q[i] * (2.0 * scale);
}

/* updateQuat (quaternion_algebra.cpp:302-315) */
void kbo_update_quat(const double q[4], const double dq[3], double r[4]) {
  double d[4];
  kbo_axis_angle2quat(dq, d);
  double ca = d[3];
  r[0] = q[0] * ca + d[0] * q[3] - d[1] * q[2] + d[2] * q[1];
  r[1] = q[1] * ca + d[0] * q[2] + d[1] * q[3] - d[2] * q[0];
  r[2] = q[2] * ca - d[0] * q[1] + d[1] * q[0] + d[2] * q[3];
  r[3] = q[3] * ca - d[0] * q[0] - d[1] * q[1] - d[2] * q[2];
}

/* ------------------------------------------------------------------ */
/* camera models                                                       */
/* ------------------------------------------------------------------ */

int kbo_model_nintr(int model) {
  switch (model) {
    case KBO_PINHOLE_RADTAN: return 8;
    case KBO_OMNI_RADTAN: return 9;
    case KBO_EUCM: return 6;
    case KBO_OMNI: return 5;
    case KBO_DS: return 6;
    case KBO_PINHOLE_EQUI: return 8;
    case KBO_PINHOLE_FOV: return 5;
    default: return -1;
  }
}

/* RadialTangentialDistortion::distort(y, J) (aslam_cameras/include/aslam/cameras/
 * implementation/RadialTangentialDistortion.hpp:28-65) */
static void radtan_distort(const double* d, double y[2], double Jd[4]) {
  const double k1 = d[0], k2 = d[1], p1 = d[2], p2 = d[3];
  double mx2 = y[0] * y[0], my2 = y[1] * y[1], mxy = y[0] * y[1], rho2 = mx2 + my2;
  double rad = k1 * rho2 + k2 * rho2 * rho2;
  if (Jd) {
    Jd[0] = 1 + rad + k1 * 2.0 * mx2 + k2 * rho2 * 4 * mx2 + 2.0 * p1 * y[1] + 6 * p2 * y[0];
    Jd[2] = k1 * 2.0 * y[0] * y[1] + k2 * 4 * rho2 * y[0] * y[1] + p1 * 2.0 * y[0] + 2.0 * p2 * y[1];
    Jd[1] = Jd[2];
    Jd[3] = 1 + rad + k1 * 2.0 * my2 + k2 * rho2 * 4 * my2 + 6 * p1 * y[1] + 2.0 * p2 * y[0];
  }
  y[0] += y[0] * rad + 2.0 * p1 * mxy + p2 * (rho2 + 2.0 * mx2);
  y[1] += y[1] * rad + 2.0 * p2 * mxy + p1 * (rho2 + 2.0 * my2);
}

/* RadialTangentialDistortion::distortParameterJacobian (...RadialTangentialDistortion.hpp:152-182): 2x4 */
static void radtan_param_jac(const double y[2], double J[8]) {
  double y0 = y[0], y1 = y[1], r2 = y0 * y0 + y1 * y1, r4 = r2 * r2;
  J[0] = y0 * r2; J[1] = y0 * r4; J[2] = 2.0 * y0 * y1; J[3] = r2 + 2.0 * y0 * y0;
  J[4] = y1 * r2; J[5] = y1 * r4; J[6] = r2 + 2.0 * y1 * y1; J[7] = 2.0 * y0 * y1;
}

/* EquidistantDistortion::distort(y, J) and distortParameterJacobian (aslam_cameras/include/aslam/cameras/
 * implementation/EquidistantDistortion.hpp:31-200, :244-273): y <- y * thetad(theta)/r, theta = atan r,
 * thetad = theta (1 + k1 theta^2 + k2 theta^4 + k3 theta^6 + k4 theta^8); scaling 1 for r <= 1e-8.
 * The Jacobians are the reference's closed forms, written as the chain rule through r (they are not
 * guarded at r = 0, as in the reference). */
static void equi_distort(const double* k, double y[2], double Jd[4], double Jk[8]) {
  const double x0 = y[0], x1 = y[1];
  const double r2 = x0 * x0 + x1 * x1, r = sqrt(r2), th = atan(r), t2 = th * th;
  const double P = 1.0 + t2 * (k[0] + t2 * (k[1] + t2 * (k[2] + t2 * k[3])));
  const double thd = th * P;
  if (Jd) {
    /* d(thetad)/d(theta) */
    const double dP = 1.0 + t2 * (3.0 * k[0] + t2 * (5.0 * k[1] + t2 * (7.0 * k[2] + t2 * 9.0 * k[3])));
    const double s = thd / r;
    const double g = (dP / (1.0 + r2) - s) / r2; /* (ds/dr) / r */
    Jd[0] = s + x0 * x0 * g;
    Jd[1] = x0 * x1 * g;
    Jd[2] = Jd[1];
    Jd[3] = s + x1 * x1 * g;
  }
  if (Jk) {
    const double t3r = th * t2 / r;
    const double pw[4] = {t3r, t3r * t2, t3r * t2 * t2, t3r * t2 * t2 * t2};
    for (int j = 0; j < 4; ++j) {
      Jk[j] = x0 * pw[j];
      Jk[4 + j] = x1 * pw[j];
    }
  }
  const double sc = (r > 1e-8) ? thd / r : 1.0;
  y[0] *= sc;
  y[1] *= sc;
}

/* FovDistortion::distort(y, J) and distortParameterJacobian (aslam_cameras/include/aslam/cameras/
 * implementation/FovDistortion.hpp:19-83, :130-168), including the reference's limits: w^2 < 1e-5 -> identity;
 * r_u^2 < 1e-5 -> scale 2 tan(w/2)/w with J = that scale times I and the parameter column set to
 * (w - sin w) / (w^2 cos^2(w/2)) in both rows (not multiplied by u, v). */
static void fov_distort(double w, double y[2], double Jd[4], double Jw[2]) {
  const double u = y[0], v = y[1];
  const double ru2 = u * u + v * v, ru = sqrt(ru2);
  const double tw = tan(w / 2.0), tw2 = tw * tw;
  const double at = atan(2.0 * tw * ru);
  double s;
  if (w * w < 1e-5) {
    s = 1.0;
    if (Jd) { Jd[0] = 1.0; Jd[1] = 0.0; Jd[2] = 0.0; Jd[3] = 1.0; }
    if (Jw) { Jw[0] = 0.0; Jw[1] = 0.0; }
  } else if (ru2 < 1e-5) {
    s = 2.0 * tw / w;
    if (Jd) { Jd[0] = s; Jd[1] = 0.0; Jd[2] = 0.0; Jd[3] = s; }
    if (Jw) {
      const double c = cos(w / 2.0);
      Jw[0] = Jw[1] = (w - sin(w)) / (w * w * c * c);
    }
  } else {
    s = at / (ru * w);
    if (Jd) {
      /* d(u s)/du = s + u^2 (ds/dr)/r, ds/dr = (2 tw / (1 + 4 tw^2 r^2)) / (w r) - s / r */
      const double q = (2.0 * tw / (w * (1.0 + 4.0 * tw2 * ru2)) - s) / ru2;
      Jd[0] = s + u * u * q;
      Jd[1] = u * v * q;
      Jd[2] = Jd[1];
      Jd[3] = s + v * v * q;
    }
    if (Jw) {
      /* d s / dw = (1 + tw^2) / (w (1 + 4 tw^2 r^2)) - s / w */
      const double ds = (1.0 + tw2) / (w * (1.0 + 4.0 * tw2 * ru2)) - s / w;
      Jw[0] = u * ds;
      Jw[1] = v * ds;
    }
  }
  y[0] = u * s;
  y[1] = v * s;
}

/* Returns 1 if the keypoint is defined.  Ji is 2 x nintr row-major with stride KBO_MAX_INTR.
 * Pinhole: PinholeProjection.hpp(impl):99-145 (keypoint + Jp), :310-353 (intrinsics), :355-378 (distortion).
 * Omni:    OmniProjection.hpp(impl):117-183, :383-420, :422-445.
 * EUCM:    ExtendedUnifiedProjection.hpp(impl):131-198, :399-457 (note the reference uses fu for
 *          both rows of the alpha/beta columns, :440-441 -- reproduced). */
int kbo_project(int model, const double* in, const double p[3], double y[2], double Jp[6], double Ji[2 * KBO_MAX_INTR]) {
  if (Ji) memset(Ji, 0, 2 * KBO_MAX_INTR * sizeof(double));
  if (model == KBO_PINHOLE_RADTAN) {
    const double fu = in[0], fv = in[1], cu = in[2], cv = in[3];
    double rz = 1.0 / p[2], rz2 = rz * rz;
    double kp[2] = {p[0] * rz, p[1] * rz};
    double un[2] = {kp[0], kp[1]};
    double Jd[4];
    radtan_distort(in + 4, kp, Jd);
    if (Jp) {
      Jp[0] = fu * Jd[0] * rz;
      Jp[1] = fu * Jd[1] * rz;
      Jp[2] = -fu * (p[0] * Jd[0] + p[1] * Jd[1]) * rz2;
      Jp[3] = fv * Jd[2] * rz;
      Jp[4] = fv * Jd[3] * rz;
      Jp[5] = -fv * (p[0] * Jd[2] + p[1] * Jd[3]) * rz2;
    }
    if (Ji) {
      Ji[0] = kp[0]; Ji[2] = 1.0;
      Ji[KBO_MAX_INTR + 1] = kp[1]; Ji[KBO_MAX_INTR + 3] = 1.0;
      double Jr[8];
      radtan_param_jac(un, Jr);
      for (int c = 0; c < 4; ++c) {
        Ji[4 + c] = Jr[c] * fu;
        Ji[KBO_MAX_INTR + 4 + c] = Jr[4 + c] * fv;
      }
    }
    y[0] = fu * kp[0] + cu;
    y[1] = fv * kp[1] + cv;
    return p[2] > 0;
  }
  if (model == KBO_OMNI_RADTAN || model == KBO_OMNI) {
    const double xi = in[0], fu = in[1], fv = in[2], cu = in[3], cv = in[4];
    const int has_dist = (model == KBO_OMNI_RADTAN);
    double d = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    double fovp = (xi <= 1.0) ? xi : 1.0 / xi;
    if (p[2] <= -(fovp * d)) return 0;
    double rz = 1.0 / (p[2] + xi * d);
    double kp[2] = {p[0] * rz, p[1] * rz};
    double un[2] = {kp[0], kp[1]};
    double J[6] = {0};
    double rzj = rz * rz / d;
    J[0] = rzj * (d * p[2] + xi * (p[1] * p[1] + p[2] * p[2]));
    J[3] = -rzj * xi * p[0] * p[1];
    J[1] = J[3];
    J[4] = rzj * (d * p[2] + xi * (p[0] * p[0] + p[2] * p[2]));
    rzj = rzj * (-xi * p[2] - d);
    J[2] = p[0] * rzj;
    J[5] = p[1] * rzj;
    double Jd[4] = {1, 0, 0, 1};
    if (has_dist) radtan_distort(in + 5, kp, Jd);
    if (Jp) {
      for (int c = 0; c < 3; ++c) {
        Jp[c] = fu * (J[c] * Jd[0] + J[3 + c] * Jd[1]);
        Jp[3 + c] = fv * (J[c] * Jd[2] + J[3 + c] * Jd[3]);
      }
    }
    if (Ji) {
      double Jxi0 = -un[0] * d * rz, Jxi1 = -un[1] * d * rz;
      Ji[0] = fu * (Jd[0] * Jxi0 + Jd[1] * Jxi1);
      Ji[KBO_MAX_INTR] = fv * (Jd[2] * Jxi0 + Jd[3] * Jxi1);
      Ji[1] = kp[0]; Ji[3] = 1.0;
      Ji[KBO_MAX_INTR + 2] = kp[1]; Ji[KBO_MAX_INTR + 4] = 1.0;
      if (has_dist) {
        double Jr[8];
        radtan_param_jac(un, Jr);
        for (int c = 0; c < 4; ++c) {
          Ji[5 + c] = Jr[c] * fu;
          Ji[KBO_MAX_INTR + 5 + c] = Jr[4 + c] * fv;
        }
      }
    }
    y[0] = fu * kp[0] + cu;
    y[1] = fv * kp[1] + cv;
    return 1;
  }
  if (model == KBO_EUCM) {
    const double al = in[0], be = in[1], fu = in[2], fv = in[3], cu = in[4], cv = in[5];
    const double x = p[0], yy_ = p[1], z = p[2];
    double xx = x * x, yy = yy_ * yy_, zz = z * z, r2 = xx + yy;
    double d2 = be * r2 + zz, d = sqrt(d2), d_inv = 1.0 / d;
    double fovp = (al <= 0.5) ? al / (1 - al) : (1 - al) / al;
    if (z <= -(fovp * d)) return 0;
    double norm = al * d + (1 - al) * z, norm_inv = 1.0 / norm;
    double mx = x * norm_inv, my = yy_ * norm_inv;
    if (Jp) {
      double denom = norm_inv * norm_inv * d_inv;
      double mid = -(al * be * x * yy_) * denom;
      double add = norm * d;
      double addz = (al * z + (1 - al) * d);
      Jp[0] = fu * (add - x * x * al * be) * denom;
      Jp[3] = fv * mid;
      Jp[1] = fu * mid;
      Jp[4] = fv * (add - yy_ * yy_ * al * be) * denom;
      Jp[2] = -fu * x * addz * denom;
      Jp[5] = -fv * yy_ * addz * denom;
    }
    if (Ji) {
      double norm_inv2 = norm_inv * norm_inv;
      const double tmp_x = -fu * x * norm_inv2;
      const double tmp_y = -fu * yy_ * norm_inv2; /* sic: fu (reference :440-441) */
      const double tmp4 = (d - z);
      const double tmp5 = 0.5 * al * r2 * d_inv;
      Ji[0] = tmp_x * tmp4; Ji[KBO_MAX_INTR + 0] = tmp_y * tmp4;
      Ji[1] = tmp_x * tmp5; Ji[KBO_MAX_INTR + 1] = tmp_y * tmp5;
      Ji[2] = mx; Ji[4] = 1.0;
      Ji[KBO_MAX_INTR + 3] = my; Ji[KBO_MAX_INTR + 5] = 1.0;
    }
    y[0] = fu * mx + cu;
    y[1] = fv * my + cv;
    return 1;
  }
  if (model == KBO_DS) {
    /* DoubleSphereProjection.hpp(impl):140-221 (keypoint + Jp), :443-505 (intrinsics) */
    const double xi = in[0], al = in[1], fu = in[2], fv = in[3], cu = in[4], cv = in[5];
    const double x = p[0], yv = p[1], z = p[2];
    const double r2 = x * x + yv * yv, d1 = sqrt(r2 + z * z), d1_inv = 1.0 / d1;
    const double tmp = (al <= 0.5) ? al / (1 - al) : (1 - al) / al;
    const double fovp = (tmp + xi) / sqrt(2 * tmp * xi + xi * xi + 1);
    if (z <= -(fovp * d1)) return 0;
    const double k = xi * d1 + z, d2 = sqrt(r2 + k * k), d2_inv = 1.0 / d2;
    const double norm = al * d2 + (1 - al) * k, ninv = 1.0 / norm, ninv2 = ninv * ninv;
    const double mx = x * ninv, my = yv * ninv;
    if (Jp) {
      const double tt2 = xi * z * d1_inv + 1;
      const double dn = (xi * (1 - al) * d1_inv + al * (xi * k * d1_inv + 1) * d2_inv) * ninv2;
      const double t2 = ((1 - al) * tt2 + al * k * tt2 * d2_inv) * ninv2;
      Jp[0] = fu * (ninv - x * x * dn);
      Jp[1] = -fu * x * yv * dn;
      Jp[2] = -fu * x * t2;
      Jp[3] = -fv * x * yv * dn;
      Jp[4] = fv * (ninv - yv * yv * dn);
      Jp[5] = -fv * yv * t2;
    }
    if (Ji) {
      const double t4 = (al - 1 - al * k * d2_inv) * d1 * ninv2;
      const double t5 = (k - d2) * ninv2;
      Ji[0] = fu * x * t4; Ji[KBO_MAX_INTR + 0] = fv * yv * t4;
      Ji[1] = fu * x * t5; Ji[KBO_MAX_INTR + 1] = fv * yv * t5;
      Ji[2] = mx; Ji[4] = 1.0;
      Ji[KBO_MAX_INTR + 3] = my; Ji[KBO_MAX_INTR + 5] = 1.0;
    }
    y[0] = fu * mx + cu;
    y[1] = fv * my + cv;
    return 1;
  }
  if (model == KBO_PINHOLE_EQUI || model == KBO_PINHOLE_FOV) {
    /* PinholeProjection.hpp(impl):99-145, :324-378 with the Equidistant / FOV distortion */
    const double fu = in[0], fv = in[1], cu = in[2], cv = in[3];
    const double rz = 1.0 / p[2], rz2 = rz * rz;
    double kp[2] = {p[0] * rz, p[1] * rz};
    double Jd[4], Jk[8];
    const int nd = (model == KBO_PINHOLE_EQUI) ? 4 : 1;
    if (model == KBO_PINHOLE_EQUI)
      equi_distort(in + 4, kp, Jd, Jk);
    else
      fov_distort(in[4], kp, Jd, Jk);
    if (Jp) {
      Jp[0] = fu * Jd[0] * rz;
      Jp[1] = fu * Jd[1] * rz;
      Jp[2] = -fu * (p[0] * Jd[0] + p[1] * Jd[1]) * rz2;
      Jp[3] = fv * Jd[2] * rz;
      Jp[4] = fv * Jd[3] * rz;
      Jp[5] = -fv * (p[0] * Jd[2] + p[1] * Jd[3]) * rz2;
    }
    if (Ji) {
      Ji[0] = kp[0]; Ji[2] = 1.0;
      Ji[KBO_MAX_INTR + 1] = kp[1]; Ji[KBO_MAX_INTR + 3] = 1.0;
      for (int c = 0; c < nd; ++c) {
        Ji[4 + c] = Jk[c] * fu;
        Ji[KBO_MAX_INTR + 4 + c] = Jk[nd + c] * fv;
      }
    }
    y[0] = fu * kp[0] + cu;
    y[1] = fv * kp[1] + cv;
    return p[2] > 0;
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* problem layout                                                      */
/* ------------------------------------------------------------------ */

int kbo_state_size(int n_cams, int n_frames) { return n_cams * KBO_MAX_INTR + KBO_POSE * (n_cams - 1) + KBO_POSE * n_frames; }
static int off_base(const kbo_problem* P) { return P->n_cams * KBO_MAX_INTR; }
static int off_frame(const kbo_problem* P) { return P->n_cams * KBO_MAX_INTR + KBO_POSE * (P->n_cams - 1); }

int kbo_cam_cols(const kbo_problem* P) {
  int c = 0;
  for (int i = 0; i < P->n_cams; ++i) c += kbo_model_nintr(P->cam_model[i]);
  return c + 6 * (P->n_cams - 1);
}
int kbo_total_cols(const kbo_problem* P) { return kbo_cam_cols(P) + 6 * P->n_frames; }

static void col_layout(const kbo_problem* P, int* col_intr, int* col_base) {
  int c = 0;
  for (int i = 0; i < P->n_cams; ++i) { col_intr[i] = c; c += kbo_model_nintr(P->cam_model[i]); }
  for (int j = 0; j < P->n_cams - 1; ++j) { col_base[j] = c; c += 6; }
}

static void pose_matrix(const double* pose, double T[16]) {
  double R[9];
  kbo_quat2r(pose, R);
  memset(T, 0, 16 * sizeof(double));
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T[r * 4 + c] = R[r * 3 + c];
    T[r * 4 + 3] = pose[4 + r];
  }
  T[15] = 1.0;
}

static void rigid_inverse(const double T[16], double Ti[16]) {
  memset(Ti, 0, 16 * sizeof(double));
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) Ti[r * 4 + c] = T[c * 4 + r];
  for (int r = 0; r < 3; ++r) Ti[r * 4 + 3] = -(Ti[r * 4 + 0] * T[3] + Ti[r * 4 + 1] * T[7] + Ti[r * 4 + 2] * T[11]);
  Ti[15] = 1.0;
}

/* TransformationBasic chain maps (aslam_backend_expressions/src/TransformationBasic.cpp:49-66):
 * a 2x6 chain ch (in [rho, phi] perturbation space) -> rotation DV 2x3 and translation DV 2x3,
 * written as J[0..2] = rotation, J[3..5] = translation (DV insertion order q then t,
 * CalibrationTools.hpp:32-45). */
static void basic_dv_jac(const double ch[12], const double t[3], double J[12]) {
  double tx[9];
  cross_mx(t, tx);
  for (int r = 0; r < 2; ++r) {
    for (int c = 0; c < 3; ++c) {
      double s = 0.0;
      for (int l = 0; l < 3; ++l) s += ch[r * 6 + l] * (-tx[l * 3 + c]);
      J[r * 6 + c] = s + ch[r * 6 + 3 + c];
      J[r * 6 + 3 + c] = ch[r * 6 + c];
    }
  }
}

/* One ReprojectionError<Geometry> term, following the expression graph of
 * CalibrateMultiCameraRig (CalibrationTools.hpp:404-408):
 *   T_cam_w = B_{i-1} * ( ... (B_0 * T_f^-1))      p_c = T_cam_w * P
 * Residual: ReprojectionError.hpp(impl):49-60.  Jacobians: impl:62-77 ->
 * HomogeneousExpressionNode.cpp:71-81 (boxMinus), TransformationExpressionNode.cpp:61-72
 * (Multiply: rhs gets chain*boxTimes(T_lhs)), :92-101 (Inverse: -boxTimes(T^-1)),
 * TransformationBasic.cpp:49-66, CameraDesignVariable.hpp(impl):38-54 (-Jp, -Jd).
 * invR = I (CalibrationTools.hpp:391-393), NoMEstimator, DV scaling 1.
 * Outputs: e = y - yhat; Jin 2 x nintr (stride KBO_MAX_INTR); JB[j] 2x6 for j<i; JF 2x6. */
static double term_blocks(const kbo_problem* P, const double* st, int v, int k, double e[2], double* Jin, double (*JB)[12], double JF[12]) {
  const int f = P->view_frame[v], i = P->view_cam[v];
  const int model = P->cam_model[i];
  const double* intr = st + i * KBO_MAX_INTR;
  const double* fp = st + off_frame(P) + KBO_POSE * f;
  double Tf[16], Tinv[16], T[16], tmp[16];
  pose_matrix(fp, Tf);
  rigid_inverse(Tf, Tinv);
  memcpy(T, Tinv, sizeof(T));
  double Tb[16][16];
  for (int j = 0; j < i; ++j) {
    pose_matrix(st + off_base(P) + KBO_POSE * j, Tb[j]);
    mat_mul(Tb[j], T, tmp, 4, 4, 4);
    memcpy(T, tmp, sizeof(T));
  }
  const int cid = P->corner_id[P->view_offset[v] + k];
  const double* X = P->target + 3 * cid;
  double ph[4];
  for (int r = 0; r < 4; ++r) ph[r] = T[r * 4 + 0] * X[0] + T[r * 4 + 1] * X[1] + T[r * 4 + 2] * X[2] + T[r * 4 + 3];
  double yh[2], Jp[6], Ji[2 * KBO_MAX_INTR];
  kbo_project(model, intr, ph, yh, Jp, Ji);
  const double* y = P->y + 2 * (P->view_offset[v] + k);
  e[0] = y[0] - yh[0];
  e[1] = y[1] - yh[1];
  if (Jin) {
    const int n = kbo_model_nintr(model);
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < n; ++c) Jin[r * KBO_MAX_INTR + c] = -Ji[r * KBO_MAX_INTR + c];
  }
  if (JF) {
    /* chain0 = -[Jp | 0] (2x4); lhs of the homogeneous multiply gets chain0 * boxMinus(T p) */
    double ch0[8] = {-Jp[0], -Jp[1], -Jp[2], 0.0, -Jp[3], -Jp[4], -Jp[5], 0.0};
    double Bm[24], ch[12], ch2[12], A[36];
    box_minus(ph, Bm);
    mat_mul(ch0, Bm, ch, 2, 4, 6);
    for (int j = i - 1; j >= 0; --j) {
      double tb[3] = {Tb[j][3], Tb[j][7], Tb[j][11]};
      basic_dv_jac(ch, tb, JB[j]);
      box_times(Tb[j], A);
      mat_mul(ch, A, ch2, 2, 6, 6);
      memcpy(ch, ch2, sizeof(ch));
    }
    box_times(Tinv, A);
    for (int q = 0; q < 36; ++q) A[q] = -A[q];
    mat_mul(ch, A, ch2, 2, 6, 6);
    basic_dv_jac(ch2, fp + 4, JF);
  }
  return e[0] * e[0] + e[1] * e[1];
}

double kbo_term_dense(const kbo_problem* P, const double* st, int v, int k, double e[2], double* Jrow, int ncols) {
  int col_intr[64], col_base[64];
  col_layout(P, col_intr, col_base);
  const int C = kbo_cam_cols(P);
  const int f = P->view_frame[v], i = P->view_cam[v], n = kbo_model_nintr(P->cam_model[i]);
  double Jin[2 * KBO_MAX_INTR], JB[16][12], JF[12];
  double chi2 = term_blocks(P, st, v, k, e, Jin, JB, JF);
  for (int r = 0; r < 2; ++r) {
    double* row = Jrow + (size_t)r * ncols;
    for (int c = 0; c < n; ++c) row[col_intr[i] + c] = Jin[r * KBO_MAX_INTR + c];
    for (int j = 0; j < i; ++j)
      for (int c = 0; c < 6; ++c) row[col_base[j] + c] = JB[j][r * 6 + c];
    for (int c = 0; c < 6; ++c) row[C + 6 * f + c] = JF[r * 6 + c];
  }
  return chi2;
}

/* ------------------------------------------------------------------ */
/* reprojection-error statistics: CameraCalibrator.hpp:368-411 (two passes, in term order) */
/* ------------------------------------------------------------------ */
void kbo_reprojection_stats(const kbo_problem* P, const double* st, double* out) {
  for (int c = 0; c < P->n_cams; ++c) {
    double n = 0.0, s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
    for (int v = 0; v < P->n_views; ++v) { /* pass 1: std::accumulate of the error vectors */
      if (P->view_cam[v] != c) continue;
      const int nk = P->view_offset[v + 1] - P->view_offset[v];
      for (int k = 0; k < nk; ++k) {
        double e[2];
        term_blocks(P, st, v, k, e, NULL, NULL, NULL);
        s0 += e[0];
        s1 += e[1];
        n += 1.0;
      }
    }
    double* o = out + 6 * c;
    for (int q = 0; q < 6; ++q) o[q] = 0.0;
    if (n == 0.0) continue;
    const double m0 = s0 / n, m1 = s1 / n;
    if (n > 1.0) { /* pass 2: squared differences from the mean, divided by N - 1 */
      for (int v = 0; v < P->n_views; ++v) {
        if (P->view_cam[v] != c) continue;
        const int nk = P->view_offset[v + 1] - P->view_offset[v];
        for (int k = 0; k < nk; ++k) {
          double e[2];
          term_blocks(P, st, v, k, e, NULL, NULL, NULL);
          q0 += (e[0] - m0) * (e[0] - m0);
          q1 += (e[1] - m1) * (e[1] - m1);
        }
      }
      o[3] = sqrt(q0 / (n - 1.0));
      o[4] = sqrt(q1 / (n - 1.0));
    }
    o[0] = n;
    o[1] = m0;
    o[2] = m1;
    o[5] = sqrt(s0 * s0 + s1 * s1) / sqrt(n); /* sum_of_errors.norm() / sqrt(size) */
  }
}

/* ------------------------------------------------------------------ */
/* cost: LinearSystemSolver::evaluateError (LinearSystemSolver.cpp:12-23,81-92) */
/* ------------------------------------------------------------------ */

typedef struct {
  const kbo_problem* P;
  const double* st;
  double part[256];
} cost_ctx;

static void cost_job(void* a, int tid, int nt) {
  cost_ctx* c = (cost_ctx*)a;
  const kbo_problem* P = c->P;
  int v0 = (int)((long long)P->n_views * tid / nt), v1 = (int)((long long)P->n_views * (tid + 1) / nt);
  double s = 0.0;
  for (int v = v0; v < v1; ++v) {
    int nk = P->view_offset[v + 1] - P->view_offset[v];
    for (int k = 0; k < nk; ++k) {
      double e[2];
      s += term_blocks(P, c->st, v, k, e, NULL, NULL, NULL);
    }
  }
  c->part[tid] = s;
}

double kbo_eval_cost(const kbo_problem* P, const double* st, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  cost_ctx c;
  c.P = P;
  c.st = st;
  kbo_parallel(nthreads, cost_job, &c);
  double s = 0.0;
  for (int t = 0; t < nthreads; ++t) s += c.part[t];
  return s;
}

/* ------------------------------------------------------------------ */
/* CCS J^T (CompressedColumnJacobianTransposeBuilder(impl).hpp:19-101,  */
/* CompressedColumnMatrix(impl).hpp:236-304,376-387)                    */
/* ------------------------------------------------------------------ */

struct kbo_jt {
  const kbo_problem* P;
  int C, ncols, nrows;        /* rows of J = 2 * n_corners */
  long long* col_ptr;         /* [nrows + 1] (a J^T column per residual row) */
  int* row_ind;               /* [nnz] sorted DV columns */
  double* values;             /* [nnz] */
  double* e_neg;              /* [nrows]  _e = -e_w */
  double cost;
  int col_intr[64], col_base[64];
};

long long kbo_jt_nnz(const kbo_jt* jt) { return jt->col_ptr[jt->nrows]; }

kbo_jt* kbo_jt_create(const kbo_problem* P) {
  kbo_jt* jt = (kbo_jt*)calloc(1, sizeof(kbo_jt));
  jt->P = P;
  jt->C = kbo_cam_cols(P);
  jt->ncols = kbo_total_cols(P);
  jt->nrows = 2 * P->n_corners;
  col_layout(P, jt->col_intr, jt->col_base);
  jt->col_ptr = (long long*)malloc(sizeof(long long) * (jt->nrows + 1));
  long long nnz = 0;
  jt->col_ptr[0] = 0;
  for (int v = 0; v < P->n_views; ++v) {
    int i = P->view_cam[v];
    int per = kbo_model_nintr(P->cam_model[i]) + 6 * i + 6;
    for (int k = P->view_offset[v]; k < P->view_offset[v + 1]; ++k) {
      jt->col_ptr[2 * k + 1] = nnz + per;
      jt->col_ptr[2 * k + 2] = nnz + 2 * per;
      nnz += 2 * per;
    }
  }
  jt->row_ind = (int*)malloc(sizeof(int) * nnz);
  jt->values = (double*)malloc(sizeof(double) * nnz);
  jt->e_neg = (double*)malloc(sizeof(double) * jt->nrows);
  /* symbolic: appendJacobiansSymbolic, blocks sorted by block index (impl:255) */
  for (int v = 0; v < P->n_views; ++v) {
    int i = P->view_cam[v], f = P->view_frame[v], n = kbo_model_nintr(P->cam_model[i]);
    for (int k = P->view_offset[v]; k < P->view_offset[v + 1]; ++k) {
      for (int r = 0; r < 2; ++r) {
        int* ri = jt->row_ind + jt->col_ptr[2 * k + r];
        int q = 0;
        for (int c = 0; c < n; ++c) ri[q++] = jt->col_intr[i] + c;
        for (int j = 0; j < i; ++j)
          for (int c = 0; c < 6; ++c) ri[q++] = jt->col_base[j] + c;
        for (int c = 0; c < 6; ++c) ri[q++] = jt->C + 6 * f + c;
      }
    }
  }
  return jt;
}

void kbo_jt_destroy(kbo_jt* jt) {
  if (!jt) return;
  free(jt->col_ptr);
  free(jt->row_ind);
  free(jt->values);
  free(jt->e_neg);
  free(jt);
}

typedef struct {
  kbo_jt* jt;
  const double* st;
  double part[256];
} jtb_ctx;

static void jt_build_job(void* a, int tid, int nt) {
  jtb_ctx* c = (jtb_ctx*)a;
  kbo_jt* jt = c->jt;
  const kbo_problem* P = jt->P;
  int v0 = (int)((long long)P->n_views * tid / nt), v1 = (int)((long long)P->n_views * (tid + 1) / nt);
  double s = 0.0;
  double Jin[2 * KBO_MAX_INTR], JB[16][12], JF[12], e[2];
  for (int v = v0; v < v1; ++v) {
    int i = P->view_cam[v], n = kbo_model_nintr(P->cam_model[i]);
    int nk = P->view_offset[v + 1] - P->view_offset[v];
    for (int k = 0; k < nk; ++k) {
      int gk = P->view_offset[v] + k;
      s += term_blocks(P, c->st, v, k, e, Jin, JB, JF);
      for (int r = 0; r < 2; ++r) {
        double* val = jt->values + jt->col_ptr[2 * gk + r];
        int q = 0;
        for (int cc = 0; cc < n; ++cc) val[q++] = Jin[r * KBO_MAX_INTR + cc];
        for (int j = 0; j < i; ++j)
          for (int cc = 0; cc < 6; ++cc) val[q++] = JB[j][r * 6 + cc];
        for (int cc = 0; cc < 6; ++cc) val[q++] = JF[r * 6 + cc];
        jt->e_neg[2 * gk + r] = -e[r];
      }
    }
  }
  c->part[tid] = s;
}

void kbo_jt_build(kbo_jt* jt, const double* st, int nthreads, double* rhs) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  jtb_ctx c;
  c.jt = jt;
  c.st = st;
  kbo_parallel(nthreads, jt_build_job, &c);
  double s = 0.0;
  for (int t = 0; t < nthreads; ++t) s += c.part[t];
  jt->cost = s;
  /* rhs = J^T * _e, single-threaded (SparseCholeskyLinearSystemSolver.cpp:39-46;
   * CompressedColumnMatrix::rightMultiply impl:376-387) */
  if (rhs) {
    memset(rhs, 0, sizeof(double) * jt->ncols);
    for (int r = 0; r < jt->nrows; ++r) {
      double er = jt->e_neg[r];
      for (long long q = jt->col_ptr[r]; q < jt->col_ptr[r + 1]; ++q) rhs[jt->row_ind[q]] += jt->values[q] * er;
    }
  }
}

typedef struct {
  kbo_jt* jt;
  kbo_arrow* A;
  double* Hcc_part; /* [nt][C*C] */
  double* gc_part;  /* [nt][C] */
} jtn_ctx;

static void jt_normal_job(void* a, int tid, int nt) {
  jtn_ctx* c = (jtn_ctx*)a;
  kbo_jt* jt = c->jt;
  const kbo_problem* P = jt->P;
  kbo_arrow* A = c->A;
  const int C = jt->C;
  double* Hcc = c->Hcc_part + (size_t)tid * C * C;
  double* gc = c->gc_part + (size_t)tid * C;
  memset(Hcc, 0, sizeof(double) * C * C);
  memset(gc, 0, sizeof(double) * C);
  /* frame-aligned ranges: views are sorted by frame */
  int f0 = (int)((long long)P->n_frames * tid / nt), f1 = (int)((long long)P->n_frames * (tid + 1) / nt);
  for (int f = f0; f < f1; ++f) {
    memset(A->Hff + 36 * (size_t)f, 0, 36 * sizeof(double));
    memset(A->Hfc + (size_t)6 * C * f, 0, 6 * C * sizeof(double));
    memset(A->gf + 6 * (size_t)f, 0, 6 * sizeof(double));
  }
  for (int v = 0; v < P->n_views; ++v) {
    int f = P->view_frame[v];
    if (f < f0 || f >= f1) continue;
    double* Hff = A->Hff + 36 * (size_t)f;
    double* Hfc = A->Hfc + (size_t)6 * C * f;
    double* gf = A->gf + 6 * (size_t)f;
    for (int k = P->view_offset[v]; k < P->view_offset[v + 1]; ++k) {
      for (int r = 2 * k; r < 2 * k + 2; ++r) {
        long long b = jt->col_ptr[r], e = jt->col_ptr[r + 1];
        int ncam = (int)(e - b) - 6; /* camera entries come first (sorted) */
        const int* ri = jt->row_ind + b;
        const double* va = jt->values + b;
        const double* vf = va + ncam;
        double er = jt->e_neg[r];
        for (int p = 0; p < 6; ++p) {
          gf[p] += vf[p] * er;
          for (int q = 0; q < 6; ++q) Hff[p * 6 + q] += vf[p] * vf[q];
          for (int q = 0; q < ncam; ++q) Hfc[p * C + ri[q]] += vf[p] * va[q];
        }
        for (int p = 0; p < ncam; ++p) {
          gc[ri[p]] += va[p] * er;
          for (int q = 0; q < ncam; ++q) Hcc[ri[p] * C + ri[q]] += va[p] * va[q];
        }
      }
    }
  }
}

void kbo_jt_normal_arrow(kbo_jt* jt, int nthreads, kbo_arrow* A) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > jt->P->n_frames) nthreads = jt->P->n_frames > 0 ? jt->P->n_frames : 1;
  if (nthreads > 256) nthreads = 256;
  const int C = jt->C;
  jtn_ctx c;
  c.jt = jt;
  c.A = A;
  c.Hcc_part = (double*)malloc(sizeof(double) * (size_t)nthreads * C * C);
  c.gc_part = (double*)malloc(sizeof(double) * (size_t)nthreads * C);
  kbo_parallel(nthreads, jt_normal_job, &c);
  memset(A->Hcc, 0, sizeof(double) * C * C);
  memset(A->gc, 0, sizeof(double) * C);
  for (int t = 0; t < nthreads; ++t) {
    for (int q = 0; q < C * C; ++q) A->Hcc[q] += c.Hcc_part[(size_t)t * C * C + q];
    for (int q = 0; q < C; ++q) A->gc[q] += c.gc_part[(size_t)t * C + q];
  }
  A->cost = jt->cost;
  free(c.Hcc_part);
  free(c.gc_part);
}

void kbo_build_arrow(const kbo_problem* P, const double* st, int nthreads, kbo_arrow* A) {
  kbo_jt* jt = kbo_jt_create(P);
  kbo_jt_build(jt, st, nthreads, NULL);
  kbo_jt_normal_arrow(jt, nthreads, A);
  kbo_jt_destroy(jt);
}

/* ------------------------------------------------------------------ */
/* solve: (J^T J + lambda^2 I) dx = rhs                                */
/* SparseCholeskyLinearSystemSolver.cpp:48-89 + Cholmod(impl).hpp:287-328,387-399:
 * CHOLMOD factors A A^T with A = [J^T | lambda I] (stype 0).  The restatement
 * eliminates the frame poses first (what AMD yields on the arrow) and does a
 * dense Cholesky of the camera-block Schur complement.                         */
/* ------------------------------------------------------------------ */

static int chol_inplace(double* A, int n) {
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0.0)) return 0;
    d = sqrt(d);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / d;
    }
    for (int k = j + 1; k < n; ++k) A[j * n + k] = 0.0;
  }
  return 1;
}

static void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
    b[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
    b[i] = s / L[i * n + i];
  }
}

typedef struct {
  const kbo_arrow* A;
  double lam2;
  int f0, f1;
  double* L;   /* [F][36] */
  double* Y;   /* [F][6*C] */
  double* z;   /* [F][6] */
  double* S_part;
  double* b_part;
  int* ok_part;
  const double* dxc;
  double* dx;
} schur_ctx;

static void schur_frame(const kbo_arrow* A, double lam2, int f, double* L, double* Y, double* z, int* ok) {
  const int C = A->C;
  memcpy(L, A->Hff + 36 * (size_t)f, 36 * sizeof(double));
  for (int d = 0; d < 6; ++d) L[d * 6 + d] += lam2;
  if (!chol_inplace(L, 6)) { *ok = 0; return; }
  const double* Hfc = A->Hfc + (size_t)6 * C * f;
  for (int c = 0; c < C; ++c)
    for (int r = 0; r < 6; ++r) {
      double s = Hfc[r * C + c];
      for (int k = 0; k < r; ++k) s -= L[r * 6 + k] * Y[k * C + c];
      Y[r * C + c] = s / L[r * 6 + r];
    }
  const double* g = A->gf + 6 * (size_t)f;
  for (int r = 0; r < 6; ++r) {
    double s = g[r];
    for (int k = 0; k < r; ++k) s -= L[r * 6 + k] * z[k];
    z[r] = s / L[r * 6 + r];
  }
}

static void schur_job(void* a, int tid, int nt) {
  schur_ctx* c = (schur_ctx*)a;
  const kbo_arrow* A = c->A;
  const int C = A->C;
  int F = c->f1 - c->f0;
  int f0 = c->f0 + (int)((long long)F * tid / nt), f1 = c->f0 + (int)((long long)F * (tid + 1) / nt);
  double* S = c->S_part + (size_t)tid * C * C;
  double* b = c->b_part + (size_t)tid * C;
  memset(S, 0, sizeof(double) * C * C);
  memset(b, 0, sizeof(double) * C);
  c->ok_part[tid] = 1;
  for (int f = f0; f < f1; ++f) {
    double* L = c->L + 36 * (size_t)f;
    double* Y = c->Y + (size_t)6 * C * f;
    double* z = c->z + 6 * (size_t)f;
    schur_frame(A, c->lam2, f, L, Y, z, &c->ok_part[tid]);
    if (!c->ok_part[tid]) return;
    for (int r = 0; r < 6; ++r) {
      const double* y = Y + r * C;
      for (int p = 0; p < C; ++p) {
        b[p] += y[p] * z[r];
        for (int q = 0; q < C; ++q) S[p * C + q] += y[p] * y[q];
      }
    }
  }
}

static void backsub_job(void* a, int tid, int nt) {
  schur_ctx* c = (schur_ctx*)a;
  const kbo_arrow* A = c->A;
  const int C = A->C;
  int f0 = (int)((long long)A->F * tid / nt), f1 = (int)((long long)A->F * (tid + 1) / nt);
  for (int f = f0; f < f1; ++f) {
    const double* L = c->L + 36 * (size_t)f;
    const double* Y = c->Y + (size_t)6 * C * f;
    const double* z = c->z + 6 * (size_t)f;
    double w[6];
    for (int r = 0; r < 6; ++r) {
      double s = z[r];
      for (int q = 0; q < C; ++q) s -= Y[r * C + q] * c->dxc[q];
      w[r] = s;
    }
    for (int r = 5; r >= 0; --r) {
      double s = w[r];
      for (int k = r + 1; k < 6; ++k) s -= L[k * 6 + r] * w[k];
      w[r] = s / L[r * 6 + r];
    }
    for (int r = 0; r < 6; ++r) c->dx[C + 6 * f + r] = w[r];
  }
}

void kbo_arrow_schur_partial(const kbo_arrow* A, double conditioner, int f0, int f1, double* S_part, double* b_part, int* ok) {
  const int C = A->C;
  schur_ctx c;
  memset(&c, 0, sizeof(c));
  c.A = A;
  c.lam2 = conditioner * conditioner;
  c.f0 = f0;
  c.f1 = f1;
  c.L = (double*)malloc(sizeof(double) * 36 * (size_t)A->F);
  c.Y = (double*)malloc(sizeof(double) * 6 * (size_t)C * A->F);
  c.z = (double*)malloc(sizeof(double) * 6 * (size_t)A->F);
  c.S_part = S_part;
  c.b_part = b_part;
  int okp = 1;
  c.ok_part = &okp;
  schur_job(&c, 0, 1);
  *ok = okp;
  free(c.L);
  free(c.Y);
  free(c.z);
}

/* ------------------------------------------------------------------ */
/* marginal SVD solve (aslam_incremental_calibration LinearSolver)     */
/* ------------------------------------------------------------------ */

/* Symmetric eigen-decomposition by cyclic Jacobi with the round-robin ("circle") parallel ordering the GPU kernel
 * uses: m = n rounded up to even, m - 1 rounds per sweep, round r pairs (r, m-1) and ((r+k) mod (m-1),
 * (r-k) mod (m-1)), k = 1 .. m/2-1; an index >= n is a bye.  Per round all rotations are computed first, then
 * every 2x2 block (pair k, pair l) is rotated as rows-then-columns (the GPU's per-block formula).  Stops after a
 * sweep without rotations.  Out: w[n] sorted by |w| descending, V[n*n] row-major with eigenvector j in column j.
 * Replaces Eigen::JacobiSVD of the symmetric Omega (linalg.cpp:412-424): for a symmetric matrix the singular
 * values are |w| and U = V up to the signs of negative eigenvalues. */
static void jacobi_pair(int m, int r, int k, int* p, int* q) {
  int a, b;
  if (k == 0) {
    a = r;
    b = m - 1;
  } else {
    a = (r + k) % (m - 1);
    b = (r - k + (m - 1)) % (m - 1);
  }
  *p = a < b ? a : b;
  *q = a < b ? b : a;
}

int kbo_sym_eig(int n, const double* Ain, double* w, double* V) {
  const int m = n + (n & 1), h = m / 2;
  double* A = (double*)malloc(sizeof(double) * (size_t)n * n);
  double* Vw = (double*)malloc(sizeof(double) * (size_t)n * n);
  double* cs = (double*)malloc(sizeof(double) * 2 * h);
  int* pp = (int*)malloc(sizeof(int) * 2 * h);
  memcpy(A, Ain, sizeof(double) * (size_t)n * n);
  for (int i = 0; i < n * n; ++i) Vw[i] = 0.0;
  for (int i = 0; i < n; ++i) Vw[i * n + i] = 1.0;
  int sweeps = 0;
  for (; sweeps < KBO_JACOBI_MAX_SWEEPS; ++sweeps) {
    int nrot = 0;
    for (int r = 0; r < m - 1; ++r) {
      for (int k = 0; k < h; ++k) {
        int p, q;
        jacobi_pair(m, r, k, &p, &q);
        pp[2 * k] = p;
        pp[2 * k + 1] = q;
        double c = 1.0, s = 0.0;
        if (q < n) {
          const double apq = A[p * n + q], app = A[p * n + p], aqq = A[q * n + q];
          if (apq != 0.0 && fabs(apq) > KBO_JACOBI_TOL * sqrt(fabs(app * aqq))) {
            const double th = (aqq - app) / (2.0 * apq);
            const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
            c = 1.0 / sqrt(t * t + 1.0);
            s = t * c;
            ++nrot;
          }
        }
        cs[2 * k] = c;
        cs[2 * k + 1] = s;
      }
      /* 2x2 blocks (k, l), l >= k: rows by rotation k, columns by rotation l; mirrored below the diagonal */
      for (int k = 0; k < h; ++k) {
        const int p = pp[2 * k], q = pp[2 * k + 1];
        const double ck = cs[2 * k], sk = cs[2 * k + 1];
        for (int l = k; l < h; ++l) {
          const int r2 = pp[2 * l], s2 = pp[2 * l + 1];
          const double cl = cs[2 * l], sl = cs[2 * l + 1];
          if (l == k) {
            if (q >= n || sk == 0.0) continue;
            const double apq = A[p * n + q], t = sk / ck;
            A[p * n + p] -= t * apq;
            A[q * n + q] += t * apq;
            A[p * n + q] = A[q * n + p] = 0.0;
            continue;
          }
          const int rv = r2 < n, sv = s2 < n, qv = q < n;
          const double apr = rv ? A[p * n + r2] : 0.0, aps = sv ? A[p * n + s2] : 0.0;
          const double aqr = (qv && rv) ? A[q * n + r2] : 0.0, aqs = (qv && sv) ? A[q * n + s2] : 0.0;
          const double tpr = ck * apr - sk * aqr, tps = ck * aps - sk * aqs;
          const double tqr = sk * apr + ck * aqr, tqs = sk * aps + ck * aqs;
          const double npr = cl * tpr - sl * tps, nps = sl * tpr + cl * tps;
          const double nqr = cl * tqr - sl * tqs, nqs = sl * tqr + cl * tqs;
          if (rv) A[p * n + r2] = A[r2 * n + p] = npr;
          if (sv) A[p * n + s2] = A[s2 * n + p] = nps;
          if (qv && rv) A[q * n + r2] = A[r2 * n + q] = nqr;
          if (qv && sv) A[q * n + s2] = A[s2 * n + q] = nqs;
        }
      }
      for (int k = 0; k < h; ++k) { /* V <- V J: columns p, q */
        const int p = pp[2 * k], q = pp[2 * k + 1];
        const double c = cs[2 * k], s = cs[2 * k + 1];
        if (q >= n || s == 0.0) continue;
        for (int i = 0; i < n; ++i) {
          const double vp = Vw[i * n + p], vq = Vw[i * n + q];
          Vw[i * n + p] = c * vp - s * vq;
          Vw[i * n + q] = s * vp + c * vq;
        }
      }
    }
    if (nrot == 0) break;
  }
  /* sort by |w| descending (ties: lower index first) */
  for (int i = 0; i < n; ++i) {
    const double ai = fabs(A[i * n + i]);
    int pos = 0;
    for (int j = 0; j < n; ++j) {
      const double aj = fabs(A[j * n + j]);
      if (aj > ai || (aj == ai && j < i)) ++pos;
    }
    w[pos] = A[i * n + i];
    for (int r = 0; r < n; ++r) V[r * n + pos] = Vw[r * n + i];
  }
  free(A);
  free(Vw);
  free(cs);
  free(pp);
  return sweeps;
}

/* LinearSolver::solve's camera-block part (LinearSolver.cpp:299-466) on the Schur-reduced system: column scaling
 * G_j = 1/||A_r col j|| = 1/sqrt(Hcc_jj), 0 below sqrt(nrows * epsNorm) (linalg.cpp:128-152); Omega = G S G,
 * b_r = G b (the SPQR route forms the same Schur complement, reduceLeftHandSide / reduceRightHandSide,
 * linalg.cpp:284-410); SVD (analyzeSVD :412-424); tolerance rankTol = sv_0 * epsSVD * n (:256-261) unless svdTol
 * != -1; rank by estimateNumericalRank (:243-254); svGap (:273-282); x_r = G V_r diag(1/sv) U_r^T b_r (solveSVD
 * :426-443).  scaling = 0 gives analyzeMarginal's unscaled SVD (LinearSolver.cpp:468-528). */
void kbo_marginal_solve(int C, const double* S, const double* b, const double* hdiag, const kbo_marg_opts* o,
                        double* x, kbo_marg_info* info) {
  double* G = (double*)malloc(sizeof(double) * C);
  double* Om = (double*)malloc(sizeof(double) * (size_t)C * C);
  double* w = (double*)malloc(sizeof(double) * C);
  double* V = info->V ? info->V : (double*)malloc(sizeof(double) * (size_t)C * C);
  const double normTol = sqrt(o->n_rows * o->eps_norm);
  for (int j = 0; j < C; ++j) {
    if (!o->column_scaling) {
      G[j] = 1.0;
      continue;
    }
    const double nrm = sqrt(hdiag[j]);
    G[j] = (nrm < normTol) ? 0.0 : 1.0 / nrm;
  }
  for (int i = 0; i < C; ++i)
    for (int j = 0; j < C; ++j) Om[i * C + j] = G[i] * S[i * C + j] * G[j];
  info->sweeps = kbo_sym_eig(C, Om, w, V);
  for (int i = 0; i < C; ++i) info->sv[i] = fabs(w[i]);
  info->tol = (o->svd_tol != -1.0) ? o->svd_tol : info->sv[0] * o->eps_svd * C;
  int rank = C;
  for (int i = C - 1; i > 0; --i) {
    if (info->sv[i] > info->tol) break;
    --rank;
  }
  info->rank = rank;
  info->gap = rank < C ? info->sv[rank - 1] / info->sv[rank] : INFINITY;
  double l2 = 0.0;
  for (int i = 0; i < rank; ++i) l2 += log(info->sv[i]);
  info->log2sum = l2 / log(2.0);
  if (x) {
    for (int i = 0; i < C; ++i) x[i] = 0.0;
    for (int j = 0; j < rank; ++j) {
      double vb = 0.0;
      for (int i = 0; i < C; ++i) vb += V[i * C + j] * G[i] * b[i];
      const double a = vb / w[j];
      for (int i = 0; i < C; ++i) x[i] += V[i * C + j] * a;
    }
    for (int i = 0; i < C; ++i) x[i] *= G[i];
  }
  if (!info->V) free(V);
  free(G);
  free(Om);
  free(w);
}

int kbo_arrow_solve(const kbo_arrow* A, double conditioner, int nthreads, double* dx) {
  return kbo_arrow_solve_ex(A, conditioner, nthreads, dx, NULL, NULL);
}

/* marg != NULL: the calibration::LinearSolver (QR + marginal SVD) in place of CHOLMOD: the conditioner is
 * ignored (LinearSolver does not use it), the camera block is solved by kbo_marginal_solve and the frame blocks
 * by back-substitution (solveQR, linalg.cpp:445-501: least squares of A_l x_l = b - A_r x_r). */
int kbo_arrow_solve_ex(const kbo_arrow* A, double conditioner, int nthreads, double* dx, const kbo_marg_opts* marg,
                       kbo_marg_info* info) {
  const int C = A->C, F = A->F;
  if (marg) conditioner = 0.0;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > F) nthreads = F > 0 ? F : 1;
  if (nthreads > 256) nthreads = 256;
  schur_ctx c;
  memset(&c, 0, sizeof(c));
  c.A = A;
  c.lam2 = conditioner * conditioner;
  c.f0 = 0;
  c.f1 = F;
  c.L = (double*)malloc(sizeof(double) * 36 * (size_t)F);
  c.Y = (double*)malloc(sizeof(double) * 6 * (size_t)C * F);
  c.z = (double*)malloc(sizeof(double) * 6 * (size_t)F);
  c.S_part = (double*)malloc(sizeof(double) * (size_t)nthreads * C * C);
  c.b_part = (double*)malloc(sizeof(double) * (size_t)nthreads * C);
  c.ok_part = (int*)malloc(sizeof(int) * nthreads);
  kbo_parallel(nthreads, schur_job, &c);
  int ok = 1;
  for (int t = 0; t < nthreads; ++t) ok &= c.ok_part[t];
  double* S = (double*)malloc(sizeof(double) * C * C);
  double* b = (double*)malloc(sizeof(double) * C);
  if (ok) {
    for (int q = 0; q < C * C; ++q) {
      double s = 0.0;
      for (int t = 0; t < nthreads; ++t) s += c.S_part[(size_t)t * C * C + q];
      S[q] = A->Hcc[q] - s;
    }
    for (int d = 0; d < C; ++d) S[d * C + d] += c.lam2;
    for (int q = 0; q < C; ++q) {
      double s = 0.0;
      for (int t = 0; t < nthreads; ++t) s += c.b_part[(size_t)t * C + q];
      b[q] = A->gc[q] - s;
    }
    if (marg) {
      double* hd = (double*)malloc(sizeof(double) * C);
      double* xr = (double*)malloc(sizeof(double) * C);
      for (int q = 0; q < C; ++q) hd[q] = A->Hcc[q * C + q];
      kbo_marginal_solve(C, S, b, hd, marg, xr, info);
      memcpy(b, xr, sizeof(double) * C);
      free(hd);
      free(xr);
    } else {
      ok = chol_inplace(S, C);
    }
  }
  if (ok) {
    if (!marg) chol_solve(S, C, b);
    for (int q = 0; q < C; ++q) dx[q] = b[q];
    c.dxc = b;
    c.dx = dx;
    kbo_parallel(nthreads, backsub_job, &c);
  }
  free(S);
  free(b);
  free(c.L);
  free(c.Y);
  free(c.z);
  free(c.S_part);
  free(c.b_part);
  free(c.ok_part);
  return ok;
}

int kbo_dense_solve(const kbo_arrow* A, double conditioner, double* dx) {
  const int C = A->C, F = A->F, n = C + 6 * F;
  double* H = (double*)calloc((size_t)n * n, sizeof(double));
  for (int p = 0; p < C; ++p)
    for (int q = 0; q < C; ++q) H[(size_t)p * n + q] = A->Hcc[p * C + q];
  for (int f = 0; f < F; ++f) {
    int o = C + 6 * f;
    for (int p = 0; p < 6; ++p) {
      for (int q = 0; q < 6; ++q) H[(size_t)(o + p) * n + o + q] = A->Hff[36 * (size_t)f + p * 6 + q];
      for (int q = 0; q < C; ++q) {
        double v = A->Hfc[(size_t)6 * C * f + p * C + q];
        H[(size_t)(o + p) * n + q] = v;
        H[(size_t)q * n + o + p] = v;
      }
    }
  }
  for (int d = 0; d < n; ++d) H[(size_t)d * n + d] += conditioner * conditioner;
  int ok = chol_inplace(H, n);
  if (ok) {
    for (int q = 0; q < C; ++q) dx[q] = A->gc[q];
    for (int q = 0; q < 6 * F; ++q) dx[C + q] = A->gf[q];
    chol_solve(H, n, dx);
  }
  free(H);
  return ok;
}

/* ------------------------------------------------------------------ */
/* block-Jacobi PCG on the arrow system (H + c^2 I) dx = g:              */
/* sparse_block_matrix LinearSolverPCG::solve                            */
/* (sparse_block_matrix/include/sparse_block_matrix/implementation/     */
/*  linear_solver_pcg.hpp:58-130; defaults linear_solver_pcg.h:39-47).   */
/* Preconditioner blocks are the design-variable blocks of the diagonal  */
/* (_J = diag block inverse, :72-75): the camera DV blocks given by the  */
/* caller, then per frame the rotation DV (3) and translation DV (3).    */
/* ------------------------------------------------------------------ */

/* y = (H + lam2 I) x on the arrow (the reference's mult(): diagonal blocks + upper blocks and their
 * transposes, linear_solver_pcg.hpp:153-171 -- the same product) */
static void arrow_mult(const kbo_arrow* A, double lam2, const double* x, double* y) {
  const int C = A->C, F = A->F;
  for (int p = 0; p < C; ++p) {
    double s = lam2 * x[p];
    for (int q = 0; q < C; ++q) s += A->Hcc[(size_t)p * C + q] * x[q];
    y[p] = s;
  }
  for (int f = 0; f < F; ++f) {
    const double* Hf = A->Hff + 36 * (size_t)f;
    const double* Bf = A->Hfc + (size_t)6 * C * f;
    const double* xf = x + C + 6 * f;
    for (int a = 0; a < 6; ++a) {
      double s = lam2 * xf[a];
      for (int b = 0; b < 6; ++b) s += Hf[a * 6 + b] * xf[b];
      for (int q = 0; q < C; ++q) s += Bf[a * C + q] * x[q];
      y[C + 6 * f + a] = s;
    }
    for (int q = 0; q < C; ++q) {
      double s = 0.0;
      for (int a = 0; a < 6; ++a) s += Bf[a * C + q] * xf[a];
      y[q] += s;
    }
  }
}

/* in-place inverse of an n x n block by Gauss-Jordan with partial pivoting; 0 if singular */
static int block_inverse(double* M, int n) {
  double Aug[6 * 12];
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < 2 * n; ++c) Aug[r * 12 + c] = c < n ? M[r * n + c] : (c - n == r ? 1.0 : 0.0);
  for (int k = 0; k < n; ++k) {
    int piv = k;
    for (int r = k + 1; r < n; ++r)
      if (fabs(Aug[r * 12 + k]) > fabs(Aug[piv * 12 + k])) piv = r;
    if (!(fabs(Aug[piv * 12 + k]) > 0.0)) return 0;
    if (piv != k)
      for (int c = 0; c < 2 * n; ++c) {
        const double t = Aug[k * 12 + c];
        Aug[k * 12 + c] = Aug[piv * 12 + c];
        Aug[piv * 12 + c] = t;
      }
    const double inv = 1.0 / Aug[k * 12 + k];
    for (int c = 0; c < 2 * n; ++c) Aug[k * 12 + c] *= inv;
    for (int r = 0; r < n; ++r) {
      if (r == k) continue;
      const double m = Aug[r * 12 + k];
      if (m != 0.0)
        for (int c = 0; c < 2 * n; ++c) Aug[r * 12 + c] -= m * Aug[k * 12 + c];
    }
  }
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) M[r * n + c] = Aug[r * 12 + n + c];
  return 1;
}

int kbo_arrow_pcg(const kbo_arrow* A, double conditioner, int n_cam_blocks, const int* cam_block_size,
                  const kbo_pcg_opts* o, double* x, kbo_pcg_info* info) {
  const int C = A->C, F = A->F, n = C + 6 * F;
  const double lam2 = conditioner * conditioner;
  const int nb = n_cam_blocks + 2 * F;
  int* bstart = (int*)malloc(sizeof(int) * (nb + 1));
  int* bsize = (int*)malloc(sizeof(int) * nb);
  int c = 0;
  for (int b = 0; b < n_cam_blocks; ++b) {
    bstart[b] = c;
    bsize[b] = cam_block_size[b];
    c += cam_block_size[b];
  }
  for (int b = n_cam_blocks; b < nb; ++b) {
    bstart[b] = c;
    bsize[b] = 3;
    c += 3;
  }
  bstart[nb] = c;
  int ok = (c == n);
  /* _J: inverses of the diagonal DV blocks of H + lam2 I */
  double* Jinv = (double*)malloc(sizeof(double) * 36 * (size_t)nb);
  for (int b = 0; ok && b < nb; ++b) {
    const int s = bstart[b], m = bsize[b];
    double* M = Jinv + 36 * (size_t)b;
    if (m < 1 || m > 6) {
      ok = 0;
      break;
    }
    for (int r = 0; r < m; ++r)
      for (int q = 0; q < m; ++q) {
        double v;
        const int gr = s + r, gq = s + q;
        if (gr < C)
          v = A->Hcc[(size_t)gr * C + gq];
        else {
          const int f = (gr - C) / 6;
          v = A->Hff[36 * (size_t)f + ((gr - C) % 6) * 6 + (gq - C) % 6];
        }
        M[r * m + q] = v + (r == q ? lam2 : 0.0);
      }
    ok = block_inverse(M, m);
  }
  double *r = (double*)malloc(sizeof(double) * n), *d = (double*)malloc(sizeof(double) * n);
  double *q = (double*)malloc(sizeof(double) * n), *s = (double*)malloc(sizeof(double) * n);
  int it = 0;
  double dn = 0.0, d0 = 0.0;
  if (ok) {
    for (int p = 0; p < C; ++p) r[p] = A->gc[p];
    for (int p = 0; p < 6 * F; ++p) r[C + p] = A->gf[p];
    for (int p = 0; p < n; ++p) x[p] = 0.0;
    /* multDiag(_J, r, d) */
    for (int b = 0; b < nb; ++b) {
      const int s0 = bstart[b], m = bsize[b];
      const double* M = Jinv + 36 * (size_t)b;
      for (int a = 0; a < m; ++a) {
        double v = 0.0;
        for (int k = 0; k < m; ++k) v += M[a * m + k] * r[s0 + k];
        d[s0 + a] = v;
      }
    }
    for (int p = 0; p < n; ++p) dn += r[p] * d[p];
    d0 = o->tolerance * dn;
    if (o->absolute_tolerance && o->prev_residual > 0.0 && o->prev_residual > d0) d0 = o->prev_residual;
    const int max_it = o->max_iterations < 0 ? n : o->max_iterations;
    for (it = 0; it < max_it; ++it) {
      if (dn <= d0) break;
      arrow_mult(A, lam2, d, q);
      double dq = 0.0;
      for (int p = 0; p < n; ++p) dq += d[p] * q[p];
      if (!(dq > 0.0) || !isfinite(dq)) { /* breakdown: not positive definite (reported, the reference has no check) */
        ok = 0;
        break;
      }
      const double a = dn / dq;
      for (int p = 0; p < n; ++p) {
        x[p] += a * d[p];
        r[p] -= a * q[p];
      }
      for (int b = 0; b < nb; ++b) {
        const int s0 = bstart[b], m = bsize[b];
        const double* M = Jinv + 36 * (size_t)b;
        for (int e = 0; e < m; ++e) {
          double v = 0.0;
          for (int k = 0; k < m; ++k) v += M[e * m + k] * r[s0 + k];
          s[s0 + e] = v;
        }
      }
      const double dold = dn;
      dn = 0.0;
      for (int p = 0; p < n; ++p) dn += r[p] * s[p];
      const double ba = dn / dold;
      for (int p = 0; p < n; ++p) d[p] = s[p] + ba * d[p];
    }
  }
  if (info) {
    info->iterations = it;
    info->residual = 0.5 * dn; /* _residual (:127) */
    info->d0 = d0;
  }
  free(bstart);
  free(bsize);
  free(Jinv);
  free(r);
  free(d);
  free(q);
  free(s);
  return ok;
}

/* ------------------------------------------------------------------ */
/* state update: Optimizer2::applyStateUpdate (Optimizer2.cpp:290-307)  */
/* ------------------------------------------------------------------ */

double kbo_apply_update(const kbo_problem* P, double* st, const double* dx) {
  int col_intr[64], col_base[64];
  col_layout(P, col_intr, col_base);
  const int C = kbo_cam_cols(P);
  /* intrinsics: additive (PinholeProjection.hpp(impl):509-518; RadialTangentialDistortion.cpp:40-45;
   * OmniProjection.hpp(impl):637-646; ExtendedUnifiedProjection.hpp(impl):661-670) */
  for (int i = 0; i < P->n_cams; ++i) {
    int n = kbo_model_nintr(P->cam_model[i]);
    for (int c = 0; c < n; ++c) st[i * KBO_MAX_INTR + c] += dx[col_intr[i] + c];
  }
  /* poses: RotationQuaternion::updateImplementation (RotationQuaternion.cpp:27-34),
   * EuclideanPoint::updateImplementation (EuclideanPoint.cpp:23-31) */
  for (int j = 0; j < P->n_cams - 1; ++j) {
    double* pose = st + off_base(P) + KBO_POSE * j;
    double q[4];
    kbo_update_quat(pose, dx + col_base[j], q);
    memcpy(pose, q, sizeof(q));
    for (int c = 0; c < 3; ++c) pose[4 + c] += dx[col_base[j] + 3 + c];
  }
  for (int f = 0; f < P->n_frames; ++f) {
    double* pose = st + off_frame(P) + KBO_POSE * f;
    double q[4];
    kbo_update_quat(pose, dx + C + 6 * f, q);
    memcpy(pose, q, sizeof(q));
    for (int c = 0; c < 3; ++c) pose[4 + c] += dx[C + 6 * f + 3 + c];
  }
  double m = 0.0;
  int n = C + 6 * P->n_frames;
  for (int q = 0; q < n; ++q) m = fabs(dx[q]) > m ? fabs(dx[q]) : m;
  return m;
}

/* ------------------------------------------------------------------ */
/* Optimizer2::optimize (Optimizer2.cpp:183-273) with                   */
/* TrustRegionPolicy::solveSystem (TrustRegionPolicy.cpp:39-52),        */
/* LevenbergMarquardtTrustRegionPolicy (LevenbergMarquardtTrustRegionPolicy.cpp:7-113),
 * GaussNewtonTrustRegionPolicy (GaussNewtonTrustRegionPolicy.cpp:18-39). */
/* ------------------------------------------------------------------ */

static void arrow_alloc(kbo_arrow* A, int C, int F) {
  A->C = C;
  A->F = F;
  A->Hff = (double*)calloc(36 * (size_t)F, sizeof(double));
  A->Hfc = (double*)calloc(6 * (size_t)C * F, sizeof(double));
  A->Hcc = (double*)calloc((size_t)C * C, sizeof(double));
  A->gf = (double*)calloc(6 * (size_t)F, sizeof(double));
  A->gc = (double*)calloc(C, sizeof(double));
}
static void arrow_free(kbo_arrow* A) {
  free(A->Hff);
  free(A->Hfc);
  free(A->Hcc);
  free(A->gf);
  free(A->gc);
}

int kbo_optimize(const kbo_problem* P, double* st, const kbo_options* o, kbo_srv* srv, double* trace, int trace_cap) {
  const int C = kbo_cam_cols(P), ncols = kbo_total_cols(P), ns = kbo_state_size(P->n_cams, P->n_frames);
  const int nt = o->nthreads < 1 ? 1 : o->nthreads;
  const int lm = (o->policy == 0);
  kbo_jt* jt = kbo_jt_create(P);
  kbo_arrow A;
  arrow_alloc(&A, C, P->n_frames);
  double* dx = (double*)calloc(ncols, sizeof(double));
  double* rhs = (double*)calloc(ncols, sizeof(double));
  double* backup = (double*)malloc(sizeof(double) * ns);
  memset(srv, 0, sizeof(*srv));

  double J = kbo_eval_cost(P, st, nt);
  double p_J = J;
  srv->J_start = p_J;
  double deltaX = o->eps_x + 1.0, deltaJ = o->eps_j + 1.0;
  int prevFailed = 0, linFail = 0, ntrace = 0;
  /* policy state: optimizationStarting (TrustRegionPolicy.cpp:30-37; LM :38-46) */
  double pol_J = J, pol_pJ = J, last_succ = J;
  int first = 1;
  double lambda = o->lambda0, gamma = 3.0, beta = 2.0, mu = 2.0;
  const int pexp = 3;

  while (srv->iterations < o->max_iterations && srv->failed_iterations < o->max_iterations &&
         ((deltaX > o->eps_x && fabs(deltaJ) > o->eps_j) || linFail)) {
    if (prevFailed) {
      pol_J = J;
    } else {
      pol_pJ = last_succ;
      last_succ = J;
      pol_J = J;
    }
    int success;
    if (lm) {
      if (first) {
        kbo_jt_build(jt, st, nt, rhs);
        kbo_jt_normal_arrow(jt, nt, &A);
      } else {
        double d2 = 0.0;
        for (int q = 0; q < ncols; ++q) d2 += dx[q] * (lambda * dx[q] + rhs[q]);
        double rho = (pol_pJ - pol_J) / d2;
        if (prevFailed) {
          mu *= 2;
          lambda *= mu;
        } else if (rho <= 0) {
          mu *= 10;
          lambda *= mu;
        } else {
          kbo_jt_build(jt, st, nt, rhs);
          kbo_jt_normal_arrow(jt, nt, &A);
          if (lambda > 1e-16) {
            double u1 = 1 / gamma;
            double u2 = 1 - (beta - 1) * pow((2 * rho - 1), pexp);
            if (u1 > u2)
              lambda *= u1;
            else
              lambda *= u2;
            mu = beta;
          } else {
            lambda = 1e-15;
          }
        }
      }
      double* tmp = (double*)malloc(sizeof(double) * ncols);
      success = kbo_arrow_solve_ex(&A, lambda, nt, tmp, o->marg, o->solve_info);
      if (success) memcpy(dx, tmp, sizeof(double) * ncols);
      free(tmp);
    } else {
      kbo_jt_build(jt, st, nt, rhs);
      kbo_jt_normal_arrow(jt, nt, &A);
      success = kbo_arrow_solve_ex(&A, 0.0, nt, dx, o->marg, o->solve_info);
    }
    first = 0;
    int accepted = 0;
    if (!success) {
      prevFailed = 1;
      linFail = 1;
      srv->failed_iterations++;
    } else {
      memcpy(backup, st, sizeof(double) * ns);
      deltaX = kbo_apply_update(P, st, dx);
      J = kbo_eval_cost(P, st, nt);
      deltaJ = p_J - J;
      if (lm) {
        if (deltaJ < 0.0) {
          memcpy(st, backup, sizeof(double) * ns); /* revertLastStateUpdate (Optimizer2.cpp:313-318) */
          srv->failed_iterations++;
          prevFailed = 1;
        } else {
          p_J = J;
          prevFailed = 0;
          accepted = 1;
        }
      } else {
        p_J = J;
        accepted = 1;
      }
      srv->iterations++;
    }
    if (trace && ntrace < trace_cap) {
      trace[4 * ntrace + 0] = success ? J : NAN;
      trace[4 * ntrace + 1] = lm ? lambda : 0.0;
      trace[4 * ntrace + 2] = deltaX;
      trace[4 * ntrace + 3] = accepted;
      ntrace++;
    }
  }
  if (o->marg && o->analyze_info) {
    /* LinearSolver::analyzeMarginal (LinearSolver.cpp:468-528): unscaled Omega of the last built system; the
     * rank, tolerance and gap stay those of the last solve when there was one (_svdRank != -1) */
    kbo_marg_opts un = *o->marg;
    un.column_scaling = 0;
    double* S = (double*)malloc(sizeof(double) * C * C);
    double* b = (double*)malloc(sizeof(double) * C);
    int okp = 1;
    kbo_arrow_schur_partial(&A, 0.0, 0, A.F, S, b, &okp);
    for (int q = 0; q < C * C; ++q) S[q] = A.Hcc[q] - S[q];
    kbo_marginal_solve(C, S, b, NULL, &un, NULL, o->analyze_info);
    if (o->solve_info && srv->iterations + srv->failed_iterations > 0) {
      kbo_marg_info* ai = o->analyze_info;
      ai->rank = o->solve_info->rank;
      ai->tol = o->solve_info->tol;
      ai->gap = o->solve_info->gap;
      double l2 = 0.0;
      for (int i = 0; i < ai->rank; ++i) l2 += log(ai->sv[i]);
      ai->log2sum = l2 / log(2.0);
    }
    free(S);
    free(b);
  }
  srv->J_final = p_J;
  srv->dx_final = deltaX;
  srv->dj_final = deltaJ;
  srv->linear_solver_failure = linFail;
  arrow_free(&A);
  kbo_jt_destroy(jt);
  free(dx);
  free(rhs);
  free(backup);
  return ntrace;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

double kbo_time_gn(const kbo_problem* P, double* st, int n_iter, int nthreads) {
  const int C = kbo_cam_cols(P), ncols = kbo_total_cols(P);
  kbo_jt* jt = kbo_jt_create(P);
  kbo_arrow A;
  arrow_alloc(&A, C, P->n_frames);
  double* dx = (double*)calloc(ncols, sizeof(double));
  double* rhs = (double*)calloc(ncols, sizeof(double));
  double t0 = now_s();
  for (int it = 0; it < n_iter; ++it) {
    kbo_jt_build(jt, st, nthreads, rhs);
    kbo_jt_normal_arrow(jt, nthreads, &A);
    if (kbo_arrow_solve(&A, 0.0, nthreads, dx)) kbo_apply_update(P, st, dx);
    (void)kbo_eval_cost(P, st, nthreads);
  }
  double t = now_s() - t0;
  arrow_free(&A);
  kbo_jt_destroy(jt);
  free(dx);
  free(rhs);
  return t;
}
