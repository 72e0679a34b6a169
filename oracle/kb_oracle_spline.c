/*
 * kb_oracle_spline.c -- CPU restatement of the continuous-time (B-spline pose) calibration path of
 * configs[4] ("2-cam + IMU continuous-time B-spline (aslam_splines) calibration").
 *
 * TEST INFRASTRUCTURE ONLY (see kb_oracle.h): the checker for the device spline path and the CPU baseline
 * of bench.py --config 5.  Nothing in kalibr_amd/ links this code.
 *
 * What is restated (paths relative to /root/reference):
 *   B-spline basis      aslam_nonparametric_estimation/bsplines/src/BSpline.cpp:58-152 (M(k,i) recursion,
 *                       d_0 / d_1), :198-221 (segment / coefficient counts), :237-318 (computeTIndex,
 *                       computeUAndTIndex, computeU, dmul), :351-387 (evalDAndJacobian: v = C_local B^T u)
 *   pose curve          bsplines/src/BSplinePose.cpp:21-41 (transformationAndJacobian, J = JT JS),
 *                       :207-219 (angularVelocityBodyFrame), :175-180 (linearAccelerationBodyFrame),
 *                       :394-412 (curveValueToTransformationAndJacobian: JT = [I, -[p]x S; 0, S])
 *   rotation vector     Schweizer-Messer/sm_kinematics/src/RotationVector.cpp:10-52
 *                       (parametersToRotationMatrix), :54-78 (rotationMatrixToParameters), :80-103 (S)
 *   spline DVs          aslam_splines/src/BSplinePoseDesignVariable.cpp:9-19 (one DesignVariableMappedVector<6>
 *                       per coefficient column, additive update), BSplineExpressions.cpp:23-45
 *                       (transformation node Jacobians J.block<6,6>(0, 6i) per active coefficient)
 *   chain               as kb_oracle.c term_blocks (TransformationExpressionNode.cpp:54-101) with the camera
 *                       chain T_ci_w = B_{i-1} ... B_0 * T_c0_b * T_wb(t)^-1
 *
 * The IMU error terms are NOT in the reference (Kalibr2 has no IMU term): they are
 * defined here and their parity is "unpinned" beyond the finite-difference checks of
 * tests/test_spline_oracle.py.  d(S(theta) v)/dtheta is our own forward-mode derivation, not the reference's
 * RotationVector::angularVelocityAndJacobian expansion.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "kb_oracle.h"

/* ------------------------------------------------------------------ small linear algebra */
static void sp_cross(const double v[3], double M[9]) {
  M[0] = 0; M[1] = -v[2]; M[2] = v[1];
  M[3] = v[2]; M[4] = 0; M[5] = -v[0];
  M[6] = -v[1]; M[7] = v[0]; M[8] = 0;
}
static void sp_mm(const double* A, const double* B, double* Cm, int m, int k, int n) {
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += A[i * k + l] * B[l * n + j];
      Cm[i * n + j] = s;
    }
}
static void sp_pose_T(const double* pose, double T[16]) {
  double R[9];
  kbo_quat2r(pose, R);
  memset(T, 0, 16 * sizeof(double));
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T[r * 4 + c] = R[r * 3 + c];
    T[r * 4 + 3] = pose[4 + r];
  }
  T[15] = 1.0;
}
static void sp_inv_T(const double T[16], double Ti[16]) {
  memset(Ti, 0, 16 * sizeof(double));
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) Ti[r * 4 + c] = T[c * 4 + r];
  for (int r = 0; r < 3; ++r) Ti[r * 4 + 3] = -(Ti[r * 4 + 0] * T[3] + Ti[r * 4 + 1] * T[7] + Ti[r * 4 + 2] * T[11]);
  Ti[15] = 1.0;
}
/* sm::kinematics::boxTimes (transformations.cpp:132-141): [C, -[t]x C; 0, C] */
static void sp_box_times(const double T[16], double A[36]) {
  double Cm[9], t[3], tx[9], txC[9];
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) Cm[r * 3 + c] = T[r * 4 + c];
    t[r] = T[r * 4 + 3];
  }
  sp_cross(t, tx);
  sp_mm(tx, Cm, txC, 3, 3, 3);
  memset(A, 0, 36 * sizeof(double));
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      A[r * 6 + c] = Cm[r * 3 + c];
      A[r * 6 + 3 + c] = -txC[r * 3 + c];
      A[(3 + r) * 6 + 3 + c] = Cm[r * 3 + c];
    }
}
/* sm::kinematics::boxMinus (transformations.cpp:45-53) for a homogeneous point p: [p3 I, [p]x] */
static void sp_box_minus(const double p[4], double B[24]) {
  memset(B, 0, 24 * sizeof(double));
  for (int r = 0; r < 3; ++r) B[r * 6 + r] = p[3];
  double px[9];
  sp_cross(p, px);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) B[r * 6 + 3 + c] = px[r * 3 + c];
}
/* TransformationBasic DV map (TransformationBasic.cpp:49-66): chain (m x 6) -> [rotation DV | translation DV] */
static void sp_basic_dv(const double* ch, int m, const double t[3], double* J) {
  double tx[9];
  sp_cross(t, tx);
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < 3; ++c) {
      double s = 0.0;
      for (int l = 0; l < 3; ++l) s += ch[r * 6 + l] * (-tx[l * 3 + c]);
      J[r * 6 + c] = s + ch[r * 6 + 3 + c];
      J[r * 6 + 3 + c] = ch[r * 6 + c];
    }
}

/* ------------------------------------------------------------------ B-spline (BSpline.cpp) */
/* d_0 / d_1 (BSpline.cpp:130-152) */
static double bs_d0(const double* kn, int k, int i, int j) {
  const double den = kn[j + k - 1] - kn[j];
  return den <= 0.0 ? 0.0 : (kn[i] - kn[j]) / den;
}
static double bs_d1(const double* kn, int k, int i, int j) {
  const double den = kn[j + k - 1] - kn[j];
  return den <= 0.0 ? 0.0 : (kn[i + 1] - kn[i]) / den;
}
/* M(k, i) (BSpline.cpp:70-128): M_k = [M_{k-1}; 0] A + [0; M_{k-1}] B, out k x k row-major */
static void bs_M(const double* kn, int k, int i, double* out) {
  if (k == 1) {
    out[0] = 1.0;
    return;
  }
  double Mp[64];
  bs_M(kn, k - 1, i, Mp);
  double M1[64], M2[64], A[64], B[64];
  memset(M1, 0, sizeof(M1));
  memset(M2, 0, sizeof(M2));
  memset(A, 0, sizeof(A));
  memset(B, 0, sizeof(B));
  const int n = k - 1; /* M_{k-1} is n x n; M1, M2 are k x n */
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) {
      M1[r * n + c] = Mp[r * n + c];
      M2[(r + 1) * n + c] = Mp[r * n + c];
    }
  for (int idx = 0; idx < n; ++idx) { /* A, B are (k-1) x k */
    const int j = i - k + 2 + idx;
    const double d0 = bs_d0(kn, k, i, j), d1 = bs_d1(kn, k, i, j);
    A[idx * k + idx] = 1.0 - d0;
    A[idx * k + idx + 1] = d0;
    B[idx * k + idx] = -d1;
    B[idx * k + idx + 1] = d1;
  }
  double P1[64], P2[64];
  sp_mm(M1, A, P1, k, n, k);
  sp_mm(M2, B, P2, k, n, k);
  for (int q = 0; q < k * k; ++q) out[q] = P1[q] + P2[q];
}

int kbo_bspline_num_coeffs(int order, int n_knots) {
  const int nseg = n_knots - 2 * order + 1; /* numValidTimeSegments (BSpline.cpp:198-202) */
  return nseg > 0 ? nseg + order - 1 : 0;   /* numCoefficientsRequired (:214-217) */
}

void kbo_bspline_basis(int order, const double* knots, int segment, double* M) {
  bs_M(knots, order, segment + order - 1, M); /* initializeBasisMatrices (:58-67) */
}

int kbo_bspline_weights(int order, const double* knots, int n_knots, double t, int deriv, double* w) {
  /* computeTIndex (:237-264): t in [t_min, t_max], t == t_max -> last segment */
  const double tmin = knots[order - 1], tmax = knots[n_knots - order];
  if (t < tmin || t > tmax + 1e-10) return -1;
  if (fabs(tmax - t) < 1e-10) t = tmax;
  int idx;
  if (t == tmax) {
    idx = n_knots - order - 1;
  } else {
    int lo = 0, hi = n_knots; /* upper_bound */
    while (lo < hi) {
      const int mid = (lo + hi) / 2;
      if (knots[mid] <= t) lo = mid + 1; else hi = mid;
    }
    idx = lo - 1;
  }
  const double den = knots[idx + 1] - knots[idx];
  const double u = den <= 0.0 ? 0.0 : (t - knots[idx]) / den; /* computeUAndTIndex (:266-287) */
  /* computeU (:300-318) */
  double uv[8] = {0};
  const double dt = knots[idx + 1] - knots[idx];
  const double mult = dt > 0.0 ? 1.0 / pow(dt, deriv) : 0.0;
  double uu = 1.0;
  for (int i = deriv; i < order; ++i) {
    int dm = 1; /* dmul(i, deriv) */
    for (int q = 0; q < deriv; ++q) dm *= (i - q);
    uv[i] = mult * uu * dm;
    uu *= u;
  }
  const int bidx = idx - order + 1;
  double M[64];
  kbo_bspline_basis(order, knots, bidx, M);
  for (int j = 0; j < order; ++j) { /* Bt_u = M^T u */
    double s = 0.0;
    for (int i = 0; i < order; ++i) s += M[i * order + j] * uv[i];
    w[j] = s;
  }
  return bidx;
}

/* ------------------------------------------------------------------ rotation vector (RotationVector.cpp) */
void kbo_rv_to_C(const double a[3], double Cm[9]) {
  const double ang = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  if (ang < 1e-14) {
    memset(Cm, 0, 9 * sizeof(double));
    Cm[0] = Cm[4] = Cm[8] = 1.0;
    return;
  }
  const double ra = 1.0 / ang, ax = a[0] * ra, ay = a[1] * ra, az = a[2] * ra;
  const double sa = sin(ang), ca = cos(ang);
  const double ax2 = ax * ax, ay2 = ay * ay, az2 = az * az;
  Cm[0] = ax2 + ca * (1.0 - ax2);
  Cm[1] = ax * ay - ca * ax * ay + sa * az;
  Cm[2] = ax * az - ca * ax * az - sa * ay;
  Cm[3] = ax * ay - ca * ax * ay - sa * az;
  Cm[4] = ay2 + ca * (1.0 - ay2);
  Cm[5] = ay * az - ca * ay * az + sa * ax;
  Cm[6] = ax * az - ca * ax * az + sa * ay;
  Cm[7] = ay * az - ca * ay * az - sa * ax;
  Cm[8] = az2 + ca * (1.0 - az2);
}

void kbo_rv_S(const double a[3], double S[9]) {
  const double ang = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  memset(S, 0, 9 * sizeof(double));
  S[0] = S[4] = S[8] = 1.0;
  if (ang < 1e-14) return;
  const double ra = 1.0 / ang;
  const double ax[3] = {a[0] * ra, a[1] * ra, a[2] * ra};
  const double st2 = sin(ang * 0.5), st = sin(ang);
  const double c1 = -2.0 * st2 * st2 * ra, c2 = (ang - st) * ra;
  double X[9], X2[9];
  sp_cross(ax, X);
  sp_mm(X, X, X2, 3, 3, 3);
  for (int q = 0; q < 9; ++q) S[q] += c1 * X[q] + c2 * X2[q];
}

/* D = d(S(a) v)/da (3x3).  S v = v + alpha(|a|) a x v + beta(|a|) a x (a x v) with
 * alpha = (cos f - 1)/f^2, beta = (f - sin f)/f^3 (the same S as kbo_rv_S); differentiated by hand. */
void kbo_rv_dSv(const double a[3], const double v[3], double D[9]) {
  const double f2 = a[0] * a[0] + a[1] * a[1] + a[2] * a[2], f = sqrt(f2);
  double al, be, dal, dbe; /* dal = alpha'(f)/f, dbe = beta'(f)/f */
  if (f < 1e-4) {
    al = -0.5 + f2 / 24.0;
    be = 1.0 / 6.0 - f2 / 120.0;
    dal = 1.0 / 12.0 - f2 / 180.0;
    dbe = -1.0 / 60.0 + f2 / 1260.0;
  } else {
    const double s = sin(f), c = cos(f);
    al = (c - 1.0) / f2;
    be = (f - s) / (f2 * f);
    dal = (-s / f2 - 2.0 * (c - 1.0) / (f2 * f)) / f;
    dbe = ((1.0 - c) / (f2 * f) - 3.0 * (f - s) / (f2 * f2)) / f;
  }
  double axv[3] = {a[1] * v[2] - a[2] * v[1], a[2] * v[0] - a[0] * v[2], a[0] * v[1] - a[1] * v[0]};
  const double av = a[0] * v[0] + a[1] * v[1] + a[2] * v[2];
  double aaxv[3]; /* a x (a x v) = a (a.v) - v f^2 */
  for (int r = 0; r < 3; ++r) aaxv[r] = a[r] * av - v[r] * f2;
  double vx[9];
  sp_cross(v, vx);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      /* d(a x v)/da = -[v]x ; d(a x (a x v))/da = (a.v) I + a v^T - 2 v a^T */
      const double daxv = -vx[r * 3 + c];
      const double daaxv = (r == c ? av : 0.0) + a[r] * v[c] - 2.0 * v[r] * a[c];
      D[r * 3 + c] = al * daxv + axv[r] * dal * a[c] + be * daaxv + aaxv[r] * dbe * a[c];
    }
}

/* ------------------------------------------------------------------ problem layout */
static int sp_ncoef(const kbo_sp_problem* P) { return kbo_bspline_num_coeffs(P->order, P->n_knots); }
static int sp_off_base(const kbo_sp_problem* P) { return P->n_cams * KBO_MAX_INTR; }
static int sp_off_cb(const kbo_sp_problem* P) { return sp_off_base(P) + KBO_POSE * (P->n_cams - 1); }
static int sp_off_imu(const kbo_sp_problem* P) { return sp_off_cb(P) + KBO_POSE; }
static int sp_off_coef(const kbo_sp_problem* P) { return sp_off_imu(P) + 9; }

int kbo_sp_state_size(const kbo_sp_problem* P) { return sp_off_coef(P) + 6 * sp_ncoef(P); }
int kbo_sp_num_coeffs(const kbo_sp_problem* P) { return sp_ncoef(P); }
int kbo_sp_cam_cols(const kbo_sp_problem* P) {
  int c = 0;
  for (int i = 0; i < P->n_cams; ++i) c += kbo_model_nintr(P->cam_model[i]);
  return c + 6 * (P->n_cams - 1) + 6 + 9;
}
int kbo_sp_total_cols(const kbo_sp_problem* P) { return kbo_sp_cam_cols(P) + 6 * sp_ncoef(P); }

typedef struct {
  int intr[16], base[16], cb, bg, ba, g, C;
} sp_cols;
static void sp_layout(const kbo_sp_problem* P, sp_cols* L) {
  int c = 0;
  for (int i = 0; i < P->n_cams; ++i) { L->intr[i] = c; c += kbo_model_nintr(P->cam_model[i]); }
  for (int j = 0; j < P->n_cams - 1; ++j) { L->base[j] = c; c += 6; }
  L->cb = c; c += 6;
  L->bg = c; c += 3;
  L->ba = c; c += 3;
  L->g = c; c += 3;
  L->C = c;
}

/* spline curve value (deriv d) at time t: v[6] = sum_j w_j c_{bidx+j} */
static int sp_eval(const kbo_sp_problem* P, const double* st, double t, int deriv, double v[6], double* w) {
  double wl[8];
  if (!w) w = wl;
  const int b = kbo_bspline_weights(P->order, P->knots, P->n_knots, t, deriv, w);
  if (b < 0) return -1;
  const double* c = st + sp_off_coef(P) + 6 * b;
  for (int r = 0; r < 6; ++r) {
    double s = 0.0;
    for (int j = 0; j < P->order; ++j) s += w[j] * c[6 * j + r];
    v[r] = s;
  }
  return b;
}

/* ------------------------------------------------------------------ reprojection term */
/* e = y - pi_i(T_ci_w P), T_ci_w = B_{i-1} ... B_0 * T_c0_b * T_wb(t_f)^-1.
 * Outputs (optional): Jin [2][KBO_MAX_INTR], JB [i][2x6], Jcb [2x6], Js [2][6*order] (coefficients bidx..),
 * returns chi^2, *bidx. */
static double sp_reproj(const kbo_sp_problem* P, const double* st, int v, int k, double e[2], double* Jin,
                        double (*JB)[12], double* Jcb, double* Js, int* bidx) {
  const int f = P->view_frame[v], i = P->view_cam[v], model = P->cam_model[i];
  const double* intr = st + i * KBO_MAX_INTR;
  double pv[6], w[8];
  const int b = sp_eval(P, st, P->frame_time[f], 0, pv, w);
  if (bidx) *bidx = b;
  double Twb[16], Tbw[16], Tcb[16], T[16], tmp[16], Cwb[9];
  kbo_rv_to_C(pv + 3, Cwb);
  memset(Twb, 0, sizeof(Twb));
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) Twb[r * 4 + c] = Cwb[r * 3 + c];
    Twb[r * 4 + 3] = pv[r];
  }
  Twb[15] = 1.0;
  sp_inv_T(Twb, Tbw);
  sp_pose_T(st + sp_off_cb(P), Tcb);
  sp_mm(Tcb, Tbw, T, 4, 4, 4);
  double Tb[16][16];
  for (int j = 0; j < i; ++j) {
    sp_pose_T(st + sp_off_base(P) + KBO_POSE * j, Tb[j]);
    sp_mm(Tb[j], T, tmp, 4, 4, 4);
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
  if (Js) {
    double ch0[8] = {-Jp[0], -Jp[1], -Jp[2], 0.0, -Jp[3], -Jp[4], -Jp[5], 0.0};
    double Bm[24], ch[12], ch2[12], A[36];
    sp_box_minus(ph, Bm);
    sp_mm(ch0, Bm, ch, 2, 4, 6);
    for (int j = i - 1; j >= 0; --j) { /* Multiply: lhs B_j gets ch, rhs gets ch boxTimes(B_j) */
      const double tb[3] = {Tb[j][3], Tb[j][7], Tb[j][11]};
      sp_basic_dv(ch, 2, tb, JB[j]);
      sp_box_times(Tb[j], A);
      sp_mm(ch, A, ch2, 2, 6, 6);
      memcpy(ch, ch2, sizeof(ch));
    }
    const double tcb[3] = {Tcb[3], Tcb[7], Tcb[11]};
    sp_basic_dv(ch, 2, tcb, Jcb);
    sp_box_times(Tcb, A);
    sp_mm(ch, A, ch2, 2, 6, 6);
    /* Inverse node: -boxTimes(T_wb^-1) */
    sp_box_times(Tbw, A);
    for (int q = 0; q < 36; ++q) A[q] = -A[q];
    sp_mm(ch2, A, ch, 2, 6, 6);
    /* spline node: J = JT JS, JT = [I, -[p]x S; 0, S] (BSplinePose.cpp:394-412) */
    double S[9], px[9], pxS[9], JT[36];
    kbo_rv_S(pv + 3, S);
    sp_cross(pv, px);
    sp_mm(px, S, pxS, 3, 3, 3);
    memset(JT, 0, sizeof(JT));
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        JT[r * 6 + c] = (r == c) ? 1.0 : 0.0;
        JT[r * 6 + 3 + c] = -pxS[r * 3 + c];
        JT[(3 + r) * 6 + 3 + c] = S[r * 3 + c];
      }
    double chJ[12];
    sp_mm(ch, JT, chJ, 2, 6, 6);
    const int ns = 6 * P->order;
    for (int r = 0; r < 2; ++r)
      for (int j = 0; j < P->order; ++j)
        for (int c = 0; c < 6; ++c) Js[r * ns + 6 * j + c] = chJ[r * 6 + c] * w[j];
  }
  return e[0] * e[0] + e[1] * e[1];
}

/* ------------------------------------------------------------------ IMU term (defined here) */
/* Whitened residual [e_gyro / sigma_g; e_acc / sigma_a] of sample m:
 *   e_gyro = w_m - (w_b(t) + b_g),      w_b = -C^T S(theta) theta_dot      (BSplinePose.cpp:207-219)
 *   e_acc  = a_m - (C^T (p_ddot - g_w) + b_a)                                (cf. :175-180, minus gravity)
 * Js [6][6*order] (coefficients bidx..), Jimu [6][9] (b_g | b_a | g_w). */
static double sp_imu(const kbo_sp_problem* P, const double* st, int m, double e[6], double* Js, double* Jimu,
                     int* bidx) {
  const double t = P->imu_time[m];
  double v0[6], v1[6], v2[6], w0[8], w1[8], w2[8];
  const int b = sp_eval(P, st, t, 0, v0, w0);
  sp_eval(P, st, t, 1, v1, w1);
  sp_eval(P, st, t, 2, v2, w2);
  if (bidx) *bidx = b;
  const double* th = v0 + 3;
  const double* thd = v1 + 3;
  double Cm[9], S[9], Ct[9];
  kbo_rv_to_C(th, Cm);
  kbo_rv_S(th, S);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) Ct[r * 3 + c] = Cm[c * 3 + r];
  const double* ib = st + sp_off_imu(P);
  const double *bg = ib, *ba = ib + 3, *g = ib + 6;
  double wv[3], om[3], vv[3], fb[3];
  sp_mm(S, thd, wv, 3, 3, 1);
  sp_mm(Ct, wv, om, 3, 3, 1);
  for (int r = 0; r < 3; ++r) om[r] = -om[r];
  for (int r = 0; r < 3; ++r) vv[r] = v2[r] - g[r];
  sp_mm(Ct, vv, fb, 3, 3, 1);
  const double ig = 1.0 / P->sigma_gyro, ia = 1.0 / P->sigma_acc;
  const double* wm = P->imu_gyro + 3 * m;
  const double* am = P->imu_acc + 3 * m;
  for (int r = 0; r < 3; ++r) {
    e[r] = (wm[r] - om[r] - bg[r]) * ig;
    e[3 + r] = (am[r] - fb[r] - ba[r]) * ia;
  }
  if (Js) {
    /* d w_b / d theta = -C^T D + C^T [w]x S ; d w_b / d theta_dot = -C^T S
     * d f_b / d theta = -C^T [v]x S ;        d f_b / d p_ddot = C^T ;  d f_b / d g = -C^T */
    double D[9], CtD[9], wx[9], wxS[9], CtwxS[9], CtS[9], vx[9], vxS[9], CtvxS[9];
    kbo_rv_dSv(th, thd, D);
    sp_mm(Ct, D, CtD, 3, 3, 3);
    sp_cross(wv, wx);
    sp_mm(wx, S, wxS, 3, 3, 3);
    sp_mm(Ct, wxS, CtwxS, 3, 3, 3);
    sp_mm(Ct, S, CtS, 3, 3, 3);
    sp_cross(vv, vx);
    sp_mm(vx, S, vxS, 3, 3, 3);
    sp_mm(Ct, vxS, CtvxS, 3, 3, 3);
    const int ns = 6 * P->order;
    for (int j = 0; j < P->order; ++j)
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          const int rc = r * 3 + c;
          /* e_gyro = -w_b: translation columns 0, rotation columns -(w0 (-C^T D + C^T[w]xS) + w1 (-C^T S)) */
          Js[r * ns + 6 * j + c] = 0.0;
          Js[r * ns + 6 * j + 3 + c] = -(w0[j] * (-CtD[rc] + CtwxS[rc]) - w1[j] * CtS[rc]) * ig;
          /* e_acc = -f_b */
          Js[(3 + r) * ns + 6 * j + c] = -(w2[j] * Ct[rc]) * ia;
          Js[(3 + r) * ns + 6 * j + 3 + c] = -(w0[j] * (-CtvxS[rc])) * ia;
        }
  }
  if (Jimu) {
    memset(Jimu, 0, 54 * sizeof(double));
    for (int r = 0; r < 3; ++r) {
      Jimu[r * 9 + r] = -ig;           /* d e_gyro / d b_g */
      Jimu[(3 + r) * 9 + 3 + r] = -ia; /* d e_acc / d b_a */
      for (int c = 0; c < 3; ++c) Jimu[(3 + r) * 9 + 6 + c] = Ct[r * 3 + c] * ia; /* d e_acc / d g = C^T */
    }
  }
  double s = 0.0;
  for (int r = 0; r < 6; ++r) s += e[r] * e[r];
  return s;
}

/* dense rows (finite-difference tests): reprojection 2 x ncols, IMU 6 x ncols */
double kbo_sp_reproj_dense(const kbo_sp_problem* P, const double* st, int v, int k, double e[2], double* J, int ncols) {
  sp_cols L;
  sp_layout(P, &L);
  const int i = P->view_cam[v], n = kbo_model_nintr(P->cam_model[i]), ns = 6 * P->order;
  double Jin[2 * KBO_MAX_INTR], JB[16][12], Jcb[12], Js[2 * 36];
  int b;
  const double chi2 = sp_reproj(P, st, v, k, e, Jin, JB, Jcb, Js, &b);
  if (J) {
    memset(J, 0, sizeof(double) * 2 * ncols);
    for (int r = 0; r < 2; ++r) {
      double* row = J + (size_t)r * ncols;
      for (int c = 0; c < n; ++c) row[L.intr[i] + c] = Jin[r * KBO_MAX_INTR + c];
      for (int j = 0; j < i; ++j)
        for (int c = 0; c < 6; ++c) row[L.base[j] + c] = JB[j][r * 6 + c];
      for (int c = 0; c < 6; ++c) row[L.cb + c] = Jcb[r * 6 + c];
      for (int c = 0; c < ns; ++c) row[L.C + 6 * b + c] = Js[r * ns + c];
    }
  }
  return chi2;
}

double kbo_sp_imu_dense(const kbo_sp_problem* P, const double* st, int m, double e[6], double* J, int ncols) {
  sp_cols L;
  sp_layout(P, &L);
  const int ns = 6 * P->order;
  double Js[6 * 36], Ji[54];
  int b;
  const double chi2 = sp_imu(P, st, m, e, Js, Ji, &b);
  if (J) {
    memset(J, 0, sizeof(double) * 6 * ncols);
    for (int r = 0; r < 6; ++r) {
      double* row = J + (size_t)r * ncols;
      for (int c = 0; c < 9; ++c) row[L.bg + c] = Ji[r * 9 + c];
      for (int c = 0; c < ns; ++c) row[L.C + 6 * b + c] = Js[r * ns + c];
    }
  }
  return chi2;
}

/* ------------------------------------------------------------------ threading */
typedef struct {
  void (*fn)(void*, int, int);
  void* ctx;
  int tid, nt;
} sp_job;
static void* sp_job_run(void* a) {
  sp_job* j = (sp_job*)a;
  j->fn(j->ctx, j->tid, j->nt);
  return NULL;
}
static void sp_parallel(int nt, void (*fn)(void*, int, int), void* ctx) {
  if (nt <= 1) {
    fn(ctx, 0, 1);
    return;
  }
  pthread_t th[256];
  sp_job jobs[256];
  for (int t = 0; t < nt; ++t) {
    jobs[t].fn = fn;
    jobs[t].ctx = ctx;
    jobs[t].tid = t;
    jobs[t].nt = nt;
    pthread_create(&th[t], NULL, sp_job_run, &jobs[t]);
  }
  for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------ cost (evaluateError) */
typedef struct {
  const kbo_sp_problem* P;
  const double* st;
  double part[256];
} sp_cost_ctx;
static void sp_cost_job(void* a, int tid, int nt) {
  sp_cost_ctx* c = (sp_cost_ctx*)a;
  const kbo_sp_problem* P = c->P;
  double s = 0.0, e[6];
  for (int v = tid; v < P->n_views; v += nt)
    for (int k = 0; k < P->view_offset[v + 1] - P->view_offset[v]; ++k)
      s += sp_reproj(P, c->st, v, k, e, NULL, NULL, NULL, NULL, NULL);
  for (int m = tid; m < P->n_imu; m += nt) s += sp_imu(P, c->st, m, e, NULL, NULL, NULL);
  c->part[tid] = s;
}
/* ------------------------------------------------------------------ BSplineMotionError */
/* Q = curveQuadraticIntegralSparse(W, m) (BSpline.cpp:1585-1622; segmentQuadraticIntegral :1512-1548) is
 * sum over the valid segments of int (d^m f/dt^m)^T W (d^m f/dt^m) dt as a quadratic form in the coefficients:
 * Q_(k,l) = W * int b_k^(m)(t) b_l^(m)(t) dt.  Restated by 4-point Gauss-Legendre quadrature per segment of the
 * basis-weight products (exact: the integrand is a polynomial of degree <= 2 (order - 1 - m) <= 6), an
 * independent route from the reference's moment matrices V (Vi :1276-1300) and derivative matrices Dii. */
int kbo_sp_motion_band(const kbo_sp_problem* P, double* q) {
  if (!P->motion_W) return 0;
  const int o = P->order, K = sp_ncoef(P), m = P->motion_order;
  static const double gx[4] = {-0.86113631159405257522, -0.33998104358485626480, 0.33998104358485626480,
                               0.86113631159405257522};
  static const double gw[4] = {0.34785484513745385737, 0.65214515486254614263, 0.65214515486254614263,
                               0.34785484513745385737};
  memset(q, 0, sizeof(double) * (size_t)K * o);
  for (int sgi = 0; sgi + o <= K; ++sgi) {
    const double t0 = P->knots[sgi + o - 1], t1 = P->knots[sgi + o];
    if (!(t1 > t0)) continue;
    for (int g = 0; g < 4; ++g) {
      const double t = t0 + 0.5 * (t1 - t0) * (1.0 + gx[g]), wt = 0.5 * (t1 - t0) * gw[g];
      double w[8];
      const int b = kbo_bspline_weights(o, P->knots, P->n_knots, t, m, w);
      if (b < 0) continue;
      for (int j = 0; j < o; ++j)
        for (int l = j; l < o; ++l) q[(size_t)(b + j) * o + (l - j)] += wt * w[j] * w[l];
    }
  }
  return 1;
}

static double sp_motion_terms(const kbo_sp_problem* P, const double* st, double* Hband, double* gs) {
  const int o = P->order, K = sp_ncoef(P);
  double* q = (double*)malloc(sizeof(double) * (size_t)K * o);
  if (!kbo_sp_motion_band(P, q)) {
    free(q);
    return 0.0;
  }
  const double* c = st + sp_off_coef(P);
  const double* W = P->motion_W;
  double cost = 0.0;
  for (int k = 0; k < K; ++k)
    for (int d = 0; d < o && k + d < K; ++d) {
      const double qk = q[(size_t)k * o + d];
      double Wc[6], Wc2[6];  /* W c_(k+d), W c_k */
      for (int a = 0; a < 6; ++a) {
        Wc[a] = Wc2[a] = 0.0;
        for (int bb = 0; bb < 6; ++bb) {
          Wc[a] += W[a * 6 + bb] * c[6 * (k + d) + bb];
          Wc2[a] += W[a * 6 + bb] * c[6 * k + bb];
        }
      }
      double e = 0.0;
      for (int a = 0; a < 6; ++a) e += c[6 * k + a] * Wc[a];
      cost += (d == 0 ? 1.0 : 2.0) * qk * e;
      if (Hband)
        for (int a = 0; a < 36; ++a) Hband[((size_t)k * o + d) * 36 + a] += qk * W[a];
      if (gs)
        for (int a = 0; a < 6; ++a) {  /* buildHessianImplementation: rhs -= Q c (BSplineMotionError.hpp:154) */
          gs[6 * k + a] -= qk * Wc[a];
          if (d > 0) gs[6 * (k + d) + a] -= qk * Wc2[a];
        }
    }
  free(q);
  return cost;
}

double kbo_sp_motion_cost(const kbo_sp_problem* P, const double* st) { return sp_motion_terms(P, st, NULL, NULL); }

/* ------------------------------------------------------------------ ErrorTermEuclidean priors on p(t) */
/* evaluateErrorImplementation (ErrorTermEuclidean.cpp:50-57): e = t.toEuclidean() - prior, chi^2 = e^T invR e;
 * t = BSplinePositionExpressionNode: p(t) = eval(t).head<3>() (BSplineExpressions.cpp:132-136), its Jacobian the
 * first three rows of evalDAndJacobian(t, 0) per coefficient DV (:138-149): w_j(t) on the coefficient's p columns.
 * Returns chi^2; *bidx = the first coefficient (-1 outside the time range: the term is skipped). */
static double sp_pos(const kbo_sp_problem* P, const double* st, int k, double e[3], double* w, int* bidx) {
  double v[6];
  const int b = sp_eval(P, st, P->pos_time[k], 0, v, w);
  *bidx = b;
  if (b < 0) {
    e[0] = e[1] = e[2] = 0.0;
    return 0.0;
  }
  for (int a = 0; a < 3; ++a) e[a] = v[a] - P->pos_prior[3 * k + a];
  const double* W = P->pos_invR + 9 * k;
  double c = 0.0;
  for (int a = 0; a < 3; ++a)
    for (int bb = 0; bb < 3; ++bb) c += e[a] * W[3 * a + bb] * e[bb];
  return c;
}

double kbo_sp_pos_dense(const kbo_sp_problem* P, const double* st, int k, double e[3], double* J, int ncols) {
  double w[8];
  int b;
  const double c = sp_pos(P, st, k, e, w, &b);
  memset(J, 0, sizeof(double) * 3 * (size_t)ncols);
  if (b < 0) return 0.0;
  const int c0 = kbo_sp_cam_cols(P);
  for (int j = 0; j < P->order; ++j)
    for (int a = 0; a < 3; ++a) J[(size_t)a * ncols + c0 + 6 * (b + j) + a] = w[j];
  return c;
}

/* the priors' share of the normal equations (ErrorTermFs: H += J^T invR J, rhs -= J^T invR e) and of the cost */
static double sp_pos_terms(const kbo_sp_problem* P, const double* st, double* Hband, double* gs) {
  const int o = P->order;
  double cost = 0.0;
  for (int k = 0; k < P->n_pos; ++k) {
    double e[3], w[8];
    int b;
    cost += sp_pos(P, st, k, e, w, &b);
    if (b < 0) continue;
    const double* W = P->pos_invR + 9 * k;
    double We[3];
    for (int a = 0; a < 3; ++a) We[a] = W[3 * a] * e[0] + W[3 * a + 1] * e[1] + W[3 * a + 2] * e[2];
    for (int i = 0; i < o; ++i) {
      if (gs)
        for (int a = 0; a < 3; ++a) gs[6 * (b + i) + a] -= w[i] * We[a];
      if (Hband)
        for (int j = i; j < o; ++j) {
          double* Hb = Hband + ((size_t)(b + i) * o + (j - i)) * 36;
          for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) Hb[6 * a + c] += w[i] * w[j] * W[3 * a + c];
        }
    }
  }
  return cost;
}

double kbo_sp_pos_cost(const kbo_sp_problem* P, const double* st) { return sp_pos_terms(P, st, NULL, NULL); }

double kbo_sp_eval_cost(const kbo_sp_problem* P, const double* st, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  sp_cost_ctx c;
  c.P = P;
  c.st = st;
  sp_parallel(nthreads, sp_cost_job, &c);
  double s = 0.0;
  for (int t = 0; t < nthreads; ++t) s += c.part[t];
  return s + sp_motion_terms(P, st, NULL, NULL)  /* evaluateErrorImplementation: c^T Q c */
           + sp_pos_terms(P, st, NULL, NULL);    /* ErrorTermEuclidean priors */
}

/* ------------------------------------------------------------------ normal equations */
/* kbo_sp_system: Hcc [C][C], Hsc [6K][C], Hband [K][order][6][6] (block (k, k+d)), gc [C], gs [6K];
 * g = -J^T e (the rhs of the reference, LinearSystemSolver.cpp:21 + SparseCholeskyLinearSystemSolver.cpp:44). */
typedef struct {
  const kbo_sp_problem* P;
  const double* st;
  int nt;
  double** Hcc;  /* per thread */
  double** Hsc;
  double** Hb;
  double** gc;
  double** gs;
  double* cost;
} sp_build_ctx;

static void sp_accum(const kbo_sp_problem* P, int C, int b, int rows, const double* Jc /* rows x C */,
                     const double* Js /* rows x ns */, const double* e, double* Hcc, double* Hsc, double* Hb,
                     double* gc, double* gs) {
  const int ns = 6 * P->order, K = sp_ncoef(P);
  (void)K;
  for (int a = 0; a < C; ++a) {
    double g = 0.0;
    for (int r = 0; r < rows; ++r) g += Jc[r * C + a] * e[r];
    gc[a] -= g;
    for (int c = 0; c < C; ++c) {
      double s = 0.0;
      for (int r = 0; r < rows; ++r) s += Jc[r * C + a] * Jc[r * C + c];
      Hcc[a * C + c] += s;
    }
  }
  for (int a = 0; a < ns; ++a) {
    const int ga = 6 * b + a; /* global spline column */
    double g = 0.0;
    for (int r = 0; r < rows; ++r) g += Js[r * ns + a] * e[r];
    gs[ga] -= g;
    for (int c = 0; c < C; ++c) {
      double s = 0.0;
      for (int r = 0; r < rows; ++r) s += Js[r * ns + a] * Jc[r * C + c];
      Hsc[(size_t)ga * C + c] += s;
    }
    for (int bb = 0; bb < ns; ++bb) {
      const int ka = a / 6, kb = bb / 6;
      if (kb < ka) continue; /* upper block band (k, k+d) */
      double s = 0.0;
      for (int r = 0; r < rows; ++r) s += Js[r * ns + a] * Js[r * ns + bb];
      Hb[((size_t)(b + ka) * P->order + (kb - ka)) * 36 + (a % 6) * 6 + (bb % 6)] += s;
    }
  }
}

static void sp_build_job(void* a, int tid, int nt) {
  sp_build_ctx* c = (sp_build_ctx*)a;
  const kbo_sp_problem* P = c->P;
  sp_cols L;
  sp_layout(P, &L);
  const int C = L.C, ns = 6 * P->order;
  double* Jc = (double*)malloc(sizeof(double) * 6 * C);
  double Js[6 * 36], e[6], Jin[2 * KBO_MAX_INTR], JB[16][12], Jcb[12], Ji[54];
  double cost = 0.0;
  for (int v = tid; v < P->n_views; v += nt) {
    const int i = P->view_cam[v], n = kbo_model_nintr(P->cam_model[i]);
    for (int k = 0; k < P->view_offset[v + 1] - P->view_offset[v]; ++k) {
      int b;
      cost += sp_reproj(P, c->st, v, k, e, Jin, JB, Jcb, Js, &b);
      memset(Jc, 0, sizeof(double) * 2 * C);
      for (int r = 0; r < 2; ++r) {
        for (int q = 0; q < n; ++q) Jc[r * C + L.intr[i] + q] = Jin[r * KBO_MAX_INTR + q];
        for (int j = 0; j < i; ++j)
          for (int q = 0; q < 6; ++q) Jc[r * C + L.base[j] + q] = JB[j][r * 6 + q];
        for (int q = 0; q < 6; ++q) Jc[r * C + L.cb + q] = Jcb[r * 6 + q];
      }
      sp_accum(P, C, b, 2, Jc, Js, e, c->Hcc[tid], c->Hsc[tid], c->Hb[tid], c->gc[tid], c->gs[tid]);
    }
  }
  for (int m = tid; m < P->n_imu; m += nt) {
    int b;
    cost += sp_imu(P, c->st, m, e, Js, Ji, &b);
    memset(Jc, 0, sizeof(double) * 6 * C);
    for (int r = 0; r < 6; ++r)
      for (int q = 0; q < 9; ++q) Jc[r * C + L.bg + q] = Ji[r * 9 + q];
    sp_accum(P, C, b, 6, Jc, Js, e, c->Hcc[tid], c->Hsc[tid], c->Hb[tid], c->gc[tid], c->gs[tid]);
  }
  (void)ns;
  c->cost[tid] = cost;
  free(Jc);
}

void kbo_sp_build(const kbo_sp_problem* P, const double* st, int nthreads, kbo_sp_system* A) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  const int C = kbo_sp_cam_cols(P), K = sp_ncoef(P), o = P->order;
  const size_t nHcc = (size_t)C * C, nHsc = (size_t)6 * K * C, nHb = (size_t)K * o * 36;
  sp_build_ctx c;
  double *Hcc[64], *Hsc[64], *Hb[64], *gc[64], *gs[64], cost[64];
  for (int t = 0; t < nthreads; ++t) {
    Hcc[t] = (double*)calloc(nHcc, sizeof(double));
    Hsc[t] = (double*)calloc(nHsc, sizeof(double));
    Hb[t] = (double*)calloc(nHb, sizeof(double));
    gc[t] = (double*)calloc(C, sizeof(double));
    gs[t] = (double*)calloc((size_t)6 * K, sizeof(double));
  }
  c.P = P;
  c.st = st;
  c.nt = nthreads;
  c.Hcc = Hcc;
  c.Hsc = Hsc;
  c.Hb = Hb;
  c.gc = gc;
  c.gs = gs;
  c.cost = cost;
  sp_parallel(nthreads, sp_build_job, &c);
  A->C = C;
  A->K = K;
  A->order = o;
  memset(A->Hcc, 0, nHcc * sizeof(double));
  memset(A->Hsc, 0, nHsc * sizeof(double));
  memset(A->Hband, 0, nHb * sizeof(double));
  memset(A->gc, 0, C * sizeof(double));
  memset(A->gs, 0, (size_t)6 * K * sizeof(double));
  A->cost = 0.0;
  for (int t = 0; t < nthreads; ++t) { /* fixed-order reduction */
    for (size_t q = 0; q < nHcc; ++q) A->Hcc[q] += Hcc[t][q];
    for (size_t q = 0; q < nHsc; ++q) A->Hsc[q] += Hsc[t][q];
    for (size_t q = 0; q < nHb; ++q) A->Hband[q] += Hb[t][q];
    for (int q = 0; q < C; ++q) A->gc[q] += gc[t][q];
    for (int q = 0; q < 6 * K; ++q) A->gs[q] += gs[t][q];
    A->cost += cost[t];
    free(Hcc[t]);
    free(Hsc[t]);
    free(Hb[t]);
    free(gc[t]);
    free(gs[t]);
  }
  /* symmetrise Hcc (full) */
  for (int a = 0; a < C; ++a)
    for (int b = 0; b < a; ++b) A->Hcc[a * C + b] = A->Hcc[b * C + a];
  A->cost += sp_motion_terms(P, st, A->Hband, A->gs);  /* BSplineMotionError::buildHessianImplementation */
  A->cost += sp_pos_terms(P, st, A->Hband, A->gs);     /* ErrorTermEuclidean priors */
}

/* ------------------------------------------------------------------ solve */
/* The CHOLMOD stand-in for the spline system: band Cholesky of the coefficient block (half bandwidth
 * 6*order - 1 scalars, the fill-free AMD-like elimination of a banded arrow), Schur complement onto the
 * C camera/IMU columns, dense Cholesky, back-substitution.  (H + lambda^2 I) dx = g. */
static int sp_dense_chol(double* A, int n) {
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
    if (!(s > 0.0)) return 0;
    const double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double t = A[i * n + j];
      for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 1;
}
static void sp_dense_solve_L(const double* L, int n, double* x) {
  for (int i = 0; i < n; ++i) {
    double s = x[i];
    for (int k = 0; k < i; ++k) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = x[i];
    for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

int kbo_sp_solve(const kbo_sp_system* A, double lambda, double* dx) {
  const int C = A->C, K = A->K, o = A->order, n = 6 * K, bw = 6 * o; /* band storage: row i, cols i..i+bw-1 */
  const double lam2 = lambda * lambda;
  double* Bd = (double*)calloc((size_t)n * bw, sizeof(double));
  for (int k = 0; k < K; ++k)
    for (int d = 0; d < o && k + d < K; ++d)
      for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) {
          const int i = 6 * k + a, j = 6 * (k + d) + b;
          if (j < i) continue;
          Bd[(size_t)i * bw + (j - i)] = A->Hband[((size_t)k * o + d) * 36 + a * 6 + b] + (i == j ? lam2 : 0.0);
        }
  /* band Cholesky H_ss = U^T U (upper band) */
  int ok = 1;
  for (int i = 0; i < n && ok; ++i) {
    double s = Bd[(size_t)i * bw];
    if (!(s > 0.0)) { ok = 0; break; }
    const double d = sqrt(s);
    Bd[(size_t)i * bw] = d;
    const int jmax = i + bw - 1 < n - 1 ? i + bw - 1 : n - 1;
    for (int j = i + 1; j <= jmax; ++j) Bd[(size_t)i * bw + (j - i)] /= d;
    for (int j = i + 1; j <= jmax; ++j) {
      const double uij = Bd[(size_t)i * bw + (j - i)];
      if (uij == 0.0) continue;
      for (int l = j; l <= jmax; ++l) Bd[(size_t)j * bw + (l - j)] -= uij * Bd[(size_t)i * bw + (l - i)];
    }
  }
  if (!ok) {
    free(Bd);
    return 0;
  }
  /* X = H_ss^-1 [H_sc | g_s]  (C + 1 columns) */
  const int m = C + 1;
  double* X = (double*)malloc(sizeof(double) * (size_t)n * m);
  for (int i = 0; i < n; ++i) {
    for (int c = 0; c < C; ++c) X[(size_t)i * m + c] = A->Hsc[(size_t)i * C + c];
    X[(size_t)i * m + C] = A->gs[i];
  }
  for (int i = 0; i < n; ++i) { /* U^T y = rhs */
    const double d = Bd[(size_t)i * bw];
    for (int c = 0; c < m; ++c) X[(size_t)i * m + c] /= d;
    const int jmax = i + bw - 1 < n - 1 ? i + bw - 1 : n - 1;
    for (int j = i + 1; j <= jmax; ++j) {
      const double u = Bd[(size_t)i * bw + (j - i)];
      for (int c = 0; c < m; ++c) X[(size_t)j * m + c] -= u * X[(size_t)i * m + c];
    }
  }
  for (int i = n - 1; i >= 0; --i) { /* U x = y */
    const int jmax = i + bw - 1 < n - 1 ? i + bw - 1 : n - 1;
    for (int j = i + 1; j <= jmax; ++j) {
      const double u = Bd[(size_t)i * bw + (j - i)];
      for (int c = 0; c < m; ++c) X[(size_t)i * m + c] -= u * X[(size_t)j * m + c];
    }
    const double d = Bd[(size_t)i * bw];
    for (int c = 0; c < m; ++c) X[(size_t)i * m + c] /= d;
  }
  /* S = H_cc + lam2 I - H_sc^T X_c ; b = g_c - H_sc^T X_g */
  double* S = (double*)malloc(sizeof(double) * C * C);
  double* bv = (double*)malloc(sizeof(double) * C);
  for (int a = 0; a < C; ++a) {
    for (int c = 0; c < C; ++c) S[a * C + c] = A->Hcc[a * C + c] + (a == c ? lam2 : 0.0);
    bv[a] = A->gc[a];
  }
  for (int i = 0; i < n; ++i) {
    const double* h = A->Hsc + (size_t)i * C;
    const double* x = X + (size_t)i * m;
    for (int a = 0; a < C; ++a) {
      for (int c = 0; c < C; ++c) S[a * C + c] -= h[a] * x[c];
      bv[a] -= h[a] * x[C];
    }
  }
  for (int a = 0; a < C; ++a) /* symmetrise the accumulated S */
    for (int c = 0; c < a; ++c) S[a * C + c] = S[c * C + a] = 0.5 * (S[a * C + c] + S[c * C + a]);
  ok = sp_dense_chol(S, C);
  if (ok) {
    sp_dense_solve_L(S, C, bv);
    for (int a = 0; a < C; ++a) dx[a] = bv[a];
    for (int i = 0; i < n; ++i) {
      double s = X[(size_t)i * m + C];
      for (int c = 0; c < C; ++c) s -= X[(size_t)i * m + c] * bv[c];
      dx[C + i] = s;
    }
  }
  free(S);
  free(bv);
  free(X);
  free(Bd);
  return ok;
}

/* dense check of the same system (small problems only) */
int kbo_sp_dense_solve(const kbo_sp_system* A, double lambda, double* dx) {
  const int C = A->C, K = A->K, o = A->order, n = C + 6 * K;
  double* H = (double*)calloc((size_t)n * n, sizeof(double));
  for (int a = 0; a < C; ++a)
    for (int c = 0; c < C; ++c) H[(size_t)a * n + c] = A->Hcc[a * C + c];
  for (int i = 0; i < 6 * K; ++i)
    for (int c = 0; c < C; ++c) H[(size_t)(C + i) * n + c] = H[(size_t)c * n + C + i] = A->Hsc[(size_t)i * C + c];
  for (int k = 0; k < K; ++k)
    for (int d = 0; d < o && k + d < K; ++d)
      for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) {
          const double v = A->Hband[((size_t)k * o + d) * 36 + a * 6 + b];
          const int i = C + 6 * k + a, j = C + 6 * (k + d) + b;
          H[(size_t)i * n + j] = v;
          H[(size_t)j * n + i] = v;
        }
  for (int i = 0; i < n; ++i) H[(size_t)i * n + i] += lambda * lambda;
  for (int a = 0; a < C; ++a) dx[a] = A->gc[a];
  for (int i = 0; i < 6 * K; ++i) dx[C + i] = A->gs[i];
  const int ok = sp_dense_chol(H, n);
  if (ok) sp_dense_solve_L(H, n, dx);
  free(H);
  return ok;
}

/* ------------------------------------------------------------------ update (Optimizer2::applyStateUpdate) */
double kbo_sp_apply_update(const kbo_sp_problem* P, double* st, const double* dx) {
  sp_cols L;
  sp_layout(P, &L);
  for (int i = 0; i < P->n_cams; ++i) {
    const int n = kbo_model_nintr(P->cam_model[i]);
    for (int c = 0; c < n; ++c) st[i * KBO_MAX_INTR + c] += dx[L.intr[i] + c];
  }
  double* poses[17];
  int cols[17], np = 0;
  for (int j = 0; j < P->n_cams - 1; ++j) {
    poses[np] = st + sp_off_base(P) + KBO_POSE * j;
    cols[np++] = L.base[j];
  }
  poses[np] = st + sp_off_cb(P);
  cols[np++] = L.cb;
  for (int q = 0; q < np; ++q) { /* RotationQuaternion / EuclideanPoint updates */
    double qn[4];
    kbo_update_quat(poses[q], dx + cols[q], qn);
    memcpy(poses[q], qn, sizeof(qn));
    for (int c = 0; c < 3; ++c) poses[q][4 + c] += dx[cols[q] + 3 + c];
  }
  for (int c = 0; c < 9; ++c) st[sp_off_imu(P) + c] += dx[L.bg + c]; /* EuclideanPoint-style additive */
  const int K = sp_ncoef(P);
  for (int q = 0; q < 6 * K; ++q) st[sp_off_coef(P) + q] += dx[L.C + q]; /* DesignVariableMappedVector<6> */
  double m = 0.0;
  const int n = L.C + 6 * K;
  for (int q = 0; q < n; ++q) m = fabs(dx[q]) > m ? fabs(dx[q]) : m;
  return m;
}

/* ------------------------------------------------------------------ system alloc */
int kbo_sp_system_alloc(const kbo_sp_problem* P, kbo_sp_system* A) {
  const int C = kbo_sp_cam_cols(P), K = sp_ncoef(P), o = P->order;
  A->C = C;
  A->K = K;
  A->order = o;
  A->Hcc = (double*)calloc((size_t)C * C, sizeof(double));
  A->Hsc = (double*)calloc((size_t)6 * K * C, sizeof(double));
  A->Hband = (double*)calloc((size_t)K * o * 36, sizeof(double));
  A->gc = (double*)calloc(C, sizeof(double));
  A->gs = (double*)calloc((size_t)6 * K, sizeof(double));
  A->cost = 0.0;
  return (A->Hcc && A->Hsc && A->Hband && A->gc && A->gs) ? 0 : -1;
}
void kbo_sp_system_free(kbo_sp_system* A) {
  free(A->Hcc);
  free(A->Hsc);
  free(A->Hband);
  free(A->gc);
  free(A->gs);
  memset(A, 0, sizeof(*A));
}

/* ------------------------------------------------------------------ Optimizer2 loop (GN / LM), as kbo_optimize */
int kbo_sp_optimize(const kbo_sp_problem* P, double* st, const kbo_options* o, kbo_srv* srv, double* trace,
                    int trace_cap) {
  const int ncols = kbo_sp_total_cols(P), ns = kbo_sp_state_size(P);
  const int nt = o->nthreads < 1 ? 1 : o->nthreads, lm = (o->policy == 0);
  kbo_sp_system A;
  kbo_sp_system_alloc(P, &A);
  double* dx = (double*)calloc(ncols, sizeof(double));
  double* tmp = (double*)calloc(ncols, sizeof(double));
  double* rhs = (double*)calloc(ncols, sizeof(double));
  double* backup = (double*)malloc(sizeof(double) * ns);
  memset(srv, 0, sizeof(*srv));
  double J = kbo_sp_eval_cost(P, st, nt), p_J = J;
  srv->J_start = p_J;
  double deltaX = o->eps_x + 1.0, deltaJ = o->eps_j + 1.0;
  int prevFailed = 0, linFail = 0, ntrace = 0, first = 1;
  double pol_J = J, pol_pJ = J, last_succ = J;
  double lambda = o->lambda0, gamma = 3.0, beta = 2.0, mu = 2.0;
  while (srv->iterations < o->max_iterations && srv->failed_iterations < o->max_iterations &&
         ((deltaX > o->eps_x && fabs(deltaJ) > o->eps_j) || linFail)) {
    if (prevFailed) {
      pol_J = J;
    } else {
      pol_pJ = last_succ;
      last_succ = J;
      pol_J = J;
    }
    int success, rebuild = 1;
    if (lm && !first) {
      double d2 = 0.0;
      for (int q = 0; q < ncols; ++q) d2 += dx[q] * (lambda * dx[q] + rhs[q]);
      const double rho = (pol_pJ - pol_J) / d2;
      if (prevFailed) {
        mu *= 2;
        lambda *= mu;
        rebuild = 0;
      } else if (rho <= 0) {
        mu *= 10;
        lambda *= mu;
        rebuild = 0;
      } else {
        if (lambda > 1e-16) {
          const double u1 = 1 / gamma, u2 = 1 - (beta - 1) * pow((2 * rho - 1), 3);
          lambda *= (u1 > u2) ? u1 : u2;
          mu = beta;
        } else {
          lambda = 1e-15;
        }
      }
    }
    if (rebuild) {
      kbo_sp_build(P, st, nt, &A);
      memcpy(rhs, A.gc, sizeof(double) * A.C);
      memcpy(rhs + A.C, A.gs, sizeof(double) * 6 * A.K);
    }
    success = kbo_sp_solve(&A, lm ? lambda : 0.0, tmp);
    if (success) memcpy(dx, tmp, sizeof(double) * ncols);
    first = 0;
    int accepted = 0;
    if (!success) {
      prevFailed = 1;
      linFail = 1;
      srv->failed_iterations++;
    } else {
      memcpy(backup, st, sizeof(double) * ns);
      deltaX = kbo_sp_apply_update(P, st, dx);
      J = kbo_sp_eval_cost(P, st, nt);
      deltaJ = p_J - J;
      if (lm) {
        if (deltaJ < 0.0) {
          memcpy(st, backup, sizeof(double) * ns);
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
  srv->J_final = p_J;
  srv->dx_final = deltaX;
  srv->dj_final = deltaJ;
  srv->linear_solver_failure = linFail;
  kbo_sp_system_free(&A);
  free(dx);
  free(tmp);
  free(rhs);
  free(backup);
  return ntrace;
}

static double sp_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

double kbo_sp_time_gn(const kbo_sp_problem* P, double* st, int n_iter, int nthreads) {
  kbo_sp_system A;
  kbo_sp_system_alloc(P, &A);
  double* dx = (double*)calloc(kbo_sp_total_cols(P), sizeof(double));
  const double t0 = sp_now();
  for (int it = 0; it < n_iter; ++it) {
    kbo_sp_build(P, st, nthreads, &A);
    if (kbo_sp_solve(&A, 0.0, dx)) kbo_sp_apply_update(P, st, dx);
    (void)kbo_sp_eval_cost(P, st, nthreads);
  }
  const double t1 = sp_now();
  kbo_sp_system_free(&A);
  free(dx);
  return t1 - t0;
}
