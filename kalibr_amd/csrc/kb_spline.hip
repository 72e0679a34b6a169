// kb_spline.hip -- configs[4] on the device: the rig (IMU body) on a cubic B-spline pose trajectory,
// camera ReprojectionError terms through the spline pose and IMU gyro / accelerometer terms, assembled
// into the block-banded normal equations and solved by block cyclic reduction + a Schur complement onto
// the camera / IMU block.  Entry points: include/kalibr_hip.h (kb_sp_*).
//
// Reference map (paths relative to the reference repository):
//   BSplinePose::transformationAndJacobian      bsplines/src/BSplinePose.cpp:26-41 (J = JT JS)
//   curveValueToTransformationAndJacobian       bsplines/src/BSplinePose.cpp:394-412 (JT = [I, -[p]x S; 0, S])
//   angularVelocityBodyFrame                    bsplines/src/BSplinePose.cpp:207-219
//   RotationVector                              Schweizer-Messer/sm_kinematics/src/RotationVector.cpp:10-103
//   BSplineTransformationExpressionNode         aslam_splines/src/BSplineExpressions.cpp:23-45
//   spline DVs (additive 6-vectors)             aslam_splines/src/BSplinePoseDesignVariable.cpp:9-19
//   B-spline basis (host side, kb_sp_upload)    bsplines/src/BSpline.cpp:58-152, 237-387
#include <hip/hip_runtime.h>
#include <type_traits>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kalibr_hip.h"
#include "kb_math.h"

// diagnostic build only (KB_STAMPS, tools/gpu_sp_stops.sh): the timed kernels return after phase i when
// KSP_DBG_STOP = i; the product library never reads the variable and has no early returns
#ifdef KB_STAMPS
#define KSP_STOP(i)                 \
  do {                              \
    if (d.dbg_stop == (i)) return;  \
  } while (0)
// timeline stamp (100 MHz s_memrealtime) of thread 0 of block 0 at slot i (tools/diag_sp_ts.py)
#define KSP_TS(i)                                                                                          \
  do {                                                                                                     \
    if (blockIdx.x == 0 && threadIdx.x == 0 && d.dbg_ts && (i) < 320) d.dbg_ts[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// the same for thread 0 of block b
#define KSP_TSB(b, i)                                                                                      \
  do {                                                                                                     \
    if (blockIdx.x == (b) && threadIdx.x == 0 && d.dbg_ts && (i) < 320) d.dbg_ts[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define KSP_TSB(b, i) \
  do {                \
  } while (0)
#define KSP_STOP(i) \
  do {              \
  } while (0)
#define KSP_TS(i) \
  do {            \
  } while (0)
#endif

namespace kb_internal {
int fail(const std::string& m);
}

namespace ksp {
using kb::kMmAll;

constexpr int ORD = 4;      // spline order of the device path
constexpr int SB = 3;       // coefficients per cyclic-reduction node: couplings reach only the next node
constexpr int NB = 6 * SB;  // 18 rows per node
constexpr int MAXC = 64;    // camera + IMU block
constexpr int FPB = 2;      // frames per k_sp_frames block (600 blocks at configs[4]; 1 frame per block measured no faster: its 1,200 partial rows cost k_sp_reduce_cc 4 us)
constexpr int RW = 16;      // waves of the column-sum kernels (k_sp_reduce_cc, k_sp_schur_red)
constexpr int XS = 17;      // LDS row stride of the 64 x 16 Jacobian-row tile
constexpr int WI = 55;      // IMU theta partial row: 9x9 upper (45) | g (9) | cost
constexpr int NPB = 4;      // nodes per k_sp_schur block
constexpr int TCH = 32;     // IMU samples staged per k_sp_assemble chunk
constexpr int TCF = 8;      // frames staged per k_sp_assemble chunk
constexpr int IRQ = 42;     // IMU record: T1 [9] | T2 [9] | T3 [9] | C^T [9] | e [6] (imu_sample)
constexpr int IRS = IRQ + 13;  // LDS stride of a staged IMU record: record | w0 w1 w2 [12] | pad
constexpr int PNS = 8;      // IMU samples per k_sp_assemble operand panel (48 residual rows = 12 MFMA k-steps)
constexpr int PST = 49;     // LDS row stride of the panel (48 columns: Jw [36] | J_theta [9] | -e | 0 0)
enum { SC_COST_BUILD = 0, SC_OK = 1, SC_DX = 2, SC_COST = 3, SC_LAM2 = 4, SC_NSC = 8 };

struct SpDev {
  int N, C, K, F, M, n, m, n_target;
  int nin[KB_MAX_CAMS], model[KB_MAX_CAMS], col_intr[KB_MAX_CAMS];
  int col_pose[KB_MAX_CAMS];  // pose DV q: B_q (q < N-1), T_c0_b (q = N-1)
  int col_imu;
  int ckind[MAXC], cidx[MAXC], csub[MAXC];  // column -> (0 intr | 1 pose | 2 imu, cam / q, sub-index)
  int off_base, off_cb, off_imu, off_coef, S;
  int nblk_f, nblk_s, nblk_ci, nblk_ic, Wc, Ws, FHS;
  double ig, ia;
  const double* target;
  const double2* y;
  const uint16_t* cid;
  const int2* fview;      // [F][N]
  const int* fb;          // [F] first coefficient of the frame's support
  const double* fw;       // [F][4] basis weights (derivative 0)
  const int* ib;          // [M]
  const double* iw;       // [M][12] weights of derivatives 0, 1, 2
  const double* imeas;    // [M][6] gyro | accel
  const int* node_fr;     // [n][2] frame range with bidx in [3i-3, 3i+2]
  const int* node_im;     // [n][2]
  double* state;
  double* backup;
  double* FH;             // [F][FHS]: H_vv (36) | H_vtheta (6 C) | g_v (6)
  double* part;           // [nblk_f][Wc] theta-theta partial rows of the frames
  double* ipart;          // [nblk_ic][WI]
  double* Hcc;            // [C][C] | gc [C] | cost
  double *D0, *U0, *R0;   // built node blocks [n][324], [n][324], [n][18 m]
  double *D, *U, *R;      // working copies (cyclic reduction in place)
  double *Lf, *Z, *X;     // [n][324], [n][18 (36 + m)], [n][18 m]
  double* Lid;            // [n][18] inverse diagonal of Lf
  double* spart;          // [nblk_s][Ws]
  double* dx;             // [C + 6K]
  double* dmax;           // [n]
  double* cpart;          // [nblk_f + nblk_ci + nblk_q]
  double* sc;             // scalars
  double* Sf;             // [C][C] Schur complement (+ lam2 I) | b [C]
  const short2* uab;      // [Wc] (a, b) of upper-triangle entry q; (a, C) for g_a; (C, C) for the cost
  // BSplineMotionError (kb_sp_set_motion_error): cost c^T Q c, H += Q, g -= Q c on the coefficient band
  int mot;                // 1: active
  int nblk_q;             // k_sp_cost_motion blocks (64 nodes each)
  const double* QD;       // [n][324] Q blocks within node i
  const double* QU;       // [n][324] Q block node i (rows) -> node i + 1 (columns)
  double* mcost;          // [n] per-node motion (+ prior) cost at the build state
  // ErrorTermEuclidean priors on p(t) (kb_sp_set_position_priors), sorted by first coefficient: e = p(t_k) - prior_k,
  // chi^2 = e^T invR e, J = w_j [I_3 | 0] on coefficient pb + j
  int npos;               // 0: none
  int cq;                 // coefficient-only terms present (motion or priors): node cost kernels + reductions run
  const int* pb;          // [npos] first coefficient
  const double* pw;       // [npos][4] value weights
  const double* pp;       // [npos][3] prior
  const double* pW;       // [npos][9] invR
  const int* node_pp;     // [n][4] priors touching node i (b in [3i-3, 3i+2]) | owned by it (b in [3i, 3i+2])
  long long* dbg_ts;      // diagnostics only: [320] KSP_TS stamps
  int dbg_stop;           // diagnostics only (KSP_DBG_STOP): 0, or the phase after which the timed kernels return
  int zero_lam;           // GN pass: k_sp_imu_cc sets lambda^2 = 0 (no separate launch)
  int cc_fused;           // GN pass: k_sp_reduce_cc's column sums run as extra blocks of k_sp_elim1 (one launch less)
  int zsf;                // zs: the Schur sums of nodes 1.. run as extra blocks of the top level's launch (beside its
                          // one block), the top node's own term added by k_sp_schur_red
  // round 6: the Schur complement from the forward reduction alone (S = H_tt - sum_i Z_R,i^T Z_R,i over every node's
  // eliminated right-hand side, the top node's included) and the back substitution with ONE right-hand side
  // v = [-dtheta | 1] after the camera solve (k_sp_bvec*), instead of X = D^-1 [H_st | g_s] for all C + 1 columns
  int zs;
  double* xs;             // [n][18] the nodes' spline steps x_j = X_j v (zs)
  double* bm;             // [n][18][37] L_j^-T [Z_Uin,j | Z_U,j | Z_R,j v] (zs, k_sp_bprep)
  double* irec;           // [IRQ][M] per-sample IMU records (k_sp_imu_cc -> k_sp_assemble): T1 | T2 | T3 | C^T | e
};

typedef double v4d_t __attribute__((ext_vector_type(4)));

// a per-camera kernel-argument array read at a run-time index, by selects: a dynamic index into a kernel argument
// makes the compiler copy the array into per-lane scratch (k_sp_frames: 160 B per lane, ~11 MB of scratch writes per
// launch at configs[4])
__device__ __forceinline__ int sp_cam_arg(const int (&a)[KB_MAX_CAMS], int i) {
  int v = a[0];
#pragma unroll
  for (int k = 1; k < KB_MAX_CAMS; ++k) v = (i == k) ? a[k] : v;
  return v;
}
#define KSP_WAVE_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// ---------------------------------------------------------------- segment-wise staging (round 5)
// A segment is `len` consecutive doubles.  Thread tid takes items tid + u nth, u < U, with the source index clamped
// (no branch around the load), so the loads of all of a kernel's segments are in flight before its first store; items
// from U nth on (rigs wider than the U sizing) follow one by one.  An item's address is one add: the packed
// ksp_batched staging of the cyclic-reduction kernels spent ~50 VALU instructions per item on segment selects and
// run-time divisions, 3.1-3.4 us of each 11 us level (tools/diag_sp_levels.py).
template <int U>
__device__ __forceinline__ void seg_ld(double (&v)[U], const double* src, int len, int tid, int nth) {
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = src[min(tid + u * nth, len - 1)];
}
template <int U, class St>
__device__ __forceinline__ void seg_st(const double (&v)[U], const double* src, int len, int tid, int nth, St st) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = tid + u * nth;
    if (q < len) st(q, v[u]);
  }
  for (int q = tid + U * nth; q < len; q += nth) st(q, src[q]);
}
// q / m for q < 2^20 and m <= 128 by a float product: (q + 1/2) / m keeps >= 1/(2m) from an integer, far above the
// float rounding error
__device__ __forceinline__ int div_small(int q, float rinv) { return (int)(((float)q + 0.5f) * rinv); }

// ---------------------------------------------------------------- batched staging
// Copies with U independent loads in flight per thread.  A runtime-bounded loop of load / store pairs waits for
// each load before it issues the next one, i.e. one memory round trip per iteration: that latency chain, not
// bytes or flops, was what the cyclic-reduction and Schur kernels spent their time on.  ld(q) is called for
// clamped q in [0, n) only (n >= 1) and must not depend on a loaded value; st(q, v) stores item q.
template <int U, class Ld, class St>
__device__ __forceinline__ void ksp_batched(int n, int tid, int nth, Ld ld, St st) {
  for (int q0 = tid; q0 < n; q0 += U * nth) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld(min(q0 + u * nth, n - 1));
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q0 + u * nth < n) st(q0 + u * nth, v[u]);
  }
}

// ---------------------------------------------------------------- rotation vector (RotationVector.cpp)
__device__ __forceinline__ void rv_C(const double* a, double* Cm) {
  const double ang = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  if (ang < 1e-14) {
#pragma unroll
    for (int q = 0; q < 9; ++q) Cm[q] = (q % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double ra = 1.0 / ang, ax = a[0] * ra, ay = a[1] * ra, az = a[2] * ra;
  double sa, ca;
  sincos(ang, &sa, &ca);
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

__device__ __forceinline__ void rv_S(const double* a, double* S) {
  const double ang = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
#pragma unroll
  for (int q = 0; q < 9; ++q) S[q] = (q % 4 == 0) ? 1.0 : 0.0;
  if (ang < 1e-14) return;
  const double ra = 1.0 / ang;
  const double x = a[0] * ra, y = a[1] * ra, z = a[2] * ra;
  const double st2 = sin(ang * 0.5), st = sin(ang);
  const double c1 = -2.0 * st2 * st2 * ra, c2 = (ang - st) * ra;
  // [x]x and [x]x^2 = x x^T - I
  const double X[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  const double X2[9] = {x * x - 1, x * y, x * z, x * y, y * y - 1, y * z, x * z, y * z, z * z - 1};
#pragma unroll
  for (int q = 0; q < 9; ++q) S[q] += c1 * X[q] + c2 * X2[q];
}

// d(S(a) v)/da: S v = v + alpha a x v + beta a x (a x v), alpha = (cos f - 1)/f^2, beta = (f - sin f)/f^3
__device__ __forceinline__ void rv_dSv(const double* a, const double* v, double* Dm) {
  const double f2 = a[0] * a[0] + a[1] * a[1] + a[2] * a[2], f = sqrt(f2);
  double al, be, dal, dbe;
  if (f < 1e-4) {
    al = -0.5 + f2 / 24.0;
    be = 1.0 / 6.0 - f2 / 120.0;
    dal = 1.0 / 12.0 - f2 / 180.0;
    dbe = -1.0 / 60.0 + f2 / 1260.0;
  } else {
    double s, c;
    sincos(f, &s, &c);
    al = (c - 1.0) / f2;
    be = (f - s) / (f2 * f);
    dal = (-s / f2 - 2.0 * (c - 1.0) / (f2 * f)) / f;
    dbe = ((1.0 - c) / (f2 * f) - 3.0 * (f - s) / (f2 * f2)) / f;
  }
  const double axv[3] = {a[1] * v[2] - a[2] * v[1], a[2] * v[0] - a[0] * v[2], a[0] * v[1] - a[1] * v[0]};
  const double av = a[0] * v[0] + a[1] * v[1] + a[2] * v[2];
  const double aaxv[3] = {a[0] * av - v[0] * f2, a[1] * av - v[1] * f2, a[2] * av - v[2] * f2};
  const double vx[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double daaxv = (r == c ? av : 0.0) + a[r] * v[c] - 2.0 * v[r] * a[c];
      Dm[r * 3 + c] = al * (-vx[r * 3 + c]) + axv[r] * dal * a[c] + be * daaxv + aaxv[r] * dbe * a[c];
    }
}

// ---------------------------------------------------------------- small SE(3) helpers
// entry (r, c) of boxTimes(R, t) M(tb), M = [[-[tb]x, I], [I, 0]] (TransformationBasic.cpp:49-66):
// maps a TransformationBasic DV perturbation (dphi, dt) to the 6-D left perturbation of the chain.
__device__ __forceinline__ double bt_basic(const double* R, const double* t, const double* tb, int r, int c) {
  // boxTimes = [[R, -[t]x R], [0, R]]
  double bt[6];
  const double tx[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if (r < 3) {
      if (k < 3) {
        bt[k] = R[r * 3 + k];
      } else {
        const int kk = k - 3;
        bt[k] = -(tx[r * 3 + 0] * R[0 * 3 + kk] + tx[r * 3 + 1] * R[1 * 3 + kk] + tx[r * 3 + 2] * R[2 * 3 + kk]);
      }
    } else {
      bt[k] = (k < 3) ? 0.0 : R[(r - 3) * 3 + (k - 3)];
    }
  }
  const double tbx[9] = {0, -tb[2], tb[1], tb[2], 0, -tb[0], -tb[1], tb[0], 0};
  double s = 0.0;
  if (c < 3) {  // rotation DV column: rows 0-2 -[tb]x, rows 3-5 I
#pragma unroll
    for (int k = 0; k < 3; ++k) s += bt[k] * (-tbx[k * 3 + c]);
    s += bt[3 + c];
  } else {  // translation DV column: rows 0-2 I
    s = bt[c - 3];
  }
  return s;
}

// LDS staging of n consecutive elements with U loads in flight per thread before their stores (a plain strided loop
// waits on every load: ~1 us per iteration when one wave per SIMD runs)
template <int U, class T>
__device__ __forceinline__ void stage_lds(T* dst, const T* src, int n, int tid, int nth) {
  for (int q0 = tid; q0 < n; q0 += U * nth) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[min(q0 + u * nth, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q0 + u * nth < n) dst[q0 + u * nth] = v[u];
  }
}

// ---------------------------------------------------------------- k_sp_frames: camera terms
// One block = FPB frames, one wave per camera.  Per frame: spline pose T_wb(t_f) and JT; per view the
// 16 x 16 local Hessian of [J_delta | J_intr | -e] by f64 MFMA SYRK through an LDS tile; then the frame's
// spline-side blocks (H_vv, H_vtheta, g_v in the curve-value coordinates v, JT folded in) to HBM and the
// camera-side (theta-theta) sums into the block's partial row.
__device__ __forceinline__ void imu_cc_wave(const SpDev& d, int blk, int lane, double* X);

template <unsigned MM>
__global__ void __launch_bounds__(512) k_sp_frames(SpDev d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int N = d.N, C = d.C, nth = blockDim.x, tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  double* Xw = sm + wave * 64 * XS;
  if ((int)blockIdx.x >= d.nblk_f) {  // the extra blocks: k_sp_imu_cc's work, one of its 64-sample blocks per wave
    const int blk = ((int)blockIdx.x - d.nblk_f) * N + wave;
    if (blk < d.nblk_ic) imu_cc_wave(d, blk, lane, Xw);
    return;
  }
  double* Hv = sm + N * 64 * XS;   // [N][256]
  double* Gv = Hv + N * 256;       // [N][36]
  double* Pv = Gv + N * 36;        // [N][36]
  double* Gp = Pv + N * 36;        // [N][N][36]
  double* Qp = Gp + N * N * 36;    // [N][N][36]
  double* tg = Qp + N * N * 36;    // [n_target][3]
  // frame-independent column tables, read per entry of every frame: (a, b) of the theta-theta entries and
  // column -> (kind, index, sub) (a load per entry and frame otherwise puts a dependent round trip in each
  // iteration of the per-frame loops)
  short2* tuab = (short2*)(tg + 3 * d.n_target);  // [Wc]
  int* tck = (int*)(tuab + d.Wc);                 // [C] kind | [C] index | [C] sub
  int* tci = tck + C;
  int* tcs = tci + C;
  __shared__ double tz[12];  // zeros | unit vector e1
  const int cam = wave;
  const double* st = d.state;
  KSP_TSB(300, 256);  // diagnostics: block 300's timeline in slots 256..271 (tools/diag_sp_asm.py)
  stage_lds<8>(tg, d.target, 3 * d.n_target, tid, nth);
  stage_lds<8>(tuab, d.uab, d.Wc, tid, nth);
  if (tid < 12) tz[tid] = tid == 6 ? 1.0 : 0.0;
  for (int q = tid; q < C; q += nth) {
    tck[q] = d.ckind[q];
    tci[q] = d.cidx[q];
    tcs[q] = d.csub[q];
  }
  // chain A_cam = B_{cam-1} .. B_0 T_c0_b (frame independent) and the pose-DV maps Gp[cam][q]
  double RA[9], tA[3];
  kb::quat2r(st + d.off_cb, RA);
  tA[0] = st[d.off_cb + 4];
  tA[1] = st[d.off_cb + 5];
  tA[2] = st[d.off_cb + 6];
  {
    double RP[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, tP[3] = {0, 0, 0};  // P = B_{cam-1} .. B_{q+1}
    for (int q = cam - 1; q >= 0; --q) {
      const double* bq = st + d.off_base + 7 * q;
      if (lane < 36) Gp[(cam * N + q) * 36 + lane] = bt_basic(RP, tP, bq + 4, lane / 6, lane % 6);
      double RB[9], R2[9], t2[3];
      kb::quat2r(bq, RB);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          R2[r * 3 + c] = RP[r * 3 + 0] * RB[0 * 3 + c] + RP[r * 3 + 1] * RB[1 * 3 + c] + RP[r * 3 + 2] * RB[2 * 3 + c];
        t2[r] = RP[r * 3 + 0] * bq[4] + RP[r * 3 + 1] * bq[5] + RP[r * 3 + 2] * bq[6] + tP[r];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) RP[k] = R2[k];
      tP[0] = t2[0];
      tP[1] = t2[1];
      tP[2] = t2[2];
    }
    if (lane < 36) Gp[(cam * N + (N - 1)) * 36 + lane] = bt_basic(RP, tP, st + d.off_cb + 4, lane / 6, lane % 6);
    double R2[9], t2[3];  // A = P T_c0_b
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
        R2[r * 3 + c] = RP[r * 3 + 0] * RA[0 * 3 + c] + RP[r * 3 + 1] * RA[1 * 3 + c] + RP[r * 3 + 2] * RA[2 * 3 + c];
      t2[r] = RP[r * 3 + 0] * tA[0] + RP[r * 3 + 1] * tA[1] + RP[r * 3 + 2] * tA[2] + tP[r];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) RA[k] = R2[k];
    tA[0] = t2[0];
    tA[1] = t2[1];
    tA[2] = t2[2];
  }
  __syncthreads();  // target, accumulators and Gp staged
  KSP_TSB(300, 257);
  const int model = sp_cam_arg(d.model, cam), nin = sp_cam_arg(d.nin, cam);
  const double* intr = st + cam * KB_MAX_INTR;
  const int mrow = lane >> 4, mcol = lane & 15;
  const int f0 = blockIdx.x * FPB, f1 = min(d.F, f0 + FPB);
  // The entries of the frame's spline side and of the block's camera side are sums over the views i of 6-term products
  // x[r xs] y[r ys] (the 12 reads issued before one fma chain), with the operands of each (entry, view) picked by selects
  // rather than branches: a single H entry is x = H[.] (stride 0) against the unit vector e1, a term the view does not
  // have is x = the zero vector
  const double* Z0 = tz;      // [6] zeros
  const double* E1 = tz + 6;  // [6] 1, 0, 0, 0, 0, 0
  auto dot6 = [&](const double* x, int xs, const double* y, int ys, double s) {
    double xv[6], yv[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      xv[r] = x[r * xs];
      yv[r] = y[r * ys];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) s += xv[r] * yv[r];
    return s;
  };
  v4d_t hs = {0.0, 0.0, 0.0, 0.0};  // this lane's entries of its view's H summed over the block's frames
  for (int f = f0; f < f1; ++f) {
    // spline pose at t_f (uniform across the block)
    const int b = d.fb[f];
    const double* w = d.fw + 4 * f;
    const double* cf = st + d.off_coef + 6 * b;
    double v[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[r] = w[0] * cf[r] + w[1] * cf[6 + r] + w[2] * cf[12 + r] + w[3] * cf[18 + r];
    double Rwb[9];
    rv_C(v + 3, Rwb);
    // T_cam_w = A T_wb^-1: R = RA Rwb^T, t = tA - R p
    double R[9], t[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        R[r * 3 + c] = RA[r * 3 + 0] * Rwb[c * 3 + 0] + RA[r * 3 + 1] * Rwb[c * 3 + 1] + RA[r * 3 + 2] * Rwb[c * 3 + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) t[r] = tA[r] - (R[r * 3 + 0] * v[0] + R[r * 3 + 1] * v[1] + R[r * 3 + 2] * v[2]);
    // G_v = -boxTimes(T_cam_w) JT, JT = [I, -[p]x S; 0, S], all 36 entries by lane 0 with compile-time indices (a
    // lane-per-entry form indexes R, S and [t]x at run time, which puts those arrays in per-lane scratch)
    if (lane == 0) {
      double S[9];
      rv_S(v + 3, S);
      const double tx[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
      const double px[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
      double JT[6][6], BT[6][6];
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          if (c < 3) {
            JT[k][c] = (k == c) ? 1.0 : 0.0;
            JT[3 + k][c] = 0.0;
          } else {
            const int cc = c - 3;
            JT[k][c] = -(px[k * 3 + 0] * S[0 * 3 + cc] + px[k * 3 + 1] * S[1 * 3 + cc] + px[k * 3 + 2] * S[2 * 3 + cc]);
            JT[3 + k][c] = S[k * 3 + cc];
          }
        }
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = 0; k < 6; ++k) {  // boxTimes(R, t)[r][k]
          if (r < 3)
            BT[r][k] = k < 3 ? R[r * 3 + k]
                             : -(tx[r * 3 + 0] * R[0 * 3 + k - 3] + tx[r * 3 + 1] * R[1 * 3 + k - 3] +
                                 tx[r * 3 + 2] * R[2 * 3 + k - 3]);
          else
            BT[r][k] = k < 3 ? 0.0 : R[(r - 3) * 3 + (k - 3)];
        }
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k < 6; ++k) s += BT[r][k] * JT[k][c];
          Gv[cam * 36 + r * 6 + c] = -s;
        }
    }
    KSP_TSB(300, 258 + 6 * (f - f0));
    // corners of view (f, cam): [J_delta | J_intr | -e] rows, SYRK on MFMA
    const int2 fv = d.fview[(size_t)f * N + cam];
    v4d_t acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    for (int base = fv.x; base < fv.y; base += 64) {
      const int k = base + lane;
      double xr[2][16];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 16; ++q) xr[r][q] = 0.0;
      if (k < fv.y) {
        const int ci = d.cid[k];
        const double2 yv = d.y[k];
        const double X0 = tg[3 * ci], X1 = tg[3 * ci + 1], X2 = tg[3 * ci + 2];
        const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
        const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
        const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
        double u, wv, Jp[6], Ji[2 * KB_MAX_INTR];
        kb::project_jac<MM>(model, intr, p0, p1, p2, u, wv, Jp, Ji);
        const double e0 = yv.x - u, e1 = yv.y - wv;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const double j0 = Jp[3 * r], j1 = Jp[3 * r + 1], j2 = Jp[3 * r + 2];
          xr[r][0] = -j0;
          xr[r][1] = -j1;
          xr[r][2] = -j2;
          xr[r][3] = -(j1 * p2 - j2 * p1);
          xr[r][4] = -(-j0 * p2 + j2 * p0);
          xr[r][5] = -(j0 * p1 - j1 * p0);
#pragma unroll
          for (int q = 0; q < 9; ++q) xr[r][6 + q] = (q < nin) ? -Ji[r * KB_MAX_INTR + q] : 0.0;
          xr[r][15] = -(r == 0 ? e0 : e1);
        }
      }
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        if (ph == 1 && base + 32 >= fv.y) break;  // wave-uniform
        if ((lane >> 5) == ph) {
          const int rr = 2 * (lane & 31);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            Xw[rr * XS + q] = xr[0][q];
            Xw[(rr + 1) * XS + q] = xr[1][q];
          }
        }
        KSP_WAVE_SYNC();
#pragma unroll
        for (int ks = 0; ks < 16; ks += 2) {
          const double xa = Xw[(4 * ks + mrow) * XS + mcol];
          const double xb = Xw[(4 * ks + 4 + mrow) * XS + mcol];
          acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, xa, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(xb, xb, acc1, 0, 0, 0);
        }
        KSP_WAVE_SYNC();
      }
    }
    // f64 MFMA C/D layout: lane l, reg r -> row (l >> 4) + 4 r, col l & 15
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double h = acc0[r] + acc1[r];
      Hv[cam * 256 + (mrow + 4 * r) * 16 + mcol] = h;
      hs[r] += h;
    }
    KSP_TSB(300, 259 + 6 * (f - f0));
    __syncthreads();
    KSP_TSB(300, 260 + 6 * (f - f0));
    // P_i = H_dd,i G_v,i ; Q_i[q] = H_dd,i Gp[i][q]
    for (int q = tid; q < N * 36 + N * N * 36; q += nth) {
      const bool isP = q < N * 36;
      const int qq = isP ? q : q - N * 36;
      const int i = isP ? qq / 36 : qq / (N * 36);
      const int e = qq % 36, r = e / 6, c = e % 6;
      const double* G = isP ? Gv + i * 36 : Gp + (qq / 36) * 36;
      const double* H = Hv + i * 256;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += H[r * 16 + k] * G[k * 6 + c];
      if (isP)
        Pv[qq] = s;
      else
        Qp[qq] = s;
    }
    __syncthreads();
    KSP_TSB(300, 261 + 6 * (f - f0));
    // spline side of the frame: [H_vv | H_vtheta | g_v]
    double* out = d.FH + (size_t)f * d.FHS;
    for (int q = tid; q < d.FHS; q += nth) {
      double s = 0.0;
      const bool vv = q < 36, vt = !vv && q < 36 + 6 * C;
      const int a = vv ? q / 6 : vt ? (q - 36) / C : q - 36 - 6 * C;
      const int col = vt ? (q - 36) % C : 0, bb = q % 6;
      const int kind = tck[col], idx = tci[col], sub = tcs[col];
      for (int i = 0; i < N; ++i) {
        const double* G = Gv + i * 36 + a;
        const double* H = Hv + i * 256;
        const bool in0 = kind == 0 && idx == i, in1 = kind == 1 && (idx == N - 1 || idx < i);
        const double* y = vv ? Pv + i * 36 + bb
                             : !vt ? H + 15 : in0 ? H + 6 + sub : in1 ? Qp + (i * N + idx) * 36 + sub : Z0;
        const int ys = vv ? 6 : (!vt || in0) ? 16 : in1 ? 6 : 1;
        s = dot6(G, 6, y, ys, s);
      }
      out[q] = s;
    }
    KSP_TSB(300, 262 + 6 * (f - f0));
    __syncthreads();  // the frame's Gv, Hv, Pv, Qp consumed
    KSP_TSB(300, 263 + 6 * (f - f0));
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) Hv[cam * 256 + (mrow + 4 * r) * 16 + mcol] = hs[r];
  __syncthreads();
  for (int qq = tid; qq < N * N * 36; qq += nth) {  // Q_i[q] = H_dd,i Gp[i][q] of the summed H
    const int i = qq / (N * 36), e = qq % 36, r = e / 6, c = e % 6;
    const double* G = Gp + (qq / 36) * 36;
    const double* H = Hv + i * 256;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += H[r * 16 + k] * G[k * 6 + c];
    Qp[qq] = s;
  }
  __syncthreads();
  KSP_TSB(300, 271);
  // camera side of the block: theta-theta upper | g_theta | cost.  Linear in each view's H (the maps Gp are frame
  // independent), so it is formed once from the views' H summed over the block's frames (per frame it cost ~5-9 us of
  // LDS round trips)
  const int nup = C * (C + 1) / 2;
  for (int q = tid; q < d.Wc; q += nth) {
    double s = 0.0;
    const bool up = q < nup, gt = !up && q < nup + C;
    const short2 ab = tuab[up ? q : 0];
    const int a = up ? ab.x : q - nup, bcol = up ? ab.y : 0;
    const int ka = tck[a], ia = tci[a], sa = tcs[a];
    const int kb2 = tck[bcol], ib2 = tci[bcol], sb = tcs[bcol];
    for (int i = 0; i < N; ++i) {
      const double* H = Hv + i * 256;
      const bool okA = (ka == 0 && ia == i) || (ka == 1 && (ia == N - 1 || ia < i));
      const bool okB = (kb2 == 0 && ib2 == i) || (kb2 == 1 && (ib2 == N - 1 || ib2 < i));
      const double* GA = Gp + (i * N + ia) * 36 + sa;
      const double* x;
      const double* y;
      int xs, ys;
      if (up) {  // (pose | intr) x (pose | intr)
        // an absent term reads zeros on both sides: Gp holds only the pairs (cam, q < cam | N - 1), the rest of its
        // LDS is whatever the last kernel left there (0 x NaN would poison the sum)
        const bool pa = ka == 1, pb = kb2 == 1, live = okA && okB;
        x = !live ? Z0 : pa ? GA : (pb ? H + 6 + sa : H + (6 + sa) * 16 + 6 + sb);
        xs = !live ? 1 : pa ? 6 : (pb ? 16 : 0);
        y = !live ? Z0 : pa ? (pb ? Qp + (i * N + ib2) * 36 + sb : H + 6 + sb) : (pb ? Gp + (i * N + ib2) * 36 + sb : E1);
        ys = !live ? 1 : pa ? (pb ? 6 : 16) : (pb ? 6 : 1);
      } else if (gt) {  // g_theta: intr a -> H[6 + sa][15]; pose a -> Gp^T H[.][15]
        x = !okA ? Z0 : ka == 1 ? GA : H + (6 + sa) * 16 + 15;
        xs = !okA ? 1 : ka == 1 ? 6 : 0;
        y = !okA ? Z0 : ka == 1 ? H + 15 : E1;
        ys = !okA || ka != 1 ? 1 : 16;
      } else {  // cost
        x = H + 255;
        xs = 0;
        y = E1;
        ys = 1;
      }
      s = dot6(x, xs, y, ys, s);
    }
    d.part[(size_t)blockIdx.x * d.Wc + q] = s;
  }
  KSP_TSB(300, 270);
}

// ---------------------------------------------------------------- IMU sample (defined in DESIGN.md 10)
// Whitened residual e[6] of sample m, Ct (C_wb^T) for the gravity columns and, when T is given, the three 3 x 3 factors
// T1 | T2 | T3 of its Jacobian blocks (J[6][24], 4 coefficients x [p | theta]; expanded in k_sp_assemble's panels).  Mirrors
// oracle/kb_oracle_spline.c:sp_imu (independently written).
__device__ void imu_sample(const SpDev& d, int m, double* e, double* T, double* Ct) {
  const int b = d.ib[m];
  const double* w = d.iw + 12 * m;  // w0[4] | w1[4] | w2[4]
  const double* cf = d.state + d.off_coef + 6 * b;
  double v0[6], v1[6], v2[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double c = cf[6 * j + r];
      s0 += w[j] * c;
      s1 += w[4 + j] * c;
      s2 += w[8 + j] * c;
    }
    v0[r] = s0;
    v1[r] = s1;
    v2[r] = s2;
  }
  double Cm[9], S[9];
  rv_C(v0 + 3, Cm);
  rv_S(v0 + 3, S);
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) Ct[r * 3 + c] = Cm[c * 3 + r];
  const double* ib = d.state + d.off_imu;
  double wv[3], om[3], vv[3], fb[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) wv[r] = S[r * 3 + 0] * v1[3] + S[r * 3 + 1] * v1[4] + S[r * 3 + 2] * v1[5];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    om[r] = -(Ct[r * 3 + 0] * wv[0] + Ct[r * 3 + 1] * wv[1] + Ct[r * 3 + 2] * wv[2]);
    vv[r] = v2[r] - ib[6 + r];
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) fb[r] = Ct[r * 3 + 0] * vv[0] + Ct[r * 3 + 1] * vv[1] + Ct[r * 3 + 2] * vv[2];
  const double* mm = d.imeas + 6 * m;
  const double ig = d.ig, ia = d.ia;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    e[r] = (mm[r] - om[r] - ib[r]) * ig;
    e[3 + r] = (mm[3 + r] - fb[r] - ib[3 + r]) * ia;
  }
  if (!T) return;
  double Dm[9];
  rv_dSv(v0 + 3, v1 + 3, Dm);
  const double wx[9] = {0, -wv[2], wv[1], wv[2], 0, -wv[0], -wv[1], wv[0], 0};
  const double vx[9] = {0, -vv[2], vv[1], vv[2], 0, -vv[0], -vv[1], vv[0], 0};
  double* T1 = T;  // T1 = -C^T D + C^T [w]x S ; T2 = C^T S ; T3 = C^T [v]x S
  double* T2 = T + 9;
  double* T3 = T + 18;
  {
    double wxS[9], vxS[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        wxS[r * 3 + c] = wx[r * 3 + 0] * S[0 * 3 + c] + wx[r * 3 + 1] * S[1 * 3 + c] + wx[r * 3 + 2] * S[2 * 3 + c];
        vxS[r * 3 + c] = vx[r * 3 + 0] * S[0 * 3 + c] + vx[r * 3 + 1] * S[1 * 3 + c] + vx[r * 3 + 2] * S[2 * 3 + c];
      }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        double a1 = 0.0, a2 = 0.0, a3 = 0.0, a4 = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          a1 += Ct[r * 3 + k] * Dm[k * 3 + c];
          a2 += Ct[r * 3 + k] * wxS[k * 3 + c];
          a3 += Ct[r * 3 + k] * S[k * 3 + c];
          a4 += Ct[r * 3 + k] * vxS[k * 3 + c];
        }
        T1[r * 3 + c] = -a1 + a2;
        T2[r * 3 + c] = a3;
        T3[r * 3 + c] = a4;
      }
  }
}



// ---------------------------------------------------------------- k_sp_assemble
// One block per cyclic-reduction node i (coefficients 3i..3i+2): D_i (18 x 18), U_i (coupling to node
// i+1) and R_i = [H_s,theta | g_s] (18 x (C+1)) from the frames and IMU samples whose support touches the
// node.
__global__ void __launch_bounds__(256) k_sp_assemble(SpDev d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  // XCD-aware node order: blocks are dealt to the 8 XCDs round-robin (block b on XCD b % 8), and a frame or an IMU sample
  // is read by the two neighbouring nodes, so each XCD takes a contiguous run of nodes (node i + 1 on the same L2 as
  // node i, one block later) instead of neighbours on different XCDs fetching the same rows twice from HBM
  const int nn = gridDim.x, xcd = blockIdx.x & 7, q8 = nn >> 3, r8 = nn & 7;
  const int i = xcd * q8 + min(xcd, r8) + (blockIdx.x >> 3);
  const int tid = threadIdx.x, nth = blockDim.x, C = d.C, m = d.m;
  const int nout = 2 * NB * NB + NB * m;
  double* out = sm;                       // [nout]
  // frame chunk [TCF][FHS] (FH rows) | IMU records [TCH][IRS] + operand panel [6 PNS][PST] share one region: a node
  // has ~3 frames and ~25 IMU samples, so a 32-term region of FHS rows would cut the blocks per CU
  double* tj = out + nout;
  const int stride = d.FHS;
  __shared__ int tb[TCH];
  __shared__ double tw[TCH][4];
  KSP_TSB(500, 241);  // diagnostics: block 500's timeline in slots 241..252 (tools/diag_sp_asm.py)
  for (int q = tid; q < nout; q += nth) out[q] = 0.0;
  const int k0 = SB * i;
  // ---- frames
  const int fa = d.node_fr[2 * i], fz = d.node_fr[2 * i + 1];
  for (int c0 = fa; c0 < fz; c0 += TCF) {
    const int nt = min(TCF, fz - c0);
    __syncthreads();
    const double* FHc = d.FH + (size_t)c0 * d.FHS;  // nt consecutive rows
    ksp_batched<8>(
        nt * d.FHS + 5 * nt, tid, nth,
        [&](int q) {
          const int e = q - nt * d.FHS;
          return e < 0 ? FHc[q] : e < nt ? (double)d.fb[c0 + e] : d.fw[4 * c0 + e - nt];
        },
        [&](int q, double v) {
          const int e = q - nt * d.FHS;
          if (e < 0)
            tj[q] = v;
          else if (e < nt)
            tb[e] = (int)v;
          else
            tw[(e - nt) / 4][(e - nt) % 4] = v;
        });
    __syncthreads();
    // the chunk's frames outer, this thread's UQ entries inner (independent LDS reads in flight); each entry sums its
    // frames in order.  Entry constants: D | U: coefficient rows kr, columns kc; R: kc = -1 (weight of the row only)
    constexpr int UQ = (2 * NB * NB + NB * (MAXC + 1) + 255) / 256;
    int ekr[UQ], ekc[UQ], eoff[UQ];
    double eacc[UQ];
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int q = min(tid + 256 * u, nout - 1);
      eacc[u] = 0.0;
      if (q < 2 * NB * NB) {
        const int blk = q / (NB * NB), e = q % (NB * NB), r = e / NB, c = e % NB;
        ekr[u] = k0 + r / 6;
        ekc[u] = k0 + SB * blk + c / 6;
        eoff[u] = (r % 6) * 6 + (c % 6);
      } else {
        const int e = q - 2 * NB * NB, r = e / m, a = e % m;
        ekr[u] = k0 + r / 6;
        ekc[u] = -1;
        eoff[u] = (a < C) ? 36 + (r % 6) * C + a : 36 + 6 * C + (r % 6);
      }
    }
    for (int t = 0; t < nt; ++t) {
      const int b = tb[t];
      const double* W = tw[t];
      const double* T = tj + t * stride;
#pragma unroll
      for (int u = 0; u < UQ; ++u) {
        const int jr = ekr[u] - b, jc = ekc[u] - b;
        const bool okr = jr >= 0 && jr <= 3, okc = jc >= 0 && jc <= 3;
        const double wr = W[min(max(jr, 0), 3)], wc = W[min(max(jc, 0), 3)], h = T[eoff[u]];
        if (ekc[u] >= 0)
          eacc[u] += (okr && okc) ? wr * wc * h : 0.0;
        else
          eacc[u] += okr ? wr * h : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u)
      if (tid + 256 * u < nout) out[tid + 256 * u] += eacc[u];
  }
  KSP_STOP(1);
  KSP_TSB(500, 242);
  // ---- IMU samples: per chunk of TCH, the records k_sp_imu_cc wrote (T1 | T2 | T3 | C^T | e) and the basis weights staged
  // in LDS; then per PNS samples an operand panel of 6 PNS residual rows x [Jw (nodes i, i + 1) | J_theta | -e | 0 0] built
  // by every thread, followed by its MFMA steps: Jn^T [Jw | J_theta | -e] with Jn = the panel's first 18 columns (this
  // node's rows), k = 4 st + (lane >> 4) = 6 t + z.  Waves 0..2: rows 0..15 x columns 16 w .. 16 w + 15 on
  // v_mfma_f64_16x16x4f64; wave 3: rows 16, 17 (padded to 4) x the 48 columns as three v_mfma_f64_4x4x4f64 per step
  // (4 blocks of 4 x 4: operand lane 16 k + 4 b + i, result (row 16 + (lane >> 4), column 16 g + (lane & 15)))
  const int ma = d.node_im[2 * i], mz = d.node_im[2 * i + 1];
  const int wave = tid >> 6, lane = tid & 63;
  v4d_t iacc = {0.0, 0.0, 0.0, 0.0};
  double iac4[3] = {0.0, 0.0, 0.0};
  double* rec = tj;              // [TCH][IRS]
  double* P = tj + TCH * IRS;    // [6 PNS][PST]
  for (int c0 = ma; c0 < mz; c0 += TCH) {
    const int nt = min(TCH, mz - c0);
    __syncthreads();
    {  // every load in flight before the stores: the IRQ field segments of nt samples, then the chunk's 12 nt weights
      constexpr int U = (TCH * (IRQ + 12) + 255) / 256;
      const int nr = IRQ * nt, nall = (IRQ + 12) * nt;
      double v[U];
      int dst[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = min(tid + u * 256, nall - 1);
        if (q < nr) {
          const int a = q / nt, t = q - a * nt;
          v[u] = d.irec[(size_t)a * d.M + c0 + t];
          dst[u] = t * IRS + a;
        } else {
          const int e = q - nr, t = e / 12;
          v[u] = d.iw[(size_t)12 * c0 + e];
          dst[u] = t * IRS + IRQ + (e - 12 * t);
        }
      }
      const int tbv = tid < nt ? d.ib[c0 + tid] : 0;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (tid + u * 256 < nall) rec[dst[u]] = v[u];
      if (tid < nt) tb[tid] = tbv;
    }
    KSP_STOP(2);
    KSP_TSB(500, 243);
    for (int s0 = 0; s0 < nt; s0 += PNS) {
      const int ns = min(PNS, nt - s0);
      __syncthreads();  // records staged / the previous panel consumed
      // one (column c, sample tt) item per thread and pass (48 x PNS = 384 items), its 6 residual rows unrolled: every
      // candidate operand read at a clamped in-record index, the entry chosen by selects
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int item = tid + 256 * u;
        if (item < 48 * PNS) {
          const int tt = item / 48, c = item - 48 * tt;
          const int t = min(s0 + tt, nt - 1);
          const double* R = rec + t * IRS;
          const double* w = R + IRQ;
          const int cb = c / 6, cc = c - 6 * cb, jj = k0 + cb - tb[t], j = min(max(jj, 0), 3);
          const bool lo = cc < 3, inj = c < 2 * NB && jj >= 0 && jj <= 3, live = tt < ns;
          const int cr = lo ? cc : cc - 3, ci = min(max(c - 2 * NB, 0), 8), cg = min(max(ci - 6, 0), 2);
          const double wj = w[j], w4 = w[4 + j], w8 = w[8 + j];
#pragma unroll
          for (int z = 0; z < 6; ++z) {
            const int zr = z % 3;
            double vj, vt;
            if (z < 3) {
              const double p1 = wj * R[3 * zr + cr], p2 = w4 * R[9 + 3 * zr + cr];
              vj = lo ? 0.0 : -(p1 - p2) * d.ig;
              vt = ci == z ? -d.ig : 0.0;
            } else {
              const double p1 = (lo ? w8 : wj) * R[(lo ? 27 : 18) + 3 * zr + cr];
              vj = lo ? -p1 * d.ia : p1 * d.ia;
              vt = ci < 3 ? 0.0 : ci < 6 ? (ci - 3 == zr ? -d.ia : 0.0) : R[27 + 3 * zr + cg] * d.ia;
            }
            const double v = c < 2 * NB ? (inj ? vj : 0.0) : c < 2 * NB + 9 ? vt : c == 2 * NB + 9 ? -R[36 + z] : 0.0;
            P[(6 * tt + z) * PST + c] = live ? v : 0.0;
          }
        }
      }
      __syncthreads();
      if (s0 / PNS < 4) KSP_TSB(500, 244 + 2 * (s0 / PNS));
      const int ks = (6 * ns + 3) / 4;  // rows k >= 6 ns of the panel are zeros
      if (wave < 3) {
        const double* pa = P + (lane >> 4) * PST + (lane & 15);
        const double* pb = pa + 16 * wave;
        for (int st = 0; st < ks; st += 2) {
          const double a0 = pa[4 * st * PST], b0 = pb[4 * st * PST];
          const double a1 = pa[4 * (st + 1) * PST], b1 = pb[4 * (st + 1) * PST];
          iacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, iacc, 0, 0, 0);
          iacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, iacc, 0, 0, 0);
        }
      } else {
        const int i4 = lane & 3;
        const double* pk = P + (lane >> 4) * PST;
        const int cb4 = 4 * ((lane >> 2) & 3) + i4;
        for (int st = 0; st < ks; ++st) {
          const double* row = pk + 4 * st * PST;
          const double a = i4 < 2 ? row[16 + i4] : 0.0;
          const double b0 = row[cb4], b1 = row[16 + cb4], b2 = row[32 + cb4];
          iac4[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b0, iac4[0], 0, 0, 0);
          iac4[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b1, iac4[1], 0, 0, 0);
          iac4[2] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b2, iac4[2], 0, 0, 0);
        }
      }
      if (s0 / PNS < 4 && wave == 0) KSP_TSB(500, 245 + 2 * (s0 / PNS));
    }
  }
  KSP_STOP(3);
  __syncthreads();  // frame sums complete (they are owned per entry q, the tiles per lane)
  // f64 MFMA C/D layout: lane l, reg r -> row (l >> 4) + 4 r, column l & 15 (waves 0..2, columns 16 w ..);
  // wave 3: row 16 + (l >> 4), column 16 g + (l & 15) of its 4x4x4 accumulator g
  if (ma < mz) {
    auto put = [&](int row, int jc, double v) {
      if (row >= NB) return;
      if (jc < 2 * NB)
        out[(jc < NB ? 0 : NB * NB) + row * NB + jc % NB] += v;
      else if (jc < 2 * NB + 9)
        out[2 * NB * NB + row * m + d.col_imu + jc - 2 * NB] += v;
      else if (jc == 2 * NB + 9)
        out[2 * NB * NB + row * m + C] += v;
    };
    if (wave < 3) {
#pragma unroll
      for (int r = 0; r < 4; ++r) put((lane >> 4) + 4 * r, 16 * wave + (lane & 15), iacc[r]);
    } else {
#pragma unroll
      for (int g = 0; g < 3; ++g) put(16 + (lane >> 4), 16 * g + (lane & 15), iac4[g]);
    }
  }
  __syncthreads();
  double node_cost = 0.0;  // thread 0: the node's coefficient-only terms at the build state (motion, own priors)
  if (d.mot) {  // BSplineMotionError::buildHessianImplementation (BSplineMotionError.hpp:96-160): H += Q, g -= Q c
    __shared__ double cn[3 * NB];  // coefficients of nodes i - 1, i, i + 1 (0 outside [0, K))
    for (int q = tid; q < 3 * NB; q += nth) {
      const int k = SB * (i - 1) + q / 6;
      cn[q] = (k >= 0 && k < d.K) ? d.state[d.off_coef + 6 * k + q % 6] : 0.0;
    }
    const double* QDi = d.QD + (size_t)i * NB * NB;
    const double* QUi = d.QU + (size_t)i * NB * NB;
    const double* QUl = d.QU + (size_t)(i > 0 ? i - 1 : 0) * NB * NB;
    for (int q = tid; q < 2 * NB * NB; q += nth) out[q] += q < NB * NB ? QDi[q] : QUi[q - NB * NB];
    __syncthreads();
    double nc = 0.0;
    if (tid < 64) {
      if (tid < NB) {
        const int r = tid;
        double a = 0.0, w = 0.0, l = 0.0;
        for (int c = 0; c < NB; ++c) {
          a += QDi[r * NB + c] * cn[NB + c];
          w += QUi[r * NB + c] * cn[2 * NB + c];
          l += (i > 0) ? QUl[c * NB + r] * cn[c] : 0.0;
        }
        out[2 * NB * NB + r * m + C] -= (a + w) + l;  // rows of node i of Q c
        nc = cn[NB + r] * (a + 2.0 * w);           // c_i^T QD_i c_i + 2 c_i^T QU_i c_(i+1)
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) nc += __shfl_xor(nc, o);
      if (tid == 0) node_cost = nc;
    }
    __syncthreads();
  }
  if (d.npos) {
    // ErrorTermEuclidean priors touching the node (ErrorTermEuclidean.cpp:50-66 over BSplinePositionExpressionNode,
    // BSplineExpressions.cpp:132-149): per prior e, invR e and chi^2 staged in LDS (one thread per prior), then every
    // output entry sums its priors in order: D / U += w_r w_c invR (position rows / columns), rhs -= w_r (invR e)
    __shared__ double pe[TCH][4];    // invR e | chi^2
    __shared__ double pwl[TCH][13];  // w [4] | invR [9]
    __shared__ int pbl[TCH];
    const int pa = d.node_pp[4 * i], pz = d.node_pp[4 * i + 1], oa = d.node_pp[4 * i + 2], oz = d.node_pp[4 * i + 3];
    double pc = 0.0;
    for (int c0 = pa; c0 < pz; c0 += TCH) {
      const int nt = min(TCH, pz - c0);
      __syncthreads();
      if (tid < nt) {
        const int k = c0 + tid, b = d.pb[k];
        const double* w = d.pw + 4 * k;
        const double* cf = d.state + d.off_coef + 6 * b;
        double e[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          double v = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) v += w[j] * cf[6 * j + a];
          e[a] = v - d.pp[3 * k + a];
        }
        const double* W = d.pW + 9 * k;
        double c2 = 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const double we = W[3 * a] * e[0] + W[3 * a + 1] * e[1] + W[3 * a + 2] * e[2];
          pe[tid][a] = we;
          c2 += e[a] * we;
        }
        pe[tid][3] = c2;
#pragma unroll
        for (int j = 0; j < 4; ++j) pwl[tid][j] = w[j];
#pragma unroll
        for (int q = 0; q < 9; ++q) pwl[tid][4 + q] = W[q];
        pbl[tid] = b;
      }
      __syncthreads();
      for (int q = tid; q < nout; q += nth) {
        double sacc = 0.0;
        if (q < 2 * NB * NB) {
          const int blk = q / (NB * NB), e = q % (NB * NB), r = e / NB, c = e % NB, a = r % 6, bb = c % 6;
          if (a < 3 && bb < 3) {
            const int kr = k0 + r / 6, kc = k0 + SB * blk + c / 6;
            for (int t = 0; t < nt; ++t) {
              const int jr = kr - pbl[t], jc = kc - pbl[t];
              if (jr < 0 || jr > 3 || jc < 0 || jc > 3) continue;
              sacc += pwl[t][jr] * pwl[t][jc] * pwl[t][4 + 3 * a + bb];
            }
          }
        } else {
          const int e = q - 2 * NB * NB, r = e / m, col = e % m, a = r % 6;
          if (col == C && a < 3) {
            const int kr = k0 + r / 6;
            for (int t = 0; t < nt; ++t) {
              const int jr = kr - pbl[t];
              if (jr < 0 || jr > 3) continue;
              sacc -= pwl[t][jr] * pe[t][a];
            }
          }
        }
        out[q] += sacc;
      }
      if (tid == 0)  // the node's own priors' chi^2, in order
        for (int t = max(oa, c0) - c0; t < min(oz, c0 + nt) - c0; ++t) pc += pe[t][3];
    }
    node_cost += pc;
    __syncthreads();
  }
  if (d.cq && tid == 0) d.mcost[i] = node_cost;
  KSP_TSB(500, 252);
  // padded rows (coefficients >= K): identity diagonal, no coupling
  for (int q = tid; q < nout; q += nth) {
    double v = out[q];
    if (q < NB * NB) {
      const int r = q / NB, c = q % NB;
      if (k0 + r / 6 >= d.K || k0 + c / 6 >= d.K) v = (r == c) ? 1.0 : 0.0;
    } else if (q < 2 * NB * NB) {
      const int e = q - NB * NB, r = e / NB, c = e % NB;
      if (k0 + r / 6 >= d.K || k0 + SB + c / 6 >= d.K) v = 0.0;
    } else {
      const int e = q - 2 * NB * NB, r = e / m;
      if (k0 + r / 6 >= d.K) v = 0.0;
    }
    if (q < NB * NB)
      d.D0[(size_t)i * NB * NB + q] = v;
    else if (q < 2 * NB * NB)
      d.U0[(size_t)i * NB * NB + q - NB * NB] = v;
    else
      d.R0[(size_t)i * NB * m + q - 2 * NB * NB] = v;
  }
}

// ---------------------------------------------------------------- IMU theta-theta (b_g | b_a | g_w)
// 64 samples per block (one wave): each lane's J_theta^T J_theta upper (45), -J_theta^T e (9), e^T e staged in
// LDS, summed per entry in sample order -> one partial row [WI].
// k_sp_imu_cc's work for its block blk (64 samples) on one wave: the samples' records for k_sp_assemble and the partial
// row [WI] of their theta-theta terms, each entry summed over the 64 samples in order through the wave's 64 x XS LDS
// tile X, 16 entries at a time.  Run by k_sp_imu_cc and by the extra blocks of k_sp_frames (one launch less per pass).
__device__ __forceinline__ void imu_cc_wave(const SpDev& d, int blk, int lane, double* X) {
  const int m = blk * 64 + lane;
  double e[6] = {0, 0, 0, 0, 0, 0}, Ct[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const bool has = m < d.M;
  if (d.zero_lam && m == 0) {  // k_sp_set_lam(0) of a GN pass, before the reduction reads it (same stream)
    d.sc[SC_LAM2] = 0.0;
    d.sc[SC_OK] = 1.0;
  }
  double T[27];
  if (has) {
    imu_sample(d, m, e, T, Ct);
#pragma unroll
    for (int q = 0; q < 27; ++q) d.irec[(size_t)q * d.M + m] = T[q];  // field-major: coalesced over the wave
#pragma unroll
    for (int q = 0; q < 9; ++q) d.irec[(size_t)(27 + q) * d.M + m] = Ct[q];
#pragma unroll
    for (int q = 0; q < 6; ++q) d.irec[(size_t)(36 + q) * d.M + m] = e[q];
  }
  double v[WI];
  // J_theta = [-ig I, 0, 0; 0, -ia I, ia C^T] (rows gyro | accel; columns b_g | b_a | g_w)
  const double ig2 = d.ig * d.ig, ia2 = d.ia * d.ia;
  int q = 0;
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int b = a; b < 9; ++b, ++q) {
      double t;
      if (a < 3)
        t = (b == a) ? ig2 : 0.0;
      else if (a < 6)
        t = (b == a) ? ia2 : (b >= 6 ? -ia2 * Ct[(a - 3) * 3 + (b - 6)] : 0.0);
      else
        t = (b == a) ? ia2 : 0.0;  // (C^T)^T C^T = I
      v[q] = has ? t : 0.0;
    }
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    double t;
    if (a < 3) {
      t = d.ig * e[a];
    } else if (a < 6) {
      t = d.ia * e[a];
    } else {
      t = -d.ia * (Ct[0 * 3 + (a - 6)] * e[3] + Ct[1 * 3 + (a - 6)] * e[4] + Ct[2 * 3 + (a - 6)] * e[5]);
    }
    v[45 + a] = has ? t : 0.0;
  }
  v[54] = has ? ((e[0] * e[0] + e[1] * e[1]) + (e[2] * e[2] + e[3] * e[3])) + (e[4] * e[4] + e[5] * e[5]) : 0.0;
#pragma unroll
  for (int q0 = 0; q0 < WI; q0 += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (q0 + j < WI) X[lane * XS + j] = v[q0 + j];
    KSP_WAVE_SYNC();
    if (lane < 16 && q0 + lane < WI) {
      double s = 0.0;
      for (int k = 0; k < 64; ++k) s += X[k * XS + lane];
      d.ipart[(size_t)blk * WI + q0 + lane] = s;
    }
    KSP_WAVE_SYNC();  // the tile is rewritten by the next 16 entries
  }
}

__global__ void __launch_bounds__(64) k_sp_imu_cc(SpDev d) {
  __shared__ double X[64 * XS];
  imu_cc_wave(d, blockIdx.x, threadIdx.x, X);
}

// ---------------------------------------------------------------- k_sp_reduce_cc: H_cc, g_c, cost
// 64 entries per block; the 4 waves sum interleaved partial rows (8 independent loads in flight per lane),
// combined in a fixed order.
// the RW waves' partial sums of one column, combined as a fixed pairwise tree
__device__ __forceinline__ double red_waves(const double (*red)[64], int lane) {
  double t[RW];
#pragma unroll
  for (int w = 0; w < RW; ++w) t[w] = red[w][lane];
#pragma unroll
  for (int h = RW / 2; h > 0; h /= 2)
#pragma unroll
    for (int w = 0; w < h; ++w) t[w] += t[w + h];
  return t[0];
}

__device__ __forceinline__ double col_sum(const double* p, int rows, int stride, int q, int w0, int ws) {
  double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int r = w0;
  for (; r + 7 * ws < rows; r += 8 * ws) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += p[(size_t)(r + u * ws) * stride + q];
  }
  for (int u = 0; r < rows; r += ws, ++u) a[u & 7] += p[(size_t)r * stride + q];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

__global__ void __launch_bounds__(64 * RW) k_sp_reduce_cc(SpDev d) {
  __shared__ double red[RW][64];
  const int C = d.C, nup = C * (C + 1) / 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * 64 + lane;
  const bool act = q < d.Wc;
  int ii = -1, a = 0, bcol = 0;
  if (act) {
    if (q < nup) {
      const short2 ab = d.uab[q];
      a = ab.x;
      bcol = ab.y;
      const int ia = a - d.col_imu, ib = bcol - d.col_imu;
      if (ia >= 0 && ia < 9 && ib >= 0 && ib < 9) ii = ia * 9 - ia * (ia - 1) / 2 + (ib - ia);
    } else if (q < nup + C) {
      const int ia = q - nup - d.col_imu;
      if (ia >= 0 && ia < 9) ii = 45 + ia;
    } else {
      ii = 54;
    }
  }
  double s = act ? col_sum(d.part, d.nblk_f, d.Wc, q, wave, RW) : 0.0;
  if (ii >= 0) s += col_sum(d.ipart, d.nblk_ic, WI, ii, wave, RW);
  red[wave][lane] = s;
  __syncthreads();
  if (wave != 0 || !act) return;
  s = red_waves(red, lane);
  if (q < nup) {
    d.Hcc[a * C + bcol] = s;
    d.Hcc[bcol * C + a] = s;
  } else if (q < nup + C) {
    d.Hcc[C * C + (q - nup)] = s;
  } else {
    d.Hcc[C * C + C] = s;
    d.sc[SC_COST_BUILD] = s;
  }
}

// ---------------------------------------------------------------- cyclic reduction
// The first elimination level and the first fused level read the built blocks D0 / U0 / R0 directly (the working
// copies D / U / R are written from the second level on): D_i = D0_i + lambda^2 I on the rows of real
// coefficients (padded rows keep their identity diagonal).
__device__ __forceinline__ double lam_diag(const SpDev& d, int i, int q, double lam2) {
  return (q / NB == q % NB && SB * i + q / (6 * NB) < d.K) ? lam2 : 0.0;
}

// Block-tridiagonal SPD system over nodes: D_i x_i + U_{i-1}^T x_{i-1} + U_i x_{i+1} = R_i (18 x m RHS).
// Level stride s: nodes i % 2s == s are eliminated (Cholesky L_j, Z_j = L_j^-1 [U_l^T | U_j | R_j]),
// nodes i % 2s == 0 absorb them; the back-substitution runs the levels in reverse.
// broadcast of lane l's double (l wave-uniform)
__device__ __forceinline__ double rdlane(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffull), l);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// 1/x by v_rcp_f64 + two Newton steps (within an ulp of the IEEE quotient)
__device__ __forceinline__ double ksp_recip(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
// the pivot chain's reciprocal: v_rcp_f64 + one Newton step (as k_solve's panel factor; two FMAs shorter per pivot)
__device__ __forceinline__ double ksp_recip1(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// ---- the 18 x 18 Cholesky with the pivot-row broadcasts fused into the FMAs (chol18_dpp, the default)
// x += (lane L's y within the lane's 16-lane row) * f by one v_fmac_f64 with a DPP row_newbcast source (64-bit DPP,
// gfx90a+); y may be x itself (operands are read before the write)
template <int L>
__device__ __forceinline__ void ksp_fmac_bc(double& x, double y, double f) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(y), "v"(f), "i"(L));
}
template <int L>
__device__ __forceinline__ void ksp_fmac_bc_self(double& x, double f) {
  asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(f), "i"(L));
}
// lane L's v within its 16-lane row after 2 wait states (the compiler does not see the DPP hazard of a VGPR an inline
// asm VALU instruction has just written)
template <int L>
__device__ __forceinline__ double ksp_bcast_dep(double v) {
  const unsigned long long b = __double_as_longlong(v);
  unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32), olo, ohi;
  asm volatile(
      "s_nop 1\n\tv_mov_b32_dpp %0, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xf\n\t"
      "v_mov_b32_dpp %1, %3 row_newbcast:%4 row_mask:0xf bank_mask:0xf"
      : "=&v"(olo), "=&v"(ohi)
      : "v"(lo), "v"(hi), "i"(L));
  return __longlong_as_double(((unsigned long long)ohi << 32) | olo);
}
template <int K, int J>
__device__ __forceinline__ void chol18_cols(double (&dr)[NB], double (&br)[NB], double nfd, double nfb) {
  if constexpr (J < NB) {
    ksp_fmac_bc<K>(br[J], dr[J], nfb);  // the below row first: it reads the pivot row's column J before its update
    ksp_fmac_bc_self<K>(dr[J], nfd);
    chol18_cols<K, J + 1>(dr, br, nfd, nfb);
  }
}
// pivot steps K .. 15 (the LDL^T form: W = L D kept in place, D_K on the diagonal), 1/sqrt(D_K) collected in rs[K]
template <int K>
__device__ __forceinline__ void chol18_steps(double (&dr)[NB], double (&br)[NB], double (&rs)[16], bool& ok) {
  if constexpr (K < 16) {
    const double Dk = ksp_bcast_dep<K>(dr[K]);
    const bool pos = Dk > 0.0;
    const double rdk = pos ? ksp_recip1(Dk) : 0.0;
    const double nfd = -(dr[K] * rdk), nfb = -(br[K] * rdk);
    chol18_cols<K, K + 1>(dr, br, nfd, nfb);
    ok = ok && pos;
    // 1 / sqrt(D_K) by v_rsq_f64 + two Newton steps, off the pivot chain (only the final scaling reads it)
    const double dpos = pos ? Dk : 1.0;
    double r = __builtin_amdgcn_rsq(dpos);
    r = r * fma(-0.5 * dpos * r, r, 1.5);
    rs[K] = r * fma(-0.5 * dpos * r, r, 1.5);
    chol18_steps<K + 1>(dr, br, rs, ok);
  }
}

// one-wave Cholesky of an 18 x 18 SPD matrix in LDS (row-major, both triangles), written back as the lower factor L
// with id = 1 / diag(L).  Columns 0..15 as one panel: every 16-lane row of the wave holds rows 0..15 (lane r: row r)
// and lanes 16, 17 also rows 16, 17 of the matrix; step K takes D_K and the pivot row from lane K of its own 16-lane row
// by DPP (fused into the FMAs: no v_readlane / SGPR round trip, which the readlane version pays twice per broadcast
// double).  Then the 2 x 2 trailing block (rows 16, 17) and the scaling W D^-1/2 -> L.  Returns false if not positive
// definite.  Call from one whole wave.
__device__ __forceinline__ bool chol18_dpp(double* A, double* id, int lane) {
  const int r = lane & 15, g = lane >> 4;
  const int br_row = (g == 1 && r < 2) ? 16 + r : r;  // lanes 16, 17: rows 16, 17 (the others: a copy, unused)
  double dr[NB], br[NB], rs[16];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    dr[c] = A[r * NB + c];
    br[c] = A[br_row * NB + c];
  }
  bool ok = true;
  chol18_steps<0>(dr, br, rs, ok);
  // trailing 2 x 2 (rows 16, 17 after the panel): D_16 = br[16] of lane 16, w = br[16] of lane 17, D_17 = br[17] of
  // lane 17 - w^2 / D_16
  // v_readlane of VGPRs the inline-asm FMAs just wrote: the wait states inside the statement
  auto rl_dep = [](double v, auto lane_c) {
    constexpr int LN = decltype(lane_c)::value;
    const unsigned long long b = __double_as_longlong(v);
    unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32), slo, shi;
    asm volatile("s_nop 4\n\tv_readlane_b32 %0, %2, %4\n\tv_readlane_b32 %1, %3, %4\n\ts_nop 1"
                 : "=s"(slo), "=s"(shi)
                 : "v"(lo), "v"(hi), "i"(LN));
    return __longlong_as_double(((unsigned long long)shi << 32) | slo);
  };
  const double d16 = rl_dep(br[16], std::integral_constant<int, 16>{});
  const double w17 = rl_dep(br[16], std::integral_constant<int, 17>{});
  const double a17 = rl_dep(br[17], std::integral_constant<int, 17>{});
  const bool p16 = d16 > 0.0;
  const double r16 = p16 ? ksp_recip(d16) : 0.0;
  const double d17 = a17 - w17 * w17 * r16;
  const bool p17 = d17 > 0.0;
  ok = ok && p16 && p17;
  auto rsq2 = [](double x) {
    const double dp = x > 0.0 ? x : 1.0;
    double q = __builtin_amdgcn_rsq(dp);
    q = q * fma(-0.5 * dp * q, q, 1.5);
    return q * fma(-0.5 * dp * q, q, 1.5);
  };
  const double s16 = rsq2(d16), s17 = rsq2(d17);
  KSP_WAVE_SYNC();
  if (lane < NB) {  // rows 0..15: lanes 0..15 (dr); rows 16, 17: lanes 16, 17 (br)
    const double* row = lane < 16 ? dr : br;
    double out[NB];
    double idr = 1.0;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      // W[row][c] / sqrt(D_c) below the diagonal, sqrt(D_row) = D_row / sqrt(D_row) on it, zero above
      const double v = row[c] * rs[c];
      out[c] = c <= lane ? v : 0.0;
      idr = (c == lane) ? rs[c] : idr;
    }
    out[16] = lane == 16 ? d16 * s16 : lane == 17 ? w17 * s16 : 0.0;
    out[17] = lane == 17 ? d17 * s17 : 0.0;
    idr = lane == 16 ? s16 : lane == 17 ? s17 : idr;
#pragma unroll
    for (int c = 0; c < NB; ++c) A[lane * NB + c] = out[c];
    id[lane] = idr;
  }
  KSP_WAVE_SYNC();
  return ok;
}

// one-wave register Cholesky of an 18 x 18 SPD matrix held in LDS (lower, row-major): lane r keeps row r in
// registers, column k broadcast by v_readlane; the factor is written back.  Returns false if not positive
// definite.  Call from one whole wave.
__device__ __forceinline__ bool chol18_wave(double* A, double* id, int lane) {
#ifndef KSP_CHOL_READLANE
  return chol18_dpp(A, id, lane);
#endif
  double a[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) a[c] = lane < NB ? A[lane * NB + c] : 0.0;
  bool ok = true;
  double rid = 1.0;  // lane k: 1 / L_kk
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const double dkk = rdlane(a[k], k);
    ok = ok && (dkk > 0.0);
    // 1 / sqrt(d_kk) by v_rsq_f64 + two Newton steps and L_kk = d_kk / sqrt(d_kk): a shorter dependent chain than
    // an IEEE square root followed by a reciprocal (wave-uniform, one per pivot)
    const double dpos = dkk > 0.0 ? dkk : 1.0;
    double rdk = __builtin_amdgcn_rsq(dpos);
    rdk = rdk * fma(-0.5 * dpos * rdk, rdk, 1.5);
    rdk = rdk * fma(-0.5 * dpos * rdk, rdk, 1.5);
    const double dk = dpos * rdk;
    // no masks on the updates: for lanes r <= k (and r < c) the update only touches the upper triangle
    // a[c > r], which is never read (column k's entries L[c][k] come from lanes c > k) and is written back as zero
    rid = (lane == k) ? rdk : rid;
    a[k] = (lane == k) ? dk : a[k] * rdk;
    const double lk = a[k];
#pragma unroll
    for (int c = k + 1; c < NB; ++c) {
      const double lck = rdlane(a[k], c);
      a[c] = fma(-lk, lck, a[c]);
    }
  }
  KSP_WAVE_SYNC();
  if (lane < NB) {
#pragma unroll
    for (int c = 0; c < NB; ++c) A[lane * NB + c] = c <= lane ? a[c] : 0.0;
    id[lane] = rid;
  }
  KSP_WAVE_SYNC();
  return ok;
}

// L Z = W (lower L in LDS, inverse diagonal id), one thread per column of the [18][ws] LDS tile W, written to
// dst (row stride ds)
__device__ __forceinline__ void node_forward(const double* L, const double* id, const double* W, int ws, int ncol,
                                             double* dst, int ds, int tid, int nth = -1) {
  if (nth < 0) nth = blockDim.x;
  for (int c = tid; c < ncol; c += nth) {
    // right-looking: once z[k] is final it updates every later row, so the dependent chain is one FMA and one
    // multiply per row (the left-looking dot products chained all 153 FMAs)
    double z[NB];
#pragma unroll
    for (int row = 0; row < NB; ++row) z[row] = W[row * ws + c];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      z[k] *= id[k];
#pragma unroll
      for (int row = k + 1; row < NB; ++row) z[row] -= L[row * NB + k] * z[k];
    }
#pragma unroll
    for (int row = 0; row < NB; ++row) dst[row * ds + c] = z[row];
  }
}

// node_forward with the L loads kept per row (a compiler barrier between rows): the kernels that keep the next
// node's operands in registers across the solve cannot hold all 171 hoisted L entries as well
__device__ __forceinline__ void node_forward_lean(const double* L, const double* id, const double* W, int ws,
                                                  int ncol, double* dst, int ds, int tid, int nth = -1) {
  if (nth < 0) nth = blockDim.x;
  for (int c = tid; c < ncol; c += nth) {
    double z[NB];
#pragma unroll
    for (int row = 0; row < NB; ++row) z[row] = W[row * ws + c];
#pragma unroll
    for (int k = 0; k < NB; ++k) {  // the arithmetic of node_forward, in the same order
      asm volatile("" ::: "memory");
      z[k] *= id[k];
#pragma unroll
      for (int row = k + 1; row < NB; ++row) z[row] -= L[row * NB + k] * z[k];
    }
#pragma unroll
    for (int row = 0; row < NB; ++row) dst[row * ds + c] = z[row];
  }
}

// back substitution of one 18-row node with LDS-staged operands: x = L^-T T (T row stride ts), one thread per
// RHS column, written to out (row stride m)
__device__ __forceinline__ void node_backsolve(const double* L, const double* id, const double* T, int ts, int m,
                                               double* out, int tid, int nth = -1) {
  if (nth < 0) nth = blockDim.x;
  for (int c = tid; c < m; c += nth) {
    double z[NB];
#pragma unroll
    for (int row = 0; row < NB; ++row) z[row] = T[row * ts + c];
    // right-looking (see node_forward)
#pragma unroll
    for (int k = NB - 1; k >= 0; --k) {
      z[k] *= id[k];
#pragma unroll
      for (int row = 0; row < k; ++row) z[row] -= L[k * NB + row] * z[k];
    }
#pragma unroll
    for (int row = 0; row < NB; ++row) out[row * m + c] = z[row];
  }
}

// node_backsolve with the L loads kept per row (see node_forward_lean)
__device__ __forceinline__ void node_backsolve_lean(const double* L, const double* id, const double* T, int ts, int m,
                                                    double* out, int tid, int nth) {
  for (int c = tid; c < m; c += nth) {
    double z[NB];
#pragma unroll
    for (int row = 0; row < NB; ++row) z[row] = T[row * ts + c];
#pragma unroll
    for (int k = NB - 1; k >= 0; --k) {  // the arithmetic of node_backsolve, in the same order
      asm volatile("" ::: "memory");
      z[k] *= id[k];
#pragma unroll
      for (int row = 0; row < k; ++row) z[row] -= L[k * NB + row] * z[k];
    }
#pragma unroll
    for (int row = 0; row < NB; ++row) out[row * m + c] = z[row];
  }
}

// first level (stride 1): odd nodes j eliminated, Z_j = L_j^-1 [U_{j-1}^T | U_j | R_j]
// k_sp_reduce_cc's column sums for columns 4 e .. 4 e + 3 of the theta partial rows on a 256-thread block (the extra
// blocks of k_sp_elim1 in a GN pass: H_cc is first read by the Schur sums, after the levels): thread (phase ph, column
// c) sums rows ph, ph + 64, .. of the frame and IMU partials, then the 64 phases in a fixed tree through red [320]
__device__ __forceinline__ void cc_sums_block(const SpDev& d, int e, double* red) {
  const int C = d.C, nup = C * (C + 1) / 2, tid = threadIdx.x, c = tid & 3, ph = tid >> 2;
  const int q = 4 * e + c;
  const bool act = q < d.Wc;
  int ii = -1, a = 0, bcol = 0;
  if (act) {
    if (q < nup) {
      const short2 ab = d.uab[q];
      a = ab.x;
      bcol = ab.y;
      const int ia = a - d.col_imu, ib = bcol - d.col_imu;
      if (ia >= 0 && ia < 9 && ib >= 0 && ib < 9) ii = ia * 9 - ia * (ia - 1) / 2 + (ib - ia);
    } else if (q < nup + C) {
      const int ia = q - nup - d.col_imu;
      if (ia >= 0 && ia < 9) ii = 45 + ia;
    } else {
      ii = 54;
    }
  }
  double s = act ? col_sum(d.part, d.nblk_f, d.Wc, q, ph, 64) : 0.0;
  if (ii >= 0) s += col_sum(d.ipart, d.nblk_ic, WI, ii, ph, 64);
  red[ph * 4 + c] = s;
  __syncthreads();
  if (tid < 64) {
    const int g = tid >> 2;
    red[256 + tid] = (red[16 * g + c] + red[16 * g + 4 + c]) + (red[16 * g + 8 + c] + red[16 * g + 12 + c]);
  }
  __syncthreads();
  if (tid >= 4 || !act) return;
  double t[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) t[g] = red[256 + 4 * g + c];
#pragma unroll
  for (int h = 8; h > 0; h >>= 1)
#pragma unroll
    for (int g = 0; g < h; ++g) t[g] += t[g + h];
  s = t[0];
  if (q < nup) {
    d.Hcc[a * C + bcol] = s;
    d.Hcc[bcol * C + a] = s;
  } else if (q < nup + C) {
    d.Hcc[C * C + (q - nup)] = s;
  } else {
    d.Hcc[C * C + C] = s;
    d.sc[SC_COST_BUILD] = s;
  }
}

__global__ void __launch_bounds__(256) k_sp_elim1(SpDev d) {
  __shared__ double L[NB * NB];
  __shared__ double id[NB];
  extern __shared__ __attribute__((aligned(16))) double W[];  // [18][36 + m]
  if ((int)blockIdx.x >= d.n / 2) {  // GN pass (cc_fused): the camera block's column sums
    cc_sums_block(d, (int)blockIdx.x - d.n / 2, L);
    return;
  }
  const int j = 1 + 2 * blockIdx.x, tid = threadIdx.x, m = d.m, wc = 36 + m;
  if (j >= d.n) return;
  KSP_TSB(1, 112);
  const int l = j - 1, r = j + 1;
  const double* Ul = d.U0 + (size_t)l * NB * NB;
  const double* Uj = d.U0 + (size_t)j * NB * NB;
  const double* Rj = d.R0 + (size_t)j * NB * m;
  const double* Dj = d.D0 + (size_t)j * NB * NB;
  const double lam2 = d.sc[SC_LAM2];
  const bool hr = r < d.n;
  const int nth = blockDim.x;
  // D_j | U_{j-1} | U_j | R_j as four segments, written as L and W = [U_{j-1}^T | U_j | R_j]
  double vd[2], vul[2], vuj[2], vr[3];
  seg_ld(vd, Dj, NB * NB, tid, nth);
  seg_ld(vul, Ul, NB * NB, tid, nth);
  seg_ld(vuj, Uj, NB * NB, tid, nth);
  seg_ld(vr, Rj, NB * m, tid, nth);
  seg_st(vd, Dj, NB * NB, tid, nth, [&](int q, double v) { L[q] = v + lam_diag(d, j, q, lam2); });
  seg_st(vul, Ul, NB * NB, tid, nth, [&](int q, double v) { W[(q % NB) * wc + q / NB] = v; });
  seg_st(vuj, Uj, NB * NB, tid, nth, [&](int q, double v) { W[(q / NB) * wc + NB + q % NB] = hr ? v : 0.0; });
  const float rinv = 1.0f / (float)m;
  seg_st(vr, Rj, NB * m, tid, nth, [&](int q, double v) {
    const int r = div_small(q, rinv);
    W[r * wc + 2 * NB + (q - r * m)] = v;
  });
  __syncthreads();
  KSP_TSB(1, 113);
  if (tid < 64) {
    const bool ok = chol18_wave(L, id, tid);
    if (!ok && tid == 0) d.sc[SC_OK] = 0.0;
  }
  __syncthreads();
  KSP_TSB(1, 114);
  // the L loads kept per row: the hoisted form held all 171 entries (256 VGPRs + 188 AGPRs, one block per CU, the
  // 500 blocks in two rounds); lean: 114 VGPRs, every block resident at once.  Same arithmetic, same bits.
  node_forward_lean(L, id, W, wc, wc, d.Z + (size_t)j * NB * wc, wc, tid);
  for (int q = tid; q < NB * NB; q += blockDim.x) d.Lf[(size_t)j * NB * NB + q] = L[q];
  if (tid < NB) d.Lid[(size_t)j * NB + tid] = id[tid];
  KSP_TSB(1, 115);
}

// the absorption products of level_step on f64 MFMA tiles (round 5; the scalar loops before read 72 LDS operands per
// entry and took 4.5 us of a 12 us level).  With P_l = Zl_U^T Zl and P_r = Zr_Uin^T Zr (18 x wc each):
//   D' = D - P_l[:, U] - P_r[:, Uin],  R' = R - P_l[:, R] - P_r[:, R]   (both sides: 8 tiles over [D | R], 2 x 4)
//   Ui = -P_l[:, Uin]^T                                                  (left only: 4 tiles, 2 x 2)
//   Uo = -P_r[:, U]                                                      (right only: 4 tiles, 2 x 2)
// K = 18 in five steps of 4 per side.  The tile kind is wave-uniform and no operand is masked but the k >= 18 rows of
// the last step: rows >= 18 and columns past a part's end read valid LDS (the Z tiles run on into the next buffer) and
// their outputs are not stored.  ~100 instructions per tile instead of ~400 with per-lane part selects and masks.
// Ui^T and Uo go straight into W's first 36 columns (the forward solve's [Ui^T | Uo | R']).  With chol (4 waves only) the
// four tiles holding D' (tj = 0, 1 of kind 0) come first, on waves 0 and 1; wave 1 then raises *dflag and wave 0, once
// it sees it, factors D' (chol18_wave) while waves 1..3 finish the other tiles, none of which touches L.
__device__ __forceinline__ void level_products(const SpDev& d, const double* Zl, const double* Zr, double* L, double* id,
                                               double* W, int m, int wc, int tid, int nth, int tsb, bool chol,
                                               int* dflag) {
  // the wave index as a scalar: tile indices and kinds are wave-uniform (scalar branches, no exec masking)
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, nw = nth >> 6, i16 = lane & 15, kq = lane >> 4;
  const int ncb = (NB + m + 15) >> 4;  // column tiles of [D | R]
  const int nt = 2 * ncb + 8;
  const bool k4 = 16 + kq < NB;  // the last k step's rows 16 + kq exist
  int ko[5];                     // the lane's Z row offsets of the five k steps
#pragma unroll
  for (int st = 0; st < 5; ++st) ko[st] = min(4 * st + kq, NB - 1) * wc;
  __shared__ double junk[64];    // the stores of rows / columns outside a part land here (no branch per store)
  KSP_TSB(tsb, 240);
  // chol: D' tiles (ti, tj) = (0,0), (1,0) on wave 0 and (0,1), (1,1) on wave 1 (order slots 0..3), the rest (slots
  // 4..nt-1) round-robin over waves 1..3; otherwise slot = t round-robin over all waves
  const bool ord = chol && nw == 4;
  const int first = ord ? (wave == 0 ? 0 : wave == 1 ? 2 : 3 + wave) : wave;
  int step = ord ? (wave <= 1 ? 1 : 3) : nw;
  for (int slot = first;; slot += step) {
    if (ord) {
      if (wave == 0 && slot == 2) {  // both D' tiles of wave 0 stored: wait for wave 1's, then factor
        while (__hip_atomic_load(dflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
        const bool ok = chol18_wave(L, id, lane);
        if (!ok && lane == 0) d.sc[SC_OK] = 0.0;
        break;
      }
      if (wave == 1 && slot == 4) {  // wave 1's D' tiles stored: release them to wave 0, then slots 4, 7, 10, ..
        __hip_atomic_store(dflag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        step = 3;
      }
    }
    if (slot >= nt) break;
    // slot -> tile: with ord, slots 0..3 are the D' tiles and 4.. the others in the plain order without them
    int t = slot;
    if (ord) {
      if (slot < 4) {
        t = (slot & 1) * ncb + (slot >> 1);  // (ti, tj) = (slot & 1, slot >> 1)
      } else {
        const int o = slot - 4;  // the non-D' tiles: kind 0 with tj >= 2 (2 (ncb - 2) of them), then kinds 1 and 2
        const int n0 = ncb - 2;
        t = o < 2 * n0 ? (o / n0) * ncb + 2 + o % n0 : 2 * ncb + o - 2 * n0;
      }
    }
    int kind, ti, tj;
    if (t < 2 * ncb) {
      kind = 0, ti = t / ncb, tj = t % ncb;
    } else {
      const int u = t - 2 * ncb;
      kind = 1 + (u >> 2), ti = (u >> 1) & 1, tj = u & 1;
    }
    const int r = 16 * ti + i16, c = 16 * tj + i16;  // the lane's A row and B column within the tile's part
    // column offsets in a Z row: kind 0: [D | R] column c -> U / Uin + c, then R; kind 1 (Ui, left): Uin + c;
    // kind 2 (Uo, right): U + c
    const int cl = kind == 0 ? (c < NB ? NB + c : 2 * NB + c - NB) : c;
    const int cr = kind == 0 ? (c < NB ? c : 2 * NB + c - NB) : NB + c;
    double al[5], bl[5], ar[5], br[5];
#pragma unroll
    for (int st = 0; st < 5; ++st) {
      al[st] = Zl[ko[st] + NB + r];
      bl[st] = Zl[ko[st] + cl];
      ar[st] = Zr[ko[st] + r];
      br[st] = Zr[ko[st] + cr];
    }
    al[4] = k4 ? al[4] : 0.0;
    ar[4] = k4 ? ar[4] : 0.0;
    __builtin_amdgcn_sched_barrier(0);
    v4d_t accl = {0.0, 0.0, 0.0, 0.0}, accr = {0.0, 0.0, 0.0, 0.0};
    if (kind != 2) {
#pragma unroll
      for (int st = 0; st < 5; ++st) accl = __builtin_amdgcn_mfma_f64_16x16x4f64(al[st], bl[st], accl, 0, 0, 0);
    }
    if (kind != 1) {
#pragma unroll
      for (int st = 0; st < 5; ++st) accr = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[st], br[st], accr, 0, 0, 0);
    }
    const v4d_t acc = accl + accr;
    // output column c of this lane, rows 16 ti + kq + 4 rr: the destination by selects, the store unconditional
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * ti + kq + 4 * rr;
      const bool rv = row < NB;
      double* dst = junk + lane;
      if (kind == 0) {
        dst = (rv && c < NB) ? L + row * NB + c : (rv && c < NB + m) ? W + row * wc + NB + c : dst;
        *dst = *dst - acc[rr];
      } else {
        // W[row][c] = Ui^T[row][c] = Ui[c][row]; W[row][NB + c] = Uo[row][c]
        dst = (rv && c < NB) ? W + row * wc + (kind == 1 ? 0 : NB) + c : dst;
        *dst = -acc[rr];
      }
    }
  }
}

// fused level: node i (i % 2s == 0) absorbs its level-s eliminated neighbours i -+ s, then either is
// eliminated at level 2s (Cholesky + Z_i with the couplings to i -+ 2s it computes itself), stays for the next
// level, or -- node 0 once no partner is left -- solves X_0 = D_0^-1 R_0.
// level_step: one node's share, by the `nth` threads of a node group (tid = the thread's index in the group); every
// thread of the block calls it (act: the group has a node at this level), with the same three block barriers on every
// path, so that k_sp_deep can run several groups (and several levels) in one block.  L, id and sm (Zl | Zr | W,
// [18][wc] each) are the group's LDS (the couplings Ui, Uo are formed in W, the forward solve's operand).
// LEAN: k_sp_deep's 1024-thread block (128 VGPRs): fewer loads in flight, per-row forward solve.  LF: only the solves
// with per-row L loads (the first level's 501 blocks: 132 VGPRs, all resident at once, 22.7 -> 16.5 us; the hoisted
// solves are ~2 us faster on the narrower levels, whose blocks fit in one round anyway).  Same arithmetic, same bits.
template <bool LEAN, bool LF = LEAN>
__device__ __forceinline__ void level_step(const SpDev& d, int s, int i, bool act, int tid, int nth, double* L,
                                           double* id, double* sm) {
  const int m = d.m, wc = 36 + m;
  const int jl = i - s, jr = i + s;
  const bool hl = jl >= 0, hr = jr < d.n;
  const bool elim = (i % (4 * s)) == 2 * s;  // eliminated at level 2s
  const bool top = (i == 0) && (2 * s >= d.n);
  double* Zl = sm;
  double* Zr = Zl + NB * wc;
  double* W = Zr + NB * wc;  // [Ui^T | Uo | R']
  // diagnostics: block 1 of the level (block 0 once it is alone), slots 120 + 6 lv + k (tools/diag_sp_levels.py)
  const int tsb = gridDim.x > 1 ? 1 : 0, tsl = 120 + 6 * (31 - __clz(s));
  if (!LEAN) KSP_TSB(tsb, tsl);
  const bool fin = act && (elim || top);
  __shared__ int dflag;  // level_products: wave 1's D' tiles stored (reset before the first barrier)
  if (tid == 0) dflag = 0;
  if (act) {
    // Zl | Zr | D_i (into L) | R_i (into W's R columns) in one batch of loads; absent neighbours read node i's Z
    // slot (any valid address) and store zeros
    const double* Zsl = d.Z + (size_t)(hl ? jl : i) * NB * wc;
    const double* Zsr = d.Z + (size_t)(hr ? jr : i) * NB * wc;
    const double* Di = (s == 1 ? d.D0 : d.D) + (size_t)i * NB * NB;
    const double* Ri = (s == 1 ? d.R0 : d.R) + (size_t)i * NB * m;
    const double lam2 = s == 1 ? d.sc[SC_LAM2] : 0.0;
    const int nz = NB * wc;
    constexpr int UZ = LEAN ? 3 : 6, UD = LEAN ? 3 : 2, UR = LEAN ? 3 : 3;
    double vl[UZ], vr[UZ], vd[UD], vq[UR];
    seg_ld(vl, Zsl, nz, tid, nth);
    seg_ld(vr, Zsr, nz, tid, nth);
    seg_ld(vd, Di, NB * NB, tid, nth);
    seg_ld(vq, Ri, NB * m, tid, nth);
    seg_st(vl, Zsl, nz, tid, nth, [&](int q, double v) { Zl[q] = hl ? v : 0.0; });
    seg_st(vr, Zsr, nz, tid, nth, [&](int q, double v) { Zr[q] = hr ? v : 0.0; });
    seg_st(vd, Di, NB * NB, tid, nth, [&](int q, double v) { L[q] = v + lam_diag(d, i, q, lam2); });
    const float rinv = 1.0f / (float)m;
    seg_st(vq, Ri, NB * m, tid, nth, [&](int q, double v) {
      const int r = div_small(q, rinv);
      W[r * wc + 2 * NB + (q - r * m)] = v;
    });
  }
  __syncthreads();
  KSP_STOP(1);
  if (!LEAN) KSP_TSB(tsb, tsl + 1);
  // (4-wave groups: a finishing node's Cholesky inside, on wave 0, behind its D' tiles)
  const bool early = !LEAN && fin && nth == 256;
  if (act) level_products(d, Zl, Zr, L, id, W, m, wc, tid, nth, LEAN ? -1 : tsb, early, &dflag);
  __syncthreads();
  KSP_STOP(2);
  if (!LEAN) KSP_TSB(tsb, tsl + 2);
  if (act && !fin) {  // stays active: D', R' for the next level (the coupling is recomputed from Z by both nodes)
    for (int q = tid; q < NB * NB; q += nth) d.D[(size_t)i * NB * NB + q] = L[q];
    for (int q = tid; q < NB * m; q += nth) d.R[(size_t)i * NB * m + q] = W[(q / m) * wc + 2 * NB + q % m];
  }
  if (LEAN || !early) {  // the Cholesky after the products (k_sp_deep's groups: the same barriers on every path)
    if (fin && tid < 64) {
      const bool ok = chol18_wave(L, id, tid);
      if (!ok && tid == 0) d.sc[SC_OK] = 0.0;
    }
    __syncthreads();
  }
  KSP_STOP(3);
  if (!LEAN) KSP_TSB(tsb, tsl + 3);
  if (fin && top && d.zs) {  // Z_R,0 = L^-1 R' and the factor: the back substitution solves x_0 with one column later
    if (LF) node_forward_lean(L, id, W + 2 * NB, wc, m, d.Z + 2 * NB, wc, tid, nth);
    else node_forward(L, id, W + 2 * NB, wc, m, d.Z + 2 * NB, wc, tid, nth);
    for (int q = tid; q < NB * NB; q += nth) d.Lf[q] = L[q];
    if (tid < NB) d.Lid[tid] = id[tid];
  } else if (fin && top) {  // X_0 = L^-T L^-1 R' (forward in place in W, then backward into X_0)
    if (LF) {
      node_forward_lean(L, id, W + 2 * NB, wc, m, W + 2 * NB, wc, tid, nth);
      node_backsolve_lean(L, id, W + 2 * NB, wc, m, d.X, tid, nth);
    } else {
      node_forward(L, id, W + 2 * NB, wc, m, W + 2 * NB, wc, tid, nth);
      node_backsolve(L, id, W + 2 * NB, wc, m, d.X, tid, nth);
    }
  } else if (fin) {
    if (LF) node_forward_lean(L, id, W, wc, wc, d.Z + (size_t)i * NB * wc, wc, tid, nth);
    else node_forward(L, id, W, wc, wc, d.Z + (size_t)i * NB * wc, wc, tid, nth);
    KSP_STOP(4);
    for (int q = tid; q < NB * NB; q += nth) d.Lf[(size_t)i * NB * NB + q] = L[q];
    if (tid < NB) d.Lid[(size_t)i * NB + tid] = id[tid];
  }
  if (!LEAN) KSP_TSB(tsb, tsl + 4);
}

__device__ __forceinline__ void zschur_block(const SpDev& d, int blk, double* sm);

template <bool LF>
__global__ void __launch_bounds__(256) k_sp_level(SpDev d, int s) {
  __shared__ double L[NB * NB];
  __shared__ double id[NB];
  extern __shared__ __attribute__((aligned(16))) double sm[];  // Zl [18][wc] | Zr [18][wc] | W [18][wc]
  const int nlb = (d.n + 2 * s - 1) / (2 * s);
  if ((int)blockIdx.x >= nlb) {  // zsf, top level: the Schur sums of nodes 1.. (all final by now) beside the top node
    zschur_block(d, (int)blockIdx.x - nlb, sm);
    return;
  }
  const int i = 2 * s * blockIdx.x;
  if (i >= d.n) return;  // block-uniform
  level_step<false, LF>(d, s, i, true, threadIdx.x, blockDim.x, L, id, sm);
}

__global__ void __launch_bounds__(256) k_sp_top(SpDev d) {
  __shared__ double L[NB * NB];
  __shared__ double id[NB];
  extern __shared__ __attribute__((aligned(16))) double T[];  // [18][m]
  const int tid = threadIdx.x, m = d.m;
  const double lam2 = d.sc[SC_LAM2];
  for (int q = tid; q < NB * NB; q += blockDim.x) L[q] = d.D0[q] + lam_diag(d, 0, q, lam2);
  for (int q = tid; q < NB * m; q += blockDim.x) T[q] = d.R0[q];
  __syncthreads();
  if (tid < 64) {
    const bool ok = chol18_wave(L, id, tid);
    if (!ok && tid == 0) d.sc[SC_OK] = 0.0;
  }
  __syncthreads();
  if (d.zs) {  // Z_R,0 and the factor (see level_step)
    node_forward(L, id, T, m, m, d.Z + 2 * NB, 36 + m, tid);
    for (int q = tid; q < NB * NB; q += blockDim.x) d.Lf[q] = L[q];
    if (tid < NB) d.Lid[tid] = id[tid];
    return;
  }
  node_forward(L, id, T, m, m, T, m, tid);
  node_backsolve(L, id, T, m, m, d.X, tid);
}

// T = Z_R - Z_Uin x_l - Z_U x_r of one node on MFMA tiles (the node group's nth threads): T[row][c] = Z_R[row][c] -
// sum_k (Z[row][k] xl[k][c] + Z[row][NB + k] xr[k][c]); A = Z^T is read from the Z rows (stride 1 in k), B from xl / xr
__device__ __forceinline__ void back_T(const double* Z, const double* xl, const double* xr, double* T, int m, int wc,
                                       int tid, int nth) {
  const int wave = tid >> 6, lane = tid & 63, nw = nth >> 6, nct = (m + 15) >> 4;
  for (int t = wave; t < 2 * nct; t += nw) {
    const int ti = t / nct, tj = t % nct, i = lane & 15;
    const int rc = min(16 * ti + i, NB - 1), cc = min(16 * tj + i, m - 1);
    const bool rv = 16 * ti + i < NB, cv = 16 * tj + i < m;
    // operands first (see level_products), the two sides in two accumulator chains
    double av[2][5], bv[2][5];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double* B = h ? xr : xl;
#pragma unroll
      for (int st = 0; st < 5; ++st) {
        const int kc = min(4 * st + (lane >> 4), NB - 1);
        av[h][st] = Z[rc * wc + h * NB + kc];
        bv[h][st] = B[kc * m + cc];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    v4d_t ac[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int st = 0; st < 5; ++st) {
      const bool kv = 4 * st + (lane >> 4) < NB;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        ac[h] = __builtin_amdgcn_mfma_f64_16x16x4f64((kv && rv) ? av[h][st] : 0.0, (kv && cv) ? bv[h][st] : 0.0, ac[h], 0, 0, 0);
    }
    const v4d_t acc = ac[0] + ac[1];
    const int c = 16 * tj + (lane & 15);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * ti + (lane >> 4) + 4 * rr;
      if (row < NB && c < m) T[row * m + c] = Z[row * wc + 2 * NB + c] - acc[rr];
    }
  }
}

// back_step: node j's back substitution by a node group (the contract of level_step: every thread of the block
// calls it, two block barriers on every path); L, id and sm (Z [18][wc] | xl | xr | T [18][m]) are the group's LDS
template <bool LEAN>
__device__ __forceinline__ void back_step(const SpDev& d, int s, int j, bool act, int tid, int nth, double* L,
                                          double* id, double* sm) {
  const int m = d.m, wc = 36 + m;
  const int l = j - s, r = j + s;
  const bool hr = r < d.n;
  double* Z = sm;
  double* xl = Z + NB * wc;
  double* xr = xl + NB * m;
  double* T = xr + NB * m;
  const int tsl = 190 + 4 * (31 - __clz(s));
  if (!LEAN) KSP_TSB(0, tsl);
  if (act) {
    // L_j | 1/diag | Z_j | x_l | x_r in one batch of loads (x_r of an absent neighbour: zeros)
    const double* Ls = d.Lf + (size_t)j * NB * NB;
    const double* Is = d.Lid + (size_t)j * NB;
    const double* Zs = d.Z + (size_t)j * NB * wc;
    const double* Xl = d.X + (size_t)l * NB * m;
    const double* Xr = d.X + (size_t)(hr ? r : l) * NB * m;
    constexpr int UL = 2, UZ = LEAN ? 3 : 6, UX = LEAN ? 3 : 3;
    double vL[UL], vI[1], vZ[UZ], vxl[UX], vxr[UX];
    seg_ld(vL, Ls, NB * NB, tid, nth);
    seg_ld(vI, Is, NB, tid, nth);
    seg_ld(vZ, Zs, NB * wc, tid, nth);
    seg_ld(vxl, Xl, NB * m, tid, nth);
    seg_ld(vxr, Xr, NB * m, tid, nth);
    seg_st(vL, Ls, NB * NB, tid, nth, [&](int q, double v) { L[q] = v; });
    seg_st(vI, Is, NB, tid, nth, [&](int q, double v) { id[q] = v; });
    seg_st(vZ, Zs, NB * wc, tid, nth, [&](int q, double v) { Z[q] = v; });
    seg_st(vxl, Xl, NB * m, tid, nth, [&](int q, double v) { xl[q] = v; });
    seg_st(vxr, Xr, NB * m, tid, nth, [&](int q, double v) { xr[q] = hr ? v : 0.0; });
  }
  __syncthreads();
  KSP_STOP(1);
  if (!LEAN) KSP_TSB(0, tsl + 1);
  if (act) back_T(Z, xl, xr, T, m, wc, tid, nth);
  __syncthreads();
  KSP_STOP(2);
  if (!LEAN) KSP_TSB(0, tsl + 2);
  if (act) {
    if (LEAN) node_backsolve_lean(L, id, T, m, m, d.X + (size_t)j * NB * m, tid, nth);
    else node_backsolve(L, id, T, m, m, d.X + (size_t)j * NB * m, tid, nth);
  }
  if (!LEAN) KSP_TSB(0, tsl + 3);
}

__global__ void __launch_bounds__(256) k_sp_back(SpDev d, int s) {
  __shared__ double L[NB * NB];
  __shared__ double id[NB];
  extern __shared__ __attribute__((aligned(16))) double sm[];  // Z [18][wc] | xl [18][m] | xr [18][m] | T [18][m]
  const int j = s + 2 * s * blockIdx.x;
  if (j >= d.n) return;  // block-uniform
  back_step<false>(d, s, j, true, threadIdx.x, blockDim.x, L, id, sm);
}

// two back-substitution levels in one launch (round 5): strides 2s and s.  Block b takes node j = s + 2sb of stride s.
// Of its neighbours j -+ s (multiples of 2s) the odd multiple of 2s, k, belongs to stride 2s: the block solves it first
// (x_{k -+ 2s} are known), then j from x_k (in LDS) and its other neighbour o.  x_k is solved by the blocks on both
// sides of it from the same operands by the same instructions, so both copies are bitwise equal; the block with
// k = j + s stores it (node k - s always exists).  One launch, one batch of operand loads and one launch gap instead
// of two; every value is computed as by two k_sp_back launches.
__global__ void __launch_bounds__(256) k_sp_back2(SpDev d, int s) {
  __shared__ double L[2][NB * NB];
  __shared__ double id[2][NB];
  // node k: Zk [18][wc] | xa | xb [18][m]; node j: Zj [18][wc] | xjl | xjr [18][m]; T [18][m]
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int b = blockIdx.x, j = s + 2 * s * b, tid = threadIdx.x, nth = blockDim.x;
  if (j >= d.n) return;  // block-uniform
  const int tsl = 190 + 4 * (31 - __clz(s));  // diagnostics: the stride-s slots (x_k done in place of T)
  KSP_TSB(0, tsl);
  const int m = d.m, wc = 36 + m, n = d.n;
  const bool kl = (b & 1) != 0;  // k = j - s (b odd) or k = j + s (b even)
  const int k = kl ? j - s : j + s, o = kl ? j + s : j - s;
  const bool hk = k < n, ho = o < n, hkb = k + 2 * s < n;
  double* Zk = sm;
  double* xa = Zk + NB * wc;
  double* xb = xa + NB * m;
  double* Zj = xb + NB * m;
  double* xjl = Zj + NB * wc;
  double* xjr = xjl + NB * m;
  double* T = xjr + NB * m;
  double* xk = kl ? xjl : xjr;  // x_k among node j's operands
  double* xo = kl ? xjr : xjl;
  {
    // L_k | 1/diag_k | Z_k | x_{k-2s} | x_{k+2s} | L_j | 1/diag_j | Z_j | x_o in one batch (absent nodes: zeros; their
    // loads read node j's slots)
    const int kc = hk ? k : j;
    const double* Lks = d.Lf + (size_t)kc * NB * NB;
    const double* Iks = d.Lid + (size_t)kc * NB;
    const double* Zks = d.Z + (size_t)kc * NB * wc;
    const double* Xas = d.X + (size_t)(hk ? k - 2 * s : j - s) * NB * m;
    const double* Xbs = d.X + (size_t)(hkb ? k + 2 * s : j - s) * NB * m;
    const double* Ljs = d.Lf + (size_t)j * NB * NB;
    const double* Ijs = d.Lid + (size_t)j * NB;
    const double* Zjs = d.Z + (size_t)j * NB * wc;
    const double* Xos = d.X + (size_t)(ho ? o : j - s) * NB * m;
    if (!hk)
      for (int q = tid; q < NB * m; q += nth) xk[q] = 0.0;
    double vLk[2], vIk[1], vZk[6], vxa[3], vxb[3], vLj[2], vIj[1], vZj[6], vxo[3];
    seg_ld(vLk, Lks, NB * NB, tid, nth);
    seg_ld(vIk, Iks, NB, tid, nth);
    seg_ld(vZk, Zks, NB * wc, tid, nth);
    seg_ld(vxa, Xas, NB * m, tid, nth);
    seg_ld(vxb, Xbs, NB * m, tid, nth);
    seg_ld(vLj, Ljs, NB * NB, tid, nth);
    seg_ld(vIj, Ijs, NB, tid, nth);
    seg_ld(vZj, Zjs, NB * wc, tid, nth);
    seg_ld(vxo, Xos, NB * m, tid, nth);
    seg_st(vLk, Lks, NB * NB, tid, nth, [&](int q, double v) { L[0][q] = v; });
    seg_st(vIk, Iks, NB, tid, nth, [&](int q, double v) { id[0][q] = v; });
    seg_st(vZk, Zks, NB * wc, tid, nth, [&](int q, double v) { Zk[q] = v; });
    seg_st(vxa, Xas, NB * m, tid, nth, [&](int q, double v) { xa[q] = v; });
    seg_st(vxb, Xbs, NB * m, tid, nth, [&](int q, double v) { xb[q] = hkb ? v : 0.0; });
    seg_st(vLj, Ljs, NB * NB, tid, nth, [&](int q, double v) { L[1][q] = v; });
    seg_st(vIj, Ijs, NB, tid, nth, [&](int q, double v) { id[1][q] = v; });
    seg_st(vZj, Zjs, NB * wc, tid, nth, [&](int q, double v) { Zj[q] = v; });
    seg_st(vxo, Xos, NB * m, tid, nth, [&](int q, double v) { xo[q] = ho ? v : 0.0; });
  }
  __syncthreads();
  KSP_TSB(0, tsl + 1);
  if (hk) back_T(Zk, xa, xb, T, m, wc, tid, nth);  // block-uniform branches
  __syncthreads();
  if (hk) node_backsolve(L[0], id[0], T, m, m, xk, tid, nth);
  __syncthreads();
  KSP_TSB(0, tsl + 2);
  if (hk && !kl)
    for (int q = tid; q < NB * m; q += nth) d.X[(size_t)k * NB * m + q] = xk[q];
  back_T(Zj, xjl, xjr, T, m, wc, tid, nth);
  __syncthreads();
  node_backsolve(L[1], id[1], T, m, m, d.X + (size_t)j * NB * m, tid, nth);
  KSP_TSB(0, tsl + 3);
}

// the deep levels in one block (round 4): once a level has at most kSpDeepGroups nodes, the remaining levels down to
// the top and back up to the same stride run in one block of kSpDeepGroups node groups of kSpDeepGT threads, a block
// barrier between levels instead of a kernel boundary (the L2 writeback and the launch of every level, and the
// operands come back from the CU's own cache).  Levels s_deep .. top, then the back substitution top .. s_deep.
constexpr int kSpDeepGroups = 4;
// LDS of one k_sp_deep node group, in doubles: L | id | Zl | Zr | W ([18][36 + m] each)
__host__ __device__ constexpr int kSpDeepPer(int m) { return NB * NB + NB + 3 * NB * (36 + m); }
constexpr int kSpDeepGT = 128;  // threads per node group: the block keeps the per-level kernels' 256-VGPR budget
__global__ void __launch_bounds__(kSpDeepGT * kSpDeepGroups) k_sp_deep(SpDev d, int s_deep) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  // wave-uniform group index: the per-node branches (active, eliminated, top) are scalar branches
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x / kSpDeepGT), tid = threadIdx.x % kSpDeepGT;
  // the group size as an opaque value, as blockDim.x is in k_sp_level / k_sp_back: a compile-time stride lets the
  // compiler unroll the strided output loops and hoist their operands (hundreds of spilled VGPRs)
  int nth = kSpDeepGT;
  asm volatile("" : "+s"(nth));
  const int wc = 36 + d.m, per = kSpDeepPer(d.m);  // the group's LDS: L | id | Zl | Zr | W
  double* L = sm + (size_t)g * per;
  double* id = L + NB * NB;
  double* gsm = id + NB;
  int s = s_deep;
  for (;; s *= 2) {
    const int i = 2 * s * g;
    level_step<true>(d, s, i, i < d.n, tid, nth, L, id, gsm);
    __syncthreads();  // this level's D / U / R / Z / X stores before the next level's loads
    if (2 * s >= d.n) break;
  }
  for (; s >= s_deep; s /= 2) {
    const int j = s + 2 * s * g;
    back_step<true>(d, s, j, j < d.n, tid, nth, L, id, gsm);
    __syncthreads();
  }
}

// ---------------------------------------------------------------- partitioned band solve (default)
// The block-tridiagonal coefficient system solved by nested partitioning instead of cyclic reduction: the nodes of
// a level are cut into chunks of q consecutive nodes whose last node is the chunk's separator.  One block per chunk
// eliminates the chunk's interior nodes in order (block Thomas: Cholesky of the node, Z = L^-1 [U_j | F_j | R_j],
// the next node's D, its fill coupling F to the left separator and its right-hand side updated by Z_U^T Z), which
// leaves a block-tridiagonal system over the separators (level l + 1: P = ceil(n / q) nodes).  The levels repeat
// until at most kSpTop nodes remain; one block solves that system by the same elimination and a back-substitution
// sweep, and the back kernels walk the levels down again (x_j = L_j^-T (Z_R - Z_U x_{j+1} - Z_F x_sepL)).
//   configs[4]: n = 1001 -> 63 (q = 16) -> 8 (q = 8) -> top: 5 launches whose dependent chain is 15 + 7 + 8
//   eliminations and 8 + 7 + 15 substitution steps, instead of 21 launches of one cyclic-reduction level each.
// Level l's system: D_i = Dt_i + Dh_i (the separator's own chunk / the next chunk's elimination; Dh of the last
// node is absent), U_i (block (i, i + 1)), R_i = Rt_i + Rh_i.  Level 0 reads the built blocks D0 + lambda^2 I, U0, R0.
constexpr int kSpTop = 16;  // largest system the one-block top kernel solves
constexpr int kSpWc = 36 + MAXC + 1;  // LDS row stride of [U | F | R] (m <= MAXC + 1)

struct SpLvl {
  int n, q, lvl;                          // nodes, chunk length (interior nodes + the separator), level
  const double *Dt, *Dh, *U, *Rt, *Rh;    // this level's system (lvl 0: D0, -, U0, R0, -)
  double *Lf, *Lid, *Z, *X;               // factors [n][324], [n][18], [n][18][36 + m]; solution [n][18][m]
  double *nDt, *nDh, *nU, *nRt, *nRh;     // chunk kernel: the next level's system
  const double* Xup;                      // back kernel: the next level's solution
};

// raw entry e of node i's [D (324) | U (324) | R (18 m)] at level L
__device__ __forceinline__ double lvl_raw(const SpDev& d, const SpLvl& L, int i, int e, double lam2) {
  const int m = d.m;
  const bool nx = i + 1 < L.n;
  if (e < NB * NB) {
    const size_t o = (size_t)i * NB * NB + e;
    return L.lvl == 0 ? L.Dt[o] + lam_diag(d, i, e, lam2) : L.Dt[o] + (nx ? L.Dh[o] : 0.0);
  }
  if (e < 2 * NB * NB) return L.U[(size_t)i * NB * NB + e - NB * NB];
  const size_t o = (size_t)i * NB * m + e - 2 * NB * NB;
  return L.lvl == 0 ? L.Rt[o] : L.Rt[o] + (nx ? L.Rh[o] : 0.0);
}

constexpr int kSpRawU = (2 * NB * NB + NB * (MAXC + 1) + 255) / 256;  // raw items per thread (256 threads)

// the node update of chunk_forward on f64 MFMA tiles (see there); U tiles: rows = the 18 Z_U columns, columns =
// [U | F | R] (D~, F, R~ of the next node); F tiles (hasL): rows = the Z_F columns, columns = [F | R] (Dh, Rh)
__device__ __forceinline__ void chunk_update_mfma(const double* Zs, int wc, int m, const double* Raw, double* Lc,
                                                  double* W, double* Dh, double* Rh, bool hasL, int tid) {
  const int wave = tid >> 6, lane = tid & 63, li = lane & 15, kq = lane >> 4;
  const int nct_u = (36 + m + 15) >> 4, nct_f = (NB + m + 15) >> 4;
  const int nt_u = 2 * nct_u, nt = nt_u + (hasL ? 2 * nct_f : 0);
  for (int t = wave; t < nt; t += 4) {
    const bool fu = t >= nt_u;
    const int tt = fu ? t - nt_u : t, nct = fu ? nct_f : nct_u;
    const int ti = tt / nct, tj = tt - ti * nct;
    const int ca = fu ? NB : 0, ncb = fu ? NB + m : 36 + m;
    const int arc = min(16 * ti + li, NB - 1), bcc = min(16 * tj + li, ncb - 1);
    v4d_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int st = 0; st < 5; ++st) {
      const int k = 4 * st + kq, kc = min(k, NB - 1);
      const double av = Zs[kc * wc + ca + arc], bv = Zs[kc * wc + ca + bcc];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(k < NB ? av : 0.0, bv, acc, 0, 0, 0);
    }
    const int c = 16 * tj + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = 16 * ti + kq + 4 * r;
      if (a < NB && c < ncb) {
        const double val = acc[r];
        if (!fu) {
          if (c < NB) Lc[a * NB + c] = Raw[a * NB + c] - val;
          else if (c < 2 * NB) W[a * wc + c] = -val;
          else W[a * wc + c] = Raw[2 * NB * NB + a * m + c - 2 * NB] - val;
        } else {
          if (c < NB) Dh[a * NB + c] -= val;
          else Rh[a * m + c - NB] -= val;
        }
      }
    }
  }
  for (int q = tid; q < NB * NB; q += 256) W[(q / NB) * wc + q % NB] = Raw[NB * NB + q];  // U of node j + 1: raw
}

// forward elimination of nodes a .. e - 1 of one chunk (e = its separator; sepL = a - 1 when hasL) by one 256-thread
// block.  On return Lc holds D~_e (whole), W = [U_e raw | F_e | R~_e], Dh / Rh the left separator's accumulated
// updates (hasL).  Writes L_j, 1/diag, Z_j of every interior node.  Returns false if a node block is not PD.
__device__ bool chunk_forward(const SpDev& d, const SpLvl& L, int a, int e, bool hasL, double lam2, double* Lc,
                              double* idc, double* W, double* Zs, double* Dh, double* Rh, double* Raw) {
  const int tid = threadIdx.x, m = d.m, wc = 36 + m, nraw = 2 * NB * NB + NB * m;
  bool ok = true;
  // node a: D -> Lc, U -> W[:, 0:18], U_{a-1}^T -> W[:, 18:36] (block (a, a-1)), R -> W[:, 36:]
  double v[kSpRawU];
#pragma unroll
  for (int u = 0; u < kSpRawU; ++u) v[u] = lvl_raw(d, L, a, min(tid + 256 * u, nraw - 1), lam2);
  double fl[2];
  const int ua = hasL ? a - 1 : a;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = min(tid + 256 * u, NB * NB - 1), r = q / NB, c = q % NB;
    fl[u] = L.U[(size_t)ua * NB * NB + c * NB + r];
  }
#pragma unroll
  for (int u = 0; u < kSpRawU; ++u) {
    const int q = tid + 256 * u;
    if (q < NB * NB) Lc[q] = v[u];
    else if (q < 2 * NB * NB) W[((q - NB * NB) / NB) * wc + (q - NB * NB) % NB] = v[u];
    else if (q < nraw) W[((q - 2 * NB * NB) / m) * wc + 36 + (q - 2 * NB * NB) % m] = v[u];
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = tid + 256 * u;
    if (q < NB * NB) W[(q / NB) * wc + NB + q % NB] = hasL ? fl[u] : 0.0;
  }
  for (int q = tid; q < NB * NB + NB * m; q += 256) {
    if (q < NB * NB) Dh[q] = 0.0;
    else Rh[q - NB * NB] = 0.0;
  }
  // node a + 1's raw blocks in flight
#pragma unroll
  for (int u = 0; u < kSpRawU; ++u) v[u] = lvl_raw(d, L, min(a + 1, e), min(tid + 256 * u, nraw - 1), lam2);
  KSP_TS(100 + L.lvl);
  for (int j = a; j < e; ++j) {
    __syncthreads();  // Lc, W of node j complete; the previous update's Raw reads done
    const int ts = 4 * (j - a) + 64 * L.lvl;
    if (j - a < 12) KSP_TS(ts);
    // node j + 1's raw blocks to LDS (their loads went out during the previous step): no registers held across the
    // factorisation and the forward solve
#pragma unroll
    for (int u = 0; u < kSpRawU; ++u)
      if (tid + 256 * u < nraw) Raw[tid + 256 * u] = v[u];
    if (tid < 64) {
      const bool okj = chol18_wave(Lc, idc, tid);
      ok = ok && okj;
    }
    __syncthreads();
    if (j - a < 12) KSP_TS(ts + 1);
    node_forward_lean(Lc, idc, W, wc, wc, Zs, wc, tid);  // Z = L^-1 [U | F | R]
    double* Lg = L.Lf + (size_t)j * NB * NB;
    for (int q = tid; q < NB * NB; q += 256) Lg[q] = Lc[q];
    if (tid < NB) L.Lid[(size_t)j * NB + tid] = idc[tid];
    __syncthreads();  // Zs complete; Lc, W free
    if (j - a < 12) KSP_TS(ts + 2);
    // node j + 2's raw blocks in flight while node j + 1's are consumed
    const int jn = min(j + 2, e);
#pragma unroll
    for (int u = 0; u < kSpRawU; ++u) v[u] = lvl_raw(d, L, jn, min(tid + 256 * u, nraw - 1), lam2);
    double* Zg = L.Z + (size_t)j * NB * wc;
    for (int q = tid; q < NB * wc; q += 256) Zg[q] = Zs[q];
    // node j + 1: D~ = D - Z_U^T Z_U -> Lc, W = [U raw | -Z_U^T Z_F | R - Z_U^T Z_R]; the left separator (hasL):
    // Dh -= Z_F^T Z_F, Rh -= Z_F^T Z_R.  The Z^T products on f64 MFMA tiles (out[a][c] = sum_k Zs[k][ca + a]
    // Zs[k][cb + c], k < 18 in 5 steps of 4), tiles dealt round-robin to the 4 waves
    chunk_update_mfma(Zs, wc, m, Raw, Lc, W, Dh, Rh, hasL, tid);
    if (j - a < 12) KSP_TS(ts + 3);
  }
  if (a == e) {  // no interior node: the separator's raw blocks
#pragma unroll
    for (int u = 0; u < kSpRawU; ++u) {
      const int q = tid + 256 * u;
      if (q < NB * NB) Lc[q] = v[u];
      else if (q < 2 * NB * NB) W[((q - NB * NB) / NB) * wc + (q - NB * NB) % NB] = v[u];
      else if (q < nraw) W[((q - 2 * NB * NB) / m) * wc + 36 + (q - 2 * NB * NB) % m] = v[u];
    }
  }
  __syncthreads();
  return ok;
}

// one block per chunk of level L: eliminate the interior, write the separators' system for level L + 1
__global__ void __launch_bounds__(256) k_sp_chunk(SpDev d, SpLvl L) {
  __shared__ double Lc[NB * NB], idc[NB], Dh[NB * NB];
  __shared__ __attribute__((aligned(16))) double W[NB * kSpWc], Zs[NB * kSpWc], Rh[NB * (MAXC + 1)],
      Raw[2 * NB * NB + NB * (MAXC + 1)];
  const int p = blockIdx.x, tid = threadIdx.x, m = d.m, wc = 36 + m;
  const int a = p * L.q, e = min(L.n, a + L.q) - 1;
  const bool hasL = p > 0;
  const double lam2 = L.lvl == 0 ? d.sc[SC_LAM2] : 0.0;
  const bool ok = chunk_forward(d, L, a, e, hasL, lam2, Lc, idc, W, Zs, Dh, Rh, Raw);
  if (tid == 0 && !ok) d.sc[SC_OK] = 0.0;
  // separator p of level L + 1: Dt = D~_e, Rt = R~_e; the left separator: U_{p-1} = F_e^T, Dh_{p-1}, Rh_{p-1}
  for (int q = tid; q < NB * NB; q += 256) {
    L.nDt[(size_t)p * NB * NB + q] = Lc[q];
    if (hasL) {
      const int r = q / NB, c = q % NB;
      L.nU[(size_t)(p - 1) * NB * NB + q] = W[c * wc + NB + r];
      L.nDh[(size_t)(p - 1) * NB * NB + q] = Dh[q];
    }
  }
  for (int q = tid; q < NB * m; q += 256) {
    L.nRt[(size_t)p * NB * m + q] = W[(q / m) * wc + 36 + q % m];
    if (hasL) L.nRh[(size_t)(p - 1) * NB * m + q] = Rh[q];
  }
}

// x_j = L_j^-T (Z_R - Z_U x_{j+1} - Z_F xl) for j = e - 1 down to a, x_e given (LDS xs); the node operands of the
// next step in flight during each step.  X rows [18][m] of each node written to L.X.
__device__ void chunk_back(const SpDev& d, const SpLvl& L, int a, int e, bool hasL, double* Ls, double* ids,
                           double* Zs, double* xs, double* xl, double* T) {
  const int tid = threadIdx.x, m = d.m, wc = 36 + m, nop = NB * NB + NB + NB * wc;
  constexpr int U = (NB * NB + NB + NB * kSpWc + 255) / 256;
  double v[U];
  auto load = [&](int j) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = min(tid + 256 * u, nop - 1);
      v[u] = q < NB * NB ? L.Lf[(size_t)j * NB * NB + q]
             : q < NB * NB + NB ? L.Lid[(size_t)j * NB + q - NB * NB]
                                : L.Z[(size_t)j * NB * wc + q - NB * NB - NB];
    }
  };
  if (e > a) load(e - 1);
  KSP_TS(104 + L.lvl);
  for (int j = e - 1; j >= a; --j) {
    __syncthreads();  // xs = x_{j+1} complete; the previous step's Ls / Zs reads done
    const int tb = 200 + 3 * (e - 1 - j);
    if (L.lvl == 0 && e - 1 - j < 12) KSP_TS(tb);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = tid + 256 * u;
      if (q < NB * NB) Ls[q] = v[u];
      else if (q < NB * NB + NB) ids[q - NB * NB] = v[u];
      else if (q < nop) Zs[q - NB * NB - NB] = v[u];
    }
    if (j > a) load(j - 1);
    __syncthreads();
    {
      // T = Z_R - [Z_U | Z_F] [x_{j+1}; xl] on f64 MFMA tiles (K = 18, or 36 with the left separator)
      const int wave = tid >> 6, lane = tid & 63, li = lane & 15, kq = lane >> 4, nct = (m + 15) >> 4;
      const int nst = hasL ? 9 : 5;
      for (int t = wave; t < 2 * nct; t += 4) {
        const int ti = t / nct, tj = t - ti * nct;
        const int arc = min(16 * ti + li, NB - 1), bcc = min(16 * tj + li, m - 1);
        v4d_t acc = {0.0, 0.0, 0.0, 0.0};
        for (int st = 0; st < nst; ++st) {
          const int k = 4 * st + kq;
          const bool kv = hasL ? k < 2 * NB : k < NB;
          const int kc = min(k, 2 * NB - 1);
          const double av = Zs[arc * wc + kc];
          const double bv = kc < NB ? xs[kc * m + bcc] : xl[(kc - NB) * m + bcc];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(kv ? av : 0.0, bv, acc, 0, 0, 0);
        }
        const int c = 16 * tj + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = 16 * ti + kq + 4 * r;
          if (a < NB && c < m) T[a * m + c] = Zs[a * wc + 36 + c] - acc[r];
        }
      }
    }
    __syncthreads();
    if (L.lvl == 0 && e - 1 - j < 12) KSP_TS(tb + 1);
    node_backsolve(Ls, ids, T, m, m, xs, tid);  // x_j replaces x_{j+1}
    __syncthreads();
    if (L.lvl == 0 && e - 1 - j < 12) KSP_TS(tb + 2);
    double* Xg = L.X + (size_t)j * NB * m;
    for (int q = tid; q < NB * m; q += 256) Xg[q] = xs[q];
  }
}

// one block: the whole top-level system (n <= kSpTop) by elimination, the last node's solve and back-substitution
__global__ void __launch_bounds__(256) k_sp_ctop(SpDev d, SpLvl L) {
  __shared__ double Lc[NB * NB], idc[NB], Dh[NB * NB];
  __shared__ __attribute__((aligned(16))) double W[NB * kSpWc], Zs[NB * kSpWc], Rh[NB * (MAXC + 1)],
      Raw[2 * NB * NB + NB * (MAXC + 1)];
  double* T = Raw;  // the back-substitution's T (Raw is free once the elimination is done)
  const int tid = threadIdx.x, m = d.m, wc = 36 + m, e = L.n - 1;
  const double lam2 = L.lvl == 0 ? d.sc[SC_LAM2] : 0.0;
  bool ok = chunk_forward(d, L, 0, e, false, lam2, Lc, idc, W, Zs, Dh, Rh, Raw);
  if (tid < 64) {
    const bool okj = chol18_wave(Lc, idc, tid);
    ok = ok && okj;
  }
  if (tid == 0 && !ok) d.sc[SC_OK] = 0.0;
  __syncthreads();
  // x_e = L^-T L^-1 R~_e (forward in place in W's R columns, backward into Rh as the x_{j+1} buffer)
  node_forward_lean(Lc, idc, W + 36, wc, m, W + 36, wc, tid);
  __syncthreads();
  node_backsolve(Lc, idc, W + 36, wc, m, Rh, tid);
  __syncthreads();
  for (int q = tid; q < NB * m; q += 256) L.X[(size_t)e * NB * m + q] = Rh[q];
  chunk_back(d, L, 0, e, false, Lc, idc, Zs, Rh, W, T);
}

// one block per chunk of level L: x of the separator and the left separator from level L + 1, then the interior
__global__ void __launch_bounds__(256) k_sp_cback(SpDev d, SpLvl L) {
  __shared__ double Ls[NB * NB], ids[NB];
  __shared__ __attribute__((aligned(16))) double Zs[NB * kSpWc], xs[NB * (MAXC + 1)], xl[NB * (MAXC + 1)],
      T[NB * (MAXC + 1)];
  const int p = blockIdx.x, tid = threadIdx.x, m = d.m;
  const int a = p * L.q, e = min(L.n, a + L.q) - 1;
  const bool hasL = p > 0;
  for (int q = tid; q < NB * m; q += 256) {
    const double x = L.Xup[(size_t)p * NB * m + q];
    xs[q] = x;
    L.X[(size_t)e * NB * m + q] = x;
    xl[q] = hasL ? L.Xup[(size_t)(p - 1) * NB * m + q] : 0.0;
  }
  chunk_back(d, L, a, e, hasL, Ls, ids, Zs, xs, xl, T);
}

// ---------------------------------------------------------------- Schur complement onto theta
// partial rows of sum_i R0_i^T X_i over NPB nodes: upper C x C | C (the g column)
__global__ void __launch_bounds__(256) k_sp_schur(SpDev d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];  // R0 [18][m] | X [18][m]
  const int tid = threadIdx.x, m = d.m;
  double* Rl = sm;
  double* Xl = sm + NB * m;
  double* acc = Xl + NB * m;  // [Ws]
  short2* tab = (short2*)(acc + d.Ws);  // [Ws] (a, b) of the entries, read for every node
  for (int q = tid; q < d.Ws; q += blockDim.x) {
    acc[q] = 0.0;
    tab[q] = d.uab[q];
  }
  const int i0 = blockIdx.x * NPB, i1 = min(d.n, i0 + NPB);
  // node i + 1's R0 | X rows are loaded into registers while node i's products run (2 * 18 * m <= SCH_U * 256 for
  // m = C + 1 <= MAXC + 1; launched with 256 threads)
  constexpr int SCH_U = (2 * NB * (MAXC + 1) + 255) / 256;
  const int nq = 2 * NB * m;
  double v[SCH_U];
  auto load = [&](int i) {
    const double* R0 = d.R0 + (size_t)i * NB * m;
    const double* X = d.X + (size_t)i * NB * m;
#pragma unroll
    for (int u = 0; u < SCH_U; ++u) {
      const int q = min(tid + u * 256, nq - 1);
      v[u] = q < NB * m ? R0[q] : X[q - NB * m];
    }
  };
  if (i0 < i1) load(i0);
  for (int i = i0; i < i1; ++i) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SCH_U; ++u) {
      const int q = tid + u * 256;
      if (q < NB * m)
        Rl[q] = v[u];
      else if (q < nq)
        Xl[q - NB * m] = v[u];
    }
    __syncthreads();
    if (i + 1 < i1) load(i + 1);
    for (int q = tid; q < d.Ws; q += blockDim.x) {
      const short2 ab = tab[q];
      const int a = ab.x, b = ab.y;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NB; ++k) s += Rl[k * m + a] * Xl[k * m + b];
      acc[q] += s;
    }
  }
  __syncthreads();
  for (int q = tid; q < d.Ws; q += blockDim.x) d.spart[(size_t)blockIdx.x * d.Ws + q] = acc[q];
}

// zs: the camera-block partial sums of sum_i Z_R,i^T Z_R,i (Z_R,i = L_i^-1 R_i', the right-hand-side part of node i's
// elimination at any level, the top node's included) = R0^T D^-1 R0 of k_sp_schur's sum_i R0_i^T X_i, from the forward
// reduction alone; same blocks of NPB nodes, same entry table and k_sp_schur_red
__device__ __forceinline__ void zschur_block(const SpDev& d, int blk, double* sm) {
  // sm: Z_R [18][m] | acc [Ws] | tab
  const int tid = threadIdx.x, m = d.m, wc = 36 + m;
  double* Zl = sm;
  double* acc = sm + 2 * NB * m;  // (k_sp_schur's layout: the LDS size is the host's lds_schur)
  short2* tab = (short2*)(acc + d.Ws);
  for (int q = tid; q < d.Ws; q += blockDim.x) {
    acc[q] = 0.0;
    tab[q] = d.uab[q];
  }
  const int i0 = max(blk * NPB, d.zsf ? 1 : 0), i1 = min(d.n, blk * NPB + NPB);  // zsf: node 0 by k_sp_schur_red
  constexpr int ZS_U = (NB * (MAXC + 1) + 255) / 256;
  const int nq = NB * m;
  const float rinv = 1.0f / (float)m;
  double v[ZS_U];
  auto load = [&](int i) {
    const double* Z = d.Z + (size_t)i * NB * wc + 2 * NB;
#pragma unroll
    for (int u = 0; u < ZS_U; ++u) {
      const int q = min(tid + u * 256, nq - 1), r = div_small(q, rinv);
      v[u] = Z[r * wc + (q - r * m)];
    }
  };
  if (i0 < i1) load(i0);
  for (int i = i0; i < i1; ++i) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < ZS_U; ++u) {
      const int q = tid + u * 256;
      if (q < nq) Zl[q] = v[u];
    }
    __syncthreads();
    if (i + 1 < i1) load(i + 1);
    for (int q = tid; q < d.Ws; q += blockDim.x) {
      const short2 ab = tab[q];
      const int a = ab.x, b = ab.y;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NB; ++k) s += Zl[k * m + a] * Zl[k * m + b];
      acc[q] += s;
    }
  }
  __syncthreads();
  for (int q = tid; q < d.Ws; q += blockDim.x) d.spart[(size_t)blk * d.Ws + q] = acc[q];
}

__global__ void __launch_bounds__(256) k_sp_zschur(SpDev d) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  zschur_block(d, blockIdx.x, sm);
}

// zs, step 1 (every node at once, after the camera solve): with v = [-dtheta | 1], node j's operands of the
// one-column back substitution, [M_l | M_r | u] = L_j^-T [Z_Uin,j | Z_U,j | Z_R,j v] (18 x 37, row-major into bm):
// the chain of strides then needs no triangular solve, x_j = u_j - M_l x_{j-s} - M_r x_{j+s}
__global__ void __launch_bounds__(256) k_sp_bprep(SpDev d) {
  // one wave per node (4 per block), wave-local LDS: L | 1/diag | T = [Z_Uin | Z_U | y] (18 x 37) | y partials | v
  __shared__ double Ls[4][NB * NB];
  __shared__ double ids[4][NB];
  __shared__ double Ts[4][NB * 37];
  __shared__ double yp[4][3 * NB];
  __shared__ double vs[4][MAXC + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, m = d.m, wc = 36 + m, C = d.C;
  const int j = 4 * blockIdx.x + wave;
  if (j >= d.n) return;  // wave-uniform
  KSP_TSB(100, 272);  // diagnostics: block 100's (wave 0's) timeline in slots 272..276 (tools/diag_sp_asm.py)
  double* L = Ls[wave];
  double* id = ids[wave];
  double* T = Ts[wave];
  const double* Z = d.Z + (size_t)j * NB * wc;
  {  // every load in flight before the LDS stores (the loops' per-iteration waits took ~5 us)
    constexpr int UL = (NB * NB + 63) / 64, UT = (NB * 36 + 63) / 64;
    double lv[UL], tv[UT];
    const double* Lj = d.Lf + (size_t)j * NB * NB;
#pragma unroll
    for (int u = 0; u < UL; ++u) lv[u] = Lj[min(lane + 64 * u, NB * NB - 1)];
#pragma unroll
    for (int u = 0; u < UT; ++u) {
      const int q = min(lane + 64 * u, NB * 36 - 1), r = q / 36;
      tv[u] = Z[r * wc + q - 36 * r];
    }
    const double iv = d.Lid[(size_t)j * NB + min(lane, NB - 1)];
    const double xv = d.dx[min(lane, C - 1)];
#pragma unroll
    for (int u = 0; u < UL; ++u)
      if (lane + 64 * u < NB * NB) L[lane + 64 * u] = lv[u];
#pragma unroll
    for (int u = 0; u < UT; ++u) {
      const int q = lane + 64 * u, r = q / 36;
      if (q < NB * 36) T[r * 37 + q - 36 * r] = tv[u];
    }
    if (lane < NB) id[lane] = iv;
    if (lane < m) vs[wave][lane] = lane < C ? -xv : 1.0;  // m = C + 1 <= MAXC + 1 = 65: lanes 0..63 and
    if (lane == 0 && m > 64) vs[wave][64] = 1.0;            // (C = 64) the rhs slot
  }
  KSP_WAVE_SYNC();
  KSP_TSB(100, 273);
  if (lane < 3 * NB) {  // y = Z_R v: three lanes per row over interleaved columns, summed in a fixed order; the
                        // row's loads all issued before the chain (a run-time trip count serialised them)
    const int r = lane % NB, pp = lane / NB;
    constexpr int UY = (MAXC + 1 + 2) / 3;
    double zv[UY];
#pragma unroll
    for (int u = 0; u < UY; ++u) zv[u] = Z[r * wc + 36 + min(pp + 3 * u, m - 1)];
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < UY; ++u)
      if (pp + 3 * u < m) t = fma(zv[u], vs[wave][pp + 3 * u], t);
    yp[wave][pp * NB + r] = t;
  }
  KSP_WAVE_SYNC();
  if (lane < NB) T[lane * 37 + 36] = (yp[wave][lane] + yp[wave][NB + lane]) + yp[wave][2 * NB + lane];
  KSP_WAVE_SYNC();
  KSP_TSB(100, 274);
  node_backsolve_lean(L, id, T, 37, 37, d.bm + (size_t)j * NB * 37, lane, 64);
  KSP_TSB(100, 275);
}

// zs, step 2: node j of stride s on one wave (s = 0: the top node, x_0 = u_0): lane r < 18 forms row r of
// x_j = u_j - M_l x_{j-s} - M_r x_{j+s} (every load in one round), written to xs and as the node's coefficient steps
// into dx
__device__ __forceinline__ void bvec_node(const SpDev& d, int j, int s, int lane) {
  const int C = d.C;
  const int l = j - s, r = j + s;
  const bool hl = s > 0, hr = s > 0 && r < d.n;
  const int row = lane < NB ? lane : 0;
  const double* M = d.bm + (size_t)j * NB * 37 + row * 37;
  double mr[37], xl[NB], xr[NB];
#pragma unroll
  for (int k = 0; k < 37; ++k) mr[k] = M[k];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    xl[k] = d.xs[(size_t)(hl ? l : j) * NB + k];
    xr[k] = d.xs[(size_t)(hr ? r : j) * NB + k];
  }
  double t = mr[36];
#pragma unroll
  for (int k = 0; k < NB; ++k) t = fma(-mr[k], hl ? xl[k] : 0.0, t);
#pragma unroll
  for (int k = 0; k < NB; ++k) t = fma(-mr[NB + k], hr ? xr[k] : 0.0, t);
  if (lane < NB) {
    d.xs[(size_t)j * NB + lane] = t;
    const int k = SB * j + lane / 6;
    if (k < d.K) d.dx[C + 6 * k + lane % 6] = t;
  }
}

// zs, step 2 for the deep strides in one block of 8 waves: the top node, then strides s_hi .. s_lo (at most 16 nodes
// each, one or two per wave), a block barrier between strides (the xs stores are block-visible after it)
constexpr int kBvecDeepWaves = 8;
__global__ void __launch_bounds__(64 * kBvecDeepWaves) k_sp_bvec_deep(SpDev d, int s_hi, int s_lo) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int nst = 1;
  for (int s = s_hi; s >= s_lo && s >= 1; s >>= 1) ++nst;
  for (int t = 0; t < nst; ++t) {
    const int s = t == 0 ? 0 : (s_hi >> (t - 1));
    for (int b = wave; b < (t == 0 ? 1 : 16); b += kBvecDeepWaves) {
      const int j = t == 0 ? 0 : s + 2 * s * b;
      if (j < d.n) bvec_node(d, j, s, lane);
    }
    __syncthreads();
  }
}

// zs, step 2 for one wider stride s: one node per wave (4 per block)
__global__ void __launch_bounds__(256) k_sp_bvec(SpDev d, int s) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = s + 2 * s * (4 * blockIdx.x + wave);
  if (j >= d.n) return;  // wave-uniform
  bvec_node(d, j, s, lane);
}

// S = H_cc + lam2 I - sum_i R0_i^T X_i, b = g_c - sum (4-wave interleaved partial sums), written full
__global__ void __launch_bounds__(64 * RW) k_sp_schur_red(SpDev d) {
  __shared__ double red[RW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, C = d.C, nup = C * (C + 1) / 2;
  const int q = blockIdx.x * 64 + lane;
  const bool act = q < d.Ws;
  red[wave][lane] = act ? col_sum(d.spart, d.nblk_s, d.Ws, q, wave, RW) : 0.0;
  __syncthreads();
  if (wave != 0 || !act) return;
  double t = red_waves(red, lane);
  const short2 ab = d.uab[q];
  const int a = ab.x, b = ab.y;
  if (d.zsf) {  // the top node's Z_R,0^T Z_R,0 (its Schur sums were not in the top level's extra blocks)
    const int wc = 36 + d.m;
    const double* Z0 = d.Z + 2 * NB;
    double z = 0.0;
#pragma unroll
    for (int k = 0; k < NB; ++k) z += Z0[k * wc + a] * Z0[k * wc + b];
    t += z;
  }
  if (q < nup) {
    const double v = d.Hcc[a * C + b] + (a == b ? d.sc[SC_LAM2] : 0.0) - t;
    d.Sf[a * C + b] = v;
    d.Sf[b * C + a] = v;
  } else {
    d.Sf[C * C + a] = d.Hcc[C * C + a] - t;
  }
}

// dense camera / IMU block solve on one wave: lane r holds row r of S in registers (CM >= C, padded with the
// identity so that no step depends on the run-time C), LDL^T with row k broadcast by v_readlane and 1/D_k by
// rcp + Newton (no square roots or IEEE divisions on the dependent chain), then L y = b, z = D^-1 y, L^T x = z.
// Lanes i > k apply S[i][j] -= (S[i][k] / D_k) S[k][j]; row i freezes at step i, so lane i ends holding
// Ltilde[i][k] D_k (k < i) and D_i.  dtheta -> dx[0..C)
template <int CM>
__global__ void __launch_bounds__(64) k_sp_camsolve(SpDev d) {
  const int lane = threadIdx.x, C = d.C;
  const int li = lane < C ? lane : 0;
  double a[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) a[c] = d.Sf[li * C + (c < C ? c : 0)];  // clamped: every load unconditional
  double x = d.Sf[C * C + li];
#pragma unroll
  for (int c = 0; c < CM; ++c) a[c] = (lane < C && c < C) ? a[c] : (lane == c ? 1.0 : 0.0);
  x = lane < C ? x : 0.0;
  bool ok = true;
  double rD = 1.0;
#pragma unroll
  for (int k = 0; k < CM; ++k) {
    const double Dk = rdlane(a[k], k);
    ok = ok && (Dk > 0.0);
    const double rdk = ksp_recip1(Dk);
    rD = (lane == k) ? rdk : rD;
    const double f = (lane > k) ? a[k] * rdk : 0.0;
#pragma unroll
    for (int j = k + 1; j < CM; ++j) a[j] -= f * rdlane(a[j], k);
  }
#pragma unroll
  for (int k = 0; k < CM; ++k) {
    const double yk = rdlane(x, k) * rdlane(rD, k);
    x -= ((lane > k) ? a[k] : 0.0) * yk;
  }
  x *= rD;
#pragma unroll
  for (int k = CM - 1; k > 0; --k) {
    const double wk = rdlane(x, k);
    x -= ((lane < k) ? a[k] * rD : 0.0) * wk;
  }
  if (lane < C) d.dx[lane] = x;
  if (lane == 0 && !ok) d.sc[SC_OK] = 0.0;
}

// coefficient steps ds_i = X_i[:, C] - X_i[:, :C] dtheta; with `apply` (and a successful solve) the state
// update: backup copy, additive coefficients, theta DVs (block 0); per-block max |dx|.
__global__ void __launch_bounds__(64) k_sp_update(SpDev d, int apply) {
  const int i = blockIdx.x, tid = threadIdx.x, C = d.C, m = d.m;
  const bool go = apply && d.sc[SC_OK] != 0.0;
  double mx = 0.0;
  if (tid < NB) {
    const int k = SB * i + tid / 6;
    if (k < d.K) {
      double v;
      if (d.zs) {  // written by the one-column back substitution (k_sp_bvec*)
        v = d.dx[C + 6 * k + tid % 6];
      } else {
        const double* x = d.X + (size_t)i * NB * m + tid * m;
        v = x[C];
#pragma unroll 16
        for (int c = 0; c < C; ++c) v -= x[c] * d.dx[c];
        d.dx[C + 6 * k + tid % 6] = v;
      }
      mx = fabs(v);
      const int o = d.off_coef + 6 * k + tid % 6;
      if (go) {
        d.backup[o] = d.state[o];
        d.state[o] += v;
      }
    }
  }
  if (i == 0) {
    for (int c = tid; c < C; c += 64) mx = fmax(mx, fabs(d.dx[c]));
    if (go) {
      for (int q = tid; q < d.off_coef; q += 64) d.backup[q] = d.state[q];
      __syncthreads();
      for (int c = tid; c < C; c += 64) {
        const int kind = d.ckind[c], idx = d.cidx[c], sub = d.csub[c];
        if (kind == 0) d.state[idx * KB_MAX_INTR + sub] += d.dx[c];
        if (kind == 2) d.state[d.off_imu + sub] += d.dx[c];
      }
      if (tid < d.N) {  // pose DVs q = tid: B_q (q < N-1) or T_c0_b
        const int q = tid;
        double* pose = d.state + (q < d.N - 1 ? d.off_base + 7 * q : d.off_cb);
        double np[7];
        kb::update_pose(pose, d.dx + d.col_pose[q], np);
#pragma unroll
        for (int k = 0; k < 7; ++k) pose[k] = np[k];
      }
    }
  }
  // wave max
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if (tid == 0) d.dmax[i] = mx;
}

// ---------------------------------------------------------------- cost (evaluateError)
template <unsigned MM>
__global__ void __launch_bounds__(512) k_sp_cost_frames(SpDev d) {
  __shared__ double red[8];
  const int N = d.N, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, cam = wave;
  if ((int)blockIdx.x >= d.nblk_f) {  // the extra blocks: the IMU samples' chi^2, 64 N samples per block
    const int m = ((int)blockIdx.x - d.nblk_f) * 64 * N + tid;
    double s = 0.0;
    if (m < d.M) {
      double e[6], Ct[9];
      imu_sample(d, m, e, nullptr, Ct);
#pragma unroll
      for (int r = 0; r < 6; ++r) s += e[r] * e[r];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[wave] = s;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int q = 0; q < N; ++q) t += red[q];
      d.cpart[blockIdx.x] = t;  // cpart[nblk_f + IMU block]
    }
    return;
  }
  const double* st = d.state;
  double RA[9], tA[3];
  kb::quat2r(st + d.off_cb, RA);
  tA[0] = st[d.off_cb + 4];
  tA[1] = st[d.off_cb + 5];
  tA[2] = st[d.off_cb + 6];
  for (int q = 0; q < cam; ++q) {  // A = B_{cam-1} .. B_0 T_c0_b
    const double* bq = st + d.off_base + 7 * q;
    double RB[9], R2[9], t2[3];
    kb::quat2r(bq, RB);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
        R2[r * 3 + c] = RB[r * 3 + 0] * RA[0 * 3 + c] + RB[r * 3 + 1] * RA[1 * 3 + c] + RB[r * 3 + 2] * RA[2 * 3 + c];
      t2[r] = RB[r * 3 + 0] * tA[0] + RB[r * 3 + 1] * tA[1] + RB[r * 3 + 2] * tA[2] + bq[4 + r];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) RA[k] = R2[k];
    tA[0] = t2[0];
    tA[1] = t2[1];
    tA[2] = t2[2];
  }
  const int model = sp_cam_arg(d.model, cam);
  const double* intr = st + cam * KB_MAX_INTR;
  double s = 0.0;
  const int f0 = blockIdx.x * FPB, f1 = min(d.F, f0 + FPB);
  for (int f = f0; f < f1; ++f) {
    const int b = d.fb[f];
    const double* w = d.fw + 4 * f;
    const double* cf = st + d.off_coef + 6 * b;
    double v[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[r] = w[0] * cf[r] + w[1] * cf[6 + r] + w[2] * cf[12 + r] + w[3] * cf[18 + r];
    double Rwb[9], R[9], t[3];
    rv_C(v + 3, Rwb);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        R[r * 3 + c] = RA[r * 3 + 0] * Rwb[c * 3 + 0] + RA[r * 3 + 1] * Rwb[c * 3 + 1] + RA[r * 3 + 2] * Rwb[c * 3 + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) t[r] = tA[r] - (R[r * 3 + 0] * v[0] + R[r * 3 + 1] * v[1] + R[r * 3 + 2] * v[2]);
    const int2 fv = d.fview[(size_t)f * N + cam];
    for (int k = fv.x + lane; k < fv.y; k += 64) {
      const int ci = d.cid[k];
      const double2 yv = d.y[k];
      const double* X = d.target + 3 * ci;
      const double p0 = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
      const double p1 = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
      const double p2 = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
      double u, wv;
      kb::project<MM>(model, intr, p0, p1, p2, u, wv);
      const double e0 = yv.x - u, e1 = yv.y - wv;
      s += e0 * e0 + e1 * e1;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int q = 0; q < N; ++q) t += red[q];
    d.cpart[blockIdx.x] = t;
  }
}

// BSplineMotionError::evaluateErrorImplementation (BSplineMotionError.hpp:62-78): c^T Q c of the current state,
// one node per lane (c_i^T QD_i c_i + 2 c_i^T QU_i c_(i+1), + the node's own priors' chi^2) -> cpart[nblk_f + nblk_ci +
// block]
__global__ void __launch_bounds__(64) k_sp_cost_motion(SpDev d) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  double s = 0.0;
  if (i < d.n) {
    double ci[NB], cj[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int k = SB * i + q / 6, k1 = k + SB;
      ci[q] = k < d.K ? d.state[d.off_coef + 6 * k + q % 6] : 0.0;
      cj[q] = k1 < d.K ? d.state[d.off_coef + 6 * k1 + q % 6] : 0.0;
    }
    if (d.mot) {
      const double* QDi = d.QD + (size_t)i * NB * NB;
      const double* QUi = d.QU + (size_t)i * NB * NB;
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        double a = 0.0, w = 0.0;
#pragma unroll
        for (int c = 0; c < NB; ++c) {
          a += QDi[r * NB + c] * ci[c];
          w += QUi[r * NB + c] * cj[c];
        }
        s += ci[r] * (a + 2.0 * w);
      }
    }
    if (d.npos) {  // the node's own ErrorTermEuclidean priors (first coefficient in 3i .. 3i+2), as k_sp_assemble
      double pc = 0.0;
      for (int k = d.node_pp[4 * i + 2]; k < d.node_pp[4 * i + 3]; ++k) {
        const int b = d.pb[k];
        const double* w = d.pw + 4 * k;
        const double* cf = d.state + d.off_coef + 6 * b;
        double e[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          double v = 0.0;
#pragma unroll
          for (int j = 0; j < 4; ++j) v += w[j] * cf[6 * j + a];
          e[a] = v - d.pp[3 * k + a];
        }
        const double* W = d.pW + 9 * k;
        double c2 = 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) c2 += e[a] * (W[3 * a] * e[0] + W[3 * a + 1] * e[1] + W[3 * a + 2] * e[2]);
        pc += c2;
      }
      s += pc;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (threadIdx.x == 0) d.cpart[d.nblk_f + d.nblk_ci + blockIdx.x] = s;
}

// motion cost of the build state: fixed-order sum of k_sp_assemble's per-node values, added to the build cost
__global__ void __launch_bounds__(256) k_sp_mcost_build(SpDev d) {
  __shared__ double red[4];
  double s = 0.0;
  for (int q = threadIdx.x; q < d.n; q += 256) s += d.mcost[q];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = (red[0] + red[1]) + (red[2] + red[3]);
    d.Hcc[d.C * d.C + d.C] += t;
    d.sc[SC_COST_BUILD] += t;
  }
}

// fixed-order sums: cost -> sc[SC_COST], max |dx| -> sc[SC_DX]
__global__ void __launch_bounds__(64) k_sp_cost_reduce(SpDev d, int with_dx) {
  const int tid = threadIdx.x;
  double s = 0.0, mx = 0.0;
#pragma unroll 8
  for (int q = tid; q < d.nblk_f + d.nblk_ci + (d.cq ? d.nblk_q : 0); q += 64) s += d.cpart[q];
  if (with_dx) {
#pragma unroll 8
    for (int q = tid; q < d.n; q += 64) mx = fmax(mx, d.dmax[q]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    mx = fmax(mx, __shfl_xor(mx, o));
  }
  if (tid == 0) {
    d.sc[SC_COST] = s;
    if (with_dx) d.sc[SC_DX] = mx;
  }
}

__global__ void k_sp_revert(SpDev d) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < d.S) d.state[q] = d.backup[q];
}

// lambda^2 of the next solve, and its success flag reset (the reduction kernels clear it on a failed factorisation)
__global__ void k_sp_set_lam(SpDev d, double lam2) {
  if (threadIdx.x == 0) {
    d.sc[SC_LAM2] = lam2;
    d.sc[SC_OK] = 1.0;
  }
}

}  // namespace ksp

// ==================================================================================================
// host side
// ==================================================================================================
using namespace ksp;

namespace {
int fail(const std::string& m) { return kb_internal::fail(m); }

#define KSP_HIP(call)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess) return fail(std::string(#call) + ": " + hipGetErrorString(e_));        \
  } while (0)

int nintr_of(int m) {
  switch (m) {
    case KB_PINHOLE_RADTAN: return 8;
    case KB_OMNI_RADTAN: return 9;
    case KB_EUCM: return 6;
    case KB_OMNI: return 5;
    case KB_DS: return 6;
    case KB_PINHOLE_EQUI: return 8;
    case KB_PINHOLE_FOV: return 5;
    default: return -1;
  }
}

// B-spline basis matrix of valid segment `seg` (BSpline.cpp:70-152) and basis weights (BSpline.cpp:237-387)
void basis_matrix(const std::vector<double>& kn, int k, int i, double* out) {
  if (k == 1) {
    out[0] = 1.0;
    return;
  }
  double Mp[64];
  basis_matrix(kn, k - 1, i, Mp);
  const int n = k - 1;
  double M1[64] = {0}, M2[64] = {0}, A[64] = {0}, B[64] = {0};
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) {
      M1[r * n + c] = Mp[r * n + c];
      M2[(r + 1) * n + c] = Mp[r * n + c];
    }
  for (int idx = 0; idx < n; ++idx) {
    const int j = i - k + 2 + idx;
    const double den = kn[j + k - 1] - kn[j];
    const double d0 = den <= 0.0 ? 0.0 : (kn[i] - kn[j]) / den;
    const double d1 = den <= 0.0 ? 0.0 : (kn[i + 1] - kn[i]) / den;
    A[idx * k + idx] = 1.0 - d0;
    A[idx * k + idx + 1] = d0;
    B[idx * k + idx] = -d1;
    B[idx * k + idx + 1] = d1;
  }
  for (int r = 0; r < k; ++r)
    for (int c = 0; c < k; ++c) {
      double s = 0.0;
      for (int l = 0; l < n; ++l) s += M1[r * n + l] * A[l * k + c] + M2[r * n + l] * B[l * k + c];
      out[r * k + c] = s;
    }
}

int basis_weights(const std::vector<double>& kn, int order, double t, int deriv, double* w) {
  const int nk = (int)kn.size();
  const double tmin = kn[order - 1], tmax = kn[nk - order];
  if (t < tmin || t > tmax + 1e-10) return -1;
  if (std::fabs(tmax - t) < 1e-10) t = tmax;
  int idx;
  if (t == tmax) {
    idx = nk - order - 1;
  } else {
    idx = (int)(std::upper_bound(kn.begin(), kn.end(), t) - kn.begin()) - 1;
  }
  const double dt = kn[idx + 1] - kn[idx];
  const double u = dt <= 0.0 ? 0.0 : (t - kn[idx]) / dt;
  const double mult = dt > 0.0 ? 1.0 / std::pow(dt, deriv) : 0.0;
  double uv[8] = {0}, uu = 1.0;
  for (int i = deriv; i < order; ++i) {
    int dm = 1;
    for (int q = 0; q < deriv; ++q) dm *= (i - q);
    uv[i] = mult * uu * dm;
    uu *= u;
  }
  const int bidx = idx - order + 1;
  double M[64];
  basis_matrix(kn, order, bidx + order - 1, M);
  for (int j = 0; j < order; ++j) {
    double s = 0.0;
    for (int i = 0; i < order; ++i) s += M[i * order + j] * uv[i];
    w[j] = s;
  }
  return bidx;
}

// segmentQuadraticIntegral (BSpline.cpp:1512-1548) of valid segment s without the W factor:
// Q_s = M^T (Dm^T)^m V Dm^m M with V(r, c) = dt / (r + c + 1) (Vi, :1276-1300), Dm(i, i + 1) = (i + 1) / dt
// (Dii, :1483-1500) and M the segment's basis matrix (Mi, :1391-1403); Q_s[j][l] couples coefficients s + j, s + l.
void segment_quadratic(const std::vector<double>& kn, int s, int m, double* Q) {
  double M[64], V[16], Dm[16] = {0}, T[16];
  basis_matrix(kn, ORD, s + ORD - 1, M);
  const double dt = kn[s + ORD] - kn[s + ORD - 1];
  const double rdt = dt > 0.0 ? 1.0 / dt : 0.0;
  for (int r = 0; r < ORD; ++r)
    for (int c = 0; c < ORD; ++c) V[r * ORD + c] = dt / (r + c + 1.0);
  for (int i = 0; i + 1 < ORD; ++i) Dm[i * ORD + i + 1] = (i + 1.0) * rdt;
  for (int it = 0; it < m; ++it) {  // V <- Dm^T V Dm
    for (int r = 0; r < ORD; ++r)
      for (int c = 0; c < ORD; ++c) {
        double a = 0.0;
        for (int k = 0; k < ORD; ++k) a += V[r * ORD + k] * Dm[k * ORD + c];
        T[r * ORD + c] = a;
      }
    for (int r = 0; r < ORD; ++r)
      for (int c = 0; c < ORD; ++c) {
        double a = 0.0;
        for (int k = 0; k < ORD; ++k) a += Dm[k * ORD + r] * T[k * ORD + c];
        V[r * ORD + c] = a;
      }
  }
  for (int j = 0; j < ORD; ++j)
    for (int l = 0; l < ORD; ++l) {
      double a = 0.0;
      for (int r = 0; r < ORD; ++r)
        for (int c = 0; c < ORD; ++c) a += M[r * ORD + j] * V[r * ORD + c] * M[c * ORD + l];
      Q[j * ORD + l] = a;
    }
}
}  // namespace

struct kb_sp_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  SpDev d{};
  int N = 0, C = 0, K = 0, F = 0, M = 0, n = 0, S = 0, ncols = 0, n_target = 0, NCo = 0;
  std::vector<double> knots;
  std::vector<void*> allocs;
  double lambda = 0.0;
  bool uploaded = false, built = false, solved = false;
  size_t lds_frames = 0, lds_asm = 0, lds_elim = 0, lds_level = 0, lds_schur = 0, lds_back = 0, lds_back2 = 0;
  bool back2 = true;       // k_sp_back2: two back-substitution strides per launch
  const void* fn_frames = nullptr;
  const void* fn_cost = nullptr;
  const void* fn_camsolve = nullptr;
  hipGraphExec_t gn_graph = nullptr;
  int gn_graph_n = 0;
  std::vector<SpLvl> lv;  // partitioned band solve: lv[0 .. nl) chunk levels, lv[nl] the top system
  bool use_cr = true;     // block cyclic reduction; KSP_PARTITION=1: the partitioned band solve
  int s_deep = 0;         // first stride run by k_sp_deep (0: one launch per level)
  int s_top = 0;          // zs: the stride the forward reduction ended at (the top node solved there)
  int deep_groups = 0;    // k_sp_deep's node groups (kSpDeepGT threads each)
  size_t lds_deep = 0;
  std::vector<double> trace;
  double* host_sc = nullptr;  // pinned scalars

  template <class T>
  int alloc(T** p, size_t cnt) {
    void* q = nullptr;
    if (cnt == 0) cnt = 1;
    hipError_t e = hipMalloc(&q, cnt * sizeof(T));
    if (e != hipSuccess) return fail(std::string("hipMalloc: ") + hipGetErrorString(e));
    hipMemsetAsync(q, 0, cnt * sizeof(T), stream);
    allocs.push_back(q);
    *p = (T*)q;
    return 0;
  }
  // free a buffer alloc() made (nullptr: no-op); the stream must be idle with respect to it
  void release(const void* p) {
    if (!p) return;
    auto it = std::find(allocs.begin(), allocs.end(), const_cast<void*>(p));
    if (it == allocs.end()) return;
    allocs.erase(it);
    hipFree(const_cast<void*>(p));
  }
};

namespace {
template <unsigned MM>
void pick_mm(kb_sp_handle* h) {
  h->fn_frames = (const void*)k_sp_frames<MM>;
  h->fn_cost = (const void*)k_sp_cost_frames<MM>;
}

// k_sp_frames' grid: the frame blocks, then ceil(nblk_ic / N) blocks whose N waves each take one of k_sp_imu_cc's
// 64-sample blocks
int frames_grid(const kb_sp_handle* h) { return h->d.nblk_f + (h->d.nblk_ic + h->N - 1) / h->N; }

int launch_build(kb_sp_handle* h) {
  SpDev& d = h->d;
  void* args[] = {&d};
  // the frames and, in its extra blocks, the IMU samples (k_sp_imu_cc's work: records, partial rows, lambda^2 = 0 of a
  // GN pass)
  KSP_HIP(hipLaunchKernel(h->fn_frames, dim3(frames_grid(h)), dim3(64 * h->N), args, h->lds_frames, h->stream));
  KSP_HIP(hipLaunchKernel((const void*)k_sp_assemble, dim3(d.n), dim3(256), args, h->lds_asm, h->stream));
  if (!d.cc_fused) hipLaunchKernelGGL(k_sp_reduce_cc, dim3((d.Wc + 63) / 64), dim3(64 * RW), 0, h->stream, d);
  if (d.cq) hipLaunchKernelGGL(k_sp_mcost_build, dim3(1), dim3(256), 0, h->stream, d);
  return 0;
}

int launch_reduction(kb_sp_handle* h) {
  SpDev& d = h->d;
  if (!h->use_cr) {  // partitioned: chunk levels down, the top system, back-substitution levels up
    const int nl = (int)h->lv.size() - 1;
    for (int l = 0; l < nl; ++l) {
      const SpLvl& L = h->lv[l];
      hipLaunchKernelGGL(k_sp_chunk, dim3((L.n + L.q - 1) / L.q), dim3(256), 0, h->stream, d, L);
    }
    hipLaunchKernelGGL(k_sp_ctop, dim3(1), dim3(256), 0, h->stream, d, h->lv[nl]);
    for (int l = nl - 1; l >= 0; --l) {
      const SpLvl& L = h->lv[l];
      hipLaunchKernelGGL(k_sp_cback, dim3((L.n + L.q - 1) / L.q), dim3(256), 0, h->stream, d, L);
    }
    return 0;
  }
  if (d.n == 1) {
    hipLaunchKernelGGL(k_sp_top, dim3(1), dim3(256), sizeof(double) * NB * d.m, h->stream, d);
    h->s_top = 1;
    return 0;
  }
  hipLaunchKernelGGL(k_sp_elim1, dim3(d.n / 2 + (d.cc_fused ? (d.Wc + 3) / 4 : 0)), dim3(256), h->lds_elim, h->stream, d);
  int s = 1;
  const int sd = h->s_deep;
  for (; s < d.n && !(sd && s >= sd); s *= 2) {
    const bool last = d.zsf && 2 * s >= d.n;  // the top level: one block, the Schur sums beside it
    hipLaunchKernelGGL(s == 1 ? k_sp_level<true> : k_sp_level<false>,
                       dim3((d.n + 2 * s - 1) / (2 * s) + (last ? d.nblk_s : 0)), dim3(256),
                       last ? std::max(h->lds_level, h->lds_schur) : h->lds_level, h->stream, d, s);
  }
  if (d.zs) {  // the back substitution runs after the camera solve, with one column (launch_bvec)
    h->s_top = s;
    return 0;
  }
  if (sd && s < d.n) {  // the remaining levels down and back up to stride sd in one block
    hipLaunchKernelGGL(k_sp_deep, dim3(1), dim3(kSpDeepGT * h->deep_groups), h->lds_deep, h->stream, d, sd);
    s = sd;
  }
  // back-substitution strides s/2 .. 1: with k_sp_back2 two per launch (an odd count leaves the top one single)
  int nb = 0;
  for (int t = s / 2; t >= 1; t /= 2) ++nb;
  for (s /= 2; s >= 1;) {
    if (h->back2 && (nb & 1) == 0) {
      const int sl = s / 2, ne = (d.n - sl + 2 * sl - 1) / (2 * sl);
      hipLaunchKernelGGL(k_sp_back2, dim3(ne), dim3(256), h->lds_back2, h->stream, d, sl);
      s /= 4;
      nb -= 2;
    } else {
      const int ne = (d.n - s + 2 * s - 1) / (2 * s);
      hipLaunchKernelGGL(k_sp_back, dim3(ne), dim3(256), h->lds_back, h->stream, d, s);
      s /= 2;
      nb -= 1;
    }
  }
  return 0;
}

// zs: the back substitution with v = [-dtheta | 1]: the top node and the strides with at most 16 nodes in one block
// (k_sp_bvec_deep), the wider strides one launch each (a wave per node)
int launch_bvec(kb_sp_handle* h) {
  SpDev& d = h->d;
  auto count = [&](int s) { return d.n > s ? (d.n - s + 2 * s - 1) / (2 * s) : 0; };
  int s = h->s_top / 2, s_lo = s;
  while (s_lo > 1 && count(s_lo / 2) <= 16) s_lo /= 2;
  hipLaunchKernelGGL(k_sp_bprep, dim3((d.n + 3) / 4), dim3(256), 0, h->stream, d);
  hipLaunchKernelGGL(k_sp_bvec_deep, dim3(1), dim3(64 * kBvecDeepWaves), 0, h->stream, d, s, s >= 1 ? s_lo : 1 << 30);
  for (s = s_lo / 2; s >= 1; s /= 2) hipLaunchKernelGGL(k_sp_bvec, dim3((count(s) + 3) / 4), dim3(256), 0, h->stream, d, s);
  KSP_HIP(hipGetLastError());
  return 0;
}

int launch_solve(kb_sp_handle* h) {
  SpDev& d = h->d;
  void* args[] = {&d};
  launch_reduction(h);
  if (!d.zsf) hipLaunchKernelGGL(d.zs ? k_sp_zschur : k_sp_schur, dim3(d.nblk_s), dim3(256), h->lds_schur, h->stream, d);
  hipLaunchKernelGGL(k_sp_schur_red, dim3((d.Ws + 63) / 64), dim3(64 * RW), 0, h->stream, d);
  KSP_HIP(hipLaunchKernel(h->fn_camsolve, dim3(1), dim3(64), args, 0, h->stream));
  if (d.zs) return launch_bvec(h);
  return 0;
}

int launch_cost(kb_sp_handle* h, int with_dx) {
  SpDev& d = h->d;
  void* args[] = {&d};
  // the frames' cost and, in its extra nblk_ci blocks, the IMU samples'
  KSP_HIP(hipLaunchKernel(h->fn_cost, dim3(d.nblk_f + d.nblk_ci), dim3(64 * h->N), args, 0, h->stream));
  if (d.cq) hipLaunchKernelGGL(k_sp_cost_motion, dim3(d.nblk_q), dim3(64), 0, h->stream, d);
  hipLaunchKernelGGL(k_sp_cost_reduce, dim3(1), dim3(64), 0, h->stream, d, with_dx);
  return 0;
}

// one GN pass: build, solve (lambda = 0), update, cost
int enqueue_gn_pass(kb_sp_handle* h) {
  SpDev& d = h->d;
  d.zero_lam = 1;  // lambda = 0 written by the build's k_sp_imu_cc
  // H_cc's column sums inside k_sp_elim1 (the cyclic reduction, no motion-error build cost to add after them)
  d.cc_fused = (h->use_cr && d.n > 1 && !d.cq && !std::getenv("KSP_CC_SEPARATE")) ? 1 : 0;
  const int rb = launch_build(h);
  d.zero_lam = 0;
  const int rs = rb ? 0 : launch_solve(h);
  d.cc_fused = 0;
  if (rb || rs) return -1;
  hipLaunchKernelGGL(k_sp_update, dim3(d.n), dim3(64), 0, h->stream, d, 1);
  return launch_cost(h, 1);
}

int read_scalars(kb_sp_handle* h) {
  KSP_HIP(hipMemcpyAsync(h->host_sc, h->d.sc, sizeof(double) * SC_NSC, hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  return 0;
}
}  // namespace

extern "C" {

kb_sp_handle* kb_sp_create(const kb_sp_layout* L) {
  if (!L || !L->cam_model || !L->target_points || !L->knots) {
    fail("kb_sp_create: null layout");
    return nullptr;
  }
  if (L->order != ORD) {
    fail("kb_sp_create: the device spline path supports order 4 (cubic) only");
    return nullptr;
  }
  if (L->n_cams < 1 || L->n_cams > 8 || L->n_target < 1 || L->n_target > 65535) {
    fail("kb_sp_create: n_cams / n_target out of range");
    return nullptr;
  }
  if (!(L->sigma_gyro > 0.0) || !(L->sigma_acc > 0.0)) {
    fail("kb_sp_create: IMU sigmas must be positive");
    return nullptr;
  }
  for (int q = 1; q < L->n_knots; ++q)
    if (L->knots[q] < L->knots[q - 1]) {
      fail("kb_sp_create: knots must be non-decreasing");
      return nullptr;
    }
  const int K = L->n_knots - 2 * L->order + 1 > 0 ? L->n_knots - L->order : 0;
  if (K < ORD) {
    fail("kb_sp_create: not enough knots for one valid time segment");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    fail("kb_sp_create: no HIP device available (the product path has no CPU fallback)");
    return nullptr;
  }
  kb_sp_handle* h = new kb_sp_handle();
  h->device = L->device;
  if (hipSetDevice(h->device) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    fail("kb_sp_create: cannot select device / create stream");
    delete h;
    return nullptr;
  }
  h->N = L->n_cams;
  h->K = K;
  h->knots.assign(L->knots, L->knots + L->n_knots);
  h->n_target = L->n_target;
  SpDev& d = h->d;
  d.N = h->N;
  d.K = K;
  d.n_target = L->n_target;
  int c = 0;
  for (int i = 0; i < h->N; ++i) {
    const int ni = nintr_of(L->cam_model[i]);
    if (ni < 0) {
      fail("kb_sp_create: unknown camera model");
      kb_sp_destroy(h);
      return nullptr;
    }
    d.model[i] = L->cam_model[i];
    d.nin[i] = ni;
    d.col_intr[i] = c;
    for (int q = 0; q < ni; ++q, ++c) {
      d.ckind[c] = 0;
      d.cidx[c] = i;
      d.csub[c] = q;
    }
  }
  for (int q = 0; q < h->N; ++q) {  // B_0 .. B_{N-2}, then T_c0_b
    d.col_pose[q] = c;
    for (int e = 0; e < 6; ++e, ++c) {
      d.ckind[c] = 1;
      d.cidx[c] = q;
      d.csub[c] = e;
    }
  }
  d.col_imu = c;
  for (int e = 0; e < 9; ++e, ++c) {
    d.ckind[c] = 2;
    d.cidx[c] = 0;
    d.csub[c] = e;
  }
  h->C = d.C = c;
  if (h->C > MAXC) {
    fail("kb_sp_create: camera + IMU block larger than 64 columns");
    kb_sp_destroy(h);
    return nullptr;
  }
  d.m = h->C + 1;
  d.off_base = h->N * KB_MAX_INTR;
  d.off_cb = d.off_base + 7 * (h->N - 1);
  d.off_imu = d.off_cb + 7;
  d.off_coef = d.off_imu + 9;
  h->S = d.S = d.off_coef + 6 * K;
  h->ncols = h->C + 6 * K;
  h->n = d.n = (K + SB - 1) / SB;
  d.ig = 1.0 / L->sigma_gyro;
  d.ia = 1.0 / L->sigma_acc;
  d.Wc = h->C * (h->C + 1) / 2 + h->C + 1;
  d.Ws = h->C * (h->C + 1) / 2 + h->C;
  d.FHS = 36 + 6 * h->C + 6;
  unsigned mm = 0;
  for (int i = 0; i < h->N; ++i) mm |= 1u << d.model[i];
  if (mm == (1u << KB_PINHOLE_RADTAN))
    pick_mm<1u << KB_PINHOLE_RADTAN>(h);
  else
    pick_mm<kMmAll>(h);
  int rc = 0;
  double* tgt = nullptr;
  rc |= h->alloc(&tgt, 3 * (size_t)L->n_target);
  d.target = tgt;
  rc |= h->alloc(&d.state, (size_t)h->S);
  rc |= h->alloc(&d.backup, (size_t)h->S);
  rc |= h->alloc(&d.Hcc, (size_t)h->C * h->C + h->C + 1);
  rc |= h->alloc(&d.D0, (size_t)h->n * NB * NB);
  rc |= h->alloc(&d.U0, (size_t)h->n * NB * NB);
  rc |= h->alloc(&d.R0, (size_t)h->n * NB * d.m);
  rc |= h->alloc(&d.D, (size_t)h->n * NB * NB);
  rc |= h->alloc(&d.R, (size_t)h->n * NB * d.m);
  rc |= h->alloc(&d.Lf, (size_t)h->n * NB * NB);
  rc |= h->alloc(&d.Lid, (size_t)h->n * NB);
  rc |= h->alloc(&d.Z, (size_t)h->n * NB * (36 + d.m));
  rc |= h->alloc(&d.X, (size_t)h->n * NB * d.m);
  {
    // partitioned band solve: level 0 is the built system; chunks of 16 nodes, then 8, until <= kSpTop remain
    const char* ev = std::getenv("KSP_PARTITION");
    h->use_cr = !(ev && std::atoi(ev) != 0);
    SpLvl L0{};
    L0.n = h->n;
    L0.Dt = d.D0;
    L0.U = d.U0;
    L0.Rt = d.R0;
    L0.Lf = d.Lf;
    L0.Lid = d.Lid;
    L0.Z = d.Z;
    L0.X = d.X;
    h->lv.push_back(L0);
    while (h->lv.back().n > kSpTop) {
      SpLvl& Lc = h->lv.back();
      Lc.q = Lc.lvl == 0 ? 16 : 8;
      SpLvl Ln{};
      Ln.lvl = Lc.lvl + 1;
      Ln.n = (Lc.n + Lc.q - 1) / Lc.q;
      const size_t nn = (size_t)Ln.n;
      double *Dt = nullptr, *Dh = nullptr, *U = nullptr, *Rt = nullptr, *Rh = nullptr;
      rc |= h->alloc(&Dt, nn * NB * NB);
      rc |= h->alloc(&Dh, nn * NB * NB);
      rc |= h->alloc(&U, nn * NB * NB);
      rc |= h->alloc(&Rt, nn * NB * d.m);
      rc |= h->alloc(&Rh, nn * NB * d.m);
      rc |= h->alloc(&Ln.Lf, nn * NB * NB);
      rc |= h->alloc(&Ln.Lid, nn * NB);
      rc |= h->alloc(&Ln.Z, nn * NB * (36 + d.m));
      rc |= h->alloc(&Ln.X, nn * NB * d.m);
      Ln.Dt = Lc.nDt = Dt;
      Ln.Dh = Lc.nDh = Dh;
      Ln.U = Lc.nU = U;
      Ln.Rt = Lc.nRt = Rt;
      Ln.Rh = Lc.nRh = Rh;
      Lc.Xup = Ln.X;
      if (rc) break;
      h->lv.push_back(Ln);
    }
    h->lv.back().q = h->lv.back().n;
  }
  d.nblk_s = (h->n + NPB - 1) / NPB;
  rc |= h->alloc(&d.spart, (size_t)d.nblk_s * d.Ws);
  rc |= h->alloc(&d.dx, (size_t)h->ncols);
  rc |= h->alloc(&d.dmax, (size_t)h->n);
  rc |= h->alloc(&d.sc, (size_t)SC_NSC);
  rc |= h->alloc(&d.Sf, (size_t)h->C * h->C + h->C);
  {
    std::vector<short2> tab((size_t)d.Wc);
    int q = 0;
    for (int a = 0; a < h->C; ++a)
      for (int b = a; b < h->C; ++b) tab[q++] = make_short2((short)a, (short)b);
    for (int a = 0; a < h->C; ++a) tab[q++] = make_short2((short)a, (short)h->C);
    tab[q++] = make_short2((short)h->C, (short)h->C);
    short2* dt = nullptr;
    rc |= h->alloc(&dt, tab.size());
    if (!rc) rc |= hipMemcpyAsync(dt, tab.data(), sizeof(short2) * tab.size(), hipMemcpyHostToDevice, h->stream) != hipSuccess;
    d.uab = dt;
  }
  h->fn_camsolve = h->C <= 16 ? (const void*)k_sp_camsolve<16>
                   : h->C <= 32 ? (const void*)k_sp_camsolve<32>
                   : h->C <= 40 ? (const void*)k_sp_camsolve<40>  // configs[4]: C = 37
                   : h->C <= 48 ? (const void*)k_sp_camsolve<48>
                                : (const void*)k_sp_camsolve<64>;
  if (rc || hipHostMalloc((void**)&h->host_sc, sizeof(double) * SC_NSC) != hipSuccess ||
      hipMemcpyAsync(tgt, L->target_points, sizeof(double) * 3 * L->n_target, hipMemcpyHostToDevice, h->stream) !=
          hipSuccess) {
    if (!rc) fail("kb_sp_create: pinned scalars / target upload failed");
    kb_sp_destroy(h);
    return nullptr;
  }
  h->lds_elim = sizeof(double) * NB * (36 + d.m);
  h->lds_level = 3 * h->lds_elim;
  h->lds_back = h->lds_elim + sizeof(double) * 3 * NB * d.m;
  h->lds_back2 = 2 * h->lds_elim + sizeof(double) * 5 * NB * d.m;
  {
    const char* ev = std::getenv("KSP_BACK2");  // two back-substitution strides per launch (default on)
    h->back2 = !(ev && std::atoi(ev) == 0);
  }
  h->lds_schur = sizeof(double) * (2 * NB * d.m + d.Ws) + sizeof(short2) * d.Ws;
  h->lds_asm = sizeof(double) * (2 * NB * NB + NB * d.m + std::max(TCH * IRS + 6 * PNS * PST, TCF * d.FHS));
  h->lds_frames = sizeof(double) * (h->N * 64 * XS + h->N * 256 + 2 * h->N * 36 + 2 * h->N * h->N * 36 +
                                    3 * L->n_target) +
                  sizeof(short2) * d.Wc + sizeof(int) * 3 * d.C;
  if (h->lds_frames > 160 * 1024 || h->lds_asm > 160 * 1024 || h->lds_schur > 160 * 1024) {
    fail("kb_sp_create: LDS budget exceeded for this rig");
    kb_sp_destroy(h);
    return nullptr;
  }
  hipFuncSetAttribute(h->fn_frames, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_frames);
  hipFuncSetAttribute((const void*)k_sp_assemble, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_asm);
  // (the top level's launch may carry the Schur sums' blocks: zsf)
  hipFuncSetAttribute((const void*)k_sp_level<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)std::max(h->lds_level, h->lds_schur));
  hipFuncSetAttribute((const void*)k_sp_level<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)std::max(h->lds_level, h->lds_schur));
  hipFuncSetAttribute((const void*)k_sp_elim1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_elim);
  hipFuncSetAttribute((const void*)k_sp_back, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_back);
  hipFuncSetAttribute((const void*)k_sp_back2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_back2);
  {
    // the deep levels in one block (k_sp_deep, KSP_DEEP=1; measured and not kept: configs[4] 2,227 -> 1,998 GN it/s,
    // the one-block kernel 118 us against 74 us for the six launches it replaces -- four nodes share one CU's SIMDs
    // and LDS port where each level kernel gives a node a CU of its own, which outweighs the saved launches): as
    // many node groups as the LDS holds (<= kSpDeepGroups), from the first stride whose level has at most that many
    // nodes
    const size_t per = sizeof(double) * kSpDeepPer(d.m);
    h->deep_groups = (int)std::min<size_t>(kSpDeepGroups, (160 * 1024) / per);
    h->s_deep = 0;
    const char* ev = std::getenv("KSP_DEEP");
    if (h->deep_groups >= 2 && h->n >= 2 && ev && std::atoi(ev) != 0) {
      int sd = 1;
      while ((h->n + 2 * sd - 1) / (2 * sd) > h->deep_groups) sd *= 2;
      h->s_deep = sd;
      h->lds_deep = per * h->deep_groups;
      hipFuncSetAttribute((const void*)k_sp_deep, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_deep);
    }
  }
  hipFuncSetAttribute((const void*)k_sp_schur, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_schur);
  hipFuncSetAttribute((const void*)k_sp_zschur, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_schur);
  {
    // the Schur complement from the forward reduction and the one-column back substitution (default with the cyclic
    // reduction; KSP_ZS=0 keeps the C + 1 column back substitution and X)
    const char* ev = std::getenv("KSP_ZS");
    d.zs = (h->use_cr && h->s_deep == 0 && !(ev && std::atoi(ev) == 0)) ? 1 : 0;
    // the Schur sums beside the top level's block (one launch less; KSP_ZSF=0 keeps k_sp_zschur)
    const char* ef = std::getenv("KSP_ZSF");
    d.zsf = (d.zs && h->n > 1 && !(ef && std::atoi(ef) == 0)) ? 1 : 0;
    if (d.zs && (h->alloc(&d.xs, (size_t)h->n * NB) || h->alloc(&d.bm, (size_t)h->n * NB * 37))) {
      kb_sp_destroy(h);
      return nullptr;
    }
  }
  if (hipStreamSynchronize(h->stream) != hipSuccess) {
    fail("kb_sp_create: stream sync failed");
    kb_sp_destroy(h);
    return nullptr;
  }
  return h;
}

void kb_sp_destroy(kb_sp_handle* h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->gn_graph) hipGraphExecDestroy(h->gn_graph);
  for (void* p : h->allocs) hipFree(p);
  if (h->host_sc) hipHostFree(h->host_sc);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
}

int kb_sp_upload(kb_sp_handle* h, int32_t n_frames, const double* frame_time, int32_t n_views, int32_t n_corners,
                 const double* y, const uint16_t* corner_id, const uint32_t* view_offsets,
                 const uint32_t* view_frame, const uint8_t* view_cam, int32_t n_imu, const double* imu_time,
                 const double* imu_gyro, const double* imu_acc) {
  if (!h) return fail("kb_sp_upload: null handle");
  if (h->uploaded) return fail("kb_sp_upload: observations already uploaded (create a new handle)");
  if (n_frames < 1 || n_views < 0 || n_corners < 0 || n_imu < 0) return fail("kb_sp_upload: bad sizes");
  if (!frame_time || (n_views && (!view_offsets || !view_frame || !view_cam)) || (n_corners && (!y || !corner_id)) ||
      (n_imu && (!imu_time || !imu_gyro || !imu_acc)))
    return fail("kb_sp_upload: null array");
  KSP_HIP(hipSetDevice(h->device));
  SpDev& d = h->d;
  const int N = h->N, F = n_frames, M = n_imu;
  // frames: basis weights, views (sorted by frame, one per camera)
  std::vector<int> fb(F), ib(M);
  std::vector<double> fw(4 * (size_t)F), iw(12 * (size_t)M), imeas(6 * (size_t)M);
  for (int f = 0; f < F; ++f) {
    if (f && frame_time[f] < frame_time[f - 1]) return fail("kb_sp_upload: frame times must be non-decreasing");
    fb[f] = basis_weights(h->knots, ORD, frame_time[f], 0, &fw[4 * (size_t)f]);
    if (fb[f] < 0) return fail("kb_sp_upload: frame time outside the spline interval");
  }
  for (int m = 0; m < M; ++m) {
    if (m && imu_time[m] < imu_time[m - 1]) return fail("kb_sp_upload: IMU times must be non-decreasing");
    ib[m] = basis_weights(h->knots, ORD, imu_time[m], 0, &iw[12 * (size_t)m]);
    if (ib[m] < 0) return fail("kb_sp_upload: IMU time outside the spline interval");
    basis_weights(h->knots, ORD, imu_time[m], 1, &iw[12 * (size_t)m + 4]);
    basis_weights(h->knots, ORD, imu_time[m], 2, &iw[12 * (size_t)m + 8]);
    for (int r = 0; r < 3; ++r) {
      imeas[6 * (size_t)m + r] = imu_gyro[3 * (size_t)m + r];
      imeas[6 * (size_t)m + 3 + r] = imu_acc[3 * (size_t)m + r];
    }
  }
  std::vector<int2> fview((size_t)F * N, make_int2(0, 0));
  for (int v = 0; v < n_views; ++v) {
    const uint32_t f = view_frame[v], cam = view_cam[v];
    if (f >= (uint32_t)F || cam >= (uint32_t)N) return fail("kb_sp_upload: view frame / camera out of range");
    if (v && view_frame[v] < view_frame[v - 1]) return fail("kb_sp_upload: views must be sorted by frame");
    if (view_offsets[v + 1] < view_offsets[v] || view_offsets[v + 1] > (uint32_t)n_corners)
      return fail("kb_sp_upload: bad view offsets");
    int2& e = fview[(size_t)f * N + cam];
    if (e.y > e.x) return fail("kb_sp_upload: two views of one (frame, camera)");
    e = make_int2((int)view_offsets[v], (int)view_offsets[v + 1]);
  }
  for (int k = 0; k < n_corners; ++k)
    if (corner_id[k] >= h->n_target) return fail("kb_sp_upload: corner id out of range");
  // per node: terms whose support [b, b+3] touches coefficients 3i .. 3i+2
  std::vector<int> nfr(2 * (size_t)h->n), nim(2 * (size_t)h->n);
  for (int i = 0; i < h->n; ++i) {
    const int lo = SB * i - 3, hi = SB * i + 2;
    nfr[2 * i] = (int)(std::lower_bound(fb.begin(), fb.end(), lo) - fb.begin());
    nfr[2 * i + 1] = (int)(std::upper_bound(fb.begin(), fb.end(), hi) - fb.begin());
    nim[2 * i] = (int)(std::lower_bound(ib.begin(), ib.end(), lo) - ib.begin());
    nim[2 * i + 1] = (int)(std::upper_bound(ib.begin(), ib.end(), hi) - ib.begin());
  }
  h->F = d.F = F;
  h->M = d.M = M;
  h->NCo = n_corners;
  d.nblk_f = (F + FPB - 1) / FPB;
  d.nblk_ci = std::max(1, (M + 64 * N - 1) / (64 * N));  // k_sp_cost_frames' IMU blocks (64 N samples each)
  d.nblk_ic = std::max(1, (M + 63) / 64);
  int rc = 0;
  double2* dy = nullptr;
  uint16_t* dcid = nullptr;
  int2* dfv = nullptr;
  int *dfb = nullptr, *dib = nullptr, *dnf = nullptr, *dni = nullptr;
  double *dfw = nullptr, *diw = nullptr, *dim = nullptr;
  rc |= h->alloc(&dy, (size_t)n_corners);
  rc |= h->alloc(&dcid, (size_t)n_corners);
  rc |= h->alloc(&dfv, (size_t)F * N);
  rc |= h->alloc(&dfb, (size_t)F);
  rc |= h->alloc(&dfw, 4 * (size_t)F);
  rc |= h->alloc(&dib, (size_t)M);
  rc |= h->alloc(&diw, 12 * (size_t)M);
  rc |= h->alloc(&dim, 6 * (size_t)M);
  rc |= h->alloc(&dnf, 2 * (size_t)h->n);
  rc |= h->alloc(&dni, 2 * (size_t)h->n);
  rc |= h->alloc(&d.FH, (size_t)F * d.FHS);
  rc |= h->alloc(&d.part, (size_t)d.nblk_f * d.Wc);
  d.nblk_q = (h->n + 63) / 64;
#ifdef KB_STAMPS
  if (const char* e = std::getenv("KSP_DBG_STOP")) d.dbg_stop = std::atoi(e);  // diagnostic build only
  if (!d.dbg_ts) rc |= h->alloc(&d.dbg_ts, 320);
#endif
  rc |= h->alloc(&d.cpart, (size_t)(d.nblk_f + d.nblk_ci + d.nblk_q));
  rc |= h->alloc(&d.mcost, (size_t)h->n);
  rc |= h->alloc(&d.ipart, (size_t)d.nblk_ic * WI);
  rc |= h->alloc(&d.irec, (size_t)IRQ * std::max(M, 1));
  if (rc) return -1;
  if (n_corners) {
    KSP_HIP(hipMemcpyAsync(dy, y, sizeof(double) * 2 * n_corners, hipMemcpyHostToDevice, h->stream));
    KSP_HIP(hipMemcpyAsync(dcid, corner_id, sizeof(uint16_t) * n_corners, hipMemcpyHostToDevice, h->stream));
  }
  KSP_HIP(hipMemcpyAsync(dfv, fview.data(), sizeof(int2) * fview.size(), hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dfb, fb.data(), sizeof(int) * F, hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dfw, fw.data(), sizeof(double) * fw.size(), hipMemcpyHostToDevice, h->stream));
  if (M) {
    KSP_HIP(hipMemcpyAsync(dib, ib.data(), sizeof(int) * M, hipMemcpyHostToDevice, h->stream));
    KSP_HIP(hipMemcpyAsync(diw, iw.data(), sizeof(double) * iw.size(), hipMemcpyHostToDevice, h->stream));
    KSP_HIP(hipMemcpyAsync(dim, imeas.data(), sizeof(double) * imeas.size(), hipMemcpyHostToDevice, h->stream));
  }
  KSP_HIP(hipMemcpyAsync(dnf, nfr.data(), sizeof(int) * nfr.size(), hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dni, nim.data(), sizeof(int) * nim.size(), hipMemcpyHostToDevice, h->stream));
  d.y = dy;
  d.cid = dcid;
  d.fview = dfv;
  d.fb = dfb;
  d.fw = dfw;
  d.ib = dib;
  d.iw = diw;
  d.imeas = dim;
  d.node_fr = dnf;
  d.node_im = dni;
  KSP_HIP(hipStreamSynchronize(h->stream));
  h->uploaded = true;
  return 0;
}

int kb_sp_state_size(const kb_sp_handle* h) { return h ? h->S : -1; }
int kb_sp_num_cols(const kb_sp_handle* h) { return h ? h->ncols : -1; }
int kb_sp_camera_cols(const kb_sp_handle* h) { return h ? h->C : -1; }

int kb_sp_set_state(kb_sp_handle* h, const double* state) {
  if (!h || !state) return fail("kb_sp_set_state: null");
  KSP_HIP(hipSetDevice(h->device));
  KSP_HIP(hipMemcpyAsync(h->d.state, state, sizeof(double) * h->S, hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(h->d.backup, state, sizeof(double) * h->S, hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  h->built = h->solved = false;
  return 0;
}

int kb_sp_get_state(kb_sp_handle* h, double* state) {
  if (!h || !state) return fail("kb_sp_get_state: null");
  KSP_HIP(hipSetDevice(h->device));
  KSP_HIP(hipMemcpyAsync(state, h->d.state, sizeof(double) * h->S, hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kb_sp_eval_cost(kb_sp_handle* h, double* J_out) {
  if (!h || !J_out) return fail("kb_sp_eval_cost: null");
  if (!h->uploaded) return fail("kb_sp_eval_cost: upload observations first");
  KSP_HIP(hipSetDevice(h->device));
  if (launch_cost(h, 0)) return -1;
  if (read_scalars(h)) return -1;
  *J_out = h->host_sc[SC_COST];
  return 0;
}

int kb_sp_build(kb_sp_handle* h) {
  if (!h) return fail("kb_sp_build: null");
  if (!h->uploaded) return fail("kb_sp_build: upload observations first");
  KSP_HIP(hipSetDevice(h->device));
  if (launch_build(h)) return -1;
  KSP_HIP(hipGetLastError());
  h->built = true;
  h->solved = false;
  return 0;
}

// BSplineMotionError (aslam_splines BSplineMotionError.hpp:29-160) over the pose spline: Q =
// curveQuadraticIntegralSparse(W, order) (BSpline.cpp:1585-1622) split into the node blocks of the cyclic reduction
// (nodes of SB coefficients; Q's band reaches order - 1 = 3 coefficients, i.e. the next node only).
int kb_sp_set_motion_error(kb_sp_handle* h, const double* W, int32_t derivative_order) {
  if (!h) return fail("kb_sp_set_motion_error: null handle");
  KSP_HIP(hipSetDevice(h->device));
  if (h->gn_graph) {  // captured passes hold the old SpDev
    hipGraphExecDestroy(h->gn_graph);
    h->gn_graph = nullptr;
  }
  if (!W) {
    h->d.mot = 0;
    h->d.cq = h->d.npos > 0;
    return 0;
  }
  int m = derivative_order;
  if (m < 0) return fail("kb_sp_set_motion_error: negative derivative order");
  if (m >= ORD) m = ORD - 1;  // BSplineMotionError::initialize: "Invalid ErrorTermOrder reduced" (:33-36)
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c)
      if (std::fabs(W[r * 6 + c] - W[c * 6 + r]) > 1e-14)  // segmentQuadraticIntegral: "W must be symmetric"
        return fail("kb_sp_set_motion_error: W must be symmetric");
  const int K = h->K, n = h->n;
  std::vector<double> q((size_t)K * ORD, 0.0);  // q[k][d]: scalar Q of coefficients (k, k + d)
  double Qs[ORD * ORD];
  for (int sg = 0; sg + ORD <= K; ++sg) {
    if (!(h->knots[sg + ORD] > h->knots[sg + ORD - 1])) continue;
    segment_quadratic(h->knots, sg, m, Qs);
    for (int j = 0; j < ORD; ++j)
      for (int l = j; l < ORD; ++l) q[(size_t)(sg + j) * ORD + (l - j)] += Qs[j * ORD + l];
  }
  std::vector<double> QD((size_t)n * NB * NB, 0.0), QU((size_t)n * NB * NB, 0.0);
  auto qv = [&](int k, int l) {  // scalar Q(k, l), symmetric, 0 outside the band / beyond K
    if (k > l) std::swap(k, l);
    return (k < 0 || l >= K || l - k >= ORD) ? 0.0 : q[(size_t)k * ORD + (l - k)];
  };
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < NB; ++r)
      for (int c = 0; c < NB; ++c) {
        const int k = SB * i + r / 6, w = (r % 6) * 6 + c % 6;
        QD[((size_t)i * NB + r) * NB + c] = qv(k, SB * i + c / 6) * W[w];
        QU[((size_t)i * NB + r) * NB + c] = qv(k, SB * (i + 1) + c / 6) * W[w];
      }
  SpDev& d = h->d;
  if (!d.QD) {
    double *qd = nullptr, *qu = nullptr;
    if (h->alloc(&qd, (size_t)n * NB * NB) || h->alloc(&qu, (size_t)n * NB * NB)) return -1;
    d.QD = qd;
    d.QU = qu;
  }
  KSP_HIP(hipMemcpyAsync(const_cast<double*>(d.QD), QD.data(), sizeof(double) * QD.size(), hipMemcpyHostToDevice,
                         h->stream));
  KSP_HIP(hipMemcpyAsync(const_cast<double*>(d.QU), QU.data(), sizeof(double) * QU.size(), hipMemcpyHostToDevice,
                         h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  d.mot = 1;
  d.cq = 1;
  return 0;
}

int kb_sp_set_position_priors(kb_sp_handle* h, int32_t n, const double* times, const double* priors,
                              const double* N) {
  if (!h) return fail("kb_sp_set_position_priors: null handle");
  if (n < 0 || (n > 0 && (!times || !priors || !N))) return fail("kb_sp_set_position_priors: bad arguments");
  KSP_HIP(hipSetDevice(h->device));
  if (h->gn_graph) {  // captured passes hold the old SpDev
    hipGraphExecDestroy(h->gn_graph);
    h->gn_graph = nullptr;
  }
  SpDev& d = h->d;
  // the previous call's prior tables go (repeated calls do not accumulate device buffers)
  auto drop_priors = [&]() -> int {
    KSP_HIP(hipStreamSynchronize(h->stream));
    h->release(d.pb);
    h->release(d.pw);
    h->release(d.pp);
    h->release(d.pW);
    h->release(d.node_pp);
    d.pb = nullptr;
    d.pw = d.pp = d.pW = nullptr;
    d.node_pp = nullptr;
    d.npos = 0;
    d.cq = d.mot;
    return 0;
  };
  if (n == 0) return drop_priors();
  // per prior: first coefficient and value weights (BSpline::evalDAndJacobian(t, 0)), invR = N^-1 (ErrorTermEuclidean's
  // first constructor, ErrorTermEuclidean.cpp:10-23: setInvR(N.inverse())); sorted by first coefficient, then time
  std::vector<int> ord(n), b(n);
  std::vector<double> w(4 * (size_t)n), W(9 * (size_t)n);
  for (int k = 0; k < n; ++k) {
    b[k] = basis_weights(h->knots, ORD, times[k], 0, &w[4 * (size_t)k]);
    if (b[k] < 0) return fail("kb_sp_set_position_priors: prior time outside the spline interval");
    const double* M = N + 9 * (size_t)k;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < r; ++c)
        if (std::fabs(M[3 * r + c] - M[3 * c + r]) > 1e-12 * (std::fabs(M[3 * r + c]) + std::fabs(M[3 * c + r])))
          return fail("kb_sp_set_position_priors: N must be symmetric");
    const double c00 = M[4] * M[8] - M[5] * M[7], c01 = M[5] * M[6] - M[3] * M[8], c02 = M[3] * M[7] - M[4] * M[6];
    const double det = M[0] * c00 + M[1] * c01 + M[2] * c02;
    // Sylvester: all three leading principal minors positive (diag(1, -1, -1) has det > 0 and M00 > 0)
    if (!(M[0] > 0.0) || !(M[0] * M[4] - M[1] * M[3] > 0.0) || !(det > 0.0))
      return fail("kb_sp_set_position_priors: N must be positive definite");
    double* I = &W[9 * (size_t)k];  // adjugate / det
    I[0] = c00 / det;
    I[1] = (M[2] * M[7] - M[1] * M[8]) / det;
    I[2] = (M[1] * M[5] - M[2] * M[4]) / det;
    I[3] = c01 / det;
    I[4] = (M[0] * M[8] - M[2] * M[6]) / det;
    I[5] = (M[2] * M[3] - M[0] * M[5]) / det;
    I[6] = c02 / det;
    I[7] = (M[1] * M[6] - M[0] * M[7]) / det;
    I[8] = (M[0] * M[4] - M[1] * M[3]) / det;
    ord[k] = k;
  }
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return b[x] < b[y]; });
  std::vector<int> pb(n);
  std::vector<double> pw(4 * (size_t)n), pp(3 * (size_t)n), pW(9 * (size_t)n);
  for (int q = 0; q < n; ++q) {
    const int k = ord[q];
    pb[q] = b[k];
    for (int j = 0; j < 4; ++j) pw[4 * (size_t)q + j] = w[4 * (size_t)k + j];
    for (int a = 0; a < 3; ++a) pp[3 * (size_t)q + a] = priors[3 * (size_t)k + a];
    for (int e = 0; e < 9; ++e) pW[9 * (size_t)q + e] = W[9 * (size_t)k + e];
  }
  std::vector<int> npp(4 * (size_t)h->n);
  for (int i = 0; i < h->n; ++i) {
    npp[4 * i] = (int)(std::lower_bound(pb.begin(), pb.end(), SB * i - 3) - pb.begin());
    npp[4 * i + 1] = (int)(std::upper_bound(pb.begin(), pb.end(), SB * i + 2) - pb.begin());
    npp[4 * i + 2] = (int)(std::lower_bound(pb.begin(), pb.end(), SB * i) - pb.begin());
    npp[4 * i + 3] = npp[4 * i + 1];
  }
  int *dpb = nullptr, *dnp = nullptr;
  double *dpw = nullptr, *dpp = nullptr, *dpW = nullptr;
  if (drop_priors()) return -1;  // inputs validated: the old tables are replaced
  if (h->alloc(&dpb, n) || h->alloc(&dpw, 4 * (size_t)n) || h->alloc(&dpp, 3 * (size_t)n) ||
      h->alloc(&dpW, 9 * (size_t)n) || h->alloc(&dnp, npp.size()))
    return -1;
  KSP_HIP(hipMemcpyAsync(dpb, pb.data(), sizeof(int) * n, hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dpw, pw.data(), sizeof(double) * pw.size(), hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dpp, pp.data(), sizeof(double) * pp.size(), hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dpW, pW.data(), sizeof(double) * pW.size(), hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipMemcpyAsync(dnp, npp.data(), sizeof(int) * npp.size(), hipMemcpyHostToDevice, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  d.pb = dpb;
  d.pw = dpw;
  d.pp = dpp;
  d.pW = dpW;
  d.node_pp = dnp;
  d.npos = n;
  d.cq = 1;
  return 0;
}

int kb_sp_set_constant_conditioner(kb_sp_handle* h, double diag) {
  if (!h) return fail("kb_sp_set_constant_conditioner: null");
  h->lambda = diag;
  return 0;
}

int kb_sp_solve(kb_sp_handle* h, double* dx_out, int* ok) {
  if (!h || !ok) return fail("kb_sp_solve: null");
  if (!h->built) return fail("kb_sp_solve: build first");
  KSP_HIP(hipSetDevice(h->device));
  hipLaunchKernelGGL(k_sp_set_lam, dim3(1), dim3(64), 0, h->stream, h->d, h->lambda * h->lambda);
  if (launch_solve(h)) return -1;
  hipLaunchKernelGGL(k_sp_update, dim3(h->d.n), dim3(64), 0, h->stream, h->d, 0);
  KSP_HIP(hipGetLastError());
  if (read_scalars(h)) return -1;
  *ok = h->host_sc[SC_OK] != 0.0;
  if (*ok && dx_out)
    KSP_HIP(hipMemcpy(dx_out, h->d.dx, sizeof(double) * h->ncols, hipMemcpyDeviceToHost));
  h->solved = *ok != 0;
  return 0;
}

int kb_sp_get_rhs(kb_sp_handle* h, double* rhs_out) {
  if (!h || !rhs_out) return fail("kb_sp_get_rhs: null");
  if (!h->built) return fail("kb_sp_get_rhs: build first");
  KSP_HIP(hipSetDevice(h->device));
  const int C = h->C, m = C + 1;
  std::vector<double> R0((size_t)h->n * NB * m);
  KSP_HIP(hipMemcpyAsync(rhs_out, h->d.Hcc + (size_t)C * C, sizeof(double) * C, hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipMemcpyAsync(R0.data(), h->d.R0, sizeof(double) * R0.size(), hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  for (int k = 0; k < h->K; ++k)
    for (int c = 0; c < 6; ++c) rhs_out[C + 6 * k + c] = R0[(size_t)(k / SB) * NB * m + (6 * (k % SB) + c) * m + C];
  return 0;
}

int kb_sp_apply_update(kb_sp_handle* h, const double* dx, double* deltaX_out) {
  if (!h) return fail("kb_sp_apply_update: null");
  KSP_HIP(hipSetDevice(h->device));
  SpDev& d = h->d;
  if (dx) {
    // host dx: write it as the solve output (X rows are not used when dx is given): theta + coefficients
    KSP_HIP(hipMemcpyAsync(d.dx, dx, sizeof(double) * h->ncols, hipMemcpyHostToDevice, h->stream));
    std::vector<double> st(h->S);
    KSP_HIP(hipMemcpyAsync(st.data(), d.state, sizeof(double) * h->S, hipMemcpyDeviceToHost, h->stream));
    KSP_HIP(hipStreamSynchronize(h->stream));
    KSP_HIP(hipMemcpyAsync(d.backup, d.state, sizeof(double) * h->S, hipMemcpyDeviceToDevice, h->stream));
    // host-side DV update (same rules as k_sp_update), then upload
    double mx = 0.0;
    for (int c = 0; c < h->ncols; ++c) mx = std::max(mx, std::fabs(dx[c]));
    for (int c = 0; c < h->C; ++c) {
      if (d.ckind[c] == 0) st[d.cidx[c] * KB_MAX_INTR + d.csub[c]] += dx[c];
      if (d.ckind[c] == 2) st[d.off_imu + d.csub[c]] += dx[c];
    }
    for (int q = 0; q < h->N; ++q) {
      double* pose = st.data() + (q < h->N - 1 ? d.off_base + 7 * q : d.off_cb);
      const double* a = dx + d.col_pose[q];
      const double th = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
      double na, ca;
      if (th < 1.220703125e-4) {
        na = 0.5 + th * th / 48.0;
        ca = 1.0 - th * th / 8.0;
      } else {
        na = std::sin(0.5 * th) / th;
        ca = std::cos(0.5 * th);
      }
      const double d0 = a[0] * na, d1 = a[1] * na, d2 = a[2] * na;
      const double q0 = pose[0], q1 = pose[1], q2 = pose[2], q3 = pose[3];
      pose[0] = q0 * ca + d0 * q3 - d1 * q2 + d2 * q1;
      pose[1] = q1 * ca + d0 * q2 + d1 * q3 - d2 * q0;
      pose[2] = q2 * ca - d0 * q1 + d1 * q0 + d2 * q3;
      pose[3] = q3 * ca - d0 * q0 - d1 * q1 - d2 * q2;
      for (int k = 0; k < 3; ++k) pose[4 + k] += a[3 + k];
    }
    for (int q = 0; q < 6 * h->K; ++q) st[d.off_coef + q] += dx[h->C + q];
    KSP_HIP(hipMemcpyAsync(d.state, st.data(), sizeof(double) * h->S, hipMemcpyHostToDevice, h->stream));
    KSP_HIP(hipStreamSynchronize(h->stream));
    if (deltaX_out) *deltaX_out = mx;
  } else {
    if (!h->solved) return fail("kb_sp_apply_update: no device solution");
    hipLaunchKernelGGL(k_sp_update, dim3(d.n), dim3(64), 0, h->stream, d, 1);
    hipLaunchKernelGGL(k_sp_cost_reduce, dim3(1), dim3(64), 0, h->stream, d, 1);
    if (read_scalars(h)) return -1;
    if (deltaX_out) *deltaX_out = h->host_sc[SC_DX];
  }
  h->built = h->solved = false;
  return 0;
}

int kb_sp_revert(kb_sp_handle* h) {
  if (!h) return fail("kb_sp_revert: null");
  KSP_HIP(hipSetDevice(h->device));
  hipLaunchKernelGGL(k_sp_revert, dim3((h->S + 255) / 256), dim3(256), 0, h->stream, h->d);
  KSP_HIP(hipStreamSynchronize(h->stream));
  h->built = h->solved = false;
  return 0;
}

int kb_sp_get_system(kb_sp_handle* h, double* Hcc, double* Hsc, double* Hband, double* gc, double* gs,
                     double* cost) {
  if (!h) return fail("kb_sp_get_system: null");
  if (!h->built) return fail("kb_sp_get_system: build first");
  KSP_HIP(hipSetDevice(h->device));
  const int C = h->C, m = C + 1, n = h->n, K = h->K;
  std::vector<double> hc((size_t)C * C + C + 1), D0((size_t)n * NB * NB), U0((size_t)n * NB * NB),
      R0((size_t)n * NB * m);
  KSP_HIP(hipMemcpyAsync(hc.data(), h->d.Hcc, sizeof(double) * hc.size(), hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipMemcpyAsync(D0.data(), h->d.D0, sizeof(double) * D0.size(), hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipMemcpyAsync(U0.data(), h->d.U0, sizeof(double) * U0.size(), hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipMemcpyAsync(R0.data(), h->d.R0, sizeof(double) * R0.size(), hipMemcpyDeviceToHost, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  if (Hcc) std::memcpy(Hcc, hc.data(), sizeof(double) * C * C);
  if (gc) std::memcpy(gc, hc.data() + (size_t)C * C, sizeof(double) * C);
  if (cost) *cost = hc[(size_t)C * C + C];
  for (int k = 0; k < K; ++k) {
    const int i = k / SB, rk = 6 * (k % SB);
    for (int a = 0; a < 6; ++a) {
      for (int c = 0; c < C; ++c)
        if (Hsc) Hsc[(size_t)(6 * k + a) * C + c] = R0[(size_t)i * NB * m + (rk + a) * m + c];
      if (gs) gs[6 * k + a] = R0[(size_t)i * NB * m + (rk + a) * m + C];
    }
    if (!Hband) continue;
    for (int dd = 0; dd < ORD; ++dd) {
      const int k2 = k + dd;
      for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) {
          double v = 0.0;
          if (k2 < K) {
            const int i2 = k2 / SB, rk2 = 6 * (k2 % SB);
            if (i2 == i)
              v = D0[(size_t)i * NB * NB + (rk + a) * NB + rk2 + b];
            else if (i2 == i + 1)
              v = U0[(size_t)i * NB * NB + (rk + a) * NB + rk2 + b];
          }
          Hband[((size_t)k * ORD + dd) * 36 + a * 6 + b] = v;
        }
    }
  }
  return 0;
}

int kb_sp_optimize(kb_sp_handle* h, const kb_optimizer_options* o, kb_solution* out) {
  if (!h || !o || !out) return fail("kb_sp_optimize: null");
  if (!h->uploaded) return fail("kb_sp_optimize: upload observations first");
  // Optimizer2::optimize (Optimizer2.cpp:183-273) + LM / GN policies, host-driven over the device passes
  std::memset(out, 0, sizeof(*out));
  h->trace.clear();
  const bool lm = o->policy == 0;
  const int ncols = h->ncols;
  std::vector<double> dx(ncols, 0.0), rhs(ncols, 0.0), tmp(ncols);
  double J;
  if (kb_sp_eval_cost(h, &J)) return -1;
  double p_J = J;
  out->J_start = p_J;
  double deltaX = o->convergence_dx + 1.0, deltaJ = o->convergence_dj + 1.0;
  bool prevFailed = false, linFail = false, first = true;
  double pol_J = J, pol_pJ = J, last_succ = J;
  double lambda = o->lambda_init, gamma = 3.0, beta = 2.0, mu = 2.0;
  while (out->iterations < o->max_iterations && out->failed_iterations < o->max_iterations &&
         ((deltaX > o->convergence_dx && std::fabs(deltaJ) > o->convergence_dj) || linFail)) {
    if (prevFailed) {
      pol_J = J;
    } else {
      pol_pJ = last_succ;
      last_succ = J;
      pol_J = J;
    }
    bool rebuild = true;
    if (lm && !first) {
      double d2 = 0.0;
      for (int q = 0; q < ncols; ++q) d2 += dx[q] * (lambda * dx[q] + rhs[q]);
      const double rho = (pol_pJ - pol_J) / d2;
      if (prevFailed) {
        mu *= 2;
        lambda *= mu;
        rebuild = false;
      } else if (rho <= 0) {
        mu *= 10;
        lambda *= mu;
        rebuild = false;
      } else if (lambda > 1e-16) {
        const double u1 = 1 / gamma, u2 = 1 - (beta - 1) * std::pow((2 * rho - 1), 3);
        lambda *= (u1 > u2) ? u1 : u2;
        mu = beta;
      } else {
        lambda = 1e-15;
      }
    }
    if (rebuild) {
      if (kb_sp_build(h)) return -1;
      if (kb_sp_get_rhs(h, rhs.data())) return -1;
    } else {
      h->built = true;  // same system, new conditioner
    }
    h->lambda = lm ? lambda : 0.0;
    int ok = 0;
    if (kb_sp_solve(h, tmp.data(), &ok)) return -1;
    if (ok) dx = tmp;
    first = false;
    int accepted = 0;
    if (!ok) {
      prevFailed = true;
      linFail = true;
      out->failed_iterations++;
    } else {
      if (kb_sp_apply_update(h, nullptr, &deltaX)) return -1;
      if (kb_sp_eval_cost(h, &J)) return -1;
      deltaJ = p_J - J;
      if (lm) {
        if (deltaJ < 0.0) {
          if (kb_sp_revert(h)) return -1;
          out->failed_iterations++;
          prevFailed = true;
        } else {
          p_J = J;
          prevFailed = false;
          accepted = 1;
        }
      } else {
        p_J = J;
        accepted = 1;
      }
      out->iterations++;
    }
    h->trace.push_back(ok ? J : NAN);
    h->trace.push_back(lm ? lambda : 0.0);
    h->trace.push_back(deltaX);
    h->trace.push_back(accepted);
    out->passes++;
  }
  out->J_final = p_J;
  out->dx_final = deltaX;
  out->dj_final = deltaJ;
  out->linear_solver_failure = linFail;
  return 0;
}

int kb_sp_get_trace(kb_sp_handle* h, double* trace, int32_t cap) {
  if (!h || !trace) return fail("kb_sp_get_trace: null");
  const int n = std::min<int>(cap, (int)(h->trace.size() / 4));
  std::memcpy(trace, h->trace.data(), sizeof(double) * 4 * n);
  return n;
}

int kb_sp_run_gn_iterations(kb_sp_handle* h, int32_t n_iter, double* seconds) {
  if (!h || n_iter < 0) return fail("kb_sp_run_gn_iterations: bad arguments");
  if (!h->uploaded) return fail("kb_sp_run_gn_iterations: upload observations first");
  KSP_HIP(hipSetDevice(h->device));
  if (!h->gn_graph) {
    hipGraph_t g = nullptr;
    KSP_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    const int rc = enqueue_gn_pass(h);
    hipError_t e = hipStreamEndCapture(h->stream, &g);
    if (rc || e != hipSuccess) return fail("kb_sp_run_gn_iterations: graph capture failed");
    e = hipGraphInstantiate(&h->gn_graph, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    if (e != hipSuccess) return fail("kb_sp_run_gn_iterations: graph instantiate failed");
  }
  KSP_HIP(hipStreamSynchronize(h->stream));
  const auto t0 = std::chrono::steady_clock::now();
  for (int it = 0; it < n_iter; ++it) KSP_HIP(hipGraphLaunch(h->gn_graph, h->stream));
  KSP_HIP(hipStreamSynchronize(h->stream));
  const auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  h->built = h->solved = false;
  return 0;
}

int kb_sp_assemble_stats(kb_sp_handle* h, int32_t n, double* ms, double* bytes) {
  if (!h || !ms || !bytes || n < 1) return fail("kb_sp_assemble_stats: bad arguments");
  if (!h->uploaded) return fail("kb_sp_assemble_stats: upload observations first");
  KSP_HIP(hipSetDevice(h->device));
  SpDev& d = h->d;
  void* args[] = {&d};
  hipEvent_t e0, e1;
  KSP_HIP(hipEventCreate(&e0));
  KSP_HIP(hipEventCreate(&e1));
  double acc = 0.0;
  for (int it = -1; it < n; ++it) {  // it = -1: warm-up
    hipLaunchKernelGGL(k_sp_set_lam, dim3(1), dim3(64), 0, h->stream, d, 0.0);
    KSP_HIP(hipLaunchKernel(h->fn_frames, dim3(frames_grid(h)), dim3(64 * h->N), args, h->lds_frames, h->stream));
    KSP_HIP(hipEventRecord(e0, h->stream));
    KSP_HIP(hipLaunchKernel((const void*)k_sp_assemble, dim3(d.n), dim3(256), args, h->lds_asm, h->stream));
    KSP_HIP(hipEventRecord(e1, h->stream));
    KSP_HIP(hipStreamSynchronize(h->stream));
    float t = 0.0f;
    KSP_HIP(hipEventElapsedTime(&t, e0, e1));
    if (it >= 0) acc += t;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  *ms = acc / n;
  // algorithmic bytes, each once: the frames' spline blocks (FHS doubles) with their basis (4 weights + index), the
  // IMU samples (k_sp_imu_cc's record of IRQ doubles, 12 weights, index), the coefficients and camera / IMU state, the
  // node tables, the node blocks D0, U0, R0 written (+ the motion-error blocks when active)
  *bytes = 8.0 * h->F * (d.FHS + 4) + 4.0 * h->F + h->M * (8.0 * (IRQ + 12) + 4.0) + 8.0 * d.S + 16.0 * h->n +
           8.0 * h->n * (2 * NB * NB + NB * d.m) + (d.mot ? 8.0 * h->n * 2 * NB * NB : 0.0);
  h->built = h->solved = false;
  return 0;
}

int kb_sp_kernel_stats(kb_sp_handle* h, int32_t n, double* ms_out6, double* frames_bytes) {
  if (!h || !ms_out6 || n < 1) return fail("kb_sp_kernel_stats: bad arguments");
  if (!h->uploaded) return fail("kb_sp_kernel_stats: upload observations first");
  KSP_HIP(hipSetDevice(h->device));
  SpDev& d = h->d;
  hipEvent_t ev[7];
  for (auto& e : ev) KSP_HIP(hipEventCreate(&e));
  double acc[6] = {0, 0, 0, 0, 0, 0};
  void* args[] = {&d};
  for (int it = 0; it < n; ++it) {
    hipLaunchKernelGGL(k_sp_set_lam, dim3(1), dim3(64), 0, h->stream, d, 0.0);
    KSP_HIP(hipEventRecord(ev[0], h->stream));
    KSP_HIP(hipLaunchKernel(h->fn_frames, dim3(frames_grid(h)), dim3(64 * h->N), args, h->lds_frames, h->stream));
    KSP_HIP(hipEventRecord(ev[1], h->stream));
    KSP_HIP(hipLaunchKernel((const void*)k_sp_assemble, dim3(d.n), dim3(256), args, h->lds_asm, h->stream));
    hipLaunchKernelGGL(k_sp_reduce_cc, dim3((d.Wc + 63) / 64), dim3(64 * RW), 0, h->stream, d);
    if (d.cq) hipLaunchKernelGGL(k_sp_mcost_build, dim3(1), dim3(256), 0, h->stream, d);
    KSP_HIP(hipEventRecord(ev[2], h->stream));
    launch_reduction(h);  // (zs: the forward half; the one-column back substitution follows the camera solve)
    KSP_HIP(hipEventRecord(ev[3], h->stream));
    if (!d.zsf) hipLaunchKernelGGL(d.zs ? k_sp_zschur : k_sp_schur, dim3(d.nblk_s), dim3(256), h->lds_schur, h->stream, d);
    hipLaunchKernelGGL(k_sp_schur_red, dim3((d.Ws + 63) / 64), dim3(64 * RW), 0, h->stream, d);
    KSP_HIP(hipLaunchKernel(h->fn_camsolve, dim3(1), dim3(64), args, 0, h->stream));
    KSP_HIP(hipEventRecord(ev[4], h->stream));
    if (d.zs && launch_bvec(h)) return -1;
    KSP_HIP(hipEventRecord(ev[5], h->stream));
    hipLaunchKernelGGL(k_sp_update, dim3(d.n), dim3(64), 0, h->stream, d, 1);
    if (launch_cost(h, 1)) return -1;
    KSP_HIP(hipEventRecord(ev[6], h->stream));
    KSP_HIP(hipStreamSynchronize(h->stream));
    float t[6];
    for (int q = 0; q < 6; ++q) KSP_HIP(hipEventElapsedTime(&t[q], ev[q], ev[q + 1]));
    // frames | assemble | reduction (forward + back substitution) | Schur + camera solve | update + cost | pass
    acc[0] += t[0];
    acc[1] += t[1];
    acc[2] += t[2] + t[4];
    acc[3] += t[3];
    acc[4] += t[5];
    float tt;
    KSP_HIP(hipEventElapsedTime(&tt, ev[0], ev[6]));
    acc[5] += tt;
  }
  for (auto& e : ev) hipEventDestroy(e);
  for (int q = 0; q < 6; ++q) ms_out6[q] = acc[q] / n;
  if (frames_bytes) {
    // algorithmic bytes of one k_sp_frames launch: corners (y 16 B + id 2 B), view ranges (8 B per (frame,
    // camera)), frame basis (4 weights + index), the 4 active coefficients per frame, the camera-side state,
    // the per-frame spline blocks written (FHS doubles) and one theta partial row per block; the extra blocks' IMU
    // samples (index, 12 weights, 6 measurements, 4 coefficients read; the IRQ-double record and the partial rows
    // written)
    *frames_bytes = 18.0 * h->NCo + 8.0 * h->F * h->N + 36.0 * h->F + 8.0 * 24 * h->F + 8.0 * d.off_coef +
                    8.0 * d.FHS * h->F + 8.0 * d.Wc * d.nblk_f +
                    h->M * (4.0 + 8.0 * (12 + 6 + 24 + IRQ)) + 8.0 * WI * d.nblk_ic;
  }
  h->built = h->solved = false;
  return 0;
}

}  // extern "C"

#ifdef KB_STAMPS
// diagnostic build only: the KSP_TS timeline (100 MHz ticks) of the last pass
extern "C" int kb_sp_diag_read_ts(kb_sp_handle* h, long long* out, int n) {
  if (!h->d.dbg_ts) return fail("kb_sp_diag_read_ts: no stamp buffer");
  KSP_HIP(hipStreamSynchronize(h->stream));
  KSP_HIP(hipMemcpy(out, h->d.dbg_ts, sizeof(long long) * std::min(n, 320), hipMemcpyDeviceToHost));
  return 0;
}
#endif
