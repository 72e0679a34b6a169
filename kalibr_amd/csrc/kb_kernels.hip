// kb_kernels.hip -- CDNA4 (gfx950) kernels of one Gauss-Newton / Levenberg-Marquardt pass
// over Kalibr2 ReprojectionError terms, FP64 throughout.
//
//   k_prep       camera-only chain quantities L_i = B_{i-1}..B_0 and K_{i,j} (frame independent)
//   k_build      K1+K2+K3: per view, residual + 2x16 Jacobian rows staged in LDS, local
//                16x16 [J|-e]^T[J|-e] by v_mfma_f64_16x16x4; per frame the 6-D adjoint expansion into
//                H_ff, H_fc, g_f; per camera deterministic partial sums for the camera block
//   k_colsum     deterministic column sums of per-block partials
//   k_camexpand  camera block H_cc, g_c from the per-camera sums (K_{i,j} expansion)
//   k_schur      K4a: per frame chol(H_ff + lambda^2 I), Y = L^-1 H_fc, z = L^-1 g_f, sum Y^T Y
//   k_solve      K4b: dense Cholesky of S = H_cc + lambda^2 I - sum Y^T Y, camera dx, camera update
//   k_backsub    K4c+K5: frame dx = L^-T (z - Y dx_c), frame pose update, step statistics
//   k_cost       K1 (cost only) on either state buffer
//   k_pol_*      the Optimizer2 / trust-region state machine, device resident
//
// Reference data flow replaced (paths relative to the reference repository):
//   LinearSystemSolver.cpp:12-92, CompressedColumnJacobianTransposeBuilder(impl).hpp:19-101,
//   SparseCholeskyLinearSystemSolver.cpp:39-89, Cholmod(impl).hpp:180-399, Optimizer2.cpp:183-318,
//   LevenbergMarquardtTrustRegionPolicy.cpp:50-113, GaussNewtonTrustRegionPolicy.cpp:18-39.
#include "kb_device.h"

namespace kb {

typedef double v4d __attribute__((ext_vector_type(4)));

#define KB_WAVE_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// ---------------------------------------------------------------------------------------------
// camera chain: L_i (R|t, 12 doubles) and K_{i,j} = boxTimes(B_{i-1}..B_{j+1}) * M(t_Bj)
// (TransformationExpressionNode.cpp:61-72 chain of boxTimes; TransformationBasic.cpp:49-66 M(t))
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void pose_rt(const double* pose, double* R, double* t) {
  quat2r(pose, R);
  t[0] = pose[4];
  t[1] = pose[5];
  t[2] = pose[6];
}

// (R1|t1) * (R2|t2)
__device__ __forceinline__ void rt_mul(const double* R1, const double* t1, const double* R2, const double* t2,
                                       double* R, double* t) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) R[r * 3 + c] = R1[r * 3 + 0] * R2[0 * 3 + c] + R1[r * 3 + 1] * R2[1 * 3 + c] + R1[r * 3 + 2] * R2[2 * 3 + c];
    t[r] = R1[r * 3 + 0] * t2[0] + R1[r * 3 + 1] * t2[1] + R1[r * 3 + 2] * t2[2] + t1[r];
  }
}

// G = -boxTimes(T_q) M(t_m) = [[R [t_m]x + [t_q]x R, -R], [-R, 0]]  (6x6, row-major), entry (a,b).
// Used with T_q = T_cam_w, t_m = t_f for the frame DV and, negated, for K_{i,j}.
__device__ __forceinline__ double chain_entry(const double* R, const double* tq, const double* tm, int a, int b) {
  if (a < 3 && b < 3) {
    // (R [tm]x)[a][b] + ([tq]x R)[a][b]
    // [x]x = [[0,-x2,x1],[x2,0,-x0],[-x1,x0,0]]
    double s;
    const double r0 = R[a * 3 + 0], r1 = R[a * 3 + 1], r2 = R[a * 3 + 2];
    if (b == 0) s = r1 * tm[2] - r2 * tm[1];
    else if (b == 1) s = -r0 * tm[2] + r2 * tm[0];
    else s = r0 * tm[1] - r1 * tm[0];
    double u;
    const double c0 = R[0 * 3 + b], c1 = R[1 * 3 + b], c2 = R[2 * 3 + b];
    if (a == 0) u = -tq[2] * c1 + tq[1] * c2;
    else if (a == 1) u = tq[2] * c0 - tq[0] * c2;
    else u = -tq[1] * c0 + tq[0] * c1;
    return s + u;
  }
  if (a < 3) return -R[a * 3 + (b - 3)];
  if (b < 3) return -R[(a - 3) * 3 + b];
  return 0.0;
}

__global__ void k_prep(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || !c->do_build)) return;
  // one block; thread t < N: L_t ; threads over (i,j,entry) for K
  __shared__ double sR[KB_MAX_CAMS][9], st[KB_MAX_CAMS][3];  // baseline B_j
  __shared__ double LR[KB_MAX_CAMS][9], Lt[KB_MAX_CAMS][3];
  const double* s = d.state + (size_t)c->cur * d.S;
  const int N = d.N;
  if (threadIdx.x < N - 1) pose_rt(s + d.off_base + 7 * threadIdx.x, sR[threadIdx.x], st[threadIdx.x]);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 0; q < 9; ++q) LR[0][q] = (q % 4 == 0) ? 1.0 : 0.0;
    Lt[0][0] = Lt[0][1] = Lt[0][2] = 0.0;
    for (int i = 1; i < N; ++i) rt_mul(sR[i - 1], st[i - 1], LR[i - 1], Lt[i - 1], LR[i], Lt[i]);
    for (int i = 0; i < N; ++i) {
      for (int q = 0; q < 9; ++q) d.camL[i * 12 + q] = LR[i][q];
      for (int q = 0; q < 3; ++q) d.camL[i * 12 + 9 + q] = Lt[i][q];
    }
  }
  __syncthreads();
  // K_{i,j} for j < i: Q = B_{i-1}..B_{j+1} (identity when j = i-1); K = -G(Q, t_Bj)
  for (int idx = threadIdx.x; idx < N * N * 36; idx += blockDim.x) {
    const int e = idx % 36, ij = idx / 36, i = ij / N, j = ij % N;
    double val = 0.0;
    if (j < i) {
      double QR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, Qt[3] = {0, 0, 0};
      for (int k = j + 1; k < i; ++k) {
        double R2[9], t2[3];
        rt_mul(sR[k], st[k], QR, Qt, R2, t2);
        for (int q = 0; q < 9; ++q) QR[q] = R2[q];
        for (int q = 0; q < 3; ++q) Qt[q] = t2[q];
      }
      val = -chain_entry(QR, Qt, st[j], e / 6, e % 6);
    }
    d.camK[idx] = val;
  }
}

// ---------------------------------------------------------------------------------------------
// k_build: one block = a group of frames, one wave per camera slot (cameras w, w+WPB, ...).
// ---------------------------------------------------------------------------------------------
constexpr int XS = 17;  // LDS row stride (doubles) of the 64 x 16 Jacobian-row tile

__global__ void __launch_bounds__(256) k_build(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || !c->do_build)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int WPB = blockDim.x >> 6;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int N = d.N, C = d.C;
  double* Xw = sm + wave * 64 * XS;                 // [64][XS]
  double* Hw = sm + WPB * 64 * XS + wave * 256;     // per-wave local 16x16
  double* Ww = sm + WPB * 64 * XS + WPB * 256 + wave * 64;  // wave scratch: R(9) t(3) tf(3) G(36)
  double* camsum = sm + WPB * 64 * XS + WPB * 256 + WPB * 64;  // [N][256]
  double* Pv = camsum + N * 256;                    // [N][36]
  double* dH = Pv + N * 36;                         // [N][36]
  double* dg = dH + N * 36;                         // [N][8]
  const double* s = d.state + (size_t)c->cur * d.S;

  for (int q = threadIdx.x; q < N * 256; q += blockDim.x) camsum[q] = 0.0;
  __syncthreads();

  const int f0 = blockIdx.x * d.gframes;
  const int f1 = min(d.F, f0 + d.gframes);
  const int mrow = lane >> 4, mcol = lane & 15;
  for (int f = f0; f < f1; ++f) {
    const double* fp = s + d.off_frame + 7 * f;
    // T_f^-1 = (Rf^T | -Rf^T tf)
    double Rf[9];
    quat2r(fp, Rf);
    const double tf[3] = {fp[4], fp[5], fp[6]};
    double Ri[9], ti[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) Ri[r * 3 + cc] = Rf[cc * 3 + r];
      ti[r] = -(Ri[r * 3 + 0] * tf[0] + Ri[r * 3 + 1] * tf[1] + Ri[r * 3 + 2] * tf[2]);
    }
    for (int cam = wave; cam < N; cam += WPB) {
      const int v = d.frame_vcam[f * N + cam];
      const int model = d.model[cam], nin = d.nintr[cam];
      const double* intr = s + cam * KB_MAX_INTR;
      // T_cam_w = L_cam * T_f^-1
      double R[9], t[3];
      rt_mul(d.camL + cam * 12, d.camL + cam * 12 + 9, Ri, ti, R, t);
      v4d acc = {0.0, 0.0, 0.0, 0.0};
      if (v >= 0) {
        const int o0 = d.view_off[v], o1 = d.view_off[v + 1];
        for (int base = o0; base < o1; base += 64) {
          const int k = base + lane;
          double xr[2][16];
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int q = 0; q < 16; ++q) xr[r][q] = 0.0;
          if (k < o1) {
            const int cid = d.cid[k];
            const double X0 = d.target[3 * cid], X1 = d.target[3 * cid + 1], X2 = d.target[3 * cid + 2];
            const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
            const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
            const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
            double u, w, Jp[6], Ji[2 * KB_MAX_INTR];
            project_jac(model, intr, p0, p1, p2, u, w, Jp, Ji);
            const double2 yv = d.y[k];
            const double e0 = yv.x - u, e1 = yv.y - w;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
              const double j0 = Jp[3 * r], j1 = Jp[3 * r + 1], j2 = Jp[3 * r + 2];
              // J_delta = -Jp [I | [p]x]   (HomogeneousExpressionNode.cpp:71-81, boxMinus)
              xr[r][0] = -j0;
              xr[r][1] = -j1;
              xr[r][2] = -j2;
              xr[r][3] = -(j1 * p2 - j2 * p1);
              xr[r][4] = -(-j0 * p2 + j2 * p0);
              xr[r][5] = -(j0 * p1 - j1 * p0);
              // intrinsics: -Jp, -Jd (CameraDesignVariable.hpp(impl):38-54)
#pragma unroll
              for (int q = 0; q < 9; ++q) xr[r][6 + q] = (q < nin) ? -Ji[r * KB_MAX_INTR + q] : 0.0;
              xr[r][15] = -(r == 0 ? e0 : e1);  // column 15 carries -e: H[:,15] = rhs, H[15][15] = chi^2
            }
          }
          // two phases of 32 corners (64 rows) through the LDS tile, 16 MFMA k-steps each
#pragma unroll
          for (int ph = 0; ph < 2; ++ph) {
            if (ph == 1 && base + 32 >= o1) break;  // wave-uniform
            if ((lane >> 5) == ph) {
              const int rr = 2 * (lane & 31);
#pragma unroll
              for (int q = 0; q < 16; ++q) {
                Xw[rr * XS + q] = xr[0][q];
                Xw[(rr + 1) * XS + q] = xr[1][q];
              }
            }
            KB_WAVE_SYNC();
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
              const double xv = Xw[(4 * ks + mrow) * XS + mcol];
              acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xv, xv, acc, 0, 0, 0);
            }
            KB_WAVE_SYNC();
          }
        }
      }
      // f64 MFMA C/D layout: lane l, reg r -> row (l>>4) + 4r, col l&15
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int idx = (mrow + 4 * r) * 16 + mcol;
        Hw[idx] = acc[r];
        camsum[cam * 256 + idx] += acc[r];
      }
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 9; ++q) Ww[q] = R[q];
        Ww[9] = t[0]; Ww[10] = t[1]; Ww[11] = t[2];
        Ww[12] = tf[0]; Ww[13] = tf[1]; Ww[14] = tf[2];
      }
      KB_WAVE_SYNC();
      // frame-DV chain G_v = -boxTimes(T_cam_w) M(t_f) (6x6)
      double* G = Ww + 16;
      if (lane < 36) G[lane] = chain_entry(Ww, Ww + 9, Ww + 12, lane / 6, lane % 6);
      KB_WAVE_SYNC();
      const bool has = v >= 0;
      if (lane < 36) {
        const int a = lane / 6, b = lane % 6;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += G[k * 6 + a] * Hw[k * 16 + b];
        Pv[cam * 36 + lane] = has ? sacc : 0.0;  // P_v = G^T H_dd
      } else if (lane < 42) {
        const int a = lane - 36;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += G[k * 6 + a] * Hw[k * 16 + 15];
        dg[cam * 8 + a] = has ? sacc : 0.0;  // G^T g_d
      }
      KB_WAVE_SYNC();
      if (lane < 36) {
        const int a = lane / 6, b = lane % 6;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += Pv[cam * 36 + a * 6 + k] * G[k * 6 + b];
        dH[cam * 36 + lane] = sacc;  // P_v G_v
      }
      if (lane < 6 * nin) {
        const int a = lane / nin, q = lane % nin;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += G[k * 6 + a] * Hw[k * 16 + 6 + q];
        d.Hfc[((size_t)f * 6 + a) * C + d.col_intr[cam] + q] = has ? sacc : 0.0;  // G^T H_dI
      }
      KB_WAVE_SYNC();
    }
    __syncthreads();
    // frame outputs: sums over the frame's views in camera order
    for (int q = threadIdx.x; q < 42 + 36 * (N - 1); q += blockDim.x) {
      if (q < 36) {
        double sacc = 0.0;
        for (int cam = 0; cam < N; ++cam) sacc += dH[cam * 36 + q];
        d.Hff[(size_t)f * 36 + q] = sacc;
      } else if (q < 42) {
        double sacc = 0.0;
        for (int cam = 0; cam < N; ++cam) sacc += dg[cam * 8 + q - 36];
        d.gf[(size_t)f * 6 + q - 36] = sacc;
      } else {
        // H_f,B_j = sum_{i > j} P_i K_{i,j}
        const int e = q - 42, j = e / 36, ab = e % 36, a = ab / 6, b = ab % 6;
        double sacc = 0.0;
        for (int i = j + 1; i < N; ++i) {
          const double* K = d.camK + (size_t)(i * N + j) * 36;
#pragma unroll
          for (int k = 0; k < 6; ++k) sacc += Pv[i * 36 + a * 6 + k] * K[k * 6 + b];
        }
        d.Hfc[((size_t)f * 6 + a) * C + d.col_base[j] + b] = sacc;
      }
    }
    __syncthreads();
  }
  // per-camera partial sums (upper triangle of the 16x16) of this block
  for (int q = threadIdx.x; q < N * 136; q += blockDim.x) {
    const int cam = q / 136, e = q % 136;
    const int a = d16_row(e), b = d16_col(e);
    d.campart[(size_t)blockIdx.x * N * 136 + q] = camsum[cam * 256 + a * 16 + b];
  }
}

// ---------------------------------------------------------------------------------------------
// deterministic column sums: out[w] = sum_b in[b][w] (fixed order)
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_colsum(KbDev d, const double* in, int B, int W, double* out, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate == 1 && (c->done || !c->do_build)) return;
  if (gate == 2 && c->done) return;
  __shared__ double part[4][64];
  const int l = threadIdx.x & 63, w4 = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + l;
  double s = 0.0;
  if (e < W)
    for (int b = w4; b < B; b += 4) s += in[(size_t)b * W + e];
  part[w4][l] = s;
  __syncthreads();
  if (w4 == 0 && e < W) out[e] = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
}

// ---------------------------------------------------------------------------------------------
// camera block H_cc, g_c from the per-camera local sums
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_camexpand(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || !c->do_build)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int N = d.N, C = d.C;
  double* Hs = sm;                    // [N][256] full per-camera 16x16 sums
  double* T = Hs + N * 256;           // [N][N][36]: T_{i,k} = H_dd,i K_{i,k}
  const double* cs = d.camsum;        // [N][136] upper packed
  for (int q = threadIdx.x; q < N * 256; q += blockDim.x) {
    const int cam = q / 256, a = (q % 256) / 16, b = q % 16;
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    Hs[q] = cs[cam * 136 + d16_index(lo, hi)];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < N * N * 36; q += blockDim.x) {
    const int e = q % 36, ik = q / 36, i = ik / N, k = ik % N;
    double s = 0.0;
    if (k < i) {
      const int a = e / 6, b = e % 6;
      const double* K = d.camK + (size_t)(i * N + k) * 36;
#pragma unroll
      for (int m = 0; m < 6; ++m) s += Hs[i * 256 + a * 16 + m] * K[m * 6 + b];
    }
    T[q] = s;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < C * C + C + 1; q += blockDim.x) {
    if (q == C * C + C) {
      double s = 0.0;
      for (int i = 0; i < N; ++i) s += Hs[i * 256 + 255];
      d.cost_build[0] = s;
      continue;
    }
    const bool isg = q >= C * C;
    const int p = isg ? q - C * C : q / C;
    const int r = isg ? 15 : q % C;  // r == 15 marks the gradient column
    const int kp = d.colinfo[p] >> 16, ip = (d.colinfo[p] >> 8) & 0xff, xp = d.colinfo[p] & 0xff;
    double s = 0.0;
    if (isg) {
      if (kp == 0) {
        s = Hs[ip * 256 + (6 + xp) * 16 + 15];
      } else {
        for (int i = ip + 1; i < N; ++i) {
          const double* K = d.camK + (size_t)(i * N + ip) * 36;
#pragma unroll
          for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Hs[i * 256 + a * 16 + 15];
        }
      }
      d.gc[p] = s;
      continue;
    }
    const int kq = d.colinfo[r] >> 16, iq = (d.colinfo[r] >> 8) & 0xff, xq = d.colinfo[r] & 0xff;
    if (kp == 0 && kq == 0) {
      if (ip == iq) s = Hs[ip * 256 + (6 + xp) * 16 + 6 + xq];
    } else if (kp == 0 && kq == 1) {
      if (iq < ip) {
        const double* K = d.camK + (size_t)(ip * N + iq) * 36;
#pragma unroll
        for (int b = 0; b < 6; ++b) s += Hs[ip * 256 + (6 + xp) * 16 + b] * K[b * 6 + xq];
      }
    } else if (kp == 1 && kq == 0) {
      if (ip < iq) {
        const double* K = d.camK + (size_t)(iq * N + ip) * 36;
#pragma unroll
        for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Hs[iq * 256 + a * 16 + 6 + xq];
      }
    } else {
      const int m = ip > iq ? ip : iq;
      for (int i = m + 1; i < N; ++i) {
        const double* K = d.camK + (size_t)(i * N + ip) * 36;
        const double* Tq = T + (size_t)(i * N + iq) * 36;
#pragma unroll
        for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Tq[a * 6 + xq];
      }
    }
    d.Hcc[q] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// k_schur: per frame chol(H_ff + lambda^2 I), Y = L^-1 H_fc, z = L^-1 g_f; sum Y^T Y, Y^T z
// ---------------------------------------------------------------------------------------------
constexpr int kSchurM = 24;  // entries per thread (256 threads) -> W <= 6144, C <= 109

__global__ void __launch_bounds__(256) k_schur(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && c->done) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int C = d.C, Wt = C * (C + 1) / 2, W = Wt + C;
  double* Y = sm;            // [6][C]
  double* L = Y + 6 * C;     // [36]
  double* z = L + 36;        // [8]
  __shared__ int okl;
  const double lam = gate ? c->lambda : d.host_lambda;
  const double lam2 = lam * lam;
  double acc[kSchurM];
  int ab[kSchurM];
#pragma unroll
  for (int m = 0; m < kSchurM; ++m) {
    acc[m] = 0.0;
    const int e = threadIdx.x + 256 * m;
    ab[m] = (e < Wt) ? d.tri[e] : -1;
  }
  if (threadIdx.x == 0) okl = 1;
  const int f0 = blockIdx.x * d.gframes, f1 = min(d.F, f0 + d.gframes);
  for (int f = f0; f < f1; ++f) {
    if (threadIdx.x < 36) L[threadIdx.x] = d.Hff[(size_t)f * 36 + threadIdx.x] + ((threadIdx.x % 7 == 0) ? lam2 : 0.0);
    __syncthreads();
    if (threadIdx.x == 0) {
      // in-place Cholesky, lower
      for (int j = 0; j < 6; ++j) {
        double dd = L[j * 6 + j];
        for (int k = 0; k < j; ++k) dd -= L[j * 6 + k] * L[j * 6 + k];
        if (!(dd > 0.0)) okl = 0;
        dd = sqrt(dd);
        L[j * 6 + j] = dd;
        for (int i = j + 1; i < 6; ++i) {
          double s2 = L[i * 6 + j];
          for (int k = 0; k < j; ++k) s2 -= L[i * 6 + k] * L[j * 6 + k];
          L[i * 6 + j] = s2 / dd;
        }
      }
      for (int q = 0; q < 36; ++q) d.Lf[(size_t)f * 36 + q] = L[q];
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < C) {
      double yv[6];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        double s2 = d.Hfc[((size_t)f * 6 + r) * C + t];
#pragma unroll
        for (int k = 0; k < r; ++k) s2 -= L[r * 6 + k] * yv[k];
        yv[r] = s2 / L[r * 6 + r];
        Y[r * C + t] = yv[r];
        d.Yf[((size_t)f * 6 + r) * C + t] = yv[r];
      }
    } else if (t == 255) {
      double zv[6];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        double s2 = d.gf[(size_t)f * 6 + r];
#pragma unroll
        for (int k = 0; k < r; ++k) s2 -= L[r * 6 + k] * zv[k];
        zv[r] = s2 / L[r * 6 + r];
        z[r] = zv[r];
        d.zf[(size_t)f * 6 + r] = zv[r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kSchurM; ++m) {
      const int e = threadIdx.x + 256 * m;
      if (e < Wt) {
        const int a = ab[m] >> 16, b = ab[m] & 0xffff;
        double s2 = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) s2 += Y[r * C + a] * Y[r * C + b];
        acc[m] += s2;
      } else if (e < W) {
        const int a = e - Wt;
        double s2 = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) s2 += Y[r * C + a] * z[r];
        acc[m] += s2;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int m = 0; m < kSchurM; ++m) {
    const int e = threadIdx.x + 256 * m;
    if (e < W) d.schurpart[(size_t)blockIdx.x * (W + 1) + e] = acc[m];
  }
  // entry W counts blocks with a non-positive-definite H_ff + lambda^2 I (summed over blocks and ranks)
  if (threadIdx.x == 0) d.schurpart[(size_t)blockIdx.x * (W + 1) + W] = okl ? 0.0 : 1.0;
}

// ---------------------------------------------------------------------------------------------
// k_solve: S = H_cc + lambda^2 I - sum Y^T Y, b = g_c - sum Y^T z; chol; dx_c; camera update
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_solve(KbDev d, int gate, int do_update) {
  KbCtrl* c = d.ctrl;
  if (gate && c->done) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int C = d.C, Wt = C * (C + 1) / 2;
  double* S = sm;  // [C][C]
  __shared__ int okl;
  __shared__ double red[4][64];
  const double lam = gate ? c->lambda : d.host_lambda;
  const double lam2 = lam * lam;
  const double* ss = d.schursum;
  for (int q = threadIdx.x; q < C * C; q += blockDim.x) {
    const int a = q / C, b = q % C;
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    const int e = lo * C - lo * (lo - 1) / 2 + (hi - lo);
    S[q] = d.Hcc[q] + ((a == b) ? lam2 : 0.0) - ss[e];
  }
  if (threadIdx.x == 0) okl = (c->solve_ok != 0) && !(ss[Wt + C] > 0.0);
  __syncthreads();
  // right-looking Cholesky (lower), 3 barriers per column
  for (int k = 0; k < C; ++k) {
    if (threadIdx.x == 0) {
      const double dd = S[k * C + k];
      if (!(dd > 0.0)) okl = 0;
      S[k * C + k] = sqrt(dd);
    }
    __syncthreads();
    const double dk = S[k * C + k];
    for (int i = k + 1 + threadIdx.x; i < C; i += blockDim.x) S[i * C + k] /= dk;
    __syncthreads();
    const int n = C - k - 1;
    for (int q = threadIdx.x; q < n * n; q += blockDim.x) {
      const int i = k + 1 + q / n, j = k + 1 + q % n;
      if (j <= i) S[i * C + j] -= S[i * C + k] * S[j * C + k];
    }
    __syncthreads();
  }
  const bool ok = okl != 0;
  if (!ok) {
    if (threadIdx.x == 0) c->solve_ok = 0;
    return;
  }
  // triangular solves by wave 0; row i held by lane i & 63 (slot i >> 6)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double bv[2];
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int i = lane + 64 * sl;
      bv[sl] = (i < C) ? d.gc[i] - ss[Wt + i] : 0.0;
    }
    for (int k = 0; k < C; ++k) {
      const double bk = __shfl(bv[k >> 6], k & 63) / S[k * C + k];
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        const int i = lane + 64 * sl;
        if (i == k) bv[sl] = bk;
        else if (i > k && i < C) bv[sl] -= S[i * C + k] * bk;
      }
    }
    for (int k = C - 1; k >= 0; --k) {
      const double xk = __shfl(bv[k >> 6], k & 63) / S[k * C + k];
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        const int i = lane + 64 * sl;
        if (i == k) bv[sl] = xk;
        else if (i < k) bv[sl] -= S[k * C + i] * xk;
      }
    }
    double mx = 0.0, dd = 0.0, dr = 0.0;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int i = lane + 64 * sl;
      if (i < C) {
        const double g = d.gc[i];
        d.dx[i] = bv[sl];
        d.rhs[i] = g;
        mx = fmax(mx, fabs(bv[sl]));
        dd += bv[sl] * bv[sl];
        dr += bv[sl] * g;
      }
    }
    red[0][lane] = mx;
    red[1][lane] = dd;
    red[2][lane] = dr;
    KB_WAVE_SYNC();
    if (lane == 0) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0;
      for (int q = 0; q < 64; ++q) {
        a0 = fmax(a0, red[0][q]);
        a1 += red[1][q];
        a2 += red[2][q];
      }
      d.camstat[0] = a0;
      d.camstat[1] = a1;
      d.camstat[2] = a2;
    }
  }
  if (do_update) {
    __syncthreads();
    const double* in = d.state + (size_t)c->cur * d.S;
    double* out = d.state + (size_t)(1 - c->cur) * d.S;
    const int N = d.N;
    for (int q = threadIdx.x; q < N * KB_MAX_INTR; q += blockDim.x) {
      const int cam = q / KB_MAX_INTR, x = q % KB_MAX_INTR;
      out[q] = in[q] + ((x < d.nintr[cam]) ? d.dx[d.col_intr[cam] + x] : 0.0);
    }
    if (threadIdx.x < N - 1) {
      const int j = threadIdx.x;
      update_pose(in + d.off_base + 7 * j, d.dx + d.col_base[j], out + d.off_base + 7 * j);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// k_backsub: one wave per frame: dx_f = L^-T (z - Y dx_c); optional pose update; statistics
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_backsub(KbDev d, int gate, int do_update) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || !c->solve_ok)) return;
  __shared__ double st4[4][3];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int f = blockIdx.x * 4 + wave;
  const int C = d.C;
  double mx = 0.0, dd = 0.0, dr = 0.0;
  if (f < d.F) {
    double w[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      double s = 0.0;
      for (int q = lane; q < C; q += 64) s += d.Yf[((size_t)f * 6 + r) * C + q] * d.dx[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
      w[r] = d.zf[(size_t)f * 6 + r] - s;
    }
    const double* L = d.Lf + (size_t)f * 36;
#pragma unroll
    for (int r = 5; r >= 0; --r) {
      double s = w[r];
#pragma unroll
      for (int k = r + 1; k < 6; ++k) s -= L[k * 6 + r] * w[k];
      w[r] = s / L[r * 6 + r];
    }
    if (lane < 6) {
      double xv = w[0];
#pragma unroll
      for (int r = 1; r < 6; ++r) xv = (lane == r) ? w[r] : xv;
      const double g = d.gf[(size_t)f * 6 + lane];
      d.dx[C + 6 * f + lane] = xv;
      d.rhs[C + 6 * f + lane] = g;
    }
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const double g = d.gf[(size_t)f * 6 + r];
        mx = fmax(mx, fabs(w[r]));
        dd += w[r] * w[r];
        dr += w[r] * g;
      }
      if (do_update) {
        const double* in = d.state + (size_t)c->cur * d.S + d.off_frame + 7 * f;
        double* out = d.state + (size_t)(1 - c->cur) * d.S + d.off_frame + 7 * f;
        update_pose(in, w, out);
      }
    }
  }
  if (lane == 0) {
    st4[wave][0] = mx;
    st4[wave][1] = dd;
    st4[wave][2] = dr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
      a0 = fmax(a0, st4[q][0]);
      a1 += st4[q][1];
      a2 += st4[q][2];
    }
    d.statpart[(size_t)blockIdx.x * 3 + 0] = a0;
    d.statpart[(size_t)blockIdx.x * 3 + 1] = a1;
    d.statpart[(size_t)blockIdx.x * 3 + 2] = a2;
  }
}

// ---------------------------------------------------------------------------------------------
// k_cost: one wave per view on state buffer (cur ^ which); per-block partial sums
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_cost(KbDev d, int gate, int which) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || !c->solve_ok)) return;
  __shared__ double part[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + wave;
  const double* s = d.state + (size_t)(c->cur ^ which) * d.S;
  double acc = 0.0;
  if (v < d.V) {
    const int f = d.view_frame[v], cam = d.view_cam[v];
    // T_cam_w = B_{cam-1} .. B_0 T_f^-1 on this state
    double R[9], t[3], Rf[9];
    const double* fp = s + d.off_frame + 7 * f;
    quat2r(fp, Rf);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) R[r * 3 + cc] = Rf[cc * 3 + r];
      t[r] = -(Rf[0 * 3 + r] * fp[4] + Rf[1 * 3 + r] * fp[5] + Rf[2 * 3 + r] * fp[6]);
    }
    for (int j = 0; j < cam; ++j) {
      double RB[9], tB[3], R2[9], t2[3];
      pose_rt(s + d.off_base + 7 * j, RB, tB);
      rt_mul(RB, tB, R, t, R2, t2);
#pragma unroll
      for (int q = 0; q < 9; ++q) R[q] = R2[q];
#pragma unroll
      for (int q = 0; q < 3; ++q) t[q] = t2[q];
    }
    const int model = d.model[cam];
    const double* intr = s + cam * KB_MAX_INTR;
    const int o0 = d.view_off[v], o1 = d.view_off[v + 1];
    for (int k = o0 + lane; k < o1; k += 64) {
      const int cid = d.cid[k];
      const double X0 = d.target[3 * cid], X1 = d.target[3 * cid + 1], X2 = d.target[3 * cid + 2];
      const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
      const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
      const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
      double u, w;
      project(model, intr, p0, p1, p2, u, w);
      const double2 yv = d.y[k];
      const double e0 = yv.x - u, e1 = yv.y - w;
      acc += e0 * e0 + e1 * e1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  }
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) d.costpart[blockIdx.x] = ((part[0] + part[1]) + part[2]) + part[3];
}

// fixed-order block reduction helper (one block of 256)
__device__ double block_sum(const double* in, int n, double* sh) {
  double s = 0.0;
  for (int q = threadIdx.x; q < n; q += blockDim.x) s += in[q];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}
__device__ double block_max(const double* in, int n, int stride, double* sh) {
  double s = 0.0;
  for (int q = threadIdx.x; q < n; q += blockDim.x) s = fmax(s, in[(size_t)q * stride]);
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}
__device__ double block_sum_strided(const double* in, int n, int stride, double* sh) {
  double s = 0.0;
  for (int q = threadIdx.x; q < n; q += blockDim.x) s += in[(size_t)q * stride];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

// red[0] = cost (sum of costpart); with stats: red[1] = dx.dx, red[2] = dx.rhs, red[3] = max|dx|
__global__ void __launch_bounds__(256) k_reduce(KbDev d, int gate, int with_stats) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || !c->solve_ok)) return;
  __shared__ double sh[256];
  const double cost = block_sum(d.costpart, d.nblk_cost, sh);
  double dd = 0.0, dr = 0.0, mx = 0.0;
  if (with_stats) {
    mx = block_max(d.statpart, d.nblk_bs, 3, sh);
    dd = block_sum_strided(d.statpart + 1, d.nblk_bs, 3, sh);
    dr = block_sum_strided(d.statpart + 2, d.nblk_bs, 3, sh);
  }
  if (threadIdx.x == 0) {
    d.red_local[0] = cost;
    d.red_local[1] = dd + (with_stats ? d.camstat[1] : 0.0);
    d.red_local[2] = dr + (with_stats ? d.camstat[2] : 0.0);
    d.red_local[3] = with_stats ? fmax(mx, d.camstat[0]) : 0.0;
  }
}

// ---------------------------------------------------------------------------------------------
// Optimizer2 + trust-region state machine
// ---------------------------------------------------------------------------------------------
__global__ void k_pol_init(KbDev d, KbOpts o) {
  KbCtrl* c = d.ctrl;
  const double J = d.red[0];
  c->J = J;
  c->p_J = J;
  c->J_start = J;
  c->deltaX = o.eps_x + 1.0;
  c->deltaJ = o.eps_j + 1.0;
  c->prev_failed = 0;
  c->lin_fail = 0;
  c->iterations = 0;
  c->failed_iterations = 0;
  c->max_iterations = o.max_iterations;
  c->eps_x = o.eps_x;
  c->eps_j = o.eps_j;
  c->policy = o.policy;
  // TrustRegionPolicy::optimizationStarting (TrustRegionPolicy.cpp:30-37), LM (:38-46)
  c->pol_J = J;
  c->pol_pJ = J;
  c->last_succ = J;
  c->first = 1;
  c->lambda = o.policy == 0 ? o.lambda_init : 0.0;
  c->mu = 2.0;
  c->dxdx = 0.0;
  c->dxrhs = 0.0;
  c->done = 0;
  c->do_build = 0;
  c->solve_ok = 1;
  c->n_trace = 0;
  c->passes = 0;
}

// while-condition (Optimizer2.cpp:215-219) + TrustRegionPolicy::solveSystem prelude (:39-52)
// + LM lambda schedule (LevenbergMarquardtTrustRegionPolicy.cpp:50-84) or GN (always build).
__global__ void k_pol_pre(KbDev d) {
  KbCtrl* c = d.ctrl;
  if (c->done) return;
  const bool cont = c->iterations < c->max_iterations && c->failed_iterations < c->max_iterations &&
                    ((c->deltaX > c->eps_x && fabs(c->deltaJ) > c->eps_j) || c->lin_fail);
  if (!cont) {
    c->done = 1;
    return;
  }
  const double J = c->J;
  if (c->prev_failed) {
    c->pol_J = J;
  } else {
    c->pol_pJ = c->last_succ;
    c->last_succ = J;
    c->pol_J = J;
  }
  c->solve_ok = 1;
  if (c->policy == 0) {
    if (c->first) {
      c->do_build = 1;
    } else {
      const double d2 = c->lambda * c->dxdx + c->dxrhs;  // dx^T (lambda dx + rhs)
      const double rho = (c->pol_pJ - c->pol_J) / d2;
      if (c->prev_failed) {
        c->mu *= 2;
        c->lambda *= c->mu;
        c->do_build = 0;
      } else if (rho <= 0) {
        c->mu *= 10;
        c->lambda *= c->mu;
        c->do_build = 0;
      } else {
        c->do_build = 1;
        if (c->lambda > 1e-16) {
          const double gamma = 3.0, beta = 2.0;
          const double u1 = 1 / gamma;
          const double u2 = 1 - (beta - 1) * pow((2 * rho - 1), 3.0);
          if (u1 > u2)
            c->lambda *= u1;
          else
            c->lambda *= u2;
          c->mu = beta;
        } else {
          c->lambda = 1e-15;
        }
      }
    }
  } else {
    c->do_build = 1;
  }
  c->first = 0;
}

// accept / revert (Optimizer2.cpp:221-259)
__global__ void k_pol_post(KbDev d) {
  KbCtrl* c = d.ctrl;
  if (c->done) return;
  double J = 0.0, dX = c->deltaX;
  int accepted = 0;
  if (!c->solve_ok) {
    c->prev_failed = 1;
    c->lin_fail = 1;
    c->failed_iterations++;
    J = NAN;
  } else {
    J = d.red[0];
    dX = d.red[3];
    c->dxdx = d.red[1];
    c->dxrhs = d.red[2];
    c->deltaX = dX;
    c->J = J;
    c->deltaJ = c->p_J - J;
    if (c->policy == 0) {
      if (c->deltaJ < 0.0) {
        c->failed_iterations++;
        c->prev_failed = 1;
      } else {
        c->cur = 1 - c->cur;
        c->p_J = J;
        c->prev_failed = 0;
        accepted = 1;
      }
    } else {
      c->cur = 1 - c->cur;
      c->p_J = J;
      accepted = 1;
    }
    c->iterations++;
  }
  if (c->n_trace < d.trace_cap) {
    double* tr = d.trace + 4 * c->n_trace;
    tr[0] = J;
    tr[1] = c->lambda;
    tr[2] = dX;
    tr[3] = accepted;
    c->n_trace++;
  }
  c->passes++;
}

// per-call update (kb_apply_update): all DVs from state[cur] -> state[1-cur]
__global__ void __launch_bounds__(256) k_update_all(KbDev d) {
  KbCtrl* c = d.ctrl;
  const double* in = d.state + (size_t)c->cur * d.S;
  double* out = d.state + (size_t)(1 - c->cur) * d.S;
  const int N = d.N;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < N * KB_MAX_INTR) {
    const int cam = t / KB_MAX_INTR, x = t % KB_MAX_INTR;
    out[t] = in[t] + ((x < d.nintr[cam]) ? d.dx[d.col_intr[cam] + x] : 0.0);
  }
  if (t < N - 1) update_pose(in + d.off_base + 7 * t, d.dx + d.col_base[t], out + d.off_base + 7 * t);
  if (t < d.F) update_pose(in + d.off_frame + 7 * t, d.dx + d.C + 6 * t, out + d.off_frame + 7 * t);
}

__global__ void k_set_cur(KbDev d, int flip) {
  if (flip) d.ctrl->cur = 1 - d.ctrl->cur;
}

// f64 MFMA fragment-layout self test: D = A * B (16x16x16 in 4 k-steps) with asymmetric A and B;
// lane l supplies A[l&15][k0 + (l>>4)] and B[k0 + (l>>4)][l&15]; D read back through the C/D map
// row = (l>>4) + 4r, col = l&15 (the layout k_build relies on).
__device__ __forceinline__ double st_a(int i, int k) { return (i == k) ? 1.0 : 0.0; }
__device__ __forceinline__ double st_b(int k, int j) { return k * 16.0 + j + 0.25 * ((k * 5 + j * 3) % 7); }
__global__ void k_selftest_mfma(double* out, int use_identity) {
  const int lane = threadIdx.x;
  v4d acc = {0, 0, 0, 0};
  for (int ks = 0; ks < 4; ++ks) {
    const int k = 4 * ks + (lane >> 4), ij = lane & 15;
    const double a = use_identity ? st_a(ij, k) : (ij * 0.5 + k * 0.125 + ((ij * 3 + k) % 5));
    const double b = st_b(k, ij);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) out[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
}

}  // namespace kb
