// kb_kernels.hip -- CDNA4 (gfx950) kernels of one Gauss-Newton / Levenberg-Marquardt pass
// over Kalibr2 ReprojectionError terms, FP64 throughout.
//
// One optimizer pass (device-resident loop, every kernel gated on ctrl):
//   k_pre        (loop start / per-call) policy prelude + camera chains L_i, K_{i,j} of the current state
//   k_build      K1+K2+K3 (+K4a fused): per view residual + 2x16 Jacobian rows staged in LDS,
//                local 16x16 [J|-e]^T[J|-e] on v_mfma_f64_16x16x4; per frame the 6-D adjoint expansion
//                into H_ff, H_fc, g_f and, fused, chol(H_ff + lambda^2 I), Y = L^-1 H_fc, z = L^-1 g_f,
//                block partials of sum Y^T Y, Y^T z and of the per-camera local sums
//   k_schur      K4a alone (LM passes that do not rebuild: lambda changed only)
//   k_colsum     stage-1 deterministic column sums of the block partials (8 row splits)
//   k_solve      K4b: camera block H_cc / g_c expansion, S = H_cc + lambda^2 I - sum Y^T Y, LDL^T,
//                camera dx, camera DV update, camera chains of the candidate state
//   k_backsub    K4c+K5(+K1): frame dx = L^-T (z - Y dx_c), pose update, cost of the frame's views at the
//                new state, step statistics; its last block reduces them and runs the accept/revert policy
//                and the next pass's prelude (k_policy after an all-reduce when sharded)
//
// Reference data flow replaced (paths relative to the reference repository):
//   LinearSystemSolver.cpp:12-92, CompressedColumnJacobianTransposeBuilder(impl).hpp:19-101,
//   SparseCholeskyLinearSystemSolver.cpp:39-89, Cholmod(impl).hpp:180-399, Optimizer2.cpp:183-318,
//   TrustRegionPolicy.cpp:39-57, LevenbergMarquardtTrustRegionPolicy.cpp:50-113,
//   GaussNewtonTrustRegionPolicy.cpp:18-39.
#include "kb_device.h"

namespace kb {

typedef double v4d __attribute__((ext_vector_type(4)));

#define KB_WAVE_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
// an (empty) use of an accumulation register: the compiler then selects the AGPR-accumulator form of every MFMA in
// the kernel.  With VGPR accumulators, a wave issuing back-to-back f64 MFMAs slows the VALU instructions of the other
// waves on its SIMD ~5x (38 vs 7 cycles each); with AGPR accumulators ~2x (tools/micro/simd_share.hip)
#define KB_MFMA_AGPR() asm volatile("" ::"a"(0))
// materialise a loaded value at this point (an empty asm use): loads issued above cannot sink below it
#define KB_KEEP(x) asm volatile("" ::"v"(x))
#define KB_KEEPS(x) asm volatile("" ::"s"(x))

// per-camera kernel-argument arrays read at a run-time index by selects: a dynamically indexed kernel argument
// would make the compiler copy the whole KbDev into scratch (private memory), which costs every launch
__device__ __forceinline__ int cam_arg(const int (&a)[KB_MAX_CAMS], int i) {
  int v = a[0];
#pragma unroll
  for (int k = 1; k < KB_MAX_CAMS; ++k) v = (i == k) ? a[k] : v;
  return v;
}

// broadcast of a double from a wave-uniform lane (v_readlane_b32 x2, no LDS round trip)
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffull), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

constexpr int XS = 17;       // LDS row stride (doubles) of the 64 x 16 Jacobian-row tile
constexpr int kTargetLds = 1536;  // target corners staged in k_build's LDS when 3 * n_target <= this
// the camera block of the C > 64 solve in LDS (and in its global image): lower 16 x 16 tiles, tile (it, jt) at
// (it(it+1)/2 + jt) * kTileSz, row stride kTS (see ldl_panels)
constexpr int kTS = 17;             // tile row stride (doubles): 16 + 1 keeps row-parallel LDS accesses conflict-free
constexpr int kTileSz = 16 * kTS;
__device__ __forceinline__ int tile_base(int it, int jt) { return (it * (it + 1) / 2 + jt) * kTileSz; }
__device__ __forceinline__ int tidx(int i, int j) { return tile_base(i >> 4, j >> 4) + (i & 15) * kTS + (j & 15); }

// 1/x by v_rcp_f64 + two Newton steps (a short dependent chain; within an ulp of the IEEE quotient)
__device__ __forceinline__ double recip_d(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// 64-bit DPP move within rows of 16 lanes (VALU, no LDS round trip); CTRL = DPP control (0x121.. = row_ror:1..)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffull), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// lane k's value to every lane of its 16-lane row (DPP row_newbcast, gfx90a+): a plain VALU move, without the
// v_readlane -> SGPR -> VALU round trip.  k must fold to a constant (unrolled loops).
__device__ __forceinline__ double bcast16(double v, int k) {
  switch (k) {
    case 0: return dpp_d<0x150>(v);
    case 1: return dpp_d<0x151>(v);
    case 2: return dpp_d<0x152>(v);
    case 3: return dpp_d<0x153>(v);
    case 4: return dpp_d<0x154>(v);
    case 5: return dpp_d<0x155>(v);
    case 6: return dpp_d<0x156>(v);
    case 7: return dpp_d<0x157>(v);
    case 8: return dpp_d<0x158>(v);
    case 9: return dpp_d<0x159>(v);
    case 10: return dpp_d<0x15A>(v);
    case 11: return dpp_d<0x15B>(v);
    case 12: return dpp_d<0x15C>(v);
    case 13: return dpp_d<0x15D>(v);
    case 14: return dpp_d<0x15E>(v);
    default: return dpp_d<0x15F>(v);
  }
}

// wave-wide sum / max, fixed order, result uniform: row butterflies by rotation, then the 4 row values
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0x128>(v);
  v += dpp_d<0x124>(v);
  v += dpp_d<0x122>(v);
  v += dpp_d<0x121>(v);
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}
__device__ __forceinline__ double wave_max_d(double v) {
  v = fmax(v, dpp_d<0x128>(v));
  v = fmax(v, dpp_d<0x124>(v));
  v = fmax(v, dpp_d<0x122>(v));
  v = fmax(v, dpp_d<0x121>(v));
  return fmax(fmax(readlane_d(v, 0), readlane_d(v, 16)), fmax(readlane_d(v, 32), readlane_d(v, 48)));
}

__device__ __forceinline__ int tri_row(int q) {  // row of packed-lower index q
  int r = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
  while (r * (r + 1) / 2 > q) --r;
  while ((r + 1) * (r + 2) / 2 <= q) ++r;
  return r;
}

// ---------------------------------------------------------------------------------------------
// rigid-transform helpers
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
    for (int c = 0; c < 3; ++c)
      R[r * 3 + c] = R1[r * 3 + 0] * R2[0 * 3 + c] + R1[r * 3 + 1] * R2[1 * 3 + c] + R1[r * 3 + 2] * R2[2 * 3 + c];
    t[r] = R1[r * 3 + 0] * t2[0] + R1[r * 3 + 1] * t2[1] + R1[r * 3 + 2] * t2[2] + t1[r];
  }
}

// T_f^-1 of a pose DV
__device__ __forceinline__ void pose_inverse(const double* fp, double* Ri, double* ti) {
  double Rf[9];
  quat2r(fp, Rf);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) Ri[r * 3 + cc] = Rf[cc * 3 + r];
    ti[r] = -(Ri[r * 3 + 0] * fp[4] + Ri[r * 3 + 1] * fp[5] + Ri[r * 3 + 2] * fp[6]);
  }
}

// T_cam_w = B_{cam-1} .. B_0 T_f^-1 computed from a state vector (cost passes, where the chain is new)
__device__ __forceinline__ void cam_from_state(const KbDev& d, const double* s, int cam, const double* fp, double* R,
                                               double* t) {
  pose_inverse(fp, R, t);
  for (int j = 0; j < cam; ++j) {
    double RB[9], tB[3], R2[9], t2[3];
    pose_rt(s + d.off_base + 7 * j, RB, tB);
    rt_mul(RB, tB, R, t, R2, t2);
#pragma unroll
    for (int q = 0; q < 9; ++q) R[q] = R2[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) t[q] = t2[q];
  }
}

// G = -boxTimes(T_q) M(t_m) = [[R [t_m]x + [t_q]x R, -R], [-R, 0]]  (6x6, row-major), entry (a,b).
// boxTimes: sm_kinematics/src/transformations.cpp:132-141; M(t): TransformationBasic.cpp:49-66
// (rotation DV chain [-[t]x; I], translation DV chain [I; 0]); the inverse node contributes
// -boxTimes(T^-1) (TransformationExpressionNode.cpp:92-101).  With T_q = T_cam_w this is the chain of the
// frame DV; -G(Q, t_Bj) with Q = B_{i-1}..B_{j+1} is the chain of baseline B_j.
__device__ __forceinline__ double chain_entry(const double* R, const double* tq, const double* tm, int a, int b) {
  if (a < 3 && b < 3) {
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

// chain_entry from wave-uniform registers (R, t_q, t_m) for a lane-dependent entry (a, b): the same products, the
// lane's row / column of R picked by 0/1 weights (exact: one weight is 1, the others 0).  s = (R_a x t_m)_b and
// u = (t_q x R_{:,b})_a are chain_entry's two terms of the rotation block.  (Selects among R's entries here were
// folded by the compiler into a run-time index into R, which put R in per-lane scratch.)
__device__ __forceinline__ double chain_entry_reg(const double (&R)[9], const double (&tq)[3], const double* tm, int a,
                                                  int b) {
  const int ra = a < 3 ? a : a - 3, rb = b < 3 ? b : b - 3;
  const double ma0 = ra == 0 ? 1.0 : 0.0, ma1 = ra == 1 ? 1.0 : 0.0, ma2 = ra == 2 ? 1.0 : 0.0;
  const double mb0 = rb == 0 ? 1.0 : 0.0, mb1 = rb == 1 ? 1.0 : 0.0, mb2 = rb == 2 ? 1.0 : 0.0;
  const double r0 = ma0 * R[0] + ma1 * R[3] + ma2 * R[6];
  const double r1 = ma0 * R[1] + ma1 * R[4] + ma2 * R[7];
  const double r2 = ma0 * R[2] + ma1 * R[5] + ma2 * R[8];
  const double c0 = mb0 * R[0] + mb1 * R[1] + mb2 * R[2];
  const double c1 = mb0 * R[3] + mb1 * R[4] + mb2 * R[5];
  const double c2 = mb0 * R[6] + mb1 * R[7] + mb2 * R[8];
  const double rab = mb0 * r0 + mb1 * r1 + mb2 * r2;
  const double s0 = r1 * tm[2] - r2 * tm[1], s1 = -r0 * tm[2] + r2 * tm[0], s2 = r0 * tm[1] - r1 * tm[0];
  const double u0 = -tq[2] * c1 + tq[1] * c2, u1 = tq[2] * c0 - tq[0] * c2, u2 = -tq[1] * c0 + tq[0] * c1;
  const double sv = mb0 * s0 + mb1 * s1 + mb2 * s2, uv = ma0 * u0 + ma1 * u1 + ma2 * u2;
  return (a < 3 && b < 3) ? sv + uv : (a < 3 || b < 3) ? -rab : 0.0;
}

// ---------------------------------------------------------------------------------------------
// policy: while-condition (Optimizer2.cpp:215-219) + TrustRegionPolicy::solveSystem prelude
// (TrustRegionPolicy.cpp:39-52) + LM lambda schedule (LevenbergMarquardtTrustRegionPolicy.cpp:50-84)
// or GN (build every pass, no conditioner: GaussNewtonTrustRegionPolicy.cpp:25-29).
// ---------------------------------------------------------------------------------------------
template <bool GN_ONLY = false>
__device__ __forceinline__ void pol_pre(KbCtrl* c) {
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
  if (!GN_ONLY && c->policy == 0) {
    if (c->first) {
      c->do_build = 1;
    } else {
      const double d2 = c->lambda * c->dxdx + c->dxrhs;  // dx^T (lambda dx + rhs), getLmRho (:107-113)
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

// accept / revert (Optimizer2.cpp:221-259); red = [cost, dx.dx, dx.rhs, max|dx|] (all ranks)
__device__ __forceinline__ void pol_post(KbCtrl* c, const KbDev& d, const double* red, bool write_trace = true) {
  double J = 0.0, dX = c->deltaX;
  int accepted = 0;
  if (!c->solve_ok) {
    c->prev_failed = 1;
    c->lin_fail = 1;
    c->failed_iterations++;
    J = NAN;
  } else {
    J = red[0];
    dX = red[3];
    c->dxdx = red[1];
    c->dxrhs = red[2];
    c->deltaX = dX;
    c->J = J;
    c->deltaJ = c->p_J - J;
    if (c->policy == 0 && c->deltaJ < 0.0) {  // regression: revertLastStateUpdate (state[cur] untouched)
      c->failed_iterations++;
      c->prev_failed = 1;
    } else {
      c->cur = 1 - c->cur;
      c->p_J = J;
      c->prev_failed = 0;
      accepted = 1;
    }
    c->iterations++;
  }
  if (c->n_trace < d.trace_cap) {
    double* tr = d.trace + 4 * c->n_trace;
    if (write_trace) {
    tr[0] = J;
    tr[1] = c->lambda;
    tr[2] = dX;
    tr[3] = accepted;
    }
    c->n_trace++;
  }
  c->passes++;
}

constexpr int kPassPre = 2;  // per-frame rows per thread prefetched by k_build's first load round

// ---------------------------------------------------------------------------------------------
// the pending pass end on one GPU: fixed-order reduction of the per-frame rows [cost, max|dx|, dx.dx, dx.rhs]
// (+ camera statistics) -> red; pol_post (accept / revert) + pol_pre (next prelude) on a register copy of ctrl.
// Every thread of the block calls it; every block that calls it computes the same bits.  Returns the updated
// control block in *out (LDS); block `writer` stores it (and the trace entry) to HBM.
// ---------------------------------------------------------------------------------------------
__device__ void pass_end_block(const KbDev& d, const KbCtrl& cin, KbCtrl* out, bool writer, int nth,
                               bool apply_policy = true, const double4* pre = nullptr) {
  __shared__ double sh[8][4];
  const int tid = threadIdx.x;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (cin.solve_ok) {
    const double4* bp = reinterpret_cast<const double4*>(d.bsrc);
    const int nrows = d.bsrc_rows;
    int q0 = tid;
    if (pre) {  // the caller's first kPassPre rows of this thread, already loaded
#pragma unroll
      for (int u = 0; u < kPassPre; ++u)
        if (q0 + u * nth < nrows) {
          s0 += pre[u].x;
          s1 = fmax(s1, pre[u].y);
          s2 += pre[u].z;
          s3 += pre[u].w;
        }
      q0 += kPassPre * nth;
    }
    for (; q0 < nrows; q0 += 4 * nth) {
      double4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = bp[min(q0 + u * nth, nrows - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (q0 + u * nth < nrows) {
          s0 += v[u].x;
          s1 = fmax(s1, v[u].y);
          s2 += v[u].z;
          s3 += v[u].w;
        }
    }
    s0 = wave_sum_d(s0);
    s1 = wave_max_d(s1);
    s2 = wave_sum_d(s2);
    s3 = wave_sum_d(s3);
    if ((tid & 63) == 0 && tid < nth) {
      sh[tid >> 6][0] = s0;
      sh[tid >> 6][1] = s1;
      sh[tid >> 6][2] = s2;
      sh[tid >> 6][3] = s3;
    }
  }
  __syncthreads();
  if (tid == 0) {
    double red[4] = {0.0, 0.0, 0.0, 0.0};
    if (cin.solve_ok) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      for (int q = 0; q < (nth >> 6); ++q) {
        a0 += sh[q][0];
        a1 = fmax(a1, sh[q][1]);
        a2 += sh[q][2];
        a3 += sh[q][3];
      }
      red[0] = a0;
      red[1] = a2 + d.camstat[1];
      red[2] = a3 + d.camstat[2];
      red[3] = fmax(a1, d.camstat[0]);
      if (writer)
#pragma unroll
        for (int q = 0; q < 4; ++q) d.red_local[q] = red[q];
    }
    if (!apply_policy) goto done_tid0;
    {
    KbCtrl cl = cin;
    pol_post(&cl, d, red, writer);
    if (!cl.done) pol_pre(&cl);
    cl.pending = 0;
    cl.have_dx = 0;
    *out = cl;
    if (writer) *d.ctrl = cl;
    }
  done_tid0:;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// camera chains of a state: L_i (R|t) = B_{i-1}..B_0 and K_{i,j} (one block) -> slot `slot` of camL / camK.
// `base` points at the N-1 baseline poses (7-stride, HBM or LDS).
// ---------------------------------------------------------------------------------------------
// P(i, j) = B_{i-1} ... B_{j+1} for -1 <= j < i (P(i, i-1) = I): L_i = P(i, -1), K_{i,j} from P(i, j) and B_j.
// One thread per pair builds its product in the reference association order (Q <- B_k Q, k = j+1 .. i-1), so
// every chain equals the former per-entry recomputation bit for bit; the 36 entries of K_{i,j} then read it.
struct ChainLds {
  double sR[KB_MAX_CAMS][9], st[KB_MAX_CAMS][3];  // baseline B_j
  double PR[64][12];  // pair (i, j) at i(i+1)/2 + j + 1: R (9) | t (3); C <= 111 bounds the rig to N <= 10 (55 pairs)
};
// part 1: the baselines and the pair products (threads tx < np; WAVE: one wave alone, wave-level LDS syncs)
template <bool WAVE>
__device__ __forceinline__ void chain_pairs(const KbDev& d, const double* base, ChainLds& L, int tx) {
  const int N = d.N, np = N * (N + 1) / 2;
  if (tx < N - 1) pose_rt(base + 7 * tx, L.sR[tx], L.st[tx]);
  if (WAVE) KB_WAVE_SYNC();
  else __syncthreads();
  if (tx < np) {
    const int q = tx, i = tri_row(q), j = q - i * (i + 1) / 2 - 1;
    double QR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, Qt[3] = {0, 0, 0};
#pragma unroll 1
    for (int k = j + 1; k < i; ++k) {
      double R2[9], t2[3];
      rt_mul(L.sR[k], L.st[k], QR, Qt, R2, t2);
#pragma unroll
      for (int e = 0; e < 9; ++e) QR[e] = R2[e];
#pragma unroll
      for (int e = 0; e < 3; ++e) Qt[e] = t2[e];
    }
#pragma unroll
    for (int e = 0; e < 9; ++e) L.PR[q][e] = QR[e];
#pragma unroll
    for (int e = 0; e < 3; ++e) L.PR[q][9 + e] = Qt[e];
  }
}
// part 2 (after a barrier that follows part 1): L_i and K_{i,j} into slot `slot`
__device__ __forceinline__ void chain_write(const KbDev& d, const ChainLds& L, int slot, int tx, int nth) {
  const int N = d.N;
  double* Lo = cam_L(d, slot);
  double* Ko = cam_K(d, slot);
  for (int q = tx; q < N * 12; q += nth) {  // L_i = P(i, -1)
    const int i = q / 12, e = q % 12;
    Lo[q] = L.PR[i * (i + 1) / 2][e];
  }
  for (int idx = tx; idx < N * N * 36; idx += nth) {
    const int e = idx % 36, ij = idx / 36, i = ij / N, j = ij % N;
    double val = 0.0;
    if (j < i) {
      const double* P = L.PR[i * (i + 1) / 2 + j + 1];
      val = -chain_entry(P, P + 9, L.st[j], e / 6, e % 6);
    }
    Ko[idx] = val;
  }
}
__device__ __forceinline__ void chain_block(const KbDev& d, const double* base, int slot, int nth) {
  __shared__ ChainLds L;
  chain_pairs<false>(d, base, L, threadIdx.x);
  __syncthreads();
  chain_write(d, L, slot, threadIdx.x, nth);
}

// k_pre: camera chains of the current state (slot cur); gate 1 also runs the policy prelude of the first pass.
// Inside the optimizer loop k_solve computes the chains of each candidate state, so the accepted state's are
// always in slot cur.
__global__ void __launch_bounds__(256) k_pre(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && threadIdx.x == 0 && !c->done) pol_pre(c);
  const int cur = c->cur;
  chain_block(d, d.state + (size_t)cur * d.S + d.off_base, cur, blockDim.x);
}

// Schur sums of a block on MFMA: P = [H_fc | g_f] and Q = [A | b] (8 x CZ in LDS, rows 6..7 and columns > C
// zero, CZ = 16 nbz, nbz = ceil((C + 1) / 16)); wave w owns lower tiles q = w, w + nw, ... (at most TW) and
// accumulates acc[t] += P_ii^T Q_jj over the block's frames (two 16x16x4 steps per frame).  Tile entry (r, c)
// is sum_k P[k][r] Q[k][c]: r, c < C -> H_fc^T H_ff^-1 H_fc, r == C -> g_f^T H_ff^-1 H_fc = (H_fc^T b)^T.
template <int TW>
__device__ __forceinline__ void schur_tiles_accumulate(const double* P, const double* Q, int CZ, const int* tii,
                                                       const int* tjj, v4d* acc) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    if (tii[t] < 0) break;  // wave-uniform
    const double* ya = P + 16 * tii[t] + (lane & 15);
    const double* yb = Q + 16 * tjj[t] + (lane & 15);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = 4 * s + (lane >> 4);
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[k * CZ], yb[k * CZ], acc[t], 0, 0, 0);
    }
  }
}

// this wave's tiles (-1 terminated)
template <int TW>
__device__ __forceinline__ void schur_tiles_assign(int nbz, int* tii, int* tjj) {
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6, ntiles = nbz * (nbz + 1) / 2;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int q = wave + t * nw;
    const int ii = q < ntiles ? tri_row(q) : -1;
    tii[t] = ii;
    tjj[t] = q < ntiles ? q - ii * (ii + 1) / 2 : -1;
  }
}

// the tiles' entries into the block's partial row: sum Y^T Y upper packed (a <= b) | sum Y^T z.  kT: the tiles are
// held transposed (schur_tiles_accumulate6: lane l, reg r -> tile row l & 15, column (l >> 4) + 4 r), so that the 16
// lanes of a row group write 16 consecutive entries of a packed row (coalesced) instead of 16 rows
template <int TW, bool kT = false>
__device__ __forceinline__ void schur_tiles_store(double* prow_schur, int C, const int* tii, const int* tjj,
                                                  const v4d* acc) {
  const int lane = threadIdx.x & 63, Wt = C * (C + 1) / 2;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    if (tii[t] < 0) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ra = kT ? (lane & 15) : (lane >> 4) + 4 * r, ca = kT ? (lane >> 4) + 4 * r : (lane & 15);
      const int rg = 16 * tii[t] + ra, cg = 16 * tjj[t] + ca;
      if (rg < C && cg <= rg)
        prow_schur[upper_index(cg, rg, C)] = acc[t][r];
      else if (rg == C && cg < C)
        prow_schur[Wt + cg] = acc[t][r];
    }
  }
}

// expanded partials (GN fused, C > 64): the tiles' entries stored as EX - sum, EX = the block's camera-block expansion
// (same packing: S upper | b), so that the column sums are S - lambda^2 I and b themselves
template <int TW, bool kT = false>
__device__ __forceinline__ void schur_tiles_store_x(double* prow_schur, int C, const int* tii, const int* tjj,
                                                    const v4d* acc, const double* EX) {
  const int lane = threadIdx.x & 63, Wt = C * (C + 1) / 2;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    if (tii[t] < 0) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ra = kT ? (lane & 15) : (lane >> 4) + 4 * r, ca = kT ? (lane >> 4) + 4 * r : (lane & 15);
      const int rg = 16 * tii[t] + ra, cg = 16 * tjj[t] + ca;
      if (rg < C && cg <= rg) {
        const int u = upper_index(cg, rg, C);
        prow_schur[u] = EX[u] - acc[t][r];
      } else if (rg == C && cg < C) {
        prow_schur[Wt + cg] = EX[Wt + cg] - acc[t][r];
      }
    }
  }
}

// column of col-major packed lower index e (C columns) == row of row-major packed upper index e
__device__ __forceinline__ int cidx_col(int e, int C) {
  int j = (int)((2.0f * C + 1.0f - sqrtf((2.0f * C + 1.0f) * (2.0f * C + 1.0f) - 8.0f * (float)e)) * 0.5f);
  j = max(0, min(j, C - 1));
  while (j > 0 && j * (2 * C - j + 1) / 2 > e) --j;
  while ((j + 1) * (2 * C - j) / 2 <= e) ++j;
  return j;
}

// pair index of the chain K_{i,j} (j < i) in the pair-packed LDS arrays of k_buildp
__device__ __forceinline__ int pidx(int i, int j) { return i * (i - 1) / 2 + j; }

// entry (p, q) of H_cc (any order) or, q < 0, entry p of g_c, expanded from one block's per-camera sums:
//   H_{I_i,I_i} = Hs_i[II]; H_{I_i,B_j} = Hs_i[Id] K_{i,j} (j < i); H_{B_j,B_k} = sum_{i > max(j,k)} K_{i,j}^T T_{i,k};
//   g_{I_i} = Hs_i[I,15]; g_{B_j} = sum_{i > j} K_{i,j}^T Hs_i[d,15]
// Hs [N][16][16] (rows 0..5 pose, 6..14 intrinsics, 15 the -e column), Kp / Tp [pair][6][6] with T_{i,k} = Hs_i[dd] K_{i,k}
// (the same algebra as cam_entry_l / cam_grad_l over the finished sums; CalibrationTools.hpp:32-45 chain order)
__device__ __forceinline__ double cam_expand_entry(int N, const int* ci, const double* Hs, const double* Tp,
                                                   const double* Kp, int p, int q) {
  const int kp = ci[p] >> 16, ip = (ci[p] >> 8) & 0xff, xp = ci[p] & 0xff;
  double s = 0.0;
  if (q < 0) {
    if (kp == 0) return Hs[ip * 256 + (6 + xp) * 16 + 15];
    for (int i = ip + 1; i < N; ++i) {
      const double* K = Kp + pidx(i, ip) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Hs[i * 256 + a * 16 + 15];
    }
    return s;
  }
  const int kq = ci[q] >> 16, iq = (ci[q] >> 8) & 0xff, xq = ci[q] & 0xff;
  if (kp == 0 && kq == 0) {
    if (ip == iq) s = Hs[ip * 256 + (6 + xp) * 16 + 6 + xq];
  } else if (kp == 0 && kq == 1) {
    if (iq < ip) {
      const double* K = Kp + pidx(ip, iq) * 36;
#pragma unroll
      for (int b = 0; b < 6; ++b) s += Hs[ip * 256 + (6 + xp) * 16 + b] * K[b * 6 + xq];
    }
  } else if (kp == 1 && kq == 0) {
    if (ip < iq) {
      const double* K = Kp + pidx(iq, ip) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Hs[iq * 256 + a * 16 + 6 + xq];
    }
  } else {
    const int m = ip > iq ? ip : iq;
    for (int i = m + 1; i < N; ++i) {
      const double* K = Kp + pidx(i, ip) * 36;
      const double* T = Tp + pidx(i, iq) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * T[a * 6 + xq];
    }
  }
  return s;
}

// Gauss-Jordan elimination of [H_ff + lam2 I | H_fc | g_f] by one wave, lanes = columns (slot s: column
// lane + 64 s), rows 0..5 in registers; pivot column k broadcast with v_readlane.  No pivoting: H_ff is SPD,
// the pivots are the squared Cholesky diagonal (all > 0 iff positive definite).  Ends with [I | A | b]:
// A = (H_ff + lam2 I)^-1 H_fc, b = (H_ff + lam2 I)^-1 g_f (solveSystem's frame blocks of the Schur solve)
// into Q (row stride CZ) and HBM.  P holds rows 0..5 of [H_fc | g_f] (stride CZ).  Returns false if not PD.
__device__ __forceinline__ bool frame_gj(const KbDev& d, int f, const double* Hff, double lam2, const double* P,
                                         double* Q, int CZ, int lane, bool store = true) {
  const int C = d.C;
  double col[2][6];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int q = lane + 64 * sl, qh = min(q, 5), qp = min(max(q - 6, 0), C);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double dg = d.cond2 ? d.cond2[C + 6 * f + i] : lam2;  // setConditioner's squares, or lambda^2
      const double h = Hff[i * 6 + qh] + (i == qh ? dg : 0.0), pv = P[i * CZ + qp];
      col[sl][i] = q < 6 ? h : (q - 6 <= C ? pv : 0.0);
    }
  }
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double a[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) a[i] = readlane_d(col[0][i], k);  // column k (lane k, slot 0)
    ok = ok && (a[k] > 0.0);
    const double r = 1.0 / a[k];
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const double ck = col[sl][k] * r;
#pragma unroll
      for (int i = 0; i < 6; ++i)
        if (i != k) col[sl][i] -= a[i] * ck;
      col[sl][k] = ck;
    }
  }
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int c = lane + 64 * sl - 6;
    if (c >= 0 && c <= C) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        Q[i * CZ + c] = col[sl][i];
        if (!store) continue;
        if (c < C)
          d.Af[((size_t)f * 6 + i) * C + c] = col[sl][i];
        else
          d.bf[(size_t)f * 6 + i] = col[sl][i];
      }
    }
  }
  return ok;
}

// [A | b] = (H_ff + lam2 I)^-1 [H_fc | g_f] by LDL^T of the 6 x 6 block, factored redundantly in every lane's
// registers (no cross-lane broadcast: a short dependent chain, which matters when the wave shares its SIMD with
// MFMA-heavy waves), then each lane solves its columns lane and lane + 64 of [H_fc | g_f] (P, rows of 6).
// Writes Q (rows of 6, columns 0..C) and, if `store`, A_f / b_f to HBM.  Returns false if not positive definite.
__device__ __forceinline__ bool frame_ldl(const KbDev& d, int f, const double* Hff, double lam2, const double* P,
                                          double* Q, int CZ, int lane, bool store, bool stamp = false) {
  const int C = d.C;
  double L[6][6], Di[6];
  if (stamp) KB_TSB(d, 140);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) L[i][j] = Hff[i * 6 + j] + (i == j ? lam2 : 0.0);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double v[6];
#pragma unroll
    for (int j = 0; j < k; ++j) v[j] = L[k][j] * L[j][j];  // L_kj D_j (D_j kept on the diagonal)
    double dk = L[k][k];
#pragma unroll
    for (int j = 0; j < k; ++j) dk -= L[k][j] * v[j];
    ok = ok && (dk > 0.0);
    L[k][k] = dk;
    Di[k] = recip_d(dk);
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      double s = L[i][k];
#pragma unroll
      for (int j = 0; j < k; ++j) s -= L[i][j] * v[j];
      L[i][k] = s * Di[k];
    }
  }
  if (stamp) KB_TSB(d, 141);
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int c = lane + 64 * sl, cc = min(c, C);
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {  // L y = b
      double s = P[i * CZ + cc];
#pragma unroll
      for (int j = 0; j < i; ++j) s -= L[i][j] * x[j];
      x[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] *= Di[i];
#pragma unroll
    for (int i = 5; i >= 0; --i) {  // L^T x = D^-1 y
      double s = x[i];
#pragma unroll
      for (int j = i + 1; j < 6; ++j) s -= L[j][i] * x[j];
      x[i] = s;
    }
    if (c <= C) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        Q[i * CZ + c] = x[i];
        if (!store) continue;
        if (c < C)
          d.Af[((size_t)f * 6 + i) * C + c] = x[i];
        else
          d.bf[(size_t)f * 6 + i] = x[i];
      }
    }
    if (stamp) KB_TSB(d, 142 + sl);
  }
  return ok;
}

// frame_ldl for a column range: each of the k_buildp frame waves factors the 6 x 6 block redundantly and solves its
// own columns c0 <= c < c1 of [H_fc | g_f] into the shared Q (the frame waves meet before the Schur tiles read it)
__device__ __forceinline__ bool frame_ldl_cols(const KbDev& d, int f, const double* Hff, double lam2, const double* P,
                                               double* Q, int CZ, int lane, int c0, int c1, bool stamp = false) {
  const int C = d.C;
  double L[6][6], Di[6];
  if (stamp) KB_TSB(d, 140);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) L[i][j] = Hff[i * 6 + j] + (i == j ? lam2 : 0.0);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double v[6];
#pragma unroll
    for (int j = 0; j < k; ++j) v[j] = L[k][j] * L[j][j];
    double dk = L[k][k];
#pragma unroll
    for (int j = 0; j < k; ++j) dk -= L[k][j] * v[j];
    ok = ok && (dk > 0.0);
    L[k][k] = dk;
    Di[k] = recip_d(dk);
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      double s = L[i][k];
#pragma unroll
      for (int j = 0; j < k; ++j) s -= L[i][j] * v[j];
      L[i][k] = s * Di[k];
    }
  }
  if (stamp) KB_TSB(d, 141);
  for (int c = c0 + lane; c < c1; c += 64) {
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {  // L y = b
      double s = P[i * CZ + c];
#pragma unroll
      for (int j = 0; j < i; ++j) s -= L[i][j] * x[j];
      x[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] *= Di[i];
#pragma unroll
    for (int i = 5; i >= 0; --i) {  // L^T x = D^-1 y
      double s = x[i];
#pragma unroll
      for (int j = i + 1; j < 6; ++j) s -= L[j][i] * x[j];
      x[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      Q[i * CZ + c] = x[i];
      if (c < C)
        d.Af[((size_t)f * 6 + i) * C + c] = x[i];
      else
        d.bf[(size_t)f * 6 + i] = x[i];
    }
  }
  if (stamp) KB_TSB(d, 142);
  return ok;
}

// dx_f = b_f - A_f dx_c.  Lane slot sl holds column lane + 64 sl of A_f (zero beyond C); lanes 0..5 hold b_f.
__device__ __forceinline__ void fdx_load(const KbDev& d, int f, int lane, double (&ar)[6][2], double& bq) {
  const int C = d.C;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int q = lane + 64 * sl, qc = min(q, C - 1);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double v = d.Af[((size_t)f * 6 + r) * C + qc];
      ar[r][sl] = q < C ? v : 0.0;
    }
  }
  bq = d.bf[(size_t)f * 6 + min(lane, 5)];
}

// every lane ends with all six entries of dx_f
__device__ __forceinline__ void fdx_solve(const double (&ar)[6][2], const double* dxv, double bq, double* w) {
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double s = ar[r][0] * dxv[0] + ar[r][1] * dxv[1];
    s = wave_sum_d(s);
    w[r] = readlane_d(bq, r) - s;
  }
}

// pose of frame f moved by its step (in place), stored to the candidate buffer if `store`; wmax = max |dx_f|
__device__ __forceinline__ void frame_step(const KbDev& d, int f, bool store, int lane, const double (&ar)[6][2],
                                           const double* dxv, double bq, double* fp, double* snew, double& wmax) {
  double w[6], np[7];
#ifdef KB_STAMPS
  if (d.dbg_flags & 32) {  // diagnostic: no wave sums
#pragma unroll
    for (int r = 0; r < 6; ++r) w[r] = ar[r][0] * dxv[0] + bq;
  } else
#endif
  fdx_solve(ar, dxv, bq, w);
#ifdef KB_STAMPS
  if (d.dbg_flags & 4) {  // diagnostic: additive pose update
#pragma unroll
    for (int q = 0; q < 7; ++q) np[q] = fp[q] + w[q % 6];
  } else
#endif
  update_pose(fp, w, np);
#pragma unroll
  for (int q = 0; q < 7; ++q) fp[q] = np[q];
#pragma unroll
  for (int r = 0; r < 6; ++r) wmax = fmax(wmax, fabs(w[r]));
#ifdef KB_STAMPS
  if (d.dbg_flags & 8) return;  // diagnostic: no pose store
#endif
  if (store && lane < 7) {
    double pv = np[0];
#pragma unroll
    for (int q = 1; q < 7; ++q) pv = (lane == q) ? np[q] : pv;
    snew[d.off_frame + 7 * f + lane] = pv;
  }
}

// ---------------------------------------------------------------------------------------------
// k_build: one block = a group of frames; waves = N * nsplit, wave w -> camera w % N, corner split w / N.
// ---------------------------------------------------------------------------------------------
// GNF: Gauss-Newton fused variant (applies the previous solve's frame steps; no folded pass end)
// MM: camera-model set of the rig (kMmAll = any model; a single-model set compiles one projection)
template <int TW, bool GNF, unsigned MM>
__global__ void __launch_bounds__(512) k_build(KbDev d, int gate, int fuse) {
  pass_stamp(d);
  KbCtrl* c = d.ctrl;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int N = d.N, C = d.C, WPB = d.wpb, NS = d.nsplit;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nth = blockDim.x, tid = threadIdx.x;
  double* Xw = sm + wave * 64 * XS;
  double* Hw = sm + WPB * 64 * XS;   // [WPB][256] per-wave partial local Hessians
  double* Hv = Hw + WPB * 256;       // [N][256] per-view local Hessian of the current frame
  double* camsum = Hv + N * 256;     // [N][256] per-camera sums over the block's frames
  double* Wv = camsum + N * 256;     // [N][64]: R(9) t(3) tf(3) | G(36) at +16
  double* Pv = Wv + N * 64;          // [N][36]  G^T H_dd
  double* dH = Pv + N * 36;          // [N][36]  G^T H_dd G
  double* dg = dH + N * 36;          // [N][8]   G^T g_d
  double* Fh = dg + N * 8;           // frame H_ff [36]
  const int nbz = (C + 16) >> 4, CZ = 16 * nbz;
  double* P = Fh + 36;               // [8][CZ]: [H_fc | g_f] of the current frame, zero-padded
  double* Q = P + 8 * CZ;            // [8][CZ]: [A | b] (frame_gj), zero-padded
  double* Kl = Q + 8 * CZ;           // [N(N-1)/2][36] K_{i,j}, j < i, at (i(i-1)/2 + j)
  double* tg = Kl + 18 * N * (N - 1);  // [n_target][3] target corners (when staged)
  __shared__ double wmx[8];            // GN fused: per-wave max |dx_f|
  __shared__ int okl;
  __shared__ double cst[KB_MAX_CAMS][24];  // per camera: chain L (12) | intrinsics (10)
  __shared__ int ctab[2][KB_MAX_CAMS];      // per camera: first intrinsic column | baseline column
  const int W = d.W, Wt = W - C;
  const int f0 = blockIdx.x * d.gframes, f1 = min(d.F, f0 + d.gframes);
  const int cam = __builtin_amdgcn_readfirstlane(wave % N), sp = __builtin_amdgcn_readfirstlane(wave / N);
  // ---- round 1: launch-independent loads, unconditional (clamped) and pinned before the gate
  __shared__ KbCtrl cnew;
  const KbCtrl cin = *c;
  int done = cin.done, dob = cin.do_build, cur = cin.cur;
  double lam = gate ? cin.lambda : d.host_lambda;
  const bool tg_lds = d.K * 3 <= kTargetLds;
  const int nt3 = 3 * d.K;
  constexpr int kTgU = 2;  // 2 x 256 threads >= 3 x 120 AprilGrid corners
  double tv[kTgU];
#pragma unroll
  for (int u = 0; u < kTgU; ++u) tv[u] = d.target[min(tid + u * nth, nt3 - 1)];
  int2 fv = d.fview[(size_t)f0 * N + cam];
  const bool fold = !GNF && gate && d.fold;
  double4 pre[kPassPre];  // previous pass's per-frame rows (fold): loaded with this round
#pragma unroll
  for (int u = 0; u < kPassPre; ++u)
    pre[u] = fold ? reinterpret_cast<const double4*>(d.bsrc)[min(tid + u * nth, d.bsrc_rows - 1)]
                  : make_double4(0.0, 0.0, 0.0, 0.0);
#pragma unroll
  for (int u = 0; u < kTgU; ++u) KB_KEEP(tv[u]);
  KB_KEEPS(fv.x);
  KB_KEEPS(fv.y);
  // GN fused passes: the previous solve's frame steps are applied here (back-substitution of frame f0)
  const bool gfu = GNF && gate;
  double yr[6][2], dxv[2] = {0.0, 0.0}, bq = 0.0;
  if (gfu) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int q = lane + 64 * sl;
      const double v = d.dx[min(q, C - 1)];
      dxv[sl] = q < C ? v : 0.0;
    }
#ifdef KB_STAMPS
    if (d.dbg_flags & 2) {  // diagnostic: no A_f / b_f loads
#pragma unroll
      for (int r = 0; r < 6; ++r) yr[r][0] = yr[r][1] = 1e-3 * r;
      bq = 1e-3 * lane;
    } else
#endif
    fdx_load(d, f0, lane, yr, bq);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      KB_KEEP(dxv[sl]);
#pragma unroll
      for (int r = 0; r < 6; ++r) KB_KEEP(yr[r][sl]);
    }
    KB_KEEP(bq);
  }
  if (fold && cin.pending && !cin.done) {  // previous pass's end (accept / revert, next prelude)
    pass_end_block(d, cin, &cnew, blockIdx.x == 0, nth, true, pre);
    done = cnew.done;
    dob = cnew.do_build;
    cur = cnew.cur;
    lam = cnew.lambda;
  }
  if (gate && (done || !dob)) return;
  // GN fused with a pending step: build at the candidate state (buffer / chain slot 1 - cur: cameras updated by
  // the previous k_solve, frames updated below from the accepted poses of buffer cur)
  const bool upd = gfu && cin.have_dx;
  const int bs = upd ? 1 - cur : cur;
  // ---- round 2: loads indexed by round 1 (state buffer, chains of slot bs, corners of the view)
  const double* s = d.state + (size_t)bs * d.S;
  const double* sf = d.state + (size_t)cur * d.S;  // frame poses (the step is applied on top when upd)
  double* snew = d.state + (size_t)(1 - cur) * d.S;
  if (tid < N * 22) {
    const int cm = tid / 22, e = tid % 22;
    cst[cm][e] = e < 12 ? cam_L(d, bs)[cm * 12 + e] : s[cm * KB_MAX_INTR + e - 12];
  }
  if (tid < 2 * N) ctab[tid / N][tid % N] = (tid < N) ? cam_arg(d.col_intr, tid) : cam_arg(d.col_base, tid - N);
  double* fpl = tg + (tg_lds ? nt3 : 0);  // [gframes][8] the block's frame poses (after their steps)
  double fp0[7];  // pose of the block's first frame
#pragma unroll
  for (int q = 0; q < 7; ++q) fp0[q] = sf[d.off_frame + 7 * f0 + q];
  int cidn;
  double2 yn;
  {
    const int k = min(fv.x + sp * 64 + lane, max(fv.y - 1, 0));
    cidn = d.cid[k];
    yn = d.y[k];
  }
  const double* Kc = cam_K(d, bs);
  for (int q = tid; q < 18 * N * (N - 1); q += nth) {
    const int e = q % 36, ij = q / 36;
    int i = 1;
    while (i * (i + 1) / 2 <= ij) ++i;
    const int j = ij - i * (i - 1) / 2;
    Kl[q] = Kc[(size_t)(i * N + j) * 36 + e];
  }
  KB_KEEPS(cidn);  // issued before the frame step's arithmetic (their latency overlaps it)
  double wmax = 0.0;  // GN fused: max |dx_f| over this wave's frames
  if (upd) frame_step(d, f0, wave == 0, lane, yr, dxv, bq, fp0, snew, wmax);  // frame f0 (its loads in round 1)
  if (wave == 0 && lane < 7) {
    double pv = fp0[0];
#pragma unroll
    for (int q = 1; q < 7; ++q) pv = (lane == q) ? fp0[q] : pv;
    fpl[lane] = pv;
  }
  // further frames of a multi-frame block: one wave each
  for (int j = 1 + wave; j < f1 - f0; j += WPB) {
    double fp[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) fp[q] = sf[d.off_frame + 7 * (f0 + j) + q];
    if (upd) {
      double af[6][2], bfq;
      fdx_load(d, f0 + j, lane, af, bfq);
      frame_step(d, f0 + j, true, lane, af, dxv, bfq, fp, snew, wmax);
    }
    if (lane < 7) {
      double pv = fp[0];
#pragma unroll
      for (int q = 1; q < 7; ++q) pv = (lane == q) ? fp[q] : pv;
      fpl[8 * j + lane] = pv;
    }
  }
  if (lane == 0) wmx[wave] = wmax;
  KB_STAMP(d, 14);
  if (tg_lds) {
#pragma unroll
    for (int u = 0; u < kTgU; ++u)
      if (tid + u * nth < nt3) tg[tid + u * nth] = tv[u];
    for (int q = tid + kTgU * nth; q < nt3; q += nth) tg[q] = d.target[q];
  }
  const double* tgt = tg_lds ? tg : d.target;
  const double lam2 = lam * lam;
  v4d acc[TW];
  int tii[TW], tjj[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
  schur_tiles_assign<TW>(fuse ? nbz : 0, tii, tjj);
  for (int q = tid; q < 8 * CZ; q += nth)  // P, Q padding (rows 6, 7 and columns > C stay zero)
    if (q >= 6 * CZ || (q % CZ) > C) P[q] = Q[q] = 0.0;
  if (tid == 0) okl = 1;
  KB_STAMP(d, 16);
  for (int q = tid; q < N * 256; q += nth) camsum[q] = 0.0;
  __syncthreads();

  const int mrow = lane >> 4, mcol = lane & 15;
  const int model = cam_arg(d.model, cam), nin = cam_arg(d.nintr, cam);
  const double* Lc = cst[cam];
  const double* intr = cst[cam] + 12;
  for (int f = f0; f < f1; ++f) {
    double fp[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) fp[q] = fpl[8 * (f - f0) + q];
    double Ri[9], ti[3], R[9], t[3];
    pose_inverse(fp, Ri, ti);
    rt_mul(Lc, Lc + 9, Ri, ti, R, t);  // T_cam_w = L_cam T_f^-1 (chain of the accepted state)
    KB_STAMP(d, 26);
    if (f > f0) {  // next frame of a multi-frame block
      fv = d.fview[(size_t)f * N + cam];
      const int k = min(fv.x + sp * 64 + lane, max(fv.y - 1, 0));
      cidn = d.cid[k];
      yn = d.y[k];
    }
    v4d acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    {
      const int o0 = fv.x, o1 = fv.y;
      for (int base = o0 + sp * 64; base < o1; base += NS * 64) {
        const int k = base + lane;
        const int cid = cidn;
        const double2 yv = yn;
        if (base + NS * 64 < o1) {  // software-pipelined: next chunk's corner ids and keypoints
          const int kn = min(k + NS * 64, o1 - 1);
          cidn = d.cid[kn];
          yn = d.y[kn];
        }
        double xr[2][16];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int q = 0; q < 16; ++q) xr[r][q] = 0.0;
        if (k < o1) {
          const double X0 = tgt[3 * cid], X1 = tgt[3 * cid + 1], X2 = tgt[3 * cid + 2];
          const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
          const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
          const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
          double u, w, Jp[6], Ji[2 * KB_MAX_INTR];
          project_jac<MM>(model, intr, p0, p1, p2, u, w, Jp, Ji);
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
            xr[r][15] = -(r == 0 ? e0 : e1);  // column 15 carries -e: H[:,15] = rhs part, H[15][15] = chi^2
          }
        }
        KB_STAMP(d, 27);
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
          for (int ks = 0; ks < 16; ks += 2) {
            const double xa = Xw[(4 * ks + mrow) * XS + mcol];
            const double xb = Xw[(4 * ks + 4 + mrow) * XS + mcol];
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, xa, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(xb, xb, acc1, 0, 0, 0);
          }
          KB_WAVE_SYNC();
        }
      }
    }
    // f64 MFMA C/D layout: lane l, reg r -> row (l>>4) + 4r, col l&15
#pragma unroll
    for (int r = 0; r < 4; ++r) Hw[wave * 256 + (mrow + 4 * r) * 16 + mcol] = acc0[r] + acc1[r];
    if (sp == 0 && lane == 0) {
      double* wv = Wv + cam * 64;
#pragma unroll
      for (int q = 0; q < 9; ++q) wv[q] = R[q];
      wv[9] = t[0]; wv[10] = t[1]; wv[11] = t[2];
      wv[12] = fp[4]; wv[13] = fp[5]; wv[14] = fp[6];
    }
    KB_STAMP(d, 17);
    __syncthreads();
    KB_STAMP(d, 18);
    for (int q = threadIdx.x; q < N * 256; q += nth) {
      const int qc = q >> 8, e = q & 255;
      double hv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double h = Hw[((k < NS ? k : 0) * N + qc) * 256 + e];
        hv[k] = (k < NS) ? h : 0.0;
      }
      const double cs = camsum[q];
      const double sacc = ((hv[0] + hv[1]) + hv[2]) + hv[3];
      Hv[q] = sacc;
      camsum[q] = cs + sacc;
    }
    __syncthreads();
    KB_STAMP(d, 19);
    if (wave < N) {  // expansion of view (f, cam = wave) through the 6-D chains
      const int vc = __builtin_amdgcn_readfirstlane(wave);
      const bool has = fv.y > fv.x;  // this wave's camera == vc
      const int nv = cam_arg(d.nintr, vc);
      const double* H = Hv + vc * 256;
      double* wv = Wv + vc * 64;
      double* G = wv + 16;
      if (lane < 36) G[lane] = chain_entry(wv, wv + 9, wv + 12, lane / 6, lane % 6);
      KB_WAVE_SYNC();
      KB_STAMP(d, 28);
      if (lane < 36) {
        const int a = lane / 6, b = lane % 6;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += G[k * 6 + a] * H[k * 16 + b];
        Pv[vc * 36 + lane] = has ? sacc : 0.0;  // P_v = G^T H_dd
      } else if (lane < 42) {
        const int a = lane - 36;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += G[k * 6 + a] * H[k * 16 + 15];
        dg[vc * 8 + a] = has ? sacc : 0.0;  // G^T g_d
      }
      KB_WAVE_SYNC();
      if (lane < 36) {
        const int a = lane / 6, b = lane % 6;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += Pv[vc * 36 + a * 6 + k] * G[k * 6 + b];
        dH[vc * 36 + lane] = sacc;  // P_v G_v
      }
      KB_STAMP(d, 29);
      if (lane < 6 * nv) {
        const int a = lane / nv, q = lane % nv;
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) sacc += G[k * 6 + a] * H[k * 16 + 6 + q];
        sacc = has ? sacc : 0.0;  // G^T H_dI
        P[a * CZ + ctab[0][vc] + q] = sacc;
        if (!gfu) d.Hfc[((size_t)f * 6 + a) * C + ctab[0][vc] + q] = sacc;
      }
    }
    __syncthreads();
    // frame outputs: sums over the frame's views in camera order
    for (int q = threadIdx.x; q < 42 + 36 * (N - 1); q += nth) {
      if (q < 36) {
        double sacc = 0.0;
        for (int i = 0; i < N; ++i) sacc += dH[i * 36 + q];
        Fh[q] = sacc;
        if (!gfu) d.Hff[(size_t)f * 36 + q] = sacc;
      } else if (q < 42) {
        double sacc = 0.0;
        for (int i = 0; i < N; ++i) sacc += dg[i * 8 + q - 36];
        P[(q - 36) * CZ + C] = sacc;
        d.gf[(size_t)f * 6 + q - 36] = sacc;
      } else {  // H_f,B_j = sum_{i > j} P_i K_{i,j}
        const int e = q - 42, j = e / 36, ab2 = e % 36, a = ab2 / 6, b = ab2 % 6;
        double sacc = 0.0;
        for (int i = j + 1; i < N; ++i) {
          const double* K = Kl + (i * (i - 1) / 2 + j) * 36;
#pragma unroll
          for (int k = 0; k < 6; ++k) sacc += Pv[i * 36 + a * 6 + k] * K[k * 6 + b];
        }
        P[a * CZ + ctab[1][j] + b] = sacc;
        if (!gfu) d.Hfc[((size_t)f * 6 + a) * C + ctab[1][j] + b] = sacc;
      }
    }
    KB_STAMP(d, 20);
    if (fuse) {
      __syncthreads();
      KB_STAMP(d, 21);
      if (wave == 0) {
        const bool ok = frame_gj(d, f, Fh, lam2, P, Q, CZ, lane);
        if (!ok && lane == 0) okl = 0;
      }
      __syncthreads();
      KB_STAMP(d, 23);
      schur_tiles_accumulate<TW>(P, Q, CZ, tii, tjj, acc);
    }
    __syncthreads();
    KB_STAMP(d, 24);
  }
  double* prow = d.part + (size_t)blockIdx.x * d.Wr;
  for (int q = threadIdx.x; q < N * 136; q += nth) {
    const int qc = q / 136;
    int a, b;
    d16_rowcol_fast(q % 136, a, b);
    prow[q] = camsum[qc * 256 + a * 16 + b];
  }
  if (fuse) {
    schur_tiles_store<TW>(prow + N * 136, C, tii, tjj, acc);
    if (threadIdx.x == 0) prow[N * 136 + W] = okl ? 0.0 : 1.0;  // non-PD frame blocks (summed)
  }
  if (GNF && threadIdx.x == 0) {  // the block's max |dx_f| (reduced with max by k_colsum)
    double m = 0.0;
    for (int q = 0; q < WPB; ++q) m = fmax(m, wmx[q]);
    prow[d.Wp] = m;
  }
  KB_STAMP(d, 25);
}

// ---------------------------------------------------------------------------------------------
// k_buildp: k_build for rigs with one wave per camera (nsplit == 1, 4 <= N <= kBuildpMaxCams), pipelined over
// the block's frames.  Waves 0..N-1 (view waves) own camera w: per frame the view's corners (projection, one
// Jacobian row per lane, 32-row LDS tiles, v_mfma_f64_16x16x4 SYRK), the camera's running local sums (registers)
// and the view's 6-D chain expansion (G, P_v = G^T H_dd, G^T g_d, P_v G, G^T H_dI: the camera's intrinsic
// columns of [H_fc | g_f], and P_v K_{v,j}: its share of the baseline columns), all wave-local; the next frame's
// first loads are issued before the expansion.  NF frame waves run one frame behind on the view outputs
// (double-buffered by frame parity): the frame sums H_ff, g_f and sum_{i>j} P_i K_{i,j}, the Gauss-Jordan
// elimination into [A_f | b_f] (every frame wave, identical bits; frame wave 0 stores) and the Schur tiles
// [H_fc | g_f]^T [A_f | b_f], split over the frame waves.  One block barrier per frame: the SYRK of frame f (MFMA)
// overlaps the elimination and Schur sums of frame f - 1 on the same CU.  The sums follow k_build's order except
// the baseline columns (per-camera products summed over cameras).
// ---------------------------------------------------------------------------------------------
constexpr int kBuildpMaxCams = 8;

// frame waves of k_buildp: the Schur tiles per frame wave TT picks them (<= 5 tiles: 2 waves, else 4: one frame wave
// per SIMD beside its two view waves)
template <int TT>
constexpr int buildp_nf() { return TT > 5 ? 4 : 2; }

// intrinsics count of a one-model set (0 for a mix): a constant count lets the compiler drop the unused columns
template <unsigned MM>
constexpr int mm_nintr() {
  if (MM == 0u || (MM & (MM - 1u))) return 0;
  int m = 0;
  while (!((MM >> m) & 1u)) ++m;
  return (m == KB_PINHOLE_RADTAN || m == KB_PINHOLE_EQUI) ? 8 : m == KB_OMNI_RADTAN ? 9
         : (m == KB_EUCM || m == KB_DS)                   ? 6 : 5;
}

// lower tiles of [P | .]^T [Q | .] owned by frame wave fw of NF (q = fw, fw + NF, ...), -1 terminated
template <int TT>
__device__ __forceinline__ void schur_tiles_assign_fw(int nbz, int fw, int* tii, int* tjj) {
  const int ntiles = nbz * (nbz + 1) / 2;
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int q = fw + buildp_nf<TT>() * t;
    const int ii = (fw >= 0 && q < ntiles) ? tri_row(q) : -1;
    tii[t] = __builtin_amdgcn_readfirstlane(ii);  // wave-uniform: scalar registers, not 2 x TT VGPRs
    tjj[t] = __builtin_amdgcn_readfirstlane(ii >= 0 ? q - ii * (ii + 1) / 2 : -1);
  }
}

// schur_tiles_accumulate over 6-row P, Q (the MFMA k rows 6, 7 are zero operands, not LDS rows)
template <int TT>
__device__ __forceinline__ void schur_tiles_accumulate6(const double* P, const double* Q, int CZ, const int* tii,
                                                        const int* tjj, v4d* acc, int lane) {
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    if (tii[t] < 0) break;  // wave-uniform
    const double* ya = P + 16 * tii[t] + (lane & 15);
    const double* yb = Q + 16 * tjj[t] + (lane & 15);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = 4 * s + (lane >> 4);
      const int kc = min(k, 5);
      const double a = ya[kc * CZ], b = yb[kc * CZ];
      // the tile transposed (B = the P rows, A = the Q columns): the stores write packed rows coalesced (kT)
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(k < 6 ? b : 0.0, k < 6 ? a : 0.0, acc[t], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);  // one tile's operands at a time (hoisting all of them spills)
  }
}

// MW: the most waves a block may have.  12 (8 cameras + 4 frame waves) caps the kernel at 168 VGPRs, so that two
// 6-wave blocks share a CU; rigs with N + frame waves <= 8 whose view role compiles two projection models
// (configs[2]) take MW = 8 (256 VGPRs, no spills, one block per CU) -- kb_capi.hip `buildp_wide`.
template <int TT, bool GNF, unsigned MM, int MW>
__global__ void __launch_bounds__(64 * MW) k_buildp(KbDev d, int gate, int fuse) {
  KB_MFMA_AGPR();
  pass_stamp(d);
  KbCtrl* c = d.ctrl;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int NF = buildp_nf<TT>();
  const int N = d.N, C = d.C, NW = N + NF, NP = N * (N - 1) / 2;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, nth = blockDim.x;
  const int tid = threadIdx.x;
  const int nbz = (C + 16) >> 4, CZ = 16 * nbz;
  const int VBS = 44 * N + 6 * CZ, FBS = 6 * CZ;
  double* Xw = sm + wave * 64 * XS;     // [N][64][XS] view waves' Jacobian-row tiles (P_v after the SYRK)
  double* PvL = sm + N * 64 * XS;       // [2][N][128] each view's P_v[:, d] (MFMA A-operand layout), by frame parity
  double* Wv = PvL + N * 256;           // [N][36]: each view's chain G
  double* VB = Wv + N * 36;             // [VBS] view outputs: dH [N][36] | dg [N][8] |
                                        //   intrinsic columns [6][CZ]
  double* FI = VB + VBS;                // [40] frame sums: H_ff ([H_fc | g_f] is summed into the view buffer's
                                        //   intrinsic-column rows, whose other columns the views leave free)
  double* FB = FI + 40;                 // [FBS] the frame's [A_f | b_f] (each frame wave solves a column range)
  double* Kl = FB + FBS;           // [NP][36] K_{i,j}, j < i, at (i(i-1)/2 + j)
  double* tg = Kl + 36 * NP;            // [n_target][3] target corners (when staged) | frame poses [gframes][8]
  __shared__ double wmx[kBuildpMaxCams + 4];
  __shared__ int okl;
  __shared__ double cst[KB_MAX_CAMS][24];  // per camera: chain L (12) | intrinsics (10)
  __shared__ int ctab[2][KB_MAX_CAMS];      // per camera: first intrinsic column | baseline column
  __shared__ int cil[112];                  // expanded partials: column info (kind << 16 | camera << 8 | index)
  __shared__ int xcnt;                      // expanded partials: view waves done with their camera's share
  __shared__ int fcnt;                      // frame waves done with their share of a frame's sums (monotonic)
  const int W = d.W;
  const int f0 = blockIdx.x * d.gframes, f1 = min(d.F, f0 + d.gframes), G = f1 - f0;
  const bool vw = wave < N;  // view wave (camera = wave) | frame wave fw = wave - N
  const int cam = __builtin_amdgcn_readfirstlane(vw ? wave : 0), fw = __builtin_amdgcn_readfirstlane(wave - N);
  if (wave == 0) KB_TSB(d, 0);
  // ---- round 1: launch-independent loads, unconditional (clamped) and pinned before the gate
  const KbCtrl cin = *c;
  const int done = cin.done, dob = cin.do_build, cur = cin.cur;
  const double lam = gate ? cin.lambda : d.host_lambda;
  const bool tg_lds = d.bp_tg;  // the host decides (its LDS budget holds a second view-output buffer)
  const int nt3 = 3 * d.K;
  constexpr int kTgU = 2;
  double tv[kTgU];
#pragma unroll
  for (int u = 0; u < kTgU; ++u) tv[u] = d.target[min(tid + u * nth, nt3 - 1)];
  int2 fv = d.fview[(size_t)f0 * N + cam];
#pragma unroll
  for (int u = 0; u < kTgU; ++u) KB_KEEP(tv[u]);
  KB_KEEPS(fv.x);
  KB_KEEPS(fv.y);
  // GN fused: the previous solve's frame steps are applied here, and H_ff / H_fc are not stored (only the per-call
  // path reads them back: kb_build, k_schur, k_pcg; the fused pass consumes A_f, b_f and the Schur sums)
  const bool gfu = GNF && gate;
  double yr[6][2], dxv[2] = {0.0, 0.0}, bq = 0.0;
  if (gfu) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int q = lane + 64 * sl;
      const double v = d.dx[min(q, C - 1)];
      dxv[sl] = q < C ? v : 0.0;
    }
    fdx_load(d, f0 + min(wave, G - 1), lane, yr, bq);  // wave j steps frame f0 + j (its rows in this round)
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      KB_KEEP(dxv[sl]);
#pragma unroll
      for (int r = 0; r < 6; ++r) KB_KEEP(yr[r][sl]);
    }
    KB_KEEP(bq);
  }
  // the state-slot-indexed loads (camera chains and intrinsics of the build state, K_{i,j}, the block's first frame
  // poses) from both ping-pong slots in this round too, picked once the control block is in: one dependent round trip
  // less before the first corner pass
  const int nK = 18 * N * (N - 1);
  double csv[2] = {0.0, 0.0}, kv[2][2] = {{0.0, 0.0}, {0.0, 0.0}}, fps[2][7];
  {
    const int cm = min(tid / 22, N - 1), e = tid % 22;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
      csv[sl] = e < 12 ? cam_L(d, sl)[cm * 12 + e] : d.state[(size_t)sl * d.S + cm * KB_MAX_INTR + e - 12];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = min(tid + u * nth, nK - 1), ee = q % 36, ij = q / 36;
      int i = 1;
      while (i * (i + 1) / 2 <= ij) ++i;
      const int j = ij - i * (i - 1) / 2;
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) kv[sl][u] = nK > 0 ? cam_K(d, sl)[(size_t)(i * N + j) * 36 + ee] : 0.0;
    }
    const int fj = f0 + min(wave, G - 1);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
#pragma unroll
      for (int q = 0; q < 7; ++q) fps[sl][q] = d.state[(size_t)sl * d.S + d.off_frame + 7 * fj + q];
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      KB_KEEP(csv[sl]);
#pragma unroll
      for (int u = 0; u < 2; ++u) KB_KEEP(kv[sl][u]);
#pragma unroll
      for (int q = 0; q < 7; ++q) KB_KEEP(fps[sl][q]);
    }
  }
  if (gate && (done || !dob)) return;
  const bool upd = gfu && cin.have_dx;
  const int bs = upd ? 1 - cur : cur;
  // ---- round 2: loads indexed by round 1
  const double* sf = d.state + (size_t)cur * d.S;
  double* snew = d.state + (size_t)(1 - cur) * d.S;
  if (tid < N * 22) cst[tid / 22][tid % 22] = bs ? csv[1] : csv[0];
  if (tid < 2 * N) ctab[tid / N][tid % N] = (tid < N) ? cam_arg(d.col_intr, tid) : cam_arg(d.col_base, tid - N);
  // expanded partials (GN fused, C > 64, KbDev::xexp): the block expands its own per-camera sums in the epilogue
  const bool xp = GNF && gfu && fuse && d.xexp;
  if (xp && tid < C) cil[tid] = d.colinfo[tid];
  double* fpl = tg + (tg_lds ? nt3 : 0);
  // the view outputs are double-buffered: frame f's in VB (f - f0 even) or VB1 (odd), so that the frame waves sum
  // frame f - 1 while the view waves run frame f
  double* VB1 = fpl + 8 * d.gframes;
  int cidn;  // view waves: lane = corner of a 64-corner pass
  double2 yn;
  {
    const int k = min(fv.x + lane, max(fv.y - 1, 0));
    cidn = d.cid[k];
    yn = d.y[k];
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (tid + u * nth < nK) Kl[tid + u * nth] = bs ? kv[1][u] : kv[0][u];
  if (nK > 2 * nth) {  // rigs whose chain table outgrows two entries per thread
    const double* Kc = cam_K(d, bs);
    for (int q = tid + 2 * nth; q < nK; q += nth) {
      const int e = q % 36, ij = q / 36;
      int i = 1;
      while (i * (i + 1) / 2 <= ij) ++i;
      const int j = ij - i * (i - 1) / 2;
      Kl[q] = Kc[(size_t)(i * N + j) * 36 + e];
    }
  }
  KB_KEEPS(cidn);
  // the previous solve's frame steps: wave j moves frame f0 + j (then f0 + j + NW, ...) and stages its pose
  double wmax = 0.0;
  for (int j = wave; j < G; j += NW) {
    double fp[7];
    if (j == wave) {
#pragma unroll
      for (int q = 0; q < 7; ++q) fp[q] = cur ? fps[1][q] : fps[0][q];
    } else {
#pragma unroll
      for (int q = 0; q < 7; ++q) fp[q] = sf[d.off_frame + 7 * (f0 + j) + q];
    }
    if (upd) {
      if (j == wave) {
        frame_step(d, f0 + j, true, lane, yr, dxv, bq, fp, snew, wmax);
      } else {
        double af[6][2], bfq;
        fdx_load(d, f0 + j, lane, af, bfq);
        frame_step(d, f0 + j, true, lane, af, dxv, bfq, fp, snew, wmax);
      }
    }
    if (lane < 7) {
      double pv = fp[0];
#pragma unroll
      for (int q = 1; q < 7; ++q) pv = (lane == q) ? fp[q] : pv;
      fpl[8 * j + lane] = pv;
    }
  }
  if (lane == 0) wmx[wave] = wmax;
  if (tg_lds) {
#pragma unroll
    for (int u = 0; u < kTgU; ++u)
      if (tid + u * nth < nt3) tg[tid + u * nth] = tv[u];
    for (int q = tid + kTgU * nth; q < nt3; q += nth) tg[q] = d.target[q];
  }
  const double* tgt = tg_lds ? tg : d.target;  // (KB_CORNER_OLD; the corner passes branch on tg_lds)
  (void)tgt;
  const double lam2 = lam * lam;
  if (tid == 0) {
    okl = 1;
    xcnt = 0;
    fcnt = 0;
  }
  __syncthreads();
  if (wave == 0) KB_TSB(d, 1);

  const int mrow = lane >> 4, mcol = lane & 15;
  double* prow = d.part + (size_t)blockIdx.x * d.Wr;
  double* Fh = FI;      // frame inputs of the frame being eliminated: H_ff (40); [H_fc | g_f] [6][CZ] in its view buffer
  // iteration it: the view waves run the views of frame it -> VB[it & 1]; the frame waves sum frame it - 1 over its
  // views (VB[(it - 1) & 1] -> FI, split over the frame waves, an LDS counter between them) and eliminate it; one
  // block barrier per frame.  The roles run separate loops with the same barrier count (G, then one after the last
  // frame), so neither holds the other's registers; the frame sums are off the view waves' chain.
  if (vw) {
    const int model = cam_arg(d.model, cam), nin = mm_nintr<MM>() ? mm_nintr<MM>() : cam_arg(d.nintr, cam);
    const double* Lc = cst[cam];
    const double* intr = cst[cam] + 12;
    v4d creg = {0.0, 0.0, 0.0, 0.0};  // the camera's local sums over the block's frames
    for (int it = 0; it < G; ++it) {
      {
        // ---------------- phase B: view (f, cam)
        const int f = f0 + it;
        int lane = threadIdx.x & 63;  // opaque per frame (see the frame waves)
        asm volatile("" : "+v"(lane));
        const int mrow = lane >> 4, mcol = lane & 15;
        if (wave == 0 && it < 8) KB_TSB(d, 2 + 2 * it);
        double* vb = (it & 1) ? VB1 : VB;
        const int2 fvn = d.fview[(size_t)min(f + 1, f1 - 1) * N + cam];  // the next frame's view (first loads below)
        double fp[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) fp[q] = fpl[8 * it + q];
        double Ri[9], ti[3], R[9], t[3];
        pose_inverse(fp, Ri, ti);
        rt_mul(Lc, Lc + 9, Ri, ti, R, t);  // T_cam_w = L_cam T_f^-1
        // the view's chain G (6 x 6) for the expansion, formed while the first pass's MFMAs run: every lane holds
        // T_cam_w and the frame translation in registers, so lane e < 36 picks entry e by selects (no LDS staging;
        // wave 0's first v-row segment 2.2 -> 1.2 us, the frame period unchanged: the second view wave of each SIMD
        // sets it)
        double* Gm = Wv + cam * 36;
        auto make_g = [&]() {
          if (lane < 36) Gm[lane] = chain_entry_reg(R, t, fp + 4, lane / 6, lane % 6);
        };
#ifdef KB_SYRK16
        v4d acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#else
        // the SYRK on v_mfma_f64_4x4x4f64 (4 blocks of 4 x 4): only the 10 upper 4 x 4 blocks of the symmetric 16 x 16
        // [J | e]^T [J | e] are formed (2.5 instructions of ~17 cycles per 4 rows, against one 64-cycle 16x16x4 that
        // also forms the 6 lower blocks).  accD: the diagonal blocks (b, b); accO1: (b, b+1 mod 4); accO2: (0,2), (1,3)
        // of two row quads.  Operand lane 16k + 4b + c supplies row k, column 4I_b + c (A) / 4J_b + c (B); block b's
        // entry (i, j) lands at lane 16i + 4b + j (tools/micro/mfma_f64_4x4_layout.hip).
        double accD = 0.0, accO1 = 0.0, accO2 = 0.0;
#endif
        const int o0 = fv.x, o1 = fv.y;
        const bool stv = (wave == 0 || wave == N - 1) && it == 2;  // diagnostic stamps: one steady-state frame
        const int sto = wave == 0 ? 130 : 160;
        int pass = 0;
        for (int base = o0; base < o1; base += 64, ++pass) {  // 64 corners per pass: the u rows, then the v rows
          const int k = base + lane;
          if (stv && pass < 2) KB_TSB(d, sto + 4 * pass);
          const int cid = cidn;
          const double2 yv = yn;
          if (base + 64 < o1) {  // software-pipelined: next pass's corner ids and keypoints
            const int kn = min(k + 64, o1 - 1);
            cidn = d.cid[kn];
            yn = d.y[kn];
          }
#ifdef KB_CORNER_OLD
          double xu[16], xv[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            xu[q] = 0.0;
            xv[q] = 0.0;
          }
          if (k < o1) {  // one projection per corner: both Jacobian rows from the lane
            const double X0 = tgt[3 * cid], X1 = tgt[3 * cid + 1], X2 = tgt[3 * cid + 2];
            const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
            const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
            const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
            double u, w, Jp[6], Ji[2 * KB_MAX_INTR];
            project_jac<MM>(model, intr, p0, p1, p2, u, w, Jp, Ji);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
              double* xr = r ? xv : xu;
              const double j0 = Jp[3 * r], j1 = Jp[3 * r + 1], j2 = Jp[3 * r + 2];
              // J_delta = -Jp [I | [p]x]   (HomogeneousExpressionNode.cpp:71-81, boxMinus)
              xr[0] = -j0;
              xr[1] = -j1;
              xr[2] = -j2;
              xr[3] = -(j1 * p2 - j2 * p1);
              xr[4] = -(-j0 * p2 + j2 * p0);
              xr[5] = -(j0 * p1 - j1 * p0);
              // intrinsics: -Jp, -Jd (CameraDesignVariable.hpp(impl):38-54)
#pragma unroll
              for (int q = 0; q < 9; ++q) xr[6 + q] = (q < nin) ? -Ji[KB_MAX_INTR * r + q] : 0.0;
              xr[15] = -(r ? yv.y - w : yv.x - u);  // column 15 carries -e: H[:,15] = rhs part, H[15][15] = chi^2
            }
          }
          const bool valid = true;
#else
          // one projection per corner: both Jacobian rows from the lane.  The rows are written un-negated,
          // [dy/dtheta | e] = -[de/dtheta | -e]: the SYRK of a row and of its negation are bitwise equal, so the sign
          // flips of J_delta = -Jp [I | [p]x] and of the intrinsic rows -Jp, -Jd (CameraDesignVariable.hpp(impl):38-54)
          // are not spent.  Lanes past the view's last corner leave xu / xv undefined and store zero rows instead (no
          // 32-register zero initialisation per pass).
          // (KB_CORNER_CLAMP: every lane projects a real corner -- lanes past the view's end hold the clamped last
          // corner -- without the exec-mask branch and the zero initialisation, those lanes storing zero rows: more
          // VGPRs spilled to AGPRs, k_buildp 93.1 -> 96.9 us; not the default)
          const bool valid = k < o1;
          double xu[16], xv[16];
#if !defined(KB_CORNER_NOZERO) && !defined(KB_CORNER_CLAMP)
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            xu[q] = 0.0;
            xv[q] = 0.0;
          }
#endif
#ifdef KB_CORNER_CLAMP
          {
#else
          if (valid) {
#endif
            double X0, X1, X2;
#ifdef KB_CORNER_TGB
            if (tg_lds) {  // the staged corners through ds_read (a select of the two pointers compiles to flat loads)
              X0 = tg[3 * cid];
              X1 = tg[3 * cid + 1];
              X2 = tg[3 * cid + 2];
            } else {
              X0 = d.target[3 * cid];
              X1 = d.target[3 * cid + 1];
              X2 = d.target[3 * cid + 2];
            }
#else
            X0 = tgt[3 * cid];
            X1 = tgt[3 * cid + 1];
            X2 = tgt[3 * cid + 2];
#endif
            const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
            const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
            const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
            double u, w, Jp[6], Ji[2 * KB_MAX_INTR];
#ifdef KB_DIAG_NOPROJ  // diagnostic timing variant only (wrong results): the projection and its Jacobian skipped
            u = p0;
            w = p1;
#pragma unroll
            for (int q = 0; q < 6; ++q) Jp[q] = p2 * q;
#pragma unroll
            for (int q = 0; q < 2 * KB_MAX_INTR; ++q) Ji[q] = p0 + q;
#else
            project_jac<MM>(model, intr, p0, p1, p2, u, w, Jp, Ji);
#endif
#pragma unroll
            for (int r = 0; r < 2; ++r) {
              double* xr = r ? xv : xu;
              const double j0 = Jp[3 * r], j1 = Jp[3 * r + 1], j2 = Jp[3 * r + 2];
              // Jp [I | [p]x]   (HomogeneousExpressionNode.cpp:71-81, boxMinus)
              xr[0] = j0;
              xr[1] = j1;
              xr[2] = j2;
              xr[3] = j1 * p2 - j2 * p1;
              xr[4] = -j0 * p2 + j2 * p0;
              xr[5] = j0 * p1 - j1 * p0;
#pragma unroll
              for (int q = 0; q < 9; ++q) xr[6 + q] = (q < nin) ? Ji[KB_MAX_INTR * r + q] : 0.0;
              xr[15] = r ? yv.y - w : yv.x - u;  // column 15 carries e: H[:,15] = rhs part, H[15][15] = chi^2
            }
          }
#endif
          if (stv && pass < 2) KB_TSB(d, sto + 4 * pass + 1);
          // rows n .. 63 of a partial pass are zero: only the groups of 4 k-steps (16 rows) holding valid rows are
          // issued (k-step ks = rows 4ks .. 4ks + 3, even ks into acc0, odd into acc1), the next group's operands in
          // flight during the current group's MFMAs (one LDS round trip per group, not per MFMA).  Row = lane: the
          // lanes of a write hit distinct LDS bank pairs at the 17-double row stride.
#ifdef KB_SYRK16
          const int ng = (min(64, o1 - base) + 15) >> 4;
#else
          const int np = (min(64, o1 - base) + 7) >> 3;  // pairs of row quads holding valid rows (the rest are zero)
#endif
#pragma unroll
          for (int r = 0; r < 2; ++r) {
#if defined(KB_CORNER_NOZERO) || defined(KB_CORNER_CLAMP)
            if (valid) {
#pragma unroll
              for (int q = 0; q < 16; ++q) Xw[lane * XS + q] = r ? xv[q] : xu[q];
            } else {
#pragma unroll
              for (int q = 0; q < 16; ++q) Xw[lane * XS + q] = 0.0;
            }
#else
            (void)valid;
#pragma unroll
            for (int q = 0; q < 16; ++q) Xw[lane * XS + q] = r ? xv[q] : xu[q];
#endif
            KB_WAVE_SYNC();
#ifndef KB_SYRK16
            {
              // per pair of row quads (rows 8p .. 8p + 7): the diagonal-block operand of each quad (row mrow, column
              // mcol: the 16x16x4 operand), the (b, b+1) operand of each (column (mcol + 4) & 15), and the A / B
              // operands of the paired (0,2), (1,3) instruction (lanes b < 2: quad 0, columns mcol | mcol + 8; b >= 2:
              // quad 1, columns mcol - 8 | mcol); the next pair's six loads issued before this pair's five MFMAs
              const int bq = (lane >> 2) & 3;
              const int oD = mrow * XS + mcol, oE = mrow * XS + ((mcol + 4) & 15);
              const int oA = bq < 2 ? oD : (4 + mrow) * XS + mcol - 8, oB = bq < 2 ? oD + 8 : (4 + mrow) * XS + mcol;
              double xr[3][6];  // the operands of two pairs (the next pair's loads in flight during this pair's MFMAs)
              auto ld = [&](double* x, int pp) {
                const double* xp = Xw + 8 * pp * XS;
                x[0] = xp[oD];
                x[1] = xp[oE];
                x[2] = xp[4 * XS + oD];
                x[3] = xp[4 * XS + oE];
                x[4] = xp[oA];
                x[5] = xp[oB];
                __builtin_amdgcn_sched_barrier(0);
              };
              auto mf = [&](const double* x) {
                accD = __builtin_amdgcn_mfma_f64_4x4x4f64(x[0], x[0], accD, 0, 0, 0);
                accO1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x[0], x[1], accO1, 0, 0, 0);
                accD = __builtin_amdgcn_mfma_f64_4x4x4f64(x[2], x[2], accD, 0, 0, 0);
                accO1 = __builtin_amdgcn_mfma_f64_4x4x4f64(x[2], x[3], accO1, 0, 0, 0);
                accO2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x[4], x[5], accO2, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
              };
#ifndef KB_SYRK44_RING3  // (a ring of three pairs spills more to AGPRs and measured 0.4 % slower)
#ifdef KB_DIAG_NOSYRK  // diagnostic timing variant only (wrong results): the SYRK MFMAs and their loads skipped
              (void)ld;
              (void)mf;
              (void)np;
#else
              ld(xr[0], 0);
#pragma unroll
              for (int pp = 0; pp < 8; ++pp) {
                if (pp >= np) break;  // wave-uniform
                if (pp + 1 < np) ld(xr[(pp + 1) & 1], pp + 1);
                mf(xr[pp & 1]);
              }
#endif
#else
              ld(xr[0], 0);
              if (np > 1) ld(xr[1], 1);
#pragma unroll
              for (int pp = 0; pp < 8; ++pp) {
                if (pp >= np) break;  // wave-uniform
                if (pp + 2 < np) ld(xr[(pp + 2) % 3], pp + 2);
                mf(xr[pp % 3]);
              }
#endif
            }
#else
            // groups g = 0..3 ping-pong between xa and xb: group g + 1's loads are issued before group g's MFMAs
            double xa[4], xb[4];
            auto ld = [&](double* x, int g) {
#pragma unroll
              for (int u = 0; u < 4; ++u) x[u] = Xw[(16 * g + 4 * u + mrow) * XS + mcol];
              __builtin_amdgcn_sched_barrier(0);
            };
            auto mf = [&](const double* x) {
              acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], x[0], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], x[1], acc1, 0, 0, 0);
              acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], x[2], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], x[3], acc1, 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            };
            ld(xa, 0);
            if (ng > 1) ld(xb, 1);
            mf(xa);
            if (ng > 1) {
              if (ng > 2) ld(xa, 2);
              mf(xb);
              if (ng > 2) {
                if (ng > 3) ld(xb, 3);
                mf(xa);
                if (ng > 3) mf(xb);
              }
            }
#endif
            if (stv && pass < 2) KB_TSB(d, sto + 4 * pass + 2 + r);
            if (r == 0 && pass == 0) make_g();
            KB_WAVE_SYNC();
          }
        }
        if (o1 <= o0) make_g();  // a view without corners (no pass ran)
        {  // the next frame's first corner ids and keypoints, in flight during the expansion and the barrier
          fv = fvn;
          const int k = min(fvn.x + lane, max(fvn.y - 1, 0));
          cidn = d.cid[k];
          yn = d.y[k];
        }
        if (wave == 0 && it < 8) KB_TSB(d, 3 + 2 * it);
        if (it == 3 && wave < 8) KB_TSB(d, 144 + wave);
        // f64 MFMA C/D layout: lane l, reg r -> row (l>>4) + 4r, col l&15
        v4d hv;
#ifdef KB_SYRK16
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          hv[q] = acc0[q] + acc1[q];
          creg[q] = creg[q] + hv[q];
        }
#else
        {
          // the upper blocks to the 16 x 16 C layout (hv[q] = H[mrow + 4q][mcol]) through the view's tile (free after
          // the SYRK): each block and its mirror written, the two quads' (0,2), (1,3) parts added first (lane + 8)
          const int bq = (lane >> 2) & 3, ii = lane >> 4, jj = lane & 3;
          const double o2 = accO2 + dpp_d<0x128>(accO2);
          const int rb = 4 * bq + ii, c1 = 4 * ((bq + 1) & 3) + jj;
          Xw[rb * XS + 4 * bq + jj] = accD;
          Xw[rb * XS + c1] = accO1;
          Xw[c1 * XS + rb] = accO1;
          if (bq < 2) {
            const int c2 = 4 * (bq + 2) + jj;
            Xw[rb * XS + c2] = o2;
            Xw[c2 * XS + rb] = o2;
          }
          KB_WAVE_SYNC();
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            hv[q] = Xw[(mrow + 4 * q) * XS + mcol];
            creg[q] = creg[q] + hv[q];
          }
        }
#endif
        // expansion of view (f, cam) through the 6-D chain G on MFMA steps whose operands stay in registers:
        //   D = H[:, d] G  (A = the lane's own H registers: H is symmetric, so C-layout row r of a lane is A's k-step r;
        //   B = G from LDS), i.e. D[i][a] = P_v[a][i] with P_v = G^T H[d, :]: G^T H_dd, G^T H_dI, G^T g_d;
        //   then D's C layout is the A operand P_v[:, d] of dH = P_v G and of this camera's share P_v K_{v,j} of the
        //   baseline columns.  No LDS transposition; the chain's loads were issued before the SYRK.
        double* dHv = vb + cam * 36;
        double* dgv = vb + N * 36 + cam * 8;
        double* Pi = vb + N * 44;
        const int i16 = lane & 15, k0 = lane >> 4;
        double gb[2];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int k = k0 + 4 * st;
          const double g = Gm[min(k, 5) * 6 + min(i16, 5)];
          gb[st] = (k < 6 && i16 < 6) ? g : 0.0;
        }
        v4d dv = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 2; ++st) dv = __builtin_amdgcn_mfma_f64_16x16x4f64(hv[st], gb[st], dv, 0, 0, 0);
        double pa[2];  // A = P_v[:, d]: lane supplies P_v[i16][k0 + 4 st] = D[k0 + 4 st][i16]
#pragma unroll
        for (int st = 0; st < 2; ++st) pa[st] = (k0 + 4 * st < 6) ? dv[st] : 0.0;
        v4d t2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 2; ++st) t2 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[st], gb[st], t2, 0, 0, 0);
        // this camera's share P_v K_{v,j} of the baseline columns is formed by the frame waves (their per-frame chain
        // has the slack): the A operand goes to LDS in its register layout, buffer it & 1
        if (cam > 0) {
#pragma unroll
          for (int st = 0; st < 2; ++st) PvL[(it & 1) * N * 128 + cam * 128 + st * 64 + lane] = pa[st];
        }
        // D entry (i, a) at lane (i & 3) * 16 + a, reg i >> 2: G^T H_dI (the camera's intrinsic columns), G^T g_d
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const int i = k0 + 4 * r;
          if (i16 < 6) {
            if (i >= 6 && i < 6 + nin) {
              Pi[i16 * CZ + ctab[0][cam] + i - 6] = dv[r];
              if (!gfu) d.Hfc[((size_t)f * 6 + i16) * C + ctab[0][cam] + i - 6] = dv[r];
            } else if (i == 15) {
              dgv[i16] = dv[r];
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {  // dH = P_v G: entry (a, b) at lane, reg: a = k0 + 4 r, b = i16
          const int arow = k0 + 4 * r;
          if (arow < 6 && i16 < 6) dHv[arow * 6 + i16] = t2[r];
        }
        if (stv) KB_TSB(d, sto + 8);
        if (it == 3 && wave < 8) KB_TSB(d, 152 + wave);
      }
      __syncthreads();
    }
    if (xp) {
      // ---- expanded partials, while the frame waves eliminate the block's last frame (the view waves
      // are idle in that phase, and the Xw tiles the image overlaps are no longer read).  The block's share of the
      // camera block, H_cc and g_c upper packed, expanded from the view waves' local sums creg = Hs (C layout: lane l,
      // reg q -> row (l >> 4) + 4 q, column l & 15) through the chains K of the build state (Kl):
      //   step 1 (each view wave, its camera i): H_{I_i,I_i} and g_{I_i} directly; D = Hs[:, d] [K_{i,0} | .. |
      //     K_{i,i-1}] on MFMA (the symmetric Hs is its own A operand): rows 6 .. 5 + nin -> H_{I_i,B_j}, row 15 -> the
      //     camera's share of g_B, rows 0 .. 5 -> T_i = Hs_dd K_i; the structural zeros of its rows;
      //   step 2 (after the view waves meet): H_{B_j,B_k} = sum_{i > max(j,k)} K_{i,j}^T T_{i,k}, one 16 x 16 tile per
      //     view wave accumulated over the cameras in order on MFMA; g_B; the cost.
      // The column sums k_colsumx forms are then S - lambda^2 I = H_cc - sum H_fc^T A_f and b = g_c - sum H_fc^T b_f.
      double* EX = sm;            // [W] H_cc upper packed | g_c
      double* Tl = EX + W;        // [N][6][48] T_i
      double* gB = Tl + N * 288;  // [N][48] camera i's share of g_B
      double* cc = gB + N * 48;   // [N] chi^2 of camera i
      const int Wt = W - C, NB = 6 * (N - 1), CI = C - NB, ci0 = ctab[0][cam];
      const int i16 = lane & 15, k0 = lane >> 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int a = mrow + 4 * q, b = mcol, x = a - 6, y = b - 6;
        if (x >= 0 && x < nin && y >= x && y < nin) EX[upper_index(ci0 + x, ci0 + y, C)] = creg[q];
        if (b == 15 && x >= 0 && x < nin) EX[Wt + ci0 + x] = creg[q];
        if (a == 15 && b == 15) cc[cam] = creg[q];
      }
      if (cam > 0) {
        const int nct = (6 * cam + 15) >> 4;
        const double* Kv = Kl + (cam * (cam - 1) / 2) * 36;
        double kb[3][2];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int k = k0 + 4 * st;
#pragma unroll
          for (int ct = 0; ct < 3; ++ct) {
            const int c = 16 * ct + i16, cc2 = min(c, 6 * cam - 1), jj = cc2 / 6, bb = cc2 - 6 * jj;
            const double v = Kv[jj * 36 + min(k, 5) * 6 + bb];
            kb[ct][st] = (k < 6 && c < 6 * cam) ? v : 0.0;
          }
        }
#pragma unroll
        for (int ct = 0; ct < 3; ++ct) {
          if (ct >= nct) break;  // wave-uniform
          v4d t = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int st = 0; st < 2; ++st) t = __builtin_amdgcn_mfma_f64_16x16x4f64(creg[st], kb[ct][st], t, 0, 0, 0);
          const int n = 16 * ct + i16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = k0 + 4 * r;
            if (n < 6 * cam) {
              if (m < 6) Tl[cam * 288 + m * 48 + n] = t[r];
              else if (m - 6 < nin) EX[upper_index(ci0 + m - 6, CI + n, C)] = t[r];
              else if (m == 15) gB[cam * 48 + n] = t[r];
            }
          }
        }
      }
      {  // the structural zeros of the camera's rows: H_{I_cam, I_k} (k > cam) and H_{I_cam, B_j} (j >= cam)
        const int nz1 = CI - (ci0 + nin), nzr = nz1 + NB - 6 * cam;
        for (int e = lane; e < nin * nzr; e += 64) {
          const int x = e / nzr, k = e - x * nzr;
          const int q = k < nz1 ? ci0 + nin + k : CI + 6 * cam + (k - nz1);
          EX[upper_index(ci0 + x, q, C)] = 0.0;
        }
      }
      // the view waves meet (an LDS counter: the frame waves are not at a block barrier now) before the baseline
      // tiles read every camera's T_i
      KB_WAVE_SYNC();
      if (lane == 0) atomicAdd(&xcnt, 1);
      while (__hip_atomic_load(&xcnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < N) __builtin_amdgcn_s_sleep(1);
      const int ntb = (NB + 15) >> 4;
      for (int tq = wave; tq < ntb * (ntb + 1) / 2; tq += N) {  // tile (ta, tb), ta <= tb, upper tiles in row order
        int ta = 0, q = tq;
        while (q >= ntb - ta) {
          q -= ntb - ta;
          ++ta;
        }
        const int tb = ta + q;
        v4d acc = {0.0, 0.0, 0.0, 0.0};
        for (int i = 1; i < N; ++i) {
          const double* Kv = Kl + (i * (i - 1) / 2) * 36;
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int k = k0 + 4 * st, ca = 16 * ta + i16, cb = 16 * tb + i16;
            const int cac = min(ca, 6 * i - 1), ja = cac / 6, ya = cac - 6 * ja;
            const double av = Kv[ja * 36 + min(k, 5) * 6 + ya];
            const double bv = Tl[i * 288 + min(k, 5) * 48 + min(cb, 47)];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64((k < 6 && ca < 6 * i) ? av : 0.0,
                                                       (k < 6 && cb < 6 * i) ? bv : 0.0, acc, 0, 0, 0);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * ta + k0 + 4 * r, col = 16 * tb + i16;
          if (row <= col && col < NB) EX[upper_index(CI + row, CI + col, C)] = acc[r];
        }
      }
      for (int n = tid; n < NB; n += 64 * N) {
        double g = 0.0;
        for (int i = n / 6 + 1; i < N; ++i) g += gB[i * 48 + n];
        EX[Wt + CI + n] = g;
      }
      if (tid == 0) {
        double sc = 0.0;
        for (int i = 0; i < N; ++i) sc += cc[i];
        prow[C] = sc;  // the block's chi^2 (the cost column)
      }
    }
    __syncthreads();  // the frame waves' last barrier (after the last frame's sums and elimination)
    if (!xp) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // the camera's local sums, upper packed
        const int a = mrow + 4 * q, b = mcol;
        if (a <= b) prow[cam * 136 + d16_index(a, b)] = creg[q];
      }
    }
  } else {
    // the frame waves are the youngest waves of their SIMDs, so age-ordered issue serves them last; their frame sums
    // and elimination are on the per-frame critical path (priority 1: configs[3] 7,187 -> 7,232 GN it/s, the 250-frame
    // shard 14,568 -> 14,750; priority 3 measured the same)
#ifndef KB_FW_PRIO
#define KB_FW_PRIO 1
#endif
    __builtin_amdgcn_s_setprio(KB_FW_PRIO);
    v4d acc[TT];
    int tii[TT], tjj[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    schur_tiles_assign_fw<TT>(fuse ? nbz : 0, fw, tii, tjj);
    double* Q = FB;  // [A_f | b_f] [6][CZ]
    const int qcw = (C + NF) / NF, qc0 = fw * qcw, qc1 = min(C + 1, qc0 + qcw);  // this wave's columns
    int mt = 0;  // frame-wave meetings so far (x NF arrivals)
    // the baseline columns (36 (N - 1): the N - 1 - j products of column block j first, so the costliest lanes are
    // spread over waves 0..1), then H_ff (its upper triangle, mirrored: 21 sums) and g_f on the cheapest wave: one
    // lane per output (243 at N = 7) over the 4 frame waves; the intrinsic columns are in place
    const int nbl = 36 * (N - 1), nsum = nbl + 27;
    for (int it = 0; it <= G; ++it) {
      if (it > 0) {
        // ---------------- phase A: sums of frame f = f0 + it - 1 over its views (camera order), the frame waves' share
        const int f = f0 + it - 1;
        if (fw == 0 && it <= 8) KB_TSB(d, 51 + it);
        double* VBp = ((it - 1) & 1) ? VB1 : VB;
        const double* dHv = VBp;
        const double* dgv = VBp + N * 36;
        double* P = VBp + N * 44;  // [H_fc | g_f]: the views wrote the intrinsic columns in place
        // the views' P_v (their MFMA A operands, entry (a, k) at register k >> 2, lane 16 (k & 3) + a)
        const double* pab = PvL + ((it - 1) & 1) * N * 128;
#ifdef KB_DIAG_NOFW  // diagnostic timing variant only (wrong results): the frame waves' sums skipped
        for (int q = nsum; q < nsum; q += 64 * NF) {
#else
        for (int q = fw * 64 + lane; q < nsum; q += 64 * NF) {
#endif
          double sacc = 0.0;
          if (q < nbl) {
            // H_f,B_j = sum_{i > j} P_i K_{i,j}: each camera's product (6 FMAs on the VALU: the MFMA pipes are busy with
            // the views' SYRK) added in camera order, two cameras' operands loaded at once (the second clamped to a
            // valid chain and dropped past the last camera)
            const int j = q / 36, ab2 = q - 36 * j, a = ab2 / 6, b = ab2 - 6 * a;
            for (int i = j + 1; i < N; i += 2) {
              const int i1 = min(i + 1, N - 1);
              const double* pv0 = pab + i * 128 + a;
              const double* pv1 = pab + i1 * 128 + a;
              const double* kp0 = Kl + (i * (i - 1) / 2 + j) * 36 + b;
              const double* kp1 = Kl + (i1 * (i1 - 1) / 2 + j) * 36 + b;
              double x0[6], x1[6], k0[6], k1[6];
#pragma unroll
              for (int k = 0; k < 6; ++k) {
                x0[k] = pv0[(k >> 2) * 64 + 16 * (k & 3)];
                k0[k] = kp0[k * 6];
                x1[k] = pv1[(k >> 2) * 64 + 16 * (k & 3)];
                k1[k] = kp1[k * 6];
              }
              double pr0 = 0.0, pr1 = 0.0;
#pragma unroll
              for (int k = 0; k < 6; ++k) {
                pr0 = fma(x0[k], k0[k], pr0);
                pr1 = fma(x1[k], k1[k], pr1);
              }
              sacc += pr0;
              if (i + 1 < N) sacc += pr1;
            }
            P[a * CZ + ctab[1][j] + b] = sacc;
            if (!gfu) d.Hfc[((size_t)f * 6 + a) * C + ctab[1][j] + b] = sacc;
          } else {
            const int e = q - nbl;
            int hr = 0, hc = e;  // H_ff entry (hr, hc), hr <= hc (e < 21), else g_f entry e - 21
            if (e < 21)
              while (hc >= 6 - hr) hc -= 6 - hr++;
            hc += hr;
            const double* src = e < 21 ? dHv + hr * 6 + hc : dgv + e - 21;
            const int stride = e < 21 ? 36 : 8;
            double v[kBuildpMaxCams];
#pragma unroll
            for (int i = 0; i < kBuildpMaxCams; ++i) v[i] = src[min(i, N - 1) * stride];
#pragma unroll
            for (int i = 0; i < kBuildpMaxCams; ++i)
              if (i < N) sacc += v[i];
            if (e < 21) {
              Fh[hr * 6 + hc] = sacc;
              Fh[hc * 6 + hr] = sacc;
              if (!gfu) {
                d.Hff[(size_t)f * 36 + hr * 6 + hc] = sacc;
                d.Hff[(size_t)f * 36 + hc * 6 + hr] = sacc;
              }
            } else {
              P[(e - 21) * CZ + C] = sacc;
              d.gf[(size_t)f * 6 + e - 21] = sacc;
            }
          }
        }
        // the frame waves meet (an LDS counter: the view waves are in their next frame) before the elimination reads
        // every sum
        KB_WAVE_SYNC();
        if (it == 3) KB_TSB(d, 184 + fw);
        mt += NF;
        if (lane == 0) atomicAdd(&fcnt, 1);
        while (__hip_atomic_load(&fcnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < mt) __builtin_amdgcn_s_sleep(1);
      }
      if (it > 0 && fuse) {
        // ---------------- frame f = it - 1 (one behind the views): elimination + Schur tiles
        const int f = f0 + it - 1;
        // an opaque lane id per frame: the lane-dependent addresses and selects of the elimination are recomputed
        // here instead of being hoisted out of the loop (which spills at this kernel's register budget)
        int lane = threadIdx.x & 63;
        asm volatile("" : "+v"(lane));
        if (fw == 0 && it <= 8) KB_TSB(d, 20 + 4 * (it - 1));
        double* P = (((it - 1) & 1) ? VB1 : VB) + N * 44;
#ifdef KB_DIAG_NOFW
        const bool ok = true;
#else
        const bool ok = frame_ldl_cols(d, f, Fh, lam2, P, Q, CZ, lane, qc0, qc1, fw == 0 && it == 3);
#endif
        if (!ok && lane == 0 && fw == 0) okl = 0;
        // the frame waves meet again before the Schur tiles read every column of Q (the next frame's elimination
        // writes Q only after the next frame's sums meeting, which every wave reaches after its Schur tiles)
        KB_WAVE_SYNC();
        mt += NF;
        if (lane == 0) atomicAdd(&fcnt, 1);
        while (__hip_atomic_load(&fcnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < mt) __builtin_amdgcn_s_sleep(1);
        if (fw == 0 && it <= 8) KB_TSB(d, 22 + 4 * (it - 1));
#ifndef KB_DIAG_NOFW
        schur_tiles_accumulate6<TT>(P, Q, CZ, tii, tjj, acc, lane);
#endif
        if (fw == 0 && it <= 8) KB_TSB(d, 23 + 4 * (it - 1));
      }
      if (it < G) __syncthreads();  // the view waves' frame it is in VB[it & 1]
    }
    __syncthreads();  // the view waves' last barrier (their expansion of the block's camera sums is done)
    if (fuse && !xp) schur_tiles_store<TT, true>(prow + N * 136, C, tii, tjj, acc);
    // expanded partials: the view waves expanded the camera block during the last frame's elimination
    if (xp) schur_tiles_store_x<TT, true>(prow + N * 136, C, tii, tjj, acc, sm);
  }
  if (xp && vw) {
    // expanded partials: the g_c columns of the block's partial row (the cost column was written in the idle phase)
    const double* EX = sm;
    for (int e = tid; e < C; e += 64 * N) prow[e] = EX[W - C + e];
  }
  __syncthreads();  // okl final
  if (wave == 0) KB_TSB(d, 63);
  if (fuse && tid == 0) prow[N * 136 + W] = okl ? 0.0 : 1.0;  // non-PD frame blocks (summed)
  if (GNF && tid == 0) {  // the block's max |dx_f| (reduced with max by k_colsum)
    double m = 0.0;
    for (int q = 0; q < NW; ++q) m = fmax(m, wmx[q]);
    prow[d.Wp] = m;
  }
}

// ---------------------------------------------------------------------------------------------
// k_schur: Schur step from the stored arrow blocks (LM passes with a new lambda, per-call solve)
// ---------------------------------------------------------------------------------------------
template <int TW>
__global__ void __launch_bounds__(256) k_schur(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && (c->done || c->do_build)) return;  // rebuild passes ran it fused in k_build
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int C = d.C, W = d.W, N = d.N;
  const int nbz = (C + 16) >> 4, CZ = 16 * nbz;
  double* P = sm;           // [8][CZ]: [H_fc | g_f], zero-padded
  double* Q = P + 8 * CZ;   // [8][CZ]: [A | b], zero-padded
  __shared__ int okl;
  const double lam = gate ? c->lambda : d.host_lambda;
  const double lam2 = lam * lam;
  v4d acc[TW];
  int tii[TW], tjj[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
  schur_tiles_assign<TW>(nbz, tii, tjj);
  for (int q = threadIdx.x; q < 8 * CZ; q += blockDim.x)
    if (q >= 6 * CZ || (q % CZ) > C) P[q] = Q[q] = 0.0;
  if (threadIdx.x == 0) okl = 1;
  const int f0 = blockIdx.x * d.gframes, f1 = min(d.F, f0 + d.gframes);
  for (int f = f0; f < f1; ++f) {
    __syncthreads();
    for (int q = threadIdx.x; q < 6 * (C + 1); q += blockDim.x) {  // [H_fc | g_f] of frame f
      const int i = q / (C + 1), cc = q % (C + 1);
      P[i * CZ + cc] = cc < C ? d.Hfc[((size_t)f * 6 + i) * C + cc] : d.gf[(size_t)f * 6 + i];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const bool ok = frame_gj(d, f, d.Hff + (size_t)f * 36, lam2, P, Q, CZ, threadIdx.x);
      if (!ok && threadIdx.x == 0) okl = 0;
    }
    __syncthreads();
    schur_tiles_accumulate<TW>(P, Q, CZ, tii, tjj, acc);
  }
  double* prow = d.part + (size_t)blockIdx.x * d.Wr + N * 136;
  schur_tiles_store<TW>(prow, C, tii, tjj, acc);
  __syncthreads();
  if (threadIdx.x == 0) prow[W] = okl ? 0.0 : 1.0;
}

// ---------------------------------------------------------------------------------------------
// k_colsum: column sums of the block partials in fixed order: block (bx, ry) sums rows b = ry (mod 8) of
// 64 columns into part8[ry] (8 loads in flight per thread).  Grid (ceil(Wtot/64), 8).  The 8 rows are
// finished by the consumer: k_solve's staging (one GPU) or k_colfin (per-call path, all-reduce input).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_colsum(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  __shared__ double part[4][64];
  const int l = threadIdx.x & 63, w4 = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + l, ry = blockIdx.y;
  const bool mx = e >= d.Wp;  // max|dx_f| column(s): reduced with max (non-negative values)
  const int ec = min(e, d.Wp);
  double s = 0.0;
  constexpr int U = 16, step = 4 * kColsumRows;
  // the first batch of partial-row loads is issued with the gate's ctrl load (one round trip, not two): the
  // rows are always valid addresses, the values are only used once the pass is known to be live
  const int b00 = ry + kColsumRows * w4;
  const int done = c->done;
  double v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = d.part[(size_t)min(b00 + u * step, d.nblk - 1) * d.Wr + ec];
#pragma unroll
  for (int u = 0; u < U; ++u) KB_KEEP(v[u]);
  if (gate && done) return;
  for (int b0 = b00; b0 < d.nblk; b0 += U * step) {
    if (b0 != b00) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = d.part[(size_t)min(b0 + u * step, d.nblk - 1) * d.Wr + ec];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double x = (b0 + u * step < d.nblk) ? v[u] : 0.0;
      s = mx ? fmax(s, x) : s + x;
    }
  }
  part[w4][l] = s;
  __syncthreads();
  if (w4 == 0 && e < d.Wtot) {
    double v = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
    if (mx)  // one column per rank: this rank's max in its own column (GN fused passes), zero elsewhere
      v = (d.gn_fused && e - d.Wp == d.rank) ? fmax(fmax(part[0][l], part[1][l]), fmax(part[2][l], part[3][l]))
                                             : 0.0;
    d.part8[(size_t)ry * d.Wtot + e] = v;
  }
}

// k_colsum1: the column sums of the block partials in one pass, into part8 row 0 (the C > 64 path, whose consumer
// k_colimg then reads one row instead of kColsumRows): block bx sums 64 columns with 16 waves, wave w the rows
// b = w (mod 16) (all of a wave's row loads in flight at once for nblk <= 16 x 24), then the 16 wave sums in fixed
// order.  max for the max|dx_f| columns, as k_colsum.
constexpr int kColsum1Waves = 16;
__global__ void __launch_bounds__(64 * kColsum1Waves) k_colsum1(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  __shared__ double part[kColsum1Waves][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + l;
  const bool mx = e >= d.Wp;
  const int ec = min(e, d.Wp);
  constexpr int U = 24;
  const int done = c->done;
  double v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = d.part[(size_t)min(w + u * kColsum1Waves, d.nblk - 1) * d.Wr + ec];
#pragma unroll
  for (int u = 0; u < U; ++u) KB_KEEP(v[u]);
  if (gate && done) return;
  double s = 0.0;
  for (int b0 = w; b0 < d.nblk; b0 += U * kColsum1Waves) {
    if (b0 != w) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = d.part[(size_t)min(b0 + u * kColsum1Waves, d.nblk - 1) * d.Wr + ec];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double x = (b0 + u * kColsum1Waves < d.nblk) ? v[u] : 0.0;
      s = mx ? fmax(s, x) : s + x;
    }
  }
  part[w][l] = s;
  __syncthreads();
  if (w == 0 && e < d.Wtot) {
    double t = 0.0, m = 0.0;
#pragma unroll
    for (int q = 0; q < kColsum1Waves; ++q) {
      t += part[q][l];
      m = fmax(m, part[q][l]);
    }
    // one max column per rank: this rank's max in its own column (GN fused passes), zero elsewhere
    if (mx) t = (d.gn_fused && e - d.Wp == d.rank) ? m : 0.0;
    d.part8[e] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// k_colsumx (GN fused passes with expanded partials, KbDev::xexp): the column sums of the block partials in one pass
// (as k_colsum1: 16 waves x 64 columns, all of a wave's row loads in flight, the wave sums in fixed order), written
// straight into the k_solve image d.ximg instead of a row that k_colimg would expand:
//   S - lambda^2 I entry (a, b) -> its lower tile position (both triangles inside a diagonal tile), b_j -> row C,
//   g_c -> the aux slots [0, C), non-PD count -> aux slot C, cost -> aux slot n16, max|dx_f| of rank r -> n16 + 1 + r.
// Work column x: [0, C] = the g_c | cost columns, then every column from N * 136 on (S, b, non-PD, max|dx_f|).
// The identity padding and lambda^2 are k_solve's (they must not be summed over ranks).
// ---------------------------------------------------------------------------------------------
// a store of the direct all-reduce's exchange region: system scope (a write-through to memory, acknowledged there)
__device__ __forceinline__ void xar_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64 * kColsum1Waves) k_colsumx(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  __shared__ double part[kColsum1Waves][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = d.N, C = d.C, nb = (C + 16) >> 4, n16 = 16 * nb;
  const int x = blockIdx.x * 64 + l;
  const int nx = (C + 1) + (d.Wtot - N * 136);
  const int e = x <= C ? x : x - (C + 1) + N * 136;
  const bool mx = e >= d.Wp;
  const int ec = min(e, d.Wp);  // the block rows hold one max|dx_f| column (Wp); rank r's image slot takes it
  constexpr int U = 24;
  const int done = c->done;
  double v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = d.part[(size_t)min(w + u * kColsum1Waves, d.nblk - 1) * d.Wr + ec];
#pragma unroll
  for (int u = 0; u < U; ++u) KB_KEEP(v[u]);
  if (gate && done) return;
  double s = 0.0;
  for (int b0 = w; b0 < d.nblk; b0 += U * kColsum1Waves) {
    if (b0 != w) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = d.part[(size_t)min(b0 + u * kColsum1Waves, d.nblk - 1) * d.Wr + ec];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double y = (b0 + u * kColsum1Waves < d.nblk) ? v[u] : 0.0;
      s = mx ? fmax(s, y) : s + y;
    }
  }
  part[w][l] = s;
  __syncthreads();
  if (w != 0 || x >= nx) return;
  double t = 0.0, m = 0.0;
#pragma unroll
  for (int q = 0; q < kColsum1Waves; ++q) {
    t += part[q][l];
    m = fmax(m, part[q][l]);
  }
  const int ntz = kTileSz * nb * (nb + 1) / 2, aux = ntz;
  const int Wt = C * (C + 1) / 2, o = N * 136;
  double* img = d.ximg;
  const bool sys = d.xar != 0;
  if (sys) {  // direct all-reduce: the partial image of launch v = flags + 1 goes to region half v & 1 (k_xar)
    const unsigned long long f0 = reinterpret_cast<const unsigned long long*>(d.xar_buf)[0];
    img = d.xar_buf + kXarFlagDoubles + (size_t)((f0 + 1) & 1) * d.img_n;
  }
  // the exchange region is written with system-scope stores: each is acknowledged only once it is in memory, past
  // every L2, so when this kernel has completed the peers' system-scope loads (k_xar) see it, whatever any L2 holds
  auto put = [&](int i, double v) {
    if (sys)
      xar_store(img + i, v);
    else
      img[i] = v;
  };
  if (e < C) {
    put(aux + e, t);  // g_c
  } else if (e == C) {
    put(aux + n16, t);  // cost
  } else if (e < o + Wt) {
    const int u = e - o, a = cidx_col(u, C), b = u - (a * C - a * (a - 1) / 2) + a;  // a <= b
    put(tidx(b, a), t);
    if (a != b && (a >> 4) == (b >> 4)) put(tidx(a, b), t);  // diagonal tiles are whole
  } else if (e < o + Wt + C) {
    const int j = e - o - Wt;
    put(tidx(C, j), t);  // b as row C
    if ((j >> 4) == (C >> 4)) put(tidx(j, C), t);
  } else if (e < d.Wp) {
    put(aux + C, t);  // non-PD frame blocks
  } else {
    const int r = e - d.Wp;  // one max column per rank: this rank's max in its own slot, zero elsewhere
    put(aux + n16 + 1 + r, (d.gn_fused && r == d.rank) ? m : 0.0);
  }
}

// ---------------------------------------------------------------------------------------------
// k_xar: the direct all-reduce of the sharded k_solve image over xGMI (replaces the one collective
// of LinearSystemSolver.cpp:81-92's host sum): every rank's k_colsumx left its partial image in its own exchange
// region (half v & 1 of launch v); block b publishes "launch v" in its flag slot (system-scope release after an L2
// write-back), waits until every rank's block b has published v, then sums chunk b of the image over the ranks in
// rank order, reading the peers' regions over xGMI (system-scope loads), into d.simg.  Every rank sums the same
// values in the same order: bitwise-identical images on all ranks, and identical to the in-process group's rank-order
// sums.  Reuse: a rank overwrites half v & 1 at launch v + 2, which needs every peer at v + 1, i.e. done reading v.
// Ordering: k_colsumx wrote the partial image with system-scope stores and has completed (same stream), so the image is
// in memory before the flag's system-scope release; a peer reads the halves with system-scope loads only after its
// system-scope acquire of that flag.  A peer that never arrives ends the wait after d.xar_timeout ticks
// (KB_XAR_TIMEOUT_MS, default 10 s): ctrl->comm_err and ctrl->done, so every later kernel of the enqueued passes
// skips, and the host fails the call and agrees with the other ranks on the RCCL collective from then on.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_xar(KbDev d, int gate) {
  KbCtrl* c = d.ctrl;
  if (gate && c->done) return;
  __shared__ unsigned long long sv;
  __shared__ int err;
  __shared__ const double* pp[kXMaxRanksDev];
  const int b = blockIdx.x, tid = threadIdx.x, R = d.nranks;
  unsigned long long* own = reinterpret_cast<unsigned long long*>(d.xar_buf);
  if (tid < R) pp[tid] = d.xar_peers[tid];
  if (tid == 0) {
    const unsigned long long v = own[b] + 1;  // only block b of this rank writes slot b
    sv = v;
    err = 0;
    __hip_atomic_store(own + b, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const unsigned long long v = sv;
  if (tid < R) {  // lane q waits for rank q's block b
    const unsigned long long* pf = reinterpret_cast<const unsigned long long*>(pp[tid]) + b;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(pf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > d.xar_timeout) {
        err = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int n = d.img_n, per = (n + gridDim.x - 1) / gridDim.x, i0 = b * per, i1 = min(n, i0 + per);
  const size_t off = kXarFlagDoubles + (size_t)(v & 1) * n;
  // every rank's value of an entry is requested before any is summed (8 remote loads in flight per group), the sum
  // itself in rank order
  constexpr int kG = 8;
  for (int i = i0 + tid; i < i1; i += blockDim.x) {
    double s = 0.0;
    for (int q0 = 0; q0 < R; q0 += kG) {
      double v[kG];
#pragma unroll
      for (int u = 0; u < kG; ++u) {
        const int q = min(q0 + u, R - 1);
        v[u] = __longlong_as_double(__hip_atomic_load(reinterpret_cast<const unsigned long long*>(pp[q] + off + i),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      }
#pragma unroll
      for (int u = 0; u < kG; ++u)
        if (q0 + u < R) s = (q0 + u == 0) ? v[u] : s + v[u];
    }
    d.simg[i] = s;
  }
  if (tid == 0 && err) {  // the pass results are void: the rest of the enqueued passes skips (every kernel checks done)
    c->comm_err = 1;
    c->done = 1;
  }
}

// k_xar self-test input: rank r's image half `half` = (r + 1) / 8 + (i % 7) (exact sums in any order)
__global__ void __launch_bounds__(256) k_xar_fill(KbDev d, int half) {
  double* img = d.xar_buf + kXarFlagDoubles + (size_t)half * d.img_n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < d.img_n; i += gridDim.x * blockDim.x)
    xar_store(img + i, (d.rank + 1) * 0.125 + (double)(i % 7));  // the stores k_colsumx uses
}

// psum_local[e] = sum_r part8[r][e] (fixed order)
__global__ void __launch_bounds__(256) k_colfin(KbDev d, int gate) {
  if (gate && d.ctrl->done) return;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.Wtot) return;
  double v[kColsumRows];
#pragma unroll
  for (int r = 0; r < kColsumRows; ++r) v[r] = d.part8[(size_t)r * d.Wtot + q];
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < kColsumRows; ++r) acc = (q >= d.Wp) ? fmax(acc, v[r]) : acc + v[r];
  d.psum_local[q] = acc;
}

// entry e of the column sums: psum_rows rows (stride Wtot) summed in fixed order
__device__ __forceinline__ double psum_at(const KbDev& d, int e) {
  double v[kColsumRows];
#pragma unroll
  for (int r = 0; r < kColsumRows; ++r) v[r] = d.psum[(size_t)(r < d.psum_rows ? r : 0) * d.Wtot + e];
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < kColsumRows; ++r) acc += (r < d.psum_rows) ? v[r] : 0.0;
  return acc;
}

// max over the psum_rows rows (the max|dx_f| columns)
__device__ __forceinline__ double psum_max_at(const KbDev& d, int e) {
  double v[kColsumRows];
#pragma unroll
  for (int r = 0; r < kColsumRows; ++r) v[r] = d.psum[(size_t)(r < d.psum_rows ? r : 0) * d.Wtot + e];
  double m = v[0];
#pragma unroll
  for (int r = 1; r < kColsumRows; ++r) m = fmax(m, v[r]);
  return m;
}


// ---------------------------------------------------------------------------------------------
// camera block from the per-camera local sums (H_cc, g_c), shared by k_camexpand and k_solve
// H_{I_i,I_i} = Hs_i[II]; H_{I_i,B_j} = Hs_i[Id] K_{i,j}; H_{B_j,B_k} = sum_{i>max} K_{i,j}^T Hs_i[dd] K_{i,k}
// ---------------------------------------------------------------------------------------------
__device__ void cam_load(const KbDev& d, double* Hs, double* T) {
  const int N = d.N;
  for (int q = threadIdx.x; q < N * 256; q += blockDim.x) {
    const int cam = q >> 8, a = (q & 255) >> 4, b = q & 15;
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    Hs[q] = psum_at(d, cam * 136 + d16_index(lo, hi));
  }
  __syncthreads();
  for (int q = threadIdx.x; q < N * N * 36; q += blockDim.x) {
    const int e = q % 36, ik = q / 36, i = ik / N, k = ik % N;
    double s = 0.0;
    if (k < i) {
      const int a = e / 6, b = e % 6;
      const double* K = cam_K(d, d.ctrl->cur) + (size_t)(i * N + k) * 36;
#pragma unroll
      for (int m = 0; m < 6; ++m) s += Hs[i * 256 + a * 16 + m] * K[m * 6 + b];
    }
    T[q] = s;  // T_{i,k} = Hs_i[dd] K_{i,k}
  }
  __syncthreads();
}

__device__ double cam_entry(const KbDev& d, const double* Hs, const double* T, int p, int q) {
  const int N = d.N;
  const int kp = d.colinfo[p] >> 16, ip = (d.colinfo[p] >> 8) & 0xff, xp = d.colinfo[p] & 0xff;
  const int kq = d.colinfo[q] >> 16, iq = (d.colinfo[q] >> 8) & 0xff, xq = d.colinfo[q] & 0xff;
  double s = 0.0;
  if (kp == 0 && kq == 0) {
    if (ip == iq) s = Hs[ip * 256 + (6 + xp) * 16 + 6 + xq];
  } else if (kp == 0 && kq == 1) {
    if (iq < ip) {
      const double* K = cam_K(d, d.ctrl->cur) + (size_t)(ip * N + iq) * 36;
#pragma unroll
      for (int b = 0; b < 6; ++b) s += Hs[ip * 256 + (6 + xp) * 16 + b] * K[b * 6 + xq];
    }
  } else if (kp == 1 && kq == 0) {
    if (ip < iq) {
      const double* K = cam_K(d, d.ctrl->cur) + (size_t)(iq * N + ip) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Hs[iq * 256 + a * 16 + 6 + xq];
    }
  } else {
    const int m = ip > iq ? ip : iq;
    for (int i = m + 1; i < N; ++i) {
      const double* K = cam_K(d, d.ctrl->cur) + (size_t)(i * N + ip) * 36;
      const double* Tq = T + (size_t)(i * N + iq) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Tq[a * 6 + xq];
    }
  }
  return s;
}

__device__ double cam_grad(const KbDev& d, const double* Hs, int p) {
  const int N = d.N;
  const int kp = d.colinfo[p] >> 16, ip = (d.colinfo[p] >> 8) & 0xff, xp = d.colinfo[p] & 0xff;
  if (kp == 0) return Hs[ip * 256 + (6 + xp) * 16 + 15];
  double s = 0.0;
  for (int i = ip + 1; i < N; ++i) {
    const double* K = cam_K(d, d.ctrl->cur) + (size_t)(i * N + ip) * 36;
#pragma unroll
    for (int a = 0; a < 6; ++a) s += K[a * 6 + xp] * Hs[i * 256 + a * 16 + 15];
  }
  return s;
}

// per-call path: H_cc, g_c, cost at the build state (kb_get_normal_blocks / kb_get_rhs)
__global__ void __launch_bounds__(256) k_camexpand(KbDev d, int gate) {
  if (gate && d.ctrl->done) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int N = d.N, C = d.C;
  double* Hs = sm;
  double* T = Hs + N * 256;
  cam_load(d, Hs, T);
  for (int q = threadIdx.x; q < C * C; q += blockDim.x) d.Hcc[q] = cam_entry(d, Hs, T, q / C, q % C);
  for (int p = threadIdx.x; p < C; p += blockDim.x) d.gc[p] = cam_grad(d, Hs, p);
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < N; ++i) s += Hs[i * 256 + 255];
    d.cost_build[0] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// k_marg: the camera-block solve of aslam_incremental_calibration's LinearSolver (LinearSolver.cpp:299-466,
// analyzeMarginal :468-528) on the Schur-reduced system the build + k_schur (lambda = 0) + k_colsum produced:
//   S = H_cc - sum H_fc^T A_f,  b = g_c - sum H_fc^T b_f   (= Omega, b_r of reduceLeft/RightHandSide)
//   column scaling G_j = 1/sqrt(H_cc[j][j]) (0 below sqrt(rows * epsNorm), linalg.cpp:128-152)
//   SVD of G S G (Eigen::JacobiSVD, linalg.cpp:412-424) by cyclic two-sided Jacobi: the off-diagonal of the symmetric
//   matrix packed upper in LDS, V in LDS; the round-robin parallel ordering applies C/2 disjoint rotations per round.
//   One barrier per round: every thread owns one 2x2 block (pair k, pair l) or one (row of V, pair k) and derives the
//   rotations it needs itself from ping-pong copies of the diagonal and of the round's pair entries a_pq, which the
//   previous round's block owners wrote (each next-round pair entry lies in exactly one of this round's blocks);
//   a parallel threshold test before each sweep replaces the rotation-free sweep that ends the cyclic Jacobi
//   truncation at rankTol = sv_0 epsSVD C, x_r = G V_r diag(1/w) V_r^T G b (solveSVD, linalg.cpp:426-443)
// Warm start (mo.warm): the sweeps run on V0^T (G S G) V0 from the previous call's V0 (sorted columns, any orthogonal
// matrix is a valid start), V = V0 J...; the successive systems of a GN loop differ little, so the start is nearly
// diagonal and the quadratic convergence takes 2-3 sweeps instead of 8-10.  Every kMargWarmMax-th call is cold.
// One block of marg_threads(C).  LDS: marg_lds_doubles(C) doubles (C <= kMargMaxC).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int pk_up(int i, int j, int n) {  // packed upper index, any order
  const int a = min(i, j), b = max(i, j);
  return a * n - a * (a - 1) / 2 + (b - a);
}

// pair k of round r (M1 = m - 1 rounds per sweep): {r, M1} for k = 0, {(r + k) % M1, (r - k) % M1} otherwise
__device__ __forceinline__ void rr_pair(int M1, int r, int k, int& p, int& q) {
  int a = r + k, b = r - k;
  if (a >= M1) a -= M1;
  if (b < 0) b += M1;
  if (k == 0) b = M1;
  p = min(a, b);
  q = max(a, b);
}

// pair k of round r in the round-robin's own orientation: a = (r + k) % M1, b = (r - k) % M1 (b = M1 for k = 0)
__device__ __forceinline__ void rr_ab(int M1, int r, int k, int& a, int& b) {
  a = r + k;
  b = r - k;
  if (a >= M1) a -= M1;
  if (b < 0) b += M1;
  if (k == 0) b = M1;
}

// the pair of round r holding index i: its slot k, and i's partner
__device__ __forceinline__ int rr_slot(int M1, int h, int r, int i, int& partner) {
  if (i == M1) {
    partner = r;
    return 0;
  }
  int k1 = i - r;
  if (k1 < 0) k1 += M1;
  if (k1 == 0) {
    partner = M1;
    return 0;
  }
  if (k1 < h) {
    int b = r - k1;
    partner = b < 0 ? b + M1 : b;
    return k1;
  }
  const int k = M1 - k1;
  int a = r + k;
  partner = a >= M1 ? a - M1 : a;
  return k;
}

// 1/sqrt(x), x a normal double: v_rsq_f64 + two Newton steps
__device__ __forceinline__ double marg_rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = fma(y, fma(-hx * y, y, 0.5), y);
  return fma(y, fma(-hx * y, y, 0.5), y);
}

// the rotation threshold (Eigen's JacobiSVD test) |a_pq| > tol sqrt|a_pp a_qq|, squared (no sqrt on the chain);
// a_pq^2 underflowing against a zero diagonal product still rotates, as the unsquared test does
__device__ __forceinline__ bool marg_big(double app, double aqq, double apq) {
  const double a2 = apq * apq, pq = fabs(app * aqq);
  return (apq != 0.0) & ((a2 > (kMargJacobiTol * kMargJacobiTol) * pq) | ((a2 == 0.0) & (pq == 0.0)));
}

// sym.schur2's quotient form for magnitudes outside the half-angle form's range
__device__ __attribute__((noinline)) void marg_rot_wide(double dd, double e, double& c, double& s, double& t) {
  const double th = dd / e, ath = fabs(th);
  t = ath > 1e150 ? 0.5 / th : (th >= 0.0 ? 1.0 : -1.0) / (ath + sqrt(th * th + 1.0));
  c = 1.0 / sqrt(t * t + 1.0);
  s = t * c;
}

// the symmetric Schur rotation of one pair (the 2x2 step of the two-sided Jacobi), c = 1, s = t = 0 at or below the
// threshold.  t = tan(theta) is the root of t^2 + 2 th t - 1 = 0 of smaller magnitude, th = (a_qq - a_pp) / (2 a_pq)
// (Golub & Van Loan's sym.schur2); here from the half-angle identities without a division or an IEEE sqrt on the
// serial chain: d = a_qq - a_pp, e = 2 a_pq, r = |(d, e)|, cos 2theta = |d| / r, c^2 = (1 + cos 2theta) / 2,
// s = sgn(d) e / (2 r c), t = s / c -- two Newton-refined v_rsq.  Magnitudes outside [1e-140, 1e140] (never met by
// the scaled system) take the quotient form.
__device__ __forceinline__ bool marg_rot(double app, double aqq, double apq, double& c, double& s, double& t) {
  const bool big = marg_big(app, aqq, apq);
  const double dd = aqq - app, e = 2.0 * apq, ad = fabs(dd), ae = fabs(e);
  const double ir = marg_rsq(fma(dd, dd, e * e));
  const double hh = fma(0.5 * ad, ir, 0.5);
  const double ic = marg_rsq(hh);
  double ss = (dd >= 0.0 ? 0.5 : -0.5) * e * ir * ic, cc = hh * ic, tt = ss * ic;
  if (__builtin_expect(big & !((ad < 1e140) & (ae < 1e140) & ((ad > 1e-140) | (ae > 1e-140))), 0))
    marg_rot_wide(dd, e, cc, ss, tt);
  c = big ? cc : 1.0;
  s = big ? ss : 0.0;
  t = big ? tt : 0.0;
  return big;
}

// LDS of k_marg in doubles.  Full storage (kFull: both triangles of Omega, C padded to even m, V [C][m]) while it fits,
// else packed upper Omega and V [C][C]; then G, b_s, and V0 (the warm start) when it fits beside them
__host__ __device__ __forceinline__ bool marg_full(int C) {
  const int m = C + (C & 1);
  return m * m + C * m + 2 * C <= kMargLdsStage;
}
__host__ __device__ __forceinline__ int marg_lds_doubles(int C, bool& stage_v0) {
  const int m = C + (C & 1);
  const int base = marg_full(C) ? m * m + C * m + 2 * C : C * (C + 1) / 2 + C * C + 2 * C;
  stage_v0 = base + C * C <= kMargLdsStage;
  return stage_v0 ? base + C * C : base;
}

// k_marg's block: one thread per item (marg_threads), plus wave 0 for the rotations when Omega is stored full
__host__ __device__ __forceinline__ int marg_block(int C) {
  const int t = marg_threads(C) + (marg_full(C) ? 64 : 0);
  return t < kMargThreads ? t : kMargThreads;
}

// round r's partner test of an entry (x, y), x != y (round-robin: {r, M1} and pairs with x + y = 2r mod M1)
__device__ __forceinline__ bool rr_is_pair(int M1, int r, int c2, int x, int y) {
  if (y == M1) return x == r;
  if (x == M1) return y == r;
  const int s = x + y;
  return (s >= M1 ? s - M1 : s) == c2;
}

__device__ void marg_tail(const KbDev& d, double* nbase, int sok);

template <bool kFull>
__global__ void __launch_bounds__(kMargThreads) k_marg(KbDev d, KbMarg mo, int gate) {
  __shared__ double nbase[KB_MAX_CAMS * 7];  // gated: the candidate baselines (marg_tail)
  __shared__ int sok0;
  if (gate) {
    if (d.ctrl->done) return;
    if (!d.ctrl->do_build) {  // no new system: the camera step's tail alone, as the separate tail kernel ran it
      marg_tail(d, nbase, d.ctrl->solve_ok);
      return;
    }
  }
  extern __shared__ __attribute__((aligned(16))) double sm[];
  KB_TSM(d, 0);
  const int C = d.C, n = C, m = C + (C & 1), h = m / 2, M1 = m - 1, tid = threadIdx.x, nth = blockDim.x;
  const int lane = tid & 63;
  const int Wt = d.W - C, o0 = d.N * 136;
  const int ld = kFull ? m : n;  // row stride of V (and of A when full)
  bool stage;
  marg_lds_doubles(C, stage);
  double* A = sm;                                          // Omega: [m][m] full, or [C(C+1)/2] packed upper
  double* V = A + (kFull ? m * m : n * (n + 1) / 2);       // [n][ld]
  double* G = V + n * ld;                                  // [n]
  double* bs = G + n;                                      // [n]
  double* V0s = bs + n;                                    // [n][n] when staged
  auto aix = [&](int i, int j) { return kFull ? i * m + j : pk_up(i, j, n); };
  __shared__ double dg[2][kMargMaxC];          // diagonal, ping-pong by round
  __shared__ double ap[2][kMargMaxC];          // a_pq of the round's pairs: by slot k (packed: ping-pong by round)
  __shared__ double csr[2 * kMargMaxC];        // full storage: (c, s) of round r's pairs at (r & 1) kMargMaxC + 2k
  __shared__ int prodkl[64], prodsel[64], nprod;  // full storage: the producer blocks (k | l << 8, selectors)
  __shared__ int flag[3];
  __shared__ int okl, swarm;
  __shared__ double wsort[kMargMaxC];
  __shared__ int perm[kMargMaxC];
  __shared__ double tco[kMargMaxC];
  __shared__ double stat[4];
  __shared__ int srank;
  // ---- load: scaling, Omega = G S G, b_s = G b
  for (int i = tid; i < n; i += nth) {
    const double nrm = sqrt(d.Hcc[(size_t)i * C + i]);
    G[i] = mo.scaling ? (nrm < mo.norm_tol ? 0.0 : 1.0 / nrm) : 1.0;
  }
  if (tid == 0) {
    okl = !(psum_at(d, o0 + Wt + C) > 0.0);  // non-PD frame blocks
    sok0 = gate ? d.ctrl->solve_ok : 1;
    const int chain = (int)mo.info[5];
    swarm = (mo.warm && chain >= 1 && chain < kMargWarmMax) ? chain : 0;
    flag[0] = flag[1] = flag[2] = 0;
  }
  __syncthreads();
  KB_TSM(d, 1);
  const int warm = swarm;
  for (int e = tid; e < n * n; e += nth) {
    const int i = e / n, j = e - i * n;
    if (j >= i) {
      const double v = G[i] * (d.Hcc[(size_t)i * C + j] - psum_at(d, o0 + upper_index(i, j, C))) * G[j];
      A[aix(i, j)] = v;
      if (kFull) A[j * m + i] = v;
    }
    if (warm && stage) V0s[e] = mo.V[e];
  }
  if (kFull && m > n)  // the padding row / column of an odd C: the dummy index of the round-robin, never rotated
    for (int i = tid; i < m; i += nth) {
      A[n * m + i] = 0.0;
      A[i * m + n] = 0.0;
      if (i < n) V[i * ld + n] = 0.0;
    }
  for (int i = tid; i < n; i += nth) bs[i] = G[i] * (d.gc[i] - psum_at(d, o0 + Wt + i));
  __syncthreads();
  KB_TSM(d, 2);
  if (warm) {  // Omega <- V0^T Omega V0 (T = Omega V0 staged in V), V <- V0
    const double* V0 = stage ? V0s : mo.V;
    for (int e = tid; e < n * n; e += nth) {
      const int i = e / n, j = e - i * n;
      double s0 = 0.0, s1 = 0.0;
      int a = 0;
      for (; a + 1 < n; a += 2) {
        s0 += A[aix(i, a)] * V0[a * n + j];
        s1 += A[aix(i, a + 1)] * V0[(a + 1) * n + j];
      }
      if (a < n) s0 += A[aix(i, a)] * V0[a * n + j];
      V[i * ld + j] = s0 + s1;
    }
    __syncthreads();
    for (int e = tid; e < n * n; e += nth) {
      const int i = e / n, j = e - i * n;
      if (j < i) continue;
      double s0 = 0.0, s1 = 0.0;
      int a = 0;
      for (; a + 1 < n; a += 2) {
        s0 += V0[a * n + i] * V[a * ld + j];
        s1 += V0[(a + 1) * n + i] * V[(a + 1) * ld + j];
      }
      if (a < n) s0 += V0[a * n + i] * V[a * ld + j];
      A[aix(i, j)] = s0 + s1;
      if (kFull) A[j * m + i] = s0 + s1;
    }
    __syncthreads();
    for (int e = tid; e < n * n; e += nth) {
      const int i = e / n, j = e - i * n;
      V[i * ld + j] = V0[e];
    }
  } else {
    for (int e = tid; e < n * n; e += nth) {
      const int i = e / n, j = e - i * n;
      V[i * ld + j] = (i == j) ? 1.0 : 0.0;
    }
  }
  KB_TSM(d, 3);
  int sweeps = 0;
  const double* w;
  if constexpr (kFull) {
    // ---- full storage: one barrier per round, the rotations one round ahead.  Round r's rotations (c, s) are in
    // csr[r & 1] before round r starts.  During round r, wave 0 (a) applies round r to the off-diagonal blocks that hold
    // the next round's pair entries ("producer" blocks: fixed over the rounds, since the round-robin is
    // shift-invariant; each holds one or two of them), writes those entries into ap by slot, then (b) lanes k < h
    // compute round r + 1's rotation of pair k from the diagonal and ap (division-free half-angle form), publish it in
    // csr[(r + 1) & 1], and apply the pair's own 2x2 step (diagonal, pair entry exactly 0).  Meanwhile the other waves
    // apply round r (csr[r & 1]) to the remaining off-diagonal blocks (rows by pair k, columns by pair l) and to V
    // (row i, pair k).  Wave 0 owns everything round r + 1's rotations read, so the two run side by side; the round
    // ends in one block barrier.  Round 0 of a sweep is computed after the sweep's convergence test (one extra barrier).
    double* dgs = dg[0];
    double* aps = ap[0];
    for (int i = tid; i < m; i += nth) dgs[i] = A[i * m + i];
    for (int k = tid; k < h; k += nth) {
      int a, b;
      rr_ab(M1, 0, k, a, b);
      aps[k] = A[a * m + b];
    }
    if (tid == 0) nprod = 0;
    const int nob = h * (h - 1) / 2, total = nob + n * h, ith = nth - 64, nit = (total + ith - 1) / ith;
    static_assert((kMargFullMaxC / 2) * (kMargFullMaxC / 2 - 1) / 2 + kMargFullMaxC * (kMargFullMaxC / 2) <=
                      (kMargThreads - 64) * kMargItems,
                  "k_marg items per thread (full storage)");
    int ik[kMargItems], il[kMargItems], isel[kMargItems];
    const int rn0 = M1 > 1 ? 1 : 0, c20 = (2 * rn0) % M1;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kMargItems; ++j) {
      const int bI = tid - 64 + j * ith;
      ik[j] = -1;
      il[j] = 0;
      isel[j] = 0;
      if (tid < 64) continue;
      if (bI < nob) {  // strictly upper (k, l): index k (2h - k - 1) / 2 + (l - k - 1)
        const float b2 = 2.0f * h - 1.0f;
        int k = (int)((b2 - sqrtf(b2 * b2 - 8.0f * bI)) * 0.5f);
        k = max(0, min(k, h - 2));
        while (k > 0 && k * (2 * h - k - 1) / 2 > bI) --k;
        while (k + 1 < h - 1 && (k + 1) * (2 * h - k - 2) / 2 <= bI) ++k;
        const int l = bI - k * (2 * h - k - 1) / 2 + k + 1;
        ik[j] = k;
        il[j] = l;
        int ak, bk, al, bl, sel = 0, ns = 0;
        rr_ab(M1, 0, k, ak, bk);
        rr_ab(M1, 0, l, al, bl);
        for (int e = 0; e < 4; ++e) {  // entry e = (row a_k | b_k) x (column a_l | b_l), its slot next round
          const int x = (e >> 1) ? bk : ak, y = (e & 1) ? bl : al;
          if (ns < 2 && rr_is_pair(M1, rn0, c20, x, y)) {
            int partner;
            const int K = rr_slot(M1, h, rn0, x, partner);
            sel |= (1 | (e << 1) | (K << 3)) << (12 * ns);
            ++ns;
          }
        }
        if (sel) {  // a producer block: wave 0's
          const int q = atomicAdd(&nprod, 1);
          prodkl[q] = k | (l << 8);
          prodsel[q] = sel;
          ik[j] = -1;
        }
      } else if (bI < total) {
        const int e = bI - nob, i = e / h;
        ik[j] = e - i * h;
        il[j] = -1 - i;
      }
    }
    __syncthreads();
    // wave 0: lane L < nprod owns producer block L
    int pk = 0, pl = 0, psel = 0;
    if (tid < 64 && lane < nprod) {
      pk = prodkl[lane] & 0xff;
      pl = prodkl[lane] >> 8;
      psel = prodsel[lane];
    }
    KB_TSM(d, 4);
    // the rotation of pair k of round rr (lanes k < h of wave 0) into csr[rr & 1], and the pair's own 2x2 step
    auto pair_step = [&](int rr, int k) {
      int a, b;
      rr_ab(M1, rr, k, a, b);
      const double aaa = dgs[a], abb = dgs[b], aab = aps[k];
      double c, sn, t;
#ifdef KB_STAMPS
      const bool rot = (d.dbg_flags & 4) ? (c = 1.0, sn = 0.0, t = 0.0, false) : marg_rot(aaa, abb, aab, c, sn, t);
#else
      const bool rot = marg_rot(aaa, abb, aab, c, sn, t);
#endif
      double* cs = csr + (rr & 1) * kMargMaxC;
      cs[2 * k] = c;
      cs[2 * k + 1] = sn;
      if (rot) {
        dgs[a] = aaa - t * aab;
        dgs[b] = abb + t * aab;
        A[a * m + b] = 0.0;
        A[b * m + a] = 0.0;
      }
      if (M1 == 1) aps[k] = rot ? 0.0 : aab;  // one round per sweep: the same pair next round
    };
    // an off-diagonal block (k, l) of round r with the rotations cs (unrotated: y = x exactly); returns y
    auto block_step = [&](int r, int k, int l, const double* cs, double (&y)[4]) {
      int ak, bk, al, bl;
      rr_ab(M1, r, k, ak, bk);
      rr_ab(M1, r, l, al, bl);
      const double ck = cs[2 * k], sk = cs[2 * k + 1], cl = cs[2 * l], sl = cs[2 * l + 1];
      const double x00 = A[ak * m + al], x01 = A[ak * m + bl], x10 = A[bk * m + al], x11 = A[bk * m + bl];
      const double t00 = ck * x00 - sk * x10, t01 = ck * x01 - sk * x11;
      const double t10 = sk * x00 + ck * x10, t11 = sk * x01 + ck * x11;
      y[0] = cl * t00 - sl * t01;
      y[1] = sl * t00 + cl * t01;
      y[2] = cl * t10 - sl * t11;
      y[3] = sl * t10 + cl * t11;
      if (sk != 0.0 || sl != 0.0) {
        A[ak * m + al] = y[0];
        A[al * m + ak] = y[0];
        A[ak * m + bl] = y[1];
        A[bl * m + ak] = y[1];
        A[bk * m + al] = y[2];
        A[al * m + bk] = y[2];
        A[bk * m + bl] = y[3];
        A[bl * m + bk] = y[3];
      }
    };
    for (;; ++sweeps) {
      {
        bool v = false;
        for (int e = tid; e < n * n; e += nth) {
          const int i = e / n, j = e - i * n;
          if (j > i) v = v || marg_big(dgs[i], dgs[j], A[i * m + j]);
        }
        if (tid == 0) flag[(sweeps + 1) % 3] = 0;  // last read after sweep - 2's test
        if (__any(v) && lane == 0) flag[sweeps % 3] = 1;
        __syncthreads();
        if (flag[sweeps % 3] == 0 || sweeps == kMargMaxSweeps) break;
      }
      if (tid < h) pair_step(0, tid);  // round 0's rotations
      __syncthreads();
      if (sweeps == 0) KB_TSM(d, 5);
      for (int r = 0; r < M1; ++r) {
        const double* cs = csr + (r & 1) * kMargMaxC;
        if (tid < 64) {
          if (lane < nprod) {  // (a) the producer blocks: round r, then the next round's pair entries by slot
            double y[4];
            block_step(r, pk, pl, cs, y);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int su = psel >> (12 * u);
              if (su & 1) {
                const int e = (su >> 1) & 3;
                aps[(su >> 3) & 0x1ff] = e == 0 ? y[0] : e == 1 ? y[1] : e == 2 ? y[2] : y[3];
              }
            }
          }
          if (r + 1 < M1 && lane < h) pair_step(r + 1, lane);  // (b) round r + 1's rotations (the wave's own writes)
        } else {
#pragma unroll
          for (int j = 0; j < kMargItems; ++j) {
            if (j >= nit) break;  // block-uniform
            const int k = ik[j], l = il[j];
            if (k < 0) continue;
            if (l >= 0) {
              double y[4];
              block_step(r, k, l, cs, y);
            } else {
              const double ck = cs[2 * k], sk = cs[2 * k + 1];
              if (sk != 0.0) {  // V <- V J: row i, pair k
                int ak, bk;
                rr_ab(M1, r, k, ak, bk);
                double* Vi = V + (-1 - l) * ld;
                const double va = Vi[ak], vb = Vi[bk];
                Vi[ak] = ck * va - sk * vb;
                Vi[bk] = sk * va + ck * vb;
              }
            }
          }
        }
        __syncthreads();
        if (sweeps == 0 && r == 0) KB_TSM(d, 6);
      }
      if (sweeps == 0) KB_TSM(d, 7);
    }
    w = dgs;
  } else {
    // ---- round 0's diagonal and pair entries
    for (int i = tid; i < n; i += nth) dg[0][i] = A[aix(i, i)];
    if (kFull && m > n && tid == 0) dg[0][n] = 0.0;
    __syncthreads();
    for (int k = tid; k < h; k += nth) {
      int p, q;
      rr_pair(M1, 0, k, p, q);
      if (kFull) ap[0][p] = A[p * m + q];
      else ap[0][k] = q < n ? A[pk_up(p, q, n)] : 0.0;
    }
    // ---- this thread's items, fixed over the rounds: [0, nblk) the 2x2 blocks (k <= l) of the pairs, then
    // [nblk, nblk + n h) (row i of V, pair k); il = -1 - i marks a V item, ik = -1 an idle slot
    const int nblk = h * (h + 1) / 2, total = nblk + n * h, nit = (total + nth - 1) / nth;
    static_assert(kMargThreads * kMargItems >= (kMargMaxC / 2) * (kMargMaxC / 2 + 1) / 2 + kMargMaxC * (kMargMaxC / 2),
                  "k_marg items per thread");
    int ik[kMargItems], il[kMargItems];
  #pragma unroll
    for (int j = 0; j < kMargItems; ++j) {
      const int bI = tid + j * nth;
      ik[j] = -1;
      il[j] = 0;
      if (bI < nblk) {  // upper (k, l): index k (2h - k + 1) / 2 + (l - k)
        int k = (int)((2.0f * h + 1.0f - sqrtf((2.0f * h + 1.0f) * (2.0f * h + 1.0f) - 8.0f * bI)) * 0.5f);
        k = max(0, min(k, h - 1));
        while (k > 0 && k * (2 * h - k + 1) / 2 > bI) --k;
        while (k + 1 < h && (k + 1) * (2 * h - k) / 2 <= bI) ++k;
        ik[j] = k;
        il[j] = k + (bI - k * (2 * h - k + 1) / 2);
      } else if (bI < total) {
        const int e = bI - nblk, i = e / h;
        ik[j] = e - i * h;
        il[j] = -1 - i;
      }
    }
    __syncthreads();
    KB_TSM(d, 4);
    // ---- Jacobi sweeps.  Each sweep is preceded by the convergence test of the sweep it would be: no pair above the
    // rotation threshold means no rotation anywhere in it (nothing changes), so the loop ends without running it.
    // One barrier per round: every item derives the rotations it needs from dg / ap of the round, which the previous
    // round's owners wrote (each next-round pair entry lies in exactly one of this round's off-diagonal blocks).
    int it = 0;
    for (;; ++sweeps) {
      {
        const double* dgc = dg[it & 1];
        bool v = false;
        for (int e = tid; e < n * n; e += nth) {
          const int i = e / n, j = e - i * n;
          if (j > i) v = v || marg_big(dgc[i], dgc[j], A[aix(i, j)]);
        }
        if (tid == 0) flag[(sweeps + 1) % 3] = 0;  // last read after sweep - 2's test
        if (__any(v) && lane == 0) flag[sweeps % 3] = 1;
        __syncthreads();
        if (flag[sweeps % 3] == 0 || sweeps == kMargMaxSweeps) break;
      }
      if (sweeps == 0) KB_TSM(d, 5);
      for (int r = 0; r < M1; ++r, ++it) {
        const int cur = it & 1, nx = cur ^ 1, rn = (r + 1 == M1) ? 0 : r + 1;
        const int c2 = (2 * rn) % M1;
        const double* dgc = dg[cur];
        const double* apc = ap[cur];
        double* dgn = dg[nx];
        double* apn = ap[nx];
  #ifdef KB_STAMPS
        if (d.dbg_flags & 2) {
          __syncthreads();
          continue;
        }
  #endif
  #pragma unroll
        for (int j = 0; j < kMargItems; ++j) {
          if (j >= nit) break;  // block-uniform
          const int k = ik[j], l = il[j];
          if (k < 0) continue;
          int p, q;
          rr_pair(M1, r, k, p, q);
          if constexpr (kFull) {
            // padded: every index < m is valid storage, the dummy pair's a_pq is 0 and never rotates.  Straight-line:
            // every item reads its pairs' diagonal / a_pq and its 2x2 entries (rows p, q of Omega for a block, row i of
            // V twice for a V item) up front, derives both rotations, and only the writes are predicated
            const bool isV = l < 0, isD = l == k;
            int r2, s2;
            rr_pair(M1, r, isV ? k : l, r2, s2);
            const int row0 = isV ? -1 - l : p, row1 = isV ? row0 : q;
            const double* base = isV ? V : A;
            const double app = dgc[p], aqq = dgc[q], apq = apc[p];
            const double arr = dgc[r2], ass = dgc[s2], ars = apc[r2];
            const double x00 = base[row0 * ld + r2], x01 = base[row0 * ld + s2];
            const double x10 = base[row1 * ld + r2], x11 = base[row1 * ld + s2];
            double ck, sk, tk, cl, sl, tl;
  #ifdef KB_STAMPS
            const bool rk = (d.dbg_flags & 4) ? (ck = 1.0, sk = 0.0, tk = 0.0, false) : marg_rot(app, aqq, apq, ck, sk, tk);
            const bool rl = (d.dbg_flags & 4) ? (cl = 1.0, sl = 0.0, tl = 0.0, false) : marg_rot(arr, ass, ars, cl, sl, tl);
  #else
            const bool rk = marg_rot(app, aqq, apq, ck, sk, tk);
            const bool rl = marg_rot(arr, ass, ars, cl, sl, tl);
  #endif
            const double cr = isV ? 1.0 : ck, sr = isV ? 0.0 : sk;  // a V item rotates its columns only
            const double t00 = cr * x00 - sr * x10, t01 = cr * x01 - sr * x11;
            const double t10 = sr * x00 + cr * x10, t11 = sr * x01 + cr * x11;
            const double y00 = cl * t00 - sl * t01, y01 = sl * t00 + cl * t01;
            const double y10 = cl * t10 - sl * t11, y11 = sl * t10 + cl * t11;
            if (isD) {  // diagonal block: the pair's own 2x2 step, the pair entry exactly 0
              dgn[p] = rk ? app - tk * apq : app;
              dgn[q] = rk ? aqq + tk * apq : aqq;
              if (rk) {
                A[p * m + q] = 0.0;
                A[q * m + p] = 0.0;
              }
              if (M1 == 1) apn[p] = rk ? 0.0 : apq;  // one round per sweep: the same pair next round
            } else if (isV) {  // V <- V J: row i, pair k
              if (rl) {
                V[row0 * ld + r2] = y00;
                V[row0 * ld + s2] = y01;
              }
            } else {  // off-diagonal block (k, l): rows by pair k, columns by pair l (unrotated: y = x exactly)
              if (rk || rl) {
                A[p * m + r2] = y00;
                A[r2 * m + p] = y00;
                A[p * m + s2] = y01;
                A[s2 * m + p] = y01;
                A[q * m + r2] = y10;
                A[r2 * m + q] = y10;
                A[q * m + s2] = y11;
                A[s2 * m + q] = y11;
              }
              if (rr_is_pair(M1, rn, c2, p, r2)) apn[min(p, r2)] = y00;
              if (rr_is_pair(M1, rn, c2, p, s2)) apn[min(p, s2)] = y01;
              if (rr_is_pair(M1, rn, c2, q, r2)) apn[min(q, r2)] = y10;
              if (rr_is_pair(M1, rn, c2, q, s2)) apn[min(q, s2)] = y11;
            }
          } else {
            const bool qv = q < n;
            const double app = dgc[p], aqq = qv ? dgc[q] : 0.0, apq = qv ? apc[k] : 0.0;
            double ck, sk, tk;
            const bool rk = marg_rot(app, aqq, apq, ck, sk, tk);
            if (l == k) {
              if (rk) {
                dgn[p] = app - tk * apq;
                dgn[q] = aqq + tk * apq;
                A[pk_up(p, q, n)] = 0.0;
              } else {
                dgn[p] = app;
                if (qv) dgn[q] = aqq;
              }
              if (M1 == 1) apn[k] = rk ? 0.0 : apq;
            } else if (l >= 0) {
              int r2, s2;
              rr_pair(M1, r, l, r2, s2);
              const bool sv = s2 < n;
              const int ipr = pk_up(p, r2, n), ips = pk_up(p, s2, n), iqr = pk_up(q, r2, n), iqs = pk_up(q, s2, n);
              double apr = A[ipr], aps = sv ? A[ips] : 0.0, aqr = qv ? A[iqr] : 0.0, aqs = (qv && sv) ? A[iqs] : 0.0;
              double cl, sl, tl;
              const bool rl = marg_rot(dgc[r2], sv ? dgc[s2] : 0.0, sv ? apc[l] : 0.0, cl, sl, tl);
              if (rk || rl) {
                const double tpr = ck * apr - sk * aqr, tps = ck * aps - sk * aqs;
                const double tqr = sk * apr + ck * aqr, tqs = sk * aps + ck * aqs;
                apr = cl * tpr - sl * tps;
                aps = sl * tpr + cl * tps;
                aqr = cl * tqr - sl * tqs;
                aqs = sl * tqr + cl * tqs;
                A[ipr] = apr;
                if (sv) A[ips] = aps;
                if (qv) A[iqr] = aqr;
                if (qv && sv) A[iqs] = aqs;
              }
              int pa;
              int kk = rr_slot(M1, h, rn, p, pa);
              if (pa == r2) apn[kk] = apr;
              else if (sv && pa == s2) apn[kk] = aps;
              if (qv) {
                kk = rr_slot(M1, h, rn, q, pa);
                if (pa == r2) apn[kk] = aqr;
                else if (sv && pa == s2) apn[kk] = aqs;
              }
            } else if (rk) {
              double* Vi = V + (-1 - l) * ld;
              const double vp = Vi[p], vq = Vi[q];
              Vi[p] = ck * vp - sk * vq;
              Vi[q] = sk * vp + ck * vq;
            }
          }
        }
        __syncthreads();
        if (sweeps == 0 && r == 0) KB_TSM(d, 6);
      }
      if (sweeps == 0) KB_TSM(d, 7);
    }
    w = dg[it & 1];
  }
  KB_TSM(d, 8);
  // ---- sort by |w| descending (ties: lower index first); singular values |w|
  for (int i = tid; i < n; i += nth) {
    const double wi = w[i], ai = fabs(wi);
    int pos = 0;
    for (int j = 0; j < n; ++j) {
      const double aj = fabs(w[j]);
      pos += (aj > ai || (aj == ai && j < i)) ? 1 : 0;
    }
    wsort[pos] = wi;
    perm[pos] = i;
  }
  __syncthreads();
  KB_TSM(d, 9);
  for (int e = tid; e < n * n; e += nth) {
    const int r = e / n, j = e - r * n;
    mo.V[e] = V[r * ld + perm[j]];
  }
  for (int j = tid; j < n; j += nth) mo.sv[j] = fabs(wsort[j]);
  if (tid < 64) {  // rankTol, estimateNumericalRank, svGap, log2 sum (linalg.cpp:243-282; LinearSolver.cpp:197-201)
    const double tol = (mo.svd_tol != -1.0) ? mo.svd_tol : fabs(wsort[0]) * mo.eps_svd * n;
    // estimateNumericalRank counts down from the end while |w| <= tol: rank = 1 + the last index above tol (>= 1)
    int last = 0;
    for (int i = lane; i < n; i += 64)
      if (fabs(wsort[i]) > tol) last = max(last, i);
    for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o));
    const int rank = last + 1;
    double l2 = 0.0;
    for (int i = lane; i < rank; i += 64) l2 += log(fabs(wsort[i]));
    for (int o = 32; o > 0; o >>= 1) l2 += __shfl_xor(l2, o);
    if (lane == 0) {
      srank = rank;
      stat[0] = tol;
      stat[1] = rank < n ? fabs(wsort[rank - 1]) / fabs(wsort[rank]) : __builtin_inf();
      stat[2] = l2 / log(2.0);
    }
  }
  __syncthreads();
  KB_TSM(d, 10);
  const int rank = srank;
  // ---- truncated solve: t_j = (v_j . b_s) / w_j, x = G V_r t
  for (int j = tid; j < rank; j += nth) {
    const int pj = perm[j];
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += V[i * ld + pj] * bs[i];
    tco[j] = s / wsort[j];
  }
  __syncthreads();
  if (mo.write_dx) {
    for (int i = tid; i < n; i += nth) {
      double s = 0.0;
      for (int j = 0; j < rank; ++j) s += V[i * ld + perm[j]] * tco[j];
      d.dx[i] = G[i] * s;
    }
  }
  if (tid == 0) {
    mo.info[0] = rank;
    mo.info[1] = sweeps;
    mo.info[2] = stat[0];
    mo.info[3] = stat[1];
    mo.info[4] = stat[2];
    bool fin = true;
    for (int i = 0; i < n; ++i) fin = fin && isfinite(wsort[i]);
    mo.info[5] = fin ? (double)(warm ? warm + 1 : 1) : 0.0;  // a non-finite result restarts cold
    if (!okl) d.ctrl->solve_ok = 0;
  }
  KB_TSM(d, 11);
  if (gate) {  // the device loop: the camera step's statistics, design variables and chains (marg_tail)
    __syncthreads();  // dx_c written
    marg_tail(d, nbase, sok0 && okl);
  }
}

// ---------------------------------------------------------------------------------------------
// marg_tail (kb_optimize_marginal, the device-resident IncrementalEstimator loop; the end of the gated k_marg): after its truncated-SVD
// camera step, what k_solve's tail does after its LDL^T -- the camera dx statistics (max |dx_c|, dx_c.dx_c, dx_c.g_c),
// the camera design variables of the candidate slot (intrinsics additive, baselines by the pose update) and the
// candidate's camera chains -- and the pass is marked pending for k_backsub / k_post
// ---------------------------------------------------------------------------------------------
// sok: the solve succeeded (ctrl->solve_ok after k_marg); every thread of the block calls it
__device__ void marg_tail(const KbDev& d, double* nbase, int sok) {
  KbCtrl* c = d.ctrl;
  const int cur = c->cur;
  const int tid = threadIdx.x, nth = blockDim.x, C = d.C, N = d.N;
  if (tid == 0) c->pending = 1;
  if (!sok) return;
  if (tid < 64) {
    double mx = 0.0, dd = 0.0, dr = 0.0;
    for (int i = tid; i < C; i += 64) {
      const double x = d.dx[i], g = d.gc[i];
      mx = fmax(mx, fabs(x));
      dd += x * x;
      dr += x * g;
    }
    mx = wave_max_d(mx);
    dd = wave_sum_d(dd);
    dr = wave_sum_d(dr);
    if (tid == 0) {
      d.camstat[0] = mx;
      d.camstat[1] = dd;
      d.camstat[2] = dr;
    }
  }
  const double* in = d.state + (size_t)cur * d.S;
  double* out = d.state + (size_t)(1 - cur) * d.S;
  for (int q = tid; q < N * KB_MAX_INTR; q += nth) {
    const int cm = q / KB_MAX_INTR, x = q - KB_MAX_INTR * cm;
    out[q] = in[q] + (x < cam_arg(d.nintr, cm) ? d.dx[cam_arg(d.col_intr, cm) + x] : 0.0);
  }
  for (int j = tid; j < N - 1; j += nth) {
    double bq[7], d6[6], nb[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) bq[q] = in[d.off_base + 7 * j + q];
    const int cb = cam_arg(d.col_base, j);
#pragma unroll
    for (int q = 0; q < 6; ++q) d6[q] = d.dx[cb + q];
    update_pose(bq, d6, nb);
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      out[d.off_base + 7 * j + q] = nb[q];
      nbase[7 * j + q] = nb[q];
    }
  }
  __syncthreads();
  chain_block(d, nbase, 1 - cur, nth);  // chains of the candidate (k_backsub's cost, the next build if accepted)
}

// ---------------------------------------------------------------------------------------------
// k_solve: S = H_cc + lambda^2 I - sum Y^T Y, b = g_c - sum Y^T z (packed lower, staged in LDS);
// LDL^T (one wave when C <= 64, else the block with one barrier per column); dx_c; camera DV update
// ---------------------------------------------------------------------------------------------

__device__ __forceinline__ double cam_entry_l(const int N, const int* ci, const double* Hs, const double* T, const double* K, int p,
                              int q) {
  const int kp = ci[p] >> 16, ip = (ci[p] >> 8) & 0xff, xp = ci[p] & 0xff;
  const int kq = ci[q] >> 16, iq = (ci[q] >> 8) & 0xff, xq = ci[q] & 0xff;
  double s = 0.0;
  if (kp == 0 && kq == 0) {
    if (ip == iq) s = Hs[ip * 256 + (6 + xp) * 16 + 6 + xq];
  } else if (kp == 0 && kq == 1) {
    if (iq < ip) {
      const double* Kk = K + (size_t)(ip * N + iq) * 36;
#pragma unroll
      for (int b = 0; b < 6; ++b) s += Hs[ip * 256 + (6 + xp) * 16 + b] * Kk[b * 6 + xq];
    }
  } else if (kp == 1 && kq == 0) {
    if (ip < iq) {
      const double* Kk = K + (size_t)(iq * N + ip) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += Kk[a * 6 + xp] * Hs[iq * 256 + a * 16 + 6 + xq];
    }
  } else {
    const int m = ip > iq ? ip : iq;
    for (int i = m + 1; i < N; ++i) {
      const double* Kk = K + (size_t)(i * N + ip) * 36;
      const double* Tq = T + (size_t)(i * N + iq) * 36;
#pragma unroll
      for (int a = 0; a < 6; ++a) s += Kk[a * 6 + xp] * Tq[a * 6 + xq];
    }
  }
  return s;
}

__device__ __forceinline__ double cam_grad_l(const int N, const int* ci, const double* Hs, const double* K, int p) {
  const int kp = ci[p] >> 16, ip = (ci[p] >> 8) & 0xff, xp = ci[p] & 0xff;
  if (kp == 0) return Hs[ip * 256 + (6 + xp) * 16 + 15];
  double s = 0.0;
  for (int i = ip + 1; i < N; ++i) {
    const double* Kk = K + (size_t)(i * N + ip) * 36;
#pragma unroll
    for (int a = 0; a < 6; ++a) s += Kk[a * 6 + xp] * Hs[i * 256 + a * 16 + 15];
  }
  return s;
}

// column-major packed lower index of (i, j), i >= j (== row-major packed upper index of (j, i))
__device__ __forceinline__ int cidx(int i, int j, int C) { return j * (2 * C - j - 1) / 2 + i; }

// ---------------------------------------------------------------------------------------------
// Blocked LDL^T of the camera block for C > 64 (configs[3]: C = 106), the right-hand side appended as row C.
// LDS layout: lower 16 x 16 tiles, tile (it, jt) at (it(it+1)/2 + jt) * kTileSz, row stride kTS, nb = ceil((C+1)/16)
// tile rows.  Row C holds b (diagonal 1), rows C+1 .. 16 nb - 1 the identity.  After the factorisation tile (i, q),
// i > q, holds W = L D (the unscaled sub-diagonal rows), a diagonal tile W strictly below its diagonal and D on it,
// rD = 1 / D.  Row C then holds y = Ltilde^-1 b: the forward solve comes out of the factorisation, z = y D^-1.
//
// Panel q (columns 16q .. 16q+15) is factored by nF(q) <= 2 "factor" waves with one matrix row per lane:
//   lanes 0..15 the rows of the diagonal tile (symmetric, read from the lower storage), lanes 16..63 the rows of three
//   tiles below (factor wave fw: tiles q+1+3fw .. q+3+3fw).  Step k broadcasts the current row k (lane k) with
//   v_readlane, so the diagonal factor and the panel's triangular solve are one 16-step register loop.
// Before that, each factor wave applies panel q-1 to its own tiles on v_mfma_f64_16x16x4f64 (the lookahead column;
// the diagonal tile into a private scratch copy), while 4 "update" waves apply panel q-1 to the remaining trailing
// tiles (i, j), j > q.  One block barrier per panel; the 106-pivot chain runs on the factor waves only.
// Same algebra as the scalar right-looking LDL^T (SparseCholeskyLinearSystemSolver.cpp:48-89 / Cholmod(impl).hpp:
// 387-399 factor the same matrix); only the accumulation order of the trailing updates differs.
// ---------------------------------------------------------------------------------------------

// LDS index of lower entry (i, j), i >= j, of the staged camera block: packed column-major (CM > 0) or tiles
template <int CM>
__device__ __forceinline__ int sidx(int i, int j, int C) {
  if constexpr (CM > 0)
    return cidx(i, j, C);
  else
    return tidx(i, j);
}

// W_a (W_b D_q^-1)^T of two 16 x 16 tiles on MFMA (lane l: A[l & 15][k], B[k][l & 15]; acc[r] = entry
// ((l >> 4) + 4 r, l & 15))
__device__ __forceinline__ v4d tile_prod(const double* Wa, const double* Wb, const double* rdq, int lane) {
  v4d acc = {0.0, 0.0, 0.0, 0.0};
  const int r = lane & 15;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + (lane >> 4);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Wa[r * kTS + k], Wb[r * kTS + k] * rdq[k], acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ void tile_sub(const double* src, double* dst, const v4d& acc, int lane) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int e = ((lane >> 4) + 4 * r) * kTS + (lane & 15);
    dst[e] = src[e] - acc[r];
  }
}

// v_readlane of M doubles of one lane in one asm statement: each value gets its own SGPR pair, so the reads
// issue back to back and the FMAs that consume them do not wait on one readlane each (separate readlanes are
// scheduled into one reused SGPR pair under k_solve's SGPR pressure, which serialises them).  L: the lane.
template <int L>
__device__ __forceinline__ void rl1(double v0, double& o0) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  asm("s_nop 1\nv_readlane_b32 %0, %2, %4\nv_readlane_b32 %1, %3, %4\ns_nop 1"
      : "=s"(sl0), "=s"(sh0)
      : "v"(l0), "v"(h0), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
}
template <int L>
__device__ __forceinline__ void rl2(double v0, double v1, double& o0, double& o1) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  const unsigned long long b1 = __double_as_longlong(v1);
  const unsigned l1 = (unsigned)b1, h1 = (unsigned)(b1 >> 32);
  unsigned sl1, sh1;
  asm("s_nop 1\nv_readlane_b32 %0, %4, %8\nv_readlane_b32 %1, %5, %8\nv_readlane_b32 %2, %6, %8\nv_readlane_b32 %3, %7, %8\ns_nop 1"
      : "=s"(sl0), "=s"(sh0), "=s"(sl1), "=s"(sh1)
      : "v"(l0), "v"(h0), "v"(l1), "v"(h1), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
  o1 = __longlong_as_double(((unsigned long long)sh1 << 32) | sl1);
}
template <int L>
__device__ __forceinline__ void rl3(double v0, double v1, double v2, double& o0, double& o1, double& o2) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  const unsigned long long b1 = __double_as_longlong(v1);
  const unsigned l1 = (unsigned)b1, h1 = (unsigned)(b1 >> 32);
  unsigned sl1, sh1;
  const unsigned long long b2 = __double_as_longlong(v2);
  const unsigned l2 = (unsigned)b2, h2 = (unsigned)(b2 >> 32);
  unsigned sl2, sh2;
  asm("s_nop 1\nv_readlane_b32 %0, %6, %12\nv_readlane_b32 %1, %7, %12\nv_readlane_b32 %2, %8, %12\nv_readlane_b32 %3, %9, %12\nv_readlane_b32 %4, %10, %12\nv_readlane_b32 %5, %11, %12\ns_nop 1"
      : "=s"(sl0), "=s"(sh0), "=s"(sl1), "=s"(sh1), "=s"(sl2), "=s"(sh2)
      : "v"(l0), "v"(h0), "v"(l1), "v"(h1), "v"(l2), "v"(h2), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
  o1 = __longlong_as_double(((unsigned long long)sh1 << 32) | sl1);
  o2 = __longlong_as_double(((unsigned long long)sh2 << 32) | sl2);
}
template <int L>
__device__ __forceinline__ void rl4(double v0, double v1, double v2, double v3, double& o0, double& o1, double& o2, double& o3) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  const unsigned long long b1 = __double_as_longlong(v1);
  const unsigned l1 = (unsigned)b1, h1 = (unsigned)(b1 >> 32);
  unsigned sl1, sh1;
  const unsigned long long b2 = __double_as_longlong(v2);
  const unsigned l2 = (unsigned)b2, h2 = (unsigned)(b2 >> 32);
  unsigned sl2, sh2;
  const unsigned long long b3 = __double_as_longlong(v3);
  const unsigned l3 = (unsigned)b3, h3 = (unsigned)(b3 >> 32);
  unsigned sl3, sh3;
  asm("s_nop 1\nv_readlane_b32 %0, %8, %16\nv_readlane_b32 %1, %9, %16\nv_readlane_b32 %2, %10, %16\nv_readlane_b32 %3, %11, %16\nv_readlane_b32 %4, %12, %16\nv_readlane_b32 %5, %13, %16\nv_readlane_b32 %6, %14, %16\nv_readlane_b32 %7, %15, %16\ns_nop 1"
      : "=s"(sl0), "=s"(sh0), "=s"(sl1), "=s"(sh1), "=s"(sl2), "=s"(sh2), "=s"(sl3), "=s"(sh3)
      : "v"(l0), "v"(h0), "v"(l1), "v"(h1), "v"(l2), "v"(h2), "v"(l3), "v"(h3), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
  o1 = __longlong_as_double(((unsigned long long)sh1 << 32) | sl1);
  o2 = __longlong_as_double(((unsigned long long)sh2 << 32) | sl2);
  o3 = __longlong_as_double(((unsigned long long)sh3 << 32) | sl3);
}
template <int L>
__device__ __forceinline__ void rl5(double v0, double v1, double v2, double v3, double v4, double& o0, double& o1, double& o2, double& o3, double& o4) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  const unsigned long long b1 = __double_as_longlong(v1);
  const unsigned l1 = (unsigned)b1, h1 = (unsigned)(b1 >> 32);
  unsigned sl1, sh1;
  const unsigned long long b2 = __double_as_longlong(v2);
  const unsigned l2 = (unsigned)b2, h2 = (unsigned)(b2 >> 32);
  unsigned sl2, sh2;
  const unsigned long long b3 = __double_as_longlong(v3);
  const unsigned l3 = (unsigned)b3, h3 = (unsigned)(b3 >> 32);
  unsigned sl3, sh3;
  const unsigned long long b4 = __double_as_longlong(v4);
  const unsigned l4 = (unsigned)b4, h4 = (unsigned)(b4 >> 32);
  unsigned sl4, sh4;
  asm("s_nop 1\nv_readlane_b32 %0, %10, %20\nv_readlane_b32 %1, %11, %20\nv_readlane_b32 %2, %12, %20\nv_readlane_b32 %3, %13, %20\nv_readlane_b32 %4, %14, %20\nv_readlane_b32 %5, %15, %20\nv_readlane_b32 %6, %16, %20\nv_readlane_b32 %7, %17, %20\nv_readlane_b32 %8, %18, %20\nv_readlane_b32 %9, %19, %20\ns_nop 1"
      : "=s"(sl0), "=s"(sh0), "=s"(sl1), "=s"(sh1), "=s"(sl2), "=s"(sh2), "=s"(sl3), "=s"(sh3), "=s"(sl4), "=s"(sh4)
      : "v"(l0), "v"(h0), "v"(l1), "v"(h1), "v"(l2), "v"(h2), "v"(l3), "v"(h3), "v"(l4), "v"(h4), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
  o1 = __longlong_as_double(((unsigned long long)sh1 << 32) | sl1);
  o2 = __longlong_as_double(((unsigned long long)sh2 << 32) | sl2);
  o3 = __longlong_as_double(((unsigned long long)sh3 << 32) | sl3);
  o4 = __longlong_as_double(((unsigned long long)sh4 << 32) | sl4);
}
template <int L>
__device__ __forceinline__ void rl6(double v0, double v1, double v2, double v3, double v4, double v5, double& o0, double& o1, double& o2, double& o3, double& o4, double& o5) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  const unsigned long long b1 = __double_as_longlong(v1);
  const unsigned l1 = (unsigned)b1, h1 = (unsigned)(b1 >> 32);
  unsigned sl1, sh1;
  const unsigned long long b2 = __double_as_longlong(v2);
  const unsigned l2 = (unsigned)b2, h2 = (unsigned)(b2 >> 32);
  unsigned sl2, sh2;
  const unsigned long long b3 = __double_as_longlong(v3);
  const unsigned l3 = (unsigned)b3, h3 = (unsigned)(b3 >> 32);
  unsigned sl3, sh3;
  const unsigned long long b4 = __double_as_longlong(v4);
  const unsigned l4 = (unsigned)b4, h4 = (unsigned)(b4 >> 32);
  unsigned sl4, sh4;
  const unsigned long long b5 = __double_as_longlong(v5);
  const unsigned l5 = (unsigned)b5, h5 = (unsigned)(b5 >> 32);
  unsigned sl5, sh5;
  asm("s_nop 1\nv_readlane_b32 %0, %12, %24\nv_readlane_b32 %1, %13, %24\nv_readlane_b32 %2, %14, %24\nv_readlane_b32 %3, %15, %24\nv_readlane_b32 %4, %16, %24\nv_readlane_b32 %5, %17, %24\nv_readlane_b32 %6, %18, %24\nv_readlane_b32 %7, %19, %24\nv_readlane_b32 %8, %20, %24\nv_readlane_b32 %9, %21, %24\nv_readlane_b32 %10, %22, %24\nv_readlane_b32 %11, %23, %24\ns_nop 1"
      : "=s"(sl0), "=s"(sh0), "=s"(sl1), "=s"(sh1), "=s"(sl2), "=s"(sh2), "=s"(sl3), "=s"(sh3), "=s"(sl4), "=s"(sh4), "=s"(sl5), "=s"(sh5)
      : "v"(l0), "v"(h0), "v"(l1), "v"(h1), "v"(l2), "v"(h2), "v"(l3), "v"(h3), "v"(l4), "v"(h4), "v"(l5), "v"(h5), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
  o1 = __longlong_as_double(((unsigned long long)sh1 << 32) | sl1);
  o2 = __longlong_as_double(((unsigned long long)sh2 << 32) | sl2);
  o3 = __longlong_as_double(((unsigned long long)sh3 << 32) | sl3);
  o4 = __longlong_as_double(((unsigned long long)sh4 << 32) | sl4);
  o5 = __longlong_as_double(((unsigned long long)sh5 << 32) | sl5);
}
template <int L>
__device__ __forceinline__ void rl7(double v0, double v1, double v2, double v3, double v4, double v5, double v6, double& o0, double& o1, double& o2, double& o3, double& o4, double& o5, double& o6) {
  const unsigned long long b0 = __double_as_longlong(v0);
  const unsigned l0 = (unsigned)b0, h0 = (unsigned)(b0 >> 32);
  unsigned sl0, sh0;
  const unsigned long long b1 = __double_as_longlong(v1);
  const unsigned l1 = (unsigned)b1, h1 = (unsigned)(b1 >> 32);
  unsigned sl1, sh1;
  const unsigned long long b2 = __double_as_longlong(v2);
  const unsigned l2 = (unsigned)b2, h2 = (unsigned)(b2 >> 32);
  unsigned sl2, sh2;
  const unsigned long long b3 = __double_as_longlong(v3);
  const unsigned l3 = (unsigned)b3, h3 = (unsigned)(b3 >> 32);
  unsigned sl3, sh3;
  const unsigned long long b4 = __double_as_longlong(v4);
  const unsigned l4 = (unsigned)b4, h4 = (unsigned)(b4 >> 32);
  unsigned sl4, sh4;
  const unsigned long long b5 = __double_as_longlong(v5);
  const unsigned l5 = (unsigned)b5, h5 = (unsigned)(b5 >> 32);
  unsigned sl5, sh5;
  const unsigned long long b6 = __double_as_longlong(v6);
  const unsigned l6 = (unsigned)b6, h6 = (unsigned)(b6 >> 32);
  unsigned sl6, sh6;
  asm("s_nop 1\nv_readlane_b32 %0, %14, %28\nv_readlane_b32 %1, %15, %28\nv_readlane_b32 %2, %16, %28\nv_readlane_b32 %3, %17, %28\nv_readlane_b32 %4, %18, %28\nv_readlane_b32 %5, %19, %28\nv_readlane_b32 %6, %20, %28\nv_readlane_b32 %7, %21, %28\nv_readlane_b32 %8, %22, %28\nv_readlane_b32 %9, %23, %28\nv_readlane_b32 %10, %24, %28\nv_readlane_b32 %11, %25, %28\nv_readlane_b32 %12, %26, %28\nv_readlane_b32 %13, %27, %28\ns_nop 1"
      : "=s"(sl0), "=s"(sh0), "=s"(sl1), "=s"(sh1), "=s"(sl2), "=s"(sh2), "=s"(sl3), "=s"(sh3), "=s"(sl4), "=s"(sh4), "=s"(sl5), "=s"(sh5), "=s"(sl6), "=s"(sh6)
      : "v"(l0), "v"(h0), "v"(l1), "v"(h1), "v"(l2), "v"(h2), "v"(l3), "v"(h3), "v"(l4), "v"(h4), "v"(l5), "v"(h5), "v"(l6), "v"(h6), "i"(L));
  o0 = __longlong_as_double(((unsigned long long)sh0 << 32) | sl0);
  o1 = __longlong_as_double(((unsigned long long)sh1 << 32) | sl1);
  o2 = __longlong_as_double(((unsigned long long)sh2 << 32) | sl2);
  o3 = __longlong_as_double(((unsigned long long)sh3 << 32) | sl3);
  o4 = __longlong_as_double(((unsigned long long)sh4 << 32) | sl4);
  o5 = __longlong_as_double(((unsigned long long)sh5 << 32) | sl5);
  o6 = __longlong_as_double(((unsigned long long)sh6 << 32) | sl6);
}

// row[J0 .. J0 + M - 1] of lane L into bc[] (M <= 7: one asm statement)
template <int L, int J0, int M>
__device__ __forceinline__ void rl_chunk(const double (&row)[16], double (&bc)[16]) {
  if constexpr (M == 1) rl1<L>(row[J0], bc[J0]);
  else if constexpr (M == 2) rl2<L>(row[J0], row[J0 + 1], bc[J0], bc[J0 + 1]);
  else if constexpr (M == 3) rl3<L>(row[J0], row[J0 + 1], row[J0 + 2], bc[J0], bc[J0 + 1], bc[J0 + 2]);
  else if constexpr (M == 4)
    rl4<L>(row[J0], row[J0 + 1], row[J0 + 2], row[J0 + 3], bc[J0], bc[J0 + 1], bc[J0 + 2], bc[J0 + 3]);
  else if constexpr (M == 5)
    rl5<L>(row[J0], row[J0 + 1], row[J0 + 2], row[J0 + 3], row[J0 + 4], bc[J0], bc[J0 + 1], bc[J0 + 2], bc[J0 + 3],
           bc[J0 + 4]);
  else if constexpr (M == 6)
    rl6<L>(row[J0], row[J0 + 1], row[J0 + 2], row[J0 + 3], row[J0 + 4], row[J0 + 5], bc[J0], bc[J0 + 1], bc[J0 + 2],
           bc[J0 + 3], bc[J0 + 4], bc[J0 + 5]);
  else
    rl7<L>(row[J0], row[J0 + 1], row[J0 + 2], row[J0 + 3], row[J0 + 4], row[J0 + 5], row[J0 + 6], bc[J0], bc[J0 + 1],
           bc[J0 + 2], bc[J0 + 3], bc[J0 + 4], bc[J0 + 5], bc[J0 + 6]);
}
// row[J0 .. 15] of lane L into bc[], chunks of 7
template <int L, int J0>
__device__ __forceinline__ void rl_tail(const double (&row)[16], double (&bc)[16]) {
  if constexpr (J0 < 16) {
    constexpr int M = (16 - J0) < 7 ? (16 - J0) : 7;
    rl_chunk<L, J0, M>(row, bc);
    rl_tail<L, J0 + M>(row, bc);
  }
}

// 1/x by v_rcp_f64 + one Newton step (the pivot chain of the panel factorisation: one FMA pair shorter)
__device__ __forceinline__ double recip_d1(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// pivot steps K .. 15 of the lane-row panel factorisation (row k of the trailing matrix broadcast from lane k).
// Every lane applies f = row[k] / D_k: lanes above the pivot hold zeros right of their own pivot (their own step
// cancelled them: f = 1 against their own row), so no lane mask sits in the pivot chain.
template <int K>
__device__ __forceinline__ void panel_steps(double (&row)[16], int lane, int q, int C, bool& ok, double& rd) {
  if constexpr (K < 16) {
    double bc[16];
    rl_tail<K, K>(row, bc);  // bc[K] = D_K, bc[j] = S[K][j] (reading D_K on its own first measured no faster)
    const double Dk = bc[K];
    const double rdk = Dk > 0.0 ? recip_d1(Dk) : 0.0;
    const double f = row[K] * rdk;
#pragma unroll
    for (int j = K + 1; j < 16; ++j) row[j] -= f * bc[j];
    ok = ok & ((Dk > 0.0) | (16 * q + K >= C));  // bitwise: no branch per pivot
    rd = (lane == K) ? rdk : rd;
    panel_steps<K + 1>(row, lane, q, C, ok, rd);
  }
}

// x += (lane L's y within the lane's 16-lane row) * f: one v_fmac_f64 whose src0 is read through DPP row_newbcast:L
// (64-bit DPP, gfx90a+), so the broadcast of the pivot row costs no instruction of its own.  y and x may be the same
// register (operands are read before the write).
template <int L>
__device__ __forceinline__ void fmac_bc(double& x, double y, double f) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(y), "v"(f), "i"(L));
}
// the same after 2 wait states, for a source a VALU instruction has just written (a dependent chain of DPP reads)
template <int L>
__device__ __forceinline__ void fmac_bc_dep(double& x, double y, double f) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(x) : "v"(y), "v"(f), "i"(L));
}
template <int L>
__device__ __forceinline__ void fmac_bc_self(double& x, double f) {
  asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(f), "i"(L));
}

// lane L's v within the lane's 16-lane row (64-bit DPP row_newbcast as two 32-bit moves), after 2 wait states: the
// DPP read hazard of a VGPR that a VALU instruction has just written is not seen by the compiler through inline asm,
// so the wait sits inside the statement
template <int L>
__device__ __forceinline__ double bcast16_dep(double v) {
  const unsigned long long b = __double_as_longlong(v);
  unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32), olo, ohi;
  asm volatile(
      "s_nop 1\n\tv_mov_b32_dpp %0, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xf\n\t"
      "v_mov_b32_dpp %1, %3 row_newbcast:%4 row_mask:0xf bank_mask:0xf"
      : "=&v"(olo), "=&v"(ohi)
      : "v"(lo), "v"(hi), "i"(L));
  return __longlong_as_double(((unsigned long long)ohi << 32) | olo);
}

// updates of step K for columns J .. 15: the below row first (it reads the pivot row's column J before the diagonal
// row's own update of it), then the diagonal row
template <int K, int J>
__device__ __forceinline__ void panel2_cols(double (&dr)[16], double (&br)[16], double nfd, double nfb) {
  if constexpr (J < 16) {
    fmac_bc<K>(br[J], dr[J], nfb);
    fmac_bc_self<K>(dr[J], nfd);
    panel2_cols<K, J + 1>(dr, br, nfd, nfb);
  }
}

// pivot steps K .. 15 of the replicated-diagonal panel factorisation (panel_factor2): every 16-lane row holds the
// diagonal tile (lane r: its row r) and one tile below (lane r: that tile's row r).  Step K reads D_K and the pivot row's
// entries from lane K of the lane's own 16-lane row, by DPP row_newbcast fused into the FMAs (no v_readlane / SGPR hop,
// no LDS round trip).  Lanes above the pivot hold zeros right of their own pivot (their own step cancelled them), so no
// lane mask sits in the pivot chain.
template <int K>
__device__ __forceinline__ void panel2_steps(double (&dr)[16], double (&br)[16], int r, int q, int C, bool& ok,
                                             double& rd) {
  if constexpr (K < 16) {
    // D_K from lane K (its row's pivot), with the DPP wait inside the statement: dr[K] may have been written by the
    // previous step's last FMA just before (K = 15); every later DPP read of this step follows it
    const double Dk = bcast16_dep<K>(dr[K]);
    const double rdk = Dk > 0.0 ? recip_d1(Dk) : 0.0;
    const double nfd = -(dr[K] * rdk), nfb = -(br[K] * rdk);
    panel2_cols<K, K + 1>(dr, br, nfd, nfb);
    ok = ok & ((Dk > 0.0) | (16 * q + K >= C));  // bitwise: no branch per pivot
    rd = (r == K) ? rdk : rd;
    panel2_steps<K + 1>(dr, br, r, q, C, ok, rd);
  }
}

// panel2_steps with a one-step lookahead: step K's column K + 1 first, then step K + 1's pivot (D_{K+1} by DPP, the
// reciprocal, its multipliers), then step K's columns K + 2 .. 15, so that the pivot's broadcast -> v_rcp -> Newton
// chain issues while the bulk of step K's FMAs is still in the wave's stream (in-order issue: without the lookahead
// every pivot waits behind the previous step's 2 (15 - K) FMAs).  Same operations and operands per entry as
// panel2_steps: bitwise the same factor.  nfd / nfb: step K's multipliers (computed by the caller / the previous step).
template <int K>
__device__ __forceinline__ void panel3_steps(double (&dr)[16], double (&br)[16], int r, int q, int C, bool& ok,
                                             double& rd, double nfd, double nfb) {
  if constexpr (K < 16) {
    if constexpr (K + 1 < 16) {
      fmac_bc<K>(br[K + 1], dr[K + 1], nfb);
      fmac_bc_self<K>(dr[K + 1], nfd);
      const double Dn = bcast16_dep<K + 1>(dr[K + 1]);
      const double rdn = Dn > 0.0 ? recip_d1(Dn) : 0.0;
      const double nfdn = -(dr[K + 1] * rdn), nfbn = -(br[K + 1] * rdn);
      panel2_cols<K, K + 2>(dr, br, nfd, nfb);
      ok = ok & ((Dn > 0.0) | (16 * q + K + 1 >= C));
      rd = (r == K + 1) ? rdn : rd;
      panel3_steps<K + 1>(dr, br, r, q, C, ok, rd, nfdn, nfbn);
    }
  }
}

// the same after 2 wait states (its DPP source was written by the previous VALU instruction)
template <int L>
__device__ __forceinline__ void fmac_bc_self_dep(double& x, double f) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "+v"(x) : "v"(f), "i"(L));
}

// columns J .. 15 of a 2 x 2 pivot step (panel4_steps): per column the below row from the ORIGINAL pivot rows K, K + 1
// (DPP reads before the diagonal rows change), then the diagonal row's step-K part; its step-(K + 1) part is issued
// after the next column's below-row updates, so that its DPP read of the register the step-K part just wrote has its
// two wait states without an s_nop (the pivot lanes' own values move by rounding only: their multipliers are 1 / 0 up
// to rounding, and they are never read again as pivot rows)
template <int K, int J>
__device__ __forceinline__ void panel4_cols(double (&dr)[16], double (&br)[16], double nd1, double nd2, double nb1,
                                            double nb2) {
  if constexpr (J < 16) {
    fmac_bc<K>(br[J], dr[J], nb1);
    fmac_bc<K + 1>(br[J], dr[J], nb2);
    if constexpr (J > K + 2) fmac_bc_self<K + 1>(dr[J - 1], nd2);
    fmac_bc_self<K>(dr[J], nd1);
    if constexpr (J == 15) fmac_bc_self_dep<K + 1>(dr[15], nd2);
    panel4_cols<K, J + 1>(dr, br, nd1, nd2, nb1, nb2);
  }
}

// (KB_PANEL_2X2, not the default: the factor wave is issue-bound, ~7 cycles per f64 FMA of one wave, on the 240 column
// FMAs per lane of a panel (2 rows x 120), and the block form's three reciprocal chains and multiplier selects add ~40 VALU per pivot
// pair: 16 pivots 1.0 -> 1.5 us.)  The panel factorisation two pivots at a time: pivots K, K + 1 eliminated together
// through the 2 x 2 block
// [[a, b], [b, c]] (rows K, K + 1 from lanes K, K + 1 by DPP): one reciprocal chain per two pivots (1/a, 1/det and 1/c
// are independent), so the pivot chain of a panel is 8 steps instead of 16.  A lane's multipliers are its two entries
// times the block inverse, [f1 f2] = [x_K x_K+1] B^-1, and column K + 1 takes the step-K part only, so the factor is
// the sequential one's (the W = L D form, D on the diagonal, 1/D in rd) up to rounding; when a pivot fails the
// multipliers follow the sequential semantics (a <= 0: step K skipped, c alone; det <= 0: step K + 1 skipped).
template <int K>
__device__ __forceinline__ void panel4_steps(double (&dr)[16], double (&br)[16], int r, int q, int C, bool& ok,
                                             double& rd) {
  if constexpr (K < 16) {
    const double a = bcast16_dep<K>(dr[K]);
    const double b = bcast16_dep<K>(dr[K + 1]);
    const double c = bcast16_dep<K + 1>(dr[K + 1]);
    const double det = fma(a, c, -(b * b));
    const bool pa = a > 0.0, pd = pa && det > 0.0, pc = c > 0.0;
    const double rda = pa ? recip_d1(a) : 0.0;
    const double rdt = pd ? recip_d1(det) : 0.0;
    const double rc = pc ? recip_d1(c) : 0.0;
    // B^-1 with the sequential semantics of failed pivots
    const double i11 = pd ? c * rdt : rda, i12 = pd ? -(b * rdt) : 0.0, i22 = pd ? a * rdt : (pa ? 0.0 : rc);
    const double xd0 = dr[K], xd1 = dr[K + 1], xb0 = br[K], xb1 = br[K + 1];
    const double nd1 = -fma(xd0, i11, xd1 * i12), nd2 = -fma(xd0, i12, xd1 * i22);
    const double nb1 = -fma(xb0, i11, xb1 * i12), nb2 = -fma(xb0, i12, xb1 * i22);
    // column K + 1: the step-K update only (W form: W[j][K + 1] = S[j][K + 1] - S[j][K] b / a, D_{K+1} on lane K + 1)
    br[K + 1] = fma(-(xb0 * rda), b, xb1);
    dr[K + 1] = fma(-(xd0 * rda), b, xd1);
    panel4_cols<K, K + 2>(dr, br, nd1, nd2, nb1, nb2);
    ok = ok & (pa | (16 * q + K >= C)) & ((pa ? pd : pc) | (16 * q + K + 1 >= C));  // bitwise: no branch per pivot
    rd = (r == K) ? rda : ((r == K + 1) ? (pa ? a * rdt : rc) : rd);
    panel4_steps<K + 2>(dr, br, r, q, C, ok, rd);
  }
}

// panel q by factor wave fw: lane (t = lane >> 4, r = lane & 15) holds row r of the diagonal tile (every 16-lane row
// the same copy) and row r of tile q + 1 + 4 fw + t.  The tiles of column q are complete (every earlier panel applied).
// The below rows' W go back in place; the factored diagonal tile (W strictly below, D on the diagonal) to Dfac and 1/D
// to rD (wave 0, lanes 0..15).  Returns false on a non-positive pivot of a real row (< C); the b row's pivot and the
// identity padding are not tested.
__device__ __forceinline__ bool panel_factor2(const KbDev& d, double* S, double* rD, double* Dfac, int q, int nb, int C,
                                              int fw) {
  const int lane = threadIdx.x & 63, r = lane & 15, t = lane >> 4;
  const int ti = q + 1 + 4 * fw + t;
  const bool live = ti < nb;
  const double* dbase = S + tile_base(q, q) + r * kTS;
  double* bbase = S + tile_base(live ? ti : q, q) + r * kTS;
  double dr[16], br[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    dr[c] = dbase[c];
    br[c] = bbase[c];
  }
  bool ok = true;
  double rd = 1.0;
  if (q == 2 && fw == 0) KB_TS(d, 41);
#ifdef KB_PANEL_NOLOOK
  panel2_steps<0>(dr, br, r, q, C, ok, rd);
#elif defined(KB_PANEL_2X2)  // measured slower (configs[3] pass 0.1237 -> 0.1300 ms): see DESIGN.md 9
  panel4_steps<0>(dr, br, r, q, C, ok, rd);
#else
  {
    const double D0 = bcast16_dep<0>(dr[0]);
    const double rd0 = D0 > 0.0 ? recip_d1(D0) : 0.0;
    ok = ok & ((D0 > 0.0) | (16 * q >= C));
    rd = (r == 0) ? rd0 : rd;
    panel3_steps<0>(dr, br, r, q, C, ok, rd, -(dr[0] * rd0), -(br[0] * rd0));
  }
#endif
#ifdef KB_STAMPS
#pragma unroll
  for (int c = 0; c < 16; ++c) KB_KEEP(br[c]);
  KB_KEEP(rd);
#endif
  if (q == 2 && fw == 0) KB_TS(d, 42);
  if (live) {
#pragma unroll
    for (int c = 0; c < 16; ++c) bbase[c] = br[c];
  }
  if (t == 0 && fw == 0) {
    double* dd = Dfac + q * kTileSz + r * kTS;
#pragma unroll
    for (int c = 0; c < 16; ++c) dd[c] = dr[c];
    rD[16 * q + r] = rd;
  }
  return ok;
}

// panel q by factor wave fw (rows in registers, one per lane: lanes 0..15 the diagonal tile, lanes 16..63 the rows of
// tiles q+1+3fw .. q+3+3fw).  The tiles of column q are complete (every earlier panel applied).  W rows go back in
// place, the factored diagonal tile (W strictly below, D on the diagonal) to Dfac (wave 0), 1/D to rD.  Returns false
// on a non-positive pivot of a real row (< C); the b row's pivot and the identity padding are not tested.
__device__ __forceinline__ bool panel_factor(const KbDev& d, double* S, double* rD, double* Dfac, int q, int nb, int C,
                                             int fw) {
  const int lane = threadIdx.x & 63, r = lane & 15, t = lane >> 4;
  const int ti_raw = q + 3 * fw + t;
  const bool live = t == 0 || ti_raw < nb;
  // the lane's row (diagonal tiles are whole, so every lane reads 16 consecutive entries)
  double* base = S + tile_base(t == 0 ? q : (live ? ti_raw : q), q) + r * kTS;
  double row[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) row[c] = base[c];
  bool ok = true;
  double rd = 1.0;
#ifdef KB_STAMPS
#pragma unroll
  for (int c = 0; c < 16; ++c) KB_KEEP(row[c]);
#endif
  if (q == 2 && fw == 0) KB_TS(d, 41);
  panel_steps<0>(row, lane, q, C, ok, rd);  // (row K through LDS instead of readlanes: 16 steps 1.36 -> 2.72 us)
#ifdef KB_STAMPS
#pragma unroll
  for (int c = 0; c < 16; ++c) KB_KEEP(row[c]);
  KB_KEEP(rd);
#endif
  if (q == 2 && fw == 0) KB_TS(d, 42);
  if (t > 0 && live) {
#pragma unroll
    for (int c = 0; c < 16; ++c) base[c] = row[c];
  } else if (t == 0 && fw == 0) {
    double* dd = Dfac + q * kTileSz + r * kTS;
#pragma unroll
    for (int c = 0; c < 16; ++c) dd[c] = row[c];
    rD[16 * q + r] = rd;
  }
  return ok;
}

// X = Ltilde_tt^-1 of factored diagonal tile t (unit lower, Ltilde = W D^-1) into Xinv[t] (row-major, stride kTS), by
// one wave: lane (g, r) holds X[r][4g .. 4g+3]; step m subtracts L[r][m] X[m][:] from the rows r > m, X[m] broadcast
// within each 16-lane group by DPP (off the factorisation's critical path: the backsolve's tile mat-vecs use it)
__device__ __forceinline__ void tile_unit_inverse(const double* Dfac, const double* rD, double* Xinv, int t) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const double* Lr = Dfac + t * kTileSz + r * kTS;
  double L[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) L[m] = (m < r) ? Lr[m] * rD[16 * t + m] : 0.0;
  double X[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) X[j] = (4 * g + j == r) ? 1.0 : 0.0;
#pragma unroll
  for (int m = 0; m < 15; ++m) {
#pragma unroll
    for (int j = 0; j < 4; ++j) X[j] = fma(-L[m], bcast16(X[j], m), X[j]);
  }
  double* xo = Xinv + t * kTileSz + r * kTS + 4 * g;
#pragma unroll
  for (int j = 0; j < 4; ++j) xo[j] = X[j];
}

// tile_unit_inverse with the broadcasts fused into the FMAs (DPP row_newbcast source operand): 60 dependent-free FMAs
// per lane in 15 steps of 4 independent columns
template <int M>
__device__ __forceinline__ void tui_steps(double (&X)[4], const double (&nL)[16]) {
  if constexpr (M < 15) {
    if constexpr (M == 0) fmac_bc_dep<M>(X[0], X[0], nL[M]);  // X was just initialised by VALU moves
    else fmac_bc<M>(X[0], X[0], nL[M]);
    fmac_bc<M>(X[1], X[1], nL[M]);
    fmac_bc<M>(X[2], X[2], nL[M]);
    fmac_bc<M>(X[3], X[3], nL[M]);
    tui_steps<M + 1>(X, nL);
  }
}
__device__ __forceinline__ void tile_unit_inverse2(const double* Dfac, const double* rD, double* Xinv, int t) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const double* Lr = Dfac + t * kTileSz + r * kTS;
  double nL[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) nL[m] = (m < r) ? -(Lr[m] * rD[16 * t + m]) : 0.0;
  double X[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) X[j] = (4 * g + j == r) ? 1.0 : 0.0;
  tui_steps<0>(X, nL);
  double* xo = Xinv + t * kTileSz + r * kTS + 4 * g;
#pragma unroll
  for (int j = 0; j < 4; ++j) xo[j] = X[j];
}

// the factorisation (every thread of the 8-wave block calls it); two phases per panel q:
//   A (q > 0): column q of the trailing matrix gets panel q-1 (tiles (q + w, q), one per wave w, on MFMA);
//   B: factor waves 0 (and 1 while panel q has more than three tiles below it) factor panel q; update waves 2, 3, 6, 7
//      apply panel q-1 to the remaining trailing tiles (i, j), j > q (waves 4 and 5 share the factor waves' SIMDs and
//      stay idle so that the MFMA tiles do not slow the pivot chain); wave 7 then inverts the previous panel's factored
//      diagonal tile (Xinv, for the backsolve's mat-vecs).
// okl is cleared on a non-positive real pivot.
__device__ __forceinline__ void ldl_panels(const KbDev& d, double* S, double* rD, double* Dfac, double* Xinv, int C, int nb,
                                           int* okl) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ow = wave == 2 ? 0 : wave == 3 ? 1 : wave == 6 ? 2 : wave == 7 ? 3 : -1;
#pragma unroll 1
  for (int q = 0; q < nb; ++q) {
    if (q > 0) {
      const int i = q + wave;
      if (i < nb) {
        const v4d acc = tile_prod(S + tile_base(i, q - 1), S + tile_base(q, q - 1), rD + 16 * (q - 1), lane);
        tile_sub(S + tile_base(i, q), S + tile_base(i, q), acc, lane);
      }
      __syncthreads();
    }
#ifdef KB_PANEL_READLANE
    const int nf = (nb - 1 - q) > 3 ? 2 : 1;  // the readlane panel: 3 tiles below per factor wave
#else
    const int nf = (nb - 1 - q) > 4 ? 2 : 1;  // the DPP panel: 4 tiles below per factor wave
#endif
    if (wave < nf) {
      if (wave == 0) KB_TS(d, 20 + 2 * q);
#ifdef KB_PANEL_READLANE
      const bool ok = panel_factor(d, S, rD, Dfac, q, nb, C, wave);
#else
      const bool ok = panel_factor2(d, S, rD, Dfac, q, nb, C, wave);
#endif
      if (wave == 0) {
        if (!ok && lane == 0) *okl = 0;
        KB_WAVE_SYNC();
        KB_TS(d, 21 + 2 * q);
      }
    } else if (ow >= 0 && q > 0) {
      // panel q-1 on tiles (q+1+ii, q+1+jj), 0 <= jj <= ii < m
      const int m = nb - 1 - q, ntiles = m * (m + 1) / 2;
      const double* rdq = rD + 16 * (q - 1);
      // two tiles at a time: all their operands in one round of LDS loads, then 8 MFMAs in two chains
      // (four tiles per round, one round for the 15 tiles of the first trailing update at C = 106, measured slower:
      // panel 1 2.52 -> 2.76 us, tools/micro/camera_solve)
#pragma unroll 1
      for (int qq = ow; qq < ntiles; qq += 8) {
        const int qb = min(qq + 4, ntiles - 1);
        const int ia = tri_row(qq), ja = qq - ia * (ia + 1) / 2, ib = tri_row(qb), jb = qb - ib * (ib + 1) / 2;
        const double* Wia = S + tile_base(q + 1 + ia, q - 1);
        const double* Wja = S + tile_base(q + 1 + ja, q - 1);
        const double* Wib = S + tile_base(q + 1 + ib, q - 1);
        const double* Wjb = S + tile_base(q + 1 + jb, q - 1);
        const int r16 = lane & 15, kq = lane >> 4;
        double aa[4], ba[4], ab[4], bb[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const int k = 4 * st + kq;
          const double rk = rdq[k];
          aa[st] = Wia[r16 * kTS + k];
          ba[st] = Wja[r16 * kTS + k] * rk;
          ab[st] = Wib[r16 * kTS + k];
          bb[st] = Wjb[r16 * kTS + k] * rk;
        }
        v4d acca = {0.0, 0.0, 0.0, 0.0}, accb = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          acca = __builtin_amdgcn_mfma_f64_16x16x4f64(aa[st], ba[st], acca, 0, 0, 0);
          accb = __builtin_amdgcn_mfma_f64_16x16x4f64(ab[st], bb[st], accb, 0, 0, 0);
        }
        double* Ta = S + tile_base(q + 1 + ia, q + 1 + ja);
        tile_sub(Ta, Ta, acca, lane);
        if (qq + 4 < ntiles) {  // wave-uniform
          double* Tb = S + tile_base(q + 1 + ib, q + 1 + jb);
          tile_sub(Tb, Tb, accb, lane);
        }
      }
    } else if ((wave == 1 || wave == 5) && q >= 2) {
      // the factored diagonal tiles' inverses for the backsolve on SIMD 1, idle once panel q has one factor wave
      // (q >= 2 for C <= 111): tile t at panel t + 2 on wave 1, the last one (t = nb - 2) at the last panel on wave 5;
      // the last tile, holding row C, is solved by its chain
      // (while wave 1 still factors, i.e. nf == 2 in the readlane variant, wave 5 takes tile q - 2)
      const int t = (wave == 1 || nf == 2) ? q - 2 : (q == nb - 1 ? nb - 2 : -1);
      if (t >= 0) tile_unit_inverse2(Dfac, rD, Xinv, t);
    }
    __syncthreads();
    KB_TS(d, 10 + q);
  }
}

// one tile ti of the backsolve (panel_backsolve).  CHAIN: the tile's own triangle by 16 dependent DPP steps (the
// last tile: its rows from C on are masked, and no inverse of it exists); otherwise by the precomputed inverse
// X = Ltilde_tt^-1: x_t[r] = sum_{c >= r} X[c][r] y[c], 16 independent products (two accumulators).  Then the tile's
// final values go to every lane through pub, which subtracts them from the rows of the earlier tiles.
template <bool CHAIN>
__device__ __forceinline__ void bs_tile(const double* S, const double* Dfac, const double* Xinv, int C, int ti,
                                        const int (&row)[2], const double (&rdv)[2], double* pub, double (&x)[2]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const int tg = ti & 3, ts = ti >> 2, i0 = 16 * ti;
  double M[16], Le[2][16];
  const double* pm = (CHAIN ? Dfac : Xinv) + ti * kTileSz + r;  // column r of the factored tile / of its inverse
#pragma unroll
  for (int u = 0; u < 16; ++u) M[u] = pm[u * kTS];
  // rows of the earlier tiles: Ltilde[i0 + u][row] (row < i0; other lanes read a valid tile and discard it)
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const double* pe = S + tile_base(ti, min(row[sl] >> 4, ti)) + (row[sl] & 15);
#pragma unroll
    for (int u = 0; u < 16; ++u) Le[sl][u] = pe[u * kTS];
  }
  double xt = ts ? x[1] : x[0];
  const int lim = C - i0;  // rows of this tile below C (CHAIN only; the other tiles are whole)
  if constexpr (CHAIN) {
    const double rdt = ts ? rdv[1] : rdv[0];
#pragma unroll
    for (int u = 0; u < 16; ++u) M[u] = (r < u && u < lim) ? M[u] * rdt : 0.0;
#pragma unroll
    for (int u = 15; u >= 0; --u) xt = fma(-M[u], bcast16(xt, u), xt);
  } else {
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      a0 = fma(c >= r ? M[c] : 0.0, bcast16(xt, c), a0);
      a1 = fma(c + 1 >= r ? M[c + 1] : 0.0, bcast16(xt, c + 1), a1);
    }
    xt = a0 + a1;
  }
  if (g == tg) {
    if (ts) x[1] = xt;
    else x[0] = xt;
    pub[r] = xt;
  }
  KB_WAVE_SYNC();
  double xp[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) xp[u] = (!CHAIN || u < lim) ? pub[u] : 0.0;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = fma(Le[sl][u], xp[u], acc);
    if (row[sl] < i0) x[sl] -= acc * rdv[sl];
  }
  KB_WAVE_SYNC();  // pub is rewritten by the next tile
}

// x = Ltilde^-T z, z = (row C of the factor) D^-1, by one wave.  Lane l = 16 g + r holds the rows 16 (g + 4 s) + r,
// s = 0, 1: tile t lives in the 16-lane group t & 3, slot t >> 2.  Tiles from the last (bs_tile); the result comes
// back in x[s] = x_{l + 64 s}.
// Once tile pub_tile is done (xb != nullptr), the final x of rows >= 16 pub_tile go to xb[] and *bflag is set: the
// baseline columns, for the wave that updates the baselines and builds the camera chains meanwhile.
__device__ __forceinline__ void bs_publish(int C, int pub_tile, double* xb, volatile int* bflag, const double (&x)[2]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int row = 16 * (g + 4 * sl) + r;
    if (row >= 16 * pub_tile && row < C) xb[row] = x[sl];
  }
  KB_WAVE_SYNC();
  if (lane == 0) *bflag = 1;
}

__device__ __forceinline__ void panel_backsolve(const KbDev& d, const double* S, const double* Dfac, const double* Xinv,
                                                const double* rD, int C, int nb, double* pub, double (&x)[2],
                                                int pub_tile = -1, double* xb = nullptr, volatile int* bflag = nullptr) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  int row[2];
  double rdv[2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    row[sl] = 16 * (g + 4 * sl) + r;
    const int rc = min(row[sl], C - 1);
    // row C's W: in place off the diagonal tile, in Dfac inside it
    const double* zp = (rc >> 4) == (C >> 4) ? Dfac + (C >> 4) * kTileSz + (C & 15) * kTS + (rc & 15) : S + tidx(C, rc);
    const double z = *zp, rd = rD[rc];
    rdv[sl] = rd;
    x[sl] = row[sl] < C ? z * rd : 0.0;
  }
  int ti = (C - 1) >> 4;
  if (ti == nb - 1) {
    bs_tile<true>(S, Dfac, Xinv, C, ti, row, rdv, pub, x);  // the tile holding row C
    if (xb && ti == pub_tile) bs_publish(C, pub_tile, xb, bflag, x);
    --ti;
  }
#pragma unroll 1
  for (; ti >= 0; --ti) {
    bs_tile<false>(S, Dfac, Xinv, C, ti, row, rdv, pub, x);
    if (xb && ti == pub_tile) bs_publish(C, pub_tile, xb, bflag, x);
  }
}

// ---- the backsolve with DPP-fused broadcasts (panel_backsolve2): the tile's mat-vec and its dependent chain take their
// broadcasts through DPP fused into the FMAs, and the tile's values reach the other 16-lane groups through one LDS slot
// without a wave-wide wait (one wave's LDS accesses complete in order).
struct BsOps {
  double M[16];       // column r of X_ti = Ltilde_tt^-1 (CHAIN: of the factored tile), masked to the entries it uses
  double Le[2][16];   // Ltilde[16 ti + u][row[sl]] for the lane's rows (slots 0, 1)
};

template <bool CHAIN>
__device__ __forceinline__ void bs2_load(const double* S, const double* Dfac, const double* Xinv, int C, int ti,
                                         const int (&row)[2], const double (&rdv)[2], BsOps& o) {
  const int lane = threadIdx.x & 63, r = lane & 15, ts = ti >> 2;
  const double* pm = (CHAIN ? Dfac : Xinv) + ti * kTileSz + r;
#pragma unroll
  for (int u = 0; u < 16; ++u) o.M[u] = pm[u * kTS];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const double* pe = S + tile_base(ti, min(row[sl] >> 4, ti)) + (row[sl] & 15);
#pragma unroll
    for (int u = 0; u < 16; ++u) o.Le[sl][u] = pe[u * kTS];
  }
  (void)C;
  (void)rdv;
  (void)ts;
}

template <bool CHAIN>
__device__ __forceinline__ void bs2_solve(const BsOps& o, int C, int ti, const int (&row)[2], const double (&rdv)[2],
                                          double* pub, double (&x)[2]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  const int tg = ti & 3, ts = ti >> 2, i0 = 16 * ti;
  double xt = ts ? x[1] : x[0];
  const int lim = C - i0;  // rows of this tile below C (CHAIN only; the other tiles are whole)
  if constexpr (CHAIN) {
    const double rdt = ts ? rdv[1] : rdv[0];
    double M[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) M[u] = (r < u && u < lim) ? -(o.M[u] * rdt) : 0.0;
    // x[r] -= sum_{u > r} L[u][r] x[u], u from the last: 16 dependent steps, x[u] read from lane u by DPP
#define KB_BS2_STEP(U) fmac_bc_dep<U>(xt, xt, M[U]);
    KB_BS2_STEP(15) KB_BS2_STEP(14) KB_BS2_STEP(13) KB_BS2_STEP(12) KB_BS2_STEP(11) KB_BS2_STEP(10) KB_BS2_STEP(9)
    KB_BS2_STEP(8) KB_BS2_STEP(7) KB_BS2_STEP(6) KB_BS2_STEP(5) KB_BS2_STEP(4) KB_BS2_STEP(3) KB_BS2_STEP(2)
    KB_BS2_STEP(1) KB_BS2_STEP(0)
#undef KB_BS2_STEP
  } else {
    // x_t[r] = sum_{c >= r} X[c][r] y[c]: 16 independent products (two accumulators), y[c] from lane c by DPP
    double a0 = 0.0, a1 = 0.0;
    double M[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) M[u] = (u >= r) ? o.M[u] : 0.0;
    // the first DPP read of xt waits inside its statement (xt was just selected by a VALU instruction)
    fmac_bc_dep<0>(a0, xt, M[0]);
    fmac_bc<1>(a1, xt, M[1]);
#define KB_BS2_MV(U) fmac_bc<U>(a0, xt, M[U]); fmac_bc<U + 1>(a1, xt, M[U + 1]);
    KB_BS2_MV(2) KB_BS2_MV(4) KB_BS2_MV(6) KB_BS2_MV(8) KB_BS2_MV(10) KB_BS2_MV(12) KB_BS2_MV(14)
#undef KB_BS2_MV
    xt = a0 + a1;
  }
  if (g == tg) {
    if (ts) x[1] = xt;
    else x[0] = xt;
    pub[r] = xt;
  }
  asm volatile("" ::: "memory");  // compiler order only: the wave's LDS write completes before its reads below
  double xp[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) xp[u] = (!CHAIN || u < lim) ? pub[u] : 0.0;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int u = 0; u < 16; u += 2) {
      acc0 = fma(o.Le[sl][u], xp[u], acc0);
      acc1 = fma(o.Le[sl][u + 1], xp[u + 1], acc1);
    }
    if (row[sl] < i0) x[sl] -= (acc0 + acc1) * rdv[sl];
  }
  asm volatile("" ::: "memory");  // pub is rewritten by the next tile after these reads
}

__device__ __forceinline__ void panel_backsolve2(const KbDev& d, const double* S, const double* Dfac, const double* Xinv,
                                                 const double* rD, int C, int nb, double* pub, double (&x)[2],
                                                 int pub_tile = -1, double* xb = nullptr, volatile int* bflag = nullptr) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  int row[2];
  double rdv[2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    row[sl] = 16 * (g + 4 * sl) + r;
    const int rc = min(row[sl], C - 1);
    const double* zp = (rc >> 4) == (C >> 4) ? Dfac + (C >> 4) * kTileSz + (C & 15) * kTS + (rc & 15) : S + tidx(C, rc);
    const double z = *zp, rd = rD[rc];
    rdv[sl] = rd;
    x[sl] = row[sl] < C ? z * rd : 0.0;
  }
  // one tile's operands at a time (a ping-pong prefetch of the next tile's 48 doubles spilled the kernel): they do not
  // depend on x, so their LDS loads go out ahead of the tile's dependent chain anyway
  int ti = (C - 1) >> 4;
  BsOps A;
  if (ti == nb - 1) {  // the tile holding row C: no inverse, solved by its dependent chain
    bs2_load<true>(S, Dfac, Xinv, C, ti, row, rdv, A);
    bs2_solve<true>(A, C, ti, row, rdv, pub, x);
    if (xb && ti == pub_tile) bs_publish(C, pub_tile, xb, bflag, x);
    --ti;
  }
#pragma unroll 1
  for (; ti >= 0; --ti) {
    bs2_load<false>(S, Dfac, Xinv, C, ti, row, rdv, A);
    bs2_solve<false>(A, C, ti, row, rdv, pub, x);
    if (xb && ti == pub_tile) bs_publish(C, pub_tile, xb, bflag, x);
  }
}

// ---- the replicated backsolve (panel_backsolve3, measured and not kept: KB_BACKSOLVE3): every 16-lane row of the
// wave runs the whole
// backward solve, lane (g, r) holding y_t[r] (row 16 t + r) of every tile t.  Tile t's values then reach the rows of
// the earlier tiles by DPP row_newbcast inside the lane's own 16-lane row: no LDS publication and no cross-row move.
// The solve is a fixed sequence of ops, each 16 DPP-fused FMAs over one column of a tile: op (T, T) forms x_T (the
// mat-vec X_T^T y_T, or the last tile's dependent chain), ops (T, s), s = T-1 .. 0, update y_s by x_T.  Each op's 16
// operands are loaded from LDS before the previous op's FMAs issue (inline asm is a scheduling boundary, so the
// prefetch is written out), and masks are multiplications so that no load becomes conditional.  On one CU
// (tools/micro/camera_solve) it takes 4.7 us with a warm instruction cache and 8.4 us cold (its ~6 KB of straight-line
// code runs once per launch), against 3.4 us for panel_backsolve2's tile loop either way.
struct Bs3 {
  const KbDev* d;  // diagnostic stamps only
  const double* S;
  const double* Dfac;
  const double* Xinv;
  int C, nb, r;
};

// operand column of op (T, SS): column r of X_T (the unit-lower tile inverse, exact zeros above its diagonal) or, for
// the last tile (its chain), of the factored diagonal tile; of tile (T, SS) for an update
template <int T, int SS>
__device__ __forceinline__ void bs3_load(const Bs3& b, double (&w)[16]) {
  const double* pe = (SS == T ? ((T == b.nb - 1) ? b.Dfac : b.Xinv) + T * kTileSz : b.S + tile_base(T, SS)) + b.r;
#pragma unroll
  for (int u = 0; u < 16; ++u) w[u] = pe[u * kTS];
}

template <int T, int SS, int P>
__device__ __forceinline__ void bs3_op(const Bs3& b, double (&y)[8], const double (&rdv)[8], double& xt,
                                       double (&w0)[16], double (&w1)[16], int pub_tile, double* xb,
                                       volatile int* bflag) {
  if constexpr (T >= 0) {
    double(&w)[16] = P ? w1 : w0;   // this op's operands (loaded by the previous op)
    double(&wn)[16] = P ? w0 : w1;  // the next op's
    constexpr int NT = SS > 0 ? T : T - 1, NS = SS > 0 ? SS - 1 : T - 1;
    if constexpr (NT >= 0) bs3_load<NT, NS>(b, wn);
    if constexpr (SS == T) {
      const int r = b.r, lim = b.C - 16 * T;
      KB_TS(*b.d, 240 + T);
      xt = y[T];
      if (T == b.nb - 1) {  // wave-uniform: the tile holding row C, solved by its dependent chain (rows >= C: x = 0)
        double M[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) M[u] = -(w[u] * rdv[T]) * ((r < u && u < lim) ? 1.0 : 0.0);
        // x[r] -= sum_{u > r} L[u][r] x[u], u from the last: 16 dependent steps, x[u] read from lane u by DPP
#define KB_BS3_STEP(U) fmac_bc_dep<U>(xt, xt, M[U]);
        KB_BS3_STEP(15) KB_BS3_STEP(14) KB_BS3_STEP(13) KB_BS3_STEP(12) KB_BS3_STEP(11) KB_BS3_STEP(10)
        KB_BS3_STEP(9) KB_BS3_STEP(8) KB_BS3_STEP(7) KB_BS3_STEP(6) KB_BS3_STEP(5) KB_BS3_STEP(4) KB_BS3_STEP(3)
        KB_BS3_STEP(2) KB_BS3_STEP(1) KB_BS3_STEP(0)
#undef KB_BS3_STEP
      } else {
        // x_t[r] = sum_{c >= r} X[c][r] y[c] (X lower: the c < r terms are exact zeros), y[c] from lane c by DPP
        double a0 = 0.0, a1 = 0.0;
        fmac_bc_dep<0>(a0, xt, w[0]);
        fmac_bc<1>(a1, xt, w[1]);
#define KB_BS3_MV(U) fmac_bc<U>(a0, xt, w[U]); fmac_bc<U + 1>(a1, xt, w[U + 1]);
        KB_BS3_MV(2) KB_BS3_MV(4) KB_BS3_MV(6) KB_BS3_MV(8) KB_BS3_MV(10) KB_BS3_MV(12) KB_BS3_MV(14)
#undef KB_BS3_MV
        xt = a0 + a1;
      }
      y[T] = xt;
      if (xb && T == pub_tile) {  // the baseline rows are final: publish them for the baseline / chain wave
        if ((threadIdx.x & 63) < 16) {
#pragma unroll
          for (int t = T; t < 8; ++t)
            if (t < b.nb && 16 * t + r < b.C) xb[16 * t + r] = y[t];
        }
        KB_WAVE_SYNC();
        if ((threadIdx.x & 63) == 0) *bflag = 1;
      }
    } else {
      // y_s[r] -= (1/D of row 16 s + r) sum_u W[16 T + u][16 s + r] x_T[u], x_T[u] from lane u by DPP (rows >= C of the
      // last tile carry x = 0)
      double a0 = 0.0, a1 = 0.0;
      if constexpr (SS == T - 1) fmac_bc_dep<0>(a0, xt, w[0]);
      else fmac_bc<0>(a0, xt, w[0]);
      fmac_bc<1>(a1, xt, w[1]);
#define KB_BS3_MV(U) fmac_bc<U>(a0, xt, w[U]); fmac_bc<U + 1>(a1, xt, w[U + 1]);
      KB_BS3_MV(2) KB_BS3_MV(4) KB_BS3_MV(6) KB_BS3_MV(8) KB_BS3_MV(10) KB_BS3_MV(12) KB_BS3_MV(14)
#undef KB_BS3_MV
      y[SS] -= (a0 + a1) * rdv[SS];
    }
    bs3_op<NT, NS, 1 - P>(b, y, rdv, xt, w0, w1, pub_tile, xb, bflag);
  }
}

// entry at the last tile T = nb - 1 (nb in 5..7 for 64 < C <= 111)
template <int T>
__device__ __forceinline__ void bs3_run(const Bs3& b, double (&y)[8], const double (&rdv)[8], int pub_tile, double* xb,
                                        volatile int* bflag) {
  double w0[16], w1[16], xt = 0.0;
  bs3_load<T, T>(b, w0);
  bs3_op<T, T, 0>(b, y, rdv, xt, w0, w1, pub_tile, xb, bflag);
}

// x = Ltilde^-T z as panel_backsolve (same operands, same result layout: x[s] = x_{l + 64 s}), nb <= 7
__device__ __forceinline__ void panel_backsolve3(const KbDev& d, const double* S, const double* Dfac, const double* Xinv,
                                                 const double* rD, int C, int nb, double (&x)[2], int pub_tile = -1,
                                                 double* xb = nullptr, volatile int* bflag = nullptr) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  Bs3 b{&d, S, Dfac, Xinv, C, nb, r};
  double y[8], rdv[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int row = 16 * t + r, rc = min(row, C - 1);
    // row C's W: in place off the diagonal tile, in Dfac inside it
    const double* zp = (rc >> 4) == (C >> 4) ? Dfac + (C >> 4) * kTileSz + (C & 15) * kTS + (rc & 15) : S + tidx(C, rc);
    const double z = *zp, rd = rD[rc];
    rdv[t] = rd;
    y[t] = (t < nb && row < C) ? z * rd : 0.0;
  }
  if (nb == 7) bs3_run<6>(b, y, rdv, pub_tile, xb, bflag);
  else if (nb == 6) bs3_run<5>(b, y, rdv, pub_tile, xb, bflag);
  else bs3_run<4>(b, y, rdv, pub_tile, xb, bflag);
  double x0 = y[0], x1 = y[4];
#pragma unroll
  for (int t = 1; t < 4; ++t) {
    x0 = g == t ? y[t] : x0;
    x1 = g == t ? y[t + 4] : x1;
  }
  x[0] = x0;
  x[1] = x1;
}

// ---------------------------------------------------------------------------------------------
// k_colimg (C > 64): finishes the column sums as k_colfin does (out[e] = sum_r rows[r][e] over the nrows rows: the 8
// stage-1 rows, or 1 all-reduced row when sharded; fixed order; max for the max|dx_f| columns) and writes k_solve's
// LDS image of the complete camera system from the same rows:
//   [S lower 16 x 16 tiles, stride kTS (diagonal tiles whole):
//      H_cc + lambda^2 I (or the per-call conditioner) - sum Y^T Y, row C = b = g_c - sum Y^T z, rows C+1.. the identity |
//    n16 + 2 slots: g_c (the gradient, for the step statistics), slot C: the non-PD frame-block count].
// H_cc and g_c are the expansion of the per-camera sums through the chains K of the build state (cam_entry_l /
// cam_grad_l: H_{I_i,I_i} = Hs_i[II], H_{B_j,I_i} = K_{i,j}^T Hs_i[dI], H_{B_j,B_k} = sum_{i > max(j,k)} K_{i,j}^T
// Hs_i[dd] K_{i,k}).  Every block that writes image entries first stages the finished per-camera sums Hs, the chains K
// and T = Hs[dd] K in LDS (the same fixed-order sums for every block), so the expansion runs wide here instead of in
// the one-block camera solve.  One thread per output entry; the block holding the first image entry also writes
// cost_build, the threads of the gradient slots gc and rhs.
// ---------------------------------------------------------------------------------------------
constexpr int kColimgThreads = 1024;  // few, wide blocks: each image block stages the camera sums once
__global__ void __launch_bounds__(kColimgThreads) k_colimg(KbDev d, const double* rows, double* out, int gate, int nrows) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const KbCtrl* c = d.ctrl;
  const int done = c->done, cur = c->cur, have = c->have_dx;
  const double lamc = c->lambda;
  if (gate && done) return;
  const int tid = threadIdx.x, q = blockIdx.x * blockDim.x + tid, nth = blockDim.x;
  const bool stamp_block = blockIdx.x == d.Wtot / (int)blockDim.x;  // diagnostic timeline: the first image block
  if (stamp_block) KB_TS(d, 50);
  const int N = d.N, C = d.C, Wt = d.W - d.C;
  const int nb = (C + 16) >> 4, ntz = kTileSz * nb * (nb + 1) / 2;  // + the b row (row C)
  const int q0 = blockIdx.x * blockDim.x;
  const bool img_block = q0 + nth > d.Wtot && q0 < d.Wtot + ntz + 16 * nb + 2;  // block-uniform
  // ---- this thread's output: which column sum it needs (src) and what it is
  // kind: 0 none / zero, 1 finished column sum (out), 2 camera entry (i, j), 3 b entry j, 4 identity, 5 g_c k,
  //       6 non-PD count
  int kind = 0, src = -1, ei = 0, ej = 0;
  const int e = q - d.Wtot;
  if (q < d.Wtot) {
    kind = 1;
    src = q;
  } else if (e < ntz) {
    const int t = e / kTileSz, w = e - t * kTileSz, r = w / kTS, cc = w - r * kTS;
    const int it = tri_row(t), jt = t - it * (it + 1) / 2;
    const int i0 = 16 * it + r, j0 = 16 * jt + cc;
    // diagonal tiles are stored whole (both triangles), so that a lane loads its row with constant offsets
    ei = max(i0, j0);
    ej = min(i0, j0);
    if (cc < 16) {
      if (ei < C) {
        kind = 2;
        src = N * 136 + upper_index(ej, ei, C);
      } else if (ei == C && ej < C) {
        kind = 3;
        src = N * 136 + Wt + ej;
      } else if (ei == ej) {
        kind = 4;
      }
    }
  } else if (e < d.img_n) {
    const int k = e - ntz;
    ej = k;
    if (k < C) kind = 5;
    else if (k == C) {
      kind = 6;
      src = N * 136 + Wt + C;
    }
  }
  // ---- round 1: the thread's column-sum rows and (image blocks) every staging load, all in flight together
  double v8[kColsumRows];
  {
    const int sc = src < 0 ? 0 : src;
#pragma unroll
    for (int r = 0; r < kColsumRows; ++r) v8[r] = rows[(size_t)(r < nrows ? r : 0) * d.Wtot + sc];
  }
  double* Hs = sm;              // [N][256] symmetric per-camera sums
  double* K = Hs + N * 256;     // [N][N][36] chains of the build state
  double* T = K + N * N * 36;   // [N][N][36] T_{i,k} = Hs_i[dd] K_{i,k}
  int* ci = (int*)(T + N * N * 36);  // [C] column info
  if (img_block) {
    const bool gfu = gate && d.gn_fused;
    const int bslot = (gfu && have) ? 1 - cur : cur;  // as k_solve: the state the system was built at
    const double* Kc = cam_K(d, bslot);
    // C <= 111 bounds the rig to N <= 10 cameras: at most 2 sums of 8 rows and 4 chain entries per thread
    constexpr int kHsU = 2, kKU = 4;
    const int nHs = N * 136, nK = N * N * 36;
    double kv[kKU], hv[kHsU][kColsumRows];
#pragma unroll
    for (int u = 0; u < kKU; ++u) kv[u] = Kc[min(tid + u * nth, nK - 1)];
#pragma unroll
    for (int u = 0; u < kHsU; ++u)
#pragma unroll
      for (int r = 0; r < kColsumRows; ++r)
        hv[u][r] = rows[(size_t)(r < nrows ? r : 0) * d.Wtot + min(tid + u * nth, nHs - 1)];
    const int civ = d.colinfo[min(tid, C - 1)];
#pragma unroll
    for (int u = 0; u < kKU; ++u)
      if (tid + u * nth < nK) K[tid + u * nth] = kv[u];
#pragma unroll
    for (int u = 0; u < kHsU; ++u) {
      const int eh = tid + u * nth;
      if (eh < nHs) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < kColsumRows; ++r)
          if (r < nrows) v += hv[u][r];
        const int cam = eh / 136;
        int a, b;
        d16_rowcol_fast(eh - 136 * cam, a, b);
        Hs[cam * 256 + a * 16 + b] = v;
        Hs[cam * 256 + b * 16 + a] = v;
      }
    }
    if (tid < C) ci[tid] = civ;
    if (stamp_block) KB_TS(d, 51);
    __syncthreads();
    if (stamp_block) KB_TS(d, 52);
    for (int et = tid; et < nK; et += nth) {
      const int x = et % 36, ik = et / 36, i = ik / N, k = ik - i * N;
      double sacc = 0.0;
      if (k < i) {
        const int a = x / 6, b = x % 6;
#pragma unroll
        for (int m = 0; m < 6; ++m) sacc += Hs[i * 256 + a * 16 + m] * K[(i * N + k) * 36 + m * 6 + b];
      }
      T[et] = sacc;
    }
    __syncthreads();
    if (stamp_block) KB_TS(d, 53);
    if (tid == 0 && blockIdx.x == d.Wtot / nth) {
      double sc = 0.0;
      for (int i = 0; i < N; ++i) sc += Hs[i * 256 + 255];
      d.cost_build[0] = sc;
    }
  }
  if (kind == 0 && e >= d.img_n) return;
  // the finished column sum (fixed order; max for the max|dx_f| columns)
  double cs = 0.0;
  if (src >= 0) {
    const bool mx = src >= d.Wp;
#pragma unroll
    for (int r = 0; r < kColsumRows; ++r)
      if (r < nrows) cs = mx ? fmax(cs, v8[r]) : cs + v8[r];
  }
  if (kind == 1) {
    out[q] = cs;
    return;
  }
  double v = 0.0;
  if (kind == 2) {
    v = cam_entry_l(N, ci, Hs, T, K, ei, ej) - cs;
    if (ei == ej) v += gate ? lamc * lamc : (d.cond2 ? d.cond2[ei] : d.host_lambda * d.host_lambda);
  } else if (kind == 3) {
    v = cam_grad_l(N, ci, Hs, K, ej) - cs;  // b
  } else if (kind == 4) {
    v = 1.0;  // identity padding (and the b row's diagonal)
  } else if (kind == 5) {
    v = cam_grad_l(N, ci, Hs, K, ej);  // g_c
    d.gc[ej] = v;
    d.rhs[ej] = v;
  } else if (kind == 6) {
    v = cs;  // non-PD frame blocks
  }
  d.simg[e] = v;
  if (stamp_block) KB_TS(d, 54);
}

// batched global -> LDS staging of the k_solve inputs: every thread keeps U independent loads in flight
// (a runtime-bounded copy loop would otherwise wait for each load before the next).  Items are laid out as
// [camK N*N*36 | per-camera sums N*256 | Schur sums Wt | Schur rhs C | colinfo C] over one index space.
template <int U, int CM, bool ONE_ROW>
__device__ __forceinline__ void solve_stage(const KbDev& d, int bslot, double* K, double* Hs, double* S, double* bv,
                                            int* ci, int tid, int nth) {
  const int N = d.N, C = d.C, Wt = d.W - C;
  // [camK N*N*36 | per-camera upper sums N*136 | Schur sums Wt + rhs C + non-PD count 1 | colinfo C]
  const int n0 = N * N * 36, n1 = n0 + N * 136, n2 = n1 + Wt, n3 = n2 + C + 1, n4 = n3 + C;
  const double* Kc = cam_K(d, bslot);  // chains of the state the system was built at
  for (int q0 = tid; q0 < n4; q0 += U * nth) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = min(q0 + u * nth, n4 - 1);
      if (q < n0)
        v[u] = Kc[q];
      else if (q < n3)
        v[u] = ONE_ROW ? d.psum[q - n0] : psum_at(d, q - n0);  // camera sums, Schur sums, rhs, count: contiguous
      else
        v[u] = (double)d.colinfo[q - n3];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * nth;
      if (q < n0) {
        K[q] = v[u];
      } else if (q < n1) {
        const int r = q - n0, cam = r / 136;
        int a, b;
        d16_rowcol_fast(r % 136, a, b);
        Hs[cam * 256 + a * 16 + b] = v[u];
        Hs[cam * 256 + b * 16 + a] = v[u];
      } else if (q < n2) {
        const int e = q - n1;  // upper (a,b) row-major == lower (b,a) col-major packed index e
        if constexpr (CM > 0) {
          S[e] = -v[u];
        } else {
          const int a = cidx_col(e, C), b = e - a * (2 * C - a - 1) / 2;
          S[tidx(b, a)] = -v[u];
        }
      } else if (q < n2 + C) {
        bv[q - n2] = -v[u];
      } else if (q < n3) {
        bv[C] = v[u];  // non-PD frame-block count (bv has C + 1 slots)
      } else if (q < n4) {
        ci[q - n3] = (int)v[u];
      }
    }
  }
}



// LDL^T + the three triangular solves of one wave, matrix rows in registers (lane i holds row i of the
// trailing matrix, CM >= C padded with the identity).  Step k broadcasts row k with v_readlane (no LDS), and
// lanes i > k apply S[i][j] -= (S[i][k] / D_k) S[k][j].  Row i freezes at step i, so lane i ends holding
// Ltilde[i][k] D_k (k < i), D_i, and by symmetry of the trailing matrix Ltilde[k][i] D_i (k > i).
template <int CM, int K0, int K1>
__device__ __forceinline__ void ldl_steps(double (&row)[CM], int lane, bool& ok, double& rD) {
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const double Dk = readlane_d(row[k], k);
    ok = ok && (Dk > 0.0);
    const double rdk = recip_d(Dk);
    rD = (lane == k) ? rdk : rD;
    const double f = (lane > k) ? row[k] * rdk : 0.0;
#pragma unroll
    for (int j = k + 1; j < CM; ++j) row[j] -= f * readlane_d(row[j], k);
  }
}

struct LdlOut {
  double x;
  int ok;
};

// One factorisation step set with the column broadcast through LDS instead of v_readlane: at step k every lane j
// publishes its S[j][k] (column k of the trailing matrix, D_k at j = k) and lanes i > k read the column back as
// broadcasts (ds_read_b128 pairs): ~1.5 instructions per updated entry instead of ~3.5.
template <int CM, int K0, int K1>
__device__ __forceinline__ void ldl_steps_lds(double (&row)[CM], int lane, bool& ok, double& rD, double* pub) {
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    if (lane < CM) pub[lane] = row[k];
    KB_WAVE_SYNC();  // the other lanes' column entries: no reuse of an earlier read across this point
    const double Dk = pub[k];
    ok = ok && (Dk > 0.0);
    const double rdk = recip_d(Dk);
    rD = (lane == k) ? rdk : rD;
    const double f = (lane > k) ? row[k] * rdk : 0.0;
#pragma unroll
    for (int j = k + 1; j < CM; ++j) row[j] -= f * pub[j];
  }
}

template <int CM>
__device__ __forceinline__ LdlOut ldl_solve_reg(const KbDev& d, const double* S, const double* bv, int C, int lane,
                                                double* pub) {
  // all CM + 1 loads unconditional (clamped) and materialised together: a select on a loaded value otherwise
  // becomes one exec-masked branch (and one wait) per load
  double row[CM];
  const int li = lane < C ? lane : 0;
  const int cs_i = li * (2 * C - li - 1) / 2;  // start of packed column li
#pragma unroll
  for (int j = 0; j < CM; ++j) {
    const int jc = j < C ? j : 0;
    const int cs_j = jc * (2 * C - jc - 1) / 2;  // wave-uniform
    row[j] = S[(li >= jc) ? cs_j + li : cs_i + jc];  // lower (max, min) of (lane, j); clamped outside C
  }
  double x = bv[li];
#pragma unroll
  for (int j = 0; j < CM; ++j) KB_KEEP(row[j]);
  KB_KEEP(x);
#pragma unroll
  for (int j = 0; j < CM; ++j) {
    const bool in = lane < C && j < C;
    row[j] = in ? row[j] : (lane == j ? 1.0 : 0.0);
  }
  x = lane < C ? x : 0.0;
  bool ok = true;
  double rD = 1.0;
#ifdef KB_STAMPS
  KB_KEEP(x);
#pragma unroll
  for (int j = 0; j < CM; ++j) KB_KEEP(row[j]);
  if (d.dbg_stop == 45) return LdlOut{x, 1};
#endif
  ldl_steps<CM, 0, CM>(row, lane, ok, rD);  // (ldl_steps_lds: same speed at CM = 24, spills at CM >= 32)
#ifdef KB_STAMPS
  KB_KEEP(rD);
#pragma unroll
  for (int j = 0; j < CM; ++j) KB_KEEP(row[j]);
  if (d.dbg_stop == 46) return LdlOut{x, 1};
#endif
  // Ltilde y = b ; z = D^-1 y ; Ltilde^T x = z
#pragma unroll
  for (int k = 0; k < CM; ++k) {
    const double yk = readlane_d(x, k) * readlane_d(rD, k);
    x -= ((lane > k) ? row[k] : 0.0) * yk;
  }
  x *= rD;
#pragma unroll
  for (int k = CM - 1; k > 0; --k) {
    const double wk = readlane_d(x, k);
    x -= ((lane < k) ? row[k] * rD : 0.0) * wk;
  }
  return LdlOut{x, ok ? 1 : 0};
}

// Camera block H_cc from the per-camera local sums, added to the staged S (lower entries), one wave per block
// of H_cc (lanes = the block's entries):  intrinsics_i x intrinsics_i = Hs_i[II];
// intrinsics_i x B_j = Hs_i[Id] K_{i,j} (j < i);  B_j x B_k = sum_{i > max(j,k)} K_{i,j}^T T_{i,k}, T = Hs_i[dd] K
template <int CM>
__device__ __forceinline__ void cam_expand_blocks(double* S, int C, int N, const int (*ctab)[KB_MAX_CAMS], const double* Hs,
                                  const double* T, const double* K, double lam2, int nw, const double* cond2) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nA = N, nB = N * (N - 1) / 2, nC = (N - 1) * N / 2;
  for (int it = wave; it < nA + nB + nC; it += nw) {
    if (it < nA) {
      const int i = it, nin = ctab[0][i], c0 = ctab[1][i];
      for (int e = lane; e < nin * nin; e += 64) {
        const int x = e / nin, y = e % nin;
        if (y <= x)
          S[sidx<CM>(c0 + x, c0 + y, C)] +=
              Hs[i * 256 + (6 + x) * 16 + 6 + y] + ((x == y) ? (cond2 ? cond2[c0 + x] : lam2) : 0.0);
      }
    } else if (it < nA + nB) {
      const int q = it - nA, i = tri_row(q) + 1, j = q - (i - 1) * i / 2;  // j < i
      const int nin = ctab[0][i], x = lane / 6, a = lane % 6;
      if (x < nin) {
        const double* Kk = K + (size_t)(i * N + j) * 36;
        double v = 0.0;
#pragma unroll
        for (int b = 0; b < 6; ++b) v += Hs[i * 256 + (6 + x) * 16 + b] * Kk[b * 6 + a];
        S[sidx<CM>(ctab[2][j] + a, ctab[1][i] + x, C)] += v;  // baseline columns follow all intrinsics
      }
    } else {
      const int q = it - nA - nB, k = tri_row(q), j = q - k * (k + 1) / 2;  // j <= k < N - 1
      const int a = lane / 6, b = lane % 6;
      if (lane < 36 && (j < k || a >= b)) {
        double v = 0.0;
        for (int i = k + 1; i < N; ++i) {
          const double* Kj = K + (size_t)(i * N + j) * 36;
          const double* Tk = T + (size_t)(i * N + k) * 36;
#pragma unroll
          for (int m = 0; m < 6; ++m) v += Kj[m * 6 + a] * Tk[m * 6 + b];
        }
        // entry (B_j a, B_k b) -> lower (B_k b, B_j a) when j < k
        const int r = (j < k) ? ctab[2][k] + b : ctab[2][j] + a, cc = (j < k) ? ctab[2][j] + a : ctab[2][j] + b;
        S[sidx<CM>(r, cc, C)] += v + ((j == k && a == b) ? (cond2 ? cond2[r] : lam2) : 0.0);
      }
    }
  }
}

// KB_SOLVER_PCG_SCHUR: LinearSolverPCG::solve (sparse_block_matrix linear_solver_pcg.hpp:58-130) on the camera
// block's Schur complement S x = b (S = H_cc + lambda^2 I - sum H_fc^T H_ff^-1 H_fc, the frame blocks eliminated
// exactly), M = the inverses of S's diagonal camera DV blocks (d.pcs_cb), by the whole block with S in LDS (sget).
// Four threads per row in the mat-vec (fixed order: j = t (mod 4) partial sums, then a 2-step butterfly); dots by a
// fixed-order block sum.  Wave 0 gets x[s] = x_{lane + 64 s}; returns false on a singular DV block or non-positive
// curvature (the reference has no check).  Every thread of the block must call it.
template <class SGet>
__device__ bool schur_pcg(const KbDev& d, SGet sget, const double* b, int C, int nth, double (&xo)[2]) {
  __shared__ double v_x[128], v_r[128], v_z[128], v_p[128], v_q[128], Minv[128][6], red[16], scal[4];
  __shared__ int blk_ok;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = nth >> 6;
  auto bsum = [&](double v) {  // fixed-order block sum, result uniform
    v = wave_sum_d(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < nw; ++w) s += red[w];
    return s;
  };
  if (tid == 0) blk_ok = 1;
  __syncthreads();
  // preconditioner: one thread per DV block inverts its m x m diagonal block of S in place in its Minv rows (LDS):
  // Gauss-Jordan without pivoting (the block is SPD); no private array, so k_solve needs no scratch
  for (int p = tid; p < C; p += nth) {
    const int s0 = d.pcs_cb[p], m = d.pcs_cb[C + p];
    if (s0 != p) continue;
    double(*A)[6] = Minv + p;  // rows p .. p + m - 1
    for (int r = 0; r < m; ++r)
      for (int c = 0; c < 6; ++c) A[r][c] = c < m ? sget(p + r, p + c) : 0.0;
    bool good = true;
    for (int k = 0; k < m; ++k) {
      const double piv = A[k][k];
      if (!(piv > 0.0)) {
        good = false;
        break;
      }
      const double inv = 1.0 / piv;
      A[k][k] = 1.0;
      for (int c = 0; c < m; ++c) A[k][c] *= inv;
      for (int r = 0; r < m; ++r) {
        if (r == k) continue;
        const double f = A[r][k];
        A[r][k] = 0.0;
        for (int c = 0; c < m; ++c) A[r][c] -= f * A[k][c];
      }
    }
    if (!good) {
      blk_ok = 0;
      for (int r = 0; r < m; ++r)
        for (int c = 0; c < 6; ++c) A[r][c] = 0.0;
    }
  }
  for (int i = tid; i < 128; i += nth) {
    v_x[i] = 0.0;
    v_r[i] = i < C ? b[i] : 0.0;
  }
  __syncthreads();
  auto precond = [&]() {  // z = M^-1 r
    for (int i = tid; i < C; i += nth) {
      const int s0 = d.pcs_cb[i], m = d.pcs_cb[C + i];
      double v = 0.0;
      for (int k = 0; k < m; ++k) v += Minv[i][k] * v_r[s0 + k];
      v_z[i] = v;
    }
  };
  precond();
  __syncthreads();
  for (int i = tid; i < 128; i += nth) v_p[i] = i < C ? v_z[i] : 0.0;
  double dn = bsum(tid < C ? v_r[tid] * v_z[tid] : 0.0);
  double d0 = d.pcs_tol * dn;
  if (d.pcs_abs && d.pcs_prev > 0.0 && d.pcs_prev > d0) d0 = d.pcs_prev;
  bool ok = blk_ok != 0;
  int it = 0;
  for (; ok && it < d.pcs_maxit; ++it) {
    if (dn <= d0) break;
    // q = S p: row i by threads 4i .. 4i + 3
    const int row = tid >> 2, part = tid & 3;
    double acc = 0.0;
    if (row < C)
      for (int j = part; j < C; j += 4) acc += sget(row, j) * v_p[j];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (row < C && part == 0) v_q[row] = acc;
    __syncthreads();
    const double pq = bsum(tid < C ? v_p[tid] * v_q[tid] : 0.0);
    if (!(pq > 0.0) || !isfinite(pq)) {
      ok = false;
      break;
    }
    const double alpha = dn / pq;
    if (tid < C) {
      v_x[tid] += alpha * v_p[tid];
      v_r[tid] -= alpha * v_q[tid];
    }
    __syncthreads();
    precond();
    __syncthreads();
    const double dnew = bsum(tid < C ? v_r[tid] * v_z[tid] : 0.0);
    const double beta = dnew / dn;
    dn = dnew;
    if (tid < C) v_p[tid] = v_z[tid] + beta * v_p[tid];
    __syncthreads();
  }
  if (tid == 0) {
    scal[0] = ok ? 1.0 : 0.0;
    d.pcs_info[0] = it;
    d.pcs_info[1] = 0.5 * dn;
    d.pcs_info[2] = d0;
    d.pcs_info[3] = ok ? 1.0 : 0.0;
  }
  __syncthreads();
  if (wave == 0) {
    xo[0] = lane < C ? v_x[lane] : 0.0;
    xo[1] = lane + 64 < C ? v_x[lane + 64] : 0.0;
  }
  return scal[0] != 0.0;
}

// Camera solve of one pass (one block): S = H_cc + lambda^2 I - sum Y^T Y, b = g_c - sum Y^T z staged in LDS,
// LDL^T + solves (CM > 0: one-wave register LDL^T for C <= CM <= 64; CM == 0: block LDL^T in LDS), camera DV
// update into state[1 - cur] and the camera chains of that candidate state into slot 1 - cur.
// Every thread of the block must call it (barriers inside).
template <int CM>
__device__ void solve_body(const KbDev& d, int gate, int do_update, int nth) {
  KbCtrl* c = d.ctrl;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int N = d.N, C = d.C, W = d.W, tid = threadIdx.x;
  const int Cp = C * (C + 1) / 2;
  const int nb = (C + 16) >> 4, n16 = 16 * nb;  // CM == 0: 16 x 16 tiles, rows 0 .. C (b appended as row C)
  // CM > 0: S column-major packed lower [Cp] | bv [C + 1] (slot C: non-PD frame-block count) | gl [C] | Hs [N][256] |
  //   T, K [N][N][36] | ci [C]
  // CM == 0: the k_colimg image [S lower tiles, complete (b as row C) | gl = g_c (n16 + 2 slots, slot C: non-PD
  //   frame-block count)] | Dfac | Xinv | 1/D
  double* S = sm;
  double* bv = S + (CM > 0 ? Cp : kTileSz * nb * (nb + 1) / 2);
  double* Hs = CM > 0 ? bv + 2 * C + 1 : bv;
  double* gl = CM > 0 ? bv + C + 1 : bv;
  double* T = CM > 0 ? Hs + N * 256 : bv;
  double* K = T + N * N * 36;        // CM > 0: [N][N][36]
  double* Dfac = CM > 0 ? K + N * N * 36 : bv + ((n16 + 2 + 1) & ~1);  // CM == 0: [nb][kTileSz] factored diagonal tiles
  double* Xinv = Dfac + (CM > 0 ? 0 : nb * kTileSz);  // CM == 0: [nb][kTileSz] their unit-lower inverses
  double* rDv = Xinv + (CM > 0 ? 0 : nb * kTileSz);   // CM == 0: [n16] 1/D
  int* ci = (int*)(rDv + (CM > 0 ? 0 : n16));      // [C]
  __shared__ int okl;
  __shared__ double nbase[KB_MAX_CAMS * 7];  // candidate baselines
  __shared__ int ctab[3][KB_MAX_CAMS];       // per camera: #intrinsics | first intrinsic column | baseline column
  __shared__ __attribute__((aligned(16))) double pubcol[CM > 0 ? CM : 16];  // LDL^T column / solve broadcast
  __shared__ int fin[2];  // GN fused: done, cur after the previous pass's end
  __shared__ KbCtrl cls;
  __shared__ double cl_red[4];
  __shared__ ChainLds chl;                     // CM == 0: the candidate chains' pair products (wave 1)
  __shared__ int bflag;                        // CM == 0: baseline x published by the backsolve wave
  __shared__ double xb[CM == 0 ? 128 : 1];     // CM == 0: those x (rows >= 16 pub_tile)
  if (CM == 0 && tid == 0) bflag = 0;
  const double lam = gate ? c->lambda : d.host_lambda;
  const double lam2 = lam * lam;
  int cur = c->cur;
  const bool gfu = gate && d.gn_fused;
  // GN fused: a pending step means the system was built at the candidate state (slot 1 - cur)
  const int bslot = (gfu && c->have_dx) ? 1 - cur : cur;
  double x[2] = {0.0, 0.0};
  // GN fused: the previous pass's end runs in wave kFinWave while the factorisation runs (CM == 0: wave 2, an
  // update wave, idle during the first panel)
  constexpr int kFinWave = CM > 0 ? 1 : 2;
  const bool fwave = (tid >> 6) == kFinWave;
  double dxr = 0.0;  // GN fused: max|dx_f| of the previous step, one column per rank
  const bool xexp = CM == 0 && gfu && d.xexp;  // expanded partials: the image holds the finished sums (k_colsumx)
  if (gfu && fwave && !xexp) {
    const int tid = threadIdx.x & 63;
    const int nr = d.Wtot - d.Wp;
    dxr = psum_max_at(d, d.Wp + min(tid, nr - 1));
    for (int r = tid + 64; r < nr; r += 64) dxr = fmax(dxr, psum_max_at(d, d.Wp + r));
  }
  // the camera DVs of both state slots (the DV update reads slot cur, which the previous pass's end may still flip),
  // loaded with the staging round instead of one dependent round trip after the solves
  __shared__ double camst[2][KB_MAX_CAMS * KB_MAX_INTR + 7 * (KB_MAX_CAMS - 1)];
  const int nst = N * KB_MAX_INTR + 7 * (N - 1);
  double cpv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = min(tid + u * nth, 2 * nst - 1), sl = q >= nst ? 1 : 0, e = q - sl * nst;
    cpv[u] = d.state[(size_t)sl * d.S + (e < N * KB_MAX_INTR ? e : d.off_base + e - N * KB_MAX_INTR)];
  }
  KB_TS(d, 0);
  KB_STAMP(d, 0);
  // phase A: stage K, column info, per-camera sums and the Schur sums in LDS (one row: psum)
  if constexpr (CM == 0) {
    // the k_colimg image (the complete system): one contiguous 16-byte copy, 12 loads in flight per thread (one round
    // trip for an 8-camera rig); the build's cost (k_colimg) in the same round
    const int n2 = d.img_n >> 1;
    const double2* gi = reinterpret_cast<const double2*>(d.simg);
    double2* li = reinterpret_cast<double2*>(S);
    const double cb0 = d.cost_build[0];
    constexpr int U = 12;
#pragma unroll 1
    for (int q0 = tid; q0 < n2; q0 += U * nth) {
      double2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = gi[min(q0 + u * nth, n2 - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * nth;
        if (q < n2) li[q] = v[u];
      }
    }
    if (tid == 0) cl_red[0] = cb0;
  } else {
    solve_stage<4, CM, false>(d, bslot, K, Hs, S, bv, ci, tid, nth);
  }
  if (tid < 3 * N) ctab[tid / N][tid % N] = tid < N ? cam_arg(d.nintr, tid) : (tid < 2 * N ? cam_arg(d.col_intr, tid - N) : cam_arg(d.col_base, tid - 2 * N));
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = tid + u * nth;
    if (q < 2 * nst) (&camst[0][0])[q >= nst ? (q - nst) + (KB_MAX_CAMS * KB_MAX_INTR + 7 * (KB_MAX_CAMS - 1)) : q] = cpv[u];
  }
  __syncthreads();
  if (xexp) {
    // k_colsumx wrote the summed S - lambda^2 I, b and aux slots; lambda^2 and the identity padding (rows C ..) are
    // added here, since the image may be an all-reduce over ranks; the cost and the per-rank max|dx_f| are aux slots
    for (int i = tid; i < n16; i += nth) {
      const int q = tidx(i, i);
      S[q] = i < C ? S[q] + lam2 : 1.0;
    }
    if (tid == 0) cl_red[0] = bv[n16];
    if (fwave) {
      const int l = tid & 63, nr = d.nranks;
      dxr = bv[n16 + 1 + min(l, nr - 1)];
    }
  }
  if (tid == 0) okl = (c->solve_ok != 0) && !(bv[C] > 0.0);
  // the loop's done flag is tested only here: the ctrl and staging loads above went out in one round trip, and
  // nothing global has been written yet
  if (gate && c->done) return;
  if (gate && !d.gn_fused && tid == 0) c->pending = 1;
  KB_TS(d, 1);
  KB_STAMP(d, 1);
  // phase B: camera block expansion (CM == 0: done by k_colimg)
  if constexpr (CM > 0) {
    for (int q = tid; q < N * N * 36; q += nth) {
      const int e = q % 36, ik = q / 36, i = ik / N, k = ik % N;
      double s = 0.0;
      if (k < i) {
        const int a = e / 6, b = e % 6;
#pragma unroll
        for (int m = 0; m < 6; ++m) s += Hs[i * 256 + a * 16 + m] * K[(i * N + k) * 36 + m * 6 + b];
      }
      T[q] = s;
    }
    if (tid == 0) {
      double s = 0.0;
      for (int i = 0; i < N; ++i) s += Hs[i * 256 + 255];
      d.cost_build[0] = s;
      cl_red[0] = s;
    }
  }
  // GN fused: the previous pass's end.  Its cost is this build's (the system was built at its candidate):
  // accept (GN always does) and the next prelude (Optimizer2.cpp:221-259, TrustRegionPolicy.cpp:39-52)
  auto finish_prev = [&]() {
    dxr = wave_max_d(dxr);
    if ((tid & 63) == 0) {
      KbCtrl& cl = cls;  // LDS copy (a private one would put the kernel arguments in scratch)
      cl = *c;
      if (cl.have_dx) {
        cl_red[1] = cl_red[2] = 0.0;
        cl_red[3] = fmax(dxr, d.camstat[0]);
        pol_post(&cl, d, cl_red);
        if (!cl.done) pol_pre<true>(&cl);
        cl.have_dx = 0;
        cl.pending = 0;
        *c = cl;
      }
      fin[0] = cl.done;
      fin[1] = cl.cur;
    }
  };
  // wave 0 after the solves: camera dx, its statistics, the intrinsic (and, CM > 0, baseline) DV update into the
  // candidate slot 1 - cu
  auto wave0_tail = [&](int cur) {
    const int lane = tid;
    double mx = 0.0, dd = 0.0, dr = 0.0;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int i = lane + 64 * sl;
      if (i < C) {
        const double g = gl[i];
        d.dx[i] = x[sl];
        mx = fmax(mx, fabs(x[sl]));
        dd += x[sl] * x[sl];
        dr += x[sl] * g;
      }
    }
    mx = wave_max_d(mx);
    dd = wave_sum_d(dd);
    dr = wave_sum_d(dr);
    if (lane == 0) {
      d.camstat[0] = mx;
      d.camstat[1] = dd;
      d.camstat[2] = dr;
      if (gfu) {  // the step is applied by the next pass's build (or the finishing back-substitution)
        c->have_dx = 1;
        c->pending = 1;
      }
    }
    if (do_update) {
      // camera design variables: intrinsics (additive, one lane per slot) and baselines (one lane per pose)
      const double* in = camst[cur];  // [intrinsics N * KB_MAX_INTR | baselines 7 (N - 1)] of slot cur
      double* out = d.state + (size_t)(1 - cur) * d.S;
      constexpr int kIntrSlots = (KB_MAX_CAMS * KB_MAX_INTR + 63) / 64;
      double vin[kIntrSlots];
#pragma unroll
      for (int r = 0; r < kIntrSlots; ++r) {
        const int q = lane + 64 * r;
        vin[r] = (q < N * KB_MAX_INTR) ? in[q] : 0.0;
      }
      double bq[7];
      const int jb = lane < N - 1 ? lane : 0;
#pragma unroll
      for (int q = 0; q < 7; ++q) bq[q] = in[N * KB_MAX_INTR + 7 * jb + q];
#pragma unroll
      for (int r = 0; r < kIntrSlots; ++r) {
        if (64 * r >= N * KB_MAX_INTR) break;  // wave-uniform
        const int q = lane + 64 * r;
        const int cm = min(q / KB_MAX_INTR, N - 1), xi = q % KB_MAX_INTR;
        const bool act = q < N * KB_MAX_INTR && xi < ctab[0][cm];
        const int col = act ? ctab[1][cm] + xi : 0;
        const double v0 = __shfl(x[0], col & 63), v1 = __shfl(x[1], col & 63);
        const double dv = (col >> 6) ? v1 : v0;
        if (q < N * KB_MAX_INTR) out[q] = vin[r] + (act ? dv : 0.0);
      }
      if (CM > 0 && N > 1) {  // CM == 0: wave 1 did the baselines (and the chains) beside the backsolve
        double d6[6], nb[7];
        const int cb = ctab[2][jb];
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const int col = cb + q;
          const double v0 = __shfl(x[0], col & 63), v1 = __shfl(x[1], col & 63);
          d6[q] = (col >> 6) ? v1 : v0;
        }
        update_pose(bq, d6, nb);
        if (lane < N - 1)
#pragma unroll
          for (int q = 0; q < 7; ++q) {
            out[d.off_base + 7 * lane + q] = nb[q];
            nbase[7 * lane + q] = nb[q];
          }
      }
    }
  };
  __syncthreads();
  KB_TS(d, 2);
  if constexpr (CM > 0) {
    cam_expand_blocks<CM>(S, C, N, ctab, Hs, T, K, lam2, nth >> 6, gate ? nullptr : d.cond2);
    for (int p = tid; p < C; p += nth) {
      const double g = cam_grad_l(N, ci, Hs, K, p);
      bv[p] += g;
      gl[p] = g;
      d.gc[p] = g;
      d.rhs[p] = g;
    }
  }
  __syncthreads();
  KB_TS(d, 3);
  KB_STAMP(d, 2);
  if constexpr (CM > 0) {
#ifdef KB_STAMPS
    const int reps = (d.dbg_flags & 1) ? 2 : 1;  // diagnostic: factor twice (rolled: same code, warm)
#pragma unroll 1
    for (int rep = 0; rep < reps; ++rep)
#endif
    if (d.pcs_cb) {  // KB_SOLVER_PCG_SCHUR (per-call path: no pass end to fold in)
      auto sget = [&](int i, int j) { return S[i >= j ? cidx(i, j, C) : cidx(j, i, C)]; };
      if (!schur_pcg(d, sget, bv, C, nth, x)) okl = 0;
    } else if (tid < 64) {
      const LdlOut r = ldl_solve_reg<CM>(d, S, bv, C, tid, pubcol);
      x[0] = r.x;
      if (!r.ok) okl = 0;
    } else if (gfu && fwave) {
      finish_prev();
    }
    KB_STAMP(d, 3);
    KB_STAMP(d, 4);
  } else {
    // phase C: blocked LDL^T with the forward solve (row C); the previous pass's end beside the first panel
    if (gfu && fwave) finish_prev();
    if (d.pcs_cb) {  // KB_SOLVER_PCG_SCHUR (per-call path): S and b = row C of the k_colimg image
      auto sget = [&](int i, int j) { return S[i >= j ? tidx(i, j) : tidx(j, i)]; };
      double* bcol = rDv;  // b (row C of the image) as a vector; rDv is unused without the LDL^T
      for (int j = tid; j < C; j += nth) bcol[j] = S[tidx(C, j)];
      __syncthreads();
      if (!schur_pcg(d, sget, bcol, C, nth, x)) okl = 0;
      __syncthreads();
      if (tid < 64 && okl && !(gfu && fin[0])) wave0_tail(gfu ? fin[1] : cur);
    } else {
    ldl_panels(d, S, rDv, Dfac, Xinv, C, nb, &okl);  // ends with a block barrier: okl and fin are final
    KB_TS(d, 4);
    KB_STAMP(d, 3);
    // phase D: Ltilde^T x = z on wave 0; wave 1 updates the baselines from the published baseline rows and builds the
    // candidate state's camera chains while wave 0 finishes the intrinsic rows (the baselines follow every intrinsic
    // column, so their rows are final first)
    const int cb0 = ctab[2][0], pub_tile = N > 1 ? cb0 >> 4 : -1;
    const bool upd = do_update && okl && !(gfu && fin[0]);
    if (tid < 64) {
#if defined(KB_BACKSOLVE1)
      panel_backsolve(d, S, Dfac, Xinv, rDv, C, nb, pubcol, x, pub_tile, xb, &bflag);
#elif defined(KB_BACKSOLVE3)
      panel_backsolve3(d, S, Dfac, Xinv, rDv, C, nb, x, pub_tile, xb, &bflag);
#else
      panel_backsolve2(d, S, Dfac, Xinv, rDv, C, nb, pubcol, x, pub_tile, xb, &bflag);
#endif
      KB_TS(d, 8);
      if (okl && !(gfu && fin[0])) wave0_tail(gfu ? fin[1] : cur);
    } else if ((tid >> 6) == 1 && upd) {
      const int lane = tid & 63, cu = gfu ? fin[1] : cur;
      if (N > 1) {
        while (*(volatile int*)&bflag == 0) __builtin_amdgcn_s_sleep(1);
        KB_WAVE_SYNC();
        const int jb = lane < N - 1 ? lane : 0;
        double bq[7], d6[6], nbv[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) bq[q] = camst[cu][N * KB_MAX_INTR + 7 * jb + q];
        const int cb = ctab[2][jb];
#pragma unroll
        for (int q = 0; q < 6; ++q) d6[q] = *(volatile double*)&xb[cb + q];
        update_pose(bq, d6, nbv);
        if (lane < N - 1) {
          double* out = d.state + (size_t)(1 - cu) * d.S;
#pragma unroll
          for (int q = 0; q < 7; ++q) {
            out[d.off_base + 7 * lane + q] = nbv[q];
            nbase[7 * lane + q] = nbv[q];
          }
        }
        KB_WAVE_SYNC();
      }
      chain_pairs<true>(d, nbase, chl, lane);  // the K entries: all waves after the barrier (chain_write)
    }
    }
    KB_STAMP(d, 4);
  }
  __syncthreads();  // okl final
  KB_TS(d, 5);
  if (gfu) {
    if (fin[0]) return;  // the loop ended at the previous pass: this solve is discarded
    cur = fin[1];
  }
  if (!okl) {
    if (tid == 0) {
      c->solve_ok = 0;
      if (gfu) {  // GN fused: the failed pass ends here (nothing to apply)
        KbCtrl& cl = cls;
        cl = *c;
        cl_red[0] = cl_red[1] = cl_red[2] = cl_red[3] = 0.0;
        pol_post(&cl, d, cl_red);
        if (!cl.done) pol_pre<true>(&cl);
        cl.pending = 0;
        cl.have_dx = 0;
        *c = cl;
      }
    }
    return;
  }
  if (CM > 0 && tid < 64) wave0_tail(cur);  // CM == 0: ran right after the backsolve
  KB_TS(d, 6);
  KB_STAMP(d, 5);
  if (CM > 0 && do_update) {
    __syncthreads();
    chain_block(d, nbase, 1 - cur, nth);  // chains of the candidate state (k_backsub's cost, next build if accepted)
  }
  if (CM == 0 && do_update) chain_write(d, chl, 1 - cur, tid, nth);  // pair products by wave 1 before the barrier
  KB_TS(d, 7);
}

// CM > 0: 4 waves (one factors); CM == 0: 8 waves
template <int CM>
__global__ void __launch_bounds__(CM == 0 ? 512 : 256) k_solve(KbDev d, int gate, int do_update) {
  if constexpr (CM == 0) KB_MFMA_AGPR();
  solve_body<CM>(d, gate, do_update, blockDim.x);  // returns early once ctrl->done (after its staging loads)
}

// ---------------------------------------------------------------------------------------------
// k_backsub: one wave per frame, kBsFrames frames per block (a 2000-frame problem is 2000 waves, resident in one
// round).  The wave forms dx_f = b_f - A_f dx_c (6 wave dot products), stores dx and the new pose, then evaluates the
// cost of the frame's views at the candidate state (evaluateError fused), view after view in 64-corner passes with
// the next pass's loads in flight: per-frame [cost, max|dx|, dx.dx, dx.rhs].  The launch-independent loads go out in
// one round before the gate; the candidate chains and intrinsics are staged in LDS once per block.
// k_post (one block) reduces the per-frame rows (+ camera stats) into red_local and, on one GPU, runs the
// policy (accept / revert, next pass prelude); sharded runs all-reduce red first and run k_policy.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_post(KbDev d, int policy) {
  __shared__ KbCtrl cnew;
  const KbCtrl cin = *d.ctrl;
  if (cin.done) return;
  if (policy && !cin.pending) return;  // nothing pending (already applied by a folding k_build)
  pass_end_block(d, cin, &cnew, true, blockDim.x, policy != 0);
}

constexpr int kBsFrames = 4;  // k_backsub: frames (waves) per block
__global__ void __launch_bounds__(64 * kBsFrames) k_backsub(KbDev d, int gate, int do_update, int with_cost) {
  KbCtrl* c = d.ctrl;
  __shared__ double tg[kTargetLds];
  __shared__ double cch[KB_MAX_CAMS][24];  // candidate chains L (12) | intrinsics (KB_MAX_INTR) of every camera
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, nth = blockDim.x;
  const int C = d.C, N = d.N, F = d.F;
  const int f = blockIdx.x * kBsFrames + wave, fc = min(f, F - 1);  // waves beyond F: loads clamped, no stores
  const bool cost_pass = do_update && with_cost;
  // ---- round 1: launch-independent loads, straight-line and unconditional (clamped) so that they are all in
  // flight together; the gate and the LDS stores come after
  const int done = c->done || (gate && d.gn_fused && !c->have_dx), sok = c->solve_ok, cur = c->cur;
  const bool tg_lds = 3 * d.K <= kTargetLds;
  const int nt3 = 3 * d.K;
  constexpr int kTgU = 6;  // 6 x 256 >= 3 x 512 target corners staged in one round
  double tv[kTgU];
#pragma unroll
  for (int u = 0; u < kTgU; ++u) tv[u] = d.target[min(tid + u * nth, nt3 - 1)];
  double yr[6][2], dxv[2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int q = lane + 64 * sl, qc = min(q, C - 1);
    const double v = d.dx[qc];
    dxv[sl] = q < C ? v : 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double yv = d.Af[((size_t)fc * 6 + r) * C + qc];
      yr[r][sl] = q < C ? yv : 0.0;
    }
  }
  const double bq = d.bf[(size_t)fc * 6 + min(lane, 5)];
  const int2 fvl = d.fview[(size_t)fc * N + min(lane, N - 1)];  // lane cm: the corner range of view (f, cm)
  // pin the round-1 values here: keeps the compiler from sinking the loads below the gate (one round trip)
  KB_KEEP(fvl.x);
  KB_KEEP(fvl.y);
  KB_KEEP(bq);
#pragma unroll
  for (int u = 0; u < kTgU; ++u) KB_KEEP(tv[u]);
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    KB_KEEP(dxv[sl]);
#pragma unroll
    for (int r = 0; r < 6; ++r) KB_KEEP(yr[r][sl]);
  }
  if (gate && done) return;  // block-uniform
  KB_STAMP(d, 30);
  const bool work = (!gate || sok) && f < F;
  const double* s0 = d.state + (size_t)cur * d.S;
  double* s1 = d.state + (size_t)(1 - cur) * d.S;
  // ---- round 2: loads indexed by round 1 (state buffers); the per-camera chains and intrinsics of the candidate state
  // go to LDS once per block
  if (cost_pass) {
    if (tg_lds) {
#pragma unroll
      for (int u = 0; u < kTgU; ++u)
        if (tid + u * nth < nt3) tg[tid + u * nth] = tv[u];
      for (int q = tid + kTgU * nth; q < nt3; q += nth) tg[q] = d.target[q];
    }
    const double* Lp = cam_L(d, 1 - cur);
    for (int q = tid; q < N * 22; q += nth) {
      const int cm = q / 22, e = q - 22 * cm;
      cch[cm][e] = e < 12 ? Lp[cm * 12 + e] : s1[cm * KB_MAX_INTR + e - 12];
    }
  }
  double pose[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) pose[q] = do_update ? s0[d.off_frame + 7 * fc + q] : 0.0;
  const double gq = d.gf[(size_t)fc * 6 + min(lane, 5)];
  // dx_f = b_f - A_f dx_c (every lane ends with all six entries)
  double w[6];
  fdx_solve(yr, dxv, bq, w);
  KB_STAMP(d, 31);
  if (work && lane < 6) {
    double xv = w[0];
#pragma unroll
    for (int r = 1; r < 6; ++r) xv = (lane == r) ? w[r] : xv;
    d.dx[C + 6 * f + lane] = xv;
    d.rhs[C + 6 * f + lane] = gq;
  }
  double cost = 0.0;
  if (do_update) {
    double np[7];
    update_pose(pose, w, np);  // every lane: the new pose stays in registers
    if (work && lane < 7) {
      double pv = np[0];
#pragma unroll
      for (int q = 1; q < 7; ++q) pv = (lane == q) ? np[q] : pv;
      s1[d.off_frame + 7 * f + lane] = pv;
    }
    KB_STAMP(d, 32);
    if (with_cost) {
      const double* tgt = tg_lds ? tg : d.target;
      __syncthreads();  // target and camera tables staged (every wave of the block reaches this)
      double Ri[9], ti[3];
      pose_inverse(np, Ri, ti);
      // the frame's views one after the other in 64-corner passes; the next pass's corner ids and keypoints are in
      // flight while the current pass projects (the views of a frame are contiguous, empty views are (0, 0))
      auto lo = [&](int cm) { return __builtin_amdgcn_readlane(fvl.x, cm); };
      auto hi = [&](int cm) { return __builtin_amdgcn_readlane(fvl.y, cm); };
      int cm = 0, k0 = lo(0);
      while (cm < N && k0 >= hi(cm)) {
        ++cm;
        if (cm < N) k0 = lo(cm);
      }
      int cidn = 0;
      double2 yn = make_double2(0.0, 0.0);
      if (cm < N) {
        const int k = min(k0 + lane, hi(cm) - 1);
        cidn = d.cid[k];
        yn = d.y[k];
      }
      int lastc = -1;
      double R[9], t[3];
      while (cm < N && work) {  // wave-uniform
        const int cc = cm, kk = k0, hc = hi(cm);
        const int cid = cidn;
        const double2 yv = yn;
        k0 += 64;
        while (cm < N && k0 >= hi(cm)) {
          ++cm;
          if (cm < N) k0 = lo(cm);
        }
        if (cm < N) {
          const int k = min(k0 + lane, hi(cm) - 1);
          cidn = d.cid[k];
          yn = d.y[k];
        }
        if (cc != lastc) {
          rt_mul(cch[cc], cch[cc] + 9, Ri, ti, R, t);  // T_cam_w = L_cam(candidate) T_f^-1
          lastc = cc;
        }
        if (kk + lane < hc) {
          const double X0 = tgt[3 * cid], X1 = tgt[3 * cid + 1], X2 = tgt[3 * cid + 2];
          const double p0 = R[0] * X0 + R[1] * X1 + R[2] * X2 + t[0];
          const double p1 = R[3] * X0 + R[4] * X1 + R[5] * X2 + t[1];
          const double p2 = R[6] * X0 + R[7] * X1 + R[8] * X2 + t[2];
          double u0, u1;
          project(cam_arg(d.model, cc), cch[cc] + 12, p0, p1, p2, u0, u1);
          const double e0 = yv.x - u0, e1 = yv.y - u1;
          cost += e0 * e0 + e1 * e1;
        }
      }
      cost = wave_sum_d(cost);
    }
  }
  KB_STAMP(d, 33);
  if (work && lane == 0) {
    double a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double g = readlane_d(gq, r);
      a1 = fmax(a1, fabs(w[r]));
      a2 += w[r] * w[r];
      a3 += w[r] * g;
    }
    reinterpret_cast<double4*>(d.bpart)[f] = make_double4(cost, a1, a2, a3);
  }
}

// ---------------------------------------------------------------------------------------------
// k_cost: one wave per view on state buffer (cur ^ which); per-block partial sums (kb_eval_cost, loop start)
// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
// rhs^T (J^T J) rhs of the last build (LinearSystemSolver::rhsJtJrhs, LinearSystemSolver.hpp:66-69; the reference
// forms ||J rhs||^2, SparseCholeskyLinearSystemSolver.cpp:106-111), from the arrow blocks: one wave per frame forms
// t_f = r_f^T H_ff r_f + 2 r_f^T H_fc r_c into part[f]; k_rjr_final sums the frames in a fixed order and adds
// r_c^T H_cc r_c.  r = [g_c | g_f] (the rhs kb_build left).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_rjr_frames(KbDev d, double* part) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int f = blockIdx.x * 4 + wave;
  if (f >= d.F) return;
  const int C = d.C;
  const double* gf = d.gf + (size_t)f * 6;
  double rf[6];
#pragma unroll
  for (int a = 0; a < 6; ++a) rf[a] = gf[a];
  double s = 0.0;
  for (int c = lane; c < C; c += 64) {
    const double rc = d.gc[c];
    double w = 0.0;
#pragma unroll
    for (int a = 0; a < 6; ++a) w = fma(rf[a], d.Hfc[((size_t)f * 6 + a) * C + c], w);
    s = fma(2.0 * w, rc, s);
  }
  if (lane < 36) s = fma(rf[lane / 6] * d.Hff[(size_t)f * 36 + lane], rf[lane % 6], s);
  s = wave_sum_d(s);
  if (lane == 0) part[f] = s;
}

__global__ void __launch_bounds__(256) k_rjr_final(KbDev d, const double* part, double* out) {
  __shared__ double sh[4];
  const int tid = threadIdx.x, C = d.C;
  double s = 0.0;
  for (int f = tid; f < d.F; f += blockDim.x) s += part[f];
  for (int q = tid; q < C * C; q += blockDim.x) s = fma(d.gc[q / C] * d.Hcc[q], d.gc[q % C], s);
  s = wave_sum_d(s);
  if ((tid & 63) == 0) sh[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) out[0] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__global__ void __launch_bounds__(256) k_cost(KbDev d, int which) {
  KbCtrl* c = d.ctrl;
  __shared__ double part[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + wave;
  const double* s = d.state + (size_t)(c->cur ^ which) * d.S;
  double acc = 0.0;
  if (v < d.V) {
    const int f = d.view_frame[v], cam = d.view_cam[v];
    double R[9], t[3];
    cam_from_state(d, s, cam, s + d.off_frame + 7 * f, R, t);
    const int model = cam_arg(d.model, cam);
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
    acc = wave_sum_d(acc);
  }
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) d.costpart[blockIdx.x] = ((part[0] + part[1]) + part[2]) + part[3];
}

// fixed-order block reduction (one block of 256)
__device__ double block_reduce(double s, double* sh, bool is_max) {
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      sh[threadIdx.x] = is_max ? fmax(sh[threadIdx.x], sh[threadIdx.x + o]) : sh[threadIdx.x] + sh[threadIdx.x + o];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(256) k_reduce_cost(KbDev d) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int q = threadIdx.x; q < d.nblk_cost; q += blockDim.x) s += d.costpart[q];
  s = block_reduce(s, sh, false);
  if (threadIdx.x == 0) {
    d.red_local[0] = s;
    d.red_local[1] = d.red_local[2] = d.red_local[3] = 0.0;
  }
}

// red = fixed-order reduction of the all-gathered per-rank [cost, dx.dx, dx.rhs] (sum) and max|dx| (max)
// ---------------------------------------------------------------------------------------------
// Reprojection-error statistics of the current state (CameraCalibrator.hpp:368-411, printed per camera by
// CalibrateCameras.cpp:318): e = y - yhat of every term (ReprojectionError::getPredictedMeasurement,
// ReprojectionError.hpp(impl):98-106).  Two passes as the reference's: k_rstats with sums == null gives per view
// [count, sum e_u, sum e_v]; with the per-camera sums of pass one it gives [count, sum (e_u - mean_u)^2,
// sum (e_v - mean_v)^2] (one wave per view, fixed-order wave sums); k_rstats_red sums a camera's views in a fixed
// order (one block per camera).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_rstats(KbDev d, const double* sums, double* vpart) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + wave;
  if (v >= d.V) return;  // wave-uniform
  const double* s = d.state + (size_t)d.ctrl->cur * d.S;
  const int f = d.view_frame[v], cam = d.view_cam[v];
  double R[9], t[3];
  cam_from_state(d, s, cam, s + d.off_frame + 7 * f, R, t);
  const int model = cam_arg(d.model, cam);
  const double* intr = s + cam * KB_MAX_INTR;
  double mu = 0.0, mv = 0.0;
  if (sums) {
    const double n = sums[3 * cam];
    mu = sums[3 * cam + 1] / n;
    mv = sums[3 * cam + 2] / n;
  }
  const int o0 = d.view_off[v], o1 = d.view_off[v + 1];
  double a0 = 0.0, a1 = 0.0;
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
    if (sums) {
      a0 += (e0 - mu) * (e0 - mu);
      a1 += (e1 - mv) * (e1 - mv);
    } else {
      a0 += e0;
      a1 += e1;
    }
  }
  a0 = wave_sum_d(a0);
  a1 = wave_sum_d(a1);
  if (lane == 0) {
    vpart[3 * (size_t)v] = (double)(o1 - o0);
    vpart[3 * (size_t)v + 1] = a0;
    vpart[3 * (size_t)v + 2] = a1;
  }
}

__global__ void __launch_bounds__(256) k_rstats_red(KbDev d, const double* vpart, double* out) {
  __shared__ double sh[256];
  const int cam = blockIdx.x;
  double a[3] = {0.0, 0.0, 0.0};
  for (int v = threadIdx.x; v < d.V; v += blockDim.x)
    if (d.view_cam[v] == cam)
#pragma unroll
      for (int q = 0; q < 3; ++q) a[q] += vpart[3 * (size_t)v + q];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double r = block_reduce(a[q], sh, false);
    if (threadIdx.x == 0) out[3 * cam + q] = r;
    __syncthreads();
  }
}

__device__ __forceinline__ void red_gather(const KbDev& d, double* red) {
  red[0] = red[1] = red[2] = red[3] = 0.0;
  for (int r = 0; r < d.nranks; ++r) {
    const double* q = d.red_all + 4 * r;
    red[0] += q[0];
    red[1] += q[1];
    red[2] += q[2];
    red[3] = fmax(red[3], q[3]);
  }
}

__global__ void k_red_gather(KbDev d) {
  double red[4];
  red_gather(d, red);
  for (int q = 0; q < 4; ++q) d.red[q] = red[q];
}

// sharded runs: the policy after the all-gather of red (accept / revert, next pass prelude)
__global__ void k_policy(KbDev d) {
  KbCtrl* c = d.ctrl;
  if (c->done) return;
  double red[4];
  red_gather(d, red);
  KbCtrl cl = *c;
  pol_post(&cl, d, red);
  if (!cl.done) pol_pre(&cl);
  cl.pending = 0;
  cl.have_dx = 0;
  *c = cl;
}

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
  c->pending = 0;
  c->have_dx = 0;
  c->comm_err = 0;  // (the host agreed on the transport at the loop start: a failed direct path is off by now)
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
    out[t] = in[t] + ((x < cam_arg(d.nintr, cam)) ? d.dx[cam_arg(d.col_intr, cam) + x] : 0.0);
  }
  if (t < N - 1) update_pose(in + d.off_base + 7 * t, d.dx + cam_arg(d.col_base, t), out + d.off_base + 7 * t);
  if (t < d.F) update_pose(in + d.off_frame + 7 * t, d.dx + d.C + 6 * t, out + d.off_frame + 7 * t);
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
