// kb_device.h -- device-side data layout of one calibration problem (one handle / rank).
//
// HBM layout (FP64 unless noted), sized at kb_upload_observations:
//   y        double2 [Nc]          measured keypoints, views contiguous, views sorted by frame
//   cid      uint16  [Nc]          target corner of each term
//   view_off uint32  [V+1]; view_frame int32 [V]; view_cam int32 [V]; frame_vcam int32 [F][N] (-1 = none)
//   state    [2][S]                ping-pong design-variable buffers, ctrl->cur = accepted one
//   Hff [F][36], Hfc [F][6][C], gf [F][6]     arrow blocks written by k_build
//   Af [F][6][C], bf [F][6]                   dx_f = b_f - A_f dx_c (k_build fused / k_schur)
//   part [nblk][Wr]                per-block partials: per-camera 16x16 upper sums (N*136) |
//                                  sum Y^T Y upper (C(C+1)/2) | sum Y^T z (C) | #non-PD frames (1) | max|dx_f| (1)
//   part8 [8][Wtot]                stage-1 column sums of part (k_colsum) | per-rank max|dx_f| (GN fused);
//                                  psum_local [Wtot] the finished sums
//   bpart [nblk_bs][4]             k_backsub_cost: cost, max|dx|, dx.dx, dx.rhs per block
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kb_math.h"

namespace kb {

struct KbCtrl {
  int cur, done, do_build, solve_ok, first, prev_failed, lin_fail;
  int iterations, failed_iterations, max_iterations, policy, n_trace, passes;
  int pending;  // a pass ran its solve: its accept/revert + the next prelude are still to apply
  int have_dx;  // GN fused passes: the last solve's dx is still to apply (by the next build or the finish)
  int comm_err;  // k_xar: a peer rank did not arrive within the wait bound (the pass batch ends, the host fails the call)
  double J, p_J, J_start, deltaX, deltaJ, eps_x, eps_j;
  double pol_J, pol_pJ, last_succ, lambda, mu;
  double dxdx, dxrhs;
};

struct KbOpts {
  int policy, max_iterations;
  double lambda_init, eps_x, eps_j;
};

constexpr int kColsumRows = 8;  // stage-1 row splits of the block partial reduction
constexpr int kXarBlocks = 32;        // k_xar blocks (each sums one chunk of the image over the ranks)
constexpr int kXMaxRanksDev = 64;     // k_xar ranks (peer table in LDS)
constexpr int kXarFlagDoubles = 64;   // flag area of an exchange region (kXarBlocks u64, padded to 512 B)
constexpr unsigned long long kXarTimeoutTicks = 1000000000ull;  // default wait bound: 10 s of s_memrealtime (100 MHz)

// k_marg (marginal truncated-SVD camera solve, aslam_incremental_calibration LinearSolver)
constexpr int kMargThreads = 1024;
constexpr int kMargMaxC = 112;         // packed Omega + V in LDS: C(C+1)/2 + C^2 + 2C doubles <= 160 KB
constexpr int kMargMaxSweeps = 40;
constexpr double kMargJacobiTol = 1.1102230246251565e-16;  // skip |a_pq| <= 2^-53 sqrt|a_pp a_qq|
constexpr int kMargItems = 8;    // k_marg items (2x2 blocks, rows of V) per thread at C <= kMargMaxC
constexpr int kMargWarmMax = 32;     // consecutive warm starts before a cold (identity) start bounds V's orthogonality drift
constexpr int kMargFullMaxC = 96;   // largest C whose full-storage Omega (padded to even) + V fit kMargLdsStage
constexpr int kMargLdsStage = 19000;  // dynamic LDS doubles up to which V0 is staged in LDS too (static ~7 KB beside)
// block size of k_marg: one thread per 2x2 block of pairs and per (row of V, pair), whole waves
__host__ __device__ inline int marg_threads(int C) {
  const int h = (C + (C & 1)) / 2, items = h * (h + 1) / 2 + C * h;
  const int t = (items + 63) / 64 * 64;
  return t < kMargThreads ? t : kMargThreads;
}
struct KbMarg {
  int scaling;      // LinearSolverOptions::columnScaling
  int write_dx;     // 1: solve (dx_c into d.dx); 0: analyzeMarginal (SVD only)
  int warm;         // 1: start the sweeps from the previous call's V (info[5] counts the warm chain)
  double norm_tol;  // sqrt(rows * epsNorm)
  double eps_svd, svd_tol;
  double* sv;    // [C] singular values, descending
  double* V;     // [C][C] row-major, right singular vector j in column j
  double* info;  // [8]: rank, sweeps, tolerance, sv gap, log2 sum of the first rank singular values, warm chain
};

struct KbDev {
  int N, F, V, NC, C, ncols, S, K;  // K = target corners
  int off_base, off_frame;
  int gframes, nblk, nblk_bs, nblk_cost;
  int nsplit, wpb;   // k_build: waves per block = N * nsplit
  int W, Wp, Wr, Wtot;  // W = C(C+1)/2 + C ; Wp = N*136 + W + 1 summed entries of a block partial row ;
                       // Wr = Wp + 1 (+ the block's max|dx_f|, GN fused) ; Wtot = Wp + max(nranks, 1)
  int trace_cap;
  int fold;          // 1: the next pass's k_build applies the pending policy (non-fused passes)
  int gn_fused;      // 1: Gauss-Newton passes fused as [update + build] -> colsum -> [GN policy + solve]
  int rank;
  double host_lambda;  // conditioner for the per-call (non-gated) path
  const double* cond2;  // per-call solve with a diagonal conditioner: its squares [C + 6F] (canonical order), or null
  int model[KB_MAX_CAMS], nintr[KB_MAX_CAMS], col_intr[KB_MAX_CAMS], col_base[KB_MAX_CAMS];
  const double* target;
  const double2* y;
  const uint16_t* cid;
  const uint32_t* view_off;
  const int32_t* view_frame;
  const int32_t* view_cam;
  const int32_t* frame_vcam;
  const int2* fview;       // [F][N]: corner range (o0, o1) of view (f, cam); o0 == o1 when absent
  const int32_t* colinfo;  // [C]: kind<<16 | cam_or_baseline<<8 | index
  const int32_t* tri;      // [C(C+1)/2]: a<<16 | b
  double* state;
  double* camL;  // [2][N][12]    camera chains L_i of state buffer `slot` (ping-pong with ctrl->cur)
  double* camK;  // [2][N][N][36] baseline chains K_{i,j} of state buffer `slot`
  double *Hff, *Hfc, *gf;
  double *Af, *bf;  // [F][6][C], [F][6]: frame back-substitution rows L_f^-T Y_f, L_f^-T z_f
  double* part;   // [nblk][Wr]
  double* part8;       // [8][Wtot] stage-1 column sums
  double* psum_local;  // [Wtot] finished column sums of this rank (last k_colsum block)
  const double* psum;  // consumer view of the column sums: psum_rows rows of Wtot summed in fixed order
  int psum_rows;       // 1 (psum_local or its all-reduce over ranks) or kColsumRows (part8, one GPU loop)
  unsigned* ticket;    // [2] arrival counters: k_colsum, k_backsub (re-armed by the last block)
  double *Hcc, *gc, *cost_build;
  double *dx, *rhs;
  double* bpart;     // [nblk_bs][4] (sharded: padded to the largest rank's frame count, zero rows beyond F)
  const double* bsrc;  // rows the pass end reduces: bpart (one GPU) or the all-gathered [nranks][F_max][4]
  int bsrc_rows;
  double* camstat;   // [4]
  double* costpart;  // [nblk_cost]
  double* red_local; // [4]: cost, dx.dx, dx.rhs, max|dx|
  double* red;       // [4] (reduced over ranks; aliases red_local on one GPU)
  const double* red_all;  // [nranks][4] all-gathered red_local (sharded runs)
  int nranks;
  double* trace;
  double* simg;  // C > 64: k_solve's LDS image of the camera block (k_colimg / k_colsumx) [img_n]
  int img_n;
  // GN fused passes of the pipelined build with C > 64 ("expanded" partials): k_buildp expands its block's per-camera
  // sums through the chains itself, so a block partial row holds [g_c (C) | cost (1) | unused .. | S - lambda^2 I
  // (upper packed) | b | non-PD | max|dx_f|], and k_colsumx writes the column sums straight into the k_solve image
  // (no k_colimg).  Image aux slots after the tiles: [g_c | non-PD at C] (n16) | cost | max|dx_f| per rank.
  int xexp;
  int bp_tg;   // k_buildp: the target corners staged in LDS (the host's LDS budget decides)
  double* ximg;  // image the column sums are written to: simg (one GPU) or this rank's partial image (sharded)
  // direct all-reduce of the sharded image (k_xar, kb_comm_init / kb_comm_init_local): this rank's exchange region
  // [kXarFlagDoubles flags (one u64 per k_xar block) | partial image, even launches | odd launches] and the regions of
  // every rank (rank order; peers mapped by IPC handles), k_colsumx writes its partial image into the region
  int xar;
  double* xar_buf;
  double* const* xar_peers;
  unsigned long long xar_timeout;  // k_xar's wait bound in s_memrealtime ticks (KB_XAR_TIMEOUT_MS, default kXarTimeoutTicks)
  // per-pass timing query only (kb_gn_pass_times): [0] arrival counter | [1 ..] s_memrealtime (100 MHz) at the start of
  // each pass's build kernel (block 0), null otherwise
  unsigned long long* pass_ts;
  KbCtrl* ctrl;
  // KB_SOLVER_PCG_SCHUR (per-call kb_solve only): k_solve runs block-Jacobi PCG on the Schur complement instead of
  // the LDL^T.  pcs_cb: [2][C] camera DV block start / size per column (null: the LDL^T); pcs_info [4]: iterations,
  // residual (dn / 2), d0, ok
  const int* pcs_cb;
  double pcs_tol, pcs_prev;
  int pcs_maxit, pcs_abs;
  double* pcs_info;
  int dbg_stop;   // diagnostic build only (KB_STAMPS): stop point of the timed kernel (-1: run to the end)
  int dbg_flags;  // diagnostic build only: bit 0 run the camera LDL^T twice (rolled)
  long long* dbg_ts;  // diagnostic build only: [128] s_memrealtime stamps: k_solve (KB_TS) | k_buildp (KB_TSB, +64)
};

#ifdef KB_STAMPS
// diagnostic build only: every thread leaves the kernel at stop point i when d.dbg_stop == i, so the kernel's
// duration up to that point can be timed from the host (tools/diag_stamps.py); stop points sit where the
// whole block is converged
#define KB_STAMP(d, i)          \
  do {                          \
    if ((d).dbg_stop == (i)) return; \
  } while (0)
// timeline stamp (100 MHz s_memrealtime) of thread 0 at point i of the last launch, without leaving the kernel
#define KB_TS(d, i)                                                                      \
  do {                                                                                   \
    if (threadIdx.x == 0 && (d).dbg_ts) {                                                \
      (d).dbg_ts[i] = __builtin_amdgcn_s_memrealtime();                                  \
      if ((i) == 0 || (i) == 7) (d).dbg_ts[60 + ((i) == 7)] = __builtin_amdgcn_s_memtime(); \
    }                                                                                    \
  } while (0)
// build-kernel timeline (k_buildp): lane 0 of the calling wave of block 0 stamps slot 64 + i
#define KB_TSB(d, i)                                                                                        \
  do {                                                                                                      \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (d).dbg_ts) (d).dbg_ts[64 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// k_marg timeline: thread 0 stamps slot 200 + i (s_memtime shader clock at i = 0 and 11 into 216 / 217)
#define KB_TSM(d, i)                                                                     \
  do {                                                                                   \
    if (threadIdx.x == 0 && (d).dbg_ts) {                                                \
      (d).dbg_ts[200 + (i)] = __builtin_amdgcn_s_memrealtime();                          \
      if ((i) == 0 || (i) == 11) (d).dbg_ts[216 + ((i) == 11)] = __builtin_amdgcn_s_memtime(); \
    }                                                                                    \
  } while (0)
#else
#define KB_TSM(d, i) \
  do {               \
  } while (0)
#define KB_TSB(d, i) \
  do {               \
  } while (0)
#define KB_STAMP(d, i) \
  do {                 \
  } while (0)
#define KB_TS(d, i) \
  do {              \
  } while (0)
#endif

// kb_gn_pass_times: one timestamp per pass at the build kernel's start (block 0, one lane; a vector atomic picks the
// slot), so that the per-pass durations come from inside the captured graph without extra graph nodes
constexpr int kPassTsCap = 255;
__device__ __forceinline__ void pass_stamp(const KbDev& d) {
  if (d.pass_ts && blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned i = atomicAdd(reinterpret_cast<unsigned*>(d.pass_ts), 1u);
    if (i < (unsigned)kPassTsCap) d.pass_ts[1 + i] = t;
  }
}

__device__ __forceinline__ double* cam_L(const KbDev& d, int slot) { return d.camL + (size_t)slot * d.N * 12; }
__device__ __forceinline__ double* cam_K(const KbDev& d, int slot) { return d.camK + (size_t)slot * d.N * d.N * 36; }

// 16x16 upper-packed helpers (row-major upper: a <= b)
__host__ __device__ __forceinline__ int d16_index(int a, int b) { return a * 16 - a * (a - 1) / 2 + (b - a); }
__device__ __forceinline__ void d16_rowcol(int e, int& a, int& b) {
  int r = 0;
  while (e >= 16 - r) {
    e -= 16 - r;
    ++r;
  }
  a = r;
  b = r + e;
}
// closed form of d16_rowcol: row a = largest with a(33 - a)/2 <= e
__device__ __forceinline__ void d16_rowcol_fast(int e, int& a, int& b) {
  int r = (int)((33.0f - sqrtf(1089.0f - 8.0f * (float)e)) * 0.5f);
  r = r < 0 ? 0 : (r > 15 ? 15 : r);
  if (r * (33 - r) / 2 > e) --r;
  else if (r < 15 && (r + 1) * (32 - r) / 2 <= e) ++r;
  a = r;
  b = r + e - r * (33 - r) / 2;
}
__host__ __device__ __forceinline__ int upper_index(int a, int b, int n) { return a * n - a * (a - 1) / 2 + (b - a); }

}  // namespace kb
