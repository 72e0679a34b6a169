// kb_device.h -- device-side data layout of one calibration problem (one handle / rank).
//
// HBM layout (FP64 unless noted), sized at kb_upload_observations:
//   y        double2 [Nc]          measured keypoints, views contiguous, views sorted by frame
//   cid      uint16  [Nc]          target corner of each term
//   view_off uint32  [V+1]; view_frame int32 [V]; view_cam int32 [V]; frame_vcam int32 [F][N] (-1 = none)
//   state    [2][S]                ping-pong design-variable buffers, ctrl->cur = accepted one
//   Hff [F][36], Hfc [F][6][C], gf [F][6]     arrow blocks written by k_build
//   campart [nblk][N][136]         per-block per-camera partial sums (16x16 upper)
//   Lf [F][36], Yf [F][6][C], zf [F][6]       Schur factors written by k_schur
//   schurpart [nblk][W]            per-block sum Y^T Y (upper packed) | Y^T z, W = C(C+1)/2 + C
//   redA_local = [camsum N*136 | schursum W] (all-reduced into redA when sharded)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kb_math.h"

namespace kb {

struct KbCtrl {
  int cur, done, do_build, solve_ok, first, prev_failed, lin_fail;
  int iterations, failed_iterations, max_iterations, policy, n_trace, passes, pad_;
  double J, p_J, J_start, deltaX, deltaJ, eps_x, eps_j;
  double pol_J, pol_pJ, last_succ, lambda, mu;
  double dxdx, dxrhs;
};

struct KbOpts {
  int policy, max_iterations;
  double lambda_init, eps_x, eps_j;
};

struct KbDev {
  int N, F, V, NC, C, ncols, S;
  int off_base, off_frame;
  int gframes, nblk, nblk_bs, nblk_cost;
  int trace_cap;
  double host_lambda;  // conditioner for the per-call (non-gated) path
  int model[KB_MAX_CAMS], nintr[KB_MAX_CAMS], col_intr[KB_MAX_CAMS], col_base[KB_MAX_CAMS];
  const double* target;
  const double2* y;
  const uint16_t* cid;
  const uint32_t* view_off;
  const int32_t* view_frame;
  const int32_t* view_cam;
  const int32_t* frame_vcam;
  const int32_t* colinfo;  // [C]: kind<<16 | cam_or_baseline<<8 | index
  const int32_t* tri;      // [C(C+1)/2]: a<<16 | b
  double* state;
  double* camL;  // [N][12]
  double* camK;  // [N][N][36]
  double *Hff, *Hfc, *gf;
  double* campart;
  double* camsum_local;  // colsum output (this rank)
  double* camsum;        // reduced over ranks (aliases camsum_local on one GPU)
  double *Hcc, *gc, *cost_build;
  double *Lf, *Yf, *zf;
  double* schurpart;
  double* schursum_local;
  double* schursum;
  double *dx, *rhs;
  double* statpart;
  double* camstat;   // [3]
  double* costpart;
  double* red_local; // [4]
  double* red;       // [4] (reduced)
  double* trace;
  KbCtrl* ctrl;
};

// 16x16 upper-packed helpers (row-major upper: a <= b)
__host__ __device__ __forceinline__ int d16_index(int a, int b) { return a * 16 - a * (a - 1) / 2 + (b - a); }
__device__ __forceinline__ int d16_row(int e) {
  int a = 0;
  while (e >= 16 - a) {
    e -= 16 - a;
    ++a;
  }
  return a;
}
__device__ __forceinline__ int d16_col(int e) {
  int a = 0;
  while (e >= 16 - a) {
    e -= 16 - a;
    ++a;
  }
  return a + e;
}

}  // namespace kb
