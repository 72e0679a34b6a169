// kb_pcg.hip -- block-Jacobi preconditioned conjugate gradients on the arrow normal equations, the
// iterative alternative to the direct Schur solve (SURVEY.md 7 step 5, 8(b) "direct or PCG by mode").
//
// Restates sparse_block_matrix's LinearSolverPCG::solve (aslam_optimizer/sparse_block_matrix/include/
// sparse_block_matrix/implementation/linear_solver_pcg.hpp:58-130, defaults linear_solver_pcg.h:39-47):
//   x = 0, r = b, d = M^-1 r, dn = r.d, d0 = tol dn (absolute mode: d0 = max(d0, previous _residual))
//   while it < maxIter and dn > d0:  q = A d; a = dn / d.q; x += a d; r -= a q; s = M^-1 r;
//                                    dn' = r.s; d = s + (dn'/dn) d
//   _residual = dn / 2
// with A = H + lambda^2 I of the last kb_build (H_ff, H_fc, H_cc in HBM) and M the diagonal design-variable
// blocks of A (the reference inverts each diagonal block of its SparseBlockMatrix, :72-75): the camera DV
// blocks (projection, distortion, baseline rotation / translation) and per frame the rotation and translation
// DVs (3 x 3 each).
//
// One cooperative launch runs the whole solve.  Block b owns frames [b fpb, (b+1) fpb): their H_fc rows, H_ff
// blocks, preconditioner blocks and vector segments stay in LDS for the whole solve; the C camera entries of
// every vector are kept redundantly by every block (identical bits: every block reduces the same partials in
// the same order).  Per iteration two grid barriers:
//   A  q_f = A_ff d_f + H_fc d_c (rows of the block); partial P_b = sum_f H_fc^T d_f (+ rows p = b mod nblk
//      of H_cc d_c + lambda^2 d_c); partial d_f.q_f                                      -> barrier
//   B  q_c = sum_b P_b (fixed order), a, x/r updates, s = M^-1 r, partial r_f.s_f       -> barrier
//   C  dn' = sum_b partials + r_c.s_c, d = s + (dn'/dn) d; loop test (uniform: same bits in every block)
// The barrier is a monotonic arrival counter with release / acquire at agent scope and a bounded spin (a
// missing block ends the solve with an error flag instead of hanging the GPU); after it every wave runs an
// agent-scope acquire fence, so the cross-block partials are read with plain (batched) loads.
#include "kb_device.h"

namespace kb {

// diagnostic build only: s_memrealtime stamps of block 0, thread 0 (slot 200 + 6 it + phase, first 8 iterations)
#ifdef KB_STAMPS
#define KB_PCG_TS(slot)                                                                                         \
  do {                                                                                                          \
    if (blockIdx.x == 0 && threadIdx.x == 0 && d.dbg_ts && (slot) < 256) d.dbg_ts[slot] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define KB_PCG_TS(slot) \
  do {                  \
  } while (0)
#endif

constexpr int kPcgThreads = 256;
constexpr int kPcgMaxFpb = 16;      // frames per block
constexpr unsigned kPcgSpinLimit = 1u << 26;

struct KbPcg {
  double lam2, tol, prev_residual;
  int max_it, abs_tol, fpb, nblk;
  const int* cb_start;  // [C] first column of the camera DV block of column p
  const int* cb_size;   // [C] its size (1..6)
  double* part;         // [nblk][C + 1]   phase A partials
  double* part2;        // [nblk]          phase B partials (r_f . s_f)
  unsigned* bar;        // arrival counter (zeroed before the launch)
  double* info;         // [5]: iterations, residual (dn / 2), d0, ok (1; 0 breakdown / singular block),
                        //      barrier timeout (1)
};

// cross-block partials are read with plain loads after pcg_barrier: every wave executes an agent-scope acquire
// fence there (vL1D invalidate), so no stale line of a previous round survives
__device__ __forceinline__ double ld_part(const double* p) { return *p; }

// grid barrier number `k` (1, 2, ...), two levels: block b arrives on the counter of its group b % kPcgGroups (one
// 128-byte line each, bar[32 (1 + g)]); the block that completes its group (fetch_add returns k * size_g - 1)
// arrives on the top counter bar[0], and every block waits for bar[0] >= k * ngroups.  The top counter takes
// ngroups atomics instead of nblk (one counter serialised ~250 same-address agent-scope atomics per barrier).
// Release / acquire at agent scope on every step; bounded spin: returns false on a timeout.
constexpr int kPcgGroups = 16;
constexpr int kPcgBarWords = 32 * (1 + kPcgGroups);
__device__ __forceinline__ bool pcg_barrier(unsigned* bar, unsigned nblk, unsigned k, int* lds_flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned ng = nblk < (unsigned)kPcgGroups ? nblk : (unsigned)kPcgGroups;
    const unsigned g = blockIdx.x % ng;
    const unsigned gsize = nblk / ng + (g < nblk % ng ? 1u : 0u);
    const unsigned old = __hip_atomic_fetch_add(bar + 32 * (1 + g), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == k * gsize) __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = k * ng;
    unsigned spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kPcgSpinLimit) {
        *lds_flag = 1;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return *lds_flag == 0;
}

// in-place inverse of an m x m diagonal DV block (row stride ld, in LDS) by Gauss-Jordan without pivoting: the blocks
// are diagonal blocks of the PSD system, so a zero pivot means a singular block (false).  No private array: a
// run-time sized one would put the kernel in per-lane scratch.
__device__ bool pcg_block_inverse(double* M, int m, int ld) {
  for (int k = 0; k < m; ++k) {
    const double piv = M[k * ld + k];
    if (!(fabs(piv) > 0.0)) return false;
    const double inv = 1.0 / piv;
    M[k * ld + k] = 1.0;
    for (int c = 0; c < m; ++c) M[k * ld + c] *= inv;
    for (int r = 0; r < m; ++r) {
      if (r == k) continue;
      const double f = M[r * ld + k];
      M[r * ld + k] = 0.0;
      for (int c = 0; c < m; ++c) M[r * ld + c] -= f * M[k * ld + c];
    }
  }
  return true;
}

// fixed-order block sum of one value per thread (all threads call; result uniform)
__device__ __forceinline__ double pcg_block_sum(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += red[q];
  return s;
}

// sum of part[0 .. nblk) by one wave in a fixed order: kPcgRU loads per lane in flight per round, then the DPP tree
__device__ __forceinline__ double pcg_sum_vec(const double* part, int nblk, int lane) {
  double a = 0.0;
  for (int b0 = 0; b0 < nblk; b0 += 256) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld_part(part + min(b0 + lane + 64 * u, nblk - 1));
#pragma unroll
    for (int u = 0; u < 4; ++u) a += (b0 + lane + 64 * u < nblk) ? v[u] : 0.0;
  }
  return wave_sum_d(a);
}

// out[p] = sum_b part[b * stride + p] for p < ncol - 1 and *last = the sum of column ncol - 1, every column in the
// same fixed order (lane-strided partial sums over the blocks, then the wave's DPP tree).  A wave takes kPcgCB
// columns at a time with all their loads in flight (kPcgRU per lane and column), so the ~27 k cross-block partials
// of an 8-camera rig arrive in a couple of memory round trips instead of nblk / 16 dependent rounds of one thread
// per column.
constexpr int kPcgCB = 14, kPcgRU = 4;
__device__ __forceinline__ void pcg_sum_columns(const double* part, int stride, int ncol, int nblk, double* out,
                                                double* last) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int p0 = wave * kPcgCB; p0 < ncol; p0 += nw * kPcgCB) {
    double acc[kPcgCB];
#pragma unroll
    for (int c = 0; c < kPcgCB; ++c) acc[c] = 0.0;
    for (int b0 = 0; b0 < nblk; b0 += 64 * kPcgRU) {
      double v[kPcgCB][kPcgRU];
#pragma unroll
      for (int c = 0; c < kPcgCB; ++c)
#pragma unroll
        for (int u = 0; u < kPcgRU; ++u) {
          const int b = min(b0 + lane + 64 * u, nblk - 1), p = min(p0 + c, ncol - 1);
          v[c][u] = ld_part(part + (size_t)b * stride + p);
        }
#pragma unroll
      for (int c = 0; c < kPcgCB; ++c)
#pragma unroll
        for (int u = 0; u < kPcgRU; ++u) acc[c] += (b0 + lane + 64 * u < nblk) ? v[c][u] : 0.0;
    }
#pragma unroll
    for (int c = 0; c < kPcgCB; ++c) {
      const double s = wave_sum_d(acc[c]);
      const int p = p0 + c;
      if (lane == 0 && p < ncol) {
        if (p < ncol - 1) out[p] = s;
        else *last = s;
      }
    }
  }
}

__global__ void __launch_bounds__(kPcgThreads) k_pcg(KbDev d, KbPcg P) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ double red[kPcgThreads / 64];
  __shared__ int flag;
  __shared__ double sh_scalar[4];
  const int C = d.C, F = d.F, tid = threadIdx.x, b = blockIdx.x, fpb = P.fpb, nblk = P.nblk;
  const int f0 = b * fpb, nf = max(0, min(F, f0 + fpb) - f0), R = 6 * fpb, nr = 6 * nf;
  const int CP = C + 1;
  // LDS carve-up
  double* Hfc = sm;                  // [R][C]
  double* Hff = Hfc + (size_t)R * C; // [fpb][36] (+ lambda^2 on the diagonal)
  double* Mf = Hff + 36 * fpb;       // [fpb][2][9] frame DV block inverses
  double* xf = Mf + 18 * fpb;        // [R] x, r, d, s, q of the block's frames
  double* rf = xf + R;
  double* df = rf + R;
  double* sf = df + R;
  double* qf = sf + R;
  double* Mc = qf + R;               // [C][6] row p of the inverse of p's camera DV block
  double* xc = Mc + 6 * C;           // [C] x, r, d, s, q camera entries
  double* rc = xc + C;
  double* dc = rc + C;
  double* sc = dc + C;
  double* qc = sc + C;
  const int nrow = (C + nblk - 1) / nblk;  // camera rows p = b + k nblk of H_cc owned by this block
  double* Hcr = qc + C;                    // [nrow][C] those rows (+ lambda^2 on the diagonal)
  int* cbs = reinterpret_cast<int*>(Hcr + (size_t)nrow * C);  // [C]
  int* cbm = cbs + C;                          // [C]
  if (tid == 0) {
    flag = 0;
    sh_scalar[0] = 1.0;  // ok
  }
  const double lam2 = P.lam2;
  // ---- load the block's system, right-hand side
  for (int q = tid; q < nr * C; q += blockDim.x) Hfc[q] = d.Hfc[(size_t)f0 * 6 * C + q];
  for (int q = tid; q < 36 * nf; q += blockDim.x) {
    const int e = q % 36;
    const double v = d.Hff[(size_t)f0 * 36 + q];
    Hff[q] = (e / 6 == e % 6) ? v + lam2 : v;
  }
  for (int q = tid; q < R; q += blockDim.x) {
    rf[q] = q < nr ? d.gf[(size_t)f0 * 6 + q] : 0.0;
    xf[q] = 0.0;
  }
  for (int q = tid; q < nrow * C; q += blockDim.x) {
    const int k = q / C, c = q % C, p = b + k * nblk;
    Hcr[q] = p < C ? d.Hcc[(size_t)p * C + c] + (c == p ? lam2 : 0.0) : 0.0;
  }
  for (int p = tid; p < C; p += blockDim.x) {
    rc[p] = d.gc[p];
    xc[p] = 0.0;
    cbs[p] = P.cb_start[p];
    cbm[p] = P.cb_size[p];
  }
  __syncthreads();
  // ---- preconditioner: inverses of the diagonal DV blocks (camera blocks redundantly in every block)
  for (int q = tid; q < 2 * nf; q += blockDim.x) {
    const int fl = q >> 1, dv = q & 1;
    double* M = Mf + 18 * fl + 9 * dv;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) M[r * 3 + c] = Hff[36 * fl + (3 * dv + r) * 6 + 3 * dv + c];
    if (!pcg_block_inverse(M, 3, 3)) sh_scalar[0] = 0.0;
  }
  for (int p = tid; p < C; p += blockDim.x) {
    if (cbs[p] != p) continue;  // one thread per camera DV block (its first column)
    const int m = cbm[p];
    double* M = Mc + p * 6;  // rows p .. p + m - 1 of Mc, inverted in place (stride 6)
    for (int r = 0; r < m; ++r)
      for (int c = 0; c < 6; ++c) M[r * 6 + c] = c < m ? d.Hcc[(size_t)(p + r) * C + p + c] + (r == c ? lam2 : 0.0) : 0.0;
    if (!pcg_block_inverse(M, m, 6)) sh_scalar[0] = 0.0;
  }
  __syncthreads();
  // s = M^-1 r (frame rows and camera entries of this block)
  auto precond = [&]() {
    for (int t = tid; t < nr; t += blockDim.x) {
      const int fl = t / 6, a = t % 6, dv = a / 3;
      const double* M = Mf + 18 * fl + 9 * dv + 3 * (a % 3);
      const double* rr = rf + 6 * fl + 3 * dv;
      sf[t] = M[0] * rr[0] + M[1] * rr[1] + M[2] * rr[2];
    }
    for (int p = tid; p < C; p += blockDim.x) {
      const int s0 = cbs[p], m = cbm[p];
      double v = 0.0;
      for (int k = 0; k < m; ++k) v += Mc[p * 6 + k] * rc[s0 + k];
      sc[p] = v;
    }
  };
  unsigned nbar = 0;
  precond();
  __syncthreads();
  for (int t = tid; t < R; t += blockDim.x) df[t] = t < nr ? sf[t] : 0.0;
  for (int p = tid; p < C; p += blockDim.x) dc[p] = sc[p];
  {
    double v = 0.0;
    for (int t = tid; t < nr; t += blockDim.x) v += rf[t] * sf[t];
    v = pcg_block_sum(v, red);
    if (tid == 0) P.part2[b] = v;
  }
  if (!pcg_barrier(P.bar, nblk, ++nbar, &flag)) goto timeout;
  double dn, d0;
  {
    // dn = sum_b (r_f.s_f)_b + r_c.s_c, fixed order in every block
    double v = 0.0;
    if (tid < 64) {
      v = pcg_sum_vec(P.part2, nblk, tid);
      double c = 0.0;
      for (int p = tid; p < C; p += 64) c += rc[p] * sc[p];
      c = wave_sum_d(c);
      if (tid == 0) sh_scalar[1] = v + c;
    }
    __syncthreads();
    dn = sh_scalar[1];
    d0 = P.tol * dn;
    if (P.abs_tol && P.prev_residual > 0.0 && P.prev_residual > d0) d0 = P.prev_residual;
  }
  {
    const int max_it = P.max_it;
    // a singular DV block (camera blocks: the same in every block; frame blocks: local) poisons this block's
    // d.q partial, so every block sees a non-finite d.q in the first iteration and stops with ok = false
    bool ok = sh_scalar[0] != 0.0;
    int it = 0;
    for (it = 0; it < max_it; ++it) {
      if (dn <= d0) break;
      const int tsb = 200 + 6 * it;
      if (it < 8) KB_PCG_TS(tsb);
      // ---- phase A: q_f, camera partials, d_f.q_f
      double dq_part = 0.0;
      for (int t = tid; t < nr; t += blockDim.x) {
        const int fl = t / 6, a = t % 6;
        const double* hf = Hff + 36 * fl + 6 * a;
        const double* dd = df + 6 * fl;
        double v = hf[0] * dd[0] + hf[1] * dd[1] + hf[2] * dd[2] + hf[3] * dd[3] + hf[4] * dd[4] + hf[5] * dd[5];
        const double* hc = Hfc + (size_t)t * C;
        double w0 = 0.0, w1 = 0.0;
        int c = 0;
        for (; c + 2 <= C; c += 2) {
          w0 += hc[c] * dc[c];
          w1 += hc[c + 1] * dc[c + 1];
        }
        if (c < C) w0 += hc[c] * dc[c];
        v += w0 + w1;
        qf[t] = v;
        dq_part += dd[a] * v;
      }
      for (int p = tid; p < C; p += blockDim.x) {
        double v = 0.0;
        for (int t = 0; t < nr; ++t) v += Hfc[(size_t)t * C + p] * df[t];
        if (p % nblk == b) {
          const double* hr = Hcr + (size_t)(p / nblk) * C;
          double w0 = 0.0, w1 = 0.0;
          int c = 0;
          for (; c + 2 <= C; c += 2) {
            w0 += hr[c] * dc[c];
            w1 += hr[c + 1] * dc[c + 1];
          }
          if (c < C) w0 += hr[c] * dc[c];
          v += w0 + w1;
        }
        P.part[(size_t)b * CP + p] = v;
      }
      dq_part = pcg_block_sum(dq_part, red);
      if (tid == 0) P.part[(size_t)b * CP + C] = ok ? dq_part : NAN;  // a failed block poisons d.q
      if (it < 8) KB_PCG_TS(tsb + 1);
      if (!pcg_barrier(P.bar, nblk, ++nbar, &flag)) goto timeout;
      if (it < 8) KB_PCG_TS(tsb + 2);
      // ---- phase B: q_c, alpha, updates, s = M^-1 r, partial r_f.s_f
      pcg_sum_columns(P.part, CP, C + 1, nblk, qc, &sh_scalar[2]);
      __syncthreads();
      if (it < 8) KB_PCG_TS(tsb + 3);
      if (tid < 64) {
        double c = 0.0;
        for (int p = tid; p < C; p += 64) c += dc[p] * qc[p];
        c = wave_sum_d(c);
        if (tid == 0) sh_scalar[3] = sh_scalar[2] + c;
      }
      __syncthreads();
      const double dq = sh_scalar[3];
      if (!(dq > 0.0) || !isfinite(dq)) {  // breakdown (uniform: every block holds the same dq)
        ok = false;
        break;
      }
      const double alpha = dn / dq;
      for (int t = tid; t < nr; t += blockDim.x) {
        xf[t] += alpha * df[t];
        rf[t] -= alpha * qf[t];
      }
      for (int p = tid; p < C; p += blockDim.x) {
        xc[p] += alpha * dc[p];
        rc[p] -= alpha * qc[p];
      }
      __syncthreads();
      precond();
      __syncthreads();
      {
        double v = 0.0;
        for (int t = tid; t < nr; t += blockDim.x) v += rf[t] * sf[t];
        v = pcg_block_sum(v, red);
        if (tid == 0) P.part2[b] = v;
      }
      if (it < 8) KB_PCG_TS(tsb + 4);
      if (!pcg_barrier(P.bar, nblk, ++nbar, &flag)) goto timeout;
      if (it < 8) KB_PCG_TS(tsb + 5);
      // ---- phase C: dn', beta, d = s + beta d
      if (tid < 64) {
        double v = 0.0;
        v = pcg_sum_vec(P.part2, nblk, tid);
        double c = 0.0;
        for (int p = tid; p < C; p += 64) c += rc[p] * sc[p];
        c = wave_sum_d(c);
        if (tid == 0) sh_scalar[1] = v + c;
      }
      __syncthreads();
      const double dnew = sh_scalar[1];
      const double beta = dnew / dn;
      dn = dnew;
      for (int t = tid; t < nr; t += blockDim.x) df[t] = sf[t] + beta * df[t];
      for (int p = tid; p < C; p += blockDim.x) dc[p] = sc[p] + beta * dc[p];
      __syncthreads();
    }
    // ---- results: x (canonical column order [camera | frames]), info
    for (int t = tid; t < nr; t += blockDim.x) d.dx[C + 6 * f0 + t] = xf[t];
    if (b == 0) {
      for (int p = tid; p < C; p += blockDim.x) d.dx[p] = xc[p];
      if (tid == 0) {
        P.info[0] = it;
        P.info[1] = 0.5 * dn;
        P.info[2] = d0;
        P.info[3] = ok ? 1.0 : 0.0;
      }
    }
    return;
  }
timeout:
  if (tid == 0) P.info[4] = 1.0;  // barrier spin limit hit (the host zeroes info[4] before the launch)
}

}  // namespace kb
