// Microbenchmark: how VALU work (the k_buildp frame waves' elimination, the view waves' projections) runs while
// another wave on the same SIMD issues FP64 MFMA (the view waves' SYRK).  One block of 8 waves: waves w and w + 4
// share a SIMD.  Waves 0..3 time a probe with s_memtime (shader clock); waves 4..7 run the load.
//   probes: 0 dependent f64 FMA chain, 1 eight independent f64 FMA chains, 2 dependent f32 FMA chain,
//           3 independent f32 chains (all unrolled x16 per loop trip);
//   loads:  0 none, 1 f64 MFMA 16x16x4 (accumulators in VGPRs), 2 the same with AGPR accumulators (inline asm),
//           3 f64 VALU (independent chains), 4 LDS reads.
// Also the MFMA issue rate of one wave alone (cycles per v_mfma_f64_16x16x4f64, VGPR and AGPR accumulators).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o simd_share simd_share.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma_agpr(v4d& c, double a, double b) {
  asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <int load>
__global__ void __launch_bounds__(512) k_share(int probe, double* out, long long* cyc, int n) {
  __shared__ double lds[4096];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int q = threadIdx.x; q < 4096; q += 512) lds[q] = q * 1e-3;
  __syncthreads();
  double r = 0.0;
  if (w < 4) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (probe == 0) {
      double x = 1.0 + lane * 1e-6;
      for (int i = 0; i < n / 16; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) x = fma(x, 0.999999, 1e-7);
      r = x;
    } else if (probe == 1) {
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = 1.0 + (lane + u) * 1e-6;
      for (int i = 0; i < n / 16; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u & 7] = fma(x[u & 7], 0.999999, 1e-7);
#pragma unroll
      for (int u = 0; u < 8; ++u) r += x[u];
    } else if (probe == 2) {
      float x = 1.0f + lane * 1e-6f;
      for (int i = 0; i < n / 16; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) x = fmaf(x, 0.999999f, 1e-7f);
      r = x;
    } else {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = 1.0f + (lane + u) * 1e-6f;
      for (int i = 0; i < n / 16; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u & 7] = fmaf(x[u & 7], 0.999999f, 1e-7f);
#pragma unroll
      for (int u = 0; u < 8; ++u) r += x[u];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[w] = t1 - t0;
  } else if constexpr (load == 1 || load == 2) {
    const double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    const int m = n / 8;  // MFMAs per accumulator: about 4x the probe's length
    for (int i = 0; i < m / 4; ++i) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (load == 1) {
          c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
          c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
          c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        } else {
          mfma_agpr(c0, a, b);
          mfma_agpr(c1, a, b);
          mfma_agpr(c2, a, b);
          mfma_agpr(c3, a, b);
        }
      }
    }
    r = c0[0] + c1[1] + c2[2] + c3[3];
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[w] = t1 - t0;
    if (lane == 0) cyc[8 + w] = 4 * m;  // MFMAs issued
  } else if constexpr (load == 3) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = 1.0 + (lane + u) * 1e-6;
    for (int i = 0; i < 4 * n / 16; ++i)
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u & 7] = fma(x[u & 7], 0.999999, 1e-7);
#pragma unroll
    for (int u = 0; u < 8; ++u) r += x[u];
  } else if constexpr (load == 4) {
    for (int i = 0; i < 4 * n / 8; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u) r += lds[(lane * 17 + i * 8 + u) & 4095];
    }
  }
  out[threadIdx.x] = r;
}

int main() {
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, 512 * 8);
  (void)hipMalloc(&cyc, 16 * 8);
  const char* pn[4] = {"dependent f64 FMA chain", "8 independent f64 chains", "dependent f32 FMA chain",
                       "8 independent f32 chains"};
  const char* ln[5] = {"alone", "+ f64 MFMA (VGPR acc)", "+ f64 MFMA (AGPR acc)", "+ f64 VALU wave", "+ LDS-read wave"};
  const int n = 8192;
  for (int p = 0; p < 4; ++p)
    for (int l = 0; l < 5; ++l) {
      (void)hipMemset(cyc, 0, 16 * 8);
      for (int nn : {64, n}) {
        if (l == 0) hipLaunchKernelGGL(k_share<0>, dim3(1), dim3(512), 0, 0, p, out, cyc, nn);
        if (l == 1) hipLaunchKernelGGL(k_share<1>, dim3(1), dim3(512), 0, 0, p, out, cyc, nn);
        if (l == 2) hipLaunchKernelGGL(k_share<2>, dim3(1), dim3(512), 0, 0, p, out, cyc, nn);
        if (l == 3) hipLaunchKernelGGL(k_share<3>, dim3(1), dim3(512), 0, 0, p, out, cyc, nn);
        if (l == 4) hipLaunchKernelGGL(k_share<4>, dim3(1), dim3(512), 0, 0, p, out, cyc, nn);
      }
      (void)hipDeviceSynchronize();
      long long c[16];
      (void)hipMemcpy(c, cyc, 16 * 8, hipMemcpyDeviceToHost);
      double m = 0;
      for (int w = 0; w < 4; ++w) m += c[w];
      std::printf("%-26s %-24s %6.2f cycles per FMA", pn[p], ln[l], m / 4 / n);
      if (l == 1 || l == 2) std::printf("   (MFMA wave: %.2f cycles per MFMA)", (double)c[4] / c[12]);
      std::printf("\n");
    }
  return 0;
}
