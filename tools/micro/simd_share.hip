// Microbenchmark: how a dependent FP64 VALU chain (the k_buildp frame waves' elimination) runs while another wave on
// the same SIMD issues FP64 MFMA (the view waves' SYRK).  One block of 8 waves: waves w and w + 4 share a SIMD.
// Waves 0..3 time a probe with s_memtime; waves 4..7 run the load.  Modes: probe {dependent f64 FMA chain,
// 8 independent f64 chains, dependent f32 chain} x load {none, f64 MFMA 16x16x4, f64 VALU, LDS reads}.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o simd_share simd_share.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) k_share(int probe, int load, double* out, long long* cyc, int n) {
  __shared__ double lds[4096];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int q = threadIdx.x; q < 4096; q += 512) lds[q] = q * 1e-3;
  __syncthreads();
  double r = 0.0;
  if (w < 4) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (probe == 0) {
      double x = 1.0 + lane * 1e-6;
      for (int i = 0; i < n; ++i) x = fma(x, 0.999999, 1e-7);
      r = x;
    } else if (probe == 1) {
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = 1.0 + (lane + u) * 1e-6;
      for (int i = 0; i < n / 8; ++i)
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = fma(x[u], 0.999999, 1e-7);
#pragma unroll
      for (int u = 0; u < 8; ++u) r += x[u];
    } else {
      float x = 1.0f + lane * 1e-6f;
      for (int i = 0; i < n; ++i) x = fmaf(x, 0.999999f, 1e-7f);
      r = x;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[w] = t1 - t0;
  } else if (load == 1) {
    const double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < 4 * n / 64; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    r = c0[0] + c1[1] + c2[2] + c3[3];
  } else if (load == 2) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = 1.0 + (lane + u) * 1e-6;
    for (int i = 0; i < 4 * n / 8; ++i)
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = fma(x[u], 0.999999, 1e-7);
#pragma unroll
    for (int u = 0; u < 8; ++u) r += x[u];
  } else if (load == 3) {
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
  (void)hipMalloc(&cyc, 8 * 8);
  const char* pn[3] = {"dependent f64 FMA chain", "8 independent f64 FMA chains", "dependent f32 FMA chain"};
  const char* ln[4] = {"alone", "+ f64 MFMA wave", "+ f64 VALU wave", "+ LDS-read wave"};
  const int n = 4096;
  for (int p = 0; p < 3; ++p)
    for (int l = 0; l < 4; ++l) {
      hipLaunchKernelGGL(k_share, dim3(1), dim3(512), 0, 0, p, l, out, cyc, 64);
      hipLaunchKernelGGL(k_share, dim3(1), dim3(512), 0, 0, p, l, out, cyc, n);
      (void)hipDeviceSynchronize();
      long long c[8];
      (void)hipMemcpy(c, cyc, 8 * 8, hipMemcpyDeviceToHost);
      double m = 0;
      for (int w = 0; w < 4; ++w) m += c[w];
      std::printf("%-30s %-18s %6.2f cycles per FMA (s_memtime)\n", pn[p], ln[l], m / 4 / n);
    }
  return 0;
}
