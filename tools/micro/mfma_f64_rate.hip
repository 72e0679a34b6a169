// Microbenchmark: issue rate of the two FP64 MFMA shapes on one SIMD (one wave, 4 independent accumulators),
// cycles per instruction from s_memtime around an unrolled loop.  Also the FLOP rate of a full-chip launch.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ void k_rate(double* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
  long long t0 = __builtin_readcyclecounter();
  if constexpr (SHAPE == 16) {
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
      }
    }
    long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
  } else {
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
      }
    }
    long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
  }
}

template <int SHAPE>
void run(const char* name, int flops_per_inst) {
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * 1024 * 4096);
  hipMalloc(&cyc, sizeof(long long));
  const int iters = 2000;
  k_rate<SHAPE><<<1, 64>>>(out, cyc, 10);
  k_rate<SHAPE><<<1, 64>>>(out, cyc, iters);
  long long c = 0;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  const double insts = 32.0 * iters;
  // full chip: 4 waves per CU x 256 CUs x 4 (one per SIMD)
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_rate<SHAPE><<<1024, 256>>>(out, cyc, 100);
  hipEventRecord(e0);
  k_rate<SHAPE><<<1024, 256>>>(out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 1024.0 * 4 * insts * flops_per_inst;
  printf("%s: %.2f cycles/inst (one wave), chip %.1f TFLOP/s\n", name, (double)c / insts, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<16>("v_mfma_f64_16x16x4f64", 16 * 16 * 4 * 2);
  run<4>("v_mfma_f64_4x4x4f64 (4 blocks)", 4 * 4 * 4 * 2 * 4);
  return 0;
}
