// Microbenchmark / layout probe for v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4): for every pair (la, lb) of lanes a wave
// runs one MFMA with A = one-hot(la), B = one-hot(lb), C = 0 and records which output lanes become 1.  The host prints
// the derived operand layout (block, row i, k of A; block, k, column j of B; block, i, j of D) and the issue rate of
// the 4x4x4 and 16x16x4 shapes with 1..4 independent accumulators.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void k_probe(unsigned long long* out) {
  const int w = blockIdx.x, lane = threadIdx.x;  // one wave per (la, lb)
  const int la = w / 64, lb = w % 64;
  double a = lane == la ? 1.0 : 0.0, b = lane == lb ? 1.0 : 0.0;
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  const unsigned long long m = __ballot(d != 0.0);
  if (lane == 0) out[w] = m;
}

template <int SHAPE, int NACC>
__global__ void k_rate(double* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
  long long t0 = __builtin_readcyclecounter();
  if constexpr (SHAPE == 16) {
    v4d c[NACC];
    for (int q = 0; q < NACC; ++q) c[q] = v4d{0, 0, 0, 0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[q], 0, 0, 0);
    }
    long long t1 = __builtin_readcyclecounter();
    double s = 0;
    for (int q = 0; q < NACC; ++q) s += c[q][q & 3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
  } else {
    double c[NACC];
    for (int q = 0; q < NACC; ++q) c[q] = 0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[q], 0, 0, 0);
    }
    long long t1 = __builtin_readcyclecounter();
    double s = 0;
    for (int q = 0; q < NACC; ++q) s += c[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
  }
}

template <int SHAPE, int NACC>
void rate(const char* name) {
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * 64);
  hipMalloc(&cyc, sizeof(long long));
  const int iters = 2000;
  k_rate<SHAPE, NACC><<<1, 64>>>(out, cyc, 10);
  k_rate<SHAPE, NACC><<<1, 64>>>(out, cyc, iters);
  long long c = 0;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%s, %d accumulators: %.2f cycles/inst (one wave)\n", name, NACC, (double)c / (8.0 * NACC * iters));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * 4096);
  hipLaunchKernelGGL(k_probe, dim3(4096), dim3(64), 0, 0, d);
  std::vector<unsigned long long> h(4096);
  hipMemcpy(h.data(), d, sizeof(unsigned long long) * 4096, hipMemcpyDeviceToHost);
  // for each output lane: the (la, lb) pairs feeding it
  for (int o = 0; o < 64; ++o) {
    printf("D lane %2d <-", o);
    for (int w = 0; w < 4096; ++w)
      if ((h[w] >> o) & 1ull) printf(" (%d,%d)", w / 64, w % 64);
    printf("\n");
  }
  rate<4, 1>("v_mfma_f64_4x4x4f64");
  rate<4, 2>("v_mfma_f64_4x4x4f64");
  rate<4, 4>("v_mfma_f64_4x4x4f64");
  rate<4, 8>("v_mfma_f64_4x4x4f64");
  rate<16, 1>("v_mfma_f64_16x16x4f64");
  rate<16, 2>("v_mfma_f64_16x16x4f64");
  rate<16, 4>("v_mfma_f64_16x16x4f64");
  return 0;
}
