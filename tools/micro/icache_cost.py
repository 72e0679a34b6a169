"""Generates tools/micro/icache_cost.hip: cost of executing K KB of straight-line code in one wave, cold (after a
kernel that streams 512 MB through the caches) and warm (relaunched right away)."""
import os
HERE = os.path.dirname(os.path.abspath(__file__))
sizes = [4, 16, 32, 64]
src = ['#include <hip/hip_runtime.h>', '#include <cstdio>']
for kb in sizes:
    n = kb * 1024 // 8  # v_fma_f64 is 8 bytes
    body = "\n".join(f'    "v_fma_f64 v[0:1], v[2:3], v[4:5], v[0:1]\\n"' for _ in range(n // 8))
    src.append(f'''__global__ void k_code{kb}(double* out, long long* cyc) {{
  double a = out[threadIdx.x];
  long long t0 = __builtin_readcyclecounter();
  for (int r = 0; r < 8; ++r)
  asm volatile(
{body}
    : : : "v0", "v1", "v2", "v3", "v4", "v5");
  long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = a;
}}''')
src.append('''__global__ void k_thrash(const double4* in, double* out, size_t n) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += in[i].x;
  if (s == 1.2345) out[0] = s;
}
template <class K>
void run(K k, const char* name, double* out, long long* cyc, const double4* big, size_t nbig) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode) {
    long long best = 0; float tms = 0;
    for (int rep = 0; rep < 5; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(k_thrash, dim3(4096), dim3(256), 0, 0, big, out, nbig);
      else hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      long long c = 0; hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      float ms = 0; hipEventElapsedTime(&ms, e0, e1);
      best += c; tms += ms;
    }
    printf("%s %s: %.0f cycles in-kernel (8 passes over the code), %.2f us per launch (events)\\n", name,
           mode == 0 ? "cold (after 512 MB stream)" : "warm", best / 5.0, 1e3 * tms / 5);
  }
}
int main() {
  double* out; long long* cyc; double4* big;
  const size_t nbig = (512ull << 20) / sizeof(double4);
  (void)hipMalloc(&out, 4096); (void)hipMalloc(&cyc, 64); (void)hipMalloc(&big, nbig * sizeof(double4));
  (void)hipMemset(big, 0, nbig * sizeof(double4)); (void)hipMemset(out, 0, 4096);
''')
for kb in sizes:
    src.append(f'  run(k_code{kb}, "{kb} KB", out, cyc, big, nbig);')
src.append('  return 0;\n}')
open(os.path.join(HERE, "icache_cost.hip"), "w").write("\n".join(src) + "\n")
