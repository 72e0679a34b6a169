// Semantics check of the cross-lane operations the camera solve relies on (gfx950): v_fmac_f64_dpp with
// row_newbcast (64-bit DPP fused into the FMA) and __builtin_amdgcn_permlane16_swap / permlane32_swap.
// Prints, per lane, what each op produced, and "OK"/"MISMATCH" against the expected formulas.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int L>
__device__ __forceinline__ void fmac_bc(double& x, double y, double f) {
  asm volatile("s_nop 1\n v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(x) : "v"(y), "v"(f), "i"(L));
}

__global__ void k(double* out, unsigned* pout) {
  const int l = threadIdx.x;
  double x = 1000.0 * l, y = (double)l, f = 2.0;
  fmac_bc<5>(x, y, f);  // x = 1000 l + 2 * y[16 (l/16) + 5]
  out[l] = x;
  double z = 3.0 * l;
  fmac_bc<9>(z, z, 1.0);  // z = 3 l + 3 (16 (l/16) + 9)
  out[64 + l] = z;
  const unsigned v = 100u * l;
  auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  pout[4 * l + 0] = p16[0];
  pout[4 * l + 1] = p16[1];
  pout[4 * l + 2] = p32[0];
  pout[4 * l + 3] = p32[1];
}

int main() {
  double* d;
  unsigned* p;
  hipMalloc(&d, 128 * sizeof(double));
  hipMalloc(&p, 256 * sizeof(unsigned));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, p);
  double h[128];
  unsigned hp[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  hipMemcpy(hp, p, sizeof(hp), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const double ex = 1000.0 * l + 2.0 * (16 * (l / 16) + 5), ez = 3.0 * l + 3.0 * (16 * (l / 16) + 9);
    if (h[l] != ex || h[64 + l] != ez) ++bad;
  }
  printf("fmac_f64_dpp row_newbcast: %s\n", bad ? "MISMATCH" : "OK");
  for (int l = 0; l < 64; l += 8)
    printf("lane %2d: p16 = (%u, %u)  p32 = (%u, %u)\n", l, hp[4 * l] / 100, hp[4 * l + 1] / 100, hp[4 * l + 2] / 100,
           hp[4 * l + 3] / 100);
  return bad ? 1 : 0;
}
