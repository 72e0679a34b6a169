// Microbenchmark: the tiled camera-block LDL^T of k_solve<0> (ldl_panels + panel_backsolve, kb_kernels.hip) alone on
// one CU, on a random SPD 106 x 106 system staged in LDS exactly as k_solve stages it.  Timeline from the KB_TS stamps
// (s_memrealtime, 100 MHz) plus s_memtime cycles; checks the solution against a host Cholesky.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DKB_STAMPS -o camera_solve camera_solve.hip
#include "../../kalibr_amd/csrc/kb_kernels.hip"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace kb;

// bsv: the backsolve variant (1: panel_backsolve, 2: panel_backsolve2, 3: panel_backsolve3, the default)
__global__ void __launch_bounds__(512) k_cam(KbDev d, const double* img, int n_img, int C, double* x_out, int reps, int bsv) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int nb = (C + 16) >> 4;
  double* S = sm;
  double* Dfac = S + n_img;
  double* Xinv = Dfac + nb * kTileSz;
  double* rD = Xinv + nb * kTileSz;
  __shared__ int okl;
  __shared__ double pub[16];
  double x[2] = {0.0, 0.0};
  for (int rep = 0; rep < reps; ++rep) {
    for (int q = threadIdx.x; q < n_img; q += blockDim.x) S[q] = img[q];
    if (threadIdx.x == 0) okl = 1;
    __syncthreads();
    KB_TS(d, 0);
    ldl_panels(d, S, rD, Dfac, Xinv, C, nb, &okl);
    KB_TS(d, 4);
    if (threadIdx.x < 64) {
      if (bsv == 1) panel_backsolve(d, S, Dfac, Xinv, rD, C, nb, pub, x);
      else if (bsv == 2) panel_backsolve2(d, S, Dfac, Xinv, rD, C, nb, pub, x);
      else panel_backsolve3(d, S, Dfac, Xinv, rD, C, nb, x);
    }
    __syncthreads();
    KB_TS(d, 5);
  }
  if (threadIdx.x < 64) {
    x_out[threadIdx.x] = x[0];
    if (threadIdx.x + 64 < C) x_out[threadIdx.x + 64] = x[1];
    if (threadIdx.x == 0) x_out[127] = okl;
  }
}

int main() {
  const int C = 106, nb = (C + 16) / 16, n_img = kTileSz * nb * (nb + 1) / 2;
  // random SPD A = M M^T + C I, b
  std::vector<double> A(C * C), b(C);
  for (int i = 0; i < C; ++i) {
    for (int j = 0; j < C; ++j) {
      double s = 0.0;
      for (int k = 0; k < C; ++k) s += std::sin(0.37 * i + 1.1 * k + 0.1) * std::sin(0.37 * j + 1.1 * k + 0.1);
      A[i * C + j] = s + (i == j ? 2.0 : 0.0);
    }
    b[i] = std::cos(0.3 * i);
  }
  // tile image: lower tiles, identity padding, b as row C
  std::vector<double> img(n_img, 0.0);
  auto tix = [&](int i, int j) { return ((i / 16) * (i / 16 + 1) / 2 + j / 16) * kTileSz + (i % 16) * kTS + (j % 16); };
  for (int i = 0; i < 16 * nb; ++i)
    for (int j = 0; j <= i; ++j) {
      double v = 0.0;
      if (i < C) v = A[i * C + j];
      else if (i == C && j < C) v = b[j];
      else if (i == j) v = 1.0;
      img[tix(i, j)] = v;
      if (i / 16 == j / 16) img[tix(j, i)] = v;  // diagonal tiles whole (k_colimg's image)
    }
  // host solve (Cholesky)
  std::vector<double> L(A), xs(b);
  for (int k = 0; k < C; ++k) {
    L[k * C + k] = std::sqrt(L[k * C + k]);
    for (int i = k + 1; i < C; ++i) L[i * C + k] /= L[k * C + k];
    for (int j = k + 1; j < C; ++j)
      for (int i = j; i < C; ++i) L[i * C + j] -= L[i * C + k] * L[j * C + k];
  }
  for (int i = 0; i < C; ++i) {
    for (int k = 0; k < i; ++k) xs[i] -= L[i * C + k] * xs[k];
    xs[i] /= L[i * C + i];
  }
  for (int i = C - 1; i >= 0; --i) {
    for (int k = i + 1; k < C; ++k) xs[i] -= L[k * C + i] * xs[k];
    xs[i] /= L[i * C + i];
  }
  double *dimg, *dx;
  long long* ts;
  (void)hipMalloc(&dimg, n_img * 8);
  (void)hipMalloc(&dx, 128 * 8);
  (void)hipMalloc(&ts, 256 * 8);
  (void)hipMemcpy(dimg, img.data(), n_img * 8, hipMemcpyHostToDevice);
  (void)hipMemset(ts, 0, 256 * 8);
  KbDev d{};
  d.dbg_ts = ts;
  const size_t lds = 8 * (n_img + 2 * nb * kTileSz + 16 * nb);
  (void)hipFuncSetAttribute((const void*)k_cam, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int bsv : {1, 2, 3})
  for (int reps : {1, 3}) {
    hipLaunchKernelGGL(k_cam, dim3(1), dim3(512), lds, 0, d, dimg, n_img, C, dx, reps, bsv);
    (void)hipDeviceSynchronize();
    long long t[256];
    std::vector<double> x(128);
    (void)hipMemcpy(t, ts, 256 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(x.data(), dx, 128 * 8, hipMemcpyDeviceToHost);
    double err = 0.0, nx = 0.0;
    for (int i = 0; i < C; ++i) {
      err = std::fmax(err, std::fabs(x[i] - xs[i]));
      nx = std::fmax(nx, std::fabs(xs[i]));
    }
    std::printf("backsolve v%d, reps %d (last rep timed): ok %g, max|x - x_host| / max|x| = %.3g\n", bsv, reps, x[127], err / nx);
    std::printf("  factor start->end %.2f us, backsolve %.2f us\n", (t[4] - t[0]) / 100.0, (t[5] - t[4]) / 100.0);
    std::printf("  panel 2 detail: lookahead phase (panel 1 end -> factor start) %.2f, row loads %.2f, 16 steps %.2f, stores %.2f us\n",
                (t[24] - t[11]) / 100.0, (t[41] - t[24]) / 100.0, (t[42] - t[41]) / 100.0, (t[25] - t[42]) / 100.0);
    if (bsv == 3) {
      std::printf("  backsolve3 tile starts (us after factor end):");
      for (int q = nb - 1; q >= 0; --q) std::printf(" %d:%.2f", q, (t[240 + q] - t[4]) / 100.0);
      std::printf("\n");
    }
    for (int q = 0; q < nb; ++q)
      std::printf("  panel %d: factor %.2f us (start at %.2f), panel end at %.2f\n", q, (t[21 + 2 * q] - t[20 + 2 * q]) / 100.0,
                  (t[20 + 2 * q] - t[0]) / 100.0, (t[10 + q] - t[0]) / 100.0);
  }
  return 0;
}
