// Microbenchmark: the 16-column panel LDL^T of the camera solve (lane = matrix row, 16 diagonal rows + 48 rows
// below), one wave alone on a CU, cycles from s_memtime.  Variants of the broadcast of the pivot row:
//   0  v_readlane (the k_solve<0> panel_factor of round 3)
//   1  diagonal tile by DPP row_newbcast (lanes 0..15), then the 48 rows solved against it with the Ltilde entries
//      read from LDS as wave-uniform broadcasts
//   2  per step the pivot lane publishes its trailing row in LDS, every lane reads it back (ds_read_b128)
//   3  every lane factors the diagonal tile redundantly (entries read as LDS broadcasts), then its own row
// plus dependent-chain latencies: FMA -> v_readlane -> FMA, FMA -> DPP -> FMA, FMA -> LDS -> FMA.
// Build: hipcc --offload-arch=gfx950 -O3 -o panel_factor panel_factor.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffull), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffull), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int K>
__device__ __forceinline__ double bc16(double v) { return dpp_d<0x150 + K>(v); }
__device__ __forceinline__ double bcast16(double v, int k) {
  switch (k) {
    case 0: return bc16<0>(v); case 1: return bc16<1>(v); case 2: return bc16<2>(v); case 3: return bc16<3>(v);
    case 4: return bc16<4>(v); case 5: return bc16<5>(v); case 6: return bc16<6>(v); case 7: return bc16<7>(v);
    case 8: return bc16<8>(v); case 9: return bc16<9>(v); case 10: return bc16<10>(v); case 11: return bc16<11>(v);
    case 12: return bc16<12>(v); case 13: return bc16<13>(v); case 14: return bc16<14>(v); default: return bc16<15>(v);
  }
}
__device__ __forceinline__ double recip_d(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
#define WSYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
// s_memtime ordered after every instruction issued before it that produced v (asm input), and before what follows
__device__ __forceinline__ long long clk() {
  long long t;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
#define DEP(x) asm volatile("v_mov_b64 %0, %0" : "+v"(x))

// in: 64 x 16 row-major (rows 0..15 the symmetric diagonal tile), out: factored rows
template <int V>
__global__ void k_panel(const double* in, double* out, long long* cyc, int reps) {
  __shared__ double sh[64 * 17];
  __shared__ double pub[32];
  const int lane = threadIdx.x;
  double row[16];
  long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
    for (int c = 0; c < 16; ++c) row[c] = in[lane * 16 + c];
#pragma unroll
    for (int c = 0; c < 16; ++c) sh[lane * 17 + c] = row[c];
    WSYNC();
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int c = 0; c < 16; ++c) DEP(row[c]);
    t0 = clk();
    double rd = 1.0;
    if constexpr (V == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const double Dk = readlane_d(row[k], k);
        const double rdk = recip_d(Dk);
        rd = lane == k ? rdk : rd;
        const double f = lane > k ? row[k] * rdk : 0.0;
#pragma unroll
        for (int j = k + 1; j < 16; ++j) row[j] -= f * readlane_d(row[j], k);
      }
    } else if constexpr (V == 1) {
      if (lane < 16) {  // diagonal LDL^T by DPP
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const double Dk = bcast16(row[k], k);
          const double rdk = recip_d(Dk);
          rd = lane == k ? rdk : rd;
          const double f = lane > k ? row[k] * rdk : 0.0;
#pragma unroll
          for (int j = k + 1; j < 16; ++j) row[j] -= f * bcast16(row[j], k);
        }
        // Ltilde (scaled) into LDS, 1/D into pub
#pragma unroll
        for (int c = 0; c < 16; ++c) sh[lane * 17 + c] = row[c] * bcast16(rd, c);
        pub[lane] = rd;
      }
      WSYNC();
      __builtin_amdgcn_s_barrier();  // one wave: orders the LDS writes for the other lanes
      if (lane >= 16) {  // w[c] = s[c] - sum_{c2 < c} w[c2] Ltilde[c][c2]; row = w
#pragma unroll
        for (int c2 = 0; c2 < 15; ++c2)
#pragma unroll
          for (int c = c2 + 1; c < 16; ++c) row[c] -= row[c2] * sh[c * 17 + c2];
      }
    } else if constexpr (V == 2) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (lane == k)
#pragma unroll
          for (int j = k; j < 16; ++j) pub[j] = row[j];
        WSYNC();
        const double Dk = pub[k];
        const double rdk = recip_d(Dk);
        rd = lane == k ? rdk : rd;
        const double f = lane > k ? row[k] * rdk : 0.0;
#pragma unroll
        for (int j = k + 1; j < 16; ++j) row[j] -= f * pub[j];
        WSYNC();
      }
    } else if constexpr (V == 3) {
      // redundant diagonal factor in every lane: L (strictly lower, scaled) + 1/D, from LDS broadcasts
      double L[120];  // packed lower of the trailing matrix
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) L[i * (i + 1) / 2 + j] = sh[i * 17 + j];
      double rdv[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        rdv[k] = recip_d(L[k * (k + 1) / 2 + k]);
#pragma unroll
        for (int i = k + 1; i < 16; ++i) {
          const double f = L[i * (i + 1) / 2 + k] * rdv[k];
#pragma unroll
          for (int j = k + 1; j <= i; ++j) L[i * (i + 1) / 2 + j] -= f * L[j * (j + 1) / 2 + k];
        }
      }
      // own row: w[c] = s[c] - sum_{c2 < c} w[c2] Ltilde[c][c2] (lanes >= 16); diag lanes take their row of L D
#pragma unroll
      for (int c2 = 0; c2 < 15; ++c2)
#pragma unroll
        for (int c = c2 + 1; c < 16; ++c) row[c] -= row[c2] * (L[c * (c + 1) / 2 + c2] * rdv[c2]);
      rd = rdv[lane & 15];
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) DEP(row[c]);
    DEP(rd);
    t1 = clk();
    row[0] += rd * 1e-300;
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) out[lane * 16 + c] = row[c];
  if (lane == 0) cyc[V] = t1 - t0;
}

// dependent chains: 64 steps x = fma(bcast(x), a, x)
template <int V>
__global__ void k_chain(double* io, long long* cyc) {
  __shared__ double pub[64];
  const int lane = threadIdx.x;
  double x = io[lane], a = 1e-3 * (lane + 1);
  __builtin_amdgcn_s_barrier();
  DEP(x);
  const long long t0 = clk();
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    double b;
    if constexpr (V == 0) b = readlane_d(x, k);
    else if constexpr (V == 1) b = bcast16(x, k & 15);
    else if constexpr (V == 2) {
      if (lane == k) pub[0] = x;
      WSYNC();
      b = pub[0];
    } else b = x;
    x = fma(b, a, x);
  }
  DEP(x);
  const long long t1 = clk();
  io[lane] = x;
  if (lane == 0) cyc[V] = t1 - t0;
}

// tick rate of s_memtime against s_memrealtime (100 MHz) over a 20k-step dependent FMA chain
__global__ void k_calib(double* io, long long* out) {
  double x = io[threadIdx.x];
  long long r0, r1, m0, m1;
  asm volatile("s_waitcnt lgkmcnt(0)\n s_memrealtime %0\n s_memtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(r0), "=s"(m0) : : "memory");
  for (int i = 0; i < 20000; ++i) x = fma(x, 0.999999, 1e-9);
  DEP(x);
  asm volatile("s_waitcnt lgkmcnt(0)\n s_memrealtime %0\n s_memtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(r1), "=s"(m1) : : "memory");
  io[threadIdx.x] = x;
  if (threadIdx.x == 0) {
    out[0] = r1 - r0;
    out[1] = m1 - m0;
  }
}

int main() {
  std::vector<double> h(64 * 16);
  // a random SPD diagonal tile + random rows below
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 16; ++j) h[i * 16 + j] = std::sin(1.3 * i + 0.7 * j) * 0.1;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0.0;
      for (int k = 0; k < 16; ++k) s += std::sin(0.3 * i + k) * std::sin(0.3 * j + k);
      h[i * 16 + j] = s + (i == j ? 16.0 : 0.0);
    }
  double *din, *dout;
  long long* dc;
  hipMalloc(&din, 64 * 16 * 8);
  hipMalloc(&dout, 4 * 64 * 16 * 8);
  hipMalloc(&dc, 16 * 8);
  hipMemcpy(din, h.data(), 64 * 16 * 8, hipMemcpyHostToDevice);
  k_panel<0><<<1, 64>>>(din, dout, dc, 1);  // first execution of the code (cold instruction cache)
  hipDeviceSynchronize();
  long long cold = 0;
  hipMemcpy(&cold, dc, 8, hipMemcpyDeviceToHost);
  std::printf("panel readlane, first pass (cold code) %lld cycles\n", cold);
  k_panel<0><<<1, 64>>>(din, dout, dc, 3);
  k_panel<1><<<1, 64>>>(din, dout + 1024, dc, 3);
  k_panel<2><<<1, 64>>>(din, dout + 2048, dc, 3);
  k_panel<3><<<1, 64>>>(din, dout + 3072, dc, 3);
  hipDeviceSynchronize();
  long long c[16];
  hipMemcpy(c, dc, 16 * 8, hipMemcpyDeviceToHost);
  std::vector<double> o(4 * 1024);
  hipMemcpy(o.data(), dout, 4 * 1024 * 8, hipMemcpyDeviceToHost);
  const char* nm[4] = {"readlane", "diag DPP + LDS trsm", "LDS row publish", "redundant diag"};
  for (int v = 0; v < 4; ++v) {
    double md = 0.0;  // rows below (lanes >= 16) vs variant 0
    for (int q = 256; q < 1024; ++q) md = std::fmax(md, std::fabs(o[v * 1024 + q] - o[q]));
    std::printf("panel %-22s %6lld cycles  max|rows below - v0| %.3g\n", nm[v], c[v], md);
  }
  double* dio;
  hipMalloc(&dio, 64 * 8);
  hipMemcpy(dio, h.data(), 64 * 8, hipMemcpyHostToDevice);
  k_chain<0><<<1, 64>>>(dio, dc);
  k_chain<1><<<1, 64>>>(dio, dc);
  k_chain<2><<<1, 64>>>(dio, dc);
  k_chain<3><<<1, 64>>>(dio, dc);
  hipDeviceSynchronize();
  hipMemcpy(c, dc, 16 * 8, hipMemcpyDeviceToHost);
  const char* cn[4] = {"fma->readlane->fma", "fma->dpp->fma", "fma->lds->fma", "fma->fma"};
  for (int v = 0; v < 4; ++v) std::printf("chain %-20s %6.1f cycles/step\n", cn[v], c[v] / 64.0);
  k_calib<<<1, 64>>>(dio, dc);
  hipDeviceSynchronize();
  hipMemcpy(c, dc, 16 * 8, hipMemcpyDeviceToHost);
  std::printf("calibration: %lld s_memtime ticks in %lld s_memrealtime ticks (100 MHz): s_memtime at %.0f MHz; "
              "dependent f64 FMA %.2f ticks\n", c[1], c[0], 100.0 * c[1] / c[0], c[1] / 20000.0);
  return 0;
}
