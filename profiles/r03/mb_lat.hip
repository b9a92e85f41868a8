// Microbenchmark: the dependency-chain floor of the matrix-core chain
// kernels' filter step (the "latency roof" of bench.py).  One wave per block,
// 256 blocks (one per CU, as the config-2 launch), cycles from s_memtime.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_lat.hip -o mb_lat && ./mb_lat
//
// V0  v_mfma_f64_16x16x4 chained through the accumulator only (C -> C)
// V1  independent v_mfma_f64_16x16x4 back to back (issue rate)
// V2  config 2's step: 4 MFMAs chained through C, D feeds the next step's B
// V3  config 3's step (NT = 2): two output tiles, each 8 MFMAs chained
//     through C, interleaved; D feeds the next step's B operands
// V4  V2 + the evidence multiply (p = d o e, e from registers)
// V5  V4 + ldexp by a power of two on every step
// V6  V4 + the step's two ds_write_b128 of the row + a 16-state sum every
//     4th step feeding the next step's ldexp (config 2's filter step)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0)

template <int V>
__global__ __launch_bounds__(64, 1) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  const int l = threadIdx.x;
  double A[8];
#pragma unroll
  for (int i = 0; i < 8; i++) A[i] = in[l + 64 * i] * 0.01;
  v4d X = {in[l + 512], in[l + 576], in[l + 640], in[l + 704]};
  v4d Y = {in[l + 768], in[l + 832], in[l + 896], in[l + 960]};
  const v4d E = {in[l + 1024], in[l + 1088], in[l + 1152], in[l + 1216]};
  __shared__ double lds[8 * 256];
  int sc = V == 5 ? 0 : 0;
  v4d acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = v4d{0, 0, 0, 0};
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i++) {
    if (V == 0) {
#pragma unroll
      for (int j = 0; j < 4; j++) acc[0] = MFMA(A[j], X.x, acc[0]);
    } else if (V == 1) {
#pragma unroll
      for (int j = 0; j < 8; j++) acc[j] = MFMA(A[j], X.x, acc[j]);
    } else if (V == 2) {
      v4d d = {0, 0, 0, 0};
      d = MFMA(A[0], X.x, d);
      d = MFMA(A[1], X.y, d);
      d = MFMA(A[2], X.z, d);
      d = MFMA(A[3], X.w, d);
      X = d;
    } else if (V >= 4) {
      v4d d = {0, 0, 0, 0};
      d = MFMA(A[0], X.x, d);
      d = MFMA(A[1], X.y, d);
      d = MFMA(A[2], X.z, d);
      d = MFMA(A[3], X.w, d);
      if (V == 5 || V == 6) {
        d.x = __builtin_ldexp(d.x, sc); d.y = __builtin_ldexp(d.y, sc);
        d.z = __builtin_ldexp(d.z, sc); d.w = __builtin_ldexp(d.w, sc);
      }
      const v4d e = (i & 1) ? Y : E;
      X = d * e;
      if (V == 6) {
        double* L = lds + (i & 7) * 256 + l * 2;
        *reinterpret_cast<double2*>(L) = make_double2(X.x, X.y);
        *reinterpret_cast<double2*>(L + 128) = make_double2(X.z, X.w);
        if ((i & 3) == 3) {
          double z = (X.x + X.y) + (X.z + X.w);
          z += __shfl_xor(z, 32);
          z += __shfl_xor(z, 16);
          sc = -__builtin_amdgcn_frexp_exp(z);
        } else {
          sc = 0;
        }
      }
    } else {
      v4d d0 = {0, 0, 0, 0}, d1 = {0, 0, 0, 0};
      d0 = MFMA(A[0], X.x, d0); d1 = MFMA(A[4], X.x, d1);
      d0 = MFMA(A[1], X.y, d0); d1 = MFMA(A[5], X.y, d1);
      d0 = MFMA(A[2], X.z, d0); d1 = MFMA(A[6], X.z, d1);
      d0 = MFMA(A[3], X.w, d0); d1 = MFMA(A[7], X.w, d1);
      d0 = MFMA(A[4], Y.x, d0); d1 = MFMA(A[0], Y.x, d1);
      d0 = MFMA(A[5], Y.y, d0); d1 = MFMA(A[1], Y.y, d1);
      d0 = MFMA(A[6], Y.z, d0); d1 = MFMA(A[2], Y.z, d1);
      d0 = MFMA(A[7], Y.w, d0); d1 = MFMA(A[3], Y.w, d1);
      X = d0;
      Y = d1;
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = X.x + X.y + X.z + X.w + Y.x + Y.y + Y.z + Y.w;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i].x + acc[i].w;
  out[blockIdx.x * 64 + l] = s;
  if (l == 0) { cyc[blockIdx.x] = t1 - t0; cyc[1024 + blockIdx.x] = r1 - r0; }
}

template <int V>
double run(const char* name, double* din, double* dout, unsigned long long* dc, int blocks, double per) {
  const int n = V >= 2 && V != 3 ? 65536 : 4096;
  for (int rep = 0; rep < (V == 2 ? 40 : 2); rep++)      // V2: >= 2 s of back-to-back launches, then stamp
    hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, din, dout, dc, n);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(2048);
  (void)hipMemcpy(c.data(), dc, 2048 * 8, hipMemcpyDeviceToHost);
  double m = 0, rt = 0;
  for (int b = 0; b < blocks; b++) { m += c[b]; rt += c[1024 + b]; }
  m /= blocks;
  rt /= blocks;
  printf("%-62s %8.1f cycles/iter  %6.1f cycles/MFMA  clock %.3f GHz\n", name, m / n, m / n / per,
         m / rt * 0.1);
  return m / n;
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 4096 * 8);
  (void)hipMalloc(&dout, 1024 * 64 * 8);
  (void)hipMalloc(&dc, 2048 * 8);
  std::vector<double> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  for (int i = 1024; i < 1280; i++) h[i] = 1.0;
  (void)hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  run<0>("V0 MFMA f64 16x16x4 chained C->C (4 per iter)", din, dout, dc, 256, 4);
  run<1>("V1 MFMA f64 16x16x4 independent (8 per iter)", din, dout, dc, 256, 8);
  run<2>("V2 config-2 step: 4 chained, D -> next B", din, dout, dc, 256, 4);
  run<3>("V3 config-3 step: 2 x 8 chained, interleaved, D -> next B", din, dout, dc, 256, 16);
  run<4>("V4 V2 + evidence multiply", din, dout, dc, 256, 4);
  run<5>("V5 V4 + ldexp every step", din, dout, dc, 256, 4);
  run<6>("V6 V4 + row writes + sum/ldexp every 4th step", din, dout, dc, 256, 4);
  return 0;
}
