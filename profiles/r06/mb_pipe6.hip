// Microbenchmark (round 6): f64 matrix-core and vector throughput of ONE SIMD
// shared by several waves (profiles/r03/mb_pipe.hip ran one wave per SIMD).
// Block of 4 W waves on a CU (256 blocks); wave w runs on SIMD w % 4, so every
// SIMD holds W waves.  Instruction streams pinned by inline asm.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form mb_pipe6.hip -o mb_pipe6
//
// Q0  every wave: 8 independent v_mfma_f64_16x16x4 per iteration
// Q1  waves w < 4: 8 independent MFMAs; waves w >= 4: 32 independent v_fma_f64
// Q2  waves w < 4: 8 independent MFMAs; waves w >= 4: 32 independent v_fma_f32
// Q3  every wave: one MFMA accumulation chain (C -> C), 8 per iteration
// Q4  every wave: 32 v_fma_f64 (16 accumulators)
// Q5  waves w < 4: two filter steps (4 chained MFMAs + multiply, the kernels' step);
//     waves w >= 4: 32 independent v_fma_f64
// Q6  every wave: two filter steps
// Printed: cycles per iteration of wave 0 (and of wave 4), and the SIMD's
// MFMA throughput implied (W waves x 8 MFMAs per iteration).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

#define MF(acc, a, b) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define FM(x, a, b) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b))
#define FM32(x, a, b) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b))

template <int V>
__global__ __launch_bounds__(1024) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double a = in[l] * 0.001, b = in[l + 64] * 0.001;
  const float af = (float)a, bf = (float)b;
  // only what a variant uses is live (no spills at 4 waves per SIMD: 128 VGPRs)
  constexpr bool kMf = V == 0 || V == 1 || V == 2 || V == 3;
  constexpr bool kX = V == 1 || V == 4 || V == 5;
  constexpr bool kXf = V == 2;
  v4d acc[8];
  double x[16];
  float xf[16];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = v4d{kMf ? in[l + 128 + i] : 0.0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; i++) { x[i] = kX ? in[l + 256 + i] : 0.0; xf[i] = kXf ? (float)in[l + 256 + i] : 0.f; }
  const bool mf = V == 0 || V == 3 || V == 6 || ((V == 1 || V == 2 || V == 5) && w < 4);
  v4d X = {in[l + 300], in[l + 301], in[l + 302], in[l + 303]};
  const v4d E = {in[l + 304], in[l + 305], in[l + 306], in[l + 307]};
  __syncthreads();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i++) {
    if (mf) {
      if (V == 3) {
#pragma unroll
        for (int j = 0; j < 8; j++) MF(acc[0], a, b);
      } else if (V == 5 || V == 6) {
        // two filter steps: 4 MFMAs chained through C, D -> the next step's B after a multiply
#pragma unroll
        for (int j = 0; j < 2; j++) {
          v4d d = {0, 0, 0, 0};
          d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, X.x, d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f64_16x16x4f64(b, X.y, d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, X.z, d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f64_16x16x4f64(b, X.w, d, 0, 0, 0);
          X = d * E;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) MF(acc[j], a, b);
      }
    } else if (V == 2) {
#pragma unroll
      for (int j = 0; j < 32; j++) FM32(xf[j & 15], af, bf);
    } else {
#pragma unroll
      for (int j = 0; j < 32; j++) FM(x[j & 15], a, b);
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  __syncthreads();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
#pragma unroll
  for (int i = 0; i < 16; i++) s += x[i] + xf[i];
  s += X.x + X.y + X.z + X.w;
  out[blockIdx.x * 1024 + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
  if (threadIdx.x == 0) cyc[4096 + blockIdx.x] = r1 - r0;   // the whole block, 100 MHz ticks
}

template <int V>
void run(const char* name, double* din, double* dout, unsigned long long* dc, int W) {
  const int n = 2048;
  for (int r = 0; r < 6; r++) hipLaunchKernelGGL(k<V>, dim3(256), dim3(256 * W), 0, 0, din, dout, dc, n);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(4096 + 256);
  (void)hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m4 = 0, wall = 0;
  for (int b = 0; b < 256; b++) { m0 += c[b * 16]; m4 += c[b * 16 + (W > 1 ? 4 : 0)]; wall += c[4096 + b]; }
  m0 /= 256 * (double)n;
  m4 /= 256 * (double)n;
  wall /= 256 * (double)n;   // 100 MHz ticks per iteration
  // block wall time in shader cycles at the wave-0 clock ratio is not known: report ns
  printf("%-52s W=%d  wave0 %7.1f  wave4 %7.1f cycles/iter  block wall %7.2f ns/iter\n", name, W, m0, m4, wall * 10.0);
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 4096 * 8);
  (void)hipMalloc(&dout, 256 * 1024 * 8);
  (void)hipMalloc(&dc, (4096 + 256) * 8);
  (void)hipMemset(dc, 0, (4096 + 256) * 8);
  std::vector<double> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  (void)hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  for (int W : {1, 2, 3, 4}) run<0>("Q0 8 independent MFMA f64 per wave", din, dout, dc, W);
  for (int W : {1, 2, 3, 4}) run<3>("Q3 8-MFMA C chain per wave", din, dout, dc, W);
  for (int W : {1, 2, 4}) run<4>("Q4 32 independent v_fma_f64 per wave", din, dout, dc, W);
  run<1>("Q1 waves<4: 8 MFMA; waves>=4: 32 v_fma_f64", din, dout, dc, 2);
  run<2>("Q2 waves<4: 8 MFMA; waves>=4: 32 v_fma_f32", din, dout, dc, 2);
  run<5>("Q5 waves<4: 2 filter steps; waves>=4: 32 v_fma_f64", din, dout, dc, 1);
  run<5>("Q5 waves<4: 2 filter steps; waves>=4: 32 v_fma_f64", din, dout, dc, 2);
  run<6>("Q6 every wave: 2 filter steps", din, dout, dc, 1);
  run<6>("Q6 every wave: 2 filter steps", din, dout, dc, 2);
  run<6>("Q6 every wave: 2 filter steps", din, dout, dc, 3);
  return 0;
}
