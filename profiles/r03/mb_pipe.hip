// Microbenchmark: f64 matrix-core and vector issue rates on gfx950 (one wave
// per SIMD or two, 256 blocks), with the instruction stream pinned by inline
// asm so the compiler cannot reorder or re-register it.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form mb_pipe.hip -o mb_pipe
//
// P0  8 independent v_mfma_f64_16x16x4 accumulators (VGPR), back to back
// P1  4 independent accumulators
// P2  2 independent accumulators
// P3  1 accumulator (dependent chain through C)
// P4  16 independent v_fma_f64 per iteration (VALU issue rate)
// P5  8 independent MFMAs + 16 independent v_fma_f64 interleaved (shared pipe?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

#define MF(acc, a, b) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define FM(x, a, b) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b))

template <int V>
__global__ __launch_bounds__(256) void k(const double* in, double* out, unsigned long long* cyc, int n, int waves) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w >= waves) return;
  const double a = in[l] * 0.001, b = in[l + 64] * 0.001;
  v4d acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = v4d{in[l + 128 + i], 0, 0, 0};
  double x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = in[l + 256 + i];
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i++) {
    if (V == 0) {
#pragma unroll
      for (int j = 0; j < 8; j++) MF(acc[j], a, b);
    } else if (V == 1) {
#pragma unroll
      for (int j = 0; j < 8; j++) MF(acc[j & 3], a, b);
    } else if (V == 2) {
#pragma unroll
      for (int j = 0; j < 8; j++) MF(acc[j & 1], a, b);
    } else if (V == 3) {
#pragma unroll
      for (int j = 0; j < 8; j++) MF(acc[0], a, b);
    } else if (V == 4) {
#pragma unroll
      for (int j = 0; j < 16; j++) FM(x[j], a, b);
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        MF(acc[j], a, b);
        FM(x[2 * j], a, b);
        FM(x[2 * j + 1], a, b);
      }
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
#pragma unroll
  for (int i = 0; i < 16; i++) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int V>
void run(const char* name, double* din, double* dout, unsigned long long* dc, int waves, double per) {
  const int n = 2048;
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<V>, dim3(256), dim3(256), 0, 0, din, dout, dc, n, waves);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(1024);
  (void)hipMemcpy(c.data(), dc, 1024 * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int b = 0; b < 256; b++) m += c[b * 4];
  m /= 256;
  printf("%-58s waves/CU %d  %8.1f cycles/iter  %6.1f cycles per op (wave 0)\n", name, waves, m / n, m / n / per);
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 4096 * 8);
  (void)hipMalloc(&dout, 256 * 256 * 8);
  (void)hipMalloc(&dc, 1024 * 8);
  (void)hipMemset(dc, 0, 1024 * 8);
  std::vector<double> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  (void)hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  for (int waves : {1, 8}) {
    run<0>("P0 MFMA f64 16x16x4, 8 independent accumulators", din, dout, dc, waves, 8);
    run<1>("P1 MFMA f64 16x16x4, 4 accumulators", din, dout, dc, waves, 8);
    run<2>("P2 MFMA f64 16x16x4, 2 accumulators", din, dout, dc, waves, 8);
    run<3>("P3 MFMA f64 16x16x4, 1 accumulator (C chain)", din, dout, dc, waves, 8);
    run<4>("P4 v_fma_f64, 16 independent", din, dout, dc, waves, 16);
    run<5>("P5 8 MFMA + 16 v_fma_f64 interleaved (per MFMA)", din, dout, dc, waves, 8);
  }
  return 0;
}
