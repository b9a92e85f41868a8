// Microbenchmark: issue cost of the f64 matrix and vector instructions the
// chain kernels are built from, on one wave per SIMD (blocks of 64 threads,
// 1024 blocks) and two waves per SIMD (2048 blocks).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_mfma.hip -o mb_mfma && ./mb_mfma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int V>
__global__ __launch_bounds__(64) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  const int l = threadIdx.x;
  const double a = in[l] * 0.001, b = in[l + 64] * 0.001;
  v4d d[8];
  for (int i = 0; i < 8; i++) d[i] = v4d{in[l] + i, 0.0, 1.0, 2.0};
  double x[16];
  for (int i = 0; i < 16; i++) x[i] = in[l + i];
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < n; it++) {
    if (V == 0) {        // 8 independent 16x16x4 f64 MFMA
#pragma unroll
      for (int i = 0; i < 8; i++) d[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d[i], 0, 0, 0);
    } else if (V == 1) { // 8 dependent
#pragma unroll
      for (int i = 0; i < 8; i++) d[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d[0], 0, 0, 0);
    } else if (V == 2) { // 8 independent 4x4x4 (4 blocks) f64 MFMA
#pragma unroll
      for (int i = 0; i < 8; i++) d[i].x = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d[i].x, 0, 0, 0);
    } else if (V == 3) { // 16 independent v_fma_f64
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = __builtin_fma(x[i], a, b);
    } else if (V == 4) { // 8 independent MFMA interleaved with 16 independent v_fma_f64
#pragma unroll
      for (int i = 0; i < 8; i++) {
        d[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d[i], 0, 0, 0);
        x[2 * i] = __builtin_fma(x[2 * i], a, b);
        x[2 * i + 1] = __builtin_fma(x[2 * i + 1], a, b);
      }
    } else if (V == 5) { // 16 independent v_fma_f32-pair ops for comparison: v_pk_fma_f32
#pragma unroll
      for (int i = 0; i < 16; i++) {
        float2 f = make_float2((float)x[i], (float)a);
        f.x = __builtin_fmaf(f.x, f.y, 1.0f);
        x[i] = f.x;
      }
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  double acc = 0;
  for (int i = 0; i < 8; i++) acc += d[i].x + d[i].y + d[i].z + d[i].w;
  for (int i = 0; i < 16; i++) acc += x[i];
  out[blockIdx.x * 64 + l] = acc;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
void run(const char* name, int per, double* din, double* dout, unsigned long long* dc, int blocks) {
  const int n = 4096;
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, din, dout, dc, n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, din, dout, dc, n);
  hipEventRecord(e1);
  hipDeviceSynchronize();
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(blocks);
  hipMemcpy(c.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto x : c) m += x; m /= blocks;
  printf("%-48s blocks %5d  %7.1f cycles per instruction (wave view)  kernel %.3f ms\n", name, blocks,
         m / n / per, ms);
}

int main() {
  double *din, *dout; unsigned long long* dc;
  hipMalloc(&din, 4096 * 8); hipMalloc(&dout, 4096 * 64 * 8); hipMalloc(&dc, 4096 * 8);
  std::vector<double> h(4096); for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  for (int blocks : {1024, 2048}) {
    run<0>("mfma_f64_16x16x4 independent", 8, din, dout, dc, blocks);
    run<1>("mfma_f64_16x16x4 dependent", 8, din, dout, dc, blocks);
    run<2>("mfma_f64_4x4x4 independent", 8, din, dout, dc, blocks);
    run<3>("v_fma_f64 independent", 16, din, dout, dc, blocks);
    run<4>("8 mfma + 16 v_fma_f64 interleaved (per mfma)", 8, din, dout, dc, blocks);
    run<5>("v_fma_f32 (+cvt) independent", 16, din, dout, dc, blocks);
  }
  return 0;
}
