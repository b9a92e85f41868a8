// Microbenchmark (round 6): can the config-2 filter
// step be shorter than the 4-MFMA accumulation chain + evidence multiply
// (V4 of profiles/r03/mb_lat.hip, 464 cycles)?  One wave per block, 256
// blocks (one per CU, as the config-2 launch), cycles from s_memtime.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form mb_lat6.hip -o mb_lat6
//
// V4  4 v_mfma_f64_16x16x4 chained through C (K = 16 in four slices), D feeds
//     the next step's B after the evidence multiply (the kernels' step)
// V5  four independent K-slice MFMAs (each from C = 0), a VALU add tree
//     ((d0 + d1) + (d2 + d3)), then the evidence multiply
// V6  two independent 2-MFMA chains (K slices {0, 2} and {1, 3}), one add,
//     then the evidence multiply (round 2's NIPAMD_MFMA_SPLITK, in isolation)
// V7  V5 with the evidence folded into the tree: (d0 + d1) * e + (d2 + d3) * e
//     as one multiply and one fma per register
// V8  V4 run by two waves on one SIMD (two independent chains; block of 2
//     waves on a CU that holds one block): the pipe's throughput with the
//     latency chain doubled up
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0)

template <int V>
__global__ __launch_bounds__(256, 1) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  const int l = threadIdx.x & 63;
  // V8: waves 0 and 4 share SIMD 0 (round-robin placement); the others exit
  const int w = threadIdx.x >> 6;
  if (V == 8 ? (w != 0 && w != 4) : w != 0) return;
  double A[4];
#pragma unroll
  for (int i = 0; i < 4; i++) A[i] = in[l + 64 * i] * 0.01;
  v4d X = {in[l + 512], in[l + 576], in[l + 640], in[l + 704]};
  const v4d Y = {in[l + 768], in[l + 832], in[l + 896], in[l + 960]};
  const v4d E = {in[l + 1024], in[l + 1088], in[l + 1152], in[l + 1216]};
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t0 = __builtin_readcyclecounter();
  const v4d z = {0, 0, 0, 0};
  for (int i = 0; i < n; i++) {
    const v4d e = (i & 1) ? Y : E;
    if (V == 4 || V == 8) {
      v4d d = z;
      d = MFMA(A[0], X.x, d);
      d = MFMA(A[1], X.y, d);
      d = MFMA(A[2], X.z, d);
      d = MFMA(A[3], X.w, d);
      X = d * e;
    } else if (V == 5) {
      const v4d d0 = MFMA(A[0], X.x, z);
      const v4d d1 = MFMA(A[1], X.y, z);
      const v4d d2 = MFMA(A[2], X.z, z);
      const v4d d3 = MFMA(A[3], X.w, z);
      X = ((d0 + d1) + (d2 + d3)) * e;
    } else if (V == 6) {
      v4d d0 = MFMA(A[0], X.x, z);
      v4d d1 = MFMA(A[1], X.y, z);
      d0 = MFMA(A[2], X.z, d0);
      d1 = MFMA(A[3], X.w, d1);
      X = (d0 + d1) * e;
    } else if (V == 7) {
      const v4d d0 = MFMA(A[0], X.x, z);
      const v4d d1 = MFMA(A[1], X.y, z);
      const v4d d2 = MFMA(A[2], X.z, z);
      const v4d d3 = MFMA(A[3], X.w, z);
      const v4d p = (d0 + d1) * e;
      const v4d q = d2 + d3;
      X.x = __builtin_fma(q.x, e.x, p.x); X.y = __builtin_fma(q.y, e.y, p.y);
      X.z = __builtin_fma(q.z, e.z, p.z); X.w = __builtin_fma(q.w, e.w, p.w);
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = X.x + X.y + X.z + X.w;
  if (l == 0) { cyc[blockIdx.x * 2 + (w ? 1 : 0)] = t1 - t0; cyc[1024 + blockIdx.x * 2 + (w ? 1 : 0)] = r1 - r0; }
}

template <int V>
double run(const char* name, double* din, double* dout, unsigned long long* dc, int blocks) {
  const int n = 65536;
  for (int rep = 0; rep < 24; rep++)      // >= 1 s of back-to-back launches (clock settles), then stamp
    hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, din, dout, dc, n);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(2048);
  (void)hipMemcpy(c.data(), dc, 2048 * 8, hipMemcpyDeviceToHost);
  double m = 0, rt = 0;
  for (int b = 0; b < blocks; b++) { m += c[2 * b]; rt += c[1024 + 2 * b]; }
  m /= blocks;
  rt /= blocks;
  printf("%-70s %8.1f cycles/step  clock %.3f GHz\n", name, m / n, m / rt * 0.1);
  return m / n;
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 4096 * 8);
  (void)hipMalloc(&dout, 1024 * 256 * 8);
  (void)hipMalloc(&dc, 4096 * 8);
  (void)hipMemset(dc, 0, 4096 * 8);
  std::vector<double> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  for (int i = 1024; i < 1280; i++) h[i] = 1.0;
  (void)hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; rep++) {
    run<4>("V4 4 MFMAs chained through C + evidence multiply (the kernels)", din, dout, dc, 256);
    run<5>("V5 4 independent K-slice MFMAs + add tree + evidence multiply", din, dout, dc, 256);
    run<6>("V6 2 x 2-MFMA chains + add + evidence multiply", din, dout, dc, 256);
    run<7>("V7 4 independent K-slice MFMAs, evidence folded into the tree", din, dout, dc, 256);
    run<8>("V8 V4 with two waves on one SIMD (per wave)", din, dout, dc, 256);
  }
  return 0;
}
