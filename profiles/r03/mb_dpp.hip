// Microbenchmark: a DPP (VALU) filter step of a 16-state chain, as an
// alternative to config 2's matrix-core step (mb_lat.hip V4: 464 cycles).
// A 16-lane row holds one sequence's 16 states; a wave holds 4 sequences.
// Step: x' = (sum_i bcast(x_i) A(i, j)) * e  (16 v_fmac_f64_dpp into 4
// accumulators), the row to LDS, every 4th step a row sum -> frexp -> ldexp.
// W waves per block (one block per CU, 256 blocks): W/4 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_dpp.hip -o mb_dpp && ./mb_dpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int K, bool NOP_FIRST>
__device__ __forceinline__ void fmac_bcast(double& acc, double v, double c) {
  if (NOP_FIRST)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(K));
  else
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(K));
}
template <int K>
__device__ __forceinline__ double row_ror(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int rl = __builtin_amdgcn_mov_dpp(lo, 0x120 + K, 0xF, 0xF, true);
  const int rh = __builtin_amdgcn_mov_dpp(hi, 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(rh, rl);
}
__device__ __forceinline__ double row_sum(double x) {
  asm("" : "+v"(x));
  x += row_ror<8>(x);
  x += row_ror<4>(x);
  x += row_ror<2>(x);
  x += row_ror<1>(x);
  return x;
}

template <int V>
__global__ __launch_bounds__(1024, 1) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  __shared__ double lds[16 * 8 * 64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  double A[16];
#pragma unroll
  for (int i = 0; i < 16; i++) A[i] = in[(l & 15) + 16 * i] * 0.06;
  double E[8];
#pragma unroll
  for (int i = 0; i < 8; i++) E[i] = in[256 + l + i];
  double x = in[512 + l];
  int sc = 0;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i += 8) {
#pragma unroll
    for (int s = 0; s < 8; s++) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      fmac_bcast<0, true>(a0, x, A[0]);   fmac_bcast<1, false>(a1, x, A[1]);
      fmac_bcast<2, false>(a2, x, A[2]);  fmac_bcast<3, false>(a3, x, A[3]);
      fmac_bcast<4, false>(a0, x, A[4]);  fmac_bcast<5, false>(a1, x, A[5]);
      fmac_bcast<6, false>(a2, x, A[6]);  fmac_bcast<7, false>(a3, x, A[7]);
      fmac_bcast<8, false>(a0, x, A[8]);  fmac_bcast<9, false>(a1, x, A[9]);
      fmac_bcast<10, false>(a2, x, A[10]); fmac_bcast<11, false>(a3, x, A[11]);
      fmac_bcast<12, false>(a0, x, A[12]); fmac_bcast<13, false>(a1, x, A[13]);
      fmac_bcast<14, false>(a2, x, A[14]); fmac_bcast<15, false>(a3, x, A[15]);
      double u = (a0 + a1) + (a2 + a3);
      if (V >= 1) u = __builtin_ldexp(u, sc);
      x = u * E[s];
      if (V >= 1) {
        lds[(w * 8 + s) * 64 + l] = x;
        if ((s & 3) == 3) sc = -__builtin_amdgcn_frexp_exp(row_sum(x));
        else sc = 0;
      }
    }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  __syncthreads();
  out[blockIdx.x * 1024 + threadIdx.x] = x + lds[threadIdx.x];
  if (l == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
}

template <int V>
void run(const char* name, int W, double* din, double* dout, unsigned long long* dc) {
  const int n = 8192;
  for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k<V>, dim3(256), dim3(64 * W), 0, 0, din, dout, dc, n);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(256 * 16);
  (void)hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int b = 0; b < 256; b++) for (int w = 0; w < W; w++) m += c[b * 16 + w];
  m /= 256.0 * W;
  printf("%-46s waves/SIMD %2d  %7.1f cycles per wave-step  (%6.1f per step of 16 sequences x 2 directions)\n",
         name, W / 4, m / n, m / n * 8.0 / W);
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 4096 * 8);
  (void)hipMalloc(&dout, 256 * 1024 * 8);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  std::vector<double> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  (void)hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  for (int W : {4, 8, 12, 16}) {
    run<0>("D0 dot_bcast + evidence multiply", W, din, dout, dc);
    run<1>("D1 D0 + LDS row + sum/ldexp every 4th", W, din, dout, dc);
  }
  return 0;
}
