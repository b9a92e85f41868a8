// Microbenchmark: where chain_row64_kernel's filter step (config 5) spends
// its cycles.  One wave per SIMD (256-thread blocks, 256 blocks), each wave
// running 128 steps of a 64-state mat-vec in registers like r64_filter:
//   V0 the step: blocks_of(x) -> 64 v_fmac_f64_dpp (4 accumulators) -> sum -> x
//   V1 V0's instructions with x fixed (no step-to-step dependency): issue rate
//   V2 only the 64 fmacs (x fixed)
//   V3 the step without the fmacs: the serial tail's latency
//   V4 V0 with 8 accumulators
//   V5 V0 plus an LDS read waited for inside the step (the evidence entry)
//   V6 V0 plus the kernel's other per-step work: two LDS ring writes and the
//      integer-max rescale every 4th step
//   V7 V6 plus a block barrier every 8 steps (all four waves in step)
//   V8 V6 with relative blocks: row r takes block r ^ s (s = 0: x itself, no
//      lane swap on the path to the first 16 fmacs), the other blocks by
//      in-place v_permlane16/32_swap (vdst = src0), no copies but one per block
//   V9 V6 plus a bare s_barrier every 8 steps (no lgkmcnt(0) drain of the ring writes)
//   V10 V6 plus the drained barrier every 16 steps
//   V11 V6 with 2 accumulators (one zeroing and one add fewer ... per pair)
//   V12 V6 with 3 accumulators
// and swapcheck: the in-place swaps' semantics (lane l gets lane l ^ 16 / l ^ 32)
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_r64.hip -o mb_r64 && ./mb_r64
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int K, bool NOP>
__device__ __forceinline__ void fb(double& acc, double v, double c) {
  if (NOP)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(c), "n"(K));
  else
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(c), "n"(K));
}
template <int NA>
__device__ __forceinline__ void f16(double (&acc)[NA], double xb, const double (&A)[16]) {
  fb<0, true>(acc[0 % NA], xb, A[0]);   fb<1, false>(acc[1 % NA], xb, A[1]);
  fb<2, false>(acc[2 % NA], xb, A[2]);  fb<3, false>(acc[3 % NA], xb, A[3]);
  fb<4, false>(acc[4 % NA], xb, A[4]);  fb<5, false>(acc[5 % NA], xb, A[5]);
  fb<6, false>(acc[6 % NA], xb, A[6]);  fb<7, false>(acc[7 % NA], xb, A[7]);
  fb<8, false>(acc[8 % NA], xb, A[8]);  fb<9, false>(acc[9 % NA], xb, A[9]);
  fb<10, false>(acc[10 % NA], xb, A[10]); fb<11, false>(acc[11 % NA], xb, A[11]);
  fb<12, false>(acc[12 % NA], xb, A[12]); fb<13, false>(acc[13 % NA], xb, A[13]);
  fb<14, false>(acc[14 % NA], xb, A[14]); fb<15, false>(acc[15 % NA], xb, A[15]);
}
__device__ __forceinline__ void blocks_of(double x, double (&xb)[4]) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto q0l = __builtin_amdgcn_permlane32_swap(pl[0], pl[0], false, false);
  const auto q0h = __builtin_amdgcn_permlane32_swap(ph[0], ph[0], false, false);
  const auto q1l = __builtin_amdgcn_permlane32_swap(pl[1], pl[1], false, false);
  const auto q1h = __builtin_amdgcn_permlane32_swap(ph[1], ph[1], false, false);
  xb[0] = __hiloint2double((int)q0h[0], (int)q0l[0]);
  xb[2] = __hiloint2double((int)q0h[1], (int)q0l[1]);
  xb[1] = __hiloint2double((int)q1h[0], (int)q1l[0]);
  xb[3] = __hiloint2double((int)q1h[1], (int)q1l[1]);
}
typedef __attribute__((address_space(3))) double lds_d;

__device__ __forceinline__ double self_swap16(double v) {
  unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0\n\tv_permlane16_swap_b32 %1, %1\n\ts_nop 1" : "+v"(lo), "+v"(hi));
  return __hiloint2double((int)hi, (int)lo);
}
__device__ __forceinline__ double self_swap32(double v) {
  unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0\n\tv_permlane32_swap_b32 %1, %1\n\ts_nop 1" : "+v"(lo), "+v"(hi));
  return __hiloint2double((int)hi, (int)lo);
}
__global__ void swapcheck(double* out) {
  const double v = (double)threadIdx.x;
  out[threadIdx.x] = self_swap16(v);
  out[64 + threadIdx.x] = self_swap32(v);
}

__device__ __forceinline__ int max_exp_rescale(double p) {
  int e = p != 0.0 ? __builtin_amdgcn_frexp_exp(p) : -0x40000;
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x128, 0xF, 0xF, true));
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x124, 0xF, 0xF, true));
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x122, 0xF, 0xF, true));
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x121, 0xF, 0xF, true));
  { const auto r = __builtin_amdgcn_permlane16_swap((unsigned)e, (unsigned)e, false, false); e = max((int)r[0], (int)r[1]); }
  { const auto r = __builtin_amdgcn_permlane32_swap((unsigned)e, (unsigned)e, false, false); e = max((int)r[0], (int)r[1]); }
  return e > -0x40000 ? -e : 0;
}

template <int V>
__global__ __launch_bounds__(256, 1) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  extern __shared__ double smem_raw[];
  lds_d* sm = (lds_d*)smem_raw;
  const int y = threadIdx.x & 63, w = threadIdx.x >> 6;
  double Ac[4][16];
#pragma unroll
  for (int b = 0; b < 4; b++)
#pragma unroll
    for (int j = 0; j < 16; j++) Ac[b][j] = in[(16 * b + j) * 64 + y] * (1.0 / 64);
  sm[threadIdx.x] = in[threadIdx.x] + 0.5;
  __syncthreads();
  double x = in[y] + 1.0;
  const double e = 1.0 + in[y + 100] * 1e-6;
  double xbf[4];
  blocks_of(x, xbf);
  int sc = 0;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int s = 0; s < n; s++) {
    double xb[4];
    if (V == 8) {
      xb[0] = x;
      xb[1] = self_swap16(x);
      xb[2] = self_swap32(x);
      xb[3] = self_swap32(xb[1]);
    } else if (V == 1 || V == 2) {
#pragma unroll
      for (int b = 0; b < 4; b++) { xb[b] = xbf[b]; asm volatile("" : "+v"(xb[b])); }
    } else {
      blocks_of(x, xb);
    }
    constexpr int NA = V == 4 ? 8 : V == 11 ? 2 : V == 12 ? 3 : 4;
    double acc[NA];
#pragma unroll
    for (int i = 0; i < NA; i++) acc[i] = 0.0;
    if (V != 3) {
      f16<NA>(acc, xb[0], Ac[0]); f16<NA>(acc, xb[1], Ac[1]); f16<NA>(acc, xb[2], Ac[2]); f16<NA>(acc, xb[3], Ac[3]);
    } else {
      acc[0] = xb[0]; acc[1] = xb[1]; acc[2] = xb[2]; acc[3] = xb[3];
    }
    double u;
    if constexpr (V >= 6) {
      double su;
      if constexpr (NA == 2) su = acc[0] + acc[1];
      else if constexpr (NA == 3) su = (acc[0] + acc[1]) + acc[2 % NA];
      else su = (acc[0] + acc[1]) + (acc[2 % NA] + acc[3 % NA]);
      u = __builtin_ldexp(su, sc);
      const double p = u * e;
      const int slot = s & 7;
      sm[1024 + (w * 8 + slot) * 64 + y] = p;
      sm[1024 + 2048 + (w * 8 + slot) * 64 + y] = u;
      sc = (s & 3) == 3 ? max_exp_rescale(p) : 0;
      x = p;
      if (V == 7 && (s & 7) == 7) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (V == 9 && (s & 7) == 7) asm volatile("s_barrier" ::: "memory");
      if (V == 10 && (s & 15) == 15) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      continue;
    }
    if constexpr (NA == 8) u = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    else u = (acc[0] + acc[1]) + (acc[2 % NA] + acc[3 % NA]);
    double ee = e;
    if (V == 5) ee *= sm[(s & 63) * 4 + w];
    const double p = u * ee;
    if (V == 2) { asm volatile("" :: "v"(acc[0]), "v"(acc[1]), "v"(acc[2]), "v"(acc[3])); }
    else if (V == 1) { asm volatile("" :: "v"(p)); }
    else x = p;
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (y == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int V>
void run(const char* name, double* din, double* dout, unsigned long long* dc) {
  const int n = 1024;
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<V>, dim3(256), dim3(256), (1024 + 4096) * 8, 0, din, dout, dc, n);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(256 * 4);
  (void)hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (auto v : c) m += v;
  m /= c.size();
  printf("%-62s %8.1f cycles/step\n", name, m / n);
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 8192 * 8);
  (void)hipMalloc(&dout, 256 * 256 * 8);
  (void)hipMalloc(&dc, 256 * 4 * 8);
  std::vector<double> h(8192);
  for (int i = 0; i < 8192; i++) h[i] = 0.5 + (i % 7) * 0.01;
  (void)hipMemcpy(din, h.data(), 8192 * 8, hipMemcpyHostToDevice);
  run<0>("V0 step: blocks_of + 64 fmac_dpp (4 acc) + sum, x -> next", din, dout, dc);
  run<1>("V1 V0 with x fixed (no step dependency)", din, dout, dc);
  run<2>("V2 64 fmac_dpp only, x fixed", din, dout, dc);
  run<3>("V3 V0 without the fmacs (serial tail)", din, dout, dc);
  run<4>("V4 V0 with 8 accumulators", din, dout, dc);
  run<5>("V5 V0 + an LDS read waited for in the step", din, dout, dc);
  run<6>("V6 V0 + two ring writes + max-exp rescale every 4th step", din, dout, dc);
  run<7>("V7 V6 + a block barrier every 8 steps", din, dout, dc);
  run<8>("V8 V6 with relative blocks and in-place swaps", din, dout, dc);
  run<9>("V9 V6 + a bare s_barrier every 8 steps (no drain)", din, dout, dc);
  run<10>("V10 V6 + the drained barrier every 16 steps", din, dout, dc);
  run<11>("V11 V6 with 2 accumulators", din, dout, dc);
  run<12>("V12 V6 with 3 accumulators", din, dout, dc);
  {
    hipLaunchKernelGGL(swapcheck, dim3(1), dim3(64), 0, 0, dout);
    std::vector<double> h(128);
    (void)hipMemcpy(h.data(), dout, 128 * 8, hipMemcpyDeviceToHost);
    int ok16 = 1, ok32 = 1;
    for (int l = 0; l < 64; l++) { ok16 &= h[l] == (double)(l ^ 16); ok32 &= h[64 + l] == (double)(l ^ 32); }
    printf("in-place v_permlane16_swap: lane l gets l ^ 16: %s; v_permlane32_swap: l ^ 32: %s\n",
           ok16 ? "yes" : "NO", ok32 ? "yes" : "NO");
    if (!ok16 || !ok32) { for (int l = 0; l < 64; l++) printf("%d:%g/%g ", l, h[l], h[64 + l]); printf("\n"); }
  }
  return 0;
}
