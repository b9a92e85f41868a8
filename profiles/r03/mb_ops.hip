// Microbenchmark: issue cost of the f64 VALU / DPP / conversion instructions
// the chain kernels are made of, on gfx950, with two waves per SIMD
// (512-thread blocks, one per CU) and 8 independent chains per wave, the
// instruction stream pinned by inline asm.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_ops.hip -o mb_ops && ./mb_ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int V>
__global__ __launch_bounds__(512) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  double x[8];
  int e[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { x[i] = in[l + 64 * i] + 1.0; e[i] = i & 1; }
  const double c = in[l + 600] * 1e-3;
  unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < n; it++) {
#define FMA(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x[i]) : "v"(c));
#define ADD(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[i]) : "v"(c));
#define MUL(i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[i]) : "v"(c));
#define LDX(i) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(x[i]) : "v"(e[i]));
#define FRX(i) asm volatile("v_frexp_exp_i32_f64 %0, %1" : "=v"(e[i]) : "v"(x[i]));
#define DPP(i) asm volatile("v_mov_b32_dpp %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(e[i]));
#define FBC(i) asm volatile("v_fmac_f64_dpp %0, %1, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(x[i]) : "v"(c));
#define CND(i) asm volatile("v_cndmask_b32 %0, 0, %0, vcc" : "+v"(e[i]) :: "vcc");
#define I32(i) asm volatile("v_add_u32 %0, %0, %0" : "+v"(e[i]));
#define RCP(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(x[i]));
    if (V == 0) { R8(FMA) } else if (V == 1) { R8(ADD) } else if (V == 2) { R8(MUL) } else if (V == 3) { R8(LDX) }
    else if (V == 4) { R8(FRX) } else if (V == 5) { R8(DPP) } else if (V == 6) { R8(FBC) } else if (V == 7) { R8(CND) }
    else if (V == 8) { R8(I32) } else { R8(RCP) }
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += x[i] + e[i];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int V>
void run(const char* name, double* din, double* dout, unsigned long long* dc) {
  const int n = 4096;
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<V>, dim3(256), dim3(512), 0, 0, din, dout, dc, n);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(256 * 8);
  (void)hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (auto v : c) m += v;
  m /= c.size();
  // two waves per SIMD: SIMD cycles per wave-instruction = wave cycles / (2 * 8 * n)
  printf("%-34s %7.2f SIMD cycles per wave64 instruction (2 waves/SIMD, 8 chains each)\n", name, m / (16.0 * n));
}

int main() {
  double *din, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&din, 4096 * 8);
  (void)hipMalloc(&dout, 256 * 512 * 8);
  (void)hipMalloc(&dc, 256 * 8 * 8);
  std::vector<double> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  (void)hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  run<0>("v_fma_f64", din, dout, dc);
  run<1>("v_add_f64", din, dout, dc);
  run<2>("v_mul_f64", din, dout, dc);
  run<3>("v_ldexp_f64", din, dout, dc);
  run<4>("v_frexp_exp_i32_f64", din, dout, dc);
  run<5>("v_mov_b32_dpp row_ror", din, dout, dc);
  run<6>("v_fmac_f64_dpp row_newbcast", din, dout, dc);
  run<7>("v_cndmask_b32", din, dout, dc);
  run<8>("v_add_u32", din, dout, dc);
  run<9>("v_rcp_f64", din, dout, dc);
  return 0;
}
