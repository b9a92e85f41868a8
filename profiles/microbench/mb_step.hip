// Microbenchmark: cycles per filter step of the matrix-core chain kernel,
// building the step up piece by piece.  One wave per block, 256 blocks.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_step.hip -o mb_step && ./mb_step
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double sum_lanes32(double x) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
__device__ __forceinline__ double sum_lanes16(double x) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
__device__ __forceinline__ double chain_sum(v4d v) { return sum_lanes16(sum_lanes32((v.x + v.y) + (v.z + v.w))); }
__device__ __forceinline__ v4d matvec(const double (&A)[4], v4d X) {
  v4d d = {0, 0, 0, 0};
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0], X.x, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[1], X.y, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[2], X.z, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[3], X.w, d, 0, 0, 0);
  return d;
}
__device__ __forceinline__ v4d matvec2(const double (&A)[4], v4d X) {   // two chains of two
  const v4d z = {0, 0, 0, 0};
  v4d d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0], X.x, z, 0, 0, 0);
  v4d d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[2], X.z, z, 0, 0, 0);
  d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[1], X.y, d0, 0, 0, 0);
  d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[3], X.w, d1, 0, 0, 0);
  return d0 + d1;
}
__device__ __forceinline__ v4d matvec4(const double (&A)[4], v4d X) {   // four independent
  const v4d z = {0, 0, 0, 0};
  v4d d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0], X.x, z, 0, 0, 0);
  v4d d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[1], X.y, z, 0, 0, 0);
  v4d d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[2], X.z, z, 0, 0, 0);
  v4d d3 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[3], X.w, z, 0, 0, 0);
  return (d0 + d1) + (d2 + d3);
}
__device__ __forceinline__ v4d ldexp4(v4d v, int k) {
  v4d r; r.x = __builtin_ldexp(v.x, k); r.y = __builtin_ldexp(v.y, k);
  r.z = __builtin_ldexp(v.z, k); r.w = __builtin_ldexp(v.w, k); return r;
}

template <int V>
__global__ __launch_bounds__(64, 1) void k(const double* in, double* out, unsigned long long* cyc, int n) {
  __shared__ double lds[64 * 8];
  const int l = threadIdx.x;
  double A[4] = {in[l] * 0.1, in[l + 64] * 0.1, in[l + 128] * 0.1, in[l + 192] * 0.1};
  v4d X = {in[l + 256], in[l + 320], in[l + 384], in[l + 448]};
  v4d e = {in[l + 512], in[l + 576], in[l + 640], in[l + 704]};   // not constant-folded
  v4d s = {1, 1, 1, 1};
  int sc = 0; double m2 = 1, m1 = 1;
  unsigned long long t0 = __builtin_readcyclecounter();
  v4d D = matvec(A, X);
  for (int i = 0; i < n; i++) {
    if (V == 11 || V == 12 || V == 13) {         // next MFMAs interleaved with this step's VALU
      v4d u = ldexp4(D, sc);
      v4d p = u * e;
      v4d d = {0, 0, 0, 0};
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0], p.x, d, 0, 0, 0);
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      const double loc = (p.x + p.y) + (p.z + p.w);
      const double h = sum_lanes32(loc);
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[1], p.y, d, 0, 0, 0);
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      const double z2 = sum_lanes16(h);
      sc = -__builtin_amdgcn_frexp_exp(z2); m2 *= z2;
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[2], p.z, d, 0, 0, 0);
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      *reinterpret_cast<double2*>(lds + (l * 2 + (i & 3) * 128)) = make_double2(p.x, p.y);
      *reinterpret_cast<double2*>(lds + (l * 2 + (i & 3) * 128 + 256)) = make_double2(p.z, p.w);
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[3], p.w, d, 0, 0, 0);
      if (V == 13) __builtin_amdgcn_sched_barrier(0);
      if (V == 12) {
        // MFMA, VALU x4, MFMA, VALU x6, MFMA, DS write x2, MFMA
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      D = d;
      X = p;
      continue;
    }
    if (V >= 5 && V < 8) {                       // software-pipelined: next MFMAs issued before this step's sums
      v4d u = ldexp4(D, sc);
      v4d p = u * e;
      if (V >= 6) __builtin_amdgcn_sched_barrier(0);
      D = matvec(A, p);
      if (V >= 6) __builtin_amdgcn_sched_barrier(0);
      const double z2 = chain_sum(p); sc = -__builtin_amdgcn_frexp_exp(z2); m2 *= z2;
      const double z1 = chain_sum(u * s); m1 *= z1;
      if (V != 7) {
      *reinterpret_cast<double2*>(lds + (l * 2 + (i & 3) * 128)) = make_double2(p.x, p.y);
      *reinterpret_cast<double2*>(lds + (l * 2 + (i & 3) * 128 + 256)) = make_double2(p.z, p.w);
      }
      X = p;
      continue;
    }
    v4d u = V == 8 ? matvec2(A, X) : V == 9 ? matvec4(A, X) : matvec(A, X);
    if ((V >= 1 && V < 8) || V == 10) u = ldexp4(u, sc);
    v4d p = ((V >= 1 && V < 8) || V == 10) ? u * e : u;
    if (V == 10) {   // z2 through one MFMA with an all-ones A operand
      const double loc = (p.x + p.y) + (p.z + p.w);
      const v4d zz = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, loc, v4d{0, 0, 0, 0}, 0, 0, 0);
      const double z2 = zz.x; sc = -__builtin_amdgcn_frexp_exp(z2); m2 *= z2;
    }
    if (V >= 2 && V < 8) { const double z2 = chain_sum(p); sc = -__builtin_amdgcn_frexp_exp(z2); m2 *= z2; }
    if (V >= 3 && V < 8) { const double z1 = chain_sum(u * s); m1 *= z1; }
    if (V >= 4 && V < 8) { *reinterpret_cast<double2*>(lds + (l * 2 + (i & 3) * 128)) = make_double2(p.x, p.y);
                  *reinterpret_cast<double2*>(lds + (l * 2 + (i & 3) * 128 + 256)) = make_double2(p.z, p.w); }
    X = p;
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + l] = X.x + X.y + X.z + X.w + m2 + m1 + lds[l];
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
void run(const char* name, double* din, double* dout, unsigned long long* dc, int blocks) {
  const int n = 2048;
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, din, dout, dc, n);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, din, dout, dc, n);
  hipDeviceSynchronize();
  std::vector<unsigned long long> c(blocks);
  hipMemcpy(c.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto x : c) m += x; m /= blocks;
  printf("%-40s blocks %4d  %.1f cycles/step\n", name, blocks, m / n);
}

int main() {
  double *din, *dout; unsigned long long* dc;
  hipMalloc(&din, 4096 * 8); hipMalloc(&dout, 1024 * 64 * 8); hipMalloc(&dc, 1024 * 8);
  std::vector<double> h(4096); for (int i = 0; i < 4096; i++) h[i] = 0.5 + (i % 7) * 0.01;
  hipMemcpy(din, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  for (int blocks : {256}) {
    run<0>("4 chained MFMA", din, dout, dc, blocks);
    run<1>("+ ldexp, *e", din, dout, dc, blocks);
    run<2>("+ z2 chain_sum, frexp", din, dout, dc, blocks);
    run<3>("+ z1 chain_sum", din, dout, dc, blocks);
    run<4>("+ 2 ds_write_b128", din, dout, dc, blocks);
    run<5>("pipelined (next MFMA before sums)", din, dout, dc, blocks);
    run<6>("pipelined + sched_barrier", din, dout, dc, blocks);
    run<7>("pipelined + sched_barrier, no ds_write", din, dout, dc, blocks);
    run<8>("MFMA: two chains of two + add", din, dout, dc, blocks);
    run<9>("MFMA: four independent + adds", din, dout, dc, blocks);
    run<10>("ldexp,*e + z2 via ones-MFMA (cf. row 3)", din, dout, dc, blocks);
    run<11>("interleaved source order (row 4 work)", din, dout, dc, blocks);
    run<12>("interleaved + sched_group_barrier", din, dout, dc, blocks);
    run<13>("interleaved, pinned by sched_barrier", din, dout, dc, blocks);
  }
  return 0;
}
