// chain_wide.hip -- forward-backward for interface chains of up to 64 states
// with up to four observed children (SURVEY 8(d) configs 3 and 5 after the
// host folds the slice's hidden independent parents into the transition).
//
// Same recursion as chain_kernels.hip, with the evidence of step t the
// product of one table column per observed child:
//   e_t[y] = prod_k T_k[code_k(t)][y]      (T_k row M_k = the child's row sum,
//                                           row M_k + 1 = 0; T_0 also carries
//                                           the row sums of unobserved children)
// Mapping: one wave per (sequence, direction), lane y = state y; a block is
// the forward and the backward wave of one sequence (two-filter smoothing,
// phase A / barrier / phase B as the other kernels).  The mat-vec reads the
// input vector from LDS by broadcast (ds_read_b128) against this lane's
// column (forward) or row (backward) of A held in registers; chain sums are
// 16-lane DPP butterflies followed by the permlane16/32 exchanges, so every
// lane holds the same bits.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "chain_kernels.h"
#include "diag.h"

namespace nipamd {

namespace {

constexpr int kWG = kScratchGuard;
constexpr int kWChunk = 8;

template <int K>
__device__ __forceinline__ double ror64(double v) {     // row_ror:K of a double
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x120 + K, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum(double x) {
  asm("" : "+v"(x));       // one rounded value per lane: no fma contraction into the first add
  x += ror64<8>(x);
  x += ror64<4>(x);
  x += ror64<2>(x);
  x += ror64<1>(x);
  {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    x = __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
  }
  {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    x = __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
  }
  return x;
}

__device__ __forceinline__ double recip(double c) {
  double r = __builtin_amdgcn_rcp(c);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  return c != 0.0 ? r : 0.0;
}

template <bool FWD, int NP>
struct WideChain {
  double Acol[NP];   // fwd: A[x][y] (column y); bwd: A[y][x] (row y)
  double X = 0.0;    // this lane's entry of the next mat-vec input
  int sc = 0;
  double m2 = 1.0, m1 = 1.0, zmin = 1.0;
  int e2 = 0, e1 = 0;

  // u = sum_x Acol[x] * X[x], X broadcast through LDS
  __device__ __forceinline__ double matvec(double* xb, int y) {
    xb[y] = X;
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int x = 0; x < NP; x += 2) {
      const double2 v = *reinterpret_cast<const double2*>(xb + x);
      a0 = __builtin_fma(Acol[x], v.x, a0);
      a1 = __builtin_fma(Acol[x + 1], v.y, a1);
    }
    return a0 + a1;
  }

  template <bool COMBINE>
  __device__ __forceinline__ void step(const WideArgs& a, double* xb, int y, double e, double s,
                                       double other, double* Sst, double* Pst, bool renorm) {
    const double u = __builtin_ldexp(matvec(xb, y), sc);
    const double p = u * e;
    const double keep = FWD ? p : u;
    const double z2 = wave_sum(p);
    if (FWD) {
      const double z1 = wave_sum(u * s);
      zmin = __builtin_fmin(zmin, z2);
      m2 *= z2; m1 *= z1;
      if (renorm) {
        const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
        const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
      }
    }
    if (!COMBINE) {
      *Sst = keep;
    } else {
      const double pr = keep * other;
      const double q = pr * recip(wave_sum(pr));
      if (Pst) *Pst = q;
    }
    sc = -__builtin_amdgcn_frexp_exp(z2);
    X = p;
  }
};

template <bool FWD, int NP>
__device__ void wide_wave(const WideArgs& a, const uint8_t* codes, int Tr, double* xb, int y, long b) {
  const int T = a.T, H = a.H;
  if (a.filter && !FWD) {                  // forward_inference: H = 0, no backward filter
    __syncthreads();
    return;
  }
  WideChain<FWD, NP> ch;
#pragma unroll
  for (int x = 0; x < NP; x++) ch.Acol[x] = FWD ? a.A[x * 64 + y] : a.A[y * 64 + x];
  const double s = a.s[y];
  double* Srow = a.S + (size_t)b * chain_scratch_row64(T) + (size_t)kWG * 64 + y;
  double* Prow = (a.post && y < a.N) ? a.post + (size_t)b * a.post_bstride + a.post_off + y : nullptr;
  const double eb = a.ebase[y];
  auto evidence = [&](int t) {
    double e = eb;
    for (int k = 0; k < a.ncol; k++) e *= a.tab[k][codes[k * Tr + kWG + t] * 64 + y];
    return e;
  };
  if (FWD) {
    ch.X = a.pi[y];
  } else {
    const double beta = y < a.N ? 1.0 : 0.0;
    Srow[(long)(T - 1) * 64] = beta;                  // beta_{T-1}, T-1 >= H
    ch.X = evidence(T - 1) * beta;
    ch.sc = -__builtin_amdgcn_frexp_exp(wave_sum(ch.X));
  }
  constexpr int dir = FWD ? 1 : -1;
  auto phase = [&](auto combine_tag, int n, int t0) {
    constexpr bool COMBINE = decltype(combine_tag)::value;
    double o[kWChunk];
    for (int base = 0; base < n; base += kWChunk) {
      double e[kWChunk];
#pragma unroll
      for (int k = 0; k < kWChunk; k++) {
        const int t = t0 + dir * (base + k);            // guards cover the over-run
        e[k] = evidence(t);
        o[k] = COMBINE ? (a.filter ? 1.0 : Srow[(long)t * 64]) : 0.0;
      }
#pragma unroll
      for (int k = 0; k < kWChunk; k++) {
        if (base + k >= n) break;
        const int t = t0 + dir * (base + k);
        ch.template step<COMBINE>(a, xb, y, e[k], s, o[k], Srow + (long)t * 64,
                                  Prow ? Prow + (long)t * a.post_tstride : nullptr, (k & 3) == 3);
      }
    }
  };
  if (FWD) phase(std::false_type{}, H, 0);
  else phase(std::false_type{}, T - 1 - H, T - 2);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (FWD) phase(std::true_type{}, T - H, H);
  else phase(std::true_type{}, H, H - 1);
  if (FWD && y == 0) {
    double ll = log(ch.m2) - log(ch.m1) + (double)(ch.e2 - ch.e1) * 0.69314718055994530942;
    const bool dead = ch.zmin == 0.0;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    if (a.status) a.status[b] = dead ? 1u : 0u;
  }
}

template <int NP>
__global__ __launch_bounds__(128, 1)
void chain_wide_kernel(WideArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* xbuf = reinterpret_cast<double*>(smem);             // [2][64]
  uint8_t* codes = smem + 2 * 64 * sizeof(double);             // [ncol][Tr]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long b = blockIdx.x;
  const int T = a.T, Tr = chain_codes_row(T);
  for (int k = 0; k < a.ncol; k++) {
    const int M = a.M[k];
    for (int i = tid; i < Tr; i += 128) {
      const int t = i - kWG;
      int c = M;                                                // missing / guard
      if (t >= 0 && t < T) {
        const int o = a.obs[b * a.obs_bstride + (long)t * a.obs_tstride + a.col[k]];
        c = o < 0 ? M : (o < M ? o : M + 1);
      }
      codes[k * Tr + i] = (uint8_t)c;
    }
  }
  __syncthreads();
  if (wave == 0) wide_wave<true, NP>(a, codes, Tr, xbuf, lane, b);
  else wide_wave<false, NP>(a, codes, Tr, xbuf + 64, lane, b);
}

}  // namespace

size_t chain_wide_lds_bytes(int ncol, int T) {
  return 2 * 64 * sizeof(double) + (size_t)(ncol > 0 ? ncol : 1) * chain_codes_row(T);
}

int chain_wide_launch(const WideArgs& a, hipStream_t stream) {
  // 33..64 states: the four-waves-per-direction kernel (chain_wide4.hip);
  // NIPAMD_WIDE_KERNEL=wave1 keeps this one-wave form for A/B measurements
  static const bool wave1 = [] {
    const char* e = diag_env("NIPAMD_WIDE_KERNEL");
    return e && std::string(e) == "wave1";
  }();
  if (a.N > 32 && !wave1) {
    const int rc = chain_wide4_launch(a, stream);
    if (rc != -2) return rc;
  }
  const size_t lds = (chain_wide_lds_bytes(a.ncol, a.T) + 15) & ~(size_t)15;
  const dim3 grid((unsigned)a.B), block(128);
  g_last_kernel = a.N <= 16 ? "chain_wide_kernel<16>" : a.N <= 32 ? "chain_wide_kernel<32>" : "chain_wide_kernel<64>";
  if (a.N <= 16) hipLaunchKernelGGL(chain_wide_kernel<16>, grid, block, lds, stream, a);
  else if (a.N <= 32) hipLaunchKernelGGL(chain_wide_kernel<32>, grid, block, lds, stream, a);
  else hipLaunchKernelGGL(chain_wide_kernel<64>, grid, block, lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
