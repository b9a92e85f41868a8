// generate_data on the GPU (src/nip.c:2325-2478): one
// thread per series, B series of length T at once.
//
// The reference samples every variable of a slice in a fixed order
// (independent variables, then children whose parents are drawn), each from
// get_probability() after the previous draws were entered as evidence, with
// lottery() (nip.c:2507-2520) on one rand() draw.  For an interface-chain
// model those conditionals are functions of the earlier draws of the slice
// and of the previous slice's interface state only, so the host tabulates
// them once (generate.cpp) and a thread walks its series: context index ->
// table row -> lottery.  rand() is glibc's additive generator
// r[n] = r[n-3] + r[n-31] (mod 2^32), draw = r[n] >> 1; each thread starts
// from the 31-word window of its own offset in the one stream the reference
// would consume (series after series), so the draws are the reference's.
//
// A draw of a zero-probability state (lottery() returns state 0 on a draw of
// exactly 0) zeroes the reference's join tree for the rest of the series; the
// thread then samples from an all-zero row, as lottery() does there.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "chain_kernels.h"

namespace nipamd {

namespace {

constexpr int kGenBlock = 64;   // one wave per block: spreads B series over the CUs

// LDS_TAB: the running-sum tables (a.cum_n doubles) are copied into LDS first;
// otherwise every row read goes to L2 / HBM, where the output stream evicts them
template <bool LDS_TAB>
__global__ __launch_bounds__(kGenBlock) void generate_kernel(GenArgs a) {
  extern __shared__ uint32_t lds[];
  uint32_t* st = lds;                               // [31][kGenBlock] rand() state
  // draws of the last `stage` slices, [stage][nv][kGenBlock]: written out per
  // thread in one burst of stores every `stage` slices, so a load's vmcnt wait
  // (loads and stores retire in order) meets outstanding stores that rarely
  int* stage = (int*)(lds + 31 * kGenBlock);
  const int tid = threadIdx.x;
  const long b = (long)blockIdx.x * kGenBlock + tid;
  double* cum_lds = (double*)(lds + (31 + a.stage * a.nv) * kGenBlock);
  if (LDS_TAB) {
    for (long k = tid; k < a.cum_n; k += kGenBlock) cum_lds[k] = a.cum[k];
    __syncthreads();
  }
  const double* cum = LDS_TAB ? cum_lds : a.cum;
  if (b >= a.B) return;                              // no block-level sync below
  if (!a.draws)
    for (int m = 0; m < 31; m++) st[m * kGenBlock + tid] = a.win[b * 31 + m];
  int pos = 0, prev = 0;
  bool dead = false;
  int* out = a.out + b * (long)a.T * a.nv;
  int tt = 0;
  long t0 = 0;
  for (int t = 0; t < a.T; t++) {
    int* smp = stage + (long)tt * a.nv * kGenBlock;
    for (int i = 0; i < a.nv; i++) {
      const GenStep& s = a.steps[i];
      const int nctx = t ? s.nctx1 : s.nctx;
      const int* ctx = t ? s.ctx1 : s.ctx;
      const long* stride = t ? s.stride1 : s.stride;
      long idx = 0;
      for (int c = 0; c < nctx; c++) {
        const int j = ctx[c];
        idx += (long)(j >= 0 ? smp[j * kGenBlock + tid] : prev) * stride[c];
      }
      const long ro = dead ? a.zero_off : (t ? s.off1 : s.off0) + idx;
      // rand(): r[n] = r[n-31] + r[n-3]; slot pos holds r[n-31], slot pos+28 (mod 31) r[n-3]
      int draw;
      if (a.draws) {
        draw = a.draws[(b * a.T + t) * (long)a.nv + i];
      } else {
        const int p3 = pos + 28 >= 31 ? pos - 3 : pos + 28;
        const uint32_t v = st[pos * kGenBlock + tid] + st[p3 * kGenBlock + tid];
        st[pos * kGenBlock + tid] = v;
        pos = pos == 30 ? 0 : pos + 1;
        draw = (int)(v >> 1);
      }
      const double r = (double)draw / 2147483647.0;
      // lottery() (nip.c:2507-2520): the first k whose running sum is not
      // below r.  The sums (cum, added in lottery()'s order on the host) are
      // non-decreasing, so k = #{cum < r}: independent loads, no chain.
      const double* crow = cum + ro;
      int k = 0;
      for (int k0 = 0; k0 < s.card; k0 += 16) {
        double c[16];
#pragma unroll
        for (int u = 0; u < 16; u++) c[u] = k0 + u < s.card ? crow[k0 + u] : r;
#pragma unroll
        for (int u = 0; u < 16; u++) k += c[u] < r;
      }
      // a zero-probability draw: r == 0 takes state 0 (reached only with
      // row[0] == 0 then), and running off the row end takes the last state
      if (k == s.card) {
        k = s.card - 1;
        if (a.tab[ro + k] == 0.0) dead = true;
      } else if (r == 0.0 && crow[0] == 0.0) {
        dead = true;
      }
      smp[i * kGenBlock + tid] = k;
    }
    prev = smp[a.x1_step * kGenBlock + tid];
    if (++tt == a.stage || t == a.T - 1) {
      int* o = out + t0 * a.nv;
      for (int u = 0; u < tt * a.nv; u++) __builtin_nontemporal_store(stage[u * kGenBlock + tid], o + u);
      t0 += tt;
      tt = 0;
    }
  }
}

// c = a * b mod (x^31 - x^28 - 1), coefficients mod 2^32 (fully unrolled:
// every index static, the polynomials live in VGPRs)
__device__ __forceinline__ void polymulmod(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  uint32_t c[61];
#pragma unroll
  for (int k = 0; k < 61; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 31; i++)
#pragma unroll
    for (int j = 0; j < 31; j++) c[i + j] += a[i] * b[j];
#pragma unroll
  for (int d = 60; d >= 31; d--) {
    c[d - 3] += c[d];
    c[d - 31] += c[d];
  }
#pragma unroll
  for (int k = 0; k < 31; k++) out[k] = c[k];
}

// win[b] = the rand() window of series b: x^(b D) mod P = (x^D)^b by square
// and multiply on the bits of b, applied to the stream's first 61 words
__global__ __launch_bounds__(256) void rand_window_kernel(int B, const uint32_t* __restrict__ qd,
                                                          uint32_t* __restrict__ win) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  uint32_t r[31], p[31];
#pragma unroll
  for (int k = 0; k < 31; k++) { r[k] = k == 0; p[k] = qd[k]; }
  for (unsigned e = (unsigned)b; e; e >>= 1) {
    if (e & 1) polymulmod(r, p, r);
    if (e > 1) polymulmod(p, p, p);
  }
  const uint32_t* base = qd + 31;               // r[313 .. 373]
#pragma unroll
  for (int m = 0; m < 31; m++) {
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 31; j++) s += r[j] * base[m + j];
    win[(long)b * 31 + m] = s;
  }
}

}  // namespace

int rand_window_launch(int B, const uint32_t* qd_base, uint32_t* win, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(rand_window_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, stream, B,
                     qd_base, win);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int generate_launch(const GenArgs& a, hipStream_t stream) {
  g_last_kernel = "generate_kernel";
  if (a.B <= 0 || a.T <= 0) return 0;
  GenArgs g = a;
  g.stage = std::max(1, std::min(16, (256 - 31) / std::max(1, a.nv)));   // <= 64 KB LDS per block
  size_t lds = (size_t)(31 + g.stage * a.nv) * kGenBlock * sizeof(uint32_t);
  const dim3 grid((unsigned)((a.B + kGenBlock - 1) / kGenBlock));
  if (lds + a.cum_n * sizeof(double) <= 64 * 1024) {
    lds += a.cum_n * sizeof(double);
    hipLaunchKernelGGL(generate_kernel<true>, grid, dim3(kGenBlock), lds, stream, g);
  } else {
    hipLaunchKernelGGL(generate_kernel<false>, grid, dim3(kGenBlock), lds, stream, g);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
