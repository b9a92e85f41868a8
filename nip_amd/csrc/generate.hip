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

#include "chain_kernels.h"

namespace nipamd {

namespace {

constexpr int kGenBlock = 64;   // one wave per block: spreads B series over the CUs

__global__ __launch_bounds__(kGenBlock) void generate_kernel(GenArgs a) {
  extern __shared__ uint32_t lds[];
  uint32_t* st = lds;                               // [31][kGenBlock] rand() state
  int* smp = (int*)(lds + 31 * kGenBlock);          // [nv][kGenBlock] draws of this slice
  const int tid = threadIdx.x;
  const long b = (long)blockIdx.x * kGenBlock + tid;
  if (b >= a.B) return;                              // no block-level sync below
  if (!a.draws)
    for (int m = 0; m < 31; m++) st[m * kGenBlock + tid] = a.win[b * 31 + m];
  int pos = 0, prev = 0;
  bool dead = false;
  int* out = a.out + b * (long)a.T * a.nv;
  for (int t = 0; t < a.T; t++) {
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
      const double* row = dead ? a.tab + a.zero_off : a.tab + (t ? s.off1 : s.off0) + idx;
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
      // lottery() (nip.c:2507-2520)
      int k = 0;
      double sum = 0.0;
      for (;;) {
        if (k >= s.card) { k = s.card; break; }
        sum += row[k++];
        if (!(sum < r)) break;
      }
      k -= 1;
      if (row[k] == 0.0) dead = true;
      smp[i * kGenBlock + tid] = k;
      out[(long)t * a.nv + i] = k;
    }
    prev = smp[a.x1_step * kGenBlock + tid];
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
  if (a.B <= 0 || a.T <= 0) return 0;
  const size_t lds = (size_t)(31 + a.nv) * kGenBlock * sizeof(uint32_t);
  hipLaunchKernelGGL(generate_kernel, dim3((unsigned)((a.B + kGenBlock - 1) / kGenBlock)),
                     dim3(kGenBlock), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
