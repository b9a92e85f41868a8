// chain_mfma_core.h -- the matrix-core chain pieces shared by the
// forward-backward kernels of chain_mfma.hip (scratch round trip) and
// chain_ckpt.hip (checkpoints + recompute): register layout, reductions, the
// filter step (Chain), the forward partner's log-likelihood (LL).  Included
// once per translation unit, inside an anonymous namespace.
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>
#include <utility>

#include "chain_kernels.h"

namespace nipamd {
namespace {

typedef double v4d __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

#ifndef NIPAMD_MFMA_ABLATE
#define NIPAMD_MFMA_ABLATE 0       // timing-only builds: 11 no posterior stores, 12 no phase-B loads,
                                   // 14 no phase-B ll, 17 phase-B partners only load,
                                   // 19 phase-B partners idle
#endif
#ifndef NIPAMD_MFMA_DMA
#define NIPAMD_MFMA_DMA 1          // phase-B prefetch by LDS-DMA when the LDS budget allows
#endif
#ifndef NIPAMD_MFMA_RESCALE
#define NIPAMD_MFMA_RESCALE 4      // phase-A filter rescale interval in steps (1, 2, 4 or 8)
#endif
#ifndef NIPAMD_MFMA_NT
#define NIPAMD_MFMA_NT 0           // posterior stores: 1 non-temporal, 2 sc1 buffer stores, 3 plain buffer stores
#endif

constexpr int kMSeq = 16;          // sequences per block
constexpr int kMThreads = 256;     // waves: 0 fwd filter, 1 bwd filter, 2 fwd partner, 3 bwd partner
constexpr int kMChunk = 8;         // steps per chunk = ring slot
constexpr int kRescale = NIPAMD_MFMA_RESCALE;
static_assert(kRescale == 1 || kRescale == 2 || kRescale == 4 || kRescale == 8, "rescale interval");
constexpr int kMG = kScratchGuard;
constexpr int kStepD = kMSeq * 16;                 // doubles per step (2 KB)
constexpr int kSlotD = kMChunk * kStepD;           // doubles per ring slot (16 KB)
constexpr int kOutD = 2 * 2 * kSlotD;              // rings [dir][slot] (64 KB)
constexpr int kZD = 2 * kMChunk * kMSeq;           // forward z2 ring [slot][step][chain] (2 KB)
constexpr int kSStep = kMSeq * 16;                 // doubles per step of a block's scratch
constexpr int kOBRow = 130;                        // DMA buffer doubles per chain: 1 KB + 16 B, so that
                                                   // chain c starts 4c banks over (conflict-free reads)

__host__ __device__ inline long block_scratch(int T) { return (long)(T + 2 * kMG) * kSStep; }

__device__ __forceinline__ double sum_lanes32(double x) {   // x[l] + x[l ^ 32]
  double xc = x;
  asm("" : "+v"(xc));   // the swap's second operand: a whole-double copy (one v_mov_b64)
  const auto rl = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

__device__ __forceinline__ double sum_lanes16(double x) {   // x[l] + x[l ^ 16]
  double xc = x;
  asm("" : "+v"(xc));   // the swap's second operand: a whole-double copy (one v_mov_b64)
  const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

// sum of the chain's 16 states, identical in the chain's four lanes
__device__ __forceinline__ double chain_sum(v4d v) {
  return sum_lanes16(sum_lanes32((v.x + v.y) + (v.z + v.w)));
}

// DPP move of a double within a 16-lane row (32-bit halves; full row mask)
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// sum over aligned groups of 8 lanes (quad swaps, then row_half_mirror);
// every level pairs equal partial sums, so all 8 lanes get identical bits
__device__ __forceinline__ double sum8(double x) {
  asm("" : "+v"(x));       // one rounded value per lane: no fma contraction into the first add
  x += dpp64<0xB1>(x);     // quad_perm [1,0,3,2]
  x += dpp64<0x4E>(x);     // quad_perm [2,3,0,1]
  x += dpp64<0x141>(x);    // row_half_mirror
  return x;
}

// sum8 of n independent values, level by level so the n dependency chains
// interleave (one wave per SIMD: nothing else hides the f64 latency)
template <int n>
__device__ __forceinline__ void sum8_n(double (&x)[n]) {
#pragma unroll
  for (int i = 0; i < n; i++) asm("" : "+v"(x[i]));   // see sum8
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += dpp64<0xB1>(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += dpp64<0x4E>(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += dpp64<0x141>(x[i]);
}

// 1/c for n values, staged like sum8_n; 0 where c == 0
template <int n>
__device__ __forceinline__ void recip_n(const double (&c)[n], double (&r)[n]) {
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = __builtin_amdgcn_rcp(c[i]);
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = __builtin_fma(r[i], __builtin_fma(-c[i], r[i], 1.0), r[i]);
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = __builtin_fma(r[i], __builtin_fma(-c[i], r[i], 1.0), r[i]);
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = c[i] != 0.0 ? r[i] : 0.0;
}

#ifndef NIPAMD_MFMA_SPLITK
#define NIPAMD_MFMA_SPLITK 0       // 1: the K=16 contraction as two independent 2-MFMA chains + adds
#endif

__device__ __forceinline__ v4d matvec(const double (&Aop)[4], v4d X) {
#if NIPAMD_MFMA_SPLITK
  // two accumulators: the second chain's MFMAs issue in the first chain's
  // dependency shadow (one wave per SIMD: nothing else would fill it)
  v4d d0 = {0.0, 0.0, 0.0, 0.0}, d1 = {0.0, 0.0, 0.0, 0.0};
  d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0], X.x, d0, 0, 0, 0);
  d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[1], X.y, d1, 0, 0, 0);
  d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[2], X.z, d0, 0, 0, 0);
  d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[3], X.w, d1, 0, 0, 0);
  return d0 + d1;
#else
  v4d d = {0.0, 0.0, 0.0, 0.0};
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0], X.x, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[1], X.y, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[2], X.z, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[3], X.w, d, 0, 0, 0);
  return d;
#endif
}

__device__ __forceinline__ v4d ldexp4(v4d v, int k) {
  v4d r;
  r.x = __builtin_ldexp(v.x, k); r.y = __builtin_ldexp(v.y, k);
  r.z = __builtin_ldexp(v.z, k); r.w = __builtin_ldexp(v.w, k);
  return r;
}

// 1/c (v_rcp_f64 + two Newton steps); 0 when c == 0 so that an all-zero
// array stays zero (nip_normalise_array, nippotential.c:354)
__device__ __forceinline__ double recip(double c) {
  double r = __builtin_amdgcn_rcp(c);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  return c != 0.0 ? r : 0.0;
}

// actual state held by register r of lane group g
__host__ __device__ constexpr int state_of(int g, int r) { return r < 2 ? 2 * g + r : 6 + 2 * g + r; }

// this lane's four states of a 16-state row; p = row + 2g
__device__ __forceinline__ v4d load4(const double* p) {
  const double2 a = *reinterpret_cast<const double2*>(p);
  const double2 b = *reinterpret_cast<const double2*>(p + 8);
  v4d r;
  r.x = a.x; r.y = a.y; r.z = b.x; r.w = b.y;
  return r;
}

// LDS ring layout of one step: chain j's 16 states at j*16, its eight 16-byte
// pieces XOR-swizzled by (j & 7) so that the filter's writes and the
// partner's reads are bank-conflict free.
__device__ __forceinline__ int piece_off(int j, int s) { return j * 16 + ((s ^ (j & 7)) << 1); }

#ifndef NIPAMD_WAIT_TIMES
#define NIPAMD_WAIT_TIMES 0        // diagnostics build: per-wave barrier wait cycles into the stamps
#endif
struct WaitAcc {
  unsigned long long cyc = 0;
};

__device__ __forceinline__ void barrier_lds(WaitAcc* w = nullptr) {
#if NIPAMD_WAIT_TIMES
  const unsigned long long t0 = __builtin_readcyclecounter();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (w) w->cyc += __builtin_readcyclecounter() - t0;
#else
  (void)w;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
}

// LDS-DMA prefetch of the other direction's vectors (phase B).  Sixteen
// global_load_lds_dwordx4, one per chain c: lane L reads q + 128 B * c and the
// 1 KB lands lane-linearly at dst + kOBRow * 8 B * c.  No VGPR is written, so the
// compiler has nothing to reorder; the completions are counted by hand with
// s_waitcnt vmcnt (the DMA is invisible to the compiler's own waits).
template <int C>
__device__ __forceinline__ void dma1(const double* q, unsigned lds_base) {
  unsigned keep;
  // the instruction offset would move the LDS address too: the global address
  // carries the 128 B * C instead
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(q + C * 16), "s"(lds_base + C * (kOBRow * 8u))
               : "memory");
}
template <int... C>
__device__ __forceinline__ void dma16(const double* q, unsigned lds_base, std::integer_sequence<int, C...>) {
  (dma1<C>(q, lds_base), ...);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// diagnostics builds: s_memrealtime (100 MHz) stamp k of this block, lane 0
__device__ __forceinline__ void diag_stamp(const ChainArgs& a, int k, int lane) {
  if (a.diag && lane == 0) a.diag[blockIdx.x * 24 + k] = __builtin_amdgcn_s_memrealtime();
}

struct WaveCtx {
  const double* Et;         // LDS evidence table + 2g (row stride es)
  const uint8_t* codes;     // LDS codes of chain j, index t in [-kMG, T + kMG)
  double* out;              // this direction's LDS ring [2][kMChunk][kStepD]
  double* zr;               // forward: LDS ring of step masses z2 [2][kMChunk][16], else null
  int* scr;                 // e_step: LDS ring of applied scale exponents [2][kMChunk][16], else null
  int wo0, wo1;             // this lane's two piece offsets within a step
  bool zw;                  // this lane writes its chain's z2 (lane group 0)
  int es = 16;              // evidence row stride (doubles)
  int wodd = 0;             // chain-swap layouts (Chain<..., SW = 1>): offset added on odd rows
};

// SW = 1: the chain-swap ring layout of chain_ckpt.hip (odd rows hold chain
// j at position j ^ 1: row pointer + c.wodd for this lane)
template <bool FWD, bool ES = false, int SW = 0>
struct Chain {
  double Aop[4];
  v4d X;          // next mat-vec input (fwd: alpha_{t-1}; bwd: e_{t+1} o beta_{t+1})
  int sc = 0;     // power-of-two scale applied to the next mat-vec result

  // one step: the interface vector (alpha_t or beta_t, scaled) to LDS row L;
  // the forward filter also publishes its step mass z2 for the partner's ll
  template <bool SUM = true>
  __device__ __forceinline__ void step(const WaveCtx& c, double* L, double* Z, int* SC, v4d e) {
    if (ES && c.zw) *SC = sc;                  // e_step partners need the exponent applied at t
    const v4d u = ldexp4(matvec(Aop, X), sc);
    const v4d p = u * e;
    const v4d keep = FWD ? p : u;
    *reinterpret_cast<double2*>(L + c.wo0) = make_double2(keep.x, keep.y);
    *reinterpret_cast<double2*>(L + c.wo1) = make_double2(keep.z, keep.w);
    if (SUM) {
      const double z2 = chain_sum(p);
      if (FWD && c.zw) *Z = z2;
      sc = -__builtin_amdgcn_frexp_exp(z2);   // frexp exponent of 0 is 0
    } else {
      sc = 0;
    }
    X = p;
  }

  // the eight codes and evidence vectors of the chunk starting at step `base`
  __device__ __forceinline__ void load_chunk(const WaveCtx& c, int t0, int base, v4d (&e)[kMChunk]) {
    constexpr int dir = FWD ? 1 : -1;
    int code[kMChunk];
#pragma unroll
    for (int k = 0; k < kMChunk; k++) code[k] = c.codes[t0 + dir * (base + k)];   // guards cover over-run
#pragma unroll
    for (int k = 0; k < kMChunk; k++) e[k] = load4(c.Et + code[k] * c.es);
  }

  template <bool SPARSE>
  __device__ __forceinline__ void chunk(const WaveCtx& c, int n, int ci, int t0, int lane, WaitAcc* w,
                                        const v4d (&e)[kMChunk], v4d (&en)[kMChunk]) {
    double* slot = c.out + (ci & 1) * kSlotD;
    double* zs = FWD ? c.zr + (ci & 1) * kMChunk * kMSeq + (lane & 15) : nullptr;
    int* ss = ES ? c.scr + (ci & 1) * kMChunk * kMSeq + (lane & 15) : nullptr;
    const int base = ci * kMChunk;
    load_chunk(c, t0, base + kMChunk, en);       // the next chunk's inputs, one chunk ahead
    if (base + kMChunk <= n) {
#pragma unroll
      for (int k = 0; k < kMChunk; k++) {
        if (!SPARSE || (k & (kRescale - 1)) == kRescale - 1)
          step<true>(c, slot + k * kStepD + ((SW && (k & 1)) ? c.wodd : 0), zs + k * kMSeq, ss + k * kMSeq, e[k]);
        else
          step<false>(c, slot + k * kStepD + ((SW && (k & 1)) ? c.wodd : 0), zs + k * kMSeq, ss + k * kMSeq, e[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kMChunk; k++)
        if (base + k < n)
          step(c, slot + k * kStepD + ((SW && (k & 1)) ? c.wodd : 0), zs + k * kMSeq, ss + k * kMSeq, e[k]);
    }
    barrier_lds(w);
  }

  // a phase of n steps from t0 in nch chunks (uniform over the block); a
  // chunk's codes and evidence vectors are read from LDS one chunk ahead.
  // SPARSE: full chunks rescale (and publish z2) every kRescale-th step only;
  // the forward partner sums alpha_t itself (phase A, where the filter bounds
  // the time and the partner idles).  Between rescales the mass shrinks by
  // the product of kRescale steps' evidence: exact as long as that product
  // stays above 2^-1022 (each step's evidence mass above 2^-255 at 4).
  template <bool SPARSE>
  __device__ __forceinline__ void run(const WaveCtx& c, int n, int nch, int t0, int lane, WaitAcc* w) {
    v4d ea[kMChunk], eb[kMChunk];
    if (nch > 0) load_chunk(c, t0, 0, ea);
    for (int ci = 0; ci < nch; ci += 2) {
      chunk<SPARSE>(c, n, ci, t0, lane, w, ea, eb);
      if (ci + 1 >= nch) break;
      chunk<SPARSE>(c, n, ci + 1, t0, lane, w, eb, ea);
    }
  }
};

template <bool FWD, bool ES = false, bool SPARSE_B = false, int SW = 0>
__device__ __forceinline__ void filter_wave(const ChainArgs& a, const WaveCtx& c, const double* Et,
                                            double* Sw, int lane, bool active, long b,
                                            int nchA, int nchB, unsigned long long* stamps) {
  const int j = lane & 15, g = lane >> 4;
  const int sj = state_of(j & 3, j >> 2);       // actual state of D row j
  const int T = a.T, H = a.H;
  Chain<FWD, ES, SW> ch;
#pragma unroll
  for (int r = 0; r < 4; r++)
    ch.Aop[r] = FWD ? a.A[state_of(g, r) * 16 + sj] : a.A[sj * 16 + state_of(g, r)];
  if (FWD) {
    ch.X = load4(a.pi + 2 * g);
    if (ES) {                                   // S[-1] = alpha_{-1} = prior: the backward partner's P0 step
      double* q = Sw - kSStep;
      *reinterpret_cast<double2*>(q) = make_double2(ch.X.x, ch.X.y);
      *reinterpret_cast<double2*>(q + 8) = make_double2(ch.X.z, ch.X.w);
    }
  } else {
    v4d beta;                                   // beta_{T-1} = 1 on the real states
    beta.x = state_of(g, 0) < a.N ? 1.0 : 0.0; beta.y = state_of(g, 1) < a.N ? 1.0 : 0.0;
    beta.z = state_of(g, 2) < a.N ? 1.0 : 0.0; beta.w = state_of(g, 3) < a.N ? 1.0 : 0.0;
    {                                           // S[T-1] (T-1 >= H): the forward partner's in phase B
      double* q = Sw + (long)(T - 1) * kSStep;
      *reinterpret_cast<double2*>(q) = make_double2(beta.x, beta.y);
      *reinterpret_cast<double2*>(q + 8) = make_double2(beta.z, beta.w);
    }
    ch.X = load4(c.Et + c.codes[T - 1] * c.es) * beta;
    ch.sc = -__builtin_amdgcn_frexp_exp(chain_sum(ch.X));
  }
  WaitAcc wa, wb;
  // phase A: forward alpha_0..alpha_{H-1}; backward beta_{T-2}..beta_H
  if (FWD) ch.template run<true>(c, H, nchA, 0, lane, &wa);
  else ch.template run<true>(c, T - 1 - H, nchA, T - 2, lane, &wa);
  if (stamps && lane == 0) stamps[blockIdx.x * 4 + 1] = __builtin_readcyclecounter();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  if (stamps && lane == 0) stamps[blockIdx.x * 4 + 2] = __builtin_readcyclecounter();
  if (ES && FWD) diag_stamp(a, 2, lane);
  // phase B: forward alpha_H..alpha_{T-1}; backward beta_{H-1}..beta_0 (e_step:
  // ..beta_{-1}, the step against alpha_{-1} = prior that yields P0 and xi_0)
  // (SPARSE_B: phase B rescales like phase A; the partner then sums alpha itself)
  if (FWD) ch.template run<SPARSE_B>(c, T - H, nchB, H, lane, &wb);
  else ch.template run<SPARSE_B>(c, ES ? H + 1 : H, nchB, H - 1, lane, &wb);
  if (NIPAMD_WAIT_TIMES && a.counts && lane == 0) {
    unsigned long long* st = reinterpret_cast<unsigned long long*>(a.counts) + (size_t)gridDim.x * 4;
    st[blockIdx.x * 8 + (FWD ? 0 : 1)] = wa.cyc;
    st[blockIdx.x * 8 + 4 + (FWD ? 0 : 1)] = wb.cyc;
  }
  (void)active; (void)b;
}

// Log-likelihood of the forward filter (nip.c:1461-1474), kept by its
// partner: ll = sum_t log m2_t - log m1_t with m2_t = z2_t = sum(alpha_t) as
// published by the filter, and m1_t = sum(u_t o s) = 2^sc_t * y_{t-1},
// y_t = alpha_t . w (w = A s, the chain plan's `ts`), sc_t = -exp2(z2_{t-1}),
// y_{-1} = prior . w.  Products of mantissas with exponents carried apart.
// Lane L owns chain L & 15 and accumulates steps k = L >> 4 and k + 4 of
// every chunk, so y is an in-lane dot product; the four partial products of
// a chain are combined once at the end (write).
struct LL {
  double m2, m1, zmin;
  int e2, e1;
  double w[16];

  __device__ __forceinline__ void init(const ChainArgs& a, int lane, bool miss0) {
    double ym = 0.0;
#pragma unroll
    for (int i = 0; i < 16; i++) { w[i] = a.ts[i]; ym = __builtin_fma(a.pi[i], w[i], ym); }   // y_{-1}
    m2 = 1.0; m1 = ((lane >> 4) == 0 && !miss0) ? ym : 1.0; zmin = 1.0; e2 = 0; e1 = 0;
  }
  __device__ __forceinline__ double dot(const double (&v)[16]) const {
    double y0 = v[0] * w[0], y1 = v[1] * w[1], y2 = v[2] * w[2], y3 = v[3] * w[3];
#pragma unroll
    for (int i = 4; i < 16; i += 4) {
      y0 = __builtin_fma(v[i], w[i], y0); y1 = __builtin_fma(v[i + 1], w[i + 1], y1);
      y2 = __builtin_fma(v[i + 2], w[i + 2], y2); y3 = __builtin_fma(v[i + 3], w[i + 3], y3);
    }
    return (y0 + y1) + (y2 + y3);
  }
  // one step: y = alpha_t . w, z2 = sum(alpha_t); zf = the filter's z2 on
  // the steps where it rescales (rs), whose exponent is sc_{t+1}; `valid`
  // masks steps past the phase, last = (t == T-1).  Branch-free.
  // A step whose observation is missing (cm; nm: the next step's) enters
  // m1 with m2's own factor instead of y_{t-1} 2^sc_t: both masses are the
  // same there (nip.c:1461-1474 with no evidence entered), so such a step
  // contributes exactly nothing (a fully missing sequence has ll = 0).
  __device__ __forceinline__ void step(double y, double z2, double zf, bool rs, bool valid, bool last,
                                       bool cm = false, bool nm = false) {
    // factors enter as mantissa and exponent: between two rescales the
    // filter's vectors (hence z2 and y) may be far below 2^-500
    const double z = valid ? z2 : 1.0, yy = (valid && !last && !nm) ? y : 1.0;
    const double zz = (valid && cm) ? z2 : 1.0;
    zmin = __builtin_fmin(zmin, z);
    m2 *= __builtin_amdgcn_frexp_mant(z); e2 += __builtin_amdgcn_frexp_exp(z);
    m1 *= __builtin_amdgcn_frexp_mant(yy); e1 += __builtin_amdgcn_frexp_exp(yy);
    m1 *= __builtin_amdgcn_frexp_mant(zz); e1 += __builtin_amdgcn_frexp_exp(zz);
    e1 -= (valid && !last && !nm && rs) ? __builtin_amdgcn_frexp_exp(zf) : 0;   // 2^sc_{t+1}
  }
  __device__ __forceinline__ static double sum16(const double (&v)[16]) {
    double s0 = v[0] + v[1], s1 = v[2] + v[3], s2 = v[4] + v[5], s3 = v[6] + v[7];
    s0 += v[8] + v[9]; s1 += v[10] + v[11]; s2 += v[12] + v[13]; s3 += v[14] + v[15];
    return (s0 + s1) + (s2 + s3);
  }
  __device__ __forceinline__ void renorm() {
    const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
    const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
  }
  // combine the chain's four lanes (l, l ^ 32, l ^ 16) after renorm(); every
  // operation is symmetric, so all four lanes hold identical bits
  __device__ __forceinline__ void reduce(double& E2, double& E1) {
    auto pair32 = [](double x, auto f) {
      double xc = x;
      asm("" : "+v"(xc));   // the swap's second operand: a whole-double copy (one v_mov_b64)
      const auto rl = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
      const auto rh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
      return f(__hiloint2double((int)rh[0], (int)rl[0]), __hiloint2double((int)rh[1], (int)rl[1]));
    };
    auto pair16 = [](double x, auto f) {
      double xc = x;
      asm("" : "+v"(xc));   // the swap's second operand: a whole-double copy (one v_mov_b64)
      const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
      const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
      return f(__hiloint2double((int)rh[0], (int)rl[0]), __hiloint2double((int)rh[1], (int)rl[1]));
    };
    auto mul = [](double x, double y) { return x * y; };
    auto mn = [](double x, double y) { return __builtin_fmin(x, y); };
    auto add = [](double x, double y) { return x + y; };
    E2 = (double)e2; E1 = (double)e1;             // small integers: exact in a double
    m2 = pair16(pair32(m2, mul), mul);
    m1 = pair16(pair32(m1, mul), mul);
    zmin = pair16(pair32(zmin, mn), mn);
    E2 = pair16(pair32(E2, add), add);
    E1 = pair16(pair32(E1, add), add);
  }
  // lanes 0..15 (chain = lane) write the sequence's ll and status
  __device__ __forceinline__ void finish(const ChainArgs& a, long b0, int lane, double E2, double E1,
                                         unsigned dead_status) const {
    if (lane >= kMSeq) return;
    const long b = b0 + lane;
    if (b >= a.B) return;
    double ll = log(m2) - log(m1) + (E2 - E1) * 0.69314718055994530942;
    const bool dead = zmin == 0.0;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    if (a.status) a.status[b] = dead ? dead_status : 0u;
  }
  __device__ __forceinline__ void write(const ChainArgs& a, long b0, int lane, unsigned dead_status = 1u) {
    renorm();
    double E2, E1;
    reduce(E2, E1);
    finish(a, b0, lane, E2, E1, dead_status);
  }
};

// Prologue of a 16-sequence block: the evidence table and the sequences'
// observation codes into LDS (codes row Tr per chain, guard bytes = missing).
// zero() runs while the first loads are in flight (block-specific LDS init).
// The caller synchronises the block afterwards.
template <int NT, typename Z, int ESTR = 16>
__device__ __forceinline__ void stage_codes(const ChainArgs& a, long b0, int tid, double* Et, uint8_t* codes,
                                            int Tr, Z zero) {
  auto put_et = [&](int i) { Et[(i >> 4) * ESTR + (i & 15)] = a.Etab[i]; };   // row stride ESTR
  const int T = a.T;
  const int nseq = (int)((a.B - b0) < kMSeq ? (a.B - b0) : kMSeq);
  auto code_of = [&](int o) -> int { return o < 0 ? a.M : (o < a.M ? o : a.M + 1); };
  const bool fast = a.obs && a.obs_tstride == 1 && a.obs_bstride == T && (T & 3) == 0 && nseq == kMSeq;
  if (fast) {
    // contiguous [16][T] int32: every 16-byte load of the first pass issued
    // before anything else (T = 1024: all of them), the guard bytes and the
    // evidence table staged while they are in flight
    const int4* src = reinterpret_cast<const int4*>(a.obs + b0 * (long)T);
    const int n4 = (kMSeq * T) >> 2;
    constexpr int kLd = 4096 / NT;
    int4 r[kLd];
    auto load = [&](int i0) {
#pragma unroll
      for (int k = 0; k < kLd; k++) if (i0 + k * NT < n4) r[k] = src[i0 + k * NT];
    };
    auto put = [&](int i0) {
#pragma unroll
      for (int k = 0; k < kLd; k++) {
        const int i4 = i0 + k * NT;
        if (i4 < n4) {
          const int i = i4 << 2, cq = i / T, t = i - cq * T;
          const uint32_t packed = (uint32_t)code_of(r[k].x) | ((uint32_t)code_of(r[k].y) << 8) |
                                  ((uint32_t)code_of(r[k].z) << 16) | ((uint32_t)code_of(r[k].w) << 24);
          *reinterpret_cast<uint32_t*>(codes + cq * Tr + kMG + t) = packed;
        }
      }
    };
    load(tid);
    for (int i = tid; i < (a.M + 2) * 16; i += NT) put_et(i);
    const int gw = kMG / 4, tw = (Tr - kMG - T) / 4;             // guard words before / after
    for (int i = tid; i < kMSeq * (gw + tw); i += NT) {
      const int cq = i / (gw + tw), w = i - cq * (gw + tw);
      const int off = w < gw ? 4 * w : kMG + T + 4 * (w - gw);
      *reinterpret_cast<uint32_t*>(codes + cq * Tr + off) = 0x01010101u * (uint32_t)a.M;   // missing / guard
    }
    zero();
    put(tid);
    for (int i0 = tid + NT * kLd; i0 < n4; i0 += NT * kLd) {
      load(i0);
      put(i0);
    }
  } else {
    for (int i = tid; i < (a.M + 2) * 16; i += NT) put_et(i);
    for (int i = tid; i < kMSeq * Tr / 4; i += NT)
      reinterpret_cast<uint32_t*>(codes)[i] = 0x01010101u * (uint32_t)a.M;   // missing / guard
    zero();
    __syncthreads();
    if (a.obs) {
      for (int i = tid; i < nseq * T; i += NT) {
        const int cq = i / T, t = i - cq * T;
        codes[cq * Tr + kMG + t] =
            (uint8_t)code_of(a.obs[(b0 + cq) * a.obs_bstride + (long)t * a.obs_tstride + a.obs_col]);
      }
    }
  }
}

}  // namespace
}  // namespace nipamd
