// chain_kernels.hip -- gfx950 kernels for DBN slices that compile to a chain
// over one interface variable (the HMM-shaped DBN of SURVEY 8(d) config 2).
//
// What the reference computes per sequence (src/nip.c:1320-1581 over the
// join tree {prev,cur} - {cur,obs}, in == out clique) reduces to the
// following recursion over the N-state interface variable, with
//   A[x][y]  = in_clique original_p   (quirk-normalised P(cur|prev), huginnet.y:635)
//   e_t[y]   = obs clique original_p column of the observation, or its row
//              sum when the observation is missing (no evidence entered), or
//              0 for an out-of-range state (all-zero evidence vector)
//   alpha_t  = e_t o (A^T alpha_{t-1}),   alpha_{-1} = prior of prev
//   beta_t   = A (e_{t+1} o beta_{t+1}),  beta_{T-1} = 1
//   post_t   = normalise(alpha_t o beta_t)                  (nip.c:1535-1552)
//   ll       = sum_t log(sum(alpha_t)) - log(alpha_{t-1}^T A s)   (nip.c:1461-1474,
//              m2 and m1 of the reference, each measured on the same scale)
// The reference's backward pass passes gamma_{t+1}/alpha_t ratios
// (nip.c:1518-1529, "0 if den == 0", nippotential.c:488-491); algebraically
// the ratio cancels into the beta recursion above, so the two directions are
// independent and run CONCURRENTLY here (two-filter smoothing), which halves
// the sequential depth of the O(T) dependency chain.
//
// Mapping onto CDNA4: one 16-lane DPP row per (sequence, direction) chain,
// lane y owns state y.  Each step is a 16x16 mat-vec done in-lane from the
// row-gathered input vector (15 row_ror DPP moves), column of A resident in
// VGPRs, evidence table and observation codes resident in LDS.  Reductions
// are row_ror butterflies, which give bit-identical sums in all 16 lanes.
// Scale is carried as exact powers of two (ldexp/frexp), so no division or
// log is on the per-step path; ll is accumulated as a mantissa/exponent
// product and logged once.
//
// Phase A: forward computes alpha_0..alpha_{H-1}, backward beta_{T-1}..beta_H,
// both spilled to the scratch S[b][t][16].  A workgroup barrier.  Phase B:
// forward continues alpha_H..alpha_{T-1} and combines with beta_t from S;
// backward continues beta_{H-1}..beta_0 and combines with alpha_t from S.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdlib>
#include <cstdint>

#include "chain_kernels.h"
#include "diag.h"
#include "dpp_row.h"
#include "store_pol.h"

namespace nipamd {

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));   // an f64 MFMA accumulator

#ifndef NIPAMD_ESTEP_SWZ
#define NIPAMD_ESTEP_SWZ 0          // e_step: off-critical-path sums on ds_swizzle (A/B build)
#endif

// The same sum with the lane exchanges done by ds_swizzle (xor 8, 4, 2, 1
// inside the 32-lane swizzle group) on the LDS pipe instead of VALU DPP
// moves: 4 VALU instructions instead of 12, at LDS latency.  Lane i adds
// lane i ^ k where row_sum adds lane (i + k) mod 16; the partial sums are
// periodic at every level, so both pair the same values and the bits are
// identical.  Used for sums off the recursion's critical path.
template <int K>
__device__ __forceinline__ double swz_xor(double v) {
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), 0x1F | (K << 10));
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), 0x1F | (K << 10));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double row_sum_swz(double x) {
#if NIPAMD_ESTEP_SWZ
  // x is often a fresh product: keep the compiler from contracting it into
  // the first add (an fma would round differently from row_sum of the same
  // product, and e_step's missing steps rely on z2 == z1 to the bit)
  asm volatile("" : "+v"(x));
  x += swz_xor<8>(x);
  x += swz_xor<4>(x);
  x += swz_xor<2>(x);
  x += swz_xor<1>(x);
  return x;
#else
  return row_sum(x);
#endif
}

// exponent e such that x = m * 2^e, m in [0.5, 1); 0 for x == 0
__device__ __forceinline__ int exp2_of(double x) {
  return x != 0.0 ? __builtin_amdgcn_frexp_exp(x) : 0;
}

// x / c for the row-uniform normaliser c (x itself when c == 0, as
// nip_normalise_array leaves an all-zero array alone, nippotential.c:354):
// v_rcp_f64 refined by two Newton steps, then one multiply.
__device__ __forceinline__ double div_by(double x, double c) {
  if (c == 0.0) return x;
  double r = __builtin_amdgcn_rcp(c);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  return x * r;
}

#ifndef NIPAMD_ESTEP_CHUNK
#define NIPAMD_ESTEP_CHUNK 8
#endif
#ifndef NIPAMD_ESTEP_WAVES
#define NIPAMD_ESTEP_WAVES 2        // e_step: waves per SIMD the register budget is sized for
#endif

// Per-chunk prefetch registers: evidence values from LDS and (phase B) the
// other direction's interface vector from HBM, issued one chunk ahead so no
// step waits on a fresh load.  KC steps per unrolled chunk.
template <int KC>
struct Prefetch {
  double e[KC];
  double s[KC];
  int c[KC];           // observation codes (E-step: M1 count row)
};

}  // namespace

constexpr int kChainsPerBlock = 8;   // 8 sequences; waves 0-1 forward, 2-3 backward
constexpr int kThreads = 256;

namespace {

constexpr int kGuard = kScratchGuard;   // guard steps on both sides of every codes / S row

// Per-row view of a chain: rows 0,1 of every wave run the forward filter of
// sequences 2w, 2w+1; rows 2,3 run the backward filter of the same two
// sequences, so every wave issues the same instruction stream (the two
// directions differ only in data: A column vs row, time direction, and which
// of u / u*e is the interface vector).
struct ChainCtx {
  const double* Et;        // LDS evidence table, this lane's column (Et + y)
  const uint8_t* codes;    // LDS codes of this sequence; codes[-kGuard .. T+kGuard)
  const double* Sload;     // S row of this sequence (+y); guard steps both sides
  double* Sstore;          // same, or a sink for lanes that must not write
  long Sstride;            // 16, or 0 for the sink
  double* Pstore;          // posterior of this sequence (+off+y), or a sink
  long Pstride;            // post_tstride, or 0 for the sink
};

// Prefetch kChunk steps of this row starting at t0 in direction dir.  The
// guard steps make every index in [-kGuard, T + kGuard) readable, so the tail
// of a phase needs no clamping (its values are never used).
template <int KC>
__device__ __forceinline__ void load_chunk(const ChainCtx& c, Prefetch<KC>& p, int t0, int dir,
                                           bool with_s) {
  int code[KC];
#pragma unroll
  for (int j = 0; j < KC; j++) {
    const int t = t0 + dir * j;
    code[j] = c.codes[t];
    if (with_s) p.s[j] = c.Sload[(long)t * 16];
  }
#pragma unroll
  for (int j = 0; j < KC; j++) { p.e[j] = c.Et[code[j] * 16]; p.c[j] = code[j]; }
}

// n wave-uniform steps with one-chunk-ahead ping-pong prefetch.
template <int KC, typename Step>
__device__ __forceinline__ void run_phase(const ChainCtx& c, int n, int t0, int dir,
                                          bool with_s, Step&& step) {
  Prefetch<KC> pa, pb;
  if (n <= 0) return;
  load_chunk(c, pa, t0, dir, with_s);
  for (int base = 0; base < n; base += 2 * KC) {
    load_chunk(c, pb, t0 + dir * (base + KC), dir, with_s);
#pragma unroll
    for (int j = 0; j < KC; j++)
      if (base + j < n) step(t0 + dir * (base + j), pa.e[j], pa.s[j], pa.c[j], j);
    if (base + KC >= n) break;
    load_chunk(c, pa, t0 + dir * (base + 2 * KC), dir, with_s);
#pragma unroll
    for (int j = 0; j < KC; j++)
      if (base + KC + j < n) step(t0 + dir * (base + KC + j), pb.e[j], pb.s[j], pb.c[j], j);
  }
}

}  // namespace

// ESTEP = false: forward_backward_inference (posteriors + ll).
// ESTEP = true:  e_step (nip.c:1708-2007): the same two filters; phase B
// accumulates the expected counts of every family (see chain_estep_slab).
template <bool ESTEP>
__global__ __launch_bounds__(kThreads, ESTEP ? NIPAMD_ESTEP_WAVES : 2)
void chain_kernel(ChainArgs a) {
  constexpr int KC = ESTEP ? NIPAMD_ESTEP_CHUNK : 8;   // steps per unrolled chunk
  static_assert(KC % 4 == 0, "the ll products renormalise every 4th step of a chunk");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* Et = reinterpret_cast<double*>(smem);                       // [(M+2)][16]
  uint8_t* codes = smem + (size_t)(a.M + 2) * 16 * sizeof(double);    // [8][Tr]
  // E-step: per (sequence, direction) M1 count tables [(M+2)][16], lane-owned
  double* Htab = reinterpret_cast<double*>(
      codes + (((size_t)kChainsPerBlock * chain_codes_row(a.T) + 15) & ~(size_t)15));

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int y = lane & 15, row = lane >> 4;
  const bool fwd = row < 2;                       // per row (lane-varying)
  const int seq = wave * 2 + (row & 1);           // 0..7 within the block
  const long b0 = (long)blockIdx.x * kChainsPerBlock;
  const long b = b0 + seq;
  const bool active = b < a.B;
  const int T = a.T, H = a.H;
  const int Tr = chain_codes_row(T);              // kGuard + T rounded + kGuard

  // --- stage the evidence table and this block's observation codes in LDS
  for (int i = tid; i < (a.M + 2) * 16; i += kThreads) Et[i] = a.Etab[i];
  const int nseq = (int)((a.B - b0) < kChainsPerBlock ? (a.B - b0) : kChainsPerBlock);
  auto code_of = [&](int o) -> int { return o < 0 ? a.M : (o < a.M ? o : a.M + 1); };
  for (int i = tid; i < kChainsPerBlock * Tr; i += kThreads) codes[i] = (uint8_t)a.M;  // missing / guard
  if (ESTEP)
    for (int i = tid; i < kChainsPerBlock * 2 * (a.M + 2) * 16; i += kThreads) Htab[i] = 0.0;
  __syncthreads();
  if (a.obs && a.obs_tstride == 1 && a.obs_bstride == T && (T & 3) == 0 && nseq == kChainsPerBlock) {
    // contiguous [8][T] int32 block: 16-byte loads, all issued before use
    const int4* src = reinterpret_cast<const int4*>(a.obs + b0 * (long)T);
    const int n4 = (kChainsPerBlock * T) >> 2;
    for (int i0 = tid; i0 < n4; i0 += kThreads * 8) {
      int4 r[8];
#pragma unroll
      for (int k = 0; k < 8; k++) if (i0 + k * kThreads < n4) r[k] = src[i0 + k * kThreads];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i4 = i0 + k * kThreads;
        if (i4 < n4) {
          const int i = i4 << 2, c = i / T, t = i - c * T;
          const uint32_t packed = (uint32_t)code_of(r[k].x) | ((uint32_t)code_of(r[k].y) << 8) |
                                  ((uint32_t)code_of(r[k].z) << 16) | ((uint32_t)code_of(r[k].w) << 24);
          *reinterpret_cast<uint32_t*>(codes + c * Tr + kGuard + t) = packed;
        }
      }
    }
  } else if (a.obs) {
    for (int i = tid; i < nseq * T; i += kThreads) {
      const int c = i / T, t = i - c * T;
      codes[c * Tr + kGuard + t] =
          (uint8_t)code_of(a.obs[(b0 + c) * a.obs_bstride + (long)t * a.obs_tstride + a.obs_col]);
    }
  }

  double C[16];   // fwd rows: column y of A (C[k] = A[k][y]); bwd rows: row y (A[y][k])
#pragma unroll
  for (int k = 0; k < 16; k++) C[k] = fwd ? a.A[k * 16 + y] : a.A[y * 16 + k];
  __syncthreads();
  const double s_y = Et[a.M * 16 + y];                    // sum_m E[y][m]

  // per-lane pointers; lanes that must not write get a sink with stride 0
  double* const sink = a.S + (size_t)(a.B + 1) * chain_scratch_row(T) + y;
  double* const Srow = a.S + (size_t)(active ? b : 0) * chain_scratch_row(T) + (size_t)kGuard * 16 + y;
  const bool ystore = active && y < a.N && a.post;
  ChainCtx cx;
  cx.Et = Et + y;
  cx.codes = codes + seq * Tr + kGuard;
  cx.Sload = Srow;
  cx.Sstore = active ? Srow : sink;
  cx.Sstride = active ? 16 : 0;
  cx.Pstore = ystore ? a.post + (size_t)b * a.post_bstride + a.post_off + y : sink;
  cx.Pstride = ystore ? a.post_tstride : 0;

  // chain state: x = this lane's entry of the next mat-vec input
  //   fwd: alpha_{t-1} (starts at the prior of prev, nip.c:1431 use_priors)
  //   bwd: g_{t+1} = e_{t+1} o beta_{t+1}  (starts at e_{T-1} o 1)
  double x;
  int sc = 0;
  double m2 = 1.0, m1 = 1.0;   // fwd: running products of m2 / m1 (mantissas)
  int e2 = 0, e1 = 0;          //      and their binary exponents
  bool dead = false;
  if (fwd) {
    x = a.pi[y];
  } else {
    const double beta = y < a.N ? 1.0 : 0.0;
    cx.Sstore[(long)(T - 1) * cx.Sstride] = beta;        // beta_{T-1}; T-1 >= H
    x = Et[cx.codes[T - 1] * 16 + y] * beta;
  }
  {
    const int k = exp2_of(row_sum(x));
    if (!fwd) sc = -k;
  }

  // E-step accumulators.  K[k]: fwd rows (lane y) sum xi(x=k, y); bwd rows
  // (lane x) sum xi(x, y=k) -- both without the A(x,y) factor, applied once
  // after the batch reduction.  Hrow: this chain's M1 count table column y.
  double K[16];
#pragma unroll
  for (int k = 0; k < 16; k++) K[k] = 0.0;
  double* Hrow = Htab + ((size_t)(seq * 2 + (fwd ? 0 : 1)) * (a.M + 2)) * 16 + y;

  // One step of either direction, branch-free.  u = A^T x (fwd) or A x (bwd),
  // scaled; p = e o u.  fwd: alpha_t = p;  bwd: beta_t = u, next input p.
  auto step = [&](int t, double e, double other, int code, bool combine, int j) {
    const double u = __builtin_ldexp(dot_bcast(x, C), sc);
#if NIPAMD_ESTEP_SWZ
    double p = u * e;
    if (ESTEP) asm volatile("" : "+v"(p));           // the same rounded product as z1's (see row_sum_swz)
#else
    const double p = u * e;
#endif
    const double keep = fwd ? p : u;                 // interface vector at time t
    const double z2 = row_sum(p);                    // fwd: m2 ; bwd: scale
#ifdef NIPAMD_ABLATE_NO_LL
    const double z1 = 0.0;
#else
    const double z1 = ESTEP ? row_sum_swz(u * s_y) : row_sum(u * s_y);   // fwd: m1
#endif
#ifdef NIPAMD_ABLATE_NO_STORE     // timing-only ablation build (wrong results)
    if (0) {
#else
    if (!combine) {
#endif
      cx.Sstore[(long)t * cx.Sstride] = keep;
    } else if (!ESTEP) {
      const double pr = keep * other;
#ifdef NIPAMD_ABLATE_NO_POSTNORM
      cx.Pstore[(long)t * cx.Pstride] = pr;
#else
      cx.Pstore[(long)t * cx.Pstride] = div_by(pr, row_sum(pr));
#endif
    } else {
      // e_step families at time t (nip.c:1925-1967), normalised by c_t:
      //   M1:  post_t(y) at row = observation code (missing -> row M, folded
      //        into E[y][m]/s(y) after the reduction; invalid -> row M+1)
      //   P1:  xi_t(x,y) = alpha_{t-1}(x) A(x,y) e_t(y) beta_t(y) / c_t   (fwd, t >= H)
      //        xi_{t+1}(x,y) = alpha_t(x) A(x,y) g_{t+1}(y) / c_t        (bwd, t+1 < H)
      const double pr = keep * other;
      const double c = row_sum_swz(pr);
      const double q = div_by(pr, c);
      Hrow[code * 16] += q;
      const double rc = c != 0.0 ? __builtin_ldexp(div_by(1.0, c), sc) : 0.0;
      const double w = fwd ? e * other * rc : (t + 1 < a.H ? other * rc : 0.0);
      acc_bcast(K, x, w);
    }
#ifndef NIPAMD_ABLATE_NO_LL
    dead |= (z2 == 0.0);
    m2 *= z2; m1 *= z1;
    if ((j & 3) == 3) {                              // renormalise every 4 steps
      const int k2 = exp2_of(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
      const int k1 = exp2_of(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
    }
#endif
    sc = -exp2_of(z2);
    x = p;
  };

  const int dir = fwd ? 1 : -1;
  // phase A: fwd t = 0..H-1 ; bwd t = T-2 .. H  (bwd has one step fewer for even T)
  {
    const int nf = H, nb = T - 1 - H, n = nf < nb ? nf : nb;
    const int t0 = fwd ? 0 : T - 2;
    run_phase<KC>(cx, n, t0, dir, false, [&](int t, double e, double o, int c, int j) { step(t, e, o, c, false, j); });
    if (nf != nb && (fwd ? nf : nb) > n) {             // peeled tail: rows with one more step
      const int t = t0 + dir * n;
      step(t, cx.Et[cx.codes[t] * 16], 0.0, cx.codes[t], false, 3);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // phase B: fwd t = H..T-1 combined with beta_t ; bwd t = H-1..0 combined with alpha_t
  {
    const int nf = T - H, nb = H, n = nf < nb ? nf : nb;
    const int t0 = fwd ? H : H - 1;
    run_phase<KC>(cx, n, t0, dir, true, [&](int t, double e, double o, int c, int j) { step(t, e, o, c, true, j); });
    if (nf != nb && (fwd ? nf : nb) > n) {
      const int t = t0 + dir * n;
      step(t, cx.Et[cx.codes[t] * 16], cx.Sload[(long)t * 16], cx.codes[t], true, 3);
    }
  }
  if (ESTEP) {
    // one more backward step with alpha_{-1} = prior of prev: its posterior is
    // the P0 count (family of the previous-slice variable at t = 0) and its
    // xi is xi_0 (when the forward rows did not cover t = 0, i.e. H > 0)
    const double pi_y = a.pi[y];
    const double u = __builtin_ldexp(dot_bcast(x, C), sc);   // bwd: beta_{-1}
    const double pr = pi_y * u;
    const double c = row_sum(pr);
    const double q = div_by(pr, c);
    const double rc = c != 0.0 ? __builtin_ldexp(div_by(1.0, c), sc) : 0.0;
    const double w = (!fwd && a.H > 0) ? pi_y * rc : 0.0;
    acc_bcast(K, x, w);
    double* slab = a.counts + (size_t)(active ? b : 0) * chain_estep_slab(a.M);
    if (active && !fwd) slab[chain_slab_p0(a.M) + y] = q;
    if (active) {
#pragma unroll
      for (int k = 0; k < 16; k++)
        slab[(fwd ? kSlabKf + k * 16 + y : kSlabKb + y * 16 + k)] = K[k];
    }
    __syncthreads();
    for (int i = tid; i < kChainsPerBlock * 2 * (a.M + 2) * 16; i += kThreads) {
      const int sq = i / (2 * (a.M + 2) * 16), r = i - sq * 2 * (a.M + 2) * 16;
      if (b0 + sq < a.B) a.counts[(size_t)(b0 + sq) * chain_estep_slab(a.M) + kSlabH + r] = Htab[i];
    }
  }
  if (fwd && active && y == 0) {
    double ll = log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    // e_step's BAD_LUCK (m1 <= 0 || m2 <= 0, nip.c:1827-1854) is the same
    // event as a zero mass here (m2 <= m1 since e <= s elementwise)
    if (a.status) a.status[b] = dead ? (ESTEP ? 3u : 1u) : 0u;
  }
}

// ---------------------------------------------------------------------------
// e_step, direction-uniform waves (chain_estep16_kernel, the default e_step).
//
// The same two filters and per-sequence slab as chain_kernel<true>, with two
// changes to the work per step (the kernel is bound by the SIMDs' f64 issue,
// DESIGN.md 4):
//  * waves are direction-uniform: a block holds 16 sequences, waves 0-3 run
//    the forward rows (4 sequences each), waves 4-7 the backward rows, so
//    each SIMD holds one wave of each direction, and the backward rows skip
//    what only the ll needs (the m1 row sum, the mass products);
//  * phase B normalises analytically: sum_y alpha_t(y) beta_t(y) = Z for
//    every t, and both filters carry their scale as an exact power of two
//    per step (alpha^_t = alpha_t 2^Ef_t, beta^_t = beta_t 2^Eb_t; the
//    exponents travel with the phase-A messages through the scratch), so
//    c_t = Z 2^(Ef_t + Eb_t): one row sum at the phase's first step gives
//    1 / c_H, and every later step's posterior and xi weight is a multiply
//    and an ldexp instead of a row sum, a division and a reciprocal.  The
//    posteriors then sum to 1 within the filters' rounding drift (~1e-13
//    relative over T = 1024), well inside DESIGN.md's count tolerance.
// Per-sequence slabs (chain_estep_slab layout) as chain_kernel<true>, so
// tree64_kernel and estep_finalize_kernel are shared.
// NSEQ sequences per block (16: 8 waves, two per SIMD; 24: 12 waves, three
// per SIMD), waves 0 .. NSEQ/4-1 forward, the rest backward
constexpr int kE16RowMul = 48;                 // scratch rows rounded to a multiple of every NSEQ
#ifndef NIPAMD_E16_PIPE
#define NIPAMD_E16_PIPE 1                      // phase B's count cells read one step ahead (0: A/B builds)
#endif
#ifndef NIPAMD_E16_BWD_MAXEXP
#define NIPAMD_E16_BWD_MAXEXP 1                // backward rows rescale by the largest exponent (0: A/B builds)
#endif
#ifndef NIPAMD_E16_FWD_SPARSE
#define NIPAMD_E16_FWD_SPARSE 1                // proper mode: forward rows rescale every 4th step (0: A/B builds)
#endif
#ifndef NIPAMD_ESTEP_PRIO
#define NIPAMD_ESTEP_PRIO 0
#endif
#ifndef NIPAMD_WAIT_TIMES
#define NIPAMD_WAIT_TIMES 0                    // stamps builds: per-wave phase cycle stamps into a.diag
#endif

namespace {

__host__ __device__ inline long estep16_xrow(int T) { return (long)T + 2 * kGuard; }

template <int NE>
struct E16Ctx {
  const double* Et;        // LDS evidence tables, this lane's column (Et + y)
  const uint8_t* codes[NE];   // LDS codes of this sequence per leaf child; codes[k][-kGuard .. T+kGuard)
  int erow16[NE];          // first row of child k's table, times 16
  const double* Sload;     // scratch message row of this sequence (+y)
  double* Sstore;          // same, or a sink
  long Sstride;            // 16, or 0 for the sink
  const int* Xload;        // scratch exponent row of this sequence
};

template <int KC, int NE>
struct Prefetch16 {
  double e[KC];            // the step's evidence column: product over the children
  double s[KC];
  int c[KC][NE];           // count-table rows (child k's first row + its code)
  int x[KC];
};

template <int KC, int NE>
__device__ __forceinline__ void load_chunk16(const E16Ctx<NE>& c, Prefetch16<KC, NE>& p, int t0, int dir,
                                             bool with_s) {
#pragma unroll
  for (int j = 0; j < KC; j++) {
    const int t = t0 + dir * j;
#pragma unroll
    for (int k = 0; k < NE; k++) p.c[j][k] = c.erow16[k] + c.codes[k][t] * 16;
    if (with_s) {
      p.s[j] = load_pol<NIPAMD_SCR_NTLD>(c.Sload + (long)t * 16);
      p.x[j] = load_pol<NIPAMD_SCR_NTLD>(c.Xload + t);
    }
  }
#pragma unroll
  for (int j = 0; j < KC; j++) {
    double e = c.Et[p.c[j][0]];
#pragma unroll
    for (int k = 1; k < NE; k++) e *= c.Et[p.c[j][k]];
    p.e[j] = e;
  }
}

// step(t, e, s, x, count rows of t, j, count rows of the next step): the
// next step's rows are in the other buffer at a chunk's last step (loaded a
// chunk ahead; past the phase's end they are guard codes, valid rows)
template <int KC, int NE, typename Step>
__device__ __forceinline__ void run_phase16(const E16Ctx<NE>& c, int n, int t0, int dir, bool with_s, Step&& step) {
  Prefetch16<KC, NE> pa, pb;
  if (n <= 0) return;
  load_chunk16(c, pa, t0, dir, with_s);
  for (int base = 0; base < n; base += 2 * KC) {
    load_chunk16(c, pb, t0 + dir * (base + KC), dir, with_s);
#pragma unroll
    for (int j = 0; j < KC; j++)
      if (base + j < n) step(t0 + dir * (base + j), pa.e[j], pa.s[j], pa.x[j], pa.c[j], j, j + 1 < KC ? pa.c[j + 1] : pb.c[0]);
    if (base + KC >= n) break;
    load_chunk16(c, pa, t0 + dir * (base + 2 * KC), dir, with_s);
#pragma unroll
    for (int j = 0; j < KC; j++)
      if (base + KC + j < n)
        step(t0 + dir * (base + KC + j), pb.e[j], pb.s[j], pb.x[j], pb.c[j], j, j + 1 < KC ? pb.c[j + 1] : pa.c[0]);
  }
}

// sum_k x[lane k] * c[k] with two accumulators (dot_bcast has four): two
// zeroing moves and one add per mat-vec instead of four and three; the
// other wave on the SIMD covers the longer fma chains
__device__ __forceinline__ double dot2_bcast(double x, const double (&c)[16]) {
  double a0 = 0.0, a1 = 0.0;
  fmac_bcast<0, true>(a0, x, c[0]);   fmac_bcast<1, false>(a1, x, c[1]);
  fmac_bcast<2, false>(a0, x, c[2]);  fmac_bcast<3, false>(a1, x, c[3]);
  fmac_bcast<4, false>(a0, x, c[4]);  fmac_bcast<5, false>(a1, x, c[5]);
  fmac_bcast<6, false>(a0, x, c[6]);  fmac_bcast<7, false>(a1, x, c[7]);
  fmac_bcast<8, false>(a0, x, c[8]);  fmac_bcast<9, false>(a1, x, c[9]);
  fmac_bcast<10, false>(a0, x, c[10]); fmac_bcast<11, false>(a1, x, c[11]);
  fmac_bcast<12, false>(a0, x, c[12]); fmac_bcast<13, false>(a1, x, c[13]);
  fmac_bcast<14, false>(a0, x, c[14]); fmac_bcast<15, false>(a1, x, c[15]);
  return a0 + a1;
}

// 16-lane integer max of the lanes' binary exponents (zeros excluded): the
// rescale exponent of a proper model's forward rows, every step -- four DPP
// integer ops where the row's f64 sum was twelve (any power of two serves:
// the ll no longer reads the step masses, posteriors and xi are scale-free)
__device__ __forceinline__ int row_max_exp_rescale(double p) {
  int e = p != 0.0 ? __builtin_amdgcn_frexp_exp(p) : -0x40000;
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x128, 0xF, 0xF, true));   // row_ror:8
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x124, 0xF, 0xF, true));   // row_ror:4
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x122, 0xF, 0xF, true));   // row_ror:2
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x121, 0xF, 0xF, true));   // row_ror:1
  return e > -0x40000 ? -e : 0;
}

// One direction's rows of a block (FWD: waves 0-3, backward: waves 4-7).
// PR: a proper model (ChainArgs::proper): the ll is log of the final forward
// mass minus its exponent, so the forward rows keep no m2 / m1 products and
// rescale by the row's largest exponent, and the backward rows sum no m1.
template <bool FWD, int KC, int NE, int PRM>
__device__ __forceinline__ void estep16_rows(const ChainArgs& a, const double* Et, const uint8_t* codes,
                                             double* Htab, double* m1x, double* kdl, double* p0l, int lane, int grp,
                                             long b0, int nseqb) {
  constexpr bool PR = PRM != 0;                     // proper mode
  constexpr bool SP = PRM == 2;                     // and the forward rows may rescale every 4th step
  const int y = lane & 15, row = lane >> 4;
  const int seq = grp * 4 + row;                    // within the block
  const long b = b0 + seq;
  const bool active = b < a.B;
  const int T = a.T, H = a.H, M = a.M;
  const int Tr = chain_codes_row(T);

  double C[16];   // forward: column y of A (C[k] = A[k][y]); backward: row y (A[y][k])
#pragma unroll
  for (int k = 0; k < 16; k++) C[k] = FWD ? a.A[k * 16 + y] : a.A[y * 16 + k];
  // s(y): the product of the children's missing rows (each child's row
  // sums; the factor of a step that observes nothing)
  auto s_of = [&](int j) {
    double v = Et[(a.erow[0] + a.eM[0]) * 16 + j];
#pragma unroll
    for (int k = 1; k < NE; k++) v *= Et[(a.erow[k] + a.eM[k]) * 16 + j];
    return v;
  };
  const double s_y = s_of(y);
  // backward rows: (A s)(x) for lane x -- the phase-A steps' m1 (below)
  double As = 0.0;
  if (!FWD) {
#pragma unroll
    for (int k = 0; k < 16; k++) As = __builtin_fma(C[k], s_of(k), As);
  }

  const long nrow = (a.B + kE16RowMul - 1) / kE16RowMul * kE16RowMul;
  double* const sink = a.S + (size_t)(nrow + 1) * chain_scratch_row(T) + y;
  double* const Srow = a.S + (size_t)(active ? b : 0) * chain_scratch_row(T) + (size_t)kGuard * 16 + y;
  int* const X = reinterpret_cast<int*>(a.S + (size_t)(nrow + 2) * chain_scratch_row(T));
  int* const Xrow = X + (size_t)(active ? b : 0) * estep16_xrow(T) + kGuard;
  E16Ctx<NE> cx;
  cx.Et = Et + y;
#pragma unroll
  for (int k = 0; k < NE; k++) {
    cx.codes[k] = codes + ((size_t)k * nseqb + seq) * Tr + kGuard;
    cx.erow16[k] = a.erow[k] * 16;
  }
  cx.Sload = Srow;
  cx.Sstore = active ? Srow : sink;
  cx.Sstride = active ? 16 : 0;
  cx.Xload = Xrow;
  const bool xw = active && y == 0;

  // chain state: x = this lane's entry of the next mat-vec input, ex its
  // exponent (x = message * 2^ex): forward alpha^_{t-1}, backward
  // g_{t+1} = e_{t+1} o beta^_{t+1}
  double x;
  int sc = 0, ex = 0;
  // ll = sum_t log m2_t - log m1_t (nip.c:1461-1474): the forward rows carry
  // every m2 and phase B's m1; phase A's m1 (t < H), (alpha^_{t-1} . A s) at
  // scale 2^Ef_{t-1} (the scales telescope to Ef_{H-1}, the m2 being at
  // 2^Ef_t), is summed by the backward rows in their phase B, where alpha^_t
  // arrives from the scratch anyway, and handed over through LDS -- the
  // split that measured best (the phase-B backward rows are the critical ones)
  double m2 = 1.0, m1 = 1.0;   // running products (mantissas)
  int e2 = 0, e1 = 0;          // and their binary exponents
  // rows past the batch run on zeros: every product they feed the block's
  // matrix-core sums is then 0 without a select per step
  if (FWD) {
    x = active ? a.pi[y] : 0.0;
  } else {
    const double beta = (active && y < a.N) ? 1.0 : 0.0;
    cx.Sstore[(long)(T - 1) * cx.Sstride] = beta;     // beta_{T-1} = 1, exponent 0
    if (xw) Xrow[T - 1] = 0;
    double e0 = Et[cx.erow16[0] + cx.codes[0][T - 1] * 16 + y];
#pragma unroll
    for (int k = 1; k < NE; k++) e0 *= Et[cx.erow16[k] + cx.codes[k][T - 1] * 16 + y];
    x = e0 * beta;
    sc = -exp2_of(row_sum(x));
  }

  // xi of the wave's four sequences on the matrix core: the rows' x (lane:
  // row r, state i) is the A operand (i, k = r) and w (row r, state j) the B
  // operand (k = r, j) of one v_mfma_f64_16x16x4 per step, D[i][j] +=
  // sum_r x_r(i) w_r(j) -- the sixteen broadcast fmas of chain_kernel<true>'s
  // per-row outer product as one instruction, summed over the wave's rows
  v4d Kd = {0.0, 0.0, 0.0, 0.0};
  double* Hrow = Htab + ((size_t)(seq * 2 + (FWD ? 0 : 1)) * (M + 2)) * 16 + y;
  double rc0 = 0.0;           // phase B: 1 / c at the phase's first step
  int E0 = 0;                 //          and that step's exponent sum

  // phase B: the step's count cells (one per child).  E16_PIPE: read one
  // step ahead, right after this step's write (the wave's LDS operations
  // complete in order, so a next step with the same cell reads the new
  // value), and consumed a whole step later; otherwise read at the step's
  // start, pinned there (the compiler then waits for it at once)
  double hn[NE];
#pragma unroll
  for (int k = 0; k < NE; k++) hn[k] = 0.0;
  // one step; combine: phase B (posterior, M1 count, xi), first: its first step
  auto step = [&](int t, double e, double other, int xo, const int (&code)[NE], bool combine, bool first, int j,
                  const int (&cnext)[NE]) {
    double hv[NE];
#pragma unroll
    for (int k = 0; k < NE; k++) {
      hv[k] = 0.0;
      if (combine) {
        if (NIPAMD_E16_PIPE) {
          hv[k] = hn[k];
        } else {
          hv[k] = Hrow[code[k]];
          asm volatile("" : "+v"(hv[k]));            // keep the read here
        }
      }
    }
    const double u = __builtin_ldexp(dot2_bcast(x, C), sc);
    const int eu = ex + sc;                          // exponent of u (and of p)
    const double p = u * e;
    const double keep = FWD ? p : u;                 // alpha^_t / beta^_t
    // the forward rows need every step's mass (m2); the backward rows only
    // rescale, every 4th step (j is the unrolled step index: no branch) --
    // four evidence factors cannot underflow, and the exponents carry any scale
    const bool rescale = (FWD && !PR) || (j & 3) == 3;
    // (the backward rows' rescale needs no sum: the row's largest binary
    // exponent, four integer DPP maxes, serves as well -- NIPAMD_E16_BWD_MAXEXP)
    constexpr bool bmx = !FWD && NIPAMD_E16_BWD_MAXEXP;
    const double z2 = (rescale && !bmx) ? row_sum(p) : 1.0;
    if (!FWD && combine && !PR) {
      // the m1 of the forward rows' phase-A step t + 1 (< H) from alpha^_t = other
      if (!first) m1 *= row_sum(other * As);           // t + 1 < H: every step but the first
    }
    if (!combine) {
      store_pol<NIPAMD_SCR_NT>(cx.Sstore + (long)t * cx.Sstride, keep);
      if (xw) store_pol<NIPAMD_SCR_NT>(Xrow + t, eu);                          // one lane per row (exec-masked store)
    } else {
      const double pr = keep * other;                // alpha^_t beta^_t = Z gamma_t 2^(eu + xo)
      if (first) {
        const double c = row_sum(pr);
        rc0 = c != 0.0 ? div_by(1.0, c) : 0.0;
        E0 = eu + xo;
      }
      const double q = __builtin_ldexp(pr * rc0, E0 - (eu + xo));
#pragma unroll
      for (int k = 0; k < NE; k++) Hrow[code[k]] = hv[k] + q;
      if (NIPAMD_E16_PIPE) {
#pragma unroll
        for (int k = 0; k < NE; k++) hn[k] = Hrow[cnext[k]];
      }
      // xi_t (forward, x = alpha^_{t-1}) / xi_{t+1} (backward, x = g_{t+1}, t + 1 < H):
      // x(.) A e_t beta_t / Z resp. alpha_t A g_{t+1} / Z, the A factor applied after the reduction
      const double f = __builtin_ldexp(rc0, E0 - (ex + xo));
      // (backward: the phase's first step, t = H - 1, has no xi_{t+1}: xi_H is the forward rows')
      const double w = FWD ? e * other * f : (first ? 0.0 : other * f);
      Kd = FWD ? __builtin_amdgcn_mfma_f64_16x16x4f64(x, w, Kd, 0, 0, 0)
               : __builtin_amdgcn_mfma_f64_16x16x4f64(w, x, Kd, 0, 0, 0);
    }
    if (FWD && !PR) {
      m2 *= z2;
      if (combine) m1 *= row_sum(u * s_y);
    }
    if (!PR && (FWD || combine) && (j & 3) == 3) {  // renormalise every 4 steps (0 stays 0)
      if (FWD) { const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2; }
      const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
    }
    // the scale of the next step (a zero mass keeps every later vector 0,
    // whatever the exponent: no zero test)
    // (SP: the forward rows rescale every 4th step as the backward rows do,
    // when the host's bound says a product of the two directions' vectors
    // cannot underflow -- engine.cpp estep16_sparse_ok; the final ll reads
    // the exponent)
    if (FWD && PR) sc = (!(SP && NIPAMD_E16_FWD_SPARSE) || (j & 3) == 3) ? row_max_exp_rescale(p) : 0;
    else if (bmx) sc = rescale ? row_max_exp_rescale(p) : 0;
    else sc = rescale ? -__builtin_amdgcn_frexp_exp(z2) : 0;
    x = p;
    ex = eu;
  };

  constexpr int dir = FWD ? 1 : -1;
  unsigned long long st[4] = {0, 0, 0, 0};
  if (NIPAMD_WAIT_TIMES) st[0] = __builtin_readcyclecounter();
  // phase A: forward t = 0..H-1; backward t = T-2..H
  run_phase16<KC, NE>(cx, FWD ? H : T - 1 - H, FWD ? 0 : T - 2, dir, false,
                      [&](int t, double e, double o, int xo, const int (&c)[NE], int j, const int (&cn)[NE]) {
                        step(t, e, o, xo, c, false, false, j, cn);
                      });
  const int efa = ex;                                // forward: Ef_{H-1}, the phase-A m1 exponents' sum
  if (NIPAMD_WAIT_TIMES) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); st[1] = __builtin_readcyclecounter(); }
  __syncthreads();
  if (NIPAMD_WAIT_TIMES) st[2] = __builtin_readcyclecounter();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // phase B: forward t = H..T-1 with beta_t; backward t = H-1..0 with alpha_t
  {
    const int n = FWD ? T - H : H;
    const int t0 = FWD ? H : H - 1;
    if (n > 0) {
      int c0[NE];
#pragma unroll
      for (int k = 0; k < NE; k++) c0[k] = cx.erow16[k] + cx.codes[k][t0] * 16;
      double e0 = cx.Et[c0[0]];
#pragma unroll
      for (int k = 1; k < NE; k++) e0 *= cx.Et[c0[k]];
      int c1[NE];                                    // the next step's rows (t0 + dir: a guard code at most)
#pragma unroll
      for (int k = 0; k < NE; k++) {
        c1[k] = cx.erow16[k] + cx.codes[k][t0 + dir] * 16;
        if (NIPAMD_E16_PIPE) hn[k] = Hrow[c0[k]];
      }
      step(t0, e0, cx.Sload[(long)t0 * 16], cx.Xload[t0], c0, true, true, 3, c1);
      run_phase16<KC, NE>(cx, n - 1, t0 + dir, dir, true,
                          [&](int t, double e, double o, int xo, const int (&c)[NE], int j, const int (&cn)[NE]) {
                            step(t, e, o, xo, c, true, false, j, cn);
                          });
    }
  }
  if (NIPAMD_WAIT_TIMES) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); st[3] = __builtin_readcyclecounter(); }
  if (NIPAMD_WAIT_TIMES && a.diag && lane == 0) {
    unsigned long long* d = a.diag + ((size_t)blockIdx.x * 16 + (FWD ? 0 : 8) + grp) * 4;
    d[0] = st[1] - st[0];                            // phase A
    d[1] = st[2] - st[1];                            // phase barrier wait
    d[2] = st[3] - st[2];                            // phase B
  }
  if (!FWD && H > 0 && !PR) {
    // the phase-A m1 part for the forward rows: step 0's from the prior, then
    // mantissa and exponent through LDS
    m1 *= row_sum(a.pi[y] * As);
    const int k1 = __builtin_amdgcn_frexp_exp(m1);
    m1 = __builtin_ldexp(m1, -k1);
    e1 += k1;
    if (y == 0) { m1x[4 * seq] = m1; m1x[4 * seq + 1] = (double)e1; }
  }
  if (!FWD) {
    // one more backward step with alpha_{-1} = prior of prev: its posterior is
    // the P0 count and its xi is xi_0 (when the forward rows did not cover
    // t = 0, i.e. H > 0); normalised exactly, as chain_kernel<true>
    const double pi_y = a.pi[y];
    const double u = __builtin_ldexp(dot2_bcast(x, C), sc);
    const double pr = pi_y * u;
    const double c = row_sum(pr);
    const double q = div_by(pr, c);
    const double rc = c != 0.0 ? __builtin_ldexp(div_by(1.0, c), sc) : 0.0;
    const double w = H > 0 ? pi_y * rc : 0.0;
    Kd = __builtin_amdgcn_mfma_f64_16x16x4f64(w, x, Kd, 0, 0, 0);
    p0l[seq * 16 + y] = active ? q : 0.0;
  }
  // the wave's xi sum (over its four sequences) to LDS: the block sums its
  // waves' and writes one slab row (chain_estep16_kernel)
#pragma unroll
  for (int r = 0; r < 4; r++) kdl[(size_t)((FWD ? 0 : nseqb / 4) + grp) * 256 + r * 64 + lane] = Kd[r];
  // proper model: ll = log P(obs) = log(sum alpha^_{T-1}) - Ef_{T-1} ln 2
  // (the forward rows end phase B at t = T - 1: x = alpha^_{T-1}, ex its
  // exponent); m1_t = the previous mass, so the reference's per-step
  // log m2 - log m1 telescope to it
  const double zT = (FWD && PR) ? row_sum(x) : 0.0;
  __syncthreads();                                   // the backward rows' m1 part in LDS
  if (FWD && PR && active && y == 0) {
    const bool dead = zT == 0.0;
    const double ll = dead ? -DBL_MAX : log(zT) - (double)ex * 0.69314718055994530942;
    if (a.ll) a.ll[b] = ll;
    if (a.status) a.status[b] = dead ? 3u : 0u;
  }
  if (FWD && !PR && active && y == 0) {
    double lm = log(m2) - log(m1);
    int ee = e2 - e1;
    bool dead = m2 == 0.0;                             // some step's m2 == 0 (products renormalised: no underflow)
    if (H > 0) {                                       // phase A's m1, summed by the backward rows
      lm -= log(m1x[4 * seq]);
      ee -= (int)m1x[4 * seq + 1] + efa;
    }
    double ll = lm + (double)ee * 0.69314718055994530942;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    // e_step's BAD_LUCK (m1 <= 0 || m2 <= 0, nip.c:1827-1854): a zero mass here
    if (a.status) a.status[b] = dead ? 3u : 0u;
  }
}

}  // namespace

template <int NSEQ, int KC, int NE, int PR>
__global__ __launch_bounds__(NSEQ * 32, 1)
void chain_estep16_kernel(ChainArgs a) {
  constexpr int kE16Seqs = NSEQ, kE16Threads = NSEQ * 32, G = NSEQ / 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = a.M + 2;                                                // table rows, all children
  double* Et = reinterpret_cast<double*>(smem);                         // [R][16]
  uint8_t* codes = smem + (size_t)R * 16 * sizeof(double);              // [NE][NSEQ][Tr]
  double* Htab = reinterpret_cast<double*>(
      codes + (((size_t)NE * kE16Seqs * chain_codes_row(a.T) + 15) & ~(size_t)15));   // [NSEQ][2][R][16]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const long b0 = (long)blockIdx.x * kE16Seqs;
  const int T = a.T;
  const int Tr = chain_codes_row(T);
  const unsigned long long t_entry = NIPAMD_WAIT_TIMES ? __builtin_readcyclecounter() : 0;

  for (int i = tid; i < R * 16; i += kE16Threads) Et[i] = a.Etab[i];
  const int nseq = (int)((a.B - b0) < kE16Seqs ? (a.B - b0) : kE16Seqs);
  // child k's code: its state, eM[k] missing, eM[k] + 1 out of range (an all-zero row)
  auto code_of = [&](int k, int o) -> int { return o < 0 ? a.eM[k] : (o < a.eM[k] ? o : a.eM[k] + 1); };
#pragma unroll
  for (int k = 0; k < NE; k++)
    for (int i = tid; i < kE16Seqs * Tr; i += kE16Threads) codes[(size_t)k * kE16Seqs * Tr + i] = (uint8_t)a.eM[k];
  for (int i = tid; i < kE16Seqs * 2 * R * 16; i += kE16Threads) Htab[i] = 0.0;
  __syncthreads();
  if (NE == 1 && a.ecol[0] >= 0 && a.obs && a.obs_tstride == 1 && a.obs_bstride == T && (T & 3) == 0 &&
      nseq == kE16Seqs) {
    const int4* src = reinterpret_cast<const int4*>(a.obs + b0 * (long)T);
    const int n4 = (kE16Seqs * T) >> 2;
    for (int i0 = tid; i0 < n4; i0 += kE16Threads * 8) {
      int4 r[8];
#pragma unroll
      for (int k = 0; k < 8; k++) if (i0 + k * kE16Threads < n4) r[k] = src[i0 + k * kE16Threads];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i4 = i0 + k * kE16Threads;
        if (i4 < n4) {
          const int i = i4 << 2, c = i / T, t = i - c * T;
          const uint32_t packed = (uint32_t)code_of(0, r[k].x) | ((uint32_t)code_of(0, r[k].y) << 8) |
                                  ((uint32_t)code_of(0, r[k].z) << 16) | ((uint32_t)code_of(0, r[k].w) << 24);
          *reinterpret_cast<uint32_t*>(codes + c * Tr + kGuard + t) = packed;
        }
      }
    }
  } else if (a.obs) {
    for (int i = tid; i < nseq * T; i += kE16Threads) {
      const int c = i / T, t = i - c * T;
      const int* o = a.obs + (b0 + c) * a.obs_bstride + (long)t * a.obs_tstride;
#pragma unroll
      for (int k = 0; k < NE; k++)
        if (a.ecol[k] >= 0) codes[((size_t)k * kE16Seqs + c) * Tr + kGuard + t] = (uint8_t)code_of(k, o[a.ecol[k]]);
    }
  }
  __syncthreads();
  double* m1x = Htab + kE16Seqs * 2 * R * 16;                           // [NSEQ][4]
  double* kdl = m1x + kE16Seqs * 4;                                     // [NSEQ / 4 * 2 waves][4][64]
  double* p0l = kdl + (kE16Seqs / 4) * 2 * 256;                         // [NSEQ][16]
  // A/B builds: static wave priority for the backward (1) or the forward (2) rows
  if ((NIPAMD_ESTEP_PRIO == 1 && wave >= G) || (NIPAMD_ESTEP_PRIO == 2 && wave < G)) __builtin_amdgcn_s_setprio(1);
  if (wave < G) estep16_rows<true, KC, NE, PR>(a, Et, codes, Htab, m1x, kdl, p0l, lane, wave, b0, kE16Seqs);
  else estep16_rows<false, KC, NE, PR>(a, Et, codes, Htab, m1x, kdl, p0l, lane, wave - G, b0, kE16Seqs);
  __syncthreads();
  // the block's slab row (chain_estep_slab layout): the block's sums in a
  // fixed order -- Kf / Kb over the direction's waves (D[i][y]: lane
  // (i % 4) * 16 + y, register i / 4), every sequence's count tables and P0
  // in sequence order.  One row per NSEQ sequences instead of one per
  // sequence: 1/NSEQ of the slab bytes written and read back by the tree.
  double* slab = a.counts + (size_t)blockIdx.x * chain_estep_slab(a.M);
  for (int e = tid; e < 512; e += kE16Threads) {
    const int dir = e >> 8, i = (e >> 4) & 15, y = e & 15;
    const int off = (i >> 2) * 64 + (i & 3) * 16 + y;
    double v = 0.0;
#pragma unroll
    for (int g = 0; g < G; g++) v += kdl[(size_t)(dir * G + g) * 256 + off];
    slab[e] = v;                                                        // kSlabKf = 0, kSlabKb = 256
  }
  for (int e = tid; e < 2 * R * 16; e += kE16Threads) {
    double v = 0.0;
    for (int sq = 0; sq < kE16Seqs; sq++) v += Htab[(size_t)sq * 2 * R * 16 + e];
    slab[kSlabH + e] = v;
  }
  for (int y = tid; y < 16; y += kE16Threads) {
    double v = 0.0;
    for (int sq = 0; sq < kE16Seqs; sq++) v += p0l[sq * 16 + y];
    slab[chain_slab_p0(a.M) + y] = v;
  }
  if (NIPAMD_WAIT_TIMES && a.diag && lane == 0) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const int dd = wave < G ? 0 : 8, gg = wave < G ? wave : wave - G;
    a.diag[((size_t)blockIdx.x * 16 + dd + gg) * 4 + 3] = __builtin_readcyclecounter() - t_entry;   // whole block
  }
}

static int estep16_seqs() {
  static const int n = [] {
    const char* e = diag_env("NIPAMD_ESTEP16_SEQS");       // A/B builds: 16 or 24
    return e && std::atoi(e) == 24 ? 24 : 16;
  }();
  return n;
}

static size_t estep16_lds(int nseq, int M, int T, int ne) {
  const size_t n = (size_t)(M + 2) * 16 * sizeof(double) + (size_t)ne * nseq * chain_codes_row(T);
  return ((n + 15) & ~(size_t)15) + (size_t)nseq * 2 * (M + 2) * 16 * sizeof(double) +
         (size_t)nseq * 4 * sizeof(double) +                           // m1x
         (size_t)(nseq / 4) * 2 * 256 * sizeof(double) +               // the waves' xi sums
         (size_t)nseq * 16 * sizeof(double);                           // P0 per sequence
}

// sequences per block: 16, or 8 when the children's count tables of 16 do not fit
static int estep16_nseq(int M, int T, int ne) {
  if (ne == 1) return estep16_seqs();
  return estep16_lds(16, M, T, ne) <= 160 * 1024 ? 16 : 8;
}

size_t chain_estep16_lds_bytes(int M, int T, int ne) { return estep16_lds(estep16_nseq(M, T, ne), M, T, ne); }
int chain_estep16_seqs_per_row(int M, int T, int ne) { return estep16_nseq(M, T, ne); }

size_t chain_estep16_scratch_bytes(long B, int T) {
  const long nrow = (B + kE16RowMul - 1) / kE16RowMul * kE16RowMul;
  return (size_t)(nrow + 2) * chain_scratch_row(T) * sizeof(double) +
         (size_t)(nrow + 2) * estep16_xrow(T) * sizeof(int);
}

template <int NSEQ, int KC, int NE, int PR>
static int estep16_launch_pr(const ChainArgs& a, size_t lds, hipStream_t stream) {
  static size_t lds_set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_estep16_kernel<NSEQ, KC, NE, PR>), lds, lds_set)) return rc;
  const int blocks = (int)((a.B + NSEQ - 1) / NSEQ);
  hipLaunchKernelGGL((chain_estep16_kernel<NSEQ, KC, NE, PR>), dim3(blocks), dim3(NSEQ * 32), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <int NSEQ, int KC, int NE>
static int estep16_launch(const ChainArgs& a, size_t lds, hipStream_t stream) {
  return a.proper == 2 ? estep16_launch_pr<NSEQ, KC, NE, 2>(a, lds, stream)
       : a.proper      ? estep16_launch_pr<NSEQ, KC, NE, 1>(a, lds, stream)
                        : estep16_launch_pr<NSEQ, KC, NE, 0>(a, lds, stream);
}

int chain_estep16_launch(const ChainArgs& a, hipStream_t stream) {
  if (a.ne < 1 || a.ne > 3) return -2;                           // four children spill: general engine
  const int nseq = estep16_nseq(a.M, a.T, a.ne);
  const size_t lds = (estep16_lds(nseq, a.M, a.T, a.ne) + 15) & ~(size_t)15;
  if (lds > 160 * 1024 || a.N > 16 || !a.counts) return -2;
  g_last_kernel = "chain_estep16_kernel";
  constexpr int KC = NIPAMD_ESTEP_CHUNK;
  switch (a.ne) {
    case 1: return nseq == 24 ? estep16_launch<24, 4, 1>(a, lds, stream) : estep16_launch<16, KC, 1>(a, lds, stream);
    case 2: return nseq == 8 ? estep16_launch<8, KC, 2>(a, lds, stream) : estep16_launch<16, KC, 2>(a, lds, stream);
    default:                                                       // 4-step prefetch: no spills
      return nseq == 8 ? estep16_launch<8, 4, 3>(a, lds, stream) : estep16_launch<16, 4, 3>(a, lds, stream);
  }
}

size_t chain_lds_bytes(int M, int T, bool estep) {
  size_t n = (size_t)(M + 2) * 16 * sizeof(double) + (size_t)kChainsPerBlock * chain_codes_row(T);
  if (estep) n = ((n + 15) & ~(size_t)15) + (size_t)kChainsPerBlock * 2 * (M + 2) * 16 * sizeof(double);
  return n;
}

int chain_fb_launch(const ChainArgs& a, hipStream_t stream) {
  const int blocks = (int)((a.B + kChainsPerBlock - 1) / kChainsPerBlock);
  const size_t lds = (chain_lds_bytes(a.M, a.T, false) + 15) & ~(size_t)15;
  hipLaunchKernelGGL(chain_kernel<false>, dim3(blocks), dim3(kThreads), lds, stream, a);
  g_last_kernel = "chain_kernel<false>";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int chain_estep_launch(const ChainArgs& a, hipStream_t stream) {
  const int blocks = (int)((a.B + kChainsPerBlock - 1) / kChainsPerBlock);
  const size_t lds = (chain_lds_bytes(a.M, a.T, true) + 15) & ~(size_t)15;
  hipLaunchKernelGGL(chain_kernel<true>, dim3(blocks), dim3(kThreads), lds, stream, a);
  g_last_kernel = "chain_kernel<true>";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// Deterministic batch reduction: out[g][j] = binary-tree sum of in[64g .. 64g+63][j]
// (missing rows count as 0; x + 0 == x, so the tree shape is fixed by index).
// Applied repeatedly, this is one binary tree over all rows, so partials of
// power-of-two shards combine bit-identically across 1/2/4/8 GPUs.
__global__ __launch_bounds__(256)
void tree64_kernel(const double* __restrict__ in, long n, int S, double* __restrict__ out) {
  const int j = blockIdx.y * 256 + threadIdx.x;
  const long g = blockIdx.x;
  if (j >= S) return;
  double v[64];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const long r = g * 64 + i;
    v[i] = r < n ? in[r * S + j] : 0.0;
  }
#pragma unroll
  for (int w = 1; w < 64; w *= 2)
#pragma unroll
    for (int i = 0; i < 64; i += 2 * w) v[i] += v[i + w];
  out[g * S + j] = v[0];
}

int tree_reduce_launch(const double* in, long n, int S, double* out, hipStream_t stream) {
  const long groups = (n + 63) / 64;
  hipLaunchKernelGGL(tree64_kernel, dim3((unsigned)groups, (S + 255) / 256), dim3(256), 0, stream,
                     in, n, S, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// counts[layout] += finalised families from the reduced slab R (em_learn layout,
// nip.c:2101-2128: child first, then parents).
__global__ __launch_bounds__(256)
void estep_finalize_kernel(const double* __restrict__ R, ChainFinalize f, double* __restrict__ counts) {
  const int N = f.N, M = f.M;
  for (int i = threadIdx.x; i < N; i += 256) counts[f.off_prev + i] += R[chain_slab_p0(M) + i];
  for (int i = threadIdx.x; i < N * N; i += 256) {
    const int y = i % N, x = i / N;                    // index y + N*x
    counts[f.off_cur + i] += f.A[x * 16 + y] * (R[kSlabKf + x * 16 + y] + R[kSlabKb + x * 16 + y]);
  }
  for (int i = threadIdx.x; i < M * N; i += 256) {
    const int m = i % M, y = i / M;                    // index m + M*y
    const double* Hf = R + kSlabH;
    const double* Hb = R + kSlabH + (M + 2) * 16;
    const double miss = Hf[M * 16 + y] + Hb[M * 16 + y];
    const double s = f.Etab[M * 16 + y];
    const double part = s != 0.0 ? miss * f.Etab[m * 16 + y] / s : 0.0;
    counts[f.off_obs + i] += (Hf[m * 16 + y] + Hb[m * 16 + y]) + part;
  }
}

// One wave per count (CSR row): lane l sums terms l, l + 64, ... of the row,
// then a fixed butterfly -- a fixed order, independent of the launch.  (A
// thread per row summed the long rows -- a hidden parent's count over a
// whole xi block -- serially: 0.168 ms of config 3's e_step,
// profiles/r06ao_timed_region.txt.)
__global__ __launch_bounds__(256)
void estep_map_finalize_kernel(const double* __restrict__ R, int n, const int* __restrict__ ptr,
                               const int* __restrict__ idx, const double* __restrict__ coef,
                               double* __restrict__ counts) {
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (p >= n) return;                          // wave-uniform
  double acc = 0.0;
  for (int j = ptr[p] + lane; j < ptr[p + 1]; j += 64) acc += coef[j] * R[idx[j]];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) counts[p] += acc;
}

int estep_map_finalize_launch(const double* R, int n, const int* ptr, const int* idx, const double* coef,
                              double* counts, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(estep_map_finalize_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, R, n, ptr, idx,
                     coef, counts);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void estep_tag_kernel(double* tag, double a, double b, double c) {
  if (threadIdx.x == 0) { tag[0] = a; tag[1] = b; tag[2] = c; }
}

int estep_tag_launch(double* tag, double a, double b, double c, hipStream_t stream) {
  hipLaunchKernelGGL(estep_tag_kernel, dim3(1), dim3(64), 0, stream, tag, a, b, c);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// out[0] = the number of nonzero status words (an exact integer as a double):
// blocks of 4096 words (16 independent loads per thread) count into part[],
// then one block adds the parts; integer sums, so the order does not matter
constexpr int kCountPer = 4096;
__global__ __launch_bounds__(256) void count_failed_kernel(const uint32_t* status, long B, double* part) {
  __shared__ int red[256];
  const long base = (long)blockIdx.x * kCountPer;
  int n = 0;
#pragma unroll
  for (int k = 0; k < kCountPer / 256; k++) {
    const long i = base + k * 256 + threadIdx.x;
    n += (i < B && status[i] != 0u) ? 1 : 0;
  }
  red[threadIdx.x] = n;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = (double)red[0];
}

__global__ __launch_bounds__(256) void count_sum_kernel(const double* part, long n, double* out) {
  __shared__ double red[256];
  double s = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

long count_failed_work(long B) { return (B + kCountPer - 1) / kCountPer; }

int count_failed_launch(const uint32_t* status, long B, double* work, double* out, hipStream_t stream) {
  const long nb = count_failed_work(B);
  hipLaunchKernelGGL(count_failed_kernel, dim3((unsigned)nb), dim3(256), 0, stream, status, B, work);
  hipLaunchKernelGGL(count_sum_kernel, dim3(1), dim3(256), 0, stream, work, nb, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The e_step's verdict on a leading missing run (prefix.cpp): a sequence
// whose observations at steps 0..first_bad are all missing (< 0) gets
// BAD_LUCK.  One thread per sequence; almost every sequence leaves at its
// first step, so the launch reads a few bytes per sequence.
// A series whose steps 0..first_bad carry no evidence: every column missing,
// or (bit c of `trivial`) an observation of a one-state variable, whose
// indicator multiplies every table by 1.0 -- the reference's propagation
// over such a step is bit for bit the missing step's (nip_update_evidence,
// nippotential.c:499-522, divides by the likelihood 1 as well)
__global__ void estep_prefix_flag_kernel(const int32_t* obs, long bstride, int n_obs, int B, int first_bad,
                                         unsigned trivial, uint32_t* status) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int32_t* o = obs + (long)b * bstride;
  for (int t = 0; t <= first_bad; t++)
    for (int c = 0; c < n_obs; c++) {
      const int32_t v = o[(long)t * n_obs + c];
      if (v >= 0 && !(v == 0 && c < 32 && ((trivial >> c) & 1u))) return;   // the mask covers columns 0..31
    }
  status[b] |= 2u;                                   // NIPAMD_STATUS_BAD_LUCK
}

int estep_prefix_flag_launch(const int32_t* obs, int n_obs, int B, int T, int first_bad, unsigned trivial,
                             uint32_t* status, hipStream_t stream) {
  if (B <= 0) return 0;
  if (first_bad < 0 || first_bad >= T || (n_obs > 0 && !obs)) return -1;
  hipLaunchKernelGGL(estep_prefix_flag_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, obs,
                     (long)T * n_obs, n_obs, B, first_bad, trivial, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int estep_finalize_launch(const double* R, const ChainFinalize& f, double* counts, hipStream_t stream) {
  hipLaunchKernelGGL(estep_finalize_kernel, dim3(1), dim3(256), 0, stream, R, f, counts);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
