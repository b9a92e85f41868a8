// chain_mfma.hip -- batched forward-backward on the gfx950 matrix cores.
//
// Same recursion as chain_kernels.hip (see the derivation there, nip.c:1320-
// 1581), laid out for v_mfma_f64_16x16x4_f64: one wavefront carries SIXTEEN
// chains (sequences) of one direction, and every step's sixteen 16x16
// mat-vecs are one 16x16x16 product, D = M' X, done as four chained MFMAs.
//
// Register layout (MI355X_MICROARCH.md, f64 MFMA): D/C lane l, register r =
// element (row (l>>4) + 4r, column l&15); A operand lane l = (row l&15,
// k l>>4); B operand lane l = (k l>>4, column l&15).  Columns are chains
// (j = l&15).  Splitting K = 16 into four MFMAs with k' = (l>>4) + 4r makes
// register r of D exactly the B operand of MFMA r of the next step, so the
// state never leaves the lane.  Internal state i' is stored as actual state
// sigma(i') = 4 (i' mod 4) + (i' div 4): lane (g = l>>4, j) register r then
// holds actual state 4g + r of chain j, so every lane owns four CONTIGUOUS
// states -- 32-byte evidence reads from LDS and 32-byte stores to HBM.
//
//   A operand of MFMA r, lane l:  M[sigma(l&15)][4(l>>4) + r]
//   with M = A^T (forward: u = A^T alpha)  or  M = A (backward: u = A g)
//
// Sums over a chain's 16 states: three in-lane adds, then v_permlane32_swap
// and v_permlane16_swap exchanges (lanes l, l^32, l^16), each symmetric, so
// all four lanes of a chain hold bit-identical sums.
//
// Block = 2 waves on the same 16 sequences: wave 0 the forward filter, wave 1
// the backward filter.  Phase A / barrier / phase B exactly as the 16-lane
// kernel (two-filter smoothing, S[b][t] holds alpha_t for t < H, beta_t for
// t >= H).  Each wave runs its own template instance: no per-lane direction
// selects.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

#include "chain_kernels.h"

namespace nipamd {

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int kMSeq = 16;          // sequences (chains per direction) per block
constexpr int kMThreads = 128;     // wave 0 forward, wave 1 backward
constexpr int kMChunk = 8;         // steps per unrolled chunk = prefetch distance
constexpr int kMG = kScratchGuard;

__device__ __forceinline__ double sum_lanes32(double x) {   // x[l] + x[l ^ 32]
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

__device__ __forceinline__ double sum_lanes16(double x) {   // x[l] + x[l ^ 16]
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

// sum of the chain's 16 states, identical in the chain's four lanes
__device__ __forceinline__ double chain_sum(v4d v) {
  return sum_lanes16(sum_lanes32((v.x + v.y) + (v.z + v.w)));
}

__device__ __forceinline__ v4d matvec(const double (&Aop)[4], v4d X) {
  v4d d = {0.0, 0.0, 0.0, 0.0};
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0], X.x, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[1], X.y, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[2], X.z, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[3], X.w, d, 0, 0, 0);
  return d;
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

__device__ __forceinline__ v4d load4(const double* p) {
  const double2 a = *reinterpret_cast<const double2*>(p);
  const double2 b = *reinterpret_cast<const double2*>(p + 2);
  v4d r;
  r.x = a.x; r.y = a.y; r.z = b.x; r.w = b.y;
  return r;
}

__device__ __forceinline__ void store4(double* p, v4d v) {
  *reinterpret_cast<double2*>(p) = make_double2(v.x, v.y);
  *reinterpret_cast<double2*>(p + 2) = make_double2(v.z, v.w);
}

struct WaveCtx {
  const double* Et;         // LDS evidence table + 4g (row stride 16)
  const uint8_t* codes;     // LDS codes of chain j, index t in [-kMG, T + kMG)
  double* S;                // this chain's scratch row + 4g (index t * 16), or the sink row
  double* P;                // posterior of this chain + post_off + 4g, or the sink row
  long Pstride;             // post_tstride, or 0 for the sink
  int nst;                  // states of this lane that are real (N - 4g, clamped)
};

__device__ __forceinline__ v4d evidence(const WaveCtx& c, int t) {
  return load4(c.Et + c.codes[t] * 16);
}

// PVEC: N == 16 and 16-byte aligned posterior rows -> two 16-byte stores
template <bool PVEC>
__device__ __forceinline__ void store_post(double* p, int nst, v4d q) {
  if (PVEC) {
    store4(p, q);
  } else {
    if (nst > 0) p[0] = q.x;
    if (nst > 1) p[1] = q.y;
    if (nst > 2) p[2] = q.z;
    if (nst > 3) p[3] = q.w;
  }
}

template <bool FWD, bool PVEC>
struct Chain {
  double Aop[4];
  v4d X;          // next mat-vec input (fwd: alpha_{t-1}; bwd: e_{t+1} o beta_{t+1})
  v4d s;          // row sums of the evidence table (m1 weights)
  int sc = 0;     // power-of-two scale applied to the next mat-vec result
  double m2 = 1.0, m1 = 1.0;
  int e2 = 0, e1 = 0;
  double zmin = 1.0;   // min over steps of z2: 0 <=> some zero mass

  // one step; Sp / Pp point at time t's vectors, `other` is the opposite
  // direction's vector at t
  template <bool COMBINE>
  __device__ __forceinline__ void step(double* Sp, double* Pp, int nst, v4d e, v4d other, int j) {
    const v4d u = ldexp4(matvec(Aop, X), sc);
    const v4d p = u * e;
    const v4d keep = FWD ? p : u;
    const double z2 = chain_sum(p);
    const double z1 = chain_sum(u * s);
    if (!COMBINE) {
      store4(Sp, keep);
    } else {
      const v4d pr = keep * other;
      // normalise; an all-zero vector stays zero (recip(0) = 0)
      store_post<PVEC>(Pp, nst, pr * recip(chain_sum(pr)));
    }
    zmin = __builtin_fmin(zmin, z2);
    m2 *= z2; m1 *= z1;
    if ((j & 3) == 3) {
      const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
      const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
    }
    sc = -__builtin_amdgcn_frexp_exp(z2);   // frexp exponent of 0 is 0
    X = p;
  }

  // n steps starting at t0, moving forward (FWD) or backward in time
  template <bool COMBINE>
  __device__ __forceinline__ void run(const WaveCtx& c, int n, int t0) {
    constexpr int dir = FWD ? 1 : -1;
    v4d oa[kMChunk], ob[kMChunk];
    auto load_other = [&](v4d (&o)[kMChunk], int tb) {
      const double* q = c.S + (long)tb * 16;
#pragma unroll
      for (int k = 0; k < kMChunk; k++) o[k] = COMBINE ? load4(q + dir * k * 16) : v4d{};
    };
    const long pinc = dir * c.Pstride;
    int base = 0;
    if (COMBINE && n >= 2 * kMChunk) load_other(oa, t0);
    double* Pp = c.P + (long)t0 * c.Pstride;
    v4d en = evidence(c, t0);
    for (; base + 2 * kMChunk <= n; base += 2 * kMChunk) {
      if (COMBINE) load_other(ob, t0 + dir * (base + kMChunk));
      double* Sc = c.S + (long)(t0 + dir * base) * 16;
#pragma unroll
      for (int k = 0; k < kMChunk; k++) {
        const v4d e = en;
        en = evidence(c, t0 + dir * (base + k + 1));
        step<COMBINE>(Sc + dir * k * 16, Pp, c.nst, e, oa[k], k);
        Pp += pinc;
      }
      if (COMBINE) load_other(oa, t0 + dir * (base + 2 * kMChunk));
#pragma unroll
      for (int k = 0; k < kMChunk; k++) {
        const v4d e = en;
        en = evidence(c, t0 + dir * (base + kMChunk + k + 1));
        step<COMBINE>(Sc + dir * (kMChunk + k) * 16, Pp, c.nst, e, ob[k], k);
        Pp += pinc;
      }
    }
    // tail (< 2 chunks): one step at a time, renormalising every step
    for (; base < n; base++) {
      const int t = t0 + dir * base;
      step<COMBINE>(c.S + (long)t * 16, Pp, c.nst, evidence(c, t),
                    COMBINE ? load4(c.S + (long)t * 16) : v4d{}, 3);
      Pp += pinc;
    }
  }
};

template <bool FWD, bool PVEC>
__device__ __forceinline__ void run_wave(const ChainArgs& a, const WaveCtx& c, const double* Et,
                                         int lane, bool active, long b) {
  const int j = lane & 15, g = lane >> 4;
  const int sj = 4 * (j & 3) + (j >> 2);        // actual state of D row j
  const int T = a.T, H = a.H;
  Chain<FWD, PVEC> ch;
#pragma unroll
  for (int r = 0; r < 4; r++)
    ch.Aop[r] = FWD ? a.A[(4 * g + r) * 16 + sj] : a.A[sj * 16 + 4 * g + r];
  ch.s = load4(Et + a.M * 16 + 4 * g);
  if (FWD) {
    ch.X = load4(a.pi + 4 * g);
  } else {
    v4d beta;                                   // beta_{T-1} = 1 on the real states
    beta.x = 4 * g + 0 < a.N ? 1.0 : 0.0; beta.y = 4 * g + 1 < a.N ? 1.0 : 0.0;
    beta.z = 4 * g + 2 < a.N ? 1.0 : 0.0; beta.w = 4 * g + 3 < a.N ? 1.0 : 0.0;
    store4(c.S + (long)(T - 1) * 16, beta);     // T-1 >= H
    ch.X = evidence(c, T - 1) * beta;
    ch.sc = -__builtin_amdgcn_frexp_exp(chain_sum(ch.X));
  }
  // phase A: forward alpha_0..alpha_{H-1}; backward beta_{T-2}..beta_H
  if (FWD) ch.template run<false>(c, H, 0);
  else ch.template run<false>(c, T - 1 - H, T - 2);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // phase B: forward alpha_H..alpha_{T-1} with beta from S; backward
  // beta_{H-1}..beta_0 with alpha from S
  if (FWD) ch.template run<true>(c, T - H, H);
  else ch.template run<true>(c, H, H - 1);
  if (FWD && active && g == 0) {
    double ll = log(ch.m2) - log(ch.m1) + (double)(ch.e2 - ch.e1) * 0.69314718055994530942;
    const bool dead = ch.zmin == 0.0;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    if (a.status) a.status[b] = dead ? 1u : 0u;
  }
}

__global__ __launch_bounds__(kMThreads, 1)
void chain_fb_mfma_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* Et = reinterpret_cast<double*>(smem);                       // [(M+2)][16]
  uint8_t* codes = smem + (size_t)(a.M + 2) * 16 * sizeof(double);    // [16][Tr]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const long b0 = (long)blockIdx.x * kMSeq;
  const long b = b0 + j;
  const bool active = b < a.B;
  const int T = a.T;
  const int Tr = chain_codes_row(T);

  // --- stage the evidence table and the 16 sequences' observation codes
  for (int i = tid; i < (a.M + 2) * 16; i += kMThreads) Et[i] = a.Etab[i];
  const int nseq = (int)((a.B - b0) < kMSeq ? (a.B - b0) : kMSeq);
  auto code_of = [&](int o) -> int { return o < 0 ? a.M : (o < a.M ? o : a.M + 1); };
  for (int i = tid; i < kMSeq * Tr / 4; i += kMThreads)
    reinterpret_cast<uint32_t*>(codes)[i] = 0x01010101u * (uint32_t)a.M;   // missing / guard
  __syncthreads();
  if (a.obs && a.obs_tstride == 1 && a.obs_bstride == T && (T & 3) == 0 && nseq == kMSeq) {
    const int4* src = reinterpret_cast<const int4*>(a.obs + b0 * (long)T);
    const int n4 = (kMSeq * T) >> 2;
    for (int i0 = tid; i0 < n4; i0 += kMThreads * 8) {
      int4 r[8];
#pragma unroll
      for (int k = 0; k < 8; k++) if (i0 + k * kMThreads < n4) r[k] = src[i0 + k * kMThreads];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i4 = i0 + k * kMThreads;
        if (i4 < n4) {
          const int i = i4 << 2, cq = i / T, t = i - cq * T;
          const uint32_t packed = (uint32_t)code_of(r[k].x) | ((uint32_t)code_of(r[k].y) << 8) |
                                  ((uint32_t)code_of(r[k].z) << 16) | ((uint32_t)code_of(r[k].w) << 24);
          *reinterpret_cast<uint32_t*>(codes + cq * Tr + kMG + t) = packed;
        }
      }
    }
  } else if (a.obs) {
    for (int i = tid; i < nseq * T; i += kMThreads) {
      const int cq = i / T, t = i - cq * T;
      codes[cq * Tr + kMG + t] =
          (uint8_t)code_of(a.obs[(b0 + cq) * a.obs_bstride + (long)t * a.obs_tstride + a.obs_col]);
    }
  }
  __syncthreads();

  const long row = chain_scratch_row(T);
  double* const sink = a.S + (size_t)(a.B + 1) * row + kMG * 16 + 4 * g;
  WaveCtx c;
  c.Et = Et + 4 * g;
  c.codes = codes + j * Tr + kMG;
  c.S = active ? a.S + (size_t)b * row + kMG * 16 + 4 * g : sink;
  const bool pst = active && a.post;
  c.P = pst ? a.post + (size_t)b * a.post_bstride + a.post_off + 4 * g : sink;
  c.Pstride = pst ? a.post_tstride : 0;
  const bool pvec = a.N == 16 && ((a.post_off | a.post_tstride | (int)(a.post_bstride & 1)) & 1) == 0 &&
                    ((reinterpret_cast<uintptr_t>(a.post) & 15) == 0);
  c.nst = pst ? (a.N - 4 * g < 0 ? 0 : (a.N - 4 * g > 4 ? 4 : a.N - 4 * g)) : 4;
  if (pvec) {
    if (wave == 0) run_wave<true, true>(a, c, Et, lane, active, b);
    else run_wave<false, true>(a, c, Et, lane, active, b);
  } else {
    if (wave == 0) run_wave<true, false>(a, c, Et, lane, active, b);
    else run_wave<false, false>(a, c, Et, lane, active, b);
  }
}

}  // namespace

size_t chain_mfma_lds_bytes(int M, int T) {
  return (size_t)(M + 2) * 16 * sizeof(double) + (size_t)kMSeq * chain_codes_row(T);
}

int chain_fb_mfma_launch(const ChainArgs& a, hipStream_t stream) {
  const int blocks = (int)((a.B + kMSeq - 1) / kMSeq);
  const size_t lds = (chain_mfma_lds_bytes(a.M, a.T) + 15) & ~(size_t)15;
  hipLaunchKernelGGL(chain_fb_mfma_kernel, dim3(blocks), dim3(kMThreads), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
