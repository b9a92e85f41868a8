// chain_wide4.hip -- forward-backward for interface chains of 33..64 states
// (SURVEY 8(d) config 5 after the 64^4 in-clique is folded, fold.hip), up to
// four observed children.  Same recursion as chain_wide.hip:
//   alpha_t = e_t o A^T alpha_{t-1},  beta_t = A (e_{t+1} o beta_{t+1}),
//   post_t = normalise(alpha_t o beta_t),  ll = sum_t log z2_t - log z1_t
// (nip.c:1320-1581; two-filter smoothing, phase A / barrier / phase B).
//
// The 64-state mat-vec is latency-bound for one wave (a 64-deep FMA chain
// per step), and B = 256 sequences give only 512 waves, so each direction of
// a sequence gets four filter waves, wave w contracting the 16 inputs
// k in [16w, 16w + 16) against its lane's column of A for all 64 outputs:
//   part_w[y] = sum_k A[k][y] x[k]    (forward; backward: A[y][k])
// The partials meet in LDS after one block barrier per step and every filter
// wave sums them in the same order, so all four hold identical bits of u, p
// and the next input (each keeps its own LDS copy of x for its broadcasts).
// Rescaling (exact powers of two) happens every 4th step only.  Two partner
// waves take the interface vectors from an LDS ring one step behind: scratch
// stores (phase A), the other direction's vector from HBM and the normalised
// posterior (phase B), and the forward ll -- all off the recursion's path.
// Block: 8 filter waves + 2 partners = 640 threads, one sequence.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

#include "chain_kernels.h"
#include "store_pol.h"

namespace nipamd {

namespace {

constexpr int kQ = 4;                    // filter waves per direction
constexpr int kW4Threads = (2 * kQ + 2) * 64;
constexpr int kW4Ring = 16;              // LDS ring depth (steps): two partner batches
constexpr int kW4G = kScratchGuard;
constexpr int kW4Rescale = 4;            // rescale interval (steps)

template <int K>
__device__ __forceinline__ double ror(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x120 + K, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// x[l] + x[l ^ 16] (pl16) / x[l] + x[l ^ 32] (pl32) in every lane: the swap's
// second operand is a copy of x made as a whole double (one v_mov_b64; the
// two results come back in the register pairs of the two operands)
__device__ __forceinline__ double pl16(double x) {
  double xc = x;
  asm("" : "+v"(xc));
  const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
__device__ __forceinline__ double pl32(double x) {
  double xc = x;
  asm("" : "+v"(xc));
  const auto rl = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

// fixed-order sum over the wave (identical bits in every lane)
__device__ __forceinline__ double wave_sum(double x) {
  asm("" : "+v"(x));       // one rounded value per lane: no fma contraction into the first add
  x += ror<8>(x);
  x += ror<4>(x);
  x += ror<2>(x);
  x += ror<1>(x);
  x = pl16(x);
  x = pl32(x);
  return x;
}

// wave_sum of n independent values, stage by stage so their dependency
// chains interleave
template <int n>
__device__ __forceinline__ void wave_sum_n(double (&x)[n]) {
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += ror<8>(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += ror<4>(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += ror<2>(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += ror<1>(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] = pl16(x[i]);
#pragma unroll
  for (int i = 0; i < n; i++) x[i] = pl32(x[i]);
}

__device__ __forceinline__ double recip(double c) {
  double r = __builtin_amdgcn_rcp(c);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  return c != 0.0 ? r : 0.0;
}

__device__ __forceinline__ void block_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS pointers typed as such, so every access is a ds_ instruction (a flat
// access would also count in vmcnt and serialise on the HBM prefetches)
typedef __attribute__((address_space(3))) double lds_d;
typedef double v2d __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2d lds_v2d;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

struct W4Lds {
  lds_d* xb;         // [2 dirs][kQ][64]      each filter wave's copy of its next input
  lds_d* pb;         // [2 dirs][2][kQ][64]   partials, double-buffered by step parity
  lds_d* ring;       // [2 dirs][kW4Ring][64] interface vector of each step (fwd: alpha, bwd: beta)
  lds_d* uring;      // [kW4Ring][64]         forward: u_t (the ll's m1 = sum u s)
  lds_d* tab;        // evidence tables [(M_k + 2)][64] at toff_k, ebase [64] at eoff
  int toff0, toff1, toff2, toff3;
  int eoff;
  lds_u8* codes;     // [ncol][Tr]
  int Tr;
  // chain_row64_kernel: each column's codes once more per direction and
  // phase in the filter's processing order, [ncol][2 dirs][PA | PB] bytes
  // (phase A at 0, phase B at PA; 8-aligned, so a chunk's 8 codes are one
  // ds_read_b64)
  lds_u8* pcodes;
  int PA, PAB;
};

// block-uniform iteration counts of the two phases (multiples of the
// partners' 8-step batches) and the filters' per-direction step counts
struct R64Iters {
  int nAf, nAb, nBf, nBb, nAi, nBi;
  __host__ __device__ R64Iters(int T, int H, bool filt) {
    nAf = filt ? 0 : H; nAb = filt ? 0 : T - 1 - H;
    nBf = filt ? T : T - H; nBb = filt ? 0 : H;
    nAi = ((nAf > nAb ? nAf : nAb) + 7) & ~7;
    nBi = ((nBf > nBb ? nBf : nBb) + 7) & ~7;
  }
  // per-phase code rows: the iterations plus two chunks of look-ahead
  __host__ __device__ int PA() const { return nAi + 16; }
  __host__ __device__ int PB() const { return nBi + 16; }
};

// e_t[y] = ebase[y] prod_k tab_k[code_k(t)][y]  (row M_k: the child's row sum,
// for a missing value and the guards; row M_k + 1: 0, out of range)
__device__ __forceinline__ double evidence(const WideArgs& a, const W4Lds& L, int t, int y) {
  double e = L.tab[L.eoff + y];
  const int toff[4] = {L.toff0, L.toff1, L.toff2, L.toff3};
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (k < a.ncol) e *= L.tab[toff[k] + L.codes[k * L.Tr + kW4G + t] * 64 + y];
  return e;
}

// Phase loops: n_iter + 1 block barriers per phase for every wave; a filter
// computes step i before barrier i + 1 (its partial before, the rest after
// barrier i), a partner processes step i - 1 after barrier i.
template <bool FWD>
__device__ __forceinline__ void w4_filter(const WideArgs& a, const W4Lds& L, int w, int y, int nA, int nAi, int nB, int nBi) {
  const int T = a.T, H = a.H;
  const int d = FWD ? 0 : 1;
  double Acol[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int kk = 16 * w + k;
    Acol[k] = FWD ? a.A[kk * 64 + y] : a.A[y * 64 + kk];
  }
  lds_d* xb = L.xb + (d * kQ + w) * 64;   // this wave's copy of the next mat-vec input
  int sc = 0;
  if (FWD) {
    xb[y] = a.pi[y];
  } else if (nA + nB > 0) {
    const double X = evidence(a, L, T - 1, y) * (y < a.N ? 1.0 : 0.0);   // e_{T-1} o beta_{T-1}
    sc = -__builtin_amdgcn_frexp_exp(wave_sum(X));
    xb[y] = X;
  }
  // diagnostics (a.diag): cycles before the barrier, waiting in it, after it
  const bool dg = a.diag != nullptr;
  unsigned long long tpre = 0, twait = 0, tpost = 0, tm = dg ? __builtin_readcyclecounter() : 0;
  auto stamp = [&](unsigned long long& acc) {
    if (dg) { const unsigned long long n = __builtin_readcyclecounter(); acc += n - tm; tm = n; }
  };
  const unsigned long long c0 = tm;
  auto phase = [&](int n, int ni, int t0) {
    double en = n > 0 ? evidence(a, L, t0, y) : 1.0;
    for (int i = 0; i <= ni; i++) {
      const bool act = i < n;
      const int t = FWD ? t0 + i : t0 - i;
      const double e = en;
      lds_d* pb = L.pb + (d * 2 + (i & 1)) * kQ * 64;
      if (act) {
        const lds_v2d* xs = reinterpret_cast<const lds_v2d*>(xb + 16 * w);   // broadcast reads
        double x[16];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const v2d v = xs[k];
          x[2 * k] = v.x; x[2 * k + 1] = v.y;
        }
        double p0 = Acol[0] * x[0], p1 = Acol[1] * x[1], p2 = Acol[2] * x[2], p3 = Acol[3] * x[3];
#pragma unroll
        for (int k = 4; k < 16; k += 4) {
          p0 = __builtin_fma(Acol[k], x[k], p0); p1 = __builtin_fma(Acol[k + 1], x[k + 1], p1);
          p2 = __builtin_fma(Acol[k + 2], x[k + 2], p2); p3 = __builtin_fma(Acol[k + 3], x[k + 3], p3);
        }
        pb[w * 64 + y] = (p0 + p1) + (p2 + p3);
        if (i + 1 < n) en = evidence(a, L, FWD ? t + 1 : t - 1, y);     // the next step's
      }
      if (dg) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stamp(tpre);
      block_barrier();
      stamp(twait);
      if (act) {
        const double u = __builtin_ldexp((pb[y] + pb[64 + y]) + (pb[128 + y] + pb[192 + y]), sc);
        const double p = u * e;
        if (w == 0) {
          const int slot = i & (kW4Ring - 1);
          L.ring[(d * kW4Ring + slot) * 64 + y] = FWD ? p : u;
          if (FWD) L.uring[slot * 64 + y] = u;
        }
        const bool rs = (i & (kW4Rescale - 1)) == kW4Rescale - 1 || i == n - 1;
        sc = 0;
        if (rs) sc = -__builtin_amdgcn_frexp_exp(wave_sum(p));   // frexp exponent of 0 is 0
        xb[y] = p;
      }
      if (dg) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stamp(tpost);
    }
  };
  // phase A: forward alpha_0..alpha_{H-1}; backward beta_{T-2}..beta_H
  phase(nA, nAi, 0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  // phase B: forward alpha_H..alpha_{T-1}; backward beta_{H-1}..beta_0
  phase(nB, nBi, 1);
  if (dg && y == 0 && w == 0) {
    a.diag[blockIdx.x * 16 + (FWD ? 0 : 4) + 0] = __builtin_readcyclecounter() - c0;
    a.diag[blockIdx.x * 16 + (FWD ? 0 : 4) + 1] = twait;
    a.diag[blockIdx.x * 16 + (FWD ? 0 : 4) + 2] = tpre;
    a.diag[blockIdx.x * 16 + (FWD ? 0 : 4) + 3] = tpost;
  }
}

// The partner processes step i - 1 after barrier i (the ring holds the
// filter's vectors of the last 16 steps).
template <bool FWD>
__device__ __forceinline__ void w4_partner(const WideArgs& a, const W4Lds& L, int y, long b, int nA, int nAi, int nB, int nBi) {
  const int T = a.T, H = a.H;
  const int d = FWD ? 0 : 1;
  double* const Srow = a.S + (size_t)b * chain_scratch_row64(T) + (size_t)kW4G * 64 + y;
  double* const Prow = (a.post && y < a.N) ? a.post + (size_t)b * a.post_bstride + a.post_off + y : nullptr;
  const double s = a.s[y];
  double m2 = 1.0, m1 = 1.0, zmin = 1.0;
  int e2 = 0, e1 = 0;
  // forward ll (nip.c:1461-1474): z2 = sum alpha_t, z1 = sum u_t s, both on
  // the same (power-of-two) scale; mantissas and exponents kept apart
  auto ll_step = [&](int slot) {
    double z[2] = {L.ring[slot * 64 + y], L.uring[slot * 64 + y] * s};
    wave_sum_n<2>(z);
    zmin = __builtin_fmin(zmin, z[0]);
    m2 *= __builtin_amdgcn_frexp_mant(z[0]); e2 += __builtin_amdgcn_frexp_exp(z[0]);
    m1 *= __builtin_amdgcn_frexp_mant(z[1]); e1 += __builtin_amdgcn_frexp_exp(z[1]);
    const int k2 = __builtin_amdgcn_frexp_exp(m2), k1 = __builtin_amdgcn_frexp_exp(m1);
    m2 = __builtin_ldexp(m2, -k2); e2 += k2;
    m1 = __builtin_ldexp(m1, -k1); e1 += k1;
  };
  const unsigned long long c0 = a.diag ? __builtin_readcyclecounter() : 0;
  if (!FWD && !a.filter) Srow[(long)(T - 1) * 64] = y < a.N ? 1.0 : 0.0;   // beta_{T-1}, T-1 >= H
  // phase A: the interface vectors to the scratch
  for (int i = 0; i <= nAi; i++) {
    block_barrier();
    const int j = i - 1;
    if (j >= 0 && j < nA) {
      const int slot = j & (kW4Ring - 1);
      Srow[(long)(FWD ? j : T - 2 - j) * 64] = L.ring[(d * kW4Ring + slot) * 64 + y];
      if (FWD) ll_step(slot);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // phase B: posterior = normalise(this o other); the other direction's
  // vectors come from the scratch one 8-step chunk ahead, ping-ponged between
  // two register sets (no register copy of a pending load)
  const int tB = FWD ? H : H - 1;
  auto tof = [&](int j) { return FWD ? tB + j : tB - j; };
  // forward_inference reads a valid dummy row instead of the scratch
  const double* const Sld = a.filter ? a.S + y : Srow;
  const long sstr = a.filter ? 0 : 64;
  auto load8 = [&](double (&r)[8], int c) {
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = load_pol<NIPAMD_SCR_NTLD>(Sld + (long)tof(8 * c + k) * sstr);   // guards cover the over-run
  };
  auto chunk = [&](const double (&r)[8], int c) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      block_barrier();                               // iteration 8c + k + 1: step 8c + k is in the ring
      const int j = 8 * c + k;
      if (j < nB) {
        const int slot = j & (kW4Ring - 1);
        const double pr = L.ring[(d * kW4Ring + slot) * 64 + y] * (a.filter ? 1.0 : r[k]);
        const double q = pr * recip(wave_sum(pr));   // an all-zero row stays zero
        if (Prow) store_pol<NIPAMD_POST_NT>(Prow + (long)tof(j) * a.post_tstride, q);
        if (FWD) ll_step(slot);
      }
    }
  };
  const int nch = nBi / 8;                           // nBi: a multiple of 8 (kernel)
  double ra[8], rb[8];
  load8(ra, 0);
  block_barrier();                                   // iteration 0
  for (int c = 0; c < nch; c += 2) {
    load8(rb, c + 1);
    chunk(ra, c);
    if (c + 1 >= nch) break;
    load8(ra, c + 2);
    chunk(rb, c + 1);
  }
  if (a.diag && y == 0) a.diag[blockIdx.x * 16 + (FWD ? 8 : 12)] = __builtin_readcyclecounter() - c0;
  if (FWD && y == 0) {
    double ll = log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
    const bool dead = zmin == 0.0;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    if (a.status) a.status[b] = dead ? 1u : 0u;
  }
}

// ---- chain_row64_kernel: one filter wave per direction (round 3) ----
//
// chain_wide4_kernel splits a direction's 64-deep contraction over four
// waves whose partials meet in LDS behind a block barrier every step: ≈ 1.4K
// cycles per step, all of it LDS round trips and barrier waits on one
// sequence's dependency chain (profiles/r02/r02h_config5_wide4_stamps.txt).
// Here one wave does the whole contraction in registers: lane y holds x(y)
// and column y of A; two lane-swap levels (v_permlane16_swap, then
// v_permlane32_swap of both results) leave in every lane the four 16-state
// blocks of x in canonical order (block 0, 2 from the first value's swap, 1,
// 3 from the second's), and 64 v_fmac_f64_dpp row_newbcast take x(16b + j)
// from lane j of the row of block b's copy.  No LDS on the recursion's path
// and one block barrier per 8 steps, when a partner takes the ring's chunk.
// Block: 4 waves, one per SIMD: forward filter, backward filter, forward
// partner, backward partner (the partners as in chain_wide4_kernel).
constexpr int kR64Threads = 256;

template <int K, bool NOP_FIRST>
__device__ __forceinline__ void fmac_b(double& acc, double v, double c) {
  if (NOP_FIRST)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(K));
  else
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(K));
}

// acc[j & 3] += x_block(lane j of the row) * Ac[j], j = 0..15 (sixteen
// accumulators measured slower: 139K vs 128K cycles per block, the extra
// zeroing and adds cost more issue slots than the shorter chains save; a
// single wave per SIMD issues f64 VALU work every ~6.3 cycles)
__device__ __forceinline__ void fmac16(double (&acc)[4], double xb, const double (&Ac)[16]) {
  fmac_b<0, true>(acc[0], xb, Ac[0]);    fmac_b<1, false>(acc[1], xb, Ac[1]);
  fmac_b<2, false>(acc[2], xb, Ac[2]);   fmac_b<3, false>(acc[3], xb, Ac[3]);
  fmac_b<4, false>(acc[0], xb, Ac[4]);   fmac_b<5, false>(acc[1], xb, Ac[5]);
  fmac_b<6, false>(acc[2], xb, Ac[6]);   fmac_b<7, false>(acc[3], xb, Ac[7]);
  fmac_b<8, false>(acc[0], xb, Ac[8]);   fmac_b<9, false>(acc[1], xb, Ac[9]);
  fmac_b<10, false>(acc[2], xb, Ac[10]); fmac_b<11, false>(acc[3], xb, Ac[11]);
  fmac_b<12, false>(acc[0], xb, Ac[12]); fmac_b<13, false>(acc[1], xb, Ac[13]);
  fmac_b<14, false>(acc[2], xb, Ac[14]); fmac_b<15, false>(acc[3], xb, Ac[15]);
}

// the four 16-state blocks of x (lane l holds x(l)) in every lane: xb[b] at
// lane (row r, i) = x(16 b + i)
__device__ __forceinline__ void blocks_of(double x, double (&xb)[4]) {
  // the copies the in-place swaps need, made as whole doubles (one
  // v_mov_b64 each instead of two v_mov_b32: each swap's two results sit in
  // the register pairs of its two operands)
  double xc = x;
  asm("" : "+v"(xc));
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const unsigned clo = (unsigned)__double2loint(xc), chi = (unsigned)__double2hiint(xc);
  const auto pl = __builtin_amdgcn_permlane16_swap(lo, clo, false, false);   // [0]: block r & ~1, [1]: r | 1
  const auto ph = __builtin_amdgcn_permlane16_swap(hi, chi, false, false);
  double p0 = __hiloint2double((int)ph[0], (int)pl[0]), p1 = __hiloint2double((int)ph[1], (int)pl[1]);
  double p0c = p0, p1c = p1;
  asm("" : "+v"(p0c));
  asm("" : "+v"(p1c));
  const auto q0l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(p0), (unsigned)__double2loint(p0c), false, false);
  const auto q0h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(p0), (unsigned)__double2hiint(p0c), false, false);
  const auto q1l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(p1), (unsigned)__double2loint(p1c), false, false);
  const auto q1h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(p1), (unsigned)__double2hiint(p1c), false, false);
  xb[0] = __hiloint2double((int)q0h[0], (int)q0l[0]);
  xb[2] = __hiloint2double((int)q0h[1], (int)q0l[1]);
  xb[1] = __hiloint2double((int)q1h[0], (int)q1l[0]);
  xb[3] = __hiloint2double((int)q1h[1], (int)q1l[1]);
}

// The rescale exponent from the largest element instead of the sum: any
// power of two serves (the ring's vectors and the partners' sums carry it
// exactly, posteriors and ll are scale-free), and an integer max over the
// wave is 32-bit DPP work (about 16 instructions) where the f64 wave sum was
// 43.  Zeros do not count; an all-zero vector keeps the scale (-> 0).
__device__ __forceinline__ int max_exp_rescale(double p) {
  int e = p != 0.0 ? __builtin_amdgcn_frexp_exp(p) : -0x40000;
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x128, 0xF, 0xF, true));   // row_ror:8
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x124, 0xF, 0xF, true));   // row_ror:4
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x122, 0xF, 0xF, true));   // row_ror:2
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x121, 0xF, 0xF, true));   // row_ror:1
  {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)e, (unsigned)e, false, false);
    e = max((int)r[0], (int)r[1]);
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)e, (unsigned)e, false, false);
    e = max((int)r[0], (int)r[1]);
  }
  return e > -0x40000 ? -e : 0;
}

// NC: observed columns (0..4).  The step's evidence e_t(y) = ebase(y) x one
// table entry per column: the codes of the next 8 steps are read a chunk
// ahead and each entry one step ahead, so no LDS load waits on the
// recursion's path (evidence() did two dependent LDS round trips per step).
// the filter wave's column (forward) / row (backward) of A: Ac[b][j] =
// A(16 b + j, y) / A(y, 16 b + j), loaded before the block stages its tables
// so that the loads' latency overlaps the staging
__device__ __forceinline__ void r64_load_A(const WideArgs& a, bool fwd, int y, double (&Ac)[4][16]) {
#pragma unroll
  for (int b = 0; b < 4; b++)
#pragma unroll
    for (int j = 0; j < 16; j++) Ac[b][j] = fwd ? a.A[(16 * b + j) * 64 + y] : a.A[y * 64 + 16 * b + j];
}

// timing-only diagnostics builds (wrong results): 1 -- the filters run their
// steps without the chunk, phase and closing barriers and the partners do
// nothing, so the stamps give the filter step's own cost in the kernel's
// code; 2 -- every barrier kept, the partners doing nothing else
#ifndef NIPAMD_R64_SOLO
#define NIPAMD_R64_SOLO 0
#endif
template <bool FWD, int NC>
__device__ __forceinline__ void r64_filter(const WideArgs& a, const W4Lds& L, int y, const double (&Ac)[4][16],
                                           int nA, int nAi, int nB, int nBi) {
  const int T = a.T, H = a.H;
  const int d = FWD ? 0 : 1;
  double x;
  int sc = 0;
  if (FWD) {
    x = a.pi[y];
  } else {
    x = (nA + nB > 0) ? evidence(a, L, T - 1, y) * (y < a.N ? 1.0 : 0.0) : 0.0;   // e_{T-1} o beta_{T-1}
    sc = -__builtin_amdgcn_frexp_exp(wave_sum(x));
  }
  const double eb = L.tab[L.eoff + y];
  const int toff[4] = {L.toff0, L.toff1, L.toff2, L.toff3};
  constexpr int NK = NC > 0 ? NC : 1;
  const bool dg = a.diag != nullptr;
  const unsigned long long c0 = dg ? __builtin_readcyclecounter() : 0;
  unsigned long long twait = 0;
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
  auto phase = [&](int n, int ni, int ph) {
    const lds_u8* pc[NK];
#pragma unroll
    for (int k = 0; k < NK; k++) pc[k] = L.pcodes + (k * 2 + d) * L.PAB + (ph ? L.PA : 0);
    // a chunk's 8 codes (two dwords, in VGPRs until the next chunk), and its
    // table entries from them -- both one chunk ahead, so that every LDS
    // load has a whole chunk and the chunk's barrier (lgkmcnt(0)) behind it
    // before its value is used, and no wait lands on the recursion's path
    auto ldw = [&](int c, u32x2 (&w)[NK]) {
#pragma unroll
      for (int k = 0; k < NC; k++) w[k] = *(const lds_u32x2*)(pc[k] + c);
    };
    auto ldt = [&](const u32x2 (&w)[NK], double (&tv)[NK][8]) {
#pragma unroll
      for (int k = 0; k < NC; k++) {
        const unsigned w0 = __builtin_amdgcn_readfirstlane(w[k].x), w1 = __builtin_amdgcn_readfirstlane(w[k].y);
#pragma unroll
        for (int j = 0; j < 8; j++) tv[k][j] = L.tab[toff[k] + (((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 0xff) * 64 + y];
      }
    };
    u32x2 wn[NK];                               // codes of the next chunk
    double tc[NK][8];                           // table entries of this chunk
    {
      u32x2 w0[NK];
      ldw(0, w0);
      ldt(w0, tc);
    }
    ldw(8, wn);
    // one step i (j = i mod 8, the unrolled position; rs: rescale after it)
    auto step = [&](int i, int j, bool rs) {
      double xb[4];
      blocks_of(x, xb);
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      fmac16(acc, xb[0], Ac[0]);
      fmac16(acc, xb[1], Ac[1]);
      fmac16(acc, xb[2], Ac[2]);
      fmac16(acc, xb[3], Ac[3]);
      double e = eb;                              // evidence(): the same products in the same order
#pragma unroll
      for (int k = 0; k < NC; k++) e *= tc[k][j];
      const double u = __builtin_ldexp((acc[0] + acc[1]) + (acc[2] + acc[3]), sc);
      const double p = u * e;
      const int slot = i & (kW4Ring - 1);
      L.ring[(d * kW4Ring + slot) * 64 + y] = FWD ? p : u;
      if (FWD) L.uring[slot * 64 + y] = u;
      sc = rs ? max_exp_rescale(p) : 0;
      x = p;
    };
    for (int c = 0; c < ni; c += 8) {
      double tn[NK][8];
      ldt(wn, tn);                              // the next chunk's entries
      u32x2 w2[NK];
      ldw(c + 16, w2);                          // the codes of the one after
      if (c + 8 <= n) {
        // a full chunk: no bounds checks, the rescales at compile-time positions
        // (every 4th step; the phase's last step, if it ends here, is j = 7)
#pragma unroll
        for (int j = 0; j < 8; j++) step(c + j, j, (j & (kW4Rescale - 1)) == kW4Rescale - 1);
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int i = c + j;
          if (i < n) step(i, j, (i & (kW4Rescale - 1)) == kW4Rescale - 1 || i == n - 1);
        }
      }
#pragma unroll
      for (int k = 0; k < NC; k++) {
        wn[k] = w2[k];
#pragma unroll
        for (int j = 0; j < 8; j++) tc[k][j] = tn[k][j];
      }
      const unsigned long long tb = dg ? __builtin_readcyclecounter() : 0;
      if (NIPAMD_R64_SOLO == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else block_barrier();                             // the chunk to the partner
      if (dg) twait += __builtin_readcyclecounter() - tb;
    }
  };
  // phase A: forward alpha_0..alpha_{H-1}; backward beta_{T-2}..beta_H
  phase(nA, nAi, 0);
  if (NIPAMD_R64_SOLO != 1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  // phase B: forward alpha_H..alpha_{T-1}; backward beta_{H-1}..beta_0
  phase(nB, nBi, 1);
  if (NIPAMD_R64_SOLO != 1) block_barrier();            // the partners' ll hand-over
  if (dg && y == 0) {
    a.diag[blockIdx.x * 16 + (FWD ? 0 : 4) + 0] = __builtin_readcyclecounter() - c0;
    a.diag[blockIdx.x * 16 + (FWD ? 0 : 4) + 1] = twait;
  }
}

// The partner takes the ring's chunk c (steps 8c..8c+7) after the chunk's
// barrier, while the filter writes chunk c + 1 into the ring's other half.
template <bool FWD>
__device__ __forceinline__ void r64_partner(const WideArgs& a, const W4Lds& L, int y, long b, int nA, int nAi,
                                            int nB, int nBi, int nAf, int nBf) {
  const int T = a.T, H = a.H;
  const int d = FWD ? 0 : 1;
  double* const Srow = a.S + (size_t)b * chain_scratch_row64(T) + (size_t)kW4G * 64 + y;
  double* const Prow = (a.post && y < a.N) ? a.post + (size_t)b * a.post_bstride + a.post_off + y : nullptr;
  const double s = a.s[y];
  double m = 1.0, zmin = 1.0;
  int e = 0;
  // the forward ll (nip.c:1461-1474) split between the partners: the forward
  // one sums z2 = sum alpha_t, the backward one z1 = sum u_t s, per forward
  // step (both on the same power-of-two scale; mantissa and exponent kept
  // apart); they meet in LDS after the last chunk
  auto zval = [&](int slot) { return FWD ? L.ring[slot * 64 + y] : L.uring[slot * 64 + y] * s; };
  auto ll_acc = [&](double z) {
    if (FWD) zmin = __builtin_fmin(zmin, z);
    m *= __builtin_amdgcn_frexp_mant(z); e += __builtin_amdgcn_frexp_exp(z);
    const int k = __builtin_amdgcn_frexp_exp(m);
    m = __builtin_ldexp(m, -k); e += k;
  };
  const unsigned long long c0 = a.diag ? __builtin_readcyclecounter() : 0;
  if (!FWD && !a.filter) Srow[(long)(T - 1) * 64] = y < a.N ? 1.0 : 0.0;   // beta_{T-1}, T-1 >= H
  // phase A: the interface vectors to the scratch
  for (int c = 0; c < nAi; c += 8) {
    block_barrier();
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int j = c + k;
      const int slot = j & (kW4Ring - 1);
      if (j < nA) store_pol<NIPAMD_WIDE_SCR_NT>(Srow + (long)(FWD ? j : T - 2 - j) * 64, (double)L.ring[(d * kW4Ring + slot) * 64 + y]);
      if (j < nAf) ll_acc(wave_sum(zval(slot)));
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // phase B: posterior = normalise(this o other); the other direction's
  // vectors come from the scratch one chunk ahead, ping-ponged between two
  // register sets
  const int tB = FWD ? H : H - 1;
  auto tof = [&](int j) { return FWD ? tB + j : tB - j; };
  const double* const Sld = a.filter ? a.S + y : Srow;   // forward_inference: a valid dummy row
  const long sstr = a.filter ? 0 : 64;
  auto load8 = [&](double (&r)[8], int c) {
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = load_pol<NIPAMD_SCR_NTLD>(Sld + (long)tof(8 * c + k) * sstr);   // guards cover the over-run
  };
  auto chunk = [&](const double (&r)[8], int c) {
    block_barrier();                                 // the filter's chunk c is in the ring
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int j = 8 * c + k;
      const int slot = j & (kW4Ring - 1);
      // the posterior's sum and the ll's, interleaved
      double z[2] = {L.ring[(d * kW4Ring + slot) * 64 + y] * (a.filter ? 1.0 : r[k]), zval(slot)};
      const double pr = z[0];
      wave_sum_n<2>(z);
      if (j < nB) {
        const double q = pr * recip(z[0]);           // an all-zero row stays zero
        if (Prow) store_pol<NIPAMD_POST_NT>(Prow + (long)tof(j) * a.post_tstride, q);
      }
      if (j < nBf) ll_acc(z[1]);
    }
  };
  const int nch = nBi / 8;                           // nBi: a multiple of 8 (kernel)
  double ra[8], rb[8];
  load8(ra, 0);
  for (int c = 0; c < nch; c += 2) {
    load8(rb, c + 1);
    chunk(ra, c);
    if (c + 1 >= nch) break;
    load8(ra, c + 2);
    chunk(rb, c + 1);
  }
  if (a.diag && y == 0) a.diag[blockIdx.x * 16 + (FWD ? 8 : 12)] = __builtin_readcyclecounter() - c0;
  // z1's mantissa and exponent to the forward partner (L.xb: unused by this
  // kernel); every wave of the block takes this last barrier
  if (!FWD && y == 0) {
    L.xb[0] = m;
    L.xb[1] = (double)e;
  }
  block_barrier();
  if (FWD && y == 0) {
    const double m1 = L.xb[0];
    const int e1 = (int)L.xb[1];
    double ll = log(m) - log(m1) + (double)(e - e1) * 0.69314718055994530942;
    const bool dead = zmin == 0.0;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    if (a.status) a.status[b] = dead ? 1u : 0u;
  }
}

// R64: chain_row64_kernel's roles (one filter wave per direction, 4 waves);
// NC: its observed columns
template <bool R64, int NC>
__global__ __launch_bounds__(R64 ? kR64Threads : kW4Threads, 1)
void chain_wide4_kernel(WideArgs a) {
  constexpr int kThreads = R64 ? kR64Threads : kW4Threads;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  lds_d* sm = (lds_d*)(smem);
  W4Lds L;
  L.xb = sm;
  L.pb = L.xb + 2 * kQ * 64;
  L.ring = L.pb + 2 * 2 * kQ * 64;
  L.uring = L.ring + 2 * kW4Ring * 64;
  lds_d* tab = L.uring + kW4Ring * 64;
  int rows = 0, toff[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (k < a.ncol) { toff[k] = rows * 64; rows += a.M[k] + 2; }
  L.toff0 = toff[0]; L.toff1 = toff[1]; L.toff2 = toff[2]; L.toff3 = toff[3];
  L.eoff = rows * 64;
  L.tab = tab;
  lds_u8* codes = (lds_u8*)(tab + (rows + 1) * 64);
  L.codes = codes;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long b = blockIdx.x;
  const int T = a.T, Tr = chain_codes_row(T);
  L.Tr = Tr;
  const unsigned long long k0 = a.diag ? __builtin_readcyclecounter() : 0;   // diagnostics: the block's entry
  if (a.diag && tid == 0) a.diag[b * 16 + 11] = __builtin_amdgcn_s_memrealtime();
  double Ac[4][16];
  if (R64 && wave < 2) r64_load_A(a, wave == 0, lane, Ac);
  // stage the evidence tables and this sequence's codes
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (k < a.ncol)
      for (int i = tid; i < (a.M[k] + 2) * 64; i += kThreads) tab[toff[k] + i] = a.tab[k][i];
  for (int i = tid; i < 64; i += kThreads) tab[L.eoff + i] = a.ebase[i];
  for (int k = 0; k < a.ncol; k++) {
    const int M = a.M[k];
    for (int i = tid; i < Tr; i += kThreads) {
      const int t = i - kW4G;
      int c = M;                                      // missing / guard
      if (t >= 0 && t < T) {
        const int o = a.obs[b * a.obs_bstride + (long)t * a.obs_tstride + a.col[k]];
        c = o < 0 ? M : (o < M ? o : M + 1);
      }
      codes[k * Tr + i] = (uint8_t)c;
    }
  }
  __syncthreads();
  const int H = a.H;
  const R64Iters it(T, H, a.filter != 0);
  const int nAf = it.nAf, nAb = it.nAb, nBf = it.nBf, nBb = it.nBb, nAi = it.nAi, nBi = it.nBi;
  if constexpr (R64) {
    // the filters' codes in processing order (R64Iters; guards: row M_k)
    L.PA = it.PA();
    L.PAB = it.PA() + it.PB();
    L.pcodes = codes + ((a.ncol * Tr + 7) & ~7);
    for (int k = 0; k < a.ncol; k++)
      for (int i = tid; i < 2 * L.PAB; i += kThreads) {
        const int dd = i >= L.PAB, r = i - dd * L.PAB, ph = r >= L.PA, j = r - ph * L.PA;
        const int n = dd ? (ph ? nBb : nAb) : (ph ? nBf : nAf);
        const int t = dd ? (ph ? H - 1 - j : T - 2 - j) : (ph ? H + j : j);
        L.pcodes[k * 2 * L.PAB + i] = j < n ? codes[k * Tr + kW4G + t] : (uint8_t)a.M[k];
      }
    __syncthreads();
    if (a.diag && tid == 0) a.diag[b * 16 + 9] = __builtin_readcyclecounter() - k0;   // staging
    if (wave == 0) r64_filter<true, NC>(a, L, lane, Ac, nAf, nAi, nBf, nBi);
    else if (wave == 1) r64_filter<false, NC>(a, L, lane, Ac, nAb, nAi, nBb, nBi);
    else if (NIPAMD_R64_SOLO == 1) return;
    else if (NIPAMD_R64_SOLO == 2) {
      // the partners' barriers only (the filters' chunk, phase and closing ones)
      for (int c = 0; c < nAi; c += 8) block_barrier();
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      for (int c = 0; c < nBi; c += 8) block_barrier();
      block_barrier();
    }
    else if (wave == 2) r64_partner<true>(a, L, lane, b, nAf, nAi, nBf, nBi, nAf, nBf);
    else r64_partner<false>(a, L, lane, b, nAb, nAi, nBb, nBi, nAf, nBf);
    if (a.diag && tid == 0) {
      a.diag[b * 16 + 10] = __builtin_readcyclecounter() - k0;  // the block, entry to exit
      a.diag[b * 16 + 13] = __builtin_amdgcn_s_memrealtime();
    }
  } else {
    if (wave < kQ) w4_filter<true>(a, L, wave, lane, nAf, nAi, nBf, nBi);
    else if (wave < 2 * kQ) w4_filter<false>(a, L, wave - kQ, lane, nAb, nAi, nBb, nBi);
    else if (wave == 2 * kQ) w4_partner<true>(a, L, lane, b, nAf, nAi, nBf, nBi);
    else w4_partner<false>(a, L, lane, b, nAb, nAi, nBb, nBi);
  }
}

}  // namespace

size_t chain_wide4_lds_bytes(const WideArgs& a) {
  int rows = 0;
  for (int k = 0; k < a.ncol; k++) rows += a.M[k] + 2;
  const R64Iters it(a.T, a.H, a.filter != 0);
  return (size_t)(2 * kQ * 64 + 2 * 2 * kQ * 64 + 2 * kW4Ring * 64 + kW4Ring * 64 + (rows + 1) * 64) *
             sizeof(double) +
         (((size_t)(a.ncol > 0 ? a.ncol : 1) * chain_codes_row(a.T) + 7) & ~(size_t)7) +
         (size_t)a.ncol * 2 * (it.PA() + it.PB());          // chain_row64_kernel's pcodes
}

#ifndef NIPAMD_R64
#define NIPAMD_R64 1               // 33..64 states: chain_row64_kernel (0: chain_wide4_kernel, four waves per direction)
#endif

namespace {
template <int NC>
int launch_r64(const WideArgs& a, size_t lds, hipStream_t stream) {
  static size_t lds_set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_wide4_kernel<true, NC>), lds, lds_set)) return rc;
  hipLaunchKernelGGL((chain_wide4_kernel<true, NC>), dim3((unsigned)a.B), dim3(kR64Threads), lds, stream, a);
  return 0;
}
}  // namespace

int chain_wide4_launch(const WideArgs& a, hipStream_t stream) {
  const size_t lds = (chain_wide4_lds_bytes(a) + 15) & ~(size_t)15;
  if (lds > 160 * 1024) return -2;
  if (NIPAMD_R64) {
    switch (a.ncol) {
      case 0: if (int rc = launch_r64<0>(a, lds, stream)) return rc; break;
      case 1: if (int rc = launch_r64<1>(a, lds, stream)) return rc; break;
      case 2: if (int rc = launch_r64<2>(a, lds, stream)) return rc; break;
      case 3: if (int rc = launch_r64<3>(a, lds, stream)) return rc; break;
      default: if (int rc = launch_r64<4>(a, lds, stream)) return rc; break;
    }
    g_last_kernel = "chain_row64_kernel";
  } else {
    static size_t lds_set[kMaxDevices] = {};
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_wide4_kernel<false, 0>), lds, lds_set)) return rc;
    hipLaunchKernelGGL((chain_wide4_kernel<false, 0>), dim3((unsigned)a.B), dim3(kW4Threads), lds, stream, a);
    g_last_kernel = "chain_wide4_kernel";
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
