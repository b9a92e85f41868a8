// chain_mfma_wide.hip -- matrix-core forward-backward for interface chains of
// up to 32 states with up to four observed children (SURVEY 8(d) config 3:
// demo1 @ 32 states, after the host folds D1 into the transition; and N <= 16
// chains observed through several children).
//
// The recursion is the one in chain_kernels.hip / chain_mfma.hip (two-filter
// smoothing, nip.c:1320-1581), with the evidence of step t the product of one
// LDS table row per observed child (the unobserved children's row sums are
// folded into the first table by the host):
//   e_t[y] = prod_k T_k[code_k(t)][y]
//
// Layout: NT = N / 16 state tiles.  Sixteen chains of one direction share a
// wave; the 16 x 16 tile (qo, qi) of the mat-vec is four v_mfma_f64_16x16x4
// whose D registers are the next step's B operands (see chain_mfma.hip for the
// register algebra).  Internal row g + 4r of tile q is state
// 16q + state_of(g, r), so lane (g = l >> 4, j = l & 15) owns states
// 16q + {2g, 2g+1, 8+2g, 9+2g} of chain j in every tile q.
// Block = two groups of 16 sequences, eight waves, two per SIMD: each SIMD
// runs one group's filter (matrix core) and one group's partner (VALU), so
// all four matrix pipes carry a filter:
//   waves 0, 1: group 0 forward / backward filter   (MFMA + evidence)
//   waves 2, 3: group 1 forward / backward filter
//   waves 4, 5: group 0 forward / backward partner (scratch copy, ll,
//               posteriors of t >= H / t < H)
//   waves 6, 7: group 1 forward / backward partner
// (a workgroup's waves go to the CU's SIMDs round robin, wave w and w + 4 on
// one SIMD).  With one group per block (round 2) the filters had two SIMDs
// to themselves, the 93 KB of LDS allowed one block per CU, and the other two
// matrix pipes idled.  LDS rings hold two chunks of CH steps per direction
// and group (CH = 8 / NT, a slot is 16 KB); one s_barrier per chunk hands a
// slot from filter to partner.  The observation codes are read from HBM by
// the filters, two chunks ahead, instead of being staged in LDS.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

#include "chain_kernels.h"
#include "store_pol.h"

namespace nipamd {

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

#ifndef NIPAMD_MW_ABLATE
#define NIPAMD_MW_ABLATE 0     // timing-only builds: 1 partners only keep the barriers,
#endif                         // 2 filters skip the mat-vec
#ifndef NIPAMD_MW_SPARSE
#define NIPAMD_MW_SPARSE 0     // timing-only builds: the filters rescale once per chunk (the ll is then wrong)
#endif
#ifndef NIPAMD_MW_ANALYTIC
#define NIPAMD_MW_ANALYTIC 1   // smoothing: analytic posterior normalisation, the ll in the forward filter (0: A/B builds)
#endif
constexpr int kWSeq = 16;                  // sequences per group
constexpr int kWGroups = 2;                // groups per block
constexpr int kWThreads = 512;
constexpr int kWG = kScratchGuard;

__host__ __device__ constexpr int state_of(int g, int r) { return r < 2 ? 2 * g + r : 6 + 2 * g + r; }

__device__ __forceinline__ double swap32_sum(double x) {     // x[l] + x[l ^ 32]
  double xc = x;
  asm("" : "+v"(xc));   // the swap's second operand: a whole-double copy (one v_mov_b64)
  const auto rl = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

__device__ __forceinline__ double swap16_sum(double x) {     // x[l] + x[l ^ 16]
  double xc = x;
  asm("" : "+v"(xc));   // the swap's second operand: a whole-double copy (one v_mov_b64)
  const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// sums over aligned groups of L = 8 or 16 lanes, level by level over n
// independent values; every level pairs equal partial sums (or adds a value
// to its mirror), so all lanes of a group hold identical bits
template <int L, int n>
__device__ __forceinline__ void sumL_n(double (&x)[n]) {
#pragma unroll
  for (int i = 0; i < n; i++) asm("" : "+v"(x[i]));   // one rounded value per lane: no fma contraction
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += dpp64<0xB1>(x[i]);     // quad_perm [1,0,3,2]
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += dpp64<0x4E>(x[i]);     // quad_perm [2,3,0,1]
#pragma unroll
  for (int i = 0; i < n; i++) x[i] += dpp64<0x141>(x[i]);    // row_half_mirror
  if (L == 16) {
#pragma unroll
    for (int i = 0; i < n; i++) x[i] += dpp64<0x140>(x[i]);  // row_mirror
  }
}

template <int n>
__device__ __forceinline__ void recip_n(const double (&c)[n], double (&r)[n]) {
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = __builtin_amdgcn_rcp(c[i]);
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = __builtin_fma(r[i], __builtin_fma(-c[i], r[i], 1.0), r[i]);
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = __builtin_fma(r[i], __builtin_fma(-c[i], r[i], 1.0), r[i]);
#pragma unroll
  for (int i = 0; i < n; i++) r[i] = c[i] != 0.0 ? r[i] : 0.0;   // all-zero rows stay zero
}

__device__ __forceinline__ v4d ldexp4(v4d v, int k) {
  v4d r;
  r.x = __builtin_ldexp(v.x, k); r.y = __builtin_ldexp(v.y, k);
  r.z = __builtin_ldexp(v.z, k); r.w = __builtin_ldexp(v.w, k);
  return r;
}

__device__ __forceinline__ v4d load4(const double* p) {      // p = row + 16q + 2g
  const v2d a = *reinterpret_cast<const v2d*>(p);
  const v2d b = *reinterpret_cast<const v2d*>(p + 8);
  return v4d{a.x, a.y, b.x, b.y};
}

#ifndef NIPAMD_WAIT_TIMES
#define NIPAMD_WAIT_TIMES 0        // stamps builds: per-wave phase and barrier-wait cycles (a.diag)
#endif
// per-wave cycle stamps of the stamps build: phase A / its barrier waits /
// phase B / its barrier waits, into a.diag[block][wave][4]
struct MwDiag {
  unsigned long long t0 = 0, ta = 0, wa = 0, wb = 0;
  bool inB = false;
  __device__ __forceinline__ void start() { if (NIPAMD_WAIT_TIMES) t0 = __builtin_readcyclecounter(); }
  __device__ __forceinline__ void phase() {
    if (NIPAMD_WAIT_TIMES) { ta = __builtin_readcyclecounter(); inB = true; }
  }
  // unit: the block's group (blocks of 16 sequences, as the host counts them)
  __device__ __forceinline__ void write(unsigned long long* d, long unit, int wave, int lane) {
    if (!NIPAMD_WAIT_TIMES || !d || lane != 0) return;
    unsigned long long* p = d + (size_t)unit * 16 + wave * 4;
    p[0] = ta - t0; p[1] = wa; p[2] = __builtin_readcyclecounter() - ta; p[3] = wb;
  }
};

__device__ __forceinline__ void barrier_lds(MwDiag* dg = nullptr) {
#if NIPAMD_WAIT_TIMES
  const unsigned long long t = __builtin_readcyclecounter();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (dg) (dg->inB ? dg->wb : dg->wa) += __builtin_readcyclecounter() - t;
#else
  (void)dg;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
}

template <int NT>
struct Geo {
  static constexpr int NP = 16 * NT;          // states per chain row
  static constexpr int LPC = NP / 2;          // partner lanes per chain (2 states each)
  static constexpr int CH = 64 / LPC;         // steps per chunk (= chains per partner pass)
  static constexpr int QN = kWSeq / CH;       // partner passes over the 16 chains
  static constexpr int kStep = kWSeq * NP;    // doubles per step of 16 chains
  // LDS evidence-table row stride: NP + 2 doubles, so that sixteen chains
  // reading sixteen different rows start at banks 4 * row apart instead of
  // all at bank 0 (an NP-double row is 128 or 256 B: 16-way conflicts)
  static constexpr int NPS = NP + 2;
  static constexpr int kSlot = CH * kStep;    // doubles per ring slot (16 KB)
  // chain j's piece p (16 bytes) within a step, XOR-swizzled by j & 7
  __device__ static int piece_off(int j, int p) { return j * NP + ((p ^ (j & 7)) << 1); }
};

__host__ __device__ inline long wblock_scratch(int NT, int T) { return (long)(T + 2 * kWG) * kWSeq * 16 * NT; }
__host__ __device__ inline long wblock_exps(int T) { return (long)(T + 2 * kWG) * kWSeq; }   // ints

struct WCtx {
  const double* tab;       // LDS tables
  const int* obs;          // this chain's observations (null: an absent sequence or no observed column)
  int ots;                 // their time stride
  int col[4], M[4];        // per observed column: offset within a time step, states
  int T;
  int tab_off[4];          // per column: LDS offset of its table + 2g
  int ncol;
  double* out;             // this direction's ring [2][kSlot]
  double* zr;              // forward: z2 ring [2][CH][16]
  int* er;                 // AN: this direction's exponent ring [2][CH][16]
  int wo[2][2];            // [tile][half] piece offsets of this lane
  bool zw;
  int j;                   // this lane's chain
};

// NC: observed columns (1..4; 0 runs as 1, column 0 carrying the row sums),
// a template parameter so that the per-step evidence gather is branch-free and
// its LDS loads can be scheduled under the MFMAs
// AN (smoothing, round 5): every step's accumulated exponent goes to the
// exponent ring (alpha^_t = alpha_t 2^Ef_t, beta^_t = beta_t 2^Eb_t), so the
// partners normalise the posteriors analytically (wpartner), and the forward
// filter keeps the ll itself (nip.c:1458-1474: m2_t = z2_t, m1_{t+1} =
// 2^sc_{t+1} alpha^_t . A s), off its recursion's dependency chain
template <bool FWD, int NT, int NC, bool AN = false>
struct WChain {
  using G = Geo<NT>;
  double Aop[NT][NT][4];
  v4d X[NT];
  int sc = 0;
  int E = 0;                               // AN: the last message's accumulated exponent
  double m2 = 1.0, m1 = 1.0, zmin = 1.0;   // AN, forward: ll mantissas (exponents apart)
  int e2 = 0, e1 = 0;
  v4d wv[NT];                              // AN, forward: this lane's states of w = A s_all
  __device__ __forceinline__ void renorm() {
    const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
    const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
  }

  // column k's observation at t, raw (-1: missing, also outside 0..T-1)
  __device__ __forceinline__ int raw(const WCtx& c, int k, int t) const {
    return (c.obs && t >= 0 && t < c.T) ? c.obs[(long)t * c.ots + c.col[k]] : -1;
  }
  // its table row: the state, M (missing) or M + 1 (out of range: all zero)
  __device__ __forceinline__ int code(const WCtx& c, int k, int o) const {
    return o < 0 ? c.M[k] : (o < c.M[k] ? o : c.M[k] + 1);
  }
  __device__ __forceinline__ void evidence(const WCtx& c, int t, v4d (&e)[NT]) const {
    int cd[NC];
#pragma unroll
    for (int k = 0; k < NC; k++) cd[k] = code(c, k, raw(c, k, t));
    v4d r[NC][NT];
    rows_of(c, cd, r);
    product(c, r, e);
  }

  __device__ __forceinline__ void rows_of(const WCtx& c, const int (&cd)[NC], v4d (&r)[NC][NT]) const {
#pragma unroll
    for (int k = 0; k < NC; k++) {
#pragma unroll
      for (int q = 0; q < NT; q++) r[k][q] = load4(c.tab + c.tab_off[k] + cd[k] * G::NPS + 16 * q);
    }
  }
  __device__ __forceinline__ void product(const WCtx& c, const v4d (&r)[NC][NT], v4d (&e)[NT]) const {
#pragma unroll
    for (int q = 0; q < NT; q++) e[q] = r[0][q];
#pragma unroll
    for (int k = 1; k < NC; k++) {
#pragma unroll
      for (int q = 0; q < NT; q++) e[q] *= r[k][q];
    }
  }

  // one step with the evidence rows loaded at its start: the MFMAs first, the
  // evidence product after them (its LDS loads complete under the MFMAs)
  template <bool RS = true>
  __device__ __forceinline__ void step_rows(const WCtx& c, double* L, double* Z, const v4d (&r)[NC][NT],
                                            int* Ez = nullptr, bool last = false) {
    v4d d[NT];
    matvec(d);
    v4d e[NT];
    product(c, r, e);
    finish<RS>(c, L, Z, d, e, Ez, last);
  }

  __device__ __forceinline__ void step(const WCtx& c, double* L, double* Z, const v4d (&e)[NT]) {
    v4d d[NT];
    matvec(d);
    finish(c, L, Z, d, e);
  }

  __device__ __forceinline__ void matvec(v4d (&d)[NT]) {
#pragma unroll
    for (int qo = 0; qo < NT; qo++) d[qo] = v4d{0.0, 0.0, 0.0, 0.0};
#if NIPAMD_MW_ABLATE == 2
#pragma unroll
    for (int qo = 0; qo < NT; qo++) d[qo] = X[qo] * 0.5;
    if (0)
#endif
    // the NT output tiles' accumulation chains interleave
#pragma unroll
    for (int qi = 0; qi < NT; qi++) {
      d[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0][qi][0], X[qi].x, d[0], 0, 0, 0);
      if (NT > 1) d[NT - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[NT - 1][qi][0], X[qi].x, d[NT - 1], 0, 0, 0);
      d[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0][qi][1], X[qi].y, d[0], 0, 0, 0);
      if (NT > 1) d[NT - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[NT - 1][qi][1], X[qi].y, d[NT - 1], 0, 0, 0);
      d[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0][qi][2], X[qi].z, d[0], 0, 0, 0);
      if (NT > 1) d[NT - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[NT - 1][qi][2], X[qi].z, d[NT - 1], 0, 0, 0);
      d[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[0][qi][3], X[qi].w, d[0], 0, 0, 0);
      if (NT > 1) d[NT - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[NT - 1][qi][3], X[qi].w, d[NT - 1], 0, 0, 0);
    }
  }

  template <bool RS = true>
  __device__ __forceinline__ void finish(const WCtx& c, double* L, double* Z, const v4d (&d)[NT],
                                         const v4d (&e)[NT], int* Ez = nullptr, bool last = false) {
    double part = 0.0, py = 0.0;
    if (AN) E += sc;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      const v4d u = ldexp4(d[q], sc);
      const v4d p = u * e[q];
      const v4d keep = FWD ? p : u;
      *reinterpret_cast<v2d*>(L + c.wo[q][0]) = v2d{keep.x, keep.y};
      *reinterpret_cast<v2d*>(L + c.wo[q][1]) = v2d{keep.z, keep.w};
      if (RS) part += (p.x + p.y) + (p.z + p.w);
      if (AN && FWD) py += (p.x * wv[q].x + p.y * wv[q].y) + (p.z * wv[q].z + p.w * wv[q].w);
      X[q] = p;
    }
    if (AN && c.zw) Ez[c.j] = E;
    if (!RS) { sc = 0; return; }
    const double z2 = swap16_sum(swap32_sum(part));
    const int k = __builtin_amdgcn_frexp_exp(z2);
    if (AN && FWD) {
      // m2_t = z2_t; m1_{t+1} = 2^sc_{t+1} y_t, y_t = alpha^_t . w
      asm("" : "+v"(py));
      const double y = swap16_sum(swap32_sum(py));
      zmin = __builtin_fmin(zmin, z2);
      m2 *= z2;
      if (!last) { m1 *= y; e1 -= k; }
      renorm();
    }
    if (!AN && FWD && c.zw) *Z = z2;
    sc = -k;
  }

  // n steps from t0 in nch chunks; the codes of chunk ci + 2 are loaded from
  // HBM when chunk ci ends (two chunks of latency cover), a step's table rows
  // from LDS at its start (under its MFMAs)
  __device__ __forceinline__ void run(const WCtx& c, int n, int nch, int t0, int lane, MwDiag& dg) {
    constexpr int dir = FWD ? 1 : -1;
    constexpr int CH = G::CH;
    int ca[CH][NC], cb[CH][NC];
    auto ldc = [&](int ci, int (&cc)[CH][NC]) {
#pragma unroll
      for (int k = 0; k < CH; k++)
#pragma unroll
        for (int q = 0; q < NC; q++) cc[k][q] = raw(c, q, t0 + dir * (ci * CH + k));
    };
    auto chunk = [&](int ci, int (&cc)[CH][NC]) {
      double* slot = c.out + (ci & 1) * G::kSlot;
      double* zs = (FWD && !AN) ? c.zr + (ci & 1) * CH * kWSeq + (lane & 15) : nullptr;
      int* es = AN ? c.er + (ci & 1) * CH * kWSeq : nullptr;
      const int base = ci * CH;
      const bool full = base + CH <= n;
#pragma unroll
      for (int k = 0; k < CH; k++) {
        if (!full && base + k >= n) break;
        int cd[NC];
#pragma unroll
        for (int q = 0; q < NC; q++) cd[q] = code(c, q, cc[k][q]);
        v4d r[NC][NT];
        rows_of(c, cd, r);
#if NIPAMD_MW_SPARSE
        // timing-only builds: rescale (and publish z2) on the chunk's last step only
        if (k == CH - 1) step_rows<true>(c, slot + k * G::kStep, zs + k * kWSeq, r);
        else step_rows<false>(c, slot + k * G::kStep, zs + k * kWSeq, r);
#else
        if (AN) step_rows(c, slot + k * G::kStep, nullptr, r, es + k * kWSeq, t0 + dir * (base + k) == c.T - 1);
        else step_rows(c, slot + k * G::kStep, zs + k * kWSeq, r);
#endif
      }
      barrier_lds(&dg);
      ldc(ci + 2, cc);
    };
    ldc(0, ca);
    ldc(1, cb);
    for (int ci = 0; ci < nch; ci += 2) {
      chunk(ci, ca);
      if (ci + 1 >= nch) break;
      chunk(ci + 1, cb);
    }
  }
};

template <bool FWD, int NT, int NC, bool AN>
__device__ __forceinline__ void wfilter(const WideMfmaArgs& a, const WCtx& c, double* Sblk, int* Eblk, int lane,
                                        long b0, int nchA, int nchB) {
  using G = Geo<NT>;
  const int j = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  WChain<FWD, NT, NC, AN> ch;
#pragma unroll
  for (int qo = 0; qo < NT; qo++)
#pragma unroll
    for (int qi = 0; qi < NT; qi++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int out = 16 * qo + state_of(j & 3, j >> 2), in = 16 * qi + state_of(g, r);
        ch.Aop[qo][qi][r] = FWD ? a.A[in * 64 + out] : a.A[out * 64 + in];
      }
  if (FWD) {
    double py = 0.0;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      ch.X[q] = load4(a.pi + 16 * q + 2 * g);
      if (AN) {
        ch.wv[q] = load4(a.w + 16 * q + 2 * g);
        py += (ch.X[q].x * ch.wv[q].x + ch.X[q].y * ch.wv[q].y) + (ch.X[q].z * ch.wv[q].z + ch.X[q].w * ch.wv[q].w);
      }
    }
    if (AN) {
      asm("" : "+v"(py));
      ch.m1 = swap16_sum(swap32_sum(py));                 // y_{-1} = prior . w
      ch.renorm();
    }
  } else {
    v4d e[NT];
    ch.evidence(c, T - 1, e);
    double part = 0.0;
    double* row = Sblk + (long)(T - 1) * G::kStep + j * G::NP;   // beta_{T-1} (T-1 >= H)
#pragma unroll
    for (int q = 0; q < NT; q++) {
      v4d beta;
      beta.x = 16 * q + state_of(g, 0) < a.N ? 1.0 : 0.0; beta.y = 16 * q + state_of(g, 1) < a.N ? 1.0 : 0.0;
      beta.z = 16 * q + state_of(g, 2) < a.N ? 1.0 : 0.0; beta.w = 16 * q + state_of(g, 3) < a.N ? 1.0 : 0.0;
      *reinterpret_cast<v2d*>(row + 16 * q + 2 * g) = v2d{beta.x, beta.y};
      *reinterpret_cast<v2d*>(row + 16 * q + 8 + 2 * g) = v2d{beta.z, beta.w};
      ch.X[q] = e[q] * beta;
      part += (ch.X[q].x + ch.X[q].y) + (ch.X[q].z + ch.X[q].w);
    }
    if (AN && g == 0) Eblk[(long)(T - 1) * kWSeq + j] = 0;     // its exponent
    ch.sc = -__builtin_amdgcn_frexp_exp(swap16_sum(swap32_sum(part)));
  }
  MwDiag dg;
  dg.start();
  if (FWD) ch.run(c, H, nchA, 0, lane, dg);
  else ch.run(c, T - 1 - H, nchA, T - 2, lane, dg);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  dg.phase();
  if (FWD) ch.run(c, T - H, nchB, H, lane, dg);
  else ch.run(c, H, nchB, H - 1, lane, dg);
  dg.write(a.diag, b0 / kWSeq, FWD ? 0 : 1, lane);
  if (AN && FWD && g == 0 && b0 + j < a.B) {
    double ll = log(ch.m2) - log(ch.m1) + (double)(ch.e2 - ch.e1) * 0.69314718055994530942;
    const bool dead = ch.zmin == 0.0;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b0 + j] = ll;
    if (a.status) a.status[b0 + j] = dead ? 1u : 0u;
  }
}

// ll of the forward filter (nip.c:1461-1474), kept by the forward partner:
// ll = sum_t log m2_t - log m1_t with m2_t = z2_t (published by the filter)
// and m1_t = 2^sc_t * y_{t-1}, y_t = alpha_t . w, w = A s (s: the product of
// every child's row sums), y_{-1} = prior . w.  Lane: chain q * CH + (L / LPC),
// piece s = L % LPC.
template <int NT>
struct WLL {
  using G = Geo<NT>;
  double m2[G::QN], m1[G::QN], zmin[G::QN];
  int e2[G::QN], e1[G::QN];
  double w0, w1;

  // first: the forward partner's accumulators start with y_{-1} = prior . w;
  // the backward partner's share (phase-B chunks it takes over) starts at 1
  __device__ __forceinline__ void init(const WideMfmaArgs& a, int s, bool first = true) {
    w0 = a.w[2 * s]; w1 = a.w[2 * s + 1];
    double y[1] = {a.pi[2 * s] * w0 + a.pi[2 * s + 1] * w1};
    sumL_n<G::LPC>(y);
#pragma unroll
    for (int q = 0; q < G::QN; q++) { m2[q] = 1.0; m1[q] = first ? y[0] : 1.0; zmin[q] = 1.0; e2[q] = 0; e1[q] = 0; }
  }
  // the backward partner's share to LDS (5 values per lane and pass), and its product into this one
  __device__ __forceinline__ void put(double* L, int lane) const {
#pragma unroll
    for (int q = 0; q < G::QN; q++) {
      double* p = L + (q * 64 + lane) * 5;
      p[0] = m2[q]; p[1] = m1[q]; p[2] = zmin[q]; p[3] = (double)e2[q]; p[4] = (double)e1[q];
    }
  }
  __device__ __forceinline__ void take(const double* L, int lane) {
#pragma unroll
    for (int q = 0; q < G::QN; q++) {
      const double* p = L + (q * 64 + lane) * 5;
      m2[q] *= p[0]; m1[q] *= p[1]; zmin[q] = __builtin_fmin(zmin[q], p[2]);
      e2[q] += (int)p[3]; e1[q] += (int)p[4];
      const int k2 = __builtin_amdgcn_frexp_exp(m2[q]); m2[q] = __builtin_ldexp(m2[q], -k2); e2[q] += k2;
      const int k1 = __builtin_amdgcn_frexp_exp(m1[q]); m1[q] = __builtin_ldexp(m1[q], -k1); e1[q] += k1;
    }
  }
  __device__ __forceinline__ void step(int q, double y, double z2, bool last, bool renorm) {
    zmin[q] = __builtin_fmin(zmin[q], z2);
    m2[q] *= z2;
    if (!last) { m1[q] *= y; e1[q] -= __builtin_amdgcn_frexp_exp(z2); }
    if (renorm) {
      const int k2 = __builtin_amdgcn_frexp_exp(m2[q]); m2[q] = __builtin_ldexp(m2[q], -k2); e2[q] += k2;
      const int k1 = __builtin_amdgcn_frexp_exp(m1[q]); m1[q] = __builtin_ldexp(m1[q], -k1); e1[q] += k1;
    }
  }
  __device__ __forceinline__ void write(const WideMfmaArgs& a, long b0, int lane) {
    if (lane % G::LPC != 0) return;
#pragma unroll
    for (int q = 0; q < G::QN; q++) {
      const long b = b0 + q * G::CH + lane / G::LPC;
      if (b >= a.B) continue;
      double ll = log(m2[q]) - log(m1[q]) + (double)(e2[q] - e1[q]) * 0.69314718055994530942;
      const bool dead = zmin[q] == 0.0;
      if (dead) ll = -DBL_MAX;
      if (a.ll) a.ll[b] = ll;
      if (a.status) a.status[b] = dead ? 1u : 0u;
    }
  }
};

// Partner wave of one direction.  Phase A: the slot's steps to the block's
// scratch S[t][16 chains][NP] (coalesced, 1 KB per store instruction).  Phase
// B: lane (hi = L / LPC, s = L % LPC) takes step hi of the chunk in address
// order and states 2s, 2s+1 of every chain: ring value times the other
// direction's vector (scratch, one chunk prefetched), normalised over the
// chain's LPC lanes; with N == NP and dense rows, one contiguous 1 KB
// posterior run per store instruction.
// Phase B's ll work is shared: the forward partner takes the forward ring's
// even chunks, the backward partner (which has no ll of its own and waits at
// the barriers otherwise) the odd ones; its partial products join the forward
// partner's through LDS after the block's closing barrier.
// AN (smoothing, round 5): the filters publish each message's accumulated
// exponent (alpha^_t = alpha_t 2^Ef_t, beta^_t = beta_t 2^Eb_t; phase A's go
// to the scratch next to the messages), so sum_y alpha^_t beta^_t =
// Z 2^(Ef_t + Eb_t) for every t: one sum per chain at the partner's first
// phase-B step (c*, exponent E*, kept in LDS) normalises every posterior,
//   posterior_t = alpha^_t o beta^_t 2^(E* - Ef_t - Eb_t) / c*
// -- a multiply and an ldexp where each (chain, step) took a 16-lane DPP sum
// and a Newton reciprocal.  The ll is the forward filter's (WChain).
template <bool FWD, bool PVEC, int NT, bool FILT, bool AN = false>
__device__ __forceinline__ void wpartner(const WideMfmaArgs& a, const double* out, const double* fring,
                                         const double* zr, double* Sblk, int lane, long b0, int nchA, int nchB,
                                         const int* er = nullptr, int* Eblk = nullptr, double* cz = nullptr) {
  using G = Geo<NT>;
  constexpr int NP = G::NP, LPC = G::LPC, CH = G::CH, QN = G::QN;
  const int T = a.T, H = a.H;
  const int s = lane % LPC, hi = lane / LPC;
  const int nA = FWD ? H : T - 1 - H, nB = FWD ? T - H : H;
  const int tA = FWD ? 0 : T - 2, tB = FWD ? H : H - 1;
  constexpr int dir = FWD ? 1 : -1;
  const int kB = FWD ? hi : CH - 1 - hi;
  auto tlow = [&](int ci) { return FWD ? tB + ci * CH : tB - ci * CH - (CH - 1); };

  MwDiag dg;
  dg.start();
  WLL<NT> ll;
  ll.init(a, s, FWD);
  auto ll_chunk = [&](int ci, int n, int t0) {
    const double* slot = fring + (ci & 1) * G::kSlot;
    const double* zs = zr + (ci & 1) * CH * kWSeq;
    const bool full = ci * CH + CH <= n;
    double y[CH * QN];
#pragma unroll
    for (int k = 0; k < CH; k++)
#pragma unroll
      for (int q = 0; q < QN; q++) {
        const v2d v = *reinterpret_cast<const v2d*>(slot + k * G::kStep + G::piece_off(q * CH + hi, s));
        y[k * QN + q] = v.x * ll.w0 + v.y * ll.w1;
      }
    sumL_n<LPC>(y);
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const int i = ci * CH + k;
      if (i >= n) break;
      const bool last = t0 + i == T - 1;
#pragma unroll
      for (int q = 0; q < QN; q++)
        ll.step(q, y[k * QN + q], zs[k * kWSeq + q * CH + hi], last, !full || (k & 3) == 3);
    }
  };
  double* const sink = FILT ? a.S + 2 * s
                            : a.S + (size_t)((a.B + kWSeq - 1) / kWSeq) * wblock_scratch(NT, T) + 2 * s;
  const bool st0 = 2 * s < a.N, st1 = 2 * s + 1 < a.N;
  // normalised posteriors of ring step kk (time t) times o, for the 16 chains
  auto emit = [&](const double* slot, int kk, int t, bool ok, const v2d (&o)[kWSeq]) {
#pragma unroll
    for (int q0 = 0; q0 < kWSeq; q0 += 8) {
      double px[8], py[8], z[8], r[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const v2d v = *reinterpret_cast<const v2d*>(slot + kk * G::kStep + G::piece_off(q0 + i, s));
        px[i] = v.x * o[q0 + i].x; py[i] = v.y * o[q0 + i].y;
        z[i] = px[i] + py[i];
      }
      sumL_n<LPC>(z);
      recip_n(z, r);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const long bb = b0 + q0 + i;
        if constexpr (PVEC) {
          double* p = (ok && bb < a.B) ? a.post + (size_t)bb * a.post_bstride + (long)t * NP + a.post_off + 2 * s
                                       : sink;
          store_pol<NIPAMD_POST_NT>(reinterpret_cast<v2d*>(p), v2d{px[i] * r[i], py[i] * r[i]});
        } else {
          if (ok && bb < a.B) {
            double* p = a.post + (size_t)bb * a.post_bstride + (long)t * a.post_tstride + a.post_off + 2 * s;
            if (st0) store_pol<NIPAMD_POST_NT>(p, px[i] * r[i]);
            if (st1) store_pol<NIPAMD_POST_NT>(p + 1, py[i] * r[i]);
          }
        }
      }
    }
  };
  // phase A copy: 16 * LPC pieces per step, 64 per store instruction
  // (filtering: the normalised alpha_t are the posteriors, nip.c:1103-1315)
  auto drainA = [&](int ci) {
    if (NIPAMD_MW_ABLATE == 1) return;
    const double* slot = out + (ci & 1) * G::kSlot;
    if (FWD && !AN) ll_chunk(ci, nA, tA);
    if constexpr (FILT) {
      if (!PVEC && !a.post) return;
      v2d ones[kWSeq];
#pragma unroll
      for (int q = 0; q < kWSeq; q++) ones[q] = v2d{1.0, 1.0};
      emit(slot, hi, ci * CH + hi, ci * CH + hi < nA, ones);
      return;
    }
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const int i = ci * CH + k;
      if (i >= nA) break;
      const int t = tA + dir * i;
#pragma unroll
      for (int u0 = 0; u0 < kWSeq * LPC; u0 += 64) {
        const int u = u0 + lane, jj = u / LPC, p = u % LPC;
        const v2d v = *reinterpret_cast<const v2d*>(slot + k * G::kStep + G::piece_off(jj, p));
        store_pol<NIPAMD_WIDE_SCR_NT>(reinterpret_cast<v2d*>(Sblk + (long)t * G::kStep + 2 * u), v);
      }
      if (AN && lane < kWSeq) Eblk[(long)t * kWSeq + lane] = er[((ci & 1) * CH + k) * kWSeq + lane];
    }
  };
  for (int ci = 0; ci < nchA; ci++) {
    if (ci > 0) drainA(ci - 1);
    barrier_lds(&dg);
  }
  if (nchA > 0) drainA(nchA - 1);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  dg.phase();

  if constexpr (FILT) {
    if (FWD) ll.write(a, b0, lane);
    return;
  }
  v2d oa[kWSeq];
  int eo[kWSeq];                                 // AN: the other direction's exponents
  auto load_other = [&](v2d (&o)[kWSeq], int ci) {
    if (NIPAMD_MW_ABLATE == 1) return;
    const double* q = Sblk + (long)(tlow(ci) + hi) * G::kStep + 2 * s;
#pragma unroll
    for (int c = 0; c < kWSeq; c++) o[c] = load_pol<NIPAMD_SCR_NTLD>(reinterpret_cast<const v2d*>(q + c * NP));
    if (AN) {
      const int* qe = Eblk + (long)(tlow(ci) + hi) * kWSeq;
#pragma unroll
      for (int c = 0; c < kWSeq; c++) eo[c] = qe[c];
    }
  };
  // AN: this ring step's posteriors, 2^(E* - Ef_t - Eb_t) / c* per chain
  auto emit_an = [&](const double* slot, const int* es, int kk, int t, bool ok, const v2d (&o)[kWSeq]) {
#pragma unroll
    for (int q = 0; q < kWSeq; q++) {
      const v2d v = *reinterpret_cast<const v2d*>(slot + kk * G::kStep + G::piece_off(q, s));
      const v2d z = *reinterpret_cast<const v2d*>(cz + 2 * q);
      const double f = __builtin_ldexp(z.x, (int)z.y - es[kk * kWSeq + q] - eo[q]);
      const double px = v.x * o[q].x * f, py = v.y * o[q].y * f;
      const long bb = b0 + q;
      if constexpr (PVEC) {
        double* p = (ok && bb < a.B) ? a.post + (size_t)bb * a.post_bstride + (long)t * NP + a.post_off + 2 * s : sink;
        store_pol<NIPAMD_POST_NT>(reinterpret_cast<v2d*>(p), v2d{px, py});
      } else {
        if (ok && bb < a.B) {
          double* p = a.post + (size_t)bb * a.post_bstride + (long)t * a.post_tstride + a.post_off + 2 * s;
          if (st0) store_pol<NIPAMD_POST_NT>(p, px);
          if (st1) store_pol<NIPAMD_POST_NT>(p + 1, py);
        }
      }
    }
  };
  const int nBf = T - H;                         // the forward side's phase-B steps (from t = H)
  auto drainB = [&](int ci, const v2d (&o)[kWSeq]) {
    if (NIPAMD_MW_ABLATE == 1) return;
    if (!AN && FWD == ((ci & 1) == 0) && ci * CH < nBf) ll_chunk(ci, nBf, H);
    if (!PVEC && !a.post) return;
    const double* slot = out + (ci & 1) * G::kSlot;
    const int nk = nB - ci * CH < CH ? nB - ci * CH : CH;
    if constexpr (AN) {
      const int* es = er + (ci & 1) * CH * kWSeq;
      if (ci == 0) {
        // c* and E* of the 16 chains at this partner's first step (ring index 0:
        // forward lanes hi = 0, backward hi = CH - 1)
#pragma unroll
        for (int q0 = 0; q0 < kWSeq; q0 += 8) {
          double z[8];
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const v2d v = *reinterpret_cast<const v2d*>(slot + kB * G::kStep + G::piece_off(q0 + i, s));
            z[i] = v.x * o[q0 + i].x + v.y * o[q0 + i].y;
          }
          sumL_n<LPC>(z);
          double r[8];
          recip_n(z, r);
          if (kB == 0 && s == 0) {
#pragma unroll
            for (int i = 0; i < 8; i++)
              *reinterpret_cast<v2d*>(cz + 2 * (q0 + i)) = v2d{r[i], (double)(es[q0 + i] + eo[q0 + i])};
          }
        }
      }
      emit_an(slot, es, kB, tlow(ci) + hi, kB < nk, o);
    } else {
      emit(slot, kB, tlow(ci) + hi, kB < nk, o);
    }
  };
  // one buffer (two groups' partners share the register file with the
  // filters): the next chunk's vectors are requested as soon as this chunk's
  // posteriors have used them, a chunk of latency ahead
  const int last = nchB > 0 ? nchB - 1 : 0;
  load_other(oa, 0);
  for (int ci = 0; ci < nchB; ci++) {
    barrier_lds(&dg);
    drainB(ci, oa);
    load_other(oa, ci + 1 < last ? ci + 1 : last);
  }
  // the forward side has nchB chunks when T - H > H (odd T): the last one is
  // the forward partner's or the backward partner's by its parity like the rest
  dg.write(a.diag, b0 / kWSeq, FWD ? 2 : 3, lane);
  // the forward ring slot the last chunk did not use (its readers passed the last loop barrier)
  double* share = const_cast<double*>(fring) + ((((nchB > 0 ? nchB : 1) - 1) & 1) ^ 1) * G::kSlot;
  if (!AN && !FWD) ll.put(share, lane);
  barrier_lds();                                 // the block's closing barrier
  if (!AN && FWD) {
    ll.take(share, lane);
    ll.write(a, b0, lane);
  }
}

// FILT: forward_inference (filtering only): per group one filter wave and one
// partner wave (waves 0, 1 the groups' filters, 2, 3 their partners), H = T
#ifndef NIPAMD_WIDE_PRIO
#define NIPAMD_WIDE_PRIO 0
#endif
template <int NT, bool FILT, int NC>
__global__ __launch_bounds__(FILT ? kWThreads / 2 : kWThreads, 1)
void chain_mfma_wide_kernel(WideMfmaArgs a) {
  constexpr int kThreads = FILT ? kWThreads / 2 : kWThreads;
  constexpr int F = FILT ? 1 : 2;                           // filter waves per group
  using G = Geo<NT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool filter = wave < kWGroups * F;
  const int role = filter ? wave : wave - kWGroups * F;
  const int grp = role / F;
  const bool fwd = FILT || (role % F) == 0;
  constexpr bool AN = !FILT && NIPAMD_MW_ANALYTIC;
  double* out = reinterpret_cast<double*>(smem) + grp * 4 * G::kSlot;   // this group's [2 dirs][2 slots][kSlot]
  double* zr = reinterpret_cast<double*>(smem) + kWGroups * 4 * G::kSlot + grp * 2 * G::CH * kWSeq;
  // AN: the same area as the group's exponent rings [2 dirs][2 slots][CH][16] ints
  int* er = reinterpret_cast<int*>(zr) + (fwd ? 0 : 2 * G::CH * kWSeq);
  double* tab = reinterpret_cast<double*>(smem) + kWGroups * (4 * G::kSlot + 2 * G::CH * kWSeq);
  // AN: per partner (1/c*, E*) of its 16 chains, after the tables
  double* cz = tab + a.tab_rows * G::NPS + (grp * 2 + (fwd ? 0 : 1)) * 2 * kWSeq;
  const int ncol = a.ncol > 0 ? a.ncol : 1;
  const int j = lane & 15, g = lane >> 4;
  const long b0 = (long)blockIdx.x * (kWGroups * kWSeq) + grp * kWSeq;
  const int T = a.T;

  for (int i = tid; i < a.tab_rows * G::NP; i += kThreads) tab[(i / G::NP) * G::NPS + i % G::NP] = a.tab[i];
  __syncthreads();

  const int H = a.H;
  const int nA = (H > T - 1 - H ? H : T - 1 - H), nB = (T - H > H ? T - H : H);
  const int nchA = (nA + G::CH - 1) / G::CH, nchB = FILT ? 0 : (nB + G::CH - 1) / G::CH;
  double* ring = out + (fwd ? 0 : 2 * G::kSlot);
  double* Sblk = FILT ? nullptr : a.S + (size_t)(b0 / kWSeq) * wblock_scratch(NT, T) + (size_t)kWG * G::kStep;
  // AN: the phase-A messages' exponents [T + 2G][16] per group, after every group's messages and the sink group
  int* Eblk = FILT ? nullptr
                   : reinterpret_cast<int*>(a.S + (size_t)((a.B + kWSeq - 1) / kWSeq + 1) * wblock_scratch(NT, T)) +
                         (size_t)(b0 / kWSeq) * wblock_exps(T) + (size_t)kWG * kWSeq;
  // A/B builds: static wave priority for the partners (1) or the filters (2)
  if ((NIPAMD_WIDE_PRIO == 1 && !filter) || (NIPAMD_WIDE_PRIO == 2 && filter)) __builtin_amdgcn_s_setprio(1);
  if (!filter) {
    const bool pvec = a.post && a.N == G::NP && a.post_tstride == G::NP && (a.post_off & 1) == 0 &&
                      (a.post_bstride & 1) == 0 && (reinterpret_cast<uintptr_t>(a.post) & 15) == 0;
    if (pvec) {
      if (fwd) wpartner<true, true, NT, FILT, AN>(a, ring, out, zr, Sblk, lane, b0, nchA, nchB, er, Eblk, cz);
      else wpartner<false, true, NT, FILT, AN>(a, ring, out, zr, Sblk, lane, b0, nchA, nchB, er, Eblk, cz);
    } else {
      if (fwd) wpartner<true, false, NT, FILT, AN>(a, ring, out, zr, Sblk, lane, b0, nchA, nchB, er, Eblk, cz);
      else wpartner<false, false, NT, FILT, AN>(a, ring, out, zr, Sblk, lane, b0, nchA, nchB, er, Eblk, cz);
    }
    return;
  }
  WCtx c;
  c.tab = tab;
  c.obs = (a.ncol > 0 && b0 + j < a.B) ? a.obs + (b0 + j) * a.obs_bstride : nullptr;
  c.ots = a.obs_tstride;
  c.T = T;
  c.ncol = ncol;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    c.col[k] = a.col[k];
    c.M[k] = a.ncol > 0 ? a.M[k] : 0;              // no observed column: row 0 (the row sums) every step
    c.tab_off[k] = (k < ncol ? a.tab_off[k] / G::NP * G::NPS : 0) + 2 * g;
  }
  c.out = ring;
  c.zr = zr;
  c.er = er;
  c.zw = g == 0;
  c.j = j;
#pragma unroll
  for (int q = 0; q < NT; q++) {
    c.wo[q][0] = Geo<NT>::piece_off(j, 8 * q + g);
    c.wo[q][1] = Geo<NT>::piece_off(j, 8 * q + 4 + g);
  }
  if (fwd) wfilter<true, NT, NC, AN>(a, c, Sblk, Eblk, lane, b0, nchA, nchB);
  else if (!FILT) wfilter<false, NT, NC, AN>(a, c, Sblk, Eblk, lane, b0, nchA, nchB);
  if (!FILT) barrier_lds();                       // the block's closing barrier (wpartner)
}

}  // namespace

size_t chain_mfma_wide_lds_bytes(int NT, int tab_rows, int ncol, int T) {
  (void)ncol; (void)T;                                       // codes are read from HBM
  const size_t slot = 2048;                                  // doubles per ring slot
  const size_t ch = 8 / NT;
  return (kWGroups * (4 * slot + 2 * ch * kWSeq) + (size_t)tab_rows * (16 * NT + 2) +
          kWGroups * 2 * 2 * kWSeq) * sizeof(double);        // + the partners' (1/c*, E*)
}

size_t chain_mfma_wide_scratch_bytes(int NT, long B, int T) {
  const long groups = (B + kWSeq - 1) / kWSeq + 1;
  return (size_t)groups * wblock_scratch(NT, T) * sizeof(double) + (size_t)groups * wblock_exps(T) * sizeof(int);
}

namespace {
template <int NT, bool FILT, int NC>
int launch_wide_nc(const WideMfmaArgs& a, size_t lds, hipStream_t stream) {
  static size_t set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_mfma_wide_kernel<NT, FILT, NC>), lds, set)) return rc;
  const int blocks = (int)((a.B + kWGroups * kWSeq - 1) / (kWGroups * kWSeq));
  hipLaunchKernelGGL((chain_mfma_wide_kernel<NT, FILT, NC>), dim3(blocks), dim3(FILT ? kWThreads / 2 : kWThreads),
                     lds, stream, a);
  g_last_kernel = NT == 1 ? "chain_mfma_wide_kernel<1>" : "chain_mfma_wide_kernel<2>";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <int NT, bool FILT>
int launch_wide(const WideMfmaArgs& a, size_t lds, hipStream_t stream) {
  switch (a.ncol > 1 ? a.ncol : 1) {
    case 1: return launch_wide_nc<NT, FILT, 1>(a, lds, stream);
    case 2: return launch_wide_nc<NT, FILT, 2>(a, lds, stream);
    case 3: return launch_wide_nc<NT, FILT, 3>(a, lds, stream);
    default: return launch_wide_nc<NT, FILT, 4>(a, lds, stream);
  }
}
}  // namespace

int chain_mfma_wide_launch(const WideMfmaArgs& a, int NT, bool filter_only, hipStream_t stream) {
  const size_t lds = (chain_mfma_wide_lds_bytes(NT, a.tab_rows, a.ncol, a.T) + 15) & ~(size_t)15;
  if (lds > 160 * 1024 || (filter_only && a.H != a.T)) return kLaunchRefused;
  if (NT == 1) return filter_only ? launch_wide<1, true>(a, lds, stream) : launch_wide<1, false>(a, lds, stream);
  return filter_only ? launch_wide<2, true>(a, lds, stream) : launch_wide<2, false>(a, lds, stream);
}

}  // namespace nipamd
