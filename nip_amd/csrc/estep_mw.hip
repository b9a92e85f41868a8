// estep_mw.hip -- fused e_step of interface chains of 17..32 states on the
// matrix cores (round 5; SURVEY 8(d) config 3's model, demo1 @ 32 states).
//
// The reference's e_step (src/nip.c:1708-2007, families :1925-1967) sums per
// sequence and step the family marginals of every variable.  For an interface
// chain they follow from three sums (estep_wide.hip):
//   K(x, y) = sum_t alpha_{t-1}(x) e_t(y) beta_t(y) / Z   (alpha_{-1} = prior)
//   H[r][y] = sum_t [r = row of child k's code at t] gamma_t(y)
//   P0(x)   = gamma_{-1}(x) = prior(x) beta_{-1}(x) / Z
// The round-4 route stored every message (chain_msgs_kernel) and read them
// back (chain_stats_kernel): 1056 B per sequence-step.  Here the block is the
// fb kernel's (chain_mfma_wide.hip): two groups of 16 sequences, per group a
// matrix-core filter wave and a partner wave per direction, so every SIMD runs
// one filter and one partner.  Phase A is the fb's (the partners copy the
// first half of each direction's messages to HBM scratch); in phase B each
// partner forms its half of the steps' three sums on the matrix cores from
// its own direction's LDS ring and the other direction's scratch rows, and
// nothing but one slab row per 16 sequences leaves the chip: 16 B of codes
// and 512 B of scratch round trip per sequence-step at 32 states.
//
// Scales.  Both filters rescale by exact powers of two and publish each
// message's accumulated exponent (alpha^_t = alpha_t 2^Ef_t, beta^_t =
// beta_t 2^Eb_t), so c_t = sum_y alpha^_t beta^_t = Z 2^(Ef_t + Eb_t) for
// every t: one sum per sequence (c*, at the partner's first phase-B step,
// exponent E*) normalises every step,
//   gamma_t = alpha^_t o beta^_t 2^(E* - Ef_t - Eb_t) / c*
//   w_t     = e_t o beta^_t 2^(E* - Ef_{t-1} - Eb_t) / c*   (paired with alpha^_{t-1})
// -- the 16-state e_step's analytic normalisation (chain_estep16_kernel).
//
// Phase-B split: the forward partner takes t = H..T-1 (gamma_t; xi_t for
// t > H, alpha^_{t-1} from its ring), the backward partner t = H-1..-1
// (gamma_t, or P0 at t = -1; xi_{t+1} with alpha^_t from the scratch and
// beta^_{t+1} from its ring) -- the backward filter runs one extra step to
// beta^_{-1}.  A ring slot holds the chunk's CH steps after a copy of the
// previous chunk's last message (row 0), so both neighbours of every step are
// in the slot the partner reads.
//
// The sums on the matrix cores (v_mfma_f64_16x16x4, K = 4 (sequence, step)
// pairs: lane l = (s, hi, c2) holds states 2s, 2s+1 of chain 2 qp + c2 at the
// chunk's step hi; the even / odd states are the two 16-wide tiles):
//   K tiles (xt, yt) += alpha^ (x) w       (4 MFMAs per pass)
//   H tiles (mt, yt) += onehot(code) (x) gamma over the observed children's
//                       in-range codes, concatenated as virtual rows (<= 64)
// and the rare rows on the VALU: a column's missing row (a wave-uniform branch
// taken only when some pair is missing), the unobserved children's missing
// rows (every step's gamma), P0.  Fixed-order sums throughout: the two
// partners' sums meet in LDS and the forward partner writes the group's slab
// row, which tree64_kernel reduces like every e_step slab (shard invariance
// for whole 16-sequence groups).
//
// The ll (nip.c:1458-1474) is the forward filter's: m2_t = z2_t, m1_t =
// 2^sc_t (alpha^_{t-1} . A s), as chain_mfma_wide.hip's partners keep it.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <cstdint>

#include "chain_kernels.h"
#include "store_pol.h"

namespace nipamd {

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

constexpr int kSeq = 16;               // sequences (chains) per group
constexpr int kGroups = 2;             // groups per block
constexpr int kThreads = 512;
constexpr int NT = 2, NP = 32;         // state tiles, states per chain row
constexpr int CH = 2;                  // steps per chunk (one block barrier each)
constexpr int kRows = CH + 1;          // ring rows per slot: the previous chunk's last message, then the chunk
constexpr int kStep = kSeq * NP;       // doubles per ring row (16 chains)
constexpr int kSlot = kRows * kStep;
constexpr int NPS = NP + 2;            // LDS table row stride (doubles): rows start 4 banks apart
constexpr int kG = kScratchGuard;
constexpr int kMaxMT = 4;              // matrix-core count-row tiles: sum of the observed children's M <= 64
constexpr int kPass = kSeq / 2;
constexpr int kMaxCols = 2;            // evidence columns the kernel takes        // partner passes per chunk: two chains x CH steps x 16 lanes each

__host__ __device__ constexpr int state_of(int g, int r) { return r < 2 ? 2 * g + r : 6 + 2 * g + r; }
// chain j's piece p (states 2p, 2p + 1) within a ring row, XOR-swizzled by j & 7
__device__ __forceinline__ int piece_off(int j, int p) { return j * NP + ((p ^ (j & 7)) << 1); }

__device__ __forceinline__ double swap32_sum(double x) {     // x[l] + x[l ^ 32]
  double xc = x;
  asm("" : "+v"(xc));
  const auto rl = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
__device__ __forceinline__ double swap16_sum(double x) {     // x[l] + x[l ^ 16]
  double xc = x;
  asm("" : "+v"(xc));
  const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
// the four lanes l, l ^ 16, l ^ 32, l ^ 48 (a chain's lanes in the filter
// layout, a state pair's lanes in the partner layout): identical bits in all
__device__ __forceinline__ double quad_sum(double x) {
  asm("" : "+v"(x));        // one rounded value per lane: no fma contraction into the first add
  return swap16_sum(swap32_sum(x));
}
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// sum over the 16 lanes of a DPP row (identical bits in all of them)
__device__ __forceinline__ double row_sum16(double x) {
  asm("" : "+v"(x));
  x += dpp64<0xB1>(x);      // quad_perm [1,0,3,2]
  x += dpp64<0x4E>(x);      // quad_perm [2,3,0,1]
  x += dpp64<0x141>(x);     // row_half_mirror
  x += dpp64<0x140>(x);     // row_mirror
  return x;
}
__device__ __forceinline__ double recip(double c) {
  double r = __builtin_amdgcn_rcp(c);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  return c != 0.0 ? r : 0.0;
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
__device__ __forceinline__ v4d mfma(double a, double b, v4d d) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
}
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void barrier_phase() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// the block's LDS: rings [group][dir][2 slots][kRows][kStep], their exponents
// [group][dir][2][kRows][16], per partner (1/c*, E*) of its 16 chains, the
// backward partners' small sums [group][6][32], then the tables
constexpr int kRingD = kGroups * 2 * 2 * kSlot;
constexpr int kRowI = 5 * kSeq;       // ints per ring row: the 16 messages' exponents, then their raw codes [4][16]
constexpr int kExpI = kGroups * 2 * 2 * kRows * kRowI;
constexpr int kCzD = kGroups * 2 * kSeq * 2;
constexpr int kSmallD = kGroups * 6 * NP;
__host__ __device__ constexpr size_t lds_doubles(int tab_rows) {
  return (size_t)kRingD + kExpI / 2 + kCzD + kSmallD + (size_t)tab_rows * NPS;
}

// per-group HBM scratch: messages [T + 2G][16][NP] doubles, exponents [T + 2G][16] ints
__host__ __device__ inline long group_msgs(int T) { return (long)(T + 2 * kG) * kStep; }
__host__ __device__ inline long group_exps(int T) { return (long)(T + 2 * kG) * kSeq; }

struct FCtx {
  const double* tab;       // LDS tables
  const int* obs;          // this chain's observations (null: an absent sequence or no observed column)
  int ots;
  int col[4], M[4];
  int T;
  int tab_off[4];          // per column: LDS offset of its table + 2g
  double* ring;            // this direction's [2][kSlot]
  int* rexp;               // [2][kRows][kRowI]: exponents, raw codes
  int wo[NT][2];           // [tile][half] piece offsets of this lane
  int j, g;
};

// One direction's filter: the fb kernel's matrix-core recursion (see
// chain_mfma_wide.hip for the register algebra), every step's message and
// accumulated exponent into the ring, the previous chunk's last message in
// row 0 of each slot; the forward filter also keeps the ll.
template <bool FWD, int NC>
struct EFilter {
  double Aop[NT][NT][4];
  v4d X[NT];               // the next step's input: forward alpha^_{t-1}, backward e_{t+1} o beta^_{t+1}
  v4d U[NT];               // backward: beta^ of the last step (row 0 of the next slot)
  int sc = 0;              // the next step's rescale exponent
  int E = 0;               // the last message's accumulated exponent
  double m2 = 1.0, m1 = 1.0, zmin = 1.0;   // forward ll: mantissas and exponents of prod z2, prod m1
  int e2 = 0, e1 = 0;
  v4d wv[NT];              // this lane's states of w = A s_all
  int lastraw[NC];         // the last step's raw codes (row 0 of the next slot)

  __device__ __forceinline__ int raw(const FCtx& c, int k, int t) const {
    return (c.obs && t >= 0 && t < c.T) ? c.obs[(long)t * c.ots + c.col[k]] : -1;
  }
  __device__ __forceinline__ int code(const FCtx& c, int k, int o) const {
    return o < 0 ? c.M[k] : (o < c.M[k] ? o : c.M[k] + 1);
  }
  __device__ __forceinline__ void rows_of(const FCtx& c, const int (&cd)[NC], v4d (&r)[NC][NT]) const {
#pragma unroll
    for (int k = 0; k < NC; k++)
#pragma unroll
      for (int q = 0; q < NT; q++) r[k][q] = load4(c.tab + c.tab_off[k] + cd[k] * NPS + 16 * q);
  }
  __device__ __forceinline__ void product(const v4d (&r)[NC][NT], v4d (&e)[NT]) const {
#pragma unroll
    for (int q = 0; q < NT; q++) e[q] = r[0][q];
#pragma unroll
    for (int k = 1; k < NC; k++)
#pragma unroll
      for (int q = 0; q < NT; q++) e[q] *= r[k][q];
  }
  __device__ __forceinline__ void matvec(v4d (&d)[NT]) {
#pragma unroll
    for (int qo = 0; qo < NT; qo++) d[qo] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int qi = 0; qi < NT; qi++) {
      d[0] = mfma(Aop[0][qi][0], X[qi].x, d[0]);
      d[NT - 1] = mfma(Aop[NT - 1][qi][0], X[qi].x, d[NT - 1]);
      d[0] = mfma(Aop[0][qi][1], X[qi].y, d[0]);
      d[NT - 1] = mfma(Aop[NT - 1][qi][1], X[qi].y, d[NT - 1]);
      d[0] = mfma(Aop[0][qi][2], X[qi].z, d[0]);
      d[NT - 1] = mfma(Aop[NT - 1][qi][2], X[qi].z, d[NT - 1]);
      d[0] = mfma(Aop[0][qi][3], X[qi].w, d[0]);
      d[NT - 1] = mfma(Aop[NT - 1][qi][3], X[qi].w, d[NT - 1]);
    }
  }
  __device__ __forceinline__ void renorm() {
    const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
    const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
  }
  // one step into ring row L (exponent and code row Le); last: t = T - 1 (forward ll)
  __device__ __forceinline__ void step(const FCtx& c, double* L, int* Le, const int (&raw)[NC], const v4d (&r)[NC][NT],
                                       bool last) {
    v4d d[NT];
    matvec(d);
    v4d e[NT];
    product(r, e);
    E += sc;
    double part = 0.0, py = 0.0;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      const v4d u = ldexp4(d[q], sc);
      const v4d p = u * e[q];
      const v4d keep = FWD ? p : u;
      *reinterpret_cast<v2d*>(L + c.wo[q][0]) = v2d{keep.x, keep.y};
      *reinterpret_cast<v2d*>(L + c.wo[q][1]) = v2d{keep.z, keep.w};
      part += (p.x + p.y) + (p.z + p.w);
      if (FWD) {
        py += (p.x * wv[q].x + p.y * wv[q].y) + (p.z * wv[q].z + p.w * wv[q].w);
      } else {
        U[q] = u;
      }
      X[q] = p;
    }
    if (c.g == 0) {
      Le[c.j] = E;
#pragma unroll
      for (int k = 0; k < NC; k++) { Le[(1 + k) * kSeq + c.j] = raw[k]; lastraw[k] = raw[k]; }
    }
    const double z2 = quad_sum(part);
    const int k = __builtin_amdgcn_frexp_exp(z2);
    if (FWD) {
      // m2_t = z2_t; m1_{t+1} = 2^sc_{t+1} y_t, y_t = alpha^_t . w (nip.c:1458-1474)
      const double y = quad_sum(py);
      zmin = __builtin_fmin(zmin, z2);
      m2 *= z2;
      if (!last) { m1 *= y; e1 -= k; }
      renorm();
    }
    sc = z2 != 0.0 ? -k : 0;
  }
  // n steps from t0 (forward up, backward down) in nch chunks; the codes of
  // chunk ci + 2 are loaded when chunk ci ends, a step's table rows from LDS
  // at its start (under its MFMAs)
  __device__ __forceinline__ void run(const FCtx& c, int n, int nch, int t0) {
    constexpr int dir = FWD ? 1 : -1;
    int ca[CH][NC], cb[CH][NC];
    auto ldc = [&](int ci, int (&cc)[CH][NC]) {
#pragma unroll
      for (int k = 0; k < CH; k++)
#pragma unroll
        for (int q = 0; q < NC; q++) cc[k][q] = raw(c, q, t0 + dir * (ci * CH + k));
    };
    auto chunk = [&](int ci, int (&cc)[CH][NC]) {
      double* slot = c.ring + (ci & 1) * kSlot;
      int* es = c.rexp + (ci & 1) * kRows * kRowI;
      // row 0: the previous step's message, exponent and codes (the slot's
      // readers passed the barrier that ended the chunk before last)
#pragma unroll
      for (int q = 0; q < NT; q++) {
        const v4d keep = FWD ? X[q] : U[q];
        *reinterpret_cast<v2d*>(slot + c.wo[q][0]) = v2d{keep.x, keep.y};
        *reinterpret_cast<v2d*>(slot + c.wo[q][1]) = v2d{keep.z, keep.w};
      }
      if (c.g == 0) {
        es[c.j] = E;
#pragma unroll
        for (int k = 0; k < NC; k++) es[(1 + k) * kSeq + c.j] = lastraw[k];
      }
      const int base = ci * CH;
#pragma unroll
      for (int k = 0; k < CH; k++) {
        if (base + k >= n) break;
        int cd[NC];
#pragma unroll
        for (int q = 0; q < NC; q++) cd[q] = code(c, q, cc[k][q]);
        v4d r[NC][NT];
        rows_of(c, cd, r);
        step(c, slot + (k + 1) * kStep, es + (k + 1) * kRowI, cc[k], r, t0 + dir * (base + k) == c.T - 1);
      }
      barrier_lds();
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

template <bool FWD, int NC>
__device__ __forceinline__ void efilter(const EMwArgs& a, const FCtx& c, int lane, long b0, int nchA, int nchB) {
  const int j = lane & 15, g = lane >> 4;
  const int T = a.T, H = a.H;
  EFilter<FWD, NC> f;
#pragma unroll
  for (int qo = 0; qo < NT; qo++)
#pragma unroll
    for (int qi = 0; qi < NT; qi++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int out = 16 * qo + state_of(j & 3, j >> 2), in = 16 * qi + state_of(g, r);
        f.Aop[qo][qi][r] = FWD ? a.A[in * 64 + out] : a.A[out * 64 + in];
      }
  if (FWD) {
    double py = 0.0;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      f.X[q] = load4(a.pi + 16 * q + 2 * g);
      f.wv[q] = load4(a.w + 16 * q + 2 * g);
      py += (f.X[q].x * f.wv[q].x + f.X[q].y * f.wv[q].y) + (f.X[q].z * f.wv[q].z + f.X[q].w * f.wv[q].w);
    }
    f.m1 = quad_sum(py);                   // y_{-1} = prior . w
#pragma unroll
    for (int q = 0; q < NC; q++) f.lastraw[q] = -1;
    f.renorm();
    f.run(c, H, nchA, 0);
    barrier_phase();
    f.run(c, T - H, nchB, H);
    if (g == 0 && b0 + j < a.B) {
      double ll = log(f.m2) - log(f.m1) + (double)(f.e2 - f.e1) * 0.69314718055994530942;
      const bool dead = f.zmin == 0.0;
      if (dead) ll = -DBL_MAX;
      if (a.ll) a.ll[b0 + j] = ll;
      // e_step's BAD_LUCK (m1 <= 0 || m2 <= 0, nip.c:1827-1854): a zero mass
      if (a.status) a.status[b0 + j] = dead ? 3u : 0u;
    }
  } else {
    // beta^_{T-1} = 1 (exponent 0), the input of the first step e_{T-1} o beta^_{T-1}
    int cd[NC];
#pragma unroll
    for (int q = 0; q < NC; q++) {
      f.lastraw[q] = f.raw(c, q, T - 1);
      cd[q] = f.code(c, q, f.lastraw[q]);
    }
    v4d r[NC][NT], e[NT];
    f.rows_of(c, cd, r);
    f.product(r, e);
    double part = 0.0;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      v4d beta;
      beta.x = 16 * q + state_of(g, 0) < a.N ? 1.0 : 0.0; beta.y = 16 * q + state_of(g, 1) < a.N ? 1.0 : 0.0;
      beta.z = 16 * q + state_of(g, 2) < a.N ? 1.0 : 0.0; beta.w = 16 * q + state_of(g, 3) < a.N ? 1.0 : 0.0;
      f.U[q] = beta;
      f.X[q] = e[q] * beta;
      part += (f.X[q].x + f.X[q].y) + (f.X[q].z + f.X[q].w);
    }
    const double z = quad_sum(part);
    f.sc = z != 0.0 ? -__builtin_amdgcn_frexp_exp(z) : 0;
    f.run(c, T - 1 - H, nchA, T - 2);
    barrier_phase();
    f.run(c, H + 1, nchB, H - 1);          // down to beta^_{-1}
  }
  barrier_lds();                            // the block's closing barrier (epartner)
}

// A partner wave's matrix-core sums over its half of the steps.
template <int NC>
struct Acc {
  v4d K[2][2];             // [xt][yt]: K(2i + xt, 2j + yt)
  v4d Hc[kMaxMT][2];       // [mt][yt]: H(virtual row 16 mt + i, 2j + yt)
  v2d hm[NC];              // per column: its missing row (this lane's pairs)
  v2d gt;                  // every step's gamma (the unobserved children's missing rows)
  v2d p0;                  // gamma_{-1} (backward partner)
};

// Partner wave of one direction and group (module comment).
template <bool FWD, int NC>
__device__ __forceinline__ void epartner(const EMwArgs& a, double* ring, int* rexp, double* cz, double* small,
                                         const double* tab, double* Sblk, int* Eblk, int lane, long b0,
                                         int nchA, int nchB) {
  const int T = a.T, H = a.H;
  const int nA = FWD ? H : T - 1 - H;
  // ---- phase A: the first half of this direction's messages to the scratch
  if (FWD) {
    // alpha^_{-1} = the prior (exponent 0), read by the backward partner at t = -1
    for (int u = lane; u < kSeq * NP / 2; u += 64) {
      const int p = u & 15;
      *reinterpret_cast<v2d*>(Sblk - kStep + 2 * u) = v2d{a.pi[2 * p], a.pi[2 * p + 1]};
    }
    if (lane < kSeq) Eblk[-kSeq + lane] = 0;
  } else {
    // beta^_{T-1} = 1 (exponent 0)
    for (int u = lane; u < kSeq * NP / 2; u += 64) {
      const int p = u & 15;
      *reinterpret_cast<v2d*>(Sblk + (long)(T - 1) * kStep + 2 * u) =
          v2d{2 * p < a.N ? 1.0 : 0.0, 2 * p + 1 < a.N ? 1.0 : 0.0};
    }
    if (lane < kSeq) Eblk[(long)(T - 1) * kSeq + lane] = 0;
  }
  auto drainA = [&](int ci) {
    const double* slot = ring + (ci & 1) * kSlot;
    const int* es = rexp + (ci & 1) * kRows * kRowI;
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const int i = ci * CH + k;
      if (i >= nA) break;
      const long t = FWD ? i : T - 2 - i;
#pragma unroll
      for (int u0 = 0; u0 < kSeq * NP / 2; u0 += 64) {
        const int u = u0 + lane, jj = u >> 4, p = u & 15;
        const v2d v = *reinterpret_cast<const v2d*>(slot + (k + 1) * kStep + piece_off(jj, p));
        store_pol<NIPAMD_WIDE_SCR_NT>(reinterpret_cast<v2d*>(Sblk + t * kStep + 2 * u), v);
      }
      if (lane < kSeq) Eblk[t * kSeq + lane] = es[(k + 1) * kRowI + lane];
    }
  };
  for (int ci = 0; ci < nchA; ci++) {
    if (ci > 0) drainA(ci - 1);
    barrier_lds();
  }
  if (nchA > 0) drainA(nchA - 1);
  barrier_phase();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");

  // ---- phase B
  const int s = lane & 15, k4 = lane >> 4, hi = k4 & 1, c2 = k4 >> 1;
  const int nB = FWD ? T - H : H + 1;
  Acc<NC> acc;
#pragma unroll
  for (int xt = 0; xt < 2; xt++)
#pragma unroll
    for (int yt = 0; yt < 2; yt++) acc.K[xt][yt] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int mt = 0; mt < kMaxMT; mt++) acc.Hc[mt][0] = acc.Hc[mt][1] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < NC; c++) acc.hm[c] = v2d{0.0, 0.0};
  acc.gt = acc.p0 = v2d{0.0, 0.0};
  int mtn = 0;                                       // count-row tiles in use
#pragma unroll
  for (int c = 0; c < NC; c++)
    if (c < a.ncol) mtn = max(mtn, (a.voff[c] + a.M[c] + 15) >> 4);
  const bool unobs = a.n_unobs > 0;

  // the other direction's vectors (scratch) and exponents one chunk ahead:
  // forward t = H + i, backward t = H - 1 - i; the codes come from the ring's
  // rows (the filters publish them)
  struct Pre {
    v2d o[kPass];
    int eo[kPass];
  };
  auto tstep = [&](int ci) { const int i = ci * CH + hi; return FWD ? H + i : H - 1 - i; };
  auto load = [&](int ci, Pre& P) {
    const int t = tstep(ci);
    const int tc = t < -1 ? -1 : (t > T - 1 ? T - 1 : t);
#pragma unroll
    for (int qp = 0; qp < kPass; qp++) {
      const int j = 2 * qp + c2;
      P.o[qp] = *reinterpret_cast<const v2d*>(Sblk + (long)tc * kStep + j * NP + 2 * s);
      P.eo[qp] = Eblk[(long)tc * kSeq + j];
    }
  };
  auto ev_row = [&](int c, int o) {                  // this lane's two states of column c's row for raw code o
    const int M = a.ncol > 0 ? a.M[c] : 0;
    const int r = o < 0 ? M : (o < M ? o : M + 1);
    return *reinterpret_cast<const v2d*>(tab + a.tab_off[c] / NP * NPS + r * NPS + 2 * s);
  };

  Pre P;
  load(0, P);
  for (int ci = 0; ci < nchB; ci++) {
    barrier_lds();
    const double* slot = ring + (ci & 1) * kSlot;
    const int* es = rexp + (ci & 1) * kRows * kRowI;
    const int i = ci * CH + hi, t = tstep(ci);
    const bool valid = i < nB;
    if (ci == 0) {
      // c* and E* of the 16 chains at this partner's first step (i = 0)
#pragma unroll
      for (int qp = 0; qp < kPass; qp++) {
        const int j = 2 * qp + c2;
        const v2d m = *reinterpret_cast<const v2d*>(slot + kStep + piece_off(j, s));
        const double cs = row_sum16(m.x * P.o[qp].x + m.y * P.o[qp].y);
        if (hi == 0 && s == 0) {
          const bool live = b0 + j < a.B;
          cz[2 * j] = live ? recip(cs) : 0.0;
          cz[2 * j + 1] = (double)(es[kRowI + j] + P.eo[qp]);
        }
      }
    }
#pragma unroll
    for (int qp = 0; qp < kPass; qp++) {
      const int j = 2 * qp + c2;
      const bool live = valid && b0 + j < a.B;
      const v2d mc = *reinterpret_cast<const v2d*>(slot + (hi + 1) * kStep + piece_off(j, s));
      const v2d ma = *reinterpret_cast<const v2d*>(slot + hi * kStep + piece_off(j, s));
      const int Ec = es[(hi + 1) * kRowI + j], Ea = es[hi * kRowI + j];
      // raw codes at this step (row hi + 1) and at its neighbour (row hi:
      // backward, t + 1, whose evidence w takes)
      int cd[NC], ce[NC];
#pragma unroll
      for (int c = 0; c < NC; c++) {
        cd[c] = es[(hi + 1) * kRowI + (1 + c) * kSeq + j];
        ce[c] = es[hi * kRowI + (1 + c) * kSeq + j];
      }
      const v2d z = *reinterpret_cast<const v2d*>(cz + 2 * j);
      const int Es = (int)z.y;
      const v2d o = P.o[qp];
      const int Eo = P.eo[qp];
      // the step's evidence (forward: at t; backward: at t + 1)
      v2d ev = ev_row(0, FWD ? cd[0] : ce[0]);
#pragma unroll
      for (int c = 1; c < NC; c++) ev *= ev_row(c, FWD ? cd[c] : ce[c]);
      v2d g, w, xa;
      if (FWD) {
        // alpha^_t = mc, alpha^_{t-1} = ma, beta^_t = o
        const double fg = __builtin_ldexp(z.x, Es - Ec - Eo);
        const double fw = t == H ? 0.0 : __builtin_ldexp(z.x, Es - Ea - Eo);   // xi_H is the backward side's
        g = mc * o * fg;
        w = ev * o * fw;
        xa = ma;
      } else {
        // beta^_t = mc, beta^_{t+1} = ma, alpha^_t = o
        const double fg = __builtin_ldexp(z.x, Es - Eo - Ec);
        const double fw = __builtin_ldexp(z.x, Es - Eo - Ea);
        g = o * mc * fg;
        w = ev * ma * fw;
        xa = o;
      }
      // (a step past this direction's last, or an absent sequence: its ring
      // rows may be stale, even never written -- nothing of it may reach a sum)
      if (!live) { g = v2d{0.0, 0.0}; w = v2d{0.0, 0.0}; xa = v2d{0.0, 0.0}; }
      // (no divergent control flow around the MFMAs: they ignore EXEC)
      acc.K[0][0] = mfma(xa.x, w.x, acc.K[0][0]);
      acc.K[0][1] = mfma(xa.x, w.y, acc.K[0][1]);
      acc.K[1][0] = mfma(xa.y, w.x, acc.K[1][0]);
      acc.K[1][1] = mfma(xa.y, w.y, acc.K[1][1]);
      const bool pz = !FWD && t < 0;                 // gamma_{-1}: P0, no count rows
      if (pz) acc.p0 += g;
      const bool cnt = live && !pz;
      // H: the in-range codes' virtual rows on the matrix cores
      int vr[NC];
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const int o = cd[c];
        vr[c] = (cnt && a.ncol > 0 && o >= 0 && o < a.M[c]) ? a.voff[c] + o : -1;
      }
#pragma unroll
      for (int mt = 0; mt < kMaxMT; mt++) {
        if (mt >= mtn) break;
        bool hit = false;
#pragma unroll
        for (int c = 0; c < NC; c++) hit |= vr[c] == 16 * mt + s;
        const double oh = hit ? 1.0 : 0.0;
        acc.Hc[mt][0] = mfma(oh, g.x, acc.Hc[mt][0]);
        acc.Hc[mt][1] = mfma(oh, g.y, acc.Hc[mt][1]);
      }
      // the observed columns' missing rows: only when some pair of the pass misses
      bool miss = false;
#pragma unroll
      for (int c = 0; c < NC; c++) miss |= cnt && a.ncol > 0 && cd[c] < 0;
      if (__builtin_amdgcn_ballot_w64(miss)) {
#pragma unroll
        for (int c = 0; c < NC; c++)
          if (cnt && a.ncol > 0 && cd[c] < 0) acc.hm[c] += g;
      }
      if (unobs && cnt) acc.gt += g;
    }
    if (ci + 1 < nchB) load(ci + 1, P);
  }

  // ---- the two partners' sums: the backward partner's into LDS (its own
  // ring, which only it reads), the forward partner adds them and writes the
  // group's slab row
  v2d sm[6];                                         // hm[0..3], gt, p0 summed over the lane's 4 pairs
#pragma unroll
  for (int c = 0; c < 4; c++) sm[c] = c < NC ? acc.hm[c < NC ? c : 0] : v2d{0.0, 0.0};
  sm[4] = acc.gt;
  sm[5] = acc.p0;
#pragma unroll
  for (int f = 0; f < 6; f++) { sm[f].x = quad_sum(sm[f].x); sm[f].y = quad_sum(sm[f].y); }
  double* kb = ring;                                 // backward partner's tiles: [tile][r][64 lanes]
  if (!FWD) {
#pragma unroll
    for (int xt = 0; xt < 2; xt++)
#pragma unroll
      for (int yt = 0; yt < 2; yt++)
#pragma unroll
        for (int r = 0; r < 4; r++) kb[((xt * 2 + yt) * 4 + r) * 64 + lane] = acc.K[xt][yt][r];
#pragma unroll
    for (int mt = 0; mt < kMaxMT; mt++)
#pragma unroll
      for (int yt = 0; yt < 2; yt++)
#pragma unroll
        for (int r = 0; r < 4; r++) kb[((4 + mt * 2 + yt) * 4 + r) * 64 + lane] = acc.Hc[mt][yt][r];
    if (k4 == 0) {
#pragma unroll
      for (int f = 0; f < 6; f++) *reinterpret_cast<v2d*>(small + f * NP + 2 * s) = sm[f];
    }
  }
  barrier_lds();                                     // the block's closing barrier
  if (!FWD || b0 >= a.B) return;
  // the backward partner's tiles: its ring in the LDS, right after this one's
  const double* ob = ring + 2 * kSlot;
  double* slab = a.slab + (size_t)(b0 / kSeq) * a.slab_size;
#pragma unroll
  for (int xt = 0; xt < 2; xt++)
#pragma unroll
    for (int yt = 0; yt < 2; yt++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int x = 2 * (k4 + 4 * r) + xt, y = 2 * s + yt;
        slab[x * NP + y] = acc.K[xt][yt][r] + ob[((xt * 2 + yt) * 4 + r) * 64 + lane];
      }
  double* Hs = slab + NP * NP;
#pragma unroll
  for (int mt = 0; mt < kMaxMT; mt++)
#pragma unroll
    for (int yt = 0; yt < 2; yt++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int vr = 16 * mt + k4 + 4 * r, y = 2 * s + yt;
        int row = -1;
#pragma unroll
        for (int c = 0; c < NC; c++)
          if (c < a.ncol && vr >= a.voff[c] && vr < a.voff[c] + a.M[c]) row = a.crow[c] + vr - a.voff[c];
        if (row >= 0) Hs[(size_t)row * NP + y] = acc.Hc[mt][yt][r] + ob[((4 + mt * 2 + yt) * 4 + r) * 64 + lane];
      }
  // the rows the matrix cores do not hold: the small sums of both partners
  // (the backward one's in LDS) staged in LDS as [field][NP], then every
  // observed column's missing row (and its all-zero out-of-range row), every
  // unobserved child's rows (missing: every step's gamma, the rest 0), P0
  if (k4 == 0) {
#pragma unroll
    for (int f = 0; f < 6; f++) {
      v2d* q = reinterpret_cast<v2d*>(small + f * NP + 2 * s);
      *q = sm[f] + *q;
    }
  }
  if (lane < NP) {
    const int y = lane;
    for (int c = 0; c < a.ncol && c < 4; c++) {
      Hs[(size_t)(a.crow[c] + a.M[c]) * NP + y] = small[c * NP + y];
      Hs[(size_t)(a.crow[c] + a.M[c] + 1) * NP + y] = 0.0;
    }
    for (int u = 0; u < a.n_unobs && u < 4; u++)
      for (int m = 0; m <= a.uM[u] + 1; m++) Hs[(size_t)(a.urow[u] + m) * NP + y] = m == a.uM[u] ? small[4 * NP + y] : 0.0;
    Hs[(size_t)a.R * NP + y] = small[5 * NP + y];
  }
}

template <int NC>
__global__ __launch_bounds__(kThreads, 1) void chain_estep_mw_kernel(EMwArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* lds = reinterpret_cast<double*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool filter = wave < 2 * kGroups;
  const int role = filter ? wave : wave - 2 * kGroups;
  const int grp = role >> 1;
  const bool fwd = (role & 1) == 0;
  double* ring = lds + (grp * 2 + (fwd ? 0 : 1)) * 2 * kSlot;
  int* rexp = reinterpret_cast<int*>(lds + kRingD) + (grp * 2 + (fwd ? 0 : 1)) * 2 * kRows * kRowI;
  double* cz = lds + kRingD + kExpI / 2 + (grp * 2 + (fwd ? 0 : 1)) * kSeq * 2;
  double* small = lds + kRingD + kExpI / 2 + kCzD + grp * 6 * NP;
  double* tab = lds + kRingD + kExpI / 2 + kCzD + kSmallD;
  const int j = lane & 15, g = lane >> 4;
  const long b0 = (long)blockIdx.x * (kGroups * kSeq) + grp * kSeq;
  const int T = a.T, H = a.H;

  for (int i = tid; i < a.tab_rows * NP; i += kThreads) tab[(i / NP) * NPS + i % NP] = a.tab[i];
  __syncthreads();
#ifndef NIPAMD_MW_PRIO
#define NIPAMD_MW_PRIO 0   // A/B builds: 1 the filters above the partners sharing their SIMDs
#endif
  if (NIPAMD_MW_PRIO == 1 && filter) __builtin_amdgcn_s_setprio(1);

  const int nA = H > T - 1 - H ? H : T - 1 - H, nB = T - H > H + 1 ? T - H : H + 1;
  const int nchA = (nA + CH - 1) / CH, nchB = (nB + CH - 1) / CH;
  const long gi = b0 / kSeq;                               // the group's scratch
  const long ngroups = (a.B + kGroups * kSeq - 1) / (kGroups * kSeq) * kGroups;
  double* Sblk = a.S + gi * group_msgs(T) + (long)kG * kStep;
  int* Eblk = reinterpret_cast<int*>(a.S + ngroups * group_msgs(T)) + gi * group_exps(T) + (long)kG * kSeq;
  if (!filter) {
    if (fwd) epartner<true, NC>(a, ring, rexp, cz, small, tab, Sblk, Eblk, lane, b0, nchA, nchB);
    else epartner<false, NC>(a, ring, rexp, cz, small, tab, Sblk, Eblk, lane, b0, nchA, nchB);
    return;
  }
  FCtx c;
  c.tab = tab;
  c.obs = (a.ncol > 0 && b0 + j < a.B) ? a.obs + (b0 + j) * a.obs_bstride : nullptr;
  c.ots = a.obs_tstride;
  c.T = T;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    c.col[k] = a.col[k];
    c.M[k] = a.ncol > 0 ? a.M[k] : 0;                    // no observed column: row 0 (the row sums) every step
    c.tab_off[k] = (k < (a.ncol > 0 ? a.ncol : 1) ? a.tab_off[k] / NP * NPS : 0) + 2 * g;
  }
  c.ring = ring;
  c.rexp = rexp;
  c.j = j;
  c.g = g;
#pragma unroll
  for (int q = 0; q < NT; q++) {
    c.wo[q][0] = piece_off(j, 8 * q + g);
    c.wo[q][1] = piece_off(j, 8 * q + 4 + g);
  }
  if (fwd) efilter<true, NC>(a, c, lane, b0, nchA, nchB);
  else efilter<false, NC>(a, c, lane, b0, nchA, nchB);
}

template <int NC>
int launch_nc(const EMwArgs& a, size_t lds, hipStream_t stream) {
  static size_t set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_estep_mw_kernel<NC>), lds, set)) return rc;
  const int blocks = (int)((a.B + kGroups * kSeq - 1) / (kGroups * kSeq));
  hipLaunchKernelGGL((chain_estep_mw_kernel<NC>), dim3(blocks), dim3(kThreads), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

int estep_mw_max_cols() { return kMaxCols; }

size_t estep_mw_lds_bytes(int tab_rows) { return (lds_doubles(tab_rows) * sizeof(double) + 15) & ~(size_t)15; }

size_t estep_mw_scratch_bytes(long B, int T) {
  const long ngroups = (B + kGroups * kSeq - 1) / (kGroups * kSeq) * kGroups;
  return (size_t)ngroups * (group_msgs(T) * sizeof(double) + group_exps(T) * sizeof(int)) + 256;
}

int estep_mw_launch(const EMwArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  const int nc = a.ncol > 0 ? a.ncol : 1;
  int rows = 0;
  for (int c = 0; c < a.ncol; c++) rows = std::max(rows, a.voff[c] + a.M[c]);
  const size_t lds = estep_mw_lds_bytes(a.tab_rows);
  // up to two evidence columns (three or four spill the partner's registers:
  // the two-kernel route of estep_wide.hip takes them)
  if (a.N > NP || a.N < 1 || nc > kMaxCols || rows > kMaxMT * 16 || a.n_unobs > 4 || lds > 160 * 1024) return -2;
  const int rc = nc == 1 ? launch_nc<1>(a, lds, stream) : launch_nc<2>(a, lds, stream);
  g_last_kernel = "chain_estep_mw_kernel";
  return rc;
}

}  // namespace nipamd
