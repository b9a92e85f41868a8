// estep_wide.hip -- e_step for interface chains of up to 64 states (the chain
// plans of SURVEY 8(d) configs 3 and 5: demo1's structure at 32 states, the
// 64^4 wide clique after its GPU fold), any number of hidden independent
// parents, up to four leaf children.
//
// The reference's e_step (src/nip.c:1708-2007, families nip.c:1925-1967)
// sums, per sequence and step, the normalised family marginals of every
// variable.  For an interface chain they all follow from three sums
// (the general chain e_step):
//   K(x, y)   = sum_t alpha_{t-1}(x) e_t(y) beta_t(y) / Z_t   (the in-clique's
//               joint posterior without its table factor; alpha_{-1} = prior)
//   H[r][y]   = sum_t [r = row of child k's code at t] gamma_t(y)   (the
//               children's count tables, one row per state + missing + zero)
//   P0(x)     = gamma_{-1}(x) = prior(x) beta_{-1}(x) / Z   (the previous
//               interface at t = 0; OLD_OUTGOING is skipped at t > 0)
// and the finalize projects them onto the em_learn layout (a CSR map built
// once per model version, engine.cpp ensure_chain_map).
//
// Two kernels:
//  * chain_msgs_kernel<NP>: the two filters, every message stored.  One wave
//    per direction holds 64 / NP sequences, lane = state; the mat-vec takes
//    the input by DPP row broadcast (v_fmac_f64_dpp row_newbcast, after
//    v_permlane16/32_swap put the sequence's 16-state blocks in each of its
//    rows) against the lane's column (forward) or row (backward) of A in
//    registers -- no LDS on the recursion's path.  alpha^_t = alpha_t 2^Ef_t (Ef_t stored,
//    one int per step) and beta^_t (t = -1 .. T-1, scale free for the
//    statistics) go to HBM; the forward wave keeps the ll (m2 / m1 per step,
//    nip.c:1461-1474) as chain_wide.hip does.
//  * chain_stats_kernel<NT, HR>: the three sums on the matrix cores.  With
//    c_t = sum_y alpha^_t(y) beta^_t(y) and w_t(y) = e_t(y) beta^_t(y)
//    2^(Ef_t - Ef_{t-1}) / c_t (the 2^Ef factors cancel the scales of the
//    stored messages), K = sum_t alpha^_{t-1} (x) w_t is a GEMM whose inner
//    dimension is time: one v_mfma_f64_16x16x4 per 16x16 tile and four steps
//    (lane l: step l >> 4, state 16 tile + (l & 15)).  H is the same GEMM with
//    a one-hot A operand (row = child code) against gamma_t = alpha^ beta^ / c.
//    A block of four waves owns 16 sequences (four per wave, one after
//    another); the waves' sums meet in LDS in a fixed order and the block
//    writes one slab row, which tree64_kernel reduces like every e_step slab.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <type_traits>

#include "chain_kernels.h"
#include "dpp_row.h"
#include "opchain.h"
#include "store_pol.h"

namespace nipamd {

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int kMsgWaves = 4;                 // 2 forward + 2 backward (no LDS: blocks just group waves)
constexpr int kMsgChunk = 8;                 // steps of evidence prefetched ahead
constexpr int kStatSeqs = 16;                // sequences per stats block (one slab row)
constexpr int kStatWaves = 4;

template <int K>
__device__ __forceinline__ double rorK(double v) {     // row_ror:K of a double (16-lane rows)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x120 + K, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// x[l ^ 16] + x[l] in both lanes: the pair's sum (the swap's second operand
// a copy of x made as a whole double: one v_mov_b64)
__device__ __forceinline__ double swap16(double x) {
  double xc = x;
  asm("" : "+v"(xc));
  const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
__device__ __forceinline__ double swap32(double x) {
  double xc = x;
  asm("" : "+v"(xc));
  const auto rl = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
  const auto rh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
  return __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
}
// sum over aligned groups of L lanes (16, 32 or 64); every level pairs equal
// partial sums, so all L lanes end with the same bits
template <int L>
__device__ __forceinline__ double group_sum(double x) {
  asm("" : "+v"(x));       // one rounded value per lane: no fma contraction into the first add
  x += rorK<8>(x);
  x += rorK<4>(x);
  x += rorK<2>(x);
  x += rorK<1>(x);
  if (L >= 32) x = swap16(x);
  if (L >= 64) x = swap32(x);
  return x;
}

__device__ __forceinline__ double recip(double c) {
  double r = __builtin_amdgcn_rcp(c);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-c, r, 1.0), r);
  return c != 0.0 ? r : 0.0;
}

// child c's code at step t: its state, M missing, M + 1 out of range
__device__ __forceinline__ int code_of(int o, int M) { return o < 0 ? M : (o < M ? o : M + 1); }

// the step's evidence e_t(y): the unobserved children's row sums times each
// observed child's table row
__device__ __forceinline__ double evidence(const EWideArgs& a, const int* o, int y) {
  double e = a.ebase[y];
  for (int c = 0; c < a.ncol; c++) e *= a.tab[a.tab_off[c] + code_of(o[a.col[c]], a.M[c]) * 64 + y];
  return e;
}

// acc[j & 3] += x(lane j of the row) * Ac[j], j = 0..15 (four chains, the
// broadcast by DPP row_newbcast, as chain_row64_kernel does)
__device__ __forceinline__ void fmac16(double (&acc)[4], double xb, const double (&Ac)[16]) {
  fmac_bcast<0, true>(acc[0], xb, Ac[0]);    fmac_bcast<1, false>(acc[1], xb, Ac[1]);
  fmac_bcast<2, false>(acc[2], xb, Ac[2]);   fmac_bcast<3, false>(acc[3], xb, Ac[3]);
  fmac_bcast<4, false>(acc[0], xb, Ac[4]);   fmac_bcast<5, false>(acc[1], xb, Ac[5]);
  fmac_bcast<6, false>(acc[2], xb, Ac[6]);   fmac_bcast<7, false>(acc[3], xb, Ac[7]);
  fmac_bcast<8, false>(acc[0], xb, Ac[8]);   fmac_bcast<9, false>(acc[1], xb, Ac[9]);
  fmac_bcast<10, false>(acc[2], xb, Ac[10]); fmac_bcast<11, false>(acc[3], xb, Ac[11]);
  fmac_bcast<12, false>(acc[0], xb, Ac[12]); fmac_bcast<13, false>(acc[1], xb, Ac[13]);
  fmac_bcast<14, false>(acc[2], xb, Ac[14]); fmac_bcast<15, false>(acc[3], xb, Ac[15]);
}

// the NB = NP / 16 blocks of 16 states of this lane's sequence, each in
// every lane of the sequence's rows: xb[b](lane 16 r + j) = x(state 16 b + j).
// One row per sequence (NB 1): x itself; two rows (NB 2): one
// v_permlane16_swap per half ([0]: the pair's even row, [1]: its odd row);
// four rows (NB 4): a v_permlane32_swap level on both results.
template <int NB>
__device__ __forceinline__ void seq_blocks(double x, double (&xb)[NB]) {
  if constexpr (NB == 1) {
    xb[0] = x;
  } else {
    // the swaps' second operands are copies made as whole doubles (one
    // v_mov_b64 each)
    double xc = x;
    asm("" : "+v"(xc));
    const auto pl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(xc), false, false);
    const auto ph = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(xc), false, false);
    if constexpr (NB == 2) {
      xb[0] = __hiloint2double((int)ph[0], (int)pl[0]);
      xb[1] = __hiloint2double((int)ph[1], (int)pl[1]);
    } else {
      double p0 = __hiloint2double((int)ph[0], (int)pl[0]), p1 = __hiloint2double((int)ph[1], (int)pl[1]);
      double p0c = p0, p1c = p1;
      asm("" : "+v"(p0c));
      asm("" : "+v"(p1c));
      const auto q0l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(p0), (unsigned)__double2loint(p0c), false, false);   // blocks 0, 2
      const auto q0h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(p0), (unsigned)__double2hiint(p0c), false, false);
      const auto q1l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(p1), (unsigned)__double2loint(p1c), false, false);   // blocks 1, 3
      const auto q1h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(p1), (unsigned)__double2hiint(p1c), false, false);
      xb[0] = __hiloint2double((int)q0h[0], (int)q0l[0]);
      xb[2] = __hiloint2double((int)q0h[1], (int)q0l[1]);
      xb[1] = __hiloint2double((int)q1h[0], (int)q1l[0]);
      xb[3] = __hiloint2double((int)q1h[1], (int)q1l[1]);
    }
  }
}

// u(y) = sum_x Ac[x / 16][x % 16] x(x) over this lane's sequence: NP
// v_fmac_f64_dpp in registers, no LDS on the recursion's path
template <int NB>
__device__ __forceinline__ double matvec_dpp(double x, const double (&Ac)[NB][16]) {
  double xb[NB];
  seq_blocks<NB>(x, xb);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int b = 0; b < NB; b++) fmac16(acc, xb[b], Ac[b]);
  return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// the rescale exponent of a proper model's forward filter: minus the largest
// binary exponent over the sequence's NP lanes (zeros excluded; 0 for an
// all-zero vector), integer DPP / permlane work instead of an f64 sum
template <int NP>
__device__ __forceinline__ int group_max_exp_rescale(double p) {
  int e = p != 0.0 ? __builtin_amdgcn_frexp_exp(p) : -0x40000;
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x128, 0xF, 0xF, true));   // row_ror:8
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x124, 0xF, 0xF, true));   // row_ror:4
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x122, 0xF, 0xF, true));   // row_ror:2
  e = max(e, __builtin_amdgcn_mov_dpp(e, 0x121, 0xF, 0xF, true));   // row_ror:1
  if (NP >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)e, (unsigned)e, false, false);
    e = max((int)r[0], (int)r[1]);
  }
  if (NP >= 64) {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)e, (unsigned)e, false, false);
    e = max((int)r[0], (int)r[1]);
  }
  return e > -0x40000 ? -e : 0;
}

// PR: a proper model (EWideArgs::proper): the forward filter keeps no step
// masses -- the reference's per-step log m2 - log m1 telescope to log P(obs)
// (m1_t is the previous step's mass when A's and the children's rows sum to
// 1) -- and rescales by the group's largest exponent
template <int NP, bool PR>
__global__ __launch_bounds__(kMsgWaves * 64) void chain_msgs_kernel(EWideArgs a) {
  constexpr int SPW = 64 / NP;                        // sequences per wave
  constexpr int NB = NP / 16;                         // 16-lane rows per sequence
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int WD = kMsgWaves / 2;                  // waves per direction
  const bool fwd = wave < WD;
  const int s = lane / NP, y = lane % NP;
  const long b = (long)blockIdx.x * (WD * SPW) + (wave % WD) * SPW + s;
  const bool active = b < a.B;
  const long bb = active ? b : 0;
  const int T = a.T, N = a.N;
  // the lane's column (forward) / row (backward) of A, in 16-state blocks
  double Ac[NB][16];
#pragma unroll
  for (int k = 0; k < NB; k++)
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int x = 16 * k + j;
      Ac[k][j] = (x < N && y < N) ? (fwd ? a.A[x * 64 + y] : a.A[y * 64 + x]) : 0.0;
    }
  const int* obs = a.obs + bb * a.obs_bstride;
  const double eb = (active && y < N) ? a.ebase[y] : 0.0;
  // evidence of a chunk of steps in processing order (forward t = j, backward
  // t = T - 1 - j): the children's codes two chunks ahead, the table entries
  // (and e) one chunk ahead, so no global load's latency meets the recursion
  int cd[4][kMsgChunk];
  auto ldcodes = [&](int j0) {
#pragma unroll
    for (int c = 0; c < 4; c++)
      if (c < a.ncol)
#pragma unroll
        for (int k = 0; k < kMsgChunk; k++) {
          const int t = fwd ? j0 + k : T - 1 - (j0 + k);
          cd[c][k] = (t >= 0 && t < T) ? code_of(obs[(long)t * a.obs_tstride + a.col[c]], a.M[c]) : a.M[c];
        }
  };
  auto evc = [&](double (&e)[kMsgChunk]) {
#pragma unroll
    for (int k = 0; k < kMsgChunk; k++) e[k] = eb;
#pragma unroll
    for (int c = 0; c < 4; c++)
      if (c < a.ncol)
#pragma unroll
        for (int k = 0; k < kMsgChunk; k++) e[k] *= a.tab[a.tab_off[c] + cd[c][k] * 64 + y];
  };
  double e[kMsgChunk], en[kMsgChunk];
  ldcodes(0);
  evc(e);
  ldcodes(kMsgChunk);
  if (fwd) {
    double* Sa = a.Sa + (size_t)bb * T * NP + y;
    int* Ea = a.Ea + (size_t)bb * T;
    double x = (active && y < N) ? a.pi[y] : 0.0;
    const double sy = y < N ? a.s[y] : 0.0;
    int sc = 0, E = 0;
    double m2 = 1.0, m1 = 1.0, zmin = 1.0;
    int e2 = 0, e1 = 0;
    for (int t0 = 0; t0 < T; t0 += kMsgChunk) {
      evc(en);
      ldcodes(t0 + 2 * kMsgChunk);
#pragma unroll
      for (int k = 0; k < kMsgChunk; k++) {
        const int t = t0 + k;
        if (t >= T) break;
        const double u = __builtin_ldexp(matvec_dpp<NB>(x, Ac), sc);
        const double p = u * e[k];
        E += sc;
        if (active) {
          store_pol<NIPAMD_MSG_NT>(Sa + (size_t)t * NP, p);
          if (y == 0) Ea[t] = E;
        }
        if (PR) {
          sc = group_max_exp_rescale<NP>(p);
        } else {
          const double z2 = group_sum<NP>(p);
          const double z1 = group_sum<NP>(u * sy);
          zmin = __builtin_fmin(zmin, z2);
          m2 *= z2; m1 *= z1;
          if ((k & 3) == 3) {
            const int k2 = __builtin_amdgcn_frexp_exp(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2;
            const int k1 = __builtin_amdgcn_frexp_exp(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1;
          }
          sc = z2 != 0.0 ? -__builtin_amdgcn_frexp_exp(z2) : 0;
        }
        x = p;
      }
#pragma unroll
      for (int k = 0; k < kMsgChunk; k++) e[k] = en[k];
    }
    // proper: ll = log(sum alpha^_{T-1}) - E_{T-1} ln 2 (x = alpha^_{T-1})
    const double zT = PR ? group_sum<NP>(x) : 0.0;
    if (active && y == 0) {
      double ll = PR ? log(zT) - (double)E * 0.69314718055994530942
                     : log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
      const bool dead = PR ? zT == 0.0 : zmin == 0.0;
      if (dead) ll = -DBL_MAX;
      if (a.ll) a.ll[b] = ll;
      // e_step's BAD_LUCK (m1 <= 0 || m2 <= 0, nip.c:1827-1854): a zero mass
      if (a.status) a.status[b] = dead ? 3u : 0u;
    }
  } else {
    // beta^_{T-1} = 1 at row T, then beta^_{t-1} = A (e_t o beta^_t) 2^sc at row t
    double* Sb = a.Sb + (size_t)bb * (T + 1) * NP + y;
    double xbeta = (active && y < N) ? 1.0 : 0.0;
    if (active) Sb[(size_t)T * NP] = xbeta;
    for (int j0 = 0; j0 < T; j0 += kMsgChunk) {
      evc(en);
      ldcodes(j0 + 2 * kMsgChunk);
#pragma unroll
      for (int k = 0; k < kMsgChunk; k++) {
        const int t = T - 1 - (j0 + k);
        if (t < 0) break;
        const double g = e[k] * xbeta;
        const double z = group_sum<NP>(g);
        const int sc = z != 0.0 ? -__builtin_amdgcn_frexp_exp(z) : 0;
        const double u = __builtin_ldexp(matvec_dpp<NB>(g, Ac), sc);
        if (active) Sb[(size_t)t * NP] = u;
        xbeta = u;
      }
#pragma unroll
      for (int k = 0; k < kMsgChunk; k++) e[k] = en[k];
    }
  }
}

// One 16x16x4 f64 MFMA: D += A (16 x 4) B (4 x 16); lane l supplies
// A[l & 15][l >> 4] and B[l >> 4][l & 15], and holds D[(l >> 4) + 4 r][l & 15].
__device__ __forceinline__ v4d mfma(double a, double b, v4d d) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
}

// the children's evidence tables [(M_k + 2)][64] and ebase [64], staged in
// LDS for the statistics kernel (doubles)
__host__ __device__ inline int stats_tab_doubles(const EWideArgs& a) {
  int n = 0;
  for (int c = 0; c < a.ncol; c++) n = max(n, a.tab_off[c] + (a.M[c] + 2) * 64);
  return n + 64;
}

// TL: the tables fit the LDS (otherwise they are read from HBM / L2)
template <int NT, int HR, bool TL>
__global__ __launch_bounds__(kStatWaves * 64, 1) void chain_stats_kernel(EWideArgs a) {
  constexpr int NP = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* red = reinterpret_cast<double*>(smem);     // [2][NT*NT + HR*NT][4][64]: the waves' sums
  // the evidence tables share the LDS with the reduction (used before it)
  double* tabs = reinterpret_cast<double*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k4 = lane >> 4, i = lane & 15;
  const int T = a.T, N = a.N;
  if (TL) {
    const int nt = stats_tab_doubles(a) - 64;
    for (int j = tid; j < nt; j += kStatWaves * 64) tabs[j] = a.tab[j];
    for (int j = tid; j < 64; j += kStatWaves * 64) tabs[nt + j] = a.ebase[j];
    __syncthreads();
  }
  const double* tabl = TL ? tabs : a.tab;
  const double* ebl = TL ? tabs + (stats_tab_doubles(a) - 64) : a.ebase;
  constexpr int NK = NT * NT, NH = HR * NT;
  v4d K[NK], Hc[NH];
#pragma unroll
  for (int q = 0; q < NK; q++) K[q] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < NH; q++) Hc[q] = v4d{0.0, 0.0, 0.0, 0.0};
  double p0 = 0.0;                                   // P0 of state `lane` (lane < NP)
  const int hr = (a.R + 15) >> 4;                    // row tiles in use (<= HR)

  // this wave's sequences one after another, 4 steps per iteration (lane:
  // step t0 + k4); every global operand of iteration it + 1 is loaded while
  // iteration it runs on the matrix cores
  const long b0 = (long)blockIdx.x * kStatSeqs + wave * (kStatSeqs / kStatWaves);
  const long nb = a.B - b0;
  const int nseq = nb <= 0 ? 0 : (nb < kStatSeqs / kStatWaves ? (int)nb : kStatSeqs / kStatWaves);
  const int nit = (T + 3) >> 2;
  const int total = nseq * nit;
  struct Ops {
    double ap[NT], al[NT], be[NT];
    int ef, oc[4], orow[4];
  };
  auto load = [&](int it, Ops& o) {
    const int sq = it / nit, t0 = (it - sq * nit) * 4;
    const long b = b0 + sq;
    const double* Sa = a.Sa + (size_t)b * T * NP;
    const double* Sb = a.Sb + (size_t)b * (T + 1) * NP;
    const int* Ea = a.Ea + (size_t)b * T;
    const int t = t0 + k4;
    const int tc = t < T ? t : T - 1;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      const int st = 16 * q + i;
      o.ap[q] = tc >= 1 ? Sa[(size_t)(tc - 1) * NP + st] : (st < N ? a.pi[st] : 0.0);
      o.al[q] = Sa[(size_t)tc * NP + st];
      o.be[q] = Sb[(size_t)(tc + 1) * NP + st];
    }
    o.ef = Ea[tc] - (tc >= 1 ? Ea[tc - 1] : 0);
    const int* ob = a.obs + b * a.obs_bstride + (long)tc * a.obs_tstride;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      o.oc[c] = c < a.ncol ? code_of(ob[a.col[c]], a.M[c]) : 0;
      o.orow[c] = c < a.nchild ? a.erow[c] + (a.ccol[c] >= 0 ? code_of(ob[a.ccol[c]], a.cM[c]) : a.cM[c]) : -1;
    }
  };
  Ops cur, nxt;
  if (total > 0) load(0, cur);
  for (int it = 0; it < total; it++) {
    if (it + 1 < total) load(it + 1, nxt);
    const int sq = it / nit, t0 = (it - sq * nit) * 4;
    if (t0 == 0) {
      // P0: gamma_{-1} = prior o beta^_{-1} / its sum (lanes 0 .. NP-1: state = lane)
      const double* Sb = a.Sb + (size_t)(b0 + sq) * (T + 1) * NP;
      const int x = lane < NP ? lane : 0;
      const double v = (lane < NP && x < N) ? a.pi[x] * Sb[x] : 0.0;
      const double z = group_sum<64>(v);
      p0 += v * recip(z);
    }
    const bool ok = t0 + k4 < T;
    double ev[NT];
#pragma unroll
    for (int q = 0; q < NT; q++) {
      const int st = 16 * q + i;
      double e = ebl[st];
#pragma unroll
      for (int c = 0; c < 4; c++)
        if (c < a.ncol) e *= tabl[a.tab_off[c] + cur.oc[c] * 64 + st];
      ev[q] = st < N ? e : 0.0;
    }
    double pr[NT];
    double zz = 0.0;
#pragma unroll
    for (int q = 0; q < NT; q++) { pr[q] = cur.al[q] * cur.be[q]; zz += pr[q]; }
    const double c = group_sum<16>(zz);
    const double rc = ok ? recip(c) : 0.0;
    const double f = __builtin_ldexp(rc, cur.ef);
    double w[NT], g[NT];
#pragma unroll
    for (int q = 0; q < NT; q++) { w[q] = ev[q] * cur.be[q] * f; g[q] = pr[q] * rc; }
#pragma unroll
    for (int xi = 0; xi < NT; xi++)
#pragma unroll
      for (int yj = 0; yj < NT; yj++) K[xi * NT + yj] = mfma(cur.ap[xi], w[yj], K[xi * NT + yj]);
#pragma unroll
    for (int mi = 0; mi < HR; mi++) {
      if (mi >= hr) break;
      const int r = 16 * mi + i;
      const double oh = (r == cur.orow[0] || r == cur.orow[1] || r == cur.orow[2] || r == cur.orow[3]) ? 1.0 : 0.0;
#pragma unroll
      for (int yj = 0; yj < NT; yj++) Hc[mi * NT + yj] = mfma(oh, g[yj], Hc[mi * NT + yj]);
    }
    cur = nxt;
  }
  __syncthreads();                                   // the tables' LDS becomes the reduction's
  // the waves' sums in a fixed order: (w0 + w2) + (w1 + w3)
  constexpr int NA = NK + NH;
  auto put = [&](int slot) {
    double* d = red + (size_t)slot * NA * 256;
#pragma unroll
    for (int q = 0; q < NK; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) d[(q * 4 + r) * 64 + lane] = K[q][r];
#pragma unroll
    for (int q = 0; q < NH; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) d[((NK + q) * 4 + r) * 64 + lane] = Hc[q][r];
  };
  auto add = [&](int slot) {
    const double* d = red + (size_t)slot * NA * 256;
#pragma unroll
    for (int q = 0; q < NK; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) K[q][r] += d[(q * 4 + r) * 64 + lane];
#pragma unroll
    for (int q = 0; q < NH; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) Hc[q][r] += d[((NK + q) * 4 + r) * 64 + lane];
  };
  double* p0s = red + (size_t)2 * NA * 256;          // [4][64]
  p0s[wave * 64 + lane] = p0;
  if (wave >= 2) put(wave - 2);
  __syncthreads();
  if (wave < 2) add(wave);
  __syncthreads();
  if (wave == 1) put(0);
  __syncthreads();
  if (wave != 0) return;
  add(0);
  const double pz = (p0s[lane] + p0s[128 + lane]) + (p0s[64 + lane] + p0s[192 + lane]);
  double* slab = a.slab + (size_t)blockIdx.x * a.slab_size;
  // K[x][y]: tile (xi, yj), D[(l >> 4) + 4r][l & 15]
#pragma unroll
  for (int xi = 0; xi < NT; xi++)
#pragma unroll
    for (int yj = 0; yj < NT; yj++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        slab[(size_t)(16 * xi + k4 + 4 * r) * NP + 16 * yj + i] = K[xi * NT + yj][r];
  double* Hs = slab + NP * NP;
#pragma unroll
  for (int mi = 0; mi < HR; mi++)
#pragma unroll
    for (int yj = 0; yj < NT; yj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * mi + k4 + 4 * r;
        if (row < a.R) Hs[(size_t)row * NP + 16 * yj + i] = Hc[mi * NT + yj][r];
      }
  if (lane < NP) slab[(size_t)NP * NP + (size_t)a.R * NP + lane] = pz;
}

template <int NT, int HR>
int stats_launch(const EWideArgs& a, hipStream_t stream) {
  constexpr int NA = NT * NT + HR * NT;
  const size_t red = (size_t)2 * NA * 256 * sizeof(double) + 4 * 64 * sizeof(double);
  const size_t tabs = (size_t)stats_tab_doubles(a) * sizeof(double);
  const bool tl = std::max(red, tabs) <= 160 * 1024;
  const size_t lds = tl ? std::max(red, tabs) : red;
  static size_t set[2][kMaxDevices] = {};
  const void* k = tl ? reinterpret_cast<const void*>(&chain_stats_kernel<NT, HR, true>)
                     : reinterpret_cast<const void*>(&chain_stats_kernel<NT, HR, false>);
  if (int rc = ensure_dyn_lds(k, lds, set[tl])) return rc;
  const int blocks = (int)((a.B + kStatSeqs - 1) / kStatSeqs);
  if (tl) hipLaunchKernelGGL((chain_stats_kernel<NT, HR, true>), dim3(blocks), dim3(kStatWaves * 64), lds, stream, a);
  else hipLaunchKernelGGL((chain_stats_kernel<NT, HR, false>), dim3(blocks), dim3(kStatWaves * 64), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- the operator chain at 17..64 joint interface states (opchain.h) ----
//
// op_fb_kernel's recursion (opchain.hip) with the wide e_step's layout: a
// wave per direction holds 64 / NP sequences (lane = state), the step's
// operator column (forward: T'(x, y) for lane y) or row (backward: T'(y, x))
// is read per step -- from LDS when the operators fit (TL), else through the
// caches -- one step ahead of its use, and the mat-vec takes the input by DPP
// row broadcasts.  With the leaf factors e_t(y) = prod_j F_j[c_j,t](y):
//   forward:  alpha_t = e_t o T'^T alpha_{t-1}  (alpha_{-1} = prior), stored
//   backward: beta_{t-1} = T' (e_t o beta_t)   (beta_{T-1} = 1), stored
//   ll = sum over steps with evidence of log m2_t - log m1_t (nip.c:1458-1474)
// the step's operator index c' | (the step has evidence) << 30
constexpr int kOpEv = 1 << 30;
__device__ __forceinline__ int op_code(const OpWideArgs& a, const int32_t* o) {
  int c = 0;
  bool ev = false, oor = false;
  for (int k = 0; k < a.onobs; k++) {
    const int v = o[a.ocol[k]];
    oor |= v >= a.ocard[k];
    ev |= v >= 0;
    if (v >= 0) c += (v + 1) * a.ocstride[k];
  }
  for (int j = 0; j < a.nleaf; j++) ev |= o[a.lcol[j]] >= 0;
  return (oor ? a.oncomb : c) | (ev ? kOpEv : 0);
}

// the leaf factors' product at state y (1 without leaves)
__device__ __forceinline__ double op_leaf_e(const OpWideArgs& a, const int32_t* o, int y) {
  double e = 1.0;
  for (int j = 0; j < a.nleaf; j++) {
    const int v = o[a.lcol[j]], M = a.lcard[j];
    const int r = v < 0 ? M : (v < M ? v : M + 1);
    e *= a.ltab[a.loff[j] + r * a.K + y];
  }
  return e;
}

typedef __attribute__((address_space(3))) double op_lds_d;
typedef double op_d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) op_d2 op_lds_d2;

// op_wide_msgs_kernel's LDS row stride: K rounded up to 2 mod 4 entries
__host__ __device__ inline int op_lds_row(int K) { return (K + 1) / 4 * 4 + 2; }
// ... and its LDS copy's length: (oncomb + 1) operators of K rows, NP - K
// zero rows, NP zeros (the last lane's reads run NP entries from its row)
__host__ __device__ inline int op_lds_doubles(int oncomb, int K, int NP) {
  return (oncomb * K + NP) * op_lds_row(K) + NP;
}

// op_wide_msgs_kernel per width: waves per block, steps of evidence prepared
// a chunk ahead, and the waves per SIMD the registers are held to.  The
// operators' LDS copy is staged once per block and at most two blocks fit a
// CU, so at NP = 32 the block is wide (8 waves) and a 3-step chunk keeps it
// within 128 registers: four waves per SIMD (estep_opchain_wide 3.95 ->
// 3.46 ms, opchain_wide 2.46 -> 1.97 ms: profiles/r05/gpu/r05x_*).  At NP = 64
// (64 coefficient registers more) the narrow block stays.
template <int NP>
struct MsgCfg {
  static constexpr int waves = 4, chunk = 8, wpe = 1;
};
template <>
struct MsgCfg<32> {
  static constexpr int waves = 8, chunk = 3, wpe = 4;
};

template <int NP, bool TL>
__global__ __launch_bounds__(MsgCfg<NP>::waves * 64) __attribute__((amdgpu_waves_per_eu(MsgCfg<NP>::wpe))) void op_wide_msgs_kernel(OpWideArgs a) {
  constexpr int kOpMsgWaves = MsgCfg<NP>::waves, kOpMsgChunk = MsgCfg<NP>::chunk;
  extern __shared__ __attribute__((aligned(16))) unsigned char op_smem[];
  constexpr int SPW = 64 / NP, NB = NP / 16;
  constexpr int SPB = kOpMsgWaves * SPW;                      // sequences per block
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T, K = a.K, KK = K * K;
  // blocks [0, nbd) run forward filters, [nbd, 2 nbd) backward ones: each
  // block stages one orientation of the operators, every state's row
  // contiguous -- forward T'^T (TtabT), backward T' -- so a lane reads its
  // step's coefficients at fixed offsets from one base, with no predicate
  const int nbd = (int)((a.B + SPB - 1) / SPB);
  const bool fwd = (int)blockIdx.x < nbd;
  const int blk = fwd ? (int)blockIdx.x : (int)blockIdx.x - nbd;
  const double* const src = fwd ? a.TtabT : a.Ttab;         // [(oncomb + 1)][K][K] + NP zeros
  // TL: the same in LDS, rows padded to Kp = op_lds_row(K) entries (zeros),
  // and NP - K zero rows after the last operator: every lane reads its own
  // row (lanes y >= K too), so a lane's 16-byte reads fall on distinct bank
  // slots across every 16-lane group of ds_read_b128 (the row stride is an
  // odd number of slots)
  op_lds_d* const Tl = (op_lds_d*)(op_smem);
  const int Kp = TL ? op_lds_row(K) : K;
  if (TL) {
    const int rows = (a.oncomb + 1) * K;
    for (int i = tid; i < op_lds_doubles(a.oncomb, K, NP); i += kOpMsgWaves * 64) {
      const int r = i / Kp, x = i - r * Kp;
      Tl[i] = (r < rows && x < K) ? src[r * K + x] : 0.0;
    }
    __syncthreads();
  }
  const int s = lane / NP, y = lane % NP;
  const long b = (long)blk * SPB + wave * SPW + s;
  const bool active = b < a.B;
  const long bb = active ? b : 0;
  const bool ys = y < K;
  const int yc = ys ? y : 0;
  const int32_t* obs = a.obs ? a.obs + bb * a.obs_bstride : nullptr;
  const bool est = a.estep != 0;
  int* const scrow = est ? a.sc + (size_t)bb * T : nullptr;
  // a chunk's steps: operator codes and leaf factors, a chunk ahead
  const int dir = fwd ? 1 : -1, t0 = fwd ? 0 : T - 1;
  // a chunk's 8 steps at once (t = t0 + dir * (j + k)): each observed
  // column's 8 loads issue together, then the leaves' table loads -- two
  // waits per column and chunk, not a chain of dependent loads per step
  auto prep = [&](int j, int (&code)[kOpMsgChunk], double (&e)[kOpMsgChunk]) {
    int c[kOpMsgChunk];
    bool ev[kOpMsgChunk], oor[kOpMsgChunk], in[kOpMsgChunk];
    const int32_t* o[kOpMsgChunk];
#pragma unroll
    for (int k = 0; k < kOpMsgChunk; k++) {
      const int t = t0 + dir * (j + k);
      in[k] = obs && t >= 0 && t < T;
      o[k] = obs + (long)(in[k] ? t : 0) * a.obs_tstride;
      c[k] = 0; ev[k] = false; oor[k] = false; e[k] = 1.0;
    }
    for (int q = 0; q < a.onobs; q++) {
      const int col = a.ocol[q], card = a.ocard[q], st = a.ocstride[q];
      int v[kOpMsgChunk];
#pragma unroll
      for (int k = 0; k < kOpMsgChunk; k++) v[k] = in[k] ? o[k][col] : -1;
#pragma unroll
      for (int k = 0; k < kOpMsgChunk; k++) {
        oor[k] |= v[k] >= card;
        ev[k] |= v[k] >= 0;
        if (v[k] >= 0) c[k] += (v[k] + 1) * st;
      }
    }
    for (int q = 0; q < a.nleaf; q++) {
      const int col = a.lcol[q], M = a.lcard[q];
      const double* lt = a.ltab + a.loff[q] + yc;
      int v[kOpMsgChunk];
#pragma unroll
      for (int k = 0; k < kOpMsgChunk; k++) v[k] = in[k] ? o[k][col] : -1;
#pragma unroll
      for (int k = 0; k < kOpMsgChunk; k++) {
        ev[k] |= v[k] >= 0;
        const int r = v[k] < 0 ? M : (v[k] < M ? v[k] : M + 1);
        e[k] *= in[k] ? lt[r * K] : 1.0;
      }
    }
#pragma unroll
    for (int k = 0; k < kOpMsgChunk; k++) code[k] = (oor[k] ? a.oncomb : c[k]) | (ev[k] ? kOpEv : 0);
  };
  // this lane's column (forward) / row (backward) of T'_c, in 16-state
  // blocks: entries x >= K read the next row or the padding (finite), and
  // meet x = 0 in the mat-vec; lanes y >= K read row 0 and are zeroed after
  auto coef = [&](int code, double (&C)[NB][16]) {
    const int base = (code & (kOpEv - 1)) * K * Kp + (TL ? y : yc) * Kp;
    if (TL) {
      const op_lds_d2* const p = (const op_lds_d2*)(Tl + base);   // 16-byte aligned: Kp even
#pragma unroll
      for (int k = 0; k < NB; k++)
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const op_d2 v = p[8 * k + j];
          C[k][2 * j] = v.x;
          C[k][2 * j + 1] = v.y;
        }
    } else {
#pragma unroll
      for (int k = 0; k < NB; k++)
#pragma unroll
        for (int j = 0; j < 16; j++) C[k][j] = src[base + 16 * k + j];
    }
  };
  int cc[kOpMsgChunk], cn[kOpMsgChunk];
  double ec[kOpMsgChunk], en[kOpMsgChunk];
  prep(0, cc, ec);
  double x;
  int sc = 0;
  double m2 = 1.0, m1 = 1.0;
  int e2 = 0, e1 = 0;
  bool dead = false, bad = false;
  const double wy = ys ? a.w[y] : 0.0;
  double* const Srow = (fwd ? a.Sa : a.Sb) + (size_t)bb * T * NP + y;
  if (fwd) {
    x = ys ? a.pi[y] : 0.0;
  } else {
    x = ys ? 1.0 : 0.0;                                 // beta_{T-1}
    if (active) Srow[(size_t)(T - 1) * NP] = x;
  }
  double C[NB][16];
  coef(cc[0], C);
  // forward: steps t = 0..T-1; backward: t = T-1..1 (each making beta_{t-1})
  const int n = fwd ? T : T - 1;
  for (int j0 = 0; j0 < n; j0 += kOpMsgChunk) {
    prep(j0 + kOpMsgChunk, cn, en);
#pragma unroll
    for (int k = 0; k < kOpMsgChunk; k++) {
      const int j = j0 + k;
      if (j >= n) break;
      const int t = t0 + dir * j;
      const double m1v = fwd ? group_sum<NP>(x * wy) : 0.0;
      const double acc = matvec_dpp<NB>(fwd ? x : x * ec[k], C);
      coef(k + 1 < kOpMsgChunk ? cc[k + 1] : cn[0], C);   // the next step's operator, under this step's work
      double u = ys ? __builtin_ldexp(acc, sc) : 0.0;
      if (fwd) u *= ec[k];
      const double z = group_sum<NP>(u);
      if (fwd) {
        if (cc[k] & kOpEv) {                            // a step with evidence
          m2 *= z;
          m1 *= __builtin_ldexp(m1v, sc);
          const int k2 = m2 != 0.0 ? __builtin_amdgcn_frexp_exp(m2) : 0;
          const int k1 = m1 != 0.0 ? __builtin_amdgcn_frexp_exp(m1) : 0;
          m2 = __builtin_ldexp(m2, -k2); e2 += k2;
          m1 = __builtin_ldexp(m1, -k1); e1 += k1;
          // e_step's BAD_LUCK (nip.c:1827-1854), as op_fb_kernel checks it
          if (est && (m2 <= 0.0 || m1 <= 0.0 || e2 > e1 || (e2 == e1 && m2 > m1))) bad = true;
        }
        dead |= z == 0.0;
        if (est && active && y == 0) scrow[t] = sc;
        if (active) store_pol<NIPAMD_MSG_NT>(Srow + (size_t)t * NP, u);   // alpha^_t
      } else {
        if (active) store_pol<NIPAMD_MSG_NT>(Srow + (size_t)(t - 1) * NP, u);   // beta^_{t-1}
      }
      sc = z != 0.0 ? -__builtin_amdgcn_frexp_exp(z) : 0;
      x = u;
    }
#pragma unroll
    for (int k = 0; k < kOpMsgChunk; k++) {
      cc[k] = cn[k];
      ec[k] = en[k];
    }
  }
  if (fwd && active && y == 0) {
    double ll = log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    // NIPAMD_STATUS_ZERO_MASS (1); in e_step mode also NIPAMD_STATUS_BAD_LUCK (2)
    if (a.status) a.status[b] = (dead ? 1u : 0u) | (est && (dead || bad) ? 2u : 0u);
  }
}

// posterior_t = normalise(alpha^_t o beta^_t) (filtering: alpha^_t), an
// all-zero row kept as is (nip_normalise_array, nippotential.c:354)
template <int NP>
__global__ __launch_bounds__(256) void op_wide_post_kernel(OpWideArgs a) {
  constexpr int SPW = 64 / NP;
  const int lane = threadIdx.x & 63, y = lane % NP;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * SPW + lane / NP;   // (b, t)
  const long nrow = a.B * a.T;
  const bool ok = row < nrow;
  const long r = ok ? row : 0;
  const double al = a.Sa[(size_t)r * NP + y];
  const double pr = a.filter ? al : al * a.Sb[(size_t)r * NP + y];
  const double z = group_sum<NP>(pr);
  const double q = z != 0.0 ? pr / z : pr;
  if (ok && y < a.K) {
    const long b = r / a.T, t = r - b * a.T;
    a.post[(size_t)b * a.post_bstride + (size_t)t * a.post_tstride + a.post_off + y] = q;
  }
}

// The operator chain's e_step at 17..64 states: op_xi_sort_kernel's sums
// (opchain.hip) from the stored messages.  Step t's xi weights are
//   W_t(x, y) = alpha^_{t-1}(x) e_t(y) beta^_t(y) f_t,  f_t = 2^sc_t / sum_y alpha^_t(y) beta^_t(y)
// (alpha^_t = 2^sc_t e_t o T'^T alpha^_{t-1}, so f_t = 1 / Z'_t, the step's xi
// mass; alpha^_{-1} = the prior; e_t the leaf factors, 1 without leaves), the
// same products as op_fb_kernel's xi_row.  They are summed per operator index
// c' (Xi'); each leaf's count rows sum the interface posterior gamma_t(y) =
// alpha^_t beta^_t / sum by the leaf's code at t.
// A block owns kOpWideSeqs = 8 sequences and one slab row (opchain.h; two
// blocks per CU).  The group's steps (sequence-major; at most kXwTileMax at a
// time, the whole group when T <= 2048) are sorted by (key, position) in LDS
// -- a bitonic sort of packed keys, so every key's steps keep their stream
// order -- then staged kXwBatch at a time, two batches in flight (the weights'
// two vectors and gamma per step in LDS, f_t by a wave sum), and summed in
// sorted order on the matrix cores (below).  A fixed summation order,
// independent of the launch (shard invariance).
#ifndef NIPAMD_XI_SKIP
#define NIPAMD_XI_SKIP 0   // timing-only builds (wrong results): 1 no sort, 2 no sums, 3 no message loads, 4 no keys
#endif
constexpr int kXwTileBits = 14;
constexpr int kXwTileMax = 1 << kXwTileBits;   // steps per sorted tile (the key's low bits)
constexpr int kXwBatch = 32;                 // sorted steps staged per pass (4 per wave)
constexpr int kXwThreads = 512;
constexpr int kXwWaves = kXwThreads / 64;
static_assert(kXwTileBits + kOpWideKeyBits <= 32, "packed sort key");

// the sorted tile's length: the group's stream rounded up to a power of two
__host__ __device__ inline int op_xi_tile(int T) {
  const long n = (long)kOpWideSeqs * T;
  int L = 64;
  while (L < n && L < kXwTileMax) L <<= 1;
  return L;
}

// a step's sort key c' << Lbits | code_j << lsh[j] (code: state, M missing,
// M + 1 out of range)
__device__ __forceinline__ int op_key(const OpWideArgs& a, const int32_t* o) {
  int k = (op_code(a, o) & (kOpEv - 1)) << a.Lbits;
  for (int j = 0; j < a.nleaf; j++) {
    const int v = o[a.lcol[j]], M = a.lcard[j];
    k |= (v < 0 ? M : (v < M ? v : M + 1)) << a.lsh[j];
  }
  return k;
}

// Per instantiation: batches in flight (register sets), step groups unrolled
// and the waves per SIMD the registers are held to.  At 16 states per tile
// pair and two slots per wave (NP = 32, TPW = 2: the 17..32-state case) one batch in flight keeps
// the kernel within 128 registers: two blocks, four waves per SIMD, which
// beats two batches in flight at one block per CU (5.73 -> 4.97 ms,
// profiles/r05/gpu/r05u_ab_estep_opchain_wide.txt); with the empty slots
// skipped, one step group per iteration (3.50 -> 3.29 ms, r05ai_*)
template <int NP, int TPW>
struct XiCfg {
  static constexpr int pipe = 2, gu = 2, wpe = 1;
};
template <>
struct XiCfg<32, 2> {
  static constexpr int pipe = 1, gu = 1, wpe = 4;
};

template <int NP, int TPW>
__global__ __launch_bounds__(kXwThreads) __attribute__((amdgpu_waves_per_eu(XiCfg<NP, TPW>::wpe))) void op_wide_xi_kernel(OpWideArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned key[];   // [op_xi_tile(T)]
  __shared__ double Ab[kXwBatch][NP], Gb[kXwBatch][NP], Gm[kXwBatch][NP];
  __shared__ int kb[kXwBatch];
  __shared__ double p0s[kOpWideSeqs][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = a.K, KK = K * K, T = a.T;
  const int L = op_xi_tile(T);
  const long b0 = (long)blockIdx.x * kOpWideSeqs;
  const int nseq = (int)((a.B - b0) < kOpWideSeqs ? (a.B - b0) : kOpWideSeqs);
  const int n = nseq * T;
  double* const out = a.slab + (size_t)blockIdx.x * a.xrow;
  // The sums on the matrix cores (v_mfma_f64_16x16x4, the steps as the inner
  // dimension, four per MFMA): Xi' tiles D[x][y] += sum_k A_k(x) G_k(y)
  // (NT x NT tiles of 16 x 16), the leaf count rows D[r][y] += sum_k
  // [code_j,k = r] gamma_k(y) (a one-hot A operand; RT_j x NT tiles per leaf).
  // Tile w + 8 i goes to wave w's accumulator i: the Xi' tiles first, then
  // the leaves' in leaf order.  An MFMA ignores EXEC, so steps outside a sum
  // enter as zero A operands, never by branching.
  constexpr int NT = NP / 16;
  int tkind[TPW], tx[TPW], ty[TPW], tj[TPW];      // kind 0 none, 1 Xi' (x tile, y tile), 2 leaf (j, row tile, y tile)
  const int wv = __builtin_amdgcn_readfirstlane(wave);   // (so that every tile parameter is wave-uniform)
#pragma unroll
  for (int i = 0; i < TPW; i++) {
    int ti = wv + kXwWaves * i;
    tkind[i] = 0; tx[i] = 0; ty[i] = 0; tj[i] = 0;
    if (ti < NT * NT) {
      tkind[i] = 1; tx[i] = ti / NT; ty[i] = ti % NT;
    } else {
      ti -= NT * NT;
      for (int j = 0; j < a.nleaf; j++) {
        const int rt = (a.lcard[j] + 2 + 15) / 16;
        if (tkind[i] == 0 && ti < rt * NT) { tkind[i] = 2; tj[i] = j; tx[i] = ti / NT; ty[i] = ti % NT; }
        ti -= rt * NT;
      }
    }
  }
  // a leaf tile's code field, row count and row offset (static-index copies:
  // an argument array indexed by a lane-varying value would live in scratch)
  int tsh[TPW], tmk[TPW], trows[TPW], thoff[TPW];
#pragma unroll
  for (int i = 0; i < TPW; i++) {
    tsh[i] = 0; tmk[i] = 0; trows[i] = 0; thoff[i] = 0;
#pragma unroll
    for (int j = 0; j < kOpMaxLeaf; j++)
      if (tkind[i] == 2 && tj[i] == j) {
        tsh[i] = a.lsh[j]; tmk[i] = (1 << a.lbits[j]) - 1; trows[i] = a.lcard[j] + 2; thoff[i] = a.hoff[j];
      }
  }
  v4d D[TPW];
#pragma unroll
  for (int i = 0; i < TPW; i++) D[i] = v4d{0.0, 0.0, 0.0, 0.0};
  int na = 0;                                      // slots with a tile (wave-uniform)
#pragma unroll
  for (int i = 0; i < TPW; i++) na += tkind[i] != 0;
  const int li = lane & 15, lk = lane >> 4;
  // the row's Xi' part zeroed by the lanes that own its cells (each cell is
  // later written, or read and written, by the same lane only)
  for (int c = 0; c <= a.oncomb; c++)
#pragma unroll
    for (int i = 0; i < TPW; i++)
      if (tkind[i] == 1)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int x = 16 * tx[i] + lk + 4 * r, yy = 16 * ty[i] + li;
          if (x < K && yy < K) out[(size_t)c * KK + x * K + yy] = 0.0;
        }
  int cur = -1;
  auto flush = [&](bool first) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TPW; i++)
      if (tkind[i] == 1) {
        if (cur >= 0)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int x = 16 * tx[i] + lk + 4 * r, yy = 16 * ty[i] + li;
            double* o = out + (size_t)cur * KK + x * K + yy;
            if (x < K && yy < K) *o = first ? D[i][r] : *o + D[i][r];
          }
        D[i] = v4d{0.0, 0.0, 0.0, 0.0};
      }
    cur = -1;
  };
  // the MFMAs of the batch's steps [k0, k1): Xi' tiles (xi) and / or leaf tiles (h)
  constexpr int GU = XiCfg<NP, TPW>::gu;              // step groups unrolled
  // Branch-free over the wave's tiles (every tile parameter is wave-uniform):
  // a group's operands are read for all of them first, then their MFMAs issue
  // back to back; a step outside [k0, k1) or a sum not asked for enters as a
  // zero A operand.
  // NA: the wave's slots that hold a tile (a prefix of its TPW slots); the
  // empty ones take no operands and no MFMAs
  auto mfma_pass_n = [&](int k0, int k1, bool xi, bool h, auto na_c) __attribute__((always_inline)) {
    constexpr int NA = decltype(na_c)::value;
#pragma unroll GU
    for (int g = 0; g < kXwBatch / 4; g++) {
      const int k = 4 * g + lk;
      const bool in = k >= k0 && k < k1;
      const int kc = kb[k];
      double av[NA], bv[NA];
#pragma unroll
      for (int i = 0; i < NA; i++) {
        const bool isx = tkind[i] == 1;
        const int col = 16 * ty[i] + li;
        const int xcol = min(16 * tx[i] + li, NP - 1);
        const double ax = Ab[k][xcol];
        bv[i] = isx ? Gb[k][col] : Gm[k][col];
        const int r = (kc >> tsh[i]) & tmk[i];
        const bool hot = r == 16 * tx[i] + li;
        av[i] = in ? (isx ? (xi ? ax : 0.0) : (h && hot ? 1.0 : 0.0)) : 0.0;
      }
      // every held slot's MFMA issues: no lane-varying branch around a
      // matrix instruction
#pragma unroll
      for (int i = 0; i < NA; i++) D[i] = mfma(av[i], bv[i], D[i]);
    }
  };
#define NIPAMD_XI_NA(n)                                                        \
  if constexpr (TPW >= n)                                                      \
    if (na == n) {                                                             \
      mfma_pass_n(k0, k1, xi, h, std::integral_constant<int, n>{});            \
      return;                                                                  \
    }
  auto mfma_pass = [&](int k0, int k1, bool xi, bool h) __attribute__((always_inline)) {
    NIPAMD_XI_NA(1) NIPAMD_XI_NA(2) NIPAMD_XI_NA(3) NIPAMD_XI_NA(4) NIPAMD_XI_NA(5) NIPAMD_XI_NA(6)
  };
#undef NIPAMD_XI_NA
  constexpr int SPW = 64 / NP;
  const int y = lane % NP;
  const bool ys = y < K;
#ifndef NIPAMD_XI_STAMPS
#define NIPAMD_XI_STAMPS 0   // timing builds: block 0 prints its phase cycles (keys, sort, sums)
#endif
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  for (int i0 = 0; i0 < n; i0 += L) {
    const int m = (n - i0) < L ? (n - i0) : L;
    if (NIPAMD_XI_STAMPS) st0 = __builtin_readcyclecounter();
    for (int i = tid; i < L; i += kXwThreads) {
      unsigned v = 0xFFFFFFFFu;                       // padding sorts last
      if (i < m) {
        const int g = i0 + i, s = g / T, t = g - s * T;
        const int c = (a.obs && NIPAMD_XI_SKIP != 4) ? op_key(a, a.obs + (b0 + s) * a.obs_bstride + (long)t * a.obs_tstride) : 0;
        v = ((unsigned)c << kXwTileBits) | (unsigned)i;
      }
      key[i] = v;
    }
    __syncthreads();
    if (NIPAMD_XI_STAMPS) st1 = __builtin_readcyclecounter();
    for (int k2 = 2; k2 <= (NIPAMD_XI_SKIP == 1 ? 1 : L); k2 <<= 1)
      for (int j = k2 >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < L; i += kXwThreads) {
          const int p = i ^ j;
          if (p > i) {
            const unsigned u = key[i], w = key[p];
            if ((u > w) == ((i & k2) == 0)) { key[i] = w; key[p] = u; }
          }
        }
        __syncthreads();
      }
    if (NIPAMD_XI_STAMPS) st2 = __builtin_readcyclecounter();
    // Staging, software-pipelined: the next batch's loads (messages, scale
    // exponent, leaf factors -- all addressed from the sorted key alone) are
    // issued before this batch's sums and land in LDS after them (XiCfg::pipe
    // batches in flight).  Wave w
    // stages slots SL_w .. SL_w + SL - 1, 64 / NP per pass.
    constexpr int SL = kXwBatch / kXwWaves / SPW;
    // two batches in flight: the one in LDS is summed while the next one's
    // loads land in one register set and the one after that is issued into
    // the other (the random-order message reads are latency-bound)
    // (register sets indexed by a compile-time buffer number: a struct passed
    // by reference would live in scratch)
    constexpr int NPB = XiCfg<NP, TPW>::pipe;
    double P_at[NPB][SL], P_bt[NPB][SL], P_ap[NPB][SL], P_e[NPB][SL];
    int P_sc[NPB][SL], P_kc[NPB][SL];              // P_kc: the key's code, -1 past the tile's end
    auto load_batch = [&](int j0, auto buf) __attribute__((always_inline)) {
      constexpr int u = decltype(buf)::value;
#pragma unroll
      for (int q = 0; q < SL; q++) {
        const int jj = wave * (kXwBatch / kXwWaves) + q * SPW + lane / NP;
        const int j = j0 + jj;
        const bool ok = j < m;
        const unsigned v = key[ok ? j : 0];
        const int g = i0 + (int)(v & (kXwTileMax - 1)), s = g / T, t = g - s * T;
        const long b = b0 + s;
        const double* sa = a.Sa + ((size_t)b * T + t) * NP + y;
        const double* sb = a.Sb + ((size_t)b * T + t) * NP + y;
        const bool on = ok && ys && NIPAMD_XI_SKIP != 3;
        P_at[u][q] = on ? sa[0] : 0.0;
        P_bt[u][q] = on ? sb[0] : 0.0;
        P_ap[u][q] = on ? (t > 0 ? sa[-NP] : a.pi[y]) : 0.0;
        P_sc[u][q] = ok ? a.sc[(size_t)b * T + t] : 0;
        const int kc = (int)(v >> kXwTileBits);
        P_kc[u][q] = ok ? kc : -1;
        // the leaf factors from the key's codes (no observation re-read), in
        // op_leaf_e's order
        double e = 1.0;
#pragma unroll
        for (int q2 = 0; q2 < kOpMaxLeaf; q2++)
          if (q2 < a.nleaf)
            e *= a.ltab[a.loff[q2] + ((kc >> a.lsh[q2]) & ((1 << a.lbits[q2]) - 1)) * K + (ys ? y : 0)];
        P_e[u][q] = e;
      }
    };
    auto store_batch = [&](auto buf) __attribute__((always_inline)) {
      constexpr int u = decltype(buf)::value;
#pragma unroll
      for (int q = 0; q < SL; q++) {
        const int jj = wave * (kXwBatch / kXwWaves) + q * SPW + lane / NP;
        const double pr = P_at[u][q] * P_bt[u][q];
        const double z = group_sum<NP>(pr);
        const double rz = z != 0.0 ? 1.0 / z : 0.0;
        Ab[jj][y] = P_ap[u][q];
        Gb[jj][y] = P_bt[u][q] * P_e[u][q] * __builtin_ldexp(rz, P_sc[u][q]);
        Gm[jj][y] = pr * rz;
        if (y == 0) kb[jj] = P_kc[u][q];
      }
    };
    auto accumulate = [&](int j0) __attribute__((always_inline)) {
      const int nj = (m - j0) < kXwBatch ? (m - j0) : kXwBatch;
      if (NIPAMD_XI_SKIP == 2) return;
      const int cl = kb[nj - 1] >> a.Lbits;
      if ((kb[0] >> a.Lbits) == cl) {
        // one operator index over the batch (the common case: runs are long)
        if (cl != cur) { flush(i0 == 0); cur = cl; }
        mfma_pass(0, nj, true, true);
        return;
      }
      mfma_pass(0, nj, false, true);
      int k0 = 0;
      while (k0 < nj) {
        const int c = kb[k0] >> a.Lbits;
        int k1 = k0 + 1;
        while (k1 < nj && (kb[k1] >> a.Lbits) == c) k1++;
        if (c != cur) { flush(i0 == 0); cur = c; }
        mfma_pass(k0, k1, true, false);
        k0 = k1;
      }
    };
    // a barrier that waits for LDS only: __syncthreads() also waits for every
    // outstanding global load (s_waitcnt vmcnt(0)), which would drain the
    // next batches' prefetches at every hand-over
    auto lds_barrier = [] __attribute__((always_inline)) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    const std::integral_constant<int, 0> pa{};
    const std::integral_constant<int, 1> pb{};
    if constexpr (NPB == 1) {
      // one batch in flight: its loads are issued before the batch in LDS is summed
      load_batch(0, pa);
      unsigned long long cs = 0, cb1 = 0, cl = 0, ca = 0, cb2 = 0, tq = 0;
      auto lap = [&](unsigned long long& acc) __attribute__((always_inline)) {
        if (NIPAMD_XI_STAMPS) {
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          const unsigned long long t = __builtin_readcyclecounter();
          acc += t - tq;
          tq = t;
        }
      };
      if (NIPAMD_XI_STAMPS) tq = __builtin_readcyclecounter();
      for (int j0 = 0; j0 < m; j0 += kXwBatch) {
        store_batch(pa);
        lap(cs);
        lds_barrier();
        lap(cb1);
        if (j0 + kXwBatch < m) load_batch(j0 + kXwBatch, pa);
        if (NIPAMD_XI_STAMPS == 2) lap(cl);
        accumulate(j0);
        lap(ca);
        lds_barrier();
        lap(cb2);
      }
      if (NIPAMD_XI_STAMPS && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2) && lane == 0)
        printf("[xi] block %d wave %d: store %llu bar1 %llu loads %llu accum %llu bar2 %llu\n", (int)blockIdx.x, wave,
               cs, cb1, cl, ca, cb2);
    } else {
      load_batch(0, pa);
      store_batch(pa);
      if (kXwBatch < m) load_batch(kXwBatch, pa);
      for (int j0 = 0; j0 < m; j0 += 2 * kXwBatch) {
        // batch j0 in LDS, batch j0 + 32 in register set 0
        lds_barrier();
        if (j0 + 2 * kXwBatch < m) load_batch(j0 + 2 * kXwBatch, pb);
        accumulate(j0);
        lds_barrier();
        if (j0 + kXwBatch >= m) break;
        store_batch(pa);
        // batch j0 + 32 in LDS, batch j0 + 64 in register set 1
        lds_barrier();
        if (j0 + 3 * kXwBatch < m) load_batch(j0 + 3 * kXwBatch, pa);
        accumulate(j0 + kXwBatch);
        lds_barrier();
        if (j0 + 2 * kXwBatch < m) store_batch(pb);
      }
    }
    flush(i0 == 0);
    if (NIPAMD_XI_STAMPS) {
      st3 = __builtin_readcyclecounter();
      if ((blockIdx.x == 0 || blockIdx.x == gridDim.x / 2) && tid == 0)
        printf("[xi] block %d tile %d: keys %llu sort %llu sums %llu cycles (m %d)\n", (int)blockIdx.x, i0 / L,
               st1 - st0, st2 - st1, st3 - st2, m);
    }
  }
  // P0 per sequence: normalise(prior o T_{c_0} (e_0 o beta^_0)), as op_fb_kernel's
  // extra backward step; then summed over the group in sequence order
  for (int s = wave; s < nseq; s += kXwWaves) {
    const long b = b0 + s;
    const int32_t* o0 = a.obs ? a.obs + b * a.obs_bstride : nullptr;
    const int c0 = o0 ? (op_code(a, o0) & (kOpEv - 1)) : 0;
    const double* Tc = a.Ttab + (size_t)c0 * KK;
    const double* bz = a.Sb + (size_t)b * T * NP;
    const bool xs = lane < K;
    double u = 0.0;
    if (xs)
      for (int k = 0; k < K; k++)
        u = __builtin_fma(Tc[lane * K + k], (o0 && a.nleaf ? op_leaf_e(a, o0, k) : 1.0) * bz[k], u);
    const double pr = xs ? a.pi[lane] * u : 0.0;
    const double z = group_sum<64>(pr);
    p0s[s][lane] = z != 0.0 ? pr / z : pr;
  }
  __syncthreads();
  if (tid < K) {
    double p = 0.0;
    for (int s = 0; s < nseq; s++) p += p0s[s][tid];
    out[a.xrow - K + tid] = p;
  }
#pragma unroll
  for (int i = 0; i < TPW; i++)
    if (tkind[i] == 2)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * tx[i] + lk + 4 * r, yy = 16 * ty[i] + li;
        if (row < trows[i] && yy < K) out[(size_t)thoff[i] + row * K + yy] = D[i][r];
      }
}

}  // namespace

// the operators in LDS (padded rows) while two blocks per CU still fit
constexpr size_t kOpWideTl = 80 * 1024;

template <int NP>
int msgs_launch(const OpWideArgs& a, hipStream_t stream) {
  const int spb = MsgCfg<NP>::waves * (64 / NP);
  const int nbd = (int)((a.B + spb - 1) / spb);
  const dim3 g((unsigned)(a.filter ? nbd : 2 * nbd)), th(MsgCfg<NP>::waves * 64);
  const size_t tl = (size_t)op_lds_doubles(a.oncomb, a.K, NP) * sizeof(double);
  if (tl <= kOpWideTl) {
    static size_t set[kMaxDevices] = {};
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&op_wide_msgs_kernel<NP, true>), tl, set)) return rc;
    hipLaunchKernelGGL((op_wide_msgs_kernel<NP, true>), g, th, tl, stream, a);
  } else {
    hipLaunchKernelGGL((op_wide_msgs_kernel<NP, false>), g, th, 0, stream, a);
  }
  if (a.post) {
    const long prow = (a.B * a.T + 4 * (64 / NP) - 1) / (4 * (64 / NP));
    hipLaunchKernelGGL(op_wide_post_kernel<NP>, dim3((unsigned)prow), dim3(256), 0, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int op_wide_launch(const OpWideArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  if (a.K > 64 || a.K < 1 || a.nleaf > kOpMaxLeaf) return -2;
  g_last_kernel = "op_wide_msgs_kernel + op_wide_post_kernel";
  return op_wide_np(a.K) == 32 ? msgs_launch<32>(a, stream) : msgs_launch<64>(a, stream);
}

template <int NP, int TPW>
int xi_launch_t(const OpWideArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)op_xi_tile(a.T) * sizeof(unsigned);
  static size_t set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&op_wide_xi_kernel<NP, TPW>), lds, set)) return rc;
  const dim3 g((unsigned)((a.B + kOpWideSeqs - 1) / kOpWideSeqs)), th(kXwThreads);
  hipLaunchKernelGGL((op_wide_xi_kernel<NP, TPW>), g, th, lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// accumulator slots per wave: the NT^2 Xi' tiles and the leaves' tiles over
// the block's waves (an empty slot costs an MFMA on zeros)
template <int NP>
int xi_launch(const OpWideArgs& a, hipStream_t stream) {
  constexpr int NT = NP / 16;
  int tiles = NT * NT;
  for (int j = 0; j < a.nleaf; j++) tiles += (a.lcard[j] + 2 + 15) / 16 * NT;
  if (tiles <= 2 * kXwWaves) return xi_launch_t<NP, 2>(a, stream);
  if (tiles <= 4 * kXwWaves) return xi_launch_t<NP, 4>(a, stream);
  if constexpr (NP == 64) {
    if (tiles <= 6 * kXwWaves) return xi_launch_t<NP, 6>(a, stream);
  }
  return -2;
}

int op_wide_xi_launch(const OpWideArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  if (a.K > 64 || a.K < 17 || a.oncomb > 65534 || !a.sc || !a.slab || a.Lbits < 0 ||
      ((long)(a.oncomb + 1) << a.Lbits) > (1L << kOpWideKeyBits) ||
      a.xrow - a.K - (a.oncomb + 1) * a.K * a.K > kOpWideMaxH || (long)kOpWideSeqs * a.T >= (1L << 31))
    return -2;
  return op_wide_np(a.K) == 32 ? xi_launch<32>(a, stream) : xi_launch<64>(a, stream);
}

int estep_wide_np(int N) { return N <= 16 ? 16 : N <= 32 ? 32 : N <= 64 ? 64 : 0; }

// the slab row's size (doubles): K [NP][NP], H [R][NP], P0 [NP]
int estep_wide_slab(int N, int R) {
  const int NP = estep_wide_np(N);
  return NP * NP + R * NP + NP;
}

bool estep_wide_fits(int N, int R) {
  const int NP = estep_wide_np(N);
  const int hr = (R + 15) / 16;
  return NP != 0 && (NP <= 32 ? hr <= 8 : hr <= 2);
}

size_t estep_wide_scratch_bytes(int N, long B, int T) {
  const int NP = estep_wide_np(N);
  return (size_t)B * (2 * (size_t)T + 1) * NP * sizeof(double) + (size_t)B * T * sizeof(int) + 256;
}

int estep_wide_launch(const EWideArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  const int NP = estep_wide_np(a.N);
  if (!estep_wide_fits(a.N, a.R) || a.nchild > 4 || a.ncol > 4) return -2;
  {
    const int spb = kMsgWaves / 2 * (64 / NP);
    const int blocks = (int)((a.B + spb - 1) / spb);
    const dim3 g(blocks), th(kMsgWaves * 64);
    if (a.proper) {
      if (NP == 16) hipLaunchKernelGGL((chain_msgs_kernel<16, true>), g, th, 0, stream, a);
      else if (NP == 32) hipLaunchKernelGGL((chain_msgs_kernel<32, true>), g, th, 0, stream, a);
      else hipLaunchKernelGGL((chain_msgs_kernel<64, true>), g, th, 0, stream, a);
    } else {
      if (NP == 16) hipLaunchKernelGGL((chain_msgs_kernel<16, false>), g, th, 0, stream, a);
      else if (NP == 32) hipLaunchKernelGGL((chain_msgs_kernel<32, false>), g, th, 0, stream, a);
      else hipLaunchKernelGGL((chain_msgs_kernel<64, false>), g, th, 0, stream, a);
    }
    if (hipGetLastError() != hipSuccess) return -1;
  }
  g_last_kernel = "chain_msgs_kernel + chain_stats_kernel";
  if (NP == 16) return stats_launch<1, 8>(a, stream);
  if (NP == 32) return stats_launch<2, 8>(a, stream);
  return stats_launch<4, 2>(a, stream);
}

}  // namespace nipamd
