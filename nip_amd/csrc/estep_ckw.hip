// estep_ckw.hip -- the checkpoint + recompute e_step (estep_ck.hip) for
// interface chains of 17..32 states with up to two observed leaf children,
// any unobserved children and hidden independent parents: SURVEY 8(d)
// config 3's model (demo1 @ 32 states, A1 and B1 observed, D1 hidden).
// Round 6, VERDICT r05 item 2.
//
// The same scheme as estep_ck.hip at two 16-state tiles (NT = 2): a wave owns
// 16 sequences and runs the forward pass (every 4th message to HBM as a
// checkpoint), then the backward pass in chunks of four steps with the
// chunk's other messages recomputed from the checkpoint below it, the
// backward message kept normalised against the forward one (beta~, no
// normaliser), and the three sums of the reference's families
// (src/nip.c:1925-1967; DESIGN.md 4, estep_wide.hip):
//   K(x, y) = sum_t alpha_{t-1}(x) e_t(y) beta_t(y) / Z   (alpha_{-1} = prior)
//   H[r][y] = sum_t [r = row of child k's code at t] gamma_t(y)
//   P0(x)   = gamma_{-1}(x)
// into the wide slab row of estep_mw.hip (K [32][32], H [R][32], P0 [32]),
// which tree64_kernel and the CSR map finalize turn into every family's
// counts.  K is sixteen v_mfma_f64_16x16x4 per step (two by two tiles, K =
// the wave's sequences, after an LDS transpose).  The count rows take one LDS
// add per sequence and step: lanes 0-31 the state y of column 0's row, lanes
// 32-63 column 1's -- no two lanes of an instruction share a cell, a wave's
// LDS operations execute in program order, so each cell sums in a fixed
// order.  The unobserved children's missing rows (every step's gamma) are
// register sums.
//
// One wave per SIMD: at 32 states a step's mat-vec is sixteen MFMAs in two
// independent accumulation chains, which keep the matrix pipe ~90% busy even
// alone (profiles/r03/r03_mb_lat.txt V3); the 4-wave block's LDS (two
// evidence tables, per wave a 69 x 32 count table and three transposes)
// leaves room for one block per CU.
#include "chain_mfma_core.h"
#include "store_pol.h"

#include <type_traits>

namespace nipamd {

namespace {

constexpr int kWWaves = 4;                     // waves per block; a wave owns 16 sequences
constexpr int kWThreads = 64 * kWWaves;
constexpr int NT = 2, NP = 32;                 // state tiles, states per sequence row
constexpr int NPS = NP + 2;                    // LDS table / transpose row stride (doubles)
constexpr int kXD = 16 * NPS;                  // one transpose buffer [16 sequences][NPS]
constexpr int kMaxCol = 2;

// per-wave LDS (doubles): the count table [rows][NP] (observed columns' rows,
// then one dummy row for the unused half of a single-column add), three
// transposes (alpha^_{t-1}, w_t, gamma_t), the chunk's count-row offsets
// [4 steps][2 halves][16 sequences] ints
__host__ __device__ inline int ckw_wave_doubles(int rows) { return (rows + 1) * NP + 3 * kXD + 64; }
__host__ __device__ inline int ckw_tab_doubles(int tab_rows) { return (tab_rows * NPS + 1) & ~1; }
__host__ __device__ inline int ckw_count(int T) { return (T + 3) >> 2; }
// checkpoints per group: [nck][16][32] doubles, then [nck][16] int exponents
__host__ __device__ inline long ckw_group_doubles(int T) { return (long)ckw_count(T) * (16 * NP + 8); }

__device__ __forceinline__ unsigned byte_of4(unsigned w, int k) { return (w >> (8 * k)) & 0xFFu; }

__device__ __forceinline__ v4d mfma1(double a, double b, v4d d) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
}

// the mat-vec of the fb kernels at NT = 2 (chain_mfma_wide.hip): d[qo] =
// sum over the input tiles qi; the two output tiles' chains interleaved
__device__ __forceinline__ void matvec2(const double (&Aop)[NT][NT][4], const v4d (&X)[NT], v4d (&d)[NT]) {
  d[0] = v4d{0.0, 0.0, 0.0, 0.0};
  d[1] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int qi = 0; qi < NT; qi++) {
    d[0] = mfma1(Aop[0][qi][0], X[qi].x, d[0]);
    d[1] = mfma1(Aop[1][qi][0], X[qi].x, d[1]);
    d[0] = mfma1(Aop[0][qi][1], X[qi].y, d[0]);
    d[1] = mfma1(Aop[1][qi][1], X[qi].y, d[1]);
    d[0] = mfma1(Aop[0][qi][2], X[qi].z, d[0]);
    d[1] = mfma1(Aop[1][qi][2], X[qi].z, d[1]);
    d[0] = mfma1(Aop[0][qi][3], X[qi].w, d[0]);
    d[1] = mfma1(Aop[1][qi][3], X[qi].w, d[1]);
  }
}

// matvec2 with the operands read from LDS ([qo][qi][r][lane] doubles, the
// block's copy: every wave's lane l holds the same A entries)
__device__ __forceinline__ void matvec2_lds(const double* Al, int lane, const v4d (&X)[NT], v4d (&d)[NT]) {
  double Aop[NT][NT][4];
#pragma unroll
  for (int qo = 0; qo < NT; qo++)
#pragma unroll
    for (int qi = 0; qi < NT; qi++)
#pragma unroll
      for (int r = 0; r < 4; r++) Aop[qo][qi][r] = Al[((qo * NT + qi) * 4 + r) * 64 + lane];
  matvec2(Aop, X, d);
}

// sum of a sequence's 32 states (its two tiles in the sequence's 4 lanes)
__device__ __forceinline__ double seq_sum(const v4d (&v)[NT]) {
  return sum_lanes16(sum_lanes32(((v[0].x + v[0].y) + (v[0].z + v[0].w)) + ((v[1].x + v[1].y) + (v[1].z + v[1].w))));
}

// transpose row j (16 sequences x NPS doubles): filter layout (lane (g, j):
// tile q's states 16q + 2g, 2g+1 and 16q + 2g+8, 2g+9) -> row j; rows 34
// doubles apart, so the 16 lanes of one piece write 64 different banks
__device__ __forceinline__ void tp_write2(double* buf, int j, int g, const v4d (&v)[NT]) {
#pragma unroll
  for (int q = 0; q < NT; q++) {
    *reinterpret_cast<v2d*>(buf + j * NPS + 16 * q + 2 * g) = v2d{v[q].x, v[q].y};
    *reinterpret_cast<v2d*>(buf + j * NPS + 16 * q + 2 * g + 8) = v2d{v[q].z, v[q].w};
  }
}
// sequence-major: lane l gets state 16 xt + (l & 15) of sequence 4q + (l >> 4):
// r[xt][q], the operands of the tile's v_mfma_f64_16x16x4 q
__device__ __forceinline__ void tp_read2(const double* buf, int lane, double (&r)[NT][4]) {
  const int y = lane & 15, k = lane >> 4;
#pragma unroll
  for (int xt = 0; xt < NT; xt++)
#pragma unroll
    for (int q = 0; q < 4; q++) r[xt][q] = buf[(4 * q + k) * NPS + 16 * xt + y];
}

// POST: forward_backward_inference's smoothed interface posteriors instead of
// the e_step's sums (the backward pass writes gamma_t, normalised exactly, and
// keeps no transposes, count tables or xi accumulators)
// VL (POST only): the chunk's recomputed messages in LDS, not registers
// ([3 slots][4 pieces][64 lanes] 16-byte pieces per wave, 12 KB): the wave
// fits 256 registers and two of them share a SIMD (eight waves per block)
template <int PR, int NC, bool POST, bool VL = false>
__global__ __launch_bounds__(VL ? 512 : kWThreads, 1) void chain_estep_ckw_kernel(EMwArgs a) {
  static_assert(POST || !VL, "messages in LDS: the posterior mode only");
  constexpr int WV = VL ? 8 : kWWaves, WT = 64 * WV;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = a.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // count-table rows of the observed columns: column c's M_c + 2 rows (its
  // states, missing, out of range) from cro[c]
  int cro[kMaxCol], crows = 0;
#pragma unroll
  for (int c = 0; c < kMaxCol; c++) {
    cro[c] = crows;
    crows += c < a.ncol ? a.M[c] + 2 : 0;
  }
  double* tab = reinterpret_cast<double*>(smem);                               // [tab_rows][NPS]
  // VL: the block's copy of the forward operands (the backward pass's
  // recomputation reads them from LDS: 32 registers fewer), then the waves'
  double* const AfL = tab + ckw_tab_doubles(a.tab_rows);                    // VL: [2][2][4][64]
  double* wl = AfL + (VL ? NT * NT * 4 * 64 : 0) + (size_t)wave * (VL ? 3 * 512 : ckw_wave_doubles(crows));
  double* const Vl = wl;                                                     // VL: [3][4][64] v2d
  double* Hl = wl;                                                           // [crows + 1][NP]
  double* XA = Hl + (crows + 1) * NP;
  double* XW = XA + kXD;
  double* XG = XW + kXD;
  int* AD = reinterpret_cast<int*>(XG + kXD);                                // [4][2][16]

  for (int i = tid; i < a.tab_rows * NP; i += WT) tab[(i / NP) * NPS + i % NP] = a.tab[i];
  if constexpr (VL)
    for (int i = tid; i < NT * NT * 4 * 64; i += WT) {
      const int l = i & 63, r = (i >> 6) & 3, qi = (i >> 8) & 1, qo = i >> 9;
      const int gl = l >> 4, jl = l & 15;
      AfL[i] = a.A[(16 * qi + state_of(gl, r)) * 64 + 16 * qo + state_of(jl & 3, jl >> 2)];
    }
  if constexpr (!POST)
    for (int i = lane; i < (crows + 1) * NP; i += 64) Hl[i] = 0.0;
  __syncthreads();                                                           // the block's only barrier

  const long grp = (long)blockIdx.x * WV + wave;
  const long b0 = grp * 16;
  if (b0 >= a.B) return;
  const int j = lane & 15, g = lane >> 4;
  const int sj = state_of(j & 3, j >> 2);
  const bool active = b0 + j < a.B;
  const int* orow = a.obs + (active ? (b0 + j) * a.obs_bstride : 0);      // the launcher requires obs
  const int nck = ckw_count(T);
  double* Sg = a.S + (size_t)grp * ckw_group_doubles(T);                     // [nck][16][32]
  int* Xg = reinterpret_cast<int*>(Sg + (size_t)nck * 16 * NP);              // [nck][16]

  // the chunk's raw codes (per column: four int32 steps; steps past T and
  // sequences past B select missing where they are packed, a chunk later)
  struct Raw {
    int v[NC][4];
  };
  auto codes_raw = [&](int c) -> Raw {
    Raw r;
    const int t0 = 4 * c;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int t = t0 + k < 0 ? 0 : (t0 + k > T - 1 ? T - 1 : t0 + k);
#pragma unroll
      for (int q = 0; q < NC; q++) r.v[q][k] = orow[(long)t * a.obs_tstride + a.col[q]];
    }
    return r;
  };
  // packed: byte k of word q = column q's table row at step 4c + k
  auto codes_pack = [&](const Raw& r, int c, unsigned (&w)[NC]) {
    const int t0 = 4 * c;
#pragma unroll
    for (int q = 0; q < NC; q++) {
      const int M = a.ncol > 0 ? a.M[q] : 0;
      unsigned x = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const bool in = active && t0 + k >= 0 && t0 + k < T;
        const int o = in ? r.v[q][k] : -1;
        const int cd = o < 0 ? M : (o < M ? o : M + 1);
        x |= (unsigned)cd << (8 * k);
      }
      w[q] = x;
    }
  };
  int toff[NC];
#pragma unroll
  for (int q = 0; q < NC; q++) toff[q] = (a.tab_off[q] / NP) * NPS + 2 * g;
  // evidence of step k: the product of the columns' rows (column 0's table
  // carries the unobserved children's row sums)
  auto evid = [&](const unsigned (&w)[NC], int k, v4d (&e)[NT]) {
#pragma unroll
    for (int q = 0; q < NT; q++) e[q] = load4(tab + toff[0] + (int)byte_of4(w[0], k) * NPS + 16 * q);
#pragma unroll
    for (int c = 1; c < NC; c++)
#pragma unroll
      for (int q = 0; q < NT; q++) e[q] *= load4(tab + toff[c] + (int)byte_of4(w[c], k) * NPS + 16 * q);
  };

  double Af[NT][NT][4], Ab[NT][NT][4];
#pragma unroll
  for (int qo = 0; qo < NT; qo++)
#pragma unroll
    for (int qi = 0; qi < NT; qi++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int out = 16 * qo + sj, in = 16 * qi + state_of(g, r);
        Af[qo][qi][r] = a.A[in * 64 + out];
        Ab[qo][qi][r] = a.A[out * 64 + in];
      }
  const v4d zero = {0.0, 0.0, 0.0, 0.0};
  // the prior and s_all (the evidence of a step that observes nothing: every
  // column at its missing row, in the evidence's own product order) are read
  // where used: registers are the budget at 32 states
  auto prior = [&](v4d (&p)[NT]) {
#pragma unroll
    for (int q = 0; q < NT; q++) p[q] = active ? load4(a.pi + 16 * q + 2 * g) : zero;
  };
  unsigned wmiss[NC];
#pragma unroll
  for (int q = 0; q < NC; q++) wmiss[q] = 0x01010101u * (unsigned)(a.ncol > 0 ? a.M[q] : 0);
  auto ck_store = [&](int slot, const v4d (&p)[NT], int e) {
    double* s = Sg + (size_t)slot * 16 * NP + j * NP + 2 * g;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      store_pol<false>(reinterpret_cast<v2d*>(s + 16 * q), v2d{p[q].x, p[q].y});
      store_pol<false>(reinterpret_cast<v2d*>(s + 16 * q + 8), v2d{p[q].z, p[q].w});
    }
    if (g == 0) Xg[slot * 16 + j] = e;
  };

  // ---------------------------------------------------------------- forward
  v4d X[NT];
  prior(X);
  int Ef = 0;
  double m2 = 1.0, m1 = 1.0;
  int e2 = 0, e1 = 0;
  bool dead = false;
  auto renorm = [](double& m, int& e) {
    const int k = __builtin_amdgcn_frexp_exp(m);
    m = __builtin_ldexp(m, -k);
    e += k;
  };
  v4d srow[NT];                                  // s_all on this lane's states (live in the forward pass only)
  evid(wmiss, 0, srow);
  auto fstep = [&](const v4d (&e)[NT], bool rescale, int slot) {
    v4d u[NT];
    matvec2(Af, X, u);
    v4d p[NT];
#pragma unroll
    for (int q = 0; q < NT; q++) p[q] = u[q] * e[q];
    double z = 0.0;
    if (!PR) {
      z = seq_sum(p);
      v4d us[NT];
#pragma unroll
      for (int q = 0; q < NT; q++) us[q] = u[q] * srow[q];
      m2 *= z;
      m1 *= seq_sum(us);
      renorm(m2, e2);
      renorm(m1, e1);
      dead |= z == 0.0;
    }
    if (rescale) {
      if (PR) z = seq_sum(p);
      const int sc = -__builtin_amdgcn_frexp_exp(z);
#pragma unroll
      for (int q = 0; q < NT; q++) p[q] = ldexp4(p[q], sc);
      Ef += sc;
      ck_store(slot, p, Ef);
    }
#pragma unroll
    for (int q = 0; q < NT; q++) X[q] = p[q];
  };
  {
    auto fchunk = [&](int c, Raw& wr) {
      unsigned w[NC];
      codes_pack(wr, c, w);
      wr = codes_raw(c + 2);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        v4d e[NT];
        evid(w, k, e);
        fstep(e, k == 3, c);
      }
    };
    Raw wA = codes_raw(0), wB = codes_raw(1);
    const int nfull = T >> 2;
    int c = 0;
    for (; c + 2 <= nfull; c += 2) {
      fchunk(c, wA);
      fchunk(c + 1, wB);
    }
    if (c < nfull) fchunk(c++, wA);
    unsigned wl[NC];
    codes_pack((nfull & 1) ? wB : wA, nfull, wl);
    for (int t = nfull * 4; t < T; t++) {
      v4d e[NT];
      evid(wl, t & 3, e);
      fstep(e, false, 0);
    }
  }
  if (PR) {
    const double zT = seq_sum(X);
    dead = zT == 0.0;
    if (active && g == 0) {
      const double ll = dead ? -DBL_MAX : log(zT) - (double)Ef * 0.69314718055994530942;
      if (a.ll) a.ll[b0 + j] = ll;
      if (a.status) a.status[b0 + j] = dead ? (POST ? 1u : 3u) : 0u;
    }
  } else if (active && g == 0) {
    double ll = log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
    const bool dd = dead || m2 == 0.0;
    if (dd) ll = -DBL_MAX;
    if (a.ll) a.ll[b0 + j] = ll;
    if (a.status) a.status[b0 + j] = dd ? (POST ? 1u : 3u) : 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");

  // --------------------------------------------------------------- backward
  // Chunk c (steps 4c..4c+3) needs the checkpoints c (message 4c+3), c - 1
  // (4c-1: the chunk's first previous message) and c - 2 (the start of chunk
  // c - 1's recomputation); a chunk passes the last two down and loads one,
  // checkpoint c - 3, with chunk c - 2's raw codes: issued at the chunk's
  // start, consumed (converted) at its end.
  struct CkRaw {
    v2d p[NT][2];
    int e;
  };
  auto ck_raw = [&](int k) -> CkRaw {
    const int kc = k < 0 ? 0 : k;
    const double* s = Sg + (size_t)kc * 16 * NP + j * NP + 2 * g;
    CkRaw r;
#pragma unroll
    for (int q = 0; q < NT; q++) {
      r.p[q][0] = *reinterpret_cast<const v2d*>(s + 16 * q);
      r.p[q][1] = *reinterpret_cast<const v2d*>(s + 16 * q + 8);
    }
    r.e = Xg[kc * 16 + j];
    return r;
  };
  // checkpoint k's message (the prior below step 0) and exponent
  auto ck_val = [&](const CkRaw& r, int k, v4d (&v)[NT], int& e) {
    if (k < 0) {
      prior(v);
      e = 0;
      return;
    }
#pragma unroll
    for (int q = 0; q < NT; q++) v[q] = v4d{r.p[q][0].x, r.p[q][0].y, r.p[q][1].x, r.p[q][1].y};
    e = r.e;
  };

  const int ctop = (T - 1) >> 2;
  // beta~_{T-1} = 1 / z_T on the real states (estep_ck.hip)
  const double rz = recip(seq_sum(X));
  v4d Bt[NT];
#pragma unroll
  for (int q = 0; q < NT; q++) {
    Bt[q].x = 16 * q + state_of(g, 0) < a.N ? rz : 0.0;
    Bt[q].y = 16 * q + state_of(g, 1) < a.N ? rz : 0.0;
    Bt[q].z = 16 * q + state_of(g, 2) < a.N ? rz : 0.0;
    Bt[q].w = 16 * q + state_of(g, 3) < a.N ? rz : 0.0;
  }
  v4d Kd[NT][NT];
#pragma unroll
  for (int xt = 0; xt < NT; xt++)
#pragma unroll
    for (int yt = 0; yt < NT; yt++) Kd[xt][yt] = zero;
  // count adds: lane half h = lane >> 5 takes column h's row (a dummy row
  // past the table when the request has one column), state lane & 31
  const int ch = lane >> 5, cy = lane & 31;
  auto recomp = [&](v4d (&x)[NT], const v4d (&e)[NT]) {
    v4d u[NT];
    if constexpr (VL) matvec2_lds(AfL, lane, x, u);
    else matvec2(Af, x, u);
#pragma unroll
    for (int q = 0; q < NT; q++) x[q] = u[q] * e[q];
  };

  // VL: slot s of the wave's message buffer
  auto vstore = [&](int sl, const v4d (&m)[NT]) {
    v2d* v = reinterpret_cast<v2d*>(Vl + sl * 512) + lane;
    v[0] = v2d{m[0].x, m[0].y};
    v[64] = v2d{m[0].z, m[0].w};
    v[128] = v2d{m[1].x, m[1].y};
    v[192] = v2d{m[1].z, m[1].w};
  };
  auto vload = [&](int sl, v4d (&m)[NT]) {
    const v2d* v = reinterpret_cast<const v2d*>(Vl + sl * 512) + lane;
    const v2d p0 = v[0], p1 = v[64], p2 = v[128], p3 = v[192];
    m[0] = v4d{p0.x, p0.y, p1.x, p1.y};
    m[1] = v4d{p2.x, p2.y, p3.x, p3.y};
  };
  // the top chunk's state
  v4d C3[NT], Cb[NT], Cr[NT], V[VL ? 1 : 3][NT];
  int E3, Es, Er;
  unsigned wc[NC], wn[NC];
  {
    const CkRaw r3 = ck_raw(ctop), rb = ck_raw(ctop - 1), rr = ck_raw(ctop - 2);
    const Raw c0 = codes_raw(ctop), c1 = codes_raw(ctop - 1);
    ck_val(r3, ctop, C3, E3);                    // unused (and unwritten) unless T % 4 == 0
    if ((T & 3) == 0) {
      C3[0] = X[0];
      C3[1] = X[1];
      E3 = Ef;
    }
    ck_val(rb, ctop - 1, Cb, Es);
    ck_val(rr, ctop - 2, Cr, Er);
    codes_pack(c0, ctop, wc);
    codes_pack(c1, ctop - 1, wn);
    v4d x[NT] = {Cb[0], Cb[1]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      v4d e[NT];
      evid(wc, k, e);
      recomp(x, e);
      if constexpr (VL) vstore(k, x);            // the top chunk: slot k (parity 0)
      else
#pragma unroll
        for (int q = 0; q < NT; q++) V[k][q] = x[q];
    }
  }

  // gamma_t normalised exactly (the reference's per-step posteriors) to
  // post[b][t]: 16-byte pieces where the rows are 32 wide and aligned
  const bool pvec = POST && a.post_tstride == NP && (a.post_off & 1) == 0 && (a.post_bstride & 1) == 0 &&
                    (reinterpret_cast<uintptr_t>(a.post) & 15) == 0;
  double* const prow = POST ? a.post + (size_t)(active ? b0 + j : 0) * a.post_bstride + a.post_off : nullptr;
  auto post_store = [&](int t, const v4d (&G)[NT]) {
    const double r = recip(seq_sum(G));
    if (!active) return;
    double* p = prow + t * a.post_tstride;
    if (pvec) {
#pragma unroll
      for (int q = 0; q < NT; q++) {
        store_pol<NIPAMD_POST_NT>(reinterpret_cast<v2d*>(p + 16 * q + 2 * g), v2d{G[q].x * r, G[q].y * r});
        store_pol<NIPAMD_POST_NT>(reinterpret_cast<v2d*>(p + 16 * q + 2 * g + 8), v2d{G[q].z * r, G[q].w * r});
      }
    } else {
#pragma unroll
      for (int q = 0; q < NT; q++) {
        const double v[4] = {G[q].x * r, G[q].y * r, G[q].z * r, G[q].w * r};
#pragma unroll
        for (int rr = 0; rr < 4; rr++)
          if (16 * q + state_of(g, rr) < a.N) store_pol<NIPAMD_POST_NT>(p + 16 * q + state_of(g, rr), v[rr]);
      }
    }
  };

  // VL: chunk c's message k lives in slot k (parity 0) or 2 - k (parity 1);
  // the recomputation writes chunk c - 1's message m where chunk c's message
  // 2 - m was (read at step 2 - m, before the write)
  auto chunk = [&](int c, auto full, auto parity) {
    constexpr bool FULL = decltype(full)::value;
    constexpr int P = decltype(parity)::value;
    auto sig = [](int pp, int k) { return pp ? 2 - k : k; };
    const CkRaw L = ck_raw(c - 3);
    const Raw Lc = codes_raw(c - 2);
    // the count rows of step g, both halves, for sequence j (element offsets
    // into the table; half 1 of a one-column request: the dummy row)
    if constexpr (!POST) {
#pragma unroll
      for (int h = 0; h < 2; h++)
        AD[(g * 2 + h) * 16 + j] = (h < NC ? cro[h] + (int)byte_of4(wc[h < NC ? h : 0], g) : crows) * NP;
    }
    v4d x[NT] = {Cr[0], Cr[1]};                  // chunk c - 1's recomputation chain
    v4d nV[VL ? 1 : 3][NT];
    const int kmax = FULL ? 3 : ((T - 1) & 3);
    // backward step k of chunk c
    auto bstep = [&](int k) {
      v4d curv[NT];
      if constexpr (VL) {
        if (k == 3) { curv[0] = C3[0]; curv[1] = C3[1]; }
        else vload(sig(P, k), curv);
      }
      const v4d(&cur)[NT] = VL ? curv : (k == 3 ? C3 : V[k]);
      const v4d(&prv)[NT] = k == 0 ? Cb : V[VL ? 0 : k - 1];
      v4d e[NT], Xb[NT], G[NT];
      evid(wc, k, e);
#pragma unroll
      for (int q = 0; q < NT; q++) {
        Xb[q] = e[q] * Bt[q];
        if (k == 3) Xb[q] = ldexp4(Xb[q], E3 - Es);
        G[q] = cur[q] * Bt[q];
      }
      if constexpr (POST) {
        matvec2(Ab, Xb, Bt);                     // beta~_{t-1} = A w_t
        post_store(4 * c + k, G);
        return;
      }
      tp_write2(XA, j, g, prv);
      tp_write2(XW, j, g, Xb);
      tp_write2(XG, j, g, G);
      matvec2(Ab, Xb, Bt);                       // beta~_{t-1} = A w_t
      double aT[NT][4], wT[NT][4];
      tp_read2(XA, lane, aT);
      tp_read2(XW, lane, wT);
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int xt = 0; xt < NT; xt++)
#pragma unroll
          for (int yt = 0; yt < NT; yt++) Kd[xt][yt] = mfma1(aT[xt][q], wT[yt][q], Kd[xt][yt]);
      // count rows: one add per sequence (lanes 0-31 column 0's row, 32-63
      // column 1's); every operand read before the first add, so the adds
      // (which the compiler must order against later LDS reads) cost one wait
      const int4* ad = reinterpret_cast<const int4*>(AD + (k * 2 + ch) * 16);
      const int4 o4[4] = {ad[0], ad[1], ad[2], ad[3]};
      double gv[16];
#pragma unroll
      for (int s = 0; s < 16; s++) gv[s] = XG[s * NPS + cy];
      const int off[16] = {o4[0].x, o4[0].y, o4[0].z, o4[0].w, o4[1].x, o4[1].y, o4[1].z, o4[1].w,
                           o4[2].x, o4[2].y, o4[2].z, o4[2].w, o4[3].x, o4[3].y, o4[3].z, o4[3].w};
#pragma unroll
      for (int s = 0; s < 16; s++)
        (void)__hip_atomic_fetch_add(Hl + cy + off[s], gv[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
#pragma unroll
    for (int k = 3; k >= 0; k--) {
#if NIPAMD_CKW_RECOMP_FIRST
      if (k < 3) {                               // chunk c - 1's recomputation, one step per step
        v4d e[NT];
        evid(wn, 2 - k, e);
        recomp(x, e);
#pragma unroll
        for (int q = 0; q < NT; q++) nV[2 - k][q] = x[q];
      }
      if (FULL || k <= kmax) bstep(k);
#else
      if (FULL || k <= kmax) bstep(k);
      if (k < 3) {                               // chunk c - 1's recomputation, one step per step (after
        v4d e[NT];                               // step k: V[k] is dead, nV[2 - k] may take its registers)
        evid(wn, 2 - k, e);
        recomp(x, e);
        if constexpr (VL) vstore(sig(1 - P, 2 - k), x);
        else
#pragma unroll
          for (int q = 0; q < NT; q++) nV[2 - k][q] = x[q];
      }
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
    // down one chunk
#pragma unroll
    for (int q = 0; q < NT; q++) {
      C3[q] = Cb[q];
      Cb[q] = Cr[q];
      if constexpr (!VL)
#pragma unroll
        for (int k = 0; k < 3; k++) V[k][q] = nV[k][q];
    }
    E3 = Es;
    Es = Er;
    ck_val(L, c - 3, Cr, Er);
#pragma unroll
    for (int q = 0; q < NC; q++) wc[q] = wn[q];
    codes_pack(Lc, c - 2, wn);
  };
  const std::integral_constant<int, 0> p0c{};
  const std::integral_constant<int, 1> p1c{};
  if (((T - 1) & 3) == 3) chunk(ctop, std::true_type{}, p0c);
  else chunk(ctop, std::false_type{}, p0c);
  int c = ctop - 1;
  for (; c >= 1; c -= 2) {
    chunk(c, std::true_type{}, p1c);
    chunk(c - 1, std::true_type{}, p0c);
  }
  if (c == 0) chunk(0, std::true_type{}, p1c);

  if constexpr (POST) return;
  // P0 = gamma_{-1}, normalised exactly, summed over the wave's sequences in
  // a fixed order (transpose, in-lane, then lane quarters)
  v4d p0[NT];
  prior(p0);
#pragma unroll
  for (int q = 0; q < NT; q++) p0[q] = p0[q] * Bt[q];
  const double rp = recip(seq_sum(p0));
#pragma unroll
  for (int q = 0; q < NT; q++) p0[q] = p0[q] * rp;
  double p0s[NT];
  {
    double r[NT][4];
    tp_write2(XA, j, g, p0);
    tp_read2(XA, lane, r);
#pragma unroll
    for (int xt = 0; xt < NT; xt++) p0s[xt] = sum_lanes16(sum_lanes32((r[xt][0] + r[xt][1]) + (r[xt][2] + r[xt][3])));
  }

  // the slab row: K [32][32], H [R][32], P0 [32]
  double* slab = a.slab + (size_t)grp * a.slab_size;
  const int tk = lane >> 4, ty = lane & 15;
#pragma unroll
  for (int xt = 0; xt < NT; xt++)
#pragma unroll
    for (int yt = 0; yt < NT; yt++)
#pragma unroll
      for (int r = 0; r < 4; r++) slab[(16 * xt + 4 * r + tk) * NP + 16 * yt + ty] = Kd[xt][yt][r];
  double* Hs = slab + NP * NP;
  for (int c2 = 0; c2 < NC && c2 < a.ncol; c2++)
    for (int i = lane; i < (a.M[c2] + 2) * NP; i += 64) Hs[(size_t)a.crow[c2] * NP + i] = Hl[cro[c2] * NP + i];
  // the unobserved children: every step's gamma on the missing row (the sum
  // of column 0's count rows, in row order), zeros elsewhere
  for (int u = 0; u < a.n_unobs && u < 4; u++)
    for (int i = lane; i < (a.uM[u] + 2) * NP; i += 64) {
      const int m = i / NP, y = i % NP;
      double v = 0.0;
      if (m == a.uM[u])
        for (int rr = 0; rr < a.M[0] + 2; rr++) v += Hl[(cro[0] + rr) * NP + y];
      Hs[(size_t)a.urow[u] * NP + i] = v;
    }
  if (lane < 16) {
#pragma unroll
    for (int xt = 0; xt < NT; xt++) Hs[(size_t)a.R * NP + 16 * xt + lane] = p0s[xt];
  }
}

}  // namespace

template <int PR, int NC, bool POST, bool VL>
static int ckw_launch(const EMwArgs& a, size_t lds, hipStream_t stream) {
  static size_t set[kMaxDevices] = {};
  const void* k = reinterpret_cast<const void*>(&chain_estep_ckw_kernel<PR, NC, POST, VL>);
  if (int rc = ensure_dyn_lds(k, lds, set)) return rc;
  const int wv = VL ? 8 : kWWaves;
  const long groups = (a.B + 15) / 16;
  const int blocks = (int)((groups + wv - 1) / wv);
  hipLaunchKernelGGL((chain_estep_ckw_kernel<PR, NC, POST, VL>), dim3(blocks), dim3(64 * wv), lds, stream, a);
  return 0;
}

size_t chain_estep_ckw_lds_bytes(int tab_rows, int count_rows) {
  const size_t d = (size_t)ckw_tab_doubles(tab_rows) + (size_t)kWWaves * ckw_wave_doubles(count_rows);
  return (d * sizeof(double) + 15) & ~(size_t)15;
}

size_t chain_estep_ckw_scratch_bytes(long B, int T) {
  return (size_t)((B + 15) / 16) * (size_t)ckw_group_doubles(T) * sizeof(double);
}

template <bool POST, bool VL>
static int ckw_dispatch(const EMwArgs& a, bool proper, hipStream_t stream) {
  if (!a.obs || a.N < 1 || a.N > NP || a.ncol < 1 || a.ncol > kMaxCol || a.T < 1 || a.n_unobs > 4)
    return kLaunchRefused;
  if (POST && !a.post) return kLaunchRefused;
  int crows = 0;
  for (int c = 0; c < a.ncol; c++) {
    if (a.M[c] < 1 || a.M[c] + 2 > 255 || a.tab_off[c] % NP != 0) return kLaunchRefused;
    crows += a.M[c] + 2;
  }
  const size_t tabb = (size_t)ckw_tab_doubles(a.tab_rows) * sizeof(double);
  const size_t lds = POST ? ((tabb + (VL ? (size_t)(NT * NT * 4 * 64 + 8 * 3 * 512) * sizeof(double) : 0)) + 15) & ~(size_t)15
                          : chain_estep_ckw_lds_bytes(a.tab_rows, crows);
  if (lds > (size_t)kLdsPerCU) return kLaunchRefused;
  int rc = 0;
  if (proper) rc = a.ncol == 1 ? ckw_launch<1, 1, POST, VL>(a, lds, stream) : ckw_launch<1, 2, POST, VL>(a, lds, stream);
  else rc = a.ncol == 1 ? ckw_launch<0, 1, POST, VL>(a, lds, stream) : ckw_launch<0, 2, POST, VL>(a, lds, stream);
  if (rc) return rc;
  g_last_kernel = POST ? "chain_fb_ckw_kernel" : "chain_estep_ckw_kernel";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int chain_estep_ckw_launch(const EMwArgs& a, bool proper, hipStream_t stream) {
  return ckw_dispatch<false, false>(a, proper, stream);
}

int chain_fb_ckw_launch(const EMwArgs& a, bool proper, bool vl, hipStream_t stream) {
  return vl ? ckw_dispatch<true, true>(a, proper, stream) : ckw_dispatch<true, false>(a, proper, stream);
}

}  // namespace nipamd
