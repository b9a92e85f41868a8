// estep_ck.hip -- e_step of 16-state interface chains with one observed child
// (the HMM-shaped DBN of SURVEY 8(d) config 4) on the matrix cores, with
// checkpoints and recomputation instead of the interface-message round trip
// (round 6).
//
// What the reference computes per sequence (src/nip.c:1708-2007; families
// :1925-1967) follows from three sums over the sequence:
//   K(x, y)  = sum_t alpha_{t-1}(x) e_t(y) beta_t(y) / Z      (alpha_{-1} = prior)
//   H[m][y]  = sum_t [m = code of o_t] gamma_t(y)             (M1 counts, rows M + 2)
//   P0(x)    = gamma_{-1}(x) = prior(x) beta_{-1}(x) / Z      (OLD_OUTGOING at t = 0)
// with the transition factor A(x, y) applied to K and the missing row split
// by the finalize (estep_finalize_kernel), and ll the forward filter's.
//
// chain_estep16_kernel stores every interface message to HBM and reads it
// back: 256 of its 260 B per sequence-step.  Here a WAVE owns 16 sequences
// and does everything itself, with no barrier and no other wave:
//   forward pass   t = 0..T-1: alpha^_t = e_t o (A^T alpha^_{t-1}), four
//                  v_mfma_f64_16x16x4 per step (the fb kernels' register
//                  algebra, chain_mfma_core.h); every 4th message (t = 4k+3,
//                  rescaled to sum ~1) and its exponent go to HBM: 32 B per
//                  sequence-step written, the same read back;
//   backward pass  t = T-1..0 in chunks of four steps: beta^ by the same
//                  matrix-core recursion with A; the chunk's three other
//                  alpha^ recomputed from the checkpoint below it (one chunk
//                  ahead, so the recomputation overlaps the steps); per step
//                  alpha^_{t-1}, the xi weight w_t and gamma_t go through a
//                  wave-private LDS transpose into sequence-major lanes, xi
//                  is four v_mfma_f64_16x16x4 (K = the wave's 16 sequences)
//                  and the M1 counts are read-add-writes into four LDS count
//                  tables (lane quarter k owns table k, so no two lanes of an
//                  instruction touch one cell: deterministic, no atomics).
// HBM per sequence-step: the observation (4 B, read by both passes) and the
// checkpoints (2 x 8 B amortised: 128 B per 4 steps written, read once): 72 B
// against chain_estep16_kernel's 260.
//
// Normalisation: both recursions rescale by exact powers of two every 4th step
// (only where the host's bound rules out underflow between rescales,
// engine.cpp estep16_sparse_ok) and carry the exponents (Ef, Eb), so
// c_t = sum_y alpha^_t beta^_t = Z 2^(Ef_t + Eb_t) for every t: one exact sum
// per chunk (c*, E*) normalises the chunk's four steps,
//   gamma_t = alpha^_t o beta^_t 2^(E* - Ef_t - Eb_t) / c*
//   w_t     = e_t o beta^_t 2^(E* - Ef_{t-1} - Eb_t) / c*   (paired with alpha^_{t-1})
// -- the drift of chain_estep16_kernel's per-phase c* cannot build up here.
// P0 is normalised exactly.  Sums in a fixed order throughout; one slab row per
// wave (chain_estep_slab layout: Kf = K, Kb = 0, Hf = H, Hb = 0, P0), reduced
// by tree64_kernel and applied by estep_finalize_kernel like every 16-state
// e_step slab, so partials of whole 16-sequence groups combine bit-identically.
//
// ll (nip.c:1458-1474): proper models (rows of A and of the child sum to 1:
// the per-step masses telescope) log of the final forward mass minus its
// exponent; otherwise m2_t = sum(alpha_t), m1_t = sum(u_t o s) per step (u_t =
// A^T alpha^_{t-1}; a missing step has e = s, so both are the same bits and
// the step adds exactly 0), as mantissa / exponent products.
#include "chain_mfma_core.h"
#include "store_pol.h"

#include <type_traits>

namespace nipamd {

namespace {

constexpr int kCkWaves = 4;                  // waves per block, one per SIMD; a wave owns 16 sequences
constexpr int kCkThreads = 64 * kCkWaves;
constexpr int kCkEt = 18;                    // evidence row stride (doubles): rows 144 B apart (chain_ckpt.hip)
constexpr int kCkXD = 256;                   // one transpose buffer: [16 sequences][16 states]
#ifndef NIPAMD_CK_SCR_NT
#define NIPAMD_CK_SCR_NT 0                   // A/B builds: checkpoints stored / loaded nontemporal
#endif

// per-wave LDS (doubles): four count tables [4][R][16], three transpose
// buffers (alpha^_{t-1}, w_t, gamma_t), the chunk's packed codes [16] words
__host__ __device__ inline int ck_wave_doubles(int R) { return 4 * R * 16 + 3 * kCkXD + 8; }
__host__ __device__ inline int ck_et_doubles(int R) { return (R * kCkEt + 1) & ~1; }
// checkpoint slot c per group: alpha^_{4c+3}; [nck][16][16] doubles, then [nck][16] int exponents
__host__ __device__ inline int ck_count(int T) { return (T + 3) >> 2; }
__host__ __device__ inline long ck_group_doubles(int T) { return (long)ck_count(T) * (256 + 8); }

// transpose buffer [row][16]: the 16-byte piece p of row r at (p ^ (r & 7)):
// the filter-layout writes (lane (g, j): pieces g and g + 4 of row j) and the
// sequence-major reads (a row's 16 doubles per 16 lanes) are conflict-free
__device__ __forceinline__ int tp_off(int row, int piece) { return row * 16 + ((piece ^ (row & 7)) << 1); }

// filter layout (lane (g, j): states 2g, 2g+1, 2g+8, 2g+9 of sequence j) -> row j
__device__ __forceinline__ void tp_write(double* buf, int j, int g, const v4d& v) {
  *reinterpret_cast<v2d*>(buf + tp_off(j, g)) = v2d{v.x, v.y};
  *reinterpret_cast<v2d*>(buf + tp_off(j, g + 4)) = v2d{v.z, v.w};
}

// sequence-major: lane l gets state l & 15 of sequences 4q + (l >> 4), q = 0..3 --
// exactly the A (i = state, k = sequence) and B (k = sequence, j = state)
// operands of v_mfma_f64_16x16x4 q
__device__ __forceinline__ v4d tp_read(const double* buf, int lane) {
  const int y = lane & 15, k = lane >> 4;
  const int p = y >> 1, e = y & 1;
  v4d r;
  r.x = buf[tp_off(k, p) + e];
  r.y = buf[tp_off(4 + k, p) + e];
  r.z = buf[tp_off(8 + k, p) + e];
  r.w = buf[tp_off(12 + k, p) + e];
  return r;
}

__device__ __forceinline__ v4d mfma4(const v4d& a, const v4d& b, v4d d) {
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, b.x, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, b.y, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(a.z, b.z, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(a.w, b.w, d, 0, 0, 0);
  return d;
}

__device__ __forceinline__ unsigned byte_of(unsigned w, int k) { return (w >> (8 * k)) & 0xFFu; }

#ifndef NIPAMD_CK_LDS_ADD
#define NIPAMD_CK_LDS_ADD 1                  // A/B builds: 0 = read-add-write
#endif
__device__ __forceinline__ void count_add(double* cell, double v) {
#if NIPAMD_CK_LDS_ADD
  (void)__hip_atomic_fetch_add(cell, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  *cell += v;
#endif
}

// mantissa / exponent running product
struct MProd {
  double m = 1.0;
  int e = 0;
  __device__ __forceinline__ void mul(double x) { m *= x; }
  __device__ __forceinline__ void renorm() {
    const int k = __builtin_amdgcn_frexp_exp(m);
    m = __builtin_ldexp(m, -k);
    e += k;
  }
};

template <int PR, bool VEC>
__global__ __launch_bounds__(kCkThreads, 2) void chain_estep_ck_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.M, R = M + 2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* Et = reinterpret_cast<double*>(smem);                                // [R][kCkEt]
  double* wl = Et + ck_et_doubles(R) + (size_t)wave * ck_wave_doubles(R);
  double* H = wl;                                                             // [4][R][16]
  double* XA = H + 4 * R * 16;                                                // alpha^_{t-1}
  double* XW = XA + kCkXD;                                                    // w_t
  double* XG = XW + kCkXD;                                                    // gamma_t
  unsigned* CW = reinterpret_cast<unsigned*>(XG + kCkXD);                     // [16] packed codes

  for (int i = tid; i < R * 16; i += kCkThreads) Et[(i >> 4) * kCkEt + (i & 15)] = a.Etab[i];
  for (int i = lane; i < 4 * R * 16; i += 64) H[i] = 0.0;
  __syncthreads();                                                            // the block's only barrier

  const long grp = (long)blockIdx.x * kCkWaves + wave;
  const long b0 = grp * 16;
  if (b0 >= a.B) return;
  // diagnostics builds (a.diag): per group the wall clock at entry and exit
  // (s_memrealtime, 100 MHz), the forward and backward passes' shader cycles
  // and the SIMD
  const unsigned long long r_in = a.diag ? __builtin_amdgcn_s_memrealtime() : 0;
  const unsigned long long c_in = a.diag ? __builtin_readcyclecounter() : 0;
  unsigned long long c_mid = 0;
  const int j = lane & 15, g = lane >> 4;
  const int sj = state_of(j & 3, j >> 2);
  const bool active = b0 + j < a.B;
  const int* orow = a.obs ? a.obs + (active ? (b0 + j) * a.obs_bstride : 0) + a.obs_col : nullptr;
  const int nck = ck_count(T);
  double* Sg = a.S + (size_t)grp * ck_group_doubles(T);                      // [nck][16][16]
  int* Xg = reinterpret_cast<int*>(Sg + (size_t)nck * 256);                   // [nck][16]

  // the four codes of chunk c (steps 4c..4c+3) of this lane's sequence, one
  // byte each: the state, M missing, M + 1 out of range; steps past T and
  // sequences past B read as missing.  Loaded raw (codes_raw) and packed
  // where they are used (codes_pack), a chunk later: nothing consumes a load
  // in the chunk that issues it, so no wait for it lands there.
  // (VEC: [B][T] int32 rows, T % 4 == 0, 16-byte aligned: one int4 load at a
  // clamped step)
  auto codes_raw = [&](int c) -> int4 {
    const int t0 = 4 * c;
    if (VEC) {
      const int tc = t0 < 0 ? 0 : (t0 > T - 4 ? T - 4 : t0);
      return *reinterpret_cast<const int4*>(orow + tc);
    }
    int o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int t = t0 + k < 0 ? 0 : (t0 + k > T - 1 ? T - 1 : t0 + k);
      o[k] = orow ? orow[(long)t * a.obs_tstride] : -1;
    }
    return int4{o[0], o[1], o[2], o[3]};
  };
  auto codes_pack = [&](const int4& v, int c) -> unsigned {
    const int t0 = 4 * c;
    const int o[4] = {v.x, v.y, v.z, v.w};
    unsigned w = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const bool in = active && t0 + k >= 0 && t0 + k < T;
      const int ok = in ? o[k] : -1;
      const int cd = ok < 0 ? M : (ok < M ? ok : M + 1);
      w |= (unsigned)cd << (8 * k);
    }
    return w;
  };
  const double* Etg = Et + 2 * g;
  auto evid = [&](unsigned w, int k) { return load4(Etg + byte_of(w, k) * kCkEt); };

  // the matrix-core operands: forward u(y) = sum_x A[x][y] X(x), backward u(x) = sum_y A[x][y] X(y)
  double Af[4], Ab[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    Af[r] = a.A[state_of(g, r) * 16 + sj];
    Ab[r] = a.A[sj * 16 + state_of(g, r)];
  }
  const v4d zero = {0.0, 0.0, 0.0, 0.0};
  const v4d prior = active ? load4(a.pi + 2 * g) : zero;
  const v4d srow = load4(Etg + M * kCkEt);                                    // s: the missing row

  auto ck_store = [&](int slot, const v4d& p, int e) {
    double* q = Sg + (size_t)slot * 256 + j * 16 + 2 * g;
    store_pol<NIPAMD_CK_SCR_NT>(reinterpret_cast<v2d*>(q), v2d{p.x, p.y});
    store_pol<NIPAMD_CK_SCR_NT>(reinterpret_cast<v2d*>(q + 8), v2d{p.z, p.w});
    if (g == 0) Xg[slot * 16 + j] = e;
  };

  // ---------------------------------------------------------------- forward
  v4d X = prior;                 // alpha^_{t-1}
  int Ef = 0;
  MProd m2, m1;
  bool dead = false;
  {
    // one full chunk of four steps from the codes w (loaded two chunks ago);
    // w is reloaded with chunk c + 2's.  Two chunks per loop iteration with
    // fixed registers (wA, wB): a loaded register is never copied, so no wait
    // on a load still in flight lands in the loop (a copy at the back edge
    // would wait for the load issued in the same iteration)
    auto fchunk = [&](int c, int4& wr) {
      const unsigned w = codes_pack(wr, c);
      v4d e[4];
#pragma unroll
      for (int k = 0; k < 4; k++) e[k] = evid(w, k);
      wr = codes_raw(c + 2);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const v4d u = matvec(Af, X);
        v4d p = u * e[k];
        double z = 0.0;
        if (!PR) {
          z = chain_sum(p);
          m2.mul(z);
          m1.mul(chain_sum(u * srow));
          m2.renorm();
          m1.renorm();
          dead |= z == 0.0;
        }
        if (k == 3) {
          if (PR) z = chain_sum(p);
          const int sc = -__builtin_amdgcn_frexp_exp(z);     // frexp exponent of 0 is 0
          p = ldexp4(p, sc);
          Ef += sc;
          ck_store(c, p, Ef);
        }
        X = p;
      }
    };
    int4 wA = codes_raw(0), wB = codes_raw(1);
    const int nfull = T >> 2;
    int c = 0;
    for (; c + 2 <= nfull; c += 2) {
      fchunk(c, wA);
      fchunk(c + 1, wB);
    }
    if (c < nfull) fchunk(c++, wA);
    // the last, partial chunk (T % 4 steps): no checkpoint; its codes are in
    // wA when nfull is even, wB when odd
    const unsigned wl = codes_pack((nfull & 1) ? wB : wA, nfull);
    for (int t = nfull * 4; t < T; t++) {
      const v4d u = matvec(Af, X);
      const v4d p = u * evid(wl, t & 3);
      if (!PR) {
        const double z = chain_sum(p);
        m2.mul(z);
        m1.mul(chain_sum(u * srow));
        m2.renorm();
        m1.renorm();
        dead |= z == 0.0;
      }
      X = p;
    }
  }
  // ll and status (nip.c:1458-1474; e_step's BAD_LUCK on a zero mass, nip.c:1827-1854)
  if (PR) {
    const double zT = chain_sum(X);
    dead = zT == 0.0;
    if (active && g == 0) {
      const double ll = dead ? -DBL_MAX : log(zT) - (double)Ef * 0.69314718055994530942;
      if (a.ll) a.ll[b0 + j] = ll;
      if (a.status) a.status[b0 + j] = dead ? 3u : 0u;
    }
  } else {
    if (active && g == 0) {
      double ll = log(m2.m) - log(m1.m) + (double)(m2.e - m1.e) * 0.69314718055994530942;
      if (dead || m2.m == 0.0) ll = -DBL_MAX;
      if (a.ll) a.ll[b0 + j] = ll;
      if (a.status) a.status[b0 + j] = (dead || m2.m == 0.0) ? 3u : 0u;
    }
  }
  // the checkpoints back from HBM by this wave: its own stores first
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (a.diag) c_mid = __builtin_readcyclecounter();

  // --------------------------------------------------------------- backward
  // checkpoint slot k (exponent in Xg); k < 0: the prior, exponent 0.
  // Loaded raw (slot 0 for k < 0) and selected where used, a chunk later.
  struct CkRaw {
    v2d lo, hi;
    int e;
  };
  auto ck_raw = [&](int k) -> CkRaw {
    const int kc = k < 0 ? 0 : k;
    const double* q = Sg + (size_t)kc * 256 + j * 16 + 2 * g;
    CkRaw r;
    r.lo = load_pol<NIPAMD_CK_SCR_NT>(reinterpret_cast<const v2d*>(q));
    r.hi = load_pol<NIPAMD_CK_SCR_NT>(reinterpret_cast<const v2d*>(q + 8));
    r.e = Xg[kc * 16 + j];
    return r;
  };
  auto ck_val = [&](const CkRaw& r, int k) -> v4d {
    return k < 0 ? prior : v4d{r.lo.x, r.lo.y, r.hi.x, r.hi.y};
  };
  auto ck_exp = [&](const CkRaw& r, int k) -> int { return k < 0 ? 0 : r.e; };
  const int ctop = (T - 1) >> 2;
  // beta~_t = beta_t 2^-Ef_t / Z: the backward message normalised against
  // the forward one, sum_y alpha^_t beta~_t = 1 for every t -- gamma_t =
  // alpha^_t o beta~_t and the xi weight w_t = e_t o beta~_t 2^(Ef_t - Ef_{t-1})
  // need no per-step or per-chunk normaliser, and beta~_{t-1} = A w_t is the
  // recursion itself (no rescaling: its size follows alpha^'s).  Start:
  // beta~_{T-1} = 1 / z_T on the real states, z_T = sum_y alpha^_{T-1}
  // (0 for a dead or absent sequence: everything it adds is then 0).
  const double rz = recip(chain_sum(X));
  v4d Bt;                                       // beta~_t
  Bt.x = state_of(g, 0) < a.N ? rz : 0.0;
  Bt.y = state_of(g, 1) < a.N ? rz : 0.0;
  Bt.z = state_of(g, 2) < a.N ? rz : 0.0;
  Bt.w = state_of(g, 3) < a.N ? rz : 0.0;
  v4d Kd = zero;                                // xi sums (D[i][y]: lane (i % 4) * 16 + y, register i / 4)
  const int tk = lane >> 4, ty = lane & 15;     // sequence-major lane: table tk, state ty
  double* Hk = H + tk * R * 16 + ty;

  // What chunk c needs, all at hand when it starts (loaded or recomputed
  // during chunk c + 1): V[0..2] = alpha^_{4c..4c+2} (recomputed from the
  // checkpoint below, exponent Es), C3 = alpha^_{4c+3} (checkpoint c, E3;
  // the top chunk's is the forward pass's X when T % 4 == 0, unused
  // otherwise), Cb = alpha^_{4c-1} (checkpoint c - 1 or the prior, Es), Cr =
  // checkpoint c - 2 (chunk c - 1's recomputation starts from it), the packed
  // codes of chunk c (wc) and of chunk c - 1 (wn).  A chunk passes C3, Cb, Cr
  // and wn down and loads one checkpoint (c - 3) and the raw codes of chunk
  // c - 2: issued at its start, converted at its end (round 6: the earlier
  // form reloaded checkpoints c - 1 and c - 2 from L2 in every chunk, 0.95 GB
  // of extra fetches per config-4 launch, profiles/pmc_traffic.json r06y).
  v4d V[3], C3, Cb, Cr;
  int E3, Es, Er;
  unsigned wc, wn;
  {
    const CkRaw r3 = ck_raw(ctop), rb = ck_raw(ctop - 1), rr = ck_raw(ctop - 2);
    const int4 c0 = codes_raw(ctop), c1 = codes_raw(ctop - 1);
    const bool top = (T & 3) == 0;
    C3 = top ? X : ck_val(r3, ctop);
    E3 = top ? Ef : ck_exp(r3, ctop);
    Cb = ck_val(rb, ctop - 1);
    Es = ck_exp(rb, ctop - 1);
    Cr = ck_val(rr, ctop - 2);
    Er = ck_exp(rr, ctop - 2);
    wc = codes_pack(c0, ctop);
    wn = codes_pack(c1, ctop - 1);
    v4d x = Cb;
#pragma unroll
    for (int k = 0; k < 3; k++) { x = matvec(Af, x) * evid(wc, k); V[k] = x; }
  }

  // one chunk: its steps t = 4c + k, k = kmax..0 (kmax = 3 but in a short top
  // chunk), chunk c - 1's recomputation one step after each step
  auto chunk = [&](int c, auto full) {
    constexpr bool FULL = decltype(full)::value;
    const CkRaw L = ck_raw(c - 3);
    const int4 Lc = codes_raw(c - 2);
    if (g == 0) CW[j] = wc;                      // this chunk's packed codes, for the sequence-major lanes
    const unsigned cq0 = CW[tk], cq1 = CW[4 + tk], cq2 = CW[8 + tk], cq3 = CW[12 + tk];
    const int kmax = FULL ? 3 : ((T - 1) & 3);
    v4d x = Cr;                                  // chunk c - 1's recomputation chain
    v4d nV[3];
#pragma unroll
    for (int k = 3; k >= 0; k--) {
      if (FULL || k <= kmax) {                   // (the top chunk's steps past T - 1 skipped)
        const v4d cur = k == 3 ? C3 : V[k];      // alpha^_t
        const v4d prv = k == 0 ? Cb : V[k - 1];  // alpha^_{t-1}
        // w_t = e_t o beta~_t, times 2^(Ef_t - Ef_{t-1}) at the chunk's top step
        // (alpha^_{4c+3} carries the forward pass's rescale, the others Es)
        v4d Xb = evid(wc, k) * Bt;
        if (k == 3) Xb = ldexp4(Xb, E3 - Es);
        tp_write(XA, j, g, prv);
        tp_write(XW, j, g, Xb);
        tp_write(XG, j, g, cur * Bt);            // gamma_t
        Bt = matvec(Ab, Xb);                     // beta~_{t-1} = A w_t
        const v4d aT = tp_read(XA, lane), wT = tp_read(XW, lane), gT = tp_read(XG, lane);
        Kd = mfma4(aT, wT, Kd);
        // M1 counts: lane (tk, ty) adds gamma_t(ty) of sequences 4q + tk to
        // table tk, row = its code.  LDS adds without return (ds_add_f64): no
        // two lanes of one instruction share a cell, and a wave's LDS operations
        // execute in program order, so every cell sums its terms in a fixed
        // order -- deterministic -- without the read-add-write chain's waits
        count_add(Hk + byte_of(cq0, k) * 16, gT.x);
        count_add(Hk + byte_of(cq1, k) * 16, gT.y);
        count_add(Hk + byte_of(cq2, k) * 16, gT.z);
        count_add(Hk + byte_of(cq3, k) * 16, gT.w);
      }
      if (k < 3) {                               // chunk c - 1's recomputation (after step k: V[k] is dead);
        x = matvec(Af, x) * evid(wn, 2 - k);     // at c = 0 it runs on missing codes and is never used
        nV[2 - k] = x;
      }
    }
    // keep the next chunk's unpacking of these loads out of this chunk: the
    // scheduler would hoist it here and wait for loads issued a moment ago
    __builtin_amdgcn_sched_barrier(0);
    // down one chunk
    C3 = Cb;
    Cb = Cr;
    E3 = Es;
    Es = Er;
    Cr = ck_val(L, c - 3);
    Er = ck_exp(L, c - 3);
#pragma unroll
    for (int k = 0; k < 3; k++) V[k] = nV[k];
    wc = wn;
    wn = codes_pack(Lc, c - 2);
  };
  if (((T - 1) & 3) == 3) chunk(ctop, std::true_type{});
  else chunk(ctop, std::false_type{});
  int c = ctop - 1;
  for (; c >= 1; c -= 2) {
    chunk(c, std::true_type{});
    chunk(c - 1, std::true_type{});
  }
  if (c == 0) chunk(0, std::true_type{});

  // P0 = gamma_{-1}: prior o beta^_{-1}, normalised exactly; summed over the
  // wave's sequences in a fixed order (transpose, in-lane, then lane quarters)
  const v4d p0 = prior * Bt;
  const v4d q0 = p0 * recip(chain_sum(p0));
  tp_write(XG, j, g, q0);
  const v4d q0T = tp_read(XG, lane);
  const double p0s = sum_lanes16(sum_lanes32((q0T.x + q0T.y) + (q0T.z + q0T.w)));

  // the slab row (chain_estep_slab layout)
  double* slab = a.counts + (size_t)grp * chain_estep_slab(M);
#pragma unroll
  for (int r = 0; r < 4; r++) slab[kSlabKf + (4 * r + tk) * 16 + ty] = Kd[r];
  for (int i = lane; i < 256; i += 64) slab[kSlabKb + i] = 0.0;
  for (int i = lane; i < R * 16; i += 64) {
    const int row = i >> 4, y = i & 15;
    const double v = ((H[row * 16 + y] + H[R * 16 + row * 16 + y]) + H[2 * R * 16 + row * 16 + y]) +
                     H[3 * R * 16 + row * 16 + y];
    slab[kSlabH + i] = v;
    slab[kSlabH + R * 16 + i] = 0.0;
  }
  if (lane < 16) slab[chain_slab_p0(M) + lane] = p0s;
  if (a.diag && lane == 0) {
    unsigned long long* d = a.diag + (size_t)grp * 5;
    d[0] = r_in;
    d[1] = __builtin_amdgcn_s_memrealtime();
    d[2] = c_mid - c_in;
    d[3] = __builtin_readcyclecounter() - c_mid;
    d[4] = (__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3;   // hwreg(HW_REG_HW_ID): SIMD
  }
}

}  // namespace

template <int PR, bool VEC>
static int ck_launch(const ChainArgs& a, size_t lds, int blocks, hipStream_t stream) {
  static size_t set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_estep_ck_kernel<PR, VEC>), lds, set)) return rc;
  hipLaunchKernelGGL((chain_estep_ck_kernel<PR, VEC>), dim3(blocks), dim3(kCkThreads), lds, stream, a);
  return 0;
}

size_t chain_estep_ck_lds_bytes(int M) {
  const int R = M + 2;
  return ((size_t)ck_et_doubles(R) + (size_t)kCkWaves * ck_wave_doubles(R)) * sizeof(double);
}

size_t chain_estep_ck_scratch_bytes(long B, int T) {
  return (size_t)((B + 15) / 16) * (size_t)ck_group_doubles(T) * sizeof(double);
}

int chain_estep_ck_launch(const ChainArgs& a, hipStream_t stream) {
  const size_t lds = (chain_estep_ck_lds_bytes(a.M) + 15) & ~(size_t)15;
  if (a.N > 16 || a.ne != 1 || !a.counts || a.T < 1 || lds > 160 * 1024) return kLaunchRefused;
  const long groups = (a.B + 15) / 16;
  const int blocks = (int)((groups + kCkWaves - 1) / kCkWaves);
  const bool vec = a.obs && a.obs_tstride == 1 && (a.obs_bstride & 3) == 0 && (a.T & 3) == 0 &&
                   ((reinterpret_cast<uintptr_t>(a.obs) & 15) == 0) && a.obs_col == 0;
  int rc = 0;
  if (a.proper) rc = vec ? ck_launch<1, true>(a, lds, blocks, stream) : ck_launch<1, false>(a, lds, blocks, stream);
  else rc = vec ? ck_launch<0, true>(a, lds, blocks, stream) : ck_launch<0, false>(a, lds, blocks, stream);
  if (rc) return rc;
  g_last_kernel = "chain_estep_ck_kernel";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
