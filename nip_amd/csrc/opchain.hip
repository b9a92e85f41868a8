// opchain.hip -- forward-backward over an evidence-indexed interface chain
// (opchain.h): the two-filter recursion of chain_kernels.hip with the
// transition chosen per step from LDS-resident operators T_c (evidence folded
// in) instead of a fixed transition times an evidence column.
//
// Block = 8 sequences, 4 waves; a 16-lane row per (sequence, direction),
// lane y owns joint interface state y (y < K): rows 0-1 of a wave run the
// forward filter of two sequences, rows 2-3 the backward filter of the same
// two.  Per step a lane reads its column (forward) or row (backward) of
// T_{c_t} from LDS and does the K-term mat-vec with DPP row broadcasts; sums
// over the row are DPP butterflies (bit-identical in every lane).
//   forward:  alpha_t = T_{c_t}^T alpha_{t-1}, alpha_{-1} = prior of the previous interface
//   backward: beta_t  = T_{c_{t+1}} beta_{t+1},  beta_{T-1} = 1
//   posterior_t = normalise(alpha_t o beta_t)
//   ll = sum over steps with evidence of log m2_t - log m1_t, m2_t = sum alpha_t,
//        m1_t = alpha_{t-1} . w (the mass the step would have without its
//        evidence); a step without evidence adds nothing, as the general
//        engine's filter (jtree.hip) and the reference (nip.c:1458-1474)
// Messages carry their scale as exact powers of two (the ratio m2 / m1 is
// taken at one scale).  Phase A / barrier / phase B with the scratch holding
// alpha_t (t < H) and beta_t (t >= H), as chain_kernel<false>.
#include <cfloat>

#include "chain_kernels.h"
#include "opchain.h"
#include "diag.h"

namespace nipamd {
namespace {

constexpr int kOpSeqs = 8;
constexpr int kOpThreads = 256;
constexpr int kOpGuard = 1;

template <int K>
__device__ __forceinline__ double ror(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int rl = __builtin_amdgcn_mov_dpp(lo, 0x120 + K, 0xF, 0xF, true);
  const int rh = __builtin_amdgcn_mov_dpp(hi, 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(rh, rl);
}

__device__ __forceinline__ double rsum(double x) {
  asm("" : "+v"(x));                       // one rounded value per lane (no fma contraction)
  x += ror<8>(x);
  x += ror<4>(x);
  x += ror<2>(x);
  x += ror<1>(x);
  return x;
}

template <int J, bool NOP>
__device__ __forceinline__ void fbc(double& acc, double v, double c) {
  if (NOP)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(J));
  else
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(J));
}

// sum_k x[lane k] * c[k] over the row (c[k] = 0 for k >= K)
__device__ __forceinline__ double dot16(double x, const double (&c)[16]) {
  double a0 = 0.0, a1 = 0.0;
  fbc<0, true>(a0, x, c[0]);   fbc<1, false>(a1, x, c[1]);
  fbc<2, false>(a0, x, c[2]);  fbc<3, false>(a1, x, c[3]);
  fbc<4, false>(a0, x, c[4]);  fbc<5, false>(a1, x, c[5]);
  fbc<6, false>(a0, x, c[6]);  fbc<7, false>(a1, x, c[7]);
  fbc<8, false>(a0, x, c[8]);  fbc<9, false>(a1, x, c[9]);
  fbc<10, false>(a0, x, c[10]); fbc<11, false>(a1, x, c[11]);
  fbc<12, false>(a0, x, c[12]); fbc<13, false>(a1, x, c[13]);
  fbc<14, false>(a0, x, c[14]); fbc<15, false>(a1, x, c[15]);
  return a0 + a1;
}

__device__ __forceinline__ double div_or_keep(double x, double c) { return c != 0.0 ? x / c : x; }

// the value of lane J of this lane's 16-lane row (v_mov_b64_dpp row_newbcast)
template <int J>
__device__ __forceinline__ double bcast(double v) { return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xF, 0xF, false); }

// e_step: lane y of a row writes W(x', y) = a(x') b(y) for x' < K (a(x') from
// lane x' of the row) to dst[x' K + y]
__device__ __forceinline__ void xi_row(double av, double bv, double* dst, int K, int y, bool w) {
#define NIPAMD_XI(J) { const double v = bcast<J>(av) * bv; if (w && J < K) dst[J * K + y] = v; }
  NIPAMD_XI(0) NIPAMD_XI(1) NIPAMD_XI(2) NIPAMD_XI(3) NIPAMD_XI(4) NIPAMD_XI(5) NIPAMD_XI(6) NIPAMD_XI(7)
  NIPAMD_XI(8) NIPAMD_XI(9) NIPAMD_XI(10) NIPAMD_XI(11) NIPAMD_XI(12) NIPAMD_XI(13) NIPAMD_XI(14) NIPAMD_XI(15)
#undef NIPAMD_XI
}

__host__ __device__ __forceinline__ int op_row(int T) { return T + 2 * kOpGuard; }

}  // namespace

__global__ __launch_bounds__(kOpThreads, 2)
void op_fb_kernel(OpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int K = a.K, KK = K * K;
  // operators in LDS when they fit (a.tlds), else read through the caches
  const bool tl = a.tlds != 0;
  double* Tl = reinterpret_cast<double*>(smem);                          // [(ncomb+1)][K][K] (tlds)
  uint16_t* codes = reinterpret_cast<uint16_t*>(smem + (tl ? (size_t)(a.ncomb + 1) * KK * sizeof(double) : 0));
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int y = lane & 15, row = lane >> 4;
  const bool fwd = row < 2;
  const int seq = wave * 2 + (row & 1);
  const long b0 = (long)blockIdx.x * kOpSeqs;
  const long b = b0 + seq;
  const bool active = b < a.B;
  const int T = a.T, H = a.H;

  if (tl)
    for (int i = tid; i < (a.ncomb + 1) * KK; i += kOpThreads) Tl[i] = a.Ttab[i];
  const int nseq = (int)((a.B - b0) < kOpSeqs ? (a.B - b0) : kOpSeqs);
  for (int i = tid; i < kOpSeqs * T; i += kOpThreads) {
    const int s = i / T, t = i - s * T;
    int c = 0;
    if (s < nseq && a.obs) {
      const int32_t* o = a.obs + (b0 + s) * a.obs_bstride + (long)t * a.obs_tstride;
      for (int k = 0; k < a.nobs; k++) {
        const int v = o[a.col[k]];
        if (v >= a.card[k]) { c = a.ncomb; break; }            // all-zero evidence: the zero table
        if (v >= 0) c += (v + 1) * a.cstride[k];
      }
    }
    codes[s * T + t] = (uint16_t)c;
    if (a.estep && s < nseq) a.C[(size_t)(b0 + s) * T + t] = (uint16_t)c;
  }
  __syncthreads();

  const uint16_t* cd = codes + seq * T;
  const double* const Tsrc = tl ? Tl : a.Ttab;
  const bool ys = y < K;
  const double wy = ys ? a.w[y] : 0.0;
  // filter mode keeps no rows in S: its sink is S's first 16 doubles (the
  // host allocates op_scratch_bytes(1, 1) for it); smoothing puts the sink
  // row past the last sequence's rows
  double* const sink = a.filter ? a.S + y : a.S + (size_t)(a.B + 1) * op_row(T) * 16 + y;
  double* const Srow = a.S + ((size_t)(active ? b : 0) * op_row(T) + kOpGuard) * 16 + y;
  double* const Sst = active ? Srow : sink;
  const long sst = active ? 16 : 0;
  const bool pst = active && ys && a.post;
  double* const Pst = pst ? a.post + (size_t)b * a.post_bstride + a.post_off + y : sink;
  const long pstr = pst ? a.post_tstride : 0;

  // this lane's column (forward) / row (backward) of T_c
  auto coef = [&](int c, double (&C)[16]) {
    const double* t = Tsrc + (size_t)c * KK;
#pragma unroll
    for (int k = 0; k < 16; k++)
      C[k] = (k < K && ys) ? (fwd ? t[k * K + y] : t[y * K + k]) : 0.0;
  };

  double x;                      // forward: alpha^_{t-1}; backward: beta^_{t+1}
  int sc = 0;
  double m2 = 1.0, m1 = 1.0;
  int e2 = 0, e1 = 0;
  bool dead = false, bad = false;
  if (fwd) {
    x = ys ? a.pi[y] : 0.0;
  } else {
    x = ys ? 1.0 : 0.0;                                 // beta_{T-1}
    if (!a.filter) Sst[(long)(T - 1) * sst] = x;
  }

  // One step of either direction, branch-free (the rows of a wave differ only
  // in data): j-th step of the phase, t per direction; a row whose phase is
  // shorter idles through its last steps (valid = false: state kept, stores
  // to the sink).  combine: phase B (the posterior from the other
  // direction's message).
  // operator of the step at t (forward: c_t; backward: c_{t+1}), clamped
  auto code_at = [&](int t) {
    const int tc = t < 0 ? 0 : (t > T - 1 ? T - 1 : t);
    return (int)cd[fwd ? tc : (tc + 1 < T ? tc + 1 : T - 1)];
  };
  double Cn[16];                 // the next step's coefficients, loaded one step ahead
  const bool est = a.estep != 0;
  auto step = [&](int t, int tnext, bool valid, bool combine, bool first) {
    const int tc = t < 0 ? 0 : (t > T - 1 ? T - 1 : t);
    const int c = code_at(t);
    double C[16];
#pragma unroll
    for (int k = 0; k < 16; k++) C[k] = Cn[k];
    coef(code_at(tnext), Cn);
    const double m1v = rsum(x * wy);
    const double u = __builtin_ldexp(dot16(x, C), sc);
    const double z = rsum(u);
    if (fwd && valid && c != 0) {                       // a forward step with evidence
      m2 *= z;
      m1 *= __builtin_ldexp(m1v, sc);
      const int k2 = m2 != 0.0 ? __builtin_amdgcn_frexp_exp(m2) : 0;
      const int k1 = m1 != 0.0 ? __builtin_amdgcn_frexp_exp(m1) : 0;
      m2 = __builtin_ldexp(m2, -k2); e2 += k2;
      m1 = __builtin_ldexp(m1, -k1); e1 += k1;
      // e_step's BAD_LUCK (nip.c:1827-1854): a mass <= 0, or the running ll
      // > 0, i.e. m2 2^e2 > m1 2^e1 (both mantissas in [0.5, 1)), as the
      // general engine's e_step checks it after every step with evidence
      if (est && (m2 <= 0.0 || m1 <= 0.0 || e2 > e1 || (e2 == e1 && m2 > m1))) bad = true;
    }
    if (fwd && valid) dead |= z == 0.0;
    if (a.filter) {
      if (fwd) (valid ? Pst : sink)[(long)tc * (valid ? pstr : 0)] = div_or_keep(u, z);
    } else if (!combine) {
      (valid ? Sst : sink)[(long)tc * (valid ? sst : 0)] = u;
    } else {
      const double o = Srow[(long)tc * 16];
      const double pr = u * o;
      const double z = rsum(pr);
      if (est) {
        // the step's xi weights: sum_y u o = 2^sc Z' (Z' the xi mass at the
        // messages' own scale); forward rows W_t = alpha^_{t-1} (x) beta^_t,
        // backward rows W_{t+1} = alpha^_t (x) beta^_{t+1} -- except at their
        // first phase-B step (t = H - 1): W_H is the forward rows'
        const double f = z != 0.0 ? __builtin_ldexp(1.0 / z, sc) : 0.0;
        const int tw = fwd ? tc : tc + 1;
        xi_row(fwd ? x : o, (fwd ? o : x) * f, a.W + ((size_t)b * T + tw) * KK, K, y,
               valid && active && ys && (fwd || !first));
      } else {
        const double q = div_or_keep(pr, z);
        (valid ? Pst : sink)[(long)tc * (valid ? pstr : 0)] = q;
      }
    }
    if (valid) {
      sc = z != 0.0 ? -__builtin_amdgcn_frexp_exp(z) : 0;
      x = u;
    }
  };

  if (a.filter) {
    coef(code_at(0), Cn);
    for (int t = 0; t < T; t++) step(t, t + 1, fwd, false, false);
  } else {
    // phase A: forward t = 0..H-1, backward t = T-2..H
    const int nA = H > T - 1 - H ? H : T - 1 - H;
    const int dir = fwd ? 1 : -1;
    coef(code_at(fwd ? 0 : T - 2), Cn);
    for (int j = 0; j < nA; j++) {
      const int t = fwd ? j : T - 2 - j;
      step(t, t + dir, fwd ? j < H : t >= H, false, false);
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // phase B: forward t = H..T-1 with beta_t, backward t = H-1..0 with alpha_t
    const int nB = T - H > H ? T - H : H;
    coef(code_at(fwd ? H : H - 1), Cn);
    for (int j = 0; j < nB; j++) {
      const int t = fwd ? H + j : H - 1 - j;
      step(t, t + dir, fwd ? t < T : t >= 0, true, j == 0);
    }
    if (est && !fwd) {
      // one more backward step with alpha_{-1} = prior of the previous
      // interface (x = beta^_0): its posterior is the t = 0 marginal of the
      // previous interface (P0), its xi weights W_0 (the forward rows took
      // t = 0 when H = 0)
      double C0[16];
      coef(cd[0], C0);
      const double u0 = __builtin_ldexp(dot16(x, C0), sc);
      const double piy = ys ? a.pi[y] : 0.0;
      const double pr = piy * u0;
      const double z = rsum(pr);
      if (active && ys) a.P0[(size_t)b * K + y] = div_or_keep(pr, z);
      const double f = z != 0.0 ? __builtin_ldexp(1.0 / z, sc) : 0.0;
      xi_row(piy, x * f, a.W + (size_t)b * T * KK, K, y, H > 0 && active && ys);
    }
  }
  if (fwd && active && y == 0) {
    double ll = log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
    if (dead) ll = -DBL_MAX;
    if (a.ll) a.ll[b] = ll;
    // NIPAMD_STATUS_ZERO_MASS (1); in e_step mode also NIPAMD_STATUS_BAD_LUCK
    // (2), which a zero mass implies, as the general engine's e_step sets them
    if (a.status) a.status[b] = (dead ? 1u : 0u) | (est && (dead || bad) ? 2u : 0u);
  }
}

// The e_step's per-combination sums: a block per 16 sequences; one lane owns
// cell l of a combination's K x K block in LDS and adds the group's W_t(l) in
// sequence and step order (one lane per cell and combination: no races, a
// fixed summation order); then P0 over the group; one slab row out.
__global__ __launch_bounds__(256)
void op_xi_kernel(OpXiArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* X = reinterpret_cast<double*>(smem);
  const int KK = a.K * a.K, R = op_xi_row(a.K, a.ncomb);
  const int tid = threadIdx.x;
  for (int i = tid; i < R; i += 256) X[i] = 0.0;
  __syncthreads();
  const long b0 = (long)blockIdx.x * kOpXiSeqs;
  const int T = a.T;
  const int nseq = (int)((a.B - b0) < kOpXiSeqs ? (a.B - b0) : kOpXiSeqs);
  // K*K <= 64: each of the four waves owns the combinations c = wave (mod 4)
  // and scans every step (a quarter of the read-add-write chains per wave);
  // larger K: lane l < K*K of the block owns cell l of every combination
  const bool split = KK <= 64;
  const int cell = split ? (tid & 63) : tid, part = split ? (tid >> 6) : 0, nparts = split ? 4 : 1;
  if (cell < KK) {
    // the group's steps as one stream (sequence-major), loaded a batch of U
    // steps ahead of their sums so no global load's latency meets the chain
    // of LDS read-add-writes
    constexpr int U = 16;
    const long n = (long)nseq * T;
    const double* Wg = a.W + (size_t)b0 * T * KK + cell;
    const uint16_t* Cg = a.C + (size_t)b0 * T;
    double w[2][U];
    int c[2][U];
    auto load = [&](long i0, double (&wv)[U], int (&cv)[U]) {
#pragma unroll
      for (int k = 0; k < U; k++) {
        const long i = i0 + k < n ? i0 + k : n - 1;
        cv[k] = Cg[i];
        wv[k] = Wg[(size_t)i * KK];
      }
    };
    load(0, w[0], c[0]);
    for (long i0 = 0; i0 < n; i0 += 2 * U) {
      load(i0 + U, w[1], c[1]);
#pragma unroll
      for (int k = 0; k < U; k++)
        if (i0 + k < n && c[0][k] % nparts == part) X[(size_t)c[0][k] * KK + cell] += w[0][k];
      if (i0 + U >= n) break;
      load(i0 + 2 * U, w[0], c[0]);
#pragma unroll
      for (int k = 0; k < U; k++)
        if (i0 + U + k < n && c[1][k] % nparts == part) X[(size_t)c[1][k] * KK + cell] += w[1][k];
    }
  }
  if (tid < a.K)
    for (int s = 0; s < nseq; s++) X[(size_t)(a.ncomb + 1) * KK + tid] += a.P0[(size_t)(b0 + s) * a.K + tid];
  __syncthreads();
  double* out = a.slab + (size_t)blockIdx.x * R;
  for (int i = tid; i < R; i += 256) out[i] = X[i];
}

// The projection of the operator chain's e_step: a wave per count cell (its
// CSR row can hold thousands of entries), lane l summing entries l, l + 64,
// ... in order, then a fixed-order wave tree -- deterministic, and the long
// rows no longer serialise one thread each
__global__ __launch_bounds__(256)
void op_finalize_kernel(const double* __restrict__ R, int n, const int* __restrict__ ptr,
                        const int* __restrict__ idx, const double* __restrict__ coef, double* __restrict__ counts) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n) return;
  double acc = 0.0;
  for (int j = ptr[row] + lane; j < ptr[row + 1]; j += 64) acc = __builtin_fma(coef[j], R[idx[j]], acc);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) counts[row] += acc;
}

int op_finalize_launch(const double* R, int n, const int* ptr, const int* idx, const double* coef, double* counts,
                       hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(op_finalize_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, R, n, ptr, idx, coef, counts);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The same sums by a counting sort (op_xi_sort_kernel): the group's steps
// are bucketed by combination in LDS -- stable, so every bucket lists its
// steps in stream order -- and a lane per cell then adds a bucket's W rows in
// a register: the same additions in the same order as op_xi_kernel (each sum
// starts at 0 and takes its steps in stream order), without op_xi_kernel's
// chain of LDS read-add-writes.  Four waves: each ranks a quarter of the
// stream (ballots over the keys of 64 steps at a time), then sums a quarter
// of the buckets.  LDS: keys [n] u16, per-wave counts -> offsets [4][NC] u32,
// bucket starts [NC + 1] u32, the sorted step list [n] u32 (n = 16 T).
__host__ __device__ inline size_t op_xi_sort_lds(int ncomb, int T) {
  const size_t n = (size_t)kOpXiSeqs * T, NC = (size_t)ncomb + 1;
  return ((n * 2 + 15) & ~(size_t)15) + (4 * NC + NC + 1) * 4 + n * 4;
}

__global__ __launch_bounds__(256)
void op_xi_sort_kernel(OpXiArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int KK = a.K * a.K, R = op_xi_row(a.K, a.ncomb), NC = a.ncomb + 1;
  const long b0 = (long)blockIdx.x * kOpXiSeqs;
  const int T = a.T;
  const int nseq = (int)((a.B - b0) < kOpXiSeqs ? (a.B - b0) : kOpXiSeqs);
  const int n = nseq * T;
  uint16_t* key = reinterpret_cast<uint16_t*>(smem);
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + (((size_t)kOpXiSeqs * T * 2 + 15) & ~(size_t)15));   // [4][NC]
  unsigned* start = cnt + 4 * NC;                                                                            // [NC + 1]
  unsigned* idx = start + NC + 1;                                                                            // [n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint16_t* Cg = a.C + (size_t)b0 * T;
  for (int i = tid; i < n; i += 256) key[i] = Cg[i];
  for (int i = tid; i < 4 * NC; i += 256) cnt[i] = 0;
  __syncthreads();
  const int qn = (n + 3) / 4, q0 = min(n, wave * qn), q1 = min(n, q0 + qn);   // this wave's quarter
  unsigned* my = cnt + wave * NC;
  const unsigned long long lt = (1ull << lane) - 1;
  // pass 1: the wave's count per combination
  for (int i0 = q0; i0 < q1; i0 += 64) {
    const int i = i0 + lane;
    const bool v = i < q1;
    const int k = v ? (int)key[i] : -1;
    unsigned long long act = __ballot(v);
    while (act) {
      const int lk = __shfl(k, __builtin_ctzll(act));
      const unsigned long long peers = __ballot(v && k == lk);
      if (lane == __builtin_ctzll(act)) my[lk] += (unsigned)__builtin_popcountll(peers);
      act &= ~peers;
    }
  }
  __syncthreads();
  // bucket sizes, and each wave's offset inside each bucket (after the waves
  // before it: stable across the quarters)
  for (int c = tid; c < NC; c += 256) {
    unsigned t = 0;
    for (int w = 0; w < 4; w++) { const unsigned x = cnt[w * NC + c]; cnt[w * NC + c] = t; t += x; }
    start[c] = t;
  }
  __syncthreads();
  if (tid == 0) {                                    // exclusive scan of the bucket sizes
    unsigned t = 0;
    for (int c = 0; c < NC; c++) { const unsigned x = start[c]; start[c] = t; t += x; }
    start[NC] = t;
  }
  __syncthreads();
  for (int i = tid; i < 4 * NC; i += 256) cnt[i] += start[i % NC];
  __syncthreads();
  // pass 2: scatter, each step to its bucket in stream order
  for (int i0 = q0; i0 < q1; i0 += 64) {
    const int i = i0 + lane;
    const bool v = i < q1;
    const int k = v ? (int)key[i] : -1;
    unsigned long long act = __ballot(v);
    while (act) {
      const int leader = __builtin_ctzll(act);
      const int lk = __shfl(k, leader);
      const unsigned long long peers = __ballot(v && k == lk);
      const unsigned base = my[lk];
      if (v && k == lk) idx[base + (unsigned)__builtin_popcountll(peers & lt)] = (unsigned)i;
      if (lane == leader) my[lk] = base + (unsigned)__builtin_popcountll(peers);
      act &= ~peers;
    }
  }
  __syncthreads();
  // sums: wave w takes the buckets c = w (mod 4), a lane per cell
  double* out = a.slab + (size_t)blockIdx.x * R;
  const double* Wg = a.W + (size_t)b0 * T * KK;
  for (int cb = 0; cb < KK; cb += 64) {
    const int cell = cb + lane;
    const bool on = cell < KK;
    for (int c = wave; c < NC; c += 4) {
      const int j0 = (int)start[c], j1 = (int)start[c + 1];
      double acc = 0.0;
      int j = j0;
      for (; j + 8 <= j1; j += 8) {
        double w[8];
#pragma unroll
        for (int u = 0; u < 8; u++) w[u] = on ? Wg[(size_t)idx[j + u] * KK + cell] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; u++) acc += w[u];
      }
      for (; j < j1; j++) acc += on ? Wg[(size_t)idx[j] * KK + cell] : 0.0;
      if (on) out[(size_t)c * KK + cell] = acc;
    }
  }
  if (wave == 0 && lane < a.K) {
    double p0 = 0.0;
    for (int sq = 0; sq < nseq; sq++) p0 += a.P0[(size_t)(b0 + sq) * a.K + lane];
    out[(size_t)NC * KK + lane] = p0;
  }
}

bool op_xi_fits(int K, int ncomb) { return (size_t)op_xi_row(K, ncomb) * sizeof(double) <= 160 * 1024; }
bool op_xi_sort_fits(int ncomb, int T) { return op_xi_sort_lds(ncomb, T) <= 160 * 1024 - 16; }

int op_xi_launch(const OpXiArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  if (a.K > 16) return -2;
  const size_t slds = (op_xi_sort_lds(a.ncomb, a.T) + 15) & ~(size_t)15;
  if (slds <= 160 * 1024) {
    static size_t sort_set[kMaxDevices] = {};
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&op_xi_sort_kernel), slds, sort_set)) return rc;
    const int blocks = (int)((a.B + kOpXiSeqs - 1) / kOpXiSeqs);
    hipLaunchKernelGGL(op_xi_sort_kernel, dim3(blocks), dim3(256), slds, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (!op_xi_fits(a.K, a.ncomb)) return -2;
  const size_t lds = ((size_t)op_xi_row(a.K, a.ncomb) * sizeof(double) + 15) & ~(size_t)15;
  static size_t lds_set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&op_xi_kernel), lds, lds_set)) return rc;
  const int blocks = (int)((a.B + kOpXiSeqs - 1) / kOpXiSeqs);
  hipLaunchKernelGGL(op_xi_kernel, dim3(blocks), dim3(256), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t op_lds_bytes(int K, int ncomb, int T, bool tables) {
  return (tables ? (size_t)(ncomb + 1) * K * K * sizeof(double) : 0) + (size_t)kOpSeqs * T * sizeof(uint16_t);
}

size_t op_scratch_bytes(long B, int T) { return (size_t)(B + 2) * op_row(T) * 16 * sizeof(double); }

int op_fb_launch(const OpArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
  OpArgs b = a;
  // operators in LDS while two blocks still fit a CU (80 KB each); the
  // diagnostics build can force either (NIPAMD_OP_TLDS=0/1)
  b.tlds = op_lds_bytes(a.K, a.ncomb, a.T, true) <= 80 * 1024 ? 1 : 0;
  if (const char* e = diag_env("NIPAMD_OP_TLDS")) b.tlds = (e[0] == '1' && op_lds_bytes(a.K, a.ncomb, a.T, true) <= 150 * 1024) ? 1 : 0;
  const size_t lds = (op_lds_bytes(a.K, a.ncomb, a.T, b.tlds != 0) + 15) & ~(size_t)15;
  if (lds > 160 * 1024 || a.K > 16 || a.ncomb > 65534) return -2;
  static size_t lds_set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&op_fb_kernel), lds, lds_set)) return rc;
  const int blocks = (int)((a.B + kOpSeqs - 1) / kOpSeqs);
  hipLaunchKernelGGL(op_fb_kernel, dim3(blocks), dim3(kOpThreads), lds, stream, b);
  g_last_kernel = "op_fb_kernel";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
