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
#include <cstdint>

#include "chain_kernels.h"

namespace nipamd {

namespace {

template <int K>
__device__ __forceinline__ double row_ror(double v) {
  static_assert(K > 0 && K < 16, "row_ror");
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int rl = __builtin_amdgcn_update_dpp(0, lo, 0x120 + K, 0xF, 0xF, false);
  const int rh = __builtin_amdgcn_update_dpp(0, hi, 0x120 + K, 0xF, 0xF, false);
  return __hiloint2double(rh, rl);
}

template <int K>
__device__ __forceinline__ int row_ror_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x120 + K, 0xF, 0xF, false);
}

// out[k] = value held by the lane that row_ror:k reads from (out[0] = own)
__device__ __forceinline__ void row_gather(double v, double (&out)[16]) {
  out[0] = v;
  out[1] = row_ror<1>(v);   out[2] = row_ror<2>(v);   out[3] = row_ror<3>(v);
  out[4] = row_ror<4>(v);   out[5] = row_ror<5>(v);   out[6] = row_ror<6>(v);
  out[7] = row_ror<7>(v);   out[8] = row_ror<8>(v);   out[9] = row_ror<9>(v);
  out[10] = row_ror<10>(v); out[11] = row_ror<11>(v); out[12] = row_ror<12>(v);
  out[13] = row_ror<13>(v); out[14] = row_ror<14>(v); out[15] = row_ror<15>(v);
}

__device__ __forceinline__ void row_sources(int y, int (&src)[16]) {
  src[0] = y;
  src[1] = row_ror_i<1>(y);   src[2] = row_ror_i<2>(y);   src[3] = row_ror_i<3>(y);
  src[4] = row_ror_i<4>(y);   src[5] = row_ror_i<5>(y);   src[6] = row_ror_i<6>(y);
  src[7] = row_ror_i<7>(y);   src[8] = row_ror_i<8>(y);   src[9] = row_ror_i<9>(y);
  src[10] = row_ror_i<10>(y); src[11] = row_ror_i<11>(y); src[12] = row_ror_i<12>(y);
  src[13] = row_ror_i<13>(y); src[14] = row_ror_i<14>(y); src[15] = row_ror_i<15>(y);
}

// Sum over the 16 lanes of the row; identical bits in every lane (each level
// pairs lanes whose partial sums are equal, and IEEE addition commutes).
__device__ __forceinline__ double row_sum(double x) {
  x += row_ror<8>(x);
  x += row_ror<4>(x);
  x += row_ror<2>(x);
  x += row_ror<1>(x);
  return x;
}

__device__ __forceinline__ double dot16(const double (&a)[16], const double (&c)[16]) {
  double s0 = a[0] * c[0], s1 = a[1] * c[1], s2 = a[2] * c[2], s3 = a[3] * c[3];
#pragma unroll
  for (int k = 4; k < 16; k += 4) {
    s0 = __builtin_fma(a[k], c[k], s0);
    s1 = __builtin_fma(a[k + 1], c[k + 1], s1);
    s2 = __builtin_fma(a[k + 2], c[k + 2], s2);
    s3 = __builtin_fma(a[k + 3], c[k + 3], s3);
  }
  return (s0 + s1) + (s2 + s3);
}

// exponent e such that x = m * 2^e, m in [0.5, 1); 0 for x == 0
__device__ __forceinline__ int exp2_of(double x) {
  return x != 0.0 ? __builtin_amdgcn_frexp_exp(x) : 0;
}

}  // namespace

constexpr int kChainsPerBlock = 8;   // 8 sequences; waves 0-1 forward, 2-3 backward
constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads)
void chain_fb_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* Et = reinterpret_cast<double*>(smem);                       // [(M+2)][16]
  uint8_t* codes = smem + (size_t)(a.M + 2) * 16 * sizeof(double);    // [8][T]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int y = lane & 15, row = lane >> 4;
  const bool fwd = wave < 2;
  const int chain = (wave & 1) * 4 + row;
  const long b0 = (long)blockIdx.x * kChainsPerBlock;
  const long b = b0 + chain;
  const bool active = b < a.B;
  const int T = a.T, H = a.H;

  // --- stage the evidence table and this block's observation codes in LDS
  for (int i = tid; i < (a.M + 2) * 16; i += kThreads) Et[i] = a.Etab[i];
  for (long i = tid; i < (long)kChainsPerBlock * T; i += kThreads) {
    const int c = (int)(i / T), t = (int)(i - (long)c * T);
    int code = a.M;                                      // missing
    if (b0 + c < a.B && a.obs) {
      const int o = a.obs[(b0 + c) * a.obs_bstride + (long)t * a.obs_tstride + a.obs_col];
      code = o < 0 ? a.M : (o < a.M ? o : a.M + 1);
    }
    codes[c * T + t] = (uint8_t)code;
  }

  // --- per-lane coefficients: column (fwd) / row (bwd) of A, rotated to
  //     match the row_gather order
  int src[16];
  row_sources(y, src);
  double C[16], TS[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    C[k] = fwd ? a.A[src[k] * 16 + y] : a.A[y * 16 + src[k]];
    TS[k] = a.ts[src[k]];
  }
  __syncthreads();

  const uint8_t* mycodes = codes + chain * T;
  double* Sb = a.S + (size_t)(active ? b : 0) * T * 16;
  double* Pb = a.post + (size_t)(active ? b : 0) * a.post_bstride;
  const bool ystore = active && y < a.N;

  // forward state
  double vin[16];          // gathered input vector (alpha_{t-1}, scaled)
  int sc = 0;              // pending power-of-two scale for the next mat-vec
  double m2 = 1.0, m1 = 1.0;
  int e2 = 0, e1 = 0;
  bool dead = false;

  if (fwd) {
    const double p = a.pi[y];
    row_gather(p, vin);
  } else {
    // beta_{T-1} = 1 on the real states; g = e_{T-1} o beta
    const double beta = y < a.N ? 1.0 : 0.0;
    if (active && T - 1 >= H) Sb[(size_t)(T - 1) * 16 + y] = beta;
    const double g = Et[mycodes[T - 1] * 16 + y] * beta;
    const double s = row_sum(g);
    sc = -exp2_of(s);
    row_gather(g, vin);
  }

  // one forward step producing alpha_t; combine with beta_t when `combine`
  auto fstep = [&](int t, bool combine) {
    const double e = Et[mycodes[t] * 16 + y];
    double bt = 0.0;
    if (combine && active) bt = Sb[(size_t)t * 16 + y];
    const double u = __builtin_ldexp(dot16(vin, C), sc);
    const double z1 = __builtin_ldexp(dot16(vin, TS), sc);
    const double v = u * e;
    const double z2 = row_sum(v);
    if (!combine) {
      if (active) Sb[(size_t)t * 16 + y] = v;
    } else {
      const double pr = v * bt;
      const double c = row_sum(pr);
      if (ystore) Pb[(size_t)t * a.post_tstride + a.post_off + y] = c != 0.0 ? pr / c : pr;
    }
    // ll: product of z2 / product of z1, as mantissa * 2^exponent
    dead |= (z2 == 0.0);
    m2 *= z2; m1 *= z1;
    { const int k2 = exp2_of(m2); m2 = __builtin_ldexp(m2, -k2); e2 += k2; }
    { const int k1 = exp2_of(m1); m1 = __builtin_ldexp(m1, -k1); e1 += k1; }
    sc = -exp2_of(z2);
    row_gather(v, vin);
  };

  // one backward step producing beta_{t} from g_{t+1}; combine with alpha_t
  auto bstep = [&](int t, bool combine) {
    const double e = Et[mycodes[t] * 16 + y];
    double at = 0.0;
    if (combine && active) at = Sb[(size_t)t * 16 + y];
    const double w = __builtin_ldexp(dot16(vin, C), sc);   // beta_t (scaled)
    if (!combine) {
      if (active) Sb[(size_t)t * 16 + y] = w;
    } else {
      const double pr = at * w;
      const double c = row_sum(pr);
      if (ystore) Pb[(size_t)t * a.post_tstride + a.post_off + y] = c != 0.0 ? pr / c : pr;
    }
    const double g = e * w;
    const double s = row_sum(g);
    sc = -exp2_of(s);
    row_gather(g, vin);
  };

  // ---------------- phase A
  if (fwd) {
    for (int t = 0; t < H; t++) fstep(t, false);
  } else {
    for (int t = T - 2; t >= H; t--) bstep(t, false);
  }

  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");

  // ---------------- phase B
  if (fwd) {
    for (int t = H; t < T; t++) fstep(t, true);
    if (active && y == 0) {
      double ll = log(m2) - log(m1) + (double)(e2 - e1) * 0.69314718055994530942;
      if (dead) ll = -DBL_MAX;
      if (a.ll) a.ll[b] = ll;
      if (a.status) a.status[b] = dead ? 1u : 0u;
    }
  } else {
    // beta_{T-1} itself may belong to phase B (only when T == 1, H == 0 ...
    // handled by the forward side reading S[T-1]); continue from H-1 down
    for (int t = (T - 2 < H - 1 ? T - 2 : H - 1); t >= 0; t--) bstep(t, true);
  }
}

size_t chain_fb_lds_bytes(int M, int T) {
  return (size_t)(M + 2) * 16 * sizeof(double) + (size_t)kChainsPerBlock * T;
}

int chain_fb_launch(const ChainArgs& a, hipStream_t stream) {
  const int blocks = (int)((a.B + kChainsPerBlock - 1) / kChainsPerBlock);
  const size_t lds = (chain_fb_lds_bytes(a.M, a.T) + 15) & ~(size_t)15;
  hipLaunchKernelGGL(chain_fb_kernel, dim3(blocks), dim3(kThreads), lds, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
