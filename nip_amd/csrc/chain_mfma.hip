// chain_mfma.hip -- batched forward-backward on the gfx950 matrix cores.
//
// Same recursion as chain_kernels.hip (see the derivation there, nip.c:1320-
// 1581), laid out for v_mfma_f64_16x16x4_f64: sixteen chains (sequences) of
// one direction share one wavefront, and each step's sixteen 16x16 mat-vecs
// are one 16x16x16 product, D = M' X, done as four chained MFMAs.
//
// Register layout (MI355X_MICROARCH.md, f64 MFMA): D/C lane l, register r =
// element (row (l>>4) + 4r, column l&15); A operand lane l = (row l&15,
// k l>>4); B operand lane l = (k l>>4, column l&15).  Columns are chains
// (j = l&15).  Splitting K = 16 into four MFMAs with k' = (l>>4) + 4r makes
// register r of D exactly the B operand of MFMA r of the next step, so the
// state never leaves the lane.  Internal state i' = g + 4r is stored as
// actual state f(g, r) = 2g + r (r < 2), 8 + 2g + (r - 2) (r >= 2): lane
// (g = l>>4, j) owns states {2g, 2g+1} and {8+2g, 9+2g} of chain j.
//
//   A operand of MFMA r, lane l:  M[f(j & 3, j >> 2)][f(l>>4, r)],  j = l&15
//   with M = A^T (forward: u = A^T alpha)  or  M = A (backward: u = A g)
//
// Sums over a chain's 16 states: three in-lane adds, then v_permlane32_swap
// and v_permlane16_swap exchanges (lanes l, l^32, l^16), each symmetric, so
// all four lanes of a chain hold bit-identical sums.
//
// On gfx950 the f64 MFMA and f64 VALU work share the SIMD's double-precision
// pipe (SQ_VALU_MFMA_COEXEC_CYCLES = 0), so a step costs its MFMA cycles PLUS
// its vector instructions: the compute waves keep only the recursion itself,
// and everything else moves to a partner wave on another SIMD.  Block = 16
// sequences, four waves, one per SIMD:
//   wave 0  forward filter:  alpha_t (scaled) -> LDS ring; ll
//   wave 1  backward filter: beta_t (scaled)  -> LDS ring
//   wave 2  forward partner:  phase A alpha -> HBM scratch;
//                             phase B posterior = normalise(alpha o beta), beta
//                             read from the scratch, -> HBM
//   wave 3  backward partner: the same for the backward half
// The rings hold two 8-step slots per direction; one s_barrier per chunk
// hands a slot from filter to partner.  Phase A / barrier / phase B as the
// 16-lane kernel (two-filter smoothing, the scratch holds alpha_t for t < H,
// beta_t for t >= H).
//
// HBM layouts chosen for streaming: the scratch is block-major,
// S[block][kMG + t][16 chains][16 states], one step of a block = 2 KB
// contiguous; posteriors (the caller's [B][T][N]) are written per chain as
// one contiguous 1 KB run of 8 steps per store instruction when N == 16.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <utility>

#include "chain_kernels.h"
#include "chain_mfma_core.h"
#include "diag.h"

namespace nipamd {

namespace {

// e_step partner context (LDS): the direction's applied-exponent ring, the
// partner's M1 count table, the block's observation codes and evidence table.
struct EsCtx {
  const int* scr;           // [2 slots][kMChunk][16 chains]
  double* H;                // M1 counts [M][16] (this partner's, block sums)
  const uint8_t* codes;     // chain c at codes + c * Tr + kMG
  int Tr;
  const double* Et;         // [(M+2)][16]
};

// e_step, phase B of one partner (nip.c:1925-1967 per sequence, summed over
// the block's 16 sequences).  Per chunk, after the filter's barrier:
//   1. in-lane pass (lane: chain c = L & 15, slot steps kq = L >> 4 and kq + 4),
//      from the ring vector v, the other direction's vector o (LDS-DMA, one
//      chunk ahead, as the fb partner) and the evidence row e of the step:
//      c_t = v . o, the posterior q = v o / c_t (kept in registers), the ll
//      (forward), and the xi operands written back in place:
//        forward  (t >= H):   o <- e o 2^sc_t / c_t           (b of xi_t)
//        backward (t <  H-1): o <- o 2^sc_t / c_t             (a of xi_{t+1})
//                             v <- e o v  (= e_t o beta_t, b of xi_t for step t-1)
//      (xi without the A(x,y) factor, applied once by estep_finalize; sc_t =
//      the exponent the filter applied at t, published per step);
//   2. matrix-core pass (lane: step kq, state y), per chain and 4-step half:
//        xi += a (x) b over the four steps, one v_mfma_f64_16x16x4 (K = time),
//        forward a = alpha_{t-1} (ring, previous step), backward b = e_{t+1} o
//        beta_{t+1} (ring, previous step); the chunk's first step takes the
//        previous chunk's last vector, kept in registers;
//   3. q written over o;
//   4. M1 counts: H[code][y] += q(y), one ds_add_f64 per 16-lane row at a time
//      (rows in a fixed order: no two lanes of an instruction share an
//      address, so the sums are deterministic); missing observations summed
//      apart (row M, split by finalize); P0 = posterior at t = -1 (backward).
// The accumulators are the block's slab row (the tree over blocks replaces
// the tree over sequences: sums of the same terms in a fixed order).
template <bool FWD>
__device__ __forceinline__ void estep_phase_b(const ChainArgs& a, double* out, const double* zr, double* Sblk,
                                              double* ob_lds, int lane, long b0, int nchB, const EsCtx& es,
                                              LL& ll, double (&pv)[kMSeq]) {
  const int T = a.T, H = a.H, M = a.M;
  const int s = lane & 7, hi = lane >> 3;
  const int c = lane & 15, kq = lane >> 4, y = lane & 15;
  const int nB = FWD ? T - H : H + 1;                    // this direction's phase-B steps
  const int tB = FWD ? H : H - 1;
  auto tlow = [&](int ci) { return FWD ? tB + ci * kMChunk : tB - ci * kMChunk - (kMChunk - 1); };
  const unsigned ob_base = (unsigned)(uintptr_t)ob_lds;
  auto dma_other = [&](int k, int ci) {
    const double* q = Sblk + (long)(tlow(ci) + hi) * kSStep + 2 * s;
    dma16(q, __builtin_amdgcn_readfirstlane(ob_base + (unsigned)k * (kMSeq * kOBRow * 8u)),
          std::make_integer_sequence<int, kMSeq>{});
  };
  const int nact = (int)(a.B - b0 < kMSeq ? a.B - b0 : kMSeq);    // sequences present in this block
  const v4d zero4 = {0.0, 0.0, 0.0, 0.0};
  v4d dx0 = zero4, dx1 = zero4;
  v4d hc0 = zero4, hc1 = zero4;                          // M1 count accumulators (D rows = codes)
  double miss = 0.0, p0 = 0.0;
  const uint8_t* cdl = es.codes + c * es.Tr + kMG;       // in-lane pass: chain c's codes
  const int last = nchB > 0 ? nchB - 1 : 0;
  unsigned long long pc[5] = {0, 0, 0, 0, 0}, tc = 0;   // diagnostics: cycles per pass
  auto tick = [&](int k) {
    if (a.diag) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const unsigned long long n = __builtin_readcyclecounter();
      pc[k] += n - tc; tc = n;
    }
  };
  dma_other(0, 0);
  for (int ci = 0; ci < nchB; ci++) {
    dma_other((ci + 1) & 1, ci + 1 < last ? ci + 1 : last);    // over-run reloads the last chunk
    if (a.diag) tc = __builtin_readcyclecounter();
    barrier_lds();
    wait_vm<16>();
    tick(0);
    double* slot = out + (ci & 1) * kSlotD;
    double* obb = ob_lds + (ci & 1) * (kMSeq * kOBRow);
    const int* scs = es.scr + (ci & 1) * kMChunk * kMSeq;
    // 1. in-lane pass
    double q[2][16];
    {
      const double* zs = zr + (ci & 1) * kMChunk * kMSeq;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = kq + 4 * h;
        const int row = FWD ? k : kMChunk - 1 - k;
        const int i = ci * kMChunk + k;
        const int t = FWD ? tB + i : tB - i;
        double* vr = slot + k * kStepD;
        double* orow = obb + c * kOBRow + row * 16;
        const int code = cdl[t];
        const double* er = es.Et + code * 16;
        double v[16], o[16], e[16];
#pragma unroll
        for (int p = 0; p < 8; p++) {
          const double2 x = *reinterpret_cast<const double2*>(vr + piece_off(c, p));
          v[2 * p] = x.x; v[2 * p + 1] = x.y;
          const double2 w = *reinterpret_cast<const double2*>(orow + 2 * p);
          o[2 * p] = w.x; o[2 * p + 1] = w.y;
          const double2 u = *reinterpret_cast<const double2*>(er + 2 * p);
          e[2 * p] = u.x; e[2 * p + 1] = u.y;
        }
        if (FWD) {
          const double zf = zs[k * kMSeq + c];
          ll.step(ll.dot(v), zf, zf, true, i < nB, t == T - 1, code == M, cdl[t + 1] == M);
        }
        double z0 = v[0] * o[0], z1 = v[1] * o[1], z2 = v[2] * o[2], z3 = v[3] * o[3];
#pragma unroll
        for (int p = 4; p < 16; p += 4) {
          z0 = __builtin_fma(v[p], o[p], z0); z1 = __builtin_fma(v[p + 1], o[p + 1], z1);
          z2 = __builtin_fma(v[p + 2], o[p + 2], z2); z3 = __builtin_fma(v[p + 3], o[p + 3], z3);
        }
        const double ct = (z0 + z1) + (z2 + z3);
        const double rc = recip(ct);
        const bool ok = i < nB && c < nact && ct != 0.0;  // a present sequence's step with alpha.beta != 0
        const double fs = __builtin_ldexp(rc, scs[k * kMSeq + c]);
        const bool okx = FWD ? ok : ok && i > 0;          // xi_H belongs to the forward partner
        double w[16];
#pragma unroll
        for (int p = 0; p < 16; p++) {
          q[h][p] = ok ? v[p] * o[p] * rc : 0.0;
          w[p] = okx ? (FWD ? e[p] * o[p] * fs : o[p] * fs) : 0.0;
        }
#pragma unroll
        for (int p = 0; p < 8; p++)
          *reinterpret_cast<double2*>(orow + 2 * p) = make_double2(w[2 * p], w[2 * p + 1]);
        if (!FWD) {
#pragma unroll
          for (int p = 0; p < 8; p++)
            *reinterpret_cast<double2*>(vr + piece_off(c, p)) =
                make_double2(ok ? e[2 * p] * v[2 * p] : 0.0, ok ? e[2 * p + 1] * v[2 * p + 1] : 0.0);
        }
      }
      if (FWD) ll.renorm();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tick(1);
    // 2. xi on the matrix cores
#pragma unroll
    for (int cc = 0; cc < kMSeq; cc++) {
      const int po = piece_off(cc, y >> 1) + (y & 1);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = 4 * h + kq;
        const int row = FWD ? k : kMChunk - 1 - k;
        const double rp = slot[(k > 0 ? k - 1 : 0) * kStepD + po];
        const double ringv = k > 0 ? rp : pv[cc];
        const double dmav = obb[cc * kOBRow + row * 16 + y];
        if (h == 0)
          dx0 = __builtin_amdgcn_mfma_f64_16x16x4f64(FWD ? ringv : dmav, FWD ? dmav : ringv, dx0, 0, 0, 0);
        else
          dx1 = __builtin_amdgcn_mfma_f64_16x16x4f64(FWD ? ringv : dmav, FWD ? dmav : ringv, dx1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int cc = 0; cc < kMSeq; cc++) pv[cc] = slot[(kMChunk - 1) * kStepD + piece_off(cc, y >> 1) + (y & 1)];
    tick(2);
    // 3. posteriors over the xi operands
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int k = kq + 4 * h;
      double* orow = obb + c * kOBRow + (FWD ? k : kMChunk - 1 - k) * 16;
#pragma unroll
      for (int p = 0; p < 8; p++)
        *reinterpret_cast<double2*>(orow + 2 * p) = make_double2(q[h][2 * p], q[h][2 * p + 1]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    tick(3);
    // 4. M1 counts on the matrix cores: H[m][y] += sum over (chain, step) of
    //    [code == m] q(y), one v_mfma_f64_16x16x4 per chain and 4-step half
    //    (K = the half's four steps; A = the one-hot code rows, lane (m = L &
    //    15, step kq); B = the posteriors, lane (step kq, state y)); a fixed
    //    accumulation order, no atomics.  Missing observations summed apart
    //    (row M, split by finalize); P0 = posterior at t = -1 (backward).
#pragma unroll 4
    for (int cc = 0; cc < kMSeq; cc++) {
      const uint8_t* cd = es.codes + cc * es.Tr + kMG;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = 4 * h + kq;
        const int i = ci * kMChunk + k;
        const int t = FWD ? tB + i : tB - i;
        const double qv = obb[cc * kOBRow + (FWD ? k : kMChunk - 1 - k) * 16 + y];
        const int code = cd[t];
        miss += (t >= 0 && code == M) ? qv : 0.0;
        if (!FWD) p0 += t == -1 ? qv : 0.0;
        const double oh = (t >= 0 && code == y && code < M) ? 1.0 : 0.0;
        if (h == 0) hc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(oh, qv, hc0, 0, 0, 0);
        else hc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(oh, qv, hc1, 0, 0, 0);
      }
    }
    tick(4);
  }
  if (a.diag && lane == 0)
    for (int k = 0; k < 5; k++) a.diag[blockIdx.x * 24 + 8 + (FWD ? 0 : 5) + k] = pc[k];
  wait_vm<0>();                      // no DMA left in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // the block's slab row (chain_estep_slab layout, summed over its sequences)
  double* slab = a.counts + (size_t)blockIdx.x * chain_estep_slab(M);
  const v4d dx = dx0 + dx1;
  const int hoff = kSlabH + (FWD ? 0 : (M + 2) * 16);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int x = (lane >> 4) + 4 * r;                   // D row: the previous state
    slab[(FWD ? kSlabKf : kSlabKb) + x * 16 + y] = dx[r];
  }
  const v4d hc = hc0 + hc1;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int m = (lane >> 4) + 4 * r;                   // D row: the observation code
    if (m < M) slab[hoff + m * 16 + y] = hc[r];
  }
  miss = sum_lanes16(sum_lanes32(miss));                  // the four steps kq of state y
  if (!FWD) p0 = sum_lanes16(sum_lanes32(p0));
  if (lane < 16) {
    slab[hoff + M * 16 + y] = miss;
    slab[hoff + (M + 1) * 16 + y] = 0.0;
    if (!FWD) slab[chain_slab_p0(M) + y] = p0;
  }
}

// Partner wave of one direction.
// Phase A: each step's 2 KB of the block's scratch as two contiguous 1 KB
// instructions (lane L: chain q*8 + (L >> 3), piece L & 7); the forward
// partner also keeps the ll.
// Phase B: lane L owns chain c = L & 15 at slot steps k = L >> 4 and k + 4:
// it reads the whole 16-state ring vector and the other direction's vector
// (scratch, by LDS-DMA one chunk ahead), forms normalise(alpha o beta) in
// lane and writes it back over the ring vector; a store pass then sends
// each chain's 8 steps as one contiguous 1 KB run per instruction (lane
// L: step L >> 3 in address order, piece L & 7).  Without the 16-state
// layout (PVEC false) or the LDS-DMA budget, the older 8-lane form is used.
template <bool FWD, bool PVEC, bool DMA, bool ES = false>
__device__ __forceinline__ void partner_wave(const ChainArgs& a, double* out, const double* zr,
                                             double* Sblk, double* ob_lds, int lane, long b0, int nchA, int nchB,
                                             const uint8_t* codes, int Tr, const EsCtx* es = nullptr) {
  const int T = a.T, H = a.H;
  const int s = lane & 7, hi = lane >> 3;
  const int c = lane & 15, kq = lane >> 4;
  constexpr bool pvec = PVEC;        // posterior rows of 16 contiguous, 16-byte aligned doubles
  const int nA = FWD ? H : T - 1 - H, nB = FWD ? T - H : H;
  const int tA = FWD ? 0 : T - 2, tB = FWD ? H : H - 1;
  constexpr int dir = FWD ? 1 : -1;
  const bool st0 = 2 * s < a.N, st1 = 2 * s + 1 < a.N;
  // phase-B geometry of the store lanes: slot step kB, time offset hi in address order
  const int kB = FWD ? hi : kMChunk - 1 - hi;
  auto tlow = [&](int ci) { return FWD ? tB + ci * kMChunk : tB - ci * kMChunk - (kMChunk - 1); };

  // e_step: chain c's codes, for the missing-step pairing of the ll (its
  // em_learn stops on a positive total ll, nip.c:2224-2234); fb keeps the
  // plain products (a missing step there contributes only rounding)
  const uint8_t* lc = codes + c * Tr + kMG;
  auto miss = [&](int t) { return ES && lc[t] == a.M; };
  LL ll;
  if (FWD) ll.init(a, lane, miss(0));
  // chain c's ring vector at slot step k (16 states, in lane)
  auto ring_vec = [&](const double* slot, int k, double (&v)[16]) {
#pragma unroll
    for (int p = 0; p < 8; p++) {
      const double2 x = *reinterpret_cast<const double2*>(slot + k * kStepD + piece_off(c, p));
      v[2 * p] = x.x; v[2 * p + 1] = x.y;
    }
  };
  // forward ll of chunk ci, steps kq and kq + 4: in phase A the filter
  // rescaled every kRescale-th step of full chunks and at every step of a
  // partial one (Chain::run<true>), in phase B (dense) at every step; z2 is
  // summed here
  auto ll_chunk = [&](int ci, int n, int t0, bool dense) {
    const double* slot = out + (ci & 1) * kSlotD;
    const double* zs = zr + (ci & 1) * kMChunk * kMSeq;
    double v0[16], v1[16];
    ring_vec(slot, kq, v0);
    ring_vec(slot, kq + 4, v1);
    const double za = zs[kq * kMSeq + c], zb = zs[(kq + 4) * kMSeq + c];
    const int i = ci * kMChunk + kq;
    const bool all = dense || ci * kMChunk + kMChunk > n;
    const bool rs0 = all || (kq & (kRescale - 1)) == kRescale - 1;
    const bool rs1 = all || ((kq + 4) & (kRescale - 1)) == kRescale - 1;
    const int ta = t0 + i, tb = t0 + i + 4;
    ll.step(ll.dot(v0), LL::sum16(v0), za, rs0, i < n, ta == T - 1, miss(ta), miss(ta + 1));
    ll.step(ll.dot(v1), LL::sum16(v1), zb, rs1, i + 4 < n, tb == T - 1, miss(tb), miss(tb + 1));
    ll.renorm();
  };
  auto drainA = [&](int ci) {
    const double* slot = out + (ci & 1) * kSlotD;
    if (FWD) ll_chunk(ci, nA, tA, false);
#pragma unroll
    for (int k = 0; k < kMChunk; k++) {
      const int i = ci * kMChunk + k;
      if (i >= nA) break;
      const int t = tA + dir * i;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int jj = q * 8 + hi;
        const double2 v = *reinterpret_cast<const double2*>(slot + k * kStepD + piece_off(jj, s));
        *reinterpret_cast<double2*>(Sblk + (long)t * kSStep + jj * 16 + 2 * s) = v;
      }
    }
  };
  WaitAcc wa, wb;
  for (int ci = 0; ci < nchA; ci++) {
    if (ci > 0) drainA(ci - 1);
    barrier_lds(&wa);
  }
  if (nchA > 0) drainA(nchA - 1);
  double pv[kMSeq];                  // e_step: previous step's vectors (lane: state lane & 15)
  if (ES) {
    // the forward partner's first xi (t = H) needs alpha_{H-1}: the last step
    // of phase A in the ring (overwritten by phase B's first chunk), or the
    // prior; the backward partner's first xi operand is unused (zero)
    const int kl = (nA - 1) - (nchA - 1) * kMChunk;
    const double* src = out + ((nchA - 1) & 1) * kSlotD + (kl > 0 ? kl : 0) * kStepD;
    const int yy = lane & 15;
#pragma unroll
    for (int cc = 0; cc < kMSeq; cc++)
      pv[cc] = !FWD ? 0.0 : nA > 0 ? src[piece_off(cc, yy >> 1) + (yy & 1)] : a.pi[yy];
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");

  // spare scratch rows past the last block: target of masked lanes' stores
  double* const sink = a.S + (size_t)((a.B + kMSeq - 1) / kMSeq) * block_scratch(T) + 2 * s;
  unsigned long long pw = 0, pl = 0, pd = 0;     // NIPAMD_WAIT_TIMES: DMA wait / drain / store cycles

  if constexpr (ES) {
    estep_phase_b<FWD>(a, out, zr, Sblk, ob_lds, lane, b0, nchB, *es, ll, pv);
  } else if constexpr (PVEC && DMA) {
    // LDS-DMA prefetch of the other direction's vectors: buffer k, chain C at
    // C * kOBRow doubles, rows = the chunk's 8 steps in address order
    const unsigned ob_base = (unsigned)(uintptr_t)ob_lds;
    auto dma_other = [&](int k, int ci) {
      const double* q = Sblk + (long)(tlow(ci) + hi) * kSStep + 2 * s;
      dma16(q, __builtin_amdgcn_readfirstlane(ob_base + (unsigned)k * (kMSeq * kOBRow * 8u)),
            std::make_integer_sequence<int, kMSeq>{});
    };
    // chain c, slot steps kq and kq + 4: posterior in lane, written over the ring vector
    auto drainV = [&](int ci, int buf) {
      double* slot = out + (ci & 1) * kSlotD;
      const double* ob = ob_lds + buf * (kMSeq * kOBRow) + c * kOBRow;
      const double* zs = zr + (ci & 1) * kMChunk * kMSeq;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = kq + 4 * h;
        const int row = FWD ? k : kMChunk - 1 - k;     // DMA row (address order) of slot step k
        double v[16], o[16];
        ring_vec(slot, k, v);
#pragma unroll
        for (int p = 0; p < 8; p++) {
          const double2 x = *reinterpret_cast<const double2*>(ob + row * 16 + 2 * p);
          o[2 * p] = x.x; o[2 * p + 1] = x.y;
        }
        if (FWD && NIPAMD_MFMA_ABLATE != 14) {
          const int i = ci * kMChunk + k;
          const double zf = zs[k * kMSeq + c];           // phase B: the filter rescales every step
          ll.step(ll.dot(v), zf, zf, true, i < nB, tB + i == T - 1);
        }
        double pr[16];
#pragma unroll
        for (int i = 0; i < 16; i++) pr[i] = v[i] * o[i];
        double z0 = pr[0] + pr[1], z1 = pr[2] + pr[3], z2 = pr[4] + pr[5], z3 = pr[6] + pr[7];
        z0 += pr[8] + pr[9]; z1 += pr[10] + pr[11]; z2 += pr[12] + pr[13]; z3 += pr[14] + pr[15];
        const double r = recip((z0 + z1) + (z2 + z3));    // an all-zero row stays zero
#pragma unroll
        for (int p = 0; p < 8; p++)
          *reinterpret_cast<double2*>(slot + k * kStepD + piece_off(c, p)) = make_double2(pr[2 * p] * r, pr[2 * p + 1] * r);
      }
      if (FWD) ll.renorm();
    };
    // chain q's 8 steps as one contiguous 1 KB run per store instruction
    auto store_pass = [&](int ci) {
      const double* slot = out + (ci & 1) * kSlotD;
      const int nk = nB - ci * kMChunk < kMChunk ? nB - ci * kMChunk : kMChunk;
      const bool ok = kB < nk;
#if NIPAMD_MFMA_NT >= 2
      // buffer stores into this block's rows: a masked lane's offset lies past
      // num_records and the store is dropped; aux 16 = sc1 (write-through)
      const long nq = a.B - b0 < kMSeq ? a.B - b0 : kMSeq;
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(a.post + (size_t)b0 * a.post_bstride, (short)0,
                                                          (int)(nq * a.post_bstride * 8), 0x00020000);
      const int vbase = (int)(((long)(tlow(ci) + hi) * 16 + a.post_off + 2 * s) * 8);
#else
      double* const base = a.post + (size_t)b0 * a.post_bstride + (long)(tlow(ci) + hi) * 16 + a.post_off + 2 * s;
#endif
#pragma unroll
      for (int q = 0; q < kMSeq; q++) {
        const double2 v = *reinterpret_cast<const double2*>(slot + kB * kStepD + piece_off(q, s));
#if NIPAMD_MFMA_ABLATE == 11
        if (v.x == 12345.0)
#endif
#if NIPAMD_MFMA_NT >= 2
        {
          typedef unsigned v4u __attribute__((ext_vector_type(4)));
          const int vo = ok ? vbase + (int)(q * a.post_bstride * 8) : (int)0x80000000;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rsrc, vo, 0,
                                                 NIPAMD_MFMA_NT == 2 ? 16 : 0);
        }
#else
        double* p = (ok && b0 + q < a.B) ? base + q * a.post_bstride : sink;
#if NIPAMD_MFMA_NT
        __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d*>(p));
#else
        *reinterpret_cast<double2*>(p) = v;
#endif
#endif
      }
    };
    // The phase barrier drained every memory operation.  Before the first
    // drain, chunk 1's sixteen DMAs follow chunk 0's (vmcnt 16); before every
    // later drain, its DMAs are followed by the previous chunk's sixteen
    // posterior stores and the next chunk's sixteen DMAs (vmcnt 32): the
    // counter retires loads, stores and DMAs together in issue order.
    const int last = nchB > 0 ? nchB - 1 : 0;
    if (NIPAMD_MFMA_ABLATE != 19) dma_other(0, 0);
    for (int ci = 0; ci < nchB; ci++) {
      if (NIPAMD_MFMA_ABLATE != 19)
        dma_other((ci + 1) & 1, ci + 1 < last ? ci + 1 : last);   // over-run reloads the last chunk
      barrier_lds(&wb);
      const unsigned long long c0 = NIPAMD_WAIT_TIMES ? __builtin_readcyclecounter() : 0;
      if (NIPAMD_MFMA_ABLATE == 19) {}
      else if (ci == 0) wait_vm<16>();
      else wait_vm<32>();
      unsigned long long c1 = 0;
      if (NIPAMD_WAIT_TIMES) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        c1 = __builtin_readcyclecounter();
        pw += c1 - c0;
      }
      if (NIPAMD_MFMA_ABLATE != 17 && NIPAMD_MFMA_ABLATE != 19) {
        drainV(ci, ci & 1);
        if (NIPAMD_WAIT_TIMES) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const unsigned long long c2 = __builtin_readcyclecounter();
          pl += c2 - c1; c1 = c2;
        }
        store_pass(ci);
        if (NIPAMD_WAIT_TIMES) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          pd += __builtin_readcyclecounter() - c1;
        }
      }
    }
    wait_vm<0>();                    // no DMA left in flight
  } else {
    // other direction's vectors of chunk ci, all 16 chains, this lane's piece
    v2d oa[kMSeq], ob[kMSeq];
    auto load_other = [&](v2d (&o)[kMSeq], int ci) {
      const double* q = Sblk + (long)(tlow(ci) + hi) * kSStep + 2 * s;
#pragma unroll
      for (int cc = 0; cc < kMSeq; cc++) o[cc] = *reinterpret_cast<const v2d*>(q + cc * 16);
    };
    auto drainB = [&](int ci, const v2d (&o)[kMSeq]) {
      if (FWD) ll_chunk(ci, nB, tB, true);
      if (!PVEC && !a.post) return;
      const double* slot = out + (ci & 1) * kSlotD;
      const int nk = nB - ci * kMChunk < kMChunk ? nB - ci * kMChunk : kMChunk;   // valid steps
      const bool ok = kB < nk;
      const int t = tlow(ci) + hi;
      if constexpr (pvec) {
        // branch-free, eight chains at a time with their dependency chains interleaved
#pragma unroll
        for (int q0 = 0; q0 < kMSeq; q0 += 8) {
          double px[8], py[8], z[8], r[8];
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const double2 v = *reinterpret_cast<const double2*>(slot + kB * kStepD + piece_off(q0 + i, s));
            px[i] = v.x * o[q0 + i].x; py[i] = v.y * o[q0 + i].y;
            z[i] = px[i] + py[i];
          }
          sum8_n(z);
          recip_n(z, r);                                 // an all-zero row stays zero
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const long bb = b0 + q0 + i;
            double* p = (ok && bb < a.B)
                            ? a.post + (size_t)bb * a.post_bstride + (long)t * 16 + a.post_off + 2 * s
                            : sink;
            *reinterpret_cast<double2*>(p) = make_double2(px[i] * r[i], py[i] * r[i]);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < kMSeq; q++) {
          const double2 v = *reinterpret_cast<const double2*>(slot + kB * kStepD + piece_off(q, s));
          const double px = v.x * o[q].x, py = v.y * o[q].y;
          const double r = recip(sum8(px + py));
          const long bb = b0 + q;
          if (!ok || bb >= a.B) continue;
          double* p = a.post + (size_t)bb * a.post_bstride + (long)t * a.post_tstride + a.post_off + 2 * s;
          if (st0) p[0] = px * r;
          if (st1) p[1] = py * r;
        }
      }
    };
    // chunk ci is drained right after the barrier that ends it, while the
    // filter computes chunk ci + 1; its inputs were loaded one chunk earlier.
    // Prefetches are unconditional (an over-run reloads the last chunk).
    const int last = nchB > 0 ? nchB - 1 : 0;
    load_other(oa, 0);
    for (int ci = 0; ci < nchB; ci += 2) {
      load_other(ob, ci + 1 < last ? ci + 1 : last);
      barrier_lds(&wb);
      drainB(ci, oa);
      if (ci + 1 >= nchB) break;
      load_other(oa, ci + 2 < last ? ci + 2 : last);
      barrier_lds(&wb);
      drainB(ci + 1, ob);
    }
  }
  if (FWD) ll.write(a, b0, lane, ES ? 3u : 1u);   // e_step: BAD_LUCK (nip.c:1827-1854)
  if (!ES && NIPAMD_WAIT_TIMES && a.counts && lane == 0) {
    unsigned long long* st = reinterpret_cast<unsigned long long*>(a.counts) + (size_t)gridDim.x * 4;
    st[blockIdx.x * 8 + 2 + (FWD ? 0 : 1)] = wa.cyc;
    st[blockIdx.x * 8 + 6 + (FWD ? 0 : 1)] = wb.cyc;
    unsigned long long* pp = reinterpret_cast<unsigned long long*>(a.counts) + (size_t)gridDim.x * 16;
    pp[blockIdx.x * 8 + (FWD ? 0 : 4) + 0] = pw;
    pp[blockIdx.x * 8 + (FWD ? 0 : 4) + 1] = pl;
    pp[blockIdx.x * 8 + (FWD ? 0 : 4) + 2] = pd;
  }
}

constexpr int kOBD = 2 * 2 * kMSeq * kOBRow;       // DMA buffers [2 partners][2][16 chains][1 KB + 16 B pad]

// e_step extras after the evidence table: applied-exponent rings [2 dirs][2][8][16]
// (ints), the partners' M1 count tables [2][M][16]
constexpr int kEsScrI = 2 * 2 * kMChunk * kMSeq;


template <bool DMA, bool ES>
__global__ __launch_bounds__(kMThreads, 1)
void chain_fb_mfma_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* out = reinterpret_cast<double*>(smem);                      // [2 dirs][2 slots][8][16][16]
  double* zr = out + kOutD;                                          // [2 slots][8][16]
  double* obuf = zr + kZD;                                           // DMA ? [2][2][16][128] : none
  double* Et = obuf + (DMA ? kOBD : 0);                              // [(M+2)][16]
  int* scr = reinterpret_cast<int*>(Et + (a.M + 2) * 16);            // ES: [2 dirs][2][8][16]
  double* Hc = reinterpret_cast<double*>(scr + (ES ? kEsScrI : 0));  // ES: [2][M][16]
  uint8_t* codes = reinterpret_cast<uint8_t*>(Hc + (ES ? 2 * a.M * 16 : 0));   // [16][Tr]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const long b0 = (long)blockIdx.x * kMSeq;
  // diagnostics (fb only): a.counts carries the stamp buffer
  unsigned long long* rts = (!ES && a.counts) ? reinterpret_cast<unsigned long long*>(a.counts) + (size_t)gridDim.x * 12
                                              : nullptr;     // wall-clock stamps
  if (rts && tid == 0) {
    rts[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memrealtime();
    rts[blockIdx.x * 4 + 1] = __builtin_readcyclecounter();
  }
  const int T = a.T;
  const int Tr = chain_codes_row(T);
  if (ES) diag_stamp(a, 0, tid);

  // --- stage the evidence table and the 16 sequences' observation codes
  stage_codes<kMThreads>(a, b0, tid, Et, codes, Tr, [&] {
    if (ES) {   // e_step: ring slots a partial chunk leaves unwritten stay finite; counts start at 0
      for (int i = tid; i < kOutD / 2; i += kMThreads) reinterpret_cast<double2*>(out)[i] = make_double2(0.0, 0.0);
      for (int i = tid; i < 2 * a.M * 16; i += kMThreads) Hc[i] = 0.0;
    }
  });
  __syncthreads();

  if (ES) diag_stamp(a, 1, tid);
  // optional phase timestamps (a.counts != nullptr in fb: NIPAMD_PHASE_TIMES)
  unsigned long long* stamps = ES ? nullptr : reinterpret_cast<unsigned long long*>(a.counts);
  if (stamps && tid == 0) stamps[blockIdx.x * 4 + 0] = __builtin_readcyclecounter();
  const int H = a.H;
  const int nA = (H > T - 1 - H ? H : T - 1 - H);
  const int nB = ES ? (T - H > H + 1 ? T - H : H + 1) : (T - H > H ? T - H : H);
  const int nchA = (nA + kMChunk - 1) / kMChunk, nchB = (nB + kMChunk - 1) / kMChunk;
  const bool fwd = (wave & 1) == 0;
  double* ring = out + (fwd ? 0 : 2 * kSlotD);
  int* scr_d = scr + (fwd ? 0 : kEsScrI / 2);
  double* Sblk = a.S + (size_t)blockIdx.x * block_scratch(T) + kMG * kSStep;   // t = 0
  if (wave >= 2) {
    double* ob = obuf + (fwd ? 0 : kOBD / 2);
    if constexpr (ES) {
      EsCtx es;
      es.scr = scr_d;
      es.H = Hc + (fwd ? 0 : a.M * 16);
      es.codes = codes;
      es.Tr = Tr;
      es.Et = Et;
      if (fwd) partner_wave<true, true, true, true>(a, ring, zr, Sblk, ob, lane, b0, nchA, nchB, codes, Tr, &es);
      else partner_wave<false, true, true, true>(a, ring, zr, Sblk, ob, lane, b0, nchA, nchB, codes, Tr, &es);
      diag_stamp(a, fwd ? 5 : 6, lane);
      return;
    } else {
      const bool pvec = a.post && a.N == 16 && a.post_tstride == 16 &&
                        ((a.post_off | (int)(a.post_bstride & 1)) & 1) == 0 &&
                        ((reinterpret_cast<uintptr_t>(a.post) & 15) == 0);
      if (pvec) {
        if (fwd) partner_wave<true, true, DMA>(a, ring, zr, Sblk, ob, lane, b0, nchA, nchB, codes, Tr);
        else partner_wave<false, true, DMA>(a, ring, zr, Sblk, ob, lane, b0, nchA, nchB, codes, Tr);
      } else {
        if (fwd) partner_wave<true, false, false>(a, ring, zr, Sblk, ob, lane, b0, nchA, nchB, codes, Tr);
        else partner_wave<false, false, false>(a, ring, zr, Sblk, ob, lane, b0, nchA, nchB, codes, Tr);
      }
      if (rts && fwd && lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rts[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
        rts[blockIdx.x * 4 + 3] = __builtin_readcyclecounter();
      }
      return;
    }
  }
  const long b = b0 + j;
  const bool active = b < a.B;
  double* Sw = Sblk + j * 16 + 2 * g;          // inactive chains compute garbage, never stored
  WaveCtx c;
  c.Et = Et + 2 * g;
  c.codes = codes + j * Tr + kMG;
  c.out = ring;
  c.zr = zr;
  c.scr = ES ? scr_d : nullptr;
  c.zw = g == 0;
  c.wo0 = piece_off(j, g);
  c.wo1 = piece_off(j, 4 + g);
  if (fwd) filter_wave<true, ES>(a, c, Et, Sw, lane, active, b, nchA, nchB, stamps);
  else filter_wave<false, ES>(a, c, Et, Sw, lane, active, b, nchA, nchB, nullptr);
  if (ES) diag_stamp(a, fwd ? 3 : 4, lane);
  if (stamps && tid == 0) stamps[blockIdx.x * 4 + 3] = __builtin_readcyclecounter();
}

}  // namespace

size_t chain_mfma_lds_bytes(int M, int T) {       // without the DMA buffers
  return (size_t)(kOutD + kZD) * sizeof(double) + (size_t)(M + 2) * 16 * sizeof(double) +
         (size_t)kMSeq * chain_codes_row(T);
}

size_t chain_estep_mfma_lds_bytes(int M, int T) {
  return chain_mfma_lds_bytes(M, T) + (size_t)kOBD * sizeof(double) + (size_t)kEsScrI * sizeof(int) +
         (size_t)2 * M * 16 * sizeof(double);
}

namespace {
template <bool DMA, bool ES>
int launch_mfma(const ChainArgs& a, size_t lds, hipStream_t stream) {
  static size_t lds_set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_fb_mfma_kernel<DMA, ES>), lds, lds_set)) return rc;
  const int blocks = (int)((a.B + kMSeq - 1) / kMSeq);
  hipLaunchKernelGGL((chain_fb_mfma_kernel<DMA, ES>), dim3(blocks), dim3(kMThreads), lds, stream, a);
  g_last_kernel = ES ? "chain_fb_mfma_kernel<estep>" : "chain_fb_mfma_kernel";
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace

int chain_fb_mfma_launch(const ChainArgs& a, hipStream_t stream) {
  // 16-wide posterior rows: the checkpoint + recompute kernel (chain_ckpt.hip)
  // unless NIPAMD_FB_KERNEL=scratch asks for this file's scratch round trip
  static const bool ckpt = [] {
    const char* e = diag_env("NIPAMD_FB_KERNEL");
    return !(e && std::strcmp(e, "scratch") == 0);
  }();
  if (ckpt) {
    const int rc = chain_fb_ckpt_launch(a, stream);
    if (rc != -2) return rc;
  }
  const size_t base = (chain_mfma_lds_bytes(a.M, a.T) + 15) & ~(size_t)15;
  const size_t with_dma = base + (size_t)kOBD * sizeof(double);
  if (NIPAMD_MFMA_DMA && NIPAMD_MFMA_ABLATE != 12 && with_dma <= 160 * 1024)
    return launch_mfma<true, false>(a, with_dma, stream);
  return launch_mfma<false, false>(a, base, stream);
}

int chain_estep_mfma_launch(const ChainArgs& a, hipStream_t stream) {
  const size_t lds = (chain_estep_mfma_lds_bytes(a.M, a.T) + 15) & ~(size_t)15;
  if (lds > 160 * 1024 || a.N > 16 || a.M > 16 || !a.counts) return -2;
  return launch_mfma<true, true>(a, lds, stream);
}

}  // namespace nipamd
