// chain_ckpt.hip -- forward-backward for 16-state interface chains with
// checkpoints and recomputation instead of the scratch round trip (config 2).
//
// chain_fb_mfma_kernel (chain_mfma.hip) hands every phase-A message to phase
// B through HBM: alpha_t (t < H) and beta_t (t >= H) are written once and read
// once, 256 of its 388 bytes per sequence-step.  Here phase A keeps one
// message in four (checkpoints), and phase B rebuilds each chunk's eight
// messages from two of them -- each checkpoint is one of the chunk's rows and
// seeds a 3-step chain for the other three of its half (two independent
// chains, interleaved) -- on the partner SIMDs, one chunk at a time, in step
// with the filter that consumes them:
//
//   SIMD 0: wave 0 forward filter (alpha, rings, z2)        wave 4 backward posteriors,
//                                                                    chains 8-15
//   SIMD 1: wave 1 backward filter (beta)                    wave 5 forward posteriors,
//                                                                    chains 8-15
//   SIMD 2: wave 2 forward partner (ll; alpha checkpoints    wave 6 recomputes
//           in phase A; posteriors t >= H, chains 0-7)               beta of t >= H
//   SIMD 3: wave 3 backward partner (beta checkpoints         wave 7 recomputes
//           in phase A; posteriors t < H, chains 0-7)                alpha of t < H
//
// (a workgroup's waves go to the CU's SIMDs round robin: wave w on SIMD w % 4).
// The filters keep their SIMD's double-precision pipe to themselves; the
// recompute wave's matrix-core chain shares a SIMD with the partner's in-lane
// normalisation and stores.  HBM per sequence-step: the observation (4 B),
// the posterior (128 B), checkpoints (2 x 32 B: written once, read once).
//
// Phase B rescales sparsely, like phase A (the forward partner sums alpha
// itself for the ll).  Results agree with chain_fb_mfma_kernel's to the last
// bits (tests/test_gpu_ckpt.py) and with the oracle within DESIGN.md's
// tolerances.
// The same recursion as nip.c:1320-1581 (forward_backward_inference), see
// chain_kernels.hip for the derivation.
#include "chain_mfma_core.h"
#include "store_pol.h"

namespace nipamd {

namespace {

constexpr int kCThreads = 512;   // 8 waves, two per SIMD
// Evidence rows 144 B apart: row r starts at bank 36r mod 64, so sixteen
// chains reading sixteen different rows (16 B per lane) conflict at most
// 2-way (a 128-B stride maps every row to bank 0 or 32: 4-way;
// profiles/r02/ck_banks.py)
constexpr int kEtStride = 18;

// Ring layout (one step = 16 chains x 16 states): chain j of row k at
// position j ^ (k & 1), its eight 16-byte pieces XOR-swizzled by j >> 1.
// Every access pattern of this kernel is then free of LDS bank conflicts
// (filter and recompute row writes, the partner's per-chain reads and writes,
// the store pass's per-step reads, the checkpoint reads), where chain_mfma.hip's
// (j & 7) swizzle leaves the partner's reads 2-way.
__device__ __forceinline__ int ck_off(int k, int j, int p) {
  return k * kStepD + ((j ^ (k & 1)) << 4) + ((p ^ ((j >> 1) & 7)) << 1);
}

// diagnostics builds (NIPAMD_WAIT_TIMES): per-wave cycle stamps, a.diag[block][wave][5] =
// phase A, phase-barrier wait, phase B, phase-B barrier waits, SIMD id (HW_ID[5:4])
struct CkDiag {
  unsigned long long t0 = 0, ta = 0, tb = 0;
  unsigned long long x1 = 0, x2 = 0, tx = 0;   // recompute waves: chunk set-up / steps cycles
  bool rc = false;
  WaitAcc wb;
  __device__ __forceinline__ void lap(unsigned long long* acc) {
    if (!NIPAMD_WAIT_TIMES) return;
    const unsigned long long t = __builtin_readcyclecounter();
    if (acc) *acc += t - tx;
    tx = t;
  }
  __device__ __forceinline__ void stamp(unsigned long long& t) {
    if (NIPAMD_WAIT_TIMES) t = __builtin_readcyclecounter();
  }
  __device__ __forceinline__ void write(const ChainArgs& a, int wave, int lane) {
    if (!NIPAMD_WAIT_TIMES || !a.diag || lane != 0) return;
    unsigned long long* d = a.diag + (size_t)blockIdx.x * 40 + wave * 5;
    d[0] = rc ? x1 : ta - t0; d[1] = rc ? x2 : tb - ta; d[2] = __builtin_readcyclecounter() - tb; d[3] = wb.cyc;
    d[4] = (__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3;   // hwreg(HW_REG_HW_ID)
  }
};

// Message recomputation for the other direction's phase-B chunks.  Sub-chain
// h of chunk ci covers the rows 4h..4h+3; its checkpoint is one of them:
//   !FWD (wave 6): beta_t for the forward filter's chunk ci, t = H + 8ci + k, into
//     ring row k; sub-chain h from beta_{H+8ci+4h+3} (its top row: a
//     checkpoint, or beta_{T-1} = 1 written by the backward filter) down;
//   FWD (wave 7): alpha_t for the backward filter's chunk ci, t = H - 1 - 8ci - k,
//     into row k; sub-chain h from alpha_{H-4-8ci-4h} (its lowest t: a
//     checkpoint) up, or from the prior alpha_{-1} where that t is negative.
// A full chunk is then 2 x 3 mat-vecs, not 2 x 4: the matrix-core pipe (64
// cycles per v_mfma_f64_16x16x4, dependent or not: profiles/r03/r03_mb_pipe.txt)
// is what this wave's time is made of.  The two sub-chains of a chunk are
// independent and interleaved.  Each starts from a vector rescaled to sum ~1
// and runs at most three steps without rescaling (phase A's sparse rescaling
// relies on four); the posterior normalisation removes the scale.  The next
// chunk's evidence vectors and the checkpoints two chunks ahead are loaded
// while a chunk runs.
template <bool FWD>
__device__ __forceinline__ void recompute_wave(const ChainArgs& a, const WaveCtx& c, const double* Sw, int lane,
                                               int nchA, int nchB, CkDiag& dg) {
  const int j = lane & 15, g = lane >> 4;
  const int sj = state_of(j & 3, j >> 2);
  const int T = a.T, H = a.H;
  double Aop[4];
#pragma unroll
  for (int r = 0; r < 4; r++) Aop[r] = FWD ? a.A[state_of(g, r) * 16 + sj] : a.A[sj * 16 + state_of(g, r)];
  const v4d prior = load4(a.pi + 2 * g);
  for (int ci = 0; ci < nchA; ci++) barrier_lds();
  dg.stamp(dg.ta);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");                         // the partners' checkpoints
  dg.stamp(dg.tb);

  const int n = FWD ? H : T - H;                 // steps of the consuming filter's phase B
  auto tof = [&](int ci, int k) { return FWD ? H - 1 - 8 * ci - k : H + 8 * ci + k; };   // t of row k
  // the checkpoint row of sub-chain h: backward its top t (clamped to T-1),
  // forward its lowest t (-1: none, the chain starts from the prior)
  auto start = [&](int ci, int h) {
    if (FWD) {
      const int lo = H - 4 - 8 * ci - 4 * h;
      return lo >= 0 ? lo : -1;
    }
    const int ts = H + 8 * ci + 4 * h + 3;
    return ts < T - 1 ? ts : T - 1;
  };
  auto ld = [&](int ci, int h) {
    const double* p = Sw + (long)start(ci < nchB ? ci : nchB - 1, h) * kSStep;
    const v2d u = load_pol<NIPAMD_SCR_NTLD>(reinterpret_cast<const v2d*>(p));
    const v2d w = load_pol<NIPAMD_SCR_NTLD>(reinterpret_cast<const v2d*>(p + 8));
    return v4d{u.x, u.y, w.x, w.y};
  };
  // a chunk's evidence rows
  constexpr int kE = kMChunk;
  // codes two chunks ahead, evidence rows one chunk ahead: no load waits on
  // another load issued in the same chunk
  auto ldC = [&](int ci, int (&C)[kE]) {
    const int cc = ci < nchB ? ci : nchB - 1;
#pragma unroll
    for (int k = 0; k < kE; k++) C[k] = c.codes[tof(cc, k)];
  };
  auto ldE = [&](const int (&C)[kE], v4d (&E)[kE]) {
#pragma unroll
    for (int k = 0; k < kE; k++) E[k] = load4(c.Et + C[k] * c.es);
  };
  auto row = [&](double* slot, int k, const v4d& v) {
    double* L = slot + k * kStepD + ((k & 1) ? c.wodd : 0);
    *reinterpret_cast<double2*>(L + c.wo0) = make_double2(v.x, v.y);
    *reinterpret_cast<double2*>(L + c.wo1) = make_double2(v.z, v.w);
  };
  // one step of a sub-chain: X -> the row's vector, X <- the next input
  auto step = [&](v4d& X, int sc, double* slot, int k, const v4d& e) {
    const v4d u = ldexp4(matvec(Aop, X), sc);
    const v4d p = u * e;
    row(slot, k, FWD ? p : u);
    X = p;
  };
  auto norm_exp = [](const v4d& v) { return -__builtin_amdgcn_frexp_exp(chain_sum(v)); };

  v4d P0 = ld(0, 0), P1 = ld(0, 1), Q0 = ld(1, 0), Q1 = ld(1, 1);
  v4d Ea[kE], Eb[kE];
  int Ca[kE], Cb[kE];
  ldC(0, Ca);
  ldE(Ca, Ea);
  ldC(1, Ca);                                      // chunk 1's codes (Cb: chunk 2's, loaded in chunk 0)
  dg.rc = true;
  auto chunk = [&](int ci, v4d& R0, v4d& R1, const v4d (&E)[kE], v4d (&En)[kE], const int (&Cn)[kE],
                   int (&Cnn)[kE]) {
    dg.lap(nullptr);
    double* slot = c.out + (ci & 1) * kSlotD;
    const v4d cur0 = R0, cur1 = R1;
    R0 = ld(ci + 2, 0);
    R1 = ld(ci + 2, 1);
    // chunk ci + 1's evidence and chunk ci + 2's codes, issued after the
    // first step pair so that no step waits behind them
    auto issue = [&] {
      ldE(Cn, En);
      ldC(ci + 2, Cnn);
    };
    const int rem = n - 8 * ci;                  // rows of this chunk (<= 0: none)
    if (rem >= kMChunk) {
      // the checkpoints are rows 3 and 7 (they sum to ~1, beta_{T-1} = 1 to
      // N: three evidence factors per sub-chain at most, no rescale); rows
      // 2..0 and 6..4 follow, forward in increasing t, backward in decreasing t
      row(slot, 3, cur0);
      row(slot, 7, cur1);
      v4d X0 = FWD ? cur0 : cur0 * E[3], X1 = FWD ? cur1 : cur1 * E[7];
      dg.lap(&dg.x1);
      issue();
#pragma unroll
      for (int q = 2; q >= 0; q--) {
        step(X0, 0, slot, q, E[q]);
        step(X1, 0, slot, q + 4, E[q + 4]);
      }
    } else if (rem > 0) {
      issue();
      // the phase's last chunk: short, or reaching t = T - 1 (rare; plain loops)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int ts = start(ci, h);
        const v4d cur = h ? cur1 : cur0;
        if (FWD) {
          const int hiT = H - 1 - 8 * ci;
          if (hiT - 4 * h < 0) continue;          // no valid row
          if (ts >= 0) row(slot, hiT - ts, cur);  // the checkpoint row
          v4d X = ts >= 0 ? cur : prior;
          int sc = ts >= 0 ? norm_exp(cur) : 0;
          for (int t = ts + 1; t <= hiT - 4 * h; t++) {
            const int k = hiT - t;
            step(X, sc, slot, k, load4(c.Et + c.codes[t] * c.es));
            sc = 0;
          }
        } else {
          const int lo = H + 8 * ci + 4 * h;
          if (lo > T - 1) continue;               // no valid row
          row(slot, ts - (H + 8 * ci), cur);      // the checkpoint row (or beta_{T-1})
          v4d X = cur * load4(c.Et + c.codes[ts] * c.es);
          int sc = norm_exp(X);
          for (int t = ts - 1; t >= lo; t--) {
            step(X, sc, slot, t - (H + 8 * ci), load4(c.Et + c.codes[t] * c.es));
            sc = 0;
          }
        }
      }
    } else {
      issue();
    }
    if (NIPAMD_WAIT_TIMES) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    dg.lap(&dg.x2);
    barrier_lds(&dg.wb);
  };
  for (int ci = 0; ci < nchB; ci += 2) {
    chunk(ci, P0, P1, Ea, Eb, Ca, Cb);
    if (ci + 1 >= nchB) break;
    chunk(ci + 1, Q0, Q1, Eb, Ea, Cb, Ca);
  }
}

// Phase B, one side's chunk ci, chains 8 part .. 8 part + 7 (the side's
// partner takes part 0, a wave on a filter SIMD part 1): normalise(v o o)
// with v from the filter's ring slot and o from the recomputed ring slot
// (lane L: chain 8 part + (L & 7), slot step L >> 3), written over o; then
// each chain's 8 steps leave as one contiguous 1 KB run per store
// instruction (lane L: step L >> 3 in address order, piece L & 7).
template <bool FWD, int PROJ>
__device__ __forceinline__ void norm_store(const ChainArgs& a, const double* fslot, double* rslot, int part,
                                           int lane, long b0, int ci, double* sink) {
  const int T = a.T, H = a.H;
  const int nB = FWD ? T - H : H, tB = FWD ? H : H - 1;
  {
    const int c = 8 * part + (lane & 7), k = lane >> 3;
    double v[16], o[16];
#pragma unroll
    for (int p = 0; p < 8; p++) {
      const double2 x = *reinterpret_cast<const double2*>(fslot + ck_off(k, c, p));
      v[2 * p] = x.x; v[2 * p + 1] = x.y;
      const double2 y = *reinterpret_cast<const double2*>(rslot + ck_off(k, c, p));
      o[2 * p] = y.x; o[2 * p + 1] = y.y;
    }
    double pr[16];
#pragma unroll
    for (int i = 0; i < 16; i++) pr[i] = v[i] * o[i];
    double z0 = pr[0] + pr[1], z1 = pr[2] + pr[3], z2 = pr[4] + pr[5], z3 = pr[6] + pr[7];
    z0 += pr[8] + pr[9]; z1 += pr[10] + pr[11]; z2 += pr[12] + pr[13]; z3 += pr[14] + pr[15];
    const double r = recip((z0 + z1) + (z2 + z3));    // an all-zero row stays zero
    if constexpr (PROJ > 0) {
      // joint interface: each requested variable's marginal straight from the
      // normalised joint posterior -- digit sums in increasing joint-state
      // order, then normalised, as derive.hip's project_digit + its
      // normaliser do on the stored joint (same operations, same bits: a
      // term outside the digit is an fma with 0, one inside an fma with 1,
      // i.e. the same add); the joint itself never leaves the CU.  PROJ
      // accumulators per variable (its cardinality <= PROJ).
      const int t = FWD ? tB + ci * kMChunk + k : tB - ci * kMChunk - k;
      const long b = b0 + c;
      if (ci * kMChunk + k < nB && b < a.B) {
        double* const dst = a.post + (size_t)b * a.post_bstride + (long)t * a.post_tstride;
        double nv[16];
#pragma unroll
        for (int i = 0; i < 16; i++) nv[i] = pr[i] * r;
        for (int jv = 0; jv < a.nproj; jv++) {
          double sd[PROJ > 0 ? PROJ : 1];
#pragma unroll
          for (int d = 0; d < PROJ; d++) sd[d] = 0.0;
#pragma unroll
          for (int i = 0; i < 16; i++) {
            const int dig = a.proj_digit[jv][i];
#pragma unroll
            for (int d = 0; d < PROJ; d++) sd[d] = __builtin_fma(nv[i], dig == d ? 1.0 : 0.0, sd[d]);
          }
          double zm = 0.0;
#pragma unroll
          for (int d = 0; d < PROJ; d++) zm += sd[d];
          const double rz = zm != 0.0 ? 1.0 / zm : 1.0;
          const int card = a.proj_card[jv];
          double* const o = dst + a.proj_off[jv];
#pragma unroll
          for (int d = 0; d < PROJ; d++)
            if (d < card) o[d] = zm != 0.0 ? sd[d] * rz : sd[d];
        }
      }
      return;
    }
#pragma unroll
    for (int p = 0; p < 8; p++)
      *reinterpret_cast<double2*>(rslot + ck_off(k, c, p)) = make_double2(pr[2 * p] * r, pr[2 * p + 1] * r);
  }
  const int s = lane & 7, hi = lane >> 3;
  const int kB = FWD ? hi : kMChunk - 1 - hi;
  const int tlow = FWD ? tB + ci * kMChunk : tB - ci * kMChunk - (kMChunk - 1);
  const int nk = nB - ci * kMChunk < kMChunk ? nB - ci * kMChunk : kMChunk;
  const bool ok = kB < nk;
  double* const base = a.post + (size_t)b0 * a.post_bstride + (long)(tlow + hi) * 16 + a.post_off + 2 * s;
#ifndef NIPAMD_CKPT_NO_STORES
#define NIPAMD_CKPT_NO_STORES 0    // timing-only builds: posteriors not written (wrong results)
#endif
#pragma unroll
  for (int q = 8 * part; q < 8 * part + 8; q++) {
    const double2 v = *reinterpret_cast<const double2*>(rslot + ck_off(kB, q, s));
    double* p = (ok && b0 + q < a.B) ? base + q * a.post_bstride : sink;
    if (NIPAMD_CKPT_NO_STORES && v.x != 12345.0) continue;
    store_pol<NIPAMD_POST_NT>(reinterpret_cast<v2d*>(p), v2d{v.x, v.y});
  }
}

template <bool FWD, int PROJ>
__device__ __forceinline__ void ck_partner(const ChainArgs& a, double* out, double* rring, const double* zr,
                                           double* Sblk, int lane, long b0, int nchA, int nchB, CkDiag& dg) {
  const int T = a.T, H = a.H;
  const int s = lane & 7, hi = lane >> 3;
  const int c = lane & 15, kq = lane >> 4;
  const int nA = FWD ? H : T - 1 - H, nB = FWD ? T - H : H;
  const int tA = FWD ? 0 : T - 2, tB = FWD ? H : H - 1;
  constexpr int dir = FWD ? 1 : -1;

  LL ll;
  if (FWD) ll.init(a, lane, false);
  auto ring_vec = [&](const double* slot, int k, double (&v)[16]) {
#pragma unroll
    for (int p = 0; p < 8; p++) {
      const double2 x = *reinterpret_cast<const double2*>(slot + ck_off(k, c, p));
      v[2 * p] = x.x; v[2 * p + 1] = x.y;
    }
  };
  // phase A: the forward ll (as chain_mfma.hip's partner) and the checkpoints
  auto drainA = [&](int ci) {
    const double* slot = out + (ci & 1) * kSlotD;
    if (FWD) {
      double v0[16], v1[16];
      ring_vec(slot, kq, v0);
      ring_vec(slot, kq + 4, v1);
      const double* zs = zr + (ci & 1) * kMChunk * kMSeq;
      const double za = zs[kq * kMSeq + c], zb = zs[(kq + 4) * kMSeq + c];
      const int i = ci * kMChunk + kq;
      const bool all = ci * kMChunk + kMChunk > nA;
      const bool rs0 = all || (kq & (kRescale - 1)) == kRescale - 1;
      const bool rs1 = all || ((kq + 4) & (kRescale - 1)) == kRescale - 1;
      const int ta = tA + i, tb = tA + i + 4;
      ll.step(ll.dot(v0), LL::sum16(v0), za, rs0, i < nA, ta == T - 1);
      ll.step(ll.dot(v1), LL::sum16(v1), zb, rs1, i + 4 < nA, tb == T - 1);
      ll.renorm();
    }
#pragma unroll
    for (int k = 0; k < kMChunk; k++) {
      const int i = ci * kMChunk + k;
      const int t = tA + dir * i;
      // forward: alpha_{H-4-4m} >= 0; backward: beta_{H+3+4m} <= T-2 (recompute_wave)
      const bool ck = i < nA && (FWD ? (((H - t) & 3) == 0 && t <= H - 4) : (((t - H) & 3) == 3 && t >= H + 3));
      if (!ck) continue;
      // stored rescaled to sum ~1 (the chain's 16 states are the 8 lanes of
      // an aligned DPP row group): a recompute chain starts from it as is
      double2 v[2];
      double z[2];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        v[q] = *reinterpret_cast<const double2*>(slot + ck_off(k, q * 8 + hi, s));
        z[q] = v[q].x + v[q].y;
      }
      sum8_n(z);
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int e = -__builtin_amdgcn_frexp_exp(z[q]);
        store_pol<NIPAMD_SCR_NT>(reinterpret_cast<v2d*>(Sblk + (long)t * kSStep + (q * 8 + hi) * 16 + 2 * s),
                                 v2d{__builtin_ldexp(v[q].x, e), __builtin_ldexp(v[q].y, e)});
      }
    }
  };
  for (int ci = 0; ci < nchA; ci++) {
    if (ci > 0) drainA(ci - 1);
    barrier_lds();
  }
  if (nchA > 0) drainA(nchA - 1);
  dg.stamp(dg.ta);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // phase barrier
  dg.stamp(dg.tb);

  double* const sink = a.S + (size_t)((a.B + kMSeq - 1) / kMSeq) * block_scratch(T) + 2 * s;
  // phase B: the forward ll from the filter's ring (phase B rescales like
  // phase A: z2 summed here, zf published on rescales); posteriors of chains
  // 0-7 of each chunk here, 8-15 on a filter SIMD's spare wave (wave 5
  // forward, wave 4 backward)
  for (int ci = 0; ci < nchB; ci++) {
    barrier_lds(&dg.wb);
    if (FWD) {
      const double* slot = out + (ci & 1) * kSlotD;
      const double* zs = zr + (ci & 1) * kMChunk * kMSeq;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int k = kq + 4 * h;
        double v[16];
        ring_vec(slot, k, v);
        const int i = ci * kMChunk + k;
        const bool rs = ci * kMChunk + kMChunk > nB || (k & (kRescale - 1)) == kRescale - 1;
        ll.step(ll.dot(v), LL::sum16(v), zs[k * kMSeq + c], rs, i < nB, tB + i == T - 1);
      }
      ll.renorm();
    }
    norm_store<FWD, PROJ>(a, out + (ci & 1) * kSlotD, rring + (ci & 1) * kSlotD, 0, lane, b0, ci, sink);
  }
  if (FWD) ll.write(a, b0, lane, 1u);
  barrier_lds();                                     // the block's closing barrier
}

template <int PROJ>
#ifndef NIPAMD_CK_PRIO
// 5: the filters at s_setprio 2, the recompute waves at 1, the partners at 0:
// -1.2% against 3 in 10 of 12 interleaved pairs (profiles/r05/gpu/r05af_ab_fb_prio.txt,
// r05ag_ab_fb_prio.txt; phase B's binding wave is the beta recompute).
// 3: the partners at 1 and the filters at 2: -3.6% against 2 in 5 of 5 pairs
// and 4 of 4 on a second box (r05q_ab_fb.txt, r05o_ab_fb_ckprio3.txt);
// 2: the partners only (round 4)
#define NIPAMD_CK_PRIO 5
#endif
__global__ __launch_bounds__(kCThreads, 1) void chain_fb_ckpt_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* out = reinterpret_cast<double*>(smem);     // filter rings [2 dirs][2 slots][8][16][16]
  double* rr = out + kOutD;                          // recomputed rings [2 dirs][2 slots][8][16][16]
  double* zr = rr + kOutD;                           // [2 slots][8][16]
  double* Et = zr + kZD;                             // [(M+2)][kEtStride]
  uint8_t* codes = reinterpret_cast<uint8_t*>(Et + (a.M + 2) * kEtStride);   // [16][Tr]
  auto nozero = [] {};
  const unsigned long long t_entry = NIPAMD_WAIT_TIMES ? __builtin_readcyclecounter() : 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const long b0 = (long)blockIdx.x * kMSeq;
  const int T = a.T;
  const int Tr = chain_codes_row(T);
  stage_codes<kCThreads, decltype(nozero), kEtStride>(a, b0, tid, Et, codes, Tr, nozero);
  __syncthreads();
  CkDiag dg;
  dg.stamp(dg.t0);

  const int H = a.H;
  const int nA = (H > T - 1 - H ? H : T - 1 - H);
  const int nB = (T - H > H ? T - H : H);
  const int nchA = (nA + kMChunk - 1) / kMChunk, nchB = (nB + kMChunk - 1) / kMChunk;
  double* Sblk = a.S + (size_t)blockIdx.x * block_scratch(T) + kMG * kSStep;   // t = 0
  const int role = wave & 3;
  const bool fwd = (wave & 1) == 0;
  double* ring = out + (fwd ? 0 : 2 * kSlotD);      // the filter's ring of this side
  // recomputed ring consumed with it: the forward side's beta (wave 6), the backward side's alpha (wave 7)
  double* rring = rr + (fwd ? 0 : 2 * kSlotD);
  // waves 4 and 5 (the filters' SIMDs): chains 8-15 of the other side's
  // posteriors -- wave 4 the backward side's, wave 5 the forward side's
  double* const sink = a.S + (size_t)((a.B + kMSeq - 1) / kMSeq) * block_scratch(T) + 2 * (lane & 7);
  if (wave == 4 || wave == 5) {
    const bool f = wave == 5;
    for (int ci = 0; ci < nchA; ci++) barrier_lds();
    dg.stamp(dg.ta);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    dg.stamp(dg.tb);
    const int side = f ? 0 : 2 * kSlotD;
    for (int ci = 0; ci < nchB; ci++) {
      barrier_lds(&dg.wb);
      if (f) norm_store<true, PROJ>(a, out + side + (ci & 1) * kSlotD, rr + side + (ci & 1) * kSlotD, 1, lane, b0, ci, sink);
      else norm_store<false, PROJ>(a, out + side + (ci & 1) * kSlotD, rr + side + (ci & 1) * kSlotD, 1, lane, b0, ci, sink);
    }
    barrier_lds();
    dg.write(a, wave, lane);
    return;
  }
  // A/B builds: static wave priority for the recompute waves (1) or the partners (2)
  // (4: filters 2, partners and recompute waves 1; 5: filters 2, recompute 1,
  // partners 0; 6: filters and recompute waves 2, partners 1)
  if ((NIPAMD_CK_PRIO == 1 && wave >= 6) || ((NIPAMD_CK_PRIO == 2 || NIPAMD_CK_PRIO == 3) && role >= 2 && wave < 4))
    __builtin_amdgcn_s_setprio(1);
  if (NIPAMD_CK_PRIO >= 3 && wave < 2) __builtin_amdgcn_s_setprio(2);
  if ((NIPAMD_CK_PRIO == 4 || NIPAMD_CK_PRIO == 6) && role >= 2 && wave < 4) __builtin_amdgcn_s_setprio(1);
  if ((NIPAMD_CK_PRIO == 4 || NIPAMD_CK_PRIO == 5) && wave >= 6) __builtin_amdgcn_s_setprio(1);
  if (NIPAMD_CK_PRIO == 6 && wave >= 6) __builtin_amdgcn_s_setprio(2);
  if (role >= 2 && wave < 4) {
    if (fwd) ck_partner<true, PROJ>(a, ring, rring, zr, Sblk, lane, b0, nchA, nchB, dg);
    else ck_partner<false, PROJ>(a, ring, rring, zr, Sblk, lane, b0, nchA, nchB, dg);
    dg.write(a, wave, lane);
    return;
  }
  WaveCtx c;
  c.Et = Et + 2 * g;
  c.es = kEtStride;
  c.codes = codes + j * Tr + kMG;
  c.zr = zr;
  c.scr = nullptr;
  c.wo0 = ck_off(0, j, g);
  c.wo1 = ck_off(0, j, 4 + g);
  c.wodd = ck_off(1, j, g) - kStepD - c.wo0;     // = (j & 1) ? -16 : 16, for both pieces
  double* Sw = Sblk + j * 16 + 2 * g;
  if (wave >= 6) {
    c.out = rring;
    c.zw = false;
    if (fwd) recompute_wave<false>(a, c, Sw, lane, nchA, nchB, dg);   // wave 6: beta for the forward side
    else recompute_wave<true>(a, c, Sw, lane, nchA, nchB, dg);        // wave 7: alpha for the backward side
    barrier_lds();
    dg.write(a, wave, lane);
    return;
  }
  c.out = ring;
  c.zw = g == 0;
  if (fwd) filter_wave<true, false, true, 1>(a, c, Et, Sw, lane, true, b0 + j, nchA, nchB, nullptr);
  else filter_wave<false, false, true, 1>(a, c, Et, Sw, lane, true, b0 + j, nchA, nchB, nullptr);
  barrier_lds();
  dg.tb = dg.ta = dg.t0;                             // the filters: total only (slot 2)
  dg.x2 = dg.t0 - t_entry;                           // and the prologue (staging) in slot 1
  dg.rc = true;
  dg.x1 = 0;
  dg.write(a, wave, lane);
}

}  // namespace

size_t chain_fb_ckpt_lds_bytes(int M, int T) {
  return (size_t)(2 * kOutD + kZD) * sizeof(double) + (size_t)(M + 2) * kEtStride * sizeof(double) +
         (size_t)kMSeq * chain_codes_row(T);
}

int chain_fb_ckpt_launch(const ChainArgs& a, hipStream_t stream) {
  const size_t lds = (chain_fb_ckpt_lds_bytes(a.M, a.T) + 15) & ~(size_t)15;
  const bool pvec = a.post && a.N == 16 && a.post_tstride == 16 &&
                    ((a.post_off | (int)(a.post_bstride & 1)) & 1) == 0 &&
                    ((reinterpret_cast<uintptr_t>(a.post) & 15) == 0);
  const bool proj = a.post && a.nproj > 0 && a.nproj <= 4;
  if (lds > 160 * 1024 || !(proj || (pvec && a.nproj == 0)) || a.T < 2) return -2;
  const int blocks = (int)((a.B + kMSeq - 1) / kMSeq);
  if (proj) {
    int cmax = 0;
    for (int jv = 0; jv < a.nproj; jv++) cmax = a.proj_card[jv] > cmax ? a.proj_card[jv] : cmax;
    if (cmax <= 4) {
      static size_t s4[kMaxDevices] = {};
      if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_fb_ckpt_kernel<4>), lds, s4)) return rc;
      hipLaunchKernelGGL(chain_fb_ckpt_kernel<4>, dim3(blocks), dim3(kCThreads), lds, stream, a);
    } else if (cmax <= 8) {
      static size_t s8[kMaxDevices] = {};
      if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_fb_ckpt_kernel<8>), lds, s8)) return rc;
      hipLaunchKernelGGL(chain_fb_ckpt_kernel<8>, dim3(blocks), dim3(kCThreads), lds, stream, a);
    } else {
      static size_t s16[kMaxDevices] = {};
      if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_fb_ckpt_kernel<16>), lds, s16)) return rc;
      hipLaunchKernelGGL(chain_fb_ckpt_kernel<16>, dim3(blocks), dim3(kCThreads), lds, stream, a);
    }
    g_last_kernel = "chain_fb_ckpt_kernel<proj>";
  } else {
    static size_t lds_set[kMaxDevices] = {};
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&chain_fb_ckpt_kernel<0>), lds, lds_set)) return rc;
    hipLaunchKernelGGL(chain_fb_ckpt_kernel<0>, dim3(blocks), dim3(kCThreads), lds, stream, a);
    g_last_kernel = "chain_fb_ckpt_kernel";
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
