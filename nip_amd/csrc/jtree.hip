// jtree.hip -- gfx950 kernels of the general join-tree engine (jtree.h).
//
// A "unit" is L lanes (16 or 64) of a 64-lane wave working on one sequence
// (filters) or one (sequence, time range) (posterior sweep); a block is one
// wave holding 64/L units that run the same schedule in lock step, so the
// only synchronisation is the wave's own barrier.  Inside a unit, clique
// entries are strided over the lanes: the factor multiply of a clique is one
// pass over its table (up to kJtMaxFac factors fused, nip_update_potential /
// nip_update_evidence, src/nippotential.c:436-522), and a marginalisation
// (nip_general_marginalise, :267-311) gives each sepset entry to a team of
// lanes that sums its pre-image and reduces by butterfly shuffles -- fixed
// order, no atomics.  Working tables live in LDS when the unit's workspace
// fits (64 KB per wave), else in an HBM workspace slot per unit.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "chain_kernels.h"
#include "jtree.h"
#include "nip_amd.h"

namespace nipamd {
namespace {

// the units of a wave run the schedule in lock step and share nothing with
// other waves: a wave-level fence orders their workspace traffic (a wave's
// LDS operations execute in program order; the fence waits for its global
// ones), no block barrier (round 6: several waves per block share the staged
// pools, and units of one wave may skip an output at different steps)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// the plan's pools in LDS (once per block, before any unit starts; the
// workspace units follow them), or read from global memory as uploaded
__device__ __forceinline__ double* stage_pools(const JtRun& r, JtPlanDev& P, double* lds) {
  if (!r.stage) return lds;
  int* ip = reinterpret_cast<int*>(lds);
  double* dp = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (((size_t)P.n_ip * sizeof(int) + 15) & ~(size_t)15));
  for (int i = threadIdx.x; i < P.n_ip; i += blockDim.x) ip[i] = P.ip[i];
  for (int i = threadIdx.x; i < P.n_dp; i += blockDim.x) dp[i] = P.dp[i];
  __syncthreads();
  P.ip = ip;
  P.dp = dp;
  return dp + P.n_dp;
}

// sum over the L lanes of a unit (every lane receives the total)
template <int L>
__device__ __forceinline__ double unit_sum(double v) {
  asm("" : "+v"(v));       // one rounded value per lane: no fma contraction into the first add
#pragma unroll
  for (int o = L / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// dst[j] = sum of src over the pre-image of j (D entries of R = size / D each)
template <int L>
__device__ void marg(const double* src, int size, const int* __restrict__ pre, int D, double* dst,
                     int sub) {
  const int R = size / D;
  if (D >= L) {
    for (int j = sub; j < D; j += L) {
      const int* p = pre + (long)j * R;
      double s = 0.0;
      for (int r = 0; r < R; r++) s += src[p[r]];
      dst[j] = s;
    }
    return;
  }
  int G = L;
  while (G * D > L) G >>= 1;           // team of G lanes per entry (power of two)
  const int j = sub / G, g = sub % G;
  double s = 0.0;
  if (j < D) {
    const int* p = pre + (long)j * R;
    for (int r = g; r < R; r += G) s += src[p[r]];
  }
  for (int o = G / 2; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (j < D && g == 0) dst[j] = s;
}

// the clique's working table = base x its factors (fused passes)
template <int L>
__device__ void visit_factors(const JtPlanDev& P, const JtVisit& v, double* ws,
                              const int32_t* orow, int sub) {
  const JtFac* F = reinterpret_cast<const JtFac*>(P.ip + P.fac) + v.fac0;
  const int* maps = P.ip + P.maps;
  const int nf = v.nfac;
  for (int f0 = 0; f0 == 0 || f0 < nf; f0 += kJtMaxFac) {
    int kind[kJtMaxFac], code[kJtMaxFac];
    const int* map[kJtMaxFac];
    const double* vec[kJtMaxFac];
#pragma unroll
    for (int k = 0; k < kJtMaxFac; k++) {
      kind[k] = -1; code[k] = 0; map[k] = maps; vec[k] = ws;
      if (f0 + k < nf) {
        const JtFac f = F[f0 + k];
        map[k] = maps + f.proj;
        if (f.kind == kJtFacObs) {
          const int c = orow ? orow[f.arg] : -1;
          if (c >= 0) { kind[k] = 0; code[k] = c; }   // missing (< 0): nothing entered (nip.c:994)
        } else {
          kind[k] = 1;
          vec[k] = ws + f.arg;
        }
      }
    }
    const double* src = f0 == 0 ? P.dp + v.base : ws + v.psi;
    for (int i = sub; i < v.size; i += L) {
      double x = src[i];
#pragma unroll
      for (int k = 0; k < kJtMaxFac; k++) {
        if (kind[k] == 0) x = map[k][i] == code[k] ? x : 0.0;   // one-hot evidence
        else if (kind[k] == 1) x *= vec[k][map[k][i]];
      }
      ws[v.psi + i] = x;
    }
    wave_sync();
  }
}

// one collect sweep (post-order); the root's table ends in ws[root.psi]
template <int L>
__device__ void collect(const JtPlanDev& P, const JtVisit* V, double* ws, const int32_t* orow, int sub) {
  const int* pres = P.ip + P.pres;
  for (int c = 0; c < P.ncl; c++) {
    const JtVisit v = V[c];
    visit_factors<L>(P, v, ws, orow, sub);
    if (v.up_proj >= 0) {
      marg<L>(ws + v.psi, v.size, pres + v.up_proj, v.up_D, ws + v.up_msg, sub);
      wave_sync();
    }
  }
}

// x[0..n) /= sum (no-op if the sum is 0: nip_normalise_array, nippotential.c:349-359);
// returns the sum
template <int L>
__device__ double normalise(double* x, int n, int sub) {
  double s = 0.0;
  for (int j = sub; j < n; j += L) s += x[j];
  s = unit_sum<L>(s);
  if (s != 0.0)
    for (int j = sub; j < n; j += L) x[j] /= s;
  wave_sync();
  return s;
}

// a unit's workspace: in LDS, or its own HBM slot -- per block of the whole
// grid, blockIdx.y included (the two filter directions run as blockIdx.y = 0
// and 1 of one launch; the host sizes wsg for 2 x r.gunits slots)
template <bool LDS>
__device__ __forceinline__ double* unit_ws(const JtRun& r, double* lds, int u, int U) {
  if (LDS) return lds + (long)u * r.p.ws;
  return r.wsg + (((long)blockIdx.y * gridDim.x + blockIdx.x) * U + u) * r.p.ws;
}

// units of the block: 64 / L per wave
template <int L>
__device__ __forceinline__ int block_units() { return (int)(blockDim.x / L); }

// any evidence entered at this step (a step without any contributes exactly 0
// to ll; DESIGN.md 6, the missing-value note)
__device__ __forceinline__ bool row_has_evidence(const int32_t* orow, int nobs) {
  for (int c = 0; c < nobs; c++) if (orow[c] >= 0) return true;
  return false;
}

// ---------------------------------------------------------------------------
// filters: blockIdx.y = direction (0 forward, 1 backward) + dir_base
template <int L, bool LDS>
__global__ __launch_bounds__(256) void jt_filter_kernel(JtRun r, int dir_base) {
  extern __shared__ double lds[];
  const int U = block_units<L>();
  const int u = threadIdx.x / L, sub = threadIdx.x % L;
  const int dir = dir_base + (int)blockIdx.y;
  JtPlanDev P = r.p;
  double* const wsl = stage_pools(r, P, lds);
  double* ws = unit_ws<LDS>(r, wsl, u, U);
  const int K = P.K;
  const JtVisit* V = reinterpret_cast<const JtVisit*>(P.ip + (dir == 0 ? P.fwd : P.bwd));
  const int* pres = P.ip + P.pres;
  for (long b0 = (long)blockIdx.x * U; b0 < r.B; b0 += (long)gridDim.x * U) {
    const long b = b0 + u;
    const bool act = b < r.B;
    const long bc = act ? b : r.B - 1;
    const int32_t* obs = r.obs ? r.obs + bc * r.obs_bstride : nullptr;
    if (dir == 0) {
      for (int j = sub; j < K; j += L) ws[P.ws_alpha + j] = P.dp[P.pi_off + j];
      wave_sync();
      double ll = 0.0;
      unsigned st = 0;
      for (int t = 0; t < r.T; t++) {
        const int32_t* orow = obs ? obs + (long)t * r.obs_tstride : nullptr;
        double m1 = 0.0;
        for (int j = sub; j < K; j += L) m1 += ws[P.ws_alpha + j] * P.dp[P.w_off + j];
        m1 = unit_sum<L>(m1);
        collect<L>(P, V, ws, orow, sub);
        marg<L>(ws + P.fwd_root_psi, P.fwd_root_size, pres + P.fwd_root_proj, K, ws + P.ws_out, sub);
        wave_sync();
        double m2 = 0.0;
        for (int j = sub; j < K; j += L) m2 += ws[P.ws_out + j];
        m2 = unit_sum<L>(m2);
        // start_timeslice_message_pass: alpha_t = normalise(marginal)  (nip.c:1031-1065)
        double* ga = r.msgA + (bc * r.T + t) * (long)K;
        for (int j = sub; j < K; j += L) {
          const double a = m2 != 0.0 ? ws[P.ws_out + j] / m2 : ws[P.ws_out + j];
          ws[P.ws_alpha + j] = a;
          if (act && t + 1 < r.T) ga[j] = a;
        }
        // ll = sum log m2 - log m1 (nip.c:1458-1474; e_step's checks :1827-1854)
        const bool ev = orow && row_has_evidence(orow, r.nobs);
        if (ev && m1 > 0.0 && m2 > 0.0) ll += log(m2) - log(m1);
        if (m2 == 0.0) { ll = -DBL_MAX; st |= NIPAMD_STATUS_ZERO_MASS; }
        if (r.estep && (m1 <= 0.0 || m2 <= 0.0 || ll > 0.0)) st |= NIPAMD_STATUS_BAD_LUCK;
        wave_sync();
      }
      if (act && sub == 0) {
        if (r.ll) r.ll[b] = ll;
        if (r.status) r.status[b] = st;
      }
    } else {
      for (int j = sub; j < K; j += L) ws[P.ws_beta + j] = 1.0;
      wave_sync();
      for (int t = r.T - 1; t >= 1; t--) {
        const int32_t* orow = obs ? obs + (long)t * r.obs_tstride : nullptr;
        collect<L>(P, V, ws, orow, sub);
        marg<L>(ws + P.bwd_root_psi, P.bwd_root_size, pres + P.bwd_root_proj, K, ws + P.ws_out, sub);
        wave_sync();
        double s = 0.0;
        for (int j = sub; j < K; j += L) s += ws[P.ws_out + j];
        s = unit_sum<L>(s);
        double* gb = r.msgB + (bc * r.T + (t - 1)) * (long)K;
        for (int j = sub; j < K; j += L) {
          const double x = s != 0.0 ? ws[P.ws_out + j] / s : ws[P.ws_out + j];
          ws[P.ws_beta + j] = x;
          if (act) gb[j] = x;
        }
        wave_sync();
      }
    }
  }
}

// m1 weights: the backward sweep of an evidence-free slice with beta = 1,
// unnormalised: w(I_{t-1}) = mass of the slice given the previous interface
template <int L, bool LDS>
__global__ __launch_bounds__(64) void jt_w_kernel(JtRun r, double* w_out) {
  extern __shared__ double lds[];
  constexpr int U = 64 / L;                 // one wave, pools from global memory (r.stage == 0)
  const int u = threadIdx.x / L, sub = threadIdx.x % L;
  const JtPlanDev& P = r.p;
  double* ws = unit_ws<LDS>(r, lds, u, U);
  const JtVisit* V = reinterpret_cast<const JtVisit*>(P.ip + P.bwd);
  for (int j = sub; j < P.K; j += L) ws[P.ws_beta + j] = 1.0;
  wave_sync();
  collect<L>(P, V, ws, nullptr, sub);
  marg<L>(ws + P.bwd_root_psi, P.bwd_root_size, P.ip + P.pres + P.bwd_root_proj, P.K, ws + P.ws_out, sub);
  wave_sync();
  if (u == 0)
    for (int j = sub; j < P.K; j += L) w_out[j] = ws[P.ws_out + j];
}

// ---------------------------------------------------------------------------
// posterior sweep: unit = (sequence, chunk of r.chunk steps)
template <int L, bool LDS>
__global__ __launch_bounds__(256) void jt_post_kernel(JtRun r) {
  extern __shared__ double lds[];
  const int U = block_units<L>();
  const int u = threadIdx.x / L, sub = threadIdx.x % L;
  JtPlanDev P = r.p;
  double* const wsl = stage_pools(r, P, lds);
  double* ws = unit_ws<LDS>(r, wsl, u, U);
  const int K = P.K;
  const JtVisit* V = reinterpret_cast<const JtVisit*>(P.ip + P.post);
  const JtDown* Dn = reinterpret_cast<const JtDown*>(P.ip + P.down);
  const JtOut* O = reinterpret_cast<const JtOut*>(P.ip + P.out);
  const int* pres = P.ip + P.pres;
  const int* maps = P.ip + P.maps;
  const long nch = (r.T + r.chunk - 1) / r.chunk;
  const long units = r.B * nch;
  for (long u0 = (long)blockIdx.x * U; u0 < units; u0 += (long)gridDim.x * U) {
    const long un = u0 + u;
    const bool act = un < units;
    const long uc = act ? un : units - 1;
    const long b = uc / nch;
    const int t0 = (int)(uc % nch) * r.chunk;
    const int t1 = min(r.T, t0 + r.chunk);
    const int32_t* obs = r.obs ? r.obs + b * r.obs_bstride : nullptr;
    if (r.estep) {
      for (int j = sub; j < P.slab; j += L) ws[P.ws_slab + j] = 0.0;
    }
    // all units of the wave run the same number of steps (uniform barriers)
    const int nsteps = r.chunk;
    for (int k = 0; k < nsteps; k++) {
      const int t = t0 + k;
      const bool live = t < t1;
      const int tc = live ? t : t1 - 1;
      const int32_t* orow = obs ? obs + (long)tc * r.obs_tstride : nullptr;
      // interface messages: alpha_{t-1} (the previous interface's prior at t = 0,
      // use_priors, nip.c:88-119) and beta_t (1 at the last step / when filtering)
      const double* ga = tc == 0 ? P.dp + P.pi_off : r.msgA + (b * r.T + (tc - 1)) * (long)K;
      const bool ones = r.filter || tc == r.T - 1;
      const double* gb = r.msgB + (b * r.T + tc) * (long)K;
      for (int j = sub; j < K; j += L) {
        ws[P.ws_alpha + j] = ga[j];
        ws[P.ws_beta + j] = ones ? 1.0 : gb[j];
      }
      wave_sync();
      collect<L>(P, V, ws, orow, sub);
      // Hugin distribute: child *= marg(parent) / old sepset (0 where old is 0)
      for (int e = 0; e < P.ndown; e++) {
        const JtDown d = Dn[e];
        marg<L>(ws + d.p_psi, d.p_size, pres + d.pS_proj, d.S_D, ws + d.tmp, sub);
        wave_sync();
        const int* cm = maps + d.cS_proj;
        for (int i = sub; i < d.c_size; i += L) {
          const int j = cm[i];
          const double old = ws[d.mu + j];
          const double x = ws[d.c_psi + i] * ws[d.tmp + j];
          ws[d.c_psi + i] = old != 0.0 ? x / old : 0.0;
        }
        wave_sync();
      }
      // outputs from the family cliques (nip.c:1535-1552; e_step :1925-1967)
      for (int q = 0; q < P.nout; q++) {
        const JtOut o = O[q];
        if (r.estep && o.t0_only && tc > 0) continue;
        marg<L>(ws + o.psi, o.size, pres + o.proj, o.D, ws + P.ws_out, sub);
        wave_sync();
        normalise<L>(ws + P.ws_out, o.D, sub);
        if (r.estep) {
          if (live)
            for (int j = sub; j < o.D; j += L) ws[P.ws_slab + o.dst + j] += ws[P.ws_out + j];
        } else if (act && live) {
          double* dst = r.post + b * r.post_bstride + (long)tc * r.post_tstride + o.dst;
          for (int j = sub; j < o.D; j += L) dst[j] = ws[P.ws_out + j];
        }
        wave_sync();
      }
    }
    if (r.estep && act) {
      double* s = r.slabs + un * (long)P.slab;     // one slab row per unit: (sequence, time chunk)
      for (int j = sub; j < P.slab; j += L) s[j] = ws[P.ws_slab + j];
    }
    wave_sync();
  }
}

__global__ void jt_add_kernel(const double* __restrict__ src, double* __restrict__ dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] += src[i];
}

// the block: r.waves waves (1 unless the pools are staged), its LDS the
// staged pools and, with LDS workspaces, every unit's workspace
template <int L, bool LDS>
static size_t block_lds(const JtRun& r, int U) {
  return (r.stage ? jt_stage_bytes(r.p) : 0) + (LDS ? (size_t)U * r.p.ws * sizeof(double) : 0);
}

template <int L, bool LDS>
int filter_launch(const JtRun& r, int dirs, hipStream_t st) {
  const int W = r.stage ? r.waves : 1, U = W * (64 / L);
  long blocks = (r.B + U - 1) / U;
  if (!LDS && blocks > r.gunits / U) blocks = r.gunits / U;
  const size_t shm = block_lds<L, LDS>(r, U);
  static size_t set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&jt_filter_kernel<L, LDS>), shm, set)) return rc;
  const int dir_base = dirs == 2 ? 0 : (dirs == 0 ? 0 : 1);   // dirs: 0 fwd only, 1 bwd only, 2 both
  hipLaunchKernelGGL((jt_filter_kernel<L, LDS>), dim3((unsigned)blocks, dirs == 2 ? 2 : 1), dim3(64 * W),
                     shm, st, r, dir_base);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int L, bool LDS>
int post_launch(const JtRun& r, hipStream_t st) {
  const int W = r.stage ? r.waves : 1, U = W * (64 / L);
  const long nch = (r.T + r.chunk - 1) / r.chunk;
  long blocks = (r.B * nch + U - 1) / U;
  if (!LDS && blocks > r.gunits / U) blocks = r.gunits / U;
  const size_t shm = block_lds<L, LDS>(r, U);
  static size_t set[kMaxDevices] = {};
  if (int rc = ensure_dyn_lds(reinterpret_cast<const void*>(&jt_post_kernel<L, LDS>), shm, set)) return rc;
  hipLaunchKernelGGL((jt_post_kernel<L, LDS>), dim3((unsigned)blocks), dim3(64 * W), shm, st, r);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

int jt_filter_launch(const JtRun& r, int L, bool lds, int dirs, hipStream_t st) {
  g_last_kernel = "jt_filter_kernel + jt_post_kernel";
  if (L == 16) return lds ? filter_launch<16, true>(r, dirs, st) : filter_launch<16, false>(r, dirs, st);
  if (L == 32) return lds ? filter_launch<32, true>(r, dirs, st) : filter_launch<32, false>(r, dirs, st);
  return lds ? filter_launch<64, true>(r, dirs, st) : filter_launch<64, false>(r, dirs, st);
}

int jt_post_launch(const JtRun& r, int L, bool lds, hipStream_t st) {
  if (L == 16) return lds ? post_launch<16, true>(r, st) : post_launch<16, false>(r, st);
  if (L == 32) return lds ? post_launch<32, true>(r, st) : post_launch<32, false>(r, st);
  return lds ? post_launch<64, true>(r, st) : post_launch<64, false>(r, st);
}

int jt_w_launch(const JtRun& r, double* w_out, int L, hipStream_t st) {
  // one block; its workspace is the first global slot
  if (L == 16)
    hipLaunchKernelGGL((jt_w_kernel<16, false>), dim3(1), dim3(64), 0, st, r, w_out);
  else if (L == 32)
    hipLaunchKernelGGL((jt_w_kernel<32, false>), dim3(1), dim3(64), 0, st, r, w_out);
  else
    hipLaunchKernelGGL((jt_w_kernel<64, false>), dim3(1), dim3(64), 0, st, r, w_out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int jt_add_launch(const double* src, double* dst, int n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jt_add_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
