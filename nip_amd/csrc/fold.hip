// fold.hip -- the interface chain's transition on the GPU: the in-clique's
// hidden independent parents summed out under their priors,
//
//   A[x][y]     = sum_h  original[x, h, y] * prod_k prior_k(h_k)        (keep = -1)
//   G_j[g][x][y] = the same sum restricted to h_j = g                    (keep = j)
//
// (compile.cpp build_chain_plan / hidden_table, which do it on the host for
// small cliques).  The reference never folds: it multiplies and marginalises
// the whole in-clique potential every time slice (nip_update_potential /
// nip_general_marginalise over the clique, src/nippotential.c:267-311,
// 436-496); this contraction is that marginalisation done once per model
// version, for config 5's 64^4-entry {X0, Y1, Z1, X1} a 134 MB stream.
//
// Mapping: one wave per output (x, y) -- or (g, x, y) -- and 16 waves per
// block on consecutive values of the faster of x / y, so the waves of a
// block read adjacent doubles of the same cache lines; lanes walk the hidden
// combinations h = lane + 64 i in the host loop's order (the first hidden
// parent fastest), whose (offset, weight) table the block stages in LDS.
// Each lane keeps four partial sums in a fixed order, the wave combines them
// by a fixed butterfly: deterministic, and HBM-bound (every entry read once).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "model.h"

namespace nipamd {

namespace {

constexpr int kFoldWaves = 16;          // outputs per block
constexpr long kFoldLdsMax = 4096;      // table entries staged in LDS (64 KB)

struct FoldArgs {
  const double* T;        // the in-clique's original_p (dimension 0 fastest)
  const long* off;        // [G][R] offset of each hidden combination
  const double* w;        // [G][R] its prior weight
  long R;                 // combinations per output group
  int G;                  // output groups (the kept parent's card, or 1)
  int N;
  long sx, sy;            // strides of prev (x) and cur (y)
  int xfast;              // x is the faster of the two (waves of a block step x)
  int lds;                // the block's table slice is staged in LDS
  double* out;            // [G][64][64]
};

template <int K>
__device__ __forceinline__ double ror(double v) {     // row_ror:K of a double
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x120 + K, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// sum over the wave in a fixed order (every lane ends with the same bits)
__device__ __forceinline__ double wave_sum(double x) {
  asm("" : "+v"(x));       // one rounded value per lane: no fma contraction into the first add
  x += ror<8>(x);
  x += ror<4>(x);
  x += ror<2>(x);
  x += ror<1>(x);
  {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    x = __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
  }
  {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    x = __hiloint2double((int)rh[0], (int)rl[0]) + __hiloint2double((int)rh[1], (int)rl[1]);
  }
  return x;
}

__global__ __launch_bounds__(kFoldWaves * 64, 1)
void fold_kernel(FoldArgs f) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long nout = (long)f.G * f.N * f.N;
  const long o0 = (long)blockIdx.x * kFoldWaves;
  const long o = o0 + wave;
  const int g = (int)(o / ((long)f.N * f.N));
  const long* off = f.off + (size_t)g * f.R;
  const double* w = f.w + (size_t)g * f.R;
  if (f.lds) {                  // every wave of the block shares group g (host-checked)
    const int g0 = (int)(o0 / ((long)f.N * f.N));
    long* so = reinterpret_cast<long*>(smem);
    double* sw = reinterpret_cast<double*>(smem + f.R * sizeof(long));
    for (long i = tid; i < f.R; i += kFoldWaves * 64) {
      so[i] = f.off[(size_t)g0 * f.R + i];
      sw[i] = f.w[(size_t)g0 * f.R + i];
    }
    __syncthreads();
    off = so;
    w = sw;
  }
  if (o >= nout) return;
  const int fast = (int)(o % f.N), slow = (int)((o / f.N) % f.N);
  const int x = f.xfast ? fast : slow, y = f.xfast ? slow : fast;
  const double* base = f.T + x * f.sx + y * f.sy;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  long h = lane;
  for (; h + 192 < f.R; h += 256) {
    const double t0 = base[off[h]], t1 = base[off[h + 64]], t2 = base[off[h + 128]], t3 = base[off[h + 192]];
    a0 = __builtin_fma(t0, w[h], a0);
    a1 = __builtin_fma(t1, w[h + 64], a1);
    a2 = __builtin_fma(t2, w[h + 128], a2);
    a3 = __builtin_fma(t3, w[h + 192], a3);
  }
  for (int r = 0; h < f.R; h += 64, r++) {
    const double t = base[off[h]] * w[h];
    if (r == 0) a0 += t; else if (r == 1) a1 += t; else a2 += t;
  }
  const double s = wave_sum((a0 + a1) + (a2 + a3));
  if (lane == 0) f.out[((size_t)g * 64 + x) * 64 + y] = s;
}

// When prev or cur is the clique's fastest dimension (config 5: X0), lanes
// span that dimension instead -- every wave load is 64 consecutive doubles --
// each lane owning its own output; the 16 waves of a block and HG blocks
// split the hidden combinations, summed in a fixed order (waves in LDS, then
// fold_sum_kernel over the HG partials).
struct FoldLaneArgs {
  const double* T;
  const long* off;        // [G][R]
  const double* w;
  long R;
  int G, N, HG;           // groups, card(prev) = card(cur), hidden-combination groups
  long sl, so;            // strides of the lane dimension and of the other output dimension
  int lane_is_x;
  double* part;           // [G][HG][64][64]
};

__global__ __launch_bounds__(kFoldWaves * 64, 1)
void fold_lane_kernel(FoldLaneArgs f) {
  __shared__ double red[kFoldWaves][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hg = (int)(blockIdx.x % f.HG);
  const int ov = (int)((blockIdx.x / f.HG) % f.N);
  const int g = (int)(blockIdx.x / ((long)f.HG * f.N));
  const long Rg = (f.R + f.HG - 1) / f.HG;
  const long h0 = hg * Rg, h1 = h0 + Rg < f.R ? h0 + Rg : f.R;
  const long* off = f.off + (size_t)g * f.R;
  const double* w = f.w + (size_t)g * f.R;
  const double* base = f.T + (lane < f.N ? lane : 0) * f.sl + ov * f.so;
  // eight 512-byte loads in flight per wave (wave-uniform h: scalar table
  // loads), four accumulators in a fixed order
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  long h = h0 + wave;
  for (; h + 7 * kFoldWaves < h1; h += 8 * kFoldWaves) {
    double t[8];
#pragma unroll
    for (int k = 0; k < 8; k++) t[k] = base[off[h + k * kFoldWaves]];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k & 3] = __builtin_fma(t[k], w[h + k * kFoldWaves], a[k & 3]);
  }
  for (int k = 0; h < h1; h += kFoldWaves, k++) a[k & 3] = __builtin_fma(base[off[h]], w[h], a[k & 3]);
  red[wave][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (wave == 0) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kFoldWaves; k++) s += red[k][lane];
    if (lane < f.N) {
      const int x = f.lane_is_x ? lane : ov, y = f.lane_is_x ? ov : lane;
      f.part[(((size_t)g * f.HG + hg) * 64 + x) * 64 + y] = s;
    }
  }
}

// out[g][x][y] = sum over hg of part[g][hg][x][y], hg in order
__global__ void fold_sum_kernel(const double* part, int G, int HG, double* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)G * 4096) return;
  const long g = i / 4096, xy = i % 4096;
  double s = 0.0;
  for (int k = 0; k < HG; k++) s += part[((size_t)g * HG + k) * 4096 + xy];
  out[i] = s;
}

struct FoldPlan {
  int cin = -1, N = 0;
  long sx = 0, sy = 0;
  std::vector<long> stride;   // per hidden parent
  std::vector<int> card;
  long hsize = 1;
  long n = 0;                 // entries of the in-clique
};

FoldPlan plan_of(const Model& m) {
  const ChainPlan& P = m.chain;
  FoldPlan f;
  f.cin = P.c_trans;
  f.N = P.N;
  const auto& cv = m.cliques[f.cin].vars;
  std::vector<long> st(m.vars.size(), 0);
  long s = 1;
  for (int v : cv) { st[v] = s; s *= m.vars[v].card; }
  f.n = s;
  f.sx = st[P.v_prev];
  f.sy = st[P.v_cur];
  for (int h : P.hidden) {
    f.stride.push_back(st[h]);
    f.card.push_back(m.vars[h].card);
    f.hsize *= m.vars[h].card;
  }
  return f;
}

#define FOLD_OK(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); goto done; } \
  } while (0)

}  // namespace

long chain_fold_entries(const Model& m) {
  const ChainPlan& P = m.chain;
  if (P.c_trans < 0) return 0;
  return (long)m.cliques[P.c_trans].original.size();
}

// keep = -1: out = A [64][64]; keep = j: out = G_j [card_j][64][64].  Runs on
// the current device and returns when the result is on the host; *ms = the
// fold kernel's time (HIP events), *bytes = the clique entries it streamed.
int chain_fold_gpu(const Model& m, int keep, std::vector<double>& out, double* ms, double* bytes, std::string& err) {
  const ChainPlan& P = m.chain;
  if (!P.valid && P.c_trans < 0) { err = "no interface-chain plan"; return -1; }
  const FoldPlan f = plan_of(m);
  const int K = (int)f.card.size();
  if (keep >= K) { err = "bad hidden parent"; return -1; }
  const int G = keep >= 0 ? f.card[keep] : 1;
  const long R = f.hsize / G;
  // (offset, weight) of every combination in the host loop's order
  // (build_chain_plan: hidden parent 0 fastest, weight = prod_k prior_k in k
  // order), grouped by the kept parent's value
  std::vector<long> off((size_t)f.hsize);
  std::vector<double> w((size_t)f.hsize);
  {
    std::vector<long> fill(G, 0);
    std::vector<int> hv(K, 0);
    for (long hi = 0; hi < f.hsize; hi++) {
      long r = hi, o = 0;
      double ww = 1.0;
      for (int k = 0; k < K; k++) {
        hv[k] = (int)(r % f.card[k]); r /= f.card[k];
        o += hv[k] * f.stride[k];
        ww *= m.vars[P.hidden[k]].prior[hv[k]];
      }
      const int g = keep >= 0 ? hv[keep] : 0;
      const size_t at = (size_t)g * R + fill[g]++;
      off[at] = o;
      w[at] = ww;
    }
  }
  out.assign((size_t)G * 64 * 64, 0.0);
  double* dT = nullptr; long* dOff = nullptr; double* dW = nullptr; double* dOut = nullptr;
  double* dPart = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = -1;
  {
    const auto& T = m.cliques[f.cin].original;
    FOLD_OK(hipMalloc(&dT, T.size() * sizeof(double)));
    FOLD_OK(hipMalloc(&dOff, off.size() * sizeof(long)));
    FOLD_OK(hipMalloc(&dW, w.size() * sizeof(double)));
    FOLD_OK(hipMalloc(&dOut, out.size() * sizeof(double)));
    FOLD_OK(hipMemcpy(dT, T.data(), T.size() * sizeof(double), hipMemcpyHostToDevice));
    FOLD_OK(hipMemcpy(dOff, off.data(), off.size() * sizeof(long), hipMemcpyHostToDevice));
    FOLD_OK(hipMemcpy(dW, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice));
    FOLD_OK(hipMemset(dOut, 0, out.size() * sizeof(double)));
    const long nout = (long)G * f.N * f.N;
    // lanes over prev or cur when it is the clique's fastest dimension
    const bool lane_x = f.sx == 1, lane_y = f.sy == 1;
    FOLD_OK(hipEventCreate(&e0));
    FOLD_OK(hipEventCreate(&e1));
    if ((lane_x || lane_y) && f.N >= 32) {
      FoldLaneArgs a{};
      a.T = dT; a.off = dOff; a.w = dW; a.R = R; a.G = G; a.N = f.N;
      long hg = (1024 + (long)G * f.N - 1) / ((long)G * f.N);  // >= 1024 blocks of 16 waves
      hg = std::max(1L, std::min(hg, R / (2 * kFoldWaves)));
      a.HG = (int)hg;
      a.sl = lane_x ? f.sx : f.sy;
      a.so = lane_x ? f.sy : f.sx;
      a.lane_is_x = lane_x ? 1 : 0;
      FOLD_OK(hipMalloc(&dPart, (size_t)G * a.HG * 4096 * sizeof(double)));
      FOLD_OK(hipMemset(dPart, 0, (size_t)G * a.HG * 4096 * sizeof(double)));
      a.part = dPart;
      FOLD_OK(hipEventRecord(e0, nullptr));
      hipLaunchKernelGGL(fold_lane_kernel, dim3((unsigned)((long)G * f.N * a.HG)), dim3(kFoldWaves * 64), 0,
                         nullptr, a);
      FOLD_OK(hipGetLastError());
      hipLaunchKernelGGL(fold_sum_kernel, dim3((unsigned)((G * 4096 + 255) / 256)), dim3(256), 0, nullptr,
                         (const double*)dPart, G, a.HG, dOut);
      FOLD_OK(hipGetLastError());
    } else {
      FoldArgs a{};
      a.T = dT; a.off = dOff; a.w = dW; a.R = R; a.G = G; a.N = f.N;
      a.sx = f.sx; a.sy = f.sy; a.xfast = f.sx <= f.sy ? 1 : 0;
      a.out = dOut;
      a.lds = (R <= kFoldLdsMax && ((long)f.N * f.N) % kFoldWaves == 0) ? 1 : 0;
      const size_t lds = a.lds ? (size_t)R * (sizeof(long) + sizeof(double)) : 0;
      if (lds > 65536)
        FOLD_OK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fold_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      FOLD_OK(hipEventRecord(e0, nullptr));
      hipLaunchKernelGGL(fold_kernel, dim3((unsigned)((nout + kFoldWaves - 1) / kFoldWaves)),
                         dim3(kFoldWaves * 64), lds, nullptr, a);
      FOLD_OK(hipGetLastError());
    }
    FOLD_OK(hipEventRecord(e1, nullptr));
    FOLD_OK(hipMemcpy(out.data(), dOut, out.size() * sizeof(double), hipMemcpyDeviceToHost));
    float t = 0.0f;
    FOLD_OK(hipEventElapsedTime(&t, e0, e1));
    if (ms) *ms = t;
    if (bytes) *bytes = (double)R * G * f.N * f.N * sizeof(double);
    rc = 0;
  }
done:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(dT); (void)hipFree(dOff); (void)hipFree(dW); (void)hipFree(dOut); (void)hipFree(dPart);
  return rc;
}

}  // namespace nipamd
