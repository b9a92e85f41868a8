// chain_kernels.h -- launch interface of the gfx950 chain (HMM-shaped slice) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdlib>

#include "diag.h"

namespace nipamd {

// Launchers return 0, kLaunchRefused when the host refuses the request before
// anything is queued (a shape or an LDS budget the kernel does not take), or
// -1 when a HIP call fails.  The engine reports a refusal as
// NIPAMD_ERROR_UNSUPPORTED with the kernel's name and a HIP failure as
// NIPAMD_ERROR_DEVICE (engine.cpp launch_fail).
constexpr int kLaunchRefused = -2;
constexpr size_t kLdsPerCU = 160 * 1024;

// The dynamic-LDS limit of a kernel is a per-device attribute: raise it on
// the current device when a launch needs more than the default 64 KB,
// remembering (per kernel, per device) the largest value already set.  More
// than a CU holds is a refusal.  Diagnostics builds: NIPAMD_LDS_CAP (bytes)
// lowers that bound, so that tests can force a refusal through the C ABI.
constexpr int kMaxDevices = 64;
inline int ensure_dyn_lds(const void* kernel, size_t lds, size_t (&set)[kMaxDevices]) {
  size_t cap = kLdsPerCU;
  if (const char* e = diag_env("NIPAMD_LDS_CAP")) cap = (size_t)std::strtoull(e, nullptr, 10);
  if (lds > cap) return kLaunchRefused;
  if (lds <= 65536) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return -1;
  if (lds <= set[dev]) return 0;
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -1;
  set[dev] = lds;
  return 0;
}

// Name of the dominant kernel of the library's last hot-path launch (set by
// the launch functions; nipamd_last_kernel), for measurement labels.
extern const char* g_last_kernel;

struct ChainArgs {
  const int* obs;        // int32 observations
  long obs_bstride;      // elements between sequences
  int obs_tstride;       // elements between time steps (= n_obs)
  int obs_col;           // column of the observed variable
  long B;
  int T, H, N, M;        // H = T / 2: split point of the two filter phases
  const double* A;       // [16][16]  A[x*16 + y]
  const double* Etab;    // [(M+2)][16]
  const double* pi;      // [16]
  const double* ts;      // [16]
  double* S;             // scratch, chain_scratch_bytes(B, T)
  double* post;          // posterior output
  long post_bstride;     // elements between sequences
  int post_tstride;      // elements between time steps
  int post_off;          // offset of the variable's block within a step
  double* ll;            // [B] or nullptr
  unsigned* status;      // [B] or nullptr
  double* counts;        // E-step only: per-sequence slabs [B][chain_estep_slab(M)]
  unsigned long long* diag;   // diagnostics builds only: per-block wall-clock stamps, else null
  // chain_estep16_kernel, one evidence table per leaf child of the plan
  // (ChainPlan::emits, at most 4): its column in obs (-1: never observed, the
  // code is always "missing"), cardinality and first row in Etab / the count
  // tables (rows M_k + 2 each; a.M + 2 = their sum)
  int ne;
  int ecol[4], eM[4], erow[4];
  // chain_estep16_kernel: the transition's rows and every child's rows sum to
  // 1 (to 1e-15): the missing mass m1_t equals the previous step's mass, so
  // the ll telescopes to log(final mass) and neither per-step sum is needed
  int proper;
  // chain_fb_ckpt_kernel, joint interface: write the marginals of up to four of
  // its variables instead of the joint posterior (post_tstride = their summed
  // cardinalities).  proj_digit[j][i]: variable j's value at joint state i (-1
  // for a padding state); its marginal goes to proj_off[j] .. + proj_card[j].
  int nproj;
  int proj_off[4], proj_card[4];
  signed char proj_digit[4][16];
};

// Scratch layout: per sequence kGuard + T + kGuard steps of 16 doubles
// (alpha_t for t < H, beta_t for t >= H), plus one sink row after the last
// sequence for lanes that must not write.  Guards let prefetch over-run.
constexpr int kScratchGuard = 16;   // >= 2 chunks: the deepest prefetch over-run
__host__ __device__ inline long chain_scratch_row(int T) { return (long)(T + 2 * kScratchGuard) * 16; }
__host__ __device__ inline int chain_codes_row(int T) { return ((T + 7) & ~7) + 2 * kScratchGuard; }
// (B rounded up to the matrix-core kernel's 16-sequence blocks, plus two spare rows)
inline size_t chain_scratch_bytes(long B, int T) {
  return (size_t)(((B + 15) & ~15L) + 2) * chain_scratch_row(T) * sizeof(double);
}

// E-step per-sequence slab (doubles): Kf[16][16], Kb[16][16] (xi sums of the
// forward / backward rows, without the A factor), H[2][M+2][16] (M1 count
// tables of the two rows), P0[16].
constexpr int kSlabKf = 0, kSlabKb = 256, kSlabH = 512;
__host__ __device__ inline int chain_estep_slab(int M) { return 512 + 2 * (M + 2) * 16 + 16; }
__host__ __device__ inline int chain_slab_p0(int M) { return 512 + 2 * (M + 2) * 16; }

struct ChainFinalize {
  int N, M;
  int off_prev, off_cur, off_obs;   // em_learn layout offsets of the three families
  const double* A;                  // [16][16]
  const double* Etab;               // [(M+2)][16]
};

// wide interface chains (chain_wide.hip): N <= 64 states, up to 4 observed children
struct WideArgs {
  const int* obs;        // int32 observations [B][T][n_obs]
  long obs_bstride;      // elements between sequences
  int obs_tstride;       // elements between time steps
  int ncol;              // observed children used (columns)
  int col[4];            // their columns in obs
  int M[4];              // their cardinalities
  const double* tab[4];  // [(M+2)][64] per column: E, then the row sums, then 0
  const double* ebase;   // [64] product of the unobserved children's row sums
  long B;
  int T, H, N;
  const double* A;       // [64][64]
  const double* pi;      // [64]
  const double* s;       // [64] m1 weights: product of all children's row sums
  double* S;             // scratch [B][T + 2G][64]
  double* post;
  long post_bstride;
  int post_tstride;
  int post_off;
  double* ll;
  unsigned* status;
  int filter;            // forward_inference: H = 0, filtered posteriors, no scratch reads
  unsigned long long* diag;   // diagnostics builds only (chain_wide4): per-block cycle counts, else null
};
__host__ __device__ inline long chain_scratch_row64(int T) { return (long)(T + 2 * kScratchGuard) * 64; }
size_t chain_wide_lds_bytes(int ncol, int T);
int chain_wide_launch(const WideArgs& a, hipStream_t stream);
// 33..64 states, four filter waves per direction (chain_wide4.hip); -2: LDS does not fit
size_t chain_wide4_lds_bytes(const WideArgs& a);
int chain_wide4_launch(const WideArgs& a, hipStream_t stream);

// matrix-core interface chains (chain_mfma_wide.hip): N <= 16 * NT states (NT = 1, 2),
// up to four observed children, 16 sequences per 4-wave block
struct WideMfmaArgs {
  const int* obs;        // int32 observations [B][T][n_obs]
  long obs_bstride;
  int obs_tstride;
  int ncol;              // observed children (0: evidence = the unobserved row sums only)
  int col[4];
  int M[4];
  int tab_off[4];        // doubles: column k's table [(M_k + 2)][16 NT] within tab
  int tab_rows;          // total rows of tab (>= 2)
  const double* tab;     // column 0 carries the unobserved children's row sums
  long B;
  int T, H, N;
  const double* A;       // [64][64]
  const double* pi;      // [64]
  const double* w;       // [64] = A s_all (ll weights)
  double* S;             // chain_mfma_wide_scratch_bytes
  double* post;
  long post_bstride;
  int post_tstride;
  int post_off;
  double* ll;
  unsigned* status;
  unsigned long long* diag;   // stamps builds (NIPAMD_WAIT_TIMES): per block [4 waves][4] cycles, else null
};
size_t chain_mfma_wide_lds_bytes(int NT, int tab_rows, int ncol, int T);
size_t chain_mfma_wide_scratch_bytes(int NT, long B, int T);
// filter_only: forward_inference (filtered posteriors + ll), requires H == T, no scratch
// beyond one sink row (S needs >= 64 doubles)
int chain_mfma_wide_launch(const WideMfmaArgs& a, int NT, bool filter_only, hipStream_t stream);

// marginals of the chain's other variables from the interface variable's
// (derive.hip): the previous-slice copy, a hidden parent, a leaf child
// kDeriveProject: a joint interface's variable, the digit (prev_stride,
// prev_card) of the joint posterior
enum : int { kDerivePrev = 0, kDeriveChild = 1, kDeriveHidden = 2, kDeriveProject = 3 };
struct DeriveArgs {
  int kind;
  int filter;            // 1: forward_inference marginals (cur = filtered)
  long B;
  int T, N;
  const double* cur;     // the interface variable's marginals [B][T] rows
  long cur_bstride;
  int cur_tstride;
  const double* alpha;   // its filtered marginals (the forward messages); = cur when filtering
  long al_bstride;
  int al_tstride;
  double* out;
  long out_bstride;
  int out_tstride;
  int out_off;
  const double* A;       // [64][64]
  const double* pi;      // [64]
  const int* obs;        // the request's evidence (e_t of filtering)
  long obs_bstride;
  int obs_tstride;
  int ncol;
  int col[4];
  int M[4];
  const double* tab[4];  // [(M+2)][64] per observed column
  const double* ebase;   // [64]
  int child_col;         // kDeriveChild: the child's column in obs, or -1
  int child_M;
  const double* child_E; // [(M+1)][64]: E, then the row sums
  int hid_card;          // kDeriveHidden
  const double* G;       // [card][64][64]
  int prev_stride;       // kDerivePrev of a joint interface / kDeriveProject: the variable's digit
  int prev_card;         // of the joint state (state / stride % card); prev_card 0: the whole interface
};
int derive_launch(const DeriveArgs& a, hipStream_t stream);

// generate_data (generate.hip): one sampling step per variable, in sampling
// order.  In the first slice the conditional row of step i starts at
// tab[off0 + idx], idx = sum_c value(ctx[c]) * stride[c] (in elements) with
// value(j) = this slice's draw of step j (j >= 0) or the previous slice's
// draw of the interface variable (j = -1); later slices use off1 / ctx1 /
// stride1.
constexpr int kGenMaxCtx = 6;
constexpr int kGenMaxVars = 64;
struct GenStep {
  int card = 0;
  int nctx = 0, nctx1 = 0;
  long off0 = 0, off1 = 0;
  int ctx[kGenMaxCtx] = {}, ctx1[kGenMaxCtx] = {};
  long stride[kGenMaxCtx] = {}, stride1[kGenMaxCtx] = {};
};
struct GenArgs {
  int B = 0, T = 0, nv = 0;
  int x1_step = 0;                  // the step drawing the interface variable
  const GenStep* steps = nullptr;   // [nv] device
  const double* tab = nullptr;      // device tables
  long zero_off = 0;                // an all-zero row (>= every card)
  const double* cum = nullptr;      // running row sums of tab (same offsets)
  long cum_n = 0;                   // their size (doubles)
  const uint32_t* win = nullptr;    // [B][31] rand() state of each series
  const int* draws = nullptr;       // or the rand() values themselves, [B][T][nv]
  int* out = nullptr;               // [B][T][nv] draws, sampling-order columns
  int stage = 1;                    // slices buffered in LDS per store burst (launch sets it)
};
int generate_launch(const GenArgs& a, hipStream_t stream);
// win [B][31] from qd_base = {x^D mod (x^31 - x^28 - 1) [31], r[313..373] [61]}
int rand_window_launch(int B, const uint32_t* qd_base, uint32_t* win, hipStream_t stream);

// e_step of interface chains up to 64 states (estep_wide.hip): the two
// filters store every message (chain_msgs_kernel), then the xi sums, the
// children's count tables and P0 per 16-sequence block on the matrix cores
// (chain_stats_kernel), one slab row per block:
//   K [NP][NP] (xi sums without the transition factor), H [R][NP] (every
//   plan child's rows M_k + 2, concatenated), P0 [NP];  NP = 16, 32 or 64
struct EWideArgs {
  const int* obs;        // int32 observations [B][T][n_obs]
  long obs_bstride;
  int obs_tstride;
  int ncol;              // observed children (their evidence)
  int col[4];            // their columns in obs
  int M[4];
  const double* tab;     // [(M_k + 2)][64] per observed child, concatenated
  int tab_off[4];        // doubles: child column k's table within tab
  const double* ebase;   // [64] the unobserved children's row sums
  const double* s;       // [64] m1 weights: every child's row sum
  const double* A;       // [64][64]
  const double* pi;      // [64]
  long B;
  int T, N;
  double* Sa;            // [B][T][NP] alpha^_t
  double* Sb;            // [B][T + 1][NP] beta^_{t-1} at row t
  int* Ea;               // [B][T] exponent of alpha^_t
  double* ll;
  unsigned* status;
  double* slab;          // [ceil(B / 16)][slab_size]
  int slab_size;
  int R;                 // count-table rows: sum over the plan's children of M_k + 2
  int nchild;            // the plan's leaf children (count tables)
  int ccol[4];           // their columns in obs, or -1 (never observed: always missing)
  int cM[4];
  int erow[4];           // first count-table row of each
  int proper;            // rows of A and of every child sum to 1 (engine.cpp chain_proper): the
                         // ll from the final forward mass, no per-step masses in the filters
};
int estep_wide_np(int N);
int estep_wide_slab(int N, int R);
bool estep_wide_fits(int N, int R);
size_t estep_wide_scratch_bytes(int N, long B, int T);
int estep_wide_launch(const EWideArgs& a, hipStream_t stream);

// fused matrix-core e_step for interface chains of 17..32 states (estep_mw.hip,
// round 5): chain_mfma_wide_kernel's block (two groups of 16 sequences, a
// matrix-core filter and a partner wave per direction and group), whose
// partners form the e_step's three sums in phase B on the matrix cores
// instead of writing posteriors -- the messages never leave the chip beyond
// the phase-A scratch round trip.  Writes the wide slab (estep_wide_slab,
// NP = 32) one row per 16 sequences.
struct EMwArgs {
  const int* obs;        // int32 observations [B][T][n_obs]
  long obs_bstride;
  int obs_tstride;
  int ncol;              // observed children (evidence columns, 0: the row sums only)
  int col[4], M[4];
  int tab_off[4];        // doubles: column k's table [(M_k + 2)][32] within tab (column 0 x ebase)
  int tab_rows;
  const double* tab;
  long B;
  int T, H, N;
  const double* A;       // [64][64]
  const double* pi;      // [64]
  const double* w;       // [64] = A s_all (ll weights)
  double* S;             // estep_mw_scratch_bytes
  double* ll;
  unsigned* status;
  double* slab;          // [ceil(B / 16)][slab_size]: K [32][32], H [R][32], P0 [32]
  int slab_size, R;
  // per evidence column: first virtual row of its in-range codes (the
  // matrix-core count rows, sum_k M_k <= 64) and its child's first slab row
  int voff[4], crow[4];
  // the plan's children no column observes: their missing rows take every
  // step's posterior (the code is always "missing"); their other rows are 0
  int n_unobs;
  int urow[4], uM[4];
  unsigned long long* diag;   // stamps builds: per group [4 waves][4] cycles, else null
  // chain_fb_ckw_launch only: the interface posteriors [B][T] rows
  double* post;
  long post_bstride;
  int post_tstride, post_off;
};
size_t estep_mw_lds_bytes(int tab_rows);
int estep_mw_max_cols();
size_t estep_mw_scratch_bytes(long B, int T);
// -2: the request does not fit the kernel (N > 32, more than 64 count rows, LDS)
int estep_mw_launch(const EMwArgs& a, hipStream_t stream);
// checkpoint + recompute e_step at 17..32 states (estep_ckw.hip, round 6):
// one or two observed columns, the same wide slab row per 16 sequences;
// count_rows = sum over the observed columns of M_k + 2.  Needs the host's
// underflow bound for rescaling every 4th step (engine.cpp ckw_sparse_ok);
// proper: ll from the final forward mass.  kLaunchRefused when it does not fit.
size_t chain_estep_ckw_lds_bytes(int tab_rows, int count_rows);
size_t chain_estep_ckw_scratch_bytes(long B, int T);
int chain_estep_ckw_launch(const EMwArgs& a, bool proper, hipStream_t stream);
// the same kernel's forward_backward_inference form (chain_fb_ckw_kernel):
// the interface posteriors to post (normalised per step), ll, status (1 for
// zero mass); scratch chain_estep_ckw_scratch_bytes; no slab
// vl: the recomputed messages in LDS, two waves per SIMD (the default; false:
// in registers, one wave per SIMD)
int chain_fb_ckw_launch(const EMwArgs& a, bool proper, bool vl, hipStream_t stream);

size_t chain_lds_bytes(int M, int T, bool estep);
int chain_fb_launch(const ChainArgs& a, hipStream_t stream);
// matrix-core variant (chain_mfma.hip): 16 sequences per 4-wave block
size_t chain_mfma_lds_bytes(int M, int T);
int chain_fb_mfma_launch(const ChainArgs& a, hipStream_t stream);
// checkpoint + recompute variant (chain_ckpt.hip, 8-wave block, N = 16
// posterior rows); -2 when the request does not fit it
size_t chain_fb_ckpt_lds_bytes(int M, int T);
int chain_fb_ckpt_launch(const ChainArgs& a, hipStream_t stream);
// matrix-core e_step (N, M <= 16): one slab row per 16-sequence block (the
// sums over its sequences); -2 when the request does not fit the kernel
size_t chain_estep_mfma_lds_bytes(int M, int T);
int chain_estep_mfma_launch(const ChainArgs& a, hipStream_t stream);
int chain_estep_launch(const ChainArgs& a, hipStream_t stream);
// the default e_step kernel (chain_kernels.hip chain_estep16_kernel): 16
// sequences per block, direction-uniform waves, analytic phase-B normalisation;
// its scratch holds the messages plus one exponent per (sequence, step)
int chain_estep16_launch(const ChainArgs& a, hipStream_t stream);
size_t chain_estep16_lds_bytes(int M, int T, int ne);
// sequences per slab row of chain_estep16_kernel (one row per block: 16, or 8 / 24)
int chain_estep16_seqs_per_row(int M, int T, int ne);
size_t chain_estep16_scratch_bytes(long B, int T);
// checkpoint + recompute e_step (estep_ck.hip, round 6): 16-state interface
// chains with one observed child; a wave per 16 sequences, one slab row each
// (chain_estep_slab); kLaunchRefused when the request does not fit it
size_t chain_estep_ck_lds_bytes(int M);
size_t chain_estep_ck_scratch_bytes(long B, int T);
int chain_estep_ck_launch(const ChainArgs& a, hipStream_t stream);
int tree_reduce_launch(const double* in, long n, int S, double* out, hipStream_t stream);
int estep_finalize_launch(const double* R, const ChainFinalize& f, double* counts, hipStream_t stream);
// the e_step partial's route tag: tag[0] = a, tag[1] = b, tag[2] = c
int estep_tag_launch(double* tag, double a, double b, double c, hipStream_t stream);
// nonzero status words -> out[0]; work: count_failed_work(B) doubles
long count_failed_work(long B);
int count_failed_launch(const uint32_t* status, long B, double* work, double* out, hipStream_t stream);
// BAD_LUCK for sequences missing every observation at steps 0..first_bad (prefix.cpp)
// trivial: bit c set when column c observes a one-state variable (no evidence)
int estep_prefix_flag_launch(const int32_t* obs, int n_obs, int B, int T, int first_bad, unsigned trivial,
                             uint32_t* status,
                             hipStream_t stream);
// counts[p] += sum_j coef[j] * R[idx[j]] over j in [ptr[p], ptr[p + 1]) (a
// linear map of the reduced slab, e.g. a joint interface's counts projected
// onto every family), in index order
int estep_map_finalize_launch(const double* R, int n, const int* ptr, const int* idx, const double* coef,
                              double* counts, hipStream_t stream);

}  // namespace nipamd
