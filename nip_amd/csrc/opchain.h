// opchain.h -- the evidence-indexed interface chain (opchain.cpp, opchain.hip).
//
// Any DBN time slice maps the previous interface's distribution to the
// current one linearly: with I_{t-1} = x and I_t = y the joint interface
// states (K = prod of the outgoing variables' cardinalities),
//   alpha_t(y) = sum_x alpha_{t-1}(x) T_{c_t}(x, y),
//   T_c(x, y)  = sum over the slice's other variables of the product of its
//                CPTs, the priors entered every slice and the evidence
//                indicators of combination c,
// where c indexes the step's evidence row (each observed variable missing or
// one of its states).  When K <= 16 and the slice is small enough to
// enumerate, the operators T_c are built once per model version and request
// on the host, and forward-backward runs as a chain over K states whose
// transition is chosen per step by the evidence row -- the slices the
// interface-chain plan rejects (evidence on a hidden parent or a non-leaf
// variable, interfaces that do not factorise) then run as chains too instead
// of on the general join-tree engine.
#pragma once

#include <cstdint>
#include <hip/hip_runtime.h>

namespace nipamd {

constexpr int kOpMaxObs = 8;

struct OpArgs {
  const int32_t* obs;      // [B][T][n_obs]
  long obs_bstride;
  int obs_tstride;
  int nobs;                // observed columns used
  int col[kOpMaxObs];      // their columns in obs
  int card[kOpMaxObs];     // their cardinalities
  int cstride[kOpMaxObs];  // combination radix: prod_{j<i} (card_j + 1)
  long B;
  int T, H, K;
  int ncomb;               // combinations; table ncomb is all zeros (an out-of-range state)
  int filter;              // forward_inference: the forward rows' normalised messages
  int tlds;                // set by op_fb_launch: the operators fit in LDS
  const double* Ttab;      // [(ncomb + 1)][K][K], table ncomb all zeros
  const double* w;         // [K] slice mass without evidence given x (m1 weights)
  const double* pi;        // [K] prior of the previous interface
  double* S;               // scratch: op_scratch_bytes(B, T)
  double* post;            // [B][T][post_tstride], the joint interface marginal at post_off
  long post_bstride;
  int post_tstride;
  int post_off;
  double* ll;
  unsigned* status;
  // e_step (estep = 1, smoothing only): instead of posteriors, every step's
  // xi weights W_t(x, y) = alpha^_{t-1}(x) beta^_t(y) / Z'_t (Z'_t: the step's
  // xi mass, so sum_{x,y} W_t T_{c_t} = 1) into W [B][T][K*K] (x-major), and
  // the previous interface's t = 0 marginal into P0 [B][K]
  int estep;
  double* W;
  double* P0;
  uint16_t* C;             // e_step: every step's evidence combination [B][T] (op_xi_kernel's keys)
};

size_t op_lds_bytes(int K, int ncomb, int T, bool tables);
size_t op_scratch_bytes(long B, int T);
int op_fb_launch(const OpArgs& a, hipStream_t stream);

// The e_step's per-combination sums (op_xi_kernel): one slab row per 16
// sequences, Xi[c][x][y] = sum over the group's steps with evidence
// combination c of W_t(x, y), then P0 [K] summed over the group.
struct OpXiArgs {
  const int32_t* obs;      // as OpArgs
  long obs_bstride;
  int obs_tstride;
  int nobs;
  int col[kOpMaxObs];
  int card[kOpMaxObs];
  int cstride[kOpMaxObs];
  long B;
  int T, K, ncomb;
  const double* W;         // [B][T][K*K]
  const double* P0;        // [B][K]
  const uint16_t* C;       // [B][T] evidence combinations (op_fb_kernel's codes)
  double* slab;            // [ceil(B / 16)][op_xi_row(K, ncomb)]
};
constexpr int kOpXiSeqs = 16;
__host__ __device__ inline int op_xi_row(int K, int ncomb) { return (ncomb + 1) * K * K + K; }
bool op_xi_fits(int K, int ncomb);

// 17 <= K <= 64 joint interface states (estep_wide.hip op_wide_*): one
// wave per direction holds 64 / NP sequences (NP = 32 or 64 lanes each, lane
// = state), the step's column (forward) or row (backward) of its operator
// read per step (from LDS when the operators fit, else through the caches),
// the mat-vec by DPP row broadcasts.  Every message is stored (alpha^_t in
// Sa, beta^_t in Sb), then op_wide_post_kernel normalises alpha^ beta^ (or
// alpha^ alone, filtering) into the caller's joint rows.
//
// Leaf factorisation (opchain.cpp build): an observed variable that appears
// in one clique only, over itself and current-interface variables, factors
// out of the operators, T_c(x, y) = T'_{c'}(x, y) prod_j F_j[c_j](y): c' indexes
// the other observed variables only (onobs, ocol, ...), and leaf j selects
// row c_j of its table F_j (its state, card_j: missing = the row sum,
// card_j + 1: out of range = 0).  The full combination c (nobs, col, ...,
// ncomb) still keys the e_step's sums.
constexpr int kOpMaxLeaf = 4;
struct OpWideArgs {
  const int32_t* obs;
  long obs_bstride;
  int obs_tstride;
  int nobs;                // the full combination (e_step keys, the ll's evidence test)
  int col[kOpMaxObs];
  int card[kOpMaxObs];
  int cstride[kOpMaxObs];
  long B;
  int T, K, ncomb;
  int filter;
  int onobs;               // the operator index c'
  int ocol[kOpMaxObs];
  int ocard[kOpMaxObs];
  int ocstride[kOpMaxObs];
  int oncomb;              // operators: oncomb + 1 (the last all zero)
  int nleaf;               // leaf factors
  int lcol[kOpMaxLeaf];
  int lcard[kOpMaxLeaf];
  int loff[kOpMaxLeaf];    // F_j at ltab + loff[j]: [(lcard[j] + 2)][K]
  const double* ltab;
  const double* Ttab;      // [(oncomb + 1)][K][K] + 64 zeros: T'_c(x, y) at c K^2 + x K + y
  const double* TtabT;     // the same transposed per operator: T'_c(x, y) at c K^2 + y K + x
  const double* w;         // [K]
  const double* pi;        // [K]
  double* Sa;              // [B][T][NP]
  double* Sb;              // [B][T][NP]
  double* post;            // joint rows: post + b * post_bstride + t * post_tstride + post_off
  long post_bstride;
  int post_tstride;
  int post_off;
  double* ll;
  unsigned* status;
  // e_step (estep = 1): the forward filter also writes every step's scale
  // exponent sc [B][T] (alpha^_t = 2^sc_t T_{c_t}^T alpha^_{t-1}) and the
  // e_step's BAD_LUCK status; op_wide_xi_launch then sums the steps' xi
  // weights per evidence combination into slab rows (op_xi_kernel's layout)
  int estep;
  int* sc;
  double* slab;
  // the e_step's slab row (op_wide_xi_kernel): Xi' [(oncomb + 1)][K][K] keyed
  // by the operator index, then per leaf j its count rows H_j [(lcard[j] + 2)][K]
  // at hoff[j] (gamma_t summed by the leaf's code), then P0 [K] at xrow - K.
  // Sort key of a step: c' << Lbits | code_j << lsh[j] (code_j in lbits[j] bits)
  int Lbits;
  int lsh[kOpMaxLeaf];
  int lbits[kOpMaxLeaf];
  int hoff[kOpMaxLeaf];
  int xrow;
};
constexpr int kOpWideSeqs = 8;         // op_wide_xi_kernel: sequences per block and slab row
constexpr int kOpWideMaxH = 2048;      // doubles of leaf count rows (op_wide_xi_kernel's LDS)
constexpr int kOpWideKeyBits = 18;     // (oncomb + 1) << Lbits <= 2^18
inline int op_wide_np(int K) { return K <= 32 ? 32 : 64; }
inline size_t op_wide_scratch_bytes(int K, long B, int T) {
  return (size_t)2 * B * T * op_wide_np(K) * sizeof(double);
}
int op_wide_launch(const OpWideArgs& a, hipStream_t stream);
int op_wide_xi_launch(const OpWideArgs& a, hipStream_t stream);
bool op_xi_sort_fits(int ncomb, int T);
int op_finalize_launch(const double* R, int n, const int* ptr, const int* idx, const double* coef, double* counts,
                       hipStream_t stream);
int op_xi_launch(const OpXiArgs& a, hipStream_t stream);

}  // namespace nipamd
