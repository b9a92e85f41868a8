// chain_kernels.h -- launch interface of the gfx950 chain (HMM-shaped slice) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>

namespace nipamd {

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
  double* S;             // scratch [B][T][16]: alpha_t (t < H), beta_t (t >= H)
  double* post;          // posterior output
  long post_bstride;     // elements between sequences
  int post_tstride;      // elements between time steps
  int post_off;          // offset of the variable's block within a step
  double* ll;            // [B] or nullptr
  unsigned* status;      // [B] or nullptr
  double* counts;        // E-step only: per-block partial counts
};

size_t chain_fb_lds_bytes(int M, int T);
int chain_fb_launch(const ChainArgs& a, hipStream_t stream);

}  // namespace nipamd
