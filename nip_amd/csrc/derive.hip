// derive.hip -- marginals of the chain's other variables, derived on the GPU
// from the interface variable's marginals (forward_backward_inference /
// forward_inference of a query that names them: the reference reads every
// queried variable's marginal off its family clique, src/nip.c:1535-1552 and
// 1273-1290).
//
// With the chain plan's tables (compile.cpp: A = the in-clique folded over
// the hidden parents, pi = prior of prev, E_k / s_k = leaf child k's clique
// and its row sums, G_j = the in-clique folded over all hidden parents but
// h_j), the family-clique marginals of slice t reduce to, with a_t = the
// normalised forward message into slice t (pi at t = 0, use_priors,
// nip.c:88-119; the filtered interface marginal of slice t-1 otherwise) and
// lambda_t(y) = the evidence and backward message on cur (e_t when
// filtering; post_t / (A^T a_t) when smoothing, 0 where A^T a_t = 0, where
// post_t is 0 too):
//
//   prev (OLD_OUTGOING)   ~ a_t(x) sum_y A(x,y) lambda_t(y)
//                           (smoothing, t >= 1: exactly post_{t-1}(x))
//   hidden parent h_j = d ~ sum_x a_t(x) sum_y G_j[d](x,y) lambda_t(y)
//   leaf child k, missing or never observed at t:
//                         ~ sum_y cur_t(y) E_k(y,m) / s_k(y)   (s_k(y) = 0: cur_t(y) = 0)
//   leaf child k observed at t (state o): the one-hot of o, or all zero
//                           when the slice has no mass (an out-of-range state
//                           enters an all-zero likelihood, nipjointree.c:832-856)
//
// each normalised as nip_normalise_array does (a zero sum is left alone,
// nippotential.c:349-360).  e_t(y) = ebase(y) prod_i tab_i[code_i][y] is the
// evidence the kernels use (code: state, M = missing, M+1 = out of range).
// One thread per (sequence, slice); these are the optional extra outputs of
// a query, not the hot path.
#include <hip/hip_runtime.h>

#include "chain_kernels.h"

namespace nipamd {

namespace {

constexpr int kMaxN = 64;

__device__ __forceinline__ int code_of(int o, int M) { return o < 0 ? M : (o < M ? o : M + 1); }

// e_t(y) (wide tables: [(M_i + 2)][64] per observed column)
__device__ __forceinline__ double evidence(const DeriveArgs& a, long b, int t, int y) {
  double e = a.ebase[y];
  for (int i = 0; i < a.ncol; i++) {
    const int o = a.obs[b * a.obs_bstride + (long)t * a.obs_tstride + a.col[i]];
    e *= a.tab[i][(size_t)code_of(o, a.M[i]) * 64 + y];
  }
  return e;
}

// one variable's marginal from a joint interface vector: out[k] = sum of v[x]
// over the joint states x whose digit (x / stride % card) is k
// (states in increasing order; each output written once)
__device__ __forceinline__ int project_digit(const double* v, int N, int stride, int card, double* out) {
  for (int k = 0; k < card; k++) {
    double s = 0.0;
    for (int hi = k * stride; hi < N; hi += stride * card)
      for (int lo = 0; lo < stride; lo++) s += v[hi + lo];
    out[k] = s;
  }
  return card;
}

__global__ __launch_bounds__(256)
void derive_kernel(DeriveArgs a) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.B * (long)a.T) return;
  const long b = i / a.T;
  const int t = (int)(i - b * a.T);
  const int N = a.N;
  const double* pc = a.cur + b * a.cur_bstride + (long)t * a.cur_tstride;
  double* out = a.out + b * a.out_bstride + (long)t * a.out_tstride + a.out_off;
  int n = 0;
  if (a.kind == kDeriveProject) {
    n = project_digit(pc, N, a.prev_stride, a.prev_card, out);
  } else if (a.kind == kDeriveChild) {
    const int M = a.child_M;
    n = M;
    const int o = a.child_col >= 0 ? a.obs[b * a.obs_bstride + (long)t * a.obs_tstride + a.child_col] : -1;
    double mass = 0.0;
    for (int y = 0; y < N; y++) mass += pc[y];
    for (int m = 0; m < M; m++) out[m] = (o >= 0 && m == o && mass > 0.0) ? 1.0 : 0.0;
    if (o < 0) {
      const double* s = a.child_E + (size_t)M * 64;
      for (int y = 0; y < N; y++) {
        if (s[y] == 0.0 || pc[y] == 0.0) continue;
        const double r = pc[y] / s[y];
        for (int m = 0; m < M; m++) out[m] += r * a.child_E[(size_t)m * 64 + y];
      }
    }
  } else if (a.kind == kDerivePrev && !a.filter && t > 0) {
    n = N;
    const double* q = pc - a.cur_tstride;
    if (a.prev_card > 0) n = project_digit(q, N, a.prev_stride, a.prev_card, out);
    else for (int x = 0; x < N; x++) out[x] = q[x];
  } else {
    // a_t and lambda_t
    double av[kMaxN], lam[kMaxN];
    const double* al = t > 0 ? a.alpha + b * a.al_bstride + (long)(t - 1) * a.al_tstride : a.pi;
    for (int x = 0; x < N; x++) av[x] = al[x];
    for (int y = 0; y < N; y++) {
      if (a.filter) {
        lam[y] = evidence(a, b, t, y);
      } else {
        double u = 0.0;
        for (int x = 0; x < N; x++) u += av[x] * a.A[x * 64 + y];
        lam[y] = u > 0.0 ? pc[y] / u : 0.0;
      }
    }
    if (a.kind == kDerivePrev) {
      n = N;
      double pj[kMaxN];
      for (int x = 0; x < N; x++) {
        double acc = 0.0;
        for (int y = 0; y < N; y++) acc += a.A[x * 64 + y] * lam[y];
        pj[x] = av[x] * acc;
      }
      if (a.prev_card > 0) n = project_digit(pj, N, a.prev_stride, a.prev_card, out);
      else for (int x = 0; x < N; x++) out[x] = pj[x];
    } else {
      n = a.hid_card;
      for (int d = 0; d < n; d++) {
        const double* g = a.G + (size_t)d * 4096;
        double acc = 0.0;
        for (int x = 0; x < N; x++) {
          if (av[x] == 0.0) continue;
          double r = 0.0;
          for (int y = 0; y < N; y++) r += g[x * 64 + y] * lam[y];
          acc += av[x] * r;
        }
        out[d] = acc;
      }
    }
  }
  double z = 0.0;
  for (int k = 0; k < n; k++) z += out[k];
  if (z != 0.0) {                                  // nip_normalise_array: a zero sum is left alone
    const double r = 1.0 / z;
    for (int k = 0; k < n; k++) out[k] *= r;
  }
}

// kDeriveProject over a dense [B][T][N] joint posterior (the engine's work
// buffer): a block's rows (256, fewer past 31 states: 64 KB of LDS) are
// staged in LDS by coalesced loads (rows
// padded to N + 1 doubles, so a wave's per-thread row reads spread over the
// banks), then each thread projects and normalises its row as derive_kernel
// does -- same sums in the same order, so the same bits.
__host__ __device__ inline int project_rows(int N) {
  const int r = 65536 / (8 * (N + 1));
  return r < 256 ? r : 256;
}

__global__ __launch_bounds__(256)
void project_kernel(DeriveArgs a) {
  extern __shared__ double rows[];
  const int N = a.N, P = N + 1, R = project_rows(N);
  const long total = a.B * (long)a.T;
  const long r0 = (long)blockIdx.x * R;
  const int nr = (int)(total - r0 < R ? total - r0 : R);
  const double* src = a.cur + r0 * N;
  for (int i = threadIdx.x; i < nr * N; i += 256) rows[(i / N) * P + (i % N)] = src[i];
  __syncthreads();
  if ((int)threadIdx.x >= nr) return;
  const long i = r0 + threadIdx.x;
  const long b = i / a.T;
  const int t = (int)(i - b * a.T);
  double* out = a.out + b * a.out_bstride + (long)t * a.out_tstride + a.out_off;
  const int n = project_digit(rows + threadIdx.x * P, N, a.prev_stride, a.prev_card, out);
  double z = 0.0;
  for (int k = 0; k < n; k++) z += out[k];
  if (z != 0.0) {
    const double r = 1.0 / z;
    for (int k = 0; k < n; k++) out[k] *= r;
  }
}

}  // namespace

int derive_launch(const DeriveArgs& a, hipStream_t stream) {
  const long n = a.B * (long)a.T;
  if (n == 0) return 0;
  if (a.kind == kDeriveProject && a.cur_tstride == a.N && a.cur_bstride == (long)a.T * a.N) {
    const int R = project_rows(a.N);
    const size_t lds = (size_t)R * (a.N + 1) * sizeof(double);        // <= 64 KB
    hipLaunchKernelGGL(project_kernel, dim3((unsigned)((n + R - 1) / R)), dim3(256), lds, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  hipLaunchKernelGGL(derive_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace nipamd
