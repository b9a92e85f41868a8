// niplikelihood (util/niplikelihood.c) on the GPU.
//
// For every time step of every series, independently (the reference resets
// the join tree after each step and passes no message between slices,
// niplikelihood.c:111-133):
//   m1 = model_prob_mass after the UNMARKED variables' evidence of the step,
//   m2 = the same after the marked variables' evidence is added,
//   ll = log(m2) - log(m1)   (ln p(marked | unmarked)).
// The slice's priors are entered as use_priors does: every independent
// variable's in the first step, all but the previous-slice copy's after
// (niplikelihood.c:114, 132; nip.c:88-119), so X0 carries weight 1 then.
// For an interface chain the mass of a step is
//   m = sum_y u(y) e(y),  u(y) = sum_x w(x) A(x, y)
// with A the transition folded over the hidden parents' priors (model.h
// ChainPlan), w = the prior of X0 (first step) or 1, and e(y) the product
// over X1's children of E_k(y, o) (observed) or the row sum s_k(y) (not), and
// an indicator of X1's own state when it is observed.  One thread per
// (series, step); the reference's sums run in a different order, so the
// masses agree to rounding (tests: 1e-12 relative).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "model.h"
#include "nip_amd.h"

namespace nipamd {
namespace {

constexpr int kLikMaxCols = 8;

struct LikArgs {
  const int* obs;
  long obs_bstride;
  int obs_tstride;
  int ncol;
  int col[kLikMaxCols];
  int M[kLikMaxCols];
  long tab_off[kLikMaxCols];   // [(M+2)][64]: E rows, the row sums (missing), zeros (out of range)
  unsigned marked;             // bit c: column c is marked
  const double* tab;
  const double* u;             // [2][64]: first step, later steps
  const double* ebase;         // [64]: row sums of the children without a column
  long B;
  int T, N;
  double *m1, *m2, *ll;        // [B][T]
};

__global__ __launch_bounds__(256) void likelihood_kernel(LikArgs a) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.B * a.T) return;
  const long b = i / a.T;
  const int t = (int)(i - b * a.T);
  const int* o = a.obs + b * a.obs_bstride + (long)t * a.obs_tstride;
  int row1[kLikMaxCols], row2[kLikMaxCols];
  for (int c = 0; c < a.ncol; c++) {
    const int v = o[a.col[c]];
    const int ev = v < 0 ? a.M[c] : (v < a.M[c] ? v : a.M[c] + 1);   // missing: row sums; out of range: 0
    row2[c] = ev;
    row1[c] = (a.marked >> c) & 1 ? a.M[c] : ev;
  }
  const double* u = a.u + (t ? 64 : 0);
  double m1 = 0.0, m2 = 0.0;
  for (int y = 0; y < a.N; y++) {
    double e1 = a.ebase[y], e2 = e1;
    for (int c = 0; c < a.ncol; c++) {
      const double* tb = a.tab + a.tab_off[c];
      e1 *= tb[(long)row1[c] * 64 + y];
      e2 *= tb[(long)row2[c] * 64 + y];
    }
    m1 += u[y] * e1;
    m2 += u[y] * e2;
  }
  a.m1[i] = m1;
  a.m2[i] = m2;
  a.ll[i] = std::log(m2) - std::log(m1);
}

}  // namespace
}  // namespace nipamd

using namespace nipamd;

namespace {
struct LikCache {
  std::vector<int> key;      // model version, device, marked mask, column variables
  int dev = -1;
  double* d_all = nullptr;   // tables, then u [128], then ebase [64]
};
}  // namespace

extern "C" int nipamd_likelihood(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                                 const int* marked, int B, int T, double* d_m1, double* d_m2,
                                 double* d_ll, void* stream) {
  if (!mm || B < 0 || T < 0 || n_obs < 0 || n_obs > kLikMaxCols || (n_obs && (!obs_vars || !marked)) ||
      (B > 0 && T > 0 && (!d_m1 || !d_m2 || !d_ll || (n_obs && !d_obs))))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "likelihood: bad arguments");
  const ChainPlan& P = mm->m.chain;
  if (!P.valid || P.joint) return set_error(NIPAMD_ERROR_UNSUPPORTED, "likelihood: the model has no single-variable interface-chain plan");
  if (int rc = ensure_fold(mm)) return rc;
  const int N = P.N;
  LikArgs a{};
  a.ncol = n_obs;
  std::vector<double> tab;
  std::vector<char> has_col(P.emits.size() + 1, 0);
  for (int c = 0; c < n_obs; c++) {
    int k = -1;
    for (size_t e = 0; e < P.emits.size(); e++)
      if (P.emits[e].var == obs_vars[c]) k = (int)e;
    if (obs_vars[c] == P.v_cur) k = (int)P.emits.size();
    if (k < 0) return set_error(NIPAMD_ERROR_UNSUPPORTED, "likelihood: evidence on a variable outside X1 and its leaf children");
    if (has_col[k]) return set_error(NIP_ERROR_INVALID_ARGUMENT, "likelihood: a variable in two columns");
    has_col[k] = 1;
    const ChainEmit& E = P.emit(k);
    a.col[c] = c;
    a.M[c] = E.M;
    a.tab_off[c] = (long)tab.size();
    a.marked |= marked[c] ? 1u << c : 0u;
    tab.insert(tab.end(), E.E.begin(), E.E.begin() + (size_t)E.M * 64);
    tab.insert(tab.end(), E.s.begin(), E.s.end());
    tab.insert(tab.end(), 64, 0.0);
  }
  std::vector<double> ebase(64, 0.0), u(128, 0.0);
  for (int y = 0; y < N; y++) {
    double s = 1.0;
    for (size_t e = 0; e < P.emits.size(); e++)
      if (!has_col[e]) s *= P.emits[e].s[y];
    ebase[y] = s;
    double u0 = 0.0, u1 = 0.0;
    for (int x = 0; x < N; x++) {
      u0 += P.pi64[x] * P.A64[x * 64 + y];
      u1 += P.A64[x * 64 + y];
    }
    u[y] = u0;
    u[64 + y] = u1;
  }
  if (B == 0 || T == 0) return NIP_NO_ERROR;
  tab.resize(tab.size() + 1);
  std::vector<double> all(tab);
  const long off_u = (long)all.size();
  all.insert(all.end(), u.begin(), u.end());
  const long off_e = (long)all.size();
  all.insert(all.end(), ebase.begin(), ebase.end());
  // device tables cached per model, keyed by the model version, the device
  // and the column set (as the fb path caches its request tables): a repeat
  // call uploads nothing and stays asynchronous on `stream`
  int dev = -1;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return set_error(NIPAMD_ERROR_DEVICE, std::string("likelihood: ") + hipGetErrorString(e));
  std::vector<int> key{(int)mm->version, dev, (int)a.marked};
  key.insert(key.end(), obs_vars, obs_vars + n_obs);
  LikCache* lc = static_cast<LikCache*>(mm->lik);
  if (!lc) mm->lik = lc = new LikCache();
  hipStream_t st = (hipStream_t)stream;
  if (!lc->d_all || lc->key != key) {
    if (lc->d_all) {
      (void)hipDeviceSynchronize();                // an earlier launch may still read them
      (void)hipSetDevice(lc->dev);
      (void)hipFree(lc->d_all);
      (void)hipSetDevice(dev);
      lc->d_all = nullptr;
    }
    e = hipMalloc(&lc->d_all, all.size() * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(lc->d_all, all.data(), all.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(lc->d_all);
      lc->d_all = nullptr;
      return set_error(NIPAMD_ERROR_DEVICE, std::string("likelihood: ") + hipGetErrorString(e));
    }
    lc->key = key;
    lc->dev = dev;
  }
  double* d_all = lc->d_all;
  a.obs = d_obs;
  a.obs_bstride = (long)T * n_obs;
  a.obs_tstride = n_obs;
  a.tab = d_all;
  a.u = d_all + off_u;
  a.ebase = d_all + off_e;
  a.B = B;
  a.T = T;
  a.N = N;
  a.m1 = d_m1;
  a.m2 = d_m2;
  a.ll = d_ll;
  const long n = (long)B * T;
  hipLaunchKernelGGL(likelihood_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  e = hipGetLastError();
  if (e != hipSuccess) return set_error(NIPAMD_ERROR_DEVICE, std::string("likelihood: ") + hipGetErrorString(e));
  return NIP_NO_ERROR;
}

void nipamd::likelihood_release(nipamd_model* mm) {
  LikCache* lc = static_cast<LikCache*>(mm->lik);
  if (!lc) return;
  if (lc->d_all) {
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(lc->dev);
    (void)hipFree(lc->d_all);
    if (cur >= 0) (void)hipSetDevice(cur);
  }
  delete lc;
  mm->lik = nullptr;
}

extern "C" int nipamd_likelihood_host(nipamd_model* mm, const int32_t* obs, int n_obs, const int* obs_vars,
                                      const int* marked, int B, int T, double* m1, double* m2, double* ll) {
  const size_t n = (size_t)B * T;
  if (B < 0 || T < 0 || (n && (!m1 || !m2 || !ll || (n_obs > 0 && !obs))))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "likelihood: bad arguments");
  int32_t* d_obs = nullptr;
  double* d_out = nullptr;
  hipError_t e = hipSuccess;
  if (n) {
    e = hipMalloc(&d_obs, (n * (n_obs > 0 ? n_obs : 1)) * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&d_out, 3 * n * sizeof(double));
    if (e == hipSuccess && n_obs > 0) e = hipMemcpy(d_obs, obs, n * n_obs * sizeof(int32_t), hipMemcpyHostToDevice);
  }
  int rc = e == hipSuccess ? NIP_NO_ERROR : set_error(NIPAMD_ERROR_DEVICE, std::string("likelihood: ") + hipGetErrorString(e));
  if (rc == NIP_NO_ERROR)
    rc = nipamd_likelihood(mm, d_obs, n_obs, obs_vars, marked, B, T, d_out, d_out + n, d_out + 2 * n, nullptr);
  if (rc == NIP_NO_ERROR && n) {
    e = hipMemcpy(m1, d_out, n * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(m2, d_out + n, n * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(ll, d_out + 2 * n, n * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = set_error(NIPAMD_ERROR_DEVICE, std::string("likelihood: ") + hipGetErrorString(e));
  }
  (void)hipFree(d_obs);
  (void)hipFree(d_out);
  return rc;
}
