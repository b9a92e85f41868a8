// opchain.cpp -- host side of the evidence-indexed interface chain (opchain.h).
//
// For a request (its observed variables) the slice's operators are built by
// enumerating every joint assignment of the slice's variables once:
//   W(a)  = prod over cliques of the clique's original potential at a
//           (each CPT lives in its family clique, nipjointree.c:713-772)
//         x prod of the priors use_priors enters at every step after the
//           first: independent variables without the OLD_OUTGOING flag
//           (nip.c:88-119; the previous interface gets the forward message)
//   x(a) / y(a): the joint previous / current interface state (first
//           variable fastest, the joint chain plan's order)
//   T_c[x][y] += W(a) for every evidence combination c the assignment is
//           consistent with (each observed variable: missing, or its state)
// so T_c is the slice's map from the previous interface to the current one
// given the step's evidence -- the propagation's result for any clique tree,
// summed in one fixed order.  w[x] = sum_y T_missing[x][y] is the mass of a
// step without evidence (m1 of the reference, nip.c:1458-1474), pi the
// product of the previous interface's priors (alpha_{-1}, use_priors at t =
// 0).  Plans are cached per model version and observed-variable list.
#include "model.h"

#include "chain_kernels.h"
#include "nip_amd.h"
#include "opchain.h"

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

namespace nipamd {
namespace {

constexpr long kOpMaxWork = 1L << 26;     // assignments x consistent combinations
constexpr size_t kOpMaxTableBytes = 64L << 20;   // operators in HBM (LDS when <= 96 KB)

struct OpPlan {
  std::vector<int> ov;
  unsigned version = 0;
  int device = -1;
  bool ok = false;
  std::string why;
  int K = 0, ncomb = 0;
  std::vector<int> card, stride;
  std::vector<double> T, w, pi;
  double* dT = nullptr;
  double* dw = nullptr;
  double* dpi = nullptr;
  double* S = nullptr;
  size_t S_bytes = 0;
  ~OpPlan() { (void)hipFree(dT); (void)hipFree(dw); (void)hipFree(dpi); (void)hipFree(S); }
};

struct OpCache {
  std::vector<std::unique_ptr<OpPlan>> plans;
};

OpCache* cache_of(nipamd_model* mm) {
  if (!mm->op) mm->op = new OpCache();
  return static_cast<OpCache*>(mm->op);
}

bool build(const Model& m, OpPlan& P) {
  const auto& prev = m.previous_outgoing;
  const auto& cur = m.outgoing;
  const int nv = (int)m.vars.size();
  if (cur.empty() || prev.size() != cur.size()) { P.why = "no interface"; return false; }
  long K = 1, Kp = 1;
  for (int v : cur) K *= m.vars[v].card;
  for (int v : prev) Kp *= m.vars[v].card;
  if (K > 16 || K != Kp) { P.why = "joint interface above 16 states"; return false; }
  for (int v : prev)
    if (!m.vars[v].has_prior) { P.why = "previous interface variable without a prior"; return false; }
  const int no = (int)P.ov.size();
  if (no > kOpMaxObs) { P.why = "more than 8 observed variables"; return false; }
  long ncomb = 1;
  for (int i = 0; i < no; i++) {
    const int v = P.ov[i];
    if (v < 0 || v >= nv) { P.why = "bad observed variable"; return false; }
    for (int j = 0; j < i; j++) if (P.ov[j] == v) { P.why = "observed variable listed twice"; return false; }
    P.card.push_back(m.vars[v].card);
    P.stride.push_back((int)ncomb);
    ncomb *= m.vars[v].card + 1;
  }
  if (ncomb > 65534 || (size_t)(ncomb + 1) * K * K * sizeof(double) > kOpMaxTableBytes) {
    P.why = "too many evidence combinations";
    return false;
  }
  long total = 1;
  for (const Var& V : m.vars) {
    total *= V.card;
    if (total > kOpMaxWork) break;
  }
  if (total * (1L << no) > kOpMaxWork) { P.why = "slice too large to enumerate"; return false; }

  P.K = (int)K;
  P.ncomb = (int)ncomb;
  P.T.assign((size_t)(ncomb + 1) * K * K, 0.0);     // + the zero operator of an out-of-range state
  // per clique: the flat-index stride of every variable (dimension 0 fastest)
  std::vector<std::vector<std::pair<int, long>>> cst(m.cliques.size());
  for (size_t c = 0; c < m.cliques.size(); c++) {
    long st = 1;
    for (int v : m.cliques[c].vars) { cst[c].push_back({v, st}); st *= m.vars[v].card; }
  }
  std::vector<int> pri;
  for (int v : m.independent)
    if (m.vars[v].has_prior && !(m.vars[v].ifs & IF_OLD_OUTGOING)) pri.push_back(v);
  std::vector<int> a(nv, 0);
  for (long it = 0; it < total; it++) {
    double W = 1.0;
    for (size_t c = 0; c < m.cliques.size() && W != 0.0; c++) {
      long idx = 0;
      for (const auto& e : cst[c]) idx += a[e.first] * e.second;
      W *= m.cliques[c].original[(size_t)idx];
    }
    for (size_t i = 0; i < pri.size() && W != 0.0; i++) W *= m.vars[pri[i]].prior[a[pri[i]]];
    if (W != 0.0) {
      long x = 0, y = 0, sx = 1, sy = 1;
      for (size_t i = 0; i < cur.size(); i++) {
        x += a[prev[i]] * sx; sx *= m.vars[prev[i]].card;
        y += a[cur[i]] * sy; sy *= m.vars[cur[i]].card;
      }
      for (long mask = 0; mask < (1L << no); mask++) {
        long c = 0;
        for (int i = 0; i < no; i++)
          if (mask >> i & 1) c += (long)(a[P.ov[i]] + 1) * P.stride[i];
        P.T[(size_t)c * K * K + x * K + y] += W;
      }
    }
    for (int v = 0; v < nv; v++) {                      // odometer, variable 0 fastest
      if (++a[v] < m.vars[v].card) break;
      a[v] = 0;
    }
  }
  P.w.assign(K, 0.0);
  for (long x = 0; x < K; x++)
    for (long y = 0; y < K; y++) P.w[x] += P.T[x * K + y];
  P.pi.assign(K, 1.0);
  for (long x = 0; x < K; x++) {
    long r = x;
    for (int v : prev) { P.pi[x] *= m.vars[v].prior[r % m.vars[v].card]; r /= m.vars[v].card; }
  }
  return true;
}

OpPlan* plan_for(nipamd_model* mm, int n_obs, const int* obs_vars) {
  OpCache* C = cache_of(mm);
  std::vector<int> ov(obs_vars, obs_vars + n_obs);
  for (auto& p : C->plans)
    if (p->ov == ov && p->version == mm->version) return p.get();
  C->plans.erase(std::remove_if(C->plans.begin(), C->plans.end(),
                                [&](const std::unique_ptr<OpPlan>& p) { return p->version != mm->version; }),
                 C->plans.end());
  auto P = std::make_unique<OpPlan>();
  P->ov = ov;
  P->version = mm->version;
  P->ok = build(mm->m, *P);
  C->plans.push_back(std::move(P));
  return C->plans.back().get();
}

template <typename V>
int upload(double** dst, const V& v) {
  if (hipMalloc(dst, (v.size() ? v.size() : 1) * sizeof(double)) != hipSuccess) return -1;
  if (v.size() && hipMemcpy(*dst, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    return -1;
  return 0;
}

}  // namespace

// Does the evidence-indexed chain take this request?  Queries: the current
// interface's variables (their marginals are digits of the joint one).
bool op_supported(nipamd_model* mm, int n_obs, const int* obs_vars, int n_query, const int* query,
                  std::string& why) {
  OpPlan* P = plan_for(mm, n_obs, obs_vars);
  if (!P->ok) { why = P->why; return false; }
  for (int i = 0; i < n_query; i++)
    if (std::find(mm->m.outgoing.begin(), mm->m.outgoing.end(), query[i]) == mm->m.outgoing.end()) {
      why = "query outside the current interface";
      return false;
    }
  return true;
}

// The kernel stages the block's evidence codes in LDS: does T fit?
bool op_fits(nipamd_model* mm, int n_obs, const int* obs_vars, int T) {
  OpPlan* P = plan_for(mm, n_obs, obs_vars);
  return P->ok && op_lds_bytes(P->K, P->ncomb, T, false) <= 150 * 1024;
}

// The joint interface's posterior (or filtered) marginals into d_joint
// [B][T][K] (or straight into the caller's rows when jts == K), ll, status.
int op_fb(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T, double* d_joint,
          long jbs, int jts, int joff, double* d_ll, uint32_t* d_status, void* stream, bool filt, int* K_out,
          std::string& err) {
  OpPlan* P = plan_for(mm, n_obs, obs_vars);
  if (!P->ok) { err = P->why; return NIPAMD_ERROR_UNSUPPORTED; }
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) { err = "no device"; return NIPAMD_ERROR_DEVICE; }
  if (P->device != dev || !P->dT) {
    (void)hipFree(P->dT); (void)hipFree(P->dw); (void)hipFree(P->dpi); (void)hipFree(P->S);
    P->dT = P->dw = P->dpi = P->S = nullptr;
    P->S_bytes = 0;
    if (upload(&P->dT, P->T) || upload(&P->dw, P->w) || upload(&P->dpi, P->pi)) {
      err = "device tables";
      return NIPAMD_ERROR_DEVICE;
    }
    P->device = dev;
  }
  // Smoothing keeps every sequence's rows plus a sink row past them; filter
  // mode keeps no rows, and its masked lanes (inactive sequences, states
  // y >= K) write to a sink at the start of S (op_fb_kernel).
  const size_t need = filt ? op_scratch_bytes(1, 1) : op_scratch_bytes(B, T);
  if (P->S_bytes < need) {
    (void)hipFree(P->S);
    P->S = nullptr;
    P->S_bytes = 0;
    if (hipMalloc(&P->S, need) != hipSuccess) { err = "scratch"; return NIPAMD_ERROR_DEVICE; }
    P->S_bytes = need;
  }
  OpArgs a{};
  a.obs = d_obs;
  const long ocols = n_obs > 0 ? n_obs : 1;
  a.obs_bstride = (long)T * ocols;
  a.obs_tstride = (int)ocols;
  a.nobs = n_obs;
  for (int i = 0; i < n_obs; i++) { a.col[i] = i; a.card[i] = P->card[i]; a.cstride[i] = P->stride[i]; }
  a.B = B; a.T = T; a.H = filt ? T : T / 2; a.K = P->K; a.ncomb = P->ncomb;
  a.filter = filt ? 1 : 0;
  a.Ttab = P->dT; a.w = P->dw; a.pi = P->dpi;
  a.S = P->S;
  a.post = d_joint; a.post_bstride = jbs; a.post_tstride = jts; a.post_off = joff;
  a.ll = d_ll; a.status = d_status;
  if (K_out) *K_out = P->K;
  const int rc = op_fb_launch(a, (hipStream_t)stream);
  if (rc == -2) { err = "operators do not fit the kernel's LDS"; return NIPAMD_ERROR_UNSUPPORTED; }
  if (rc) { err = std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()); return NIPAMD_ERROR_DEVICE; }
  return 0;
}

void op_release(nipamd_model* mm) {
  delete static_cast<OpCache*>(mm->op);
  mm->op = nullptr;
}

}  // namespace nipamd
