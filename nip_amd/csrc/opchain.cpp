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
#include "diag.h"
#include "nip_amd.h"
#include "opchain.h"

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

namespace nipamd {

// a launcher's nonzero return: kLaunchRefused (the host refused the request)
// -> NIPAMD_ERROR_UNSUPPORTED, anything else -> NIPAMD_ERROR_DEVICE
static int op_launch_fail(int rc, const char* what, std::string& err) {
  if (rc == kLaunchRefused) {
    err = std::string(what) + ": the request does not fit the kernel (refused on the host)";
    return NIPAMD_ERROR_UNSUPPORTED;
  }
  err = std::string(what) + ": kernel launch failed: " + hipGetErrorString(hipGetLastError());
  return NIPAMD_ERROR_DEVICE;
}
namespace {

constexpr long kOpMaxWork = 1L << 26;     // assignments x consistent combinations
constexpr size_t kOpMaxTableBytes = 64L << 20;   // operators in HBM (LDS when <= 96 KB)
constexpr size_t kOpMaxWideRow = 32L << 20;      // 17..64 states: an e_step slab row (kOpWideSeqs = 8 sequences)

struct OpPlan {
  std::vector<int> ov;
  unsigned version = 0;
  int device = -1;
  bool ok = false;
  std::string why;
  int K = 0, ncomb = 0;
  std::vector<int> card, stride;
  // the operators' index (K > 16: the observed variables that are not leaf
  // factors, opchain.h) and the leaf factors' tables
  int oncomb = 0;
  std::vector<int> oi, ostride;      // positions in ov, radix
  std::vector<int> li, loff;         // positions in ov, offsets into lt
  std::vector<int> lcl;              // the leaves' cliques
  // the e_step's slab row (opchain.h OpWideArgs): sort-key radix, leaf count
  // rows' offsets, row size
  int Lbits = 0;
  std::vector<int> lsh, lbits, hoff;
  long xrow = 0;
  std::vector<double> lt;
  std::vector<double> T, w, pi;      // T: [(oncomb + 1)][K][K] + 64 zeros (the wide kernels' over-reads)
  std::vector<double> TT;            // K > 16: T transposed per operator, + 64 zeros
  double* dT = nullptr;
  double* dTT = nullptr;
  double* dw = nullptr;
  double* dpi = nullptr;
  double* dlt = nullptr;
  double* S = nullptr;
  size_t S_bytes = 0;
  // e_step: the projection of the per-combination xi sums onto the em_learn
  // layout (CSR over count cells, built on demand per model version) and the
  // launch buffers (W rows, P0, slab rows, tree work)
  int map_state = 0;                 // 0 not built, 1 built, -1 unsupported
  std::string map_why;
  int map_n = 0;
  int* d_mptr = nullptr;
  int* d_midx = nullptr;
  double* d_mcoef = nullptr;
  double* E = nullptr;
  size_t E_bytes = 0;
  ~OpPlan() {
    (void)hipFree(dT); (void)hipFree(dTT); (void)hipFree(dw); (void)hipFree(dpi); (void)hipFree(dlt); (void)hipFree(S);
    (void)hipFree(d_mptr); (void)hipFree(d_midx); (void)hipFree(d_mcoef); (void)hipFree(E);
  }
};

struct OpCache {
  std::vector<std::unique_ptr<OpPlan>> plans;
};

OpCache* cache_of(nipamd_model* mm) {
  if (!mm->op) mm->op = new OpCache();
  return static_cast<OpCache*>(mm->op);
}

template <typename V>
bool has(const V& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); }

bool build(const Model& m, OpPlan& P) {
  const auto& prev = m.previous_outgoing;
  const auto& cur = m.outgoing;
  const int nv = (int)m.vars.size();
  if (cur.empty() || prev.size() != cur.size()) { P.why = "no interface"; return false; }
  long K = 1, Kp = 1;
  for (int v : cur) K *= m.vars[v].card;
  for (int v : prev) Kp *= m.vars[v].card;
  if (K > 64 || K != Kp) { P.why = "joint interface above 64 states"; return false; }
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
  if (ncomb > 65534) { P.why = "too many evidence combinations"; return false; }
  std::vector<int> pri;
  for (int v : m.independent)
    if (m.vars[v].has_prior && !(m.vars[v].ifs & IF_OLD_OUTGOING)) pri.push_back(v);
  // Leaf factors (17..64 states, op_wide_msgs_kernel): an observed variable
  // in exactly one clique whose other variables are all current-interface
  // ones carries every factor it appears in within that clique, so summing it
  // out under its evidence leaves a function of y alone, F[c_v](y), and
  // T_c = T'_{c'} diag(prod F) -- c' over the other observed variables.
  std::vector<char> leaf(no, 0);
  std::vector<int> lcl;
  // (the e_step's limits: leaf codes a byte each, the leaf count rows within
  // kOpWideMaxH doubles, sort keys below 2^kOpWideKeyBits)
  long hsz = 0;
  if (K > 16)
    for (int i = 0; i < no && (int)lcl.size() < kOpMaxLeaf; i++) {
      const int v = P.ov[i];
      if (has(cur, v) || has(prev, v) || has(pri, v) || P.card[i] + 2 > 255) continue;
      if (hsz + (long)(P.card[i] + 2) * K > kOpWideMaxH) continue;
      int cl = -1, nc = 0;
      for (size_t c = 0; c < m.cliques.size(); c++)
        if (has(m.cliques[c].vars, v)) { cl = (int)c; nc++; }
      if (nc != 1 || has(lcl, cl)) continue;
      bool ok = true;
      for (int u : m.cliques[cl].vars) ok = ok && (u == v || has(cur, u));
      if (!ok) continue;
      leaf[i] = 1;
      lcl.push_back(cl);
      hsz += (long)(P.card[i] + 2) * K;
    }
  // the sort key c' << Lbits | leaf codes must fit: drop leaves from the back
  auto code_bits = [](int card) { int b = 0; while ((1 << b) < card + 2) b++; return b; };
  for (;;) {
    long oc = 1;
    int lb = 0;
    for (int i = 0; i < no; i++) {
      if (leaf[i]) lb += code_bits(P.card[i]);
      else oc *= P.card[i] + 1;
    }
    if (((oc + 1) << lb) <= (1L << kOpWideKeyBits) || lcl.empty()) break;
    for (int i = no - 1; i >= 0; i--)
      if (leaf[i]) { leaf[i] = 0; lcl.pop_back(); break; }
  }
  long oncomb = 1;
  for (int i = 0; i < no; i++)
    if (!leaf[i]) {
      P.oi.push_back(i);
      P.ostride.push_back((int)oncomb);
      oncomb *= P.card[i] + 1;
    }
  if ((size_t)(oncomb + 1) * K * K * sizeof(double) > kOpMaxTableBytes) {
    P.why = "too many evidence combinations";
    return false;
  }
  P.lcl = lcl;
  std::vector<char> skip(nv, 0);                        // leaf variables: not enumerated
  for (int i = 0; i < no; i++) if (leaf[i]) skip[P.ov[i]] = 1;
  long total = 1;
  for (int v = 0; v < nv; v++) {
    if (skip[v]) continue;
    total *= m.vars[v].card;
    if (total > kOpMaxWork) break;
  }
  if (total * (1L << P.oi.size()) > kOpMaxWork) { P.why = "slice too large to enumerate"; return false; }

  P.K = (int)K;
  P.ncomb = (int)ncomb;
  P.oncomb = (int)oncomb;
  P.T.assign((size_t)(oncomb + 1) * K * K, 0.0);    // + the zero operator of an out-of-range state
  // per clique: the flat-index stride of every variable (dimension 0 fastest)
  std::vector<std::vector<std::pair<int, long>>> cst(m.cliques.size());
  for (size_t c = 0; c < m.cliques.size(); c++) {
    long st = 1;
    for (int v : m.cliques[c].vars) { cst[c].push_back({v, st}); st *= m.vars[v].card; }
  }
  std::vector<char> lc(m.cliques.size(), 0);
  for (int c : lcl) lc[c] = 1;
  const int nop = (int)P.oi.size();
  std::vector<int> a(nv, 0);
  for (long it = 0; it < total; it++) {
    double W = 1.0;
    for (size_t c = 0; c < m.cliques.size() && W != 0.0; c++) {
      if (lc[c]) continue;
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
      for (long mask = 0; mask < (1L << nop); mask++) {
        long c = 0;
        for (int q = 0; q < nop; q++)
          if (mask >> q & 1) c += (long)(a[P.ov[P.oi[q]]] + 1) * P.ostride[q];
        P.T[(size_t)c * K * K + x * K + y] += W;
      }
    }
    for (int v = 0; v < nv; v++) {                      // odometer, variable 0 fastest
      if (skip[v]) continue;
      if (++a[v] < m.vars[v].card) break;
      a[v] = 0;
    }
  }
  // the leaf tables: F[r][y] = the clique's entry at (v = r, y's components),
  // row M the sum over r (a missing value), row M + 1 zero (out of range)
  std::vector<double> eall(K, 1.0);                     // prod_j F_j[missing](y)
  for (size_t j = 0; j < lcl.size(); j++) {
    int i = 0;
    for (int q = 0, n = 0; q < no; q++) if (leaf[q] && n++ == (int)j) i = q;
    const int v = P.ov[i], M = P.card[i], cl = lcl[j];
    P.li.push_back(i);
    P.loff.push_back((int)P.lt.size());
    const size_t base = P.lt.size();
    P.lt.resize(base + (size_t)(M + 2) * K, 0.0);
    for (long y = 0; y < K; y++) {
      std::vector<int> comp(nv, 0);
      long r = y;
      for (int u : cur) { comp[u] = (int)(r % m.vars[u].card); r /= m.vars[u].card; }
      double sum = 0.0;
      for (int val = 0; val < M; val++) {
        long idx = 0;
        for (const auto& e : cst[cl]) idx += (e.first == v ? val : comp[e.first]) * e.second;
        const double f = m.cliques[cl].original[(size_t)idx];
        P.lt[base + (size_t)val * K + y] = f;
        sum += f;
      }
      P.lt[base + (size_t)M * K + y] = sum;
      eall[y] *= sum;
    }
  }
  P.Lbits = 0;
  P.xrow = (long)(oncomb + 1) * K * K;
  for (size_t j = 0; j < P.li.size(); j++) {
    int b = 0;
    while ((1 << b) < P.card[P.li[j]] + 2) b++;
    P.lsh.push_back(P.Lbits);
    P.lbits.push_back(b);
    P.Lbits += b;
    P.hoff.push_back((int)P.xrow);
    P.xrow += (long)(P.card[P.li[j]] + 2) * K;
  }
  P.xrow += K;
  P.w.assign(K, 0.0);
  for (long x = 0; x < K; x++)
    for (long y = 0; y < K; y++) P.w[x] += P.T[x * K + y] * eall[y];
  P.pi.assign(K, 1.0);
  for (long x = 0; x < K; x++) {
    long r = x;
    for (int v : prev) { P.pi[x] *= m.vars[v].prior[r % m.vars[v].card]; r /= m.vars[v].card; }
  }
  P.T.resize(P.T.size() + 64, 0.0);
  if (K > 16) {
    P.TT.assign(P.T.size(), 0.0);
    for (long c = 0; c <= oncomb; c++)
      for (long x = 0; x < K; x++)
        for (long y = 0; y < K; y++) P.TT[(size_t)c * K * K + y * K + x] = P.T[(size_t)c * K * K + x * K + y];
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

// the wide kernels' request fields: the full combination, the operator index
// and the leaf factors (opchain.h OpWideArgs)
void fill_wide(const OpPlan* P, int n_obs, OpWideArgs& w) {
  w.nobs = n_obs;
  for (int i = 0; i < n_obs; i++) { w.col[i] = i; w.card[i] = P->card[i]; w.cstride[i] = P->stride[i]; }
  w.K = P->K;
  w.ncomb = P->ncomb;
  w.onobs = (int)P->oi.size();
  for (int q = 0; q < w.onobs; q++) {
    w.ocol[q] = P->oi[q]; w.ocard[q] = P->card[P->oi[q]]; w.ocstride[q] = P->ostride[q];
  }
  w.oncomb = P->oncomb;
  w.nleaf = (int)P->li.size();
  for (int j = 0; j < w.nleaf; j++) { w.lcol[j] = P->li[j]; w.lcard[j] = P->card[P->li[j]]; w.loff[j] = P->loff[j]; }
  w.ltab = P->dlt;
  w.Ttab = P->dT; w.TtabT = P->dTT; w.w = P->dw; w.pi = P->dpi;
  w.Lbits = P->Lbits;
  for (int j = 0; j < w.nleaf; j++) { w.lsh[j] = P->lsh[j]; w.lbits[j] = P->lbits[j]; w.hoff[j] = P->hoff[j]; }
  w.xrow = (int)P->xrow;
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
  if (P->ok && P->K > 16) return true;                  // the wide kernels read the codes from HBM
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
    (void)hipFree(P->dT); (void)hipFree(P->dTT); (void)hipFree(P->dw); (void)hipFree(P->dpi); (void)hipFree(P->dlt);
    (void)hipFree(P->S);
    P->dT = P->dTT = P->dw = P->dpi = P->dlt = P->S = nullptr;
    P->S_bytes = 0;
    if (upload(&P->dT, P->T) || upload(&P->dTT, P->TT) || upload(&P->dw, P->w) || upload(&P->dpi, P->pi) ||
        upload(&P->dlt, P->lt)) {
      err = "device tables";
      return NIPAMD_ERROR_DEVICE;
    }
    P->device = dev;
  }
  if (P->K > 16) {
    // 17..64 states (op_wide_launch): every message stored, launched in
    // chunks of sequences whose two message arrays stay within ~4 GB
    const size_t per = op_wide_scratch_bytes(P->K, 1, T);
    long chunk = (long)std::max<size_t>(1, ((size_t)4 << 30) / per);
    chunk = std::min<long>(chunk, B > 0 ? B : 1);
    const size_t need = op_wide_scratch_bytes(P->K, chunk, T);
    if (P->S_bytes < need) {
      (void)hipFree(P->S);
      P->S = nullptr;
      P->S_bytes = 0;
      if (hipMalloc(&P->S, need) != hipSuccess) { err = "scratch"; return NIPAMD_ERROR_DEVICE; }
      P->S_bytes = need;
    }
    const long ocols = n_obs > 0 ? n_obs : 1;
    for (long b0 = 0; b0 < B; b0 += chunk) {
      const long nb = std::min<long>(chunk, B - b0);
      OpWideArgs w{};
      w.obs = d_obs ? d_obs + b0 * T * ocols : nullptr;
      w.obs_bstride = (long)T * ocols;
      w.obs_tstride = (int)ocols;
      fill_wide(P, n_obs, w);
      w.B = nb; w.T = T;
      w.filter = filt ? 1 : 0;
      w.Sa = P->S;
      w.Sb = P->S + (size_t)nb * T * op_wide_np(P->K);
      w.post = d_joint ? d_joint + b0 * jbs : nullptr;
      w.post_bstride = jbs; w.post_tstride = jts; w.post_off = joff;
      w.ll = d_ll ? d_ll + b0 : nullptr;
      w.status = d_status ? d_status + b0 : nullptr;
      if (int rc = op_wide_launch(w, (hipStream_t)stream)) return op_launch_fail(rc, "op_wide_msgs_kernel", err);
    }
    if (K_out) *K_out = P->K;
    return 0;
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
  if (rc) return op_launch_fail(rc, "op_fb_kernel", err);
  return 0;
}

// ---------------------------------------------------------------------------
// e_step on the operator chain.  The reference's e_step (nip.c:1708-2007)
// sums every variable's normalised family marginal over the steps
// (nip.c:1925-1967; the previous interface's prior families at t = 0 only).
// On the operator chain the slice's joint posterior at step t is
//   P_t(a) = alpha^_{t-1}(x(a)) W(a) [a consistent with c_t] beta^_t(y(a)) / Z'_t
// (W as in build()), so every family count is linear in the per-combination
// sums Xi_c(x, y) = sum over the steps with combination c of
// alpha^_{t-1}(x) beta^_t(y) / Z'_t (op_fb_kernel's xi weights, summed per
// 16-sequence group by op_xi_kernel and over the batch by the fixed-order
// tree):  count(v, family cell) = sum over assignments a in the cell and
// combinations c consistent with a of W(a) Xi_c(x(a), y(a)); the previous
// interface's families come from P0 (its t = 0 marginal).  That projection
// is a CSR map over the count cells, built per model version by the same
// enumeration as the operators; the finalize applies it.
//
// Partial section (after the model's route tag, nipamd_estep_partial_size_req):
//   [count, f[kOpFields], f^2[kOpFields] | Xi [(ncomb + 1) K K] | P0 [K]]
// with the request's fields f = (n_obs, ov[kOpMaxObs], K, ncomb) -- the
// header's entries are summed with the partials and read back divided by the
// count (exact for these small integers); the squares make the check exact:
// sum(f^2) / n == (sum(f) / n)^2 only when every partial had the same f, so
// partials of different requests whose fields merely average to integers
// ([1] and [3] giving [2], permuted lists) are refused.
namespace {

constexpr int kOpFields = 3 + kOpMaxObs;
constexpr int kOpHdr = 1 + 2 * kOpFields;
constexpr long kOpMaxMapEntries = 1L << 27;

bool build_map(const Model& m, OpPlan& P) {
  const auto& prev = m.previous_outgoing;
  const auto& cur = m.outgoing;
  const int nv = (int)m.vars.size(), K = P.K, no = (int)P.ov.size();
  std::vector<long> off(nv + 1, 0);
  for (int v = 0; v < nv; v++) {
    long sz = m.vars[v].card;
    for (int q : m.vars[v].parents) sz *= m.vars[q].card;
    off[v + 1] = off[v] + sz;
  }
  for (int v = 0; v < nv; v++)
    if ((m.vars[v].ifs & IF_OLD_OUTGOING) &&
        (!m.vars[v].parents.empty() || std::find(prev.begin(), prev.end(), v) == prev.end())) {
      P.map_why = "previous-interface variable with parents or outside the interface";
      return false;
    }
  struct Ent { long row; int idx; double coef; };
  std::vector<Ent> ents;
  std::vector<std::vector<std::pair<int, long>>> cst(m.cliques.size());
  for (size_t c = 0; c < m.cliques.size(); c++) {
    long st = 1;
    for (int v : m.cliques[c].vars) { cst[c].push_back({v, st}); st *= m.vars[v].card; }
  }
  std::vector<int> pri;
  for (int v : m.independent)
    if (m.vars[v].has_prior && !(m.vars[v].ifs & IF_OLD_OUTGOING)) pri.push_back(v);
  // the leaf factors (K > 16, build()): their variables are not enumerated
  // and their cliques leave the product; a counted variable whose family holds
  // a leaf takes its counts from that leaf's count rows instead of Xi'
  std::vector<char> skip(nv, 0), lc(m.cliques.size(), 0);
  for (int i : P.li) skip[P.ov[i]] = 1;
  for (int c : P.lcl) lc[c] = 1;
  auto leaf_of = [&](int v) {                         // the leaf in v's family, -1: none
    for (size_t j = 0; j < P.li.size(); j++) {
      const int l = P.ov[P.li[j]];
      if (v == l || has(m.vars[v].parents, l)) return (int)j;
    }
    return -1;
  };
  std::vector<int> cnt;                               // the counted variables (every step), via Xi'
  for (int v = 0; v < nv; v++)
    if (!(m.vars[v].ifs & IF_OLD_OUTGOING) && leaf_of(v) < 0) cnt.push_back(v);
  long total = 1;
  for (int v = 0; v < nv; v++)
    if (!skip[v]) total *= m.vars[v].card;
  const int nop = (int)P.oi.size();
  std::vector<int> a(nv, 0);
  const long KK = (long)K * K;
  for (long it = 0; it < total; it++) {
    double W = 1.0;                                   // the same product, in the same order, as build()
    for (size_t c = 0; c < m.cliques.size() && W != 0.0; c++) {
      if (lc[c]) continue;
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
      for (long mask = 0; mask < (1L << nop); mask++) {
        long c = 0;
        for (int q = 0; q < nop; q++)
          if (mask >> q & 1) c += (long)(a[P.ov[P.oi[q]]] + 1) * P.ostride[q];
        const int idx = (int)(c * KK + x * K + y);
        for (int v : cnt) {
          long cell = a[v], st = m.vars[v].card;
          for (int q : m.vars[v].parents) { cell += (long)a[q] * st; st *= m.vars[q].card; }
          ents.push_back({off[v] + cell, idx, W});
        }
        if ((long)ents.size() > kOpMaxMapEntries) { P.map_why = "e_step projection too large"; return false; }
      }
    }
    for (int v = 0; v < nv; v++) {                    // odometer, variable 0 fastest
      if (skip[v]) continue;
      if (++a[v] < m.vars[v].card) break;
      a[v] = 0;
    }
  }
  // families holding leaf j: sum_t gamma_t(y) P(leaf = r | y, its code at t)
  // -- the count row of code r (observed r), plus the missing row times
  // F_j[r](y) / F_j[missing](y)
  for (size_t j = 0; j < P.li.size(); j++) {
    const int l = P.ov[P.li[j]], M = P.card[P.li[j]];
    const double* F = P.lt.data() + P.loff[j];
    for (int v = 0; v < nv; v++) {
      if ((m.vars[v].ifs & IF_OLD_OUTGOING) || leaf_of(v) != (int)j) continue;
      for (long y = 0; y < K; y++) {
        std::vector<int> comp(nv, 0);
        long r = y;
        for (int u : cur) { comp[u] = (int)(r % m.vars[u].card); r /= m.vars[u].card; }
        for (int val = 0; val < M; val++) {
          comp[l] = val;
          long cell = comp[v], st = m.vars[v].card;
          for (int q : m.vars[v].parents) { cell += (long)comp[q] * st; st *= m.vars[q].card; }
          ents.push_back({off[v] + cell, (int)(P.hoff[j] + (long)val * K + y), 1.0});
          const double miss = F[(size_t)M * K + y];
          if (miss != 0.0) ents.push_back({off[v] + cell, (int)(P.hoff[j] + (long)M * K + y), F[(size_t)val * K + y] / miss});
        }
      }
    }
  }
  // the previous interface at t = 0: P0 digits
  const int p0 = (int)(P.xrow - K);
  for (int x = 0; x < K; x++) {
    long r = x;
    for (int v : prev) {
      const int card = m.vars[v].card;
      ents.push_back({off[v] + r % card, p0 + x, 1.0});
      r /= card;
    }
  }
  // CSR by a stable counting sort on the row
  const long nrows = off[nv];
  std::vector<int> ptr((size_t)nrows + 1, 0);
  for (const Ent& e : ents) ptr[(size_t)e.row + 1]++;
  for (long r = 0; r < nrows; r++) ptr[(size_t)r + 1] += ptr[(size_t)r];
  std::vector<int> fill(ptr.begin(), ptr.end() - 1), idx(ents.size());
  std::vector<double> coef(ents.size());
  for (const Ent& e : ents) {
    const int q = fill[(size_t)e.row]++;
    idx[(size_t)q] = e.idx;
    coef[(size_t)q] = e.coef;
  }
  if (hipMalloc(&P.d_mptr, ptr.size() * sizeof(int)) != hipSuccess ||
      hipMemcpy(P.d_mptr, ptr.data(), ptr.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
      hipMalloc(&P.d_midx, std::max<size_t>(1, idx.size()) * sizeof(int)) != hipSuccess ||
      (!idx.empty() && hipMemcpy(P.d_midx, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) ||
      upload(&P.d_mcoef, coef)) {
    P.map_why = "device map";
    return false;
  }
  P.map_n = (int)nrows;
  return true;
}

// sequences per launch: a power of two (chunk trees are subtrees of the
// batch tree), the W rows within ~2 GB
long op_estep_chunk(int K, int T) {
  const size_t per = (size_t)T * K * K * sizeof(double) + (size_t)(T + 2) * 16 * sizeof(double);
  long c = 16;
  while (c < 16384 && (size_t)(c * 2) * per <= ((size_t)2 << 30)) c *= 2;
  return c;
}

// 17..64 states: op_wide_msgs_kernel in e_step mode stores every message and
// scale exponent, op_wide_xi_kernel sums the xi weights per combination into
// one slab row per kOpWideSeqs = 8 sequences, and the fixed-order tree reduces the rows --
// per launch a power-of-two chunk of sequences whose messages stay within
// ~4 GB and slab rows within ~8 GB (a row holds (ncomb + 1) K^2 + K doubles:
// 29.6 MB at 20 states and 9261 combinations, so 256 rows fill the chip).
int op_wide_estep(OpPlan* P, const int32_t* d_obs, int n_obs, int B, int T, double* out, double* d_ll,
                  uint32_t* d_status, hipStream_t st, std::string& err) {
  const int K = P->K;
  const long R = P->xrow;
  const size_t per = op_wide_scratch_bytes(K, 1, T) + (size_t)T * sizeof(int);
  size_t budget = (size_t)4 << 30;
  // diagnostics builds: a smaller message budget, so that tests run one batch
  // as several launch chunks
  if (const char* e = diag_env("NIPAMD_OP_WIDE_BYTES")) budget = (size_t)std::atoll(e);
  long chunk = 16;
  while (chunk < 65536 && (size_t)(chunk * 2) * per <= budget &&
         (size_t)(chunk * 2 / kOpWideSeqs) * R * sizeof(double) <= ((size_t)8 << 30))
    chunk *= 2;
  chunk = std::min<long>(chunk, std::max(16, B));
  const long nchunks = (B + chunk - 1) / chunk;
  const long rows = (chunk + kOpWideSeqs - 1) / kOpWideSeqs;
  const long lvl = (rows + 63) / 64;
  const size_t nsc = ((size_t)chunk * T * sizeof(int) + sizeof(double) - 1) / sizeof(double);
  const size_t nE = nsc + (size_t)(rows + 2 * lvl + nchunks + 2 * ((nchunks + 63) / 64) + 1) * R;
  const size_t need = op_wide_scratch_bytes(K, chunk, T);
  if (P->S_bytes < need) {
    (void)hipFree(P->S);
    P->S = nullptr;
    P->S_bytes = 0;
    if (hipMalloc(&P->S, need) != hipSuccess) { err = "scratch"; return NIPAMD_ERROR_DEVICE; }
    P->S_bytes = need;
  }
  if (P->E_bytes < nE * sizeof(double)) {
    (void)hipFree(P->E);
    P->E = nullptr;
    P->E_bytes = 0;
    if (hipMalloc(&P->E, nE * sizeof(double)) != hipSuccess) { err = "e_step buffers"; return NIPAMD_ERROR_DEVICE; }
    P->E_bytes = nE * sizeof(double);
  }
  int* sc = reinterpret_cast<int*>(P->E);
  double* slab = P->E + nsc;
  double* work = slab + (size_t)rows * R;
  double* cres = work + (size_t)2 * lvl * R;
  double* cwork = cres + (size_t)nchunks * R;
  const long ocols = n_obs > 0 ? n_obs : 1;
  for (long c = 0; c < nchunks; c++) {
    const long b0 = c * chunk;
    const long nb = std::min<long>(chunk, B - b0);
    OpWideArgs w{};
    w.obs = d_obs ? d_obs + b0 * T * ocols : nullptr;
    w.obs_bstride = (long)T * ocols;
    w.obs_tstride = (int)ocols;
    fill_wide(P, n_obs, w);
    w.B = nb; w.T = T;
    w.filter = 0;
    w.Sa = P->S;
    w.Sb = P->S + (size_t)nb * T * op_wide_np(K);
    w.post = nullptr;
    w.ll = d_ll ? d_ll + b0 : nullptr;
    w.status = d_status ? d_status + b0 : nullptr;
    w.estep = 1;
    w.sc = sc;
    w.slab = slab;
    if (int rc = op_wide_launch(w, st)) return op_launch_fail(rc, "op_wide_msgs_kernel (e_step)", err);
    if (int rc = op_wide_xi_launch(w, st)) return op_launch_fail(rc, "op_wide_xi_kernel", err);
    const long nr = (nb + kOpWideSeqs - 1) / kOpWideSeqs;
    if (nipamd_tree_sum(slab, nr, (int)R, work, nchunks == 1 ? out : cres + (size_t)c * R, st)) {
      err = "tree launch failed";
      return NIPAMD_ERROR_DEVICE;
    }
  }
  if (nchunks > 1 && nipamd_tree_sum(cres, nchunks, (int)R, cwork, out, st)) {
    err = "tree launch failed";
    return NIPAMD_ERROR_DEVICE;
  }
  g_last_kernel = "op_wide_msgs_kernel (e_step) + op_wide_xi_kernel";
  return 0;
}

}  // namespace

bool op_estep_supported(nipamd_model* mm, int n_obs, const int* obs_vars, int T, std::string& why) {
  OpPlan* P = plan_for(mm, n_obs, obs_vars);
  if (!P->ok) { why = P->why; return false; }
  if (P->K > 16) {
    // op_wide_msgs_kernel + op_wide_xi_kernel: one slab row per 8 sequences (kOpWideSeqs); every
    // block zeroes and writes its row's whole (ncomb + 1) K^2 section, so the slab traffic per
    // sequence is R / 8 doubles whatever the sequence touches (a cost, not a bound)
    if ((size_t)P->xrow * sizeof(double) > kOpMaxWideRow) {
      why = "too many evidence combinations for the wide e_step's slab rows";
      return false;
    }
  } else if (!op_fits(mm, n_obs, obs_vars, T)) {
    why = "sequence too long for the operator chain's LDS codes";
    return false;
  } else if (!op_xi_fits(P->K, P->ncomb) && !op_xi_sort_fits(P->ncomb, T)) {
    why = "too many evidence combinations for the e_step's LDS sums";
    return false;
  }
  const long total = [&] { long t = 1; for (const Var& V : mm->m.vars) t *= V.card; return t; }();
  if (total * (1L << P->ov.size()) * (long)mm->m.vars.size() > kOpMaxMapEntries) {
    why = "e_step projection too large";
    return false;
  }
  return true;
}

long op_estep_section(nipamd_model* mm, int n_obs, const int* obs_vars) {
  OpPlan* P = plan_for(mm, n_obs, obs_vars);
  if (!P->ok) return 0;
  return kOpHdr + P->xrow;
}

int op_estep_partial(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T,
                     double* d_sec, double* d_ll, uint32_t* d_status, void* stream, std::string& err) {
  OpPlan* P = plan_for(mm, n_obs, obs_vars);
  if (!P->ok) { err = P->why; return NIPAMD_ERROR_UNSUPPORTED; }
  hipStream_t st = (hipStream_t)stream;
  const int K = P->K, R = (int)P->xrow;
  // the header (pageable host source: staged before the call returns)
  double hdr[kOpHdr];
  hdr[0] = 1.0;
  hdr[1] = n_obs;
  for (int i = 0; i < kOpMaxObs; i++) hdr[2 + i] = i < n_obs ? obs_vars[i] : -1.0;
  hdr[2 + kOpMaxObs] = K;
  hdr[3 + kOpMaxObs] = P->ncomb;
  for (int i = 0; i < kOpFields; i++) hdr[1 + kOpFields + i] = hdr[1 + i] * hdr[1 + i];
  if (hipMemcpyAsync(d_sec, hdr, sizeof(hdr), hipMemcpyHostToDevice, st) != hipSuccess) {
    err = "header copy";
    return NIPAMD_ERROR_DEVICE;
  }
  double* out = d_sec + kOpHdr;
  if (B == 0) {
    if (hipMemsetAsync(out, 0, (size_t)R * sizeof(double), st) != hipSuccess) { err = "memset"; return NIPAMD_ERROR_DEVICE; }
    return 0;
  }
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) { err = "no device"; return NIPAMD_ERROR_DEVICE; }
  if (P->device != dev || !P->dT) {
    (void)hipFree(P->dT); (void)hipFree(P->dTT); (void)hipFree(P->dw); (void)hipFree(P->dpi); (void)hipFree(P->dlt);
    (void)hipFree(P->S); (void)hipFree(P->E);
    P->dT = P->dTT = P->dw = P->dpi = P->dlt = P->S = P->E = nullptr;
    P->S_bytes = P->E_bytes = 0;
    if (upload(&P->dT, P->T) || upload(&P->dTT, P->TT) || upload(&P->dw, P->w) || upload(&P->dpi, P->pi) ||
        upload(&P->dlt, P->lt)) {
      err = "device tables";
      return NIPAMD_ERROR_DEVICE;
    }
    P->device = dev;
  }
  if (K > 16) return op_wide_estep(P, d_obs, n_obs, B, T, out, d_ll, d_status, st, err);
  const long chunk = std::min<long>(op_estep_chunk(K, T), std::max(16, B));
  const long nchunks = (B + chunk - 1) / chunk;
  const long rows = (chunk + kOpXiSeqs - 1) / kOpXiSeqs;
  const long lvl = (rows + 63) / 64;
  const size_t nW = (size_t)chunk * T * K * K, nP0 = (size_t)chunk * K;
  const size_t nC = ((size_t)chunk * T * sizeof(uint16_t) + sizeof(double) - 1) / sizeof(double);
  const size_t nE = nW + nP0 + nC + (size_t)(rows + 2 * lvl + nchunks + 2 * ((nchunks + 63) / 64) + 1) * R;
  if (P->S_bytes < op_scratch_bytes(chunk, T)) {
    (void)hipFree(P->S);
    P->S = nullptr;
    P->S_bytes = 0;
    if (hipMalloc(&P->S, op_scratch_bytes(chunk, T)) != hipSuccess) { err = "scratch"; return NIPAMD_ERROR_DEVICE; }
    P->S_bytes = op_scratch_bytes(chunk, T);
  }
  if (P->E_bytes < nE * sizeof(double)) {
    (void)hipFree(P->E);
    P->E = nullptr;
    P->E_bytes = 0;
    if (hipMalloc(&P->E, nE * sizeof(double)) != hipSuccess) { err = "e_step buffers"; return NIPAMD_ERROR_DEVICE; }
    P->E_bytes = nE * sizeof(double);
  }
  double* W = P->E;
  double* P0 = W + nW;
  uint16_t* Cc = reinterpret_cast<uint16_t*>(P0 + nP0);
  double* slab = P0 + nP0 + nC;
  double* work = slab + (size_t)rows * R;
  double* cres = work + (size_t)2 * lvl * R;
  double* cwork = cres + (size_t)nchunks * R;
  const long ocols = n_obs > 0 ? n_obs : 1;
  for (long c = 0; c < nchunks; c++) {
    const long b0 = c * chunk;
    const long nb = (B - b0) < chunk ? (B - b0) : chunk;
    OpArgs a{};
    a.obs = d_obs ? d_obs + b0 * T * ocols : nullptr;
    a.obs_bstride = (long)T * ocols;
    a.obs_tstride = (int)ocols;
    a.nobs = n_obs;
    for (int i = 0; i < n_obs; i++) { a.col[i] = i; a.card[i] = P->card[i]; a.cstride[i] = P->stride[i]; }
    a.B = nb; a.T = T; a.H = T / 2; a.K = K; a.ncomb = P->ncomb;
    a.filter = 0;
    a.Ttab = P->dT; a.w = P->dw; a.pi = P->dpi;
    a.S = P->S;
    a.post = nullptr;
    a.ll = d_ll ? d_ll + b0 : nullptr;
    a.status = d_status ? d_status + b0 : nullptr;
    a.estep = 1;
    a.W = W;
    a.P0 = P0;
    a.C = Cc;
    const int rc = op_fb_launch(a, st);
    if (rc) return op_launch_fail(rc, "op_fb_kernel (e_step)", err);
    OpXiArgs x{};
    x.obs = a.obs; x.obs_bstride = a.obs_bstride; x.obs_tstride = a.obs_tstride; x.nobs = n_obs;
    for (int i = 0; i < n_obs; i++) { x.col[i] = i; x.card[i] = P->card[i]; x.cstride[i] = P->stride[i]; }
    x.B = nb; x.T = T; x.K = K; x.ncomb = P->ncomb;
    x.W = W; x.P0 = P0; x.C = Cc; x.slab = slab;
    if (int rc = op_xi_launch(x, st)) return op_launch_fail(rc, "op_xi_kernel", err);
    const long nr = (nb + kOpXiSeqs - 1) / kOpXiSeqs;
    if (nipamd_tree_sum(slab, nr, R, work, nchunks == 1 ? out : cres + (size_t)c * R, stream)) {
      err = "tree launch failed";
      return NIPAMD_ERROR_DEVICE;
    }
  }
  if (nchunks > 1 && nipamd_tree_sum(cres, nchunks, R, cwork, out, stream)) {
    err = "tree launch failed";
    return NIPAMD_ERROR_DEVICE;
  }
  g_last_kernel = op_xi_sort_fits(P->ncomb, T) ? "op_fb_kernel (e_step) + op_xi_sort_kernel"
                                               : "op_fb_kernel (e_step) + op_xi_kernel";
  return 0;
}

int op_estep_finalize(nipamd_model* mm, const double* d_sec, double* d_counts, void* stream, std::string& err) {
  double hdr[kOpHdr];
  if (hipMemcpyAsync(hdr, d_sec, sizeof(hdr), hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
      hipStreamSynchronize((hipStream_t)stream) != hipSuccess) {
    err = "header read";
    return NIPAMD_ERROR_DEVICE;
  }
  const double n = hdr[0];
  // field i of every combined partial was the same integer
  auto val = [&](int i, int& out) {
    const double q = hdr[1 + i] / n;
    out = (int)q;
    return q == (double)out && hdr[1 + kOpFields + i] / n == q * q;
  };
  int nobs = 0, ov[kOpMaxObs], K = 0, ncomb = 0;
  bool ok = n >= 1.0 && n == (double)(long)n && val(0, nobs) && nobs >= 0 && nobs <= kOpMaxObs &&
            val(1 + kOpMaxObs, K) && val(2 + kOpMaxObs, ncomb);
  for (int i = 0; ok && i < kOpMaxObs; i++) {
    int v = 0;
    ok = val(1 + i, v);
    if (i < nobs) ov[i] = v;
  }
  if (!ok) { err = "operator-chain e_step partial: inconsistent header (partials of different requests combined?)"; return NIP_ERROR_INVALID_ARGUMENT; }
  OpPlan* P = plan_for(mm, nobs, ov);
  if (!P->ok || P->K != K || P->ncomb != ncomb) {
    err = "operator-chain e_step partial does not match this model";
    return NIP_ERROR_INVALID_ARGUMENT;
  }
  if (P->map_state == 0) P->map_state = build_map(mm->m, *P) ? 1 : -1;
  if (P->map_state < 0) { err = P->map_why; return NIPAMD_ERROR_UNSUPPORTED; }
  if (op_finalize_launch(d_sec + kOpHdr, P->map_n, P->d_mptr, P->d_midx, P->d_mcoef, d_counts,
                         (hipStream_t)stream)) {
    err = "finalize launch failed";
    return NIPAMD_ERROR_DEVICE;
  }
  return 0;
}

void op_release(nipamd_model* mm) {
  delete static_cast<OpCache*>(mm->op);
  mm->op = nullptr;
}

}  // namespace nipamd
