// jtree_plan.cpp -- host side of the general join-tree engine (jtree.h):
// compiles a request (observed columns, queried variables or e_step
// families) against the model's join tree into a flat schedule, keeps it
// device-resident per model version, and drives the kernels.
//
// Reference correspondence:
//   tables       nip_potential, flat index dimension 0 fastest (src/nippotential.c:58-68)
//   projections  nip_mapper + nip_general_marginalise (src/nipvariable.c:560-589,
//                src/nippotential.c:267-311)
//   base tables  nip_global_retraction (orig_p, src/nipjointree.c:791-817) x use_priors
//                of the independent variables entered every slice (src/nip.c:88-119;
//                a zero prior is never entered, nip_enter_prior :904-943)
//   pi           the OLD_OUTGOING priors entered at t = 0 only
//   evidence     nip_enter_index_observation into the family clique (:832-901)
//   sweeps       nip_collect_evidence / nip_distribute_evidence (:580-673) and the
//                interface messages start_/finish_timeslice_message_pass (src/nip.c:1031-1098)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <vector>

#include "chain_kernels.h"
#include "jtree.h"
#include "model.h"
#include "nip_amd.h"
#include "diag.h"

namespace nipamd {
namespace {

#define JT_HIP(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return set_error(NIPAMD_ERROR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct Plan {
  std::string key;
  JtPlanDev p{};
  int L = 64;
  bool lds = false;
  int* d_ip = nullptr;
  double* d_dp = nullptr;
  int slab = 0;
  int stride = 0;           // query row width
  int stage = 0, waves = 1; // the pools staged in LDS, waves per block (jt_stage_bytes)
  std::vector<int> hI;      // host copies of the pools (until uploaded)
  std::vector<double> hD;
};

struct JtState {
  int device = -1;
  unsigned version = 0;
  std::deque<Plan> plans;          // deque: pointers to plans stay valid
  double* msg = nullptr;    // msgA | msgB
  size_t msg_bytes = 0;
  double* wsg = nullptr;
  size_t wsg_bytes = 0;
  double* work = nullptr;   // e_step slabs + tree levels + chunk results
  size_t work_bytes = 0;
};

void free_plans(JtState* s) {
  for (auto& p : s->plans) { (void)hipFree(p.d_ip); (void)hipFree(p.d_dp); }
  s->plans.clear();
}

void release(JtState* s) {
  free_plans(s);
  (void)hipFree(s->msg); (void)hipFree(s->wsg); (void)hipFree(s->work);
  *s = JtState();
}

JtState* state_of(nipamd_model* mm) {
  if (!mm->m.jt) mm->m.jt = new JtState();
  return static_cast<JtState*>(mm->m.jt);
}

int ensure_buf(double** p, size_t* have, size_t bytes) {
  if (*have >= bytes) return 0;
  (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  JT_HIP(hipMalloc(p, bytes));
  *have = bytes;
  return 0;
}

// ------------------------------------------------------------------ builder
struct Builder {
  const Model& m;
  std::vector<int> card;
  std::vector<int> maps, pres;                 // projection pools (same offsets)
  std::map<std::string, int> proj_cache;
  std::vector<double> dp;
  std::vector<int> visits_f, visits_b, visits_p, downs, outs, facs;
  explicit Builder(const Model& mm) : m(mm) {
    for (const auto& v : m.vars) card.push_back(v.card);
  }

  long clique_size(int c) const {
    long s = 1;
    for (int v : m.cliques[c].vars) s *= card[v];
    return s;
  }

  // projection of clique c onto the ordered variables U: map[i] = index of
  // entry i's sub-index in the U-table, pres = entries of each U-index in
  // increasing i.  Returns the pool offset.
  int proj(int c, const std::vector<int>& U) {
    std::string key = std::to_string(c) + ":";
    for (int v : U) key += std::to_string(v) + ",";
    auto it = proj_cache.find(key);
    if (it != proj_cache.end()) return it->second;
    const auto& cv = m.cliques[c].vars;
    const long size = clique_size(c);
    std::vector<long> ustride(cv.size(), 0);   // contribution of clique dim k to the U index
    long us = 1, D = 1;
    for (int v : U) {
      const auto pos = std::find(cv.begin(), cv.end(), v) - cv.begin();
      ustride[pos] = us;
      us *= card[v];
      D *= card[v];
    }
    const int off = (int)maps.size();
    std::vector<int> idx(cv.size(), 0);
    std::vector<int> mp(size);
    for (long i = 0; i < size; i++) {
      long j = 0;
      for (size_t k = 0; k < cv.size(); k++) j += idx[k] * ustride[k];
      mp[i] = (int)j;
      for (size_t k = 0; k < cv.size(); k++) {           // odometer, dim 0 fastest
        if (++idx[k] < card[cv[k]]) break;
        idx[k] = 0;
      }
    }
    std::vector<int> cnt(D, 0), pr(size);
    const long R = size / D;
    for (long i = 0; i < size; i++) pr[(long)mp[i] * R + cnt[mp[i]]++] = (int)i;
    maps.insert(maps.end(), mp.begin(), mp.end());
    pres.insert(pres.end(), pr.begin(), pr.end());
    proj_cache[key] = off;
    return off;
  }
};

long table_size(const std::vector<int>& card, const std::vector<int>& vs) {
  long s = 1;
  for (int v : vs) s *= card[v];
  return s;
}

// tree rooted at `root`: parent, the sepset to the parent, post-order
void rooted(const Model& m, int root, std::vector<int>& parent, std::vector<int>& psep,
            std::vector<int>& post) {
  const int n = (int)m.cliques.size();
  parent.assign(n, -1);
  psep.assign(n, -1);
  post.clear();
  std::vector<int> stack{root}, order;
  std::vector<char> seen(n, 0);
  seen[root] = 1;
  while (!stack.empty()) {                   // pre-order by the c->sepsets list order
    const int c = stack.back();
    stack.pop_back();
    order.push_back(c);
    const auto& lk = m.cliques[c].links;
    for (auto it = lk.rbegin(); it != lk.rend(); ++it) {
      const auto& s = m.sepsets[*it];
      const int o = s.a == c ? s.b : s.a;
      if (seen[o]) continue;
      seen[o] = 1;
      parent[o] = c;
      psep[o] = *it;
      stack.push_back(o);
    }
  }
  post.assign(order.rbegin(), order.rend());  // children before parents
}

bool prior_entered(const Var& v) {
  if (!v.parents.empty() || !v.has_prior) return false;
  for (double x : v.prior) if (x > 0) return true;       // nip_enter_prior rejects a zero vector
  return false;
}

}  // namespace

// Build the plan of one request.  estep: outputs are the em_learn families of
// every variable; else the queried variables' marginals.
static int build_plan(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query,
                      const int* query, bool estep, Plan& P, std::string& why) {
  const Model& m = mm->m;
  const int nc = (int)m.cliques.size();
  const int nv = (int)m.vars.size();
  if (nc == 0) { why = "model has no cliques"; return NIPAMD_ERROR_UNSUPPORTED; }
  Builder B(m);
  for (int i = 0; i < n_obs; i++) {
    if (obs_vars[i] < 0 || obs_vars[i] >= nv) { why = "bad observed variable"; return NIPAMD_ERROR_UNSUPPORTED; }
    for (int j = 0; j < i; j++) if (obs_vars[j] == obs_vars[i]) { why = "observed variable listed twice"; return NIPAMD_ERROR_UNSUPPORTED; }
  }
  const bool iface = !m.outgoing.empty();
  const int cin = iface ? m.in_clique : 0, cout = iface ? m.out_clique : 0;
  if (iface && (cin < 0 || cout < 0)) { why = "no in/out clique"; return NIPAMD_ERROR_UNSUPPORTED; }
  const std::vector<int> outv = iface ? m.outgoing : std::vector<int>();
  const std::vector<int> prevv = iface ? m.previous_outgoing : std::vector<int>();
  const long K = table_size(B.card, outv);
  if (K != table_size(B.card, prevv)) { why = "interface cardinalities differ"; return NIPAMD_ERROR_UNSUPPORTED; }
  long maxc = 0, total = 0;
  for (int c = 0; c < nc; c++) { maxc = std::max(maxc, B.clique_size(c)); total += B.clique_size(c); }
  if (total > (1L << 28) || K > (1L << 22)) { why = "clique tables too large for the general engine"; return NIPAMD_ERROR_UNSUPPORTED; }

  // workspace: clique tables, one upward-message slot per clique, the
  // interface slots, scratch for marginals, the e_step slab
  std::vector<int> psi(nc), upm(nc);
  long w = 0;
  for (int c = 0; c < nc; c++) { psi[c] = (int)w; w += B.clique_size(c); }
  long maxs = 1;
  for (int c = 0; c < nc; c++) {
    long mx = 1;
    for (int s : m.cliques[c].links) mx = std::max(mx, table_size(B.card, m.sepsets[s].vars));
    upm[c] = (int)w;
    w += mx;
    maxs = std::max(maxs, mx);
  }
  JtPlanDev& p = P.p;
  p.ncl = nc;
  p.K = (int)K;
  p.ws_alpha = (int)w; w += K;
  p.ws_beta = (int)w; w += K;
  long maxout = std::max(K, maxs);
  // outputs
  std::vector<JtOut> outs;
  if (estep) {
    int off = 0;
    for (int v = 0; v < nv; v++) {
      const auto& V = m.vars[v];
      std::vector<int> U{v};
      for (int q : V.parents) U.push_back(q);
      JtOut o{};
      o.psi = psi[V.family];
      o.size = (int)B.clique_size(V.family);
      o.proj = B.proj(V.family, U);
      o.D = (int)table_size(B.card, U);
      o.dst = off;
      o.t0_only = (V.ifs & IF_OLD_OUTGOING) ? 1 : 0;
      off += o.D;
      maxout = std::max(maxout, (long)o.D);
      outs.push_back(o);
    }
    P.slab = off;
  } else {
    int off = 0;
    for (int i = 0; i < n_query; i++) {
      const int q = query[i];
      if (q < 0 || q >= nv) { why = "bad query variable"; return NIPAMD_ERROR_UNSUPPORTED; }
      JtOut o{};
      o.psi = psi[m.vars[q].family];
      o.size = (int)B.clique_size(m.vars[q].family);
      o.proj = B.proj(m.vars[q].family, {q});
      o.D = B.card[q];
      o.dst = off;
      off += o.D;
      maxout = std::max(maxout, (long)o.D);
      outs.push_back(o);
    }
    P.stride = off;
  }
  p.ws_out = (int)w; w += maxout;
  p.ws_slab = (int)w;
  p.slab = estep ? P.slab : 0;
  w += p.slab;
  p.ws = (int)w;

  // base tables: orig_p x the priors entered every slice; pi over the
  // previous interface: the OLD_OUTGOING priors (t = 0)
  std::vector<int> base(nc);
  for (int c = 0; c < nc; c++) {
    base[c] = (int)B.dp.size();
    std::vector<double> t = m.cliques[c].original;
    t.resize(B.clique_size(c), 1.0);
    for (int v = 0; v < nv; v++) {
      const auto& V = m.vars[v];
      if (V.family != c || !prior_entered(V) || (V.ifs & IF_OLD_OUTGOING)) continue;
      const int pr = B.proj(c, {v});
      for (size_t i = 0; i < t.size(); i++) t[i] *= V.prior[B.maps[pr + i]];
    }
    B.dp.insert(B.dp.end(), t.begin(), t.end());
  }
  p.pi_off = (int)B.dp.size();
  {
    std::vector<double> pi(K, 1.0);
    std::vector<int> idx(prevv.size(), 0);
    for (long j = 0; j < K; j++) {
      double x = 1.0;
      for (size_t k = 0; k < prevv.size(); k++)
        if (prior_entered(m.vars[prevv[k]])) x *= m.vars[prevv[k]].prior[idx[k]];
      pi[j] = x;
      for (size_t k = 0; k < prevv.size(); k++) {
        if (++idx[k] < B.card[prevv[k]]) break;
        idx[k] = 0;
      }
    }
    B.dp.insert(B.dp.end(), pi.begin(), pi.end());
  }
  p.w_off = (int)B.dp.size();
  B.dp.resize(B.dp.size() + K, 0.0);          // filled on the device (jt_w_kernel)

  // sweeps
  std::vector<std::vector<JtFac>> obsf(nc);    // evidence factors per clique
  for (int i = 0; i < n_obs; i++) {
    const int v = obs_vars[i], c = m.vars[v].family;
    obsf[c].push_back(JtFac{kJtFacObs, B.proj(c, {v}), i});
  }
  std::vector<JtFac> fac;
  auto sweep = [&](int root, bool with_alpha, bool with_beta, std::vector<JtVisit>& vis,
                   std::vector<int>& parent, std::vector<int>& psep, std::vector<int>& post) {
    rooted(m, root, parent, psep, post);
    vis.clear();
    for (int c : post) {
      JtVisit v{};
      v.size = (int)B.clique_size(c);
      v.base = base[c];
      v.psi = psi[c];
      v.fac0 = (int)fac.size();
      for (const auto& f : obsf[c]) fac.push_back(f);
      if (iface && with_alpha && c == cin) fac.push_back(JtFac{kJtFacMsg, B.proj(c, prevv), p.ws_alpha});
      if (iface && with_beta && c == cout) fac.push_back(JtFac{kJtFacMsg, B.proj(c, outv), p.ws_beta});
      for (int k = 0; k < nc; k++)
        if (parent[k] == c) fac.push_back(JtFac{kJtFacMsg, B.proj(c, m.sepsets[psep[k]].vars), upm[k]});
      v.nfac = (int)fac.size() - v.fac0;
      if (parent[c] >= 0) {
        const auto& sv = m.sepsets[psep[c]].vars;
        v.up_proj = B.proj(c, sv);
        v.up_D = (int)table_size(B.card, sv);
        v.up_msg = upm[c];
      } else {
        v.up_proj = -1;
      }
      vis.push_back(v);
    }
  };
  std::vector<JtVisit> vf, vb, vp;
  std::vector<int> parent, psep, post;
  sweep(cout, true, false, vf, parent, psep, post);
  sweep(cin, false, true, vb, parent, psep, post);
  sweep(cin, true, true, vp, parent, psep, post);
  std::vector<JtDown> dn;
  for (auto it = post.rbegin(); it != post.rend(); ++it) {      // pre-order of the posterior tree
    const int c = *it;
    if (parent[c] < 0) continue;
    const auto& sv = m.sepsets[psep[c]].vars;
    JtDown d{};
    d.p_psi = psi[parent[c]];
    d.p_size = (int)B.clique_size(parent[c]);
    d.pS_proj = B.proj(parent[c], sv);
    d.S_D = (int)table_size(B.card, sv);
    d.mu = upm[c];
    d.tmp = p.ws_out;
    d.c_psi = psi[c];
    d.c_size = (int)B.clique_size(c);
    d.cS_proj = B.proj(c, sv);
    dn.push_back(d);
  }
  p.fwd_root_proj = B.proj(cout, outv);
  p.bwd_root_proj = B.proj(cin, prevv);
  p.fwd_root_psi = psi[cout];
  p.fwd_root_size = (int)B.clique_size(cout);
  p.bwd_root_psi = psi[cin];
  p.bwd_root_size = (int)B.clique_size(cin);

  // int pool: visits | downs | outs | factors | maps | pres
  std::vector<int> I;
  auto put = [&I](const void* s, size_t bytes) {
    const int* q = static_cast<const int*>(s);
    I.insert(I.end(), q, q + bytes / sizeof(int));
  };
  p.fwd = (int)I.size(); put(vf.data(), vf.size() * sizeof(JtVisit));
  p.bwd = (int)I.size(); put(vb.data(), vb.size() * sizeof(JtVisit));
  p.post = (int)I.size(); put(vp.data(), vp.size() * sizeof(JtVisit));
  p.down = (int)I.size(); p.ndown = (int)dn.size(); put(dn.data(), dn.size() * sizeof(JtDown));
  p.out = (int)I.size(); p.nout = (int)outs.size(); put(outs.data(), outs.size() * sizeof(JtOut));
  p.fac = (int)I.size(); put(fac.data(), fac.size() * sizeof(JtFac));
  p.maps = (int)I.size(); I.insert(I.end(), B.maps.begin(), B.maps.end());
  p.pres = (int)I.size(); I.insert(I.end(), B.pres.begin(), B.pres.end());
  if (I.size() > (size_t)0x7fffffff) { why = "schedule too large"; return NIPAMD_ERROR_UNSUPPORTED; }

  P.L = maxc <= 64 && K <= 64 && maxout <= 64 ? 16 : 64;
  if (const char* e = diag_env("NIPAMD_JT_L")) {       // A/B: lanes per unit (16, 32 or 64)
    const int l = std::atoi(e);
    if (l == 16 || l == 32 || l == 64) P.L = l;
  }
  P.lds = (size_t)(64 / P.L) * p.ws * sizeof(double) <= 64 * 1024;
  // round 6: every block stages the pools (schedule, index maps, pre-images,
  // base tables) in LDS once and runs up to four waves on them, instead of
  // each unit reading them from L2 at every step; NIPAMD_JT_STAGE=0 in
  // diagnostics builds keeps the round-3 form
  p.n_ip = (int)I.size();
  p.n_dp = (int)B.dp.size();
  {
    const size_t sb = jt_stage_bytes(p), wsb = P.lds ? (size_t)(64 / P.L) * p.ws * sizeof(double) : 0;
    int W = 4;
    while (W > 1 && sb + W * wsb > 160 * 1024) W /= 2;
    P.stage = sb + W * wsb <= 160 * 1024 ? 1 : 0;
    P.waves = P.stage ? W : 1;
    if (const char* e = diag_env("NIPAMD_JT_STAGE"))
      if (std::atoi(e) == 0) { P.stage = 0; P.waves = 1; }
  }
  P.hI = std::move(I);
  P.hD = std::move(B.dp);
  return 0;
}

static int upload_plan(Plan& P) {
  JT_HIP(hipMalloc(&P.d_ip, P.hI.size() * sizeof(int)));
  JT_HIP(hipMemcpy(P.d_ip, P.hI.data(), P.hI.size() * sizeof(int), hipMemcpyHostToDevice));
  JT_HIP(hipMalloc(&P.d_dp, P.hD.size() * sizeof(double)));
  JT_HIP(hipMemcpy(P.d_dp, P.hD.data(), P.hD.size() * sizeof(double), hipMemcpyHostToDevice));
  P.p.ip = P.d_ip;
  P.p.dp = P.d_dp;
  P.hI.clear(); P.hI.shrink_to_fit();
  P.hD.clear(); P.hD.shrink_to_fit();
  return 0;
}

static std::string request_key(int n_obs, const int* obs_vars, int n_query, const int* query, bool estep) {
  std::string k = estep ? "E|" : "Q|";
  for (int i = 0; i < n_obs; i++) k += std::to_string(obs_vars[i]) + ",";
  k += "|";
  if (!estep) for (int i = 0; i < n_query; i++) k += std::to_string(query[i]) + ",";
  return k;
}

// the plan of a request on the current device (built and uploaded once per
// model version), with its m1 weights computed on the device
static int get_plan(nipamd_model* mm, int n_obs, const int* obs_vars, int n_query, const int* query,
                    bool estep, Plan** out, hipStream_t st) {
  JtState* s = state_of(mm);
  int dev = -1;
  JT_HIP(hipGetDevice(&dev));
  if (s->device != dev) { release(s); s->device = dev; }
  if (s->version != mm->version) { free_plans(s); s->version = mm->version; }
  const std::string key = request_key(n_obs, obs_vars, n_query, query, estep);
  for (auto& p : s->plans) if (p.key == key) { *out = &p; return 0; }
  Plan P;
  P.key = key;
  std::string why;
  if (int rc = build_plan(mm, n_obs, obs_vars, n_query, query, estep, P, why))
    return rc == NIPAMD_ERROR_UNSUPPORTED ? set_error(rc, "general engine: " + why) : rc;
  if (int rc = upload_plan(P)) {
    (void)hipFree(P.d_ip); (void)hipFree(P.d_dp);
    return rc;
  }
  // m1 weights (one block, workspace in the global slot)
  if (int rc = ensure_buf(&s->wsg, &s->wsg_bytes, (size_t)(64 / P.L) * P.p.ws * sizeof(double))) return rc;
  JtRun r{};
  r.p = P.p;
  r.wsg = s->wsg;
  r.gunits = jt_global_units(P.p.ws);
  if (jt_w_launch(r, P.d_dp + P.p.w_off, P.L, st)) {
    (void)hipFree(P.d_ip); (void)hipFree(P.d_dp);
    return set_error(NIPAMD_ERROR_DEVICE, "jtree: m1-weight launch failed");
  }
  s->plans.push_back(P);
  *out = &s->plans.back();
  return 0;
}

// sequences per launch: bounds the message scratch (2 x B x T x K doubles)
static long seq_chunk(long B, int T, int K, long cap_units = 1L << 27) {
  long c = cap_units / ((long)T * K);
  if (c < 1) c = 1;
  long p2 = 1;
  while (p2 * 2 <= c) p2 *= 2;
  return std::min(B, p2);
}

int jt_supported(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query, const int* query,
                 std::string& why) {
  const Model& m = mm->m;
  const int nv = (int)m.vars.size();
  if (m.cliques.empty()) { why = "model has no cliques"; return 0; }
  for (int i = 0; i < n_obs; i++) {
    if (!obs_vars || obs_vars[i] < 0 || obs_vars[i] >= nv) { why = "bad observed variable"; return 0; }
    for (int j = 0; j < i; j++) if (obs_vars[j] == obs_vars[i]) { why = "observed variable listed twice"; return 0; }
  }
  for (int i = 0; i < n_query; i++)
    if (!query || query[i] < 0 || query[i] >= nv) { why = "bad query variable"; return 0; }
  long total = 0;
  for (const auto& c : m.cliques) {
    long s = 1;
    for (int v : c.vars) s *= m.vars[v].card;
    total += s;
  }
  if (total > (1L << 28)) { why = "clique tables too large for the general engine"; return 0; }
  return 1;
}

int jt_fb(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T,
          int n_query, const int* query, double* d_post, double* d_ll, uint32_t* d_status,
          void* stream, bool filt) {
  hipStream_t st = (hipStream_t)stream;
  Plan* P = nullptr;
  if (int rc = get_plan(mm, n_obs, obs_vars, n_query, query, false, &P, st)) return rc;
  JtState* s = state_of(mm);
  const int K = P->p.K;
  const long chunk = seq_chunk(B, T, K);
  if (int rc = ensure_buf(&s->msg, &s->msg_bytes, (size_t)2 * chunk * T * K * sizeof(double))) return rc;
  if (!P->lds)
    if (int rc = ensure_buf(&s->wsg, &s->wsg_bytes, (size_t)2 * jt_global_units(P->p.ws) * P->p.ws * sizeof(double))) return rc;
  const long ocols = n_obs > 0 ? n_obs : 1;
  for (long b0 = 0; b0 < B; b0 += chunk) {
    const long nb = std::min<long>(chunk, B - b0);
    JtRun r{};
    r.p = P->p;
    r.obs = n_obs > 0 ? d_obs + b0 * T * ocols : nullptr;
    r.obs_bstride = (long)T * ocols;
    r.obs_tstride = (int)ocols;
    r.nobs = n_obs;
    r.B = nb;
    r.T = T;
    r.msgA = s->msg;
    r.msgB = s->msg + (size_t)chunk * T * K;
    r.wsg = s->wsg;
    r.gunits = jt_global_units(P->p.ws);
    r.post = d_post ? d_post + b0 * (long)T * P->stride : nullptr;
    r.post_bstride = (long)T * P->stride;
    r.post_tstride = P->stride;
    r.ll = d_ll ? d_ll + b0 : nullptr;
    r.status = d_status ? (unsigned*)d_status + b0 : nullptr;
    r.filter = filt ? 1 : 0;
    r.stage = P->stage;
    r.waves = P->waves;
    // posterior units: (sequence, chunk of steps), enough of them to fill the chip
    long nch = std::max<long>(1, std::min<long>(T, 16384 / std::max<long>(1, nb)));
    r.chunk = (int)((T + nch - 1) / nch);
    if (jt_filter_launch(r, P->L, P->lds, filt ? 0 : 2, st))
      return set_error(NIPAMD_ERROR_DEVICE, std::string("jtree filter launch: ") + hipGetErrorString(hipGetLastError()));
    if (P->stride > 0 && d_post)
      if (jt_post_launch(r, P->L, P->lds, st))
        return set_error(NIPAMD_ERROR_DEVICE, std::string("jtree posterior launch: ") + hipGetErrorString(hipGetLastError()));
  }
  return 0;
}

int jt_estep_partial(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T,
                     double* d_partial, double* d_ll, uint32_t* d_status, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  Plan* P = nullptr;
  if (int rc = get_plan(mm, n_obs, obs_vars, 0, nullptr, true, &P, st)) return rc;
  JtState* s = state_of(mm);
  const int S = P->slab;
  if (B == 0) { JT_HIP(hipMemsetAsync(d_partial, 0, (size_t)S * sizeof(double), st)); return 0; }
  const int K = P->p.K;
  // the posterior sweep's units: (sequence, one of nch time chunks), nch a
  // power of two that depends on T only, one slab row per unit in (sequence,
  // chunk) order -- a batch's tree over them contains every power-of-two
  // shard's as a subtree, so shard partials still combine bit for bit
  // (and exactly nch units: ceil(T / ceil(T / nch)) == nch, true whenever
  // (nch - 1)^2 < T, so a short T takes fewer chunks)
  int nch = 16;
  while (nch > 1 && (nch - 1) * ((T + nch - 1) / nch) >= T) nch /= 2;
  const int tch = (T + nch - 1) / nch;
  // power-of-two sequence chunks: chunk trees are subtrees of the batch tree
  long chunk = std::min(seq_chunk(B, T, K), seq_chunk(B, 1, (int)std::min<long>((long)S * nch, 1L << 30), 1L << 26));
  chunk = std::min<long>(chunk, 16384);
  const long nchunks = (B + chunk - 1) / chunk;
  const long rows = chunk * nch;
  const long lvl = (rows + 63) / 64;
  if (int rc = ensure_buf(&s->msg, &s->msg_bytes, (size_t)2 * chunk * T * K * sizeof(double))) return rc;
  if (!P->lds)
    if (int rc = ensure_buf(&s->wsg, &s->wsg_bytes, (size_t)2 * jt_global_units(P->p.ws) * P->p.ws * sizeof(double))) return rc;
  if (int rc = ensure_buf(&s->work, &s->work_bytes,
                          ((size_t)rows + 2 * lvl + nchunks + 64) * S * sizeof(double))) return rc;
  double* slab = s->work;
  double* tA = slab + (size_t)rows * S;
  double* tB = tA + (size_t)lvl * S;
  double* cres = tB + (size_t)lvl * S;
  const long ocols = n_obs > 0 ? n_obs : 1;
  auto reduce = [&](const double* in, long n, double* out) -> int {
    const double* cur = in;
    while (n > 64) {
      double* dst = (cur == tA) ? tB : tA;
      if (tree_reduce_launch(cur, n, S, dst, st)) return -1;
      cur = dst;
      n = (n + 63) / 64;
    }
    return tree_reduce_launch(cur, n, S, out, st);
  };
  for (long c = 0; c < nchunks; c++) {
    const long b0 = c * chunk;
    const long nb = std::min<long>(chunk, B - b0);
    JtRun r{};
    r.p = P->p;
    r.obs = n_obs > 0 ? d_obs + b0 * T * ocols : nullptr;
    r.obs_bstride = (long)T * ocols;
    r.obs_tstride = (int)ocols;
    r.nobs = n_obs;
    r.B = nb;
    r.T = T;
    r.msgA = s->msg;
    r.msgB = s->msg + (size_t)chunk * T * K;
    r.wsg = s->wsg;
    r.gunits = jt_global_units(P->p.ws);
    r.ll = d_ll ? d_ll + b0 : nullptr;
    r.status = d_status ? (unsigned*)d_status + b0 : nullptr;
    r.slabs = slab;
    r.estep = 1;
    r.chunk = tch;
    r.stage = P->stage;
    r.waves = P->waves;
    if (jt_filter_launch(r, P->L, P->lds, 2, st) || jt_post_launch(r, P->L, P->lds, st))
      return set_error(NIPAMD_ERROR_DEVICE, std::string("jtree e_step launch: ") + hipGetErrorString(hipGetLastError()));
    double* out = nchunks == 1 ? d_partial : cres + (size_t)c * S;
    if (reduce(slab, nb * nch, out))
      return set_error(NIPAMD_ERROR_DEVICE, "jtree e_step reduction launch failed");
  }
  if (nchunks > 1 && reduce(cres, nchunks, d_partial))
    return set_error(NIPAMD_ERROR_DEVICE, "jtree e_step reduction launch failed");
  return 0;
}

int jt_estep_finalize(const nipamd_model* mm, const double* d_partial, double* d_counts, void* stream) {
  if (jt_add_launch(d_partial, d_counts, param_size(mm->m), (hipStream_t)stream))
    return set_error(NIPAMD_ERROR_DEVICE, "jtree finalize launch failed");
  return 0;
}

int jt_query_stride(const nipamd_model* mm, int n_query, const int* query) {
  int s = 0;
  for (int i = 0; i < n_query; i++) s += mm->m.vars[query[i]].card;
  return s;
}

// The host-compiled schedule of a request without touching the device (test
// hook: tests/jt_emul.py interprets it step by step against the oracle).
int jt_plan_dump(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query, const int* query,
                 int estep, int* hdr, int hdr_cap, int* ip, long ip_cap, double* dp, long dp_cap,
                 long* sizes) {
  Plan P;
  std::string why;
  if (int rc = build_plan(mm, n_obs, obs_vars, n_query, query, estep != 0, P, why))
    return rc == NIPAMD_ERROR_UNSUPPORTED ? set_error(rc, why) : rc;
  const JtPlanDev& p = P.p;
  const int h[] = {p.ncl, p.K, p.ws, p.fwd, p.bwd, p.post, p.down, p.ndown, p.out, p.nout, p.fac,
                   p.maps, p.pres, p.fwd_root_proj, p.bwd_root_proj, p.fwd_root_psi, p.fwd_root_size,
                   p.bwd_root_psi, p.bwd_root_size, p.pi_off, p.w_off, p.ws_alpha, p.ws_beta,
                   p.ws_out, p.ws_slab, p.slab, P.L, P.lds ? 1 : 0, P.stride};
  const int nh = (int)(sizeof(h) / sizeof(h[0]));
  for (int i = 0; i < nh && i < hdr_cap; i++) hdr[i] = h[i];
  sizes[0] = (long)P.hI.size();
  sizes[1] = (long)P.hD.size();
  if (ip) std::memcpy(ip, P.hI.data(), std::min<long>(ip_cap, sizes[0]) * sizeof(int));
  if (dp) std::memcpy(dp, P.hD.data(), std::min<long>(dp_cap, sizes[1]) * sizeof(double));
  return 0;
}

void jt_release(nipamd_model* mm) {
  if (!mm->m.jt) return;
  JtState* s = static_cast<JtState*>(mm->m.jt);
  release(s);
  delete s;
  mm->m.jt = nullptr;
}

}  // namespace nipamd
