// generate_data (src/nip.c:2325-2478) on the GPU: host side.
//
// For an interface-chain model (model.h ChainPlan: prev X0, cur X1, hidden
// independent parents H of X1, leaf children O of X1) the reference draws,
// in every slice, the variables in the order of nip.c:2343-2375 (independent
// variables in model order, then repeated passes over the model picking the
// variables whose parents are drawn), each from get_probability() after the
// earlier draws were entered.  With the slice factor
//     W(x0, h, x1, o) = pi'(x0) prod_h p_h(h) F(x0, h, x1) prod_k E_k(x1, o_k)
// (F, E_k: the compiled clique tables, normalised as the reference's parser
// leaves them; pi' the prior of X0 in the first slice, the forward message
// -- a point mass at the previous X1 -- after) those conditionals are:
//   independent u_i:  W summed over the undrawn independents, x1 and o, with
//                     S(x1) = prod_k sum_o E_k(x1, o) for the children
//   X1:               F(x0, h, x1) S(x1) at the drawn x0, h
//   O_k:              E_k(x1, o) at the drawn x1
// each normalised as nip_normalise_array (no-op on a zero sum).  The tables
// are built once per model version and kept on the device; the kernel
// (generate.hip) only indexes them.  The summation order differs from the
// reference's join-tree propagation, so a conditional may differ in its last
// bits; a draw can then differ only when rand()/RAND_MAX lands within those
// bits of a cumulative boundary.
//
// glibc rand() (TYPE_3): srand(seed) fills r[0..30] by 16807 * r mod 2^31-1,
// r[31..33] = r[0..2], r[n] = r[n-31] + r[n-3] (mod 2^32) after, and the k-th
// rand() is r[344 + k] >> 1.  Series b starts at draw o = b * T * nv; its
// window r[313 + o .. 343 + o] is x^o mod (x^31 - x^28 - 1) (the
// recurrence's characteristic polynomial) applied to r[313..373]: the host
// computes x^(T nv) once, rand_window_kernel raises it to the b-th power per
// series (nipamd_rand_windows is the host form, for tests).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "chain_kernels.h"
#include "model.h"
#include "nip_amd.h"

namespace nipamd {

namespace {

using Poly = std::vector<uint32_t>;   // 31 coefficients, mod 2^32

Poly polymulmod(const Poly& a, const Poly& b) {
  std::vector<uint32_t> c(61, 0);
  for (int i = 0; i < 31; i++)
    if (a[i])
      for (int j = 0; j < 31; j++) c[i + j] += a[i] * b[j];
  for (int d = 60; d >= 31; d--) {       // x^31 = x^28 + 1
    c[d - 3] += c[d];
    c[d - 31] += c[d];
  }
  return Poly(c.begin(), c.begin() + 31);
}

Poly xpow(long n) {
  Poly r(31, 0), base(31, 0);
  r[0] = 1;
  base[1] = 1;
  while (n > 0) {
    if (n & 1) r = polymulmod(r, base);
    base = polymulmod(base, base);
    n >>= 1;
  }
  return r;
}

// r[0..count) of glibc's srand(seed) state sequence
std::vector<uint32_t> glibc_state(unsigned seed, int count) {
  std::vector<uint32_t> r(std::max(count, 34));
  int32_t word = (int32_t)(seed == 0 ? 1u : seed);
  r[0] = (uint32_t)word;
  for (int i = 1; i < 31; i++) {
    const long hi = word / 127773, lo = word % 127773;
    long w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    word = (int32_t)w;
    r[i] = (uint32_t)word;
  }
  for (int i = 31; i < 34; i++) r[i] = r[i - 31];
  for (int i = 34; i < (int)r.size(); i++) r[i] = r[i - 31] + r[i - 3];
  return r;
}

void normalise_rows(double* t, size_t n, int card) {
  for (size_t i = 0; i < n; i += card) {
    double s = 0.0;
    for (int k = 0; k < card; k++) s += t[i + k];
    if (s != 0.0)
      for (int k = 0; k < card; k++) t[i + k] /= s;
  }
}

struct GenCache {
  unsigned version = 0;
  int device = -1;
  std::vector<int> order;             // sampling order (model variables)
  std::vector<GenStep> steps;
  int x1_step = 0;
  long zero_off = 0;
  long cum_off = 0;                   // the running-sum tables follow the tables
  GenStep* d_steps = nullptr;
  double* d_tab = nullptr;
  uint32_t* d_win = nullptr;
  size_t win_cap = 0;
};

std::mutex g_mu;
std::unordered_map<const nipamd_model*, GenCache> g_cache;

void release(GenCache& c) {
  (void)hipFree(c.d_steps);
  (void)hipFree(c.d_tab);
  (void)hipFree(c.d_win);
  c.d_steps = nullptr;
  c.d_tab = nullptr;
  c.d_win = nullptr;
  c.win_cap = 0;
}

// the order of nip.c:2343-2375
std::vector<int> sampling_order(const Model& m) {
  const int n = (int)m.vars.size();
  std::vector<int> order;
  std::vector<char> mark(n, 0);
  for (int i = 0; i < n; i++)
    if (m.vars[i].parents.empty()) { order.push_back(i); mark[i] = 1; }
  while ((int)order.size() < n) {
    const size_t before = order.size();
    for (int i = 0; i < n; i++) {
      if (mark[i]) continue;
      bool ok = true;
      for (int p : m.vars[i].parents) ok &= mark[p] != 0;
      if (ok) { order.push_back(i); mark[i] = 1; }
    }
    if (order.size() == before) break;   // a cycle: cannot happen in a parsed DAG
  }
  return order;
}

long clique_idx(const Model& m, int c, const std::vector<int>& val) {
  long idx = 0, stride = 1;
  for (int v : m.cliques[c].vars) { idx += val[v] * stride; stride *= m.vars[v].card; }
  return idx;
}

#define GEN_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_error(NIPAMD_ERROR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

int build_tables(const nipamd_model* mm, GenCache& g) {
  const Model& m = mm->m;
  const ChainPlan& P = m.chain;
  const auto& V = m.vars;
  if (!P.valid || P.joint) return set_error(NIPAMD_ERROR_UNSUPPORTED, "generate: the model has no single-variable interface-chain plan");
  if (P.hidden.size() + 2 > (size_t)kGenMaxCtx || V.size() > (size_t)kGenMaxVars)
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "generate: too many variables in the slice");
  const int N = P.N, vp = P.v_prev, vc = P.v_cur, cin = P.c_trans;
  g.order = sampling_order(m);
  const int nv = (int)g.order.size();
  if (nv != (int)V.size()) return set_error(NIP_ERROR_GENERAL, "generate: no sampling order");
  std::vector<int> step_of(V.size(), -1);
  for (int i = 0; i < nv; i++) step_of[g.order[i]] = i;
  std::vector<int> ind, hid;                  // independents (X0 and H) / H, sampling order
  for (int v : g.order)
    if (V[v].parents.empty()) {
      ind.push_back(v);
      if (v != vp) hid.push_back(v);
    }
  long hsize = 1;
  for (int h : hid) hsize *= V[h].card;
  // F(x0, h, x1) S(x1) (X1's table) and K(x0, h) = sum_x1 F S
  const std::vector<double>& S = P.s_all64;
  std::vector<double> X1tab((size_t)N * hsize * N);      // [x0][h, first slowest][x1]
  std::vector<double> K((size_t)N * hsize, 0.0);
  std::vector<int> val(V.size(), 0);
  for (int x0 = 0; x0 < N; x0++)
    for (long hi = 0; hi < hsize; hi++) {
      long r = hi;
      for (int q = (int)hid.size() - 1; q >= 0; q--) { val[hid[q]] = (int)(r % V[hid[q]].card); r /= V[hid[q]].card; }
      val[vp] = x0;
      double k = 0.0;
      double* row = X1tab.data() + ((size_t)x0 * hsize + hi) * N;
      for (int x1 = 0; x1 < N; x1++) {
        val[vc] = x1;
        row[x1] = m.cliques[cin].original[clique_idx(m, cin, val)] * S[x1];
        k += row[x1];
      }
      K[(size_t)x0 * hsize + hi] = k;
    }
  normalise_rows(X1tab.data(), X1tab.size(), N);
  std::vector<double> tab;
  std::vector<std::pair<long, int>> segs;     // (offset, row length) of every table
  auto append = [&](const std::vector<double>& t, int card) {
    const long off = (long)tab.size();
    tab.insert(tab.end(), t.begin(), t.end());
    segs.push_back({off, card});
    return off;
  };
  auto hweight = [&](long hi) {               // prod p_h over the H of index hi
    double w = 1.0;
    for (int q = (int)hid.size() - 1; q >= 0; q--) {
      w *= V[hid[q]].prior[hi % V[hid[q]].card];
      hi /= V[hid[q]].card;
    }
    return w;
  };
  g.steps.assign(nv, GenStep());
  // first slice: W0 over the independents in sampling order (first slowest)
  {
    std::vector<int> cards;
    for (int u : ind) cards.push_back(V[u].card);
    long wsize = 1;
    for (int c : cards) wsize *= c;
    std::vector<double> W0(wsize);
    std::vector<int> uv(ind.size());
    for (long wi = 0; wi < wsize; wi++) {
      long r = wi;
      for (int q = (int)ind.size() - 1; q >= 0; q--) { uv[q] = (int)(r % cards[q]); r /= cards[q]; }
      long hi = 0;
      int x0 = 0;
      for (size_t q = 0; q < ind.size(); q++) {
        if (ind[q] == vp) x0 = uv[q];
        else hi = hi * cards[q] + uv[q];
      }
      W0[wi] = V[vp].prior[x0] * hweight(hi) * K[(size_t)x0 * hsize + hi];
    }
    long prefix = 1;
    for (size_t q = 0; q < ind.size(); q++) {
      prefix *= cards[q];
      const long block = wsize / prefix;
      std::vector<double> Tq(prefix, 0.0);
      for (long i = 0; i < prefix; i++)
        for (long j = 0; j < block; j++) Tq[i] += W0[i * block + j];
      normalise_rows(Tq.data(), Tq.size(), cards[q]);
      GenStep& s = g.steps[step_of[ind[q]]];
      s.card = cards[q];
      s.off0 = append(Tq, cards[q]);
      s.nctx = (int)q;
      long stride = cards[q];
      for (int c = (int)q - 1; c >= 0; c--) {
        s.ctx[c] = step_of[ind[c]];
        s.stride[c] = stride;
        stride *= cards[c];
      }
    }
  }
  // later slices: X0 is the previous X1 (a point mass: identity rows); the H
  // are drawn from W1[x0][h] = prod p_h K given x0 and the H drawn before
  {
    std::vector<double> I((size_t)N * N, 0.0);
    for (int x = 0; x < N; x++) I[(size_t)x * N + x] = 1.0;
    GenStep& s0 = g.steps[step_of[vp]];
    s0.off1 = append(I, N);
    s0.nctx1 = 1;
    s0.ctx1[0] = -1;
    s0.stride1[0] = N;
    std::vector<double> W1((size_t)N * hsize);
    for (int x0 = 0; x0 < N; x0++)
      for (long hi = 0; hi < hsize; hi++) W1[(size_t)x0 * hsize + hi] = hweight(hi) * K[(size_t)x0 * hsize + hi];
    long prefix = N;
    for (size_t q = 0; q < hid.size(); q++) {
      const int cq = V[hid[q]].card;
      prefix *= cq;
      const long block = (long)N * hsize / prefix;
      std::vector<double> Tq(prefix, 0.0);
      for (long i = 0; i < prefix; i++)
        for (long j = 0; j < block; j++) Tq[i] += W1[i * block + j];
      normalise_rows(Tq.data(), Tq.size(), cq);
      GenStep& s = g.steps[step_of[hid[q]]];
      s.off1 = append(Tq, cq);
      s.nctx1 = (int)q + 1;
      long stride = cq;
      for (int c = (int)q - 1; c >= 0; c--) {
        s.ctx1[c + 1] = step_of[hid[c]];
        s.stride1[c + 1] = stride;
        stride *= V[hid[c]].card;
      }
      s.ctx1[0] = -1;
      s.stride1[0] = stride;
    }
  }
  // X1 given x0 and h (every slice)
  {
    GenStep& s = g.steps[step_of[vc]];
    s.card = N;
    s.off0 = s.off1 = append(X1tab, N);
    s.nctx = s.nctx1 = 1 + (int)hid.size();
    long stride = N;
    for (int q = (int)hid.size() - 1; q >= 0; q--) {
      s.ctx[q + 1] = s.ctx1[q + 1] = step_of[hid[q]];
      s.stride[q + 1] = s.stride1[q + 1] = stride;
      stride *= V[hid[q]].card;
    }
    s.ctx[0] = s.ctx1[0] = step_of[vp];
    s.stride[0] = s.stride1[0] = stride;
  }
  // leaf children given x1
  for (const ChainEmit& E : P.emits) {
    std::vector<double> T((size_t)N * E.M);
    for (int y = 0; y < N; y++)
      for (int o = 0; o < E.M; o++) T[(size_t)y * E.M + o] = E.E[(size_t)o * 64 + y];
    normalise_rows(T.data(), T.size(), E.M);
    GenStep& s = g.steps[step_of[E.var]];
    s.card = E.M;
    s.off0 = s.off1 = append(T, E.M);
    s.nctx = s.nctx1 = 1;
    s.ctx[0] = s.ctx1[0] = step_of[vc];
    s.stride[0] = s.stride1[0] = E.M;
  }
  int maxc = 1;
  for (const GenStep& s : g.steps) maxc = std::max(maxc, s.card);
  g.zero_off = append(std::vector<double>(maxc, 0.0), maxc);
  // running sums of every row, added in lottery()'s order (sum += d[i++],
  // nip.c:2512-2518) so the kernel compares exactly the reference's sums
  std::vector<double> cum(tab.size());
  for (size_t k = 0; k < segs.size(); k++) {
    const long end = k + 1 < segs.size() ? segs[k + 1].first : (long)tab.size();
    for (long i = segs[k].first; i < end; i += segs[k].second) {
      double sum = 0.0;
      for (int j = 0; j < segs[k].second; j++) cum[i + j] = (sum += tab[i + j]);
    }
  }
  tab.insert(tab.end(), cum.begin(), cum.end());
  g.cum_off = (long)cum.size();
  g.x1_step = step_of[vc];
  release(g);
  GEN_HIP(hipMalloc(&g.d_steps, sizeof(GenStep) * nv));
  GEN_HIP(hipMemcpy(g.d_steps, g.steps.data(), sizeof(GenStep) * nv, hipMemcpyHostToDevice));
  GEN_HIP(hipMalloc(&g.d_tab, sizeof(double) * tab.size()));
  GEN_HIP(hipMemcpy(g.d_tab, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice));
  g.version = mm->version;
  return NIP_NO_ERROR;
}

int prepare(const nipamd_model* mm, GenCache*& out) {
  int dev = -1;
  GEN_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_mu);
  GenCache& g = g_cache[mm];
  if (g.d_tab && g.version == mm->version && g.device == dev) {
    out = &g;
    return NIP_NO_ERROR;
  }
  if (g.device != dev) { release(g); g.device = dev; }
  if (int rc = build_tables(mm, g)) return rc;
  out = &g;
  return NIP_NO_ERROR;
}

int rand_windows(long seed, int B, long draws, uint32_t* win) {
  const std::vector<uint32_t> r = glibc_state((unsigned)seed, 374);
  const Poly Q = xpow(draws);
  std::vector<uint32_t> w(r.begin() + 313, r.begin() + 344), ext(61);
  for (int b = 0; b < B; b++) {
    std::memcpy(win + (size_t)b * 31, w.data(), 31 * sizeof(uint32_t));
    if (b + 1 == B) break;
    std::copy(w.begin(), w.end(), ext.begin());
    for (int i = 31; i < 61; i++) ext[i] = ext[i - 31] + ext[i - 3];
    for (int k = 0; k < 31; k++) {
      uint32_t s = 0;
      for (int j = 0; j < 31; j++) s += Q[j] * ext[k + j];
      w[k] = s;
    }
  }
  return NIP_NO_ERROR;
}

}  // namespace

void generate_release(const nipamd_model* mm) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_cache.find(mm);
  if (it == g_cache.end()) return;
  release(it->second);
  g_cache.erase(it);
}

}  // namespace nipamd

using namespace nipamd;

extern "C" {

int nipamd_generate_order(const nipamd_model* mm, int* order) {
  if (!mm) return -1;
  const std::vector<int> o = sampling_order(mm->m);
  if (order) std::copy(o.begin(), o.end(), order);
  return (int)o.size();
}

int nipamd_rand_windows(long seed, int B, long draws_per_series, uint32_t* win) {
  if (B < 0 || draws_per_series < 0 || (B > 0 && !win))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "rand_windows: bad arguments");
  return rand_windows(seed, B, draws_per_series, win);
}

int nipamd_generate(nipamd_model* mm, long seed, int B, int T, int32_t* d_data, void* stream) {
  if (!mm || B < 0 || T < 0 || (B > 0 && T > 0 && !d_data))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "generate: bad arguments");
  GenCache* g = nullptr;
  if (int rc = prepare(mm, g)) return rc;
  if (B == 0 || T == 0) return NIP_NO_ERROR;
  const int nv = (int)g->order.size();
  // x^(T nv) mod P and the stream's words r[313..373]: the kernel derives
  // every series' window from them (rand_window_kernel)
  const std::vector<uint32_t> r = glibc_state((unsigned)seed, 374);
  const Poly Q = xpow((long)T * nv);
  std::vector<uint32_t> qd(Q.begin(), Q.end());
  qd.insert(qd.end(), r.begin() + 313, r.begin() + 374);
  hipStream_t st = (hipStream_t)stream;
  const size_t need = (size_t)B * 31 + qd.size();
  if (g->win_cap < need) {
    GEN_HIP(hipStreamSynchronize(st));
    (void)hipFree(g->d_win);
    g->d_win = nullptr;
    g->win_cap = 0;
    GEN_HIP(hipMalloc(&g->d_win, need * sizeof(uint32_t)));
    g->win_cap = need;
  }
  uint32_t* d_qd = g->d_win + (size_t)B * 31;
  GEN_HIP(hipMemcpyAsync(d_qd, qd.data(), qd.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  GEN_HIP(hipStreamSynchronize(st));     // 368 bytes; the host vector ends here
  if (rand_window_launch(B, d_qd, g->d_win, st)) return set_error(NIPAMD_ERROR_DEVICE, "generate: window launch failed");
  GenArgs a;
  a.B = B;
  a.T = T;
  a.nv = nv;
  a.x1_step = g->x1_step;
  a.steps = g->d_steps;
  a.tab = g->d_tab;
  a.zero_off = g->zero_off;
  a.cum = g->d_tab + g->cum_off;
  a.cum_n = g->cum_off;
  a.win = g->d_win;
  a.out = d_data;
  if (generate_launch(a, st)) return set_error(NIPAMD_ERROR_DEVICE, "generate: kernel launch failed");
  return NIP_NO_ERROR;
}

int nipamd_generate_host_draws(nipamd_model* mm, int B, int T, const int32_t* draws, int32_t* data) {
  if (!mm || B < 0 || T < 0 || (B > 0 && T > 0 && (!draws || !data)))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "generate: bad arguments");
  GenCache* g = nullptr;
  if (int rc = prepare(mm, g)) return rc;
  const size_t n = (size_t)B * T * g->order.size();
  if (n == 0) return NIP_NO_ERROR;
  int32_t *d_draws = nullptr, *d_out = nullptr;
  int rc = NIP_NO_ERROR;
  hipError_t e = hipMalloc(&d_draws, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&d_out, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpy(d_draws, draws, n * sizeof(int32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    GenArgs a;
    a.B = B;
    a.T = T;
    a.nv = (int)g->order.size();
    a.x1_step = g->x1_step;
    a.steps = g->d_steps;
    a.tab = g->d_tab;
    a.zero_off = g->zero_off;
    a.cum = g->d_tab + g->cum_off;
  a.cum_n = g->cum_off;
    a.draws = d_draws;
    a.out = d_out;
    if (generate_launch(a, nullptr)) rc = set_error(NIPAMD_ERROR_DEVICE, "generate: kernel launch failed");
    else e = hipMemcpy(data, d_out, n * sizeof(int32_t), hipMemcpyDeviceToHost);
  }
  if (rc == NIP_NO_ERROR && e != hipSuccess)
    rc = set_error(NIPAMD_ERROR_DEVICE, std::string("generate: ") + hipGetErrorString(e));
  (void)hipFree(d_draws);
  (void)hipFree(d_out);
  return rc;
}

int nipamd_generate_host(nipamd_model* mm, long seed, int B, int T, int32_t* data) {
  if (!mm || B < 0 || T < 0 || (B > 0 && T > 0 && !data))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "generate: bad arguments");
  const size_t n = (size_t)B * T * mm->m.vars.size();
  int32_t* d = nullptr;
  if (n) GEN_HIP(hipMalloc(&d, n * sizeof(int32_t)));
  int rc = nipamd_generate(mm, seed, B, T, d, nullptr);
  if (rc == NIP_NO_ERROR && n) {
    const hipError_t e = hipMemcpy(data, d, n * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = set_error(NIPAMD_ERROR_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  (void)hipFree(d);
  return rc;
}

}  // extern "C"
