// prefix.cpp -- the e_step's BAD_LUCK verdict on a leading run of missing
// observations, decided on the host once per model version.
//
// The reference's e_step (src/nip.c:1786-1880) fails a series with BAD_LUCK as
// soon as m1 <= 0, m2 <= 0 or the running log-likelihood is > 0 after a step.
// While a series has observed nothing yet, the increment log(m2) - log(m1) is
// 0 in exact arithmetic: both masses come from make_consistent over the same
// evidence (nothing was inserted between the two propagations), and differ
// only by the rounding of the second propagation's new/old sepset ratios.  The
// running sum can therefore round to a positive value (+1e-16) and the series
// is rejected for data that is fine.  The GPU kernels compute the
// log-likelihood in their own order, so they cannot reproduce those last
// bits; but the join tree's state over a leading missing run does not depend
// on the series at all -- only on the model -- so the verdict is a single
// number per model: the first step k at which the reference's test fires on a
// series that has observed nothing up to and including k.  A series whose
// first observation comes after step k is rejected (the flag kernel,
// chain_kernels.hip estep_prefix_flag_kernel); every other series has left the
// rounding regime before ll could turn positive (an observed step contributes
// log of a probability, orders of magnitude above the rounding).
//
// This file restates that prefix exactly, in the reference's operation order:
//   reset_model          nip.c:61-73 (global retraction, nipjointree.c:791-817;
//                        the retraction DFS nipjointree.c:1089-1105)
//   use_priors           nip.c:88-119, nip_enter_prior nipjointree.c:904-943
//   finish / start pass  nip.c:1031-1098 (forward direction)
//   make_consistent      nip.c:1600-1617 with nip_collect_evidence /
//                        nip_distribute_evidence / nip_message_pass
//                        (nipjointree.c:580-709)
//   model_prob_mass      nipjointree.c:1108-1188 (clique sums minus sepset sums
//                        along the DFS)
//   table kernels        nip_general_marginalise, nip_update_potential,
//                        nip_update_evidence, nip_normalise_array
//                        (nippotential.c:267-311, 349-359, 436-522)
// with the flat-index maps precomputed per table pair, the loops running in
// the same element order and every floating-point operation the same one.
//
// The state entering step t + 1 (t >= 0) is a function of the forward message
// alpha_t alone (reset, the priors of the non-interface variables, alpha_t
// multiplied into the in-clique), so once alpha_t repeats an earlier
// alpha_{t-p} bit for bit, the increments repeat with period p and only the
// running sum is carried on: the simulation costs the mixing time of the
// chain (tens of steps), not T.
#include "model.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <vector>

namespace nipamd {
namespace {

// flat index of a table over `sub` (dimension 0 fastest) for every entry of a
// table over `vars` (dimension 0 fastest): nip_mapper + the odometer of
// nippotential.c:58-81
std::vector<int> projection(const Model& m, const std::vector<int>& vars, const std::vector<int>& sub) {
  const int d = (int)vars.size();
  std::vector<int> card(d), stride(d, 0);
  long size = 1;
  for (int k = 0; k < d; k++) { card[k] = m.vars[vars[k]].card; size *= card[k]; }
  int st = 1;
  for (int v : sub) {
    const int k = (int)(std::find(vars.begin(), vars.end(), v) - vars.begin());
    if (k < d) stride[k] = st;
    st *= m.vars[v].card;
  }
  std::vector<int> out((size_t)size);
  std::vector<int> idx(d, 0);
  int j = 0;
  for (long i = 0; i < size; i++) {
    out[(size_t)i] = j;
    for (int k = 0; k < d; k++) {
      j += stride[k];
      if (++idx[k] < card[k]) break;
      j -= stride[k] * card[k];
      idx[k] = 0;
    }
  }
  return out;
}

long table_size(const Model& m, const std::vector<int>& vars) {
  long s = 1;
  for (int v : vars) s *= m.vars[v].card;
  return s;
}

struct Sim {
  const Model& m;
  std::vector<std::vector<double>> P, Snew, Sold;
  std::vector<std::vector<int>> map_a, map_b;    // clique a / b entry -> sepset entry
  std::vector<std::vector<int>> prior_map;       // family-clique entry -> the variable's state
  std::vector<int> in_map, out_map;              // in-clique -> previous_outgoing, out-clique -> outgoing
  std::vector<char> mark;

  explicit Sim(const Model& mm) : m(mm) {
    const int nc = (int)m.cliques.size(), ns = (int)m.sepsets.size();
    P.resize(nc);
    Snew.resize(ns); Sold.resize(ns); map_a.resize(ns); map_b.resize(ns);
    for (int s = 0; s < ns; s++) {
      const Sepset& S = m.sepsets[s];
      Snew[s].assign((size_t)table_size(m, S.vars), 1.0);
      Sold[s] = Snew[s];
      map_a[s] = projection(m, m.cliques[S.a].vars, S.vars);
      map_b[s] = projection(m, m.cliques[S.b].vars, S.vars);
    }
    prior_map.resize(m.vars.size());
    for (int v : m.independent)
      if (m.vars[v].has_prior) prior_map[v] = projection(m, m.cliques[m.vars[v].family].vars, {v});
    if (!m.outgoing.empty()) {
      in_map = projection(m, m.cliques[m.in_clique].vars, m.previous_outgoing);
      out_map = projection(m, m.cliques[m.out_clique].vars, m.outgoing);
    }
    mark.assign(nc, 0);
  }

  const std::vector<int>& side(int s, int c) const { return m.sepsets[s].a == c ? map_a[s] : map_b[s]; }
  void unmark() { std::fill(mark.begin(), mark.end(), 0); }

  // nip_message_pass: swap old / new, marginalise c1 into new, c2 *= new / old
  void message_pass(int c1, int s, int c2) {
    std::swap(Sold[s], Snew[s]);
    std::vector<double>& nw = Snew[s];
    const std::vector<double>& od = Sold[s];
    std::fill(nw.begin(), nw.end(), 0.0);
    const std::vector<int>& m1 = side(s, c1);
    const std::vector<double>& p1 = P[c1];
    for (size_t i = 0; i < p1.size(); i++) nw[m1[i]] += p1[i];
    const std::vector<int>& m2 = side(s, c2);
    std::vector<double>& p2 = P[c2];
    for (size_t i = 0; i < p2.size(); i++) {
      const int j = m2[i];
      p2[i] *= nw[j];
      if (od[j] != 0) p2[i] /= od[j];
      else p2[i] = 0;
    }
  }

  // nip_collect_evidence: both neighbour tests, no else (nipjointree.c:630-673)
  void collect(int c1, int s12, int c2) {
    mark[c2] = 1;
    for (int s : m.cliques[c2].links) {
      if (!mark[m.sepsets[s].a]) collect(c2, s, m.sepsets[s].a);
      if (!mark[m.sepsets[s].b]) collect(c2, s, m.sepsets[s].b);
    }
    if (c1 >= 0) message_pass(c2, s12, c1);
  }

  // nip_distribute_evidence: every pass out of c first, then the recursion
  void distribute(int c) {
    mark[c] = 1;
    const auto& L = m.cliques[c].links;
    for (int s : L) {
      if (!mark[m.sepsets[s].a]) message_pass(c, s, m.sepsets[s].a);
      else if (!mark[m.sepsets[s].b]) message_pass(c, s, m.sepsets[s].b);
    }
    for (int s : L) {
      if (!mark[m.sepsets[s].a]) distribute(m.sepsets[s].a);
      else if (!mark[m.sepsets[s].b]) distribute(m.sepsets[s].b);
    }
  }

  void make_consistent() {
    unmark(); collect(-1, -1, 0);
    unmark(); distribute(0);
  }

  void mass_dfs(int c, double& acc) {
    mark[c] = 1;
    double t = 0;
    for (double x : P[c]) t += x;
    acc += t;
    for (int s : m.cliques[c].links) {
      int nb;
      if (!mark[m.sepsets[s].a]) nb = m.sepsets[s].a;
      else if (!mark[m.sepsets[s].b]) nb = m.sepsets[s].b;
      else continue;
      t = 0;
      for (double x : Snew[s]) t += x;
      acc -= t;
      mass_dfs(nb, acc);
    }
  }
  double mass() { double r = 0; unmark(); mass_dfs(0, r); return r; }

  // the retraction DFS: tables back to the originals, sepsets to 1 (the
  // likelihoods are all 1 after reset_model, so re-entering them is exact)
  void retract_dfs(int c) {
    mark[c] = 1;
    P[c] = m.cliques[c].original;
    for (int s : m.cliques[c].links) {
      int nb;
      if (!mark[m.sepsets[s].a]) nb = m.sepsets[s].a;
      else if (!mark[m.sepsets[s].b]) nb = m.sepsets[s].b;
      else continue;
      std::fill(Sold[s].begin(), Sold[s].end(), 1.0);
      std::fill(Snew[s].begin(), Snew[s].end(), 1.0);
      retract_dfs(nb);
    }
  }
  void reset() { unmark(); retract_dfs(0); }

  void use_priors(bool has_history) {
    for (int v : m.independent) {
      const Var& V = m.vars[v];
      if (has_history && (V.ifs & IF_OLD_OUTGOING)) continue;
      if (!V.has_prior) continue;
      bool any = false;
      for (double x : V.prior) any |= x > 0;
      if (!any) continue;                              // nip_enter_prior refuses a zero vector
      std::vector<double>& p = P[V.family];
      const std::vector<int>& mp = prior_map[v];
      for (size_t i = 0; i < p.size(); i++) p[i] *= V.prior[mp[i]];
    }
  }

  void finish(const std::vector<double>& alpha) {
    if (m.outgoing.empty()) return;
    std::vector<double>& p = P[m.in_clique];
    for (size_t i = 0; i < p.size(); i++) p[i] *= alpha[in_map[i]];
  }

  void start(std::vector<double>& alpha) {
    alpha.assign((size_t)table_size(m, m.outgoing), 0.0);
    if (m.outgoing.empty()) { alpha.assign(1, 1.0); return; }
    const std::vector<double>& p = P[m.out_clique];
    for (size_t i = 0; i < p.size(); i++) alpha[out_map[i]] += p[i];
    double sum = 0;
    for (double x : alpha) sum += x;
    if (sum == 0) return;
    for (double& x : alpha) x /= sum;
  }
};

constexpr int kMaxPeriod = 32;
// Work bound: table entries x propagated steps.  A chain whose forward message
// has not repeated (bit for bit, period <= kMaxPeriod) within this budget is
// not simulated further (-2: its leading missing runs are accepted), so the
// host work per model version stays within about a second whatever T, the
// chain's mixing time or its period.
constexpr long kPrefixWork = 1L << 29;

}  // namespace

// First step k < T at which the reference's e_step would reject a series that
// has observed nothing at steps 0..k; -1 if there is none; -2 if the work
// bound ran out first.  `steps` (if not null) receives the number of steps
// actually propagated.
int estep_prefix_first_bad(const Model& m, int T, int* steps) {
  const long entries = std::max(1L, estep_prefix_entries(m));
  const long budget = std::max(16L, kPrefixWork / entries);
  Sim S(m);
  S.reset();
  S.use_priors(false);
  double ll = 0.0;
  std::vector<double> alpha;
  std::deque<std::vector<double>> hist;   // alpha_{t-1}, alpha_{t-2}, ...
  std::vector<double> inc;                // the increment of every step so far
  int t = 0;
  for (; t < T; t++) {
    if (t >= budget) { if (steps) *steps = t; return -2; }
    if (t > 0) S.finish(alpha);
    S.make_consistent();
    const double m1 = S.mass();
    S.make_consistent();
    const double m2 = S.mass();
    double d = 0.0;
    if (m1 > 0 && m2 > 0) {
      d = std::log(m2) - std::log(m1);
      ll = ll + d;
    }
    inc.push_back(d);
    if (m1 <= 0 || m2 <= 0 || ll > 0) { if (steps) *steps = t + 1; return t; }
    S.start(alpha);
    S.reset();
    S.use_priors(T > 1);
    int p = 0;
    for (int q = 0; q < (int)hist.size() && !p; q++)
      if (hist[q] == alpha) p = q + 1;
    if (p) {
      // step t + 1 + j repeats step t + 1 - p + (j mod p)
      if (steps) *steps = t + 1;
      const int base = t + 1 - p;
      for (int u = t + 1; u < T; u++) {
        ll = ll + inc[base + (u - base) % p];
        if (ll > 0) return u;
      }
      return -1;
    }
    hist.push_front(alpha);
    if ((int)hist.size() > kMaxPeriod) hist.pop_back();
  }
  if (steps) *steps = t;
  return -1;
}

}  // namespace nipamd

namespace nipamd {
// table entries one propagation touches (the engine's size cap, engine.cpp)
long estep_prefix_entries(const Model& m) {
  long n = 0;
  for (const Clique& c : m.cliques) n += table_size(m, c.vars);
  for (const Sepset& s : m.sepsets) n += table_size(m, s.vars);
  return n;
}
}  // namespace nipamd
