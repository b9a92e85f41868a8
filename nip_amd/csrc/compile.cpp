// compile.cpp -- Bayes-net spec -> DBN time-slice join tree, host side.
//
// Re-derives, bit for bit, the structures the reference builds at parse time:
//   * variable IDs = declaration order        (src/nipvariable.c:56-128)
//   * parsed CPT reorder + normalisation      (src/nipjointree.c:341-480,
//                                              src/huginnet.y:582-780)
//   * interface flags                         (src/huginnet.y:1155-1254)
//   * moralise / interface edges / triangulate / cliques / sepsets
//                                             (src/nipgraph.c:300-612, 616-822,
//                                              src/nipheap.c:42-298)
//   * family cliques and mappings             (src/nipjointree.c:967-1064)
//   * clique initialisation with the CPTs     (src/nipjointree.c:713-772)
//   * model assembly, in/out cliques          (src/nip.c:147-264)
// The heap, the cluster/sepset cost keys (including the sepset secondary key
// that is always 0 because of `if(!s)`, nipgraph.c:656) and every tie-break are
// reproduced, since the clique array order depends on them.
#include "model.h"

#include "nip_amd.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <sstream>

namespace nipamd {
namespace {

// ------------------------------------------------------------------
// Binary min-heap with the reference's (non-standard) update semantics.
// ------------------------------------------------------------------
struct HeapItem {
  std::vector<int> content;   // cluster: [v, neighbours...]; sepset: {index}
  int primary = 0, secondary = 0;
};

class RefHeap {
 public:
  using KeyFn = std::function<void(HeapItem&)>;
  explicit RefHeap(KeyFn keys) : keys_(std::move(keys)) {}

  void insert(std::vector<int> content) {
    auto it = std::make_unique<HeapItem>();
    it->content = std::move(content);
    keys_(*it);
    items_.push_back(std::move(it));
    heapified_ = false;
  }
  // nip_build_min_heap (nipheap.c:167-190): full heapify unless already
  // heapified, in which case only the updated indices are sifted DOWN.
  void build() {
    if (!heapified_) {
      for (int i = parent(size() - 1); i >= 0; i--) heapify(i);
    } else {
      for (int idx : updated_) heapify(idx);
    }
    updated_.clear();
    heapified_ = true;
  }
  // nip_heap_extract_min (nipheap.c:193-220)
  bool extract(std::vector<int>& out) {
    if (size() < 1) return false;
    std::unique_ptr<HeapItem> mn = std::move(items_[0]);
    items_[0] = std::move(items_[size() - 1]);
    items_.pop_back();
    if (size() > 0) heapify(0);
    out = std::move(mn->content);
    return true;
  }
  int search_first(int v) const {  // nip_search_heap_item with nip_family_cluster
    for (int n = 0; n < size(); n++)
      if (!items_[n]->content.empty() && items_[n]->content[0] == v) return n;
    return -1;
  }
  const std::vector<int>& get(int i) const { return items_[i]->content; }
  void set(int i, std::vector<int> c) {  // nip_set_heap_item (nipheap.c:152-164)
    items_[i]->content = std::move(c);
    keys_(*items_[i]);
    updated_.push_back(i);
  }
  int size() const { return (int)items_.size(); }

 private:
  static int parent(int i) { return (i - 1) / 2; }
  static bool less(const HeapItem* a, const HeapItem* b) {  // nipheap.c:247-258
    if (a) {
      if (b) return a->primary < b->primary ||
                    (a->primary == b->primary && a->secondary < b->secondary);
      return true;
    }
    return false;
  }
  void heapify(int i) {  // nip_min_heapify (nipheap.c:261-285)
    for (;;) {
      int l = 2 * i + 1, r = 2 * (i + 1), mn = i;
      if (l < size() && less(items_[l].get(), items_[i].get())) mn = l;
      if (r < size() && less(items_[r].get(), items_[mn].get())) mn = r;
      if (mn == i) break;
      std::swap(items_[mn], items_[i]);
      i = mn;
    }
  }
  KeyFn keys_;
  std::vector<std::unique_ptr<HeapItem>> items_;
  std::vector<int> updated_;
  bool heapified_ = false;
};

bool is_parent(const std::vector<std::vector<int>>& parents, int p, int c) {
  for (int q : parents[c]) if (q == p) return true;
  return false;
}

// nip_variable_union(a, b) (nipvariable.c:446-502): a, then b's missing ones.
std::vector<int> var_union(const std::vector<int>& a, const std::vector<int>& b) {
  std::vector<int> c = a;
  for (int x : b) if (std::find(c.begin(), c.end(), x) == c.end()) c.push_back(x);
  return c;
}

// nip_variable_isect(a, b) (nipvariable.c:506-557): a's order.
std::vector<int> var_isect(const std::vector<int>& a, const std::vector<int>& b) {
  std::vector<int> c;
  for (int x : a) if (std::find(b.begin(), b.end(), x) != b.end()) c.push_back(x);
  return c;
}

struct Graph {
  int n;
  std::vector<int> adj;  // adj[i*n+j]
  int& at(int i, int j) { return adj[(size_t)i * n + j]; }
};

// Triangulation + clique array (nipgraph.c:443-515, 389-440).  Returns the
// clique variable lists (ascending index) in clique-array order.
int triangulate(Graph& gu, const std::vector<int>& card,
                const std::vector<std::vector<int>>& parents,
                std::vector<std::vector<int>>& cliques, std::string& err) {
  const int n = gu.n;
  RefHeap h([&](HeapItem& it) {
    const auto& vs = it.content;
    int sum = 0;                         // nip_cluster_primary_cost (nipgraph.c:616-636)
    for (size_t i = 0; i < vs.size(); i++)
      for (size_t j = i + 1; j < vs.size(); j++) sum += !is_parent(parents, vs[i], vs[j]);
    uint32_t prod = 1;                   // nip_cluster_secondary_cost (:638-644), int wrap
    for (int v : vs) prod *= (uint32_t)card[v];
    it.primary = sum;
    it.secondary = (int)prod;
  });
  for (int i = 0; i < n; i++) {          // nip_build_cluster_heap (:670-713)
    std::vector<int> cl{i};
    for (int j = 0; j < n; j++) if (gu.at(i, j)) cl.push_back(j);
    h.insert(std::move(cl));
  }
  h.build();

  std::vector<std::vector<char>> sets;   // prepend-ordered list (front = newest)
  for (int i = 0; i < n; i++) {
    std::vector<int> cl;
    if (!h.extract(cl)) { err = "cluster heap exhausted"; return -1; }
    std::vector<char> vset(n, 0);
    for (size_t j = 0; j < cl.size(); j++) {
      vset[cl[j]] = 1;
      for (size_t k = j + 1; k < cl.size(); k++) { gu.at(cl[j], cl[k]) = 1; gu.at(cl[k], cl[j]) = 1; }
    }
    // nip_update_cluster_heap (:725-778)
    const int removed = cl[0];
    for (size_t k = 1; k < cl.size(); k++) {
      int idx = h.search_first(cl[k]);
      if (idx < 0) { err = "neighbour cluster missing from heap (reference would assert)"; return -1; }
      std::vector<int> u = var_union(h.get(idx), cl), nc;
      for (int x : u) if (x != removed) nc.push_back(x);
      h.set(idx, std::move(nc));
    }
    h.build();
    // nip_int_array_list_contains_subset (niplists.c:598-619)
    bool subset = false;
    for (const auto& s : sets) {
      bool ok = true;
      for (int v = 0; v < n; v++) if (vset[v] && !s[v]) { ok = false; break; }
      if (ok) { subset = true; break; }
    }
    if (!subset) sets.insert(sets.begin(), std::move(vset));
  }
  // nip_cluster_list_to_clique_array: list head fills the LAST slot.
  const int nc = (int)sets.size();
  cliques.assign(nc, {});
  int counter = nc;
  for (const auto& s : sets) {
    std::vector<int> cv;
    for (int v = 0; v < n; v++) if (s[v]) cv.push_back(v);
    cliques[--counter] = cv;             // ids ascend with index: already sorted
  }
  return nc;
}

// nip_cliques_connected (nipjointree.c:546-577)
bool connected(const std::vector<Clique>& cq, const std::vector<Sepset>& ss,
               std::vector<char>& mark, int one, int two) {
  mark[one] = 1;
  if (one == two) return true;
  for (int s : cq[one].links) {
    if (!mark[ss[s].a]) { if (connected(cq, ss, mark, ss[s].a, two)) return true; }
    else if (!mark[ss[s].b]) { if (connected(cq, ss, mark, ss[s].b, two)) return true; }
  }
  return false;
}

// nip_create_sepsets (nipgraph.c:547-612) with the sepset heap (:781-822).
void create_sepsets(std::vector<Clique>& cq, std::vector<Sepset>& ss) {
  const int nc = (int)cq.size();
  std::vector<Sepset> cand;
  for (int i = 0; i < nc - 1; i++)
    for (int j = i + 1; j < nc; j++) {
      Sepset s; s.a = i; s.b = j; s.vars = var_isect(cq[i].vars, cq[j].vars);
      cand.push_back(std::move(s));
    }
  RefHeap h([&](HeapItem& it) {
    it.primary = -(int)cand[it.content[0]].vars.size();  // nip_sepset_primary_cost
    it.secondary = 0;                                    // :652-667, always 0
  });
  for (size_t k = 0; k < cand.size(); k++) h.insert({(int)k});
  h.build();
  std::vector<Sepset> confirmed;
  int inserted = 0;
  while (inserted < nc - 1) {
    std::vector<int> item;
    if (!h.extract(item)) break;
    const Sepset& s = cand[item[0]];
    std::vector<char> mark(nc, 0);
    if (!connected(cq, confirmed, mark, s.a, s.b)) {
      int id = (int)confirmed.size();
      confirmed.push_back(s);
      // nip_confirm_sepset (nipjointree.c:211-234): prepend to both lists
      cq[s.a].links.insert(cq[s.a].links.begin(), id);
      cq[s.b].links.insert(cq[s.b].links.begin(), id);
      inserted++;
    }
  }
  ss = std::move(confirmed);
}

// nip_find_clique (nipjointree.c:1043-1064)
int find_clique(const std::vector<Clique>& cq, const std::vector<int>& vs) {
  for (size_t i = 0; i < cq.size(); i++) {
    size_t ok = 0;
    for (int v : vs)
      if (std::find(cq[i].vars.begin(), cq[i].vars.end(), v) != cq[i].vars.end()) ok++;
    if (ok == vs.size()) return (int)i;
  }
  return -1;
}

void normalise_array(double* r, int n) {  // nippotential.c:349-359
  double sum = 0;
  for (int i = 0; i < n; i++) sum += r[i];
  if (sum == 0) return;
  for (int i = 0; i < n; i++) r[i] /= sum;
}

// Multiply probs (dims = `pvars`, ascending IDs) into a clique table through
// the positions of pvars in the clique (nip_init_potential, nippotential.c:525-564).
void init_into(const std::vector<int>& cvars, const std::vector<int>& card,
               std::vector<double>& tgt, const std::vector<int>& pvars,
               const std::vector<double>& probs, const std::vector<int>& map) {
  const int cd = (int)cvars.size();
  std::vector<int> idx(cd, 0);
  for (size_t i = 0; i < tgt.size(); i++) {
    int j = 0, stride = 1;
    for (size_t k = 0; k < pvars.size(); k++) { j += idx[map[k]] * stride; stride *= card[pvars[k]]; }
    tgt[i] *= probs[j];
    for (int k = 0; k < cd; k++) { if (++idx[k] < card[cvars[k]]) break; idx[k] = 0; }
  }
}

}  // namespace

int compile_graph_only(int n, const std::vector<int>& card,
                       const std::vector<std::pair<int, int>>& edges, bool set_parents,
                       std::vector<std::vector<int>>& cliques_out, std::string& err) {
  Graph g{n, std::vector<int>((size_t)n * n, 0)};
  std::vector<std::vector<int>> parents(n);
  for (auto& e : edges) {
    g.at(e.first, e.second) = 1;
    if (set_parents) parents[e.second].push_back(e.first);
  }
  Graph gm = g;  // nip_moralise_graph (nipgraph.c:325-351)
  for (int v = 0; v < n; v++)
    for (int i = 0; i < n; i++)
      if (g.at(i, v))
        for (int j = i + 1; j < n; j++) { gm.at(i, j) |= g.at(j, v); gm.at(j, i) |= g.at(j, v); }
  Graph gu = gm;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) gu.at(i, j) = gm.at(i, j) || gm.at(j, i);
  return triangulate(gu, card, parents, cliques_out, err);
}

int compile_model(const NetSpec& spec, Model& m, std::string& err) {
  const int n = (int)spec.card.size();
  m = Model();
  m.vars.resize(n);
  for (int i = 0; i < n; i++) {
    m.vars[i].symbol = i < (int)spec.symbols.size() ? spec.symbols[i] : ("V" + std::to_string(i));
    m.vars[i].card = spec.card[i];
    if (spec.card[i] <= 0) { err = "non-positive cardinality"; return NIP_ERROR_INVALID_ARGUMENT; }
    if (i < (int)spec.labels.size()) m.vars[i].label = spec.labels[i];
    if (i < (int)spec.positions.size()) {
      m.vars[i].pos_x = spec.positions[i].first;
      m.vars[i].pos_y = spec.positions[i].second;
    }
    if (i < (int)spec.states.size() && (int)spec.states[i].size() == spec.card[i]) {
      m.vars[i].states = spec.states[i];
    } else {
      for (int s = 0; s < spec.card[i]; s++) m.vars[i].states.push_back(std::to_string(s));
    }
  }
  m.node_size_x = spec.node_size_x;
  m.node_size_y = spec.node_size_y;
  auto& V = m.vars;

  // --- potentialDeclaration actions (huginnet.y:582-780) ---
  struct Parsed { int child; std::vector<int> parents; std::vector<int> ids; std::vector<double> data; };
  std::vector<Parsed> parsed;
  for (const auto& p : spec.pots) {
    Parsed q;
    q.child = p.child;
    q.parents.assign(p.parents.rbegin(), p.parents.rend());  // prepend (:753-766)
    std::vector<int> fam{p.child};
    fam.insert(fam.end(), q.parents.begin(), q.parents.end());
    // nip_create_potential (nipjointree.c:341-480): reorder to ascending ID
    std::vector<int> sorted = fam;
    std::sort(sorted.begin(), sorted.end());
    size_t size = 1;
    for (int v : fam) size *= (size_t)V[v].card;
    q.ids = sorted;
    q.data.assign(size, 1.0);
    if (p.has_data) {
      if (p.data.size() < size) { err = "not enough elements in potential"; return NIP_ERROR_INVALID_ARGUMENT; }
      const int d = (int)fam.size();
      std::vector<int> rank(d);
      for (int j = 0; j < d; j++) rank[j] = (int)(std::find(sorted.begin(), sorted.end(), fam[j]) - sorted.begin());
      std::vector<int> idx(d, 0);  // multi-index over sorted dims
      for (size_t i = 0; i < size; i++) {
        size_t src = 0, stride = 1;
        for (int j = 0; j < d; j++) { src += (size_t)idx[rank[j]] * stride; stride *= (size_t)V[fam[j]].card; }
        q.data[i] = p.data[src];
        for (int k = 0; k < d; k++) { if (++idx[k] < V[sorted[k]].card) break; idx[k] = 0; }
      }
    }
    if (!q.parents.empty()) {
      // nip_normalise_cpd over dimension 0 = lowest ID of the family (:635-636)
      const int c0 = V[sorted[0]].card;
      for (size_t i = 0; i < size; i += c0) normalise_array(q.data.data() + i, c0);
    } else if (p.has_data) {
      normalise_array(q.data.data(), (int)size);           // :665-666
    }
    parsed.push_back(std::move(q));
  }

  // --- parsed_vars_to_graph (huginnet.y:1058-1103) ---
  Graph g{n, std::vector<int>((size_t)n * n, 0)};
  std::vector<std::vector<int>> parents(n);
  for (const auto& q : parsed) {
    for (int p : q.parents) g.at(p, q.child) = 1;
    V[q.child].parents = q.parents;                        // nip_set_parents
    parents[q.child] = q.parents;
  }

  // --- interface_to_vars (huginnet.y:1155-1254) ---
  for (int i = 0; i < n; i++) {
    int nx = spec.next[i];
    if (nx >= 0) {
      if (V[nx].card != V[i].card) { err = "invalid NIP_next: cardinalities differ"; return NIP_ERROR_GENERAL; }
      V[i].next = nx; V[nx].previous = i;
    }
  }
  for (int k = 0; k < n; k++) {
    bool mm = false;
    for (int p : V[k].parents)
      if (V[p].next >= 0) {
        V[p].ifs |= IF_OLD_OUTGOING; V[V[p].next].ifs |= IF_OUTGOING; V[k].ifs |= IF_INCOMING; mm = true;
      }
    if (mm)
      for (int p : V[k].parents) if (V[p].next < 0) V[p].ifs |= IF_INCOMING;
  }

  // --- nip_graph_to_cliques (nipgraph.c:518-544) ---
  Graph gm = g;
  for (int v = 0; v < n; v++)
    for (int i = 0; i < n; i++)
      if (g.at(i, v))
        for (int j = i + 1; j < n; j++) { gm.at(i, j) |= g.at(j, v); gm.at(j, i) |= g.at(j, v); }
  Graph gi = gm;  // nip_add_interface_edges (:354-386)
  for (int i = 0; i < n; i++)
    for (int j = i + 1; j < n; j++)
      if (((V[i].ifs & IF_OLD_OUTGOING) && (V[j].ifs & IF_OLD_OUTGOING)) ||
          ((V[i].ifs & IF_OUTGOING) && (V[j].ifs & IF_OUTGOING))) { gi.at(i, j) = 1; gi.at(j, i) = 1; }
  Graph gu = gi;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) gu.at(i, j) = gi.at(i, j) || gi.at(j, i);
  std::vector<std::vector<int>> cl;
  std::vector<int> card(n);
  for (int i = 0; i < n; i++) card[i] = V[i].card;
  if (triangulate(gu, card, parents, cl, err) < 0) return NIP_ERROR_GENERAL;
  m.cliques.resize(cl.size());
  for (size_t c = 0; c < cl.size(); c++) {
    m.cliques[c].vars = cl[c];
    size_t sz = 1;
    for (int v : cl[c]) sz *= (size_t)V[v].card;
    m.cliques[c].original.assign(sz, 1.0);
  }
  std::vector<Sepset> ss;
  create_sepsets(m.cliques, ss);

  // sepset numbering: first appearance walking cliques in order, then each
  // clique's link list in order (the order the index contract is dumped in)
  {
    std::vector<int> remap(ss.size(), -1);
    int next_id = 0;
    for (auto& c : m.cliques)
      for (int s : c.links) if (remap[s] < 0) remap[s] = next_id++;
    m.sepsets.resize(ss.size());
    for (size_t s = 0; s < ss.size(); s++) m.sepsets[remap[s]] = ss[s];
    for (auto& c : m.cliques) for (int& s : c.links) s = remap[s];
  }

  // --- families (nipjointree.c:967-1040) ---
  for (int v = 0; v < n; v++) {
    std::vector<int> fam = V[v].parents;
    fam.push_back(v);
    V[v].family = find_clique(m.cliques, fam);
    if (V[v].family < 0) { err = "no family clique for " + V[v].symbol; return NIP_ERROR_GENERAL; }
    const auto& cv = m.cliques[V[v].family].vars;
    V[v].family_mapping.assign(V[v].parents.size() + 1, 0);
    for (size_t i = 0; i < cv.size(); i++) if (cv[i] == v) { V[v].family_mapping[0] = (int)i; break; }
    size_t found = 0;
    for (size_t i = 0; i < cv.size() && found < V[v].parents.size(); i++)
      for (size_t j = 0; j < V[v].parents.size(); j++)
        if (cv[i] == V[v].parents[j]) { V[v].family_mapping[j + 1] = (int)i; found++; break; }
    V[v].family_pos = V[v].family_mapping[0];
  }

  // --- parsed_potentials_to_jtree (huginnet.y:1110-1152) ---
  for (const auto& q : parsed) {
    const int fc = V[q.child].family;
    if (q.ids.size() > 1) {
      // nip_init_clique (nipjointree.c:713-772): positions of the potential's
      // (ascending-ID) variables in the clique, in clique order
      const auto& cv = m.cliques[fc].vars;
      std::vector<int> map;
      if (q.ids.size() < cv.size()) {
        for (size_t i = 0; i < cv.size() && map.size() < q.ids.size(); i++) {
          int var = cv[i];
          for (int p : q.parents) if (var == p) map.push_back((int)i);
          if (var == q.child) map.push_back((int)i);
        }
      } else {
        for (size_t i = 0; i < cv.size(); i++) map.push_back((int)i);
      }
      init_into(cv, card, m.cliques[fc].original, q.ids, q.data, map);
    } else {
      V[q.child].has_prior = true;                         // nip_set_prior
      V[q.child].prior = q.data;
    }
  }

  // --- model assembly (nip.c:147-264) ---
  for (int v = 0; v < n; v++)
    if (V[v].parents.empty() && !V[v].has_prior) { V[v].has_prior = true; V[v].prior.assign(V[v].card, 0.0); }
  for (int v = 0; v < n; v++) {
    if (V[v].ifs & IF_OLD_OUTGOING) { m.previous_outgoing.push_back(v); m.outgoing.push_back(V[v].next); }
    if (!V[v].parents.empty()) m.children.push_back(v); else m.independent.push_back(v);
  }
  if (!m.outgoing.empty()) {
    m.in_clique = find_clique(m.cliques, m.previous_outgoing);
    m.out_clique = find_clique(m.cliques, m.outgoing);
  }
  build_chain_plan(m);
  return 0;
}

int param_size(const Model& m) {
  int tot = 0;
  for (const auto& v : m.vars) {
    int s = v.card;
    for (int p : v.parents) s *= m.vars[p].card;
    tot += s;
  }
  return tot;
}

// m_step (src/nip.c:2010-2071) on the host tables.
int m_step(Model& m, const double* params) {
  std::vector<int> card(m.vars.size());
  for (size_t i = 0; i < m.vars.size(); i++) card[i] = m.vars[i].card;
  std::vector<std::vector<double>> P;
  size_t off = 0;
  for (const auto& v : m.vars) {
    size_t s = v.card;
    for (int p : v.parents) s *= m.vars[p].card;
    std::vector<double> t(params + off, params + off + s);
    for (size_t i = 0; i < s; i += v.card) normalise_array(t.data() + i, v.card);  // normalise_cpd
    P.push_back(std::move(t));
    off += s;
  }
  for (auto& c : m.cliques) std::fill(c.original.begin(), c.original.end(), 1.0);  // total_reset
  for (size_t i = 0; i < m.vars.size(); i++) {
    auto& v = m.vars[i];
    if (!v.parents.empty()) {
      // nip_init_potential(params, family->original_p, family_mapping): the
      // parameter dims are (child, parents...) in v->parents order
      std::vector<int> pvars{(int)i};
      pvars.insert(pvars.end(), v.parents.begin(), v.parents.end());
      init_into(m.cliques[v.family].vars, card, m.cliques[v.family].original, pvars, P[i], v.family_mapping);
    } else {
      v.prior = P[i];  // nip_total_marginalise(params, prior, 0) of a 1-D table
    }
  }
  build_chain_plan(m);
  return 0;
}

// ------------------------------------------------------------------
// Index-contract dump (same schema as oracle/ref/nipref_harness.c nh_desc)
// ------------------------------------------------------------------
namespace {
void put_ints(std::ostringstream& o, const std::vector<int>& v) {
  o << "[";
  for (size_t i = 0; i < v.size(); i++) o << (i ? "," : "") << v[i];
  o << "]";
}
void put_doubles(std::ostringstream& o, const std::vector<double>& v) {
  char b[40];
  o << "[";
  for (size_t i = 0; i < v.size(); i++) { std::snprintf(b, sizeof b, "%.17g", v[i]); o << (i ? "," : "") << b; }
  o << "]";
}
}  // namespace

std::string model_desc_json(const Model& m) {
  std::ostringstream o;
  o << "{\"vars\":[";
  for (size_t i = 0; i < m.vars.size(); i++) {
    const auto& v = m.vars[i];
    o << (i ? "," : "") << "{\"symbol\":\"" << v.symbol << "\",\"card\":" << v.card
      << ",\"if\":" << v.ifs << ",\"next\":" << v.next << ",\"previous\":" << v.previous
      << ",\"parents\":";
    put_ints(o, v.parents);
    o << ",\"prior\":";
    if (v.parents.empty() && v.has_prior) put_doubles(o, v.prior); else o << "null";
    o << ",\"family\":" << v.family << ",\"family_mapping\":";
    put_ints(o, v.family_mapping);
    o << "}";
  }
  o << "],\"cliques\":[";
  for (size_t c = 0; c < m.cliques.size(); c++) {
    o << (c ? "," : "") << "{\"vars\":";
    put_ints(o, m.cliques[c].vars);
    o << ",\"links\":";
    put_ints(o, m.cliques[c].links);
    o << ",\"original\":";
    put_doubles(o, m.cliques[c].original);
    o << "}";
  }
  o << "],\"sepsets\":[";
  for (size_t s = 0; s < m.sepsets.size(); s++) {
    o << (s ? "," : "") << "{\"a\":" << m.sepsets[s].a << ",\"b\":" << m.sepsets[s].b << ",\"vars\":";
    put_ints(o, m.sepsets[s].vars);
    o << "}";
  }
  o << "],\"in_clique\":" << m.in_clique << ",\"out_clique\":" << m.out_clique << ",\"outgoing\":";
  put_ints(o, m.outgoing);
  o << ",\"previous_outgoing\":";
  put_ints(o, m.previous_outgoing);
  o << ",\"independent\":";
  put_ints(o, m.independent);
  o << ",\"children\":";
  put_ints(o, m.children);
  o << "}";
  return o.str();
}

// ------------------------------------------------------------------
// Interface-chain execution plan (model.h).
// ------------------------------------------------------------------
namespace {
// flat index of an assignment in a clique table (dimension 0 fastest)
long clique_index(const Model& m, int c, const std::vector<int>& val_of_var) {
  long idx = 0, stride = 1;
  for (int v : m.cliques[c].vars) { idx += val_of_var[v] * stride; stride *= m.vars[v].card; }
  return idx;
}

void build_single_chain_plan(Model& m);
void build_joint_chain_plan(Model& m);
}  // namespace

void build_chain_plan(Model& m) {
  build_single_chain_plan(m);
  if (!m.chain.valid) build_joint_chain_plan(m);
}

namespace {
void build_single_chain_plan(Model& m) {
  ChainPlan& P = m.chain;
  P = ChainPlan();
  if (m.outgoing.size() != 1 || m.previous_outgoing.size() != 1) return;
  const int vp = m.previous_outgoing[0], vc = m.outgoing[0];
  const auto& V = m.vars;
  const int N = V[vc].card;
  if (N < 1 || N > 64 || V[vp].card != N) return;
  if (!V[vp].parents.empty() || !V[vp].has_prior) return;
  // the in-clique: the one clique holding prev; it must hold cur too
  int cin = -1;
  for (size_t c = 0; c < m.cliques.size(); c++) {
    const auto& cv = m.cliques[c].vars;
    if (std::find(cv.begin(), cv.end(), vp) != cv.end()) {
      if (cin >= 0) return;
      cin = (int)c;
    }
  }
  if (cin < 0) return;
  const auto& inv = m.cliques[cin].vars;
  if (std::find(inv.begin(), inv.end(), vc) == inv.end()) return;
  if (V[vc].family != cin) return;
  // cur's parents: prev plus hidden independent variables living only in the in-clique
  std::vector<int> hidden;
  for (int v : inv) {
    if (v == vp || v == vc) continue;
    // (an independent parent of cur is flagged INCOMING; its prior is entered every slice)
    if (!V[v].parents.empty() || !V[v].has_prior || (V[v].ifs & (IF_OUTGOING | IF_OLD_OUTGOING))) return;
    if (std::find(V[vc].parents.begin(), V[vc].parents.end(), v) == V[vc].parents.end()) return;
    hidden.push_back(v);
  }
  if (V[vc].parents.size() != hidden.size() + 1 ||
      std::find(V[vc].parents.begin(), V[vc].parents.end(), vp) == V[vc].parents.end()) return;
  long hsize = 1;
  for (int h : hidden) { hsize *= V[h].card; if (hsize > (1L << 24)) return; }
  // every other clique: {cur, o}, o a leaf child of cur in no other clique
  std::vector<int> seen(V.size(), 0);
  for (int v : inv) seen[v] = 1;
  std::vector<ChainEmit> emits;
  for (size_t c = 0; c < m.cliques.size(); c++) {
    if ((int)c == cin) continue;
    const auto& cv = m.cliques[c].vars;
    if (cv.size() != 2 || std::find(cv.begin(), cv.end(), vc) == cv.end()) return;
    const int o = cv[0] == vc ? cv[1] : cv[0];
    if (seen[o] || V[o].parents != std::vector<int>{vc} || V[o].family != (int)c ||
        (V[o].ifs & (IF_OUTGOING | IF_OLD_OUTGOING))) return;
    seen[o] = 1;
    ChainEmit E;
    E.var = o; E.clique = (int)c; E.M = V[o].card;
    if (E.M < 1 || E.M > 253) return;
    E.E.assign((size_t)E.M * 64, 0.0);
    E.s.assign(64, 0.0);
    std::vector<int> val(V.size(), 0);
    for (int y = 0; y < N; y++)
      for (int mm = 0; mm < E.M; mm++) {
        val[vc] = y; val[o] = mm;
        const double e = m.cliques[c].original[clique_index(m, (int)c, val)];
        E.E[(size_t)mm * 64 + y] = e;
        E.s[y] += e;
      }
    emits.push_back(std::move(E));
  }
  for (size_t v = 0; v < V.size(); v++) if (!seen[v]) return;   // every variable accounted for
  // transition with the hidden parents summed out under their priors (large
  // in-cliques: on the GPU, fold.hip, when the engine first needs it)
  P.A64.assign(64 * 64, 0.0);
  std::vector<int> val(V.size(), 0);
  std::vector<int> hv(hidden.size(), 0);
  P.fold_gpu = !hidden.empty() && hsize * N * N >= kGpuFoldMin;
  for (long hi = 0; hi < (P.fold_gpu ? 0 : hsize); hi++) {
    long r = hi;
    double w = 1.0;
    for (size_t k = 0; k < hidden.size(); k++) {
      const int c = V[hidden[k]].card;
      hv[k] = (int)(r % c); r /= c;
      val[hidden[k]] = hv[k];
      w *= V[hidden[k]].prior[hv[k]];
    }
    for (int x = 0; x < N; x++)
      for (int y = 0; y < N; y++) {
        val[vp] = x; val[vc] = y;
        P.A64[x * 64 + y] += m.cliques[cin].original[clique_index(m, cin, val)] * w;
      }
  }
  P.N = N; P.v_prev = vp; P.v_cur = vc; P.c_trans = cin;
  P.hidden = hidden;
  P.emits = std::move(emits);
  P.pi64.assign(64, 0.0);
  for (int x = 0; x < N; x++) P.pi64[x] = V[vp].prior[x];
  P.s_all64.assign(64, 0.0);
  for (int y = 0; y < N; y++) {
    double s = 1.0;
    for (const auto& E : P.emits) s *= E.s[y];
    P.s_all64[y] = s;
  }
  if (N <= 16) {
    P.A.assign(256, 0.0);
    P.pi.assign(16, 0.0);
    for (int x = 0; x < N; x++) {
      P.pi[x] = P.pi64[x];
      for (int y = 0; y < N; y++) P.A[x * 16 + y] = P.A64[x * 64 + y];
    }
  }
  P.self.var = vc;
  P.self.M = N;
  P.self.E.assign((size_t)N * 64, 0.0);
  P.self.s.assign(64, 0.0);
  for (int y = 0; y < N; y++) { P.self.E[(size_t)y * 64 + y] = 1.0; P.self.s[y] = 1.0; }
  P.hmm = hidden.empty() && P.emits.size() == 1 && V.size() == 3 && N <= 16;
  P.valid = true;
}

// Several interface variables (a factorial HMM, coupled chains): the slice is
// still an interface chain over the JOINT interface state when its
// distribution over (previous interface x, interface y, observation
// candidates o_k) factorises as A[x][y] prod_k E_k[y][o_k].  x and y index the
// joint states as the general engine's interface messages do (dimension 0
// fastest over previous_outgoing / outgoing, paired by position), the other
// variables of the slice are summed out, and the factorisation is checked
// numerically on the slice's joint -- the product of the clique tables the
// reference propagates (orig_p, nip_global_retraction, src/nipjointree.c:791-817)
// and the priors use_priors enters every slice (src/nip.c:88-119) -- so a
// slice that does not factorise keeps the general engine.  Candidates are
// leaf variables whose parents are all interface variables; each interface
// variable is a pseudo-child with an indicator table, so its marginal is
// derived from the joint posterior (derive.hip, kDeriveChild) and evidence on
// it is an indicator row.
bool every_slice_prior(const Var& v) {
  if (!v.parents.empty() || !v.has_prior || (v.ifs & IF_OLD_OUTGOING)) return false;
  for (double x : v.prior) if (x > 0) return true;            // nip_enter_prior rejects a zero vector
  return false;
}

void build_joint_chain_plan(Model& m) {
  ChainPlan& P = m.chain;
  P = ChainPlan();
  const auto& V = m.vars;
  const int nv = (int)V.size();
  const auto &prev = m.previous_outgoing, &cur = m.outgoing;
  if (cur.size() < 2 || cur.size() != prev.size()) return;
  long K = 1;
  for (size_t i = 0; i < cur.size(); i++) {
    if (V[cur[i]].card != V[prev[i]].card || !V[prev[i]].parents.empty()) return;
    K *= V[cur[i]].card;
    if (K > 64) return;
  }
  std::vector<int> role(nv, 3);                               // 0 prev, 1 cur, 2 candidate, 3 summed
  for (int v : prev) role[v] = 0;
  for (int v : cur) role[v] = 1;
  std::vector<char> has_child(nv, 0);
  for (int v = 0; v < nv; v++) for (int q : V[v].parents) has_child[q] = 1;
  std::vector<int> cand;
  long C = 1;
  for (int v = 0; v < nv; v++) {
    if (role[v] != 3 || has_child[v] || V[v].parents.empty() || V[v].card > 253) continue;
    bool ok = true;
    for (int q : V[v].parents) ok &= role[q] == 1;
    if (!ok) continue;
    role[v] = 2;
    cand.push_back(v);
    C *= V[v].card;
    if (K * K * C > (1L << 22)) return;
  }
  long total = 1;
  for (int v = 0; v < nv; v++) { total *= V[v].card; if (total > (1L << 20)) return; }
  // F[(x * K + y) * C + c]: the slice joint with everything else summed out
  std::vector<double> F((size_t)(K * K * C), 0.0);
  std::vector<int> val(nv, 0);
  for (long i = 0; i < total; i++) {
    double w = 1.0;
    for (size_t c = 0; c < m.cliques.size() && w != 0.0; c++) {
      const auto& o = m.cliques[c].original;
      const long k = clique_index(m, (int)c, val);
      w *= k < (long)o.size() ? o[k] : 1.0;
    }
    for (int v = 0; v < nv && w != 0.0; v++) if (every_slice_prior(V[v])) w *= V[v].prior[val[v]];
    long x = 0, y = 0, cc = 0, sx = 1, sc = 1;
    for (size_t k = 0; k < cur.size(); k++) {
      x += val[prev[k]] * sx; y += val[cur[k]] * sx; sx *= V[cur[k]].card;
    }
    for (int v : cand) { cc += val[v] * sc; sc *= V[v].card; }
    F[(size_t)((x * K + y) * C + cc)] += w;
    for (int v = 0; v < nv; v++) {                              // odometer, variable 0 fastest
      if (++val[v] < V[v].card) break;
      val[v] = 0;
    }
  }
  // A and the candidates' tables, then the factorisation check
  std::vector<double> A((size_t)(K * K), 0.0);
  double fmax = 0.0;
  for (long xy = 0; xy < K * K; xy++)
    for (long c = 0; c < C; c++) { A[xy] += F[xy * C + c]; fmax = std::max(fmax, F[xy * C + c]); }
  std::vector<std::vector<double>> E(cand.size());
  for (size_t k = 0; k < cand.size(); k++) {
    const int M = V[cand[k]].card;
    long stride = 1;
    for (size_t j = 0; j < k; j++) stride *= V[cand[j]].card;
    E[k].assign((size_t)M * 64, 0.0);
    for (long y = 0; y < K; y++) {
      long xb = -1;
      for (long x = 0; x < K; x++) if (A[x * K + y] > 0 && (xb < 0 || A[x * K + y] > A[xb * K + y])) xb = x;
      if (xb < 0) continue;                                      // y unreachable: its evidence never matters
      for (long c = 0; c < C; c++)
        E[k][(size_t)((c / stride) % M) * 64 + y] += F[(xb * K + y) * C + c];
      for (int mm = 0; mm < M; mm++) E[k][(size_t)mm * 64 + y] /= A[xb * K + y];
    }
  }
  for (long x = 0; x < K; x++)
    for (long y = 0; y < K; y++)
      for (long c = 0; c < C; c++) {
        double f = A[x * K + y];
        long r = c;
        for (size_t k = 0; k < cand.size(); k++) {
          const int M = V[cand[k]].card;
          f *= E[k][(size_t)(r % M) * 64 + y];
          r /= M;
        }
        if (std::fabs(f - F[(x * K + y) * C + c]) > 1e-13 * fmax) return;   // does not factorise
      }
  P.N = (int)K;
  P.A64.assign(64 * 64, 0.0);
  for (long x = 0; x < K; x++)
    for (long y = 0; y < K; y++) P.A64[x * 64 + y] = A[x * K + y];
  P.pi64.assign(64, 0.0);
  for (long x = 0; x < K; x++) {
    double p = 1.0;
    long r = x;
    for (int v : prev) {
      const int d = (int)(r % V[v].card);
      r /= V[v].card;
      bool entered = V[v].has_prior;
      if (entered) { entered = false; for (double q : V[v].prior) entered |= q > 0; }
      if (entered) p *= V[v].prior[d];
    }
    P.pi64[x] = p;
  }
  for (size_t k = 0; k < cand.size(); k++) {
    ChainEmit em;
    em.var = cand[k]; em.clique = V[cand[k]].family; em.M = V[cand[k]].card;
    em.E = std::move(E[k]);
    em.s.assign(64, 0.0);
    for (long y = 0; y < K; y++)
      for (int mm = 0; mm < em.M; mm++) em.s[y] += em.E[(size_t)mm * 64 + y];
    P.emits.push_back(std::move(em));
  }
  long sx = 1;
  for (size_t i = 0; i < cur.size(); i++) {                   // the interface variables: indicator pseudo-children
    ChainEmit em;
    em.var = cur[i]; em.clique = V[cur[i]].family; em.M = V[cur[i]].card;
    em.E.assign((size_t)em.M * 64, 0.0);
    em.s.assign(64, 0.0);
    for (long y = 0; y < K; y++) { em.E[(size_t)((y / sx) % em.M) * 64 + y] = 1.0; em.s[y] = 1.0; }
    sx *= em.M;
    P.emits.push_back(std::move(em));
  }
  P.s_all64.assign(64, 0.0);
  for (long y = 0; y < K; y++) {
    double s = 1.0;
    for (const auto& em : P.emits) s *= em.s[y];
    P.s_all64[y] = s;
  }
  if (K <= 16) {
    P.A.assign(256, 0.0);
    P.pi.assign(16, 0.0);
    for (long x = 0; x < K; x++) {
      P.pi[x] = P.pi64[x];
      for (long y = 0; y < K; y++) P.A[x * 16 + y] = P.A64[x * 64 + y];
    }
  }
  P.jprev = prev;
  P.jcur = cur;
  bool summed = false;
  for (int v = 0; v < nv; v++) summed |= role[v] == 3;
  // e_step on the HMM e_step kernel over the joint state, the slab projected
  // onto every family (engine.cpp ensure_joint_map)
  P.jhmm = !summed && cand.size() == 1 && K <= 16;
  P.joint = true;
  P.valid = true;
}
}  // namespace

void hidden_table(const Model& m, int j, std::vector<double>& G) {
  const ChainPlan& P = m.chain;
  const auto& V = m.vars;
  const int N = P.N, vp = P.v_prev, vc = P.v_cur, cin = P.c_trans;
  const int cj = V[P.hidden[j]].card;
  G.assign((size_t)cj * 64 * 64, 0.0);
  long hsize = 1;
  for (int h : P.hidden) hsize *= V[h].card;
  std::vector<int> val(V.size(), 0), hv(P.hidden.size(), 0);
  for (long hi = 0; hi < hsize; hi++) {              // the order of build_chain_plan's A64 loop
    long r = hi;
    double w = 1.0;
    for (size_t k = 0; k < P.hidden.size(); k++) {
      const int c = V[P.hidden[k]].card;
      hv[k] = (int)(r % c); r /= c;
      val[P.hidden[k]] = hv[k];
      w *= V[P.hidden[k]].prior[hv[k]];
    }
    double* g = G.data() + (size_t)hv[j] * 64 * 64;
    for (int x = 0; x < N; x++)
      for (int y = 0; y < N; y++) {
        val[vp] = x; val[vc] = y;
        g[x * 64 + y] += m.cliques[cin].original[clique_index(m, cin, val)] * w;
      }
  }
}

}  // namespace nipamd
