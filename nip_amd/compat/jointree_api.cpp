// libnip.so -- cliques, sepsets and join-tree operations (src/nipjointree.h,
// declared in include/compat/nipjointree.h).
//
// Propagation goes to the GPU.  nip_collect_evidence / nip_distribute_evidence
// walk the tree exactly as the reference does (src/nipjointree.c:580-673:
// marks, sepset-list order, collect's two independent neighbour tests,
// distribute's passes-then-recursion) and record each nip_message_pass
// (:676-709) -- including its swap of the sepset's old/new potentials -- as a
// pass (source table, new message, old message, target table, the two
// mappings).  The recorded passes then run in order on the device through
// nipamd_hugin_passes (nip_amd/csrc/hugin.hip), with the reference's
// arithmetic, so the tables end bit-identical.  The traversal reads no table
// data, so recording first and executing after is the same computation.
//
// The rest is bookkeeping over the host tables: evidence entry and global
// retraction (:791-943), families (:967-1064), the probability mass
// (:1108-1188) and the joint-probability gather (:1198-1402).
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "nip_amd.h"
#include "niperrorhandler.h"
#include "nipjointree.h"

namespace {

#define REPORT(e) nip_report_error((char*)__FILE__, __LINE__, (e), 1)
#define QUIET(e) nip_report_error((char*)__FILE__, __LINE__, (e), 0)

// the caller's rand() stream is the caller's: the HIP runtime runs on a
// scratch state (as in compat.cpp)
struct RandGuard {
  char scratch[128];
  char* saved;
  RandGuard() { saved = initstate(1, scratch, sizeof scratch); }
  ~RandGuard() { setstate(saved); }
};

bool marked(nip_clique c) { return c && c->mark == NIP_MARK_ON; }

int dim(nip_potential p) { return p->dimensionality; }

// position of v among c's variables, -1 if absent (nip_clique_var_index, :950-964)
int var_index(nip_clique c, nip_variable v) {
  if (!(c && v)) {
    REPORT(EFAULT);
    return -1;
  }
  for (int i = 0; i < dim(c->p); i++)
    if (nip_equal_variables(v, c->variables[i])) return i;
  return -1;
}

// the neighbour across s from a clique that is marked (collect/distribute
// compare both neighbours' marks; see the call sites for the exact tests)
template <class F>
void for_each_link(nip_clique c, F f) {
  for (nip_sepset_link l = c->sepsets; l; l = l->fwd) f((nip_sepset)l->data);
}

// ---------------------------------------------------------------------------
// the pass recorder

struct Passes {
  std::vector<nip_potential> tables;
  std::unordered_map<nip_potential, int> index;
  std::vector<int> pass, maps;
  int err = 0;

  int table(nip_potential p) {
    auto it = index.find(p);
    if (it != index.end()) return it->second;
    index[p] = (int)tables.size();
    tables.push_back(p);
    return (int)tables.size() - 1;
  }

  // nip_message_pass(c1, s, c2): swap, then marginalise c1 into s->new and
  // absorb it into c2 divided by s->old
  void message(nip_clique c1, nip_sepset s, nip_clique c2) {
    std::swap(s->old, s->new_);
    const int nd = dim(s->new_);
    const int m1 = (int)maps.size();
    for (int k = 0; k < nd; k++) maps.push_back(var_index(c1, s->variables[k]));
    const int m2 = (int)maps.size();
    for (int k = 0; k < nd; k++) maps.push_back(var_index(c2, s->variables[k]));
    if (dim(s->new_) > dim(c1->p)) err = EINVAL;  // nip_general_marginalise's check (nippotential.c:272-273)
    for (int t : {table(c1->p), table(s->new_), table(s->old), table(c2->p), m1, m2}) pass.push_back(t);
  }

  int run() {
    if (err) return REPORT(err);
    if (pass.empty()) return 0;
    std::vector<double*> data;
    std::vector<int> nd, card;
    for (nip_potential p : tables) {
      data.push_back(p->data);
      nd.push_back(p->dimensionality);
      for (int a = 0; a < p->dimensionality; a++) card.push_back(p->cardinality[a]);
    }
    if (maps.empty()) maps.push_back(0);   // every sepset empty: no map entries, a valid pointer
    int e;
    {
      RandGuard guard;
      e = nipamd_hugin_passes((int)tables.size(), data.data(), nd.data(), card.data(),
                              (int)pass.size() / 6, pass.data(), maps.data());
    }
    if (e != NIP_NO_ERROR) {
      std::fprintf(stderr, "nip_amd: %s\n", nipamd_last_error());
      return REPORT(e == NIP_ERROR_INVALID_ARGUMENT ? EINVAL : e);
    }
    return 0;
  }
};

// nip_collect_evidence's traversal (:630-673): mark c2, recurse into every
// unmarked neighbour (both neighbours tested, no else, :642-652), then pass
// c2's message to c1
void collect(Passes& P, nip_clique c1, nip_sepset s12, nip_clique c2) {
  c2->mark = NIP_MARK_ON;
  for_each_link(c2, [&](nip_sepset s) {
    if (!marked(s->first_neighbour)) collect(P, c2, s, s->first_neighbour);
    if (!marked(s->second_neighbour)) collect(P, c2, s, s->second_neighbour);
  });
  if (c1 && s12) P.message(c2, s12, c1);
}

// nip_distribute_evidence's traversal (:580-627): mark c, pass to every
// unmarked neighbour (first, else second), then recurse in the same order
void distribute(Passes& P, nip_clique c) {
  c->mark = NIP_MARK_ON;
  auto other = [](nip_sepset s) -> nip_clique {
    if (!marked(s->first_neighbour)) return s->first_neighbour;
    if (!marked(s->second_neighbour)) return s->second_neighbour;
    return nullptr;
  };
  for_each_link(c, [&](nip_sepset s) {
    if (nip_clique n = other(s)) P.message(c, s, n);
  });
  for_each_link(c, [&](nip_sepset s) {
    if (nip_clique n = other(s)) distribute(P, n);
  });
}

// nip_join_tree_dfs (:1108-1153): the clique, then for each link with an
// unmarked neighbour (first, else second) the sepset and the subtree
template <class CF, class SF>
void dfs(nip_clique c, CF cf, SF sf) {
  c->mark = NIP_MARK_ON;
  cf(c);
  for_each_link(c, [&](nip_sepset s) {
    nip_clique n = !marked(s->first_neighbour) ? s->first_neighbour
                   : !marked(s->second_neighbour) ? s->second_neighbour : nullptr;
    if (!n) return;
    sf(s);
    dfs(n, cf, sf);
  });
}

nip_potential potential_over(nip_variable* vars, int n) {
  std::vector<int> card(n > 0 ? n : 1);
  for (int i = 0; i < n; i++) card[i] = NIP_CARDINALITY(vars[i]);
  return nip_new_potential(card.data(), n, nullptr);
}

// nip_mapper padded with zeros to `len` entries.  nip_gather_joint_probability
// hands update_potential a mapping shorter than the numerator's
// dimensionality whenever a sepset holds variables of interest
// (:1340-1345): the reference then reads past the end of the mapping, into
// the slack of its calloc'd block, which glibc hands out zeroed -- index 0.
std::vector<int> padded_map(nip_variable* set, int nset, nip_variable* sub, int nsub, int len) {
  std::vector<int> m(len > nsub ? len : (nsub > 0 ? nsub : 1), 0);
  int* r = nip_mapper(set, sub, nset, nsub);
  for (int i = 0; i < nsub && r; i++) m[i] = r[i];
  std::free(r);
  return m;
}

// Whether the reference's gather stays inside its arrays.  Where it does not
// (it reads past a mapping's allocation, indexes a table with a digit larger
// than that dimension, or writes n_vars + n_isect cardinalities into an array
// of nprod, :1372-1377), its result is undefined -- garbage or a corrupted
// heap (an abort, for some variable sets); this implementation then reports
// an error and returns NULL instead.
bool zeroed_slack(int n_alloc, int n_read) {   // glibc calloc: chunk = max(32, n*4 + 8 rounded to 16)
  const int bytes = n_alloc * 4 + 8;
  const int chunk = bytes < 32 ? 32 : (bytes + 15) & ~15;
  return n_read <= (chunk - 8) / 4;
}

// digit of big's dimension map[k] indexes small's dimension k
bool digits_fit(const nip_potential big, const std::vector<int>& map, const nip_potential small) {
  for (int k = 0; k < small->dimensionality; k++)
    if (map[k] < 0 || map[k] >= big->dimensionality || big->cardinality[map[k]] > small->cardinality[k])
      return false;
  return true;
}

}  // namespace

extern "C" {

nip_clique nip_new_clique(nip_variable vars[], int nvars) {
  auto* c = (nip_clique)std::calloc(1, sizeof(nip_clique_struct));
  if (!c) {
    REPORT(ENOMEM);
    return nullptr;
  }
  c->variables = (nip_variable*)std::calloc(nvars > 0 ? nvars : 1, sizeof(nip_variable));
  std::vector<int> card(nvars > 0 ? nvars : 1);
  if (!c->variables) {
    std::free(c);
    REPORT(ENOMEM);
    return nullptr;
  }
  // ascending ID: variable i goes to position #{j : id_j < id_i} (:122-133)
  for (int i = 0; i < nvars; i++) {
    int r = 0;
    for (int j = 0; j < nvars; j++) r += nip_variable_id(vars[j]) < nip_variable_id(vars[i]);
    c->variables[r] = vars[i];
  }
  for (int i = 0; i < nvars; i++) card[i] = NIP_CARDINALITY(c->variables[i]);
  c->p = nip_new_potential(card.data(), nvars, nullptr);
  c->original_p = nip_new_potential(card.data(), nvars, nullptr);
  if (!c->p || !c->original_p) {
    nip_free_potential(c->p);
    nip_free_potential(c->original_p);
    std::free(c->variables);
    std::free(c);
    REPORT(EFAULT);
    return nullptr;
  }
  c->sepsets = nullptr;
  c->num_of_sepsets = 0;
  c->mark = NIP_MARK_OFF;
  return c;
}

}  // extern "C"

namespace {
void remove_link(nip_clique c, nip_sepset s) {
  if (!(c && s)) {
    REPORT(EFAULT);
    return;
  }
  for (nip_sepset_link l = c->sepsets; l; l = l->fwd)
    if (l->data == s) {
      if (l->bwd) l->bwd->fwd = l->fwd; else c->sepsets = l->fwd;
      if (l->fwd) l->fwd->bwd = l->bwd;
      std::free(l);
      c->num_of_sepsets--;
      return;
    }
}
}  // namespace

extern "C" {

void nip_free_clique(nip_clique c) {
  if (!c) return;
  while (c->sepsets) {
    auto* s = (nip_sepset)c->sepsets->data;
    remove_link(s->first_neighbour, s);
    remove_link(s->second_neighbour, s);
    nip_free_sepset(s);
  }
  nip_free_potential(c->p);
  nip_free_potential(c->original_p);
  std::free(c->variables);
  std::free(c);
}

// link s at the front of both neighbours' lists (:211-234)
int nip_confirm_sepset(nip_sepset s) {
  auto* a = (nip_sepset_link)std::malloc(sizeof(nip_sepsetlink_struct));
  auto* b = (nip_sepset_link)std::malloc(sizeof(nip_sepsetlink_struct));
  if (!a || !b) {
    std::free(a);
    std::free(b);
    return REPORT(ENOMEM);
  }
  nip_clique cs[2] = {s->first_neighbour, s->second_neighbour};
  nip_sepset_link ls[2] = {a, b};
  for (int i = 0; i < 2; i++) {
    ls[i]->data = s;
    ls[i]->bwd = nullptr;
    ls[i]->fwd = cs[i]->sepsets;
    if (cs[i]->sepsets) cs[i]->sepsets->bwd = ls[i];
    cs[i]->sepsets = ls[i];
    cs[i]->num_of_sepsets++;
  }
  return 0;
}

nip_sepset nip_new_sepset(nip_clique neighbour_a, nip_clique neighbour_b) {
  if (!neighbour_a || !neighbour_b) {
    REPORT(EFAULT);
    return nullptr;
  }
  auto* s = (nip_sepset)std::calloc(1, sizeof(nip_sepset_struct));
  if (!s) {
    REPORT(ENOMEM);
    return nullptr;
  }
  s->first_neighbour = neighbour_a;
  s->second_neighbour = neighbour_b;
  int n = 0;
  s->variables = nip_variable_isect(neighbour_a->variables, neighbour_b->variables,
                                    dim(neighbour_a->p), dim(neighbour_b->p), &n);
  if (n < 0) {
    std::free(s);
    REPORT(EFAULT);
    return nullptr;
  }
  s->old = potential_over(s->variables, n);
  s->new_ = potential_over(s->variables, n);
  if (!s->old || !s->new_) {
    nip_free_sepset(s);
    REPORT(EFAULT);
    return nullptr;
  }
  return s;
}

void nip_free_sepset(nip_sepset s) {
  if (!s) return;
  nip_free_potential(s->old);
  nip_free_potential(s->new_);
  std::free(s->variables);
  std::free(s);
}

// data given in the order of `variables` (dimension 0 fastest) -> a table in
// ascending-ID order (:341-480)
nip_potential nip_create_potential(nip_variable variables[], int nvars, double data[]) {
  std::vector<int> rank(nvars > 0 ? nvars : 1), card(nvars > 0 ? nvars : 1);
  for (int i = 0; i < nvars; i++) {
    rank[i] = 0;
    for (int j = 0; j < nvars; j++) rank[i] += nip_variable_id(variables[j]) < nip_variable_id(variables[i]);
  }
  for (int i = 0; i < nvars; i++) card[rank[i]] = NIP_CARDINALITY(variables[i]);
  nip_potential p = nip_new_potential(card.data(), nvars, nullptr);
  if (!p) {
    REPORT(EFAULT);
    return nullptr;
  }
  if (data) {
    std::vector<int> idx(nvars > 0 ? nvars : 1);
    for (int i = 0; i < p->size_of_data; i++) {
      nip_inverse_mapping(p, i, idx.data());
      long src = 0, s = 1;
      for (int j = 0; j < nvars; j++) {
        src += (long)idx[rank[j]] * s;
        s *= card[rank[j]];
      }
      p->data[i] = data[src];
    }
  }
  return p;
}

void nip_unmark_clique(nip_clique c) {
  if (c) c->mark = NIP_MARK_OFF;
}

int nip_clique_size(nip_clique c) { return c ? dim(c->p) : 0; }
int nip_sepset_size(nip_sepset s) { return s ? dim(s->old) : 0; }

// :546-577 (first neighbour, else second, as the reference tests them)
int nip_cliques_connected(nip_clique one, nip_clique two) {
  if (!one || !two) return 0;
  one->mark = NIP_MARK_ON;
  if (one == two) return 1;
  for (nip_sepset_link l = one->sepsets; l; l = l->fwd) {
    auto* s = (nip_sepset)l->data;
    if (!marked(s->first_neighbour)) {
      if (nip_cliques_connected(s->first_neighbour, two)) return 1;
    } else if (!marked(s->second_neighbour)) {
      if (nip_cliques_connected(s->second_neighbour, two)) return 1;
    }
  }
  return 0;
}

int nip_distribute_evidence(nip_clique c) {
  if (!c) return REPORT(EFAULT);
  Passes P;
  distribute(P, c);
  return P.run();
}

int nip_collect_evidence(nip_clique c1, nip_sepset s12, nip_clique c2) {
  if (!c2) return REPORT(EFAULT);
  Passes P;
  collect(P, c1, s12, c2);
  return P.run();
}

int nipamd_compat_make_consistent(nip_clique* cliques, int ncliques) {
  if (!cliques || ncliques < 1 || !cliques[0]) return REPORT(EFAULT);
  Passes P;
  for (int i = 0; i < ncliques; i++) nip_unmark_clique(cliques[i]);
  collect(P, nullptr, nullptr, cliques[0]);
  for (int i = 0; i < ncliques; i++) nip_unmark_clique(cliques[i]);
  distribute(P, cliques[0]);
  return P.run();
}

// :1198-1402, operation for operation (see padded_map for the one place the
// reference reads outside its arrays)
nip_potential nip_gather_joint_probability(nip_clique start, nip_variable* vars, int n_vars,
                                           nip_variable* isect, int n_isect) {
  if (!start || n_vars < 0) {
    REPORT(EINVAL);
    return nullptr;
  }
  if (n_vars == 0) return nip_new_potential(nullptr, 0, nullptr);
  if (!vars) {
    REPORT(EFAULT);
    return nullptr;
  }
  start->mark = NIP_MARK_ON;
  int nprod = 0;
  nip_variable* prod_vars = nip_variable_union(vars, start->variables, n_vars, dim(start->p), &nprod);
  if (!prod_vars) {
    REPORT(ENOMEM);
    return nullptr;
  }
  nip_potential prod = potential_over(prod_vars, nprod);
  auto fail = [&]() -> nip_potential {
    std::free(prod_vars);
    nip_free_potential(prod);
    return nullptr;
  };
  if (!prod) return fail();
  {
    auto m = padded_map(prod_vars, nprod, start->variables, dim(start->p), dim(start->p));
    if (int e = nip_update_potential(start->p, nullptr, prod, m.data())) {
      REPORT(e);
      return fail();
    }
  }
  for (nip_sepset_link l = start->sepsets; l; l = l->fwd) {
    auto* s = (nip_sepset)l->data;
    for (nip_clique c : {s->first_neighbour, s->second_neighbour}) {
      if (marked(c)) continue;
      auto m = padded_map(prod_vars, nprod, s->variables, dim(s->new_), dim(s->new_));
      if (int e = nip_update_potential(nullptr, s->new_, prod, m.data())) {
        REPORT(e);
        return fail();
      }
      int nmsgi = 0;
      nip_variable* msg_isect = nip_variable_isect(s->variables, vars, dim(s->new_), n_vars, &nmsgi);
      if (!msg_isect) {   // also an empty intersection: isect returns NULL (:1327-1333)
        REPORT(ENOMEM);
        return fail();
      }
      nip_potential msg = nip_gather_joint_probability(c, vars, n_vars, msg_isect, nmsgi);
      if (!msg) {
        std::free(msg_isect);
        return fail();
      }
      int nmsg = 0;
      nip_variable* msg_vars = nip_variable_union(vars, msg_isect, n_vars, nmsgi, &nmsg);
      auto mm = padded_map(prod_vars, nprod, msg_vars, nmsg, dim(msg));
      std::free(msg_vars);
      std::free(msg_isect);
      if (!zeroed_slack(nmsg, dim(msg)) || !digits_fit(prod, mm, msg)) {
        nip_free_potential(msg);
        std::fprintf(stderr, "nip_amd: the reference's join-tree gather is undefined here (it reads outside its arrays)\n");
        REPORT(EINVAL);
        return fail();
      }
      const int e = nip_update_potential(msg, nullptr, prod, mm.data());
      nip_free_potential(msg);
      if (e) {
        REPORT(e);
        return fail();
      }
    }
  }
  std::free(prod_vars);
  if (nprod == n_vars + n_isect) return prod;
  std::vector<int> card(n_vars + n_isect), map(n_vars + n_isect);
  for (int i = 0; i < n_vars; i++) card[i] = NIP_CARDINALITY(vars[i]);
  for (int i = 0; i < n_isect; i++) card[n_vars + i] = NIP_CARDINALITY(isect[i]);
  for (int i = 0; i < n_vars + n_isect; i++) map[i] = i;
  nip_potential sum = nip_new_potential(card.data(), n_vars + n_isect, nullptr);
  if (sum && (n_vars + n_isect > nprod || !digits_fit(prod, map, sum))) {
    nip_free_potential(prod);
    nip_free_potential(sum);
    std::fprintf(stderr, "nip_amd: the reference's join-tree gather is undefined here (it writes outside its arrays)\n");
    REPORT(EINVAL);
    return nullptr;
  }
  const int e = sum ? nip_general_marginalise(prod, sum, map.data()) : ENOMEM;
  nip_free_potential(prod);
  if (e) {
    REPORT(e);
    nip_free_potential(sum);
    return nullptr;
  }
  return sum;
}

// :713-772: the mapping lists the family's positions in clique order (each
// clique variable that is a parent or the child, in clique order)
int nip_init_clique(nip_clique c, nip_variable child, nip_potential p, int transient) {
  nip_variable* parents = nip_get_parents(child);
  std::vector<int> mapping;
  const bool mapped = dim(p) < dim(c->p);
  if (mapped) {
    for (int i = 0; i < dim(c->p) && (int)mapping.size() < dim(p); i++) {
      nip_variable v = c->variables[i];
      for (int j = 0; j < dim(p) - 1; j++)
        if (nip_equal_variables(v, parents[j])) mapping.push_back(i);
      if (nip_equal_variables(v, child)) mapping.push_back(i);
    }
    mapping.resize(dim(p) > 0 ? dim(p) : 1, 0);
  }
  if (int e = nip_init_potential(p, c->p, mapped ? mapping.data() : nullptr)) return REPORT(e);
  if (!transient)
    if (int e = nip_init_potential(p, c->original_p, mapped ? mapping.data() : nullptr)) return REPORT(e);
  return 0;  // p stays the caller's (the reference neither stores nor frees it)
}

int nip_marginalise_clique(nip_clique c, nip_variable v, double r[]) {
  const int index = var_index(c, v);
  if (index < 0) return REPORT(EINVAL);
  const int e = nip_total_marginalise(c->p, r, index);
  if (e) REPORT(e);
  return e;
}

int nip_global_retraction(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques) {
  for (int i = 0; i < ncliques; i++) nip_unmark_clique(cliques[i]);
  if (ncliques > 0 && cliques[0])
    dfs(cliques[0], [](nip_clique c) { nip_retract_potential(c->p, c->original_p); },
        [](nip_sepset s) {
          nip_uniform_potential(s->old, 1.0);
          nip_uniform_potential(s->new_, 1.0);
        });
  for (int i = 0; i < nvars; i++) {
    nip_variable v = vars[i];
    nip_clique c = nip_find_family(cliques, ncliques, v);
    const int index = var_index(c, v);
    if (!c || index < 0) return REPORT(EINVAL);
    if (int e = nip_update_evidence(v->likelihood, nullptr, c->p, index)) return REPORT(e);
  }
  return 0;
}

// sum of clique masses minus sepset masses in DFS order from cliques[0]
// (:1156-1188); each table summed ascending, then added to the running total
double nip_probability_mass(nip_clique* cliques, int ncliques) {
  for (int i = 0; i < ncliques; i++) nip_unmark_clique(cliques[i]);
  double ret = 0.0;
  auto mass = [](nip_potential p) {
    double m = 0.0;
    for (int i = 0; i < p->size_of_data; i++) m += p->data[i];
    return m;
  };
  if (ncliques > 0 && cliques[0])
    dfs(cliques[0], [&](nip_clique c) { ret += mass(c->p); }, [&](nip_sepset s) { ret -= mass(s->new_); });
  return ret;
}

int nip_enter_observation(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                          nip_variable v, char* state) {
  const int index = nip_variable_state_index(v, state);
  if (index < 0) return 0;
  return nip_enter_index_observation(vars, nvars, cliques, ncliques, v, index);
}

int nip_enter_index_observation(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                                nip_variable v, int index) {
  if (index < 0) return 0;
  std::vector<double> e(NIP_CARDINALITY(v), 0.0);
  if (index < (int)e.size()) e[index] = 1.0;
  return nip_enter_evidence(vars, nvars, cliques, ncliques, v, e.data());
}

// :859-901: zero -> nonzero likelihood needs a global retraction (after the
// likelihood is updated); otherwise evidence / old likelihood on the family
int nip_enter_evidence(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                       nip_variable v, double evidence[]) {
  if (!v || !evidence) return REPORT(EFAULT);
  nip_clique c = nip_find_family(cliques, ncliques, v);
  if (!c) return QUIET(EINVAL);
  const int index = var_index(c, v);
  bool retraction = false;
  for (int i = 0; i < NIP_CARDINALITY(v); i++)
    if (v->likelihood[i] == 0.0 && evidence[i] != 0.0) retraction = true;
  if (!retraction)
    if (int e = nip_update_evidence(evidence, v->likelihood, c->p, index)) return REPORT(e);
  if (int e = nip_update_likelihood(v, evidence)) return REPORT(e);
  if (retraction)
    if (int e = nip_global_retraction(vars, nvars, cliques, ncliques)) return REPORT(e);
  return 0;
}

int nip_enter_prior(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                    nip_variable v, double prior[]) {
  (void)vars;
  (void)nvars;
  if (!v || !prior) return REPORT(EFAULT);
  nip_clique c = nip_find_family(cliques, ncliques, v);
  bool zero = true;
  for (int i = 0; i < NIP_CARDINALITY(v); i++)
    if (prior[i] > 0) zero = false;
  if (!c || zero) return QUIET(EINVAL);
  const int index = var_index(c, v);
  if (int e = nip_update_evidence(prior, nullptr, c->p, index)) return REPORT(e);
  return 0;
}

nip_clique nip_find_family(nip_clique* cliques, int ncliques, nip_variable var) {
  if (var->family_clique) return (nip_clique)var->family_clique;
  const int n = nip_number_of_parents(var);
  std::vector<nip_variable> family(n > 0 ? n + 1 : 1);
  for (int i = 0; i < n; i++) family[i] = var->parents[i];
  family[n > 0 ? n : 0] = var;
  nip_clique found = nip_find_clique(cliques, ncliques, family.data(), (n > 0 ? n : 0) + 1);
  var->family_clique = found;
  return found;
}

// child first, then the parents in v->parents order (:996-1040), memoised
int* nip_find_family_mapping(nip_clique family, nip_variable child) {
  if (!family || !child) {
    REPORT(EFAULT);
    return nullptr;
  }
  if (!child->family_mapping) {
    const int n = nip_number_of_parents(child) + 1;
    int* r = (int*)std::calloc(n, sizeof(int));
    if (!r) {
      REPORT(ENOMEM);
      return nullptr;
    }
    for (int i = 0; i < dim(family->p); i++)
      if (nip_equal_variables(family->variables[i], child)) {
        r[0] = i;
        break;
      }
    int found = 0;
    for (int i = 0; i < dim(family->p) && found < n - 1; i++)
      for (int j = 0; j < n - 1; j++)
        if (nip_equal_variables(family->variables[i], child->parents[j])) {
          r[j + 1] = i;
          found++;
          break;
        }
    child->family_mapping = r;
  }
  return child->family_mapping;
}

nip_clique nip_find_clique(nip_clique* cliques, int ncliques, nip_variable* variables, int nvars) {
  for (int i = 0; i < ncliques; i++) {
    int ok = 0;
    for (int j = 0; j < nvars; j++)
      if (var_index(cliques[i], variables[j]) >= 0) ok++;
    if (ok == nvars) return cliques[i];
  }
  return nullptr;
}

void nip_fprintf_clique(FILE* stream, nip_clique c) {
  std::fprintf(stream, "clique ");
  for (int i = 0; i < dim(c->p); i++) std::fprintf(stream, "%s ", nip_variable_symbol(c->variables[i]));
  std::fprintf(stream, "\n");
}

void nip_fprintf_sepset(FILE* stream, nip_sepset s) {
  std::fprintf(stream, "sepset ");
  for (int i = 0; i < dim(s->old); i++) std::fprintf(stream, "%s ", nip_variable_symbol(s->variables[i]));
  std::fprintf(stream, "\n");
}

// declared by the reference (nipjointree.h:380-381) but never defined there;
// the intersection in cl1's order, as its documentation describes
int nip_clique_intersection(nip_clique cl1, nip_clique cl2, nip_variable** vars, int* n) {
  if (!cl1 || !cl2 || !vars || !n) return REPORT(EFAULT);
  *vars = nip_variable_isect(cl1->variables, cl2->variables, dim(cl1->p), dim(cl2->p), n);
  return *n < 0 ? REPORT(ENOMEM) : 0;
}

nip_potential_list nip_new_potential_list(void) {
  auto* l = (nip_potential_list)std::calloc(1, sizeof(nip_potential_list_struct));
  if (!l) REPORT(ENOMEM);
  return l;
}

}  // extern "C"

namespace {
int add_potential(nip_potential_list l, nip_potential p, nip_variable child, nip_variable* parents,
                  bool front) {
  if (!l || !p) return REPORT(EFAULT);
  auto* k = (nip_potential_link)std::malloc(sizeof(nip_potential_link_struct));
  if (!k) return REPORT(ENOMEM);
  k->data = p;
  k->child = child;
  k->parents = parents;  // the list owns the parents array (:1431-1432)
  if (front) {
    k->bwd = nullptr;
    k->fwd = l->first;
    if (l->first) l->first->bwd = k; else l->last = k;
    l->first = k;
  } else {
    k->fwd = nullptr;
    k->bwd = l->last;
    if (l->last) l->last->fwd = k; else l->first = k;
    l->last = k;
  }
  l->length++;
  return 0;
}
}  // namespace

extern "C" {

int nip_append_potential(nip_potential_list l, nip_potential p, nip_variable child, nip_variable* parents) {
  return add_potential(l, p, child, parents, false);
}
int nip_prepend_potential(nip_potential_list l, nip_potential p, nip_variable child, nip_variable* parents) {
  return add_potential(l, p, child, parents, true);
}

void nip_free_potential_list(nip_potential_list l) {
  if (!l) return;
  for (nip_potential_link k = l->first; k;) {
    nip_potential_link n = k->fwd;
    nip_free_potential(k->data);
    std::free(k->parents);
    std::free(k);
    k = n;
  }
  std::free(l);
}

}  // extern "C"
