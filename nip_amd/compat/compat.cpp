// libnip.so -- the reference's nip.h API (src/nip.h) over the nip_amd GPU
// engine (the drop-in boundary with the reference's struct
// layouts).  Declared in include/compat/nip.h.
//
// Each nip_model owns an engine handle (nipamd_model) in a side table keyed
// by the nip_model pointer, so the public struct keeps the reference's layout
// (nip.h:71-104).  The variable records (nipvariable.h:51-78) and the join
// tree (nipjointree.h:43-63: cliques with the compiled original_p, sepsets,
// sepset lists in the reference's order) are built from the engine's
// compiled model.  Work goes to the GPU:
//   forward_inference           -> nipamd_filter_host   (nip.c:1103-1315)
//   forward_backward_inference  -> nipamd_fb_host       (nip.c:1320-1581)
//   em_learn                    -> nipamd_em_learn      (nip.c:2076-2243)
//   make_consistent             -> nipamd_hugin_passes  (nip.c:1600-1617)
// with the evidence of MARKED observed variables only (insert_ts_step with
// NIP_MARK_ON, nip.c:982-1003, 1240, 1455, 1816).  There is no CPU path: a
// request the engine has no GPU plan for fails (NULL / error code) after
// nip_report_error.  Edits a caller makes to the host join tree's
// original_p tables or to priors (nip_init_clique, nip_set_prior, ...) are
// forwarded to the engine before each engine call (sync_engine).
#include <array>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <string>
#include <unordered_map>
#include <unistd.h>
#include <vector>

#include "nip.h"

extern "C" unsigned long nipamd_compat_take_ids(int n);   // variable_api.cpp

namespace {

struct Compat {
  nip_model_struct pub{};
  nipamd_model* eng = nullptr;
  unsigned long id0 = 0;                  // ID of variable 0 (IDs are consecutive)
  // the records; their arrays are malloc'd because the reference's API frees
  // or replaces them (nip_set_parents, nip_set_prior, nip_find_family_mapping)
  std::vector<nip_variable_struct> vars;
  std::vector<nip_variable> all, next, previous, outgoing, prev_outgoing, incoming, children,
      independent;
  std::vector<nip_clique> cliques;
  std::vector<nip_sepset> sepsets;
  // the tables the engine holds (what sync_engine compares host edits against)
  std::vector<std::vector<double>> eng_orig, eng_prior;
};

std::unordered_map<const nip_model_struct*, Compat*> g_models;

Compat* lookup(nip_model m) {
  auto it = g_models.find(m);
  return it == g_models.end() ? nullptr : it->second;
}

// model variable index of v, -1 if v is not one of c's variables
int index_of(const Compat* c, nip_variable v) {
  if (!v || v->id < c->id0 || v->id >= c->id0 + c->vars.size()) return -1;
  const int i = (int)(v->id - c->id0);
  return &c->vars[i] == v ? i : -1;
}

#define REPORT(e) nip_report_error((char*)__FILE__, __LINE__, (e), 1)

// The caller's rand() stream belongs to the caller (random_seed, lottery, the
// reference's generate_data and em_learn draw from it): while the engine and
// the HIP runtime run, rand() is switched to a scratch state, so nothing they
// do (runtime initialisation included) draws from or reseeds the caller's.
struct RandGuard {
  char scratch[128];
  char* saved;
  RandGuard() { saved = initstate(1, scratch, sizeof scratch); }
  ~RandGuard() { setstate(saved); }
};

void engine_error(int e) {
  std::fprintf(stderr, "nip_amd: %s\n", nipamd_last_error());
  REPORT(e);
}

// Forward host-side edits of original_p / priors to the engine.
int sync_engine(Compat* c) {
  const int nc = (int)c->cliques.size(), nv = (int)c->vars.size();
  std::vector<const double*> orig(nc, nullptr), pri(nv, nullptr);
  bool dirty = false;
  for (int k = 0; k < nc; k++) {
    nip_potential o = c->cliques[k]->original_p;
    auto& e = c->eng_orig[k];
    if ((size_t)o->size_of_data == e.size() &&
        std::memcmp(o->data, e.data(), e.size() * sizeof(double)) != 0) {
      orig[k] = o->data;
      e.assign(o->data, o->data + e.size());
      dirty = true;
    }
  }
  for (int i = 0; i < nv; i++) {
    nip_variable v = &c->vars[i];
    auto& e = c->eng_prior[i];
    if (v->num_of_parents > 0 || !v->prior || e.size() != (size_t)v->cardinality) continue;
    if (std::memcmp(v->prior, e.data(), e.size() * sizeof(double)) != 0) {
      pri[i] = v->prior;
      e.assign(v->prior, v->prior + e.size());
      dirty = true;
    }
  }
  if (!dirty) return NIP_NO_ERROR;
  return nipamd_model_set_tables(c->eng, nc, orig.data(), nv, pri.data());
}

// After the engine changed its tables (em_learn's m_step): the host join
// tree's original_p and p, and the priors, take the engine's values.
void pull_engine(Compat* c) {
  for (size_t k = 0; k < c->cliques.size(); k++) {
    nip_potential o = c->cliques[k]->original_p;
    nipamd_model_original(c->eng, (int)k, o->data, o->size_of_data);
    std::memcpy(c->cliques[k]->p->data, o->data, sizeof(double) * o->size_of_data);
    c->eng_orig[k].assign(o->data, o->data + o->size_of_data);
  }
  for (size_t i = 0; i < c->vars.size(); i++) {
    nip_variable v = &c->vars[i];
    if (!v->prior || v->num_of_parents > 0) continue;
    if (nipamd_model_prior(c->eng, (int)i, nullptr) == v->cardinality) {
      nipamd_model_prior(c->eng, (int)i, v->prior);
      c->eng_prior[i].assign(v->prior, v->prior + v->cardinality);
    }
  }
}

// the marked observed columns of a series: (column, model variable)
void marked_columns(const time_series ts, const Compat* c, std::vector<int>& col,
                    std::vector<int>& var) {
  col.clear();
  var.clear();
  for (int i = 0; i < ts->num_of_observed; i++) {
    nip_variable v = ts->observed[i];
    if (!(NIP_MARK(v) & NIP_MARK_ON)) continue;
    col.push_back(i);
    var.push_back(index_of(c, v));
  }
}

uncertain_series new_ucs(nip_variable vars[], int nvars, int T) {
  auto* u = (uncertain_series)std::calloc(1, sizeof(uncertain_series_struct));
  if (!u) return nullptr;
  u->num_of_vars = nvars;
  u->length = T;
  u->variables = (nip_variable*)std::calloc(nvars > 0 ? nvars : 1, sizeof(nip_variable));
  u->data = (double***)std::calloc(T > 0 ? T : 1, sizeof(double**));
  bool ok = u->variables && u->data;
  if (ok && nvars > 0) std::memcpy(u->variables, vars, (size_t)nvars * sizeof(nip_variable));
  for (int t = 0; ok && t < T; t++) {
    u->data[t] = (double**)std::calloc(nvars > 0 ? nvars : 1, sizeof(double*));
    ok = u->data[t] != nullptr;
    for (int i = 0; ok && i < nvars; i++)
      ok = (u->data[t][i] = (double*)std::calloc(NIP_CARDINALITY(vars[i]), sizeof(double))) != nullptr;
  }
  if (!ok) {
    free_uncertainseries(u);
    return nullptr;
  }
  return u;
}

// n series through the engine, batched by (length, marked columns)
int run_inference(time_series* ts, int n, nip_variable vars[], int nvars, bool filter,
                  uncertain_series* out, double* ll) {
  if (!ts || n < 1 || !out || (nvars > 0 && !vars)) return NIP_ERROR_INVALID_ARGUMENT;
  for (int s = 0; s < n; s++) out[s] = nullptr;
  Compat* c = ts[0] ? lookup(ts[0]->model) : nullptr;
  if (!c) return NIP_ERROR_INVALID_ARGUMENT;
  if (int e = sync_engine(c)) return e;
  std::vector<int> q(nvars), off(nvars);
  int stride = 0;
  for (int i = 0; i < nvars; i++) {
    if ((q[i] = index_of(c, vars[i])) < 0) return NIP_ERROR_INVALID_ARGUMENT;
    off[i] = stride;
    stride += NIP_CARDINALITY(vars[i]);
  }
  std::map<std::pair<int, std::vector<int>>, std::vector<int>> groups;
  std::vector<std::vector<int>> cols(n), ovars(n);
  for (int s = 0; s < n; s++) {
    if (!ts[s] || ts[s]->model != ts[0]->model || ts[s]->length < 0) return NIP_ERROR_INVALID_ARGUMENT;
    marked_columns(ts[s], c, cols[s], ovars[s]);
    groups[{ts[s]->length, ovars[s]}].push_back(s);
  }
  int rc = NIP_NO_ERROR;
  for (const auto& [key, ids] : groups) {
    const int T = key.first, B = (int)ids.size();
    const std::vector<int>& ov = key.second;
    const int k = (int)ov.size();
    std::vector<double> post((size_t)B * T * (stride > 0 ? stride : 1)), l(B, 0.0);
    if (T > 0) {
      std::vector<int32_t> obs((size_t)B * T * (k > 0 ? k : 1), -1);
      for (int b = 0; b < B; b++) {
        const time_series x = ts[ids[b]];
        for (int t = 0; t < T; t++)
          for (int i = 0; i < k; i++) obs[((size_t)b * T + t) * k + i] = x->data[t][cols[ids[b]][i]];
      }
      std::vector<uint32_t> st(B);
      RandGuard guard;
      rc = (filter ? nipamd_filter_host : nipamd_fb_host)(c->eng, obs.data(), k, ov.data(), B, T,
                                                          nvars, q.data(), post.data(), l.data(),
                                                          st.data());
      if (rc != NIP_NO_ERROR) break;
    }
    for (int b = 0; b < B; b++) {
      uncertain_series u = new_ucs(vars, nvars, T);
      if (!u) {
        rc = NIP_ERROR_OUTOFMEMORY;
        break;
      }
      const double* p = post.data() + (size_t)b * T * stride;
      for (int t = 0; t < T; t++)
        for (int i = 0; i < nvars; i++)
          std::memcpy(u->data[t][i], p + (size_t)t * stride + off[i],
                      (size_t)NIP_CARDINALITY(vars[i]) * sizeof(double));
      out[ids[b]] = u;
      if (ll) ll[ids[b]] = l[b];
    }
    if (rc != NIP_NO_ERROR) break;
  }
  if (rc != NIP_NO_ERROR)
    for (int s = 0; s < n; s++) {
      free_uncertainseries(out[s]);
      out[s] = nullptr;
    }
  return rc;
}

}  // namespace

extern "C" {

/* ---- niperrorhandler (src/niperrorhandler.c:27-69) ---- */

static int g_error_counter = 0;
static int g_error_code = 0;

int nip_report_error(char* srcFile, int line, int error, int verbose) {
  g_error_code = error;
  g_error_counter++;
  if (verbose) {
    std::fprintf(stderr, "In %s (%d): ", srcFile, line);
    switch (error) {
      case 0: std::fprintf(stderr, "O.K.\n"); break;
      case EFAULT: std::fprintf(stderr, "Nullpointer given.\n"); break;
      case EDOM: std::fprintf(stderr, "Argument outside the defined domain.\n"); break;
      case EINVAL: std::fprintf(stderr, "Invalid argument given.\n"); break;
      case ENOMEM: std::fprintf(stderr, "Failed to allocate memory.\n"); break;
      case EIO: std::fprintf(stderr, "I/O failure.\n"); break;
      case ENOENT: std::fprintf(stderr, "Requested file not found.\n"); break;
      default: std::fprintf(stderr, "Something went wrong.\n");
    }
  }
  return error;
}

void nip_reset_error_handler(void) { g_error_code = g_error_counter = 0; }
int nip_check_error_type(void) { return g_error_code; }
int nip_check_error_counter(void) { return g_error_counter; }

/* ---- models (src/nip.c:122-508, 1584-1597, 2523-2553) ---- */

namespace {
char* copy_text(const std::string& s) {
  char* r = (char*)std::malloc(s.size() + 1);
  if (r) std::memcpy(r, s.c_str(), s.size() + 1);
  return r;
}

void free_compat(Compat* c) {
  for (nip_clique q : c->cliques) nip_free_clique(q);   // frees the sepsets too
  for (auto& v : c->vars) {
    std::free(v.symbol);
    std::free(v.name);
    if (v.state_names)
      for (int s = 0; s < v.cardinality; s++) std::free(v.state_names[s]);
    std::free(v.state_names);
    std::free(v.likelihood);
    std::free(v.prior);
    std::free(v.parents);
    std::free(v.family_mapping);
  }
  if (c->eng) nipamd_model_free(c->eng);
  delete c;
}

// the join tree of the compiled model as the reference's structs: clique c
// holds its variables in ascending ID order and p = original_p = the
// compiled CPT product (nip_init_clique into both, nipjointree.c:713-772);
// sepsets start as ones (nipjointree.c:265-325) and are linked into each
// clique's list in the compiled list order
int build_join_tree(Compat* c) {
  nipamd_model* e = c->eng;
  const int nc = nipamd_model_num_cliques(e), ns = nipamd_model_num_sepsets(e);
  const int nv = (int)c->vars.size();
  std::vector<int> vars(nv + 1), links(ns + 1);
  std::vector<std::vector<int>> clinks(nc);
  for (int k = 0; k < nc; k++) {
    int n = 0, nl = 0;
    nipamd_model_clique(e, k, vars.data(), &n, links.data(), &nl);
    std::vector<nip_variable> vs(n > 0 ? n : 1);
    for (int i = 0; i < n; i++) vs[i] = &c->vars[vars[i]];
    nip_clique q = nip_new_clique(vs.data(), n);
    if (!q) return NIP_ERROR_OUTOFMEMORY;
    c->cliques.push_back(q);
    nipamd_model_original(e, k, q->original_p->data, q->original_p->size_of_data);
    std::memcpy(q->p->data, q->original_p->data, sizeof(double) * q->p->size_of_data);
    c->eng_orig.emplace_back(q->original_p->data, q->original_p->data + q->original_p->size_of_data);
    clinks[k].assign(links.begin(), links.begin() + nl);
  }
  for (int s = 0; s < ns; s++) {
    int a = -1, b = -1, n = 0;
    nipamd_model_sepset(e, s, &a, &b, vars.data(), &n);
    nip_sepset q = nip_new_sepset(c->cliques[a], c->cliques[b]);
    if (!q) return NIP_ERROR_OUTOFMEMORY;
    c->sepsets.push_back(q);
  }
  for (int k = 0; k < nc; k++) {   // the list order of each clique, front to back
    nip_sepset_link prev = nullptr;
    for (int s : clinks[k]) {
      auto* l = (nip_sepset_link)std::malloc(sizeof(nip_sepsetlink_struct));
      if (!l) return NIP_ERROR_OUTOFMEMORY;
      l->data = c->sepsets[s];
      l->fwd = nullptr;
      l->bwd = prev;
      if (prev) prev->fwd = l; else c->cliques[k]->sepsets = l;
      prev = l;
    }
    c->cliques[k]->num_of_sepsets = (int)clinks[k].size();
  }
  return NIP_NO_ERROR;
}
}  // namespace

nip_model parse_model(char* file) {
  nipamd_model* e = nullptr;
  if (!file || nipamd_model_from_net(file, &e) != NIP_NO_ERROR) {
    std::fprintf(stderr, "nip_amd: %s\n", nipamd_last_error());
    REPORT(NIP_ERROR_GENERAL);
    return nullptr;
  }
  auto* c = new Compat;
  c->eng = e;
  const int n = nipamd_model_num_vars(e);
  c->id0 = nipamd_compat_take_ids(n);   // the parser numbers variables from the global counter
  c->vars.assign(n, nip_variable_struct{});
  c->eng_prior.resize(n);
  std::vector<std::array<int, 9>> info(n);
  std::vector<std::vector<int>> par(n);
  char buf[4096];
  bool ok = true;
  for (int i = 0; i < n && ok; i++) {
    nip_variable_struct& v = c->vars[i];
    const int np = nipamd_model_var_info(e, i, info[i].data(), nullptr, 0);
    par[i].resize(np);
    nipamd_model_var_info(e, i, info[i].data(), par[i].data(), np);
    const int card = info[i][0];
    v.id = c->id0 + (unsigned long)i;
    nipamd_model_var_symbol(e, i, buf, sizeof buf);
    v.symbol = copy_text(buf);
    nipamd_model_var_label(e, i, buf, sizeof buf);
    v.name = copy_text(buf);
    v.cardinality = card;
    v.state_names = (char**)std::calloc(card > 0 ? card : 1, sizeof(char*));
    v.likelihood = (double*)std::malloc(sizeof(double) * (card > 0 ? card : 1));
    ok = v.symbol && v.name && v.state_names && v.likelihood;
    for (int s = 0; ok && s < card; s++) {
      nipamd_model_state_name(e, i, s, buf, sizeof buf);
      ok = (v.state_names[s] = copy_text(buf)) != nullptr;
      v.likelihood[s] = 1.0;
    }
    if (ok && np == 0) {   // nip.c:175-180: a missing prior reads as zeros
      v.prior = (double*)std::calloc(card > 0 ? card : 1, sizeof(double));
      ok = v.prior != nullptr;
      if (ok) nipamd_model_prior(e, i, v.prior);
      if (ok) c->eng_prior[i].assign(v.prior, v.prior + card);
    }
  }
  for (int i = 0; i < n && ok; i++) {
    nip_variable_struct& v = c->vars[i];
    v.prior_entered = 0;
    v.next = info[i][1] >= 0 ? &c->vars[info[i][1]] : nullptr;
    v.previous = info[i][2] >= 0 ? &c->vars[info[i][2]] : nullptr;
    v.num_of_parents = (int)par[i].size();
    if (!par[i].empty()) {
      v.parents = (nip_variable*)std::calloc(par[i].size(), sizeof(nip_variable));
      if (!(ok = v.parents != nullptr)) break;
      for (size_t j = 0; j < par[i].size(); j++) v.parents[j] = &c->vars[par[i][j]];
    }
    v.family_clique = nullptr;
    v.family_mapping = nullptr;
    v.interface_status = info[i][3];
    v.mark = NIP_MARK_OFF;
    v.pos_x = info[i][4];
    v.pos_y = info[i][5];
    c->all.push_back(&v);
  }
  if (ok) ok = build_join_tree(c) == NIP_NO_ERROR;
  if (!ok) {
    REPORT(NIP_ERROR_OUTOFMEMORY);
    free_compat(c);
    return nullptr;
  }
  // the special-purpose arrays of nip.c:216-247
  for (int i = 0; i < n; i++) {
    nip_variable v = &c->vars[i];
    if (v->next) {
      c->next.push_back(v);
      c->previous.push_back(v->next);
    }
    if (v->interface_status & NIP_INTERFACE_INCOMING) c->incoming.push_back(v);
    if (v->interface_status & NIP_INTERFACE_OLD_OUTGOING) {
      c->prev_outgoing.push_back(v);
      c->outgoing.push_back(v->next);
    }
    (v->parents ? c->children : c->independent).push_back(v);
  }
  int in_c = -1, out_c = -1;
  nipamd_model_interface_cliques(e, &in_c, &out_c);
  nip_model_struct& m = c->pub;
  m.num_of_cliques = (int)c->cliques.size();
  m.cliques = c->cliques.data();
  m.num_of_vars = n;
  m.variables = c->all.data();
  m.num_of_nexts = (int)c->next.size();
  m.next = c->next.data();
  m.previous = c->previous.data();
  m.outgoing_interface_size = (int)c->outgoing.size();
  m.outgoing_interface = c->outgoing.data();
  m.previous_outgoing_interface = c->prev_outgoing.data();
  m.incoming_interface_size = (int)c->incoming.size();
  m.incoming_interface = c->incoming.data();
  m.in_clique = in_c >= 0 ? c->cliques[in_c] : nullptr;
  m.out_clique = out_c >= 0 ? c->cliques[out_c] : nullptr;
  m.num_of_children = (int)c->children.size();
  m.children = c->children.data();
  m.independent = c->independent.data();
  m.node_size_x = n > 0 ? info[0][7] : 80;
  m.node_size_y = n > 0 ? info[0][8] : 60;
  g_models[&c->pub] = c;
  return &c->pub;
}

void free_model(nip_model model) {
  Compat* c = lookup(model);
  if (!c) return;
  g_models.erase(model);
  free_compat(c);
}

int write_model(nip_model model, char* filename) {
  Compat* c = lookup(model);
  if (!c || !filename) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  if (int e = sync_engine(c)) {
    engine_error(e);
    return e;
  }
  const int e = nipamd_write_model(c->eng, filename);
  if (e != NIP_NO_ERROR) engine_error(e);
  return e;
}

nip_variable model_variable(nip_model model, char* symbol) {
  if (!model) {
    REPORT(NIP_ERROR_NULLPOINTER);
    return nullptr;
  }
  for (int i = 0; i < model->num_of_vars; i++)
    if (std::strcmp(symbol, model->variables[i]->symbol) == 0) return model->variables[i];
  return nullptr;
}

// every clique with its belief, then its sepsets in list order with their
// latest messages (nip.c:2523-2553)
void print_cliques(nip_model model) {
  if (!model) {
    REPORT(NIP_ERROR_NULLPOINTER);
    return;
  }
  std::printf("Cliques of the model:\n");
  for (int i = 0; i < model->num_of_cliques; i++) {
    nip_clique c = model->cliques[i];
    nip_fprintf_clique(stdout, c);
    nip_fprintf_potential(stdout, c->p);
    for (nip_sepset_link l = c->sepsets; l; l = l->fwd) {
      auto* s = (nip_sepset)l->data;
      nip_fprintf_sepset(stdout, s);
      nip_fprintf_potential(stdout, s->new_);
    }
    std::printf("\n");
  }
}

/* ---- time series (src/nip.c:512-931) ---- */

int read_timeseries(nip_model model, char* datafile, time_series** results) {
  Compat* c = lookup(model);
  if (!c || !datafile || !results) {
    REPORT(NIP_ERROR_INVALID_ARGUMENT);
    return 0;
  }
  nipamd_series* s = nullptr;
  if (nipamd_read_timeseries(c->eng, datafile, &s) != NIP_NO_ERROR) {
    std::fprintf(stderr, "nip_amd: %s\n", nipamd_last_error());
    REPORT(NIP_ERROR_IO);
    return 0;
  }
  const int N = nipamd_series_count(s), k = nipamd_series_num_observed(s), n = model->num_of_vars;
  std::vector<int> ov(k > 0 ? k : 1);
  nipamd_series_observed(s, ov.data());
  *results = (time_series*)std::calloc(N > 0 ? N : 1, sizeof(time_series));
  bool ok = *results != nullptr;
  for (int i = 0; ok && i < N; i++) {
    auto* ts = (time_series)std::calloc(1, sizeof(time_series_struct));
    if (!(ok = ts != nullptr)) break;
    (*results)[i] = ts;
    ts->model = model;
    ts->length = nipamd_series_length(s, i);
    ts->num_of_observed = k;
    ts->num_of_hidden = n - k;
    ts->hidden = (nip_variable*)std::calloc(n - k > 0 ? n - k : 1, sizeof(nip_variable));
    ts->observed = k > 0 ? (nip_variable*)std::calloc(k, sizeof(nip_variable)) : nullptr;
    if (!(ok = ts->hidden && (k == 0 || ts->observed))) break;
    int h = 0;
    for (int v = 0; v < n; v++) {  // nip.c:578-589: model order
      bool seen = false;
      for (int j = 0; j < k; j++) seen |= ov[j] == v;
      if (!seen) ts->hidden[h++] = model->variables[v];
    }
    for (int j = 0; j < k; j++) ts->observed[j] = model->variables[ov[j]];
    if (k > 0) {
      ts->data = (int**)std::calloc(ts->length > 0 ? ts->length : 1, sizeof(int*));
      if (!(ok = ts->data != nullptr)) break;
      const int32_t* d = nipamd_series_data(s, i);
      for (int t = 0; ok && t < ts->length; t++) {
        if (!(ok = (ts->data[t] = (int*)std::calloc(k, sizeof(int))) != nullptr)) break;
        for (int j = 0; j < k; j++) ts->data[t][j] = d[(size_t)t * k + j];
      }
    }
  }
  nipamd_series_free(s);
  if (!ok) {
    REPORT(NIP_ERROR_OUTOFMEMORY);
    if (*results)
      for (int i = 0; i < N; i++) free_timeseries((*results)[i]);
    std::free(*results);
    *results = nullptr;
    return 0;
  }
  return N;
}

int write_timeseries(time_series* ts_set, int n_series, char* filename) {
  if (!(n_series > 0 && ts_set && filename)) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  nip_model model = ts_set[0]->model;
  for (int n = 1; n < n_series; n++)
    if (ts_set[n]->model != model) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  // union of the observed variables in first-seen order (nip_variable_union)
  std::vector<nip_variable> obs;
  for (int n = 0; n < n_series; n++)
    for (int i = 0; i < ts_set[n]->num_of_observed; i++) {
      bool seen = false;
      for (nip_variable v : obs) seen |= nip_equal_variables(v, ts_set[n]->observed[i]) != 0;
      if (!seen) obs.push_back(ts_set[n]->observed[i]);
    }
  if (obs.empty()) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  FILE* f = std::fopen(filename, "w");
  if (!f) return REPORT(NIP_ERROR_IO);
  for (size_t i = 0; i < obs.size(); i++) {
    if (i) std::fprintf(f, "%c", NIP_FIELD_SEPARATOR);
    std::fprintf(f, "%s", nip_variable_symbol(obs[i]));
  }
  std::fputs("\n", f);
  std::vector<int> rec(obs.size()), map;
  for (int n = 0; n < n_series; n++) {
    const time_series ts = ts_set[n];
    map.assign(ts->num_of_observed, 0);
    for (int i = 0; i < ts->num_of_observed; i++)
      for (size_t j = 0; j < obs.size(); j++)
        if (nip_equal_variables(obs[j], ts->observed[i])) map[i] = (int)j;
    for (int t = 0; t < ts->length; t++) {
      std::fill(rec.begin(), rec.end(), -1);
      for (int i = 0; i < ts->num_of_observed; i++) rec[map[i]] = ts->data[t][i];
      for (size_t i = 0; i < obs.size(); i++) {
        if (i) std::fprintf(f, "%c", NIP_FIELD_SEPARATOR);
        if (rec[i] >= 0) std::fprintf(f, "%s", nip_variable_state_name(obs[i], rec[i]));
        else std::fputs("null", f);
      }
      std::fputs("\n", f);
    }
    std::fputs("\n", f);
  }
  if (std::fclose(f)) return REPORT(NIP_ERROR_IO);
  return NIP_NO_ERROR;
}

void free_timeseries(time_series ts) {
  if (!ts) return;
  if (ts->data) {
    for (int t = 0; t < ts->length; t++) std::free(ts->data[t]);
    std::free(ts->data);
  }
  std::free(ts->hidden);
  std::free(ts->observed);
  std::free(ts);
}

int timeseries_length(time_series ts) { return ts ? ts->length : 0; }

char* get_observation(time_series ts, nip_variable v, int time) {
  int j = -1;
  for (int i = 0; i < ts->model->num_of_vars - ts->num_of_hidden; i++)
    if (nip_equal_variables(v, ts->observed[i])) j = i;
  if (j < 0 || time < 0 || ts->length <= time) return nullptr;
  return v->state_names[ts->data[time][j]];
}

int set_observation(time_series ts, nip_variable v, int time, char* observation) {
  int j = -1;
  for (int i = 0; i < ts->model->num_of_vars - ts->num_of_hidden; i++)
    if (nip_equal_variables(v, ts->observed[i])) j = i;
  const int i = nip_variable_state_index(v, observation);
  if (j < 0 || i < 0) return NIP_ERROR_INVALID_ARGUMENT;
  ts->data[time][j] = i;
  return 0;
}

int write_uncertainseries(uncertain_series* ucs_set, int n_series, nip_variable v, char* filename) {
  const int n = v ? NIP_CARDINALITY(v) : 0;
  if (!(n > 0 && ucs_set && filename && n_series > 0)) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  std::vector<int> vi(n_series, -1);
  for (int s = 0; s < n_series; s++) {
    for (int i = 0; i < ucs_set[s]->num_of_vars; i++)
      if (nip_equal_variables(v, ucs_set[s]->variables[i])) {
        vi[s] = i;
        break;
      }
    if (vi[s] < 0) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  }
  FILE* f = std::fopen(filename, "w");
  if (!f) return REPORT(NIP_ERROR_IO);
  for (int i = 0; i < n; i++) {
    if (i) std::fprintf(f, "%c", NIP_FIELD_SEPARATOR);
    std::fprintf(f, "%s", nip_variable_state_name(v, i));
  }
  std::fputs("\n", f);
  for (int s = 0; s < n_series; s++) {
    const uncertain_series u = ucs_set[s];
    for (int t = 0; t < u->length; t++) {
      for (int i = 0; i < n; i++) {
        if (i) std::fprintf(f, "%c", NIP_FIELD_SEPARATOR);
        std::fprintf(f, "%f", u->data[t][vi[s]][i]);
      }
      std::fputs("\n", f);
    }
    std::fputs("\n", f);
  }
  if (std::fclose(f)) return REPORT(NIP_ERROR_IO);
  return NIP_NO_ERROR;
}

void free_uncertainseries(uncertain_series ucs) {
  if (!ucs) return;
  if (ucs->data) {
    for (int t = 0; t < ucs->length; t++) {
      if (!ucs->data[t]) continue;
      for (int i = 0; i < ucs->num_of_vars; i++) std::free(ucs->data[t][i]);
      std::free(ucs->data[t]);
    }
    std::free(ucs->data);
  }
  std::free(ucs->variables);
  std::free(ucs);
}

int uncertainseries_length(uncertain_series ucs) { return ucs ? ucs->length : 0; }

/* ---- inference and learning on the engine ---- */

uncertain_series forward_inference(time_series ts, nip_variable vars[], int nvars,
                                   double* loglikelihood) {
  uncertain_series u = nullptr;
  const int e = run_inference(&ts, 1, vars, nvars, true, &u, loglikelihood);
  if (e != NIP_NO_ERROR) engine_error(e);
  return u;
}

uncertain_series forward_backward_inference(time_series ts, nip_variable vars[], int nvars,
                                            double* loglikelihood) {
  uncertain_series u = nullptr;
  const int e = run_inference(&ts, 1, vars, nvars, false, &u, loglikelihood);
  if (e != NIP_NO_ERROR) engine_error(e);
  return u;
}

int forward_backward_inference_batch(time_series* ts, int n_ts, nip_variable vars[], int nvars,
                                     uncertain_series* ucs_out, double* ll_out) {
  const int e = run_inference(ts, n_ts, vars, nvars, false, ucs_out, ll_out);
  if (e != NIP_NO_ERROR) engine_error(e);
  return e;
}

int em_learn(time_series* ts, int n_ts, double threshold, nip_double_list learning_curve) {
  if (!ts || n_ts < 1 || !ts[0] || !ts[0]->model) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  Compat* c = lookup(ts[0]->model);
  if (!c) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  if (int e = sync_engine(c)) {
    engine_error(e);
    return e;
  }
  if (learning_curve && NIP_LIST_LENGTH(learning_curve) > 0) nip_empty_double_list(learning_curve);
  std::vector<int> col, var, ov;
  marked_columns(ts[0], c, col, ov);
  std::vector<int> lengths(n_ts);
  size_t total = 0;
  for (int s = 0; s < n_ts; s++) {
    if (!ts[s] || ts[s]->model != ts[0]->model) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
    marked_columns(ts[s], c, col, var);
    if (var != ov) {
      std::fprintf(stderr, "nip_amd: em_learn needs the same observed variables in every series\n");
      return REPORT(NIP_ERROR_INVALID_ARGUMENT);
    }
    total += (size_t)(lengths[s] = ts[s]->length);
  }
  const int k = (int)ov.size();
  std::vector<int32_t> obs(total * (k > 0 ? k : 1) + 1, -1);
  size_t r = 0;
  for (int s = 0; s < n_ts; s++) {
    marked_columns(ts[s], c, col, var);
    for (int t = 0; t < ts[s]->length; t++, r++)
      for (int i = 0; i < k; i++) obs[r * k + i] = ts[s]->data[t][col[i]];
  }
  std::vector<double> curve(1 << 16);
  int curve_len = 0;
  // the random start from the caller's stream, rand()/RAND_MAX per parameter
  // in the em_learn layout (nip_random_potential per variable, nip.c:2135-2138)
  std::vector<double> init(nipamd_model_param_size(c->eng) + 1);
  for (size_t i = 0; i + 1 < init.size(); i++) init[i] = std::rand() / (double)RAND_MAX;
  int e;
  {
    RandGuard guard;
    e = nipamd_em_learn(c->eng, n_ts, lengths.data(), obs.data(), k, ov.data(), threshold,
                        init.data(), 0, curve.data(), (int)curve.size(), &curve_len);
  }
  pull_engine(c);
  if (e != NIP_NO_ERROR && e != NIP_ERROR_BAD_LUCK) {
    engine_error(e);
    return e;
  }
  // on BAD_LUCK the curve so far stays (nip.c:2192-2198)
  for (int i = 0; learning_curve && i < curve_len && i < (int)curve.size(); i++) {
    const int a = nip_append_double(learning_curve, curve[i]);
    if (a != NIP_NO_ERROR) return a;
  }
  return e;
}

/* generate_data (src/nip.c:2325-2478) on the engine: the rand() draws come
 * from the caller's own stream, one per variable per step in sampling order,
 * exactly as the reference consumes them; the sampling is the GPU's.  The
 * result's observed variables are the sampling order (nip.c:2384-2389) and
 * every variable ends up marked (nip.c:2343-2375). */
time_series generate_data(nip_model model, int length) {
  Compat* c = lookup(model);
  if (!c || length < 0) {
    REPORT(NIP_ERROR_INVALID_ARGUMENT);
    return nullptr;
  }
  if (int e = sync_engine(c)) {
    engine_error(e);
    return nullptr;
  }
  const int nv = nipamd_generate_order(c->eng, nullptr);
  std::vector<int> order(nv > 0 ? nv : 1);
  nipamd_generate_order(c->eng, order.data());
  std::vector<int32_t> draws((size_t)length * nv + 1), out((size_t)length * nv + 1);
  for (size_t i = 0; i + 1 < draws.size(); i++) draws[i] = std::rand();
  int e;
  {
    RandGuard guard;
    e = nipamd_generate_host_draws(c->eng, 1, length, draws.data(), out.data());
  }
  if (e != NIP_NO_ERROR) {
    engine_error(e);
    return nullptr;
  }
  for (int i = 0; i < model->num_of_vars; i++) nip_mark_variable(model->variables[i]);
  auto* ts = (time_series)std::calloc(1, sizeof(time_series_struct));
  if (!ts) {
    REPORT(NIP_ERROR_OUTOFMEMORY);
    return nullptr;
  }
  ts->model = model;
  ts->hidden = nullptr;
  ts->num_of_hidden = model->num_of_vars - nv;
  ts->num_of_observed = nv;
  ts->length = length;
  ts->observed = (nip_variable*)std::calloc(nv > 0 ? nv : 1, sizeof(nip_variable));
  ts->data = (int**)std::calloc(length > 0 ? length : 1, sizeof(int*));
  bool ok = ts->observed && ts->data;
  for (int i = 0; ok && i < nv; i++) ts->observed[i] = model->variables[order[i]];
  for (int t = 0; ok && t < length; t++) {
    ok = (ts->data[t] = (int*)std::calloc(nv > 0 ? nv : 1, sizeof(int))) != nullptr;
    for (int i = 0; ok && i < nv; i++) ts->data[t][i] = out[(size_t)t * nv + i];
  }
  if (!ok) {
    REPORT(NIP_ERROR_OUTOFMEMORY);
    free_timeseries(ts);
    return nullptr;
  }
  return ts;
}

/* ---- the single-slice state (src/nip.c:61-119, 951-1027, 1600-1617,
 *      2254-2321): the reference's bookkeeping over the host join tree;
 *      make_consistent propagates on the GPU ---- */

void reset_model(nip_model model) {
  for (int i = 0; i < model->num_of_vars; i++) {
    nip_variable v = model->variables[i];
    nip_reset_likelihood(v);
    v->prior_entered = 0;
  }
  if (nip_global_retraction(model->variables, model->num_of_vars, model->cliques,
                            model->num_of_cliques) != NIP_NO_ERROR)
    REPORT(NIP_ERROR_GENERAL);
}

void total_reset(nip_model model) {
  for (int i = 0; i < model->num_of_cliques; i++) nip_uniform_potential(model->cliques[i]->original_p, 1.0);
  reset_model(model);
}

// priors of the independent variables, once each; with has_history the
// previous slice's interface variables get none (nip.c:88-119)
void use_priors(nip_model model, int has_history) {
  for (int i = 0; i < model->num_of_vars - model->num_of_children; i++) {
    nip_variable v = model->independent[i];
    if (v->prior_entered) continue;
    if (has_history && (v->interface_status & NIP_INTERFACE_OLD_OUTGOING)) continue;
    if (nip_enter_prior(model->variables, model->num_of_vars, model->cliques, model->num_of_cliques,
                        v, v->prior) != NIP_NO_ERROR)
      REPORT(NIP_ERROR_GENERAL);
    v->prior_entered = 1;
  }
}

void make_consistent(nip_model model) {
  if (nipamd_compat_make_consistent(model->cliques, model->num_of_cliques) != NIP_NO_ERROR)
    REPORT(NIP_ERROR_GENERAL);
}

int insert_hard_evidence(nip_model model, char* varname, char* observation) {
  nip_variable v = model_variable(model, varname);
  if (!v) return NIP_ERROR_INVALID_ARGUMENT;
  const int ret = nip_enter_observation(model->variables, model->num_of_vars, model->cliques,
                                        model->num_of_cliques, v, observation);
  if (ret != NIP_NO_ERROR) REPORT(NIP_ERROR_GENERAL);
  make_consistent(model);
  return ret;
}

int insert_soft_evidence(nip_model model, char* varname, double* distribution) {
  nip_variable v = model_variable(model, varname);
  if (!v) return NIP_ERROR_INVALID_ARGUMENT;
  const int ret = nip_enter_evidence(model->variables, model->num_of_vars, model->cliques,
                                     model->num_of_cliques, v, distribution);
  make_consistent(model);
  return ret;
}

// the observations of step t whose variables' marks match mark_mask;
// missing values (< 0) are skipped (nip.c:982-1001)
int insert_ts_step(time_series ts, int t, nip_model model, char mark_mask) {
  if (t < 0 || t >= timeseries_length(ts)) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  for (int i = 0; i < ts->model->num_of_vars - ts->num_of_hidden; i++) {
    nip_variable v = ts->observed[i];
    if ((NIP_MARK(v) & mark_mask) && ts->data[t][i] >= 0)
      nip_enter_index_observation(model->variables, model->num_of_vars, model->cliques,
                                  model->num_of_cliques, v, ts->data[t][i]);
  }
  return NIP_NO_ERROR;
}

int insert_ucs_step(uncertain_series ucs, int t, nip_model model, char mark_mask) {
  if (t < 0 || t >= uncertainseries_length(ucs)) return REPORT(NIP_ERROR_INVALID_ARGUMENT);
  for (int i = 0; i < ucs->num_of_vars; i++) {
    nip_variable v = ucs->variables[i];
    if (!(NIP_MARK(v) & mark_mask)) continue;
    const int e = nip_enter_evidence(model->variables, model->num_of_vars, model->cliques,
                                     model->num_of_cliques, v, ucs->data[t][i]);
    if (e != NIP_NO_ERROR) return REPORT(e);
  }
  return NIP_NO_ERROR;
}

double model_prob_mass(nip_model model) {
  return nip_probability_mass(model->cliques, model->num_of_cliques);
}

double* get_probability(nip_model model, nip_variable v) {
  if (!model || !v) {
    REPORT(NIP_ERROR_NULLPOINTER);
    return nullptr;
  }
  const int card = NIP_CARDINALITY(v);
  auto* r = (double*)std::calloc(card > 0 ? card : 1, sizeof(double));
  if (!r) {
    REPORT(NIP_ERROR_OUTOFMEMORY);
    return nullptr;
  }
  nip_clique c = nip_find_family(model->cliques, model->num_of_cliques, v);
  if (!c) {
    REPORT(NIP_ERROR_GENERAL);
    std::free(r);
    return nullptr;
  }
  nip_marginalise_clique(c, v, r);
  nip_normalise_array(r, card);
  return r;
}

nip_potential get_joint_probability(nip_model model, nip_variable* vars, int num_of_vars) {
  for (int i = 0; i < model->num_of_cliques; i++) nip_unmark_clique(model->cliques[i]);
  nip_potential p = nip_gather_joint_probability(model->cliques[0], vars, num_of_vars, nullptr, 0);
  if (!p) {
    REPORT(NIP_ERROR_GENERAL);
    return nullptr;
  }
  nip_normalise_potential(p);
  return p;
}

/* ---- random numbers (src/nip.c:2482-2520) ---- */

long random_seed(long* seedpointer) {
  long seed;
  if (!seedpointer) {
    const time_t now = std::time(nullptr);
    const struct tm* tp = std::localtime(&now);
    seed = tp->tm_sec + 60 * tp->tm_min + 3600 * tp->tm_hour;
    seed ^= (getpid() + (getpid() << 15));
  } else {
    seed = *seedpointer;
  }
  std::srand((unsigned)seed);
  return seed;
}

int lottery(double* distribution, int size) {
  int i = 0;
  double sum = 0;
  const double r = std::rand() / (double)RAND_MAX;
  do {
    if (i >= size) {
      REPORT(NIP_ERROR_INVALID_ARGUMENT);
      return size - 1;
    }
    sum += distribution[i++];
  } while (sum < r);
  return i - 1;
}

}  // extern "C"
