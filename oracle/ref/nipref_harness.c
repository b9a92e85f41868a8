/*
 * nipref_harness.c -- TEST INFRASTRUCTURE ONLY (oracle).
 *
 * Builds NIP models through the reference's OWN compiled code
 * (/root/reference/src: nipvariable.c, nippotential.c, nipjointree.c,
 * nipgraph.c, nipheap.c, niplists.c, nipstring.c, niperrorhandler.c, built
 * unmodified by oracle/Makefile into oracle/_ref/) and runs the reference's
 * time-slice algorithms on top of them.
 *
 * Two reference pieces cannot be built here and are RESTATED below instead:
 *   - src/huginnet.y (bison is absent): its grammar actions are replayed in
 *     file order from a token stream produced by oracle/netfile.py;
 *   - src/nip.c (needs the generated huginnet.tab.h and the NIP_ERROR_* codes
 *     that are defined nowhere in the tree): the top-level loops that sit on
 *     the hot path are restated here, each citing the nip.c lines it follows.
 * Everything below those loops -- potential algebra, Hugin propagation,
 * evidence entry, retraction, probability mass, graph compilation -- is the
 * reference's own code.
 *
 * Nothing in the product (nip_amd/) links or calls this file.  It is used to
 * generate the golden fixtures under tests/golden/ and, on the GPU box, as the
 * "reference" CPU baseline timed by bench.py.
 *
 * ABI (ctypes):
 *   int  nh_build(const char* replay)            -> model handle (>=0) or -1
 *   int  nh_desc(int h, char* buf, int cap)      -> JSON join-tree description
 *   int  nh_fb(...), nh_filter(...), nh_estep(...), nh_em(...)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <assert.h>

#include "niperrorhandler.h"
#include "niplists.h"
#include "nipvariable.h"
#include "nippotential.h"
#include "nipjointree.h"
#include "nipgraph.h"

#define NH_MAX_MODELS 65536

/* Layout-compatible subset of nip_model_struct (src/nip.h:71-104); only the
 * harness reads it, so it is declared locally instead of pulling in nip.h
 * (whose prototypes refer to the unbuildable nip.c). */
typedef struct {
  int num_of_cliques;
  nip_clique* cliques;
  int num_of_vars;
  nip_variable* variables;
  int num_of_nexts;
  nip_variable* next;
  nip_variable* previous;
  int outgoing_interface_size;
  nip_variable* outgoing_interface;
  nip_variable* previous_outgoing_interface;
  int incoming_interface_size;
  nip_variable* incoming_interface;
  nip_clique in_clique;
  nip_clique out_clique;
  int num_of_children;
  nip_variable* children;
  nip_variable* independent;
  /* harness-only bookkeeping */
  int n_sepsets;
  nip_sepset* sepsets;          /* in nip_confirm_sepset order */
} nh_model;

static nh_model* nh_models[NH_MAX_MODELS];
static int nh_n_models = 0;

/* ------------------------------------------------------------------ */
/* token reader for the replay stream                                  */
/* ------------------------------------------------------------------ */
typedef struct { const char* s; } nh_tok;

static int nh_next(nh_tok* t, char* out, int cap){
  int n = 0;
  while(*t->s == ' ' || *t->s == '\n' || *t->s == '\t' || *t->s == '\r') t->s++;
  if(!*t->s) return 0;
  while(*t->s && *t->s != ' ' && *t->s != '\n' && *t->s != '\t' && *t->s != '\r'){
    if(n < cap - 1) out[n++] = *t->s;
    t->s++;
  }
  out[n] = 0;
  return 1;
}

static int nh_int(nh_tok* t){ char b[64]; if(!nh_next(t, b, 64)) return -1; return atoi(b); }
static double nh_dbl(nh_tok* t){ char b[64]; nh_next(t, b, 64); return strtod(b, NULL); }

static int nh_var_index(nh_model* m, nip_variable v){
  int i;
  for(i = 0; i < m->num_of_vars; i++) if(m->variables[i] == v) return i;
  return -1;
}

static int nh_clique_index(nh_model* m, nip_clique c){
  int i;
  for(i = 0; i < m->num_of_cliques; i++) if(m->cliques[i] == c) return i;
  return -1;
}

/* ------------------------------------------------------------------ */
/* Replay of the huginnet.y grammar actions                            */
/* ------------------------------------------------------------------ */
typedef struct {
  nip_potential p;
  nip_variable child;
  nip_variable* parents;   /* reversed file order, as the grammar builds it */
  int nparents;
} nh_parsed_pot;

/* interface_to_vars, restated from src/huginnet.y:1155-1254 */
static void nh_interface_to_vars(nip_variable* vars, int n, const int* next){
  int i, k, m;
  for(i = 0; i < n; i++){
    if(next[i] >= 0){
      vars[i]->next = vars[next[i]];            /* huginnet.y:1186-1187 */
      vars[next[i]]->previous = vars[i];
    }
  }
  for(k = 0; k < n; k++){                        /* huginnet.y:1206-1251 */
    nip_variable v2 = vars[k];
    m = 0;
    for(i = 0; i < nip_number_of_parents(v2); i++){
      nip_variable v1 = v2->parents[i];
      if(v1->next != NULL){
        v1->interface_status |= NIP_INTERFACE_OLD_OUTGOING;
        v1->next->interface_status |= NIP_INTERFACE_OUTGOING;
        v2->interface_status |= NIP_INTERFACE_INCOMING;
        m = 1;
      }
    }
    if(m){
      for(i = 0; i < nip_number_of_parents(v2); i++){
        nip_variable v1 = v2->parents[i];
        if(v1->next == NULL)
          v1->interface_status |= NIP_INTERFACE_INCOMING;
      }
    }
  }
}

/*
 * Replay stream:
 *   V <n>  then n lines  "<symbol> <card> <next-index|-1>"
 *   P <np> then np lines "<child> <k> <parent_1..parent_k (file order)> <nd> <d_0..d_nd-1>"
 * (indices are positions in the node list).
 */
int nh_build(const char* replay){
  nh_tok t; char tok[256];
  int n, np, i, j, k;
  int* next;
  nip_variable* vars;
  nh_parsed_pot* pots;
  nip_graph g;
  nh_model* m;
  int nc;

  if(nh_n_models >= NH_MAX_MODELS) return -1;
  t.s = replay;
  nh_next(&t, tok, 256); if(strcmp(tok, "V")) return -1;
  n = nh_int(&t);
  vars = (nip_variable*) calloc(n, sizeof(nip_variable));
  next = (int*) calloc(n, sizeof(int));
  for(i = 0; i < n; i++){
    char sym[256]; int card;
    char** states;
    nh_next(&t, sym, 256);
    card = nh_int(&t);
    next[i] = nh_int(&t);
    states = (char**) calloc(card, sizeof(char*));
    for(j = 0; j < card; j++){ states[j] = (char*) malloc(16); snprintf(states[j], 16, "%d", j); }
    /* nodeDeclaration action, huginnet.y:321-387: ids follow file order */
    vars[i] = nip_new_variable(sym, sym, states, card);
    for(j = 0; j < card; j++) free(states[j]);
    free(states);
  }

  nh_next(&t, tok, 256); if(strcmp(tok, "P")) return -1;
  np = nh_int(&t);
  pots = (nh_parsed_pot*) calloc(np, sizeof(nh_parsed_pot));
  for(i = 0; i < np; i++){
    int child = nh_int(&t);
    int kp = nh_int(&t);
    int nd;
    double* data = NULL;
    nip_variable* family = (nip_variable*) calloc(kp + 1, sizeof(nip_variable));
    int* fpar = (int*) calloc(kp > 0 ? kp : 1, sizeof(int));
    for(j = 0; j < kp; j++) fpar[j] = nh_int(&t);
    nd = nh_int(&t);
    if(nd > 0){
      data = (double*) calloc(nd, sizeof(double));
      for(j = 0; j < nd; j++) data[j] = nh_dbl(&t);
    }
    pots[i].child = vars[child];
    pots[i].nparents = kp;
    if(kp > 0){
      /* the 'symbol' rule prepends (huginnet.y:753-766): parents reversed */
      pots[i].parents = (nip_variable*) calloc(kp, sizeof(nip_variable));
      for(j = 0; j < kp; j++) pots[i].parents[j] = vars[fpar[kp - 1 - j]];
    }
    family[0] = vars[child];
    for(j = 0; j < kp; j++) family[j + 1] = pots[i].parents[j];
    pots[i].p = nip_create_potential(family, kp + 1, data);
    if(kp > 0){
      nip_normalise_cpd(pots[i].p);   /* huginnet.y:635-636, 727-728 (with or without data) */
    }
    else if(nd > 0){
      nip_normalise_potential(pots[i].p);             /* huginnet.y:665-666 */
    }
    free(family); free(fpar); free(data);
  }

  /* input action, huginnet.y:202-236 */
  g = nip_new_graph(n);
  for(i = 0; i < n; i++) nip_graph_add_node(g, vars[i]);        /* :1069-1079 */
  for(i = 0; i < np; i++){                                       /* :1082-1102 */
    for(j = 0; j < pots[i].nparents; j++)
      nip_graph_add_child(g, pots[i].parents[j], pots[i].child);
    nip_set_parents(pots[i].child, pots[i].parents, pots[i].nparents);
  }
  nh_interface_to_vars(vars, n, next);

  m = (nh_model*) calloc(1, sizeof(nh_model));
  nc = nip_graph_to_cliques(g, &m->cliques);
  if(nc < 0) return -1;
  m->num_of_cliques = nc;

  /* parsed_potentials_to_jtree, huginnet.y:1110-1152 */
  for(i = 0; i < np; i++){
    nip_clique fc = nip_find_family(m->cliques, nc, pots[i].child);
    if(fc == NULL){ fprintf(stderr, "harness: find_family failed\n"); continue; }
    if(NIP_DIMENSIONALITY(pots[i].p) > 1)
      nip_init_clique(fc, pots[i].child, pots[i].p, 0);
    else
      nip_set_prior(pots[i].child, pots[i].p->data);
  }

  /* model assembly, restated from parse_model (src/nip.c:147-264) */
  m->num_of_vars = n;
  m->variables = vars;
  for(i = 0; i < n; i++){
    nip_variable v = vars[i];
    if(v->next) m->num_of_nexts++;
    if(v->interface_status & NIP_INTERFACE_INCOMING) m->incoming_interface_size++;
    if(v->interface_status & NIP_INTERFACE_OUTGOING) m->outgoing_interface_size++;
    if(v->parents) m->num_of_children++;
    else if(v->prior == NULL)
      v->prior = (double*) calloc(NIP_CARDINALITY(v), sizeof(double)); /* nip.c:175-179 */
  }
  m->next = (nip_variable*) calloc(m->num_of_nexts + 1, sizeof(nip_variable));
  m->previous = (nip_variable*) calloc(m->num_of_nexts + 1, sizeof(nip_variable));
  m->outgoing_interface = (nip_variable*) calloc(m->outgoing_interface_size + 1, sizeof(nip_variable));
  m->previous_outgoing_interface = (nip_variable*) calloc(m->outgoing_interface_size + 1, sizeof(nip_variable));
  m->incoming_interface = (nip_variable*) calloc(m->incoming_interface_size + 1, sizeof(nip_variable));
  m->children = (nip_variable*) calloc(m->num_of_children + 1, sizeof(nip_variable));
  m->independent = (nip_variable*) calloc(n - m->num_of_children + 1, sizeof(nip_variable));
  j = 0; k = 0; { int mm = 0;
    for(i = 0; i < n; i++){
      nip_variable v = vars[i];
      if(v->next){ m->next[j] = v; m->previous[j] = v->next; j++; }
      if(v->interface_status & NIP_INTERFACE_INCOMING) m->incoming_interface[k++] = v;
      if(v->interface_status & NIP_INTERFACE_OLD_OUTGOING){
        m->previous_outgoing_interface[mm] = v;
        m->outgoing_interface[mm] = v->next;
        mm++;
      }
    }
  }
  j = 0; k = 0;
  for(i = 0; i < n; i++){
    if(vars[i]->parents) m->children[j++] = vars[i];
    else m->independent[k++] = vars[i];
  }
  if(m->outgoing_interface_size > 0){
    m->in_clique = nip_find_clique(m->cliques, nc, m->previous_outgoing_interface,
                                   m->outgoing_interface_size);
    m->out_clique = nip_find_clique(m->cliques, nc, m->outgoing_interface,
                                    m->outgoing_interface_size);
  }

  /* enumerate sepsets by walking each clique's list (harness bookkeeping) */
  {
    int cap = nc > 1 ? nc : 1;
    m->sepsets = (nip_sepset*) calloc(cap, sizeof(nip_sepset));
    for(i = 0; i < nc; i++){
      nip_sepset_link l = m->cliques[i]->sepsets;
      while(l){
        nip_sepset s = (nip_sepset) l->data;
        int found = 0;
        for(j = 0; j < m->n_sepsets; j++) if(m->sepsets[j] == s) found = 1;
        if(!found && m->n_sepsets < cap) m->sepsets[m->n_sepsets++] = s;
        l = l->fwd;
      }
    }
  }

  nip_free_graph(g);
  free(next);
  free(pots);   /* potentials stay alive (leaked on purpose, like the parser list) */
  nh_models[nh_n_models] = m;
  return nh_n_models++;
}

/* ------------------------------------------------------------------ */
/* JSON dump of the join-tree description (the index contract)         */
/* ------------------------------------------------------------------ */
typedef struct { char* buf; int cap; int len; } nh_out;
static void nh_put(nh_out* o, const char* fmt, ...);
#include <stdarg.h>
static void nh_put(nh_out* o, const char* fmt, ...){
  va_list ap; int r;
  va_start(ap, fmt);
  r = vsnprintf(o->buf + (o->len < o->cap ? o->len : o->cap),
                o->len < o->cap ? (size_t)(o->cap - o->len) : 0, fmt, ap);
  va_end(ap);
  o->len += r;
}

static void nh_put_doubles(nh_out* o, const double* d, int n){
  int i;
  nh_put(o, "[");
  for(i = 0; i < n; i++) nh_put(o, "%s%.17g", i ? "," : "", d[i]);
  nh_put(o, "]");
}

static int nh_sepset_index(nh_model* m, nip_sepset s){
  int i;
  for(i = 0; i < m->n_sepsets; i++) if(m->sepsets[i] == s) return i;
  return -1;
}

int nh_desc(int h, char* buf, int cap){
  nh_model* m = nh_models[h];
  nh_out o; int i, j;
  o.buf = buf; o.cap = cap; o.len = 0;
  nh_put(&o, "{\"vars\":[");
  for(i = 0; i < m->num_of_vars; i++){
    nip_variable v = m->variables[i];
    nh_put(&o, "%s{\"symbol\":\"%s\",\"card\":%d,\"if\":%d,\"next\":%d,\"previous\":%d,\"parents\":[",
           i ? "," : "", v->symbol, v->cardinality, v->interface_status,
           v->next ? nh_var_index(m, v->next) : -1,
           v->previous ? nh_var_index(m, v->previous) : -1);
    for(j = 0; j < v->num_of_parents; j++)
      nh_put(&o, "%s%d", j ? "," : "", nh_var_index(m, v->parents[j]));
    nh_put(&o, "],\"prior\":");
    if(v->prior && !v->parents) nh_put_doubles(&o, v->prior, v->cardinality);
    else nh_put(&o, "null");
    {
      nip_clique fc = nip_find_family(m->cliques, m->num_of_cliques, v);
      int* fm = nip_find_family_mapping(fc, v);
      nh_put(&o, ",\"family\":%d,\"family_mapping\":[", nh_clique_index(m, fc));
      for(j = 0; j <= v->num_of_parents; j++) nh_put(&o, "%s%d", j ? "," : "", fm[j]);
      nh_put(&o, "]}");
    }
  }
  nh_put(&o, "],\"cliques\":[");
  for(i = 0; i < m->num_of_cliques; i++){
    nip_clique c = m->cliques[i];
    nip_sepset_link l;
    nh_put(&o, "%s{\"vars\":[", i ? "," : "");
    for(j = 0; j < NIP_DIMENSIONALITY(c->p); j++)
      nh_put(&o, "%s%d", j ? "," : "", nh_var_index(m, c->variables[j]));
    nh_put(&o, "],\"links\":[");
    j = 0;
    for(l = c->sepsets; l; l = l->fwd)
      nh_put(&o, "%s%d", j++ ? "," : "", nh_sepset_index(m, (nip_sepset) l->data));
    nh_put(&o, "],\"original\":");
    nh_put_doubles(&o, c->original_p->data, c->original_p->size_of_data);
    nh_put(&o, "}");
  }
  nh_put(&o, "],\"sepsets\":[");
  for(i = 0; i < m->n_sepsets; i++){
    nip_sepset s = m->sepsets[i];
    nh_put(&o, "%s{\"a\":%d,\"b\":%d,\"vars\":[", i ? "," : "",
           nh_clique_index(m, s->first_neighbour), nh_clique_index(m, s->second_neighbour));
    for(j = 0; j < NIP_DIMENSIONALITY(s->old); j++)
      nh_put(&o, "%s%d", j ? "," : "", nh_var_index(m, s->variables[j]));
    nh_put(&o, "]}");
  }
  nh_put(&o, "],\"in_clique\":%d,\"out_clique\":%d,\"outgoing\":[",
         m->in_clique ? nh_clique_index(m, m->in_clique) : -1,
         m->out_clique ? nh_clique_index(m, m->out_clique) : -1);
  for(i = 0; i < m->outgoing_interface_size; i++)
    nh_put(&o, "%s%d", i ? "," : "", nh_var_index(m, m->outgoing_interface[i]));
  nh_put(&o, "],\"previous_outgoing\":[");
  for(i = 0; i < m->outgoing_interface_size; i++)
    nh_put(&o, "%s%d", i ? "," : "", nh_var_index(m, m->previous_outgoing_interface[i]));
  nh_put(&o, "],\"independent\":[");
  for(i = 0; i < m->num_of_vars - m->num_of_children; i++)
    nh_put(&o, "%s%d", i ? "," : "", nh_var_index(m, m->independent[i]));
  nh_put(&o, "],\"children\":[");
  for(i = 0; i < m->num_of_children; i++)
    nh_put(&o, "%s%d", i ? "," : "", nh_var_index(m, m->children[i]));
  nh_put(&o, "]}");
  return o.len;
}

/* ------------------------------------------------------------------ */
/* nip.c restatements (time-slice layer) on top of the reference code  */
/* ------------------------------------------------------------------ */

/* reset_model, src/nip.c:61-73 */
static void h_reset_model(nh_model* m){
  int i;
  for(i = 0; i < m->num_of_vars; i++){
    nip_reset_likelihood(m->variables[i]);
    m->variables[i]->prior_entered = 0;
  }
  nip_global_retraction(m->variables, m->num_of_vars, m->cliques, m->num_of_cliques);
}

/* total_reset, src/nip.c:76-85 */
static void h_total_reset(nh_model* m){
  int i;
  for(i = 0; i < m->num_of_cliques; i++)
    nip_uniform_potential(m->cliques[i]->original_p, 1.0);
  h_reset_model(m);
}

/* use_priors, src/nip.c:88-119 */
static void h_use_priors(nh_model* m, int has_history){
  int i;
  for(i = 0; i < m->num_of_vars - m->num_of_children; i++){
    nip_variable v = m->independent[i];
    if(!v->prior_entered){
      if(!has_history || !(v->interface_status & NIP_INTERFACE_OLD_OUTGOING)){
        nip_enter_prior(m->variables, m->num_of_vars, m->cliques, m->num_of_cliques, v, v->prior);
        v->prior_entered = 1;
      }
    }
  }
}

/* make_consistent, src/nip.c:1600-1617 */
static void h_make_consistent(nh_model* m){
  int i;
  for(i = 0; i < m->num_of_cliques; i++) nip_unmark_clique(m->cliques[i]);
  nip_collect_evidence(NULL, NULL, m->cliques[0]);
  for(i = 0; i < m->num_of_cliques; i++) nip_unmark_clique(m->cliques[i]);
  nip_distribute_evidence(m->cliques[0]);
}

/* insert_ts_step, src/nip.c:982-1001 (every variable marked, as in
 * util/nipinference.c:115-116); obs row = data[t][0..nobs-1] */
static void h_insert_ts_step(nh_model* m, int nobs, const int* obs_vars, const int* row){
  int i;
  for(i = 0; i < nobs; i++){
    if(row[i] >= 0)
      nip_enter_index_observation(m->variables, m->num_of_vars, m->cliques,
                                  m->num_of_cliques, m->variables[obs_vars[i]], row[i]);
  }
}

/* start_timeslice_message_pass, src/nip.c:1031-1065 (BACKWARD=0, FORWARD=1) */
static void h_start_pass(nh_model* m, int forward, nip_potential ag){
  int nv = m->outgoing_interface_size;
  nip_variable* vs; nip_clique c; int* map;
  if(nv == 0){ nip_uniform_potential(ag, 1.0); return; }
  if(forward){ vs = m->outgoing_interface; c = m->out_clique; }
  else { vs = m->previous_outgoing_interface; c = m->in_clique; }
  map = nip_mapper(c->variables, vs, NIP_DIMENSIONALITY(c->p), nv);
  nip_general_marginalise(c->p, ag, map);
  free(map);
  nip_normalise_potential(ag);
}

/* finish_timeslice_message_pass, src/nip.c:1069-1098 */
static void h_finish_pass(nh_model* m, int forward, nip_potential num, nip_potential den){
  int nv = m->outgoing_interface_size;
  nip_variable* vs; nip_clique c; int* map;
  if(nv == 0) return;
  if(forward){ vs = m->previous_outgoing_interface; c = m->in_clique; }
  else { vs = m->outgoing_interface; c = m->out_clique; }
  map = nip_mapper(c->variables, vs, NIP_DIMENSIONALITY(c->p), nv);
  nip_update_potential(num, den, c->p, map);
  free(map);
}

static nip_potential* h_alloc_ag(nh_model* m, int T){
  int i; int* card = (int*) calloc(m->outgoing_interface_size + 1, sizeof(int));
  nip_potential* ag = (nip_potential*) calloc(T + 1, sizeof(nip_potential));
  for(i = 0; i < m->outgoing_interface_size; i++) card[i] = NIP_CARDINALITY(m->outgoing_interface[i]);
  for(i = 0; i <= T; i++) ag[i] = nip_new_potential(card, m->outgoing_interface_size, NULL);
  free(card);
  return ag;
}

static void h_free_ag(nip_potential* ag, int T){
  int i; for(i = 0; i <= T; i++) nip_free_potential(ag[i]); free(ag);
}

static void h_marks(nh_model* m){
  int i; for(i = 0; i < m->num_of_vars; i++) nip_mark_variable(m->variables[i]);
}

/* result of variable of interest: find family, marginalise, normalise
 * (src/nip.c:1535-1552) */
static void h_write_result(nh_model* m, int vi, double* out){
  nip_variable v = m->variables[vi];
  nip_clique c = nip_find_family(m->cliques, m->num_of_cliques, v);
  nip_marginalise_clique(c, v, out);
  nip_normalise_array(out, NIP_CARDINALITY(v));
}

/*
 * forward_backward_inference, restated from src/nip.c:1320-1581.
 * obs: [T][nobs] state indices (-1 = missing); post: [T][sum card(vars)];
 * *ll: log-likelihood SUM over t (nip.c:1466), as the reference returns it.
 */
int nh_fb(int h, int T, int nobs, const int* obs_vars, const int* obs,
          int nint, const int* vint, double* post, double* ll){
  nh_model* m = nh_models[h];
  nip_potential* ag; int t, i, stride = 0, off;
  double m1 = 0, m2;
  for(i = 0; i < nint; i++) stride += NIP_CARDINALITY(m->variables[vint[i]]);
  h_marks(m);
  ag = h_alloc_ag(m, T);
  h_reset_model(m);
  h_use_priors(m, 0);
  if(ll) *ll = 0;
  for(t = 0; t < T; t++){
    if(t > 0) h_finish_pass(m, 1, ag[t-1], NULL);
    if(ll){ h_make_consistent(m); m1 = nip_probability_mass(m->cliques, m->num_of_cliques); }
    h_insert_ts_step(m, nobs, obs_vars, obs + (size_t)t * nobs);
    h_make_consistent(m);
    if(ll){
      m2 = nip_probability_mass(m->cliques, m->num_of_cliques);
      if(m1 > 0 && m2 > 0) *ll = *ll + (log(m2) - log(m1));
      if(m2 == 0.0) *ll = -DBL_MAX;
    }
    h_start_pass(m, 1, ag[t]);
    h_reset_model(m);
    h_use_priors(m, T > 1 ? 1 : 0);
  }
  for(t = T - 1; t >= 0; t--){
    if(t > 0) h_finish_pass(m, 1, ag[t-1], NULL);
    h_insert_ts_step(m, nobs, obs_vars, obs + (size_t)t * nobs);
    if(t < T - 1) h_finish_pass(m, 0, ag[t+1], ag[t]);
    h_make_consistent(m);
    off = 0;
    for(i = 0; i < nint; i++){
      h_write_result(m, vint[i], post + (size_t)t * stride + off);
      off += NIP_CARDINALITY(m->variables[vint[i]]);
    }
    if(t > 0) h_start_pass(m, 0, ag[t]);
    h_reset_model(m);
    h_use_priors(m, t > 1 ? 1 : 0);
  }
  h_free_ag(ag, T);
  return 0;
}

/* forward_inference, restated from src/nip.c:1103-1315 */
int nh_filter(int h, int T, int nobs, const int* obs_vars, const int* obs,
              int nint, const int* vint, double* post, double* ll){
  nh_model* m = nh_models[h];
  nip_potential* ag; int t, i, stride = 0, off;
  double m1 = 0, m2;
  for(i = 0; i < nint; i++) stride += NIP_CARDINALITY(m->variables[vint[i]]);
  h_marks(m);
  ag = h_alloc_ag(m, 1);
  h_reset_model(m);
  h_use_priors(m, 0);
  if(ll) *ll = 0;
  for(t = 0; t < T; t++){
    if(t > 0) h_finish_pass(m, 1, ag[0], NULL);
    if(ll){ h_make_consistent(m); m1 = nip_probability_mass(m->cliques, m->num_of_cliques); }
    h_insert_ts_step(m, nobs, obs_vars, obs + (size_t)t * nobs);
    h_make_consistent(m);
    if(ll){
      m2 = nip_probability_mass(m->cliques, m->num_of_cliques);
      if(m1 > 0 && m2 > 0) *ll = *ll + (log(m2) - log(m1));
      if(m2 == 0) *ll = -DBL_MAX;
    }
    off = 0;
    for(i = 0; i < nint; i++){
      h_write_result(m, vint[i], post + (size_t)t * stride + off);
      off += NIP_CARDINALITY(m->variables[vint[i]]);
    }
    h_start_pass(m, 1, ag[0]);
    h_reset_model(m);
    h_use_priors(m, 1);
  }
  h_free_ag(ag, 1);
  return 0;
}

/* parameter potentials in em_learn layout (src/nip.c:2108-2128):
 * child first, then v->parents order */
static nip_potential* h_alloc_params(nh_model* m){
  int v, i;
  nip_potential* p = (nip_potential*) calloc(m->num_of_vars, sizeof(nip_potential));
  for(v = 0; v < m->num_of_vars; v++){
    int n = nip_number_of_parents(m->variables[v]) + 1;
    int* card = (int*) calloc(n, sizeof(int));
    card[0] = NIP_CARDINALITY(m->variables[v]);
    for(i = 1; i < n; i++) card[i] = NIP_CARDINALITY(m->variables[v]->parents[i-1]);
    p[v] = nip_new_potential(card, n, NULL);
    free(card);
  }
  return p;
}

/*
 * e_step, restated from src/nip.c:1708-2007.  Adds this series' expected
 * counts into params (caller-initialised) and returns 0, or the reference's
 * BAD_LUCK condition as 1.
 */
static int h_e_step(nh_model* m, int T, int nobs, const int* obs_vars, const int* obs,
                    nip_potential* params, double* ll){
  nip_potential* ag; nip_potential* res; int t, i;
  double m1, m2;
  res = (nip_potential*) calloc(m->num_of_vars, sizeof(nip_potential));
  for(i = 0; i < m->num_of_vars; i++)
    res[i] = nip_new_potential(params[i]->cardinality, params[i]->dimensionality, NULL);
  ag = h_alloc_ag(m, T);
  h_reset_model(m);
  h_use_priors(m, 0);
  *ll = 0;
  for(t = 0; t < T; t++){
    if(t > 0) h_finish_pass(m, 1, ag[t-1], NULL);
    h_make_consistent(m);
    m1 = nip_probability_mass(m->cliques, m->num_of_cliques);
    h_insert_ts_step(m, nobs, obs_vars, obs + (size_t)t * nobs);
    h_make_consistent(m);
    m2 = nip_probability_mass(m->cliques, m->num_of_cliques);
    if(m1 > 0 && m2 > 0) *ll = *ll + (log(m2) - log(m1));
    if(m1 <= 0 || m2 <= 0 || *ll > 0){
      for(i = 0; i < m->num_of_vars; i++) nip_free_potential(res[i]);
      free(res); h_free_ag(ag, T);
      return 1;                                    /* NIP_ERROR_BAD_LUCK */
    }
    h_start_pass(m, 1, ag[t]);
    h_reset_model(m);
    h_use_priors(m, T > 1 ? 1 : 0);
  }
  for(t = T - 1; t >= 0; t--){
    if(t > 0) h_finish_pass(m, 1, ag[t-1], NULL);
    h_insert_ts_step(m, nobs, obs_vars, obs + (size_t)t * nobs);
    if(t < T - 1) h_finish_pass(m, 0, ag[t+1], ag[t]);
    h_make_consistent(m);
    for(i = 0; i < m->num_of_vars; i++){
      nip_variable v = m->variables[i];
      nip_clique c; int* map;
      if(t > 0 && (v->interface_status & NIP_INTERFACE_OLD_OUTGOING)) continue;
      c = nip_find_family(m->cliques, m->num_of_cliques, v);
      map = nip_find_family_mapping(c, v);
      nip_general_marginalise(c->p, res[i], map);
      nip_normalise_potential(res[i]);
      nip_sum_potential(params[i], res[i]);
    }
    if(t > 0) h_start_pass(m, 0, ag[t]);
    h_reset_model(m);
    h_use_priors(m, t > 1 ? 1 : 0);
  }
  for(i = 0; i < m->num_of_vars; i++) nip_free_potential(res[i]);
  free(res);
  h_free_ag(ag, T);
  return 0;
}

/* m_step, restated from src/nip.c:2010-2071 (PARAMETER_EPSILON undefined) */
static void h_m_step(nh_model* m, nip_potential* params){
  int i;
  for(i = 0; i < m->num_of_vars; i++) nip_normalise_cpd(params[i]);
  h_total_reset(m);
  for(i = 0; i < m->num_of_vars; i++){
    nip_variable child = m->variables[i];
    if(nip_number_of_parents(child) > 0){
      nip_clique fc = nip_find_family(m->cliques, m->num_of_cliques, child);
      int* fm = nip_find_family_mapping(fc, child);
      nip_init_potential(params[i], fc->p, fm);
      nip_init_potential(params[i], fc->original_p, fm);
    }
    else nip_total_marginalise(params[i], child->prior, 0);
  }
}

/*
 * One E-step over ns series (each T long; obs [ns][T][nobs]).
 * counts_in: initial parameter values (em_learn uses 1.0, nip.c:2172), in
 * the concatenated em_learn layout; counts_out receives the sums.
 * Returns number of BAD_LUCK series; ll_out[ns].
 */
int nh_estep(int h, int ns, int T, int nobs, const int* obs_vars, const int* obs,
             const double* counts_in, double* counts_out, double* ll_out, int* bad){
  nh_model* m = nh_models[h];
  nip_potential* params = h_alloc_params(m);
  int n, i, off = 0, nbad = 0;
  h_marks(m);
  for(i = 0; i < m->num_of_vars; i++){
    memcpy(params[i]->data, counts_in + off, sizeof(double) * params[i]->size_of_data);
    off += params[i]->size_of_data;
  }
  for(n = 0; n < ns; n++){
    int r = h_e_step(m, T, nobs, obs_vars, obs + (size_t)n * T * nobs, params, ll_out + n);
    if(bad) bad[n] = r;
    nbad += r;
  }
  off = 0;
  for(i = 0; i < m->num_of_vars; i++){
    memcpy(counts_out + off, params[i]->data, sizeof(double) * params[i]->size_of_data);
    off += params[i]->size_of_data;
    nip_free_potential(params[i]);
  }
  free(params);
  return nbad;
}

/* number of doubles in the em_learn parameter layout */
int nh_param_size(int h){
  nh_model* m = nh_models[h];
  int v, i, tot = 0;
  for(v = 0; v < m->num_of_vars; v++){
    int s = NIP_CARDINALITY(m->variables[v]);
    for(i = 0; i < m->variables[v]->num_of_parents; i++) s *= NIP_CARDINALITY(m->variables[v]->parents[i]);
    tot += s;
  }
  return tot;
}

/* m_step applied to given parameter values (em_learn layout) */
int nh_m_step(int h, const double* params_in){
  nh_model* m = nh_models[h];
  nip_potential* params = h_alloc_params(m);
  int i, off = 0;
  for(i = 0; i < m->num_of_vars; i++){
    memcpy(params[i]->data, params_in + off, sizeof(double) * params[i]->size_of_data);
    off += params[i]->size_of_data;
  }
  h_m_step(m, params);
  for(i = 0; i < m->num_of_vars; i++) nip_free_potential(params[i]);
  free(params);
  return 0;
}

/*
 * em_learn, restated from src/nip.c:2076-2250 with the random initial
 * parameters (nip.c:2135-2138) replaced by init (em_learn layout), so the
 * run is deterministic.  curve[max_iter] receives the learning curve;
 * returns the number of iterations, or -1 for BAD_LUCK.
 */
int nh_em(int h, int ns, int T, int nobs, const int* obs_vars, const int* obs,
          const double* init, double threshold, int max_iter, double* curve){
  nh_model* m = nh_models[h];
  nip_potential* params = h_alloc_params(m);
  double old_ll, ll = -DBL_MAX, probe;
  int i, n, v, off = 0, it = 0, steps = ns * T;
  h_marks(m);
  for(v = 0; v < m->num_of_vars; v++){
    memcpy(params[v]->data, init + off, sizeof(double) * params[v]->size_of_data);
    off += params[v]->size_of_data;
  }
  do {
    h_m_step(m, params);
    old_ll = ll; ll = 0.0;
    for(v = 0; v < m->num_of_vars; v++) nip_uniform_potential(params[v], 1.0);
    for(n = 0; n < ns; n++){
      if(h_e_step(m, T, nobs, obs_vars, obs + (size_t)n * T * nobs, params, &probe)){
        it = -1; goto done;
      }
      ll += probe;
    }
    if(it < max_iter) curve[it] = ll / steps;
    if(old_ll > ll + (steps * threshold) || ll > 0 || ll == -HUGE_VAL){ it = -1; goto done; }
    i = ++it;
    if(it >= max_iter) break;
  } while((ll - old_ll) > (steps * threshold) || i < 3);
done:
  for(v = 0; v < m->num_of_vars; v++) nip_free_potential(params[v]);
  free(params);
  return it;
}

/* current clique original tables (after nh_m_step) for inspection */
int nh_clique_original(int h, int c, double* out, int cap){
  nh_model* m = nh_models[h];
  nip_potential p = m->cliques[c]->original_p;
  int n = p->size_of_data < cap ? p->size_of_data : cap;
  memcpy(out, p->data, sizeof(double) * n);
  return p->size_of_data;
}

int nh_prior(int h, int v, double* out){
  nh_model* m = nh_models[h];
  nip_variable var = m->variables[v];
  if(!var->prior) return 0;
  memcpy(out, var->prior, sizeof(double) * var->cardinality);
  return var->cardinality;
}

/*
 * util/niplikelihood.c:111-133 restated over the reference's code: per step
 * of each series on its own, the mass after the unmarked columns' evidence
 * (m1), after the marked ones' too (m2), ll = log(m2) - log(m1).
 * obs [ns][T][nobs]; marked [nobs]; out [ns][T][3] = (m1, m2, ll).
 */
int nh_likelihood(int h, int ns, int T, int nobs, const int* obs_vars, const int* marked,
                  const int* obs, double* out){
  nh_model* m = nh_models[h];
  int s, t, i;
  for(s = 0; s < ns; s++){
    h_reset_model(m);
    h_use_priors(m, 0);
    for(t = 0; t < T; t++){
      const int* row = obs + ((size_t)s * T + t) * nobs;
      double* o = out + ((size_t)s * T + t) * 3;
      for(i = 0; i < nobs; i++)
        if(!marked[i] && row[i] >= 0)
          nip_enter_index_observation(m->variables, m->num_of_vars, m->cliques,
                                      m->num_of_cliques, m->variables[obs_vars[i]], row[i]);
      h_make_consistent(m);
      o[0] = nip_probability_mass(m->cliques, m->num_of_cliques);
      for(i = 0; i < nobs; i++)
        if(marked[i] && row[i] >= 0)
          nip_enter_index_observation(m->variables, m->num_of_vars, m->cliques,
                                      m->num_of_cliques, m->variables[obs_vars[i]], row[i]);
      h_make_consistent(m);
      o[1] = nip_probability_mass(m->cliques, m->num_of_cliques);
      o[2] = log(o[1]) - log(o[0]);
      h_reset_model(m);
      h_use_priors(m, 1);
    }
  }
  return 0;
}

/* lottery, src/nip.c:2507-2520 */
static int h_lottery(const double* d, int size){
  int i = 0;
  double sum = 0;
  double r = rand() / (double)RAND_MAX;
  do{
    if(i >= size) return size - 1;
    sum += d[i++];
  } while(sum < r);
  return i - 1;
}

/*
 * generate_data, restated from src/nip.c:2325-2478, for n_series series of
 * length T drawn one after the other from one rand() stream seeded with
 * srand(seed) (random_seed(&seed), nip.c:2482-2502, then generate_data per
 * series as a sampling program would).  order[nv]: the sampling order
 * (independent variables first, then children whose parents are all drawn,
 * nip.c:2343-2375) = the column order of data[n_series][T][nv].
 */
int nh_generate(int h, long seed, int n_series, int T, int* order, int* data){
  nh_model* m = nh_models[h];
  int nv = m->num_of_vars, i, j, k, t, s, ok;
  char* mark = (char*) calloc(nv, 1);
  double* dist;
  nip_potential* alpha;
  int maxc = 1;
  j = 0;
  for(i = 0; i < nv; i++)
    if(m->variables[i]->num_of_parents == 0){ order[j++] = i; mark[i] = 1; }
  while(j < nv){
    for(i = 0; i < nv; i++){
      nip_variable v = m->variables[i];
      if(mark[i]) continue;
      ok = 1;
      for(k = 0; k < v->num_of_parents; k++)
        if(!mark[nh_var_index(m, v->parents[k])]){ ok = 0; break; }
      if(ok){ order[j++] = i; mark[i] = 1; }
    }
  }
  free(mark);
  for(i = 0; i < nv; i++)
    if(NIP_CARDINALITY(m->variables[i]) > maxc) maxc = NIP_CARDINALITY(m->variables[i]);
  dist = (double*) calloc(maxc, sizeof(double));
  alpha = h_alloc_ag(m, 0);
  srand((unsigned)seed);
  for(s = 0; s < n_series; s++){
    int* d = data + (size_t)s * T * nv;
    h_reset_model(m);
    h_use_priors(m, 0);
    for(t = 0; t < T; t++){
      if(t > 0) h_finish_pass(m, 1, alpha[0], NULL);
      for(i = 0; i < nv; i++){
        h_make_consistent(m);
        h_write_result(m, order[i], dist);
        k = h_lottery(dist, NIP_CARDINALITY(m->variables[order[i]]));
        d[(size_t)t * nv + i] = k;
        nip_enter_index_observation(m->variables, m->num_of_vars, m->cliques,
                                    m->num_of_cliques, m->variables[order[i]], k);
      }
      h_make_consistent(m);
      h_start_pass(m, 1, alpha[0]);
      h_reset_model(m);
      h_use_priors(m, 1);
    }
  }
  h_free_ag(alpha, 0);
  free(dist);
  return nv;
}

/*
 * Cliques of an explicit graph through the reference's own triangulation
 * (nip_moralise_graph, nip_make_graph_undirected, nip_triangulate_graph --
 * the sequence of test/graphtest.c:182-230 Test 6/7).  edges: [2*ne]
 * (parent, child).  With set_parents == 0 the variables carry no parent lists,
 * exactly as graphtest builds them.  out: clique variable lists (node
 * indices), CSR offsets in off[ncliques+1].  Returns ncliques.
 */
int nh_graph_cliques(int n, const int* card, int ne, const int* edges, int set_parents,
                     int* off, int* out, int cap){
  nip_variable* v = (nip_variable*) calloc(n, sizeof(nip_variable));
  nip_graph g, gm, gu;
  nip_clique* cl;
  char* st[256];
  int i, j, k, nc, pos = 0;
  for(i = 0; i < 256; i++){ st[i] = (char*) malloc(8); snprintf(st[i], 8, "%d", i); }
  for(i = 0; i < n; i++){
    char sym[16]; snprintf(sym, 16, "G%d", i);
    v[i] = nip_new_variable(sym, "", st, card[i]);
  }
  g = nip_new_graph(n);
  for(i = 0; i < n; i++) nip_graph_add_node(g, v[i]);
  for(i = 0; i < ne; i++) nip_graph_add_child(g, v[edges[2*i]], v[edges[2*i+1]]);
  if(set_parents){
    for(i = 0; i < n; i++){
      nip_variable par[64]; int np = 0;
      for(j = 0; j < ne; j++) if(edges[2*j+1] == i) par[np++] = v[edges[2*j]];
      if(np) nip_set_parents(v[i], par, np);
    }
  }
  gm = nip_moralise_graph(g);
  gu = nip_make_graph_undirected(gm);
  nc = nip_triangulate_graph(gu, &cl);
  off[0] = 0;
  for(i = 0; i < nc; i++){
    for(j = 0; j < NIP_DIMENSIONALITY(cl[i]->p); j++){
      for(k = 0; k < n; k++) if(cl[i]->variables[j] == v[k]) break;
      if(pos < cap) out[pos] = k;
      pos++;
    }
    off[i + 1] = pos;
  }
  for(i = 0; i < 256; i++) free(st[i]);
  return nc;
}

/* ------------------------------------------------------------------ */
/* single-slice scripts (oracle/ref/slice_script.h) over the reference */
/* ------------------------------------------------------------------ */

/* get_probability, src/nip.c:2261-2298 */
static double* h_get_probability(nh_model* m, nip_variable v){
  nip_clique c = nip_find_family(m->cliques, m->num_of_cliques, v);
  double* r;
  if(!c) return NULL;
  r = (double*) calloc(NIP_CARDINALITY(v), sizeof(double));
  nip_marginalise_clique(c, v, r);
  nip_normalise_array(r, NIP_CARDINALITY(v));
  return r;
}

/* get_joint_probability, src/nip.c:2301-2321 */
static nip_potential h_get_joint(nh_model* m, nip_variable* vars, int n){
  int i;
  nip_potential p;
  for(i = 0; i < m->num_of_cliques; i++) nip_unmark_clique(m->cliques[i]);
  p = nip_gather_joint_probability(m->cliques[0], vars, n, NULL, 0);
  if(p) nip_normalise_potential(p);
  return p;
}

#define SS_MODEL nh_model*
#define SS_RESET(m) h_reset_model(m)
#define SS_PRIORS(m, h) h_use_priors(m, h)
#define SS_CONSISTENT(m) h_make_consistent(m)
#define SS_PROB(m, v) h_get_probability(m, v)
#define SS_JOINT(m, vs, n) h_get_joint(m, vs, n)
#define ss_put(ctx, ...) nh_put((nh_out*)(ctx), __VA_ARGS__)
#include "slice_script.h"

/* run a slice script (slice_script.h) on model h; the output text goes to
 * buf (returns its length, which may exceed cap: call again with more room),
 * -1 on a bad script */
int nh_slice(int h, const char* script, char* buf, int cap){
  nh_out o = { buf, cap, 0 };
  if(cap > 0) buf[0] = 0;
  if(ss_run(&o, nh_models[h], script)) return -1;
  return o.len;
}
