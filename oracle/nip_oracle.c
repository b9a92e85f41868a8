/*
 * nip_oracle.c -- TEST INFRASTRUCTURE ONLY (the "port" oracle).
 *
 * A plain-C restatement of the reference's forward-backward / filtering / EM
 * path, operating on the flat join-tree description of nip_oracle.h.  Every
 * floating-point operation is done in the same order as the reference so the
 * results are bit-identical to it; tests/test_oracle.py pins that against the
 * outputs of the reference's own code (oracle/_ref) stored in tests/golden/.
 *
 * The product (nip_amd/) never links, calls or imports this file.
 */
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include "nip_oracle.h"

#define IF_INCOMING     1
#define IF_OUTGOING     2
#define IF_OLD_OUTGOING 4

typedef struct {
  int dim;
  int card[16];
  int size;
  double* data;
} pot;

typedef struct {
  /* owned copy of the description */
  no_desc d;
  int* ibuf; double* dbuf;
  /* state */
  pot* p;        /* clique beliefs */
  pot* orig;     /* clique original_p */
  pot* sold;     /* sepset old */
  pot* snew;     /* sepset new */
  int** smap_a;  /* positions of sepset vars in first neighbour */
  int** smap_b;
  double** lik;  /* per-variable likelihood */
  double** prior;
  int* prior_entered;
  int* fam_pos;  /* index of v among its family clique's variables */
  char* mark;
} model;

/* ------------------------------------------------------------------ */
/* potential helpers                                                    */
/* ------------------------------------------------------------------ */
static void pot_init(pot* q, int dim, const int* card, const int* vars){
  int i;
  q->dim = dim; q->size = 1;
  for(i = 0; i < dim; i++){ q->card[i] = vars ? card[vars[i]] : card[i]; q->size *= q->card[i]; }
  q->data = (double*) malloc(sizeof(double) * q->size);
  for(i = 0; i < q->size; i++) q->data[i] = 1.0;   /* nip_new_potential(NULL) */
}

/* odometer over the multi-index of a table, dimension 0 fastest
 * (nippotential.c:58-68, 251-264) */
#define ODO_STEP(q, idx) do { int _k = 0; while(_k < (q)->dim){ if(++(idx)[_k] < (q)->card[_k]) break; (idx)[_k] = 0; _k++; } } while(0)

/* flat index in dst of the sub-index chosen by map (nippotential.c:72-81) */
static int sub_flat(const pot* dst, const int* idx, const int* map){
  int k, j = 0, stride = 1;
  for(k = 0; k < dst->dim; k++){ j += idx[map[k]] * stride; stride *= dst->card[k]; }
  return j;
}

/* nip_general_marginalise, nippotential.c:267-311 */
static void marginalise(const pot* src, pot* dst, const int* map){
  int i, idx[16] = {0};
  if(dst->dim == 0){
    dst->data[0] = 0;
    for(i = 0; i < src->size; i++) dst->data[0] += src->data[i];
    return;
  }
  for(i = 0; i < dst->size; i++) dst->data[i] = 0.0;
  for(i = 0; i < src->size; i++){
    dst->data[sub_flat(dst, idx, map)] += src->data[i];
    ODO_STEP(src, idx);
  }
}

/* nip_update_potential, nippotential.c:436-496 */
static void update_potential(const pot* num, const pot* den, pot* tgt, const int* map){
  int i, j, idx[16] = {0};
  const pot* geo = num ? num : den;
  for(i = 0; i < tgt->size; i++){
    j = geo->dim ? sub_flat(geo, idx, map) : 0;
    if(num) tgt->data[i] *= num->data[j];
    if(den){
      if(den->data[j] != 0) tgt->data[i] /= den->data[j];
      else tgt->data[i] = 0;
    }
    ODO_STEP(tgt, idx);
  }
}

/* nip_update_evidence, nippotential.c:499-522 */
static void update_evidence(const double* num, const double* den, pot* tgt, int var){
  int i, idx[16] = {0};
  for(i = 0; i < tgt->size; i++){
    int s = idx[var];
    tgt->data[i] *= num[s];
    if(den != NULL && den[s] != 0) tgt->data[i] /= den[s];
    ODO_STEP(tgt, idx);
  }
}

/* nip_total_marginalise, nippotential.c:314-346 */
static void total_marginalise(const pot* src, double* dst, int var){
  int i, idx[16] = {0};
  if(src->dim == 0){ dst[0] = src->data[0]; return; }
  for(i = 0; i < src->card[var]; i++) dst[i] = 0.0;
  for(i = 0; i < src->size; i++){ dst[idx[var]] += src->data[i]; ODO_STEP(src, idx); }
}

/* nip_normalise_array, nippotential.c:349-359 */
static void normalise_array(double* r, int n){
  int i; double sum = 0;
  for(i = 0; i < n; i++) sum += r[i];
  if(sum == 0) return;
  for(i = 0; i < n; i++) r[i] /= sum;
}

/* nip_normalise_cpd, nippotential.c:373-383 */
static void normalise_cpd(pot* q){
  int i, n = q->card[0];
  for(i = 0; i < q->size; i += n) normalise_array(q->data + i, n);
}

/* nip_init_potential with a mapping, nippotential.c:525-564 */
static void init_potential(const pot* probs, pot* tgt, const int* map){
  int i, idx[16] = {0};
  if(probs->dim == 0) return;
  for(i = 0; i < tgt->size; i++){
    tgt->data[i] *= probs->data[sub_flat(probs, idx, map)];
    ODO_STEP(tgt, idx);
  }
}

/* ------------------------------------------------------------------ */
/* model                                                                */
/* ------------------------------------------------------------------ */
#define CV(m,c)   ((m)->d.cv + (m)->d.cv_off[c])
#define NCV(m,c)  ((m)->d.cv_off[(c)+1] - (m)->d.cv_off[c])
#define SV(m,s)   ((m)->d.sv + (m)->d.sv_off[s])
#define NSV(m,s)  ((m)->d.sv_off[(s)+1] - (m)->d.sv_off[s])

static int* mapper(const int* set, int nset, const int* sub, int nsub){
  /* nip_mapper, nipvariable.c:560-589 */
  int i, j; int* r = (int*) calloc(nsub > 0 ? nsub : 1, sizeof(int));
  for(i = 0; i < nsub; i++) for(j = 0; j < nset; j++) if(sub[i] == set[j]){ r[i] = j; break; }
  return r;
}

static int* dup_i(const int* a, int n){ int* r = (int*) malloc(sizeof(int) * (n > 0 ? n : 1)); if(n > 0) memcpy(r, a, sizeof(int) * n); return r; }
static double* dup_d(const double* a, int n){ double* r = (double*) malloc(sizeof(double) * (n > 0 ? n : 1)); if(n > 0) memcpy(r, a, sizeof(double) * n); return r; }

void* no_create(const no_desc* in){
  model* m = (model*) calloc(1, sizeof(model));
  no_desc* d = &m->d;
  int nv = in->nvars, nc = in->ncliques, ns = in->nsepsets, i, v, c, s;
  int npr = 0;
  *d = *in;
  d->card = dup_i(in->card, nv); d->ifs = dup_i(in->ifs, nv);
  d->par_off = dup_i(in->par_off, nv + 1); d->par = dup_i(in->par, in->par_off[nv]);
  d->prior_off = dup_i(in->prior_off, nv);
  for(v = 0; v < nv; v++) if(in->prior_off[v] >= 0 && in->prior_off[v] + in->card[v] > npr) npr = in->prior_off[v] + in->card[v];
  d->priors = dup_d(in->priors, npr);
  d->family = dup_i(in->family, nv);
  d->fmap_off = dup_i(in->fmap_off, nv + 1); d->fmap = dup_i(in->fmap, in->fmap_off[nv]);
  d->cv_off = dup_i(in->cv_off, nc + 1); d->cv = dup_i(in->cv, in->cv_off[nc]);
  d->lk_off = dup_i(in->lk_off, nc + 1); d->lk = dup_i(in->lk, in->lk_off[nc]);
  d->orig_off = dup_i(in->orig_off, nc + 1); d->orig = dup_d(in->orig, in->orig_off[nc]);
  d->sa = dup_i(in->sa, ns); d->sb = dup_i(in->sb, ns);
  d->sv_off = dup_i(in->sv_off, ns + 1); d->sv = dup_i(in->sv, in->sv_off[ns]);
  d->outgoing = dup_i(in->outgoing, in->nout); d->prev_outgoing = dup_i(in->prev_outgoing, in->nout);
  d->independent = dup_i(in->independent, in->nindep);

  m->p = (pot*) calloc(nc, sizeof(pot)); m->orig = (pot*) calloc(nc, sizeof(pot));
  for(c = 0; c < nc; c++){
    pot_init(&m->p[c], NCV(m, c), d->card, CV(m, c));
    pot_init(&m->orig[c], NCV(m, c), d->card, CV(m, c));
    memcpy(m->orig[c].data, d->orig + d->orig_off[c], sizeof(double) * m->orig[c].size);
    memcpy(m->p[c].data, m->orig[c].data, sizeof(double) * m->orig[c].size);
  }
  m->sold = (pot*) calloc(ns > 0 ? ns : 1, sizeof(pot)); m->snew = (pot*) calloc(ns > 0 ? ns : 1, sizeof(pot));
  m->smap_a = (int**) calloc(ns > 0 ? ns : 1, sizeof(int*)); m->smap_b = (int**) calloc(ns > 0 ? ns : 1, sizeof(int*));
  for(s = 0; s < ns; s++){
    pot_init(&m->sold[s], NSV(m, s), d->card, SV(m, s));
    pot_init(&m->snew[s], NSV(m, s), d->card, SV(m, s));
    m->smap_a[s] = mapper(CV(m, d->sa[s]), NCV(m, d->sa[s]), SV(m, s), NSV(m, s));
    m->smap_b[s] = mapper(CV(m, d->sb[s]), NCV(m, d->sb[s]), SV(m, s), NSV(m, s));
  }
  m->lik = (double**) calloc(nv, sizeof(double*)); m->prior = (double**) calloc(nv, sizeof(double*));
  m->prior_entered = (int*) calloc(nv, sizeof(int)); m->fam_pos = (int*) calloc(nv, sizeof(int));
  for(v = 0; v < nv; v++){
    m->lik[v] = (double*) malloc(sizeof(double) * d->card[v]);
    for(i = 0; i < d->card[v]; i++) m->lik[v][i] = 1.0;
    if(d->prior_off[v] >= 0) m->prior[v] = dup_d(d->priors + d->prior_off[v], d->card[v]);
    c = d->family[v];
    m->fam_pos[v] = -1;
    for(i = 0; i < NCV(m, c); i++) if(CV(m, c)[i] == v){ m->fam_pos[v] = i; break; }
  }
  m->mark = (char*) calloc(nc > 0 ? nc : 1, 1);
  return m;
}

void no_free(void* mm){
  model* m = (model*) mm; int c, s, v;
  if(!m) return;
  for(c = 0; c < m->d.ncliques; c++){ free(m->p[c].data); free(m->orig[c].data); }
  for(s = 0; s < m->d.nsepsets; s++){ free(m->sold[s].data); free(m->snew[s].data); free(m->smap_a[s]); free(m->smap_b[s]); }
  for(v = 0; v < m->d.nvars; v++){ free(m->lik[v]); free(m->prior[v]); }
  free(m->p); free(m->orig); free(m->sold); free(m->snew); free(m->smap_a); free(m->smap_b);
  free(m->lik); free(m->prior); free(m->prior_entered); free(m->fam_pos); free(m->mark);
  free((void*)m->d.card); free((void*)m->d.ifs); free((void*)m->d.par_off); free((void*)m->d.par);
  free((void*)m->d.prior_off); free((void*)m->d.priors); free((void*)m->d.family);
  free((void*)m->d.fmap_off); free((void*)m->d.fmap); free((void*)m->d.cv_off); free((void*)m->d.cv);
  free((void*)m->d.lk_off); free((void*)m->d.lk); free((void*)m->d.orig_off); free((void*)m->d.orig);
  free((void*)m->d.sa); free((void*)m->d.sb); free((void*)m->d.sv_off); free((void*)m->d.sv);
  free((void*)m->d.outgoing); free((void*)m->d.prev_outgoing); free((void*)m->d.independent);
  free(m);
}

/* clone including current (possibly M-stepped) tables and priors */
static model* clone(model* m){
  model* r = (model*) no_create(&m->d);
  int c, v;
  for(c = 0; c < m->d.ncliques; c++) memcpy(r->orig[c].data, m->orig[c].data, sizeof(double) * m->orig[c].size);
  for(v = 0; v < m->d.nvars; v++) if(m->prior[v]) memcpy(r->prior[v], m->prior[v], sizeof(double) * m->d.card[v]);
  return r;
}

static int other(model* m, int s, int c){ return m->d.sa[s] == c ? m->d.sb[s] : m->d.sa[s]; }

/* nip_message_pass, nipjointree.c:676-709 */
static void message_pass(model* m, int c1, int s, int c2){
  pot tmp = m->sold[s]; m->sold[s] = m->snew[s]; m->snew[s] = tmp;
  marginalise(&m->p[c1], &m->snew[s], m->d.sa[s] == c1 ? m->smap_a[s] : m->smap_b[s]);
  update_potential(&m->snew[s], &m->sold[s], &m->p[c2], m->d.sa[s] == c2 ? m->smap_a[s] : m->smap_b[s]);
}

/* nip_collect_evidence, nipjointree.c:630-673 */
static void collect(model* m, int c1, int s12, int c2){
  int l;
  m->mark[c2] = 1;
  for(l = m->d.lk_off[c2]; l < m->d.lk_off[c2 + 1]; l++){
    int s = m->d.lk[l];
    if(!m->mark[m->d.sa[s]]) collect(m, c2, s, m->d.sa[s]);
    if(!m->mark[m->d.sb[s]]) collect(m, c2, s, m->d.sb[s]);
  }
  if(c1 >= 0 && s12 >= 0) message_pass(m, c2, s12, c1);
}

/* nip_distribute_evidence, nipjointree.c:580-627 */
static void distribute(model* m, int c){
  int l;
  m->mark[c] = 1;
  for(l = m->d.lk_off[c]; l < m->d.lk_off[c + 1]; l++){
    int s = m->d.lk[l];
    if(!m->mark[m->d.sa[s]]) message_pass(m, c, s, m->d.sa[s]);
    else if(!m->mark[m->d.sb[s]]) message_pass(m, c, s, m->d.sb[s]);
  }
  for(l = m->d.lk_off[c]; l < m->d.lk_off[c + 1]; l++){
    int s = m->d.lk[l];
    if(!m->mark[m->d.sa[s]]) distribute(m, m->d.sa[s]);
    else if(!m->mark[m->d.sb[s]]) distribute(m, m->d.sb[s]);
  }
}

static void unmark(model* m){ memset(m->mark, 0, m->d.ncliques); }

/* make_consistent, nip.c:1600-1617 */
static void make_consistent(model* m){
  unmark(m); collect(m, -1, -1, 0);
  unmark(m); distribute(m, 0);
}

/* nip_join_tree_dfs with nip_clique_mass / nip_neg_sepset_mass,
 * nipjointree.c:1108-1188 */
static void mass_dfs(model* m, int c, double* acc){
  int l, i; double s_;
  m->mark[c] = 1;
  s_ = 0; for(i = 0; i < m->p[c].size; i++) s_ += m->p[c].data[i];
  *acc += s_;
  for(l = m->d.lk_off[c]; l < m->d.lk_off[c + 1]; l++){
    int s = m->d.lk[l], nb;
    if(!m->mark[m->d.sa[s]]) nb = m->d.sa[s];
    else if(!m->mark[m->d.sb[s]]) nb = m->d.sb[s];
    else continue;
    s_ = 0; for(i = 0; i < m->snew[s].size; i++) s_ += m->snew[s].data[i];
    *acc -= s_;
    mass_dfs(m, nb, acc);
  }
}

static double prob_mass(model* m){ double r = 0; unmark(m); mass_dfs(m, 0, &r); return r; }

/* retraction DFS, nipjointree.c:1089-1105 via nip_join_tree_dfs */
static void retract_dfs(model* m, int c){
  int l, i;
  m->mark[c] = 1;
  memcpy(m->p[c].data, m->orig[c].data, sizeof(double) * m->p[c].size);
  for(l = m->d.lk_off[c]; l < m->d.lk_off[c + 1]; l++){
    int s = m->d.lk[l], nb;
    if(!m->mark[m->d.sa[s]]) nb = m->d.sa[s];
    else if(!m->mark[m->d.sb[s]]) nb = m->d.sb[s];
    else continue;
    for(i = 0; i < m->sold[s].size; i++){ m->sold[s].data[i] = 1; m->snew[s].data[i] = 1; }
    retract_dfs(m, nb);
  }
}

/* nip_global_retraction, nipjointree.c:791-817 */
static void global_retraction(model* m){
  int v;
  unmark(m); retract_dfs(m, 0);
  for(v = 0; v < m->d.nvars; v++)
    update_evidence(m->lik[v], NULL, &m->p[m->d.family[v]], m->fam_pos[v]);
}

/* nip_enter_evidence, nipjointree.c:859-901 */
static void enter_evidence(model* m, int v, const double* ev){
  int i, retr = 0;
  for(i = 0; i < m->d.card[v]; i++) if(m->lik[v][i] == 0 && ev[i] != 0) retr = 1;
  if(!retr) update_evidence(ev, m->lik[v], &m->p[m->d.family[v]], m->fam_pos[v]);
  memcpy(m->lik[v], ev, sizeof(double) * m->d.card[v]);
  if(retr) global_retraction(m);
}

/* nip_enter_index_observation, nipjointree.c:832-856 */
static void enter_index(model* m, int v, int idx){
  double* ev; int i;
  if(idx < 0) return;
  ev = (double*) malloc(sizeof(double) * m->d.card[v]);
  for(i = 0; i < m->d.card[v]; i++) ev[i] = (i == idx) ? 1 : 0;
  enter_evidence(m, v, ev);
  free(ev);
}

/* nip_enter_prior, nipjointree.c:904-943 */
static void enter_prior(model* m, int v){
  int i, zero = 1;
  for(i = 0; i < m->d.card[v]; i++) if(m->prior[v][i] > 0) zero = 0;
  if(zero) return;
  update_evidence(m->prior[v], NULL, &m->p[m->d.family[v]], m->fam_pos[v]);
}

/* reset_model, nip.c:61-73 */
static void reset_model(model* m){
  int v, i;
  for(v = 0; v < m->d.nvars; v++){
    for(i = 0; i < m->d.card[v]; i++) m->lik[v][i] = 1;
    m->prior_entered[v] = 0;
  }
  global_retraction(m);
}

/* use_priors, nip.c:88-119 */
static void use_priors(model* m, int has_history){
  int i;
  for(i = 0; i < m->d.nindep; i++){
    int v = m->d.independent[i];
    if(!m->prior_entered[v]){
      if(!has_history || !(m->d.ifs[v] & IF_OLD_OUTGOING)){
        if(m->prior[v]) enter_prior(m, v);
        m->prior_entered[v] = 1;
      }
    }
  }
}

/* insert_ts_step, nip.c:982-1001 (all variables marked) */
static void insert_step(model* m, int nobs, const int* ov, const int* row){
  int i;
  for(i = 0; i < nobs; i++) if(row[i] >= 0) enter_index(m, ov[i], row[i]);
}

/* interface message potentials */
static pot* alloc_ag(model* m, int n){
  int t; pot* a = (pot*) calloc(n, sizeof(pot));
  for(t = 0; t < n; t++) pot_init(&a[t], m->d.nout, m->d.card, m->d.outgoing);
  return a;
}
static void free_ag(pot* a, int n){ int t; for(t = 0; t < n; t++) free(a[t].data); free(a); }

/* start_timeslice_message_pass, nip.c:1031-1065 */
static void start_pass(model* m, int forward, pot* ag){
  int c, i; int* map;
  if(m->d.nout == 0){ for(i = 0; i < ag->size; i++) ag->data[i] = 1.0; return; }
  c = forward ? m->d.out_clique : m->d.in_clique;
  map = mapper(CV(m, c), NCV(m, c), forward ? m->d.outgoing : m->d.prev_outgoing, m->d.nout);
  marginalise(&m->p[c], ag, map);
  free(map);
  normalise_array(ag->data, ag->size);
}

/* finish_timeslice_message_pass, nip.c:1069-1098 */
static void finish_pass(model* m, int forward, const pot* num, const pot* den){
  int c; int* map;
  if(m->d.nout == 0) return;
  c = forward ? m->d.in_clique : m->d.out_clique;
  map = mapper(CV(m, c), NCV(m, c), forward ? m->d.prev_outgoing : m->d.outgoing, m->d.nout);
  update_potential(num, den, &m->p[c], map);
  free(map);
}

/* nip_marginalise_clique + normalise, nip.c:1535-1552 */
static void write_result(model* m, int v, double* out){
  total_marginalise(&m->p[m->d.family[v]], out, m->fam_pos[v]);
  normalise_array(out, m->d.card[v]);
}

/* forward_backward_inference, nip.c:1320-1581 */
int no_fb(void* mm, int T, int nobs, const int* ov, const int* obs,
          int nint, const int* vint, double* post, double* ll){
  model* m = (model*) mm;
  int t, i, stride = 0, off; double m1 = 0, m2;
  pot* ag;
  for(i = 0; i < nint; i++) stride += m->d.card[vint[i]];
  ag = alloc_ag(m, T + 1);
  reset_model(m); use_priors(m, 0);
  if(ll) *ll = 0;
  for(t = 0; t < T; t++){
    if(t > 0) finish_pass(m, 1, &ag[t-1], NULL);
    if(ll){ make_consistent(m); m1 = prob_mass(m); }
    insert_step(m, nobs, ov, obs + (size_t)t * nobs);
    make_consistent(m);
    if(ll){
      m2 = prob_mass(m);
      if(m1 > 0 && m2 > 0) *ll = *ll + (log(m2) - log(m1));
      if(m2 == 0.0) *ll = -DBL_MAX;
    }
    start_pass(m, 1, &ag[t]);
    reset_model(m); use_priors(m, T > 1);
  }
  for(t = T - 1; t >= 0; t--){
    if(t > 0) finish_pass(m, 1, &ag[t-1], NULL);
    insert_step(m, nobs, ov, obs + (size_t)t * nobs);
    if(t < T - 1) finish_pass(m, 0, &ag[t+1], &ag[t]);
    make_consistent(m);
    off = 0;
    for(i = 0; i < nint; i++){ write_result(m, vint[i], post + (size_t)t * stride + off); off += m->d.card[vint[i]]; }
    if(t > 0) start_pass(m, 0, &ag[t]);
    reset_model(m); use_priors(m, t > 1);
  }
  free_ag(ag, T + 1);
  return 0;
}

/* forward_inference, nip.c:1103-1315 */
int no_filter(void* mm, int T, int nobs, const int* ov, const int* obs,
              int nint, const int* vint, double* post, double* ll){
  model* m = (model*) mm;
  int t, i, stride = 0, off; double m1 = 0, m2;
  pot* ag;
  for(i = 0; i < nint; i++) stride += m->d.card[vint[i]];
  ag = alloc_ag(m, 1);
  reset_model(m); use_priors(m, 0);
  if(ll) *ll = 0;
  for(t = 0; t < T; t++){
    if(t > 0) finish_pass(m, 1, &ag[0], NULL);
    if(ll){ make_consistent(m); m1 = prob_mass(m); }
    insert_step(m, nobs, ov, obs + (size_t)t * nobs);
    make_consistent(m);
    if(ll){
      m2 = prob_mass(m);
      if(m1 > 0 && m2 > 0) *ll = *ll + (log(m2) - log(m1));
      if(m2 == 0) *ll = -DBL_MAX;
    }
    off = 0;
    for(i = 0; i < nint; i++){ write_result(m, vint[i], post + (size_t)t * stride + off); off += m->d.card[vint[i]]; }
    start_pass(m, 1, &ag[0]);
    reset_model(m); use_priors(m, 1);
  }
  free_ag(ag, 1);
  return 0;
}

/* B independent sequences (obs [B][T][nobs], post [B][T][stride]), one
 * model clone per thread -- the reference itself is single-threaded */
int no_fb_batch(void* mm, int B, int T, int nobs, const int* ov, const int* obs,
                int nint, const int* vint, double* post, double* ll, int nthreads){
  model* m = (model*) mm;
  int stride = 0, i;
  for(i = 0; i < nint; i++) stride += m->d.card[vint[i]];
  if(nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    model* mc = clone(m);
    int b;
#pragma omp for schedule(dynamic, 1)
    for(b = 0; b < B; b++)
      no_fb(mc, T, nobs, ov, obs + (size_t)b * T * nobs, nint, vint,
            post + (size_t)b * T * stride, ll ? ll + b : NULL);
    no_free(mc);
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* EM: e_step nip.c:1708-2007, m_step :2010-2071, em_learn :2076-2250  */
/* ------------------------------------------------------------------ */
static pot* alloc_params(model* m){
  int v, k; pot* p = (pot*) calloc(m->d.nvars, sizeof(pot));
  for(v = 0; v < m->d.nvars; v++){
    int card[16], n = m->d.par_off[v + 1] - m->d.par_off[v] + 1;
    card[0] = m->d.card[v];
    for(k = 1; k < n; k++) card[k] = m->d.card[m->d.par[m->d.par_off[v] + k - 1]];
    pot_init(&p[v], n, card, NULL);
  }
  return p;
}
static void free_params(model* m, pot* p){ int v; for(v = 0; v < m->d.nvars; v++) free(p[v].data); free(p); }

int no_param_size(void* mm){
  model* m = (model*) mm; pot* p = alloc_params(m); int v, n = 0;
  for(v = 0; v < m->d.nvars; v++) n += p[v].size;
  free_params(m, p); return n;
}

static int e_step(model* m, int T, int nobs, const int* ov, const int* obs, pot* params, double* ll){
  pot* ag; pot* res; int t, v, i; double m1, m2;
  res = alloc_params(m);
  ag = alloc_ag(m, T + 1);
  reset_model(m); use_priors(m, 0);
  *ll = 0;
  for(t = 0; t < T; t++){
    if(t > 0) finish_pass(m, 1, &ag[t-1], NULL);
    make_consistent(m); m1 = prob_mass(m);
    insert_step(m, nobs, ov, obs + (size_t)t * nobs);
    make_consistent(m); m2 = prob_mass(m);
    if(m1 > 0 && m2 > 0) *ll = *ll + (log(m2) - log(m1));
    if(m1 <= 0 || m2 <= 0 || *ll > 0){ free_params(m, res); free_ag(ag, T + 1); return 1; }
    start_pass(m, 1, &ag[t]);
    reset_model(m); use_priors(m, T > 1);
  }
  for(t = T - 1; t >= 0; t--){
    if(t > 0) finish_pass(m, 1, &ag[t-1], NULL);
    insert_step(m, nobs, ov, obs + (size_t)t * nobs);
    if(t < T - 1) finish_pass(m, 0, &ag[t+1], &ag[t]);
    make_consistent(m);
    for(v = 0; v < m->d.nvars; v++){
      if(t > 0 && (m->d.ifs[v] & IF_OLD_OUTGOING)) continue;
      marginalise(&m->p[m->d.family[v]], &res[v], m->d.fmap + m->d.fmap_off[v]);
      normalise_array(res[v].data, res[v].size);
      for(i = 0; i < res[v].size; i++) params[v].data[i] += res[v].data[i];
    }
    if(t > 0) start_pass(m, 0, &ag[t]);
    reset_model(m); use_priors(m, t > 1);
  }
  free_params(m, res); free_ag(ag, T + 1);
  return 0;
}

static void m_step(model* m, pot* params){
  int v, c, i;
  for(v = 0; v < m->d.nvars; v++) normalise_cpd(&params[v]);
  for(c = 0; c < m->d.ncliques; c++) for(i = 0; i < m->orig[c].size; i++) m->orig[c].data[i] = 1.0; /* total_reset */
  reset_model(m);
  for(v = 0; v < m->d.nvars; v++){
    if(m->d.par_off[v + 1] > m->d.par_off[v]){
      c = m->d.family[v];
      init_potential(&params[v], &m->p[c], m->d.fmap + m->d.fmap_off[v]);
      init_potential(&params[v], &m->orig[c], m->d.fmap + m->d.fmap_off[v]);
    }
    else if(m->prior[v]) total_marginalise(&params[v], m->prior[v], 0);
  }
}

static void load_params(model* m, pot* p, const double* src){
  int v, off = 0;
  for(v = 0; v < m->d.nvars; v++){ memcpy(p[v].data, src + off, sizeof(double) * p[v].size); off += p[v].size; }
}
static void store_params(model* m, pot* p, double* dst){
  int v, off = 0;
  for(v = 0; v < m->d.nvars; v++){ memcpy(dst + off, p[v].data, sizeof(double) * p[v].size); off += p[v].size; }
}

int no_estep(void* mm, int ns, int T, int nobs, const int* ov, const int* obs,
             const double* cin, double* cout, double* ll_out, int* bad){
  model* m = (model*) mm; pot* p = alloc_params(m); int n, nbad = 0;
  load_params(m, p, cin);
  for(n = 0; n < ns; n++){
    int r = e_step(m, T, nobs, ov, obs + (size_t)n * T * nobs, p, ll_out + n);
    if(bad) bad[n] = r;
    nbad += r;
  }
  store_params(m, p, cout);
  free_params(m, p);
  return nbad;
}

int no_m_step(void* mm, const double* params){
  model* m = (model*) mm; pot* p = alloc_params(m);
  load_params(m, p, params); m_step(m, p); free_params(m, p);
  return 0;
}

int no_em(void* mm, int ns, int T, int nobs, const int* ov, const int* obs,
          const double* init, double threshold, int max_iter, double* curve){
  model* m = (model*) mm; pot* p = alloc_params(m);
  double old_ll, ll = -DBL_MAX, probe;
  int n, v, i, it = 0, steps = ns * T;
  load_params(m, p, init);
  do {
    m_step(m, p);
    old_ll = ll; ll = 0.0;
    for(v = 0; v < m->d.nvars; v++) for(i = 0; i < p[v].size; i++) p[v].data[i] = 1.0;
    for(n = 0; n < ns; n++){
      if(e_step(m, T, nobs, ov, obs + (size_t)n * T * nobs, p, &probe)){ it = -1; goto done; }
      ll += probe;
    }
    if(it < max_iter) curve[it] = ll / steps;
    if(old_ll > ll + (steps * threshold) || ll > 0 || ll == -HUGE_VAL){ it = -1; goto done; }
    i = ++it;
    if(it >= max_iter) break;
  } while((ll - old_ll) > (steps * threshold) || i < 3);
done:
  free_params(m, p);
  return it;
}

int no_original(void* mm, int c, double* out, int cap){
  model* m = (model*) mm; int n = m->orig[c].size < cap ? m->orig[c].size : cap;
  memcpy(out, m->orig[c].data, sizeof(double) * n);
  return m->orig[c].size;
}

int no_prior(void* mm, int v, double* out){
  model* m = (model*) mm;
  if(!m->prior[v]) return 0;
  memcpy(out, m->prior[v], sizeof(double) * m->d.card[v]);
  return m->d.card[v];
}

/*
 * Soft-evidence query on a hand-built join tree, the procedure of the
 * reference's test/cliquetest.c:182-213: enter each evidence vector
 * (nip_enter_evidence), collect and distribute from `root`, then the
 * normalised marginal of q from its family clique.
 */
int no_query(void* mm, int root, int nev, const int* ev_vars, const double* ev,
             int q, double* out){
  model* m = (model*) mm;
  int v, i, off = 0;
  for(v = 0; v < m->d.nvars; v++){
    for(i = 0; i < m->d.card[v]; i++) m->lik[v][i] = 1;
  }
  global_retraction(m);
  for(i = 0; i < nev; i++){
    enter_evidence(m, ev_vars[i], ev + off);
    off += m->d.card[ev_vars[i]];
  }
  unmark(m); collect(m, -1, -1, root);
  unmark(m); distribute(m, root);
  write_result(m, q, out);
  return 0;
}
