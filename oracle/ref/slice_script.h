/*
 * slice_script.h -- TEST INFRASTRUCTURE ONLY (oracle).
 *
 * A tiny interpreter of single-slice scripts over a NIP model, included by
 * two programs so that the same script runs on both sides of the drop-in:
 *   - oracle/ref/nipref_harness.c (nh_slice): the reference's own compiled
 *     nipjointree.c / nippotential.c under the harness's restated nip.c
 *     compositions (h_reset_model, h_use_priors, h_make_consistent);
 *   - tests/capi/slice_driver.c: the same script against libnip.so through
 *     the compat headers (reset_model, use_priors, make_consistent on the GPU).
 * The including file defines SS_MODEL (a pointer type with num_of_vars,
 * variables, num_of_cliques, cliques), SS_RESET(m), SS_PRIORS(m, h),
 * SS_CONSISTENT(m), SS_PROB(m, v) (malloc'd normalised marginal) and
 * SS_JOINT(m, vars, n) (a normalised nip_potential), and an output sink
 * ss_put(ctx, fmt, ...).  Doubles print as %a, so outputs compare bit for bit.
 *
 * Script: whitespace-separated commands, variables by model index
 *   reset | priors H | obs V S | soft V p_0 .. p_{card-1} | consistent
 *   collect C | distribute C     (the nipjointree.h primitives from clique C)
 *   mass | prob V | joint N V_1 .. V_N | dump
 */
#ifndef NIP_SLICE_SCRIPT_H
#define NIP_SLICE_SCRIPT_H

#include <stdlib.h>
#include <string.h>

static void ss_doubles(void* ctx, const double* d, int n){
  int i;
  for(i = 0; i < n; i++) ss_put(ctx, " %a", d[i]);
  ss_put(ctx, "\n");
}

static void ss_unmark_all(SS_MODEL m){
  int i;
  for(i = 0; i < m->num_of_cliques; i++) nip_unmark_clique(m->cliques[i]);
}

/* every clique's belief, then -- first seen in clique / list order -- every
 * sepset's old and new message */
static void ss_dump(void* ctx, SS_MODEL m){
  int i, k, n = 0;
  nip_sepset seen[4096];
  nip_sepset_link l;
  for(i = 0; i < m->num_of_cliques; i++){
    nip_clique c = m->cliques[i];
    ss_put(ctx, "clique %d", i);
    ss_doubles(ctx, c->p->data, c->p->size_of_data);
    for(l = c->sepsets; l; l = l->fwd){
      nip_sepset s = (nip_sepset)l->data;
      int dup = 0;
      for(k = 0; k < n; k++) dup |= seen[k] == s;
      if(dup || n >= 4096) continue;
      seen[n++] = s;
      ss_put(ctx, "sepset %d old", n - 1);
      ss_doubles(ctx, s->old->data, s->old->size_of_data);
      ss_put(ctx, "sepset %d new", n - 1);
      ss_doubles(ctx, s->new->data, s->new->size_of_data);
    }
  }
}

static int ss_run(void* ctx, SS_MODEL m, const char* script){
  char tok[64];
  const char* p = script;
  int used, i, n;
#define SS_NEXT() (sscanf(p, "%63s%n", tok, &used) == 1 ? (p += used, 1) : 0)
#define SS_INT() (SS_NEXT() ? atoi(tok) : -1)
  while(SS_NEXT()){
    if(!strcmp(tok, "reset")) SS_RESET(m);
    else if(!strcmp(tok, "priors")) SS_PRIORS(m, SS_INT());
    else if(!strcmp(tok, "consistent")) SS_CONSISTENT(m);
    else if(!strcmp(tok, "obs")){
      int v = SS_INT(), s = SS_INT();
      nip_enter_index_observation(m->variables, m->num_of_vars, m->cliques, m->num_of_cliques,
                                  m->variables[v], s);
    }
    else if(!strcmp(tok, "soft")){
      int v = SS_INT();
      int card = NIP_CARDINALITY(m->variables[v]);
      double* e = (double*) calloc(card, sizeof(double));
      for(i = 0; i < card; i++){ SS_NEXT(); e[i] = strtod(tok, NULL); }
      nip_enter_evidence(m->variables, m->num_of_vars, m->cliques, m->num_of_cliques,
                         m->variables[v], e);
      free(e);
    }
    else if(!strcmp(tok, "collect")){
      int c = SS_INT();
      ss_unmark_all(m);
      nip_collect_evidence(NULL, NULL, m->cliques[c]);
    }
    else if(!strcmp(tok, "distribute")){
      int c = SS_INT();
      ss_unmark_all(m);
      nip_distribute_evidence(m->cliques[c]);
    }
    else if(!strcmp(tok, "mass"))
      ss_put(ctx, "mass %a\n", nip_probability_mass(m->cliques, m->num_of_cliques));
    else if(!strcmp(tok, "prob")){
      int v = SS_INT();
      double* r = SS_PROB(m, m->variables[v]);
      ss_put(ctx, "prob %d", v);
      if(r) ss_doubles(ctx, r, NIP_CARDINALITY(m->variables[v])); else ss_put(ctx, " null\n");
      free(r);
    }
    else if(!strcmp(tok, "joint")){
      nip_variable vs[64];
      nip_potential r;
      n = SS_INT();
      for(i = 0; i < n && i < 64; i++) vs[i] = m->variables[SS_INT()];
      r = SS_JOINT(m, vs, n);
      ss_put(ctx, "joint");
      if(r){
        for(i = 0; i < r->dimensionality; i++) ss_put(ctx, " %d", r->cardinality[i]);
        ss_put(ctx, " :");
        ss_doubles(ctx, r->data, r->size_of_data);
        nip_free_potential(r);
      } else ss_put(ctx, " null\n");
    }
    else if(!strcmp(tok, "dump")) ss_dump(ctx, m);
    else return -1;
  }
#undef SS_NEXT
#undef SS_INT
  return 0;
}

#endif
