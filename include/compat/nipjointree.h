/*
 * nipjointree.h -- drop-in for the reference's src/nipjointree.h (nip_amd
 * compat layer, libnip.so): cliques, sepsets and the join-tree operations.
 *
 * The structs keep the field order and types of nipjointree.h:33-85.  A
 * parsed model's cliques (model->cliques) are real join-tree nodes with the
 * reference's variable order, sepset lists (prepend order,
 * nipjointree.c:211-234) and tables (original_p from the compiled CPTs,
 * including the parser's normalisation quirk), so code that walks or reads
 * them -- nip_probability_mass(model->cliques, ...) in util/nipjoint.c --
 * works unchanged.
 *
 * Propagation runs on the GPU: nip_collect_evidence / nip_distribute_evidence
 * replay the reference's traversal on the host (marks, neighbour order, the
 * old/new sepset swap of nip_message_pass, nipjointree.c:580-709) to record
 * the message passes, and execute them with nipamd_hugin_passes
 * (include/nip_amd.h), bit-identical to the reference's arithmetic.
 * Everything else here is host bookkeeping over the tables
 * (nip_amd/compat/jointree_api.cpp).
 */
#ifndef NIP_AMD_COMPAT_JOINTREE_H
#define NIP_AMD_COMPAT_JOINTREE_H

#include <stdio.h>

#include "nippotential.h"
#include "nipvariable.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nip_sepsetlink {
  void* data;                      /* a nip_sepset */
  struct nip_sepsetlink* fwd;
  struct nip_sepsetlink* bwd;
} nip_sepsetlink_struct;
typedef nip_sepsetlink_struct* nip_sepset_link;

typedef struct {
  nip_potential p;                 /* current belief, with evidence */
  nip_potential original_p;        /* the model's tables, no evidence */
  nip_variable* variables;         /* ascending variable ID */
  nip_sepset_link sepsets;         /* neighbouring sepsets, most recent first */
  int num_of_sepsets;
  char mark;
} nip_clique_struct;
typedef nip_clique_struct* nip_clique;

typedef struct {
  nip_potential old;               /* the message before the latest pass */
#ifdef __cplusplus
  nip_potential new_;              /* `new` in C (a keyword in C++): same layout */
#else
  nip_potential new;               /* the latest message */
#endif
  nip_variable* variables;         /* the first neighbour's order */
  nip_clique first_neighbour;
  nip_clique second_neighbour;
} nip_sepset_struct;
typedef nip_sepset_struct* nip_sepset;

typedef struct nip_potentiallink {
  nip_potential data;
  nip_variable child;
  nip_variable* parents;
  struct nip_potentiallink* fwd;
  struct nip_potentiallink* bwd;
} nip_potential_link_struct;
typedef nip_potential_link_struct* nip_potential_link;

typedef struct {
  int length;
  nip_potential_link first;
  nip_potential_link last;
} nip_potential_list_struct;
typedef nip_potential_list_struct* nip_potential_list;

nip_clique nip_new_clique(nip_variable vars[], int nvars);
void nip_free_clique(nip_clique c);
int nip_confirm_sepset(nip_sepset s);
nip_sepset nip_new_sepset(nip_clique neighbour_a, nip_clique neighbour_b);
void nip_free_sepset(nip_sepset s);
nip_potential nip_create_potential(nip_variable variables[], int nvars, double data[]);
void nip_unmark_clique(nip_clique c);
int nip_clique_size(nip_clique c);
int nip_sepset_size(nip_sepset s);
int nip_cliques_connected(nip_clique one, nip_clique two);
int nip_distribute_evidence(nip_clique c);
int nip_collect_evidence(nip_clique c1, nip_sepset s12, nip_clique c2);
nip_potential nip_gather_joint_probability(nip_clique start, nip_variable* vars, int n_vars,
                                           nip_variable* isect, int n_isect);
int nip_init_clique(nip_clique c, nip_variable child, nip_potential p, int transient);
int nip_marginalise_clique(nip_clique c, nip_variable v, double r[]);
int nip_global_retraction(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques);
double nip_probability_mass(nip_clique* cliques, int ncliques);
int nip_enter_observation(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                          nip_variable v, char* state);
int nip_enter_index_observation(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                                nip_variable v, int index);
int nip_enter_evidence(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                       nip_variable v, double evidence[]);
int nip_enter_prior(nip_variable* vars, int nvars, nip_clique* cliques, int ncliques,
                    nip_variable v, double prior[]);
nip_clique nip_find_family(nip_clique* cliques, int ncliques, nip_variable var);
int* nip_find_family_mapping(nip_clique family, nip_variable child);
nip_clique nip_find_clique(nip_clique* cliques, int ncliques, nip_variable* variables, int nvars);
void nip_fprintf_clique(FILE* stream, nip_clique c);
void nip_fprintf_sepset(FILE* stream, nip_sepset s);
int nip_clique_intersection(nip_clique cl1, nip_clique cl2, nip_variable** vars, int* n);
nip_potential_list nip_new_potential_list(void);
int nip_append_potential(nip_potential_list l, nip_potential p, nip_variable child,
                         nip_variable* parents);
int nip_prepend_potential(nip_potential_list l, nip_potential p, nip_variable child,
                          nip_variable* parents);
void nip_free_potential_list(nip_potential_list l);

/* nip_amd extension: collect toward cliques[0] and distribute from it as one
 * GPU call (the two traversals make_consistent runs, src/nip.c:1600-1617) */
int nipamd_compat_make_consistent(nip_clique* cliques, int ncliques);

#ifdef __cplusplus
}
#endif
#endif
