/*
 * nippotential.h -- drop-in for the reference's src/nippotential.h (nip_amd
 * compat layer, libnip.so): multidimensional probability tables.
 *
 * The struct keeps the field order and types of nippotential.h:48-55 (callers
 * read p->data, p->size_of_data and p->cardinality directly, e.g.
 * src/nip.c:2020-2024, src/nipjointree.c:1159).  Tables are flat with
 * dimension 0 least significant (nippotential.c:58-68).  Every function of
 * nippotential.h:70-275 is provided (nip_amd/compat/potential_api.cpp) with
 * the reference's arithmetic, operation for operation, so results are
 * bit-identical: marginalisation sums each destination entry over its
 * pre-image in ascending source order; update_potential writes 0 where the
 * denominator is 0 while update_evidence skips that division; normalising an
 * all-zero array leaves it unchanged.
 *
 * These operate on caller-owned host tables, as in the reference.  The
 * model-level propagation built from them -- nip_collect_evidence /
 * nip_distribute_evidence / make_consistent -- runs on the GPU
 * (nipamd_hugin_passes, include/nip_amd.h).
 */
#ifndef NIP_AMD_COMPAT_POTENTIAL_H
#define NIP_AMD_COMPAT_POTENTIAL_H

#include <math.h>
#include <stdio.h>

#include "niplists.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef HUGE_DOUBLE
#define HUGE_DOUBLE HUGE_VAL
#endif

#define NIP_DIMENSIONALITY(p) ((p)->dimensionality)

typedef struct nip_pot_array {
  int dimensionality;
  int* cardinality;
  int* temp_index;                 /* scratch for index calculations */
  int size_of_data;                /* prod(cardinality); 1 for a scalar */
  double* data;
  nip_string_pair_list application_specific_properties;
} nip_potential_struct;

typedef nip_potential_struct* nip_potential;

nip_potential nip_new_potential(int cardinality[], int dimensionality, double data[]);
int nip_set_potential_property(nip_potential p, char* key, char* value);
char* nip_get_potential_property(nip_potential p, char* key);
nip_potential nip_copy_potential(nip_potential p);
int nip_retract_potential(nip_potential p, nip_potential ref);
void nip_free_potential(nip_potential p);
void nip_uniform_potential(nip_potential p, double value);
void nip_random_potential(nip_potential p);
double nip_get_potential_value(nip_potential p, int indices[]);
void nip_set_potential_value(nip_potential p, int indices[], double value);
void nip_inverse_mapping(nip_potential p, int flat_index, int indices[]);
int nip_general_marginalise(nip_potential source, nip_potential destination, int mapping[]);
int nip_total_marginalise(nip_potential source, double destination[], int variable);
void nip_normalise_array(double result[], int array_size);
int nip_normalise_potential(nip_potential p);
int nip_normalise_cpd(nip_potential p);
int nip_normalise_dimension(nip_potential p, int dimension);
int nip_sum_potential(nip_potential sum, nip_potential increment);
int nip_update_potential(nip_potential numerator, nip_potential denominator,
                         nip_potential target, int mapping[]);
int nip_update_evidence(double numerator[], double denominator[], nip_potential target, int var);
int nip_init_potential(nip_potential probs, nip_potential target, int mapping[]);
void nip_fprintf_potential(FILE* stream, nip_potential p);

#ifdef __cplusplus
}
#endif
#endif
