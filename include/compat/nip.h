/*
 * nip.h -- drop-in for the reference's src/nip.h on the nip_amd GPU engine:
 * libnip.so (the sources under nip_amd/compat).
 *
 * Programs written against the reference's nip.h -- util/nipinference.c,
 * nipmap.c, niptrain.c, nipsample.c, niplikelihood.c, nipjoint.c -- compile
 * unmodified against this header and link against libnip.so instead of the
 * reference's objects.  The structs a caller reads directly keep the
 * reference's field order and types (nip_model_struct nip.h:71-104,
 * time_series_struct nip.h:112-122, uncertain_series_struct nip.h:131-136),
 * and a parsed model carries a real join tree (model->cliques, in_clique,
 * out_clique; nipjointree.h) with the reference's clique order, variable
 * order, sepset lists and tables.
 *
 * Where the work goes:
 *   forward_inference / forward_backward_inference / em_learn / generate_data
 *       the batched GPU engine (nipamd_filter / nipamd_fb / nipamd_em_learn /
 *       nipamd_generate); a model without a GPU plan for the request fails
 *       with NULL / an error code -- there is no CPU path
 *   make_consistent (and insert_hard/soft_evidence, which end with it)
 *       GPU Hugin propagation over the model's tables (nipamd_hugin_passes)
 *   reset_model / use_priors / insert_*_step / model_prob_mass /
 *   get_probability / get_joint_probability
 *       the reference's bookkeeping over the host tables (nipjointree.h)
 */
#ifndef NIP_AMD_COMPAT_NIP_H
#define NIP_AMD_COMPAT_NIP_H

#include <assert.h>
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "niperrorhandler.h"
#include "nipjointree.h"
#include "niplists.h"
#include "nipparsers.h"
#include "nippotential.h"
#include "nipvariable.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TIME_SERIES_LENGTH(ts) ((ts)->length)
#define UNCERTAIN_SERIES_LENGTH(ucs) ((ucs)->length)
#define NIP_FIELD_SEPARATOR ','
#define NIP_HAD_A_PREVIOUS_TIMESLICE 1

enum nip_direction_type { BACKWARD, FORWARD };
typedef enum nip_direction_type nip_direction;

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
  int node_size_x;
  int node_size_y;
} nip_model_struct;
typedef nip_model_struct* nip_model;

typedef struct {
  nip_model model;
  int num_of_hidden;
  nip_variable* hidden;                     /* variables without a data column */
  int num_of_observed;
  nip_variable* observed;                   /* the data columns, file order */
  int length;
  int** data;                               /* data[t][i]: state index, -1 missing */
} time_series_struct;
typedef time_series_struct* time_series;

typedef struct {
  int num_of_vars;
  nip_variable* variables;
  int length;
  double*** data;                           /* data[t][i][state] */
} uncertain_series_struct;
typedef uncertain_series_struct* uncertain_series;

/* the single-slice state (src/nip.c:61-119, 951-1027, 1600-1617, 2254-2321) */
void reset_model(nip_model model);
void total_reset(nip_model model);
void use_priors(nip_model model, int has_history);
int insert_hard_evidence(nip_model model, char* varname, char* observation);
int insert_soft_evidence(nip_model model, char* varname, double* distribution);
int insert_ts_step(time_series ts, int t, nip_model model, char mark_mask);
int insert_ucs_step(uncertain_series ucs, int t, nip_model model, char mark_mask);
void make_consistent(nip_model model);
double model_prob_mass(nip_model model);
double* get_probability(nip_model model, nip_variable v);
nip_potential get_joint_probability(nip_model model, nip_variable* vars, int num_of_vars);

nip_model parse_model(char* file);
int write_model(nip_model model, char* filename);
void free_model(nip_model model);
nip_variable model_variable(nip_model model, char* symbol);

int read_timeseries(nip_model model, char* datafile, time_series** results);
int write_timeseries(time_series* ts_set, int n_series, char* filename);
void free_timeseries(time_series ts);
int timeseries_length(time_series ts);
char* get_observation(time_series ts, nip_variable v, int time);
int set_observation(time_series ts, nip_variable v, int time, char* observation);

int write_uncertainseries(uncertain_series* ucs_set, int n_series, nip_variable v, char* filename);
void free_uncertainseries(uncertain_series ucs);
int uncertainseries_length(uncertain_series ucs);

/* ll: the SUM of the per-step log-likelihoods, as the reference returns it */
uncertain_series forward_inference(time_series ts, nip_variable vars[], int nvars,
                                   double* loglikelihood);
uncertain_series forward_backward_inference(time_series ts, nip_variable vars[], int nvars,
                                            double* loglikelihood);
int em_learn(time_series* ts, int n_ts, double threshold, nip_double_list learning_curve);

/* sampled on the GPU from the caller's rand() stream (nip.c:2325-2478) */
time_series generate_data(nip_model model, int length);

long random_seed(long* seedpointer);
int lottery(double* distribution, int size);
void print_cliques(nip_model model);

/* Batched extension: n_ts series of one length through one
 * engine launch; ucs_out[n_ts] receives what forward_backward_inference
 * would return for each, ll_out[n_ts] their log-likelihoods. */
int forward_backward_inference_batch(time_series* ts, int n_ts, nip_variable vars[], int nvars,
                                     uncertain_series* ucs_out, double* ll_out);

#ifdef __cplusplus
}
#endif
#endif
