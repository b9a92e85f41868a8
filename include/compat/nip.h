/*
 * nip.h -- drop-in for the reference's time-series API (src/nip.h) on the
 * nip_amd GPU engine: libnip.so (nip_amd/compat/compat.cpp).
 *
 * Programs written against the reference's nip.h -- util/nipinference.c,
 * util/nipmap.c, util/niptrain.c -- compile unmodified against this header
 * and link against libnip.so instead of the reference's objects.  The structs
 * a caller reads directly keep the reference's field order and types
 * (nip_model_struct nip.h:71-104, time_series_struct nip.h:112-122,
 * uncertain_series_struct nip.h:131-136, nip_variable_struct
 * nipvariable.h:51-78).  The join tree is compiled and held by the engine
 * (an nipamd_model behind each nip_model), so the clique fields are opaque
 * and the potential / join-tree API of nippotential.h / nipjointree.h is not
 * part of this layer.
 *
 * forward_inference / forward_backward_inference / em_learn run on the GPU
 * (nipamd_filter / nipamd_fb / nipamd_em_learn); a model without a GPU plan
 * for the request fails with NULL / an error code -- there is no CPU path.
 */
#ifndef NIP_AMD_COMPAT_NIP_H
#define NIP_AMD_COMPAT_NIP_H

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "niperrorhandler.h"
#include "niplists.h"
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

/* the join tree is the engine's: cliques are opaque here */
typedef struct nip_clique_type* nip_clique;

typedef struct {
  int num_of_cliques;
  nip_clique* cliques;                      /* NULL */
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
  nip_clique in_clique;                     /* NULL */
  nip_clique out_clique;                    /* NULL */
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
