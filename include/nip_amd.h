/*
 * nip_amd.h -- C-ABI of the MI355X-native NIP forward-backward engine.
 *
 * Plain C types only (pointers and sizes); no torch or HIP types appear in the
 * signatures.  Device pointers are HIP device allocations; `stream` is a
 * hipStream_t passed as void* (NULL = default stream).
 *
 * Each entry point names the reference interface it replaces (paths relative
 * to the reference tree, manuelschmidt/nip @ v0).  Error codes follow the
 * reference's convention: 0 = NIP_NO_ERROR (src/niperrorhandler.h:32), else a
 * NIP_ERROR_* code.  The reference USES those codes (~200 call sites in nip.c,
 * nipparsers.c, huginnet.y, util/) but never defines them; the values below
 * are the only ones the project ever had (nip-2010-10-27.tar.gz,
 * errorhandler.h:5-13).  NIP_ERROR_BAD_LUCK is distinct and non-zero as
 * util/niptrain.c:153,189 requires.
 */
#ifndef NIP_AMD_H
#define NIP_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef NIP_NO_ERROR
#define NIP_NO_ERROR               0
#endif
#define NIP_ERROR_NULLPOINTER      1
#define NIP_ERROR_DIVBYZERO        2
#define NIP_ERROR_INVALID_ARGUMENT 3
#define NIP_ERROR_OUTOFMEMORY      4
#define NIP_ERROR_IO               5
#define NIP_ERROR_GENERAL          6
#define NIP_ERROR_FILENOTFOUND     7
#define NIP_ERROR_BAD_LUCK         8
/* engine-specific: the compiled slice has no GPU execution plan yet */
#define NIPAMD_ERROR_UNSUPPORTED   100
/* engine-specific: no usable gfx950 device / HIP runtime failure */
#define NIPAMD_ERROR_DEVICE        101

/* Per-sequence status bits written by the batched entry points. */
#define NIPAMD_STATUS_ZERO_MASS    1u  /* some m2 == 0: ll = -DBL_MAX (src/nip.c:1471-1473) */
#define NIPAMD_STATUS_BAD_LUCK     2u  /* e_step's m1<=0 || m2<=0 || ll>0 (src/nip.c:1827-1854);
                                          nipamd_estep sets ZERO_MASS|BAD_LUCK */

typedef struct nipamd_model nipamd_model;

/* ------------------------------------------------------------------ */
/* Model construction (host)                                            */
/* ------------------------------------------------------------------ */

/*
 * Build a model from a Bayes-net spec given in Hugin-file order.
 * Replaces parse_model() (src/nip.c:122-294) together with the grammar
 * actions it drives (src/huginnet.y:202-236, 321-387, 582-780, 1058-1254) and
 * the join-tree compiler nip_graph_to_cliques() (src/nipgraph.c:518-544).
 * Variable IDs, clique order, clique dimension order, sepsets, family
 * cliques/mappings and the parsed-CPT normalisation (huginnet.y:635-636) are
 * reproduced bit-exactly.
 *
 *   n_nodes            nodes in declaration order
 *   symbols[n]         node symbols (may be NULL)
 *   card[n]            number of states
 *   next[n]            index of the NIP_next node, or -1
 *   n_pots             potential declarations in file order
 *   pot_child[p]       child node index
 *   pot_nparents[p]    number of parents
 *   pot_parents        concatenated parent indices, FILE order
 *   pot_ndata[p]       number of data values (0 = "data" omitted)
 *   pot_data           concatenated data in textual order
 */
int nipamd_model_from_spec(int n_nodes, const char* const* symbols,
                           const int* card, const int* next, int n_pots,
                           const int* pot_child, const int* pot_nparents,
                           const int* pot_parents, const int* pot_ndata,
                           const double* pot_data, nipamd_model** out);

/* Same, reading a Hugin .net file (replaces parse_model(char*), src/nip.c:122). */
int nipamd_model_from_net(const char* path, nipamd_model** out);

/* Replaces free_model() (src/nip.c:485-508). */
void nipamd_model_free(nipamd_model* m);

/* Number of variables / index of a symbol (replaces model_variable(),
 * src/nip.c:1584-1597). */
int nipamd_model_num_vars(const nipamd_model* m);
int nipamd_model_var_index(const nipamd_model* m, const char* symbol);
int nipamd_model_var_card(const nipamd_model* m, int v);

/*
 * Index contract: JSON description of the compiled join
 * tree -- variables (cards, interface flags, parents, priors, family clique and
 * mapping), cliques (dimension order, sepset link order, original tables),
 * sepsets, in/out cliques and interface lists.  Returns the JSON length
 * (excluding the terminator); writes at most cap bytes.
 */
int nipamd_model_desc_json(const nipamd_model* m, char* buf, int cap);

/*
 * Clique array of an explicit DAG through the join-tree compiler alone
 * (moralise, triangulate: src/nipgraph.c:325-351, 443-515).  edges [2*n_edges]
 * are (parent, child) node indices; set_parents = 0 reproduces graphs built
 * without parent lists (test/graphtest.c:182-230).  clique_off [ncliques+1]
 * CSR offsets into clique_vars (at most cap entries written).  Returns the
 * number of cliques, or a negated NIP_ERROR_* code (clique_off must hold
 * n+1 entries).
 */
int nipamd_graph_cliques(int n, const int* card, int n_edges, const int* edges,
                         int set_parents, int* clique_off, int* clique_vars, int cap);

/* Size of the em_learn parameter layout (src/nip.c:2101-2128): for every
 * variable, a table with the child as dimension 0, then v->parents order. */
int nipamd_model_param_size(const nipamd_model* m);

/* 1 if the model has a GPU execution plan for this request: the interface-
 * chain kernels or the general join-tree engine (any slice whose clique
 * tables fit; include/nip_amd.h NIPAMD_ENGINE_*). */
int nipamd_model_gpu_supported(const nipamd_model* m, int n_obs,
                               const int* obs_vars, int n_query,
                               const int* query_vars);

/*
 * Engine selection for a model (not part of the reference API).
 *   NIPAMD_ENGINE_AUTO   the interface-chain kernels where the slice is an
 *                        interface chain and they fit, else (fb / filter
 *                        of current-interface variables, <= 16 joint
 *                        interface states) the evidence-indexed chain
 *                        (opchain.hip), else the general join-tree engine
 *                        (jtree.hip)
 *   NIPAMD_ENGINE_CHAIN  interface-chain kernels only (UNSUPPORTED otherwise)
 *   NIPAMD_ENGINE_JTREE  the general join-tree engine for every request
 * Both run on the GPU; there is no CPU path.  Returns the previous value.
 */
#define NIPAMD_ENGINE_AUTO  0
#define NIPAMD_ENGINE_CHAIN 1
#define NIPAMD_ENGINE_JTREE 2
int nipamd_model_set_engine(nipamd_model* m, int engine);

/*
 * The interface chain's transition folded on the GPU (fold.hip): the
 * in-clique's hidden parents summed out under their priors -- the
 * marginalisation the reference repeats every time slice
 * (nip_general_marginalise over the in-clique, src/nippotential.c:267-311),
 * done once per model version.  keep = -1: out = A [64][64] (row = previous
 * state); keep = j: out = hidden parent j's table [card_j][64][64].  cap =
 * doubles available in out.  *kernel_ms: the kernel's time (HIP events),
 * *bytes: in-clique bytes it streamed.  Synchronous, current device.  The
 * engine calls the same code itself for in-cliques of >= 2^22 summed entries
 * (config 5's 64^4); smaller ones fold on the host while compiling.
 */
int nipamd_model_fold(nipamd_model* m, int keep, double* out, long cap, double* kernel_ms, double* bytes);

/*
 * The general engine's compiled schedule for a request (host only, no device
 * work): header hdr[29] (sizes and offsets of jtree.h's JtPlanDev, then L,
 * LDS flag, query row width), the int pool and the table pool.  sizes[0..1]
 * receive the pool lengths; pass NULL pools to query them.  A test hook:
 * tests/jt_emul.py replays the schedule against the CPU oracle.
 */
int nipamd_jt_plan_dump(const nipamd_model* m, int n_obs, const int* obs_vars, int n_query,
                        const int* query, int estep, int* hdr, int hdr_cap, int* ip, long ip_cap,
                        double* dp, long dp_cap, long* sizes);

/* ------------------------------------------------------------------ */
/* Hot path (device)                                                    */
/* ------------------------------------------------------------------ */

/*
 * Batched forward_backward_inference() (src/nip.c:1320-1581) for B
 * independent sequences of equal length T, inputs and outputs resident in
 * HBM, asynchronous on `stream`.
 *
 *   d_obs     int32 [B][T][n_obs]; state index, <0 = missing (nip.c:994)
 *   obs_vars  host int[n_obs]: model variable of each column (ts->observed)
 *   query     host int[n_query]: variables of interest (vars[] of the API)
 *   d_post    double [B][T][sum card(query)]  -- uncertain_series->data
 *   d_ll      double [B] log-likelihood SUM over t as the reference returns
 *             it (nip.c:1466; the header's "average", nip.h:393, is wrong),
 *             or NULL
 *   d_status  uint32 [B] NIPAMD_STATUS_* bits, or NULL
 */
int nipamd_fb(nipamd_model* m, const int32_t* d_obs, int n_obs,
              const int* obs_vars, int B, int T, int n_query,
              const int* query, double* d_post, double* d_ll,
              uint32_t* d_status, void* stream);

/* Host-buffer convenience wrapper around nipamd_fb (copies in and out and
 * synchronises); the PCIe-inclusive path. */
int nipamd_fb_host(nipamd_model* m, const int32_t* obs, int n_obs,
                   const int* obs_vars, int B, int T, int n_query,
                   const int* query, double* post, double* ll,
                   uint32_t* status);

/*
 * Batched forward_inference() (src/nip.c:1103-1315): filtered marginals
 * P(X_t | y_0..y_t) of the query variables, same buffers and conventions as
 * nipamd_fb (d_ll = the same sum over t; the filter pass alone yields it).
 * Replaces forward_inference(ts, vars, nvars, &ll) (nip.h:382-383) batched.
 */
int nipamd_filter(nipamd_model* m, const int32_t* d_obs, int n_obs,
                  const int* obs_vars, int B, int T, int n_query,
                  const int* query, double* d_post, double* d_ll,
                  uint32_t* d_status, void* stream);
int nipamd_filter_host(nipamd_model* m, const int32_t* obs, int n_obs,
                       const int* obs_vars, int B, int T, int n_query,
                       const int* query, double* post, double* ll,
                       uint32_t* status);

/*
 * Batched e_step() (src/nip.c:1708-2007): expected counts of B sequences
 * summed into d_counts (double [param_size], em_learn layout, caller
 * initialised -- em_learn starts from 1.0, nip.c:2172).  Summation over the
 * batch is deterministic (fixed order).  d_ll [B] and d_status [B] optional.
 */
int nipamd_estep(nipamd_model* m, const int32_t* d_obs, int n_obs,
                 const int* obs_vars, int B, int T, double* d_counts,
                 double* d_ll, uint32_t* d_status, void* stream);

/* Host-buffer form of nipamd_estep (copies in, counts[] += on the host
 * array, synchronous): the em_learn seam of INTEGRATION.md. */
int nipamd_estep_host(nipamd_model* m, const int32_t* obs, int n_obs,
                      const int* obs_vars, int B, int T, double* counts,
                      double* ll, uint32_t* status);

/*
 * The two halves of nipamd_estep, for data-parallel EM (one process per GPU,
 * util/niptrain.c:142-195 over a sharded sequence set):
 *   nipamd_estep_partial  B sequences -> d_partial
 *                         [nipamd_estep_partial_size_req(m, n_obs, obs_vars, T)]
 *                         (overwritten): the fixed-order binary-tree sum of the
 *                         per-sequence count slabs, before the model's tables
 *                         are applied.  Partials of power-of-two shards combine
 *                         (pairwise, in rank order) into exactly the partial of
 *                         the whole batch.
 *   nipamd_estep_finalize d_counts += the e_step families of a partial
 *                         (synchronises the stream to read the route tag).
 * A partial ends in three tag slots counting the partials summed into it per
 * kernel route (16-state chain slab, em_learn layout, wide chain slab; the
 * route depends on the engine setting and on T); the finalize fails with
 * NIP_ERROR_INVALID_ARGUMENT on partials of different routes combined,
 * instead of summing mismatched layouts.  The operator chain's e_step
 * (slices outside the chain plan with a joint interface of <= 16 states,
 * NIPAMD_ENGINE_AUTO) tags its partials (-1, -1, -1) and appends a section
 * sized by the request -- its per-evidence-combination sums, whose count
 * depends on the observed variables -- so its partial is
 * nipamd_estep_partial_size_req doubles (nipamd_estep_partial_size for every
 * other route; the _req form is always large enough) and is written only by
 * nipamd_estep_partial_ex given that capacity.  nipamd_estep_partial requires
 * d_status (NIP_ERROR_INVALID_ARGUMENT otherwise) when the model's e_step
 * rejects series with a long leading missing run
 * (nipamd_estep_prefix_first_bad >= 0): the verdict is reported there.
 */
int nipamd_estep_partial_size(const nipamd_model* m);
int nipamd_estep_partial_size_req(nipamd_model* m, int n_obs, const int* obs_vars, int T);
int nipamd_estep_partial(nipamd_model* m, const int32_t* d_obs, int n_obs,
                         const int* obs_vars, int B, int T, double* d_partial,
                         double* d_ll, uint32_t* d_status, void* stream);
/* The same with the partial's capacity in doubles.  nipamd_estep_partial
 * promises only nipamd_estep_partial_size doubles, so it never takes the
 * operator chain's e_step (whose partial is larger): such requests run on the
 * general engine there.  With capacity >= nipamd_estep_partial_size_req the
 * operator chain takes them; capacity < nipamd_estep_partial_size fails with
 * NIP_ERROR_INVALID_ARGUMENT.  The two forms therefore route such a request
 * differently -- nipamd_estep_partial to the general engine (slower; route tag
 * (0, 1, 0), nipamd_last_kernel says so), nipamd_estep_partial_ex to the
 * operator chain (tag (-1, -1, -1)) -- and their partials do not combine:
 * every rank of a data-parallel e_step uses the same entry point. */
int nipamd_estep_partial_ex(nipamd_model* m, const int32_t* d_obs, int n_obs,
                            const int* obs_vars, int B, int T, double* d_partial,
                            long capacity, double* d_ll, uint32_t* d_status,
                            void* stream);
int nipamd_estep_finalize(nipamd_model* m, const double* d_partial,
                          double* d_counts, void* stream);

/*
 * d_out[S] = the fixed-order binary-tree sum of the n rows d_rows[n][S]
 * (pairs (2i, 2i + 1) level by level, an odd tail paired with 0): the tree
 * nipamd_estep_partial reduces its count slabs with, so a data-parallel
 * em_learn sums its per-sequence log-likelihoods in the same shape as its
 * counts (nip_amd/em.py exchange).  d_work: at least 2 * ceil(n / 64) * S
 * doubles of device workspace when n > 64 (else may be null).  Queued on
 * stream, no synchronisation.
 */
int nipamd_tree_sum(const double* d_rows, long n, int S, double* d_work, double* d_out,
                    void* stream);

/*
 * The scalars an em_learn iteration exchanges with its counts (nip_amd/em.py):
 * d_out2[0] = nipamd_tree_sum of the n = B per-sequence log-likelihoods
 * d_ll[B], d_out2[1] = the number of nonzero status words d_status[B] (the
 * series nip.c:2182-2198 fails on).  Written next to the partial (d_out2 =
 * d_partial + size), the pack needs no copy.  d_work: at least
 * 2 * ceil(B / 64) + ceil(B / 4096) doubles of device workspace (B > 0).
 * Queued on stream, no synchronisation.
 */
int nipamd_estep_tail(const double* d_ll, const uint32_t* d_status, long B, double* d_work, double* d_out2,
                      void* stream);

/*
 * The e_step's verdict on a leading run of missing observations: the first
 * step k < T at which the reference's e_step rejects (BAD_LUCK, nip.c:1836-
 * 1840) a series that observed nothing at steps 0..k -- its running ll of pure
 * rounding turned > 0, or a mass was <= 0 -- or -1 if no such step exists.
 * nipamd_estep / _partial set NIPAMD_STATUS_BAD_LUCK on every such series in
 * d_status.  Computed on the host once per model version (the join tree's
 * state over missing steps does not depend on the data); -2 when the run was
 * not simulated -- the model's tables exceed 2^26 entries, or the simulation's
 * work bound (2^29 table entries x steps for a chain whose forward message has
 * not repeated within 32 steps) ran out -- and its leading missing runs are
 * accepted.
 */
int nipamd_estep_prefix_first_bad(nipamd_model* m, int T);

/* m_step() (src/nip.c:2010-2071): normalise params (host, em_learn layout)
 * and re-initialise the model's tables and priors from them. */
int nipamd_m_step(nipamd_model* m, const double* params);

/*
 * em_learn(ts, n_ts, threshold, learning_curve) (src/nip.c:2076-2243) for
 * series of any lengths on one GPU.  obs: the series back to back
 * ([sum lengths][n_obs], state index, -1 missing); init: initial parameters
 * in the em_learn layout, or NULL to draw rand()/RAND_MAX like the reference
 * (seed with srand first); max_iterations: 0 = the reference's stopping rule
 * only.  The learning curve (average log-likelihood per time step per
 * iteration) goes to curve[0..curve_cap).  Returns NIP_NO_ERROR or
 * NIP_ERROR_BAD_LUCK (or an argument / device error); the model keeps the
 * parameters of the last m_step.
 */
int nipamd_em_learn(nipamd_model* m, int n_series, const int* lengths, const int32_t* obs,
                    int n_obs, const int* obs_vars, double threshold, const double* init,
                    int max_iterations, double* curve, int curve_cap, int* curve_len);

/* write_model (src/nip.c:298-484): the model as a Hugin .net file in the
 * reference's layout (learned CPTs from the family cliques, "%f" values). */
int nipamd_write_model(const nipamd_model* m, const char* path);

/* Current clique original table / prior of an independent variable. */
int nipamd_model_original(const nipamd_model* m, int clique, double* out, int cap);
int nipamd_model_prior(const nipamd_model* m, int v, double* out);
/* The compiled join tree: clique c's variables
 * (ascending ID = model index order) and its sepset list in the reference's
 * list order (nipjointree.c:211-234); sepset s's neighbours (first, second)
 * and variables (the first neighbour's order, nipvariable.c:506-557); the
 * in / out cliques of src/nip.c:249-264 (-1 without an interface).  Arrays
 * need room for the model's variable / sepset counts. */
int nipamd_model_num_cliques(const nipamd_model* m);
int nipamd_model_num_sepsets(const nipamd_model* m);
int nipamd_model_clique(const nipamd_model* m, int c, int* vars, int* n_vars, int* links, int* n_links);
int nipamd_model_sepset(const nipamd_model* m, int s, int* a, int* b, int* vars, int* n_vars);
int nipamd_model_interface_cliques(const nipamd_model* m, int* in_clique, int* out_clique);
/* Replace the model's tables: originals[c] (NULL: keep) is clique c's
 * original_p, priors[v] (NULL: keep; ignored for variables with parents) the
 * prior of variable v.  What a caller of the reference achieves by writing
 * clique->original_p / nip_set_prior before inference; libnip.so forwards
 * such edits of its host join tree before every engine call. */
int nipamd_model_set_tables(nipamd_model* m, int n_cliques, const double* const* originals,
                            int n_vars, const double* const* priors);

/* Last error message (thread-local), for diagnostics. */
const char* nipamd_last_error(void);
/* Name of the dominant kernel of the library's last hot-path launch (e.g.
 * "chain_fb_ckpt_kernel"), for measurement labels; "" before any launch. */
const char* nipamd_last_kernel(void);

/* Name of state `state` of variable `var` (the .net `states` field; "0".."card-1"
 * for models built from a spec).  Copies at most cap-1 bytes into buf; returns
 * the full length, -1 on bad arguments.  Replaces nip_variable_state_name
 * (src/nipvariable.c:250-254). */
int nipamd_model_state_name(const nipamd_model* m, int var, int state, char* buf, int cap);
/* Symbol of variable `var` (nip_variable_symbol, src/nipvariable.c); same
 * buffer convention. */
int nipamd_model_var_symbol(const nipamd_model* m, int var, char* buf, int cap);
/* The .net `label` of a variable (v->name, src/nipvariable.h:54); same buffer
 * convention. */
int nipamd_model_var_label(const nipamd_model* m, int var, char* buf, int cap);
/* The rest of a variable record (src/nipvariable.h:51-78) for the nip.h
 * compat layer: info[9] = {cardinality, next, previous (variable index or
 * -1), interface_status (NIP_INTERFACE_* bits), pos_x, pos_y, num_of_parents,
 * model node_size_x, node_size_y}; parents[0..cap) in v->parents order.
 * Returns num_of_parents, -1 on bad arguments. */
int nipamd_model_var_info(const nipamd_model* m, int var, int* info, int* parents, int cap);

/*
 * Time-series data files, the reference's text format:
 * a line of node symbols, then one line per time step (tokens separated by
 * ',' and/or white space), series separated by empty lines; unknown tokens
 * ("null", "N/A", "<null>", ...) are missing (-1).  Columns whose symbol is
 * not a model variable are ignored.
 *   nipamd_read_timeseries  replaces read_timeseries (src/nip.c:512-667) with
 *                           nip_open_data_file / nip_next_line_tokens
 *                           (src/nipparsers.c:48-522)
 *   nipamd_write_uncertainseries replaces write_uncertainseries
 *                           (src/nip.c:815-893): state names, then "%f" rows.
 */
typedef struct nipamd_series nipamd_series;
int nipamd_read_timeseries(const nipamd_model* m, const char* path, nipamd_series** out);
int nipamd_series_count(const nipamd_series* s);
int nipamd_series_num_observed(const nipamd_series* s);
int nipamd_series_observed(const nipamd_series* s, int* vars);   /* model variable per column */
int nipamd_series_length(const nipamd_series* s, int i);
const int32_t* nipamd_series_data(const nipamd_series* s, int i); /* [length][n_observed] */
void nipamd_series_free(nipamd_series* s);
/* post: the series' posteriors back to back, rows of `stride` doubles, the
 * variable's card() values at `offset` in each row */
int nipamd_write_uncertainseries(const nipamd_model* m, const char* path, int var, int n_series,
                                 const int* lengths, const double* post, int stride, int offset);

/*
 * generate_data (src/nip.c:2325-2478) for B series of
 * length T on the GPU, for models with an interface-chain plan.  The draws
 * are the ones the reference makes after random_seed(&seed) (srand) when it
 * calls generate_data B times in a row (util/nipsample.c:100-110): series b
 * uses rand() draws [b T nv, (b+1) T nv) of that one stream.
 *   d_data  int32 [B][T][nv] device, column i = variable order[i]
 *   order   nipamd_generate_order: the sampling order of nip.c:2343-2375
 *           (independent variables, then children of drawn parents) =
 *           time_series->observed of the reference's result; returns nv
 * nipamd_generate is asynchronous on `stream` once the tables are resident
 * (the first call per model builds them); _host copies out and synchronises.
 */
int nipamd_generate_order(const nipamd_model* m, int* order);
int nipamd_generate(nipamd_model* m, long seed, int B, int T, int32_t* d_data, void* stream);
int nipamd_generate_host(nipamd_model* m, long seed, int B, int T, int32_t* data);
/* Same with the rand() values given ([B][T][nv], what rand() returned, in
 * draw order): the compat generate_data draws them from the caller's own
 * rand() stream, whatever state it is in. */
int nipamd_generate_host_draws(nipamd_model* m, int B, int T, const int32_t* draws, int32_t* data);
/* The 31-word glibc rand() state window of each of B series that use
 * draws_per_series draws each after srand(seed): win[b][m] = r[313 + b d + m]
 * (the next draw is (r[n-31] + r[n-3]) >> 1).  Exposed for tests. */
int nipamd_rand_windows(long seed, int B, long draws_per_series, uint32_t* win);

/*
 * util/niplikelihood.c batched: for every step of B
 * series of length T, independently (no message between slices), the
 * probability mass after the evidence of the UNMARKED columns (m1), after all
 * columns (m2), and ll = log(m2) - log(m1) = ln p(marked | unmarked)
 * (niplikelihood.c:111-133).  marked[n_obs]: 1 for the variables of interest.
 * d_obs int32 [B][T][n_obs]; d_m1, d_m2, d_ll double [B][T].  Synchronous.
 */
int nipamd_likelihood(nipamd_model* m, const int32_t* d_obs, int n_obs, const int* obs_vars,
                      const int* marked, int B, int T, double* d_m1, double* d_m2, double* d_ll,
                      void* stream);
int nipamd_likelihood_host(nipamd_model* m, const int32_t* obs, int n_obs, const int* obs_vars,
                           const int* marked, int B, int T, double* m1, double* m2, double* ll);

/*
 * Hugin message passes on the GPU over explicit potential tables: the
 * propagation under libnip.so's single-slice API (nip_collect_evidence /
 * nip_distribute_evidence, src/nipjointree.c:580-673; make_consistent,
 * src/nip.c:1600-1617), which records the passes of the reference's
 * traversal and hands them here.
 *   tables[k]   host pointer to table k (flat, dimension 0 fastest,
 *               src/nippotential.c:58-68); ndim[k] dimensions with the
 *               cardinalities concatenated in card[] (table after table)
 *   passes[6p]  (src, s_new, s_old, dst, map_src, map_dst) for pass p =
 *               nip_message_pass(src, s, dst) (nipjointree.c:676-709):
 *                 s_new := marginalise(src) onto the sepset
 *                          (nip_general_marginalise, nippotential.c:267-311)
 *                 dst   *= s_new / s_old, 0 where s_old is 0
 *                          (nip_update_potential, :436-496)
 *               maps[map_src ...] / maps[map_dst ...]: the position of each
 *               sepset dimension in src / dst (nip_mapper)
 * Passes run in order with the reference's arithmetic, so the tables end
 * bit-identical to the reference's.  Synchronous: the tables are read before
 * and the written ones (s_new, dst) copied back after.
 */
int nipamd_hugin_passes(int n_tables, double* const* tables, const int* ndim, const int* card,
                        int n_passes, const int* passes, const int* maps);

#ifdef __cplusplus
}
#endif
#endif /* NIP_AMD_H */
