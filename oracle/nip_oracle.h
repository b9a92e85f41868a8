/*
 * nip_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Standalone CPU restatement of the reference's fwd-bwd / EM path over a
 * compiled join tree (no reference code linked).  Pinned against the
 * reference's own outputs (oracle/_ref, tests/golden/).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it; the
 * product (nip_amd/) never does.
 */
#ifndef NIP_ORACLE_H
#define NIP_ORACLE_H

/* Flat join-tree description: the "index contract" of SURVEY.md 8(a)
 * rows A18-A20, exactly what nh_desc()/the product compiler emit.
 * Variable-length lists use CSR offsets (n+1 entries). */
typedef struct {
  int nvars;
  const int* card;        /* [nvars] */
  const int* ifs;         /* [nvars] NIP_INTERFACE_* flags */
  const int* par_off;     /* [nvars+1] */
  const int* par;         /* v->parents order */
  const int* prior_off;   /* [nvars] offset into priors, -1 if none */
  const double* priors;
  const int* family;      /* [nvars] family clique */
  const int* fmap_off;    /* [nvars+1] */
  const int* fmap;        /* family mapping, child first */
  int ncliques;
  const int* cv_off;      /* [ncliques+1] */
  const int* cv;          /* clique variables, clique dimension order */
  const int* lk_off;      /* [ncliques+1] */
  const int* lk;          /* sepset indices, c->sepsets list order */
  const int* orig_off;    /* [ncliques+1] */
  const double* orig;     /* original_p tables */
  int nsepsets;
  const int* sa;          /* first_neighbour */
  const int* sb;          /* second_neighbour */
  const int* sv_off;      /* [nsepsets+1] */
  const int* sv;          /* sepset variables */
  int in_clique, out_clique;
  int nout;
  const int* outgoing;
  const int* prev_outgoing;
  int nindep;
  const int* independent;
} no_desc;

void* no_create(const no_desc* d);
void  no_free(void* m);
int   no_param_size(void* m);

int no_fb(void* m, int T, int nobs, const int* obs_vars, const int* obs,
          int nint, const int* vint, double* post, double* ll);
int no_filter(void* m, int T, int nobs, const int* obs_vars, const int* obs,
              int nint, const int* vint, double* post, double* ll);
int no_fb_batch(void* m, int B, int T, int nobs, const int* obs_vars,
                const int* obs, int nint, const int* vint, double* post,
                double* ll, int nthreads);
int no_estep(void* m, int ns, int T, int nobs, const int* obs_vars,
             const int* obs, const double* counts_in, double* counts_out,
             double* ll_out, int* bad);
int no_m_step(void* m, const double* params);
int no_em(void* m, int ns, int T, int nobs, const int* obs_vars, const int* obs,
          const double* init, double threshold, int max_iter, double* curve);
int no_original(void* m, int c, double* out, int cap);
int no_prior(void* m, int v, double* out);
int no_query(void* m, int root, int nev, const int* ev_vars, const double* ev,
             int q, double* out);

#endif
