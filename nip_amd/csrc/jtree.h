// jtree.h -- the general join-tree engine: a compiled per-slice message
// schedule (host, jtree_plan.cpp) interpreted by gfx950 kernels (jtree.hip)
// for B independent sequences.
//
// It serves every slice the interface-chain kernels do not: several
// interface variables, evidence on hidden parents or on non-leaf variables,
// arbitrary clique trees (SURVEY 8(a) A1-A17 in their general form).  Per
// time slice the reference runs Hugin propagation over the whole join tree
// (make_consistent, src/nip.c:1600-1617; nip_collect_evidence /
// nip_distribute_evidence, src/nipjointree.c:580-673) with the interface
// messages of src/nip.c:1031-1098.  Here the same sum-product runs as three
// sweeps over the tree:
//   forward filter   collect toward out_clique with alpha_{t-1} entered at
//                    in_clique -> alpha_t (normalised, as
//                    start_timeslice_message_pass does), masses m1 / m2
//   backward filter  collect toward in_clique with beta_t entered at
//                    out_clique -> beta_{t-1} (two-filter smoothing: the
//                    reference's gamma_{t+1}/alpha_t ratio is beta_t)
//   posterior        collect + Hugin distribute (division, 0 where the old
//                    sepset is 0: nip_update_potential, src/nippotential.c:
//                    436-496) with both messages; marginals of the queried
//                    variables / em_learn families from their family cliques
// Clique tables are flat, dimension 0 fastest (nippotential.c:58-68);
// projections onto ordered variable subsets are precomputed index maps
// (nip_general_marginalise's choose-index, :267-311) plus their inverse
// (pre-image lists), so marginalisation is a gather-sum with no atomics.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace nipamd {

enum : int { kJtFacObs = 0, kJtFacMsg = 1 };
enum : int { kJtMaxFac = 8 };     // factors fused per pass over a clique (more: extra passes)

// One factor multiplied into a clique table: an observation indicator
// (evidence of the variable whose family clique this is, nip_enter_index_
// observation, src/nipjointree.c:832-856) or a message vector in the unit's
// workspace (an interface message or a child's upward sepset message).
struct JtFac {
  int kind;      // kJtFacObs / kJtFacMsg
  int proj;      // projection (clique -> the factor's variables): offset into the map pool
  int arg;       // obs column, or workspace offset of the message
};

// One clique visited by a collect sweep (post-order toward the root).
struct JtVisit {
  int size;      // |C|
  int base;      // table offset of orig_p x the priors entered every slice
  int psi;       // workspace offset of the clique's working table
  int fac0;      // first factor (JtFac index)
  int nfac;
  int up_proj;   // projection onto the sepset toward the parent (-1 at the root)
  int up_D;      // sepset size
  int up_msg;    // workspace offset of the upward message
};

// One Hugin pass parent -> child of the distribute sweep (pre-order).
struct JtDown {
  int p_psi, p_size, pS_proj;   // parent table and its projection onto the sepset
  int S_D, mu, tmp;             // sepset size, the child's upward message (the old sepset), scratch
  int c_psi, c_size, cS_proj;   // child table and its projection onto the sepset
};

// One output marginal of the posterior sweep.
struct JtOut {
  int psi, size, proj, D;       // family clique table, projection onto the output's variables
  int dst;                      // offset within the output row (query) / parameter slab (e_step)
  int t0_only;                  // e_step: OLD_OUTGOING variables count at t = 0 only (nip.c:1931-1933)
};

// Device-resident plan of one (model version, request).  Offsets are in
// elements of the int pool `ip` (visits, downs, outs, factors, maps, pres as
// structs of ints) or the double pool `dp` (tables).
struct JtPlanDev {
  const int* ip;
  const double* dp;
  int ncl;                // cliques
  int K;                  // interface table size (1 with no interface)
  int ws;                 // doubles of workspace per unit
  int fwd, bwd, post;     // JtVisit arrays (ip offsets, in ints)
  int down, ndown;        // JtDown array
  int out, nout;          // JtOut array
  int fac;                // JtFac array
  int maps, pres;         // map / pre-image pools
  int fwd_root_proj;      // out_clique -> outgoing (alpha_t)
  int bwd_root_proj;      // in_clique -> previous outgoing (beta_{t-1})
  int fwd_root_psi, fwd_root_size, bwd_root_psi, bwd_root_size;
  int pi_off, w_off;      // dp: prior of the previous interface (t = 0), m1 weights
  int ws_alpha, ws_beta, ws_out, ws_slab;   // workspace slots (ws_slab: e_step counts)
  int slab;               // e_step slab size (param_size), 0 otherwise
  int n_ip, n_dp;         // pool sizes (ints, doubles): the kernels stage both in LDS when they fit
};

struct JtRun {
  JtPlanDev p;
  const int32_t* obs;     // [B][T][n_obs] (nullptr: nothing observed)
  long obs_bstride;
  int obs_tstride;
  int nobs;
  long B;
  int T;
  double* msgA;           // [B][T][K] normalised alpha_t
  double* msgB;           // [B][T][K] beta_t
  double* wsg;            // global workspace (nullptr: LDS)
  double* post;           // query rows
  long post_bstride;
  int post_tstride;
  double* ll;
  unsigned* status;
  double* slabs;          // e_step: [B][slab]
  int filter;             // forward_inference: no beta, the posterior sweep uses ones
  int estep;              // status BAD_LUCK rules of e_step (nip.c:1827-1854)
  int chunk;              // posterior: time steps per unit
  int gunits;             // HBM workspace: slots per direction (<= kJtGlobalUnits; wsg holds 2 x gunits)
  // round 6: the pools staged in LDS once per block, W waves per block
  // sharing them (jt_stage_bytes; 0 / 1: the round-3 form, pools read from
  // global memory, one wave per block)
  int stage;
  int waves;
};

// LDS bytes of the staged pools (ints, then doubles, 16-byte aligned)
inline size_t jt_stage_bytes(const JtPlanDev& p) {
  return (((size_t)p.n_ip * sizeof(int) + 15) & ~(size_t)15) + (size_t)p.n_dp * sizeof(double);
}

// launches (jtree.hip); L = lanes per sequence unit (16, 32 or 64)
int jt_w_launch(const JtRun& r, double* w_out, int L, hipStream_t st);
int jt_filter_launch(const JtRun& r, int L, bool lds, int dirs, hipStream_t st);
int jt_post_launch(const JtRun& r, int L, bool lds, hipStream_t st);
int jt_add_launch(const double* src, double* dst, int n, hipStream_t st);
// workspace units per launch when the workspace lives in HBM (at most; the
// host lowers it so that the 2 x units slots stay within kJtGlobalBytes)
constexpr int kJtGlobalUnits = 4096;
constexpr size_t kJtGlobalBytes = (size_t)8 << 30;
inline int jt_global_units(int ws) {
  const size_t per = (size_t)2 * ws * sizeof(double);
  size_t u = per ? kJtGlobalBytes / per : kJtGlobalUnits;
  if (u > (size_t)kJtGlobalUnits) u = kJtGlobalUnits;
  u = u / 64 * 64;
  return u < 64 ? 64 : (int)u;
}

}  // namespace nipamd
