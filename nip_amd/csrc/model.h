// model.h -- host-side model representation of the nip_amd engine.
//
// A compiled DBN time slice: variables, join-tree cliques and sepsets with the
// exact indexing the reference produces, plus the GPU
// execution plan derived from it.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace nipamd {

// Interface flags, same bit values as src/nipvariable.h:31-34.
enum : int { IF_NONE = 0, IF_INCOMING = 1, IF_OUTGOING = 2, IF_OLD_OUTGOING = 4 };

struct Var {
  std::string symbol;
  int card = 0;
  std::vector<std::string> states;  // state names (the .net `states` field)
  std::string label = " ";          // v->name
  int pos_x = 100, pos_y = 100;
  int next = -1, previous = -1;     // next-slice / previous-slice variable
  std::vector<int> parents;         // v->parents order (reversed file order)
  bool has_prior = false;           // independent variable with a prior vector
  std::vector<double> prior;
  int ifs = IF_NONE;
  int family = -1;                  // nip_find_family(), memoised
  std::vector<int> family_mapping;  // nip_find_family_mapping(): child first
  int family_pos = -1;              // nip_clique_var_index(family, v)
};

struct Clique {
  std::vector<int> vars;            // ascending variable ID (= declaration order)
  std::vector<int> links;           // sepset indices, c->sepsets list order
  std::vector<double> original;     // original_p, dimension 0 fastest
};

struct Sepset {
  int a = -1, b = -1;               // first / second neighbour
  std::vector<int> vars;            // nip_variable_isect(a, b): a's order
};

// Parsed spec in Hugin-file order (what the grammar actions see).
struct NetSpec {
  std::vector<std::string> symbols;
  std::vector<int> card;
  std::vector<std::vector<std::string>> states;   // may be empty: names "0".."card-1"
  std::vector<std::string> labels;                // `label` (" " if absent, huginnet.y:328-329)
  std::vector<std::pair<int, int>> positions;     // `position` (100 100 if absent, huginnet.y:49-50)
  int node_size_x = 80, node_size_y = 60;         // net-level `node_size` (huginnet.y:51-52)
  std::vector<int> next;
  struct Pot { int child; std::vector<int> parents; std::vector<double> data; bool has_data; };
  std::vector<Pot> pots;
};

// Interface-chain plan: the slice reduces to a chain over its one interface
// variable (prev -> cur).  The in-clique holds prev, cur and hidden
// independent parents H of cur, which are summed out with their priors into
// the transition A[x][y] = sum_H orig(x, y, H) prod_h prior_h; every other
// clique is {cur, o} for a leaf child o of cur (an "emission" child, observed
// or not).  SURVEY 8(d) configs 2 (HMM), 3 (demo1, H = {D1}) and 5 (wide
// clique, H = {Y1, Z1}) are all of this shape.
struct ChainEmit {
  int var = -1;                     // the child variable
  int clique = -1;                  // its clique {cur, o}
  int M = 0;                        // card(o)
  std::vector<double> E;            // [M][64]: E[m*64 + y] = clique original at (cur = y, o = m)
  std::vector<double> s;            // [64]: sum_m E (factor of a missing observation)
};

struct ChainPlan {
  bool valid = false;
  int N = 0;                        // card(prev) == card(cur), <= 64
  int v_prev = -1, v_cur = -1;
  int c_trans = -1;                 // the in-clique
  std::vector<int> hidden;          // H
  std::vector<ChainEmit> emits;
  // evidence on cur itself (read_timeseries marks every variable, so data
  // files can observe the interface variable): an indicator "child" with
  // E = identity and s = 1, addressed as emit index emits.size()
  ChainEmit self;
  const ChainEmit& emit(int k) const { return k == (int)emits.size() ? self : emits[k]; }
  std::vector<double> A64;          // [64][64]
  std::vector<double> pi64;         // [64] prior of prev
  std::vector<double> s_all64;      // [64] product of every child's s
  // the 16-state layout of the same tables (N <= 16 kernels)
  std::vector<double> A;            // [16][16]
  std::vector<double> pi;           // [16]
  // classic HMM (exactly prev, cur and one child): the e_step plan
  bool hmm = false;
  // large in-cliques (>= kGpuFoldMin entries summed): A64 / A are folded on
  // the GPU when the engine first needs them (fold.hip), not here
  bool fold_gpu = false;
  bool folded = false;
  // joint interface chain (several interface variables, compile.cpp
  // build_joint_chain_plan): N = the joint interface's states, v_prev = v_cur =
  // -1, no hidden parents, emits = the observation candidates followed by one
  // indicator pseudo-child per interface variable; fb / filter only
  bool joint = false;
  std::vector<int> jprev;           // joint: previous_outgoing (their marginals: derive.hip kDerivePrev, projected)
  std::vector<int> jcur;            // joint: outgoing (their marginals: derive.hip kDeriveProject)
  // joint, <= 16 joint states, one observation candidate (emits[0]) and no
  // summed-out variable: the HMM e_step kernel runs on the joint state and the
  // finalize projects the joint counts onto every family (engine.cpp)
  bool jhmm = false;
};
constexpr long kGpuFoldMin = 1L << 22;
struct Model {
  std::vector<Var> vars;
  int node_size_x = 80, node_size_y = 60;
  std::vector<Clique> cliques;
  std::vector<Sepset> sepsets;
  int in_clique = -1, out_clique = -1;
  std::vector<int> outgoing, previous_outgoing, independent, children;

  ChainPlan chain;
  // device-side state (engine.cpp) and the general engine's caches (jtree_plan.cpp)
  void* dev = nullptr;
  void* jt = nullptr;
};

// compile.cpp
int compile_model(const NetSpec& spec, Model& m, std::string& err);
// Pure join-tree compilation of an explicit graph (used by tests: the
// reference's test/graphtest.c Test 7 builds a graph without parent lists).
int compile_graph_only(int n, const std::vector<int>& card,
                       const std::vector<std::pair<int, int>>& edges,
                       bool set_parents, std::vector<std::vector<int>>& cliques_out,
                       std::string& err);
std::string model_desc_json(const Model& m);
int param_size(const Model& m);
void build_chain_plan(Model& m);
// [card(h_j)][64][64]: the in-clique folded under the priors over every
// hidden parent but h_j, at h_j = d (sum_d G[d] = A64); derived marginals
void hidden_table(const Model& m, int j, std::vector<double>& G);
int m_step(Model& m, const double* params);

// netfile.cpp
int parse_net_file(const std::string& text, NetSpec& spec, std::string& err);
// engine.cpp: record the message behind a C-ABI error code (nipamd_last_error)
int set_error(int code, const std::string& msg);
// netwrite.cpp: write_model (src/nip.c:298-484)
int write_net_file(const Model& m, const std::string& path, std::string& err);

}  // namespace nipamd

// The opaque handle of the C-ABI (include/nip_amd.h).
struct nipamd_model {
  nipamd::Model m;
  unsigned version = 1;          // bumped whenever the tables change
  int engine = 0;                // NIPAMD_ENGINE_* (nipamd_model_set_engine)
  double fold_ms = 0.0;          // the last GPU fold: kernel time and clique bytes streamed
  double fold_bytes = 0.0;
  void* lik = nullptr;           // likelihood.hip: device tables of the last column set
  void* op = nullptr;            // opchain.cpp: evidence-indexed chain plans
  // prefix.cpp: the e_step's leading-missing-run verdict for `version`, valid
  // for T <= pf_T (-1: none below pf_T; -2: not decided, model too large)
  unsigned pf_version = 0;
  int pf_T = 0, pf_first_bad = -1;
};

namespace nipamd {
// fold.hip: the chain plan's transition (keep = -1: A [64][64]) or hidden
// parent j's table (keep = j: G_j [card][64][64]) summed on the current GPU
int chain_fold_gpu(const Model& m, int keep, std::vector<double>& out, double* ms, double* bytes,
                   std::string& err);
// engine.cpp: complete a deferred fold (ChainPlan::fold_gpu) before host use of A64
int ensure_fold(nipamd_model* mm);
// prefix.cpp: the first step k < T at which the reference's e_step rejects a
// series that observed nothing at steps 0..k (-1: none)
int estep_prefix_first_bad(const Model& m, int T, int* steps);
long estep_prefix_entries(const Model& m);
// likelihood.hip: drop a model's cached likelihood tables (nipamd_model_free)
void likelihood_release(nipamd_model* mm);
// generate.cpp: drop a model's cached generate_data tables (nipamd_model_free)
void generate_release(const nipamd_model* mm);
// opchain.cpp: the evidence-indexed interface chain (opchain.h)
bool op_supported(nipamd_model* mm, int n_obs, const int* obs_vars, int n_query, const int* query,
                  std::string& why);
int op_fb(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T, double* d_joint,
          long jbs, int jts, int joff, double* d_ll, uint32_t* d_status, void* stream, bool filt, int* K_out,
          std::string& err);
bool op_fits(nipamd_model* mm, int n_obs, const int* obs_vars, int T);
// its e_step: a partial section of op_estep_section doubles after the route tag
bool op_estep_supported(nipamd_model* mm, int n_obs, const int* obs_vars, int T, std::string& why);
long op_estep_section(nipamd_model* mm, int n_obs, const int* obs_vars);
int op_estep_partial(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T,
                     double* d_sec, double* d_ll, uint32_t* d_status, void* stream, std::string& err);
int op_estep_finalize(nipamd_model* mm, const double* d_sec, double* d_counts, void* stream, std::string& err);
void op_release(nipamd_model* mm);
// jtree_plan.cpp: the general join-tree engine (jtree.h)
int jt_supported(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query,
                 const int* query, std::string& why);
int jt_fb(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B, int T,
          int n_query, const int* query, double* d_post, double* d_ll, uint32_t* d_status,
          void* stream, bool filt);
int jt_estep_partial(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars, int B,
                     int T, double* d_partial, double* d_ll, uint32_t* d_status, void* stream);
int jt_estep_finalize(const nipamd_model* mm, const double* d_partial, double* d_counts, void* stream);
void jt_release(nipamd_model* mm);
int jt_plan_dump(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query, const int* query,
                 int estep, int* hdr, int hdr_cap, int* ip, long ip_cap, double* dp, long dp_cap,
                 long* sizes);
}  // namespace nipamd
