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
  std::vector<int> next;
  struct Pot { int child; std::vector<int> parents; std::vector<double> data; bool has_data; };
  std::vector<Pot> pots;
};

// Chain plan: the slice is an HMM over one interface variable
// (SURVEY 8(d) config 2): transition table A[x][y] = in_clique original over
// (previous x, current y), emission table E[y][m] = the observation clique's
// original over (current y, observed m), prior pi over the previous-slice
// variable.  Padded to 16 states for the gfx950 kernels.
struct ChainPlan {
  bool valid = false;
  int N = 0, M = 0;                 // hidden / observed cardinalities
  int v_prev = -1, v_cur = -1, v_obs = -1;
  int c_trans = -1, c_emit = -1;
  std::vector<double> A;            // [16][16]  A[x*16+y]
  std::vector<double> Etab;         // [(M+2)][16]: rows 0..M-1 = E[.,m], M = column sums (missing), M+1 = 0
  std::vector<double> pi;           // [16]
  std::vector<double> ts;           // [16]  ts[x] = sum_y A[x][y] * s[y]
};

struct Model {
  std::vector<Var> vars;
  std::vector<Clique> cliques;
  std::vector<Sepset> sepsets;
  int in_clique = -1, out_clique = -1;
  std::vector<int> outgoing, previous_outgoing, independent, children;

  ChainPlan chain;
  // device-side state (engine.cpp)
  void* dev = nullptr;
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
int m_step(Model& m, const double* params);

// netfile.cpp
int parse_net_file(const std::string& text, NetSpec& spec, std::string& err);

}  // namespace nipamd
