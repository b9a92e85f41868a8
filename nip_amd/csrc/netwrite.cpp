// netwrite.cpp -- write_model (src/nip.c:298-484): the model as a Hugin .net
// file, in the reference's exact layout (the niptrain counterpart writes the
// learned model with it).
//
//   net { node_size = (x y); }
//   one `node` block per variable (label, position, states, NIP_next of the
//     variable's `previous`, nip.c:361-363);
//   the priors of the independent variables ("%f  " values, 7 per line);
//   one conditional table per child: the family clique's original_p
//     marginalised onto (child, parents...) with the family mapping
//     (nip_general_marginalise, nippotential.c:267-311), normalised along the
//     child (nip_normalise_cpd, :363-383), parents printed in reverse order,
//     " %f " values, a new line at every new parent configuration (with a
//     comment naming it) and every 7 values when the child has more than 7
//     states (POTENTIAL_ELEMENTS_PER_LINE, nip.c:26).
#include <cstdio>
#include <string>
#include <vector>

#include "model.h"
#include "nip_amd.h"

namespace nipamd {

namespace {

constexpr int kPerLine = 7;   // POTENTIAL_ELEMENTS_PER_LINE, nip.c:26

// dest[choose(idx)] += src[i] over the clique in flat order (dimension 0 fastest)
std::vector<double> family_table(const Model& m, int v) {
  const Var& V = m.vars[v];
  const Clique& c = m.cliques[V.family];
  std::vector<int> ccard;
  for (int u : c.vars) ccard.push_back(m.vars[u].card);
  std::vector<int> dcard = {V.card};
  for (int p : V.parents) dcard.push_back(m.vars[p].card);
  size_t dsize = 1;
  for (int d : dcard) dsize *= (size_t)d;
  std::vector<double> dest(dsize, 0.0);
  std::vector<int> idx(ccard.size(), 0);
  for (size_t i = 0; i < c.original.size(); i++) {
    size_t di = 0, stride = 1;
    for (size_t k = 0; k < dcard.size(); k++) {
      di += (size_t)idx[V.family_mapping[k]] * stride;
      stride *= (size_t)dcard[k];
    }
    dest[di] += c.original[i];
    for (size_t k = 0; k < idx.size(); k++) {            // next clique index
      if (++idx[k] < ccard[k]) break;
      idx[k] = 0;
    }
  }
  // nip_normalise_cpd: along dimension 0 for every parent configuration, no-op on a zero sum
  for (size_t b = 0; b < dsize; b += (size_t)V.card) {
    double sum = 0.0;
    for (int x = 0; x < V.card; x++) sum += dest[b + x];
    if (sum != 0.0)
      for (int x = 0; x < V.card; x++) dest[b + x] /= sum;
  }
  return dest;
}

}  // namespace

int write_net_file(const Model& m, const std::string& path, std::string& err) {
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) { err = "cannot write " + path; return NIP_ERROR_IO; }
  std::fputs("net\n", f);
  std::fputs("{\n", f);
  std::fprintf(f, "    node_size = (%d %d);\n", m.node_size_x, m.node_size_y);
  std::fputs("}\n", f);

  for (const Var& v : m.vars) {
    const int n = v.card - 1;
    std::fputs("\n", f);
    std::fprintf(f, "node %s\n", v.symbol.c_str());
    std::fputs("{\n", f);
    std::fprintf(f, "    label = \"%s\";\n", v.label.c_str());
    std::fprintf(f, "    position = (%d %d);\n", v.pos_x, v.pos_y);
    std::fputs("    states = (", f);
    for (int j = 0; j < n; j++) std::fprintf(f, " \"%s\" \n              ", v.states[j].c_str());
    std::fprintf(f, " \"%s\" );\n", v.states[n].c_str());
    if (v.previous >= 0) std::fprintf(f, "    NIP_next = \"%s\";\n", m.vars[v.previous].symbol.c_str());
    std::fputs("}\n", f);
  }

  for (int iv : m.independent) {
    const Var& v = m.vars[iv];
    std::fputs("\n", f);
    std::fprintf(f, "potential (%s)\n", v.symbol.c_str());
    std::fputs("{\n", f);
    std::fputs("    data = ( ", f);
    for (int j = 0; j < v.card; j++) {
      if (j > 0 && (j % kPerLine) == 0) std::fputs("\n             ", f);
      std::fprintf(f, "%f  ", j < (int)v.prior.size() ? v.prior[j] : 0.0);
    }
    std::fputs(");\n", f);
    std::fputs("}\n", f);
  }

  for (int ic : m.children) {
    const Var& v = m.vars[ic];
    const int np = (int)v.parents.size();
    std::fputs("\n", f);
    std::fprintf(f, "potential (%s | ", v.symbol.c_str());
    for (int j = np - 1; j > 0; j--) std::fprintf(f, "%s ", m.vars[v.parents[j]].symbol.c_str());
    std::fprintf(f, "%s)\n", m.vars[v.parents[0]].symbol.c_str());
    std::fputs("{ \n", f);
    std::fputs("    data = (", f);
    const std::vector<double> p = family_table(m, ic);
    int y = 0;
    for (size_t j = 0; j < p.size(); j++) {
      const bool n = (j % (size_t)v.card) == 0;     // a new parent configuration
      if (j > 0 && (n || (v.card > kPerLine && y % kPerLine == 0))) {
        if (n) {
          // comment naming the previous line's parent values (nip_inverse_mapping of j-1)
          std::fputs(" % ", f);
          size_t r = (j - 1) / (size_t)v.card;
          std::vector<int> pv(np);
          for (int k = 0; k < np; k++) {
            const int ck = m.vars[v.parents[k]].card;
            pv[k] = (int)(r % (size_t)ck);
            r /= (size_t)ck;
          }
          for (int x = np - 1; x >= 0; x--)
            std::fprintf(f, "%s=%s ", m.vars[v.parents[x]].symbol.c_str(),
                         m.vars[v.parents[x]].states[pv[x]].c_str());
        }
        std::fputs("\n            ", f);
        y = 0;
      }
      std::fprintf(f, " %f ", p[j]);
      y++;
    }
    std::fputs(");\n", f);
    std::fputs("}\n", f);
  }
  if (std::fclose(f)) { err = "cannot close " + path; return NIP_ERROR_IO; }
  return NIP_NO_ERROR;
}

}  // namespace nipamd

extern "C" int nipamd_write_model(const nipamd_model* mm, const char* path) {
  if (!mm || !path) return NIP_ERROR_NULLPOINTER;
  std::string err;
  const int rc = nipamd::write_net_file(mm->m, path, err);
  if (rc) nipamd::set_error(rc, err);
  return rc;
}
