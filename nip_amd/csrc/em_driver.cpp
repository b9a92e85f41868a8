// em_driver.cpp -- em_learn (src/nip.c:2076-2243) over the batched GPU e_step,
// for a set of series of any lengths on one GPU (the niptrain counterpart;
// the data-parallel multi-GPU driver is nip_amd/em.py).
//
// The reference's loop exactly: random initial parameters rand()/RAND_MAX in
// the em_learn layout (nippotential.c:222-229, the caller seeds srand as
// niptrain does with random_seed, nip.c:2482-2502), m_step first, counts
// start at 1.0 (nip.c:2172), the log-likelihood summed over the series in
// their order, the learning curve of average log-likelihood per time step,
// BAD_LUCK on an e_step failure or on a decreasing / positive / -inf
// likelihood (nip.c:2182-2234), and the stopping rule with
// MIN_EM_ITERATIONS = 3 (nip.c:29, 2240-2241).  The per-series e_step loop is
// one batched nipamd_estep_host call per distinct series length.
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "model.h"
#include "nip_amd.h"

namespace {
constexpr int kMinEmIterations = 3;   // src/nip.c:29
}

extern "C" int nipamd_em_learn(nipamd_model* m, int n_series, const int* lengths, const int32_t* obs,
                               int n_obs, const int* obs_vars, double threshold, const double* init,
                               int max_iterations, double* curve, int curve_cap, int* curve_len) {
  if (curve_len) *curve_len = 0;
  if (!m || n_series <= 0 || !lengths || (n_obs > 0 && (!obs || !obs_vars)))
    return nipamd::set_error(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const int P = nipamd_model_param_size(m);
  if (P <= 0) return nipamd::set_error(NIP_ERROR_INVALID_ARGUMENT, "model has no parameters");
  std::vector<double> params(P);
  for (int i = 0; i < P; i++) params[i] = init ? init[i] : std::rand() / (double)RAND_MAX;

  // series grouped by length, packed once ([B][T][n_obs] per group)
  std::vector<size_t> row0(n_series + 1, 0);
  for (int i = 0; i < n_series; i++) {
    if (lengths[i] < 1) return nipamd::set_error(NIP_ERROR_INVALID_ARGUMENT, "empty series");
    row0[i + 1] = row0[i] + (size_t)lengths[i];
  }
  struct Group { int T; std::vector<int> ids; std::vector<int32_t> obs; };
  std::map<int, Group> groups;
  for (int i = 0; i < n_series; i++) {
    Group& g = groups[lengths[i]];
    g.T = lengths[i];
    g.ids.push_back(i);
    if (n_obs > 0)
      g.obs.insert(g.obs.end(), obs + row0[i] * n_obs, obs + row0[i + 1] * n_obs);
    else
      g.obs.insert(g.obs.end(), (size_t)lengths[i], -1);
  }
  const double ts_steps = (double)row0[n_series];             // nip.c:2141-2143

  double loglikelihood = -DBL_MAX;                            // nip.c:2082
  std::vector<double> counts(P), lls(n_series);
  int it = 0, n_curve = 0;
  for (;;) {
    int rc = nipamd_m_step(m, params.data());                 // nip.c:2154
    if (rc) return rc;
    const double old = loglikelihood;
    std::fill(counts.begin(), counts.end(), 1.0);             // nip.c:2172
    for (auto& kv : groups) {
      Group& g = kv.second;
      const int B = (int)g.ids.size();
      std::vector<double> l(B);
      std::vector<uint32_t> st(B);
      rc = nipamd_estep_host(m, g.obs.data(), n_obs, obs_vars, B, g.T, counts.data(), l.data(), st.data());
      if (rc) return rc;
      for (int b = 0; b < B; b++) {
        if (st[b]) return NIP_ERROR_BAD_LUCK;                 // e_step failure, nip.c:2182-2198
        lls[g.ids[b]] = l[b];
      }
    }
    loglikelihood = 0.0;
    for (int i = 0; i < n_series; i++) loglikelihood += lls[i];   // series order, as the reference
    params = counts;
    if (curve && n_curve < curve_cap) curve[n_curve] = loglikelihood / ts_steps;
    n_curve++;
    if (curve_len) *curve_len = n_curve < curve_cap ? n_curve : curve_cap;
    if (old > loglikelihood + ts_steps * threshold || loglikelihood > 0 || std::isinf(loglikelihood))
      return NIP_ERROR_BAD_LUCK;                              // nip.c:2224-2234
    it++;
    if (max_iterations > 0 && it >= max_iterations) return NIP_NO_ERROR;
    if (!((loglikelihood - old) > ts_steps * threshold || it < kMinEmIterations)) return NIP_NO_ERROR;
  }
}
