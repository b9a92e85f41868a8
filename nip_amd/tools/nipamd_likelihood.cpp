// nipamd_likelihood -- counterpart of the reference's util/niplikelihood.c on
// the GPU engine.
//
//   nipamd_likelihood <MODEL.NET> <DATA.TXT> <A> [B C ...]
//
// For every time step of every series, on its own: the mass after the
// evidence of the data columns that are not variables of interest (m1), after
// all columns (m2), and ln p(A B C | rest) = log(m2) - log(m1), printed as
// "%g %g %g" per step with an empty line after each series, as
// niplikelihood.c:111-135 does.  Series are batched by length (one
// nipamd_likelihood_host call per length).
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "nip_amd.h"

int main(int argc, char* argv[]) {
  std::printf("nipamd_likelihood:\n");
  if (argc < 4) {
    std::printf("You must specify: \n");
    std::printf(" - the NET file, e.g. model.net, \n");
    std::printf(" - the data file, e.g. data.txt, and \n");
    std::printf(" - variable(s) of interest, e.g. A B C \n");
    return 0;
  }
  nipamd_model* m = nullptr;
  if (nipamd_model_from_net(argv[1], &m) != NIP_NO_ERROR) {
    std::fprintf(stderr, "Unable to parse the NET file: %s?\n", argv[1]);
    return -1;
  }
  nipamd_series* s = nullptr;
  if (nipamd_read_timeseries(m, argv[2], &s) != NIP_NO_ERROR || nipamd_series_count(s) < 1) {
    std::fprintf(stderr, "Unable to parse the data file: %s?\n", argv[2]);
    if (s) nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  const int n = nipamd_series_count(s), k = nipamd_series_num_observed(s);
  std::vector<int> ov(k > 0 ? k : 1), marked(k > 0 ? k : 1, 0);
  nipamd_series_observed(s, ov.data());
  for (int a = 3; a < argc; a++) {           // unknown symbols are ignored (niplikelihood.c:92-108)
    const int v = nipamd_model_var_index(m, argv[a]);
    for (int i = 0; i < k; i++)
      if (ov[i] == v) marked[i] = 1;
  }
  std::map<int, std::vector<int>> by_len;
  std::vector<int> len(n);
  for (int i = 0; i < n; i++) by_len[len[i] = nipamd_series_length(s, i)].push_back(i);
  std::vector<std::vector<double>> res(n);
  int rc = NIP_NO_ERROR;
  for (const auto& [T, ids] : by_len) {
    const int B = (int)ids.size();
    std::vector<int32_t> obs((size_t)B * T * (k > 0 ? k : 1), -1);
    for (int b = 0; b < B && k > 0; b++) {
      const int32_t* d = nipamd_series_data(s, ids[b]);
      std::copy(d, d + (size_t)T * k, obs.begin() + (size_t)b * T * k);
    }
    std::vector<double> m1((size_t)B * T), m2(m1.size()), ll(m1.size());
    rc = nipamd_likelihood_host(m, obs.data(), k, ov.data(), marked.data(), B, T, m1.data(), m2.data(),
                                ll.data());
    if (rc != NIP_NO_ERROR) break;
    for (int b = 0; b < B; b++) {
      auto& r = res[ids[b]];
      for (int t = 0; t < T; t++) {
        const size_t i = (size_t)b * T + t;
        r.insert(r.end(), {m1[i], m2[i], ll[i]});
      }
    }
  }
  if (rc != NIP_NO_ERROR) {
    std::fprintf(stderr, "nipamd_likelihood: %s\n", nipamd_last_error());
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  for (int i = 0; i < n; i++) {
    for (int t = 0; t < len[i]; t++)
      std::printf("%g %g %g\n", res[i][3 * t], res[i][3 * t + 1], res[i][3 * t + 2]);
    std::printf("\n");
  }
  nipamd_series_free(s);
  nipamd_model_free(m);
  return 0;
}
