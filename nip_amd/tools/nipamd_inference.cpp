// nipamd_inference -- counterpart of the reference's util/nipinference.c on
// the batched GPU engine.
//
//   nipamd_inference <MODEL.NET> <INPUT_DATA.TXT> <VARIABLE> <OUTPUT_DATA.TXT>
//
// Same behaviour and output as nipinference: every variable with a data
// column is evidence (nip_mark_variable on all, nipinference.c:115-116), the
// smoothed marginals of VARIABLE are written with write_uncertainseries
// (state names, "%f" rows, a blank line after each series) and the average
// over series of (log-likelihood / length) is printed (nipinference.c:124-136).
// The series are batched by length, one nipamd_fb_host call per length, so
// every series is computed exactly as on its own.  Models or requests outside
// the GPU plan fail with the engine's message; there is no CPU path.
#include <cstdio>
#include <map>
#include <vector>

#include "nip_amd.h"

int main(int argc, char* argv[]) {
  std::printf("nipamd_inference:\n");
  if (argc < 5) {
    std::printf("Specify the names of the net file, input data file, ");
    std::printf("variable, and output data file.\n");
    return 0;
  }
  nipamd_model* m = nullptr;
  if (nipamd_model_from_net(argv[1], &m) != NIP_NO_ERROR) {
    std::fprintf(stderr, "%s: %s\n", argv[1], nipamd_last_error());
    return -1;
  }
  nipamd_series* s = nullptr;
  if (nipamd_read_timeseries(m, argv[2], &s) != NIP_NO_ERROR || nipamd_series_count(s) < 1) {
    std::fprintf(stderr, "%s: %s\n", argv[2], nipamd_last_error());
    nipamd_model_free(m);
    return -1;
  }
  const int v = nipamd_model_var_index(m, argv[3]);
  if (v < 0) {
    std::fprintf(stderr, "No such variable (%s) in the model.\n", argv[3]);
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  const int n = nipamd_series_count(s), k = nipamd_series_num_observed(s), card = nipamd_model_var_card(m, v);
  std::vector<int> ov(k > 0 ? k : 1);
  nipamd_series_observed(s, ov.data());

  std::printf("  Computing...\n");
  std::map<int, std::vector<int>> by_len;          // length -> series
  std::vector<int> len(n);
  for (int i = 0; i < n; i++) by_len[len[i] = nipamd_series_length(s, i)].push_back(i);
  std::vector<size_t> row0(n + 1, 0);
  for (int i = 0; i < n; i++) row0[i + 1] = row0[i] + len[i];
  std::vector<double> post(row0[n] * card), ll(n);
  int rc = NIP_NO_ERROR;
  for (const auto& [T, ids] : by_len) {
    const int B = (int)ids.size();
    std::vector<int32_t> obs((size_t)B * T * (k > 0 ? k : 1), -1);
    for (int b = 0; b < B && k > 0; b++) {
      const int32_t* d = nipamd_series_data(s, ids[b]);
      std::copy(d, d + (size_t)T * k, obs.begin() + (size_t)b * T * k);
    }
    std::vector<double> p((size_t)B * T * card), l(B);
    std::vector<uint32_t> st(B);
    rc = nipamd_fb_host(m, obs.data(), k, ov.data(), B, T, 1, &v, p.data(), l.data(), st.data());
    if (rc != NIP_NO_ERROR) break;
    for (int b = 0; b < B; b++) {
      std::copy(p.begin() + (size_t)b * T * card, p.begin() + (size_t)(b + 1) * T * card,
                post.begin() + row0[ids[b]] * card);
      ll[ids[b]] = l[b];
    }
  }
  if (rc != NIP_NO_ERROR) {
    std::fprintf(stderr, "nipamd_inference: %s\n", nipamd_last_error());
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  double avg = 0.0;
  for (int i = 0; i < n; i++) avg += ll[i] / len[i];
  avg /= n;
  rc = nipamd_write_uncertainseries(m, argv[4], v, n, len.data(), post.data(), card, 0);
  if (rc != NIP_NO_ERROR) std::fprintf(stderr, "%s: %s\n", argv[4], nipamd_last_error());
  std::printf("  Average log. likelihood = %g\n", avg);
  std::printf("  ...done.\n");
  nipamd_series_free(s);
  nipamd_model_free(m);
  return rc == NIP_NO_ERROR ? 0 : -1;
}
