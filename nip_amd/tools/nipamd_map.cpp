// nipamd_map -- counterpart of the reference's util/nipmap.c on the batched
// GPU engine.
//
//   nipamd_map <MODEL.NET> <INPUT_DATA.TXT> <OUTPUT_DATA.TXT>
//
// The maximum a posteriori state of every hidden variable (the model's
// variables without a data column, in model order: read_timeseries,
// nip.c:578-589) at every time step, from the smoothed marginals of all of
// them at once (nipmap.c:145).  The output has nipmap.c's layout: the hidden
// variables' symbols on the first line, then per time step each variable's
// MAP state name followed by one space (the last one by " \n"), and an empty
// line after each series (nipmap.c:124-178).  The MAP state is the first
// state whose marginal is strictly greater than every earlier one, starting
// from 0 (state 0 for an all-zero marginal), as nipmap.c:154-160.  Series are
// batched by length, one nipamd_fb_host call per length.
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "nip_amd.h"

static std::string symbol(const nipamd_model* m, int v) {
  char buf[256];
  nipamd_model_var_symbol(m, v, buf, sizeof buf);
  return buf;
}

static std::string state(const nipamd_model* m, int v, int s) {
  char buf[256];
  nipamd_model_state_name(m, v, s, buf, sizeof buf);
  return buf;
}

int main(int argc, char* argv[]) {
  std::printf("nipamd_map:\n");
  if (argc < 4) {
    std::printf("Specify the names of the net file and input/output data files.\n");
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
    if (s) nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  const int nv = nipamd_model_num_vars(m), n = nipamd_series_count(s), k = nipamd_series_num_observed(s);
  std::vector<int> ov(k > 0 ? k : 1);
  nipamd_series_observed(s, ov.data());
  std::vector<int> hidden;
  for (int v = 0; v < nv; v++) {
    bool seen = false;
    for (int i = 0; i < k; i++) seen |= ov[i] == v;
    if (!seen) hidden.push_back(v);
  }
  FILE* f = std::fopen(argv[3], "w");
  if (!f) {
    std::fprintf(stderr, "%s: cannot open\n", argv[3]);
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  if (hidden.empty()) {
    std::fprintf(stderr, "No hidden variables to estimate.\n");
    std::fclose(f);
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  std::printf("  Observed variables:\n  ");
  for (int i = 0; i < k; i++) std::printf("%s ", symbol(m, ov[i]).c_str());
  std::printf("\n  Hidden variables:\n  ");
  for (int v : hidden) std::printf("%s ", symbol(m, v).c_str());
  std::printf("\n");
  std::fprintf(f, "%s", symbol(m, hidden[0]).c_str());
  for (size_t i = 1; i < hidden.size(); i++) std::fprintf(f, " %s", symbol(m, hidden[i]).c_str());
  std::fputs("\n", f);

  std::printf("  Computing...\n");
  std::vector<int> card(hidden.size()), off(hidden.size());
  int stride = 0;
  for (size_t i = 0; i < hidden.size(); i++) {
    card[i] = nipamd_model_var_card(m, hidden[i]);
    off[i] = stride;
    stride += card[i];
  }
  std::map<int, std::vector<int>> by_len;          // length -> series
  std::vector<int> len(n);
  for (int i = 0; i < n; i++) by_len[len[i] = nipamd_series_length(s, i)].push_back(i);
  std::vector<std::vector<double>> post(n);
  int rc = NIP_NO_ERROR;
  for (const auto& [T, ids] : by_len) {
    const int B = (int)ids.size();
    std::vector<int32_t> obs((size_t)B * T * (k > 0 ? k : 1), -1);
    for (int b = 0; b < B && k > 0; b++) {
      const int32_t* d = nipamd_series_data(s, ids[b]);
      std::copy(d, d + (size_t)T * k, obs.begin() + (size_t)b * T * k);
    }
    std::vector<double> p((size_t)B * T * stride), l(B);
    std::vector<uint32_t> st(B);
    rc = nipamd_fb_host(m, obs.data(), k, ov.data(), B, T, (int)hidden.size(), hidden.data(),
                        p.data(), l.data(), st.data());
    if (rc != NIP_NO_ERROR) break;
    for (int b = 0; b < B; b++)
      post[ids[b]].assign(p.begin() + (size_t)b * T * stride, p.begin() + (size_t)(b + 1) * T * stride);
  }
  if (rc != NIP_NO_ERROR) {
    std::fprintf(stderr, "nipamd_map: %s\n", nipamd_last_error());
    std::fclose(f);
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  for (int i = 0; i < n; i++) {
    for (int t = 0; t < len[i]; t++) {
      const double* row = post[i].data() + (size_t)t * stride;
      for (size_t h = 0; h < hidden.size(); h++) {
        int best = 0;
        double m_max = 0.0;
        for (int j = 0; j < card[h]; j++)
          if (row[off[h] + j] > m_max) { m_max = row[off[h] + j]; best = j; }
        std::fprintf(f, h + 1 < hidden.size() ? "%s " : "%s \n", state(m, hidden[h], best).c_str());
      }
    }
    std::fputs("\n", f);
  }
  std::printf("  ...done\n");
  rc = std::fclose(f) ? -1 : 0;
  nipamd_series_free(s);
  nipamd_model_free(m);
  return rc;
}
