// nipamd_train -- counterpart of the reference's util/niptrain.c on the
// batched GPU e_step (config 4's EM on one GPU).
//
//   nipamd_train <MODEL.NET> <DATA.TXT> <THRESHOLD> <MIN_LL> <RESULT.NET>
//
// Same flow and output as niptrain: every variable with a data column is
// evidence; em_learn from random parameters (rand() seeded like
// random_seed(NULL), nip.c:2482-2502, or by NIPAMD_SEED) is restarted until it
// ends without BAD_LUCK at an average log-likelihood >= MIN_LL; the run
// summaries and the learning curve are printed as niptrain prints them
// (niptrain.c:120-205) and the model is written with write_model.
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <vector>

#include "nip_amd.h"

static long random_seed() {                     // nip.c:2482-2502 with seedpointer == NULL
  if (const char* e = std::getenv("NIPAMD_SEED")) {
    const long s = std::strtol(e, nullptr, 10);
    std::srand((unsigned)s);
    return s;
  }
  const time_t now = std::time(nullptr);
  const struct tm* t = std::localtime(&now);
  long seed = t->tm_sec + 60 * t->tm_min + 3600 * t->tm_hour;
  seed ^= (getpid() + (getpid() << 15));
  std::srand((unsigned)seed);
  return seed;
}

int main(int argc, char* argv[]) {
  std::printf("nipamd_train:\n");
  if (argc < 6) {
    std::printf("You must specify: \n");
    std::printf(" - the original NET file, \n");
    std::printf(" - data file, \n");
    std::printf(" - threshold value (0...1), \n");
    std::printf(" - minimum required log. likelihood/time step (<<0), and \n");
    std::printf(" - file name for the resulting model, please!\n");
    return 0;
  }
  nipamd_model* m = nullptr;
  if (nipamd_model_from_net(argv[1], &m) != NIP_NO_ERROR) {
    std::fprintf(stderr, "Unable to parse the NET file: %s? (%s)\n", argv[1], nipamd_last_error());
    return -1;
  }
  nipamd_series* s = nullptr;
  if (nipamd_read_timeseries(m, argv[2], &s) != NIP_NO_ERROR) {
    std::fprintf(stderr, "Unable to parse the data file: %s?\n", argv[2]);
    nipamd_model_free(m);
    return -1;
  }
  const int n = nipamd_series_count(s), k = nipamd_series_num_observed(s), nv = nipamd_model_num_vars(m);
  std::vector<int> ov(k > 0 ? k : 1);
  nipamd_series_observed(s, ov.data());
  std::printf("  Hidden variables are:\n");
  char name[256];
  for (int v = 0; v < nv; v++) {
    bool seen = false;
    for (int i = 0; i < k; i++) seen |= ov[i] == v;
    if (!seen) {
      nipamd_model_var_symbol(m, v, name, sizeof name);
      std::printf("  %s", name);
    }
  }
  std::printf("\n  Observed variables are:\n");
  for (int i = 0; i < k; i++) {
    nipamd_model_var_symbol(m, ov[i], name, sizeof name);
    std::printf("  %s", name);
  }
  std::printf("\n");

  char* tail = nullptr;
  const double threshold = std::strtod(argv[3], &tail);
  if (threshold <= 0.0 || threshold > 1 || tail == argv[3]) {
    std::fprintf(stderr, "Specify a valid threshold value: %s?\n", argv[3]);
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }
  tail = nullptr;
  const double min_ll = std::strtod(argv[4], &tail);
  if (min_ll >= 0.0 || tail == argv[4]) {
    std::fprintf(stderr, "Specify a valid value for minimum log. likelihood");
    std::fprintf(stderr, " / time step: %s?\n", argv[4]);
    nipamd_series_free(s);
    nipamd_model_free(m);
    return -1;
  }

  std::printf("  Computing... \n");
  std::printf("  Random seed = %ld\n", random_seed());
  std::vector<int> len(n);
  size_t rows = 0;
  for (int i = 0; i < n; i++) rows += (size_t)(len[i] = nipamd_series_length(s, i));
  std::vector<int32_t> obs(rows * (k > 0 ? k : 1));
  size_t off = 0;
  for (int i = 0; i < n && k > 0; i++) {
    const int32_t* d = nipamd_series_data(s, i);
    std::copy(d, d + (size_t)len[i] * k, obs.begin() + off);
    off += (size_t)len[i] * k;
  }
  std::vector<double> curve(100000);
  int nc = 0, e = 0, t = 0;
  double last = 0;
  do {
    t++;
    last = 0;
    e = nipamd_em_learn(m, n, len.data(), obs.data(), k, ov.data(), threshold, nullptr, 0,
                        curve.data(), (int)curve.size(), &nc);
    if (!(e == NIP_NO_ERROR || e == NIP_ERROR_BAD_LUCK)) {
      std::fprintf(stderr, "There were errors during learning: %s\n", nipamd_last_error());
      nipamd_series_free(s);
      nipamd_model_free(m);
      return -1;
    }
    if (nc == 0) {
      std::printf("  Run %d failed 0.0  with 0 iterations, delta = 0.0 \n", t);
    } else {
      last = curve[nc - 1];
      if (nc > 1)
        std::printf("  Run %d reached %g  with %d iterations, delta = %g \n", t, last, nc, last - curve[nc - 2]);
      else
        std::printf("  Run %d reached %g  with %d iterations, delta = 0.0 \n", t, last, nc);
    }
  } while (e == NIP_ERROR_BAD_LUCK || last < min_ll);
  std::printf("  ...done.\n");
  for (int i = 0; i < nc; i++)
    std::printf("  Iteration %d: \t average loglikelihood = %g\n", i, std::rint(curve[i] / threshold) * threshold);

  const int rc = nipamd_write_model(m, argv[5]);
  if (rc != NIP_NO_ERROR) std::fprintf(stderr, "Failed to write the model into %s\n", argv[5]);
  nipamd_series_free(s);
  nipamd_model_free(m);
  return rc == NIP_NO_ERROR ? 0 : -1;
}
