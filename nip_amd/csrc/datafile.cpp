// datafile.cpp -- the time-series data files around the hot path (SURVEY
// 8(f) row 2): reading observations for a batch and writing posteriors.
//
// Restates the reference's text format exactly:
//  * tokens (nipstring.c:36-99 nip_count_tokens / :101- nip_tokenise with
//    q_strings = 0, sep_tokens = 0, wspace_sep = 1): maximal runs of
//    characters that are neither white space nor the field separator ','
//    (NIP_FIELD_SEPARATOR, nip.h:54); empty fields vanish;
//  * structure (nipparsers.c:48-367 nip_open_data_file, nodenames = 1): the
//    first non-empty line holds the node symbols; empty lines before it and
//    right after it are ignored; after the first data line, one or more empty
//    lines end a time series; lines are read with a 10000-byte buffer
//    (MAX_LINELENGTH, nipparsers.h:30);
//  * values (nip.c:512-667 read_timeseries): columns whose symbol is not a
//    model variable are skipped; the others are the observed variables, in
//    file order; a token is the index of the equal state name, else -1
//    (missing: "null", "N/A", "<null>" or anything unknown,
//    nipvariable.c:239-247); a line with fewer tokens than symbols leaves the
//    remaining observed entries at 0 (calloc'd, nip.c:620-651: the loop stops
//    at the short line's end);
//  * output (nip.c:815-893 write_uncertainseries): the state names joined by
//    ',', then one line of "%f" probabilities per time step, a blank line
//    after each series.
// Batches for the GPU are assembled by the caller (nip_amd/tools, Python).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "model.h"
#include "nip_amd.h"

struct nipamd_series {
  std::vector<int> obs_vars;           // model variable per observed column (file order)
  std::vector<int> lengths;            // per series
  std::vector<size_t> offset;          // first row of each series in data
  std::vector<int32_t> data;           // [sum lengths][n_obs]
};

namespace {

constexpr int kMaxLine = 10000;
constexpr char kSep = ',';

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

// tokens of one line, exactly as nip_tokenise(line, n, 0, ",", 1, 0, 1)
std::vector<std::string> tokens_of(const char* s) {
  std::vector<std::string> out;
  std::string cur;
  bool in = false;
  for (; *s; s++) {
    const char c = *s;
    if (c == kSep || is_space(c)) {
      if (in) { out.push_back(cur); cur.clear(); in = false; }
    } else {
      cur.push_back(c);
      in = true;
    }
  }
  if (in) out.push_back(cur);
  return out;
}

// fgets-style line reader with the reference's buffer size (a longer line
// continues as the next "line")
bool next_line(FILE* f, std::string& line) {
  char buf[kMaxLine];
  if (!std::fgets(buf, kMaxLine, f)) return false;
  line = buf;
  return true;
}

}  // namespace

extern "C" {

int nipamd_read_timeseries(const nipamd_model* mm, const char* path, nipamd_series** out) {
  if (!mm || !path || !out) return nipamd::set_error(NIP_ERROR_NULLPOINTER, "bad arguments");
  *out = nullptr;
  FILE* f = std::fopen(path, "r");
  if (!f) return nipamd::set_error(NIP_ERROR_FILENOTFOUND, std::string("cannot open ") + path);
  // one pass over the lines, with the two-pass reference's outcome
  std::vector<std::string> symbols;
  std::vector<std::vector<std::vector<std::string>>> series;   // [series][row][token]
  bool have_labels = false, in_series = false;
  std::string line;
  while (next_line(f, line)) {
    std::vector<std::string> toks = tokens_of(line.c_str());
    if (toks.empty()) {                 // an empty line ends the current series
      in_series = false;
      continue;
    }
    if (!have_labels) { symbols = toks; have_labels = true; continue; }
    if (!in_series) { series.emplace_back(); in_series = true; }
    series.back().push_back(std::move(toks));
  }
  std::fclose(f);
  if (!have_labels || series.empty())
    return nipamd::set_error(NIP_ERROR_INVALID_ARGUMENT, std::string("no time series in ") + path);

  const auto& V = mm->m.vars;
  auto var_of = [&](const std::string& sym) -> int {
    for (size_t v = 0; v < V.size(); v++) if (V[v].symbol == sym) return (int)v;
    return -1;
  };
  auto* s = new nipamd_series();
  std::vector<int> col_var(symbols.size());
  for (size_t i = 0; i < symbols.size(); i++) {
    col_var[i] = var_of(symbols[i]);
    if (col_var[i] >= 0) s->obs_vars.push_back(col_var[i]);
  }
  const size_t nobs = s->obs_vars.size();
  for (const auto& rows : series) {
    s->offset.push_back(s->data.size() / (nobs ? nobs : 1));
    s->lengths.push_back((int)rows.size());
    for (const auto& toks : rows) {
      std::vector<int32_t> rec(nobs, 0);           // calloc'd: a short line leaves zeros
      size_t k = 0;
      for (size_t i = 0; i < symbols.size(); i++) {
        if (i == toks.size()) break;              // the line was too short
        const int v = col_var[i];
        if (v < 0) continue;
        int idx = -1;
        for (int st = 0; st < V[v].card; st++)
          if (V[v].states[st] == toks[i]) { idx = st; break; }
        rec[k++] = idx;
      }
      s->data.insert(s->data.end(), rec.begin(), rec.end());
    }
  }
  *out = s;
  return NIP_NO_ERROR;
}

int nipamd_series_count(const nipamd_series* s) { return s ? (int)s->lengths.size() : -1; }

int nipamd_series_num_observed(const nipamd_series* s) { return s ? (int)s->obs_vars.size() : -1; }

int nipamd_series_observed(const nipamd_series* s, int* vars) {
  if (!s || !vars) return NIP_ERROR_NULLPOINTER;
  for (size_t i = 0; i < s->obs_vars.size(); i++) vars[i] = s->obs_vars[i];
  return NIP_NO_ERROR;
}

int nipamd_series_length(const nipamd_series* s, int i) {
  if (!s || i < 0 || i >= (int)s->lengths.size()) return -1;
  return s->lengths[i];
}

const int32_t* nipamd_series_data(const nipamd_series* s, int i) {
  if (!s || i < 0 || i >= (int)s->lengths.size() || s->obs_vars.empty()) return nullptr;
  return s->data.data() + s->offset[i] * s->obs_vars.size();
}

void nipamd_series_free(nipamd_series* s) { delete s; }

int nipamd_write_uncertainseries(const nipamd_model* mm, const char* path, int var, int n_series,
                                 const int* lengths, const double* post, int stride, int offset) {
  if (!mm || !path || !lengths || !post || n_series <= 0 || var < 0 || var >= (int)mm->m.vars.size())
    return nipamd::set_error(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const auto& v = mm->m.vars[var];
  if (offset < 0 || offset + v.card > stride) return nipamd::set_error(NIP_ERROR_INVALID_ARGUMENT, "bad stride");
  FILE* f = std::fopen(path, "w");
  if (!f) return nipamd::set_error(NIP_ERROR_IO, std::string("cannot write ") + path);
  for (int i = 0; i < v.card; i++) {
    if (i > 0) std::fputc(kSep, f);
    std::fputs(v.states[i].c_str(), f);
  }
  std::fputs("\n", f);
  size_t row = 0;
  for (int s = 0; s < n_series; s++) {
    for (int t = 0; t < lengths[s]; t++, row++) {
      const double* p = post + row * (size_t)stride + offset;
      for (int i = 0; i < v.card; i++) {
        if (i > 0) std::fputc(kSep, f);
        std::fprintf(f, "%f", p[i]);
      }
      std::fputs("\n", f);
    }
    std::fputs("\n", f);
  }
  if (std::fclose(f)) return nipamd::set_error(NIP_ERROR_IO, std::string("cannot close ") + path);
  return NIP_NO_ERROR;
}

int nipamd_model_var_symbol(const nipamd_model* mm, int var, char* buf, int cap) {
  if (!mm || var < 0 || var >= (int)mm->m.vars.size()) return -1;
  const std::string& n = mm->m.vars[var].symbol;
  if (buf && cap > 0) {
    std::strncpy(buf, n.c_str(), (size_t)cap - 1);
    buf[cap - 1] = '\0';
  }
  return (int)n.size();
}

int nipamd_model_state_name(const nipamd_model* mm, int var, int state, char* buf, int cap) {
  if (!mm || var < 0 || var >= (int)mm->m.vars.size()) return -1;
  const auto& v = mm->m.vars[var];
  if (state < 0 || state >= v.card) return -1;
  const std::string& n = v.states[state];
  if (buf && cap > 0) {
    std::strncpy(buf, n.c_str(), (size_t)cap - 1);
    buf[cap - 1] = '\0';
  }
  return (int)n.size();
}

int nipamd_model_var_label(const nipamd_model* mm, int var, char* buf, int cap) {
  if (!mm || var < 0 || var >= (int)mm->m.vars.size()) return -1;
  const std::string& n = mm->m.vars[var].label;
  if (buf && cap > 0) {
    std::strncpy(buf, n.c_str(), (size_t)cap - 1);
    buf[cap - 1] = '\0';
  }
  return (int)n.size();
}

int nipamd_model_var_info(const nipamd_model* mm, int var, int* info, int* parents, int cap) {
  if (!mm || var < 0 || var >= (int)mm->m.vars.size() || !info) return -1;
  const auto& v = mm->m.vars[var];
  info[0] = v.card;
  info[1] = v.next;
  info[2] = v.previous;
  info[3] = v.ifs;
  info[4] = v.pos_x;
  info[5] = v.pos_y;
  info[6] = (int)v.parents.size();
  info[7] = mm->m.node_size_x;
  info[8] = mm->m.node_size_y;
  for (int i = 0; parents && i < (int)v.parents.size() && i < cap; i++) parents[i] = v.parents[i];
  return (int)v.parents.size();
}

}  // extern "C"
