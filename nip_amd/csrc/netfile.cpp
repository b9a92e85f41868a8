// netfile.cpp -- Hugin .net reader for the nip_amd host side.
//
// Covers the subset of the Hugin net language that src/huginnet.y accepts
// (grammar at huginnet.y:202-834, lexer at :845-1047): an optional `net { }`
// block (contents ignored), `node`/`discrete node` declarations with `states`,
// `NIP_next`, `label`, `position` (other fields ignored), the net block's
// `node_size`, and `potential`
// declarations `(child)`, `(child | parents...)` with an optional `data` list.
// `%` starts a comment outside quotes.  Declaration order is preserved because
// it fixes the variable IDs (nipvariable.c:60,72).
#include "model.h"
#include "nip_amd.h"

#include <cctype>
#include <cstdlib>

namespace nipamd {
namespace {

struct Lexer {
  const std::string& s;
  size_t i = 0;
  explicit Lexer(const std::string& text) : s(text) {}

  void skip() {
    for (;;) {
      while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
      if (i < s.size() && s[i] == '%') { while (i < s.size() && s[i] != '\n') i++; continue; }
      return;
    }
  }
  // token kinds: 'q' quoted, 'w' word/number, or the punctuation char itself
  bool next(char& kind, std::string& tok) {
    skip();
    if (i >= s.size()) return false;
    char c = s[i];
    if (c == '"') {
      size_t j = s.find('"', i + 1);
      if (j == std::string::npos) j = s.size();
      tok = s.substr(i + 1, j - i - 1);
      kind = 'q';
      i = j + 1;
      return true;
    }
    if (std::string("(){}=;|").find(c) != std::string::npos) { tok = std::string(1, c); kind = c; i++; return true; }
    size_t j = i;
    while (j < s.size() && !std::isspace((unsigned char)s[j]) &&
           std::string("(){}=;|\"%").find(s[j]) == std::string::npos) j++;
    tok = s.substr(i, j - i);
    kind = 'w';
    i = j;
    return true;
  }
};

}  // namespace

int parse_net_file(const std::string& text, NetSpec& spec, std::string& err) {
  Lexer L(text);
  std::vector<std::pair<char, std::string>> toks;
  char k; std::string t;
  while (L.next(k, t)) toks.emplace_back(k, t);
  size_t i = 0;
  auto expect = [&](char c) -> bool {
    if (i < toks.size() && toks[i].first == c) { i++; return true; }
    err = std::string("net parser: expected '") + c + "'";
    return false;
  };
  auto skip_block = [&]() {
    int depth = 0;
    while (i < toks.size()) {
      if (toks[i].first == '{') depth++;
      else if (toks[i].first == '}') { if (--depth == 0) { i++; return; } }
      i++;
    }
  };
  std::vector<std::string> next_sym;
  struct RawPot { std::string child; std::vector<std::string> parents; std::vector<double> data; bool has; };
  std::vector<RawPot> raw;
  while (i < toks.size()) {
    const std::string& w = toks[i].second;
    if (toks[i].first == 'w' && (w == "net" || w == "class")) {
      i++;
      if (w == "class" && i < toks.size()) i++;  // class name
      if (w == "class") { if (!expect('{')) return NIP_ERROR_IO; continue; }
      // net { ... node_size = (x y); ... }  (huginnet.y:572-574)
      const size_t b0 = i;
      skip_block();
      for (size_t q = b0; q + 5 < i; q++)
        if (toks[q].first == 'w' && toks[q].second == "node_size" && toks[q + 1].first == '=' &&
            toks[q + 2].first == '(') {
          spec.node_size_x = std::abs((int)std::strtod(toks[q + 3].second.c_str(), nullptr));
          spec.node_size_y = std::abs((int)std::strtod(toks[q + 4].second.c_str(), nullptr));
        }
    } else if (toks[i].first == 'w' && (w == "node" || w == "discrete")) {
      if (w == "discrete") i++;
      i++;
      if (i >= toks.size()) { err = "net parser: truncated node"; return NIP_ERROR_IO; }
      std::string sym = toks[i++].second;
      if (!expect('{')) return NIP_ERROR_IO;
      std::vector<std::string> states;
      std::string nx, label = " ";
      int px = 100, py = 100;
      while (i < toks.size() && toks[i].first != '}') {
        std::string key = toks[i++].second;
        if (!expect('=')) return NIP_ERROR_IO;
        std::vector<std::string> vals;
        if (i < toks.size() && toks[i].first == '(') {
          i++;
          while (i < toks.size() && toks[i].first != ')') vals.push_back(toks[i++].second);
          if (!expect(')')) return NIP_ERROR_IO;
        } else if (i < toks.size()) {
          vals.push_back(toks[i++].second);
        }
        if (!expect(';')) return NIP_ERROR_IO;
        if (key == "states") states = vals;
        else if (key == "NIP_next" && !vals.empty()) nx = vals[0];
        else if (key == "label" && !vals.empty()) label = vals[0];
        else if (key == "position" && vals.size() == 2) {
          px = std::abs((int)std::strtod(vals[0].c_str(), nullptr));
          py = std::abs((int)std::strtod(vals[1].c_str(), nullptr));
        }
      }
      if (!expect('}')) return NIP_ERROR_IO;
      if (states.empty()) { err = "net parser: the states field is missing (node " + sym + ")"; return NIP_ERROR_IO; }
      spec.symbols.push_back(sym);
      spec.card.push_back((int)states.size());
      spec.states.push_back(states);
      spec.labels.push_back(label);
      spec.positions.emplace_back(px, py);
      next_sym.push_back(nx);
    } else if (toks[i].first == 'w' && w == "potential") {
      i++;
      if (!expect('(')) return NIP_ERROR_IO;
      RawPot p; p.has = false;
      if (i >= toks.size()) return NIP_ERROR_IO;
      p.child = toks[i++].second;
      if (i < toks.size() && toks[i].first == '|') {
        i++;
        while (i < toks.size() && toks[i].first != ')') p.parents.push_back(toks[i++].second);
      }
      if (!expect(')')) return NIP_ERROR_IO;
      if (!expect('{')) return NIP_ERROR_IO;
      while (i < toks.size() && toks[i].first != '}') {
        std::string key = toks[i++].second;
        if (!expect('=')) return NIP_ERROR_IO;
        if (key == "data") {
          p.has = true;
          while (i < toks.size() && toks[i].first != ';') {
            if (toks[i].first == 'w') p.data.push_back(std::strtod(toks[i].second.c_str(), nullptr));
            i++;
          }
        } else {
          while (i < toks.size() && toks[i].first != ';') i++;
        }
        if (!expect(';')) return NIP_ERROR_IO;
      }
      if (!expect('}')) return NIP_ERROR_IO;
      raw.push_back(std::move(p));
    } else {
      i++;
    }
  }
  auto index = [&](const std::string& s) -> int {
    for (size_t j = 0; j < spec.symbols.size(); j++) if (spec.symbols[j] == s) return (int)j;
    return -1;
  };
  spec.next.assign(spec.symbols.size(), -1);
  for (size_t j = 0; j < next_sym.size(); j++)
    if (!next_sym[j].empty()) {
      spec.next[j] = index(next_sym[j]);
      if (spec.next[j] < 0) { err = "net parser: unknown NIP_next " + next_sym[j]; return NIP_ERROR_GENERAL; }
    }
  for (auto& r : raw) {
    NetSpec::Pot p;
    p.child = index(r.child);
    if (p.child < 0) { err = "net parser: unknown child " + r.child; return NIP_ERROR_GENERAL; }
    for (auto& ps : r.parents) {
      int q = index(ps);
      if (q < 0) { err = "net parser: unknown parent " + ps; return NIP_ERROR_GENERAL; }
      p.parents.push_back(q);
    }
    p.data = std::move(r.data);
    p.has_data = r.has;
    spec.pots.push_back(std::move(p));
  }
  return 0;
}

}  // namespace nipamd
