// engine.cpp -- C-ABI of the nip_amd engine (include/nip_amd.h).
//
// Host side of the hot path: owns the compiled model, its device-resident
// tables and scratch, validates the request against the GPU execution plan
// and launches the gfx950 kernels on the caller's stream.  There is no CPU
// fallback: a request the GPU plan does not cover fails with
// NIPAMD_ERROR_UNSUPPORTED, and a missing/unusable device with
// NIPAMD_ERROR_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "chain_kernels.h"
#include "diag.h"
#include "model.h"
#include "nip_amd.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// A launcher's nonzero return (chain_kernels.h): kLaunchRefused -- the host
// refused the request before queueing anything (a shape or LDS budget the
// kernel does not take) -- is NIPAMD_ERROR_UNSUPPORTED; anything else is a
// failed HIP call, NIPAMD_ERROR_DEVICE with HIP's last error.
int launch_fail(int rc, const char* what) {
  if (rc == nipamd::kLaunchRefused)
    return fail(NIPAMD_ERROR_UNSUPPORTED, std::string(what) + ": the request does not fit the kernel (refused on the host)");
  return fail(NIPAMD_ERROR_DEVICE, std::string(what) + ": kernel launch failed: " + hipGetErrorString(hipGetLastError()));
}

#define HIP_OK(expr)                                                         \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return fail(NIPAMD_ERROR_DEVICE, std::string(#expr) + ": " +          \
                                           hipGetErrorString(e_));           \
  } while (0)

// Device tables that depend on which children a request observes.
struct ReqTables {
  std::string key;                // emit index per observed column
  int M0 = 0;                     // narrow kernels: rows of Etab16 are M0 + 2
  double* Etab16 = nullptr;       // [(M0+2)][16]
  double* ts16 = nullptr;         // [16] w = A s_all (matrix-core kernel's ll)
  double* tabw = nullptr;         // wide kernel: per column [(M_k+2)][64], concatenated
  std::vector<size_t> tabw_off;
  double* ebase = nullptr;        // [64] product of the unobserved children's row sums
  // matrix-core wide kernel: per column [(M_k+2)][NP], column 0 times ebase
  // (a single [2][NP] pseudo column = ebase when nothing is observed)
  double* mtab = nullptr;
  int mtab_rows = 0;
  int mtab_off[4] = {0, 0, 0, 0};
  double* wv = nullptr;           // [64] A s_all
  double* arena = nullptr;        // the pool buffer all of the above live in (one upload)
};

struct DevState {
  int device = -1;
  unsigned version = 0;
  double* A = nullptr;            // [16][16]  (N <= 16)
  double* pi = nullptr;           // [16]
  double* A64 = nullptr;          // [64][64]
  double* pi64 = nullptr;         // [64]
  double* sall64 = nullptr;       // [64]
  double* arena = nullptr;        // the pool buffer A .. sall64 and childE live in (one upload)
  std::deque<ReqTables> reqs;      // deque: pointers returned by ensure_req_tables stay valid
  double* S = nullptr;
  size_t S_bytes = 0;
  double* R = nullptr;     // E-step partial [nipamd_estep_partial_size] of nipamd_estep
  int R_size = 0;
  double* W = nullptr;     // E-step work: slabs + tree levels + chunk results + partial
  size_t W_bytes = 0;
  double* Q = nullptr;     // derived marginals: interface marginals / forward messages
  size_t Q_bytes = 0;
  std::vector<double*> childE;   // per leaf child [(M+1)][64]: E, then the row sums
  std::vector<double*> G;        // per hidden parent [card][64][64], built on first use
  // joint-interface e_step finalize: the slab -> em_learn layout map (CSR)
  int* jm_ptr = nullptr;
  int* jm_idx = nullptr;
  double* jm_coef = nullptr;
  int jm_n = 0;
  int jm_kind = 0;                // 1 joint map, 2 16-state chain slab, 3 wide chain slab
  // general chain e_step (several leaf children, hidden parents): every
  // child's table, rows M_k + 2 each (E, the row sums, zeros), 16 columns
  double* etab_all = nullptr;
  // model-table buffers of earlier versions, kept for the next version's
  // tables of the same sizes (an em_learn iteration re-uploads every table
  // after its m_step: no hipMalloc / hipFree pair per table and iteration)
  std::unordered_map<void*, size_t> live;        // pool-managed buffers in use -> bytes
  std::vector<std::pair<void*, size_t>> pool;     // free ones
};

void* dalloc(DevState* d, size_t bytes) {
  for (size_t i = 0; i < d->pool.size(); i++)
    if (d->pool[i].second == bytes) {
      void* p = d->pool[i].first;
      d->pool[i] = d->pool.back();
      d->pool.pop_back();
      d->live[p] = bytes;
      return p;
    }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  d->live[p] = bytes;
  return p;
}

// back to the pool (the caller has synchronised the device), or hipFree for
// buffers the pool did not hand out
void dfree(DevState* d, void* p) {
  if (!p) return;
  auto it = d->live.find(p);
  if (it == d->live.end()) { (void)hipFree(p); return; }
  d->pool.push_back(*it);
  d->live.erase(it);
}

DevState* dev_of(nipamd_model* mm) {
  if (!mm->m.dev) mm->m.dev = new DevState();
  return static_cast<DevState*>(mm->m.dev);
}

void free_tables(DevState* d) {
  // queued kernels may still read the tables: they return to the pool only
  // once the device is idle (hipFree synchronised the same way)
  if (!d->live.empty()) (void)hipDeviceSynchronize();
  dfree(d, d->arena);
  d->A = d->pi = d->A64 = d->pi64 = d->sall64 = d->arena = nullptr;
  for (auto& r : d->reqs) dfree(d, r.arena);
  d->reqs.clear();
  for (double* p : d->G) dfree(d, p);
  d->childE.clear();
  d->G.clear();
  dfree(d, d->jm_ptr); dfree(d, d->jm_idx); dfree(d, d->jm_coef);
  d->jm_ptr = nullptr; d->jm_idx = nullptr; d->jm_coef = nullptr; d->jm_n = 0; d->jm_kind = 0;
  dfree(d, d->etab_all);
  d->etab_all = nullptr;
}

void dev_release(DevState* d) {
  if (!d) return;
  free_tables(d);
  for (auto& e : d->pool) (void)hipFree(e.first);
  d->pool.clear();
  (void)hipFree(d->S); (void)hipFree(d->W); (void)hipFree(d->R); (void)hipFree(d->Q);
  *d = DevState();
}

// Several tables in one pool buffer with one host-to-device copy: every
// em_learn iteration re-uploads the model's tables after its m_step, and a
// synchronous copy per table kept the device idle for ~0.2 ms per iteration
// (profiles/r05/em_phases.py).  Each table starts on a 64-byte boundary.
struct Staged {
  std::vector<double> host;
  std::vector<std::pair<double**, size_t>> dst;
  template <typename V>
  void add(double** p, const V& v) {
    dst.push_back({p, host.size()});
    host.insert(host.end(), v.begin(), v.end());
    host.resize((host.size() + 8) & ~(size_t)7, 0.0);     // >= 1 double, 64-byte aligned
  }
  int commit(DevState* d, double** arena);
};

template <typename V>
int upload(DevState* d, double** dst, const V& v) {
  *dst = static_cast<double*>(dalloc(d, (v.size() ? v.size() : 1) * sizeof(double)));
  if (!*dst) return fail(NIPAMD_ERROR_DEVICE, "device allocation failed");
  if (v.size()) HIP_OK(hipMemcpy(*dst, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice));
  return 0;
}

int Staged::commit(DevState* d, double** arena) {
  *arena = static_cast<double*>(dalloc(d, host.size() * sizeof(double)));
  if (!*arena) return fail(NIPAMD_ERROR_DEVICE, "device allocation failed");
  HIP_OK(hipMemcpy(*arena, host.data(), host.size() * sizeof(double), hipMemcpyHostToDevice));
  for (auto& e : dst) *e.first = *arena + e.second;
  return 0;
}

// Bind the model's device state to the current device (a different device
// drops every buffer of the old one).  Call before taking any DevState
// pointer that a later ensure_* must not free.
int ensure_device(nipamd_model* mm) {
  int dev = -1;
  HIP_OK(hipGetDevice(&dev));
  DevState* d = dev_of(mm);
  if (d->device != dev) { dev_release(d); d->device = dev; }
  return 0;
}

}  // namespace

// A deferred fold (large in-clique, ChainPlan::fold_gpu): A64 on the GPU, then
// on the host for every host-side use (derived tables, likelihood, P.A).
int nipamd::ensure_fold(nipamd_model* mm) {
  auto& P = mm->m.chain;
  if (!P.valid || !P.fold_gpu || P.folded) return 0;
  if (int rc = ensure_device(mm)) return rc;
  std::vector<double> A;
  std::string err;
  if (nipamd::chain_fold_gpu(mm->m, -1, A, &mm->fold_ms, &mm->fold_bytes, err))
    return fail(NIPAMD_ERROR_DEVICE, "transition fold: " + err);
  P.A64 = std::move(A);
  if (P.N <= 16)
    for (int x = 0; x < P.N; x++)
      for (int y = 0; y < P.N; y++) P.A[x * 16 + y] = P.A64[x * 64 + y];
  P.folded = true;
  return 0;
}

namespace {

// Upload the chain plan's tables to the current device (once per version).
int ensure_tables(nipamd_model* mm) {
  if (int rc = ensure_device(mm)) return rc;
  DevState* d = dev_of(mm);
  if (d->version == mm->version && d->A64) return 0;
  if (int rc = nipamd::ensure_fold(mm)) return rc;
  const auto& P = mm->m.chain;
  free_tables(d);
  Staged sg;
  if (P.N <= 16) {
    sg.add(&d->A, P.A);
    sg.add(&d->pi, P.pi);
  }
  sg.add(&d->A64, P.A64);
  sg.add(&d->pi64, P.pi64);
  sg.add(&d->sall64, P.s_all64);
  d->childE.assign(P.emits.size(), nullptr);
  for (size_t k = 0; k < P.emits.size(); k++) {
    std::vector<double> t(P.emits[k].E);
    t.insert(t.end(), P.emits[k].s.begin(), P.emits[k].s.end());
    sg.add(&d->childE[k], t);
  }
  if (int rc = sg.commit(d, &d->arena)) return rc;
  d->G.assign(P.hidden.size(), nullptr);
  d->version = mm->version;
  return 0;
}

// G table of hidden parent j on the device (derived marginals)
int ensure_hidden(nipamd_model* mm, int j) {
  DevState* d = dev_of(mm);
  if (d->G[j]) return 0;
  std::vector<double> g;
  if (mm->m.chain.fold_gpu) {
    std::string err;
    double ms = 0, bytes = 0;
    if (nipamd::chain_fold_gpu(mm->m, j, g, &ms, &bytes, err)) return fail(NIPAMD_ERROR_DEVICE, "hidden fold: " + err);
  } else {
    nipamd::hidden_table(mm->m, j, g);
  }
  return upload(d, &d->G[j], g);
}

// A request's routing through the chain plan: which emission child each
// observation column is, and which kernel family serves it.
struct Route {
  int ncol = 0;                   // observed emission children
  int col[4] = {-1, -1, -1, -1};  // their columns in obs
  int emit[4] = {-1, -1, -1, -1}; // their plan.emits index
  int primary = -1;               // narrow kernels: the child whose table is used
  int pcol = -1;                  // its column (or -1: never observed)
  bool narrow = false;            // N <= 16 and at most one observed child
};

// Tables of a route (built and uploaded once per model version).
int ensure_req_tables(nipamd_model* mm, const Route& r, ReqTables** out) {
  DevState* d = dev_of(mm);
  const auto& P = mm->m.chain;
  std::string key;
  for (int i = 0; i < r.ncol; i++) key += std::to_string(r.emit[i]) + ",";
  key += "|" + std::to_string(r.primary);
  for (auto& t : d->reqs) if (t.key == key) { *out = &t; return 0; }
  ReqTables t;
  t.key = key;
  Staged sg;                                 // every table of the request, one upload
  const int N = P.N;
  if (N <= 16) {
    // narrow: the primary child's table times the other children's row sums
    std::vector<double> b(16, 0.0);
    for (int y = 0; y < N; y++) {
      double v = 1.0;
      for (size_t k = 0; k < P.emits.size(); k++) if ((int)k != r.primary) v *= P.emits[k].s[y];
      b[y] = v;
    }
    const int M = r.primary >= 0 ? P.emit(r.primary).M : 0;
    std::vector<double> E((size_t)(M + 2) * 16, 0.0);
    for (int y = 0; y < N; y++) {
      for (int m = 0; m < M; m++) E[(size_t)m * 16 + y] = P.emit(r.primary).E[(size_t)m * 64 + y] * b[y];
      E[(size_t)M * 16 + y] = (r.primary >= 0 ? P.emit(r.primary).s[y] : 1.0) * b[y];
    }
    std::vector<double> ts(16, 0.0);
    for (int x = 0; x < N; x++) {
      double acc = 0.0;
      for (int y = 0; y < N; y++) acc += P.A[x * 16 + y] * E[(size_t)M * 16 + y];
      ts[x] = acc;
    }
    t.M0 = M;
    sg.add(&t.Etab16, E);
    sg.add(&t.ts16, ts);
  }
  // wide: one unscaled table per observed child, the unobserved ones in ebase
  std::vector<double> W;
  for (int i = 0; i < r.ncol; i++) {
    const auto& em = P.emit(r.emit[i]);
    t.tabw_off.push_back(W.size());
    const size_t base = W.size();
    W.resize(base + (size_t)(em.M + 2) * 64, 0.0);
    for (int y = 0; y < N; y++) {
      for (int m = 0; m < em.M; m++) W[base + (size_t)m * 64 + y] = em.E[(size_t)m * 64 + y];
      W[base + (size_t)em.M * 64 + y] = em.s[y];
    }
  }
  std::vector<double> eb(64, 0.0);
  for (int y = 0; y < N; y++) {
    double v = 1.0;
    for (size_t k = 0; k < P.emits.size(); k++) {
      bool obs = false;
      for (int i = 0; i < r.ncol; i++) obs |= r.emit[i] == (int)k;
      if (!obs) v *= P.emits[k].s[y];
    }
    eb[y] = v;
  }
  sg.add(&t.tabw, W);
  sg.add(&t.ebase, eb);
  if (N <= 32) {
    const int NP = N <= 16 ? 16 : 32;
    std::vector<double> MT;
    const int nc = r.ncol > 0 ? r.ncol : 1;
    for (int i = 0; i < nc; i++) {
      const int M = r.ncol > 0 ? P.emit(r.emit[i]).M : 0;
      t.mtab_off[i] = (int)MT.size();
      const size_t base = MT.size();
      MT.resize(base + (size_t)(M + 2) * NP, 0.0);
      for (int y = 0; y < N; y++) {
        const double f = i == 0 ? eb[y] : 1.0;
        if (r.ncol > 0) {
          const auto& em = P.emit(r.emit[i]);
          for (int m = 0; m < M; m++) MT[base + (size_t)m * NP + y] = em.E[(size_t)m * 64 + y] * f;
          MT[base + (size_t)M * NP + y] = em.s[y] * f;
        } else {
          MT[base + y] = f;
        }
      }
    }
    t.mtab_rows = (int)(MT.size() / NP);
    std::vector<double> wv(64, 0.0);
    for (int x = 0; x < N; x++) {
      double acc = 0.0;
      for (int y = 0; y < N; y++) acc += P.A64[(size_t)x * 64 + y] * P.s_all64[y];
      wv[x] = acc;
    }
    sg.add(&t.mtab, MT);
    sg.add(&t.wv, wv);
  }
  if (int rc = sg.commit(d, &t.arena)) return rc;
  d->reqs.push_back(std::move(t));
  *out = &d->reqs.back();
  return 0;
}

int ensure_scratch(nipamd_model* mm, size_t bytes) {
  DevState* d = dev_of(mm);
  if (d->S_bytes >= bytes) return 0;
  (void)hipFree(d->S);
  d->S = nullptr;
  d->S_bytes = 0;
  HIP_OK(hipMalloc(&d->S, bytes));
  d->S_bytes = bytes;
  return 0;
}

int ensure_q(nipamd_model* mm, size_t bytes) {
  DevState* d = dev_of(mm);
  if (d->Q_bytes >= bytes) return 0;
  (void)hipFree(d->Q);
  d->Q = nullptr;
  d->Q_bytes = 0;
  HIP_OK(hipMalloc(&d->Q, bytes));
  d->Q_bytes = bytes;
  return 0;
}

int ensure_work(nipamd_model* mm, size_t bytes) {
  DevState* d = dev_of(mm);
  if (d->W_bytes >= bytes) return 0;
  (void)hipFree(d->W);
  d->W = nullptr;
  d->W_bytes = 0;
  HIP_OK(hipMalloc(&d->W, bytes));
  d->W_bytes = bytes;
  return 0;
}

// Sequences per E-step launch: bounds the slab + scratch memory.  A power of
// two times 64^k, so chunk trees are subtrees of the one binary tree over the
// batch (see tree64_kernel).
#ifndef NIPAMD_ESTEP_SEQS
#define NIPAMD_ESTEP_SEQS 16384
#endif
constexpr long kEstepChunk = NIPAMD_ESTEP_SEQS;
// chain_estep_ck_kernel's launches: its scratch holds one checkpoint per four
// steps (~4.4 GB at 131072 x 1024), so a whole config-4 shard is one launch
constexpr long kEstepCkChunk = 131072;

// rows [n][S] -> out [S] by repeated radix-64 tree levels (ping-pong tA/tB)
int reduce_rows(const double* in, long n, int S, double* tA, double* tB, double* out, hipStream_t st) {
  const double* cur = in;
  while (n > 64) {
    double* dst = (cur == tA) ? tB : tA;
    if (nipamd::tree_reduce_launch(cur, n, S, dst, st)) return -1;
    cur = dst;
    n = (n + 63) / 64;
  }
  return nipamd::tree_reduce_launch(cur, n, S, out, st);
}

// fb kernel choice: the matrix-core kernels (chain_fb_ckpt_kernel for 16-wide
// posterior rows, NIPAMD_FB_KERNEL=scratch for chain_fb_mfma_kernel) unless NIPAMD_FB_KERNEL=dpp
// (the 16-lane DPP kernel, kept for the e_step and for A/B measurements)
bool use_mfma() {
  static const bool v = [] {
    const char* e = nipamd::diag_env("NIPAMD_FB_KERNEL");
    return !(e && std::string(e) == "dpp");
  }();
  return v;
}

// Role of a query variable in the chain plan: 0 the interface variable, 1 its
// previous-slice copy, 2 + k leaf child k, 500 + i / 700 + i previous-slice /
// current interface variable i of a joint interface, 1000 + j hidden parent j;
// -1 none.
// Every variable of a single-variable plan has one (build_chain_plan accounts
// for all); a joint plan covers the interface variables, their previous-slice
// copies and the leaf children it factorises.
int query_kind(const nipamd::ChainPlan& P, int v) {
  if (v == P.v_cur) return 0;
  if (v == P.v_prev) return 1;
  for (size_t i = 0; i < P.jprev.size(); i++) if (P.jprev[i] == v) return 500 + (int)i;
  for (size_t i = 0; i < P.jcur.size(); i++) if (P.jcur[i] == v) return 700 + (int)i;
  for (size_t k = 0; k < P.emits.size(); k++) if (P.emits[k].var == v) return 2 + (int)k;
  for (size_t j = 0; j < P.hidden.size(); j++) if (P.hidden[j] == v) return 1000 + (int)j;
  return -1;
}

// Which GPU plan (if any) covers this request.
int route_request(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query,
                  const int* query, Route& r, std::string& why) {
  const auto& P = mm->m.chain;
  if (!P.valid) {
    why = "model slice is not an interface chain (GPU plan: one interface variable, hidden "
          "independent parents, leaf children; see DESIGN.md)";
    return 0;
  }
  r = Route();
  for (int i = 0; i < n_obs; i++) {
    int k = -1;
    for (size_t e = 0; e < P.emits.size(); e++) if (P.emits[e].var == obs_vars[i]) k = (int)e;
    if (obs_vars[i] == P.v_cur) k = (int)P.emits.size();          // the interface variable itself
    if (k < 0) {
      why = "evidence on a variable that is neither the interface variable nor a leaf child of it";
      return 0;
    }
    for (int j = 0; j < r.ncol; j++) if (r.emit[j] == k) { why = "observed variable listed twice"; return 0; }
    if (r.ncol == 4) { why = "more than four observed children"; return 0; }
    r.col[r.ncol] = i; r.emit[r.ncol] = k; r.ncol++;
  }
  for (int i = 0; i < n_query; i++)
    if (query_kind(P, query[i]) < 0) { why = "query variable outside the chain plan"; return 0; }
  r.narrow = P.N <= 16 && r.ncol <= 1;
  if (r.ncol == 1) { r.primary = r.emit[0]; r.pcol = r.col[0]; }
  else if (!P.emits.empty()) { r.primary = 0; r.pcol = -1; }
  return 1;
}

// device buffers of a host-buffer call, freed on every return path
struct DevBufs {
  std::vector<void*> p;
  template <typename T> int alloc(T** out, size_t n) {
    *out = nullptr;
    HIP_OK(hipMalloc(out, (n ? n : 1) * sizeof(T)));
    p.push_back(*out);
    return 0;
  }
  ~DevBufs() { for (void* q : p) (void)hipFree(q); }
};

}  // namespace

namespace nipamd {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
const char* g_last_kernel = "";
}  // namespace nipamd

extern "C" {

const char* nipamd_last_error(void) { return g_err.c_str(); }

const char* nipamd_last_kernel(void) { return nipamd::g_last_kernel; }

int nipamd_model_from_spec(int n_nodes, const char* const* symbols, const int* card,
                           const int* next, int n_pots, const int* pot_child,
                           const int* pot_nparents, const int* pot_parents,
                           const int* pot_ndata, const double* pot_data,
                           nipamd_model** out) {
  if (!out || !card || n_nodes <= 0) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  nipamd::NetSpec spec;
  for (int i = 0; i < n_nodes; i++) {
    spec.symbols.push_back(symbols && symbols[i] ? symbols[i] : ("V" + std::to_string(i)));
    spec.card.push_back(card[i]);
    spec.next.push_back(next ? next[i] : -1);
  }
  size_t po = 0, dof = 0;
  for (int p = 0; p < n_pots; p++) {
    nipamd::NetSpec::Pot q;
    q.child = pot_child[p];
    for (int k = 0; k < pot_nparents[p]; k++) q.parents.push_back(pot_parents[po++]);
    q.has_data = pot_ndata[p] > 0;
    q.data.assign(pot_data + dof, pot_data + dof + pot_ndata[p]);
    dof += pot_ndata[p];
    if (q.child < 0 || q.child >= n_nodes) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad child index");
    for (int v : q.parents) if (v < 0 || v >= n_nodes) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad parent index");
    spec.pots.push_back(std::move(q));
  }
  auto* mm = new nipamd_model();
  std::string err;
  int rc = nipamd::compile_model(spec, mm->m, err);
  if (rc) { delete mm; return fail(rc, err); }
  *out = mm;
  return 0;
}

int nipamd_model_from_net(const char* path, nipamd_model** out) {
  if (!path || !out) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  std::ifstream f(path);
  if (!f) return fail(NIP_ERROR_FILENOTFOUND, std::string("cannot open ") + path);
  std::stringstream ss;
  ss << f.rdbuf();
  nipamd::NetSpec spec;
  std::string err;
  int rc = nipamd::parse_net_file(ss.str(), spec, err);
  if (rc) return fail(rc, err);
  auto* mm = new nipamd_model();
  rc = nipamd::compile_model(spec, mm->m, err);
  if (rc) { delete mm; return fail(rc, err); }
  *out = mm;
  return 0;
}

void nipamd_model_free(nipamd_model* mm) {
  if (!mm) return;
  nipamd::generate_release(mm);
  nipamd::jt_release(mm);
  nipamd::op_release(mm);
  nipamd::likelihood_release(mm);
  DevState* d = static_cast<DevState*>(mm->m.dev);
  dev_release(d);
  delete d;
  delete mm;
}

int nipamd_model_num_vars(const nipamd_model* mm) { return mm ? (int)mm->m.vars.size() : -1; }

int nipamd_model_var_index(const nipamd_model* mm, const char* symbol) {
  if (!mm || !symbol) return -1;
  for (size_t i = 0; i < mm->m.vars.size(); i++)
    if (mm->m.vars[i].symbol == symbol) return (int)i;
  return -1;
}

int nipamd_model_var_card(const nipamd_model* mm, int v) {
  if (!mm || v < 0 || v >= (int)mm->m.vars.size()) return -1;
  return mm->m.vars[v].card;
}

int nipamd_model_desc_json(const nipamd_model* mm, char* buf, int cap) {
  if (!mm) return -1;
  std::string s = nipamd::model_desc_json(mm->m);
  if (buf && cap > 0) {
    size_t n = s.size() < (size_t)(cap - 1) ? s.size() : (size_t)(cap - 1);
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int)s.size();
}

int nipamd_model_param_size(const nipamd_model* mm) { return mm ? nipamd::param_size(mm->m) : -1; }

int nipamd_model_gpu_supported(const nipamd_model* mm, int n_obs, const int* obs_vars,
                               int n_query, const int* query) {
  if (!mm) return 0;
  Route r; std::string why;
  if (mm->engine != NIPAMD_ENGINE_JTREE && route_request(mm, n_obs, obs_vars, n_query, query, r, why)) return 1;
  if (mm->engine == NIPAMD_ENGINE_AUTO &&
      nipamd::op_supported(const_cast<nipamd_model*>(mm), n_obs, obs_vars, n_query, query, why))
    return 1;
  return mm->engine != NIPAMD_ENGINE_CHAIN && nipamd::jt_supported(mm, n_obs, obs_vars, n_query, query, why);
}

int nipamd_jt_plan_dump(const nipamd_model* mm, int n_obs, const int* obs_vars, int n_query,
                        const int* query, int estep, int* hdr, int hdr_cap, int* ip, long ip_cap,
                        double* dp, long dp_cap, long* sizes) {
  if (!mm || !hdr || !sizes || (n_obs > 0 && !obs_vars) || (n_query > 0 && !query))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  return nipamd::jt_plan_dump(mm, n_obs, obs_vars, n_query, query, estep, hdr, hdr_cap, ip, ip_cap, dp,
                              dp_cap, sizes);
}

int nipamd_model_fold(nipamd_model* mm, int keep, double* out, long cap, double* kernel_ms, double* bytes) {
  if (!mm || !out) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const auto& P = mm->m.chain;
  if (!P.valid || P.joint) return fail(NIPAMD_ERROR_UNSUPPORTED, "the model has no single-variable interface-chain plan");
  if (keep < -1 || keep >= (int)P.hidden.size()) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad hidden parent");
  const long need = (keep < 0 ? 1L : (long)mm->m.vars[P.hidden[keep]].card) * 64 * 64;
  if (cap < need) return fail(NIP_ERROR_INVALID_ARGUMENT, "output buffer too small");
  if (int rc = ensure_device(mm)) return rc;
  std::vector<double> v;
  std::string err;
  double ms = 0, by = 0;
  if (nipamd::chain_fold_gpu(mm->m, keep, v, &ms, &by, err)) return fail(NIPAMD_ERROR_DEVICE, "fold: " + err);
  std::copy(v.begin(), v.end(), out);
  if (kernel_ms) *kernel_ms = ms;
  if (bytes) *bytes = by;
  return 0;
}

int nipamd_model_set_engine(nipamd_model* mm, int engine) {
  if (!mm || engine < NIPAMD_ENGINE_AUTO || engine > NIPAMD_ENGINE_JTREE) return -1;
  const int prev = mm->engine;
  mm->engine = engine;
  return prev;
}

int nipamd_model_original(const nipamd_model* mm, int c, double* out, int cap) {
  if (!mm || c < 0 || c >= (int)mm->m.cliques.size()) return -1;
  const auto& o = mm->m.cliques[c].original;
  size_t n = o.size() < (size_t)cap ? o.size() : (size_t)cap;
  if (out) std::memcpy(out, o.data(), n * sizeof(double));
  return (int)o.size();
}

int nipamd_model_prior(const nipamd_model* mm, int v, double* out) {
  if (!mm || v < 0 || v >= (int)mm->m.vars.size()) return -1;
  const auto& var = mm->m.vars[v];
  if (!var.has_prior || !var.parents.empty()) return 0;
  if (out) std::memcpy(out, var.prior.data(), var.prior.size() * sizeof(double));
  return (int)var.prior.size();
}

int nipamd_model_num_cliques(const nipamd_model* mm) { return mm ? (int)mm->m.cliques.size() : -1; }
int nipamd_model_num_sepsets(const nipamd_model* mm) { return mm ? (int)mm->m.sepsets.size() : -1; }

int nipamd_model_clique(const nipamd_model* mm, int c, int* vars, int* n_vars, int* links, int* n_links) {
  if (!mm || c < 0 || c >= (int)mm->m.cliques.size()) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad clique");
  const auto& q = mm->m.cliques[c];
  if (n_vars) *n_vars = (int)q.vars.size();
  if (n_links) *n_links = (int)q.links.size();
  if (vars) std::copy(q.vars.begin(), q.vars.end(), vars);
  if (links) std::copy(q.links.begin(), q.links.end(), links);
  return NIP_NO_ERROR;
}

int nipamd_model_sepset(const nipamd_model* mm, int s, int* a, int* b, int* vars, int* n_vars) {
  if (!mm || s < 0 || s >= (int)mm->m.sepsets.size()) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad sepset");
  const auto& q = mm->m.sepsets[s];
  if (a) *a = q.a;
  if (b) *b = q.b;
  if (n_vars) *n_vars = (int)q.vars.size();
  if (vars) std::copy(q.vars.begin(), q.vars.end(), vars);
  return NIP_NO_ERROR;
}

int nipamd_model_interface_cliques(const nipamd_model* mm, int* in_clique, int* out_clique) {
  if (!mm) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad model");
  if (in_clique) *in_clique = mm->m.in_clique;
  if (out_clique) *out_clique = mm->m.out_clique;
  return NIP_NO_ERROR;
}

int nipamd_model_set_tables(nipamd_model* mm, int n_cliques, const double* const* originals,
                            int n_vars, const double* const* priors) {
  if (!mm || n_cliques != (int)mm->m.cliques.size() || n_vars != (int)mm->m.vars.size() ||
      (n_cliques > 0 && !originals) || (n_vars > 0 && !priors))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "nipamd_model_set_tables: bad arguments");
  for (int c = 0; c < n_cliques; c++) {
    auto& o = mm->m.cliques[c].original;
    if (originals[c]) std::memcpy(o.data(), originals[c], o.size() * sizeof(double));
  }
  for (int v = 0; v < n_vars; v++) {
    auto& var = mm->m.vars[v];
    if (!priors[v] || !var.parents.empty()) continue;
    var.prior.assign(priors[v], priors[v] + var.card);
    var.has_prior = true;
  }
  nipamd::build_chain_plan(mm->m);
  mm->version++;
  return NIP_NO_ERROR;
}

int nipamd_graph_cliques(int n, const int* card, int n_edges, const int* edges,
                         int set_parents, int* clique_off, int* clique_vars, int cap) {
  if (n <= 0 || !card || (n_edges > 0 && !edges) || !clique_off) return -NIP_ERROR_INVALID_ARGUMENT;
  std::vector<int> cd(card, card + n);
  std::vector<std::pair<int, int>> e;
  for (int i = 0; i < n_edges; i++) e.emplace_back(edges[2 * i], edges[2 * i + 1]);
  std::vector<std::vector<int>> cl;
  std::string err;
  int nc = nipamd::compile_graph_only(n, cd, e, set_parents != 0, cl, err);
  if (nc < 0) { g_err = err; return -NIP_ERROR_GENERAL; }
  int pos = 0;
  clique_off[0] = 0;
  for (int c = 0; c < nc; c++) {
    for (int v : cl[c]) { if (clique_vars && pos < cap) clique_vars[pos] = v; pos++; }
    clique_off[c + 1] = pos;
  }
  return nc;
}

int nipamd_m_step(nipamd_model* mm, const double* params) {
  if (!mm || !params) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  int rc = nipamd::m_step(mm->m, params);
  mm->version++;
  return rc;
}

// Interface-chain kernel for a route, in order of preference; each kernel
// stages the block's observation codes in LDS, so a long sequence may not fit
// one and falls through to the next (the 64-state kernel last).  kNoChain:
// no chain kernel fits -- the request goes to the general engine.
enum ChainKernel { kNoChain = 0, kMfmaWide, kNarrowMfma, kNarrowDpp, kWide64 };

static int pick_kernel(const nipamd_model* mm, const Route& r, const ReqTables* rt, int T, bool filt) {
  const auto& P = mm->m.chain;
  static const bool force_wide = [] {
    const char* e = nipamd::diag_env("NIPAMD_FB_KERNEL");
    return e && std::string(e) == "wide";
  }();
  if ((!r.narrow || filt) && P.N <= 32 && !force_wide &&
      nipamd::chain_mfma_wide_lds_bytes(P.N <= 16 ? 1 : 2, rt->mtab_rows, r.ncol, T) <= 160 * 1024)
    return kMfmaWide;
  if (r.narrow && !filt) {
    if (use_mfma() && nipamd::chain_mfma_lds_bytes(rt->M0, T) <= 160 * 1024) return kNarrowMfma;
    if (nipamd::chain_lds_bytes(rt->M0, T, false) <= 96 * 1024) return kNarrowDpp;
  }
  if (nipamd::chain_wide_lds_bytes(r.ncol, T) <= 64 * 1024) return kWide64;
  return kNoChain;
}

#ifdef NIPAMD_DIAGNOSTICS
// Timing-only builds: per-block phase timestamps of the matrix-core fb kernel
// (NIPAMD_PHASE_TIMES=1), printed as a summary after the launch.
static void phase_report(const unsigned long long* h, int nblk) {
  double sa = 0, sb = 0, sc = 0;
  for (int k = 0; k < nblk; k++) {
    sa += (double)(h[k * 4 + 1] - h[k * 4 + 0]);
    sb += (double)(h[k * 4 + 2] - h[k * 4 + 1]);
    sc += (double)(h[k * 4 + 3] - h[k * 4 + 2]);
  }
  std::fprintf(stderr, "[nipamd] phase cycles (mean over %d blocks): A %.0f  barrier %.0f  B %.0f\n",
               nblk, sa / nblk, sb / nblk, sc / nblk);
  double w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < nblk; k++)
    for (int i = 0; i < 8; i++) w[i] += (double)h[(size_t)nblk * 4 + k * 8 + i];
  if (w[0] + w[4] > 0)
    std::fprintf(stderr, "[nipamd] barrier wait cycles A/B: fwd filter %.0f/%.0f  bwd filter %.0f/%.0f  "
                 "fwd partner %.0f/%.0f  bwd partner %.0f/%.0f\n", w[0] / nblk, w[4] / nblk, w[1] / nblk,
                 w[5] / nblk, w[2] / nblk, w[6] / nblk, w[3] / nblk, w[7] / nblk);
  double pp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < nblk; k++)
    for (int i = 0; i < 8; i++) pp[i] += (double)h[(size_t)nblk * 16 + k * 8 + i];
  if (pp[0] + pp[4] > 0)
    std::fprintf(stderr, "[nipamd] phase-B partner cycles (DMA wait / ll / drain): fwd %.0f/%.0f/%.0f  "
                 "bwd %.0f/%.0f/%.0f\n", pp[0] / nblk, pp[1] / nblk, pp[2] / nblk, pp[4] / nblk, pp[5] / nblk,
                 pp[6] / nblk);
  const unsigned long long* rt = h + (size_t)nblk * 12;   // s_memrealtime (100 MHz)
  unsigned long long t0 = ~0ull, e0 = 0, e1 = ~0ull, s1 = 0;
  double mhz = 0, me = 0, st0 = 0;
  for (int k = 0; k < nblk; k++) {
    t0 = std::min(t0, rt[k * 4 + 0]); s1 = std::max(s1, rt[k * 4 + 0]);
    e0 = std::max(e0, rt[k * 4 + 2]); e1 = std::min(e1, rt[k * 4 + 2]);
    me += (double)(rt[k * 4 + 2] - rt[k * 4 + 0]);
    st0 += (double)(h[k * 4] - rt[k * 4 + 1]);
    if (rt[k * 4 + 2] > rt[k * 4 + 0])
      mhz += 100.0 * (double)(rt[k * 4 + 3] - rt[k * 4 + 1]) / (double)(rt[k * 4 + 2] - rt[k * 4 + 0]);
  }
  std::fprintf(stderr, "[nipamd] wall us: last entry %.2f  first end %.2f  last end %.2f  mean block %.2f  "
               "clock %.0f MHz; entry->stamp0 cycles %.0f\n", (s1 - t0) / 100.0, (e1 - t0) / 100.0,
               (e0 - t0) / 100.0, me / nblk / 100.0, mhz / nblk, st0 / nblk);
}
#endif

static bool chain_proper(const nipamd::ChainPlan& P);
static bool ckw_sparse_ok(const nipamd::ChainPlan& P, const Route& r, const bool (&seen)[4]);

// One launch of the chain kernel `kind` for route r: the interface
// variable's marginals (smoothed, or filtered) into dst rows (dbs / dts /
// doff), or only ll / status when dst is null.
static int launch_cur(nipamd_model* mm, const Route& r, ReqTables* rt, int kind, const int32_t* d_obs,
                      int n_obs, int B, int T, double* dst, long dbs, int dts, int doff,
                      double* d_ll, uint32_t* d_status, void* stream, bool filt) {
  const auto& P = mm->m.chain;
  DevState* d = dev_of(mm);
  const long ocols = n_obs > 0 ? n_obs : 1;
  if (kind == kMfmaWide) {
    // matrix-core interface chain: N <= 32, up to four observed children
    const int NT = P.N <= 16 ? 1 : 2;
    // chain_fb_ckw_kernel (round 6): smoothing at 17..32 states with one or
    // two observed columns where every recursion may rescale every 4th step
    // (ckw_sparse_ok): checkpoints + recomputation, no message round trip;
    // NIPAMD_FB_WIDE_KERNEL=mw in diagnostics builds keeps chain_mfma_wide_kernel
    if (NT == 2 && !filt && dst && r.ncol >= 1 && r.ncol <= 2 && P.emits.size() <= 4) {
      bool seen[4] = {false, false, false, false}, ok = true;
      int crows = 0;
      for (int i = 0; i < r.ncol; i++) {
        const int k = r.emit[i];
        if (k < 0 || k >= (int)P.emits.size() || seen[k]) ok = false;
        else seen[k] = true;
        if (ok) crows += P.emits[k].M + 2;
      }
      const char* wk = nipamd::diag_env("NIPAMD_FB_WIDE_KERNEL");
      if (ok && !(wk && std::string(wk) == "mw") && ckw_sparse_ok(P, r, seen)) {
        if (int rc = ensure_scratch(mm, nipamd::chain_estep_ckw_scratch_bytes(B, T))) return rc;
        nipamd::EMwArgs a{};
        a.obs = d_obs; a.obs_bstride = (long)T * ocols; a.obs_tstride = (int)ocols;
        a.ncol = r.ncol;
        for (int i = 0; i < 4; i++) {
          a.col[i] = i < r.ncol ? r.col[i] : 0;
          a.M[i] = i < r.ncol ? P.emit(r.emit[i]).M : 0;
          a.tab_off[i] = rt->mtab_off[i];
        }
        a.tab_rows = rt->mtab_rows; a.tab = rt->mtab;
        a.B = B; a.T = T; a.H = T / 2; a.N = P.N;
        a.A = d->A64; a.pi = d->pi64; a.w = rt->wv; a.S = d->S;
        a.ll = d_ll; a.status = d_status;
        a.post = dst; a.post_bstride = dbs; a.post_tstride = dts; a.post_off = doff;
#ifndef NIPAMD_FB_CKW_VL
#define NIPAMD_FB_CKW_VL 1          // A/B builds: 0 = the recomputed messages in registers, one wave per SIMD
#endif
        const char* vl = nipamd::diag_env("NIPAMD_FB_CKW_VL");
        const bool use_vl = vl ? std::atoi(vl) != 0 : NIPAMD_FB_CKW_VL != 0;
        const int lrc = nipamd::chain_fb_ckw_launch(a, chain_proper(P), use_vl, (hipStream_t)stream);
        if (lrc != nipamd::kLaunchRefused) return lrc ? launch_fail(lrc, "chain_fb_ckw_kernel") : 0;
      }
    }
    if (int rc = ensure_scratch(mm, filt ? 64 * sizeof(double) : nipamd::chain_mfma_wide_scratch_bytes(NT, B, T)))
      return rc;
    nipamd::WideMfmaArgs w{};
    w.obs = d_obs; w.obs_bstride = (long)T * ocols; w.obs_tstride = (int)ocols;
    w.ncol = r.ncol;
    for (int i = 0; i < 4; i++) {
      w.col[i] = i < r.ncol ? r.col[i] : 0;
      w.M[i] = i < r.ncol ? P.emit(r.emit[i]).M : 0;
      w.tab_off[i] = rt->mtab_off[i];
    }
    w.tab_rows = rt->mtab_rows; w.tab = rt->mtab;
    w.B = B; w.T = T; w.H = filt ? T : T / 2; w.N = P.N;
    w.A = d->A64; w.pi = d->pi64; w.w = rt->wv; w.S = d->S;
    w.post = dst;
    w.post_bstride = dbs; w.post_tstride = dts; w.post_off = doff;
    w.ll = d_ll; w.status = d_status;
#ifdef NIPAMD_DIAGNOSTICS
    static const bool mtimes = std::getenv("NIPAMD_PHASE_TIMES") != nullptr;
    const int nblk = (B + 15) / 16;
    if (mtimes && !filt) {
      HIP_OK(hipMalloc(&w.diag, (size_t)nblk * 16 * sizeof(unsigned long long)));
      HIP_OK(hipMemsetAsync(w.diag, 0, (size_t)nblk * 16 * sizeof(unsigned long long), (hipStream_t)stream));
    }
#endif
    if (int rc = nipamd::chain_mfma_wide_launch(w, NT, filt, (hipStream_t)stream))
      return launch_fail(rc, "chain_mfma_wide_kernel");
#ifdef NIPAMD_DIAGNOSTICS
    if (w.diag) {
      std::vector<unsigned long long> h((size_t)nblk * 16);
      HIP_OK(hipStreamSynchronize((hipStream_t)stream));
      HIP_OK(hipMemcpy(h.data(), w.diag, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      (void)hipFree(w.diag);
      double m[16] = {0};
      for (int k = 0; k < nblk; k++)
        for (int i = 0; i < 16; i++) m[i] += (double)h[(size_t)k * 16 + i] / nblk;
      static const char* names[4] = {"fwd filter", "bwd filter", "fwd partner", "bwd partner"};
      std::fprintf(stderr, "[nipamd] mfma_wide cycles per wave (phase A / its barrier waits / phase B / its barrier waits):\n");
      for (int v = 0; v < 4; v++)
        std::fprintf(stderr, "[nipamd]   %-12s %9.0f %9.0f %9.0f %9.0f\n", names[v], m[v * 4], m[v * 4 + 1], m[v * 4 + 2],
                     m[v * 4 + 3]);
    }
#endif
    return 0;
  }
  if (kind == kWide64) {
    // wide interface chain: N <= 64, up to four observed children
    if (int rc = ensure_scratch(mm, filt ? 64 * sizeof(double)
                                         : (size_t)(B + 2) * nipamd::chain_scratch_row64(T) * sizeof(double)))
      return rc;
    nipamd::WideArgs w{};
    w.filter = filt ? 1 : 0;
    w.obs = d_obs; w.obs_bstride = (long)T * ocols; w.obs_tstride = (int)ocols;
    w.ncol = r.ncol;
    for (int i = 0; i < r.ncol; i++) {
      w.col[i] = r.col[i];
      w.M[i] = P.emit(r.emit[i]).M;
      w.tab[i] = rt->tabw + rt->tabw_off[i];
    }
    w.ebase = rt->ebase;
    w.B = B; w.T = T; w.H = filt ? 0 : T / 2; w.N = P.N;
    w.A = d->A64; w.pi = d->pi64; w.s = d->sall64; w.S = d->S;
    w.post = dst;
    w.post_bstride = dbs; w.post_tstride = dts; w.post_off = doff;
    w.ll = d_ll; w.status = d_status;
#ifdef NIPAMD_DIAGNOSTICS
    static const bool wtimes = std::getenv("NIPAMD_PHASE_TIMES") != nullptr;
    if (wtimes && P.N > 32) {
      HIP_OK(hipMalloc(&w.diag, (size_t)B * 16 * sizeof(unsigned long long)));
      HIP_OK(hipMemsetAsync(w.diag, 0, (size_t)B * 16 * sizeof(unsigned long long), (hipStream_t)stream));
    }
#endif
    if (int rc = nipamd::chain_wide_launch(w, (hipStream_t)stream))
      return launch_fail(rc, "wide chain kernel");
#ifdef NIPAMD_DIAGNOSTICS
    if (w.diag) {
      std::vector<unsigned long long> h((size_t)B * 16);
      HIP_OK(hipStreamSynchronize((hipStream_t)stream));
      HIP_OK(hipMemcpy(h.data(), w.diag, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      (void)hipFree(w.diag);
      double m[16] = {0};
      for (int b = 0; b < B; b++)
        for (int i = 0; i < 16; i++) m[i] += (double)h[(size_t)b * 16 + i] / B;
      std::fprintf(stderr, "[nipamd] wide4 cycles (total / wait / before / after barrier): fwd filter %.0f / %.0f / %.0f / %.0f  "
                   "bwd filter %.0f / %.0f / %.0f / %.0f  partners %.0f %.0f  staging %.0f  block %.0f\n", m[0], m[1],
                   m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[12], m[9], m[10]);
      unsigned long long e0 = ~0ull, e1 = 0, x0 = ~0ull, x1 = 0;
      for (int b = 0; b < B; b++) {
        e0 = std::min(e0, h[(size_t)b * 16 + 11]); e1 = std::max(e1, h[(size_t)b * 16 + 11]);
        x0 = std::min(x0, h[(size_t)b * 16 + 13]); x1 = std::max(x1, h[(size_t)b * 16 + 13]);
      }
      std::fprintf(stderr, "[nipamd] wide4 wall us: entries spread %.2f  first exit %.2f  last exit %.2f\n",
                   (e1 - e0) / 100.0, (x0 - e0) / 100.0, (x1 - e0) / 100.0);
    }
#endif
    return 0;
  }
  if (kind != kNarrowMfma && kind != kNarrowDpp)
    return fail(NIPAMD_ERROR_UNSUPPORTED, "no interface-chain kernel fits this request");
  if (int rc = ensure_scratch(mm, nipamd::chain_scratch_bytes(B, T))) return rc;
  nipamd::ChainArgs a{};
  a.obs = r.pcol >= 0 ? d_obs : nullptr;
  a.obs_bstride = (long)T * ocols;
  a.obs_tstride = (int)ocols;
  a.obs_col = r.pcol;
  a.B = B; a.T = T; a.H = T / 2; a.N = P.N; a.M = rt->M0;
  a.A = d->A; a.Etab = rt->Etab16; a.pi = d->pi; a.ts = rt->ts16; a.S = d->S;
  a.post = dst;
  a.post_bstride = dbs;
  a.post_tstride = dts;
  a.post_off = doff;
  a.ll = d_ll;
  a.status = d_status;
#ifdef NIPAMD_DIAGNOSTICS
  static const bool times = std::getenv("NIPAMD_PHASE_TIMES") != nullptr;
  unsigned long long* stamps = nullptr;
  const int nblk = (int)((B + 15) / 16);
  if (kind == kNarrowMfma && times) {
    HIP_OK(hipMalloc(&stamps, (size_t)nblk * 24 * sizeof(unsigned long long)));
    HIP_OK(hipMemsetAsync(stamps, 0, (size_t)nblk * 24 * sizeof(unsigned long long), (hipStream_t)stream));
    a.counts = reinterpret_cast<double*>(stamps);
    // chain_ckpt.hip's per-wave stamps [block][8 waves][5]
    HIP_OK(hipMalloc(&a.diag, (size_t)nblk * 40 * sizeof(unsigned long long)));
    HIP_OK(hipMemsetAsync(a.diag, 0, (size_t)nblk * 40 * sizeof(unsigned long long), (hipStream_t)stream));
  }
#endif
  const int rc = kind == kNarrowMfma ? nipamd::chain_fb_mfma_launch(a, (hipStream_t)stream)
                                     : nipamd::chain_fb_launch(a, (hipStream_t)stream);
#ifdef NIPAMD_DIAGNOSTICS
  if (stamps) {
    std::vector<unsigned long long> h((size_t)nblk * 24);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    HIP_OK(hipMemcpy(h.data(), stamps, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    (void)hipFree(stamps);
    phase_report(h.data(), nblk);
    std::vector<unsigned long long> w((size_t)nblk * 40);
    HIP_OK(hipMemcpy(w.data(), a.diag, w.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    (void)hipFree(a.diag);
    double m[40] = {0};
    for (int k = 0; k < nblk; k++)
      for (int i = 0; i < 40; i++) m[i] += (double)w[(size_t)k * 40 + i] / nblk;
    if (m[2] > 0) {
      std::fprintf(stderr, "[nipamd] ckpt kernel cycles per wave (phase A / phase-barrier wait / phase B / "
                   "phase-B barrier waits / mean SIMD id; block 0's SIMD ids):\n");
      static const char* names[8] = {"fwd filter", "bwd filter", "fwd partner", "bwd partner", "idle 4", "idle 5",
                                     "beta recompute", "alpha recompute"};
      for (int v = 0; v < 8; v++)
        std::fprintf(stderr, "[nipamd]   %-16s %9.0f %9.0f %9.0f %9.0f %5.2f %llu\n", names[v], m[v * 5], m[v * 5 + 1],
                     m[v * 5 + 2], m[v * 5 + 3], m[v * 5 + 4], w[v * 5 + 4]);
    }
  }
#endif
  if (rc) return launch_fail(rc, kind == kNarrowMfma ? "chain_fb_mfma_kernel" : "chain_kernel");
  return 0;
}


// Joint interface, smoothing, every query one of the interface's current-slice
// variables: chain_fb_ckpt_kernel writes their marginals itself (digit sums of
// the normalised joint posterior, chain_ckpt.hip norm_store) instead of the
// joint posterior plus one project_kernel pass per variable.  *taken = false
// when the checkpoint kernel does not take the request (the caller falls back).
static int launch_joint_marginals(nipamd_model* mm, const Route& r, ReqTables* rt, const int32_t* d_obs,
                                  int n_obs, int B, int T, int n_query, const int* query, double* d_post,
                                  double* d_ll, uint32_t* d_status, void* stream, bool* taken) {
  *taken = false;
  const auto& P = mm->m.chain;
  if (!P.joint || P.N > 16 || n_query < 1 || n_query > 4) return 0;
  nipamd::ChainArgs a{};
  int stride = 0;
  for (int i = 0; i < n_query; i++) {
    const int kind = query_kind(P, query[i]);
    if (kind < 700 || kind >= 1000) return 0;
    const int k = kind - 700;
    int st = 1;
    for (int j = 0; j < k; j++) st *= mm->m.vars[P.jcur[j]].card;
    const int card = mm->m.vars[P.jcur[k]].card;
    a.proj_off[i] = stride;
    a.proj_card[i] = card;
    for (int s = 0; s < 16; s++) a.proj_digit[i][s] = (signed char)(s < P.N ? (s / st) % card : -1);
    stride += card;
  }
  a.nproj = n_query;
  if (int rc = ensure_scratch(mm, nipamd::chain_scratch_bytes(B, T))) return rc;
  DevState* d = dev_of(mm);
  const long ocols = n_obs > 0 ? n_obs : 1;
  a.obs = r.pcol >= 0 ? d_obs : nullptr;
  a.obs_bstride = (long)T * ocols;
  a.obs_tstride = (int)ocols;
  a.obs_col = r.pcol;
  a.B = B; a.T = T; a.H = T / 2; a.N = P.N; a.M = rt->M0;
  a.A = d->A; a.Etab = rt->Etab16; a.pi = d->pi; a.ts = rt->ts16; a.S = d->S;
  a.post = d_post;
  a.post_bstride = (long)T * stride;
  a.post_tstride = stride;
  a.ll = d_ll;
  a.status = d_status;
  const int rc = nipamd::chain_fb_ckpt_launch(a, (hipStream_t)stream);
  if (rc == -2) return 0;                            // not taken: the next kernel serves it
  if (rc) return launch_fail(rc, "chain_fb_ckpt_kernel");
  *taken = true;
  return 0;
}

static int rc_or_fail(int rc, const std::string& err) { return rc ? fail(rc, err) : 0; }

// forward_backward_inference (filt = false) / forward_inference (filt = true).
// The interface variable's marginals come from the chain kernels; every
// other queried variable's are derived from them (derive.hip), with the
// forward messages of a filter pass when a hidden parent is smoothed.
static int fb_impl(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                   int B, int T, int n_query, const int* query, double* d_post,
                   double* d_ll, uint32_t* d_status, void* stream, bool filt) {
  if (!mm || B < 0 || T < 1 || (n_obs > 0 && (!d_obs || !obs_vars)) || (n_query > 0 && (!query || !d_post)))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  for (int i = 0; i < n_query; i++)
    if (query[i] < 0 || query[i] >= (int)mm->m.vars.size()) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad query variable");
  if (B == 0) return 0;
  Route r;
  std::string why;
  int kk = kNoChain;
  ReqTables* rt = nullptr;
  if (mm->engine != NIPAMD_ENGINE_JTREE && route_request(mm, n_obs, obs_vars, n_query, query, r, why)) {
    if (int rc = ensure_tables(mm)) return rc;
    if (int rc = ensure_req_tables(mm, r, &rt)) return rc;
    kk = pick_kernel(mm, r, rt, T, filt);
    // smoothed hidden parents also need the forward messages of a filter pass
    for (int i = 0; i < n_query && kk != kNoChain && !filt; i++)
      if (query_kind(mm->m.chain, query[i]) >= 1000 && pick_kernel(mm, r, rt, T, true) == kNoChain) kk = kNoChain;
    if (kk == kNoChain) why = "sequence too long for the interface-chain kernels' LDS-resident codes";
  }
  if (kk == kNoChain && mm->engine == NIPAMD_ENGINE_AUTO) {
    // the evidence-indexed interface chain (opchain.h): the slice as one K x K
    // operator per evidence combination, K <= 16 joint interface states
    // (automatic engine choice only: NIPAMD_ENGINE_CHAIN is the chain plan's
    // kernels, NIPAMD_ENGINE_JTREE the general engine)
    std::string why2;
    if (nipamd::op_supported(mm, n_obs, obs_vars, n_query, query, why2) &&
        nipamd::op_fits(mm, n_obs, obs_vars, T)) {
      if (int rc = ensure_device(mm)) return rc;
      const auto& out = mm->m.outgoing;
      std::string err;
      int K = 0;
      if (n_query == 1 && out.size() == 1) {           // the interface variable itself: straight into its rows
        const int card = mm->m.vars[query[0]].card;
        return (rc_or_fail(nipamd::op_fb(mm, d_obs, n_obs, obs_vars, B, T, d_post, (long)T * card, card, 0, d_ll,
                                         d_status, stream, filt, &K, err), err));
      }
      long stride = 0;
      for (int i = 0; i < n_query; i++) stride += mm->m.vars[query[i]].card;
      long Kj = 1;
      for (int v : out) Kj *= mm->m.vars[v].card;
      if (int rc = ensure_q(mm, (size_t)B * T * Kj * sizeof(double))) return rc;
      double* q = dev_of(mm)->Q;
      if (int rc = nipamd::op_fb(mm, d_obs, n_obs, obs_vars, B, T, q, (long)T * Kj, (int)Kj, 0, d_ll, d_status,
                                 stream, filt, &K, err))
        return fail(rc, err);
      long off = 0;
      for (int i = 0; i < n_query; i++) {
        nipamd::DeriveArgs g{};
        g.kind = nipamd::kDeriveProject;
        g.filter = filt ? 1 : 0;
        g.B = B; g.T = T; g.N = (int)Kj;
        g.cur = q; g.cur_bstride = (long)T * Kj; g.cur_tstride = (int)Kj;
        g.alpha = q; g.al_bstride = g.cur_bstride; g.al_tstride = g.cur_tstride;
        g.out = d_post; g.out_bstride = (long)T * stride; g.out_tstride = (int)stride; g.out_off = (int)off;
        g.prev_stride = 1;
        for (size_t j = 0; j < out.size() && out[j] != query[i]; j++) g.prev_stride *= mm->m.vars[out[j]].card;
        g.prev_card = mm->m.vars[query[i]].card;
        g.child_col = -1;
        if (int rc = nipamd::derive_launch(g, (hipStream_t)stream))
          return launch_fail(rc, "derive_kernel");
        off += g.prev_card;
      }
      return 0;
    }
  }
  if (kk == kNoChain) {
    // the general join-tree engine (jtree.hip): any slice, any T
    if (mm->engine == NIPAMD_ENGINE_CHAIN) return fail(NIPAMD_ERROR_UNSUPPORTED, why);
    return nipamd::jt_fb(mm, d_obs, n_obs, obs_vars, B, T, n_query, query, d_post, d_ll, d_status,
                         stream, filt);
  }
  if (!filt && kk == kNarrowMfma && mm->m.chain.joint) {
    bool taken = false;
    if (int rc = launch_joint_marginals(mm, r, rt, d_obs, n_obs, B, T, n_query, query, d_post, d_ll, d_status,
                                        stream, &taken))
      return rc;
    if (taken) return 0;
  }
  const auto& P = mm->m.chain;
  std::vector<int> kind(n_query), off(n_query);
  int stride = 0, first_cur = -1;
  bool derived = false, fwd_msgs = false;
  for (int i = 0; i < n_query; i++) {
    kind[i] = query_kind(P, query[i]);
    off[i] = stride;
    stride += mm->m.vars[query[i]].card;
    if (kind[i] == 0) { if (first_cur < 0) first_cur = i; }
    else { derived = true; fwd_msgs |= kind[i] >= 1000 && !filt; }
  }
  const long pbs = (long)T * stride;
  const int N = P.N;
  const size_t per = (size_t)B * T * N;
  // where the interface marginals live: the first query slot naming the
  // interface variable, or (derived queries only) the work buffer Q
  double* cur = nullptr;
  long cbs = 0;
  int cts = 0;
  double* fwd = nullptr;
  if (derived) {
    const size_t need = (first_cur < 0 ? per : 0) + (fwd_msgs ? per : 0);
    if (need) if (int rc = ensure_q(mm, need * sizeof(double))) return rc;
    double* q = dev_of(mm)->Q;
    if (first_cur < 0) { cur = q; cbs = (long)T * N; cts = N; q += per; }
    else { cur = d_post + off[first_cur]; cbs = pbs; cts = stride; }
    if (fwd_msgs) fwd = q;
  }
  bool first = true;
  for (int i = 0; i < n_query; i++) {
    if (kind[i] != 0) continue;
    if (int rc = launch_cur(mm, r, rt, kk, d_obs, n_obs, B, T, d_post, pbs, stride, off[i],
                            first ? d_ll : nullptr, first ? d_status : nullptr, stream, filt)) return rc;
    first = false;
  }
  if (first)       // no query slot names the interface variable
    if (int rc = launch_cur(mm, r, rt, kk, d_obs, n_obs, B, T, cur, cbs, cts, 0, d_ll, d_status, stream, filt)) return rc;
  if (fwd_msgs)    // the forward messages: a filter pass
    if (int rc = launch_cur(mm, r, rt, pick_kernel(mm, r, rt, T, true), d_obs, n_obs, B, T, fwd, (long)T * N, N, 0,
                            nullptr, nullptr, stream, true))
      return rc;
  if (!derived) return 0;
  DevState* d = dev_of(mm);
  const long ocols = n_obs > 0 ? n_obs : 1;
  for (int i = 0; i < n_query; i++) {
    if (kind[i] == 0) continue;
    nipamd::DeriveArgs g{};
    g.filter = filt ? 1 : 0;
    g.B = B; g.T = T; g.N = N;
    g.cur = cur; g.cur_bstride = cbs; g.cur_tstride = cts;
    if (fwd) { g.alpha = fwd; g.al_bstride = (long)T * N; g.al_tstride = N; }
    else { g.alpha = cur; g.al_bstride = cbs; g.al_tstride = cts; }
    g.out = d_post; g.out_bstride = pbs; g.out_tstride = stride; g.out_off = off[i];
    g.A = d->A64; g.pi = d->pi64;
    g.obs = d_obs; g.obs_bstride = (long)T * ocols; g.obs_tstride = (int)ocols;
    g.ncol = r.ncol;
    for (int c = 0; c < r.ncol; c++) {
      g.col[c] = r.col[c];
      g.M[c] = P.emit(r.emit[c]).M;
      g.tab[c] = rt->tabw + rt->tabw_off[c];
    }
    g.ebase = rt->ebase;
    g.child_col = -1;
    if (kind[i] == 1) {
      g.kind = nipamd::kDerivePrev;
    } else if (kind[i] >= 500 && kind[i] < 1000) {
      // a joint interface's variable: its digit of the joint interface
      // marginal (current slice), or of the derived previous-interface one
      const bool is_prev = kind[i] < 700;
      const int k = kind[i] - (is_prev ? 500 : 700);
      const auto& vs = is_prev ? P.jprev : P.jcur;
      g.kind = is_prev ? nipamd::kDerivePrev : nipamd::kDeriveProject;
      g.prev_stride = 1;
      for (int j = 0; j < k; j++) g.prev_stride *= mm->m.vars[vs[j]].card;
      g.prev_card = mm->m.vars[vs[k]].card;
    } else if (kind[i] < 1000) {
      const int k = kind[i] - 2;
      g.kind = nipamd::kDeriveChild;
      g.child_M = P.emits[k].M;
      g.child_E = d->childE[k];
      for (int c = 0; c < r.ncol; c++) if (r.emit[c] == k) g.child_col = r.col[c];
    } else {
      const int j = kind[i] - 1000;
      if (int rc = ensure_hidden(mm, j)) return rc;
      g.kind = nipamd::kDeriveHidden;
      g.hid_card = mm->m.vars[P.hidden[j]].card;
      g.G = d->G[j];
    }
    if (int rc = nipamd::derive_launch(g, (hipStream_t)stream))
      return launch_fail(rc, "derive_kernel");
  }
  return 0;
}

int nipamd_fb(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
              int B, int T, int n_query, const int* query, double* d_post,
              double* d_ll, uint32_t* d_status, void* stream) {
  return fb_impl(mm, d_obs, n_obs, obs_vars, B, T, n_query, query, d_post, d_ll, d_status, stream, false);
}

int nipamd_filter(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                  int B, int T, int n_query, const int* query, double* d_post,
                  double* d_ll, uint32_t* d_status, void* stream) {
  return fb_impl(mm, d_obs, n_obs, obs_vars, B, T, n_query, query, d_post, d_ll, d_status, stream, true);
}

// host-buffer form of fb_impl (PCIe-inclusive, synchronous)
static int fb_host_impl(nipamd_model* mm, const int32_t* obs, int n_obs, const int* obs_vars,
                        int B, int T, int n_query, const int* query, double* post,
                        double* ll, uint32_t* status, bool filt) {
  if (!mm || B < 0 || T < 1 || n_query < 0 || (n_query > 0 && !query) || (n_obs > 0 && (!obs || !obs_vars)))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  for (int i = 0; i < n_query; i++)
    if (query[i] < 0 || query[i] >= (int)mm->m.vars.size()) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad query variable");
  if (B == 0) return 0;
  int stride = 0;
  for (int i = 0; i < n_query; i++) stride += mm->m.vars[query[i]].card;
  DevBufs db;
  int32_t* d_obs = nullptr; double* d_post = nullptr; double* d_ll = nullptr; uint32_t* d_st = nullptr;
  const size_t nob = (size_t)B * T * (n_obs > 0 ? n_obs : 1);
  const size_t npo = (size_t)B * T * (stride > 0 ? stride : 1);
  if (int rc = db.alloc(&d_obs, nob)) return rc;
  if (int rc = db.alloc(&d_post, npo)) return rc;
  if (int rc = db.alloc(&d_ll, (size_t)B)) return rc;
  if (int rc = db.alloc(&d_st, (size_t)B)) return rc;
  if (n_obs > 0) HIP_OK(hipMemcpy(d_obs, obs, nob * sizeof(int32_t), hipMemcpyHostToDevice));
  int rc = fb_impl(mm, d_obs, n_obs, obs_vars, B, T, n_query, query, d_post, d_ll, d_st, nullptr, filt);
  if (rc == 0) {
    HIP_OK(hipDeviceSynchronize());
    if (post && stride > 0) HIP_OK(hipMemcpy(post, d_post, npo * sizeof(double), hipMemcpyDeviceToHost));
    if (ll) HIP_OK(hipMemcpy(ll, d_ll, (size_t)B * sizeof(double), hipMemcpyDeviceToHost));
    if (status) HIP_OK(hipMemcpy(status, d_st, (size_t)B * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  return rc;
}

int nipamd_fb_host(nipamd_model* mm, const int32_t* obs, int n_obs, const int* obs_vars,
                   int B, int T, int n_query, const int* query, double* post,
                   double* ll, uint32_t* status) {
  return fb_host_impl(mm, obs, n_obs, obs_vars, B, T, n_query, query, post, ll, status, false);
}

int nipamd_filter_host(nipamd_model* mm, const int32_t* obs, int n_obs, const int* obs_vars,
                       int B, int T, int n_query, const int* query, double* post,
                       double* ll, uint32_t* status) {
  return fb_host_impl(mm, obs, n_obs, obs_vars, B, T, n_query, query, post, ll, status, true);
}

// The chain e_step kernels serve interface chains with evidence on their
// leaf children; every other e_step runs on the general engine, whose partial
// is the em_learn layout itself.  The partial is [body | route tag]: the body
// holds any layout the model's routes produce (the largest of the sizes), the
// three tag slots count the partials summed into it per route -- (1, 0, 0)
// the 16-state chain slab, (0, 1, 0) em_learn layout, (0, 0, 1) the wide
// chain slab (estep_wide.hip) -- so partials of different routes (another T,
// another engine setting, another rank) that were combined are detected by
// the finalize instead of being summed silently.
// A chain plan the general 16-state chain e_step takes: one interface
// variable of at most 16 states, 1..3 leaf children, hidden independent
// parents (their families follow from the xi sums, ensure_chain_map).
static bool estep_general_plan(const nipamd::ChainPlan& P) {
  return P.valid && !P.joint && !P.hmm && P.N <= 16 && !P.emits.empty() && P.emits.size() <= 3 &&
         !P.fold_gpu;
}
// the count-table rows of every child: sum_k (M_k + 2)
static int estep_rows(const nipamd::ChainPlan& P) {
  int R = 0;
  for (const auto& e : P.emits) R += e.M + 2;
  return R;
}
static bool chain_map_supported(const nipamd::Model& m);
// A chain plan the wide chain e_step takes (estep_wide.hip): one interface
// variable of at most 64 states, 1..4 leaf children, hidden independent
// parents, in-cliques folded on the GPU (config 3's and config 5's models).
static bool estep_wide_plan(const nipamd::Model& m) {
  const auto& P = m.chain;
  return P.valid && !P.joint && !P.emits.empty() && P.emits.size() <= 4 &&
         nipamd::estep_wide_fits(P.N, estep_rows(P)) && chain_map_supported(m);
}
constexpr int kTagSlots = 3;

// The body is the larger of the layouts this model's routes can produce,
// whatever the engine setting, so the tag sits at the same offset for every
// partial of a model version (a set_engine between partial and finalize
// cannot move it into the counts).
static bool has_chain_estep(const nipamd::Model& m) {
  const auto& P = m.chain;
  return P.valid && (P.hmm || P.jhmm || estep_general_plan(P) || estep_wide_plan(m));
}
static int estep_body_size(const nipamd_model* mm) {
  int body = nipamd::param_size(mm->m);
  const auto& P = mm->m.chain;
  if (P.valid && (P.hmm || P.jhmm)) body = std::max(body, nipamd::chain_estep_slab(P.emits[0].M));
  if (estep_general_plan(P)) body = std::max(body, nipamd::chain_estep_slab(estep_rows(P) - 2));
  if (estep_wide_plan(mm->m)) body = std::max(body, nipamd::estep_wide_slab(P.N, estep_rows(P)));
  return body;
}

int nipamd_estep_partial_size(const nipamd_model* mm) {
  if (!mm) return -1;
  if (mm->engine == NIPAMD_ENGINE_CHAIN && !has_chain_estep(mm->m)) return -1;
  return estep_body_size(mm) + kTagSlots;
}

static bool chain_estep_ok(const nipamd_model* mm, int n_obs, const int* obs_vars, int T, Route& r);
static bool wide_estep_ok(const nipamd_model* mm, int n_obs, const int* obs_vars, Route& r);

// The request's route is the operator chain's e_step (the chain and wide
// routes decline it, the engine choice is automatic and the operator chain
// takes it): its partial carries a section after the route tag.
// capacity: the caller's partial in doubles (-1: unbounded, the size query).
// The operator chain's partial is larger than nipamd_estep_partial_size, so a
// partial of that size (nipamd_estep_partial, which takes no capacity) runs
// such requests on the general engine, whose partial fits.
static bool op_estep_route(nipamd_model* mm, int n_obs, const int* obs_vars, int T, long capacity) {
  Route r;
  if (mm->engine != NIPAMD_ENGINE_AUTO || chain_estep_ok(mm, n_obs, obs_vars, T, r) ||
      wide_estep_ok(mm, n_obs, obs_vars, r))
    return false;
  std::string why;
  if (!nipamd::op_estep_supported(mm, n_obs, obs_vars, T, why)) return false;
  return capacity < 0 ||
         capacity >= (long)nipamd_estep_partial_size(mm) + (long)nipamd::op_estep_section(mm, n_obs, obs_vars);
}

int nipamd_estep_partial_size_req(nipamd_model* mm, int n_obs, const int* obs_vars, int T) {
  if (!mm || T < 1 || (n_obs > 0 && !obs_vars)) return -1;
  const int base = nipamd_estep_partial_size(mm);
  if (base < 0 || !op_estep_route(mm, n_obs, obs_vars, T, -1)) return base;
  return base + (int)nipamd::op_estep_section(mm, n_obs, obs_vars);
}

// e_step kernel of the chain route: 3 = chain_estep16_kernel (16-lane DPP
// rows, direction-uniform waves, analytic phase-B normalisation; the
// default), 2 = chain_kernel<true> (the round-2 DPP kernel, mixed-direction
// waves; NIPAMD_ESTEP_KERNEL=dpp8 in diagnostics builds, or when the 16-seq
// block's LDS does not fit), 1 = the matrix-core kernel (NIPAMD_ESTEP_KERNEL=mfma).
// Measured on config 4.
static bool estep16_sparse_ok(const nipamd::ChainPlan& P, int ne);
static int chain_estep_kernel(const nipamd_model* mm, int T) {
  const auto& P = mm->m.chain;
  if (estep_general_plan(P))                       // only chain_estep16_kernel takes several children
    return nipamd::chain_estep16_lds_bytes(estep_rows(P) - 2, T, (int)P.emits.size()) <= 160 * 1024 ? 3 : 0;
  const int M = P.emits[0].M;
  const char* ek = nipamd::diag_env("NIPAMD_ESTEP_KERNEL");
  const std::string want = ek ? ek : "";
  // 4 = chain_estep_ck_kernel (checkpoints + recomputation, round 6): the
  // default where both recursions may rescale every 4th step (the host's
  // underflow bound) and its count tables fit; NIPAMD_ESTEP_KERNEL=e16 in
  // diagnostics builds runs chain_estep16_kernel instead
  if (want != "mfma" && want != "dpp8" && want != "e16" && P.N <= 16 && P.hmm &&
      nipamd::chain_estep_ck_lds_bytes(M) <= 160 * 1024 && estep16_sparse_ok(P, 1))
    return 4;
  if (want == "mfma" && P.N <= 16 && M <= 16 && nipamd::chain_estep_mfma_lds_bytes(M, T) <= 160 * 1024) return 1;
  if (want != "dpp8" && P.N <= 16 && nipamd::chain_estep16_lds_bytes(M, T, 1) <= 160 * 1024) return 3;
  if (nipamd::chain_lds_bytes(M, T, true) <= 96 * 1024) return 2;
  return 0;
}

// The chain's transition rows and every child's rows sum to 1 within 1e-15
// (normalised CPTs; every m_step's output): the reference's per-step
// log m2 - log m1 then telescope to log P(obs) (m1_t is the previous step's
// mass), which chain_estep16_kernel's proper mode computes from the final
// forward mass -- the ll differs by the tables' rounding, <= T x 1e-15.
static bool chain_proper(const nipamd::ChainPlan& P) {
  if (P.N > 64) return false;
  for (int x = 0; x < P.N; x++) {
    double r = 0.0;
    for (int y = 0; y < P.N; y++) r += P.A64[x * 64 + y];
    if (!(std::fabs(r - 1.0) <= 1e-15)) return false;
  }
  for (const auto& E : P.emits)
    for (int y = 0; y < P.N; y++)
      if (!(std::fabs(E.s[y] - 1.0) <= 1e-15)) return false;
  return true;
}

// chain_estep16_kernel's proper mode may let the forward rows rescale every
// 4th step (as the backward rows do) when no step can shrink a vector's
// largest entry by more than 1e-30: then either direction's vector keeps its
// largest entry above 1e-120 between rescales and phase B's products
// alpha^ beta^ stay far above the subnormals.  Bound: for every previous
// state x and every code o (the missing row included), the largest entry of
// row x of A times the evidence column of o.  One child only (the HMM shape);
// otherwise every step rescales (tests/test_gpu_estep.py peaked models).
static bool estep16_sparse_ok(const nipamd::ChainPlan& P, int ne) {
  if (ne != 1 || P.emits.empty() || P.N > 64) return false;
  const auto& E = P.emits[0];
  for (int o = 0; o <= E.M; o++)
    for (int x = 0; x < P.N; x++) {
      double best = 0.0;
      for (int y = 0; y < P.N; y++)
        best = std::max(best, P.A64[x * 64 + y] * (o < E.M ? E.E[(size_t)o * 64 + y] : E.s[y]));
      if (!(best >= 1e-30)) return false;
    }
  return true;
}

static bool chain_estep_ok(const nipamd_model* mm, int n_obs, const int* obs_vars, int T, Route& r) {
  std::string why;
  const auto& P = mm->m.chain;
  const bool general = estep_general_plan(P);
  if (mm->engine == NIPAMD_ENGINE_JTREE || !P.valid || !(P.hmm || P.jhmm || general)) return false;
  if (!route_request(mm, n_obs, obs_vars, 0, nullptr, r, why)) return false;
  if (general) {                                   // evidence on leaf children only (not on the interface)
    for (int i = 0; i < r.ncol; i++) if (r.emit[i] >= (int)P.emits.size()) return false;
  } else if (r.ncol > 1 || (r.ncol == 1 && r.emit[0] != 0)) {
    return false;                                  // evidence on the child only
  }
  return chain_estep_kernel(mm, T) != 0;
}

// the wide chain e_step: evidence on leaf children only
static bool wide_estep_ok(const nipamd_model* mm, int n_obs, const int* obs_vars, Route& r) {
  std::string why;
  const auto& P = mm->m.chain;
  if (mm->engine == NIPAMD_ENGINE_JTREE || !estep_wide_plan(mm->m)) return false;
  if (!route_request(mm, n_obs, obs_vars, 0, nullptr, r, why)) return false;
  for (int i = 0; i < r.ncol; i++) if (r.emit[i] >= (int)P.emits.size()) return false;
  return true;
}

// The reference's verdict on a leading run of missing observations
// (prefix.cpp), once per model version and T; -1: no step is rejected.
// prefix.cpp bounds its own work (entries x steps); models whose join tree
// holds more than kPrefixMaxEntries table entries are not simulated at all
// (-2: their leading missing runs are accepted).
constexpr long kPrefixMaxEntries = 1L << 26;

static int prefix_first_bad(nipamd_model* mm, int T) {
  const int c = mm->pf_first_bad;
  // -1 holds for every shorter T, a step >= 0 for every T, -2 (the work bound
  // ran out) for every longer T
  const bool hit = mm->pf_version == mm->version &&
                   (c >= 0 || (c == -1 && T <= mm->pf_T) || (c == -2 && T >= mm->pf_T));
  if (!hit) {
    mm->pf_first_bad = nipamd::estep_prefix_entries(mm->m) > kPrefixMaxEntries
                           ? -2 : nipamd::estep_prefix_first_bad(mm->m, T, nullptr);
    mm->pf_version = mm->version;
    mm->pf_T = T;
  }
  const int k = mm->pf_first_bad;
  return k >= 0 && k < T ? k : -1;
}

static int estep_partial_routes(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                                int B, int T, double* d_partial, long capacity, double* d_ll,
                                uint32_t* d_status, void* stream);
static int ensure_etab_all(nipamd_model* mm);
static int estep_partial_cap(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                             int B, int T, double* d_partial, long capacity, double* d_ll,
                             uint32_t* d_status, void* stream);

int nipamd_estep_partial(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                         int B, int T, double* d_partial, double* d_ll, uint32_t* d_status,
                         void* stream) {
  if (!mm) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const int base = nipamd_estep_partial_size(mm);
  return estep_partial_cap(mm, d_obs, n_obs, obs_vars, B, T, d_partial, base > 0 ? base : 0, d_ll, d_status,
                           stream);
}

int nipamd_estep_partial_ex(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                            int B, int T, double* d_partial, long capacity, double* d_ll,
                            uint32_t* d_status, void* stream) {
  if (!mm) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const int base = nipamd_estep_partial_size(mm);
  if (base >= 0 && capacity < base)
    return fail(NIP_ERROR_INVALID_ARGUMENT, "partial capacity below nipamd_estep_partial_size");
  return estep_partial_cap(mm, d_obs, n_obs, obs_vars, B, T, d_partial, capacity, d_ll, d_status, stream);
}

static int estep_partial_cap(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                             int B, int T, double* d_partial, long capacity, double* d_ll,
                             uint32_t* d_status, void* stream) {
  if (!mm || B < 0 || T < 1 || !d_partial || (n_obs > 0 && (!d_obs || !obs_vars)))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  // The reference rejects series whose leading missing run reaches the
  // model's verdict step (BAD_LUCK): without d_status that verdict could not
  // be reported, and the partial would include counts the reference drops.
  if (!d_status && B > 0 && prefix_first_bad(mm, T) >= 0)
    return fail(NIP_ERROR_INVALID_ARGUMENT,
                "d_status is required: this model's e_step rejects series with a long leading missing run");
  if (int rc = estep_partial_routes(mm, d_obs, n_obs, obs_vars, B, T, d_partial, capacity, d_ll, d_status,
                                    stream))
    return rc;
  if (!d_status || B == 0) return 0;
  // the kernels are queued: this host work overlaps them
  const int k = prefix_first_bad(mm, T);
  if (k < 0) return 0;
  unsigned trivial = 0;                          // columns observing a one-state variable
  for (int c = 0; c < n_obs && c < 32; c++)
    if (obs_vars[c] >= 0 && obs_vars[c] < (int)mm->m.vars.size() && mm->m.vars[obs_vars[c]].card == 1)
      trivial |= 1u << c;
  if (nipamd::estep_prefix_flag_launch(d_obs, n_obs, B, T, k, trivial, d_status, (hipStream_t)stream))
    return fail(NIPAMD_ERROR_DEVICE, "prefix flag launch failed");
  return 0;
}

int nipamd_tree_sum(const double* d_rows, long n, int S, double* d_work, double* d_out, void* stream) {
  if (n < 0 || S < 1 || !d_out || (n > 0 && !d_rows) || (n > 64 && !d_work))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  if (n == 0) {
    HIP_OK(hipMemsetAsync(d_out, 0, (size_t)S * sizeof(double), (hipStream_t)stream));
    return 0;
  }
  double* tA = d_work;
  double* tB = d_work ? d_work + (size_t)((n + 63) / 64) * S : nullptr;
  if (reduce_rows(d_rows, n, S, tA, tB, d_out, (hipStream_t)stream))
    return fail(NIPAMD_ERROR_DEVICE, "tree launch failed");
  return 0;
}

int nipamd_estep_tail(const double* d_ll, const uint32_t* d_status, long B, double* d_work, double* d_out2,
                      void* stream) {
  if (B < 0 || !d_out2 || (B > 0 && (!d_ll || !d_status || !d_work)))
    return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  if (int rc = nipamd_tree_sum(d_ll, B, 1, d_work, d_out2, stream)) return rc;
  if (B == 0) {
    HIP_OK(hipMemsetAsync(d_out2 + 1, 0, sizeof(double), (hipStream_t)stream));
    return 0;
  }
  // the count's block parts after the tree's levels in the workspace
  double* cw = d_work + (B > 64 ? 2 * ((B + 63) / 64) : 0);
  if (nipamd::count_failed_launch(d_status, B, cw, d_out2 + 1, (hipStream_t)stream))
    return fail(NIPAMD_ERROR_DEVICE, "count launch failed");
  return 0;
}

int nipamd_estep_prefix_first_bad(nipamd_model* mm, int T) {
  if (!mm || T < 1) { fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments"); return -2; }
  if (nipamd::estep_prefix_entries(mm->m) > kPrefixMaxEntries) return -2;
  const int k = prefix_first_bad(mm, T);
  // -2: the simulation's work bound ran out (not simulated), not "no step"
  return k < 0 && mm->pf_first_bad == -2 ? -2 : k;
}

// A route writes the first `written` doubles of the body; the rest (another
// route's larger layout) is zeroed, so every partial is fully defined and
// partials of one route combine and compare bit for bit.
static int zero_tail(nipamd_model* mm, double* d_partial, int written, hipStream_t st) {
  const int body = estep_body_size(mm);
  if (written < body) HIP_OK(hipMemsetAsync(d_partial + written, 0, (size_t)(body - written) * sizeof(double), st));
  return 0;
}

// chain_estep_ckw_kernel rescales each recursion every 4th step: allowed when
// no step can shrink a vector's largest entry by more than 1e-30 (the bound of
// estep16_sparse_ok at several columns).  For every previous state x: the
// largest over y of A[x][y] times the smallest evidence any code combination
// gives y (per column the smallest of its rows, missing included; column 0
// carries the unobserved children's row sums).
static bool ckw_sparse_ok(const nipamd::ChainPlan& P, const Route& r, const bool (&seen)[4]) {
  if (P.N > 64) return false;
  std::vector<double> ev(P.N, 1.0);
  for (int k = 0; k < (int)P.emits.size() && k < 4; k++)
    if (!seen[k])
      for (int y = 0; y < P.N; y++) ev[y] *= P.emits[k].s[y];
  for (int i = 0; i < r.ncol; i++) {
    const auto& E = P.emit(r.emit[i]);
    for (int y = 0; y < P.N; y++) {
      double lo = E.s[y];
      for (int o = 0; o < E.M; o++) lo = std::min(lo, E.E[(size_t)o * 64 + y]);
      ev[y] *= lo;
    }
  }
  for (int x = 0; x < P.N; x++) {
    double best = 0.0;
    for (int y = 0; y < P.N; y++) best = std::max(best, P.A64[x * 64 + y] * ev[y]);
    if (!(best >= 1e-30)) return false;
  }
  return true;
}

// The wide chain e_step (estep_wide.hip): the filters store every message of
// a chunk of sequences, the statistics kernel writes one slab row per 16
// sequences, and the fixed-order tree sums the rows (per chunk, then over
// the chunks) into the partial.
// The fused matrix-core e_step (estep_mw.hip) for 17..32 states: the wide
// slab layout (K [32][32], H [R][32], P0 [32]), one row per 16 sequences.
// taken = false (nothing done) when the request does not fit the kernel: the
// caller takes the two-kernel route.
static int estep_mw_partial(nipamd_model* mm, const Route& r, const int32_t* d_obs, int n_obs, int B, int T,
                            double* d_partial, double* d_ll, uint32_t* d_status, void* stream, bool& taken) {
  const auto& P = mm->m.chain;
  taken = false;
  if (nipamd::estep_wide_np(P.N) != 32 || r.ncol > nipamd::estep_mw_max_cols() || P.emits.size() > 4) return 0;
  if (nipamd::diag_env("NIPAMD_ESTEP_WIDE_TWO_KERNELS")) return 0;   // A/B: the round-4 route
  int rows = 0;
  bool seen[4] = {false, false, false, false};
  for (int i = 0; i < r.ncol; i++) {
    const int k = r.emit[i];
    if (k < 0 || k >= (int)P.emits.size() || seen[k]) return 0;
    seen[k] = true;
    rows += P.emits[k].M;
  }
  if (rows > 64) return 0;
  if (int rc = ensure_tables(mm)) return rc;
  ReqTables* rt = nullptr;
  if (int rc = ensure_req_tables(mm, r, &rt)) return rc;
  if (nipamd::estep_mw_lds_bytes(rt->mtab_rows) > 160 * 1024) return 0;
  taken = true;
  const int R = estep_rows(P);
  const int S = nipamd::estep_wide_slab(P.N, R);
  hipStream_t st = (hipStream_t)stream;
  if (nipamd::estep_tag_launch(d_partial + estep_body_size(mm), 0.0, 0.0, 1.0, st))
    return fail(NIPAMD_ERROR_DEVICE, "tag launch failed");
  if (int rc = zero_tail(mm, d_partial, S, st)) return rc;
  if (B == 0) { HIP_OK(hipMemsetAsync(d_partial, 0, (size_t)S * sizeof(double), st)); return 0; }
  // chain_estep_ckw_kernel (checkpoints + recomputation, round 6): the
  // default where every step may rescale every 4th step (ckw_sparse_ok) and
  // its LDS fits; NIPAMD_ESTEP_WIDE_KERNEL=mw in diagnostics builds runs
  // chain_estep_mw_kernel instead
  int crows = 0;
  for (int i = 0; i < r.ncol; i++) crows += P.emit(r.emit[i]).M + 2;
  const char* wk = nipamd::diag_env("NIPAMD_ESTEP_WIDE_KERNEL");
  const bool ck = !(wk && std::string(wk) == "mw") && r.ncol >= 1 && r.ncol <= 2 &&
                  nipamd::chain_estep_ckw_lds_bytes(rt->mtab_rows, crows) <= 160 * 1024 && ckw_sparse_ok(P, r, seen);
  // sequences per launch: a power of two (the chunk trees are subtrees of the
  // batch's tree), scratch within ~8 GB: config 3's 65,536 x 256 in one launch
  const size_t per_seq = ck ? nipamd::chain_estep_ckw_scratch_bytes(16, T) / 16 + 1
                            : nipamd::estep_mw_scratch_bytes(32, T) / 32 + 1;
  const size_t cap = std::min<size_t>(65536, std::max<size_t>(32, ((size_t)8 << 30) / per_seq));
  long chunk = 32;
  while ((size_t)chunk * 2 <= cap) chunk *= 2;
  if (B < chunk) chunk = B;
  const long nchunks = (B + chunk - 1) / chunk;
  const long srows = (chunk + 15) / 16;
  const long lvl = (srows + 63) / 64;
  const size_t work = ((size_t)srows + 2 * lvl + nchunks + 64) * S * sizeof(double);
  if (int rc = ensure_scratch(mm, ck ? nipamd::chain_estep_ckw_scratch_bytes(chunk, T)
                                     : nipamd::estep_mw_scratch_bytes(chunk, T))) return rc;
  if (int rc = ensure_work(mm, work)) return rc;
  DevState* d = dev_of(mm);
  double* slab = d->W;
  double* tA = slab + (size_t)srows * S;
  double* tB = tA + (size_t)lvl * S;
  double* cres = tB + (size_t)lvl * S;
  const long ocols = n_obs > 0 ? n_obs : 1;
  nipamd::EMwArgs a{};
  a.obs_bstride = (long)T * ocols;
  a.obs_tstride = (int)ocols;
  a.ncol = r.ncol;
  for (int i = 0, v = 0; i < 4; i++) {
    a.col[i] = i < r.ncol ? r.col[i] : 0;
    a.M[i] = i < r.ncol ? P.emit(r.emit[i]).M : 0;
    a.tab_off[i] = rt->mtab_off[i];
    a.voff[i] = v;
    v += a.M[i];
  }
  for (int k = 0, row = 0; k < (int)P.emits.size(); k++) {
    for (int i = 0; i < r.ncol; i++)
      if (r.emit[i] == k) a.crow[i] = row;
    if (!seen[k]) {
      a.urow[a.n_unobs] = row;
      a.uM[a.n_unobs++] = P.emits[k].M;
    }
    row += P.emits[k].M + 2;
  }
  a.tab_rows = rt->mtab_rows; a.tab = rt->mtab;
  a.T = T; a.H = T / 2; a.N = P.N;
  a.A = d->A64; a.pi = d->pi64; a.w = rt->wv; a.S = d->S;
  a.slab = slab; a.slab_size = S; a.R = R;
  for (long c = 0; c < nchunks; c++) {
    const long b0 = c * chunk;
    const long nb = (B - b0) < chunk ? (B - b0) : chunk;
    a.obs = d_obs ? d_obs + b0 * T * ocols : nullptr;
    a.B = nb;
    a.ll = d_ll ? d_ll + b0 : nullptr;
    a.status = d_status ? d_status + b0 : nullptr;
    const int lrc = ck ? nipamd::chain_estep_ckw_launch(a, chain_proper(P), st) : nipamd::estep_mw_launch(a, st);
    if (lrc) return launch_fail(lrc, ck ? "chain_estep_ckw_kernel" : "chain_estep_mw_kernel");
    double* out = nchunks == 1 ? d_partial : cres + (size_t)c * S;
    if (reduce_rows(slab, (nb + 15) / 16, S, tA, tB, out, st))
      return fail(NIPAMD_ERROR_DEVICE, "reduction launch failed");
  }
  if (nchunks > 1 && reduce_rows(cres, nchunks, S, tA, tB, d_partial, st))
    return fail(NIPAMD_ERROR_DEVICE, "reduction launch failed");
  return 0;
}

static int estep_wide_partial(nipamd_model* mm, const Route& r, const int32_t* d_obs, int n_obs, int B, int T,
                              double* d_partial, double* d_ll, uint32_t* d_status, void* stream) {
  const auto& P = mm->m.chain;
  {
    bool taken = false;
    const int rc = estep_mw_partial(mm, r, d_obs, n_obs, B, T, d_partial, d_ll, d_status, stream, taken);
    if (rc || taken) return rc;
  }
  const int R = estep_rows(P);
  const int S = nipamd::estep_wide_slab(P.N, R);
  hipStream_t st = (hipStream_t)stream;
  if (nipamd::estep_tag_launch(d_partial + estep_body_size(mm), 0.0, 0.0, 1.0, st))
    return fail(NIPAMD_ERROR_DEVICE, "tag launch failed");
  if (int rc = zero_tail(mm, d_partial, S, st)) return rc;
  if (B == 0) { HIP_OK(hipMemsetAsync(d_partial, 0, (size_t)S * sizeof(double), st)); return 0; }
  if (int rc = ensure_tables(mm)) return rc;
  ReqTables* rt = nullptr;
  if (int rc = ensure_req_tables(mm, r, &rt)) return rc;
  // sequences per launch: the messages of a chunk stay within ~4 GB of HBM,
  // and the chunk is a power of two (>= 16), so every chunk's tree is a
  // subtree of the batch's tree and power-of-two shards combine into exactly
  // the whole batch's partial (nip_amd.h).  NIPAMD_ESTEP_WIDE_BYTES lowers the
  // byte budget in diagnostics builds (the multi-chunk shard-invariance test).
  const size_t per_seq = nipamd::estep_wide_scratch_bytes(P.N, 1, T);
  size_t budget = (size_t)4 << 30;
  if (const char* wb = nipamd::diag_env("NIPAMD_ESTEP_WIDE_BYTES")) budget = (size_t)std::atoll(wb);
  const size_t cap = std::min<size_t>(kEstepChunk, std::max<size_t>(16, budget / per_seq));
  long chunk = 16;
  while ((size_t)chunk * 2 <= cap) chunk *= 2;
  if (B < chunk) chunk = B;
  const long nchunks = (B + chunk - 1) / chunk;
  const long rows = (chunk + 15) / 16;
  const long lvl = (rows + 63) / 64;
  const size_t work = ((size_t)rows + 2 * lvl + nchunks + 64) * S * sizeof(double);
  if (int rc = ensure_scratch(mm, nipamd::estep_wide_scratch_bytes(P.N, chunk, T))) return rc;
  if (int rc = ensure_work(mm, work)) return rc;
  DevState* d = dev_of(mm);
  const int NP = nipamd::estep_wide_np(P.N);
  double* slab = d->W;
  double* tA = slab + (size_t)rows * S;
  double* tB = tA + (size_t)lvl * S;
  double* cres = tB + (size_t)lvl * S;
  const long ocols = n_obs > 0 ? n_obs : 1;
  for (long c = 0; c < nchunks; c++) {
    const long b0 = c * chunk;
    const long nb = (B - b0) < chunk ? (B - b0) : chunk;
    nipamd::EWideArgs a{};
    a.obs = d_obs ? d_obs + b0 * T * ocols : nullptr;
    a.obs_bstride = (long)T * ocols;
    a.obs_tstride = (int)ocols;
    a.ncol = r.ncol;
    for (int i = 0; i < r.ncol; i++) {
      a.col[i] = r.col[i];
      a.M[i] = P.emit(r.emit[i]).M;
      a.tab_off[i] = (int)rt->tabw_off[i];
    }
    a.tab = rt->tabw; a.ebase = rt->ebase; a.s = d->sall64; a.A = d->A64; a.pi = d->pi64;
    a.B = nb; a.T = T; a.N = P.N;
    a.Sa = d->S;
    a.Sb = a.Sa + (size_t)chunk * T * NP;
    a.Ea = reinterpret_cast<int*>(a.Sb + (size_t)chunk * (T + 1) * NP);
    a.ll = d_ll ? d_ll + b0 : nullptr;
    a.status = d_status ? d_status + b0 : nullptr;
    a.slab = slab; a.slab_size = S; a.R = R;
    a.proper = chain_proper(P) ? 1 : 0;
    a.nchild = (int)P.emits.size();
    for (int k = 0, row = 0; k < a.nchild; k++) {
      a.ccol[k] = -1;
      for (int i = 0; i < r.ncol; i++) if (r.emit[i] == k) a.ccol[k] = r.col[i];
      a.cM[k] = P.emits[k].M;
      a.erow[k] = row;
      row += P.emits[k].M + 2;
    }
    const int lrc = nipamd::estep_wide_launch(a, st);
    if (lrc) return launch_fail(lrc, "wide chain e_step (chain_msgs_kernel + chain_stats_kernel)");
    double* out = nchunks == 1 ? d_partial : cres + (size_t)c * S;
    if (reduce_rows(slab, (nb + 15) / 16, S, tA, tB, out, st))
      return fail(NIPAMD_ERROR_DEVICE, "reduction launch failed");
  }
  if (nchunks > 1 && reduce_rows(cres, nchunks, S, tA, tB, d_partial, st))
    return fail(NIPAMD_ERROR_DEVICE, "reduction launch failed");
  return 0;
}

static int estep_partial_routes(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                                int B, int T, double* d_partial, long capacity, double* d_ll,
                                uint32_t* d_status, void* stream) {
  Route r;
  if (!chain_estep_ok(mm, n_obs, obs_vars, T, r)) {
    Route rw;
    if (wide_estep_ok(mm, n_obs, obs_vars, rw))
      return estep_wide_partial(mm, rw, d_obs, n_obs, B, T, d_partial, d_ll, d_status, stream);
    if (mm->engine == NIPAMD_ENGINE_CHAIN)
      return fail(NIPAMD_ERROR_UNSUPPORTED, "chain e_step covers interface chains with evidence on their children");
    if (op_estep_route(mm, n_obs, obs_vars, T, capacity)) {
      // the operator chain (opchain.cpp): body zeros, the tag (-1, -1, -1)
      // that no other route's tag combines with, then its section
      const int body = estep_body_size(mm);
      hipStream_t st = (hipStream_t)stream;
      HIP_OK(hipMemsetAsync(d_partial, 0, (size_t)body * sizeof(double), st));
      if (nipamd::estep_tag_launch(d_partial + body, -1.0, -1.0, -1.0, st))
        return fail(NIPAMD_ERROR_DEVICE, "tag launch failed");
      std::string err;
      if (int rc = nipamd::op_estep_partial(mm, d_obs, n_obs, obs_vars, B, T, d_partial + body + kTagSlots, d_ll,
                                            d_status, stream, err))
        return fail(rc, err);
      return 0;
    }
    std::string why;
    if (!nipamd::jt_supported(mm, n_obs, obs_vars, 0, nullptr, why)) return fail(NIPAMD_ERROR_UNSUPPORTED, why);
    if (int rc = nipamd::jt_estep_partial(mm, d_obs, n_obs, obs_vars, B, T, d_partial, d_ll, d_status, stream))
      return rc;
    // an operator-chain request on a partial too small for its section (the
    // capacity-free nipamd_estep_partial): say so in nipamd_last_kernel
    if (capacity >= 0 && op_estep_route(mm, n_obs, obs_vars, T, -1))
      nipamd::g_last_kernel =
          "jt_filter_kernel + jt_post_kernel (general engine: an operator-chain request on a partial without room "
          "for its section)";
    if (nipamd::estep_tag_launch(d_partial + estep_body_size(mm), 0.0, 1.0, 0.0, (hipStream_t)stream))
      return fail(NIPAMD_ERROR_DEVICE, "tag launch failed");
    return zero_tail(mm, d_partial, nipamd::param_size(mm->m), (hipStream_t)stream);
  }
  const auto& P = mm->m.chain;
  const bool general = estep_general_plan(P);
  const int col = r.pcol;
  const int Mo = general ? estep_rows(P) - 2 : P.emits[0].M;   // the slab's count-table rows - 2
  const int S = nipamd::chain_estep_slab(Mo);
  const int ek = chain_estep_kernel(mm, T);
  const bool mfma = ek == 1;
  // sequences per slab row: the matrix-core kernel's and chain_estep16_kernel's
  // blocks (one row each), the round-2 DPP kernel's sequences
  const bool ck = ek == 4;
  const int per_row = (mfma || ck) ? 16 : ek == 3 ? nipamd::chain_estep16_seqs_per_row(Mo, T, general ? (int)P.emits.size() : 1) : 1;
  const long echunk = ck ? kEstepCkChunk : kEstepChunk;
  hipStream_t st = (hipStream_t)stream;
  if (nipamd::estep_tag_launch(d_partial + estep_body_size(mm), 1.0, 0.0, 0.0, st))
    return fail(NIPAMD_ERROR_DEVICE, "tag launch failed");
  if (int rc = zero_tail(mm, d_partial, S, st)) return rc;
  if (B == 0) { HIP_OK(hipMemsetAsync(d_partial, 0, (size_t)S * sizeof(double), st)); return 0; }
  if (int rc = ensure_tables(mm)) return rc;
  Route rh;
  rh.primary = 0;
  ReqTables* rt = nullptr;
  if (int rc = ensure_req_tables(mm, rh, &rt)) return rc;
  if (general)
    if (int rc = ensure_etab_all(mm)) return rc;
  const long chunk = B < echunk ? B : echunk;
  const long nchunks = (B + echunk - 1) / echunk;
  const long rows = (chunk + per_row - 1) / per_row;
  const long lvl = (rows + 63) / 64;
  const size_t work = ((size_t)rows + 2 * lvl + nchunks + 64) * S * sizeof(double);
  if (int rc = ensure_scratch(mm, ck ? nipamd::chain_estep_ck_scratch_bytes(chunk, T)
                                  : ek == 3 ? nipamd::chain_estep16_scratch_bytes(chunk, T)
                                            : nipamd::chain_scratch_bytes((int)chunk, T))) return rc;
  if (int rc = ensure_work(mm, work)) return rc;
  DevState* d = dev_of(mm);
  double* slab = d->W;
  double* tA = slab + (size_t)rows * S;
  double* tB = tA + (size_t)lvl * S;
  double* cres = tB + (size_t)lvl * S;
  const long ocols = n_obs > 0 ? n_obs : 1;
  for (long c = 0; c < nchunks; c++) {
    const long b0 = c * echunk;
    const int nb = (int)((B - b0) < echunk ? (B - b0) : echunk);
    nipamd::ChainArgs a{};
    a.obs = (general ? r.ncol > 0 : col >= 0) ? d_obs + b0 * T * ocols : nullptr;
    a.obs_bstride = (long)T * ocols;
    a.obs_tstride = ocols;
    a.obs_col = col;
    a.B = nb; a.T = T; a.H = T / 2; a.N = P.N; a.M = Mo;
    if (const char* hp = nipamd::diag_env("NIPAMD_ESTEP_H"))    // split point in % of T (A/B builds)
      if (ek == 3) a.H = std::min(T - 1, std::max(0, (int)((long)T * std::atoi(hp) / 100)));
    a.A = d->A; a.Etab = general ? d->etab_all : rt->Etab16; a.pi = d->pi; a.ts = rt->ts16; a.S = d->S;
    // chain_estep16_kernel's children: the HMM's one (the primary table), or every leaf child
    a.ne = general ? (int)P.emits.size() : 1;
    for (int k = 0, row = 0; k < a.ne; k++) {
      a.eM[k] = general ? P.emits[k].M : Mo;
      a.erow[k] = row;
      row += a.eM[k] + 2;
      a.ecol[k] = general ? -1 : col;
      if (general)
        for (int i = 0; i < r.ncol; i++) if (r.emit[i] == k) a.ecol[k] = r.col[i];
    }
    a.ll = d_ll ? d_ll + b0 : nullptr;
    a.status = d_status ? d_status + b0 : nullptr;
    a.counts = slab;
    a.proper = ck ? (chain_proper(P) ? 1 : 0)
                  : ek == 3 && chain_proper(P) ? (estep16_sparse_ok(P, a.ne) ? 2 : 1) : 0;
#ifdef NIPAMD_DIAGNOSTICS
    static const bool times = std::getenv("NIPAMD_PHASE_TIMES") != nullptr;
    const int nblk = (nb + 15) / 16;
    if (mfma && times && c == 0) {
      HIP_OK(hipMalloc(&a.diag, (size_t)nblk * 24 * sizeof(unsigned long long)));
      HIP_OK(hipMemsetAsync(a.diag, 0, (size_t)nblk * 24 * sizeof(unsigned long long), st));
    }
    unsigned long long* ckd = nullptr;               // chain_estep_ck_kernel's per-group stamps [group][5]
    const long ngrp = (nb + 15) / 16;
    if (ck && times && c == 0) {
      HIP_OK(hipMalloc(&ckd, (size_t)ngrp * 5 * sizeof(unsigned long long)));
      HIP_OK(hipMemsetAsync(ckd, 0, (size_t)ngrp * 5 * sizeof(unsigned long long), st));
      a.diag = ckd;
    }
    unsigned long long* e16d = nullptr;              // chain_estep16_kernel's per-wave stamps [block][16][4]
    const int nblk8 = (nb + 7) / 8;                  // blocks of 8 or 16 sequences: room for either
    if (ek == 3 && times && c == 0) {
      HIP_OK(hipMalloc(&e16d, (size_t)nblk8 * 64 * sizeof(unsigned long long)));
      HIP_OK(hipMemsetAsync(e16d, 0, (size_t)nblk8 * 64 * sizeof(unsigned long long), st));
      a.diag = e16d;
    }
#endif
    const int lrc = ck ? nipamd::chain_estep_ck_launch(a, st)
                    : mfma ? nipamd::chain_estep_mfma_launch(a, st)
                    : ek == 3 ? nipamd::chain_estep16_launch(a, st) : nipamd::chain_estep_launch(a, st);
    if (lrc)
      return launch_fail(lrc, ck ? "chain_estep_ck_kernel" : mfma ? "chain_fb_mfma_kernel (e_step)"
                              : ek == 3 ? "chain_estep16_kernel" : "chain_kernel<true>");
#ifdef NIPAMD_DIAGNOSTICS
    if (ckd) {
      std::vector<unsigned long long> h((size_t)ngrp * 5);
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(h.data(), ckd, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      (void)hipFree(ckd);
      a.diag = nullptr;
      unsigned long long t0 = ~0ull, t1 = 0;
      double fw = 0, bw = 0, wall = 0;
      for (long k = 0; k < ngrp; k++) {
        const unsigned long long* r = h.data() + k * 5;
        t0 = std::min(t0, r[0]);
        t1 = std::max(t1, r[1]);
        fw += (double)r[2];
        bw += (double)r[3];
        wall += (double)(r[1] - r[0]);
      }
      std::fprintf(stderr, "[nipamd] estep_ck groups %ld, launch span %.1f us; per group: forward %.0f cycles, "
                   "backward %.0f cycles, wall %.1f us\n", ngrp, (t1 - t0) / 100.0, fw / ngrp, bw / ngrp,
                   wall / ngrp / 100.0);
    }
    if (e16d) {
      std::vector<unsigned long long> h((size_t)nblk8 * 64);
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(h.data(), e16d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      (void)hipFree(e16d);
      a.diag = nullptr;
      double m[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
      int nw[2] = {0, 0};
      for (int k = 0; k < nblk8; k++)
        for (int w = 0; w < 16; w++) {
          const unsigned long long* r = h.data() + ((size_t)k * 16 + w) * 4;
          if (r[0] + r[2] == 0) continue;
          const int dd = w < 8 ? 0 : 1;
          for (int i = 0; i < 4; i++) m[dd][i] += (double)r[i];
          nw[dd]++;
        }
      for (int dd = 0; dd < 2; dd++)
        if (nw[dd])
          std::fprintf(stderr, "[nipamd] estep16 %s waves: phase A %.0f  barrier wait %.0f  phase B %.0f  "
                       "block entry to exit %.0f cycles (mean of %d)\n", dd ? "backward" : "forward",
                       m[dd][0] / nw[dd], m[dd][1] / nw[dd], m[dd][2] / nw[dd], m[dd][3] / nw[dd], nw[dd]);
    }
    if (a.diag) {
      std::vector<unsigned long long> h((size_t)nblk * 24);
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(h.data(), a.diag, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      (void)hipFree(a.diag);
      unsigned long long t0 = ~0ull, tend = 0;
      double d[7] = {0, 0, 0, 0, 0, 0, 0};
      for (int k = 0; k < nblk; k++) {
        const unsigned long long* r = h.data() + (size_t)k * 24;
        t0 = std::min(t0, r[0]);
        for (int i = 1; i < 7; i++) { d[i] += (double)(r[i] - r[0]); tend = std::max(tend, r[i]); }
      }
      std::fprintf(stderr, "[nipamd] e_step blocks %d, launch span %.1f us; mean us from block entry: staged %.1f  "
                   "phase A end %.1f  fwd filter end %.1f  bwd filter end %.1f  fwd partner end %.1f  "
                   "bwd partner end %.1f\n", nblk, (tend - t0) / 100.0, d[1] / nblk / 100.0, d[2] / nblk / 100.0,
                   d[3] / nblk / 100.0, d[4] / nblk / 100.0, d[5] / nblk / 100.0, d[6] / nblk / 100.0);
      double pcs[10] = {0};
      for (int k = 0; k < nblk; k++)
        for (int i = 0; i < 10; i++) pcs[i] += (double)h[(size_t)k * 24 + 8 + i];
      std::fprintf(stderr, "[nipamd] e_step partner phase-B cycles (wait / in-lane / xi / q / counts): "
                   "fwd %.0f %.0f %.0f %.0f %.0f  bwd %.0f %.0f %.0f %.0f %.0f\n", pcs[0] / nblk, pcs[1] / nblk,
                   pcs[2] / nblk, pcs[3] / nblk, pcs[4] / nblk, pcs[5] / nblk, pcs[6] / nblk, pcs[7] / nblk,
                   pcs[8] / nblk, pcs[9] / nblk);
    }
#endif
    double* out = nchunks == 1 ? d_partial : cres + (size_t)c * S;
    if (reduce_rows(slab, (nb + per_row - 1) / per_row, S, tA, tB, out, st))
      return fail(NIPAMD_ERROR_DEVICE, "reduction launch failed");
  }
  if (nchunks > 1 && reduce_rows(cres, nchunks, S, tA, tB, d_partial, st))
    return fail(NIPAMD_ERROR_DEVICE, "reduction launch failed");
  return 0;
}

// A joint interface's e_step counts (the HMM e_step kernel's slab over the
// joint states: xi sums Kf / Kb without the A factor, M1 tables of the
// observation, the t = 0 posterior P0) projected onto every family of the
// em_learn layout (child first, then its parents, nip.c:2101-2128): the
// family's value at a joint (x, y) is its variables' digits, previous-slice
// variables from x and interface variables from y.  Built on the host once
// per model version; each count is one fixed-order sum (CSR row).
static int ensure_joint_map(nipamd_model* mm) {
  DevState* d = dev_of(mm);
  if (d->jm_ptr) return 0;
  const nipamd::Model& m = mm->m;
  const auto& P = m.chain;
  const int nv = (int)m.vars.size(), K = P.N, M = P.emits[0].M, ov = P.emits[0].var;
  const int Kb = nipamd::kSlabKb, Hf = nipamd::kSlabH, Hb = nipamd::kSlabH + (M + 2) * 16;
  const int p0 = nipamd::chain_slab_p0(M);
  std::vector<int> off(nv + 1, 0);
  for (int v = 0; v < nv; v++) {
    int sz = m.vars[v].card;
    for (int q : m.vars[v].parents) sz *= m.vars[q].card;
    off[v + 1] = off[v] + sz;
  }
  // value of variable w at joint (x, y): -1 if it is neither interface's
  auto value = [&](int w, int x, int y) {
    long sx = 1;
    for (size_t i = 0; i < P.jprev.size(); i++) {
      const int c = m.vars[P.jprev[i]].card;
      if (P.jprev[i] == w) return (int)((x / sx) % c);
      if (P.jcur[i] == w) return (int)((y / sx) % c);
      sx *= c;
    }
    return -1;
  };
  std::vector<std::vector<std::pair<int, double>>> rows(off[nv]);
  for (int v = 0; v < nv; v++) {
    const auto& V = m.vars[v];
    std::vector<int> U{v};
    U.insert(U.end(), V.parents.begin(), V.parents.end());
    auto family_index = [&](int x, int y, int first) {     // first: v's own value (child first)
      long idx = first, st = V.card;
      for (size_t k = 1; k < U.size(); k++) {
        const int u = value(U[k], x, y);
        if (u < 0) return -1L;
        idx += u * st;
        st *= m.vars[U[k]].card;
      }
      return idx;
    };
    const bool is_prev = std::find(P.jprev.begin(), P.jprev.end(), v) != P.jprev.end();
    const bool is_cur = std::find(P.jcur.begin(), P.jcur.end(), v) != P.jcur.end();
    if (is_prev) {
      if (U.size() != 1) return fail(NIPAMD_ERROR_UNSUPPORTED, "joint e_step: previous-slice variable with parents");
      for (int x = 0; x < K; x++) rows[off[v] + value(v, x, 0)].push_back({p0 + x, 1.0});
    } else if (is_cur) {
      for (int x = 0; x < K; x++)
        for (int y = 0; y < K; y++) {
          const long i = family_index(x, y, value(v, x, y));
          if (i < 0) return fail(NIPAMD_ERROR_UNSUPPORTED, "joint e_step: family outside the interfaces");
          const double a = P.A[x * 16 + y];
          rows[off[v] + i].push_back({x * 16 + y, a});
          rows[off[v] + i].push_back({Kb + x * 16 + y, a});
        }
    } else if (v == ov) {
      const auto& E = P.emits[0];
      for (int y = 0; y < K; y++)
        for (int o = 0; o < M; o++) {
          const long i = family_index(0, y, o);
          if (i < 0) return fail(NIPAMD_ERROR_UNSUPPORTED, "joint e_step: observation family outside the interface");
          rows[off[v] + i].push_back({Hf + o * 16 + y, 1.0});
          rows[off[v] + i].push_back({Hb + o * 16 + y, 1.0});
          if (E.s[y] != 0.0) {                   // missing observations, split as E(y, o) / s(y)
            const double w = E.E[(size_t)o * 64 + y] / E.s[y];
            rows[off[v] + i].push_back({Hf + M * 16 + y, w});
            rows[off[v] + i].push_back({Hb + M * 16 + y, w});
          }
        }
    } else {
      return fail(NIPAMD_ERROR_UNSUPPORTED, "joint e_step: variable outside the joint chain");
    }
  }
  std::vector<int> ptr{0}, idx;
  std::vector<double> coef;
  for (const auto& r : rows) {
    for (const auto& e : r) { idx.push_back(e.first); coef.push_back(e.second); }
    ptr.push_back((int)idx.size());
  }
  HIP_OK(hipMalloc(&d->jm_ptr, ptr.size() * sizeof(int)));
  HIP_OK(hipMemcpy(d->jm_ptr, ptr.data(), ptr.size() * sizeof(int), hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&d->jm_idx, std::max<size_t>(1, idx.size()) * sizeof(int)));
  if (!idx.empty()) HIP_OK(hipMemcpy(d->jm_idx, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice));
  if (int rc = upload(d, &d->jm_coef, coef)) return rc;
  d->jm_n = off[nv];
  return 0;
}

// Every leaf child's evidence table for the general chain e_step: rows
// M_k + 2 per child (E_k[m][y], the row sums, an all-zero row for an
// out-of-range state), 16 columns, children in plan order.
static int ensure_etab_all(nipamd_model* mm) {
  DevState* d = dev_of(mm);
  if (d->etab_all) return 0;
  const auto& P = mm->m.chain;
  std::vector<double> E;
  for (const auto& em : P.emits) {
    const size_t base = E.size();
    E.resize(base + (size_t)(em.M + 2) * 16, 0.0);
    for (int y = 0; y < P.N; y++) {
      for (int m = 0; m < em.M; m++) E[base + (size_t)m * 16 + y] = em.E[(size_t)m * 64 + y];
      E[base + (size_t)em.M * 16 + y] = em.s[y];
    }
  }
  return upload(d, &d->etab_all, E);
}

// The general chain e_step's slab (xi sums without the transition, the
// children's count tables, the t = 0 posterior P0) projected onto every
// family of the em_learn layout (nip.c:2101-2128: child first, then its
// parents in v->parents order), as one fixed-order sum per count (CSR):
//   previous interface variable: P0
//   interface variable y | x, hidden parents h: in-clique(x, y, h)
//       x prod_j prior_j(h_j) x K(x, y)   (the joint posterior of the
//       in-clique's variables is alpha_{t-1}(x) P(y | x, h) prod prior(h)
//       e_t(y) beta_t(y) / Z; the xi sums K hold everything but the first factors)
//   hidden parent h_j: the same summed over everything but h_j
//   leaf child o_k | y: its count table, a missing observation split as
//       E_k(y, o) / s_k(y) (the child's posterior given y)
// Two slab layouts: the 16-state kernels' (Kf and Kb, two count tables, row
// stride 16) and estep_wide.hip's (one K, one table, row stride NP).  Built
// as (row, slab index, coefficient) triples in a fixed generation order, then
// grouped by row with a stable counting sort: the in-clique of config 5 has
// 16.7M entries, one CSR row each.
// the cached slab -> em_learn map serves one slab layout: drop it when a
// partial of another layout comes to be finalized
static int ensure_map_kind(nipamd_model* mm, int kind) {
  DevState* d = dev_of(mm);
  if (d->jm_ptr && d->jm_kind != kind) {
    HIP_OK(hipDeviceSynchronize());
    dfree(d, d->jm_ptr); dfree(d, d->jm_idx); dfree(d, d->jm_coef);
    d->jm_ptr = nullptr; d->jm_idx = nullptr; d->jm_coef = nullptr; d->jm_n = 0;
  }
  d->jm_kind = kind;
  return 0;
}

struct SlabLayout {
  int ns;          // row stride of K and H
  int kf, kb;      // K sums (kb < 0: one sum)
  int hf, hb;      // count tables (hb < 0: one table)
  int p0;
};

// the projection's structural preconditions (ensure_chain_map's checks)
static bool chain_map_supported(const nipamd::Model& m) {
  const auto& P = m.chain;
  if (!P.valid || P.joint || P.c_trans < 0) return false;
  for (int v : m.cliques[P.c_trans].vars)
    if (v != P.v_prev && v != P.v_cur && std::find(P.hidden.begin(), P.hidden.end(), v) == P.hidden.end())
      return false;
  if (!m.vars[P.v_prev].parents.empty()) return false;
  for (const auto& E : P.emits) {
    const auto& Vo = m.vars[E.var];
    if (Vo.parents.size() != 1 || Vo.parents[0] != P.v_cur) return false;
  }
  for (int v = 0; v < (int)m.vars.size(); v++) {
    const bool known = v == P.v_prev || v == P.v_cur ||
                       std::find(P.hidden.begin(), P.hidden.end(), v) != P.hidden.end() ||
                       std::any_of(P.emits.begin(), P.emits.end(), [&](const nipamd::ChainEmit& e) { return e.var == v; });
    if (!known) return false;
  }
  return true;
}

static int ensure_chain_map(nipamd_model* mm, const SlabLayout& L) {
  DevState* d = dev_of(mm);
  if (d->jm_ptr) return 0;
  const nipamd::Model& m = mm->m;
  if (!chain_map_supported(m)) return fail(NIPAMD_ERROR_UNSUPPORTED, "chain e_step: slice outside the chain plan");
  const auto& P = m.chain;
  const int nv = (int)m.vars.size(), N = P.N;
  std::vector<long> off(nv + 1, 0);
  for (int v = 0; v < nv; v++) {
    long sz = m.vars[v].card;
    for (int q : m.vars[v].parents) sz *= m.vars[q].card;
    off[v + 1] = off[v] + sz;
  }
  struct Ent { long row; int idx; double coef; };
  std::vector<Ent> ents;
  auto kidx = [&](int base, int x, int y) { return base + x * L.ns + y; };
  // the in-clique's entries: (x, y, hidden values) -> coefficient
  const auto& cin = m.cliques[P.c_trans];
  const size_t nc = cin.vars.size();
  long total = 1;
  for (size_t i = 0; i < nc; i++) total *= m.vars[cin.vars[i]].card;
  ents.reserve((size_t)total * (L.kb >= 0 ? 2 : 1) + 4096);
  const int nh = (int)P.hidden.size();
  // hidden parent j, value d: sum over the in-clique entries of each (x, y),
  // in entry order, and the order in which the (x, y) first occur
  std::vector<std::vector<double>> hacc(nh);
  std::vector<std::vector<char>> hseen(nh);
  std::vector<std::vector<std::vector<int>>> horder(nh);
  for (int j = 0; j < nh; j++) {
    const int c = m.vars[P.hidden[j]].card;
    hacc[j].assign((size_t)c * N * N, 0.0);
    hseen[j].assign((size_t)c * N * N, 0);
    horder[j].resize(c);
  }
  std::vector<int> val(nv, 0);
  const auto& Vc = m.vars[P.v_cur];
  std::vector<int> cardc(nc);
  for (size_t k = 0; k < nc; k++) cardc[k] = m.vars[cin.vars[k]].card;
  std::vector<int> digit(nc, 0);
  for (long i = 0; i < total; i++) {
    for (size_t k = 0; k < nc; k++) val[cin.vars[k]] = digit[k];
    double coef = cin.original[(size_t)i];
    for (int h : P.hidden) coef *= m.vars[h].prior[val[h]];
    const int x = val[P.v_prev], y = val[P.v_cur];
    // the interface variable's family: y first, then its parents in order
    long idx = y, st = Vc.card;
    for (int q : Vc.parents) { idx += (long)val[q] * st; st *= m.vars[q].card; }
    ents.push_back({off[P.v_cur] + idx, kidx(L.kf, x, y), coef});
    if (L.kb >= 0) ents.push_back({off[P.v_cur] + idx, kidx(L.kb, x, y), coef});
    for (int j = 0; j < nh; j++) {
      const int dv = val[P.hidden[j]];
      const size_t c = ((size_t)dv * N + x) * N + y;
      if (!hseen[j][c]) { hseen[j][c] = 1; horder[j][dv].push_back(x * N + y); }
      hacc[j][c] += coef;
    }
    for (size_t k = 0; k < nc; k++) {                     // odometer, dimension 0 fastest
      if (++digit[k] < cardc[k]) break;
      digit[k] = 0;
    }
  }
  for (int j = 0; j < nh; j++) {
    const int h = P.hidden[j];
    for (int dv = 0; dv < m.vars[h].card; dv++) {
      for (int xy : horder[j][dv])
        ents.push_back({off[h] + dv, kidx(L.kf, xy / N, xy % N), hacc[j][((size_t)dv * N) * N + xy]});
      if (L.kb >= 0)
        for (int xy : horder[j][dv])
          ents.push_back({off[h] + dv, kidx(L.kb, xy / N, xy % N), hacc[j][((size_t)dv * N) * N + xy]});
    }
  }
  for (int x = 0; x < N; x++) ents.push_back({off[P.v_prev] + x, L.p0 + x, 1.0});
  for (size_t k = 0, row0 = 0; k < P.emits.size(); k++) {
    const auto& E = P.emits[k];
    for (int y = 0; y < N; y++)
      for (int o = 0; o < E.M; o++) {
        const long r = off[E.var] + o + (long)E.M * y;
        ents.push_back({r, L.hf + (int)(row0 + o) * L.ns + y, 1.0});
        if (L.hb >= 0) ents.push_back({r, L.hb + (int)(row0 + o) * L.ns + y, 1.0});
        if (E.s[y] != 0.0) {                   // missing observations, split as E(y, o) / s(y)
          const double w = E.E[(size_t)o * 64 + y] / E.s[y];
          ents.push_back({r, L.hf + (int)(row0 + E.M) * L.ns + y, w});
          if (L.hb >= 0) ents.push_back({r, L.hb + (int)(row0 + E.M) * L.ns + y, w});
        }
      }
    row0 += E.M + 2;
  }
  // CSR by a stable counting sort on the row
  const long nrows = off[nv];
  if ((long)ents.size() >= (1L << 31) || nrows >= (1L << 31))
    return fail(NIPAMD_ERROR_UNSUPPORTED, "chain e_step: projection beyond 2^31 entries");
  std::vector<int> ptr((size_t)nrows + 1, 0);
  for (const Ent& e : ents) ptr[(size_t)e.row + 1]++;
  for (long r = 0; r < nrows; r++) ptr[(size_t)r + 1] += ptr[(size_t)r];
  std::vector<int> fill(ptr.begin(), ptr.end() - 1), idx(ents.size());
  std::vector<double> coef(ents.size());
  for (const Ent& e : ents) {
    const int q = fill[(size_t)e.row]++;
    idx[(size_t)q] = e.idx;
    coef[(size_t)q] = e.coef;
  }
  HIP_OK(hipMalloc(&d->jm_ptr, ptr.size() * sizeof(int)));
  HIP_OK(hipMemcpy(d->jm_ptr, ptr.data(), ptr.size() * sizeof(int), hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&d->jm_idx, std::max<size_t>(1, idx.size()) * sizeof(int)));
  if (!idx.empty()) HIP_OK(hipMemcpy(d->jm_idx, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice));
  if (int rc = upload(d, &d->jm_coef, coef)) return rc;
  d->jm_n = (int)nrows;
  return 0;
}

int nipamd_estep_finalize(nipamd_model* mm, const double* d_partial, double* d_counts, void* stream) {
  if (!mm || !d_partial || !d_counts) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const int body = estep_body_size(mm);
  // the route tag (see nipamd_estep_partial_size): one 24-byte read, once per EM iteration
  double tag[kTagSlots] = {0.0, 0.0, 0.0};
  HIP_OK(hipMemcpyAsync(tag, d_partial + body, sizeof(tag), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  int route = -1, nz = 0;
  for (int k = 0; k < kTagSlots; k++)
    if (tag[k] != 0.0) { nz++; if (tag[k] >= 1.0) route = k; }
  if (tag[0] <= -1.0 && tag[1] == tag[0] && tag[2] == tag[0]) {
    // the operator chain's partial (its header names the request)
    std::string err;
    if (int rc = nipamd::op_estep_finalize(mm, d_partial + body + kTagSlots, d_counts, stream, err))
      return fail(rc, err);
    return 0;
  }
  if (nz != 1 || route < 0)
    return fail(NIP_ERROR_INVALID_ARGUMENT, "e_step partial: partials of different routes (chain slab / em_learn "
                                            "layout / wide chain slab) were combined, or the buffer is not an "
                                            "e_step partial");
  if (route == 1) return nipamd::jt_estep_finalize(mm, d_partial, d_counts, stream);
  const auto& P = mm->m.chain;
  if (!has_chain_estep(mm->m)) return fail(NIPAMD_ERROR_UNSUPPORTED, "no chain e_step plan for this model");
  if (int rc = ensure_tables(mm)) return rc;
  DevState* d = dev_of(mm);
  if (route == 2) {
    if (!estep_wide_plan(mm->m)) return fail(NIPAMD_ERROR_UNSUPPORTED, "no wide chain e_step plan for this model");
    const int NP = nipamd::estep_wide_np(P.N), R = estep_rows(P);
    const SlabLayout L{NP, 0, -1, NP * NP, -1, NP * NP + R * NP};
    if (int rc = ensure_map_kind(mm, 3)) return rc;
    if (int rc = ensure_chain_map(mm, L)) return rc;
    if (nipamd::estep_map_finalize_launch(d_partial, d->jm_n, d->jm_ptr, d->jm_idx, d->jm_coef, d_counts,
                                          (hipStream_t)stream))
      return fail(NIPAMD_ERROR_DEVICE, "finalize launch failed");
    return 0;
  }
  Route rh;
  rh.primary = 0;
  ReqTables* rt = nullptr;
  if (int rc = ensure_req_tables(mm, rh, &rt)) return rc;
  if (P.jhmm || !P.hmm) {
    const int R = estep_rows(P);
    const SlabLayout L{16, nipamd::kSlabKf, nipamd::kSlabKb, nipamd::kSlabH, nipamd::kSlabH + R * 16,
                       nipamd::chain_slab_p0(R - 2)};
    if (int rc = ensure_map_kind(mm, P.jhmm ? 1 : 2)) return rc;
    if (int rc = P.jhmm ? ensure_joint_map(mm) : ensure_chain_map(mm, L)) return rc;
    if (nipamd::estep_map_finalize_launch(d_partial, d->jm_n, d->jm_ptr, d->jm_idx, d->jm_coef, d_counts,
                                          (hipStream_t)stream))
      return fail(NIPAMD_ERROR_DEVICE, "finalize launch failed");
    return 0;
  }
  nipamd::ChainFinalize f{};
  f.N = P.N; f.M = P.emits[0].M;
  int off = 0;
  for (size_t v = 0; v < mm->m.vars.size(); v++) {
    if ((int)v == P.v_prev) f.off_prev = off;
    if ((int)v == P.v_cur) f.off_cur = off;
    if ((int)v == P.emits[0].var) f.off_obs = off;
    int s = mm->m.vars[v].card;
    for (int p : mm->m.vars[v].parents) s *= mm->m.vars[p].card;
    off += s;
  }
  f.A = d->A; f.Etab = rt->Etab16;
  if (nipamd::estep_finalize_launch(d_partial, f, d_counts, (hipStream_t)stream))
    return fail(NIPAMD_ERROR_DEVICE, "finalize launch failed");
  return 0;
}

int nipamd_estep(nipamd_model* mm, const int32_t* d_obs, int n_obs, const int* obs_vars,
                 int B, int T, double* d_counts, double* d_ll, uint32_t* d_status, void* stream) {
  if (!mm || !d_counts || T < 1) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const int S = nipamd_estep_partial_size_req(mm, n_obs, obs_vars, T);
  if (S < 0) return fail(NIPAMD_ERROR_UNSUPPORTED, "no e_step plan for this model under the selected engine");
  if (int rc = ensure_device(mm)) return rc;
  DevState* d = dev_of(mm);
  if (d->R_size < S) {
    (void)hipFree(d->R);
    d->R = nullptr;
    d->R_size = 0;
    HIP_OK(hipMalloc(&d->R, (size_t)S * sizeof(double)));
    d->R_size = S;
  }
  double* part = d->R;
  int rc = nipamd_estep_partial_ex(mm, d_obs, n_obs, obs_vars, B, T, part, S, d_ll, d_status, stream);
  if (rc) return rc;
  return nipamd_estep_finalize(mm, part, d_counts, stream);
}

int nipamd_estep_host(nipamd_model* mm, const int32_t* obs, int n_obs, const int* obs_vars,
                      int B, int T, double* counts, double* ll, uint32_t* status) {
  if (!mm || B < 0 || T < 1 || !counts) return fail(NIP_ERROR_INVALID_ARGUMENT, "bad arguments");
  const int P = nipamd::param_size(mm->m);
  int32_t* d_obs = nullptr; double* d_cnt = nullptr; double* d_ll = nullptr; uint32_t* d_st = nullptr;
  const size_t nob = (size_t)B * T * (n_obs > 0 ? n_obs : 1);
  HIP_OK(hipMalloc(&d_obs, nob * sizeof(int32_t)));
  HIP_OK(hipMalloc(&d_cnt, (size_t)P * sizeof(double)));
  HIP_OK(hipMalloc(&d_ll, (size_t)(B > 0 ? B : 1) * sizeof(double)));
  HIP_OK(hipMalloc(&d_st, (size_t)(B > 0 ? B : 1) * sizeof(uint32_t)));
  if (n_obs > 0 && B > 0) HIP_OK(hipMemcpy(d_obs, obs, nob * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_cnt, counts, (size_t)P * sizeof(double), hipMemcpyHostToDevice));
  int rc = nipamd_estep(mm, d_obs, n_obs, obs_vars, B, T, d_cnt, d_ll, d_st, nullptr);
  if (rc == 0) {
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(counts, d_cnt, (size_t)P * sizeof(double), hipMemcpyDeviceToHost));
    if (ll && B > 0) HIP_OK(hipMemcpy(ll, d_ll, (size_t)B * sizeof(double), hipMemcpyDeviceToHost));
    if (status && B > 0) HIP_OK(hipMemcpy(status, d_st, (size_t)B * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  (void)hipFree(d_obs); (void)hipFree(d_cnt); (void)hipFree(d_ll); (void)hipFree(d_st);
  return rc;
}

}  // extern "C"
