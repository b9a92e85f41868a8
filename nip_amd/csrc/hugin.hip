// hugin.hip -- Hugin message passes over explicit potential tables on gfx950
// (nipamd_hugin_passes, include/nip_amd.h): the propagation behind the
// single-slice API of libnip.so (nip_collect_evidence /
// nip_distribute_evidence / make_consistent, src/nipjointree.c:580-709,
// src/nip.c:1600-1617).
//
// One pass (nip_message_pass, nipjointree.c:676-709) is
//   marginalise  s_new[j] = sum of src over the pre-image of j
//                (nip_general_marginalise, src/nippotential.c:267-311)
//   absorb       dst[i] = dst[i] * s_new[j(i)]; then / s_old[j(i)], or 0
//                where s_old is 0 (nip_update_potential, :436-496)
// and the passes of a traversal run in order.  Both halves keep the
// reference's arithmetic exactly: one lane owns a sepset entry and adds its
// pre-image in ascending source order starting from 0.0 (the reference's
// "dest[choose(i)] += src[i] for i ascending" restricted to that entry), and
// the absorption is the same multiply-then-divide per entry.  Results are
// therefore bit-identical to the reference.
//
// Small trees (every table <= kSmall entries) run as ONE launch of one
// 1024-lane block that walks all passes with a barrier between the halves.
// Larger tables launch each half of each pass as its own grid (marginalise:
// one lane per sepset entry; absorb: one lane per clique entry).
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "model.h"
#include "nip_amd.h"

namespace nipamd {
namespace {

constexpr int kMaxDim = 24;            // dimensions per table
constexpr int kSmall = 1 << 16;        // entries: single-block path
constexpr int kBlock = 1024;

struct HPass {
  long long src, snew, sold, dst;      // table offsets (doubles) in the packed buffer
  int D;                               // sepset entries
  int nsd;                             // sepset dimensions
  int scard[kMaxDim];                  // sepset cardinalities
  long long sstride[kMaxDim];          // source stride of the source dimension of sepset dim k
  int nfree;                           // source dimensions not in the sepset, ascending
  int fcard[kMaxDim];
  long long fstride[kMaxDim];
  int N;                               // destination clique entries
  int ndd;
  int dcard[kMaxDim];
  int dproj[kMaxDim];                  // sepset stride of destination dim a (0: not in the sepset)
};

// s_new[j] for one sepset entry j
__device__ __forceinline__ void marg_entry(const HPass& P, double* buf, int j) {
  long long base = P.src;
  int r = j;
  for (int k = 0; k < P.nsd; k++) {
    const int d = r % P.scard[k];
    r /= P.scard[k];
    base += (long long)d * P.sstride[k];
  }
  int idx[kMaxDim];
  for (int a = 0; a < P.nfree; a++) idx[a] = 0;
  const double* src = buf;
  double s = 0.0;
  long long off = base;
  for (;;) {
    s += src[off];
    int a = 0;
    for (; a < P.nfree; a++) {       // odometer over the free dimensions, lowest fastest
      off += P.fstride[a];
      if (++idx[a] < P.fcard[a]) break;
      off -= P.fstride[a] * idx[a];
      idx[a] = 0;
    }
    if (a == P.nfree) break;
  }
  buf[P.snew + j] = s;
}

// dst[i] *= s_new / s_old (0 where s_old is 0)
__device__ __forceinline__ void absorb_entry(const HPass& P, double* buf, int i) {
  int r = i, j = 0;
  for (int a = 0; a < P.ndd; a++) {
    const int d = r % P.dcard[a];
    r /= P.dcard[a];
    j += d * P.dproj[a];
  }
  double x = buf[P.dst + i] * buf[P.snew + j];
  const double old = buf[P.sold + j];
  buf[P.dst + i] = old != 0.0 ? x / old : 0.0;
}

__global__ __launch_bounds__(kBlock) void hugin_block_kernel(const HPass* __restrict__ passes, int np,
                                                            double* buf) {
  for (int p = 0; p < np; p++) {
    const HPass& P = passes[p];
    for (int j = threadIdx.x; j < P.D; j += kBlock) marg_entry(P, buf, j);
    __syncthreads();
    for (int i = threadIdx.x; i < P.N; i += kBlock) absorb_entry(P, buf, i);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void hugin_marg_kernel(const HPass* __restrict__ passes, int p,
                                                         double* buf) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < passes[p].D) marg_entry(passes[p], buf, j);
}

__global__ __launch_bounds__(256) void hugin_absorb_kernel(const HPass* __restrict__ passes, int p,
                                                           double* buf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < passes[p].N) absorb_entry(passes[p], buf, i);
}

// per-device scratch, grown on demand (the API is single-threaded, like the
// reference's: SURVEY 8(b) threading)
struct Scratch {
  double* buf = nullptr;
  size_t buf_n = 0;
  HPass* passes = nullptr;
  size_t passes_n = 0;
};
std::map<int, Scratch> g_scratch;

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return set_error(NIPAMD_ERROR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

}  // namespace
}  // namespace nipamd

using namespace nipamd;

extern "C" int nipamd_hugin_passes(int n_tables, double* const* tables, const int* ndim,
                                   const int* card, int n_passes, const int* passes,
                                   const int* maps) {
  if (n_tables < 0 || n_passes < 0 || (n_tables > 0 && (!tables || !ndim || !card)) ||
      (n_passes > 0 && (!passes || !maps)))
    return set_error(NIP_ERROR_INVALID_ARGUMENT, "nipamd_hugin_passes: null argument");
  if (n_passes == 0) return NIP_NO_ERROR;
  // table geometry
  std::vector<long long> off(n_tables + 1, 0);
  std::vector<int> coff(n_tables + 1, 0);
  std::vector<long long> size(n_tables);
  for (int k = 0; k < n_tables; k++) {
    if (ndim[k] < 0 || ndim[k] > kMaxDim || !tables[k])
      return set_error(NIP_ERROR_INVALID_ARGUMENT, "nipamd_hugin_passes: bad table " + std::to_string(k));
    long long s = 1;
    for (int a = 0; a < ndim[k]; a++) {
      if (card[coff[k] + a] < 1) return set_error(NIP_ERROR_INVALID_ARGUMENT, "nipamd_hugin_passes: bad cardinality");
      s *= card[coff[k] + a];
    }
    if (s > (1LL << 31) - 1) return set_error(NIPAMD_ERROR_UNSUPPORTED, "nipamd_hugin_passes: table too large");
    size[k] = s;
    off[k + 1] = off[k] + s;
    coff[k + 1] = coff[k] + ndim[k];
  }
  auto dims = [&](int k, int a) { return card[coff[k] + a]; };
  // pass descriptors
  std::vector<HPass> H(n_passes);
  long long largest = 0;
  for (int p = 0; p < n_passes; p++) {
    const int* q = passes + 6 * p;
    const int src = q[0], sn = q[1], so = q[2], dst = q[3];
    for (int t : {src, sn, so, dst})
      if (t < 0 || t >= n_tables) return set_error(NIP_ERROR_INVALID_ARGUMENT, "nipamd_hugin_passes: table index");
    if (ndim[sn] != ndim[so] || size[sn] != size[so])
      return set_error(NIP_ERROR_INVALID_ARGUMENT, "nipamd_hugin_passes: old/new sepset geometry differs");
    const int* m_src = maps + q[4];
    const int* m_dst = maps + q[5];
    HPass& P = H[p];
    std::memset(&P, 0, sizeof P);
    P.src = off[src]; P.snew = off[sn]; P.sold = off[so]; P.dst = off[dst];
    P.D = (int)size[sn];
    P.nsd = ndim[sn];
    P.N = (int)size[dst];
    P.ndd = ndim[dst];
    std::vector<long long> sstride(ndim[src]);
    long long s = 1;
    for (int a = 0; a < ndim[src]; a++) { sstride[a] = s; s *= dims(src, a); }
    std::vector<bool> used(ndim[src], false);
    long long sep_stride = 1;
    for (int k = 0; k < P.nsd; k++) {
      const int a = m_src[k], b = m_dst[k];
      if (a < 0 || a >= ndim[src] || b < 0 || b >= ndim[dst] || dims(src, a) != dims(sn, k) ||
          dims(dst, b) != dims(sn, k) || used[a])
        return set_error(NIP_ERROR_INVALID_ARGUMENT, "nipamd_hugin_passes: mapping does not match the sepset");
      used[a] = true;
      P.scard[k] = dims(sn, k);
      P.sstride[k] = sstride[a];
      P.dproj[b] = (int)sep_stride;
      sep_stride *= dims(sn, k);
    }
    for (int a = 0; a < ndim[src]; a++)
      if (!used[a]) {
        P.fcard[P.nfree] = dims(src, a);
        P.fstride[P.nfree] = sstride[a];
        P.nfree++;
      }
    for (int b = 0; b < P.ndd; b++) P.dcard[b] = dims(dst, b);
    largest = std::max(largest, std::max(size[src], size[dst]));
  }
  // pack, run, unpack
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  Scratch& S = g_scratch[dev];
  const size_t total = (size_t)off[n_tables];
  if (S.buf_n < total) {
    (void)hipFree(S.buf);
    S.buf = nullptr;
    S.buf_n = 0;
    HIP_TRY(hipMalloc(&S.buf, total * sizeof(double)));
    S.buf_n = total;
  }
  if (S.passes_n < H.size()) {
    (void)hipFree(S.passes);
    S.passes = nullptr;
    S.passes_n = 0;
    HIP_TRY(hipMalloc(&S.passes, H.size() * sizeof(HPass)));
    S.passes_n = H.size();
  }
  std::vector<double> stage(total);
  for (int k = 0; k < n_tables; k++)
    std::memcpy(stage.data() + off[k], tables[k], (size_t)size[k] * sizeof(double));
  HIP_TRY(hipMemcpy(S.buf, stage.data(), total * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(S.passes, H.data(), H.size() * sizeof(HPass), hipMemcpyHostToDevice));
  if (largest <= kSmall) {
    hipLaunchKernelGGL(hugin_block_kernel, dim3(1), dim3(kBlock), 0, 0, S.passes, n_passes, S.buf);
    HIP_TRY(hipGetLastError());
  } else {
    for (int p = 0; p < n_passes; p++) {
      hipLaunchKernelGGL(hugin_marg_kernel, dim3((H[p].D + 255) / 256), dim3(256), 0, 0, S.passes, p, S.buf);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(hugin_absorb_kernel, dim3((H[p].N + 255) / 256), dim3(256), 0, 0, S.passes, p, S.buf);
      HIP_TRY(hipGetLastError());
    }
  }
  HIP_TRY(hipMemcpy(stage.data(), S.buf, total * sizeof(double), hipMemcpyDeviceToHost));
  std::vector<bool> written(n_tables, false);
  for (int p = 0; p < n_passes; p++) written[passes[6 * p + 1]] = written[passes[6 * p + 3]] = true;
  for (int k = 0; k < n_tables; k++)
    if (written[k]) std::memcpy(tables[k], stage.data() + off[k], (size_t)size[k] * sizeof(double));
  return NIP_NO_ERROR;
}
