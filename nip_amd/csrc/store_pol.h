// Store policy of the chain kernels' global streams (device code only).
//
// Posteriors are write-once streams nothing on the GPU reads back: they
// leave with nontemporal stores, so they do not evict the scratch rows a
// block reads back in its phase B (interleaved A/B on one box: config 2
// 0.291 -> 0.278 ms, config 3 3.14 -> 3.06 ms, profiles/r04/gpu/r04z_*).
// Scratch rows (messages written in phase A, read in phase B by the same
// block): nontemporal in the wide kernels (config 3's chain_mfma_wide_kernel
// 3.07 -> 2.91 ms, config 5's chain_row64_kernel 0.0476 -> 0.0471 ms,
// profiles/r04/gpu/r04za_*), the default policy in chain_fb_ckpt_kernel and
// chain_estep16_kernel (nontemporal there: 0.284 -> 0.296 ms and 10.0 ->
// 17.4 ms -- the e_step's per-lane 8-byte rows and 4-byte exponents).
#pragma once
#include <hip/hip_runtime.h>

#ifndef NIPAMD_POST_NT
#define NIPAMD_POST_NT 1
#endif
#ifndef NIPAMD_SCR_NT
#define NIPAMD_SCR_NT 0         // chain_fb_ckpt_kernel, chain_estep16_kernel
#endif
#ifndef NIPAMD_WIDE_SCR_NT
#define NIPAMD_WIDE_SCR_NT 1    // chain_mfma_wide_kernel, chain_row64_kernel
#endif
#ifndef NIPAMD_MSG_NT
#define NIPAMD_MSG_NT 1         // the wide e_step message kernels' rows (estep_wide.hip): 0.3-0.5%
#endif
#ifndef NIPAMD_SCR_NTLD
#define NIPAMD_SCR_NTLD 0       // A/B builds: scratch rows read back (their last use) nontemporal
#endif

namespace nipamd {

template <bool NT, typename V>
__device__ __forceinline__ void store_pol(V* p, const V& v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT, typename V>
__device__ __forceinline__ V load_pol(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

}  // namespace nipamd
