// Store policy of the chain kernels' global streams (device code only).
//
// Posteriors are write-once streams nothing on the GPU reads back: they
// leave with nontemporal stores, so they do not evict the scratch rows a
// block reads back in its phase B (interleaved A/B on one box: config 2
// 0.291 -> 0.278 ms, config 3 3.14 -> 3.06 ms, profiles/r04/gpu/r04z_*).
// Scratch rows (messages written in phase A, read in phase B by the same
// block) keep the default policy unless NIPAMD_SCR_NT (A/B builds).
#pragma once
#include <hip/hip_runtime.h>

#ifndef NIPAMD_POST_NT
#define NIPAMD_POST_NT 1
#endif
#ifndef NIPAMD_SCR_NT
#define NIPAMD_SCR_NT 0
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
