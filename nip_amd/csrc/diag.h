// diag.h -- measurement switches.  Kernel-selection A/B switches
// (NIPAMD_FB_KERNEL, NIPAMD_ESTEP_KERNEL, NIPAMD_WIDE_KERNEL, NIPAMD_JT_L) are
// read from the environment only in diagnostics builds (-DNIPAMD_DIAGNOSTICS,
// nip_amd/_lib/diag/libnip_amd_diag.so, selected with NIPAMD_LIB); the product
// library always runs the default kernels.
#pragma once

#include <cstdlib>

namespace nipamd {

inline const char* diag_env(const char* name) {
#ifdef NIPAMD_DIAGNOSTICS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

}  // namespace nipamd
