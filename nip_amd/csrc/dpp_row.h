// dpp_row.h -- 16-lane DPP row primitives shared by the row-form chain
// kernels (chain_kernels.hip: the e_step; chain_ckpt.hip: the row-form
// filters of chain_fb_ckd_kernel).  One 16-lane row holds one chain's 16
// states, lane y state y.  Included inside an anonymous namespace user.
#pragma once
#include <hip/hip_runtime.h>

namespace nipamd {
namespace {

// DPP row_ror:K -- every lane of a 16-lane row has a source, so no "old"
// operand is needed (mov_dpp with bound_ctrl)
template <int K>
__device__ __forceinline__ double row_ror(double v) {
  static_assert(K > 0 && K < 16, "row_ror");
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int rl = __builtin_amdgcn_mov_dpp(lo, 0x120 + K, 0xF, 0xF, true);
  const int rh = __builtin_amdgcn_mov_dpp(hi, 0x120 + K, 0xF, 0xF, true);
  return __hiloint2double(rh, rl);
}



// acc += (value of lane K of this row) * c   -- one v_fmac_f64 with a 64-bit
// DPP row_newbcast source (gfx950 DP-ALU DPP); the broadcast costs nothing
// extra.  hipcc neither pads nor schedules inside asm, so the VALU->DPP read
// hazard (2 wait states) is covered by the s_nop in the first term (NOP_FIRST).
template <int K, bool NOP_FIRST>
__device__ __forceinline__ void fmac_bcast(double& acc, double v, double c) {
  if (NOP_FIRST)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(K));
  else
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(v), "v"(c), "n"(K));
}

// sum_k x[lane k] * c[k] over the 16 lanes of the row, x read by broadcast;
// the result is identical in every lane (fixed k order).
__device__ __forceinline__ double dot_bcast(double x, const double (&c)[16]) {
#ifdef NIPAMD_ABLATE_NO_DOT      // timing-only ablation build (wrong results)
  return x * c[0];
#endif
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  fmac_bcast<0, true>(a0, x, c[0]);   fmac_bcast<1, false>(a1, x, c[1]);
  fmac_bcast<2, false>(a2, x, c[2]);  fmac_bcast<3, false>(a3, x, c[3]);
  fmac_bcast<4, false>(a0, x, c[4]);  fmac_bcast<5, false>(a1, x, c[5]);
  fmac_bcast<6, false>(a2, x, c[6]);  fmac_bcast<7, false>(a3, x, c[7]);
  fmac_bcast<8, false>(a0, x, c[8]);  fmac_bcast<9, false>(a1, x, c[9]);
  fmac_bcast<10, false>(a2, x, c[10]); fmac_bcast<11, false>(a3, x, c[11]);
  fmac_bcast<12, false>(a0, x, c[12]); fmac_bcast<13, false>(a1, x, c[13]);
  fmac_bcast<14, false>(a2, x, c[14]); fmac_bcast<15, false>(a3, x, c[15]);
  return (a0 + a1) + (a2 + a3);
}

// K[k] += (value of lane k of this row) * w, k = 0..15 (E-step outer products)
__device__ __forceinline__ void acc_bcast(double (&K)[16], double x, double w) {
  fmac_bcast<0, true>(K[0], x, w);    fmac_bcast<1, false>(K[1], x, w);
  fmac_bcast<2, false>(K[2], x, w);   fmac_bcast<3, false>(K[3], x, w);
  fmac_bcast<4, false>(K[4], x, w);   fmac_bcast<5, false>(K[5], x, w);
  fmac_bcast<6, false>(K[6], x, w);   fmac_bcast<7, false>(K[7], x, w);
  fmac_bcast<8, false>(K[8], x, w);   fmac_bcast<9, false>(K[9], x, w);
  fmac_bcast<10, false>(K[10], x, w); fmac_bcast<11, false>(K[11], x, w);
  fmac_bcast<12, false>(K[12], x, w); fmac_bcast<13, false>(K[13], x, w);
  fmac_bcast<14, false>(K[14], x, w); fmac_bcast<15, false>(K[15], x, w);
}

// Sum over the 16 lanes of the row; identical bits in every lane (each level
// pairs lanes whose partial sums are equal, and IEEE addition commutes).
__device__ __forceinline__ double row_sum(double x) {
#ifdef NIPAMD_ABLATE_NO_REDUCE   // timing-only ablation build (wrong results)
  return x;
#endif
  // x must be one rounded value in every lane: if x is a fresh product the
  // compiler may contract this lane's term of the first add into an fma
  // (x = a*b; x += ror(x) -> fma(a, b, ror(x))), the lanes then disagree in
  // the last bit, and a scale exponent taken from the sum can differ by one
  // between lanes (a sum of probabilities sits right at 1.0)
  asm("" : "+v"(x));
  x += row_ror<8>(x);
  x += row_ror<4>(x);
  x += row_ror<2>(x);
  x += row_ror<1>(x);
  return x;
}

}  // namespace
}  // namespace nipamd
