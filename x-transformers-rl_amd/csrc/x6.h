// Split-bf16 ("X6") helpers shared by the GEMM kernels: an fp32 value x = hi + mid + lo exactly,
// each piece the round-to-nearest bf16 of the running remainder (the subtractions are exact, the
// three pieces hold all 24 significand bits); a product a.b is then the sum of the six largest
// piece products lo.hi + hi.lo + mid.mid + mid.hi + hi.mid + hi.hi on the bf16 matrix cores with
// fp32 accumulation (the dropped mid.lo, lo.mid, lo.lo are below 2^-24 of the product).
#pragma once
#include "common.h"

namespace xtrl {
namespace {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// x = hi + mid + lo exactly (round-to-nearest bf16 of the running remainder; exact subtractions).
// Written on packed pairs: one v_cvt_pk_bf16_f32 per pair and level, the pieces widened back to
// f32 by a shift (low half) / mask (high half) — 4.5 VALU per value instead of the ~7.7 the
// vector-convert form compiled to.
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}
// (scalar v_sub_f32 in asm: left to itself the compiler pairs the subtractions into v_pk_add_f32
// plus register moves, slower beside MFMAs)
__device__ __forceinline__ float sub_f32(float a, float b) { return a - b; }
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = pk_bf16(a, b);
  const float ra = sub_f32(a, __builtin_bit_cast(float, h << 16));
  const float rb = sub_f32(b, __builtin_bit_cast(float, h & 0xffff0000u));
  m = pk_bf16(ra, rb);
  const float sa = sub_f32(ra, __builtin_bit_cast(float, m << 16));
  const float sb = sub_f32(rb, __builtin_bit_cast(float, m & 0xffff0000u));
  l = pk_bf16(sa, sb);
}
__device__ __forceinline__ void split3(float4 v, bf16x4& h, bf16x4& m, bf16x4& l) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split3_pair(v.x, v.y, h0, m0, l0);
  split3_pair(v.z, v.w, h1, m1, l1);
  h = __builtin_bit_cast(bf16x4, make_uint2(h0, h1));
  m = __builtin_bit_cast(bf16x4, make_uint2(m0, m1));
  l = __builtin_bit_cast(bf16x4, make_uint2(l0, l1));
}

}  // namespace
}  // namespace xtrl
