// Shared device helpers for libxtrl_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/xtrl_hip.h"

namespace xtrl {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ----------------------------------------------------------------------------------------------
// error reporting (host)
// ----------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define XTRL_REQUIRE(cond, ...)                                                                   \
  do {                                                                                            \
    if (!(cond)) {                                                                                \
      ::xtrl::set_error(__VA_ARGS__);                                                             \
      return XTRL_E_ARG;                                                                          \
    }                                                                                             \
  } while (0)

#define XTRL_LAUNCHED(what)                                                                       \
  do {                                                                                            \
    int rc__ = ::xtrl::check_launch(what);                                                        \
    if (rc__) return rc__;                                                                        \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ----------------------------------------------------------------------------------------------
// wave reductions (64 lanes)
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// DPP forms for latency-bound kernels: four intra-row steps as DPP moves (quad xor 1, xor 2, half-row
// mirror, row mirror — after the quad steps every lane of a quad holds the same value, so the
// mirrors pair whole groups), then two cross-row shuffles.  A different association from wave_sum.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
#ifndef XTRL_DPP_BCAST
#define XTRL_DPP_BCAST 1
#endif
// a row's value broadcast into the next row(s) (row_bcast:15 into rows 1 and 3, row_bcast:31 into
// rows 2 and 3; the other rows get 0 / -inf): the cross-row steps on the VALU instead of two LDS
// permutes.  The last lane then holds ((r3 + r2) + (r1 + r0)) — the xor-shuffle form's
// ((r0 + r1) + (r2 + r3)) with each add commuted, so the same bits — and readlane broadcasts it.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_bcast(float v, float fill) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, fill), __builtin_bit_cast(int, v),
                                                                CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
#if XTRL_DPP_BCAST
  v += dpp_bcast<0x142, 0xA>(v, 0.f);   // row_bcast:15 -> rows 1, 3
  v += dpp_bcast<0x143, 0xC>(v, 0.f);   // row_bcast:31 -> rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
#else
  v += __shfl_xor(v, 16, kWave);
  v += __shfl_xor(v, 32, kWave);
  return v;
#endif
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
#if XTRL_DPP_BCAST
  v = fmaxf(v, dpp_bcast<0x142, 0xA>(v, -INFINITY));
  v = fmaxf(v, dpp_bcast<0x143, 0xC>(v, -INFINITY));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
#else
  v = fmaxf(v, __shfl_xor(v, 16, kWave));
  v = fmaxf(v, __shfl_xor(v, 32, kWave));
  return v;
#endif
}

// 4 x 4 transpose across the four lanes of a quad (lanes with equal lane >> 2): on entry lane
// c = lane & 3 holds column c of the block (x[q] = element (q, c)), on exit its row c
// (x[k] = element (c, k)).  Two exchange stages: lane ^ 2 swaps the off-diagonal 2 x 2 blocks,
// lane ^ 1 transposes each 2 x 2 block.
template <typename T>
__device__ __forceinline__ void quad_transpose(T (&x)[4], int lane) {
  const bool b1 = (lane & 2) != 0, b0 = (lane & 1) != 0;
  T s0 = b1 ? x[0] : x[2], s1 = b1 ? x[1] : x[3];
  T r0 = __shfl_xor(s0, 2, kWave), r1 = __shfl_xor(s1, 2, kWave);
  if (b1) {
    x[0] = r0;
    x[1] = r1;
  } else {
    x[2] = r0;
    x[3] = r1;
  }
  s0 = b0 ? x[0] : x[1];
  s1 = b0 ? x[2] : x[3];
  r0 = __shfl_xor(s0, 1, kWave);
  r1 = __shfl_xor(s1, 1, kWave);
  if (b0) {
    x[0] = r0;
    x[2] = r1;
  } else {
    x[1] = r0;
    x[3] = r1;
  }
}

// LDS hand-off between lanes of ONE wave (no workgroup barrier: waves of a block may have exited)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// activations, written the way PyTorch's CPU kernels evaluate them
// x-transformers pre-norms: LayerNorm (no affine, eps 1e-5; sq = the centred second moment) or,
// rms (Decoder use_rmsnorm), RMSNorm = F.normalize(x, eps 1e-12) sqrt(d) (the caller takes mean 0, so
// sq = the raw sum of squares) — the row's multiplier either way: y = (x - mean) * rstd * g
__device__ __forceinline__ float norm_rstd(float sq, float d, bool rms) {
  return rms ? sqrtf(d) / fmaxf(sqrtf(sq), 1e-12f) : 1.0f / sqrtf(sq / d + 1e-5f);
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float geluf_(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float siluf_(float x) { return x / (1.0f + expf(-x)); }
// torch.lerp(start, end, w): two-branch form
__device__ __forceinline__ float lerpf_(float s, float e, float w) {
  return (fabsf(w) < 0.5f) ? s + w * (e - s) : e - (e - s) * (1.0f - w);
}

}  // namespace xtrl
