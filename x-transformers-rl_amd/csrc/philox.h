// Counter-based random streams shared by the rollout, the synthetic Sim and dropout.
// Bit-identical with oracle/philox.py (integer arithmetic + a fixed order of f32 adds, no FMA-able
// expressions, no transcendental functions):
//   philox4x32-10(counter = (c0, c1, c2, c3), key = (seed_lo, seed_hi))
//   c0 = slot / env / minibatch, c1 = timestep / epoch, c2 = learning update,
//   c3 = (field << 24) | sub-index
//   uniform(x) = (x >> 8) * 2^-24,  normal = (((u0 + u1) + u2) + u3 - 2) * sqrt(3)  (Irwin-Hall 4)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xtrl {

enum RngField : uint32_t {
  FIELD_STATE = 1,
  FIELD_REWARD = 2,
  FIELD_TERM = 3,
  FIELD_SAMPLE = 4,
  FIELD_COIN = 5,
  FIELD_DROPOUT = 6,      // attention probabilities (learn)
  FIELD_FF_DROPOUT = 7,   // feed-forward hidden units (learn)
};

struct u32x4_t {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ __forceinline__ u32x4_t philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                           uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

__host__ __device__ __forceinline__ uint32_t rng_c3(uint32_t field, uint32_t sub) {
  return (field << 24) | (sub & 0xFFFFFFu);
}

__host__ __device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-8f; }

__host__ __device__ __forceinline__ float rng_uniform(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t,
                                                      uint32_t field, uint32_t sub) {
  return u01(philox4x32_10(slot, t, update, rng_c3(field, sub), seed).x);
}

__host__ __device__ __forceinline__ uint32_t rng_u32(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t,
                                                     uint32_t field, uint32_t sub) {
  return philox4x32_10(slot, t, update, rng_c3(field, sub), seed).x;
}

__host__ __device__ __forceinline__ float rng_normal(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t,
                                                     uint32_t field, uint32_t sub) {
  const u32x4_t r = philox4x32_10(slot, t, update, rng_c3(field, sub), seed);
  // u01() is an exact power-of-two scaling, so FMA contraction of these adds cannot change bits
  float s = u01(r.x) + u01(r.y);
  s = s + u01(r.z);
  s = s + u01(r.w);
  const float c = s - 2.0f;
  return c * 1.7320508075688772f;
}

}  // namespace xtrl
