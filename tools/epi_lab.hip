// Epilogue ALU lab: the FF1 forward epilogue (GELU + saved derivative + FF dropout) alone over a
// 16384 x 1024 output, without the GEMM, to price its parts.  hipcc -O3 --offload-arch=gfx950
// tools/epi_lab.hip -o tools/epi_lab.bin -I x-transformers-rl_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include "philox.h"
using namespace xtrl;

// VAR: 0 = copy, 1 = GELU + derivative (erff/expf), 2 = 1 + Philox-10 per 4 rows,
//      3 = 2 with the derivative from one erff and one expf (shared terms)
template <int VAR>
__global__ __launch_bounds__(256) void k_epi(float* __restrict__ y, float* __restrict__ dy, int M, int N,
                                               uint32_t thresh, float inv_keep, uint64_t seed) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int mb = (blockIdx.y * 4 + (threadIdx.x >> 6)) * 16;
  for (int g = 0; g < 4; ++g) {
    const int m0 = mb + 4 * g;
    u32x4_t kw{0u, 0u, 0u, 0u};
    if (VAR >= 2) kw = philox4x32_10((uint32_t)n, (uint32_t)(m0 >> 2), 7u, rng_c3(FIELD_FF_DROPOUT, 0), seed);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = m0 + q;
      float x = (float)((m * 131 + n * 7) % 977) * 0.005f - 2.4f;
      float a = 1.f;
      if (VAR >= 1) {
        const float e = erff(x * 0.70710678118654752f);
        const float cdf = 0.5f * (1.0f + e);
        const float pdf = 0.3989422804014327f * expf(x * x * -0.5f);
        a = cdf + x * pdf;
        x = (0.5f * x) * (1.0f + e);
      }
      if (VAR >= 2) {
        const uint32_t word = q == 0 ? kw.x : (q == 1 ? kw.y : (q == 2 ? kw.z : kw.w));
        const bool keep = word >= thresh;
        x = keep ? x * inv_keep : 0.f;
        a = keep ? a * inv_keep : 0.f;
      }
      y[(size_t)m * N + n] = x;
      dy[(size_t)m * N + n] = a;
    }
  }
}

template <int VAR>
float run(float* y, float* dy, int M, int N) {
  dim3 grid(N / 64, M / 64);
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  k_epi<VAR><<<grid, 256>>>(y, dy, M, N, 0x40000000u, 1.f / 0.75f, 1234);
  hipEventRecord(s);
  for (int i = 0; i < 20; ++i) k_epi<VAR><<<grid, 256>>>(y, dy, M, N, 0x40000000u, 1.f / 0.75f, 1234);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms / 20 * 1e3f;
}

int main() {
  const int M = 16384, N = 1024;
  float *y, *dy;
  hipMalloc(&y, (size_t)M * N * 4);
  hipMalloc(&dy, (size_t)M * N * 4);
  printf("copy          %8.1f us\n", run<0>(y, dy, M, N));
  printf("gelu+deriv    %8.1f us\n", run<1>(y, dy, M, N));
  printf("+philox10     %8.1f us\n", run<2>(y, dy, M, N));
  return 0;
}
