// Cost of the row-resident step's phase shapes in isolation (one 512-thread workgroup, shader-clock
// stamps): an empty barrier, a wave-0 LayerNorm + barrier over an LDS row, a 4 x 16-float GEMV with
// its LDS reduction.  Build: hipcc --offload-arch=gfx950 -O3 -o row_phase_lab tools/row_phase_lab.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float dpp_b1(float v) { return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)); }
__device__ __forceinline__ float dpp_4e(float v) { return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)); }
__device__ __forceinline__ float dpp_141(float v) { return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)); }
__device__ __forceinline__ float dpp_140(float v) { return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)); }
__device__ __forceinline__ float wsum(float v) {
  v += dpp_b1(v); v += dpp_4e(v); v += dpp_141(v); v += dpp_140(v);
  v += __shfl_xor(v, 16, 64); v += __shfl_xor(v, 32, 64);
  return v;
}

__device__ __forceinline__ float xsum16(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
}
__device__ __forceinline__ float wsum_pl(float v) {
  v += dpp_b1(v); v += dpp_4e(v); v += dpp_141(v); v += dpp_140(v);
  return xsum32(xsum16(v));
}
// the two reductions agree bit for bit on random-ish data
__global__ void k_check(const float* x, int* bad) {
  const float v = x[threadIdx.x] * 1.37f + 0.11f * threadIdx.x;
  if (wsum(v) != wsum_pl(v)) atomicAdd(bad, 1);
}

template <int MODE>
__global__ __launch_bounds__(512) void k_lab(const float* g, float* out, uint64_t* cyc, int iters, int d) {
  __shared__ float xs[256], xn[256], part[4096];
  const int tid = threadIdx.x;
  if (tid < 256) xs[tid] = 0.01f * tid;
  __syncthreads();
  const uint64_t t0 = clock64();
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {   // barrier only
      __syncthreads();
    } else if (MODE == 3) {   // MODE 1 with permlane swaps for the cross-row steps
      if (tid < 64) {
        float v[4], gv[4], sm = 0.f;
        for (int k = 0; k < 4; ++k) { const int c = tid + 64 * k; gv[k] = c < d ? g[c] : 0.f; v[k] = c < d ? xs[c] : 0.f; sm += v[k]; }
        const float mean = wsum_pl(sm) / d;
        float qq = 0.f;
        for (int k = 0; k < 4; ++k) { const float dl = v[k] - mean; qq += tid + 64 * k < d ? dl * dl : 0.f; }
        const float rstd = 1.f / sqrtf(wsum_pl(qq) / d + 1e-5f);
        for (int k = 0; k < 4; ++k) { const int c = tid + 64 * k; if (c < d) xn[c] = (v[k] - mean) * rstd * gv[k]; }
      }
      __syncthreads();
    } else if (MODE == 1) {   // wave-0 LayerNorm from LDS, gain from global, + barrier
      if (tid < 64) {
        float v[4], gv[4], sm = 0.f;
        for (int k = 0; k < 4; ++k) { const int c = tid + 64 * k; gv[k] = c < d ? g[c] : 0.f; v[k] = c < d ? xs[c] : 0.f; sm += v[k]; }
        const float mean = wsum(sm) / d;
        float qq = 0.f;
        for (int k = 0; k < 4; ++k) { const float dl = v[k] - mean; qq += tid + 64 * k < d ? dl * dl : 0.f; }
        const float rstd = 1.f / sqrtf(wsum(qq) / d + 1e-5f);
        for (int k = 0; k < 4; ++k) { const int c = tid + 64 * k; if (c < d) xn[c] = (v[k] - mean) * rstd * gv[k]; }
      }
      __syncthreads();
    } else if (MODE == 6) {   // MODE 5 with the partials loaded 8 at a time (adds in the same order)
      const int N = d, NC4 = N / 4, KG = min(32, 512 / NC4), Kc = (d + KG - 1) / KG;
      if (tid < KG * NC4) {
        const int gg = tid / NC4, n4 = 4 * (tid - gg * NC4), k0 = gg * Kc;
        float4 a = make_float4(xn[k0], 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(part + gg * N + n4) = a;
      }
      __syncthreads();
      for (int n = tid; n < N; n += 512) {
        float v = part[n];
        for (int g0 = 1; g0 < KG; g0 += 8) {
          float pv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) pv[u] = part[min(g0 + u, KG - 1) * N + n];
#pragma unroll
          for (int u = 0; u < 8; ++u) if (g0 + u < KG) v += pv[u];
        }
        xs[n] = v * 1e-3f + xs[n];
      }
      __syncthreads();
    } else if (MODE == 4 || MODE == 5) {   // 4: GEMV with W from LDS; 5: only the partial store + reduction
      const int N = d, NC4 = N / 4, KG = min(32, 512 / NC4), Kc = (d + KG - 1) / KG;
      if (tid < KG * NC4) {
        const int gg = tid / NC4, n4 = 4 * (tid - gg * NC4), k0 = gg * Kc, k1 = min(d, k0 + Kc);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (MODE == 4)
          for (int k = k0; k < k1; ++k) {
            const float xv = xn[k];
            const float4 w = *reinterpret_cast<const float4*>(part + 2048 + (k * N + n4) % 2048);
            a.x += xv * w.x; a.y += xv * w.y; a.z += xv * w.z; a.w += xv * w.w;
          }
        else a.x = xn[k0];
        *reinterpret_cast<float4*>(part + gg * N + n4) = a;
      }
      __syncthreads();
      for (int n = tid; n < N; n += 512) {
        float v = part[n];
        for (int gg = 1; gg < KG; ++gg) v += part[gg * N + n];
        xs[n] = v * 1e-3f + xs[n];
      }
      __syncthreads();
    } else if (MODE == 2) {   // GEMV 48 -> 48 (k-groups 32, Kc 2) with its LDS reduction, weights from global
      const int N = d, NC4 = N / 4, KG = min(32, 512 / NC4), Kc = (d + KG - 1) / KG;
      if (tid < KG * NC4) {
        const int gg = tid / NC4, n4 = 4 * (tid - gg * NC4), k0 = gg * Kc, k1 = min(d, k0 + Kc);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = k0; k < k1; ++k) {
          const float xv = xn[k];
          const float4 w = *reinterpret_cast<const float4*>(g + k * N + n4);
          a.x += xv * w.x; a.y += xv * w.y; a.z += xv * w.z; a.w += xv * w.w;
        }
        *reinterpret_cast<float4*>(part + gg * N + n4) = a;
      }
      __syncthreads();
      for (int n = tid; n < N; n += 512) {
        float v = part[n];
        for (int gg = 1; gg < KG; ++gg) v += part[gg * N + n];
        xs[n] = v * 1e-3f + xs[n];
      }
      __syncthreads();
    }
  }
  const uint64_t t1 = clock64();
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
  if (tid < 256) out[tid] = xn[tid] + xs[tid] + acc;
}

int main() {
  float *g, *out; uint64_t* cyc;
  hipMalloc(&g, 1 << 20); hipMalloc(&out, 4096); hipMalloc(&cyc, 64);
  hipMemset(g, 0, 1 << 20);
  const int iters = 1000;
  for (int rep = 0; rep < 2; ++rep) {
    for (int mode = 0; mode < 7; ++mode) {
      uint64_t h = 0;
      if (mode == 0) hipLaunchKernelGGL(k_lab<0>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      if (mode == 1) hipLaunchKernelGGL(k_lab<1>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      if (mode == 2) hipLaunchKernelGGL(k_lab<2>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      if (mode == 3) hipLaunchKernelGGL(k_lab<3>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      if (mode == 4) hipLaunchKernelGGL(k_lab<4>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      if (mode == 5) hipLaunchKernelGGL(k_lab<5>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      if (mode == 6) hipLaunchKernelGGL(k_lab<6>, dim3(1), dim3(512), 0, 0, g, out, cyc, iters, 48);
      hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
      printf("mode %d (%s): %.0f cycles per phase\n", mode, mode == 0 ? "barrier" : mode == 1 ? "LayerNorm + barrier" : mode == 2 ? "GEMV 48x48 + 2 barriers" : mode == 3 ? "LayerNorm (permlane) + barrier" : mode == 4 ? "GEMV, W from LDS" : mode == 5 ? "GEMV partial store + reduction only" : "the same, partials 8 in flight", (double)h / iters);
    }
  }
  {
    float* x; int* bad; int hb = 0;
    hipMalloc(&x, 256); hipMalloc(&bad, 4); hipMemset(bad, 0, 4);
    float hx[64]; for (int i = 0; i < 64; ++i) hx[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    hipMemcpy(x, hx, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, x, bad);
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("permlane reduction vs ds_bpermute: %d lanes differ\n", hb);
  }
  return 0;
}
