// GEMM tiling experiments for the fp32 MFMA GEMM (not part of the library).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_lab.hip -o /tmp/gemm_lab && /tmp/gemm_lab
// C[M][N] = A[M][K] . B[N][K]^T, all row-major fp32 ("N"/"N" layouts of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

#ifndef LAB_MINB
#define LAB_MINB 1
#endif
template <int BM, int BN, int BK, int WM, int WN, int NBUF>
__global__ __launch_bounds__(64 * WM * WN, LAB_MINB) void k_lab(const float* __restrict__ A, const float* __restrict__ B,
                                                     float* __restrict__ C, int M, int N, int K) {
  constexpr int NT = 64 * WM * WN, TM = BM / (32 * WM), TN = BN / (32 * WN);
  constexpr int AST = BM + 1, BST = BN + 1;
  constexpr int A_F4 = BM * BK / 4 / NT, B_F4 = BN * BK / 4 / NT;
  static_assert(A_F4 >= 1 && B_F4 >= 1, "");
  __shared__ float As[NBUF][BK][AST];
  __shared__ float Bs[NBUF][BK][BST];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  float4 ra[A_F4], rb[B_F4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      ra[i] = *reinterpret_cast<const float4*>(A + (int64_t)min(m0 + r, M - 1) * K + k0 + 4 * q);
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      rb[i] = *reinterpret_cast<const float4*>(B + (int64_t)min(n0 + r, N - 1) * K + k0 + 4 * q);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      As[buf][4 * q + 0][r] = ra[i].x; As[buf][4 * q + 1][r] = ra[i].y;
      As[buf][4 * q + 2][r] = ra[i].z; As[buf][4 * q + 3][r] = ra[i].w;
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      Bs[buf][4 * q + 0][r] = rb[i].x; Bs[buf][4 * q + 1][r] = rb[i].y;
      Bs[buf][4 * q + 2][r] = rb[i].z; Bs[buf][4 * q + 3][r] = rb[i].w;
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int fi = wm * 32 * TM + (lane & 31), fj = wn * 32 * TN + (lane & 31), fk = lane >> 5;
  auto compute = [&](int cur) {
    float av[2][TM], bv[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[0][i] = As[cur][fk][fi + 32 * i];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[0][j] = Bs[cur][fk][fj + 32 * j];
#pragma unroll
    for (int st = 0; st < BK / 2; ++st) {
      const int pb = st & 1;
      if (st + 1 < BK / 2) {
#pragma unroll
        for (int i = 0; i < TM; ++i) av[pb ^ 1][i] = As[cur][fk + 2 * st + 2][fi + 32 * i];
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[pb ^ 1][j] = Bs[cur][fk + 2 * st + 2][fj + 32 * j];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[pb][i], bv[pb][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int nk = K / BK;
  if constexpr (NBUF == 2) {
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load((kt + 1) * BK);
      __builtin_amdgcn_sched_barrier(0);
      compute(kt & 1);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) store((kt & 1) ^ 1);
      __syncthreads();
    }
  } else {   // one LDS buffer, tile t+1 in registers: write it after the barrier, re-issue t+2
    load(0);
    store(0);
    if (nk > 1) load(BK);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      compute(0);
      __syncthreads();
      if (kt + 1 < nk) {
        store(0);
        if (kt + 2 < nk) load((kt + 2) * BK);
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 32 * TN + 32 * j + (lane & 31);
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 * TM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < M) C[(int64_t)m * N + n] = acc[i][j][r];
      }
  }
}

template <int BM, int BN, int BK, int WM, int WN, int NBUF>
void run(const char* tag, const float* A, const float* B, float* C, int M, int N, int K, const std::vector<float>& hA,
         const std::vector<float>& hB) {
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);
  auto launch = [&] { hipLaunchKernelGGL((k_lab<BM, BN, BK, WM, WN, NBUF>), grid, dim3(64 * WM * WN), 0, 0, A, B, C, M, N, K); };
  launch();
  CK(hipDeviceSynchronize());
  // spot-check a few entries
  std::vector<float> hC((size_t)M * N);
  CK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0;
  for (int t = 0; t < 64; ++t) {
    const int m = (t * 7919) % M, n = (t * 104729) % N;
    double s = 0;
    for (int k = 0; k < K; ++k) s += (double)hA[(size_t)m * K + k] * hB[(size_t)n * K + k];
    maxerr = fmax(maxerr, fabs(s - hC[(size_t)m * N + n]) / (1 + fabs(s)));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int it = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  printf("%-28s M=%5d N=%5d K=%5d  %8.1f us  %6.1f TF  err %.1e\n", tag, M, N, K, us, 2.0 * M * N * K / us / 1e6, maxerr);
}


// ---- glds pipeline: global_load_lds (16 B / lane) into an XOR-swizzled [row][32] image per stage,
// k-slot permutation (MFMA step s, lane half g uses k = 16 g + s) so each lane's 16 steps are 4
// ds_read_b128; NS stages with counted vmcnt and raw barriers.
__device__ __forceinline__ void waitcnt_vm(int n) {
  // s_waitcnt vmcnt(n) expcnt(7) lgkmcnt(15)
  if (n == 0) __builtin_amdgcn_s_waitcnt(0x0F70);
  else if (n == 4) __builtin_amdgcn_s_waitcnt(0x0F74);
  else if (n == 8) __builtin_amdgcn_s_waitcnt(0x0F78);
  else if (n == 12) __builtin_amdgcn_s_waitcnt(0x0F7C);
  else __builtin_amdgcn_s_waitcnt(0x4F70);   // 16
}
typedef __attribute__((address_space(3))) void lds_void;

template <int NS, int WPB>   // WPB: 4 waves (2x2 of 64x64) for a 128x128 tile
__global__ __launch_bounds__(256) void k_glds(const float* __restrict__ A, const float* __restrict__ B,
                                             float* __restrict__ C, int M, int N, int K) {
  constexpr int BM = 128, BN = 128, BK = 32;
  constexpr int STAGE = (BM + BN) * BK;   // floats per stage
  // one __shared__ object per stage: the compiler then tracks each stage's LDS-DMA separately and
  // does not drain every outstanding load before a read of an older stage
  __shared__ __attribute__((aligned(16))) float sm0[STAGE];
  __shared__ __attribute__((aligned(16))) float sm1[STAGE];
  __shared__ __attribute__((aligned(16))) float sm2[NS > 2 ? STAGE : 4];
  __shared__ __attribute__((aligned(16))) float sm3[NS > 3 ? STAGE : 4];
  auto stage = [&]<int S>() -> float* {
    if constexpr (S == 0) return sm0;
    else if constexpr (S == 1) return sm1;
    else if constexpr (S == 2) return sm2;
    else return sm3;
  };
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int lr = lane >> 3, lp = lane & 7;
  const float* srcA[4];
  const float* srcB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (w * 4 + i) * 8 + lr;
    const int j = lp ^ ((row >> 1) & 7);
    srcA[i] = A + (int64_t)min(m0 + row, M - 1) * K + 4 * j;
    srcB[i] = B + (int64_t)min(n0 + row, N - 1) * K + 4 * j;
  }
  auto stage_load = [&]<int S>(int t) {
    float* st = stage.template operator()<S>();
    const int k0 = t * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcA[i] + k0), (lds_void*)(st + (w * 4 + i) * 8 * BK), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[i] + k0), (lds_void*)(st + BM * BK + (w * 4 + i) * 8 * BK), 16, 0, 0);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int g = lane >> 5, ml = lane & 31;
  int offa[2][4], offb[2][4];   // per fragment and quarter: float offset of its 16-byte chunk
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ra = wm * 64 + 32 * i + ml, rb = wn * 64 + 32 * i + ml;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = 4 * g + q;
      offa[i][q] = ra * BK + 4 * (j ^ ((ra >> 1) & 7));
      offb[i][q] = BM * BK + rb * BK + 4 * (j ^ ((rb >> 1) & 7));
    }
  }
  const int nk = K / BK;
  // LDS fragment reads as inline asm: the compiler's waitcnt pass cannot tell them apart from the
  // stage being filled by LDS-DMA and would otherwise drain every load first; the matching
  // lgkmcnt waits are explicit and tied to the registers they guard
  auto rd = [&](const float* p) -> f32x4 {
    f32x4 v;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
  };
  auto compute = [&](const float* st) {
    f32x4 af[2][2], bf[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[0][i] = rd(st + offa[i][0]);
      bf[0][i] = rd(st + offb[i][0]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cb = q & 1;
      if (q + 1 < 4) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          af[cb ^ 1][i] = rd(st + offa[i][q + 1]);
          bf[cb ^ 1][i] = rd(st + offb[i][q + 1]);
        }
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(af[cb][0]), "+v"(af[cb][1]), "+v"(bf[cb][0]), "+v"(bf[cb][1]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[cb][0]), "+v"(af[cb][1]), "+v"(bf[cb][0]), "+v"(bf[cb][1]));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jn = 0; jn < 2; ++jn) {
            const float a = af[cb][i][e], b = bf[cb][jn][e];
            acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i][jn], 0, 0, 0);
          }
    }
  };
  // prologue: tiles 0 .. NS-2 in flight
  stage_load.template operator()<0>(0);
  if constexpr (NS > 2) if (1 < nk) stage_load.template operator()<1>(1);
  if constexpr (NS > 3) if (2 < nk) stage_load.template operator()<2>(2);
  auto step = [&]<int S>(int t) {
    if (t >= nk) return;
    const int ahead = min(NS - 2, nk - 1 - t);   // tiles after t already issued
    waitcnt_vm(8 * ahead);
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nk) stage_load.template operator()<(S + NS - 1) % NS>(t + NS - 1);
    compute(stage.template operator()<S>());
  };
  for (int t = 0; t < nk; t += NS) {
    step.template operator()<0>(t);
    step.template operator()<1>(t + 1);
    if constexpr (NS > 2) step.template operator()<2>(t + 2);
    if constexpr (NS > 3) step.template operator()<3>(t + 3);
  }
#pragma unroll
  for (int jn = 0; jn < 2; ++jn) {
    const int n = n0 + wn * 64 + 32 * jn + ml;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * g;
        if (m < M) C[(int64_t)m * N + n] = acc[i][jn][r];
      }
  }
}

template <int NS>
void run_glds(const char* tag, const float* A, const float* B, float* C, int M, int N, int K, const std::vector<float>& hA,
              const std::vector<float>& hB) {
  dim3 grid((N + 127) / 128, (M + 127) / 128);
  auto launch = [&] { hipLaunchKernelGGL((k_glds<NS, 4>), grid, dim3(256), 0, 0, A, B, C, M, N, K); };
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> hC((size_t)M * N);
  CK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0;
  for (int t = 0; t < 64; ++t) {
    const int m = (t * 7919) % M, n = (t * 104729) % N;
    double s = 0;
    for (int k = 0; k < K; ++k) s += (double)hA[(size_t)m * K + k] * hB[(size_t)n * K + k];
    maxerr = fmax(maxerr, fabs(s - hC[(size_t)m * N + n]) / (1 + fabs(s)));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int it = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < it; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  printf("%-28s M=%5d N=%5d K=%5d  %8.1f us  %6.1f TF  err %.1e\n", tag, M, N, K, us, 2.0 * M * N * K / us / 1e6, maxerr);
}

// ---- "TT" layouts (the weight-gradient GEMM): A given as [K][M], B as [K][N] (contiguous along
// m / n); both staged with float4 writes into k-major LDS images.  ROT: row k stored rotated by
// 32 columns when k is odd, so the two half-waves of a fragment read (rows k, k+1) hit disjoint
// LDS banks.
template <int ROT, int PADC>
__global__ __launch_bounds__(256) void k_tt(const float* __restrict__ A, const float* __restrict__ B,
                                           float* __restrict__ C, int M, int N, int K) {
  constexpr int BM = 128, BN = 128, BK = 32, NT = 256, ST = BM + PADC;
  constexpr int F4 = BM * BK / 4 / NT;   // 4 float4 per thread per operand
  __shared__ __attribute__((aligned(16))) float As[2][BK][ST];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][ST];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  float4 ra[F4], rb[F4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int e = tid + i * NT, r = e / (BM / 4), q = e % (BM / 4);
      ra[i] = *reinterpret_cast<const float4*>(A + (int64_t)(k0 + r) * M + m0 + 4 * q);
      rb[i] = *reinterpret_cast<const float4*>(B + (int64_t)(k0 + r) * N + n0 + 4 * q);
    }
  };
  auto col = [&](int k, int c) { return ROT ? ((c + 32 * (k & 1)) & (BM - 1)) : c; };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int e = tid + i * NT, r = e / (BM / 4), q = e % (BM / 4);
      *reinterpret_cast<float4*>(&As[buf][r][col(r, 4 * q)]) = ra[i];
      *reinterpret_cast<float4*>(&Bs[buf][r][col(r, 4 * q)]) = rb[i];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int fi = wm * 64 + (lane & 31), fj = wn * 64 + (lane & 31), fk = lane >> 5;
  auto compute = [&](int cur) {
    float av[2][2], bv[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      av[0][i] = As[cur][fk][col(fk, fi + 32 * i)];
      bv[0][i] = Bs[cur][fk][col(fk, fj + 32 * i)];
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int pb = st & 1;
      if (st + 1 < 16) {
        const int k = fk + 2 * st + 2;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          av[pb ^ 1][i] = As[cur][k][col(k, fi + 32 * i)];
          bv[pb ^ 1][i] = Bs[cur][k][col(k, fj + 32 * i)];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[pb][i], bv[pb][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int nk = K / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load((kt + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);
    compute(kt & 1);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) store((kt & 1) ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        C[(int64_t)m * N + n] = acc[i][j][r];
      }
  }
}

template <int ROT, int PADC>
void run_tt(const char* tag, int M, int N, int K) {
  std::vector<float> hA((size_t)K * M), hB((size_t)K * N);
  srand(2);
  for (auto& x : hA) x = (float)rand() / RAND_MAX - 0.5f;
  for (auto& x : hB) x = (float)rand() / RAND_MAX - 0.5f;
  float *A, *B, *C;
  CK(hipMalloc(&A, hA.size() * 4));
  CK(hipMalloc(&B, hB.size() * 4));
  CK(hipMalloc(&C, (size_t)M * N * 4));
  CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
  dim3 grid(N / 128, M / 128);
  auto launch = [&] { hipLaunchKernelGGL((k_tt<ROT, PADC>), grid, dim3(256), 0, 0, A, B, C, M, N, K); };
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> hC((size_t)M * N);
  CK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0;
  for (int t = 0; t < 32; ++t) {
    const int m = (t * 7919) % M, n = (t * 104729) % N;
    double s = 0;
    for (int k = 0; k < K; ++k) s += (double)hA[(size_t)k * M + m] * hB[(size_t)k * N + n];
    maxerr = fmax(maxerr, fabs(s - hC[(size_t)m * N + n]) / (1 + fabs(s)));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / 20;
  printf("%-28s M=%5d N=%5d K=%5d  %8.1f us  %6.1f TF  err %.1e\n", tag, M, N, K, us, 2.0 * M * N * K / us / 1e6, maxerr);
  CK(hipFree(A));
  CK(hipFree(B));
  CK(hipFree(C));
}

int main() {
  // weight-gradient-like: M = 1024 out, N = 256 in, K = 512 tokens per split (one workgroup round)
  for (int rep = 0; rep < 1; ++rep) {
    run_tt<0, 4>("TT pad4", 1024, 256, 16384);
    run_tt<1, 4>("TT pad4 rot32", 1024, 256, 16384);
    run_tt<1, 0>("TT pad0 rot32", 1024, 256, 16384);
    run_tt<0, 32>("TT pad32", 1024, 256, 16384);
    run_tt<0, 4>("TT pad4 4k", 4096, 4096, 4096);
    run_tt<1, 0>("TT pad0 rot32 4k", 4096, 4096, 4096);
  }
  if (getenv("LAB_TT_ONLY")) return 0;
  const int shapes[][3] = {{16384, 1024, 256}, {16384, 256, 1024}, {16384, 512, 512}, {4096, 4096, 4096}};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    std::vector<float> hA((size_t)M * K), hB((size_t)N * K);
    srand(1);
    for (auto& x : hA) x = (float)rand() / RAND_MAX - 0.5f;
    for (auto& x : hB) x = (float)rand() / RAND_MAX - 0.5f;
    float *A, *B, *C;
    CK(hipMalloc(&A, hA.size() * 4));
    CK(hipMalloc(&B, hB.size() * 4));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    run<128, 128, 32, 2, 2, 2>("128x128 4w(64x64) dbuf", A, B, C, M, N, K, hA, hB);
    run<128, 128, 32, 2, 2, 1>("128x128 4w(64x64) sbuf", A, B, C, M, N, K, hA, hB);
    run<128, 128, 32, 1, 2, 2>("128x128 2w(128x64) dbuf", A, B, C, M, N, K, hA, hB);
    run<128, 128, 32, 2, 1, 2>("128x128 2w(64x128) dbuf", A, B, C, M, N, K, hA, hB);
    run<256, 128, 32, 2, 2, 1>("256x128 4w(128x64) sbuf", A, B, C, M, N, K, hA, hB);
    run<256, 128, 32, 2, 2, 2>("256x128 4w(128x64) dbuf", A, B, C, M, N, K, hA, hB);
    run<128, 256, 32, 2, 2, 1>("128x256 4w(64x128) sbuf", A, B, C, M, N, K, hA, hB);
    run<256, 256, 32, 2, 2, 1>("256x256 4w(128x128) sbuf", A, B, C, M, N, K, hA, hB);
    run<128, 128, 16, 2, 2, 2>("128x128x16 4w dbuf", A, B, C, M, N, K, hA, hB);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
  }
  return 0;
}
