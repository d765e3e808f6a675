// Split-bf16 fp32 GEMM experiment (not part of the library).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/x6_lab.hip -o tools/x6_lab.bin
// Each fp32 operand x is split into three bf16 pieces x = hi + mid + lo (+ |r| <= 2^-24 |x|) and
// C = A.B^T is computed as the sum of the NP largest piece products on the bf16 matrix cores
// (v_mfma_f32_32x32x16_bf16, fp32 accumulate):
//   NP = 6: lo.hi + hi.lo + mid.mid + mid.hi + hi.mid + hi.hi
//   NP = 8: + mid.lo + lo.mid
// against the native f32 MFMA kernel (v_mfma_f32_32x32x2_f32) on the same tiles.  Reports time and
// the error against an fp64 reference, normalised by sum_k |a_k b_k| (the scale of an fp32 dot
// product's rounding error).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// x = hi + mid + lo, each round-to-nearest bf16 of the running remainder (subtractions exact)
__device__ __forceinline__ void split3(f32x4v x, bf16x4& h, bf16x4& m, bf16x4& l) {
  h = __builtin_convertvector(x, bf16x4);
  const f32x4v r1 = x - __builtin_convertvector(h, f32x4v);
  m = __builtin_convertvector(r1, bf16x4);
  const f32x4v r2 = r1 - __builtin_convertvector(m, f32x4v);
  l = __builtin_convertvector(r2, bf16x4);
}

// ---- native f32 MFMA baseline: 128x128x32, 4 waves of 64x64, one LDS stage + next slab in regs
__global__ __launch_bounds__(256) void k_f32(const float* __restrict__ A, const float* __restrict__ B,
                                             float* __restrict__ C, int M, int N, int K) {
  constexpr int BM = 128, BN = 128, BK = 32, NT = 256, TM = 2, TN = 2, AST = BM + 1, BST = BN + 1;
  constexpr int A_F4 = BM * BK / 4 / NT, B_F4 = BN * BK / 4 / NT;
  __shared__ float As[BK][AST];
  __shared__ float Bs[BK][BST];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / 2, wn = wave % 2;
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
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      As[4 * q + 0][r] = ra[i].x; As[4 * q + 1][r] = ra[i].y; As[4 * q + 2][r] = ra[i].z; As[4 * q + 3][r] = ra[i].w;
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      Bs[4 * q + 0][r] = rb[i].x; Bs[4 * q + 1][r] = rb[i].y; Bs[4 * q + 2][r] = rb[i].z; Bs[4 * q + 3][r] = rb[i].w;
    }
  };
  f32x16 acc[TM][TN];
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int fi = wm * 64 + (lane & 31), fj = wn * 64 + (lane & 31), fk = lane >> 5;
  auto compute = [&]() {
    float av[2][TM], bv[2][TN];
    for (int i = 0; i < TM; ++i) av[0][i] = As[fk][fi + 32 * i];
    for (int j = 0; j < TN; ++j) bv[0][j] = Bs[fk][fj + 32 * j];
#pragma unroll
    for (int st = 0; st < BK / 2; ++st) {
      const int pb = st & 1;
      if (st + 1 < BK / 2) {
        for (int i = 0; i < TM; ++i) av[pb ^ 1][i] = As[fk + 2 * st + 2][fi + 32 * i];
        for (int j = 0; j < TN; ++j) bv[pb ^ 1][j] = Bs[fk + 2 * st + 2][fj + 32 * j];
      }
      __builtin_amdgcn_sched_barrier(0);
      for (int i = 0; i < TM; ++i)
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[pb][i], bv[pb][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int nk = K / BK;
  load(0);
  store();
  if (nk > 1) load(BK);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    compute();
    __syncthreads();
    if (kt + 1 < nk) {
      store();
      if (kt + 2 < nk) load((kt + 2) * BK);
      __syncthreads();
    }
  }
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 64 + 32 * j + (lane & 31);
    for (int i = 0; i < TM; ++i)
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < M && n < N) C[(int64_t)m * N + n] = acc[i][j][r];
      }
  }
}

// ---- split-bf16: LDS images [piece][row][BK + PAD] of bf16 (row = m for A, n for B) ------------
template <int NP, int BK, int PAD>
__global__ __launch_bounds__(256) void k_x6(const float* __restrict__ A, const float* __restrict__ B,
                                            float* __restrict__ C, int M, int N, int K) {
  constexpr int BM = 128, BN = 128, NT = 256, TM = 2, TN = 2, RS = BK + PAD;   // row stride (bf16)
  constexpr int A_F4 = BM * BK / 4 / NT, B_F4 = BN * BK / 4 / NT;
  __shared__ __attribute__((aligned(16))) __bf16 As[3][BM][RS];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3][BN][RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / 2, wn = wave % 2;
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
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      bf16x4 h, m, l;
      split3(f32x4v{ra[i].x, ra[i].y, ra[i].z, ra[i].w}, h, m, l);
      *reinterpret_cast<bf16x4*>(&As[0][r][4 * q]) = h;
      *reinterpret_cast<bf16x4*>(&As[1][r][4 * q]) = m;
      *reinterpret_cast<bf16x4*>(&As[2][r][4 * q]) = l;
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
      bf16x4 h, m, l;
      split3(f32x4v{rb[i].x, rb[i].y, rb[i].z, rb[i].w}, h, m, l);
      *reinterpret_cast<bf16x4*>(&Bs[0][r][4 * q]) = h;
      *reinterpret_cast<bf16x4*>(&Bs[1][r][4 * q]) = m;
      *reinterpret_cast<bf16x4*>(&Bs[2][r][4 * q]) = l;
    }
  };
  f32x16 acc[TM][TN];
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int fi = wm * 64 + (lane & 31), fj = wn * 64 + (lane & 31), fk = 8 * (lane >> 5);
  constexpr int NS = BK / 16;   // MFMA k-steps per slab
  auto compute = [&]() {
    bf16x8 av[2][3][TM], bv[2][3][TN];
    auto rd = [&](int buf, int st) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int i = 0; i < TM; ++i) av[buf][p][i] = *reinterpret_cast<const bf16x8*>(&As[p][fi + 32 * i][16 * st + fk]);
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[buf][p][j] = *reinterpret_cast<const bf16x8*>(&Bs[p][fj + 32 * j][16 * st + fk]);
      }
    };
    rd(0, 0);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int pb = st & 1;
      if (st + 1 < NS) rd(pb ^ 1, st + 1);
      __builtin_amdgcn_sched_barrier(0);
      // smallest products first
      constexpr int NPR = NP;
      // (A piece, B piece): mid.lo, lo.mid | lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, then hi.hi below;
      // NP = 6 skips the first two
      const int pa[7] = {1, 2, 2, 0, 1, 1, 0}, pbb[7] = {2, 1, 0, 2, 1, 0, 1};
#pragma unroll
      for (int t = (NPR == 8 ? 0 : 2); t < 7; ++t) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[pb][pa[t]][i], bv[pb][pbb[t]][j], acc[i][j], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[pb][0][i], bv[pb][0][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const int nk = K / BK;
  load(0);
  store();
  if (nk > 1) load(BK);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    compute();
    __syncthreads();
    if (kt + 1 < nk) {
      store();
      if (kt + 2 < nk) load((kt + 2) * BK);
      __syncthreads();
    }
  }
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 64 + 32 * j + (lane & 31);
    for (int i = 0; i < TM; ++i)
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < M && n < N) C[(int64_t)m * N + n] = acc[i][j][r];
      }
  }
}

// debug: split a few values; one MFMA of lo pieces against ones
__global__ void k_dbg(const float* x, float* out) {
  const int lane = threadIdx.x;
  bf16x4 h, m, l;
  split3(f32x4v{x[4 * lane], x[4 * lane + 1], x[4 * lane + 2], x[4 * lane + 3]}, h, m, l);
  for (int j = 0; j < 4; ++j) {
    out[16 * lane + 4 * j + 0] = (float)h[j];
    out[16 * lane + 4 * j + 1] = (float)m[j];
    out[16 * lane + 4 * j + 2] = (float)l[j];
    out[16 * lane + 4 * j + 3] = x[4 * lane + j] - ((float)h[j] + (float)m[j] + (float)l[j]);
  }
  // MFMA: A = lo pieces (lane's 8 k values = its l[0..3] twice), B = ones
  bf16x8 a, b;
  for (int j = 0; j < 4; ++j) { a[j] = l[j]; a[4 + j] = l[j]; b[j] = (__bf16)1.0f; b[4 + j] = (__bf16)1.0f; }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  out[1024 + lane] = acc[0];
  // same with a large accumulator start
  for (int r = 0; r < 16; ++r) acc[r] = 1.0f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  out[1088 + lane] = acc[0] - 1.0f;
}

struct Err { double max_rel, rms_rel; };

static Err check(const std::vector<float>& hA, const std::vector<float>& hB, const std::vector<float>& hC, int M, int N,
                 int K) {
  double mx = 0, s2 = 0;
  const int S = 512;
  for (int t = 0; t < S; ++t) {
    const int m = (int)(((int64_t)t * 7919) % M), n = (int)(((int64_t)t * 104729 + t / 3) % N);
    double s = 0, sa = 0;
    for (int k = 0; k < K; ++k) {
      const double p = (double)hA[(size_t)m * K + k] * hB[(size_t)n * K + k];
      s += p;
      sa += fabs(p);
    }
    const double e = fabs(s - hC[(size_t)m * N + n]) / sa;
    mx = fmax(mx, e);
    s2 += e * e;
  }
  return {mx, sqrt(s2 / S)};
}

template <typename F>
static void timeit(const char* tag, F launch, float* C, const std::vector<float>& hA, const std::vector<float>& hB,
                   int M, int N, int K) {
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> hC((size_t)M * N);
  CK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
  const Err e = check(hA, hB, hC, M, N, K);
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
  printf("%-22s M=%5d N=%5d K=%5d %8.1f us %6.1f TF  err max %.2e rms %.2e (x 2^-24: %.2f / %.2f)\n", tag, M, N, K, us,
         2.0 * M * N * K / us / 1e6, e.max_rel, e.rms_rel, e.max_rel / 5.96e-8, e.rms_rel / 5.96e-8);
}

int main(int argc, char** argv) {
  if (argc > 1) {
    std::vector<float> hx(256);
    srand(3);
    for (auto& v : hx) v = ((float)rand() / RAND_MAX - 0.5f);
    float *x, *o;
    CK(hipMalloc(&x, 256 * 4));
    CK(hipMalloc(&o, 2048 * 4));
    CK(hipMemcpy(x, hx.data(), 256 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_dbg, dim3(1), dim3(64), 0, 0, x, o);
    std::vector<float> ho(2048);
    CK(hipMemcpy(ho.data(), o, 2048 * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; ++i)
      printf("x %.9g hi %.9g mid %.9g lo %.9g resid %.3g\n", hx[i], ho[4 * i], ho[4 * i + 1], ho[4 * i + 2], ho[4 * i + 3]);
    // lane 0 row 0: sum over k of A[0][k] = lanes 0 (k 0..7) and 32 (k 8..15)
    double ref = 0;
    for (int j = 0; j < 4; ++j) ref += 2.0 * ho[4 * j + 2] + 2.0 * ho[4 * (128 + j) / 1 + 2 - 0 * 4];
    printf("mfma lo sum lane0 %.9g (acc 1: %.9g)\n", ho[1024], ho[1088]);
    double r0 = 0;
    for (int j = 0; j < 4; ++j) r0 += 2.0 * ho[16 * 0 + 4 * j + 2] + 2.0 * ho[16 * 32 + 4 * j + 2];
    printf("expected %.9g\n", r0);
    return 0;
  }
  const int shapes[][3] = {{16384, 1024, 256}, {16384, 256, 1024}, {16384, 512, 512}, {4096, 4096, 4096}};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    std::vector<float> hA((size_t)M * K), hB((size_t)N * K);
    srand(1);
    // activations / gradients: mixed magnitudes (normal-ish times a log-uniform scale)
    for (auto& x : hA) x = ((float)rand() / RAND_MAX - 0.5f) * powf(2.f, (float)(rand() % 8) - 4.f);
    for (auto& x : hB) x = ((float)rand() / RAND_MAX - 0.5f) * 0.1f;
    float *A, *B, *C;
    CK(hipMalloc(&A, hA.size() * 4));
    CK(hipMalloc(&B, hB.size() * 4));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    dim3 grid(N / 128, M / 128);
    timeit("f32 mfma", [&] { hipLaunchKernelGGL(k_f32, grid, dim3(256), 0, 0, A, B, C, M, N, K); }, C, hA, hB, M, N, K);
    timeit("x6 bk32 pad8", [&] { hipLaunchKernelGGL((k_x6<6, 32, 8>), grid, dim3(256), 0, 0, A, B, C, M, N, K); }, C, hA, hB, M, N, K);
    timeit("x6 bk32 pad0", [&] { hipLaunchKernelGGL((k_x6<6, 32, 0>), grid, dim3(256), 0, 0, A, B, C, M, N, K); }, C, hA, hB, M, N, K);
    timeit("x6 bk64 pad8", [&] { hipLaunchKernelGGL((k_x6<6, 64, 8>), grid, dim3(256), 0, 0, A, B, C, M, N, K); }, C, hA, hB, M, N, K);
    timeit("x8 bk32 pad8", [&] { hipLaunchKernelGGL((k_x6<8, 32, 8>), grid, dim3(256), 0, 0, A, B, C, M, N, K); }, C, hA, hB, M, N, K);
    timeit("x8 bk64 pad8", [&] { hipLaunchKernelGGL((k_x6<8, 64, 8>), grid, dim3(256), 0, 0, A, B, C, M, N, K); }, C, hA, hB, M, N, K);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
  }
  return 0;
}
