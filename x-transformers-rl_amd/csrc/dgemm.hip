// Decode-step GEMM: the rollout's projections over the COMPACTED live rows of one timestep.
//
//   C[dst(m), n] = act( LN?(A)[m, :] . W[n, :] + bias[n] ) (+ R[m, n])      m < *m_dev
//
// The rollout's GEMMs are small (M <= E live rows, N <= 1024, K <= 1024) and latency bound: the
// cost of one launch is one workgroup's chain of load latency + MFMA + epilogue.  This kernel is
// built for that regime (replaces the per-step GEMM / LayerNorm launches of the round-1 decode):
//  * the workgroup's whole A panel (16 or 32 rows x K) is fetched in ONE round of LDS-DMA loads
//    (global_load_lds, 1 KiB row pieces, rows padded by 16 B so the fragment reads are
//    conflict-free), so there is one load latency per launch instead of one per K slab;
//  * an optional LayerNorm prologue normalises the first ln_k columns of the staged rows in LDS
//    (x-transformers LayerNorm: no affine, eps 1e-5, times gamma), all 256 threads at once (a
//    wave per row, one row after another, cost 11 us a launch: LDS and shuffle round trips) —
//    the pre-norms of q|k|v, FF1 and the heads cost no launch of their own;
//  * each wave owns 16*NT output columns and streams its weights straight into registers (16
//    float4 per lane per block, the next block in flight while the current one feeds the MFMAs):
//    weights are not shared between waves, so they skip LDS.  They are stored fragment-packed
//    (xtrl_dgemm_pack, once per rollout): every load instruction reads 1 KiB contiguous — in the
//    nn.Linear layout the 16 columns of a fragment sit in 16 rows, 64 cache lines per instruction
//    (FF2: 16.7 us a launch, L1-bound);
//  * v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation); lane (r = l & 15, q = l >> 4)
//    of every fragment covers the k quarter [q K/4, (q+1) K/4), float4 j of it feeding four
//    MFMAs — any k order sums every product once; two accumulator chains per tile hide the
//    40-cycle dependent MFMA latency;
//  * M is read from device memory (the live-row count the embedding kernel produced), so one
//    captured hipGraph serves every step: row tiles past the live count exit at once;
//  * epilogue: bias, GELU / SiLU, residual, a row scatter and a column split (the heads' last
//    Linear: actor logits to a row buffer, critic logits straight into the trajectory rows of their
//    episodes).
#include <algorithm>

#include "kernels.h"

namespace xtrl {

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ f32x4v mfma4(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int DG_JB = 16;   // float4 weight loads per lane per block (per column tile: 16 / NT)

// padded K (a multiple of 16: four lane quarters of whole float4s) and the LDS row stride
__host__ __device__ __forceinline__ int dg_kp(int K) { return (K + 15) & ~15; }

template <int MT, int NT, int EPI, bool LN, bool RES>
__global__ __launch_bounds__(256) void k_dgemm(const DGemmArgs a) {
  constexpr int BM = 16 * MT, BNW = 16 * NT, BN = 4 * BNW, JB = DG_JB / NT;
  extern __shared__ float As[];
  const int M = a.m_dev ? *a.m_dev : a.M;
  const int m0 = blockIdx.y * BM;
  if (m0 >= M) return;
  const int K = a.K, Kp = dg_kp(K), LDA = Kp + 4, KQ = Kp >> 2, JN = KQ >> 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * BN + w * BNW;

  // ---- weights of this wave: fragment-packed (xtrl_dgemm_pack), so one load instruction reads
  //      1 KiB contiguous — float4 slot ((n / 16 * JN + j) * 4 + q) * 16 + n % 16 holds
  //      W[n][q KQ + 4 j .. + 3], zero-padded past N and K ----
  const float* wp[NT];
  const int ntiles = (a.N + 15) >> 4;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int t16 = min((n0 >> 4) + nt, ntiles - 1);
    wp[nt] = a.W + ((int64_t)t16 * JN * 64 + lane) * 4;
  }
  f32x4v bcur[NT][JB], bnext[NT][JB];
  auto load_b = [&](f32x4v(&b)[NT][JB], int blk) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int jj = min(blk * JB + j, JN - 1);   // (steps past JN: tail block, unused)
        b[nt][j] = *reinterpret_cast<const f32x4v*>(wp[nt] + 256 * jj);
      }
  };

  // ---- A panel: rows m0 .. m0 + BM - 1 (clamped to the last live row), 1 KiB pieces by LDS-DMA ----
  {
    const int pieces = (K + 255) >> 8;
    for (int p = w; p < BM * pieces; p += 4) {
      const int r = p / pieces, c = p - r * pieces;
      const int col = 256 * c + 4 * lane;
      const int mrow = min(m0 + r, M - 1);
      if (col < K)
        __builtin_amdgcn_global_load_lds((const void*)(a.A + (int64_t)mrow * a.lda + col),
                                         (lds_void*)(As + r * LDA + 256 * c), 16, 0, 0);
    }
    if (K < Kp)   // zero the k padding (disjoint from the DMA destinations)
      for (int i = tid; i < BM * (Kp - K); i += 256) {
        const int r = i / (Kp - K), c = K + (i - r * (Kp - K));
        As[r * LDA + c] = 0.f;
      }
  }
  float* gsh = As + BM * LDA;   // LayerNorm gains [ln_k] (LDS-DMA, wave 0)
  if constexpr (LN) {
    if (w == 0)
      for (int c = 0; c < a.ln_k; c += 256)
        if (c + 4 * lane < a.ln_k)
          __builtin_amdgcn_global_load_lds((const void*)(a.gamma + c + 4 * lane), (lds_void*)(gsh + c), 16, 0, 0);
  }
  load_b(bcur, 0);
  // epilogue operands, prefetched with the panel (clamped, unconditional: see load_b): bias,
  // residual, destination rows
  float bias[NT], resv[MT][NT][4];
  int64_t dst[MT][4], dst2[MT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = min(n0 + 16 * nt + lr, a.N - 1);
    bias[nt] = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = min(m0 + 16 * mt + 4 * q + i, M - 1);
        if constexpr (RES) resv[mt][nt][i] = a.R[(int64_t)m * a.ldr + n];
      }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(m0 + 16 * mt + 4 * q + i, M - 1);
      dst[mt][i] = a.row_map ? (int64_t)a.row_map[m] : (int64_t)m;
      dst2[mt][i] = a.row_map2 ? (int64_t)a.row_map2[m] : (int64_t)m;
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if constexpr (LN) {
    // x-transformers LayerNorm of columns [0, ln_k): mean, then the centred second moment.  TPR
    // threads per row (all 256 threads at once), each holding float4s sub + TPR i of the row in
    // registers; butterflies over the TPR lanes of the row.
    constexpr int TPR = 256 / BM, MAXF = 128 / TPR;   // ln_k <= 512
    const int row = tid / TPR, sub = tid % TPR;
    f32x4v* xr = reinterpret_cast<f32x4v*>(As + row * LDA);
    const f32x4v* g4 = reinterpret_cast<const f32x4v*>(gsh);
    const int NF = a.ln_k >> 2;
    const float D = (float)a.ln_k;
    f32x4v v[MAXF];
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < MAXF; ++i) {
      const int f = sub + TPR * i;
      v[i] = xr[min(f, NF - 1)];
      if (f < NF) sm += ((v[i].x + v[i].y) + (v[i].z + v[i].w));
    }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) sm += __shfl_xor(sm, o, 64);
    const float mean = sm / D;
    float qq = 0.f;
#pragma unroll
    for (int i = 0; i < MAXF; ++i) {
      if (sub + TPR * i < NF) {
        const f32x4v dl = v[i] - mean;
        qq += ((dl.x * dl.x + dl.y * dl.y) + (dl.z * dl.z + dl.w * dl.w));
      }
    }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) qq += __shfl_xor(qq, o, 64);
    const float rstd = 1.0f / sqrtf(qq / D + 1e-5f);
#pragma unroll
    for (int i = 0; i < MAXF; ++i) {
      const int f = sub + TPR * i;
      if (f < NF) xr[f] = ((v[i] - mean) * rstd) * g4[f];
    }
    __syncthreads();
  }

  // ---- MFMA main loop ----
  f32x4v acc[MT][NT][2];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt][0] = acc[mt][nt][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
  const float* arow = As + lr * LDA + q * KQ;
  auto step = [&](int jj, const f32x4v(&b)[NT][JB], int j) {
    f32x4v av[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) av[mt] = *reinterpret_cast<const f32x4v*>(arow + mt * 16 * LDA + 4 * jj);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt][i & 1] = mfma4(av[mt][i], b[nt][j][i], acc[mt][nt][i & 1]);
  };
  // whole blocks of JB float4 steps (K a multiple of 16 JB / ... : no per-step condition), then
  // the tail block
  const int NBF = JN / JB, JT = JN - NBF * JB;
  for (int blk = 0; blk < NBF; ++blk) {
    const bool more = blk + 1 < NBF || JT > 0;
    if (more) load_b(bnext, blk + 1);
#pragma unroll
    for (int j = 0; j < JB; ++j) step(blk * JB + j, bcur, j);
    if (more) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int j = 0; j < JB; ++j) bcur[nt][j] = bnext[nt][j];
    }
  }
  if (JT > 0) {
#pragma unroll
    for (int j = 0; j < JB; ++j)
      if (j < JT) step(NBF * JB + j, bcur, j);
  }

  // ---- epilogue: element i of a tile is (row 4 q + i, column lr) ----
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + 16 * nt + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + 16 * mt + 4 * q + i;
        float v = (acc[mt][nt][0][i] + acc[mt][nt][1][i]) + bias[nt];
        if constexpr (EPI == EPI_GELU) v = geluf_(v);
        if constexpr (EPI == EPI_SILU) v = siluf_(v);
        if constexpr (EPI == EPI_RELU) v = fmaxf(v, 0.f);
        if constexpr (RES) v += resv[mt][nt][i];
        if (m < M && n < a.N) {
          if (n < a.n_split) a.C[dst[mt][i] * a.ldc + n] = v;
          else a.C2[dst2[mt][i] * a.ldc2 + (n - a.n_split)] = v;
        }
      }
    }
}

// fragment packing of an nn.Linear weight [N][K] (one thread per float4 slot)
__global__ void k_dg_pack(const float* W, int ldw, int N, int K, float* Wp) {
  const int Kp = dg_kp(K), JN = Kp >> 4, KQ = Kp >> 2;
  const int64_t slots = (int64_t)((N + 15) >> 4) * JN * 64;
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= slots) return;
  const int lr = (int)(s & 15), q = (int)((s >> 4) & 3);
  const int64_t rest = s >> 6;
  const int j = (int)(rest % JN), t16 = (int)(rest / JN);
  const int n = t16 * 16 + lr, k0 = q * KQ + 4 * j;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (n < N && k0 + i < K) ? W[(int64_t)n * ldw + k0 + i] : 0.f;
  reinterpret_cast<float4*>(Wp)[s] = make_float4(v[0], v[1], v[2], v[3]);
}

template <int MT, int NT, int EPI, bool LN, bool RES>
void launch_dg(const DGemmArgs& a, int rows, hipStream_t s) {
  constexpr int BM = 16 * MT, BN = 64 * NT;
  dim3 grid((a.N + BN - 1) / BN, (rows + BM - 1) / BM);
  const size_t lds = ((size_t)BM * (dg_kp(a.K) + 4) + (LN ? 512 : 0)) * sizeof(float);
  hipLaunchKernelGGL((k_dgemm<MT, NT, EPI, LN, RES>), grid, dim3(256), lds, s, a);
}

template <int EPI, bool LN, bool RES>
void dispatch_dg(const DGemmArgs& a, int rows, hipStream_t s) {
  // 32-row panels where N is wide and the panel stays small (FF1, the head hidden layer: twice
  // the weight reuse, half the workgroups); 16-row panels otherwise (long K, narrow N)
  const size_t lds32 = (size_t)32 * (dg_kp(a.K) + 4) * sizeof(float);
  if (a.N >= 512 && lds32 <= 80 * 1024) launch_dg<2, 1, EPI, LN, RES>(a, rows, s);
  else launch_dg<1, 1, EPI, LN, RES>(a, rows, s);
}

}  // namespace

int64_t dgemm_packed_floats(int N, int K) { return (int64_t)((N + 15) / 16) * 16 * dg_kp(K); }

int dgemm_pack(const float* W, int ldw, int N, int K, float* Wp, hipStream_t s) {
  XTRL_REQUIRE(W && Wp && N > 0 && K > 0 && ldw >= K, "dgemm_pack: bad arguments");
  const int64_t slots = dgemm_packed_floats(N, K) / 4;
  hipLaunchKernelGGL(k_dg_pack, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, W, ldw, N, K, Wp);
  XTRL_LAUNCHED("dgemm_pack");
  return XTRL_OK;
}

int dgemm_run(const DGemmArgs& a, int rows, int epi, hipStream_t s) {
  XTRL_REQUIRE(a.A && a.W && a.C && a.K > 0 && a.N > 0 && rows >= 0, "dgemm: bad operands");
  XTRL_REQUIRE(a.K % 4 == 0 && a.lda % 4 == 0 && ((uintptr_t)a.A & 15u) == 0 && ((uintptr_t)a.W & 15u) == 0,
               "dgemm: K, lda must be multiples of 4 and A, W 16-byte aligned (K=%d lda=%d)", a.K, a.lda);
  XTRL_REQUIRE(a.K <= 2048 && a.lda >= a.K && a.ldc >= std::min(a.N, a.n_split),
               "dgemm: bad K / leading dimensions");
  XTRL_REQUIRE(!a.gamma || (a.ln_k > 0 && a.ln_k <= a.K && a.ln_k <= 512), "dgemm: bad LayerNorm width (<= 512)");
  XTRL_REQUIRE(epi == EPI_NONE || epi == EPI_GELU || epi == EPI_SILU || epi == EPI_RELU,
               "dgemm: epilogue %d unsupported", epi);
  XTRL_REQUIRE(a.n_split >= a.N || (a.C2 && a.n_split >= 0 && a.ldc2 >= a.N - a.n_split), "dgemm: bad column split");
  if (rows == 0) return XTRL_OK;
  const bool ln = a.gamma != nullptr, res = a.R != nullptr;
#define XTRL_DG(E)                                                                                \
  do {                                                                                            \
    if (ln && res) dispatch_dg<E, true, true>(a, rows, s);                                        \
    else if (ln) dispatch_dg<E, true, false>(a, rows, s);                                         \
    else if (res) dispatch_dg<E, false, true>(a, rows, s);                                        \
    else dispatch_dg<E, false, false>(a, rows, s);                                                \
  } while (0)
  if (epi == EPI_GELU) XTRL_DG(EPI_GELU);
  else if (epi == EPI_SILU) XTRL_DG(EPI_SILU);
  else if (epi == EPI_RELU) {
    XTRL_REQUIRE(!ln && !res, "dgemm: the ReLU epilogue has no LayerNorm / residual variant");
    dispatch_dg<EPI_RELU, false, false>(a, rows, s);
  }
  else XTRL_DG(EPI_NONE);
#undef XTRL_DG
  XTRL_LAUNCHED("dgemm");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int64_t xtrl_dgemm_packed_floats(int N, int K) { return xtrl::dgemm_packed_floats(N, K); }
extern "C" int xtrl_dgemm_pack(const float* W, int ldw, int N, int K, float* Wp, void* stream) {
  return xtrl::dgemm_pack(W, ldw, N, K, Wp, xtrl::as_stream(stream));
}
extern "C" int xtrl_dgemm(const float* A, int lda, const float* Wp, const float* bias, const float* ln_gamma, int ln_k,
                          const float* R, int ldr, float* C, int ldc, const int32_t* row_map, const int32_t* m_dev,
                          int M, int N, int K, int act, void* stream) {
  xtrl::DGemmArgs a;
  a.A = A; a.lda = lda; a.W = Wp; a.ldw = xtrl::dgemm_packed_floats(1, K) / 16; a.bias = bias; a.gamma = ln_gamma; a.ln_k = ln_k;
  a.R = R; a.ldr = ldr; a.C = C; a.ldc = ldc; a.row_map = row_map; a.m_dev = m_dev; a.M = M; a.N = N; a.K = K;
  return xtrl::dgemm_run(a, M, act == 3 ? xtrl::EPI_RELU : act, xtrl::as_stream(stream));
}
