// Decode-step GEMM body (dgemm.hip), shared with the fused head + sampling kernel of decode.hip.
// See dgemm.hip for the design.  A Hook adds work to the body: prefetch(m0, M) runs before the
// operand loads are issued, landed() once they have landed (the first workgroup barrier passed),
// value(row_in_tile, n, v) for every output element (also the discarded ones past M / N),
// finish(m0, M) after the epilogue.
#pragma once
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

// LDS floats of a dgemm_body launch: the A panel, the LayerNorm gains, the K-split partial tiles
__host__ __device__ __forceinline__ size_t dg_lds_floats(int MT, int NT, int KS, bool LN, int K) {
  return (size_t)16 * MT * (dg_kp(K) + 4) + (LN ? 512 : 0) + (size_t)(KS - 1) * (4 / KS) * MT * NT * 256;
}
// the 4-way K split for projections with K >= 768 over N <= 512 (16-row panels)
__host__ __device__ __forceinline__ bool dg_split_k(int N, int K) { return K >= 768 && N < 512; }

struct DgNoHook {
  __device__ __forceinline__ void prefetch(int, int) {}
  __device__ __forceinline__ void landed() {}
  __device__ __forceinline__ void value(int, int, float) {}
  __device__ __forceinline__ void finish(int, int) {}
};

// KS: waves per column group that split K (KS = 1: each of the 4 waves owns 16 NT columns over
// all of K; KS = 4: the 4 waves share 16 NT columns, each a quarter of the k steps, and their
// partial tiles meet in LDS, summed in wave order before the epilogue of wave 0).  A long-K,
// narrow-N projection over few live rows (FF2, the heads' last Linear) otherwise runs a 4x
// longer MFMA chain per wave on a quarter of the chip.
template <int MT, int NT, int KS, int EPI, bool LN, bool RES, class Hook>
__device__ __forceinline__ void dgemm_body(const DGemmArgs& a, float* As, Hook& hook) {
  constexpr int CG = 4 / KS;   // column groups per workgroup
  constexpr int BM = 16 * MT, BNW = 16 * NT, BN = CG * BNW, JB = DG_JB / NT;
  // (loading M together with the operands — rows clamped to the buffer, a workgroup past M exiting
  // after its loads — measured slower: the dead row panels' loads cost more than the round trip)
  const int M = a.m_dev ? *a.m_dev : a.M;
  const int m0 = blockIdx.y * BM, mlast = M - 1;
  if (m0 >= M) return;
  hook.prefetch(m0, M);
  const int K = a.K, Kp = dg_kp(K), LDA = Kp + 4, KQ = Kp >> 2, JN = KQ >> 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, q = lane >> 4;
  const int cg = w / KS, ks = w - cg * KS;
  const int n0 = blockIdx.x * BN + cg * BNW;
  // this wave's k steps [j_lo, j_hi) of the JN per lane quarter (JN >= KS: see dgemm_run)
  const int j_lo = ks * JN / KS, j_hi = (ks + 1) * JN / KS;

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
        const int jj = min(j_lo + blk * JB + j, j_hi - 1);   // (steps past the range: tail block, unused)
        b[nt][j] = *reinterpret_cast<const f32x4v*>(wp[nt] + 256 * jj);
      }
  };

  // ---- A panel: rows m0 .. m0 + BM - 1 (clamped to the last live row), 1 KiB pieces by LDS-DMA ----
  {
    const int pieces = (K + 255) >> 8;
    for (int p = w; p < BM * pieces; p += 4) {
      const int r = p / pieces, c = p - r * pieces;
      const int col = 256 * c + 4 * lane;
      const int mrow = min(m0 + r, mlast);
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
        const int m = min(m0 + 16 * mt + 4 * q + i, mlast);
        if constexpr (RES) resv[mt][nt][i] = a.R[(int64_t)m * a.ldr + n];
      }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(m0 + 16 * mt + 4 * q + i, mlast);
      dst[mt][i] = a.row_map ? (int64_t)a.row_map[m] : (int64_t)m;
      dst2[mt][i] = a.row_map2 ? (int64_t)a.row_map2[m] : (int64_t)m;
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  hook.landed();

  if constexpr (LN) {
    // x-transformers LayerNorm (ln_rms: RMSNorm) of columns [0, ln_k): mean, then the centred second moment.  TPR
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
    const float mean = a.ln_rms ? 0.f : sm / D;
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
    const float rstd = norm_rstd(qq, D, a.ln_rms);
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
  const int NJ = j_hi - j_lo, NBF = NJ / JB, JT = NJ - NBF * JB;
  for (int blk = 0; blk < NBF; ++blk) {
    const bool more = blk + 1 < NBF || JT > 0;
    if (more) load_b(bnext, blk + 1);
#pragma unroll
    for (int j = 0; j < JB; ++j) step(j_lo + blk * JB + j, bcur, j);
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
      if (j < JT) step(j_lo + NBF * JB + j, bcur, j);
  }
  if constexpr (KS > 1) {   // partial tiles of waves 1 .. KS-1 of each column group -> wave 0
    f32x4v* red = reinterpret_cast<f32x4v*>(As + BM * LDA + (LN ? 512 : 0));
    auto slot = [&](int k, int mt, int nt) { return ((cg * (KS - 1) + k - 1) * MT * NT + mt * NT + nt) * 64 + lane; };
    if (ks > 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) red[slot(ks, mt, nt)] = acc[mt][nt][0] + acc[mt][nt][1];
    }
    __syncthreads();
    if (ks == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          f32x4v v = acc[mt][nt][0] + acc[mt][nt][1];
          for (int k = 1; k < KS; ++k) v += red[slot(k, mt, nt)];
          acc[mt][nt][0] = v;
          acc[mt][nt][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
        }
    }
  }

  // ---- epilogue (wave 0 of each column group): element i of a tile is (row 4 q + i, column lr) ----
  if (ks == 0)
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
        hook.value(16 * mt + 4 * q + i, n, v);
      }
    }
  hook.finish(m0, M);
}


}  // namespace
}  // namespace xtrl
