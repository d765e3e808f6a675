// Fused fp32 GEMM on the CDNA4 f32 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 products,
// 64 cycles / instruction / SIMD, dependent-accumulator latency 64 -> one accumulator chain per
// wave runs at the issue rate).
//
//   C[m, n] = act( LN?(A)[m, :] . B[:, n] + bias[n] ) (+ R[m, n])          (fp32 in, fp32 out)
//
// Operand layouts (so one kernel serves forward, dgrad and wgrad of nn.Linear):
//   A "N": A[m][k] at a[m * lda + k]       A "T": A[m][k] at a[k * lda + m]
//   B "N": B[k][n] at b[n * ldb + k]  (nn.Linear weight [out][in])
//   B "T": B[k][n] at b[k * ldb + n]
//
// Geometry: WM x WN x WK waves; each wave owns a 32 x 32 output tile and a 32-deep share of every
// K-slab (so WK > 1 splits K inside the workgroup; partial tiles are summed through LDS in fixed
// order — deterministic).  Block tile (32 WM) x (32 WN), K-slab 32 WK.  Slabs are staged
// global -> registers (float4, coalesced along the contiguous dimension) -> LDS in k-major images
// [k][m + 1] / [k][n + 1] (the +1 pad keeps the MFMA fragment reads — 32 consecutive dwords per
// half-wave — conflict-free); the next slab's global loads are issued before the current slab's
// MFMAs (register double buffering, one barrier per slab).
//
// X6 (split-bf16 products, the large-tile geometry): every staged fp32 operand x is split into
// three bf16 pieces x = hi + mid + lo (each the round-to-nearest bf16 of the running remainder;
// the subtractions are exact and the three pieces hold all 24 significand bits) and the product is
// the sum of the six largest piece products lo.hi + hi.lo + mid.mid + mid.hi + hi.mid + hi.hi on
// the bf16 matrix cores (v_mfma_f32_32x32x16_bf16, fp32 accumulate, 6 x 32 cycles per 32x32x16
// step vs 8 x 64 for v_mfma_f32_32x32x2_f32).  The dropped terms (mid.lo, lo.mid, lo.lo) are
// below 2^-24 of each product: measured error vs fp64 equals the native f32 path's
// (tools/x6_lab.hip: rms 0.51-0.57 vs 0.58-0.69 x 2^-24 of sum |a b|, K = 256 ... 4096).
// XTRL_GEMM_F32=1 selects the native f32 MFMA path everywhere (A/B experiments).
//
// The optional LayerNorm prologue (x-transformers LayerNorm: no affine, eps 1e-5, times gamma;
// A "N" only) computes per-row mean / rstd for the block's rows (two-pass) and normalises A while
// staging it.
#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "philox.h"
#include "x6.h"

namespace xtrl {

namespace {

__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
__device__ __forceinline__ float f4c(const float4& v, int k) {
  return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

// the row-vector epilogue applies when every row segment it reads or writes is a 16-byte aligned float4
template <int EPI, bool RES>
__device__ __forceinline__ bool epi_v4_ok(const GemmArgs& a, const float* C) {
  constexpr bool AUX1 = (EPI == EPI_MUL_AUX || EPI == EPI_DGATE || EPI == EPI_MASK_POS), AUX2 = (EPI == EPI_DGATE);
  constexpr bool AOUT = (EPI == EPI_GELU_DROP || EPI == EPI_SILU_SAVE || EPI == EPI_DGATE);
  bool ok = (a.N & 3) == 0 && (a.ldc & 3) == 0 && al16(C);
  if constexpr (RES) ok = ok && (a.ldr & 3) == 0 && al16(a.R);
  if constexpr (AUX1) ok = ok && (a.ld_aux_in & 3) == 0 && al16(a.aux_in);
  if constexpr (AUX2) ok = ok && (a.ld_aux_in2 & 3) == 0 && al16(a.aux_in2);
  if constexpr (AOUT) ok = ok && (a.ld_aux_out & 3) == 0 && al16(a.aux_out);
  return ok;
}

// FF dropout keep bits in byte mode (GemmArgs::drop_thresh8, p a multiple of 1/256): element (m, n)
// keeps iff byte (m & 3) of word ((m >> 3) & 3) of philox(seed; n, 2 (m >> 5) + ((m >> 2) & 1),
// drop_off, FIELD_FF_DROPOUT sub 2 layer + 1) is >= drop_thresh8 — the 16 rows of a 32-row MFMA tile one lane
// holds (mb + 8 g + q, mb = 32-aligned base + 4 (lane >> 5)) share one block.  k_ff_mask (train.hip)
// draws the same bits.
__device__ __forceinline__ u32x4_t ff_block8(const GemmArgs& a, int n, int mb) {
  return philox4x32_10((uint32_t)n, (uint32_t)(((mb >> 5) << 1) | ((mb >> 2) & 1)), a.drop_off,
                       rng_c3(FIELD_FF_DROPOUT, 2 * a.drop_layer + 1), a.seed);
}
// the four bytes of word g (rows mb + 8 g + 0..3) as four "words" compared against drop_thresh8
__device__ __forceinline__ u32x4_t ff_bytes8(const u32x4_t& kb, int g) {
  const uint32_t w = g == 0 ? kb.x : (g == 1 ? kb.y : (g == 2 ? kb.z : kb.w));
  return {w & 0xFFu, (w >> 8) & 0xFFu, (w >> 16) & 0xFFu, w >> 24};
}

// torch's GELU (erf form) and its derivative with ONE exponential: erf from Abramowitz & Stegun
// 7.1.26 (|error| < 1.5e-7; with z = |x| / sqrt 2 its exp(-z^2) is the Gaussian pdf's exp(-x^2 / 2)),
// the CDF formed without cancellation on either side (1 - h or h): max |error| vs the exact GELU
// 4.2e-7 on [-12, 12], as torch's fp32 erf form (4.5e-7); 24 vector instructions instead of the
// library erff + expf (the FF1 epilogue was vector-issue bound: tools/epi_pmc.sh)
__device__ __forceinline__ void gelu_fwd_deriv(float x, float& g, float& dg) {
  const float E = __expf(-0.5f * x * x);
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  const float h = 0.5f * poly * E;
  const float cdf = x >= 0.f ? 1.0f - h : h;
  g = x * cdf;
  dg = fmaf(x, 0.3989422804014327f * E, cdf);
}

// Row-vector epilogue.  The element-wise stage that reads no operand (bias, activation, dropout,
// saved derivative) runs in the MFMA layout — one Philox block still covers a column's four rows —
// then a quad transpose gives every lane four consecutive columns of one row, so the operand reads
// (saved derivative, gate, residual, old C) and the stores are float4: 4 store instructions per
// 32 x 32 tile and output instead of 16 (the scalar tail was store-issue bound).  Per element the
// same operations in the same order as the scalar form below.
template <int TM, int TN, int EPI, bool RES>
__device__ __forceinline__ void gemm_epilogue_v4(const GemmArgs& a, f32x16 (&acc)[TM][TN], float* C, int m0, int n0,
                                                 int wm, int wn, int lane) {
  const int M = a.M, N = a.N;
  const bool acc_c = a.beta != 0.f;
  constexpr bool DROP = (EPI == EPI_GELU_DROP);
  constexpr bool SAVE = (EPI == EPI_GELU_DROP || EPI == EPI_SILU_SAVE);
  constexpr bool AUX1 = (EPI == EPI_MUL_AUX || EPI == EPI_DGATE || EPI == EPI_MASK_POS), AUX2 = (EPI == EPI_DGATE);
  const int c4 = lane & 3;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 32 * TN + 32 * j + (lane & 31);              // MFMA layout column
    const int nv = n0 + wn * 32 * TN + 32 * j + 4 * ((lane & 31) >> 2);  // row-vector first column
    const int nvc = nv < N ? nv : N - 4;
    const bool nok = n < N;
    const float bn = (a.bias && nok && n >= a.bias_col0) ? a.bias[n - a.bias_col0] : 0.f;
    const bool act = n < a.act_cols;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = m0 + wm * 32 * TM + 32 * i + 4 * (lane >> 5);
      float v[4][4], ax[4][4];
      // byte-mode keep bits (drop_thresh8): ONE Philox block covers this lane's 16 rows of column n
      const u32x4_t kb = (DROP && a.drop_thresh8) ? ff_block8(a, n, mb) : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x4_t kw{0u, 0u, 0u, 0u};
        if (DROP && a.drop_thresh && !a.drop_thresh8)
          kw = philox4x32_10((uint32_t)n, (uint32_t)((mb + 8 * g) >> 2), a.drop_off, rng_c3(FIELD_FF_DROPOUT, 2 * a.drop_layer),
                             a.seed);
        else if (DROP && a.drop_thresh8)
          kw = ff_bytes8(kb, g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float x = acc[i][j][4 * g + q] + bn;
          float aux_o = 0.f;
          const uint32_t word = q == 0 ? kw.x : (q == 1 ? kw.y : (q == 2 ? kw.z : kw.w));
          if constexpr (EPI == EPI_GELU) x = geluf_(x);
          if constexpr (EPI == EPI_SILU) x = siluf_(x);
          if constexpr (EPI == EPI_RELU) x = fmaxf(x, 0.f);
          if constexpr (EPI == EPI_GELU_DROP) {   // torch GELU (erf) and GeluBackward's factor
            gelu_fwd_deriv(x, x, aux_o);
            if (a.drop_thresh) {
              const bool keep = a.drop_thresh8 ? word >= a.drop_thresh8 : word >= a.drop_thresh;
              x = keep ? x * a.inv_keep : 0.f;
              aux_o = keep ? aux_o * a.inv_keep : 0.f;
            }
          }
          if constexpr (EPI == EPI_SILU_SAVE) {
            if (act) {
              const float sg = 1.0f / (1.0f + expf(-x));
              aux_o = sg * (1.0f + x * (1.0f - sg));
              x = x / (1.0f + expf(-x));
            } else {
              aux_o = 1.0f;
            }
          }
          v[g][q] = x;
          ax[g][q] = aux_o;
        }
        quad_transpose(v[g], lane);
        if constexpr (SAVE) quad_transpose(ax[g], lane);
      }
      // row-vector stage: this lane holds row mb + 8 g + (lane & 3), columns nv .. nv + 3; every
      // operand read comes before the stores (which may alias them as far as the compiler knows)
      float4 x1[4], x2[4], rr[4], old[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = mb + 8 * g + c4, mc = m < M ? m : M - 1;
        if constexpr (AUX1) x1[g] = *reinterpret_cast<const float4*>(a.aux_in + (int64_t)mc * a.ld_aux_in + nvc);
        if constexpr (AUX2) x2[g] = *reinterpret_cast<const float4*>(a.aux_in2 + (int64_t)mc * a.ld_aux_in2 + nvc);
        if constexpr (RES) rr[g] = *reinterpret_cast<const float4*>(a.R + (int64_t)mc * a.ldr + nvc);
        old[g] = acc_c ? *reinterpret_cast<const float4*>(C + (int64_t)mc * a.ldc + nvc)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = mb + 8 * g + c4;
        float o[4], ao[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float x = v[g][k];
          float aux_o = SAVE ? ax[g][k] : 0.f;
          if constexpr (EPI == EPI_MUL_AUX) x = x * f4c(x1[g], k);
          if constexpr (EPI == EPI_MASK_POS) x = f4c(x1[g], k) > 0.f ? x : 0.f;
          if constexpr (EPI == EPI_DGATE) {
            const float sg = sigmoidf_(f4c(x2[g], k));
            aux_o = (x * f4c(x1[g], k)) * (1.0f - sg) * sg;
            x = x * sg;
          }
          if constexpr (RES) x = x + f4c(rr[g], k);
          if (acc_c) x = a.beta * f4c(old[g], k) + x;
          o[k] = x;
          ao[k] = aux_o;
        }
        if (m < M && nv < N && (!a.row_mask || a.row_mask[m])) {
          *reinterpret_cast<float4*>(C + (int64_t)m * a.ldc + nv) = make_float4(o[0], o[1], o[2], o[3]);
          if constexpr (SAVE || EPI == EPI_DGATE)
            *reinterpret_cast<float4*>(a.aux_out + (int64_t)m * a.ld_aux_out + nv) =
                make_float4(ao[0], ao[1], ao[2], ao[3]);
        }
      }
    }
  }
}

// scalar epilogue: acc[r] -> row (r & 3) + 8 (r >> 2) + 4 (lane >> 5), col lane & 31 of the wave's 32 x 32
// tile (i, j); bias / activation / saved derivative / gate / residual / beta, then the stores
// V4ONLY: the launch guarantees the row-vector form (epi_v4_host): the scalar form is not compiled
// in (for the split-bf16 GELU + dropout kernels it cost 46 spilled registers)
template <int TM, int TN, int EPI, bool RES, bool V4ONLY = false>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, f32x16 (&acc)[TM][TN], int m0, int n0, int wm,
                                              int wn, int lane, int bz) {
  const int M = a.M, N = a.N;
  float* C = a.C;
  if (a.t_dev) C += (int64_t)(*a.t_dev) * a.c_t_stride;
  if (a.kspan > 0) C += bz * a.c_split;
  if (V4ONLY || epi_v4_ok<EPI, RES>(a, C)) {
    gemm_epilogue_v4<TM, TN, EPI, RES>(a, acc, C, m0, n0, wm, wn, lane);
    return;
  }
  const bool acc_c = a.beta != 0.f;
  constexpr bool DROP = (EPI == EPI_GELU_DROP);
  constexpr bool AUX1 = (EPI == EPI_MUL_AUX || EPI == EPI_DGATE || EPI == EPI_MASK_POS);
  constexpr bool AUX2 = (EPI == EPI_DGATE);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * 32 * TN + 32 * j + (lane & 31);
    const bool nok = n < N;
    const int nc = nok ? n : N - 1;
    const float bn = (a.bias && nok && n >= a.bias_col0) ? a.bias[n - a.bias_col0] : 0.f;
    const bool act = n < a.act_cols;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = m0 + wm * 32 * TM + 32 * i + 4 * (lane >> 5);
      // all reads of this lane's 16 elements first (aux inputs, residual, old C): the stores below
      // may alias them as far as the compiler knows, so interleaving would serialise every access
      float x1[16], x2[16], rr[16], old[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2);
        const int mc = m < M ? m : M - 1;
        if constexpr (AUX1) x1[r] = a.aux_in[(int64_t)mc * a.ld_aux_in + nc];
        if constexpr (AUX2) x2[r] = a.aux_in2[(int64_t)mc * a.ld_aux_in2 + nc];
        if constexpr (RES) rr[r] = a.R[(int64_t)mc * a.ldr + nc];
        old[r] = acc_c ? C[(int64_t)mc * a.ldc + nc] : 0.f;
      }
      const u32x4_t kb = (DROP && a.drop_thresh8) ? ff_block8(a, n, mb) : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // rows mb + 8g + 0..3 (a 4-aligned group): one Philox block gives their four keep words
        // (byte mode: the lane's one block gives all 16)
        u32x4_t kw{0u, 0u, 0u, 0u};
        if (DROP && a.drop_thresh && !a.drop_thresh8)
          kw = philox4x32_10((uint32_t)n, (uint32_t)((mb + 8 * g) >> 2), a.drop_off, rng_c3(FIELD_FF_DROPOUT, 2 * a.drop_layer),
                             a.seed);
        else if (DROP && a.drop_thresh8)
          kw = ff_bytes8(kb, g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 4 * g + q;
          const int m = mb + 8 * g + q;
          float v = acc[i][j][r] + bn;
          const uint32_t word = q == 0 ? kw.x : (q == 1 ? kw.y : (q == 2 ? kw.z : kw.w));
          float aux_o = 0.f;
          if constexpr (EPI == EPI_GELU) v = geluf_(v);
          if constexpr (EPI == EPI_SILU) v = siluf_(v);
          if constexpr (EPI == EPI_RELU) v = fmaxf(v, 0.f);
          if constexpr (EPI == EPI_GELU_DROP) {   // torch GELU (erf) and GeluBackward's factor
            gelu_fwd_deriv(v, v, aux_o);
            if (a.drop_thresh) {
              const bool keep = a.drop_thresh8 ? word >= a.drop_thresh8 : word >= a.drop_thresh;
              v = keep ? v * a.inv_keep : 0.f;
              aux_o = keep ? aux_o * a.inv_keep : 0.f;
            }
          }
          if constexpr (EPI == EPI_SILU_SAVE) {
            if (act) {
              const float sg = 1.0f / (1.0f + expf(-v));
              aux_o = sg * (1.0f + v * (1.0f - sg));
              v = v / (1.0f + expf(-v));
            } else {
              aux_o = 1.0f;
            }
          }
          if constexpr (EPI == EPI_MUL_AUX) v = v * x1[r];
          if constexpr (EPI == EPI_MASK_POS) v = x1[r] > 0.f ? v : 0.f;
          if constexpr (EPI == EPI_DGATE) {
            const float sg = sigmoidf_(x2[r]);
            aux_o = (v * x1[r]) * (1.0f - sg) * sg;
            v = v * sg;
          }
          if constexpr (RES) v = v + rr[r];
          if (acc_c) v = a.beta * old[r] + v;
          if (nok && m < M && (!a.row_mask || a.row_mask[m])) {
            C[(int64_t)m * a.ldc + n] = v;
            if constexpr (EPI == EPI_GELU_DROP || EPI == EPI_SILU_SAVE || EPI == EPI_DGATE)
              a.aux_out[(int64_t)m * a.ld_aux_out + n] = aux_o;
          }
        }
      }
    }
  }
}

template <int WM, int WN, int WK, int TM, int TN, bool TA, bool TB, int EPI, bool LN, bool RES, bool VEC,
          bool X6 = false>
__global__ __launch_bounds__(64 * WM * WN * WK, (X6 && EPI != EPI_DGATE) ? 2 : 1) void k_gemm(const GemmArgs a) {
  constexpr int BM = 32 * WM * TM, BN = 32 * WN * TN, BK = 32 * WK, NT = 64 * WM * WN * WK;
  // X6 images: [piece][row][k] bf16, rows padded to XRS = BK + 8 (conflict-light 16-byte reads)
  constexpr int XRS = BK + 8;
  static_assert(!X6 || (WK == 1 && VEC && (!TA || BM * BK % (16 * NT) == 0) && (!TB || BN * BK % (16 * NT) == 0)),
                "X6: one wave along K, vector staging, whole 4 x 4 transposed groups");
  // k-major LDS images [buf][k][m]: +1 pad ("N", transposed scalar staging writes), +4 (16-byte
  // rows, "T").  SWZ (kept for experiments, off): row stride = 32 mod 64 banks so the two
  // half-waves of a fragment read (rows k, k+1) use disjoint banks, plus an XOR-by-8 column
  // swizzle for conflict-free transposed writes.  Isolated TT GEMM at 4096^3 +22 %, but the C3
  // update measured 2 % slower with it (tools/gemm_lab.hip, A/B bench), so it is disabled.
  constexpr bool SWZ = false && (WK == 1 && BM >= 64 && BN >= 64);
  constexpr int AST = SWZ ? BM + 32 : (TA ? BM + 4 : BM + 1), BST = SWZ ? BN + 32 : (TB ? BN + 4 : BN + 1);
  constexpr int A_F4 = BM * BK / 4 / NT, B_F4 = BN * BK / 4 / NT;   // float4 loads per thread per slab
  static_assert(A_F4 >= 1 && B_F4 >= 1, "tile too small for the thread count");
  // ONE LDS stage (the next slab waits in registers; see the main loop): one static block
  constexpr int STAGE = X6 ? 3 * (BM + BN) * XRS / 2 : BK * AST + BK * BST;   // floats
  constexpr int SMEM = STAGE + (LN ? 2 * BM : 0);
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float(*As)[BK][AST] = reinterpret_cast<float(*)[BK][AST]>(smem);
  float(*Bs)[BK][BST] = reinterpret_cast<float(*)[BK][BST]>(smem + BK * AST);
  __bf16(*Xa)[BM][XRS] = reinterpret_cast<__bf16(*)[BM][XRS]>(smem);
  __bf16(*Xb)[BN][XRS] = reinterpret_cast<__bf16(*)[BN][XRS]>(reinterpret_cast<__bf16*>(smem) + 3 * BM * XRS);
  float* row_mean = smem + STAGE;
  float* row_rstd = row_mean + BM;
  auto sw = [](int k, int m) { return SWZ ? (m ^ (8 * ((k >> 2) & 7))) : m; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (WM * WN), wmn = wave % (WM * WN), wm = wmn / WN, wn = wmn % WN;
  // workgroup -> (column tile, row tile, K split).  The hardware deals workgroups to the 8 XCDs
  // round-robin by linear id; with xcd_remap the ids are permuted so each XCD runs a contiguous
  // range of logical tiles (column tile fastest): the column tiles of a row tile — which all read
  // the same A rows — then share that XCD's L2 instead of fetching A once per XCD
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (a.xcd_remap) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int total = nx * ny * gridDim.z;
    const int lin = bx + nx * (by + ny * bz);
    const int lg = (lin & 7) * (total >> 3) + (lin >> 3);
    bx = lg % nx;
    by = (lg / nx) % ny;
    bz = lg / (nx * ny);
  }
  const int m0 = by * BM, n0 = bx * BN;
  const int M = a.M, N = a.N;
  int K = a.K;
  const float* __restrict__ Ab = a.A;
  const float* __restrict__ Bb = a.B;
  if (a.kspan > 0) {   // cross-workgroup split of K: shift the operands to this split's K range
    const int kb = bz * a.kspan;
    K = min(a.kspan, a.K - kb);
    Ab += TA ? (int64_t)kb * a.lda : kb;
    Bb += TB ? (int64_t)kb * a.ldb : kb;
  }

  if constexpr (LN) {
    // per-row mean / rstd of the block's rows: each wave takes 4 rows at a time with all their
    // loads in flight (row held in registers, two-pass variance); K <= 1024 on the VEC path
    constexpr int NW = WM * WN * WK, RB = 4;
    if (VEC && K <= 1024) {
      for (int r0 = wave * RB; r0 < BM; r0 += NW * RB) {
        float4 v[RB][4];
        float s[RB];
#pragma unroll
        for (int q = 0; q < RB; ++q) {
          const int m = m0 + r0 + q;
          const float* xr = a.A + (int64_t)min(m, M - 1) * a.lda;
          s[q] = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = 4 * (lane + 64 * j);
            v[q][j] = (m < M && c < K) ? *reinterpret_cast<const float4*>(xr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            s[q] += (v[q][j].x + v[q][j].y) + (v[q][j].z + v[q][j].w);
          }
        }
#pragma unroll
        for (int q = 0; q < RB; ++q) {
          const float mean = a.ln_rms ? 0.f : wave_sum(s[q]) / (float)K;
          float sq = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (4 * (lane + 64 * j) < K) {
              const float4 x = v[q][j];
              sq += ((x.x - mean) * (x.x - mean) + (x.y - mean) * (x.y - mean)) +
                    ((x.z - mean) * (x.z - mean) + (x.w - mean) * (x.w - mean));
            }
          }
          const float rstd = norm_rstd(wave_sum(sq), (float)K, a.ln_rms);
          if (lane == 0 && r0 + q < BM) {
            row_mean[r0 + q] = mean;
            row_rstd[r0 + q] = rstd;
          }
        }
      }
    } else {
      for (int r = wave; r < BM; r += NW) {
        const int m = m0 + r;
        float mean = 0.f, rstd = 0.f;
        if (m < M) {
          const float* xr = a.A + (int64_t)m * a.lda;
          float s = 0.f;
          for (int k = lane; k < K; k += 64) s += xr[k];
          mean = a.ln_rms ? 0.f : wave_sum(s) / (float)K;
          float q = 0.f;
          for (int k = lane; k < K; k += 64) {
            const float dlt = xr[k] - mean;
            q += dlt * dlt;
          }
          rstd = norm_rstd(wave_sum(q), (float)K, a.ln_rms);
        }
        if (lane == 0) {
          row_mean[r] = mean;
          row_rstd[r] = rstd;
        }
      }
    }
    __syncthreads();
  }

  // staging registers (one slab; the buffer index P is a compile-time constant)
  float4 ra[1][A_F4], rb[1][B_F4];
  using I0 = std::integral_constant<int, 0>;
  // Branch-free staging loads.  Indices are clamped into the operand, so every load is in bounds;
  // rows / columns past M or N then hold duplicates that only feed output rows / columns the
  // epilogue discards, and only the reduction index k needs zeroing past K — which can only happen
  // in the last slab (TAIL, a workgroup-uniform branch).  Keeping selects out of the interior slabs
  // lets the next slab's loads stay in flight across the current slab's MFMAs.  VEC requires the
  // contiguous extent to be a multiple of 4, so a quad is all-in or all-out.
  auto load4 = [&](const float* base, int64_t ld, int outer, int inner, int outer_lim, int inner_lim,
                   bool outer_is_k, bool tail) -> float4 {
    const float* row = base + (int64_t)min(outer, outer_lim - 1) * ld;
    float4 f;
    if constexpr (VEC) {
      // quads are clamped into the row's 4-aligned extent (the leading dimension covers it, see
      // gemm_run): a quad straddling the end of the contiguous extent reads in-bounds padding,
      // zeroed by the tail mask when that extent is K and discarded by the epilogue otherwise
      f = *reinterpret_cast<const float4*>(row + min(inner, ((inner_lim + 3) & ~3) - 4));
    } else {
      f.x = row[min(inner + 0, inner_lim - 1)];
      f.y = row[min(inner + 1, inner_lim - 1)];
      f.z = row[min(inner + 2, inner_lim - 1)];
      f.w = row[min(inner + 3, inner_lim - 1)];
    }
    if (tail) {
      if (outer_is_k) {
        const bool ok = outer < outer_lim;
        f = make_float4(ok ? f.x : 0.f, ok ? f.y : 0.f, ok ? f.z : 0.f, ok ? f.w : 0.f);
      } else {
        f.x = inner + 0 < inner_lim ? f.x : 0.f;
        f.y = inner + 1 < inner_lim ? f.y : 0.f;
        f.z = inner + 2 < inner_lim ? f.z : 0.f;
        f.w = inner + 3 < inner_lim ? f.w : 0.f;
      }
    }
    return f;
  };
  auto load_slab = [&](auto P, int k0, bool tail) {
    float4(&RA)[A_F4] = ra[decltype(P)::value];
    float4(&RB)[B_F4] = rb[decltype(P)::value];
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int e = tid + i * NT;
      if constexpr (!TA) {   // [BM rows][BK/4 quads]
        const int r = e / (BK / 4), q = e % (BK / 4);
        float4 f = load4(Ab, a.lda, m0 + r, k0 + 4 * q, M, K, false, tail);
        if constexpr (LN) {
          const float mu = row_mean[r], rs = row_rstd[r];
          const int k = k0 + 4 * q;
          f.x = ((f.x - mu) * rs) * a.gamma[min(k + 0, K - 1)];
          f.y = ((f.y - mu) * rs) * a.gamma[min(k + 1, K - 1)];
          f.z = ((f.z - mu) * rs) * a.gamma[min(k + 2, K - 1)];
          f.w = ((f.w - mu) * rs) * a.gamma[min(k + 3, K - 1)];
          if (tail) {
            f.x = k + 0 < K ? f.x : 0.f;
            f.y = k + 1 < K ? f.y : 0.f;
            f.z = k + 2 < K ? f.z : 0.f;
            f.w = k + 3 < K ? f.w : 0.f;
          }
        }
        RA[i] = f;
      } else if constexpr (X6) {   // 4 x 4 groups: k rows 4 kq .. 4 kq + 3 of m quad q (kq fastest
                                   // over lanes: conflict-free transposed LDS writes)
        const int g = tid + (i >> 2) * NT, kq = g % (BK / 4), q = g / (BK / 4);
        RA[i] = load4(Ab, a.lda, k0 + 4 * kq + (i & 3), m0 + 4 * q, K, M, true, tail);
      } else {               // [BK rows][BM/4 quads]
        const int r = e / (BM / 4), q = e % (BM / 4);
        RA[i] = load4(Ab, a.lda, k0 + r, m0 + 4 * q, K, M, true, tail);
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int e = tid + i * NT;
      if constexpr (!TB) {
        const int r = e / (BK / 4), q = e % (BK / 4);
        RB[i] = load4(Bb, a.ldb, n0 + r, k0 + 4 * q, N, K, false, tail);
      } else if constexpr (X6) {
        const int g = tid + (i >> 2) * NT, kq = g % (BK / 4), q = g / (BK / 4);
        RB[i] = load4(Bb, a.ldb, k0 + 4 * kq + (i & 3), n0 + 4 * q, K, N, true, tail);
      } else {
        const int r = e / (BN / 4), q = e % (BN / 4);
        RB[i] = load4(Bb, a.ldb, k0 + r, n0 + 4 * q, K, N, true, tail);
      }
    }
  };
  // X6 staging: split each row's 4 consecutive k values into the three piece images
  auto store_slab_x6 = [&](auto P) {
    const float4(&RA)[A_F4] = ra[decltype(P)::value];
    const float4(&RB)[B_F4] = rb[decltype(P)::value];
    __bf16* xa = &Xa[0][0][0];
    __bf16* xb = &Xb[0][0][0];
    auto put = [&](__bf16* img, int rows, int row, int k, float4 v) {
      bf16x4 h, m, l;
      split3(v, h, m, l);
      __bf16* p = img + row * XRS + k;
      *reinterpret_cast<bf16x4*>(p) = h;
      *reinterpret_cast<bf16x4*>(p + rows * XRS) = m;
      *reinterpret_cast<bf16x4*>(p + 2 * rows * XRS) = l;
    };
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      if constexpr (!TA) {
        const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
        put(xa, BM, r, 4 * q, RA[i]);
      } else if ((i & 3) == 3) {   // transpose the 4 x 4 group: row m = 4 q + c gets k 4 kq .. 4 kq + 3
        const int g = tid + (i >> 2) * NT, kq = g % (BK / 4), q = g / (BK / 4);
        const float4 k0v = RA[i - 3], k1v = RA[i - 2], k2v = RA[i - 1], k3v = RA[i];
        put(xa, BM, 4 * q + 0, 4 * kq, make_float4(k0v.x, k1v.x, k2v.x, k3v.x));
        put(xa, BM, 4 * q + 1, 4 * kq, make_float4(k0v.y, k1v.y, k2v.y, k3v.y));
        put(xa, BM, 4 * q + 2, 4 * kq, make_float4(k0v.z, k1v.z, k2v.z, k3v.z));
        put(xa, BM, 4 * q + 3, 4 * kq, make_float4(k0v.w, k1v.w, k2v.w, k3v.w));
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      if constexpr (!TB) {
        const int e = tid + i * NT, r = e / (BK / 4), q = e % (BK / 4);
        put(xb, BN, r, 4 * q, RB[i]);
      } else if ((i & 3) == 3) {
        const int g = tid + (i >> 2) * NT, kq = g % (BK / 4), q = g / (BK / 4);
        const float4 k0v = RB[i - 3], k1v = RB[i - 2], k2v = RB[i - 1], k3v = RB[i];
        put(xb, BN, 4 * q + 0, 4 * kq, make_float4(k0v.x, k1v.x, k2v.x, k3v.x));
        put(xb, BN, 4 * q + 1, 4 * kq, make_float4(k0v.y, k1v.y, k2v.y, k3v.y));
        put(xb, BN, 4 * q + 2, 4 * kq, make_float4(k0v.z, k1v.z, k2v.z, k3v.z));
        put(xb, BN, 4 * q + 3, 4 * kq, make_float4(k0v.w, k1v.w, k2v.w, k3v.w));
      }
    }
  };
  auto store_slab = [&](auto P, int buf) {
    if constexpr (X6) {
      store_slab_x6(P);
      return;
    }
    const float4(&RA)[A_F4] = ra[decltype(P)::value];
    const float4(&RB)[B_F4] = rb[decltype(P)::value];
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int e = tid + i * NT;
      if constexpr (!TA) {
        const int r = e / (BK / 4), q = e % (BK / 4);
        As[buf][4 * q + 0][sw(4 * q + 0, r)] = RA[i].x;
        As[buf][4 * q + 1][sw(4 * q + 1, r)] = RA[i].y;
        As[buf][4 * q + 2][sw(4 * q + 2, r)] = RA[i].z;
        As[buf][4 * q + 3][sw(4 * q + 3, r)] = RA[i].w;
      } else {
        const int r = e / (BM / 4), q = e % (BM / 4);
        *reinterpret_cast<float4*>(&As[buf][r][sw(r, 4 * q)]) = RA[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int e = tid + i * NT;
      if constexpr (!TB) {
        const int r = e / (BK / 4), q = e % (BK / 4);
        Bs[buf][4 * q + 0][sw(4 * q + 0, r)] = RB[i].x;
        Bs[buf][4 * q + 1][sw(4 * q + 1, r)] = RB[i].y;
        Bs[buf][4 * q + 2][sw(4 * q + 2, r)] = RB[i].z;
        Bs[buf][4 * q + 3][sw(4 * q + 3, r)] = RB[i].w;
      } else {
        const int r = e / (BN / 4), q = e % (BN / 4);
        *reinterpret_cast<float4*>(&Bs[buf][r][sw(r, 4 * q)]) = RB[i];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  const int fi = wm * 32 * TM + (lane & 31), fj = wn * 32 * TN + (lane & 31), fk = wk * 32 + (lane >> 5);
  // MFMA fragments double-buffered in registers: the LDS reads of step s + 1 are issued (and pinned
  // by a scheduling barrier) ahead of step s's MFMAs, so their latency hides behind them
  auto compute_x6 = [&]() {
    const int xi = wm * 32 * TM + (lane & 31), xj = wn * 32 * TN + (lane & 31), xk = 8 * (lane >> 5);
    const __bf16* xa = &Xa[0][0][0];
    const __bf16* xb = &Xb[0][0][0];
    // fragments double-buffered: the reads of k-step s + 1 fly across k-step s's MFMAs
    constexpr int FB = 2;
    bf16x8 av[FB][3][TM], bv[FB][3][TN];
    auto rd = [&](int buf, int st) {   // in the order the products consume them (see k_gemm_ws)
      auto ra_ = [&](int p) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          av[buf][p][i] = *reinterpret_cast<const bf16x8*>(xa + (p * BM + xi + 32 * i) * XRS + 16 * st + xk);
      };
      auto rb_ = [&](int p) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bv[buf][p][j] = *reinterpret_cast<const bf16x8*>(xb + (p * BN + xj + 32 * j) * XRS + 16 * st + xk);
      };
      ra_(2); rb_(0); ra_(0); rb_(2); ra_(1); rb_(1);
    };
    if constexpr (FB == 2) rd(0, 0);
#pragma unroll
    for (int st = 0; st < BK / 16; ++st) {
      const int pb = FB == 2 ? (st & 1) : 0;
      if constexpr (FB == 2) {
        if (st + 1 < BK / 16) rd(pb ^ 1, st + 1);
      } else {
        rd(0, st);
      }
      __builtin_amdgcn_sched_barrier(0);
      // smallest products first: (A piece, B piece) = lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi
      constexpr int PA[6] = {2, 0, 1, 1, 0, 0}, PB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[pb][PA[t]][i], bv[pb][PB[t]][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto compute = [&](int cur) {
    if constexpr (X6) {
      compute_x6();
      return;
    }
    float av[2][TM], bv[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) av[0][i] = As[cur][fk][sw(fk, fi + 32 * i)];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[0][j] = Bs[cur][fk][sw(fk, fj + 32 * j)];
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int pb = st & 1;
      if (st + 1 < 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) av[pb ^ 1][i] = As[cur][fk + 2 * st + 2][sw(fk + 2 * st + 2, fi + 32 * i)];
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[pb ^ 1][j] = Bs[cur][fk + 2 * st + 2][sw(fk + 2 * st + 2, fj + 32 * j)];
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
  // optional row sums of A (= the bias gradient of a weight-gradient GEMM, whose A is dY^T):
  // the workgroups of the first column tile add up each staged slab from LDS
  const bool do_rs = a.rowsum != nullptr && bx == 0;
  float rs_acc = 0.f;
  auto rs_slab = [&](int cur) {
    if (do_rs && tid < BM) {
      if constexpr (X6) {   // hi + mid + lo reassembles x exactly
        const __bf16* row = &Xa[0][0][0] + tid * XRS;
#pragma unroll 8
        for (int k = 0; k < BK; ++k)
          rs_acc += ((float)row[k] + (float)row[BM * XRS + k]) + (float)row[2 * BM * XRS + k];
      } else {
#pragma unroll 8
        for (int k = 0; k < BK; ++k) rs_acc += As[cur][k][sw(k, tid)];
      }
    }
  };
  // Pipeline: one LDS stage, slab t + 1 waiting in registers.  Per slab: MFMAs from LDS, barrier,
  // write slab t + 1 to LDS, issue the global loads of slab t + 2, barrier — the loads then fly
  // across a whole compute phase (measured 5-10 % faster than two LDS stages with one barrier,
  // tools/gemm_lab.hip; a second slab in flight for X6 needs more than 256 registers and spills).
  // Only the last slab can be partial: the steady-state loop loads full slabs (no masking,
  // straight-line body); the last few iterations load masked.
  load_slab(I0{}, 0, true);
  store_slab(I0{}, 0);
  if (nk > 1) load_slab(I0{}, BK, true);
  __syncthreads();
  int kt = 0;
  for (; kt + 3 < nk; ++kt) {
    compute(0);
    __builtin_amdgcn_sched_barrier(0);
    rs_slab(0);
    __syncthreads();
    store_slab(I0{}, 0);
    load_slab(I0{}, (kt + 2) * BK, false);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  }
  for (; kt < nk; ++kt) {
    compute(0);
    rs_slab(0);
    __syncthreads();
    if (kt + 1 < nk) {
      store_slab(I0{}, 0);
      if (kt + 2 < nk) load_slab(I0{}, (kt + 2) * BK, true);
      __syncthreads();
    }
  }
  if (do_rs && tid < BM) {
    const int m = m0 + tid;
    if (m < M && m >= a.rowsum_m0) {
      if (a.kspan > 0) a.rowsum_ws[(int64_t)bz * M + m] = rs_acc;
      else a.rowsum[m - a.rowsum_m0] += rs_acc;
    }
  }

  // ---- intra-workgroup split-K: waves wk > 0 hand their tiles to wk == 0 through LDS ----------
  if constexpr (WK > 1) {
    static_assert(TM == 1 && TN == 1, "intra-workgroup split-K uses one tile per wave");
    float* red = &As[0][0][0];   // reuse the staging LDS
    static_assert((WK - 1) * WM * WN * 16 * 64 <= BK * AST + BK * BST, "reduction scratch too small");
    float* mine = red + ((wk - 1) * WM * WN + wmn) * 16 * 64;
    __syncthreads();   // every wave is done reading the last slab
    if (wk > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) mine[r * 64 + lane] = acc[0][0][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int j = 1; j < WK; ++j) {
      const float* src = red + ((j - 1) * WM * WN + wmn) * 16 * 64;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][0][r] += src[r * 64 + lane];
    }
  }

  gemm_epilogue<TM, TN, EPI, RES, X6 && EPI == EPI_GELU_DROP>(a, acc, m0, n0, wm, wn, lane, bz);
}

// LayerNorm epilogues of the warp-specialised GEMM (EPI_RES_LN / EPI_LN_BWD; N <= BN, one column
// tile).  The consumers park the accumulator tile (2 x 2 32 x 32 MFMA tiles per wave) in LDS rows;
// then each of the 8 waves takes rows w, w + 8, ... with a lane per 4 consecutive columns: every
// global operand of its rows is loaded before the first reduction, row statistics are wave sums.
// The same arithmetic per element as k_ln_fwd / k_ln_bwd (train.hip): x-transformers LayerNorm
// (no affine, eps 1e-5) times gamma, two-pass variance; d gamma partials per BM-row tile summed
// over the 8 waves in wave order (deterministic).
template <int BM, int BN, int EPI>
__device__ __forceinline__ void ln_epilogue(const GemmArgs& a, f32x16 (&acc)[2][2], float* tile, bool producer,
                                            int m0, int wm, int wn, int lane, int wave, int row_tile) {
  constexpr int LDT = BN + 4, RPW = BM / 8;
  const int M = a.M, N = a.N;
  if (!producer) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + 32 * i + 4 * (lane >> 5) + 8 * (r >> 2) + (r & 3);
          tile[row * LDT + wn * 64 + 32 * j + (lane & 31)] = acc[i][j][r];
        }
  }
  __syncthreads();
  const int c = 4 * lane;
  const bool cok = c < N;
  // every global load unconditional at an in-bounds column (a select between a global and a zero
  // operand compiles to flat loads through a scratch zero), the values selected afterwards
  const int cc = cok ? c : 0;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  auto ld4 = [&](const float* base) { return *reinterpret_cast<const float4*>(base + cc); };
  float4 gam = ld4(a.ln_g);
  if (!cok) gam = z4;
  const float inv_n = 1.0f / (float)N;
  if constexpr (EPI == EPI_RES_LN) {
    float4 bia = z4, beta = z4, add2 = z4;
    if (a.bias) bia = ld4(a.bias);
    if (a.ln_b) beta = ld4(a.ln_b);
    if (a.ln_b2) add2 = ld4(a.ln_b2);
    if (!cok) bia = beta = add2 = z4;
    float4 v[RPW], r[RPW];
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int row = wave + 8 * rr, mc = min(m0 + row, M - 1);
      v[rr] = *reinterpret_cast<const float4*>(tile + row * LDT + cc);
      r[rr] = ld4(a.R + (int64_t)mc * a.ldr);
    }
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int m = m0 + wave + 8 * rr;
      float4 x;   // (acc + bias) + residual, as the GEMM epilogue forms it
      x.x = (v[rr].x + bia.x) + r[rr].x; x.y = (v[rr].y + bia.y) + r[rr].y;
      x.z = (v[rr].z + bia.z) + r[rr].z; x.w = (v[rr].w + bia.w) + r[rr].w;
      if (!cok) x = z4;
      const float mean = a.ln_rms ? 0.f : wave_sum((x.x + x.y) + (x.z + x.w)) * inv_n;
      float4 dl = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
      if (!cok) dl = z4;
      const float sq = wave_sum((dl.x * dl.x + dl.y * dl.y) + (dl.z * dl.z + dl.w * dl.w));
      const float rstd = a.ln_rms ? norm_rstd(sq, (float)N, true) : 1.0f / sqrtf(sq * inv_n + 1e-5f);
      float4 y = make_float4((dl.x * rstd) * gam.x, (dl.y * rstd) * gam.y, (dl.z * rstd) * gam.z,
                             (dl.w * rstd) * gam.w);
      if (a.ln_b) y = make_float4(y.x + beta.x, y.y + beta.y, y.z + beta.z, y.w + beta.w);
      if (m < M) {
        if (cok) {
          *reinterpret_cast<float4*>(a.C + (int64_t)m * a.ldc + c) = x;
          *reinterpret_cast<float4*>(a.ln_y1 + (int64_t)m * a.ln_ld1 + c) = y;
          if (a.ln_y2)
            *reinterpret_cast<float4*>(a.ln_y2 + (int64_t)m * a.ln_ld2 + c) =
                make_float4(y.x + add2.x, y.y + add2.y, y.z + add2.z, y.w + add2.w);
        }
        if (lane == 0) *reinterpret_cast<float2*>(a.ln_stats + 2 * (int64_t)m) = make_float2(mean, rstd);
      }
    }
  } else {
    // EPI_LN_BWD: the x-transformers LayerNorm (no bias) with a residual gradient added after;
    // EPI_LN_BWD2: nn.LayerNorm post-norm blocks (gradient added before, d beta, optional chain)
    constexpr bool X = EPI == EPI_LN_BWD2;
    const int ps = X && a.ln_pstride ? a.ln_pstride : N;
    float4 g[RPW], xv[RPW], dr[RPW];
    float2 st[RPW];
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int row = wave + 8 * rr, mc = min(m0 + row, M - 1);
      g[rr] = *reinterpret_cast<const float4*>(tile + row * LDT + cc);
      xv[rr] = ld4(a.ln_x + (int64_t)mc * N);
      if constexpr (X) dr[rr] = a.ln_gpre ? ld4(a.ln_gpre + (int64_t)mc * (a.ln_ldg ? a.ln_ldg : N)) : z4;
      else dr[rr] = a.ln_dres ? ld4(a.ln_dres + (int64_t)mc * N) : z4;
      st[rr] = *reinterpret_cast<const float2*>(a.ln_stats + 2 * (int64_t)mc);
      if constexpr (X) {
        const float gs = a.ln_gscale;
        g[rr] = make_float4(g[rr].x * gs + dr[rr].x, g[rr].y * gs + dr[rr].y, g[rr].z * gs + dr[rr].z,
                            g[rr].w * gs + dr[rr].w);
      }
      if (!cok) g[rr] = z4;
    }
    float4 dg = z4, db = z4;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int m = m0 + wave + 8 * rr;
      const float mu = st[rr].x, rs = st[rr].y;
      float4 xh = make_float4((xv[rr].x - mu) * rs, (xv[rr].y - mu) * rs, (xv[rr].z - mu) * rs, (xv[rr].w - mu) * rs);
      if (!cok) xh = z4;
      const float4 gm = make_float4(g[rr].x * gam.x, g[rr].y * gam.y, g[rr].z * gam.z, g[rr].w * gam.w);
      if (m < M) {
        dg.x += g[rr].x * xh.x; dg.y += g[rr].y * xh.y; dg.z += g[rr].z * xh.z; dg.w += g[rr].w * xh.w;
        if constexpr (X) { db.x += g[rr].x; db.y += g[rr].y; db.z += g[rr].z; db.w += g[rr].w; }
      }
      // (RMSNorm: no mean in the forward, so no mean(g gamma) term: dx = rstd (g gamma - x^ mean(g gamma x^)))
      const float ma = a.ln_rms ? 0.f : wave_sum((gm.x + gm.y) + (gm.z + gm.w)) * inv_n;
      const float mb = wave_sum((gm.x * xh.x + gm.y * xh.y) + (gm.z * xh.z + gm.w * xh.w)) * inv_n;
      float4 o;
      o.x = rs * (gm.x - ma - xh.x * mb);
      o.y = rs * (gm.y - ma - xh.y * mb);
      o.z = rs * (gm.z - ma - xh.z * mb);
      o.w = rs * (gm.w - ma - xh.w * mb);
      if constexpr (!X) {
        o.x += dr[rr].x; o.y += dr[rr].y; o.z += dr[rr].z; o.w += dr[rr].w;
      }
      if (!cok) o = z4;
      if (m < M && cok) *reinterpret_cast<float4*>(a.C + (int64_t)m * a.ldc + c) = o;
      if constexpr (X) g[rr] = o;   // the chained LayerNorm's upstream gradient
    }
    // partials of this row tile: the 8 waves' column sums, added in wave order
    float* red = tile + BM * LDT;
    const int t = threadIdx.x;
    auto tile_sum = [&](float4 v, float* dst) {
      __syncthreads();
      if (cok) *reinterpret_cast<float4*>(red + wave * BN + c) = v;
      __syncthreads();
      if (t < N) {
        float sum = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) sum += red[w * BN + t];
        dst[(int64_t)row_tile * ps + t] = sum;
      }
    };
    tile_sum(dg, a.ln_part);
    if constexpr (X) {
      if (a.ln_part_b) tile_sum(db, a.ln_part_b);
      if (a.ln2_out) {   // chained: the LayerNorm whose output's whole gradient is the one just formed
        float4 gam2 = ld4(a.ln2_g);
        if (!cok) gam2 = z4;
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int row = wave + 8 * rr, mc = min(m0 + row, M - 1);
          xv[rr] = ld4(a.ln2_x + (int64_t)mc * N);
          st[rr] = *reinterpret_cast<const float2*>(a.ln2_stats + 2 * (int64_t)mc);
        }
        dg = db = z4;
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int m = m0 + wave + 8 * rr;
          const float mu = st[rr].x, rs = st[rr].y;
          float4 xh = make_float4((xv[rr].x - mu) * rs, (xv[rr].y - mu) * rs, (xv[rr].z - mu) * rs, (xv[rr].w - mu) * rs);
          if (!cok) xh = z4;
          const float4 gm = make_float4(g[rr].x * gam2.x, g[rr].y * gam2.y, g[rr].z * gam2.z, g[rr].w * gam2.w);
          if (m < M) {
            dg.x += g[rr].x * xh.x; dg.y += g[rr].y * xh.y; dg.z += g[rr].z * xh.z; dg.w += g[rr].w * xh.w;
            db.x += g[rr].x; db.y += g[rr].y; db.z += g[rr].z; db.w += g[rr].w;
          }
          const float ma = wave_sum((gm.x + gm.y) + (gm.z + gm.w)) * inv_n;
          const float mb = wave_sum((gm.x * xh.x + gm.y * xh.y) + (gm.z * xh.z + gm.w * xh.w)) * inv_n;
          const float4 o = make_float4(rs * (gm.x - ma - xh.x * mb), rs * (gm.y - ma - xh.y * mb),
                                       rs * (gm.z - ma - xh.z * mb), rs * (gm.w - ma - xh.w * mb));
          if (m < M && cok) *reinterpret_cast<float4*>(a.ln2_out + (int64_t)m * N + c) = o;
        }
        tile_sum(dg, a.ln2_part);
        tile_sum(db, a.ln2_part_b);
      }
    }
  }
}

#ifdef XTRL_WS_DIAG   // tools/ws_lab.hip: per-step s_memtime stamps of waves 0 and 4 of every workgroup
__device__ uint64_t* g_ws_diag;
__device__ int g_ws_mode;   // 1: consumers skip the MFMAs; 2: producers skip loads + splits; 3: skip splits
#define WS_STAMP(step, k)                                                                         \
  do {                                                                                            \
    if ((tid & 255) == 0)                                                                         \
      g_ws_diag[((int64_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 2 +   \
                 (tid >> 8)) * 4096 + (step) * 4 + (k)] = __builtin_amdgcn_s_memtime();           \
  } while (0)
#else
#define WS_STAMP(step, k) do {} while (0)
#endif

// ---- X6 warp-specialised GEMM (the large-tile path) ---------------------------------------------
// 8 waves per workgroup, one workgroup per CU.  Waves 0-3 (one per SIMD) are consumers: each owns
// 64 x 64 of the tile and only reads piece fragments from LDS and issues bf16 MFMAs.  Waves 4-7
// (their SIMD partners) are producers: they keep two fp32 slabs in flight global -> registers,
// split each staged value into its hi / mid / lo pieces and write the piece images the consumers
// read next.  Two piece images (double buffered), one barrier per 32-deep K slab: the consumers
// never wait on global memory, and the producers' split arithmetic issues in the gaps of their
// partner's MFMAs.  Float4 operands; K a multiple of 32, or of 4 with KT (the last slab's k >= K
// entries are zeroed in both operands, branch-free).
// Tiles: BM x BN = 128 x 128 (2 x 2 consumer waves) or 64 x 256 (1 x 4: a whole d = 256 row per
// tile, so the LayerNorm epilogues below see every column of their rows).
// LayerNorm epilogues (EPI_RES_LN / EPI_LN_BWD, one column tile, N <= BN): the consumers park the
// tile in LDS (the piece images are free after the last step), then all 8 waves take whole rows —
// a lane per 4 consecutive columns, every operand of the wave's rows loaded before the first
// reduction — and finish the residual + LayerNorm forward, or the LayerNorm backward with the
// incoming residual gradient and the tile's d gamma partial, in the same launch (no normalised /
// d-normalised intermediate goes through HBM, no separate LayerNorm launch).
template <bool TA, bool TB, int EPI, bool RES, int BM = 128, int BN = 128, bool KT = false>
__global__ __launch_bounds__(512, 1) void k_gemm_ws(const GemmArgs a) {
  constexpr int BK = 32, XRS = BK + 8, NP = 256, TM = 2, TN = 2, WN = BN / 64;
  constexpr bool LNE = (EPI == EPI_RES_LN || EPI == EPI_LN_BWD || EPI == EPI_LN_BWD2);
  constexpr int A_F4 = BM * BK / 4 / NP, B_F4 = BN * BK / 4 / NP;   // float4 per producer thread per slab
  constexpr int IMG = 3 * (BM + BN) * XRS;                           // bf16 per piece image
  static_assert((BM == 128 && BN == 128) || (BM == 64 && BN == 256), "tile 128 x 128 or 64 x 256");
  static_assert(!TA || A_F4 == 4, "A \"T\": one 4 x 4 transposed group per producer thread");
  static_assert(!TB || B_F4 % 4 == 0, "B \"T\": whole 4 x 4 transposed groups per producer thread");
  constexpr int LDT = BN + 4;                                        // LN epilogue: tile rows in LDS (floats)
  static_assert(!LNE || (BM * LDT + 8 * BN) * 4 <= 2 * IMG * 2, "LN tile exceeds the piece images");
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool producer = wave >= 4;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (a.xcd_remap) {   // as k_gemm: each XCD runs a contiguous range of tiles (column tile fastest)
    const int nx = gridDim.x, ny = gridDim.y;
    const int total = nx * ny * gridDim.z;
    const int lin = bx + nx * (by + ny * bz);
    const int lg = (lin & 7) * (total >> 3) + (lin >> 3);
    bx = lg % nx;
    by = (lg / nx) % ny;
    bz = lg / (nx * ny);
  }
  const int m0 = by * BM, n0 = bx * BN;
  const int M = a.M, N = a.N;
  int K = a.K;
  const float* __restrict__ Ab = a.A;
  const float* __restrict__ Bb = a.B;
  if (a.kspan > 0) {
    const int kb = bz * a.kspan;
    K = min(a.kspan, a.K - kb);
    Ab += TA ? (int64_t)kb * a.lda : kb;
    Bb += TB ? (int64_t)kb * a.ldb : kb;
  }
  const int nk = (K + BK - 1) / BK;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // ---- producer state: two register sets of one slab each ----
  const int p = tid - 256;
  float4 ra[2][A_F4], rb[2][B_F4];
  const bool do_rs = a.rowsum != nullptr && bx == 0;   // bias gradient (TA only, see gemm_run)
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  // operand element loads, clamped into the operand (rows / columns past M / N feed only outputs
  // the epilogue discards; k past K: clamped in-bounds, then zeroed with KT)
  auto ld_n = [&](const float* base, int64_t ld, int row, int row_lim, int k) -> float4 {   // [row][k]
    float4 f = *reinterpret_cast<const float4*>(base + (int64_t)min(row, row_lim - 1) * ld + (KT ? min(k, K - 4) : k));
    if constexpr (KT) {
      const bool ok = k < K;
      f = make_float4(ok ? f.x : 0.f, ok ? f.y : 0.f, ok ? f.z : 0.f, ok ? f.w : 0.f);
    }
    return f;
  };
  auto ld_t = [&](const float* base, int64_t ld, int k, int col, int col_lim) -> float4 {   // [k][col]
    float4 f = *reinterpret_cast<const float4*>(base + (int64_t)(KT ? min(k, K - 1) : k) * ld +
                                                min(col, ((col_lim + 3) & ~3) - 4));
    if constexpr (KT) {
      const bool ok = k < K;
      f = make_float4(ok ? f.x : 0.f, ok ? f.y : 0.f, ok ? f.z : 0.f, ok ? f.w : 0.f);
    }
    return f;
  };
  auto load = [&](auto S, int kt) {
    const int k0 = min(kt, nk - 1) * BK;
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      if constexpr (!TA) {
        const int e = p + i * NP, r = e / (BK / 4), q = e % (BK / 4);
        ra[S][i] = ld_n(Ab, a.lda, m0 + r, M, k0 + 4 * q);
      } else {   // 4 x 4 group: k rows 4 kq .. 4 kq + 3 of m quad q
        const int kq = p % (BK / 4), q = p / (BK / 4);
        ra[S][i] = ld_t(Ab, a.lda, k0 + 4 * kq + i, m0 + 4 * q, M);
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      if constexpr (!TB) {
        const int e = p + i * NP, r = e / (BK / 4), q = e % (BK / 4);
        rb[S][i] = ld_n(Bb, a.ldb, n0 + r, N, k0 + 4 * q);
      } else {   // group i / 4 covers column quads 32 (i / 4) + p / 8
        const int kq = p % (BK / 4), q = p / (BK / 4) + 32 * (i >> 2);
        rb[S][i] = ld_t(Bb, a.ldb, k0 + 4 * kq + (i & 3), n0 + 4 * q, N);
      }
    }
  };
  auto put = [&](__bf16* img, int rows, int row, int k, float4 v) {
    bf16x4 h, m, l;
#if defined(XTRL_WS_MODE) && XTRL_WS_MODE == 4   // tools/ws_lab.hip: the LDS writes without the split arithmetic
    h = __builtin_bit_cast(bf16x4, make_uint2(__float_as_uint(v.x), __float_as_uint(v.y)));
    m = __builtin_bit_cast(bf16x4, make_uint2(__float_as_uint(v.z), __float_as_uint(v.w)));
    l = __builtin_bit_cast(bf16x4, make_uint2(__float_as_uint(v.x), __float_as_uint(v.w)));
#else
    split3(v, h, m, l);
#endif
    __bf16* q = img + row * XRS + k;
    *reinterpret_cast<bf16x4*>(q) = h;
    *reinterpret_cast<bf16x4*>(q + rows * XRS) = m;
    *reinterpret_cast<bf16x4*>(q + 2 * rows * XRS) = l;
  };
  auto convert = [&](auto S, __bf16* img, bool live) {   // live: a real slab (row sums count it)
    __bf16* xa = img;
    __bf16* xb = img + 3 * BM * XRS;
    const int kq = p % (BK / 4), q = p / (BK / 4);
    if constexpr (!TA) {
#pragma unroll
      for (int i = 0; i < A_F4; ++i) {
        const int e = p + i * NP, r = e / (BK / 4), qq = e % (BK / 4);
        put(xa, BM, r, 4 * qq, ra[S][i]);
      }
    } else {
      const float4 k0v = ra[S][0], k1v = ra[S][1], k2v = ra[S][2], k3v = ra[S][3];
      put(xa, BM, 4 * q + 0, 4 * kq, make_float4(k0v.x, k1v.x, k2v.x, k3v.x));
      put(xa, BM, 4 * q + 1, 4 * kq, make_float4(k0v.y, k1v.y, k2v.y, k3v.y));
      put(xa, BM, 4 * q + 2, 4 * kq, make_float4(k0v.z, k1v.z, k2v.z, k3v.z));
      put(xa, BM, 4 * q + 3, 4 * kq, make_float4(k0v.w, k1v.w, k2v.w, k3v.w));
      if (do_rs) {   // this slab's sums of rows 4 q .. 4 q + 3: own 4 k, then the 8 lanes of the m quad
        float s4[4] = {(k0v.x + k1v.x) + (k2v.x + k3v.x), (k0v.y + k1v.y) + (k2v.y + k3v.y),
                       (k0v.z + k1v.z) + (k2v.z + k3v.z), (k0v.w + k1v.w) + (k2v.w + k3v.w)};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
          for (int o = 1; o < BK / 4; o <<= 1) s4[c] += __shfl_xor(s4[c], o, kWave);
          rs[c] += live ? s4[c] : 0.f;
        }
      }
    }
    if constexpr (!TB) {
#pragma unroll
      for (int i = 0; i < B_F4; ++i) {
        const int e = p + i * NP, r = e / (BK / 4), qq = e % (BK / 4);
        put(xb, BN, r, 4 * qq, rb[S][i]);
      }
    } else {
#pragma unroll
      for (int gi = 0; gi < B_F4 / 4; ++gi) {
        const int qg = q + 32 * gi;
        const float4 k0v = rb[S][4 * gi], k1v = rb[S][4 * gi + 1], k2v = rb[S][4 * gi + 2], k3v = rb[S][4 * gi + 3];
        put(xb, BN, 4 * qg + 0, 4 * kq, make_float4(k0v.x, k1v.x, k2v.x, k3v.x));
        put(xb, BN, 4 * qg + 1, 4 * kq, make_float4(k0v.y, k1v.y, k2v.y, k3v.y));
        put(xb, BN, 4 * qg + 2, 4 * kq, make_float4(k0v.z, k1v.z, k2v.z, k3v.z));
        put(xb, BN, 4 * qg + 3, 4 * kq, make_float4(k0v.w, k1v.w, k2v.w, k3v.w));
      }
    }
  };

  // ---- consumer state ----
  const int wm = (wave & 3) / WN, wn = (wave & 3) % WN;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto compute = [&](const __bf16* img) {
    const int xi = wm * 32 * TM + (lane & 31), xj = wn * 32 * TN + (lane & 31), xk = 8 * (lane >> 5);
    const __bf16* xa = img;
    const __bf16* xb = img + 3 * BM * XRS;
    bf16x8 av[2][3][TM], bv[2][3][TN];
    // fragments read in the order the products consume them (A lo, B hi, A hi, B lo, A mid, B mid),
    // so the first MFMAs of a slab wait for three reads, not for all of them
    auto rd = [&](int buf, int st) {
      auto ra_ = [&](int pc) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          av[buf][pc][i] = *reinterpret_cast<const bf16x8*>(xa + (pc * BM + xi + 32 * i) * XRS + 16 * st + xk);
      };
      auto rb_ = [&](int pc) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bv[buf][pc][j] = *reinterpret_cast<const bf16x8*>(xb + (pc * BN + xj + 32 * j) * XRS + 16 * st + xk);
      };
      ra_(2); rb_(0); ra_(0); rb_(2); ra_(1); rb_(1);
    };
    rd(0, 0);
#pragma unroll
    for (int st = 0; st < BK / 16; ++st) {
      const int pb = st & 1;
      if (st + 1 < BK / 16) rd(pb ^ 1, st + 1);
      __builtin_amdgcn_sched_barrier(0);
      // smallest products first: (A piece, B piece) = lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi
      constexpr int PA[6] = {2, 0, 1, 1, 0, 0}, PB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
      for (int t = 0; t < 6; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[pb][PA[t]][i], bv[pb][PB[t]][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- pipeline ----
  // Slab t waits in register set t & 1 until it is split into piece image t & 1.  The two roles
  // run separate loops (neither keeps the other's registers live) with the same barrier sequence:
  // one after the prologue, then one per step, 2 * ceil(nk / 2) steps.  In step t the consumers
  // multiply image t & 1 while the producers split slab t + 1 (set (t + 1) & 1) into image
  // (t + 1) & 1 and refill that set with slab t + 3.  Loads past the last slab repeat it
  // (clamped); their splits go to images no consumer reads.  (Three register sets with the loads
  // issued ahead of the split measured 13 % slower: tools/ws_lab.hip.)
  const int nsteps = 2 * ((nk + 1) / 2);
  if (producer) {
    load(I0{}, 0);
    load(I1{}, 1);
    convert(I0{}, smem, true);
    load(I0{}, 2);
    __syncthreads();
#ifdef XTRL_WS_DIAG
    const int mode = g_ws_mode;
#elif defined(XTRL_WS_MODE)   // tools/ws_lab.hip stamp-free builds: the same modes, fixed at compile time
    constexpr int mode = XTRL_WS_MODE;
#else
    constexpr int mode = 0;
#endif
    // straight-line body (no branch around a load: hipcc would wait for every load at the join);
    // scheduling barriers keep each step's split inside its step (the scheduler would otherwise
    // hoist the next step's split arithmetic above the workgroup barrier)
    auto pstep = [&](auto C, int t) {
      WS_STAMP(t, 0);
      if (mode < 2 || mode == 4) convert(C, smem + ((t + 1) & 1) * IMG, t + 1 < nk);
      else if (mode == 3) {   // consume the loads without splitting
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) s += ra[decltype(C)::value][i % A_F4].x + rb[decltype(C)::value][i].y;
        if (s == 12345.f) smem[tid] = (__bf16)s;
      }
      WS_STAMP(t, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (mode != 2) load(C, t + 3);
      WS_STAMP(t, 2);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
    };
    for (int t = 0; t < nsteps; t += 2) {
      pstep(I1{}, t);
      pstep(I0{}, t + 1);
    }
    if (TA && do_rs && (p % (BK / 4)) == 0) {
      const int q = p / (BK / 4);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int m = m0 + 4 * q + c;
        if (m < M && m >= a.rowsum_m0) {
          if (a.kspan > 0) a.rowsum_ws[(int64_t)bz * M + m] = rs[c];
          else a.rowsum[m - a.rowsum_m0] += rs[c];
        }
      }
    }
    if constexpr (!LNE) return;
  } else {
    __syncthreads();
    for (int t = 0; t < nsteps; ++t) {
      WS_STAMP(t, 0);
#ifdef XTRL_WS_DIAG
      if (t < nk && g_ws_mode != 1) compute(smem + (t & 1) * IMG);
#elif defined(XTRL_WS_MODE)
      if (t < nk && XTRL_WS_MODE != 1) compute(smem + (t & 1) * IMG);
#else
      if (t < nk) compute(smem + (t & 1) * IMG);
#endif
      WS_STAMP(t, 1);
      __syncthreads();
    }
    WS_STAMP(nsteps, 0);
    if constexpr (!LNE) {
      gemm_epilogue<TM, TN, EPI, RES, EPI == EPI_GELU_DROP>(a, acc, m0, n0, wm, wn, lane, bz);
      return;
    }
  }
  if constexpr (LNE) ln_epilogue<BM, BN, EPI>(a, acc, reinterpret_cast<float*>(smem), producer, m0, wm, wn, lane, wave,
                                              by);
}

__global__ __launch_bounds__(256) void k_layernorm(const float* X, int ldx, const float* gamma, float* Y, int ldy,
                                                   int M, int D) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const float* xr = X + (int64_t)m * ldx;
  float s = 0.f;
  for (int k = lane; k < D; k += 64) s += xr[k];
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
  for (int k = lane; k < D; k += 64) {
    const float dlt = xr[k] - mean;
    q += dlt * dlt;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + 1e-5f);
  for (int k = lane; k < D; k += 64) Y[(int64_t)m * ldy + k] = ((xr[k] - mean) * rstd) * gamma[k];
}

// phase 2 of the split-K GEMM: C = beta * C + sum_z partial[z] in a fixed order (deterministic:
// partial z goes to accumulator z % 8, the eight are summed as a fixed tree; eight loads per
// thread in flight).  Partials are dense [S][M][N]; each thread owns one float4 of C.  Optional
// row sums (bias gradient): rowsum[m - m0] += sum_z rws[z][m], spread over the grid.
// sum_z p[z * stride] for z < S in z order, sixteen loads in flight (a serial loop waits out one
// load latency per split: 64 splits cost tens of microseconds)
__device__ __forceinline__ float sum_splits(const float* p, int S, int64_t stride) {
  float acc = 0.f;
  int z = 0;
  for (; z + 16 <= S; z += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = p[(int64_t)(z + u) * stride];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += v[u];
  }
  for (; z < S; ++z) acc += p[(int64_t)z * stride];
  return acc;
}

__global__ __launch_bounds__(256) void k_splitk_reduce(const float* ws, int S, int M, int N, float* C, int ldc,
                                                       float beta, const float* rws, float* rowsum, int m0) {
  const int64_t MN = (int64_t)M * N;
  const int64_t gtid = (int64_t)blockIdx.x * 256 + threadIdx.x, gsz = (int64_t)gridDim.x * 256;
  if (rowsum) {
    for (int64_t m = m0 + gtid; m < M; m += gsz) rowsum[m - m0] += sum_splits(rws + m, S, M);
  }
  if ((N & 3) == 0) {
    // four lanes per float4 of C: lane g sums partials g, g + 4, g + 8, ... (eight loads in
    // flight), then the four lane sums combine as (l0 + l1) + (l2 + l3)
    constexpr int G = 4, U = 8;
    const int64_t Q = MN >> 2;
    const int g = threadIdx.x & (G - 1);
    const float4* w4 = reinterpret_cast<const float4*>(ws);
    for (int64_t q = gtid / G; q < Q; q += gsz / G) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int z0 = g; z0 < S; z0 += G * U) {
        float4 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int z = z0 + G * u;
          p[u] = z < S ? w4[(int64_t)z * Q + q] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          a.x += p[u].x; a.y += p[u].y; a.z += p[u].z; a.w += p[u].w;
        }
      }
      float4 b;
      b.x = __shfl_xor(a.x, 1); b.y = __shfl_xor(a.y, 1); b.z = __shfl_xor(a.z, 1); b.w = __shfl_xor(a.w, 1);
      if (g & 1) { const float4 t = a; a = b; b = t; }   // (even + odd) in both lanes, same order
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      b.x = __shfl_xor(a.x, 2); b.y = __shfl_xor(a.y, 2); b.z = __shfl_xor(a.z, 2); b.w = __shfl_xor(a.w, 2);
      if (g & 2) { const float4 t = a; a = b; b = t; }
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      if (g == 0) {
        const int64_t i = q << 2;
        const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
        float* dst = C + (int64_t)m * ldc + n;
        if (beta != 0.f) {
          a.x += beta * dst[0]; a.y += beta * dst[1]; a.z += beta * dst[2]; a.w += beta * dst[3];
        }
        dst[0] = a.x; dst[1] = a.y; dst[2] = a.z; dst[3] = a.w;
      }
    }
    return;
  }
  for (int64_t i = gtid; i < MN; i += gsz) {
    const float acc = sum_splits(ws + i, S, MN);
    const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
    float* dst = C + (int64_t)m * ldc + n;
    *dst = (beta != 0.f) ? beta * (*dst) + acc : acc;
  }
}

// every queued split-K job in one launch (SplitKQueue, kernels.h): thread unit u < total float4
// units sums the S partial float4s of its job's element group in z order (eight loads in flight),
// the remaining units the row sums (bias gradients).  Jobs are passed by value (kernel arguments).
struct SplitKJobs {
  SplitKJob job[kMaxSplitKJobs];
  int n;
  int64_t total_q, total_r;
};
__global__ __launch_bounds__(256) void k_splitk_reduce_multi(const SplitKJobs J) {
  const int64_t gsz = (int64_t)gridDim.x * 256;
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < J.total_q + J.total_r; u += gsz) {
    if (u < J.total_q) {
      int j = 0;
      while (j + 1 < J.n && J.job[j + 1].q0 <= u) ++j;
      const SplitKJob& b = J.job[j];
      const int64_t q = u - b.q0, MN4 = (int64_t)b.M * b.N / 4;
      const float4* w4 = reinterpret_cast<const float4*>(b.ws);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      int z = 0;
      for (; z + 8 <= b.S; z += 8) {
        float4 p[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) p[k] = w4[(int64_t)(z + k) * MN4 + q];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a.x += p[k].x; a.y += p[k].y; a.z += p[k].z; a.w += p[k].w;
        }
      }
      for (; z < b.S; ++z) {
        const float4 p = w4[(int64_t)z * MN4 + q];
        a.x += p.x; a.y += p.y; a.z += p.z; a.w += p.w;
      }
      const int64_t i = q << 2;
      const int m = (int)(i / b.N), n = (int)(i - (int64_t)m * b.N);
      float4* dst = reinterpret_cast<float4*>(b.C + (int64_t)m * b.ldc + n);
      if (b.beta != 0.f) {
        const float4 o = *dst;
        a.x += b.beta * o.x; a.y += b.beta * o.y; a.z += b.beta * o.z; a.w += b.beta * o.w;
      }
      *dst = a;
    } else {
      const int64_t r = u - J.total_q;
      int j = 0;
      while (j + 1 < J.n && J.job[j + 1].r0 <= r) ++j;
      const SplitKJob& b = J.job[j];
      const int m = b.m0 + (int)(r - b.r0);
      b.rowsum[m - b.m0] += sum_splits(b.rws + m, b.S, b.M);
    }
  }
}

bool xcd_env() {   // XTRL_GEMM_XCD=0: hardware workgroup order (A/B experiments)
  static const bool on = [] {
    const char* e = getenv("XTRL_GEMM_XCD");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

template <int WM, int WN, int WK, int TM, int TN, bool TA, bool TB, int EPI, bool LN, bool RES, bool VEC,
          bool X6 = false>
void launch(const GemmArgs& a, hipStream_t s) {
  constexpr int BM = 32 * WM * TM, BN = 32 * WN * TN;
  const int splits = a.kspan > 0 ? (a.K + a.kspan - 1) / a.kspan : 1;
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  if constexpr (X6) {
    if (xcd_env() && (int64_t)grid.x * grid.y * grid.z % 8 == 0) {
      GemmArgs r = a;
      r.xcd_remap = 1;
      hipLaunchKernelGGL((k_gemm<WM, WN, WK, TM, TN, TA, TB, EPI, LN, RES, VEC, X6>), grid, dim3(64 * WM * WN * WK), 0,
                         s, r);
      return;
    }
  }
  hipLaunchKernelGGL((k_gemm<WM, WN, WK, TM, TN, TA, TB, EPI, LN, RES, VEC, X6>), grid, dim3(64 * WM * WN * WK), 0, s,
                     a);
}

// split-bf16 products on the 64 x 64 geometry too (XTRL_GEMM_X6_SMALL=0: f32 products there).  On
// since the rollout's projections moved to the decode GEMM (dgemm.hip): the learn step's mid-sized
// GEMMs gain (C3 learn -0.2 ... -0.5 ms in 5 of 5 A/B rounds); round 1 had it off for the decode
// shapes (rollout 38.7 vs 38.1 ms)
bool use_x6_small() {
  static const bool on = [] {
    const char* e = getenv("XTRL_GEMM_X6_SMALL");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

bool use_ws() {   // XTRL_GEMM_WS=0: the register-staged X6 kernel instead of the warp-specialised one
  static const bool on = [] {
    const char* e = getenv("XTRL_GEMM_WS");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// the warp-specialised X6 kernel takes whole 32-deep slabs (K and the split span) and no LN prologue
// (ta: the weight-gradient "T" x "T" layout, whose staging loads every k row on its own — a K that is not
// a multiple of 32 (the packed learn step's token count) takes the KT variant, the last slab's rows past K
// zeroed; spans stay multiples of 32)
bool ws_ok(const GemmArgs& a, bool ta, bool ln) {
  if (!(use_ws() && !ln && (a.K % 32 == 0 || ta) && (a.kspan == 0 || a.kspan % 32 == 0) && (!a.rowsum || ta)))
    return false;
  // one workgroup per CU: it wins only when the whole grid is one resident round and K is long
  // (16384 x 256 x 1024: 59 vs 72 us); with several rounds or K = 256 the register-staged kernel's
  // two workgroups per CU overlap one tile's prologue / epilogue with another's main loop
  // (16384 x 1024 x 256: 94 vs 70 us; tools/gemm_bench.py, XTRL_GEMM_WS=0)
  const int splits = a.kspan > 0 ? (a.K + a.kspan - 1) / a.kspan : 1;
  const int64_t wgs = (int64_t)((a.N + 127) / 128) * ((a.M + 127) / 128) * splits;
  // (weight gradients, "T" x "T": the warp-specialised kernel wins at every split span measured, down to
  // 352 tokens — tools/wgrad_span_lab.hip, 256 x 256 over 16384 tokens: 25.4 vs 31.2 us at 47 splits,
  // 35.5 vs 48.1 at 24; the C5 fractal step's 256 x 256 / 192 x 256 weights)
  return wgs <= 256 && (a.kspan > 0 ? a.kspan : a.K) >= (ta ? 64 : 512);
}

template <bool TA, bool TB, int EPI, bool RES, int BM = 128, int BN = 128, bool KT = false>
void launch_ws(const GemmArgs& a, hipStream_t s) {
  const int splits = a.kspan > 0 ? (a.K + a.kspan - 1) / a.kspan : 1;
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  GemmArgs r = a;
  r.xcd_remap = (xcd_env() && (int64_t)grid.x * grid.y * grid.z % 8 == 0) ? 1 : 0;
  hipLaunchKernelGGL((k_gemm_ws<TA, TB, EPI, RES, BM, BN, KT>), grid, dim3(512), 0, s, r);
}

// the LayerNorm-epilogue GEMMs: one column tile per row (N <= 256), 128-row tiles up to N = 128,
// 64 x 256 above; K a multiple of 4 (KT masks a partial last slab)
int ln_gemm_run(const GemmArgs& a, int trans_a, int trans_b, int epi, bool vec, hipStream_t s) {
  const bool res = a.R != nullptr;
  XTRL_REQUIRE(!trans_a && vec && a.kspan == 0 && a.N <= 256 && a.N % 4 == 0 && a.K % 4 == 0 && a.ln_g &&
                   a.ln_stats && a.ldc % 4 == 0 && ((uintptr_t)a.C & 15u) == 0 && ((uintptr_t)a.ln_g & 15u) == 0,
               "gemm: LayerNorm epilogue needs one row tile (N=%d <= 256), float4 operands, K %% 4 == 0", a.N);
  const bool kt = a.K % 32 != 0, narrow = a.N <= 128;
  if (epi == EPI_RES_LN) {
    XTRL_REQUIRE(!trans_b && res && a.ln_y1 && a.ldr % 4 == 0 && a.ln_ld1 % 4 == 0 && (!a.ln_y2 || a.ln_ld2 % 4 == 0) &&
                     (!a.bias || ((uintptr_t)a.bias & 15u) == 0) && (!a.ln_b || ((uintptr_t)a.ln_b & 15u) == 0) &&
                     (!a.ln_b2 || (a.ln_y2 && ((uintptr_t)a.ln_b2 & 15u) == 0)),
                 "gemm: residual + LayerNorm epilogue arguments");
    if (narrow) {
      if (kt) launch_ws<false, false, EPI_RES_LN, true, 128, 128, true>(a, s);
      else launch_ws<false, false, EPI_RES_LN, true, 128, 128, false>(a, s);
    } else {
      if (kt) launch_ws<false, false, EPI_RES_LN, true, 64, 256, true>(a, s);
      else launch_ws<false, false, EPI_RES_LN, true, 64, 256, false>(a, s);
    }
  } else if (epi == EPI_LN_BWD) {
    XTRL_REQUIRE(trans_b && !res && a.ln_x && a.ln_part, "gemm: LayerNorm-backward epilogue arguments");
    if (narrow) launch_ws<false, true, EPI_LN_BWD, false, 128, 128, true>(a, s);
    else launch_ws<false, true, EPI_LN_BWD, false, 64, 256, true>(a, s);
  } else {
    XTRL_REQUIRE(trans_b && !res && a.ln_x && a.ln_part && (!a.ln_gpre || ((uintptr_t)a.ln_gpre & 15u) == 0) &&
                     a.ln_ldg % 4 == 0 &&
                     (!a.ln2_out || (a.ln2_g && a.ln2_x && a.ln2_stats && a.ln2_part && a.ln2_part_b &&
                                     ((uintptr_t)a.ln2_out & 15u) == 0 && ((uintptr_t)a.ln2_g & 15u) == 0)) &&
                     a.ldc == a.N,
                 "gemm: post-norm LayerNorm-backward epilogue arguments");
    if (narrow) launch_ws<false, true, EPI_LN_BWD2, false, 128, 128, true>(a, s);
    else launch_ws<false, true, EPI_LN_BWD2, false, 64, 256, true>(a, s);
  }
  XTRL_LAUNCHED("gemm_ln");
  return XTRL_OK;
}

bool use_x6() {   // XTRL_GEMM_F32=1: native f32 MFMA products everywhere
  static const bool x6 = [] {
    const char* e = getenv("XTRL_GEMM_F32");
    return !(e && atoi(e) != 0);
  }();
  return x6;
}

// geometry: 128 x 128 tiles (2 x 2 waves of 64 x 64, four accumulator chains each) when they fill
// the chip, else 64 x 64 tiles, else (decode-sized M) 64 x 32 tiles with a 2-way or 32 x 32 tiles
// with a 4-way split of K inside the workgroup.  Operands whose contiguous extent is not a multiple of 4 (or unaligned) take
// the scalar-load variant, instantiated for the 64 x 64 geometry only.
int forced_geom() {   // XTRL_GEMM_GEOM=<n> (tuning experiments): force geometry n for VEC launches
  static int g = [] {
    const char* e = getenv("XTRL_GEMM_GEOM");
    return e ? atoi(e) : -1;
  }();
  return g;
}

template <bool TA, bool TB, int EPI, bool LN, bool RES>
void dispatch_geom(const GemmArgs& a, bool vec, hipStream_t s) {
  const int64_t tiles128 = (int64_t)((a.M + 127) / 128) * ((a.N + 127) / 128);
  const int64_t tiles64 = (int64_t)((a.M + 63) / 64) * ((a.N + 63) / 64);
  const int fg = vec ? forced_geom() : -1;
  if (fg >= 0 && !TA) {
    switch (fg) {
      case 0: launch<1, 1, 4, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 1: launch<2, 2, 1, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 2: launch<2, 2, 1, 2, 2, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 3: launch<1, 1, 2, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 4: launch<1, 2, 2, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 5: launch<2, 1, 2, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 6: launch<1, 1, 8, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      case 7: launch<1, 2, 4, 1, 1, TA, TB, EPI, LN, RES, true>(a, s); return;
      default: break;
    }
  }
  // (decode-sized M measured on MI355X, graph-timed: M=1024 N=1024 K=256 64x64 11.6 us vs
  //  32x32/WK4 17.4; N=260 K=256 64x32/WK2 7.7 vs 8.2; N=256 K=1024 32x32/WK4 13.7 vs 64x64 24.7)
  // (learn shapes, tools/geom_probe.py learn: N <= 32 outputs over 16384 rows 64x32/WK2 9.8-10.8 us vs
  //  64x64 13.3 / 32x32-WK4 14.9; K = 64 64x64 12.3 vs 128x128 14.0)
  if (!vec) launch<2, 2, 1, 1, 1, TA, TB, EPI, LN, RES, false>(a, s);
  else if (!TA && a.N <= 32 && a.M >= 4096) launch<2, 1, 2, 1, 1, TA, TB, EPI, LN, RES, true>(a, s);
  else if (tiles128 >= 192 && a.K > 64) {
    bool done = false;
    if constexpr (EPI != EPI_DGATE && !LN) {   // (the gate epilogue needs more than 256 registers)
      if (use_x6() && ws_ok(a, TA, LN) && a.K % 32 == 0) {
        launch_ws<TA, TB, EPI, RES>(a, s);
        done = true;
      }
    }
    if (done) {
    } else if (use_x6()) launch<2, 2, 1, 2, 2, TA, TB, EPI, LN, RES, true, true>(a, s);
    else launch<2, 2, 1, 2, 2, TA, TB, EPI, LN, RES, true>(a, s);
  }
  else if (tiles64 >= 256 && a.K <= 512) {
    bool done = false;
    // 64 x 64 tiles with split-bf16 products (XTRL_GEMM_X6_SMALL=0: f32); "N" operands only (the
    // transposed staging needs whole 4 x 4 groups per thread)
    if constexpr (!TA && !TB && EPI != EPI_DGATE) {
      if (use_x6() && use_x6_small()) {
        launch<2, 2, 1, 1, 1, TA, TB, EPI, LN, RES, true, true>(a, s);
        done = true;
      }
    }
    if (!done) launch<2, 2, 1, 1, 1, TA, TB, EPI, LN, RES, true>(a, s);
  }
  else if (a.K <= 256) launch<2, 1, 2, 1, 1, TA, TB, EPI, LN, RES, true>(a, s);
  else launch<1, 1, 4, 1, 1, TA, TB, EPI, LN, RES, true>(a, s);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// host restatement of epi_v4_ok for the GELU + dropout epilogue (C and aux_out; no split-K / t_dev
// offset on this epilogue's launches): the split-bf16 kernels compile only the row-vector form of it
bool gelu_drop_v4_host(const GemmArgs& a) {
  return (a.N & 3) == 0 && (a.ldc & 3) == 0 && aligned16(a.C) && (a.ld_aux_out & 3) == 0 && aligned16(a.aux_out) &&
         !a.t_dev && a.kspan == 0;
}
int round4(int x) { return (x + 3) & ~3; }

}  // namespace

int gemm_ln_rows(int N) { return N <= 128 ? 128 : 64; }

int gemm_run(const GemmArgs& a, int trans_a, int trans_b, int epi, hipStream_t s) {
  XTRL_REQUIRE(a.A && a.B && a.C, "gemm: null operand");
  XTRL_REQUIRE(a.M >= 0 && a.N >= 0 && a.K > 0, "gemm: bad shape M=%d N=%d K=%d", a.M, a.N, a.K);
  XTRL_REQUIRE(a.lda >= (trans_a ? a.M : a.K) && a.ldb >= (trans_b ? a.N : a.K) && a.ldc >= a.N,
               "gemm: leading dims too small");
  XTRL_REQUIRE(!(a.gamma && trans_a), "gemm: LayerNorm prologue needs a row-major A");
  XTRL_REQUIRE(!((epi == EPI_GELU_DROP || epi == EPI_SILU_SAVE || epi == EPI_DGATE) && !a.aux_out),
               "gemm: epilogue %d needs aux_out", epi);
  XTRL_REQUIRE(!((epi == EPI_MUL_AUX || epi == EPI_DGATE || epi == EPI_MASK_POS) && !a.aux_in),
               "gemm: epilogue %d needs aux_in", epi);
  XTRL_REQUIRE(!(epi == EPI_DGATE && !a.aux_in2), "gemm: gate epilogue needs aux_in2");
  if (a.M == 0 || a.N == 0) return XTRL_OK;
  // float4 staging: 16-byte aligned operands whose leading dimensions are multiples of 4 and cover
  // the contiguous extent rounded up to 4 (a ragged extent such as K = d + 1 then reads in-bounds
  // padding of the row; see load4)
  const bool vec = aligned16(a.A) && aligned16(a.B) && (a.lda % 4 == 0) && (a.ldb % 4 == 0) &&
                   a.lda >= round4(trans_a ? a.M : a.K) && a.ldb >= round4(trans_b ? a.N : a.K);
  const bool ln = a.gamma != nullptr, res = a.R != nullptr;
  // (the split-bf16 GELU + dropout kernels have only the row-vector epilogue: other layouts take the
  // scalar-load kernel)
  if (epi == EPI_RES_LN || epi == EPI_LN_BWD || epi == EPI_LN_BWD2) return ln_gemm_run(a, trans_a, trans_b, epi, vec, s);
  const bool vec_k = vec && (epi != EPI_GELU_DROP || gelu_drop_v4_host(a));
#define XG(TA_, TB_, E_, L_, R_)                                                                   \
  if (trans_a == TA_ && trans_b == TB_ && epi == E_ && ln == L_ && res == R_) {                    \
    dispatch_geom<TA_, TB_, E_, L_, R_>(a, vec_k, s);                                              \
    XTRL_LAUNCHED("gemm_f32");                                                                     \
    return XTRL_OK;                                                                                \
  }
  // forward / decode (A row-major, B = nn.Linear weight)
  XG(0, 0, EPI_NONE, false, false)
  XG(0, 0, EPI_NONE, false, true)
  XG(0, 0, EPI_NONE, true, false)
  XG(0, 0, EPI_GELU, true, false)
  XG(0, 0, EPI_GELU, false, false)
  XG(0, 0, EPI_SILU, false, false)
  XG(0, 0, EPI_RELU, false, false)
  XG(0, 0, EPI_GELU_DROP, false, false)
  XG(0, 0, EPI_SILU_SAVE, false, false)
  // dgrad (B = weight used as [k][n]) with fused activation / dropout / gate backward
  XG(0, 1, EPI_NONE, false, false)
  XG(0, 1, EPI_NONE, false, true)       // input gradient + a residual-path gradient (fractal post-norm blocks)
  XG(0, 1, EPI_MASK_POS, false, false)  // input gradient through a ReLU (fractal final aggregation)
  XG(0, 1, EPI_MUL_AUX, false, false)
  XG(0, 1, EPI_DGATE, false, false)
  // wgrad (A = dY^T)
  XG(1, 1, EPI_NONE, false, false)
#undef XG
  set_error("gemm: unsupported combination ta=%d tb=%d epi=%d ln=%d residual=%d", trans_a, trans_b, epi, (int)ln,
            (int)res);
  return XTRL_E_ARG;
}

int gemm_ex(int trans_a, int trans_b, const float* A, int lda, const float* B, int ldb, const float* bias,
            const float* ln_gamma, const float* R, int ldr, float* C, int ldc, const int32_t* t_dev,
            int64_t c_t_stride, int M, int N, int K, int act, float beta, hipStream_t s) {
  XTRL_REQUIRE(act >= 0 && act <= 3, "gemm: bad activation %d", act);
  if (act == 3) act = EPI_RELU;
  GemmArgs a;
  a.A = A; a.B = B; a.bias = bias; a.gamma = ln_gamma; a.R = R; a.C = C; a.t_dev = t_dev;
  a.c_t_stride = c_t_stride; a.lda = lda; a.ldb = ldb; a.ldr = ldr; a.ldc = ldc; a.M = M; a.N = N; a.K = K;
  a.beta = beta;
  return gemm_run(a, trans_a, trans_b, act, s);
}

// ---- skinny weight gradients: dW [N][K] (+ db) where one side — N, or K plus the bias column — is
// at most 32 and the other at most 512 (the state / world-model heads: to_state_embed and
// project_in over the [states | reward] rows of S + 1 floats, to_pred's 2 (S + 1) outputs, the
// actor's action logits).  The 64 x 64 GEMM tile wastes most of its MFMA work on these and, with
// rows off the float4 grid, stages them with scalar loads: 58-123 us a launch at C3, on the side
// stream that bounds the backward's tail.  Here each workgroup owns `span` tokens: it stages SKW_R
// token rows of dY and X (+ a ones column for the bias) in LDS, a lane owns one index of the long
// side and accumulates the whole short side against LDS broadcasts (S FMAs per lane-row), and the
// workgroup's partial goes to ws in the split-K layout ([split][N][K] + bias rows [split][N]), so
// the same fixed-order reduction (immediate or deferred) finishes it.  Deterministic; the products
// are plain fp32 FMAs (a token span of 64 per partial, then the reduction's fixed tree).
constexpr int SKW_R = 64;   // token rows staged per LDS round (the whole default span: one round)
template <bool TALL, int S, int LJ>
__global__ __launch_bounds__(256) void k_wgrad_skinny(const float* __restrict__ dY, int ldy, const float* __restrict__ X,
                                                      int ldx, int M, int N, int K, int bias, int span,
                                                      float* __restrict__ P, float* __restrict__ PR) {
  constexpr int R = SKW_R / LJ;   // (the two-index lanes stage half the rows: registers)
  extern __shared__ float skw_lds[];
  const int tid = threadIdx.x, Kx = K + bias;
  const int YS = (N + 3) & ~3, XS = (Kx + 3) & ~3;   // LDS row strides (the broadcast side reads float4)
  float* Ys = skw_lds;
  // (pads: a lane past the long side, and the broadcast past the short side, read in-bounds)
  float* Xs = skw_lds + R * YS + (TALL ? 0 : 256 * LJ);
  const int t_lo = blockIdx.x * span, t_hi = min(M, t_lo + span);
  // a round: the long side lane-per-column (row offsets uniform: every load of a lane in flight at
  // once), the short side flat over its [R][cols] block; rows past the span stage zeros
  auto stage = [&](int t0) {
    const float* Lg = TALL ? dY : X;
    const int ldl = TALL ? ldy : ldx, Ln = TALL ? N : Kx, LSd = TALL ? YS : XS;
    float* Ld = TALL ? Ys : Xs;
#pragma unroll
    for (int j = 0; j < LJ; ++j) {
      const int c = tid + 256 * j;
      const bool in = c < Ln, ld = in && (TALL || c < K);
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = (t0 + r < t_hi && ld) ? Lg[(int64_t)(t0 + r) * ldl + c] : 0.f;
      if (!TALL && c == K)   // the bias column
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = t0 + r < t_hi ? 1.f : 0.f;
      if (in)
#pragma unroll
        for (int r = 0; r < R; ++r) Ld[r * LSd + c] = v[r];
    }
    const float* Sg = TALL ? X : dY;
    const int lds_ = TALL ? ldx : ldy, Sn = TALL ? Kx : N, SSd = TALL ? XS : YS;
    float* Sd = TALL ? Xs : Ys;
    for (int e = tid; e < R * Sn; e += 256) {
      const int r = e / Sn, c = e - r * Sn, t = t0 + r;
      float v = 0.f;
      if (t < t_hi) v = (!TALL || c < K) ? Sg[(int64_t)t * lds_ + c] : 1.f;   // (TALL: the bias column)
      Sd[r * SSd + c] = v;
    }
  };
  float acc[LJ][S];
#pragma unroll
  for (int j = 0; j < LJ; ++j)
#pragma unroll
    for (int c = 0; c < S; ++c) acc[j][c] = 0.f;
  const float* Ls = TALL ? Ys : Xs;   // the long side: one lane per index
  const float* Bs = TALL ? Xs : Ys;   // the short side: LDS broadcasts
  const int LS = TALL ? YS : XS, BSd = TALL ? XS : YS;
  for (int t0 = t_lo; t0 < t_hi; t0 += R) {
    if (t0 > t_lo) __syncthreads();   // the previous round's reads are done
    stage(t0);
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < R; ++r) {
      float b[S];
#pragma unroll
      for (int c4 = 0; c4 < S / 4; ++c4) {
        const float4 v = *reinterpret_cast<const float4*>(Bs + r * BSd + 4 * c4);
        b[4 * c4] = v.x; b[4 * c4 + 1] = v.y; b[4 * c4 + 2] = v.z; b[4 * c4 + 3] = v.w;
      }
#pragma unroll
      for (int j = 0; j < LJ; ++j) {
        const float l = Ls[r * LS + tid + 256 * j];
#pragma unroll
        for (int c = 0; c < S; ++c) acc[j][c] = fmaf(l, b[c], acc[j][c]);
      }
    }
  }
  // partial [split][N][K] (+ bias rows [split][N])
  float* Pb = P + (int64_t)blockIdx.x * N * K;
#pragma unroll
  for (int j = 0; j < LJ; ++j) {
    const int li = tid + 256 * j;
    if (TALL) {
      if (li < N) {
#pragma unroll
        for (int c = 0; c < S; ++c) {
          if (c < K) Pb[(int64_t)li * K + c] = acc[j][c];
          else if (c == K && bias) PR[(int64_t)blockIdx.x * N + li] = acc[j][c];
        }
      }
    } else if (li < Kx) {
#pragma unroll
      for (int c = 0; c < S; ++c) {
        if (c < N) {
          if (li < K) Pb[(int64_t)c * K + li] = acc[j][c];
          else PR[(int64_t)blockIdx.x * N + c] = acc[j][c];
        }
      }
    }
  }
}

// the skinny shape class of a weight gradient (0: not skinny), see k_wgrad_skinny
struct SkinnyPick {
  bool tall = false;
  int S = 0, LJ = 0;
};
static SkinnyPick skinny_pick(int N, int Kx) {
  SkinnyPick p;
  static const bool on = [] {   // XTRL_WGRAD_SKINNY=0: the 64 x 64 GEMM for these too
    const char* e = getenv("XTRL_WGRAD_SKINNY");
    return !(e && atoi(e) == 0);
  }();
  if (!on) return p;
  auto s_of = [](int x) { return x <= 4 ? 4 : x <= 8 ? 8 : x <= 12 ? 12 : x <= 16 ? 16 : x <= 24 ? 24 : x <= 32 ? 32 : 0; };
  if (Kx <= N && s_of(Kx) && N <= 512) {
    p.tall = true; p.S = s_of(Kx); p.LJ = (N + 255) / 256;
  } else if (N < Kx && s_of(N) && Kx <= 512) {
    p.tall = false; p.S = s_of(N); p.LJ = (Kx + 255) / 256;
  }
  return p;
}
static void launch_skinny(const SkinnyPick& p, const float* dY, int ldy, const float* X, int ldx, int M, int N, int K,
                          int bias, int span, int splits, float* P, float* PR, hipStream_t s) {
  const int Kx = K + bias, YS = (N + 3) & ~3, XS = (Kx + 3) & ~3;
  const size_t lds = sizeof(float) * ((size_t)SKW_R * (YS + XS) + 512 * p.LJ + 32);
  const dim3 g(splits), b(256);
#define SKW(T, SS, L)                                                                                   \
  if (p.tall == T && p.S == SS && p.LJ == L) {                                                          \
    hipLaunchKernelGGL((k_wgrad_skinny<T, SS, L>), g, b, lds, s, dY, ldy, X, ldx, M, N, K, bias, span, P, PR); \
    return;                                                                                             \
  }
#define SKW_L(T, L) SKW(T, 4, L) SKW(T, 8, L) SKW(T, 12, L) SKW(T, 16, L) SKW(T, 24, L) SKW(T, 32, L)
  SKW_L(true, 1) SKW_L(true, 2) SKW_L(false, 1) SKW_L(false, 2)
#undef SKW_L
#undef SKW
}

// phase 2 of k_wgrad_skinny: dW = beta dW + sum_z P[z], db[n - m0] += sum_z PR[z][n].  A workgroup
// per 64 consecutive outputs; wave w sums the splits z = w, w + 4, ... (16 loads in flight), the
// four wave sums combine in LDS in a fixed order (deterministic)
__global__ __launch_bounds__(256) void k_skinny_reduce(const float* __restrict__ P, const float* __restrict__ PR, int S,
                                                       int N, int K, float* dW, int ldw, float beta, float* db, int m0) {
  __shared__ float part[4][64];
  const int NK = N * K, nbw = (NK + 63) / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool isb = (int)blockIdx.x >= nbw;
  const int o = ((int)blockIdx.x - (isb ? nbw : 0)) * 64 + lane;
  const int len = isb ? N : NK;
  const float* src = isb ? PR : P;
  constexpr int U = 16;
  float acc = 0.f;
  if (o < len) {
    for (int z0 = w; z0 < S; z0 += 4 * U) {
      float p[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int z = z0 + 4 * u;
        p[u] = z < S ? src[(int64_t)z * len + o] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += p[u];
    }
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w == 0 && o < len) {
    const float sum = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (isb) {
      if (o >= m0) db[o - m0] += sum;
    } else {
      const int n = o / K, k = o - n * K;
      float* d = dW + (int64_t)n * ldw + k;
      *d = beta != 0.f ? beta * *d + sum : sum;
    }
  }
}

// weight gradient dW[N][K] = beta dW + sum_m dY[m][n] X[m][k] (reduction over the M tokens):
// split the token range over workgroups (partial 64x64 tiles in ws), then a fixed-order sum
int splitk_flush(SplitKQueue& q, hipStream_t s) {
  if (q.n == 0) return XTRL_OK;
  SplitKJobs J;
  J.n = q.n;
  J.total_q = J.total_r = 0;
  for (int j = 0; j < q.n; ++j) {
    J.job[j] = q.job[j];
    J.job[j].q0 = J.total_q;
    J.job[j].r0 = J.total_r;
    J.total_q += (int64_t)q.job[j].M * q.job[j].N / 4;
    J.total_r += q.job[j].rowsum ? q.job[j].M - q.job[j].m0 : 0;
  }
  const int64_t units = J.total_q + J.total_r;
  hipLaunchKernelGGL(k_splitk_reduce_multi, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((units + 255) / 256, 8192))),
                     dim3(256), 0, s, J);
  q.n = 0;
  q.used = 0;
  XTRL_LAUNCHED("splitk_flush");
  return XTRL_OK;
}

int gemm_wgrad(const float* dY, int ldy, const float* X, int ldx, float* dW, int ldw, int M, int N, int K, float beta,
               float* ws, int64_t ws_floats, hipStream_t s, float* db, int db_n0, const GemmProfile* prof,
               SplitKQueue* defer) {
  XTRL_REQUIRE(dY && X && dW && M > 0 && N > 0 && K > 0, "gemm_wgrad: bad arguments");
  XTRL_REQUIRE(ldy >= N && ldx >= K && ldw >= K, "gemm_wgrad: leading dims too small");
  XTRL_REQUIRE(!db || beta == 1.f, "gemm_wgrad: the bias gradient accumulates (beta = 1)");
  // skinny shapes (k_wgrad_skinny): a workgroup per `span` tokens (XTRL_SKINNY_SPAN, default 64; at
  // most 1024 partials), reduced at once behind any queued split-K partials in ws
  if (const SkinnyPick sk = ws ? skinny_pick(N, K + (db ? 1 : 0)) : SkinnyPick{}; sk.S && M >= 64) {
    static const int sk_span = [] {
      const char* e = getenv("XTRL_SKINNY_SPAN");
      return std::max(32, ((e ? atoi(e) : 64) + 31) / 32 * 32);
    }();
    int span = std::max(sk_span, (int)(((M + 1023) / 1024 + 31) / 32 * 32));
    int sp = (M + span - 1) / span;
    const int64_t per = (int64_t)N * K + (db ? N : 0);
    float* w = ws;
    int64_t wf = ws_floats;
    if (defer && defer->n > 0) {
      bool overlap = false;   // a queued job that writes this dW / db sums first (its beta may be 0)
      for (int j = 0; j < defer->n; ++j) {
        const SplitKJob& o = defer->job[j];
        const float *a0 = dW, *a1 = dW + (int64_t)(N - 1) * ldw + K, *b0 = o.C, *b1 = o.C + (int64_t)(o.M - 1) * o.ldc + o.N;
        if (a0 < b1 && b0 < a1) overlap = true;
        if (db && o.rowsum && db < o.rowsum + (o.M - o.m0) && o.rowsum < db + (N - db_n0)) overlap = true;
      }
      if (overlap) {
        if (int rc = splitk_flush(*defer, s)) return rc;
      }
      w += defer->used;
      wf -= defer->used;
    }
    while (sp > 1 && sp * per > wf) {
      span *= 2;
      sp = (M + span - 1) / span;
    }
    if (sp * per <= wf) {
      launch_skinny(sk, dY, ldy, X, ldx, M, N, K, db ? 1 : 0, span, sp, w, w + (int64_t)sp * N * K, s);
      const int nbw = (N * K + 63) / 64, nbb = db ? (N + 63) / 64 : 0;
      hipLaunchKernelGGL(k_skinny_reduce, dim3(nbw + nbb), dim3(256), 0, s, (const float*)w,
                         (const float*)(w + (int64_t)sp * N * K), sp, N, K, dW, ldw, beta, db, db_n0);
      XTRL_LAUNCHED("gemm_wgrad (skinny)");
      return XTRL_OK;
    }
  }
  // GEMM view: C = dW [N x K], A[n][m] = dY[m][n] ("T", lda = ldy), B[m][k] = X[m][k] ("T", ldb = ldx)
  // 128 x 128 tiles (2 workgroups / CU by registers) when the weight is large, else 64 x 64 (4 / CU);
  // split the tokens until 192 workgroups (three quarters of a resident round: the learn step runs
  // these on a side stream beside the input-gradient chain, whose kernels take the free CUs; A/B on
  // one box, learn ms: 256 / 224 / 192 / 160 / 128 workgroups = 130.0 / 129.5 / 128.6 / 128.6 / 130.1)
  // keeping at least 8 K-slabs (256 tokens) per split so the pipeline
  // reaches steady state (more splits cost more partial-tile traffic in phase 2 than they save)
  const bool big = (int64_t)N * K >= 256 * 256;
  const int tm = big ? 128 : 64;
  const int64_t tiles = (int64_t)((N + tm - 1) / tm) * ((K + tm - 1) / tm);
  static const int64_t big_target = [] {   // XTRL_WGRAD_TARGET: workgroups of the 128 x 128 launch
    const char* e = getenv("XTRL_WGRAD_TARGET");
    return (int64_t)(e ? atoi(e) : 192);
  }();
  const int64_t target = big ? big_target : 1024;
  int splits = (int)std::max<int64_t>(1, std::min<int64_t>((target + tiles - 1) / tiles, (M + 255) / 256));
  int kspan = ((M + splits - 1) / splits + 31) / 32 * 32;
  splits = (M + kspan - 1) / kspan;
  auto need = [&](int sp) { return (int64_t)sp * N * K + (db ? (int64_t)sp * N : 0); };
  // deferred reduction: float4 element groups, and a dW no queued job also writes (jobs of one
  // launch run concurrently); the partials go behind the queued jobs' in ws
  bool deferred = defer && splits > 1 && K % 4 == 0 && ldw % 4 == 0 && aligned16(dW);
  if (deferred)
    for (int j = 0; j < defer->n; ++j) {
      const SplitKJob& o = defer->job[j];
      const float *a0 = dW, *a1 = dW + (int64_t)(N - 1) * ldw + K, *b0 = o.C, *b1 = o.C + (int64_t)(o.M - 1) * o.ldc + o.N;
      if (a0 < b1 && b0 < a1) deferred = false;
      if (db && o.rowsum && db < o.rowsum + (o.M - o.m0) && o.rowsum < db + (N - db_n0)) deferred = false;
    }
  if (deferred && (defer->n == kMaxSplitKJobs || defer->used + need(splits) > ws_floats)) {
    if (int rc = splitk_flush(*defer, s)) return rc;   // the queued partials are summed first
  }
  // a split that is not queued reduces at once from the front of ws, where queued partials lie
  // (and may accumulate into a dW a queued job also writes): sum the queue first
  if (defer && !deferred && splits > 1 && defer->n > 0)
    if (int rc = splitk_flush(*defer, s)) return rc;
  if (deferred) {
    ws += defer->used;
    ws_floats -= defer->used;
  }
  while (splits > 1 && need(splits) > ws_floats) {   // fit the partial slabs in ws
    splits = std::max(1, splits / 2);
    kspan = ((M + splits - 1) / splits + 31) / 32 * 32;
    splits = (M + kspan - 1) / kspan;
  }
  const bool vec = aligned16(dY) && aligned16(X) && (ldy % 4 == 0) && (ldx % 4 == 0) && ldy >= round4(N) &&
                   ldx >= round4(K);
  GemmArgs a;
  a.A = dY; a.B = X; a.C = dW; a.lda = ldy; a.ldb = ldx; a.ldc = ldw; a.M = N; a.N = K; a.K = M; a.beta = beta;
  a.rowsum = db;
  a.rowsum_m0 = db_n0;
  if (splits > 1) {
    XTRL_REQUIRE(ws && need(splits) <= ws_floats, "gemm_wgrad: workspace too small");
    a.C = ws;
    a.ldc = K;
    a.beta = 0.f;
    a.kspan = kspan;
    a.c_split = (int64_t)N * K;
    a.rowsum_ws = ws + (int64_t)splits * N * K;
  }
  if (!vec) launch<2, 2, 1, 1, 1, true, true, EPI_NONE, false, false, false>(a, s);
  else if (big) {
    const bool timed = prof && prof->events && *prof->n < prof->cap;
    if (timed) (void)hipEventRecord((hipEvent_t)prof->events[2 * *prof->n], s);
    static const bool wgrad_ws = [] {   // XTRL_WGRAD_WS=0: register-staged kernel for weight gradients
      const char* e = getenv("XTRL_WGRAD_WS");
      return !(e && atoi(e) == 0);
    }();
    if (use_x6() && wgrad_ws && ws_ok(a, true, false)) {
      if (a.K % 32 == 0) launch_ws<true, true, EPI_NONE, false>(a, s);
      else launch_ws<true, true, EPI_NONE, false, 128, 128, true>(a, s);
    }
    else if (use_x6()) launch<2, 2, 1, 2, 2, true, true, EPI_NONE, false, false, true, true>(a, s);
    else launch<2, 2, 1, 2, 2, true, true, EPI_NONE, false, false, true>(a, s);
    if (timed) {
      (void)hipEventRecord((hipEvent_t)prof->events[2 * *prof->n + 1], s);
      prof->flops[*prof->n] = 2.0 * (double)M * (double)N * (double)K;
      ++*prof->n;
    }
  } else launch<2, 2, 1, 1, 1, true, true, EPI_NONE, false, false, true>(a, s);
  if (splits > 1 && deferred) {
    SplitKJob& j = defer->job[defer->n++];
    j.ws = ws; j.C = dW; j.rws = a.rowsum_ws; j.rowsum = db; j.S = splits; j.M = N; j.N = K; j.ldc = ldw;
    j.m0 = db_n0; j.beta = beta; j.q0 = j.r0 = 0;
    defer->used += need(splits);
  } else if (splits > 1) {
    const int64_t MN = (int64_t)N * K;
    const int64_t units = MN;   // scalar path: a thread per element; float4 path: four lanes per float4
    hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((units + 255) / 256, 4096))),
                       dim3(256), 0, s, ws, splits, N, K, dW, ldw, beta, a.rowsum_ws, db, db_n0);
  }
  XTRL_LAUNCHED("gemm_wgrad");
  return XTRL_OK;
}

int gemm_f32(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* ln_gamma,
             const float* R, int ldr, float* Y, int ldy, const int32_t* t_dev, int64_t y_t_stride, int M, int N,
             int K, int act, hipStream_t s) {
  return gemm_ex(0, 0, X, ldx, W, ldw, bias, ln_gamma, R, ldr, Y, ldy, t_dev, y_t_stride, M, N, K, act, 0.f, s);
}

int layernorm_f32(const float* X, int ldx, const float* gamma, float* Y, int ldy, int M, int D, hipStream_t s) {
  XTRL_REQUIRE(X && gamma && Y && M >= 0 && D > 0, "layernorm: bad arguments");
  if (M == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_layernorm, dim3((M + 3) / 4), dim3(256), 0, s, X, ldx, gamma, Y, ldy, M, D);
  XTRL_LAUNCHED("layernorm_f32");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_gemm_f32(const float* X, int ldx, const float* W, int ldw, const float* bias,
                             const float* ln_gamma, const float* R, int ldr, float* Y, int ldy,
                             const int32_t* t_dev, int64_t y_t_stride, int M, int N, int K, int act, void* stream) {
  return xtrl::gemm_f32(X, ldx, W, ldw, bias, ln_gamma, R, ldr, Y, ldy, t_dev, y_t_stride, M, N, K, act,
                        xtrl::as_stream(stream));
}

extern "C" int xtrl_gemm_ex(int trans_a, int trans_b, const float* A, int lda, const float* B, int ldb,
                            const float* bias, float* C, int ldc, int M, int N, int K, float beta, void* stream) {
  return xtrl::gemm_ex(trans_a, trans_b, A, lda, B, ldb, bias, nullptr, nullptr, 0, C, ldc, nullptr, 0, M, N, K,
                       XTRL_ACT_NONE, beta, xtrl::as_stream(stream));
}

extern "C" int xtrl_gemm_wgrad(const float* dY, int ldy, const float* X, int ldx, float* dW, int ldw, int M, int N,
                               int K, float beta, float* ws, int64_t ws_floats, void* stream) {
  return xtrl::gemm_wgrad(dY, ldy, X, ldx, dW, ldw, M, N, K, beta, ws, ws_floats, xtrl::as_stream(stream), nullptr, 0);
}

extern "C" int xtrl_gemm_wgrad_db(const float* dY, int ldy, const float* X, int ldx, float* dW, int ldw, int M,
                                  int N, int K, float beta, float* ws, int64_t ws_floats, float* db, int db_n0,
                                  void* stream) {
  return xtrl::gemm_wgrad(dY, ldy, X, ldx, dW, ldw, M, N, K, beta, ws, ws_floats, xtrl::as_stream(stream), db, db_n0);
}

extern "C" int xtrl_layernorm_f32(const float* X, int ldx, const float* gamma, float* Y, int ldy, int M, int D,
                                  void* stream) {
  return xtrl::layernorm_f32(X, ldx, gamma, Y, ldy, M, D, xtrl::as_stream(stream));
}
