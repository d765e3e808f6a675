// Fused fp32 GEMM on the CDNA4 f32 matrix cores (v_mfma_f32_32x32x2_f32, exact f32 products).
//
//   Y[m, n] = act( LN?(X)[m, :] . W[n, :] + bias[n] ) (+ R[m, n])
//
// Tile: 64 x 64 output per 256-thread workgroup, 2 x 2 waves of 32 x 32, BK = 16.  Operands are
// staged k-major in LDS ([BK][64 + 4]) so that an MFMA fragment read (lane l -> row l & 31,
// k = l >> 5) is 32 consecutive dwords per half-wave: conflict-free ds_read_b32.  Staging is
// register double-buffered: the next K-slab's global loads are issued before the current slab's
// MFMAs and written to the other LDS buffer after them (one barrier per K-step).
//
// The optional LayerNorm prologue (x-transformers LayerNorm: no affine, eps 1e-5, times gamma)
// computes per-row mean / rstd for the block's 64 rows (two-pass, in registers) and normalises
// the A operand while staging it, so pre-norm blocks need no separate normalisation pass.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace xtrl {

namespace {
constexpr int BM = 64, BN = 64, BK = 16, LDSW = BM + 4;

struct GemmArgs {
  const float* X;
  const float* W;
  const float* bias;
  const float* gamma;
  const float* R;
  float* Y;
  const int32_t* t_dev;
  int64_t y_t_stride;
  int ldx, ldw, ldr, ldy, M, N, K;
};

template <int ACT, bool LN, bool RES>
__global__ __launch_bounds__(256) void k_gemm_f32(const GemmArgs a) {
  __shared__ float As[2][BK][LDSW];
  __shared__ float Bs[2][BK][LDSW];
  __shared__ float row_mean[BM], row_rstd[BM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = a.M, N = a.N, K = a.K;

  if constexpr (LN) {
    // 16 rows per wave, two-pass mean / variance like F.layer_norm
    for (int rr = 0; rr < 16; ++rr) {
      const int r = wave * 16 + rr, m = m0 + r;
      float mean = 0.f, rstd = 0.f;
      if (m < M) {
        const float* xr = a.X + (int64_t)m * a.ldx;
        float s = 0.f;
        for (int k = lane; k < K; k += 64) s += xr[k];
        mean = wave_sum(s) / (float)K;
        float q = 0.f;
        for (int k = lane; k < K; k += 64) {
          const float dlt = xr[k] - mean;
          q += dlt * dlt;
        }
        const float var = wave_sum(q) / (float)K;
        rstd = 1.0f / sqrtf(var + 1e-5f);
      }
      if (lane == 0) {
        row_mean[r] = mean;
        row_rstd[r] = rstd;
      }
    }
    __syncthreads();
  }

  // staging: wave w loads k-columns [4w, 4w + 4) of the slab for all 64 rows (lane = row)
  const int sr = lane, sk = wave * 4;
  float4 ra, rb;
  auto load_slab = [&](int k0) {
    const int k = k0 + sk;
    {
      const int m = m0 + sr;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (m < M) {
        const float* p = a.X + (int64_t)m * a.ldx + k;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (k + c < K) v[c] = p[c];
        if constexpr (LN) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (k + c < K) v[c] = ((v[c] - row_mean[sr]) * row_rstd[sr]) * a.gamma[k + c];
        }
      }
      ra = make_float4(v[0], v[1], v[2], v[3]);
    }
    {
      const int n = n0 + sr;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (n < N) {
        const float* p = a.W + (int64_t)n * a.ldw + k;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (k + c < K) v[c] = p[c];
      }
      rb = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_slab = [&](int buf) {
    As[buf][sk + 0][sr] = ra.x;
    As[buf][sk + 1][sr] = ra.y;
    As[buf][sk + 2][sr] = ra.z;
    As[buf][sk + 3][sr] = ra.w;
    Bs[buf][sk + 0][sr] = rb.x;
    Bs[buf][sk + 1][sr] = rb.y;
    Bs[buf][sk + 2][sr] = rb.z;
    Bs[buf][sk + 3][sr] = rb.w;
  };

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  const int nk = (K + BK - 1) / BK;
  load_slab(0);
  store_slab(0);
  __syncthreads();
  const int fi = wm * 32 + (lane & 31), fj = wn * 32 + (lane & 31), fk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_slab((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float av = As[cur][kk + fk][fi];
      const float bv = Bs[cur][kk + fk][fj];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    if (kt + 1 < nk) store_slab(cur ^ 1);
    __syncthreads();
  }

  // epilogue: acc[r] -> row (r & 3) + 8 (r >> 2) + 4 (lane >> 5), col lane & 31
  float* Y = a.Y;
  if (a.t_dev) Y += (int64_t)(*a.t_dev) * a.y_t_stride;
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= N) return;
  const float bn = a.bias ? a.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < M) {
      float v = acc[r] + bn;
      if constexpr (ACT == XTRL_ACT_GELU) v = geluf_(v);
      if constexpr (ACT == XTRL_ACT_SILU) v = siluf_(v);
      if constexpr (RES) v = v + a.R[(int64_t)m * a.ldr + n];
      Y[(int64_t)m * a.ldy + n] = v;
    }
  }
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

template <int ACT, bool LN, bool RES>
void launch(const GemmArgs& a, hipStream_t s) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM);
  hipLaunchKernelGGL((k_gemm_f32<ACT, LN, RES>), grid, dim3(256), 0, s, a);
}

}  // namespace

int gemm_f32(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* ln_gamma,
             const float* R, int ldr, float* Y, int ldy, const int32_t* t_dev, int64_t y_t_stride, int M, int N,
             int K, int act, hipStream_t s) {
  XTRL_REQUIRE(X && W && Y, "gemm: null operand");
  XTRL_REQUIRE(M >= 0 && N >= 0 && K > 0, "gemm: bad shape M=%d N=%d K=%d", M, N, K);
  XTRL_REQUIRE(ldx >= K && ldw >= K && ldy >= N, "gemm: leading dims too small");
  XTRL_REQUIRE(act >= 0 && act <= 2, "gemm: bad activation %d", act);
  if (M == 0 || N == 0) return XTRL_OK;
  GemmArgs a{X, W, bias, ln_gamma, R, Y, t_dev, y_t_stride, ldx, ldw, ldr, ldy, M, N, K};
  const bool ln = ln_gamma != nullptr, res = R != nullptr;
#define XTRL_GEMM_CASE(A_, L_, R_) \
  if (act == A_ && ln == L_ && res == R_) { launch<A_, L_, R_>(a, s); XTRL_LAUNCHED("gemm_f32"); return XTRL_OK; }
  XTRL_GEMM_CASE(XTRL_ACT_NONE, false, false)
  XTRL_GEMM_CASE(XTRL_ACT_NONE, false, true)
  XTRL_GEMM_CASE(XTRL_ACT_NONE, true, false)
  XTRL_GEMM_CASE(XTRL_ACT_NONE, true, true)
  XTRL_GEMM_CASE(XTRL_ACT_GELU, false, false)
  XTRL_GEMM_CASE(XTRL_ACT_GELU, true, false)
  XTRL_GEMM_CASE(XTRL_ACT_SILU, false, false)
  XTRL_GEMM_CASE(XTRL_ACT_SILU, true, false)
#undef XTRL_GEMM_CASE
  set_error("gemm: unsupported combination act=%d ln=%d residual=%d", act, (int)ln, (int)res);
  return XTRL_E_ARG;
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

extern "C" int xtrl_layernorm_f32(const float* X, int ldx, const float* gamma, float* Y, int ldy, int M, int D,
                                  void* stream) {
  return xtrl::layernorm_f32(X, ldx, gamma, Y, ldy, M, D, xtrl::as_stream(stream));
}
