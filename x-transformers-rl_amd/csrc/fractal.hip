// Row kernels of the fractal encoder body (x_transformers_rl/fractal_rl.py), the §8(f)-3 policy
// body.  The encoder's matrix work runs on the library GEMM (gemm.hip) and the bidirectional
// attention kernel (attn.hip, xtrl_attn_fwd_tokens); what is left is row-wise:
//   xtrl_rows_add       y = x + v (x NULL: v)   level embedding (fractal_rl.py:312-314, :64-68)
//   xtrl_add_layernorm  y = LN(x + r) g + b     post-norm residual blocks (fractal_rl.py:127-136);
//                                               r_rep > 1 broadcasts one residual row over r_rep
//                                               rows (the cross-attention read of the one-token
//                                               global state, whose softmax over a single key is 1)
//   xtrl_seq_mean       y[b] = mean_i x[b, i]   einops reduce 'b n d -> b d' (fractal_rl.py:321, :338)
//   xtrl_safe_embed     SafeEmbedding           (x_transformers_rl.py:181-195)
//   xtrl_wm_post        Continuous.mean_variance + sigmoid done head (x_transformers_rl.py:224-241,
//                                               fractal_rl.py:402-406)
// Each row is one wave; a LayerNorm row (D <= 1024) stays in registers, sixteen floats per lane.
#include "kernels.h"

namespace xtrl {
namespace {

constexpr int RW = 4;   // rows (waves) per 256-thread block

__global__ __launch_bounds__(256) void k_rows_add(const float* x, int ldx, const float* v, float* y, int ldy, int M,
                                                  int D) {
  const int m = blockIdx.x * RW + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= M) return;
  for (int c = lane; c < D; c += 64) y[(int64_t)m * ldy + c] = (x ? x[(int64_t)m * ldx + c] : 0.f) + v[c];
}

// nn.LayerNorm(D) (eps, affine) of x + r; two-pass variance over the row held in registers
__global__ __launch_bounds__(256) void k_add_layernorm(const float* x, int ldx, const float* r, int ldr, int r_rep,
                                                       const float* g, const float* bta, float* y, int ldy, int M,
                                                       int D, float eps) {
  const int m = blockIdx.x * RW + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= M) return;
  const float* xr = x + (int64_t)m * ldx;
  const float* rr = r ? r + (int64_t)(m / r_rep) * ldr : nullptr;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? xr[c] + (rr ? rr[c] : 0.f) : 0.f;
    s += v[j];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = lane + 64 * j;
    const float d = c < D ? v[j] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = lane + 64 * j;
    if (c < D) y[(int64_t)m * ldy + c] = (v[j] - mean) * rstd * g[c] + (bta ? bta[c] : 0.f);
  }
}

// y[b][c] = mean over the n rows of sequence b (fixed summation order)
__global__ __launch_bounds__(256) void k_seq_mean(const float* x, int ldx, int B, int n, int D, float* y, int ldy) {
  const int col = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (col >= D || b >= B) return;
  const float* xb = x + (int64_t)b * n * ldx + col;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += xb[(int64_t)i * ldx];
  y[(int64_t)b * ldy + col] = s / (float)n;
}

__global__ __launch_bounds__(256) void k_safe_embed(const int32_t* actions, int M, const float* W, int D, float* y,
                                                    int ldy) {
  const int m = blockIdx.x * RW + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= M) return;
  const int a = actions[m];
  for (int c = lane; c < D; c += 64) y[(int64_t)m * ldy + c] = a >= 0 ? W[(int64_t)a * D + c] : 0.f;
}

// raw [M][2P] interleaved (mean, log-variance) pairs -> mean_var [2][M][P] with
// variance = exp(3 tanh(lv / 3)); done[m] = sigmoid(done_logit[m])
__global__ __launch_bounds__(256) void k_wm_post(const float* raw, int ldr, int M, int P, float* mean_var,
                                                 const float* done_logit, int ldd, float* done) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < M * P) {
    const int m = t / P, p = t - m * P;
    const float mu = raw[(int64_t)m * ldr + 2 * p], lv = raw[(int64_t)m * ldr + 2 * p + 1];
    mean_var[t] = mu;
    mean_var[(int64_t)M * P + t] = expf(tanhf(lv / 3.0f) * 3.0f);
  }
  if (done && t < M) done[t] = 1.0f / (1.0f + expf(-done_logit[(int64_t)t * ldd]));
}

}  // namespace

// launchers shared with the fractal decode step (decode.hip)
void rows_add_launch(const float* x, int ldx, const float* v, float* y, int ldy, int M, int D, hipStream_t s) {
  hipLaunchKernelGGL(k_rows_add, dim3((M + RW - 1) / RW), dim3(256), 0, s, x, ldx, v, y, ldy, M, D);
}
void add_layernorm_launch(const float* x, int ldx, const float* r, int ldr, const float* g, const float* b, float* y,
                          int ldy, int M, int D, float eps, hipStream_t s) {
  hipLaunchKernelGGL(k_add_layernorm, dim3((M + RW - 1) / RW), dim3(256), 0, s, x, ldx, r, ldr, 1, g, b, y, ldy, M, D,
                     eps);
}
}  // namespace xtrl

using namespace xtrl;

extern "C" int xtrl_rows_add(const float* x, int ldx, const float* v, float* y, int ldy, int M, int D, void* stream) {
  XTRL_REQUIRE(v && y && M >= 0 && D > 0 && (!x || ldx >= D) && ldy >= D, "rows_add: bad arguments");
  if (M == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_rows_add, dim3((M + RW - 1) / RW), dim3(256), 0, (hipStream_t)stream, x, ldx, v, y, ldy, M, D);
  XTRL_LAUNCHED("rows_add");
  return XTRL_OK;
}

extern "C" int xtrl_add_layernorm(const float* x, int ldx, const float* r, int ldr, int r_rep, const float* gamma,
                                  const float* beta, float* y, int ldy, int M, int D, float eps, void* stream) {
  XTRL_REQUIRE(x && gamma && y && M >= 0 && D > 0 && D <= 1024 && ldx >= D && ldy >= D,
               "add_layernorm: bad arguments (D <= 1024)");
  XTRL_REQUIRE(!r || (r_rep >= 1 && ldr >= (r_rep > 1 ? 0 : D)), "add_layernorm: bad residual");
  if (M == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_add_layernorm, dim3((M + RW - 1) / RW), dim3(256), 0, (hipStream_t)stream, x, ldx, r, ldr,
                     r_rep < 1 ? 1 : r_rep, gamma, beta, y, ldy, M, D, eps);
  XTRL_LAUNCHED("add_layernorm");
  return XTRL_OK;
}

extern "C" int xtrl_seq_mean(const float* x, int ldx, int B, int n, int D, float* y, int ldy, void* stream) {
  XTRL_REQUIRE(x && y && B >= 0 && n > 0 && D > 0 && ldx >= D && ldy >= D, "seq_mean: bad arguments");
  if (B == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_seq_mean, dim3((D + 255) / 256, B), dim3(256), 0, (hipStream_t)stream, x, ldx, B, n, D, y, ldy);
  XTRL_LAUNCHED("seq_mean");
  return XTRL_OK;
}

extern "C" int xtrl_safe_embed(const int32_t* actions, int M, const float* W, int D, float* y, int ldy,
                               void* stream) {
  XTRL_REQUIRE(actions && W && y && M >= 0 && D > 0 && ldy >= D, "safe_embed: bad arguments");
  if (M == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_safe_embed, dim3((M + RW - 1) / RW), dim3(256), 0, (hipStream_t)stream, actions, M, W, D, y,
                     ldy);
  XTRL_LAUNCHED("safe_embed");
  return XTRL_OK;
}

extern "C" int xtrl_wm_post(const float* raw, int ldr, int M, int P, float* mean_var, const float* done_logit,
                            int ldd, float* done, void* stream) {
  XTRL_REQUIRE(raw && mean_var && M >= 0 && P > 0 && ldr >= 2 * P, "wm_post: bad arguments");
  XTRL_REQUIRE(!done || done_logit, "wm_post: done needs done_logit");
  const int units = M * P > M ? M * P : M;
  if (units == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_wm_post, dim3((units + 255) / 256), dim3(256), 0, (hipStream_t)stream, raw, ldr, M, P, mean_var,
                     done_logit, ldd, done);
  XTRL_LAUNCHED("wm_post");
  return XTRL_OK;
}
