// Optimiser path over ONE flat fp32 parameter buffer (every nn.Parameter of the model is a view
// into it, so clip / step / EMA are three streaming passes instead of ~60 per-tensor launches).
//
//   xtrl_grad_norm   clip_grad_norm_ (xtrl.py:987): total L2 norm, clip coefficient
//                    min(max_norm / (norm + 1e-6), 1)  -> out[0] norm, out[1] coefficient
//   xtrl_adopt_atan2 AdoptAtan2.step (xtrl.py:749, 991; adam-atan2-pytorch, restated in
//                    oracle/thirdparty.py) with the clip coefficient folded into the gradient and
//                    the cautious-mask mean taken per parameter tensor (segment)
//   xtrl_ema_lerp    EMA post-step update (xtrl.py:747-753; ema-pytorch lerp)
// All are HBM-bound elementwise passes (16-28 B per parameter).
#include "common.h"

namespace xtrl {
namespace {

constexpr int NB = 512;   // partial-sum blocks for the norm
constexpr int ADOPT_U = 4;   // elements per thread in flight in the AdoptAtan2 passes

__global__ __launch_bounds__(256) void k_sumsq(const float* g, int64_t n, double* ws) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = g[i];
    s += v * v;
  }
  __shared__ double sh[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// 64 lanes: lane l sums partials l, l + 64, ... in order (loads in flight together), then a
// fixed-order wave reduction
__global__ void k_norm_final(const double* ws, int nb, float max_norm, float* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) s += ws[i];
  s = wave_sum_d(s);
  if (threadIdx.x != 0) return;
  const float norm = (float)sqrt(s);
  out[0] = norm;
  out[1] = fminf(max_norm / (norm + 1e-6f), 1.0f);
}

struct AdoptArgs {
  float *p, *g, *m, *v, *p_init;
  int64_t n;
  const int64_t* chunks;   // [n_chunks][3]: start, end, segment
  int n_chunks;
  const int64_t* seg;      // [n_seg + 1] segment offsets
  int n_seg;
  int* cnt;
  const float* clip;
  float lr, init_lr, beta1, beta2, a, b, wd, regen, cautious;
  int first;
};

// pass A (one workgroup per chunk of one parameter tensor): regen / weight decay, first-step
// init, m update, and the cautious alignment count of the chunk -> ONE atomic per workgroup
__global__ __launch_bounds__(256) void k_adopt_a(const AdoptArgs A) {
  const int64_t c0 = A.chunks[3 * blockIdx.x], c1 = A.chunks[3 * blockIdx.x + 1];
  const int sg = (int)A.chunks[3 * blockIdx.x + 2];
  const float coef = A.clip ? A.clip[1] : 1.f;
  int aligned = 0;
  // ADOPT_U elements per thread per round, all loaded before the first store (the stores may alias
  // the loads as far as the compiler knows): the round's loads are in flight together
  for (int64_t i0 = c0 + threadIdx.x; i0 < c1; i0 += ADOPT_U * 256) {
    float g[ADOPT_U], p[ADOPT_U], pi[ADOPT_U], v[ADOPT_U], m[ADOPT_U];
#pragma unroll
    for (int u = 0; u < ADOPT_U; ++u) {
      const int64_t i = i0 + u * 256, ic = i < c1 ? i : c0;
      g[u] = A.g[ic];
      p[u] = A.p[ic];
      pi[u] = (A.regen > 0.f && !A.first) ? A.p_init[ic] : 0.f;
      v[u] = A.first ? 0.f : A.v[ic];
      m[u] = A.first ? 0.f : A.m[ic];
    }
#pragma unroll
    for (int u = 0; u < ADOPT_U; ++u) {
      const int64_t i = i0 + u * 256;
      if (i >= c1) break;
      const float gg = g[u] * coef;
      A.g[i] = gg;
      float pp = p[u];
      if (A.regen > 0.f && !A.first) pp = lerpf_(pp, pi[u], A.lr / A.init_lr * A.regen);
      if (A.wd > 0.f) pp = pp * (1.f - A.lr * A.wd);
      A.p[i] = pp;
      if (A.first) {
        A.m[i] = 0.f;
        A.v[i] = gg * gg;
        if (A.regen > 0.f) A.p_init[i] = pp;
        continue;
      }
      const float uu = atan2f(gg, A.b * sqrtf(v[u]));
      const float mm = lerpf_(m[u], uu, 1.f - A.beta1);
      A.m[i] = mm;
      aligned += (mm * gg > 0.f) ? 1 : 0;
    }
  }
  if (A.first || A.cautious >= 1.f) return;
  __shared__ int sh[4];
  int w = aligned;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&A.cnt[sg], sh[0] + sh[1] + sh[2] + sh[3]);
}

// pass B: p -= lr * a * m * scale; v = lerp(v, g^2, 1 - beta2)
__global__ __launch_bounds__(256) void k_adopt_b(const AdoptArgs A) {
  if (A.first) return;
  const int64_t c0 = A.chunks[3 * blockIdx.x], c1 = A.chunks[3 * blockIdx.x + 1];
  const int sg = (int)A.chunks[3 * blockIdx.x + 2];
  float mean = 1.f;
  if (A.cautious < 1.f) {
    const double len = (double)(A.seg[sg + 1] - A.seg[sg]);
    const double k = (double)A.cnt[sg];
    mean = (float)((k + (double)A.cautious * (len - k)) / len);
  }
  const float inv = 1.f / fmaxf(mean, 1e-5f);
  for (int64_t i0 = c0 + threadIdx.x; i0 < c1; i0 += ADOPT_U * 256) {
    float g[ADOPT_U], m[ADOPT_U], p[ADOPT_U], v[ADOPT_U];
#pragma unroll
    for (int u = 0; u < ADOPT_U; ++u) {
      const int64_t i = i0 + u * 256, ic = i < c1 ? i : c0;
      g[u] = A.g[ic];
      m[u] = A.m[ic];
      p[u] = A.p[ic];
      v[u] = A.v[ic];
    }
#pragma unroll
    for (int u = 0; u < ADOPT_U; ++u) {
      const int64_t i = i0 + u * 256;
      if (i >= c1) break;
      float upd = m[u];
      if (A.cautious < 1.f) upd = m[u] * (((m[u] * g[u] > 0.f) ? 1.f : A.cautious) * inv);
      A.p[i] = p[u] + (-A.lr) * (upd * A.a);
      A.v[i] = lerpf_(v[u], g[u] * g[u], 1.f - A.beta2);
    }
  }
}

__global__ void k_ema(float* ema, const float* p, int64_t n, float w) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    ema[i] = lerpf_(ema[i], p[i], w);
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 4096); }

}  // namespace

int grad_norm(const float* g, int64_t n, double* ws, float max_norm, float* out, hipStream_t s) {
  XTRL_REQUIRE(g && ws && out && n > 0, "grad_norm: bad arguments");
  hipLaunchKernelGGL(k_sumsq, dim3(NB), dim3(256), 0, s, g, n, ws);
  hipLaunchKernelGGL(k_norm_final, dim3(1), dim3(64), 0, s, ws, NB, max_norm, out);
  XTRL_LAUNCHED("grad_norm");
  return XTRL_OK;
}

int adopt_atan2(const AdoptArgs& A, hipStream_t s) {
  XTRL_REQUIRE(A.p && A.g && A.m && A.v && A.n > 0 && A.seg && A.n_seg > 0 && A.cnt && A.chunks && A.n_chunks > 0,
               "adopt_atan2: bad arguments");
  XTRL_REQUIRE(A.regen <= 0.f || A.p_init, "adopt_atan2: regen needs p_init");
  if (hipMemsetAsync(A.cnt, 0, sizeof(int) * A.n_seg, s) != hipSuccess) return check_launch("adopt_atan2 memset");
  hipLaunchKernelGGL(k_adopt_a, dim3(A.n_chunks), dim3(256), 0, s, A);
  hipLaunchKernelGGL(k_adopt_b, dim3(A.n_chunks), dim3(256), 0, s, A);
  XTRL_LAUNCHED("adopt_atan2");
  return XTRL_OK;
}

int ema_lerp(float* ema, const float* p, int64_t n, float w, hipStream_t s) {
  XTRL_REQUIRE(ema && p && n > 0, "ema_lerp: bad arguments");
  hipLaunchKernelGGL(k_ema, dim3(grid_for(n)), dim3(256), 0, s, ema, p, n, w);
  XTRL_LAUNCHED("ema_lerp");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_grad_norm(const float* g, int64_t n, double* ws, float max_norm, float* out, void* stream) {
  return xtrl::grad_norm(g, n, ws, max_norm, out, xtrl::as_stream(stream));
}

extern "C" int xtrl_adopt_atan2(float* p, float* g, float* m, float* v, float* p_init, int64_t n,
                                const int64_t* chunks, int n_chunks, const int64_t* seg_start, int n_seg,
                                int* seg_ws, const float* clip, float lr, float init_lr, float beta1, float beta2,
                                float a, float b, float weight_decay, float regen_rate, float cautious, int first_step,
                                void* stream) {
  xtrl::AdoptArgs A{p,     g,      m,       v,    p_init, n, chunks, n_chunks, seg_start, n_seg, seg_ws, clip, lr,
                    init_lr, beta1, beta2, a, b, weight_decay, regen_rate, cautious, first_step};
  return xtrl::adopt_atan2(A, xtrl::as_stream(stream));
}

extern "C" int xtrl_ema_lerp(float* ema, const float* p, int64_t n, float weight, void* stream) {
  return xtrl::ema_lerp(ema, p, n, weight, xtrl::as_stream(stream));
}
