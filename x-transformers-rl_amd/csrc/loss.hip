// Fused PPO / critic / world-model / done loss of one learn minibatch, forward and backward.
//
// Restates (x_transformers_rl.py):
//   compute_actor_loss   :413-444   ratio, clipped surrogate, masked advantage normalisation
//                                   (normalize :103-112), entropy bonus
//   compute_critic_loss  :446-477   HL-Gauss value / cross-entropy (hl-gauss-pytorch), returns
//                                   clamped to +-value_clip, "between" zeroing
//   compute_autoregressive_loss :398-404 (F.gaussian_nll_loss, var clamped 1e-6 without grad)
//   compute_done_loss    :406-411   (sigmoid + F.binary_cross_entropy, log clamped at -100)
//   combination          :939-978   ((w_a actor + w_c critic)[mask].mean() + (wm.mean() + done.mean()) w_ar)
//
// k_loss_tokens (one wave per token, lanes over the value bins; each block of 16 tokens leaves the
// partial sums of the masked statistics in its tokens' spare slots) -> k_loss_stats (one workgroup:
// fixed-order sum of the block partials -> advantage mean / unbiased variance, critic means,
// gradient coefficients) -> k_loss_actor (thread per token: actor / critic terms, block partials)
// -> k_loss_final (the loss scalars) -> k_loss_bwd (one wave per token) writes d/draw_actions,
// d/dvalues, d/dpred_raw, d/ddone_logit.  Every sum is in double in a fixed order (deterministic).
// Gradients follow PyTorch's autograd rules for min (ties split), clamp (inclusive bounds),
// gaussian_nll_loss (straight-through var clamp) and binary_cross_entropy (eps 1e-12).
#include "common.h"

namespace xtrl {
namespace {

constexpr float F32_EPS = 1.1920928955078125e-07f;
constexpr int NT = XTRL_LOSS_TOK;
enum Tok { T_ADV = 0, T_V = 1, T_VOLD = 2, T_CEU = 3, T_CEC = 4, T_LP = 5, T_ENT = 6, T_WM = 7, T_BCE = 8, T_ACT = 9,
           T_LSE = 10, T_SPARE = 12 };   // T_LSE: log-sum-exp of the value logits (the backward reuses it)
// partial sums of a block: doubles in the spare slots of the block's first token
__device__ __forceinline__ double* part_slot(float* tok, int64_t first, int k) {
  return reinterpret_cast<double*>(tok + first * NT + T_SPARE + 2 * k);
}
// pass-1 statistics
enum Part { P_NMASK = 0, P_ADV, P_ADV2, P_CEU, P_CEC, P_WM, P_NWM, P_BCE, P_KCRIT, P_N1 };
enum Part2 { Q_ACTOR = 0, Q_CRITIC, Q_AC, Q_N };
static_assert(T_SPARE + 2 * P_N1 <= NT && T_SPARE % 2 == 0, "partial sums must fit a token's spare slots");

// softmax statistics of a B-bin logit row held by a wave (lanes strided over bins)
struct RowStats {
  float mx, lse, dot_centers;   // max, log-sum-exp, sum softmax * centres
};

__device__ RowStats row_stats(const float* x, const float* centers, int B, int lane) {
  float mx = -INFINITY;
  for (int k = lane; k < B; k += 64) mx = fmaxf(mx, x[k]);
  mx = wave_max(mx);
  float s = 0.f, sc = 0.f;
  for (int k = lane; k < B; k += 64) {
    const float e = expf(x[k] - mx);
    s += e;
    sc += e * centers[k];
  }
  s = wave_sum(s);
  sc = wave_sum(sc);
  return {mx, mx + logf(s), sc / s};
}

// HL-Gauss target bin probability k for target y (already clamped): (cdf[k+1] - cdf[k]) / z
__device__ __forceinline__ float hl_cdf(const float* support, int k, float y, float inv) {
  return erff((support[k] - y) * inv);
}

// HL-Gauss target probabilities of bins lane and lane + 64 (B <= 127): each lane evaluates the
// CDF at its two bin edges once and takes edge k + 1 from its neighbour, so every edge costs one
// erff per token (the same value, bit for bit, as evaluating both edges of every bin)
struct HlTargets {
  float t0, t1;
};

__device__ HlTargets hl_targets(const float* support, int B, float y, float inv, int lane) {
  const float e0 = lane <= B ? hl_cdf(support, lane, y, inv) : 0.f;
  const float e1 = lane + 64 <= B ? hl_cdf(support, lane + 64, y, inv) : 0.f;
  const int nb = (lane + 1) & 63;
  const float n0s = __shfl(e0, nb, 64), n1 = __shfl(e1, nb, 64), e64 = __shfl(e1, 0, 64);
  const float n0 = lane == 63 ? e64 : n0s;
  const float cB = B < 64 ? __shfl(e0, B, 64) : __shfl(e1, B - 64, 64);
  const float z = cB - __shfl(e0, 0, 64);
  return {lane < B ? (n0 - e0) / z : 0.f, lane + 64 < B ? (n1 - e1) / z : 0.f};
}

// cross entropy -sum_k t_k log_softmax(x)_k
__device__ float hl_ce(const XtrlLossDesc& D, const float* x, float lse, float y, int lane) {
  const int B = D.B;
  y = fminf(fmaxf(y, D.lo), D.hi);
  const float inv = 1.0f / (1.41421356237309505f * D.sigma);
  const HlTargets t = hl_targets(D.support, B, y, inv, lane);
  float acc = 0.f;
  if (lane < B) acc += t.t0 * (x[lane] - lse);
  if (lane + 64 < B) acc += t.t1 * (x[lane + 64] - lse);
  return -wave_sum(acc);
}

// discrete policy terms from raw action logits (A <= 32): torch Categorical(probs = softmax)
struct DiscreteTerms {
  float p[32];
  float S;
  float lp, ent;
};

__device__ void discrete_terms(const float* raw, int A, int a, DiscreteTerms& T) {
  float mx = -INFINITY;
  for (int i = 0; i < A; ++i) mx = fmaxf(mx, raw[i]);
  float s = 0.f;
  for (int i = 0; i < A; ++i) {
    T.p[i] = expf(raw[i] - mx);
    s += T.p[i];
  }
  float S = 0.f;
  for (int i = 0; i < A; ++i) {
    T.p[i] = T.p[i] / s;
    S += T.p[i];
  }
  T.S = S;
  float ent = 0.f;
  for (int i = 0; i < A; ++i) {
    const float q = T.p[i] / S;
    const float lg = logf(fminf(fmaxf(q, F32_EPS), 1.f - F32_EPS));
    ent += lg * q;
    if (i == a) T.lp = lg;
  }
  T.ent = -ent;
}

struct ContTerms {
  float lp, ent;
};

__device__ void cont_terms(const float* raw, float x, int i, int squash, ContTerms& C) {
  const float mean = raw[2 * i], lv = raw[2 * i + 1];
  const float var = expf(tanhf(lv / 3.f) * 3.f);
  const float sd = sqrtf(fmaxf(var, 1e-5f));
  float lp = -((x - mean) * (x - mean)) / (2.f * sd * sd) - logf(sd) - 0.91893853320467274f;
  if (squash) lp -= logf(fmaxf(1.f - x * x, 1e-20f));
  C.lp = lp;
  C.ent = squash ? -lp : 0.5f + 0.91893853320467274f + logf(sd);
}

// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool critic_zeroed(float v, float ret, float vold, float clip) {
  const float lo = vold - clip, hi = vold + clip;
  return ((ret < v) && (v < lo)) || ((hi < v) && (v < ret));
}

// LT_W waves (tokens) per block: the block partials number N / LT_W for k_loss_stats
constexpr int LT_W = 16;
__global__ __launch_bounds__(64 * LT_W) void k_loss_tokens(const XtrlLossDesc D) {
  __shared__ double shp[LT_W][P_N1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = D.b * D.n;
  const int tk0 = blockIdx.x * LT_W + w;
  const bool valid = tk0 < N;   // (waves past N evaluate the last token and store nothing)
  const int tk = valid ? tk0 : N - 1;
  const int bi = tk / D.n, ti = tk - bi * D.n;
  // every operand of the token in one batch of loads (the terms below are chains of wave
  // reductions; loading inside them cost one memory round trip per stage): value and old-value
  // logits, bin centres and edges of lanes k and k + 64, the prediction and next real row (c = lane),
  // the action logits (lane < A) and the token's scalars.  Same arithmetic, same order, as loading
  // on use.
  const int B = D.B;
  const float* vals = D.values + (int64_t)tk * B;
  const float* ovals = D.old_values + (int64_t)tk * B;
  const bool k0 = lane < B, k1 = lane + 64 < B;
  const float x0 = k0 ? vals[lane] : 0.f, x1 = k1 ? vals[lane + 64] : 0.f;
  const float y0 = k0 ? ovals[lane] : 0.f, y1 = k1 ? ovals[lane + 64] : 0.f;
  const float c0 = k0 ? D.centers[lane] : 0.f, c1 = k1 ? D.centers[lane + 64] : 0.f;
  const float e0 = lane <= B ? D.support[lane] : 0.f, e1 = lane + 64 <= B ? D.support[lane + 64] : 0.f;
  const float* pr = D.pred_raw + (int64_t)tk * 2 * D.S1;
  const bool c_in = lane < D.S1;
  const float pm = c_in ? pr[2 * lane] : 0.f, plv = c_in ? pr[2 * lane + 1] : 0.f;
  const float yr = c_in ? D.real[((int64_t)min(tk + 1, N - 1)) * D.S1 + lane] : 0.f;
  const float rawv = (!D.continuous && lane < D.A) ? D.raw_actions[(int64_t)tk * D.A + lane] : 0.f;
  const int act = D.continuous ? 0 : D.actions[tk];
  const float ret = D.returns[tk], zlog = D.done_logit[tk];
  const bool dn = D.dones[tk] != 0;
  const bool mask = ti < D.lens[bi];
  float* tok = D.tok + (int64_t)tk * NT;
  // softmax statistics of the value and old-value rows (row_stats on registers)
  auto stats = [&](float a0, float a1) -> RowStats {
    float mx = -INFINITY;
    if (k0) mx = fmaxf(mx, a0);
    if (k1) mx = fmaxf(mx, a1);
    mx = wave_max(mx);
    float sm = 0.f, sc = 0.f;
    if (k0) {
      const float e = expf(a0 - mx);
      sm += e;
      sc += e * c0;
    }
    if (k1) {
      const float e = expf(a1 - mx);
      sm += e;
      sc += e * c1;
    }
    sm = wave_sum(sm);
    sc = wave_sum(sc);
    return {mx, mx + logf(sm), sc / sm};
  };
  const RowStats rn = stats(x0, x1);
  const RowStats ro = stats(y0, y1);
  // HL-Gauss cross entropy (hl_targets / hl_ce on the edges in registers)
  const float inv = 1.0f / (1.41421356237309505f * D.sigma);
  auto ce = [&](float y) -> float {
    y = fminf(fmaxf(y, D.lo), D.hi);
    const float f0 = lane <= B ? erff((e0 - y) * inv) : 0.f;
    const float f1 = lane + 64 <= B ? erff((e1 - y) * inv) : 0.f;
    const int nb = (lane + 1) & 63;
    const float n0s = __shfl(f0, nb, 64), n1 = __shfl(f1, nb, 64), f64 = __shfl(f1, 0, 64);
    const float n0 = lane == 63 ? f64 : n0s;
    const float cB = B < 64 ? __shfl(f0, B, 64) : __shfl(f1, B - 64, 64);
    const float z = cB - __shfl(f0, 0, 64);
    const float t0 = k0 ? (n0 - f0) / z : 0.f, t1 = k1 ? (n1 - f1) / z : 0.f;
    float acc = 0.f;
    if (k0) acc += t0 * (x0 - rn.lse);
    if (k1) acc += t1 * (x1 - rn.lse);
    return -wave_sum(acc);
  };
  const float ceu = ce(ret);
  const float cec = ce(fminf(fmaxf(ret, -D.value_clip), D.value_clip));
  // world model: predictions at t predict the normalised state-with-reward at t + 1
  const bool wm_on = mask && ti < D.n - 1;
  float wm = 0.f;
  if (wm_on) {
    for (int c = lane; c < D.S1; c += 64) {
      const float mean = c == lane ? pm : pr[2 * c];
      const float var = expf(tanhf((c == lane ? plv : pr[2 * c + 1]) / 3.f) * 3.f);
      const float vv = fmaxf(var, 1e-6f);
      const float y = c == lane ? yr : D.real[((int64_t)tk + 1) * D.S1 + c];
      wm += 0.5f * (logf(vv) + (mean - y) * (mean - y) / vv);
    }
    wm = wave_sum(wm);
  }
  // the action logits to every lane (lane 0 evaluates the discrete terms)
  float rawa[32];
  if (!D.continuous) {
#pragma unroll
    for (int i = 0; i < 32; ++i) rawa[i] = __shfl(rawv, i, 64);
  }
  if (lane == 0) {
    const float adv = ret - ro.dot_centers;
    const float pd = sigmoidf_(zlog);
    const float y = dn ? 1.f : 0.f;
    const float l1 = fmaxf(logf(pd), -100.f), l0 = fmaxf(logf(1.f - pd), -100.f);
    const float bce = -(y * l1 + (1.f - y) * l0);
    if (valid) {
      tok[T_ADV] = adv;
      tok[T_V] = rn.dot_centers;
      tok[T_LSE] = rn.lse;
      tok[T_VOLD] = ro.dot_centers;
      tok[T_CEU] = ceu;
      tok[T_CEC] = cec;
      if (!D.continuous) {
        DiscreteTerms T;
        discrete_terms(rawa, D.A, act, T);
        tok[T_LP] = T.lp;
        tok[T_ENT] = T.ent;
      }
      tok[T_WM] = wm;
      tok[T_BCE] = bce;
    }
    // this token's share of the masked statistics (k_loss_stats)
    const bool m = valid && mask;
    double* sp = shp[w];
    sp[P_NMASK] = m ? 1.0 : 0.0;
    sp[P_ADV] = m ? (double)adv : 0.0;
    sp[P_ADV2] = m ? (double)adv * (double)adv : 0.0;
    sp[P_CEU] = valid ? (double)ceu : 0.0;
    sp[P_CEC] = valid ? (double)cec : 0.0;
    sp[P_WM] = (valid && wm_on) ? (double)wm : 0.0;
    sp[P_NWM] = (valid && wm_on) ? (double)D.S1 : 0.0;
    sp[P_BCE] = m ? (double)bce : 0.0;
    sp[P_KCRIT] = (m && !critic_zeroed(rn.dot_centers, ret, ro.dot_centers, D.value_clip)) ? 1.0 : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < P_N1) {
    const int k = threadIdx.x;
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < LT_W; ++j) v += shp[j][k];
    *part_slot(D.tok, (int64_t)blockIdx.x * LT_W, k) = v;
  }
}

// block-wide sum over 1024 threads (deterministic tree)
__device__ double block_sum(double v, double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (w == 0) {
    r = lane < (int)(blockDim.x >> 6) ? sh[lane] : 0.0;
    r = wave_sum_d(r);
    if (lane == 0) sh[0] = r;
  }
  __syncthreads();
  r = sh[0];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float dmin_dr(float r, float adv, float lo, float hi) {
  const float rc = fminf(fmaxf(r, lo), hi);
  const float s1 = r * adv, s2 = rc * adv;
  const float inr = (r >= lo && r <= hi) ? 1.f : 0.f;
  if (s1 < s2) return adv;
  if (s1 > s2) return adv * inr;
  return 0.5f * adv + 0.5f * adv * inr;
}

// the block partials of k_loss_tokens summed in a fixed order -> masked statistics, advantage mean
// and unbiased variance (sum of squares about zero, in double), critic means and the gradient
// coefficients of the mean-reduced HL-Gauss critic
__global__ __launch_bounds__(1024) void k_loss_stats(const XtrlLossDesc D) {
  __shared__ double sh[16][P_N1];
  const int N = D.b * D.n, P = (N + LT_W - 1) / LT_W;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc[P_N1];
#pragma unroll
  for (int k = 0; k < P_N1; ++k) acc[k] = 0.0;
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
#pragma unroll
    for (int k = 0; k < P_N1; ++k) acc[k] += *part_slot(D.tok, (int64_t)p * LT_W, k);
  }
  // all nine sums in one pass: butterfly per wave, one barrier, wave totals in a fixed order
#pragma unroll
  for (int k = 0; k < P_N1; ++k) {
    const double v = wave_sum_d(acc[k]);
    if (lane == 0) sh[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const int nw = (int)(blockDim.x >> 6);
#pragma unroll
  for (int k = 0; k < P_N1; ++k) {
    double t = 0.0;
    for (int j = 0; j < nw; ++j) t += sh[j][k];
    acc[k] = t;
  }
  const double n_mask = acc[P_NMASK], s_adv = acc[P_ADV], n_wm = acc[P_NWM], k_crit = acc[P_KCRIT];
  const float adv_mean = (float)(s_adv / n_mask);
  const double s_var = acc[P_ADV2] - s_adv * (s_adv / n_mask);
  const float var = n_mask > 1 ? (float)(s_var / (n_mask - 1)) : NAN;
  const float den = sqrtf(fmaxf(var, 1e-5f));
  const float L = (float)(acc[P_CEU] / N), Lc = (float)(acc[P_CEC] / N);
  float* st = D.stats;
  st[XTRL_LS_AUTOREG] = (float)(acc[P_WM] / n_wm);
  st[XTRL_LS_DONE] = (float)(acc[P_BCE] / n_mask);
  st[XTRL_LS_ADV_MEAN] = adv_mean;
  st[XTRL_LS_ADV_DEN] = den;
  st[XTRL_LS_L] = L;
  st[XTRL_LS_LC] = Lc;
  st[XTRL_LS_NMASK] = (float)n_mask;
  st[XTRL_LS_NWM] = (float)n_wm;
  st[XTRL_LS_KCRIT] = (float)k_crit;
  const float dmin = D.w_critic * (float)(k_crit / n_mask);
  st[XTRL_LS_DL] = L < Lc ? dmin : (L > Lc ? 0.f : 0.5f * dmin);
  st[XTRL_LS_DLC] = Lc < L ? dmin : (Lc > L ? 0.f : 0.5f * dmin);
}

// per-token actor / critic terms (thread per token) with the normalised advantage; T_ACT and the
// block partials of sum actor, sum critic (all b*n tokens) and the masked weighted sum
__global__ __launch_bounds__(256) void k_loss_actor(const XtrlLossDesc D) {
  __shared__ double sh[4][Q_N];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = D.b * D.n;
  const int tk0 = blockIdx.x * 256 + threadIdx.x;
  const bool valid = tk0 < N;
  const int tk = valid ? tk0 : N - 1;
  const int bi = tk / D.n, ti = tk - bi * D.n;
  const bool mask = ti < D.lens[bi];
  const float* st = D.stats;
  const float* tok = D.tok + (int64_t)tk * NT;
  const float advn = (tok[T_ADV] - st[XTRL_LS_ADV_MEAN]) / st[XTRL_LS_ADV_DEN];
  const float lo = 1.f - D.eps_clip, hi = 1.f + D.eps_clip;
  float actor = 0.f;
  if (!D.continuous) {
    const float r = expf(tok[T_LP] - D.old_logp[tk]);
    const float rc = fminf(fmaxf(r, lo), hi);
    actor = -fminf(r * advn, rc * advn) - D.entropy_weight * tok[T_ENT];
  } else {
    for (int i = 0; i < D.A; ++i) {
      ContTerms C;
      cont_terms(D.raw_actions + (int64_t)tk * 2 * D.A, D.actions_f[(int64_t)tk * D.A + i], i, D.squash, C);
      const float r = expf(C.lp - D.old_logp[(int64_t)tk * D.A + i]);
      const float rc = fminf(fmaxf(r, lo), hi);
      actor += -fminf(r * advn, rc * advn) - D.entropy_weight * C.ent;
    }
  }
  const bool zero = critic_zeroed(tok[T_V], D.returns[tk], tok[T_VOLD], D.value_clip);
  float critic;
  if (D.hl_reduction_mean) critic = zero ? 0.f : fminf(st[XTRL_LS_L], st[XTRL_LS_LC]);
  else critic = zero ? 0.f : fminf(tok[T_CEU], tok[T_CEC]);
  if (valid) D.tok[(int64_t)tk * NT + T_ACT] = actor;
  double q[Q_N];
  q[Q_ACTOR] = valid ? (double)actor : 0.0;
  q[Q_CRITIC] = valid ? (double)critic : 0.0;
  q[Q_AC] = (valid && mask) ? (double)(actor * D.w_actor + critic * D.w_critic) : 0.0;
#pragma unroll
  for (int k = 0; k < Q_N; ++k) {
    const double v = wave_sum_d(q[k]);
    if (lane == 0) sh[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < Q_N) {
    const int k = threadIdx.x;
    *part_slot(D.tok, (int64_t)blockIdx.x * 256, k) = ((sh[0][k] + sh[1][k]) + sh[2][k]) + sh[3][k];
  }
}

// the loss scalars from the k_loss_actor block partials (fixed order)
__global__ __launch_bounds__(256) void k_loss_final(const XtrlLossDesc D) {
  __shared__ double sh[16];
  const int N = D.b * D.n, P = (N + 255) / 256;
  double acc[Q_N] = {0.0, 0.0, 0.0};
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
#pragma unroll
    for (int k = 0; k < Q_N; ++k) acc[k] += *part_slot(D.tok, (int64_t)p * 256, k);
  }
#pragma unroll
  for (int k = 0; k < Q_N; ++k) acc[k] = block_sum(acc[k], sh);
  if (threadIdx.x != 0) return;
  float* st = D.stats;
  const double n_mask = st[XTRL_LS_NMASK];
  st[XTRL_LS_LOSS] = (float)(acc[Q_AC] / n_mask) + (st[XTRL_LS_AUTOREG] + st[XTRL_LS_DONE]) * D.w_autoreg;
  st[XTRL_LS_ACTOR] = (float)(acc[Q_ACTOR] / N);
  st[XTRL_LS_CRITIC] = (float)(acc[Q_CRITIC] / N);
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_loss_bwd(const XtrlLossDesc D, float g) {
  const int lane = threadIdx.x & 63;
  const int tk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int N = D.b * D.n;
  if (tk >= N) return;
  const int bi = tk / D.n, ti = tk - bi * D.n;
  // every operand of the token in one batch of loads (as k_loss_tokens; same arithmetic and order
  // as loading on use): the forward's per-token terms and the loss statistics, value logits and bin
  // edges of lanes k and k + 64, the prediction and next real row (c = lane), the token's scalars
  const int B = D.B;
  const bool k0 = lane < B, k1 = lane + 64 < B;
  const float* x = D.values + (int64_t)tk * B;
  const float x0 = k0 ? x[lane] : 0.f, x1 = k1 ? x[lane + 64] : 0.f;
  const float e0 = lane <= B ? D.support[lane] : 0.f, e1 = lane + 64 <= B ? D.support[lane + 64] : 0.f;
  const float* pr = D.pred_raw + (int64_t)tk * 2 * D.S1;
  const bool c_in = lane < D.S1;
  const float pm = c_in ? pr[2 * lane] : 0.f, plv = c_in ? pr[2 * lane + 1] : 0.f;
  const float yr = c_in ? D.real[((int64_t)min(tk + 1, N - 1)) * D.S1 + lane] : 0.f;
  const float* st = D.stats;
  const float* tok = D.tok + (int64_t)tk * NT;
  const float t_adv = tok[T_ADV], t_v = tok[T_V], t_vold = tok[T_VOLD], t_ceu = tok[T_CEU], t_cec = tok[T_CEC],
              t_lse = tok[T_LSE];
  const float s_nmask = st[XTRL_LS_NMASK], s_mean = st[XTRL_LS_ADV_MEAN], s_den = st[XTRL_LS_ADV_DEN],
              s_dl = st[XTRL_LS_DL], s_dlc = st[XTRL_LS_DLC], s_nwm = st[XTRL_LS_NWM];
  const float ret = D.returns[tk], zlog = D.done_logit[tk];
  const bool dn = D.dones[tk] != 0;
  const bool mask = ti < D.lens[bi];
  const float n_mask = s_nmask;
  const float coef_ac = mask ? g / n_mask : 0.f;
  const float advn = (t_adv - s_mean) / s_den;
  const float lo = 1.f - D.eps_clip, hi = 1.f + D.eps_clip;

  // ---- critic: d/dvalues
  {
    float du, dc;   // weights of the unclipped / clipped CE gradients
    if (D.hl_reduction_mean) {
      du = g * s_dl / (float)N;
      dc = g * s_dlc / (float)N;
    } else {
      const bool zero = critic_zeroed(t_v, ret, t_vold, D.value_clip);
      const float w = zero ? 0.f : coef_ac * D.w_critic;
      const float a = t_ceu, b = t_cec;
      du = a < b ? w : (a > b ? 0.f : 0.5f * w);
      dc = b < a ? w : (b > a ? 0.f : 0.5f * w);
    }
    const float lse = t_lse;   // the forward's softmax statistics of this token's value logits
    const float inv = 1.0f / (1.41421356237309505f * D.sigma);
    const float yu = fminf(fmaxf(ret, D.lo), D.hi);
    const float yc = fminf(fmaxf(fminf(fmaxf(ret, -D.value_clip), D.value_clip), D.lo), D.hi);
    // hl_targets on the edges in registers
    auto targets = [&](float y) -> HlTargets {
      const float f0 = lane <= B ? erff((e0 - y) * inv) : 0.f;
      const float f1 = lane + 64 <= B ? erff((e1 - y) * inv) : 0.f;
      const int nb = (lane + 1) & 63;
      const float n0s = __shfl(f0, nb, 64), n1 = __shfl(f1, nb, 64), f64 = __shfl(f1, 0, 64);
      const float n0 = lane == 63 ? f64 : n0s;
      const float cB = B < 64 ? __shfl(f0, B, 64) : __shfl(f1, B - 64, 64);
      const float z = cB - __shfl(f0, 0, 64);
      return {k0 ? (n0 - f0) / z : 0.f, k1 ? (n1 - f1) / z : 0.f};
    };
    const HlTargets tu = targets(yu);
    const HlTargets tc = targets(yc);
    // sum_k t_k (= 1 up to rounding) for the exact softmax * sum(t) - t gradient
    float su = 0.f, sc = 0.f;
    if (k0) {
      su += tu.t0;
      sc += tc.t0;
    }
    if (k1) {
      su += tu.t1;
      sc += tc.t1;
    }
    su = wave_sum(su);
    sc = wave_sum(sc);
    if (k0) {
      const float p = expf(x0 - lse);
      D.d_values[(int64_t)tk * B + lane] = du * (p * su - tu.t0) + dc * (p * sc - tc.t0);
    }
    if (k1) {
      const float p = expf(x1 - lse);
      D.d_values[(int64_t)tk * B + lane + 64] = du * (p * su - tu.t1) + dc * (p * sc - tc.t1);
    }
  }

  // ---- world model: d/dpred_raw (interleaved mean / log-var)
  {
    const float coef = (mask && ti < D.n - 1) ? g * D.w_autoreg / s_nwm : 0.f;
    for (int c = lane; c < D.S1; c += 64) {
      float dm = 0.f, dlv = 0.f;
      if (coef != 0.f) {
        const float mean = c == lane ? pm : pr[2 * c], lv = c == lane ? plv : pr[2 * c + 1];
        const float th = tanhf(lv / 3.f);
        const float var = expf(th * 3.f);
        const float vv = fmaxf(var, 1e-6f);
        const float y = c == lane ? yr : D.real[((int64_t)tk + 1) * D.S1 + c];
        const float df = mean - y;
        dm = coef * df / vv;
        const float dvar = coef * 0.5f * (1.f / vv - df * df / (vv * vv));
        dlv = dvar * var * (1.f - th * th);
      }
      D.d_pred_raw[(int64_t)tk * 2 * D.S1 + 2 * c] = dm;
      D.d_pred_raw[(int64_t)tk * 2 * D.S1 + 2 * c + 1] = dlv;
    }
  }

  // the action logits to every lane (lane 0 evaluates the discrete terms)
  float rawa[32];
  int act = 0;
  float olp = 0.f;
  if (!D.continuous) {
    const float rawv = lane < D.A ? D.raw_actions[(int64_t)tk * D.A + lane] : 0.f;
    act = D.actions[tk];
    olp = D.old_logp[tk];
#pragma unroll
    for (int i = 0; i < 32; ++i) rawa[i] = __shfl(rawv, i, 64);
  }
  if (lane != 0) return;
  // ---- done: BCE(sigmoid(z), y)
  {
    const float coef = mask ? g * D.w_autoreg / n_mask : 0.f;
    const float p = sigmoidf_(zlog);
    const float y = dn ? 1.f : 0.f;
    const float dp = coef * (p - y) / fmaxf((1.f - p) * p, 1e-12f);
    D.d_done_logit[tk] = dp * (1.f - p) * p;
  }
  // ---- actor: d/draw_actions
  const float ca = coef_ac * D.w_actor;
  if (!D.continuous) {
    const int A = D.A;
    float* dr = D.d_raw_actions + (int64_t)tk * A;
    if (ca == 0.f) {
      for (int i = 0; i < A; ++i) dr[i] = 0.f;
      return;
    }
    DiscreteTerms T;
    const int a = act;
    discrete_terms(rawa, A, a, T);
    const float r = expf(T.lp - olp);
    const float dlp = -dmin_dr(r, advn, lo, hi) * r * ca;   // d tok / d logp
    const float dent = -D.entropy_weight * ca;               // d tok / d entropy
    float gq[32];
    for (int i = 0; i < A; ++i) {
      const float q = T.p[i] / T.S;
      const bool inr = (q >= F32_EPS) && (q <= 1.f - F32_EPS);
      const float lg = logf(fminf(fmaxf(q, F32_EPS), 1.f - F32_EPS));
      const float dlg = inr ? 1.f / fminf(fmaxf(q, F32_EPS), 1.f - F32_EPS) : 0.f;
      float gqi = dent * -(lg + q * dlg);
      if (i == a) gqi += dlp * dlg;
      gq[i] = gqi;
    }
    float sgp = 0.f;
    for (int i = 0; i < A; ++i) sgp += gq[i] * T.p[i];
    float gp[32], sg = 0.f;
    for (int i = 0; i < A; ++i) {
      gp[i] = gq[i] / T.S - sgp / (T.S * T.S);
      sg += gp[i] * T.p[i];
    }
    for (int i = 0; i < A; ++i) dr[i] = T.p[i] * (gp[i] - sg);
  } else {
    const int A = D.A;
    const float* raw = D.raw_actions + (int64_t)tk * 2 * A;
    float* dr = D.d_raw_actions + (int64_t)tk * 2 * A;
    for (int i = 0; i < A; ++i) {
      if (ca == 0.f) {
        dr[2 * i] = 0.f;
        dr[2 * i + 1] = 0.f;
        continue;
      }
      const float x = D.actions_f[(int64_t)tk * A + i];
      ContTerms C;
      cont_terms(raw, x, i, D.squash, C);
      const float r = expf(C.lp - D.old_logp[(int64_t)tk * A + i]);
      float dlp = -dmin_dr(r, advn, lo, hi) * r * ca;
      float dsd_extra = 0.f;
      if (D.squash) dlp += D.entropy_weight * ca;   // entropy = -logp
      const float mean = raw[2 * i], lv = raw[2 * i + 1];
      const float th = tanhf(lv / 3.f);
      const float var = expf(th * 3.f);
      const float sd = sqrtf(fmaxf(var, 1e-5f));
      if (!D.squash) dsd_extra = -D.entropy_weight * ca / sd;   // d(-beta * log sd)/d sd
      const float df = x - mean;
      const float dmean = dlp * df / (sd * sd);
      const float dsd = dlp * (df * df / (sd * sd * sd) - 1.f / sd) + dsd_extra;
      const float dvar = var >= 1e-5f ? dsd * 0.5f / sd : 0.f;
      dr[2 * i] = dmean;
      dr[2 * i + 1] = dvar * var * (1.f - th * th);
    }
  }
}

int check(const XtrlLossDesc* D) {
  XTRL_REQUIRE(D, "loss: null descriptor");
  XTRL_REQUIRE(D->b > 0 && D->n > 0 && D->A > 0 && D->A <= 32 && D->B > 0 && D->B <= 127 && D->S1 > 0,
               "loss: bad shape (A <= 32, B <= 127)");
  XTRL_REQUIRE(D->raw_actions && D->values && D->pred_raw && D->done_logit && D->old_logp && D->returns &&
                   D->old_values && D->dones && D->lens && D->real && D->support && D->centers && D->tok && D->stats,
               "loss: null operand");
  XTRL_REQUIRE(D->continuous ? D->actions_f != nullptr : D->actions != nullptr, "loss: null actions");
  return XTRL_OK;
}

}  // namespace

int loss_fwd(const XtrlLossDesc* D, hipStream_t s) {
  if (int rc = check(D)) return rc;
  const int N = D->b * D->n;
  hipLaunchKernelGGL(k_loss_tokens, dim3((N + LT_W - 1) / LT_W), dim3(64 * LT_W), 0, s, *D);
  XTRL_LAUNCHED("loss_tokens");
  hipLaunchKernelGGL(k_loss_stats, dim3(1), dim3(1024), 0, s, *D);
  XTRL_LAUNCHED("loss_stats");
  hipLaunchKernelGGL(k_loss_actor, dim3((N + 255) / 256), dim3(256), 0, s, *D);
  XTRL_LAUNCHED("loss_actor");
  hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(256), 0, s, *D);
  XTRL_LAUNCHED("loss_final");
  return XTRL_OK;
}

int loss_bwd(const XtrlLossDesc* D, float g, hipStream_t s) {
  if (int rc = check(D)) return rc;
  XTRL_REQUIRE(D->d_raw_actions && D->d_values && D->d_pred_raw && D->d_done_logit, "loss_bwd: null gradient");
  const int N = D->b * D->n;
  hipLaunchKernelGGL(k_loss_bwd, dim3((N + 3) / 4), dim3(256), 0, s, *D, g);
  XTRL_LAUNCHED("loss_bwd");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_loss_fwd(const XtrlLossDesc* desc, void* stream) {
  return xtrl::loss_fwd(desc, xtrl::as_stream(stream));
}
extern "C" int xtrl_loss_bwd(const XtrlLossDesc* desc, float grad_scale, void* stream) {
  return xtrl::loss_bwd(desc, grad_scale, xtrl::as_stream(stream));
}
