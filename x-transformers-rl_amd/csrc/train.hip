// Learn-step forward / backward of WorldModelActorCritic on one minibatch without autograd
// (Agent.learn, x_transformers_rl.py:928-935 forward with mask, :982 backward; the x-transformers
// Decoder restated in SURVEY Appendix A).  The dense layers run on the fused fp32 MFMA GEMM with
// their elementwise neighbours folded into prologues / epilogues (LayerNorm, bias, GELU + dropout,
// SiLU, residual, value gate, and their derivatives), the attention core on the strided flash
// kernels, and everything else in the handful of small kernels below.  All reductions over tokens
// (bias / LayerNorm-gain / embedding gradients) are two-phase with a fixed summation order, so the
// step is deterministic run to run.
#include <cstdlib>
#include <vector>

#include <hip/hip_ext.h>

#include "kernels.h"
#include "philox.h"

namespace xtrl {
namespace {

constexpr int kMaxDPerLane = 8;   // LayerNorm kernels: d <= 512

__device__ __forceinline__ float ldg(const float* p) { return __builtin_nontemporal_load(p); }

// ---- embeddings: x0 = project_in(state) + action_embed(prev) + reward * keep * reward_embed;
//      ac_in[:, d:2d] = to_state_embed(state); ewa[:, d:2d] = action_embed(next);
//      ac_in[:, 2d:3d] = latent_to_embed(gene)  (xtrl.py:494-503, 516-549)
struct EmbedArgs {
  const float *swr, *w_pin, *act_emb, *act_emb_b, *reward_embed, *w_se, *b_se, *lat_e, *prev_af, *next_af;
  const int32_t *prev_a, *next_a;
  float *x0, *ac_in, *ewa;
  int T, n, S, A, d, in_dim, continuous, evolutionary;
  float keep;
  const float* ln_g;   // (k_embed_ln) layer 0's attention pre-norm: gamma, output rows, (mean, rstd)
  float *xn, *st;
  int rms;             // the pre-norm is x-transformers' RMSNorm (use_rmsnorm)
  const int32_t* rows; // packed rows: token t is the minibatch's row rows[t] = episode * n + step (latent)
};

constexpr int EMB_TOK = 32, EMB_U = 8, EMB_MAXS = 32;
// block: EMB_TOK tokens x all d columns; thread c keeps its project_in / to_state_embed rows in
// registers (S <= EMB_MAXS) and walks the block's tokens EMB_U at a time, every input of a batch
// loaded before its first store (the stores may alias the inputs as far as the compiler knows)
// S_ > 0: the state width at compile time (the lander's 8: no per-element guards in the S loops)
template <int S_>
__global__ __launch_bounds__(256) void k_embed(const EmbedArgs a) {
  constexpr int MS = S_ > 0 ? S_ : EMB_MAXS;
  const int S = S_ > 0 ? S_ : a.S;
  for (int c = threadIdx.x; c < a.d; c += 256) {
    float wp[MS], ws[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      wp[s] = s < S ? a.w_pin[(int64_t)c * S + s] : 0.f;
      ws[s] = s < S ? a.w_se[(int64_t)c * S + s] : 0.f;
    }
    const float bse = a.b_se[c], re = a.reward_embed[c];
    const float bemb = a.continuous ? a.act_emb_b[c] : 0.f;
    for (int t0 = blockIdx.x * EMB_TOK; t0 < min(a.T, (int)(blockIdx.x + 1) * EMB_TOK); t0 += EMB_U) {
      float pin[EMB_U], se[EMB_U], rw[EMB_U], ap[EMB_U], an[EMB_U], le[EMB_U];
#pragma unroll
      for (int u = 0; u < EMB_U; ++u) {
        const int t = min(t0 + u, a.T - 1);
        const float* st = a.swr + (int64_t)t * (S + 1);
        float sp = 0.f, ss = 0.f;
#pragma unroll
        for (int s = 0; s < MS; ++s) {
          if (s < S) {
            const float x = st[s];
            sp += x * wp[s];
            ss += x * ws[s];
          }
        }
        pin[u] = sp;
        se[u] = ss + bse;
        rw[u] = st[S];
        if (a.continuous) {
          const float* w = a.act_emb + (int64_t)c * a.A;
          float p = 0.f, q = 0.f;
          for (int k = 0; k < a.A; ++k) {
            p += a.prev_af[(int64_t)t * a.A + k] * w[k];
            q += a.next_af[(int64_t)t * a.A + k] * w[k];
          }
          ap[u] = p + bemb;
          an[u] = q + bemb;
        } else {   // SafeEmbedding: action < 0 -> zero vector (xtrl.py:181-195)
          const int p = a.prev_a[t], q = a.next_a[t];
          ap[u] = p >= 0 ? a.act_emb[(int64_t)p * a.d + c] : 0.f;
          an[u] = q >= 0 ? a.act_emb[(int64_t)q * a.d + c] : 0.f;
        }
        le[u] = a.evolutionary ? a.lat_e[(int64_t)((a.rows ? a.rows[t] : t) / a.n) * a.d + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < EMB_U; ++u) {
        const int t = t0 + u;
        if (t >= a.T) break;
        a.x0[(int64_t)t * a.d + c] = pin[u] + (ap[u] + (rw[u] * re) * a.keep);
        a.ac_in[(int64_t)t * a.in_dim + a.d + c] = se[u];
        a.ewa[(int64_t)t * 2 * a.d + a.d + c] = an[u];
        if (a.evolutionary) a.ac_in[(int64_t)t * a.in_dim + 2 * a.d + c] = le[u];
      }
    }
  }
}

// k_embed with layer 0's attention pre-norm folded in (d <= 256: thread c owns column c): per
// batch of EMB_U tokens the row sums and the centred sums of squares meet through LDS (two
// barriers), then x0, LN(x0) gamma and (mean, rstd) are stored — k_ln_fwd's arithmetic (two-pass
// variance, eps 1e-5) with the row sum associated per wave, then over the 4 waves.  One batch per
// workgroup (EMB_LN_TOK = EMB_U): the batches' load / barrier round trips run in parallel
// workgroups instead of one after another (C3: 2048 workgroups, 45 -> see DESIGN §7 a launch)
constexpr int EMB_LN_TOK = EMB_U;
template <int S_>
__global__ __launch_bounds__(256) void k_embed_ln(const EmbedArgs a) {
  constexpr int MS = S_ > 0 ? S_ : EMB_MAXS;
  const int S = S_ > 0 ? S_ : a.S;
  __shared__ float red[2][4][EMB_U];
  const int c = threadIdx.x, lane = c & 63, w = c >> 6;
  const bool on = c < a.d;
  const int cc = on ? c : 0;
  float wp[MS], ws[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    wp[s] = s < S ? a.w_pin[(int64_t)cc * S + s] : 0.f;
    ws[s] = s < S ? a.w_se[(int64_t)cc * S + s] : 0.f;
  }
  const float bse = a.b_se[cc], re = a.reward_embed[cc], gam = on ? a.ln_g[cc] : 0.f;
  const float bemb = a.continuous ? a.act_emb_b[cc] : 0.f;
  const float inv_d = 1.0f / (float)a.d;
  for (int t0 = blockIdx.x * EMB_LN_TOK; t0 < min(a.T, (int)(blockIdx.x + 1) * EMB_LN_TOK); t0 += EMB_U) {
    float x[EMB_U], se[EMB_U], an[EMB_U], le[EMB_U];
#pragma unroll
    for (int u = 0; u < EMB_U; ++u) {
      const int t = min(t0 + u, a.T - 1);
      const float* st = a.swr + (int64_t)t * (S + 1);
      float sp = 0.f, ss = 0.f;
#pragma unroll
      for (int s = 0; s < MS; ++s) {
        if (s < S) {
          const float v = st[s];
          sp += v * wp[s];
          ss += v * ws[s];
        }
      }
      float ap;
      if (a.continuous) {
        const float* wa = a.act_emb + (int64_t)cc * a.A;
        float p = 0.f, q = 0.f;
        for (int k = 0; k < a.A; ++k) {
          p += a.prev_af[(int64_t)t * a.A + k] * wa[k];
          q += a.next_af[(int64_t)t * a.A + k] * wa[k];
        }
        ap = p + bemb;
        an[u] = q + bemb;
      } else {   // SafeEmbedding: action < 0 -> zero vector (xtrl.py:181-195)
        const int p = a.prev_a[t], q = a.next_a[t];
        ap = p >= 0 ? a.act_emb[(int64_t)p * a.d + cc] : 0.f;
        an[u] = q >= 0 ? a.act_emb[(int64_t)q * a.d + cc] : 0.f;
      }
      x[u] = on ? sp + (ap + (st[S] * re) * a.keep) : 0.f;
      se[u] = ss + bse;
      le[u] = a.evolutionary ? a.lat_e[(int64_t)((a.rows ? a.rows[t] : t) / a.n) * a.d + cc] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < EMB_U; ++u) {
      const float r = wave_sum(x[u]);
      if (lane == 0) red[0][w][u] = r;
    }
    __syncthreads();
    float mean[EMB_U], dl[EMB_U];
#pragma unroll
    for (int u = 0; u < EMB_U; ++u) {
      mean[u] = a.rms ? 0.f : ((red[0][0][u] + red[0][1][u]) + (red[0][2][u] + red[0][3][u])) * inv_d;
      dl[u] = on ? x[u] - mean[u] : 0.f;
      const float q = wave_sum(dl[u] * dl[u]);
      if (lane == 0) red[1][w][u] = q;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EMB_U; ++u) {
      const int t = t0 + u;
      if (t >= a.T) break;
      const float sq = (red[1][0][u] + red[1][1][u]) + (red[1][2][u] + red[1][3][u]);
      const float rstd = a.rms ? norm_rstd(sq, (float)a.d, true) : 1.0f / sqrtf(sq * inv_d + 1e-5f);
      if (on) {
        a.x0[(int64_t)t * a.d + c] = x[u];
        a.xn[(int64_t)t * a.d + c] = (dl[u] * rstd) * gam;
        a.ac_in[(int64_t)t * a.in_dim + a.d + c] = se[u];
        a.ewa[(int64_t)t * 2 * a.d + a.d + c] = an[u];
        if (a.evolutionary) a.ac_in[(int64_t)t * a.in_dim + 2 * a.d + c] = le[u];
      }
      if (c == 0) {
        a.st[2 * (int64_t)t] = mean[u];
        a.st[2 * (int64_t)t + 1] = rstd;
      }
    }
  }
}

// lat_e[b][c] = latent[b] . w[c] + bias[c]
__global__ void k_latent_embed(const float* latent, const float* w, const float* bias, float* out, int b, int G,
                               int d) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b * d) return;
  const int e = i / d, c = i - e * d;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += latent[(int64_t)e * G + g] * w[(int64_t)c * G + g];
  out[i] = s + bias[c];
}

// ---- LayerNorm (x-transformers: layer_norm without affine, eps 1e-5, times gamma) ------------
// one wave per row; y written to y1 (and y2 when given); stats = (mean, rstd)
__global__ __launch_bounds__(256) void k_ln_fwd(const float* x, const float* gamma, float* y1, int ld1, float* y2,
                                                int ld2, float* stats, int T, int d, int rms) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const float* xr = x + (int64_t)t * d;
  float v[kMaxDPerLane], gm[kMaxDPerLane];   // gamma loaded with the row: one round trip
#pragma unroll
  for (int k = 0; k < kMaxDPerLane; ++k) {
    const int c = lane + 64 * k;
    v[k] = c < d ? xr[c] : 0.f;
    gm[k] = c < d ? gamma[c] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxDPerLane; ++k) s += v[k];
  const float mean = rms ? 0.f : wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxDPerLane; ++k) {
    const int c = lane + 64 * k;
    const float dl = c < d ? v[k] - mean : 0.f;
    q += dl * dl;
  }
  const float rstd = norm_rstd(wave_sum(q), (float)d, rms);
#pragma unroll
  for (int k = 0; k < kMaxDPerLane; ++k) {
    const int c = lane + 64 * k;
    if (c < d) {
      const float y = ((v[k] - mean) * rstd) * gm[k];
      y1[(int64_t)t * ld1 + c] = y;
      if (y2) y2[(int64_t)t * ld2 + c] = y;
    }
  }
  if (lane == 0) {
    stats[2 * t] = mean;
    stats[2 * t + 1] = rstd;
  }
}

// LayerNorm backward, LN_ROWS rows per block of LN_WAVES waves (each wave 4 rows, loads of all
// four issued together; small blocks so they co-reside with the weight-gradient GEMM workgroups of
// the backward side stream: learn 125.3 -> 124.0 ms against 16-wave blocks): upstream gradient g = s1 * g1 + g2 (g2 optional),
// dx = rstd * (g*gamma - mean(g*gamma) - xhat * mean(g*gamma*xhat)) (+ dres; dx may alias dres);
// per-block partial d gamma = sum_rows g * xhat -> part[block][d] (and, for nn.LayerNorm's bias,
// d beta = sum_rows g -> part_b[block][d] when part_b is given)
constexpr int LN_ROWS = 16, LN_WAVES = 4, LN_R = 4;   // 256-thread blocks fit beside a side-stream GEMM workgroup on its CU
template <int DPL>
__global__ __launch_bounds__(64 * LN_WAVES) void k_ln_bwd(const float* g1, int ldg1, float s1, const float* g2,
                                                          int ldg2, const float* x, const float* stats,
                                                          const float* gamma, const float* dres, float* dx,
                                                          float* part, float* part_b, int pstride, int T, int d,
                                                          int rms) {
  __shared__ float red[LN_WAVES][64 * DPL];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float gam[DPL], dg[DPL], db[DPL];
#pragma unroll
  for (int k = 0; k < DPL; ++k) {
    const int c = lane + 64 * k;
    gam[k] = c < d ? gamma[c] : 0.f;
    dg[k] = 0.f;
    db[k] = 0.f;
  }
  const int r0 = blockIdx.x * LN_ROWS;
  for (int rb = w * LN_R; rb < LN_ROWS; rb += LN_WAVES * LN_R) {
    // every operand of the wave's LN_R rows (incoming residual gradient included) is loaded
    // before the first reduction: one memory round trip per row group
    float g[LN_R][DPL], xv[LN_R][DPL], dr[LN_R][DPL], rs[LN_R], mu[LN_R];
#pragma unroll
    for (int q = 0; q < LN_R; ++q) {
      const int t = r0 + rb + q;
      const bool ok = t < T;
      mu[q] = ok ? stats[2 * t] : 0.f;
      rs[q] = ok ? stats[2 * t + 1] : 0.f;
#pragma unroll
      for (int k = 0; k < DPL; ++k) {
        const int c = lane + 64 * k;
        const bool in = ok && c < d;
        float gv = in ? s1 * g1[(int64_t)t * ldg1 + c] : 0.f;
        if (g2 && in) gv += g2[(int64_t)t * ldg2 + c];
        g[q][k] = gv;
        xv[q][k] = in ? x[(int64_t)t * d + c] : 0.f;
        dr[q][k] = (dres && in) ? dres[(int64_t)t * d + c] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < LN_R; ++q) {
      const int t = r0 + rb + q;
      float sa = 0.f, sb = 0.f;
      float gm[DPL], xh[DPL];
#pragma unroll
      for (int k = 0; k < DPL; ++k) {
        const int c = lane + 64 * k;
        xh[k] = c < d ? (xv[q][k] - mu[q]) * rs[q] : 0.f;
        gm[k] = g[q][k] * gam[k];
        dg[k] += g[q][k] * xh[k];
        db[k] += g[q][k];
        sa += gm[k];
        sb += gm[k] * xh[k];
      }
      // (RMSNorm: no mean in the forward, no mean(g gamma) term in the backward)
      const float ma = rms ? 0.f : wave_sum(sa) / (float)d, mb = wave_sum(sb) / (float)d;
      if (t < T) {
#pragma unroll
        for (int k = 0; k < DPL; ++k) {
          const int c = lane + 64 * k;
          if (c < d) {
            float v = rs[q] * (gm[k] - ma - xh[k] * mb);
            if (dres) v += dr[q][k];
            dx[(int64_t)t * d + c] = v;
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < DPL; ++k) red[w][lane + 64 * k] = dg[k];
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 64 * LN_WAVES) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < LN_WAVES; ++j) v += red[j][c];
    part[(int64_t)blockIdx.x * pstride + c] = v;
  }
  if (!part_b) return;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < DPL; ++k) red[w][lane + 64 * k] = db[k];
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 64 * LN_WAVES) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < LN_WAVES; ++j) v += red[j][c];
    part_b[(int64_t)blockIdx.x * pstride + c] = v;
  }
}

// ---- rotary + value-residual mix (x-transformers Attention) --------------
// one thread per (token, column pair) of q | k | v (coalesced float2 traffic): q and k rotated on
// their first rot_dim channels (interleaved pairs, position = step within the episode); v mixed
// towards the first layer's v
struct PrepArgs {
  const float* proj;    // [T][n_qkv]
  const float* vfirst;  // layer-0 proj (v at column 2I)
  float* qkv;           // [T][3I]
  const float* inv_freq;
  int T, n, H, dh, I, n_qkv, ld_vfirst, rot_dim, mix_col;   // mix_col < 0: no mix
  int qk_norm;          // x-transformers qk norm: q, k l2-normalised per head before the rotary
  float xpos_base;      // rotary xPos scale base (0: off)
  const int32_t* rows;  // packed rows (grid (pair blocks, T)): token t's position is rows[t] % n
};

// x-transformers RotaryEmbedding(use_xpos): rotated pair j (even channel) at position pos of an n-token
// sequence is scaled by ((j + 0.4 rot) / (1.4 rot)) ^ ((pos - n / 2) / scale_base) for q, by its
// inverse for k (x_transformers.RotaryEmbedding.forward / apply_rotary_pos_emb)
__device__ __forceinline__ float xpos_factor(int j, int rot, int pos, int n, float base) {
  const float sc = ((float)j + 0.4f * (float)rot) / (1.4f * (float)rot);
  return powf(sc, (float)(pos - n / 2) / base);
}

// the per-head l2 norm of a (q or k) channel pair: the head's dh / 2 pairs sit on consecutive,
// aligned lanes (every lane of the group active); F.normalize: x / max(||x||, 1e-12)
__device__ __forceinline__ float head_norm(float2 x, int dh) {
  float ss = x.x * x.x + x.y * x.y;
  for (int o = dh >> 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  return fmaxf(sqrtf(ss), 1e-12f);
}

// grid (pair blocks, n steps, b episodes), PREP_T threads: token and position come from the grid
// (no 64-bit division per element); one sincosf per rotated pair
constexpr int PREP_T = 128;
__global__ __launch_bounds__(PREP_T) void k_qkv_prep(const PrepArgs a) {
  const int P = 3 * a.I / 2;
  const int pair = blockIdx.x * PREP_T + threadIdx.x;
  if (pair >= P) return;
  const int t = a.rows ? (int)blockIdx.y : blockIdx.z * a.n + blockIdx.y;
  const int pos = a.rows ? a.rows[t] % a.n : (int)blockIdx.y, col = 2 * pair;
  const int seg = col / a.I, within = col - seg * a.I, h = within / a.dh, j = within - h * a.dh;
  float2 x = *reinterpret_cast<const float2*>(a.proj + (int64_t)t * a.n_qkv + col);
  float2 y;
  if (seg < 2) {
    if (a.qk_norm) {
      const float nrm = head_norm(x, a.dh);
      x.x = x.x / nrm;
      x.y = x.y / nrm;
    }
    if (j < a.rot_dim) {
      const float f = (float)pos * a.inv_freq[j >> 1];
      float sn, cs;
      sincosf(f, &sn, &cs);
      y.x = x.x * cs + (-x.y) * sn;
      y.y = x.y * cs + x.x * sn;
      if (a.xpos_base > 0.f) {
        const float xf = xpos_factor(j, a.rot_dim, pos, a.n, a.xpos_base);
        const float sf = seg == 0 ? xf : 1.0f / xf;
        y.x *= sf;
        y.y *= sf;
      }
    } else {
      y = x;
    }
  } else if (a.mix_col >= 0) {
    const float m = sigmoidf_(a.proj[(int64_t)t * a.n_qkv + a.mix_col + h]);
    const float2 vf = *reinterpret_cast<const float2*>(a.vfirst + (int64_t)t * a.ld_vfirst + 2 * a.I + within);
    y.x = lerpf_(x.x, vf.x, m);
    y.y = lerpf_(x.y, vf.y, m);
  } else {
    y = x;
  }
  *reinterpret_cast<float2*>(a.qkv + (int64_t)t * 3 * a.I + col) = y;
}

// backward of k_qkv_prep, in place on dproj ([T][n_qkv], dq | dk | dv written by the attention
// backward): inverse rotation of dq, dk; lerp backward for v (dv -> (1 - m) dv, dvfirst += m dv,
// d mix_pre = sum over the head's channels of dv (vf - v), times m (1 - m): a shuffle reduction over
// the head's dh / 2 consecutive lanes); layer 0 adds the accumulated dvfirst to its dv
struct PrepBwdArgs {
  float* dproj;
  const float* proj;
  const float* vfirst;
  float* dvfirst;       // [T][I]
  const float* inv_freq;
  int T, n, H, dh, I, n_qkv, ld_vfirst, rot_dim, mix_col, first_layer, accumulate;
  int qk_norm;
  float xpos_base;
  const int32_t* rows;  // packed rows, as PrepArgs
};

__global__ __launch_bounds__(PREP_T) void k_qkv_prep_bwd(const PrepBwdArgs a) {
  const int P = 3 * a.I / 2;
  const int pair0 = blockIdx.x * PREP_T + threadIdx.x;
  const bool valid = pair0 < P;
  const int pair = valid ? pair0 : 0;
  const int t = a.rows ? (int)blockIdx.y : blockIdx.z * a.n + blockIdx.y;
  const int pos = a.rows ? a.rows[t] % a.n : (int)blockIdx.y, col = 2 * pair;
  const int seg = col / a.I, within = col - seg * a.I, h = within / a.dh, j = within - h * a.dh;
  float* g = a.dproj + (int64_t)t * a.n_qkv + col;
  float dm = 0.f, m = 0.f;
  float2 gqk = make_float2(0.f, 0.f);   // q / k: the gradient w.r.t. the (normalised) pre-rotary pair
  if (valid) {
    float2 gv = *reinterpret_cast<float2*>(g);
    if (seg < 2) {
      if (j < a.rot_dim) {
        const float f = (float)pos * a.inv_freq[j >> 1];
        float sn, cs;
        sincosf(f, &sn, &cs);
        float g0 = gv.x, g1 = gv.y;
        if (a.xpos_base > 0.f) {
          const float xf = xpos_factor(j, a.rot_dim, pos, a.n, a.xpos_base);
          const float sf = seg == 0 ? xf : 1.0f / xf;
          g0 *= sf;
          g1 *= sf;
        }
        gv.x = g0 * cs + g1 * sn;
        gv.y = g1 * cs + (-g0) * sn;
        if (!a.qk_norm) *reinterpret_cast<float2*>(g) = gv;
      }
      gqk = gv;
    } else {
      float2* dvf = reinterpret_cast<float2*>(a.dvfirst + (int64_t)t * a.I + within);
      if (a.mix_col >= 0) {
        const float* pr = a.proj + (int64_t)t * a.n_qkv;
        m = sigmoidf_(pr[a.mix_col + h]);
        const float2 v = *reinterpret_cast<const float2*>(pr + col);
        const float2 vf = *reinterpret_cast<const float2*>(a.vfirst + (int64_t)t * a.ld_vfirst + col);
        dm = gv.x * (vf.x - v.x) + gv.y * (vf.y - v.y);
        float2 f;
        f.x = gv.x * m;
        f.y = gv.y * m;
        if (a.accumulate) {
          const float2 o = *dvf;
          f.x += o.x;
          f.y += o.y;
        }
        *dvf = f;
        gv.x = gv.x * (1.0f - m);
        gv.y = gv.y * (1.0f - m);
        *reinterpret_cast<float2*>(g) = gv;
      } else if (a.first_layer && a.accumulate) {
        const float2 o = *dvf;
        gv.x += o.x;
        gv.y += o.y;
        *reinterpret_cast<float2*>(g) = gv;
      }
    }
  }
  if (a.qk_norm) {   // l2-norm backward of q, k: dx = (g - x^ (x^ . g)) / ||x||  (every lane shuffles)
    const float2 x = valid ? *reinterpret_cast<const float2*>(a.proj + (int64_t)t * a.n_qkv + col) : make_float2(0.f, 0.f);
    float ss = x.x * x.x + x.y * x.y;
    for (int o = a.dh >> 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    const float r = sqrtf(ss), nrm = fmaxf(r, 1e-12f);
    const float hx = x.x / nrm, hy = x.y / nrm;
    const float2 gg = gqk;
    float dot = hx * gg.x + hy * gg.y;
    for (int o = a.dh >> 2; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
    if (valid && seg < 2) {
      float2 dx;
      if (r >= 1e-12f) {
        dx.x = (gg.x - hx * dot) / nrm;
        dx.y = (gg.y - hy * dot) / nrm;
      } else {
        dx.x = gg.x / nrm;
        dx.y = gg.y / nrm;
      }
      *reinterpret_cast<float2*>(g) = dx;
    }
  }
  if (a.mix_col >= 0) {   // every lane takes part in the shuffles (groups of dh / 2 aligned lanes)
    for (int o = a.dh >> 2; o > 0; o >>= 1) dm += __shfl_xor(dm, o, 64);
    if (valid && seg == 2 && j == 0) a.dproj[(int64_t)t * a.n_qkv + a.mix_col + h] = dm * (1.0f - m) * m;
  }
}

// ---- deterministic column sums: part[chunk][c] = sum over the chunk's rows of w_r * src[r][c] --
__global__ __launch_bounds__(256) void k_colsum_part(const float* src, int ld, int rows, int cols, int chunk_rows,
                                                     const float* rw, int ld_rw, float rw_scale, float* part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * chunk_rows, r1 = min(rows, r0 + chunk_rows);
  float s = 0.f;
  if (rw) {
#pragma unroll 8
    for (int r = r0; r < r1; ++r) s += src[(int64_t)r * ld + c] * (rw[(int64_t)r * ld_rw] * rw_scale);
  } else {
#pragma unroll 8
    for (int r = r0; r < r1; ++r) s += src[(int64_t)r * ld + c];
  }
  part[(int64_t)blockIdx.y * cols + c] = s;
}

// dst[c] += sum over chunks of part[chunk][c]: CS_COLS columns per block of CS_WAVES waves; each
// lane owns (column lane % CS_COLS, chunk group) and sums its chunks in four chains (loads in flight),
// then the CS_G group totals of a column are added in a fixed order (deterministic)
constexpr int CS_WAVES = 16, CS_COLS = 16, CS_G = 64 * CS_WAVES / CS_COLS;
__device__ __forceinline__ void colsum_final_body(const float* part, int chunks, int cols, float* dst, int bx) {
  __shared__ float red[CS_G][CS_COLS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cl = lane % CS_COLS, g = w * (64 / CS_COLS) + lane / CS_COLS;
  const int c = bx * CS_COLS + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < cols) {
    int k = g;
    for (; k + 3 * CS_G < chunks; k += 4 * CS_G) {
      s0 += part[(int64_t)k * cols + c];
      s1 += part[(int64_t)(k + CS_G) * cols + c];
      s2 += part[(int64_t)(k + 2 * CS_G) * cols + c];
      s3 += part[(int64_t)(k + 3 * CS_G) * cols + c];
    }
    for (; k < chunks; k += CS_G) s0 += part[(int64_t)k * cols + c];
  }
  red[g][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (threadIdx.x < CS_COLS) {
    const int cc = bx * CS_COLS + threadIdx.x;
    if (cc < cols) {
      float v = 0.f;
#pragma unroll 8
      for (int j2 = 0; j2 < CS_G; ++j2) v += red[j2][threadIdx.x];
      dst[cc] += v;
    }
  }
}
__global__ __launch_bounds__(64 * CS_WAVES) void k_colsum_final(const float* part, int chunks, int cols, float* dst) {
  colsum_final_body(part, chunks, cols, dst, blockIdx.x);
}

// the LayerNorm d gamma column sums of a backward, deferred: each fused LayerNorm-backward GEMM
// epilogue writes its row-tile partials into a plane of its own, and ONE launch (blockIdx.y = job)
// finishes them all — each sum exactly k_colsum_final's, into a distinct gamma (bit-identical)
constexpr int kMaxColsumJobs = 16;
struct ColsumJobs {
  const float* part[kMaxColsumJobs];
  float* dst[kMaxColsumJobs];
  int chunks[kMaxColsumJobs];
  int cols[kMaxColsumJobs];
};
__global__ __launch_bounds__(64 * CS_WAVES) void k_colsum_final_multi(const ColsumJobs J) {
  const int j = blockIdx.y;
  if ((int)blockIdx.x * CS_COLS >= J.cols[j]) return;   // (workgroup-uniform)
  colsum_final_body(J.part[j], J.chunks[j], J.cols[j], J.dst[j], blockIdx.x);
}
struct ColsumQueue {
  ColsumJobs J{};
  int n = 0, max_cols = 0;
  float* base = nullptr;
  int64_t cap = 0, used = 0;
  // a plane of chunks x cols partials whose column sums go to dst, or NULL (full: sum now)
  // the plane, flushing the queued jobs first when it is full (their planes are then free)
  float* take_or_flush(int chunks, int cols, float* dst, hipStream_t s, int* rc) {
    *rc = XTRL_OK;
    float* P = take(chunks, cols, dst);
    if (!P && base && n > 0) {
      if ((*rc = flush(s))) return nullptr;
      P = take(chunks, cols, dst);
    }
    return P;
  }
  float* take(int chunks, int cols, float* dst) {
    const int64_t need = (int64_t)chunks * cols;
    if (!base || n == kMaxColsumJobs || used + need > cap) return nullptr;
    float* P = base + used;
    used += (need + 3) & ~(int64_t)3;
    J.part[n] = P; J.dst[n] = dst; J.chunks[n] = chunks; J.cols[n] = cols;
    ++n;
    max_cols = std::max(max_cols, cols);
    return P;
  }
  int flush(hipStream_t s) {
    if (n > 0) {
      hipLaunchKernelGGL(k_colsum_final_multi, dim3((max_cols + CS_COLS - 1) / CS_COLS, n), dim3(64 * CS_WAVES), 0, s,
                         J);
      XTRL_LAUNCHED("colsum_final_multi");
    }
    n = 0; max_cols = 0; used = 0;
    return XTRL_OK;
  }
};

// discrete action-embedding gradient: part[chunk][a][c] = sum over rows of the chunk with
// prev[r] == a of g1[r][c]  +  rows with next[r] == a of g2[r][c]   (A <= EMB_MAXA, registers)
constexpr int EMB_MAXA = 32;
template <int MAXA>   // a compile-time bound on A (4 / 8 / 32): the per-row select chain is MAXA long
__global__ __launch_bounds__(256) void k_embed_grad_part(const float* g1, int ld1, const int32_t* prev,
                                                         const float* g2, int ld2, const int32_t* next, int rows,
                                                         int d, int A, int chunk_rows, float* part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  const int r0 = blockIdx.y * chunk_rows, r1 = min(rows, r0 + chunk_rows);
  float acc[MAXA];
#pragma unroll
  for (int a = 0; a < MAXA; ++a) acc[a] = 0.f;
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    const int p = prev ? prev[r] : -1, q = next[r];   // (no prev: the next-action input only)
    const float x = prev ? g1[(int64_t)r * ld1 + c] : 0.f, y = g2[(int64_t)r * ld2 + c];
#pragma unroll
    for (int a = 0; a < MAXA; ++a) {
      if (a < A) {
        acc[a] += p == a ? x : 0.f;
        acc[a] += q == a ? y : 0.f;
      }
    }
  }
  float* out = part + (int64_t)blockIdx.y * A * d;
#pragma unroll
  for (int a = 0; a < MAXA; ++a)
    if (a < A) out[(int64_t)a * d + c] = acc[a];
}

// latent gradient of the evolutionary conditioning: dlat[e][c] = sum_steps dac[e*n + s][2d + c].
// Block (episode e, 64 columns): LG_G groups of 64 threads each sum a contiguous range of steps
// in order (8 loads in flight per thread), then the group partials are added in group order (a
// thread per column summing all n steps in turn took 107 us a launch at C2's n = 500)
constexpr int LG_G = 16;
// ep_off (packed rows): episode e's rows are ep_off[e] .. ep_off[e + 1] - 1
__global__ __launch_bounds__(64 * LG_G) void k_latent_grad(const float* dac, int ld, int off, int b, int n, int d,
                                                           float* dlat, const int32_t* ep_off) {
  __shared__ float red[LG_G][64];
  const int e = blockIdx.x, cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const int64_t r0 = ep_off ? (int64_t)ep_off[e] : (int64_t)e * n;
  const int ne = ep_off ? ep_off[e + 1] - ep_off[e] : n;
  const int per = (ne + LG_G - 1) / LG_G, t0 = grp * per, t1 = min(ne, t0 + per);
  float s = 0.f;
  if (c < d) {
    const float* col = dac + r0 * ld + off + c;
    int t = t0;
    for (; t + 8 <= t1; t += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = col[(int64_t)(t + u) * ld];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; t < t1; ++t) s += col[(int64_t)t * ld];
  }
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < d) {
    float tot = 0.f;
#pragma unroll
    for (int g2 = 0; g2 < LG_G; ++g2) tot += red[g2][cl];
    dlat[(int64_t)e * d + c] = tot;
  }
}

// dW[c][g] += sum_e dlat[e][c] latent[e][g];  db[c] += sum_e dlat[e][c]
__global__ void k_latent_wgrad(const float* dlat, const float* latent, int b, int d, int G, float* dw, float* db) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d * (G + 1)) return;
  const int c = i / (G + 1), g = i - c * (G + 1);
  // (episodes 8 at a time, their loads issued together; the sum in episode order)
  float s = 0.f;
  for (int e0 = 0; e0 < b; e0 += 8) {
    float x[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = min(e0 + u, b - 1);
      x[u] = dlat[(int64_t)e * d + c];
      y[u] = g < G ? latent[(int64_t)e * G + g] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (e0 + u < b) s += g < G ? x[u] * y[u] : x[u];
  }
  if (g < G) dw[(int64_t)c * G + g] += s;
  else db[c] += s;
}

__global__ void k_copy_col(const float* src, int ld, float* dst, int lddst, int rows) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) dst[(int64_t)r * lddst] = src[(int64_t)r * ld];
}

// the FF dropout keep mask of the GELU_DROP epilogue (gemm.hip): word mode (one Philox block per
// 4 rows of a column) or byte mode (thresh8 != 0: one block per 16 rows, see ff_block8)
// the feed-forward dropout's keep bit of element (m, n) of the [T][ff] hidden (the FF1 epilogue's stream)
__device__ __forceinline__ bool ff_keep(int m, int n, uint32_t thresh, uint32_t thresh8, uint64_t seed, uint32_t off,
                                        uint32_t layer) {
  if (thresh8) {
    const u32x4_t r = philox4x32_10((uint32_t)n, (uint32_t)(((m >> 5) << 1) | ((m >> 2) & 1)), off,
                                    rng_c3(FIELD_FF_DROPOUT, 2 * layer + 1), seed);
    const int g = (m >> 3) & 3;
    const uint32_t w = g == 0 ? r.x : (g == 1 ? r.y : (g == 2 ? r.z : r.w));
    return ((w >> (8 * (m & 3))) & 0xFFu) >= thresh8;
  }
  if (thresh == 0) return true;
  const u32x4_t r = philox4x32_10((uint32_t)n, (uint32_t)(m >> 2), off, rng_c3(FIELD_FF_DROPOUT, 2 * layer), seed);
  const int q = m & 3;
  const uint32_t w = q == 0 ? r.x : (q == 1 ? r.y : (q == 2 ? r.z : r.w));
  return w >= thresh;
}

__global__ void k_ff_mask(uint8_t* mask, int M, int N, uint32_t thresh, uint32_t thresh8, uint64_t seed,
                          uint32_t off, uint32_t layer) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
  mask[i] = (uint8_t)ff_keep(m, n, thresh, thresh8, seed, off, layer);
}

// x-transformers GLU project-in (ff_glu) + the feed-forward dropout: u = [value | gate] [M][2 ff] (the
// GLU projection's output), h[m][j] = drop(u[m][j] GELU(u[m][ff + j])) with the FF1 epilogue's keep
// stream (torch's erf GELU); backward du = [dh~ GELU(g) | dh~ a GELU'(g)], dh~ = drop(dh).  One
// thread per hidden element (HBM bound: 12 bytes read + 4 written forward, 16 + 8 backward)
__device__ __forceinline__ float gelu_deriv_erf(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  return cdf + x * (0.39894228040143268f * expf(-0.5f * x * x));
}
__global__ void k_glu_fwd(const float* u, int ldu, float* h, int ldh, int M, int ff, uint32_t thresh, uint32_t thresh8,
                          float inv_keep, uint64_t seed, uint32_t off, uint32_t layer) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * ff) return;
  const int m = (int)(i / ff), j = (int)(i - (int64_t)m * ff);
  const float a = u[(int64_t)m * ldu + j], g = u[(int64_t)m * ldu + ff + j];
  const bool keep = ff_keep(m, j, thresh, thresh8, seed, off, layer);
  h[(int64_t)m * ldh + j] = keep ? (a * geluf_(g)) * inv_keep : 0.f;
}
__global__ void k_glu_bwd(const float* dh, int lddh, const float* u, int ldu, float* du, int lddu, int M, int ff,
                          uint32_t thresh, uint32_t thresh8, float inv_keep, uint64_t seed, uint32_t off,
                          uint32_t layer) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * ff) return;
  const int m = (int)(i / ff), j = (int)(i - (int64_t)m * ff);
  const float a = u[(int64_t)m * ldu + j], g = u[(int64_t)m * ldu + ff + j];
  const bool keep = ff_keep(m, j, thresh, thresh8, seed, off, layer);
  const float dk = keep ? dh[(int64_t)m * lddh + j] * inv_keep : 0.f;
  du[(int64_t)m * lddu + j] = dk * geluf_(g);
  du[(int64_t)m * lddu + ff + j] = (dk * a) * gelu_deriv_erf(g);
}

int glu_fwd(const float* u, int ldu, float* h, int ldh, int M, int ff, float p, uint64_t seed, uint32_t off,
            uint32_t layer, hipStream_t s) {
  if ((int64_t)M * ff == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_glu_fwd, dim3((unsigned)(((int64_t)M * ff + 255) / 256)), dim3(256), 0, s, u, ldu, h, ldh, M, ff,
                     dropout_thresh(p), dropout_thresh8(p), p > 0.f ? 1.f / (1.f - p) : 1.f, seed, off, layer);
  XTRL_LAUNCHED("glu_fwd");
  return XTRL_OK;
}
int glu_bwd(const float* dh, int lddh, const float* u, int ldu, float* du, int lddu, int M, int ff, float p,
            uint64_t seed, uint32_t off, uint32_t layer, hipStream_t s) {
  if ((int64_t)M * ff == 0) return XTRL_OK;
  hipLaunchKernelGGL(k_glu_bwd, dim3((unsigned)(((int64_t)M * ff + 255) / 256)), dim3(256), 0, s, dh, lddh, u, ldu, du,
                     lddu, M, ff, dropout_thresh(p), dropout_thresh8(p), p > 0.f ? 1.f / (1.f - p) : 1.f, seed, off,
                     layer);
  XTRL_LAUNCHED("glu_bwd");
  return XTRL_OK;
}

// ---- fractal learn step (fractal_rl.py:116-136, 274-346 made causal; xtrl_amd/fractal.py) -------
// causal running mean over each episode's steps (the reference's sequence mean made causal)
//   REV = 0: dst[e, t] = (sum_{s <= t} src[e, s]) / (t + 1)                       (x3.cumsum(1) / cnt)
//   REV = 1: dst[e, s] = add[e, s] + sum_{t >= s} src[e, t] / (t + 1)            (its backward)
// Block (episode e, 64 columns), CM_G groups of 64 threads each owning a contiguous range of steps:
// pass 1 sums the range, the group totals are combined through LDS, pass 2 rescans the range from
// the carried-in total (coalesced: a group reads 64 consecutive floats of a row per step)
constexpr int CM_G = 16;
template <int REV>
__global__ __launch_bounds__(64 * CM_G) void k_causal_mean(const float* src, int lds, const float* add, int ldadd,
                                                          float* dst, int ldd, int n, int d) {
  __shared__ float tot[CM_G][64];
  const int e = blockIdx.x, cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const int per = (n + CM_G - 1) / CM_G, t0 = min(n, grp * per), t1 = min(n, t0 + per);
  const bool ok = c < d;
  const int64_t base = (int64_t)e * n;
  float s = 0.f;
  if (ok)
    for (int t = t0; t < t1; ++t) {
      const float v = src[(base + t) * lds + c];
      s += REV ? v / (float)(t + 1) : v;
    }
  tot[grp][cl] = s;
  __syncthreads();
  float carry = 0.f;
  if (REV) {
    for (int j = CM_G - 1; j > grp; --j) carry += tot[j][cl];
  } else {
    for (int j = 0; j < grp; ++j) carry += tot[j][cl];
  }
  if (!ok) return;
  if (REV) {
    for (int t = t1 - 1; t >= t0; --t) {
      carry += src[(base + t) * lds + c] / (float)(t + 1);
      dst[(base + t) * ldd + c] = (add ? add[(base + t) * ldadd + c] : 0.f) + carry;
    }
  } else {
    for (int t = t0; t < t1; ++t) {
      carry += src[(base + t) * lds + c];
      dst[(base + t) * ldd + c] = carry / (float)(t + 1);
    }
  }
}

// out[i] = a[i] + b[i]
__global__ void k_vec_add(const float* a, const float* b, float* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

// dst[r][c] = alpha * a[r][c] + (b ? b[r][c] : 0)   (a row vector broadcast when lda == 0)
__global__ void k_rows_axpb(const float* a, int lda, float alpha, const float* b, int ldb, float* dst, int ldd,
                            int rows, int cols) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * cols) return;
  const int64_t r = i / cols;
  const int c = (int)(i - r * cols);
  float v = alpha * a[r * lda + c];
  if (b) v += b[r * ldb + c];
  dst[r * ldd + c] = v;
}

// SafeEmbedding of the next action (xtrl.py:181-195): out[r] = W[a_r] for 0 <= a_r < A, else 0
__global__ void k_action_rows(const int32_t* act, const float* W, int A, float* out, int ldo, int rows, int d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * d) return;
  const int64_t r = i / d;
  const int c = (int)(i - r * d), a = act[r];
  out[r * ldo + c] = (a >= 0 && a < A) ? W[(int64_t)a * d + c] : 0.f;
}

// dst[r][c] = src[r / n][c]: one row per episode broadcast over its n steps (the gene embedding)
__global__ void k_rows_bcast_ep(const float* src, float* dst, int ldd, int rows, int n, int d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * d) return;
  const int64_t r = i / d;
  const int c = (int)(i - r * d);
  dst[r * ldd + c] = src[(r / n) * d + c];
}

// ---- host helpers -----------------------------------------------------------------------------
inline unsigned blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

struct Ctx {
  const XtrlTrainDesc* D;
  hipStream_t s;
  int T;
  SplitKQueue* q = nullptr;   // weight gradients: split-K reductions deferred to one launch
  const float* P(int64_t off) const { return off >= 0 ? D->flat + off : nullptr; }
  float* G(int64_t off) const { return off >= 0 ? D->grad + off : nullptr; }
};

// row stride of the [T][ff] feed-forward buffers (hd, u, dff; fractal h, u, dz): ld_ff >= ff, 0 = ff
// (a stride off the 4 KiB power of two spreads the FF1 epilogue's two store streams: 93 -> 82 us)
inline int ld_ff(const XtrlTrainDesc* D) { return D->ld_ff > 0 ? D->ld_ff : D->ff; }

// ---- weight gradients on a side stream ---------------------------------------------------------
// The weight-gradient GEMMs (and their split-K reduces) are off the backward's critical path: only
// the optimiser step reads dW.  They run on a low-priority side stream, each after an event on the
// main stream marks its dY ready; the main stream waits for a specific side event before it
// overwrites a buffer a pending weight gradient still reads (dx, dff, dproj), and for all of them
// at the end of the backward.  The side stream and its event pool are created once per process
// (one device per process, grown to the deepest model seen) and hold no data.
// XTRL_WGRAD_STREAM=0: everything on one stream.
struct SideStream {
  hipStream_t s = nullptr;
  std::vector<hipEvent_t> ev;
  bool ok = false;
  // at least n events (false: creation failed, the caller runs single-stream).  The fork / join
  // events only order two streams of this device, so they are recorded with a device-scope
  // release instead of the default system-scope fence (the kernels' own end-of-kernel release and
  // start-of-kernel acquire carry the data): the main stream's gap at a fork shrinks, C3 learn
  // −0.7 ms.  XTRL_FORK_FENCE=0: system scope (the HIP default); 2: no fence at all (A/B only)
  bool ensure(size_t n) {
    static const unsigned flags = [] {
      const char* f = getenv("XTRL_FORK_FENCE");
      const int v = f ? atoi(f) : 1;
      return (unsigned)hipEventDisableTiming |
             (v == 1 ? (unsigned)hipEventReleaseToDevice : v == 2 ? (unsigned)hipEventDisableSystemFence : 0u);
    }();
    while (ok && ev.size() < n) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return false;
      ev.push_back(e);
    }
    return ok;
  }
};
SideStream& side_stream() {
  static SideStream S = [] {
    SideStream x;
    const char* e = getenv("XTRL_WGRAD_STREAM");
    if (e && atoi(e) == 0) return x;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
    // XTRL_WGRAD_CUS=n (experiments): the side stream confined to n CUs, every (CUs / n)-th one
    const char* cus = getenv("XTRL_WGRAD_CUS");
    int dev = 0, ncu = 0;
    if (cus && atoi(cus) > 0 && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0) {
      const int want = std::min(atoi(cus), ncu), step = std::max(1, ncu / want);
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int i = 0, n = 0; i < ncu && n < want; i += step, ++n) mask[i / 32] |= 1u << (i % 32);
      x.ok = hipExtStreamCreateWithCUMask(&x.s, (uint32_t)mask.size(), mask.data()) == hipSuccess;
      return x;
    }
    // XTRL_WGRAD_PRIO=1 (experiments): the side stream at the highest priority instead of the lowest
    const char* pr = getenv("XTRL_WGRAD_PRIO");
    x.ok = hipStreamCreateWithPriority(&x.s, hipStreamNonBlocking, (pr && atoi(pr) == 1) ? greatest : least) ==
           hipSuccess;
    return x;
  }();
  return S;
}
// events one backward takes: 4 forks before the decoder blocks, 4 forks + 4 marks per block, one
// fork + one mark for the embeddings and the final join
constexpr size_t side_events_needed(int L) { return 8 * (size_t)L + 6; }

// fork / mark / wait helpers of one backward call (no-ops on a single stream)
struct Fork {
  hipStream_t main, side;
  SideStream* S;
  int next = 0;
  bool failed = false;   // a mark() could not record: the final join reports it
  bool on() const { return S != nullptr; }
  hipEvent_t take() {
    if ((size_t)next >= S->ev.size()) return nullptr;   // (sized by side_events_needed: never)
    return S->ev[next++];
  }
  // the side stream waits for everything issued on the main stream so far
  int fork() {
    if (!on()) return XTRL_OK;
    hipEvent_t e = take();
    if (!e || hipEventRecord(e, main) != hipSuccess || hipStreamWaitEvent(side, e, 0) != hipSuccess) {
      set_error("train: side-stream fork failed");
      return XTRL_E_HIP;
    }
    return XTRL_OK;
  }
  // an event after everything issued on the side stream so far
  hipEvent_t mark() {
    if (!on()) return nullptr;
    hipEvent_t e = take();
    if (!e || hipEventRecord(e, side) != hipSuccess) {
      failed = true;
      return nullptr;
    }
    return e;
  }
  // the main stream waits for a side event (nullptr: nothing to wait for)
  int wait(hipEvent_t e) {
    if (!on() || !e) return XTRL_OK;
    if (hipStreamWaitEvent(main, e, 0) != hipSuccess) {
      set_error("train: side-stream join failed");
      return XTRL_E_HIP;
    }
    return XTRL_OK;
  }
};

// C[M][N] = A[M][K] . W[N][K]^T (+ bias) with an epilogue
int linear_fwd(const Ctx& c, const float* A, int lda, const float* W, const float* bias, float* C, int ldc, int M,
               int N, int K, int epi, const float* R = nullptr, float* aux_out = nullptr, int ld_aux = 0,
               int act_cols = 1 << 30, int bias_col0 = 0, uint32_t drop_off = 0, uint32_t drop_layer = 0) {
  GemmArgs g;
  g.A = A; g.lda = lda; g.B = W; g.ldb = K; g.bias = bias; g.C = C; g.ldc = ldc; g.M = M; g.N = N; g.K = K;
  g.R = R; g.ldr = ldc; g.aux_out = aux_out; g.ld_aux_out = ld_aux; g.act_cols = act_cols; g.bias_col0 = bias_col0;
  if (epi == EPI_GELU_DROP) {
    g.seed = c.D->seed;
    g.drop_off = drop_off;
    g.drop_layer = drop_layer;
    g.drop_thresh = dropout_thresh(c.D->dropout);
    g.drop_thresh8 = dropout_thresh8(c.D->dropout);
    g.inv_keep = c.D->dropout > 0.f ? 1.f / (1.f - c.D->dropout) : 1.f;
  }
  return gemm_run(g, 0, 0, epi, c.s);
}

// dX[M][K] = dY[M][N] . W[N][K] with an epilogue
int linear_dgrad(const Ctx& c, const float* dY, int ldy, const float* W, float* dX, int ldx, int M, int N, int K,
                 int epi, const float* aux_in = nullptr, int ld_aux = 0, int act_cols = 1 << 30,
                 const float* aux_in2 = nullptr, int ld_aux2 = 0, float* aux_out = nullptr, int ld_aux_out = 0) {
  GemmArgs g;
  g.A = dY; g.lda = ldy; g.B = W; g.ldb = K; g.C = dX; g.ldc = ldx; g.M = M; g.N = K; g.K = N;
  g.aux_in = aux_in; g.ld_aux_in = ld_aux; g.act_cols = act_cols;
  g.aux_in2 = aux_in2; g.ld_aux_in2 = ld_aux2; g.aux_out = aux_out; g.ld_aux_out = ld_aux_out;
  return gemm_run(g, 0, 1, epi, c.s);
}

// dW += dY^T X (and the bias gradient db[n - db_n0] += column sums of dY for n >= db_n0)
int wgrad(const Ctx& c, const float* dY, int ldy, const float* X, int ldx, float* dW, int M, int N, int K,
          float* db = nullptr, int db_n0 = 0) {
  const GemmProfile prof{c.D->prof_events, c.D->prof_flops, c.D->prof_cap, c.D->prof_n};
  return gemm_wgrad(dY, ldy, X, ldx, dW, K, M, N, K, 1.f, c.D->ws, c.D->ws_floats, c.s, db, db_n0,
                    c.D->prof_events && c.D->prof_n ? &prof : nullptr, c.q);
}

// dst[0:cols] += sum over rows of src (optionally weighted by rw[r * ld_rw] * rw_scale)
int colsum(const Ctx& c, const float* src, int ld, int rows, int cols, float* dst, const float* rw = nullptr,
           int ld_rw = 0, float rw_scale = 1.f) {
  if (!dst || cols <= 0) return XTRL_OK;
  int chunks = std::min(1024, std::max(1, rows / 16));   // 16 rows per partial (loads in flight)
  const int chunk_rows = (rows + chunks - 1) / chunks;
  chunks = (rows + chunk_rows - 1) / chunk_rows;
  XTRL_REQUIRE((int64_t)chunks * cols <= c.D->part_floats, "train: partial-sum workspace too small");
  hipLaunchKernelGGL(k_colsum_part, dim3(blocks(cols, 256), chunks), dim3(256), 0, c.s, src, ld, rows, cols,
                     chunk_rows, rw, ld_rw, rw_scale, c.D->part);
  hipLaunchKernelGGL(k_colsum_final, dim3(blocks(cols, CS_COLS)), dim3(64 * CS_WAVES), 0, c.s, c.D->part, chunks, cols, dst);
  XTRL_LAUNCHED("train colsum");
  return XTRL_OK;
}

int ln_fwd(const Ctx& c, const float* x, const float* gamma, float* y1, int ld1, float* y2, int ld2, float* st) {
  hipLaunchKernelGGL(k_ln_fwd, dim3(blocks(c.T, 4)), dim3(256), 0, c.s, x, gamma, y1, ld1, y2, ld2, st, c.T,
                     c.D->d, c.D->rms_norm);
  XTRL_LAUNCHED("train ln_fwd");
  return XTRL_OK;
}

int ln_bwd(const Ctx& c, const float* g1, int ldg1, float s1, const float* g2, int ldg2, const float* x,
           const float* st, const float* gamma, const float* dres, float* dx, float* dgamma, float* dbeta = nullptr) {
  const int d = c.D->d, nb = (int)blocks(c.T, LN_ROWS);
  XTRL_REQUIRE((int64_t)nb * d * (dbeta ? 2 : 1) <= c.D->part_floats, "train: partial-sum workspace too small");
  // with d beta: the two partial rows of a block side by side ([gamma | beta], stride 2d), so one
  // column-sum launch finishes both when the parameters are adjacent (nn.LayerNorm weight, bias)
  const int ps = dbeta ? 2 * d : d;
  float* pb = dbeta ? c.D->part + d : nullptr;
  const dim3 g(nb), bl(64 * LN_WAVES);
  float* P = c.D->part;
  if (d <= 64) hipLaunchKernelGGL(k_ln_bwd<1>, g, bl, 0, c.s, g1, ldg1, s1, g2, ldg2, x, st, gamma, dres, dx, P, pb, ps, c.T, d, c.D->rms_norm);
  else if (d <= 128) hipLaunchKernelGGL(k_ln_bwd<2>, g, bl, 0, c.s, g1, ldg1, s1, g2, ldg2, x, st, gamma, dres, dx, P, pb, ps, c.T, d, c.D->rms_norm);
  else if (d <= 256) hipLaunchKernelGGL(k_ln_bwd<4>, g, bl, 0, c.s, g1, ldg1, s1, g2, ldg2, x, st, gamma, dres, dx, P, pb, ps, c.T, d, c.D->rms_norm);
  else hipLaunchKernelGGL(k_ln_bwd<8>, g, bl, 0, c.s, g1, ldg1, s1, g2, ldg2, x, st, gamma, dres, dx, P, pb, ps, c.T, d, c.D->rms_norm);
  if (!dbeta) {
    hipLaunchKernelGGL(k_colsum_final, dim3(blocks(d, CS_COLS)), dim3(64 * CS_WAVES), 0, c.s, P, nb, d, dgamma);
  } else if (dbeta == dgamma + d) {
    hipLaunchKernelGGL(k_colsum_final, dim3(blocks(2 * d, CS_COLS)), dim3(64 * CS_WAVES), 0, c.s, P, nb, 2 * d, dgamma);
  } else {
    XTRL_REQUIRE(false, "train: LayerNorm weight and bias gradients must be adjacent");
  }
  XTRL_LAUNCHED("train ln_bwd");
  return XTRL_OK;
}

// LayerNorm folded into the GEMM that produces / consumes its rows (gemm.hip EPI_RES_LN /
// EPI_LN_BWD): possible when one column tile holds the whole row and every operand is float4
bool ln_fusable(const XtrlTrainDesc* D) {
  static const bool on = [] {   // XTRL_FUSED_LN=0: separate LayerNorm launches (A/B experiments)
    const char* e = getenv("XTRL_FUSED_LN");
    return !(e && atoi(e) == 0);
  }();
  if (!on || D->d % 4 || D->d > 256 || (D->H * D->dh) % 4 || D->ff % 4 || D->in_dim % 4) return false;
  for (int li = 0; li < D->L; ++li)
    if (D->layers[li].n_qkv % 4) return false;
  return true;
}

// x_out = A W^T (+ bias) + R, then y1 (= y2) = LN(x_out) gamma and the row statistics, one launch
int linear_res_ln(const Ctx& c, const float* A, int lda, const float* W, const float* bias, const float* R,
                  float* x_out, int K, const float* gamma, float* y1, int ld1, float* y2, int ld2, float* st) {
  const int d = c.D->d;
  GemmArgs g;
  g.A = A; g.lda = lda; g.B = W; g.ldb = K; g.bias = bias; g.C = x_out; g.ldc = d; g.M = c.T; g.N = d; g.K = K;
  g.R = R; g.ldr = d; g.ln_g = gamma; g.ln_y1 = y1; g.ln_ld1 = ld1; g.ln_y2 = y2; g.ln_ld2 = ld2; g.ln_stats = st;
  g.ln_rms = c.D->rms_norm;
  return gemm_run(g, 0, 0, EPI_RES_LN, c.s);
}

// dx = LN_backward(dY W; x, stats, gamma) + dres in one launch; d gamma accumulated from the
// per-row-tile partials
int dgrad_ln_bwd(const Ctx& c, const float* dY, int ldy, const float* W, int N, const float* x, const float* st,
                 const float* gamma, const float* dres, float* dx, float* dgamma, ColsumQueue* cq = nullptr) {
  const int d = c.D->d, nb = (c.T + gemm_ln_rows(d) - 1) / gemm_ln_rows(d);
  XTRL_REQUIRE((int64_t)nb * d <= c.D->part_floats, "train: partial-sum workspace too small");
  int rc = XTRL_OK;
  float* P = cq ? cq->take_or_flush(nb, d, dgamma, c.s, &rc) : nullptr;   // deferred: the queue's one launch
  if (rc) return rc;
  GemmArgs g;
  g.A = dY; g.lda = ldy; g.B = W; g.ldb = d; g.C = dx; g.ldc = d; g.M = c.T; g.N = d; g.K = N;
  g.ln_g = gamma; g.ln_x = x; g.ln_stats = const_cast<float*>(st); g.ln_dres = dres; g.ln_part = P ? P : c.D->part;
  g.ln_rms = c.D->rms_norm;
  if ((rc = gemm_run(g, 0, 1, EPI_LN_BWD, c.s))) return rc;
  if (!P)
    hipLaunchKernelGGL(k_colsum_final, dim3(blocks(d, CS_COLS)), dim3(64 * CS_WAVES), 0, c.s, c.D->part, nb, d, dgamma);
  XTRL_LAUNCHED("train dgrad_ln_bwd");
  return XTRL_OK;
}

AttnProblem attn_problem(const Ctx& c, const XtrlTrainLayer& Ly, int li) {
  const XtrlTrainDesc* D = c.D;
  const int I = D->H * D->dh;
  AttnProblem p{};
  p.b = D->b;
  p.H = D->H;
  p.n = D->n;
  p.dh = D->dh;
  p.lens = D->lens;
  p.scale = D->attn_scale;
  p.dropout = D->dropout;
  p.seed = D->seed;
  p.offset = D->attn_offset;
  p.sub = (uint32_t)li;
  p.in = attn_layout_tokens(D->n, 3 * I, D->dh);
  p.out = attn_layout_tokens(D->n, I, D->dh);
  p.grad = attn_layout_tokens(D->n, Ly.n_qkv, D->dh);
  p.gate = attn_layout_tokens(D->n, Ly.n_qkv, D->dh);
  p.ep_off = D->packed ? D->ep_off : nullptr;
  p.dq_part = D->dq_part;
  p.dq_part_floats = D->dq_part_floats;
  return p;
}

int validate(const XtrlTrainDesc* D) {
  XTRL_REQUIRE(D && D->layers && D->flat && D->grad, "train: null descriptor / layers / parameters");
  XTRL_REQUIRE(D->b > 0 && D->n > 0 && D->d > 0 && D->L > 0 && D->H > 0 && D->dh > 0, "train: bad sizes");
  XTRL_REQUIRE(D->d <= 64 * kMaxDPerLane, "train: d = %d > %d unsupported", D->d, 64 * kMaxDPerLane);
  XTRL_REQUIRE(D->dh % 2 == 0 && D->rot_dim <= D->dh, "train: bad rotary dims");
  XTRL_REQUIRE(D->in_dim == D->d * (D->evolutionary ? 3 : 2), "train: in_dim mismatch");
  XTRL_REQUIRE(D->ld_ff == 0 || (D->ld_ff >= D->ff && D->ld_ff % 4 == 0), "train: ld_ff %d (ff %d)", D->ld_ff, D->ff);
  XTRL_REQUIRE(!D->ff_glu || (D->ld_u2 >= 2 * D->ff && D->ld_u2 % 4 == 0 && D->glu_dh),
               "train: ff_glu needs ld_u2 >= 2 ff (a multiple of 4) and glu_dh");
  XTRL_REQUIRE(!D->evolutionary || (D->latent && D->lat_e), "train: evolutionary needs latent buffers");
  XTRL_REQUIRE(D->S <= EMB_MAXS, "train: state_dim %d > %d unsupported", D->S, EMB_MAXS);
  XTRL_REQUIRE(D->continuous || D->A <= EMB_MAXA, "train: %d discrete actions > %d unsupported", D->A, EMB_MAXA);
  XTRL_REQUIRE(D->continuous ? (D->prev_action_f && D->next_action_f) : (D->prev_action && D->next_action),
               "train: missing action inputs");
  return XTRL_OK;
}

}  // namespace

// ---- valid-token rows of a minibatch (the world-model heads' compact form, XtrlTrainDesc.Tv) ---
namespace {
constexpr int VR_MAXB = 4096;
// vrows[0 .. Tv): the valid tokens' rows e n + t (t < lens[e]) in episode, then step order;
// vinv[r]: a row's index in that list, -1 for padding.  One workgroup (b <= VR_MAXB).  Tv (the
// host's count, sizing the compact GEMMs) is trusted for nothing: list entries at or past Tv are
// never written and their rows scatter as padding, and list slots past the device count read row 0,
// so a wrong Tv gives wrong heads outputs but no out-of-range or stale access.
__global__ __launch_bounds__(1024) void k_valid_rows(const int32_t* lens, int b, int n, int Tv, int32_t* vrows,
                                                     int32_t* vinv, int32_t* ep_off = nullptr) {
  __shared__ int off[VR_MAXB + 1];
  for (int e = threadIdx.x; e < b; e += 1024) off[e + 1] = min(max(lens[e], 0), n);
  __syncthreads();
  if (threadIdx.x == 0) {
    off[0] = 0;
    for (int e = 0; e < b; ++e) off[e + 1] += off[e];
  }
  __syncthreads();
  for (int r = threadIdx.x; r < b * n; r += 1024) {
    const int e = r / n, t = r - e * n;
    const int j = off[e] + t;
    if (t < off[e + 1] - off[e] && j < Tv) {
      vrows[j] = r;
      vinv[r] = j;
    } else {
      vinv[r] = -1;
    }
  }
  for (int j = off[b] + threadIdx.x; j < Tv; j += 1024) vrows[j] = 0;
  if (ep_off)   // (the packed learn step's episode row offsets; the prefix is final after the barrier)
    for (int e = threadIdx.x; e <= b; e += 1024) ep_off[e] = min(off[e], Tv);
}
// dst[i][0:cols] = src[rows[i]][0:cols] (V = 4: float4 columns)
template <int V>
__global__ void k_gather_rows(const float* src, int lds, const int32_t* rows, int nr, int cols, float* dst, int ldd) {
  const int cv = cols / V;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)nr * cv) return;
  const int r = (int)(i / cv), c = V * (int)(i - (int64_t)r * cv);
  const float* sp = src + (int64_t)rows[r] * lds + c;
  float* dp = dst + (int64_t)r * ldd + c;
  if constexpr (V == 4) *reinterpret_cast<float4*>(dp) = *reinterpret_cast<const float4*>(sp);
  else *dp = *sp;
}
// dst[r][0:cols] = inv[r] >= 0 ? src[inv[r]][0:cols] : 0 for r < T
template <int V>
__global__ void k_scatter_rows(const float* src, int lds, const int32_t* inv, int T, int cols, float* dst, int ldd) {
  const int cv = cols / V;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)T * cv) return;
  const int r = (int)(i / cv), c = V * (int)(i - (int64_t)r * cv);
  const int j = inv[r];
  float* dp = dst + (int64_t)r * ldd + c;
  if constexpr (V == 4)
    *reinterpret_cast<float4*>(dp) = j >= 0 ? *reinterpret_cast<const float4*>(src + (int64_t)j * lds + c)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
  else
    *dp = j >= 0 ? src[(int64_t)j * lds + c] : 0.f;
}
bool vec4_ok(const float* a, int lda, const float* b, int ldb, int cols) {
  return cols % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0;
}
void gather_rows(const float* src, int lds, const int32_t* rows, int nr, int cols, float* dst, int ldd, hipStream_t s) {
  const bool v4 = vec4_ok(src, lds, dst, ldd, cols);
  const int64_t units = (int64_t)nr * (v4 ? cols / 4 : cols);
  if (v4) hipLaunchKernelGGL(k_gather_rows<4>, dim3(blocks(units, 256)), dim3(256), 0, s, src, lds, rows, nr, cols, dst, ldd);
  else hipLaunchKernelGGL(k_gather_rows<1>, dim3(blocks(units, 256)), dim3(256), 0, s, src, lds, rows, nr, cols, dst, ldd);
}
void scatter_rows(const float* src, int lds, const int32_t* inv, int T, int cols, float* dst, int ldd, hipStream_t s) {
  const bool v4 = vec4_ok(src, lds, dst, ldd, cols);
  const int64_t units = (int64_t)T * (v4 ? cols / 4 : cols);
  if (v4) hipLaunchKernelGGL(k_scatter_rows<4>, dim3(blocks(units, 256)), dim3(256), 0, s, src, lds, inv, T, cols, dst, ldd);
  else hipLaunchKernelGGL(k_scatter_rows<1>, dim3(blocks(units, 256)), dim3(256), 0, s, src, lds, inv, T, cols, dst, ldd);
}
// the world-model heads run on the valid rows only (XtrlTrainDesc.Tv; XTRL_HEADS_COMPACT=0: every row)
bool heads_compact(const Ctx& c) {
  static const bool on = [] {
    const char* e = getenv("XTRL_HEADS_COMPACT");
    return !(e && atoi(e) == 0);
  }();
  const XtrlTrainDesc* D = c.D;
  return on && D->Tv > 0 && D->Tv < c.T && D->b <= VR_MAXB && D->vrows && D->vinv && D->ewa_v && D->hp_v &&
         D->zp_v && D->pred_v && D->d_pred_v && D->dzp_v && D->dewa_v;
}
}  // namespace

// ---- the heads every policy body shares (xtrl.py:533-557, fractal_rl.py:586-619) -------------
// input: ac_in = [embed | state embed (| latent embed)], ewa = [embed | next-action embed]
int heads_forward(const Ctx& c) {
  const XtrlTrainDesc* D = c.D;
  const int T = c.T, d = D->d, ldp = d + 4;
  const hipStream_t s = c.s;
  int rc;
  const int S1x2 = 2 * (D->S + 1);
  if (heads_compact(c)) {
    // world-model heads over the Tv valid rows: their outputs feed only masked losses (xtrl.py:944,
    // 949), the padded rows' pred / done are stored as zeros
    const int Tv = D->Tv;
    hipLaunchKernelGGL(k_valid_rows, dim3(1), dim3(1024), 0, s, D->lens, D->b, D->n, D->Tv, D->vrows, D->vinv);
    gather_rows(D->ewa, 2 * d, D->vrows, Tv, 2 * d, D->ewa_v, 2 * d, s);
    if ((rc = linear_fwd(c, D->ewa_v, 2 * d, c.P(D->w_pd), c.P(D->b_pd), D->hp_v, ldp, Tv, d + 1, 2 * d, EPI_SILU_SAVE,
                         nullptr, D->zp_v, ldp, d)))
      return rc;
    if ((rc = linear_fwd(c, D->hp_v, ldp, c.P(D->w_pred2), c.P(D->b_pred2), D->pred_v, S1x2, Tv, S1x2, d, EPI_NONE)))
      return rc;
    scatter_rows(D->pred_v, S1x2, D->vinv, T, S1x2, D->pred, S1x2, s);
    scatter_rows(D->hp_v + d, ldp, D->vinv, T, 1, D->done, 1, s);
  } else {
    // world-model heads: to_pred.0 | to_pred_done in one GEMM (SiLU on the first d columns)
    if ((rc = linear_fwd(c, D->ewa, 2 * d, c.P(D->w_pd), c.P(D->b_pd), D->hp, ldp, T, d + 1, 2 * d, EPI_SILU_SAVE,
                         nullptr, D->zp, ldp, d)))
      return rc;
    if ((rc = linear_fwd(c, D->hp, ldp, c.P(D->w_pred2), c.P(D->b_pred2), D->pred, S1x2, T, S1x2, d, EPI_NONE)))
      return rc;
    hipLaunchKernelGGL(k_copy_col, dim3(blocks(T, 256)), dim3(256), 0, s, D->hp + d, ldp, D->done, 1, T);
  }
  // actor | critic first layers in one GEMM, then the two output layers
  if ((rc = linear_fwd(c, D->ac_in, D->in_dim, c.P(D->w_h1), c.P(D->b_h1), D->h1, 4 * d, T, 4 * d, D->in_dim,
                       EPI_SILU_SAVE, nullptr, D->z1, 4 * d)))
    return rc;
  if ((rc = linear_fwd(c, D->h1, 4 * d, c.P(D->w_a2), c.P(D->b_a2), D->raw, D->n_out, T, D->n_out, 2 * d, EPI_NONE)))
    return rc;
  if ((rc = linear_fwd(c, D->h1 + 2 * d, 4 * d, c.P(D->w_c2), c.P(D->b_c2), D->values, D->B, T, D->B, 2 * d,
                       EPI_NONE)))
    return rc;
  XTRL_LAUNCHED("train heads");
  return XTRL_OK;
}

// heads backward -> dac (gradient of ac_in), dewa (of ewa); the weight gradients of the heads, the
// state embedding and the gene conditioning (c: main stream, cw: weight-gradient stream)
int heads_backward(const Ctx& c, const Ctx& cw, Fork& F, bool embed_cols = true) {
  const XtrlTrainDesc* D = c.D;
  const int T = c.T, d = D->d, ldp = d + 4, S1x2 = 2 * (D->S + 1);
  const hipStream_t s = c.s;
  int rc;
  // (compact world-model heads) their output gradients on the valid rows, before the first fork so
  // the weight-gradient stream sees them: d_pred -> d_pred_v, d_done -> column d of dzp_v
  const bool cmp = heads_compact(c);
  if (cmp) {
    gather_rows(D->d_pred, S1x2, D->vrows, D->Tv, S1x2, D->d_pred_v, S1x2, s);
    gather_rows(D->d_done, 1, D->vrows, D->Tv, 1, D->dzp_v + d, ldp, s);
  }
  // ---- actor / critic heads
  if ((rc = F.fork())) return rc;
  if ((rc = wgrad(cw, D->d_raw, D->n_out, D->h1, 4 * d, c.G(D->w_a2), T, D->n_out, 2 * d, c.G(D->b_a2)))) return rc;
  if ((rc = wgrad(cw, D->d_values, D->B, D->h1 + 2 * d, 4 * d, c.G(D->w_c2), T, D->B, 2 * d, c.G(D->b_c2)))) return rc;
  if ((rc = linear_dgrad(c, D->d_raw, D->n_out, c.P(D->w_a2), D->dz1, 4 * d, T, D->n_out, 2 * d, EPI_MUL_AUX, D->z1,
                         4 * d)))
    return rc;
  if ((rc = linear_dgrad(c, D->d_values, D->B, c.P(D->w_c2), D->dz1 + 2 * d, 4 * d, T, D->B, 2 * d, EPI_MUL_AUX,
                         D->z1 + 2 * d, 4 * d)))
    return rc;
  if ((rc = F.fork())) return rc;
  if ((rc = wgrad(cw, D->dz1, 4 * d, D->ac_in, D->in_dim, c.G(D->w_h1), T, 4 * d, D->in_dim, c.G(D->b_h1)))) return rc;
  if (embed_cols) {
    if ((rc = linear_dgrad(c, D->dz1, 4 * d, c.P(D->w_h1), D->dac, D->in_dim, T, 4 * d, D->in_dim, EPI_NONE))) return rc;
  } else {   // columns [d, in_dim) only: the caller folds the embed columns into its final-norm backward
    GemmArgs g;
    g.A = D->dz1; g.lda = 4 * d; g.B = c.P(D->w_h1) + d; g.ldb = D->in_dim; g.C = D->dac + d; g.ldc = D->in_dim;
    g.M = T; g.N = D->in_dim - d; g.K = 4 * d;
    if ((rc = gemm_run(g, 0, 1, EPI_NONE, c.s))) return rc;
  }
  // state embedding and gene conditioning
  if ((rc = F.fork())) return rc;
  if ((rc = wgrad(cw, D->dac + d, D->in_dim, D->swr, D->S + 1, c.G(D->w_se), T, d, D->S, c.G(D->b_se)))) return rc;
  if (D->evolutionary) {
    XTRL_REQUIRE((int64_t)D->b * d <= D->part_floats, "train: partial-sum workspace too small");
    hipLaunchKernelGGL(k_latent_grad, dim3(D->b, (d + 63) / 64), dim3(64 * LG_G), 0, s, D->dac, D->in_dim, 2 * d,
                       D->b, D->n, d, D->part, D->packed ? D->ep_off : nullptr);
    hipLaunchKernelGGL(k_latent_wgrad, dim3(blocks(d * (D->G + 1), 256)), dim3(256), 0, s, D->part, D->latent, D->b,
                       d, D->G, c.G(D->w_lat), c.G(D->b_lat));
    XTRL_LAUNCHED("train latent grad");
  }
  // ---- world-model heads
  if (cmp) {   // on the Tv valid rows; dewa's padded rows are zero (their dzp rows were)
    const int Tv = D->Tv;
    if ((rc = wgrad(cw, D->d_pred_v, S1x2, D->hp_v, ldp, c.G(D->w_pred2), Tv, S1x2, d, c.G(D->b_pred2)))) return rc;
    if ((rc = linear_dgrad(c, D->d_pred_v, S1x2, c.P(D->w_pred2), D->dzp_v, ldp, Tv, S1x2, d, EPI_MUL_AUX, D->zp_v,
                           ldp)))
      return rc;
    if ((rc = F.fork())) return rc;
    if ((rc = wgrad(cw, D->dzp_v, ldp, D->ewa_v, 2 * d, c.G(D->w_pd), Tv, d + 1, 2 * d, c.G(D->b_pd)))) return rc;
    if ((rc = linear_dgrad(c, D->dzp_v, ldp, c.P(D->w_pd), D->dewa_v, 2 * d, Tv, d + 1, 2 * d, EPI_NONE))) return rc;
    scatter_rows(D->dewa_v, 2 * d, D->vinv, T, 2 * d, D->dewa, 2 * d, s);
    XTRL_LAUNCHED("train heads backward (compact)");
    return XTRL_OK;
  }
  if ((rc = wgrad(cw, D->d_pred, S1x2, D->hp, ldp, c.G(D->w_pred2), T, S1x2, d, c.G(D->b_pred2)))) return rc;
  if ((rc = linear_dgrad(c, D->d_pred, S1x2, c.P(D->w_pred2), D->dzp, ldp, T, S1x2, d, EPI_MUL_AUX, D->zp, ldp))) return rc;
  hipLaunchKernelGGL(k_copy_col, dim3(blocks(T, 256)), dim3(256), 0, s, D->d_done, 1, D->dzp + d, ldp, T);
  if ((rc = F.fork())) return rc;
  if ((rc = wgrad(cw, D->dzp, ldp, D->ewa, 2 * d, c.G(D->w_pd), T, d + 1, 2 * d, c.G(D->b_pd)))) return rc;
  if ((rc = linear_dgrad(c, D->dzp, ldp, c.P(D->w_pd), D->dewa, 2 * d, T, d + 1, 2 * d, EPI_NONE))) return rc;
  return XTRL_OK;
}

// ============================================================================================
int train_forward_rows(const XtrlTrainDesc* D, int Trows, hipStream_t s) {
  if (int rc = validate(D)) return rc;
  const Ctx c{D, s, Trows};
  const int32_t* rows = D->packed ? D->vrows : nullptr;
  const int T = c.T, d = D->d, I = D->H * D->dh, ff = D->ff, lf = ld_ff(D);
  int rc;
  // embeddings
  if (D->evolutionary) {
    hipLaunchKernelGGL(k_latent_embed, dim3(blocks(D->b * d, 256)), dim3(256), 0, s, D->latent, c.P(D->w_lat),
                       c.P(D->b_lat), D->lat_e, D->b, D->G, d);
  }
  EmbedArgs ea{D->swr, c.P(D->w_pin), c.P(D->act_emb), c.P(D->act_emb_b), c.P(D->reward_embed), c.P(D->w_se),
               c.P(D->b_se), D->lat_e, D->prev_action_f, D->next_action_f, D->prev_action, D->next_action,
               D->layers[0].x_attn, D->ac_in, D->ewa, T, D->n, D->S, D->A, d, D->in_dim, D->continuous,
               D->evolutionary, D->reward_keep, nullptr, nullptr, nullptr, D->rms_norm, rows};
  // fused: every LayerNorm is formed by the kernel that completes its rows — layer 0's attention
  // pre-norm by the embedding, the others in the epilogue of the GEMM before them (out-projection +
  // residual, FF2 + residual)
  const bool fuse = ln_fusable(D);
  if (fuse) {
    const XtrlTrainLayer& L0 = D->layers[0];
    ea.ln_g = c.P(L0.ln_attn);
    ea.xn = L0.xn_attn;
    ea.st = L0.st_attn;
    if (D->S == 8) hipLaunchKernelGGL(k_embed_ln<8>, dim3(blocks(T, EMB_LN_TOK)), dim3(256), 0, s, ea);
    else hipLaunchKernelGGL(k_embed_ln<0>, dim3(blocks(T, EMB_LN_TOK)), dim3(256), 0, s, ea);
  } else if (D->S == 8) {
    hipLaunchKernelGGL(k_embed<8>, dim3(blocks(T, EMB_TOK)), dim3(256), 0, s, ea);
  } else {
    hipLaunchKernelGGL(k_embed<0>, dim3(blocks(T, EMB_TOK)), dim3(256), 0, s, ea);
  }
  XTRL_LAUNCHED("train embed");
  for (int li = 0; li < D->L; ++li) {
    const XtrlTrainLayer& Ly = D->layers[li];
    if (!fuse)
      if ((rc = ln_fwd(c, Ly.x_attn, c.P(Ly.ln_attn), Ly.xn_attn, d, nullptr, 0, Ly.st_attn))) return rc;
    if ((rc = linear_fwd(c, Ly.xn_attn, d, c.P(Ly.w_proj), c.P(Ly.b_proj), Ly.proj, Ly.n_qkv, T, Ly.n_qkv, d,
                         EPI_NONE, nullptr, nullptr, 0, 1 << 30, 3 * I)))
      return rc;
    const int mix_col = Ly.mix ? 3 * I + (D->gate_values ? I : 0) : -1;
    PrepArgs pa{Ly.proj, D->layers[0].proj, Ly.qkv, D->inv_freq, T, D->n, D->H, D->dh, I, Ly.n_qkv,
                D->layers[0].n_qkv, D->rot_dim, mix_col, D->qk_norm, D->xpos_base, rows};
    const dim3 pg = rows ? dim3(blocks(3 * I / 2, PREP_T), T) : dim3(blocks(3 * I / 2, PREP_T), D->n, D->b);
    hipLaunchKernelGGL(k_qkv_prep, pg, dim3(PREP_T), 0, s, pa);
    XTRL_LAUNCHED("train qkv_prep");
    const AttnProblem ap = attn_problem(c, Ly, li);
    if ((rc = attn_fwd_ex(ap, Ly.qkv, Ly.qkv + I, Ly.qkv + 2 * I, Ly.o, Ly.lse,
                          D->gate_values ? Ly.proj + 3 * I : nullptr, D->gate_values ? Ly.og : nullptr, s)))
      return rc;
    if (fuse) {
      if ((rc = linear_res_ln(c, D->gate_values ? Ly.og : Ly.o, I, c.P(Ly.w_out), nullptr, Ly.x_attn, Ly.x_ff, I,
                              c.P(Ly.ln_ff), Ly.xn_ff, d, nullptr, 0, Ly.st_ff)))
        return rc;
    } else {
      if ((rc = linear_fwd(c, D->gate_values ? Ly.og : Ly.o, I, c.P(Ly.w_out), nullptr, Ly.x_ff, d, T, d, I, EPI_NONE,
                           Ly.x_attn)))
        return rc;
      if ((rc = ln_fwd(c, Ly.x_ff, c.P(Ly.ln_ff), Ly.xn_ff, d, nullptr, 0, Ly.st_ff))) return rc;
    }
    if (D->ff_glu) {   // GLU projection [T][2 ff] into u, then drop(value * GELU(gate)) into hd
      if ((rc = linear_fwd(c, Ly.xn_ff, d, c.P(Ly.w_ff1), c.P(Ly.b_ff1), Ly.u, D->ld_u2, T, 2 * ff, d, EPI_NONE)))
        return rc;
      if ((rc = glu_fwd(Ly.u, D->ld_u2, Ly.hd, lf, T, ff, D->dropout, D->seed, D->ff_offset, (uint32_t)li, s)))
        return rc;
    } else if ((rc = linear_fwd(c, Ly.xn_ff, d, c.P(Ly.w_ff1), c.P(Ly.b_ff1), Ly.hd, lf, T, ff, d, EPI_GELU_DROP,
                                nullptr, Ly.u, lf, 1 << 30, 0, D->ff_offset, (uint32_t)li))) {
      return rc;
    }
    float* x_out = li + 1 < D->L ? D->layers[li + 1].x_attn : D->x_final;
    if (fuse && li + 1 < D->L) {   // + the next block's attention pre-norm
      const XtrlTrainLayer& Ln = D->layers[li + 1];
      if ((rc = linear_res_ln(c, Ly.hd, lf, c.P(Ly.w_ff2), c.P(Ly.b_ff2), Ly.x_ff, x_out, ff, c.P(Ln.ln_attn),
                              Ln.xn_attn, d, nullptr, 0, Ln.st_attn)))
        return rc;
    } else if (fuse) {             // + the final norm -> embed, into ac_in[:, :d] and ewa[:, :d]
      if ((rc = linear_res_ln(c, Ly.hd, lf, c.P(Ly.w_ff2), c.P(Ly.b_ff2), Ly.x_ff, x_out, ff, c.P(D->ln_final),
                              D->ac_in, D->in_dim, D->ewa, 2 * d, D->st_final)))
        return rc;
    } else {
      if ((rc = linear_fwd(c, Ly.hd, lf, c.P(Ly.w_ff2), c.P(Ly.b_ff2), x_out, d, T, d, ff, EPI_NONE, Ly.x_ff))) return rc;
    }
  }
  // final norm -> embed, into ac_in[:, :d] and ewa[:, :d]
  if (!fuse)
    if ((rc = ln_fwd(c, D->x_final, c.P(D->ln_final), D->ac_in, D->in_dim, D->ewa, 2 * d, D->st_final))) return rc;
  if ((rc = heads_forward(c))) return rc;
  XTRL_LAUNCHED("train forward");
  return XTRL_OK;
}

// ============================================================================================
int train_backward_rows(const XtrlTrainDesc* D, int Trows, hipStream_t s) {
  if (int rc = validate(D)) return rc;
  XTRL_REQUIRE(D->d_raw && D->d_values && D->d_pred && D->d_done, "train: missing loss gradients");
  const Ctx c{D, s, Trows};
  const int32_t* rows = D->packed ? D->vrows : nullptr;
  const int T = c.T, d = D->d, I = D->H * D->dh, ff = D->ff, lf = ld_ff(D);
  int rc;
  SideStream& side = side_stream();
  const bool two = side.ok && side.ensure(side_events_needed(D->L));
  Fork F{s, side.s, two ? &side : nullptr};
  // weight gradients (side stream); their split-K partials are summed by one launch at the end
  // (XTRL_SPLITK_DEFER=0: a reduce launch after every weight-gradient GEMM)
  static const bool defer = [] {
    const char* e = getenv("XTRL_SPLITK_DEFER");
    return !(e && atoi(e) == 0);
  }();
  // the LayerNorm d gamma sums of the final norm and the decoder blocks: deferred to one launch after
  // the blocks (nothing else writes the partial workspace until the embeddings), or at each gradient
  // bucket; XTRL_LN_COLSUM_DEFER=0: a column-sum launch after every LayerNorm-backward GEMM
  static const bool cs_defer = [] {
    const char* e = getenv("XTRL_LN_COLSUM_DEFER");
    return !(e && atoi(e) == 0);
  }();
  ColsumQueue csq;
  if (cs_defer && ln_fusable(D) && D->scratch_per_layer) {
    csq.base = D->part;
    csq.cap = D->part_floats;
  }
  SplitKQueue skq;
  const Ctx cw{D, two ? side.s : s, T, defer ? &skq : nullptr};
  // data-parallel gradient buckets: flush the bucket's deferred reductions, then record its events
  int bucket = 0;
  auto bucket_done = [&]() -> int {
    if (!D->grad_events) return XTRL_OK;
    if (int rc = csq.flush(s)) return rc;
    if (int rc = splitk_flush(skq, cw.s)) return rc;
    if (hipEventRecord((hipEvent_t)D->grad_events[2 * bucket], s) != hipSuccess ||
        hipEventRecord((hipEvent_t)D->grad_events[2 * bucket + 1], cw.s) != hipSuccess) {
      set_error("train: gradient bucket event record failed");
      return XTRL_E_HIP;
    }
    ++bucket;
    return XTRL_OK;
  };
  const bool per_layer = ln_fusable(D) && D->scratch_per_layer;
  float* dx_top = per_layer ? D->dx + (int64_t)D->L * T * d : D->dx;   // (scratch_per_layer: slot L)
  // ---- final norm: d embed = frac * dac[:, :d] + dewa[:, :d].  Fused: the embed columns of the
  // actor | critic input gradient finish the final norm's backward in their GEMM's epilogue (no
  // LayerNorm launch); otherwise dac in full, then k_ln_bwd
  const bool fold = ln_fusable(D);
  if ((rc = heads_backward(c, cw, F, !fold))) return rc;
  if (fold) {
    const int nb = (T + gemm_ln_rows(d) - 1) / gemm_ln_rows(d);
    XTRL_REQUIRE((int64_t)nb * d <= D->part_floats, "train: partial-sum workspace too small");
    GemmArgs g;
    g.A = D->dz1; g.lda = 4 * d; g.B = c.P(D->w_h1); g.ldb = D->in_dim; g.C = dx_top; g.ldc = d;
    g.M = T; g.N = d; g.K = 4 * d;
    g.ln_g = c.P(D->ln_final); g.ln_x = D->x_final; g.ln_stats = D->st_final; g.ln_rms = D->rms_norm;
    float* P = csq.take_or_flush(nb, d, c.G(D->ln_final), s, &rc);
    if (rc) return rc;
    g.ln_gpre = D->dewa; g.ln_ldg = 2 * d; g.ln_gscale = D->frac_head_grad; g.ln_part = P ? P : D->part;
    if ((rc = gemm_run(g, 0, 1, EPI_LN_BWD2, s))) return rc;
    if (!P)
      hipLaunchKernelGGL(k_colsum_final, dim3(blocks(d, CS_COLS)), dim3(64 * CS_WAVES), 0, s, D->part, nb, d,
                         c.G(D->ln_final));
    XTRL_LAUNCHED("train final-norm backward");
  } else if ((rc = ln_bwd(c, D->dac, D->in_dim, D->frac_head_grad, D->dewa, 2 * d, D->x_final, D->st_final,
                          c.P(D->ln_final), nullptr, dx_top, c.G(D->ln_final)))) {
    return rc;
  }
  if ((rc = bucket_done())) return rc;   // bucket 0: heads, state / gene embeddings, final norm
  // ---- decoder blocks, last to first.  Side events of the weight gradients whose dY buffer the
  // main stream overwrites later: dx (FF2 / out-projection), dff (FF1, by the next layer's FF2
  // input gradient), dproj (q|k|v projection, by the next layer's gate / attention backward).
  // Fused LayerNorm backward (ln_fusable): the FF1 and q|k|v input-gradient GEMMs finish the
  // LayerNorm backward and add the residual gradient in their epilogue, alternating between dx and
  // dx2, so neither overwrites the buffer a pending side-stream weight gradient still reads: the FF
  // block writes dx2 (read by the out-projection weight gradient), the attention block writes dx
  // (read by the next FF2 weight gradient).
  const bool fuse = ln_fusable(D);
  XTRL_REQUIRE(!fuse || D->dx2, "train: fused LayerNorm backward needs dx2");
  // scratch_per_layer (fused path): every buffer a side-stream weight gradient reads is a per-layer
  // plane written once per backward — dx [L + 1][T][d] (slot l + 1: the gradient w.r.t. block l's
  // output, slot 0 w.r.t. the embedding), dx2 [L][T][d] (w.r.t. block l's attention output), dff
  // [L][T][ld_ff], dproj [L][T][max n_qkv] — so the main stream never waits for the side stream
  // before the final join (the waits below are skipped)
  const bool per = per_layer;
  int maxq = 0;
  for (int li = 0; li < D->L; ++li) maxq = std::max(maxq, D->layers[li].n_qkv);
  const int64_t Td = (int64_t)T * d;
  auto Gx = [&](int slot) { return per ? D->dx + slot * Td : D->dx; };
  auto Gx2 = [&](int li) { return per ? D->dx2 + li * Td : D->dx2; };
  // dff: the FF1 output gradient [T][ld_f1] (GLU: the projection's [T][2 ff] on the ld_u2 stride)
  const int f1 = D->ff_glu ? 2 * ff : ff, ld_f1 = D->ff_glu ? D->ld_u2 : lf;
  auto Gff = [&](int li) { return per ? D->dff + (int64_t)li * T * ld_f1 : D->dff; };
  auto Gpr = [&](int li) { return per ? D->dproj + (int64_t)li * T * maxq : D->dproj; };
  auto wait = [&](hipEvent_t e) { return per ? XTRL_OK : F.wait(e); };
  hipEvent_t e_ff1 = nullptr, e_proj = nullptr, e_out_prev = nullptr;
  for (int li = D->L - 1; li >= 0; --li) {
    const XtrlTrainLayer& Ly = D->layers[li];
    float* gout = Gx(li + 1);   // gradient w.r.t. the block output
    float* dff = Gff(li);
    float* dproj = Gpr(li);
    // FF2 (+ residual)
    if ((rc = F.fork())) return rc;
    if ((rc = wgrad(cw, gout, d, Ly.hd, lf, c.G(Ly.w_ff2), T, d, ff, c.G(Ly.b_ff2)))) return rc;
    hipEvent_t e_ff2 = F.mark();
    if ((rc = wait(e_ff1))) return rc;
    if (D->ff_glu) {   // d hd, then the GLU backward into the projection gradient
      if ((rc = linear_dgrad(c, gout, d, c.P(Ly.w_ff2), D->glu_dh, lf, T, d, ff, EPI_NONE))) return rc;
      if ((rc = glu_bwd(D->glu_dh, lf, Ly.u, D->ld_u2, dff, ld_f1, T, ff, D->dropout, D->seed, D->ff_offset,
                        (uint32_t)li, s)))
        return rc;
    } else if ((rc = linear_dgrad(c, gout, d, c.P(Ly.w_ff2), dff, lf, T, d, ff, EPI_MUL_AUX, Ly.u, lf))) {
      return rc;
    }
    if ((rc = F.fork())) return rc;
    if ((rc = wgrad(cw, dff, ld_f1, Ly.xn_ff, d, c.G(Ly.w_ff1), T, f1, d, c.G(Ly.b_ff1)))) return rc;
    e_ff1 = F.mark();
    float* xg = D->dx;   // gradient w.r.t. the attention block's output
    if (fuse) {
      if ((rc = wait(e_out_prev))) return rc;   // the deeper block's out-projection weight gradient read dx2
      if ((rc = dgrad_ln_bwd(c, dff, ld_f1, c.P(Ly.w_ff1), f1, Ly.x_ff, Ly.st_ff, c.P(Ly.ln_ff), gout, Gx2(li),
                             c.G(Ly.ln_ff), &csq)))
        return rc;
      xg = Gx2(li);
    } else {
      if ((rc = linear_dgrad(c, dff, ld_f1, c.P(Ly.w_ff1), D->dxn, d, T, f1, d, EPI_NONE))) return rc;
      if ((rc = F.wait(e_ff2))) return rc;
      if ((rc = ln_bwd(c, D->dxn, d, 1.f, nullptr, 0, Ly.x_ff, Ly.st_ff, c.P(Ly.ln_ff), D->dx, D->dx, c.G(Ly.ln_ff))))
        return rc;
    }
    // attention out-projection (+ residual) and the value gate
    if ((rc = F.fork())) return rc;
    if ((rc = wgrad(cw, xg, d, D->gate_values ? Ly.og : Ly.o, I, c.G(Ly.w_out), T, d, I))) return rc;
    hipEvent_t e_out = F.mark();
    if ((rc = wait(e_proj))) return rc;
    if (D->gate_values) {
      if ((rc = linear_dgrad(c, xg, d, c.P(Ly.w_out), D->dog, I, T, d, I, EPI_DGATE, Ly.o, I, 1 << 30,
                             Ly.proj + 3 * I, Ly.n_qkv, dproj + 3 * I, Ly.n_qkv)))
        return rc;
    } else {
      if ((rc = linear_dgrad(c, xg, d, c.P(Ly.w_out), D->dog, I, T, d, I, EPI_NONE))) return rc;
    }
    const AttnProblem ap = attn_problem(c, Ly, li);
    if ((rc = attn_bwd_ex(ap, Ly.qkv, Ly.qkv + I, Ly.qkv + 2 * I, Ly.o, Ly.lse, D->dog, dproj, dproj + I,
                          dproj + 2 * I, D->delta, s)))
      return rc;
    const int mix_col = Ly.mix ? 3 * I + (D->gate_values ? I : 0) : -1;
    const bool any_mix = [&] {
      for (int j = 1; j < D->L; ++j)
        if (D->layers[j].mix) return true;
      return false;
    }();
    // dvfirst: the first mixing layer processed (the deepest) writes, the others accumulate
    bool deeper_mix = false;
    for (int j = li + 1; j < D->L; ++j) deeper_mix = deeper_mix || D->layers[j].mix;
    PrepBwdArgs pb{dproj, Ly.proj, D->layers[0].proj, D->dvfirst, D->inv_freq, T, D->n, D->H, D->dh, I,
                   Ly.n_qkv, D->layers[0].n_qkv, D->rot_dim, mix_col, li == 0 ? 1 : 0,
                   (li == 0 ? any_mix : deeper_mix) ? 1 : 0, D->qk_norm, D->xpos_base, rows};
    const dim3 pg = rows ? dim3(blocks(3 * I / 2, PREP_T), T) : dim3(blocks(3 * I / 2, PREP_T), D->n, D->b);
    hipLaunchKernelGGL(k_qkv_prep_bwd, pg, dim3(PREP_T), 0, s, pb);
    XTRL_LAUNCHED("train qkv_prep_bwd");
    // q | k | v | gate | mix projection
    if ((rc = F.fork())) return rc;
    if ((rc = wgrad(cw, dproj, Ly.n_qkv, Ly.xn_attn, d, c.G(Ly.w_proj), T, Ly.n_qkv, d, c.G(Ly.b_proj), 3 * I)))
      return rc;
    e_proj = F.mark();
    if (fuse) {
      if ((rc = wait(e_ff2))) return rc;   // this block's FF2 weight gradient read dx
      if ((rc = dgrad_ln_bwd(c, dproj, Ly.n_qkv, c.P(Ly.w_proj), Ly.n_qkv, Ly.x_attn, Ly.st_attn, c.P(Ly.ln_attn),
                             Gx2(li), Gx(li), c.G(Ly.ln_attn), &csq)))
        return rc;
      e_out_prev = e_out;
    } else {
      if ((rc = linear_dgrad(c, dproj, Ly.n_qkv, c.P(Ly.w_proj), D->dxn, d, T, Ly.n_qkv, d, EPI_NONE))) return rc;
      if ((rc = F.wait(e_out))) return rc;
      if ((rc = ln_bwd(c, D->dxn, d, 1.f, nullptr, 0, Ly.x_attn, Ly.st_attn, c.P(Ly.ln_attn), D->dx, D->dx,
                       c.G(Ly.ln_attn))))
        return rc;
    }
    if ((rc = bucket_done())) return rc;   // bucket L - li: decoder block li
  }
  if ((rc = csq.flush(s))) return rc;   // (before the embeddings reuse the partial workspace)
  // ---- embeddings: dx is d x0.  The deferred split-K sums start now on the side stream, beside the
  // embedding backward, and project_in's small weight gradient runs on the main stream into the
  // workspace behind them (its immediate reduce; the backward's tail was that gradient waiting for its
  // fork, then the whole flush).  XTRL_WPIN_MAIN=0: on the side stream, before the flush.
  static const bool wpin_main = [] {
    const char* e = getenv("XTRL_WPIN_MAIN");
    return !(e && atoi(e) == 0);
  }();
  const bool wpin_on_main = wpin_main && !D->continuous && !D->grad_events && skq.used < D->ws_floats;
  if (wpin_on_main) {
    const int64_t used0 = skq.used;
    if ((rc = splitk_flush(skq, cw.s))) return rc;
    if ((rc = gemm_wgrad(D->dx, d, D->swr, D->S + 1, c.G(D->w_pin), D->S, T, d, D->S, 1.f, D->ws + used0,
                         D->ws_floats - used0, s, nullptr, 0, nullptr, nullptr)))
      return rc;
  } else {
    if ((rc = F.fork())) return rc;
    if ((rc = wgrad(cw, D->dx, d, D->swr, D->S + 1, c.G(D->w_pin), T, d, D->S))) return rc;
  }
  if ((rc = colsum(c, D->dx, d, T, d, c.G(D->reward_embed), D->swr + D->S, D->S + 1, D->reward_keep))) return rc;
  if (D->continuous) {
    if ((rc = wgrad(cw, D->dx, d, D->prev_action_f, D->A, c.G(D->act_emb), T, d, D->A))) return rc;
    if ((rc = wgrad(cw, D->dewa + d, 2 * d, D->next_action_f, D->A, c.G(D->act_emb), T, d, D->A))) return rc;
    if ((rc = colsum(c, D->dx, d, T, d, c.G(D->act_emb_b)))) return rc;
    if ((rc = colsum(c, D->dewa + d, 2 * d, T, d, c.G(D->act_emb_b)))) return rc;
  } else {
    // 16-row partials (loads in flight), as many as the partial workspace holds
    int chunks = std::min<int64_t>(std::min(1024, std::max(1, T / 16)),
                                   std::max<int64_t>(1, D->part_floats / ((int64_t)D->A * d)));
    const int chunk_rows = (T + chunks - 1) / chunks;
    chunks = (T + chunk_rows - 1) / chunk_rows;
    XTRL_REQUIRE((int64_t)chunks * D->A * d <= D->part_floats, "train: partial-sum workspace too small");
    const dim3 eg(blocks(d, 256), chunks);
    if (D->A <= 4)
      hipLaunchKernelGGL(k_embed_grad_part<4>, eg, dim3(256), 0, s, D->dx, d, D->prev_action, D->dewa + d, 2 * d,
                         D->next_action, T, d, D->A, chunk_rows, D->part);
    else if (D->A <= 8)
      hipLaunchKernelGGL(k_embed_grad_part<8>, eg, dim3(256), 0, s, D->dx, d, D->prev_action, D->dewa + d, 2 * d,
                         D->next_action, T, d, D->A, chunk_rows, D->part);
    else
      hipLaunchKernelGGL(k_embed_grad_part<EMB_MAXA>, eg, dim3(256), 0, s, D->dx, d, D->prev_action, D->dewa + d,
                         2 * d, D->next_action, T, d, D->A, chunk_rows, D->part);
    hipLaunchKernelGGL(k_colsum_final, dim3(blocks(D->A * d, CS_COLS)), dim3(64 * CS_WAVES), 0, s, D->part, chunks, D->A * d,
                       c.G(D->act_emb));
    XTRL_LAUNCHED("train embed grad");
  }
  // every weight gradient is in before the caller's optimiser step
  if ((rc = splitk_flush(skq, cw.s))) return rc;
  if ((rc = bucket_done())) return rc;   // bucket L + 1: embeddings (and the flat buffer's tail)
  if ((rc = F.wait(F.mark()))) return rc;
  XTRL_REQUIRE(!F.failed, "train: side-stream event record failed");
  XTRL_REQUIRE(!F.on() || (size_t)F.next == side_events_needed(D->L) - (wpin_on_main ? 1 : 0),
               "train: side events %d != %d", F.next, (int)side_events_needed(D->L) - (wpin_on_main ? 1 : 0));
  return XTRL_OK;
}

// ============================================================================================
// Packed learn step (XtrlTrainDesc.packed): the minibatch without its padding.  With the per-token
// critic reduction every loss term is a masked mean over the valid tokens (xtrl.py:944-978) and a
// valid token sees only earlier valid keys (causal + key padding), so the padded tokens change
// neither the loss nor any gradient: the step runs on the Tv valid tokens, episode after episode.
namespace {
struct PackBufs {   // carved from pack_ws, 16-byte aligned segments of T rows each
  float *swr, *pa, *na, *raw, *values, *pred, *done, *d_raw, *d_values, *d_pred, *d_done;
  int64_t floats;
};
int64_t r4(int64_t x) { return (x + 3) & ~int64_t(3); }
PackBufs pack_bufs(float* base, int T, int S, int A, int n_out, int B) {
  PackBufs P{};
  int64_t at = 0;
  auto take = [&](int cols) {
    float* q = base ? base + at : nullptr;
    at += r4((int64_t)T * cols);
    return q;
  };
  const int a = std::max(A, 1);
  P.swr = take(S + 1); P.pa = take(a); P.na = take(a);
  P.raw = take(n_out); P.values = take(B); P.pred = take(2 * (S + 1)); P.done = take(1);
  P.d_raw = take(n_out); P.d_values = take(B); P.d_pred = take(2 * (S + 1)); P.d_done = take(1);
  P.floats = at;
  return P;
}
// the descriptor the row-wise step runs on: packed inputs / outputs, no compact heads (every row valid)
int packed_view(const XtrlTrainDesc* D, XtrlTrainDesc& P, PackBufs& B) {
  XTRL_REQUIRE(D->Tv > 0 && D->Tv <= D->b * D->n, "train (packed): Tv = %d outside (0, b n = %d]", D->Tv, D->b * D->n);
  XTRL_REQUIRE(D->b <= VR_MAXB && D->vrows && D->vinv && D->ep_off && D->pack_ws, "train (packed): row list buffers");
  XTRL_REQUIRE(D->Tv <= 65535, "train (packed): %d tokens exceed the prep kernels' grid", D->Tv);
  B = pack_bufs(D->pack_ws, D->Tv, D->S, D->A, D->n_out, D->B);
  XTRL_REQUIRE(B.floats <= D->pack_ws_floats, "train (packed): pack_ws %lld < %lld floats",
               (long long)D->pack_ws_floats, (long long)B.floats);
  P = *D;
  P.swr = B.swr;
  if (D->continuous) {
    P.prev_action_f = B.pa;
    P.next_action_f = B.na;
  } else {
    P.prev_action = reinterpret_cast<const int32_t*>(B.pa);
    P.next_action = reinterpret_cast<const int32_t*>(B.na);
  }
  P.raw = B.raw; P.values = B.values; P.pred = B.pred; P.done = B.done;
  P.d_raw = B.d_raw; P.d_values = B.d_values; P.d_pred = B.d_pred; P.d_done = B.d_done;
  P.Tv = 0;
  return XTRL_OK;
}
}  // namespace

int train_forward(const XtrlTrainDesc* D, hipStream_t s) {
  if (!D || !D->packed) return train_forward_rows(D, D ? D->b * D->n : 0, s);
  if (int rc = validate(D)) return rc;
  XtrlTrainDesc P;
  PackBufs B;
  if (int rc = packed_view(D, P, B)) return rc;
  const int T = D->b * D->n, Tv = D->Tv, S1 = D->S + 1, A = D->continuous ? D->A : 1;
  hipLaunchKernelGGL(k_valid_rows, dim3(1), dim3(1024), 0, s, D->lens, D->b, D->n, Tv, D->vrows, D->vinv, D->ep_off);
  gather_rows(D->swr, S1, D->vrows, Tv, S1, B.swr, S1, s);
  // (discrete actions: int32 moved as 4-byte words)
  gather_rows(D->continuous ? D->prev_action_f : reinterpret_cast<const float*>(D->prev_action), A, D->vrows, Tv, A,
              B.pa, A, s);
  gather_rows(D->continuous ? D->next_action_f : reinterpret_cast<const float*>(D->next_action), A, D->vrows, Tv, A,
              B.na, A, s);
  XTRL_LAUNCHED("train packed gather");
  if (int rc = train_forward_rows(&P, Tv, s)) return rc;
  // the heads' outputs back to the minibatch's [b][n] layout for the loss kernels (zeros on the padding)
  scatter_rows(B.raw, D->n_out, D->vinv, T, D->n_out, D->raw, D->n_out, s);
  scatter_rows(B.values, D->B, D->vinv, T, D->B, D->values, D->B, s);
  scatter_rows(B.pred, 2 * S1, D->vinv, T, 2 * S1, D->pred, 2 * S1, s);
  scatter_rows(B.done, 1, D->vinv, T, 1, D->done, 1, s);
  XTRL_LAUNCHED("train packed scatter");
  return XTRL_OK;
}

int train_backward(const XtrlTrainDesc* D, hipStream_t s) {
  if (!D || !D->packed) return train_backward_rows(D, D ? D->b * D->n : 0, s);
  if (int rc = validate(D)) return rc;
  XTRL_REQUIRE(D->d_raw && D->d_values && D->d_pred && D->d_done, "train: missing loss gradients");
  XtrlTrainDesc P;
  PackBufs B;
  if (int rc = packed_view(D, P, B)) return rc;
  const int Tv = D->Tv, S1 = D->S + 1;
  gather_rows(D->d_raw, D->n_out, D->vrows, Tv, D->n_out, B.d_raw, D->n_out, s);
  gather_rows(D->d_values, D->B, D->vrows, Tv, D->B, B.d_values, D->B, s);
  gather_rows(D->d_pred, 2 * S1, D->vrows, Tv, 2 * S1, B.d_pred, 2 * S1, s);
  gather_rows(D->d_done, 1, D->vrows, Tv, 1, B.d_done, 1, s);
  XTRL_LAUNCHED("train packed gradient gather");
  return train_backward_rows(&P, Tv, s);
}

// ============================================================================================
// Fractal policy body learn step (include/xtrl_hip.h XtrlFractalTrainDesc; the reference-mode
// autograd forward it replaces: xtrl_amd/fractal.py FractalPolicyActorCritic.forward_train)
namespace {
int validate_fractal(const XtrlTrainDesc* D, const XtrlFractalTrainDesc* F) {
  XTRL_REQUIRE(D && F && F->level && D->flat && D->grad, "fractal train: null descriptor / levels / parameters");
  XTRL_REQUIRE(F->levels > 0 && D->b > 0 && D->n > 0 && D->d > 0 && D->H > 0 && D->dh > 0 && D->ff > 0,
               "fractal train: bad sizes");
  XTRL_REQUIRE(D->d % 4 == 0 && D->d <= 256 && (D->H * D->dh) % 4 == 0 && D->ff % 4 == 0,
               "fractal train: needs d %% 4 == 0, d <= 256, H dh %% 4 == 0, ff %% 4 == 0 (d = %d)", D->d);
  XTRL_REQUIRE(D->in_dim == D->d * (D->evolutionary ? 3 : 2), "fractal train: in_dim mismatch");
  XTRL_REQUIRE(D->ld_ff == 0 || (D->ld_ff >= D->ff && D->ld_ff % 4 == 0), "fractal train: ld_ff %d (ff %d)", D->ld_ff,
               D->ff);
  XTRL_REQUIRE(!D->evolutionary || (D->latent && D->lat_e), "fractal train: evolutionary needs latent buffers");
  XTRL_REQUIRE(D->continuous ? D->next_action_f != nullptr : D->next_action != nullptr,
               "fractal train: missing next actions");
  XTRL_REQUIRE(D->continuous || D->A <= EMB_MAXA, "fractal train: %d discrete actions > %d unsupported", D->A, EMB_MAXA);
  XTRL_REQUIRE(D->w_pin >= 0 && F->b_in >= 0 && F->g_init >= 0 && F->w_gu >= 0 && F->w_fa0 >= 0 && F->w_fa2 >= 0,
               "fractal train: missing encoder parameters");
  XTRL_REQUIRE(F->scale_embeds && F->le && F->bias0 && F->cat && F->hfa, "fractal train: missing buffers");
  for (int l = 0; l < F->levels; ++l) {
    const XtrlFractalTrainLevel& V = F->level[l];
    XTRL_REQUIRE(V.w_qkv >= 0 && V.w_out >= 0 && V.w_gv >= 0 && V.w_go >= 0 && V.w_ff1 >= 0 && V.w_ff2 >= 0 &&
                     V.w_proj >= 0 && V.ln1_w >= 0 && V.ln2_w >= 0 && V.ln3_w >= 0 && V.level_embed >= 0,
                 "fractal train: level %d misses parameters", l);
    XTRL_REQUIRE(V.xin && V.qkv && V.o && V.lse && V.s1 && V.x1 && V.st1 && V.g && V.gv && V.s2 && V.x2 && V.st2 &&
                     V.h && V.u && V.s3 && V.x3 && V.st3 && V.mean,
                 "fractal train: level %d misses activation buffers", l);
  }
  return XTRL_OK;
}

// x_out = A W^T (+ bias) + R; y1 = nn.LayerNorm(x_out) (weight, bias); y2 = y1 + b2 (optional): one launch
int linear_res_ln_affine(const Ctx& c, const float* A, int lda, const float* W, int K, const float* bias,
                         const float* R, float* x_out, const float* gamma, const float* beta, float* y1, float* st,
                         float* y2 = nullptr, const float* b2 = nullptr) {
  const int d = c.D->d;
  GemmArgs g;
  g.A = A; g.lda = lda; g.B = W; g.ldb = K; g.bias = bias; g.C = x_out; g.ldc = d; g.M = c.T; g.N = d; g.K = K;
  g.R = R; g.ldr = d; g.ln_g = gamma; g.ln_b = beta; g.ln_b2 = b2; g.ln_y1 = y1; g.ln_ld1 = d; g.ln_y2 = y2;
  g.ln_ld2 = d; g.ln_stats = st;
  return gemm_run(g, 0, 0, EPI_RES_LN, c.s);
}

// C = A W^T + bias + R with R's own leading dimension
int linear_fwd_res(const Ctx& c, const float* A, int lda, const float* W, const float* bias, const float* R, int ldr,
                   float* C, int ldc, int N, int K) {
  GemmArgs g;
  g.A = A; g.lda = lda; g.B = W; g.ldb = K; g.bias = bias; g.C = C; g.ldc = ldc; g.M = c.T; g.N = N; g.K = K;
  g.R = R; g.ldr = ldr;
  return gemm_run(g, 0, 0, EPI_NONE, c.s);
}

// dX = dY W + R (R: a residual-path gradient, may alias dX)
int dgrad_res(const Ctx& c, const float* dY, int ldy, const float* W, int N, int K, const float* R, int ldr, float* dX,
              int ldx) {
  GemmArgs g;
  g.A = dY; g.lda = ldy; g.B = W; g.ldb = K; g.C = dX; g.ldc = ldx; g.M = c.T; g.N = K; g.K = N;
  g.R = R; g.ldr = ldr;
  return gemm_run(g, 0, 1, EPI_NONE, c.s);
}

// dx = dY W + gpre -> ds_a = norm2 backward(dx) and ds_b = norm1 backward(ds_a), one launch; the four
// partial rows of a row tile side by side [d gamma1 | d beta1 | d gamma2 | d beta2] -> one column sum
// into the adjacent norm1.weight | norm1.bias | norm2.weight | norm2.bias gradients
int dgrad_post_ln2(const Ctx& c, const float* dY, int ldy, const float* W, const float* gpre,
                   const XtrlFractalTrainLevel& V, float* ds_a, float* ds_b) {
  const int d = c.D->d, K = c.D->ff, nb = (c.T + gemm_ln_rows(d) - 1) / gemm_ln_rows(d);
  XTRL_REQUIRE(V.ln1_b == V.ln1_w + d && V.ln2_w == V.ln1_w + 2 * d && V.ln2_b == V.ln1_w + 3 * d,
               "fractal train: norm1 / norm2 parameters must be adjacent in the flat buffer");
  XTRL_REQUIRE((int64_t)nb * 4 * d <= c.D->part_floats, "fractal train: partial-sum workspace too small");
  float* P = c.D->part;
  GemmArgs g;
  g.A = dY; g.lda = ldy; g.B = W; g.ldb = d; g.C = ds_a; g.ldc = d; g.M = c.T; g.N = d; g.K = K;
  g.ln_g = c.P(V.ln2_w); g.ln_x = V.s2; g.ln_stats = V.st2; g.ln_gpre = gpre;
  g.ln_part = P + 2 * d; g.ln_part_b = P + 3 * d; g.ln_pstride = 4 * d;
  g.ln2_g = c.P(V.ln1_w); g.ln2_x = V.s1; g.ln2_stats = V.st1; g.ln2_out = ds_b; g.ln2_part = P;
  g.ln2_part_b = P + d;
  if (int rc = gemm_run(g, 0, 1, EPI_LN_BWD2, c.s)) return rc;
  hipLaunchKernelGGL(k_colsum_final, dim3(blocks(4 * d, CS_COLS)), dim3(64 * CS_WAVES), 0, c.s, P, nb, 4 * d,
                     c.G(V.ln1_w));
  XTRL_LAUNCHED("fractal dgrad_post_ln2");
  return XTRL_OK;
}

bool ln_fusable_fractal(const XtrlTrainDesc* D) {
  static const bool on = [] {
    const char* e = getenv("XTRL_FUSED_LN");
    return !(e && atoi(e) == 0);
  }();
  return on && D->d % 4 == 0 && D->d <= 256 && D->ff % 4 == 0;
}

AttnProblem fractal_attn(const Ctx& c, int level) {
  const XtrlTrainDesc* D = c.D;
  const int I = D->H * D->dh;
  AttnProblem p{};
  p.b = D->b; p.H = D->H; p.n = D->n; p.dh = D->dh; p.lens = D->lens; p.scale = D->attn_scale;
  p.dropout = D->dropout; p.seed = D->seed; p.offset = D->attn_offset; p.sub = (uint32_t)level;
  p.in = attn_layout_tokens(D->n, 3 * I, D->dh);
  p.out = attn_layout_tokens(D->n, I, D->dh);
  p.grad = attn_layout_tokens(D->n, 3 * I, D->dh);
  p.gate = p.grad;
  p.dq_part = D->dq_part;
  p.dq_part_floats = D->dq_part_floats;
  return p;
}

int causal_mean(const Ctx& c, const float* src, int lds, const float* add, int ldadd, float* dst, int ldd, bool rev) {
  const XtrlTrainDesc* D = c.D;
  const dim3 g(D->b, (D->d + 63) / 64), bl(64 * CM_G);
  if (rev) hipLaunchKernelGGL(k_causal_mean<1>, g, bl, 0, c.s, src, lds, add, ldadd, dst, ldd, D->n, D->d);
  else hipLaunchKernelGGL(k_causal_mean<0>, g, bl, 0, c.s, src, lds, add, ldadd, dst, ldd, D->n, D->d);
  XTRL_LAUNCHED("fractal causal_mean");
  return XTRL_OK;
}

int rows_axpb(const Ctx& c, const float* a, int lda, float alpha, const float* b, int ldb, float* dst, int ldd, int rows,
              int cols) {
  hipLaunchKernelGGL(k_rows_axpb, dim3(blocks((int64_t)rows * cols, 256)), dim3(256), 0, c.s, a, lda, alpha, b, ldb, dst,
                     ldd, rows, cols);
  XTRL_LAUNCHED("fractal rows_axpb");
  return XTRL_OK;
}
}  // namespace

int fractal_train_forward(const XtrlTrainDesc* D, const XtrlFractalTrainDesc* F, hipStream_t s) {
  if (int rc = validate_fractal(D, F)) return rc;
  const Ctx c{D, s, D->b * D->n};
  const int T = c.T, d = D->d, I = D->H * D->dh, ff = D->ff, lf = ld_ff(D), Lv = F->levels, S = D->S,
            ldcat = (Lv + 1) * d;
  int rc;
  // level embeddings le[l] = level_embeds[l] + scale_embeds[l] (level_embeds: one [levels][d]
  // parameter, level 0's offset its base) and the level-0 input bias b_in + le[0]
  hipLaunchKernelGGL(k_vec_add, dim3(blocks(Lv * d, 256)), dim3(256), 0, s, c.P(F->level[0].level_embed),
                     F->scale_embeds, F->le, Lv * d);
  hipLaunchKernelGGL(k_vec_add, dim3(blocks(d, 256)), dim3(256), 0, s, c.P(F->b_in), F->le, F->bias0, d);
  XTRL_LAUNCHED("fractal embeds");
  // x_in,0 = input_embed(state) + le[0];  g_0 = global_state_init on every row
  if ((rc = linear_fwd(c, D->swr, S + 1, c.P(D->w_pin), F->bias0, F->level[0].xin, d, T, d, S, EPI_NONE))) return rc;
  if ((rc = rows_axpb(c, c.P(F->g_init), 0, 1.f, nullptr, 0, F->level[0].g, d, T, d))) return rc;
  // heads' inputs besides the features: to_state_embed(state) -> ac_in[:, d:2d], the gene embedding
  // broadcast -> ac_in[:, 2d:], the next action's embedding -> ewa[:, d:]
  if ((rc = linear_fwd(c, D->swr, S + 1, c.P(D->w_se), c.P(D->b_se), D->ac_in + d, D->in_dim, T, d, S, EPI_NONE)))
    return rc;
  if (D->evolutionary) {
    hipLaunchKernelGGL(k_latent_embed, dim3(blocks(D->b * d, 256)), dim3(256), 0, s, D->latent, c.P(D->w_lat),
                       c.P(D->b_lat), D->lat_e, D->b, D->G, d);
    hipLaunchKernelGGL(k_rows_bcast_ep, dim3(blocks((int64_t)T * d, 256)), dim3(256), 0, s, D->lat_e, D->ac_in + 2 * d,
                       D->in_dim, T, D->n, d);
  }
  if (D->continuous) {
    if ((rc = linear_fwd(c, D->next_action_f, D->A, c.P(D->act_emb), c.P(D->act_emb_b), D->ewa + d, 2 * d, T, d, D->A,
                         EPI_NONE)))
      return rc;
  } else {
    hipLaunchKernelGGL(k_action_rows, dim3(blocks((int64_t)T * d, 256)), dim3(256), 0, s, D->next_action,
                       c.P(D->act_emb), D->A, D->ewa + d, 2 * d, T, d);
  }
  XTRL_LAUNCHED("fractal inputs");
  for (int l = 0; l < Lv; ++l) {
    const XtrlFractalTrainLevel& V = F->level[l];
    // self-attention: q | k | v (adjacent weights, one GEMM), causal flash attention with dropout
    if ((rc = linear_fwd(c, V.xin, d, c.P(V.w_qkv), nullptr, V.qkv, 3 * I, T, 3 * I, d, EPI_NONE))) return rc;
    const AttnProblem ap = fractal_attn(c, l);
    if ((rc = attn_fwd_ex(ap, V.qkv, V.qkv + I, V.qkv + 2 * I, V.o, V.lse, nullptr, nullptr, s))) return rc;
    // s1 = x_in + o W_out^T, x1 = norm1(s1)
    if ((rc = linear_res_ln_affine(c, V.o, I, c.P(V.w_out), I, nullptr, V.xin, V.s1, c.P(V.ln1_w), c.P(V.ln1_b), V.x1,
                                   V.st1)))
      return rc;
    // cross-attention to the one-token global state (softmax over one key == 1): s2 = x1 + (g W_gv^T) W_go^T
    if ((rc = linear_fwd(c, V.g, d, c.P(V.w_gv), nullptr, V.gv, I, T, I, d, EPI_NONE))) return rc;
    if ((rc = linear_res_ln_affine(c, V.gv, I, c.P(V.w_go), I, nullptr, V.x1, V.s2, c.P(V.ln2_w), c.P(V.ln2_b), V.x2,
                                   V.st2)))
      return rc;
    // feed-forward: h = drop(gelu(x2 W1^T + b1)); s3 = x2 + h W2^T + b2, x3 = norm3(s3) (and the next
    // level's input x3 + le[l + 1] from the same epilogue)
    if ((rc = linear_fwd(c, V.x2, d, c.P(V.w_ff1), c.P(V.b_ff1), V.h, lf, T, ff, d, EPI_GELU_DROP, nullptr, V.u, lf,
                         1 << 30, 0, D->ff_offset, (uint32_t)l)))
      return rc;
    const bool last = l + 1 == Lv;
    if ((rc = linear_res_ln_affine(c, V.h, lf, c.P(V.w_ff2), ff, c.P(V.b_ff2), V.x2, V.s3, c.P(V.ln3_w), c.P(V.ln3_b),
                                   V.x3, V.st3, last ? nullptr : F->level[l + 1].xin, last ? nullptr : F->le + (l + 1) * d)))
      return rc;
    // causal running mean; level projection into cat[:, l d:]; g <- g + mean W_gu^T + b_gu
    if ((rc = causal_mean(c, V.x3, d, nullptr, 0, V.mean, d, false))) return rc;
    if ((rc = linear_fwd(c, V.mean, d, c.P(V.w_proj), c.P(V.b_proj), F->cat + l * d, ldcat, T, d, d, EPI_NONE))) return rc;
    if ((rc = linear_fwd_res(c, V.mean, d, c.P(F->w_gu), c.P(F->b_gu), V.g, d, last ? F->cat + Lv * d : F->level[l + 1].g,
                             last ? ldcat : d, d, d)))
      return rc;
  }
  // features = final_aggregation(cat) -> ac_in[:, :d] and ewa[:, :d]
  if ((rc = linear_fwd(c, F->cat, ldcat, c.P(F->w_fa0), c.P(F->b_fa0), F->hfa, 2 * d, T, 2 * d, ldcat, EPI_RELU))) return rc;
  if ((rc = linear_fwd(c, F->hfa, 2 * d, c.P(F->w_fa2), c.P(F->b_fa2), D->ac_in, D->in_dim, T, d, 2 * d, EPI_NONE)))
    return rc;
  if ((rc = rows_axpb(c, D->ac_in, D->in_dim, 1.f, nullptr, 0, D->ewa, 2 * d, T, d))) return rc;
  if ((rc = heads_forward(c))) return rc;
  XTRL_LAUNCHED("fractal train forward");
  return XTRL_OK;
}

// events one fractal backward takes: forks — heads 4, action embedding 1, aggregation 1, 7 per level,
// input embedding 1 — and the final join's mark
constexpr size_t fractal_events_needed(int Lv) { return 7 * (size_t)Lv + 8; }

int fractal_train_backward(const XtrlTrainDesc* D, const XtrlFractalTrainDesc* F, hipStream_t s) {
  if (int rc = validate_fractal(D, F)) return rc;
  XTRL_REQUIRE(D->d_raw && D->d_values && D->d_pred && D->d_done, "fractal train: missing loss gradients");
  XTRL_REQUIRE(F->dxa && F->dxb && F->ds && F->dmean && F->dga && F->dgv && F->dz && F->dqkv && F->dob && F->dcat &&
                   F->dhfa,
               "fractal train: missing backward scratch");
  const Ctx c{D, s, D->b * D->n};
  const int T = c.T, d = D->d, I = D->H * D->dh, ff = D->ff, lf = ld_ff(D), Lv = F->levels, S = D->S,
            ldcat = (Lv + 1) * d;
  const int64_t Td = (int64_t)T * d;
  int rc;
  SideStream& side = side_stream();
  const bool two = side.ok && side.ensure(fractal_events_needed(Lv));
  Fork Fk{s, side.s, two ? &side : nullptr};
  static const bool defer = [] {
    const char* e = getenv("XTRL_SPLITK_DEFER");
    return !(e && atoi(e) == 0);
  }();
  SplitKQueue skq;
  const Ctx cw{D, two ? side.s : s, T, defer ? &skq : nullptr};
  // data-parallel gradient buckets (FractalPolicyActorCritic.flat_buckets_names): [heads, action
  // embedding, final aggregation], one per level (last to first), [the rest]; each flushes its
  // deferred split-K reductions and records an event on both streams once its gradients are final
  int bucket = 0;
  auto bucket_done = [&]() -> int {
    if (!D->grad_events) return XTRL_OK;
    if (int rc = splitk_flush(skq, cw.s)) return rc;
    if (hipEventRecord((hipEvent_t)D->grad_events[2 * bucket], s) != hipSuccess ||
        hipEventRecord((hipEvent_t)D->grad_events[2 * bucket + 1], cw.s) != hipSuccess) {
      set_error("fractal train: gradient bucket event record failed");
      return XTRL_E_HIP;
    }
    ++bucket;
    return XTRL_OK;
  };
  if ((rc = heads_backward(c, cw, Fk))) return rc;
  // d features = frac * dac[:, :d] + dewa[:, :d]  (frac_gradient: the actor / critic share scaled)
  // every backward scratch plane a side-stream weight gradient reads is written once per backward
  // (per-level planes): the main stream never waits for the side stream before the final join
  float* dfeat = F->ds + 3 * (int64_t)Lv * Td;   // after the levels' [3][T][d] planes
  if ((rc = rows_axpb(c, D->dac, D->in_dim, D->frac_head_grad, D->dewa, 2 * d, dfeat, d, T, d))) return rc;
  // next-action embedding
  if (D->continuous) {
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, D->dewa + d, 2 * d, D->next_action_f, D->A, c.G(D->act_emb), T, d, D->A, c.G(D->act_emb_b))))
      return rc;
  } else {
    int chunks = (int)std::min<int64_t>(std::min(1024, std::max(1, T / 16)),
                                        std::max<int64_t>(1, D->part_floats / ((int64_t)D->A * d)));
    const int chunk_rows = (T + chunks - 1) / chunks;
    chunks = (T + chunk_rows - 1) / chunk_rows;
    XTRL_REQUIRE((int64_t)chunks * D->A * d <= D->part_floats, "fractal train: partial-sum workspace too small");
    const dim3 eg(blocks(d, 256), chunks);
    if (D->A <= 4)
      hipLaunchKernelGGL(k_embed_grad_part<4>, eg, dim3(256), 0, s, nullptr, 0, nullptr, D->dewa + d, 2 * d,
                         D->next_action, T, d, D->A, chunk_rows, D->part);
    else if (D->A <= 8)
      hipLaunchKernelGGL(k_embed_grad_part<8>, eg, dim3(256), 0, s, nullptr, 0, nullptr, D->dewa + d, 2 * d,
                         D->next_action, T, d, D->A, chunk_rows, D->part);
    else
      hipLaunchKernelGGL(k_embed_grad_part<EMB_MAXA>, eg, dim3(256), 0, s, nullptr, 0, nullptr, D->dewa + d, 2 * d,
                         D->next_action, T, d, D->A, chunk_rows, D->part);
    hipLaunchKernelGGL(k_colsum_final, dim3(blocks(D->A * d, CS_COLS)), dim3(64 * CS_WAVES), 0, s, D->part, chunks,
                       D->A * d, c.G(D->act_emb));
    XTRL_LAUNCHED("fractal action embed grad");
    if ((rc = Fk.fork())) return rc;   // (keeps the event count independent of the action kind)
  }
  // final aggregation: feat = hfa W_fa2^T + b; hfa = ReLU(cat W_fa0^T + b)
  if ((rc = wgrad(cw, dfeat, d, F->hfa, 2 * d, c.G(F->w_fa2), T, d, 2 * d, c.G(F->b_fa2)))) return rc;
  if ((rc = linear_dgrad(c, dfeat, d, c.P(F->w_fa2), F->dhfa, 2 * d, T, d, 2 * d, EPI_MASK_POS, F->hfa, 2 * d))) return rc;
  if ((rc = Fk.fork())) return rc;
  if ((rc = wgrad(cw, F->dhfa, 2 * d, F->cat, ldcat, c.G(F->w_fa0), T, 2 * d, ldcat, c.G(F->b_fa0)))) return rc;
  if ((rc = linear_dgrad(c, F->dhfa, 2 * d, c.P(F->w_fa0), F->dcat, ldcat, T, 2 * d, ldcat, EPI_NONE))) return rc;
  if ((rc = bucket_done())) return rc;   // bucket 0: heads, action embedding, final aggregation
  // levels, last to first.  dgn: gradient of g_{l+1} (the final g: cat's last d columns); dxn:
  // gradient of x3_l from level l + 1's input (none for the last level).
  // the chained post-norm LayerNorm backward epilogue (XTRL_FUSED_LN=0: separate launches)
  const bool post2 = ln_fusable_fractal(D);
  const float* dgn = F->dcat + Lv * d;
  int lddgn = ldcat;
  const float* dxn = nullptr;
  for (int l = Lv - 1; l >= 0; --l) {
    const XtrlFractalTrainLevel& V = F->level[l];
    float* ds1 = F->ds + 3 * (int64_t)l * Td;   // this level's planes
    float* ds2 = ds1 + Td;
    float* ds3 = ds1 + 2 * Td;
    float* dz = F->dz + (int64_t)l * T * lf;
    float* dgv = F->dgv + (int64_t)l * T * I;
    float* dqkv = F->dqkv + (int64_t)l * T * 3 * I;
    float* dgc = F->dga + (int64_t)l * Td;
    // g_{l+1} = g_l + mean W_gu^T + b_gu;  cat[:, l d:] = mean W_p^T + b_p
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, dgn, lddgn, V.mean, d, c.G(F->w_gu), T, d, d, c.G(F->b_gu)))) return rc;
    if ((rc = wgrad(cw, F->dcat + l * d, ldcat, V.mean, d, c.G(V.w_proj), T, d, d, c.G(V.b_proj)))) return rc;
    if ((rc = linear_dgrad(c, dgn, lddgn, c.P(F->w_gu), F->dmean, d, T, d, d, EPI_NONE))) return rc;
    if ((rc = dgrad_res(c, F->dcat + l * d, ldcat, c.P(V.w_proj), d, d, F->dmean, d, F->dmean, d))) return rc;
    // mean = causal running mean of x3: dx3 = dxn + reverse scan of dmean / (t + 1)
    if ((rc = causal_mean(c, F->dmean, d, dxn, d, F->dxa, d, true))) return rc;
    // norm3 backward -> ds3 (d gamma, d beta)
    if ((rc = ln_bwd(c, F->dxa, d, 1.f, nullptr, 0, V.s3, V.st3, c.P(V.ln3_w), nullptr, ds3, c.G(V.ln3_w),
                     c.G(V.ln3_b))))
      return rc;
    // feed-forward: s3 = x2 + h W2^T + b2
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, ds3, d, V.h, lf, c.G(V.w_ff2), T, d, ff, c.G(V.b_ff2)))) return rc;
    if ((rc = linear_dgrad(c, ds3, d, c.P(V.w_ff2), dz, lf, T, d, ff, EPI_MUL_AUX, V.u, lf))) return rc;
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, dz, lf, V.x2, d, c.G(V.w_ff1), T, ff, d, c.G(V.b_ff1)))) return rc;
    // dx2 = ds3 + dz W1; norm2 backward -> ds2; norm1 backward (x1's whole gradient is ds2, the
    // residual path of s2) -> ds1: one launch (the LayerNorm backward of both in the epilogue)
    if (post2) {
      if ((rc = dgrad_post_ln2(c, dz, lf, c.P(V.w_ff1), ds3, V, ds2, ds1))) return rc;
    } else {
      if ((rc = dgrad_res(c, dz, lf, c.P(V.w_ff1), ff, d, ds3, d, F->dxb, d))) return rc;
      if ((rc = ln_bwd(c, F->dxb, d, 1.f, nullptr, 0, V.s2, V.st2, c.P(V.ln2_w), nullptr, ds2, c.G(V.ln2_w),
                       c.G(V.ln2_b))))
        return rc;
      if ((rc = ln_bwd(c, ds2, d, 1.f, nullptr, 0, V.s1, V.st1, c.P(V.ln1_w), nullptr, ds1, c.G(V.ln1_w),
                       c.G(V.ln1_b))))
        return rc;
    }
    // cross-attention: s2 = x1 + gv W_go^T, gv = g W_gv^T
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, ds2, d, V.gv, I, c.G(V.w_go), T, d, I))) return rc;
    if ((rc = linear_dgrad(c, ds2, d, c.P(V.w_go), dgv, I, T, d, I, EPI_NONE))) return rc;
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, dgv, I, V.g, d, c.G(V.w_gv), T, I, d))) return rc;
    // dg_l = dg_{l+1} + dgv W_gv
    if ((rc = dgrad_res(c, dgv, I, c.P(V.w_gv), I, d, dgn, lddgn, dgc, d))) return rc;
    // self-attention: s1 = x_in + o W_out^T
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, ds1, d, V.o, I, c.G(V.w_out), T, d, I))) return rc;
    if ((rc = linear_dgrad(c, ds1, d, c.P(V.w_out), F->dob, I, T, d, I, EPI_NONE))) return rc;
    const AttnProblem ap = fractal_attn(c, l);
    if ((rc = attn_bwd_ex(ap, V.qkv, V.qkv + I, V.qkv + 2 * I, V.o, V.lse, F->dob, dqkv, dqkv + I, dqkv + 2 * I,
                          D->delta, s)))
      return rc;
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, dqkv, 3 * I, V.xin, d, c.G(V.w_qkv), T, 3 * I, d))) return rc;
    // d x_in = ds1 + dqkv W_qkv; the level embedding's gradient is its column sum
    if ((rc = dgrad_res(c, dqkv, 3 * I, c.P(V.w_qkv), 3 * I, d, ds1, d, F->dxa, d))) return rc;
    if ((rc = colsum(c, F->dxa, d, T, d, c.G(V.level_embed)))) return rc;
    dxn = F->dxa;
    dgn = dgc;
    lddgn = d;
    if ((rc = bucket_done())) return rc;   // bucket Lv - l: level l's block and projection
  }
  // input embedding (x_in,0 = state W_in^T + b_in + le[0]) and global_state_init (g_0 on every row).
  // As the decoder step's backward: the queued split-K sums start on the side stream here and the
  // small input-projection gradient runs on the main stream behind them in the workspace
  static const bool wpin_main = [] {
    const char* e = getenv("XTRL_WPIN_MAIN");
    return !(e && atoi(e) == 0);
  }();
  const bool wpin_on_main = wpin_main && !D->grad_events && skq.used < D->ws_floats;
  if (wpin_on_main) {
    const int64_t used0 = skq.used;
    if ((rc = splitk_flush(skq, cw.s))) return rc;
    if ((rc = gemm_wgrad(F->dxa, d, D->swr, S + 1, c.G(D->w_pin), S, T, d, S, 1.f, D->ws + used0,
                         D->ws_floats - used0, c.s, c.G(F->b_in), 0, nullptr, nullptr)))
      return rc;
  } else {
    if ((rc = Fk.fork())) return rc;
    if ((rc = wgrad(cw, F->dxa, d, D->swr, S + 1, c.G(D->w_pin), T, d, S, c.G(F->b_in)))) return rc;
  }
  if ((rc = colsum(c, dgn, lddgn, T, d, c.G(F->g_init)))) return rc;
  if ((rc = splitk_flush(skq, cw.s))) return rc;
  if ((rc = bucket_done())) return rc;   // bucket Lv + 1: embeddings, global state, level embeddings
  if ((rc = Fk.wait(Fk.mark()))) return rc;
  XTRL_REQUIRE(!Fk.failed, "fractal train: side-stream event record failed");
  XTRL_REQUIRE(!Fk.on() || (size_t)Fk.next == fractal_events_needed(Lv) - (wpin_on_main ? 1 : 0),
               "fractal train: side events %d != %d", Fk.next, (int)fractal_events_needed(Lv) - (wpin_on_main ? 1 : 0));
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_train_forward(const XtrlTrainDesc* desc, void* stream) {
  return xtrl::train_forward(desc, xtrl::as_stream(stream));
}

extern "C" int xtrl_train_backward(const XtrlTrainDesc* desc, void* stream) {
  return xtrl::train_backward(desc, xtrl::as_stream(stream));
}

extern "C" int xtrl_fractal_train_forward(const XtrlTrainDesc* base, const XtrlFractalTrainDesc* f, void* stream) {
  return xtrl::fractal_train_forward(base, f, xtrl::as_stream(stream));
}

extern "C" int xtrl_fractal_train_backward(const XtrlTrainDesc* base, const XtrlFractalTrainDesc* f, void* stream) {
  return xtrl::fractal_train_backward(base, f, xtrl::as_stream(stream));
}

extern "C" int64_t xtrl_train_part_floats(int T, int b, int d, int A) {
  if (T <= 0 || d <= 0) return 0;
  const int64_t ln = (int64_t)((T + xtrl::LN_ROWS - 1) / xtrl::LN_ROWS) * d;            // ln_bwd partials
  const int64_t cs = (int64_t)std::min(1024, std::max(1, T / 16)) * d;                  // colsum partials
  const int64_t lat = (int64_t)std::max(b, 1) * d;                                      // latent gradient
  const int64_t emb = (int64_t)std::max(A, 1) * d;                                      // >= 1 embedding chunk
  return std::max(std::max(ln, cs), std::max(lat, emb));
}

extern "C" int64_t xtrl_train_pack_floats(int T, int S, int A, int n_out, int B) {
  if (T <= 0) return 0;
  return xtrl::pack_bufs(nullptr, T, S, A, n_out, B).floats;
}

extern "C" int xtrl_linear_gelu_drop(const float* X, int ldx, const float* W, const float* bias, float* Y, int ldy,
                                     float* deriv, int ld_deriv, int M, int N, int K, float p, uint64_t seed,
                                     uint32_t offset, uint32_t layer, void* stream) {
  XTRL_REQUIRE(layer < (1u << 22), "linear_gelu_drop: layer %u out of range", layer);
  XTRL_REQUIRE(X && W && Y && deriv && M >= 0 && N > 0 && K > 0 && p >= 0.f && p < 1.f && ldx >= K && ldy >= N &&
                   ld_deriv >= N,
               "linear_gelu_drop: bad arguments");
  if (M == 0) return XTRL_OK;
  xtrl::GemmArgs g;
  g.A = X; g.lda = ldx; g.B = W; g.ldb = K; g.bias = bias; g.C = Y; g.ldc = ldy; g.M = M; g.N = N; g.K = K;
  g.aux_out = deriv; g.ld_aux_out = ld_deriv;
  g.seed = seed; g.drop_off = offset; g.drop_layer = layer;
  g.drop_thresh = xtrl::dropout_thresh(p);
  g.drop_thresh8 = xtrl::dropout_thresh8(p);
  g.inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  return xtrl::gemm_run(g, 0, 0, xtrl::EPI_GELU_DROP, xtrl::as_stream(stream));
}

extern "C" int xtrl_glu_drop_fwd(const float* u, int ldu, float* h, int ldh, int M, int ff, float p, uint64_t seed,
                                 uint32_t offset, uint32_t layer, void* stream) {
  XTRL_REQUIRE(layer < (1u << 22), "glu_drop_fwd: layer %u out of range", layer);
  XTRL_REQUIRE(u && h && M >= 0 && ff > 0 && ldu >= 2 * ff && ldh >= ff && p >= 0.f && p < 1.f,
               "glu_drop_fwd: bad arguments");
  return xtrl::glu_fwd(u, ldu, h, ldh, M, ff, p, seed, offset, layer, xtrl::as_stream(stream));
}

extern "C" int xtrl_glu_drop_bwd(const float* dh, int lddh, const float* u, int ldu, float* du, int lddu, int M, int ff,
                                 float p, uint64_t seed, uint32_t offset, uint32_t layer, void* stream) {
  XTRL_REQUIRE(layer < (1u << 22), "glu_drop_bwd: layer %u out of range", layer);
  XTRL_REQUIRE(dh && u && du && M >= 0 && ff > 0 && lddh >= ff && ldu >= 2 * ff && lddu >= 2 * ff && p >= 0.f && p < 1.f,
               "glu_drop_bwd: bad arguments");
  return xtrl::glu_bwd(dh, lddh, u, ldu, du, lddu, M, ff, p, seed, offset, layer, xtrl::as_stream(stream));
}

extern "C" int xtrl_ff_dropout_mask(uint8_t* mask, int M, int N, float p, uint64_t seed, uint32_t offset,
                                    uint32_t layer, void* stream) {
  XTRL_REQUIRE(layer < (1u << 22), "ff_dropout_mask: layer %u out of range", layer);
  XTRL_REQUIRE(mask && M >= 0 && N >= 0 && p >= 0.f && p < 1.f, "ff_dropout_mask: bad arguments");
  if ((int64_t)M * N == 0) return XTRL_OK;
  hipLaunchKernelGGL(xtrl::k_ff_mask, dim3((unsigned)(((int64_t)M * N + 255) / 256)), dim3(256), 0,
                     xtrl::as_stream(stream), mask, M, N, xtrl::dropout_thresh(p), xtrl::dropout_thresh8(p), seed, offset, layer);
  XTRL_LAUNCHED("ff_dropout_mask");
  return XTRL_OK;
}
