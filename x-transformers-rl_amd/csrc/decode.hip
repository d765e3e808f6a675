// Rollout: one policy timestep for E concurrent episodes, entirely on device.
//
// Replaces the batch-1, host-synchronised body of the reference rollout loop
// (x_transformers_rl.py:1250-1341) with a vectorised step:
//
//   k_embed        RSNorm eval of [state, prev_reward] (xtrl.py:1254-1259, 591), project_in +
//                  action embedding + reward embedding (xtrl.py:492-503), to_state_embed;
//                  writes the raw state into the trajectory (Memory.state, xtrl.py:1315)
//   per layer      LN -> [q|k|v|gate|mix] GEMM (gemm.hip)
//                  k_attn_decode: value-residual mix, rotary, KV append at t, softmax(q k^T) v
//                  over positions 0..t, value gate        (x-transformers Attention, cached)
//                  out-proj GEMM + residual, LN -> FF1 GELU GEMM, FF2 GEMM + residual
//   final LN       into ac_in[:, 0:d]; heads: [actor|critic] hidden GEMM (SiLU), logits GEMMs
//                  (critic logits straight into traj_values[:, t, :] of live envs)
//   k_sample       softmax -> Categorical -> inverse-CDF sample on Philox uniforms, log_prob
//                  (xtrl.py:1280-1289; torch Categorical(probs) semantics), then the synthetic
//                  LunarLander-shaped Sim step (philox.h): reward, termination, next state, alive
//                  mask, episode length, cumulative reward (xtrl.py:1297-1351)
//
// Layouts in HBM: activations are [E][·] row-major; KV caches [E][H][Tmax][dh] so one (env, head)
// streams a contiguous Tmax*dh block; trajectories [E][Tmax][·] so the learner reads whole
// episodes contiguously.
#include "kernels.h"
#include "philox.h"

namespace xtrl {

namespace {

constexpr float F32_EPS = 1.1920928955078125e-07f;

// ---------------------------------------------------------------------------------------------
// embeddings (one wave per env)
// ---------------------------------------------------------------------------------------------
// ln_gamma != NULL (d <= 256): the row is also layer-normalised into xn with the first layer's
// pre-norm gamma, in k_layernorm's order of operations (bit-identical; one launch less per step)
__global__ __launch_bounds__(256) void k_embed(const XtrlDecodeDesc D, int t, const float* ln_gamma) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= D.E) return;
  const int S = D.S, d = D.d;
  __shared__ float ns_sh[4][64];
  float* ns = ns_sh[threadIdx.x >> 6];
  const float* st = D.state + (int64_t)e * S;
  const bool alive = D.alive[e] != 0;
  // RSNorm eval on the packed [state, prev_reward] vector: (x - mean) / clamp(sqrt(var), eps)
  if (lane <= S) {
    const float xv = lane < S ? st[lane] : D.prev_reward[e];
    ns[lane] = (xv - D.rs_mean[lane]) / fmaxf(sqrtf(D.rs_var[lane]), D.rs_eps);
    if (lane < S && alive) D.traj_states[((int64_t)e * D.Tmax + t) * S + lane] = xv;
  }
  wave_sync();
  const float nr = ns[S];
  const int a = D.continuous ? 0 : D.prev_action[e];
  float xs[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c = lane, k = 0; c < d; c += 64, ++k) {
    float p = 0.f, se = 0.f;
    for (int s = 0; s < S; ++s) {
      p += ns[s] * D.w_pin[c * S + s];
      se += ns[s] * D.w_se[c * S + s];
    }
    if (D.b_pin) p += D.b_pin[c];
    float act;
    if (D.continuous) {
      float acc = 0.f;
      for (int i = 0; i < D.A; ++i) acc += D.prev_action_f[e * D.A + i] * D.act_emb[c * D.A + i];
      act = acc + D.act_emb_b[c];
    } else {
      act = a >= 0 ? D.act_emb[a * d + c] : 0.f;
    }
    const float rew = D.no_reward_cond ? 0.f : nr * D.reward_embed[c];
    const float xv = p + (act + rew);
    D.x[(int64_t)e * d + c] = xv;
    if (k < 4) xs[k] = xv;
    D.ac_in[(int64_t)e * D.in_dim + d + c] = se + D.b_se[c];
  }
  if (ln_gamma) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lane + 64 * k < d) s += xs[k];
    const float mean = wave_sum(s) / (float)d;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (lane + 64 * k < d) {
        const float dlt = xs[k] - mean;
        q += dlt * dlt;
      }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)d + 1e-5f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = lane + 64 * k;
      if (c < d) D.xn[(int64_t)e * d + c] = ((xs[k] - mean) * rstd) * ln_gamma[c];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// attention decode: one wave per (env, head), keys 0..t
// ---------------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(256) void k_attn_decode(const XtrlDecodeDesc D, const XtrlDecodeLayer Ly, int layer,
                                                     int t) {
  extern __shared__ float smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int idx = blockIdx.x * 4 + w;
  const int H = D.H, I = H * DH;
  const int e = idx / H, h = idx - e * H;
  const bool valid = e < D.E;
  float* sc = smem + w * (D.Tmax + 3 * DH);   // scores [Tmax] | q | k_new | v_new
  float* qs = sc + D.Tmax;
  float* ks = qs + DH;
  float* vs = ks + DH;
  const bool alive = valid && D.alive[e] != 0;
  if (!alive) return;   // wave-uniform
  const float* row = D.qkv + (int64_t)e * D.n_qkv;
  constexpr int G = 64 / DH;   // lane groups for the P.V product
  const int c = lane % DH, g = lane / DH;
  float q = row[h * DH + c], k = row[I + h * DH + c], v = row[2 * I + h * DH + c];
  // value residual (first layer stores its values; later layers lerp toward them)
  if (D.value_residual) {
    float* v1 = D.v1 + (int64_t)e * I + h * DH + c;
    if (layer == 0) {
      if (g == 0) *v1 = v;
    } else if (D.learned_mix) {
      const int mix_col = 3 * I + (D.gate_values ? I : 0) + h;
      const float mix = sigmoidf_(row[mix_col]);
      v = lerpf_(v, *v1, mix);
    }
  }
  // rotary (interleaved pairs on the first rot_dim channels); 'zero' mode = position 0 = identity
  if (D.rotary_abs && c < D.rot_dim) {
    const float f = (float)t * D.inv_freq[c >> 1];
    const float cs = cosf(f), sn = sinf(f);
    const float qp = __shfl_xor(q, 1, 64), kp = __shfl_xor(k, 1, 64);
    const float sgn = (c & 1) ? 1.f : -1.f;   // rotate_half: (-x2, x1)
    q = q * cs + (sgn * qp) * sn;
    k = k * cs + (sgn * kp) * sn;
  }
  const int64_t cache_base = ((int64_t)e * H + h) * D.Tmax * DH;
  if (g == 0) {
    qs[c] = q;
    ks[c] = k;
    vs[c] = v;
    Ly.k_cache[cache_base + (int64_t)t * DH + c] = k;
    Ly.v_cache[cache_base + (int64_t)t * DH + c] = v;
  }
  wave_sync();
  const float scale = 1.0f / sqrtf((float)DH);
  float qreg[DH];
#pragma unroll
  for (int i = 0; i < DH; ++i) qreg[i] = qs[i];
  const float* Kc = Ly.k_cache + cache_base;
  const float* Vc = Ly.v_cache + cache_base;
  float mx = -INFINITY;
#pragma unroll 2
  for (int j = lane; j <= t; j += 64) {
    float s = 0.f;
    if (j < t) {
      const float4* kr = reinterpret_cast<const float4*>(Kc + (int64_t)j * DH);
#pragma unroll
      for (int i = 0; i < DH / 4; ++i) {
        const float4 kv = kr[i];
        s += qreg[4 * i] * kv.x;
        s += qreg[4 * i + 1] * kv.y;
        s += qreg[4 * i + 2] * kv.z;
        s += qreg[4 * i + 3] * kv.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < DH; ++i) s += qreg[i] * ks[i];
    }
    s *= scale;
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j <= t; j += 64) {
    const float p = expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  wave_sync();
  float acc = 0.f;
  // eight V rows in flight per lane group (the loads are independent; only the adds chain).
  // (A one-key-per-lane P.V with a reduce-scatter butterfly measured slower: 14.9 vs 11.5 us.)
#pragma unroll 8
  for (int j = g; j <= t; j += G) {
    const float p = sc[j] / sum;
    const float vv = (j < t) ? Vc[(int64_t)j * DH + c] : vs[c];
    acc += p * vv;
  }
#pragma unroll
  for (int o = DH; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (g == 0) {
    float out = acc;
    if (D.gate_values) out *= sigmoidf_(row[3 * I + h * DH + c]);
    D.att[(int64_t)e * I + h * DH + c] = out;
  }
}

// ---------------------------------------------------------------------------------------------
// sampling (one thread per env)
// ---------------------------------------------------------------------------------------------
// sampling (xtrl.py:197-277) and, for the device Sim, its step (one thread per live env).  The
// value logits were written straight into the trajectory by the critic GEMM (masked to live envs).
__device__ __forceinline__ float reward_factor(int a) { return (float)(1.0 + 0.1 * (double)a); }

__device__ __forceinline__ void sim_step_env(const XtrlDecodeDesc& D, int e, int t, const XtrlRngState& R) {
  const uint32_t ep = (uint32_t)D.episode_of_slot[e];
  const float z = rng_normal(R.seed, R.update, ep, t, FIELD_REWARD, 0);
  const float reward = (D.sim_mode == 1 && !D.continuous) ? z * reward_factor(D.prev_action[e]) : z;
  bool term = false;
  if (D.sim_mode == 1 && D.hazard_log2 > 0)
    term = (rng_u32(R.seed, R.update, ep, t, FIELD_TERM, 0) & ((1u << D.hazard_log2) - 1u)) == 0u;
  D.traj_rewards[(int64_t)e * D.Tmax + t] = reward;
  D.traj_bounds[(int64_t)e * D.Tmax + t] = term ? 1 : 0;
  D.prev_reward[e] = reward;
  D.cum_reward[e] += (double)reward;
  D.lens[e] = t + 1;   // (the next state was written by the env's lanes in k_sample)
  if (term || t + 1 >= D.Tmax) D.alive[e] = 0;
}

// SAMPLE_L lanes per env (one wave holds whole envs): lane 0 samples the action and steps the Sim;
// the next state's S normals are spread over the env's lanes (they do not depend on the action)
constexpr int SAMPLE_L = 8;
__global__ void k_sample(const XtrlDecodeDesc D, int t) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = gid / SAMPLE_L, sub = gid % SAMPLE_L;
  if (e >= D.E || !D.alive[e]) return;   // (every lane of the env reads alive before lane 0 clears it)
  if (D.alive[e] == 2) {   // truncation-bootstrap step of a host env: its value logits are all it needed
    if (sub == 0) D.alive[e] = 0;
    return;
  }
  const XtrlRngState R = *D.rng;
  if (D.sim_mode >= 0) {
    const uint32_t ep = (uint32_t)D.episode_of_slot[e];
    for (int i = sub; i < D.S; i += SAMPLE_L)
      D.state[(int64_t)e * D.S + i] = rng_normal(R.seed, R.update, ep, t + 1, FIELD_STATE, i);
  }
  if (sub != 0) return;
  const uint32_t slot = D.slot_of_row ? (uint32_t)D.slot_of_row[e] : R.slot_offset + (uint32_t)e;
  const int A = D.A;
  const float* lg = D.logits + (int64_t)e * (D.continuous ? 2 * A : A);
  if (!D.continuous) {
    // softmax (xtrl.py:203), Categorical(probs) re-normalisation, inverse CDF on the supplied
    // uniform; probabilities recomputed on the fly (no per-thread array)
    float mx = -INFINITY;
    for (int i = 0; i < A; ++i) mx = fmaxf(mx, lg[i]);
    float s = 0.f;
    for (int i = 0; i < A; ++i) s += expf(lg[i] - mx);
    float s2 = 0.f;
    for (int i = 0; i < A; ++i) s2 += expf(lg[i] - mx) / s;
    const float u = rng_uniform(R.seed, R.update, slot, t, FIELD_SAMPLE, 0);
    int a = 0;
    float cdf = 0.f, pa = 0.f;
    for (int i = 0; i < A; ++i) {
      const float p = (expf(lg[i] - mx) / s) / s2;
      if (i < A - 1) {
        cdf += p;
        a += (u >= cdf) ? 1 : 0;
      }
    }
    for (int i = 0; i < A; ++i)
      if (i == a) pa = (expf(lg[i] - mx) / s) / s2;
    pa = fminf(fmaxf(pa, F32_EPS), 1.f - F32_EPS);
    D.traj_actions[(int64_t)e * D.Tmax + t] = a;
    D.traj_logp[(int64_t)e * D.Tmax + t] = logf(pa);
    D.prev_action[e] = a;
  } else {
    for (int i = 0; i < A; ++i) {
      const float mean = lg[2 * i], lv = lg[2 * i + 1];
      const float var = expf(tanhf(lv / 3.f) * 3.f);
      const float sd = sqrtf(fmaxf(var, 1e-5f));
      const float z = rng_normal(R.seed, R.update, slot, t, FIELD_SAMPLE, i);
      float s = mean + sd * z;
      if (D.squash) s = tanhf(s);
      float lp = -((s - mean) * (s - mean)) / (2.f * sd * sd) - logf(sd) - 0.91893853320467274f;
      if (D.squash) lp -= logf(fmaxf(1.f - s * s, 1e-20f));
      if (D.has_clamp) s = fminf(fmaxf(s, D.clamp_lo), D.clamp_hi);
      D.traj_actions_f[((int64_t)e * D.Tmax + t) * A + i] = s;
      D.traj_logp[((int64_t)e * D.Tmax + t) * A + i] = lp;
      D.prev_action_f[e * A + i] = s;
    }
  }
  if (D.sim_mode >= 0) sim_step_env(D, e, t, R);
}

// host env results of step t (xtrl.py:1297-1336): the memory stores is_boundary = terminated;
// done = terminated | truncated ends the episode; a truncated (not terminated) episode with
// `bootstrap` stays for one more decode step (alive = 2) whose critic logits land in the padding
// slot traj_values[e][t + 1] — the value of the next state the reference computes at :1323-1336.
__global__ void k_env_feedback(const XtrlDecodeDesc D, int t, const float* next_state, const float* reward,
                               const uint8_t* terminated, const uint8_t* truncated, int t_limit, int bootstrap) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D.E || D.alive[e] != 1) return;
  const bool term = terminated[e] != 0, trunc = truncated && truncated[e] != 0;
  D.traj_rewards[(int64_t)e * D.Tmax + t] = reward[e];
  D.traj_bounds[(int64_t)e * D.Tmax + t] = term ? 1 : 0;
  D.prev_reward[e] = reward[e];
  D.cum_reward[e] += (double)reward[e];
  D.lens[e] = t + 1;
  for (int i = 0; i < D.S; ++i) D.state[(int64_t)e * D.S + i] = next_state[(int64_t)e * D.S + i];
  if (term || t + 1 >= t_limit) D.alive[e] = 0;
  else if (trunc) D.alive[e] = (bootstrap && t + 1 < D.Tmax) ? 2 : 0;
}

__global__ void k_rollout_begin(const XtrlDecodeDesc D) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D.E) return;
  const XtrlRngState R = *D.rng;
  if (D.sim_mode >= 0) {
    const uint32_t ep = (uint32_t)D.episode_of_slot[e];
    for (int i = 0; i < D.S; ++i) D.state[(int64_t)e * D.S + i] = rng_normal(R.seed, R.update, ep, 0, FIELD_STATE, i);
  }
  D.prev_action[e] = -1;
  if (D.continuous)
    for (int i = 0; i < D.A; ++i) D.prev_action_f[e * D.A + i] = 0.f;
  D.prev_reward[e] = 0.f;
  D.alive[e] = 1;
  D.lens[e] = 0;
  D.cum_reward[e] = 0.0;
}

__global__ void k_sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update, const int32_t* ep_of_slot) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  for (int i = 0; i < S; ++i) state[(int64_t)e * S + i] = rng_normal(seed, update, (uint32_t)ep_of_slot[e], 0, FIELD_STATE, i);
}

int check_desc(const XtrlDecodeDesc* D) {
  XTRL_REQUIRE(D && D->layers, "decode: null descriptor");
  XTRL_REQUIRE(D->E > 0 && D->S > 0 && D->S < 64 && D->A > 0 && D->A <= 32, "decode: bad E/S/A (E=%d S=%d A=%d)",
               D->E, D->S, D->A);
  XTRL_REQUIRE(D->dh == 16 || D->dh == 32 || D->dh == 64, "decode: dim_head %d unsupported (16/32/64)", D->dh);
  XTRL_REQUIRE(D->H * D->dh <= 4096 && D->d > 0 && D->L > 0 && D->Tmax > 0, "decode: bad dims");
  XTRL_REQUIRE(D->in_dim == 2 * D->d + (D->evolutionary ? D->d : 0), "decode: in_dim mismatch");
  const int I = D->H * D->dh;
  XTRL_REQUIRE(D->n_qkv == 3 * I + (D->gate_values ? I : 0) + ((D->value_residual && D->learned_mix) ? D->H : 0),
               "decode: n_qkv mismatch");
  return XTRL_OK;
}

int launch_attn_decode(const XtrlDecodeDesc* D, int l, int t, hipStream_t s) {
  const int waves = D->E * D->H;
  const size_t lds = 4 * (size_t)(D->Tmax + 3 * D->dh) * sizeof(float);
  XTRL_REQUIRE(lds <= 160 * 1024, "attn_decode: Tmax %d too large for LDS", D->Tmax);
  dim3 grid((waves + 3) / 4);
  if (D->dh == 16)
    hipLaunchKernelGGL(k_attn_decode<16>, grid, dim3(256), lds, s, *D, D->layers[l], l, t);
  else if (D->dh == 32)
    hipLaunchKernelGGL(k_attn_decode<32>, grid, dim3(256), lds, s, *D, D->layers[l], l, t);
  else
    hipLaunchKernelGGL(k_attn_decode<64>, grid, dim3(256), lds, s, *D, D->layers[l], l, t);
  XTRL_LAUNCHED("attn_decode");
  return XTRL_OK;
}

}  // namespace

int decode_step(const XtrlDecodeDesc* D, int t, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  XTRL_REQUIRE(t >= 0 && t < D->Tmax, "decode: t=%d outside [0, %d)", t, D->Tmax);
  const int E = D->E, d = D->d, I = D->H * D->dh;
  const bool embed_ln = d <= 256;   // layer 0's pre-norm inside the embedding kernel
  hipLaunchKernelGGL(k_embed, dim3((E + 3) / 4), dim3(256), 0, s, *D, t,
                     embed_ln ? D->layers[0].ln_attn : (const float*)nullptr);
  XTRL_LAUNCHED("embed");
  for (int l = 0; l < D->L; ++l) {
    const XtrlDecodeLayer& Ly = D->layers[l];
    // pre-norm once per row (a LN prologue inside the GEMM would be recomputed by every column tile)
    int rc = (l == 0 && embed_ln) ? XTRL_OK : layernorm_f32(D->x, d, Ly.ln_attn, D->xn, d, E, d, s);
    if (rc) return rc;
    if ((rc = gemm_f32(D->xn, d, Ly.w_qkv, d, Ly.b_qkv, nullptr, nullptr, 0, D->qkv, D->n_qkv, nullptr, 0, E,
                       D->n_qkv, d, XTRL_ACT_NONE, s)))
      return rc;
    if (D->prof_events) (void)hipEventRecord((hipEvent_t)D->prof_events[2 * (t * D->L + l)], s);
    if ((rc = launch_attn_decode(D, l, t, s))) return rc;
    if (D->prof_events) (void)hipEventRecord((hipEvent_t)D->prof_events[2 * (t * D->L + l) + 1], s);
    if ((rc = gemm_f32(D->att, I, Ly.w_out, I, nullptr, nullptr, D->x, d, D->x, d, nullptr, 0, E, d, I,
                       XTRL_ACT_NONE, s)))
      return rc;
    if ((rc = layernorm_f32(D->x, d, Ly.ln_ff, D->xn, d, E, d, s))) return rc;
    if ((rc = gemm_f32(D->xn, d, Ly.w_ff1, d, Ly.b_ff1, nullptr, nullptr, 0, D->hff, D->ff, nullptr, 0, E, D->ff, d,
                       XTRL_ACT_GELU, s)))
      return rc;
    if ((rc = gemm_f32(D->hff, D->ff, Ly.w_ff2, D->ff, Ly.b_ff2, nullptr, D->x, d, D->x, d, nullptr, 0, E, d, D->ff,
                       XTRL_ACT_NONE, s)))
      return rc;
  }
  int rc = layernorm_f32(D->x, d, D->ln_final, D->ac_in, D->in_dim, E, d, s);
  if (rc) return rc;
  // heads: hidden [E][4d] = SiLU(ac_in . [Wa1; Wc1]^T + b); logits / critic bins from the halves
  if ((rc = gemm_f32(D->ac_in, D->in_dim, D->w_h1, D->in_dim, D->b_h1, nullptr, nullptr, 0, D->hff, 4 * d, nullptr,
                     0, E, 4 * d, D->in_dim, XTRL_ACT_SILU, s)))
    return rc;
  const int n_act = D->continuous ? 2 * D->A : D->A;
  if ((rc = gemm_f32(D->hff, 4 * d, D->w_a2, 2 * d, D->b_a2, nullptr, nullptr, 0, D->logits, n_act, nullptr, 0, E,
                     n_act, 2 * d, XTRL_ACT_NONE, s)))
    return rc;
  {   // critic bins straight into the trajectory row t (Memory.value, xtrl.py:1315), live envs only
    GemmArgs g;
    g.A = D->hff + 2 * d; g.lda = 4 * d; g.B = D->w_c2; g.ldb = 2 * d; g.bias = D->b_c2;
    g.C = D->traj_values + (int64_t)t * D->B; g.ldc = D->Tmax * D->B; g.M = E; g.N = D->B; g.K = 2 * d;
    g.row_mask = D->alive;
    if ((rc = gemm_run(g, 0, 0, EPI_NONE, s))) return rc;
  }
  hipLaunchKernelGGL(k_sample, dim3((E * SAMPLE_L + 255) / 256), dim3(256), 0, s, *D, t);
  XTRL_LAUNCHED("sample");
  return XTRL_OK;
}

int rollout_begin(const XtrlDecodeDesc* D, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  hipLaunchKernelGGL(k_rollout_begin, dim3((D->E + 255) / 256), dim3(256), 0, s, *D);
  XTRL_LAUNCHED("rollout_begin");
  return XTRL_OK;
}

int attn_decode(const XtrlDecodeDesc* D, int l, int t, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  XTRL_REQUIRE(l >= 0 && l < D->L && t >= 0 && t < D->Tmax, "attn_decode: bad layer / t");
  return launch_attn_decode(D, l, t, s);
}

int env_feedback(const XtrlDecodeDesc* D, int t, const float* next_state, const float* reward,
                 const uint8_t* terminated, const uint8_t* truncated, int t_limit, int bootstrap, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  XTRL_REQUIRE(next_state && reward && terminated && t >= 0 && t < D->Tmax && t_limit > t && t_limit <= D->Tmax,
               "env_feedback: bad arguments (t=%d t_limit=%d Tmax=%d)", t, t_limit, D->Tmax);
  hipLaunchKernelGGL(k_env_feedback, dim3((D->E + 255) / 256), dim3(256), 0, s, *D, t, next_state, reward,
                     terminated, truncated, t_limit, bootstrap);
  XTRL_LAUNCHED("env_feedback");
  return XTRL_OK;
}

int sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update, const int32_t* ep, hipStream_t s) {
  XTRL_REQUIRE(state && ep && E > 0 && S > 0, "sim_reset: bad arguments");
  hipLaunchKernelGGL(k_sim_reset, dim3((E + 255) / 256), dim3(256), 0, s, state, E, S, seed, update, ep);
  XTRL_LAUNCHED("sim_reset");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_decode_step(const XtrlDecodeDesc* desc, int t, void* stream) {
  return xtrl::decode_step(desc, t, xtrl::as_stream(stream));
}
extern "C" int xtrl_rollout_begin(const XtrlDecodeDesc* desc, void* stream) {
  return xtrl::rollout_begin(desc, xtrl::as_stream(stream));
}
extern "C" int xtrl_attn_decode(const XtrlDecodeDesc* desc, int layer, int t, void* stream) {
  return xtrl::attn_decode(desc, layer, t, xtrl::as_stream(stream));
}
extern "C" int xtrl_rollout_env_feedback(const XtrlDecodeDesc* desc, int t, const float* next_state,
                                         const float* reward, const uint8_t* terminated, const uint8_t* truncated,
                                         int t_limit, int bootstrap, void* stream) {
  return xtrl::env_feedback(desc, t, next_state, reward, terminated, truncated, t_limit, bootstrap,
                            xtrl::as_stream(stream));
}
extern "C" int xtrl_sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update,
                              const int32_t* episode_of_slot, void* stream) {
  return xtrl::sim_reset(state, E, S, seed, update, episode_of_slot, xtrl::as_stream(stream));
}
