/*
 * libxtrl_hip — C ABI of the MI355X (gfx950) Learner hot path.
 *
 * The reference (tinycrops/x-transformers-rl) is pure Python: there is no FFI of its own.  Each
 * entry point below replaces a cluster of ATen calls on the reference's rollout/update path; the
 * reference line it stands in for is cited per function ("xtrl.py" = x_transformers_rl/
 * x_transformers_rl.py).  The Python host layer (x-transformers-rl_amd/xtrl_amd) binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every function returns 0 (XTRL_OK) or an XTRL_E_* code; xtrl_last_error() has the message
 *   - all buffers are caller-allocated device memory; plain pointers + sizes, row-major, fp32
 *     unless the name says otherwise; the library keeps no state beyond its code objects
 *   - `stream` is a hipStream_t passed as void*; every call is asynchronous on it and is safe to
 *     capture into a hipGraph (no allocation, no synchronisation inside)
 */
#ifndef XTRL_HIP_H
#define XTRL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XTRL_OK 0
#define XTRL_E_ARG 1    /* invalid argument / unsupported shape */
#define XTRL_E_HIP 2    /* HIP launch or runtime error */

#define XTRL_ABI_VERSION 21

int xtrl_abi_version(void);
/* sizeof(struct) of a descriptor type named by its C name (-1: unknown); host-only */
int64_t xtrl_struct_size(const char* name);
const char* xtrl_last_error(void);
/* content hash of the sources the library was compiled from (x-transformers-rl_amd/xtrl_amd/_srchash.py);
 * bindings compare it with the sources beside the library and refuse a stale build; host-only */
const char* xtrl_source_hash(void);

/* ---------------------------------------------------------------------------------------------
 * Fused fp32 MFMA GEMM  (every nn.Linear on the path: x-transformers to_q/k/v/out, FeedForward,
 * WorldModelActorCritic heads; xtrl.py:315-369, 553-557)
 *   Y[m, n] = act( LN?(X)[m, :] . W[n, :] + bias[n] ) (+ R[m, n])
 *   X [M][K] (ldx), W [N][K] (ldw, nn.Linear layout), Y [M][N] (ldy; Y += (*t_dev) * y_t_stride)
 *   ln_gamma != NULL -> X rows are layer-normalised (eps 1e-5, no beta) and scaled by gamma
 *   act: 0 none, 1 GELU(erf), 2 SiLU, 3 ReLU;  R may alias Y (in-place residual add)
 * ------------------------------------------------------------------------------------------- */
#define XTRL_ACT_NONE 0
#define XTRL_ACT_GELU 1
#define XTRL_ACT_SILU 2
#define XTRL_ACT_RELU 3

int xtrl_gemm_f32(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* ln_gamma,
                  const float* R, int ldr, float* Y, int ldy, const int32_t* t_dev, int64_t y_t_stride, int M,
                  int N, int K, int act, void* stream);

/* General C = A . B (+ bias) with either operand transposed; C = beta * C + result.
 *   trans_a = 0: A[m][k] at A[m * lda + k]   trans_a = 1: A[m][k] at A[k * lda + m]
 *   trans_b = 0: B[k][n] at B[n * ldb + k]   trans_b = 1: B[k][n] at B[k * ldb + n]
 * (nn.Linear backward: dgrad = (0, 1), wgrad = (1, 1) with beta = 1 to accumulate) */
int xtrl_gemm_ex(int trans_a, int trans_b, const float* A, int lda, const float* B, int ldb, const float* bias,
                 float* C, int ldc, int M, int N, int K, float beta, void* stream);

/* nn.Linear weight gradient: dW[N][K] = beta dW + sum_m dY[m][n] X[m][k] over M tokens.  The token
 * range is split over workgroups (partial tiles in ws, ws_floats >= splits * N * K, up to
 * 512 / tiles splits) and summed in fixed order — deterministic. */
int xtrl_gemm_wgrad(const float* dY, int ldy, const float* X, int ldx, float* dW, int ldw, int M, int N, int K,
                    float beta, float* ws, int64_t ws_floats, void* stream);
/* the same with the bias gradient folded in: db[n - db_n0] += sum_m dY[m][n] for n >= db_n0 (from
 * the staged dY slabs of the GEMM; beta must be 1).  nn.Linear.bias.grad (xtrl.py:981 backward) */
int xtrl_gemm_wgrad_db(const float* dY, int ldy, const float* X, int ldx, float* dW, int ldw, int M, int N, int K,
                       float beta, float* ws, int64_t ws_floats, float* db, int db_n0, void* stream);

/* Y[m, :] = layer_norm(X[m, :]) * gamma  (x-transformers LayerNorm, final norm of the Decoder) */
int xtrl_layernorm_f32(const float* X, int ldx, const float* gamma, float* Y, int ldy, int M, int D, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Rollout: one timestep of the vectorised policy for E concurrent episodes.
 * Replaces the per-step body of Learner.forward (xtrl.py:1250-1341): RSNorm eval (:1254-1259),
 * WorldModelActorCritic.forward with KV cache (:479-559 -> x-transformers decode), Discrete
 * sample/log_prob (:1280-1289), env.step (:1297-1313), Memory write (:1315).
 * ------------------------------------------------------------------------------------------- */
typedef struct XtrlDecodeLayer {
  const float* ln_attn;  /* [d]  pre-attention LayerNorm gamma */
  /* decode GEMM weights (w_qkv, w_out, w_ff1, w_ff2, w_h1, w_h2) are fragment-packed (xtrl_dgemm_pack)
   * images of the nn.Linear weights described */
  const float* w_qkv;    /* [n_qkv][d]  rows: to_q | to_k | to_v | to_v_gate (opt) | value-residual mix (opt) */
  const float* b_qkv;    /* [n_qkv]     zeros for q/k/v */
  const float* w_out;    /* [d][I]      to_out */
  const float* ln_ff;    /* [d] */
  const float* w_ff1;    /* [ff][d] */
  const float* b_ff1;    /* [ff] */
  const float* w_ff2;    /* [d][ff] */
  const float* b_ff2;    /* [d] */
  float* k_cache;        /* [E][H][Tmax][dh]  keys (post-rotary) */
  float* v_cache;        /* [E][H][Tmax][dh]  values (post value-residual mix) */
  const float* w_out_t;  /* [I][d]  to_out transposed (plain fp32), or NULL: when set (and the shape
                            allows) the attention kernel applies the out-projection + residual
                            itself, x += W_out o, and no out-projection GEMM runs */
  const uint16_t* w_ff1x; /* split-bf16 images (xtrl_dgemm_pack_x6) of the unpacked [ff][d] FF1 and */
  const uint16_t* w_ff2x; /* [d][ff] FF2 weights, or NULL: when both are set (with xn, mlp_part and
                             mlp_cnt) FF1 + GELU + FF2 + residual + the next pre-norm run as one launch
                             on the bf16 matrix cores (fp32 products as six piece products) */
  /* k-major (transposed, plain fp32) copies for the row-resident step (xtrl_decode_step_rows), or NULL:
   * w_qkv_t [d][round4(n_qkv)] (padding columns zero), w_ff1_t [d][ff], w_ff2_t [ff][d] */
  const float* w_qkv_t;
  const float* w_ff1_t;
  const float* w_ff2_t;
  /* fp32 fragment images (xtrl_dgemm_pack_f8) of FF1 [ff][d] and FF2 [d][ff], or NULL: when both are
   * set the one-launch feed-forward reads these (4 bytes a weight instead of the split images' 6)
   * and splits the weight fragments into their bf16 pieces itself — the same pieces, bit-identical */
  const float* w_ff1f;
  const float* w_ff2f;
} XtrlDecodeLayer;

typedef struct XtrlRngState {   /* device memory; read by the sampling / sim kernels */
  uint64_t seed;
  uint32_t update;
  uint32_t slot_offset;
} XtrlRngState;

typedef struct XtrlDecodeDesc {
  /* shapes */
  int E, S, A, B, d, L, H, dh, Tmax, G, ff, in_dim, n_qkv;
  /* switches */
  int continuous, squash, evolutionary, gate_values, value_residual, learned_mix;
  int rotary_abs;       /* 0: rotary positions restart at 0 for every cached token (reference), 1: absolute */
  int rot_dim;          /* dh / 2 */
  int sim_mode;         /* 0 readme, 1 lander, -1 host env (no device sim step) */
  int hazard_log2;
  int no_reward_cond;   /* 1: model called with rewards=None (deploy without reward, xtrl.py:1042-1061) */
  int state_only;       /* 1: the embedding is project_in(state) alone (the fractal body ignores the action /
                           reward arguments, fractal_rl.py:540-553) */
  float rs_eps;
  float clamp_lo, clamp_hi; int has_clamp;
  /* weights (EMA model for the rollout, xtrl.py:1194) */
  const float* w_pin; const float* b_pin;           /* project_in [d][S] (+[d] or NULL) */
  const float* act_emb; const float* act_emb_b;     /* discrete [A][d]; continuous Linear [d][A] + [d] */
  const float* reward_embed;                        /* [d] */
  const float* w_se; const float* b_se;             /* to_state_embed [d][S], [d] */
  const float* ln_final;                            /* [d] */
  const float* w_h1; const float* b_h1;             /* [4d][in_dim]: action_head.0 rows then critic_head.0 rows */
  const float* w_h2; const float* b_h2;             /* [n_act + B][4d] block diagonal: action_head.2 [n_act][2d] over
                                                       the actor half of the hidden row, critic_head.2 [B][2d] over the
                                                       critic half (n_act = A or 2A); bias [n_act + B] */
  const float* inv_freq;                            /* [rot_dim/2] rotary inverse frequencies */
  const XtrlDecodeLayer* layers;                    /* HOST array of L layer descriptors */
  const float* rs_mean; const float* rs_var;        /* RSNorm running stats [S+1] */
  /* env / episode state (device) */
  float* state;            /* [E][S] current raw state */
  int32_t* prev_action;    /* [E] (-1 at t = 0) */
  float* prev_action_f;    /* [E][A] continuous */
  float* prev_reward;      /* [E] */
  uint8_t* alive;          /* [E] 0 dead, 1 live, 2 bootstrap step pending, 3 + (t & 1) ended at step t by
                              xtrl_decode_step_rows (dead from step t + 1 on; no step clears the markers
                              of the last step: read alive >= 3 as dead — the Python RolloutEngine
                              zeroes them when a rollout ends) */
  int32_t* lens;           /* [E] episode length so far */
  double* cum_reward;      /* [E] cumulative reward (fitness, xtrl.py:1310, 1345-1346) */
  const int32_t* episode_of_slot;  /* [E] episode index keying the Sim stream */
  const int32_t* slot_of_row;      /* [E] global (episode, gene) pair index keying the sampling stream, or
                                      NULL: rng->slot_offset + row (contiguous shards) */
  const XtrlRngState* rng;
  /* trajectory (device), row e = one episode, padded with zeros past its length */
  float* traj_states;      /* [E][Tmax][S] */
  int32_t* traj_actions;   /* [E][Tmax] */
  float* traj_actions_f;   /* [E][Tmax][A] continuous */
  float* traj_logp;        /* [E][Tmax] (continuous: [E][Tmax][A]) */
  float* traj_rewards;     /* [E][Tmax] */
  uint8_t* traj_bounds;    /* [E][Tmax] terminated flags */
  float* traj_values;      /* [E][Tmax][B] critic logits */
  /* scratch (device) */
  /* (per-step activations are indexed by live row, not by episode slot) */
  float* x;      /* [E][d] residual stream */
  float* qkv;    /* [E][n_qkv] */
  float* att;    /* [E][I] */
  float* hff;    /* [E][max(ff or 2 ff with ff_glu, 4d)] */
  float* ac_in;  /* [E][in_dim]  (final-normed embed | state embed | latent embed) */
  float* logits; /* [E][A or 2A] */
  float* v1;     /* [E][I] first layer's values (value residual) */
  float* xn;     /* [E][d] or NULL: LayerNorm(x) * gain of the next projection, written by the kernel
                    that completes the row (the embedding for layer 0's q|k|v, the fused attention
                    for FF1), so that projection runs without a LayerNorm prologue */
  /* live-row compaction: the step-t kernels run over rows 0..live_count[t & 1]-1 only; row r is
   * episode slot live_rows[(t & 1) * E + r] (written by the step's embedding kernel) */
  int32_t* live_rows;        /* [2][E] */
  int32_t* live_count;       /* [2] */
  /* the one-launch feed-forward block: partial outputs of the hidden chunks [ceil(E / 32)][ff / 128]
   * [32][d] and one arrival counter per 16-row panel [ceil(E / 16)] (zero-initialised; every launch
   * leaves them zero), or NULL */
  float* mlp_part;
  uint32_t* mlp_cnt;
  const float* lat_embed;    /* [E][d] latent_to_embed(gene) per episode slot (evolutionary) or NULL */
  /* optional profiling: 2 * Tmax * L hipEvent_t recorded around each attention-decode launch
   * (events[2 (t L + l)] before, [2 (t L + l) + 1] after); NULL = off */
  void** prof_events;
  /* k-major heads, or NULL: w_h1_t [in_dim][4d] (w_h1 transposed; the row-resident step),
   * w_h2_t [4d][round4(n_act + B)] (the block-diagonal w_h2 transposed, padding columns zero; the
   * row-resident step and the one-launch heads) */
  const float* w_h1_t;
  const float* w_h2_t;
  const XtrlDecodeLayer* layers_dev;   /* DEVICE copy of the L layer descriptors (the row-resident step) */
  /* the one-launch heads (hidden layer + SiLU + last projection + sampling), or NULL: w_h1x = the
   * split-bf16 image of w_h1 (xtrl_dgemm_pack_x6 with N = 4d, K = in_dim), heads_part = partial
   * outputs [ceil(E / 16)][4d / 64][16][round4(n_act + B)], heads_cnt = one arrival counter per
   * 16-row panel [ceil(E / 16)] (zero-initialised; every launch leaves them zero) */
  const uint16_t* w_h1x;
  float* heads_part;
  uint32_t* heads_cnt;
  /* the row-resident step's split heads (up to 4 workgroups per row), or NULL (one workgroup per
   * row): row_part = partial outputs [E][4][round4(n_act + B)], row_cnt = one arrival counter per
   * row [E] (zero-initialised; every launch leaves them zero) */
  float* row_part;
  uint32_t* row_cnt;
  /* world_model['ff_glu']: FF1 (w_ff1 / b_ff1) is the GLU projection [2 ff][d]; the step forms
   * hglu [E][ff] = value * gelu(gate) from it (the one-launch feed-forward and the row-resident step
   * are not used) */
  int ff_glu;
  float* hglu;
  /* world_model['attn_qk_norm']: q and k of the new token l2-normalised per head before the rotary
   * (the cache holds normalised, rotated keys); attn_scale: the score scale (qk_norm_scale with qk
   * norm), 0 = dh^-0.5.  xpos_base: rotary xPos scale base (0 = off) — with rotary_abs the rotated
   * pair j of q at position t is scaled by ((j + 0.4 rot_dim) / (1.4 rot_dim)) ^ ((t - (t + 1) / 2) /
   * xpos_base), k by its inverse (the reference's cached decode rotates at position 0: identity) */
  int qk_norm;
  float attn_scale;
  float xpos_base;
  /* world_model['use_rmsnorm']: every pre-norm and the final norm are x-transformers' RMSNorm
   * (F.normalize(x) sqrt(d) g) instead of its LayerNorm; 0: LayerNorm */
  int rms_norm;
  /* host-env loop (xtrl_host_decode): pinned host memory the device can address (int32 [E] actions,
   * continuous: float [E][A]), or NULL.  When set, the sampling also stores each row's action
   * there (and the rollout start its -1 / 0 reset), so xtrl_host_decode passed this same buffer only
   * synchronises — no device->host copy per step */
  void* act_host;
} XtrlDecodeDesc;

/* Reset: state_0 = sim reset, prev_action = -1 / 0, prev_reward = 0, alive = 1, lens = 0, and
 * the latent embedding columns of ac_in must already hold latent_to_embed(gene) (evolutionary). */
int xtrl_rollout_begin(const XtrlDecodeDesc* desc, void* stream);
/* one timestep t for all E episodes; with sim_mode == -1 the env step happens on the host and
 * xtrl_rollout_env_feedback() writes its results back. */
int xtrl_decode_step(const XtrlDecodeDesc* desc, int t, void* stream);
/* The same step, row-resident (replaces xtrl_decode_step for few live rows / small models; same
 * outputs to fp32 rounding): one workgroup carries a live row through compaction, embeddings, every
 * layer, the heads and the sampling + Sim step in ONE launch, min(max_rows, E) workgroups taking
 * live rows b, b + grid, ...  Needs the k-major weights (w_qkv_t / w_ff1_t / w_ff2_t, w_out_t,
 * w_h1_t / w_h2_t), d <= 256, E <= 8192, L <= 64, n_act <= 64, layers_dev, its LDS within 96 KiB (the
 * reference loop it replaces: x_transformers_rl.py:1250-1341).  Its GEMVs read whole float4 columns:
 * b_qkv must hold round4(n_qkv) floats and b_h2 round4(n_act + B), the padding zero.  The step never
 * turns a slot it ranks from live to dead: a Sim episode it ends reads alive = 3 + (t & 1) until the
 * next step's compaction clears it to 0 (every compaction treats 3 + (t & 1) as live at step t only). */
int xtrl_decode_step_rows(const XtrlDecodeDesc* desc, int t, int max_rows, void* stream);
/* Diagnostics of the row-resident step (no reference counterpart): synchronises the device, copies
 * the phase stamps of the last stamped launch (wall-clock ticks taken by workgroup 0 after each
 * phase of its first row: start, compaction, embedding, 7 per layer — LN, q|k|v, attention,
 * out-projection, LN, FF1, FF2 — final LN, hidden, last Linear, sampling) into out[0..cap) — the
 * wall-clock stamps at [0, n), the same points' shader-clock counters at [n, 2 n), n the returned
 * capacity — stores the wall-clock tick rate, then turns stamping on (on != 0) or off for later
 * launches. */
int xtrl_row_stamps(int on, uint64_t* out, int cap, int64_t* ticks_per_sec);
/* Host env results of step t (xtrl.py:1297-1336) for the live rows: next_state [E][S], reward [E],
 * terminated [E] (stored as is_boundary), truncated [E] or NULL.  An episode ends when terminated,
 * truncated or t + 1 == t_limit (max_timesteps); with `bootstrap` a truncated, not terminated
 * episode takes one more decode step that only writes its critic logits (the next state's value,
 * xtrl.py:1323-1336) into the padding slot traj_values[e][t + 1] (needs t + 1 < Tmax); a row still
 * flagged for that step (alive 2: the row-resident step leaves the flag) is cleared here. */
int xtrl_rollout_env_feedback(const XtrlDecodeDesc* desc, int t, const float* next_state, const float* reward,
                              const uint8_t* terminated, const uint8_t* truncated, int t_limit, int bootstrap,
                              void* stream);
/* Host-env loop helpers (the reference's `env.step(action.tolist())` loop, xtrl.py:1284-1341), one call
 * per half of a step.  The exception to the no-synchronisation rule above: xtrl_host_decode runs
 * decode step t (rows_max > 0: xtrl_decode_step_rows), copies the rows' actions (prev_action [E]
 * int32, continuous prev_action_f [E][A]) to act_host (pinned host memory) and synchronises the
 * stream — the one host wait of a step; when act_host is desc->act_host the sampling already stored
 * the actions there and no copy runs.  xtrl_host_feedback copies the pinned stage (next_state
 * [E][S] fp32 | reward [E] fp32 | terminated [E] u8 | truncated [E] u8) to dev_stage (device, same
 * layout) and runs xtrl_rollout_env_feedback on it; dev_stage NULL: the kernel reads the pinned
 * stage in place (device-addressable pinned memory), no host->device copy. */
int xtrl_host_decode(const XtrlDecodeDesc* desc, int t, int rows_max, void* act_host, void* stream);
int xtrl_host_feedback(const XtrlDecodeDesc* desc, int t, const void* host_stage, void* dev_stage, int t_limit,
                       int bootstrap, void* stream);
/* The gated form of the scalar-env loop (one row, E == 1, the row-resident step; ABI 21): step t is
 * queued ahead of the host's env step.  gate = pinned uint32 [3], zeroed per wave: gate[0] the host's
 * step counter ("go"), gate[1] the last completed step + 1 ("done"), gate[2] the last step + 1 that
 * gave up.  The launch waits ON THE DEVICE until gate[0] >= t + 1, applies step t - 1's env results
 * from the pinned stage (xtrl_host_feedback's layout and arithmetic; none at t = 0), runs decode step
 * t (desc->act_host receives the action) and stores gate[1] = t + 1.  gate[0] = 0xFFFFFFFF cancels every
 * queued step (they exit untouched); no go within XTRL_HOST_GATE_WAIT_MS (default 4000 ms): the launch
 * exits untouched and stores gate[2] = t + 1.  xtrl_host_wait(gate + 1, value, timeout_s) spins on the
 * host until gate[1] >= value (returns 0), gate[2] >= value (1: the device gave up; cancel, feed back
 * and run the step the ungated way) or timeout_s passed (-1).  Replaces the per-step launch + stream
 * synchronisation + feedback launch of the reference loop's device half (xtrl.py:1284-1341). */
int xtrl_host_row_step(const XtrlDecodeDesc* desc, int t, const void* host_stage, int t_limit, int bootstrap,
                       uint32_t* gate, void* stream);
int xtrl_host_wait(const uint32_t* done, uint32_t value, double timeout_s);

/* Decode-step projection (the rollout's GEMM):
 *   C[dst(m), n] = act( LN?(A)[m, :] . W[n, :] + bias[n] ) (+ R[m, n])   for m < (m_dev ? *m_dev : M)
 * W an nn.Linear weight [N][K] (xtrl.py's Linear layers, x-transformers projections) in the
 * fragment-packed layout of xtrl_dgemm_pack; ln_gamma != NULL applies the x-transformers LayerNorm
 * (no affine, eps 1e-5, times gamma) to A's columns [0, ln_k) first (Decoder pre-norms / final
 * norm, ln_k <= 512); dst(m) = row_map ? row_map[m] : m; act 0 / 1 GELU / 2 SiLU.  K, lda
 * multiples of 4, A 16-byte aligned. */
int xtrl_dgemm(const float* A, int lda, const float* Wp, const float* bias, const float* ln_gamma, int ln_k,
               const float* R, int ldr, float* C, int ldc, const int32_t* row_map, const int32_t* m_dev, int M, int N,
               int K, int act, void* stream);
/* Fragment packing of W [N][K] (row stride ldw) into Wp (xtrl_dgemm_packed_floats(N, K) floats):
 * float4 slot ((n / 16 * JN + j) * 4 + q) * 16 + n % 16 holds W[n][q Kp/4 + 4 j .. + 3], Kp = K
 * rounded up to 16, JN = Kp / 16, zero-padded past N and K — each MFMA fragment load of the
 * decode GEMM reads 1 KiB contiguous.  Done once per rollout (the EMA weights are fixed for it). */
int64_t xtrl_dgemm_packed_floats(int N, int K);
int xtrl_dgemm_pack(const float* W, int ldw, int N, int K, float* Wp, void* stream);
/* Split-bf16 fragment packing of W [N][K] (K a multiple of 32) for the v_mfma_f32_16x16x32_bf16
 * operand: every value w = hi + mid + lo exactly (bf16 pieces); three planes (hi, mid, lo) of
 * xtrl_dgemm_packed_x6_elems(N, K) / 3 bf16 each, the 16-byte slot (n / 16 * K / 32 + s) * 64 + lane
 * of a plane holding W[16 (n / 16) + lane % 16][32 s + 8 (lane / 16) .. + 7], zero past N. */
int64_t xtrl_dgemm_packed_x6_elems(int N, int K);
int xtrl_dgemm_pack_x6(const float* W, int ldw, int N, int K, uint16_t* Wp, void* stream);
/* The same fragment order in fp32 (K a multiple of 32): two planes of xtrl_dgemm_packed_f8_floats(N, K)
 * / 2 floats, float4 slot (n / 16 * K / 32 + s) * 64 + lane of plane h holding
 * W[16 (n / 16) + lane % 16][32 s + 8 (lane / 16) + 4 h .. + 3], zero past N. */
int64_t xtrl_dgemm_packed_f8_floats(int N, int K);
int xtrl_dgemm_pack_f8(const float* W, int ldw, int N, int K, float* Wp, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fractal policy body, one decode step (fractal_rl.py:37-346, 510-619 restated per timestep and
 * causal so it can stand in for the Decoder in the rollout / PPO loop — DESIGN §6).  Per live row
 * (the XtrlDecodeDesc's compaction, embedding (state_only = 1, b_pin = input_embed.bias + level
 * embedding 0), heads and sampling are reused; its layers[l] hold level l's K/V caches and
 * n_qkv = 3 I):
 *   for each level l:
 *     c  = W_c,l g  (W_c = W_out,g W_v,g; level 0: the constant row c0)   cross-attention to the one-token
 *                                                                           global state (softmax over one key)
 *     x2 = LN2(LN1(x + W_out attn(W_q x, W_k x, W_v x)) + c)               causal self-attention over the
 *                                                                           cache; both add + LayerNorms in one
 *     x3 = LN3(x2 + FF(x2)); m = mean over this episode's steps 0..t of x3 (running sums per slot);
 *     x <- x3 + level_embed[l+1]                                           one launch
 *     [g | p_l] = [g | 0] + m [W_gu; W_p,l]^T + [b_gu; b_p,l]               one GEMM
 *   features = W_fa2 ReLU(W_fa0 [p_0 | ... | p_{L-1} | g] + b) + b  -> ac_in[:, 0:d] -> heads
 * GEMM weights fragment-packed (xtrl_dgemm_pack); LayerNorms nn.LayerNorm (eps, weight, bias). */
typedef struct XtrlFractalLevel {
  const float* w_qkv;                       /* [3I][d]  self_attn.to_q | to_k | to_v */
  const float* w_out;                       /* [d][I]   self_attn.to_out */
  const float* ln1_w; const float* ln1_b;   /* [d] norm1 */
  const float* w_c;                         /* [d][d]   global_attn.to_out . to_v (the one-key cross-attention,
                                             *          one operand: W_out W_v g) */
  const float* ln2_w; const float* ln2_b;
  const float* w_ff1; const float* b_ff1;   /* [ff][d], [ff] */
  const float* w_ff2; const float* b_ff2;   /* [d][ff], [d] */
  const float* ln3_w; const float* ln3_b;
  const float* w_pg; const float* b_pg;     /* [2d][d], [2d]: global_state_update | level_projections[l] — one
                                             * GEMM over the running mean: columns [0, d) update g in place,
                                             * [d, 2d) the level's projection into allf */
  const float* level_emb;                   /* [d] level_embeds[l] + scale_embeds[l] (added for l > 0) */
  float* sums;                              /* [E][d] running sum of this level's outputs per episode slot */
} XtrlFractalLevel;

typedef struct XtrlFractalDesc {
  int levels;
  float ln_eps;
  const XtrlFractalLevel* level;            /* HOST array of `levels` descriptors */
  const float* g_init;                      /* [2d] global_state_init | zeros */
  const float* c0;                          /* [d] level 0's cross-attention row W_c,0 g_init (every row) */
  const float* w_fa0; const float* b_fa0;   /* final_aggregation.0 [2d][(L+1) d], [2d] */
  const float* w_fa2; const float* b_fa2;   /* final_aggregation.2 [d][2d], [d] */
  float* g;                                 /* [E][2d] global state of the step's rows | zeros (the columns the
                                             * fused update GEMM's residual reads for its projection half) */
  float* c2;                                /* [E][d] cross-attention rows (levels > 0) */
  float* tmp;                               /* [E][d] projection outputs before their add + LayerNorm */
  float* x2;                                /* [E][d] norm2 output (the feed-forward input) */
  float* mean;                              /* [E][d] the level's running mean */
  float* allf;                              /* [E][(L+1) d] */
  float* hagg;                              /* [E][2d] */
} XtrlFractalDesc;

/* one timestep of the fractal policy for the live rows of `desc` (xtrl_rollout_begin first; the
 * level sums are zeroed by the caller at the start of an episode batch) */
int xtrl_fractal_decode_step(const XtrlDecodeDesc* desc, const XtrlFractalDesc* fd, int t, void* stream);

/* ---------------------------------------------------------------------------------------------
 * HL-Gauss value decode + GAE   (xtrl.py:843-852 -> calc_gae :616-640, HLGaussLoss value)
 *   values[e, t] = softmax(logits[e, t, :]) . centres     (B bins over [lo, hi])
 *   returns = reverse scan of delta_t = r_t + gamma v_{t+1} m_t - v_t, gate = gamma lam m_t;
 *   m_t = !bounds[e, t]; sequential order per row (bitwise stable)
 *   logits row (e, t) at logits + e*ld_row + t*B; rewards / bounds at e*ld_seq + t;
 *   values / returns written densely [E][n]; gamma_lam = float32(gamma * lam) as the reference
 *   multiplies the Python product into the mask
 *   boot [E] (or NULL): the value of the state after a truncated episode's last step (NaN: none);
 *   it stands in for v at index lens[e] (xtrl.py:1323-1336 bootstrap memory)
 * ------------------------------------------------------------------------------------------- */
int xtrl_hlgauss_gae(const float* logits, int64_t ld_row, const float* rewards, const uint8_t* bounds,
                     int64_t ld_seq, const float* centers, float* values, float* returns, int E, int n, int B,
                     float gamma, float gamma_lam, const float* boot, const int32_t* lens, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Training attention (x-transformers Attend with causal + key-padding mask, post-softmax dropout)
 *   q, k, v: [b][H][n][dh]; lens[b] valid keys per row; out o [b][H][n][dh]; lse [b][H][n]
 * ------------------------------------------------------------------------------------------- */
/* dropout keep(b, h, i, j), c2 = offset + b * H + h: when 256 p is an integer (p = 0.25), byte (i & 3)
 * of word ((j >> 4) & 3) of philox(seed; i >> 2, 16 (j >> 6) + (j & 15), c2, (6 << 24) | sub | 1 << 23)
 * >= 256 p; otherwise word (i & 3) of philox(seed; i >> 2, j, c2, (6 << 24) | sub) >= p * 2^32;
 * sub (< 2^23) names the decoder layer */
int xtrl_attn_fwd(const float* q, const float* k, const float* v, const int32_t* lens, float* o, float* lse,
                  int b, int H, int n, int dh, float scale, float dropout_p, uint64_t seed, uint32_t offset,
                  uint32_t sub, void* stream);
int xtrl_attn_bwd(const float* q, const float* k, const float* v, const int32_t* lens, const float* o,
                  const float* lse, const float* dout, float* dq, float* dk, float* dv, float* delta_ws, int b,
                  int H, int n, int dh, float scale, float dropout_p, uint64_t seed, uint32_t offset, uint32_t sub,
                  void* stream);
/* xtrl_attn_bwd with a workspace for long episodes (n > 128, dh = 16; same backward, xtrl.py:981 over
 * the attention of :928-935): the dK / dV kernel forms dQ from the same P / dS per (key tile, query
 * tile) pair — rows with one contributing key tile get dQ directly (bit-identical to xtrl_attn_bwd),
 * the others one partial per key tile in dq_part, summed in key-tile order by a reduce launch.
 * dq_part_floats >= xtrl_attn_bwd_part_floats(b, H, n, dh) = ceil(n / 64) * b * H * n * dh; a smaller
 * (or NULL) workspace takes xtrl_attn_bwd's kernel pair. */
int64_t xtrl_attn_bwd_part_floats(int b, int H, int n, int dh);
int xtrl_attn_bwd_part(const float* q, const float* k, const float* v, const int32_t* lens, const float* o,
                       const float* lse, const float* dout, float* dq, float* dk, float* dv, float* delta_ws,
                       float* dq_part, int64_t dq_part_floats, int b, int H, int n, int dh, float scale,
                       float dropout_p, uint64_t seed, uint32_t offset, uint32_t sub, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Learn-step forward / backward of WorldModelActorCritic on one minibatch, hand-scheduled (no
 * autograd): replaces `model(..., mask=mask)` + `loss.backward()` of Agent.learn
 * (xtrl.py:928-935, 982) with the x-transformers Decoder inside.
 *   T = b * n tokens (token t = episode * n + step), activations token-major [T][features].
 *   Parameters live in ONE fp32 buffer `flat`; gradients at the same offsets of `grad`
 *   (accumulated: the caller zeroes `grad`).  Offsets are in floats, -1 = absent.
 * Forward writes raw / values / pred / done (the inputs of xtrl_loss_fwd) and saves what the
 * backward needs; backward consumes d_raw / d_values / d_pred / d_done (xtrl_loss_bwd).
 * Dropout streams (Philox counter (c0, c1, c2, c3), c3 = field << 24 | sub):
 *   feed-forward  keep(m, n) = word (m & 3) of philox(seed; n, m >> 2, ff_offset, (7 << 24) | 2 layer)
 *                 >= p * 2^32; when 256 p is an integer, byte (m & 3) of word ((m >> 3) & 3) of
 *                 philox(seed; n, 2 (m >> 5) + ((m >> 2) & 1), ff_offset, (7 << 24) | (2 layer + 1)) >= 256 p;
 *   attention     as xtrl_attn_fwd with offset attn_offset and sub = layer.
 * The caller gives every minibatch its own ff_offset and a disjoint [attn_offset, attn_offset + b H)
 * range (xtrl_amd/learner.py: minibatch ordinal and ordinal * batch_size * H).
 * ------------------------------------------------------------------------------------------- */
typedef struct XtrlTrainLayer {
  int64_t ln_attn, w_proj, b_proj, w_out, ln_ff, w_ff1, b_ff1, w_ff2, b_ff2;
  int n_qkv;            /* 3I (+ I value gates) (+ H value-residual mix, layers >= 2) */
  int mix;              /* learned value-residual mix in this layer */
  float* x_attn;        /* [T][d] residual stream entering the attention block */
  float* x_ff;          /* [T][d] entering the feed-forward block */
  float* xn_attn;       /* [T][d] LayerNorm outputs */
  float* xn_ff;
  float* st_attn;       /* [T][2] LayerNorm (mean, rstd) */
  float* st_ff;
  float* proj;          /* [T][n_qkv] q | k | v | gate | mix pre-activations */
  float* qkv;           /* [T][3I] rotary q, k and (mixed) v */
  float* o;             /* [T][I] attention output */
  float* og;            /* [T][I] gated output (== o when there are no value gates) */
  float* lse;           /* [b][H][n] */
  float* u;             /* [T][ff] FF1 local derivative: dropout-masked GELU'(pre-activation) */
  float* hd;            /* [T][ff] GELU + dropout output */
} XtrlTrainLayer;

typedef struct XtrlTrainDesc {
  int b, n, S, A, d, L, H, dh, ff, B, in_dim, n_out, G;
  int continuous, evolutionary, gate_values, rot_dim;
  float dropout, frac_head_grad, reward_keep, attn_scale;
  uint64_t seed;
  uint32_t attn_offset, ff_offset;
  float* flat;
  float* grad;
  int64_t w_pin, act_emb, act_emb_b, reward_embed, w_se, b_se, ln_final;
  int64_t w_pd, b_pd;   /* to_pred.0 | to_pred_done: weights [d + 1][2d], biases [d + 1], adjacent */
  int64_t w_pred2, b_pred2, w_lat, b_lat, w_h1, b_h1, w_a2, b_a2, w_c2, b_c2;
  const float* inv_freq;         /* [rot_dim / 2] */
  /* minibatch */
  const float* swr;              /* [T][S + 1] normalised states | normalised previous reward */
  const int32_t* prev_action;    /* [T] discrete, -1 = none */
  const int32_t* next_action;    /* [T] */
  const float* prev_action_f;    /* [T][A] continuous */
  const float* next_action_f;
  const float* latent;           /* [b][G] (evolutionary) */
  const int32_t* lens;           /* [b] */
  /* forward outputs */
  float* raw;                    /* [T][n_out] */
  float* values;                 /* [T][B] */
  float* pred;                   /* [T][2 (S + 1)] */
  float* done;                   /* [T] */
  /* head activations */
  float* x_final;                /* [T][d] residual stream after the last block */
  float* st_final;               /* [T][2] */
  float* ac_in;                  /* [T][in_dim] embed | state_embed | latent_embed */
  float* ewa;                    /* [T][2d] embed | next-action embed */
  float* zp;                     /* [T][d + 4] local derivative of SiLU(to_pred.0) | 1 (done column) */
  float* hp;                     /* [T][d + 4] SiLU(to_pred.0) | done logit */
  float* z1;                     /* [T][4d] local derivative of SiLU(action_head.0 | critic_head.0) */
  float* h1;                     /* [T][4d] SiLU */
  float* lat_e;                  /* [b][d] */
  /* loss gradients */
  const float* d_raw;
  const float* d_values;
  const float* d_pred;
  const float* d_done;
  /* backward scratch */
  float* dx;                     /* [T][d] */
  float* dx2;                    /* [T][d] second residual-gradient buffer (fused LayerNorm backward) */
  float* dxn;                    /* [T][d] */
  float* dff;                    /* [T][ff] */
  float* dproj;                  /* [T][max n_qkv] */
  float* dog;                    /* [T][I] */
  float* dvfirst;                /* [T][I] */
  float* dz1;                    /* [T][4d] */
  float* dac;                    /* [T][in_dim] */
  float* dzp;                    /* [T][d + 4] */
  float* dewa;                   /* [T][2d] */
  float* delta;                  /* [b][H][n] */
  float* part;                   /* deterministic partial sums */
  int64_t part_floats;
  float* ws;                     /* split-K weight-gradient partial tiles */
  int64_t ws_floats;
  const XtrlTrainLayer* layers;  /* host array [L] */
  /* optional live timing of the dominant kernel (the 128x128-tile weight-gradient GEMM): event pair
   * (prof_events[2i], prof_events[2i+1]) brackets its i-th launch and prof_flops[i] = 2 M N K;
   * *prof_n counts launches (the caller resets it); NULL prof_events = off */
  void** prof_events;
  double* prof_flops;
  int prof_cap;
  int* prof_n;
  /* optional data-parallel gradient buckets (NULL = off): the backward records, for bucket i =
   * 0 .. L + 1 in completion order (0: heads + final norm, 1 + j: decoder block L - 1 - j, L + 1:
   * embeddings / everything), grad_events[2i] on the caller's stream and grad_events[2i + 1] on the
   * weight-gradient stream once every gradient of the bucket is final, so the caller can all-reduce
   * bucket i (a contiguous range of the flat gradient, xtrl_amd.model flat_order) while the backward
   * continues (DDP's bucketed all-reduce, xtrl.py:885/981).  xtrl_fractal_train_backward: buckets
   * 0 .. levels + 1 (0: heads + action embedding + final aggregation, 1 + j: level levels - 1 - j,
   * levels + 1: input embedding / global state / level embeddings / everything else;
   * xtrl_amd.fractal flat_buckets_names) */
  void** grad_events;
  /* row stride (floats) of the [T][ff] feed-forward buffers hd, u, dff (the fractal body's h, u, dz):
   * >= ff, a multiple of 4; 0 = ff.  A stride off the 4 KiB power of two (e.g. ff + 16) spreads the
   * FF1 epilogue's two store streams over the memory channels */
  int ld_ff;
  /* 1 (decoder step with the fused LayerNorms): the backward buffers the weight-gradient stream reads
   * are per-layer planes — dx [L + 1][T][d], dx2 [L][T][d], dff [L][T][ld_ff], dproj [L][T][max n_qkv]
   * — written once per backward, so the caller's stream never waits for the weight-gradient stream
   * before the final join; 0: one plane each, reused layer by layer behind events */
  int scratch_per_layer;
  /* world_model['ff_glu'] (x-transformers FeedForward glu = True): w_ff1 / b_ff1 are the GLU
   * projection [2 ff][d] / [2 ff] (value rows, then gate rows); per layer u holds its output
   * [T][ld_u2] (ld_u2 >= 2 ff, a multiple of 4) for the backward, dff is the projection's gradient
   * ([L][T][ld_u2] planes), glu_dh [T][ld_ff] the gradient w.r.t. the GLU + dropout output.  0: GELU */
  int ff_glu;
  int ld_u2;
  float* glu_dh;
  /* world_model['attn_qk_norm'] (x-transformers qk norm): q and k are l2-normalised per head
   * (F.normalize, eps 1e-12) before the rotary, and attn_scale carries qk_norm_scale (default 10).
   * 0: off */
  int qk_norm;
  /* world_model['rotary_xpos'] (x-transformers RotaryEmbedding use_xpos): the rotary scale base
   * (rotary_xpos_scale_base, default 512), 0 = off.  Rotated channel pair j (even) of q at position p
   * of the n-step minibatch is multiplied by ((j + 0.4 rot_dim) / (1.4 rot_dim)) ^ ((p - n / 2) /
   * xpos_base), that of k divided by it */
  float xpos_base;
  /* world_model['use_rmsnorm'] (x-transformers RMSNorm: F.normalize(x) sqrt(d) g, no mean, eps 1e-12
   * on the norm) for every pre-norm and the final norm, forward and backward; 0: LayerNorm */
  int rms_norm;
  /* world-model heads over the valid tokens only: Tv = sum over the minibatch of min(lens[e], n)
   * (from the host), 0 < Tv < b n.  Their outputs feed only masked losses (xtrl.py:944, 949: the
   * world-model and done terms of padded tokens are dropped), so to_pred / to_pred_done run on the
   * Tv valid rows, gathered in (episode, step) order (vrows [T], vinv [T] int32 scratch: the row
   * list and its inverse, -1 for padding), and pred / done / dewa are scattered back with zeros on
   * the padded rows.  Tv = 0 (or vrows NULL): every row.  Compact buffers, Tv rows each:
   * ewa_v [2d], hp_v / zp_v / dzp_v [d + 4], pred_v / d_pred_v [2 (S + 1)], dewa_v [2d] */
  int Tv;
  int32_t* vrows;
  int32_t* vinv;
  float* ewa_v;
  float* hp_v;
  float* zp_v;
  float* pred_v;
  float* d_pred_v;
  float* dzp_v;
  float* dewa_v;
  /* long episodes (n > 128, dh = 16): the attention backward's dQ partial workspace
   * (xtrl_attn_bwd_part_floats(b, H, n, dh) floats), or NULL for the dK / dV + dQ kernel pair */
  float* dq_part;
  int64_t dq_part_floats;
  /* packed learn step (per-token critic reduction only, Agent(packed_learn=True); xtrl.py:936-978 with
   * hl_reduction_mean=False): the minibatch's Tv = sum(min(lens, n)) valid tokens are computed in
   * episode-then-step order without the padding — the inputs (swr, actions; the minibatch's [b][n]
   * layout as usual) are gathered into pack_ws, every row-wise kernel runs on Tv rows, the attention
   * on per-episode row ranges (ep_off [b + 1], written by the forward), rotary positions from the
   * row list (vrows), the FF dropout keyed by the packed row; raw / values / pred / done are
   * scattered back to [b][n] (zeros on the padding) for xtrl_loss_*, whose gradients the backward
   * gathers again.  pack_ws_floats >= xtrl_train_pack_floats(b * n, S, A, n_out, B). */
  int packed;
  int32_t* ep_off;
  float* pack_ws;
  int64_t pack_ws_floats;
} XtrlTrainDesc;

int xtrl_train_forward(const XtrlTrainDesc* desc, void* stream);
int xtrl_train_backward(const XtrlTrainDesc* desc, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Hand-scheduled learn step of the causal fractal policy body (xtrl_amd.fractal
 * FractalPolicyActorCritic: fractal_rl.py:116-132, 274-346 made causal per timestep, DESIGN.md
 * decision log).  Replaces the reference-mode autograd step (model.forward_train + loss.backward,
 * xtrl.py:928-983): the base XtrlTrainDesc carries the minibatch, the heads (identical to the
 * decoder's: to_pred / to_pred_done / actor / critic / state and gene embeddings), the loss
 * gradients and the workspaces (its layers / L / H-projection fields are unused; w_pin / ln_final
 * unused); the fractal descriptor the encoder.  Per level: x_in = x + level_embed; q|k|v; causal
 * flash attention (dropout); s1 = x_in + o W_out^T, x1 = LN1(s1); s2 = x1 + (g W_gv^T) W_go^T,
 * x2 = LN2(s2); h = drop(gelu(x2 W1^T + b1)); s3 = x2 + h W2^T + b2, x3 = LN3(s3); mean = causal
 * running mean of x3; cat[:, l d:] = mean W_p^T + b_p; g <- g + mean W_gu^T + b_gu.  Then
 * features = ReLU(cat W_fa0^T + b) W_fa2^T + b (cat's last d columns: the final g).
 * nn.LayerNorm (weight and bias) is formed in the epilogue of the GEMM completing its rows.
 * --------------------------------------------------------------------------------------------- */
typedef struct XtrlFractalTrainLevel {
  int64_t w_qkv;                   /* self_attn.to_q | to_k | to_v [3I][d], adjacent in the flat buffer */
  int64_t w_out, w_gv, w_go;       /* self_attn.to_out [d][I], global_attn.to_v [I][d], .to_out [d][I] */
  int64_t ln1_w, ln1_b, ln2_w, ln2_b, ln3_w, ln3_b;
  int64_t w_ff1, b_ff1, w_ff2, b_ff2, w_proj, b_proj, level_embed;
  /* activations [T][.] kept for the backward */
  float* xin;                      /* [T][d] level input (x + level embedding) */
  float* qkv;                      /* [T][3I] */
  float* o;                        /* [T][I] attention output */
  float* lse;                      /* [b][H][n] */
  float* s1; float* x1; float* st1;   /* pre-norm sum, normalised, (mean, rstd) [T][2] */
  float* g;                        /* [T][d] global state entering the level */
  float* gv;                       /* [T][I] g W_gv^T */
  float* s2; float* x2; float* st2;
  float* h; float* u;              /* [T][ff] drop(gelu) and its saved derivative */
  float* s3; float* x3; float* st3;
  float* mean;                     /* [T][d] causal running mean of x3 */
} XtrlFractalTrainLevel;

typedef struct XtrlFractalTrainDesc {
  int levels;
  int64_t b_in;                    /* input_embed.bias (its weight: the base's w_pin) */
  int64_t g_init, w_gu, b_gu, w_fa0, b_fa0, w_fa2, b_fa2;
  const float* scale_embeds;       /* [levels][d] (level_embedding.scale_embeds buffer) */
  float* le;                       /* [levels][d] scratch: level_embeds + scale_embeds */
  float* bias0;                    /* [d] scratch: input_embed.bias + le[0] */
  float* cat;                      /* [T][(levels + 1) d] level projections | final global state */
  float* hfa;                      /* [T][2d] ReLU(final_aggregation[0]) */
  /* backward scratch; the planes a side-stream weight gradient reads are per level, so the main
   * stream never waits for the side stream before the final join */
  float* dxa; float* dxb; float* dmean;   /* [T][d] */
  float* ds;                       /* [3 levels + 1][T][d]: per level the norm1 / norm2 / norm3 input
                                    * gradients, then d features */
  float* dga;                      /* [levels][T][d] gradient of each level's global state */
  float* dgb;                      /* unused (NULL) */
  float* dgv;                      /* [levels][T][I] */
  float* dz;                       /* [levels][T][ld_ff] */
  float* dqkv;                     /* [levels][T][3I] */
  float* dob;                      /* [T][I] */
  float* dcat;                     /* [T][(levels + 1) d] */
  float* dhfa;                     /* [T][2d] */
  const XtrlFractalTrainLevel* level;   /* host array [levels] */
} XtrlFractalTrainDesc;

int xtrl_fractal_train_forward(const XtrlTrainDesc* base, const XtrlFractalTrainDesc* f, void* stream);
int xtrl_fractal_train_backward(const XtrlTrainDesc* base, const XtrlFractalTrainDesc* f, void* stream);
/* Y = drop(gelu(X W^T + b)) and deriv = drop(gelu'(X W^T + b)) (x-transformers FeedForward's first
 * Linear + GELU + Dropout, xtrl.py Decoder ff; fractal_rl.py FeedForward), dropout keep bits the
 * stream of xtrl_ff_dropout_mask(seed, offset, layer) and of the fused learn step */
int xtrl_linear_gelu_drop(const float* X, int ldx, const float* W, const float* bias, float* Y, int ldy, float* deriv,
                          int ld_deriv, int M, int N, int K, float p, uint64_t seed, uint32_t offset, uint32_t layer,
                          void* stream);
/* the feed-forward dropout keep mask of layer `layer` as uint8 [M][N] (tests / reference mode) */
int xtrl_ff_dropout_mask(uint8_t* mask, int M, int N, float p, uint64_t seed, uint32_t offset, uint32_t layer,
                         void* stream);
/* x-transformers FeedForward with glu = True (world_model['ff_glu']): u [M][2 ff] = the GLU projection's
 * output [value | gate], h[m][j] = drop(u[m][j] * gelu(u[m][ff + j])) (erf GELU, the dropout keep bits
 * of xtrl_ff_dropout_mask(seed, offset, layer) over [M][ff]); the backward writes du [M][2 ff] from dh */
int xtrl_glu_drop_fwd(const float* u, int ldu, float* h, int ldh, int M, int ff, float p, uint64_t seed,
                      uint32_t offset, uint32_t layer, void* stream);
int xtrl_glu_drop_bwd(const float* dh, int lddh, const float* u, int ldu, float* du, int lddu, int M, int ff, float p,
                      uint64_t seed, uint32_t offset, uint32_t layer, void* stream);
/* floats of XtrlTrainDesc.part (the partial-sum workspace) a learn step of T = b * n tokens needs;
 * host-only, no device call */
int64_t xtrl_train_part_floats(int T, int b, int d, int A);
/* floats of XtrlTrainDesc.pack_ws for up to T packed tokens */
int64_t xtrl_train_pack_floats(int T, int S, int A, int n_out, int B);

/* ---------------------------------------------------------------------------------------------
 * Minibatch assembly for the learn step (Agent.learn data prep, xtrl.py:816-924): gathers the
 * minibatch's episodes (idx) from the device trajectory, shifts actions / rewards right by one
 * step (pad_at_dim, xtrl.py:127-138, fill -1 for discrete actions), normalises [state, previous
 * reward] with the RSNorm statistics (xtrl.py:591), and produces the masked column mean of the
 * normalised rows that feeds the RSNorm copy update (xtrl.py:598-610, 1005).
 * ------------------------------------------------------------------------------------------- */
typedef struct XtrlBatchDesc {
  int N, Tmax, n, b, S, A, B, continuous;
  /* trajectory [N][Tmax][.] (rollout buffers) and per-update tensors */
  const float* states;        /* [N][Tmax][S] */
  const int32_t* actions;     /* [N][Tmax] discrete */
  const float* actions_f;     /* [N][Tmax][A] continuous */
  const float* rewards;       /* [N][Tmax] */
  const float* logp;          /* [N][Tmax] (continuous [N][Tmax][A]) */
  const uint8_t* bounds;      /* [N][Tmax] */
  const float* values;        /* [N][Tmax][B] */
  const float* returns;       /* [N][n] */
  const int32_t* lens;        /* [N] */
  const int64_t* idx;         /* [b] episode indices of the minibatch */
  const float* rs_mean;       /* [S + 1] normalisation statistics */
  const float* rs_var;
  /* outputs [b][n][.] */
  float* swr;                 /* [b][n][S + 1] */
  int32_t* prev_action;       /* [b][n] discrete (-1 at step 0) */
  int32_t* action;
  float* prev_action_f;       /* [b][n][A] continuous (0 at step 0) */
  float* action_f;
  float* old_logp;            /* [b][n] (continuous [b][n][A]) */
  float* mb_returns;          /* [b][n] */
  float* old_values;          /* [b][n][B] */
  uint8_t* dones;             /* [b][n] */
  int32_t* mb_lens;           /* [b] */
  float* rs_part;             /* workspace >= 64 * (S + 2) floats */
  float* rs_m;                /* [S + 1] masked mean of swr over the valid steps */
} XtrlBatchDesc;

int xtrl_minibatch_gather(const XtrlBatchDesc* desc, void* stream);
/* RSNorm running update with a batch mean m (xtrl.py:602-610): mean += (m - mean) / t;
 * var = (t - 1) / t * (var + (m - mean_old)^2 / t) */
int xtrl_rsnorm_update(float* mean, float* var, const float* m, int D, int t, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused PPO / critic / world-model / done loss   (xtrl.py:398-477 losses, :939-978 combination)
 * ------------------------------------------------------------------------------------------- */
typedef struct XtrlLossDesc {
  int b, n, A, B, S1;     /* S1 = state_dim + 1 */
  int continuous, squash, hl_reduction_mean;
  float eps_clip, value_clip, entropy_weight, w_actor, w_critic, w_autoreg, lo, hi, sigma;
  /* inputs */
  const float* raw_actions;   /* [b][n][A or 2A] */
  const float* values;        /* [b][n][B] */
  const float* pred_raw;      /* [b][n][2 S1]  to_pred output (interleaved mean / log-var) */
  const float* done_logit;    /* [b][n] */
  const int32_t* actions;     /* [b][n] discrete */
  const float* actions_f;     /* [b][n][A] continuous */
  const float* old_logp;      /* [b][n] (continuous [b][n][A]) */
  const float* returns;       /* [b][n] */
  const float* old_values;    /* [b][n][B] */
  const uint8_t* dones;       /* [b][n] */
  const int32_t* lens;        /* [b] */
  const float* real;          /* [b][n][S1] normalised states-with-rewards */
  const float* support;       /* [B + 1] HL-Gauss bin edges (torch.linspace, host-computed) */
  const float* centers;       /* [B]     bin centres */
  /* workspace + outputs */
  float* tok;                 /* [b][n][XTRL_LOSS_TOK] per-token scratch */
  float* stats;               /* [XTRL_LOSS_STATS] scalars, see XTRL_LS_* */
  /* gradients (backward) */
  float* d_raw_actions; float* d_values; float* d_pred_raw; float* d_done_logit;
} XtrlLossDesc;

#define XTRL_LOSS_TOK 30       /* 11 per-token terms (+1 pad) + 18 floats: per-block partial sums (doubles) */
#define XTRL_LOSS_STATS 32
/* stats[] slots */
#define XTRL_LS_LOSS 0         /* total loss (xtrl.py:975-978) */
#define XTRL_LS_ACTOR 1        /* actor_loss.mean() over all b*n (log, xtrl.py:997) */
#define XTRL_LS_CRITIC 2       /* critic_loss.mean() over all b*n */
#define XTRL_LS_AUTOREG 3      /* world_model_loss.mean() over the masked elements */
#define XTRL_LS_DONE 4         /* pred_done_loss.mean() over the mask */
#define XTRL_LS_ADV_MEAN 5
#define XTRL_LS_ADV_DEN 6      /* sqrt(clamp(unbiased var, 1e-5)) */
#define XTRL_LS_L 7            /* HL-Gauss CE(values, returns), mean reduction */
#define XTRL_LS_LC 8           /* HL-Gauss CE(values, clamp(returns)), mean reduction */
#define XTRL_LS_NMASK 9
#define XTRL_LS_NWM 10         /* number of world-model loss elements */
#define XTRL_LS_KCRIT 11       /* masked tokens whose critic loss is not clipped to 0 */
#define XTRL_LS_DL 12          /* d loss / d L   (per unit upstream gradient) */
#define XTRL_LS_DLC 13         /* d loss / d Lc */

int xtrl_loss_fwd(const XtrlLossDesc* desc, void* stream);
int xtrl_loss_bwd(const XtrlLossDesc* desc, float grad_scale, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Optimiser path over one flat fp32 parameter buffer  (xtrl.py:987-992, 747-753)
 * ------------------------------------------------------------------------------------------- */
/* clip_grad_norm_ (xtrl.py:987): ws = 512 doubles of scratch; out[0] = total L2 norm,
 * out[1] = min(max_norm / (norm + 1e-6), 1) */
int xtrl_grad_norm(const float* g, int64_t n, double* ws, float max_norm, float* out, void* stream);
/* AdoptAtan2 step (xtrl.py:749, 991) on n parameters split into n_seg tensors
 * (seg_start[n_seg + 1] device offsets) and processed as n_chunks contiguous pieces
 * (chunks[n_chunks][3] = start, end, tensor index; one workgroup each, so the per-tensor cautious
 * mean needs one atomic per workgroup); g is scaled in place by clip[1] (clip may be NULL);
 * seg_ws = n_seg ints of scratch; first_step != 0 initialises m = 0, v = g^2, p_init = p. */
int xtrl_adopt_atan2(float* p, float* g, float* m, float* v, float* p_init, int64_t n, const int64_t* chunks,
                     int n_chunks, const int64_t* seg_start, int n_seg, int* seg_ws, const float* clip, float lr,
                     float init_lr, float beta1, float beta2, float a, float b, float weight_decay, float regen_rate,
                     float cautious, int first_step, void* stream);
/* ema = lerp(ema, p, 1 - decay) */
int xtrl_ema_lerp(float* ema, const float* p, int64_t n, float weight, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Synthetic vectorised Sim (stands in for gym LunarLander, which is not available)
 * ------------------------------------------------------------------------------------------- */
/* host-side evaluation of the device random streams (csrc/philox.h), e.g. the reward-dropout coin */
float xtrl_rng_uniform(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t, uint32_t field, uint32_t sub);
float xtrl_rng_normal(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t, uint32_t field, uint32_t sub);

int xtrl_sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update, const int32_t* episode_of_slot,
                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fractal encoder body (x_transformers_rl/fractal_rl.py FractalEncoder :137-346 and
 * FractalWorldModelActorCritic.forward :549-619).  The reference composes x-transformers modules
 * in Python; its matrix work maps to xtrl_gemm_f32 (Linear, act 3 = the ReLU of
 * final_aggregation :235-239) and xtrl_attn_fwd_tokens (Attention, bidirectional: the
 * FractalProcessingBlock self-attention :127-129); the rest is these row kernels.  The host side
 * (xtrl_amd/fractal.py) mirrors the reference modules and their state_dict names.
 * ------------------------------------------------------------------------------------------- */
/* attention forward on token-major q/k/v (rows b*n + i, head h at columns h*dh, one row stride);
 * causal = 0: key-padding mask only (keys j < lens[b]) */
int xtrl_attn_fwd_tokens(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                         const int32_t* lens, float* o, int ldo, float* lse, int b, int H, int n, int dh, float scale,
                         int causal, void* stream);
/* y = x + v (v broadcast over rows; x NULL: y = v): level embedding add, fractal_rl.py:312-314 */
int xtrl_rows_add(const float* x, int ldx, const float* v, float* y, int ldy, int M, int D, void* stream);
/* y = LayerNorm(x + r) * gamma + beta (nn.LayerNorm, eps): post-norm blocks fractal_rl.py:127-136.
 * Residual row m / r_rep (r_rep = n broadcasts one row per sequence: the cross-attention read of
 * the one-token global state, whose softmax over a single key is exactly 1). r may be NULL. */
int xtrl_add_layernorm(const float* x, int ldx, const float* r, int ldr, int r_rep, const float* gamma,
                       const float* beta, float* y, int ldy, int M, int D, float eps, void* stream);
/* y[b, :] = mean over the n rows of sequence b (einops reduce 'b n d -> b d', fractal_rl.py:321, :338) */
int xtrl_seq_mean(const float* x, int ldx, int B, int n, int D, float* y, int ldy, void* stream);
/* SafeEmbedding (x_transformers_rl.py:181-195): y[m] = actions[m] >= 0 ? W[actions[m]] : 0 */
int xtrl_safe_embed(const int32_t* actions, int M, const float* W, int D, float* y, int ldy, void* stream);
/* Continuous(raw).mean_variance (x_transformers_rl.py:224-241) -> mean_var [2][M][P];
 * optional done = sigmoid(done_logit) (to_pred_done, fractal_rl.py:402-406) */
int xtrl_wm_post(const float* raw, int ldr, int M, int P, float* mean_var, const float* done_logit, int ldd,
                 float* done, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* XTRL_HIP_H */
