// Rollout: one policy timestep for E concurrent episodes, entirely on device.
//
// Replaces the batch-1, host-synchronised body of the reference rollout loop
// (x_transformers_rl.py:1250-1341) with a vectorised step over the LIVE episodes only:
//
//   k_compact      lists the live episodes (alive != 0) in slot order: row r of every per-step
//                  buffer is episode slot live_rows[t & 1][r], r < live_count[t & 1]
//   k_embed        RSNorm eval of [state, prev_reward]
//                  (xtrl.py:1254-1259, 591), project_in + action embedding + reward embedding
//                  (xtrl.py:492-503), to_state_embed, latent embedding; writes the raw state into
//                  the trajectory (Memory.state, xtrl.py:1315)
//   per layer      [LN -> q|k|v|gate|mix] dgemm (LayerNorm in the GEMM prologue)
//                  k_attn_decode: value-residual mix, rotary, KV append at t, softmax(q k^T) v
//                  over positions 0..t, value gate        (x-transformers Attention, cached)
//                  out-proj dgemm + residual, [LN -> FF1 GELU] dgemm, FF2 dgemm + residual
//                  (the last layer's FF2 writes the final-norm input straight into ac_in[:, 0:d])
//   heads          [final LN -> actor|critic hidden SiLU] dgemm; the last Linear layers as one
//                  block-diagonal dgemm: actor logits to the row buffer, critic logits straight
//                  into traj_values[slot][t] (row scatter)
//   k_sample       softmax -> Categorical ->
//                  inverse-CDF sample on Philox uniforms, log_prob (xtrl.py:1280-1289; torch
//                  Categorical(probs) semantics), then the synthetic LunarLander-shaped Sim step
//                  (philox.h): reward, termination, next state, alive mask, episode length,
//                  cumulative reward (xtrl.py:1297-1351)
// 5 L + 5 launches per step (C3: 25; round 1: 33), and terminated episodes cost nothing.
//
// Layouts in HBM: per-step activations are [live row][.] row-major; KV caches [E][H][Tmax][dh]
// (per episode slot) so one (episode, head) streams a contiguous Tmax*dh block; trajectories
// [E][Tmax][.] so the learner reads whole episodes contiguously.
#include <chrono>
#include "dgemm_body.h"
#include "kernels.h"
#include "x6.h"
#include "philox.h"

namespace xtrl {

namespace {

constexpr float F32_EPS = 1.1920928955078125e-07f;

__device__ __forceinline__ float f4c(const float4& v, int k) {
  return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

__device__ __forceinline__ const int32_t* rows_of(const XtrlDecodeDesc& D, int t) { return D.live_rows + (t & 1) * D.E; }

// The alive byte of an episode slot: 0 dead, 1 live, 2 truncation-bootstrap step pending (host envs),
// ALIVE_END + (t & 1): a Sim episode the row-resident step ended at step t.  That step's workgroups
// rank the live slots while others already step theirs, so the step never turns a slot it ranks
// from live to dead: a row it ends goes 1 -> ALIVE_END + (t & 1), live for step t, dead for step
// t + 1 (whose compaction clears it to 0 — before step t + 2, where the parity would repeat).  One
// byte, one store: the ranking needs no ordering between stores of different arrays.
constexpr uint8_t ALIVE_END = 3;
__device__ __forceinline__ bool live_at(uint8_t al, int t) {
  return al == 1 || al == 2 || al == (uint8_t)(ALIVE_END + (t & 1));
}
__device__ __forceinline__ bool ended_before(uint8_t al, int t) { return al == (uint8_t)(ALIVE_END + ((t + 1) & 1)); }

// ---------------------------------------------------------------------------------------------
// live-row compaction: one workgroup lists the episode slots with alive != 0 in slot order
// (live_rows[t & 1][0 .. n-1], live_count[t & 1] = n) — deterministic, one launch
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_compact(const XtrlDecodeDesc D, int t) {
  __shared__ int wsum[16];
  __shared__ int base_sh;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int32_t* rows = D.live_rows + (t & 1) * D.E;
  if (tid == 0) base_sh = 0;
  for (int e0 = 0; e0 < D.E; e0 += 1024) {
    const int e = e0 + tid;
    const uint8_t a8 = e < D.E ? D.alive[e] : 0;
    const bool al = live_at(a8, t);
    if (ended_before(a8, t)) D.alive[e] = 0;
    const uint64_t bal = __ballot(al);
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base_sh;
    for (int i = 0; i < w; ++i) off += wsum[i];
    if (al) rows[off + __popcll(bal & ((1ull << lane) - 1ull))] = e;
    __syncthreads();
    if (tid == 0) {
      int tot = 0;
      for (int i = 0; i < 16; ++i) tot += wsum[i];
      base_sh += tot;
    }
    __syncthreads();
  }
  if (tid == 0) D.live_count[t & 1] = base_sh;
}

// ---------------------------------------------------------------------------------------------
// embeddings of the live rows: one wave per row, 16 rows per 1024-thread workgroup; project_in and
// to_state_embed weights staged once per workgroup in LDS as [s][column] images.  The kernel is
// latency bound, so it is written as four batches of independent global loads (live count ->
// slot -> state / previous action -> action-embedding rows), nothing loaded inside a loop
// ---------------------------------------------------------------------------------------------
constexpr int EMB_ROWS = 16;
constexpr int EMB_LDS_FLOATS = 8192;   // 2 d S <= 8192 (C3: 4096); larger: weights read from global
constexpr int EMB_MAX_E = 8192;        // E up to this: the compaction runs inside k_embed (CMP)
constexpr int EMB_AREG = 8;            // discrete A up to this: action embeddings held in registers
// CMP: every workgroup ranks the live slots itself (one load of the alive bytes, ballots, an LDS
// scan — the same slot order as k_compact) and stores its own rows' entries of live_rows[t & 1];
// workgroup 0 stores live_count[t & 1].  No separate compaction launch, and the embedding's
// first dependent load (the live count) is gone.  Otherwise k_compact ran before.
template <int NC, bool CMP>   // columns per lane: lane + 64 k, k < NC (d <= 64 NC)
__global__ __launch_bounds__(1024) void k_embed(const XtrlDecodeDesc D, int t, const float* g_ln0) {
  __shared__ float wsh[EMB_LDS_FLOATS];
  __shared__ float ns_sh[EMB_ROWS][64];
  __shared__ int rows_sh[CMP ? EMB_MAX_E : 1];
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int S = D.S, d = D.d, dS = d * S;
  const bool staged = 2 * dS <= EMB_LDS_FLOATS;
  // weights (independent of the rows): two float4 per thread per matrix cover 2 d S <= 8192
  float4 wv[2][2];
  if (staged) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = min(tid + 1024 * u, (dS >> 2) - 1);
      wv[0][u] = reinterpret_cast<const float4*>(D.w_pin)[f];
      wv[1][u] = reinterpret_cast<const float4*>(D.w_se)[f];
    }
  }
  int n_live = 0;   // (CMP: the live count, the same in every thread)
  if constexpr (CMP) {   // rank the live slots (live_at) in slot order
    uint8_t alv[EMB_MAX_E / 1024];
#pragma unroll
    for (int c = 0; c < EMB_MAX_E / 1024; ++c) {
      const int e = min(1024 * c + tid, D.E - 1);
      alv[c] = D.alive[e];
    }
    int base = 0;
#pragma unroll
    for (int c = 0; c < EMB_MAX_E / 1024; ++c) {
      if (1024 * c >= D.E) break;   // (uniform)
      const int e = 1024 * c + tid;
      const bool al = e < D.E && live_at(alv[c], t);
      if (blockIdx.x == 0 && e < D.E && ended_before(alv[c], t)) D.alive[e] = 0;
      const uint64_t bal = __ballot(al);
      if (lane == 0) wsum[w] = __popcll(bal);
      __syncthreads();
      int off = base, tot = 0;
      for (int i = 0; i < 16; ++i) {
        off += i < w ? wsum[i] : 0;
        tot += wsum[i];
      }
      if (al) rows_sh[off + __popcll(bal & ((1ull << lane) - 1ull))] = e;
      base += tot;
      __syncthreads();
    }
    const int r = blockIdx.x * EMB_ROWS + tid;
    if (tid < EMB_ROWS && r < base) D.live_rows[(t & 1) * D.E + r] = rows_sh[r];
    if (blockIdx.x == 0 && tid == 0) D.live_count[t & 1] = base;
    n_live = base;
  }
  // per-column constants of this lane
  float remb[NC], bse[NC], bpin[NC], gln[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = min(lane + 64 * k, d - 1);
    remb[k] = D.reward_embed[c];
    bse[k] = D.b_se[c];
    bpin[k] = D.b_pin ? D.b_pin[c] : 0.f;
    gln[k] = g_ln0 ? g_ln0[c] : 0.f;
  }
  // discrete actions, A <= EMB_AREG: every action's embedding columns of this lane, loaded up front
  // (the row's action then selects among registers: no dependent load after the previous action)
  constexpr int AR = NC <= 4 ? EMB_AREG : 1;   // (d > 256: the table stays in memory, registers are short)
  const bool areg = NC <= 4 && !D.continuous && D.A <= EMB_AREG;
  float emb_a[AR][NC];
  if (areg) {
#pragma unroll
    for (int i = 0; i < AR; ++i)
#pragma unroll
      for (int k = 0; k < NC; ++k) emb_a[i][k] = D.act_emb[min(i, D.A - 1) * d + min(lane + 64 * k, d - 1)];
  }
  const int n = CMP ? n_live : D.live_count[t & 1];
  const int r0 = blockIdx.x * EMB_ROWS;
  if (r0 >= n) return;   // (whole workgroup)
  if (staged) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = tid + 1024 * u;
      if (f < (dS >> 2)) {   // (c, s) -> [s][c] and [S + s][c]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = 4 * f + i, c = idx / S, sidx = idx - c * S;
          wsh[sidx * d + c] = f4c(wv[0][u], i);
          wsh[(S + sidx) * d + c] = f4c(wv[1][u], i);
        }
      }
    }
  }
  __syncthreads();
  const int r = r0 + w;
  if (r >= n) return;   // wave-uniform
  const int e = CMP ? rows_sh[r] : D.live_rows[(t & 1) * D.E + r];
  float* ns = ns_sh[w];
  // RSNorm eval on the packed [state, prev_reward] vector: (x - mean) / clamp(sqrt(var), eps)
  const float xv = lane < S ? D.state[(int64_t)e * S + lane] : D.prev_reward[e];
  const int a = D.continuous ? 0 : D.prev_action[e];
  float lat[NC];
  if (D.evolutionary && D.lat_embed) {
#pragma unroll
    for (int k = 0; k < NC; ++k) lat[k] = D.lat_embed[(int64_t)e * d + min(lane + 64 * k, d - 1)];
  }
  if (lane <= S) {
    ns[lane] = (xv - D.rs_mean[lane]) / fmaxf(sqrtf(D.rs_var[lane]), D.rs_eps);
    if (lane < S) D.traj_states[((int64_t)e * D.Tmax + t) * S + lane] = xv;
  }
  float act[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = min(lane + 64 * k, d - 1);
    if (D.continuous) {
      float acc = 0.f;
      for (int i = 0; i < D.A; ++i) acc += D.prev_action_f[e * D.A + i] * D.act_emb[c * D.A + i];
      act[k] = acc + D.act_emb_b[c];
    } else if (areg) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < AR; ++i) v = (i == max(a, 0)) ? emb_a[i][k] : v;
      act[k] = v;
    } else {
      act[k] = D.act_emb[max(a, 0) * d + c];
    }
  }
  wave_sync();
  const float nr = ns[S];
  float xo[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = lane + 64 * k;
    xo[k] = 0.f;
    if (c >= d) break;
    float p = 0.f, se = 0.f;
    for (int sidx = 0; sidx < S; ++sidx) {
      const float wp = staged ? wsh[sidx * d + c] : D.w_pin[c * S + sidx];
      const float wsv = staged ? wsh[(S + sidx) * d + c] : D.w_se[c * S + sidx];
      p += ns[sidx] * wp;
      se += ns[sidx] * wsv;
    }
    p += bpin[k];
    const float ak = D.state_only ? 0.f : ((D.continuous || a >= 0) ? act[k] : 0.f);   // SafeEmbedding: -1 -> 0
    const float rew = (D.no_reward_cond || D.state_only) ? 0.f : nr * remb[k];
    xo[k] = p + (ak + rew);
    D.x[(int64_t)r * d + c] = xo[k];
    D.ac_in[(int64_t)r * D.in_dim + d + c] = se + bse[k];
    if (D.evolutionary && D.lat_embed) D.ac_in[(int64_t)r * D.in_dim + 2 * d + c] = lat[k];
  }
  if (g_ln0 && D.xn) {   // layer 0's pre-attention LayerNorm (two-pass, as the GEMM prologue)
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) sm += lane + 64 * k < d ? xo[k] : 0.f;
    const float mean = D.rms_norm ? 0.f : wave_sum_dpp(sm) / (float)d;
    float qq = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float dl = xo[k] - mean;
      qq += lane + 64 * k < d ? dl * dl : 0.f;
    }
    const float rstd = norm_rstd(wave_sum_dpp(qq), (float)d, D.rms_norm);
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = lane + 64 * k;
      if (c < d) D.xn[(int64_t)r * d + c] = ((xo[k] - mean) * rstd) * gln[k];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// attention decode: one wave per (live row, head), keys 0..t.  Latency bound: the keys are taken in
// chunks of CK, and the first chunk's K rows (one key per lane) and V rows (a key per DH/4 lanes,
// float4 per lane) are loaded in ONE batch right after the row's q|k|v — for t < CK (C3: every
// step) the whole cache read is one memory round trip.  Reductions by DPP.
// ---------------------------------------------------------------------------------------------
// sum over the N consecutive lanes of an aligned group (N = 4, 8 or 16), every lane of the group
// receiving it (DPP: quad xor steps, half-row and row mirrors)
template <int N>
__device__ __forceinline__ float kpi_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  if constexpr (N >= 8) v += dpp_mov<0x141>(v);
  if constexpr (N >= 16) v += dpp_mov<0x140>(v);
  return v;
}

// FUSE: one workgroup per live row (H waves), and the out-projection + residual applied here:
// wave h multiplies its head's output by rows [h DH, (h+1) DH) of W_out^T (prefetched with the
// cache rows: float4 columns 4 lane + 256 j), the H partial rows meet in LDS and are summed in head
// order onto the residual row x[r] — the out-projection GEMM launch of the layer is gone.
// FJ = ceil(d / 256) float4 column groups per lane (FJ = 0: not fused, the output goes to D.att)
// FrPost (fractal body, g1 non-NULL): the fused tail forms the post-norm rows instead —
// out = LN2(LN1(x + attn W_out^T) g1 + b1 + c[r] ) g2 + b2 (nn.LayerNorm, eps), x itself is not
// stored (nothing reads it) and no pre-norm is written
// x-transformers qk norm of the new token's q and k (F.normalize over the head's DH channels, eps
// 1e-12): lane c = lane % DH holds channel c, a head's DH channels on DH aligned lanes
template <int DH>
__device__ __forceinline__ void qk_l2norm(float& q, float& k) {
  float sq = q * q, sk = k * k;
#pragma unroll
  for (int o = DH / 2; o > 0; o >>= 1) {
    sq += __shfl_xor(sq, o, 64);
    sk += __shfl_xor(sk, o, 64);
  }
  q = q / fmaxf(sqrtf(sq), 1e-12f);
  k = k / fmaxf(sqrtf(sk), 1e-12f);
}

// rotary at absolute position t of channel c (< rot_dim; pairs on adjacent lanes), with the xPos scale
// of an input whose last position is t (max_pos = t + 1): q times, k divided by the pair's factor
__device__ __forceinline__ void rotary_row(const XtrlDecodeDesc& D, int t, int c, float& q, float& k) {
  const float f = (float)t * D.inv_freq[c >> 1];
  const float cs = cosf(f), sn = sinf(f);
  const float qp = dpp_mov<0xB1>(q), kp = dpp_mov<0xB1>(k);   // the pair partner (lane ^ 1; DPP, no permute)
  const float sgn = (c & 1) ? 1.f : -1.f;   // rotate_half: (-x2, x1)
  q = q * cs + (sgn * qp) * sn;
  k = k * cs + (sgn * kp) * sn;
  if (D.xpos_base > 0.f) {
    const float rot = (float)D.rot_dim;
    const float xf = powf(((float)(c & ~1) + 0.4f * rot) / (1.4f * rot), (float)(t - (t + 1) / 2) / D.xpos_base);
    q *= xf;
    k *= 1.0f / xf;
  }
}

struct FrPost {
  const float *g1 = nullptr, *b1 = nullptr, *g2 = nullptr, *b2 = nullptr, *c = nullptr;
  int ldc = 0;
  float* out = nullptr;
  float eps = 1e-5f;
};

template <int DH, int FJ>
__global__ __launch_bounds__(FJ > 0 ? 512 : 256) void k_attn_decode(const XtrlDecodeDesc D, const XtrlDecodeLayer Ly, int layer,
                                                      int t, const FrPost fp) {
  constexpr int CK = DH <= 32 ? 128 : 64;          // keys per chunk
  constexpr int KL = CK / 64, F4 = DH / 4;         // keys per lane (scores), float4 per key row
  constexpr int LPK = DH / 4, KPI = 64 / LPK;      // P.V: lanes per key row, keys per load instruction
  constexpr int VU = CK / KPI;                     // V loads per lane per chunk
  extern __shared__ float smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int idx = blockIdx.x * nw + w;
  const int H = D.H, I = H * DH, d = D.d;
  const int r = idx / H, h = idx - r * H;
  constexpr bool FUSE = FJ > 0;
  // the live count and the row's slot in one round trip (live_rows past the count: a stale slot)
  const int n_live = D.live_count[t & 1];
  const int e = rows_of(D, t)[min(r, D.E - 1)];
  if (r >= n_live) return;   // wave-uniform (FUSE: workgroup-uniform)
  // fused out-projection operands: this head's rows of W_out^T and the residual row
  float4 wt[FUSE ? FJ : 1][FUSE ? DH : 1];
  float4 xres[FUSE ? FJ : 1], gff[FUSE ? FJ : 1];   // wave 0: the residual row and FF1's LayerNorm gain
  float4 pg1[FUSE ? FJ : 1], pb1[FUSE ? FJ : 1], pg2[FUSE ? FJ : 1], pb2[FUSE ? FJ : 1], pc[FUSE ? FJ : 1];
  const bool post = fp.g1 != nullptr;
  if constexpr (FUSE) {
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int n = min(4 * lane + 256 * j, d - 4);
#pragma unroll
      for (int c = 0; c < DH; ++c)
        wt[j][c] = *reinterpret_cast<const float4*>(Ly.w_out_t + (int64_t)(h * DH + c) * d + n);
      if (w == 0) {
        xres[j] = *reinterpret_cast<const float4*>(D.x + (int64_t)r * d + n);
        if (post) {
          if constexpr (FJ == 1) {   // (prefetched with the residual row; FJ = 2 loads them in the tail)
            pg1[j] = *reinterpret_cast<const float4*>(fp.g1 + n);
            pb1[j] = *reinterpret_cast<const float4*>(fp.b1 + n);
            pg2[j] = *reinterpret_cast<const float4*>(fp.g2 + n);
            pb2[j] = *reinterpret_cast<const float4*>(fp.b2 + n);
            pc[j] = *reinterpret_cast<const float4*>(fp.c + (int64_t)r * fp.ldc + n);
          }
        } else {
          gff[j] = *reinterpret_cast<const float4*>(Ly.ln_ff + n);
        }
      }
    }
  }
  float* sc = smem + w * (D.Tmax + 3 * DH);   // scores / probabilities [Tmax] | q | k_new | v_new
  float* qs = sc + D.Tmax;
  float* ks = qs + DH;
  float* vs = ks + DH;
  const float* row = D.qkv + (int64_t)r * D.n_qkv;
  const int c = lane % DH, g = lane / DH;
  float q = row[h * DH + c], k = row[I + h * DH + c], v = row[2 * I + h * DH + c];
  float v1v = 0.f, mixv = 0.f, gate4[4] = {0.f, 0.f, 0.f, 0.f};
  // P.V lane roles: key kk = lane % KPI of a load instruction's KPI rows, channel quad cq = lane / KPI
  // (the KPI rows of one instruction are consecutive: 1 KiB contiguous; the reduction over kk stays
  // inside a 16-lane row: DPP steps, no cross-lane permutes)
  const int kk = lane % KPI, cq = lane / KPI;
  if (D.value_residual && layer > 0) {
    v1v = D.v1[(int64_t)r * I + h * DH + c];
    if (D.learned_mix) mixv = row[3 * I + (D.gate_values ? I : 0) + h];
  }
  if (D.gate_values) {
#pragma unroll
    for (int i = 0; i < 4; ++i) gate4[i] = row[3 * I + h * DH + 4 * cq + i];
  }
  // the first chunk of the cache (rows written by earlier steps; rows >= t clamped, masked below)
  const int64_t cache_base = ((int64_t)e * H + h) * D.Tmax * DH;
  const float* Kc = Ly.k_cache + cache_base;
  const float* Vc = Ly.v_cache + cache_base;
  const int tl = max(t - 1, 0);
  float4 kpre[KL][F4], vpre[VU];
#pragma unroll
  for (int u = 0; u < KL; ++u)
#pragma unroll
    for (int i = 0; i < F4; ++i) kpre[u][i] = reinterpret_cast<const float4*>(Kc + (int64_t)min(lane + 64 * u, tl) * DH)[i];
#pragma unroll
  for (int u = 0; u < VU; ++u)
    vpre[u] = *reinterpret_cast<const float4*>(Vc + (int64_t)min(kk + KPI * u, tl) * DH + 4 * cq);
  // value residual (first layer stores its values; later layers lerp toward them)
  if (D.value_residual) {
    if (layer == 0) {
      if (g == 0) D.v1[(int64_t)r * I + h * DH + c] = v;
    } else if (D.learned_mix) {
      v = lerpf_(v, v1v, sigmoidf_(mixv));
    }
  }
  if (D.qk_norm) qk_l2norm<DH>(q, k);
  // rotary (interleaved pairs on the first rot_dim channels); 'zero' mode = position 0 = identity
  if (D.rotary_abs && c < D.rot_dim) rotary_row(D, t, c, q, k);
  if (g == 0) {
    qs[c] = q;
    ks[c] = k;
    vs[c] = v;
    Ly.k_cache[cache_base + (int64_t)t * DH + c] = k;
    Ly.v_cache[cache_base + (int64_t)t * DH + c] = v;
  }
  wave_sync();
  const float scale = D.attn_scale > 0.f ? D.attn_scale : 1.0f / sqrtf((float)DH);
  float qreg[DH];
#pragma unroll
  for (int i = 0; i < DH; ++i) qreg[i] = qs[i];
  // scores, one key per lane; chunk 0 from the prefetched rows
  float mx = -INFINITY;
  for (int j0 = 0; j0 <= t; j0 += CK) {
    float4 kc[KL][F4];
    if (j0 == 0) {
#pragma unroll
      for (int u = 0; u < KL; ++u)
#pragma unroll
        for (int i = 0; i < F4; ++i) kc[u][i] = kpre[u][i];
    } else {
#pragma unroll
      for (int u = 0; u < KL; ++u)
#pragma unroll
        for (int i = 0; i < F4; ++i)
          kc[u][i] = reinterpret_cast<const float4*>(Kc + (int64_t)min(j0 + lane + 64 * u, tl) * DH)[i];
    }
#pragma unroll
    for (int u = 0; u < KL; ++u) {
      const int j = j0 + lane + 64 * u;
      float s = 0.f;
      if (j < t) {
#pragma unroll
        for (int i = 0; i < F4; ++i) {
          s += qreg[4 * i] * kc[u][i].x;
          s += qreg[4 * i + 1] * kc[u][i].y;
          s += qreg[4 * i + 2] * kc[u][i].z;
          s += qreg[4 * i + 3] * kc[u][i].w;
        }
      } else {
#pragma unroll
        for (int i = 0; i < DH; ++i) s += qreg[i] * ks[i];
      }
      s *= scale;
      if (j <= t) {
        sc[j] = s;
        mx = fmaxf(mx, s);
      }
    }
  }
  mx = wave_max_dpp(mx);
  float sum = 0.f;
  for (int j = lane; j <= t; j += 64) {
    const float p = expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = wave_sum_dpp(sum);
  wave_sync();
  // P.V (unnormalised probabilities; one division at the end)
  const float4 vnew = make_float4(vs[4 * cq], vs[4 * cq + 1], vs[4 * cq + 2], vs[4 * cq + 3]);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j0 = 0; j0 <= t; j0 += CK) {
    float4 vc[VU];
    if (j0 == 0) {
#pragma unroll
      for (int u = 0; u < VU; ++u) vc[u] = vpre[u];
    } else {
#pragma unroll
      for (int u = 0; u < VU; ++u)
        vc[u] = *reinterpret_cast<const float4*>(Vc + (int64_t)min(j0 + kk + KPI * u, tl) * DH + 4 * cq);
    }
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const int j = j0 + kk + KPI * u;
      if (j <= t) {
        const float p = sc[j];
        const float4 v4 = j < t ? vc[u] : vnew;
        acc.x += p * v4.x;
        acc.y += p * v4.y;
        acc.z += p * v4.z;
        acc.w += p * v4.w;
      }
    }
  }
  acc.x = kpi_sum<KPI>(acc.x);
  acc.y = kpi_sum<KPI>(acc.y);
  acc.z = kpi_sum<KPI>(acc.z);
  acc.w = kpi_sum<KPI>(acc.w);
  if (kk == 0) {
    float o4[4] = {acc.x / sum, acc.y / sum, acc.z / sum, acc.w / sum};
    if (D.gate_values) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o4[i] *= sigmoidf_(gate4[i]);
    }
    if constexpr (FUSE) *reinterpret_cast<float4*>(qs + 4 * cq) = make_float4(o4[0], o4[1], o4[2], o4[3]);
    else *reinterpret_cast<float4*>(D.att + (int64_t)r * I + h * DH + 4 * cq) = make_float4(o4[0], o4[1], o4[2], o4[3]);
  }
  if constexpr (FUSE) {
    wave_sync();
    float* part = smem + nw * (D.Tmax + 3 * DH);   // [H][d] partial output rows
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int n = 4 * lane + 256 * j;
      float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int c = 0; c < DH; ++c) {
        const float o = qs[c];
        y.x += o * wt[j][c].x;
        y.y += o * wt[j][c].y;
        y.z += o * wt[j][c].z;
        y.w += o * wt[j][c].w;
      }
      if (n < d) *reinterpret_cast<float4*>(part + h * d + n) = y;
    }
    __syncthreads();
    if (w == 0) {   // the row: residual + the head partials in head order; then FF1's LayerNorm
      float4 y[FJ];
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int n = 4 * lane + 256 * j;
        y[j] = xres[j];
        if (n < d) {
          for (int hh = 0; hh < H; ++hh) {
            const float4 p = *reinterpret_cast<const float4*>(part + hh * d + n);
            y[j].x += p.x;
            y[j].y += p.y;
            y[j].z += p.z;
            y[j].w += p.w;
          }
          if (!post) *reinterpret_cast<float4*>(D.x + (int64_t)r * d + n) = y[j];
          sm += (y[j].x + y[j].y) + (y[j].z + y[j].w);
        }
      }
      if (post) {   // LN1 (affine), + the cross-attention row, LN2 (affine) -> out
        if constexpr (FJ > 1) {
#pragma unroll
          for (int j = 0; j < FJ; ++j) {
            const int n = min(4 * lane + 256 * j, d - 4);
            pg1[j] = *reinterpret_cast<const float4*>(fp.g1 + n);
            pb1[j] = *reinterpret_cast<const float4*>(fp.b1 + n);
            pg2[j] = *reinterpret_cast<const float4*>(fp.g2 + n);
            pb2[j] = *reinterpret_cast<const float4*>(fp.b2 + n);
            pc[j] = *reinterpret_cast<const float4*>(fp.c + (int64_t)r * fp.ldc + n);
          }
        }
        auto affine_ln = [&](float4 (&v)[FJ], float s1, const float4 (&g)[FJ], const float4 (&b)[FJ]) {
          const float mean = wave_sum_dpp(s1) / (float)d;
          float qq = 0.f;
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            if (4 * lane + 256 * j < d) {
              const float4 dl = make_float4(v[j].x - mean, v[j].y - mean, v[j].z - mean, v[j].w - mean);
              qq += (dl.x * dl.x + dl.y * dl.y) + (dl.z * dl.z + dl.w * dl.w);
            }
          const float rstd = 1.0f / sqrtf(wave_sum_dpp(qq) / (float)d + fp.eps);
#pragma unroll
          for (int j = 0; j < FJ; ++j)
            v[j] = make_float4((v[j].x - mean) * rstd * g[j].x + b[j].x, (v[j].y - mean) * rstd * g[j].y + b[j].y,
                               (v[j].z - mean) * rstd * g[j].z + b[j].z, (v[j].w - mean) * rstd * g[j].w + b[j].w);
        };
        affine_ln(y, sm, pg1, pb1);
        float s2 = 0.f;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          y[j] = make_float4(y[j].x + pc[j].x, y[j].y + pc[j].y, y[j].z + pc[j].z, y[j].w + pc[j].w);
          if (4 * lane + 256 * j < d) s2 += (y[j].x + y[j].y) + (y[j].z + y[j].w);
        }
        affine_ln(y, s2, pg2, pb2);
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          const int n = 4 * lane + 256 * j;
          if (n < d) *reinterpret_cast<float4*>(fp.out + (int64_t)r * d + n) = y[j];
        }
      } else if (D.xn) {
        const float mean = D.rms_norm ? 0.f : wave_sum_dpp(sm) / (float)d;
        float qq = 0.f;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          if (4 * lane + 256 * j < d) {
            const float4 dl = make_float4(y[j].x - mean, y[j].y - mean, y[j].z - mean, y[j].w - mean);
            qq += (dl.x * dl.x + dl.y * dl.y) + (dl.z * dl.z + dl.w * dl.w);
          }
        }
        const float rstd = norm_rstd(wave_sum_dpp(qq), (float)d, D.rms_norm);
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          const int n = 4 * lane + 256 * j;
          if (n < d)
            *reinterpret_cast<float4*>(D.xn + (int64_t)r * d + n) =
                make_float4(((y[j].x - mean) * rstd) * gff[j].x, ((y[j].y - mean) * rstd) * gff[j].y,
                            ((y[j].z - mean) * rstd) * gff[j].z, ((y[j].w - mean) * rstd) * gff[j].w);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// actor logits + sampling + device Sim step (SAMPLE_L lanes per live row)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float reward_factor(int a) { return (float)(1.0 + 0.1 * (double)a); }

// SAMPLE_L lanes per row (a wave holds whole rows).  The row's lanes stage its logits in LDS and
// draw its random numbers in parallel (none depends on the action): the next state's S normals
// (lane i), the sampling uniform (lane 0), the Sim's reward normal (lane 1) and termination word
// (lane 2); lane 0 then samples the action and finishes the Sim step.
constexpr int SAMPLE_L = 8;

// per-row inputs of the sampling / Sim step, loaded in one batch
struct SampleIn {
  XtrlRngState R;
  int al;
  uint32_t ep, slot;
  double cum;
};
__device__ __forceinline__ SampleIn sample_load(const XtrlDecodeDesc& D, int e) {
  SampleIn in;
  in.R = *D.rng;
  in.al = D.alive[e];   // (every lane of the row reads alive before lane 0 clears it)
  in.ep = D.sim_mode >= 0 ? (uint32_t)D.episode_of_slot[e] : 0u;
  in.slot = D.slot_of_row ? (uint32_t)D.slot_of_row[e] : 0u;
  in.cum = D.cum_reward[e];
  return in;
}

// the sample and the Sim step of one live row (slot e) by its SAMPLE_L lanes (sub = lane of the
// row's aligned group, every lane of the group active); lg = the row's actor outputs in LDS.
// row_step: the row-resident step, whose workgroups rank the live rows while others already sample —
// a truncation-bootstrap row (alive 2) keeps alive = 2 (the next k_env_feedback clears it) and a Sim
// row ending here is marked ALIVE_END + (t & 1), never 0 (live_at)
__device__ __forceinline__ void sample_row(const XtrlDecodeDesc& D, int t, int e, int sub, const float* lg,
                                           const SampleIn& in, bool row_step = false) {
  const XtrlRngState& R = in.R;
  const int al = in.al;
  const uint32_t ep = in.ep;
  const uint32_t slot = D.slot_of_row ? in.slot : R.slot_offset + (uint32_t)e;
  const double cum = in.cum;
  const int A = D.A;
  // random numbers of the step, spread over the row's lanes
  float u = 0.f, zr = 0.f;
  uint32_t tw = 0u;
  if (sub == 0 && !D.continuous) u = rng_uniform(R.seed, R.update, slot, t, FIELD_SAMPLE, 0);
  if (D.sim_mode >= 0) {
    if (sub == 1) zr = rng_normal(R.seed, R.update, ep, t, FIELD_REWARD, 0);
    if (sub == 2) tw = rng_u32(R.seed, R.update, ep, t, FIELD_TERM, 0);
    if (al != 2)
      for (int i = sub; i < D.S; i += SAMPLE_L)
        D.state[(int64_t)e * D.S + i] = rng_normal(R.seed, R.update, ep, t + 1, FIELD_STATE, i);
  }
  const int base = (threadIdx.x & 63) & ~(SAMPLE_L - 1);
  zr = __shfl(zr, base + 1, 64);
  tw = __shfl(tw, base + 2, 64);
  if (sub != 0) return;
  if (al == 2) {   // truncation-bootstrap step of a host env: its value logits are all it needed
    if (!row_step) D.alive[e] = 0;
    return;
  }
  int a = 0;
  if (!D.continuous) {
    // softmax (xtrl.py:203), Categorical(probs) re-normalisation, inverse CDF on the supplied
    // uniform; probabilities recomputed on the fly (no per-thread array)
    float mx = -INFINITY;
    for (int i = 0; i < A; ++i) mx = fmaxf(mx, lg[i]);
    float s = 0.f;
    for (int i = 0; i < A; ++i) s += expf(lg[i] - mx);
    float s2 = 0.f;
    for (int i = 0; i < A; ++i) s2 += expf(lg[i] - mx) / s;
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
    if (D.act_host) static_cast<int32_t*>(D.act_host)[e] = a;
  } else {
    for (int i = 0; i < A; ++i) {
      const float mean = lg[2 * i], lv = lg[2 * i + 1];
      const float var = expf(tanhf(lv / 3.f) * 3.f);
      const float sd = sqrtf(fmaxf(var, 1e-5f));
      const float z = rng_normal(R.seed, R.update, slot, t, FIELD_SAMPLE, i);
      float sv = mean + sd * z;
      if (D.squash) sv = tanhf(sv);
      float lp = -((sv - mean) * (sv - mean)) / (2.f * sd * sd) - logf(sd) - 0.91893853320467274f;
      if (D.squash) lp -= logf(fmaxf(1.f - sv * sv, 1e-20f));
      if (D.has_clamp) sv = fminf(fmaxf(sv, D.clamp_lo), D.clamp_hi);
      D.traj_actions_f[((int64_t)e * D.Tmax + t) * A + i] = sv;
      D.traj_logp[((int64_t)e * D.Tmax + t) * A + i] = lp;
      D.prev_action_f[e * A + i] = sv;
      if (D.act_host) static_cast<float*>(D.act_host)[e * A + i] = sv;
    }
  }
  if (D.sim_mode >= 0) {   // the synthetic Sim's step (reward, termination, bookkeeping)
    const float reward = (D.sim_mode == 1 && !D.continuous) ? zr * reward_factor(a) : zr;
    const bool term = D.sim_mode == 1 && D.hazard_log2 > 0 && (tw & ((1u << D.hazard_log2) - 1u)) == 0u;
    D.traj_rewards[(int64_t)e * D.Tmax + t] = reward;
    D.traj_bounds[(int64_t)e * D.Tmax + t] = term ? 1 : 0;
    D.prev_reward[e] = reward;
    D.cum_reward[e] = cum + (double)reward;
    D.lens[e] = t + 1;
    if (term || t + 1 >= D.Tmax) D.alive[e] = row_step ? (uint8_t)(ALIVE_END + (t & 1)) : (uint8_t)0;
  }
}

// SAMPLE_L lanes per row (a wave holds whole rows).  The row's lanes stage its logits in LDS and
// draw its random numbers in parallel (none depends on the action): the next state's S normals
// (lane i), the sampling uniform (lane 0), the Sim's reward normal (lane 1) and termination word
// (lane 2); lane 0 then samples the action and finishes the Sim step.  (Used where the head
// projection and the sampling are not fused: n_act > 64.)
__global__ __launch_bounds__(256) void k_sample(const XtrlDecodeDesc D, int t) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = gid / SAMPLE_L, sub = gid % SAMPLE_L;
  if (r >= D.live_count[t & 1]) return;   // (whole rows: SAMPLE_L divides the wave)
  const int e = rows_of(D, t)[r];
  const SampleIn in = sample_load(D, e);
  const int n_act = D.continuous ? 2 * D.A : D.A;
  __shared__ float lg_sh[256 / SAMPLE_L][64];
  float* lg = lg_sh[threadIdx.x / SAMPLE_L];
  for (int o = sub; o < n_act; o += SAMPLE_L) lg[o] = D.logits[(int64_t)r * n_act + o];
  wave_sync();
  sample_row(D, t, e, sub, lg, in);
}

// the heads' last projection (block-diagonal [actor | critic], 16-row panels) with the sampling of
// its rows fused: the column-block-0 workgroups hold every actor output of their 16 rows (n_act <=
// 64), keep them in LDS and run sample_row for each row (SAMPLE_L lanes per row, the per-row
// inputs prefetched with the GEMM operands) — no sampling launch, no logits round trip
struct SampleHook {
  const XtrlDecodeDesc& D;
  int t, n_act;
  bool on;
  float (*lg)[64];
  int row, sub, e;
  SampleIn in;
  // the row's slot first (its load lands with the GEMM operands), the loads that depend on it
  // once they have landed (in flight during the MFMA loop)
  __device__ __forceinline__ void prefetch(int m0, int M) {
    row = threadIdx.x / SAMPLE_L;
    sub = threadIdx.x % SAMPLE_L;
    if (on && row < 16) e = rows_of(D, t)[min(m0 + row, M - 1)];
  }
  __device__ __forceinline__ void landed() {
    if (on && row < 16) in = sample_load(D, e);
  }
  __device__ __forceinline__ void value(int r, int n, float v) {
    if (on && n < n_act) lg[r][n] = v;
  }
  __device__ __forceinline__ void finish(int m0, int M) {
    if (!on) return;   // (workgroup-uniform)
    __syncthreads();
    if (row < 16 && m0 + row < M) sample_row(D, t, e, sub, lg[row], in);
  }
};

template <int KS>
__global__ __launch_bounds__(256) void k_heads_sample(const DGemmArgs a, const XtrlDecodeDesc D, int t) {
  extern __shared__ float As[];
  __shared__ float lg_sh[16][64];
  SampleHook hook{D, t, D.continuous ? 2 * D.A : D.A, blockIdx.x == 0, lg_sh};
  dgemm_body<1, 1, KS, EPI_NONE, false, false>(a, As, hook);
}

// host env results of step t (xtrl.py:1297-1336): the memory stores is_boundary = terminated;
// done = terminated | truncated ends the episode; a truncated (not terminated) episode with
// `bootstrap` stays for one more decode step (alive = 2) whose critic logits land in the padding
// slot traj_values[e][t + 1] — the value of the next state the reference computes at :1323-1336.
// (al: the row's alive byte as loaded by the caller; copy_state false: the caller copies the state)
__device__ __forceinline__ void env_feedback_row(const XtrlDecodeDesc& D, int e, uint8_t al, int t,
                                                 const float* next_state, const float* reward,
                                                 const uint8_t* terminated, const uint8_t* truncated, int t_limit,
                                                 int bootstrap, bool copy_state = true) {
  if (al == 2) {   // its bootstrap step ran (the row-resident step leaves the flag to this kernel)
    D.alive[e] = 0;
    return;
  }
  if (al != 1) return;
  const bool term = terminated[e] != 0, trunc = truncated && truncated[e] != 0;
  D.traj_rewards[(int64_t)e * D.Tmax + t] = reward[e];
  D.traj_bounds[(int64_t)e * D.Tmax + t] = term ? 1 : 0;
  D.prev_reward[e] = reward[e];
  D.cum_reward[e] += (double)reward[e];
  D.lens[e] = t + 1;
  if (copy_state)
    for (int i = 0; i < D.S; ++i) D.state[(int64_t)e * D.S + i] = next_state[(int64_t)e * D.S + i];
  // the bootstrap is taken on any truncated, not terminated step — the last allowed step included
  // (an env TimeLimit equal to max_timesteps: the engine holds Tmax = max_timesteps + 1 positions)
  if (term) D.alive[e] = 0;
  else if (trunc && bootstrap && t + 1 < D.Tmax) D.alive[e] = 2;
  else if (trunc || t + 1 >= t_limit) D.alive[e] = 0;
}
__global__ void k_env_feedback(const XtrlDecodeDesc D, int t, const float* next_state, const float* reward,
                               const uint8_t* terminated, const uint8_t* truncated, int t_limit, int bootstrap) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < D.E) env_feedback_row(D, e, D.alive[e], t, next_state, reward, terminated, truncated, t_limit, bootstrap);
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
  if (D.act_host) {   // (the host-side copy of the actions starts as the device one)
    if (D.continuous)
      for (int i = 0; i < D.A; ++i) static_cast<float*>(D.act_host)[e * D.A + i] = 0.f;
    else
      static_cast<int32_t*>(D.act_host)[e] = -1;
  }
  D.prev_reward[e] = 0.f;
  D.alive[e] = 1;
  D.lens[e] = 0;
  D.cum_reward[e] = 0.0;
  // the fused feed-forward's panel arrival counters (every launch leaves them zero; reset here so an
  // interrupted rollout cannot leave one behind)
  if (D.mlp_cnt && e < (D.E + 15) / 16) D.mlp_cnt[e] = 0u;
}

__global__ void k_sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update, const int32_t* ep_of_slot) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  for (int i = 0; i < S; ++i) state[(int64_t)e * S + i] = rng_normal(seed, update, (uint32_t)ep_of_slot[e], 0, FIELD_STATE, i);
}

// fractal body: running mean of a level's outputs over this episode's steps 0..t (one thread per
// element of the live rows); sums[slot] accumulates in step order, restarting at t = 0
__global__ __launch_bounds__(256) void k_copy_rows(const float* src, int lds, float* dst, int ldd, int M, int D) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(i / D), c = (int)(i - (int64_t)r * D);
  if (r < M) dst[(int64_t)r * ldd + c] = src[(int64_t)r * lds + c];
}

// fractal body, the post-norm rows of one level (wave per live row, the row in registers, nn.LayerNorm
// as k_add_layernorm: two-pass variance, eps): x2 = LN2(LN1(x + o) + c) with c the row's
// cross-attention read (ldc 0: one row for every live row)
constexpr int FR_MAXF = 8;   // floats per lane: d <= 512
__device__ __forceinline__ void fr_layernorm(float (&v)[FR_MAXF], int lane, int d, float eps, const float* g,
                                             const float* b) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) s += v[j];
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) {
    const int c = lane + 64 * j;
    const float dl = c < d ? v[j] - mean : 0.f;
    q += dl * dl;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)d + eps);
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < d ? (v[j] - mean) * rstd * g[c] + b[c] : 0.f;
  }
}

__global__ __launch_bounds__(256) void k_fr_ln12(const XtrlDecodeDesc D, int t, const float* o, const float* cx,
                                                 int ldcx, const float* g1, const float* b1, const float* g2,
                                                 const float* b2, float* x2, float eps) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63, d = D.d;
  if (r >= D.live_count[t & 1]) return;
  const float* xr = D.x + (int64_t)r * d;
  const float* orow = o + (int64_t)r * d;
  const float* crow = cx + (int64_t)r * ldcx;
  float v[FR_MAXF], cv[FR_MAXF];
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < d ? xr[c] + orow[c] : 0.f;
    cv[j] = c < d ? crow[c] : 0.f;
  }
  fr_layernorm(v, lane, d, eps, g1, b1);
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) v[j] += cv[j];
  fr_layernorm(v, lane, d, eps, g2, b2);
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) {
    const int c = lane + 64 * j;
    if (c < d) x2[(int64_t)r * d + c] = v[j];
  }
}

// x3 = LN3(s3) (s3 = x2 + FF(x2)); the episode slot's running sum of x3 (restarting at t = 0) and the running mean
// of the live row; the next level's input x3 + level_embed[l + 1] into D.x (xnext NULL: last level)
__global__ __launch_bounds__(256) void k_fr_ln3_tail(const XtrlDecodeDesc D, int t, const float* s3, const float* g3,
                                                     const float* b3, float* sums, float* mean, const float* le_next,
                                                     float eps) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63, d = D.d;
  if (r >= D.live_count[t & 1]) return;
  const int e = rows_of(D, t)[r];
  float v[FR_MAXF], sp[FR_MAXF];
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < d ? s3[(int64_t)r * d + c] : 0.f;
    sp[j] = (c < d && t > 0) ? sums[(int64_t)e * d + c] : 0.f;   // step 0 starts the episode's sum
  }
  fr_layernorm(v, lane, d, eps, g3, b3);
#pragma unroll
  for (int j = 0; j < FR_MAXF; ++j) {
    const int c = lane + 64 * j;
    if (c < d) {
      const float sm = sp[j] + v[j];
      sums[(int64_t)e * d + c] = sm;
      mean[(int64_t)r * d + c] = sm / (float)(t + 1);
      if (le_next) D.x[(int64_t)r * d + c] = v[j] + le_next[c];
    }
  }
}

int check_desc(const XtrlDecodeDesc* D) {
  XTRL_REQUIRE(D && D->layers, "decode: null descriptor");
  XTRL_REQUIRE(D->live_rows && D->live_count, "decode: live_rows / live_count missing");
  XTRL_REQUIRE(D->E > 0 && D->S > 0 && D->S < 64 && D->A > 0 && D->A <= 32, "decode: bad E/S/A (E=%d S=%d A=%d)",
               D->E, D->S, D->A);
  XTRL_REQUIRE(D->dh == 16 || D->dh == 32 || D->dh == 64, "decode: dim_head %d unsupported (16/32/64)", D->dh);
  XTRL_REQUIRE(D->H * D->dh <= 4096 && D->d > 0 && D->d <= 512 && D->d % 4 == 0 && D->L > 0 && D->Tmax > 0,
               "decode: bad dims (d must be a multiple of 4, at most 512)");
  XTRL_REQUIRE(D->in_dim == 2 * D->d + (D->evolutionary ? D->d : 0), "decode: in_dim mismatch");
  const int I = D->H * D->dh;
  XTRL_REQUIRE(D->n_qkv == 3 * I + (D->gate_values ? I : 0) + ((D->value_residual && D->learned_mix) ? D->H : 0),
               "decode: n_qkv mismatch");
  XTRL_REQUIRE(!D->ff_glu || (D->hglu && D->hff), "decode: ff_glu needs hglu");
  return XTRL_OK;
}

// compaction (inside the embedding for E <= EMB_MAX_E) + embeddings of step t
template <bool CMP>
void launch_embed_t(const XtrlDecodeDesc* D, int t, const float* g, hipStream_t s) {
  const dim3 grid((D->E + EMB_ROWS - 1) / EMB_ROWS), blk(1024);
  switch ((D->d + 63) / 64) {
    case 1: hipLaunchKernelGGL((k_embed<1, CMP>), grid, blk, 0, s, *D, t, g); break;
    case 2: hipLaunchKernelGGL((k_embed<2, CMP>), grid, blk, 0, s, *D, t, g); break;
    case 3: hipLaunchKernelGGL((k_embed<3, CMP>), grid, blk, 0, s, *D, t, g); break;
    case 4: hipLaunchKernelGGL((k_embed<4, CMP>), grid, blk, 0, s, *D, t, g); break;
    default: hipLaunchKernelGGL((k_embed<8, CMP>), grid, blk, 0, s, *D, t, g); break;
  }
}
// g_ln0: the gain of layer 0's pre-attention LayerNorm when the embedding also writes xn, else NULL
int launch_embed(const XtrlDecodeDesc* D, int t, const float* g_ln0, hipStream_t s) {
  if (D->E <= EMB_MAX_E) {
    launch_embed_t<true>(D, t, g_ln0, s);
  } else {
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, *D, t);
    XTRL_LAUNCHED("compact");
    launch_embed_t<false>(D, t, g_ln0, s);
  }
  XTRL_LAUNCHED("embed");
  return XTRL_OK;
}

// whether layer l's attention launch applies its out-projection + residual (k_attn_decode FUSE)
bool attn_fused(const XtrlDecodeDesc* D, int l) {
  const size_t lds = ((size_t)D->H * (D->Tmax + 3 * D->dh) + (size_t)D->H * D->d) * sizeof(float);
  // (dh = 16 only: the dh = 32 forms would spill the prefetched W_out^T rows)
  return D->layers[l].w_out_t && D->dh == 16 && D->H <= 8 && D->d % 4 == 0 && D->d <= 512 &&
         D->d <= 4 * 64 * D->H && lds <= 160 * 1024;
}

// ---------------------------------------------------------------------------------------------
// the feed-forward block of a decode layer in ONE launch (replaces the FF1 and FF2 projections):
// workgroup (hidden chunk c, 16-row panel p) computes h_c = GELU(xn W1[c]^T + b1[c]) for its 16
// live rows and 128 hidden units (kept in LDS) and the partial output h_c W2[:, c]^T (16 x d).  The
// ff / 128 partials of a panel meet through the cross-workgroup hand-off of the MI355X guide (sc1
// stores and loads, no fences): every workgroup stores its partial tile with sc1 stores, every wave
// waits for them, and behind a workgroup barrier one lane adds to the panel's arrival counter
// (agent scope); the workgroup whose add returned ff/128 - 1 sums the partials in chunk order
// (sc1 loads) onto the residual row and b2, stores the layer output and the next pre-norm of it,
// and zeroes the counter.  Every chunk workgroup of a live panel is live, so the count always
// completes; nothing waits or polls.  Both products run on the bf16 matrix cores as split-bf16
// ("X6", x6.h: fp32-accurate): the weights pre-split at pack time (xtrl_dgemm_pack_x6), the
// activations split as their fragments are read from LDS (6 x 16 cycles per 32-deep step instead
// of 8 x 32 for the f32 MFMA: at E = 1024 the fp32 feed-forward was matrix-core bound).
// ---------------------------------------------------------------------------------------------
constexpr int MLP_HW = 128;   // hidden units per workgroup

// fp32 operands as split-bf16 pieces: 8 consecutive values -> hi / mid / lo bf16x8 fragments
__device__ __forceinline__ void split3x8(const f32x4v a, const f32x4v b, bf16x8& h, bf16x8& m, bf16x8& l) {
  uint32_t hh[4], mm[4], ll[4];
  split3_pair(a[0], a[1], hh[0], mm[0], ll[0]);
  split3_pair(a[2], a[3], hh[1], mm[1], ll[1]);
  split3_pair(b[0], b[1], hh[2], mm[2], ll[2]);
  split3_pair(b[2], b[3], hh[3], mm[3], ll[3]);
  h = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
  m = __builtin_bit_cast(bf16x8, make_uint4(mm[0], mm[1], mm[2], mm[3]));
  l = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
}
// acc += a . b over 32 k as the six largest piece products, smallest first (x6.h)
__device__ __forceinline__ f32x4v mfma_x6(const bf16x8 (&a)[3], const uint4 (&b)[3], f32x4v c) {
  const bf16x8 bh = __builtin_bit_cast(bf16x8, b[0]), bm = __builtin_bit_cast(bf16x8, b[1]),
               bl = __builtin_bit_cast(bf16x8, b[2]);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bh, c, 0, 0, 0);
}

// FrMlp (fractal body, g3 non-NULL): the tail forms x3 = LN3(s3) g3 + b3 (nn.LayerNorm, eps) of the
// completed rows instead of a pre-norm, adds it to the episode slot's running sum (restarting at
// t = 0), stores the running mean and, for all but the last level, the next level's input
// x3 + le_next into D.x
struct FrMlp {
  const float *g3 = nullptr, *b3 = nullptr;
  float* sums = nullptr;
  float* mean = nullptr;
  const float* le_next = nullptr;
  float eps = 1e-5f;
};

// a weight fragment as its three bf16 piece fragments: WR = 3 (the split image, as loaded) or WR = 2
// (the fp32 image: 8 consecutive k of the lane's column, split here exactly as xtrl_dgemm_pack_x6 does)
template <int WR>
__device__ __forceinline__ void frag_pieces(const uint4 (&w)[WR], uint4 (&b)[3]) {
  if constexpr (WR == 3) {
    b[0] = w[0]; b[1] = w[1]; b[2] = w[2];
  } else {
    const float4 u = __builtin_bit_cast(float4, w[0]), v = __builtin_bit_cast(float4, w[1]);
    uint32_t h[4], m[4], l[4];
    split3_pair(u.x, u.y, h[0], m[0], l[0]);
    split3_pair(u.z, u.w, h[1], m[1], l[1]);
    split3_pair(v.x, v.y, h[2], m[2], l[2]);
    split3_pair(v.z, v.w, h[3], m[3], l[3]);
    b[0] = make_uint4(h[0], h[1], h[2], h[3]);
    b[1] = make_uint4(m[0], m[1], m[2], m[3]);
    b[2] = make_uint4(l[0], l[1], l[2], l[3]);
  }
}

// FI: the weights come from the fp32 fragment images (Ly.w_ff1f / w_ff2f: 2/3 of the split images'
// bytes, the split done per fragment before its MFMAs) instead of the split images.  EW (FI only):
// the W2 fragments are loaded in the same batch as W1 (one weight round trip instead of two; 256
// registers of weights: one workgroup per SIMD set)
template <int NT2, int MT, bool FI, bool EW = false>   // d = 64 NT2 (d <= 256): output columns per wave 16 NT2; panel rows 16 MT
__global__ __launch_bounds__(256, EW ? 1 : 2) void k_mlp(const XtrlDecodeDesc D, const XtrlDecodeLayer Ly, int t, const float* xin,
                                             const float* res, float* C, int ldc, const float* g_next, float* Y,
                                             int ldy, const FrMlp fm) {
  constexpr int d = 64 * NT2, NT1 = MLP_HW / 64, BM = 16 * MT;
  constexpr int LDA = d + 4, JS1 = d / 32;              // FF1: K = d, 32-deep k steps
  constexpr int LDH = MLP_HW + 4, JSC = MLP_HW / 32;    // FF2: the chunk's 128 k
  __shared__ __attribute__((aligned(16))) float A1[BM * LDA];
  __shared__ __attribute__((aligned(16))) float Hs[BM * LDH];
  __shared__ int last_sh;
  const int HC = D.ff / MLP_HW, JS2 = D.ff / 32;
  const int c = blockIdx.x, p = blockIdx.y, m0 = p * BM;
  const int M = D.live_count[t & 1];
  if (m0 >= M) return;   // (workgroup-uniform)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, q = lane >> 4;
  // ---- operands: the panel's xn rows (LDS-DMA, one 1 KiB piece per row; the destination is the
  //      wave's row base, lane i lands 16 i bytes further), this wave's W1 piece fragments of the
  //      chunk (all of K in one batch), b1
  if (4 * lane < d)
    for (int r = w; r < BM; r += 4)
      __builtin_amdgcn_global_load_lds((const void*)(xin + (int64_t)min(m0 + r, M - 1) * d + 4 * lane),
                                       (lds_void*)(A1 + r * LDA), 16, 0, 0);
  constexpr int WR = FI ? 2 : 3;   // 16-byte registers per weight fragment
  const uint4* w1 = reinterpret_cast<const uint4*>(FI ? (const void*)Ly.w_ff1f : (const void*)Ly.w_ff1x);
  const int64_t P1 = (int64_t)D.ff / 16 * JS1 * 64;   // slots per piece plane
  uint4 bw[NT1][JS1][WR];
  float b1v[NT1];
#pragma unroll
  for (int nt = 0; nt < NT1; ++nt) {
    const int t16 = c * (MLP_HW / 16) + w * NT1 + nt;
    const uint4* wp = w1 + (int64_t)t16 * JS1 * 64 + lane;
#pragma unroll
    for (int s = 0; s < JS1; ++s)
#pragma unroll
      for (int pc = 0; pc < WR; ++pc) bw[nt][s][pc] = wp[pc * P1 + 64 * s];
    b1v[nt] = Ly.b_ff1[t16 * 16 + lr];
  }
  // this wave's W2 fragments: tiles w NT2 + nt, k steps of chunk c (EW: in this batch; else issued
  // after FF1: with the first batch they would double the registers)
  const uint4* w2 = reinterpret_cast<const uint4*>(FI ? (const void*)Ly.w_ff2f : (const void*)Ly.w_ff2x);
  const int64_t P2 = (int64_t)(d / 16) * JS2 * 64;
  uint4 b2w[NT2][JSC][WR];
  auto load_w2 = [&]() {
#pragma unroll
    for (int nt = 0; nt < NT2; ++nt) {
      const uint4* wp = w2 + ((int64_t)(w * NT2 + nt) * JS2 + c * JSC) * 64 + lane;
#pragma unroll
      for (int s = 0; s < JSC; ++s)
#pragma unroll
        for (int pc = 0; pc < WR; ++pc) b2w[nt][s][pc] = wp[pc * P2 + 64 * s];
    }
  };
  if constexpr (EW) load_w2();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- FF1 chunk + GELU -> Hs
  {
    f32x4v acc[MT][NT1][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT1; ++nt) acc[mt][nt][0] = acc[mt][nt][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < JS1; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float* ap = A1 + (16 * mt + lr) * LDA + 32 * s + 8 * q;
        bf16x8 a[3];
        split3x8(*reinterpret_cast<const f32x4v*>(ap), *reinterpret_cast<const f32x4v*>(ap + 4), a[0], a[1], a[2]);
#pragma unroll
        for (int nt = 0; nt < NT1; ++nt) {
          uint4 b[3];
          frag_pieces<WR>(bw[nt][s], b);
          acc[mt][nt][s & 1] = mfma_x6(a, b, acc[mt][nt][s & 1]);
        }
      }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT1; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          Hs[(16 * mt + 4 * q + i) * LDH + w * 16 * NT1 + 16 * nt + lr] =
              geluf_((acc[mt][nt][0][i] + acc[mt][nt][1][i]) + b1v[nt]);
  }
  if constexpr (!EW) load_w2();
  __syncthreads();   // (Hs complete)
  // ---- FF2 partial of the chunk -> sc1 stores
  {
    f32x4v acc[MT][NT2][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT2; ++nt) acc[mt][nt][0] = acc[mt][nt][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < JSC; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float* ap = Hs + (16 * mt + lr) * LDH + 32 * s + 8 * q;
        bf16x8 a[3];
        split3x8(*reinterpret_cast<const f32x4v*>(ap), *reinterpret_cast<const f32x4v*>(ap + 4), a[0], a[1], a[2]);
#pragma unroll
        for (int nt = 0; nt < NT2; ++nt) {
          uint4 b[3];
          frag_pieces<WR>(b2w[nt][s], b);
          acc[mt][nt][s & 1] = mfma_x6(a, b, acc[mt][nt][s & 1]);
        }
      }
    float* part = D.mlp_part + ((int64_t)p * HC + c) * BM * d;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT2; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          __hip_atomic_store(part + (16 * mt + 4 * q + i) * d + w * 16 * NT2 + 16 * nt + lr,
                             acc[mt][nt][0][i] + acc[mt][nt][1][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Ordering (not the HIP memory model's release/acquire: a relaxed counter is formally a race
  // there): the gfx950 visibility rules of /opt/skills/guides/MI355X_MICROARCH.md § visibility,
  // "Valid forms", consumer bullet (1)-(4) — (2) every partial byte is stored sc1 (relaxed
  // agent-scope atomic store = global_store ... sc1, write-through to the memory side), (3) every
  // storing wave waits vmcnt(0) for its stores and the one counter add comes after a workgroup
  // barrier behind all those waits, (1) the last arriver reads every partial with sc1 loads
  // (relaxed agent-scope atomic load = global_load ... sc1, bypassing its CU's L1), so no
  // agent-scope release (buffer_wbl2) or acquire (buffer_inv) is needed.  Checked in the ISA of
  // this kernel: the partial stores / loads are global_store/load_dword ... sc1, never flat_.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its partial stores have completed
  __syncthreads();
  if (tid == 0)
    last_sh = __hip_atomic_fetch_add(D.mlp_cnt + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(HC - 1);
  __syncthreads();
  if (!last_sh) return;   // (workgroup-uniform)
  // ---- the last chunk workgroup of the panel: residual + b2 + the partials in chunk order (every
  //      load issued before the first store: C may be the residual row itself)
  //      The partials are loaded HB chunks at a time, all HB x EPT loads of a batch in flight together
  //      (a loop of one chunk per round trip measured ~8 memory round trips in this tail), clamped
  //      past the last chunk and added in chunk order
  constexpr int EPT = BM * d / 256;   // elements per thread
  constexpr int HB = EPT <= 16 ? 8 : 4;
  const float* part0 = D.mlp_part + (int64_t)p * HC * BM * d;
  float v[EPT], rv[EPT], bv[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = tid + 256 * k, r = e / d, col = e - r * d;
    rv[k] = res[(int64_t)min(m0 + r, M - 1) * d + col];
    bv[k] = Ly.b_ff2[col];
  }
  for (int c0 = 0; c0 < HC; c0 += HB) {
    float pv[HB][EPT];
#pragma unroll
    for (int u = 0; u < HB; ++u) {
      const int cc = min(c0 + u, HC - 1);
#pragma unroll
      for (int k = 0; k < EPT; ++k) {
        const int e = tid + 256 * k, r = e / d, col = e - r * d;
        pv[u][k] = __hip_atomic_load(part0 + ((int64_t)cc * BM + r) * d + col, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (c0 == 0) {
#pragma unroll
      for (int k = 0; k < EPT; ++k) v[k] = rv[k] + bv[k];
    }
#pragma unroll
    for (int u = 0; u < HB; ++u)
      if (c0 + u < HC) {   // (uniform; no load under it)
#pragma unroll
        for (int k = 0; k < EPT; ++k) v[k] += pv[u][k];
      }
  }
  if (tid == 0) __hip_atomic_store(D.mlp_cnt + p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = tid + 256 * k, r = e / d, col = e - r * d, m = m0 + r;
    if (C && m < M) C[(int64_t)m * ldc + col] = v[k];
    A1[r * LDA + col] = v[k];   // (A1 is free: every wave is past its FF1)
  }
  // the next pre-norm of the completed rows (the next layer's attention LayerNorm, or the final norm
  // in the heads' input row), two-pass as the GEMM prologue: one wave per BM / 4 rows (Y NULL: none)
  if (fm.g3) {   // fractal: LayerNorm 3, the running sums / mean and the next level's input
    __syncthreads();
    float g3v[NT2], b3v[NT2], lev[NT2];
#pragma unroll
    for (int j = 0; j < NT2; ++j) {
      g3v[j] = fm.g3[lane + 64 * j];
      b3v[j] = fm.b3[lane + 64 * j];
      lev[j] = fm.le_next ? fm.le_next[lane + 64 * j] : 0.f;
    }
    const int32_t* slots = rows_of(D, t);
#pragma unroll
    for (int rr = 0; rr < BM / 4; ++rr) {
      const int r = (BM / 4) * w + rr, m = m0 + r;
      const int e = slots[min(m, M - 1)];
      float xv[NT2], sp[NT2], sm = 0.f;
#pragma unroll
      for (int j = 0; j < NT2; ++j) {
        xv[j] = A1[r * LDA + lane + 64 * j];
        sp[j] = t > 0 ? fm.sums[(int64_t)e * d + lane + 64 * j] : 0.f;
        sm += xv[j];
      }
      const float mean = wave_sum_dpp(sm) / (float)d;
      float qq = 0.f;
#pragma unroll
      for (int j = 0; j < NT2; ++j) {
        const float dl = xv[j] - mean;
        qq += dl * dl;
      }
      const float rstd = 1.0f / sqrtf(wave_sum_dpp(qq) / (float)d + fm.eps);
      if (m < M)
#pragma unroll
        for (int j = 0; j < NT2; ++j) {
          const int col = lane + 64 * j;
          const float x3 = (xv[j] - mean) * rstd * g3v[j] + b3v[j];
          const float s2 = sp[j] + x3;
          fm.sums[(int64_t)e * d + col] = s2;
          fm.mean[(int64_t)m * d + col] = s2 / (float)(t + 1);
          if (fm.le_next) D.x[(int64_t)m * d + col] = x3 + lev[j];
        }
    }
    return;
  }
  if (!Y) return;
  __syncthreads();
#pragma unroll
  for (int rr = 0; rr < BM / 4; ++rr) {
    const int r = (BM / 4) * w + rr, m = m0 + r;
    float xv[NT2], sm = 0.f;
#pragma unroll
    for (int j = 0; j < NT2; ++j) {
      xv[j] = A1[r * LDA + lane + 64 * j];
      sm += xv[j];
    }
    const float mean = D.rms_norm ? 0.f : wave_sum_dpp(sm) / (float)d;
    float qq = 0.f;
#pragma unroll
    for (int j = 0; j < NT2; ++j) {
      const float dl = xv[j] - mean;
      qq += dl * dl;
    }
    const float rstd = norm_rstd(wave_sum_dpp(qq), (float)d, D.rms_norm);
    if (m < M)
#pragma unroll
      for (int j = 0; j < NT2; ++j)
        Y[(int64_t)m * ldy + lane + 64 * j] = ((xv[j] - mean) * rstd) * g_next[lane + 64 * j];
  }
}

// panel rows of the fused feed-forward: 16; XTRL_MLP_ROWS=32 (experiments) feeds every weight
// fragment to twice the rows on half the workgroups — measured slower at C3 (26.2 vs 19.7 us a
// launch, rollout 26.5 vs 23.2 ms: the per-wave MFMA chain doubles and one workgroup per CU is left)
int mlp_rows() {
  static const int r = [] {
    const char* e = getenv("XTRL_MLP_ROWS");
    return (e && atoi(e) == 32) ? 32 : 16;
  }();
  return r;
}

// XTRL_MLP_EW=1: the fp32-image feed-forward loads W1 and W2 in one batch (one workgroup per SIMD set)
bool mlp_ew() {
  static const bool on = [] {
    const char* e = getenv("XTRL_MLP_EW");
    return e && atoi(e) == 1;
  }();
  return on;
}

// the one-launch feed-forward's weights: the fp32 fragment images (preferred) or the split images
bool mlp_weights(const XtrlDecodeLayer& Ly) { return (Ly.w_ff1f && Ly.w_ff2f) || (Ly.w_ff1x && Ly.w_ff2x); }

bool mlp_fused(const XtrlDecodeDesc* D, int l) {
  return !D->ff_glu && D->xn && D->mlp_part && D->mlp_cnt && mlp_weights(D->layers[l]) && attn_fused(D, l) &&
         D->d % 64 == 0 &&
         D->d <= 256 && D->ff % MLP_HW == 0;
}

// layer l's feed-forward: x += FF(xn), then the next pre-norm of the rows — the last layer writes only
// the final-normed row into the heads' input (nothing reads its raw output), the others x and xn
// the one-launch feed-forward over the live rows: C = res + FF(xin) (C NULL: not stored), then
// (Y non-NULL) the pre-norm LN(C) g into Y
int launch_mlp_rows(const XtrlDecodeDesc* D, int l, int t, const float* xin, const float* res, float* C, int ldc,
                    const float* g, float* Y, int ldy, hipStream_t s, const FrMlp& fm = FrMlp{}) {
  const int bm = mlp_rows();
  const dim3 grid(D->ff / MLP_HW, (D->E + bm - 1) / bm);
  const XtrlDecodeLayer& Ly = D->layers[l];
  const bool fi = Ly.w_ff1f && Ly.w_ff2f;
#define XTRL_MLP(NT2)                                                                              \
  do {                                                                                             \
    if (bm == 32 && fi)                                                                            \
      hipLaunchKernelGGL((k_mlp<NT2, 2, true>), grid, dim3(256), 0, s, *D, Ly, t, xin, res, C, ldc, g, Y, ldy, fm); \
    else if (bm == 32)                                                                             \
      hipLaunchKernelGGL((k_mlp<NT2, 2, false>), grid, dim3(256), 0, s, *D, Ly, t, xin, res, C, ldc, g, Y, ldy, fm); \
    else if (fi && mlp_ew()) hipLaunchKernelGGL((k_mlp<NT2, 1, true, true>), grid, dim3(256), 0, s, *D, Ly, t, xin, res, C, ldc, g, Y, ldy, fm); \
    else if (fi) hipLaunchKernelGGL((k_mlp<NT2, 1, true>), grid, dim3(256), 0, s, *D, Ly, t, xin, res, C, ldc, g, Y, ldy, fm); \
    else hipLaunchKernelGGL((k_mlp<NT2, 1, false>), grid, dim3(256), 0, s, *D, Ly, t, xin, res, C, ldc, g, Y, ldy, fm); \
  } while (0)
  switch (D->d / 64) {
    case 1: XTRL_MLP(1); break;
    case 2: XTRL_MLP(2); break;
    case 3: XTRL_MLP(3); break;
    default: XTRL_MLP(4); break;
  }
#undef XTRL_MLP
  XTRL_LAUNCHED("mlp");
  return XTRL_OK;
}

int launch_mlp(const XtrlDecodeDesc* D, int l, int t, hipStream_t s) {
  const bool last = l == D->L - 1;
  return launch_mlp_rows(D, l, t, D->xn, D->x, last ? nullptr : D->x, D->d,
                         last ? D->ln_final : D->layers[l + 1].ln_attn, last ? D->ac_in : D->xn,
                         last ? D->in_dim : D->d, s);
}

int launch_attn_decode(const XtrlDecodeDesc* D, int l, int t, hipStream_t s, const FrPost& fp = FrPost{}) {
  if (attn_fused(D, l)) {   // one workgroup of H waves per live row
    const size_t lds = ((size_t)D->H * (D->Tmax + 3 * D->dh) + (size_t)D->H * D->d) * sizeof(float);
    const dim3 grid(D->E), blk(64 * D->H);
    if (D->d > 256) hipLaunchKernelGGL((k_attn_decode<16, 2>), grid, blk, lds, s, *D, D->layers[l], l, t, fp);
    else hipLaunchKernelGGL((k_attn_decode<16, 1>), grid, blk, lds, s, *D, D->layers[l], l, t, fp);
    XTRL_LAUNCHED("attn_decode");
    return XTRL_OK;
  }
  const int waves = D->E * D->H;
  const size_t lds = 4 * (size_t)(D->Tmax + 3 * D->dh) * sizeof(float);
  XTRL_REQUIRE(lds <= 160 * 1024, "attn_decode: Tmax %d too large for LDS", D->Tmax);
  dim3 grid((waves + 3) / 4);
  if (D->dh == 16)
    hipLaunchKernelGGL((k_attn_decode<16, 0>), grid, dim3(256), lds, s, *D, D->layers[l], l, t, fp);
  else if (D->dh == 32)
    hipLaunchKernelGGL((k_attn_decode<32, 0>), grid, dim3(256), lds, s, *D, D->layers[l], l, t, fp);
  else
    hipLaunchKernelGGL((k_attn_decode<64, 0>), grid, dim3(256), lds, s, *D, D->layers[l], l, t, fp);
  XTRL_LAUNCHED("attn_decode");
  return XTRL_OK;
}

// one decode projection over the live rows of step t
// ff_glu: hglu[r][j] = hff[r][j] * gelu(hff[r][ff + j]) over the step's live rows (x-transformers GLU;
// the rollout runs the model in eval: no dropout)
__global__ void k_glu_rows(const XtrlDecodeDesc D, int t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int ff = D.ff, M = D.live_count[t & 1];
  if (i >= (int64_t)M * ff) return;
  const int r = (int)(i / ff), j = (int)(i - (int64_t)r * ff);
  const float* u = D.hff + (int64_t)r * 2 * ff;
  D.hglu[(int64_t)r * ff + j] = u[j] * geluf_(u[ff + j]);
}

int dproj(const XtrlDecodeDesc* D, int t, const float* A, int lda, const float* W, int K, const float* bias,
          const float* gamma, int ln_k, const float* R, int ldr, float* C, int ldc, int N, int epi, hipStream_t s,
          const int32_t* row_map = nullptr, int n_split = 1 << 30, float* C2 = nullptr, int ldc2 = 0,
          const int32_t* row_map2 = nullptr) {
  DGemmArgs g;
  g.n_split = n_split; g.C2 = C2; g.ldc2 = ldc2; g.row_map2 = row_map2;
  g.A = A; g.lda = lda; g.W = W; g.ldw = K; g.bias = bias; g.gamma = gamma; g.ln_k = ln_k; g.ln_rms = D->rms_norm;
  g.R = R; g.ldr = ldr; g.C = C; g.ldc = ldc; g.row_map = row_map;
  g.m_dev = D->live_count + (t & 1);
  g.M = D->E; g.N = N; g.K = K;
  return dgemm_run(g, D->E, epi, s);
}

// heads + sampling of a decode step: hidden [n][4d] = SiLU([LN_final?(x) | state embed | latent] .
// [Wa1; Wc1]^T + b); the last Linear layers as one block-diagonal projection (actor logits to the
// logits rows, critic bins straight into the trajectory row t of each live episode: Memory.value,
// xtrl.py:1315); then sampling and the Sim step
// ---------------------------------------------------------------------------------------------
// the actor-critic heads in ONE launch (replaces the hidden-layer projection and the last
// projection + sampling pair): workgroup (hidden chunk c of 64 units, 16-row panel p), 8 waves —
// wave w multiplies the panel's [final-normed x | state embed | latent] rows (ac_in, staged in LDS)
// by hidden tile w & 3 of the chunk over k half w >> 2 (split-bf16 products on the bf16 matrix
// cores, the weight pre-split by xtrl_dgemm_pack_x6), the two k halves meet in LDS in order, + b1,
// SiLU; then the chunk's partial of the block-diagonal last Linear (actor chunks c < HC / 2 feed the
// n_act actor outputs, critic chunks the B value logits; fp32 FMAs over the chunk's 64 hidden units,
// W2 rows staged in LDS) goes out with sc1 stores and the panel's arrival counter (k_mlp's hand-off)
// elects the last chunk workgroup, which sums the partials in chunk order + b2, stores the logits /
// value logits and runs the sampling + Sim step of its rows (SAMPLE_L lanes per row, the rows'
// sampling inputs loaded while the matrix cores run).
// ---------------------------------------------------------------------------------------------
__host__ __device__ inline int round4i(int x) { return (x + 3) & ~3; }
constexpr int HD_HW = 64;   // hidden units per workgroup
constexpr int HD_T = 512;   // threads
struct HeadsLds {   // floats, carved from the dynamic LDS
  int a, hp, hs, w2, lg, tot;
};
__host__ __device__ inline HeadsLds heads_lds(int in_dim, int np) {
  HeadsLds o;
  int at = 0;
  o.a = at; at += 16 * (in_dim + 4);
  o.hp = at; at += 2 * 16 * (HD_HW + 4);
  o.hs = at; at += 16 * (HD_HW + 4);
  o.w2 = at; at += HD_HW * np;
  o.lg = at; at += 16 * 64;
  o.tot = at;
  return o;
}

template <int JH>   // k steps (32 deep) per wave: in_dim = 64 JH
__global__ __launch_bounds__(HD_T) void k_heads_mlp(const XtrlDecodeDesc D, int t) {
  extern __shared__ __attribute__((aligned(16))) float hl[];
  __shared__ int e_sh[16];
  __shared__ int last_sh;
  constexpr int in_dim = 64 * JH, LDA = in_dim + 4, LDH = HD_HW + 4;
  constexpr int AV = (16 * in_dim / 4 + HD_T - 1) / HD_T;   // A panel float4 per thread
  constexpr int W2V = 8;                                    // W2 chunk float4 per thread (np <= 128)
  constexpr int CHM = 8;                                    // chunks per head half at most (d <= 256)
  const int n_act = D.continuous ? 2 * D.A : D.A, na2 = n_act + D.B, np = round4i(na2);
  const int HC = 4 * D.d / HD_HW, HCh = HC / 2;
  const int c = blockIdx.x, p = blockIdx.y, m0 = 16 * p;
  const int M = D.live_count[t & 1];
  if (m0 >= M) return;   // (workgroup-uniform)
  const HeadsLds Lo = heads_lds(in_dim, np);
  float *As = hl + Lo.a, *Hp = hl + Lo.hp, *Hs = hl + Lo.hs, *W2s = hl + Lo.w2, *lg = hl + Lo.lg;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, q = lane >> 4;
  const int tile = w & 3, kh = w >> 2;
  const bool actor = c < HCh;
  const int n0 = actor ? 0 : n_act, nn = actor ? n_act : D.B;
  // ---- one batch: the panel's rows, this wave's W1 fragments, b1, the chunk's W2 rows, b2, slots
  float4 av[AV];
#pragma unroll
  for (int u = 0; u < AV; ++u) {
    const int f = min(tid + HD_T * u, 16 * (in_dim / 4) - 1), r = f / (in_dim / 4), k4 = f - r * (in_dim / 4);
    av[u] = reinterpret_cast<const float4*>(D.ac_in + (int64_t)min(m0 + r, M - 1) * D.in_dim)[k4];
  }
  const uint4* w1 = reinterpret_cast<const uint4*>(D.w_h1x);
  const int JS = in_dim / 32;
  const int64_t P1 = (int64_t)(4 * D.d / 16) * JS * 64;   // slots per piece plane
  const int t16 = c * (HD_HW / 16) + tile;
  uint4 bw[JH][3];
  {
    const uint4* wp = w1 + ((int64_t)t16 * JS + kh * JH) * 64 + lane;
#pragma unroll
    for (int s = 0; s < JH; ++s)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) bw[s][pc] = wp[pc * P1 + 64 * s];
  }
  float b1v[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b1v[j] = D.b_h1[c * HD_HW + ((tid + HD_T * j) & (HD_HW - 1))];
  const int w2n = HD_HW * np / 4;
  float4 w2v[W2V];
#pragma unroll
  for (int u = 0; u < W2V; ++u)
    w2v[u] = reinterpret_cast<const float4*>(D.w_h2_t + (int64_t)c * HD_HW * np)[min(tid + HD_T * u, w2n - 1)];
  float b2v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b2v[j] = D.b_h2[min((tid + HD_T * j) % na2, np - 1)];
  const int srow = tid / SAMPLE_L, sub = tid % SAMPLE_L;
  int e = 0;
  if (srow < 16) e = rows_of(D, t)[min(m0 + srow, M - 1)];
  // ---- to LDS
#pragma unroll
  for (int u = 0; u < AV; ++u) {
    const int f = tid + HD_T * u;
    if (f < 16 * (in_dim / 4)) {
      const int r = f / (in_dim / 4), k4 = f - r * (in_dim / 4);
      *reinterpret_cast<float4*>(As + r * LDA + 4 * k4) = av[u];
    }
  }
#pragma unroll
  for (int u = 0; u < W2V; ++u)
    if (tid + HD_T * u < w2n) reinterpret_cast<float4*>(W2s)[tid + HD_T * u] = w2v[u];
  if (srow < 16 && sub == 0) e_sh[srow] = e;
  SampleIn in{};
  if (srow < 16) in = sample_load(D, e);   // (in flight during the products)
  __syncthreads();
  // ---- hidden tile over this wave's k half -> Hp[kh]
  {
    f32x4v acc[2] = {f32x4v{0.f, 0.f, 0.f, 0.f}, f32x4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < JH; ++s) {
      const float* ap = As + lr * LDA + 32 * (kh * JH + s) + 8 * q;
      bf16x8 a[3];
      split3x8(*reinterpret_cast<const f32x4v*>(ap), *reinterpret_cast<const f32x4v*>(ap + 4), a[0], a[1], a[2]);
      acc[s & 1] = mfma_x6(a, bw[s], acc[s & 1]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) Hp[(kh * 16 + 4 * q + i) * LDH + 16 * tile + lr] = acc[0][i] + acc[1][i];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {   // 16 x 64 hidden values, two per thread
    const int i = tid + HD_T * j, r = i / HD_HW, col = i & (HD_HW - 1);
    Hs[r * LDH + col] = siluf_((Hp[r * LDH + col] + Hp[(16 + r) * LDH + col]) + b1v[j]);
  }
  __syncthreads();
  // ---- the chunk's partial of its head's outputs (16 rows x nn over the chunk's 64 hidden units on
  //      v_mfma_f32_16x16x4_f32, wave w: output columns n0 + 16 w ...) -> sc1 stores
  float* part = D.heads_part + ((int64_t)p * HC + c) * 16 * np;
  if (w < (nn + 15) / 16) {   // (wave-uniform)
    const int n = n0 + 16 * w + lr;
    const bool nv = n < n0 + nn;
    const int nc = nv ? n : n0;
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < HD_HW / 4; ++s) {
      const float b = W2s[(4 * s + q) * np + nc];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Hs[lr * LDH + 4 * s + q], nv ? b : 0.f, acc, 0, 0, 0);
    }
    if (nv) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __hip_atomic_store(part + (4 * q + i) * np + n, acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // the hand-off of k_mlp (MI355X_MICROARCH.md visibility, "Valid forms": sc1 stores, per-wave
  // vmcnt(0), a workgroup barrier, one agent-scope counter add; the last arriver reads with sc1 loads)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    last_sh = __hip_atomic_fetch_add(D.heads_cnt + p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(HC - 1);
  __syncthreads();
  if (!last_sh) return;   // (workgroup-uniform)
  // ---- the last arriver: outputs = the partials of the head's chunks in chunk order + b2, every
  //      partial load of a thread in flight together
  const float* part0 = D.heads_part + (int64_t)p * HC * 16 * np;
  float pv[4][CHM];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int it = min(tid + HD_T * j, 16 * na2 - 1), r = it / na2, n = it - r * na2, cb = n < n_act ? 0 : HCh;
#pragma unroll
    for (int u = 0; u < CHM; ++u)
      pv[j][u] = __hip_atomic_load(part0 + ((int64_t)(cb + min(u, HCh - 1)) * 16 + r) * np + n, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) __hip_atomic_store(D.heads_cnt + p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int it = tid + HD_T * j;
    if (it < 16 * na2) {
      const int r = it / na2, n = it - r * na2, m = m0 + r;
      float v = 0.f;
#pragma unroll
      for (int u = 0; u < CHM; ++u)
        if (u < HCh) v += pv[j][u];
      v += b2v[j];
      if (m < M) {
        if (n < n_act) {
          lg[r * 64 + n] = v;
          D.logits[(int64_t)m * n_act + n] = v;
        } else {
          D.traj_values[((int64_t)e_sh[r] * D.Tmax + t) * D.B + (n - n_act)] = v;
        }
      }
    }
  }
  __syncthreads();
  if (srow < 16 && m0 + srow < M) sample_row(D, t, e, sub, lg + srow * 64, in);
}

bool heads_fused(const XtrlDecodeDesc* D, bool final_norm) {
  const int n_act = D->continuous ? 2 * D->A : D->A, np = round4i(n_act + D->B);
  const int jh = D->in_dim / 64;
  return !final_norm && D->w_h1x && D->w_h2_t && D->heads_part && D->heads_cnt && D->in_dim % 64 == 0 &&
         (jh == 2 || jh == 3 || jh == 4 || jh == 6 || jh == 8 || jh == 12) && D->d % 32 == 0 && D->d <= 256 &&
         n_act <= 64 && np <= 128 && (size_t)heads_lds(D->in_dim, np).tot * sizeof(float) <= 160 * 1024;
}

int decode_heads(const XtrlDecodeDesc* D, int t, bool final_norm, hipStream_t s) {
  const int E = D->E, d = D->d;
  int rc;
  const int n_act = D->continuous ? 2 * D->A : D->A;
  if (heads_fused(D, final_norm)) {   // hidden layer + SiLU + last projection + sampling: one launch
    const dim3 grid(4 * d / HD_HW, (E + 15) / 16);
    const size_t lds = (size_t)heads_lds(D->in_dim, round4i(n_act + D->B)).tot * sizeof(float);
    switch (D->in_dim / 64) {
      case 2: hipLaunchKernelGGL(k_heads_mlp<2>, grid, dim3(HD_T), lds, s, *D, t); break;
      case 3: hipLaunchKernelGGL(k_heads_mlp<3>, grid, dim3(HD_T), lds, s, *D, t); break;
      case 4: hipLaunchKernelGGL(k_heads_mlp<4>, grid, dim3(HD_T), lds, s, *D, t); break;
      case 6: hipLaunchKernelGGL(k_heads_mlp<6>, grid, dim3(HD_T), lds, s, *D, t); break;
      case 8: hipLaunchKernelGGL(k_heads_mlp<8>, grid, dim3(HD_T), lds, s, *D, t); break;
      default: hipLaunchKernelGGL(k_heads_mlp<12>, grid, dim3(HD_T), lds, s, *D, t); break;
    }
    XTRL_LAUNCHED("heads_mlp");
    return XTRL_OK;
  }
  if ((rc = dproj(D, t, D->ac_in, D->in_dim, D->w_h1, D->in_dim, D->b_h1, final_norm ? D->ln_final : nullptr,
                  final_norm ? d : 0, nullptr, 0, D->hff, 4 * d, 4 * d, EPI_SILU, s)))
    return rc;
  const int ks = dg_ks(n_act + D->B, 4 * d);
  if (n_act <= 64 / ks) {   // block-diagonal projection + sampling in one launch (actor columns in block 0)
    DGemmArgs g;
    g.A = D->hff; g.lda = 4 * d; g.W = D->w_h2; g.ldw = 4 * d; g.bias = D->b_h2;
    g.C = D->logits; g.ldc = n_act; g.n_split = n_act;
    g.C2 = D->traj_values + (int64_t)t * D->B; g.ldc2 = D->Tmax * D->B; g.row_map2 = D->live_rows + (t & 1) * E;
    g.m_dev = D->live_count + (t & 1); g.M = E; g.N = n_act + D->B; g.K = 4 * d;
    XTRL_REQUIRE(g.K % 4 == 0 && g.K <= 2048, "decode heads: 4 d must be a multiple of 4, at most 2048");
    const int bn = 64 / ks;
    const dim3 grid((g.N + bn - 1) / bn, (E + 15) / 16);
    const size_t lds = dg_lds_floats(1, 1, ks, false, g.K) * sizeof(float);
    if (ks == 4) hipLaunchKernelGGL(k_heads_sample<4>, grid, dim3(256), lds, s, g, *D, t);
    else if (ks == 2) hipLaunchKernelGGL(k_heads_sample<2>, grid, dim3(256), lds, s, g, *D, t);
    else hipLaunchKernelGGL(k_heads_sample<1>, grid, dim3(256), lds, s, g, *D, t);
    XTRL_LAUNCHED("heads_sample");
    return XTRL_OK;
  }
  if ((rc = dproj(D, t, D->hff, 4 * d, D->w_h2, 4 * d, D->b_h2, nullptr, 0, nullptr, 0, D->logits, n_act,
                  n_act + D->B, EPI_NONE, s, nullptr, n_act, D->traj_values + (int64_t)t * D->B, D->Tmax * D->B,
                  D->live_rows + (t & 1) * E)))
    return rc;
  hipLaunchKernelGGL(k_sample, dim3((E * SAMPLE_L + 255) / 256), dim3(256), 0, s, *D, t);
  XTRL_LAUNCHED("sample");
  return XTRL_OK;
}

// ---------------------------------------------------------------------------------------------
// Row-resident decode step (few live rows, small models): ONE workgroup carries a live row through
// the whole step — compaction, RSNorm + embeddings, every layer (LayerNorm, q|k|v|gate|mix, value
// residual, rotary, KV append, attention over 0..t, gate, out-projection + residual, LayerNorm,
// FF1 + GELU, FF2 + residual), the final norm, the heads and the sampling + Sim step — with the
// activations in LDS.  Same semantics as the multi-launch step (k_embed / dgemm / k_attn_decode /
// k_mlp / k_heads_sample); the products are plain fp32 FMAs (different summation order, fp32
// rounding level).  The multi-launch step pays ~15 dependent launches whatever the live count
// (C2's long tail: one or two live episodes for hundreds of steps; a scalar host env: one row per
// step); here a step is one launch whose time is the row's weight stream (k-major copies, float4
// per lane, L2-resident for d <= 128) plus its dependent latency chain.
// ROW_T threads; workgroup b takes live rows b, b + gridDim.x, ...
// ---------------------------------------------------------------------------------------------
constexpr int ROW_T = 512;      // 8 waves (2 per SIMD, up to 256 VGPRs: no spills), 8 float4 loads in flight per lane
constexpr int ROW_PART = 4096;  // GEMV partial sums: k-groups x N <= 8 x ROW_T floats
// k-groups of a row GEMV at most: fewer groups = a longer per-thread chain of in-flight loads and
// FMAs but fewer partial rows to sum after the barrier.  32 / 16 / 8 / 4 (tools/r06_kg*.sh, phase
// stamps at the lander_host shape): 63.8 / 62.2 / 59.6 / 64.1 us a step (the out-projection 1.44 ->
// 0.96 us, FF2 2.04 -> 1.72; at 4 FF2's 48-deep chains lose), C2 rollout 27.3 / 26.9 / 27.0 / 29.0 ms
#ifndef ROW_KG_MAX
#define ROW_KG_MAX 8
#endif

// out[n] = act(sum_k x[k] WT[k ldw + n] + bias[n]) (+ res[n]) for n < N (N % 4 == 0, k-major WT, 16-byte
// aligned rows).  The ROW_T threads form KG = ROW_T / (N / 4) k-groups (at most 32) x N / 4 float4
// columns: thread (g, c4) sums its k-group's k sequentially (8 loads in flight), the KG partial rows
// meet in LDS in group order.  ACT: 0 none, 1 GELU, 2 SiLU.  Called by every thread of the workgroup.
template <int ACT>
__device__ __forceinline__ void row_gemv(const float* x, int K, const float* WT, int ldw, const float* bias, int N,
                                         float* out, float* part, const float* res = nullptr) {
  const int tid = threadIdx.x, NC4 = N >> 2;
  const int KG = NC4 >= ROW_T ? 1 : min(ROW_KG_MAX, ROW_T / NC4);
  const int Kc = (K + KG - 1) / KG;
  // the bias of this thread's first two output columns, loaded beside the weights (after the
  // barrier below it would be one more dependent round trip)
  float bpre[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = tid + ROW_T * j;
    bpre[j] = (bias && n < N) ? bias[n] : 0.f;
  }
  for (int item = tid; item < KG * NC4; item += ROW_T) {
    const int g = item / NC4, n4 = 4 * (item - g * NC4);
    const int k0 = g * Kc, k1 = min(K, k0 + Kc);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* wp = WT + n4;
#pragma unroll 8
    for (int k = k0; k < k1; ++k) {
      const float xv = x[k];
      const float4 wv = *reinterpret_cast<const float4*>(wp + (int64_t)k * ldw);
      acc.x = fmaf(xv, wv.x, acc.x);
      acc.y = fmaf(xv, wv.y, acc.y);
      acc.z = fmaf(xv, wv.z, acc.z);
      acc.w = fmaf(xv, wv.w, acc.w);
    }
    *reinterpret_cast<float4*>(part + g * N + n4) = acc;
  }
  __syncthreads();
  for (int n = tid, j = 0; n < N; n += ROW_T, ++j) {
    // the KG partial rows in group order, 8 LDS loads in flight per batch (one load per add left
    // every add waiting a full LDS latency: ~2.9 k cycles for KG = 32, tools/row_phase_lab.hip)
    float v = part[n];
    for (int g0 = 1; g0 < KG; g0 += 8) {
      float pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) pv[u] = part[min(g0 + u, KG - 1) * N + n];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (g0 + u < KG) v += pv[u];
    }
    v += bias ? (j == 0 ? bpre[0] : (j == 1 ? bpre[1] : bias[n])) : 0.f;
    if constexpr (ACT == 1) v = geluf_(v);
    if constexpr (ACT == 2) v = siluf_(v);
    if (res) v += res[n];
    out[n] = v;
  }
  __syncthreads();
}

// out[c] = LayerNorm(x)[c] * g[c] (x-transformers: no affine, eps 1e-5, two-pass) by wave 0; d <= 256
__device__ __forceinline__ void row_layernorm(const float* x, const float* g, int d, float* out, bool rms) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    float v[4], gv[4], sm = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // (the gain issued first: its round trip overlaps the reductions)
      const int c = tid + 64 * k;
      gv[k] = c < d ? g[c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = tid + 64 * k;
      v[k] = c < d ? x[c] : 0.f;
      sm += v[k];
    }
    const float mean = rms ? 0.f : wave_sum_dpp(sm) / (float)d;
    float qq = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float dl = v[k] - mean;
      qq += tid + 64 * k < d ? dl * dl : 0.f;
    }
    const float rstd = norm_rstd(wave_sum_dpp(qq), (float)d, rms);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = tid + 64 * k;
      if (c < d) out[c] = ((v[k] - mean) * rstd) * gv[k];
    }
  }
  __syncthreads();
}

struct RowLds {   // floats, carved from the dynamic LDS
  int x, xn, qkv, att, v1, h, ac, part, sc, lg, tot;
};
__host__ __device__ inline RowLds row_lds(const XtrlDecodeDesc& D) {
  RowLds o;
  const int I = D.H * D.dh, nq = round4i(D.n_qkv), hw = D.ff > 4 * D.d ? D.ff : 4 * D.d;
  const int n2 = round4i((D.continuous ? 2 * D.A : D.A) + D.B);
  int at = 0;
  o.x = at; at += round4i(D.d);
  o.xn = at; at += round4i(D.d);
  o.qkv = at; at += nq;
  o.att = at; at += round4i(I);
  o.v1 = at; at += round4i(I);
  o.h = at; at += round4i(hw);
  o.ac = at; at += round4i(D.in_dim);
  o.part = at; at += ROW_PART + n2;   // partial rows (+ the heads' output row behind them)
  o.sc = at; at += D.H * (round4i(D.Tmax) + 64);   // per head: the scores, then the new value row
  o.lg = at; at += 64;
  o.tot = at;
  return o;
}

constexpr int ROW_MAX_L = 64;
// phase stamps of the row-resident step (xtrl_row_stamps, diagnostics): thread 0 of workgroup 0
// records the wall clock after each phase of its first row — start, compaction, embedding, 7 per
// layer (LN, q|k|v, attention, out-projection, LN, FF1, FF2), final LN, hidden, last Linear, sample
constexpr int ROW_STAMP_MAX = 8 + 7 * ROW_MAX_L;
__device__ int g_row_stamp_on;
__device__ uint64_t g_row_stamps[2 * ROW_STAMP_MAX];   // wall clock | shader clock (s_memtime)
constexpr int ROW_G = 4;      // workgroups per row at most (the heads split across them)
constexpr int ROW_CUS = 256;  // (rows x workgroups per row kept within one workgroup per CU)

// The gated host-env step (xtrl_host_row_step; one workgroup, E == 1): the launch is queued ahead of
// the host's env step; thread 0 waits for the host's step counter in pinned memory (go >= go_val,
// system-scope acquire loads, s_sleep between polls), the workgroup applies the env's results of step
// t - 1 from the pinned stage (k_env_feedback's arithmetic), runs decode step t, and thread 0 — the
// thread whose sampling stored the action into pinned memory — publishes go_val in `done` (system
// release).  So neither the launch nor a stream synchronisation sits between the env step and the
// decode.  go == HG_CANCEL: exit at once (the host ends the wave); no go within wait_ticks: exit
// untouched, done[1] = go_val (the host falls back to launching the step itself).  done[0] only ever
// holds completed steps, so a later launch giving up cannot hide an earlier completion.
struct HostGate {
  const uint32_t* go;   // null: not gated
  uint32_t* done;        // [0] the last completed step's go_val, [1] the last go_val that gave up
  const float* stage;   // [E][S] next state | [E] reward | [E] terminated u8 | [E] truncated u8
  uint32_t go_val;
  int t_prev, t_limit, bootstrap;
  uint64_t wait_ticks;   // of the 100 MHz constant clock (XTRL_HOST_GATE_WAIT_MS, default 4000)
};
constexpr uint32_t HG_CANCEL = 0xFFFFFFFFu;

// G > 1: with few live rows, Ge in {4, 2} (<= G, rows x Ge <= 256) workgroups carry each row — every one runs the
// row's embedding and layers (identical arithmetic; only the first stores the shared state), then
// takes 4 d / Ge of the heads' hidden units and its partial of the last Linear; the partials meet
// through k_mlp's hand-off (sc1 stores, one counter per row) and the last arriver sums them in
// workgroup order, adds b2 and samples.  The heads are ~40 % of a row's weight bytes (C2).
template <int DH, int KP = (DH == 16 ? 2 : 1)>   // KP: 64-key K passes per round trip
__global__ __launch_bounds__(ROW_T) void k_decode_row(const XtrlDecodeDesc D, int t, int G, const HostGate hg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ int rows_sh[EMB_MAX_E];
  __shared__ int wsum[ROW_T / 64];
  const RowLds Lo = row_lds(D);
  float *xs = lds + Lo.x, *xn = lds + Lo.xn, *qkv = lds + Lo.qkv, *att = lds + Lo.att, *v1s = lds + Lo.v1;
  float *hs = lds + Lo.h, *ac = lds + Lo.ac, *part = lds + Lo.part, *lg = lds + Lo.lg;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (hg.go) {   // the gated host-env step: the host's go, then the env's results of step t - 1
    __shared__ uint32_t go_sh;
    if (tid == 0) {
      const uint64_t c0 = wall_clock64();
      uint32_t v = __hip_atomic_load(hg.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      while (v < hg.go_val) {
        if (wall_clock64() - c0 > hg.wait_ticks) break;
        __builtin_amdgcn_s_sleep(4);
        v = __hip_atomic_load(hg.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      go_sh = v;
    }
    __syncthreads();
    const uint32_t v = go_sh;
    if (v == HG_CANCEL) return;
    if (v < hg.go_val) {   // the host never came: nothing done, the host takes the step over
      if (tid == 0) __hip_atomic_store(hg.done + 1, hg.go_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    if (hg.t_prev >= 0 && tid < 64) {   // (E == 1; wave 0: one load of the alive byte for every lane)
      const int S = D.S;
      const uint8_t al = D.alive[0];
      if (al == 1 && tid < S) D.state[tid] = hg.stage[tid];   // (the next state, a lane per column)
      if (tid == 0) {
        const uint8_t* fl = reinterpret_cast<const uint8_t*>(hg.stage + (S + 1));
        env_feedback_row(D, 0, al, hg.t_prev, hg.stage, hg.stage + S, fl, fl + 1, hg.t_limit, hg.bootstrap, false);
      }
    }
    __threadfence();   // (agent-scope acquire: no stale L1 line of the fed-back alive / state bytes)
    __syncthreads();
  }
  bool stamp = blockIdx.x == 0 && tid == 0 && g_row_stamp_on;
  int ns = 0;
  auto mark = [&]() {
    if (stamp && ns < ROW_STAMP_MAX) {
      g_row_stamps[ROW_STAMP_MAX + ns] = (uint64_t)clock64();
      g_row_stamps[ns++] = (uint64_t)wall_clock64();
    }
  };
  mark();
  const int S = D.S, d = D.d, H = D.H, I = H * DH, L = D.L;
  // the layer descriptors (pointers) copied to LDS in one batch of vector loads: read lazily from
  // layers_dev, each layer phase's pointers were a cold scalar load ahead of its data (a round trip per phase)
  __shared__ XtrlDecodeLayer ly_sh[ROW_MAX_L];
  {
    constexpr int LW = (int)(sizeof(XtrlDecodeLayer) / sizeof(uint32_t));
    const uint32_t* src = reinterpret_cast<const uint32_t*>(D.layers_dev);
    uint32_t* dst = reinterpret_cast<uint32_t*>(ly_sh);
    for (int i = tid; i < L * LW; i += ROW_T) dst[i] = src[i];   // (visible after the compaction's barriers)
  }
  // ---- compaction (as k_embed<CMP>): every workgroup ranks the live slots itself.  Workgroups that
  //      start late (the grid need not be resident at once) may find rows that others have already
  //      stepped: a Sim row ended at this step reads ALIVE_END + (t & 1) and a bootstrap row keeps
  //      alive 2 through the launch (sample_row row_step) — both still live_at(t) — so every workgroup
  //      ranks the rows live at the step's start, whichever value of the one byte it sees
  // (every chunk's alive byte loaded in one batch, then ranked chunk by chunk)
  int n_live = 0;
  // E <= 64 (a scalar host env, small tests): every wave ballots the alive bytes itself and a row's
  // slot is the r-th set bit of the live mask — no LDS scan, one barrier (the layer descriptors)
  const bool small_e = D.E <= 64;
  uint64_t live_mask = 0;
  if (small_e) {
    const uint8_t a = D.alive[min(lane, D.E - 1)];
    const bool al = lane < D.E && live_at(a, t);
    if (blockIdx.x == 0 && w == 0 && lane < D.E && ended_before(a, t)) D.alive[lane] = 0;
    live_mask = __ballot(al);
    n_live = __popcll(live_mask);
    __syncthreads();
  }
  constexpr int CH = EMB_MAX_E / ROW_T;
  uint8_t alv[CH];
#pragma unroll
  for (int ci = 0; ci < CH; ++ci) {
    const int ec = min(ROW_T * ci + tid, D.E - 1);
    alv[ci] = small_e ? 0 : D.alive[ec];
  }
#pragma unroll
  for (int ci = 0; ci < CH; ++ci) {
    const int c0 = ROW_T * ci;
    if (small_e || c0 >= D.E) break;   // (uniform)
    const int e = c0 + tid;
    const bool al = e < D.E && live_at(alv[ci], t);
    // (a slot ended at step t - 1 is dead here: cleared before step t + 1 reads the same parity)
    if (blockIdx.x == 0 && e < D.E && ended_before(alv[ci], t)) D.alive[e] = 0;
    const uint64_t bal = __ballot(al);
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = n_live, tot = 0;
    for (int i = 0; i < ROW_T / 64; ++i) {
      off += i < w ? wsum[i] : 0;
      tot += wsum[i];
    }
    if (al) rows_sh[off + __popcll(bal & ((1ull << lane) - 1ull))] = e;
    n_live += tot;
    __syncthreads();
  }
  if (blockIdx.x == 0 && tid == 0) D.live_count[t & 1] = n_live;
  mark();
  const int n_act = D.continuous ? 2 * D.A : D.A;
  const int nq4 = round4i(D.n_qkv), n2 = round4i(n_act + D.B), ff = D.ff;
  const float scale = D.attn_scale > 0.f ? D.attn_scale : 1.0f / sqrtf((float)DH);
  constexpr int F4 = DH / 4, LPK = DH / 4, KPI = 64 / LPK;   // P.V: lanes per key row, key rows per wave pass
  // workgroups per row (uniform): 4, 2 or 1 — a divisor of 4 d / 4 hidden units — with rows x Ge <= 256
  const int Ge = min(G, n_live <= ROW_CUS / 4 ? 4 : (n_live <= ROW_CUS / 2 ? 2 : 1));
  const int gs = blockIdx.x % Ge, nrw = (int)gridDim.x / Ge;
  const bool lead = gs == 0;   // stores the row's shared state
  __shared__ int last_sh;
  for (int r = (int)blockIdx.x / Ge; r < n_live && (int)blockIdx.x < nrw * Ge; r += nrw) {
    int e;
    if (small_e) {   // the r-th live slot: clear the r lowest set bits
      uint64_t m = live_mask;
      for (int i = 0; i < r; ++i) m &= m - 1ull;
      e = __builtin_ctzll(m);
    } else {
      e = rows_sh[r];
    }
    if (lead && tid == 0) D.live_rows[(t & 1) * D.E + r] = e;
    // ---- RSNorm of [state, prev reward], embeddings (k_embed's arithmetic and order)
    if (tid <= S) {
      const float xv = tid < S ? D.state[(int64_t)e * S + tid] : D.prev_reward[e];
      part[tid] = (xv - D.rs_mean[tid]) / fmaxf(sqrtf(D.rs_var[tid]), D.rs_eps);
      if (lead && tid < S) D.traj_states[((int64_t)e * D.Tmax + t) * S + tid] = xv;
    }
    __syncthreads();
    if (tid < d) {
      const int c = tid;
      float p = 0.f, se = 0.f;
      for (int sidx = 0; sidx < S; ++sidx) {
        p += part[sidx] * D.w_pin[c * S + sidx];
        se += part[sidx] * D.w_se[c * S + sidx];
      }
      p += D.b_pin ? D.b_pin[c] : 0.f;
      float ak;
      if (D.continuous) {
        float acc = 0.f;
        for (int i = 0; i < D.A; ++i) acc += D.prev_action_f[e * D.A + i] * D.act_emb[c * D.A + i];
        ak = acc + D.act_emb_b[c];
      } else {
        const int a = D.prev_action[e];
        ak = a >= 0 ? D.act_emb[a * d + c] : 0.f;   // SafeEmbedding: -1 -> 0
      }
      if (D.state_only) ak = 0.f;
      const float rew = (D.no_reward_cond || D.state_only) ? 0.f : part[S] * D.reward_embed[c];
      xs[c] = p + (ak + rew);
      ac[d + c] = se + D.b_se[c];
      if (D.evolutionary && D.lat_embed) ac[2 * d + c] = D.lat_embed[(int64_t)e * d + c];
    }
    __syncthreads();
    mark();
    // ---- decoder layers
    for (int l = 0; l < L; ++l) {
      const XtrlDecodeLayer& Ly = ly_sh[l];   // (the LDS copy of layers_dev)
      row_layernorm(xs, Ly.ln_attn, d, xn, D.rms_norm);
      mark();
      row_gemv<0>(xn, d, Ly.w_qkv_t, nq4, Ly.b_qkv, nq4, qkv, part);
      mark();
      // attention: head h on wave h (waves past H idle); k_attn_decode's arithmetic and lane roles
      for (int h = w; h < H; h += ROW_T / 64) {
        const int c = lane % DH, g = lane / DH;
        float* sc = lds + Lo.sc + h * (round4i(D.Tmax) + 64);
        float q = qkv[h * DH + c], k = qkv[I + h * DH + c], v = qkv[2 * I + h * DH + c];
        if (D.value_residual) {
          if (l == 0) {
            if (g == 0) {
              v1s[h * DH + c] = v;
              if (lead) D.v1[(int64_t)r * I + h * DH + c] = v;
            }
          } else if (D.learned_mix) {
            v = lerpf_(v, v1s[h * DH + c], sigmoidf_(qkv[3 * I + (D.gate_values ? I : 0) + h]));
          }
        }
        if (D.qk_norm) qk_l2norm<DH>(q, k);
        if (D.rotary_abs && c < D.rot_dim) rotary_row(D, t, c, q, k);
        const int64_t cb = ((int64_t)e * H + h) * D.Tmax * DH;
        if (g == 0) {
          if (lead) {
            Ly.k_cache[cb + (int64_t)t * DH + c] = k;
            Ly.v_cache[cb + (int64_t)t * DH + c] = v;
          }
          sc[round4i(D.Tmax) + c] = v;   // (the new value row, read by the P.V lanes below; q is broadcast
          att[h * DH + c] = q;           //  from LDS, its head's att slot is written only after the scores)
        }
        float kn = 0.f;
        if constexpr (DH == 16) {   // a row of 16 lanes holds the head's q and k: DPP row sum (no permutes)
          kn = kpi_sum<16>(q * k);
        } else {
#pragma unroll
          for (int i = 0; i < DH; ++i) kn += __shfl(q, i, 64) * __shfl(k, i, 64);
        }
        kn *= scale;   // the new key's score, k_attn_decode's channel order
        wave_sync();
        const float4* q4 = reinterpret_cast<const float4*>(att + h * DH);
        // scores of the cached keys, one key per lane, NP 64-key passes in flight
        constexpr int NP = KP;   // (DH 16: 128 keys per round trip; 256 measured slower: C2 rollout
                                 //  31.06-31.26 vs 30.80-30.92 ms, A/B x3)
        float mx = kn;
        for (int j0 = 0; j0 < t; j0 += 64 * NP) {
          float4 kr[NP][F4];
#pragma unroll
          for (int u = 0; u < NP; ++u) {
            const int j = min(j0 + lane + 64 * u, t - 1);
#pragma unroll
            for (int i = 0; i < F4; ++i) kr[u][i] = reinterpret_cast<const float4*>(Ly.k_cache + cb + (int64_t)j * DH)[i];
          }
#pragma unroll
          for (int u = 0; u < NP; ++u) {
            const int j = j0 + lane + 64 * u;
            float s_ = 0.f;
#pragma unroll
            for (int i = 0; i < F4; ++i) {
              const float4 qv = q4[i];
              s_ += qv.x * kr[u][i].x;
              s_ += qv.y * kr[u][i].y;
              s_ += qv.z * kr[u][i].z;
              s_ += qv.w * kr[u][i].w;
            }
            s_ *= scale;
            if (j < t) {
              sc[j] = s_;
              mx = fmaxf(mx, s_);
            }
          }
        }
        mx = wave_max_dpp(mx);
        float sum = 0.f;
        for (int j = lane; j < t; j += 64) {
          const float p = expf(sc[j] - mx);
          sc[j] = p;
          sum += p;
        }
        const float pn = expf(kn - mx);
        sum = wave_sum_dpp(sum) + pn;
        wave_sync();
        // P.V: lane (kk = key in a pass, cq = channel quad), float4 value rows, 8 passes in flight
        const int kk = lane % KPI, cq = lane / KPI;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        constexpr int VB = 8;   // value rows in flight per lane (128 / 64 / 32 keys a pass; 16 spilled)
        for (int j0 = 0; j0 < t; j0 += VB * KPI) {
          float4 vr[VB];
#pragma unroll
          for (int u = 0; u < VB; ++u) {
            const int j = min(j0 + kk + KPI * u, t - 1);
            vr[u] = *reinterpret_cast<const float4*>(Ly.v_cache + cb + (int64_t)j * DH + 4 * cq);
          }
#pragma unroll
          for (int u = 0; u < VB; ++u) {
            const int j = j0 + kk + KPI * u;
            const float p = j < t ? sc[j] : 0.f;
            acc.x += p * vr[u].x;
            acc.y += p * vr[u].y;
            acc.z += p * vr[u].z;
            acc.w += p * vr[u].w;
          }
        }
        acc.x = kpi_sum<KPI>(acc.x);
        acc.y = kpi_sum<KPI>(acc.y);
        acc.z = kpi_sum<KPI>(acc.z);
        acc.w = kpi_sum<KPI>(acc.w);
        if (kk == 0) {   // + the new key's term, normalise, gate
          const float* vn = sc + round4i(D.Tmax) + 4 * cq;
          float o4[4] = {(acc.x + pn * vn[0]) / sum, (acc.y + pn * vn[1]) / sum, (acc.z + pn * vn[2]) / sum,
                         (acc.w + pn * vn[3]) / sum};
          if (D.gate_values) {
#pragma unroll
            for (int i = 0; i < 4; ++i) o4[i] *= sigmoidf_(qkv[3 * I + h * DH + 4 * cq + i]);
          }
          *reinterpret_cast<float4*>(att + h * DH + 4 * cq) = make_float4(o4[0], o4[1], o4[2], o4[3]);
        }
      }
      __syncthreads();
      mark();
      // out-projection + residual (W_out^T is k-major), then FF: LN, FF1 + GELU, FF2 + residual
      row_gemv<0>(att, I, Ly.w_out_t, d, nullptr, d, xs, part, xs);
      mark();
      row_layernorm(xs, Ly.ln_ff, d, xn, D.rms_norm);
      mark();
      row_gemv<1>(xn, d, Ly.w_ff1_t, ff, Ly.b_ff1, ff, hs, part);
      mark();
      row_gemv<0>(hs, ff, Ly.w_ff2_t, d, Ly.b_ff2, d, xs, part, xs);
      mark();
    }
    // ---- heads: [final LN(x) | state embed | latent] -> SiLU hidden -> block-diagonal last layer
    row_layernorm(xs, D.ln_final, d, ac, D.rms_norm);
    mark();
    const int hw = 4 * d / Ge, hc0 = gs * hw;   // this workgroup's hidden units
    row_gemv<2>(ac, D.in_dim, D.w_h1_t + hc0, 4 * d, D.b_h1 + hc0, hw, hs, part);
    mark();
    float* out2 = part + ROW_PART;
    row_gemv<0>(hs, hw, D.w_h2_t + (int64_t)hc0 * n2, n2, Ge == 1 ? D.b_h2 : nullptr, n2, out2, part);
    mark();
    if (Ge > 1) {   // the partials meet (k_mlp's hand-off); the last arriver sums them in order + b2
      float* rp = D.row_part + (int64_t)r * ROW_G * n2;
      for (int n = tid; n < n2; n += ROW_T)
        __hip_atomic_store(rp + gs * n2 + n, out2[n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        last_sh = __hip_atomic_fetch_add(D.row_cnt + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(Ge - 1);
      __syncthreads();
      if (!last_sh) continue;   // (workgroup-uniform)
      for (int n = tid; n < n2; n += ROW_T) {
        float pv[ROW_G];
#pragma unroll
        for (int g2 = 0; g2 < ROW_G; ++g2)
          pv[g2] = __hip_atomic_load(rp + min(g2, Ge - 1) * n2 + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float v = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < ROW_G; ++g2)
          if (g2 < Ge) v += pv[g2];
        out2[n] = v + D.b_h2[n];
      }
      if (tid == 0) __hip_atomic_store(D.row_cnt + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
    }
    for (int n = tid; n < n_act + D.B; n += ROW_T) {
      if (n < n_act) {
        lg[n] = out2[n];
        D.logits[(int64_t)r * n_act + n] = out2[n];
      } else {
        D.traj_values[((int64_t)e * D.Tmax + t) * D.B + (n - n_act)] = out2[n];
      }
    }
    __syncthreads();
    if (tid < SAMPLE_L) {
      const SampleIn in = sample_load(D, e);
      sample_row(D, t, e, tid, lg, in, true);
    }
    __syncthreads();
    mark();
    stamp = false;   // (the first row only)
  }
  if (hg.go) {   // thread 0 stored the row's action into pinned memory (sample_row): publish the step
    __syncthreads();
    if (tid == 0) {
      __threadfence_system();
      __hip_atomic_store(hg.done, hg.go_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

bool row_ok(const XtrlDecodeDesc* D) {
  if (D->ff_glu || !D->layers_dev || !D->w_h1_t || !D->w_h2_t || D->d > 256 || D->E > EMB_MAX_E || (D->continuous ? 2 * D->A : D->A) > 64 ||
      D->L > ROW_MAX_L)
    return false;
  for (int l = 0; l < D->L; ++l)
    if (!D->layers[l].w_qkv_t || !D->layers[l].w_ff1_t || !D->layers[l].w_ff2_t || !D->layers[l].w_out_t) return false;
  return D->ff % 4 == 0 && (size_t)row_lds(*D).tot * sizeof(float) <= 96 * 1024;
}

}  // namespace

int decode_step(const XtrlDecodeDesc* D, int t, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  XTRL_REQUIRE(t >= 0 && t < D->Tmax, "decode: t=%d outside [0, %d)", t, D->Tmax);
  const int d = D->d, I = D->H * D->dh, ff = D->ff;
  int rc;
  // xn: the LayerNorm of a row computed by the kernel that completes it (embedding -> layer 0's
  // q|k|v, fused attention -> FF1, fused feed-forward -> the next q|k|v or the heads); the other
  // pre-norms run in the GEMM prologue
  const bool xn = D->xn != nullptr;
  if ((rc = launch_embed(D, t, xn ? D->layers[0].ln_attn : nullptr, s))) return rc;
  for (int l = 0; l < D->L; ++l) {
    const XtrlDecodeLayer& Ly = D->layers[l];
    const bool xn_qkv = xn && (l == 0 || mlp_fused(D, l - 1)), xn_ff = xn && attn_fused(D, l);
    if ((rc = dproj(D, t, xn_qkv ? D->xn : D->x, d, Ly.w_qkv, d, Ly.b_qkv, xn_qkv ? nullptr : Ly.ln_attn,
                    xn_qkv ? 0 : d, nullptr, 0, D->qkv, D->n_qkv, D->n_qkv, EPI_NONE, s)))
      return rc;
    if (D->prof_events) (void)hipEventRecord((hipEvent_t)D->prof_events[2 * (t * D->L + l)], s);
    if ((rc = launch_attn_decode(D, l, t, s))) return rc;
    if (D->prof_events) (void)hipEventRecord((hipEvent_t)D->prof_events[2 * (t * D->L + l) + 1], s);
    if (!attn_fused(D, l) &&
        (rc = dproj(D, t, D->att, I, Ly.w_out, I, nullptr, nullptr, 0, D->x, d, D->x, d, d, EPI_NONE, s)))
      return rc;
    // the last layer's output goes straight into the heads' input row (final norm in their prologue)
    const bool last = l == D->L - 1;
    if (mlp_fused(D, l)) {   // FF1 + GELU + FF2 + residual + the next pre-norm: one launch
      if ((rc = launch_mlp(D, l, t, s))) return rc;
      continue;
    }
    if (D->ff_glu) {   // the GLU projection [2 ff], then value * gelu(gate)
      if ((rc = dproj(D, t, xn_ff ? D->xn : D->x, d, Ly.w_ff1, d, Ly.b_ff1, xn_ff ? nullptr : Ly.ln_ff,
                      xn_ff ? 0 : d, nullptr, 0, D->hff, 2 * ff, 2 * ff, EPI_NONE, s)))
        return rc;
      hipLaunchKernelGGL(k_glu_rows, dim3((unsigned)(((int64_t)D->E * ff + 255) / 256)), dim3(256), 0, s, *D, t);
      XTRL_LAUNCHED("glu_rows");
    } else if ((rc = dproj(D, t, xn_ff ? D->xn : D->x, d, Ly.w_ff1, d, Ly.b_ff1, xn_ff ? nullptr : Ly.ln_ff,
                           xn_ff ? 0 : d, nullptr, 0, D->hff, ff, ff, EPI_GELU, s))) {
      return rc;
    }
    const float* h = D->ff_glu ? D->hglu : D->hff;
    if ((rc = dproj(D, t, h, ff, Ly.w_ff2, ff, Ly.b_ff2, nullptr, 0, D->x, d, last ? D->ac_in : D->x,
                    last ? D->in_dim : d, d, EPI_NONE, s)))
      return rc;
  }
  return decode_heads(D, t, !mlp_fused(D, D->L - 1), s);
}


// the row-resident step over the live rows (workgroup b: rows b, b + grid, ...)
int decode_step_rows(const XtrlDecodeDesc* D, int t, int max_rows, hipStream_t s, const HostGate& hg = HostGate{}) {
  if (int rc = check_desc(D)) return rc;
  XTRL_REQUIRE(t >= 0 && t < D->Tmax, "decode rows: t=%d outside [0, %d)", t, D->Tmax);
  XTRL_REQUIRE(row_ok(D), "decode rows: the row-resident step needs the k-major weights (w_*_t), d <= 256, "
                          "E <= %d, at most %d layers, layers_dev and its LDS within 96 KiB", EMB_MAX_E, ROW_MAX_L);
  XTRL_REQUIRE(max_rows > 0, "decode rows: max_rows %d", max_rows);
  // XTRL_ROW_G: workgroups per row at most (1, 2 or 4; default 1 — on one box C2 rollout 30.8–31.7
  // vs 31.3–31.5 ms and the host-env decode step 57.6 vs 74.1 us at 1 vs 4: the redundant layer work
  // and the hand-off cost more than the split heads save; the step is bound by its ~20 dependent
  // phases, not by its weight stream)
  static const int g_env = [] {
    const char* e = getenv("XTRL_ROW_G");
    const int v = e ? atoi(e) : 1;
    return (v == 1 || v == 2 || v == 4) ? v : 1;
  }();
  const int G = (D->row_part && D->row_cnt && D->d % 4 == 0) ? g_env : 1;
  const dim3 grid(std::min(max_rows, D->E) * G);
  const size_t lds = (size_t)row_lds(*D).tot * sizeof(float);
  if (hg.go) XTRL_REQUIRE(grid.x == 1 && D->act_host, "decode rows: the gated host step takes one row (E == 1) "
                                                       "and the pinned action buffer");
  if (D->dh == 16) hipLaunchKernelGGL(k_decode_row<16>, grid, dim3(ROW_T), lds, s, *D, t, G, hg);
  else if (D->dh == 32) hipLaunchKernelGGL(k_decode_row<32>, grid, dim3(ROW_T), lds, s, *D, t, G, hg);
  else hipLaunchKernelGGL(k_decode_row<64>, grid, dim3(ROW_T), lds, s, *D, t, G, hg);
  XTRL_LAUNCHED("decode_row");
  return XTRL_OK;
}

int fractal_decode_step(const XtrlDecodeDesc* D, const XtrlFractalDesc* F, int t, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  XTRL_REQUIRE(F && F->level && F->levels == D->L && F->levels > 0, "fractal_decode: levels mismatch");
  XTRL_REQUIRE(t >= 0 && t < D->Tmax, "fractal_decode: t=%d outside [0, %d)", t, D->Tmax);
  XTRL_REQUIRE(D->state_only && !D->gate_values && !D->value_residual && !D->rotary_abs && !D->qk_norm &&
                   D->n_qkv == 3 * D->H * D->dh && D->d <= 64 * FR_MAXF,
               "fractal_decode: the descriptor must describe plain attention (n_qkv = 3 I) with state_only = 1");
  XTRL_REQUIRE(F->g_init && F->c0 && F->g && F->c2 && F->tmp && F->x2 && F->mean && F->allf && F->hagg,
               "fractal_decode: missing buffers");
  const int E = D->E, d = D->d, I = D->H * D->dh, ff = D->ff, Lv = F->levels;
  const dim3 rows_grid((E + 3) / 4), rows_blk(256);
  if (int rc = launch_embed(D, t, nullptr, s)) return rc;   // x = W_in s + b_in + le_0
  int rc;
  for (int l = 0; l < Lv; ++l) {
    const XtrlFractalLevel& Q = F->level[l];
    // the cross-attention read of the global state (level 0: the same row c0 for every row)
    if (l > 0 &&
        (rc = dproj(D, t, F->g, 2 * d, Q.w_c, d, nullptr, nullptr, 0, nullptr, 0, F->c2, d, d, EPI_NONE, s)))
      return rc;
    if ((rc = dproj(D, t, D->x, d, Q.w_qkv, d, nullptr, nullptr, 0, nullptr, 0, D->qkv, D->n_qkv, 3 * I, EPI_NONE, s)))
      return rc;
    // x2 = LN2(LN1(x + attn W_out^T) + c): inside the attention launch (one workgroup per live row,
    // the head partials of the out-projection meeting in LDS) or as projection + row kernel
    FrPost fp;
    fp.g1 = Q.ln1_w; fp.b1 = Q.ln1_b; fp.g2 = Q.ln2_w; fp.b2 = Q.ln2_b;
    fp.c = l > 0 ? F->c2 : F->c0; fp.ldc = l > 0 ? d : 0; fp.out = F->x2; fp.eps = F->ln_eps;
    const bool fused = attn_fused(D, l);
    if (D->prof_events) (void)hipEventRecord((hipEvent_t)D->prof_events[2 * (t * D->L + l)], s);
    if ((rc = launch_attn_decode(D, l, t, s, fused ? fp : FrPost{}))) return rc;
    if (D->prof_events) (void)hipEventRecord((hipEvent_t)D->prof_events[2 * (t * D->L + l) + 1], s);
    if (!fused) {
      if ((rc = dproj(D, t, D->att, I, Q.w_out, I, nullptr, nullptr, 0, nullptr, 0, F->tmp, d, d, EPI_NONE, s)))
        return rc;
      hipLaunchKernelGGL(k_fr_ln12, rows_grid, rows_blk, 0, s, *D, t, F->tmp, l > 0 ? F->c2 : F->c0, l > 0 ? d : 0,
                         Q.ln1_w, Q.ln1_b, Q.ln2_w, Q.ln2_b, F->x2, F->ln_eps);
      XTRL_LAUNCHED("fractal ln12");
    }
    // s3 = x2 + FF(x2): one launch (k_mlp, split-bf16 weight images) or the two projections
    const XtrlDecodeLayer& Ly = D->layers[l];
    const bool mlp = D->mlp_part && D->mlp_cnt && mlp_weights(Ly) && d % 64 == 0 && d <= 256 &&
                     ff % MLP_HW == 0;
    // x3 = LN3(s3), its running mean, the next level's input: in the k_mlp tail, or a row kernel
    const float* le_next = l + 1 < Lv ? F->level[l + 1].level_emb : nullptr;
    if (mlp) {
      FrMlp fm;
      fm.g3 = Q.ln3_w; fm.b3 = Q.ln3_b; fm.sums = Q.sums; fm.mean = F->mean; fm.le_next = le_next; fm.eps = F->ln_eps;
      if ((rc = launch_mlp_rows(D, l, t, F->x2, F->x2, nullptr, d, nullptr, nullptr, 0, s, fm))) return rc;
    } else {
      if ((rc = dproj(D, t, F->x2, d, Q.w_ff1, d, Q.b_ff1, nullptr, 0, nullptr, 0, D->hff, ff, ff, EPI_GELU, s)))
        return rc;
      if ((rc = dproj(D, t, D->hff, ff, Q.w_ff2, ff, Q.b_ff2, nullptr, 0, F->x2, d, F->tmp, d, d, EPI_NONE, s)))
        return rc;
      hipLaunchKernelGGL(k_fr_ln3_tail, rows_grid, rows_blk, 0, s, *D, t, F->tmp, Q.ln3_w, Q.ln3_b, Q.sums, F->mean,
                         le_next, F->ln_eps);
      XTRL_LAUNCHED("fractal ln3 tail");
    }
    // [g | p_l] = [g | 0] + mean [W_gu; W_p,l]^T + [b_gu; b_p,l]: g in place (level 0 from g_init),
    // the level projection into allf
    if ((rc = dproj(D, t, F->mean, d, Q.w_pg, d, Q.b_pg, nullptr, 0, l > 0 ? F->g : F->g_init, l > 0 ? 2 * d : 0, F->g,
                    2 * d, 2 * d, EPI_NONE, s, nullptr, d, F->allf + (int64_t)l * d, (Lv + 1) * d)))
      return rc;
  }
  hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)(((int64_t)E * d + 255) / 256)), dim3(256), 0, s, F->g, 2 * d,
                     F->allf + (int64_t)Lv * d, (Lv + 1) * d, E, d);
  XTRL_LAUNCHED("copy_rows");
  // final aggregation -> the heads' input row (no final norm: the encoder has none)
  if ((rc = dproj(D, t, F->allf, (Lv + 1) * d, F->w_fa0, (Lv + 1) * d, F->b_fa0, nullptr, 0, nullptr, 0, F->hagg,
                  2 * d, 2 * d, EPI_RELU, s)))
    return rc;
  if ((rc = dproj(D, t, F->hagg, 2 * d, F->w_fa2, 2 * d, F->b_fa2, nullptr, 0, nullptr, 0, D->ac_in, D->in_dim, d,
                  EPI_NONE, s)))
    return rc;
  return decode_heads(D, t, false, s);
}

int rollout_begin(const XtrlDecodeDesc* D, hipStream_t s) {
  if (int rc = check_desc(D)) return rc;
  hipLaunchKernelGGL(k_rollout_begin, dim3((D->E + 255) / 256), dim3(256), 0, s, *D);
  XTRL_LAUNCHED("rollout_begin");
  return XTRL_OK;
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

// host-env loop (Learner.rollout_host), the device half of a step: decode step t (rows_max > 0: the
// row-resident step), the rows' actions to pinned host memory, one stream synchronisation
int host_decode(const XtrlDecodeDesc* D, int t, int rows_max, void* act_host, hipStream_t s) {
  XTRL_REQUIRE(act_host, "host_decode: null action buffer");
  if (int rc = rows_max > 0 ? decode_step_rows(D, t, rows_max, s) : decode_step(D, t, s)) return rc;
  const size_t bytes = (size_t)D->E * (D->continuous ? D->A : 1) * 4;
  const void* src = D->continuous ? (const void*)D->prev_action_f : (const void*)D->prev_action;
  if ((act_host != D->act_host && hipMemcpyAsync(act_host, src, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) ||
      hipStreamSynchronize(s) != hipSuccess) {
    set_error("host_decode: action copy / synchronisation failed");
    return XTRL_E_HIP;
  }
  return XTRL_OK;
}

// the gated form of a host-env step (one row, E == 1): queued ahead, waits on the device for the
// host's go (gate[0] >= t + 1), applies step t - 1's env results from the pinned stage, runs decode
// step t and publishes gate[1] = t + 1 (k_decode_row's HostGate)
int host_row_step(const XtrlDecodeDesc* D, int t, const void* host_stage, int t_limit, int bootstrap, uint32_t* gate,
                  hipStream_t s) {
  XTRL_REQUIRE(host_stage && gate && D && D->E == 1 && t >= 0 && t_limit > 0 && t_limit <= D->Tmax,
               "host_row_step: bad arguments (one row, pinned stage and gate)");
  HostGate hg;
  hg.go = gate;
  hg.done = gate + 1;
  hg.stage = static_cast<const float*>(host_stage);
  hg.go_val = (uint32_t)t + 1u;
  hg.t_prev = t - 1;
  hg.t_limit = t_limit;
  hg.bootstrap = bootstrap;
  const char* we = getenv("XTRL_HOST_GATE_WAIT_MS");   // (read per call: tests shorten it)
  const long wait_ms = we && atol(we) > 0 ? atol(we) : 4000;
  hg.wait_ticks = (uint64_t)wait_ms * 100000ull;
  return decode_step_rows(D, t, 1, s, hg);
}

// ... and the env's results back: the pinned stage [E][S] next state | [E] reward | [E] terminated
// (u8) | [E] truncated (u8) to the device stage (same layout), then the feedback kernel on it
int host_feedback(const XtrlDecodeDesc* D, int t, const void* host_stage, void* dev_stage, int t_limit, int bootstrap,
                  hipStream_t s) {
  XTRL_REQUIRE(host_stage, "host_feedback: null stage");
  const int E = D->E, S = D->S;
  if (dev_stage && hipMemcpyAsync(dev_stage, host_stage, (size_t)4 * E * (S + 1) + 2 * (size_t)E,
                                  hipMemcpyHostToDevice, s) != hipSuccess) {
    set_error("host_feedback: stage copy failed");
    return XTRL_E_HIP;
  }
  // (dev_stage NULL: the feedback kernel reads the pinned stage in place)
  const float* f = static_cast<const float*>(dev_stage ? dev_stage : host_stage);
  const uint8_t* flags = reinterpret_cast<const uint8_t*>(f + (int64_t)E * (S + 1));
  return env_feedback(D, t, f, f + (int64_t)E * S, flags, flags + E, t_limit, bootstrap, s);
}

int sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update, const int32_t* ep, hipStream_t s) {
  XTRL_REQUIRE(state && ep && E > 0 && S > 0, "sim_reset: bad arguments");
  hipLaunchKernelGGL(k_sim_reset, dim3((E + 255) / 256), dim3(256), 0, s, state, E, S, seed, update, ep);
  XTRL_LAUNCHED("sim_reset");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_decode_step_rows(const XtrlDecodeDesc* desc, int t, int max_rows, void* stream) {
  return xtrl::decode_step_rows(desc, t, max_rows, xtrl::as_stream(stream));
}
extern "C" int xtrl_row_stamps(int on, uint64_t* out, int cap, int64_t* ticks_per_sec) {
  XTRL_REQUIRE(cap >= 0 && (cap == 0 || out), "row_stamps: bad arguments");
  if (hipDeviceSynchronize() != hipSuccess) return XTRL_E_HIP;
  const int n = std::min(cap, 2 * xtrl::ROW_STAMP_MAX);
  if (n > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(xtrl::g_row_stamps), n * sizeof(uint64_t)) != hipSuccess)
    return XTRL_E_HIP;
  if (ticks_per_sec) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
      return XTRL_E_HIP;
    *ticks_per_sec = (int64_t)khz * 1000;
  }
  const int v = on ? 1 : 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(xtrl::g_row_stamp_on), &v, sizeof(int)) != hipSuccess) return XTRL_E_HIP;
  return xtrl::ROW_STAMP_MAX;
}
extern "C" int xtrl_decode_step(const XtrlDecodeDesc* desc, int t, void* stream) {
  return xtrl::decode_step(desc, t, xtrl::as_stream(stream));
}
extern "C" int xtrl_rollout_begin(const XtrlDecodeDesc* desc, void* stream) {
  return xtrl::rollout_begin(desc, xtrl::as_stream(stream));
}
extern "C" int xtrl_rollout_env_feedback(const XtrlDecodeDesc* desc, int t, const float* next_state,
                                         const float* reward, const uint8_t* terminated, const uint8_t* truncated,
                                         int t_limit, int bootstrap, void* stream) {
  return xtrl::env_feedback(desc, t, next_state, reward, terminated, truncated, t_limit, bootstrap,
                            xtrl::as_stream(stream));
}
extern "C" int xtrl_host_decode(const XtrlDecodeDesc* desc, int t, int rows_max, void* act_host, void* stream) {
  return xtrl::host_decode(desc, t, rows_max, act_host, xtrl::as_stream(stream));
}
extern "C" int xtrl_host_row_step(const XtrlDecodeDesc* desc, int t, const void* host_stage, int t_limit, int bootstrap,
                                  uint32_t* gate, void* stream) {
  return xtrl::host_row_step(desc, t, host_stage, t_limit, bootstrap, gate, xtrl::as_stream(stream));
}
// the host half: spin until done[0] >= value (0), done[1] >= value — the awaited launch (or, once it
// gave up, a later one) found no go in time (1) — or timeout_s passed on the host (-1)
extern "C" int xtrl_host_wait(const uint32_t* done, uint32_t value, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0;; ++spin) {
    if (__atomic_load_n(done, __ATOMIC_ACQUIRE) >= value) return 0;
    if (__atomic_load_n(done + 1, __ATOMIC_ACQUIRE) >= value) return 1;
    if ((spin & 1023u) == 0u &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return -1;
    __builtin_ia32_pause();
  }
}
extern "C" int xtrl_host_feedback(const XtrlDecodeDesc* desc, int t, const void* host_stage, void* dev_stage,
                                  int t_limit, int bootstrap, void* stream) {
  return xtrl::host_feedback(desc, t, host_stage, dev_stage, t_limit, bootstrap, xtrl::as_stream(stream));
}
extern "C" int xtrl_sim_reset(float* state, int E, int S, uint64_t seed, uint32_t update,
                              const int32_t* episode_of_slot, void* stream) {
  return xtrl::sim_reset(state, E, S, seed, update, episode_of_slot, xtrl::as_stream(stream));
}
extern "C" int xtrl_fractal_decode_step(const XtrlDecodeDesc* desc, const XtrlFractalDesc* fd, int t, void* stream) {
  return xtrl::fractal_decode_step(desc, fd, t, xtrl::as_stream(stream));
}
