// Training attention for the learn step: causal + key-padding mask, softmax in fp32, post-softmax
// dropout (x-transformers Attend, called from WorldModelActorCritic.forward in Agent.learn,
// x_transformers_rl.py:928-935 with mask = arange(n) < episode_lens, :908-909).
//
// All products run on the f32 matrix cores (v_mfma_f32_16x16x4_f32):
//   forward   S = Q K^T, online softmax, O = P~ V              (flash style, no n x n in HBM)
//   backward  D = rowsum(dO * O); dK, dV per key tile; dQ per query tile (no atomics, deterministic)
// Geometry: 64-row tiles, 4 waves x 16 rows; K/V (or Q/dO) tiles staged in LDS with a 2-float
// row pad; the probability tile crosses LDS once per wave to turn the MFMA C layout (rows on
// lane groups) into the A layout (rows on lanes), in a 66-float-stride image (conflict-free read).
// Dropout keep bits, with c2 = offset + b*H + h (sub = the decoder layer / fractal level):
//   byte mode (256 p an integer, e.g. p = 0.25): byte (i & 3) of word ((j >> 4) & 3) of
//     philox(seed; i >> 2, 16 (j >> 6) + (j & 15), c2, FIELD_DROPOUT << 24 | (sub | 1 << 23)) >= 256 p —
//     one block covers rows 4 (i >> 2) + 0..3 and columns j, j + 16, j + 32, j + 48 of a 64-key tile:
//     exactly the 16 scores one lane holds in the forward and dQ kernels (one block per lane and tile)
//   word mode: word (i & 3) of philox(seed; i >> 2, j, c2, FIELD_DROPOUT << 24 | sub) >= p 2^32.
#include "kernels.h"
#include "philox.h"

namespace xtrl {
namespace {

constexpr int TQ = 64, TK = 64, PST = 66;

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t keep_word(uint64_t seed, uint32_t off, uint32_t c3, int i, int j) {
  const u32x4_t r = philox4x32_10((uint32_t)(i >> 2), (uint32_t)j, off, c3, seed);
  const int w = i & 3;
  return w == 0 ? r.x : (w == 1 ? r.y : (w == 2 ? r.z : r.w));
}
__device__ __forceinline__ uint32_t qword(const u32x4_t& u, int r) {
  return r == 0 ? u.x : (r == 1 ? u.y : (r == 2 ? u.z : u.w));
}
// byte-mode keep byte (row & 3) of word (16-column group) of a lane's block
__device__ __forceinline__ uint32_t qbyte(const u32x4_t& u, int word, int r) {
  return (qword(u, word) >> (8 * r)) & 0xFFu;
}

struct AttnArgs {
  const float *Q, *K, *V, *O, *LSE, *dO, *Dl, *G;
  float *Oout, *LSEout, *dQ, *dK, *dV, *Dout, *OGout;
  float* dQp;         // k_attn_bwd_dkdv<DH, true>: per-key-tile dQ partials [n_key_tiles][b H][n][DH]
  const int32_t* ep_off;   // packed rows: episode b's tokens are rows ep_off[b] .. + min(lens[b], n) - 1
  const int32_t* lens;
  int H, n;
  AttnLayout in, out, grad, gate;   // q/k/v; o/do/og; dq/dk/dv; gate
  float scale, inv_keep;
  uint32_t thresh;    // keep iff word >= thresh (thresh = 0: no dropout)
  uint32_t thresh8;   // != 0: byte mode, keep iff byte >= thresh8
  uint64_t seed;
  uint32_t offset;
  uint32_t c3;        // rng_c3(FIELD_DROPOUT, layer); byte mode: rng_c3(FIELD_DROPOUT, layer | 1 << 23)
  int causal;
};

// first row of episode b in layout L: b * sb (padded [b][n] tokens), or ep_off[b] rows (packed)
__device__ __forceinline__ int64_t ebase(const AttnArgs& a, const AttnLayout& L, int b) {
  return a.ep_off ? (int64_t)a.ep_off[b] * L.si : (int64_t)b * L.sb;
}

// ---------------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(256) void k_attn_fwd(const AttnArgs a) {
  constexpr int KS = DH / 4, ND = DH / 16, KST = DH + 2;
  __shared__ float Ks[TK][KST], Vs[TK][KST];
  __shared__ float Ps[4][16][PST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int bh = blockIdx.y, b = bh / a.H, ns = a.n;
  const int q0 = blockIdx.x * TQ;
  const int len = a.lens[b];
  const int n = a.ep_off ? min(len, ns) : ns;   // packed rows: the episode's own length
  const int h = bh - b * a.H;
  if (q0 >= n) return;   // (packed rows: a query tile past the episode; workgroup-uniform)
  const int64_t ib = ebase(a, a.in, b) + h * a.in.sh, ob = ebase(a, a.out, b) + h * a.out.sh;
  const int isi = a.in.si, osi = a.out.si;
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t off = a.offset + (uint32_t)bh;

  float qa[KS];
  {
    const int i = q0 + 16 * w + lr;
#pragma unroll
    for (int s = 0; s < KS; ++s) qa[s] = (i < n) ? a.Q[ib + (int64_t)i * isi + 4 * s + lg] : 0.f;
  }
  float m[4], l[4];
  f32x4v o[ND];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int last_key = min(min(a.causal ? q0 + TQ - 1 : n - 1, n - 1), len - 1);
  for (int kt = 0; kt * TK <= last_key; ++kt) {
    __syncthreads();
    for (int x = tid; x < TK * DH; x += 256) {
      const int j = x / DH, c = x - j * DH, jj = kt * TK + j;
      Ks[j][c] = jj < n ? a.K[ib + (int64_t)jj * isi + c] : 0.f;
      Vs[j][c] = jj < n ? a.V[ib + (int64_t)jj * isi + c] : 0.f;
    }
    __syncthreads();
    f32x4v sacc[4];
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      sacc[sub] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) sacc[sub] = mfma16(qa[s], Ks[16 * sub + lr][4 * s + lg], sacc[sub]);
    }
    // keep words: this lane's rows q0 + 16 w + 4 lg + 0..3 share one Philox block per key column
    // (word = row & 3), so one block per column instead of one per element
    u32x4_t kws[4] = {};
    if (a.thresh8) {   // byte mode: one block holds all 16 keep bytes of this lane's scores
      kws[0] = philox4x32_10((uint32_t)((q0 + 16 * w + 4 * lg) >> 2), (uint32_t)(kt * 16 + lr), off, a.c3, a.seed);
    } else if (a.thresh) {
#pragma unroll
      for (int sub = 0; sub < 4; ++sub)
        kws[sub] = philox4x32_10((uint32_t)((q0 + 16 * w + 4 * lg) >> 2), (uint32_t)(kt * TK + 16 * sub + lr), off,
                                 a.c3, a.seed);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q0 + 16 * w + 4 * lg + r;
      float sv[4];
      float mx = -INFINITY;
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const int j = kt * TK + 16 * sub + lr;
        const bool ok = (j <= i || !a.causal) && (j < len);
        sv[sub] = ok ? sacc[sub][r] * a.scale : -INFINITY;
        mx = fmaxf(mx, sv[sub]);
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, 64));
      const float mnew = fmaxf(m[r], mx);
      const float alpha = (m[r] == -INFINITY) ? 0.f : expf(m[r] - mnew);
      float rs = 0.f;
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const float p = (sv[sub] == -INFINITY) ? 0.f : expf(sv[sub] - mnew);
        rs += p;
        float pd = p;
        if (a.thresh8) pd = (qbyte(kws[0], sub, r) >= a.thresh8) ? p * a.inv_keep : 0.f;
        else if (a.thresh) pd = (qword(kws[sub], r) >= a.thresh) ? p * a.inv_keep : 0.f;
        Ps[w][4 * lg + r][16 * sub + lr] = pd;
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) rs += __shfl_xor(rs, o2, 64);
      l[r] = l[r] * alpha + rs;
      m[r] = mnew;
#pragma unroll
      for (int d = 0; d < ND; ++d) o[d][r] *= alpha;
    }
    wave_sync();
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int s = 0; s < TK / 4; ++s) o[d] = mfma16(Ps[w][lr][4 * s + lg], Vs[4 * s + lg][16 * d + lr], o[d]);
    wave_sync();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q0 + 16 * w + 4 * lg + r;
    if (i < n) {
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int64_t at = ob + (int64_t)i * osi + 16 * d + lr;
        const float ov = o[d][r] / l[r];
        a.Oout[at] = ov;
        if (a.OGout)   // gated values (x-transformers attn_gate_values)
          a.OGout[at] = ov * sigmoidf_(a.G[ebase(a, a.gate, b) + h * a.gate.sh + (int64_t)i * a.gate.si + 16 * d + lr]);
      }
      if (lr == 0) a.LSEout[(int64_t)bh * ns + i] = m[r] + logf(l[r]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// DQ (long episodes, n > FB_MAXN): the dQ kernel's pass is folded in as in k_attn_bwd_fused — per
// (key tile, query tile) pair, once the four waves' dS images are in LDS, wave w multiplies its 16
// query rows of dS by the key tile (staged once per workgroup) — but the key tiles stay spread over
// the grid: a query row whose only contributing key tile is tile 0 (query tile 0, or an episode of
// <= 64 steps: min(qt, (len - 1) / 64) = 0) gets dQ written here, bit-identical to k_attn_bwd_dq;
// the other rows get one partial per contributing key tile in dQp, summed in ascending key-tile
// order by k_attn_dq_reduce.  (141 registers, 3 waves per SIMD: held to 128 it spilled 12.)
template <int DH, bool DQ = false>
__global__ __launch_bounds__(256, DH == 16 ? (DQ ? 3 : 4) : 1) void k_attn_bwd_dkdv(const AttnArgs a) {
  constexpr int KS = DH / 4, ND = DH / 16, KST = DH + 2;
  __shared__ float Qs[TQ][KST], dOs[TQ][KST];
  __shared__ float Ks[DQ ? TK : 1][KST];
  __shared__ float Ls[TQ], Dls[TQ];
  // one per-wave tile image, used for P~ (dV) and then for dS (dK): 26.6 KB of LDS per workgroup,
  // six resident per CU; at dh = 16 the register budget is held to 128 (4 waves per SIMD: 168 gave
  // 3, and a quarter of the C3 grid ran as a second round), so the C3 grid is one round
  __shared__ float Ps[4][16][PST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int bh = blockIdx.y, b = bh / a.H, ns = a.n;
  const int j0 = blockIdx.x * TK;
  const int len = a.lens[b];
  const int n = a.ep_off ? min(len, ns) : ns;   // packed rows: the episode's own length
  const int h = bh - b * a.H;
  const int64_t ib = ebase(a, a.in, b) + h * a.in.sh, ob = ebase(a, a.out, b) + h * a.out.sh, gb = ebase(a, a.grad, b) + h * a.grad.sh;
  const int isi = a.in.si, osi = a.out.si, gsi = a.grad.si;
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t off = a.offset + (uint32_t)bh;

  float ka[KS], va[KS];
  {
    const int j = j0 + 16 * w + lr;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      ka[s] = (j < n) ? a.K[ib + (int64_t)j * isi + 4 * s + lg] : 0.f;
      va[s] = (j < n) ? a.V[ib + (int64_t)j * isi + 4 * s + lg] : 0.f;
    }
  }
  f32x4v dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    dk[d] = f32x4v{0.f, 0.f, 0.f, 0.f};
    dv[d] = f32x4v{0.f, 0.f, 0.f, 0.f};
  }
  const int kmax = len > 0 ? (len - 1) / TK : 0;   // DQ: the last key tile holding a valid key
  if constexpr (DQ) {
    for (int x = tid; x < TK * DH; x += 256) {
      const int j = x / DH, c = x - j * DH, jj = j0 + j;
      Ks[j][c] = jj < n ? a.K[ib + (int64_t)jj * isi + c] : 0.f;
    }
    if (j0 == 0 && len <= 0) {   // no valid key: the rows' dQ is 0, this workgroup its only writer
      for (int x = tid; x < n * DH; x += 256) {
        const int i = x / DH, c = x - i * DH;
        a.dQ[gb + (int64_t)i * gsi + c] = 0.f;
      }
    }
  }
  if (j0 < len) {
    for (int qt = j0 / TQ; qt * TQ < n; ++qt) {
      __syncthreads();
      for (int x = tid; x < TQ * DH; x += 256) {
        const int i = x / DH, c = x - i * DH, ii = qt * TQ + i;
        Qs[i][c] = ii < n ? a.Q[ib + (int64_t)ii * isi + c] : 0.f;
        dOs[i][c] = ii < n ? a.dO[ob + (int64_t)ii * osi + c] : 0.f;
      }
      // D_i = rowsum(dO_i * O_i) of the tile's query rows, computed here (the O row in registers
      // while the tile stages) in the order of a sequential sum over the head dimension; the
      // key-tile-0 workgroup, which visits every query tile, stores it for k_attn_bwd_dq
      float orow[DH];
      if (tid < TQ) {
        const int ii = qt * TQ + tid;
        Ls[tid] = ii < n ? a.LSE[(int64_t)bh * ns + ii] : 0.f;
#pragma unroll
        for (int c = 0; c < DH; ++c) orow[c] = ii < n ? a.O[ob + (int64_t)ii * osi + c] : 0.f;
      }
      __syncthreads();
      if (tid < TQ) {
        const int ii = qt * TQ + tid;
        float dsum = 0.f;
#pragma unroll
        for (int c = 0; c < DH; ++c) dsum += dOs[tid][c] * orow[c];
        Dls[tid] = dsum;
        if (j0 == 0 && ii < n) a.Dout[(int64_t)bh * ns + ii] = dsum;
      }
      __syncthreads();
      float dsr[4][4];
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        f32x4v st = f32x4v{0.f, 0.f, 0.f, 0.f}, dpt = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          st = mfma16(ka[s], Qs[16 * sub + lr][4 * s + lg], st);
          dpt = mfma16(va[s], dOs[16 * sub + lr][4 * s + lg], dpt);
        }
        const int il = 16 * sub + lr, i = qt * TQ + il;
        // keep words of row i at key columns j0 + 16 w + 4 lg + 0..3: the four lanes of a quad hold
        // rows 4 (i >> 2) + 0..3; lane c computes the block of column 4 lg + c (its four words are
        // the quad's four rows) and a quad transpose hands every lane its row's word of each column
        // (byte mode: lane c computes the block of column class 4 lg + c, takes word w — this wave's
        // 16-column group — and the quad transpose deals byte (row & 3) of each column's word)
        uint32_t kq[4] = {0u, 0u, 0u, 0u};
        if (a.thresh8) {
          const u32x4_t kb = philox4x32_10((uint32_t)(i >> 2), (uint32_t)((j0 >> 6) * 16 + 4 * lg + (lr & 3)), off,
                                           a.c3, a.seed);
          const uint32_t wd = qword(kb, w);
#pragma unroll
          for (int c = 0; c < 4; ++c) kq[c] = (wd >> (8 * c)) & 0xFFu;
          quad_transpose(kq, lane);
        } else if (a.thresh) {
          const u32x4_t kb = philox4x32_10((uint32_t)(i >> 2), (uint32_t)(j0 + 16 * w + 4 * lg + (lr & 3)), off,
                                           a.c3, a.seed);
          kq[0] = kb.x;
          kq[1] = kb.y;
          kq[2] = kb.z;
          kq[3] = kb.w;
          quad_transpose(kq, lane);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = j0 + 16 * w + 4 * lg + r;
          const bool ok = (j <= i) && (j < len) && (i < n);
          const float p = ok ? expf(st[r] * a.scale - Ls[il]) : 0.f;
          float z = 1.f;
          if (a.thresh8 && ok) z = (kq[r] >= a.thresh8) ? a.inv_keep : 0.f;
          else if (a.thresh && ok) z = (kq[r] >= a.thresh) ? a.inv_keep : 0.f;
          Ps[w][4 * lg + r][il] = p * z;
          dsr[sub][r] = p * (dpt[r] * z - Dls[il]);
        }
      }
      wave_sync();
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int s = 0; s < TQ / 4; ++s) dv[d] = mfma16(Ps[w][lr][4 * s + lg], dOs[4 * s + lg][16 * d + lr], dv[d]);
      wave_sync();
#pragma unroll
      for (int sub = 0; sub < 4; ++sub)
#pragma unroll
        for (int r = 0; r < 4; ++r) Ps[w][4 * lg + r][16 * sub + lr] = dsr[sub][r];
      wave_sync();
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int s = 0; s < TQ / 4; ++s) dk[d] = mfma16(Ps[w][lr][4 * s + lg], Qs[4 * s + lg][16 * d + lr], dk[d]);
      if constexpr (DQ) {
        __syncthreads();   // every wave's dS image of the pair is in LDS
        // dQ rows 16 w .. 16 w + 15 of this query tile: dS[query][key] = image [key / 16][key % 16][query]
        f32x4v dq[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          dq[d] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < TK / 4; ++s) {
            const int j = 4 * s + lg;
            dq[d] = mfma16(Ps[j >> 4][j & 15][16 * w + lr], Ks[j][16 * d + lr], dq[d]);
          }
        }
        const bool sole = min(qt, kmax) == 0;   // (then this is key tile 0)
        const int64_t pb = ((int64_t)blockIdx.x * gridDim.y + bh) * ns;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = qt * TQ + 16 * w + 4 * lg + r;
          if (i < n) {
#pragma unroll
            for (int d = 0; d < ND; ++d) {
              if (sole) a.dQ[gb + (int64_t)i * gsi + 16 * d + lr] = dq[d][r] * a.scale;
              else a.dQp[(pb + i) * DH + 16 * d + lr] = dq[d][r];
            }
          }
        }
      } else {
        wave_sync();
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = j0 + 16 * w + 4 * lg + r;
    if (j < n) {
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        a.dK[gb + (int64_t)j * gsi + 16 * d + lr] = dk[d][r] * a.scale;
        a.dV[gb + (int64_t)j * gsi + 16 * d + lr] = dv[d][r];
      }
    }
  }
}

// dQ of the rows with more than one contributing key tile: the partials of key tiles
// 0 .. min(qt, (len - 1) / 64) summed in ascending order (k_attn_bwd_dkdv<DH, true>); thread per
// (row, 4 channels)
template <int DH>
__global__ __launch_bounds__(256) void k_attn_dq_reduce(const AttnArgs a, int BH) {
  constexpr int C4 = DH / 4;
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int ns = a.n;
  if (x >= (int64_t)BH * ns * C4) return;
  const int c4 = (int)(x % C4);
  const int64_t row = x / C4;
  const int bh = (int)(row / ns), i = (int)(row - (int64_t)bh * ns);
  const int b = bh / a.H, h = bh - b * a.H;
  const int len = a.lens[b];
  if (a.ep_off && i >= min(len, ns)) return;   // packed rows: past the episode's own length
  const int m = min(i / TQ, len > 0 ? (len - 1) / TK : 0);
  if (m == 0) return;   // written by key tile 0
  float4 acc = *reinterpret_cast<const float4*>(a.dQp + ((int64_t)bh * ns + i) * DH + 4 * c4);
  for (int kt = 1; kt <= m; ++kt) {
    const float4 p = *reinterpret_cast<const float4*>(a.dQp + (((int64_t)kt * BH + bh) * ns + i) * DH + 4 * c4);
    acc.x += p.x;
    acc.y += p.y;
    acc.z += p.z;
    acc.w += p.w;
  }
  float* dst = a.dQ + ebase(a, a.grad, b) + h * a.grad.sh + (int64_t)i * a.grad.si + 4 * c4;
  dst[0] = acc.x * a.scale;
  dst[1] = acc.y * a.scale;
  dst[2] = acc.z * a.scale;
  dst[3] = acc.w * a.scale;
}

// ---------------------------------------------------------------------------------------------
template <int DH>
__global__ __launch_bounds__(256) void k_attn_bwd_dq(const AttnArgs a) {
  constexpr int KS = DH / 4, ND = DH / 16, KST = DH + 2;
  __shared__ float Ks[TK][KST], Vs[TK][KST];
  __shared__ float Ds[4][16][PST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int bh = blockIdx.y, b = bh / a.H, ns = a.n;
  const int q0 = blockIdx.x * TQ;
  const int len = a.lens[b];
  const int n = a.ep_off ? min(len, ns) : ns;   // packed rows: the episode's own length
  const int h = bh - b * a.H;
  if (q0 >= n) return;   // (packed rows: a query tile past the episode; workgroup-uniform)
  const int64_t ib = ebase(a, a.in, b) + h * a.in.sh, ob = ebase(a, a.out, b) + h * a.out.sh, gb = ebase(a, a.grad, b) + h * a.grad.sh;
  const int isi = a.in.si, osi = a.out.si, gsi = a.grad.si;
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t off = a.offset + (uint32_t)bh;

  float qa[KS], da[KS];
  {
    const int i = q0 + 16 * w + lr;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qa[s] = (i < n) ? a.Q[ib + (int64_t)i * isi + 4 * s + lg] : 0.f;
      da[s] = (i < n) ? a.dO[ob + (int64_t)i * osi + 4 * s + lg] : 0.f;
    }
  }
  float lse[4], dl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q0 + 16 * w + 4 * lg + r;
    lse[r] = i < n ? a.LSE[(int64_t)bh * ns + i] : 0.f;
    dl[r] = i < n ? a.Dl[(int64_t)bh * ns + i] : 0.f;
  }
  f32x4v dq[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dq[d] = f32x4v{0.f, 0.f, 0.f, 0.f};
  const int last_key = min(min(a.causal ? q0 + TQ - 1 : n - 1, n - 1), len - 1);
  for (int kt = 0; kt * TK <= last_key; ++kt) {
    __syncthreads();
    for (int x = tid; x < TK * DH; x += 256) {
      const int j = x / DH, c = x - j * DH, jj = kt * TK + j;
      Ks[j][c] = jj < n ? a.K[ib + (int64_t)jj * isi + c] : 0.f;
      Vs[j][c] = jj < n ? a.V[ib + (int64_t)jj * isi + c] : 0.f;
    }
    __syncthreads();
    // byte mode: one block per lane and key tile holds all 16 keep bytes of its scores
    const u32x4_t kb8 = a.thresh8 ? philox4x32_10((uint32_t)((q0 + 16 * w + 4 * lg) >> 2), (uint32_t)(kt * 16 + lr),
                                                  off, a.c3, a.seed)
                                  : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      f32x4v s_ = f32x4v{0.f, 0.f, 0.f, 0.f}, dp = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s_ = mfma16(qa[s], Ks[16 * sub + lr][4 * s + lg], s_);
        dp = mfma16(da[s], Vs[16 * sub + lr][4 * s + lg], dp);
      }
      const int jl = 16 * sub + lr, j = kt * TK + jl;
      // this lane's rows q0 + 16 w + 4 lg + 0..3 share one Philox block (word = row & 3)
      const u32x4_t kw = (a.thresh && !a.thresh8) ? philox4x32_10((uint32_t)((q0 + 16 * w + 4 * lg) >> 2), (uint32_t)j,
                                                                  off, a.c3, a.seed)
                                                  : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = q0 + 16 * w + 4 * lg + r;
        const bool ok = (j <= i) && (j < len) && (i < n);
        const float p = ok ? expf(s_[r] * a.scale - lse[r]) : 0.f;
        float z = 1.f;
        if (a.thresh8 && ok) z = (qbyte(kb8, sub, r) >= a.thresh8) ? a.inv_keep : 0.f;
        else if (a.thresh && ok) z = (qword(kw, r) >= a.thresh) ? a.inv_keep : 0.f;
        Ds[w][4 * lg + r][jl] = p * (dp[r] * z - dl[r]);
      }
    }
    wave_sync();
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int s = 0; s < TK / 4; ++s) dq[d] = mfma16(Ds[w][lr][4 * s + lg], Ks[4 * s + lg][16 * d + lr], dq[d]);
    wave_sync();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q0 + 16 * w + 4 * lg + r;
    if (i < n) {
#pragma unroll
      for (int d = 0; d < ND; ++d) a.dQ[gb + (int64_t)i * gsi + 16 * d + lr] = dq[d][r] * a.scale;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused backward for short episodes (n <= FB_MAXN, dh = 16): one workgroup per (episode, head)
// walks its key tiles; per (key tile, query tile) pair it forms P, P~ and dS ONCE and takes dV, dK
// (as k_attn_bwd_dkdv) and dQ from them — the dQ kernel's second pass over the same pairs (scores,
// softmax, keep bits and dP recomputed) is gone.  dQ: after the four waves' dS images of the pair are
// in LDS, wave w multiplies rows 16 w .. 16 w + 15 of dS (queries) by the key tile (staged in LDS)
// into its register accumulator of that query tile; the pairs are visited in (key tile, query tile)
// order, the same for every workgroup (deterministic).  Keep bits, masks and D = rowsum(dO * O) as
// k_attn_bwd_dkdv (bit-identical dK / dV; dQ sums key tiles in ascending order like k_attn_bwd_dq).
constexpr int FB_MAXN = 128, FB_QT = FB_MAXN / TQ;
template <int DH>
__global__ __launch_bounds__(256) void k_attn_bwd_fused(const AttnArgs a) {
  constexpr int KS = DH / 4, ND = DH / 16, KST = DH + 2;
  __shared__ float Qs[TQ][KST], dOs[TQ][KST], Ks[TK][KST];
  __shared__ float Ls[TQ], Dls[TQ];
  __shared__ float Ps[4][16][PST];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int bh = blockIdx.x, b = bh / a.H, ns = a.n;
  const int len = a.lens[b];
  const int n = a.ep_off ? min(len, ns) : ns;   // packed rows: the episode's own length
  const int h = bh - b * a.H;
  const int64_t ib = ebase(a, a.in, b) + h * a.in.sh, ob = ebase(a, a.out, b) + h * a.out.sh, gb = ebase(a, a.grad, b) + h * a.grad.sh;
  const int isi = a.in.si, osi = a.out.si, gsi = a.grad.si;
  const int lr = lane & 15, lg = lane >> 4;
  const uint32_t off = a.offset + (uint32_t)bh;
  const int nq = (n + TQ - 1) / TQ;

  f32x4v dq[FB_QT][ND];
#pragma unroll
  for (int q = 0; q < FB_QT; ++q)
#pragma unroll
    for (int d = 0; d < ND; ++d) dq[q][d] = f32x4v{0.f, 0.f, 0.f, 0.f};

  for (int kt = 0; kt < nq; ++kt) {
    const int j0 = kt * TK;
    float ka[KS], va[KS];
    {
      const int j = j0 + 16 * w + lr;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        ka[s] = (j < n) ? a.K[ib + (int64_t)j * isi + 4 * s + lg] : 0.f;
        va[s] = (j < n) ? a.V[ib + (int64_t)j * isi + 4 * s + lg] : 0.f;
      }
    }
    f32x4v dk[ND], dv[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      dk[d] = f32x4v{0.f, 0.f, 0.f, 0.f};
      dv[d] = f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    if (j0 < len) {
#pragma unroll
      for (int qt = 0; qt < FB_QT; ++qt) {
        if (qt < kt || qt >= nq) continue;   // (workgroup-uniform) causal: query tiles from the key tile on
        __syncthreads();
        for (int x = tid; x < TQ * DH; x += 256) {
          const int i = x / DH, c = x - i * DH, ii = qt * TQ + i, jj = j0 + i;
          Qs[i][c] = ii < n ? a.Q[ib + (int64_t)ii * isi + c] : 0.f;
          dOs[i][c] = ii < n ? a.dO[ob + (int64_t)ii * osi + c] : 0.f;
          Ks[i][c] = jj < n ? a.K[ib + (int64_t)jj * isi + c] : 0.f;
        }
        float orow[DH];
        if (tid < TQ) {
          const int ii = qt * TQ + tid;
          Ls[tid] = ii < n ? a.LSE[(int64_t)bh * ns + ii] : 0.f;
#pragma unroll
          for (int c = 0; c < DH; ++c) orow[c] = ii < n ? a.O[ob + (int64_t)ii * osi + c] : 0.f;
        }
        __syncthreads();
        if (tid < TQ) {
          float dsum = 0.f;
#pragma unroll
          for (int c = 0; c < DH; ++c) dsum += dOs[tid][c] * orow[c];
          Dls[tid] = dsum;
          const int ii = qt * TQ + tid;
          if (kt == 0 && ii < n) a.Dout[(int64_t)bh * ns + ii] = dsum;   // as k_attn_bwd_dkdv's key tile 0
        }
        __syncthreads();
        float dsr[4][4];
#pragma unroll
        for (int sub = 0; sub < 4; ++sub) {
          f32x4v st = f32x4v{0.f, 0.f, 0.f, 0.f}, dpt = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            st = mfma16(ka[s], Qs[16 * sub + lr][4 * s + lg], st);
            dpt = mfma16(va[s], dOs[16 * sub + lr][4 * s + lg], dpt);
          }
          const int il = 16 * sub + lr, i = qt * TQ + il;
          uint32_t kq[4] = {0u, 0u, 0u, 0u};
          if (a.thresh8) {
            const u32x4_t kb = philox4x32_10((uint32_t)(i >> 2), (uint32_t)((j0 >> 6) * 16 + 4 * lg + (lr & 3)), off,
                                             a.c3, a.seed);
            const uint32_t wd = qword(kb, w);
#pragma unroll
            for (int c = 0; c < 4; ++c) kq[c] = (wd >> (8 * c)) & 0xFFu;
            quad_transpose(kq, lane);
          } else if (a.thresh) {
            const u32x4_t kb = philox4x32_10((uint32_t)(i >> 2), (uint32_t)(j0 + 16 * w + 4 * lg + (lr & 3)), off,
                                             a.c3, a.seed);
            kq[0] = kb.x;
            kq[1] = kb.y;
            kq[2] = kb.z;
            kq[3] = kb.w;
            quad_transpose(kq, lane);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = j0 + 16 * w + 4 * lg + r;
            const bool ok = (j <= i) && (j < len) && (i < n);
            const float p = ok ? expf(st[r] * a.scale - Ls[il]) : 0.f;
            float z = 1.f;
            if (a.thresh8 && ok) z = (kq[r] >= a.thresh8) ? a.inv_keep : 0.f;
            else if (a.thresh && ok) z = (kq[r] >= a.thresh) ? a.inv_keep : 0.f;
            Ps[w][4 * lg + r][il] = p * z;
            dsr[sub][r] = p * (dpt[r] * z - Dls[il]);
          }
        }
        wave_sync();
#pragma unroll
        for (int d = 0; d < ND; ++d)
#pragma unroll
          for (int s = 0; s < TQ / 4; ++s) dv[d] = mfma16(Ps[w][lr][4 * s + lg], dOs[4 * s + lg][16 * d + lr], dv[d]);
        wave_sync();
#pragma unroll
        for (int sub = 0; sub < 4; ++sub)
#pragma unroll
          for (int r = 0; r < 4; ++r) Ps[w][4 * lg + r][16 * sub + lr] = dsr[sub][r];
        wave_sync();
#pragma unroll
        for (int d = 0; d < ND; ++d)
#pragma unroll
          for (int s = 0; s < TQ / 4; ++s) dk[d] = mfma16(Ps[w][lr][4 * s + lg], Qs[4 * s + lg][16 * d + lr], dk[d]);
        __syncthreads();   // every wave's dS image of the pair is in LDS
        // dQ rows 16 w .. 16 w + 15 of this query tile: dS[query][key] = image [key / 16][key % 16][query]
#pragma unroll
        for (int d = 0; d < ND; ++d)
#pragma unroll
          for (int s = 0; s < TK / 4; ++s) {
            const int j = 4 * s + lg;
            dq[qt][d] = mfma16(Ps[j >> 4][j & 15][16 * w + lr], Ks[j][16 * d + lr], dq[qt][d]);
          }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = j0 + 16 * w + 4 * lg + r;
      if (j < n) {
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          a.dK[gb + (int64_t)j * gsi + 16 * d + lr] = dk[d][r] * a.scale;
          a.dV[gb + (int64_t)j * gsi + 16 * d + lr] = dv[d][r];
        }
      }
    }
  }
#pragma unroll
  for (int qt = 0; qt < FB_QT; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = qt * TQ + 16 * w + 4 * lg + r;
      if (qt < nq && i < n) {
#pragma unroll
        for (int d = 0; d < ND; ++d) a.dQ[gb + (int64_t)i * gsi + 16 * d + lr] = dq[qt][d][r] * a.scale;
      }
    }
}

bool attn_fused_bwd_on() {   // XTRL_ATTN_FUSED_BWD=0: the kernel pair (read per launch: tests flip it)
  const char* e = getenv("XTRL_ATTN_FUSED_BWD");
  return !(e && atoi(e) == 0);
}

int fill_args(AttnArgs& a, const AttnProblem& p) {
  XTRL_REQUIRE(p.dh == 16 || p.dh == 32 || p.dh == 64, "attn: dim_head %d unsupported (16/32/64)", p.dh);
  XTRL_REQUIRE(p.lens && p.H > 0 && p.n > 0 && p.b > 0, "attn: bad arguments");
  XTRL_REQUIRE(p.dropout >= 0.f && p.dropout < 1.f, "attn: dropout %f outside [0, 1)", p.dropout);
  a.lens = p.lens;
  a.H = p.H;
  a.n = p.n;
  a.in = p.in;
  a.out = p.out;
  a.grad = p.grad;
  a.gate = p.gate;
  a.scale = p.scale;
  a.inv_keep = p.dropout > 0.f ? 1.f / (1.f - p.dropout) : 1.f;
  a.thresh = dropout_thresh(p.dropout);
  a.thresh8 = dropout_thresh8(p.dropout);
  a.seed = p.seed;
  a.offset = p.offset;
  XTRL_REQUIRE(p.sub < (1u << 23), "attn: dropout stream sub-index %u does not fit 23 bits", p.sub);
  a.c3 = rng_c3(FIELD_DROPOUT, a.thresh8 ? (p.sub | (1u << 23)) : p.sub);
  a.causal = p.causal;
  a.ep_off = p.ep_off;
  return XTRL_OK;
}

}  // namespace

int attn_fwd_ex(const AttnProblem& p, const float* q, const float* k, const float* v, float* o, float* lse,
                const float* gate, float* og, hipStream_t s) {
  AttnArgs a{};
  if (int rc = fill_args(a, p)) return rc;
  XTRL_REQUIRE(q && k && v && o && lse, "attn_fwd: null operand");
  XTRL_REQUIRE(!gate == !og, "attn_fwd: gate and og go together");
  a.Q = q;
  a.K = k;
  a.V = v;
  a.Oout = o;
  a.LSEout = lse;
  a.G = gate;
  a.OGout = og;
  dim3 grid((p.n + TQ - 1) / TQ, p.b * p.H);
  if (p.dh == 16) hipLaunchKernelGGL(k_attn_fwd<16>, grid, dim3(256), 0, s, a);
  else if (p.dh == 32) hipLaunchKernelGGL(k_attn_fwd<32>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_attn_fwd<64>, grid, dim3(256), 0, s, a);
  XTRL_LAUNCHED("attn_fwd");
  return XTRL_OK;
}

int attn_bwd_ex(const AttnProblem& p, const float* q, const float* k, const float* v, const float* o,
                const float* lse, const float* dout, float* dq, float* dk, float* dv, float* delta_ws,
                hipStream_t s) {
  AttnArgs a{};
  if (int rc = fill_args(a, p)) return rc;
  XTRL_REQUIRE(q && k && v && o && lse && dout && dq && dk && dv && delta_ws, "attn_bwd: null operand");
  XTRL_REQUIRE(p.causal, "attn_bwd: bidirectional attention is forward-only");
  a.Q = q;
  a.K = k;
  a.V = v;
  a.O = o;
  a.LSE = lse;
  a.dO = dout;
  a.Dl = delta_ws;
  a.Dout = delta_ws;
  a.dQ = dq;
  a.dK = dk;
  a.dV = dv;
  // (D = rowsum(dO * O) is formed inside k_attn_bwd_dkdv, whose key-tile-0 workgroups store it for dq)
  dim3 grid((p.n + TQ - 1) / TQ, p.b * p.H);
  const int64_t part_need = attn_dq_part_floats(p.b, p.H, p.n, p.dh);
  if (p.dh == 16 && p.n <= FB_MAXN && attn_fused_bwd_on()) {   // short episodes: one fused launch
    hipLaunchKernelGGL(k_attn_bwd_fused<16>, dim3(p.b * p.H), dim3(256), 0, s, a);
  } else if (p.dh == 16 && p.dq_part && p.dq_part_floats >= part_need && attn_fused_bwd_on()) {
    // long episodes: dK / dV with the dQ pass folded in (partials for multi-key-tile rows) + their sum
    a.dQp = p.dq_part;
    hipLaunchKernelGGL((k_attn_bwd_dkdv<16, true>), grid, dim3(256), 0, s, a);
    const int64_t units = (int64_t)p.b * p.H * p.n * 4;
    hipLaunchKernelGGL(k_attn_dq_reduce<16>, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, s, a, p.b * p.H);
  } else if (p.dh == 16) {
    hipLaunchKernelGGL(k_attn_bwd_dkdv<16>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_attn_bwd_dq<16>, grid, dim3(256), 0, s, a);
  } else if (p.dh == 32) {
    hipLaunchKernelGGL(k_attn_bwd_dkdv<32>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_attn_bwd_dq<32>, grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_attn_bwd_dkdv<64>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_attn_bwd_dq<64>, grid, dim3(256), 0, s, a);
  }
  XTRL_LAUNCHED("attn_bwd");
  return XTRL_OK;
}

int64_t attn_dq_part_floats(int b, int H, int n, int dh) {
  return (int64_t)((n + TK - 1) / TK) * b * H * n * dh;
}

AttnProblem contiguous_problem(const int32_t* lens, int b, int H, int n, int dh, float scale, float p, uint64_t seed,
                               uint32_t offset, uint32_t sub) {
  AttnProblem pr{b, H, n, dh, lens, scale, p, seed, offset, {}, {}, {}, {}};
  pr.sub = sub;
  pr.in = pr.out = pr.grad = attn_layout_bhnd(H, n, dh);
  return pr;
}

}  // namespace xtrl

extern "C" int xtrl_attn_fwd(const float* q, const float* k, const float* v, const int32_t* lens, float* o,
                             float* lse, int b, int H, int n, int dh, float scale, float dropout_p, uint64_t seed,
                             uint32_t offset, uint32_t sub, void* stream) {
  return xtrl::attn_fwd_ex(xtrl::contiguous_problem(lens, b, H, n, dh, scale, dropout_p, seed, offset, sub), q, k, v, o,
                           lse, nullptr, nullptr, xtrl::as_stream(stream));
}

extern "C" int64_t xtrl_attn_bwd_part_floats(int b, int H, int n, int dh) {
  return xtrl::attn_dq_part_floats(b, H, n, dh);
}

extern "C" int xtrl_attn_bwd_part(const float* q, const float* k, const float* v, const int32_t* lens, const float* o,
                                  const float* lse, const float* dout, float* dq, float* dk, float* dv, float* delta_ws,
                                  float* dq_part, int64_t dq_part_floats, int b, int H, int n, int dh, float scale,
                                  float dropout_p, uint64_t seed, uint32_t offset, uint32_t sub, void* stream) {
  xtrl::AttnProblem pr = xtrl::contiguous_problem(lens, b, H, n, dh, scale, dropout_p, seed, offset, sub);
  pr.dq_part = dq_part;
  pr.dq_part_floats = dq_part_floats;
  return xtrl::attn_bwd_ex(pr, q, k, v, o, lse, dout, dq, dk, dv, delta_ws, xtrl::as_stream(stream));
}

extern "C" int xtrl_attn_bwd(const float* q, const float* k, const float* v, const int32_t* lens, const float* o,
                             const float* lse, const float* dout, float* dq, float* dk, float* dv, float* delta_ws,
                             int b, int H, int n, int dh, float scale, float dropout_p, uint64_t seed,
                             uint32_t offset, uint32_t sub, void* stream) {
  return xtrl::attn_bwd_ex(xtrl::contiguous_problem(lens, b, H, n, dh, scale, dropout_p, seed, offset, sub), q, k, v, o,
                           lse, dout, dq, dk, dv, delta_ws, xtrl::as_stream(stream));
}

/* bidirectional / causal attention forward on token-major operands (rows b * n + i, head h at
 * columns h * dh): q, k, v with row strides ldq / ldk / ldv, out o [b * n][ldo]. */
extern "C" int xtrl_attn_fwd_tokens(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                                    const int32_t* lens, float* o, int ldo, float* lse, int b, int H, int n, int dh,
                                    float scale, int causal, void* stream) {
  XTRL_REQUIRE(ldq == ldk && ldk == ldv, "attn_fwd_tokens: q, k, v share one row stride (got %d %d %d)", ldq, ldk,
               ldv);
  xtrl::AttnProblem pr{b, H, n, dh, lens, scale, 0.f, 0, 0, {}, {}, {}, {}};
  pr.in = xtrl::attn_layout_tokens(n, ldq, dh);
  pr.out = xtrl::attn_layout_tokens(n, ldo, dh);
  pr.causal = causal;
  // q, k, v are addressed from their own bases with the same layout
  return xtrl::attn_fwd_ex(pr, q, k, v, o, lse, nullptr, nullptr, (hipStream_t)stream);
}
