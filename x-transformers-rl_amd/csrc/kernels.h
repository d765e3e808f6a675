// Internal (C++) interfaces shared between the translation units of libxtrl_hip.
// Not part of the C-ABI: include/xtrl_hip.h is.
#pragma once
#include "common.h"

namespace xtrl {

// ---------------------------------------------------------------------------------------------
// fp32 MFMA GEMM (gemm.hip)
//   C[m, n] = epi( LN?(A)[m, :] . B[:, n] + bias ) (+ R[m, n]);   C = beta * C + result
// Operand layouts:  A "N": A[m][k] at A[m * lda + k]    A "T": A[m][k] at A[k * lda + m]
//                   B "N": B[k][n] at B[n * ldb + k]    B "T": B[k][n] at B[k * ldb + n]
// ---------------------------------------------------------------------------------------------
enum GemmEpi : int {
  EPI_NONE = 0,        // (bias)
  EPI_GELU = 1,        // gelu(v)
  EPI_SILU = 2,        // silu(v)
  // forward epilogues that also save the local derivative for the backward (so the backward
  // epilogue is one multiply: no erf / exp / dropout RNG recomputation)
  EPI_GELU_DROP = 3,   // C = drop(gelu(v)); aux_out = drop(gelu'(v))   (drop: keep ? x / (1 - p) : 0)
  EPI_SILU_SAVE = 4,   // n < act_cols: C = silu(v), aux_out = silu'(v);  else C = v, aux_out = 1
  EPI_MUL_AUX = 5,     // C = v * aux_in                                 (dgrad through a saved derivative)
  EPI_RELU = 8,        // max(v, 0)   (fractal encoder final aggregation, fractal_rl.py:235-239)
  EPI_DGATE = 7,       // s = sigmoid(aux_in2): C = v * s; aux_out = v * aux_in * (1 - s) * s   (value gate)
  // full-row LayerNorm epilogues (warp-specialised kernel, one column tile holds every column of a row:
  // N <= 256; x-transformers LayerNorm = layer_norm without affine, eps 1e-5, times gamma)
  EPI_RES_LN = 9,      // C = v (+ bias) + R;  ln_y1 / ln_y2 = LN(C) * ln_g;  ln_stats[m] = (mean, rstd)
  EPI_LN_BWD = 10,     // g = v; xhat = (ln_x - mean) rstd; C = rstd (g ln_g - mean_n(g ln_g) - xhat
                       //   mean_n(g ln_g xhat)) + ln_dres;  ln_part[row tile][n] = sum_tile rows g xhat
  EPI_MASK_POS = 11,   // C = aux_in > 0 ? v : 0        (dgrad through a ReLU whose output is aux_in)
  EPI_LN_BWD2 = 12,    // post-norm (nn.LayerNorm) backward: g = v + ln_gpre; C = LN_bwd(g) (+ d gamma / d beta
                       //   partials); with ln2_out also C2 = LN_bwd(C; ln2_x, ln2_stats, ln2_g) (+ partials):
                       //   two chained post-norm LayerNorms whose residual path has no other branch
};

struct GemmArgs {
  const float* A = nullptr;
  const float* B = nullptr;
  const float* bias = nullptr;    // bias[n - bias_col0] for n >= bias_col0
  const float* gamma = nullptr;   // LayerNorm prologue (A "N" only)
  const float* R = nullptr;       // residual
  float* C = nullptr;
  const int32_t* t_dev = nullptr; // C += (*t_dev) * c_t_stride (decode writes into trajectory rows)
  int64_t c_t_stride = 0;
  int lda = 0, ldb = 0, ldr = 0, ldc = 0, M = 0, N = 0, K = 0;
  float beta = 0.f;
  int kspan = 0;                  // > 0: split K over blockIdx.z (partial tiles at C + z * c_split)
  int64_t c_split = 0;
  int bias_col0 = 0;
  int act_cols = 1 << 30;
  const float* aux_in = nullptr;  int ld_aux_in = 0;
  const float* aux_in2 = nullptr; int ld_aux_in2 = 0;
  float* aux_out = nullptr;       int ld_aux_out = 0;
  uint64_t seed = 0;              // dropout (EPI_GELU_DROP): keep(m, n) =
  uint32_t drop_off = 0;          //   philox(seed; n, m >> 2, drop_off, FIELD_FF_DROPOUT sub 2 layer) word (m & 3)
  uint32_t drop_layer = 0;        //   (c3 sub-index = 2 * drop_layer + byte mode)
  uint32_t drop_thresh = 0;       //   >= drop_thresh (0: no dropout)
  uint32_t drop_thresh8 = 0;      // != 0: byte-mode keep bits (p = drop_thresh8 / 256 exactly), see ff_block8
  float inv_keep = 1.f;
  const uint8_t* row_mask = nullptr;   // rows m with row_mask[m] == 0 are not stored (dead envs)
  float* rowsum = nullptr;        // += row sums of A (rows >= rowsum_m0, at rowsum[m - rowsum_m0]) —
  int rowsum_m0 = 0;              //   the bias gradient when A = dY^T; with split-K the per-split
  float* rowsum_ws = nullptr;     //   sums go to rowsum_ws[z][M] and the reduce kernel adds them
  int xcd_remap = 0;              // 1: workgroup ids permuted so each XCD runs consecutive tiles
  // LayerNorm epilogues (EPI_RES_LN / EPI_LN_BWD)
  const float* ln_g = nullptr;    // gamma [N]
  int ln_rms = 0;                 // LN prologue / RES_LN / LN_BWD: x-transformers RMSNorm (use_rmsnorm), mean 0
  const float* ln_b = nullptr;    // RES_LN: beta [N] (nn.LayerNorm bias; x-transformers LayerNorm has none)
  const float* ln_b2 = nullptr;   // RES_LN: ln_y2 = LN(C) * ln_g (+ ln_b) + ln_b2 (the next level's input)
  float* ln_y1 = nullptr; int ln_ld1 = 0;   // RES_LN: normalised rows (ln_y2 optional: a second copy)
  float* ln_y2 = nullptr; int ln_ld2 = 0;
  float* ln_stats = nullptr;      // [M][2] (mean, rstd): written by RES_LN, read by LN_BWD
  const float* ln_x = nullptr;    // LN_BWD: the LayerNorm input [M][N] (row stride N)
  const float* ln_dres = nullptr; // LN_BWD: gradient added to the output (may alias C: same element, same thread)
  float* ln_part = nullptr;       // LN_BWD: d gamma partials [ceil(M / BM)][N]
  // EPI_LN_BWD2 (partial rows of stride ln_pstride: the four partial sets of one row tile side by side)
  const float* ln_gpre = nullptr; // gradient added to the GEMM output before the LayerNorm backward [M][N]
  int ln_ldg = 0;                 //   its row stride (0: N)
  float ln_gscale = 1.f;          // the GEMM output scaled by this before the add (frac_gradient)
  float* ln_part_b = nullptr;     // d beta partials
  int ln_pstride = 0;
  const float* ln2_g = nullptr;   // the chained LayerNorm: gamma, input, (mean, rstd), output, partials
  const float* ln2_x = nullptr;
  const float* ln2_stats = nullptr;
  float* ln2_out = nullptr;
  float* ln2_part = nullptr;
  float* ln2_part_b = nullptr;
};
// rows per workgroup of the LayerNorm-epilogue GEMM for an N-column row (the column tile is the row)
int gemm_ln_rows(int N);

// launch C = op(A, B) for the combination (trans_a, trans_b, epi, LN = gamma != 0, RES = R != 0)
int gemm_run(const GemmArgs& a, int trans_a, int trans_b, int epi, hipStream_t s);
// dW[N][K] (+)= dY^T X over M tokens, split-K over workgroups with a fixed-order reduction;
// db (optional, accumulated) [n - db_n0] += sum_m dY[m][n] for n >= db_n0 (the bias gradient)
// prof (optional): events recorded around the main GEMM launch when it is the 128x128 kernel
struct GemmProfile {
  void** events;
  double* flops;
  int cap;
  int* n;
};
// Deferred split-K reductions: the weight gradients of one backward write their partial tiles to
// disjoint workspace ranges and queue their reduction; splitk_flush sums every queued job in ONE
// launch (fixed order per element: deterministic) instead of a reduce launch per weight.
struct SplitKJob {
  const float* ws;       // partials [S][M][N]
  float* C;              // C[m][n] (ldc) = beta C + sum_z partial
  const float* rws;      // optional row-sum partials [S][M] -> rowsum[m - m0] += sum_z
  float* rowsum;
  int S, M, N, ldc, m0;
  float beta;
  int64_t q0, r0;        // first float4 unit / first row-sum unit of this job in the launch
};
constexpr int kMaxSplitKJobs = 24;
struct SplitKQueue {
  SplitKJob job[kMaxSplitKJobs];
  int n = 0;
  int64_t used = 0;      // workspace floats taken by the queued jobs
};
int splitk_flush(SplitKQueue& q, hipStream_t s);

int gemm_wgrad(const float* dY, int ldy, const float* X, int ldx, float* dW, int ldw, int M, int N, int K, float beta,
               float* ws, int64_t ws_floats, hipStream_t s, float* db = nullptr, int db_n0 = 0,
               const GemmProfile* prof = nullptr, SplitKQueue* defer = nullptr);
int gemm_f32(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* ln_gamma,
             const float* R, int ldr, float* Y, int ldy, const int32_t* t_dev, int64_t y_t_stride, int M, int N,
             int K, int act, hipStream_t s);
int layernorm_f32(const float* X, int ldx, const float* gamma, float* Y, int ldy, int M, int D, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// decode-step GEMM over compacted live rows (dgemm.hip)
//   C[dst(m), n] = act( LN?(A)[m, :] . W[n, :] + bias[n] ) (+ R[m, n]),  m < (m_dev ? *m_dev : M)
//   W is an nn.Linear weight [N][K]; LN (x-transformers LayerNorm times gamma) covers A's columns
//   [0, ln_k); dst(m) = row_map ? row_map[m] : m
// ---------------------------------------------------------------------------------------------
struct DGemmArgs {
  const float* A = nullptr; int lda = 0;
  const float* W = nullptr; int ldw = 0;
  const float* bias = nullptr;
  const float* gamma = nullptr; int ln_k = 0;
  int ln_rms = 0;   // the prologue norm is x-transformers' RMSNorm (use_rmsnorm), not its LayerNorm
  const float* R = nullptr; int ldr = 0;
  float* C = nullptr; int ldc = 0;
  const int32_t* row_map = nullptr;
  const int32_t* m_dev = nullptr;
  int M = 0, N = 0, K = 0;
  // columns n >= n_split go to C2[dst2(m) * ldc2 + n - n_split], dst2(m) = row_map2 ? row_map2[m] : m
  // (the heads' last Linear: actor logits to a row buffer, critic logits into the trajectory)
  int n_split = 1 << 30;
  float* C2 = nullptr; int ldc2 = 0;
  const int32_t* row_map2 = nullptr;
};
// `rows` bounds the live-row count (sizes the grid); epi: EPI_NONE / EPI_GELU / EPI_SILU;
// W fragment-packed by dgemm_pack (dgemm_packed_floats(N, K) floats)
int dgemm_run(const DGemmArgs& a, int rows, int epi, hipStream_t s);
// waves splitting K per column group (dgemm_body KS) of a 16-row-panel projection of this shape
int dg_ks(int N, int K);
int64_t dgemm_packed_floats(int N, int K);
int dgemm_pack(const float* W, int ldw, int N, int K, float* Wp, hipStream_t s);

// fractal body row kernels (fractal.hip): y = x + v (x NULL: v); y = LN(x + r) g + b (nn.LayerNorm)
void rows_add_launch(const float* x, int ldx, const float* v, float* y, int ldy, int M, int D, hipStream_t s);
void add_layernorm_launch(const float* x, int ldx, const float* r, int ldr, const float* g, const float* b, float* y,
                          int ldy, int M, int D, float eps, hipStream_t s);

// dropout threshold of probability p on a uint32 word: keep iff word >= thresh
// p * 256 when that is an integer in [1, 255] (byte-mode FF dropout keep bits), else 0
inline uint32_t dropout_thresh8(float p) {
  const double t = (double)p * 256.0;
  return (t >= 1.0 && t <= 255.0 && t == (double)(int)t) ? (uint32_t)t : 0u;
}

inline uint32_t dropout_thresh(float p) {
  if (!(p > 0.f)) return 0u;
  const double th = (double)p * 4294967296.0;
  const uint32_t t = (uint32_t)fmin(th, 4294967295.0);
  return t ? t : 1u;
}

// ---------------------------------------------------------------------------------------------
// training attention on strided operands (attn.hip)
//   element (b, h, i, c) of a tensor with layout L is at P + b * L.sb + h * L.sh + i * L.si + c
// ---------------------------------------------------------------------------------------------
struct AttnLayout {
  int64_t sb, sh;
  int si;
};
inline AttnLayout attn_layout_bhnd(int H, int n, int dh) {
  return AttnLayout{(int64_t)H * n * dh, (int64_t)n * dh, dh};
}
inline AttnLayout attn_layout_tokens(int n, int ld, int dh) {   // [b*n][ld], head h at column h*dh
  return AttnLayout{(int64_t)n * ld, (int64_t)dh, ld};
}

struct AttnProblem {
  int b, H, n, dh;
  const int32_t* lens;
  float scale, dropout;
  uint64_t seed;
  uint32_t offset;
  AttnLayout in, out, grad;   // q/k/v; o/do (and og); dq/dk/dv
  AttnLayout gate;            // gate pre-activations (x-transformers attn_gate_values)
  int causal = 1;             // 0: bidirectional (key-padding mask only; forward only)
  uint32_t sub = 0;           // dropout stream sub-index (c3 low 24 bits): the decoder layer
  // n > 128 (past the one-launch fused backward) at dh = 16: workspace for the per-key-tile dQ
  // partials of the dK / dV kernel with the dQ pass folded in (attn_dq_part_floats); NULL: the pair
  float* dq_part = nullptr;
  int64_t dq_part_floats = 0;
  // packed rows (the learn step without padding, XtrlTrainDesc.packed): episode b's min(lens[b], n)
  // tokens are rows ep_off[b] .. of the token-major layouts (their sb unused); NULL: rows b * n + i
  const int32_t* ep_off = nullptr;
};
int64_t attn_dq_part_floats(int b, int H, int n, int dh);

// o (ungated) and lse; if gate != nullptr also og = o * sigmoid(gate) (og in the `out` layout)
int attn_fwd_ex(const AttnProblem& p, const float* q, const float* k, const float* v, float* o, float* lse,
                const float* gate, float* og, hipStream_t s);
int attn_bwd_ex(const AttnProblem& p, const float* q, const float* k, const float* v, const float* o,
                const float* lse, const float* dout, float* dq, float* dk, float* dv, float* delta_ws,
                hipStream_t s);

}  // namespace xtrl
