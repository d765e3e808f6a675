// Decode-step GEMM: the rollout's projections over the COMPACTED live rows of one timestep.
//
//   C[dst(m), n] = act( LN?(A)[m, :] . W[n, :] + bias[n] ) (+ R[m, n])      m < *m_dev
//
// The rollout's GEMMs are small (M <= E live rows, N <= 1024, K <= 1024) and latency bound: the
// cost of one launch is one workgroup's chain of load latency + MFMA + epilogue.  This kernel is
// built for that regime (replaces the per-step GEMM / LayerNorm launches of the round-1 decode):
//  * the workgroup's whole A panel (16 or 32 rows x K) is fetched in ONE round of LDS-DMA loads
//    (global_load_lds, 1 KiB row pieces, rows padded by 16 B so the fragment reads are
//    conflict-free), so there is one load latency per launch instead of one per K slab;
//  * an optional LayerNorm prologue normalises the first ln_k columns of the staged rows in LDS
//    (x-transformers LayerNorm: no affine, eps 1e-5, times gamma), all 256 threads at once (a
//    wave per row, one row after another, cost 11 us a launch: LDS and shuffle round trips) —
//    the pre-norms of q|k|v, FF1 and the heads cost no launch of their own;
//  * each wave owns 16*NT output columns and streams its weights straight into registers (16
//    float4 per lane per block, the next block in flight while the current one feeds the MFMAs):
//    weights are not shared between waves, so they skip LDS.  They are stored fragment-packed
//    (xtrl_dgemm_pack, once per rollout): every load instruction reads 1 KiB contiguous — in the
//    nn.Linear layout the 16 columns of a fragment sit in 16 rows, 64 cache lines per instruction
//    (FF2: 16.7 us a launch, L1-bound);
//  * v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation); lane (r = l & 15, q = l >> 4)
//    of every fragment covers the k quarter [q K/4, (q+1) K/4), float4 j of it feeding four
//    MFMAs — any k order sums every product once; two accumulator chains per tile hide the
//    40-cycle dependent MFMA latency;
//  * M is read from device memory (the live-row count the embedding kernel produced), so one
//    captured hipGraph serves every step: row tiles past the live count exit at once;
//  * epilogue: bias, GELU / SiLU, residual, a row scatter and a column split (the heads' last
//    Linear: actor logits to a row buffer, critic logits straight into the trajectory rows of their
//    episodes).
#include <algorithm>
#include <cstdlib>

#include "dgemm_body.h"
#include "x6.h"

namespace xtrl {

namespace {

template <int MT, int NT, int KS, int EPI, bool LN, bool RES>
__global__ __launch_bounds__(256) void k_dgemm(const DGemmArgs a) {
  extern __shared__ float As[];
  DgNoHook hook;
  dgemm_body<MT, NT, KS, EPI, LN, RES>(a, As, hook);
}

// fragment packing of an nn.Linear weight [N][K] (one thread per float4 slot)
__global__ void k_dg_pack(const float* W, int ldw, int N, int K, float* Wp) {
  const int Kp = dg_kp(K), JN = Kp >> 4, KQ = Kp >> 2;
  const int64_t slots = (int64_t)((N + 15) >> 4) * JN * 64;
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= slots) return;
  const int lr = (int)(s & 15), q = (int)((s >> 4) & 3);
  const int64_t rest = s >> 6;
  const int j = (int)(rest % JN), t16 = (int)(rest / JN);
  const int n = t16 * 16 + lr, k0 = q * KQ + 4 * j;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (n < N && k0 + i < K) ? W[(int64_t)n * ldw + k0 + i] : 0.f;
  reinterpret_cast<float4*>(Wp)[s] = make_float4(v[0], v[1], v[2], v[3]);
}

// split-bf16 fragment packing for the 16x16x32 bf16 operand (one thread per 16-byte slot of each plane)
__global__ void k_dg_pack_x6(const float* W, int ldw, int N, int K, uint4* Wp) {
  const int JS = K >> 5;
  const int64_t slots = (int64_t)((N + 15) >> 4) * JS * 64;
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= slots) return;
  const int lane = (int)(s & 63);
  const int64_t rest = s >> 6;
  const int sk = (int)(rest % JS), t16 = (int)(rest / JS);
  const int n = 16 * t16 + (lane & 15), k0 = 32 * sk + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = n < N ? W[(int64_t)n * ldw + k0 + i] : 0.f;
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) split3_pair(v[2 * i], v[2 * i + 1], h[i], m[i], l[i]);
  Wp[s] = make_uint4(h[0], h[1], h[2], h[3]);
  Wp[slots + s] = make_uint4(m[0], m[1], m[2], m[3]);
  Wp[2 * slots + s] = make_uint4(l[0], l[1], l[2], l[3]);
}

// the same fragment order in fp32: plane h of slot s holds the lane's k0 + 4 h .. + 3
__global__ void k_dg_pack_f8(const float* W, int ldw, int N, int K, float4* Wp) {
  const int JS = K >> 5;
  const int64_t slots = (int64_t)((N + 15) >> 4) * JS * 64;
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= slots) return;
  const int lane = (int)(s & 63);
  const int64_t rest = s >> 6;
  const int sk = (int)(rest % JS), t16 = (int)(rest / JS);
  const int n = 16 * t16 + (lane & 15), k0 = 32 * sk + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = n < N ? W[(int64_t)n * ldw + k0 + i] : 0.f;
  Wp[s] = make_float4(v[0], v[1], v[2], v[3]);
  Wp[slots + s] = make_float4(v[4], v[5], v[6], v[7]);
}

template <int MT, int NT, int KS, int EPI, bool LN, bool RES>
void launch_dg(const DGemmArgs& a, int rows, hipStream_t s) {
  constexpr int BM = 16 * MT, BN = 64 * NT / KS;
  dim3 grid((a.N + BN - 1) / BN, (rows + BM - 1) / BM);
  const size_t lds = dg_lds_floats(MT, NT, KS, LN, a.K) * sizeof(float);
  hipLaunchKernelGGL((k_dgemm<MT, NT, KS, EPI, LN, RES>), grid, dim3(256), lds, s, a);
}

template <int EPI, bool LN, bool RES>
void dispatch_dg(const DGemmArgs& a, int rows, hipStream_t s) {
  // 32-row panels where N is wide and the panel stays small (FF1, the head hidden layer: twice
  // the weight reuse, half the workgroups); 16-row panels otherwise (long K, narrow N)
  // (long K over narrow N: the K split across the 4 waves, see dgemm_body)
  const size_t lds32 = (size_t)32 * (dg_kp(a.K) + 4) * sizeof(float);
  const int ks = dg_ks(a.N, a.K);
  if (a.N >= 512 && lds32 <= 80 * 1024) launch_dg<2, 1, 1, EPI, LN, RES>(a, rows, s);
  else if (ks == 2) launch_dg<1, 1, 2, EPI, LN, RES>(a, rows, s);
  else if (ks == 4) launch_dg<1, 1, 4, EPI, LN, RES>(a, rows, s);
  else launch_dg<1, 1, 1, EPI, LN, RES>(a, rows, s);
}

}  // namespace

// the K split of a 16-row-panel projection: 2 for K >= 768 over N < 512 (FF2 at 440 live rows:
// 9.7 -> 7.3 us; 4: 7.3 us at 440 rows but 14.0 vs 10.0 us at 1024, every column block re-reading
// the A panel); XTRL_DG_KS overrides (1, 2, 4; experiments)
int dg_ks(int N, int K) {
  static const int ks_env = [] {
    const char* e = getenv("XTRL_DG_KS");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  if (!dg_split_k(N, K)) return 1;
  return ks_env ? ks_env : 2;
}

int64_t dgemm_packed_floats(int N, int K) { return (int64_t)((N + 15) / 16) * 16 * dg_kp(K); }

int dgemm_pack(const float* W, int ldw, int N, int K, float* Wp, hipStream_t s) {
  XTRL_REQUIRE(W && Wp && N > 0 && K > 0 && ldw >= K, "dgemm_pack: bad arguments");
  const int64_t slots = dgemm_packed_floats(N, K) / 4;
  hipLaunchKernelGGL(k_dg_pack, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, W, ldw, N, K, Wp);
  XTRL_LAUNCHED("dgemm_pack");
  return XTRL_OK;
}

int64_t dgemm_packed_x6_elems(int N, int K) { return (int64_t)3 * ((N + 15) / 16) * 16 * K; }

int64_t dgemm_packed_f8_floats(int N, int K) { return (int64_t)((N + 15) / 16) * 16 * K; }

int dgemm_pack_f8(const float* W, int ldw, int N, int K, float* Wp, hipStream_t s) {
  XTRL_REQUIRE(W && Wp && N > 0 && K > 0 && K % 32 == 0 && ldw >= K && ((uintptr_t)Wp & 15u) == 0,
               "dgemm_pack_f8: bad arguments (K a multiple of 32, Wp 16-byte aligned)");
  const int64_t slots = dgemm_packed_f8_floats(N, K) / 8;
  hipLaunchKernelGGL(k_dg_pack_f8, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, W, ldw, N, K,
                     reinterpret_cast<float4*>(Wp));
  XTRL_LAUNCHED("dgemm_pack_f8");
  return XTRL_OK;
}

int dgemm_pack_x6(const float* W, int ldw, int N, int K, uint16_t* Wp, hipStream_t s) {
  XTRL_REQUIRE(W && Wp && N > 0 && K > 0 && K % 32 == 0 && ldw >= K && ((uintptr_t)Wp & 15u) == 0,
               "dgemm_pack_x6: bad arguments (K a multiple of 32, Wp 16-byte aligned)");
  const int64_t slots = dgemm_packed_x6_elems(N, K) / 24;
  hipLaunchKernelGGL(k_dg_pack_x6, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, W, ldw, N, K,
                     reinterpret_cast<uint4*>(Wp));
  XTRL_LAUNCHED("dgemm_pack_x6");
  return XTRL_OK;
}

int dgemm_run(const DGemmArgs& a, int rows, int epi, hipStream_t s) {
  XTRL_REQUIRE(a.A && a.W && a.C && a.K > 0 && a.N > 0 && rows >= 0, "dgemm: bad operands");
  XTRL_REQUIRE(a.K % 4 == 0 && a.lda % 4 == 0 && ((uintptr_t)a.A & 15u) == 0 && ((uintptr_t)a.W & 15u) == 0,
               "dgemm: K, lda must be multiples of 4 and A, W 16-byte aligned (K=%d lda=%d)", a.K, a.lda);
  XTRL_REQUIRE(a.K <= 2048 && a.lda >= a.K && a.ldc >= std::min(a.N, a.n_split),
               "dgemm: bad K / leading dimensions");
  XTRL_REQUIRE(!a.gamma || (a.ln_k > 0 && a.ln_k <= a.K && a.ln_k <= 512), "dgemm: bad LayerNorm width (<= 512)");
  XTRL_REQUIRE(epi == EPI_NONE || epi == EPI_GELU || epi == EPI_SILU || epi == EPI_RELU,
               "dgemm: epilogue %d unsupported", epi);
  XTRL_REQUIRE(a.n_split >= a.N || (a.C2 && a.n_split >= 0 && a.ldc2 >= a.N - a.n_split), "dgemm: bad column split");
  if (rows == 0) return XTRL_OK;
  const bool ln = a.gamma != nullptr, res = a.R != nullptr;
#define XTRL_DG(E)                                                                                \
  do {                                                                                            \
    if (ln && res) dispatch_dg<E, true, true>(a, rows, s);                                        \
    else if (ln) dispatch_dg<E, true, false>(a, rows, s);                                         \
    else if (res) dispatch_dg<E, false, true>(a, rows, s);                                        \
    else dispatch_dg<E, false, false>(a, rows, s);                                                \
  } while (0)
  if (epi == EPI_GELU) XTRL_DG(EPI_GELU);
  else if (epi == EPI_SILU) XTRL_DG(EPI_SILU);
  else if (epi == EPI_RELU) {
    XTRL_REQUIRE(!ln && !res, "dgemm: the ReLU epilogue has no LayerNorm / residual variant");
    dispatch_dg<EPI_RELU, false, false>(a, rows, s);
  }
  else XTRL_DG(EPI_NONE);
#undef XTRL_DG
  XTRL_LAUNCHED("dgemm");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int64_t xtrl_dgemm_packed_floats(int N, int K) { return xtrl::dgemm_packed_floats(N, K); }
extern "C" int xtrl_dgemm_pack(const float* W, int ldw, int N, int K, float* Wp, void* stream) {
  return xtrl::dgemm_pack(W, ldw, N, K, Wp, xtrl::as_stream(stream));
}
extern "C" int64_t xtrl_dgemm_packed_x6_elems(int N, int K) { return xtrl::dgemm_packed_x6_elems(N, K); }
extern "C" int64_t xtrl_dgemm_packed_f8_floats(int N, int K) { return xtrl::dgemm_packed_f8_floats(N, K); }
extern "C" int xtrl_dgemm_pack_f8(const float* W, int ldw, int N, int K, float* Wp, void* stream) {
  return xtrl::dgemm_pack_f8(W, ldw, N, K, Wp, xtrl::as_stream(stream));
}
extern "C" int xtrl_dgemm_pack_x6(const float* W, int ldw, int N, int K, uint16_t* Wp, void* stream) {
  return xtrl::dgemm_pack_x6(W, ldw, N, K, Wp, xtrl::as_stream(stream));
}
extern "C" int xtrl_dgemm(const float* A, int lda, const float* Wp, const float* bias, const float* ln_gamma, int ln_k,
                          const float* R, int ldr, float* C, int ldc, const int32_t* row_map, const int32_t* m_dev,
                          int M, int N, int K, int act, void* stream) {
  xtrl::DGemmArgs a;
  a.A = A; a.lda = lda; a.W = Wp; a.ldw = xtrl::dgemm_packed_floats(1, K) / 16; a.bias = bias; a.gamma = ln_gamma; a.ln_k = ln_k;
  a.R = R; a.ldr = ldr; a.C = C; a.ldc = ldc; a.row_map = row_map; a.m_dev = m_dev; a.M = M; a.N = N; a.K = K;
  return xtrl::dgemm_run(a, M, act == 3 ? xtrl::EPI_RELU : act, xtrl::as_stream(stream));
}
