// Consumer-split weight-gradient GEMM (k_gemm_cs, defined here) against the warp-specialised one (k_gemm_ws<T,T>) on
// the learn step's weight-gradient shapes: timing, and bit-equality of the split-K partial tiles and
// of the bias row sums.  Not part of the library.
//   hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -Ix-transformers-rl_amd/csrc \
//         tools/cs_lab.hip -o /tmp/cs_lab && /tmp/cs_lab
#include "../x-transformers-rl_amd/csrc/gemm.hip"
#include <cstdarg>
#include <cstdio>
#include <vector>
#include <algorithm>

// ---- the kernel under test (measured slower than k_gemm_ws and kept out of the library; DESIGN §7
// round-6 negatives).  Same translation unit as gemm.hip, so its anonymous-namespace helpers are visible.
namespace xtrl {
namespace {
// ---- X6 weight-gradient GEMM with the split in the consumers (both operands "T") ------------------
// dW = dY^T X: A[m][k] = dY[k][m], B[k][n] = X[k][n], k = token.  The warp-specialised kernel's
// producers write every slab as three bf16 piece images, and those LDS stores — the VGPR -> LDS
// transfer, 6 bytes per element — not the split arithmetic are its overhead (tools/ws_lab.hip:
// loads + piece stores without the split 70.8 us, loads alone 59.5, the full kernel 68.7, MFMAs
// alone 53.5 on the C3 FF1 weight gradient).  Here the raw fp32 slabs go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, 4 bytes per element, k-major [k][128] images exactly as the
// token rows lie in memory: one 1 KiB wave-instruction = 2 token rows of a 128-column tile) into a
// ring of three slabs, two in flight across each barrier (counted vmcnt, raw s_barrier); the four
// waves (one per SIMD, 64 x 64 each) read their fragments as fp32 (8 k-strided dwords per lane,
// conflict-free: 32 consecutive columns per half-wave), split them into hi / mid / lo in registers
// and issue the same six piece products in the same order as k_gemm_ws — bit-identical outputs.
// K (tokens) and the split span are multiples of 32 (host: cs_ok).
typedef __attribute__((address_space(3))) void lds_void_t;
template <int BM = 128, bool PIPE = true>   // PIPE: both k16 steps' fragments read before the first step's split
__global__ __launch_bounds__(BM * 2, 1) void k_gemm_cs(const GemmArgs a) {
  // BM = 128: 4 waves (one per SIMD); BM = 256: 8 waves, two per SIMD (one wave's split arithmetic
  // issues beside the other's MFMAs); each wave 64 x 64, BN = 128
  constexpr int BN = 128, BK = 32, NS = 3, TM = 2, TN = 2, NW = BM / 32;
  constexpr int SLAB = (BM + BN) * BK;                             // floats: A image [k][BM], then B [k][BN]
  constexpr int PA_ = BK * BM / 256, PB_ = BK * BN / 256;          // 1 KiB DMA pieces per operand and slab
  static_assert((PA_ + PB_) % NW == 0, "DMA pieces split evenly over the waves");
  constexpr int PW = (PA_ + PB_) / NW;                             // pieces per wave and slab
  __shared__ __attribute__((aligned(16))) float smem[NS * SLAB];   // 96 / 144 KiB
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (a.xcd_remap) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int total = nx * ny * gridDim.z;
    const int lin = bx + nx * (by + ny * bz);
    const int lg = (lin & 7) * (total >> 3) + (lin >> 3);
    bx = lg % nx;
    by = (lg / nx) % ny;
    bz = lg / (nx * ny);
  }
  const int m0 = by * BM, n0 = bx * BN;
  const int M = a.M, N = a.N;
  int K = a.K;
  const float* __restrict__ Ab = a.A;
  const float* __restrict__ Bb = a.B;
  if (a.kspan > 0) {
    const int kb = bz * a.kspan;
    K = min(a.kspan, a.K - kb);
    Ab += (int64_t)kb * a.lda;
    Bb += (int64_t)kb * a.ldb;
  }
  const int nk = K / BK;
  // DMA: piece q (A pieces 0 .. PA_ - 1, then B's) holds image floats 256 q .. 256 q + 255, lane l the
  // 4 at 256 q + 4 l -> token row e / width, column e % width (clamped into the operand: columns past
  // M / N feed only discarded outputs); wave w issues pieces w, w + NW, ...
  const float* gp[PW];
  int lo[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int q = w + NW * i;
    if (q < PA_) {
      const int e = 256 * q + 4 * lane;
      gp[i] = Ab + (int64_t)(e / BM) * a.lda + min(m0 + e % BM, ((M + 3) & ~3) - 4);
      lo[i] = 256 * q;
    } else {
      const int e = 256 * (q - PA_) + 4 * lane;
      gp[i] = Bb + (int64_t)(e / BN) * a.ldb + min(n0 + e % BN, ((N + 3) & ~3) - 4);
      lo[i] = BM * BK + 256 * (q - PA_);
    }
  }
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int q = w + NW * i;
      const int64_t ko = (int64_t)kt * BK * (q < PA_ ? a.lda : a.ldb);
      __builtin_amdgcn_global_load_lds((const void*)(gp[i] + ko), (lds_void_t*)(smem + slot * SLAB + lo[i]), 16, 0, 0);
    }
  };
  const int wm = w >> 1, wn = w & 1;
  const bool do_rs = a.rowsum != nullptr && bx == 0 && wn == 0;   // bias gradient: row sums of A
  float rsum[TM] = {0.f, 0.f};
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  auto rdv = [&](const float* img, int width, int row, int k0, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = img[(k0 + j) * width + row];
  };
  auto splitv = [&](const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l, float& rs) {
    uint32_t hh[4], mm[4], ll[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) split3_pair(v[2 * q], v[2 * q + 1], hh[q], mm[q], ll[q]);
    h = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
    m = __builtin_bit_cast(bf16x8, make_uint4(mm[0], mm[1], mm[2], mm[3]));
    l = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
    rs += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));   // (kept only where do_rs)
  };
  float rs_unused = 0.f;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int t = 0; t < nk; ++t) {
    // slab t landed (this wave's 8 DMAs of it; slab t + 1's stay in flight), every wave's DMAs of it
    // retired and every wave done reading slab t - 1 (whose ring slot the next issue overwrites)
    if (t + 1 < nk) {
      if constexpr (PW == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) issue(t + 2, (t + 2) % NS);
    const float* sa = smem + (t % NS) * SLAB;
    const float* sb = sa + BM * BK;
    float va[2][TM][8], vb[2][TN][8];
    static_assert(PW == 8 || PW == 6, "vmcnt immediates above");
    auto rd_step = [&](int st) {
#pragma unroll
      for (int i = 0; i < TM; ++i) rdv(sa, BM, wm * 64 + 32 * i + fr, 16 * st + fk, va[st][i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) rdv(sb, BN, wn * 64 + 32 * j + fr, 16 * st + fk, vb[st][j]);
    };
    if constexpr (PIPE) {
      rd_step(0);
      rd_step(1);
    }
#pragma unroll
    for (int st = 0; st < BK / 16; ++st) {
      if constexpr (!PIPE) rd_step(st);
      bf16x8 av[3][TM], bv[3][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) splitv(va[st][i], av[0][i], av[1][i], av[2][i], rsum[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) splitv(vb[st][j], bv[0][j], bv[1][j], bv[2][j], rs_unused);
      // smallest products first: (A piece, B piece) = lo.hi, hi.lo, mid.mid, mid.hi, hi.mid, hi.hi
      constexpr int PA[6] = {2, 0, 1, 1, 0, 0}, PB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[PA[q]][i], bv[PB[q]][j], acc[i][j], 0, 0, 0);
    }
  }
  if (do_rs) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float r = rsum[i] + __shfl_xor(rsum[i], 32, kWave);
      const int m = m0 + wm * 64 + 32 * i + lane;
      if (lane < 32 && m < M && m >= a.rowsum_m0) {
        if (a.kspan > 0) a.rowsum_ws[(int64_t)bz * M + m] = r;
        else a.rowsum[m - a.rowsum_m0] += r;
      }
    }
  }
  gemm_epilogue<TM, TN, EPI_NONE, false>(a, acc, m0, n0, wm, wn, lane, bz);
}

void launch_cs(const GemmArgs& a, hipStream_t s) {
  const int splits = a.kspan > 0 ? (a.K + a.kspan - 1) / a.kspan : 1;
  dim3 grid((a.N + 127) / 128, (a.M + 127) / 128, splits);
  GemmArgs r = a;
  r.xcd_remap = (xcd_env() && (int64_t)grid.x * grid.y * grid.z % 8 == 0) ? 1 : 0;
  hipLaunchKernelGGL((k_gemm_cs<128, true>), grid, dim3(256), 0, s, r);
}

}  // namespace
}  // namespace xtrl

namespace xtrl {
void set_error(const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap); fputc('\n', stderr);
}
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : 1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
  // dW[Nout][Kin] = dY[T][Nout]^T X[T][Kin]; gemm view M = Nout, N = Kin, K = T
  const int shapes[][3] = {{1024, 256, 16384}, {256, 1024, 16384}, {260, 256, 16384}, {1024, 512, 16384},
                           {512, 128, 13760}, {128, 512, 13760}};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    const int ldy = (M + 3) & ~3, ldx = N;
    // the library's split rule (gemm_wgrad): 192 workgroups, spans of whole 32-token slabs
    const int64_t tiles = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
    int splits = (int)std::max<int64_t>(1, std::min<int64_t>((192 + tiles - 1) / tiles, (K + 255) / 256));
    int kspan = ((K + splits - 1) / splits + 31) / 32 * 32;
    splits = (K + kspan - 1) / kspan;
    float *A, *B, *C1, *C2, *rs1, *rs2;
    CK(hipMalloc(&A, (size_t)K * ldy * 4)); CK(hipMalloc(&B, (size_t)K * ldx * 4));
    CK(hipMalloc(&C1, (size_t)splits * M * N * 4)); CK(hipMalloc(&C2, (size_t)splits * M * N * 4));
    CK(hipMalloc(&rs1, (size_t)splits * M * 4)); CK(hipMalloc(&rs2, (size_t)splits * M * 4));
    std::vector<float> h((size_t)K * std::max(ldy, ldx));
    for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
    CK(hipMemcpy(A, h.data(), (size_t)K * ldy * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), (size_t)K * ldx * 4, hipMemcpyHostToDevice));
    xtrl::GemmArgs a;
    a.A = A; a.B = B; a.lda = ldy; a.ldb = ldx; a.M = M; a.N = N; a.K = K; a.ldc = N;
    a.kspan = kspan; a.c_split = (int64_t)M * N; a.beta = 0.f;
    float dummy_bias = 0.f;
    a.rowsum = &dummy_bias; a.rowsum_m0 = 0;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run_ws = [&]() { a.C = C1; a.rowsum_ws = rs1; xtrl::launch_ws<true, true, xtrl::EPI_NONE, false>(a, 0); };
    auto run_cs = [&]() { a.C = C2; a.rowsum_ws = rs2; xtrl::launch_cs(a, 0); };
    // 256 x 128 tiles, 8 waves (two per SIMD): half the tiles, twice the splits -> the same workgroup count
    const int64_t tiles2 = (int64_t)((M + 255) / 256) * ((N + 127) / 128);
    int splits2 = (int)std::max<int64_t>(1, std::min<int64_t>((192 + tiles2 - 1) / tiles2, (K + 255) / 256));
    int kspan2 = ((K + splits2 - 1) / splits2 + 31) / 32 * 32;
    splits2 = (K + kspan2 - 1) / kspan2;
    float* C3; CK(hipMalloc(&C3, (size_t)splits2 * M * N * 4));
    float* rs3; CK(hipMalloc(&rs3, (size_t)splits2 * M * 4));
    auto run_cs0 = [&]() {
      xtrl::GemmArgs b = a;
      b.C = C3; b.rowsum_ws = rs3; b.kspan = kspan2;
      dim3 grid((b.N + 127) / 128, (b.M + 255) / 256, splits2);
      hipLaunchKernelGGL((xtrl::k_gemm_cs<256, true>), grid, dim3(512), 0, 0, b);
    };
    auto timeit = [&](auto fn) {
      for (int i = 0; i < 3; ++i) fn();
      CK(hipEventRecord(e0)); for (int i = 0; i < 20; ++i) fn(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms * 1e3f / 20;
    };
    const float t0 = timeit(run_cs0);
    float tw = timeit(run_ws), tc = timeit(run_cs), tw2 = timeit(run_ws), tc2 = timeit(run_cs);
    CK(hipDeviceSynchronize());
    std::vector<float> c1((size_t)splits * M * N), c2(c1.size()), r1((size_t)splits * M), r2(r1.size());
    CK(hipMemcpy(c1.data(), C1, c1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c2.data(), C2, c2.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r1.data(), rs1, r1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), rs2, r2.size() * 4, hipMemcpyDeviceToHost));
    size_t diff = 0; double maxd = 0, maxr = 0;
    for (size_t i = 0; i < c1.size(); ++i) if (c1[i] != c2[i]) { ++diff; maxd = std::max(maxd, (double)fabsf(c1[i] - c2[i])); }
    for (size_t i = 0; i < r1.size(); ++i) maxr = std::max(maxr, (double)fabsf(r1[i] - r2[i]) / (fabsf(r1[i]) + 1e-3));
    const double fl = 2.0 * M * N * K;
    printf("M=%d N=%d K=%d splits=%d: ws %.1f/%.1f us (%.0f TF)  cs256 %.1f  cs %.1f/%.1f us (%.0f TF)  partials differing %zu "
           "(max %.3g)  rowsum max rel %.3g\n", M, N, K, splits, tw, tw2, fl / std::min(tw, tw2) / 1e6, t0, tc, tc2,
           fl / std::min(tc, tc2) / 1e6, diff, maxd, maxr);
    {   // the 256-row variant: its split partials summed on the host vs the 128-row kernel's
      std::vector<float> c3((size_t)splits2 * M * N);
      CK(hipMemcpy(c3.data(), C3, c3.size() * 4, hipMemcpyDeviceToHost));
      double md = 0, mag = 0;
      for (size_t e = 0; e < (size_t)M * N; e += 7) {
        double x = 0, y = 0;
        for (int z = 0; z < splits; ++z) x += c2[z * (size_t)M * N + e];
        for (int z = 0; z < splits2; ++z) y += c3[z * (size_t)M * N + e];
        md = std::max(md, fabs(x - y)); mag = std::max(mag, fabs(x));
      }
      printf("    cs256 splits %d: summed-partial max |diff| %.3g of max |C| %.3g\n", splits2, md, mag);
    }
    CK(hipFree(C3)); CK(hipFree(rs3));
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C1)); CK(hipFree(C2)); CK(hipFree(rs1)); CK(hipFree(rs2));
  }
  return 0;
}
