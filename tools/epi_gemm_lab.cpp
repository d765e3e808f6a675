// FF1-forward epilogue price inside the GEMM: xtrl::gemm_run at M=16384 N=1024 K=256 with the plain,
// GELU, GELU + saved derivative (no dropout), and GELU + derivative + dropout (byte / word mode)
// epilogues.  Build: hipcc -O2 --offload-arch=gfx950 -I x-transformers-rl_amd/csrc tools/epi_gemm_lab.cpp
//   -L x-transformers-rl_amd/xtrl_amd -lxtrl_hip -Wl,-rpath,'$ORIGIN/../x-transformers-rl_amd/xtrl_amd'
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "kernels.h"

static float time_us(const xtrl::GemmArgs& g, int epi) {
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  if (xtrl::gemm_run(g, 0, 0, epi, nullptr)) return -1.f;
  (void)hipEventRecord(s, nullptr);
  for (int i = 0; i < 20; ++i) xtrl::gemm_run(g, 0, 0, epi, nullptr);
  (void)hipEventRecord(e, nullptr);
  (void)hipEventSynchronize(e);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, s, e);
  return ms / 20 * 1e3f;
}

int main() {
  const int M = 16384, N = 1024, K = 256;
  float *A, *B, *C, *D, *bias;
  (void)hipMalloc(&A, (size_t)M * 768 * 4);
  (void)hipMalloc(&B, (size_t)N * 768 * 4);
  (void)hipMalloc(&C, (size_t)M * (N + 64) * 4);
  (void)hipMalloc(&D, (size_t)M * (N + 64) * 4);
  (void)hipMalloc(&bias, (size_t)N * 4);
  {   // non-zero operands (zero inputs run at a higher clock and skip erf's slow branches)
    std::vector<float> h((size_t)M * 768);
    uint32_t x = 1;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = ((x >> 8) * 5.96e-8f - 0.5f) * 0.25f; }
    (void)hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(B, h.data(), (size_t)N * 768 * 4, hipMemcpyHostToDevice);
  }
  (void)hipMemset(bias, 0, (size_t)N * 4);
  xtrl::GemmArgs g;
  g.A = A; g.lda = K; g.B = B; g.ldb = K; g.bias = bias; g.C = C; g.ldc = N; g.M = M; g.N = N; g.K = K;
  printf("plain             %7.1f us\n", time_us(g, xtrl::EPI_NONE));
  printf("gelu              %7.1f us\n", time_us(g, xtrl::EPI_GELU));
  g.aux_out = D; g.ld_aux_out = N;
  printf("gelu+deriv        %7.1f us\n", time_us(g, xtrl::EPI_GELU_DROP));
  g.seed = 12345; g.drop_off = 3; g.inv_keep = 1.f / 0.75f;
  g.drop_thresh = xtrl::dropout_thresh(0.25f); g.drop_thresh8 = xtrl::dropout_thresh8(0.25f);
  printf("+dropout (byte)   %7.1f us\n", time_us(g, xtrl::EPI_GELU_DROP));
  g.drop_thresh = xtrl::dropout_thresh(0.1f); g.drop_thresh8 = 0; g.inv_keep = 1.f / 0.9f;
  printf("+dropout (word)   %7.1f us\n", time_us(g, xtrl::EPI_GELU_DROP));
  // output row strides off the 4 KiB power of two (channel / bank spread of the store streams)
  g.drop_thresh = xtrl::dropout_thresh(0.25f); g.drop_thresh8 = xtrl::dropout_thresh8(0.25f); g.inv_keep = 1.f / 0.75f;
  for (int pad : {4, 16, 32, 64}) {
    g.ldc = N + pad; g.ld_aux_out = N + pad;
    printf("byte, ld %4d      %7.1f us   (plain %7.1f us)\n", N + pad, time_us(g, xtrl::EPI_GELU_DROP),
           time_us(g, xtrl::EPI_NONE));
  }
  g.ldc = N; g.ld_aux_out = N;
  // the heads' first layer (actor | critic, SiLU + saved derivative): K = 512 (C3) / 768 (C5)
  g.drop_thresh = 0; g.drop_thresh8 = 0;
  for (int k : {512, 768}) {
    g.K = k; g.lda = k; g.ldb = k;
    for (int pad : {0, 16}) {
      g.ldc = N + pad; g.ld_aux_out = N + pad;
      printf("silu_save K %d ld %4d  %7.1f us   (plain %7.1f us)\n", k, N + pad, time_us(g, xtrl::EPI_SILU_SAVE),
             time_us(g, xtrl::EPI_NONE));
    }
  }
  // the world-model heads' input gradient: dewa[T][2d] = dzp[T][d + 1] . W_pd[d + 1][2d] (K = d + 1
  // ragged) against the aligned K = d
  {
    xtrl::GemmArgs h;
    h.A = A; h.lda = 260; h.B = B; h.ldb = 512; h.C = C; h.ldc = 512; h.M = M; h.N = 512;
    for (int k : {257, 256, 260}) {
      h.K = k;
      hipEvent_t s0, s1;
      (void)hipEventCreate(&s0);
      (void)hipEventCreate(&s1);
      xtrl::gemm_run(h, 0, 1, xtrl::EPI_NONE, nullptr);
      (void)hipEventRecord(s0, nullptr);
      for (int i = 0; i < 20; ++i) xtrl::gemm_run(h, 0, 1, xtrl::EPI_NONE, nullptr);
      (void)hipEventRecord(s1, nullptr);
      (void)hipEventSynchronize(s1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, s0, s1);
      printf("dgrad NT M %d N 512 K %d      %7.1f us\n", M, k, ms / 20 * 1e3f);
    }
  }
  return 0;
}
