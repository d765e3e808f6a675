// Weight-gradient GEMM kernel choice for short split spans (gemm.hip ws_ok: the warp-specialised
// kernel only when each split spans >= 512 tokens): k_gemm_ws<T,T> vs the register-staged X6 kernel
// at several split counts, on the small-weight shapes of the fractal learn step (C5: 256 x 256 over
// 16384 tokens).  Not part of the library.
//   hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -Ix-transformers-rl_amd/csrc \
//         tools/wgrad_span_lab.hip -o /tmp/wsl && /tmp/wsl
#include "../x-transformers-rl_amd/csrc/gemm.hip"
#include <cstdarg>
#include <cstdio>
#include <vector>

namespace xtrl {
void set_error(const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap); fputc('\n', stderr);
}
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : 1; }
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
  const int shapes[][3] = {{256, 256, 16384}, {512, 256, 16384}, {256, 512, 16384}, {192, 256, 16384}};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    float *A, *B, *C;
    CK(hipMalloc(&A, (size_t)K * M * 4)); CK(hipMalloc(&B, (size_t)K * N * 4));
    CK(hipMalloc(&C, (size_t)128 * M * N * 4));
    std::vector<float> h((size_t)K * std::max(M, N));
    for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
    CK(hipMemcpy(A, h.data(), (size_t)K * M * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), (size_t)K * N * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    for (int splits : {192 / tiles, 96 / tiles, 48 / tiles, 24 / tiles}) {
      if (splits < 1) continue;
      const int kspan = ((K + splits - 1) / splits + 31) / 32 * 32;
      const int sp = (K + kspan - 1) / kspan;
      xtrl::GemmArgs a;
      a.A = A; a.B = B; a.C = C; a.lda = M; a.ldb = N; a.M = M; a.N = N; a.K = K; a.ldc = N;
      a.kspan = kspan; a.c_split = (int64_t)M * N; a.beta = 0.f;
      auto timeit = [&](auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipEventRecord(e0)); for (int i = 0; i < 20; ++i) fn(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms * 1e3f / 20;
      };
      const float tw = timeit([&] { xtrl::launch_ws<true, true, xtrl::EPI_NONE, false>(a, 0); });
      const float tr = timeit([&] { xtrl::launch<2, 2, 1, 2, 2, true, true, xtrl::EPI_NONE, false, false, true, true>(a, 0); });
      printf("M=%d N=%d K=%d splits=%d span=%d: ws %.1f us  register-staged %.1f us  (%d workgroups)\n", M, N, K, sp,
             kspan, tw, tr, tiles * sp);
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C));
  }
  return 0;
}
