// Diagnostic build of the warp-specialised X6 GEMM (not part of the library): per-step
// s_memtime stamps of one consumer and one producer wave per workgroup (-DXTRL_WS_DIAG), or, without
// stamps, one mode fixed at compile time (-DXTRL_WS_MODE=m: 1 consumers skip the MFMAs, 2 producers
// skip loads + splits, 3 producers load but do not split; production code otherwise).
//   hipcc -O3 -std=c++17 -fno-slp-vectorize --offload-arch=gfx950 -DXTRL_WS_DIAG \
//         -Ix-transformers-rl_amd/csrc tools/ws_lab.hip -o /tmp/ws_lab && /tmp/ws_lab M N K [ta tb]
#include "../x-transformers-rl_amd/csrc/gemm.hip"
#include <cstdarg>
#include <cstdio>
#include <vector>
#include <algorithm>

namespace xtrl {
void set_error(const char* fmt, ...) {
  va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap); fputc('\n', stderr);
}
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : 1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  int M = argc > 1 ? atoi(argv[1]) : 16384, N = argc > 2 ? atoi(argv[2]) : 256, K = argc > 3 ? atoi(argv[3]) : 1024;
  int ta = argc > 4 ? atoi(argv[4]) : 0, tb = argc > 5 ? atoi(argv[5]) : 0, mode = argc > 6 ? atoi(argv[6]) : 0;
  const int kspan = argc > 7 ? atoi(argv[7]) : 0;   // > 0: cross-workgroup split of K (as gemm_wgrad)
  const int splits = kspan > 0 ? (K + kspan - 1) / kspan : 1;
  float *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * K * 4)); CK(hipMalloc(&B, (size_t)N * K * 4)); CK(hipMalloc(&C, (size_t)splits * M * N * 4));
  std::vector<float> h((size_t)std::max(M, N) * K);
  for (auto& v : h) v = (float)rand() / RAND_MAX - 0.5f;
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)N * K * 4, hipMemcpyHostToDevice));
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128) * splits;
#ifdef XTRL_WS_DIAG
  uint64_t* diag;
  CK(hipMalloc(&diag, (size_t)tiles * 2 * 4096 * 8));
  CK(hipMemset(diag, 0, (size_t)tiles * 2 * 4096 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(xtrl::g_ws_diag), &diag, sizeof(diag)));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(xtrl::g_ws_mode), &mode, sizeof(mode)));
#endif
  xtrl::GemmArgs a;
  a.A = A; a.B = B; a.C = C; a.M = M; a.N = N; a.K = K; a.ldc = N;
  a.lda = ta ? M : K; a.ldb = tb ? N : K;
  if (kspan > 0) { a.kspan = kspan; a.c_split = (int64_t)M * N; }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&]() {
    if (!ta && !tb) xtrl::launch_ws<false, false, xtrl::EPI_NONE, false>(a, 0);
    else if (!ta && tb) xtrl::launch_ws<false, true, xtrl::EPI_NONE, false>(a, 0);
    else xtrl::launch_ws<true, true, xtrl::EPI_NONE, false>(a, 0);
  };
  for (int i = 0; i < 3; ++i) run();
  CK(hipEventRecord(e0)); for (int i = 0; i < 10; ++i) run(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
#ifndef XTRL_WS_DIAG
#ifdef XTRL_WS_MODE
  mode = XTRL_WS_MODE;
#endif
#endif
  printf("mode %d M=%d N=%d K=%d ta=%d tb=%d splits=%d: %.1f us/launch, %.1f TF (diag build)\n", mode, M, N, K, ta, tb, splits, ms * 100, 2.0 * M * N * K / (ms / 10 * 1e-3) / 1e12);
  if (mode == 0) {   // sampled outputs vs an fp64 dot product (split-K partials summed here)
    std::vector<float> hc((size_t)splits * M * N);
    CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
    double worst = 0;
    for (int s = 0; s < 512; ++s) {
      const int m = (int)(((uint64_t)s * 2654435761u) % M), n = (int)(((uint64_t)s * 40503u + 7) % N);
      double ref = 0, mag = 0, got = 0;
      for (int k = 0; k < K; ++k) {
        const double x = h[ta ? (size_t)k * M + m : (size_t)m * K + k], y = h[tb ? (size_t)k * N + n : (size_t)n * K + k];
        ref += x * y; mag += fabs(x * y);
      }
      for (int z = 0; z < splits; ++z) got += hc[(size_t)z * M * N + (size_t)m * N + n];
      worst = std::max(worst, fabs(got - ref) / mag);
    }
    printf("  max |C - C64| / sum|a b| over 512 samples: %.3g (2^-24 = 5.96e-8)\n", worst);
  }
#ifndef XTRL_WS_DIAG
  (void)tiles;
  return 0;
#else
  std::vector<uint64_t> d((size_t)tiles * 2 * 4096);
  CK(hipMemcpy(d.data(), diag, d.size() * 8, hipMemcpyDeviceToHost));
  const int nk = (kspan > 0 ? kspan : K) / 32, nsteps = 3 * ((nk + 2) / 3);
  // per step averages (over workgroups) in s_memtime ticks
  double cc = 0, cw = 0, pc = 0, pl = 0, pw = 0; int n = 0;
  std::vector<double> per_c(nk, 0), per_p(nk, 0);
  uint64_t tmin = ~0ull, tmax = 0;
  for (int w = 0; w < tiles; ++w) {
    const uint64_t* c = &d[(size_t)(w * 2 + 0) * 4096];
    const uint64_t* p = &d[(size_t)(w * 2 + 1) * 4096];
    for (int s = 1; s + 1 < nk; ++s) {
      cc += c[s * 4 + 1] - c[s * 4 + 0];
      cw += c[(s + 1) * 4 + 0] - c[s * 4 + 1];
      pl += p[s * 4 + 1] - p[s * 4 + 0];
      pc += p[s * 4 + 2] - p[s * 4 + 1];
      pw += p[(s + 1) * 4 + 0] - p[s * 4 + 2];
      ++n;
    }
    tmin = std::min(tmin, c[0]); tmax = std::max(tmax, c[nsteps * 4]);
  }
  printf("per step (ticks): consumer compute %.0f, consumer barrier wait %.0f | producer load issue %.0f, convert %.0f, barrier wait %.0f\n",
         cc / n, cw / n, pl / n, pc / n, pw / n);
  const uint64_t* c0 = &d[0];
  printf("wg0 loop span %llu ticks for %d steps; all-wg loop span %llu\n", (unsigned long long)(c0[(nk + (nk & 1)) * 4] - c0[0]), nk,
         (unsigned long long)(tmax - tmin));
  return 0;
#endif
}
