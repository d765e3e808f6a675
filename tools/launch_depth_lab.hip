// How far ahead of the GPU can the host enqueue?  Launches K spin kernels of a fixed duration on
// one stream with kernel arguments of ARG bytes and reports, at steady state, how many launches the
// host is ahead (launch i's call returns when kernel i - depth has finished) and how long a launch
// call blocks.  Build: hipcc --offload-arch=gfx950 -O2 tools/launch_depth_lab.hip -o tools/launch_depth_lab.bin
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

template <int BYTES>
struct Arg {
  unsigned char pad[BYTES];
};

template <int BYTES>
__global__ void k_spin(Arg<BYTES> a, long long cycles, int* out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.pad[0];
}

template <int BYTES>
void run(int K, double us, int blocks) {
  int* out;
  (void)hipMalloc(&out, 4);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  Arg<BYTES> a{};
  // wall_clock64 runs at 100 MHz on gfx9
  const long long cyc = (long long)(us * 100.0);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_spin<BYTES>, dim3(blocks), dim3(64), 0, s, a, cyc, out);
  (void)hipStreamSynchronize(s);
  std::vector<double> ret(K), dur(K);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < K; ++i) {
    const auto c0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_spin<BYTES>, dim3(blocks), dim3(64), 0, s, a, cyc, out);
    const auto c1 = std::chrono::steady_clock::now();
    ret[i] = std::chrono::duration<double, std::micro>(c1 - t0).count();
    dur[i] = std::chrono::duration<double, std::micro>(c1 - c0).count();
  }
  (void)hipStreamSynchronize(s);
  const double total = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  const double per = total / K;   // GPU time per kernel at steady state
  // host lead when launch i returns: (kernels enqueued) - (kernels finished by then)
  double lead_sum = 0;
  int n = 0;
  for (int i = K / 2; i < K; ++i) {
    lead_sum += i + 1 - ret[i] / per;
    ++n;
  }
  std::vector<double> ds(dur.begin() + K / 2, dur.end());
  std::sort(ds.begin(), ds.end());
  printf("arg %5d B  kernel %6.1f us  blocks %4d: GPU %.1f us/kernel, host ahead by %.1f launches (%.0f us) "
         "at steady state; launch call p50 %.1f p90 %.1f max %.1f us; host done enqueueing at %.0f of %.0f us\n",
         BYTES, us, blocks, per, lead_sum / n, per * lead_sum / n, ds[ds.size() / 2], ds[ds.size() * 9 / 10],
         ds.back(), ret[K - 1], total);
  (void)hipStreamDestroy(s);
  (void)hipFree(out);
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 4000;
  for (double us : {5.0, 20.0, 80.0}) {
    run<64>(K, us, 1);
    run<512>(K, us, 1);
    run<2048>(K, us, 1);
    run<64>(K, us, 1024);
  }
  return 0;
}
