// Cost of a cross-stream fork point on the forking stream (not part of the library): a chain of
// N small kernels on stream A, and after each one the side stream B is made to wait for it.
//   0: no fork (baseline)
//   1: hipEventRecord(e, A) + hipStreamWaitEvent(B, e)               (train.hip Fork::fork today)
//   2: the chain kernel launched with hipExtLaunchKernelGGL(stopEvent = e) + hipStreamWaitEvent(B, e)
//   3: an empty marker kernel with stopEvent = e after each chain kernel + hipStreamWaitEvent(B, e)
//   4: hipStreamWriteValue32(A, flag, i + 1) + hipStreamWaitValue32(B, flag >= i + 1)
//   5: every chain-kernel workgroup adds 1 to a counter after a release fence (no packet on A);
//      hipStreamWaitValue32(B, counter >= blocks (i + 1))
//   6: the NEXT chain kernel launched with startEvent = e (it starts once everything before it on A
//      is done), then hipStreamWaitEvent(B, e)
// B runs a tiny kernel after each wait (as the weight-gradient stream would).  Prints us per link.
//   hipcc -O3 --offload-arch=gfx950 tools/event_gap_lab.hip -o /tmp/event_gap_lab && /tmp/event_gap_lab
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_work(const float* x, float* y, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = x[i] * 1.0001f + 1.f;
}
__global__ void k_marker() {}
__global__ void k_work_cnt(const float* x, float* y, int n, unsigned* cnt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) y[i] = x[i] * 1.0001f + 1.f;
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_side(float* z) {
  if (threadIdx.x == 0) z[blockIdx.x] += 1.f;
}

int main() {
  const int n = 1 << 22, N = 64, reps = 20;
  float *x, *y, *z;
  CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&z, 4096));
  CK(hipMemset(x, 0, n * 4)); CK(hipMemset(z, 0, 4096));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(N);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  unsigned* flag;
  CK(hipExtMallocWithFlags((void**)&flag, 8, hipMallocSignalMemory));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
  for (int mode = 0; mode < 7; ++mode) {
    if (mode == 5) continue;   // (measured ~1 ms a link: the wait polls slowly)
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipMemset(flag, 0, 8));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, A));
      for (int i = 0; i < N; ++i) {
        if (mode == 2) {
          hipExtLaunchKernelGGL(k_work, dim3(1024), dim3(256), 0, A, nullptr, ev[i], 0, (const float*)x, y, n);
        } else if (mode == 6) {
          hipExtLaunchKernelGGL(k_work, dim3(1024), dim3(256), 0, A, ev[i], nullptr, 0, (const float*)x, y, n);
        } else if (mode == 5) {
          hipLaunchKernelGGL(k_work_cnt, dim3(1024), dim3(256), 0, A, (const float*)x, y, n, flag);
        } else {
          hipLaunchKernelGGL(k_work, dim3(1024), dim3(256), 0, A, (const float*)x, y, n);
        }
        if (mode == 1) CK(hipEventRecord(ev[i], A));
        if (mode == 3) hipExtLaunchKernelGGL(k_marker, dim3(1), dim3(64), 0, A, nullptr, ev[i], 0);
        if (mode == 4) {
          CK(hipStreamWriteValue32(A, flag, (uint32_t)(i + 1), 0));
          CK(hipStreamWaitValue32(B, flag, (uint32_t)(i + 1), hipStreamWaitValueGte, 0xffffffffu));
          hipLaunchKernelGGL(k_side, dim3(1), dim3(64), 0, B, z);
        } else if (mode == 5) {
          CK(hipStreamWaitValue32(B, flag, (uint32_t)(1024 * (i + 1)), hipStreamWaitValueGte, 0xffffffffu));
          hipLaunchKernelGGL(k_side, dim3(1), dim3(64), 0, B, z);
        } else if (mode != 0) {
          CK(hipStreamWaitEvent(B, ev[i], 0));
          hipLaunchKernelGGL(k_side, dim3(1), dim3(64), 0, B, z);
        }
      }
      CK(hipEventRecord(t1, A));
      CK(hipEventSynchronize(t1));
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      best = ms < best ? ms : best;
    }
    printf("mode %d: %.2f us per chain link (best of %d, %d links)\n", mode, best * 1e3f / N, reps, N);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
