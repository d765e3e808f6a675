// HL-Gauss value decode + generalised advantage estimation over the padded trajectory batch.
//
// Restates Agent.learn's preparation (x_transformers_rl.py:839-852):
//   scalar_values = HLGaussLoss(values)                      softmax(logits) . centres
//   returns       = calc_gae(rewards, scalar_values, ~is_boundaries, gamma, lam)   (:616-640)
// One workgroup per episode row.  Phase 1: each wave decodes values for timesteps t = w, w+4, ...
// (lanes over the bins; the logits row is read once, coalesced).  Phase 2: one lane runs the
// reverse scan gae_t = gate_t * gae_{t+1} + delta_t in sequential order — the same order as the
// oracle, so the returns are bitwise stable — with FMA contraction disabled so each step rounds
// like the reference's separate multiply and add.
// Truncation bootstrap (optional): boot[e] (not NaN) is the value of the state after a truncated
// episode's last step; it replaces V at index lens[e] (the padding value the scan would read).
#include "common.h"

namespace xtrl {
namespace {

__global__ __launch_bounds__(256) void k_hlgauss_gae(const float* logits, int64_t ld_row, const float* rewards,
                                                     const uint8_t* bounds, int64_t ld_seq, const float* centers,
                                                     float* values, float* returns, int n, int B, float gamma,
                                                     float gamma_lam, const float* boot, const int32_t* lens) {
  extern __shared__ float vs[];   // [n + 1]
  const int e = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int t = w; t < n; t += 4) {
    const float* x = logits + (int64_t)e * ld_row + (int64_t)t * B;
    float mx = -INFINITY;
    for (int k = lane; k < B; k += 64) mx = fmaxf(mx, x[k]);
    mx = wave_max(mx);
    float s = 0.f, sc = 0.f;
    for (int k = lane; k < B; k += 64) {
      const float ex = expf(x[k] - mx);
      s += ex;
      sc += ex * centers[k];
    }
    s = wave_sum(s);
    sc = wave_sum(sc);
    if (lane == 0) vs[t] = sc / s;
  }
  if (threadIdx.x == 0) vs[n] = 0.f;
  __syncthreads();
  if (boot && threadIdx.x == 0) {
    const float bv = boot[e];
    const int le = lens[e];
    if (!isnan(bv) && le >= 0 && le <= n) vs[le] = bv;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < n; t += 256) values[(int64_t)e * n + t] = vs[t];
  if (threadIdx.x != 0) return;
  {
#pragma clang fp contract(off)
    float acc = 0.f;
    for (int t = n - 1; t >= 0; --t) {
      const float m = bounds[(int64_t)e * ld_seq + t] ? 0.f : 1.f;
      const float r = rewards[(int64_t)e * ld_seq + t];
      const float delta = (r + (gamma * vs[t + 1]) * m) - vs[t];
      const float gate = gamma_lam * m;
      acc = gate * acc + delta;
      returns[(int64_t)e * n + t] = acc + vs[t];
    }
  }
}

}  // namespace

int hlgauss_gae(const float* logits, int64_t ld_row, const float* rewards, const uint8_t* bounds, int64_t ld_seq,
                const float* centers, float* values, float* returns, int E, int n, int B, float gamma,
                float gamma_lam, const float* boot, const int32_t* lens, hipStream_t s) {
  XTRL_REQUIRE(logits && rewards && bounds && centers && values && returns, "hlgauss_gae: null operand");
  XTRL_REQUIRE(!boot || lens, "hlgauss_gae: bootstrap values need the episode lengths");
  XTRL_REQUIRE(E > 0 && n > 0 && B > 0, "hlgauss_gae: bad shape E=%d n=%d B=%d", E, n, B);
  XTRL_REQUIRE((size_t)(n + 1) * 4 <= 160 * 1024, "hlgauss_gae: n=%d too long", n);
  hipLaunchKernelGGL(k_hlgauss_gae, dim3(E), dim3(256), (n + 1) * sizeof(float), s, logits, ld_row, rewards, bounds,
                     ld_seq, centers, values, returns, n, B, gamma, gamma_lam, boot, lens);
  XTRL_LAUNCHED("hlgauss_gae");
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_hlgauss_gae(const float* logits, int64_t ld_row, const float* rewards, const uint8_t* bounds,
                                int64_t ld_seq, const float* centers, float* values, float* returns, int E, int n,
                                int B, float gamma, float gamma_lam, const float* boot, const int32_t* lens,
                                void* stream) {
  return xtrl::hlgauss_gae(logits, ld_row, rewards, bounds, ld_seq, centers, values, returns, E, n, B, gamma,
                           gamma_lam, boot, lens, xtrl::as_stream(stream));
}
