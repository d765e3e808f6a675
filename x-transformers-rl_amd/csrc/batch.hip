// Minibatch assembly for the learn step (Agent.learn, x_transformers_rl.py:816-924): one wave per
// token gathers the episode's step from the device trajectory (no host round trip), shifts actions
// and rewards right by one step, normalises [state, previous reward] with the RSNorm statistics,
// and copies the loss inputs; the masked column mean of the normalised rows (the RSNorm copy
// update's batch mean, xtrl.py:1005) is reduced in fixed order.
#include "kernels.h"

namespace xtrl {
namespace {

__global__ __launch_bounds__(256) void k_gather(const XtrlBatchDesc D) {
  const int lane = threadIdx.x & 63;
  const int tk = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tk >= D.b * D.n) return;
  const int j = tk / D.n, t = tk - j * D.n;
  const int64_t ep = D.idx[j];
  const int64_t src = ep * D.Tmax + t;   // row of (episode, step) in the trajectory
  const int S1 = D.S + 1;
  // [state, previous reward], RSNorm-normalised: (x - mean) / clamp(sqrt(var), 1e-5)
  for (int c = lane; c < S1; c += 64) {
    float x;
    if (c < D.S) x = D.states[src * D.S + c];
    else x = t > 0 ? D.rewards[src - 1] : 0.f;
    const float sd = fmaxf(sqrtf(D.rs_var[c]), 1e-5f);
    D.swr[(int64_t)tk * S1 + c] = (x - D.rs_mean[c]) / sd;
  }
  for (int k = lane; k < D.B; k += 64) D.old_values[(int64_t)tk * D.B + k] = D.values[src * D.B + k];
  if (D.continuous) {
    for (int i = lane; i < D.A; i += 64) {
      D.action_f[(int64_t)tk * D.A + i] = D.actions_f[src * D.A + i];
      D.prev_action_f[(int64_t)tk * D.A + i] = t > 0 ? D.actions_f[(src - 1) * D.A + i] : 0.f;
      D.old_logp[(int64_t)tk * D.A + i] = D.logp[src * D.A + i];
    }
  }
  if (lane == 0) {
    if (!D.continuous) {
      D.action[tk] = D.actions[src];
      D.prev_action[tk] = t > 0 ? D.actions[src - 1] : -1;
      D.old_logp[tk] = D.logp[src];
    }
    D.mb_returns[tk] = D.returns[ep * D.n + t];
    D.dones[tk] = D.bounds[src];
    if (t == 0) D.mb_lens[j] = D.lens[ep];
  }
}

// masked column sums of swr: part[blk][c] (c < S + 1) and part[blk][S + 1] = valid-token count
constexpr int RS_BLOCKS = 64;
__global__ __launch_bounds__(256) void k_rs_part(const XtrlBatchDesc D) {
  __shared__ float red[256];
  const int S1 = D.S + 1, T = D.b * D.n;
  const int per = (T + RS_BLOCKS - 1) / RS_BLOCKS, t0 = blockIdx.x * per, t1 = min(T, t0 + per);
  for (int c = 0; c <= S1; ++c) {
    float s = 0.f;
    for (int tk = t0 + threadIdx.x; tk < t1; tk += 256) {
      const int j = tk / D.n, t = tk - j * D.n;
      if (t < D.lens[D.idx[j]]) s += c < S1 ? D.swr[(int64_t)tk * S1 + c] : 1.f;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) D.rs_part[blockIdx.x * (S1 + 1) + c] = red[0];
    __syncthreads();
  }
}

__global__ void k_rs_final(const XtrlBatchDesc D) {
  const int S1 = D.S + 1, c = threadIdx.x;
  if (c >= S1) return;
  float s = 0.f, n = 0.f;
  for (int k = 0; k < RS_BLOCKS; ++k) {
    s += D.rs_part[k * (S1 + 1) + c];
    n += D.rs_part[k * (S1 + 1) + S1];
  }
  D.rs_m[c] = s / n;
}

__global__ void k_rsnorm_update(float* mean, float* var, const float* m, int D, float tf, float c) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= D) return;
  const float delta = m[i] - mean[i];
  mean[i] = mean[i] + delta / tf;
  var[i] = c * (var[i] + (delta * delta) / tf);
}

}  // namespace
}  // namespace xtrl

extern "C" int xtrl_minibatch_gather(const XtrlBatchDesc* D, void* stream) {
  XTRL_REQUIRE(D && D->b > 0 && D->n > 0 && D->n <= D->Tmax && D->S > 0 && D->S < 64, "gather: bad sizes");
  XTRL_REQUIRE(D->continuous ? (D->actions_f && D->action_f && D->prev_action_f)
                             : (D->actions && D->action && D->prev_action),
               "gather: missing action buffers");
  XTRL_REQUIRE(D->states && D->rewards && D->logp && D->bounds && D->values && D->returns && D->lens && D->idx &&
                   D->rs_mean && D->rs_var && D->swr && D->old_logp && D->mb_returns && D->old_values && D->dones &&
                   D->mb_lens && D->rs_part && D->rs_m,
               "gather: null buffer");
  hipStream_t s = xtrl::as_stream(stream);
  const int T = D->b * D->n;
  hipLaunchKernelGGL(xtrl::k_gather, dim3((T + 3) / 4), dim3(256), 0, s, *D);
  hipLaunchKernelGGL(xtrl::k_rs_part, dim3(xtrl::RS_BLOCKS), dim3(256), 0, s, *D);
  hipLaunchKernelGGL(xtrl::k_rs_final, dim3(1), dim3(64), 0, s, *D);
  XTRL_LAUNCHED("minibatch_gather");
  return XTRL_OK;
}

extern "C" int xtrl_rsnorm_update(float* mean, float* var, const float* m, int D, int t, void* stream) {
  XTRL_REQUIRE(mean && var && m && D > 0 && t >= 1, "rsnorm_update: bad arguments");
  const float c = (float)((double)(t - 1) / (double)t);
  hipLaunchKernelGGL(xtrl::k_rsnorm_update, dim3((D + 63) / 64), dim3(64), 0, xtrl::as_stream(stream), mean, var, m,
                     D, (float)t, c);
  XTRL_LAUNCHED("rsnorm_update");
  return XTRL_OK;
}
