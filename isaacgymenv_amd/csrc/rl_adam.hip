// libgymrl.so -- the PPO minibatch optimizer step as three launches (include/gymrl.h rl_opt_step), or two with the
// fp16 parameter shadow written by the update (rl_opt_step_h: the finish runs in k_opt_adam's last workgroup).
//
// rl_games a2c_common.py trancate_gradients_and_step with mixed precision: scaler.unscale_(optimizer),
// clip_grad_norm_(params, grad_norm), scaler.step(optimizer) (torch.optim.Adam, skipped when a gradient
// is not finite), scaler.update().  torch spends ~20 launches on it (per-tensor unscale and found-inf,
// per-tensor norms and their norm, clip multiply, the fused Adam, the scale update); the parameters,
// gradients and Adam moments of this learner are each ONE flat buffer (rl/a2c_continuous.py), so here:
//   k_opt_norm  : per workgroup, sum of (g / scale)^2 over its slice (fixed order) and a non-finite flag
//   k_opt_adam  : every workgroup sums the partials in the same fixed order (the norm, found-inf), then the
//                 clip coefficient and Adam (torch's update: m.lerp_(g, 1 - b1), v = b2 v + (1 - b2) g^2,
//                 p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)) on its slice; nothing when found-inf
//   k_opt_finish: step += 1 unless found-inf; GradScaler.update (backoff on inf, growth every interval)
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kThreads = 256;
constexpr int kBlocks = 256;  // partials: [kBlocks] sums, [kBlocks] non-finite flags

__device__ __forceinline__ float block_sum(float x, float* sh) {
  const int t = threadIdx.x;
  sh[t] = x;
  __syncthreads();
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] += sh[t + s];
    __syncthreads();
  }
  const float r = sh[0];
  __syncthreads();
  return r;
}

__device__ __forceinline__ void slice(int64_t n, int64_t& b, int64_t& e) {
  const int64_t chunk = (n + kBlocks - 1) / kBlocks;
  b = (int64_t)blockIdx.x * chunk;
  e = b + chunk < n ? b + chunk : n;
}

__global__ __launch_bounds__(kThreads) void k_opt_norm(const float* __restrict__ grad, int64_t n,
                                                       const float* __restrict__ scale, float* __restrict__ part) {
  __shared__ float sh[kThreads];
  const float inv = scale ? 1.0f / *scale : 1.0f;
  int64_t b, e;
  slice(n, b, e);
  float acc = 0.f, bad = 0.f;
  for (int64_t i = b + threadIdx.x; i < e; i += kThreads) {
    const float g = grad[i] * inv;
    if (!isfinite(g)) bad = 1.f;
    acc += g * g;
  }
  acc = block_sum(acc, sh);
  bad = block_sum(bad, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = acc;
    part[kBlocks + blockIdx.x] = bad;
  }
}

// the partials, summed in the same order in every workgroup: (squared norm, found_inf)
__device__ __forceinline__ void totals(const float* __restrict__ part, float* sh, float& sq, bool& found) {
  sq = block_sum(threadIdx.x < kBlocks ? part[threadIdx.x] : 0.f, sh);
  found = block_sum(threadIdx.x < kBlocks ? part[kBlocks + threadIdx.x] : 0.f, sh) > 0.f;
}

// the step's bookkeeping (torch: step += 1 in Adam, GradScaler.update): after every workgroup's Adam
__device__ __forceinline__ void opt_finish(float* __restrict__ step, float* __restrict__ scale,
                                           int32_t* __restrict__ tracker, bool found, const rl_opt_hyper& h) {
  if (!found || !scale) *step += 1.f;  // (a skipped step exists only with loss scaling, k_opt_adam)
  if (scale && tracker) {  // torch._amp_update_scale_
    if (found) {
      *scale *= h.backoff;
      *tracker = 0;
    } else {
      const int32_t s = *tracker + 1;
      if (s == h.growth_interval) {
        const float grown = *scale * h.growth;
        if (isfinite(grown)) *scale = grown;  // growth only while the scale stays finite
        *tracker = 0;
      } else {
        *tracker = s;
      }
    }
  }
}

// phalf (nullable): the parameters' fp16 shadow written with the update (the next minibatch's GEMM operands);
// counter (nullable): the last workgroup to finish runs opt_finish (ONE launch instead of k_opt_adam + k_opt_finish;
// every workgroup reads step and scale before it counts itself done)
__global__ __launch_bounds__(kThreads) void k_opt_adam(float* __restrict__ param, const float* __restrict__ grad,
                                                       float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                       float* __restrict__ step, const float* __restrict__ lr,
                                                       float* __restrict__ scale, const float* __restrict__ part,
                                                       rl_opt_hyper h, __half* __restrict__ phalf,
                                                       int32_t* __restrict__ tracker, unsigned int* __restrict__ counter) {
  __shared__ float sh[kThreads];
  __shared__ bool last;
  float sq;
  bool found;
  totals(part, sh, sq, found);
  // GradScaler.step skips the optimizer step on a non-finite gradient; without loss scaling torch's Adam steps
  // anyway (and a non-finite gradient makes the parameters non-finite, as there)
  if (!(found && scale)) {
    float coef = 1.f;
    if (h.max_norm > 0.f) {  // clip_grad_norm_: max_norm / (total_norm + 1e-6), clamp(max=1) (NaN stays NaN)
      const float c = h.max_norm / (sqrtf(sq) + 1e-6f);
      coef = c > 1.f ? 1.f : c;
    }
    const float gs = (scale ? 1.0f / *scale : 1.0f) * coef;
    const float t = *step + 1.f;
    const float bc1 = 1.f - powf(h.beta1, t);
    const float bc2 = 1.f - powf(h.beta2, t);
    const float step_size = *lr / bc1;
    const float bc2_sqrt = sqrtf(bc2);
    int64_t b, e;
    slice(n, b, e);
    for (int64_t i = b + threadIdx.x; i < e; i += kThreads) {
      float g = grad[i] * gs;
      float p = param[i];
      if (h.weight_decay != 0.f) g += h.weight_decay * p;
      float mi = m[i], vi = v[i];
      mi = mi + (1.f - h.beta1) * (g - mi);
      vi = h.beta2 * vi + (1.f - h.beta2) * g * g;
      const float denom = sqrtf(vi) / bc2_sqrt + h.eps;
      p -= step_size * (mi / denom);
      m[i] = mi;
      v[i] = vi;
      param[i] = p;
      if (phalf) phalf[i] = __float2half(p);
    }
  }
  if (!counter) return;
  // nothing is handed over (each workgroup has its own found / norm): the counter only orders the last
  // workgroup's step / scale update after every workgroup's reads of them, which completed before its add
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(counter, 1u) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    opt_finish(step, scale, tracker, found, h);
    *counter = 0u;  // ready for the next launch
  }
}

__global__ __launch_bounds__(kThreads) void k_opt_finish(float* __restrict__ step, float* __restrict__ scale,
                                                         int32_t* __restrict__ tracker, const float* __restrict__ part,
                                                         rl_opt_hyper h) {
  __shared__ float sh[kThreads];
  float sq;
  bool found;
  totals(part, sh, sq, found);
  if (threadIdx.x != 0) return;
  opt_finish(step, scale, tracker, found, h);
}

}  // namespace

extern "C" int rl_opt_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float* step,
                           const float* lr, float* scale, int32_t* growth_tracker, const rl_opt_hyper* hyper,
                           float* partials, void* stream) {
  if (n <= 0 || !param || !grad || !exp_avg || !exp_avg_sq || !step || !lr || !hyper || !partials)
    return rl_set_error("rl_opt_step: null pointer or n <= 0");
  if ((scale == nullptr) != (growth_tracker == nullptr))
    return rl_set_error("rl_opt_step: scale and growth_tracker come together (both null: no loss scaling)");
  hipStream_t st = (hipStream_t)stream;
  const rl_opt_hyper h = *hyper;
  hipLaunchKernelGGL(k_opt_norm, dim3(kBlocks), dim3(kThreads), 0, st, grad, n, scale, partials);
  hipLaunchKernelGGL(k_opt_adam, dim3(kBlocks), dim3(kThreads), 0, st, param, grad, exp_avg, exp_avg_sq, n, step, lr,
                     scale, partials, h, (__half*)nullptr, growth_tracker, (unsigned int*)nullptr);
  hipLaunchKernelGGL(k_opt_finish, dim3(1), dim3(kThreads), 0, st, step, scale, growth_tracker, partials, h);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    char msg[256];
    snprintf(msg, sizeof(msg), "rl_opt_step: launch failed: %s", hipGetErrorString(e));
    return rl_set_error(msg) + 1;
  }
  return 0;
}

extern "C" int rl_opt_partials_size(void) { return 2 * kBlocks + 1; }  // + the last-workgroup counter

extern "C" int rl_opt_step_h(float* param, void* param_half, const float* grad, float* exp_avg, float* exp_avg_sq,
                             int64_t n, float* step, const float* lr, float* scale, int32_t* growth_tracker,
                             const rl_opt_hyper* hyper, float* partials, void* stream) {
  if (n <= 0 || !param || !param_half || !grad || !exp_avg || !exp_avg_sq || !step || !lr || !hyper || !partials)
    return rl_set_error("rl_opt_step_h: null pointer or n <= 0");
  if ((scale == nullptr) != (growth_tracker == nullptr))
    return rl_set_error("rl_opt_step_h: scale and growth_tracker come together (both null: no loss scaling)");
  hipStream_t st = (hipStream_t)stream;
  const rl_opt_hyper h = *hyper;
  hipLaunchKernelGGL(k_opt_norm, dim3(kBlocks), dim3(kThreads), 0, st, grad, n, scale, partials);
  hipLaunchKernelGGL(k_opt_adam, dim3(kBlocks), dim3(kThreads), 0, st, param, grad, exp_avg, exp_avg_sq, n, step, lr,
                     scale, partials, h, (__half*)param_half, growth_tracker,
                     reinterpret_cast<unsigned int*>(partials + 2 * kBlocks));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    char msg[256];
    snprintf(msg, sizeof(msg), "rl_opt_step_h: launch failed: %s", hipGetErrorString(e));
    return rl_set_error(msg) + 1;
  }
  return 0;
}
