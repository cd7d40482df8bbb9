// libgymrl.so -- the per-minibatch policy bookkeeping of the PPO update (include/gymrl.h ABI 6, rl_policy_kl and
// rl_adaptive_lr).
//
// rl_games a2c_common.py after each minibatch's optimizer step: kl_dist = policy_kl(mu, sigma, old_mu, old_sigma)
// (torch_ext.policy_kl: sum over the action dims of log(s1/s0 + 1e-5) + (s0^2 + (m1 - m0)^2) / (2 (s1^2 + 1e-5))
// - 0.5, mean over the rows), dataset.update_mu_sigma(mu, sigma), the adaptive learning-rate scheduler
// (schedulers.py AdaptiveScheduler: lr / 1.5 above 2 kl_threshold, lr * 1.5 below kl_threshold / 2, clamped to
// [1e-6, 1e-2]) and the epoch's loss / kl meters.  torch spends ~12 launches on these statements; here:
//   k_kl_part : per workgroup, the KL of its rows summed in a fixed order (+ the dataset's mu / sigma rows written
//               with the new values, the same elements each thread has just read)
//   k_kl_fin  : one workgroup sums the partials in block order, / rows -> kl
//   k_lr      : one thread: kl / world, the scheduler step in float64, the meters (a2c_continuous.py _mb_finish)
// (libgymrl builds with -ffp-contract=off: each statement rounds as torch's elementwise kernels do)
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kThreads = 256;
constexpr int kBlocks = 256;  // partials: kBlocks floats

// the single-rank minibatch: the scheduler and the meters run in the last workgroup of k_kl_part (a vector
// atomic counter; the workgroups' partials are summed in the same fixed order as k_kl_fin)
struct LrStep {
  int on;  // 0: k_kl_fin / rl_adaptive_lr do it (a KL all-reduce sits between)
  int adaptive;
  double threshold;
  double* lr;
  float* opt_lr;
  float* stats;
  const float *a_loss, *c_loss, *entropy;
  unsigned int* counter;
};

__device__ __forceinline__ void lr_step(float* kl, float k, int adaptive, double threshold, double* lr, float* opt_lr,
                                        float* stats, const float* a_loss, const float* c_loss, const float* entropy) {
  *kl = k;
  if (adaptive) {
    const double kd = (double)k, cur = *lr;
    double next = cur;
    if (kd > 2.0 * threshold) next = fmax(cur / 1.5, 1e-6);
    if (kd < 0.5 * threshold) next = fmin(cur * 1.5, 1e-2);
    *lr = next;
    if (opt_lr) *opt_lr = (float)next;
  }
  if (stats) {
    stats[0] += *a_loss;
    stats[1] += *c_loss;
    stats[2] += k;
    stats[3] += *entropy;
  }
}

__device__ __forceinline__ float tree_sum(float* sh) {
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  return sh[0];
}

template <bool HALF>
__global__ __launch_bounds__(kThreads) void k_kl_part(const void* __restrict__ mu_new, const float* __restrict__ sg_new,
                                                      int64_t sg_stride, int sg_log, float* __restrict__ mu_old,
                                                      float* __restrict__ sg_old, int M, int A, int write_back,
                                                      float* __restrict__ part, float* __restrict__ kl, LrStep L) {
  __shared__ float sh[kThreads];
  __shared__ bool last;
  const int rows_per = (M + kBlocks - 1) / kBlocks;
  const int r0 = blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  float acc = 0.f;
  for (int r = r0 + (int)threadIdx.x; r < r1; r += kThreads) {
    float row = 0.f;
    for (int a = 0; a < A; ++a) {
      const int64_t i = (int64_t)r * A + a;
      const float m0 = HALF ? __half2float(static_cast<const __half*>(mu_new)[i]) : static_cast<const float*>(mu_new)[i];
      const float sv = sg_new[r * sg_stride + a];
      const float s0 = sg_log ? expf(sv) : sv;  // sigma = exp(logstd) (the fixed-sigma parameter)
      const float m1 = mu_old[i], s1 = sg_old[i];
      const float c1 = logf(s1 / s0 + 1e-5f);
      const float dm = m1 - m0;
      const float c2 = (s0 * s0 + dm * dm) / (2.0f * (s1 * s1 + 1e-5f));
      row += c1 + c2 - 0.5f;
      if (write_back) {  // dataset.update_mu_sigma: the new policy's values replace the ones just read
        mu_old[i] = m0;
        sg_old[i] = s0;
      }
    }
    acc += row;
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  const float total = tree_sum(sh);
  if (!L.on) {
    if (threadIdx.x == 0) part[blockIdx.x] = total;
    return;
  }
  // the hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): the partial stored, waited for, released at agent
  // scope, then the agent-scope counter add; the last workgroup acquires before anyone of it loads the partials
  if (threadIdx.x == 0) {
    part[blockIdx.x] = total;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = atomicAdd(L.counter, 1u) == (unsigned)(gridDim.x - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  sh[threadIdx.x] = threadIdx.x < kBlocks ? part[threadIdx.x] : 0.f;
  __syncthreads();
  const float k = tree_sum(sh) / (float)M;
  if (threadIdx.x == 0) {
    lr_step(kl, k, L.adaptive, L.threshold, L.lr, L.opt_lr, L.stats, L.a_loss, L.c_loss, L.entropy);
    *L.counter = 0u;  // ready for the next launch
  }
}

__global__ __launch_bounds__(kThreads) void k_kl_fin(const float* __restrict__ part, int M, float* __restrict__ kl) {
  __shared__ float sh[kThreads];
  sh[threadIdx.x] = threadIdx.x < kBlocks ? part[threadIdx.x] : 0.f;
  __syncthreads();
  const float s = tree_sum(sh);
  if (threadIdx.x == 0) *kl = s / (float)M;
}

__global__ void k_lr(float* __restrict__ kl, float inv_world, int adaptive, double threshold, double* __restrict__ lr,
                     float* __restrict__ opt_lr, float* __restrict__ stats, const float* __restrict__ a_loss,
                     const float* __restrict__ c_loss, const float* __restrict__ entropy) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float k = inv_world != 1.0f ? *kl * inv_world : *kl;
  lr_step(kl, k, adaptive, threshold, lr, opt_lr, stats, a_loss, c_loss, entropy);
}

int launch_fail(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  return rl_set_error(what) + 1;
}

}  // namespace

extern "C" int rl_kl_partials_size(void) { return kBlocks + 1; }  // + the last-workgroup counter

static int launch_kl(const void* mu_new, int32_t mu_half, const float* sigma_new, int64_t sigma_row_stride,
                     int32_t sigma_is_log, float* mu_old, float* sigma_old, int32_t M, int32_t A, int32_t write_back,
                     float* kl, float* partials, const LrStep& L, hipStream_t st) {
  if (mu_half)
    hipLaunchKernelGGL(k_kl_part<true>, dim3(kBlocks), dim3(kThreads), 0, st, mu_new, sigma_new, sigma_row_stride,
                       (int)sigma_is_log, mu_old, sigma_old, M, A, write_back, partials, kl, L);
  else
    hipLaunchKernelGGL(k_kl_part<false>, dim3(kBlocks), dim3(kThreads), 0, st, mu_new, sigma_new, sigma_row_stride,
                       (int)sigma_is_log, mu_old, sigma_old, M, A, write_back, partials, kl, L);
  return launch_fail("rl_policy_kl: launch failed");
}

extern "C" int rl_policy_kl(const void* mu_new, int32_t mu_half, const float* sigma_new, int64_t sigma_row_stride,
                            int32_t sigma_is_log, float* mu_old, float* sigma_old, int32_t M, int32_t A,
                            int32_t write_back, float* kl, float* partials, void* stream) {
  if (!mu_new || !sigma_new || !mu_old || !sigma_old || !kl || !partials || M <= 0 || A <= 0 || sigma_row_stride < 0)
    return rl_set_error("rl_policy_kl: null pointer or empty shape");
  hipStream_t st = (hipStream_t)stream;
  LrStep L{};
  if (int rc = launch_kl(mu_new, mu_half, sigma_new, sigma_row_stride, sigma_is_log, mu_old, sigma_old, M, A,
                         write_back, kl, partials, L, st))
    return rc;
  hipLaunchKernelGGL(k_kl_fin, dim3(1), dim3(kThreads), 0, st, partials, M, kl);
  return launch_fail("rl_policy_kl: launch failed");
}

extern "C" int rl_policy_kl_step(const void* mu_new, int32_t mu_half, const float* sigma_new,
                                 int64_t sigma_row_stride, int32_t sigma_is_log, float* mu_old, float* sigma_old,
                                 int32_t M, int32_t A, int32_t write_back, float* kl, float* partials, int32_t adaptive,
                                 double kl_threshold, double* lr, float* opt_lr, float* stats, const float* a_loss,
                                 const float* c_loss, const float* entropy, void* stream) {
  if (!mu_new || !sigma_new || !mu_old || !sigma_old || !kl || !partials || M <= 0 || A <= 0 || sigma_row_stride < 0)
    return rl_set_error("rl_policy_kl_step: null pointer or empty shape");
  if ((adaptive && !lr) || (stats && (!a_loss || !c_loss || !entropy)))
    return rl_set_error("rl_policy_kl_step: null pointer");
  LrStep L{1, adaptive, kl_threshold, lr, opt_lr, stats, a_loss, c_loss, entropy,
           reinterpret_cast<unsigned int*>(partials + kBlocks)};
  return launch_kl(mu_new, mu_half, sigma_new, sigma_row_stride, sigma_is_log, mu_old, sigma_old, M, A, write_back, kl,
                   partials, L, (hipStream_t)stream);
}
extern "C" int rl_adaptive_lr(float* kl, float inv_world, int32_t adaptive, double kl_threshold, double* lr,
                              float* opt_lr, float* stats, const float* a_loss, const float* c_loss,
                              const float* entropy, void* stream) {
  if (!kl || (adaptive && !lr) || (stats && (!a_loss || !c_loss || !entropy)))
    return rl_set_error("rl_adaptive_lr: null pointer");
  hipLaunchKernelGGL(k_lr, dim3(1), dim3(64), 0, (hipStream_t)stream, kl, inv_world, adaptive, kl_threshold, lr, opt_lr,
                     stats, a_loss, c_loss, entropy);
  return launch_fail("rl_adaptive_lr: launch failed");
}
