// libgymrl.so -- input normalisation of the PPO model (include/gymrl.h rl_rms_normalize).
//
// rl_games algos_torch/running_mean_std.py RunningMeanStd (rl-games 1.6.x), rl/running_mean_std.py:
// in train mode every forward merges the batch moments (mean, unbiased var over axis 0) into the
// float64 running moments, then y = clamp((x - mean) / sqrt(var + eps), -5, 5) with the float32
// casts of the running moments.  torch spends ~25 launches on it (a Welford reduction of ~40 us at
// 16384 x 188, ~15 float64 elementwise ops on [C], the normalisation chain); here:
//   k_rms_part: workgroup b, lane c = column c: Welford over the workgroup's rows (fp32)
//   k_rms_fin : lane c merges the workgroups' (mean, M2) in fp64 in block order (Chan et al.), rounds the
//               batch mean / var to fp32 as torch's fp32 reductions return them, then updates the running
//               moments with the reference formula in fp64, same operation order
//   k_rms_norm: the normalisation (also the eval-mode path, update = 0)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kCols = 256;     // columns <= 256: one lane each
constexpr int kRowBlock = 128; // rows per partial

__global__ __launch_bounds__(kCols) void k_rms_part(const float* __restrict__ x, int N, int C,
                                                    float* __restrict__ part) {
    const int c = threadIdx.x;
    if (c >= C) return;
    const int r0 = blockIdx.x * kRowBlock, r1 = min(N, r0 + kRowBlock);
    float mean = 0.f, m2 = 0.f;
    int n = 0;
    for (int r = r0; r < r1; ++r) {
        const float v = x[(size_t)r * C + c];
        ++n;
        const float d = v - mean;
        mean += d / (float)n;
        m2 += d * (v - mean);
    }
    part[((size_t)blockIdx.x * C + c) * 2 + 0] = mean;
    part[((size_t)blockIdx.x * C + c) * 2 + 1] = m2;
}

__global__ __launch_bounds__(kCols) void k_rms_fin(const float* __restrict__ part, int blocks, int N, int C,
                                                   double* __restrict__ rmean, double* __restrict__ rvar,
                                                   double* __restrict__ count) {
    const int c = threadIdx.x;
    const double cnt = *count;  // every lane reads it before lane 0 updates it
    __syncthreads();
    if (c < C) {
        double na = 0.0, mean = 0.0, M2 = 0.0;
        for (int b = 0; b < blocks; ++b) {
            const double nb = (double)(min(N, (b + 1) * kRowBlock) - b * kRowBlock);
            const double pm = part[((size_t)b * C + c) * 2 + 0], pm2 = part[((size_t)b * C + c) * 2 + 1];
            const double tot = na + nb;
            const double delta = pm - mean;
            mean += delta * nb / tot;
            M2 += pm2 + delta * delta * na * nb / tot;
            na = tot;
        }
        // torch: input.mean / input.var on float32 return float32
        const double bmean = (double)(float)mean;
        const double bvar = (double)(float)(N > 1 ? M2 / (double)(N - 1) : 0.0);
        const double bc = (double)N;
        // RunningMeanStd._update_mean_var_count_from_moments, same order of operations
        const double delta = bmean - rmean[c];
        const double tot = cnt + bc;
        const double new_mean = rmean[c] + delta * bc / tot;
        const double m_a = rvar[c] * cnt;
        const double m_b = bvar * bc;
        const double m2 = m_a + m_b + delta * delta * cnt * bc / tot;
        rmean[c] = new_mean;
        rvar[c] = m2 / tot;
    }
    if (c == 0) *count = cnt + (double)N;
}

__global__ __launch_bounds__(256) void k_rms_norm(const float* __restrict__ x, int64_t n, int C,
                                                  const double* __restrict__ rmean, const double* __restrict__ rvar,
                                                  float eps, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = (int)(i % C);
    const float m = (float)rmean[c];
    const float d = sqrtf((float)rvar[c] + eps);
    y[i] = fminf(fmaxf((x[i] - m) / d, -5.f), 5.f);
}

}  // namespace

extern "C" int rl_rms_normalize(const float* x, int32_t rows, int32_t cols, double* running_mean, double* running_var,
                                double* count, double epsilon, int32_t update, float* partials, float* y,
                                void* stream) {
    if (rows <= 0 || cols <= 0 || cols > kCols) return rl_set_error("rl_rms_normalize: rows > 0, 0 < cols <= 256");
    if (!x || !running_mean || !running_var || !y || (update && (!count || !partials)))
        return rl_set_error("rl_rms_normalize: null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (update) {
        const int blocks = (rows + kRowBlock - 1) / kRowBlock;
        hipLaunchKernelGGL(k_rms_part, dim3(blocks), dim3(kCols), 0, st, x, (int)rows, (int)cols, partials);
        hipLaunchKernelGGL(k_rms_fin, dim3(1), dim3(kCols), 0, st, partials, blocks, (int)rows, (int)cols,
                           running_mean, running_var, count);
    }
    const int64_t n = (int64_t)rows * cols;
    hipLaunchKernelGGL(k_rms_norm, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, (int)cols,
                       running_mean, running_var, (float)epsilon, y);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_rms_normalize: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}
