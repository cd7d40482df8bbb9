// libgymrl.so -- input normalisation of the PPO model (include/gymrl.h rl_rms_normalize).
//
// rl_games algos_torch/running_mean_std.py RunningMeanStd (rl-games 1.6.x), rl/running_mean_std.py:
// in train mode every forward merges the batch moments (mean, unbiased var over axis 0) into the
// float64 running moments, then y = clamp((x - mean) / sqrt(var + eps), -5, 5) with the float32
// casts of the running moments.  torch spends ~25 launches on it (a Welford reduction of ~40 us at
// 16384 x 188, ~15 float64 elementwise ops on [C], the normalisation chain); here:
//   k_rms_part: workgroup b, lane c = column c: Welford over the workgroup's 64 rows (fp32, loads issued 8 ahead)
//   k_rms_fin : 64 lanes per column merge the workgroups' (mean, M2) in fp64 (Chan et al.; lane j takes blocks
//               j, j + 64, ... in order, then a fixed pairwise tree: deterministic), rounds the
//               batch mean / var to fp32 as torch's fp32 reductions return them, then updates the running
//               moments with the reference formula in fp64, same operation order
//   k_rms_norm: the normalisation (also the eval-mode path, update = 0); bumps the running count
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kCols = 256;     // columns <= 256
constexpr int kRowBlock = 64;  // rows per partial
constexpr int kPre = 8;        // loads issued ahead of the dependent Welford / merge chain
constexpr int kFinCols = 4;    // finish: columns per workgroup, kFinSub lanes per column
constexpr int kFinSub = 64;

__global__ __launch_bounds__(kCols) void k_rms_part(const float* __restrict__ x, int N, int C,
                                                    float* __restrict__ part) {
    const int c = threadIdx.x;
    if (c >= C) return;
    const int r0 = blockIdx.x * kRowBlock, r1 = min(N, r0 + kRowBlock);
    float mean = 0.f, m2 = 0.f;
    int n = 0;
    for (int r = r0; r < r1; r += kPre) {
        float v[kPre];
#pragma unroll
        for (int k = 0; k < kPre; ++k) v[k] = r + k < r1 ? x[(size_t)(r + k) * C + c] : 0.f;
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            if (r + k < r1) {
                ++n;
                const float d = v[k] - mean;
                mean += d / (float)n;
                m2 += d * (v[k] - mean);
            }
        }
    }
    part[((size_t)blockIdx.x * C + c) * 2 + 0] = mean;
    part[((size_t)blockIdx.x * C + c) * 2 + 1] = m2;
}

// Chan et al. merge of (na, mean, M2) with (nb, pm, pm2), float64
__device__ __forceinline__ void merge(double& na, double& mean, double& M2, double nb, double pm, double pm2) {
    const double tot = na + nb;
    const double delta = pm - mean;
    mean += delta * nb / tot;
    M2 += pm2 + delta * delta * na * nb / tot;
    na = tot;
}

// workgroup = kFinCols columns x kFinSub lanes; lane j merges the partials b = j, j + kFinSub, ... in order, then
// the kFinSub lane results are merged pairwise in a fixed tree (lane j with lane j + s, s = 32, 16, ..., 1):
// deterministic, and 47 workgroups of short fp64 chains instead of 3 workgroups of 64-long ones (34.5 -> ~2 us)
__global__ __launch_bounds__(kFinCols * kFinSub) void k_rms_fin(const float* __restrict__ part, int blocks, int N,
                                                                int C, double* __restrict__ rmean,
                                                                double* __restrict__ rvar,
                                                                const double* __restrict__ count) {
    __shared__ double sh[kFinCols][kFinSub][3];
    const int j = threadIdx.x % kFinSub, cl = threadIdx.x / kFinSub;
    const int c = blockIdx.x * kFinCols + cl;
    double na = 0.0, mean = 0.0, M2 = 0.0;
    if (c < C) {
        for (int b = j; b < blocks; b += kFinSub) {
            const float pm = part[((size_t)b * C + c) * 2 + 0], pm2 = part[((size_t)b * C + c) * 2 + 1];
            merge(na, mean, M2, (double)(min(N, (b + 1) * kRowBlock) - b * kRowBlock), pm, pm2);
        }
    }
    sh[cl][j][0] = na;
    sh[cl][j][1] = mean;
    sh[cl][j][2] = M2;
    __syncthreads();
    for (int st = kFinSub / 2; st > 0; st >>= 1) {
        if (j < st && sh[cl][j + st][0] > 0.0) {
            merge(na, mean, M2, sh[cl][j + st][0], sh[cl][j + st][1], sh[cl][j + st][2]);
            sh[cl][j][0] = na;
            sh[cl][j][1] = mean;
            sh[cl][j][2] = M2;
        }
        __syncthreads();
    }
    if (j != 0 || c >= C) return;
    const double cnt = *count;  // updated by k_rms_norm, after every column's update
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

template <class TY>  // float, or __half: the fp16 operand the learner's first layer casts it to anyway
__global__ __launch_bounds__(256) void k_rms_norm(const float* __restrict__ x, int64_t n, int C,
                                                  const double* __restrict__ rmean, const double* __restrict__ rvar,
                                                  float eps, TY* __restrict__ y, double* __restrict__ count,
                                                  double add) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (count && i == 0) *count += add;  // the running count, after k_rms_fin read it
    if (i >= n) return;
    const int c = (int)(i % C);
    const float m = (float)rmean[c];
    const float d = sqrtf((float)rvar[c] + eps);
    const float v = fminf(fmaxf((x[i] - m) / d, -5.f), 5.f);
    if constexpr (sizeof(TY) == 2) y[i] = __float2half(v);
    else y[i] = v;
}

}  // namespace

static int rms_normalize(const float* x, int32_t rows, int32_t cols, double* running_mean, double* running_var,
                         double* count, double epsilon, int32_t update, float* partials, void* y, bool half,
                         void* stream) {
    if (rows <= 0 || cols <= 0 || cols > kCols) return rl_set_error("rl_rms_normalize: rows > 0, 0 < cols <= 256");
    if (!x || !running_mean || !running_var || !y || (update && (!count || !partials)))
        return rl_set_error("rl_rms_normalize: null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (update) {
        const int blocks = (rows + kRowBlock - 1) / kRowBlock;
        hipLaunchKernelGGL(k_rms_part, dim3(blocks), dim3(kCols), 0, st, x, (int)rows, (int)cols, partials);
        hipLaunchKernelGGL(k_rms_fin, dim3((cols + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinSub), 0, st, partials,
                           blocks, (int)rows, (int)cols, running_mean, running_var, count);
    }
    const int64_t n = (int64_t)rows * cols;
    if (half)
        hipLaunchKernelGGL(k_rms_norm<__half>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, (int)cols,
                           running_mean, running_var, (float)epsilon, (__half*)y, update ? count : nullptr, (double)rows);
    else
        hipLaunchKernelGGL(k_rms_norm<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, (int)cols,
                           running_mean, running_var, (float)epsilon, (float*)y, update ? count : nullptr, (double)rows);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_rms_normalize: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}

extern "C" int rl_rms_normalize(const float* x, int32_t rows, int32_t cols, double* running_mean, double* running_var,
                                double* count, double epsilon, int32_t update, float* partials, float* y,
                                void* stream) {
    return rms_normalize(x, rows, cols, running_mean, running_var, count, epsilon, update, partials, y, false, stream);
}

extern "C" int rl_rms_normalize_h(const float* x, int32_t rows, int32_t cols, double* running_mean,
                                  double* running_var, double* count, double epsilon, int32_t update, float* partials,
                                  void* y_half, void* stream) {
    return rms_normalize(x, rows, cols, running_mean, running_var, count, epsilon, update, partials, y_half, true,
                         stream);
}
