// libgymrl.so -- gradient finish of the PPO learner's split-K weight gradients (include/gymrl.h).
//
// The minibatch-sized Linear layers (rl/network.py) form dW = g^T x as SPLIT_K row-block partial
// products in one batched GEMM ([P][n] partials, fp16 under the config's mixed precision).  This
// kernel finishes them in ONE pass and adds the result straight into the parameter's fp32 gradient
// (a view into the learner's flat gradient buffer): grad[i] += sum_p part[p][i], the P partials added
// in ascending p order in fp32 (bit-identical run to run).  It replaces three launches per layer
// (torch's fp32 sum over the split axis ~10.6 us at 16 x 512 x 188 fp16, and autograd's
// accumulate-into-.grad add).
//
// HBM-bound elementwise: each lane owns 4 consecutive outputs, loads 8 B (fp16) / 16 B (fp32) per
// partial per lane: every wave load is a contiguous 512 B / 1 KB run; P independent loads in flight.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip: the message rl_last_error() returns; returns 1

namespace {

constexpr int kBlock = 256;
constexpr int kVec = 4;

// vec: n % 4 == 0 and both pointers aligned for the 4-wide accesses (host-checked; a gradient view inside
// the flat buffer may sit at any float offset), else the scalar path, same order of additions
// 64-thread workgroups: a layer's gradient is 33-131 k floats, i.e. 8-32 k lanes -- spread over every CU
constexpr int kAccBlock = 64;
template <bool HALF>
__global__ __launch_bounds__(kAccBlock) void k_splitk_accum(const void* __restrict__ parts, int P, int64_t n,
                                                            float* __restrict__ grad, bool vec) {
    const int64_t i0 = ((int64_t)blockIdx.x * kAccBlock + threadIdx.x) * kVec;
    if (i0 >= n) return;
    float acc[kVec] = {0.f, 0.f, 0.f, 0.f};
    if (vec) {
        // the partials in batches of 16 loads issued before any is added (one load latency per batch, not per
        // partial); the additions stay in ascending partial order (a last batch past P reloads partial P - 1 in
        // its spare slots and never adds them)
        constexpr int kBatch = 16;
        for (int p0 = 0; p0 < P; p0 += kBatch) {
            float4 v[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const int p = p0 + b < P ? p0 + b : P - 1;
                if constexpr (HALF) {
                    const __half2* src = reinterpret_cast<const __half2*>(static_cast<const __half*>(parts) + p * n + i0);
                    const float2 a = __half22float2(src[0]), c = __half22float2(src[1]);
                    v[b] = make_float4(a.x, a.y, c.x, c.y);
                } else {
                    v[b] = *reinterpret_cast<const float4*>(static_cast<const float*>(parts) + p * n + i0);
                }
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                if (p0 + b < P) { acc[0] += v[b].x; acc[1] += v[b].y; acc[2] += v[b].z; acc[3] += v[b].w; }
            }
        }
        float4 g = *reinterpret_cast<float4*>(grad + i0);
        g.x += acc[0]; g.y += acc[1]; g.z += acc[2]; g.w += acc[3];
        *reinterpret_cast<float4*>(grad + i0) = g;
        return;
    }
    for (int k = 0; k < kVec && i0 + k < n; ++k) {
        float a = 0.f;
        for (int p = 0; p < P; ++p) {
            if constexpr (HALF) a += __half2float(static_cast<const __half*>(parts)[p * n + i0 + k]);
            else a += static_cast<const float*>(parts)[p * n + i0 + k];
        }
        grad[i0 + k] += a;
    }
}

// several layers' finishes in one launch (rl_splitk_accum_multi): blocks [first[j], first[j + 1]) finish job j;
// store: grad = sum instead of grad += sum (the learner's fused path writes every gradient exactly once, so the
// flat gradient buffer needs no zeroing)
struct MultiJobs {
    const void* parts[RL_SPLITK_MAX_JOBS];
    float* grad[RL_SPLITK_MAX_JOBS];
    int64_t n[RL_SPLITK_MAX_JOBS];
    int32_t P[RL_SPLITK_MAX_JOBS];
    int32_t half[RL_SPLITK_MAX_JOBS];
    int32_t vec[RL_SPLITK_MAX_JOBS];
    int32_t first[RL_SPLITK_MAX_JOBS + 1];
    int32_t njobs, store;
};

template <bool HALF>
__device__ __forceinline__ void accum_lanes(const void* __restrict__ parts, int P, int64_t n, float* __restrict__ grad,
                                            bool vec, int64_t i0, bool store) {
    float acc[kVec] = {0.f, 0.f, 0.f, 0.f};
    if (vec) {
        constexpr int kBatch = 16;
        for (int p0 = 0; p0 < P; p0 += kBatch) {
            float4 v[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const int p = p0 + b < P ? p0 + b : P - 1;
                if constexpr (HALF) {
                    const __half2* src = reinterpret_cast<const __half2*>(static_cast<const __half*>(parts) + p * n + i0);
                    const float2 a = __half22float2(src[0]), c = __half22float2(src[1]);
                    v[b] = make_float4(a.x, a.y, c.x, c.y);
                } else {
                    v[b] = *reinterpret_cast<const float4*>(static_cast<const float*>(parts) + p * n + i0);
                }
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                if (p0 + b < P) { acc[0] += v[b].x; acc[1] += v[b].y; acc[2] += v[b].z; acc[3] += v[b].w; }
            }
        }
        float4 g = store ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<float4*>(grad + i0);
        g.x += acc[0]; g.y += acc[1]; g.z += acc[2]; g.w += acc[3];
        *reinterpret_cast<float4*>(grad + i0) = g;
        return;
    }
    for (int k = 0; k < kVec && i0 + k < n; ++k) {
        float a = 0.f;
        for (int p = 0; p < P; ++p) {
            if constexpr (HALF) a += __half2float(static_cast<const __half*>(parts)[p * n + i0 + k]);
            else a += static_cast<const float*>(parts)[p * n + i0 + k];
        }
        grad[i0 + k] = store ? a : grad[i0 + k] + a;
    }
}

__global__ __launch_bounds__(kAccBlock) void k_splitk_accum_multi(MultiJobs J) {
    int j = 0;
    while (j + 1 < J.njobs && (int)blockIdx.x >= J.first[j + 1]) ++j;
    const int64_t i0 = ((int64_t)(blockIdx.x - J.first[j]) * kAccBlock + threadIdx.x) * kVec;
    if (i0 >= J.n[j]) return;
    if (J.half[j]) accum_lanes<true>(J.parts[j], J.P[j], J.n[j], J.grad[j], J.vec[j], i0, J.store);
    else accum_lanes<false>(J.parts[j], J.P[j], J.n[j], J.grad[j], J.vec[j], i0, J.store);
}

}  // namespace

extern "C" int rl_splitk_accum_multi(const rl_splitk_job* jobs, int32_t num_jobs, int32_t store, void* stream) {
    if (!jobs || num_jobs <= 0 || num_jobs > RL_SPLITK_MAX_JOBS)
        return rl_set_error("rl_splitk_accum_multi: 1 <= num_jobs <= RL_SPLITK_MAX_JOBS jobs required");
    MultiJobs J{};
    int64_t blocks = 0;
    for (int j = 0; j < num_jobs; ++j) {
        const rl_splitk_job& q = jobs[j];
        if (q.num_parts <= 0 || q.n < 0 || (q.n > 0 && (!q.parts || !q.grad)))
            return rl_set_error("rl_splitk_accum_multi: a job has a null pointer, num_parts <= 0 or n < 0");
        const uintptr_t align = q.parts_are_f16 ? 8 : 16;
        J.parts[j] = q.parts;
        J.grad[j] = q.grad;
        J.n[j] = q.n;
        J.P[j] = q.num_parts;
        J.half[j] = q.parts_are_f16 ? 1 : 0;
        J.vec[j] = (q.n % kVec) == 0 && ((uintptr_t)q.parts % align) == 0 && ((uintptr_t)q.grad % 16) == 0;
        J.first[j] = (int32_t)blocks;
        blocks += ((q.n + kVec - 1) / kVec + kAccBlock - 1) / kAccBlock;
        if (blocks > INT32_MAX) return rl_set_error("rl_splitk_accum_multi: too many elements");
    }
    J.first[num_jobs] = (int32_t)blocks;
    J.njobs = num_jobs;
    J.store = store ? 1 : 0;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(k_splitk_accum_multi, dim3((unsigned)blocks), dim3(kAccBlock), 0, (hipStream_t)stream, J);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_splitk_accum_multi: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}

extern "C" int rl_splitk_accum(const void* parts, int32_t num_parts, int64_t n, int32_t parts_are_f16, float* grad,
                               void* stream) {
    if (num_parts <= 0 || n < 0) return rl_set_error("rl_splitk_accum: num_parts must be positive, n >= 0");
    if (n == 0) return 0;
    if (!parts || !grad) return rl_set_error("rl_splitk_accum: null pointer");
    const uintptr_t align = parts_are_f16 ? 8 : 16;
    const bool vec = (n % kVec) == 0 && ((uintptr_t)parts % align) == 0 && ((uintptr_t)grad % 16) == 0;
    const int64_t lanes = (n + kVec - 1) / kVec;
    const dim3 grid((unsigned)((lanes + kAccBlock - 1) / kAccBlock));
    if (parts_are_f16)
        hipLaunchKernelGGL(k_splitk_accum<true>, grid, dim3(kAccBlock), 0, (hipStream_t)stream, parts, (int)num_parts, n,
                           grad, vec);
    else
        hipLaunchKernelGGL(k_splitk_accum<false>, grid, dim3(kAccBlock), 0, (hipStream_t)stream, parts, (int)num_parts,
                           n, grad, vec);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_splitk_accum: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}

// ---------------------------------------------------------------- bias gradients
// grad[c] += sum_r g[r][c] over a [rows][cols] fp16 / f32 matrix (the bias gradient of a Linear layer
// is the column sum of its output gradient).  Deterministic, two launches:
//   k_colsum_part: workgroup b sums rows [b*R, (b+1)*R) (lane = 8 consecutive columns of one row,
//                  256 / (cols/8) rows side by side, folded in a fixed order) -> work[b][cols];
//   k_colsum_fin : workgroup = 8 columns; 32 lane groups each add every 32nd partial in order, then
//                  the 32 group sums are added in order into grad.
namespace {

constexpr int kColVec = 8;
constexpr int kMaxParts = 256;
constexpr int kFinGroups = kBlock / kColVec;  // 32

template <bool HALF>
__global__ __launch_bounds__(kBlock) void k_colsum_part(const void* __restrict__ g, int rows, int cols,
                                                        float* __restrict__ work) {
    __shared__ float red[kBlock * kColVec];
    const int cv = cols / kColVec;
    const int row_lanes = kBlock / cv;
    const int t = threadIdx.x;
    const int lane_row = t / cv, lane_col = t - lane_row * cv;
    const int per = (rows + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * per, r1 = min(rows, r0 + per);
    float acc[kColVec];
#pragma unroll
    for (int k = 0; k < kColVec; ++k) acc[k] = 0.f;
    if (lane_row < row_lanes) {
        for (int r = r0 + lane_row; r < r1; r += row_lanes) {
            if constexpr (HALF) {
                const uint4 raw = *reinterpret_cast<const uint4*>(static_cast<const __half*>(g) + (size_t)r * cols +
                                                                  lane_col * kColVec);
                const __half2* h = reinterpret_cast<const __half2*>(&raw);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float2 f = __half22float2(h[k]);
                    acc[2 * k] += f.x;
                    acc[2 * k + 1] += f.y;
                }
            } else {
                const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(g) + (size_t)r * cols +
                                                                  lane_col * kColVec);
                const float4 a = p[0], b = p[1];
                acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
                acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kColVec; ++k) red[t * kColVec + k] = acc[k];
    __syncthreads();
    for (int c = t; c < cols; c += kBlock) {
        const int v = c / kColVec, k = c - v * kColVec;
        float s = 0.f;
        for (int lr = 0; lr < row_lanes; ++lr) s += red[(lr * cv + v) * kColVec + k];
        work[(size_t)blockIdx.x * cols + c] = s;
    }
}

__global__ __launch_bounds__(kBlock) void k_colsum_fin(const float* __restrict__ work, int parts, int cols,
                                                       float* __restrict__ grad) {
    __shared__ float red[kFinGroups][kColVec];
    const int t = threadIdx.x;
    const int k = t % kColVec, j = t / kColVec;
    const int c = blockIdx.x * kColVec + k;
    float s = 0.f;
    if (c < cols)
        for (int b = j; b < parts; b += kFinGroups) s += work[(size_t)b * cols + c];
    red[j][k] = s;
    __syncthreads();
    if (t < kColVec && c < cols) {
        float a = 0.f;
        for (int q = 0; q < kFinGroups; ++q) a += red[q][t];
        grad[c] += a;
    }
}

}  // namespace

extern "C" int rl_colsum_accum(const void* g, int32_t rows, int32_t cols, int32_t g_is_f16, float* grad, float* work,
                               void* stream) {
    if (rows <= 0 || cols <= 0) return rl_set_error("rl_colsum_accum: rows and cols must be positive");
    if (!g || !grad || !work) return rl_set_error("rl_colsum_accum: null pointer");
    if (cols % kColVec != 0 || cols / kColVec > kBlock || ((uintptr_t)g % 16) != 0)
        return rl_set_error("rl_colsum_accum: cols must be a multiple of 8 and <= 2048, g 16-byte aligned");
    // ~64 rows per partial: enough workgroups to cover the CUs, few enough partials for the finish
    int parts = (rows + 63) / 64;
    parts = parts < 1 ? 1 : (parts > kMaxParts ? kMaxParts : parts);
    hipStream_t st = (hipStream_t)stream;
    if (g_is_f16)
        hipLaunchKernelGGL(k_colsum_part<true>, dim3(parts), dim3(kBlock), 0, st, g, (int)rows, (int)cols, work);
    else
        hipLaunchKernelGGL(k_colsum_part<false>, dim3(parts), dim3(kBlock), 0, st, g, (int)rows, (int)cols, work);
    hipLaunchKernelGGL(k_colsum_fin, dim3((cols + kColVec - 1) / kColVec), dim3(kBlock), 0, st, work, parts, (int)cols,
                       grad);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_colsum_accum: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}
