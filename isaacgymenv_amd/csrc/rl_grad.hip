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
template <bool HALF>
__global__ __launch_bounds__(kBlock) void k_splitk_accum(const void* __restrict__ parts, int P, int64_t n,
                                                         float* __restrict__ grad, bool vec) {
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kVec;
    if (i0 >= n) return;
    float acc[kVec] = {0.f, 0.f, 0.f, 0.f};
    if (vec) {
        for (int p = 0; p < P; ++p) {
            if constexpr (HALF) {
                const __half2* src = reinterpret_cast<const __half2*>(static_cast<const __half*>(parts) + p * n + i0);
                const float2 a = __half22float2(src[0]), b = __half22float2(src[1]);
                acc[0] += a.x; acc[1] += a.y; acc[2] += b.x; acc[3] += b.y;
            } else {
                const float4 v = *reinterpret_cast<const float4*>(static_cast<const float*>(parts) + p * n + i0);
                acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
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

}  // namespace

extern "C" int rl_splitk_accum(const void* parts, int32_t num_parts, int64_t n, int32_t parts_are_f16, float* grad,
                               void* stream) {
    if (num_parts <= 0 || n < 0) return rl_set_error("rl_splitk_accum: num_parts must be positive, n >= 0");
    if (n == 0) return 0;
    if (!parts || !grad) return rl_set_error("rl_splitk_accum: null pointer");
    const uintptr_t align = parts_are_f16 ? 8 : 16;
    const bool vec = (n % kVec) == 0 && ((uintptr_t)parts % align) == 0 && ((uintptr_t)grad % 16) == 0;
    const int64_t lanes = (n + kVec - 1) / kVec;
    const dim3 grid((unsigned)((lanes + kBlock - 1) / kBlock));
    if (parts_are_f16)
        hipLaunchKernelGGL(k_splitk_accum<true>, grid, dim3(kBlock), 0, (hipStream_t)stream, parts, (int)num_parts, n,
                           grad, vec);
    else
        hipLaunchKernelGGL(k_splitk_accum<false>, grid, dim3(kBlock), 0, (hipStream_t)stream, parts, (int)num_parts,
                           n, grad, vec);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_splitk_accum: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}
