// torch_philox.h -- torch.rand's float32 stream on ROCm, evaluated per element.
//
// The task layer must draw exactly the numbers the reference draws (bit-exact resets and
// observation noise), and the reference draws them with torch.rand / torch.rand_like on the
// CUDA/HIP generator.  Rather than launching torch's generator kernel and reading its output
// back from HBM, the fused tail kernels evaluate the same stream in registers:
//
//   torch (ATen/native/cuda/DistributionTemplates.h, uniform_and_transform + calc_execution_policy):
//     grid  = min(CUs * (maxThreadsPerCU / 256), ceil(n / 256)),  T = 256 * grid threads
//     thread `idx` runs Philox4x32-10 (rocRAND) with key = seed, subsequence = idx and the
//     generator offset; each curand_uniform4 call yields 4 floats; element
//       i = it * 4T + ii * T + idx   takes component ii of call number `it` of thread idx
//     offset increment of the call = ((n - 1) / (4T) + 1) * 4
//   rocRAND philox4x32_10 (rocrand_philox4x32_10.h): counter = {c_lo, c_hi, idx_lo, idx_hi} with
//     c = offset / 4 + it (offset is a multiple of 4 -> substate 0), 10 rounds with key bumps.
//   rocrand_uniform4: u = 2^-32 + float(v) * 2^-32 in (0, 1]; torch maps u == 1 to 0.
//
// The host side (isaacgymenv_amd/gymtask.py: TorchRandPlan) reads the generator's seed and
// offset, computes T and the increment, and advances the generator exactly as torch would.
// tests/test_philox_gpu.py checks this against torch.rand bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gymtask.h"

namespace torch_philox {

__device__ __forceinline__ uint4 philox_round(uint4 c, uint32_t k0, uint32_t k1) {
  const uint64_t m0 = (uint64_t)0xD2511F53u * c.x;
  const uint64_t m1 = (uint64_t)0xCD9E8D57u * c.z;
  return uint4{(uint32_t)(m1 >> 32) ^ c.y ^ k0, (uint32_t)m1, (uint32_t)(m0 >> 32) ^ c.w ^ k1, (uint32_t)m0};
}

__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    c = philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return philox_round(c, k0, k1);
}

// element i of torch.rand(n) drawn from plan d (d.numel == n)
#ifndef GT_PHILOX_WIDE
#define GT_PHILOX_WIDE 0  // 1: always the 64-bit index math (A/B builds)
#endif

__device__ __forceinline__ float rand_at(const gt_torch_rand_plan& d, uint64_t i) {
  const uint64_t T = d.threads;
  uint64_t it, idx;
  uint32_t ii;
  if (!GT_PHILOX_WIDE && (i >> 32) == 0 && (T >> 30) == 0) {
    // the same integer quotients in 32 bits (a 64-bit division is a long software sequence on the GPU; the
    // observation draws of a 4096-env step are ~770 k elements)
    const uint32_t i32 = (uint32_t)i, T32 = (uint32_t)T;
    const uint32_t it32 = i32 / (4u * T32);
    const uint32_t r = i32 - it32 * (4u * T32);
    ii = r / T32;
    it = it32;
    idx = r - ii * T32;
  } else {
    it = i / (4 * T);
    const uint64_t r = i - it * 4 * T;
    ii = (uint32_t)(r / T);
    idx = r - (uint64_t)ii * T;
  }
  const uint64_t ctr = d.offset / 4 + it;
  const uint4 v = philox10(uint4{(uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)idx, (uint32_t)(idx >> 32)},
                           (uint32_t)d.seed, (uint32_t)(d.seed >> 32));
  const uint32_t w = ii == 0 ? v.x : ii == 1 ? v.y : ii == 2 ? v.z : v.w;
  const float u = 2.3283064365386963e-10f + (float)w * 2.3283064365386963e-10f;
  return u == 1.0f ? 0.0f : u;
}

}  // namespace torch_philox
