// libgymrl.so -- PPO learner kernels (include/gymrl.h).
//
// rl_gae: rl_games A2CBase.discount_values (a2c_common.py, rl-games 1.6.x; the reference
// pins only rl-games>=1.6.0, setup.py:22) + returns = advs + values + swap_and_flatten01.
//
// One lane per env, one wave (64 envs) per workgroup.  Pass 1 walks the horizon backwards
// reading the time-major rollout rows (each wave load = 256 contiguous bytes) and keeps the
// advantages in an LDS tile [64][H+1] (padded row: lane r writes column t of row r, the 64
// writes of one t land in distinct banks).  Pass 2 streams the tile out env-major: the 64
// envs of the workgroup own the contiguous range [n0*H, (n0+64)*H) of every output, so the
// stores are fully coalesced.  Memory-bound: 4 reads (r, v, done, + v again from L2) and up
// to 3 writes per sample.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "gymrl.h"

namespace {

thread_local char g_err[512];

int fail(const char *msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return 1;
}

constexpr int kWave = 64;
constexpr int kMaxHorizon = 240;  // LDS tile 64 x (H+1) floats <= 61.9 KB

__global__ __launch_bounds__(kWave) void k_gae(const float *__restrict__ rewards, const float *__restrict__ values,
                                               const uint8_t *__restrict__ dones,
                                               const float *__restrict__ last_values,
                                               const uint8_t *__restrict__ last_dones, int H, int N, float gamma,
                                               float gt, float *__restrict__ returns_out,
                                               float *__restrict__ advs_out, float *__restrict__ values_out) {
    extern __shared__ float tile[];  // [64][H+1]
    const int r = threadIdx.x;
    const int n0 = blockIdx.x * kWave;
    const int n = n0 + r;
    const int ld = H + 1;
    if (n < N) {
        float nv = last_values[n];
        float nn = 1.0f - (float)last_dones[n];
        float adv = 0.0f;
        for (int t = H - 1; t >= 0; --t) {
            const size_t i = (size_t)t * N + n;
            const float v = values[i];
            // same association as the reference: r + gamma * nv * nn - v ; delta + gamma * tau * nn * adv
            const float delta = rewards[i] + gamma * nv * nn - v;
            adv = delta + gt * nn * adv;
            tile[r * ld + t] = adv;
            nv = v;
            nn = 1.0f - (float)dones[i];
        }
    }
    __syncthreads();
    const int rows = min(kWave, N - n0);
    const size_t base = (size_t)n0 * H;
    for (int k = r; k < rows * H; k += kWave) {
        const int rr = k / H, t = k - rr * H;
        const float a = tile[rr * ld + t];
        const float v = values[(size_t)t * N + n0 + rr];
        returns_out[base + k] = a + v;
        if (advs_out) advs_out[base + k] = a;
        if (values_out) values_out[base + k] = v;
    }
}

}  // namespace

int rl_set_error(const char *msg) { return fail(msg); }

extern "C" {

int rl_abi_version(void) { return RL_ABI_VERSION; }

const char *rl_last_error(void) { return g_err; }

int rl_gae(const float *rewards, const float *values, const uint8_t *dones, const float *last_values,
           const uint8_t *last_dones, int32_t horizon, int32_t num_envs, double gamma, double tau,
           float *returns_out, float *advs_out, float *values_out, void *stream) {
    if (horizon <= 0 || num_envs <= 0) return fail("rl_gae: horizon and num_envs must be positive");
    if (horizon > kMaxHorizon) return fail("rl_gae: horizon exceeds 240 (LDS tile bound)");
    if (!rewards || !values || !dones || !last_values || !last_dones || !returns_out)
        return fail("rl_gae: null required pointer");
    const int blocks = (num_envs + kWave - 1) / kWave;
    const size_t lds = (size_t)kWave * (horizon + 1) * sizeof(float);
    hipLaunchKernelGGL(k_gae, dim3(blocks), dim3(kWave), lds, (hipStream_t)stream, rewards, values, dones,
                       last_values, last_dones, horizon, num_envs, (float)gamma, (float)(gamma * tau), returns_out, advs_out, values_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "rl_gae: launch failed: %s", hipGetErrorString(e));
        return 2;
    }
    return 0;
}

}  // extern "C"
