// libgymrl.so -- rollout bookkeeping after each VecTask.step of the PPO learner (include/gymrl.h).
//
// rl_games a2c_common.py play_steps (v1.6.x), the statements after `self.env_step(actions)`:
//   shaped_rewards = rewards_shaper(rewards) [+ gamma * values * time_outs  (value_bootstrap)]
//   experience rewards[n] = shaped; current_rewards += rewards; current_lengths += 1
//   game_rewards / game_lengths .update(current_* of the envs done this step)  (torch_ext.AverageMeter)
//   current_* *= 1 - dones
// as ONE workgroup (1024 lanes, 4096 envs = 4 per lane): the elementwise part is the same fp32
// arithmetic torch's kernels do (built with -ffp-contract=off); the meters' masked sums are reduced
// per lane in env order, then across the workgroup in a fixed LDS tree (deterministic, but not torch's
// reduction order: the meters agree with the torch path to fp32 rounding).  Replaces ~20 torch launches
// (~0.14 ms replayed as a HIP graph at 4096 envs) and the three static-buffer copies in front of them.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kLanes = 1024;

__device__ __forceinline__ bool flag(const void* p, int bytes, int i) {
    return bytes == 8 ? static_cast<const int64_t*>(p)[i] != 0 : static_cast<const uint8_t*>(p)[i] != 0;
}

// AverageMeter.update with the masked sums (rl/a2c_continuous.py _AverageMeter.update_masked)
__device__ void meter_update(float* m, float cnt, float vsum, float max_size) {
    if (!(cnt > 0.f)) return;
    const float new_mean = vsum / fmaxf(cnt, 1.f);
    const float size = fminf(cnt, max_size);
    const float old_size = fminf(max_size - size, m[1]);
    const float size_sum = old_size + size;
    m[0] = (m[0] * old_size + new_mean * size) / fmaxf(size_sum, 1.f);
    m[1] = size_sum;
}

__global__ __launch_bounds__(kLanes) void k_rollout_post(
    const float* __restrict__ rew, const void* __restrict__ dones_in, int dones_bytes,
    const void* __restrict__ timeouts, int timeouts_bytes, const float* __restrict__ values, float shift, float scale,
    float gamma, int N, uint8_t* __restrict__ dones_out, float* __restrict__ t_rewards, float* __restrict__ cur_rew,
    float* __restrict__ cur_len, float* __restrict__ meter_rew, float* __restrict__ meter_len, float max_size) {
    __shared__ float red[3][kLanes];
    const int t = threadIdx.x;
    float cnt = 0.f, srew = 0.f, slen = 0.f;
    for (int i = t; i < N; i += kLanes) {
        const float r = rew[i];
        const bool d = flag(dones_in, dones_bytes, i);
        dones_out[i] = d ? 1 : 0;
        float shaped = (r + shift) * scale;
        if (values && timeouts) {
            const float to = flag(timeouts, timeouts_bytes, i) ? 1.f : 0.f;
            shaped = shaped + gamma * values[i] * to;
        }
        t_rewards[i] = shaped;
        const float cr = cur_rew[i] + r;
        const float cl = cur_len[i] + 1.f;
        if (d) {
            cnt += 1.f;
            srew += cr;
            slen += cl;
        }
        const float nd = 1.f - (d ? 1.f : 0.f);
        cur_rew[i] = cr * nd;
        cur_len[i] = cl * nd;
    }
    red[0][t] = cnt;
    red[1][t] = srew;
    red[2][t] = slen;
    __syncthreads();
    for (int s = kLanes / 2; s > 0; s >>= 1) {
        if (t < s) {
            red[0][t] += red[0][t + s];
            red[1][t] += red[1][t + s];
            red[2][t] += red[2][t + s];
        }
        __syncthreads();
    }
    if (t == 0) {
        meter_update(meter_rew, red[0][0], red[1][0], max_size);
        meter_update(meter_len, red[0][0], red[2][0], max_size);
    }
}

}  // namespace

extern "C" int rl_rollout_post(const float* rewards, const void* dones, int32_t dones_bytes, const void* time_outs,
                               int32_t time_outs_bytes, const float* values, double reward_shift, double reward_scale,
                               double gamma, int32_t num_envs, uint8_t* dones_out, float* rewards_out,
                               float* current_rewards, float* current_lengths, float* meter_rewards,
                               float* meter_lengths, int32_t games_to_track, void* stream) {
    if (num_envs <= 0) return rl_set_error("rl_rollout_post: num_envs must be positive");
    if (!rewards || !dones || !dones_out || !rewards_out || !current_rewards || !current_lengths || !meter_rewards ||
        !meter_lengths)
        return rl_set_error("rl_rollout_post: null required pointer");
    if ((dones_bytes != 1 && dones_bytes != 8) || (time_outs && time_outs_bytes != 1 && time_outs_bytes != 8))
        return rl_set_error("rl_rollout_post: flags must be 1-byte (bool / uint8) or 8-byte (int64) elements");
    hipLaunchKernelGGL(k_rollout_post, dim3(1), dim3(kLanes), 0, (hipStream_t)stream, rewards, dones, (int)dones_bytes,
                       time_outs, (int)time_outs_bytes, values, (float)reward_shift, (float)reward_scale,
                       (float)gamma, (int)num_envs, dones_out, rewards_out, current_rewards, current_lengths,
                       meter_rewards, meter_lengths, (float)games_to_track);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_rollout_post: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}

// ---------------------------------------------------------------- experience slot (before env.step)
// play_steps' update_data calls of horizon slot n (rl_games a2c_common.py: obses, dones, values,
// actions, neglogpacs, mus, sigmas), one launch instead of seven strided copies: 64 lanes per env,
// four envs per workgroup; plain copies, bit-identical to the torch statements.
namespace {

__global__ __launch_bounds__(256) void k_rollout_pre(const float* __restrict__ obs, int O, const uint8_t* __restrict__ dones,
                                                     const float* __restrict__ values, int vstride,
                                                     const float* __restrict__ actions, const float* __restrict__ neglogp,
                                                     const float* __restrict__ mu, const float* __restrict__ sigma, int N,
                                                     int A, int H, int n, float* __restrict__ b_obs,
                                                     uint8_t* __restrict__ t_dones, float* __restrict__ t_values,
                                                     float* __restrict__ b_actions, float* __restrict__ b_neglogp,
                                                     float* __restrict__ b_mu, float* __restrict__ b_sigma) {
    const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int l = threadIdx.x & 63;
    if (e >= N) return;
    const float* src = obs + (size_t)e * O;
    float* dst = b_obs + ((size_t)e * H + n) * O;
    for (int k = l; k < O; k += 64) dst[k] = src[k];
    const size_t ra = (size_t)e * A, wa = ((size_t)e * H + n) * A;
    if (l < A) {
        b_actions[wa + l] = actions[ra + l];
        b_mu[wa + l] = mu[ra + l];
        b_sigma[wa + l] = sigma[ra + l];
    }
    if (l == 0) {
        t_dones[(size_t)n * N + e] = dones[e];
        t_values[(size_t)n * N + e] = values[(size_t)e * vstride];
        b_neglogp[(size_t)e * H + n] = neglogp[e];
    }
}

}  // namespace

extern "C" int rl_rollout_pre(const float* obs, int32_t obs_dim, const uint8_t* dones, const float* values,
                              int32_t values_stride, const float* actions, const float* neglogp, const float* mu,
                              const float* sigma, int32_t num_envs, int32_t num_actions, int32_t horizon, int32_t slot,
                              float* b_obs, uint8_t* t_dones, float* t_values, float* b_actions, float* b_neglogp,
                              float* b_mu, float* b_sigma, void* stream) {
    if (num_envs <= 0 || obs_dim <= 0 || num_actions <= 0 || num_actions > 64 || horizon <= 0 || slot < 0 ||
        slot >= horizon || values_stride <= 0)
        return rl_set_error("rl_rollout_pre: bad sizes (num_actions <= 64, 0 <= slot < horizon)");
    if (!obs || !dones || !values || !actions || !neglogp || !mu || !sigma || !b_obs || !t_dones || !t_values ||
        !b_actions || !b_neglogp || !b_mu || !b_sigma)
        return rl_set_error("rl_rollout_pre: null pointer");
    hipLaunchKernelGGL(k_rollout_pre, dim3((num_envs + 3) / 4), dim3(256), 0, (hipStream_t)stream, obs, (int)obs_dim,
                       dones, values, (int)values_stride, actions, neglogp, mu, sigma, (int)num_envs, (int)num_actions,
                       (int)horizon, (int)slot, b_obs, t_dones, t_values, b_actions, b_neglogp, b_mu, b_sigma);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_rollout_pre: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}

// ---------------------------------------------------------------- act forward head
// models.ModelA2CContinuousLogStd eval forward after the network (fixed sigma), rl/network.py:
//   sigma = exp(logstd); action = normal(0, 1) * sigma + mu  (the standard normals drawn by torch's
//   normal_, so the RNG stream is torch's); neglogp(action); value = RunningMeanStd unnorm (clamp to
//   [-5, 5], * sqrt(float(var) + eps) + float(mean)).  One lane per env; replaces ~14 launches.
namespace {

__global__ __launch_bounds__(256) void k_policy_head(const float* __restrict__ mu, const float* __restrict__ noise,
                                                     const float* __restrict__ logstd, const float* __restrict__ value,
                                                     const double* __restrict__ vmean, const double* __restrict__ vvar,
                                                     float veps, int N, int A, float nlp_const,
                                                     float* __restrict__ actions, float* __restrict__ sigmas,
                                                     float* __restrict__ neglogp, float* __restrict__ value_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float sq = 0.f, sls = 0.f;
    for (int a = 0; a < A; ++a) {
        const size_t k = (size_t)i * A + a;
        const float ls = logstd[a];
        const float s = expf(ls);
        const float m = mu[k];
        const float t = noise[k] * s;
        const float x = t + m;
        actions[k] = x;
        sigmas[k] = s;
        const float z = (x - m) / s;
        sq += z * z;
        sls += ls;
    }
    neglogp[i] = 0.5f * sq + nlp_const + sls;
    float v = value[i];
    if (vmean) {
        v = fminf(fmaxf(v, -5.f), 5.f);
        v = sqrtf((float)vvar[0] + veps) * v + (float)vmean[0];
    }
    value_out[i] = v;
}

}  // namespace

extern "C" int rl_policy_head(const float* mu, const float* noise, const float* logstd, const float* value,
                              const double* value_mean, const double* value_var, double value_eps, int32_t num_envs,
                              int32_t num_actions, float* actions, float* sigmas, float* neglogp, float* value_out,
                              void* stream) {
    if (num_envs <= 0 || num_actions <= 0) return rl_set_error("rl_policy_head: num_envs, num_actions must be positive");
    if (!mu || !noise || !logstd || !value || !actions || !sigmas || !neglogp || !value_out ||
        (!value_mean) != (!value_var))
        return rl_set_error("rl_policy_head: null pointer");
    const double c = 0.5 * 1.8378770664093453 * num_actions;  // 0.5 * math.log(2 pi) * A, as Python computes it
    hipLaunchKernelGGL(k_policy_head, dim3((num_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream, mu, noise, logstd,
                       value, value_mean, value_var, (float)value_eps, (int)num_envs, (int)num_actions, (float)c,
                       actions, sigmas, neglogp, value_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_policy_head: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}

// ---------------------------------------------------------------- act forward heads + head (ABI 7)
// The two Linear heads on the MLP outputs (mu = a W_mu^T + b_mu, value = c w_v^T + b_v; network.py
// ActorCriticNetwork.forward) and then rl_policy_head's statements, in one launch: 16 rows per
// workgroup, their hidden rows and the head weights staged in LDS (row strides padded by one float so
// the lanes of a dot product fall on different banks), one lane per (row, output) dot product as a
// f32 FMA chains over H, four interleaved (k mod 4) and added pairwise (the library GEMM's order differs:
// within f32 rounding of it).
namespace {

constexpr int kHeadRows = 16;

__global__ __launch_bounds__(256) void k_act_heads(const float* __restrict__ ha, int lda, const float* __restrict__ hc,
                                                   int ldc, int H, const float* __restrict__ w_mu,
                                                   const float* __restrict__ b_mu, const float* __restrict__ w_v,
                                                   const float* __restrict__ b_v, const float* __restrict__ noise,
                                                   const float* __restrict__ logstd, const double* __restrict__ vmean,
                                                   const double* __restrict__ vvar, float veps, int N, int A,
                                                   float nlp_const, float* __restrict__ mu_out,
                                                   float* __restrict__ actions, float* __restrict__ sigmas,
                                                   float* __restrict__ neglogp, float* __restrict__ value_out) {
    extern __shared__ float sm[];
    const int SH = 2 * H + 1, SW = H + 1, O = A + 1;
    float* sh = sm;                     // [kHeadRows][SH]: actor hidden | critic hidden
    float* sw = sh + kHeadRows * SH;    // [O][SW]: the A mu rows, then the value row
    float* so = sw + O * SW;            // [kHeadRows][O]: mu | value
    const int r0 = blockIdx.x * kHeadRows;
    const int nr = min(kHeadRows, N - r0);
    for (int i = threadIdx.x; i < nr * 2 * H; i += blockDim.x) {
        const int r = i / (2 * H), k = i - r * 2 * H;
        sh[r * SH + k] = k < H ? ha[(size_t)(r0 + r) * lda + k] : hc[(size_t)(r0 + r) * ldc + (k - H)];
    }
    for (int i = threadIdx.x; i < O * H; i += blockDim.x) {
        const int o = i / H, k = i - o * H;
        sw[o * SW + k] = o < A ? w_mu[(size_t)o * H + k] : w_v[k];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nr * O; t += blockDim.x) {
        const int r = t / O, o = t - r * O;
        const float* h = sh + r * SH + (o < A ? 0 : H);
        const float* w = sw + o * SW;
        // four interleaved FMA chains (k mod 4), added pairwise: a quarter of the dependent latency
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        int k = 0;
        for (; k + 4 <= H; k += 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = fmaf(h[k + q], w[k + q], acc[q]);
        }
        for (; k < H; ++k) acc[k & 3] = fmaf(h[k], w[k], acc[k & 3]);
        so[r * O + o] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + (o < A ? b_mu[o] : b_v[0]);
    }
    __syncthreads();
    if ((int)threadIdx.x < nr) {
        const int r = threadIdx.x, i = r0 + r;
        float sq = 0.f, sls = 0.f;
        for (int a = 0; a < A; ++a) {  // rl_policy_head's statements, in its order
            const size_t k = (size_t)i * A + a;
            const float ls = logstd[a];
            const float sg = expf(ls);
            const float m = so[r * O + a];
            const float x = noise[k] * sg + m;
            mu_out[k] = m;
            actions[k] = x;
            sigmas[k] = sg;
            const float z = (x - m) / sg;
            sq += z * z;
            sls += ls;
        }
        neglogp[i] = 0.5f * sq + nlp_const + sls;
        float v = so[r * O + A];
        if (vmean) {
            v = fminf(fmaxf(v, -5.f), 5.f);
            v = sqrtf((float)vvar[0] + veps) * v + (float)vmean[0];
        }
        value_out[i] = v;
    }
}

}  // namespace

extern "C" int rl_act_heads(const float* hidden_actor, int32_t ld_actor, const float* hidden_critic, int32_t ld_critic,
                            int32_t H, const float* w_mu, const float* b_mu, const float* w_v, const float* b_v,
                            const float* noise, const float* logstd, const double* value_mean, const double* value_var,
                            double value_eps, int32_t num_envs, int32_t num_actions, float* mu, float* actions,
                            float* sigmas, float* neglogp, float* value_out, void* stream) {
    if (num_envs <= 0 || num_actions <= 0 || H <= 0 || ld_actor < H || ld_critic < H)
        return rl_set_error("rl_act_heads: bad sizes");
    if (!hidden_actor || !hidden_critic || !w_mu || !b_mu || !w_v || !b_v || !noise || !logstd || !mu || !actions ||
        !sigmas || !neglogp || !value_out || (!value_mean) != (!value_var))
        return rl_set_error("rl_act_heads: null pointer");
    const size_t lds = sizeof(float) * ((size_t)kHeadRows * (2 * H + 1) + (size_t)(num_actions + 1) * (H + 1) +
                                        (size_t)kHeadRows * (num_actions + 1));
    if (lds > 64 * 1024) return rl_set_error("rl_act_heads: H / num_actions too large for the LDS stage");
    const double c = 0.5 * 1.8378770664093453 * num_actions;  // as rl_policy_head
    hipLaunchKernelGGL(k_act_heads, dim3((num_envs + kHeadRows - 1) / kHeadRows), dim3(256), lds, (hipStream_t)stream,
                       hidden_actor, (int)ld_actor, hidden_critic, (int)ld_critic, (int)H, w_mu, b_mu, w_v, b_v, noise,
                       logstd, value_mean, value_var, (float)value_eps, (int)num_envs, (int)num_actions, (float)c, mu,
                       actions, sigmas, neglogp, value_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char msg[256];
        snprintf(msg, sizeof(msg), "rl_act_heads: launch failed: %s", hipGetErrorString(e));
        return rl_set_error(msg) + 1;
    }
    return 0;
}
