// libgymrl.so -- the PPO minibatch loss and its gradient in one pass (include/gymrl.h).
//
// rl_games a2c_continuous.py calc_gradients (v1.6.x) after the network forward, restated for the
// continuous_a2c_logstd model with fixed sigma (AnymalTerrainPPO.yaml):
//   sigma = exp(logstd); neglogp = 0.5 sum_a ((x - mu) / sigma)^2 + 0.5 log(2 pi) A + sum_a logstd
//   ratio = exp(old_neglogp - neglogp); a = max(-adv ratio, -adv clamp(ratio, 1 - e, 1 + e))   (actor_loss)
//   c = max((v - R)^2, (old_v + clamp(v - old_v, -e, e) - R)^2)  [clip_value] else (R - v)^2     (critic_loss)
//   entropy = sum_a (0.5 + 0.5 log(2 pi) + log sigma)
//   b = sum_a clamp_max(mu + 1.1, 0)^2 + clamp_min(mu - 1.1, 0)^2   (bound_loss; mu +- 1.1 rounded to fp16
//       as torch's fp16 add does under autocast)
//   loss = mean(a) + 0.5 mean(c) critic_coef - mean(entropy) entropy_coef + mean(b) bounds_loss_coef
// and, in the same pass, d loss / d mu, d loss / d v, d loss / d logstd with PyTorch's autograd rules
// (maximum: ties split the gradient; clamp: passes it inside [lo, hi] inclusive).  The torch statement
// of the same loss is ~80 launches forward + backward per minibatch; this is three (rows, finish,
// and the backward's scale by the upstream gradient = the GradScaler scale).
//
// k_ppo_rows: one lane per row; per-workgroup partial sums of the four terms and of d/d logstd folded
// in a fixed LDS tree -> part[block][4 + A]; k_ppo_finish: one workgroup adds the partials in block
// order (deterministic; torch's reductions use another order: the loss agrees to fp32 rounding).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kRows = 128;  // 128 workgroups for a 16384-row minibatch
constexpr int kMaxA = 32;
constexpr int kNT = 4 + kMaxA;  // partial slots per block: a, c, entropy, b, dlogstd[A]

template <class T>
__device__ __forceinline__ float ld(const T* p, size_t i) {
    if constexpr (sizeof(T) == 2) return __half2float(reinterpret_cast<const __half*>(p)[i]);
    else return reinterpret_cast<const float*>(p)[i];
}

// d max(p, q) / d (p, q) as PyTorch's maximum backward: the larger side, ties half each
__device__ __forceinline__ void max_grad(float p, float q, float& wp, float& wq) {
    wp = p > q ? 1.f : (p < q ? 0.f : 0.5f);
    wq = 1.f - wp;
}

template <class TM, class TV>
__global__ __launch_bounds__(kRows) void k_ppo_rows(const TM* __restrict__ mu, const TV* __restrict__ values,
                                                    const float* __restrict__ logstd, const float* __restrict__ act,
                                                    const float* __restrict__ old_nlp, const float* __restrict__ adv,
                                                    const float* __restrict__ old_v, const float* __restrict__ ret,
                                                    int B, int A, float e, int clip_value, float cc, float ec,
                                                    float bc, float* __restrict__ dmu, float* __restrict__ dv,
                                                    float* __restrict__ part) {
    __shared__ float red[kNT][kRows];
    const int t = threadIdx.x;
    const int i = blockIdx.x * kRows + t;
    const float invB = 1.f / (float)B;
    const float half_log2pi = 0.5f * logf(2.f * 3.14159265358979323846f);
    float ta = 0.f, tc = 0.f, te = 0.f, tb = 0.f;
    // this row's d/d logstd goes straight to its LDS column (no runtime-indexed register array)
    for (int a = 0; a < kMaxA; ++a) red[4 + a][t] = 0.f;
    if (i < B) {
        // neglogp, entropy, bound loss
        float sq = 0.f, sls = 0.f, ent = 0.f, bl = 0.f;
        for (int a = 0; a < A; ++a) {
            const float m = ld(mu, (size_t)i * A + a);
            const float ls = logstd[a];
            const float sg = expf(ls);
            const float z = (act[(size_t)i * A + a] - m) / sg;
            sq += z * z;
            sls += ls;
            ent += 0.5f + half_log2pi + logf(sg);
            const float t1 = fminf(__half2float(__float2half(m + 1.1f)), 0.f);
            const float t2 = fmaxf(__half2float(__float2half(m - 1.1f)), 0.f);
            bl += t1 * t1 + t2 * t2;
        }
        const float nlp = 0.5f * sq + half_log2pi * (float)A + sls;
        const float r = expf(old_nlp[i] - nlp);
        const float ad = adv[i];
        const float rc = fminf(fmaxf(r, 1.f - e), 1.f + e);
        const float p = -(ad * r), q = -(ad * rc);
        const float av = fmaxf(p, q);
        // critic
        const float v = ld(values, i), ov = old_v[i], R = ret[i];
        float cv, dcdv;
        if (clip_value) {
            const float dvo = v - ov;
            const float vpc = ov + fminf(fmaxf(dvo, -e), e);
            const float q1 = (v - R) * (v - R), q2 = (vpc - R) * (vpc - R);
            cv = fmaxf(q1, q2);
            float w1, w2;
            max_grad(q1, q2, w1, w2);
            const float in = (dvo >= -e && dvo <= e) ? 1.f : 0.f;
            dcdv = w1 * 2.f * (v - R) + w2 * 2.f * (vpc - R) * in;
        } else {
            cv = (R - v) * (R - v);
            dcdv = 2.f * (v - R);
        }
        ta = av; tc = cv; te = ent; tb = bl;
        // gradients of the mean loss
        float wp, wq;
        max_grad(p, q, wp, wq);
        const float in_r = (r >= 1.f - e && r <= 1.f + e) ? 1.f : 0.f;
        const float dratio = invB * (wp * -ad + wq * -ad * in_r);
        const float dnlp = -r * dratio;
        for (int a = 0; a < A; ++a) {
            const float m = ld(mu, (size_t)i * A + a);
            const float sg = expf(logstd[a]);
            const float z = (act[(size_t)i * A + a] - m) / sg;
            const float h1 = __half2float(__float2half(m + 1.1f)), h2 = __half2float(__float2half(m - 1.1f));
            const float db = (h1 <= 0.f ? 2.f * fminf(h1, 0.f) : 0.f) + (h2 >= 0.f ? 2.f * fmaxf(h2, 0.f) : 0.f);
            dmu[(size_t)i * A + a] = dnlp * (-z / sg) + bc * invB * db;
            red[4 + a][t] = dnlp * (1.f - z * z) - ec * invB;
        }
        dv[i] = 0.5f * cc * invB * dcdv;
    }
    red[0][t] = ta;
    red[1][t] = tc;
    red[2][t] = te;
    red[3][t] = tb;
    __syncthreads();
    for (int s = kRows / 2; s > 0; s >>= 1) {
        if (t < s)
            for (int k = 0; k < 4 + A; ++k) red[k][t] += red[k][t + s];
        __syncthreads();
    }
    if (t < 4 + A) part[(size_t)blockIdx.x * kNT + t] = red[t][0];
}

__global__ __launch_bounds__(64) void k_ppo_finish(const float* __restrict__ part, int blocks, int A, float invB,
                                                   float cc, float ec, float bc, float* __restrict__ loss,
                                                   float* __restrict__ stats, float* __restrict__ dls) {
    __shared__ float m[4];
    const int t = threadIdx.x;
    if (t < 4 + A) {
        // 8 independent partial chains (b mod 8, combined pairwise): the loads issue together instead of
        // one L2 round trip per block; a fixed order, so the sums stay run-to-run identical
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int b = 0;
        for (; b + 8 <= blocks; b += 8) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += part[(size_t)(b + k) * kNT + t];
        }
        for (; b < blocks; ++b) acc[0] += part[(size_t)b * kNT + t];
        const float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        if (t < 4) {
            m[t] = s * invB;
            stats[t] = m[t];
        } else {
            dls[t - 4] = s;
        }
    }
    __syncthreads();
    if (t == 0) *loss = m[0] + 0.5f * m[1] * cc - m[2] * ec + m[3] * bc;
}

template <class T>
__device__ __forceinline__ void st(T* p, size_t i, float v) {
    if constexpr (sizeof(T) == 2) reinterpret_cast<__half*>(p)[i] = __float2half(v);
    else reinterpret_cast<float*>(p)[i] = v;
}

template <class TM, class TV>
__global__ __launch_bounds__(256) void k_ppo_scale(const float* __restrict__ g, const float* __restrict__ dmu,
                                                   const float* __restrict__ dv, const float* __restrict__ dls,
                                                   int B, int A, TM* __restrict__ dmu_out, TV* __restrict__ dv_out,
                                                   float* __restrict__ dls_out) {
    const float s = *g;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (size_t)B * A) st(dmu_out, i, dmu[i] * s);
    if (i < (size_t)B) st(dv_out, i, dv[i] * s);
    if (i < (size_t)A) dls_out[i] = dls[i] * s;
}

int launch_err(const char* where) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    char msg[256];
    snprintf(msg, sizeof(msg), "%s: launch failed: %s", where, hipGetErrorString(e));
    return rl_set_error(msg) + 1;
}

}  // namespace

extern "C" int rl_ppo_loss(const void* mu, int32_t mu_is_f16, const void* values, int32_t values_is_f16,
                           const float* logstd, const float* actions, const float* old_neglogp, const float* advantages,
                           const float* old_values, const float* returns, int32_t rows, int32_t num_actions,
                           double e_clip, int32_t clip_value, double critic_coef, double entropy_coef,
                           double bounds_loss_coef, float* dmu, float* dvalues, float* partials, float* loss,
                           float* stats, float* dlogstd, void* stream) {
    if (rows <= 0 || num_actions <= 0 || num_actions > kMaxA)
        return rl_set_error("rl_ppo_loss: rows must be positive and 0 < num_actions <= 32");
    if (!mu || !values || !logstd || !actions || !old_neglogp || !advantages || !old_values || !returns || !dmu ||
        !dvalues || !partials || !loss || !stats || !dlogstd)
        return rl_set_error("rl_ppo_loss: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const int blocks = (rows + kRows - 1) / kRows;
    const float e = (float)e_clip, cc = (float)critic_coef, ec = (float)entropy_coef, bc = (float)bounds_loss_coef;
#define RL_PPO_ROWS(TM, TV)                                                                                     \
    hipLaunchKernelGGL((k_ppo_rows<TM, TV>), dim3(blocks), dim3(kRows), 0, st, (const TM*)mu, (const TV*)values, \
                       logstd, actions, old_neglogp, advantages, old_values, returns, (int)rows, (int)num_actions, e, \
                       (int)clip_value, cc, ec, bc, dmu, dvalues, partials)
    if (mu_is_f16 && values_is_f16) RL_PPO_ROWS(__half, __half);
    else if (mu_is_f16) RL_PPO_ROWS(__half, float);
    else if (values_is_f16) RL_PPO_ROWS(float, __half);
    else RL_PPO_ROWS(float, float);
#undef RL_PPO_ROWS
    if (int rc = launch_err("rl_ppo_loss")) return rc;
    hipLaunchKernelGGL(k_ppo_finish, dim3(1), dim3(64), 0, st, partials, blocks, (int)num_actions, 1.f / (float)rows,
                       cc, ec, bc, loss, stats, dlogstd);
    return launch_err("rl_ppo_loss finish");
}

extern "C" int rl_ppo_loss_backward(const float* grad_loss, const float* dmu, const float* dvalues,
                                    const float* dlogstd, int32_t rows, int32_t num_actions, void* dmu_out,
                                    int32_t dmu_is_f16, void* dvalues_out, int32_t dvalues_is_f16,
                                    float* dlogstd_out, void* stream) {
    if (rows <= 0 || num_actions <= 0 || num_actions > kMaxA)
        return rl_set_error("rl_ppo_loss_backward: rows must be positive and 0 < num_actions <= 32");
    if (!grad_loss || !dmu || !dvalues || !dlogstd || !dmu_out || !dvalues_out || !dlogstd_out)
        return rl_set_error("rl_ppo_loss_backward: null pointer");
    size_t n = (size_t)rows * num_actions;
    if (n < (size_t)rows) n = rows;
    const dim3 grid((unsigned)((n + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
#define RL_PPO_SCALE(TM, TV)                                                                                      \
    hipLaunchKernelGGL((k_ppo_scale<TM, TV>), grid, dim3(256), 0, st, grad_loss, dmu, dvalues, dlogstd, (int)rows, \
                       (int)num_actions, (TM*)dmu_out, (TV*)dvalues_out, dlogstd_out)
    if (dmu_is_f16 && dvalues_is_f16) RL_PPO_SCALE(__half, __half);
    else if (dmu_is_f16) RL_PPO_SCALE(__half, float);
    else if (dvalues_is_f16) RL_PPO_SCALE(float, __half);
    else RL_PPO_SCALE(float, float);
#undef RL_PPO_SCALE
    return launch_err("rl_ppo_loss_backward");
}
