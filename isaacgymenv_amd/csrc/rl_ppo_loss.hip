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

__device__ __forceinline__ float sum_partials(const float* __restrict__ part, int blocks, size_t stride, int i,
                                              bool on, float (*sh)[64]);

__global__ __launch_bounds__(256) void k_ppo_finish(const float* __restrict__ part, int blocks, int A, float invB,
                                                    float cc, float ec, float bc, float* __restrict__ loss,
                                                    float* __restrict__ stats, float* __restrict__ dls) {
    // 4 lanes per slot add the blocks' partials (a fixed order, so the sums stay run-to-run identical)
    __shared__ float sh[4][64];
    __shared__ float m[4];
    const int t = threadIdx.x;
    const float s = sum_partials(part, blocks, (size_t)kNT, t & 63, (t & 63) < 4 + A, sh);
    if (t < 4) {
        m[t] = s * invB;
        stats[t] = m[t];
    } else if (t < 4 + A) {
        dls[t - 4] = s;
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

// ---------------------------------------------------------------------------------------------------------------
// The heads and the loss in one pass (rl_ppo_heads_loss / _backward).  After the grouped actor / critic MLPs the
// network has two small heads -- mu = a_out W_mu^T + b_mu [B][A] and value = c_out w_v + b_v [B][1]
// (a2c_continuous network_builder: self.mu, self.value; fp16 under autocast) -- that torch runs as six skinny
// hipBLASLt GEMMs, two column reductions and a concatenation per minibatch.  Here:
//   k_heads_fwd : a DPP quad per row, 16 rows per wave, 64 rows per workgroup: each lane loads its quarter of the
//                 row's actor / critic columns (16-byte loads, all issued before the math), dot products with the
//                 LDS-staged head weights by v_dot2_f32_f16 (fp32 accumulation), a quad butterfly, + bias, rounded
//                 to fp16 as the autocast GEMM's output; then the loss row of k_ppo_rows (same statements) -> mu
//                 (fp16, for the KL and dataset.update_mu_sigma), the unscaled d/d mu, d/d v, one partial per
//                 workgroup (k_ppo_finish)
//   k_heads_bwd : 128 rows per workgroup; the upstream scale applied (d mu, d v rounded to fp16: the torch path's
//                 fp16 head gradients), then one thread per column pair and row group: d a_out = d mu W_mu,
//                 d c_out = d v w_v (fp16, straight into the grouped MLP's [B][G*H] gradient; 16 rows' loads in
//                 flight) and the weight gradient partials, the row groups summed in LDS in a fixed order
//   k_heads_bfin: 4 lanes per output add the workgroup partials (fixed order), into the flat gradient views
constexpr int kHR = 64;    // forward rows per workgroup (4 waves x 16 quads)
constexpr int kHRB = 64;   // backward rows per workgroup

typedef _Float16 hh2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float h2f(__half h) { return __half2float(h); }
__device__ __forceinline__ float rnd_h(float v) { return __half2float(__float2half(v)); }
__device__ __forceinline__ float dot8(uint4 x, uint4 w, float c) {
    c = __builtin_amdgcn_fdot2(__builtin_bit_cast(hh2, x.x), __builtin_bit_cast(hh2, w.x), c, false);
    c = __builtin_amdgcn_fdot2(__builtin_bit_cast(hh2, x.y), __builtin_bit_cast(hh2, w.y), c, false);
    c = __builtin_amdgcn_fdot2(__builtin_bit_cast(hh2, x.z), __builtin_bit_cast(hh2, w.z), c, false);
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(hh2, x.w), __builtin_bit_cast(hh2, w.w), c, false);
}

// AM: the action count padded to the instantiation (guards a < A are uniform); NC: 16-byte chunks per lane (H / 32)
template <int AM, int NC>
__global__ __launch_bounds__(256) void k_heads_fwd(const __half* __restrict__ hid, int ld, int acol, int ccol,
                                                   const __half* __restrict__ wmu, const __half* __restrict__ bmu,
                                                   const __half* __restrict__ wv, const __half* __restrict__ bv,
                                                   const float* __restrict__ logstd, const float* __restrict__ act,
                                                   const float* __restrict__ old_nlp, const float* __restrict__ adv,
                                                   const float* __restrict__ old_v, const float* __restrict__ ret,
                                                   int B, int A, float e, int clip_value, float cc, float ec, float bc,
                                                   __half* __restrict__ mu_out, float* __restrict__ dmu,
                                                   float* __restrict__ dv, float* __restrict__ part) {
    constexpr int H = 32 * NC, K4 = 8 * NC;
    __shared__ uint4 ws[(AM + 1) * H / 8];  // W_mu rows then w_v, fp16
    __shared__ float red[4][kNT];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, q = lane & 3;
    const int row = blockIdx.x * kHR + wave * 16 + (lane >> 2);
    const bool valid = row < B;
    // the row quarter's activations first (independent loads), then the weights into LDS (2-byte loads: the
    // fp16 shadows sit at any even byte offset of the flat buffer)
    uint4 xa[NC], xc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        xa[j] = valid ? *reinterpret_cast<const uint4*>(hid + (size_t)row * ld + acol + q * K4 + 8 * j) : uint4{0, 0, 0, 0};
        xc[j] = valid ? *reinterpret_cast<const uint4*>(hid + (size_t)row * ld + ccol + q * K4 + 8 * j) : uint4{0, 0, 0, 0};
    }
    // the row's loss inputs too, before anything waits on memory
    float xact[AM], lsv[AM];
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        xact[a] = (valid && a < A) ? act[(size_t)row * A + a] : 0.f;
        lsv[a] = a < A ? logstd[a] : 0.f;
    }
    const float r_old_nlp = valid ? old_nlp[row] : 0.f, r_adv = valid ? adv[row] : 0.f;
    const float r_old_v = valid ? old_v[row] : 0.f, r_ret = valid ? ret[row] : 0.f;
    float bmu_f[AM];
#pragma unroll
    for (int a = 0; a < AM; ++a) bmu_f[a] = a < A ? h2f(bmu[a]) : 0.f;
    const float bv_f = h2f(bv[0]);
    __half* wsh = reinterpret_cast<__half*>(ws);
    constexpr int WN = (AM + 1) * H, WI = (WN + 255) / 256;
    __half wtmp[WI];
#pragma unroll
    for (int u = 0; u < WI; ++u) {
        const int i = t + 256 * u, a = i / H, k = i - a * H;
        wtmp[u] = i < WN ? (a < A ? wmu[(size_t)a * H + k] : (a == AM ? wv[k] : __float2half(0.f))) : __float2half(0.f);
    }
#pragma unroll
    for (int u = 0; u < WI; ++u)
        if (t + 256 * u < WN) wsh[t + 256 * u] = wtmp[u];
    __syncthreads();
    float m[AM];
    float vacc = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        m[a] = 0.f;
        if (a < A) {
#pragma unroll
            for (int j = 0; j < NC; ++j) m[a] = dot8(xa[j], ws[(a * H + q * K4) / 8 + j], m[a]);
        }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) vacc = dot8(xc[j], ws[(AM * H + q * K4) / 8 + j], vacc);
    // quad butterfly: every lane of the quad holds the same sums
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        if (a < A) {
            m[a] += __shfl_xor(m[a], 1, 64);
            m[a] += __shfl_xor(m[a], 2, 64);
        }
    }
    vacc += __shfl_xor(vacc, 1, 64);
    vacc += __shfl_xor(vacc, 2, 64);
    const float invB = 1.f / (float)B;
    const float half_log2pi = 0.5f * logf(2.f * 3.14159265358979323846f);
    float dls[AM];
    float ta = 0.f, tc = 0.f, te = 0.f, tb = 0.f;
#pragma unroll
    for (int a = 0; a < AM; ++a) dls[a] = 0.f;
    if (valid) {
        const size_t i = (size_t)row;
        float sq = 0.f, sls = 0.f, ent = 0.f, bl = 0.f;
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            if (a < A) {
                m[a] = rnd_h(m[a] + bmu_f[a]);  // the fp16 head output
                if ((a & 3) == q) mu_out[i * A + a] = __float2half(m[a]);
                const float ls = lsv[a];
                const float sg = expf(ls);
                const float z = (xact[a] - m[a]) / sg;
                sq += z * z;
                sls += ls;
                ent += 0.5f + half_log2pi + logf(sg);
                const float t1 = fminf(rnd_h(m[a] + 1.1f), 0.f);
                const float t2 = fmaxf(rnd_h(m[a] - 1.1f), 0.f);
                bl += t1 * t1 + t2 * t2;
            }
        }
        const float nlp = 0.5f * sq + half_log2pi * (float)A + sls;
        const float r = expf(r_old_nlp - nlp);
        const float ad = r_adv;
        const float rc = fminf(fmaxf(r, 1.f - e), 1.f + e);
        const float p = -(ad * r), qq = -(ad * rc);
        const float av = fmaxf(p, qq);
        const float v = rnd_h(vacc + bv_f), ov = r_old_v, R = r_ret;
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
        float wp, wq;
        max_grad(p, qq, wp, wq);
        const float in_r = (r >= 1.f - e && r <= 1.f + e) ? 1.f : 0.f;
        const float dratio = invB * (wp * -ad + wq * -ad * in_r);
        const float dnlp = -r * dratio;
#pragma unroll
        for (int a = 0; a < AM; ++a) {
            if (a < A) {
                const float sg = expf(lsv[a]);
                const float z = (xact[a] - m[a]) / sg;
                const float h1 = rnd_h(m[a] + 1.1f), h2 = rnd_h(m[a] - 1.1f);
                const float db = (h1 <= 0.f ? 2.f * fminf(h1, 0.f) : 0.f) + (h2 >= 0.f ? 2.f * fmaxf(h2, 0.f) : 0.f);
                if ((a & 3) == q) dmu[i * A + a] = dnlp * (-z / sg) + bc * invB * db;
                dls[a] = dnlp * (1.f - z * z) - ec * invB;
            }
        }
        if (q == 0) {
            dv[i] = 0.5f * cc * invB * dcdv;
            ta = av; tc = cv; te = ent; tb = bl;
        } else {
#pragma unroll
            for (int a = 0; a < AM; ++a) dls[a] = 0.f;  // one contribution per row
        }
    }
    // the wave's 16 rows (butterfly, a fixed order), then the 4 waves in order -> part[block][kNT]
    float vals[4 + AM];
    vals[0] = ta; vals[1] = tc; vals[2] = te; vals[3] = tb;
#pragma unroll
    for (int a = 0; a < AM; ++a) vals[4 + a] = dls[a];
#pragma unroll
    for (int k = 0; k < 4 + AM; ++k) {
        if (k < 4 + A) {
            float x = vals[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if (lane == 0) red[wave][k] = x;
        }
    }
    __syncthreads();
    if (t < 4 + A) part[(size_t)blockIdx.x * kNT + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

// one thread per column pair (actor columns 2p, 2p + 1 and the critic's) and row group: 512 / H groups of
// kHRB * H / 512 rows (16 for H = 128), every row's loads issued before the math
template <int AM>
__global__ __launch_bounds__(256) void k_heads_bwd(const float* __restrict__ g, const float* __restrict__ dmu,
                                                   const float* __restrict__ dv, const __half* __restrict__ hid,
                                                   int ld, int acol, int ccol, int H, const __half* __restrict__ wmu,
                                                   const __half* __restrict__ wv, int B, int A,
                                                   __half* __restrict__ dhid, float* __restrict__ part) {
    constexpr int SDW = (AM + 4) & ~3, NS = 2 * AM + 2, RMAX = 64;  // sd row stride; partial slots per thread
    __shared__ float sd[kHRB][SDW];  // the rows' fp16 d mu (as float) and, in column AM, d v
    __shared__ float comb[NS * 256];  // the row groups' weight partials
    const int t = threadIdx.x, row0 = blockIdx.x * kHRB;
    const int nrow = min(kHRB, B - row0);
    const float s = *g;
    const int H2 = H / 2, GR = 256 / H2, grp = t / H2, p = t - grp * H2, RPG = kHRB / GR;
    // the gradient rows (scaled, rounded to fp16 as the torch path's head gradients) and this thread's weights
    if (t < kHRB) {
#pragma unroll
        for (int a = 0; a < AM; ++a) sd[t][a] = (a < A && t < nrow) ? rnd_h(dmu[(size_t)(row0 + t) * A + a] * s) : 0.f;
        sd[t][AM] = t < nrow ? rnd_h(dv[row0 + t] * s) : 0.f;
    }
    float w0[AM], w1[AM], acc0[AM], acc1[AM];
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        w0[a] = a < A ? h2f(wmu[(size_t)a * H + 2 * p]) : 0.f;  // (the fp16 shadow: 2-byte aligned only)
        w1[a] = a < A ? h2f(wmu[(size_t)a * H + 2 * p + 1]) : 0.f;
        acc0[a] = 0.f;
        acc1[a] = 0.f;
    }
    const float wv0 = h2f(wv[2 * p]), wv1 = h2f(wv[2 * p + 1]);
    float av0 = 0.f, av1 = 0.f;
    const int r0 = grp * RPG, r1 = min(r0 + RPG, nrow);
    __half2 xa[RMAX / 4], xc[RMAX / 4];  // RPG <= 16 for H <= 128; H = 256 takes two passes below
    __syncthreads();
    for (int rb = r0; rb < r1; rb += RMAX / 4) {
#pragma unroll
        for (int k = 0; k < RMAX / 4; ++k) {
            const size_t o = (size_t)(row0 + rb + k) * ld;
            const bool in = rb + k < r1;
            xa[k] = in ? *reinterpret_cast<const __half2*>(hid + o + acol + 2 * p) : __half2{};
            xc[k] = in ? *reinterpret_cast<const __half2*>(hid + o + ccol + 2 * p) : __half2{};
        }
#pragma unroll
        for (int k = 0; k < RMAX / 4; ++k) {
            const int r = rb + k;
            if (r < r1) {
                const float x0 = __low2float(xa[k]), x1 = __high2float(xa[k]);
                float d0 = 0.f, d1 = 0.f;
#pragma unroll
                for (int a = 0; a < AM; ++a) {
                    if (a < A) {
                        const float d = sd[r][a];
                        d0 += d * w0[a];
                        d1 += d * w1[a];
                        acc0[a] += d * x0;
                        acc1[a] += d * x1;
                    }
                }
                const float dvr = sd[r][AM];
                const size_t o = (size_t)(row0 + r) * ld;
                *reinterpret_cast<__half2*>(dhid + o + acol + 2 * p) = __floats2half2_rn(d0, d1);
                *reinterpret_cast<__half2*>(dhid + o + ccol + 2 * p) = __floats2half2_rn(dvr * wv0, dvr * wv1);
                av0 += dvr * __low2float(xc[k]);
                av1 += dvr * __high2float(xc[k]);
            }
        }
    }
    // the row groups' partials in a fixed order (group 0 adds 1, 2, ...)
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        comb[(2 * a) * 256 + t] = acc0[a];
        comb[(2 * a + 1) * 256 + t] = acc1[a];
    }
    comb[(2 * AM) * 256 + t] = av0;
    comb[(2 * AM + 1) * 256 + t] = av1;
    __syncthreads();
    const size_t P = (size_t)A * H + H + A + 1;
    float* pb = part + (size_t)blockIdx.x * P;
    if (grp == 0) {
        for (int a = 0; a <= A; ++a) {
            const int sl = a < A ? 2 * a : 2 * AM;  // a == A: w_v, right after W_mu's slots
            float s0 = comb[sl * 256 + p], s1 = comb[(sl + 1) * 256 + p];
            for (int g2 = 1; g2 < GR; ++g2) {
                s0 += comb[sl * 256 + g2 * H2 + p];
                s1 += comb[(sl + 1) * 256 + g2 * H2 + p];
            }
            pb[(size_t)a * H + 2 * p] = s0;
            pb[(size_t)a * H + 2 * p + 1] = s1;
        }
    }
    if (t <= A) {  // bias partials: d b_mu (t < A), d b_v (t == A)
        const int cl = t < A ? t : AM;
        float sum = 0.f;
        for (int r = 0; r < nrow; ++r) sum += sd[r][cl];
        pb[(size_t)A * H + H + t] = sum;
    }
}

// 64 outputs per workgroup, 4 lanes each: lane group j adds the blocks b = j (mod 4) in 8 chains, then the 4 in order
__device__ __forceinline__ float sum_partials(const float* __restrict__ part, int blocks, size_t stride, int i,
                                              bool on, float (*sh)[64]) {
    const int t = threadIdx.x, j = t >> 6, o = t & 63;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (on) {
        int b = j;
        for (; b + 28 < blocks; b += 32) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += part[(size_t)(b + 4 * k) * stride + i];
        }
        for (; b < blocks; b += 4) acc[0] += part[(size_t)b * stride + i];
    }
    sh[j][o] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    return (sh[0][o] + sh[1][o]) + (sh[2][o] + sh[3][o]);
}

__global__ __launch_bounds__(256) void k_heads_bfin(const float* __restrict__ part, int blocks, int A, int H,
                                                    const float* __restrict__ g, const float* __restrict__ dls,
                                                    float* __restrict__ gw_mu, float* __restrict__ gb_mu,
                                                    float* __restrict__ gw_v, float* __restrict__ gb_v,
                                                    float* __restrict__ g_logstd, int store) {
    __shared__ float sh[4][64];
    const int P = A * H + H + A + 1;
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const float sum = sum_partials(part, blocks, (size_t)P, i, i < P, sh);
    if (threadIdx.x >= 64) return;
    float* dst = i < A * H ? gw_mu + i
                 : i < A * H + H ? gw_v + (i - A * H)
                 : i < A * H + H + A ? gb_mu + (i - A * H - H)
                 : i < P ? gb_v : i < P + A ? g_logstd + (i - P) : nullptr;
    if (!dst) return;
    const float val = i < P ? sum : dls[i - P] * *g;  // the sigma parameter: d logstd times the scale
    *dst = store ? val : *dst + val;  // AccumulateGrad's add, or the first write of a zero-free flat buffer
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
    hipLaunchKernelGGL(k_ppo_finish, dim3(1), dim3(256), 0, st, partials, blocks, (int)num_actions, 1.f / (float)rows,
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

extern "C" int rl_ppo_heads_partials_size(int32_t rows, int32_t hidden, int32_t num_actions) {
    if (rows <= 0 || hidden <= 0 || num_actions <= 0) return 0;
    const int64_t fwd = (int64_t)((rows + kHR - 1) / kHR) * kNT;
    const int64_t bwd = (int64_t)((rows + kHRB - 1) / kHRB) * ((int64_t)num_actions * hidden + hidden + num_actions + 1);
    const int64_t n = fwd > bwd ? fwd : bwd;
    return n > INT32_MAX ? -1 : (int)n;
}

static int heads_check(const char* who, int64_t ld, int32_t acol, int32_t ccol, int32_t H, int32_t rows, int32_t A) {
    char msg[320];
    if (rows <= 0 || A <= 0 || A > kMaxA || !(H == 32 || H == 64 || H == 128 || H == 256) || acol < 0 || ccol < 0 ||
        acol % 8 || ccol % 8 || acol + H > ld || ccol + H > ld || (acol < ccol + H && ccol < acol + H) || ld % 8) {
        snprintf(msg, sizeof(msg), "%s: needs 0 < num_actions <= 32, hidden 32, 64, 128 or 256, disjoint column "
                 "ranges at multiples of 8 inside a row stride in multiples of 8 (ld %lld, actor %d, critic %d, "
                 "hidden %d, actions %d)", who, (long long)ld, acol, ccol, H, A);
        return rl_set_error(msg);
    }
    return 0;
}

template <int AM>
static void launch_heads_fwd(int blocks, size_t, hipStream_t st, const __half* hid, int ld, int acol, int ccol, int H,
                             const __half* wmu, const __half* bmu, const __half* wv, const __half* bv,
                             const float* logstd, const float* act, const float* old_nlp, const float* adv,
                             const float* old_v, const float* ret, int B, int A, float e, int clip_value, float cc,
                             float ec, float bc, __half* mu_out, float* dmu, float* dv, float* part) {
#define RL_HEADS_FWD(NC)                                                                                            \
    hipLaunchKernelGGL((k_heads_fwd<AM, NC>), dim3(blocks), dim3(256), 0, st, hid, ld, acol, ccol, wmu, bmu, wv, bv, \
                       logstd, act, old_nlp, adv, old_v, ret, B, A, e, clip_value, cc, ec, bc, mu_out, dmu, dv, part)
    switch (H) {
        case 32: RL_HEADS_FWD(1); break;
        case 64: RL_HEADS_FWD(2); break;
        case 128: RL_HEADS_FWD(4); break;
        default: RL_HEADS_FWD(8); break;
    }
#undef RL_HEADS_FWD
}

#define RL_HEADS_AM_SWITCH(A, F, ...)          \
    do {                                       \
        if ((A) <= 4) F<4>(__VA_ARGS__);       \
        else if ((A) <= 8) F<8>(__VA_ARGS__);  \
        else if ((A) <= 12) F<12>(__VA_ARGS__); \
        else if ((A) <= 16) F<16>(__VA_ARGS__); \
        else if ((A) <= 24) F<24>(__VA_ARGS__); \
        else F<32>(__VA_ARGS__);               \
    } while (0)

extern "C" int rl_ppo_heads_loss(const void* hidden, int64_t ld, int32_t actor_col, int32_t critic_col,
                                 int32_t hidden_size, const void* w_mu, const void* b_mu, const void* w_v,
                                 const void* b_v, const float* logstd, const float* actions, const float* old_neglogp,
                                 const float* advantages, const float* old_values, const float* returns, int32_t rows,
                                 int32_t num_actions, double e_clip, int32_t clip_value, double critic_coef,
                                 double entropy_coef, double bounds_loss_coef, void* mu_out, float* dmu,
                                 float* dvalues, float* partials, float* loss, float* stats, float* dlogstd,
                                 void* stream) {
    if (int rc = heads_check("rl_ppo_heads_loss", ld, actor_col, critic_col, hidden_size, rows, num_actions)) return rc;
    if (!hidden || !w_mu || !b_mu || !w_v || !b_v || !logstd || !actions || !old_neglogp || !advantages ||
        !old_values || !returns || !mu_out || !dmu || !dvalues || !partials || !loss || !stats || !dlogstd)
        return rl_set_error("rl_ppo_heads_loss: null pointer");
    if (reinterpret_cast<uintptr_t>(hidden) % 16)
        return rl_set_error("rl_ppo_heads_loss: hidden must be 16-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    const int blocks = (rows + kHR - 1) / kHR;
    const float e = (float)e_clip, cc = (float)critic_coef, ec = (float)entropy_coef, bc = (float)bounds_loss_coef;
    RL_HEADS_AM_SWITCH(num_actions, launch_heads_fwd, blocks, 0, st, (const __half*)hidden, (int)ld, (int)actor_col,
                       (int)critic_col, (int)hidden_size, (const __half*)w_mu, (const __half*)b_mu,
                       (const __half*)w_v, (const __half*)b_v, logstd, actions, old_neglogp, advantages, old_values,
                       returns, (int)rows, (int)num_actions, e, (int)clip_value, cc, ec, bc, (__half*)mu_out, dmu,
                       dvalues, partials);
    if (int rc = launch_err("rl_ppo_heads_loss")) return rc;
    hipLaunchKernelGGL(k_ppo_finish, dim3(1), dim3(256), 0, st, partials, blocks, (int)num_actions, 1.f / (float)rows,
                       cc, ec, bc, loss, stats, dlogstd);
    return launch_err("rl_ppo_heads_loss finish");
}

template <int AM>
static void launch_heads_bwd(int blocks, hipStream_t st, const float* g, const float* dmu, const float* dv,
                             const __half* hid, int ld, int acol, int ccol, int H, const __half* wmu, const __half* wv,
                             int B, int A, __half* dhid, float* part) {
    hipLaunchKernelGGL((k_heads_bwd<AM>), dim3(blocks), dim3(256), 0, st, g, dmu, dv, hid, ld, acol, ccol, H, wmu, wv,
                       B, A, dhid, part);
}

extern "C" int rl_ppo_heads_loss_backward(const float* grad_loss, const float* dmu, const float* dvalues,
                                          const float* dlogstd, const void* hidden, int64_t ld, int32_t actor_col,
                                          int32_t critic_col, int32_t hidden_size, const void* w_mu, const void* w_v,
                                          int32_t rows, int32_t num_actions, void* dhidden, float* partials,
                                          float* grad_w_mu, float* grad_b_mu, float* grad_w_v, float* grad_b_v,
                                          float* grad_logstd, int32_t store_grads, void* stream) {
    if (int rc = heads_check("rl_ppo_heads_loss_backward", ld, actor_col, critic_col, hidden_size, rows, num_actions))
        return rc;
    if (!grad_loss || !dmu || !dvalues || !dlogstd || !hidden || !w_mu || !w_v || !dhidden || !partials ||
        !grad_w_mu || !grad_b_mu || !grad_w_v || !grad_b_v || !grad_logstd)
        return rl_set_error("rl_ppo_heads_loss_backward: null pointer");
    if (reinterpret_cast<uintptr_t>(hidden) % 4 || reinterpret_cast<uintptr_t>(dhidden) % 4)
        return rl_set_error("rl_ppo_heads_loss_backward: hidden / dhidden must be 4-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    const int blocks = (rows + kHRB - 1) / kHRB, H = hidden_size, A = num_actions;
    RL_HEADS_AM_SWITCH(A, launch_heads_bwd, blocks, st, grad_loss, dmu, dvalues, (const __half*)hidden, (int)ld,
                       (int)actor_col, (int)critic_col, H, (const __half*)w_mu, (const __half*)w_v, (int)rows, A,
                       (__half*)dhidden, partials);
    if (int rc = launch_err("rl_ppo_heads_loss_backward")) return rc;
    const int P = A * H + H + A + 1 + A;
    hipLaunchKernelGGL(k_heads_bfin, dim3((P + 63) / 64), dim3(256), 0, st, partials, blocks, A, H, grad_loss, dlogstd,
                       grad_w_mu, grad_b_mu, grad_w_v, grad_b_v, grad_logstd, (int)store_grads);
    return launch_err("rl_ppo_heads_loss_backward finish");
}
