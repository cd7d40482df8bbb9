// libgymrl.so -- the act forward of the actor-critic MLP as one kernel (include/gymrl.h rl_act_mlp).
//
// rl_games ModelA2CContinuousLogStd eval forward (network_builder.py A2CBuilder: running_mean_std input
// normalisation, actor MLP [and the separate critic MLP] of Linear + ELU layers, the mu and value Linear heads),
// run once per rollout step on the whole env batch.  torch spends ~15 launches on it (a normalisation pass, one
// f32 GEMM and one ELU pass per layer, the heads), each latency-bound at 4096 rows (GEMMs of 8-16 us, 4-6 us
// elementwise passes).  Here a workgroup takes R rows through every layer with the activations in LDS:
//   * the normalised rows (the reference's clamp((x - float(mean)) / sqrt(float(var) + eps), -5, 5)) in LDS;
//   * the layers' weights transposed into a workspace first (one launch, k_transpose: always the live weights);
//   * a layer of J outputs: thread t owns column t (and t + 256 when J > 256) for the workgroup's rows (or a
//     row group when J < 256); a weight load Wt[k][j] is coalesced across the wave and serves all its rows,
//     the rows' inputs are 16-B LDS broadcasts; bias + ELU (alpha 1: x > 0 ? x : exp(x) - 1) in f32, result to the other LDS buffer;
//   * the heads: one thread per (row, output).
// f32 throughout, accumulation in k order (not hipBLASLt's order: results agree with the torch statement to
// float rounding, tests/test_ppo_gpu.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

constexpr int kThreads = 256;
constexpr int kRows = 8;       // rows per workgroup (512 workgroups at 4096 envs: two per CU)
constexpr int kMaxWidth = 512;  // widest layer (and the input)

struct Mlp {
  const float* w[RL_MLP_MAX_LAYERS];
  const float* b[RL_MLP_MAX_LAYERS];
  int dims[RL_MLP_MAX_LAYERS + 1];
  int layers;
};

// one Linear + ELU layer on the workgroup's rows: in [R][K] (LDS, row stride ldi) -> out [R][J] (row stride ldo);
// Wt [K][J] is the layer's weight transposed (k_transpose), so a wave's weight load is 64 consecutive columns
__device__ __forceinline__ void layer(const float* __restrict__ Wt, const float* __restrict__ bias, int K, int J,
                                      const float* in, int ldi, float* out, int ldo, bool elu) {
  const int t = threadIdx.x;
  const int Jt = J < kThreads ? J : kThreads;
  const int G = kThreads / Jt;  // row groups (J < 256: several threads per column, on different rows)
  const int j0 = t % Jt, g = t / Jt;
  if (g >= G) return;
  const bool two = J > kThreads && j0 + kThreads < J;
  const int j1 = two ? j0 + kThreads : j0;
  float acc0[kRows], acc1[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }
  for (int k = 0; k < K; k += 4) {
    float a[4], c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = Wt[(size_t)(k + q) * J + j0];
      c[q] = two ? Wt[(size_t)(k + q) * J + j1] : 0.f;
    }
#pragma unroll
    for (int rr = 0; rr < kRows; ++rr) {
      const int r = g + rr * G;
      if (r < kRows) {
        const float4 x = *reinterpret_cast<const float4*>(in + r * ldi + k);
        acc0[rr] = fmaf(x.w, a[3], fmaf(x.z, a[2], fmaf(x.y, a[1], fmaf(x.x, a[0], acc0[rr]))));
        if (two) acc1[rr] = fmaf(x.w, c[3], fmaf(x.z, c[2], fmaf(x.y, c[1], fmaf(x.x, c[0], acc1[rr]))));
      }
    }
  }
  const float b0 = bias[j0], b1 = two ? bias[j1] : 0.f;
#pragma unroll
  for (int rr = 0; rr < kRows; ++rr) {
    const int r = g + rr * G;
    if (r < kRows) {
      float y0 = acc0[rr] + b0;
      if (elu) y0 = y0 > 0.f ? y0 : expf(y0) - 1.f;
      out[r * ldo + j0] = y0;
      if (two) {
        float y1 = acc1[rr] + b1;
        if (elu) y1 = y1 > 0.f ? y1 : expf(y1) - 1.f;
        out[r * ldo + j1] = y1;
      }
    }
  }
}

// every hidden layer's weight transposed into the workspace, one launch: workgroup b takes a 32 x 32 tile of the
// layer whose tile range holds b (tile prefix in Tr)
struct Tr {
  const float* w[2 * RL_MLP_MAX_LAYERS];
  float* wt[2 * RL_MLP_MAX_LAYERS];
  int rows[2 * RL_MLP_MAX_LAYERS], cols[2 * RL_MLP_MAX_LAYERS];  // W [rows][cols]
  int tile0[2 * RL_MLP_MAX_LAYERS + 1];
  int n;
};
__global__ __launch_bounds__(256) void k_transpose(Tr T) {
  __shared__ float tile[32][33];
  int l = 0;
  while (l + 1 < T.n && (int)blockIdx.x >= T.tile0[l + 1]) ++l;
  const int b = blockIdx.x - T.tile0[l];
  const int R = T.rows[l], Cc = T.cols[l];
  const int tc = (Cc + 31) / 32;
  const int r0 = (b / tc) * 32, c0 = (b % tc) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int y = ty; y < 32; y += 8)
    if (r0 + y < R && c0 + tx < Cc) tile[y][tx] = T.w[l][(size_t)(r0 + y) * Cc + c0 + tx];
  __syncthreads();
  for (int y = ty; y < 32; y += 8)
    if (c0 + y < Cc && r0 + tx < R) T.wt[l][(size_t)(c0 + y) * R + r0 + tx] = tile[tx][y];
}

// the hidden layers of one MLP from `x` (LDS); returns the buffer holding the last hidden layer
__device__ __forceinline__ const float* run_mlp(const Mlp& m, const float* x, float* buf0, float* buf1) {
  const float* in = x;
  float* out = buf0;
  for (int l = 0; l < m.layers; ++l) {
    layer(m.w[l], m.b[l], m.dims[l], m.dims[l + 1], in, kMaxWidth, out, kMaxWidth, true);
    __syncthreads();
    in = out;
    out = out == buf0 ? buf1 : buf0;
  }
  return in;
}

__global__ __launch_bounds__(kThreads) void k_act_mlp(const float* __restrict__ obs, int N, int IN,
                                                      const double* __restrict__ rmean, const double* __restrict__ rvar,
                                                      float eps, Mlp actor, Mlp critic, int separate,
                                                      const float* __restrict__ wmu, const float* __restrict__ bmu, int A,
                                                      const float* __restrict__ wv, const float* __restrict__ bv,
                                                      float* __restrict__ mu_out, float* __restrict__ v_out) {
  __shared__ __attribute__((aligned(16))) float x[kRows * kMaxWidth];
  __shared__ __attribute__((aligned(16))) float buf0[kRows * kMaxWidth];
  __shared__ __attribute__((aligned(16))) float buf1[kRows * kMaxWidth];
  __shared__ __attribute__((aligned(16))) float keep[kRows * kMaxWidth];
  const int row0 = blockIdx.x * kRows;
  // normalised input rows (k_rms_norm's arithmetic); rows past N are zeros
  for (int i = threadIdx.x; i < kRows * IN; i += kThreads) {
    const int r = i / IN, c = i - r * IN;
    float v = 0.f;
    if (row0 + r < N) {
      v = obs[(size_t)(row0 + r) * IN + c];
      if (rmean) {
        const float m = (float)rmean[c];
        const float d = sqrtf((float)rvar[c] + eps);
        v = fminf(fmaxf((v - m) / d, -5.f), 5.f);
      }
    }
    x[r * kMaxWidth + c] = v;
  }
  __syncthreads();
  const int Ja = actor.dims[actor.layers];
  const float* ha = run_mlp(actor, x, buf0, buf1);
  const float* hc = ha;
  if (separate) {
    for (int i = threadIdx.x; i < kRows * Ja; i += kThreads) {
      const int r = i / Ja, c = i - r * Ja;
      keep[r * kMaxWidth + c] = ha[r * kMaxWidth + c];
    }
    __syncthreads();
    ha = keep;
    hc = run_mlp(critic, x, buf0, buf1);
  }
  const int Jc = separate ? critic.dims[critic.layers] : Ja;
  // heads: mu (A outputs of the actor trunk), value (1 output of the critic trunk)
  for (int i = threadIdx.x; i < kRows * (A + 1); i += kThreads) {
    const int r = i / (A + 1), o = i - r * (A + 1);
    if (row0 + r >= N) continue;
    if (o < A) {
      const float* w = wmu + (size_t)o * Ja;
      float acc = 0.f;
      for (int k = 0; k < Ja; ++k) acc = fmaf(ha[r * kMaxWidth + k], w[k], acc);
      mu_out[(size_t)(row0 + r) * A + o] = acc + bmu[o];
    } else {
      float acc = 0.f;
      for (int k = 0; k < Jc; ++k) acc = fmaf(hc[r * kMaxWidth + k], wv[k], acc);
      v_out[row0 + r] = acc + bv[0];
    }
  }
}

}  // namespace

extern "C" int rl_act_mlp_workspace_floats(const rl_mlp* actor, const rl_mlp* critic) {
  int64_t n = 0;
  const rl_mlp* src[2] = {actor, critic};
  for (int s = 0; s < 2; ++s)
    if (src[s])
      for (int l = 0; l < src[s]->num_layers && l < RL_MLP_MAX_LAYERS; ++l) n += (int64_t)src[s]->dims[l] * src[s]->dims[l + 1];
  return (int)n;
}

extern "C" int rl_act_mlp(const float* obs, int32_t num_rows, int32_t obs_dim, const double* running_mean,
                          const double* running_var, double epsilon, const rl_mlp* actor, const rl_mlp* critic,
                          const float* mu_w, const float* mu_b, int32_t num_actions, const float* value_w,
                          const float* value_b, float* mu_out, float* value_out, float* workspace, void* stream) {
  if (!obs || !actor || !mu_w || !mu_b || !value_w || !value_b || !mu_out || !value_out || num_rows <= 0)
    return rl_set_error("rl_act_mlp: null pointer or num_rows <= 0");
  if ((running_mean == nullptr) != (running_var == nullptr))
    return rl_set_error("rl_act_mlp: running_mean and running_var come together");
  Mlp m[2];
  const rl_mlp* src[2] = {actor, critic};
  for (int s = 0; s < 2; ++s) {
    if (!src[s]) continue;
    const rl_mlp& d = *src[s];
    if (d.num_layers < 1 || d.num_layers > RL_MLP_MAX_LAYERS || d.dims[0] != obs_dim)
      return rl_set_error("rl_act_mlp: 1..RL_MLP_MAX_LAYERS layers whose input is the observation");
    m[s].layers = d.num_layers;
    for (int l = 0; l <= d.num_layers; ++l) {
      if (d.dims[l] <= 0 || d.dims[l] > kMaxWidth || d.dims[l] % 4 != 0)
        return rl_set_error("rl_act_mlp: layer widths (and the input) must be multiples of 4 up to 512");
      m[s].dims[l] = d.dims[l];
    }
    for (int l = 0; l < d.num_layers; ++l) {
      if (!d.weight[l] || !d.bias[l]) return rl_set_error("rl_act_mlp: null layer weights");
      m[s].w[l] = d.weight[l];
      m[s].b[l] = d.bias[l];
    }
  }
  if (!critic) m[1] = m[0];
  if (num_actions <= 0 || num_actions > 256) return rl_set_error("rl_act_mlp: 0 < num_actions <= 256");
  if (!workspace) return rl_set_error("rl_act_mlp: null workspace (rl_act_mlp_workspace_floats floats)");
  // transposed weights into the workspace (the MLP kernel reads them), then the MLP
  Tr T{};
  float* ws = workspace;
  T.tile0[0] = 0;
  for (int s = 0; s < 2; ++s) {
    if (!src[s]) continue;
    for (int l = 0; l < m[s].layers; ++l) {
      const int i = T.n++;
      T.w[i] = m[s].w[l];
      T.rows[i] = m[s].dims[l + 1];
      T.cols[i] = m[s].dims[l];
      T.wt[i] = ws;
      ws += (size_t)T.rows[i] * T.cols[i];
      T.tile0[i + 1] = T.tile0[i] + ((T.rows[i] + 31) / 32) * ((T.cols[i] + 31) / 32);
      m[s].w[l] = T.wt[i];
    }
  }
  if (!critic) m[1] = m[0];
  hipLaunchKernelGGL(k_transpose, dim3(T.tile0[T.n]), dim3(256), 0, (hipStream_t)stream, T);
  hipLaunchKernelGGL(k_act_mlp, dim3((num_rows + kRows - 1) / kRows), dim3(kThreads), 0, (hipStream_t)stream, obs,
                     (int)num_rows, (int)obs_dim, running_mean, running_var, (float)epsilon, m[0], m[1],
                     critic ? 1 : 0, mu_w, mu_b, (int)num_actions, value_w, value_b, mu_out, value_out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    char msg[256];
    snprintf(msg, sizeof(msg), "rl_act_mlp: launch failed: %s", hipGetErrorString(e));
    return rl_set_error(msg) + 1;
  }
  return 0;
}
