/*
 * gymrl.h -- C ABI of libgymrl.so: device kernels of the PPO learner that
 * consumes VecTask.step() (rl_games a2c_continuous, the reference's trainer:
 * isaacgymenvs/train.py:188-218 builds an rl_games Runner; rl-games>=1.6.0,
 * setup.py:22, is not vendored in /root/reference).
 *
 *   rl_gae : rl_games a2c_common.py A2CBase.discount_values (v1.6.x) fused with
 *            the "returns = advs + values" step of play_steps and the
 *            swap_and_flatten01 re-layout of the experience buffer: reads the
 *            time-major horizon buffers the rollout wrote, writes env-major
 *            [N][H] rows the PPO minibatches slice.
 *   rl_splitk_accum : finish of the learner's split-K weight gradients (the
 *            backward of rl_games' actor/critic nn.Linear layers, network_builder.py
 *            A2CBuilder, as a batched GEMM over row blocks): sums the partials in
 *            a fixed order and adds them into the parameter's fp32 gradient.
 *   rl_colsum_accum : the same layers' bias gradients (column sums), deterministic.
 *   rl_ppo_loss / rl_ppo_loss_backward : the minibatch PPO loss and its gradient.
 *   rl_rms_normalize : the model's running mean / std input normalisation.
 *   rl_policy_head : the act forward's sampling / neglogp / value unnormalisation.
 *   rl_rollout_post : the rollout bookkeeping after each env step (play_steps).
 *   rl_rollout_pre : the experience slot written before each env step (play_steps).
 *
 * All pointers are device pointers; calls are ordered on `stream` (a hipStream_t,
 * NULL = legacy default stream) and return 0 on success, otherwise a nonzero
 * code with the message in rl_last_error().
 */
#ifndef GYMRL_H
#define GYMRL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RL_ABI_VERSION 7

int rl_abi_version(void);
const char *rl_last_error(void);

/*
 * Generalised advantage estimation over one rollout of `horizon` steps x `num_envs` envs.
 *   rewards  [H][N] f32  shaped rewards (value bootstrap on time-outs already added)
 *   values   [H][N] f32  value estimates at the observations the actions were taken from
 *   dones    [H][N] u8   done flags of those observations (rl_games mb_fdones)
 *   last_values [N] f32, last_dones [N] u8  bootstrap after the last step
 * Writes (env-major, row n = env n's H steps):
 *   returns_out [N][H], advs_out [N][H] (nullable), values_out [N][H] (nullable, = values transposed)
 * gamma and tau are the config's Python floats: the kernel uses float(gamma) and float(gamma * tau),
 * the constants torch's elementwise ops see in the reference loop.
 * Recurrence (t = H-1 .. 0):  nn = 1 - done(t+1) (last_dones at t = H-1), nv = value(t+1)
 *   delta = r_t + gamma * nv * nn - v_t;   adv_t = delta + gamma * tau * nn * adv_{t+1}
 */
int rl_gae(const float *rewards, const float *values, const uint8_t *dones, const float *last_values,
           const uint8_t *last_dones, int32_t horizon, int32_t num_envs, double gamma, double tau,
           float *returns_out, float *advs_out, float *values_out, void *stream);

/*
 * grad[i] += sum_{p = 0..num_parts-1} parts[p * n + i]   (i < n; fp32 sum in ascending p order)
 *   parts  [num_parts][n]  fp16 (parts_are_f16 != 0) or f32, device
 *   grad   [n] f32, device; any float offset (a view into a flat gradient buffer)
 * Replaces `grad += parts.sum(0, dtype=float32)` (rl/network.py split-K weight gradient).
 */
int rl_splitk_accum(const void *parts, int32_t num_parts, int64_t n, int32_t parts_are_f16, float *grad,
                    void *stream);

/*
 * ABI 6: up to RL_SPLITK_MAX_JOBS rl_splitk_accum finishes in one launch (the learner's layers at the end of the
 * backward); store != 0: grad = sum (no read of grad; the fused learner writes each gradient once and skips
 * zeroing the flat buffer), else grad += sum.  Same per-job arithmetic and order as rl_splitk_accum.
 */
#define RL_SPLITK_MAX_JOBS 8
typedef struct rl_splitk_job {
    const void *parts;
    float *grad;
    int64_t n;
    int32_t num_parts;
    int32_t parts_are_f16;
} rl_splitk_job;
int rl_splitk_accum_multi(const rl_splitk_job *jobs, int32_t num_jobs, int32_t store, void *stream);

/*
 * grad[c] += sum_r g[r * cols + c]   (the bias gradient of a Linear layer: column sums of its output
 * gradient; fp32 sums, deterministic: fixed-order row-block partials, then the partials added in a
 * fixed order; two launches on `stream`)
 *   g [rows][cols] fp16 (g_is_f16 != 0) or f32, 16-byte aligned; cols % 8 == 0 and cols <= 2048
 *   grad [cols] f32 (any float offset); work >= 256 * cols f32 scratch (calls sharing it: one stream)
 */
int rl_colsum_accum(const void *g, int32_t rows, int32_t cols, int32_t g_is_f16, float *grad, float *work,
                    void *stream);

/*
 * The PPO minibatch loss and its gradient (rl_games a2c_continuous calc_gradients for the
 * continuous_a2c_logstd model with fixed sigma): actor (clipped surrogate), critic (clipped value
 * loss if clip_value), entropy and bound losses of `rows` samples with `num_actions` <= 32 actions.
 *   mu [rows][A], values [rows] (fp16 if *_is_f16 else f32), logstd [A] f32 (the sigma parameter),
 *   actions [rows][A], old_neglogp, advantages, old_values, returns [rows] f32
 * Writes loss (0-d: a + 0.5 c critic_coef - entropy entropy_coef + b bounds_loss_coef of the means),
 * stats[4] = the means (a, c, entropy, b), and the UNSCALED gradients of loss: dmu [rows][A],
 * dvalues [rows], dlogstd [A] (f32); partials >= ceil(rows / 128) * 36 f32 scratch.  Two launches.
 */
int rl_ppo_loss(const void *mu, int32_t mu_is_f16, const void *values, int32_t values_is_f16, const float *logstd,
                const float *actions, const float *old_neglogp, const float *advantages, const float *old_values,
                const float *returns, int32_t rows, int32_t num_actions, double e_clip, int32_t clip_value,
                double critic_coef, double entropy_coef, double bounds_loss_coef, float *dmu, float *dvalues,
                float *partials, float *loss, float *stats, float *dlogstd, void *stream);

/*
 * Backward of rl_ppo_loss: d(upstream) = grad_loss[0] (device f32, e.g. the GradScaler scale) times the
 * stored gradients, cast to the dtypes of mu / values: dmu_out [rows][A], dvalues_out [rows], dlogstd_out [A].
 */
int rl_ppo_loss_backward(const float *grad_loss, const float *dmu, const float *dvalues, const float *dlogstd,
                         int32_t rows, int32_t num_actions, void *dmu_out, int32_t dmu_is_f16, void *dvalues_out,
                         int32_t dvalues_is_f16, float *dlogstd_out, void *stream);

/*
 * ABI 6 -- the heads and the loss in one pass (rl_games network_builder's mu / value heads, fp16 under autocast,
 * then rl_ppo_loss).  hidden: fp16 [rows][ld] holding the actor MLP's output in columns [actor_col, +hidden_size)
 * and the critic's in [critic_col, +hidden_size) (disjoint; even columns, even ld, 4-byte aligned; hidden_size even
 * and <= 256); w_mu [A][hidden_size], b_mu [A], w_v [hidden_size], b_v [1] fp16 (the parameters' fp16 shadows).
 * mu = fp16(hidden_a w_mu^T + b_mu), value = fp16(hidden_c w_v + b_v) (fp32 accumulation), then rl_ppo_loss's
 * statements: loss, stats[4], the unscaled dmu [rows][A], dvalues [rows], dlogstd [A] f32; mu_out fp16 [rows][A].
 * partials >= rl_ppo_heads_partials_size(rows, hidden_size, A) f32 (shared by both passes).  Two launches.
 */
int rl_ppo_heads_partials_size(int32_t rows, int32_t hidden_size, int32_t num_actions);
int rl_ppo_heads_loss(const void *hidden, int64_t ld, int32_t actor_col, int32_t critic_col, int32_t hidden_size,
                      const void *w_mu, const void *b_mu, const void *w_v, const void *b_v, const float *logstd,
                      const float *actions, const float *old_neglogp, const float *advantages, const float *old_values,
                      const float *returns, int32_t rows, int32_t num_actions, double e_clip, int32_t clip_value,
                      double critic_coef, double entropy_coef, double bounds_loss_coef, void *mu_out, float *dmu,
                      float *dvalues, float *partials, float *loss, float *stats, float *dlogstd, void *stream);
/*
 * Backward: s = grad_loss[0]; d mu = fp16(dmu s), d v = fp16(dvalues s) (the fp16 head gradients), then
 * dhidden (fp16, same layout as hidden; the two column ranges written) = d mu w_mu | d v w_v, and the head
 * parameters' gradients ADDED to grad_w_mu [A][hidden_size], grad_b_mu [A], grad_w_v [hidden_size], grad_b_v [1],
 * grad_logstd [A] += dlogstd s (f32; fixed-order sums over row blocks; store_grads: = instead of +=, the fused
 * learner's zero-free flat gradient).  Two launches.
 */
int rl_ppo_heads_loss_backward(const float *grad_loss, const float *dmu, const float *dvalues, const float *dlogstd,
                               const void *hidden, int64_t ld, int32_t actor_col, int32_t critic_col,
                               int32_t hidden_size, const void *w_mu, const void *w_v, int32_t rows,
                               int32_t num_actions, void *dhidden, float *partials, float *grad_w_mu, float *grad_b_mu,
                               float *grad_w_v, float *grad_b_v, float *grad_logstd, int32_t store_grads,
                               void *stream);

/*
 * RunningMeanStd of the model input (rl_games algos_torch/running_mean_std.py): with update != 0 the
 * batch mean / unbiased var of x [rows][cols] (cols <= 256) are merged into the float64 running moments
 * running_mean / running_var [cols] and count (0-d) as the reference does in train mode; then
 * y = clamp((x - float(mean)) / sqrt(float(var) + epsilon), -5, 5).  partials >= ceil(rows / 64) * cols * 2
 * f32 scratch (update only).  Three launches (update) or one.
 */
int rl_rms_normalize(const float *x, int32_t rows, int32_t cols, double *running_mean, double *running_var,
                     double *count, double epsilon, int32_t update, float *partials, float *y, void *stream);
/* ABI 6: the same with y written as fp16 (the learner's first-layer operand; the value autocast would cast to). */
int rl_rms_normalize_h(const float *x, int32_t rows, int32_t cols, double *running_mean, double *running_var,
                       double *count, double epsilon, int32_t update, float *partials, void *y_half, void *stream);

/*
 * Act-forward head of the fixed-sigma continuous model (rl_games ModelA2CContinuousLogStd eval forward):
 *   sigmas = exp(logstd) [N][A], actions = noise * sigma + mu (noise: torch's normal_(0, 1) draws),
 *   neglogp [N] of the actions, value_out [N] = value unnormalised by the value RunningMeanStd
 *   (value_mean / value_var: its float64 moments, [1]; both null = no value normalisation).
 *   mu, noise [N][A], logstd [A], value [N]: f32.
 */
int rl_policy_head(const float *mu, const float *noise, const float *logstd, const float *value,
                   const double *value_mean, const double *value_var, double value_eps, int32_t num_envs,
                   int32_t num_actions, float *actions, float *sigmas, float *neglogp, float *value_out, void *stream);

/*
 * Rollout bookkeeping after one VecTask.step (rl_games a2c_common.py play_steps, the statements after
 * env_step: rewards_shaper + value bootstrap on time-outs, experience rewards / dones, current episode
 * reward / length, game_rewards / game_lengths AverageMeter updates of the done envs, reset of the
 * done envs' counters).  One workgroup; N <= any.
 *   rewards [N] f32; dones [N] (dones_bytes 1: bool / uint8, 8: int64)
 *   time_outs [N] (time_outs_bytes as dones) and values [N] f32: both null = no value bootstrap
 *   shaped = (r + reward_shift) * reward_scale [+ gamma * value * (time_out != 0)]   (fp32, torch's order)
 * Writes dones_out [N] u8, rewards_out [N] f32 (= shaped), current_rewards / current_lengths [N] f32
 * (+= r, += 1, then * (1 - done)), meter_rewards / meter_lengths [2] f32 = (mean, current_size) of
 * the AverageMeter(games_to_track) updated with the done envs' episode rewards / lengths.
 */
int rl_rollout_post(const float *rewards, const void *dones, int32_t dones_bytes, const void *time_outs,
                    int32_t time_outs_bytes, const float *values, double reward_shift, double reward_scale,
                    double gamma, int32_t num_envs, uint8_t *dones_out, float *rewards_out, float *current_rewards,
                    float *current_lengths, float *meter_rewards, float *meter_lengths, int32_t games_to_track,
                    void *stream);

/*
 * ABI 7 -- the act forward's heads and head in one launch: mu = a W_mu^T + b_mu (W_mu [A][H]), value =
 * c w_v^T + b_v (w_v [H], b_v [1]) from the actor / critic MLP outputs a, c (rows of H f32, row strides
 * ld_actor / ld_critic), then rl_policy_head's statements on them (noise [N][A] = torch's normal_ draws,
 * logstd [A]; value unnormalised when value_mean / value_var are given).  Outputs mu, actions, sigmas
 * [N][A], neglogp [N], value_out [N].  Each head output: four f32 FMA chains over k mod 4, added pairwise.
 */
int rl_act_heads(const float *hidden_actor, int32_t ld_actor, const float *hidden_critic, int32_t ld_critic,
                 int32_t H, const float *w_mu, const float *b_mu, const float *w_v, const float *b_v, const float *noise,
                 const float *logstd, const double *value_mean, const double *value_var, double value_eps,
                 int32_t num_envs, int32_t num_actions, float *mu, float *actions, float *sigmas, float *neglogp,
                 float *value_out, void *stream);

/*
 * ABI 7 -- play_steps' experience of horizon slot `slot` before env.step (rl_games a2c_common.py
 * update_data('obses' / 'dones' / 'values' / 'actions' / 'neglogpacs' / 'mus' / 'sigmas')), one launch:
 *   b_obs[e][slot][:] = obs[e][:]            obs [N][obs_dim] f32, b_obs [N][horizon][obs_dim]
 *   t_dones[slot][e] = dones[e]              dones [N] u8, t_dones [horizon][N] u8
 *   t_values[slot][e] = values[e * values_stride]                      t_values [horizon][N] f32
 *   b_actions / b_mu / b_sigma[e][slot][:] = actions / mu / sigma[e][:]  ([N][A] in, [N][horizon][A] out)
 *   b_neglogp[e][slot] = neglogp[e]          neglogp [N], b_neglogp [N][horizon]
 * Inputs contiguous as shown; num_actions <= 64.  Plain copies (bit-identical).
 */
int rl_rollout_pre(const float *obs, int32_t obs_dim, const uint8_t *dones, const float *values, int32_t values_stride,
                   const float *actions, const float *neglogp, const float *mu, const float *sigma, int32_t num_envs,
                   int32_t num_actions, int32_t horizon, int32_t slot, float *b_obs, uint8_t *t_dones, float *t_values,
                   float *b_actions, float *b_neglogp, float *b_mu, float *b_sigma, void *stream);

/*
 * ABI 4 -- the minibatch optimizer step over the learner's flat buffers (rl_games a2c_common.py
 * trancate_gradients_and_step: scaler.unscale_, clip_grad_norm_, scaler.step(Adam), scaler.update):
 *   g = grad / scale (scale null: 1, no skipping, no update); found_inf = any non-finite g;
 *   unless found_inf: g *= min(1, max_norm / (||g|| + 1e-6)) when max_norm > 0; g += weight_decay * p;
 *   Adam with step t = *step + 1: m = lerp(m, g, 1 - beta1), v = beta2 v + (1 - beta2) g^2,
 *   p -= lr / (1 - beta1^t) * m / (sqrt(v) / sqrt(1 - beta2^t) + eps); then *step = t.
 *   GradScaler.update on (scale, growth_tracker): found_inf -> scale *= backoff, tracker = 0; else
 *   tracker += 1, and at growth_interval scale *= growth, tracker = 0.
 * param / grad / exp_avg / exp_avg_sq [n] f32; step, lr, scale: device f32 scalars; growth_tracker: device
 * int32; partials >= rl_opt_partials_size() f32 scratch.  Three launches, no host synchronisation.
 */
typedef struct rl_opt_hyper {
    float max_norm;       /* <= 0: no clipping */
    float beta1, beta2, eps, weight_decay;
    float backoff, growth;
    int32_t growth_interval;
} rl_opt_hyper;

int rl_opt_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float *step,
                const float *lr, float *scale, int32_t *growth_tracker, const rl_opt_hyper *hyper, float *partials,
                void *stream);
int rl_opt_partials_size(void);
/*
 * ABI 6: rl_opt_step that also writes the updated parameters' fp16 shadow param_half [n] (the next minibatch's
 * GEMM operands, instead of a separate cast), with the step / scale bookkeeping in the Adam launch's last workgroup:
 * two launches.  partials (rl_opt_partials_size() f32) zero-initialised once.
 */
int rl_opt_step_h(float *param, void *param_half, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                  float *step, const float *lr, float *scale, int32_t *growth_tracker, const rl_opt_hyper *hyper,
                  float *partials, void *stream);

/*
 * ABI 5 -- the hidden Linear + ELU layers of the actor / critic MLPs on the matrix cores (rl_linear.hip; rl_games
 * network_builder.py A2CBuilder mlp, trained under fp16 autocast: AnymalTerrainPPO.yaml mixed_precision).  fp16
 * operands, f32 accumulation (v_mfma_f32_32x32x16_f16).  The act-forward MLP kernel of ABI 4 (rl_act_mlp: f32 FMA
 * chains on L2-resident weights, slower than the library GEMMs it replaced) is gone.
 *
 * rl_linear_fwd: y [M][N] fp16 = act(x [M][K] (row stride ldx) . w[N][K]^T + bias [N] fp16 (null: none)), act 1 =
 *   ELU (alpha 1), 0 = none.  M % 64 == 0, N % 128 == 0, K and ldx % 4 == 0, 8-byte aligned rows.
 * rl_linear_transpose: w [N][K] fp16 -> wt [K][N] fp16 (a utility; the backward reads w itself).
 * rl_linear_bwd: the backward of rl_linear_fwd with ELU from its output y: dZ = dy * (y > 0 ? 1 : y + 1);
 *   dx [M][K] fp16 = dZ . w (w [N][K] as in rl_linear_fwd; null dx: skipped; needs K % 128 == 0);
 *   wpart [splits][N][K] f32 = per row block of M / splits rows, dZ^T . x; bpart [splits][N] f32 = column sums of
 *   dZ (null: skipped; bpart needs wpart, computed in the same pass); pstride 0 = those layouts, else block s of both starts s * pstride floats in (the merged
 *   layout bpart = wpart + N*K, pstride = N*K + N: one rl_splitk_accum finishes a weight and its bias when their
 *   gradients are adjacent).  wpart 16-byte aligned.  Finish with rl_splitk_accum (fixed order).  M % 128 == 0,
 *   M % (64 splits) == 0.
 */
int rl_linear_fwd(const void *x, int32_t M, int32_t K, int32_t ldx, const void *w, int32_t N, const void *bias,
                  int32_t act, void *y, void *stream);
int rl_linear_transpose(const void *w, int32_t N, int32_t K, void *wt, void *stream);
int rl_linear_bwd(const void *dy, const void *y, int32_t M, int32_t N, const void *x, int32_t K, int32_t ldx,
                  const void *w, void *dx, int32_t splits, float *wpart, float *bpart, int64_t pstride, void *stream);

/*
 * ABI 6 -- grouped layers: G equal-shaped layers in one launch (the actor and critic MLPs of rl_games' separate
 * network, AnymalTerrainPPO.yaml `separate: True`; network.py _GroupedMLPFn).  Group g reads x + g x_gstride,
 * w + g w_gstride, bias + g b_gstride, y / dy + g y_gstride (row stride ldy, 0: N) and writes dx + g dx_gstride
 * (row stride lddx, 0: K) and its weight / bias partials at + g part_gstride / bpart_gstride within each block of
 * pstride floats.  Strides in elements, multiples of 4.  groups = 1 with all strides 0 is the ungrouped call; every
 * group computes exactly what its own ungrouped call would (same tiles, same reduction order).
 */
typedef struct rl_linear_groups {
    int32_t groups;
    int32_t ldy;
    int32_t lddx;
    int32_t reserved;
    int64_t x_gstride, w_gstride, b_gstride, y_gstride, dx_gstride, part_gstride, bpart_gstride;
} rl_linear_groups;
int rl_linear_fwd_g(const void *x, int32_t M, int32_t K, int32_t ldx, const void *w, int32_t N, const void *bias,
                    int32_t act, void *y, const rl_linear_groups *groups, void *stream);
int rl_linear_bwd_g(const void *dy, const void *y, int32_t M, int32_t N, const void *x, int32_t K, int32_t ldx,
                    const void *w, void *dx, int32_t splits, float *wpart, float *bpart, int64_t pstride,
                    const rl_linear_groups *groups, void *stream);
/*
 * ABI 7 -- the rollout's act forward in f32 (rl_games play_steps: no autocast): y = act(x w^T + bias) with f32
 * operands, products and accumulation (v_mfma_f32_32x32x2_f32; the kernel's own order of the sum, so within f32
 * rounding of a library GEMM), act = ELU when nonzero.  Same arguments and groups as rl_linear_fwd_g with f32
 * tensors (the weight is w [N][K] row-major, row stride K).  Requires M % 64, N % 64, K % 4, ldx % 4, ldy % 4 and
 * 16-byte aligned x / w / y; group strides % 4.
 */
int rl_linear_fwd_f32_g(const float *x, int32_t M, int32_t K, int32_t ldx, const float *w, int32_t N,
                        const float *bias, int32_t act, float *y, const rl_linear_groups *groups, void *stream);

/*
 * ABI 6 -- the minibatch's policy bookkeeping (rl_policy.hip; rl_games a2c_common.py after the optimizer step:
 * torch_ext.policy_kl, dataset.update_mu_sigma, schedulers.AdaptiveScheduler, the loss / kl meters).
 * rl_policy_kl: kl (f32 scalar) = mean over M rows of the sum over A of log(s1/s0 + 1e-5) + (s0^2 + (m1 - m0)^2) /
 *   (2 (s1^2 + 1e-5)) - 0.5 with m0 = mu_new [M][A] (mu_half: fp16, else f32), s0 = sigma_new (row r at
 *   r * sigma_row_stride: 0 = one [A] row for all; sigma_is_log: the row holds log sigma, s0 = exp of it),
 *   m1 / s1 = mu_old / sigma_old [M][A] f32; write_back: mu_old / sigma_old receive the new values
 *   (update_mu_sigma).  Fixed-order sums; partials >= rl_kl_partials_size() f32, zero-initialised once.
 * rl_adaptive_lr: kl = kl * inv_world (the rank average after a summing all-reduce); adaptive: lr (f64) /= 1.5 if kl >
 *   2 kl_threshold (>= 1e-6), *= 1.5 if kl < kl_threshold / 2 (<= 1e-2), opt_lr (f32, nullable) = lr; stats (nullable):
 *   stats[0..3] += a_loss, c_loss, kl, entropy.  One thread, no host synchronisation.
 * rl_policy_kl_step: rl_policy_kl then rl_adaptive_lr (inv_world 1) in ONE launch, the single-rank minibatch (the
 *   last workgroup to finish sums the partials -- same order -- and steps the scheduler).
 */
int rl_kl_partials_size(void);
int rl_policy_kl(const void *mu_new, int32_t mu_half, const float *sigma_new, int64_t sigma_row_stride,
                 int32_t sigma_is_log, float *mu_old, float *sigma_old, int32_t M, int32_t A, int32_t write_back,
                 float *kl, float *partials, void *stream);
int rl_adaptive_lr(float *kl, float inv_world, int32_t adaptive, double kl_threshold, double *lr, float *opt_lr,
                   float *stats, const float *a_loss, const float *c_loss, const float *entropy, void *stream);
int rl_policy_kl_step(const void *mu_new, int32_t mu_half, const float *sigma_new, int64_t sigma_row_stride,
                      int32_t sigma_is_log, float *mu_old, float *sigma_old, int32_t M, int32_t A, int32_t write_back,
                      float *kl, float *partials, int32_t adaptive, double kl_threshold, double *lr, float *opt_lr,
                      float *stats, const float *a_loss, const float *c_loss, const float *entropy, void *stream);

#ifdef __cplusplus
}
#endif
#endif
