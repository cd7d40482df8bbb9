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

#define RL_ABI_VERSION 1

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

#ifdef __cplusplus
}
#endif
#endif
