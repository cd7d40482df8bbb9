// gt_anymal.hip -- fused AnymalTerrain post-physics kernels + the libgymtask C ABI
// (include/gymtask.h).
//
// Built with -ffp-contract=off: every statement mirrors the order of the
// reference's torch expression (anymal_terrain.py:315-382, torch_jit_utils.py:94-103)
// so results track the reference's elementwise torch ops to float rounding.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "../../include/gymtask.h"

namespace {
thread_local std::string g_err;

constexpr float kTwoPi = 6.2831854820251465f;  // float(2*np.pi) as torch casts it for a float32 tensor
constexpr float kPi = 3.1415927410125732f;     // float(np.pi)

// reference quat_rotate_inverse: a - b + c with a = v(2w^2-1), b = 2w (u x v), c = 2u (u.v)
__device__ __forceinline__ void quat_rotate_inverse(const float* q, const float* v, float* o) {
  const float w = q[3];
  const float s = 2.0f * (w * w) - 1.0f;
  const float cx = q[1] * v[2] - q[2] * v[1];
  const float cy = q[2] * v[0] - q[0] * v[2];
  const float cz = q[0] * v[1] - q[1] * v[0];
  const float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  o[0] = (v[0] * s - (cx * w) * 2.0f) + (q[0] * d) * 2.0f;
  o[1] = (v[1] * s - (cy * w) * 2.0f) + (q[1] * d) * 2.0f;
  o[2] = (v[2] * s - (cz * w) * 2.0f) + (q[2] * d) * 2.0f;
}


__device__ __forceinline__ float sq(float x) { return x * x; }
__device__ __forceinline__ float norm3(const float* v) { return sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

__global__ void k_post_a(gt_anymal_params p, gt_anymal_buffers b) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.num_envs) return;
  const int nd = p.num_dofs, nb = p.num_bodies;
  const int64_t prog = b.progress_buf[e] + 1;
  b.progress_buf[e] = prog;
  b.randomize_buf[e] += 1;

  const float* root = b.root_states + (size_t)e * 13;
  float q[4] = {root[3], root[4], root[5], root[6]};
  float blv[3], bav[3], pg[3];
  quat_rotate_inverse(q, root + 7, blv);
  quat_rotate_inverse(q, root + 10, bav);
  const float gv[3] = {0.0f, 0.0f, -1.0f};
  quat_rotate_inverse(q, gv, pg);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    b.base_lin_vel[e * 3 + k] = blv[k];
    b.base_ang_vel[e * 3 + k] = bav[k];
    b.projected_gravity[e * 3 + k] = pg[k];
  }
  // heading: quat_apply(q, (1,0,0)) -> t = 2 u x f ; f + w t + u x t
  const float tx = (q[1] * 0.0f - q[2] * 0.0f) * 2.0f;
  const float ty = (q[2] * 1.0f - q[0] * 0.0f) * 2.0f;
  const float tz = (q[0] * 0.0f - q[1] * 1.0f) * 2.0f;
  const float fx = (1.0f + q[3] * tx) + (q[1] * tz - q[2] * ty);
  const float fy = (0.0f + q[3] * ty) + (q[2] * tx - q[0] * tz);
  const float heading = atan2f(fy, fx);
  float* cmd = b.commands + (size_t)e * 4;
  // wrap_to_pi (anymal_terrain.py:684-687) is TorchScript: `%=` there is C fmod, not a floored
  // remainder, so negative angles stay negative (pinned by tests/golden/anymal_terrain.npz)
  float ang = fmodf(cmd[3] - heading, kTwoPi);
  ang = ang - kTwoPi * (ang > kPi ? 1.0f : 0.0f);
  const float c2 = fminf(fmaxf(0.5f * ang, -1.0f), 1.0f);
  cmd[2] = c2;

  // ---- check_termination
  const float* cf = b.contact_forces + (size_t)e * nb * 3;
  bool reset = norm3(cf + 3 * p.base_index) > 1.0f;
  int knee_count = 0;
  for (int k = 0; k < p.num_knees; ++k) knee_count += norm3(cf + 3 * p.knee_idx[k]) > 1.0f ? 1 : 0;
  if (!p.allow_knee_contacts && knee_count > 0) reset = true;
  if (prog >= p.max_episode_length - 1) reset = true;
  b.reset_buf[e] = reset ? 1 : 0;

  // ---- compute_reward (reference order)
  const float lin_err = sq(cmd[0] - blv[0]) + sq(cmd[1] - blv[1]);
  const float ang_err = sq(c2 - bav[2]);
  const float r_lin_xy = expf(-lin_err / 0.25f) * p.s_lin_vel_xy;
  const float r_ang_z = expf(-ang_err / 0.25f) * p.s_ang_vel_z;
  const float r_lin_z = sq(blv[2]) * p.s_lin_vel_z;
  const float r_ang_xy = (sq(bav[0]) + sq(bav[1])) * p.s_ang_vel_xy;
  const float r_orient = (sq(pg[0]) + sq(pg[1])) * p.s_orient;
  const float r_height = sq(root[2] - 0.52f) * p.s_base_height;
  const float* tq = b.torques + (size_t)e * nd;
  const float* act = b.actions + (size_t)e * nd;
  const float* lact = b.last_actions + (size_t)e * nd;
  const float* lqd = b.last_dof_vel + (size_t)e * nd;
  const float* ds = b.dof_state + (size_t)e * nd * 2;
  float s_tq = 0.f, s_acc = 0.f, s_rate = 0.f;
  for (int j = 0; j < nd; ++j) {
    s_tq += sq(tq[j]);
    s_acc += sq(lqd[j] - ds[2 * j + 1]);
    s_rate += sq(lact[j] - act[j]);
  }
  const float r_torque = s_tq * p.s_torque;
  const float r_jacc = s_acc * p.s_joint_acc;
  const float r_coll = (float)knee_count * p.s_collision;
  int stumble = 0;
  float* air = b.feet_air_time + (size_t)e * 4;
  float air_sum = 0.f;
  for (int k = 0; k < p.num_feet; ++k) {
    const float* f = cf + 3 * p.feet_idx[k];
    stumble += (sqrtf(f[0] * f[0] + f[1] * f[1]) > 5.0f && fabsf(f[2]) < 1.0f) ? 1 : 0;
    const bool contact = f[2] > 1.0f;
    const bool first = (air[k] > 0.0f) && contact;
    const float a = air[k] + p.dt;
    air_sum += (a - 0.5f) * (first ? 1.0f : 0.0f);
    air[k] = a * (contact ? 0.0f : 1.0f);
  }
  const float r_stumble = (float)stumble * p.s_stumble;
  const float r_rate = s_rate * p.s_action_rate;
  float r_air = air_sum * p.s_air_time;
  r_air = r_air * (sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) > 0.1f ? 1.0f : 0.0f);
  float hip = 0.f;
  for (int k = 0; k < 4; ++k) {
    const int j = p.hip_dofs[k];
    hip += fabsf(ds[2 * j] - p.default_dof_pos[j]);
  }
  const float r_hip = hip * p.s_hip;
  float rew = r_lin_xy + r_ang_z + r_lin_z + r_ang_xy + r_orient + r_height + r_torque + r_jacc + r_coll + r_rate +
              r_air + r_hip + r_stumble;
  rew = fmaxf(rew, 0.0f);
  float not_timeout;
  if (b.timeout_is_int64) not_timeout = (float)(~((const int64_t*)b.timeout_buf)[e]);
  else not_timeout = ((const uint8_t*)b.timeout_buf)[e] ? 0.0f : 1.0f;
  rew += p.s_termination * ((reset ? 1.0f : 0.0f) * not_timeout);
  b.rew_buf[e] = rew;
  const size_t N = p.num_envs;
  float* es = b.episode_sums;
  es[0 * N + e] += r_lin_xy;
  es[1 * N + e] += r_lin_z;
  es[2 * N + e] += r_ang_z;
  es[3 * N + e] += r_ang_xy;
  es[4 * N + e] += r_orient;
  es[5 * N + e] += r_torque;
  es[6 * N + e] += r_jacc;
  es[7 * N + e] += r_height;
  es[8 * N + e] += r_air;
  es[9 * N + e] += r_coll;
  es[10 * N + e] += r_stumble;
  es[11 * N + e] += r_rate;
  es[12 * N + e] += r_hip;
}

__global__ void k_reset(gt_anymal_params p, gt_anymal_buffers b, const int32_t* __restrict__ ids, int k,
                        const float* __restrict__ off, const float* __restrict__ vel, const float* __restrict__ cx,
                        const float* __restrict__ cy, const float* __restrict__ ch, float* __restrict__ ep) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= k) return;
  const int e = ids[t];
  if (e < 0 || e >= p.num_envs) return;
  const int nd = p.num_dofs;
  float* ds = b.dof_state + (size_t)e * nd * 2;
  for (int j = 0; j < nd; ++j) {
    ds[2 * j] = p.default_dof_pos[j] * off[(size_t)t * nd + j];
    ds[2 * j + 1] = vel[(size_t)t * nd + j];
  }
  float* root = b.root_states + (size_t)e * 13;
  for (int j = 0; j < 13; ++j) root[j] = p.base_init_state[j];
  float* cmd = b.commands + (size_t)e * 4;
  cmd[0] = cx[t];
  cmd[1] = cy[t];
  cmd[3] = ch[t];
  const float m = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) > 0.25f ? 1.0f : 0.0f;
  for (int j = 0; j < 4; ++j) cmd[j] = cmd[j] * m;
  for (int j = 0; j < nd; ++j) {
    b.last_actions[(size_t)e * nd + j] = 0.0f;
    b.last_dof_vel[(size_t)e * nd + j] = 0.0f;
  }
  for (int j = 0; j < 4; ++j) b.feet_air_time[(size_t)e * 4 + j] = 0.0f;
  b.progress_buf[e] = 0;
  b.reset_buf[e] = 1;
  const size_t N = p.num_envs;
  for (int term = 0; term < GT_ANYMAL_NUM_TERMS; ++term) {
    atomicAdd(&ep[term], b.episode_sums[term * N + e]);
    b.episode_sums[term * N + e] = 0.0f;
  }
}

// one thread per observation element: coalesced obs / noise traffic
__global__ void k_post_b(gt_anymal_params p, gt_anymal_buffers b, const float* __restrict__ noise) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int no = p.num_obs;
  if (t >= (long)p.num_envs * no) return;
  const int e = (int)(t / no), k = (int)(t - (long)e * no);
  const int nd = p.num_dofs;
  float v;
  if (k < 3) {
    v = b.base_lin_vel[e * 3 + k] * p.lin_vel_scale;
  } else if (k < 6) {
    v = b.base_ang_vel[e * 3 + k - 3] * p.ang_vel_scale;
  } else if (k < 9) {
    v = b.projected_gravity[e * 3 + k - 6];
  } else if (k < 12) {
    const float sc = k < 11 ? p.lin_vel_scale : p.ang_vel_scale;
    v = b.commands[(size_t)e * 4 + k - 9] * sc;
  } else if (k < 12 + nd) {
    v = b.dof_state[((size_t)e * nd + (k - 12)) * 2] * p.dof_pos_scale;
  } else if (k < 12 + 2 * nd) {
    v = b.dof_state[((size_t)e * nd + (k - 12 - nd)) * 2 + 1] * p.dof_vel_scale;
  } else if (k < no - nd) {
    // plane terrain: measured heights are 0 (anymal_terrain.py:516-517)
    const float h = b.root_states[(size_t)e * 13 + 2] - 0.5f - 0.0f;
    v = fminf(fmaxf(h, -1.0f), 1.0f) * p.height_meas_scale;
  } else {
    v = b.actions[(size_t)e * nd + (k - (no - nd))];
  }
  if (noise) v = v + (2.0f * noise[t] - 1.0f) * b.noise_scale[k];
  b.obs_buf[t] = v;
  if (k < nd) {
    b.last_actions[(size_t)e * nd + k] = b.actions[(size_t)e * nd + k];
    b.last_dof_vel[(size_t)e * nd + k] = b.dof_state[((size_t)e * nd + k) * 2 + 1];
  }
}

int fail(const char* what, hipError_t e) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  g_err = buf;
  return -1;
}
int check_params(const gt_anymal_params* p) {
  if (!p || p->num_envs <= 0 || p->num_dofs <= 0 || p->num_dofs > 16 || p->num_feet > 4 || p->num_knees > 4 ||
      p->num_obs != 36 + 140 + p->num_dofs) {
    g_err = "gt_anymal: invalid parameters";
    return -1;
  }
  return 0;
}
}  // namespace

extern "C" {

int gt_abi_version(void) { return GT_ABI_VERSION; }
const char* gt_last_error(void) { return g_err.c_str(); }

int gt_anymal_post_physics_a(const gt_anymal_params* p, const gt_anymal_buffers* b, void* stream) {
  if (check_params(p)) return -1;
  const int blk = 256;
  hipLaunchKernelGGL(k_post_a, dim3((p->num_envs + blk - 1) / blk), dim3(blk), 0, (hipStream_t)stream, *p, *b);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_post_physics_a", e);
}

int gt_anymal_reset(const gt_anymal_params* p, const gt_anymal_buffers* b, const int32_t* env_ids, int k,
                    const float* pos_offset, const float* dof_vel, const float* cmd_x, const float* cmd_y,
                    const float* cmd_heading, float* episode_out, void* stream) {
  if (check_params(p)) return -1;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(episode_out, 0, sizeof(float) * GT_ANYMAL_NUM_TERMS, st);
  if (e != hipSuccess) return fail("gt_anymal_reset memset", e);
  if (k <= 0) return 0;
  const int blk = 256;
  hipLaunchKernelGGL(k_reset, dim3((k + blk - 1) / blk), dim3(blk), 0, st, *p, *b, env_ids, k, pos_offset, dof_vel,
                     cmd_x, cmd_y, cmd_heading, episode_out);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_reset", e);
}

int gt_anymal_post_physics_b(const gt_anymal_params* p, const gt_anymal_buffers* b, const float* noise,
                             void* stream) {
  if (check_params(p)) return -1;
  const long n = (long)p->num_envs * p->num_obs;
  const int blk = 256;
  hipLaunchKernelGGL(k_post_b, dim3((unsigned)((n + blk - 1) / blk)), dim3(blk), 0, (hipStream_t)stream, *p, *b,
                     noise);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_post_physics_b", e);
}

}  // extern "C"
