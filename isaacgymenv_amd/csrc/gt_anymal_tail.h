// gt_anymal_tail.h -- AnymalTerrain / UsefulHound post_physics_step part A for one env (anymal_terrain.py:458-475
// minus the push: counters, base-frame quantities, heading command, check_termination :294-300, compute_reward
// :315-382, episode sums), shared by libgymtask's k_post_a (gt_anymal.hip) and the lane-team physics kernel's
// fused tail (gs_team.hip, gs_pd_args.tail_*): one source, so both produce the same bits.
//
// Every statement mirrors the order of the reference's torch expression, and the functions compile without FMA
// contraction whatever the including library's flags (the pragma in each body), so results track the reference's
// elementwise torch ops to float rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gymtask.h"

struct gt_anymal_hound;

namespace gt_tail {

constexpr float kTwoPi = 6.2831854820251465f;  // float(2*np.pi) as torch casts it for a float32 tensor
constexpr float kPi = 3.1415927410125732f;     // float(np.pi)

// reference quat_rotate_inverse: a - b + c with a = v(2w^2-1), b = 2w (u x v), c = 2u (u.v)
__device__ __forceinline__ void quat_rotate_inverse(const float* q, const float* v, float* o) {
#pragma clang fp contract(off)
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
__device__ __forceinline__ float norm3(const float* v) {
#pragma clang fp contract(off)
  return sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
}

// 16-float rows (nd <= 16) as float4 loads when the row is 16-B aligned (nd % 4 == 0 and the
// tensor base is aligned; the host checks): AoS rows of 48 B per env are otherwise 12 dword
// loads that each touch 64 cache lines per wave.
template <bool VEC, int NC = 0>  // NC > 0: the row length at compile time (no per-vector guards, VEC only)
__device__ __forceinline__ void load_row16(const float* __restrict__ src, int n, float* dst) {
  if (VEC && NC > 0) {
#pragma unroll
    for (int j = 0; j < NC; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(src + j);
      dst[j] = v.x; dst[j + 1] = v.y; dst[j + 2] = v.z; dst[j + 3] = v.w;
    }
  } else if (VEC) {
#pragma unroll
    for (int j = 0; j < 16; j += 4)
      if (j < n) {
        const float4 v = *reinterpret_cast<const float4*>(src + j);
        dst[j] = v.x; dst[j + 1] = v.y; dst[j + 2] = v.z; dst[j + 3] = v.w;
      }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < n) dst[j] = src[j];
  }
}
// dof_state row [nd][2] -> q, qd
template <bool VEC, int NC = 0>
__device__ __forceinline__ void load_dof_row(const float* __restrict__ src, int n, float* q, float* qd) {
  if (VEC && NC > 0) {
#pragma unroll
    for (int j = 0; j < NC; j += 2) {
      const float4 v = *reinterpret_cast<const float4*>(src + 2 * j);
      q[j] = v.x; qd[j] = v.y; q[j + 1] = v.z; qd[j + 1] = v.w;
    }
  } else if (VEC) {
#pragma unroll
    for (int j = 0; j < 16; j += 2)
      if (j < n) {
        const float4 v = *reinterpret_cast<const float4*>(src + 2 * j);
        q[j] = v.x; qd[j] = v.y; q[j + 1] = v.z; qd[j + 1] = v.w;
      }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < n) { q[j] = src[2 * j]; qd[j] = src[2 * j + 1]; }
  }
}

constexpr int kMaxActions = 20;  // UsefulHound: 18

// One env: every input is loaded first (one memory round trip), then computed, then stored:
// the buffers may alias as far as the compiler knows, so interleaved loads and stores would
// serialise into one round trip per statement group.  HOUND: UsefulHound's tail (gymtask.h,
// gt_anymal_hound; useful_hound.py:467-567).
// NDC: num_dofs at compile time (0: runtime).  With it (and VEC) every load of the env is unconditional straight-
// line code: guarded loads put the compiler's conservative vmcnt waits at each branch join, one memory round trip
// per group (23 waits in the runtime-nd form); here the knee / foot rows of unused slots read the base row instead
// and are never used.
template <bool VEC, bool HOUND, int NDC = 0>
__device__ __forceinline__ bool post_a_env(const gt_anymal_params& p, const gt_anymal_buffers& b,
                                           const gt_anymal_hound& h, const int e) {
#pragma clang fp contract(off)
  static_assert(NDC == 0 || (VEC && !HOUND && NDC % 4 == 0 && NDC <= 16), "compile-time rows: AnymalTerrain, VEC");
  const int nd = NDC > 0 ? NDC : p.num_dofs, nb = p.num_bodies;
  const int na = HOUND ? h.num_actions : nd;  // torques / actions width and dof_state row width
  const size_t N = p.num_envs;
  // ---- loads
  const int64_t prog = b.progress_buf[e] + 1;
  const int64_t rnd = b.randomize_buf[e] + 1;
  float root[13];
#pragma unroll
  for (int k = 0; k < 13; ++k) root[k] = b.root_states[(size_t)e * 13 + k];
  float cmd[4], air[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    cmd[k] = b.commands[(size_t)e * 4 + k];
    air[k] = b.feet_air_time[(size_t)e * 4 + k];
  }
  const float* cf = b.contact_forces + (size_t)e * nb * 3;
  float fbase[3], fknee[4][3], ffoot[4][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) fbase[c] = cf[3 * p.base_index + c];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (NDC > 0) {  // (slots past num_knees / num_feet are never read below)
        fknee[k][c] = cf[3 * (k < p.num_knees ? p.knee_idx[k] : p.base_index) + c];
        ffoot[k][c] = cf[3 * (k < p.num_feet ? p.feet_idx[k] : p.base_index) + c];
      } else {
        fknee[k][c] = k < p.num_knees ? cf[3 * p.knee_idx[k] + c] : 0.0f;
        ffoot[k][c] = k < p.num_feet ? cf[3 * p.feet_idx[k] + c] : 0.0f;
      }
    }
  float fsh[4][3];
  if constexpr (HOUND) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) fsh[k][c] = k < h.num_shoulders ? cf[3 * h.shoulder_idx[k] + c] : 0.0f;
  }
  float tq[kMaxActions], act[kMaxActions], lact[kMaxActions], lqd[16], dq[16], dqd[16];
  if constexpr (HOUND) {
#pragma unroll
    for (int j = 0; j < kMaxActions; ++j)
      if (j < na) {
        tq[j] = b.torques[(size_t)e * na + j];
        act[j] = b.actions[(size_t)e * na + j];
        lact[j] = b.last_actions[(size_t)e * na + j];
      }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < nd) {
        lqd[j] = b.last_dof_vel[(size_t)e * nd + j];
        dq[j] = b.dof_state[((size_t)e * na + j) * 2];
        dqd[j] = b.dof_state[((size_t)e * na + j) * 2 + 1];
      }
  } else {
    load_row16<VEC, NDC>(b.torques + (size_t)e * nd, nd, tq);
    load_row16<VEC, NDC>(b.actions + (size_t)e * nd, nd, act);
    load_row16<VEC, NDC>(b.last_actions + (size_t)e * nd, nd, lact);
    load_row16<VEC, NDC>(b.last_dof_vel + (size_t)e * nd, nd, lqd);
    load_dof_row<VEC, NDC>(b.dof_state + (size_t)e * nd * 2, nd, dq, dqd);
  }
  float not_timeout;
  if (NDC > 0) {
    // one unconditional byte load: the int64 buffer (VecTask's initial zeros, the first step only) holds 0 / 1,
    // whose low byte is the value (little-endian)
    const uint8_t lo = ((const uint8_t*)b.timeout_buf)[b.timeout_is_int64 ? 8 * (size_t)e : (size_t)e];
    not_timeout = b.timeout_is_int64 ? (float)(~(int64_t)lo) : (lo ? 0.0f : 1.0f);
  } else if (b.timeout_is_int64) {
    not_timeout = (float)(~((const int64_t*)b.timeout_buf)[e]);
  } else {
    not_timeout = ((const uint8_t*)b.timeout_buf)[e] ? 0.0f : 1.0f;
  }
  float sums[GT_ANYMAL_NUM_TERMS];
#pragma unroll
  for (int t = 0; t < GT_ANYMAL_NUM_TERMS; ++t) sums[t] = b.episode_sums[t * N + e];

  // ---- base-frame quantities (anymal_terrain.py:461-463)
  const float q[4] = {root[3], root[4], root[5], root[6]};
  float blv[3], bav[3], pg[3];
  quat_rotate_inverse(q, root + 7, blv);
  quat_rotate_inverse(q, root + 10, bav);
  const float gv[3] = {0.0f, 0.0f, -1.0f};
  quat_rotate_inverse(q, gv, pg);
  // heading: quat_apply(q, (1,0,0)) -> t = 2 u x f ; f + w t + u x t
  const float tx = (q[1] * 0.0f - q[2] * 0.0f) * 2.0f;
  const float ty = (q[2] * 1.0f - q[0] * 0.0f) * 2.0f;
  const float tz = (q[0] * 0.0f - q[1] * 1.0f) * 2.0f;
  const float fx = (1.0f + q[3] * tx) + (q[1] * tz - q[2] * ty);
  const float fy = (0.0f + q[3] * ty) + (q[2] * tx - q[0] * tz);
  const float heading = atan2f(fy, fx);
  // wrap_to_pi (anymal_terrain.py:684-687) is TorchScript: `%=` there is C fmod, not a floored
  // remainder, so negative angles stay negative (pinned by tests/golden/anymal_terrain.npz)
  float ang = fmodf(cmd[3] - heading, kTwoPi);
  ang = ang - kTwoPi * (ang > kPi ? 1.0f : 0.0f);
  const float c2 = fminf(fmaxf(0.5f * ang, -1.0f), 1.0f);

  // ---- check_termination (:294-300)
  bool reset = norm3(fbase) > 1.0f;
  int knee_count = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) knee_count += (k < p.num_knees && norm3(fknee[k]) > 1.0f) ? 1 : 0;
  int sh_count = 0;
  if constexpr (HOUND) {
    // useful_hound.py:467-480: thigh and shoulder contacts terminate, allowKneeContacts is not read
#pragma unroll
    for (int k = 0; k < 4; ++k) sh_count += (k < h.num_shoulders && norm3(fsh[k]) > 1.0f) ? 1 : 0;
    if (knee_count > 0 || sh_count > 0) reset = true;
  } else {
    if (!p.allow_knee_contacts && knee_count > 0) reset = true;
  }
  if (prog >= p.max_episode_length - 1) reset = true;

  // ---- compute_reward (:315-382, reference order)
  const float lin_err = sq(cmd[0] - blv[0]) + sq(cmd[1] - blv[1]);
  const float ang_err = sq(c2 - bav[2]);
  const float r_lin_xy = expf(-lin_err / 0.25f) * p.s_lin_vel_xy;
  const float r_ang_z = expf(-ang_err / 0.25f) * p.s_ang_vel_z;
  const float r_lin_z = sq(blv[2]) * p.s_lin_vel_z;
  const float r_ang_xy = (sq(bav[0]) + sq(bav[1])) * p.s_ang_vel_xy;
  const float r_orient = (sq(pg[0]) + sq(pg[1])) * p.s_orient;
  const float r_height = sq(root[2] - 0.52f) * p.s_base_height;
  float s_tq = 0.f, s_acc = 0.f, s_rate = 0.f;
#pragma unroll
  for (int j = 0; j < kMaxActions; ++j) {
    if (j < na) {
      s_tq += sq(tq[j]);
      s_rate += sq(lact[j] - act[j]);
    }
    if (j < 16 && j < nd) s_acc += sq(lqd[j] - dqd[j]);
  }
  const float r_torque = s_tq * p.s_torque;
  const float r_jacc = s_acc * p.s_joint_acc;
  const float r_coll = HOUND ? (float)knee_count * p.s_collision + (float)sh_count * p.s_collision
                             : (float)knee_count * p.s_collision;
  int stumble = 0;
  float air_sum = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < p.num_feet) {
      const float* f = ffoot[k];
      stumble += (sqrtf(f[0] * f[0] + f[1] * f[1]) > 5.0f && fabsf(f[2]) < 1.0f) ? 1 : 0;
      const bool contact = f[2] > 1.0f;
      const bool first = (air[k] > 0.0f) && contact;
      const float a = air[k] + p.dt;
      air_sum += (a - 0.5f) * (first ? 1.0f : 0.0f);
      air[k] = a * (contact ? 0.0f : 1.0f);
    }
  }
  const float r_stumble = (float)stumble * p.s_stumble;
  const float r_rate = s_rate * p.s_action_rate;
  float r_air = air_sum * p.s_air_time;
  r_air = r_air * (sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) > 0.1f ? 1.0f : 0.0f);
  float hip = 0.f;
  // hip dofs are 0, 3, 6, 9 (anymal_terrain.py:378); constant indices keep dq in registers
#pragma unroll
  for (int k = 0; k < 4; ++k) hip += fabsf(dq[3 * k] - p.default_dof_pos[3 * k]);
  const float r_hip = hip * p.s_hip;
  float rew = r_lin_xy + r_ang_z + r_lin_z + r_ang_xy + r_orient + r_height + r_torque + r_jacc + r_coll + r_rate +
              r_air + r_hip + r_stumble;
  rew = fmaxf(rew, 0.0f);
  rew += p.s_termination * ((reset ? 1.0f : 0.0f) * not_timeout);
  const float terms[GT_ANYMAL_NUM_TERMS] = {r_lin_xy, r_lin_z,  r_ang_z,    r_ang_xy, r_orient, r_torque, r_jacc,
                                            r_height, r_air,    r_coll,     r_stumble, r_rate,  r_hip};

  // ---- stores
  b.progress_buf[e] = prog;
  b.randomize_buf[e] = rnd;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    b.base_lin_vel[e * 3 + k] = blv[k];
    b.base_ang_vel[e * 3 + k] = bav[k];
    b.projected_gravity[e * 3 + k] = pg[k];
  }
  b.commands[(size_t)e * 4 + 2] = c2;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < p.num_feet) b.feet_air_time[(size_t)e * 4 + k] = air[k];
  b.reset_buf[e] = reset ? 1 : 0;
  b.rew_buf[e] = rew;
#pragma unroll
  for (int t = 0; t < GT_ANYMAL_NUM_TERMS; ++t) b.episode_sums[t * N + e] = sums[t] + terms[t];
  return reset;
}

// The done count of one wave (popc envs flagged) joins the launch's total: one 64-bit atomic per wave carries
// {waves done << 32 | count}; the wave that completes the grid (nwaves waves) publishes the total (device word
// reset_count[2], and {count, seq} into host memory for the host's spin wait) and re-arms the accumulator.
// Called by one lane per wave.
__device__ __forceinline__ void publish_count(const gt_anymal_buffers& b, unsigned popc, unsigned nwaves) {
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(b.reset_count);
  const unsigned long long add = (1ull << 32) | (unsigned long long)popc;
  const unsigned long long old = atomicAdd(acc, add);
  if ((unsigned)(old >> 32) == nwaves - 1) {
    const int total = (int)((old + add) & 0xffffffffull);
    *acc = 0ull;
    b.reset_count[2] = total;
    if (b.host_count) {
      // {count, seq} as ONE 8-byte store: the host reads only this word, so no release fence
      // (a system-scope release writes back the whole L2, microseconds at the end of the tail)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(b.host_count),
                         ((unsigned long long)(uint32_t)b.seq << 32) | (uint32_t)total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace gt_tail
