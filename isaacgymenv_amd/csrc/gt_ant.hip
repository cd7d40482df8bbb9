// gt_ant.hip -- Ant post-physics tail, fused (include/gymtask.h gt_ant_post_physics).
//
// Replaces the torch statements of ant.py:299-324 (compute_observations) and :326-371
// (compute_ant_reward) that follow the resets of post_physics_step: ~100 elementwise launches
// (quaternion product and rotations, Euler angles, the 60-wide observation, reward terms, done
// mask) become one lane per env.  Built with -ffp-contract=off and written in the reference's
// expression order (torch_jit_utils quat_mul / quat_rotate / get_euler_xyz / normalize), so results
// track the torch path to float rounding (tests/test_ant_tail_gpu.py).  The number of envs the done
// mask flags is published {count, seq} into pinned host memory, so the next step's reset needs no
// nonzero() on steps where nothing is done.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#include "../../include/gymtask.h"
#include "torch_philox.h"

void gt_set_last_error(const char* msg);

namespace {

constexpr float kTwoPi = 6.2831854820251465f;  // float(2*np.pi) as torch casts it for a float32 tensor

// torch.remainder(x, m) for float32 (sign of the divisor)
__device__ __forceinline__ float py_mod(float x, float m) {
  const float r = fmodf(x, m);
  return (r != 0.f && ((r < 0.f) != (m < 0.f))) ? r + m : r;
}

// torch_jit_utils.quat_mul (xyzw), same operation order
__device__ __forceinline__ void quat_mul(const float* a, const float* b, float* o) {
  const float x1 = a[0], y1 = a[1], z1 = a[2], w1 = a[3];
  const float x2 = b[0], y2 = b[1], z2 = b[2], w2 = b[3];
  const float ww = (z1 + x1) * (x2 + y2);
  const float yy = (w1 - y1) * (w2 + z2);
  const float zz = (w1 + y1) * (w2 - z2);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
  o[3] = qq - ww + (z1 - y1) * (y2 - z2);
  o[0] = qq - xx + (x1 + w1) * (x2 + w2);
  o[1] = qq - yy + (w1 - x1) * (y2 + z2);
  o[2] = qq - zz + (z1 + y1) * (w2 - x2);
}

// quat_rotate (sign +1) / quat_rotate_inverse (sign -1): a +- b + c with a = v (2 w^2 - 1),
// b = (u x v) w 2, c = u (u . v) 2
__device__ __forceinline__ void quat_rot(const float* q, const float* v, bool inverse, float* o) {
  const float w = q[3];
  const float s = 2.0f * (w * w) - 1.0f;
  const float cx = q[1] * v[2] - q[2] * v[1];
  const float cy = q[2] * v[0] - q[0] * v[2];
  const float cz = q[0] * v[1] - q[1] * v[0];
  const float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  const float b[3] = {cx * w * 2.0f, cy * w * 2.0f, cz * w * 2.0f};
  const float a[3] = {v[0] * s, v[1] * s, v[2] * s};
  const float c[3] = {q[0] * d * 2.0f, q[1] * d * 2.0f, q[2] * d * 2.0f};
#pragma unroll
  for (int k = 0; k < 3; ++k) o[k] = inverse ? a[k] - b[k] + c[k] : a[k] + b[k] + c[k];
}

__global__ void __launch_bounds__(64) k_ant_tail(gt_ant_params p, gt_ant_buffers b) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  bool done = false;
  if (e < p.num_envs) {
    constexpr int ND = 8;
    const float* rs = b.root_states + (size_t)e * 13;
    const float pos[3] = {rs[0], rs[1], rs[2]};
    const float* tg = b.targets + (size_t)e * 3;
    // to_target with z zeroed, potentials (ant.py:387-391)
    const float tt[3] = {tg[0] - pos[0], tg[1] - pos[1], 0.0f};
    const float prev = b.potentials[e];
    const float tnorm = sqrtf(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
    const float pot = -tnorm / p.dt;
    // compute_heading_and_up (torch_jit_utils.py:248-263)
    const float tn = fmaxf(tnorm, 1e-9f);
    const float tdir[3] = {tt[0] / tn, tt[1] / tn, tt[2] / tn};
    float tq[4];
    quat_mul(rs + 3, b.inv_start_rot + (size_t)e * 4, tq);
    const float vec0[3] = {1.0f, 0.0f, 0.0f}, vec1[3] = {0.0f, 0.0f, 1.0f};
    float up[3], hd[3];
    quat_rot(tq, vec1, false, up);
    quat_rot(tq, vec0, false, hd);
    const float up_proj = up[2];
    const float heading_proj = hd[0] * tdir[0] + hd[1] * tdir[1] + hd[2] * tdir[2];
    // compute_rot (torch_jit_utils.py:266-277): local velocities, roll / yaw, angle to target
    float vl[3], avl[3];
    quat_rot(tq, rs + 7, true, vl);
    quat_rot(tq, rs + 10, true, avl);
    const float x = tq[0], y = tq[1], z = tq[2], w = tq[3];
    const float roll = py_mod(atan2f(2.0f * (w * x + y * z), w * w - x * x - y * y + z * z), kTwoPi);
    const float yaw = py_mod(atan2f(2.0f * (w * z + x * y), w * w + x * x - y * y - z * z), kTwoPi);
    const float walk = atan2f(tg[2] - pos[2], tg[0] - pos[0]);
    // observation (ant.py:400-406)
    float* ob = b.obs_buf + (size_t)e * 60;
    ob[0] = pos[2];
    ob[1] = vl[0]; ob[2] = vl[1]; ob[3] = vl[2];
    ob[4] = avl[0]; ob[5] = avl[1]; ob[6] = avl[2];
    ob[7] = yaw;
    ob[8] = roll;
    ob[9] = walk - yaw;
    ob[10] = up_proj;
    ob[11] = heading_proj;
    const float* ds = b.dof_state + (size_t)e * ND * 2;
    const float* act = b.actions + (size_t)e * ND;
    float dpos[ND], dvel[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float lo = p.dof_lower[j], hi = p.dof_upper[j];
      dpos[j] = (2.0f * ds[2 * j] - hi - lo) / (hi - lo);
      dvel[j] = ds[2 * j + 1] * p.dof_vel_scale;
      ob[12 + j] = dpos[j];
      ob[20 + j] = dvel[j];
      ob[52 + j] = act[j];
    }
    const float* sn = b.sensors + (size_t)e * 24;
#pragma unroll
    for (int k = 0; k < 24; ++k) ob[28 + k] = sn[k] * p.contact_force_scale;
    b.potentials[e] = pot;
    b.prev_potentials[e] = prev;
    float* uv = b.up_vec + (size_t)e * 3;
    float* hv = b.heading_vec + (size_t)e * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) { uv[k] = up[k]; hv[k] = hd[k]; }
    // reward and done mask (ant.py:344-369)
    const float heading_reward = heading_proj > 0.8f ? p.heading_weight : p.heading_weight * heading_proj / 0.8f;
    const float up_reward = up_proj > 0.93f ? 0.0f + p.up_weight : 0.0f;
    float ac = 0.f, el = 0.f;
    long long lim = 0;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      ac += act[j] * act[j];
      el += fabsf(act[j] * dvel[j]);
      lim += dpos[j] > 0.99f ? 1 : 0;
    }
    const float alive = 1.0f * 0.5f;
    const float progress = pot - prev;
    float total = progress + alive + up_reward + heading_reward - p.actions_cost_scale * ac -
                  p.energy_cost_scale * el - (float)lim * p.joints_at_limit_cost_scale;
    const bool fallen = pos[2] < p.termination_height;
    if (fallen) total = 1.0f * p.death_cost;
    b.rew_buf[e] = total;
    long long r = fallen ? 1ll : b.reset_buf[e];
    if ((double)b.progress_buf[e] >= (double)p.max_episode_length - 1.0) r = 1ll;
    b.reset_buf[e] = r;
    b.true_objective[e] = rs[7];
    done = r != 0;
  }
  // done count: one 64-bit atomic per wave {waves done << 32 | count}; the grid's last wave publishes
  // {count, seq} to host memory and re-arms the accumulator (the protocol of gt_anymal_post_physics_a)
  const unsigned long long m = __ballot(done);
  if (b.reset_masks && (threadIdx.x & 63) == 0) b.reset_masks[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = m;
  if ((threadIdx.x & 63) == 0) {
    const unsigned nwaves = (gridDim.x * blockDim.x + 63) / 64;
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(b.reset_count);
    const unsigned long long add = (1ull << 32) | (unsigned long long)__popcll(m);
    const unsigned long long old = atomicAdd(acc, add);
    if ((unsigned)(old >> 32) == nwaves - 1) {
      const int total = (int)((old + add) & 0xffffffffull);
      atomicExch(acc, 0ull);
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
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// reset_idx of the flagged envs (gymtask.h gt_ant_reset_flagged): one lane per env, one wave per workgroup;
// a flagged env's rank among all flagged envs is the exclusive prefix of the earlier waves' ballot popcounts
__global__ void __launch_bounds__(64) k_ant_reset_flagged(gt_ant_params p, gt_ant_buffers b, gt_ant_reset_args r) {
  constexpr int ND = 8;
  const int lane = threadIdx.x, w = blockIdx.x, e = w * 64 + lane;
  int base = 0;
  for (int c = 0; c < w; c += 64) {
    const int i = c + lane;
    base += wave_sum_i(i < w ? (int)__popcll(b.reset_masks[i]) : 0);
  }
  const unsigned long long mine = b.reset_masks[w];
  if (e >= p.num_envs || !((mine >> lane) & 1ull)) return;
  const int t = base + (int)__popcll(mine & ((1ull << lane) - 1ull));
  float* ds = r.dof_state + (size_t)e * ND * 2;
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const size_t q = (size_t)t * ND + j;
    const float up = r.u_pos ? r.u_pos[q] : torch_philox::rand_at(r.plan_pos, q);
    const float uv = r.u_vel ? r.u_vel[q] : torch_philox::rand_at(r.plan_vel, q);
    const float off = r.pos_range * up + r.pos_lower;  // torch_rand_float: (upper - lower) * rand + lower
    const float x = r.initial_dof_pos[(size_t)e * ND + j] + off;
    ds[2 * j] = fmaxf(fminf(x, p.dof_upper[j]), p.dof_lower[j]);  // tensor_clamp = max(min(t, upper), lower)
    ds[2 * j + 1] = r.vel_range * uv + r.vel_lower;
  }
  const float* tg = b.targets + (size_t)e * 3;
  const float* ir = r.initial_root_states + (size_t)e * 13;
  const float px = tg[0] - ir[0], py = tg[1] - ir[1], pz = 0.0f;
  // -torch.norm(planar) / dt: ATen divides by a host scalar as a product with its float reciprocal
  const float prev = -sqrtf(px * px + py * py + pz * pz) * (1.0f / p.dt);
  b.prev_potentials[e] = prev;
  b.potentials[e] = prev;
  r.progress_buf[e] = 0;
  b.reset_buf[e] = 0;
  r.env_ids_out[t] = e;
}

}  // namespace

extern "C" int gt_ant_reset_flagged(const gt_ant_params* p, const gt_ant_buffers* b, int k, const gt_ant_reset_args* r,
                                    void* stream) {
  if (!p || !b || !r || p->num_envs <= 0 || p->num_dofs != 8 || !b->reset_masks || !b->targets || !b->potentials ||
      !b->prev_potentials || !b->reset_buf || !r->initial_dof_pos || !r->initial_root_states || !r->dof_state ||
      !r->progress_buf || !r->env_ids_out || k < 0 || k > p->num_envs ||
      (!r->u_pos && r->plan_pos.numel != (uint32_t)k * 8u) || (!r->u_vel && r->plan_vel.numel != (uint32_t)k * 8u)) {
    gt_set_last_error("gt_ant_reset_flagged: invalid parameters, null buffers or plans that do not cover k x 8");
    return -1;
  }
  if (k == 0) return 0;
  hipLaunchKernelGGL(k_ant_reset_flagged, dim3((p->num_envs + 63) / 64), dim3(64), 0, (hipStream_t)stream, *p, *b, *r);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "gt_ant_reset_flagged: %s", hipGetErrorString(e));
    gt_set_last_error(buf);
    return -1;
  }
  return 0;
}

extern "C" int gt_ant_post_physics(const gt_ant_params* p, const gt_ant_buffers* b, void* stream) {
  if (!p || !b || p->num_envs <= 0 || p->num_dofs != 8 || !b->root_states || !b->dof_state || !b->sensors ||
      !b->actions || !b->targets || !b->inv_start_rot || !b->potentials || !b->prev_potentials || !b->up_vec ||
      !b->heading_vec || !b->obs_buf || !b->rew_buf || !b->reset_buf || !b->progress_buf || !b->true_objective ||
      !b->reset_count) {
    gt_set_last_error("gt_ant_post_physics: invalid parameters or null buffers");
    return -1;
  }
  const int blocks = (p->num_envs + 63) / 64;
  hipLaunchKernelGGL(k_ant_tail, dim3(blocks), dim3(64), 0, (hipStream_t)stream, *p, *b);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "gt_ant_post_physics: %s", hipGetErrorString(e));
    gt_set_last_error(buf);
    return -1;
  }
  return 0;
}
