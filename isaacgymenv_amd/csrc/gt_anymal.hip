// gt_anymal.hip -- fused AnymalTerrain post-physics kernels + the libgymtask C ABI
// (include/gymtask.h).
//
// Built with -ffp-contract=off: every statement mirrors the order of the
// reference's torch expression (anymal_terrain.py:315-382, torch_jit_utils.py:94-103)
// so results track the reference's elementwise torch ops to float rounding.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <cstdio>
#include <string>
#include <thread>

#include "../../include/gymtask.h"
#include "torch_philox.h"
#include "gt_anymal_tail.h"

// k_reset_flagged's episode-sum hand-off depends on gfx950's L2-served agent-scope atomics (see there)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "gt_anymal.hip targets gfx950 only (the k_reset_flagged hand-off ordering is gfx950's)"
#endif

namespace {
thread_local std::string g_err;

using namespace gt_tail;


// One lane per env, one wave per workgroup (4096 envs -> 64 workgroups on 64 CUs: the tail is
// latency bound, so spreading it over CUs beats packing 4 waves per CU).
template <bool VEC, bool HOUND, int NDC = 0>
__global__ void __launch_bounds__(64) k_post_a(gt_anymal_params p, gt_anymal_buffers b, gt_anymal_hound h) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  bool reset = false;
  if (e < p.num_envs) reset = post_a_env<VEC, HOUND, NDC>(p, b, h, e);
  // reset count (gt_tail::publish_count) and this wave's 64-bit mask of flagged envs (k_reset_flagged ranks them)
  const unsigned long long m = __ballot(reset);
  if ((threadIdx.x & 63) == 0) {
    if (b.reset_masks) b.reset_masks[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = m;
    publish_count(b, (unsigned)__popcll(m), (gridDim.x * blockDim.x + 63) / 64);
  }
}

__global__ void k_reset(gt_anymal_params p, gt_anymal_buffers b, const int32_t* __restrict__ ids, int k,
                        const float* __restrict__ off, const float* __restrict__ vel, const float* __restrict__ cx,
                        const float* __restrict__ cy, const float* __restrict__ ch) {
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
  // the episode sums were summed by k_episode_sums (launched before this kernel)
  for (int term = 0; term < GT_ANYMAL_NUM_TERMS; ++term) b.episode_sums[term * N + e] = 0.0f;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ep[term] = sum over t of episode_sums[term][ids[t]] in a FIXED order (extras["episode"] must not
// depend on how waves were scheduled): one wave per term, lane l sums t = l, l + 64, ... in order,
// then the butterfly reduction (itself a fixed order).
__global__ void __launch_bounds__(64 * GT_ANYMAL_NUM_TERMS) k_episode_sums(gt_anymal_params p,
                                                                          const float* __restrict__ sums,
                                                                          const int32_t* __restrict__ ids, int k,
                                                                          float* __restrict__ ep) {
  const int term = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t N = p.num_envs;
  float v = 0.0f;
  for (int t = lane; t < k; t += 64) {
    const int e = ids[t];
    if (e >= 0 && e < p.num_envs) v += sums[term * N + e];
  }
  v = wave_sum(v);
  if (lane == 0) ep[term] = v;
}

// reset_idx for the envs post_a flagged (anymal_terrain.py:384-425, plane terrain).  One lane
// per env, one wave per workgroup; the rank of a flagged env among all flagged envs comes from
// post_a's per-wave ballots (exclusive prefix of popcounts), so no compaction pass is needed.
template <bool HOUND>
__global__ void __launch_bounds__(64) k_reset_flagged(gt_anymal_params p, gt_anymal_buffers b, gt_anymal_hound h,
                                                      int k, gt_anymal_reset_draws d, gt_anymal_terrain_reset tr,
                                                      bool has_terrain, int32_t* __restrict__ ids_out,
                                                      float* __restrict__ ep_out, float len_s,
                                                      float* __restrict__ partial, unsigned* __restrict__ done) {
  const int lane = threadIdx.x;
  const int w = blockIdx.x;
  const int e = w * 64 + lane;
  int base = 0;
  for (int c = 0; c < w; c += 64) {
    const int i = c + lane;
    base += wave_sum(i < w ? (int)__popcll(b.reset_masks[i]) : 0);
  }
  const unsigned long long mine = b.reset_masks[w];
  const bool flagged = (mine >> lane) & 1ull;
  const int nd = p.num_dofs;
  const int na = HOUND ? h.num_actions : nd;
  const size_t N = p.num_envs;
  // The wave's draws (2*nd + 3 per flagged env) are evaluated by all 64 lanes and exchanged
  // through LDS: one Philox chain per lane instead of 2*nd + 3 serial ones per flagged lane.
  constexpr int kMaxDraws = 2 * 16 + 3 + 2 + (HOUND ? 6 : 0);
  __shared__ float u_lds[64 * kMaxDraws];
  const int m = (int)__popcll(mine);
  const int DT = 2 * nd + 3 + (has_terrain ? 2 : 0);  // pos | vel | cmd x, y, heading | root x, y
  const int D = DT + (HOUND ? 6 : 0);                  // | arm (UsefulHound)
  for (int s = lane; s < m * D; s += 64) {
    const int r = s / D, c = s - (s / D) * D;
    const int t = base + r;
    float u;
    if (c < nd) u = d.u_pos ? d.u_pos[(size_t)t * nd + c] : torch_philox::rand_at(d.plan_pos, (size_t)t * nd + c);
    else if (c < 2 * nd) {
      const size_t q = (size_t)t * nd + (c - nd);
      u = d.u_vel ? d.u_vel[q] : torch_philox::rand_at(d.plan_vel, q);
    } else if (c == 2 * nd) u = d.u_cmd_x ? d.u_cmd_x[t] : torch_philox::rand_at(d.plan_cmd_x, t);
    else if (c == 2 * nd + 1) u = d.u_cmd_y ? d.u_cmd_y[t] : torch_philox::rand_at(d.plan_cmd_y, t);
    else if (c == 2 * nd + 2) u = d.u_cmd_h ? d.u_cmd_h[t] : torch_philox::rand_at(d.plan_cmd_h, t);
    else if (c < DT) {
      const size_t q = (size_t)t * 2 + (c - 2 * nd - 3);
      u = tr.u_root_xy ? tr.u_root_xy[q] : torch_philox::rand_at(tr.plan_root_xy, q);
    } else {
      const size_t q = (size_t)t * 6 + (c - DT);
      u = h.u_arm ? h.u_arm[q] : torch_philox::rand_at(h.plan_arm, q);
    }
    u_lds[s] = u;
  }
  __syncthreads();
  float term[GT_ANYMAL_NUM_TERMS];
#pragma unroll
  for (int i = 0; i < GT_ANYMAL_NUM_TERMS; ++i) term[i] = 0.0f;
  if (flagged) {
    const int r = (int)__popcll(mine & ((1ull << lane) - 1ull));
    const int t = base + r;
    const float* u = u_lds + r * D;
    float* ds = b.dof_state + (size_t)e * na * 2;
    for (int j = 0; j < nd; ++j) {
      const float off = d.pos_range * u[j] + d.pos_lower;
      const float vel = d.vel_range * u[nd + j] + d.vel_lower;
      ds[2 * j] = p.default_dof_pos[j] * off;
      ds[2 * j + 1] = vel;
    }
    if constexpr (HOUND) {
      // useful_hound.py:592-601: tensor_clamp(default + noise * 2.0 * (u - 0.5), lower, upper)
      for (int j = 0; j < 6; ++j) {
        const float x = h.arm_default[j] + (u[DT + j] - 0.5f) * h.arm_noise2;
        const float q = fmaxf(fminf(x, h.arm_upper[j]), h.arm_lower[j]);
        ds[2 * (nd + j)] = q;
        ds[2 * (nd + j) + 1] = 0.0f;
        h.pos_control[(size_t)e * 6 + j] = q;
        h.effort_control[(size_t)e * 6 + j] = 0.0f;
      }
    }
    float* root = b.root_states + (size_t)e * 13;
    if (has_terrain) {
      // update_terrain_level (:427-435) on the state BEFORE the reset, then the origin of the new level
      long long lvl = tr.terrain_levels[e];
      if (tr.update_levels) {
        const float dx = root[0] - tr.env_origins[(size_t)e * 3 + 0];
        const float dy = root[1] - tr.env_origins[(size_t)e * 3 + 1];
        const float dist = sqrtf(dx * dx + dy * dy);
        const float c0 = b.commands[(size_t)e * 4 + 0], c1 = b.commands[(size_t)e * 4 + 1];
        const float cn = sqrtf(c0 * c0 + c1 * c1);
        lvl -= (dist < cn * tr.max_episode_length_s * 0.25f) ? 1 : 0;
        lvl += (dist > tr.env_length / 2.0f) ? 1 : 0;
        lvl = (lvl < 0 ? 0 : lvl) % tr.env_rows;
        tr.terrain_levels[e] = lvl;
        const long long ty = tr.terrain_types[e];
        for (int j = 0; j < 3; ++j)
          tr.env_origins[(size_t)e * 3 + j] = tr.terrain_origins[((size_t)lvl * tr.env_cols + ty) * 3 + j];
      }
      float o[3];
      for (int j = 0; j < 3; ++j) o[j] = tr.env_origins[(size_t)e * 3 + j];
      for (int j = 0; j < 13; ++j) root[j] = p.base_init_state[j];
      for (int j = 0; j < 3; ++j) root[j] = root[j] + o[j];
      root[0] = root[0] + (tr.xy_range * u[2 * nd + 3] + tr.xy_lower);
      root[1] = root[1] + (tr.xy_range * u[2 * nd + 4] + tr.xy_lower);
    } else {
      for (int j = 0; j < 13; ++j) root[j] = p.base_init_state[j];
    }
    float cmd[4];
    const float ux = u[2 * nd], uy = u[2 * nd + 1], uh = u[2 * nd + 2];
    cmd[0] = d.cmd_x_range * ux + d.cmd_x_lower;
    cmd[1] = d.cmd_y_range * uy + d.cmd_y_lower;
    cmd[2] = b.commands[(size_t)e * 4 + 2];
    cmd[3] = d.cmd_h_range * uh + d.cmd_h_lower;
    const float m = sqrtf(cmd[0] * cmd[0] + cmd[1] * cmd[1]) > 0.25f ? 1.0f : 0.0f;
    for (int j = 0; j < 4; ++j) b.commands[(size_t)e * 4 + j] = cmd[j] * m;
    for (int j = 0; j < na; ++j) b.last_actions[(size_t)e * na + j] = 0.0f;
    for (int j = 0; j < nd; ++j) b.last_dof_vel[(size_t)e * nd + j] = 0.0f;
    for (int j = 0; j < 4; ++j) b.feet_air_time[(size_t)e * 4 + j] = 0.0f;
    b.progress_buf[e] = 0;
    b.reset_buf[e] = 1;
#pragma unroll
    for (int i = 0; i < GT_ANYMAL_NUM_TERMS; ++i) {
      term[i] = b.episode_sums[i * N + e];
      b.episode_sums[i * N + e] = 0.0f;
    }
    ids_out[t] = e;
  }
  // Episode means, deterministic: every wave publishes its 13 wave sums (zeros when nothing was
  // flagged) to its own slot of `partial`; the last wave to finish adds the slots in wave order.
  // Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table): the
  // slots are stored and loaded sc1 (relaxed agent-scope atomics, L2-served, so no L1 staleness),
  // each wave waits for its own stores before ONE lane adds to the unsharded counter, and the wave
  // whose add returned last loads.  No __threadfence(): two of those per wave (~3.5 us each) were
  // most of this kernel's time.
  // The ordering this hand-off relies on is gfx950's (agent-scope relaxed atomics are served by L2, the one
  // coherence point of the agent; vmcnt(0) retires this wave's stores there before its counter add; the last
  // wave's loads read L2): under the scoped C++ model a release on the add and an acquire in the last wave would be
  // needed, at the cost of the cache write-back / invalidate above.  The build is gfx950-only (the #error below).
  // slot NT (terrain): the wave's sum of terrain levels after the update, for mean(terrain_levels)
  constexpr int NT = GT_ANYMAL_NUM_TERMS + 1;
#pragma unroll
  for (int i = 0; i < GT_ANYMAL_NUM_TERMS; ++i) {
    const float s = mine ? wave_sum(term[i]) : 0.0f;
    if (lane == i) __hip_atomic_store(&partial[(size_t)w * NT + i], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (has_terrain) {
    // integer levels: the float sums are exact in any order (< 2^24)
    const float lv = wave_sum(e < p.num_envs ? (float)tr.terrain_levels[e] : 0.0f);
    if (lane == 0)
      __hip_atomic_store(&partial[(size_t)w * NT + GT_ANYMAL_NUM_TERMS], lv, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old == gridDim.x - 1) {  // last wave: finalise the 13 terms in parallel lanes
    // The slots are staged through LDS 64 waves at a time, every lane issuing its NT loads at
    // once; lane `term` then adds its column in wave order from LDS (the order of the sum is
    // fixed, so extras["episode"] does not depend on wave scheduling).
    static_assert(NT <= kMaxDraws, "partial staging reuses u_lds");
    float v = 0.0f;
    for (int q0 = 0; q0 < (int)gridDim.x; q0 += 64) {
      const int nq = min(64, (int)gridDim.x - q0);
      float r[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int s = lane + 64 * i;
        r[i] = s < nq * NT ? __hip_atomic_load(&partial[(size_t)q0 * NT + s], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0f;
      }
      __syncthreads();  // u_lds (draws, or the previous chunk) is no longer read
#pragma unroll
      for (int i = 0; i < NT; ++i) u_lds[lane + 64 * i] = r[i];
      __syncthreads();
      if (lane < NT)
        for (int q = 0; q < nq; ++q) v += u_lds[q * NT + lane];
    }
    if (lane < GT_ANYMAL_NUM_TERMS + (has_terrain ? 1 : 0)) {
      if (lane < GT_ANYMAL_NUM_TERMS)
        // torch.mean(sums[env_ids]) / max_episode_length_s: mean = sum * (1/k), / scalar = * (1/scalar)
        ep_out[lane] = (v * (1.0f / (float)k)) * (1.0f / len_s);
      else
        ep_out[lane] = v * (1.0f / (float)p.num_envs);  // torch.mean(terrain_levels.float())
    }
    if (lane == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One workgroup per env, one lane per observation element (compute_observations, :302-313).
// Each lane selects its source address and scale first and then issues ONE load, so the
// ragged segments of the obs row do not serialise into one memory round trip per segment.
template <int NOISE, bool HOUND>  // NOISE: 0 none, 1 drawn buffer, 2 in-kernel torch.rand stream
__device__ __forceinline__ void post_b_elem(const gt_anymal_params& p, const gt_anymal_buffers& b,
                                            const gt_anymal_hound& h, const float* __restrict__ noise,
                                            const gt_torch_rand_plan& plan, const int e, const int k) {
  const int no = p.num_obs;
  const int nd = p.num_dofs;
  const int na = HOUND ? h.num_actions : nd;    // actions width, dof_state row width
  const int ne = HOUND ? 10 : 0;                // end-effector position, quaternion, arm command
  const int nh = no - 12 - 2 * nd - na - ne;    // height probes (140)
  const size_t t = (size_t)e * no + k;
  // side outputs: last_actions / last_dof_vel (:484-485) and VecTask's time_outs (vec_task.py:394)
  float la = 0.0f, lq = 0.0f;
  if (k < na) la = b.actions[(size_t)e * na + k];
  if (k < nd) lq = b.dof_state[((size_t)e * na + k) * 2 + 1];
  int64_t prog = 0;
  uint8_t rst = 0;
  if (k == 0 && b.time_outs) {
    prog = b.progress_buf[e];
    rst = b.reset_buf[e];
  }
  const float* src;
  float sc = 1.0f;
  bool height = false;
  if (k < 3) {
    src = b.base_lin_vel + e * 3 + k; sc = p.lin_vel_scale;
  } else if (k < 6) {
    src = b.base_ang_vel + e * 3 + k - 3; sc = p.ang_vel_scale;
  } else if (k < 9) {
    src = b.projected_gravity + e * 3 + k - 6;
  } else if (k < 12) {
    src = b.commands + (size_t)e * 4 + k - 9; sc = k < 11 ? p.lin_vel_scale : p.ang_vel_scale;
  } else if (k < 12 + nd) {
    src = b.dof_state + ((size_t)e * na + (k - 12)) * 2; sc = p.dof_pos_scale;
  } else if (k < 12 + 2 * nd) {
    src = b.dof_state + ((size_t)e * na + (k - 12 - nd)) * 2 + 1; sc = p.dof_vel_scale;
  } else if (k < 12 + 2 * nd + nh) {
    // the base height; the probe's terrain height is subtracted below
    src = b.root_states + (size_t)e * 13 + 2; height = true;
  } else if (k < 12 + 2 * nd + nh + na) {
    src = b.actions + (size_t)e * na + (k - (12 + 2 * nd + nh));
  } else if (k < no - 3) {  // UsefulHound: end-effector position | quaternion (useful_hound.py:492-493)
    src = h.eef_state + (size_t)e * h.eef_stride + (k - (no - ne));
  } else {
    src = h.arm_commands + (size_t)e * 3 + (k - (no - 3));
  }
  const float x = *src;
  const float nz = NOISE == 1 ? noise[t] : NOISE == 2 ? torch_philox::rand_at(plan, t) : 0.0f;
  const float ns = b.noise_scale[k];
  float v;
  if (height) {
    // clip(z - 0.5 - measured_height, -1, 1) * scale (:303-304); plane terrain: heights are 0
    const float mh = b.measured_heights ? b.measured_heights[(size_t)e * nh + (k - 12 - 2 * nd)] : 0.0f;
    v = fminf(fmaxf(x - 0.5f - mh, -1.0f), 1.0f) * p.height_meas_scale;
  }
  else if (k < 12 + 2 * nd && !(k >= 6 && k < 9)) v = x * sc;
  else v = x;
  if (NOISE) v = v + (2.0f * nz - 1.0f) * ns;
  b.obs_buf[t] = v;
  if (b.obs_out) {
    const float c = fminf(fmaxf(v, -b.clip_obs), b.clip_obs);
    b.obs_out[t] = c;
    if (b.obs_mirror) b.obs_mirror[t] = c;
  }
  if (k == 0 && b.time_outs) b.time_outs[e] = (prog >= p.max_episode_length - 1) && (rst != 0);
  if (k < na) b.last_actions[(size_t)e * na + k] = la;
  if (k < nd) b.last_dof_vel[(size_t)e * nd + k] = lq;
}

template <int NOISE, bool HOUND>
__global__ void __launch_bounds__(256) k_post_b(gt_anymal_params p, gt_anymal_buffers b, gt_anymal_hound h,
                                                const float* __restrict__ noise, gt_torch_rand_plan plan) {
  const int k = threadIdx.x;
  if (k < p.num_obs) post_b_elem<NOISE, HOUND>(p, b, h, noise, plan, blockIdx.x, k);
}

// post_a + post_b in one launch (gt_anymal_post_physics_ab; AnymalTerrain, 12 dofs, plane): a workgroup of 256
// lanes takes 16 envs; lanes 0-15 run post_a_env for them (the same source as k_post_a), publish their 16 done bits
// as a slice of the 64-env mask word and join the grid's count, then -- after a workgroup barrier, so post_a's
// stores of these envs are visible -- all 256 lanes run the 16 x num_obs observation elements (k_post_b's body).
// Each workgroup moves on to its observations as soon as its own envs' part A is done, without a launch boundary
// and without waiting for the rest of the grid.
constexpr int kAbEnvs = 16;
// (called, not inlined, in k_post_ab's element loop: inlining it there crashes this compiler's loop passes)
template <int NOISE>
__device__ __attribute__((noinline)) void post_b_elem_call(const gt_anymal_params& p, const gt_anymal_buffers& b,
                                                           const float* __restrict__ noise,
                                                           const gt_torch_rand_plan& plan, const int e, const int k) {
  post_b_elem<NOISE, false>(p, b, gt_anymal_hound{}, noise, plan, e, k);
}
template <int NOISE>
__global__ void __launch_bounds__(256) k_post_ab(gt_anymal_params p, gt_anymal_buffers b,
                                                 const float* __restrict__ noise, gt_torch_rand_plan plan) {
  const gt_anymal_hound h{};
  const int tid = threadIdx.x, e0 = blockIdx.x * kAbEnvs, N = p.num_envs;
  bool reset = false;
  if (tid < kAbEnvs && e0 + tid < N) reset = post_a_env<true, false, 12>(p, b, h, e0 + tid);
  const unsigned long long m = __ballot(reset);  // (wave 0: lanes 0-15 hold the envs)
  if (tid == 0) {
    uint16_t* slices = reinterpret_cast<uint16_t*>(b.reset_masks);
    slices[e0 / kAbEnvs] = (uint16_t)(m & 0xffffull);
    if (e0 + kAbEnvs >= N)  // the last workgroup clears its mask word's slices past the last env
      for (int q = e0 / kAbEnvs + 1; q % 4 != 0; ++q) slices[q] = 0;
    publish_count(b, (unsigned)__popcll(m & 0xffffull), gridDim.x);
  }
  __syncthreads();
  const int no = p.num_obs, ne = (N - e0 < kAbEnvs ? N - e0 : kAbEnvs);
  for (int i = tid; i < ne * no; i += blockDim.x) post_b_elem_call<NOISE>(p, b, noise, plan, e0 + i / no, i % no);
}

// get_heights, one lane per (env, probe).  The statement order follows the reference's torch
// expressions (normalize of the yaw-only quaternion, quat_apply = v + w t + q x t with t = 2 q x v,
// + root position, + border, / hs, truncation) and the library is built without FMA contraction,
// so the cell index matches the eager torch computation except on exact ties.
__global__ void __launch_bounds__(256) k_measure_heights(const int16_t* __restrict__ hf, int rows, int cols,
                                                         float border, float hs, float vs,
                                                         const float* __restrict__ root,
                                                         const float* __restrict__ pts, int N, int np_,
                                                         float* __restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)N * np_) return;
  const int e = (int)(t / np_);
  const float* r = root + (size_t)e * 13;
  const float qz = r[5], qw = r[6];
  const float nrm = fmaxf(sqrtf(qz * qz + qw * qw), 1e-9f);
  const float z = qz / nrm, w = qw / nrm;  // yaw-only quaternion (0, 0, z, w)
  const float* pv = pts + (size_t)t * 3;
  const float vx = pv[0], vy = pv[1], vz = pv[2];
  // t = 2 * (q x v) with q = (0, 0, z): (-z vy, z vx, 0)
  const float tx = (0.0f * vz - z * vy) * 2.0f;
  const float ty = (z * vx - 0.0f * vz) * 2.0f;
  const float tz = (0.0f * vy - 0.0f * vx) * 2.0f;
  // q x t
  const float cx = 0.0f * tz - z * ty;
  const float cy = z * tx - 0.0f * tz;
  float px = vx + w * tx + cx + r[0];
  float py = vy + w * ty + cy + r[1];
  (void)tz;
  px += border;
  py += border;
  // torch on the GPU divides by a host scalar as a multiplication by its float reciprocal
  // (ATen div_true with a CPU scalar): (pts / hs).long() is trunc(p * (1 / hs))
  const float inv_hs = 1.0f / hs;
  long ix = (long)(px * inv_hs), iy = (long)(py * inv_hs);
  ix = ix < 0 ? 0 : (ix > rows - 2 ? rows - 2 : ix);
  iy = iy < 0 ? 0 : (iy > cols - 2 ? cols - 2 : iy);
  const int h1 = hf[(size_t)ix * cols + iy];
  const int h2 = hf[(size_t)(ix + 1) * cols + iy + 1];
  out[t] = (float)(h1 < h2 ? h1 : h2) * vs;
}

__global__ void k_torch_rand(gt_torch_rand_plan plan, float* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < plan.numel) out[i] = torch_philox::rand_at(plan, i);
}

int fail(const char* what, hipError_t e) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  g_err = buf;
  return -1;
}
int check_params(const gt_anymal_params* p, const gt_anymal_buffers* b) {
  const gt_anymal_hound* h = b ? b->hound : nullptr;
  const int na = h ? h->num_actions : (p ? p->num_dofs : 0);
  if (!p || !b || p->num_envs <= 0 || p->num_dofs <= 0 || p->num_dofs > 16 || p->num_feet > 4 || p->num_knees > 4 ||
      na < p->num_dofs || na > kMaxActions || p->num_obs != 12 + 2 * p->num_dofs + 140 + na + (h ? 10 : 0)) {
    g_err = "gt_anymal: invalid parameters";
    return -1;
  }
  if (h && (h->num_shoulders < 0 || h->num_shoulders > 4 || !h->eef_state || !h->arm_commands || !h->pos_control ||
            !h->effort_control || h->num_actions != p->num_dofs + 6)) {
    g_err = "gt_anymal: invalid UsefulHound extension";
    return -1;
  }
  return 0;
}
gt_anymal_hound hound_of(const gt_anymal_buffers* b) { return b->hound ? *b->hound : gt_anymal_hound{}; }
}  // namespace

// shared with the other task kernels of libgymtask (gt_hound.hip)
void gt_set_last_error(const char* msg) { g_err = msg; }

extern "C" {

int gt_abi_version(void) { return GT_ABI_VERSION; }
const char* gt_last_error(void) { return g_err.c_str(); }

int gt_anymal_post_physics_a(const gt_anymal_params* p, const gt_anymal_buffers* b, void* stream) {
  if (check_params(p, b)) return -1;
  if (!b->reset_count) {
    g_err = "gt_anymal_post_physics_a: reset_count (int32[3], zero-initialised) is required";
    return -1;
  }
  const int blk = 64;
  const dim3 grid((p->num_envs + blk - 1) / blk);
  auto aligned = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  const bool vec = p->num_dofs % 4 == 0 && aligned(b->torques) && aligned(b->actions) && aligned(b->last_actions) &&
                   aligned(b->last_dof_vel) && aligned(b->dof_state);
  const gt_anymal_hound h = hound_of(b);
  // (GT_POST_A_GENERIC set: the runtime-nd form, an A/B switch)
  static const bool generic = std::getenv("GT_POST_A_GENERIC") != nullptr;
  if (b->hound) hipLaunchKernelGGL((k_post_a<false, true>), grid, dim3(blk), 0, (hipStream_t)stream, *p, *b, h);
  else if (vec && p->num_dofs == 12 && !generic)  // AnymalTerrain: straight-line loads (gt_anymal_tail.h NDC)
    hipLaunchKernelGGL((k_post_a<true, false, 12>), grid, dim3(blk), 0, (hipStream_t)stream, *p, *b, h);
  else if (vec) hipLaunchKernelGGL((k_post_a<true, false>), grid, dim3(blk), 0, (hipStream_t)stream, *p, *b, h);
  else hipLaunchKernelGGL((k_post_a<false, false>), grid, dim3(blk), 0, (hipStream_t)stream, *p, *b, h);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_post_physics_a", e);
}

int gt_anymal_reset(const gt_anymal_params* p, const gt_anymal_buffers* b, const int32_t* env_ids, int k,
                    const float* pos_offset, const float* dof_vel, const float* cmd_x, const float* cmd_y,
                    const float* cmd_heading, float* episode_out, void* stream) {
  if (check_params(p, b)) return -1;
  if (b->hound) {
    g_err = "gt_anymal_reset: UsefulHound resets go through gt_anymal_reset_flagged";
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  if (k <= 0) {
    hipError_t e = hipMemsetAsync(episode_out, 0, sizeof(float) * GT_ANYMAL_NUM_TERMS, st);
    return e == hipSuccess ? 0 : fail("gt_anymal_reset memset", e);
  }
  hipLaunchKernelGGL(k_episode_sums, dim3(1), dim3(64 * GT_ANYMAL_NUM_TERMS), 0, st, *p, b->episode_sums, env_ids, k,
                     episode_out);
  const int blk = 256;
  hipLaunchKernelGGL(k_reset, dim3((k + blk - 1) / blk), dim3(blk), 0, st, *p, *b, env_ids, k, pos_offset, dof_vel,
                     cmd_x, cmd_y, cmd_heading);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_reset", e);
}

int gt_anymal_post_physics_ab(const gt_anymal_params* p, const gt_anymal_buffers* b,
                              const gt_torch_rand_plan* noise_plan, void* stream) {
  if (check_params(p, b)) return -1;
  auto aligned = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
  if (b->hound || p->num_dofs != 12 || !b->reset_count || !b->reset_masks || b->measured_heights ||
      !aligned(b->torques) || !aligned(b->actions) || !aligned(b->last_actions) || !aligned(b->last_dof_vel) ||
      !aligned(b->dof_state)) {
    g_err = "gt_anymal_post_physics_ab: AnymalTerrain plane, 12 dofs, 16-byte aligned dof rows, reset_count and "
            "reset_masks required";
    return -1;
  }
  if (noise_plan && ((uint64_t)noise_plan->numel != (uint64_t)p->num_envs * p->num_obs || noise_plan->threads == 0)) {
    g_err = "gt_anymal_post_physics_ab: noise plan does not cover obs_buf";
    return -1;
  }
  const dim3 g((p->num_envs + kAbEnvs - 1) / kAbEnvs), bl(256);
  const gt_torch_rand_plan pl = noise_plan ? *noise_plan : gt_torch_rand_plan{};
  if (noise_plan) hipLaunchKernelGGL((k_post_ab<2>), g, bl, 0, (hipStream_t)stream, *p, *b, nullptr, pl);
  else hipLaunchKernelGGL((k_post_ab<0>), g, bl, 0, (hipStream_t)stream, *p, *b, nullptr, pl);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_post_physics_ab", e);
}

int gt_anymal_post_physics_b(const gt_anymal_params* p, const gt_anymal_buffers* b, const float* noise,
                             const gt_torch_rand_plan* noise_plan, void* stream) {
  if (check_params(p, b)) return -1;
  if (p->num_obs > 256) {
    g_err = "gt_anymal_post_physics_b: num_obs > 256";
    return -1;
  }
  const int blk = (p->num_obs + 63) / 64 * 64;
  gt_torch_rand_plan plan{};
  hipStream_t st = (hipStream_t)stream;
  const gt_anymal_hound h = hound_of(b);
  if (noise_plan && !noise &&
      ((uint64_t)noise_plan->numel != (uint64_t)p->num_envs * p->num_obs || noise_plan->threads == 0)) {
    g_err = "gt_anymal_post_physics_b: noise plan does not cover obs_buf";
    return -1;
  }
  const int mode = noise ? 1 : noise_plan ? 2 : 0;
  const gt_torch_rand_plan pl = (mode == 2) ? *noise_plan : plan;
  const dim3 g(p->num_envs), bl(blk);
#define GT_POST_B(M, H) hipLaunchKernelGGL((k_post_b<M, H>), g, bl, 0, st, *p, *b, h, noise, pl)
  if (b->hound) {
    if (mode == 1) GT_POST_B(1, true); else if (mode == 2) GT_POST_B(2, true); else GT_POST_B(0, true);
  } else {
    if (mode == 1) GT_POST_B(1, false); else if (mode == 2) GT_POST_B(2, false); else GT_POST_B(0, false);
  }
#undef GT_POST_B
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_post_physics_b", e);
}

int gt_anymal_reset_flagged(const gt_anymal_params* p, const gt_anymal_buffers* b, int k,
                            const gt_anymal_reset_draws* d, const gt_anymal_terrain_reset* terrain,
                            int32_t* env_ids_out, float* episode_out, float episode_length_s, void* scratch,
                            void* stream) {
  if (check_params(p, b)) return -1;
  if (!b->reset_masks || !d || !env_ids_out || !episode_out || !scratch || k < 0 || k > p->num_envs) {
    g_err = "gt_anymal_reset_flagged: invalid arguments";
    return -1;
  }
  if (terrain && (!terrain->terrain_levels || !terrain->terrain_types || !terrain->env_origins ||
                  !terrain->terrain_origins || terrain->env_rows <= 0 || terrain->env_cols <= 0)) {
    g_err = "gt_anymal_reset_flagged: incomplete terrain reset";
    return -1;
  }
  const gt_anymal_terrain_reset tr = terrain ? *terrain : gt_anymal_terrain_reset{};
  if (k == 0) return 0;
  unsigned* done = static_cast<unsigned*>(scratch);
  float* partial = static_cast<float*>(scratch) + 16;
  const gt_anymal_hound h = hound_of(b);
  const dim3 g((p->num_envs + 63) / 64), bl(64);
  if (b->hound)
    hipLaunchKernelGGL(k_reset_flagged<true>, g, bl, 0, (hipStream_t)stream, *p, *b, h, k, *d, tr, terrain != nullptr,
                       env_ids_out, episode_out, episode_length_s, partial, done);
  else
    hipLaunchKernelGGL(k_reset_flagged<false>, g, bl, 0, (hipStream_t)stream, *p, *b, h, k, *d, tr,
                       terrain != nullptr, env_ids_out, episode_out, episode_length_s, partial, done);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_anymal_reset_flagged", e);
}

int gt_anymal_reset_observe(const gt_anymal_params* p, const gt_anymal_buffers* b, int k, gt_anymal_reset_draws* d,
                            int32_t* env_ids_out, float* episode_out, float episode_length_s, void* scratch,
                            uint64_t seed, uint64_t* offset, uint32_t grid_cap, int add_noise, gt_set_state_fn set_state,
                            void* set_state_ctx, const float* root_states, const float* dof_state, void* stream) {
  if (check_params(p, b)) return -1;
  if (b->hound || !d || !offset || grid_cap == 0 || !set_state || !root_states || !dof_state || k <= 0 ||
      k > p->num_envs) {
    g_err = "gt_anymal_reset_observe: invalid arguments (AnymalTerrain plane resets, k > 0)";
    return -1;
  }
  // torch.rand(n) plans on the generator stream (gymtask.TorchRandPlanner.plan_many's arithmetic)
  uint64_t off = *offset;
  auto plan = [&](uint64_t n) {
    const uint64_t blocks = (n + 255) / 256;
    const uint32_t threads = (uint32_t)(256 * (blocks < grid_cap ? blocks : grid_cap));
    const gt_torch_rand_plan pl{seed, off, threads, (uint32_t)n};
    off += ((n - 1) / (4 * (uint64_t)threads) + 1) * 4;
    return pl;
  };
  const uint64_t kn = (uint64_t)k * p->num_dofs;
  d->u_pos = d->u_vel = d->u_cmd_x = d->u_cmd_y = d->u_cmd_h = nullptr;
  d->plan_pos = plan(kn);
  d->plan_vel = plan(kn);
  d->plan_cmd_x = plan((uint64_t)k);
  d->plan_cmd_y = plan((uint64_t)k);
  d->plan_cmd_h = plan((uint64_t)k);
  if (gt_anymal_reset_flagged(p, b, k, d, nullptr, env_ids_out, episode_out, episode_length_s, scratch, stream))
    return -1;
  if (set_state(set_state_ctx, root_states, dof_state, env_ids_out, k, stream)) {
    g_err = "gt_anymal_reset_observe: the set_state callback failed";
    return -1;
  }
  gt_torch_rand_plan noise{};
  if (add_noise) noise = plan((uint64_t)p->num_envs * p->num_obs);
  if (gt_anymal_post_physics_b(p, b, nullptr, add_noise ? &noise : nullptr, stream)) return -1;
  *offset = off;
  return 0;
}

int gt_measure_heights(const int16_t* samples, int rows, int cols, float border, float hs, float vs,
                       const float* root_states, const float* points, int num_envs, int num_points, float* heights,
                       void* stream) {
  if (!samples || !root_states || !points || !heights || rows < 2 || cols < 2 || num_envs < 0 || num_points < 0 ||
      !(hs > 0.0f)) {
    g_err = "gt_measure_heights: invalid arguments";
    return -1;
  }
  const long n = (long)num_envs * num_points;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_measure_heights, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, samples,
                     rows, cols, border, hs, vs, root_states, points, num_envs, num_points, heights);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_measure_heights", e);
}

int gt_torch_rand(const gt_torch_rand_plan* plan, float* out, void* stream) {
  if (!plan || !out || plan->threads == 0) {
    g_err = "gt_torch_rand: invalid arguments";
    return -1;
  }
  if (plan->numel == 0) return 0;
  const int blk = 256;
  hipLaunchKernelGGL(k_torch_rand, dim3((plan->numel + blk - 1) / blk), dim3(blk), 0, (hipStream_t)stream, *plan,
                     out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("gt_torch_rand", e);
}

int gt_host_alloc(uint64_t bytes, void** host_ptr, void** device_ptr) {
  if (!host_ptr || !device_ptr || bytes == 0) {
    g_err = "gt_host_alloc: invalid arguments";
    return -1;
  }
  void* h = nullptr;
  hipError_t e = hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return fail("gt_host_alloc hipHostMalloc", e);
  std::memset(h, 0, bytes);
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return fail("gt_host_alloc hipHostGetDevicePointer", e);
  }
  *host_ptr = h;
  *device_ptr = d;
  return 0;
}

int gt_host_free(void* host_ptr) {
  if (!host_ptr) return 0;
  hipError_t e = hipHostFree(host_ptr);
  return e == hipSuccess ? 0 : fail("gt_host_free", e);
}

int gt_wait_host_seq(const int32_t* words, int32_t seq, int32_t timeout_ms, int32_t* value) {
  if (!words || !value) {
    g_err = "gt_wait_host_seq: invalid arguments";
    return -1;
  }
  // Busy-poll: the count lands a few microseconds after post_a finishes, much sooner than an
  // event wake-up.  Yield after the first ~50k polls (~1 ms) so a long wait does not hog a core.
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 0;; ++i) {
    // {count, seq} arrive as one 8-byte store (words is hipHostMalloc'd, so 8-byte aligned)
    const uint64_t w = __atomic_load_n(reinterpret_cast<const uint64_t*>(words), __ATOMIC_ACQUIRE);
    if ((int32_t)(uint32_t)(w >> 32) == seq) {
      *value = (int32_t)(uint32_t)w;
      return 0;
    }
    if ((i & 4095) == 4095) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
        g_err = "gt_wait_host_seq: timed out waiting for post_a (kernel not finished)";
        return -1;
      }
      if (i > 50000) std::this_thread::yield();
    }
  }
}

int gt_anymal_wait_reset_observe(const int32_t* words, int32_t seq, int32_t timeout_ms, int32_t* count,
                                 const gt_anymal_params* p, const gt_anymal_buffers* b, gt_anymal_reset_draws* d,
                                 int32_t* env_ids_out, float* episode_out, float episode_length_s, void* scratch,
                                 uint64_t seed, uint64_t* offset, uint32_t grid_cap, int add_noise,
                                 gt_set_state_fn set_state, void* set_state_ctx, const float* root_states,
                                 const float* dof_state, void* stream) {
  if (!count || gt_wait_host_seq(words, seq, timeout_ms, count)) return -1;
  if (*count <= 0) return 0;
  return gt_anymal_reset_observe(p, b, *count, d, env_ids_out, episode_out, episode_length_s, scratch, seed, offset,
                                 grid_cap, add_noise, set_state, set_state_ctx, root_states, dof_state, stream);
}

}  // extern "C"
