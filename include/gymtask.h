/*
 * gymtask.h -- C ABI of libgymtask.so: fused task-layer kernels for the
 * post-physics tail of VecTask.step (reference tasks/anymal_terrain.py).
 *
 * The reference computes this tail as ~790 small torch/TorchScript ops per
 * step; these entry points replace, for AnymalTerrain:
 *   gt_anymal_post_physics_a : anymal_terrain.py:458-475 minus the push
 *       progress/randomize counters, base-frame velocities and gravity
 *       (quat_rotate_inverse x3), heading command (quat_apply, atan2,
 *       wrap_to_pi), check_termination (:294-300), compute_reward (:315-382)
 *       incl. feet air time and episode sums.
 *   gt_anymal_reset : reset_idx (:384-425) given the random draws the host made
 *       with torch in the reference's order (bit-exact resets).
 *   gt_anymal_post_physics_b : compute_observations (:302-313) + noise
 *       (:481-482) + last_actions / last_dof_vel (:484-485).
 * All tensors are the reference's (float32 AoS unless stated); all calls are
 * stream ordered and return 0 on success (gt_last_error() otherwise).
 */
#ifndef GYMTASK_H
#define GYMTASK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GT_ABI_VERSION 5
#define GT_ANYMAL_NUM_TERMS 13  /* lin_vel_xy lin_vel_z ang_vel_z ang_vel_xy orient torques joint_acc
                                   base_height air_time collision stumble action_rate hip */

/* One torch.rand(n) call on the device generator, evaluated in-kernel instead of launched
 * (isaacgymenv_amd/csrc/torch_philox.h): seed and offset are the generator's before the call,
 * threads = 256 * min(CUs * maxThreadsPerCU / 256, ceil(n / 256)); the host advances the
 * generator offset by ((n - 1) / (4 * threads) + 1) * 4 as torch does. */
typedef struct gt_torch_rand_plan {
    uint64_t seed, offset;
    uint32_t threads, numel;
} gt_torch_rand_plan;

typedef struct gt_anymal_params {
    int32_t num_envs, num_dofs, num_bodies, num_obs;
    int32_t base_index;
    int32_t num_feet, feet_idx[4];
    int32_t num_knees, knee_idx[4];
    int32_t hip_dofs[4];
    int32_t allow_knee_contacts;
    int64_t max_episode_length;
    float dt;                        /* policy dt = decimation * sim dt */
    /* reward scales already multiplied by dt (anymal_terrain.py:104-105) */
    float s_termination, s_lin_vel_xy, s_lin_vel_z, s_ang_vel_z, s_ang_vel_xy, s_orient, s_torque,
          s_joint_acc, s_base_height, s_air_time, s_collision, s_stumble, s_action_rate, s_hip;
    float lin_vel_scale, ang_vel_scale, dof_pos_scale, dof_vel_scale, height_meas_scale;
    float default_dof_pos[16];
    float base_init_state[13];
} gt_anymal_params;

struct gt_anymal_hound;

typedef struct gt_anymal_buffers {
    float *root_states;          /* [N][13]                                   */
    const float *contact_forces; /* [N*nb][3]                                 */
    float *dof_state;            /* [N*nd][2]                                 */
    const float *torques;        /* [N][nd]                                   */
    const float *actions;        /* [N][nd]                                   */
    float *last_actions;         /* [N][nd]                                   */
    float *last_dof_vel;         /* [N][nd]                                   */
    float *commands;             /* [N][4]                                    */
    float *feet_air_time;        /* [N][4]                                    */
    int64_t *progress_buf;       /* [N]                                       */
    int64_t *randomize_buf;      /* [N]                                       */
    uint8_t *reset_buf;          /* [N] bool                                  */
    const void *timeout_buf;     /* [N] bool (timeout_is_int64 = 0) or int64  */
    int32_t timeout_is_int64;    /* the first step sees VecTask's int64 zeros */
    float *rew_buf;              /* [N]                                       */
    float *episode_sums;         /* [13][N]                                   */
    float *base_lin_vel;         /* [N][3]                                    */
    float *base_ang_vel;         /* [N][3]                                    */
    float *projected_gravity;    /* [N][3]                                    */
    float *obs_buf;              /* [N][num_obs]                              */
    const float *noise_scale;    /* [num_obs]                                 */
    int32_t *reset_count;        /* [3] device, zero-initialised: post_a's accumulator and
                                    workgroup counter (re-armed by post_a itself), and [2] =
                                    the number of envs post_a flagged for reset               */
    int32_t *host_count;         /* [2] host-mapped words (gt_host_alloc, 8-byte aligned) or NULL:
                                    post_a's last workgroup stores {count, seq} as ONE 8-byte
                                    system-scope store                                         */
    int32_t seq;                 /* sequence number post_a publishes in host_count[1]        */
    uint64_t *reset_masks;       /* [ceil(N/64)] post_a's per-wave reset ballots (bit l of word w =
                                    env 64w+l), read by gt_anymal_reset_flagged                */
    float *obs_out;              /* [N][num_obs] or NULL: VecTask's clamped obs copy (vec_task.py:402) */
    uint8_t *time_outs;          /* [N] bool or NULL: (progress >= T-1) & reset (vec_task.py:394)     */
    float clip_obs;              /* clipObservations (inf -> plain copy)                    */
    const float *measured_heights; /* [N][140] terrain heights under the probes
                                    (gt_measure_heights), or NULL: plane terrain, heights 0 */
    const struct gt_anymal_hound *hound; /* NULL for AnymalTerrain; UsefulHound's differences (ABI 3) */
    float *obs_mirror;           /* ABI 5: [N][num_obs] or NULL: a second copy of what obs_out receives (a
                                    learner's static act-forward input: no copy launch per step); needs obs_out */
} gt_anymal_buffers;

/* UsefulHound (reference tasks/useful_hound.py) runs the same tail with these differences
 * (ABI 3; the gt_anymal_* entry points take them through gt_anymal_buffers.hound):
 *   - num_dofs in gt_anymal_params is the 12 LEG dofs (default_dof_pos, hip terms, last_dof_vel
 *     [N][12], joint_acc, dof observations); dof_state rows hold num_actions (18) dofs, legs first;
 *     torques / actions / last_actions are [N][num_actions];
 *   - check_termination (:467-480): thigh ("knee") contacts terminate regardless of
 *     allow_knee_contacts, and so do the shoulder links (base_indices);
 *   - compute_reward (:499-567): collision = knees * s + shoulders * s;
 *   - reset_idx (:569-642): after the leg draws (and the trimesh root x, y) one torch.rand(k, 6) for
 *     the arm: q_arm = clamp(arm_default + arm_noise2 * (u - 0.5), arm_lower, arm_upper), qd_arm = 0,
 *     pos_control = q_arm, effort_control = 0;
 *   - compute_observations (:482-497): 204 = 12 base | 12 dof pos | 12 dof vel | 140 heights |
 *     18 actions | end-effector position (3) and quaternion (4) from the rigid-body row eef_state
 *     + e * eef_stride | arm_commands [N][3]. */
typedef struct gt_anymal_hound {
    int32_t num_actions;                 /* 18 */
    int32_t num_shoulders, shoulder_idx[4];
    const float *eef_state;              /* env 0's end-effector rigid-body row (pos | quat | ...) */
    int32_t eef_stride;                  /* floats between consecutive envs' rows */
    const float *arm_commands;           /* [N][3] */
    float *pos_control, *effort_control; /* [N][6] */
    float arm_default[6], arm_lower[6], arm_upper[6];
    float arm_noise2;                    /* float(houndarmDofNoise * 2.0) */
    const float *u_arm;                  /* [k][6] drawn buffer, or NULL: use plan_arm */
    gt_torch_rand_plan plan_arm;
} gt_anymal_hound;

int gt_abi_version(void);
const char *gt_last_error(void);

int gt_anymal_post_physics_a(const gt_anymal_params *p, const gt_anymal_buffers *b, void *stream);

/* env_ids int32[k]; pos_offset/dof_vel [k][nd]; cmd_x/cmd_y/cmd_heading [k];
 * episode_out[13] receives the per-term sums over env_ids (then zeroed in
 * episode_sums); the caller divides by k * episodeLength_s. */
int gt_anymal_reset(const gt_anymal_params *p, const gt_anymal_buffers *b, const int32_t *env_ids, int k,
                    const float *pos_offset, const float *dof_vel, const float *cmd_x, const float *cmd_y,
                    const float *cmd_heading, float *episode_out, void *stream);

/* torch.rand draws (uniform [0,1), float32) made by the host in the reference's order
 * (anymal_terrain.py:385-398); the kernel applies torch_rand_float's map
 * `range * u + lower` in float32 (range = float(upper - lower)). */
typedef struct gt_anymal_reset_draws {
    const float *u_pos, *u_vel;              /* [k][nd] drawn buffers, or NULL: use the plan */
    const float *u_cmd_x, *u_cmd_y, *u_cmd_h; /* [k]     */
    gt_torch_rand_plan plan_pos, plan_vel, plan_cmd_x, plan_cmd_y, plan_cmd_h;
    float pos_range, pos_lower, vel_range, vel_lower;
    float cmd_x_range, cmd_x_lower, cmd_y_range, cmd_y_lower, cmd_h_range, cmd_h_lower;
} gt_anymal_reset_draws;

/* The trimesh terrain's part of reset_idx (ABI 2; custom origins, anymal_terrain.py:385-398 with
 * update_terrain_level :427-435): before the reset, an env that walked less than a quarter of its
 * commanded distance over the episode moves a level down, one that left its tile a level up
 * (clip >= 0, modulo env_rows; only when update_levels = init_done && curriculum), and takes the
 * origin terrain_origins[level][type]; the root then starts at base_init_state + origin with x, y
 * offset by U(-0.5, 0.5) draws (drawn after the dof draws, before the command draws).
 * episode_out[13] additionally receives mean(terrain_levels) over all envs (extras["episode"]
 * ["terrain_level"]). */
typedef struct gt_anymal_terrain_reset {
    int64_t *terrain_levels;          /* [N]                   */
    const int64_t *terrain_types;     /* [N]                   */
    float *env_origins;               /* [N][3]                */
    const float *terrain_origins;     /* [env_rows][env_cols][3] */
    int32_t env_rows, env_cols, update_levels;
    float env_length, max_episode_length_s;
    const float *u_root_xy;           /* [k][2] drawn buffer, or NULL: use the plan */
    gt_torch_rand_plan plan_root_xy;
    float xy_range, xy_lower;
} gt_anymal_terrain_reset;

/* reset_idx for the k envs the last post_a flagged, without the host knowing
 * which: envs are ranked by index from reset_masks (torch.nonzero's order), row t of the draws
 * goes to the t-th flagged env.  env_ids_out int32[k] receives the flagged ids ascending (for
 * set_*_tensor_indexed); episode_out[13] = mean over the flagged envs of each episode sum /
 * episode_length_s (extras["episode"], :416-420), sums then zeroed; the means are summed in a
 * fixed order (bit-identical run to run).  terrain: NULL for the plane, else the trimesh part above.  scratch: GT_ANYMAL_RESET_SCRATCH_WORDS(num_envs) words
 * of device memory, the first 16 zero-initialised (a counter the kernel re-arms). */
#define GT_ANYMAL_RESET_SCRATCH_WORDS(num_envs) (16 + (GT_ANYMAL_NUM_TERMS + 1) * (((num_envs) + 63) / 64))
int gt_anymal_reset_flagged(const gt_anymal_params *p, const gt_anymal_buffers *b, int k,
                            const gt_anymal_reset_draws *draws, const struct gt_anymal_terrain_reset *terrain,
                            int32_t *env_ids_out, float *episode_out, float episode_length_s, void *scratch,
                            void *stream);

/* ABI 5: a reset step's whole host sequence after post_a's count (anymal_terrain.py:458-485 with k > 0, plane,
 * AnymalTerrain): the reset draws' plans (torch.rand of k*nd, k*nd, k, k, k in the reference's order), the
 * gt_anymal_reset_flagged launch, the root / dof indexed sets through `set_state` (e.g. gymsim's
 * gs_sim_set_root_and_dof with ctx = the gs_sim), then gt_anymal_post_physics_b with the observation noise plan
 * (add_noise) -- one host call instead of the Python between them.  seed / *offset: the
 * device generator's seed and Philox offset before the draws (the caller's rolled-back offset); *offset returns
 * the offset after them, as torch would leave it.  grid_cap = CUs * maxThreadsPerCU / 256 (the plans' thread
 * counts, see gt_torch_rand_plan).  draws: the affine maps (its u_* / plan_* are written here).  b->obs_out /
 * time_outs / clip_obs as for post_physics_b.  UsefulHound (b->hound) and the trimesh reset are refused. */
typedef int (*gt_set_state_fn)(void *ctx, const float *root_states, const float *dof_state, const int32_t *idx,
                               int n, void *stream);
int gt_anymal_reset_observe(const gt_anymal_params *p, const gt_anymal_buffers *b, int k, gt_anymal_reset_draws *draws,
                            int32_t *env_ids_out, float *episode_out, float episode_length_s, void *scratch,
                            uint64_t seed, uint64_t *offset, uint32_t grid_cap, int add_noise,
                            gt_set_state_fn set_state, void *set_state_ctx, const float *root_states,
                            const float *dof_state, void *stream);

/* ABI 5: gt_anymal_post_physics_a + gt_anymal_post_physics_b (noise_plan or none) in one launch, for
 * AnymalTerrain on the plane (num_dofs 12, no measured heights, post_a's 16-byte aligned dof rows): each
 * workgroup runs part A for its 16 envs, then their observations; the count and the reset masks are published
 * exactly as post_physics_a publishes them. */
int gt_anymal_post_physics_ab(const gt_anymal_params *p, const gt_anymal_buffers *b,
                              const gt_torch_rand_plan *noise_plan, void *stream);

/* ABI 5: gt_wait_host_seq, then -- when the count is > 0 -- gt_anymal_reset_observe with it, so the reset's first
 * launch follows the count with no caller code in between; *count receives the count either way (*offset is only
 * advanced when it is > 0). */
int gt_anymal_wait_reset_observe(const int32_t *words, int32_t seq, int32_t timeout_ms, int32_t *count,
                                 const gt_anymal_params *p, const gt_anymal_buffers *b, gt_anymal_reset_draws *draws,
                                 int32_t *env_ids_out, float *episode_out, float episode_length_s, void *scratch,
                                 uint64_t seed, uint64_t *offset, uint32_t grid_cap, int add_noise,
                                 gt_set_state_fn set_state, void *set_state_ctx, const float *root_states,
                                 const float *dof_state, void *stream);

/* Pinned, device-mapped, coherent host memory for host_count (hipHostMalloc). */
int gt_host_alloc(uint64_t bytes, void **host_ptr, void **device_ptr);
int gt_host_free(void *host_ptr);
/* Spin until words[1] == seq (post_a published), then *value = words[0].  Returns -1 after
 * timeout_ms (a kernel that never finished): the caller raises instead of hanging. */
int gt_wait_host_seq(const int32_t *words, int32_t seq, int32_t timeout_ms, int32_t *value);

/* noise [N][num_obs] uniform draws (torch.rand_like(obs_buf)), or NULL and noise_plan for the
 * same draws evaluated in-kernel, or both NULL when addNoise is false */
int gt_anymal_post_physics_b(const gt_anymal_params *p, const gt_anymal_buffers *b, const float *noise,
                             const gt_torch_rand_plan *noise_plan, void *stream);

/* get_heights (anymal_terrain.py:515-538, trimesh terrain): for env e and probe k,
 *   p = quat_apply_yaw(root_quat[e], points[e][k]) + root_pos[e] + border,
 *   (px, py) = clip(trunc(p.xy / hs), 0, (rows-2, cols-2)),
 *   heights[e][k] = vs * min(samples[px][py], samples[px+1][py+1]).
 * samples int16 [rows][cols]; root_states [N][13]; points [N][num_points][3]; heights [N][num_points]. */
int gt_measure_heights(const int16_t *samples, int rows, int cols, float border, float hs, float vs,
                       const float *root_states, const float *points, int num_envs, int num_points, float *heights,
                       void *stream);

/* UsefulHound control (useful_hound.py:695-726 inner loop, fused): for every env,
 *   legs: torques[0:12] = clip(kp * (action_scale * a[0:12] + leg_default - q[0:12]) - kd * qd[0:12], +-torque_limit)
 *   arm : the operational-space controller of useful_hound.py:660-691 with
 *         M = mass_matrix[e][nv-6:][nv-6:], J = jacobian[e][jac_row][:][0:6], v_eef = rigid_body[e*nl+eef_link][7:13],
 *         dpose = a[12:18] * arm_cmd_limit / arm_action_scale,
 *         u = J^T M_eef (arm_kp dpose - arm_kd v_eef) + (1 - J^T M_eef J M^-1) M u_null,  M_eef = (J M^-1 J^T)^-1,
 *         u_null = -arm_kd_null qd_arm + arm_kp_null ((arm_default - q_arm + pi) mod 2 pi - pi),
 *         clamped to +-arm_effort  -> torques[12:18] and arm_control (row stride arm_control_stride floats).
 * The 6x6 algebra runs in float64 (Gauss-Jordan with partial pivoting) on one lane per env.
 * actions [N][18], dof_state [N*18][2], leg_default [12] (device), mass_matrix [N][nv][nv],
 * jacobian [N][nl][6][nv], rigid_body [N*nl][13], torques [N][18]. */
typedef struct gt_hound_control_params {
    int32_t num_envs, nv, num_links, jac_row, eef_link, arm_control_stride;
    float kp, kd, action_scale, torque_limit, arm_action_scale;
    float arm_kp[6], arm_kd[6], arm_kp_null[6], arm_kd_null[6], arm_cmd_limit[6], arm_default[6], arm_effort[6];
} gt_hound_control_params;

int gt_hound_control(const gt_hound_control_params *p, const float *actions, const float *dof_state,
                     const float *leg_default, const float *mass_matrix, const float *jacobian,
                     const float *rigid_body, float *torques, float *arm_control, void *stream);

/* Ant post-physics tail (ant.py:299-324 compute_observations + :326-371 compute_ant_reward), fused,
 * run after post_physics_step's resets and refreshes: per env, the 60-wide observation, potentials /
 * previous potentials, up and heading vectors, the reward, the done mask (int64, fallen or episode
 * end, else kept) and extras["true_objective"]; publishes the done count {count, seq} to host_count
 * (gt_host_alloc words) so the next step's reset needs no nonzero() when nothing is done.
 * root_states [N][13], dof_state [N*8][2], sensors [N][24], actions [N][8], targets [N][3],
 * inv_start_rot [N][4], potentials / prev_potentials / rew_buf / true_objective [N],
 * up_vec / heading_vec [N][3], obs_buf [N][60], reset_buf / progress_buf int64 [N]. */
typedef struct gt_ant_params {
    int32_t num_envs, num_dofs;
    float dt, dof_vel_scale, contact_force_scale, heading_weight, up_weight, actions_cost_scale,
          energy_cost_scale, joints_at_limit_cost_scale, termination_height, death_cost, max_episode_length;
    float dof_lower[8], dof_upper[8];
} gt_ant_params;

typedef struct gt_ant_buffers {
    const float *root_states, *dof_state, *sensors, *actions, *targets, *inv_start_rot;
    float *potentials, *prev_potentials, *up_vec, *heading_vec, *obs_buf, *rew_buf, *true_objective;
    int64_t *reset_buf;
    const int64_t *progress_buf;
    int32_t *reset_count;        /* [3] device, zero-initialised accumulator (re-armed by the kernel) */
    int32_t *host_count;         /* [2] host-mapped {count, seq} or NULL */
    int32_t seq;
    uint64_t *reset_masks;       /* ABI 4: [ceil(N/64)] the done mask's per-wave ballots (gt_ant_reset_flagged) */
} gt_ant_buffers;

int gt_ant_post_physics(const gt_ant_params *p, const gt_ant_buffers *b, void *stream);

/* Ant reset_idx (ant.py:252-279), fused (ABI 4), for the k envs the previous gt_ant_post_physics flagged
 * (its reset_masks ballots; env ids ascending = torch's nonzero order):
 *   offsets    = torch_rand_float(-0.2, 0.2, (k, 8)), velocities = torch_rand_float(-0.1, 0.1, (k, 8))
 *                (pos_range * u + pos_lower etc.; u from the two consecutive torch.rand plans, evaluated in-kernel
 *                bit-identically to torch's Philox, or from explicit uniforms u_pos / u_vel [k][8])
 *   dof_state[e] = (tensor_clamp(initial_dof_pos[e] + offsets, lower, upper), velocities)
 *   prev_potentials[e] = potentials[e] = -|planar(targets[e] - initial_root_states[e, 0:3])| / dt
 *   progress_buf[e] = 0, reset_buf[e] = 0, env_ids_out[rank] = e
 * The caller then applies set_actor_root_state_tensor_indexed(initial_root_states, env_ids_out, k) and
 * set_dof_state_tensor_indexed(dof_state, env_ids_out, k) as the reference does. */
typedef struct gt_ant_reset_args {
    gt_torch_rand_plan plan_pos, plan_vel;
    const float *u_pos, *u_vel;
    float pos_range, pos_lower, vel_range, vel_lower;
    const float *initial_dof_pos;      /* [N][8]  */
    const float *initial_root_states;  /* [N][13] */
    float *dof_state;                  /* [N*8][2] the task's dof tensor */
    int64_t *progress_buf;             /* [N] */
    int32_t *env_ids_out;              /* [>= k] */
} gt_ant_reset_args;

int gt_ant_reset_flagged(const gt_ant_params *p, const gt_ant_buffers *b, int k, const gt_ant_reset_args *r,
                         void *stream);

/* out[plan.numel] = torch.rand(plan.numel) for the given plan (checks torch_philox.h against torch) */
int gt_torch_rand(const gt_torch_rand_plan *plan, float *out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GYMTASK_H */
