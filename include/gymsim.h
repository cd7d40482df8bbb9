/*
 * gymsim.h -- C ABI of libgymsim.so, the MI355X-native simulator behind the
 * `isaacgym.gymapi` / `gymtorch` surface.
 *
 * The reference reaches its (closed, CUDA/PhysX) simulator only through the
 * Isaac Gym Python binding; every entry point below replaces one call the
 * reference's task layer makes on `self.gym`.  The
 * Python shim in isaacgymenv_amd/isaacgym/gymapi.py binds these with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - plain pointers and sizes; no torch types.  Device pointers are HIP
 *     device addresses (torch.Tensor.data_ptr() on cuda:k); `stream` is a
 *     hipStream_t passed as void* (0 = default stream).
 *   - every function returns int status, 0 = ok; on error gs_last_error()
 *     returns a message.  gs_sim_create returns NULL on failure, the caller's
 *     `create_sim` returns None (vec_task.py:338-340).
 *   - a gs_sim is not thread safe; all work is stream ordered (no host sync)
 *     except gs_sim_create / gs_sim_set_model / gs_sim_prepare.
 *   - host backend (ABI 3): gs_sim_create(device < 0, ...) makes a sim that runs the
 *     same solver on the CPU -- the reference's sim_device=cpu pipeline (vec_task.py:82-88,
 *     PhysX CPU with physx.num_threads workers, cfg/config.yaml:30-32).  Every buffer
 *     argument of such a sim is a HOST pointer in the same layout, `stream` is ignored and
 *     each call returns when its work is done (gym.fetch_results(sim, True) is a no-op).
 *     It makes no HIP call, so it runs on a machine without a GPU.
 *   - tensor layouts are the reference's (AoS, float32):
 *       root state  [num_envs][13]  pos(3) quat xyzw(4) lin vel of COM(3) ang vel(3)
 *       dof state   [num_envs*num_dofs][2] (pos, vel)
 *       dof force   [num_envs*num_dofs]
 *       net contact [num_envs*num_bodies][3]
 *       rigid body  [num_envs*num_bodies][13] pos(3) quat xyzw(4) lin vel of COM(3) ang vel(3)
 *       jacobian    [num_envs][num_bodies][6][nv]  rows: COM lin vel (3), ang vel (3), world axes
 *       mass matrix [num_envs][nv][nv]
 *     num_bodies counts reported links (fixed-joint links included when
 *     collapse_fixed_joints=False); nv = 6 + num_dofs (floating base: root COM
 *     linear velocity, root angular velocity, then dof velocities) or num_dofs.
 *     (one articulation actor per env; actor index == env index)
 */
#ifndef GYMSIM_H
#define GYMSIM_H

#include <stdint.h>

#include "gymtask.h"  /* gs_pd_args.tail_*: the AnymalTerrain tail structs */

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 9

typedef struct gs_sim gs_sim;

/* Articulation description after asset import (double precision on the host).
 * Built by isaacgymenv_amd/isaacgym/_model.py:flatten(). */
typedef struct gs_model_desc {
    int32_t num_bodies, num_dofs, num_candidates, num_shapes, fixed_base;
    const int32_t *parent;        /* [nb] body parent, -1 root                          */
    const int32_t *joint_kind;    /* [nb] 1 revolute, 2 prismatic, root 3 free / 0 fixed */
    const int32_t *body_dof;      /* [nb] dof moved by the body's joint, -1 root        */
    const double *joint_origin;   /* [nb][12] parent frame -> joint frame: R (9) t (3)  */
    const double *joint_axis;     /* [nb][3] in the joint frame                         */
    const double *mass;           /* [nb]                                               */
    const double *com;            /* [nb][3] body frame                                 */
    const double *inertia;        /* [nb][9] about COM, body axes                       */
    const int32_t *cand_body;     /* [nc] contact candidate: body                       */
    const double *cand_point;     /* [nc][3] body frame                                 */
    const double *cand_radius;    /* [nc]                                               */
    const int32_t *cand_shape;    /* [nc] shape index (friction lookup)                 */
    const double *dof_effort;     /* [nd] max |force|, <= 0 unlimited                   */
    const double *dof_velocity;   /* [nd] max |vel|, <= 0 unlimited                     */
    const double *dof_armature;   /* [nd]                                               */
    const double *dof_lower;      /* [nd] joint limits (rad or m), used where has_limits */
    const double *dof_upper;      /* [nd]                                               */
    const int32_t *dof_has_limits;/* [nd] 0/1 (URDF <limit>, MJCF limited="true")     */
    /* reported links (ABI 2): the tensor API's rigid bodies.  Equal to the bodies unless
     * fixed joints are kept (collapse_fixed_joints=False), then each fixed link is welded
     * into a body for the dynamics but still reported (Hound.urdf: 19 bodies, 24 links). */
    int32_t num_links;
    const int32_t *cand_link;     /* [nc] link whose net contact force the candidate adds to */
    const int32_t *link_body;     /* [nl] dynamic body the link is welded into          */
    const double *link_pose;      /* [nl][12] link frame in the body frame: R (9) t (3) */
    const double *link_com;       /* [nl][3] link COM, link frame                       */
    /* convex hulls and self-collision (ABI 5).  A convex hull (STL mesh
     * collider, useful_hound.py:329) keeps every hull vertex; against the ground it has 4 dynamic
     * candidates (cand_dyn 0..3) filled every substep from its vertices.  Filter-0 actors
     * (gym.create_actor(..., filter=0), anymal_terrain.py:282, useful_hound.py:421) collide their
     * own shapes pairwise (gs_sim_set_self_collision). */
    const int32_t *cand_dyn;      /* [nc] hull slot of a dynamic candidate, -1 fixed point */
    const int32_t *shape_kind;    /* [ns] 0 sphere 1 capsule 2 box 3 cylinder 4 hull      */
    const int32_t *shape_body;    /* [ns]                                               */
    const int32_t *shape_link;    /* [ns]                                               */
    const double *shape_pose;     /* [ns][12] shape frame in the body frame: R (9) t (3) */
    const double *shape_size;     /* [ns][3] sphere r | capsule / cylinder r, half length | box half extents */
    const double *shape_margin;   /* [ns] core radius of the pair narrowphase           */
    const double *shape_sphere;   /* [ns][4] bounding sphere, body frame centre + radius */
    int32_t num_hull_verts;
    const double *hull_verts;     /* [nhv][4] body frame xyz + core factor f (core vertex = c + f (v - c),
                                     c = shape_sphere centre) */
    const int32_t *shape_hv0;     /* [ns] hull vertex range [hv0, hv1)                   */
    const int32_t *shape_hv1;     /* [ns]                                               */
    int32_t num_pairs;
    const int32_t *pair_a;        /* [np] shape a < shape b of a link pair that may collide */
    const int32_t *pair_b;        /* [np]                                               */
    const int32_t *pair_kind;     /* [np] 0 sphere-sphere 1 sphere-capsule 2 capsule-capsule 3 GJK */
    int32_t pair_pool;            /* self-contact slots per env (the compiled topology's) */
    int32_t num_pair_verts;
    const double *pair_verts;     /* [npv][4] the hulls' self-collision core vertices (a subset of hull_verts) */
    const int32_t *shape_pv0;     /* [ns] range [pv0, pv1)                              */
    const int32_t *shape_pv1;     /* [ns]                                               */
} gs_model_desc;

/* gymapi.SimParams subset the reference sets (vec_task.py:514-562). */
typedef struct gs_sim_params {
    double dt;
    int32_t substeps;
    double gravity[3];
    int32_t num_position_iterations;
    int32_t num_velocity_iterations;
    double contact_offset;
    double rest_offset;
    double bounce_threshold_velocity;   /* accepted, restitution is 0 in every in-scope task */
    double max_depenetration_velocity;
    int32_t contact_collection;         /* 0 never, 1 last substep (2 treated as 1)        */
    int32_t kernel_variant;             /* 0 auto, 1 one env per lane, 2 lane team (4 lanes/env), 4 runtime-sized (ABI 8) */
    double joint_limit_margin;          /* a limit row is active within this distance of the limit */
    int32_t num_threads;                /* ABI 3, host backend: physx.num_threads (cfg/config.yaml:30)
                                           solver threads including the caller; <= 1 = caller only */
    int32_t solver_type;                /* ABI 7: physx.solver_type (cfg/config.yaml:31): 0 PGS with split
                                           impulse, 1 TGS -- the position iterations as sub-steps of
                                           h / num_position_iterations; every kernel form */
} gs_sim_params;

/* Fused PD decimation step (AnymalTerrain.pre_physics_step + VecTask.step's
 * simulate loop, anymal_terrain.py:441-451 + vec_task.py:379-382):
 *   repeat `decimation` times:
 *     torque = clip(kp*(action_scale*a + default_pos - q) - kd*qd, +-torque_limit)
 *     simulate()                                  (sim dt, `substeps`)
 *   then `extra_simulates` more simulate() with the last torque.
 *   Outputs mirror the refresh calls the reference makes: dof state after the
 *   decimation loop (refresh_dof_state_tensor inside the loop), root state and
 *   contact forces after the extra simulates (post_physics_step refreshes). */
typedef struct gs_pd_args {
    const float *actions;        /* [N][nd]                      */
    const float *default_pos;    /* [nd]  (device)               */
    float kp, kd, action_scale, torque_limit;
    int32_t decimation;
    int32_t extra_simulates;
    float *torques_out;          /* [N][nd]  last applied torque */
    float *dof_state_out;        /* [N*nd][2] in/out, required: the first PD torque reads q, qd
                                    from it (the task's refreshed dof_pos / dof_vel views,
                                    anymal_terrain.py:444-445), it receives the state after
                                    the decimation loop */
    float *root_state_out;       /* [N][13]   or NULL            */
    float *contact_out;          /* [N*nb][3] or NULL            */
    float *actions_copy_out;     /* [N][nd] or NULL: receives `actions` (the task's
                                    `self.actions = actions.clone()`, anymal_terrain.py:442) */
    /* ABI 9: the AnymalTerrain post_physics_step part A (include/gymtask.h gt_anymal_post_physics_a:
     * anymal_terrain.py:458-475 minus the push) run by the physics kernel's last phase on the outputs it
     * just wrote -- counters, base-frame quantities, heading command, termination, reward, episode sums,
     * the reset mask and the {count, seq} publication -- instead of a separate launch; both NULL: none
     * (the caller launches gt_anymal_post_physics_a).  Only where gs_sim_pd_tail_supported() is 1, with
     * post_a's vector rows (num_dofs % 4 == 0; torques, actions, last_actions, last_dof_vel and dof_state
     * 16-byte aligned) and buffers.torques / actions / root_states / contact_forces / dof_state being
     * this call's torques_out / actions_copy_out / root_state_out / contact_out / dof_state_out.  The
     * structs are read during the call (they may change afterwards). */
    const gt_anymal_params *tail_params;
    const gt_anymal_buffers *tail_buffers;
} gs_pd_args;

int gs_abi_version(void);
const char *gs_last_error(void);

/* 1 when gs_sim_pd_step can run the AnymalTerrain tail in its physics kernel (gs_pd_args.tail_*): the
 * lane-team kernel on the GPU (gs_sim_kernel_variant 2) of a plane scene; 0 otherwise. */
int gs_sim_pd_tail_supported(const gs_sim *sim);

/* 1 if libgymsim was compiled with a specialised kernel for this topology. */
int gs_topology_supported(const gs_model_desc *model);

/* gym.create_sim(compute_device, graphics_device, SIM_PHYSX, sim_params)   vec_task.py:337
 * device >= 0: HIP device ordinal; device < 0: host backend (physx.use_gpu = False). */
gs_sim *gs_sim_create(int device, const gs_sim_params *params);
void gs_sim_destroy(gs_sim *sim);

/* gym.add_ground(sim, PlaneParams)   anymal_terrain.py:188-194 (z-up plane only) */
int gs_sim_add_ground(gs_sim *sim, double static_friction, double dynamic_friction, double restitution);

/* gym.add_triangle_mesh(sim, vertices f32[3V], triangles u32[3T], TriangleMeshParams)
 * anymal_terrain.py:196-208.  The mesh must be a heightfield grid as produced by
 * terrain_utils.convert_heightfield_to_trimesh (rows x cols vertices, row-major; cell (i,j) ->
 * triangles (v[i,j], v[i+1,j+1], v[i,j+1]), (v[i,j], v[i+1,j], v[i+1,j+1]); every vertex within
 * one cell of its grid point); other meshes are rejected (-1, gs_last_error).  transform_p is the
 * mesh translation (TriangleMeshParams.transform.p; rotations are not supported).  One mesh per
 * sim; call before gs_sim_set_model.  Contacts: DESIGN.md 3.7. */
int gs_sim_add_triangle_mesh(gs_sim *sim, const float *vertices, int64_t num_vertices, const uint32_t *triangles,
                             int64_t num_triangles, const double *transform_p, double static_friction,
                             double dynamic_friction, double restitution);

/* gym.load_asset + create_actor for every env (one articulation type per sim)
 * anymal_terrain.py:231,282  cartpole.py:88,106 */
int gs_sim_set_model(gs_sim *sim, const gs_model_desc *model);

/* gym.prepare_sim(sim)   vec_task.py:262.
 * Binds caller-owned device buffers:
 *   state   [13 + 2*nd][N]  SoA sim state: pos(3) quat(4) v_origin(3) w(3) q(nd) qd(nd)
 *   shape_friction [ns][N]  per-env shape friction (anymal_terrain.py:279-281)
 *   contact [3*nb][N]       SoA net contact force of the last collected substep
 * The initial state must already be in `state`. */
int gs_sim_prepare(gs_sim *sim, int num_envs, float *state, const float *shape_friction, float *contact);

/* gym.simulate(sim) with dof actuation forces [N*nd] (set_dof_actuation_force_tensor,
 * anymal_terrain.py:446-448, vec_task.py:382).  `dof_force` may be NULL (zero). */
int gs_sim_simulate(gs_sim *sim, const float *dof_force, void *stream);

/* refresh_*_tensor: sim state -> reference-layout tensors (anymal_terrain.py:451,455,456) */
int gs_sim_refresh_root(gs_sim *sim, float *root_state, void *stream);
int gs_sim_refresh_dof(gs_sim *sim, float *dof_state, void *stream);
int gs_sim_refresh_contact(gs_sim *sim, float *net_contact, void *stream);

/* refresh_rigid_body_state_tensor / refresh_jacobian_tensors / refresh_mass_matrix_tensors
 * (useful_hound.py:440-455 acquire, :725-732 refresh).  Kinematics of the current state:
 * link poses and COM velocities, the link COM Jacobians in the generalized velocities
 * above, and M = sum_b J_b^T diag(m_b, I_b) J_b over the dynamic bodies (so v^T M v / 2 is
 * the kinetic energy).  Layouts in the header comment. */
int gs_sim_refresh_rigid_body(gs_sim *sim, float *rigid_body_state, void *stream);
int gs_sim_refresh_jacobian(gs_sim *sim, float *jacobian, void *stream);
int gs_sim_refresh_mass_matrix(gs_sim *sim, float *mass_matrix, void *stream);

/* set_actor_root_state_tensor(_indexed) / set_dof_state_tensor(_indexed):
 * rows `idx[0..n_idx)` (int32 actor ids) of the full source tensor; idx NULL = all envs.
 * anymal_terrain.py:401-407, 439 */
int gs_sim_set_root(gs_sim *sim, const float *root_state, const int32_t *idx, int n_idx, void *stream);
int gs_sim_set_dof(gs_sim *sim, const float *dof_state, const int32_t *idx, int n_idx, void *stream);
/* ABI 9: gs_sim_set_root + gs_sim_set_dof with the same indices in ONE launch (a reset's pair,
 * set_actor_root_state_tensor_indexed + set_dof_state_tensor_indexed, anymal_terrain.py:401-408). */
int gs_sim_set_root_and_dof(gs_sim *sim, const float *root, const float *dof, const int32_t *idx, int n_idx,
                            void *stream);

/* Fused decimation step, see gs_pd_args. */
int gs_sim_pd_step(gs_sim *sim, const gs_pd_args *args, void *stream);

/* Force sensors (gym.create_asset_force_sensor, ant.py:174-178): one per listed body, identity
 * sensor pose, leaf bodies only.  Call after gs_sim_set_model and before gs_sim_prepare.  A sensor
 * reads the wrench its body receives through its parent joint (Newton-Euler of the body with the
 * substep's solved accelerations, minus gravity and contact), force then torque at the body origin
 * in body axes, from the last substep of every simulate call. */
int gs_sim_set_force_sensors(gs_sim *sim, int n, const int32_t *bodies);
/* Caller-owned SoA readings [6*n][N], bound after gs_sim_prepare. */
int gs_sim_bind_force_sensors(gs_sim *sim, float *sensor_soa);
/* refresh_force_sensor_tensor: SoA -> [N*n][6] (ant.py:233-235) */
int gs_sim_refresh_force_sensor(gs_sim *sim, float *out, void *stream);

/* Joint drives (ABI 4): gym.set_actor_dof_properties with driveMode / stiffness / damping
 * (useful_hound.py:391-404 sets them; PhysX articulation joint drives).  Per dof of the asset:
 * mode 1 DOF_MODE_POS drives with stiffness kp and damping kd toward the position / velocity targets,
 * mode 2 DOF_MODE_VEL with damping kd toward the velocity target, other modes no drive.  Implicit
 * spring-damper per substep: kp (q* - q - h qd) + kd (qd* - qd) with (h kd + h^2 kp) added to the dof's
 * mass-matrix diagonal.  Call after gs_sim_set_model; a sim with drives runs the
 * one-env-per-lane kernel. */
int gs_sim_set_dof_drives(gs_sim *sim, const int32_t *mode, const double *stiffness, const double *damping);
/* Caller-owned drive targets [N*nd] float32 (set_dof_position_target_tensor(_indexed) /
 * set_dof_velocity_target_tensor, useful_hound.py:622-627), read by every later simulate / pd_step;
 * NULL = zero targets. */
int gs_sim_bind_dof_targets(gs_sim *sim, const float *pos_targets, const float *vel_targets);
/* Per-actor dof properties (ABI 8): gym.set_actor_dof_properties called actor by actor with differing values
 * (anymal_terrain.py:283, useful_hound.py:422 call it per actor; Isaac Gym keeps the properties per actor).
 * Caller-owned table [6][nd][N] float32 on the sim's device (host memory for the host backend): drive
 * stiffness (DOF_MODE_POS, else 0), drive damping (DOF_MODE_POS / VEL, else 0), effort (<= 0 unlimited), lower,
 * upper (lower >= upper: no limit), velocity (<= 0 unlimited) -- read by every later simulate / pd_step in
 * place of the asset's values (gs_sim_set_model, gs_sim_set_dof_drives).  any_drive / any_limits: some env has
 * a drive gain / a limit.  NULL unbinds (the asset's values again).  A sim with a table runs the
 * one-env-per-lane kernel; kernel_variant 2 (lane team forced) fails. */
int gs_sim_bind_dof_properties_env(gs_sim *sim, const float *table, int any_drive, int any_limits);

/* Self-collision (ABI 5): gym.create_actor with collision filter 0 (anymal_terrain.py:282,
 * useful_hound.py:421) makes Isaac Gym collide an actor's shapes with each other except on links joined
 * by a joint.  enable = 1 turns the model's pairs on (every actor of the sim must agree). */
int gs_sim_set_self_collision(gs_sim *sim, int enable);

/* Physics kernel selected by gs_sim_set_model: 1 one env per lane, 2 lane team, 3 host backend, 4 the
 * runtime-sized kernel (ABI 8: a topology with no compiled kernel -- any tree of revolute / prismatic joints with
 * plane contacts of sphere / capsule / cylinder / box candidates, joint limits, drives, per-actor dof properties;
 * one wave per env, dense joint-space rows; hull candidates, self-collision, terrain meshes and force sensors
 * need a compiled topology and are refused); -1 on error. */
int gs_sim_kernel_variant(gs_sim *sim);

/* Kernel time of the last gs_sim_pd_step / gs_sim_simulate launch measured with
 * HIP events on `stream` (ms; host backend: wall time of the call); -1 if not recorded.
 * Used by bench.py. */
int gs_sim_enable_timing(gs_sim *sim, int enable);
float gs_sim_last_kernel_ms(gs_sim *sim);

/* Profiling build only (libgymsim_prof.so, -DGS_PHASE_PROFILE): per-phase cycle sums of the
 * lane-team kernel over all waves since the last reset (tools/phase_profile.py); -1 otherwise. */
int gs_debug_phase_cycles(unsigned long long *out, int n, int reset);

/* Test hook: the terrain-mesh contact query of the physics kernels (gs_terrain.h)
 * for n spheres: centres [n][3] world, radii [n] (device pointers), threshold = r + contact_offset;
 * out [n][5] = (found, separation, normal xyz). */
int gs_debug_terrain_query(gs_sim *sim, const float *centres, const float *radii, int n, float *out, void *stream);

/* Test hook (ABI 6): each env's self-contact pool from the current sim state.
 * mode 0: the inline narrowphase of the one-env-per-lane / host forms; mode 1 (device, split-form topologies
 * such as UsefulHound): the near-pair records kernel then the records' gather, as the split simulate runs them.
 * out [N][npk][10] = contact point (3, relative to the root origin), normal (3, from shape b to shape a),
 * separation, friction, body a, body b; count [N] contacts kept (at most npk).  Device buffers on the GPU
 * pipeline (synchronises `stream`), host buffers on the host backend. */
int gs_debug_self_contacts(gs_sim *sim, int mode, float *out, int *count, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GYMSIM_H */
