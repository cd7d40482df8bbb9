// Internal (non-ABI) declarations shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>

#include "gs_terrain.h"
#include "../../include/gymtask.h"

#define GS_MAXB 32   // bodies per articulation
#define GS_MAXD 32   // dofs per articulation
#define GS_MAXC 192  // contact candidates per articulation (UsefulHound with its arm hulls: 175)
#define GS_MAXL 40   // reported links per articulation (fixed-joint links included)
#define GS_MAXS 8    // force sensors per articulation
#define GS_MAXSH 32  // collision shapes per articulation
#define GS_MAXHV 2048  // convex-hull vertices per articulation (UsefulHound's arm: 1503)
#define GS_MAXP 512   // self-collision shape pairs per articulation (UsefulHound: 253)
#define GS_MAXPV 512  // hull self-collision core vertices per articulation (UsefulHound: 7 x <= 48)
#define GS_MAXPOOL 8  // self-contact slots per env
#define GS_WAVE 64
// a SELF-contact row whose J M^-1 J^T falls below this -- an effective mass above 1000 kg, an overlap no dof can
// separate (UsefulHound's arm pinned on its trunk) -- takes no impulse; the oracle uses the same bound.  Ground
// and terrain rows always respond (a body heavier than 1000 kg still rests on the plane:
// tests/test_oracle_physics.py::test_heavy_body_rests_on_the_plane)
#ifndef GS_MIN_RESPONSE
#define GS_MIN_RESPONSE 1e-3f
#endif

// Model constants shared by every env, float32, one copy in device memory.
// Kernels index it with compile-time body / candidate indices from a uniform
// pointer, so every read lowers to a scalar (SGPR) load.
struct DevModel {
  float jR[GS_MAXB][9];      // parent frame -> joint frame rotation, row major
  float jt[GS_MAXB][3];      // parent frame -> joint frame translation
  float jaxis[GS_MAXB][3];   // joint axis in the joint frame
  float mass[GS_MAXB];
  float com[GS_MAXB][3];     // body frame
  float root_com[3];         // COM of the root LINK, body-0 frame (root tensor velocity point; = com[0]
                             // unless fixed-joint links are welded into the root body)
  float inertia[GS_MAXB][6]; // about COM, body axes: xx yy zz xy xz yz
  float cpoint[GS_MAXC][3];  // contact candidate, body frame
  float cradius[GS_MAXC];
  // per collision shape: bounding sphere of its candidates (body frame centre xyz, radius incl. the
  // candidates' own radii); a shape whose sphere clears the ground plane has no active candidate
  float shc[GS_MAXSH][4];
  float effort[GS_MAXD];     // <= 0 : unlimited
  float vmax[GS_MAXD];       // <= 0 : unlimited
  float armature[GS_MAXD];
  // joint drives (DOF_MODE_POS: stiffness + damping, DOF_MODE_VEL: damping; 0 otherwise), implicit
  // spring-damper folded into the substep's mass matrix and free velocity
  float dkp[GS_MAXD], dkd[GS_MAXD];
  float lower[GS_MAXD], upper[GS_MAXD];  // joint limits where has_lim
  int has_lim[GS_MAXD];
  int nsens;                    // force sensors (leaf bodies)
  int sens_of_body[GS_MAXB];    // sensor index of body b, -1 if none
  // ---- convex hulls and self-collision
  unsigned banc[GS_MAXB];       // bit a set: body a is b or an ancestor of b
  int shkind[GS_MAXSH];         // 0 sphere 1 capsule 2 box 3 cylinder 4 hull
  int shbody[GS_MAXSH], shlink[GS_MAXSH];
  float shR[GS_MAXSH][9], sht[GS_MAXSH][3];  // shape frame in the body frame
  float shsize[GS_MAXSH][3];    // sphere r | capsule r, half length | box half extents
  float shm[GS_MAXSH];          // core radius (pair narrowphase margin)
  int hv0[GS_MAXSH], hv1[GS_MAXSH];  // hull vertex range
  int np;                       // self-collision pairs
  int pa[GS_MAXP], pb[GS_MAXP], pk[GS_MAXP];  // shape a < shape b, kind 0 SS 1 SC 2 CC 3 GJK
  alignas(16) float hv[GS_MAXHV][4];  // (16-B rows: one dwordx4 load each) hull vertices, body frame xyz + core factor (core = c + f (v - c))
  int pv0[GS_MAXSH], pv1[GS_MAXSH];  // a hull's self-collision core vertices (subset of hv)
  alignas(16) float pv[GS_MAXPV][4];
};

struct DevParams {
  float h;               // substep length = dt / substeps
  int substeps;
  float g[3];
  int pos_iters, vel_iters;
  int tgs;               // physx.solver_type 1: TGS position sub-steps (every kernel form and the host backend)
  float contact_offset, rest_offset, max_depen_vel;
  float ground_mu;       // ground plane friction (0.5*(mu_shape + mu_ground) is the pair friction)
  int has_ground;
  int collect;           // contact_collection != 0
  float limit_margin;    // joint-limit rows are active within this distance
  int any_limits;        // some dof has limits (uniform: skips the limit rows entirely)
  int has_terrain;       // a heightfield triangle mesh is present (TERR kernels, gs_terrain.h)
  TerrainDev terr;
  int any_drive;         // some dof has drive gains (uniform: skips the drive terms entirely)
  int self_collide;      // filter-0 actors: self-collision pairs
  const float* ptgt;     // [N][nd] dof position targets or null (= 0)
  const float* vtgt;     // [N][nd] dof velocity targets or null (= 0)
  // per-actor dof properties (set_actor_dof_properties actor by actor; gs_sim_set_dof_properties_env):
  // [GS_DOFP_FIELDS][nd][N] -- drive stiffness, drive damping (after the drive-mode rule), effort, lower, upper
  // (lower >= upper: no limit), velocity limit; null = the model's per-asset values
  const float* dof_env;
  int dof_env_n;         // the table's env stride (N)
  // the runtime-sized kernel (gs_generic.hip, kernel_variant 4): its tree and candidate tables; null otherwise
  const struct GenTopo* gen;
  const struct DevLinks* gen_links;
  int gen_nd, gen_nr;
};
#define GS_DOFP_FIELDS 6

// SoA state: field f of env e at state[f*N + e]
//   0..2 root pos, 3..6 quat xyzw, 7..9 root ORIGIN lin vel, 10..12 ang vel,
//   13..13+nd-1 dof pos, 13+nd..13+2nd-1 dof vel
struct SimBuffers {
  float* state;
  const float* mu;       // [ns][N]
  float* cf;             // [3*nr][N]  (nr reported links)
  int N;
  float* sens;           // [6*nsens][N] force-sensor readings or null
  float* rows;           // contact-row tiles of the GLOBAL-row kernels (LaneCfg::GLOBAL), else null
};

// Candidate tables of the runtime-sized kernel (the compiled kernels have them as Topo_* constants)
struct GenTopo {
  int nc;
  int cbody[GS_MAXC], cshape[GS_MAXC], clink[GS_MAXC];
};

struct PdDev {
  const float* actions;      // [N][nd]
  const float* dof_state_in; // [N*nd][2] dof tensor as the task sees it (first PD uses it)
  const float* default_pos;  // [nd]
  float kp, kd, scale, tlim;
  int decimation, extra;
  float* torques_out;        // [N][nd]
  float* dof_out;            // [N*nd][2] or null
  float* root_out;           // [N][13]   or null
  float* cf_out;             // [N*nr][3] or null
  float* actions_copy;       // [N][nd]   or null
  // the AnymalTerrain tail (gymsim.h gs_pd_args.tail_*, gt_anymal_tail.h) run by the team kernel's last phase
  int tail_on;
  gt_anymal_params tail_p;
  gt_anymal_buffers tail_b;
};

bool team_fused_tail_available();  // gs_team.hip: the lane-team kernel can run PdDev's tail

typedef hipError_t (*launch_sim_fn)(const DevModel*, const DevParams&, const SimBuffers&, const float* tau,
                                    hipStream_t);
typedef hipError_t (*launch_pd_fn)(const DevModel*, const DevParams&, const SimBuffers&, const PdDev&,
                                   hipStream_t);

typedef hipError_t (*launch_dbg_pool_fn)(const DevModel*, const DevParams&, const SimBuffers&, int mode, float* out,
                                        int* count, hipStream_t);
struct TopoEntry {
  const char* sig;
  const char* name;
  launch_sim_fn sim;
  launch_pd_fn pd;
  launch_dbg_pool_fn dbg_pool;  // gs_debug_self_contacts
  int nb, nd, nc, ns;
  int sens;  // force sensors compiled in (T::SENS)
  int row_floats, row_lanes;  // SimBuffers::rows of the plane one-env-per-lane kernels: floats per env
                              // (0 = rows in LDS) and env lanes per workgroup (LaneCfg<T, false>)
  int npk;                    // self-contact pool slots (T::NPK)
  const int* cdyn;            // [nc] hull slot of each candidate (T::cdyn)
  int npair;                  // self-collision pair table (T::NPAIR, T::pair_a / pair_b / pair_k) and shape
  const int *pair_a, *pair_b, *pair_k, *shkind;  // kinds (T::shkind): the kernels unroll over them
};

// Kinematics of the reported links (gs_kinematics.hip): runtime-sized tree tables, one copy in
// device memory next to the DevModel.
struct DevLinks {
  int nb, nd, nr, fixed_base;
  int parent[GS_MAXB];
  int jkind[GS_MAXB];
  int bdof[GS_MAXB];
  unsigned anc_mask[GS_MAXB];  // bit a set: body a is b or an ancestor of b
  int dbody[GS_MAXD];          // body moved by dof j
  int lbody[GS_MAXL];
  float lR[GS_MAXL][9];        // link frame in the body frame
  float lt[GS_MAXL][3];
  float lcom[GS_MAXL][3];      // link COM, link frame
};

extern TopoEntry g_topologies[];
extern const int g_num_topologies;

// lane-team kernels (gs_team.hip) for "uniform star" topologies; null when not applicable
struct TeamEntry {
  const char* sig;
  launch_sim_fn sim;
  launch_pd_fn pd;
};
extern TeamEntry g_team_kernels[];
extern const int g_num_team_kernels;

// generic (runtime-sized) tensor API kernels
hipError_t launch_terrain_query(const DevParams& P, const float* c, const float* r, int n, float* out, hipStream_t s);
hipError_t launch_refresh_root(const float* state, int N, int nd, const float* com0, float* out, hipStream_t s);
hipError_t launch_refresh_dof(const float* state, int N, int nd, float* out, hipStream_t s);
hipError_t launch_refresh_contact(const float* cf, int N, int nb, float* out, hipStream_t s);
// mode bits: 1 rigid body state [N*nr][13], 2 jacobian [N][nr][6][nv], 4 mass matrix [N][nv][nv]
hipError_t launch_kinematics(const DevModel* M, const DevLinks* L, const float* state, int N, int nv, int mode,
                             float* rb, float* jac, float* mm, hipStream_t s);
hipError_t launch_refresh_sensor(const float* soa, int N, int ns, float* out, hipStream_t s);
hipError_t launch_set_root(float* state, int N, int nd, const float* com0, const float* src, const int* idx,
                           int n_idx, hipStream_t s);
hipError_t launch_set_root_dof(float* state, int N, int nd, const float* com0, const float* root, const float* dof,
                               const int* idx, int n, hipStream_t s);
hipError_t launch_set_dof(float* state, int N, int nd, const float* src, const int* idx, int n_idx,
                          hipStream_t s);
// the runtime-sized kernel (gs_generic.hip): workspace SimBuffers::rows = generic_ws_floats per env
hipError_t launch_sim_generic(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau,
                              hipStream_t st);
hipError_t launch_pd_generic(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A,
                             hipStream_t st);
inline size_t generic_ws_floats(int nc, int nd, int fixed_base) {
  return (size_t)2 * (3 * nc + nd) * ((fixed_base ? 0 : 6) + nd);
}

// ---------------------------------------------------------------- host backend (gs_host.hip)
// The sim_device=cpu pipeline: the same solver on host buffers, envs spread over a thread pool.
struct HostPool;
HostPool* host_pool_create(int threads);  // threads >= 1 (the calling thread included)
void host_pool_destroy(HostPool* p);
int host_pool_threads(const HostPool* p);
typedef void (*host_sim_fn)(const DevModel*, const DevParams&, const SimBuffers&, const float* tau, HostPool*);
typedef void (*host_pd_fn)(const DevModel*, const DevParams&, const SimBuffers&, const PdDev&, HostPool*);
typedef void (*host_dbg_pool_fn)(const DevModel*, const DevParams&, const SimBuffers&, float* out, int* count, HostPool*);
struct HostTopoEntry {
  const char* sig;
  host_sim_fn sim;
  host_pd_fn pd;
  host_dbg_pool_fn dbg_pool;  // gs_debug_self_contacts (inline narrowphase)
};
extern HostTopoEntry g_host_topologies[];
extern const int g_num_host_topologies;
void host_refresh_root(const float* st, int N, const float* com0, float* out, HostPool* pool);
void host_refresh_dof(const float* st, int N, int nd, float* out, HostPool* pool);
void host_soa_to_aos(const float* soa, int N, int n, int comp, float* out, HostPool* pool);
void host_set_root(float* st, int N, const float* com0, const float* src, const int* idx, int n);
void host_set_dof(float* st, int N, int nd, const float* src, const int* idx, int n);
void host_kinematics(const DevModel* M, const DevLinks* L, const float* st, int N, int nv, int mode, float* rb,
                     float* jac, float* mm, HostPool* pool);
void host_terrain_query(const DevParams& P, const float* c, const float* r, int n, float* out);
