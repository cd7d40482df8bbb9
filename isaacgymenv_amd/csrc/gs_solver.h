// gs_solver.h -- the per-env articulation + contact solver of libgymsim.
//
// One source, two backends: the one-env-per-lane HIP kernels (gs_physics.hip) run `substep` with
// the contact rows of LB lanes interleaved in LDS, the host backend (gs_host.hip, the reference's
// sim_device=cpu pipeline, vec_task.py:82-88) runs the very same function per env on a worker
// thread with LB = 1 and a thread-local scratch row.  Everything here is __host__ __device__;
// the few operations whose fast form differs per side are target overloads in gs_math.h.
#pragma once
#include "gs_internal.h"
#include "gs_topologies.h"
#include "gs_math.h"
#include "gs_pairs.h"

namespace {

// k-th node of the support path of a contact on the body moved by generalized dof
// `leaf`: the leaf itself, then its ancestors towards the root.
template <class T>
GS_HD constexpr int supp_node(int leaf, int si) {
  return si == 0 ? leaf : T::anc[leaf][si > 0 ? si - 1 : 0];
}

// body kk is b or one of its ancestors
template <class T>
GS_HD constexpr bool body_on_path(int kk, int b) {
  for (int x = b; x > 0; x = T::parent[x])
    if (x == kk) return true;
  return kk == 0;
}

// Lanes (= envs) per workgroup: a full wave unless the topology's LDS rows would exceed the
// 160 KB of LDS per CU (nv_ant: 25 candidates -> 748 slots -> 32 lanes).
// TERR kernels (trimesh terrain) keep each active candidate's contact normal in 3 more slots.
template <class T, bool TERR = false>
struct LaneCfg {
  // contact rows (NSLOT), [TERR: normals 3 NC], separation NC, friction NC, impulses 3 NC, self-contact pool
  static constexpr int X_POOL = T::NSLOT + (TERR ? 3 * T::NC : 0) + 5 * T::NC;
  static constexpr int SLOTS = X_POOL + PoolCfg<T>::FLOATS;
  // the self-collision prepass keeps the shapes' world data in the contact-row area (rows are written later)
  static_assert(T::NPK == 0 || kShW * T::NS <= T::NSLOT, "shape world data must fit the contact-row area");
  static_assert(T::NPK <= GS_MAXPOOL, "self-contact pool exceeds GS_MAXPOOL");
  static constexpr int FIT = (SLOTS * 64 * 4 <= 160 * 1024) ? 64 : (SLOTS * 32 * 4 <= 160 * 1024) ? 32
                           : (SLOTS * 16 * 4 <= 160 * 1024) ? 16 : 8;
  // Below 16 lanes the rows of two workgroups no longer share a CU, and halving again measured
  // ~10 % faster for Hound (2745 slots; r01n, profiles/r01n_experiments_other_configs.txt) while
  // Ant (32 lanes) got slower at 4: only the LDS-starved widths go narrower.  The mesh-contact
  // (TERR) kernels run LB env lanes in a 64-lane workgroup whose other lanes help with the terrain
  // queries (gs_physics.hip, k_*_terr): few env lanes = many query lanes per env.
#ifndef GS_NARROW_LANES
#define GS_NARROW_LANES 4
#endif
#ifndef GS_TERR_LANES
#define GS_TERR_LANES 4
#endif
  // LDS-starved topologies (FIT == 8): the widest of 4 / 2 / 1 env lanes that still lets 3 workgroups
  // share a CU (their kernels hold 512 VGPR+AGPR per lane, so at most 4 waves per CU anyway): UsefulHound
  // with its arm hulls (6,599 slots) runs 2 lanes, 3 workgroups per CU, instead of 4 lanes, 1 per CU
  static constexpr int NARROW = (SLOTS * 4 * 4 * 3 <= 160 * 1024) ? 4 : (SLOTS * 2 * 4 * 3 <= 160 * 1024) ? 2 : 1;
  // GLOBAL (compile knob GS_GLOBAL_LANES > 0, off by default): the LDS-starved plane kernels keep the
  // contact rows in a per-workgroup tile of device memory (SimBuffers::rows, [SLOTS][LB] per workgroup)
  // instead of LDS, so the lane count is no longer set by the 160 KB (GS_GLOBAL_LANES env lanes per wave;
  // 4 = 1024 waves, one per SIMD, at 4096 envs).  Same arithmetic, same order.  Measured r02x: UsefulHound
  // simulate 1.17 -> 2.34 ms per launch (the Gauss-Seidel chain waits on L2 latency instead of LDS), so
  // the default keeps the rows in LDS (profiles/r02x_experiment_global_rows.txt).
#ifndef GS_GLOBAL_LANES
#define GS_GLOBAL_LANES 0
#endif
  static constexpr bool GLOBAL = (FIT == 8) && !TERR && (GS_GLOBAL_LANES > 0);
  // GS_LANE_CAP: at most this many env lanes per workgroup for the others, so 4096 envs make >= 256
  // workgroups (one per CU) instead of 64-128: Ant simulate 0.136 -> 0.119 ms at 16 (32 = LDS fit),
  // 0.134 at 8, 0.163 at 4 (r02z A/B, profiles/r02z_experiment_lane_cap.txt)
#ifndef GS_LANE_CAP
#define GS_LANE_CAP 16
#endif
  static constexpr int LB = GLOBAL ? GS_GLOBAL_LANES
                          : FIT == 8 ? (GS_NARROW_LANES < NARROW ? GS_NARROW_LANES : NARROW)
                                     : (TERR && FIT > GS_TERR_LANES) ? GS_TERR_LANES
                                                                     : (FIT < GS_LANE_CAP ? FIT : GS_LANE_CAP);
  static_assert(GLOBAL || SLOTS * LB * 4 <= 160 * 1024, "contact rows exceed the LDS of a CU even at 8 lanes");
  // floats of SimBuffers::rows per env (0: the rows live in LDS)
  // SPLIT (plane, self-collision, LDS-starved: UsefulHound): the pair narrowphase runs as its own kernel before the
  // solver (gs_physics_impl.h k_pair_records) and hands over near-pair records in SimBuffers::rows, per env
  static constexpr bool SPLIT = T::NPK > 0 && !TERR && !GLOBAL && LB <= 4;
  static constexpr int ROW_FLOATS = GLOBAL ? SLOTS : SPLIT ? 1 + T::NPAIR * (1 + 2 * kRec) : 0;
};

// World-frame force of candidate c's impulses (normal from LDS, tangents rebuilt), / h.
template <class T, int LB>
GS_HD void contact_force_world(const float* lds, int c, const float* lam, float inv_h,
                                                    float* f) {
  const float* nsl = lds + (T::NSLOT + 3 * c) * LB;
  const float n[3] = {nsl[0], nsl[LB], nsl[2 * LB]};
  float t1[3], t2[3];
  gs_terrain::tangents(n, t1, t2);
#pragma unroll
  for (int k = 0; k < 3; ++k) f[k] = (lam[0] * n[k] + lam[1] * t1[k] + lam[2] * t2[k]) * inv_h;
}

// Register-resident env state.
template <class T>
struct EnvState {
  float p[3], quat[4], vo[3], w[3];
  float q[T::ND > 0 ? T::ND : 1], qd[T::ND > 0 ? T::ND : 1];
};

template <class T>
GS_HD void load_state(const float* __restrict__ st, int N, int e, EnvState<T>& s) {
#pragma unroll
  for (int k = 0; k < 3; ++k) s.p[k] = st[k * N + e];
#pragma unroll
  for (int k = 0; k < 4; ++k) s.quat[k] = st[(3 + k) * N + e];
#pragma unroll
  for (int k = 0; k < 3; ++k) s.vo[k] = st[(7 + k) * N + e];
#pragma unroll
  for (int k = 0; k < 3; ++k) s.w[k] = st[(10 + k) * N + e];
#pragma unroll
  for (int j = 0; j < T::ND; ++j) s.q[j] = st[(13 + j) * N + e];
#pragma unroll
  for (int j = 0; j < T::ND; ++j) s.qd[j] = st[(13 + T::ND + j) * N + e];
}
template <class T>
GS_HD void store_state(float* __restrict__ st, int N, int e, const EnvState<T>& s) {
#pragma unroll
  for (int k = 0; k < 3; ++k) st[k * N + e] = s.p[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) st[(3 + k) * N + e] = s.quat[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) st[(7 + k) * N + e] = s.vo[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) st[(10 + k) * N + e] = s.w[k];
#pragma unroll
  for (int j = 0; j < T::ND; ++j) st[(13 + j) * N + e] = s.q[j];
#pragma unroll
  for (int j = 0; j < T::ND; ++j) st[(13 + T::ND + j) * N + e] = s.qd[j];
}

// f(c) for every candidate c of every shape whose bit is set in shb, in candidate order; shapes are
// visited by compile-time recursion so each shape's candidate loop has constant bounds (and unrolls)
template <class T, int SH = 0, class F>
GS_HD __attribute__((always_inline)) void for_active_shapes(unsigned shb, F&& f) {
  if constexpr (SH < T::NS) {
    if ((shb >> SH) & 1u) {
#pragma unroll
      for (int c = T::sh_c0[SH]; c < T::sh_c1[SH]; ++c) f(c);
    }
    for_active_shapes<T, SH + 1>(shb, f);
  }
}

// Body rotations R_b and positions X_b relative to the root origin, exactly as substep's tree walk forms them.
template <class T>
GS_HD void body_poses(const DevModel* __restrict__ M, const EnvState<T>& s, float (&R)[T::NB][9], float (&X)[T::NB][3]) {
  constexpr int NB = T::NB;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    if (i == 0) {
      float qn[4];
      const float inv = gs_rsqrt(s.quat[0] * s.quat[0] + s.quat[1] * s.quat[1] + s.quat[2] * s.quat[2] +
                                 s.quat[3] * s.quat[3]);
#pragma unroll
      for (int k = 0; k < 4; ++k) qn[k] = s.quat[k] * inv;
      quat_to_mat(qn, R[0]);
      X[0][0] = X[0][1] = X[0][2] = 0.f;
    } else {
      const int pa = T::parent[i];
      float RJ[9], t[3], aw[3];
      mat3mul(R[pa], M->jR[i], RJ);
      mat3vec(R[pa], M->jt[i], t);
      X[i][0] = X[pa][0] + t[0]; X[i][1] = X[pa][1] + t[1]; X[i][2] = X[pa][2] + t[2];
      mat3vec(RJ, M->jaxis[i], aw);
      const float qj = s.q[T::bdof[i]];
      if (T::jkind[i] == 1) {
        float sn, cs;
        gs_sincos(qj, &sn, &cs);
        const float* a = M->jaxis[i];
        const float C = 1.f - cs;
        float Rq[9];
        Rq[0] = cs + a[0] * a[0] * C;        Rq[1] = a[0] * a[1] * C - a[2] * sn; Rq[2] = a[0] * a[2] * C + a[1] * sn;
        Rq[3] = a[1] * a[0] * C + a[2] * sn; Rq[4] = cs + a[1] * a[1] * C;        Rq[5] = a[1] * a[2] * C - a[0] * sn;
        Rq[6] = a[2] * a[0] * C - a[1] * sn; Rq[7] = a[2] * a[1] * C + a[0] * sn; Rq[8] = cs + a[2] * a[2] * C;
        mat3mul(RJ, Rq, R[i]);
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) R[i][k] = RJ[k];
        X[i][0] += aw[0] * qj; X[i][1] += aw[1] * qj; X[i][2] += aw[2] * qj;
      }
    }
  }
}

// One substep for one env.  `lds` points at this lane's column of the
// workgroup's [SLOTS][LB] contact-row staging area (LB = 1 in the host backend: a per-thread
// scratch row).
//
// Register budget: the tree is walked ONCE in DFS order.  Kinematics,
// velocities, RNEA forces and composite inertias are accumulated post-order,
// so only the bodies on the current root->leaf path are live at any time; a
// body's bias force and its mass-matrix row are emitted the moment its subtree
// is complete (T::subend).  Contact Jacobian rows are written to LDS during the
// same walk (they need the path's motion subspaces) and turned into scaled
// Z rows after the factorisation.
// Shape world data of env state s for the self-collision narrowphase (gs_pairs.h layout: [kShW * sh + f] at
// stride LB): R (9), centre (3), bounding-sphere centre (3), relative to the root origin.  Written into the
// contact-row area, which the substep fills only after its narrowphase.
template <class T, int LB>
GS_HD void shape_world(const DevModel* __restrict__ Min, const EnvState<T>& s, float* lds) {
  constexpr int NB = T::NB;
  const DevModel* __restrict__ M = gs_opaque(Min);
  float Rb[NB][9], Xb[NB][3];
  body_poses<T>(M, s, Rb, Xb);
#pragma unroll
  for (int sh = 0; sh < T::NS; ++sh) {
    const int b = T::sh_body[sh];
    float Rs[9], t[3];
    mat3mul(Rb[b], M->shR[sh], Rs);
    float* o = lds + kShW * sh * LB;
#pragma unroll
    for (int k = 0; k < 9; ++k) o[k * LB] = Rs[k];
    mat3vec(Rb[b], M->sht[sh], t);
#pragma unroll
    for (int k = 0; k < 3; ++k) o[(9 + k) * LB] = Xb[b][k] + t[k];
    mat3vec(Rb[b], M->shc[sh], t);
#pragma unroll
    for (int k = 0; k < 3; ++k) o[(12 + k) * LB] = Xb[b][k] + t[k];
  }
}

// Near-pair records of the wave-assisted kernels (gs_physics_impl.h pair_records), at stride PR from a base:
// in each env's LDS column behind its shape world data (base SHW, written before the contact rows reuse that area),
// or per env in SimBuffers::rows (LaneCfg::SPLIT, FLOATS per env).  [0] the env's count of pairs within reach of
// the broadphase; record r (its r-th such pair, in pair order) at 1 + RW r: q + kRecQ * (contact count), then
// contact c's x, n, separation at 1 + kRec c.
constexpr int kRecQ = 1024;
template <class T>
struct NearRec {
  static constexpr int SHW = kShW * T::NS, RW = 1 + 2 * kRec, FLOATS = 1 + T::NPAIR * RW, END = SHW + FLOATS;
  static_assert(T::NPAIR < kRecQ, "pair index must fit below kRecQ");
};

// the env's near-pair records gathered in pair order into the pool, at most T::NPK -- the entries
// self_contacts writes for the same shapes
template <class T, int LB, int PR>
GS_HD int pool_from_records(const DevModel* __restrict__ M, const float* __restrict__ mu_g, int N, int e,
                            const float* __restrict__ col, float* pool) {
  using R = NearRec<T>;
  constexpr int PE = PoolCfg<T>::PE;
  const int cnt = (int)col[0];
  int n = 0;
  for (int r = 0; r < cnt && n < T::NPK; ++r) {
    const float* rec = col + (1 + R::RW * r) * PR;
    const int code = (int)rec[0];
    const int q = code % kRecQ, nc = code / kRecQ;
    for (int c = 0; c < nc && n < T::NPK; ++c) {
      const float* x = rec + (1 + c * kRec) * PR;
      float* o = pool + PE * n * LB;
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k * LB] = x[k * PR];
      o[kPoolSep * LB] = x[kRecSep * PR];
      pool_entry_finish<LB>(M, mu_g, N, e, M->pa[q], M->pb[q], o);
      ++n;
    }
  }
  return n;
}

// QS > 0 (TERR kernels): the terrain queries of this substep were already run by the whole workgroup
// (terrain_queries, gs_physics.hip) and `qres` holds this env's results, [5 * c + k][QS] for
// candidate c: (found, separation, normal xyz); QS == 0 runs each candidate's query inline.
// SELF = false compiles the self-collision path out (kernels launched for sims without it)
// PR > 0 (wave-assisted kernels): the self-collision narrowphase of this substep was already run by the whole
// workgroup (pair_records, gs_physics_impl.h) on the shape world data shape_world wrote, and `prec` holds this
// env's pair records at stride PR (pair_records' layout); the prepass only gathers them into the pool.
template <class T, bool TERR, int LB = LaneCfg<T, TERR>::LB, int QS = 0, bool SELF = true, int PR = 0>
GS_HD void substep(const DevModel* __restrict__ Min, const DevParams& P, EnvState<T>& s,
                                        const float* tau, const float* __restrict__ mu_g, int N, int e, float* lds,
                                        float* __restrict__ cf_soa, bool collect, float* __restrict__ sens_soa,
                   const float* __restrict__ qres = nullptr, const float* __restrict__ prec = nullptr) {
  constexpr int NB = T::NB, NV = T::NV, NB6 = T::NBASE, NC = T::NC, ND = T::ND;
  constexpr int MS = T::MAXDEP + 1;
  // Keep the model pointer opaque per substep: the constants are re-read with
  // scalar loads (K$ hits) instead of being hoisted out of the substep loop
  // into hundreds of SGPRs.
  const DevModel* __restrict__ M = gs_opaque(Min);
  const float h = P.h;

  // ---- self-collision prepass: shape world data into the (not yet written) contact-row
  // area, narrowphase into the self-contact pool; the pool's J rows are filled during the tree walk
  constexpr int XP = LaneCfg<T, TERR>::X_POOL;
  constexpr int PE = PoolCfg<T>::PE;
  float* pool = lds + XP * LB;
  int npc = 0;
  if constexpr (T::NPK > 0 && SELF) {
    if (P.self_collide) {
      if constexpr (PR > 0) {
        npc = pool_from_records<T, LB, PR>(M, mu_g, N, e, prec, pool);
      } else {
        shape_world<T, LB>(M, s, lds);
        npc = self_contacts<T, LB>(M, P, mu_g, N, e, lds, pool);
      }
      for (int p = 0; p < npc; ++p)
        for (int k = 0; k < 3 * NV; ++k) pool[(PE * p + kPoolJ + k) * LB] = 0.f;
    }
  }

  float nu[NV];
  if (NB6) {
    nu[0] = s.w[0]; nu[1] = s.w[1]; nu[2] = s.w[2];
    nu[3] = s.vo[0]; nu[4] = s.vo[1]; nu[5] = s.vo[2];
  }
#pragma unroll
  for (int j = 0; j < T::ND; ++j) nu[NB6 + j] = s.qd[j];

  // per-actor dof property f of dof j (GS_DOFP_FIELDS order), else the asset's value mv
  auto dofp = [&](int f, int j, float mv) -> float {
    return P.dof_env ? P.dof_env[((size_t)f * ND + j) * P.dof_env_n + e] : mv;
  };
  // joint drives: the drive force estimate kp (q* - q - h qd) + kd (qd* - qd) of each dof;
  // within the dof's effort limit the drive is implicit ((h kd + h^2 kp) on M's diagonal), a saturated drive
  // applies the clamped force explicitly (PhysX: the drive's max force is the dof's effort property)
  float dforce[ND > 0 ? ND : 1];
  bool dimpl[ND > 0 ? ND : 1];
  if (P.any_drive) {
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float pt = P.ptgt ? P.ptgt[(size_t)e * ND + j] : 0.f;
      const float vt = P.vtgt ? P.vtgt[(size_t)e * ND + j] : 0.f;
      const float f = dofp(0, j, M->dkp[j]) * (pt - s.q[j] - h * s.qd[j]) + dofp(1, j, M->dkd[j]) * (vt - s.qd[j]);
      const float ef = dofp(2, j, M->effort[j]);
      dimpl[j] = !(ef > 0.f) || fabsf(f) <= ef;
      dforce[j] = dimpl[j] ? f : clampf(f, -ef, ef);
    }
  }

  float R[NB][9], X[NB][3], S[NB][6], V[NB][6], A[NB][6], Fc[NB][6];
  SpI Ic[NB];
  float Mm[NV][NV], bias[NV];
  // per-candidate activity as per-lane bits; separation, friction and impulses live in the lane's LDS
  // column (slots XS...: compile-time offsets), so an 84-candidate robot does not spill them to scratch
  constexpr int XS = T::NSLOT + (TERR ? 3 * NC : 0);
  constexpr int X_SEP = XS, X_MU = XS + NC, X_LAM = XS + 2 * NC;
  unsigned actb[(NC + 31) / 32];
#pragma unroll
  for (int w = 0; w < (NC + 31) / 32; ++w) actb[w] = 0u;
#define GS_ACT(c) ((actb[(c) >> 5] >> ((c) & 31)) & 1u)
  // shapes with an active candidate: the row, impulse and sweep loops visit only their candidates
  // (same global candidate order: shapes in order, a shape's candidates contiguous)
  static_assert(T::NS <= 32, "shape activity is one 32-bit word");
  unsigned shb = 0u;

#pragma unroll
  for (int i = 0; i < NB; ++i) {
    // ---- kinematics of body i (positions relative to the root origin)
    if (i == 0) {
      float qn[4];
      const float inv = gs_rsqrt(s.quat[0] * s.quat[0] + s.quat[1] * s.quat[1] + s.quat[2] * s.quat[2] +
                               s.quat[3] * s.quat[3]);
#pragma unroll
      for (int k = 0; k < 4; ++k) qn[k] = s.quat[k] * inv;
      quat_to_mat(qn, R[0]);
      X[0][0] = X[0][1] = X[0][2] = 0.f;
#pragma unroll
      for (int k = 0; k < 6; ++k) V[0][k] = NB6 ? nu[k] : 0.f;
      A[0][0] = A[0][1] = A[0][2] = 0.f;
      A[0][3] = -P.g[0]; A[0][4] = -P.g[1]; A[0][5] = -P.g[2];
    } else {
      const int pa = T::parent[i];
      float RJ[9], t[3], aw[3];
      mat3mul(R[pa], M->jR[i], RJ);
      mat3vec(R[pa], M->jt[i], t);
      X[i][0] = X[pa][0] + t[0]; X[i][1] = X[pa][1] + t[1]; X[i][2] = X[pa][2] + t[2];
      mat3vec(RJ, M->jaxis[i], aw);
      const float qj = s.q[T::bdof[i]];
      if (T::jkind[i] == 1) {
        float sn, cs;
        gs_sincos(qj, &sn, &cs);
        const float* a = M->jaxis[i];
        const float C = 1.f - cs;
        float Rq[9];
        Rq[0] = cs + a[0] * a[0] * C;        Rq[1] = a[0] * a[1] * C - a[2] * sn; Rq[2] = a[0] * a[2] * C + a[1] * sn;
        Rq[3] = a[1] * a[0] * C + a[2] * sn; Rq[4] = cs + a[1] * a[1] * C;        Rq[5] = a[1] * a[2] * C - a[0] * sn;
        Rq[6] = a[2] * a[0] * C - a[1] * sn; Rq[7] = a[2] * a[1] * C + a[0] * sn; Rq[8] = cs + a[2] * a[2] * C;
        mat3mul(RJ, Rq, R[i]);
        S[i][0] = aw[0]; S[i][1] = aw[1]; S[i][2] = aw[2];
        cross3(X[i], aw, &S[i][3]);
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) R[i][k] = RJ[k];
        X[i][0] += aw[0] * qj; X[i][1] += aw[1] * qj; X[i][2] += aw[2] * qj;
        S[i][0] = S[i][1] = S[i][2] = 0.f;
        S[i][3] = aw[0]; S[i][4] = aw[1]; S[i][5] = aw[2];
      }
      const float qd = nu[NB6 + T::bdof[i]];
      float c6[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) V[i][k] = V[pa][k] + S[i][k] * qd;
      crm(V[i], S[i], c6);
#pragma unroll
      for (int k = 0; k < 6; ++k) A[i][k] = A[pa][k] + c6[k] * qd;
    }

    // ---- self-contact rows, column of body i's dof: n.(v_A(x) - v_B(x)) takes S_i's velocity at x when i is on
    // A's path and minus it on B's (a common ancestor's column cancels; the base columns always do)
    if constexpr (T::NPK > 0 && SELF) {
      if (i > 0) {
        const int col = NB6 + T::bdof[i];
        // (unrolled over the pool with a guard: a runtime loop here would carry the tree walk's registers
        // across its back edge -- ~4 KB of scratch per lane measured)
#pragma unroll
        for (int p = 0; p < T::NPK; ++p) {
          if (p >= npc) continue;  // (a guard, not an exit: the loop stays fully unrolled)
          float* o = pool + PE * p * LB;
          const int ba = (int)o[kPoolBA * LB], bb = (int)o[kPoolBB * LB];
          const float coef = (float)((M->banc[ba] >> i) & 1u) - (float)((M->banc[bb] >> i) & 1u);
          if (coef != 0.f) {
            const float x[3] = {o[kPoolX * LB], o[(kPoolX + 1) * LB], o[(kPoolX + 2) * LB]};
            float vx[3];  // velocity of the point x under S_i: S_lin + S_ang x x
            cross3(S[i], x, vx);
#pragma unroll
            for (int k = 0; k < 3; ++k) vx[k] += S[i][3 + k];
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
              const int dofs = rr == 0 ? kPoolN : (rr == 1 ? kPoolT1 : kPoolT2);
              const float d[3] = {o[dofs * LB], o[(dofs + 1) * LB], o[(dofs + 2) * LB]};
              o[(kPoolJ + rr * NV + col) * LB] = coef * dot3f(d, vx);
            }
          }
        }
      }
    }

    // ---- spatial inertia of body i at O; RNEA force
    {
      float c[3];
      mat3vec(R[i], M->com[i], c);
      c[0] += X[i][0]; c[1] += X[i][1]; c[2] += X[i][2];
      const float* Il = M->inertia[i];  // xx yy zz xy xz yz
      const float* Rm = R[i];
      float Am[9];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        Am[3 * r + 0] = Rm[3 * r] * Il[0] + Rm[3 * r + 1] * Il[3] + Rm[3 * r + 2] * Il[4];
        Am[3 * r + 1] = Rm[3 * r] * Il[3] + Rm[3 * r + 1] * Il[1] + Rm[3 * r + 2] * Il[5];
        Am[3 * r + 2] = Rm[3 * r] * Il[4] + Rm[3 * r + 1] * Il[5] + Rm[3 * r + 2] * Il[2];
      }
      const float m = M->mass[i];
      const float cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
      SpI& I = Ic[i];
      I.m = m;
      I.h[0] = m * c[0]; I.h[1] = m * c[1]; I.h[2] = m * c[2];
      I.I[0] = Am[0] * Rm[0] + Am[1] * Rm[1] + Am[2] * Rm[2] + m * (cc - c[0] * c[0]);
      I.I[1] = Am[3] * Rm[3] + Am[4] * Rm[4] + Am[5] * Rm[5] + m * (cc - c[1] * c[1]);
      I.I[2] = Am[6] * Rm[6] + Am[7] * Rm[7] + Am[8] * Rm[8] + m * (cc - c[2] * c[2]);
      I.I[3] = Am[0] * Rm[3] + Am[1] * Rm[4] + Am[2] * Rm[5] - m * c[0] * c[1];
      I.I[4] = Am[0] * Rm[6] + Am[1] * Rm[7] + Am[2] * Rm[8] - m * c[0] * c[2];
      I.I[5] = Am[3] * Rm[6] + Am[4] * Rm[7] + Am[5] * Rm[8] - m * c[1] * c[2];
      float ia[6], iv[6], x6[6];
      spi_mul(I, A[i], ia);
      spi_mul(I, V[i], iv);
      crf(V[i], iv, x6);
#pragma unroll
      for (int k = 0; k < 6; ++k) Fc[i][k] = ia[k] + x6[k];
    }

    // ---- contact candidates on body i: activity test + Jacobian rows -> LDS
    // Plane: a shape whose bounding sphere clears the ground by contact_offset has no active candidate
    // (exact: every candidate lies inside the sphere), so its candidates are not even transformed --
    // boxes and mesh hulls away from the ground cost one test per shape instead of one per point.
    bool shape_near[T::NS];
    int hsel[T::NS][4], hn[T::NS];
#pragma unroll
    for (int sh = 0; sh < T::NS; ++sh) {
      shape_near[sh] = true;
      hn[sh] = 0;
      if constexpr (!TERR) {
        if (T::sh_body[sh] == i && T::sh_c1[sh] - T::sh_c0[sh] > 1) {
          const float* sc = M->shc[sh];
          const float cz = s.p[2] + X[i][2] + R[i][6] * sc[0] + R[i][7] * sc[1] + R[i][8] * sc[2];
          shape_near[sh] = P.has_ground && (cz - sc[3] < P.contact_offset);
        }
      }
      // a convex hull's ground contacts: the 4-point manifold of its vertices (plane only)
      if (T::shkind[sh] == 4 && T::sh_body[sh] == i && shape_near[sh] && P.has_ground)
        hn[sh] = hull_ground_select(M, sh, R[i], X[i], s.p[2], P.contact_offset, hsel[sh]);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (T::cbody[c] == i && shape_near[T::cshape[c]] && (T::cdyn[c] < 0 || T::cdyn[c] < hn[T::cshape[c]])) {
        float x[3];
        mat3vec(R[i], T::cdyn[c] < 0 ? M->cpoint[c] : M->hv[hsel[T::cshape[c]][T::cdyn[c] & 3]], x);
        x[0] += X[i][0]; x[1] += X[i][1]; x[2] += X[i][2];
        const float r = M->cradius[c];
        if constexpr (TERR) {
          // deepest of the ground plane and the terrain mesh (gs_terrain.h); the contact frame is
          // (n, t1, t2) with n stored in LDS for the force outputs
          const float cw[3] = {s.p[0] + x[0], s.p[1] + x[1], s.p[2] + x[2]};
          float dist = P.has_ground ? cw[2] - r : 3.0e38f;
          float nrm[3] = {0.f, 0.f, 1.f};
          float smu = P.ground_mu;
          float st, nt[3];
          bool found;
          if (T::cdyn[c] >= 0) {  // hull slots: ground plane only
            found = false;
          } else if constexpr (QS > 0) {
            found = qres[(5 * c) * QS] != 0.f;
            st = qres[(5 * c + 1) * QS];
            nt[0] = qres[(5 * c + 2) * QS]; nt[1] = qres[(5 * c + 3) * QS]; nt[2] = qres[(5 * c + 4) * QS];
          } else {
            found = gs_terrain::sphere_contact(P.terr, cw, r, r + P.contact_offset, st, nt);
          }
          if (found && st < dist) {
            dist = st;
            nrm[0] = nt[0]; nrm[1] = nt[1]; nrm[2] = nt[2];
            smu = P.terr.mu;
          }
          const bool actc = dist < P.contact_offset;
          if (actc) {
            actb[c >> 5] |= 1u << (c & 31);  shb |= 1u << T::cshape[c];
            lds[(X_SEP + c) * LB] = dist - P.rest_offset;
            lds[(X_MU + c) * LB] = 0.5f * (mu_g[T::cshape[c] * N + e] + smu);
            float* nsl = lds + (T::NSLOT + 3 * c) * LB;
            nsl[0] = nrm[0]; nsl[LB] = nrm[1]; nsl[2 * LB] = nrm[2];
            float dir[3][3];
            dir[0][0] = nrm[0]; dir[0][1] = nrm[1]; dir[0][2] = nrm[2];
            gs_terrain::tangents(nrm, dir[1], dir[2]);
            const float xc[3] = {x[0] - r * nrm[0], x[1] - r * nrm[1], x[2] - r * nrm[2]};
            const int SUP = T::csupp[c];
            const int leaf = T::cleaf[c];
            float* slot = lds + T::cslot[c] * LB;
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
              const float* d = dir[rr];
              float xd[3];  // the row's angular part: d.(w x xc) = w.(xc x d)
              cross3(xc, d, xd);
#pragma unroll
              for (int si = 0; si < MS; ++si) {
                if (si < SUP) {
                  const int k = supp_node<T>(leaf, si);
                  float v;
                  if (k < NB6) {
                    v = k < 3 ? xd[k] : d[k - 3];
                  } else {
                    const float* Sk = S[T::gbody[k]];
                    v = Sk[3] * d[0] + Sk[4] * d[1] + Sk[5] * d[2] + Sk[0] * xd[0] + Sk[1] * xd[1] + Sk[2] * xd[2];
                  }
                  slot[(rr * SUP + si) * LB] = v;
                }
              }
            }
          }
        } else {
        const float dist = s.p[2] + x[2] - r;
        const bool actc = P.has_ground && (dist < P.contact_offset);
        if (actc) {
          actb[c >> 5] |= 1u << (c & 31);  shb |= 1u << T::cshape[c];
          lds[(X_SEP + c) * LB] = dist - P.rest_offset;
          lds[(X_MU + c) * LB] = 0.5f * (mu_g[T::cshape[c] * N + e] + P.ground_mu);
          const float xc[3] = {x[0], x[1], x[2] - r};
          const int SUP = T::csupp[c];
          const int leaf = T::cleaf[c];
          float* slot = lds + T::cslot[c] * LB;
#pragma unroll
          for (int rr = 0; rr < 3; ++rr) {
            const int ax = (rr == 0) ? 2 : (rr == 1 ? 0 : 1);  // normal z, tangent x, tangent y
#pragma unroll
            for (int si = 0; si < MS; ++si) {
              if (si < SUP) {
                const int k = supp_node<T>(leaf, si);
                float v;
                if (k < NB6) {
                  if (k < 3) {
                    const float m3[3][3] = {{0.f, xc[2], -xc[1]}, {-xc[2], 0.f, xc[0]}, {xc[1], -xc[0], 0.f}};
                    v = m3[ax][k];  // d(w x xc)/dw = -[xc]x
                  } else {
                    v = (ax == k - 3) ? 1.f : 0.f;
                  }
                } else {
                  const float* Sk = S[T::gbody[k]];
                  float t[3];
                  cross3(Sk, xc, t);
                  v = Sk[3 + ax] + t[ax];
                }
                slot[(rr * SUP + si) * LB] = v;
              }
            }
          }
        }
        }  // !TERR
      }
    }

    // ---- subtrees completed at body i: bias + mass-matrix rows, then fold into the parent
#pragma unroll
    for (int a = NB - 1; a >= 0; --a) {
      if (a <= i && T::subend[a] == i && (a == i || true)) {
        bool on_path = false;
        // a must be i or an ancestor of i (subend == i implies that)
        on_path = true;
        if (on_path) {
          if (a > 0) {
            const int ga = NB6 + T::bdof[a];
            bias[ga] = dot6(S[a], Fc[a]);
            float F[6];
            spi_mul(Ic[a], S[a], F);
            Mm[ga][ga] = dot6(S[a], F) + M->armature[T::bdof[a]];
            if (P.any_drive && dimpl[T::bdof[a]])
              Mm[ga][ga] += h * (dofp(1, T::bdof[a], M->dkd[T::bdof[a]]) + h * dofp(0, T::bdof[a], M->dkp[T::bdof[a]]));
#pragma unroll
            for (int k = 0; k < T::MAXDEP; ++k) {
              if (k < T::depth[ga]) {
                const int an = T::anc[ga][k];
                if (an >= NB6) Mm[ga][an] = dot6(S[T::gbody[an]], F);
                else Mm[ga][an] = F[an];
              }
            }
            const int pa = T::parent[a];
            Ic[pa].m += Ic[a].m;
#pragma unroll
            for (int k = 0; k < 3; ++k) Ic[pa].h[k] += Ic[a].h[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) Ic[pa].I[k] += Ic[a].I[k];
#pragma unroll
            for (int k = 0; k < 6; ++k) Fc[pa][k] += Fc[a][k];
          } else if (NB6) {
#pragma unroll
            for (int k = 0; k < 6; ++k) bias[k] = Fc[0][k];
            const SpI& I0 = Ic[0];
            Mm[0][0] = I0.I[0]; Mm[1][1] = I0.I[1]; Mm[2][2] = I0.I[2];
            Mm[1][0] = I0.I[3]; Mm[2][0] = I0.I[4]; Mm[2][1] = I0.I[5];
            Mm[3][0] = 0.f;       Mm[3][1] = I0.h[2];  Mm[3][2] = -I0.h[1];
            Mm[4][0] = -I0.h[2];  Mm[4][1] = 0.f;      Mm[4][2] = I0.h[0];
            Mm[5][0] = I0.h[1];   Mm[5][1] = -I0.h[0]; Mm[5][2] = 0.f;
            Mm[3][3] = I0.m; Mm[4][4] = I0.m; Mm[5][5] = I0.m;
            Mm[4][3] = 0.f; Mm[5][3] = 0.f; Mm[5][4] = 0.f;
          }
        }
      }
    }
  }

  // ---------------- joint-limit activity (substep start): one unilateral row per dof within
  // limit_margin of a limit; sign +1 pushes q up (lower limit), -1 down (upper limit)
  float lsgn[ND > 0 ? ND : 1], lsep[ND > 0 ? ND : 1];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    lsgn[j] = 0.f;
    lsep[j] = 0.f;
    const float lwr = dofp(3, j, M->lower[j]), upr = dofp(4, j, M->upper[j]);
    if (P.any_limits && (P.dof_env ? lwr < upr : M->has_lim[j] != 0)) {
      const float lo = s.q[j] - lwr, hi = upr - s.q[j];
      if (lo < P.limit_margin || hi < P.limit_margin) {
        lsgn[j] = lo <= hi ? 1.f : -1.f;
        lsep[j] = lo <= hi ? lo : hi;
      }
    }
  }

  // ---------------- L^T D L (Featherstone, tree-sparse, in place)
#pragma unroll
  for (int kk = 0; kk < NV; ++kk) {
    const int k = NV - 1 - kk;
    const float dinv = 1.f / Mm[k][k];
#pragma unroll
    for (int ai = 0; ai < T::MAXDEP; ++ai) {
      if (ai < T::depth[k]) {
        const int i = T::anc[k][ai];
        const float a = Mm[k][i] * dinv;
#pragma unroll
        for (int aj = ai; aj < T::MAXDEP; ++aj) {
          if (aj < T::depth[k]) {
            const int j = T::anc[k][aj];
            Mm[i][j] -= a * Mm[k][j];
          }
        }
        Mm[k][i] = a;
      }
    }
  }
  float sD[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) sD[k] = gs_rsqrt(Mm[k][k]);

  // ---------------- free velocity: nu_f = nu + h M^-1 (tau - c) (+ mixed-frame term)
  float nuf[NV];
  {
    float r[NV];
    if (NB6) {
#pragma unroll
      for (int k = 0; k < 6; ++k) r[k] = -bias[k];
    }
#pragma unroll
    for (int j = 0; j < T::ND; ++j) {
      float t = tau[j];
      const float ef = dofp(2, j, M->effort[j]);
      if (ef > 0.f) t = clampf(t, -ef, ef);
      r[NB6 + j] = t - bias[NB6 + j];
      if (P.any_drive) r[NB6 + j] += dforce[j];
    }
#pragma unroll
    for (int kk = 0; kk < NV; ++kk) {
      const int k = NV - 1 - kk;
#pragma unroll
      for (int ai = 0; ai < T::MAXDEP; ++ai)
        if (ai < T::depth[k]) r[T::anc[k][ai]] -= Mm[k][T::anc[k][ai]] * r[k];
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) r[k] *= sD[k] * sD[k];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
      for (int ai = 0; ai < T::MAXDEP; ++ai)
        if (ai < T::depth[k]) r[k] -= Mm[k][T::anc[k][ai]] * r[T::anc[k][ai]];
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) nuf[k] = nu[k] + h * r[k];
    if (NB6) {
      float wxp[3];
      cross3(&nu[0], &nu[3], wxp);
      nuf[3] += h * wxp[0]; nuf[4] += h * wxp[1]; nuf[5] += h * wxp[2];
    }
  }

  // ---------------- contact rows: J (LDS) -> c = J nu_f, scaled Z = (L^-T J^T) D^-1/2, 1/diag
  for_active_shapes<T>(shb, [&](const int c) {
    if (GS_ACT(c)) {
      const int SUP = T::csupp[c];
      const int leaf = T::cleaf[c];
      float* slot = lds + T::cslot[c] * LB;
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        float jv[MS];
        float cj = 0.f;
#pragma unroll
        for (int si = 0; si < MS; ++si) {
          if (si < SUP) {
            jv[si] = slot[(rr * SUP + si) * LB];
            cj += jv[si] * nuf[supp_node<T>(leaf, si)];
          }
        }
#pragma unroll
        for (int si = 0; si < MS; ++si) {
          if (si < SUP) {
            const int k = supp_node<T>(leaf, si);
#pragma unroll
            for (int sj = si + 1; sj < MS; ++sj)
              if (sj < SUP) jv[sj] -= Mm[k][supp_node<T>(leaf, sj)] * jv[si];
          }
        }
        float d = 0.f;
#pragma unroll
        for (int si = 0; si < MS; ++si) {
          if (si < SUP) {
            const float zh = jv[si] * sD[supp_node<T>(leaf, si)];
            d += zh * zh;
            slot[(rr * SUP + si) * LB] = zh;
          }
        }
        slot[(3 * SUP + rr) * LB] = cj;
        // (ground rows: no response cutoff; a row the articulation cannot move along -- d == 0, e.g. a
        // fixed-base planar chain's off-plane tangent -- takes no impulse instead of 0 * inf)
        slot[(3 * SUP + 3 + rr) * LB] = d > 0.f ? 1.f / d : 0.f;
      }
    }
  });

  // ---------------- joint-limit rows: J = sign * e_dof -> c, scaled Z, 1/diag (same elimination)
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    if (lsgn[j] != 0.f) {
      const int SUP = T::lsupp[j];
      const int leaf = T::lleaf[j];
      float* slot = lds + T::lslot[j] * LB;
      float jv[MS];
#pragma unroll
      for (int si = 0; si < MS; ++si) jv[si] = si == 0 ? lsgn[j] : 0.f;
#pragma unroll
      for (int si = 0; si < MS; ++si) {
        if (si < SUP) {
          const int k = supp_node<T>(leaf, si);
#pragma unroll
          for (int sj = si + 1; sj < MS; ++sj)
            if (sj < SUP) jv[sj] -= Mm[k][supp_node<T>(leaf, sj)] * jv[si];
        }
      }
      float d = 0.f;
#pragma unroll
      for (int si = 0; si < MS; ++si) {
        if (si < SUP) {
          const float zh = jv[si] * sD[supp_node<T>(leaf, si)];
          d += zh * zh;
          slot[si * LB] = zh;
        }
      }
      slot[SUP * LB] = lsgn[j] * nuf[leaf];
      slot[(SUP + 1) * LB] = d > 0.f ? 1.f / d : 0.f;
    }
  }

  // ---------------- self-contact rows: dense J over the tree -> c = J nu_f, scaled Z = (L^-T J^T) D^-1/2, 1/diag
  if constexpr (T::NPK > 0 && SELF) {
#pragma unroll
    for (int p = 0; p < T::NPK; ++p) {
      if (p >= npc) continue;
      float* o = pool + PE * p * LB;
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        float jv[NV];
        float cj = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          jv[k] = o[(kPoolJ + rr * NV + k) * LB];
          cj += jv[k] * nuf[k];
        }
#pragma unroll
        for (int kk = 0; kk < NV; ++kk) {
          const int k = NV - 1 - kk;
#pragma unroll
          for (int ai = 0; ai < T::MAXDEP; ++ai)
            if (ai < T::depth[k]) jv[T::anc[k][ai]] -= Mm[k][T::anc[k][ai]] * jv[k];
        }
        float d = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const float zh = jv[k] * sD[k];
          d += zh * zh;
          o[(kPoolJ + rr * NV + k) * LB] = zh;
        }
        o[(kPoolC + rr) * LB] = cj;
        o[(kPoolDi + rr) * LB] = d > GS_MIN_RESPONSE ? 1.f / d : 0.f;
        o[(kPoolLam + rr) * LB] = 0.f;
      }
    }
  }

  // ---------------- projected Gauss-Seidel in w-space (joint limits, then contacts)
  float wt[NV], wpos[NV], laml[ND > 0 ? ND : 1];
  float* lamc = lds + X_LAM * LB;  // impulses of candidate c: lamc[(3 * c + rr) * LB]
#pragma unroll
  for (int j = 0; j < ND; ++j) laml[j] = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) wt[k] = 0.f;
  for_active_shapes<T>(shb, [&](const int c) {
    if (GS_ACT(c)) lamc[(3 * c) * LB] = lamc[(3 * c + 1) * LB] = lamc[(3 * c + 2) * LB] = 0.f;
  });
  const float inv_h = 1.f / h;
  const int iters = P.pos_iters + P.vel_iters;
  // TGS (physx.solver_type 1; DESIGN.md 3.5, the lane team's rule, oracle solver_type 3): the position iterations
  // are sub-steps of hs = h / pos_iters; a row's separation is advanced by J dq, dq the sub-steps' displacement --
  // in w space the row's c + z.w summed over the sub-steps done (wacc: the sum of their w); a gap closes within
  // its sub-step, a penetration is pushed out over the step (-s / h, capped); the velocity iterations target the
  // gap the sub-steps left; the positions integrate the sub-steps' mean velocity.  PGS: split impulse.
  const bool tgs = P.tgs != 0;
  const float hs = tgs ? h / (float)P.pos_iters : h, inv_hs = 1.f / hs;
  float wacc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) wacc[k] = 0.f;
  for (int it = 0; it < iters; ++it) {
    const bool pos_phase = it < P.pos_iters;
    const float na = (float)(it < P.pos_iters ? it : P.pos_iters);  // sub-steps done
    // the row's target from its separation at the sub-step (TGS) or the step's start (PGS)
    auto row_target = [&](float sc, float su) {
      if (!tgs) {
        const float t = -sc * inv_h;
        return sc < 0.f ? (pos_phase ? fminf(t, P.max_depen_vel) : 0.f) : t;
      }
      const float sep = sc + hs * su;
      return sep >= 0.f ? -sep * (pos_phase ? inv_hs : inv_h)
                        : (pos_phase ? fminf(-sep * inv_h, P.max_depen_vel) : 0.f);
    };
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      if (lsgn[j] != 0.f) {
        const int SUP = T::lsupp[j];
        const int leaf = T::lleaf[j];
        const float* slot = lds + T::lslot[j] * LB;
        const float sc = lsep[j];
        float z[MS];
        float u = slot[SUP * LB], su = na * slot[SUP * LB];
#pragma unroll
        for (int si = 0; si < MS; ++si) {
          if (si < SUP) {
            z[si] = slot[si * LB];
            u += z[si] * wt[supp_node<T>(leaf, si)];
            if (tgs) su += z[si] * wacc[supp_node<T>(leaf, si)];
          }
        }
        const float target = row_target(sc, su);
        const float nl = fmaxf(laml[j] + (target - u) * slot[(SUP + 1) * LB], 0.f);
        const float dl = nl - laml[j];
        laml[j] = nl;
#pragma unroll
        for (int si = 0; si < MS; ++si)
          if (si < SUP) wt[supp_node<T>(leaf, si)] += z[si] * dl;
      }
    }
    for_active_shapes<T>(shb, [&](const int c) {
      if (GS_ACT(c)) {
        const int SUP = T::csupp[c];
        const int leaf = T::cleaf[c];
        const float* slot = lds + T::cslot[c] * LB;
        const float sc = lds[(X_SEP + c) * LB];
        const float cmu = lds[(X_MU + c) * LB];
        float lam[3] = {lamc[(3 * c) * LB], lamc[(3 * c + 1) * LB], lamc[(3 * c + 2) * LB]};
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
          float z[MS];
          float u = slot[(3 * SUP + rr) * LB], su = na * slot[(3 * SUP + rr) * LB];
#pragma unroll
          for (int si = 0; si < MS; ++si) {
            if (si < SUP) {
              z[si] = slot[(rr * SUP + si) * LB];
              u += z[si] * wt[supp_node<T>(leaf, si)];
              if (tgs && rr == 0) su += z[si] * wacc[supp_node<T>(leaf, si)];
            }
          }
          const float dinv = slot[(3 * SUP + 3 + rr) * LB];  // 0 below GS_MIN_RESPONSE (no impulse)
          float nl;
          if (rr == 0) {
            const float target = row_target(sc, su);
            nl = fmaxf(lam[0] + (target - u) * dinv, 0.f);
          } else {
            const float lim = cmu * lam[0];
            nl = clampf(lam[rr] - u * dinv, -lim, lim);
          }
          const float dl = nl - lam[rr];
          lam[rr] = nl;
#pragma unroll
          for (int si = 0; si < MS; ++si)
            if (si < SUP) wt[supp_node<T>(leaf, si)] += z[si] * dl;
        }
        lamc[(3 * c) * LB] = lam[0];
        lamc[(3 * c + 1) * LB] = lam[1];
        lamc[(3 * c + 2) * LB] = lam[2];
      }
    });
    if constexpr (T::NPK > 0 && SELF) {
      for (int p = 0; p < npc; ++p) {
        float* o = pool + PE * p * LB;
        const float sc = o[kPoolSep * LB];
        float lam[3] = {o[kPoolLam * LB], o[(kPoolLam + 1) * LB], o[(kPoolLam + 2) * LB]};
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
          float u = o[(kPoolC + rr) * LB], su = na * o[(kPoolC + rr) * LB];
#pragma unroll
          for (int k = 0; k < NV; ++k) {
            u += o[(kPoolJ + rr * NV + k) * LB] * wt[k];
            if (tgs && rr == 0) su += o[(kPoolJ + rr * NV + k) * LB] * wacc[k];
          }
          const float dinv = o[(kPoolDi + rr) * LB];
          float nl;
          if (rr == 0) {
            const float target = row_target(sc, su);
            nl = fmaxf(lam[0] + (target - u) * dinv, 0.f);
          } else {
            const float lim = o[kPoolMu * LB] * lam[0];
            nl = clampf(lam[rr] - u * dinv, -lim, lim);
          }
          const float dl = nl - lam[rr];
          lam[rr] = nl;
#pragma unroll
          for (int k = 0; k < NV; ++k) wt[k] += o[(kPoolJ + rr * NV + k) * LB] * dl;
        }
        o[kPoolLam * LB] = lam[0];
        o[(kPoolLam + 1) * LB] = lam[1];
        o[(kPoolLam + 2) * LB] = lam[2];
      }
    }
    if (tgs && pos_phase) {  // the sub-step's velocity joins the displacement
#pragma unroll
      for (int k = 0; k < NV; ++k) wacc[k] += wt[k];
    }
    if (it == P.pos_iters - 1) {
      const float inv_n = 1.f / (float)P.pos_iters;  // TGS: the sub-steps' mean (w space is linear)
#pragma unroll
      for (int k = 0; k < NV; ++k) wpos[k] = tgs ? wacc[k] * inv_n : wt[k];
    }
  }
  if (P.pos_iters <= 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) wpos[k] = wt[k];
  }
  // dnu = L^-1 D^-1/2 w  for the velocity-phase (state) and position-phase (integration) solutions
  float nun[NV], nupos[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float v = wt[k] * sD[k], vp = wpos[k] * sD[k];
#pragma unroll
    for (int ai = 0; ai < T::MAXDEP; ++ai) {
      if (ai < T::depth[k]) {
        const float l = Mm[k][T::anc[k][ai]];
        v -= l * nun[T::anc[k][ai]];
        vp -= l * nupos[T::anc[k][ai]];
      }
    }
    nun[k] = v;
    nupos[k] = vp;
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    nun[k] += nuf[k];
    nupos[k] += nuf[k];
  }

  // ---------------- joint velocity limits
#pragma unroll
  for (int j = 0; j < T::ND; ++j) {
    const float vm = dofp(5, j, M->vmax[j]);
    if (vm > 0.f) {
      nun[NB6 + j] = clampf(nun[NB6 + j], -vm, vm);
      nupos[NB6 + j] = clampf(nupos[NB6 + j], -vm, vm);
    }
  }

  // ---------------- integrate positions with nu_pos; keep nu_new
  if (NB6) {
    s.p[0] += h * nupos[3]; s.p[1] += h * nupos[4]; s.p[2] += h * nupos[5];
    const float wx = nupos[0], wy = nupos[1], wz = nupos[2];
    float x = s.quat[0], y = s.quat[1], z = s.quat[2], w = s.quat[3];
    const float hh = 0.5f * h;
    const float dx = hh * (w * wx + wy * z - wz * y);
    const float dy = hh * (w * wy + wz * x - wx * z);
    const float dz = hh * (w * wz + wx * y - wy * x);
    const float dw = -hh * (wx * x + wy * y + wz * z);
    x += dx; y += dy; z += dz; w += dw;
    const float n = gs_rsqrt(x * x + y * y + z * z + w * w);
    s.quat[0] = x * n; s.quat[1] = y * n; s.quat[2] = z * n; s.quat[3] = w * n;
    s.w[0] = nun[0]; s.w[1] = nun[1]; s.w[2] = nun[2];
    s.vo[0] = nun[3]; s.vo[1] = nun[4]; s.vo[2] = nun[5];
  }
#pragma unroll
  for (int j = 0; j < T::ND; ++j) {
    s.q[j] += h * nupos[NB6 + j];
    s.qd[j] = nun[NB6 + j];
  }
  if (collect) {
    // net contact force per reported link of this (collecting) substep, SoA [3*nr][N]
    // (links = bodies unless fixed-joint links are kept: then a candidate adds to its own link)
#pragma unroll
    for (int b = 0; b < T::NR; ++b) {
      float f0 = 0.f, f1 = 0.f, f2 = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (T::clink[c] == b && ((shb >> T::cshape[c]) & 1u)) {
          if (GS_ACT(c)) {
            const float lam[3] = {lamc[(3 * c) * LB], lamc[(3 * c + 1) * LB], lamc[(3 * c + 2) * LB]};
            if constexpr (TERR) {
              float fw[3];
              contact_force_world<T, LB>(lds, c, lam, inv_h, fw);
              f0 += fw[0]; f1 += fw[1]; f2 += fw[2];
            } else {
              f0 += lam[1] * inv_h;
              f1 += lam[2] * inv_h;
              f2 += lam[0] * inv_h;
            }
          }
        }
      }
      cf_soa[(3 * b + 0) * N + e] = f0;
      cf_soa[(3 * b + 1) * N + e] = f1;
      cf_soa[(3 * b + 2) * N + e] = f2;
    }
    if constexpr (T::NPK > 0 && SELF) {  // self-contacts: +f on link A, -f on link B
      for (int p = 0; p < npc; ++p) {
        const float* o = pool + PE * p * LB;
        const int la = (int)o[kPoolLA * LB], lb = (int)o[kPoolLB * LB];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float f = (o[kPoolLam * LB] * o[(kPoolN + k) * LB] + o[(kPoolLam + 1) * LB] * o[(kPoolT1 + k) * LB] +
                           o[(kPoolLam + 2) * LB] * o[(kPoolT2 + k) * LB]) * inv_h;
          cf_soa[(3 * la + k) * N + e] += f;
          cf_soa[(3 * lb + k) * N + e] -= f;
        }
      }
    }
  }
  if constexpr (T::SENS) if (sens_soa && M->nsens > 0) {
    // force sensors on leaf bodies (topologies compiled with T::SENS): the wrench through the parent joint,
    //   f_joint = I_b a_b + v_b x* I_b v_b - f_contact   (a_b with the gravity offset, RNEA form)
    // with a_b = A_b (velocity products + gravity) + base acceleration + sum_path S_k qdd_k, where
    // qdd = (nu_new - nu)/h and the base's spatial acceleration is (dw/h, dpdot/h - w x pdot).
    // Fc[b] / Ic[b] of a leaf still hold the body's own RNEA force / inertia.
    float ab[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) ab[k] = 0.f;
    if (NB6) {
      float wxp[3];
      cross3(&nu[0], &nu[3], wxp);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        ab[k] = (nun[k] - nu[k]) * inv_h;
        ab[3 + k] = (nun[3 + k] - nu[3 + k]) * inv_h - wxp[k];
      }
    }
#pragma unroll
    for (int b = 1; b < NB; ++b) {
      const int si = M->sens_of_body[b];
      if (si >= 0) {
        float a[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) a[k] = ab[k];
#pragma unroll
        for (int kk = 0; kk < NB; ++kk) {  // path root -> b (compile-time ancestor test)
            if (kk > 0 && body_on_path<T>(kk, b)) {
            const int g = NB6 + T::bdof[kk];
            const float qdd = (nun[g] - nu[g]) * inv_h;
#pragma unroll
            for (int k = 0; k < 6; ++k) a[k] += S[kk][k] * qdd;
          }
        }
        float ia[6], f[6];
        spi_mul(Ic[b], a, ia);
#pragma unroll
        for (int k = 0; k < 6; ++k) f[k] = Fc[b][k] + ia[k];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (T::cbody[c] == b && GS_ACT(c)) {
            const float lamv[3] = {lamc[(3 * c) * LB], lamc[(3 * c + 1) * LB], lamc[(3 * c + 2) * LB]};
            float x[3];
            mat3vec(R[b], M->cpoint[c], x);
            float fc[3];
            if constexpr (TERR) {
              const float* nsl = lds + (T::NSLOT + 3 * c) * LB;
              const float r = M->cradius[c];
              x[0] += X[b][0] - r * nsl[0]; x[1] += X[b][1] - r * nsl[LB]; x[2] += X[b][2] - r * nsl[2 * LB];
              contact_force_world<T, LB>(lds, c, lamv, inv_h, fc);
            } else {
              x[0] += X[b][0]; x[1] += X[b][1]; x[2] += X[b][2] - M->cradius[c];
              fc[0] = lamv[1] * inv_h; fc[1] = lamv[2] * inv_h; fc[2] = lamv[0] * inv_h;
            }
            float n[3];
            cross3(x, fc, n);
#pragma unroll
            for (int k = 0; k < 3; ++k) { f[k] -= n[k]; f[3 + k] -= fc[k]; }
          }
        }
        if constexpr (T::NPK > 0 && SELF) {
          for (int p = 0; p < npc; ++p) {
            const float* o = pool + PE * p * LB;
            const int ba = (int)o[kPoolBA * LB], bbd = (int)o[kPoolBB * LB];
            if (ba != b && bbd != b) continue;
            const float sg = ba == b ? inv_h : -inv_h;
            float fc[3], x[3], n3[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              fc[k] = sg * (o[kPoolLam * LB] * o[(kPoolN + k) * LB] + o[(kPoolLam + 1) * LB] * o[(kPoolT1 + k) * LB] +
                            o[(kPoolLam + 2) * LB] * o[(kPoolT2 + k) * LB]);
              x[k] = o[(kPoolX + k) * LB];
            }
            cross3(x, fc, n3);
#pragma unroll
            for (int k = 0; k < 3; ++k) { f[k] -= n3[k]; f[3 + k] -= fc[k]; }
          }
        }
        // torque about the body origin, then body axes
        float xf[3], tq[3];
        cross3(X[b], &f[3], xf);
#pragma unroll
        for (int k = 0; k < 3; ++k) tq[k] = f[k] - xf[k];
        const float* Rb = R[b];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          sens_soa[(6 * si + k) * N + e] = Rb[k] * f[3] + Rb[3 + k] * f[4] + Rb[6 + k] * f[5];
          sens_soa[(6 * si + 3 + k) * N + e] = Rb[k] * tq[0] + Rb[3 + k] * tq[1] + Rb[6 + k] * tq[2];
        }
      }
    }
  }
}

#undef GS_ACT

template <class T>
GS_HD void com_velocity(const DevModel* __restrict__ M, const EnvState<T>& s, float* v) {
  float R[9], c[3], wc[3];
  quat_to_mat(s.quat, R);
  mat3vec(R, M->root_com, c);
  cross3(s.w, c, wc);
  v[0] = s.vo[0] + wc[0]; v[1] = s.vo[1] + wc[1]; v[2] = s.vo[2] + wc[2];
}

// World centres of env state s's contact candidates, exactly as substep's tree walk forms them
// (cw = p + R_b cpoint + X_b), written to out[(4 * c + k) * stride] with the radius as k = 3.  (A hull's
// dynamic candidates take no terrain-mesh contact: their query result is not read.)
template <class T>
GS_HD void candidate_centres(const DevModel* __restrict__ Min, const EnvState<T>& s, float* out, int stride) {
  constexpr int NB = T::NB, NC = T::NC;
  const DevModel* __restrict__ M = gs_opaque(Min);
  float R[NB][9], X[NB][3];
  body_poses<T>(M, s, R, X);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int b = T::cbody[c];
    float x[3];
    mat3vec(R[b], M->cpoint[c], x);
    x[0] += X[b][0]; x[1] += X[b][1]; x[2] += X[b][2];
    out[(4 * c + 0) * stride] = s.p[0] + x[0];
    out[(4 * c + 1) * stride] = s.p[1] + x[1];
    out[(4 * c + 2) * stride] = s.p[2] + x[2];
    out[(4 * c + 3) * stride] = M->cradius[c];
  }
}

// ---------------------------------------------------------------- per-env entry points
// gym.simulate for env e: `substeps` substeps with constant dof forces [N][nd] (or zero)
// REC: the self-collision narrowphase already ran (k_pair_records), its near-pair records are in B.rows
template <class T, bool TERR, int LB, bool SELF = true, bool REC = false>
GS_HD void simulate_env(const DevModel* __restrict__ M, const DevParams& P, const SimBuffers& B,
                        const float* __restrict__ tau_aos, int e, float* lds) {
  const int N = B.N;
  EnvState<T> s;
  load_state<T>(B.state, N, e, s);
  float tau[T::ND > 0 ? T::ND : 1];
#pragma unroll
  for (int j = 0; j < T::ND; ++j) tau[j] = tau_aos ? tau_aos[(size_t)e * T::ND + j] : 0.f;
  for (int sstep = 0; sstep < P.substeps; ++sstep) {
    const bool last = (sstep == P.substeps - 1) && P.collect;
    if constexpr (SELF && REC)  // this substep's near-pair records
      substep<T, TERR, LB, 0, SELF, 1>(M, P, s, tau, B.mu, N, e, lds, B.cf, last,
                                       sstep == P.substeps - 1 ? B.sens : nullptr, nullptr,
                                       B.rows + (size_t)e * LaneCfg<T, TERR>::ROW_FLOATS);
    else
      substep<T, TERR, LB, 0, SELF>(M, P, s, tau, B.mu, N, e, lds, B.cf, last, sstep == P.substeps - 1 ? B.sens : nullptr);
  }
  store_state<T>(B.state, N, e, s);
}

// PD torques of the fused decimation step for env e (anymal_terrain.py:444-446); the first evaluation
// of a launch reads the dof tensor the task holds (refreshed after the previous step's decimation
// loop, or written by reset_idx)
template <class T>
GS_HD void pd_torques(const PdDev& A, int e, const EnvState<T>& s, bool first, float* tau) {
  constexpr int ND = T::ND;
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const float qj = first ? A.dof_state_in[((size_t)e * ND + j) * 2 + 0] : s.q[j];
    const float qdj = first ? A.dof_state_in[((size_t)e * ND + j) * 2 + 1] : s.qd[j];
    const float aj = A.actions[(size_t)e * ND + j];
    tau[j] = clampf(A.kp * (A.scale * aj + A.default_pos[j] - qj) - A.kd * qdj, -A.tlim, A.tlim);
  }
}
template <class T>
GS_HD void pd_dof_out(const PdDev& A, int e, const EnvState<T>& s) {
  constexpr int ND = T::ND;
  if (!A.dof_out) return;
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    A.dof_out[((size_t)e * ND + j) * 2 + 0] = s.q[j];
    A.dof_out[((size_t)e * ND + j) * 2 + 1] = s.qd[j];
  }
}
// end of the fused step: state, last torques, the actions copy, root and contact tensors
template <class T>
GS_HD void pd_outputs(const DevModel* __restrict__ M, const DevParams& P, const SimBuffers& B, const PdDev& A, int e,
                      const EnvState<T>& s, const float* tau) {
  const int N = B.N;
  constexpr int ND = T::ND;
  store_state<T>(B.state, N, e, s);
#pragma unroll
  for (int j = 0; j < ND; ++j) A.torques_out[(size_t)e * ND + j] = tau[j];
  if (A.actions_copy) {
#pragma unroll
    for (int j = 0; j < ND; ++j) A.actions_copy[(size_t)e * ND + j] = A.actions[(size_t)e * ND + j];
  }
  if (A.root_out) {
    float* o = A.root_out + (size_t)e * 13;
    o[0] = s.p[0]; o[1] = s.p[1]; o[2] = s.p[2];
    o[3] = s.quat[0]; o[4] = s.quat[1]; o[5] = s.quat[2]; o[6] = s.quat[3];
    float v[3];
    com_velocity<T>(M, s, v);
    o[7] = v[0]; o[8] = v[1]; o[9] = v[2];
    o[10] = s.w[0]; o[11] = s.w[1]; o[12] = s.w[2];
  }
  if (P.collect && A.cf_out) {
#pragma unroll
    for (int b = 0; b < T::NR; ++b)
#pragma unroll
      for (int k = 0; k < 3; ++k) A.cf_out[((size_t)e * T::NR + b) * 3 + k] = B.cf[(3 * b + k) * N + e];
  }
}

// the fused decimation step (gs_pd_args, include/gymsim.h) for env e
template <class T, bool TERR, int LB, bool SELF = true>
GS_HD void pd_step_env(const DevModel* __restrict__ M, const DevParams& P, const SimBuffers& B, const PdDev& A, int e,
                       float* lds) {
  const int N = B.N;
  EnvState<T> s;
  load_state<T>(B.state, N, e, s);
  float tau[T::ND];
  // one call site for the substep so it is inlined once
  const int sub = P.substeps;
  const int n_pd = A.decimation * sub;
  const int total = (A.decimation + A.extra) * sub;
  for (int it = 0; it < total; ++it) {
    if (it < n_pd && (it % sub) == 0) pd_torques<T>(A, e, s, it == 0, tau);
    const bool last = ((it % sub) == sub - 1) && P.collect;
    substep<T, TERR, LB, 0, SELF>(M, P, s, tau, B.mu, N, e, lds, B.cf, last, it == total - 1 ? B.sens : nullptr);
    if (it == n_pd - 1) pd_dof_out<T>(A, e, s);
  }
  pd_outputs<T>(M, P, B, A, e, s, tau);
}

// refresh_actor_root_state_tensor row e: SoA state -> [13] with the root link COM velocity
GS_HD void refresh_root_env(const float* __restrict__ st, int N, const float* __restrict__ com0,
                            float* __restrict__ out, int e) {
  float q[4], R[9], c[3], w[3], wc[3];
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = st[(3 + k) * N + e];
#pragma unroll
  for (int k = 0; k < 3; ++k) w[k] = st[(10 + k) * N + e];
  quat_to_mat(q, R);
  mat3vec(R, com0, c);
  cross3(w, c, wc);
  float* o = out + (size_t)e * 13;
#pragma unroll
  for (int k = 0; k < 3; ++k) o[k] = st[k * N + e];
#pragma unroll
  for (int k = 0; k < 4; ++k) o[3 + k] = q[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) o[7 + k] = st[(7 + k) * N + e] + wc[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) o[10 + k] = w[k];
}

// set_actor_root_state_tensor row e: [13] (normalised quaternion, COM velocity) -> SoA state
GS_HD void set_root_env(float* __restrict__ st, int N, const float* __restrict__ com0, const float* __restrict__ src,
                        int e) {
  const float* r = src + (size_t)e * 13;
  float q[4], R[9], c[3], wc[3];
  const float inv = gs_rsqrt(r[3] * r[3] + r[4] * r[4] + r[5] * r[5] + r[6] * r[6]);
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = r[3 + k] * inv;
  quat_to_mat(q, R);
  mat3vec(R, com0, c);
  cross3(r + 10, c, wc);
#pragma unroll
  for (int k = 0; k < 3; ++k) st[k * N + e] = r[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) st[(3 + k) * N + e] = q[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) st[(7 + k) * N + e] = r[7 + k] - wc[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) st[(10 + k) * N + e] = r[10 + k];
}

}  // namespace
