// gs_team.hip -- lane-team form of the articulation + plane-contact substep (gfx950).
//
// Same solver specification as gs_physics.hip / oracle/physics_oracle.c,
// mapped for MI355X occupancy: at 4096 envs the one-env-per-lane kernel has 64 waves for 256
// CUs and spills (VGPR+AGPR+scratch).  Here an env is a TEAM of T::T_LANES consecutive lanes (a
// DPP quad); lane c owns serial chain c of a "uniform star" articulation (ANYmal: 4 legs x 3
// joints).  Chain kinematics, RNEA, composite inertias, the chain rows of the mass matrix, their
// L^T D L elimination, the chain's contact rows and its joint state live in lane c; the 6
// floating-base dofs are REPLICATED in every lane of the team (bit-identical: same inputs, same
// instruction stream, commutative DPP reductions).  Cross-lane traffic is DPP quad_perm only:
//   * sums of chain contributions to the base (composite inertia, RNEA force, Schur
//     complement of the base block, back-substitution residuals);
//   * per Gauss-Seidel row of chain c: broadcast of the row's impulse and activity from lane c,
//     the row itself read from lane c's LDS column (16 teams read 16 addresses, 4-way broadcast).
// Rows are processed in the oracle's global order (root candidates, then chain 0, 1, ...), so
// the iterates are the same projected Gauss-Seidel sequence, only the rounding order of the base
// sums differs.  4096 envs -> 256 waves; per-chain model constants are staged in LDS.
#include <type_traits>

#include "gs_internal.h"
#include "gs_topologies.h"
#include "gs_math.h"
#include "gs_pairs.h"
#include "gt_anymal_tail.h"

// Phase profiler (profiling build only, -DGS_PHASE_PROFILE -> libgymsim_prof.so): per-wave
// s_memtime deltas per solver phase, summed over waves into gs_phase_cycles (gs_capi.hip).
#ifdef GS_PHASE_PROFILE
// [0, 16): phase sums over waves; [16, 32): histogram of a wave's launch total (25k-cycle bins);
// [32, 48): phase sums over the slow waves (total above 250k cycles), [48]: their count
__device__ unsigned long long gs_phase_cycles[64];
#define GS_PROF_DECL long long gs_t_ = clock64(); long long gs_acc_[16] = {0};
#define GS_PROF(i) { const long long t_ = clock64(); gs_acc_[i] += t_ - gs_t_; gs_t_ = t_; }
#define GS_PROF_COUNT(i, n) { gs_acc_[i] += (n); }
#define GS_PROF_PARAM , long long &gs_t_, long long *gs_acc_
#define GS_PROF_ARGS , gs_t_, gs_acc_
#define GS_PROF_FLUSH                                                   \
  if ((threadIdx.x & 63) == 0) {                                        \
    long long tot_ = 0;                                                 \
    for (int i_ = 0; i_ < 16; ++i_) {                                   \
      atomicAdd(&gs_phase_cycles[i_], (unsigned long long)gs_acc_[i_]); \
      if (i_ < 8 || i_ == 11) tot_ += gs_acc_[i_];                      \
    }                                                                   \
    atomicAdd(&gs_phase_cycles[16 + (int)min(tot_ / 25000, 15ll)], 1ull); \
    if (tot_ > 250000) {                                                \
      for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&gs_phase_cycles[32 + i_], (unsigned long long)gs_acc_[i_]); \
      atomicAdd(&gs_phase_cycles[48], 1ull);                            \
    }                                                                   \
  }
#else
#define GS_PROF_DECL
#define GS_PROF_PARAM
#define GS_PROF_ARGS
#define GS_PROF(i)
#define GS_PROF_COUNT(i, n)
#define GS_PROF_FLUSH
#endif

namespace {

template <int CTRL>
__device__ __forceinline__ float qperm(float x) {
  // bound_ctrl: quad_perm never reads out of range; it lets the DPP fold into the consuming VALU op
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int qperm_i(int x) {
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
}
// sum over the 4 lanes of the quad; every lane receives the same bits
__device__ __forceinline__ float quad_sum(float x) {
  x = x + qperm<0xB1>(x);  // quad_perm(1,0,3,2)
  return x + qperm<0x4E>(x);  // quad_perm(2,3,0,1)
}
// packed f32 pairs (v_pk_fma_f32 on gfx950; a broadcast operand is op_sel_hi, not a move)
typedef float f2 __attribute__((ext_vector_type(2)));
#ifndef GS_TEAM_PK
#define GS_TEAM_PK 0  // 1: v_pk_fma_f32 for the row-0/1 partials -- measured slower (r06d: 0.1101 vs 0.1059 ms)
#endif
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) {
#if GS_TEAM_PK
  return __builtin_elementwise_fma(a, b, c);
#else
  return f2{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)};
#endif
}

// three independent quad sums, interleaved so no DPP read waits on the VALU write before it
__device__ __forceinline__ void quad_sum3(float* u) {
  const float a0 = qperm<0xB1>(u[0]), a1 = qperm<0xB1>(u[1]), a2 = qperm<0xB1>(u[2]);
  const float t0 = u[0] + a0, t1 = u[1] + a1, t2 = u[2] + a2;
  const float b0 = qperm<0x4E>(t0), b1 = qperm<0x4E>(t1), b2 = qperm<0x4E>(t2);
  u[0] = t0 + b0;
  u[1] = t1 + b1;
  u[2] = t2 + b2;
}
// four interleaved quad sums (a contact's three rows + its TGS displacement term): the same bits as quad_sum
// of each, one DPP latency for all four
__device__ __forceinline__ void quad_sum4(float* u) {
  const float a0 = qperm<0xB1>(u[0]), a1 = qperm<0xB1>(u[1]), a2 = qperm<0xB1>(u[2]), a3 = qperm<0xB1>(u[3]);
  const float t0 = u[0] + a0, t1 = u[1] + a1, t2 = u[2] + a2, t3 = u[3] + a3;
  const float b0 = qperm<0x4E>(t0), b1 = qperm<0x4E>(t1), b2 = qperm<0x4E>(t2), b3 = qperm<0x4E>(t3);
  u[0] = t0 + b0;
  u[1] = t1 + b1;
  u[2] = t2 + b2;
  u[3] = t3 + b3;
}
// broadcast lane L of the quad to all four lanes; L is a constant after unrolling, the switch folds
__device__ __forceinline__ float bcast(float x, int L) {
  switch (L) {
    case 0: return qperm<0x00>(x);
    case 1: return qperm<0x55>(x);
    case 2: return qperm<0xAA>(x);
    default: return qperm<0xFF>(x);
  }
}
__device__ __forceinline__ int bcast_i(int x, int L) {
  switch (L) {
    case 0: return qperm_i<0x00>(x);
    case 1: return qperm_i<0x55>(x);
    case 2: return qperm_i<0xAA>(x);
    default: return qperm_i<0xFF>(x);
  }
}

// per-chain model constants in LDS, layout [param][lane]
template <class T>
struct CM {
  static constexpr int CL = T::T_CL, CC = T::T_CC;
  static constexpr int BODY = 25;  // jR 9 | jt 3 | axis 3 | mass 1 | com 3 | inertia 6
  static constexpr int CAND = BODY * CL;  // point 3 | radius 1
  static constexpr int DOF = CAND + 4 * CC;  // effort | vmax | armature
  // self-collision broadphase: each chain shape's core segment end points in its body frame (a sphere's
  // centre twice) and its core radius
  static constexpr int SHP = DOF + 3 * CL;
  static constexpr int NP = SHP + (T::NPK > 0 ? 8 * T::T_SPC : 0);
  static constexpr int LANES = T::T_LANES;
};

#ifndef GS_TEAM_BLOCK
#define GS_TEAM_BLOCK 64
#endif
constexpr int kTeamBlock = GS_TEAM_BLOCK;  // lanes per workgroup (one wave at most): 64 -> 16 envs
static_assert(kTeamBlock % 4 == 0 && kTeamBlock <= GS_WAVE, "a workgroup holds whole teams within one wave");

// LDS row stride: one float per lane of the workgroup plus a pad, so the 4 lanes of a team reading 4
// different slots of one column land in 4 different banks (and a narrow workgroup's rows stay small
// enough for several workgroups per CU)
constexpr int RW = kTeamBlock + 1;

// LDS contact records, layout [slot][lane]: chain candidates in the owner lane's column, then root
// candidates (replicated, every lane its own column).  A record holds everything a lane needs
// to run the contact's three Gauss-Seidel rows without cross-lane traffic:
//   Z rows (3 x 16 slots: [Zb 6 | Zc CL | c] spread over the team's lanes) | 1/G_rr (3) |
//   G10/G11 G20/G22 G21/G22 | target/G00 (pos, vel phase) | mu | active
// where G = Z Z^T is the contact's 3x3 Delassus block (couples its rows within one GS pass); the
// couplings and the target are stored pre-scaled by the row's 1/G_rr so that the serial part of a
// contact's Gauss-Seidel update is as short as possible (contact_block).
template <class T>
struct RowSlots {
  static constexpr int CL = T::T_CL;
  // A Z row's 9 components (base 6 | chain 3) plus c = J nu_f in PGS-owner order, four slots per lane:
  // lane l < 3 owns base 2l, base 2l+1 and chain component l (slot 4l+3 a zero pad), lane 3 holds
  // only c (slot 15), so every lane's partial of u = c + Z w is the same three FMAs.  Rows 0 and 1 are
  // stored interleaved (zs): a slot's row-0 and row-1 values are adjacent, one paired LDS load lands them
  // in a register pair, and the two rows' partials are three v_pk_fma_f32 (round 6).
  static constexpr int ZROW = 16;
  static constexpr int RZROW = 16;
  static constexpr int CSLOT = 15;
  __device__ static constexpr int zslot(int comp) { return comp < 6 ? 4 * (comp >> 1) + (comp & 1) : 4 * (comp - 6) + 2; }
  // offset of row rr's slot s inside a record's Z block
  __device__ static constexpr int zs(int rr, int s) { return rr < 2 ? 2 * s + rr : 2 * ZROW + s; }
  // (C_SEP / R_SEP: the row's separation at the substep's start, for TGS's per-sub-step targets)
  static constexpr int C_DI = 3 * ZROW, C_G = C_DI + 3, C_TP = C_G + 3, C_TV = C_TP + 1,
                       C_MU = C_TV + 1, C_ACT = C_MU + 1, C_SEP = C_ACT + 1, PER_CONTACT = C_SEP + 1;
  static constexpr int R_DI = 3 * RZROW, R_G = R_DI + 3, R_TP = R_G + 3, R_TV = R_TP + 1,
                       R_MU = R_TV + 1, R_SEP = R_MU + 1, PER_ROOT = R_SEP + 1;
  static constexpr int CHAIN = PER_CONTACT * T::T_CC;
  static constexpr int ROOT = PER_ROOT * (T::T_RC > 0 ? T::T_RC : 1);
  // self-contact pool, replicated in every lane's column of a team: the entry's geometry
  // (gs_pairs.h kPool* layout), impulses, then per row the lane's 5 components of the distributed Z row
  // [base 2l, base 2l+1, chain A comp l, chain B comp l, c (lane 3)], 1/G_rr (3), scaled couplings (3),
  // target/G00 (pos, vel), chains A and B
  static constexpr int P_Z = kPoolLam + 3, P_DI = P_Z + 15, P_G = P_DI + 3, P_TP = P_G + 3, P_TV = P_TP + 1,
                       P_CA = P_TV + 1, P_CB = P_CA + 1, PER_POOL = P_CB + 1;
  static constexpr int POOL = CHAIN + ROOT;
  static constexpr int TOTAL = POOL + PER_POOL * T::NPK;
  __device__ static constexpr int chain(int j) { return j * PER_CONTACT; }
  __device__ static constexpr int root(int j) { return CHAIN + j * PER_ROOT; }
};

// x[lc][k] for the lane's own chain lc (runtime) out of a replicated [NCH][K] register array
template <int NCH, int K>
__device__ __forceinline__ float sel_chain(const float (&x)[NCH][K], int lc, int k) {
  float v = x[0][k];
#pragma unroll
  for (int c = 1; c < NCH; ++c) v = lc == c ? x[c][k] : v;
  return v;
}

// Distributed PGS velocity -> replicated base w (6) and this lane's chain w (3).  Owners: base 2l
// and 2l+1 lane l < 3 (wA, wA2), chain c component l lane l < 3 (wC[c]).
template <class T>
__device__ __forceinline__ void gather_w(int lc, float wA, float wA2, const float (&wC)[T::T_NCH], float* wb,
                                         float* wc) {
  wb[0] = bcast(wA, 0); wb[1] = bcast(wA2, 0); wb[2] = bcast(wA, 1); wb[3] = bcast(wA2, 1);
  wb[4] = bcast(wA, 2); wb[5] = bcast(wA2, 2);
  wc[0] = wc[1] = wc[2] = 0.f;
#pragma unroll
  for (int c = 0; c < T::T_NCH; ++c) {
    const float c0 = bcast(wC[c], 0), c1 = bcast(wC[c], 1), c2 = bcast(wC[c], 2);
    wc[0] = lc == c ? c0 : wc[0];
    wc[1] = lc == c ? c1 : wc[1];
    wc[2] = lc == c ? c2 : wc[2];
  }
}

// One contact's three projected Gauss-Seidel rows (normal, then the two box-friction rows bounded by
// mu * normal impulse) given u = c + Z w before the pass; the in-pass coupling of its rows goes
// through the Delassus block.  Arguments are pre-scaled: tdi = target/G00, s10 = G10/G11,
// s20 = G20/G22, s21 = G21/G22.  Algebraically the iterate of three scalar GS rows
// with the dependent chain cut to: max, sub | fma, med3, sub | fma, med3, sub.
__device__ __forceinline__ void contact_block(float u0, float u1, float u2, float di0, float di1, float di2,
                                              float s10, float s20, float s21, float tdi, float mu,
                                              float* lam, float& dl0, float& dl1, float& dl2) {
  const float n0 = fmaxf(fmaf(-u0, di0, lam[0] + tdi), 0.f);
  const float a1 = fmaf(-u1, di1, lam[1]);  // row 1 before the in-pass coupling to row 0
  const float a2 = fmaf(-u2, di2, lam[2]);
  dl0 = n0 - lam[0];
  lam[0] = n0;
  const float lim = mu * n0;
  const float n1 = __builtin_amdgcn_fmed3f(fmaf(-s10, dl0, a1), -lim, lim);
  const float b2 = fmaf(-s20, dl0, a2);
  dl1 = n1 - lam[1];
  lam[1] = n1;
  const float n2 = __builtin_amdgcn_fmed3f(fmaf(-s21, dl1, b2), -lim, lim);
  dl2 = n2 - lam[2];
  lam[2] = n2;
}

template <class T>
struct TeamState {
  float p[3], quat[4], vo[3], w[3];  // replicated root
  float q[T::T_CL], qd[T::T_CL];     // this lane's chain
};

template <class T>
__device__ __forceinline__ void stage_chain_model(const DevModel* __restrict__ M, float* mdl) {
  using C = CM<T>;
  for (int i = threadIdx.x; i < C::NP * T::T_NCH; i += blockDim.x) {
    const int p = i / T::T_NCH, c = i - p * T::T_NCH;
    float v;
    if (p < C::CAND) {
      const int k = p / C::BODY, f = p - k * C::BODY;
      const int b = 1 + c * C::CL + k;
      if (f < 9) v = M->jR[b][f];
      else if (f < 12) v = M->jt[b][f - 9];
      else if (f < 15) v = M->jaxis[b][f - 12];
      else if (f < 16) v = M->mass[b];
      else if (f < 19) v = M->com[b][f - 16];
      else v = M->inertia[b][f - 19];
    } else if (p < C::DOF) {
      const int j = (p - C::CAND) / 4, f = (p - C::CAND) - 4 * j;
      const int cand = T::T_RC + c * C::CC + j;
      v = f < 3 ? M->cpoint[cand][f] : M->cradius[cand];
    } else if (p < C::SHP) {
      const int k = (p - C::DOF) / 3, f = (p - C::DOF) - 3 * k;
      const int d = c * C::CL + k;
      v = f == 0 ? M->effort[d] : (f == 1 ? M->vmax[d] : M->armature[d]);
    } else {
      const int j = (p - C::SHP) / 8, f = (p - C::SHP) - 8 * j;
      const int sh = T::T_RS + c * T::T_SPC + j;
      const int kind = M->shkind[sh];
      const float hl = kind == 1 ? M->shsize[sh][1] : 0.f;  // capsules: segment; spheres (and others): centre
      if (f < 6) {
        const float sg = f < 3 ? -hl : hl;
        const int a = f % 3;
        v = kind == 0 || kind == 1 ? M->sht[sh][a] + sg * M->shR[sh][3 * a + 2] : M->shc[sh][a];
      } else if (f == 6) {
        v = kind == 0 || kind == 1 ? M->shm[sh] : M->shc[sh][3];
      } else {
        v = hl;  // half length: bounding sphere radius = hl + radius around the segment's midpoint
      }
    }
    mdl[p * C::LANES + c] = v;
  }
}

// Team-uniform shape constants of the self-collision passes, staged once per launch: per shape
// (ShapeConstsTab) bounding radius, margin, capsule half length, 256 body + link; then per root shape the core segment in
// the root frame (ends l0, l1), radius and half length (broadphase)
template <class T>
struct ShapeTab {
  static constexpr int RS = T::HAS_TEAM ? T::T_RS : 0;
  static constexpr int ROOT = kShC * T::NS;
  static constexpr int POSE = ROOT + 8 * RS;  // per shape: local R (9), t (3), bounding-sphere centre (3)
  static constexpr int SIZE = T::NPK > 0 ? POSE + 15 * T::NS : 1;
};
template <class T>
__device__ __forceinline__ void stage_shape_consts(const DevModel* __restrict__ M, float* sct) {
  if constexpr (T::NPK > 0) {
    using S = ShapeTab<T>;
    for (int i = threadIdx.x; i < S::SIZE; i += blockDim.x) {
      float v = 0.f;
      if (i < S::ROOT) {
        const int sh = i / kShC, f = i - kShC * sh;
        // (slot 3: the shape's body and link, 256 body + link -- the team narrowphase's pool entries, no global
        // load on that path)
        v = f == 0 ? M->shc[sh][3]
                   : (f == 1 ? M->shm[sh] : (f == 2 ? M->shsize[sh][1] : (float)(256 * M->shbody[sh] + M->shlink[sh])));
      } else if (i >= S::POSE) {
        const int sh = (i - S::POSE) / 15, f = (i - S::POSE) - 15 * sh;
        v = f < 9 ? M->shR[sh][f] : (f < 12 ? M->sht[sh][f - 9] : M->shc[sh][f - 12]);
      } else {
        const int sr = (i - S::ROOT) / 8, f = (i - S::ROOT) - 8 * sr;
        const int kind = T::shkind[sr];
        const bool seg = kind == 0 || kind == 1;
        const float hl = kind == 1 ? M->shsize[sr][1] : 0.f;
        if (f < 6) {
          const int a = f % 3;
          const float sg = f < 3 ? -hl : hl;
          v = seg ? M->sht[sr][a] + sg * M->shR[sr][3 * a + 2] : M->shc[sr][a];
        } else {
          v = f == 6 ? (seg ? M->shm[sr] : M->shc[sr][3]) : hl;
        }
      }
      sct[i] = v;
    }
  }
}

template <class T>
__device__ __forceinline__ void team_load(const float* __restrict__ st, int N, int e, int lc, TeamState<T>& s) {
  constexpr int ND = T::ND, CL = T::T_CL;
#pragma unroll
  for (int k = 0; k < 3; ++k) s.p[k] = st[k * N + e];
#pragma unroll
  for (int k = 0; k < 4; ++k) s.quat[k] = st[(3 + k) * N + e];
#pragma unroll
  for (int k = 0; k < 3; ++k) s.vo[k] = st[(7 + k) * N + e];
#pragma unroll
  for (int k = 0; k < 3; ++k) s.w[k] = st[(10 + k) * N + e];
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    s.q[k] = st[(13 + lc * CL + k) * N + e];
    s.qd[k] = st[(13 + ND + lc * CL + k) * N + e];
  }
}
template <class T>
__device__ __forceinline__ void team_store(float* __restrict__ st, int N, int e, int lc, const TeamState<T>& s) {
  constexpr int ND = T::ND, CL = T::T_CL;
  if (lc == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) st[k * N + e] = s.p[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) st[(3 + k) * N + e] = s.quat[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) st[(7 + k) * N + e] = s.vo[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) st[(10 + k) * N + e] = s.w[k];
  }
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    st[(13 + lc * CL + k) * N + e] = s.q[k];
    st[(13 + ND + lc * CL + k) * N + e] = s.qd[k];
  }
}

// spatial inertia of a body at O from its pose and local mass properties
__device__ __forceinline__ void body_inertia(const float* R, const float* X, float m, const float* com,
                                             const float* Il, SpI& I) {
  float c[3];
  mat3vec(R, com, c);
  c[0] += X[0]; c[1] += X[1]; c[2] += X[2];
  float Am[9];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    Am[3 * r + 0] = R[3 * r] * Il[0] + R[3 * r + 1] * Il[3] + R[3 * r + 2] * Il[4];
    Am[3 * r + 1] = R[3 * r] * Il[3] + R[3 * r + 1] * Il[1] + R[3 * r + 2] * Il[5];
    Am[3 * r + 2] = R[3 * r] * Il[4] + R[3 * r + 1] * Il[5] + R[3 * r + 2] * Il[2];
  }
  const float cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  I.m = m;
  I.h[0] = m * c[0]; I.h[1] = m * c[1]; I.h[2] = m * c[2];
  I.I[0] = Am[0] * R[0] + Am[1] * R[1] + Am[2] * R[2] + m * (cc - c[0] * c[0]);
  I.I[1] = Am[3] * R[3] + Am[4] * R[4] + Am[5] * R[5] + m * (cc - c[1] * c[1]);
  I.I[2] = Am[6] * R[6] + Am[7] * R[7] + Am[8] * R[8] + m * (cc - c[2] * c[2]);
  I.I[3] = Am[0] * R[3] + Am[1] * R[4] + Am[2] * R[5] - m * c[0] * c[1];
  I.I[4] = Am[0] * R[6] + Am[1] * R[7] + Am[2] * R[8] - m * c[0] * c[2];
  I.I[5] = Am[3] * R[6] + Am[4] * R[7] + Am[5] * R[8] - m * c[1] * c[2];
}

// Jacobian rows of a contact point xc (relative to O) for the base dofs: row ax of [-[xc]x | I]
__device__ __forceinline__ float base_jac(const float* xc, int ax, int k) {
  if (k < 3) {
    const float m3[3][3] = {{0.f, xc[2], -xc[1]}, {-xc[2], 0.f, xc[0]}, {xc[1], -xc[0], 0.f}};
    return m3[ax][k];
  }
  return (ax == k - 3) ? 1.f : 0.f;
}

// An index the compiler cannot see through: the kernels' final stores recompute their addresses from it instead
// of keeping the load addresses (64-bit, one pair of VGPRs per state row) live across the whole launch -- in the
// round-5 kernel those pairs were what spilled to scratch (184 B per lane, written back once per launch)
__device__ __forceinline__ int opaque_index(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// floats per lane of the sweeps' LDS stash (substep_team stash_io): the base block's L factors, 1/sqrt(D) and free
// velocity, then per chain dof its Mcb row, Mcc row, 1/sqrt(D) and free velocity
template <class T>
__host__ __device__ constexpr int team_stash_size() {
  return 15 + 6 + 6 + T::T_CL * (6 + 2) + T::T_CL * (T::T_CL - 1) / 2;
}

// Per-team shape table for the self-collision prepass: [(kShW * sh + f) * TPW + team] (TPW teams per workgroup)
constexpr int kTeamsPerBlock = kTeamBlock / 4;

// every self-collision pair of the topology has a closed form (pair kinds 0 sphere-sphere, 1 sphere-capsule,
// 2 capsule-capsule, gs_pairs.h self_pair): the team narrowphase forms them in the lanes that found them; a
// topology with a GJK pair (box, cylinder, hull) runs the replicated gs_pairs.h narrowphase instead
template <class T>
__host__ __device__ constexpr bool team_closed_form() {
  for (int q = 0; q < T::NPAIR; ++q)
    if (T::pair_k[q] > 2) return false;
  return true;
}
// the team narrowphase's staging: per lane its kTeamLC(T) contacts of smallest pair order (kTeamSt floats each:
// x (3), n (3), separation, shapes a, b) at [f + kTeamSt * slot][64 lanes], then the team's first NPK in pair order
// at [f + kTeamSt * rank][TPW teams].  Each lane keeping its NPK smallest keys is exact: every contact among the
// team's first NPK is among its own lane's first NPK.
constexpr int kTeamSt = 9;
template <class T>
__host__ __device__ constexpr int team_lc() { return T::NPK > 0 ? T::NPK : 1; }
// floats of the workgroup's shape / staging table (shared with the TERR query list)
template <class T>
__host__ __device__ constexpr int shw_size() {
  const int pose = kShW * T::NS * kTeamsPerBlock;
  const int stage = team_lc<T>() * kTeamSt * 64 + T::NPK * kTeamSt * kTeamsPerBlock;
  return T::NPK == 0 ? 1 : (team_closed_form<T>() ? (stage > pose ? stage : pose) : pose);
}

// Self-collision prepass of a team: every lane publishes its chain's shapes' bounding-sphere
// centres (lane 0 also the root's), the lanes split the pair list for the broadphase; a wave with a near pair
// in any team publishes the shapes' full poses and runs the narrowphase replicated in each lane of the team
// (gs_pairs.h self_contacts: the same pair order and rules as the one-env-per-lane solver and the oracle).
// Returns the team's self-contact count (the pool geometry is in the lane's own column).
// Squared distance between segments p1q1 and p2q2, branch-free (Ericson's closest points with v_rcp: s from the
// lines' closest points, t from s, s again from t, each clamped; a point segment has a = 0 or e = 0).  The
// reciprocals' ~1 ulp error is covered by the broadphase's slack; the narrowphase recomputes exactly.
__device__ __forceinline__ float seg_seg_d2(const float* p1, const float* q1, const float* p2, const float* q2) {
  float d1[3], d2[3], r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
  const float a = dot3f(d1, d1), e = dot3f(d2, d2), b = dot3f(d1, d2), c = dot3f(d1, r), f = dot3f(d2, r);
  const float ia = a > 1e-12f ? __builtin_amdgcn_rcpf(a) : 0.f;
  const float ie = e > 1e-12f ? __builtin_amdgcn_rcpf(e) : 0.f;
  const float den = a * e - b * b;
  float s = den > 1e-12f * a * e ? __builtin_amdgcn_fmed3f((b * f - c * e) * __builtin_amdgcn_rcpf(den), 0.f, 1.f) : 0.f;
  const float t = __builtin_amdgcn_fmed3f((b * s + f) * ie, 0.f, 1.f);
  s = __builtin_amdgcn_fmed3f((b * t - c) * ia, 0.f, 1.f);
  float dd = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float x = r[k] + s * d1[k] - t * d2[k];
    dd += x * x;
  }
  return dd;
}

// squared distance from point p to segment s0 s1 (v_rcp: ~1 ulp, covered by the broadphase's slack)
__device__ __forceinline__ float seg_pt_d2(const float* s0, const float* s1, const float* p) {
  float d[3], r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { d[k] = s1[k] - s0[k]; r[k] = p[k] - s0[k]; }
  const float dd = dot3f(d, d);
  const float t = dd > 1e-12f ? __builtin_amdgcn_fmed3f(dot3f(r, d) * __builtin_amdgcn_rcpf(dd), 0.f, 1.f) : 0.f;
  float out = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float x = r[k] - t * d[k];
    out += x * x;
  }
  return out;
}

// gs_pairs.h seg_seg / seg_closest_pt with v_rcp for the divisions (~1 ulp): the team narrowphase is a serial
// chain of them inside a wave-divergent block, where each IEEE division costs ~10 dependent instructions
__device__ __forceinline__ void seg_seg_rcp(const float* p1, const float* q1, const float* p2, const float* q2, float& s,
                                            float& t, float& den, float& a, float& e) {
  float d1[3], d2[3], r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
  a = dot3f(d1, d1);
  e = dot3f(d2, d2);
  const float f = dot3f(d2, r);
  s = 0.f; t = 0.f; den = 0.f;
  const float ia = __builtin_amdgcn_rcpf(a), ie = __builtin_amdgcn_rcpf(e);
  auto cl = [](float x) { return __builtin_amdgcn_fmed3f(x, 0.f, 1.f); };
  if (a <= 1e-12f && e <= 1e-12f) {
  } else if (a <= 1e-12f) {
    t = cl(f * ie);
  } else {
    const float c = dot3f(d1, r);
    if (e <= 1e-12f) {
      s = cl(-c * ia);
    } else {
      const float b = dot3f(d1, d2);
      den = a * e - b * b;
      s = den > 0.f ? cl((b * f - c * e) * __builtin_amdgcn_rcpf(den)) : 0.f;
      t = (b * s + f) * ie;
      if (t < 0.f) { t = 0.f; s = cl(-c * ia); }
      else if (t > 1.f) { t = 1.f; s = cl((b - c) * ia); }
    }
  }
}
__device__ __forceinline__ void seg_closest_pt_rcp(const float* p, const float* a, const float* b, float* q) {
  const float ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  const float l2 = dot3f(ab, ab);
  const float t = l2 > 0.f ? __builtin_amdgcn_fmed3f(dot3f(ap, ab) * __builtin_amdgcn_rcpf(l2), 0.f, 1.f) : 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) q[k] = a[k] + t * ab[k];
}

// shapes a < b of a topology collide (its self-collision pair table, gs_topologies.h)
template <class T>
__host__ __device__ constexpr bool team_pair(int a, int b) {
  for (int q = 0; q < T::NPAIR; ++q)
    if (T::pair_a[q] == a && T::pair_b[q] == b) return true;
  return false;
}
// index of the pair of shapes a, b in the pair table (-1: not a pair)
template <class T>
__host__ __device__ constexpr int team_pair_index(int a, int b) {
  for (int q = 0; q < T::NPAIR; ++q)
    if ((T::pair_a[q] == a && T::pair_b[q] == b) || (T::pair_a[q] == b && T::pair_b[q] == a)) return q;
  return -1;
}
// a pair's bit in the team's near mask, for the lane's chain lc: shapes a_c = RS + c SPC + ja (or root shape
// ra when ja < 0), b_c = RS + ((c + dl) & 3) SPC + jb, selected from the four compile-time candidates
template <class T>
__device__ __forceinline__ unsigned long long team_pair_bit(int lc, int ra, int ja, int dl, int jb) {
  unsigned long long bit = 0ull;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int a = ja < 0 ? ra : T::T_RS + c * T::T_SPC + ja;
    const int b = T::T_RS + ((c + dl) & 3) * T::T_SPC + jb;
    const int q = team_pair_index<T>(a, b);
    bit = lc == c ? (q >= 0 ? 1ull << q : 0ull) : bit;
  }
  return bit;
}
__device__ __forceinline__ unsigned long long quad_or64(unsigned long long m) {
  int lo = (int)(unsigned)m, hi = (int)(unsigned)(m >> 32);
  lo |= qperm_i<0xB1>(lo);
  hi |= qperm_i<0xB1>(hi);
  lo |= qperm_i<0x4E>(lo);
  hi |= qperm_i<0x4E>(hi);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// The replicated narrowphase (the round-4 path, now the fallback of team_self_contacts when a lane holds more
// contacts than it stages): every lane publishes its chain's shapes' full poses (lane 0 also the root's) to the
// team's LDS table, and each lane of a team runs gs_pairs.h self_contacts over the team's near pairs.
template <class T>
__device__ __forceinline__ int team_narrow_replicated(const DevModel* __restrict__ M, const DevParams& P,
                                                   const float* __restrict__ mu_g, int N, int e, int lc,
                                                   const float (&R0)[9], const float (&R)[T::T_CL][9],
                                                   const float (&X)[T::T_CL][3], unsigned long long near,
                                                   float* __restrict__ shw_tab, const float* __restrict__ sct,
                                                   float* __restrict__ pool) {
  constexpr int TPW = kTeamsPerBlock;
  const int team = threadIdx.x >> 2;
  float* tab = shw_tab + team;
  __syncthreads();  // the staging above may still be read
  // full shape poses for the narrowphase: R (9), centre (3), bounding-sphere centre (3)
#pragma unroll
  for (int j = 0; j < T::T_SPC; ++j) {
    const int sh = T::T_RS + lc * T::T_SPC + j;
    const int k = T::sh_body[T::T_RS + j] - 1;
    const float* ps = sct + ShapeTab<T>::POSE + 15 * sh;
    float Rs[9], t[3], c[3];
    mat3mul(R[k], ps, Rs);
    mat3vec(R[k], ps + 9, t);
    mat3vec(R[k], ps + 12, c);
#pragma unroll
    for (int f = 0; f < 9; ++f) tab[(kShW * sh + f) * TPW] = Rs[f];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      tab[(kShW * sh + 9 + f) * TPW] = X[k][f] + t[f];
      tab[(kShW * sh + 12 + f) * TPW] = X[k][f] + c[f];
    }
  }
  if (lc == 0) {
#pragma unroll
    for (int sh = 0; sh < T::T_RS; ++sh) {
      const float* ps = sct + ShapeTab<T>::POSE + 15 * sh;
      float Rs[9], t[3], c[3];
      mat3mul(R0, ps, Rs);
      mat3vec(R0, ps + 9, t);
      mat3vec(R0, ps + 12, c);
#pragma unroll
      for (int f = 0; f < 9; ++f) tab[(kShW * sh + f) * TPW] = Rs[f];
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        tab[(kShW * sh + 9 + f) * TPW] = t[f];
        tab[(kShW * sh + 12 + f) * TPW] = c[f];
      }
    }
  }
  __syncthreads();
  // the team's near pairs (team-uniform mask) -> the narrowphase of those pairs, replicated in the team's lanes
  const unsigned long long tmask = quad_or64(near);
  int cnt = 0;
  if (tmask) cnt = self_contacts<T, TPW, RW, RowSlots<T>::PER_POOL>(M, P, mu_g, N, e, tab, pool, ShapeConstsTab{sct},
                                                                    tmask);
  return cnt;
}

// Self-collision prepass of a team.  Broadphase in registers, every substep: each lane holds its
// chain's shapes as core segments + radius (a sphere is a point segment; boxes / hulls their bounding sphere) and
// the root's; it tests the pairs root x own chain, own chain x itself, own chain x chain lc+1 and (lanes 0, 1)
// x chain lc+2, the neighbours' shapes arriving by DPP quad rotations -- the exact core distance for sphere /
// capsule pairs, within contact_offset.  Only a wave with such a pair writes the shapes' full poses to the team's
// LDS table and runs the narrowphase, replicated in each lane of the teams concerned (gs_pairs.h self_contacts:
// the pair order and rules of the one-env-per-lane solver and the oracle).  Returns the team's self-contact count
// (the pool in the lane's own column).
template <class T>
__device__ __forceinline__ int team_self_contacts(const DevModel* __restrict__ M, const float* __restrict__ cm,
                                                  const DevParams& P, const float* __restrict__ mu_g, int N, int e,
                                                  int lc, const float (&R0)[9], const float (&R)[T::T_CL][9],
                                                  const float (&X)[T::T_CL][3], float* __restrict__ shw_tab,
                                                  const float* __restrict__ sct, float* __restrict__ pool) {
  constexpr int TPW = kTeamsPerBlock, LN = T::T_LANES, SPC = T::T_SPC, RSH = T::T_RS;
  using C = CM<T>;
  // (conservative by a hair: the narrowphase recomputes the distance in another association order)
  const float off = P.contact_offset * 1.001f + 1e-5f;
  float p0[SPC][3], p1[SPC][3], rad[SPC], hl[SPC];
#pragma unroll
  for (int j = 0; j < SPC; ++j) {
    const int k = T::sh_body[RSH + j] - 1;  // chain-local body (chain 0's layout, the same for every chain)
    const float* sp = cm + (C::SHP + 8 * j) * LN;
    const float l0[3] = {sp[0], sp[LN], sp[2 * LN]}, l1[3] = {sp[3 * LN], sp[4 * LN], sp[5 * LN]};
    mat3vec(R[k], l0, p0[j]);
    mat3vec(R[k], l1, p1[j]);
#pragma unroll
    for (int f = 0; f < 3; ++f) { p0[j][f] += X[k][f]; p1[j][f] += X[k][f]; }
    rad[j] = sp[6 * LN];
    hl[j] = sp[7 * LN];
  }
  static_assert(T::NPAIR <= 64, "the team's near-pair mask is 64 bits");
  unsigned long long near = 0ull;  // bits of the pair table: the lane's tests that found a pair within reach
  // bounding spheres first (midpoint, half length + radius); the exact segment distance only where they meet
  // (sa / sb: the shape is a capsule core segment; spheres, boxes and hulls are points here -- compile-time
  // kinds, so a point pair is exact on the midpoint test and a point-capsule pair takes the point-segment
  // distance instead of the segment-segment one)
  auto test = [&](const float* a0, const float* a1, float ra, float ha, bool sa, int, const float* b0, const float* b1,
                  float rb, float hb, bool sb, int, unsigned long long bit) {
    const float rr = ra + rb + off;
    float dc = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float x = 0.5f * ((a0[k] + a1[k]) - (b0[k] + b1[k]));
      dc += x * x;
    }
    if (!sa && !sb) {
      if (dc < rr * rr) near |= bit;
      return;
    }
    const float rs = rr + (sa ? ha : 0.f) + (sb ? hb : 0.f);
    if (!(dc < rs * rs)) return;
    float d2;
    if (sa && sb) {
      d2 = seg_seg_d2(a0, a1, b0, b1);
    } else {
      const float* s0 = sa ? a0 : b0;
      const float* s1 = sa ? a1 : b1;
      const float* pt = sa ? b0 : a0;
      d2 = seg_pt_d2(s0, s1, pt);
    }
    if (d2 < rr * rr) near |= bit;
  };
  // every pair site of the lane, in a fixed order: f(segment a, radius, half length, capsule?, shape, segment b, ...,
  // the pair's bit); the root shapes' and the neighbour chains' segments are formed here
  // (lcv: the lane's chain; the narrowphase passes it through opaque_index so its pair bits and keys are formed
  // there, not hoisted to the kernel's start and kept live across the launch)
  auto visit = [&](int lcv, auto&& f) {
#pragma unroll
    for (int sr = 0; sr < RSH; ++sr) {
      const float* rt = sct + ShapeTab<T>::ROOT + 8 * sr;
      const float l0[3] = {rt[0], rt[1], rt[2]}, l1[3] = {rt[3], rt[4], rt[5]};
      const float rr = rt[6], rhl = rt[7];
      float r0[3], r1[3];
      mat3vec(R0, l0, r0);
      mat3vec(R0, l1, r1);
#pragma unroll
      for (int j = 0; j < SPC; ++j)
        if (team_pair<T>(sr, RSH + j))
          f(r0, r1, rr, rhl, T::shkind[sr] == 1, sr, p0[j], p1[j], rad[j], hl[j], T::shkind[RSH + j] == 1,
            RSH + lcv * SPC + j, team_pair_bit<T>(lcv, sr, -1, 0, j));
    }
#pragma unroll
    for (int j = 0; j < SPC; ++j)
#pragma unroll
      for (int j2 = j + 1; j2 < SPC; ++j2)
        if (team_pair<T>(RSH + j, RSH + j2))
          f(p0[j], p1[j], rad[j], hl[j], T::shkind[RSH + j] == 1, RSH + lcv * SPC + j, p0[j2], p1[j2], rad[j2], hl[j2],
            T::shkind[RSH + j2] == 1, RSH + lcv * SPC + j2, team_pair_bit<T>(lcv, 0, j, 0, j2));
    // chains lc + 1 (every lane) and lc + 2 (lanes 0 and 1): each inter-chain pair exactly once
#pragma unroll
    for (int dl = 1; dl <= 2; ++dl) {
      float q0[SPC][3], q1[SPC][3];
#pragma unroll
      for (int j = 0; j < SPC; ++j) {
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          q0[j][g] = dl == 1 ? qperm<0x39>(p0[j][g]) : qperm<0x4E>(p0[j][g]);
          q1[j][g] = dl == 1 ? qperm<0x39>(p1[j][g]) : qperm<0x4E>(p1[j][g]);
        }
      }
      if (dl == 1 || lcv < 2) {
        const int lo = (lcv + dl) & 3;
#pragma unroll
        for (int j = 0; j < SPC; ++j)
#pragma unroll
          for (int j2 = 0; j2 < SPC; ++j2)
            if (team_pair<T>(RSH + j, RSH + SPC + j2))
              f(p0[j], p1[j], rad[j], hl[j], T::shkind[RSH + j] == 1, RSH + lcv * SPC + j, q0[j2], q1[j2], rad[j2],
                hl[j2], T::shkind[RSH + j2] == 1, RSH + lo * SPC + j2, team_pair_bit<T>(lcv, 0, j, dl, j2));
      }
    }
  };
  visit(lc, test);
  if (__ballot(near != 0ull) == 0ull) return 0;  // wave-uniform: no team of the wave has a pair within reach
#ifdef GS_PHASE_PROFILE
  if ((threadIdx.x & 63) == 0) atomicAdd(&gs_phase_cycles[12], 1ull);  // substeps a wave runs the narrowphase
  const long long np_t0 = clock64();
#endif
  if constexpr (!team_closed_form<T>()) {
    // GJK pairs: the replicated narrowphase (every pair kind of gs_pairs.h self_pair)
    return team_narrow_replicated<T>(M, P, mu_g, N, e, lc, R0, R, X, near, shw_tab, sct, pool);
  } else {
  // ---- narrowphase (round 5).  Each near pair's contacts are formed by the lane whose broadphase found it, from
  // the segments it holds in registers -- the closed-form sphere / capsule rules of gs_pairs.h self_pair (the
  // pair's a = the lower shape index, n from b to a, up to 2 contacts for a parallel capsule overlap), so the
  // pool is the one-env-per-lane solver's -- into the lane's own LDS slots; the team then ranks its contacts
  // by (pair, contact) through DPP, keeps the first NPK in pair order (self_contacts' cap) and every lane of the
  // team copies them into its pool column.  Before, every lane of the team published its shapes' full poses
  // and re-ran the whole narrowphase of the team's near pairs (10.5 k cycles per wave-substep entered: the slow
  // waves' tail).  Round 6: each lane keeps the kLC = NPK contacts of smallest pair order it finds
  // (exact for the team's first NPK, team_lc), so no lane ever falls back to the replicated narrowphase.
  constexpr int kLC = team_lc<T>(), kSt = kTeamSt;
  constexpr int kNone = 0x7fffffff;
  const int wl = threadIdx.x & 63;
  const int team = threadIdx.x >> 2;
  float* lslot = shw_tab + wl;                        // [f + kSt * slot][64 lanes]
  float* tstg = shw_tab + kLC * kSt * 64 + team;      // [f + kSt * rank][TPW teams]
  static_assert(kLC * kSt * 64 + T::NPK * kSt * TPW <= shw_size<T>(), "contact staging fits the table");
  __syncthreads();  // an earlier user of the table (the TERR query list, a previous substep) is done with it
  const float coff = P.contact_offset;
  int cnt = 0;  // the lane's contacts (all of them: the team's count caps at NPK)
  int key[kLC];
#pragma unroll
  for (int i = 0; i < kLC; ++i) key[i] = kNone;
  auto narrow = [&](const float* a0_, const float* a1_, float ra_, float, bool sa, int ia, const float* b0_,
                    const float* b1_, float rb_, float, bool sb, int ib, unsigned long long bit) {
    if (!(near & bit)) return;
    const int q = __builtin_ctzll(bit);
    // the pair table's orientation: a = the lower shape index
    const bool sw = ia > ib;
    float a0[3], a1[3], b0[3], b1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      a0[k] = sw ? b0_[k] : a0_[k]; a1[k] = sw ? b1_[k] : a1_[k];
      b0[k] = sw ? a0_[k] : b0_[k]; b1[k] = sw ? a1_[k] : b1_[k];
    }
    const float ra = sw ? rb_ : ra_, rb = sw ? ra_ : rb_;
    const int sha = sw ? ib : ia, shb = sw ? ia : ib;
    float pa[2][3], pb[2][3];
    int nct = 1;
    if (!sa && !sb) {  // sphere pair: the centres
#pragma unroll
      for (int k = 0; k < 3; ++k) { pa[0][k] = a0[k]; pb[0][k] = b0[k]; }
    } else if (sa && sb) {  // capsule pair: the segments' closest points, both ends of a parallel overlap
      float s, t, den, aa, ee;
      seg_seg_rcp(a0, a1, b0, b1, s, t, den, aa, ee);
      bool two = false;
      float lo = 0.f, hi = 0.f;
      if (aa > 1e-12f && ee > 1e-12f && den <= 1e-4f * aa * ee) {
        float d1[3], w0[3], w1[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { d1[k] = a1[k] - a0[k]; w0[k] = b0[k] - a0[k]; w1[k] = b1[k] - a0[k]; }
        const float ia = __builtin_amdgcn_rcpf(aa);
        const float s0 = dot3f(w0, d1) * ia, s1 = dot3f(w1, d1) * ia;
        lo = fminf(s0, s1);
        hi = fmaxf(s0, s1);
        lo = lo < 0.f ? 0.f : lo;
        hi = hi > 1.f ? 1.f : hi;
        two = hi - lo > 1e-3f;
      }
      if (two) {
        nct = 2;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const float sc2 = c == 0 ? lo : hi;
#pragma unroll
          for (int k = 0; k < 3; ++k) pa[c][k] = a0[k] + sc2 * (a1[k] - a0[k]);
          seg_closest_pt_rcp(pa[c], b0, b1, pb[c]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) { pa[0][k] = a0[k] + s * (a1[k] - a0[k]); pb[0][k] = b0[k] + t * (b1[k] - b0[k]); }
      }
    } else {  // sphere - capsule: the sphere centre's closest point on the core segment
      const bool capa = sw ? sb : sa;  // side a (oriented) is the capsule
      float e0[3], e1[3], pt[3], q3[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        e0[k] = capa ? a0[k] : b0[k]; e1[k] = capa ? a1[k] : b1[k]; pt[k] = capa ? b0[k] : a0[k];
      }
      seg_closest_pt_rcp(pt, e0, e1, q3);
#pragma unroll
      for (int k = 0; k < 3; ++k) { pa[0][k] = capa ? q3[k] : a0[k]; pb[0][k] = capa ? b0[k] : q3[k]; }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (c >= nct) break;
      float nn[3] = {pa[c][0] - pb[c][0], pa[c][1] - pb[c][1], pa[c][2] - pb[c][2]};
      const float d2 = dot3f(nn, nn);
      float dist = sqrtf(d2);
      if (!(dist > 1e-9f)) {  // coincident cores: the centres' direction
        float f[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) f[k] = 0.5f * ((a0[k] + a1[k]) - (b0[k] + b1[k]));
        float l = sqrtf(dot3f(f, f));
        if (!(l > 1e-9f)) { f[0] = 0.f; f[1] = 0.f; f[2] = 1.f; l = 1.f; }
#pragma unroll
        for (int k = 0; k < 3; ++k) nn[k] = f[k] / l;
        dist = 0.f;
      } else {
        const float idist = __builtin_amdgcn_rsqf(d2);
#pragma unroll
        for (int k = 0; k < 3; ++k) nn[k] *= idist;
      }
      const float sep = dist - ra - rb;
      if (!(sep < coff)) continue;
      // the slot: the next free one, else the one holding the largest key when this key is smaller
      const int kn = 2 * q + c;
      int slot = cnt < kLC ? cnt : -1;
      if (cnt >= kLC) {
        int m = 0, km = key[0];
#pragma unroll
        for (int i = 1; i < kLC; ++i) {
          m = key[i] > km ? i : m;
          km = key[i] > km ? key[i] : km;
        }
        slot = kn < km ? m : -1;
      }
      if (slot >= 0) {
        float* o = lslot + kSt * slot * 64;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          o[k * 64] = 0.5f * ((pa[c][k] - ra * nn[k]) + (pb[c][k] + rb * nn[k]));
          o[(3 + k) * 64] = nn[k];
        }
        o[6 * 64] = sep;
        o[7 * 64] = __int_as_float(sha);
        o[8 * 64] = __int_as_float(shb);
#pragma unroll
        for (int i = 0; i < kLC; ++i) key[i] = i == slot ? kn : key[i];
      }
      ++cnt;
    }
  };
  visit(opaque_index(lc), narrow);
#ifdef GS_PHASE_PROFILE
  if ((threadIdx.x & 63) == 0) atomicAdd(&gs_phase_cycles[14], (unsigned long long)(clock64() - np_t0));
#endif
  int cnt_team = 0;
  {
    // the team's contacts in pair order: each staged contact's rank among the team's staged keys (the smaller
    // keys of the team's first NPK are all staged, so the rank is the contact's place in the whole pair order)
    int rk[kLC];
#pragma unroll
    for (int i = 0; i < kLC; ++i) rk[i] = 0;
    auto tally = [&](const int (&ks)[kLC]) {
#pragma unroll
      for (int j = 0; j < kLC; ++j)
#pragma unroll
        for (int i = 0; i < kLC; ++i) rk[i] += ks[j] < key[i];
    };
    tally(key);
    {
      int ks[kLC];
#pragma unroll
      for (int j = 0; j < kLC; ++j) ks[j] = qperm_i<0x39>(key[j]);
      tally(ks);
#pragma unroll
      for (int j = 0; j < kLC; ++j) ks[j] = qperm_i<0x4E>(key[j]);
      tally(ks);
#pragma unroll
      for (int j = 0; j < kLC; ++j) ks[j] = qperm_i<0x93>(key[j]);
      tally(ks);
    }
    cnt_team = cnt + qperm_i<0xB1>(cnt);
    cnt_team += qperm_i<0x4E>(cnt_team);
#pragma unroll
    for (int i = 0; i < kLC; ++i) {
      if (i < cnt && rk[i] < T::NPK) {
        const float* src = lslot + kSt * i * 64;
        float* dst = tstg + kSt * rk[i] * TPW;
#pragma unroll
        for (int f = 0; f < kSt; ++f) dst[f * TPW] = src[f * 64];
      }
    }
    __syncthreads();
    cnt_team = cnt_team < T::NPK ? cnt_team : T::NPK;
#pragma unroll
    for (int r = 0; r < T::NPK; ++r) {
      if (r < cnt_team) {
        const float* src = tstg + kSt * r * TPW;
        float* o = pool + RowSlots<T>::PER_POOL * r * RW;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          o[(kPoolX + k) * RW] = src[k * TPW];
          o[(kPoolN + k) * RW] = src[(3 + k) * TPW];
        }
        o[kPoolSep * RW] = src[6 * TPW];
        // pool_entry_finish's fields, the bodies and links from the LDS shape table
        const int a = __float_as_int(src[7 * TPW]), b = __float_as_int(src[8 * TPW]);
        const float nn[3] = {src[3 * TPW], src[4 * TPW], src[5 * TPW]};
        float t1[3], t2[3];
        gs_terrain::tangents(nn, t1, t2);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          o[(kPoolT1 + k) * RW] = t1[k];
          o[(kPoolT2 + k) * RW] = t2[k];
        }
        o[kPoolMu * RW] = 0.5f * (mu_g[a * N + e] + mu_g[b * N + e]);
        const int bla = (int)sct[kShC * a + 3], blb = (int)sct[kShC * b + 3];
        o[kPoolBA * RW] = (float)(bla >> 8);
        o[kPoolBB * RW] = (float)(blb >> 8);
        o[kPoolLA * RW] = (float)(bla & 255);
        o[kPoolLB * RW] = (float)(blb & 255);
      }
    }
  }
#ifdef GS_PHASE_PROFILE
  {
    const unsigned long long tm = quad_or64(near);
    const unsigned long long lanes = __ballot(tm != 0ull);
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&gs_phase_cycles[13], (unsigned long long)(clock64() - np_t0));
      atomicAdd(&gs_phase_cycles[15], (unsigned long long)__popcll(lanes));  // lanes of teams with a near pair
      atomicAdd(&gs_phase_cycles[10], (unsigned long long)__popcll(tm));  // (lane 0's team) near pairs
    }
  }
#endif
  return cnt_team;
  }  // closed-form pairs
}

// TERR (trimesh terrain): a candidate sphere at x (relative to the root origin p) against the
// deepest of the ground plane and the terrain mesh, as the one-env-per-lane solver's TERR branch: returns the
// distance, the contact normal and the surface friction (the plane's (0, 0, 1) and ground friction when no mesh
// surface is nearer)
__device__ __forceinline__ float terrain_candidate(const DevParams& P, const float* p, const float* x, float r,
                                                   float* nrm, float& smu) {
  const float cw[3] = {p[0] + x[0], p[1] + x[1], p[2] + x[2]};
  float dist = P.has_ground ? cw[2] - r : 3.0e38f;
  nrm[0] = 0.f; nrm[1] = 0.f; nrm[2] = 1.f;
  smu = P.ground_mu;
  float st, nt[3];
  if (gs_terrain::sphere_contact(P.terr, cw, r, r + P.contact_offset, st, nt) && st < dist) {
    dist = st;
    nrm[0] = nt[0]; nrm[1] = nt[1]; nrm[2] = nt[2];
    smu = P.terr.mu;
  }
  return dist;
}

template <class T, bool TERR, bool TGS>
__device__ __forceinline__ void substep_team(const DevModel* __restrict__ Min, const float* __restrict__ mdl,
                                             const DevParams& P, TeamState<T>& s, const float* tau,
                                             const float* __restrict__ mu_t, int N, int e, int lc,
                                             float* __restrict__ rows_own, const float* __restrict__ rows_team,
                                             float* __restrict__ cf_soa, bool collect,
                                             float* __restrict__ cf_aos, float* __restrict__ shw_tab,
                                             const float* __restrict__ sct, float* __restrict__ stash GS_PROF_PARAM) {
  constexpr int CL = T::T_CL, CC = T::T_CC, RC = T::T_RC, NCH = T::T_NCH, LN = T::T_LANES;
  static_assert(NCH == LN && LN == 4, "lane teams are DPP quads with one chain per lane");
  using C = CM<T>;
  using RS = RowSlots<T>;
  uintptr_t mp = reinterpret_cast<uintptr_t>(Min);
  asm volatile("" : "+s"(mp));
  const DevModel* __restrict__ M = reinterpret_cast<const DevModel*>(mp);
  const float* cm = mdl + lc;  // this lane's chain constants: cm[p * LN]
  const float h = P.h;

  // ================= root (replicated)
  float R0[9];
  {
    const float inv = rsqrtf(s.quat[0] * s.quat[0] + s.quat[1] * s.quat[1] + s.quat[2] * s.quat[2] +
                             s.quat[3] * s.quat[3]);
    const float qn[4] = {s.quat[0] * inv, s.quat[1] * inv, s.quat[2] * inv, s.quat[3] * inv};
    quat_to_mat(qn, R0);
  }
  const float X0[3] = {0.f, 0.f, 0.f};
  float nub[6] = {s.w[0], s.w[1], s.w[2], s.vo[0], s.vo[1], s.vo[2]};
  const float A0[6] = {0.f, 0.f, 0.f, -P.g[0], -P.g[1], -P.g[2]};
  SpI I0;
  body_inertia(R0, X0, M->mass[0], M->com[0], M->inertia[0], I0);
  float F0[6];
  {
    float ia[6], iv[6], x6[6];
    spi_mul(I0, A0, ia);
    spi_mul(I0, nub, iv);
    crf(nub, iv, x6);
#pragma unroll
    for (int k = 0; k < 6; ++k) F0[k] = ia[k] + x6[k];
  }

  // ================= TERR: the mesh queries first, while little else is live (run inside the forward pass, where
  // the chain's spatial quantities are live, the query code spilled ~1 KB of registers per lane to scratch).  The
  // chain's body poses are walked here by the forward pass's own statements; results: distance, normal, friction.
  // (held in a type that is empty for plane scenes: dead arrays there cost the plane kernel 0.5 KB of scratch)
  struct TerrQ {
    float d[CC], n[CC][3], m[CC];                                        // chain candidates
    float rd[RC > 0 ? RC : 1], rn[RC > 0 ? RC : 1][3], rm[RC > 0 ? RC : 1];  // root candidates
  };
  struct NoTerrQ {};
  [[maybe_unused]] std::conditional_t<TERR, TerrQ, NoTerrQ> tq;
  if constexpr (TERR) {
    // each lane's queries: its chain's CC candidates, and root candidate lc (lanes lc < RC); world centres as
    // terrain_candidate forms them (root origin + the candidate's offset)
    constexpr int NQ = CC + 1;
    static_assert(RC <= LN, "one root candidate per lane of the team");
    float qc[NQ][3], qr[NQ];
    bool qv[NQ];
    float Rk[9], Xk[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < 9; ++f) Rk[f] = R0[f];
#pragma unroll
    for (int k = 0; k < CL; ++k) {
      const float* bp = cm + (k * C::BODY) * LN;
      float jR[9], jt[3], ax[3];
#pragma unroll
      for (int f = 0; f < 9; ++f) jR[f] = bp[f * LN];
#pragma unroll
      for (int f = 0; f < 3; ++f) { jt[f] = bp[(9 + f) * LN]; ax[f] = bp[(12 + f) * LN]; }
      float RJ[9], t[3], aw[3];
      mat3mul(Rk, jR, RJ);
      mat3vec(Rk, jt, t);
      Xk[0] += t[0]; Xk[1] += t[1]; Xk[2] += t[2];
      mat3vec(RJ, ax, aw);
      const float qj = s.q[k];
      if (T::jkind[1 + k] == 1) {
        float sn, cs;
        sincosf(qj, &sn, &cs);
        const float Cc = 1.f - cs;
        float Rq[9];
        Rq[0] = cs + ax[0] * ax[0] * Cc;         Rq[1] = ax[0] * ax[1] * Cc - ax[2] * sn; Rq[2] = ax[0] * ax[2] * Cc + ax[1] * sn;
        Rq[3] = ax[1] * ax[0] * Cc + ax[2] * sn; Rq[4] = cs + ax[1] * ax[1] * Cc;         Rq[5] = ax[1] * ax[2] * Cc - ax[0] * sn;
        Rq[6] = ax[2] * ax[0] * Cc - ax[1] * sn; Rq[7] = ax[2] * ax[1] * Cc + ax[0] * sn; Rq[8] = cs + ax[2] * ax[2] * Cc;
        mat3mul(RJ, Rq, Rk);
      } else {
#pragma unroll
        for (int f = 0; f < 9; ++f) Rk[f] = RJ[f];
        Xk[0] += aw[0] * qj; Xk[1] += aw[1] * qj; Xk[2] += aw[2] * qj;
      }
#pragma unroll
      for (int j = 0; j < CC; ++j) {
        if (T::T_ccb[j] == k) {
          const float* cp = cm + (C::CAND + 4 * j) * LN;
          const float pl[3] = {cp[0], cp[LN], cp[2 * LN]};
          float x[3];
          mat3vec(Rk, pl, x);
          x[0] += Xk[0]; x[1] += Xk[1]; x[2] += Xk[2];
#pragma unroll
          for (int f = 0; f < 3; ++f) qc[j][f] = s.p[f] + x[f];
          qr[j] = cp[3 * LN];
          qv[j] = true;
        }
      }
    }
    qv[CC] = lc < RC;
    qr[CC] = 0.f;
    qc[CC][0] = qc[CC][1] = qc[CC][2] = 0.f;
    if (lc < RC) {
      float x[3];
      mat3vec(R0, M->cpoint[lc], x);
#pragma unroll
      for (int f = 0; f < 3; ++f) qc[CC][f] = s.p[f] + x[f];
      qr[CC] = M->cradius[lc];
    }
    // the queries the block summary cannot rule out (gs_terrain::may_contact: sphere_contact's own first test) go
    // into one list for the whole wave -- typically a minority (knees, the base, lifted feet end here) -- and the
    // wave's 64 lanes run them side by side, instead of every lane running its NQ queries one after another (a
    // wave pays for a query slot whenever ANY of its lanes has a query in it).  The list lives in the self-collision
    // pose table (rewritten before each use there), kQItem floats per query: centre, radius, found, sep, normal.
    constexpr int kQItem = 9;
    static_assert(T::NPK > 0 && kShW * T::NS >= kQItem * (CC * LN + RC), "query list fits the pose table");
    float* ql = shw_tab;  // (the workgroup's table; a workgroup is one wave)
    const int wl = threadIdx.x & 63;
    const unsigned long long below = (1ull << wl) - 1ull;
    int slot[NQ];
    int cnt = 0;
#ifdef GS_PHASE_PROFILE
    const long long tq0 = clock64();
#endif
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool need = qv[q] && gs_terrain::may_contact(P.terr, qc[q], qr[q], qr[q] + P.contact_offset);
      const unsigned long long bal = __ballot(need);
      slot[q] = need ? cnt + __popcll(bal & below) : -1;
      if (need) {
        float* it = ql + slot[q] * kQItem;
        it[0] = qc[q][0]; it[1] = qc[q][1]; it[2] = qc[q][2]; it[3] = qr[q];
      }
      cnt += __popcll(bal);
    }
    __syncthreads();
#ifdef GS_PHASE_PROFILE
    const long long tq1 = clock64();
#endif
    // (the live lanes only: the lanes of envs past N left the kernel before the substep loop)
    const unsigned long long live = __ballot(true);
    const int nlive = __popcll(live);
    for (int i = __popcll(live & below); i < cnt; i += nlive) {
      float* it = ql + i * kQItem;
      const float cw[3] = {it[0], it[1], it[2]};
      const float r = it[3];
      float st = 0.f, nt[3] = {0.f, 0.f, 1.f};
      const bool found = gs_terrain::sphere_contact_scan(P.terr, cw, r, r + P.contact_offset, st, nt);
      it[4] = found ? 1.f : 0.f;
      it[5] = st;
      it[6] = nt[0]; it[7] = nt[1]; it[8] = nt[2];
    }
    __syncthreads();
#ifdef GS_PHASE_PROFILE
    if ((threadIdx.x & 63) == 0) {  // mesh query phases: [50] the may_contact culls, [51] the scans, [52] queries
      const long long tq2 = clock64();
      atomicAdd(&gs_phase_cycles[50], (unsigned long long)(tq1 - tq0));
      atomicAdd(&gs_phase_cycles[51], (unsigned long long)(tq2 - tq1));
      atomicAdd(&gs_phase_cycles[52], (unsigned long long)cnt);
    }
#endif
    // terrain_candidate's result: the deepest of the ground plane and the mesh surface
    float rd = 3.0e38f, rn[3] = {0.f, 0.f, 1.f}, rm = P.ground_mu;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float dist = P.has_ground ? qc[q][2] - qr[q] : 3.0e38f;
      float nrm[3] = {0.f, 0.f, 1.f};
      float smu = P.ground_mu;
      if (slot[q] >= 0) {
        const float* it = ql + slot[q] * kQItem;
        if (it[4] != 0.f && it[5] < dist) {
          dist = it[5];
          nrm[0] = it[6]; nrm[1] = it[7]; nrm[2] = it[8];
          smu = P.terr.mu;
        }
      }
      if (q < CC) {
        tq.d[q] = dist; tq.m[q] = smu;
        tq.n[q][0] = nrm[0]; tq.n[q][1] = nrm[1]; tq.n[q][2] = nrm[2];
      } else {
        rd = dist; rm = smu;
        rn[0] = nrm[0]; rn[1] = nrm[1]; rn[2] = nrm[2];
      }
    }
    // root candidate j's result lives in lane j of the team
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      tq.rd[j] = bcast(rd, j);
      tq.rm[j] = bcast(rm, j);
#pragma unroll
      for (int f = 0; f < 3; ++f) tq.rn[j][f] = bcast(rn[f], j);
    }
  }

  // ================= chain forward pass (lane-local)
  float R[CL][9], X[CL][3], S[CL][6], V[CL][6], A[CL][6], Fc[CL][6];
  SpI Ic[CL];
  bool act[CC];
  float sep[CC], cmu[CC];
  float cnrm[TERR ? CC : 1][3];  // TERR: each chain candidate's contact normal (the force outputs)
  // (a) body poses and joint axes; (b) the self-collision prepass, which needs only the poses -- run here, before
  // the chain's velocities, accelerations, inertias and forces are live, so its narrowphase spills nothing; (c)
  // the rest of the forward pass and the contact candidates
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    const float* Rp = k == 0 ? R0 : R[k - 1];
    const float* Xp = k == 0 ? X0 : X[k - 1];
    const float* bp = cm + (k * C::BODY) * LN;
    float jR[9], jt[3], ax[3];
#pragma unroll
    for (int f = 0; f < 9; ++f) jR[f] = bp[f * LN];
#pragma unroll
    for (int f = 0; f < 3; ++f) { jt[f] = bp[(9 + f) * LN]; ax[f] = bp[(12 + f) * LN]; }
    float RJ[9], t[3], aw[3];
    mat3mul(Rp, jR, RJ);
    mat3vec(Rp, jt, t);
    X[k][0] = Xp[0] + t[0]; X[k][1] = Xp[1] + t[1]; X[k][2] = Xp[2] + t[2];
    mat3vec(RJ, ax, aw);
    const float qj = s.q[k];
    if (T::jkind[1 + k] == 1) {
      float sn, cs;
      sincosf(qj, &sn, &cs);
      const float Cc = 1.f - cs;
      float Rq[9];
      Rq[0] = cs + ax[0] * ax[0] * Cc;         Rq[1] = ax[0] * ax[1] * Cc - ax[2] * sn; Rq[2] = ax[0] * ax[2] * Cc + ax[1] * sn;
      Rq[3] = ax[1] * ax[0] * Cc + ax[2] * sn; Rq[4] = cs + ax[1] * ax[1] * Cc;         Rq[5] = ax[1] * ax[2] * Cc - ax[0] * sn;
      Rq[6] = ax[2] * ax[0] * Cc - ax[1] * sn; Rq[7] = ax[2] * ax[1] * Cc + ax[0] * sn; Rq[8] = cs + ax[2] * ax[2] * Cc;
      mat3mul(RJ, Rq, R[k]);
      S[k][0] = aw[0]; S[k][1] = aw[1]; S[k][2] = aw[2];
      cross3(X[k], aw, &S[k][3]);
    } else {
#pragma unroll
      for (int f = 0; f < 9; ++f) R[k][f] = RJ[f];
      X[k][0] += aw[0] * qj; X[k][1] += aw[1] * qj; X[k][2] += aw[2] * qj;
      S[k][0] = S[k][1] = S[k][2] = 0.f;
      S[k][3] = aw[0]; S[k][4] = aw[1]; S[k][5] = aw[2];
    }
  }
  GS_PROF(0)  // root + chain poses
  // ================= self-collision prepass (rare narrowphase; the pool rows are built with the contact records)
  int npc = 0;
  float* pool = rows_own + RS::POOL * RW;
  if constexpr (T::NPK > 0) {
    if (P.self_collide) npc = team_self_contacts<T>(M, cm, P, mu_t, kTeamsPerBlock, 0, lc, R0, R, X, shw_tab, sct, pool);
  }
  GS_PROF(11)  // self-collision prepass
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    const float* Vp = k == 0 ? nub : V[k - 1];
    const float* Ap = k == 0 ? A0 : A[k - 1];
    const float* bp = cm + (k * C::BODY) * LN;
    const float qd = s.qd[k];
    float c6[6];
#pragma unroll
    for (int f = 0; f < 6; ++f) V[k][f] = Vp[f] + S[k][f] * qd;
    crm(V[k], S[k], c6);
#pragma unroll
    for (int f = 0; f < 6; ++f) A[k][f] = Ap[f] + c6[f] * qd;
    float com[3], Il[6];
#pragma unroll
    for (int f = 0; f < 3; ++f) com[f] = bp[(16 + f) * LN];
#pragma unroll
    for (int f = 0; f < 6; ++f) Il[f] = bp[(19 + f) * LN];
    body_inertia(R[k], X[k], bp[15 * LN], com, Il, Ic[k]);
    {
      float ia[6], iv[6], x6[6];
      spi_mul(Ic[k], A[k], ia);
      spi_mul(Ic[k], V[k], iv);
      crf(V[k], iv, x6);
#pragma unroll
      for (int f = 0; f < 6; ++f) Fc[k][f] = ia[f] + x6[f];
    }
    // ---- chain contact candidates on body k: activity + Jacobian rows into this lane's LDS column
#pragma unroll
    for (int j = 0; j < CC; ++j) {
      if (T::T_ccb[j] == k) {
        const float* cp = cm + (C::CAND + 4 * j) * LN;
        const float pl[3] = {cp[0], cp[LN], cp[2 * LN]};
        const float r = cp[3 * LN];
        float x[3];
        mat3vec(R[k], pl, x);
        x[0] += X[k][0]; x[1] += X[k][1]; x[2] += X[k][2];
        const int shape = T::T_RS + lc * T::T_SPC + T::T_ccs[j];
        if constexpr (TERR) {
          // deepest of the ground plane and the terrain mesh (gs_terrain.h), as the one-env-per-lane solver;
          // the contact frame (n, t1, t2) replaces the plane's (z, x, y)
          const float* nrm = tq.n[j];
          const float dist = tq.d[j], smu = tq.m[j];
          act[j] = dist < P.contact_offset;
          sep[j] = dist - P.rest_offset;
          cmu[j] = 0.5f * (mu_t[shape * kTeamsPerBlock] + smu);
          cnrm[j][0] = nrm[0]; cnrm[j][1] = nrm[1]; cnrm[j][2] = nrm[2];
          if (act[j]) {
            float dir[3][3];
            dir[0][0] = nrm[0]; dir[0][1] = nrm[1]; dir[0][2] = nrm[2];
            gs_terrain::tangents(nrm, dir[1], dir[2]);
            const float xc[3] = {x[0] - r * nrm[0], x[1] - r * nrm[1], x[2] - r * nrm[2]};
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
              const float* d = dir[rr];
              float xd[3];  // the row's angular part: d.(w x xc) = w.(xc x d)
              cross3(xc, d, xd);
              float* row = rows_own + RS::chain(j) * RW;
#pragma unroll
              for (int b = 0; b < 6; ++b) row[RS::zs(rr, RS::zslot(b)) * RW] = b < 3 ? xd[b] : d[b - 3];
#pragma unroll
              for (int kk = 0; kk < CL; ++kk) {
                float v = 0.f;
                if (kk <= k)
                  v = S[kk][3] * d[0] + S[kk][4] * d[1] + S[kk][5] * d[2] + S[kk][0] * xd[0] + S[kk][1] * xd[1] +
                      S[kk][2] * xd[2];
                row[RS::zs(rr, RS::zslot(6 + kk)) * RW] = v;
              }
            }
          }
        } else {
        const float dist = s.p[2] + x[2] - r;
        act[j] = P.has_ground && (dist < P.contact_offset);
        sep[j] = dist - P.rest_offset;
        cmu[j] = 0.5f * (mu_t[shape * kTeamsPerBlock] + P.ground_mu);
        if (act[j]) {
          const float xc[3] = {x[0], x[1], x[2] - r};
#pragma unroll
          for (int rr = 0; rr < 3; ++rr) {
            const int ax3 = (rr == 0) ? 2 : (rr == 1 ? 0 : 1);
            float* row = rows_own + RS::chain(j) * RW;
#pragma unroll
            for (int b = 0; b < 6; ++b) row[RS::zs(rr, RS::zslot(b)) * RW] = base_jac(xc, ax3, b);
#pragma unroll
            for (int kk = 0; kk < CL; ++kk) {
              float v = 0.f;
              if (kk <= k) {
                float tt[3];
                cross3(S[kk], xc, tt);
                v = S[kk][3 + ax3] + tt[ax3];
              }
              row[RS::zs(rr, RS::zslot(6 + kk)) * RW] = v;
            }
          }
        }
        }  // !TERR
      }
    }
  }

  GS_PROF(0)  // chain forward pass + contact Jacobians
  // ================= chain backward pass: composite inertia / force, bias, chain rows of M
  float Mcc[CL][CL], Mcb[CL][6], biasc[CL];
#pragma unroll
  for (int kk = 0; kk < CL; ++kk) {
    const int k = CL - 1 - kk;
    if (k < CL - 1) {
      Ic[k].m += Ic[k + 1].m;
#pragma unroll
      for (int f = 0; f < 3; ++f) Ic[k].h[f] += Ic[k + 1].h[f];
#pragma unroll
      for (int f = 0; f < 6; ++f) Ic[k].I[f] += Ic[k + 1].I[f];
#pragma unroll
      for (int f = 0; f < 6; ++f) Fc[k][f] += Fc[k + 1][f];
    }
    biasc[k] = dot6(S[k], Fc[k]);
    float Fk[6];
    spi_mul(Ic[k], S[k], Fk);
    Mcc[k][k] = dot6(S[k], Fk) + cm[(C::DOF + 3 * k + 2) * LN];
#pragma unroll
    for (int j = 0; j < k; ++j) Mcc[k][j] = dot6(S[j], Fk);
#pragma unroll
    for (int b = 0; b < 6; ++b) Mcb[k][b] = Fk[b];
  }
  // ================= root sums over the team
  float Fb[6], Mbb[6][6];
  SpI Ir;
  {
#pragma unroll
    for (int f = 0; f < 6; ++f) Fb[f] = F0[f] + quad_sum(Fc[0][f]);
    Ir.m = I0.m + quad_sum(Ic[0].m);
#pragma unroll
    for (int f = 0; f < 3; ++f) Ir.h[f] = I0.h[f] + quad_sum(Ic[0].h[f]);
#pragma unroll
    for (int f = 0; f < 6; ++f) Ir.I[f] = I0.I[f] + quad_sum(Ic[0].I[f]);
    Mbb[0][0] = Ir.I[0]; Mbb[1][1] = Ir.I[1]; Mbb[2][2] = Ir.I[2];
    Mbb[1][0] = Ir.I[3]; Mbb[2][0] = Ir.I[4]; Mbb[2][1] = Ir.I[5];
    Mbb[3][0] = 0.f;       Mbb[3][1] = Ir.h[2];  Mbb[3][2] = -Ir.h[1];
    Mbb[4][0] = -Ir.h[2];  Mbb[4][1] = 0.f;      Mbb[4][2] = Ir.h[0];
    Mbb[5][0] = Ir.h[1];   Mbb[5][1] = -Ir.h[0]; Mbb[5][2] = 0.f;
    Mbb[3][3] = Ir.m; Mbb[4][4] = Ir.m; Mbb[5][5] = Ir.m;
    Mbb[4][3] = 0.f; Mbb[5][3] = 0.f; Mbb[5][4] = 0.f;
  }

  // ================= L^T D L: chain dofs (lane-local) with the base Schur complement summed over the team
  {
    float corr[6][6];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b <= a; ++b) corr[a][b] = 0.f;
#pragma unroll
    for (int kk = 0; kk < CL; ++kk) {
      const int k = CL - 1 - kk;
      const float dinv = __builtin_amdgcn_rcpf(Mcc[k][k]);
#pragma unroll
      for (int jj = 0; jj < CL; ++jj) {
        const int j = k - 1 - jj;
        if (j >= 0) {
          const float a = Mcc[k][j] * dinv;
#pragma unroll
          for (int i = 0; i <= j; ++i) Mcc[j][i] -= a * Mcc[k][i];
#pragma unroll
          for (int b = 0; b < 6; ++b) Mcb[j][b] -= a * Mcb[k][b];
          Mcc[k][j] = a;
        }
      }
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        const int b = 5 - bb;
        const float a = Mcb[k][b] * dinv;
#pragma unroll
        for (int i = 0; i <= b; ++i) corr[b][i] -= a * Mcb[k][i];
        Mcb[k][b] = a;
      }
    }
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b <= a; ++b) Mbb[a][b] += quad_sum(corr[a][b]);
  }
#pragma unroll
  for (int kk = 0; kk < 6; ++kk) {
    const int k = 5 - kk;
    const float dinv = __builtin_amdgcn_rcpf(Mbb[k][k]);
#pragma unroll
    for (int ii = 0; ii < 6; ++ii) {
      const int i = k - 1 - ii;
      if (i >= 0) {
        const float a = Mbb[k][i] * dinv;
#pragma unroll
        for (int j = 0; j <= i; ++j) Mbb[i][j] -= a * Mbb[k][j];
        Mbb[k][i] = a;
      }
    }
  }
  float sDc[CL], sDb[6];
#pragma unroll
  for (int k = 0; k < CL; ++k) sDc[k] = rsqrtf(Mcc[k][k]);
#pragma unroll
  for (int k = 0; k < 6; ++k) sDb[k] = rsqrtf(Mbb[k][k]);

  GS_PROF(1)  // backward pass, team sums, L^T D L
  // ================= free velocity
  float nufc[CL], nufb[6];
  {
    float rc[CL], rb[6], rcorr[6];
#pragma unroll
    for (int k = 0; k < CL; ++k) {
      float t = tau[k];
      const float ef = cm[(C::DOF + 3 * k + 0) * LN];
      if (ef > 0.f) t = clampf(t, -ef, ef);
      rc[k] = t - biasc[k];
    }
#pragma unroll
    for (int b = 0; b < 6; ++b) { rb[b] = -Fb[b]; rcorr[b] = 0.f; }
#pragma unroll
    for (int kk = 0; kk < CL; ++kk) {
      const int k = CL - 1 - kk;
#pragma unroll
      for (int j = 0; j < k; ++j) rc[j] -= Mcc[k][j] * rc[k];
#pragma unroll
      for (int b = 0; b < 6; ++b) rcorr[b] -= Mcb[k][b] * rc[k];
    }
#pragma unroll
    for (int b = 0; b < 6; ++b) rb[b] += quad_sum(rcorr[b]);
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      const int k = 5 - kk;
#pragma unroll
      for (int b = 0; b < k; ++b) rb[b] -= Mbb[k][b] * rb[k];
    }
#pragma unroll
    for (int b = 0; b < 6; ++b) rb[b] *= sDb[b] * sDb[b];
#pragma unroll
    for (int k = 0; k < CL; ++k) rc[k] *= sDc[k] * sDc[k];
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int b = 0; b < k; ++b) rb[k] -= Mbb[k][b] * rb[b];
#pragma unroll
    for (int k = 0; k < CL; ++k) {
#pragma unroll
      for (int b = 0; b < 6; ++b) rc[k] -= Mcb[k][b] * rb[b];
#pragma unroll
      for (int j = 0; j < k; ++j) rc[k] -= Mcc[k][j] * rc[j];
    }
#pragma unroll
    for (int b = 0; b < 6; ++b) nufb[b] = nub[b] + h * rb[b];
#pragma unroll
    for (int k = 0; k < CL; ++k) nufc[k] = s.qd[k] + h * rc[k];
    float wxp[3];
    cross3(&nub[0], &nub[3], wxp);
    nufb[3] += h * wxp[0]; nufb[4] += h * wxp[1]; nufb[5] += h * wxp[2];
  }

  GS_PROF(2)  // free velocity
  // ================= contact records: scaled Z = (L^-T J^T) D^-1/2, c = J nu_f, Delassus block
  const float inv_h = 1.f / h;
  // chain candidates (owner lane writes its column; the whole team reads it in the sweeps)
#pragma unroll
  for (int j = 0; j < CC; ++j) {
    float* rec = rows_own + RS::chain(j) * RW;
    rec[RS::C_ACT * RW] = act[j] ? 1.f : 0.f;
    if (act[j]) {
      const int kb = T::T_ccb[j];
      float zr[3][6 + CL], dir[3];
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        float* row = rows_own + RS::chain(j) * RW;
        auto Z = [&](int sl) -> float& { return row[RS::zs(rr, sl) * RW]; };
        float zb[6], zc[CL];
        float cj = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b) { zb[b] = Z(RS::zslot(b)); cj += zb[b] * nufb[b]; }
#pragma unroll
        for (int k = 0; k < CL; ++k) { zc[k] = Z(RS::zslot(6 + k)); if (k <= kb) cj += zc[k] * nufc[k]; }
        // leaf -> root: chain nodes kb..0 then base 5..0
#pragma unroll
        for (int kk = 0; kk < CL; ++kk) {
          const int k = kb - kk;
          if (k >= 0) {
#pragma unroll
            for (int i = 0; i < k; ++i) zc[i] -= Mcc[k][i] * zc[k];
#pragma unroll
            for (int b = 0; b < 6; ++b) zb[b] -= Mcb[k][b] * zc[k];
          }
        }
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
          const int k = 5 - kk;
#pragma unroll
          for (int b = 0; b < k; ++b) zb[b] -= Mbb[k][b] * zb[k];
        }
        float d = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          zb[b] *= sDb[b];
          d += zb[b] * zb[b];
          Z(RS::zslot(b)) = zb[b];
          zr[rr][b] = zb[b];
        }
#pragma unroll
        for (int k = 0; k < CL; ++k) {
          const float z = k <= kb ? zc[k] * sDc[k] : 0.f;
          d += z * z;
          Z(RS::zslot(6 + k)) = z;
          zr[rr][6 + k] = z;
        }
        Z(3) = 0.f;  // pads: lanes 0-2 add no constant, lane 3 owns no component
        Z(7) = 0.f;
        Z(11) = 0.f;
        Z(12) = 0.f;
        Z(13) = 0.f;
        Z(14) = 0.f;
        Z(RS::CSLOT) = cj;
        dir[rr] = d > 0.f ? __builtin_amdgcn_rcpf(d) : 0.f;  // (d == 0: a row the chain cannot move along)
        rec[(RS::C_DI + rr) * RW] = dir[rr];
      }
      float g10 = 0.f, g20 = 0.f, g21 = 0.f;
#pragma unroll
      for (int f = 0; f < 6 + CL; ++f) {
        g10 += zr[1][f] * zr[0][f];
        g20 += zr[2][f] * zr[0][f];
        g21 += zr[2][f] * zr[1][f];
      }
      rec[(RS::C_G + 0) * RW] = g10 * dir[1];
      rec[(RS::C_G + 1) * RW] = g20 * dir[2];
      rec[(RS::C_G + 2) * RW] = g21 * dir[2];
      const float sc = sep[j];
      const float tgt = -sc * inv_h;
      rec[RS::C_TP * RW] = (sc < 0.f ? fminf(tgt, P.max_depen_vel) : tgt) * dir[0];
      rec[RS::C_TV * RW] = (sc < 0.f ? 0.f : tgt) * dir[0];
      rec[RS::C_MU * RW] = cmu[j];
      rec[RS::C_SEP * RW] = sc;
    }
  }
  // root candidates (replicated in every lane, own column; TERR: lane j % 4 runs root candidate j's mesh query
  // and broadcasts its result to the team)
  bool ract[RC > 0 ? RC : 1];
  float rnrm[TERR && RC > 0 ? RC : 1][3];
#pragma unroll
  for (int j = 0; j < RC; ++j) {
    float x[3];
    mat3vec(R0, M->cpoint[j], x);
    const float r = M->cradius[j];
    float dist, rmu_s = P.ground_mu;
    float rdir[3][3];
    if constexpr (TERR) {
      dist = tq.rd[j];
      rmu_s = tq.rm[j];
#pragma unroll
      for (int f = 0; f < 3; ++f) rnrm[j][f] = tq.rn[j][f];
      ract[j] = dist < P.contact_offset;
      rdir[0][0] = rnrm[j][0]; rdir[0][1] = rnrm[j][1]; rdir[0][2] = rnrm[j][2];
      gs_terrain::tangents(rnrm[j], rdir[1], rdir[2]);
    } else {
      dist = s.p[2] + x[2] - r;
      ract[j] = P.has_ground && (dist < P.contact_offset);
    }
    if (ract[j]) {
      float* rec = rows_own + RS::root(j) * RW;
      const float xc[3] = {TERR ? x[0] - r * rdir[0][0] : x[0], TERR ? x[1] - r * rdir[0][1] : x[1],
                           TERR ? x[2] - r * rdir[0][2] : x[2] - r};
      float zr[3][6], dir[3];
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        const int ax3 = (rr == 0) ? 2 : (rr == 1 ? 0 : 1);
        float zb[6], cj = 0.f;
        float xd[3] = {0.f, 0.f, 0.f};
        if constexpr (TERR) cross3(xc, rdir[rr], xd);
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          zb[b] = TERR ? (b < 3 ? xd[b] : rdir[rr][b - 3]) : base_jac(xc, ax3, b);
          cj += zb[b] * nufb[b];
        }
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
          const int k = 5 - kk;
#pragma unroll
          for (int b = 0; b < k; ++b) zb[b] -= Mbb[k][b] * zb[k];
        }
        float d = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b) {
          zb[b] *= sDb[b];
          d += zb[b] * zb[b];
          rec[RS::zs(rr, RS::zslot(b)) * RW] = zb[b];
          zr[rr][b] = zb[b];
        }
        auto Z = [&](int sl) -> float& { return rec[RS::zs(rr, sl) * RW]; };
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // no chain components; pads as in the chain records
          Z(4 * k + 2) = 0.f;
          Z(4 * k + 3) = 0.f;
        }
        Z(12) = 0.f;
        Z(13) = 0.f;
        Z(14) = 0.f;
        Z(RS::CSLOT) = cj;
        dir[rr] = d > 0.f ? __builtin_amdgcn_rcpf(d) : 0.f;  // (d == 0: a row the chain cannot move along)
        rec[(RS::R_DI + rr) * RW] = dir[rr];
      }
      float g10 = 0.f, g20 = 0.f, g21 = 0.f;
#pragma unroll
      for (int f = 0; f < 6; ++f) {
        g10 += zr[1][f] * zr[0][f];
        g20 += zr[2][f] * zr[0][f];
        g21 += zr[2][f] * zr[1][f];
      }
      rec[(RS::R_G + 0) * RW] = g10 * dir[1];
      rec[(RS::R_G + 1) * RW] = g20 * dir[2];
      rec[(RS::R_G + 2) * RW] = g21 * dir[2];
      const float sc = dist - P.rest_offset;
      const float tgt = -sc * inv_h;
      rec[RS::R_TP * RW] = (sc < 0.f ? fminf(tgt, P.max_depen_vel) : tgt) * dir[0];
      rec[RS::R_TV * RW] = (sc < 0.f ? 0.f : tgt) * dir[0];
      rec[RS::R_MU * RW] = 0.5f * (mu_t[T::T_rcs[j] * kTeamsPerBlock] + rmu_s);
      rec[RS::R_SEP * RW] = sc;
    }
  }
  // self-contact pool rows: J = n.(v_A(x) - v_B(x)) has columns only on the two chains below
  // the root (the base columns cancel); each lane forms its own chain's part, eliminates it through its L factor,
  // the base part is the team sum eliminated through the replicated base block; the lane then keeps the
  // components it owns in the distributed PGS (base 2l, 2l+1; component l of chains A and B; lane 3: c)
  if constexpr (T::NPK > 0) {
    for (int p = 0; p < npc; ++p) {
      float* o = pool + RS::PER_POOL * p * RW;
      const int ba = (int)o[kPoolBA * RW], bb = (int)o[kPoolBB * RW];
      const int ca = ba > 0 ? (ba - 1) / CL : -1, ka = ba > 0 ? (ba - 1) - ca * CL : -1;
      const int cb = bb > 0 ? (bb - 1) / CL : -1, kb = bb > 0 ? (bb - 1) - cb * CL : -1;
      const float x[3] = {o[kPoolX * RW], o[(kPoolX + 1) * RW], o[(kPoolX + 2) * RW]};
      float zr[3][6], zc3[3][CL], dd[3];
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        const int dofs = rr == 0 ? kPoolN : (rr == 1 ? kPoolT1 : kPoolT2);
        const float d[3] = {o[dofs * RW], o[(dofs + 1) * RW], o[(dofs + 2) * RW]};
        float zc[CL], zbc[6];
        float cpart = 0.f;
#pragma unroll
        for (int k = 0; k < CL; ++k) {
          const float coef = (lc == ca && k <= ka ? 1.f : 0.f) - (lc == cb && k <= kb ? 1.f : 0.f);
          float vx[3];
          cross3(S[k], x, vx);
          zc[k] = coef * (d[0] * (S[k][3] + vx[0]) + d[1] * (S[k][4] + vx[1]) + d[2] * (S[k][5] + vx[2]));
          cpart += zc[k] * nufc[k];
        }
#pragma unroll
        for (int b = 0; b < 6; ++b) zbc[b] = 0.f;
#pragma unroll
        for (int kk = 0; kk < CL; ++kk) {
          const int k = CL - 1 - kk;
#pragma unroll
          for (int i = 0; i < k; ++i) zc[i] -= Mcc[k][i] * zc[k];
#pragma unroll
          for (int b = 0; b < 6; ++b) zbc[b] -= Mcb[k][b] * zc[k];
        }
        float zb[6];
#pragma unroll
        for (int b = 0; b < 6; ++b) zb[b] = quad_sum(zbc[b]);
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
          const int k = 5 - kk;
#pragma unroll
          for (int b = 0; b < k; ++b) zb[b] -= Mbb[k][b] * zb[k];
        }
        float own = 0.f, db = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b) { zb[b] *= sDb[b]; db += zb[b] * zb[b]; zr[rr][b] = zb[b]; }
#pragma unroll
        for (int k = 0; k < CL; ++k) { zc[k] *= sDc[k]; own += zc[k] * zc[k]; zc3[rr][k] = zc[k]; }
        dd[rr] = db + quad_sum(own);
        const float cj = quad_sum(cpart);
        // distributed components: chain A / B component lc (from lane ca / cb), base 2 lc, 2 lc + 1
        float za = 0.f, zbb = 0.f;
#pragma unroll
        for (int l = 0; l < CL; ++l) {
          float va = 0.f, vb = 0.f;
#pragma unroll
          for (int L = 0; L < 4; ++L) {
            const float t = bcast(zc[l], L);
            va = L == ca ? t : va;
            vb = L == cb ? t : vb;
          }
          za = lc == l ? va : za;
          zbb = lc == l ? vb : zbb;
        }
        if (cb == ca) zbb = 0.f;  // one chain: its components carry both sides already
        const float b0 = lc == 0 ? zb[0] : (lc == 1 ? zb[2] : (lc == 2 ? zb[4] : 0.f));
        const float b1 = lc == 0 ? zb[1] : (lc == 1 ? zb[3] : (lc == 2 ? zb[5] : 0.f));
        float* zo = o + (RS::P_Z + 5 * rr) * RW;
        zo[0] = b0;
        zo[RW] = b1;
        zo[2 * RW] = za;
        zo[3 * RW] = zbb;
        zo[4 * RW] = lc == 3 ? cj : 0.f;
      }
      float g10 = 0.f, g20 = 0.f, g21 = 0.f, c10 = 0.f, c20 = 0.f, c21 = 0.f;
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        g10 += zr[1][b] * zr[0][b];
        g20 += zr[2][b] * zr[0][b];
        g21 += zr[2][b] * zr[1][b];
      }
#pragma unroll
      for (int k = 0; k < CL; ++k) {
        c10 += zc3[1][k] * zc3[0][k];
        c20 += zc3[2][k] * zc3[0][k];
        c21 += zc3[2][k] * zc3[1][k];
      }
      g10 += quad_sum(c10);
      g20 += quad_sum(c20);
      g21 += quad_sum(c21);
      float di[3];
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        di[rr] = dd[rr] > GS_MIN_RESPONSE ? __builtin_amdgcn_rcpf(dd[rr]) : 0.f;
        o[(RS::P_DI + rr) * RW] = di[rr];
        o[(kPoolLam + rr) * RW] = 0.f;
      }
      o[(RS::P_G + 0) * RW] = g10 * di[1];
      o[(RS::P_G + 1) * RW] = g20 * di[2];
      o[(RS::P_G + 2) * RW] = g21 * di[2];
      const float sc = o[kPoolSep * RW];
      const float tgt = -sc * inv_h;
      o[RS::P_TP * RW] = (sc < 0.f ? fminf(tgt, P.max_depen_vel) : tgt) * di[0];
      o[RS::P_TV * RW] = (sc < 0.f ? 0.f : tgt) * di[0];
      o[RS::P_CA * RW] = (float)ca;
      o[RS::P_CB * RW] = (float)(cb == ca ? -1 : cb);
    }
  }
  // the sweeps read other lanes' records: make this wave's LDS writes visible (one-wave block)
  __syncthreads();

  GS_PROF(3)  // contact records
  // The factorisation and the free velocity are read again only after the sweeps (back-substitution): they wait
  // in the lane's LDS stash meanwhile, so the sweeps have their registers (the records of all contacts in flight,
  // register pairs for the packed row partials) -- round 6; they spilled to scratch otherwise
  auto stash_io = [&](bool save) {
    int q = 0;
    auto io = [&](float& v) {
      if (save) stash[q * kTeamBlock] = v; else v = stash[q * kTeamBlock];
      ++q;
    };
#pragma unroll
    for (int k = 0; k < 6; ++k) {
#pragma unroll
      for (int b = 0; b < k; ++b) io(Mbb[k][b]);
      io(sDb[k]);
      io(nufb[k]);
    }
#pragma unroll
    for (int k = 0; k < CL; ++k) {
#pragma unroll
      for (int b = 0; b < 6; ++b) io(Mcb[k][b]);
#pragma unroll
      for (int j = 0; j < k; ++j) io(Mcc[k][j]);
      io(sDc[k]);
      io(nufc[k]);
    }
  };
  stash_io(true);
  // ================= projected Gauss-Seidel, global contact order: root candidates, chain 0, 1, ...
  // The 9 velocity components a chain contact row touches (base 6 | its chain's 3) are spread over
  // the team: lane l < 3 owns base 2l, base 2l+1 and chain component l (RowSlots).  Each lane forms
  // its partial of the 3 rows' u = c + Z w (lane 3: c), a DPP quad sum completes them
  // (bit-identical in the 4 lanes), the 3-row projection through the contact's Delassus couplings
  // runs replicated, and each lane updates only what it owns.
  static_assert(CL == 3, "component distribution assumes 3-dof chains");
  float wA = 0.f, wA2 = 0.f, wC[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) wC[c] = 0.f;
  float lamc[NCH][CC][3], lamr[RC > 0 ? RC : 1][3];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < CC; ++j) lamc[c][j][0] = lamc[c][j][1] = lamc[c][j][2] = 0.f;
#pragma unroll
  for (int j = 0; j < RC; ++j) lamr[j][0] = lamr[j][1] = lamr[j][2] = 0.f;
  float wbp[6], wcp[CL];
  const int iters = P.pos_iters + P.vel_iters;
  // TGS (physx.solver_type 1; oracle/physics_oracle.c solver_type 3): the position iterations are
  // sub-steps of hs = h / pos_iters; a row's separation is advanced by J dq, dq = hs (v_0 + ... + v_{k-1}) the
  // displacement of the sub-steps done (in w space: Z (w_0 + ... + w_{k-1}) + k c, the sums kept in aA / aA2 /
  // aC); its target: a gap closes within the sub-step (-s / hs), a penetration is pushed out at -s / h (capped),
  // over the whole step; the velocity iterations target the gap left after the sub-steps; the positions integrate
  // the sub-steps' mean velocity.  PGS (0): the split-impulse targets precomputed in the records.
  // (TGS is a template parameter: the PGS kernels carry none of its state, and its target is branch-free)
  constexpr bool tgs = TGS;
  const float hs = tgs ? h / (float)P.pos_iters : h, inv_hs = 1.f / hs;
  [[maybe_unused]] float aA = 0.f, aA2 = 0.f, aC[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) aC[c] = 0.f;
  for (int it = 0; it < iters; ++it) {
    const int tsel = it < P.pos_iters ? RS::C_TP : RS::C_TV;
    const int rsel = it < P.pos_iters ? RS::R_TP : RS::R_TV;
    const bool pos = it < P.pos_iters;
    const float na = (float)(it < P.pos_iters ? it : P.pos_iters);  // sub-steps done
    // the TGS target of a row at separation sep (wave-uniform factors): a gap closes at -sep / hs in a position
    // sub-step, at -sep / h in a velocity iteration; a penetration is pushed out at -sep / h capped at
    // max_depenetration_velocity in a position sub-step, not at all in a velocity iteration (the cap 0)
    const float kgap = pos ? inv_hs : inv_h, cap = pos ? P.max_depen_vel : 0.f;
    auto tgs_tdi = [&](float sc, float su, float di0) {
      const float sep = fmaf(hs, su, sc);
      const float t = sep >= 0.f ? -sep * kgap : fminf(-sep * inv_h, cap);
      return t * di0;
    };
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      if (ract[j]) {
        const float* rec = rows_own + RS::root(j) * RW;
        float z[12], u[4];
#pragma unroll
        for (int i = 0; i < 12; ++i) z[i] = rec[RS::zs(i >> 2, 4 * lc + (i & 3)) * RW];
        {
          const f2 u01 = pk_fma(f2{z[0], z[4]}, f2{wA, wA}, pk_fma(f2{z[1], z[5]}, f2{wA2, wA2}, f2{z[3], z[7]}));
          u[0] = u01.x;
          u[1] = u01.y;
        }
        u[2] = fmaf(z[8], wA, fmaf(z[9], wA2, z[11]));
        float tdi;
        if constexpr (tgs) {
          u[3] = fmaf(z[0], aA, fmaf(z[1], aA2, na * z[3]));
          quad_sum4(u);
          tdi = tgs_tdi(rec[RS::R_SEP * RW], u[3], rec[RS::R_DI * RW]);
        } else {
          quad_sum3(u);
          tdi = rec[rsel * RW];
        }
        float dl0, dl1, dl2;
        contact_block(u[0], u[1], u[2], rec[RS::R_DI * RW], rec[(RS::R_DI + 1) * RW], rec[(RS::R_DI + 2) * RW],
                      rec[RS::R_G * RW], rec[(RS::R_G + 1) * RW], rec[(RS::R_G + 2) * RW], tdi,
                      rec[RS::R_MU * RW], lamr[j], dl0, dl1, dl2);
        wA = fmaf(z[8], dl2, fmaf(z[4], dl1, fmaf(z[0], dl0, wA)));
        wA2 = fmaf(z[9], dl2, fmaf(z[5], dl1, fmaf(z[1], dl0, wA2)));
      }
    }
    // software-pipelined over the NCH*CC chain contacts: the next contact's whole record (activity,
    // this lane's Z components and c, the Delassus block, target, mu) is loaded before this
    // contact's (divergent) block, so its LDS latency overlaps the block
    float nact, nz[12], nk[8];  // nk: 1/G_rr (3) | scaled couplings (3) | target (TGS: separation) | mu
    auto fetch = [&](int n) {
      const int cc = n / CC, j = n - (n / CC) * CC;
      const float* rec = rows_team + cc + RS::chain(j) * RW;
      nact = rec[RS::C_ACT * RW];
#pragma unroll
      for (int i = 0; i < 12; ++i) nz[i] = rec[RS::zs(i >> 2, 4 * lc + (i & 3)) * RW];
#pragma unroll
      for (int i = 0; i < 6; ++i) nk[i] = rec[(RS::C_DI + i) * RW];
      nk[6] = rec[(tgs ? RS::C_SEP : tsel) * RW];
      nk[7] = rec[RS::C_MU * RW];
    };
    fetch(0);
#pragma unroll
    for (int n = 0; n < NCH * CC; ++n) {
      const int cc = n / CC, j = n - (n / CC) * CC;
      float z[12], k8[8];
      const float act_n = nact;
#pragma unroll
      for (int i = 0; i < 12; ++i) z[i] = nz[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) k8[i] = nk[i];
      // (the scheduler hoists all 12 records' loads to the top of the sweep and parks them in AGPRs;
      // measured faster than keeping the prefetch one contact deep with a scheduling fence:
      // 0.0886 vs 0.0915 ms per launch, profiles/r02o_experiments_team_pgs.txt)
#ifdef GS_PGS_FENCE
      __builtin_amdgcn_sched_barrier(0);  // (A/B: keep the prefetch one contact deep)
#endif
      if (n + 1 < NCH * CC) fetch(n + 1);
      const bool a_o = act_n != 0.f;
#ifdef GS_PHASE_PROFILE
      if (__ballot(a_o) != 0ull) GS_PROF_COUNT(8, 1)  // chain contacts the wave executes
#endif
      if (a_o) {
        float u[4];
        {  // the w terms last (they carry the Gauss-Seidel chain); rows 0 and 1 as register pairs
          const f2 u01 = pk_fma(f2{z[0], z[4]}, f2{wA, wA},
                                pk_fma(f2{z[1], z[5]}, f2{wA2, wA2}, pk_fma(f2{z[2], z[6]}, f2{wC[cc], wC[cc]},
                                                                         f2{z[3], z[7]})));
          u[0] = u01.x;
          u[1] = u01.y;
        }
        u[2] = fmaf(z[8], wA, fmaf(z[9], wA2, fmaf(z[10], wC[cc], z[11])));
        float tdi = k8[6];
        if constexpr (tgs) {
          u[3] = fmaf(z[0], aA, fmaf(z[1], aA2, fmaf(z[2], aC[cc], na * z[3])));
          quad_sum4(u);
          tdi = tgs_tdi(k8[6], u[3], k8[0]);
        } else {
          quad_sum3(u);
        }
        float dl0, dl1, dl2;
        contact_block(u[0], u[1], u[2], k8[0], k8[1], k8[2], k8[3], k8[4], k8[5], tdi, k8[7], lamc[cc][j], dl0,
                      dl1, dl2);
        wA = fmaf(z[8], dl2, fmaf(z[4], dl1, fmaf(z[0], dl0, wA)));
        wA2 = fmaf(z[9], dl2, fmaf(z[5], dl1, fmaf(z[1], dl0, wA2)));
        wC[cc] = fmaf(z[10], dl2, fmaf(z[6], dl1, fmaf(z[2], dl0, wC[cc])));
      }
    }
    if constexpr (T::NPK > 0) {
      const int psel = it < P.pos_iters ? RS::P_TP : RS::P_TV;
      // unrolled over the pool's NPK slots with the next entry's record loaded ahead (as the chain contacts);
      // the wave runs as many entries as its fullest team has (npc is per team)
      float pz[15], pk[11];  // Z components | lam (3), 1/G_rr (3), couplings (3), target (TGS: separation), mu
      int pca = 0, pcb = 0;
      auto pfetch = [&](int p) {
        const float* o = pool + RS::PER_POOL * p * RW;
#pragma unroll
        for (int i = 0; i < 15; ++i) pz[i] = o[(RS::P_Z + i) * RW];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          pk[i] = o[(kPoolLam + i) * RW];
          pk[3 + i] = o[(RS::P_DI + i) * RW];
          pk[6 + i] = o[(RS::P_G + i) * RW];
        }
        pk[9] = o[(tgs ? (int)kPoolSep : psel) * RW];
        pk[10] = o[kPoolMu * RW];
        pca = (int)o[RS::P_CA * RW];
        pcb = (int)o[RS::P_CB * RW];
      };
      const unsigned long long any_pool = __ballot(npc > 0);
      if (any_pool) pfetch(0);
#pragma unroll
      for (int p = 0; p < T::NPK; ++p) {
        if (__ballot(p < npc) == 0ull) break;
        float z[15], k11[11];
#pragma unroll
        for (int i = 0; i < 15; ++i) z[i] = pz[i];
#pragma unroll
        for (int i = 0; i < 11; ++i) k11[i] = pk[i];
        const int ca = pca, cb = pcb;
        if (p + 1 < T::NPK) pfetch(p + 1);
        if (p < npc) {
          float wa = 0.f, wb = 0.f, ana = 0.f, anb = 0.f;
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            wa = c == ca ? wC[c] : wa;
            wb = c == cb ? wC[c] : wb;
            ana = c == ca ? aC[c] : ana;
            anb = c == cb ? aC[c] : anb;
          }
          float u[4];
#pragma unroll
          for (int rr = 0; rr < 3; ++rr)
            u[rr] = fmaf(z[5 * rr], wA, fmaf(z[5 * rr + 1], wA2, fmaf(z[5 * rr + 2], wa, fmaf(z[5 * rr + 3], wb, z[5 * rr + 4]))));
          float lam[3] = {k11[0], k11[1], k11[2]};
          float tdi = k11[9];
          if constexpr (tgs) {
            u[3] = fmaf(z[0], aA, fmaf(z[1], aA2, fmaf(z[2], ana, fmaf(z[3], anb, na * z[4]))));
            quad_sum4(u);
            tdi = tgs_tdi(k11[9], u[3], k11[3]);
          } else {
            quad_sum3(u);
          }
          float dl0, dl1, dl2;
          contact_block(u[0], u[1], u[2], k11[3], k11[4], k11[5], k11[6], k11[7], k11[8], tdi, k11[10], lam, dl0, dl1,
                        dl2);
          float* o = pool + RS::PER_POOL * p * RW;
          o[kPoolLam * RW] = lam[0];
          o[(kPoolLam + 1) * RW] = lam[1];
          o[(kPoolLam + 2) * RW] = lam[2];
          wA = fmaf(z[10], dl2, fmaf(z[5], dl1, fmaf(z[0], dl0, wA)));
          wA2 = fmaf(z[11], dl2, fmaf(z[6], dl1, fmaf(z[1], dl0, wA2)));
          const float da = fmaf(z[12], dl2, fmaf(z[7], dl1, z[2] * dl0));
          const float db = fmaf(z[13], dl2, fmaf(z[8], dl1, z[3] * dl0));
#pragma unroll
          for (int c = 0; c < NCH; ++c) wC[c] += (c == ca ? da : 0.f) + (c == cb ? db : 0.f);
        }
      }
    }
#ifdef GS_PHASE_PROFILE
    for (int j = 0; j < RC; ++j)
      if (__ballot(ract[j]) != 0ull) GS_PROF_COUNT(9, 1)  // root contacts the wave executes
#endif
    if (tgs && pos) {  // the sub-step's velocity joins the displacement
      aA += wA;
      aA2 += wA2;
#pragma unroll
      for (int c = 0; c < NCH; ++c) aC[c] += wC[c];
    }
    if (it == P.pos_iters - 1) {
      if constexpr (tgs) {  // positions integrate the sub-steps' mean velocity (w space is linear)
        const float inv_n = 1.f / (float)P.pos_iters;
        float mC[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) mC[c] = aC[c] * inv_n;
        gather_w<T>(lc, aA * inv_n, aA2 * inv_n, mC, wbp, wcp);
      } else {
        gather_w<T>(lc, wA, wA2, wC, wbp, wcp);
      }
    }
  }
  float wb[6], wc[CL];
  gather_w<T>(lc, wA, wA2, wC, wb, wc);
  if (P.pos_iters <= 0) {
#pragma unroll
    for (int b = 0; b < 6; ++b) wbp[b] = wb[b];
#pragma unroll
    for (int k = 0; k < CL; ++k) wcp[k] = wc[k];
  }
  __syncthreads();  // the next substep rewrites the records other lanes just read
  stash_io(false);

  GS_PROF(4)  // PGS
  // ================= dnu = L^-1 D^-1/2 w (base first, then the chain)
  float nunb[6], nupb[6], nunc[CL], nupc[CL];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    float v = wb[k] * sDb[k], vp = wbp[k] * sDb[k];
#pragma unroll
    for (int b = 0; b < k; ++b) { v -= Mbb[k][b] * nunb[b]; vp -= Mbb[k][b] * nupb[b]; }
    nunb[k] = v;
    nupb[k] = vp;
  }
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    float v = wc[k] * sDc[k], vp = wcp[k] * sDc[k];
#pragma unroll
    for (int b = 0; b < 6; ++b) { v -= Mcb[k][b] * nunb[b]; vp -= Mcb[k][b] * nupb[b]; }
#pragma unroll
    for (int j = 0; j < k; ++j) { v -= Mcc[k][j] * nunc[j]; vp -= Mcc[k][j] * nupc[j]; }
    nunc[k] = v;
    nupc[k] = vp;
  }
#pragma unroll
  for (int b = 0; b < 6; ++b) { nunb[b] += nufb[b]; nupb[b] += nufb[b]; }
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    float vn = nunc[k] + nufc[k], vp = nupc[k] + nufc[k];
    const float vm = cm[(C::DOF + 3 * k + 1) * LN];
    if (vm > 0.f) { vn = clampf(vn, -vm, vm); vp = clampf(vp, -vm, vm); }
    nunc[k] = vn;
    nupc[k] = vp;
  }

  // ================= integrate
  s.p[0] += h * nupb[3]; s.p[1] += h * nupb[4]; s.p[2] += h * nupb[5];
  {
    const float wx = nupb[0], wy = nupb[1], wz = nupb[2];
    float x = s.quat[0], y = s.quat[1], z = s.quat[2], w = s.quat[3];
    const float hh = 0.5f * h;
    const float dx = hh * (w * wx + wy * z - wz * y);
    const float dy = hh * (w * wy + wz * x - wx * z);
    const float dz = hh * (w * wz + wx * y - wy * x);
    const float dw = -hh * (wx * x + wy * y + wz * z);
    x += dx; y += dy; z += dz; w += dw;
    const float n = rsqrtf(x * x + y * y + z * z + w * w);
    s.quat[0] = x * n; s.quat[1] = y * n; s.quat[2] = z * n; s.quat[3] = w * n;
  }
  s.w[0] = nunb[0]; s.w[1] = nunb[1]; s.w[2] = nunb[2];
  s.vo[0] = nunb[3]; s.vo[1] = nunb[4]; s.vo[2] = nunb[5];
#pragma unroll
  for (int k = 0; k < CL; ++k) {
    s.q[k] += h * nupc[k];
    s.qd[k] = nunc[k];
  }
  if (collect) {
    // (output addresses formed here: opaque_index)
    e = opaque_index(e);
#pragma unroll
    for (int k = 0; k < CL; ++k) {
      float f0 = 0.f, f1 = 0.f, f2 = 0.f;
#pragma unroll
      for (int j = 0; j < CC; ++j) {
        if (T::T_ccb[j] == k) {
          float l0 = lamc[0][j][0], l1 = lamc[0][j][1], l2 = lamc[0][j][2];
#pragma unroll
          for (int c = 1; c < NCH; ++c) {
            l0 = lc == c ? lamc[c][j][0] : l0;
            l1 = lc == c ? lamc[c][j][1] : l1;
            l2 = lc == c ? lamc[c][j][2] : l2;
          }
          if constexpr (TERR) {  // f = (l0 n + l1 t1 + l2 t2) / h in the candidate's mesh frame
            float t1[3], t2[3];
            gs_terrain::tangents(cnrm[j], t1, t2);
            f0 += (l0 * cnrm[j][0] + l1 * t1[0] + l2 * t2[0]) * inv_h;
            f1 += (l0 * cnrm[j][1] + l1 * t1[1] + l2 * t2[1]) * inv_h;
            f2 += (l0 * cnrm[j][2] + l1 * t1[2] + l2 * t2[2]) * inv_h;
          } else {
            f0 += l1 * inv_h;
            f1 += l2 * inv_h;
            f2 += l0 * inv_h;
          }
        }
      }
      if constexpr (T::NPK > 0) {  // self-contacts: +f on body A, -f on body B
        for (int p = 0; p < npc; ++p) {
          const float* o = pool + RS::PER_POOL * p * RW;
          const int bk = 1 + lc * CL + k;
          const float sg = ((int)o[kPoolBA * RW] == bk ? inv_h : 0.f) - ((int)o[kPoolBB * RW] == bk ? inv_h : 0.f);
          if (sg != 0.f) {
            const float l0 = o[kPoolLam * RW], l1 = o[(kPoolLam + 1) * RW], l2 = o[(kPoolLam + 2) * RW];
            f0 += sg * (l0 * o[kPoolN * RW] + l1 * o[kPoolT1 * RW] + l2 * o[kPoolT2 * RW]);
            f1 += sg * (l0 * o[(kPoolN + 1) * RW] + l1 * o[(kPoolT1 + 1) * RW] + l2 * o[(kPoolT2 + 1) * RW]);
            f2 += sg * (l0 * o[(kPoolN + 2) * RW] + l1 * o[(kPoolT1 + 2) * RW] + l2 * o[(kPoolT2 + 2) * RW]);
          }
        }
      }
      const int b = 1 + lc * CL + k;
      cf_soa[(3 * b + 0) * N + e] = f0;
      cf_soa[(3 * b + 1) * N + e] = f1;
      cf_soa[(3 * b + 2) * N + e] = f2;
      if (cf_aos) {  // net contact force tensor [N*nb][3] (the launch's last collecting substep)
        float* o = cf_aos + ((size_t)e * T::NB + b) * 3;
        o[0] = f0; o[1] = f1; o[2] = f2;
      }
    }
    if (lc == 0) {
      float f0 = 0.f, f1 = 0.f, f2 = 0.f;
#pragma unroll
      for (int j = 0; j < RC; ++j) {
        if constexpr (TERR) {
          float t1[3], t2[3];
          gs_terrain::tangents(rnrm[j], t1, t2);
          const float g = ract[j] ? inv_h : 0.f;
          f0 += (lamr[j][0] * rnrm[j][0] + lamr[j][1] * t1[0] + lamr[j][2] * t2[0]) * g;
          f1 += (lamr[j][0] * rnrm[j][1] + lamr[j][1] * t1[1] + lamr[j][2] * t2[1]) * g;
          f2 += (lamr[j][0] * rnrm[j][2] + lamr[j][1] * t1[2] + lamr[j][2] * t2[2]) * g;
        } else {
          f0 += lamr[j][1] * inv_h;
          f1 += lamr[j][2] * inv_h;
          f2 += lamr[j][0] * inv_h;
        }
      }
      if constexpr (T::NPK > 0) {
        for (int p = 0; p < npc; ++p) {
          const float* o = pool + RS::PER_POOL * p * RW;
          const float sg = ((int)o[kPoolBA * RW] == 0 ? inv_h : 0.f) - ((int)o[kPoolBB * RW] == 0 ? inv_h : 0.f);
          if (sg != 0.f) {
            const float l0 = o[kPoolLam * RW], l1 = o[(kPoolLam + 1) * RW], l2 = o[(kPoolLam + 2) * RW];
            f0 += sg * (l0 * o[kPoolN * RW] + l1 * o[kPoolT1 * RW] + l2 * o[kPoolT2 * RW]);
            f1 += sg * (l0 * o[(kPoolN + 1) * RW] + l1 * o[(kPoolT1 + 1) * RW] + l2 * o[(kPoolT2 + 1) * RW]);
            f2 += sg * (l0 * o[(kPoolN + 2) * RW] + l1 * o[(kPoolT1 + 2) * RW] + l2 * o[(kPoolT2 + 2) * RW]);
          }
        }
      }
      cf_soa[0 * N + e] = f0;
      cf_soa[1 * N + e] = f1;
      cf_soa[2 * N + e] = f2;
      if (cf_aos) {
        float* o = cf_aos + (size_t)e * T::NB * 3;
        o[0] = f0; o[1] = f1; o[2] = f2;
      }
    }
  }
  GS_PROF(5)  // back-substitution + integrate + contact forces
}

template <class T>
__device__ __forceinline__ void team_com_velocity(const DevModel* __restrict__ M, const TeamState<T>& s, float* v) {
  float R[9], c[3], wc[3];
  quat_to_mat(s.quat, R);
  mat3vec(R, M->root_com, c);
  cross3(s.w, c, wc);
  v[0] = s.vo[0] + wc[0]; v[1] = s.vo[1] + wc[1]; v[2] = s.vo[2] + wc[2];
}

// XCD-aware workgroup -> env-block mapping.  The dispatcher hands workgroup b to XCD b % 8, and each XCD has
// its own L2: with the identity mapping the two 64-B halves of every 128-B line of a SoA state row (16 envs x
// 4 B per wave) were read by workgroups on two different XCDs, each fetching the line from HBM (2.2x the
// algorithmic read bytes, profiles/pmc_pd_step.json r03).  Here the workgroups an XCD runs take consecutive env
// blocks (a bijection on [0, G) for any G), so neighbouring halves meet in one L2.
__device__ __forceinline__ int xcd_block(int b, int G) {
  constexpr int kXcd = 8;
  const int per = G / kXcd, rem = G % kXcd, x = b % kXcd, q = b / kXcd;
  return x * per + (x < rem ? x : rem) + q;
}

template <class T, bool TERR, bool TGS>
__global__ __launch_bounds__(kTeamBlock, 1) void k_simulate_team(const DevModel* __restrict__ M, DevParams P,
                                                                 SimBuffers B, const float* __restrict__ tau_aos) {
  constexpr int LN = T::T_LANES, CL = T::T_CL, ND = T::ND;
  __shared__ float mdl[CM<T>::NP * LN];
  __shared__ float rows[RowSlots<T>::TOTAL * RW];
  __shared__ float shw_tab[shw_size<T>()];
  __shared__ float sct[ShapeTab<T>::SIZE];
  // the team's shape friction (constant over the launch), read by the contact records and the self-contact pool
  // from LDS instead of device memory every substep: [shape][team]
  __shared__ float mu_tab[T::NS * kTeamsPerBlock];
  __shared__ float stash_tab[team_stash_size<T>() * kTeamBlock];
  stage_chain_model<T>(M, mdl);
  stage_shape_consts<T>(M, sct);
  const int lc = threadIdx.x & (LN - 1);
  const int e = (xcd_block(blockIdx.x, gridDim.x) * kTeamBlock + threadIdx.x) / LN;
  for (int sh = lc; sh < T::NS; sh += LN)
    mu_tab[sh * kTeamsPerBlock + (threadIdx.x >> 2)] = e < B.N ? B.mu[(size_t)sh * B.N + e] : 1.f;
  __syncthreads();
  if (e >= B.N) return;
  const float* mu_t = mu_tab + (threadIdx.x >> 2);
  const int N = B.N;
  TeamState<T> s;
  team_load<T>(B.state, N, e, lc, s);
  float tau[CL];
#pragma unroll
  for (int k = 0; k < CL; ++k) tau[k] = tau_aos ? tau_aos[(size_t)e * ND + lc * CL + k] : 0.f;
  float* own = rows + threadIdx.x;
  const float* team = rows + (threadIdx.x & ~(LN - 1));
  GS_PROF_DECL
  for (int sstep = 0; sstep < P.substeps; ++sstep) {
    const bool last = (sstep == P.substeps - 1) && P.collect;
    substep_team<T, TERR, TGS>(M, mdl, P, s, tau, mu_t, N, e, lc, own, team, B.cf, last, nullptr, shw_tab, sct, stash_tab + threadIdx.x GS_PROF_ARGS);
  }
  team_store<T>(B.state, N, opaque_index(e), opaque_index(lc), s);
  GS_PROF_FLUSH
}

template <class T, bool TERR, bool TGS>
__global__ __launch_bounds__(kTeamBlock, 1) void k_pd_step_team(const DevModel* __restrict__ M, DevParams P,
                                                                SimBuffers B, PdDev A) {
  constexpr int LN = T::T_LANES, CL = T::T_CL, ND = T::ND, NB = T::NB;
  __shared__ float mdl[CM<T>::NP * LN];
  __shared__ float rows[RowSlots<T>::TOTAL * RW];
  __shared__ float shw_tab[shw_size<T>()];
  __shared__ float sct[ShapeTab<T>::SIZE];
  // the team's shape friction (constant over the launch), read by the contact records and the self-contact pool
  // from LDS instead of device memory every substep: [shape][team]
  __shared__ float mu_tab[T::NS * kTeamsPerBlock];
  __shared__ float stash_tab[team_stash_size<T>() * kTeamBlock];
  stage_chain_model<T>(M, mdl);
  stage_shape_consts<T>(M, sct);
  const int lc = threadIdx.x & (LN - 1);
  const int e = (xcd_block(blockIdx.x, gridDim.x) * kTeamBlock + threadIdx.x) / LN;
  for (int sh = lc; sh < T::NS; sh += LN)
    mu_tab[sh * kTeamsPerBlock + (threadIdx.x >> 2)] = e < B.N ? B.mu[(size_t)sh * B.N + e] : 1.f;
  __syncthreads();
  if (e >= B.N) return;
  const float* mu_t = mu_tab + (threadIdx.x >> 2);
  const int N = B.N;
  TeamState<T> s;
  team_load<T>(B.state, N, e, lc, s);
  float tau[CL];
  float* own = rows + threadIdx.x;
  const float* team = rows + (threadIdx.x & ~(LN - 1));
  const int sub = P.substeps;
  const int n_pd = A.decimation * sub;
  const int total = (A.decimation + A.extra) * sub;
  // this lane's first dof in the AoS tensors (formed where each use needs it, opaque_index)
  auto dof0 = [&]() { return (size_t)opaque_index(e) * ND + lc * CL; };
  GS_PROF_DECL
  for (int it = 0; it < total; ++it) {
    if (it < n_pd && (it % sub) == 0) {
      const bool first = it == 0;
      const size_t d0 = dof0();
#pragma unroll
      for (int k = 0; k < CL; ++k) {
        const float qj = first ? A.dof_state_in[(d0 + k) * 2 + 0] : s.q[k];
        const float qdj = first ? A.dof_state_in[(d0 + k) * 2 + 1] : s.qd[k];
        const float aj = A.actions[d0 + k];
        tau[k] = clampf(A.kp * (A.scale * aj + A.default_pos[lc * CL + k] - qj) - A.kd * qdj, -A.tlim, A.tlim);
      }
    }
    const bool last = ((it % sub) == sub - 1) && P.collect;
    GS_PROF(6)  // PD torque
    float* cf_aos = (it == total - 1) ? A.cf_out : nullptr;
    substep_team<T, TERR, TGS>(M, mdl, P, s, tau, mu_t, N, e, lc, own, team, B.cf, last, cf_aos, shw_tab, sct, stash_tab + threadIdx.x GS_PROF_ARGS);
    if (it == n_pd - 1 && A.dof_out) {
      const size_t d0 = dof0();
#pragma unroll
      for (int k = 0; k < CL; ++k) {
        A.dof_out[(d0 + k) * 2 + 0] = s.q[k];
        A.dof_out[(d0 + k) * 2 + 1] = s.qd[k];
      }
    }
  }
  team_store<T>(B.state, N, opaque_index(e), opaque_index(lc), s);
  const size_t d0 = dof0();
#pragma unroll
  for (int k = 0; k < CL; ++k) A.torques_out[d0 + k] = tau[k];
  if (A.actions_copy) {
#pragma unroll
    for (int k = 0; k < CL; ++k) A.actions_copy[d0 + k] = A.actions[d0 + k];
  }
  if (A.root_out && lc == 0) {
    float* o = A.root_out + (size_t)e * 13;
    o[0] = s.p[0]; o[1] = s.p[1]; o[2] = s.p[2];
    o[3] = s.quat[0]; o[4] = s.quat[1]; o[5] = s.quat[2]; o[6] = s.quat[3];
    float v[3];
    team_com_velocity<T>(M, s, v);
    o[7] = v[0]; o[8] = v[1]; o[9] = v[2];
    o[10] = s.w[0]; o[11] = s.w[1]; o[12] = s.w[2];
  }
  if constexpr (!TERR) if (kTeamsPerBlock == 16 && A.tail_on) {  // (plane kernels only: the TERR form is at its
                                                                    // register limit, the tail cost it 12 B scratch)
    // The AnymalTerrain tail (gymsim.h gs_pd_args.tail_*; gt_anymal_tail.h, the source of libgymtask's k_post_a)
    // on the outputs this wave has just stored (root, contacts, dofs, torques, the actions copy): lane 0 of each
    // team runs its env, so the separate post_a launch and its wait behind this kernel go away.  The wave's 16
    // done bits are its 16-bit slice of the 64-env reset-mask word k_reset_flagged ranks; the wave that completes
    // the grid publishes the count.
    __syncthreads();  // (one wave per workgroup) this wave's global stores are visible to its own loads
    const bool reset = lc == 0 && (ND == 12 ? gt_tail::post_a_env<true, false, (ND == 12 ? 12 : 0)>(
                                                  A.tail_p, A.tail_b, gt_anymal_hound{}, e)
                                            : gt_tail::post_a_env<true, false>(A.tail_p, A.tail_b, gt_anymal_hound{}, e));
    const unsigned long long m = __ballot(reset);
    unsigned m16 = 0;
#pragma unroll
    for (int i = 0; i < kTeamsPerBlock; ++i) m16 |= (unsigned)((m >> (LN * i)) & 1ull) << i;
    const int e0 = e - (int)(threadIdx.x / LN);  // the wave's first env (16-aligned)
    const unsigned long long live = __ballot(true);
    if ((int)(threadIdx.x & 63) == __ffsll((long long)live) - 1) {
      uint16_t* slices = reinterpret_cast<uint16_t*>(A.tail_b.reset_masks);
      slices[e0 / kTeamsPerBlock] = (uint16_t)m16;
      // the last wave also clears the slices of its mask word past the last env
      if (e0 + kTeamsPerBlock >= N)
        for (int q = e0 / kTeamsPerBlock + 1; q % 4 != 0; ++q) slices[q] = 0;
      gt_tail::publish_count(A.tail_b, (unsigned)__popc(m16), gridDim.x);
    }
  }
  GS_PROF(7)  // outputs
  GS_PROF_FLUSH
}

}  // namespace

// the fused tail writes 16-env slices of the reset-mask words (one wave of 16 teams per workgroup)
bool team_fused_tail_available() { return kTeamsPerBlock == 16; }

template <class T>
hipError_t launch_sim_team(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau,
                           hipStream_t st) {
  if constexpr (T::HAS_TEAM) {
    static_assert(T::NR == T::NB, "the lane team reports contact forces per body (no kept fixed-joint links)");
    const long lanes = (long)B.N * T::T_LANES;
    const int blocks = (int)((lanes + kTeamBlock - 1) / kTeamBlock);
    // trimesh terrain: mesh queries by the candidates' owner lanes; TGS / PGS
    if (P.has_terrain && P.tgs)
      hipLaunchKernelGGL((k_simulate_team<T, true, true>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, tau);
    else if (P.has_terrain)
      hipLaunchKernelGGL((k_simulate_team<T, true, false>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, tau);
    else if (P.tgs)
      hipLaunchKernelGGL((k_simulate_team<T, false, true>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, tau);
    else
      hipLaunchKernelGGL((k_simulate_team<T, false, false>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, tau);
    return hipGetLastError();
  } else {
    return hipErrorInvalidConfiguration;
  }
}
template <class T>
hipError_t launch_pd_team(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  if constexpr (T::HAS_TEAM) {
    const long lanes = (long)B.N * T::T_LANES;
    const int blocks = (int)((lanes + kTeamBlock - 1) / kTeamBlock);
    if (P.has_terrain && P.tgs)
      hipLaunchKernelGGL((k_pd_step_team<T, true, true>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, A);
    else if (P.has_terrain)
      hipLaunchKernelGGL((k_pd_step_team<T, true, false>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, A);
    else if (P.tgs)
      hipLaunchKernelGGL((k_pd_step_team<T, false, true>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, A);
    else
      hipLaunchKernelGGL((k_pd_step_team<T, false, false>), dim3(blocks), dim3(kTeamBlock), 0, st, M, P, B, A);
    return hipGetLastError();
  } else {
    return hipErrorInvalidConfiguration;
  }
}

#define GS_TEAM_ENTRY(T, SIG) {SIG, T::HAS_TEAM ? &launch_sim_team<T> : nullptr, T::HAS_TEAM ? &launch_pd_team<T> : nullptr},
TeamEntry g_team_kernels[] = {GS_FOR_EACH_TOPOLOGY(GS_TEAM_ENTRY)};
const int g_num_team_kernels = sizeof(g_team_kernels) / sizeof(g_team_kernels[0]);

// Phase profile readout (include/gymsim.h); -1 outside the profiling build.
extern "C" int gs_debug_phase_cycles(unsigned long long* out, int n, int reset) {
#ifdef GS_PHASE_PROFILE
  if (!out || n <= 0 || n > 64) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs_phase_cycles), sizeof(unsigned long long) * n) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gs_phase_cycles), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
#else
  (void)out; (void)n; (void)reset;
  return -1;
#endif
}
