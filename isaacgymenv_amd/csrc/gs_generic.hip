// gs_generic.hip -- the runtime-sized articulation solver (kernel_variant 4): any robot whose topology is not
// compiled into libgymsim (tools/gen_topologies.py) still simulates, sized from the model tables at
// gs_sim_set_model instead of a compile-time Topo_* (the fork's own
// assets/urdf/Hound_new/Hound.urdf, loaded by /root/reference/isaacgymenvs/tasks/hound.py:168-183, is the proof).
//
// Same solver specification as the compiled kernels and the oracle: spatial inertias at the
// root origin O, RNEA bias with gravity as base acceleration, CRBA mass matrix in mixed coordinates
// nu = (w, p_dot_origin, q_dot) with the h (w x p_dot) term, plane contact candidates (spheres, capsule / cylinder
// ends, box corners) active within contact_offset, joint-limit rows within limit_margin, joint drives (implicit
// within the effort, clamped beyond it), PGS with split impulse or the position sub-steps of TGS (physx.solver_type
// 1), joint velocity clamp, semi-implicit integration with the position-phase velocity.  What the
// compiled kernels do with compile-time tree tables and register arrays, this one does densely in joint space:
// the mass matrix is factored (Cholesky), each contact row's response W = M^-1 J^T is two triangular solves.
//
// Mapping (MI355X): ONE WAVE PER ENV.  Body recursions (kinematics, RNEA, composite inertias) are serial over the
// tree and run in lane 0 on LDS-resident body tables; everything dense is spread over the 64 lanes -- the mass
// matrix rows (lane = body), the Cholesky columns (lane = row), candidates (lane = candidate, activity compacted
// by a ballot prefix in candidate order), Jacobian rows (lane = column), the row solves (lane = row) and the
// Gauss-Seidel sweeps (lane = velocity component: u = J v is a wave reduction, v += W dl a vector update).  The
// rows J, W live in a per-env workspace in device memory (SimBuffers::rows), the factor and the body tables in
// LDS.  Not supported here (fails loudly at set-up): hull candidates, self-collision, terrain meshes, force
// sensors -- those robots need a compiled topology.
#include <hip/hip_runtime.h>

#include "gs_internal.h"
#include "gs_math.h"

namespace {

constexpr int kGW = 64;         // lanes per env (one wave)
constexpr int kGMaxV = GS_MAXD + 6;

struct GBody {  // LDS body tables of one env
  float R[GS_MAXB][9], P[GS_MAXB][3], S[GS_MAXB][6], V[GS_MAXB][6], A[GS_MAXB][6], F[GS_MAXB][6];
  SpI Ib[GS_MAXB], Ic[GS_MAXB];
};

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kGW);
  return x;
}

__device__ __forceinline__ void axis_rot(const float* a, float q, float* Rq) {
  float s, c;
  sincosf(q, &s, &c);
  const float C = 1.f - c;
  Rq[0] = c + a[0] * a[0] * C;        Rq[1] = a[0] * a[1] * C - a[2] * s; Rq[2] = a[0] * a[2] * C + a[1] * s;
  Rq[3] = a[1] * a[0] * C + a[2] * s; Rq[4] = c + a[1] * a[1] * C;        Rq[5] = a[1] * a[2] * C - a[0] * s;
  Rq[6] = a[2] * a[0] * C - a[1] * s; Rq[7] = a[2] * a[1] * C + a[0] * s; Rq[8] = c + a[2] * a[2] * C;
}

// per-actor dof property f of dof j (GS_DOFP_FIELDS order), else the asset's value
__device__ __forceinline__ float gdofp(const DevParams& P, int nd, int e, int f, int j, float mv) {
  return P.dof_env ? P.dof_env[((size_t)f * nd + j) * P.dof_env_n + e] : mv;
}

// One substep of env e (the whole wave).  st: SoA state; tau: [N][nd] or null; ws: this env's row workspace
// (J then W, row stride nv); cf: [3 nr][N] or null (collect).
__device__ void generic_substep(const DevModel* __restrict__ M, const DevLinks* __restrict__ L,
                                const GenTopo* __restrict__ G, const DevParams& P, float* __restrict__ st,
                                const float* __restrict__ mu, int N, int e, const float* __restrict__ tau_e,
                                float* __restrict__ ws, float* __restrict__ cf, GBody& B, float* Ml, float* rowf,
                                int* rowi, float* vec) {
  const int lane = threadIdx.x & (kGW - 1);
  const int nb = L->nb, nd = L->nd, fb = L->fixed_base;
  const int nbase = fb ? 0 : 6, nv = nbase + nd;
  const float h = P.h;
  const int maxrows = 3 * G->nc + nd;
  float* Jw = ws;                             // [maxrows][nv]
  float* Ww = ws + (size_t)maxrows * nv;      // [maxrows][nv]
  // vec: nu (nv) | nuf (nv) | rhs (nv) | root (13) | q (nd) | qd (nd) | dforce (nd) | dimpl (nd)
  float* nu = vec;
  float* nuf = vec + kGMaxV;
  float* rhs = vec + 2 * kGMaxV;
  float* root = vec + 3 * kGMaxV;
  float* q = root + 13;
  float* qd = q + GS_MAXD;
  float* dforce = qd + GS_MAXD;
  float* dimpl = dforce + GS_MAXD;
  // row tables (rowf: separation, mu, normal xyz, Dr, lam | rowi: kind (0 limit, 1 contact row), candidate / dof)
  float* rsep = rowf;
  float* rmu = rowf + 1 * (3 * GS_MAXC + GS_MAXD);
  float* rD = rowf + 2 * (3 * GS_MAXC + GS_MAXD);
  float* rlam = rowf + 3 * (3 * GS_MAXC + GS_MAXD);
  float* rsg = rowf + 4 * (3 * GS_MAXC + GS_MAXD);  // limit rows: +1 lower, -1 upper

  // ---------------- state in
  if (lane < 13) root[lane] = st[(size_t)lane * N + e];
  for (int j = lane; j < nd; j += kGW) {
    q[j] = st[(size_t)(13 + j) * N + e];
    qd[j] = st[(size_t)(13 + nd + j) * N + e];
  }
  __syncthreads();

  // ---------------- lane 0: kinematics, velocities, RNEA, composite inertias (serial over the tree)
  if (lane == 0) {
    const float qn = 1.f / sqrtf(root[3] * root[3] + root[4] * root[4] + root[5] * root[5] + root[6] * root[6]);
    const float q4[4] = {root[3] * qn, root[4] * qn, root[5] * qn, root[6] * qn};
    quat_to_mat(q4, B.R[0]);
    B.P[0][0] = B.P[0][1] = B.P[0][2] = 0.f;
    for (int k = 0; k < 6; ++k) { B.S[0][k] = 0.f; B.V[0][k] = 0.f; }
    if (!fb) {
      B.V[0][0] = root[10]; B.V[0][1] = root[11]; B.V[0][2] = root[12];
      B.V[0][3] = root[7]; B.V[0][4] = root[8]; B.V[0][5] = root[9];
    }
    B.A[0][0] = B.A[0][1] = B.A[0][2] = 0.f;
    B.A[0][3] = -P.g[0]; B.A[0][4] = -P.g[1]; B.A[0][5] = -P.g[2];
    for (int i = 1; i < nb; ++i) {
      const int pa = L->parent[i];
      float RJ[9], t[3], aw[3];
      mat3mul(B.R[pa], M->jR[i], RJ);
      mat3vec(B.R[pa], M->jt[i], t);
      for (int k = 0; k < 3; ++k) B.P[i][k] = B.P[pa][k] + t[k];
      mat3vec(RJ, M->jaxis[i], aw);
      const int d = L->bdof[i];
      const float qj = q[d];
      if (L->jkind[i] == 1) {
        float Rq[9];
        axis_rot(M->jaxis[i], qj, Rq);
        mat3mul(RJ, Rq, B.R[i]);
        B.S[i][0] = aw[0]; B.S[i][1] = aw[1]; B.S[i][2] = aw[2];
        cross3(B.P[i], aw, &B.S[i][3]);
      } else {
        for (int k = 0; k < 9; ++k) B.R[i][k] = RJ[k];
        for (int k = 0; k < 3; ++k) B.P[i][k] += aw[k] * qj;
        B.S[i][0] = B.S[i][1] = B.S[i][2] = 0.f;
        B.S[i][3] = aw[0]; B.S[i][4] = aw[1]; B.S[i][5] = aw[2];
      }
      const float w = qd[d];
      float c6[6];
      for (int k = 0; k < 6; ++k) B.V[i][k] = B.V[pa][k] + B.S[i][k] * w;
      crm(B.V[i], B.S[i], c6);
      for (int k = 0; k < 6; ++k) B.A[i][k] = B.A[pa][k] + c6[k] * w;
    }
    for (int i = 0; i < nb; ++i) {
      // spatial inertia at O: m, h = m c, I_O = R I_c R^T + m ([c]^T [c])
      float c[3], Am[9];
      mat3vec(B.R[i], M->com[i], c);
      for (int k = 0; k < 3; ++k) c[k] += B.P[i][k];
      const float* Il = M->inertia[i];  // xx yy zz xy xz yz
      const float* R = B.R[i];
      for (int r = 0; r < 3; ++r) {
        Am[3 * r + 0] = R[3 * r] * Il[0] + R[3 * r + 1] * Il[3] + R[3 * r + 2] * Il[4];
        Am[3 * r + 1] = R[3 * r] * Il[3] + R[3 * r + 1] * Il[1] + R[3 * r + 2] * Il[5];
        Am[3 * r + 2] = R[3 * r] * Il[4] + R[3 * r + 1] * Il[5] + R[3 * r + 2] * Il[2];
      }
      const float m = M->mass[i], cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
      SpI& I = B.Ib[i];
      I.m = m;
      I.h[0] = m * c[0]; I.h[1] = m * c[1]; I.h[2] = m * c[2];
      I.I[0] = Am[0] * R[0] + Am[1] * R[1] + Am[2] * R[2] + m * (cc - c[0] * c[0]);
      I.I[1] = Am[3] * R[3] + Am[4] * R[4] + Am[5] * R[5] + m * (cc - c[1] * c[1]);
      I.I[2] = Am[6] * R[6] + Am[7] * R[7] + Am[8] * R[8] + m * (cc - c[2] * c[2]);
      I.I[3] = Am[0] * R[3] + Am[1] * R[4] + Am[2] * R[5] - m * c[0] * c[1];
      I.I[4] = Am[0] * R[6] + Am[1] * R[7] + Am[2] * R[8] - m * c[0] * c[2];
      I.I[5] = Am[3] * R[6] + Am[4] * R[7] + Am[5] * R[8] - m * c[1] * c[2];
      B.Ic[i] = I;
      float ia[6], iv[6], x6[6];
      spi_mul(I, B.A[i], ia);
      spi_mul(I, B.V[i], iv);
      crf(B.V[i], iv, x6);
      for (int k = 0; k < 6; ++k) B.F[i][k] = ia[k] + x6[k];
    }
    for (int i = nb - 1; i > 0; --i) {
      const int pa = L->parent[i];
      SpI& a = B.Ic[pa];
      const SpI& b = B.Ic[i];
      a.m += b.m;
      for (int k = 0; k < 3; ++k) a.h[k] += b.h[k];
      for (int k = 0; k < 6; ++k) a.I[k] += b.I[k];
      for (int k = 0; k < 6; ++k) B.F[pa][k] += B.F[i][k];
    }
    // generalized velocity and the bias c(q, nu)
    if (!fb) {
      for (int k = 0; k < 3; ++k) { nu[k] = root[10 + k]; nu[3 + k] = root[7 + k]; }
      for (int k = 0; k < 6; ++k) rhs[k] = -B.F[0][k];
    }
    for (int j = 0; j < nd; ++j) nu[nbase + j] = qd[j];
  }
  __syncthreads();

  // ---------------- drives and generalized forces (lane = dof)
  for (int j = lane; j < nd; j += kGW) {
    const int i = L->dbody[j];
    const float bias = dot6(B.S[i], B.F[i]);
    const float ef = gdofp(P, nd, e, 2, j, M->effort[j]);
    float t = tau_e ? tau_e[j] : 0.f;
    if (ef > 0.f) t = clampf(t, -ef, ef);
    float r = t - bias;
    float df = 0.f, imp = 0.f;
    if (P.any_drive) {
      const float pt = P.ptgt ? P.ptgt[(size_t)e * nd + j] : 0.f;
      const float vt = P.vtgt ? P.vtgt[(size_t)e * nd + j] : 0.f;
      const float f = gdofp(P, nd, e, 0, j, M->dkp[j]) * (pt - q[j] - h * qd[j]) + gdofp(P, nd, e, 1, j, M->dkd[j]) * (vt - qd[j]);
      const bool im = !(ef > 0.f) || fabsf(f) <= ef;
      df = im ? f : clampf(f, -ef, ef);
      imp = im ? 1.f : 0.f;
      r += df;
    }
    rhs[nbase + j] = r;
    dforce[j] = df;
    dimpl[j] = imp;
  }
  // ---------------- CRBA (lane = body): row of body i's dof, and its base block (entries of dofs on no common
  // path stay zero)
  for (int t = lane; t < nv * kGMaxV; t += kGW) Ml[t] = 0.f;
  __syncthreads();
  for (int i = lane; i < nb; i += kGW) {
    if (i == 0) {
      if (!fb) {
        const SpI& I0 = B.Ic[0];
        const float* hh = I0.h;
        const float hx[9] = {0.f, -hh[2], hh[1], hh[2], 0.f, -hh[0], -hh[1], hh[0], 0.f};
        const float Iv[9] = {I0.I[0], I0.I[3], I0.I[4], I0.I[3], I0.I[1], I0.I[5], I0.I[4], I0.I[5], I0.I[2]};
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b) {
            Ml[a * kGMaxV + b] = Iv[3 * a + b];
            Ml[(3 + a) * kGMaxV + 3 + b] = a == b ? I0.m : 0.f;
            Ml[a * kGMaxV + 3 + b] = hx[3 * a + b];
            Ml[(3 + b) * kGMaxV + a] = hx[3 * a + b];
          }
      }
      continue;
    }
    const int d = L->bdof[i], di = nbase + d;
    float Fi[6];
    spi_mul(B.Ic[i], B.S[i], Fi);
    float dd = dot6(B.S[i], Fi) + M->armature[d];
    if (P.any_drive && dimpl[d] != 0.f)
      dd += h * (gdofp(P, nd, e, 1, d, M->dkd[d]) + h * gdofp(P, nd, e, 0, d, M->dkp[d]));
    Ml[di * kGMaxV + di] = dd;
    for (int jb = L->parent[i]; jb > 0; jb = L->parent[jb]) {
      const int dj = nbase + L->bdof[jb];
      const float v = dot6(B.S[jb], Fi);
      Ml[di * kGMaxV + dj] = v;
      Ml[dj * kGMaxV + di] = v;
    }
    if (!fb)
      for (int k = 0; k < 6; ++k) { Ml[di * kGMaxV + k] = Fi[k]; Ml[k * kGMaxV + di] = Fi[k]; }
  }
  __syncthreads();
  // ---------------- Cholesky M = L L^T (lower, in place), column by column, lane = row
  for (int j = 0; j < nv; ++j) {
    float d = Ml[j * kGMaxV + j];
    for (int k = 0; k < j; ++k) d -= Ml[j * kGMaxV + k] * Ml[j * kGMaxV + k];
    d = sqrtf(d > 0.f ? d : 1e-30f);
    for (int i = j + 1 + lane; i < nv; i += kGW) {
      float t = Ml[i * kGMaxV + j];
      for (int k = 0; k < j; ++k) t -= Ml[i * kGMaxV + k] * Ml[j * kGMaxV + k];
      Ml[i * kGMaxV + j] = t / d;
    }
    __syncthreads();
    if (lane == 0) Ml[j * kGMaxV + j] = d;
    __syncthreads();
  }
  auto chol_solve = [&](const float* b, float* x, int stride) {  // x = M^-1 b (one lane, vectors at stride)
    float y[kGMaxV];
    for (int i = 0; i < nv; ++i) {
      float t = b[i * stride];
      for (int k = 0; k < i; ++k) t -= Ml[i * kGMaxV + k] * y[k];
      y[i] = t / Ml[i * kGMaxV + i];
    }
    for (int i = nv - 1; i >= 0; --i) {
      float t = y[i];
      for (int k = i + 1; k < nv; ++k) t -= Ml[k * kGMaxV + i] * x[k * stride];
      x[i * stride] = t / Ml[i * kGMaxV + i];
    }
  };
  // ---------------- free velocity (lane 0)
  if (lane == 0) {
    float acc[kGMaxV];
    chol_solve(rhs, acc, 1);
    for (int k = 0; k < nv; ++k) nuf[k] = nu[k] + h * acc[k];
    if (!fb) {
      float wxp[3];
      cross3(&nu[0], &nu[3], wxp);
      for (int k = 0; k < 3; ++k) nuf[3 + k] += h * wxp[k];
    }
  }
  __syncthreads();

  // ---------------- rows: joint limits (dof order), then plane contacts (candidate order), 3 rows each
  int nlim = 0;
  {
    bool on = false;
    float sg = 0.f, sep = 0.f;
    if (lane < nd && P.any_limits) {
      const float lo = gdofp(P, nd, e, 3, lane, M->lower[lane]), hi = gdofp(P, nd, e, 4, lane, M->upper[lane]);
      const bool lim = P.dof_env ? lo < hi : M->has_lim[lane] != 0;
      if (lim) {
        const float dl = q[lane] - lo, dh = hi - q[lane];
        on = dl < P.limit_margin || dh < P.limit_margin;
        sg = dl <= dh ? 1.f : -1.f;
        sep = dl <= dh ? dl : dh;
      }
    }
    const unsigned long long bal = __ballot(on);
    const int slot = __popcll(bal & ((1ull << lane) - 1ull));
    if (on) {
      rowi[2 * slot] = 0;
      rowi[2 * slot + 1] = lane;
      rsep[slot] = sep;
      rsg[slot] = sg;
    }
    nlim = __popcll(bal);
  }
  int nrows = nlim;
  for (int c0 = 0; c0 < G->nc; c0 += kGW) {
    const int c = c0 + lane;
    bool act = false;
    float dist = 0.f;
    if (c < G->nc && P.has_ground) {
      const int b = G->cbody[c];
      float x[3];
      mat3vec(B.R[b], M->cpoint[c], x);
      dist = root[2] + B.P[b][2] + x[2] - M->cradius[c];
      act = dist < P.contact_offset;
    }
    const unsigned long long bal = __ballot(act);
    const int slot = nrows + 3 * __popcll(bal & ((1ull << lane) - 1ull));
    if (act) {
      const float m = 0.5f * (mu[(size_t)G->cshape[c] * N + e] + P.ground_mu);
      for (int rr = 0; rr < 3; ++rr) {
        rowi[2 * (slot + rr)] = 1 + rr;
        rowi[2 * (slot + rr) + 1] = c;
        rsep[slot + rr] = dist - P.rest_offset;
        rmu[slot + rr] = m;
      }
    }
    nrows += 3 * __popcll(bal);
  }
  __syncthreads();
  // Jacobian rows (lane = column k): a limit row is +-e_dof; a contact row's direction d (normal z, tangents x, y
  // for the plane) times the velocity of the contact point xc = x - r n over the candidate body's path
  for (int r = 0; r < nrows; ++r) {
    const int kind = rowi[2 * r], id = rowi[2 * r + 1];
    float* Jr = Jw + (size_t)r * nv;
    for (int k = lane; k < nv; k += kGW) {
      float v = 0.f;
      if (kind == 0) {
        v = k == nbase + id ? rsg[r] : 0.f;
      } else {
        const int b = G->cbody[id];
        float x[3];
        mat3vec(B.R[b], M->cpoint[id], x);
        const float xc[3] = {B.P[b][0] + x[0], B.P[b][1] + x[1], B.P[b][2] + x[2] - M->cradius[id]};
        const int ax = kind == 1 ? 2 : (kind == 2 ? 0 : 1);  // normal z, tangent 1 x, tangent 2 y
        if (k < nbase) {
          if (k < 3) {  // d . (w x xc) = w . (xc x d): column k of xc x e_ax
            const float ea[3] = {ax == 0 ? 1.f : 0.f, ax == 1 ? 1.f : 0.f, ax == 2 ? 1.f : 0.f};
            float t[3];
            cross3(xc, ea, t);
            v = t[k];
          } else {
            v = (k - 3) == ax ? 1.f : 0.f;
          }
        } else {
          const int i = L->dbody[k - nbase];
          if ((L->anc_mask[b] >> i) & 1u) {
            float t[3];
            cross3(B.S[i], xc, t);
            v = B.S[i][3 + ax] + t[ax];
          }
        }
      }
      Jr[k] = v;
    }
  }
  __syncthreads();
  // responses W = M^-1 J^T and the Delassus diagonals (lane = row)
  for (int r = lane; r < nrows; r += kGW) {
    const float* Jr = Jw + (size_t)r * nv;
    float* Wr = Ww + (size_t)r * nv;
    chol_solve(Jr, Wr, 1);
    float d = 0.f;
    for (int k = 0; k < nv; ++k) d += Jr[k] * Wr[k];
    rD[r] = d;
    rlam[r] = 0.f;
  }
  __syncthreads();

  // ---------------- projected Gauss-Seidel / TGS sub-steps (lane = velocity component)
  float v = lane < nv ? nuf[lane] : 0.f;
  float dxs = 0.f, vpos = v;
  const bool tgs = P.tgs != 0;
  const float hs = tgs ? h / (float)P.pos_iters : h;
  const int iters = P.pos_iters + P.vel_iters;
  for (int it = 0; it < iters; ++it) {
    const bool pos = it < P.pos_iters;
    const float hd = pos ? hs : h;
    for (int r = 0; r < nrows; ++r) {
      const int kind = rowi[2 * r];
      const float* Jr = Jw + (size_t)r * nv;
      const float* Wr = Ww + (size_t)r * nv;
      const float jk = lane < nv ? Jr[lane] : 0.f;
      const float u = wave_sum(jk * v);
      float ln;
      if (kind <= 1) {  // limit or contact normal: unilateral, separation target
        float s = rsep[r];
        if (tgs) s += wave_sum(jk * dxs);
        float target;
        if (s >= 0.f) target = -s / hd;
        else if (pos) target = fminf(-s / h, P.max_depen_vel);  // (TGS: the push-out spread over the step)
        else target = 0.f;
        ln = rD[r] > 0.f ? rlam[r] + (target - u) / rD[r] : rlam[r];
        ln = fmaxf(ln, 0.f);
      } else {  // friction: |lambda_t| <= mu lambda_n of the contact's normal row (two rows above or one)
        const int nr0 = r - (kind - 1);
        const float lim = rmu[r] * rlam[nr0];
        ln = rD[r] > 0.f ? rlam[r] - u / rD[r] : rlam[r];
        ln = clampf(ln, -lim, lim);
      }
      const float dl = ln - rlam[r];
      rlam[r] = ln;  // (every lane the same value: a one-wave workgroup reads and writes LDS in program order)
      if (lane < nv) v += Wr[lane] * dl;
    }
    if (tgs && pos) dxs += hs * v;
    if (it == P.pos_iters - 1) vpos = tgs ? dxs / h : v;
  }
  if (P.pos_iters <= 0) vpos = v;
  // joint velocity clamp
  if (lane >= nbase && lane < nv) {
    const int j = lane - nbase;
    const float vm = gdofp(P, nd, e, 5, j, M->vmax[j]);
    if (vm > 0.f) { v = clampf(v, -vm, vm); vpos = clampf(vpos, -vm, vm); }
  }
  // ---------------- integrate and store
  if (lane < nv) { nu[lane] = v; nuf[lane] = vpos; }  // (nu: new velocity, nuf: position-phase velocity)
  __syncthreads();
  if (lane == 0) {
    if (!fb) {
      for (int k = 0; k < 3; ++k) root[k] += h * nuf[3 + k];
      const float wx = nuf[0], wy = nuf[1], wz = nuf[2];
      float x = root[3], y = root[4], z = root[5], w = root[6];
      const float hh = 0.5f * h;
      const float dx = hh * (w * wx + wy * z - wz * y), dy = hh * (w * wy + wz * x - wx * z);
      const float dz = hh * (w * wz + wx * y - wy * x), dw = -hh * (wx * x + wy * y + wz * z);
      x += dx; y += dy; z += dz; w += dw;
      const float n = 1.f / sqrtf(x * x + y * y + z * z + w * w);
      root[3] = x * n; root[4] = y * n; root[5] = z * n; root[6] = w * n;
      for (int k = 0; k < 3; ++k) { root[10 + k] = nu[k]; root[7 + k] = nu[3 + k]; }
    }
    for (int j = 0; j < nd; ++j) {
      q[j] += h * nuf[nbase + j];
      qd[j] = nu[nbase + j];
    }
  }
  __syncthreads();
  if (lane < 13) st[(size_t)lane * N + e] = root[lane];
  for (int j = lane; j < nd; j += kGW) {
    st[(size_t)(13 + j) * N + e] = q[j];
    st[(size_t)(13 + nd + j) * N + e] = qd[j];
  }
  // net contact force per reported link, sum of lambda / h over the contact's rows in its frame (plane: z, x, y)
  if (cf) {
    for (int l = lane; l < L->nr; l += kGW) {
      float f[3] = {0.f, 0.f, 0.f};
      for (int r = nlim; r < nrows; r += 3) {
        if (G->clink[rowi[2 * r + 1]] != l) continue;
        f[0] += rlam[r + 1] / h;
        f[1] += rlam[r + 2] / h;
        f[2] += rlam[r] / h;
      }
      for (int k = 0; k < 3; ++k) cf[(size_t)(3 * l + k) * N + e] = f[k];
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kGW) void k_simulate_generic(const DevModel* __restrict__ M, DevParams P, SimBuffers Bf,
                                                          const float* __restrict__ tau) {
  __shared__ GBody B;
  __shared__ float Ml[kGMaxV * kGMaxV];
  __shared__ float rowf[5 * (3 * GS_MAXC + GS_MAXD)];
  __shared__ int rowi[2 * (3 * GS_MAXC + GS_MAXD)];
  __shared__ float vec[3 * kGMaxV + 13 + 4 * GS_MAXD];
  const int e = blockIdx.x;
  if (e >= Bf.N) return;
  const DevLinks* L = P.gen_links;
  const GenTopo* G = P.gen;
  const int nv = (L->fixed_base ? 0 : 6) + L->nd;
  const size_t ws_per_env = (size_t)2 * (3 * G->nc + L->nd) * nv;
  float* ws = Bf.rows + ws_per_env * e;
  for (int s = 0; s < P.substeps; ++s) {
    const bool last = s == P.substeps - 1;
    generic_substep(M, L, G, P, Bf.state, Bf.mu, Bf.N, e, tau ? tau + (size_t)e * L->nd : nullptr, ws,
                    (last && P.collect) ? Bf.cf : nullptr, B, Ml, rowf, rowi, vec);
  }
}

__global__ void k_generic_pd_torque(const DevParams P, SimBuffers Bf, PdDev A, int nd, int first, float* tau) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= Bf.N * nd) return;
  const int e = t / nd, j = t - e * nd;
  const float q = first ? A.dof_state_in[(size_t)t * 2] : Bf.state[(size_t)(13 + j) * Bf.N + e];
  const float qd = first ? A.dof_state_in[(size_t)t * 2 + 1] : Bf.state[(size_t)(13 + nd + j) * Bf.N + e];
  const float a = A.actions[t];
  tau[t] = clampf(A.kp * (A.scale * a + A.default_pos[j] - q) - A.kd * qd, -A.tlim, A.tlim);
  (void)P;
}

}  // namespace

hipError_t launch_sim_generic(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau,
                              hipStream_t st) {
  if (!P.gen || !P.gen_links || !B.rows) return hipErrorInvalidValue;
  if (P.has_terrain || P.self_collide) return hipErrorNotSupported;
  if (B.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_simulate_generic, dim3(B.N), dim3(kGW), 0, st, M, P, B, tau);
  return hipGetLastError();
}

// The fused PD decimation step on the generic kernel: per decimation step one PD-torque launch (into
// torques_out) and one simulate launch, then the extra simulates with the last torques, and the dof / root /
// contact tensors by the refresh kernels (the compiled kernels' PdDev contract, gs_internal.h).
hipError_t launch_pd_generic(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A,
                             hipStream_t st) {
  if (!P.gen || !P.gen_links) return hipErrorInvalidValue;
  const int nd = P.gen_nd;
  const int n = B.N * nd, blocks = (n + 255) / 256;
  for (int d = 0; d < A.decimation; ++d) {
    if (n > 0)
      hipLaunchKernelGGL(k_generic_pd_torque, dim3(blocks), dim3(256), 0, st, P, B, A, nd, d == 0 ? 1 : 0,
                         A.torques_out);
    if (hipError_t e = launch_sim_generic(M, P, B, A.torques_out, st); e != hipSuccess) return e;
  }
  if (A.dof_out)
    if (hipError_t e = launch_refresh_dof(B.state, B.N, nd, A.dof_out, st); e != hipSuccess) return e;
  for (int x = 0; x < A.extra; ++x)
    if (hipError_t e = launch_sim_generic(M, P, B, A.torques_out, st); e != hipSuccess) return e;
  if (A.root_out)
    if (hipError_t e = launch_refresh_root(B.state, B.N, nd, &M->root_com[0], A.root_out, st); e != hipSuccess) return e;
  if (A.cf_out)
    if (hipError_t e = launch_refresh_contact(B.cf, B.N, P.gen_nr, A.cf_out, st); e != hipSuccess) return e;
  if (A.actions_copy && n > 0)
    if (hipError_t e = hipMemcpyAsync(A.actions_copy, A.actions, sizeof(float) * n, hipMemcpyDeviceToDevice, st);
        e != hipSuccess)
      return e;
  return hipGetLastError();
}
