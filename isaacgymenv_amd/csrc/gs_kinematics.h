// gs_kinematics.h -- link kinematics of one env (rigid-body state, Jacobians, mass matrix), shared by
// the HIP kernel (gs_kinematics.hip: lane 0 runs the forward pass into LDS, 64 lanes write the outputs)
// and the host backend (gs_host.hip: one thread per env, stride 1).  Conventions: gs_kinematics.hip.
#pragma once
#include "gs_internal.h"
#include "gs_math.h"

namespace {

struct EnvKin {
  float R[GS_MAXB][9];   // body rotation (world)
  float p[GS_MAXB][3];   // body origin (world)
  float c[GS_MAXB][3];   // body COM (world)
  float a[GS_MAXB][3];   // joint axis of the body's dof (world)
  float o[GS_MAXB][3];   // joint point (world)
  float cr[3];           // root LINK COM (world): the point the base columns refer to
  float nu[6 + GS_MAXD]; // generalized velocity
};

GS_HD void axis_angle(const float* ax, float th, float* R) {
  float s, c;
  gs_fast_sincos(th, &s, &c);
  const float t = 1.f - c, x = ax[0], y = ax[1], z = ax[2];
  R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
  R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
  R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}

// rotation matrix -> quaternion xyzw (Shepperd; same branch order as _assets.mat_to_quat_xyzw), w >= 0
GS_HD void mat_to_quat(const float* m, float* q) {
  const float tr = m[0] + m[4] + m[8];
  float x, y, z, w;
  if (tr > 0.f) {
    const float s = sqrtf(tr + 1.f) * 2.f;
    w = 0.25f * s; x = (m[7] - m[5]) / s; y = (m[2] - m[6]) / s; z = (m[3] - m[1]) / s;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    const float s = sqrtf(1.f + m[0] - m[4] - m[8]) * 2.f;
    w = (m[7] - m[5]) / s; x = 0.25f * s; y = (m[1] + m[3]) / s; z = (m[2] + m[6]) / s;
  } else if (m[4] > m[8]) {
    const float s = sqrtf(1.f + m[4] - m[0] - m[8]) * 2.f;
    w = (m[2] - m[6]) / s; x = (m[1] + m[3]) / s; y = 0.25f * s; z = (m[5] + m[7]) / s;
  } else {
    const float s = sqrtf(1.f + m[8] - m[0] - m[4]) * 2.f;
    w = (m[3] - m[1]) / s; x = (m[2] + m[6]) / s; y = (m[5] + m[7]) / s; z = 0.25f * s;
  }
  const float sg = w < 0.f ? -1.f : 1.f, n = sg * gs_rsqrt(x * x + y * y + z * z + w * w);
  q[0] = x * n; q[1] = y * n; q[2] = z * n; q[3] = w * n;
}

// Column k of the Jacobian of point x (world) rigidly attached to body b.
GS_HD void column(const DevLinks* __restrict__ L, const EnvKin& K, int nbase, int k, int b,
                                       const float* x, float* lin, float* ang) {
  lin[0] = lin[1] = lin[2] = 0.f;
  ang[0] = ang[1] = ang[2] = 0.f;
  if (k < nbase) {
    if (k < 3) {
      lin[k] = 1.f;
    } else {
      ang[k - 3] = 1.f;
      const float d[3] = {x[0] - K.cr[0], x[1] - K.cr[1], x[2] - K.cr[2]};
      cross3(ang, d, lin);
    }
    return;
  }
  const int j = k - nbase, bj = L->dbody[j];
  if (!((L->anc_mask[b] >> bj) & 1u)) return;
  const float* ax = K.a[bj];
  if (L->jkind[bj] == 2) {  // prismatic
    lin[0] = ax[0]; lin[1] = ax[1]; lin[2] = ax[2];
  } else {
    ang[0] = ax[0]; ang[1] = ax[1]; ang[2] = ax[2];
    const float d[3] = {x[0] - K.o[bj][0], x[1] - K.o[bj][1], x[2] - K.o[bj][2]};
    cross3(ax, d, lin);
  }
}

// forward pass of env e: poses, COMs, joint axes / points and the generalized velocity (parents
// before children; body order is DFS)
GS_HD void kin_forward(const DevModel* __restrict__ M, const DevLinks* __restrict__ L, const float* __restrict__ st,
                       int N, int e, EnvKin& K) {
  const int nb = L->nb, nd = L->nd, nbase = L->fixed_base ? 0 : 6;
  // ---- forward kinematics, parents before children (body order is DFS)
  float q[4];
  for (int k = 0; k < 4; ++k) q[k] = st[(3 + k) * N + e];
  quat_to_mat(q, K.R[0]);
  for (int k = 0; k < 3; ++k) K.p[0][k] = st[k * N + e];
  for (int b = 1; b < nb; ++b) {
    const int pb = L->parent[b];
    float Rj[9], t[3];
    mat3mul(K.R[pb], M->jR[b], Rj);  // joint frame (= child frame at q = 0)
    mat3vec(K.R[pb], M->jt[b], t);
    for (int k = 0; k < 3; ++k) K.o[b][k] = K.p[pb][k] + t[k];
    mat3vec(Rj, M->jaxis[b], K.a[b]);
    const int j = L->bdof[b];
    const float qj = j >= 0 ? st[(13 + j) * N + e] : 0.f;
    if (L->jkind[b] == 1) {
      float Ra[9];
      axis_angle(M->jaxis[b], qj, Ra);
      mat3mul(Rj, Ra, K.R[b]);
      for (int k = 0; k < 3; ++k) K.p[b][k] = K.o[b][k];
    } else {
      for (int k = 0; k < 9; ++k) K.R[b][k] = Rj[k];
      for (int k = 0; k < 3; ++k) K.p[b][k] = K.o[b][k] + (L->jkind[b] == 2 ? K.a[b][k] * qj : 0.f);
    }
  }
  for (int b = 0; b < nb; ++b) {
    float cw[3];
    mat3vec(K.R[b], M->com[b], cw);
    for (int k = 0; k < 3; ++k) K.c[b][k] = K.p[b][k] + cw[k];
  }
  {
    float cw[3];
    mat3vec(K.R[0], M->root_com, cw);
    for (int k = 0; k < 3; ++k) K.cr[k] = K.p[0][k] + cw[k];
  }
  // ---- generalized velocity: root link COM velocity = origin velocity + w x (c - p)
  if (nbase) {
    float wv[3], d[3], wc[3];
    for (int k = 0; k < 3; ++k) wv[k] = st[(10 + k) * N + e];
    for (int k = 0; k < 3; ++k) d[k] = K.cr[k] - K.p[0][k];
    cross3(wv, d, wc);
    for (int k = 0; k < 3; ++k) K.nu[k] = st[(7 + k) * N + e] + wc[k];
    for (int k = 0; k < 3; ++k) K.nu[3 + k] = wv[k];
  }
  for (int j = 0; j < nd; ++j) K.nu[nbase + j] = st[(13 + nd + j) * N + e];
}

// outputs of env e over items lane, lane + stride, ... (rb [N*nr][13], jac [N][nr][6][nv], mm [N][nv][nv])
GS_HD void kin_outputs(const DevModel* __restrict__ M, const DevLinks* __restrict__ L, const float* __restrict__ st,
                       int N, int nv, int mode, int e, const EnvKin& K, int lane, int stride, float* __restrict__ rb,
                       float* __restrict__ jac, float* __restrict__ mm) {
  const int nb = L->nb, nd = L->nd, nr = L->nr, nbase = L->fixed_base ? 0 : 6;
  (void)nb; (void)nd;
  if (mode & 1) {  // rigid body state [N*nr][13]
    for (int l = lane; l < nr; l += stride) {
      const int b = L->lbody[l];
      float R[9], t[3], x[3], cw[3];
      mat3mul(K.R[b], L->lR[l], R);
      mat3vec(K.R[b], L->lt[l], t);
      float* out = rb + ((size_t)e * nr + l) * 13;
      float pl[3];
      for (int k = 0; k < 3; ++k) pl[k] = K.p[b][k] + t[k];
      mat3vec(R, L->lcom[l], cw);
      for (int k = 0; k < 3; ++k) x[k] = pl[k] + cw[k];
      float qo[4];
      if (l == 0) {
        for (int k = 0; k < 4; ++k) qo[k] = st[(3 + k) * N + e];  // the root keeps the state's quaternion
      } else {
        mat_to_quat(R, qo);
      }
      float v[3] = {0.f, 0.f, 0.f}, om[3] = {0.f, 0.f, 0.f};
      for (int k = 0; k < nbase + nd; ++k) {
        float lin[3], ang[3];
        column(L, K, nbase, k, b, x, lin, ang);
        const float u = K.nu[k];
        for (int i = 0; i < 3; ++i) { v[i] += lin[i] * u; om[i] += ang[i] * u; }
      }
      for (int k = 0; k < 3; ++k) out[k] = pl[k];
      for (int k = 0; k < 4; ++k) out[3 + k] = qo[k];
      for (int k = 0; k < 3; ++k) out[7 + k] = v[k];
      for (int k = 0; k < 3; ++k) out[10 + k] = om[k];
    }
  }
  if (mode & 2) {  // jacobian [N][nr][6][nv], one float per lane per iteration (coalesced)
    const int per = nr * 6 * nv;
    float* out = jac + (size_t)e * per;
    for (int idx = lane; idx < per; idx += stride) {
      const int l = idx / (6 * nv), r = (idx / nv) % 6, k = idx % nv;
      const int b = L->lbody[l];
      float x[3], t[3], R[9], cw[3];
      mat3mul(K.R[b], L->lR[l], R);
      mat3vec(K.R[b], L->lt[l], t);
      mat3vec(R, L->lcom[l], cw);
      for (int i = 0; i < 3; ++i) x[i] = K.p[b][i] + t[i] + cw[i];
      float lin[3], ang[3];
      column(L, K, nbase, k, b, x, lin, ang);
      out[idx] = r < 3 ? lin[r] : ang[r - 3];
    }
  }
  if (mode & 4) {  // mass matrix [N][nv][nv]
    float* out = mm + (size_t)e * nv * nv;
    for (int idx = lane; idx < nv * nv; idx += stride) {
      const int i = idx / nv, j = idx % nv;
      float acc = 0.f;
      for (int b = 0; b < nb; ++b) {
        float li[3], ai[3], lj[3], aj[3];
        column(L, K, nbase, i, b, K.c[b], li, ai);
        column(L, K, nbase, j, b, K.c[b], lj, aj);
        // world inertia about the COM: R I R^T
        const float* I6 = M->inertia[b];
        const float Ib[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
        float RtA[3], IRtA[3], w2[3];
        const float* R = K.R[b];
        RtA[0] = R[0] * aj[0] + R[3] * aj[1] + R[6] * aj[2];
        RtA[1] = R[1] * aj[0] + R[4] * aj[1] + R[7] * aj[2];
        RtA[2] = R[2] * aj[0] + R[5] * aj[1] + R[8] * aj[2];
        mat3vec(Ib, RtA, IRtA);
        mat3vec(R, IRtA, w2);
        acc += M->mass[b] * (li[0] * lj[0] + li[1] * lj[1] + li[2] * lj[2]) +
               ai[0] * w2[0] + ai[1] * w2[1] + ai[2] * w2[2];
      }
      out[idx] = acc;
    }
  }
}

}  // namespace
