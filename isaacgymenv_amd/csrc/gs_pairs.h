// gs_pairs.h -- convex-hull ground contacts and self-collision narrowphase of the solver.
//
// __host__ __device__ like gs_solver.h (the host backend compiles the same source).  The fp64 restatement
// the kernels are checked against is oracle/physics_oracle.c (hull_ground_select, self_contacts); both follow
// the same rules, in the same order, so the selected vertices / pairs agree away from exact ties.
//
// Reference behaviour restated: Isaac Gym collides a filter-0 actor's shapes with each other
// (anymal_terrain.py:282, useful_hound.py:421) except on links joined by a joint, and a mesh collider is
// its convex hull (useful_hound.py:329, Hound.urdf:508-733).
#pragma once
#include "gs_internal.h"
#include "gs_math.h"
#include "gs_terrain.h"

namespace {

GS_HD float dot3f(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
// GS_GJK_TRACE=<env> (debug builds only, tools/probes/hound_pool_probe.py): device printf of GJK's iterations
// for that env in the one-thread-per-env debug kernel (gs_debug_self_contacts); on the host backend every call
#if defined(GS_GJK_TRACE) && defined(__HIP_DEVICE_COMPILE__)
#define GS_GJK_TR(...) \
  if ((int)(blockIdx.x * blockDim.x + threadIdx.x) == GS_GJK_TRACE) printf(__VA_ARGS__)
#elif defined(GS_GJK_TRACE)
#define GS_GJK_TR(...) printf(__VA_ARGS__)  // host backend: every call (run a one-env sim)
#else
#define GS_GJK_TR(...)
#endif

GS_HD void cross3f(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

// Visit rows k0 <= k < k1 of a model vertex table (4 floats per row) in index order, f(k, row).  The rows
// are read 8 at a time before any is used: a hull's index range is wave-uniform, so the 8 rows are
// independent scalar loads in flight together instead of one load-to-use wait per vertex (the tail
// batch re-reads row k1 - 1 and skips it).  Same visits, same order as the plain loop.
template <class F>
GS_HD __attribute__((always_inline)) inline void for_rows8(const float (*tab)[4], int k0, int k1, F&& f) {
  // (tab: a DevModel table declared alignas(16))
  for (int kb = k0; kb < k1; kb += 8) {
    float r[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(tab[kb + j < k1 ? kb + j : k1 - 1]);  // rows are 16-B aligned
      r[j][0] = v.x; r[j][1] = v.y; r[j][2] = v.z; r[j][3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (kb + j < k1) f(kb + j, r[j]);
  }
}

// ---------------------------------------------------------------- hull vs ground
// Vertices of hull shape sh (body pose R, X relative to the root origin; root height rootz) below
// contact_offset, reduced to at most 4: the deepest; the farthest from it horizontally; the one spanning the
// largest horizontal triangle with those two; the one farthest outside that triangle.  First index wins
// ties; a step whose best value is <= 1e-10 ends the selection.  Returns the count, vertex indices in sel.
GS_HD int hull_ground_select(const DevModel* __restrict__ M, int sh, const float* R, const float* X, float rootz,
                             float off, int* sel) {
  const int v0 = M->hv0[sh], v1 = M->hv1[sh];
  auto world = [&](const float* v, float* w) {
    w[0] = X[0] + R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
    w[1] = X[1] + R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
    w[2] = rootz + X[2] + R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  };
  int i0 = -1;
  float zmin = 3.0e38f;
  for_rows8(M->hv, v0, v1, [&](int k, const float* v) {
    float w[3];
    world(v, w);
    if (w[2] < zmin) { zmin = w[2]; i0 = k; }
  });
  if (i0 < 0 || !(zmin < off)) return 0;
  int n = 0;
  float p0[3];
  world(M->hv[i0], p0);
  sel[n++] = i0;
  int i1 = -1;
  float best = 1e-10f;
  for_rows8(M->hv, v0, v1, [&](int k, const float* v) {
    float w[3];
    world(v, w);
    if (!(w[2] < off)) return;
    const float d2 = (w[0] - p0[0]) * (w[0] - p0[0]) + (w[1] - p0[1]) * (w[1] - p0[1]);
    if (d2 > best) { best = d2; i1 = k; }
  });
  if (i1 < 0) return n;
  float p1[3];
  world(M->hv[i1], p1);
  sel[n++] = i1;
  const float ex = p1[0] - p0[0], ey = p1[1] - p0[1];
  int i2 = -1;
  best = 1e-10f;
  for_rows8(M->hv, v0, v1, [&](int k, const float* v) {
    float w[3];
    world(v, w);
    if (!(w[2] < off)) return;
    const float a = fabsf(ex * (w[1] - p0[1]) - ey * (w[0] - p0[0]));
    if (a > best) { best = a; i2 = k; }
  });
  if (i2 < 0) return n;
  float p2[3];
  world(M->hv[i2], p2);
  sel[n++] = i2;
  const float sg = (ex * (p2[1] - p0[1]) - ey * (p2[0] - p0[0])) > 0.f ? 1.f : -1.f;
  int i3 = -1;
  best = 1e-10f;
  for_rows8(M->hv, v0, v1, [&](int k, const float* v) {
    float w[3];
    world(v, w);
    if (!(w[2] < off)) return;
    const float e0 = sg * ((p1[0] - p0[0]) * (w[1] - p0[1]) - (p1[1] - p0[1]) * (w[0] - p0[0]));
    const float e1 = sg * ((p2[0] - p1[0]) * (w[1] - p1[1]) - (p2[1] - p1[1]) * (w[0] - p1[0]));
    const float e2 = sg * ((p0[0] - p2[0]) * (w[1] - p2[1]) - (p0[1] - p2[1]) * (w[0] - p2[0]));
    const float mn = fminf(fminf(e0, e1), e2);
    if (-mn > best) { best = -mn; i3 = k; }
  });
  if (i3 >= 0) sel[n++] = i3;
  return n;
}

// ---------------------------------------------------------------- self-collision
// Shape world data in the lane's LDS column: [SHW * sh + f], f: R (9), centre c (3), bounding-sphere centre (3)
constexpr int kShW = 15;
// Self-contact pool entry p at [PE * p + f]: x (3) n (3) t1 (3) t2 (3) sep mu bodyA bodyB linkA linkB | lam (3)
// | c = J nu_f (3) | 1 / diag (3) | J then scaled Z rows (3 x NV)
constexpr int kPoolX = 0, kPoolN = 3, kPoolT1 = 6, kPoolT2 = 9, kPoolSep = 12, kPoolMu = 13, kPoolBA = 14,
              kPoolBB = 15, kPoolLA = 16, kPoolLB = 17, kPoolLam = 18, kPoolC = 21, kPoolDi = 24, kPoolJ = 27;
template <class T>
struct PoolCfg {
  static constexpr int PE = kPoolJ + 3 * T::NV;
  static constexpr int FLOATS = T::NPK > 0 ? T::NPK * PE : 0;
};

// a pair record's contact: x (3) n (3) sep -- the pool entry's first 6 floats plus the separation
constexpr int kRecSep = 6, kRec = 7;

// the rest of a pool entry whose x and n are written: tangents of n, separation stays, friction (PhysX average
// of the two shapes'), bodies and links of shapes a and b
template <int LBP>
GS_HD void pool_entry_finish(const DevModel* __restrict__ M, const float* __restrict__ mu_g, int N, int e, int a, int b,
                             float* o) {
  const float nn[3] = {o[kPoolN * LBP], o[(kPoolN + 1) * LBP], o[(kPoolN + 2) * LBP]};
  float t1[3], t2[3];
  gs_terrain::tangents(nn, t1, t2);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    o[(kPoolT1 + k) * LBP] = t1[k];
    o[(kPoolT2 + k) * LBP] = t2[k];
  }
  o[kPoolMu * LBP] = 0.5f * (mu_g[a * N + e] + mu_g[b * N + e]);
  o[kPoolBA * LBP] = (float)M->shbody[a];
  o[kPoolBB * LBP] = (float)M->shbody[b];
  o[kPoolLA * LBP] = (float)M->shlink[a];
  o[kPoolLB * LBP] = (float)M->shlink[b];
}

struct ShapeW {
  float R[9], c[3], sc[3];
};

template <int LB>
GS_HD void load_shape_w(const float* shw, int sh, ShapeW& w) {
  const float* p = shw + kShW * sh * LB;
#pragma unroll
  for (int k = 0; k < 9; ++k) w.R[k] = p[k * LB];
#pragma unroll
  for (int k = 0; k < 3; ++k) { w.c[k] = p[(9 + k) * LB]; w.sc[k] = p[(12 + k) * LB]; }
}

// core support point of shape sh (world data W) in direction d; a hull's body pose is its shape pose
GS_HD void core_support(const DevModel* __restrict__ M, int sh, const ShapeW& W, const float* d, float* out) {
  const int kind = M->shkind[sh];
  const float* sz = M->shsize[sh];
  if (kind == 0) {
    out[0] = W.c[0]; out[1] = W.c[1]; out[2] = W.c[2];
  } else if (kind == 1) {
    const float ax[3] = {W.R[2], W.R[5], W.R[8]};
    const float s = dot3f(ax, d) >= 0.f ? sz[1] : -sz[1];
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k] = W.c[k] + s * ax[k];
  } else if (kind == 3) {  // flat-ended cylinder: rim point of the end disc (core radius r - m, half length h - m)
    const float mg = M->shm[sh];
    const float ax[3] = {W.R[2], W.R[5], W.R[8]};
    const float da = dot3f(ax, d);
    float pp[3] = {d[0] - da * ax[0], d[1] - da * ax[1], d[2] - da * ax[2]};
    // projected once more: for d nearly along the axis (an end disc facing the other core) the subtraction
    // cancels, and the rounding left in pp -- not orthogonal to the axis -- tilted the normalised rim direction
    // off the disc (UsefulHound, a hull face on a leg cylinder's end: the rim point 2.8 mm beyond the disc and a
    // 1.7 mm separation error, round 5)
    const float pa = dot3f(ax, pp);
#pragma unroll
    for (int k = 0; k < 3; ++k) pp[k] -= pa * ax[k];
    const float lp = sqrtf(dot3f(pp, pp));
    const float s = da >= 0.f ? sz[1] - mg : -(sz[1] - mg);
    const float rs = lp > 1e-12f ? (sz[0] - mg) / lp : 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k] = W.c[k] + s * ax[k] + rs * pp[k];
  } else if (kind == 2) {
    const float mg = M->shm[sh];
    out[0] = W.c[0]; out[1] = W.c[1]; out[2] = W.c[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float e[3] = {W.R[i], W.R[3 + i], W.R[6 + i]};
      const float s = dot3f(e, d) >= 0.f ? sz[i] - mg : -(sz[i] - mg);
#pragma unroll
      for (int k = 0; k < 3; ++k) out[k] += s * e[k];
    }
  } else {
    const float dl[3] = {W.R[0] * d[0] + W.R[3] * d[1] + W.R[6] * d[2], W.R[1] * d[0] + W.R[4] * d[1] + W.R[7] * d[2],
                         W.R[2] * d[0] + W.R[5] * d[1] + W.R[8] * d[2]};
    const float cc[3] = {M->shc[sh][0], M->shc[sh][1], M->shc[sh][2]};
    float best = -3.0e38f, bv[3] = {0.f, 0.f, 0.f};
    for_rows8(M->pv, M->pv0[sh], M->pv1[sh], [&](int, const float* v) {
      const float f = v[3];
      const float p[3] = {cc[0] + f * (v[0] - cc[0]), cc[1] + f * (v[1] - cc[1]), cc[2] + f * (v[2] - cc[2])};
      const float t = dot3f(p, dl);
      if (t > best) { best = t; bv[0] = p[0]; bv[1] = p[1]; bv[2] = p[2]; }
    });
    mat3vec(W.R, bv, out);
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k] += W.c[k];
  }
}

// Centroid of shape sh's core support feature in direction d: the core points within kFeatureEps of the
// support plane (box corners, hull vertices; a cylinder's end disc, side line or rim point; a capsule's segment
// or end; a sphere's centre).  Returns the feature's extent, 0 for a single point (the oracle's core_feature).
constexpr float kFeatureEps = 2e-3f;
#ifndef GS_DEEP_SKIP
#define GS_DEEP_SKIP 1
#endif
GS_HD float core_feature(const DevModel* __restrict__ M, int sh, const ShapeW& W, const float* d, float* cen) {
  const int kind = M->shkind[sh];
  const float* sz = M->shsize[sh];
  const float mg = M->shm[sh];
  if (kind == 0) {
    cen[0] = W.c[0]; cen[1] = W.c[1]; cen[2] = W.c[2];
    return 0.f;
  }
  if (kind == 1 || kind == 3) {
    const float ax[3] = {W.R[2], W.R[5], W.R[8]};
    const float hl = kind == 1 ? sz[1] : sz[1] - mg, rr = kind == 1 ? 0.f : sz[0] - mg;
    const float da = dot3f(ax, d);
    const float pp[3] = {d[0] - da * ax[0], d[1] - da * ax[1], d[2] - da * ax[2]};
    const float lp = sqrtf(dot3f(pp, pp));
    const bool side = 2.f * hl * fabsf(da) <= kFeatureEps;
    const bool disc = kind == 3 && 2.f * rr * lp <= kFeatureEps;
    const float s = side ? 0.f : (da >= 0.f ? hl : -hl);
    const float rs = (disc || !(lp > 1e-12f)) ? 0.f : rr / lp;
#pragma unroll
    for (int k = 0; k < 3; ++k) cen[k] = W.c[k] + s * ax[k] + rs * pp[k];
    return side ? hl : (disc ? rr : 0.f);
  }
  if (kind == 2) {
    float pts[8][3], hmax = -3.0e38f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
      for (int k = 0; k < 3; ++k) pts[c][k] = W.c[k];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float sg = ((c >> i) & 1) ? 1.f : -1.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) pts[c][k] += sg * (sz[i] - mg) * W.R[3 * k + i];
      }
      hmax = fmaxf(hmax, dot3f(pts[c], d));
    }
    float acc[3] = {0.f, 0.f, 0.f};
    int n = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (dot3f(pts[c], d) >= hmax - kFeatureEps) {
        acc[0] += pts[c][0]; acc[1] += pts[c][1]; acc[2] += pts[c][2];
        ++n;
      }
    const float inv = 1.f / (float)n;
#pragma unroll
    for (int k = 0; k < 3; ++k) cen[k] = acc[k] * inv;
    float ext = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (dot3f(pts[c], d) >= hmax - kFeatureEps) {
        const float dd[3] = {pts[c][0] - cen[0], pts[c][1] - cen[1], pts[c][2] - cen[2]};
        ext = fmaxf(ext, sqrtf(dot3f(dd, dd)));
      }
    return ext;
  }
  const float dl[3] = {W.R[0] * d[0] + W.R[3] * d[1] + W.R[6] * d[2], W.R[1] * d[0] + W.R[4] * d[1] + W.R[7] * d[2],
                       W.R[2] * d[0] + W.R[5] * d[1] + W.R[8] * d[2]};
  const float cc[3] = {M->shc[sh][0], M->shc[sh][1], M->shc[sh][2]};
  auto corev = [&](const float* v, float* p) {
    const float f = v[3];
    p[0] = cc[0] + f * (v[0] - cc[0]); p[1] = cc[1] + f * (v[1] - cc[1]); p[2] = cc[2] + f * (v[2] - cc[2]);
  };
  const int k0 = M->pv0[sh], k1 = M->pv1[sh];
  float hmax = -3.0e38f;
  for_rows8(M->pv, k0, k1, [&](int, const float* v) {
    float p[3];
    corev(v, p);
    hmax = fmaxf(hmax, dot3f(p, dl));
  });
  float acc[3] = {0.f, 0.f, 0.f};
  int n = 0;
  for_rows8(M->pv, k0, k1, [&](int, const float* v) {
    float p[3];
    corev(v, p);
    if (dot3f(p, dl) >= hmax - kFeatureEps) {
      acc[0] += p[0]; acc[1] += p[1]; acc[2] += p[2];
      ++n;
    }
  });
  const float inv = 1.f / (float)n;
  acc[0] *= inv; acc[1] *= inv; acc[2] *= inv;
  float ext = 0.f;
  for_rows8(M->pv, k0, k1, [&](int, const float* v) {
    float p[3];
    corev(v, p);
    if (dot3f(p, dl) >= hmax - kFeatureEps) {
      const float dd[3] = {p[0] - acc[0], p[1] - acc[1], p[2] - acc[2]};
      ext = fmaxf(ext, sqrtf(dot3f(dd, dd)));
    }
  });
  mat3vec(W.R, acc, cen);
#pragma unroll
  for (int k = 0; k < 3; ++k) cen[k] += W.c[k];
  return ext;
}

// Closest point of conv(W[0..k)) to the origin: every vertex subset whose affine closest point has positive
// barycentrics is a candidate, the nearest wins (first subset on ties).  Subsets are compile-time masks, so
// the simplex stays in registers.  Returns the chosen mask (0: none valid).
template <int MASK>
GS_HD void simplex_subset(const float (&W)[4][3], int k, float& best, int& bm, float* v, float* lam) {
  constexpr int n = ((MASK >> 0) & 1) + ((MASK >> 1) & 1) + ((MASK >> 2) & 1) + ((MASK >> 3) & 1);
  constexpr int top = (MASK & 8) ? 4 : (MASK & 4) ? 3 : (MASK & 2) ? 2 : 1;
  if (top > k) return;
  int id[4] = {0, 0, 0, 0};
  {
    int c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((MASK >> i) & 1) id[c++] = i;
  }
  float l[4] = {1.f, 0.f, 0.f, 0.f}, p[3];
  if constexpr (n == 1) {
    p[0] = W[id[0]][0]; p[1] = W[id[0]][1]; p[2] = W[id[0]][2];
  } else {
    constexpr int q = n - 1;
    float E[3][3], G[3][3], r[3], mu[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 1; j < n; ++j)
#pragma unroll
      for (int a = 0; a < 3; ++a) E[j - 1][a] = W[id[j]][a] - W[id[0]][a];
#pragma unroll
    for (int i = 0; i < q; ++i) {
      r[i] = -dot3f(W[id[0]], E[i]);
#pragma unroll
      for (int j = 0; j < q; ++j) G[i][j] = dot3f(E[i], E[j]);
    }
    if constexpr (q == 1) {
      if (!(G[0][0] > 1e-18f)) return;
      mu[0] = r[0] / G[0][0];
    } else if constexpr (q == 2) {
      const float det = G[0][0] * G[1][1] - G[0][1] * G[1][0];
      if (!(fabsf(det) > 1e-12f * G[0][0] * G[1][1]) || !(det != 0.f)) return;
      mu[0] = (r[0] * G[1][1] - G[0][1] * r[1]) / det;
      mu[1] = (G[0][0] * r[1] - r[0] * G[1][0]) / det;
    } else {
      auto det3 = [](const float (&A)[3][3]) {
        return A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
               A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
      };
      const float det = det3(G);
      if (!(fabsf(det) > 1e-12f * G[0][0] * G[1][1] * G[2][2]) || !(det != 0.f)) return;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float Gc[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) Gc[i][j] = j == c ? r[i] : G[i][j];
        mu[c] = det3(Gc) / det;
      }
    }
    float l0 = 1.f;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < q; ++j) {
      l0 -= mu[j];
      l[j + 1] = mu[j];
      ok = ok && (mu[j] > 1e-12f);
    }
    l[0] = l0;
    if (!ok || !(l0 > 1e-12f)) return;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      p[a] = W[id[0]][a];
#pragma unroll
      for (int j = 0; j < q; ++j) p[a] += mu[j] * E[j][a];
    }
  }
  const float d2 = dot3f(p, p);
  if (d2 < best) {
    best = d2;
    bm = MASK;
    v[0] = p[0]; v[1] = p[1]; v[2] = p[2];
    int j = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) lam[i] = ((MASK >> i) & 1) ? l[j++] : 0.f;
  }
}
template <int MASK = 1>
GS_HD void simplex_all(const float (&W)[4][3], int k, float& best, int& bm, float* v, float* lam) {
  if constexpr (MASK < 16) {
    simplex_subset<MASK>(W, k, best, bm, v, lam);
    simplex_all<MASK + 1>(W, k, best, bm, v, lam);
  }
}

// GJK distance between the cores of shapes a and b: closest points pa, pb and the separating vector
// vout = pa - pb (from the final simplex's closest point: the contact normal's direction, more accurate than
// the difference of the two closest points); returns the distance, 0 when the cores overlap (same iteration
// and termination rules as the oracle's gjk_cores)
// stop: a distance beyond which the caller has no use for the closest points -- once GJK's lower bound (the
// support plane's offset v.w / |v|) exceeds it, the search ends and returns that bound (pa, pb unset)
GS_HD float gjk_cores(const DevModel* __restrict__ M, int sa, int sb, const ShapeW& Wa, const ShapeW& Wb, float* pa,
                      float* pb, float* vout, float stop = 3.0e38f) {
  float v[3] = {Wa.sc[0] - Wb.sc[0], Wa.sc[1] - Wb.sc[1], Wa.sc[2] - Wb.sc[2]};
  if (dot3f(v, v) < 1e-18f) { v[0] = 1.f; v[1] = 0.f; v[2] = 0.f; }
  float W[4][3], A[4][3], B[4][3], lam[4] = {1.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 3; ++t) W[i][t] = A[i][t] = B[i][t] = 0.f;
  int k = 0;
  // a support plane with v.w > 1e-4 vv has certified a positive distance (at least v.w / |v|, far above rounding):
  // from then on a subset search that reads the origin as enclosed is a rounding failure, not an overlap
  bool sepd = false;
  for (int it = 0; it < 32; ++it) {
    const float nv[3] = {-v[0], -v[1], -v[2]};
    float a[3], b[3], w[3];
    core_support(M, sa, Wa, nv, a);
    core_support(M, sb, Wb, v, b);
#pragma unroll
    for (int t = 0; t < 3; ++t) w[t] = a[t] - b[t];
    const float vv = dot3f(v, v), vw = dot3f(v, w);
    GS_GJK_TR("gjk %d-%d it %d k %d v %.9g %.9g %.9g w %.9g %.9g %.9g vv %.9g vw %.9g\n", sa, sb, it, k, v[0], v[1],
              v[2], w[0], w[1], w[2], vv, vw);
    if (vw > 0.f && vw * vw > stop * stop * vv) return vw / sqrtf(vv);  // separated by more than stop
    sepd = sepd || vw > 1e-4f * vv;
    // converged: the support plane is within 1e-6 |v| of the simplex's closest point (the distance to ~1e-6
    // relative; the oracle's fp64 bound is 1e-10, which float arithmetic cannot resolve: below ~1e-7 vv the test
    // reads rounding, so a converged float search ran on until a repeated support point or the iteration cap)
    if (k > 0 && vv - vw <= 1e-6f * vv + 1e-14f) break;
    // Step along the segment from the closest point of the first kold simplex points -- a point of the Minkowski
    // difference whose witness points are the same combination of A and B -- to w: a strict decrease whenever
    // v.w < v.v, and the next simplex {that point, w} is well conditioned.  Returns false (the simplex cut back to
    // kold points, v its closest point) when rounding leaves no progress.
    auto segment_step = [&](int kold) -> bool {
      float Av[3] = {0.f, 0.f, 0.f}, Bv[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i < kold)
#pragma unroll
          for (int t = 0; t < 3; ++t) { Av[t] += lam[i] * A[i][t]; Bv[t] += lam[i] * B[i][t]; }
      const float Wv[3] = {Av[0] - Bv[0], Av[1] - Bv[1], Av[2] - Bv[2]};
      const float d[3] = {w[0] - Wv[0], w[1] - Wv[1], w[2] - Wv[2]};
      const float dd = dot3f(d, d);
      float t = dd > 0.f ? -dot3f(Wv, d) / dd : 0.f;
      t = t > 1.f ? 1.f : t;
      GS_GJK_TR("gjk %d-%d   segment step from %d points t %.9g\n", sa, sb, kold, t);
      if (!(t > 0.f)) {
        k = kold;
#pragma unroll
        for (int s = 0; s < 3; ++s) v[s] = Wv[s];
        return false;
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        W[0][s] = Wv[s]; A[0][s] = Av[s]; B[0][s] = Bv[s];
        W[1][s] = w[s]; A[1][s] = a[s]; B[1][s] = b[s];
        v[s] = Wv[s] + t * d[s];
      }
      lam[0] = 1.f - t; lam[1] = t; lam[2] = 0.f; lam[3] = 0.f;
      k = 2;
      return true;
    };
    bool dup = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d[3] = {W[i][0] - w[0], W[i][1] - w[1], W[i][2] - w[2]};
      dup = dup || (i < k && dot3f(d, d) < 1e-16f);
    }
    // A support point already in the simplex although the search has not converged (v.w < v.v beyond the
    // tolerance): in exact arithmetic v is the simplex's closest point and v.p >= v.v for every vertex p, so v is
    // off by the rounding of the subset solve -- sliver triangles of two finely tessellated hulls (UsefulHound's
    // trunk against an arm link: 0.7 degrees of contact normal, round 5).  Step instead of stopping.
    if (dup) {
      if (segment_step(k)) continue;
      break;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == k) {
#pragma unroll
        for (int t = 0; t < 3; ++t) { W[i][t] = w[t]; A[i][t] = a[t]; B[i][t] = b[t]; }
      }
    ++k;
    float best = 3.0e38f, l4[4] = {0.f, 0.f, 0.f, 0.f};
    int mask = 0;
    simplex_all(W, k, best, mask, v, l4);
    GS_GJK_TR("gjk %d-%d   mask %d best %.9g v %.9g %.9g %.9g\n", sa, sb, mask, best, v[0], v[1], v[2]);
    if (!mask && !sepd) return 0.f;
    if (!((mask >> (k - 1)) & 1) || (sepd && (mask == 15 || !(best >= 1e-18f)))) {
      // The subset search dropped the new support point w although w lies beyond the old closest point's support
      // plane (vv - vw above the tolerance) -- in exact arithmetic the grown simplex's closest point involves w --
      // or it read the origin as enclosed after a support plane had certified a positive distance.  Only rounding
      // does either: the case of a curved core (a cylinder's rim), whose support points crowd together into
      // sliver triangles and tetrahedra as the search converges.  Left alone the search re-added w until the
      // iteration cap and returned the old point, or reported overlapping cores (UsefulHound env 111 of the r04f
      // failure: a 4e-3 rad contact-normal error; the fp32 oracle dropped the contact).
      if (segment_step(k - 1)) continue;
      break;
    }
    // keep the chosen subset, in order (compile-time moves under runtime conditions)
    float W2[4][3], A2[4][3], B2[4][3];
    int n = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 3; ++t) W2[i][t] = A2[i][t] = B2[i][t] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if ((mask >> i) & 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j == n) {
#pragma unroll
            for (int t = 0; t < 3; ++t) { W2[j][t] = W[i][t]; A2[j][t] = A[i][t]; B2[j][t] = B[i][t]; }
            lam[j] = l4[i];
          }
        ++n;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < 3; ++t) { W[i][t] = W2[i][t]; A[i][t] = A2[i][t]; B[i][t] = B2[i][t]; }
    k = n;
    if (k == 4 || dot3f(v, v) < 1e-18f) return 0.f;
  }
  pa[0] = pa[1] = pa[2] = pb[0] = pb[1] = pb[2] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < k)
#pragma unroll
      for (int t = 0; t < 3; ++t) { pa[t] += lam[i] * A[i][t]; pb[t] += lam[i] * B[i][t]; }
  // The separating direction from the final simplex's geometry: its affine closest point from cross products
  // (the segment's perpendicular, the triangle's plane normal) instead of W0 + mu E, whose normal-equation
  // rounding leaves it off the perpendicular by ~cond(G) ulps -- up to ~1e-2 rad of contact-normal error for
  // near-parallel hull faces in float.  Only the direction is refined (GJK's subset choice above keeps the
  // normal-equation points, which lie in the simplex's affine hull: a cross-product point of a near-degenerate
  // subset could undercut the true distance and mislead the search), and only from a well-conditioned simplex.
  float vr[3] = {v[0], v[1], v[2]};
  if (k == 2 || k == 3) {
    float E0[3], E1[3], pr[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) { E0[t] = W[1][t] - W[0][t]; E1[t] = W[2][t] - W[0][t]; }
    bool ok = false;
    if (k == 2) {
      const float ee = dot3f(E0, E0);
      float c1[3];
      cross3f(E0, W[0], c1);
      cross3f(c1, E0, pr);
      ok = ee > 0.f;
#pragma unroll
      for (int t = 0; t < 3; ++t) pr[t] = ok ? pr[t] / ee : 0.f;
    } else {
      float nr[3];
      cross3f(E0, E1, nr);
      const float nn2 = dot3f(nr, nr);
      ok = nn2 > 1e-8f * dot3f(E0, E0) * dot3f(E1, E1);  // the triangle's angles above ~1e-4 rad
      const float s = ok ? dot3f(nr, W[0]) / nn2 : 0.f;
#pragma unroll
      for (int t = 0; t < 3; ++t) pr[t] = s * nr[t];
    }
    // (a refinement, not a new answer: it must agree with v to within a small angle)
    const float vv = dot3f(v, v), pp = dot3f(pr, pr), vp = dot3f(v, pr);
    if (ok && vp > 0.f && vp * vp >= 0.9999f * vv * pp) { vr[0] = pr[0]; vr[1] = pr[1]; vr[2] = pr[2]; }
  }
  vout[0] = vr[0]; vout[1] = vr[1]; vout[2] = vr[2];
  GS_GJK_TR("gjk %d-%d done k %d pa %.9g %.9g %.9g pb %.9g %.9g %.9g\n", sa, sb, k, pa[0], pa[1], pa[2], pb[0], pb[1],
            pb[2]);
  return sqrtf(dot3f(v, v));
}

GS_HD void seg_closest_pt(const float* p, const float* a, const float* b, float* q) {
  const float ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  const float l2 = dot3f(ab, ab);
  float t = l2 > 0.f ? dot3f(ap, ab) / l2 : 0.f;
  t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
#pragma unroll
  for (int k = 0; k < 3; ++k) q[k] = a[k] + t * ab[k];
}

// closest points of segments p1q1, p2q2 (Ericson), parameters s, t; den = a e - b^2
GS_HD void seg_seg(const float* p1, const float* q1, const float* p2, const float* q2, float& s, float& t, float& den,
                   float& a, float& e) {
  float d1[3], d2[3], r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
  a = dot3f(d1, d1);
  e = dot3f(d2, d2);
  const float f = dot3f(d2, r);
  s = 0.f; t = 0.f; den = 0.f;
  auto cl = [](float x) { return x < 0.f ? 0.f : (x > 1.f ? 1.f : x); };
  if (a <= 1e-12f && e <= 1e-12f) {
  } else if (a <= 1e-12f) {
    t = cl(f / e);
  } else {
    const float c = dot3f(d1, r);
    if (e <= 1e-12f) {
      s = cl(-c / a);
    } else {
      const float b = dot3f(d1, d2);
      den = a * e - b * b;
      s = den > 0.f ? cl((b * f - c * e) / den) : 0.f;
      t = (b * s + f) / e;
      if (t < 0.f) { t = 0.f; s = cl(-c / a); }
      else if (t > 1.f) { t = 1.f; s = cl((b - c) / a); }
    }
  }
}

constexpr int kUnrollPairs = 64;  // pair tables up to this size are unrolled at compile time

// Self-contacts of one env in pair order, at most T::NPK (later ones dropped): broadphase on the shapes'
// bounding spheres (within contact_offset), closed-form sphere / capsule pairs, GJK on margin-rounded cores
// otherwise.  Writes the pool entries' geometry (x relative to the root origin, n from B to A, tangents,
// separation, friction, bodies, links); returns the count.
// (shape data at stride LB, pool entries at stride LBP with PE floats per entry: the one-env-per-lane solver
// keeps both in its lane column; the lane team reads a per-team shape table and keeps a shorter entry)
// Per-shape constants of the narrowphase: bounding-sphere radius, margin (core rounding), capsule half length.
// ShapeConstsM reads the model; the lane team stages them in LDS once per launch (ShapeConstsTab, kShC floats
// per shape), so a pair's test waits on no scalar-cache miss.
struct ShapeConstsM {
  const DevModel* __restrict__ M;
  GS_HD float brad(int s) const { return M->shc[s][3]; }
  GS_HD float margin(int s) const { return M->shm[s]; }
  GS_HD float hlen(int s) const { return M->shsize[s][1]; }
};
constexpr int kShC = 4;
struct ShapeConstsTab {
  const float* __restrict__ t;
  GS_HD float brad(int s) const { return t[kShC * s]; }
  GS_HD float margin(int s) const { return t[kShC * s + 1]; }
  GS_HD float hlen(int s) const { return t[kShC * s + 2]; }
};

// One pair (shapes a < b, pair kind) of self_contacts: appends its contacts to the pool (n counts them).
// REC: a pair record of the wave-assisted lane kernels (gs_physics_impl.h pair_records) -- only x, n and the
// separation (kRec floats per contact); pool_entry_finish completes the entry as the full form writes it.
template <class T, int LB, int LBP, int PE, class SC, bool REC = false>
GS_HD __attribute__((always_inline)) inline void self_pair(const DevModel* __restrict__ M, const SC& sc,
                                                           const DevParams& P, const float* __restrict__ mu_g, int N,
                                                           int e, const float* shw, float* pool, int a, int b,
                                                           int kind, int& n) {
  const float off = P.contact_offset;
  {
    const float* sa = shw + (kShW * a + 12) * LB;
    const float* sb = shw + (kShW * b + 12) * LB;
    const float d[3] = {sa[0] - sb[0], sa[LB] - sb[LB], sa[2 * LB] - sb[2 * LB]};
    const float rr = sc.brad(a) + sc.brad(b) + off;
    if (!(dot3f(d, d) < rr * rr)) return;
  }
  {
    ShapeW Wa, Wb;
    load_shape_w<LB>(shw, a, Wa);
    load_shape_w<LB>(shw, b, Wb);
    const float ra = sc.margin(a), rb = sc.margin(b);
    float pa[2][3], pb[2][3];
    int nct = 1;
    bool gdeep = false, gnorm = false;
    float gn[3] = {0.f, 0.f, 1.f}, gdist = 0.f;  // GJK pairs: the contact normal and the cores' distance
    if (kind == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) { pa[0][k] = Wa.c[k]; pb[0][k] = Wb.c[k]; }
    } else if (kind == 1) {
      const bool a_sph = T::shkind[a] == 0;  // (the compiled topology's kinds: gs_sim_set_model checks them)
      const ShapeW& Wc = a_sph ? Wb : Wa;
      const ShapeW& Ws = a_sph ? Wa : Wb;
      const float hl = sc.hlen(a_sph ? b : a);
      const float ax[3] = {Wc.R[2], Wc.R[5], Wc.R[8]};
      float e0[3], e1[3], q3[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) { e0[k] = Wc.c[k] - hl * ax[k]; e1[k] = Wc.c[k] + hl * ax[k]; }
      seg_closest_pt(Ws.c, e0, e1, q3);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        pa[0][k] = a_sph ? Ws.c[k] : q3[k];
        pb[0][k] = a_sph ? q3[k] : Ws.c[k];
      }
    } else if (kind == 2) {
      const float ha = sc.hlen(a), hb = sc.hlen(b);
      float p1[3], q1[3], p2[3], q2[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float axa = Wa.R[3 * k + 2], axb = Wb.R[3 * k + 2];
        p1[k] = Wa.c[k] - ha * axa; q1[k] = Wa.c[k] + ha * axa;
        p2[k] = Wb.c[k] - hb * axb; q2[k] = Wb.c[k] + hb * axb;
      }
      float s, t, den, aa, ee;
      seg_seg(p1, q1, p2, q2, s, t, den, aa, ee);
      bool two = false;
      float lo = 0.f, hi = 0.f;
      if (aa > 1e-12f && ee > 1e-12f && den <= 1e-4f * aa * ee) {
        float d1[3], w0[3], w1[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { d1[k] = q1[k] - p1[k]; w0[k] = p2[k] - p1[k]; w1[k] = q2[k] - p1[k]; }
        const float s0 = dot3f(w0, d1) / aa, s1 = dot3f(w1, d1) / aa;
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
          for (int k = 0; k < 3; ++k) pa[c][k] = p1[k] + sc2 * (q1[k] - p1[k]);
          seg_closest_pt(pa[c], p2, q2, pb[c]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) { pa[0][k] = p1[k] + s * (q1[k] - p1[k]); pb[0][k] = p2[k] + t * (q2[k] - p2[k]); }
      }
    } else {
      // (a pair whose cores are farther apart than contact_offset + radii makes no contact: stop there, with a
      // hair of slack so the bound's rounding never drops a contact the full search would keep)
      const float stop = (off + ra + rb) * 1.001f + 1e-5f;
      float vg[3];
      const float dist = gjk_cores(M, a, b, Wa, Wb, pa[0], pb[0], vg, stop);
      if (dist > stop) return;
      if (!(dist > 1e-9f)) {
        gdeep = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) { pa[0][k] = Wa.sc[k]; pb[0][k] = Wb.sc[k]; }
      } else {
        // the contact point: the centroid of the smaller of the two support features facing each other (a
        // face's, not GJK's arbitrary point of it), kept at the cores' distance
        const float inv = 1.f / dist;
        const float nn[3] = {vg[0] * inv, vg[1] * inv, vg[2] * inv};
        gnorm = true;
        gdist = dist;
        gn[0] = nn[0]; gn[1] = nn[1]; gn[2] = nn[2];
        const float mn[3] = {-nn[0], -nn[1], -nn[2]};
        float ca[3], cb[3];
        const float ea = core_feature(M, a, Wa, mn, ca);
        const float eb = core_feature(M, b, Wb, nn, cb);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (ea <= eb) { pa[0][k] = ca[k]; pb[0][k] = ca[k] - dist * nn[k]; }
          else { pb[0][k] = cb[k]; pa[0][k] = cb[k] + dist * nn[k]; }
        }
      }
    }
    for (int c = 0; c < nct; ++c) {
      if (n >= T::NPK) break;
      float nn[3] = {pa[c][0] - pb[c][0], pa[c][1] - pb[c][1], pa[c][2] - pb[c][2]};
      float dist = sqrtf(dot3f(nn, nn));
      if (gnorm) {  // (pa - pb of the feature construction is dist * n up to the rounding of |pa| ~ 0.5 m)
#pragma unroll
        for (int k = 0; k < 3; ++k) nn[k] = gn[k];
        dist = gdist;
      } else if (!(dist > 1e-9f)) {
        float f[3] = {Wa.sc[0] - Wb.sc[0], Wa.sc[1] - Wb.sc[1], Wa.sc[2] - Wb.sc[2]};
        float l = sqrtf(dot3f(f, f));
        if (!(l > 1e-9f)) { f[0] = 0.f; f[1] = 0.f; f[2] = 1.f; l = 1.f; }
#pragma unroll
        for (int k = 0; k < 3; ++k) nn[k] = f[k] / l;
        dist = 0.f;
      } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) nn[k] /= dist;
      }
      if (gdeep && GS_DEEP_SKIP) continue;
      const float sep = gdeep ? -(ra + rb) : dist - ra - rb;
      if (!(sep < off)) continue;
      float* o = pool + PE * n * LBP;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        o[(kPoolX + k) * LBP] = 0.5f * ((pa[c][k] - ra * nn[k]) + (pb[c][k] + rb * nn[k]));
        o[(kPoolN + k) * LBP] = nn[k];
      }
      if constexpr (REC) {
        o[kRecSep * LBP] = sep;
      } else {
        o[kPoolSep * LBP] = sep;
        pool_entry_finish<LBP>(M, mu_g, N, e, a, b, o);
      }
      ++n;
    }
  }
}

// (mask: a caller's broadphase may restrict the pairs to a superset of those that can touch -- bit q of pair q;
// the result is the same as without it)
template <class T, int LB, int LBP = LB, int PE = PoolCfg<T>::PE, class SC = ShapeConstsM>
GS_HD int self_contacts(const DevModel* __restrict__ M, const DevParams& P, const float* __restrict__ mu_g, int N,
                        int e, const float* shw, float* pool, const SC& sc, unsigned long long mask = ~0ull) {
  int n = 0;
  if constexpr (T::NPAIR <= kUnrollPairs) {
    // the compiled topology's pair table (gs_sim_set_model checks it against the model's): shapes and pair
    // kinds fold into the code, the shapes' constants are independent loads
#pragma unroll
    for (int q = 0; q < T::NPAIR; ++q)
      if (n < T::NPK && ((mask >> q) & 1ull))
        self_pair<T, LB, LBP, PE>(M, sc, P, mu_g, N, e, shw, pool, T::pair_a[q], T::pair_b[q], T::pair_k[q], n);
  } else {
    // runtime pair table (UsefulHound: 253 pairs): 8 pairs' shapes and bounding spheres are read together
    // and tested, then the near ones run self_pair in pair order (which repeats the same test)
    const int np = M->np;
    const float off = P.contact_offset;
    for (int q0 = 0; q0 < np; q0 += 8) {
      if (n >= T::NPK) break;
      int pa[8], pb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int q = q0 + j < np ? q0 + j : np - 1;
        pa[j] = M->pa[q];
        pb[j] = M->pb[q];
      }
      unsigned near = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* sa = shw + (kShW * pa[j] + 12) * LB;
        const float* sb = shw + (kShW * pb[j] + 12) * LB;
        const float d[3] = {sa[0] - sb[0], sa[LB] - sb[LB], sa[2 * LB] - sb[2 * LB]};
        const float rr = sc.brad(pa[j]) + sc.brad(pb[j]) + off;
        if (q0 + j < np && dot3f(d, d) < rr * rr) near |= 1u << j;
      }
      // (one inlined narrowphase: j stays a uniform loop counter, the pair's shapes are re-read by index)
#pragma unroll 1
      for (int j = 0; j < 8; ++j)
        if (((near >> j) & 1u) && n < T::NPK)
          self_pair<T, LB, LBP, PE>(M, sc, P, mu_g, N, e, shw, pool, M->pa[q0 + j], M->pb[q0 + j], M->pk[q0 + j], n);
    }
  }
  return n;
}
template <class T, int LB, int LBP = LB, int PE = PoolCfg<T>::PE>
GS_HD int self_contacts(const DevModel* __restrict__ M, const DevParams& P, const float* __restrict__ mu_g, int N,
                        int e, const float* shw, float* pool) {
  return self_contacts<T, LB, LBP, PE, ShapeConstsM>(M, P, mu_g, N, e, shw, pool, ShapeConstsM{M});
}

}  // namespace
