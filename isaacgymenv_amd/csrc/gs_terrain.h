// gs_terrain.h -- sphere vs heightfield-grid triangle mesh (the trimesh terrain of
// anymal_terrain.py:196-208, built by terrain_utils.convert_heightfield_to_trimesh).
//
// Mesh layout (checked on the host by gs_sim_add_triangle_mesh): vertex (i, j) of a rows x cols
// grid at index i*cols + j, at most one cell away from its grid point (x0 + i*hs, y0 + j*hs)
// (the slope-threshold moves that turn steep edges into walls); cell (i, j) holds the triangles
// (v[i,j], v[i+1,j+1], v[i,j+1]) and (v[i,j], v[i+1,j], v[i+1,j+1]).
//
// Contact rule (the oracle restates it in oracle/physics_oracle.c):
//   for a candidate sphere (centre c, radius r) and threshold thr = r + contact_offset, every
//   triangle whose closest point q to c lies within thr, and whose face normal is not pointing down
//   (n_z >= TERRAIN_DOWN_NZ), is a candidate surface:
//     * q interior to the face: normal = the face normal nf, separation = nf.(c - a) - r, also
//       when the centre is below the face by at most r + TERRAIN_BACK (penetration);
//     * q on an edge or vertex: only from the front side (nf.(c - a) >= 0), normal = (c - q)/|c - q|,
//       separation = |c - q| - r;
//   the candidate keeps the surface of the triangle CLOSEST to its centre (|sd| for a face, |c - q|
//   otherwise), first found on ties, visiting first the cell under the centre, then every cell in
//   (i, j) order, the two triangles of a cell in the order above (a foot pushed into a stair riser
//   below the tread's edge is pushed back out of the riser, not lifted onto the tread, unless the
//   tread is nearer).
// Cells are culled by their top height (a centre more than thr above every vertex of a cell
// cannot touch it from the front nor lie behind one of its faces), by their (move-extended)
// footprint widened by the horizontal reach max(thr, r + TERRAIN_BACK), and -- once a surface is
// found -- by their bounding box: a triangle's key is its distance to the centre, at least the box's,
// so a cell whose box lies no nearer than the best key cannot win (strict < updates).  All three
// tests are conservative, so the result is that of a full scan in the visiting order; on flat ground
// the box test leaves the 1-4 cells around the centre of the 25-36 in the window.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_math.h"

#define TERRAIN_BACK 0.1f
#define TERRAIN_BLK 8  // cells per side of a block in TerrainDev::blk
// faces whose unit normal points down (z below this) generate no contact: a heightfield's surface
// faces up or sideways, and the slope-threshold vertex moves can invert a triangle, whose back face
// would otherwise admit a sphere centre lying inside the terrain and push it down along the
// inverted normal (trimesh AnymalTerrain blow-up, tools/probes/trimesh_nan_replay.py)
#define TERRAIN_DOWN_NZ (-0.5f)

struct TerrainDev {
  const float4* v;     // [rows*cols] world xyz (transform applied), w unused
  const uint4* cell;   // [(rows-1)*(cols-1)]: x = top height (float bits), y = footprint flags,
                       // z = bottom height (float bits), w = footprint extents (TCELL_EXT_*)
  const float* blk;    // [ceil((rows-1)/TERRAIN_BLK)][bcols]: the highest top of each block of cells
  const float* sq4;    // [(rows-1)*(cols-1)]: the highest top of the 4 x 4 cells starting at each cell (clipped)
  const float4* rec;   // [(rows-1)*(cols-1)][TERRAIN_REC]: each cell's vertices and its two face normals (below)
  int rows, cols, bcols;
  float x0, y0, hs, inv_hs;
  float mu;            // static friction of the mesh
};

// Cell record (GS_TERR_PLANES): a cell's two triangles tested from one batch of five 16-byte
// loads, with no normal reconstruction.  rec[0..3] = v00, v01, v10, v11 (xyz), their w = n0.x, n0.y, n0.z, n1.x;
// rec[4] = (n1.y, n1.z, 0, 0); n0 / n1 = unit face normals of triangles (v00, v11, v01) / (v00, v10, v11), computed
// on the host in double from the float vertices; a degenerate (|e1 x e2|^2 <= 1e-14) or downward-facing
// (n_z < TERRAIN_DOWN_NZ) triangle is stored as n = (0, 0, -1), which the face test rejects.
#define TERRAIN_REC 5
#ifndef GS_TERR_PLANES
#define GS_TERR_PLANES 1
#endif
#ifndef GS_TERR_ROWBATCH
#define GS_TERR_ROWBATCH 8  // cell words of a row loaded together in the scan (A/B builds: 4, 16)
#endif

// footprint flags of a cell: its triangles reach one cell further towards -x, +x, -y, +y
#define TCELL_XLO 1u
#define TCELL_XHI 2u
#define TCELL_YLO 4u
#define TCELL_YHI 8u
// footprint extents of a cell (its word's w): how far its vertices reach beyond the cell square towards -x, +x,
// -y, +y, one byte each, in units of hs / 64 rounded up (the flags alone bounded a vertex moved by
// less than a quarter cell -- set only past 0.25 hs -- by the bare cell square; the extents bound every vertex the
// input check admits, up to 1.001 hs = 65 units)
#define TCELL_EXT_UNITS 64.0f

namespace gs_terrain {

GS_HD float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// closest point on triangle (a, b, c) to p (Voronoi-region walk); returns true when the point is
// interior to the face
GS_HD bool closest_on_triangle(const float* p, const float* a, const float* b, const float* c,
                                                    float* q) {
  float ab[3], ac[3], ap[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = p[k] - a[k]; }
  const float d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) { q[0] = a[0]; q[1] = a[1]; q[2] = a[2]; return false; }
  float bp[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) bp[k] = p[k] - b[k];
  const float d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0.f && d4 <= d3) { q[0] = b[0]; q[1] = b[1]; q[2] = b[2]; return false; }
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
    const float t = d1 / (d1 - d3);
#pragma unroll
    for (int k = 0; k < 3; ++k) q[k] = a[k] + t * ab[k];
    return false;
  }
  float cp[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) cp[k] = p[k] - c[k];
  const float d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0.f && d5 <= d6) { q[0] = c[0]; q[1] = c[1]; q[2] = c[2]; return false; }
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
    const float t = d2 / (d2 - d6);
#pragma unroll
    for (int k = 0; k < 3; ++k) q[k] = a[k] + t * ac[k];
    return false;
  }
  const float va = d3 * d6 - d5 * d4;
  if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
    const float t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
#pragma unroll
    for (int k = 0; k < 3; ++k) q[k] = b[k] + t * (c[k] - b[k]);
    return false;
  }
  const float den = 1.f / (va + vb + vc);
  const float v = vb * den, w = vc * den;
#pragma unroll
  for (int k = 0; k < 3; ++k) q[k] = a[k] + ab[k] * v + ac[k] * w;
  return true;
}

// one triangle: update (bkey, best, n) when it is an admissible surface closer to the centre
GS_HD void triangle(const float* p, float r, float thr, const float4& A, const float4& B,
                                         const float4& C, float& bkey, float& best, float* n) {
  const float a[3] = {A.x, A.y, A.z}, b[3] = {B.x, B.y, B.z}, c[3] = {C.x, C.y, C.z};
  const float e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const float e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  float nf[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  const float l2 = dot3(nf, nf);
  if (!(l2 > 1e-14f)) return;  // degenerate (collapsed by two vertex moves)
  const float il = gs_rsqrt(l2);
  nf[0] *= il; nf[1] *= il; nf[2] *= il;
  if (nf[2] < TERRAIN_DOWN_NZ) return;  // inverted (downward-facing) triangle
  const float ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  const float sd = dot3(nf, ap);
  if (sd > thr || sd < -(r + TERRAIN_BACK)) return;
  float q[3];
  const bool face = closest_on_triangle(p, a, b, c, q);
  if (face) {
    const float key = fabsf(sd);
    if (key < bkey) { bkey = key; best = sd - r; n[0] = nf[0]; n[1] = nf[1]; n[2] = nf[2]; }
    return;
  }
  if (sd < 0.f) return;
  const float d[3] = {p[0] - q[0], p[1] - q[1], p[2] - q[2]};
  const float dd = dot3(d, d);
  if (dd > thr * thr) return;
  const float dist = sqrtf(dd);
  if (dist < bkey) {
    bkey = dist;
    best = dist - r;
    if (dist > 1e-7f) {
      const float id = 1.f / dist;
      n[0] = d[0] * id; n[1] = d[1] * id; n[2] = d[2] * id;
    } else {
      n[0] = nf[0]; n[1] = nf[1]; n[2] = nf[2];
    }
  }
}

// one triangle given its unit face normal from the cell record (triangle()'s statements past the normal)
GS_HD void triangle_n(const float* p, float r, float thr, const float4& A, const float4& B, const float4& C,
                      const float* nf, float& bkey, float& best, float* n) {
  if (nf[2] < TERRAIN_DOWN_NZ) return;  // inverted or degenerate (flagged on the host)
  const float a[3] = {A.x, A.y, A.z}, b[3] = {B.x, B.y, B.z}, c[3] = {C.x, C.y, C.z};
  const float ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  const float sd = dot3(nf, ap);
  if (sd > thr || sd < -(r + TERRAIN_BACK)) return;
  float q[3];
  const bool face = closest_on_triangle(p, a, b, c, q);
  if (face) {
    const float key = fabsf(sd);
    if (key < bkey) { bkey = key; best = sd - r; n[0] = nf[0]; n[1] = nf[1]; n[2] = nf[2]; }
    return;
  }
  if (sd < 0.f) return;
  const float d[3] = {p[0] - q[0], p[1] - q[1], p[2] - q[2]};
  const float dd = dot3(d, d);
  if (dd > thr * thr) return;
  const float dist = sqrtf(dd);
  if (dist < bkey) {
    bkey = dist;
    best = dist - r;
    if (dist > 1e-7f) {
      const float id = 1.f / dist;
      n[0] = d[0] * id; n[1] = d[1] * id; n[2] = d[2] * id;
    } else {
      n[0] = nf[0]; n[1] = nf[1]; n[2] = nf[2];
    }
  }
}

// false when no cell around sphere (p, r) can hold a surface within thr: the range of cells within the horizontal
// reach is empty, or the sphere's lowest reach lies above the highest cell top of the range (from the 4 x 4
// square maxima; ranges wider than 8 cells from the 8 x 8 block summary).  sphere_contact starts with exactly this test; the lane team runs it alone first to hand only
// the remaining queries to the wave (gs_team.hip).
GS_HD bool may_contact(const TerrainDev& T, const float* p, float r, float thr) {
  const float reach = fmaxf(thr, r + TERRAIN_BACK);
  const float gx = (p[0] - T.x0) * T.inv_hs, gy = (p[1] - T.y0) * T.inv_hs, gt = reach * T.inv_hs;
  const int i0 = gs_imax((int)floorf(gx - gt) - 1, 0), i1 = gs_imin((int)floorf(gx + gt) + 1, T.rows - 2);
  const int j0 = gs_imax((int)floorf(gy - gt) - 1, 0), j1 = gs_imin((int)floorf(gy + gt) + 1, T.cols - 2);
  if (i0 > i1 || j0 > j1) return false;
  const float zlo = p[2] - thr;
  if (i1 - i0 <= 7 && j1 - j0 <= 7) {
    // the range's highest top exactly-or-above from four overlapping 4 x 4 squares (their union covers a range
    // up to 8 cells wide; a narrower, clipped range is covered with room to spare): one batch of loads
    const int ib = gs_imax(i0, i1 - 3), jb = gs_imax(j0, j1 - 3);
    const size_t C = (size_t)(T.cols - 1);
    const float t00 = T.sq4[i0 * C + j0], t01 = T.sq4[i0 * C + jb], t10 = T.sq4[ib * C + j0], t11 = T.sq4[ib * C + jb];
    return !(zlo > t00) || !(zlo > t01) || !(zlo > t10) || !(zlo > t11);
  }
  const int bi0 = i0 / TERRAIN_BLK, bi1 = i1 / TERRAIN_BLK, bj0 = j0 / TERRAIN_BLK, bj1 = j1 / TERRAIN_BLK;
  bool reach_any = false;
  if (bi1 - bi0 <= 1 && bj1 - bj0 <= 1) {
    const float* b0 = T.blk + (size_t)bi0 * T.bcols;
    const float* b1 = T.blk + (size_t)bi1 * T.bcols;
    const float t00 = b0[bj0], t01 = b0[bj1], t10 = b1[bj0], t11 = b1[bj1];
    reach_any = !(zlo > t00) || !(zlo > t01) || !(zlo > t10) || !(zlo > t11);
  } else {
    for (int bi = bi0; bi <= bi1; ++bi)
      for (int bj = bj0; bj <= bj1; ++bj) reach_any |= !(zlo > T.blk[(size_t)bi * T.bcols + bj]);
  }
  return reach_any;
}

// The scan of sphere_contact past its first cull (callers that ran may_contact themselves: gs_team.hip).
GS_HD bool sphere_contact_scan(const TerrainDev& T, const float* p, float r, float thr, float& sep, float* n);

// Closest admissible mesh surface for sphere (p, r); false when none lies within thr.
// (1) the range of cells and its highest top: no cell can contact (a lifted foot, the knees, the base: most
//     queries end here after one batch of loads).  Everything after it skips only cells the per-cell tests would
//     skip, so the result is the full scan's.
GS_HD bool sphere_contact(const TerrainDev& T, const float* p, float r, float thr, float& sep, float* n) {
  return may_contact(T, p, r, thr) && sphere_contact_scan(T, p, r, thr, sep, n);
}

GS_HD bool sphere_contact_scan(const TerrainDev& T, const float* p, float r, float thr, float& sep, float* n) {
  // horizontal reach: a face can be admitted from behind up to r + TERRAIN_BACK away (walls)
  const float reach = fmaxf(thr, r + TERRAIN_BACK);
  const float gx = (p[0] - T.x0) * T.inv_hs, gy = (p[1] - T.y0) * T.inv_hs, gt = reach * T.inv_hs;
  const int i0 = gs_imax((int)floorf(gx - gt) - 1, 0), i1 = gs_imin((int)floorf(gx + gt) + 1, T.rows - 2);
  const int j0 = gs_imax((int)floorf(gy - gt) - 1, 0), j1 = gs_imin((int)floorf(gy + gt) + 1, T.cols - 2);
  float best = 3.0e38f, bkey = 3.0e38f;
  const float zlo = p[2] - thr;
  const float pad = 1e-4f * T.hs;
  // one cell given its info word: the culling tests, then its two triangles (vertices loaded here unless given:
  // the cell record's TERRAIN_REC float4 with GS_TERR_PLANES, else the four vertices)
  auto cell = [&](int i, int j, const uint4& cinfo, const float4* pre = nullptr) {
    const float top = gs_bits_float(cinfo.x);
    if (zlo > top) return;
    const uint32_t x = cinfo.w;
    const float cx0 = T.x0 + (float)i * T.hs, cy0 = T.y0 + (float)j * T.hs, u = T.hs * (1.f / TCELL_EXT_UNITS);
    const float bx0 = cx0 - u * (float)(x & 255u), bx1 = cx0 + T.hs + u * (float)((x >> 8) & 255u);
    const float by0 = cy0 - u * (float)((x >> 16) & 255u), by1 = cy0 + T.hs + u * (float)(x >> 24);
    if (p[0] + reach < bx0 || p[0] - reach > bx1 || p[1] + reach < by0 || p[1] - reach > by1) return;
    const float dx = fmaxf(fmaxf(bx0 - pad - p[0], p[0] - bx1 - pad), 0.f);
    const float dy = fmaxf(fmaxf(by0 - pad - p[1], p[1] - by1 - pad), 0.f);
    const float dz = fmaxf(fmaxf(gs_bits_float(cinfo.z) - pad - p[2], p[2] - top - pad), 0.f);
    if (dx * dx + dy * dy + dz * dz >= bkey * bkey) return;
#if GS_TERR_PLANES
    const float4* rc = T.rec + ((size_t)i * (T.cols - 1) + j) * TERRAIN_REC;
    const float4 v00 = pre ? pre[0] : rc[0], v01 = pre ? pre[1] : rc[1], v10 = pre ? pre[2] : rc[2],
                 v11 = pre ? pre[3] : rc[3], x4 = pre ? pre[4] : rc[4];
    const float n0[3] = {v00.w, v01.w, v10.w}, n1[3] = {v11.w, x4.x, x4.y};
    triangle_n(p, r, thr, v00, v11, v01, n0, bkey, best, n);
    triangle_n(p, r, thr, v00, v10, v11, n1, bkey, best, n);
#else
    const size_t v0 = (size_t)i * T.cols + j;
    const float4 v00 = pre ? pre[0] : T.v[v0], v01 = pre ? pre[1] : T.v[v0 + 1];
    const float4 v10 = pre ? pre[2] : T.v[v0 + T.cols], v11 = pre ? pre[3] : T.v[v0 + T.cols + 1];
    triangle(p, r, thr, v00, v11, v01, bkey, best, n);
    triangle(p, r, thr, v00, v10, v11, bkey, best, n);
#endif
  };
  const int ic = (int)floorf(gx), jc = (int)floorf(gy);
  const bool centre = ic >= 0 && ic <= T.rows - 2 && jc >= 0 && jc <= T.cols - 2;
  if (centre) {  // the centre cell's word and vertices in one batch (it is nearly always tested)
    const uint4 cw = T.cell[(size_t)ic * (T.cols - 1) + jc];
#if GS_TERR_PLANES
    const float4* rc = T.rec + ((size_t)ic * (T.cols - 1) + jc) * TERRAIN_REC;
    const float4 pre[TERRAIN_REC] = {rc[0], rc[1], rc[2], rc[3], rc[4]};
#else
    const size_t v0 = (size_t)ic * T.cols + jc;
    const float4 pre[4] = {T.v[v0], T.v[v0 + 1], T.v[v0 + T.cols], T.v[v0 + T.cols + 1]};
#endif
    cell(ic, jc, cw, pre);
  }
  // (2) the rest in (i, j) order.  Before loading a cell's word, its widest possible footprint (one cell further
  //     on every side, plus a margin far above the float rounding of the coordinates) is tested against the
  //     reach and the best key: cells beyond it are skipped unread, whole rows at once.  A row's remaining cell
  //     words are loaded together before any is tested (one load latency per row, not one per cell).
  const float marg = pad + 0.01f * T.hs;
  const float kscale = 1.f + 1e-5f;  // the key test on the widest footprint, safely on the skipping side
  constexpr int kRowBatch = GS_TERR_ROWBATCH;
  for (int i = i0; i <= i1; ++i) {
    const float cx0 = T.x0 + (float)i * T.hs;
    const float wx0 = cx0 - T.hs - marg, wx1 = cx0 + 2.f * T.hs + marg;
    if (p[0] + reach < wx0 || p[0] - reach > wx1) continue;
    const float dxw = fmaxf(fmaxf(wx0 - p[0], p[0] - wx1), 0.f);
    const float dx2 = dxw * dxw;
    auto unread = [&](int j) {
      const float cy0 = T.y0 + (float)j * T.hs;
      const float wy0 = cy0 - T.hs - marg, wy1 = cy0 + 2.f * T.hs + marg;
      if (p[1] + reach < wy0 || p[1] - reach > wy1) return true;
      const float dyw = fmaxf(fmaxf(wy0 - p[1], p[1] - wy1), 0.f);
      return dx2 + dyw * dyw >= bkey * bkey * kscale;
    };
    int ja = j0, jz = j1;
    while (ja <= jz && unread(ja)) ++ja;
    while (jz >= ja && unread(jz)) --jz;
    const uint4* crow = T.cell + (size_t)i * (T.cols - 1);
    for (int jb = ja; jb <= jz; jb += kRowBatch) {
      uint4 cw[kRowBatch];
#pragma unroll
      for (int k = 0; k < kRowBatch; ++k) cw[k] = crow[jb + k <= jz ? jb + k : jz];
#pragma unroll
      for (int k = 0; k < kRowBatch; ++k) {
        const int j = jb + k;
        if (j <= jz && !(centre && i == ic && j == jc)) cell(i, j, cw[k]);
      }
    }
  }
  if (best >= thr - r) return false;
  sep = best;
  return true;
}

// tangent basis of the contact frame: t1 = world x projected onto the contact plane (world y
// when n is along x), t2 = n x t1; for n = +z this is (x, y), the plane contact's axes
GS_HD void tangents(const float* n, float* t1, float* t2) {
  float a[3] = {1.f - n[0] * n[0], -n[0] * n[1], -n[0] * n[2]};
  float l2 = a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
  if (l2 < 1e-6f) {
    a[0] = -n[1] * n[0]; a[1] = 1.f - n[1] * n[1]; a[2] = -n[1] * n[2];
    l2 = a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
  }
  const float il = gs_rsqrt(l2);
  t1[0] = a[0] * il; t1[1] = a[1] * il; t1[2] = a[2] * il;
  t2[0] = n[1] * t1[2] - n[2] * t1[1];
  t2[1] = n[2] * t1[0] - n[0] * t1[2];
  t2[2] = n[0] * t1[1] - n[1] * t1[0];
}

}  // namespace gs_terrain
