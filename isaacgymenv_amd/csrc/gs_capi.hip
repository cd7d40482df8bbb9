// gs_capi.hip -- the C ABI of libgymsim.so (include/gymsim.h).
//
// Host-side object that replaces the Isaac Gym `sim` handle: it owns the
// float32 device copy of the articulation model, the parsed SimParams and the
// selected kernel specialisation, and binds the caller-owned (torch) device
// buffers that hold the sim state.  All launches are stream ordered; nothing
// here synchronises the host except create/set_model/prepare.
//
// A sim created with device < 0 is the host backend (gs_host.hip, the reference's
// sim_device=cpu pipeline): same entry points, caller-owned HOST buffers, the solver
// runs on a thread pool inside the call, `stream` is ignored, no HIP call is made.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "gs_internal.h"
#include "../../include/gymsim.h"

namespace {
thread_local std::string g_err;

int fail(const char* fmt, const char* arg = nullptr) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), fmt, arg ? arg : "");
  g_err = buf;
  return -1;
}
int hip_fail(hipError_t e, const char* where) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", where, hipGetErrorString(e));
  g_err = buf;
  return -1;
}

std::string signature(const gs_model_desc* m) {
  std::string s = "fb" + std::to_string(m->fixed_base) + "_p";
  for (int i = 0; i < m->num_bodies; ++i) s += (i ? "-" : "") + std::to_string(m->parent[i]);
  s += "_c";
  for (int i = 0; i < m->num_candidates; ++i) s += (i ? "-" : "") + std::to_string(m->cand_body[i]);
  // kept fixed-joint links change the compiled contact-force tables (_model.topology_signature)
  bool links_differ = m->num_links != m->num_bodies;
  for (int i = 0; i < m->num_candidates && !links_differ; ++i) links_differ = m->cand_link[i] != m->cand_body[i];
  if (links_differ) {
    s += "_l" + std::to_string(m->num_links) + "_";
    for (int i = 0; i < m->num_candidates; ++i) s += (i ? "-" : "") + std::to_string(m->cand_link[i]);
  }
  return s;
}

const TopoEntry* find_topology(const gs_model_desc* m) {
  const std::string sig = signature(m);
  for (int i = 0; i < g_num_topologies; ++i)
    if (sig == g_topologies[i].sig) return &g_topologies[i];
  return nullptr;
}
}  // namespace

struct gs_sim {
  int device = 0;
  gs_sim_params params{};
  DevParams dp{};
  bool has_ground = false;
  float ground_mu = 1.f;
  const TopoEntry* topo = nullptr;
  launch_sim_fn sim_fn = nullptr;
  launch_pd_fn pd_fn = nullptr;
  int variant = 0;  // kernel actually selected: 1 lane, 2 team
  // the kernel gs_sim_set_model selected (drives may move the sim to the lane kernel and back)
  launch_sim_fn model_sim_fn = nullptr;
  launch_pd_fn model_pd_fn = nullptr;
  int model_variant = 0;
  bool team_pairs = false;  // the lane-team kernel solves self-contacts (gs_team.hip)
  // the asset-wide (uniform) drive / limit flags; a bound per-actor property table overrides them in dp
  int uni_any_drive = 0, uni_any_limits = 0;
  // the runtime-sized kernel (gs_generic.hip, kernel_variant 4): the topology entry it stands in for and its
  // candidate tables on the device
  TopoEntry gen_entry{};
  GenTopo* d_gen = nullptr;
  int env_any_drive = 0, env_any_limits = 0;
  DevModel* d_model = nullptr;
  DevModel h_model{};             // host copy (sensors are added after set_model)
  DevLinks* d_links = nullptr;    // link kinematics tables (gs_kinematics.hip)
  int nr = 0, nv = 0;
  std::vector<int> parent;
  float* sens = nullptr;          // [6*nsens][N]
  int nb = 0, nd = 0, nc = 0, ns = 0;
  int N = 0;
  float* state = nullptr;
  const float* mu = nullptr;
  float* cf = nullptr;
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  float4* d_tverts = nullptr;     // terrain mesh (gs_terrain.h)
  uint4* d_tcells = nullptr;
  float* d_tblk = nullptr;        // highest cell top per TERRAIN_BLK x TERRAIN_BLK block of cells
  float* d_tsq4 = nullptr;        // highest cell top of the 4 x 4 cells starting at each cell
  float4* d_trec = nullptr;       // cell records: vertices + face normals (gs_terrain.h TERRAIN_REC)
  float* d_rows = nullptr;        // contact-row tiles of the GLOBAL-row kernels (TopoEntry::row_floats)
  size_t rows_cap = 0;            // floats allocated
  // host backend (device < 0)
  bool host = false;
  HostPool* pool = nullptr;
  const HostTopoEntry* htopo = nullptr;
  DevLinks h_links{};
  std::vector<float4> h_tverts;
  std::vector<uint4> h_tcells;
  std::vector<float> h_tblk;
  std::vector<float> h_tsq4;
  std::vector<float4> h_trec;
  double host_ms = -1.0;          // wall time of the last simulate / pd_step (timing enabled)
  const DevModel* model() const { return host ? &h_model : d_model; }
  const DevLinks* links() const { return host ? &h_links : d_links; }
};

extern "C" {

int gs_abi_version(void) { return GS_ABI_VERSION; }
const char* gs_last_error(void) { return g_err.c_str(); }

int gs_topology_supported(const gs_model_desc* model) { return find_topology(model) != nullptr; }

gs_sim* gs_sim_create(int device, const gs_sim_params* p) {
  if (!p) { fail("gs_sim_create: null params"); return nullptr; }
  if (!(p->dt > 0)) { fail("gs_sim_create: dt must be > 0"); return nullptr; }
  gs_sim* s = nullptr;
  if (device < 0) {
    s = new gs_sim();
    s->host = true;
    s->device = -1;
    // physx.num_threads (cfg/config.yaml:30): worker threads; 0 runs the solver on the caller only
    s->pool = host_pool_create(p->num_threads > 0 ? p->num_threads : 1);
  } else {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
      fail("gs_sim_create: no HIP device %s", std::to_string(device).c_str());
      return nullptr;
    }
    if (hipError_t e = hipSetDevice(device); e != hipSuccess) {
      hip_fail(e, "gs_sim_create hipSetDevice");
      return nullptr;
    }
    s = new gs_sim();
    s->device = device;
  }
  s->params = *p;
  const int sub = p->substeps > 0 ? p->substeps : 1;
  s->dp.h = (float)(p->dt / sub);
  s->dp.substeps = sub;
  for (int k = 0; k < 3; ++k) s->dp.g[k] = (float)p->gravity[k];
  s->dp.pos_iters = p->num_position_iterations;
  s->dp.vel_iters = p->num_velocity_iterations;
  s->dp.contact_offset = (float)p->contact_offset;
  s->dp.rest_offset = (float)p->rest_offset;
  s->dp.max_depen_vel = (float)p->max_depenetration_velocity;
  s->dp.tgs = p->solver_type == 1 && p->num_position_iterations > 0 ? 1 : 0;
  s->dp.collect = p->contact_collection != 0;
  s->dp.limit_margin = (float)(p->joint_limit_margin > 0 ? p->joint_limit_margin : 0.0);
  s->dp.any_limits = 0;
  s->dp.has_ground = 0;
  s->dp.ground_mu = 1.f;
  return s;
}

void gs_sim_destroy(gs_sim* s) {
  if (!s) return;
  if (s->host) {
    host_pool_destroy(s->pool);
    delete s;
    return;
  }
  // Teardown is best-effort: a failed free cannot be reported through a void API.
  (void)hipSetDevice(s->device);
  if (s->d_model) (void)hipFree(s->d_model);
  if (s->d_links) (void)hipFree(s->d_links);
  if (s->d_tverts) (void)hipFree(s->d_tverts);
  if (s->d_tcells) (void)hipFree(s->d_tcells);
  if (s->d_tblk) (void)hipFree(s->d_tblk);
  if (s->d_tsq4) (void)hipFree(s->d_tsq4);
  if (s->d_trec) (void)hipFree(s->d_trec);
  if (s->d_rows) (void)hipFree(s->d_rows);
  if (s->d_gen) (void)hipFree(s->d_gen);
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  delete s;
}

int gs_sim_add_ground(gs_sim* s, double static_friction, double dynamic_friction, double restitution) {
  if (!s) return fail("gs_sim_add_ground: null sim");
  (void)dynamic_friction;
  (void)restitution;
  s->has_ground = true;
  s->dp.has_ground = 1;
  s->dp.ground_mu = (float)static_friction;
  return 0;
}

int gs_sim_add_triangle_mesh(gs_sim* s, const float* vertices, int64_t num_vertices, const uint32_t* triangles,
                             int64_t num_triangles, const double* transform_p, double static_friction,
                             double dynamic_friction, double restitution) {
  (void)dynamic_friction;
  (void)restitution;
  if (!s || !vertices || !triangles) return fail("gs_sim_add_triangle_mesh: null argument");
  if (s->topo) return fail("gs_sim_add_triangle_mesh: call before the model is set (prepare_sim)");
  if (s->d_tverts) return fail("gs_sim_add_triangle_mesh: one triangle mesh per sim");
  if (num_triangles < 2) return fail("gs_sim_add_triangle_mesh: empty mesh");
  // grid shape from the first triangle (v[0,0], v[1,1], v[0,1]) = (0, cols + 1, 1)
  const int64_t cols = (int64_t)triangles[1] - 1;
  if (triangles[0] != 0 || triangles[2] != 1 || cols < 2 || num_vertices % cols != 0)
    return fail("gs_sim_add_triangle_mesh: not a heightfield grid mesh (first triangle)");
  const int64_t rows = num_vertices / cols;
  if (rows < 2 || num_triangles != 2 * (rows - 1) * (cols - 1))
    return fail("gs_sim_add_triangle_mesh: triangle count does not match a %s grid",
                (std::to_string(rows) + "x" + std::to_string(cols)).c_str());
  if (rows > (1 << 24) || cols > (1 << 24)) return fail("gs_sim_add_triangle_mesh: grid too large");
  for (int64_t i = 0; i + 1 < rows; ++i) {
    for (int64_t j = 0; j + 1 < cols; ++j) {
      const int64_t b = i * cols + j, t = 2 * (i * (cols - 1) + j);
      const uint32_t* a = triangles + 3 * t;
      if (a[0] != b || a[1] != b + cols + 1 || a[2] != b + 1 || a[3] != b || a[4] != b + cols || a[5] != b + cols + 1)
        return fail("gs_sim_add_triangle_mesh: triangle %s does not follow the heightfield grid layout",
                    std::to_string(t).c_str());
    }
  }
  // spacing: the grid points are x = i*hs, y = j*hs before the transform.  Slope correction moves a
  // vertex by up to one cell, so take the median over columns of the first-to-last-row span / (rows - 1):
  // a median single-row step carries the float32 rounding of the coordinates (1.5e-5 m at 160 m), which
  // accumulated over 2000 cells misplaces the far end of the 1200 x 2000 AnymalTerrain map by 0.2 cells
  std::vector<double> spans;
  for (int64_t j = 0; j < cols && spans.size() < 4096; j += std::max<int64_t>(1, cols / 1024))
    spans.push_back((double)vertices[3 * ((rows - 1) * cols + j)] - (double)vertices[3 * j]);
  std::sort(spans.begin(), spans.end());
  double hs = spans[spans.size() / 2] / (double)(rows - 1);
  if (!(hs > 0)) return fail("gs_sim_add_triangle_mesh: cannot infer the grid spacing");
  const double tx = transform_p ? transform_p[0] : 0.0, ty = transform_p ? transform_p[1] : 0.0,
               tz = transform_p ? transform_p[2] : 0.0;
  // grid point (0, 0): vertices of row 0 / column 0 can only move inward, so take the minimum
  double x0 = vertices[0], y0 = vertices[1];
  for (int64_t j = 0; j < cols; ++j) x0 = std::min(x0, (double)vertices[3 * j]);
  for (int64_t i = 0; i < rows; ++i) y0 = std::min(y0, (double)vertices[3 * (i * cols) + 1]);
  std::vector<float4> hv((size_t)(rows * cols));
  for (int64_t i = 0; i < rows; ++i) {
    for (int64_t j = 0; j < cols; ++j) {
      const float* v = vertices + 3 * (i * cols + j);
      const double gx = x0 + i * hs, gy = y0 + j * hs;
      if (std::fabs(v[0] - gx) > 1.001 * hs || std::fabs(v[1] - gy) > 1.001 * hs)
        return fail("gs_sim_add_triangle_mesh: a vertex lies more than one cell from its grid point");
      hv[(size_t)(i * cols + j)] = make_float4((float)(v[0] + tx), (float)(v[1] + ty), (float)(v[2] + tz), 0.f);
    }
  }
  std::vector<uint4> hc((size_t)((rows - 1) * (cols - 1)));
  for (int64_t i = 0; i + 1 < rows; ++i) {
    for (int64_t j = 0; j + 1 < cols; ++j) {
      const float4 q[4] = {hv[i * cols + j], hv[i * cols + j + 1], hv[(i + 1) * cols + j], hv[(i + 1) * cols + j + 1]};
      float zmax = q[0].z, zmin = q[0].z, xmin = q[0].x, xmax = q[0].x, ymin = q[0].y, ymax = q[0].y;
      for (int k = 1; k < 4; ++k) {
        zmax = std::max(zmax, q[k].z);
        zmin = std::min(zmin, q[k].z);
        xmin = std::min(xmin, q[k].x); xmax = std::max(xmax, q[k].x);
        ymin = std::min(ymin, q[k].y); ymax = std::max(ymax, q[k].y);
      }
      const double cx0 = x0 + tx + i * hs, cy0 = y0 + ty + j * hs;
      uint32_t f = 0;
      if (xmin < cx0 - 0.25 * hs) f |= TCELL_XLO;
      if (xmax > cx0 + 1.25 * hs) f |= TCELL_XHI;
      if (ymin < cy0 - 0.25 * hs) f |= TCELL_YLO;
      if (ymax > cy0 + 1.25 * hs) f |= TCELL_YHI;
      // the extents beyond the cell square, rounded up to hs / TCELL_EXT_UNITS (gs_terrain.h)
      auto ext = [&](double d) -> uint32_t {
        return (uint32_t)std::min(255.0, std::ceil(std::max(0.0, d) / hs * TCELL_EXT_UNITS));
      };
      const uint32_t ew = ext(cx0 - xmin) | ext(xmax - (cx0 + hs)) << 8 | ext(cy0 - ymin) << 16 |
                          ext(ymax - (cy0 + hs)) << 24;
      uint32_t zb, zl;
      std::memcpy(&zb, &zmax, 4);
      std::memcpy(&zl, &zmin, 4);
      hc[(size_t)(i * (cols - 1) + j)] = make_uint4(zb, f, zl, ew);
    }
  }
  // block summary for the query's first cull (gs_terrain.h sphere_contact): the highest cell top of each block
  const int64_t brows = (rows - 1 + TERRAIN_BLK - 1) / TERRAIN_BLK, bcols = (cols - 1 + TERRAIN_BLK - 1) / TERRAIN_BLK;
  std::vector<float> hb((size_t)(brows * bcols), -3.0e38f);
  for (int64_t i = 0; i + 1 < rows; ++i)
    for (int64_t j = 0; j + 1 < cols; ++j) {
      float top;
      std::memcpy(&top, &hc[(size_t)(i * (cols - 1) + j)].x, 4);
      float& b = hb[(size_t)((i / TERRAIN_BLK) * bcols + j / TERRAIN_BLK)];
      b = std::max(b, top);
    }
  // 4 x 4 square maxima (clipped at the grid's end): row-wise maxima of 4, then column-wise
  const int64_t cr = rows - 1, cc = cols - 1;
  std::vector<float> h4((size_t)(cr * cc)), hq((size_t)(cr * cc));
  for (int64_t i = 0; i < cr; ++i)
    for (int64_t j = 0; j < cc; ++j) {
      float m = -3.0e38f;
      for (int64_t d = 0; d < 4 && j + d < cc; ++d) {
        float top;
        std::memcpy(&top, &hc[(size_t)(i * cc + j + d)].x, 4);
        m = std::max(m, top);
      }
      h4[(size_t)(i * cc + j)] = m;
    }
  for (int64_t i = 0; i < cr; ++i)
    for (int64_t j = 0; j < cc; ++j) {
      float m = -3.0e38f;
      for (int64_t d = 0; d < 4 && i + d < cr; ++d) m = std::max(m, h4[(size_t)((i + d) * cc + j)]);
      hq[(size_t)(i * cc + j)] = m;
    }
  // cell records (gs_terrain.h TERRAIN_REC): the four vertices, the unit normals of the cell's triangles
  // (v00, v11, v01) and (v00, v10, v11) in double from the float vertices; degenerate or downward-facing: (0, 0, -1)
  std::vector<float4> hr((size_t)(cr * cc * TERRAIN_REC));
  for (int64_t i = 0; i < cr; ++i)
    for (int64_t j = 0; j < cc; ++j) {
      const float4 q00 = hv[i * cols + j], q01 = hv[i * cols + j + 1], q10 = hv[(i + 1) * cols + j],
                   q11 = hv[(i + 1) * cols + j + 1];
      auto normal = [](const float4& a, const float4& b, const float4& c, float* nf) {
        const double e1[3] = {(double)b.x - a.x, (double)b.y - a.y, (double)b.z - a.z};
        const double e2[3] = {(double)c.x - a.x, (double)c.y - a.y, (double)c.z - a.z};
        const double x[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double l2 = x[0] * x[0] + x[1] * x[1] + x[2] * x[2];
        nf[0] = 0.f; nf[1] = 0.f; nf[2] = -1.f;
        if (!(l2 > 1e-14)) return;
        const double il = 1.0 / std::sqrt(l2);
        if (x[2] * il < (double)TERRAIN_DOWN_NZ) return;
        for (int k = 0; k < 3; ++k) nf[k] = (float)(x[k] * il);
      };
      float n0[3], n1[3];
      normal(q00, q11, q01, n0);
      normal(q00, q10, q11, n1);
      float4* r = &hr[(size_t)((i * cc + j) * TERRAIN_REC)];
      r[0] = make_float4(q00.x, q00.y, q00.z, n0[0]);
      r[1] = make_float4(q01.x, q01.y, q01.z, n0[1]);
      r[2] = make_float4(q10.x, q10.y, q10.z, n0[2]);
      r[3] = make_float4(q11.x, q11.y, q11.z, n1[0]);
      r[4] = make_float4(n1[1], n1[2], 0.f, 0.f);
    }
  TerrainDev& T = s->dp.terr;
  if (s->host) {
    s->h_tverts = std::move(hv);
    s->h_tcells = std::move(hc);
    s->h_tblk = std::move(hb);
    s->h_tsq4 = std::move(hq);
    s->h_trec = std::move(hr);
    T.rec = s->h_trec.data();
    T.v = s->h_tverts.data();
    T.cell = s->h_tcells.data();
    T.blk = s->h_tblk.data();
    T.sq4 = s->h_tsq4.data();
  } else {
    float4* dv = nullptr;
    uint4* dc = nullptr;
    float* db = nullptr;
    float* dq = nullptr;
    float4* dr = nullptr;
    hipError_t e = hipSetDevice(s->device);
    if (e == hipSuccess) e = hipMalloc(&dv, hv.size() * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&dc, hc.size() * sizeof(uint4));
    if (e == hipSuccess) e = hipMalloc(&db, hb.size() * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&dq, hq.size() * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(dv, hv.data(), hv.size() * sizeof(float4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dc, hc.data(), hc.size() * sizeof(uint4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(db, hb.data(), hb.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dq, hq.data(), hq.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&dr, hr.size() * sizeof(float4));
    if (e == hipSuccess) e = hipMemcpy(dr, hr.data(), hr.size() * sizeof(float4), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (dr) (void)hipFree(dr);
      if (dv) (void)hipFree(dv);
      if (dc) (void)hipFree(dc);
      if (db) (void)hipFree(db);
      if (dq) (void)hipFree(dq);
      return hip_fail(e, "gs_sim_add_triangle_mesh");
    }
    s->d_tverts = dv;
    s->d_tcells = dc;
    s->d_tblk = db;
    s->d_tsq4 = dq;
    s->d_trec = dr;
    T.rec = s->d_trec;
    T.v = s->d_tverts;
    T.cell = s->d_tcells;
    T.blk = s->d_tblk;
    T.sq4 = s->d_tsq4;
  }
  T.bcols = (int)bcols;
  T.rows = (int)rows;
  T.cols = (int)cols;
  T.x0 = (float)(x0 + tx);
  T.y0 = (float)(y0 + ty);
  T.hs = (float)hs;
  T.inv_hs = (float)(1.0 / hs);
  T.mu = (float)static_friction;
  s->dp.has_terrain = 1;
  return 0;
}

int gs_sim_set_model(gs_sim* s, const gs_model_desc* m) {
  if (!s || !m) return fail("gs_sim_set_model: null argument");
  if (m->num_bodies > GS_MAXB || m->num_dofs > GS_MAXD || m->num_candidates > GS_MAXC || m->num_links > GS_MAXL ||
      m->num_shapes > GS_MAXSH)
    return fail("gs_sim_set_model: articulation exceeds compiled maxima (bodies/dofs/candidates/links)");
  if (m->num_links < m->num_bodies || !m->link_body || !m->link_pose || !m->link_com ||
      (m->num_candidates > 0 && !m->cand_link))
    return fail("gs_sim_set_model: link tables missing (gs_model_desc ABI 2: num_links >= num_bodies)");
  for (int l = 0; l < m->num_links; ++l)
    if (m->link_body[l] < 0 || m->link_body[l] >= m->num_bodies) return fail("gs_sim_set_model: link_body out of range");
  for (int c = 0; c < m->num_candidates; ++c)
    if (m->cand_link[c] < 0 || m->cand_link[c] >= m->num_links) return fail("gs_sim_set_model: cand_link out of range");
  const TopoEntry* t = find_topology(m);
  // A topology with no compiled kernel runs the runtime-sized kernel (gs_generic.hip, kernel_variant 4) on the GPU:
  // any tree of revolute / prismatic joints with plane contacts of point candidates (spheres, capsule / cylinder
  // ends, box corners), joint limits and drives.  Hull candidates, self-collision, terrain meshes and force
  // sensors need a compiled topology (tools/gen_topologies.py) and are refused where they are set up.
  // (kernel_variant 4 asks for it on a compiled topology too: the cross-check of the two solver forms)
  const bool generic = !t || (s->params.kernel_variant == 4 && !s->host);
  if (generic) {
    if (s->host)
      return fail("gs_sim_set_model: the runtime-sized kernel is a GPU kernel and no host solver is compiled for "
                  "this topology (add it with tools/gen_topologies.py): %s", signature(m).c_str());
    if (s->params.kernel_variant == 1 || s->params.kernel_variant == 2)
      return fail("gs_sim_set_model: kernel_variant 1 / 2 requested but topology %s is not compiled (the runtime-"
                  "sized kernel is variant 4)", signature(m).c_str());
    for (int c = 0; c < m->num_candidates; ++c)
      if (m->cand_dyn && m->cand_dyn[c] >= 0)
        return fail("gs_sim_set_model: topology %s has convex-hull candidates: the runtime-sized kernel has no hull "
                    "ground manifold (compile the topology with tools/gen_topologies.py)", signature(m).c_str());
    if (s->dp.has_terrain)
      return fail("gs_sim_set_model: topology %s with a terrain mesh: the runtime-sized kernel has plane contacts only "
                  "(compile the topology with tools/gen_topologies.py)", signature(m).c_str());
    if (m->num_dofs + 6 > GS_MAXD + 6 || (m->num_candidates > 0 && !m->cand_shape))
      return fail("gs_sim_set_model: runtime-sized kernel tables missing for %s", signature(m).c_str());
  }
  if (!generic && m->num_pairs > 0 && m->pair_pool != t->npk)
    return fail("gs_sim_set_model: self-contact pool differs from the compiled topology's %s",
                std::to_string(t->npk).c_str());
  for (int c = 0; c < m->num_candidates && !generic; ++c)
    if (m->cand_dyn && m->cand_dyn[c] != t->cdyn[c])
      return fail("gs_sim_set_model: hull slots differ from the compiled topology (tools/gen_topologies.py)");
  // the kernels unroll the self-collision pairs and shape kinds at compile time
  if (!generic && m->num_pairs > 0 && m->num_pairs != t->npair)
    return fail("gs_sim_set_model: self-collision pair count differs from the compiled topology's %s",
                std::to_string(t->npair).c_str());
  for (int q = 0; q < m->num_pairs && !generic; ++q)
    if (m->pair_a[q] != t->pair_a[q] || m->pair_b[q] != t->pair_b[q] || m->pair_kind[q] != t->pair_k[q])
      return fail("gs_sim_set_model: self-collision pairs differ from the compiled topology (tools/gen_topologies.py)");
  for (int sh = 0; sh < m->num_shapes && !generic; ++sh)
    if (m->shape_kind && m->shape_kind[sh] != t->shkind[sh])
      return fail("gs_sim_set_model: shape kinds differ from the compiled topology (tools/gen_topologies.py)");
  // Everything is built into locals first and committed at the end, so a failure leaves the sim as
  // it was (no half-set topology with a null kernel or link table).
  DevModel h;
  std::memset(&h, 0, sizeof(h));
  for (int i = 0; i < m->num_bodies; ++i) {
    for (int k = 0; k < 9; ++k) h.jR[i][k] = (float)m->joint_origin[12 * i + k];
    for (int k = 0; k < 3; ++k) h.jt[i][k] = (float)m->joint_origin[12 * i + 9 + k];
    for (int k = 0; k < 3; ++k) h.jaxis[i][k] = (float)m->joint_axis[3 * i + k];
    h.mass[i] = (float)m->mass[i];
    for (int k = 0; k < 3; ++k) h.com[i][k] = (float)m->com[3 * i + k];
    const double* I = m->inertia + 9 * i;
    h.inertia[i][0] = (float)I[0]; h.inertia[i][1] = (float)I[4]; h.inertia[i][2] = (float)I[8];
    h.inertia[i][3] = (float)I[1]; h.inertia[i][4] = (float)I[2]; h.inertia[i][5] = (float)I[5];
  }
  {  // root link COM in the body-0 frame: link pose (identity for the root link) applied to its COM
    const double* P = m->link_pose;
    const double* c = m->link_com;
    for (int k = 0; k < 3; ++k)
      h.root_com[k] = (float)(P[9 + k] + P[3 * k] * c[0] + P[3 * k + 1] * c[1] + P[3 * k + 2] * c[2]);
  }
  for (int c = 0; c < m->num_candidates; ++c) {
    for (int k = 0; k < 3; ++k) h.cpoint[c][k] = (float)m->cand_point[3 * c + k];
    h.cradius[c] = (float)m->cand_radius[c];
  }
  // shapes (ABI 5): bounding spheres widened by 1e-4 relative so that float rounding never culls an active
  // candidate or pair; hull vertices; self-collision pairs
  if (!m->shape_kind || !m->shape_body || !m->shape_link || !m->shape_pose || !m->shape_size || !m->shape_margin ||
      !m->shape_sphere || !m->shape_hv0 || !m->shape_hv1 || (m->num_candidates > 0 && !m->cand_dyn))
    return fail("gs_sim_set_model: shape tables missing (gs_model_desc ABI 5)");
  if (m->num_hull_verts < 0 || m->num_hull_verts > GS_MAXHV || m->num_pairs < 0 || m->num_pairs > GS_MAXP ||
      (m->num_hull_verts > 0 && !m->hull_verts) || (m->num_pairs > 0 && (!m->pair_a || !m->pair_b || !m->pair_kind)))
    return fail("gs_sim_set_model: hull vertices / self-collision pairs exceed compiled maxima");
  for (int sh = 0; sh < m->num_shapes; ++sh) {
    for (int k = 0; k < 3; ++k) h.shc[sh][k] = (float)m->shape_sphere[4 * sh + k];
    // the sphere must hold the shape's ground candidates too (the solver skips a shape whose sphere clears the
    // ground): a cylinder's candidates are its end points with the cylinder's radius (a capsule to the plane
    // test), which reach hl + r along the axis, beyond the cylinder's own bounding sphere
    // sqrt(hl^2 + r^2) (round 5: a UsefulHound leg cylinder's end 10 mm from the ground was skipped at a 42 mm
    // sphere clearance; the pair broadphase only gets looser by it)
    double reach = m->shape_sphere[4 * sh + 3];
    for (int c = 0; c < m->num_candidates; ++c) {
      if (m->cand_shape && m->cand_shape[c] == sh && m->cand_dyn[c] < 0) {
        double d2 = 0.0;
        for (int k = 0; k < 3; ++k) {
          const double d = m->cand_point[3 * c + k] - m->shape_sphere[4 * sh + k];
          d2 += d * d;
        }
        reach = std::max(reach, std::sqrt(d2) + m->cand_radius[c]);
      }
    }
    h.shc[sh][3] = (float)(reach * (1.0 + 1e-4) + 1e-5);
    h.shkind[sh] = m->shape_kind[sh];
    h.shbody[sh] = m->shape_body[sh];
    h.shlink[sh] = m->shape_link[sh];
    for (int k = 0; k < 9; ++k) h.shR[sh][k] = (float)m->shape_pose[12 * sh + k];
    for (int k = 0; k < 3; ++k) h.sht[sh][k] = (float)m->shape_pose[12 * sh + 9 + k];
    for (int k = 0; k < 3; ++k) h.shsize[sh][k] = (float)m->shape_size[3 * sh + k];
    h.shm[sh] = (float)m->shape_margin[sh];
    h.hv0[sh] = m->shape_hv0[sh];
    h.hv1[sh] = m->shape_hv1[sh];
    if (h.shbody[sh] < 0 || h.shbody[sh] >= m->num_bodies || h.shlink[sh] < 0 || h.shlink[sh] >= m->num_links ||
        h.hv0[sh] < 0 || h.hv1[sh] < h.hv0[sh] || h.hv1[sh] > m->num_hull_verts ||
        (h.shkind[sh] == 4 && h.hv1[sh] == h.hv0[sh]))
      return fail("gs_sim_set_model: shape %s tables out of range", std::to_string(sh).c_str());
  }
  for (int v = 0; v < m->num_hull_verts; ++v)
    for (int k = 0; k < 4; ++k) h.hv[v][k] = (float)m->hull_verts[4 * v + k];
  if (m->num_pair_verts < 0 || m->num_pair_verts > GS_MAXPV || !m->shape_pv0 || !m->shape_pv1 ||
      (m->num_pair_verts > 0 && !m->pair_verts))
    return fail("gs_sim_set_model: hull self-collision cores missing or beyond GS_MAXPV");
  for (int v = 0; v < m->num_pair_verts; ++v)
    for (int k = 0; k < 4; ++k) h.pv[v][k] = (float)m->pair_verts[4 * v + k];
  for (int sh = 0; sh < m->num_shapes; ++sh) {
    h.pv0[sh] = m->shape_pv0[sh];
    h.pv1[sh] = m->shape_pv1[sh];
    if (h.pv0[sh] < 0 || h.pv1[sh] < h.pv0[sh] || h.pv1[sh] > m->num_pair_verts ||
        (h.shkind[sh] == 4 && h.pv1[sh] == h.pv0[sh]))
      return fail("gs_sim_set_model: shape %s self-collision core out of range", std::to_string(sh).c_str());
  }
  for (int c = 0; c < m->num_candidates; ++c)
    if (m->cand_dyn[c] >= 0 && m->shape_kind[m->cand_shape[c]] != 4)
      return fail("gs_sim_set_model: dynamic candidate %s on a shape that is not a hull", std::to_string(c).c_str());
  h.np = m->num_pairs;
  for (int q = 0; q < m->num_pairs; ++q) {
    h.pa[q] = m->pair_a[q];
    h.pb[q] = m->pair_b[q];
    h.pk[q] = m->pair_kind[q];
    if (h.pa[q] < 0 || h.pb[q] <= h.pa[q] || h.pb[q] >= m->num_shapes || h.pk[q] < 0 || h.pk[q] > 3)
      return fail("gs_sim_set_model: self-collision pair %s out of range", std::to_string(q).c_str());
  }
  for (int b = 0; b < m->num_bodies; ++b) {
    unsigned mask = 0;
    for (int a = b; a >= 0; a = m->parent[a]) mask |= 1u << a;
    h.banc[b] = mask;
  }
  int any_lim = 0;
  for (int j = 0; j < m->num_dofs; ++j) {
    h.effort[j] = (float)m->dof_effort[j];
    h.vmax[j] = (float)m->dof_velocity[j];
    h.armature[j] = (float)m->dof_armature[j];
    h.has_lim[j] = m->dof_has_limits && m->dof_has_limits[j] && m->dof_upper[j] > m->dof_lower[j];
    h.lower[j] = h.has_lim[j] ? (float)m->dof_lower[j] : 0.f;
    h.upper[j] = h.has_lim[j] ? (float)m->dof_upper[j] : 0.f;
    any_lim |= h.has_lim[j];
  }
  h.nsens = 0;
  for (int b = 0; b < GS_MAXB; ++b) h.sens_of_body[b] = -1;

  DevLinks hl;
  std::memset(&hl, 0, sizeof(hl));
  hl.nb = m->num_bodies;
  hl.nd = m->num_dofs;
  hl.nr = m->num_links;
  hl.fixed_base = m->fixed_base;
  for (int b = 0; b < m->num_bodies; ++b) {
    hl.parent[b] = m->parent[b];
    hl.jkind[b] = m->joint_kind[b];
    hl.bdof[b] = m->body_dof[b];
    unsigned mask = 0;
    for (int a = b; a >= 0; a = m->parent[a]) mask |= 1u << a;
    hl.anc_mask[b] = mask;
    if (m->body_dof[b] >= 0) hl.dbody[m->body_dof[b]] = b;
  }
  for (int l = 0; l < m->num_links; ++l) {
    hl.lbody[l] = m->link_body[l];
    for (int k = 0; k < 9; ++k) hl.lR[l][k] = (float)m->link_pose[12 * l + k];
    for (int k = 0; k < 3; ++k) hl.lt[l][k] = (float)m->link_pose[12 * l + 9 + k];
    for (int k = 0; k < 3; ++k) hl.lcom[l][k] = (float)m->link_com[3 * l + k];
  }

  const int want = s->params.kernel_variant;
  launch_sim_fn sim_fn = nullptr;
  launch_pd_fn pd_fn = nullptr;
  const HostTopoEntry* htopo = nullptr;
  int variant = 0;
  GenTopo hg;
  std::memset(&hg, 0, sizeof(hg));
  if (generic) {
    hg.nc = m->num_candidates;
    for (int c = 0; c < m->num_candidates; ++c) {
      hg.cbody[c] = m->cand_body[c];
      hg.cshape[c] = m->cand_shape[c];
      hg.clink[c] = m->cand_link[c];
      if (hg.cbody[c] < 0 || hg.cbody[c] >= m->num_bodies || hg.cshape[c] < 0 || hg.cshape[c] >= m->num_shapes)
        return fail("gs_sim_set_model: candidate %s tables out of range", std::to_string(c).c_str());
    }
    TopoEntry& g = s->gen_entry;
    g = TopoEntry{};
    g.sig = "runtime";
    g.name = "runtime-sized (gs_generic.hip)";
    g.sim = launch_sim_generic;
    g.pd = launch_pd_generic;
    g.dbg_pool = nullptr;
    g.nb = m->num_bodies; g.nd = m->num_dofs; g.nc = m->num_candidates; g.ns = m->num_shapes;
    g.sens = 0;
    g.row_floats = (int)generic_ws_floats(m->num_candidates, m->num_dofs, m->fixed_base);
    g.row_lanes = 1;
    g.npk = 0;
    g.npair = 0;
    t = &g;
  }
  if (s->host) {
    for (int i = 0; i < g_num_host_topologies; ++i)
      if (std::strcmp(g_host_topologies[i].sig, t->sig) == 0) htopo = &g_host_topologies[i];
    if (!htopo) return fail("gs_sim_set_model: no host solver for topology %s", t->sig);
    if (want == 2) return fail("gs_sim_set_model: the lane-team kernel is a GPU kernel (host sim)");
    variant = 3;
  } else {
    const TeamEntry* te = nullptr;
    for (int i = 0; i < g_num_team_kernels; ++i)
      if (std::strcmp(g_team_kernels[i].sig, t->sig) == 0 && g_team_kernels[i].sim) te = &g_team_kernels[i];
    // the lane team has no joint-limit rows: the one-env-per-lane kernel runs (a trimesh terrain runs the lane
    // team's TERR form; kernel_variant 1 still selects the one-env-per-lane kernel)
    if (te && any_lim) te = nullptr;
    if (want == 2 && !te)
      return fail("gs_sim_set_model: no lane-team kernel for this topology / joint limits");
    if (generic) {
      sim_fn = launch_sim_generic;
      pd_fn = launch_pd_generic;
      variant = 4;
    } else if (te && want != 1) {
      sim_fn = te->sim;
      pd_fn = te->pd;
      variant = 2;
    } else {
      sim_fn = t->sim;
      pd_fn = t->pd;
      variant = 1;
    }
    if (hipError_t e = hipSetDevice(s->device); e != hipSuccess) return hip_fail(e, "gs_sim_set_model hipSetDevice");
    DevModel* dm = s->d_model;
    DevLinks* dl = s->d_links;
    hipError_t e = hipSuccess;
    if (!dm) e = hipMalloc(&dm, sizeof(DevModel));
    if (e == hipSuccess && !dl) e = hipMalloc(&dl, sizeof(DevLinks));
    // keep whatever was allocated (freed by gs_sim_destroy) even when a later step fails
    s->d_model = dm;
    s->d_links = dl;
    if (e == hipSuccess) e = hipMemcpy(dm, &h, sizeof(DevModel), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dl, &hl, sizeof(DevLinks), hipMemcpyHostToDevice);
    if (e == hipSuccess && generic && !s->d_gen) e = hipMalloc(&s->d_gen, sizeof(GenTopo));
    if (e == hipSuccess && generic) e = hipMemcpy(s->d_gen, &hg, sizeof(GenTopo), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "gs_sim_set_model upload");
  }
  // commit
  s->h_model = h;
  s->h_links = hl;
  s->dp.any_limits = any_lim;
  s->uni_any_limits = any_lim;
  s->parent.assign(m->parent, m->parent + m->num_bodies);
  s->sim_fn = sim_fn;
  s->pd_fn = pd_fn;
  s->htopo = htopo;
  s->variant = variant;
  s->model_sim_fn = sim_fn;
  s->model_pd_fn = pd_fn;
  s->model_variant = variant;
  s->team_pairs = variant == 2;  // the lane-team kernel solves self-contacts (gs_team.hip team_self_contacts)
  s->nr = m->num_links;
  s->nv = (m->fixed_base ? 0 : 6) + m->num_dofs;
  s->nb = m->num_bodies;
  s->nd = m->num_dofs;
  s->nc = m->num_candidates;
  s->ns = m->num_shapes;
  s->topo = t;
  s->dp.gen = generic ? s->d_gen : nullptr;
  s->dp.gen_links = generic ? s->d_links : nullptr;
  s->dp.gen_nd = m->num_dofs;
  s->dp.gen_nr = m->num_links;
  return 0;
}

int gs_sim_prepare(gs_sim* s, int num_envs, float* state, const float* shape_friction, float* contact) {
  if (!s || !s->topo) return fail("gs_sim_prepare: model not set");
  if (num_envs <= 0 || !state || !shape_friction || !contact) return fail("gs_sim_prepare: bad buffers");
  s->N = num_envs;
  s->state = state;
  s->mu = shape_friction;
  s->cf = contact;
  return 0;
}

static SimBuffers buffers(gs_sim* s) { return SimBuffers{s->state, s->mu, s->cf, s->N, s->sens, s->d_rows}; }

// floats of contact-row tiles the selected GPU kernel needs for N envs (0: its rows live in LDS)
static size_t rows_needed(const gs_sim* s) {
  if (s->host || !s->topo || (s->variant != 1 && s->variant != 4) || (s->variant == 1 && s->dp.has_terrain) ||
      s->topo->row_floats <= 0 || s->N <= 0)
    return 0;
  const size_t lanes = (size_t)s->topo->row_lanes;
  return ((size_t)s->N + lanes - 1) / lanes * lanes * (size_t)s->topo->row_floats;
}

static int ready(gs_sim* s, const char* where) {
  if (!s || !s->topo || !s->state) return fail("%s: sim not prepared", where);
  if (s->host ? !s->htopo : (!s->sim_fn || !s->pd_fn || !s->d_model || !s->d_links))
    return fail("%s: sim model incomplete", where);
  if (const size_t need = rows_needed(s); need > s->rows_cap) {
    // first step of an LDS-starved topology (or more envs than before): the row tiles, once
    if (hipError_t e = hipSetDevice(s->device); e != hipSuccess) return hip_fail(e, where);
    if (s->d_rows) (void)hipFree(s->d_rows);
    s->d_rows = nullptr;
    s->rows_cap = 0;
    if (hipError_t e = hipMalloc(&s->d_rows, need * sizeof(float)); e != hipSuccess) {
      s->d_rows = nullptr;
      return hip_fail(e, where);
    }
    s->rows_cap = need;
  }
  return 0;
}

static void timing_begin(gs_sim* s, hipStream_t st) {
  if (!s->timing || s->host) return;
  if (!s->ev0) {
    // Timing is diagnostic: if the events cannot be made, switch it off rather than fail the step.
    if (hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess) {
      s->timing = false;
      return;
    }
  }
  (void)hipEventRecord(s->ev0, st);
}
static void timing_end(gs_sim* s, hipStream_t st) {
  if (!s->timing || s->host) return;
  s->timed = hipEventRecord(s->ev1, st) == hipSuccess;
}

namespace {
using host_clock = std::chrono::steady_clock;
double ms_since(host_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(host_clock::now() - t0).count();
}
}  // namespace

int gs_sim_simulate(gs_sim* s, const float* dof_force, void* stream) {
  if (ready(s, "gs_sim_simulate")) return -1;
  if (s->host) {
    const auto t0 = host_clock::now();
    s->htopo->sim(&s->h_model, s->dp, buffers(s), dof_force, s->pool);
    s->host_ms = ms_since(t0);
    return 0;
  }
  hipStream_t st = (hipStream_t)stream;
  timing_begin(s, st);
  hipError_t e = s->sim_fn(s->d_model, s->dp, buffers(s), dof_force, st);
  timing_end(s, st);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_simulate");
}

int gs_sim_pd_step(gs_sim* s, const gs_pd_args* a, void* stream) {
  if (ready(s, "gs_sim_pd_step")) return -1;
  if (!a || !a->actions || !a->default_pos || !a->torques_out || !a->dof_state_out)
    return fail("gs_sim_pd_step: actions/default_pos/torques_out/dof_state_out required");
  PdDev d;
  d.actions = a->actions;
  d.dof_state_in = a->dof_state_out;
  d.default_pos = a->default_pos;
  d.kp = a->kp; d.kd = a->kd; d.scale = a->action_scale; d.tlim = a->torque_limit;
  d.decimation = a->decimation;
  d.extra = a->extra_simulates;
  d.torques_out = a->torques_out;
  d.dof_out = a->dof_state_out;
  d.root_out = a->root_state_out;
  d.cf_out = a->contact_out;
  d.actions_copy = a->actions_copy_out;
  d.tail_on = 0;
  if (a->tail_params || a->tail_buffers) {
    // the AnymalTerrain tail in the team kernel's last phase (gymsim.h ABI 9): the checks gt_anymal_post_physics_a
    // makes, post_a's vector rows, and the buffers the kernel has just written being the tail's inputs
    const gt_anymal_params* tp = a->tail_params;
    const gt_anymal_buffers* tb = a->tail_buffers;
    auto aligned = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
    if (!gs_sim_pd_tail_supported(s)) return fail("gs_sim_pd_step: this sim's kernel has no fused tail");
    if (!tp || !tb || tb->hound || tp->num_envs != s->N || tp->num_dofs != s->nd || tp->num_dofs % 4 != 0 ||
        tp->num_bodies != s->nr || tp->num_feet > 4 || tp->num_knees > 4 || tp->num_feet < 0 || tp->num_knees < 0 ||
        tp->base_index < 0 || tp->base_index >= s->nr || !tb->reset_count || !tb->reset_masks || !tb->reset_buf ||
        !tb->timeout_buf || !tb->rew_buf || !tb->episode_sums || !tb->base_lin_vel || !tb->base_ang_vel ||
        !tb->projected_gravity || !tb->progress_buf || !tb->randomize_buf || !tb->commands || !tb->feet_air_time ||
        !tb->last_actions || !tb->last_dof_vel)
      return fail("gs_sim_pd_step: invalid tail parameters / buffers");
    for (int k = 0; k < tp->num_feet; ++k)
      if (tp->feet_idx[k] < 0 || tp->feet_idx[k] >= s->nr) return fail("gs_sim_pd_step: tail foot index");
    for (int k = 0; k < tp->num_knees; ++k)
      if (tp->knee_idx[k] < 0 || tp->knee_idx[k] >= s->nr) return fail("gs_sim_pd_step: tail knee index");
    if (tb->torques != a->torques_out || tb->actions != a->actions_copy_out || tb->root_states != a->root_state_out ||
        tb->contact_forces != a->contact_out || tb->dof_state != a->dof_state_out)
      return fail("gs_sim_pd_step: the tail must read this call's outputs");
    if (!aligned(tb->torques) || !aligned(tb->actions) || !aligned(tb->last_actions) || !aligned(tb->last_dof_vel) ||
        !aligned(tb->dof_state))
      return fail("gs_sim_pd_step: the tail's dof rows must be 16-byte aligned");
    d.tail_on = 1;
    d.tail_p = *tp;
    d.tail_b = *tb;
  }
  if (s->host) {
    const auto t0 = host_clock::now();
    s->htopo->pd(&s->h_model, s->dp, buffers(s), d, s->pool);
    s->host_ms = ms_since(t0);
    return 0;
  }
  hipStream_t st = (hipStream_t)stream;
  timing_begin(s, st);
  hipError_t e = s->pd_fn(s->d_model, s->dp, buffers(s), d, st);
  timing_end(s, st);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_pd_step");
}

int gs_sim_refresh_root(gs_sim* s, float* out, void* stream) {
  if (ready(s, "gs_sim_refresh_root")) return -1;
  if (s->host) {
    host_refresh_root(s->state, s->N, &s->h_model.root_com[0], out, s->pool);
    return 0;
  }
  hipError_t e = launch_refresh_root(s->state, s->N, s->nd, &s->d_model->root_com[0], out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_refresh_root");
}
int gs_sim_refresh_dof(gs_sim* s, float* out, void* stream) {
  if (ready(s, "gs_sim_refresh_dof")) return -1;
  if (s->host) {
    host_refresh_dof(s->state, s->N, s->nd, out, s->pool);
    return 0;
  }
  hipError_t e = launch_refresh_dof(s->state, s->N, s->nd, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_refresh_dof");
}
int gs_sim_refresh_contact(gs_sim* s, float* out, void* stream) {
  if (ready(s, "gs_sim_refresh_contact")) return -1;
  if (s->host) {
    host_soa_to_aos(s->cf, s->N, s->nr, 3, out, s->pool);
    return 0;
  }
  hipError_t e = launch_refresh_contact(s->cf, s->N, s->nr, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_refresh_contact");
}
static int kinematics(gs_sim* s, int mode, float* rb, float* jac, float* mm, void* stream, const char* where) {
  if (ready(s, where)) return -1;
  if (!rb && !jac && !mm) return fail("%s: null output", where);
  if (s->host) {
    host_kinematics(&s->h_model, &s->h_links, s->state, s->N, s->nv, mode, rb, jac, mm, s->pool);
    return 0;
  }
  hipError_t e = launch_kinematics(s->d_model, s->d_links, s->state, s->N, s->nv, mode, rb, jac, mm,
                                   (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, where);
}
int gs_sim_refresh_rigid_body(gs_sim* s, float* out, void* stream) {
  return kinematics(s, 1, out, nullptr, nullptr, stream, "gs_sim_refresh_rigid_body");
}
int gs_sim_refresh_jacobian(gs_sim* s, float* out, void* stream) {
  return kinematics(s, 2, nullptr, out, nullptr, stream, "gs_sim_refresh_jacobian");
}
int gs_sim_refresh_mass_matrix(gs_sim* s, float* out, void* stream) {
  return kinematics(s, 4, nullptr, nullptr, out, stream, "gs_sim_refresh_mass_matrix");
}
int gs_sim_set_root(gs_sim* s, const float* src, const int32_t* idx, int n_idx, void* stream) {
  if (ready(s, "gs_sim_set_root")) return -1;
  if (s->host) {
    host_set_root(s->state, s->N, &s->h_model.root_com[0], src, idx, idx ? n_idx : s->N);
    return 0;
  }
  hipError_t e = launch_set_root(s->state, s->N, s->nd, &s->d_model->root_com[0], src, idx, n_idx,
                                 (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_set_root");
}
int gs_sim_set_dof(gs_sim* s, const float* src, const int32_t* idx, int n_idx, void* stream) {
  if (ready(s, "gs_sim_set_dof")) return -1;
  if (s->host) {
    host_set_dof(s->state, s->N, s->nd, src, idx, idx ? n_idx : s->N);
    return 0;
  }
  hipError_t e = launch_set_dof(s->state, s->N, s->nd, src, idx, n_idx, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_set_dof");
}

int gs_sim_set_root_and_dof(gs_sim* s, const float* root, const float* dof, const int32_t* idx, int n_idx,
                            void* stream) {
  if (ready(s, "gs_sim_set_root_and_dof")) return -1;
  if (!root || !dof || !idx || n_idx < 0) return fail("gs_sim_set_root_and_dof: root, dof and idx required");
  if (s->host) {
    host_set_root(s->state, s->N, &s->h_model.root_com[0], root, idx, n_idx);
    host_set_dof(s->state, s->N, s->nd, dof, idx, n_idx);
    return 0;
  }
  hipError_t e = launch_set_root_dof(s->state, s->N, s->nd, &s->d_model->root_com[0], root, dof, idx, n_idx,
                                     (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_set_root_and_dof");
}

int gs_sim_set_force_sensors(gs_sim* s, int n, const int32_t* bodies) {
  if (!s || !s->topo) return fail("gs_sim_set_force_sensors: model not set");
  if (s->state) return fail("gs_sim_set_force_sensors: call before gs_sim_prepare");
  if (n < 0 || n > GS_MAXS || (n > 0 && !bodies)) return fail("gs_sim_set_force_sensors: at most 8 sensors");
  if (n > 0 && s->variant == 2)
    return fail("gs_sim_set_force_sensors: the lane-team kernel has no force sensors (use kernel_variant 1)");
  if (n > 0 && s->variant == 4)
    return fail("gs_sim_set_force_sensors: the runtime-sized kernel has no force sensors (compile the topology)");
  if (n > 0 && !s->topo->sens)
    return fail("gs_sim_set_force_sensors: topology %s is compiled without force sensors (sensors flag in "
                "tools/gen_topologies.py MODELS)", s->topo->name);
  DevModel& h = s->h_model;
  for (int b = 0; b < GS_MAXB; ++b) h.sens_of_body[b] = -1;
  for (int i = 0; i < n; ++i) {
    const int b = bodies[i];
    if (b <= 0 || b >= s->nb) return fail("gs_sim_set_force_sensors: sensor body out of range (or the root)");
    for (int c = 0; c < s->nb; ++c)
      if (s->parent[c] == b) return fail("gs_sim_set_force_sensors: sensors on non-leaf bodies are not supported");
    if (h.sens_of_body[b] >= 0) return fail("gs_sim_set_force_sensors: two sensors on one body");
    h.sens_of_body[b] = i;
  }
  h.nsens = n;
  if (s->host) return 0;
  hipError_t e = hipSetDevice(s->device);
  if (e == hipSuccess) e = hipMemcpy(s->d_model, &h, sizeof(DevModel), hipMemcpyHostToDevice);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_set_force_sensors hipMemcpy");
}

// The kernel form for the sim's current features: the one gs_sim_set_model selected, or the one-env-per-lane
// kernel where the lane team lacks a feature in use (joint drives, a per-actor dof property table)
static int kernel_select(gs_sim* s, const char* who) {
  launch_sim_fn sim_fn = s->model_sim_fn;
  launch_pd_fn pd_fn = s->model_pd_fn;
  int variant = s->model_variant;
  const bool lane = s->dp.any_drive || s->dp.dof_env || (s->dp.self_collide && !s->team_pairs);
  if (lane && variant == 2) {  // (the runtime-sized kernel, variant 4, has drives and per-actor properties)
    if (s->params.kernel_variant == 2)
      return fail("%s: the lane-team kernel (kernel_variant 2) has no joint drives or per-actor dof properties", who);
    sim_fn = s->topo->sim;
    pd_fn = s->topo->pd;
    variant = 1;
  }
  s->sim_fn = sim_fn;
  s->pd_fn = pd_fn;
  s->variant = variant;
  return 0;
}

int gs_sim_set_dof_drives(gs_sim* s, const int32_t* mode, const double* stiffness, const double* damping) {
  if (!s || !s->topo) return fail("gs_sim_set_dof_drives: model not set");
  if (s->nd > 0 && (!mode || !stiffness || !damping)) return fail("gs_sim_set_dof_drives: null argument");
  DevModel h = s->h_model;
  int any = 0;
  for (int j = 0; j < s->nd; ++j) {
    // gymapi.DofDriveMode: 1 POS (stiffness, damping), 2 VEL (damping); NONE / EFFORT: no drive
    const double kp = mode[j] == 1 ? stiffness[j] : 0.0;
    const double kd = (mode[j] == 1 || mode[j] == 2) ? damping[j] : 0.0;
    if (!(kp >= 0.0) || !(kd >= 0.0)) return fail("gs_sim_set_dof_drives: negative or NaN drive gain");
    h.dkp[j] = (float)kp;
    h.dkd[j] = (float)kd;
    any |= (kp > 0.0 || kd > 0.0);
  }
  // the lane-team kernel has no drive terms: drives run the one-env-per-lane kernel; the kernel
  // gs_sim_set_model selected comes back once every gain is zero again
  if (any && s->model_variant == 2 && s->params.kernel_variant == 2)
    return fail("gs_sim_set_dof_drives: the lane-team kernel (kernel_variant 2) has no joint drives");
  if (!s->host) {
    // the physics kernels read d_model: the blocking upload must not overtake a launch still queued on
    // a caller's (non-blocking) stream, so the device drains first (cold path: dof property changes)
    hipError_t e = hipSetDevice(s->device);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(s->d_model, &h, sizeof(DevModel), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "gs_sim_set_dof_drives hipMemcpy");
  }
  s->h_model = h;
  s->uni_any_drive = any;
  s->dp.any_drive = s->dp.dof_env ? s->env_any_drive : any;
  return kernel_select(s, "gs_sim_set_dof_drives");
}

int gs_sim_set_self_collision(gs_sim* s, int enable) {
  if (!s || !s->topo) return fail("gs_sim_set_self_collision: model not set");
  if (enable && s->h_model.np > 0 && s->topo->npk <= 0)
    return fail("gs_sim_set_self_collision: the compiled topology has no self-contact pool");
  if (enable && s->h_model.np > 0 && s->variant == 4)
    return fail("gs_sim_set_self_collision: the runtime-sized kernel has no self-collision (compile the topology "
                "with tools/gen_topologies.py, or create the actors with collision filter 1)");
  s->dp.self_collide = enable && s->h_model.np > 0;
  if (s->dp.self_collide && s->variant == 2 && !s->team_pairs) {  // this lane-team build has no pair rows
    if (s->params.kernel_variant == 2)
      return fail("gs_sim_set_self_collision: the lane-team kernel (kernel_variant 2) has no self-collision");
    s->sim_fn = s->topo->sim;
    s->pd_fn = s->topo->pd;
    s->variant = 1;
  }
  return 0;
}

int gs_sim_bind_dof_targets(gs_sim* s, const float* pos_targets, const float* vel_targets) {
  if (!s || !s->topo) return fail("gs_sim_bind_dof_targets: model not set");
  s->dp.ptgt = pos_targets;
  s->dp.vtgt = vel_targets;
  return 0;
}

int gs_sim_bind_dof_properties_env(gs_sim* s, const float* table, int any_drive, int any_limits) {
  if (ready(s, "gs_sim_bind_dof_properties_env")) return -1;
  if (table) {
    s->dp.dof_env = table;
    s->dp.dof_env_n = s->N;
    s->env_any_drive = any_drive != 0;
    s->env_any_limits = any_limits != 0;
    s->dp.any_drive = s->env_any_drive;
    s->dp.any_limits = s->env_any_limits;
  } else {
    s->dp.dof_env = nullptr;
    s->dp.dof_env_n = 0;
    s->dp.any_drive = s->uni_any_drive;
    s->dp.any_limits = s->uni_any_limits;
  }
  return kernel_select(s, "gs_sim_bind_dof_properties_env");
}

int gs_sim_bind_force_sensors(gs_sim* s, float* soa) {
  if (ready(s, "gs_sim_bind_force_sensors")) return -1;
  if (s->h_model.nsens > 0 && !soa) return fail("gs_sim_bind_force_sensors: buffer required");
  s->sens = soa;
  return 0;
}

int gs_sim_refresh_force_sensor(gs_sim* s, float* out, void* stream) {
  if (ready(s, "gs_sim_refresh_force_sensor")) return -1;
  if (s->h_model.nsens == 0) return 0;
  if (!s->sens) return fail("gs_sim_refresh_force_sensor: sensors not bound");
  if (s->host) {
    host_soa_to_aos(s->sens, s->N, s->h_model.nsens, 6, out, s->pool);
    return 0;
  }
  hipError_t e = launch_refresh_sensor(s->sens, s->N, s->h_model.nsens, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_sim_refresh_force_sensor");
}

int gs_debug_terrain_query(gs_sim* s, const float* centres, const float* radii, int n, float* out, void* stream) {
  if (!s || !s->dp.has_terrain) return fail("gs_debug_terrain_query: no terrain mesh");
  if (n < 0 || (n > 0 && (!centres || !radii || !out))) return fail("gs_debug_terrain_query: bad buffers");
  if (s->host) {
    host_terrain_query(s->dp, centres, radii, n, out);
    return 0;
  }
  hipError_t e = launch_terrain_query(s->dp, centres, radii, n, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_debug_terrain_query");
}

int gs_debug_self_contacts(gs_sim* s, int mode, float* out, int* count, void* stream) {
  if (ready(s, "gs_debug_self_contacts")) return -1;
  if (!out || !count) return fail("gs_debug_self_contacts: bad buffers");
  if (s->host) {
    if (mode != 0) return fail("gs_debug_self_contacts: the host backend has the inline form only (mode 0)");
    s->htopo->dbg_pool(&s->h_model, s->dp, buffers(s), out, count, s->pool);
    return 0;
  }
  const hipError_t e = s->topo->dbg_pool(s->d_model, s->dp, buffers(s), mode, out, count, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(e, "gs_debug_self_contacts (mode 1 needs a split-form topology)");
}

int gs_sim_kernel_variant(gs_sim* s) { return s ? s->variant : -1; }

int gs_sim_pd_tail_supported(const gs_sim* s) {
  return s && !s->host && s->topo && s->variant == 2 && !s->dp.has_terrain && team_fused_tail_available() ? 1 : 0;
}

int gs_sim_enable_timing(gs_sim* s, int enable) {
  if (!s) return fail("gs_sim_enable_timing: null sim");
  s->timing = enable != 0;
  return 0;
}
float gs_sim_last_kernel_ms(gs_sim* s) {
  if (s && s->host) return s->timing ? (float)s->host_ms : -1.f;
  if (!s || !s->timed) return -1.f;
  float ms = -1.f;
  if (hipEventSynchronize(s->ev1) != hipSuccess) return -1.f;
  if (hipEventElapsedTime(&ms, s->ev0, s->ev1) != hipSuccess) return -1.f;
  return ms;
}

}  // extern "C"
