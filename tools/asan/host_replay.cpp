// ASan + UBSan replay driver for libgymsim's host backend (SURVEY section 5 sanitizers).
// Reads a case written by tools/asan/dump_case.py, builds the sim through the public C ABI (include/gymsim.h) on
// the host backend (device -1: no HIP call), runs the fused PD step (gs_sim_pd_step: 4 x PD + 1 simulates) and
// writes the final SoA state and the torques to <case>.out.  Built by tools/asan/run.sh with the host-side
// sanitizers on gs_host.hip / gs_capi.hip (the solver, narrowphase and kinematics headers they instantiate).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gymsim.h"

namespace {
FILE* g_in = nullptr;
template <class T>
void rd(T* p, size_t n) {
  if (fread(p, sizeof(T), n, g_in) != n) {
    fprintf(stderr, "host_replay: truncated case file\n");
    exit(2);
  }
}
struct Arr {
  std::vector<int32_t> i;
  std::vector<double> d;
  const void* ptr() const { return i.empty() ? (const void*)d.data() : (const void*)i.data(); }
};
void check(int rc, const char* what) {
  if (rc != 0) {
    fprintf(stderr, "host_replay: %s failed: %s\n", what, gs_last_error());
    exit(3);
  }
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: host_replay <case.bin>\n");
    return 1;
  }
  g_in = fopen(argv[1], "rb");
  if (!g_in) {
    perror("host_replay");
    return 1;
  }
  uint32_t magic = 0;
  rd(&magic, 1);
  if (magic != 0x47534153u) {
    fprintf(stderr, "host_replay: not a case file\n");
    return 1;
  }
  constexpr int NF = 39;  // pointer fields of gs_model_desc, dump_case.py _FIELDS order
  std::vector<Arr> a(NF);
  for (int f = 0; f < NF; ++f) {
    int64_t n = 0;
    int32_t kind = 0;
    rd(&n, 1);
    rd(&kind, 1);
    if (kind == 0) { a[f].i.resize(n); rd(a[f].i.data(), n); }
    else { a[f].d.resize(n); rd(a[f].d.data(), n); }
  }
  int32_t sc[10];
  rd(sc, 10);
  gs_model_desc m{};
  m.num_bodies = sc[0]; m.num_dofs = sc[1]; m.num_candidates = sc[2]; m.num_shapes = sc[3]; m.fixed_base = sc[4];
  m.num_links = sc[5]; m.num_hull_verts = sc[6]; m.num_pairs = sc[7]; m.pair_pool = sc[8]; m.num_pair_verts = sc[9];
  int f = 0;
  auto I = [&]() { return (const int32_t*)a[f++].ptr(); };
  auto D = [&]() { return (const double*)a[f++].ptr(); };
  m.parent = I(); m.joint_kind = I(); m.body_dof = I(); m.joint_origin = D(); m.joint_axis = D(); m.mass = D();
  m.com = D(); m.inertia = D(); m.cand_body = I(); m.cand_point = D(); m.cand_radius = D(); m.cand_shape = I();
  m.dof_effort = D(); m.dof_velocity = D(); m.dof_armature = D(); m.dof_lower = D(); m.dof_upper = D();
  m.dof_has_limits = I(); m.cand_link = I(); m.link_body = I(); m.link_pose = D(); m.link_com = D();
  m.cand_dyn = I(); m.shape_kind = I(); m.shape_body = I(); m.shape_link = I(); m.shape_pose = D();
  m.shape_size = D(); m.shape_margin = D(); m.shape_sphere = D(); m.hull_verts = D(); m.shape_hv0 = I();
  m.shape_hv1 = I(); m.pair_a = I(); m.pair_b = I(); m.pair_kind = I(); m.pair_verts = D(); m.shape_pv0 = I();
  m.shape_pv1 = I();
  gs_sim_params p{};
  rd(&p.dt, 1); rd(&p.substeps, 1); rd(p.gravity, 3); rd(&p.num_position_iterations, 1);
  rd(&p.num_velocity_iterations, 1); rd(&p.contact_offset, 1); rd(&p.rest_offset, 1);
  rd(&p.bounce_threshold_velocity, 1); rd(&p.max_depenetration_velocity, 1); rd(&p.contact_collection, 1);
  rd(&p.kernel_variant, 1); rd(&p.joint_limit_margin, 1);
  p.num_threads = 1;
  int32_t hdr[5];
  rd(hdr, 5);
  double gnd[3];
  rd(gnd, 3);
  const int N = hdr[0], nd = hdr[1], ns = hdr[2], self_collide = hdr[3], ground = hdr[4];
  std::vector<float> state((size_t)(13 + 2 * nd) * N), mu((size_t)ns * N), act((size_t)N * nd), def(nd), g(4);
  rd(state.data(), state.size());
  rd(mu.data(), mu.size());
  rd(act.data(), act.size());
  rd(def.data(), def.size());
  rd(g.data(), 4);
  fclose(g_in);

  gs_sim* sim = gs_sim_create(-1, &p);
  if (!sim) {
    fprintf(stderr, "host_replay: gs_sim_create failed: %s\n", gs_last_error());
    return 3;
  }
  check(gs_sim_set_model(sim, &m), "gs_sim_set_model");
  check(gs_sim_set_self_collision(sim, self_collide), "gs_sim_set_self_collision");
  if (ground) check(gs_sim_add_ground(sim, gnd[0], gnd[1], gnd[2]), "gs_sim_add_ground");
  std::vector<float> cf((size_t)3 * m.num_links * N, 0.f);
  check(gs_sim_prepare(sim, N, state.data(), mu.data(), cf.data()), "gs_sim_prepare");
  std::vector<float> tau((size_t)N * nd, 0.f), dof_out((size_t)N * nd * 2, 0.f), root_out((size_t)N * 13, 0.f),
      contact_out((size_t)N * m.num_links * 3, 0.f);
  for (int i = 0; i < N; ++i)  // the refreshed dof state tensor the first PD torque reads (gs_pd_args)
    for (int d = 0; d < nd; ++d) {
      dof_out[((size_t)i * nd + d) * 2] = state[(size_t)(13 + d) * N + i];
      dof_out[((size_t)i * nd + d) * 2 + 1] = state[(size_t)(13 + nd + d) * N + i];
    }
  gs_pd_args pd{};
  pd.actions = act.data();
  pd.default_pos = def.data();
  pd.kp = g[0]; pd.kd = g[1]; pd.action_scale = g[2]; pd.torque_limit = g[3];
  pd.decimation = 4;
  pd.extra_simulates = 1;
  pd.torques_out = tau.data();
  pd.dof_state_out = dof_out.data();
  pd.root_state_out = root_out.data();
  pd.contact_out = contact_out.data();
  check(gs_sim_pd_step(sim, &pd, nullptr), "gs_sim_pd_step");
  gs_sim_destroy(sim);
  std::string out = std::string(argv[1]) + ".out";
  FILE* fo = fopen(out.c_str(), "wb");
  if (!fo) {
    perror("host_replay");
    return 1;
  }
  fwrite(state.data(), sizeof(float), state.size(), fo);
  fwrite(tau.data(), sizeof(float), tau.size(), fo);
  fclose(fo);
  printf("host_replay: %d envs, 4 x PD + 1 on the host backend, outputs in %s\n", N, out.c_str());
  return 0;
}
