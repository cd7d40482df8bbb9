// gs_host.hip -- the host backend of libgymsim: the reference's `sim_device=cpu pipeline=cpu` path.
//
// Isaac Gym runs PhysX on the CPU when sim_device is "cpu" (vec_task.py:82-88; physx.use_gpu is
// `contains("cuda", sim_device)`, cfg/task/*.yaml) with `physx.num_threads` worker threads
// (cfg/config.yaml:30-32).  This backend steps the same solver source as the HIP kernels
// (gs_solver.h, gs_kinematics.h: every function there is __host__ __device__) one env per task on
// a persistent pool of `num_threads` threads (the caller included), on caller-owned HOST buffers
// in the same SoA / AoS layouts as the device backend.  Nothing here touches the HIP runtime, so
// the backend runs on a machine without a GPU.  Selected by gs_sim_create(device < 0, ...).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
#include <limits>
#include <algorithm>
#include <cstdlib>

#include "gs_host_impl.h"
#include "gs_kinematics.h"

using gs_hostimpl::host_sim;
using gs_hostimpl::host_pd;
using gs_hostimpl::host_dbg_pool;

HostPool* host_pool_create(int threads) {
  HostPool* p = new HostPool();
  for (int i = 1; i < threads; ++i) p->workers.emplace_back([p] { p->worker(); });
  return p;
}
void host_pool_destroy(HostPool* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(p->m);
    p->stop = true;
  }
  p->wake.notify_all();
  for (auto& t : p->workers) t.join();
  delete p;
}
int host_pool_threads(const HostPool* p) { return p ? (int)p->workers.size() + 1 : 0; }


#define GS_HOST_TOPO_ENTRY(T, SIG) {SIG, &host_sim<T>, &host_pd<T>, &host_dbg_pool<T>},
HostTopoEntry g_host_topologies[] = {GS_FOR_EACH_TOPOLOGY(GS_HOST_TOPO_ENTRY)};
const int g_num_host_topologies = sizeof(g_host_topologies) / sizeof(g_host_topologies[0]);

// ---------------------------------------------------------------- tensor API (host buffers)
void host_refresh_root(const float* st, int N, const float* com0, float* out, HostPool* pool) {
  pool->run(N, [&](int b, int e1) {
    for (int e = b; e < e1; ++e) refresh_root_env(st, N, com0, out, e);
  });
}
void host_refresh_dof(const float* st, int N, int nd, float* out, HostPool* pool) {
  pool->run(N, [&](int b, int e1) {
    for (int e = b; e < e1; ++e)
      for (int j = 0; j < nd; ++j) {
        out[2 * ((size_t)e * nd + j) + 0] = st[(size_t)(13 + j) * N + e];
        out[2 * ((size_t)e * nd + j) + 1] = st[(size_t)(13 + nd + j) * N + e];
      }
  });
}
// SoA [comp*n][N] -> AoS [N*n][comp]
void host_soa_to_aos(const float* soa, int N, int n, int comp, float* out, HostPool* pool) {
  pool->run(N, [&](int b, int e1) {
    for (int e = b; e < e1; ++e)
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < comp; ++k) out[((size_t)e * n + i) * comp + k] = soa[(size_t)(comp * i + k) * N + e];
  });
}
void host_set_root(float* st, int N, const float* com0, const float* src, const int* idx, int n) {
  for (int t = 0; t < n; ++t) {
    const int e = idx ? idx[t] : t;
    if (e >= 0 && e < N) set_root_env(st, N, com0, src, e);
  }
}
void host_set_dof(float* st, int N, int nd, const float* src, const int* idx, int n) {
  for (int t = 0; t < n; ++t) {
    const int e = idx ? idx[t] : t;
    if (e < 0 || e >= N) continue;
    for (int j = 0; j < nd; ++j) {
      st[(size_t)(13 + j) * N + e] = src[((size_t)e * nd + j) * 2 + 0];
      st[(size_t)(13 + nd + j) * N + e] = src[((size_t)e * nd + j) * 2 + 1];
    }
  }
}
void host_kinematics(const DevModel* M, const DevLinks* L, const float* st, int N, int nv, int mode, float* rb,
                     float* jac, float* mm, HostPool* pool) {
  pool->run(N, [&](int b, int e1) {
    thread_local EnvKin K;
    for (int e = b; e < e1; ++e) {
      kin_forward(M, L, st, N, e, K);
      kin_outputs(M, L, st, N, nv, mode, e, K, 0, 1, rb, jac, mm);
    }
  });
}
void host_terrain_query(const DevParams& P, const float* c, const float* r, int n, float* out) {
  for (int t = 0; t < n; ++t) {
    const float p[3] = {c[3 * t], c[3 * t + 1], c[3 * t + 2]};
    float sep = 0.f, nn[3] = {0.f, 0.f, 0.f};
    const bool f = gs_terrain::sphere_contact(P.terr, p, r[t], r[t] + P.contact_offset, sep, nn);
    out[5 * t] = f ? 1.f : 0.f;
    out[5 * t + 1] = sep;
    out[5 * t + 2] = nn[0]; out[5 * t + 3] = nn[1]; out[5 * t + 4] = nn[2];
  }
}
