// gs_host_impl.h -- the host backend's thread pool and per-topology solver drivers (gs_host.hip): one env per
// pool task, the solver's LDS column as a thread-local scratch row; GS_HOST_QS=1 replays the GPU wave-assisted
// kernels' order of work (terrain queries first, then the substep) on the host.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <limits>
#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "gs_solver.h"

// ---------------------------------------------------------------- thread pool
struct HostPool {
  std::vector<std::thread> workers;
  std::mutex m;
  std::condition_variable wake, done;
  const std::function<void(int, int)>* job = nullptr;  // (begin, end) of a chunk of envs
  std::atomic<int> next{0};
  int n = 0, chunk = 1;
  unsigned long gen = 0;
  int busy = 0;
  bool stop = false;

  void drain() {
    for (;;) {
      const int b = next.fetch_add(chunk);
      if (b >= n) return;
      (*job)(b, b + chunk < n ? b + chunk : n);
    }
  }
  void worker() {
    unsigned long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m);
        wake.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      drain();
      std::lock_guard<std::mutex> lk(m);
      if (--busy == 0) done.notify_one();
    }
  }
  // run f over [0, n) in chunks; the calling thread works too; returns when every chunk is done
  void run(int n_items, const std::function<void(int, int)>& f) {
    if (n_items <= 0) return;
    const int threads = (int)workers.size() + 1;
    if (threads == 1 || n_items == 1) {
      f(0, n_items);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m);
      job = &f;
      n = n_items;
      // ~8 chunks per thread: envs differ in cost (contacts, terrain cells), so balance dynamically
      chunk = n_items / (threads * 8) > 0 ? n_items / (threads * 8) : 1;
      next.store(0);
      busy = (int)workers.size();
      ++gen;
    }
    wake.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(m);
    done.wait(lk, [&] { return busy == 0; });
    job = nullptr;
  }
};

namespace gs_hostimpl {

// per-thread contact-row scratch (the LDS column of one lane in the kernels, LB = 1).  GS_HOST_POISON=1 fills it
// with NaN before every env (debug: any read of a slot the env did not write shows up as a NaN state)
inline bool host_poison() {
  static const bool on = [] { const char* v = std::getenv("GS_HOST_POISON"); return v && v[0] == '1'; }();
  return on;
}
inline float* scratch(int slots) {
  thread_local std::vector<float> buf;
  if ((int)buf.size() < slots) buf.resize(slots);
  return buf.data();
}
inline void poison(float* lds, int slots) {
  if (host_poison()) std::fill(lds, lds + slots, std::numeric_limits<float>::quiet_NaN());
}

// GS_HOST_QS=1 (debug): mesh scenes take the GPU TERR kernels' route -- candidate centres, the terrain queries
// run first into a result table, the substep reads them (substep QS > 0) -- instead of the inline queries
inline bool host_qs() {
  static const bool on = [] { const char* v = std::getenv("GS_HOST_QS"); return v && v[0] == '1'; }();
  return on;
}
template <class T>
void simulate_env_qs(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau_aos, int e, float* lds) {
  const int N = B.N;
  EnvState<T> s;
  load_state<T>(B.state, N, e, s);
  float tau[T::ND > 0 ? T::ND : 1];
  for (int j = 0; j < T::ND; ++j) tau[j] = tau_aos ? tau_aos[(size_t)e * T::ND + j] : 0.f;
  float qin[4 * T::NC], qout[5 * T::NC];
  for (int sstep = 0; sstep < P.substeps; ++sstep) {
    candidate_centres<T>(M, s, qin, 1);
    for (int c = 0; c < T::NC; ++c) {
      const float p[3] = {qin[4 * c], qin[4 * c + 1], qin[4 * c + 2]};
      const float r = qin[4 * c + 3];
      float sep = 0.f, n[3] = {0.f, 0.f, 0.f};
      const bool f = gs_terrain::sphere_contact(P.terr, p, r, r + P.contact_offset, sep, n);
      qout[5 * c] = f ? 1.f : 0.f;
      qout[5 * c + 1] = sep;
      qout[5 * c + 2] = n[0]; qout[5 * c + 3] = n[1]; qout[5 * c + 4] = n[2];
    }
    const bool last = (sstep == P.substeps - 1) && P.collect;
    substep<T, true, 1, 1, true>(M, P, s, tau, B.mu, N, e, lds, B.cf, last, sstep == P.substeps - 1 ? B.sens : nullptr,
                                 qout);
  }
  store_state<T>(B.state, N, e, s);
}

template <class T>
void host_sim(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, HostPool* pool) {
  if (P.has_terrain && host_qs()) {
    pool->run(B.N, [&](int b, int e1) {
      float* lds = scratch(LaneCfg<T, true>::SLOTS);
      for (int e = b; e < e1; ++e) { poison(lds, LaneCfg<T, true>::SLOTS); simulate_env_qs<T>(M, P, B, tau, e, lds); }
    });
  } else if (P.has_terrain) {
    pool->run(B.N, [&](int b, int e1) {
      float* lds = scratch(LaneCfg<T, true>::SLOTS);
      for (int e = b; e < e1; ++e) { poison(lds, LaneCfg<T, true>::SLOTS); simulate_env<T, true, 1>(M, P, B, tau, e, lds); }
    });
  } else {
    pool->run(B.N, [&](int b, int e1) {
      float* lds = scratch(LaneCfg<T, false>::SLOTS);
      for (int e = b; e < e1; ++e) { poison(lds, LaneCfg<T, false>::SLOTS); simulate_env<T, false, 1>(M, P, B, tau, e, lds); }
    });
  }
}

template <class T>
void host_pd(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, HostPool* pool) {
  if (P.has_terrain) {
    pool->run(B.N, [&](int b, int e1) {
      float* lds = scratch(LaneCfg<T, true>::SLOTS);
      for (int e = b; e < e1; ++e) { poison(lds, LaneCfg<T, true>::SLOTS); pd_step_env<T, true, 1>(M, P, B, A, e, lds); }
    });
  } else {
    pool->run(B.N, [&](int b, int e1) {
      float* lds = scratch(LaneCfg<T, false>::SLOTS);
      for (int e = b; e < e1; ++e) { poison(lds, LaneCfg<T, false>::SLOTS); pd_step_env<T, false, 1>(M, P, B, A, e, lds); }
    });
  }
}

// gs_debug_self_contacts on the host: each env's self-contact pool from the current state (the inline
// narrowphase of the host substep); out [N][npk][10], count [N] as gs_physics_impl.h k_dbg_pool
template <class T>
void host_dbg_pool(const DevModel* M, const DevParams& P, const SimBuffers& B, float* out, int* count, HostPool* pool) {
  using C = LaneCfg<T, false>;
  pool->run(B.N, [&](int b, int e1) {
    float* col = scratch(C::SLOTS);
    for (int e = b; e < e1; ++e) {
      int n = 0;
      if constexpr (T::NPK > 0) {
        constexpr int PE = PoolCfg<T>::PE;
        poison(col, C::SLOTS);
        EnvState<T> s;
        load_state<T>(B.state, B.N, e, s);
        shape_world<T, 1>(M, s, col);
        float* pl = col + C::X_POOL;
        n = self_contacts<T, 1>(M, P, B.mu, B.N, e, col, pl);
        for (int p = 0; p < n; ++p) {
          const float* o = pl + PE * p;
          float* d = out + ((size_t)e * T::NPK + p) * 10;
          for (int k = 0; k < 6; ++k) d[k] = o[kPoolX + k];
          d[6] = o[kPoolSep];
          d[7] = o[kPoolMu];
          d[8] = o[kPoolBA];
          d[9] = o[kPoolBB];
        }
      }
      count[e] = n;
    }
  });
}

}  // namespace gs_hostimpl
