// gs_physics_impl.h -- the per-env physics kernels (one env per lane, and the terrain-mesh form) and
// their launchers as templates.  Each (topology, kernel form) is instantiated in its own translation
// unit (gs_phys_inst.hip compiled once per pair by isaacgymenv_amd/build.py), so the large solver
// instantiations compile in parallel; gs_physics.hip holds the registry and the tensor API kernels.
#pragma once
#include "gs_solver.h"

namespace gs_phys {

// ---------------------------------------------------------------- kernels
template <class T, bool TERR, bool SELF>
__global__ __launch_bounds__((LaneCfg<T, TERR>::LB), 1) void k_simulate(const DevModel* __restrict__ M, DevParams P,
                                                                SimBuffers B, const float* __restrict__ tau_aos) {
  using C = LaneCfg<T, TERR>;
  constexpr int LB = C::LB;
  __shared__ float lds[C::GLOBAL ? 1 : C::SLOTS * LB];
  const int e = blockIdx.x * LB + threadIdx.x;
  if (e >= B.N) return;
  float* rows = C::GLOBAL ? B.rows + (size_t)blockIdx.x * C::SLOTS * LB + threadIdx.x : lds + threadIdx.x;
  simulate_env<T, TERR, LB, SELF, SELF && C::SPLIT>(M, P, B, tau_aos, e, rows);
}

template <class T, bool TERR, bool SELF>
__global__ __launch_bounds__((LaneCfg<T, TERR>::LB), 1) void k_pd_step(const DevModel* __restrict__ M, DevParams P,
                                                               SimBuffers B, PdDev A) {
  using C = LaneCfg<T, TERR>;
  constexpr int LB = C::LB;
  __shared__ float lds[C::GLOBAL ? 1 : C::SLOTS * LB];
  const int e = blockIdx.x * LB + threadIdx.x;
  if (e >= B.N) return;
  float* rows = C::GLOBAL ? B.rows + (size_t)blockIdx.x * C::SLOTS * LB + threadIdx.x : lds + threadIdx.x;
  pd_step_env<T, TERR, LB, SELF>(M, P, B, A, e, rows);
}

// ---------------------------------------------------------------- wave-assisted kernels (TERR, SELF)
// The mesh narrowphase (gs_terrain::sphere_contact, a scan of the grid cells around a candidate) and the
// self-collision narrowphase (gs_pairs.h self_pair: bounding spheres, closed-form sphere / capsule pairs, GJK)
// are independent per candidate / per shape pair, and inline in an env's substep they run serially in its lane.
// A 64-lane workgroup holds LB env lanes (the per-env solver, as in k_simulate) and, before every substep, the
// WHOLE wave runs the LB x NC terrain queries and the LB x NPAIR pair tests of its envs: env lanes publish their
// candidate centres (candidate_centres) and shape world data (shape_world), every lane takes work items
// l, l + 64, ..., and the env lanes' substep reads the results instead of computing them inline
// (substep<..., QS = LB, ..., PR = LB>).  Same results as the inline form; the serial chain per env shrinks from
// NC queries + NPAIR pair tests to ~(NC + NPAIR) * LB / 64.  The env lanes' substep then carries no mesh / GJK
// code, so its register allocation is the plane solver's.
constexpr int kTerrWave = 64;

// Phase profiler of the wave-assisted kernels (profiling build only, -DGS_PHASE_PROFILE -> libgymsim_prof.so):
// per-wave s_memtime cycles of 0 publish (shape world / candidate centres), 1 terrain queries, 2 pair broadphase,
// 3 pair narrowphase, 4 env-lane substep; summed over waves into this translation unit's gs_wave_cycles, read by
// gs_debug_wave_cycles_<topology>_<form> (gs_phys_inst.hip, tools/probes/wave_phases.py); [8] counts waves.
#ifdef GS_PHASE_PROFILE
static __device__ unsigned long long gs_wave_cycles[16];
#define GS_WPROF_DECL long long wt_ = clock64(); long long wacc_[5] = {0, 0, 0, 0, 0};
#define GS_WPROF(i) { const long long t_ = clock64(); wacc_[i] += t_ - wt_; wt_ = t_; }
#define GS_WPROF_PARAM , long long &wt_, long long *wacc_
#define GS_WPROF_ARGS , wt_, wacc_
#define GS_WPROF_FLUSH                                                                      \
  if (threadIdx.x == 0) {                                                                   \
    for (int i_ = 0; i_ < 5; ++i_) atomicAdd(&gs_wave_cycles[i_], (unsigned long long)wacc_[i_]); \
    atomicAdd(&gs_wave_cycles[8], 1ull);                                                    \
  }
#else
#define GS_WPROF_DECL
#define GS_WPROF(i)
#define GS_WPROF_PARAM
#define GS_WPROF_ARGS
#define GS_WPROF_FLUSH
#endif

template <class T, int LB>
__device__ __forceinline__ void terrain_queries(const DevParams& P, int N, int e0, const float* __restrict__ qin,
                                                float* __restrict__ qout) {
  constexpr int NQ = T::NC * LB;
  for (int q = threadIdx.x; q < NQ; q += kTerrWave) {
    const int c = q / LB, l = q - c * LB;
    if (e0 + l >= N) continue;
    const float p[3] = {qin[(4 * c + 0) * LB + l], qin[(4 * c + 1) * LB + l], qin[(4 * c + 2) * LB + l]};
    const float r = qin[(4 * c + 3) * LB + l];
    float sep = 0.f, n[3] = {0.f, 0.f, 0.f};
    const bool f = gs_terrain::sphere_contact(P.terr, p, r, r + P.contact_offset, sep, n);
    qout[(5 * c + 0) * LB + l] = f ? 1.f : 0.f;
    qout[(5 * c + 1) * LB + l] = sep;
    qout[(5 * c + 2) * LB + l] = n[0];
    qout[(5 * c + 3) * LB + l] = n[1];
    qout[(5 * c + 4) * LB + l] = n[2];
  }
}

// Near-pair records of the workgroup's envs (gs_solver.h NearRec layout, in each env's LDS column, stride LB)
// from the shape world data the env lanes wrote there.  Two passes over the wave:
//  1. broadphase, env by env, 64 pairs per round (lane = pair): the pairs within reach are ranked by a ballot
//     prefix, so each env's list comes out in pair order;
//  2. narrowphase of the listed pairs, one (env, pair) per lane -- the ~10-20 near pairs of every env of the
//     workgroup run side by side instead of one after another in the env's lane.
// The pair's shapes differ per lane in pass 2 (vector loads of their constants and hull vertices).
// (shape world at stride LB from shw; env l's records at stride RS from rb0 + l * rstep)
template <class T, int LB, int RS>
__device__ __forceinline__ void pair_records(const DevModel* __restrict__ M, const DevParams& P,
                                             const float* __restrict__ mu_g, int N, int e0, const float* shw,
                                             float* rb0, size_t rstep GS_WPROF_PARAM) {
  using R = NearRec<T>;
  const int lane = threadIdx.x;
  const float off = P.contact_offset;
  const ShapeConstsM sc{M};
  int tot = 0;
#pragma unroll
  for (int l = 0; l < LB; ++l) {
    const float* col = shw + l;
    float* rb = rb0 + l * rstep;
    const bool live = e0 + l < N;
    int cnt = 0;
    for (int q0 = 0; q0 < T::NPAIR; q0 += kTerrWave) {
      const int q = q0 + lane;
      bool near = false;
      if (live && q < T::NPAIR) {
        const int a = M->pa[q], b = M->pb[q];
        const float* sa = col + (kShW * a + 12) * LB;
        const float* sb = col + (kShW * b + 12) * LB;
        const float d[3] = {sa[0] - sb[0], sa[LB] - sb[LB], sa[2 * LB] - sb[2 * LB]};
        const float rr = sc.brad(a) + sc.brad(b) + off;
        near = dot3f(d, d) < rr * rr;
      }
      const unsigned long long bal = __ballot(near);
      if (near) rb[(1 + R::RW * (cnt + __popcll(bal & ((1ull << lane) - 1ull)))) * RS] = (float)q;
      cnt += __popcll(bal);
    }
    if (lane == 0 && live) rb[0] = (float)cnt;
    tot += cnt;
  }
  __syncthreads();  // the lists are read across lanes
  GS_WPROF(2)
  for (int i = lane; i < tot; i += kTerrWave) {
    int l = 0, r = i;
#pragma unroll
    for (int k = 0; k + 1 < LB; ++k) {
      const int c = (int)rb0[l * rstep];
      if (r >= c) { r -= c; ++l; }
    }
    float* rec = rb0 + l * rstep + (1 + R::RW * r) * RS;
    const int q = (int)rec[0];
    int n = 0;
    self_pair<T, LB, RS, kRec, ShapeConstsM, true>(M, sc, P, mu_g, N, e0 + l, shw + l, rec + RS, M->pa[q], M->pb[q],
                                                   M->pk[q], n);
    rec[0] = (float)(q + kRecQ * n);
  }
}

// The split form's narrowphase kernel (LaneCfg::SPLIT): kPairEnvs envs per 64-lane workgroup (2: 0.60 ms per
// UsefulHound launch vs 0.74 ms with 4, more waves in flight for the same pair tests) publish their
// shape world data to LDS, the wave runs pair_records, the records go to SimBuffers::rows for the solver kernel
// (k_simulate, substep PR = 1) that follows on the stream.  Its own launch: a small register footprint and
// several waves per SIMD to hide the narrowphase's load latency, which the solver kernel (512 VGPR, scratch,
// 3 waves per CU) cannot.  Two waves per SIMD (<= 256 VGPR): unbounded, the 4 publishing lanes' link poses (the
// forward kinematics of shape_world) took the kernel to 383 VGPR + AGPR, one wave per SIMD.
#ifndef GS_PAIR_ENVS
#define GS_PAIR_ENVS 2  // (A/B builds: 1)
#endif
constexpr int kPairEnvs = GS_PAIR_ENVS;
template <class T>
__global__ __launch_bounds__(kTerrWave, 2) void k_pair_records(const DevModel* __restrict__ M, DevParams P, SimBuffers B) {
  __shared__ float shw[kShW * T::NS * kPairEnvs];
  const int N = B.N, e0 = blockIdx.x * kPairEnvs, l = threadIdx.x;
  if (l < kPairEnvs && e0 + l < N) {
    EnvState<T> s;
    load_state<T>(B.state, N, e0 + l, s);
    shape_world<T, kPairEnvs>(M, s, shw + l);
  }
  __syncthreads();
  GS_WPROF_DECL
  constexpr int FL = LaneCfg<T, false>::ROW_FLOATS;
  pair_records<T, kPairEnvs, 1>(M, P, B.mu, N, e0, shw, B.rows + (size_t)e0 * FL, FL GS_WPROF_ARGS);
}

template <class T, bool TERR, bool SELF>
struct WaveCfg {
  static constexpr int LB = LaneCfg<T, TERR>::LB;
  static constexpr bool PAIRS = SELF && T::NPK > 0;
  static constexpr int QIN = TERR ? 4 * T::NC * LB : 1, QOUT = TERR ? 5 * T::NC * LB : 1;
  // the near-pair records live in the env columns' contact-row area (written after the records are read)
  static_assert(!PAIRS || NearRec<T>::END <= LaneCfg<T, TERR>::X_POOL, "near-pair records exceed the env column");
};

// the work of the whole workgroup before an env substep: env lanes publish, every lane queries / tests
template <class T, bool TERR, bool SELF>
__device__ __forceinline__ void wave_prepass(const DevModel* __restrict__ M, const DevParams& P, const SimBuffers& B,
                                             int e0, bool env_lane, const EnvState<T>& s, float* lds, float* qin,
                                             float* qout GS_WPROF_PARAM) {
  using W = WaveCfg<T, TERR, SELF>;
  constexpr int LB = W::LB;
  if (env_lane) {
    if constexpr (TERR) candidate_centres<T>(M, s, qin + threadIdx.x, LB);
    if constexpr (W::PAIRS) if (P.self_collide) shape_world<T, LB>(M, s, lds + threadIdx.x);
  }
  __syncthreads();
  GS_WPROF(0)
  if constexpr (TERR) terrain_queries<T, LB>(P, B.N, e0, qin, qout);
  GS_WPROF(1)
#ifndef GS_NO_PAIR_REC
  if constexpr (W::PAIRS)
    if (P.self_collide)
      pair_records<T, LB, LB>(M, P, B.mu, B.N, e0, lds, lds + NearRec<T>::SHW * LB, 1 GS_WPROF_ARGS);
#endif
  __syncthreads();
  GS_WPROF(3)
}

template <class T, bool TERR, bool SELF>
__global__ __launch_bounds__(kTerrWave, 1) void k_simulate_wave(const DevModel* __restrict__ M, DevParams P,
                                                                SimBuffers B, const float* __restrict__ tau_aos) {
  using W = WaveCfg<T, TERR, SELF>;
  constexpr int LB = W::LB;
  __shared__ float lds[LaneCfg<T, TERR>::SLOTS * LB];
  __shared__ float qin[W::QIN], qout[W::QOUT];
  const int N = B.N, e0 = blockIdx.x * LB, e = e0 + threadIdx.x;
  const bool env_lane = threadIdx.x < LB && e < N;
  EnvState<T> s;
  float tau[T::ND > 0 ? T::ND : 1];
  if (env_lane) {
    load_state<T>(B.state, N, e, s);
#pragma unroll
    for (int j = 0; j < T::ND; ++j) tau[j] = tau_aos ? tau_aos[(size_t)e * T::ND + j] : 0.f;
  }
  GS_WPROF_DECL
  for (int sstep = 0; sstep < P.substeps; ++sstep) {  // uniform trip count: every lane meets every barrier
    wave_prepass<T, TERR, SELF>(M, P, B, e0, env_lane, s, lds, qin, qout GS_WPROF_ARGS);
    if (env_lane) {
      const bool last = (sstep == P.substeps - 1) && P.collect;
      substep<T, TERR, LB, TERR ? LB : 0, SELF, W::PAIRS ? LB : 0>(
          M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last, sstep == P.substeps - 1 ? B.sens : nullptr,
          qout + threadIdx.x, lds + threadIdx.x + NearRec<T>::SHW * LB);
    }
    GS_WPROF(4)
  }
  GS_WPROF_FLUSH
  if (env_lane) store_state<T>(B.state, N, e, s);
}

template <class T, bool TERR, bool SELF>
__global__ __launch_bounds__(kTerrWave, 1) void k_pd_step_wave(const DevModel* __restrict__ M, DevParams P,
                                                               SimBuffers B, PdDev A) {
  using W = WaveCfg<T, TERR, SELF>;
  constexpr int LB = W::LB;
  __shared__ float lds[LaneCfg<T, TERR>::SLOTS * LB];
  __shared__ float qin[W::QIN], qout[W::QOUT];
  const int N = B.N, e0 = blockIdx.x * LB, e = e0 + threadIdx.x;
  const bool env_lane = threadIdx.x < LB && e < N;
  EnvState<T> s;
  float tau[T::ND];
  if (env_lane) load_state<T>(B.state, N, e, s);
  const int sub = P.substeps;
  const int n_pd = A.decimation * sub;
  const int total = (A.decimation + A.extra) * sub;
  GS_WPROF_DECL
  for (int it = 0; it < total; ++it) {  // uniform trip count: every lane meets every barrier
    if (env_lane && it < n_pd && (it % sub) == 0) pd_torques<T>(A, e, s, it == 0, tau);
    wave_prepass<T, TERR, SELF>(M, P, B, e0, env_lane, s, lds, qin, qout GS_WPROF_ARGS);
    if (env_lane) {
      const bool last = ((it % sub) == sub - 1) && P.collect;
      substep<T, TERR, LB, TERR ? LB : 0, SELF, W::PAIRS ? LB : 0>(
          M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last, it == total - 1 ? B.sens : nullptr,
          qout + threadIdx.x, lds + threadIdx.x + NearRec<T>::SHW * LB);
      if (it == n_pd - 1) pd_dof_out<T>(A, e, s);
    }
    GS_WPROF(4)
  }
  GS_WPROF_FLUSH
  if (env_lane) pd_outputs<T>(M, P, B, A, e, s, tau);
}

}  // namespace gs_phys

// launchers, one per kernel form (instantiated per topology in gs_phys_inst.hip).  Mesh sims run the
// wave-assisted kernels.  Plane sims with self-collision whose envs are LDS-starved (<= 4 env lanes per
// workgroup: UsefulHound): the simulate takes the split form when LaneCfg::SPLIT (k_pair_records, then
// k_simulate reading the records; r03: 1.64 vs 2.05 ms per substep for the wave form), and the fused PD step
// (gs_sim_pd_step) the wave-assisted form when GS_WAVE_PLANE_SELF (default 1) -- two narrowphase routes for one
// topology, each pinned against the oracle on the GPU (test_hound_gpu.py: the simulate and the fused PD step).
#ifndef GS_WAVE_PLANE_SELF
#define GS_WAVE_PLANE_SELF 1
#endif
template <class T>
constexpr bool kWavePlaneSelf = GS_WAVE_PLANE_SELF && T::NPK > 0 && LaneCfg<T, false>::LB <= 4 && !LaneCfg<T, false>::GLOBAL;

template <class T>
hipError_t launch_sim_plane(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  constexpr int LB = LaneCfg<T, false>::LB;
  const dim3 grid((B.N + LB - 1) / LB);
  if (P.self_collide) {
    if constexpr (LaneCfg<T, false>::SPLIT) {
      // narrowphase kernel, then the solver reading its records: one pair of launches per substep
      if (!B.rows) return hipErrorInvalidValue;
      const dim3 pgrid((B.N + gs_phys::kPairEnvs - 1) / gs_phys::kPairEnvs);
      DevParams P1 = P;
      P1.substeps = 1;
      for (int ss = 0; ss < P.substeps; ++ss) {
        P1.collect = P.collect && ss == P.substeps - 1;
        hipLaunchKernelGGL((gs_phys::k_pair_records<T>), pgrid, dim3(gs_phys::kTerrWave), 0, st, M, P1, B);
        hipLaunchKernelGGL((gs_phys::k_simulate<T, false, true>), grid, dim3(LB), 0, st, M, P1, B, tau);
      }
    } else if constexpr (kWavePlaneSelf<T>) {
      hipLaunchKernelGGL((gs_phys::k_simulate_wave<T, false, true>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, tau);
    } else {
      hipLaunchKernelGGL((gs_phys::k_simulate<T, false, true>), grid, dim3(LB), 0, st, M, P, B, tau);
    }
  } else {
    hipLaunchKernelGGL((gs_phys::k_simulate<T, false, false>), grid, dim3(LB), 0, st, M, P, B, tau);
  }
  return hipGetLastError();
}
// ---------------------------------------------------------------- self-contact pool dump (test hook)
// gs_debug_self_contacts: each env's self-contact pool from the current state, one env per thread with its
// column in device memory (LB = 1).  MODE 0: the inline narrowphase (self_contacts, what the lane / host forms
// run); MODE 1: the split form's route -- k_pair_records into SimBuffers::rows, then pool_from_records.
// out [N][npk][10] = x (3, root-origin relative), n (3), separation, friction, body a, body b; count [N].
namespace gs_phys {
template <class T, int MODE>
__global__ void k_dbg_pool(const DevModel* __restrict__ M, DevParams P, SimBuffers B, float* __restrict__ work,
                           float* __restrict__ out, int* __restrict__ count) {
  using C = LaneCfg<T, false>;
  const int N = B.N, e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  int n = 0;
  constexpr int NPK = T::NPK > 0 ? T::NPK : 1;
  if constexpr (T::NPK > 0) {
    constexpr int PE = PoolCfg<T>::PE;
    float* col = work + (size_t)e * C::SLOTS;
    float* pool = col + C::X_POOL;
    if constexpr (MODE == 0) {
      EnvState<T> s;
      load_state<T>(B.state, N, e, s);
      shape_world<T, 1>(M, s, col);
      n = self_contacts<T, 1>(M, P, B.mu, N, e, col, pool);
    } else {
      n = pool_from_records<T, 1, 1>(M, B.mu, N, e, B.rows + (size_t)e * C::ROW_FLOATS, pool);
    }
    for (int p = 0; p < n; ++p) {
      const float* o = pool + PE * p;
      float* d = out + ((size_t)e * NPK + p) * 10;
      for (int k = 0; k < 6; ++k) d[k] = o[kPoolX + k];
      d[6] = o[kPoolSep];
      d[7] = o[kPoolMu];
      d[8] = o[kPoolBA];
      d[9] = o[kPoolBB];
    }
  }
  count[e] = n;
}
}  // namespace gs_phys

template <class T>
hipError_t launch_dbg_pool(const DevModel* M, const DevParams& P, const SimBuffers& B, int mode, float* out,
                           int* count, hipStream_t st) {
  using C = LaneCfg<T, false>;
  if (mode != 0 && !(mode == 1 && C::SPLIT && B.rows)) return hipErrorInvalidValue;
  float* work = nullptr;
  hipError_t e = hipMalloc(&work, sizeof(float) * (size_t)B.N * C::SLOTS);
  if (e != hipSuccess) return e;
  DevParams P1 = P;
  P1.substeps = 1;
  if (mode == 1) {
    if constexpr (C::SPLIT)
      hipLaunchKernelGGL((gs_phys::k_pair_records<T>), dim3((B.N + gs_phys::kPairEnvs - 1) / gs_phys::kPairEnvs),
                         dim3(gs_phys::kTerrWave), 0, st, M, P1, B);
    hipLaunchKernelGGL((gs_phys::k_dbg_pool<T, 1>), dim3((B.N + 63) / 64), dim3(64), 0, st, M, P1, B, work, out, count);
  } else {
    hipLaunchKernelGGL((gs_phys::k_dbg_pool<T, 0>), dim3((B.N + 63) / 64), dim3(64), 0, st, M, P1, B, work, out, count);
  }
  e = hipGetLastError();
  const hipError_t e2 = hipStreamSynchronize(st);
  (void)hipFree(work);
  return e != hipSuccess ? e : e2;
}

template <class T>
hipError_t launch_sim_terr(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  constexpr int LB = LaneCfg<T, true>::LB;
  const dim3 grid((B.N + LB - 1) / LB);
  if (P.self_collide)
    hipLaunchKernelGGL((gs_phys::k_simulate_wave<T, true, true>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, tau);
  else
    hipLaunchKernelGGL((gs_phys::k_simulate_wave<T, true, false>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, tau);
  return hipGetLastError();
}
template <class T>
hipError_t launch_pd_plane(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  constexpr int LB = LaneCfg<T, false>::LB;
  const dim3 grid((B.N + LB - 1) / LB);
  if (P.self_collide) {
    if constexpr (kWavePlaneSelf<T>)
      hipLaunchKernelGGL((gs_phys::k_pd_step_wave<T, false, true>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, A);
    else
      hipLaunchKernelGGL((gs_phys::k_pd_step<T, false, true>), grid, dim3(LB), 0, st, M, P, B, A);
  } else {
    hipLaunchKernelGGL((gs_phys::k_pd_step<T, false, false>), grid, dim3(LB), 0, st, M, P, B, A);
  }
  return hipGetLastError();
}
template <class T>
hipError_t launch_pd_terr(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  constexpr int LB = LaneCfg<T, true>::LB;
  const dim3 grid((B.N + LB - 1) / LB);
  if (P.self_collide)
    hipLaunchKernelGGL((gs_phys::k_pd_step_wave<T, true, true>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, A);
  else
    hipLaunchKernelGGL((gs_phys::k_pd_step_wave<T, true, false>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, A);
  return hipGetLastError();
}
