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
  simulate_env<T, TERR, LB, SELF>(M, P, B, tau_aos, e, rows);
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

// pair records of the workgroup's envs (gs_solver.h pool_from_records layout, stride LB) from the shape world
// data the env lanes wrote into their LDS columns (stride LB)
template <class T, int LB>
__device__ __forceinline__ void pair_records(const DevModel* __restrict__ M, const DevParams& P,
                                             const float* __restrict__ mu_g, int N, int e0, const float* shw,
                                             float* __restrict__ prec) {
  constexpr int NI = T::NPAIR * LB;
  for (int it = threadIdx.x; it < NI; it += kTerrWave) {
    const int q = it / LB, l = it - q * LB;
    int n = 0;
    if (e0 + l < N)
      self_pair<T, LB, LB, kRec, ShapeConstsM, true>(M, ShapeConstsM{M}, P, mu_g, N, e0 + l, shw + l,
                                                     prec + (T::NPAIR + 2 * q * kRec) * LB + l, M->pa[q], M->pb[q],
                                                     M->pk[q], n);
    prec[q * LB + l] = (float)n;
  }
}

template <class T, bool TERR, bool SELF>
struct WaveCfg {
  static constexpr int LB = LaneCfg<T, TERR>::LB;
  static constexpr bool PAIRS = SELF && T::NPK > 0;
  static constexpr int QIN = TERR ? 4 * T::NC * LB : 1, QOUT = TERR ? 5 * T::NC * LB : 1;
  static constexpr int PREC = PAIRS ? T::NPAIR * (1 + 2 * kRec) * LB : 1;
};

// the work of the whole workgroup before an env substep: env lanes publish, every lane queries / tests
template <class T, bool TERR, bool SELF>
__device__ __forceinline__ void wave_prepass(const DevModel* __restrict__ M, const DevParams& P, const SimBuffers& B,
                                             int e0, bool env_lane, const EnvState<T>& s, float* lds, float* qin,
                                             float* qout, float* prec) {
  using W = WaveCfg<T, TERR, SELF>;
  constexpr int LB = W::LB;
  if (env_lane) {
    if constexpr (TERR) candidate_centres<T>(M, s, qin + threadIdx.x, LB);
    if constexpr (W::PAIRS) if (P.self_collide) shape_world<T, LB>(M, s, lds + threadIdx.x);
  }
  __syncthreads();
  if constexpr (TERR) terrain_queries<T, LB>(P, B.N, e0, qin, qout);
#ifndef GS_NO_PAIR_REC
  if constexpr (W::PAIRS) if (P.self_collide) pair_records<T, LB>(M, P, B.mu, B.N, e0, lds, prec);
#endif
  __syncthreads();
}

template <class T, bool TERR, bool SELF>
__global__ __launch_bounds__(kTerrWave, 1) void k_simulate_wave(const DevModel* __restrict__ M, DevParams P,
                                                                SimBuffers B, const float* __restrict__ tau_aos) {
  using W = WaveCfg<T, TERR, SELF>;
  constexpr int LB = W::LB;
  __shared__ float lds[LaneCfg<T, TERR>::SLOTS * LB];
  __shared__ float qin[W::QIN], qout[W::QOUT], prec[W::PREC];
  const int N = B.N, e0 = blockIdx.x * LB, e = e0 + threadIdx.x;
  const bool env_lane = threadIdx.x < LB && e < N;
  EnvState<T> s;
  float tau[T::ND > 0 ? T::ND : 1];
  if (env_lane) {
    load_state<T>(B.state, N, e, s);
#pragma unroll
    for (int j = 0; j < T::ND; ++j) tau[j] = tau_aos ? tau_aos[(size_t)e * T::ND + j] : 0.f;
  }
  for (int sstep = 0; sstep < P.substeps; ++sstep) {  // uniform trip count: every lane meets every barrier
    wave_prepass<T, TERR, SELF>(M, P, B, e0, env_lane, s, lds, qin, qout, prec);
    if (env_lane) {
      const bool last = (sstep == P.substeps - 1) && P.collect;
      substep<T, TERR, LB, TERR ? LB : 0, SELF, W::PAIRS ? LB : 0>(
          M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last, sstep == P.substeps - 1 ? B.sens : nullptr,
          qout + threadIdx.x, prec + threadIdx.x);
    }
  }
  if (env_lane) store_state<T>(B.state, N, e, s);
}

template <class T, bool TERR, bool SELF>
__global__ __launch_bounds__(kTerrWave, 1) void k_pd_step_wave(const DevModel* __restrict__ M, DevParams P,
                                                               SimBuffers B, PdDev A) {
  using W = WaveCfg<T, TERR, SELF>;
  constexpr int LB = W::LB;
  __shared__ float lds[LaneCfg<T, TERR>::SLOTS * LB];
  __shared__ float qin[W::QIN], qout[W::QOUT], prec[W::PREC];
  const int N = B.N, e0 = blockIdx.x * LB, e = e0 + threadIdx.x;
  const bool env_lane = threadIdx.x < LB && e < N;
  EnvState<T> s;
  float tau[T::ND];
  if (env_lane) load_state<T>(B.state, N, e, s);
  const int sub = P.substeps;
  const int n_pd = A.decimation * sub;
  const int total = (A.decimation + A.extra) * sub;
  for (int it = 0; it < total; ++it) {  // uniform trip count: every lane meets every barrier
    if (env_lane && it < n_pd && (it % sub) == 0) pd_torques<T>(A, e, s, it == 0, tau);
    wave_prepass<T, TERR, SELF>(M, P, B, e0, env_lane, s, lds, qin, qout, prec);
    if (env_lane) {
      const bool last = ((it % sub) == sub - 1) && P.collect;
      substep<T, TERR, LB, TERR ? LB : 0, SELF, W::PAIRS ? LB : 0>(
          M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last, it == total - 1 ? B.sens : nullptr,
          qout + threadIdx.x, prec + threadIdx.x);
      if (it == n_pd - 1) pd_dof_out<T>(A, e, s);
    }
  }
  if (env_lane) pd_outputs<T>(M, P, B, A, e, s, tau);
}

}  // namespace gs_phys

// launchers, one per kernel form (instantiated per topology in gs_phys_inst.hip).  Mesh sims run the
// wave-assisted kernels; with GS_WAVE_PLANE_SELF plane sims with self-collision whose envs are LDS-starved
// (<= 4 env lanes per workgroup: UsefulHound) do too.
// (off: measured slower for UsefulHound, the only such topology -- 4.68 vs 4.17 ms per substep: the pair records
// cost it a workgroup per CU of LDS while its substep is bound by the solver lane's scratch latency, not by the
// narrowphase; profiles/r03f_hound_ab.txt)
#ifndef GS_WAVE_PLANE_SELF
#define GS_WAVE_PLANE_SELF 0
#endif
template <class T>
constexpr bool kWavePlaneSelf = GS_WAVE_PLANE_SELF && T::NPK > 0 && LaneCfg<T, false>::LB <= 4 && !LaneCfg<T, false>::GLOBAL;

template <class T>
hipError_t launch_sim_plane(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  constexpr int LB = LaneCfg<T, false>::LB;
  const dim3 grid((B.N + LB - 1) / LB);
  if (P.self_collide) {
    if constexpr (kWavePlaneSelf<T>)
      hipLaunchKernelGGL((gs_phys::k_simulate_wave<T, false, true>), grid, dim3(gs_phys::kTerrWave), 0, st, M, P, B, tau);
    else
      hipLaunchKernelGGL((gs_phys::k_simulate<T, false, true>), grid, dim3(LB), 0, st, M, P, B, tau);
  } else {
    hipLaunchKernelGGL((gs_phys::k_simulate<T, false, false>), grid, dim3(LB), 0, st, M, P, B, tau);
  }
  return hipGetLastError();
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
