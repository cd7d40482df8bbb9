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

// ---------------------------------------------------------------- terrain-mesh (TERR) kernels
// The mesh narrowphase (gs_terrain::sphere_contact, a scan of the grid cells around a candidate) is
// most of a TERR substep, and the candidates' queries are independent.  A 64-lane workgroup holds
// LB env lanes (the per-env solver, as in k_simulate) and, before every substep, the WHOLE wave runs
// the LB x NC queries of its envs: env lanes publish their candidate centres (candidate_centres, the
// positions the solver's tree walk forms), every lane takes queries l, l + 64, ..., and the env lanes'
// substep reads the results instead of querying inline (substep<..., QS = LB>).  Same results as the
// inline query; the serial query chain per env shrinks from NC to ~NC * LB / 64.
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

template <class T, bool SELF>
__global__ __launch_bounds__(kTerrWave, 1) void k_simulate_terr(const DevModel* __restrict__ M, DevParams P,
                                                                SimBuffers B, const float* __restrict__ tau_aos) {
  constexpr int LB = LaneCfg<T, true>::LB, NC = T::NC;
  __shared__ float lds[LaneCfg<T, true>::SLOTS * LB];
  __shared__ float qin[4 * NC * LB], qout[5 * NC * LB];
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
    if (env_lane) candidate_centres<T>(M, s, qin + threadIdx.x, LB);
    __syncthreads();
    terrain_queries<T, LB>(P, N, e0, qin, qout);
    __syncthreads();
    if (env_lane) {
      const bool last = (sstep == P.substeps - 1) && P.collect;
      substep<T, true, LB, LB, SELF>(M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last,
                               sstep == P.substeps - 1 ? B.sens : nullptr, qout + threadIdx.x);
    }
  }
  if (env_lane) store_state<T>(B.state, N, e, s);
}

template <class T, bool SELF>
__global__ __launch_bounds__(kTerrWave, 1) void k_pd_step_terr(const DevModel* __restrict__ M, DevParams P,
                                                               SimBuffers B, PdDev A) {
  constexpr int LB = LaneCfg<T, true>::LB, NC = T::NC;
  __shared__ float lds[LaneCfg<T, true>::SLOTS * LB];
  __shared__ float qin[4 * NC * LB], qout[5 * NC * LB];
  const int N = B.N, e0 = blockIdx.x * LB, e = e0 + threadIdx.x;
  const bool env_lane = threadIdx.x < LB && e < N;
  EnvState<T> s;
  float tau[T::ND];
  if (env_lane) load_state<T>(B.state, N, e, s);
  const int sub = P.substeps;
  const int n_pd = A.decimation * sub;
  const int total = (A.decimation + A.extra) * sub;
  for (int it = 0; it < total; ++it) {  // uniform trip count: every lane meets every barrier
    if (env_lane) {
      if (it < n_pd && (it % sub) == 0) pd_torques<T>(A, e, s, it == 0, tau);
      candidate_centres<T>(M, s, qin + threadIdx.x, LB);
    }
    __syncthreads();
    terrain_queries<T, LB>(P, N, e0, qin, qout);
    __syncthreads();
    if (env_lane) {
      const bool last = ((it % sub) == sub - 1) && P.collect;
      substep<T, true, LB, LB, SELF>(M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last,
                               it == total - 1 ? B.sens : nullptr, qout + threadIdx.x);
      if (it == n_pd - 1) pd_dof_out<T>(A, e, s);
    }
  }
  if (env_lane) pd_outputs<T>(M, P, B, A, e, s, tau);
}

}  // namespace gs_phys

// launchers, one per kernel form (instantiated per topology in gs_phys_inst.hip)
template <class T>
hipError_t launch_sim_plane(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  constexpr int LB = LaneCfg<T, false>::LB;
  if (P.self_collide)
    hipLaunchKernelGGL((gs_phys::k_simulate<T, false, true>), dim3((B.N + LB - 1) / LB), dim3(LB), 0, st, M, P, B, tau);
  else
    hipLaunchKernelGGL((gs_phys::k_simulate<T, false, false>), dim3((B.N + LB - 1) / LB), dim3(LB), 0, st, M, P, B, tau);
  return hipGetLastError();
}
template <class T>
hipError_t launch_sim_terr(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  constexpr int LB = LaneCfg<T, true>::LB;
  if (P.self_collide)
    hipLaunchKernelGGL((gs_phys::k_simulate_terr<T, true>), dim3((B.N + LB - 1) / LB), dim3(gs_phys::kTerrWave), 0, st, M, P,
                       B, tau);
  else
    hipLaunchKernelGGL((gs_phys::k_simulate_terr<T, false>), dim3((B.N + LB - 1) / LB), dim3(gs_phys::kTerrWave), 0, st, M,
                       P, B, tau);
  return hipGetLastError();
}
template <class T>
hipError_t launch_pd_plane(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  constexpr int LB = LaneCfg<T, false>::LB;
  if (P.self_collide)
    hipLaunchKernelGGL((gs_phys::k_pd_step<T, false, true>), dim3((B.N + LB - 1) / LB), dim3(LB), 0, st, M, P, B, A);
  else
    hipLaunchKernelGGL((gs_phys::k_pd_step<T, false, false>), dim3((B.N + LB - 1) / LB), dim3(LB), 0, st, M, P, B, A);
  return hipGetLastError();
}
template <class T>
hipError_t launch_pd_terr(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  constexpr int LB = LaneCfg<T, true>::LB;
  if (P.self_collide)
    hipLaunchKernelGGL((gs_phys::k_pd_step_terr<T, true>), dim3((B.N + LB - 1) / LB), dim3(gs_phys::kTerrWave), 0, st, M, P,
                       B, A);
  else
    hipLaunchKernelGGL((gs_phys::k_pd_step_terr<T, false>), dim3((B.N + LB - 1) / LB), dim3(gs_phys::kTerrWave), 0, st, M, P,
                       B, A);
  return hipGetLastError();
}
