// gs_physics.hip -- articulation dynamics + plane contact solve for gfx950.
//
// Replaces the PhysX GPU articulation/contact pipeline that the reference runs
// inside `gym.simulate` (vec_task.py:382, anymal_terrain.py:448).  The solver
// specification is shared with the fp64 CPU oracle in
// oracle/physics_oracle.c, which is written independently (dense Cholesky,
// joint-space impulses); this file is the MI355X form:
//
//   * one env per lane, 64 envs per wave / workgroup; state loads and stores
//     are SoA so every wave-instruction moves 256 contiguous bytes;
//   * the articulation topology is a template parameter (gs_topologies.h), all
//     tree walks unroll at compile time and the per-body quantities (poses,
//     motion subspaces, composite inertias, the L^T D L factor of the mass
//     matrix) live in VGPRs;
//   * contact rows are staged in LDS ([slot][lane], conflict-free) because
//     their count (3 per candidate) would not fit the register file;
//   * model constants are read through a uniform pointer -> SGPR loads.
//
// Per substep (h = dt / substeps):
//   FK -> spatial inertias at the root origin O -> RNEA bias (gravity as base
//   acceleration) -> CRBA mass matrix -> tree-sparse L^T D L -> free velocity
//   -> plane contact candidates (contact_offset) -> per row scaled
//   Z = J L^-1 D^-1/2 -> projected Gauss-Seidel in w-space
//   (pos iterations with depenetration bias, then velocity iterations without)
//   -> velocity limits -> semi-implicit integration with the position-phase
//   velocity; the velocity-phase velocity is kept as state.

#include "gs_solver.h"

namespace {

// ---------------------------------------------------------------- kernels
template <class T, bool TERR>
__global__ __launch_bounds__((LaneCfg<T, TERR>::LB), 1) void k_simulate(const DevModel* __restrict__ M, DevParams P,
                                                                SimBuffers B, const float* __restrict__ tau_aos) {
  constexpr int LB = LaneCfg<T, TERR>::LB;
  __shared__ float lds[LaneCfg<T, TERR>::SLOTS * LB];
  const int e = blockIdx.x * LB + threadIdx.x;
  if (e >= B.N) return;
  simulate_env<T, TERR, LB>(M, P, B, tau_aos, e, lds + threadIdx.x);
}

template <class T, bool TERR>
__global__ __launch_bounds__((LaneCfg<T, TERR>::LB), 1) void k_pd_step(const DevModel* __restrict__ M, DevParams P,
                                                               SimBuffers B, PdDev A) {
  constexpr int LB = LaneCfg<T, TERR>::LB;
  __shared__ float lds[LaneCfg<T, TERR>::SLOTS * LB];
  const int e = blockIdx.x * LB + threadIdx.x;
  if (e >= B.N) return;
  pd_step_env<T, TERR, LB>(M, P, B, A, e, lds + threadIdx.x);
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

template <class T>
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
      substep<T, true, LB, LB>(M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last,
                               sstep == P.substeps - 1 ? B.sens : nullptr, qout + threadIdx.x);
    }
  }
  if (env_lane) store_state<T>(B.state, N, e, s);
}

template <class T>
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
      substep<T, true, LB, LB>(M, P, s, tau, B.mu, N, e, lds + threadIdx.x, B.cf, last,
                               it == total - 1 ? B.sens : nullptr, qout + threadIdx.x);
      if (it == n_pd - 1) pd_dof_out<T>(A, e, s);
    }
  }
  if (env_lane) pd_outputs<T>(M, P, B, A, e, s, tau);
}

// ---------------------------------------------------------------- tensor API kernels
__global__ void k_refresh_root(const float* __restrict__ st, int N, const float* __restrict__ com0,
                               float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  refresh_root_env(st, N, com0, out, e);
}
__global__ void k_refresh_dof(const float* __restrict__ st, int N, int nd, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // t = e*nd + j
  if (t >= N * nd) return;
  const int e = t / nd, j = t - e * nd;
  out[2 * (size_t)t + 0] = st[(13 + j) * N + e];
  out[2 * (size_t)t + 1] = st[(13 + nd + j) * N + e];
}
__global__ void k_refresh_contact(const float* __restrict__ cf, int N, int nb, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // t = (e*nb + b)*3 + k
  if (t >= N * nb * 3) return;
  const int k = t % 3, eb = t / 3, b = eb % nb, e = eb / nb;
  out[t] = cf[(3 * b + k) * N + e];
}
__global__ void k_refresh_sensor(const float* __restrict__ soa, int N, int ns, float* __restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)N * ns * 6) return;
  const int k = (int)(t % 6);
  const long eb = t / 6;
  const int sidx = (int)(eb % ns);
  const int e = (int)(eb / ns);
  out[t] = soa[(6 * sidx + k) * (long)N + e];
}
__global__ void k_set_root(float* __restrict__ st, int N, const float* __restrict__ com0,
                           const float* __restrict__ src, const int* __restrict__ idx, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int e = idx ? idx[t] : t;
  if (e < 0 || e >= N) return;
  set_root_env(st, N, com0, src, e);
}
__global__ void k_set_dof(float* __restrict__ st, int N, int nd, const float* __restrict__ src,
                          const int* __restrict__ idx, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;  // t over n*nd
  if (t >= n * nd) return;
  const int r = t / nd, j = t - r * nd;
  const int e = idx ? idx[r] : r;
  if (e < 0 || e >= N) return;
  st[(13 + j) * N + e] = src[((size_t)e * nd + j) * 2 + 0];
  st[(13 + nd + j) * N + e] = src[((size_t)e * nd + j) * 2 + 1];
}

__global__ void k_terrain_query(TerrainDev T, float offset, const float* __restrict__ c, const float* __restrict__ r,
                                int n, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float p[3] = {c[3 * t], c[3 * t + 1], c[3 * t + 2]};
  float sep = 0.f, nn[3] = {0.f, 0.f, 0.f};
  const bool f = gs_terrain::sphere_contact(T, p, r[t], r[t] + offset, sep, nn);
  out[5 * t] = f ? 1.f : 0.f;
  out[5 * t + 1] = sep;
  out[5 * t + 2] = nn[0]; out[5 * t + 3] = nn[1]; out[5 * t + 4] = nn[2];
}

inline int nblk(long n, int b) { return (int)((n + b - 1) / b); }

}  // namespace

hipError_t launch_terrain_query(const DevParams& P, const float* c, const float* r, int n, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_terrain_query, dim3(nblk(n, 256)), dim3(256), 0, s, P.terr, P.contact_offset, c, r, n, out);
  return hipGetLastError();
}
hipError_t launch_refresh_root(const float* state, int N, int nd, const float* com0, float* out, hipStream_t s) {
  (void)nd;
  hipLaunchKernelGGL(k_refresh_root, dim3(nblk(N, 256)), dim3(256), 0, s, state, N, com0, out);
  return hipGetLastError();
}
hipError_t launch_refresh_dof(const float* state, int N, int nd, float* out, hipStream_t s) {
  if (nd == 0) return hipSuccess;
  hipLaunchKernelGGL(k_refresh_dof, dim3(nblk((long)N * nd, 256)), dim3(256), 0, s, state, N, nd, out);
  return hipGetLastError();
}
hipError_t launch_refresh_contact(const float* cf, int N, int nb, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_refresh_contact, dim3(nblk((long)N * nb * 3, 256)), dim3(256), 0, s, cf, N, nb, out);
  return hipGetLastError();
}
hipError_t launch_refresh_sensor(const float* soa, int N, int ns, float* out, hipStream_t s) {
  // [6*ns][N] -> [N*ns][6]: the same transpose as the contact refresh with 6 components
  hipLaunchKernelGGL(k_refresh_sensor, dim3(nblk((long)N * ns * 6, 256)), dim3(256), 0, s, soa, N, ns, out);
  return hipGetLastError();
}
hipError_t launch_set_root(float* state, int N, int nd, const float* com0, const float* src, const int* idx, int n_idx,
                           hipStream_t s) {
  (void)nd;
  const int n = idx ? n_idx : N;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_root, dim3(nblk(n, 256)), dim3(256), 0, s, state, N, com0, src, idx, n);
  return hipGetLastError();
}
hipError_t launch_set_dof(float* state, int N, int nd, const float* src, const int* idx, int n_idx, hipStream_t s) {
  const int n = idx ? n_idx : N;
  if (n <= 0 || nd == 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_dof, dim3(nblk((long)n * nd, 256)), dim3(256), 0, s, state, N, nd, src, idx, n);
  return hipGetLastError();
}

template <class T>
hipError_t launch_sim(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  if (P.has_terrain) {
    constexpr int LB = LaneCfg<T, true>::LB;
    hipLaunchKernelGGL((k_simulate_terr<T>), dim3((B.N + LB - 1) / LB), dim3(kTerrWave), 0, st, M, P, B, tau);
  } else {
    constexpr int LB = LaneCfg<T, false>::LB;
    hipLaunchKernelGGL((k_simulate<T, false>), dim3((B.N + LB - 1) / LB), dim3(LB), 0, st, M, P, B, tau);
  }
  return hipGetLastError();
}
template <class T>
hipError_t launch_pd(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  if (P.has_terrain) {
    constexpr int LB = LaneCfg<T, true>::LB;
    hipLaunchKernelGGL((k_pd_step_terr<T>), dim3((B.N + LB - 1) / LB), dim3(kTerrWave), 0, st, M, P, B, A);
  } else {
    constexpr int LB = LaneCfg<T, false>::LB;
    hipLaunchKernelGGL((k_pd_step<T, false>), dim3((B.N + LB - 1) / LB), dim3(LB), 0, st, M, P, B, A);
  }
  return hipGetLastError();
}

#define GS_TOPO_ENTRY(T, SIG) {SIG, T::kName, &launch_sim<T>, &launch_pd<T>, T::NB, T::ND, T::NC, T::NS, T::SENS ? 1 : 0},
TopoEntry g_topologies[] = {GS_FOR_EACH_TOPOLOGY(GS_TOPO_ENTRY)};
const int g_num_topologies = sizeof(g_topologies) / sizeof(g_topologies[0]);
