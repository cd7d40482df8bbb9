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

#include "gs_solver.h"  // (kernels: gs_physics_impl.h)

namespace {

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

// a reset's two indexed sets in one launch: threads [0, n nd) the dofs (as k_set_dof), [n nd, n nd + n) the roots
__global__ void k_set_root_dof(float* __restrict__ st, int N, int nd, const float* __restrict__ com0,
                               const float* __restrict__ root, const float* __restrict__ dof,
                               const int* __restrict__ idx, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nt = n * nd;
  if (t < nt) {
    const int r = t / nd, j = t - r * nd;
    const int e = idx[r];
    if (e < 0 || e >= N) return;
    st[(13 + j) * N + e] = dof[((size_t)e * nd + j) * 2 + 0];
    st[(13 + nd + j) * N + e] = dof[((size_t)e * nd + j) * 2 + 1];
  } else if (t < nt + n) {
    const int e = idx[t - nt];
    if (e < 0 || e >= N) return;
    set_root_env(st, N, com0, root, e);
  }
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
hipError_t launch_set_root_dof(float* state, int N, int nd, const float* com0, const float* root, const float* dof,
                               const int* idx, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_root_dof, dim3(nblk((long)n * (nd + 1), 256)), dim3(256), 0, s, state, N, nd, com0, root, dof,
                     idx, n);
  return hipGetLastError();
}
hipError_t launch_set_dof(float* state, int N, int nd, const float* src, const int* idx, int n_idx, hipStream_t s) {
  const int n = idx ? n_idx : N;
  if (n <= 0 || nd == 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_dof, dim3(nblk((long)n * nd, 256)), dim3(256), 0, s, state, N, nd, src, idx, n);
  return hipGetLastError();
}

// per-form launchers: defined in gs_physics_impl.h, instantiated in gs_phys_inst.hip
template <class T>
hipError_t launch_sim_plane(const DevModel*, const DevParams&, const SimBuffers&, const float*, hipStream_t);
template <class T>
hipError_t launch_sim_terr(const DevModel*, const DevParams&, const SimBuffers&, const float*, hipStream_t);
template <class T>
hipError_t launch_pd_plane(const DevModel*, const DevParams&, const SimBuffers&, const PdDev&, hipStream_t);
template <class T>
hipError_t launch_pd_terr(const DevModel*, const DevParams&, const SimBuffers&, const PdDev&, hipStream_t);

template <class T>
hipError_t launch_dbg_pool(const DevModel*, const DevParams&, const SimBuffers&, int, float*, int*, hipStream_t);

template <class T>
hipError_t launch_sim(const DevModel* M, const DevParams& P, const SimBuffers& B, const float* tau, hipStream_t st) {
  return P.has_terrain ? launch_sim_terr<T>(M, P, B, tau, st) : launch_sim_plane<T>(M, P, B, tau, st);
}
template <class T>
hipError_t launch_pd(const DevModel* M, const DevParams& P, const SimBuffers& B, const PdDev& A, hipStream_t st) {
  return P.has_terrain ? launch_pd_terr<T>(M, P, B, A, st) : launch_pd_plane<T>(M, P, B, A, st);
}

#define GS_TOPO_ENTRY(T, SIG)                                                                          \
  {SIG, T::kName, &launch_sim<T>, &launch_pd<T>, &launch_dbg_pool<T>, T::NB, T::ND, T::NC, T::NS, T::SENS ? 1 : 0,            \
   LaneCfg<T, false>::ROW_FLOATS, LaneCfg<T, false>::LB, T::NPK, T::cdyn, T::NPAIR, T::pair_a, T::pair_b,      \
   T::pair_k, T::shkind},
TopoEntry g_topologies[] = {GS_FOR_EACH_TOPOLOGY(GS_TOPO_ENTRY)};
const int g_num_topologies = sizeof(g_topologies) / sizeof(g_topologies[0]);
