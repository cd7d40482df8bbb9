// gs_kinematics.hip -- link kinematics for the tensor API: rigid-body state, Jacobians, mass matrix.
//
// Replaces what Isaac Gym computes behind refresh_rigid_body_state_tensor /
// refresh_jacobian_tensors / refresh_mass_matrix_tensors (useful_hound.py:440-455, 725-732).
// Conventions (include/gymsim.h): generalized velocity nu = [root link COM linear velocity (world),
// root angular velocity (world), dof velocities] (floating base) or the dof velocities (fixed base);
// Jacobian rows of a link are the linear velocity of the link's COM and its angular velocity, world
// axes; the mass matrix is M = sum_b J_b^T diag(m_b 1, I_b) J_b over the dynamic bodies (J_b at the
// body COM), i.e. the kinetic-energy metric of nu.
//
// Layout: one wave per env (4 envs per 256-thread block).  Lane 0 walks the tree once (FK is a
// serial parent->child recurrence of ~30 FLOP per body) into LDS; then all 64 lanes produce the
// outputs with the env's contiguous output block split across lanes, so stores are coalesced
// (jacobian: nr*6*nv = 3456 floats per env for Hound, 13.8 KB, the dominant HBM traffic).
#include <hip/hip_runtime.h>

#include "gs_kinematics.h"

namespace {

constexpr int kEnvsPerBlock = 4;

__global__ __launch_bounds__(64 * kEnvsPerBlock) void k_kinematics(const DevModel* __restrict__ M,
                                                                    const DevLinks* __restrict__ L,
                                                                    const float* __restrict__ st, int N, int nv,
                                                                    int mode, float* __restrict__ rb,
                                                                    float* __restrict__ jac, float* __restrict__ mm) {
  __shared__ EnvKin kin[kEnvsPerBlock];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int e = blockIdx.x * kEnvsPerBlock + w;
  EnvKin& K = kin[w];
  if (e < N && lane == 0) kin_forward(M, L, st, N, e, K);
  __syncthreads();
  if (e >= N) return;
  kin_outputs(M, L, st, N, nv, mode, e, K, lane, 64, rb, jac, mm);
}

}  // namespace

hipError_t launch_kinematics(const DevModel* M, const DevLinks* L, const float* state, int N, int nv, int mode,
                             float* rb, float* jac, float* mm, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const int blocks = (N + kEnvsPerBlock - 1) / kEnvsPerBlock;
  hipLaunchKernelGGL(k_kinematics, dim3(blocks), dim3(64 * kEnvsPerBlock), 0, s, M, L, state, N, nv, mode, rb, jac,
                     mm);
  return hipGetLastError();
}
