// gt_hound.hip -- UsefulHound control, fused (include/gymtask.h gt_hound_control).
//
// Replaces the torch statements of useful_hound.py:695-726 that run before every simulate of the
// decimation loop: the leg PD and the arm's operational-space controller (_compute_osc_torques,
// useful_hound.py:660-691).  In torch the OSC is ~40 launches per decimation step including two
// batched torch.inverse calls, each of which checks its LU info on the host (a device sync); here
// it is one lane per env: the env's 6x6 arm mass-matrix block, the 6x6 Jacobian block and the
// end-effector velocity are loaded once and the whole controller runs in registers in float64.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#include "../../include/gymtask.h"

void gt_set_last_error(const char* msg);

namespace {

// In-place inverse of a 6x6 row-major matrix, Gauss-Jordan with partial pivoting (as LU-based
// torch.inverse, no error on singular input: a zero pivot yields inf/nan like torch's result would).
__device__ __forceinline__ void inv6(double* A) {
  double B[36];
#pragma unroll
  for (int i = 0; i < 36; ++i) B[i] = (i % 7 == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    int piv = c;
    double best = fabs(A[c * 6 + c]);
#pragma unroll
    for (int r = c + 1; r < 6; ++r) {
      const double v = fabs(A[r * 6 + c]);
      if (v > best) { best = v; piv = r; }
    }
    // row swap by predicated selects (registers stay statically indexed)
#pragma unroll
    for (int r = c + 1; r < 6; ++r) {
      if (r == piv) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const double ta = A[c * 6 + k], tb = B[c * 6 + k];
          A[c * 6 + k] = A[r * 6 + k]; B[c * 6 + k] = B[r * 6 + k];
          A[r * 6 + k] = ta; B[r * 6 + k] = tb;
        }
      }
    }
    const double inv = 1.0 / A[c * 6 + c];
#pragma unroll
    for (int k = 0; k < 6; ++k) { A[c * 6 + k] *= inv; B[c * 6 + k] *= inv; }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      if (r == c) continue;
      const double f = A[r * 6 + c];
#pragma unroll
      for (int k = 0; k < 6; ++k) { A[r * 6 + k] -= f * A[c * 6 + k]; B[r * 6 + k] -= f * B[c * 6 + k]; }
    }
  }
#pragma unroll
  for (int i = 0; i < 36; ++i) A[i] = B[i];
}

// C = A B (6x6)
__device__ __forceinline__ void mul6(const double* A, const double* B, double* C) {
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += A[i * 6 + k] * B[k * 6 + j];
      C[i * 6 + j] = s;
    }
}

__global__ __launch_bounds__(64) void k_hound_control(gt_hound_control_params p, const float* __restrict__ actions,
                                                     const float* __restrict__ dof, const float* __restrict__ leg_default,
                                                     const float* __restrict__ mm, const float* __restrict__ jac,
                                                     const float* __restrict__ rb, float* __restrict__ torques,
                                                     float* __restrict__ arm_control) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.num_envs) return;
  constexpr int ND = 18, NL = 12;
  const float* a = actions + (size_t)e * ND;
  const float* ds = dof + (size_t)e * ND * 2;
  float* tq = torques + (size_t)e * ND;
  // ---- legs: reference float32 expression order
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const float t = p.kp * (p.action_scale * a[j] + leg_default[j] - ds[2 * j]) - p.kd * ds[2 * j + 1];
    tq[j] = fminf(fmaxf(t, -p.torque_limit), p.torque_limit);
  }
  // ---- arm OSC (float64)
  const int nv = p.nv, o = nv - 6;
  double M[36], Minv[36], J[36];
  const float* mme = mm + (size_t)e * nv * nv;
  const float* je = jac + (((size_t)e * p.num_links + p.jac_row) * 6) * nv;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      M[i * 6 + j] = mme[(o + i) * nv + o + j];
      J[i * 6 + j] = je[i * nv + j];
    }
#pragma unroll
  for (int i = 0; i < 36; ++i) Minv[i] = M[i];
  inv6(Minv);
  double JMi[36], Meef[36], T[36];
  mul6(J, Minv, JMi);  // J M^-1
  // M_eef^-1 = J M^-1 J^T
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += JMi[i * 6 + k] * J[j * 6 + k];
      Meef[i * 6 + j] = s;
    }
  inv6(Meef);
  const float* eef = rb + ((size_t)e * p.num_links + p.eef_link) * 13;
  double f[6], g[6], u[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double dpose = (double)(a[NL + k] * p.arm_cmd_limit[k] / p.arm_action_scale);
    f[k] = (double)p.arm_kp[k] * dpose - (double)p.arm_kd[k] * (double)eef[7 + k];
  }
  // u = J^T (M_eef f)
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += Meef[i * 6 + k] * f[k];
    g[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += J[k * 6 + i] * g[k];
    u[i] = s;
  }
  // null space: u_null = M (-kd_null qd + kp_null wrap(default - q)),  u += (1 - J^T M_eef J M^-1) u_null
  const double kTwoPi = 2.0 * M_PI;
  double un[6], mun[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double q = ds[2 * (NL + k)], qd = ds[2 * (NL + k) + 1];
    const double x = (double)p.arm_default[k] - q + M_PI;
    const double w = x - kTwoPi * floor(x / kTwoPi) - M_PI;  // torch.remainder (floor mod)
    un[k] = (double)p.arm_kd_null[k] * -qd + (double)p.arm_kp_null[k] * w;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += M[i * 6 + k] * un[k];
    mun[i] = s;
  }
  mul6(Meef, JMi, T);  // j_eef_inv = M_eef J M^-1
  // (J^T T) mun
  double tm[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += T[i * 6 + k] * mun[k];
    tm[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += J[k * 6 + i] * tm[k];
    u[i] += mun[i] - s;
  }
  float* ac = arm_control + (size_t)e * p.arm_control_stride;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const float lim = p.arm_effort[k];
    const float v = fminf(fmaxf((float)u[k], -lim), lim);
    tq[NL + k] = v;
    ac[k] = v;
  }
}

}  // namespace

extern "C" int gt_hound_control(const gt_hound_control_params* p, const float* actions, const float* dof_state,
                                const float* leg_default, const float* mass_matrix, const float* jacobian,
                                const float* rigid_body, float* torques, float* arm_control, void* stream) {
  if (!p || p->num_envs <= 0 || p->nv < 6 || p->num_links <= 0 || p->jac_row < 0 || p->jac_row >= p->num_links ||
      p->eef_link < 0 || p->eef_link >= p->num_links || p->arm_control_stride < 6 || !actions || !dof_state ||
      !leg_default || !mass_matrix || !jacobian || !rigid_body || !torques || !arm_control) {
    gt_set_last_error("gt_hound_control: invalid parameters or null buffers");
    return -1;
  }
  const int blocks = (p->num_envs + 63) / 64;
  hipLaunchKernelGGL(k_hound_control, dim3(blocks), dim3(64), 0, (hipStream_t)stream, *p, actions, dof_state,
                     leg_default, mass_matrix, jacobian, rigid_body, torques, arm_control);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "gt_hound_control: %s", hipGetErrorString(e));
    gt_set_last_error(buf);
    return -1;
  }
  return 0;
}
