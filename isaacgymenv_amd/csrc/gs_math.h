// gs_math.h -- small fp32 rigid-body / spatial-algebra helpers shared by the physics kernels.
// Spatial vectors are (angular, linear); inertias are about the env's root origin O in world axes.
//
// Every helper is __host__ __device__: the same solver source runs in the HIP kernels and in the
// host backend of libgymsim (the sim_device=cpu pipeline, gs_host.hip).  The few operations whose
// fast form differs per side are target overloads (clang picks the __device__ or the __host__ one
// for the side being compiled), so the device code is what it was before the host build existed.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define GS_HD __host__ __device__ __forceinline__

namespace {

__device__ __forceinline__ float gs_rsqrt(float x) { return rsqrtf(x); }
__host__ inline float gs_rsqrt(float x) { return 1.f / sqrtf(x); }
__device__ __forceinline__ void gs_sincos(float x, float* s, float* c) { sincosf(x, s, c); }
__host__ inline void gs_sincos(float x, float* s, float* c) { *s = sinf(x); *c = cosf(x); }
// the kinematics kernel's fast sine / cosine (v_sin / v_cos)
__device__ __forceinline__ void gs_fast_sincos(float x, float* s, float* c) { __sincosf(x, s, c); }
__host__ inline void gs_fast_sincos(float x, float* s, float* c) { *s = sinf(x); *c = cosf(x); }
// Hide a uniform pointer from loop-invariant code motion (kernels: keep it in SGPRs, re-read the
// constants through the scalar cache instead of hoisting hundreds of them into registers).
template <class P>
__device__ __forceinline__ const P* gs_opaque(const P* p) {
  uintptr_t mp = reinterpret_cast<uintptr_t>(p);
  asm volatile("" : "+s"(mp));
  return reinterpret_cast<const P*>(mp);
}
template <class P>
__host__ inline const P* gs_opaque(const P* p) { return p; }
GS_HD int gs_imax(int a, int b) { return a > b ? a : b; }
GS_HD int gs_imin(int a, int b) { return a < b ? a : b; }
GS_HD float gs_bits_float(uint32_t u) { return __builtin_bit_cast(float, u); }

GS_HD void cross3(const float* a, const float* b, float* o) {
  const float x = a[1] * b[2] - a[2] * b[1];
  const float y = a[2] * b[0] - a[0] * b[2];
  const float z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
GS_HD void mat3vec(const float* R, const float* v, float* o) {
  const float x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  const float y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  const float z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
GS_HD void mat3mul(const float* A, const float* B, float* C) {
  float T[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int k = 0; k < 9; ++k) C[k] = T[k];
}
GS_HD void quat_to_mat(const float* q, float* R) {
  const float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - z * w);       R[2] = 2.f * (x * z + y * w);
  R[3] = 2.f * (x * y + z * w);       R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - x * w);
  R[6] = 2.f * (x * z - y * w);       R[7] = 2.f * (y * z + x * w);       R[8] = 1.f - 2.f * (x * x + y * y);
}

// spatial inertia about O in world axes: f = (I w + h x v, m v - h x w)
struct SpI {
  float m, h[3], I[6];  // I: xx yy zz xy xz yz
};
GS_HD void spi_mul(const SpI& I, const float* mv, float* f) {
  const float n0 = I.I[0] * mv[0] + I.I[3] * mv[1] + I.I[4] * mv[2];
  const float n1 = I.I[3] * mv[0] + I.I[1] * mv[1] + I.I[5] * mv[2];
  const float n2 = I.I[4] * mv[0] + I.I[5] * mv[1] + I.I[2] * mv[2];
  float hv[3], hw[3];
  cross3(I.h, mv + 3, hv);
  cross3(I.h, mv, hw);
  f[0] = n0 + hv[0]; f[1] = n1 + hv[1]; f[2] = n2 + hv[2];
  f[3] = I.m * mv[3] - hw[0]; f[4] = I.m * mv[4] - hw[1]; f[5] = I.m * mv[5] - hw[2];
}
// motion x motion
GS_HD void crm(const float* a, const float* b, float* o) {
  float t1[3], t2[3], t3[3];
  cross3(a, b, t1); cross3(a, b + 3, t2); cross3(a + 3, b, t3);
  o[0] = t1[0]; o[1] = t1[1]; o[2] = t1[2];
  o[3] = t2[0] + t3[0]; o[4] = t2[1] + t3[1]; o[5] = t2[2] + t3[2];
}
// motion x* force
GS_HD void crf(const float* a, const float* b, float* o) {
  float t1[3], t2[3], t3[3];
  cross3(a, b, t1); cross3(a + 3, b + 3, t2); cross3(a, b + 3, t3);
  o[0] = t1[0] + t2[0]; o[1] = t1[1] + t2[1]; o[2] = t1[2] + t2[2];
  o[3] = t3[0]; o[4] = t3[1]; o[5] = t3[2];
}
GS_HD float dot6(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
GS_HD float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }


}  // namespace
