// hbm_calib.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the physics kernel's own
// access shapes (MI355X_MICROARCH.md: "other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern").  Each kernel moves a KNOWN number of bytes with one of the
// shapes k_pd_step_team uses, at the same sizes (4096 envs):
//   soa_rw      : the SoA sim state, field f of env e at st[f * N + e], one dword per lane
//                 (37 fields read, 37 written: load_state / store_state, team_load / team_store)
//   aos_dof_rw  : the AoS dof tensor [N * 12][2], a lane reading / writing its env's 24 dwords
//                 (the first PD evaluation's read and the dof_out write)
//   aos13_write : the AoS root tensor [N][13] written one dword per (env, field)
// plus a 64 MB streaming dwordx4 copy (the guide's reference shape) as the control.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_calib tools/hbm_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir> -- tools/hbm_calib
// The program prints the known bytes per launch of each kernel (tools/hbm_calib_summary.py joins them
// with the counter CSVs).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

constexpr int kF = 37;  // SoA fields of the ANYmal state: 13 + 2 * 12

__global__ void soa_rw(float* __restrict__ st, int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  float v[kF];
#pragma unroll
  for (int f = 0; f < kF; ++f) v[f] = st[(size_t)f * N + e];
#pragma unroll
  for (int f = 0; f < kF; ++f) st[(size_t)f * N + e] = v[f] * 1.0001f + 1.0f;
}

__global__ void aos_dof_rw(float* __restrict__ dof, int N, int nd) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  float v[24];
#pragma unroll
  for (int j = 0; j < 2 * 12; ++j) v[j] = dof[(size_t)e * 2 * nd + j];
#pragma unroll
  for (int j = 0; j < 2 * 12; ++j) dof[(size_t)e * 2 * nd + j] = v[j] + 1.0f;
}

__global__ void aos13_write(float* __restrict__ out, int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
#pragma unroll
  for (int k = 0; k < 13; ++k) out[(size_t)e * 13 + k] = (float)(e + k);
}

__global__ void stream_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

int main() {
  const int N = 4096, F = kF, ND = 12, REPS = 20;
  float *st, *dof, *root;
  CHECK(hipMalloc(&st, sizeof(float) * F * N));
  CHECK(hipMalloc(&dof, sizeof(float) * 2 * ND * N));
  CHECK(hipMalloc(&root, sizeof(float) * 13 * N));
  CHECK(hipMemset(st, 0, sizeof(float) * F * N));
  CHECK(hipMemset(dof, 0, sizeof(float) * 2 * ND * N));
  const size_t n4 = (size_t)64 << 20 >> 4;  // 64 MB of float4
  float4 *a, *b;
  CHECK(hipMalloc(&a, n4 * 16));
  CHECK(hipMalloc(&b, n4 * 16));
  CHECK(hipMemset(a, 0, n4 * 16));
  for (int r = 0; r < REPS; ++r) {
    hipLaunchKernelGGL(soa_rw, dim3(N / 64), dim3(64), 0, 0, st, N);
    hipLaunchKernelGGL(aos_dof_rw, dim3(N / 64), dim3(64), 0, 0, dof, N, ND);
    hipLaunchKernelGGL(aos13_write, dim3(N / 64), dim3(64), 0, 0, root, N);
    hipLaunchKernelGGL(stream_copy, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, a, b, n4);
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::printf("{\"soa_rw\": {\"read\": %zu, \"write\": %zu}, ", sizeof(float) * F * N, sizeof(float) * F * N);
  std::printf("\"aos_dof_rw\": {\"read\": %zu, \"write\": %zu}, ", sizeof(float) * 2 * ND * N, sizeof(float) * 2 * ND * N);
  std::printf("\"aos13_write\": {\"read\": 0, \"write\": %zu}, ", sizeof(float) * 13 * N);
  std::printf("\"stream_copy\": {\"read\": %zu, \"write\": %zu}, \"reps\": %d}\n", n4 * 16, n4 * 16, REPS);
  CHECK(hipFree(st));
  CHECK(hipFree(dof));
  CHECK(hipFree(root));
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  return 0;
}
