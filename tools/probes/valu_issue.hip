// valu_issue.hip -- issue cost of scalar vs packed FP32 VALU for ONE wave per SIMD (the lane-team
// physics kernel's regime) and for two waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_issue tools/probes/valu_issue.hip && /tmp/valu_issue
// Prints s_memtime cycles per instruction (median over waves) for independent v_fma_f32,
// v_pk_fma_f32 and dependent v_fma_f32 chains.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

template <int MODE>
__global__ void probe(float* out, long long* cyc) {
  float a[8];
  f2 p[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 0.001f + i;
    p[i] = f2{a[i], a[i] + 1.f};
  }
  const float b = 1.0001f, c = 0.0001f;
  const f2 pb = {b, b}, pc = {c, c};
  const long long t0 = clock64();
  for (int it = 0; it < kIters; ++it) {
    if constexpr (MODE == 0) {  // 8 independent scalar FMAs
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
    } else if constexpr (MODE == 1) {  // 8 independent packed FMAs (16 flops per lane)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(pb), "v"(pc));
    } else {  // one dependent chain of 8 scalar FMAs
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += a[i] + p[i].x + p[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
double run(int blocks, int threads, float* out, long long* cyc) {
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc);
  hipDeviceSynchronize();
  const int nw = blocks * threads / 64;
  std::vector<long long> h(nw);
  hipMemcpy(h.data(), cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  return (double)h[nw / 2] / (kIters * 8.0);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float) * 256 * 1024);
  hipMalloc(&cyc, sizeof(long long) * 256 * 16);
  const char* names[3] = {"v_fma_f32 independent", "v_pk_fma_f32 independent", "v_fma_f32 dependent"};
  // 256 blocks x 64 = one wave per CU; 256 x 512 = two waves per SIMD
  for (int cfg = 0; cfg < 2; ++cfg) {
    const int threads = cfg == 0 ? 64 : 512;
    std::printf("%s\n", cfg == 0 ? "one wave per CU (one SIMD busy):" : "8 waves per CU (two per SIMD):");
    std::printf("  %-26s %.2f cyc/instr per wave\n", names[0], run<0>(256, threads, out, cyc));
    std::printf("  %-26s %.2f cyc/instr per wave\n", names[1], run<1>(256, threads, out, cyc));
    std::printf("  %-26s %.2f cyc/instr per wave\n", names[2], run<2>(256, threads, out, cyc));
  }
  hipFree(out);
  hipFree(cyc);
  return 0;
}
