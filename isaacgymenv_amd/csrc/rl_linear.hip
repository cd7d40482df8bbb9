// libgymrl.so -- the PPO learner's hidden Linear + ELU layers on the matrix cores (include/gymrl.h ABI 5).
//
// rl_games' actor / critic MLPs (network_builder.py A2CBuilder: Linear -> ELU per hidden layer; AnymalTerrainPPO.yaml
// units 512-256-128, separate networks, fp16 autocast under mixed_precision) train on 16384-row minibatches.  On
// hipBLASLt each hidden layer was a GEMM (~12 us at these skinny shapes), an ELU pass and its backward, and a
// split-K weight-gradient GEMM with its finish (network.py).  Here a layer is:
//   forward   Y  = ELU(X W^T + b)                     one kernel (k_gemm_nt<ELU>), bias and ELU in the epilogue
//   backward  dZ = dY * ELU'(Y)  (ELU' = 1 for Y > 0, Y + 1 otherwise: torch's elu_backward on the result)
//             dX = dZ W                               k_gemm_nn (dZ formed on load, W through transpose reads)
//             dW = dZ^T X, db = colsum dZ             k_gemm_tn: S row-block partials [S][N][K] / [S][N] in f32,
//                                                     finished in a fixed order by rl_splitk_accum (rl_grad.hip)
// Operands fp16, accumulation f32 (v_mfma_f32_32x32x16_f16), outputs rounded once to fp16 (Y, dX) or kept f32
// (weight / bias partials).  Tiles: 256 threads = 4 waves in 2 x 2, each wave 2 x 2 (or 1 x 2) MFMA tiles of
// 32 x 32; the reduction in steps of 32 through double-buffered LDS.  NT: both operands are contiguous along the
// reduction index (X rows, W rows; dZ rows, W^T rows) and go to LDS as they are; TN (weight gradient): both
// operands are [M][*] row-major and the reduction runs over M, so each 16-B global chunk is written to LDS
// transposed (8 scalar stores) and the fragments read contiguous along M.
//
// MFMA 32x32x16 operand / result maps (gfx950): lane l, r = l & 31, h = l >> 5 holds A[row r][k = 8h + j] and
// B[k = 8h + j][col r] (j = 0..7); result register i of lane l is C[row (i & 3) + 8 (i >> 2) + 4 h][col r].
// (tests/test_ppo_gpu.py test_linear_kernels_exact_on_integers pins them with exact integer data.)
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "gymrl.h"

int rl_set_error(const char* msg);  // rl_gae.hip

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int kTnStep = 64;        // TN: rows of the reduction per LDS stage (four MFMA k-steps)
constexpr int kNtStep = 64;        // NT: reduction step per LDS stage (four MFMA k-steps); LDS rows of 72 halves

__device__ __forceinline__ float elu_f(float z) { return z > 0.f ? z : expm1f(z); }
// torch elu_backward with is_result: y > 0 -> 1, else y + 1 (= exp(z))
__device__ __forceinline__ float elu_d(float y) { return y > 0.f ? 1.f : y + 1.f; }

// 8 consecutive halves of a row from global memory: 16 B as two 8-B loads (rows are 8-B aligned: host check),
// zero beyond `valid`
__device__ __forceinline__ h8 load8(const _Float16* __restrict__ p, int valid) {
  h8 v;
  if (valid >= 8) {
    const uint2 a = *reinterpret_cast<const uint2*>(p);
    const uint2 b = *reinterpret_cast<const uint2*>(p + 4);
    uint4 u = make_uint4(a.x, a.y, b.x, b.y);
    v = __builtin_bit_cast(h8, u);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = j < valid ? p[j] : (_Float16)0.f;
  }
  return v;
}

// XCD-aware tile order (MI355X_MICROARCH.md, workgroup dispatch: blocks are dealt round-robin over the 8 XCDs):
// the 1-D grid's block b is renumbered so that each XCD takes a contiguous run of the row-major (group, m, n) tile
// order -- n fastest: the blocks resident on an XCD at once cover whole rows of the output (full-line, page-local
// writes) and share their A row tiles in that XCD's L2.  Bijective for any tile count.
__device__ __forceinline__ void tile_of(int MT, int NT, int& g, int& mt, int& nt) {
  const int T = gridDim.x, id = blockIdx.x, q = T / 8, r = T % 8, xcd = id % 8;
  const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
  g = w / (MT * NT);
  const int rem = w - g * (MT * NT);
  mt = rem / NT;
  nt = rem - mt * NT;
}

// The output tile through LDS: a lane's fp16 results (4 consecutive columns of one row per register group) are
// written to `stage` ([BM][BN + 8] halves, the K loop's buffers reused), then the workgroup stores whole rows with
// 16-byte stores -- each wave store a contiguous 1 KB of 4 rows.  Stored straight from the registers (8-byte
// stores, 32 rows apart per wave instruction) the 32 MB of the first layer's output went out at ~1 TB/s.
// o(j, i, g) gives the 4 halves of register group g of fragment (j, i).  Falls back to the direct stores when C
// or its row stride is not 16-byte aligned.
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
template <int BM, int BN, class F>
__device__ __forceinline__ void store_tile(_Float16* __restrict__ stage, _Float16* __restrict__ C, int ldc, int m0,
                                           int c0, int wm, int wn, int r, int hh, F&& o) {
  constexpr int TM = BM / 64, TN = BN / 64, SLD = BN + 8;
  if (((reinterpret_cast<uintptr_t>(C) | (uintptr_t)(ldc * 2)) & 15) != 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = m0 + wm * (BM / 2) + i * 32 + r, cg = c0 + wn * (BN / 2) + j * 32 + 8 * g + 4 * hh;
          *reinterpret_cast<h4*>(C + (size_t)m * ldc + cg) = o(j, i, g);
        }
    return;
  }
  __syncthreads();  // every wave is done with the K loop's buffers
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ml = wm * (BM / 2) + i * 32 + r, cl = wn * (BN / 2) + j * 32 + 8 * g + 4 * hh;
        *reinterpret_cast<h4*>(stage + ml * SLD + cl) = o(j, i, g);
      }
  __syncthreads();
  constexpr int CPR = BN / 8, IT = BM * CPR / kThreads;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = threadIdx.x + it * kThreads, row = c / CPR, cc = (c % CPR) * 8;
    *reinterpret_cast<uint4*>(C + (size_t)(m0 + row) * ldc + c0 + cc) = *reinterpret_cast<const uint4*>(stage + row * SLD + cc);
  }
}

// ---------------------------------------------------------------- NT: C[m][c] = sum_r A[m][r] Bt[c][r]
// ACT: ELU epilogue.  bias: fp16 [C] or null.  C fp16 [M][ldc].  M % BM == 0, Cn % BN == 0 (host).  The MFMA takes the Bt tile as its row operand,
// so a lane's result registers 4g .. 4g+3 are 4 consecutive columns c of one row m: one 8-byte store each.
// Groups (blockIdx.z = g): group g reads A + g gA, Bt + g gB, bias + g gBias and writes C + g gC -- the actor and
// critic MLPs' equal-shaped layers in one launch (rl_linear_fwd_g).
template <int BM, int BN, bool ACT>
__global__ __launch_bounds__(kThreads) void k_gemm_nt(const _Float16* __restrict__ A,
                                                      int lda, const _Float16* __restrict__ Bt, int ldb,
                                                      const _Float16* __restrict__ bias, _Float16* __restrict__ C,
                                                      int ldc, int R, int64_t gA, int64_t gB, int64_t gBias,
                                                      int64_t gC, int MT, int NT) {
  int gi, mt, nt;
  tile_of(MT, NT, gi, mt, nt);
  {
    const int64_t g = gi;
    A += g * gA;
    Bt += g * gB;
    if (bias) bias += g * gBias;
    C += g * gC;
  }
  constexpr int TM = BM / 64, TN = BN / 64;                  // MFMA tiles per wave
  constexpr int KS = kNtStep, LD = KS + 8, CPR = KS / 8;      // reduction step, LDS row stride, chunks per row
  constexpr int CA = BM * KS / 8 / kThreads, CB = BN * KS / 8 / kThreads;  // 16-B chunks per thread
  static_assert(CA >= 1 && CB >= 1, "tile too small for the thread block");
  __shared__ _Float16 sA[2][BM * LD];
  __shared__ _Float16 sB[2][BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = mt * BM, c0 = nt * BN;
  const int r = lane & 31, hh = lane >> 5;
  f16v acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[j][i][q] = 0.f;

  // the bias of this lane's output columns, loaded before the K loop (its latency hides there): columns
  // c0 + wn BN/2 + 32 j + 8 g + 4 hh + e
  float bcol[TN][4][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        bcol[j][g][e] = bias ? (float)bias[c0 + wn * (BN / 2) + j * 32 + 8 * g + 4 * hh + e] : 0.f;
  h8 ra[CA], rb[CB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 8;
      const int valid = R - (k0 + kc);
      const size_t off = (size_t)(m0 + row) * lda + k0 + kc;
      ra[i] = load8(A + off, valid);
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 8;
      rb[i] = load8(Bt + (size_t)(c0 + row) * ldb + k0 + kc, R - (k0 + kc));
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 8;
      *reinterpret_cast<h8*>(&sA[buf][row * LD + kc]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 8;
      *reinterpret_cast<h8*>(&sB[buf][row * LD + kc]) = rb[i];
    }
  };
  const int steps = (R + KS - 1) / KS;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    const int buf = s & 1;
    if (s + 1 < steps) gload((s + 1) * KS);
#pragma unroll
    for (int ks = 0; ks < KS / 16; ++ks) {
      h8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const h8*>(&sA[buf][(wm * (BM / 2) + i * 32 + r) * LD + ks * 16 + 8 * hh]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const h8*>(&sB[buf][(wn * (BN / 2) + j * 32 + r) * LD + ks * 16 + 8 * hh]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[j], fa[i], acc[j][i], 0, 0, 0);
    }
    if (s + 1 < steps) lstore(buf ^ 1);
    __syncthreads();
  }
  // epilogue: + bias, ELU, one rounding to fp16; registers 4g .. 4g+3 -> columns cg .. cg+3 of row m
  static_assert(BM * (BN + 8) <= 2 * BM * LD, "the output stage fits the A buffers");
  store_tile<BM, BN>(&sA[0][0], C, ldc, m0, c0, wm, wn, r, hh, [&](int j, int i, int g) {
    h4 ov;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float z = acc[j][i][4 * g + e] + bcol[j][g][e];
      if constexpr (ACT) z = elu_f(z);
      ov[e] = (_Float16)z;
    }
    return ov;
  });
}

// ---------------------------------------------------------------- NT in f32: the rollout's act forward
// rl_games play_steps runs the act forward in f32 (no autocast).  C[m][c] = act(sum_r A[m][r] Bt[c][r] + bias[c])
// with f32 operands on v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation; the order of the sum is this
// kernel's, so the result agrees with a library f32 GEMM to f32 rounding), bias and ELU in the epilogue.  64 x 64
// tiles, 4 waves in 2 x 2, one 32 x 32 MFMA tile each; the reduction in stages of KS = 32 or 64 through
// double-buffered LDS (row stride KS + 4 floats: the 16-B fragment reads of 16 rows hit disjoint banks).  A lane reads 4 consecutive k of its row (one 16-B LDS read per operand) and feeds them
// to 4 MFMAs: in MFMA s, half h of the wave carries k = 8 ks + 4 h + s -- the A and Bt fragments use the same map,
// so every k is summed exactly once.  The output tile goes out through LDS as whole 256-B row segments.
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 load4f(const float* __restrict__ p, int valid) {
  if (valid >= 4) return *reinterpret_cast<const f4*>(p);
  f4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = j < valid ? p[j] : 0.f;
  return v;
}

template <bool ACT, int KS>
__global__ __launch_bounds__(kThreads) void k_gemm_nt_f32(const float* __restrict__ A, int lda,
                                                          const float* __restrict__ Bt, int ldb,
                                                          const float* __restrict__ bias, float* __restrict__ C,
                                                          int ldc, int R, int64_t gA, int64_t gB, int64_t gBias,
                                                          int64_t gC, int MT, int NT) {
  constexpr int BM = 64, BN = 64, LD = KS + 4, CPR = KS / 4;
  constexpr int CA = BM * KS / 4 / kThreads, CB = BN * KS / 4 / kThreads;  // 16-B chunks per thread (2, 2)
  int gi, mt, nt;
  tile_of(MT, NT, gi, mt, nt);
  {
    const int64_t g = gi;
    A += g * gA;
    Bt += g * gB;
    if (bias) bias += g * gBias;
    C += g * gC;
  }
  __shared__ float sA[2][BM * LD];
  __shared__ float sB[2][BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = mt * BM, c0 = nt * BN;
  const int r = lane & 31, hh = lane >> 5;
  f16v acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  float bcol[4][4];  // this lane's output columns c0 + 32 wn + 8 g + 4 hh + e
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) bcol[g][e] = bias ? bias[c0 + wn * 32 + 8 * g + 4 * hh + e] : 0.f;
  f4 ra[CA], rb[CB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 4;
      ra[i] = load4f(A + (size_t)(m0 + row) * lda + k0 + kc, R - (k0 + kc));
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 4;
      rb[i] = load4f(Bt + (size_t)(c0 + row) * ldb + k0 + kc, R - (k0 + kc));
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 4;
      *reinterpret_cast<f4*>(&sA[buf][row * LD + kc]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 4;
      *reinterpret_cast<f4*>(&sB[buf][row * LD + kc]) = rb[i];
    }
  };
  const int steps = (R + KS - 1) / KS;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    const int buf = s & 1;
    if (s + 1 < steps) gload((s + 1) * KS);
#pragma unroll
    for (int ks = 0; ks < KS / 8; ++ks) {
      const f4 fa = *reinterpret_cast<const f4*>(&sA[buf][(wm * 32 + r) * LD + ks * 8 + 4 * hh]);
      const f4 fb = *reinterpret_cast<const f4*>(&sB[buf][(wn * 32 + r) * LD + ks * 8 + 4 * hh]);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[q], fa[q], acc, 0, 0, 0);
    }
    if (s + 1 < steps) lstore(buf ^ 1);
    __syncthreads();
  }
  // epilogue: registers 4g .. 4g+3 are columns 32 wn + 8 g + 4 hh + (0..3) of tile row 32 wm + r
  constexpr int SLD = BN + 4;
  static_assert(BM * SLD <= 2 * BM * LD, "the output stage fits the A buffers");
  float* stage = &sA[0][0];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    f4 ov;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float z = acc[4 * g + e] + bcol[g][e];
      if constexpr (ACT) z = elu_f(z);
      ov[e] = z;
    }
    *reinterpret_cast<f4*>(stage + (wm * 32 + r) * SLD + wn * 32 + 8 * g + 4 * hh) = ov;
  }
  __syncthreads();
  constexpr int OPR = BN / 4, IT = BM * OPR / kThreads;  // 16 chunks per row, 4 per thread
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = tid + it * kThreads, row = c / OPR, cc = (c % OPR) * 4;
    *reinterpret_cast<f4*>(C + (size_t)(m0 + row) * ldc + c0 + cc) = *reinterpret_cast<const f4*>(stage + row * SLD + cc);
  }
}

// ---------------------------------------------------------------- TN: weight / bias gradient partials
// part[s][n][k] = sum_{m in block s} dZ[m][n] X[m][k] with dZ = dY * elu'(Y) (dY, Y [M][N], X [M][K]);
// bpart[s][n] = sum_{m in block s} dZ[m][n] (written by the blocks of k-tile 0); consecutive blocks wstride /
// bstride floats apart.  Tiles 128 (k) x 128 (n); the rows of a block in stages of 64.  Both operands sum over their ROW
// index m, so they are staged in LDS as they lie in memory ([m][n], [m][k]: 16-byte stores) and the MFMA fragments
// (8 consecutive m of one column) come from the hardware transpose read ds_read_b64_tr_b16: lane 4q + p of each
// 16-lane group addresses row q, columns 4p .. 4p+3 of a 4 x 16 block and receives one column of it.  Row stride
// 160 halves (320 B): the four rows of a block fall on disjoint bank ranges.  X^T is the MFMA's row operand, so a
// lane's result registers 4g .. 4g+3 are 4 consecutive k of one n: one 16-byte store each.
constexpr int kTN = 128;
constexpr int kTLd = kTN + 32;
typedef short s4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ h8 tr_frag(const _Float16* tile, int lane) {
  // the 8 consecutive rows (8h .. 8h+7, h = lane >> 5) of column (lane & 31) of `tile` ([row][kTLd] halves)
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const _Float16* a = tile + (8 * (g >> 1) + q) * kTLd + 16 * (g & 1) + 4 * p;
  typedef __attribute__((address_space(3))) s4 lds_s4;
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a + 4 * kTLd));
  const s4 v[2] = {lo, hi};
  return __builtin_bit_cast(h8, v);
}

// Groups: blockIdx.z = g * splits + s; group g reads dY / Y + g gY (row stride ldy), X + g gX and writes its
// partials at + g gP / + g gBP within each block.
__global__ __launch_bounds__(kThreads) void k_gemm_tn(const _Float16* __restrict__ dY, const _Float16* __restrict__ Y,
                                                      int N, int ldy, const _Float16* __restrict__ X, int ldx, int K,
                                                      int rows_per_split, float* __restrict__ part,
                                                      float* __restrict__ bpart, int64_t wstride, int64_t bstride,
                                                      int splits, int64_t gY, int64_t gX, int64_t gP, int64_t gBP) {
  {
    const int64_t g = blockIdx.z / splits;
    dY += g * gY;
    Y += g * gY;
    X += g * gX;
    part += g * gP;
    if (bpart) bpart += g * gBP;
  }
  constexpr int TS = kTnStep, CH = TS / 16;  // rows per stage, 16-B chunks per thread per operand
  __shared__ _Float16 sZ[2][TS * kTLd];  // [m][n]
  __shared__ _Float16 sX[2][TS * kTLd];  // [m][k]
  __shared__ float sbias[16][kTN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.x * kTN, k0 = blockIdx.y * kTN, s = blockIdx.z % splits;
  const int mb = s * rows_per_split;
  const int r = lane & 31, hh = lane >> 5;
  const bool do_bias = blockIdx.y == 0 && bpart != nullptr;
  f16v acc[2][2];  // [k tile][n tile]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  // each thread: CH chunks of 8 along n (resp. k) at rows m = tid / 16 + 16 i of the stage
  const int crow = tid >> 4, ccol = (tid & 15) * 8;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  h8 ra[CH], rb[CH], ry[CH];
  // the loads of a stage are issued before the previous stage's MFMAs and consumed after them (dZ and the bias
  // sums formed in gfinish), so their latency hides behind the matrix work
  auto gload = [&](int m) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const size_t row = (size_t)(m + crow + 16 * i);
      const size_t off = row * ldy + n0 + ccol;
      ra[i] = load8(dY + off, N - (n0 + ccol));
      ry[i] = load8(Y + off, N - (n0 + ccol));
      rb[i] = load8(X + row * ldx + k0 + ccol, K - (k0 + ccol));
    }
  };
  auto gfinish = [&]() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ra[i][j] = (_Float16)((float)ra[i][j] * elu_d((float)ry[i][j]));
        bsum[j] += (float)ra[i][j];  // the bias gradient sums the same rounded dZ the weight gradient uses
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int m = crow + 16 * i;
      *reinterpret_cast<h8*>(&sZ[buf][m * kTLd + ccol]) = ra[i];
      *reinterpret_cast<h8*>(&sX[buf][m * kTLd + ccol]) = rb[i];
    }
  };
  const int steps = rows_per_split / TS;
  gload(mb);
  gfinish();
  lstore(0);
  __syncthreads();
  for (int st = 0; st < steps; ++st) {
    const int buf = st & 1;
    if (st + 1 < steps) gload(mb + (st + 1) * TS);
#pragma unroll
    for (int ks = 0; ks < TS / 16; ++ks) {
      h8 fx[2], fz[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fx[i] = tr_frag(&sX[buf][ks * 16 * kTLd + wk * 64 + i * 32], lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fz[j] = tr_frag(&sZ[buf][ks * 16 * kTLd + wn * 64 + j * 32], lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fx[i], fz[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < steps) {
      gfinish();
      lstore(buf ^ 1);
    }
    __syncthreads();
  }
  float* out = part + (size_t)s * wstride;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + r;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k = k0 + wk * 64 + i * 32 + 8 * g + 4 * hh;
        if (k < K)  // K % 4 == 0: a group of 4 is wholly inside or outside
          *reinterpret_cast<float4*>(out + (size_t)n * K + k) =
              make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
      }
  }
  if (do_bias) {  // the 16 row groups' sums of each column, added in a fixed order
#pragma unroll
    for (int j = 0; j < 8; ++j) sbias[crow][ccol + j] = bsum[j];
    __syncthreads();
    if (tid < kTN) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) t += sbias[g][tid];
      bpart[(size_t)s * bstride + n0 + tid] = t;
    }
  }
}

// ---------------------------------------------------------------- NN: dX[m][k] = sum_n dZ[m][n] W[n][k]
// dZ = dY * elu'(Y) formed on load (dY, Y [M][N]); W [N][K] as the forward uses it, staged in LDS as it lies
// ([n][k], 16-byte stores) and read with the transpose read (8 consecutive n of one k per lane), so no W^T copy
// is needed.  As in k_gemm_nt the k rows are the MFMA's row operand: registers 4g .. 4g+3 are 4 consecutive k of
// one row m, one 8-byte store.  M % BM == 0, K % 128 == 0 (host).
// Groups (blockIdx.z = g): dY / Y + g gY (row stride ldy), W + g gW, dX + g gDX (row stride lddx).
template <int BM>
__global__ __launch_bounds__(kThreads) void k_gemm_nn(const _Float16* __restrict__ dY, const _Float16* __restrict__ Y,
                                                      int N, int ldy, const _Float16* __restrict__ W, int K,
                                                      _Float16* __restrict__ dX, int lddx, int64_t gY, int64_t gW,
                                                      int64_t gDX, int MT, int NT) {
  int gi, mt, nt;
  tile_of(MT, NT, gi, mt, nt);
  {
    const int64_t g = gi;
    dY += g * gY;
    Y += g * gY;
    W += g * gW;
    dX += g * gDX;
  }
  constexpr int BN = 128, TM = BM / 64, TN = BN / 64;
  constexpr int KS = kNtStep, LD = KS + 8, CPR = KS / 8;
  constexpr int CA = BM * KS / 8 / kThreads, CB = KS * BN / 8 / kThreads;
  __shared__ _Float16 sA[2][BM * LD];     // [m][n]
  __shared__ _Float16 sB[2][KS * kTLd];   // [n][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = mt * BM, c0 = nt * BN;
  const int r = lane & 31, hh = lane >> 5;
  f16v acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[j][i][q] = 0.f;
  h8 ra[CA], ry[CA], rb[CB];
  // loads issued before the previous step's MFMAs, dZ formed after them (gfinish): the latency hides behind them
  auto gload = [&](int n0) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 8;
      const int valid = N - (n0 + kc);
      const size_t off = (size_t)(m0 + row) * ldy + n0 + kc;
      ra[i] = load8(dY + off, valid);
      ry[i] = load8(Y + off, valid);
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * kThreads, row = c >> 4, kc = (c & 15) * 8;
      rb[i] = n0 + row < N ? load8(W + (size_t)(n0 + row) * K + c0 + kc, 8) : h8{};
    }
  };
  auto gfinish = [&]() {
#pragma unroll
    for (int i = 0; i < CA; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) ra[i][j] = (_Float16)((float)ra[i][j] * elu_d((float)ry[i][j]));
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int c = tid + i * kThreads, row = c / CPR, kc = (c % CPR) * 8;
      *reinterpret_cast<h8*>(&sA[buf][row * LD + kc]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = tid + i * kThreads, row = c >> 4, kc = (c & 15) * 8;
      *reinterpret_cast<h8*>(&sB[buf][row * kTLd + kc]) = rb[i];
    }
  };
  const int steps = (N + KS - 1) / KS;
  gload(0);
  gfinish();
  lstore(0);
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    const int buf = s & 1;
    if (s + 1 < steps) gload((s + 1) * KS);
#pragma unroll
    for (int ks = 0; ks < KS / 16; ++ks) {
      h8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const h8*>(&sA[buf][(wm * (BM / 2) + i * 32 + r) * LD + ks * 16 + 8 * hh]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = tr_frag(&sB[buf][ks * 16 * kTLd + wn * (BN / 2) + j * 32], lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[j], fa[i], acc[j][i], 0, 0, 0);
    }
    if (s + 1 < steps) {
      gfinish();
      lstore(buf ^ 1);
    }
    __syncthreads();
  }
  static_assert(BM * (BN + 8) <= 2 * BM * LD, "the output stage fits the A buffers");
  store_tile<BM, BN>(&sA[0][0], dX, lddx, m0, c0, wm, wn, r, hh,
                     [&](int j, int i, int g) {
                       const h4 ov = {(_Float16)acc[j][i][4 * g], (_Float16)acc[j][i][4 * g + 1],
                                      (_Float16)acc[j][i][4 * g + 2], (_Float16)acc[j][i][4 * g + 3]};
                       return ov;
                     });
}

// W [N][K] fp16 -> W^T [K][N] fp16 (32 x 32 tiles through LDS)
__global__ __launch_bounds__(256) void k_transpose_f16(const _Float16* __restrict__ w, int N, int K,
                                                       _Float16* __restrict__ wt) {
  __shared__ _Float16 t[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int bk = blockIdx.x * 32, bn = blockIdx.y * 32;
#pragma unroll
  for (int i = 0; i < 32; i += 8) {
    const int n = bn + ty + i, k = bk + tx;
    if (n < N && k < K) t[ty + i][tx] = w[(size_t)n * K + k];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 32; i += 8) {
    const int k = bk + ty + i, n = bn + tx;
    if (n < N && k < K) wt[(size_t)k * N + n] = t[tx][ty + i];
  }
}

bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }

int launch_fail(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  char msg[256];
  snprintf(msg, sizeof(msg), "%s: launch failed: %s", what, hipGetErrorString(e));
  return rl_set_error(msg) + 1;
}

}  // namespace

extern "C" int rl_linear_fwd_g(const void* x, int32_t M, int32_t K, int32_t ldx, const void* w, int32_t N,
                               const void* bias, int32_t act, void* y, const rl_linear_groups* grp, void* stream) {
  if (!x || !w || !y || M <= 0 || K <= 0 || N <= 0) return rl_set_error("rl_linear_fwd: null pointer or empty shape");
  const int G = grp ? grp->groups : 1;
  const int ldy = grp && grp->ldy ? grp->ldy : N;
  if (G < 1 || G > 65535 || ldy < N || ldy % 4) return rl_set_error("rl_linear_fwd: bad groups or output row stride");
  if (M % 64 || N % 128 || ldx % 4 || K % 4 || !aligned8(x) || !aligned8(w) || !aligned8(y))
    return rl_set_error("rl_linear_fwd: M % 64, N % 128, K % 4 and 8-byte aligned rows required");
  const int64_t gx = grp ? grp->x_gstride : 0, gw = grp ? grp->w_gstride : 0, gb = grp ? grp->b_gstride : 0,
                gy = grp ? grp->y_gstride : 0;
  if (G > 1 && ((gx | gw | gb | gy) % 4 != 0)) return rl_set_error("rl_linear_fwd: group strides must be % 4");
  hipStream_t st = (hipStream_t)stream;
  const auto* X = static_cast<const _Float16*>(x);
  const auto* W = static_cast<const _Float16*>(w);
  const auto* B = static_cast<const _Float16*>(bias);
  auto* Y = static_cast<_Float16*>(y);
  // 128 x 128 tiles when that still gives >= 256 workgroups (over all groups), else 64-row tiles
  // (RL_NT_WG: that workgroup threshold, an A/B switch)
  static const int nt_wg = getenv("RL_NT_WG") ? atoi(getenv("RL_NT_WG")) : 256;
  if ((M / 128) * (N / 128) * G >= nt_wg && M % 128 == 0) {
    const int MT = M / 128, NT = N / 128;
    const dim3 g(MT * NT * G);
    if (act) hipLaunchKernelGGL((k_gemm_nt<128, 128, true>), g, dim3(kThreads), 0, st, X, ldx, W, K, B, Y, ldy, K, gx, gw, gb, gy, MT, NT);
    else hipLaunchKernelGGL((k_gemm_nt<128, 128, false>), g, dim3(kThreads), 0, st, X, ldx, W, K, B, Y, ldy, K, gx, gw, gb, gy, MT, NT);
  } else {
    const int MT = M / 64, NT = N / 128;
    const dim3 g(MT * NT * G);
    if (act) hipLaunchKernelGGL((k_gemm_nt<64, 128, true>), g, dim3(kThreads), 0, st, X, ldx, W, K, B, Y, ldy, K, gx, gw, gb, gy, MT, NT);
    else hipLaunchKernelGGL((k_gemm_nt<64, 128, false>), g, dim3(kThreads), 0, st, X, ldx, W, K, B, Y, ldy, K, gx, gw, gb, gy, MT, NT);
  }
  return launch_fail("rl_linear_fwd");
}

extern "C" int rl_linear_fwd_f32_g(const float* x, int32_t M, int32_t K, int32_t ldx, const float* w, int32_t N,
                                   const float* bias, int32_t act, float* y, const rl_linear_groups* grp,
                                   void* stream) {
  if (!x || !w || !y || M <= 0 || K <= 0 || N <= 0) return rl_set_error("rl_linear_fwd_f32: null pointer or empty shape");
  const int G = grp ? grp->groups : 1;
  const int ldy = grp && grp->ldy ? grp->ldy : N;
  if (G < 1 || G > 65535 || ldy < N || ldy % 4) return rl_set_error("rl_linear_fwd_f32: bad groups or output row stride");
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (M % 64 || N % 64 || ldx % 4 || K % 4 || ldx < K || !a16(x) || !a16(w) || !a16(y) || (bias && (N % 4)))
    return rl_set_error("rl_linear_fwd_f32: M % 64, N % 64, K % 4, ldx % 4 and 16-byte aligned x / w / y required");
  const int64_t gx = grp ? grp->x_gstride : 0, gw = grp ? grp->w_gstride : 0, gb = grp ? grp->b_gstride : 0,
                gy = grp ? grp->y_gstride : 0;
  if (G > 1 && ((gx | gw | gy) % 4 != 0)) return rl_set_error("rl_linear_fwd_f32: group strides must be % 4");
  const int MT = M / 64, NT = N / 64;
  const dim3 g(MT * NT * G);
  hipStream_t st = (hipStream_t)stream;
  // K stage: 64 (two MFMA kilocycles per wave per stage against the next stage's loads; 70 KB of LDS, two
  // workgroups per CU) when the grid has at most two workgroups per CU, else 32 (37 KB, four per CU)
  int ks = (int64_t)MT * NT * G <= 512 ? 64 : 32;
  if (const char* e = getenv("RL_F32_KSTEP")) ks = atoi(e) == 64 ? 64 : 32;  // A/B switch (tools/probes)
  if (ks == 64) {
    if (act) hipLaunchKernelGGL((k_gemm_nt_f32<true, 64>), g, dim3(kThreads), 0, st, x, ldx, w, K, bias, y, ldy, K, gx, gw, gb, gy, MT, NT);
    else hipLaunchKernelGGL((k_gemm_nt_f32<false, 64>), g, dim3(kThreads), 0, st, x, ldx, w, K, bias, y, ldy, K, gx, gw, gb, gy, MT, NT);
  } else {
    if (act) hipLaunchKernelGGL((k_gemm_nt_f32<true, 32>), g, dim3(kThreads), 0, st, x, ldx, w, K, bias, y, ldy, K, gx, gw, gb, gy, MT, NT);
    else hipLaunchKernelGGL((k_gemm_nt_f32<false, 32>), g, dim3(kThreads), 0, st, x, ldx, w, K, bias, y, ldy, K, gx, gw, gb, gy, MT, NT);
  }
  return launch_fail("rl_linear_fwd_f32");
}

extern "C" int rl_linear_fwd(const void* x, int32_t M, int32_t K, int32_t ldx, const void* w, int32_t N,
                             const void* bias, int32_t act, void* y, void* stream) {
  return rl_linear_fwd_g(x, M, K, ldx, w, N, bias, act, y, nullptr, stream);
}

extern "C" int rl_linear_transpose(const void* w, int32_t N, int32_t K, void* wt, void* stream) {
  if (!w || !wt || N <= 0 || K <= 0) return rl_set_error("rl_linear_transpose: null pointer or empty shape");
  hipLaunchKernelGGL(k_transpose_f16, dim3((K + 31) / 32, (N + 31) / 32), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const _Float16*>(w), N, K, static_cast<_Float16*>(wt));
  return launch_fail("rl_linear_transpose");
}

extern "C" int rl_linear_bwd_g(const void* dy, const void* y, int32_t M, int32_t N, const void* x, int32_t K,
                               int32_t ldx, const void* w, void* dx, int32_t splits, float* wpart, float* bpart,
                               int64_t pstride, const rl_linear_groups* grp, void* stream) {
  if (!dy || !y || !x || M <= 0 || N <= 0 || K <= 0) return rl_set_error("rl_linear_bwd: null pointer or empty shape");
  const int G = grp ? grp->groups : 1;
  const int ldy = grp && grp->ldy ? grp->ldy : N, lddx = grp && grp->lddx ? grp->lddx : K;
  if (G < 1 || G > 65535 || ldy < N || ldy % 4 || lddx < K || lddx % 4)
    return rl_set_error("rl_linear_bwd: bad groups or row strides");
  if (M % 128 || N % 128 || K % 4 || ldx % 4 || !aligned8(dy) || !aligned8(y) || !aligned8(x))
    return rl_set_error("rl_linear_bwd: M % 128, N % 128, K % 4 and 8-byte aligned rows required");
  if (splits <= 0 || M % (splits * kTnStep) != 0 || (int64_t)splits * G > 65535)
    return rl_set_error("rl_linear_bwd: M must split into row blocks of multiples of 64");
  // (the bias partials come out of the weight-gradient kernel's pass: bpart alone would be left unwritten)
  if (bpart && !wpart) return rl_set_error("rl_linear_bwd: bias partials (bpart) need the weight partials (wpart)");
  const int64_t gx = grp ? grp->x_gstride : 0, gw = grp ? grp->w_gstride : 0, gy = grp ? grp->y_gstride : 0,
                gdx = grp ? grp->dx_gstride : 0, gp = grp ? grp->part_gstride : 0, gbp = grp ? grp->bpart_gstride : 0;
  if (G > 1 && ((gx | gw | gy | gdx | gp | gbp) % 4 != 0)) return rl_set_error("rl_linear_bwd: group strides must be % 4");
  hipStream_t st = (hipStream_t)stream;
  const auto* DY = static_cast<const _Float16*>(dy);
  const auto* Yv = static_cast<const _Float16*>(y);
  const auto* X = static_cast<const _Float16*>(x);
  if (dx) {
    if (!w || !aligned8(w) || !aligned8(dx) || K % 128)
      return rl_set_error("rl_linear_bwd: dX needs W, 8-byte aligned rows and K % 128");
    const auto* Wp = static_cast<const _Float16*>(w);
    auto* DX = static_cast<_Float16*>(dx);
    static const int nn_wg = getenv("RL_NN_WG") ? atoi(getenv("RL_NN_WG")) : 256;  // (A/B switch)
    if ((M / 128) * (K / 128) * G >= nn_wg)
      hipLaunchKernelGGL((k_gemm_nn<128>), dim3((M / 128) * (K / 128) * G), dim3(kThreads), 0, st, DY, Yv, N, ldy, Wp,
                         K, DX, lddx, gy, gw, gdx, M / 128, K / 128);
    else
      hipLaunchKernelGGL((k_gemm_nn<64>), dim3((M / 64) * (K / 128) * G), dim3(kThreads), 0, st, DY, Yv, N, ldy, Wp,
                         K, DX, lddx, gy, gw, gdx, M / 64, K / 128);
    if (int rc = launch_fail("rl_linear_bwd (dX)")) return rc;
  }
  if (wpart) {
    // pstride 0: wpart [splits][N][K], bpart [splits][N]; else both advance pstride floats per block (the merged
    // layout: each block's bias partials right behind its weight partials, pstride = N*K + N; grouped: the groups'
    // weight partials then their bias partials within a block, pstride = G (N*K + N))
    const int64_t ws = pstride ? pstride : (int64_t)N * K, bs = pstride ? pstride : (int64_t)N;
    if ((reinterpret_cast<uintptr_t>(wpart) & 15) || ws % 4 || ws < (int64_t)N * K)
      return rl_set_error("rl_linear_bwd: weight partials need 16-byte alignment and a block stride >= N*K, % 4");
    hipLaunchKernelGGL(k_gemm_tn, dim3(N / kTN, (K + kTN - 1) / kTN, splits * G), dim3(kThreads), 0, st, DY, Yv, N,
                       ldy, X, ldx, K, M / splits, wpart, bpart, ws, bs, splits, gy, gx, gp, gbp);
    return launch_fail("rl_linear_bwd (dW)");
  }
  return 0;
}

extern "C" int rl_linear_bwd(const void* dy, const void* y, int32_t M, int32_t N, const void* x, int32_t K,
                             int32_t ldx, const void* w, void* dx, int32_t splits, float* wpart, float* bpart,
                             int64_t pstride, void* stream) {
  return rl_linear_bwd_g(dy, y, M, N, x, K, ldx, w, dx, splits, wpart, bpart, pstride, nullptr, stream);
}
