// Dense feature-transform GEMMs of the GCN layer on fp32 MFMA (gfx950).
//
// mgcn_gemm_tn:  C[M, N] (+)= A^T B  with A [K, M], B [K, N] row-major and
// K = number of nodes (1M at config 2) -- the weight gradient
// dW = X^T dH of `x @ W` (gcn_base_models.py:201).  hipBLASLt picks a
// 32x32x256 macro-tile for this tall-K shape and runs it at ~18 TFLOP/s;
// here K is split across the whole chip instead:
//
//   * grid = (C tiles of 128 x 128) x (K splits); 4 waves per workgroup,
//     wave (wi, wj) owns the 64 x 64 quadrant = 2 x 2 tiles of
//     v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate);
//   * operands stream straight from HBM into registers (each k-step is two
//     contiguous 128-B row segments per operand per wave), U k-steps in flight;
//   * every split writes its 128 x 128 f32 partial to a workspace slab, and a
//     second kernel folds the slabs in split order: deterministic, no atomics.
//
// Roofline: at K = 1M, M = N = 128 the kernel moves 4K(M+N) = 1 GB and does
// 2KMN = 33.6 GFLOP -> 0.21 ms at the 157 TF fp32 MFMA peak vs 0.13 ms at
// 8 TB/s: MFMA-bound (the GEMMs are compute-bound at F=128).

#include "mgcn_internal.h"

namespace mgcn {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 128;   // C tile per workgroup (M and N)
constexpr int kU = 4;        // k-steps (of 2 rows) in flight per iteration

__global__ __launch_bounds__(256) void gemm_tn_partial_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t ldb,
    int64_t K, int M, int N, int64_t k_per_split, int tiles_n, float *__restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int tile_m = blockIdx.x / tiles_n, tile_n = blockIdx.x % tiles_n;
  const int i0 = tile_m * kTile + wi * 64;
  const int j0 = tile_n * kTile + wj * 64;
  const int64_t kb = (int64_t)blockIdx.y * k_per_split;
  const int64_t ke = (kb + k_per_split < K) ? kb + k_per_split : K;
  const int lr = lane >> 5;   // k offset within a k-step (0/1)
  const int lc = lane & 31;   // row of A^T tile / column of B tile

  // column indices this lane reads (clamped; out-of-range lanes read column 0 and
  // their products land only in C entries that are never stored)
  int ia[2], jb[2];
  bool oka[2], okb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    ia[t] = i0 + t * 32 + lc;
    oka[t] = ia[t] < M;
    if (!oka[t]) ia[t] = 0;
    jb[t] = j0 + t * 32 + lc;
    okb[t] = jb[t] < N;
    if (!okb[t]) jb[t] = 0;
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][s][r] = 0.0f;

  for (int64_t k = kb; k < ke; k += 2 * kU) {
    float a[kU][2], b[kU][2];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t kr = k + 2 * u + lr;
      const bool okk = kr < ke;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[u][t] = (okk && oka[t]) ? A[kr * lda + ia[t]] : 0.0f;
        b[u][t] = (okk && okb[t]) ? B[kr * ldb + jb[t]] : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[t][s] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][t], b[u][s], acc[t][s], 0, 0, 0);
  }

  // partial slab [split][M][N]; C/D map: col = lane & 31,
  // row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  float *slab = partial + (int64_t)blockIdx.y * M * N;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lr;
        const int col = j0 + s * 32 + lc;
        if (row < M && col < N) slab[(int64_t)row * N + col] = acc[t][s][r];
      }
}

// C[e] (+)= sum over splits of partial[split][e], in split order within each of
// 4 interleaved groups, the groups then folded in order: deterministic.
__global__ __launch_bounds__(256) void gemm_reduce_kernel(const float *__restrict__ partial,
                                                          int splits, int64_t MN, int N,
                                                          float *__restrict__ C, int64_t ldc,
                                                          int accumulate) {
  __shared__ float red[4][64];
  const int g = threadIdx.x >> 6;  // split group
  const int64_t e = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  float s = 0.0f;
  if (e < MN) {
#pragma unroll 8
    for (int sp = g; sp < splits; sp += 4) s = __fadd_rn(s, partial[(int64_t)sp * MN + e]);
  }
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && e < MN) {
    float v = __fadd_rn(__fadd_rn(red[0][threadIdx.x], red[1][threadIdx.x]),
                        __fadd_rn(red[2][threadIdx.x], red[3][threadIdx.x]));
    const int64_t row = e / N, col = e % N;
    float *dst = C + row * ldc + col;
    *dst = accumulate ? __fadd_rn(*dst, v) : v;
  }
}

int gemm_splits(int64_t K, int tiles) {
  // ~2048 workgroups in flight over 256 CUs, at least 64 rows of K per split
  int64_t s = 2048 / (tiles > 0 ? tiles : 1);
  int64_t max_s = (K + 63) / 64;
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  return (int)s;
}

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" size_t mgcn_gemm_tn_workspace_bytes(int64_t K, int32_t M, int32_t N) {
  const int tiles = ((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  return align_up((size_t)gemm_splits(K, tiles) * (size_t)M * (size_t)N * sizeof(float), 256);
}

extern "C" int mgcn_gemm_tn(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda,
                            const float *B, int64_t ldb, float *C, int64_t ldc, int accumulate,
                            void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(K >= 0 && M >= 0 && N >= 0, "mgcn_gemm_tn: negative size");
  hipStream_t s = as_stream(stream);
  if (M == 0 || N == 0) return MGCN_OK;
  MGCN_REQUIRE(C != nullptr && ldc >= N, "mgcn_gemm_tn: bad C");
  if (K == 0) {
    if (!accumulate)
      for (int32_t r = 0; r < M; ++r)
        MGCN_HIP_TRY(hipMemsetAsync(C + r * ldc, 0, sizeof(float) * N, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(A && B && lda >= M && ldb >= N, "mgcn_gemm_tn: bad A/B");
  const int tiles_m = (M + kTile - 1) / kTile, tiles_n = (N + kTile - 1) / kTile;
  const int splits = gemm_splits(K, tiles_m * tiles_n);
  const size_t need = mgcn_gemm_tn_workspace_bytes(K, M, N);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_gemm_tn: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  int64_t kps = (K + splits - 1) / splits;
  kps = (kps + 2 * kU - 1) / (2 * kU) * (2 * kU);
  const int used = (int)((K + kps - 1) / kps);
  float *partial = static_cast<float *>(workspace);
  hipLaunchKernelGGL(gemm_tn_partial_kernel, dim3(tiles_m * tiles_n, used), dim3(256), 0, s, A,
                     lda, B, ldb, K, M, N, kps, tiles_n, partial);
  if (int rc = check_launch("gemm_tn_partial_kernel")) return rc;
  const int64_t MN = (int64_t)M * N;
  hipLaunchKernelGGL(gemm_reduce_kernel, dim3((unsigned)((MN + 63) / 64)), dim3(256), 0, s,
                     partial, used, MN, N, C, ldc, accumulate);
  return check_launch("gemm_reduce_kernel");
}
