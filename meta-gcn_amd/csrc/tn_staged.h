// Split-K workgroup of the staged small-C GEMM  C = A^T B  (M = 32 columns
// of A, N = 32 NT columns of B, 16-byte aligned rows), shared by
// gemm_tn_staged_kernel (gemm.hip) and the residual stack's heavy-row
// transform launch (residual.hip), which runs the layer's weight GEMM in the
// same launch.  Device code only, internal.
//
// Workgroup `blk` (256 threads) reduces rows [blk kps, (blk + 1) kps) of K:
// chunks of CK rows stream in as float4 buffer loads (one register bank of
// prefetch, the tail past the split reads zeros), are staged in LDS and feed
// v_mfma_f32_32x32x2f32 from there (rows of 32 / 64 floats: conflict-free
// operand reads); the four waves take interleaved k-steps of each chunk and
// fold through LDS in wave order into the [32][N] slab partial + blk 32 N.
// `stage` is LDS of max(CK (32 + N), 4 x 16 x 64) floats.
#pragma once

#include "mgcn_internal.h"
#include "x6.h"

namespace mgcn {

template <int NT, int CK>
__device__ inline void tn_staged_block(const float *__restrict__ A, int64_t lda,
                                       const float *__restrict__ B, int64_t ldb, int64_t K,
                                       int64_t k_per_split, float *__restrict__ partial, int blk,
                                       float *stage) {
  using namespace x6;
  constexpr int NB = 32 * NT;  // columns of B (and C)
  constexpr int QA = CK * 32 / 4 / 256, QB = CK * NB / 4 / 256;  // float4 per thread
  static_assert(QA >= 1 && QB >= 1, "CK too small for 256 threads");
  float(*As)[32] = reinterpret_cast<float(*)[32]>(stage);
  float(*Bs)[NB] = reinterpret_cast<float(*)[NB]>(stage + CK * 32);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane >> 5, lc = lane & 31;
  const int64_t kb = (int64_t)blk * k_per_split;
  const int64_t ke = (kb + k_per_split < K) ? kb + k_per_split : K;
  const int64_t n = ke > kb ? ke - kb : 0;
  const auto ra_ = buf_rsrc(A + kb * lda, (uint32_t)(n * lda * 4));
  const auto rb_ = buf_rsrc(B + kb * ldb, (uint32_t)(n * ldb * 4));
  u32x4 ra[QA], rb[QB];
  auto load = [&](int64_t r0) {  // chunk at split row r0 (relative)
#pragma unroll
    for (int j = 0; j < QA; ++j) {
      const int i = tid + 256 * j, row = i >> 3, c4 = i & 7;
      ra[j] = __builtin_amdgcn_raw_buffer_load_b128(
          ra_, (int)(((r0 + row) * lda + 4 * c4) * 4), 0, 0);
    }
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      const int i = tid + 256 * j, row = i / (NB / 4), c4 = i % (NB / 4);
      rb[j] = __builtin_amdgcn_raw_buffer_load_b128(
          rb_, (int)(((r0 + row) * ldb + 4 * c4) * 4), 0, 0);
    }
  };
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
  if (n > 0) load(0);
  for (int64_t r0 = 0; r0 < n; r0 += CK) {
    __syncthreads();  // the previous chunk's operand reads are done
#pragma unroll
    for (int j = 0; j < QA; ++j) {
      const int i = tid + 256 * j;
      *reinterpret_cast<u32x4 *>(&As[i >> 3][4 * (i & 7)]) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      const int i = tid + 256 * j;
      *reinterpret_cast<u32x4 *>(&Bs[i / (NB / 4)][4 * (i % (NB / 4))]) = rb[j];
    }
    __syncthreads();
    if (r0 + CK < n) load(r0 + CK);  // in flight under this chunk's MFMAs
    // wave w: k-steps w, w + 4, ... of two rows each (rows past the split are 0)
#pragma unroll
    for (int st = 0; st < CK / 8; ++st) {
      const int k = 2 * (wave + 4 * st) + lr;
      const float a = As[k][lc];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bs[k][32 * t + lc], acc[t], 0, 0, 0);
    }
  }
  // fold the four waves' accumulators in wave order (4 x 16 x 64 floats)
  float(*red)[16][64] = reinterpret_cast<float(*)[16][64]>(stage);
  float *slab = partial + (int64_t)blk * 32 * NB;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave][r][lane] = acc[t][r];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = __fadd_rn(__fadd_rn(red[0][r][lane], red[1][r][lane]),
                                  __fadd_rn(red[2][r][lane], red[3][r][lane]));
        const int row = (r & 3) + 8 * (r >> 2) + 4 * lr;
        slab[row * NB + 32 * t + lc] = v;
      }
    }
  }
}

}  // namespace mgcn
