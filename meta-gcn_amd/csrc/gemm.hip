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
constexpr int kU = 4;        // k-steps (of 2 rows) in flight per iteration (8: -25%, occupancy 3 -> 2)

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

  // operands for kU k-steps; the next group's loads are issued before the
  // current group's MFMAs (register double buffer)
  float a[kU][2], b[kU][2], na[kU][2], nb[kU][2];
  auto load = [&](int64_t k, float (&x)[kU][2], float (&y)[kU][2]) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t kr = k + 2 * u + lr;
      const bool okk = kr < ke;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        x[u][t] = (okk && oka[t]) ? A[kr * lda + ia[t]] : 0.0f;
        y[u][t] = (okk && okb[t]) ? B[kr * ldb + jb[t]] : 0.0f;
      }
    }
  };
  if (kb < ke) load(kb, a, b);
  for (int64_t k = kb; k < ke; k += 2 * kU) {
    if (k + 2 * kU < ke) load(k + 2 * kU, na, nb);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[t][s] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][t], b[u][s], acc[t][s], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[u][t] = na[u][t];
        b[u][t] = nb[u][t];
      }
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

// Small C (M, N <= 32: F = 32 layers and the 32 -> 2 projection of config 3):
// one 32 x 32 MFMA tile per workgroup; the four waves take interleaved
// k-steps of the split's K range (wave-level split-K) and their accumulators
// are folded in wave order through LDS, then one slab per split.
__global__ __launch_bounds__(256) void gemm_tn_small_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t ldb,
    int64_t K, int M, int N, int64_t k_per_split, float *__restrict__ partial) {
  constexpr int U = 8;
  __shared__ float red[4][16][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int lr = lane >> 5, lc = lane & 31;
  const int64_t kb = (int64_t)blockIdx.x * k_per_split;
  const int64_t ke = (kb + k_per_split < K) ? kb + k_per_split : K;
  const bool oka = lc < M, okb = lc < N;
  const int ia = oka ? lc : 0, jb = okb ? lc : 0;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  // wave w takes k-steps w, w + 4, w + 8, ... (2 rows each)
  for (int64_t k = kb + 2 * wave; k < ke; k += 2 * 4 * U) {
    float a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t kr = k + 8 * u + lr;
      const bool okk = kr < ke;
      a[u] = (okk && oka) ? A[kr * lda + ia] : 0.0f;
      b[u] = (okk && okb) ? B[kr * ldb + jb] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][r][lane] = acc[r];
  __syncthreads();
  if (wave == 0) {
    float *slab = partial + (int64_t)blockIdx.x * M * N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = __fadd_rn(__fadd_rn(red[0][r][lane], red[1][r][lane]),
                                __fadd_rn(red[2][r][lane], red[3][r][lane]));
      const int row = (r & 3) + 8 * (r >> 2) + 4 * lr;
      if (row < M && lc < N) slab[row * N + lc] = v;
    }
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
  // one resident round: 256 CUs x 3 workgroups (3 waves/SIMD at 134 VGPRs);
  // at least 64 rows of K per split (partials: splits x 64 KB per tile)
  int64_t s = 768 / (tiles > 0 ? tiles : 1);
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
  if (M <= 32 && N <= 32) {
    hipLaunchKernelGGL(gemm_tn_small_kernel, dim3(used), dim3(256), 0, s, A, lda, B, ldb, K, M, N,
                       kps, partial);
    if (int rc = check_launch("gemm_tn_small_kernel")) return rc;
  } else {
    hipLaunchKernelGGL(gemm_tn_partial_kernel, dim3(tiles_m * tiles_n, used), dim3(256), 0, s, A,
                       lda, B, ldb, K, M, N, kps, tiles_n, partial);
    if (int rc = check_launch("gemm_tn_partial_kernel")) return rc;
  }
  const int64_t MN = (int64_t)M * N;
  hipLaunchKernelGGL(gemm_reduce_kernel, dim3((unsigned)((MN + 63) / 64)), dim3(256), 0, s,
                     partial, used, MN, N, C, ldc, accumulate);
  return check_launch("gemm_reduce_kernel");
}

// ---------------------------------------------------------------------------
// mgcn_gemm_nn: C[M, N] = A[M, K] . B[K, N]   (tall-skinny: M = nodes, K, N = F)
//
// The forward transform H = X W (gcn_base_models.py:201) and the input
// gradient dX = dH W^T of a layer (B = W^T through strides).  One workgroup
// per 128-row tile of A; wave w owns output columns [32w, 32w + 32) and the
// four 32-row M sub-tiles (4 accumulators of v_mfma_f32_32x32x2_f32).
//   * the wave's 32-column slab of B stays in registers for the whole tile
//     (K/2 floats per lane);
//   * the A tile is staged once through LDS ([128][K + 4] floats: the +4 pad
//     makes the ds_read_b128 fragment reads conflict-free) and read by all
//     four waves;
//   * K order inside the MFMA chain is permuted (lane half h takes
//     k = s + h K/2) so one ds_read_b128 feeds four consecutive k-steps.
// Epilogue modes:
//   EPI_STORE  C = acc
//   EPI_RELU   (the previous layer's ReLU backward fused into dX):
//              C = Z > 0 ? acc : 0, and per-tile column sums of C written to
//              colsum_partial[tile][N] (the bias gradient, folded in tile order
//              by mgcn_colsum_finish -- deterministic).
// Roofline: 2 M K N FLOP on 157 TF fp32 MFMA vs 4 M (K + N) bytes;
// at K = N = 128 the MFMA side is the bound (0.21 ms vs 0.13 ms at 8 TB/s).

namespace mgcn {
namespace {

constexpr int kNNRows = 128;  // rows of A per workgroup
constexpr int EPI_STORE = 0, EPI_RELU = 1;

// NTP = 32-column tiles of N per workgroup (1, 2 or 4): wave w owns column
// tile w % NTP and the 32-row subtiles t = w / NTP + j * (4 / NTP), so a small
// N (F = 32 layers, config 3) still keeps all four waves busy.
template <int K, int EPI, int NTP>
__global__ __launch_bounds__(256, 2) void gemm_nn_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t sbk,
    int64_t sbn, float *__restrict__ C, int64_t ldc, int64_t M, int N,
    const float *__restrict__ Z, int64_t ldz, float *__restrict__ colsum_partial) {
  constexpr int LDA = K + 4;
  constexpr int KH = K / 2;  // k-steps per lane half
  constexpr int V4_PER_ROW = K / 4;
  constexpr int V4_PER_THREAD = kNNRows * V4_PER_ROW / 256;
  // register prefetch of the next A tile, except where it would spill (the
  // K = 128 ReLU epilogue needs those registers; the co-resident workgroup
  // still overlaps its loads with this one's MFMAs)
  constexpr bool kPrefetch = true;
  __shared__ __attribute__((aligned(16))) float sA[kNNRows * LDA];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int h = lane >> 5, lc = lane & 31;
  constexpr int SUBS = 4 / NTP;  // waves sharing a column tile
  const int mg = wave / NTP;     // first 32-row subtile of this wave
  const int n = (wave % NTP) * 32 + lc;  // output column of this lane
  const bool n_ok = n < N;
  const int64_t n_tiles = (M + kNNRows - 1) / kNNRows;

  // B slab of this wave's 32 columns: b[s] = B[k = s + h*KH][n] (whole kernel)
  float b[KH];
#pragma unroll
  for (int s = 0; s < KH; ++s)
    b[s] = n_ok ? B[(int64_t)(s + h * KH) * sbk + (int64_t)n * sbn] : 0.0f;

  // register prefetch of one A tile: thread t holds float4 #(t + 256 i)
  float4 pre[V4_PER_THREAD];
  auto fetch = [&](int64_t tile) {
    const int64_t m0 = tile * kNNRows;
#pragma unroll
    for (int i = 0; i < V4_PER_THREAD; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / V4_PER_ROW, c4 = idx % V4_PER_ROW;
      pre[i] = (m0 + r < M) ? *reinterpret_cast<const float4 *>(A + (m0 + r) * lda + c4 * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  float csum = 0.0f;
  int64_t tile = blockIdx.x;
  if (kPrefetch && tile < n_tiles) fetch(tile);
  for (; tile < n_tiles; tile += gridDim.x) {
    const int64_t m0 = tile * kNNRows;
    if (!kPrefetch) fetch(tile);
    __syncthreads();  // previous tile's LDS reads are done
#pragma unroll
    for (int i = 0; i < V4_PER_THREAD; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / V4_PER_ROW, c4 = idx % V4_PER_ROW;
      *reinterpret_cast<float4 *>(&sA[r * LDA + c4 * 4]) = pre[i];
    }
    __syncthreads();
    if (kPrefetch && tile + gridDim.x < n_tiles) fetch(tile + gridDim.x);  // overlaps MFMAs

    // one 32-row subtile at a time: 16 accumulator registers, fragment reads
    // double-buffered one step ahead, epilogue of subtile t overlapping the
    // MFMAs of subtile t + 1.  C/D map: col = lane & 31 (-> n),
    // row = (r & 3) + 8 (r >> 2) + 4 h.
    const bool full = (m0 + kNNRows <= M) && n_ok;
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const int t = mg + j * SUBS;
      const float *arow = &sA[(t * 32 + lc) * LDA + h * KH];
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
      float4 cur = *reinterpret_cast<const float4 *>(arow);
#pragma unroll
      for (int s4 = 0; s4 < KH; s4 += 4) {
        float4 nxt = cur;
        if (s4 + 4 < KH) nxt = *reinterpret_cast<const float4 *>(arow + s4 + 4);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.x, b[s4 + 0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.y, b[s4 + 1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.z, b[s4 + 2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.w, b[s4 + 3], acc, 0, 0, 0);
        cur = nxt;
      }
      const int64_t rbase = m0 + t * 32 + 4 * h;
      if (full) {  // unguarded: guarded loads would serialise (one wait per element)
        if constexpr (EPI == EPI_RELU) {
          float zv[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) zv[r] = Z[(rbase + (r & 3) + 8 * (r >> 2)) * ldz + n];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = (zv[r] > 0.0f) ? acc[r] : 0.0f;
            csum = __fadd_rn(csum, v);
            C[(rbase + (r & 3) + 8 * (r >> 2)) * ldc + n] = v;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) C[(rbase + (r & 3) + 8 * (r >> 2)) * ldc + n] = acc[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < M && n_ok) {
            float v = acc[r];
            if constexpr (EPI == EPI_RELU) {
              v = (Z[row * ldz + n] > 0.0f) ? v : 0.0f;
              csum = __fadd_rn(csum, v);
            }
            C[row * ldc + n] = v;
          }
        }
      }
    }
  }
  if constexpr (EPI == EPI_RELU) {
    // fold the waves that share a column tile, in subtile order (deterministic)
    __shared__ float red[4][32];
    const float both = __fadd_rn(csum, __shfl_xor(csum, 32, 64));
    if (h == 0) red[wave][lc] = both;
    __syncthreads();
    if (wave < NTP && h == 0 && n_ok) {
      float v = red[wave][lc];
      for (int g = 1; g < SUBS; ++g) v = __fadd_rn(v, red[g * NTP + wave][lc]);
      colsum_partial[(int64_t)blockIdx.x * N + n] = v;
    }
  }
}

int nn_grid(int64_t M) {
  const int64_t tiles = (M + kNNRows - 1) / kNNRows;
  return (int)(tiles < 512 ? (tiles > 0 ? tiles : 1) : 512);  // 2 persistent WGs per CU
}

template <int K>
int launch_nn(int64_t M, int N, const float *A, int64_t lda, const float *B, int64_t sbk,
              int64_t sbn, float *C, int64_t ldc, int epi, const float *Z, int64_t ldz,
              float *partial, hipStream_t s) {
  const unsigned blocks = (unsigned)nn_grid(M);
#define MGCN_NN(NTP_)                                                                          \
  if (epi == EPI_RELU)                                                                        \
    hipLaunchKernelGGL((gemm_nn_kernel<K, EPI_RELU, NTP_>), dim3(blocks), dim3(256), 0, s, A, \
                       lda, B, sbk, sbn, C, ldc, M, N, Z, ldz, partial);                      \
  else                                                                                        \
    hipLaunchKernelGGL((gemm_nn_kernel<K, EPI_STORE, NTP_>), dim3(blocks), dim3(256), 0, s, A,\
                       lda, B, sbk, sbn, C, ldc, M, N, Z, ldz, partial);
  // NTP = 1 only where it compiles without spills (K = 32, N <= 32: the
  // config-3 F = 32 layers); elsewhere idle column tiles are cheaper than spills
  if constexpr (K == 32) {
    if (N <= 32) {
      MGCN_NN(1)
    } else {
      MGCN_NN(4)
    }
  } else {
    MGCN_NN(4)
  }
#undef MGCN_NN
  return check_launch("gemm_nn_kernel");
}

__global__ __launch_bounds__(256) void colsum_fold_kernel(const float *__restrict__ partial,
                                                          int64_t nparts, int N,
                                                          float *__restrict__ out) {
  __shared__ float red[4][64];
  const int g = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + (threadIdx.x & 63);
  float s = 0.0f;
  if (f < N) {
#pragma unroll 8
    for (int64_t p = g; p < nparts; p += 4) s = __fadd_rn(s, partial[p * N + f]);
  }
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && f < N)
    out[f] = __fadd_rn(__fadd_rn(red[0][threadIdx.x], red[1][threadIdx.x]),
                       __fadd_rn(red[2][threadIdx.x], red[3][threadIdx.x]));
}

}  // namespace
}  // namespace mgcn

extern "C" int mgcn_gemm_nn_supported(int32_t K, int32_t N) {
  return (K == 32 || K == 64 || K == 128) && N >= 1 && N <= 128;
}

extern "C" size_t mgcn_gemm_nn_workspace_bytes(int64_t M, int32_t N) {
  return align_up((size_t)nn_grid(M) * (size_t)(N > 0 ? N : 1) * 4, 256);
}

extern "C" int mgcn_gemm_nn(int64_t M, int32_t K, int32_t N, const float *A, int64_t lda,
                            const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                            const float *Z, int64_t ldz, float *colsum, void *workspace,
                            size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(M >= 0 && K >= 0 && N >= 0, "mgcn_gemm_nn: negative size");
  MGCN_REQUIRE(mgcn_gemm_nn_supported(K, N), "mgcn_gemm_nn: unsupported K=%d N=%d", K, N);
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    if (colsum) MGCN_HIP_TRY(hipMemsetAsync(colsum, 0, sizeof(float) * N, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(A && B && C && lda >= K && ldc >= N, "mgcn_gemm_nn: bad A/B/C");
  MGCN_REQUIRE(lda % 4 == 0 && reinterpret_cast<uintptr_t>(A) % 16 == 0,
               "mgcn_gemm_nn: A must be 16-byte aligned with lda % 4 == 0");
  const int epi = (Z != nullptr) ? EPI_RELU : EPI_STORE;
  MGCN_REQUIRE(epi == EPI_STORE || colsum != nullptr, "mgcn_gemm_nn: Z given without colsum");
  float *partial = nullptr;
  if (epi == EPI_RELU) {
    const size_t need = mgcn_gemm_nn_workspace_bytes(M, N);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_gemm_nn: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    partial = static_cast<float *>(workspace);
  }
  int rc;
  if (K == 32)
    rc = launch_nn<32>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, ldz, partial, s);
  else if (K == 64)
    rc = launch_nn<64>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, ldz, partial, s);
  else
    rc = launch_nn<128>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, ldz, partial, s);
  if (rc || epi != EPI_RELU) return rc;
  const int64_t parts = nn_grid(M);
  hipLaunchKernelGGL(colsum_fold_kernel, dim3((N + 63) / 64), dim3(256), 0, s, partial, parts, N,
                     colsum);
  return check_launch("colsum_fold_kernel");
}
