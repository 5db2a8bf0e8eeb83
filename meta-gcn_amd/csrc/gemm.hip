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
#include "x6.h"
#include "tn_staged.h"

// cache policy of gemm_bwd's X / Z rows (streamed once): 2 = nt (fused.hip)
#ifndef MGCN_NT_AUX
#define MGCN_NT_AUX 2
#endif

namespace mgcn {
namespace {

using namespace x6;

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

// LDS-staged variant for M, N multiples of 128 (the F = 128 layers).  The
// per-lane dword loads of gemm_tn_partial_kernel are fragment-shaped (every
// wave-instruction 2 x 128 B) and keep the texture-address path busy at full
// MFMA rate; here each 32-row chunk of both operands moves in 1-KiB
// global_load_lds_dwordx4 instructions (2 rows of 512 B, lane-linear image)
// into one of two LDS buffers, and the MFMA fragments come from LDS with
// ds_read_b32.  One barrier per chunk; the next chunk's loads are issued
// right after it, so they run under the current chunk's MFMAs (2 BK per
// wave).  K order inside a chunk is permuted (lane half h takes rows
// h BK/2 .. (h + 1) BK/2 - 1): the same products per output, summed in a
// different order.
typedef __attribute__((address_space(3))) void lds_void_t;

// ---------------------------------------------------------------------------
// bf16x6 product arithmetic (mgcn_set_option "gemm_precision" 1): every fp32
// operand split exactly-rounded into three bf16 terms x = hi + mid + lo (RNE
// at each step; x - hi and r - mid are exact, |mid| <= 2^-9 |x|, |lo| <=
// 2^-18 |x|, |x - (hi + mid + lo)| <= 2^-27 |x|) and the six products whose
// magnitude reaches 2^-18 (hh, hm, mh, mm, hl, lh) summed on
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate) into one fp32
// accumulator.  Dropped terms (ml, lm, ll) are below 2^-27 of |a b|; the
// accumulator takes 6 K / 16 roundings per output against K for the f32
// form.  Error vs fp64: scripts/bench_gemm.py, tests/test_gpu_parity.py.
constexpr int PREC_F32 = 0, PREC_BF16X6 = 1;
int g_gemm_precision = PREC_BF16X6;


// dW for M, N multiples of 128 in bf16x6.  Per chunk of 16 k-rows, each
// thread loads 2 float4 of each operand (coalesced 512-B rows), splits them
// and writes the three bf16 terms into [k][128] images (256-B rows, 16-B
// chunks XOR-swizzled: chunk ch of row r at ch ^ ((r & 3) << 2 | (r >> 2) & 3)),
// from which every MFMA fragment (8 consecutive k of one column) is two
// ds_read_b64_tr_b16 (each 16-lane group transposes a 4-row x 16-column
// block; conflict-free on this swizzle).  The next chunk's loads are in
// flight in registers while the current chunk's 24 MFMAs per wave run.
constexpr int kTnX6Rows = 16;                       // k-rows per chunk
constexpr int kTnX6Img = kTnX6Rows * 256;           // bytes per term image
__device__ __forceinline__ int tn_x6_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__global__ __launch_bounds__(256, 3) void gemm_tn_x6_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t ldb,
    int64_t K, int M, int N, int64_t k_per_split, int tiles_n, float *__restrict__ partial) {
  // images: [operand A/B][term hi/mid/lo] x kTnX6Img bytes
  __shared__ __attribute__((aligned(16))) char lds[6 * kTnX6Img];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  // XCD-aware order (1-D grid of tiles x splits): workgroup L runs on XCD
  // L % 8; consecutive logical ids -- the C tiles of one split, which read
  // the same K rows of A and B -- go to one XCD, so the second read of each
  // row is an L2 hit instead of a second HBM read
  const int tiles = (M / kTile) * tiles_n;
  const int64_t G = gridDim.x, G8 = G - G % 8;
  const int64_t L = blockIdx.x;
  const int64_t lj = L < G8 ? (L % 8) * (G8 / 8) + L / 8 : L;
  const int tile = (int)(lj % tiles);
  const int tile_m = tile / tiles_n, tile_n = tile % tiles_n;
  const int64_t split = lj / tiles;
  const int64_t kb = split * k_per_split;
  const int64_t ke = (kb + k_per_split < K) ? kb + k_per_split : K;
  const int h = lane >> 5, lc = lane & 31;

  // staging: thread -> float4 items tid and tid + 256 of a [16][32] float4 chunk
  const float *a_base = A + (int64_t)tile_m * kTile;
  const float *b_base = B + (int64_t)tile_n * kTile;
  float4 ra[2], rb[2];
  auto load_chunk = [&](int64_t k0) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int f = tid + 256 * m;
      const int64_t row = k0 + (f >> 5);
      const bool ok = row < ke;
      const int64_t rr = ok ? row : kb;  // a valid row, zeroed below
      const float4 va = *reinterpret_cast<const float4 *>(a_base + rr * lda + 4 * (f & 31));
      const float4 vb = *reinterpret_cast<const float4 *>(b_base + rr * ldb + 4 * (f & 31));
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      ra[m] = ok ? va : z;
      rb[m] = ok ? vb : z;
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int f = tid + 256 * m;
      const int row = f >> 5, c4 = f & 31;
      const int off = tn_x6_off(row, c4 >> 1) + 8 * (c4 & 1);
#pragma unroll
      for (int op = 0; op < 2; ++op) {
        const float4 v = op ? rb[m] : ra[m];
        uint32_t hi[2], mid[2], lo[2];
        split3_pair(f32x2{v.x, v.y}, hi[0], mid[0], lo[0]);
        split3_pair(f32x2{v.z, v.w}, hi[1], mid[1], lo[1]);
        char *img = lds + op * 3 * kTnX6Img + off;
        *reinterpret_cast<uint2 *>(img) = make_uint2(hi[0], hi[1]);
        *reinterpret_cast<uint2 *>(img + kTnX6Img) = make_uint2(mid[0], mid[1]);
        *reinterpret_cast<uint2 *>(img + 2 * kTnX6Img) = make_uint2(lo[0], lo[1]);
      }
    }
  };

  // fragment addresses: lane = 16 g + 4 q + p reads rows 8 h + q (+ 4) and
  // chunk (col0 >> 3) + 2 (g & 1) + (p >> 1), half p & 1
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto frag_off = [&](int col0, int second) {
    const int row = 8 * h + q + 4 * second;
    return tn_x6_off(row, (col0 >> 3) + 2 * (g & 1) + (p >> 1)) + 8 * (p & 1);
  };
  int offa[2][2], offb[2][2];  // [tile][read]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      offa[t][r] = frag_off(wi * 64 + 32 * t, r);
      offb[t][r] = 3 * kTnX6Img + frag_off(wj * 64 + 32 * t, r);
    }
  auto read8 = [&](const int (&o)[2], int term) {
    const v4i16 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4i16_t *)(lds + o[0] + term * kTnX6Img));
    const v4i16 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4i16_t *)(lds + o[1] + term * kTnX6Img));
    const short y[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, y);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][s2][r] = 0.0f;

  const int64_t nchunks = (ke - kb + kTnX6Rows - 1) / kTnX6Rows;
  if (nchunks > 0) load_chunk(kb);
  for (int64_t c = 0; c < nchunks; ++c) {
    __syncthreads();  // the previous chunk's fragments are read
    store_chunk();
    if (c + 1 < nchunks) load_chunk(kb + (c + 1) * kTnX6Rows);
    __syncthreads();
    bf16x8 fa[2][3], fb[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int term = 0; term < 3; ++term) {
        fa[t][term] = read8(offa[t], term);
        fb[t][term] = read8(offb[t], term);
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        acc[t][s2] = mfma_x6(fa[t][0], fa[t][1], fa[t][2], fb[s2][0], fb[s2][1], fb[s2][2],
                             acc[t][s2]);
  }

  float *slab = partial + split * M * N;
  const int i0 = tile_m * kTile + wi * 64, j0 = tile_n * kTile + wj * 64;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        slab[(int64_t)row * N + j0 + s2 * 32 + lc] = acc[t][s2][r];
      }
}



template <int BK, int WPS>
__global__ __launch_bounds__(256, WPS) void gemm_tn_lds_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t ldb,
    int64_t K, int M, int N, int64_t k_per_split, int tiles_n, float *__restrict__ partial) {
  constexpr int kTnChunkFloats = BK * kTile;  // one operand's chunk image
  constexpr int HS = BK / 2;                  // k-steps per chunk
  __shared__ __attribute__((aligned(16))) float lds[2][2][kTnChunkFloats];  // [buf][A/B]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  // XCD-aware order (1-D grid of tiles x splits): workgroup L runs on XCD
  // L % 8; consecutive logical ids -- the C tiles of one split, which read
  // the same K rows of A and B -- go to one XCD, so the second read of each
  // row is an L2 hit instead of a second HBM read
  const int tiles = (M / kTile) * tiles_n;
  const int64_t G = gridDim.x, G8 = G - G % 8;
  const int64_t L = blockIdx.x;
  const int64_t lj = L < G8 ? (L % 8) * (G8 / 8) + L / 8 : L;
  const int tile = (int)(lj % tiles);
  const int tile_m = tile / tiles_n, tile_n = tile % tiles_n;
  const int64_t split = lj / tiles;
  const int64_t kb = split * k_per_split;
  const int64_t ke = (kb + k_per_split < K) ? kb + k_per_split : K;
  const int h = lane >> 5, lc = lane & 31;
  // glds source: lane -> row pair half (lane >> 5), 4 floats at column 4 (lane & 31)
  const int g_row = lane >> 5, g_col = (lane & 31) * 4;
  const float *a_src = A + (int64_t)tile_m * kTile + g_col;
  const float *b_src = B + (int64_t)tile_n * kTile + g_col;

  auto issue = [&](int64_t k0, int buf) {
    // wave w moves row pairs w, w + 4, ... of both operands
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      const int pair = wave + 4 * q;
      int64_t row = k0 + 2 * pair + g_row;
      row = row < K ? row : K - 1;  // past the end: a valid row, masked in compute
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a_src + row * lda),
                                       (lds_void_t *)(&lds[buf][0][pair * 2 * kTile]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(b_src + row * ldb),
                                       (lds_void_t *)(&lds[buf][1][pair * 2 * kTile]), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][s][r] = 0.0f;

  auto compute = [&](int buf, int valid) {  // valid: rows of this chunk below ke
    const float *la = &lds[buf][0][wi * 64 + lc];
    const float *lb = &lds[buf][1][wj * 64 + lc];
    float a[2], b[2], na[2], nb[2];
    auto frag = [&](int m, float (&x)[2], float (&y)[2]) {
      const int k = m + HS * h;
      const bool ok = k < valid;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        x[t] = ok ? la[k * kTile + 32 * t] : 0.0f;
        y[t] = ok ? lb[k * kTile + 32 * t] : 0.0f;
      }
    };
    frag(0, a, b);
#pragma unroll
    for (int m = 0; m < HS; ++m) {
      if (m + 1 < HS) frag(m + 1, na, nb);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          acc[t][s2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[s2], acc[t][s2], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = na[t];
        b[t] = nb[t];
      }
    }
  };

  const int64_t nchunks = (ke - kb + BK - 1) / BK;
  if (nchunks > 0) issue(kb, 0);
  for (int64_t c = 0; c < nchunks; ++c) {
    const int64_t k0 = kb + c * BK;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's loads of chunk c have landed
    __syncthreads();                // everyone's have; buffer (c + 1) & 1 is free
    if (c + 1 < nchunks) issue(k0 + BK, (int)((c + 1) & 1));
    const int64_t left = ke - k0;
    if (left >= BK)
      compute((int)(c & 1), BK);
    else
      compute((int)(c & 1), (int)left);
  }

  float *slab = partial + split * M * N;
  const int i0 = tile_m * kTile + wi * 64, j0 = tile_n * kTile + wj * 64;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        slab[(int64_t)row * N + j0 + s2 * 32 + lc] = acc[t][s2][r];
      }
}

// Small C (M <= 32, N <= 32 NT: F = 32 layers, the 32 -> 2 projection and,
// with NT = 2, the [W | Wr^T] pair of a fused residual layer, config 3):
// NT 32 x 32 MFMA tiles per workgroup; the four waves take interleaved
// k-steps of the split's K range (wave-level split-K) and their accumulators
// are folded in wave order through LDS, then one slab per split.
template <int NT>
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
  const bool oka = lc < M;
  const int ia = oka ? lc : 0;
  bool okb[NT];
  int jb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    okb[t] = 32 * t + lc < N;
    jb[t] = okb[t] ? 32 * t + lc : 0;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
  // wave w takes k-steps w, w + 4, w + 8, ... (2 rows each)
  for (int64_t k = kb + 2 * wave; k < ke; k += 2 * 4 * U) {
    float a[U], b[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t kr = k + 8 * u + lr;
      const bool okk = kr < ke;
      a[u] = (okk && oka) ? A[kr * lda + ia] : 0.0f;
#pragma unroll
      for (int t = 0; t < NT; ++t) b[u][t] = (okk && okb[t]) ? B[kr * ldb + jb[t]] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u][t], acc[t], 0, 0, 0);
  }
  float *slab = partial + (int64_t)blockIdx.x * M * N;
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
        if (row < M && okb[t]) slab[row * N + 32 * t + lc] = v;
      }
    }
  }
}

// Staged small C for M = 32, N = 32 NT with 16-byte aligned rows (the F = 32
// weight GEMMs of config 3, [W | Wr^T] with NT = 2): tn_staged.h's split-K
// workgroups (64-row chunks), plus the side-fold workgroups of an independent
// job at the end of the grid.  The 4-byte-per-lane loads of
// gemm_tn_small_kernel leave ~6 dependent round trips per split at config 3
// (26 us per launch; this one 20 us).
template <int NT>
__global__ __launch_bounds__(256) void gemm_tn_staged_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t ldb,
    int64_t K, int64_t k_per_split, float *__restrict__ partial, SideFold sf) {
  constexpr int CK = 64;
  __shared__ __attribute__((aligned(16))) float stage[CK * 32 + CK * 32 * NT > 4096
                                                          ? CK * 32 + CK * 32 * NT
                                                          : 4096];
  if (blockIdx.x >= gridDim.x - (unsigned)sf.blocks) {
    // a side job riding in the same launch (an independent fold)
    side_fold_block(sf, (int)(blockIdx.x - (gridDim.x - (unsigned)sf.blocks)), stage);
    return;
  }
  tn_staged_block<NT, CK>(A, lda, B, ldb, K, k_per_split, partial, (int)blockIdx.x, stage);
}

// dW at M = N = 256 (config 5's F = 256 layers: C = Z^T dY over K = the
// rank's rows).  gemm_tn_x6_kernel's 128 x 128 tiles would split (and read)
// every element of A and B twice -- once per C tile sharing its K rows; here
// one 512-thread workgroup per split owns the whole 256 x 256 C: wave w the
// 64 x 128 block (rows 64 (w >> 1), columns 128 (w & 1)) = 2 x 4 tiles of
// v_mfma_f32_32x32x16_bf16 (bf16x6), 128 accumulators.  Per 16-row chunk the
// rows of A and B (16 KB each) are split once into twelve 4-KB term images
// ([operand][128-column half][term], gemm_tn_x6's swizzle), double-buffered
// (96 KB: one workgroup per CU, one barrier per chunk); the next chunk's
// loads (buffer loads: the split's tail reads zeros) are in flight in
// registers under the current chunk's 48 MFMAs per wave.  K = 6.2M: 4.66 ms
// (6.18 for the 128 x 128 tiles; 5.49 here with the loads' zero select,
// which made every load wait at once).  Same products as gemm_tn_x6 (each C element a sum over its split's
// rows in k-step order), partial slabs folded in split order.
constexpr int kTnWideChunk = 12 * kTnX6Img;  // one chunk's images: 48 KB

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void
gemm_tn_x6_wide_kernel(const float *__restrict__ A, int64_t lda, const float *__restrict__ B,
                       int64_t ldb, int64_t K, int64_t k_per_split, float *__restrict__ partial) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kTnWideChunk];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t kb = (int64_t)blockIdx.x * k_per_split;
  const int64_t ke = (kb + k_per_split < K) ? kb + k_per_split : K;
  const int h = lane >> 5, lc = lane & 31;

  // staging: thread -> float4 items tid, tid + 512 of a [16][64] float4
  // chunk, per operand (one chunk in flight in registers)
  struct Regs {
    float4 a[2], b[2];
  };
  // buffer loads over the split's rows: a row past its end reads zeros with
  // no select on the loaded value (a select would make the load synchronous);
  // the nt policy (streamed once: 4.70 vs 4.75 ms at K = 6.24M, round 6)
  const auto rsa = buf_rsrc(A + kb * lda, (uint32_t)((ke - kb) * lda * 4));
  const auto rsb = buf_rsrc(B + kb * ldb, (uint32_t)((ke - kb) * ldb * 4));
  auto load_chunk = [&](int64_t k0, Regs &R) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int f = tid + 512 * m;
      const int64_t row = k0 - kb + (f >> 6);  // split-relative
      R.a[m] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rsa, (int)((row * lda + 4 * (f & 63)) * 4), 0, MGCN_NT_AUX));
      R.b[m] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rsb, (int)((row * ldb + 4 * (f & 63)) * 4), 0, MGCN_NT_AUX));
    }
  };
  auto store_chunk = [&](char *img0, const Regs &R) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int f = tid + 512 * m;
      const int row = f >> 6, c4 = f & 63;
      const int half = c4 >> 5, c = c4 & 31;
      const int off = tn_x6_off(row, c >> 1) + 8 * (c & 1);
#pragma unroll
      for (int op = 0; op < 2; ++op) {
        const float4 v = op ? R.b[m] : R.a[m];
        uint32_t hi[2], mid[2], lo[2];
        split3_pair(f32x2{v.x, v.y}, hi[0], mid[0], lo[0]);
        split3_pair(f32x2{v.z, v.w}, hi[1], mid[1], lo[1]);
        char *img = img0 + (op * 2 + half) * 3 * kTnX6Img + off;
        *reinterpret_cast<uint2 *>(img) = make_uint2(hi[0], hi[1]);
        *reinterpret_cast<uint2 *>(img + kTnX6Img) = make_uint2(mid[0], mid[1]);
        *reinterpret_cast<uint2 *>(img + 2 * kTnX6Img) = make_uint2(lo[0], lo[1]);
      }
    }
  };
  // fragment addresses (gemm_tn_x6_kernel's): lane = 16 g + 4 q + p reads
  // rows 8 h + q (+ 4) and chunk (col0 >> 3) + 2 (g & 1) + (p >> 1), half p & 1
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto frag_off = [&](int op, int gcol0, int second) {
    const int half = gcol0 >> 7, col0 = gcol0 & 127;
    const int row = 8 * h + q + 4 * second;
    return (op * 2 + half) * 3 * kTnX6Img +
           tn_x6_off(row, (col0 >> 3) + 2 * (g & 1) + (p >> 1)) + 8 * (p & 1);
  };
  int offa[2][2], offb[4][2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int t = 0; t < 2; ++t) offa[t][r] = frag_off(0, wm * 64 + 32 * t, r);
#pragma unroll
    for (int u = 0; u < 4; ++u) offb[u][r] = frag_off(1, wn * 128 + 32 * u, r);
  }
  auto read8 = [&](const char *img0, const int (&o)[2], int term) {
    const v4i16 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4i16_t *)(img0 + o[0] + term * kTnX6Img));
    const v4i16 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4i16_t *)(img0 + o[1] + term * kTnX6Img));
    const short y[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, y);
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.0f;

  // (tried: chunk c's MFMAs in one basic block with the split and store of
  // chunk c + 1 -- 4.84 vs 4.66 ms at K = 6.2M; two chunks of register
  // prefetch -- slower again)
  const int64_t nchunks = (ke - kb + kTnX6Rows - 1) / kTnX6Rows;
  Regs R;
  if (nchunks > 0) load_chunk(kb, R);
  for (int64_t c = 0; c < nchunks; ++c) {
    char *img0 = lds + (c & 1) * kTnWideChunk;
    // this buffer was last read two chunks ago, before the previous barrier
    store_chunk(img0, R);
    if (c + 1 < nchunks) load_chunk(kb + (c + 1) * kTnX6Rows, R);
    __syncthreads();
    bf16x8 fa[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int term = 0; term < 3; ++term) fa[t][term] = read8(img0, offa[t], term);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      bf16x8 fb[3];
#pragma unroll
      for (int term = 0; term < 3; ++term) fb[term] = read8(img0, offb[u], term);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc[t][u] = mfma_x6(fa[t][0], fa[t][1], fa[t][2], fb[0], fb[1], fb[2], acc[t][u]);
    }
  }

  float *slab = partial + (int64_t)blockIdx.x * 256 * 256;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        slab[(int64_t)row * 256 + wn * 128 + u * 32 + lc] = acc[t][u][r];
      }
}


bool tn_wide(int M, int N) { return M == 256 && N == 256; }
// gemm_tn_x6_wide_kernel addresses a split's rows with 32-bit buffer offsets
bool tn_wide_fits(int64_t kps, int64_t lda, int64_t ldb) {
  return (kps + 16) * (lda > ldb ? lda : ldb) * 4 < (int64_t(1) << 31);
}

bool tn_lds(int M, int N) { return M % kTile == 0 && N % kTile == 0; }

// LDS-staged dW variants (mgcn_set_option "gemm_tn_variant"; measured at
// K = 1M, M = N = 128: 0.321 / 0.335 / 0.337 ms): 0 = BK 64, one workgroup
// per CU; 1 = BK 32, two; 2 = BK 16, three
int g_tn_lds_variant = 0;
int g_tn_staged = 1;  // M = 32, N = 32 / 64: gemm_tn_staged_kernel (0: gemm_tn_small_kernel)
int tn_lds_wgs() { return g_tn_lds_variant == 1 ? 2 : g_tn_lds_variant == 2 ? 3 : 1; }

int gemm_splits(int64_t K, int M, int N) {
  // one resident round: 256 CUs x 3 workgroups (3 waves/SIMD at 134 VGPRs),
  // or x 2 for the LDS-staged kernel (64 KB of LDS each); at least 64 rows of
  // K per split (partials: splits x 64 KB per tile).  256 x 256 bf16x6
  // (gemm_tn_x6_wide_kernel): one workgroup per CU
  if (tn_wide(M, N) && g_gemm_precision == PREC_BF16X6) {
    int64_t s = 256, max_s = (K + 63) / 64;
    if (s > max_s) s = max_s;
    return (int)(s < 1 ? 1 : s);
  }
  const int tiles = ((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  const int per_cu = !tn_lds(M, N) ? 3 : g_gemm_precision == PREC_BF16X6 ? 3 : tn_lds_wgs();
  int64_t s = 256 * per_cu / (tiles > 0 ? tiles : 1);
  int64_t max_s = (K + 63) / 64;
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  return (int)s;
}

}  // namespace

int gemm_set_tn_variant(int value) {
  if (value < 0 || value > 2) return MGCN_EINVAL;
  g_tn_lds_variant = value;
  return MGCN_OK;
}

int gemm_set_tn_staged(int value) {
  if (value < 0 || value > 1) return MGCN_EINVAL;
  g_tn_staged = value;
  return MGCN_OK;
}

}  // namespace mgcn

using namespace mgcn;

extern "C" size_t mgcn_gemm_tn_workspace_bytes(int64_t K, int32_t M, int32_t N) {
  return align_up((size_t)gemm_splits(K, M, N) * (size_t)M * (size_t)N * sizeof(float), 256);
}

namespace {
// C = A^T B; columns [N1, N) go transposed to C2 (N1 == N: plain C)
int gemm_tn_core(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda, const float *B,
                 int64_t ldb, float *C, int64_t ldc, int32_t N1, float *C2, int64_t ldc2,
                 int accumulate, void *workspace, size_t workspace_bytes, hipStream_t s,
                 const SideFold *side, bool *side_done, SideFold *defer) {
  if (M == 0 || N == 0) return MGCN_OK;
  if (K == 0) {
    if (!accumulate) {
      for (int32_t r = 0; r < M && N1 > 0; ++r)
        MGCN_HIP_TRY(hipMemsetAsync(C + r * ldc, 0, sizeof(float) * N1, s));
      for (int32_t r = 0; r < N - N1; ++r)
        MGCN_HIP_TRY(hipMemsetAsync(C2 + r * ldc2, 0, sizeof(float) * M, s));
    }
    return MGCN_OK;
  }
  const int tiles_m = (M + kTile - 1) / kTile, tiles_n = (N + kTile - 1) / kTile;
  const int splits = gemm_splits(K, M, N);
  const size_t need = mgcn_gemm_tn_workspace_bytes(K, M, N);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_gemm_tn: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  int64_t kps = (K + splits - 1) / splits;
  kps = (kps + 63) / 64 * 64;  // whole chunks of every variant (and whole kU groups)
  const int used = (int)((K + kps - 1) / kps);
  float *partial = static_cast<float *>(workspace);
  TnJob job{};
  if (K > 0 && tn_staged_plan(K, M, N, A, lda, B, ldb, workspace, workspace_bytes, &job)) {
    const int used2 = job.blocks;
    const int64_t kps2 = job.kps;
    SideFold sf{};
    if (side != nullptr && side->blocks > 0) {
      sf = *side;
      *side_done = true;
    }
    const dim3 grid((unsigned)(used2 + sf.blocks));
    if (N == 32)
      hipLaunchKernelGGL(gemm_tn_staged_kernel<1>, grid, dim3(256), 0, s, A, lda, B, ldb, K,
                         kps2, partial, sf);
    else
      hipLaunchKernelGGL(gemm_tn_staged_kernel<2>, grid, dim3(256), 0, s, A, lda, B, ldb, K,
                         kps2, partial, sf);
    if (int rc = check_launch("gemm_tn_staged_kernel")) return rc;
    if (defer != nullptr && !accumulate) {
      *defer = make_side_fold(partial, used2, (int64_t)M * N, N, C, ldc, N1, C2, ldc2);
      return MGCN_OK;
    }
    return launch_fold_split(partial, used2, (int64_t)M * N, N, C, ldc, N1, C2, ldc2, accumulate,
                             s);
  }
  if (M <= 32 && N <= 64) {
    if (N <= 32)
      hipLaunchKernelGGL(gemm_tn_small_kernel<1>, dim3(used), dim3(256), 0, s, A, lda, B, ldb, K,
                         M, N, kps, partial);
    else
      hipLaunchKernelGGL(gemm_tn_small_kernel<2>, dim3(used), dim3(256), 0, s, A, lda, B, ldb, K,
                         M, N, kps, partial);
    if (int rc = check_launch("gemm_tn_small_kernel")) return rc;
  } else if (tn_lds(M, N) && reinterpret_cast<uintptr_t>(A) % 16 == 0 &&
             reinterpret_cast<uintptr_t>(B) % 16 == 0 && lda % 4 == 0 && ldb % 4 == 0) {
    // 1-D grids of tiles x splits in the kernels' XCD-aware order
    const dim3 grid(tiles_m * tiles_n * used);
    if (g_gemm_precision == PREC_BF16X6 && tn_wide(M, N) && tn_wide_fits(kps, lda, ldb))
      hipLaunchKernelGGL(gemm_tn_x6_wide_kernel, dim3(used), dim3(512), 0, s, A, lda, B, ldb, K,
                         kps, partial);
    else if (g_gemm_precision == PREC_BF16X6)
      hipLaunchKernelGGL(gemm_tn_x6_kernel, grid, dim3(256), 0, s, A, lda, B, ldb, K, M, N, kps,
                         tiles_n, partial);
    else if (g_tn_lds_variant == 1)
      hipLaunchKernelGGL((gemm_tn_lds_kernel<32, 2>), grid, dim3(256), 0, s, A, lda, B, ldb, K, M,
                         N, kps, tiles_n, partial);
    else if (g_tn_lds_variant == 2)
      hipLaunchKernelGGL((gemm_tn_lds_kernel<16, 3>), grid, dim3(256), 0, s, A, lda, B, ldb, K, M,
                         N, kps, tiles_n, partial);
    else
      hipLaunchKernelGGL((gemm_tn_lds_kernel<64, 1>), grid, dim3(256), 0, s, A, lda, B, ldb, K, M,
                         N, kps, tiles_n, partial);
    if (int rc = check_launch("gemm_tn_lds/x6_kernel")) return rc;
  } else {
    hipLaunchKernelGGL(gemm_tn_partial_kernel, dim3(tiles_m * tiles_n, used), dim3(256), 0, s, A,
                       lda, B, ldb, K, M, N, kps, tiles_n, partial);
    if (int rc = check_launch("gemm_tn_partial_kernel")) return rc;
  }
  const int64_t MN = (int64_t)M * N;
  return launch_fold_split(partial, used, MN, N, C, ldc, N1, C2, ldc2, accumulate, s);
}

int gemm_tn_impl(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda, const float *B,
                 int64_t ldb, float *C, int64_t ldc, int32_t N1, float *C2, int64_t ldc2,
                 int accumulate, void *workspace, size_t workspace_bytes, hipStream_t s,
                 const SideFold *side = nullptr, SideFold *defer = nullptr) {
  bool done = false;
  if (defer != nullptr) *defer = SideFold{};
  if (int rc = gemm_tn_core(K, M, N, A, lda, B, ldb, C, ldc, N1, C2, ldc2, accumulate, workspace,
                            workspace_bytes, s, side, &done, defer))
    return rc;
  if (side == nullptr || done) return MGCN_OK;
  return launch_side_fold(*side, s);
}
}  // namespace

extern "C" int mgcn_gemm_tn(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda,
                            const float *B, int64_t ldb, float *C, int64_t ldc, int accumulate,
                            void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(K >= 0 && M >= 0 && N >= 0, "mgcn_gemm_tn: negative size");
  if (M == 0 || N == 0) return MGCN_OK;
  MGCN_REQUIRE(C != nullptr && ldc >= N, "mgcn_gemm_tn: bad C");
  MGCN_REQUIRE(K == 0 || (A && B && lda >= M && ldb >= N), "mgcn_gemm_tn: bad A/B");
  return gemm_tn_impl(K, M, N, A, lda, B, ldb, C, ldc, N, nullptr, 0, accumulate, workspace,
                      workspace_bytes, as_stream(stream));
}

namespace mgcn {
int gemm_tn_split_fold(int64_t K, int32_t M, int32_t N, int32_t N1, const float *A, int64_t lda,
                       const float *B, int64_t ldb, float *C1, int64_t ldc1, float *C2t,
                       int64_t ldc2t, void *workspace, size_t workspace_bytes,
                       const SideFold &side, hipStream_t s, SideFold *defer) {
  return gemm_tn_impl(K, M, N, A, lda, B, ldb, C1, ldc1, N1, C2t, ldc2t, 0, workspace,
                      workspace_bytes, s, &side, defer);
}
}  // namespace mgcn

extern "C" int mgcn_gemm_tn_split(int64_t K, int32_t M, int32_t N, int32_t N1, const float *A,
                                  int64_t lda, const float *B, int64_t ldb, float *C1,
                                  int64_t ldc1, float *C2t, int64_t ldc2t, int accumulate,
                                  void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(K >= 0 && M >= 0 && N >= 0 && 0 <= N1 && N1 <= N,
               "mgcn_gemm_tn_split: need K, M, N >= 0 and 0 <= N1 <= N");
  if (M == 0 || N == 0) return MGCN_OK;
  MGCN_REQUIRE(N1 == 0 || (C1 != nullptr && ldc1 >= N1), "mgcn_gemm_tn_split: bad C1");
  MGCN_REQUIRE(N1 == N || (C2t != nullptr && ldc2t >= M), "mgcn_gemm_tn_split: bad C2t");
  MGCN_REQUIRE(K == 0 || (A && B && lda >= M && ldb >= N), "mgcn_gemm_tn_split: bad A/B");
  return gemm_tn_impl(K, M, N, A, lda, B, ldb, C1, ldc1, N1, C2t, ldc2t, accumulate, workspace,
                      workspace_bytes, as_stream(stream));
}

// ---------------------------------------------------------------------------
// mgcn_gemm_nn: C[M, N] = A[M, K] . B[K, N]   (tall-skinny: M = nodes, K, N = F)
//
// The forward transform H = X W (gcn_base_models.py:201) and the input
// gradient dX = dH W^T of a layer (B = W^T through strides).
//   * B (at most 128 x 128) is staged ONCE per workgroup into LDS as B^T
//     ([n][K + 4]), so a lane reads the 4 consecutive k of its column with one
//     ds_read_b128 (K order inside the MFMA chain is permuted: lane half h
//     takes k = m + h K/2, identically for A and B);
//   * every wave streams its own 32-row subtiles of A straight from HBM into
//     registers -- no LDS staging of A, no barriers, no re-reads: lane
//     (h, r) reads row r's k-range [h K/2, h K/2 + K/2) as float4s;
//   * A arrives in bursts of 8 float4 per lane (one 128-byte line), issued
//     back to back so the line's 8 requests meet in L1, double-buffered in
//     registers: the next burst loads while the current one feeds up to 128
//     v_mfma_f32_32x32x2_f32;
//   * persistent workgroups of 8 waves (grid = resident capacity).
// Epilogue modes:
//   EPI_STORE  C = acc
//   EPI_RELU   (the previous layer's ReLU backward fused into dX):
//              C = Z > 0 ? acc : 0, and per-workgroup column sums of C written
//              to colsum_partial[workgroup][N] (the bias gradient, folded in
//              workgroup order by launch_colsum_fold -- deterministic).
// Roofline: 2 M K N FLOP on 157 TF fp32 MFMA vs 4 M (K + N) bytes (+ 4 M N
// for Z); at K = N = 128: 0.21 ms MFMA vs 0.13 ms (0.19 with Z) at 8 TB/s.

namespace mgcn {
namespace {
using namespace x6;

// the product's rows leave with the nt cache policy (with the SpMM outputs',
// spmm.hip: measured together); MGCN_NT_EXTRA=0 builds the default-policy form
#ifndef MGCN_NT_EXTRA
#define MGCN_NT_EXTRA 1
#endif
__device__ __forceinline__ void nn_store(float *p, float v) {
  if constexpr (MGCN_NT_EXTRA != 0)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

constexpr int kNNWaves = 8;  // waves per workgroup
constexpr int kNNThreads = 64 * kNNWaves;
constexpr int kNNMaxGrid = 1024;  // colsum partial slots
constexpr int EPI_STORE = 0, EPI_RELU = 1, EPI_RELU_DIV = 2;  // DIV: C stored / row_div

template <int K, int NT, int P>
constexpr int nn_lds_bytes() {
  return P == PREC_BF16X6 ? 3 * NT * 32 * (K + 8) * 2 : NT * 32 * (K + 4) * 4;
}

// Column groups (N wider than one workgroup's B^T fits in LDS: K = 256 holds
// 64 columns, K <= 128 holds 128): workgroup b takes column group
// (b >> 3) % n_groups of row stream ((b >> 3) / n_groups) * 8 + (b & 7).  The
// workgroups of one row stream are 8 apart in dispatch order, so they land
// on the same XCD (round-robin dispatch) at the same time and walk the same
// rows in the same order: A is read from HBM once and re-read from that
// XCD's L2 by the other groups.  The grid is a multiple of 8 n_groups
// (n_groups = 1: any grid, b = the row stream).
template <int K, int NT, int EPI, int P>
__global__ __launch_bounds__(kNNThreads, P == PREC_BF16X6 ? 1 : 2) void gemm_nn_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t sbk,
    int64_t sbn, float *__restrict__ C, int64_t ldc, int64_t M, int N,
    const uint32_t *__restrict__ relu_mask, const float *__restrict__ row_div,
    float *__restrict__ colsum_partial, int n_groups) {
  constexpr int KH = K / 2;              // k per lane half
  constexpr int S4 = KH / 4;             // float4 steps per 32-row subtile
  constexpr int GS = (K == 32) ? 2 : 1;  // subtiles per unit (>= 8 steps per unit)
  constexpr int S = GS * S4;             // float4 steps per unit
  constexpr int LDB = K + 4;             // f32: B^T row stride in LDS (floats)
  constexpr int LDK = K + 8;             // bf16x6: split-B^T row stride (bf16)
  __shared__ __attribute__((aligned(16))) char smem[nn_lds_bytes<K, NT, P>()];
  float *BT = reinterpret_cast<float *>(smem);    // f32: [n][LDB]
  __bf16 *BS = reinterpret_cast<__bf16 *>(smem);  // bf16x6: [term][n][LDK]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, lc = lane & 31;
  const int bx = (int)blockIdx.x;
  const int cg = (bx >> 3) % n_groups;                       // column group
  const int rs = ((bx >> 3) / n_groups) * 8 + (bx & 7);      // row stream
  const int n_streams = (int)gridDim.x / n_groups;
  const int n0 = cg * NT * 32;                               // first column of the group

  if constexpr (P == PREC_BF16X6) {
    // B^T split into its three bf16 terms, 8 k per item; columns past N zero
    for (int idx = tid; idx < NT * 32 * (K / 8); idx += kNNThreads) {
      const int n = idx / (K / 8), k8 = (idx % (K / 8)) * 8;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = (n0 + n < N) ? B[(int64_t)(k8 + j) * sbk + (int64_t)(n0 + n) * sbn] : 0.0f;
      bf16x8 th, tm, tl;
      split3_bf16(v, th, tm, tl);
      *reinterpret_cast<bf16x8 *>(&BS[(0 * NT * 32 + n) * LDK + k8]) = th;
      *reinterpret_cast<bf16x8 *>(&BS[(1 * NT * 32 + n) * LDK + k8]) = tm;
      *reinterpret_cast<bf16x8 *>(&BS[(2 * NT * 32 + n) * LDK + k8]) = tl;
    }
  } else {
    // B^T into LDS, columns past N zero
    for (int idx = tid; idx < NT * 32 * (K / 4); idx += kNNThreads) {
      const int n = idx / (K / 4), k4 = (idx % (K / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n0 + n < N) {
        const float *bp = B + (int64_t)k4 * sbk + (int64_t)(n0 + n) * sbn;
        v.x = bp[0];
        v.y = bp[sbk];
        v.z = bp[2 * sbk];
        v.w = bp[3 * sbk];
      }
      *reinterpret_cast<float4 *>(&BT[n * LDB + k4]) = v;
    }
  }
  __syncthreads();

  const int64_t n_sub = (M + 31) / 32;
  const int64_t n_units = (n_sub + GS - 1) / GS;
  const int64_t wstride = (int64_t)n_streams * kNNWaves;
  // A is read in BURSTS of 8 float4 steps = one 128-byte line per lane,
  // issued back to back (the 8 requests of a line meet in L1), into two
  // register banks: burst t + 1 loads while burst t feeds the MFMAs.
  constexpr int NB = S / 8;  // bursts per unit: 4 (K = 256), 2 (K = 128), 1 (K = 64; K = 32: 2 subtiles)
  auto load_burst = [&](int64_t unit, int part, float4 (&bk)[8]) {
    const float4 *rp[GS];
#pragma unroll
    for (int g = 0; g < GS; ++g) {
      int64_t row = (unit * GS + g) * 32 + lc;
      row = row < M ? row : M - 1;  // the tail's rows past M: loaded, never stored
      rp[g] = reinterpret_cast<const float4 *>(A + row * lda + h * KH);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int st = part * 8 + i;
      bk[i] = rp[st / S4][st % S4];
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  const float *bt_lane = &BT[lc * LDB + h * KH];
  float csum[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) csum[j] = 0.0f;
  f32x16 acc[GS][NT];
  auto zero_acc = [&]() {
#pragma unroll
    for (int g = 0; g < GS; ++g)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][j][r] = 0.0f;
  };
  // bf16x6: lane (h, lc) fragment of k-step ks covers k = h KH + 8 ks + j
  // (j = 0..7) of A row lc and of B^T row j * 32 + lc: two float4 of the
  // burst, one ds_read_b128 per term and column tile.
  const __bf16 *bs_lane = &BS[lc * LDK + h * KH];
  // Software pipeline over the burst's 4 k-steps x NT column tiles: the next
  // tile's three B fragments (ds_read_b128) and the next k-step's A split
  // (VALU) are issued before the current tile's six MFMAs, double-buffered
  // in registers, so LDS latency and split work hide under the MFMA chain.
  auto compute_burst_x6 = [&](const float4 (&bk)[8], int part) {
    constexpr int STEPS = 4;  // k-steps per burst (8 float4)
    uint32_t ah[2][4], am[2][4], al[2][4];
    bf16x8 bh[2], bm[2], bl[2];
    auto split_pair = [&](int i, int p, int slot) {  // pair p of k-step i
      const float4 v = bk[2 * i + (p >> 1)];
      const f32x2 x = (p & 1) ? f32x2{v.z, v.w} : f32x2{v.x, v.y};
      split3_pair(x, ah[slot][p], am[slot][p], al[slot][p]);
    };
    auto load_b = [&](int i, int j, int slot) {
      const int ks = ((part * 8 + 2 * i) % S4) / 2;
      const __bf16 *bp = bs_lane + j * 32 * LDK + 8 * ks;
      bh[slot] = *reinterpret_cast<const bf16x8 *>(bp);
      bm[slot] = *reinterpret_cast<const bf16x8 *>(bp + NT * 32 * LDK);
      bl[slot] = *reinterpret_cast<const bf16x8 *>(bp + 2 * NT * 32 * LDK);
    };
    load_b(0, 0, 0);
#pragma unroll
    for (int p = 0; p < 4; ++p) split_pair(0, p, 0);
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {
      const int sub = (part * 8 + 2 * i) / S4;
      const bf16x8 xh = __builtin_bit_cast(bf16x8, ah[i & 1]);
      const bf16x8 xm = __builtin_bit_cast(bf16x8, am[i & 1]);
      const bf16x8 xl = __builtin_bit_cast(bf16x8, al[i & 1]);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int t = i * NT + j;
        // next tile's fragments and a share of the next k-step's split,
        // interleaved with this tile's six MFMAs (MFMA, DS read, 2 VALU, ...)
        if (t + 1 < STEPS * NT) load_b((t + 1) / NT, (t + 1) % NT, (t + 1) & 1);
        if (i + 1 < STEPS) {
#pragma unroll
          for (int p = 0; p < 4; ++p)
            if (p % NT == j) split_pair(i + 1, p, (i + 1) & 1);
        }
        acc[sub][j] = mfma_x6(xh, xm, xl, bh[t & 1], bm[t & 1], bl[t & 1], acc[sub][j]);
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          if (q < 3) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto compute_burst = [&](const float4 (&bk)[8], int part) {
    if constexpr (P == PREC_BF16X6) {
      compute_burst_x6(bk, part);
      return;
    }
    float4 bcur[NT], bnxt[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
      bcur[j] = *reinterpret_cast<const float4 *>(bt_lane + j * 32 * LDB + 4 * ((part * 8) % S4));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int st = part * 8 + i;
      const int sub = st / S4;
      if (i + 1 < 8) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
          bnxt[j] = *reinterpret_cast<const float4 *>(bt_lane + j * 32 * LDB + 4 * ((st + 1) % S4));
      }
      const float4 a = bk[i];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[sub][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bcur[j].x, acc[sub][j], 0, 0, 0);
        acc[sub][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bcur[j].y, acc[sub][j], 0, 0, 0);
        acc[sub][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bcur[j].z, acc[sub][j], 0, 0, 0);
        acc[sub][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bcur[j].w, acc[sub][j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) bcur[j] = bnxt[j];
    }
  };
  // ReLU mask words of the unit's rows (EPI_RELU*): column n = 32 j + lc is
  // bit 8 j + (lc >> 2) of word lc & 3, so a lane needs one word per row --
  // 16 per subtile, loaded when the unit starts (in flight under the MFMAs)
  uint32_t mword[GS][16];
  auto load_mask = [&](int64_t unit) {
    if constexpr (EPI != EPI_STORE) {
#pragma unroll
      for (int g = 0; g < GS; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int64_t row = (unit * GS + g) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          row = row < M ? row : M - 1;
          mword[g][r] = relu_mask[row * 4 + (lc & 3)];
        }
    }
  };
  // epilogue; C/D map: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 h.
  // Addresses = lane pointer + wave-uniform row offset; full subtiles store
  // unguarded, the M tail per element.
  auto epilogue = [&](int64_t unit) {
#pragma unroll
    for (int g = 0; g < GS; ++g) {
      const int64_t r0 = (unit * GS + g) * 32;
      const bool rows_full = r0 + 32 <= M;  // wave-uniform
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + j * 32 + lc;
        const bool n_ok = n < N;
        const int bit = n >> 2;  // EPI_RELU*: N <= 128, one 4-word mask row
        float *cp = C + (r0 + 4 * h) * ldc + n;
        if (rows_full) {
          if constexpr (EPI != EPI_STORE) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float v = ((mword[g][r] >> bit) & 1u) ? acc[g][j][r] : 0.0f;
              if (n_ok) {
                csum[j] = __fadd_rn(csum[j], v);  // bias gradient: undivided
                const int rr = (r & 3) + 8 * (r >> 2);
                if constexpr (EPI == EPI_RELU_DIV)
                  nn_store(cp + rr * ldc, __fdiv_rn(v, row_div[r0 + 4 * h + rr]));
                else
                  nn_store(cp + rr * ldc, v);
              }
            }
          } else {
            if (n_ok) {
#pragma unroll
              for (int r = 0; r < 16; ++r) nn_store(cp + ((r & 3) + 8 * (r >> 2)) * ldc, acc[g][j][r]);
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rr = (r & 3) + 8 * (r >> 2);
            if (n_ok && r0 + 4 * h + rr < M) {
              float v = acc[g][j][r];
              if constexpr (EPI != EPI_STORE) {
                v = ((mword[g][r] >> bit) & 1u) ? v : 0.0f;
                csum[j] = __fadd_rn(csum[j], v);
                if constexpr (EPI == EPI_RELU_DIV) v = __fdiv_rn(v, row_div[r0 + 4 * h + rr]);
              }
              cp[rr * ldc] = v;
            }
          }
        }
      }
    }
  };

  float4 bank0[8], bank1[8];
  int64_t u = (int64_t)rs * kNNWaves + wave;
  if (u < n_units) load_burst(u, 0, bank0);
  if constexpr (NB == 4) {
    for (; u < n_units; u += wstride) {
      const int64_t un = (u + wstride < n_units) ? u + wstride : u;  // last: harmless reload
      zero_acc();
      load_mask(u);
      load_burst(u, 1, bank1);
      compute_burst(bank0, 0);
      load_burst(u, 2, bank0);
      compute_burst(bank1, 1);
      load_burst(u, 3, bank1);
      compute_burst(bank0, 2);
      load_burst(un, 0, bank0);
      compute_burst(bank1, 3);
      epilogue(u);
    }
  } else if constexpr (NB == 2) {
    for (; u < n_units; u += wstride) {
      const int64_t un = (u + wstride < n_units) ? u + wstride : u;  // last: harmless reload
      zero_acc();
      load_mask(u);
      load_burst(u, 1, bank1);
      compute_burst(bank0, 0);
      load_burst(un, 0, bank0);
      compute_burst(bank1, 1);
      epilogue(u);
    }
  } else {
    for (; u < n_units; u += 2 * wstride) {
      const int64_t u1 = u + wstride;
      load_burst(u1 < n_units ? u1 : u, 0, bank1);
      zero_acc();
      load_mask(u);
      compute_burst(bank0, 0);
      epilogue(u);
      if (u1 >= n_units) break;
      const int64_t u2 = u + 2 * wstride;
      load_burst(u2 < n_units ? u2 : u1, 0, bank0);
      zero_acc();
      load_mask(u1);
      compute_burst(bank1, 0);
      epilogue(u1);
    }
  }
  if constexpr (EPI != EPI_STORE) {
    // fold the lane halves, then the waves in wave order (deterministic)
    __syncthreads();  // BT is free
    float *red = BT;  // [kNNWaves][NT * 32]
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float both = __fadd_rn(csum[j], __shfl_xor(csum[j], 32, 64));
      if (h == 0) red[wave * NT * 32 + j * 32 + lc] = both;
    }
    __syncthreads();
    for (int c = tid; c < NT * 32 && n0 + c < N; c += kNNThreads) {
      float v = red[c];
      for (int w = 1; w < kNNWaves; ++w) v = __fadd_rn(v, red[w * NT * 32 + c]);
      colsum_partial[(int64_t)rs * N + n0 + c] = v;  // [row stream][N]
    }
  }
}

// Resident capacity of this instantiation (queried once), capped by work;
// with column groups a multiple of 8 groups (module comment above the kernel).
template <int K, int NT, int EPI, int P>
int nn_blocks(int64_t M, int n_groups) {
  static std::atomic<int> per_cu_cache{0};  // same code object on every device
  int per_cu = per_cu_cache.load(std::memory_order_relaxed);
  if (per_cu == 0) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, gemm_nn_kernel<K, NT, EPI, P>, kNNThreads,
                                                     0) != hipSuccess || b < 1)
      b = 1;
    per_cu = b;
    per_cu_cache.store(b, std::memory_order_relaxed);
  }
  constexpr int GS = (K == 32) ? 2 : 1;
  const int64_t units = ((M + 31) / 32 + GS - 1) / GS;
  int64_t streams = (units + kNNWaves - 1) / kNNWaves;
  int64_t cap = 256LL * per_cu / n_groups;
  if (cap > kNNMaxGrid) cap = kNNMaxGrid;  // colsum partial slots: one per row stream
  if (streams > cap) streams = cap;
  if (n_groups > 1) streams = streams < 8 ? 8 : streams / 8 * 8;
  return (int)((streams > 0 ? streams : 1) * n_groups);
}

template <int K, int NT, int EPI, int P>
int launch_nn_epi(int64_t M, int N, const float *A, int64_t lda, const float *B, int64_t sbk,
                  int64_t sbn, float *C, int64_t ldc, const uint32_t *mask,
                  const float *row_div, float *partial, int *streams_out, hipStream_t s) {
  const int n_groups = (N + NT * 32 - 1) / (NT * 32);
  const int g = nn_blocks<K, NT, EPI, P>(M, n_groups);
  hipLaunchKernelGGL((gemm_nn_kernel<K, NT, EPI, P>), dim3(g), dim3(kNNThreads), 0, s, A, lda, B,
                     sbk, sbn, C, ldc, M, N, mask, row_div, partial, n_groups);
  *streams_out = g / n_groups;
  return check_launch("gemm_nn_kernel");
}

template <int K, int NT, int P>
int launch_nn_nt(int64_t M, int N, const float *A, int64_t lda, const float *B, int64_t sbk,
                 int64_t sbn, float *C, int64_t ldc, int epi, const uint32_t *Z,
                 const float *rd, float *partial, int *grid_out, hipStream_t s) {
  if (epi == EPI_RELU_DIV)
    return launch_nn_epi<K, NT, EPI_RELU_DIV, P>(M, N, A, lda, B, sbk, sbn, C, ldc, Z, rd,
                                                 partial, grid_out, s);
  if (epi == EPI_RELU)
    return launch_nn_epi<K, NT, EPI_RELU, P>(M, N, A, lda, B, sbk, sbn, C, ldc, Z, rd, partial,
                                             grid_out, s);
  return launch_nn_epi<K, NT, EPI_STORE, P>(M, N, A, lda, B, sbk, sbn, C, ldc, Z, rd, partial,
                                            grid_out, s);
}

// Column tiles per workgroup: the split B^T (3 bf16 terms, K + 8 per row)
// must fit the 160 KB of LDS -- K = 256: 64 columns (101 KB), K <= 128: 128.
// Wider N runs as column groups.
template <int K, int P>
int launch_nn_p(int64_t M, int N, const float *A, int64_t lda, const float *B, int64_t sbk,
                int64_t sbn, float *C, int64_t ldc, int epi, const uint32_t *Z,
                const float *rd, float *partial, int *grid_out, hipStream_t s) {
  const int nt = (N + 31) / 32;
  if constexpr (K == 256) {
    if (nt == 1)
      return launch_nn_nt<K, 1, P>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial, grid_out, s);
    return launch_nn_nt<K, 2, P>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial, grid_out, s);
  } else {
    if (nt == 1)
      return launch_nn_nt<K, 1, P>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial, grid_out, s);
    if (nt == 2)
      return launch_nn_nt<K, 2, P>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial, grid_out, s);
    if (nt == 3)
      return launch_nn_nt<K, 3, P>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial, grid_out, s);
    return launch_nn_nt<K, 4, P>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial, grid_out, s);
  }
}

template <int K>
int launch_nn(int64_t M, int N, const float *A, int64_t lda, const float *B, int64_t sbk,
              int64_t sbn, float *C, int64_t ldc, int epi, const uint32_t *Z,
              const float *rd, float *partial, int *grid_out, hipStream_t s) {
  if (g_gemm_precision == PREC_BF16X6)
    return launch_nn_p<K, PREC_BF16X6>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial,
                                       grid_out, s);
  return launch_nn_p<K, PREC_F32>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, Z, rd, partial,
                                  grid_out, s);
}

// ---------------------------------------------------------------------------
// Any other shape (K not in {32, 64, 128, 256}, rows not 16-byte aligned, B
// through any strides): C[M, N] = A[M, K] B[K, N] on 64 x 64 output tiles,
// one per 256-thread workgroup (four waves of 32 x 32), the K range in
// chunks of 16 staged through LDS -- bounds-checked element loads, the
// fp32 operands split into their three bf16 terms (row-major [row][16 k]
// images, B transposed) and multiplied on v_mfma_f32_32x32x16_bf16 (bf16x6),
// or kept fp32 for v_mfma_f32_32x32x2_f32 (gemm_precision 0).  Two LDS
// buffers, one barrier per chunk.  Not a roofline kernel: it covers the
// shapes of the module surface the tuned kernels do not take (TU input
// widths such as 3 / 21 / 89, hidden 16, classifier heads) so that no
// product GEMM runs on a vendor library.
constexpr int kGenT = 64, kGenK = 16, kGenThreads = 256;

template <int P>
__global__ __launch_bounds__(kGenThreads) void gemm_gen_kernel(
    const float *__restrict__ A, int64_t lda, const float *__restrict__ B, int64_t sbk,
    int64_t sbn, float *__restrict__ C, int64_t ldc, int64_t M, int K, int N) {
  // x6: [buf][A | B^T][term][64][16] bf16; f32: [buf][A | B^T][64][16 + 1] fp32
  constexpr int kImg = kGenT * kGenK * 2;            // one bf16 term image (2 KB)
  constexpr int kF32Ld = kGenK + 1;
  constexpr int kBufBytes = P == PREC_BF16X6 ? 2 * 3 * kImg : 2 * kGenT * kF32Ld * 4;
  __shared__ __attribute__((aligned(16))) char lds[2 * kBufBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int h = lane >> 5, lc = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * kGenT;
  const int n0 = (int)blockIdx.y * kGenT;
  // staging: A element (row t >> 2, k 4 (t & 3) + i), B element (k 4 (t >> 6) + i, col t & 63)
  const int ar = tid >> 2, ak = 4 * (tid & 3);
  const int bn = tid & 63, bk = 4 * (tid >> 6);
  const bool a_row_ok = m0 + ar < M;
  const bool b_col_ok = n0 + bn < N;
  const float *ap = A + (m0 + ar) * lda;
  const float *bp = B + (int64_t)(n0 + bn) * sbn;
  float ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ka = k0 + ak + i, kb = k0 + bk + i;
      ra[i] = (a_row_ok && ka < K) ? ap[ka] : 0.0f;
      rb[i] = (b_col_ok && kb < K) ? bp[(int64_t)kb * sbk] : 0.0f;
    }
  };
  auto store = [&](char *buf) {
    if constexpr (P == PREC_BF16X6) {
#pragma unroll
      for (int op = 0; op < 2; ++op) {
        const float *v = op ? rb : ra;
        uint32_t hi[2], mid[2], lo[2];
        split3_pair(f32x2{v[0], v[1]}, hi[0], mid[0], lo[0]);
        split3_pair(f32x2{v[2], v[3]}, hi[1], mid[1], lo[1]);
        const int row = op ? bn : ar, k = op ? bk : ak;
        char *img = buf + op * 3 * kImg + (row * kGenK + k) * 2;
        *reinterpret_cast<uint2 *>(img) = make_uint2(hi[0], hi[1]);
        *reinterpret_cast<uint2 *>(img + kImg) = make_uint2(mid[0], mid[1]);
        *reinterpret_cast<uint2 *>(img + 2 * kImg) = make_uint2(lo[0], lo[1]);
      }
    } else {
      float *fa = reinterpret_cast<float *>(buf);
      float *fb = fa + kGenT * kF32Ld;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[ar * kF32Ld + ak + i] = ra[i];
        fb[bn * kF32Ld + bk + i] = rb[i];
      }
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  const int nk = (K + kGenK - 1) / kGenK;
  load(0);
  store(lds);
  __syncthreads();
  for (int c = 0; c < nk; ++c) {
    const char *buf = lds + (c & 1) * kBufBytes;
    if (c + 1 < nk) load((c + 1) * kGenK);
    if constexpr (P == PREC_BF16X6) {
      // lane (h, lc): row lc of the wave's 32-row A tile / column lc of its
      // B tile, k = 8 h .. 8 h + 7 of the chunk
      const char *pa = buf + ((32 * wi + lc) * kGenK + 8 * h) * 2;
      const char *pb = buf + 3 * kImg + ((32 * wj + lc) * kGenK + 8 * h) * 2;
      const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(pa);
      const bf16x8 am = *reinterpret_cast<const bf16x8 *>(pa + kImg);
      const bf16x8 al = *reinterpret_cast<const bf16x8 *>(pa + 2 * kImg);
      const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(pb);
      const bf16x8 bm = *reinterpret_cast<const bf16x8 *>(pb + kImg);
      const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(pb + 2 * kImg);
      acc = mfma_x6(ah, am, al, bh, bm, bl, acc);
    } else {
      const float *fa = reinterpret_cast<const float *>(buf) + (32 * wi + lc) * kF32Ld;
      const float *fb = reinterpret_cast<const float *>(buf) + kGenT * kF32Ld + (32 * wj + lc) * kF32Ld;
#pragma unroll
      for (int ks = 0; ks < kGenK / 2; ++ks)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[2 * ks + h], fb[2 * ks + h], acc, 0, 0, 0);
    }
    if (c + 1 < nk) store(lds + ((c + 1) & 1) * kBufBytes);
    __syncthreads();
  }
  // C/D map: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 h
  const int n = n0 + 32 * wj + lc;
  if (n < N) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = m0 + 32 * wi + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row < M) C[row * ldc + n] = acc[r];
    }
  }
}

int launch_gen(int64_t M, int K, int N, const float *A, int64_t lda, const float *B, int64_t sbk,
               int64_t sbn, float *C, int64_t ldc, hipStream_t s) {
  const dim3 grid((unsigned)((M + kGenT - 1) / kGenT), (unsigned)((N + kGenT - 1) / kGenT));
  if (g_gemm_precision == PREC_BF16X6)
    hipLaunchKernelGGL(gemm_gen_kernel<PREC_BF16X6>, grid, dim3(kGenThreads), 0, s, A, lda, B, sbk,
                       sbn, C, ldc, M, K, N);
  else
    hipLaunchKernelGGL(gemm_gen_kernel<PREC_F32>, grid, dim3(kGenThreads), 0, s, A, lda, B, sbk,
                       sbn, C, ldc, M, K, N);
  return check_launch("gemm_gen_kernel");
}

// Deterministic fold of split partial sums: C[e] (+)= sum over sp of
// partial[sp][e] (C[e] at row e / N, column e % N).  A 256-thread block owns
// EB consecutive elements and T = 256 / EB interleaved split groups per
// element; group g adds splits g, g + T, ... in order, then the T group sums
// meet in a fixed binary tree.  EB shrinks with MN so that small folds (dW of
// F = 32 layers, bias column sums) still spread over many lanes: the 4-group
// form of round 1 left 12-13 us per fold of 32 x 32 or 32 values.
__global__ __launch_bounds__(256) void fold_partials_kernel(const float *__restrict__ partial,
                                                            int64_t splits, int64_t MN, int N,
                                                            float *__restrict__ C, int64_t ldc,
                                                            int accumulate, int log_eb, int N1,
                                                            float *__restrict__ C2,
                                                            int64_t ldc2) {
  __shared__ float red[256];
  const int EB = 1 << log_eb, T = 256 >> log_eb;
  const int el = threadIdx.x & (EB - 1), g = threadIdx.x >> log_eb;
  const int64_t e = (int64_t)blockIdx.x * EB + el;
  float acc = 0.0f;
  if (e < MN) {
#pragma unroll 4
    for (int64_t sp = g; sp < splits; sp += T) acc = __fadd_rn(acc, partial[sp * MN + e]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = T >> 1; h >= 1; h >>= 1) {
    if (g < h) red[threadIdx.x] = __fadd_rn(red[threadIdx.x], red[threadIdx.x + h * EB]);
    __syncthreads();
  }
  if (g == 0 && e < MN) {
    const float v = red[el];
    const int64_t row = e / N, col = e % N;
    float *dst = col < N1 ? C + row * ldc + col : C2 + (col - N1) * ldc2 + row;
    *dst = accumulate ? __fadd_rn(*dst, v) : v;
  }
}

}  // namespace

// launchers of the split-K / column-sum folds, also for other translation
// units (fused.hip's backward and elementwise.hip write the same partial slabs)
int launch_fold(const float *partial, int64_t splits, int64_t MN, int N, float *C, int64_t ldc,
                int accumulate, hipStream_t s) {
  return launch_fold_split(partial, splits, MN, N, C, ldc, N, nullptr, 0, accumulate, s);
}

// columns [N1, N) of the folded [MN / N, N] result go transposed to C2
int launch_fold_split(const float *partial, int64_t splits, int64_t MN, int N, float *C,
                      int64_t ldc, int N1, float *C2, int64_t ldc2, int accumulate, hipStream_t s) {
  if (MN <= 0) return MGCN_OK;
  int log_eb = 0;  // EB = clamp(pow2 <= MN / 256, 1, 16)
  while (log_eb < 4 && (MN >> (log_eb + 9)) > 0) ++log_eb;
  const int64_t blocks = (MN + (1 << log_eb) - 1) >> log_eb;
  hipLaunchKernelGGL(fold_partials_kernel, dim3((unsigned)blocks), dim3(256), 0, s, partial,
                     splits, MN, N, C, ldc, accumulate, log_eb, N1, C2, ldc2);
  return check_launch("fold_partials_kernel");
}

SideFold make_side_fold(const float *partial, int64_t parts, int64_t MN, int N, float *C,
                        int64_t ldc, int N1, float *C2, int64_t ldc2) {
  SideFold f{};
  if (MN <= 0) return f;
  int log_eb = 0;  // as launch_fold_split
  while (log_eb < 4 && (MN >> (log_eb + 9)) > 0) ++log_eb;
  f.partial = partial;
  f.parts = parts;
  f.MN = MN;
  f.N = N;
  f.N1 = N1;
  f.log_eb = log_eb;
  f.blocks = (int)((MN + (1 << log_eb) - 1) >> log_eb);
  f.C = C;
  f.C2 = C2;
  f.ldc = ldc;
  f.ldc2 = ldc2;
  return f;
}

int launch_side_fold(const SideFold &f, hipStream_t s) {
  if (f.blocks <= 0) return MGCN_OK;
  hipLaunchKernelGGL(fold_partials_kernel, dim3((unsigned)f.blocks), dim3(256), 0, s, f.partial,
                     f.parts, f.MN, f.N, f.C, f.ldc, 0, f.log_eb, f.N1, f.C2, f.ldc2);
  return check_launch("fold_partials_kernel");
}

int launch_split_reduce(const float *partial, int splits, int64_t MN, int N, float *C,
                        int64_t ldc, int accumulate, hipStream_t s) {
  return launch_fold(partial, splits, MN, N, C, ldc, accumulate, s);
}

int launch_colsum_fold(const float *partial, int64_t nparts, int N, float *out, hipStream_t s) {
  return launch_fold(partial, nparts, N, N, out, N, 0, s);
}

int gemm_precision_is_x6() { return g_gemm_precision == PREC_BF16X6; }

int gemm_set_precision(int value) {
  if (value != PREC_F32 && value != PREC_BF16X6) return MGCN_EINVAL;
  g_gemm_precision = value;
  return MGCN_OK;
}

}  // namespace mgcn

namespace {
// the tuned tall-skinny kernel: K in {32, 64, 128, 256}, 16-byte aligned A rows
bool nn_fast(int32_t K, const float *A, int64_t lda) {
  return (K == 32 || K == 64 || K == 128 || K == 256) && lda % 4 == 0 &&
         reinterpret_cast<uintptr_t>(A) % 16 == 0;
}
}  // namespace

extern "C" int mgcn_gemm_nn_supported(int32_t K, int32_t N) {
  return K >= 1 && N >= 1;  // every shape: the tuned kernel or gemm_gen_kernel
}

extern "C" int mgcn_gemm_nn_fast(int32_t K, int32_t N) {
  return (K == 32 || K == 64 || K == 128 || K == 256) && N >= 1;
}

extern "C" int mgcn_gemm_nn_epi_supported(int32_t K, int32_t N) {
  // the fused ReLU-mask epilogue: the tuned kernel, one 4-word mask row (N <= 128)
  return mgcn_gemm_nn_fast(K, N) && N <= 128;
}

extern "C" size_t mgcn_gemm_nn_workspace_bytes(int64_t M, int32_t N) {
  (void)M;
  return align_up((size_t)kNNMaxGrid * (size_t)(N > 0 ? N : 1) * 4, 256);
}

extern "C" int mgcn_gemm_nn(int64_t M, int32_t K, int32_t N, const float *A, int64_t lda,
                            const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                            const uint32_t *relu_mask, const float *row_div, float *colsum,
                            void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(M >= 0 && K >= 0 && N >= 0, "mgcn_gemm_nn: negative size");
  MGCN_REQUIRE(K >= 1 && N >= 1, "mgcn_gemm_nn: unsupported K=%d N=%d", K, N);
  hipStream_t s = as_stream(stream);
  const int epi = relu_mask == nullptr ? EPI_STORE : row_div != nullptr ? EPI_RELU_DIV : EPI_RELU;
  if (M == 0) {
    if (colsum) MGCN_HIP_TRY(hipMemsetAsync(colsum, 0, sizeof(float) * N, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(A && B && C && lda >= K && ldc >= N, "mgcn_gemm_nn: bad A/B/C");
  MGCN_REQUIRE(epi == EPI_STORE || colsum != nullptr, "mgcn_gemm_nn: relu_mask given without colsum");
  MGCN_REQUIRE(row_div == nullptr || relu_mask != nullptr, "mgcn_gemm_nn: row_div needs relu_mask");
  const bool fast = nn_fast(K, A, lda);
  MGCN_REQUIRE(epi == EPI_STORE || (fast && N <= 128),
               "mgcn_gemm_nn: the ReLU-mask epilogue needs K in {32, 64, 128, 256}, N <= 128 and "
               "16-byte aligned A rows (K=%d N=%d)", K, N);
  if (!fast) return launch_gen(M, K, N, A, lda, B, sbk, sbn, C, ldc, s);
  float *partial = nullptr;
  if (epi != EPI_STORE) {
    const size_t need = mgcn_gemm_nn_workspace_bytes(M, N);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_gemm_nn: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    partial = static_cast<float *>(workspace);
  }
  int rc;
  int streams = 0;
  if (K == 32)
    rc = launch_nn<32>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, relu_mask, row_div, partial, &streams, s);
  else if (K == 64)
    rc = launch_nn<64>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, relu_mask, row_div, partial, &streams, s);
  else if (K == 128)
    rc = launch_nn<128>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, relu_mask, row_div, partial, &streams, s);
  else
    rc = launch_nn<256>(M, N, A, lda, B, sbk, sbn, C, ldc, epi, relu_mask, row_div, partial, &streams, s);
  if (rc || epi == EPI_STORE) return rc;
  return launch_colsum_fold(partial, streams, N, colsum, s);
}

// ---------------------------------------------------------------------------
// mgcn_gemm_bwd: both dense adjoints of H = X W from ONE pass over X and dH
// (F_in = F_out = 128, bf16x6):
//   dW  = X^T dH                                (split over the chip, as gemm_tn)
//   dX  = relu'(X) * (dH W^T) [/ row_div]       (as gemm_nn with EPI_RELU*)
//   colsum[n] = sum_m relu'(X) (dH W^T)[m, n]   (the lower layer's bias gradient)
// The separate kernels read dH twice and X once (1.5 GB at config 2) plus
// write dX; here every 32-row chunk of X and dH is loaded once, split into
// its three bf16 terms in LDS, and feeds both products: 1 GB read + 0.5 GB
// written per launch.
//   * persistent grid of kBwGrid 512-thread workgroups (one per CU, fixed so
//     the split-K fold order is fixed); chunk c goes to workgroup c % grid;
//   * register prefetch two chunks ahead (two banks of 4 float4 per thread),
//     LDS double buffer, one barrier per chunk;
//   * dW: wave w owns the 32 x 32 tiles (w >> 1, 2 (w & 1) + {0, 1}) on
//     v_mfma_f32_32x32x16_bf16 (operands by ds_read_b64_tr_b16 transposed
//     reads of the row-major images, as gemm_tn_x6);
//   * dX: wave w owns output columns 16 w .. 16 w + 15 of the chunk's 32 rows
//     (two 16 x 16 tiles) on v_mfma_f32_16x16x32_bf16; its W^T fragments are
//     split once and stay in registers (48 VGPRs), the dH fragments are
//     ds_read_b128 row reads of the same image the dW pass reads transposed;
//   * image swizzle: 16-B chunk ch of row r at ch ^ ((r & 3) << 2 | G[(r >> 2) & 3]),
//     G = {0, 2, 3, 1}: conflict-free for the transposed reads (the four rows
//     of a read differ in bits 2-3) AND for the 16x16x32 row reads (the lane
//     groups {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31} of ds_read_b128 land
//     on 16 distinct chunks; with G = {0, 1, 2, 3} they are 2-way).
// Roofline at M = 1M: 1.54 GB (X, dH read; dX written; 16 B/row mask) ->
// 0.24 ms at 6.3 TB/s; 2 x 33.6 GFLOP x 6 bf16 products = 403 GFLOP -> 0.16 ms
// at 2.5 PF: HBM-bound.

namespace mgcn {
namespace {
using namespace x6;


constexpr int kBwF = 128;
constexpr int kBwRows = 32;
constexpr int kBwWaves = 8;
constexpr int kBwThreads = 64 * kBwWaves;
constexpr int kBwGrid = 256;
constexpr int kBwImg = kBwRows * 256;             // one bf16 term image of a chunk operand
constexpr int kBwMaskOff = 6 * kBwImg;            // [32 rows][4] u32 ReLU mask words
constexpr int kBwDivOff = kBwMaskOff + kBwRows * 16;  // [32] row divisors
constexpr int kBwBuf = kBwDivOff + kBwRows * 4;

struct BwBank {
  u32x4 v[4];  // X rows q, 16 + q and dH rows q, 16 + q (q = tid >> 5), float4 tid & 31
  u32x4 mk;    // mask words of row tid & 31
  uint32_t rd; // row divisor of row tid & 31
  u32x4 sv[2]; // SCS: rows q, 16 + q of S
};

// HCS (dW only): also the column sums of dH -- the bias gradient of the
// layer whose output gradient dH is (gcn_base_models.py:240) -- from the
// staged rows, so that pass needs no second read of dH.
// SCS (dW only, ABI v20): also the column sums of another [M, 128] matrix S
// streamed beside X and dH (a stack's top-layer bias gradient folded into the
// bottom layer's pass) into s_partial.
template <int EPI, bool DX, bool HCS = false, bool SCS = false>
__global__ __launch_bounds__(kBwThreads, 1) void gemm_bwd_kernel(
    const float *__restrict__ X, int64_t ldx, const float *__restrict__ dH, int64_t lddh,
    const float *__restrict__ W, int64_t ldw, int64_t M, float *__restrict__ dX, int64_t lddx,
    const uint32_t *__restrict__ relu_mask, const float *__restrict__ row_div,
    float *__restrict__ dw_partial, float *__restrict__ colsum_partial,
    const float *__restrict__ S = nullptr, int64_t lds_ = 0, float *__restrict__ s_partial = nullptr) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kBwBuf];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, lc = lane & 31;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int64_t n_chunks = (M + kBwRows - 1) / kBwRows;
  auto rows_in = [&](int64_t chunk) -> uint32_t {  // valid rows of a chunk (0 past the end)
    const int64_t r = M - chunk * kBwRows;
    return (uint32_t)(r <= 0 ? 0 : r >= kBwRows ? kBwRows : r);
  };

  // dX: W^T fragments of this wave's 16 columns, split once (B[k][n] = W[n][k])
  bf16x8 wb[4][3];
  if constexpr (DX) {
    const float *wp = W + (int64_t)(16 * wave + l16) * ldw + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = wp[32 * ks + j];
      split3_bf16(v, wb[ks][0], wb[ks][1], wb[ks][2]);
    }
  }

  const int ld_off_x = 4 * (int)((tid >> 5) * ldx + 4 * (tid & 31));
  const int ld_off_h = 4 * (int)((tid >> 5) * lddh + 4 * (tid & 31));
  auto load = [&](int64_t chunk, BwBank &b) {
    const int64_t r0 = chunk * kBwRows;
    const uint32_t rv = rows_in(chunk);
    const auto rx = buf_rsrc(X + r0 * ldx, rv * (uint32_t)ldx * 4u);
    const auto rh = buf_rsrc(dH + r0 * lddh, rv * (uint32_t)lddh * 4u);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      b.v[m] = __builtin_amdgcn_raw_buffer_load_b128(rx, ld_off_x + m * 64 * (int)ldx, 0,
                                                     MGCN_NT_AUX);
      b.v[2 + m] = __builtin_amdgcn_raw_buffer_load_b128(rh, ld_off_h + m * 64 * (int)lddh, 0, 0);
    }
    if constexpr (SCS) {
      const auto rs = buf_rsrc(S + r0 * lds_, rv * (uint32_t)lds_ * 4u);
#pragma unroll
      for (int m = 0; m < 2; ++m)
        b.sv[m] = __builtin_amdgcn_raw_buffer_load_b128(
            rs, 4 * (int)((tid >> 5) * lds_ + 4 * (tid & 31)) + m * 64 * (int)lds_, 0, MGCN_NT_AUX);
    }
    if constexpr (DX && EPI != EPI_STORE) {
      const auto rm = buf_rsrc(relu_mask + r0 * 4, rv * 16u);
      b.mk = __builtin_amdgcn_raw_buffer_load_b128(rm, 16 * (tid & 31), 0, 0);
      if constexpr (EPI == EPI_RELU_DIV) {
        const auto rd = buf_rsrc(row_div + r0, rv * 4u);
        b.rd = __builtin_amdgcn_raw_buffer_load_b32(rd, 4 * (tid & 31), 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // issue the prefetch here, not where the scheduler sinks it
  };
  // staging of one float4 per thread (m = 0, 1: X rows q, 16 + q; 2, 3: dH),
  // the mask / divisor words with the last part; called in pieces between the
  // MFMA steps of the previous chunk so the split VALU work and the LDS
  // writes run under them
  float hc[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // HCS: dH column sums of float4 tid & 31
  float sc[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // SCS: S column sums of float4 tid & 31
  auto stage_part = [&](const BwBank &b, char *buf, int m) {
    const int c4 = tid & 31;
    const int row = 16 * (m & 1) + (tid >> 5);
    const int off = img_off(row, c4 >> 1) + 8 * (c4 & 1);
    const float4 v = __builtin_bit_cast(float4, b.v[m]);
    if constexpr (SCS) {
      if (m >= 2) {  // rows q then 16 + q of every chunk, as hc
        const float4 u = __builtin_bit_cast(float4, b.sv[m - 2]);
        sc[0] = __fadd_rn(sc[0], u.x);
        sc[1] = __fadd_rn(sc[1], u.y);
        sc[2] = __fadd_rn(sc[2], u.z);
        sc[3] = __fadd_rn(sc[3], u.w);
      }
    }
    if constexpr (HCS) {
      // every chunk is staged once (chunks past the end as zeros), rows q
      // then 16 + q: a fixed summation order
      if (m >= 2) {
        hc[0] = __fadd_rn(hc[0], v.x);
        hc[1] = __fadd_rn(hc[1], v.y);
        hc[2] = __fadd_rn(hc[2], v.z);
        hc[3] = __fadd_rn(hc[3], v.w);
      }
    }
    uint32_t hi[2], mid[2], lo[2];
    split3_pair(f32x2{v.x, v.y}, hi[0], mid[0], lo[0]);
    split3_pair(f32x2{v.z, v.w}, hi[1], mid[1], lo[1]);
    char *img = buf + (m >> 1) * 3 * kBwImg + off;
    *reinterpret_cast<uint2 *>(img) = make_uint2(hi[0], hi[1]);
    *reinterpret_cast<uint2 *>(img + kBwImg) = make_uint2(mid[0], mid[1]);
    *reinterpret_cast<uint2 *>(img + 2 * kBwImg) = make_uint2(lo[0], lo[1]);
    if constexpr (DX && EPI != EPI_STORE) {
      if (m == 3 && wave == 0) {
        if (h == 0) *reinterpret_cast<u32x4 *>(buf + kBwMaskOff + 16 * lc) = b.mk;
        if constexpr (EPI == EPI_RELU_DIV)
          if (h == 1) *reinterpret_cast<uint32_t *>(buf + kBwDivOff + 4 * lc) = b.rd;
      }
    }
  };
  auto stage = [&](const BwBank &b, char *buf) {
#pragma unroll
    for (int m = 0; m < 4; ++m) stage_part(b, buf, m);
  };

  // dW fragment offsets (gemm_tn_x6 mapping): lane = 16 g + 4 q + p reads
  // row 8 h + q (+ 4) of chunk (col0 >> 3) + 2 (g & 1) + (p >> 1), half p & 1
  const int q = (lane >> 2) & 3, p = lane & 3;
  auto frag_off = [&](int col0, int second) {
    return img_off(8 * h + q + 4 * second, (col0 >> 3) + 2 * (g4 & 1) + (p >> 1)) + 8 * (p & 1);
  };
  const int ti = wave >> 1, tj0 = 2 * (wave & 1);
  int offa[2], offb[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    offa[r] = frag_off(32 * ti, r);
    offb[0][r] = 3 * kBwImg + frag_off(32 * tj0, r);
    offb[1][r] = 3 * kBwImg + frag_off(32 * (tj0 + 1), r);
  }
  auto read8 = [&](const char *base, const int (&o)[2]) {
    const v4i16 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t *)(base + o[0]));
    const v4i16 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t *)(base + o[1]));
    const short y[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, y);
  };

  f32x16 accw[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int r = 0; r < 16; ++r) accw[s][r] = 0.0f;
  float csum = 0.0f;
  const int ncol = 16 * wave + l16;  // dX column of this lane
  const int mword = ncol & 3, mbit = 8 * (ncol >> 5) + ((ncol & 31) >> 2);

  auto compute = [&](int64_t chunk, const char *buf, const BwBank &nb, char *nbuf) {
    // dW: two 16-row k-steps
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const char *kb = buf + ks * 16 * 256;
      bf16x8 fa[3], fb[2][3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        fa[t] = read8(kb + t * kBwImg, offa);
        fb[0][t] = read8(kb + t * kBwImg, offb[0]);
        fb[1][t] = read8(kb + t * kBwImg, offb[1]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
        accw[s] = mfma_x6(fa[0], fa[1], fa[2], fb[s][0], fb[s][1], fb[s][2], accw[s]);
      stage_part(nb, nbuf, ks);
      if constexpr (!DX) stage_part(nb, nbuf, 2 + ks);
    }
    if constexpr (DX) {
      f32x4_t acc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][r] = 0.0f;
      const char *hb = buf + 3 * kBwImg;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int off = img_off(16 * t + l16, 4 * ks + g4);
          const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(hb + off);
          const bf16x8 am = *reinterpret_cast<const bf16x8 *>(hb + kBwImg + off);
          const bf16x8 al = *reinterpret_cast<const bf16x8 *>(hb + 2 * kBwImg + off);
          acc[t] = mfma16_x6(ah, am, al, wb[ks][0], wb[ks][1], wb[ks][2], acc[t]);
          if (t == 1 && ks < 2) stage_part(nb, nbuf, 2 + ks);
        }
      // epilogue: lane holds rows 16 t + 4 g4 + r of column ncol; rows past M
      // are zero (their loads returned 0) and their stores fall off the buffer
      const int64_t r0 = chunk * kBwRows;
      const auto rx = buf_rsrc(dX + r0 * lddx, rows_in(chunk) * (uint32_t)lddx * 4u);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * t + 4 * g4 + r;
          float v = acc[t][r];
          if constexpr (EPI != EPI_STORE) {
            const uint32_t wd = *reinterpret_cast<const uint32_t *>(buf + kBwMaskOff + 16 * lr + 4 * mword);
            v = ((wd >> mbit) & 1u) ? v : 0.0f;
            csum = __fadd_rn(csum, v);
            if constexpr (EPI == EPI_RELU_DIV)
              v = __fdiv_rn(v, *reinterpret_cast<const float *>(buf + kBwDivOff + 4 * lr));
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rx,
                                                4 * (int)(lr * lddx + ncol), 0,
                                                MGCN_NT_EXTRA ? 2 : 0);
        }
    }
  };

  // D = 2 register banks: chunk i + 2 is loaded while chunk i is computed
  // (four banks, three chunks in flight, measured 0.224 vs 0.214 ms for the
  // dW-only pass: it is issue-bound)
  constexpr int D = 2;
  static_assert(D % 2 == 0, "chunk i reads LDS buffer i & 1: the bank count must be even");
  BwBank bk[D];
  const int64_t c0 = blockIdx.x;
  const int64_t G = gridDim.x;
#pragma unroll
  for (int j = 0; j < D; ++j) load(c0 + j * G, bk[j]);
  stage(bk[0], lds);  // the grid never exceeds the chunk count
  __syncthreads();
  // chunk i (= c0 + i G, bank i % D, LDS buffer i & 1): its bank was staged
  // during chunk i - 1, so it takes the prefetch of chunk i + D; the MFMAs
  // read buffer i & 1 while chunk i + 1 is staged into the other buffer
  // (a chunk past the end stages zeros that are never read: no branches)
  // 32-bit chunk counters: the loop tests stay scalar (a 64-bit compare
  // takes a VGPR temporary, whose reuse made the latch wait for every load)
  const int n_my = c0 < n_chunks ? (int)((n_chunks - 1 - c0) / G) + 1 : 0;
  for (int i = 0; i < n_my; i += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      // leave both loops at once: a break into the latch would merge the
      // partial iterations' load counts into the back edge (vmcnt(4) waits)
      if (j > 0 && i + j >= n_my) goto chunks_done;
      const int64_t ci = c0 + (int64_t)(i + j) * G;
      load(ci + D * G, bk[j]);
      compute(ci, lds + (j & 1) * kBwBuf, bk[(j + 1) % D], lds + ((j + 1) & 1) * kBwBuf);
      __syncthreads();
    }
  }
chunks_done:

  // dW partial slab of this workgroup; C map: col = lc, row = (r & 3) + 8 (r >> 2) + 4 h
  float *slab = dw_partial + (int64_t)blockIdx.x * kBwF * kBwF;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * ti + (r & 3) + 8 * (r >> 2) + 4 * h;
      slab[row * kBwF + 32 * (tj0 + s) + lc] = accw[s][r];
    }
  if constexpr (HCS) {
    // fold the 16 row groups (tid >> 5) of each column in fixed order; the
    // loop's last barrier has retired every read of the LDS images
    float *red = reinterpret_cast<float *>(lds);
    *reinterpret_cast<float4 *>(red + 4 * tid) = make_float4(hc[0], hc[1], hc[2], hc[3]);
    __syncthreads();
    if (tid < kBwF) {
      float c = 0.0f;
#pragma unroll
      for (int g = 0; g < 16; ++g) c = __fadd_rn(c, red[4 * (32 * g + (tid >> 2)) + (tid & 3)]);
      colsum_partial[(int64_t)blockIdx.x * kBwF + tid] = c;
    }
  }
  if constexpr (SCS) {
    __syncthreads();  // (HCS's fold, if any, has read its LDS)
    float *red = reinterpret_cast<float *>(lds);
    *reinterpret_cast<float4 *>(red + 4 * tid) = make_float4(sc[0], sc[1], sc[2], sc[3]);
    __syncthreads();
    if (tid < kBwF) {
      float c = 0.0f;
#pragma unroll
      for (int g = 0; g < 16; ++g) c = __fadd_rn(c, red[4 * (32 * g + (tid >> 2)) + (tid & 3)]);
      s_partial[(int64_t)blockIdx.x * kBwF + tid] = c;
    }
  }
  if constexpr (DX && EPI != EPI_STORE) {
    // fold the four row groups of each column in fixed order
    const float a = __fadd_rn(csum, __shfl_xor(csum, 16, 64));
    const float b = __fadd_rn(a, __shfl_xor(a, 32, 64));
    if (lane < 16) colsum_partial[(int64_t)blockIdx.x * kBwF + ncol] = b;
  }
}

template <int EPI, bool DX, bool HCS = false>
int launch_bwd(int grid, const float *X, int64_t ldx, const float *dH, int64_t lddh,
               const float *W, int64_t ldw, int64_t M, float *dX, int64_t lddx,
               const uint32_t *mask, const float *rd, float *dwp, float *csp, hipStream_t s) {
  hipLaunchKernelGGL((gemm_bwd_kernel<EPI, DX, HCS>), dim3(grid), dim3(kBwThreads), 0, s, X, ldx, dH,
                     lddh, W, ldw, M, dX, lddx, mask, rd, dwp, csp);
  return check_launch("gemm_bwd_kernel");
}

// ----------------------------------------------------------------------------
}  // namespace
}  // namespace mgcn

extern "C" int mgcn_gemm_bwd_supported(int32_t F_in, int32_t F_out) {
  return F_in == kBwF && F_out == kBwF && g_gemm_precision == PREC_BF16X6;
}

extern "C" size_t mgcn_gemm_bwd_workspace_bytes(int64_t M, int32_t F_in, int32_t F_out) {
  (void)M;
  return align_up((size_t)kBwGrid * (size_t)F_in * (size_t)F_out * 4, 256) +
         align_up((size_t)kBwGrid * (size_t)F_in * 4, 256);
}

extern "C" int mgcn_gemm_bwd(int64_t M, int32_t F_in, int32_t F_out, const float *X, int64_t ldx,
                             const float *dH, int64_t lddh, const float *W, int64_t ldw,
                             float *dW, int64_t lddw, int accumulate, float *dX, int64_t lddx,
                             const uint32_t *relu_mask, const float *row_div, float *colsum,
                             void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(M >= 0, "mgcn_gemm_bwd: negative size");
  MGCN_REQUIRE(mgcn_gemm_bwd_supported(F_in, F_out),
               "mgcn_gemm_bwd: unsupported F_in=%d F_out=%d (needs 128 x 128, bf16x6)", F_in, F_out);
  MGCN_REQUIRE(dW != nullptr && lddw >= F_out, "mgcn_gemm_bwd: bad dW");
  const int epi = relu_mask == nullptr ? EPI_STORE : row_div != nullptr ? EPI_RELU_DIV : EPI_RELU;
  MGCN_REQUIRE(epi == EPI_STORE || (dX != nullptr && colsum != nullptr),
               "mgcn_gemm_bwd: relu_mask needs dX and colsum");
  MGCN_REQUIRE(row_div == nullptr || relu_mask != nullptr, "mgcn_gemm_bwd: row_div needs relu_mask");
  hipStream_t s = as_stream(stream);
  // dW only with colsum: colsum = the column sums of dH (F_out entries)
  const bool hcs = dX == nullptr && colsum != nullptr;
  if (M == 0) {
    if (!accumulate)
      for (int32_t r = 0; r < F_in; ++r)
        MGCN_HIP_TRY(hipMemsetAsync(dW + r * lddw, 0, sizeof(float) * F_out, s));
    if (colsum) MGCN_HIP_TRY(hipMemsetAsync(colsum, 0, sizeof(float) * (hcs ? F_out : F_in), s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(X && dH && ldx >= F_in && lddh >= F_out && ldx % 4 == 0 && lddh % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(X) % 16 == 0 && reinterpret_cast<uintptr_t>(dH) % 16 == 0,
               "mgcn_gemm_bwd: X/dH must be 16-byte aligned rows");
  MGCN_REQUIRE(dX == nullptr || (W != nullptr && ldw >= F_out && lddx >= F_in),
               "mgcn_gemm_bwd: bad W/dX");
  const size_t need = mgcn_gemm_bwd_workspace_bytes(M, F_in, F_out);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_gemm_bwd: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  float *dwp = static_cast<float *>(workspace);
  float *csp = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                         align_up((size_t)kBwGrid * F_in * F_out * 4, 256));
  const int64_t n_chunks = (M + kBwRows - 1) / kBwRows;
  const int grid = (int)(n_chunks < kBwGrid ? n_chunks : kBwGrid);
  int rc;
  const int fold_grid = grid;
  if (dX == nullptr && hcs)
    rc = launch_bwd<EPI_STORE, false, true>(grid, X, ldx, dH, lddh, W, ldw, M, dX, lddx,
                                            relu_mask, row_div, dwp, csp, s);
  else if (dX == nullptr)
    rc = launch_bwd<EPI_STORE, false>(grid, X, ldx, dH, lddh, W, ldw, M, dX, lddx, relu_mask,
                                      row_div, dwp, csp, s);
  else if (epi == EPI_RELU_DIV)
    rc = launch_bwd<EPI_RELU_DIV, true>(grid, X, ldx, dH, lddh, W, ldw, M, dX, lddx, relu_mask,
                                        row_div, dwp, csp, s);
  else if (epi == EPI_RELU)
    rc = launch_bwd<EPI_RELU, true>(grid, X, ldx, dH, lddh, W, ldw, M, dX, lddx, relu_mask,
                                    row_div, dwp, csp, s);
  else
    rc = launch_bwd<EPI_STORE, true>(grid, X, ldx, dH, lddh, W, ldw, M, dX, lddx, relu_mask,
                                     row_div, dwp, csp, s);
  if (rc) return rc;
  const int64_t MN = (int64_t)F_in * F_out;
  if (int rc2 = launch_fold(dwp, fold_grid, MN, F_out, dW, lddw, accumulate, s)) return rc2;
  if (hcs) return launch_colsum_fold(csp, fold_grid, F_out, colsum, s);
  if (epi == EPI_STORE) return MGCN_OK;
  return launch_colsum_fold(csp, grid, F_in, colsum, s);
}

extern "C" size_t mgcn_gemm_bwd_dw_cs_workspace_bytes(int64_t M) {
  return mgcn_gemm_bwd_workspace_bytes(M, kBwF, kBwF) + align_up((size_t)kBwGrid * kBwF * 4, 256);
}

extern "C" int mgcn_gemm_bwd_dw_cs(int64_t M, const float *X, int64_t ldx, const float *dH,
                                   int64_t lddh, float *dW, int64_t lddw, int accumulate,
                                   float *colsum, const float *S, int64_t lds, float *s_colsum,
                                   void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(M >= 0, "mgcn_gemm_bwd_dw_cs: negative size");
  MGCN_REQUIRE(g_gemm_precision == PREC_BF16X6, "mgcn_gemm_bwd_dw_cs: needs the bf16x6 products");
  MGCN_REQUIRE(dW != nullptr && lddw >= kBwF && s_colsum != nullptr,
               "mgcn_gemm_bwd_dw_cs: bad dW / s_colsum");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    if (!accumulate)
      for (int32_t r = 0; r < kBwF; ++r)
        MGCN_HIP_TRY(hipMemsetAsync(dW + r * lddw, 0, sizeof(float) * kBwF, s));
    if (colsum) MGCN_HIP_TRY(hipMemsetAsync(colsum, 0, sizeof(float) * kBwF, s));
    MGCN_HIP_TRY(hipMemsetAsync(s_colsum, 0, sizeof(float) * kBwF, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(X && dH && S && ldx >= kBwF && lddh >= kBwF && lds >= kBwF && ldx % 4 == 0 &&
                   lddh % 4 == 0 && lds % 4 == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(dH) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(S) % 16 == 0,
               "mgcn_gemm_bwd_dw_cs: X / dH / S must be 16-byte aligned rows");
  const size_t need = mgcn_gemm_bwd_dw_cs_workspace_bytes(M);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_gemm_bwd_dw_cs: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  float *dwp = static_cast<float *>(workspace);
  float *csp = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                         align_up((size_t)kBwGrid * kBwF * kBwF * 4, 256));
  float *ssp = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                         mgcn_gemm_bwd_workspace_bytes(M, kBwF, kBwF));
  const int64_t n_chunks = (M + kBwRows - 1) / kBwRows;
  const int grid = (int)(n_chunks < kBwGrid ? n_chunks : kBwGrid);
  if (colsum)
    hipLaunchKernelGGL((gemm_bwd_kernel<EPI_STORE, false, true, true>), dim3(grid),
                       dim3(kBwThreads), 0, s, X, ldx, dH, lddh, nullptr, 0, M, nullptr, 0,
                       nullptr, nullptr, dwp, csp, S, lds, ssp);
  else
    hipLaunchKernelGGL((gemm_bwd_kernel<EPI_STORE, false, false, true>), dim3(grid),
                       dim3(kBwThreads), 0, s, X, ldx, dH, lddh, nullptr, 0, M, nullptr, 0,
                       nullptr, nullptr, dwp, csp, S, lds, ssp);
  if (int rc = check_launch("gemm_bwd_kernel")) return rc;
  if (int rc = launch_fold(dwp, grid, (int64_t)kBwF * kBwF, kBwF, dW, lddw, accumulate, s)) return rc;
  if (colsum)
    if (int rc = launch_colsum_fold(csp, grid, kBwF, colsum, s)) return rc;
  return launch_colsum_fold(ssp, grid, kBwF, s_colsum, s);
}

namespace mgcn {
// The staged kernel takes C = A^T B when M = 32, N = 32 / 64, rows 16-byte
// aligned and a split's byte offsets within 32 bits: at most gemm_splits
// (the workspace's count, K >= 64 rows each) workgroups of >= 256 rows.
bool tn_staged_plan(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda, const float *B,
                    int64_t ldb, void *workspace, size_t workspace_bytes, TnJob *job) {
  if (!g_tn_staged || K <= 0 || M != 32 || (N != 32 && N != 64) ||
      reinterpret_cast<uintptr_t>(A) % 16 || reinterpret_cast<uintptr_t>(B) % 16 || lda % 4 ||
      ldb % 4 || workspace == nullptr ||
      workspace_bytes < mgcn_gemm_tn_workspace_bytes(K, M, N))
    return false;
  const int splits = gemm_splits(K, M, N);
  int64_t s2 = (K + 255) / 256;
  if (s2 > 512) s2 = 512;
  if (s2 > splits) s2 = splits;
  int64_t kps2 = (K + s2 - 1) / s2;
  kps2 = (kps2 + 63) / 64 * 64;
  if ((kps2 + 64) * (lda > ldb ? lda : ldb) * 4 >= (int64_t(1) << 31)) return false;
  *job = TnJob{A, lda, B, ldb, K, kps2, static_cast<float *>(workspace),
               (int)((K + kps2 - 1) / kps2)};
  return true;
}
}  // namespace mgcn
