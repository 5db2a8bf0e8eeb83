// Zero-skipping row packing for the sharded path's table exchange
// (mgcn.dist): the tables the ranks all-gather between
// layers are ReLU outputs (forward) or gradients masked by the same ReLU
// (backward), about half exact zeros.  A chunk of rows travels as
//
//   [offs: n int32][masks: n x F/32 uint32][vals: the nonzero words, row-major]
//
// bit b of mask word w of a row <=> word 32 w + b of the row is not +0.0 (a
// BIT-PATTERN test: -0.0, NaN and denormals travel as values, so unpacking
// restores every row bit for bit); offs[i] = the index in vals of row i's
// first value (exclusive prefix sum of the rows' popcounts).
//
// Kernels (one wave per row, 64 words per step; F % 32 == 0):
//   pack_count   row -> mask words (into the send buffer) + popcount
//   pack_values  row + mask + offs -> its nonzero words at vals + offs[i]
//   unpack       for every received segment p and row i: mask + offs + vals
//                -> the dense row at T[(p n + i) ldt]
// HBM-bound: pack reads the chunk once per kernel (4 F bytes per row) and
// writes 4 (1 + F/32) + 4 nnz; unpack reads the segment and writes 4 F.

#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kPkWaves = 4;

__global__ __launch_bounds__(64 * kPkWaves) void pack_count_kernel(int64_t n, int F,
                                                                   const float *__restrict__ X,
                                                                   int64_t ldx,
                                                                   uint32_t *__restrict__ masks,
                                                                   int32_t *__restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * kPkWaves;
  const int words = F >> 5;
  for (int64_t r = (int64_t)blockIdx.x * kPkWaves + (threadIdx.x >> 6); r < n; r += stride) {
    const uint32_t *x = reinterpret_cast<const uint32_t *>(X + r * ldx);
    int cnt = 0;
    for (int f0 = 0; f0 < F; f0 += 64) {
      const int f = f0 + lane;
      const bool nz = f < F && x[f] != 0u;
      const uint64_t b = __ballot(nz);
      cnt += __popcll(b);
      const int w = f0 >> 5;
      if (lane == 0) masks[r * words + w] = (uint32_t)b;
      if (lane == 1 && w + 1 < words) masks[r * words + w + 1] = (uint32_t)(b >> 32);
    }
    if (lane == 0) counts[r] = cnt;
  }
}

__global__ __launch_bounds__(64 * kPkWaves) void pack_values_kernel(
    int64_t n, int F, const float *__restrict__ X, int64_t ldx,
    const uint32_t *__restrict__ masks, const int32_t *__restrict__ offs,
    uint32_t *__restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * kPkWaves;
  const int words = F >> 5;
  for (int64_t r = (int64_t)blockIdx.x * kPkWaves + (threadIdx.x >> 6); r < n; r += stride) {
    const uint32_t *x = reinterpret_cast<const uint32_t *>(X + r * ldx);
    int64_t pos = offs[r];
    for (int f0 = 0; f0 < F; f0 += 64) {
      const int f = f0 + lane;
      const uint32_t v = f < F ? x[f] : 0u;
      const int w = f0 >> 5;
      const uint64_t m = (uint64_t)masks[r * words + w] |
                         (w + 1 < words ? (uint64_t)masks[r * words + w + 1] << 32 : 0ull);
      const bool nz = (m >> lane) & 1ull;
      // lanes below this one holding a value
      const int below = __popcll(m & ((1ull << lane) - 1ull));
      if (nz) vals[pos + below] = v;
      pos += __popcll(m);
    }
  }
}

__global__ __launch_bounds__(64 * kPkWaves) void unpack_kernel(int64_t n_seg, int64_t n, int F,
                                                               const uint32_t *__restrict__ buf,
                                                               int64_t seg_words,
                                                               float *__restrict__ T,
                                                               int64_t ldt) {
  const int lane = threadIdx.x & 63;
  const int64_t total = n_seg * n;
  const int64_t stride = (int64_t)gridDim.x * kPkWaves;
  const int words = F >> 5;
  for (int64_t k = (int64_t)blockIdx.x * kPkWaves + (threadIdx.x >> 6); k < total; k += stride) {
    const int64_t p = k / n, i = k - p * n;
    const uint32_t *seg = buf + p * seg_words;
    const int32_t *offs = reinterpret_cast<const int32_t *>(seg);
    const uint32_t *mk = seg + n + i * words;
    const uint32_t *vals = seg + n + n * words;
    int64_t pos = offs[i];
    uint32_t *t = reinterpret_cast<uint32_t *>(T + k * ldt);
    for (int f0 = 0; f0 < F; f0 += 64) {
      const int f = f0 + lane;
      const int w = f0 >> 5;
      const uint64_t m = (uint64_t)mk[w] | (w + 1 < words ? (uint64_t)mk[w + 1] << 32 : 0ull);
      const bool nz = (m >> lane) & 1ull;
      const int below = __popcll(m & ((1ull << lane) - 1ull));
      const uint32_t v = nz ? vals[pos + below] : 0u;
      if (f < F) t[f] = v;
      pos += __popcll(m);
    }
  }
}

unsigned pk_grid(int64_t rows) { return grid_for((rows + kPkWaves - 1) / kPkWaves, 1); }

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" int mgcn_pack_rows_count(int64_t n, int32_t F, const float *X, int64_t ldx,
                                    uint32_t *masks, int32_t *counts, void *stream) {
  clear_error();
  MGCN_REQUIRE(n >= 0 && F > 0 && F % 32 == 0 && ldx >= F,
               "mgcn_pack_rows_count: need n >= 0, F a multiple of 32, ldx >= F");
  if (n == 0) return MGCN_OK;
  MGCN_REQUIRE(X && masks && counts, "mgcn_pack_rows_count: null array");
  hipLaunchKernelGGL(pack_count_kernel, dim3(pk_grid(n)), dim3(64 * kPkWaves), 0,
                     as_stream(stream), n, (int)F, X, ldx, masks, counts);
  return check_launch("pack_count_kernel");
}

extern "C" int mgcn_pack_rows_values(int64_t n, int32_t F, const float *X, int64_t ldx,
                                     const uint32_t *masks, const int32_t *offs, uint32_t *vals,
                                     void *stream) {
  clear_error();
  MGCN_REQUIRE(n >= 0 && F > 0 && F % 32 == 0 && ldx >= F,
               "mgcn_pack_rows_values: need n >= 0, F a multiple of 32, ldx >= F");
  if (n == 0) return MGCN_OK;
  MGCN_REQUIRE(X && masks && offs && vals, "mgcn_pack_rows_values: null array");
  hipLaunchKernelGGL(pack_values_kernel, dim3(pk_grid(n)), dim3(64 * kPkWaves), 0,
                     as_stream(stream), n, (int)F, X, ldx, masks, offs, vals);
  return check_launch("pack_values_kernel");
}

extern "C" int mgcn_unpack_rows(int64_t n_seg, int64_t n, int32_t F, const uint32_t *buf,
                                int64_t seg_words, float *T, int64_t ldt, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_seg >= 0 && n >= 0 && F > 0 && F % 32 == 0 && ldt >= F,
               "mgcn_unpack_rows: need n_seg, n >= 0, F a multiple of 32, ldt >= F");
  if (n_seg == 0 || n == 0) return MGCN_OK;
  MGCN_REQUIRE(buf && T, "mgcn_unpack_rows: null array");
  MGCN_REQUIRE(seg_words >= n * (1 + F / 32), "mgcn_unpack_rows: segment of %lld words < header",
               (long long)seg_words);
  hipLaunchKernelGGL(unpack_kernel, dim3(pk_grid(n_seg * n)), dim3(64 * kPkWaves), 0,
                     as_stream(stream), n_seg, n, (int)F, buf, seg_words, T, ldt);
  return check_launch("unpack_kernel");
}
