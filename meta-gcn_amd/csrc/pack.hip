// Zero-skipping row packing for the sharded path's table exchange
// (mgcn.dist): the tables the ranks all-gather between
// layers are ReLU outputs (forward) or gradients masked by the same ReLU
// (backward), about half exact zeros.  A chunk of n rows travels as
//
//   [hdr: n x W pairs (mask_w, pos_w) uint32][vals: the nonzero words, row-major]
//
// with W = F / 32.  Bit b of mask_w of a row <=> word 32 w + b of the row is
// not +0.0 (a BIT-PATTERN test: -0.0, NaN and denormals travel as values, so
// every row comes back bit for bit); pos_w = the index in vals of the row's
// first value at or after word 32 w (the row's offset -- exclusive prefix sum
// of the rows' popcounts -- plus the popcounts of its words below w).  The
// pairs make the packed rows GATHERABLE in place (round 6): the lane that
// holds words 4 j .. 4 j + 3 of a row reads one 8-B pair (w = j / 8) and
// finds its values at pos_w + popc(mask_w below bit 4 (j % 8)) -- no scan over
// the row (fused_wide.hip, spmm_xw_wide_ws_kernel<.., PK>).
//
// Layout of the work: a row is cut into segments of 256 words; a group of
// G = min(64, F/4) lanes (a power of two) takes one segment, lane gl words
// 4 gl .. 4 gl + 3 as one 16-B access, so a wave moves 1 KB per instruction
// (G = 32 at F = 128: two rows per wave).  Four ballots give the group's
// nonzero bits by word position j; a value's place in the packed row is the
// values of the lanes below it (popcounts of the ballots under a lane mask)
// plus those of its own lane's lower words.  Mask word w of a segment is
// lanes 8 w .. 8 w + 7's nibbles, interleaved out of the four ballots.
// HBM-bound: pack reads the chunk once per kernel (4 F bytes per row) and
// writes F/4 (+ 4 nnz); unpack reads F/4 + 4 nnz and writes 4 F.

#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kPkWaves = 4;
typedef unsigned int wl_u32x4 __attribute__((ext_vector_type(4)));

// word w (w < G / 8) of a segment from the group's four ballots (bit gl of
// b[j] <=> word 4 gl + j is nonzero): bit 4 i + j <- bit 8 w + i of b[j]
__device__ __forceinline__ uint32_t seg_word(const uint64_t (&b)[4], int w) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t byte = (uint32_t)(b[j] >> (8 * w)) & 0xffu;
    // spread the 8 bits of `byte` to positions 0, 4, 8, ..., 28
    uint32_t x = byte;
    x = (x | (x << 12)) & 0x000f000fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    r |= x << j;
  }
  return r;
}

template <int G>
struct PkLane {
  int gl, grp;
  uint64_t gmask;  // the group's lanes
  uint64_t below;  // the group's lanes below this one
};

template <int G>
__device__ __forceinline__ PkLane<G> pk_lane() {
  PkLane<G> p;
  const int lane = threadIdx.x & 63;
  p.gl = lane & (G - 1);
  p.grp = lane / G;
  const uint64_t g = G == 64 ? ~0ull : ((1ull << G) - 1ull);
  p.gmask = g << (p.grp * G);
  p.below = ((1ull << lane) - 1ull) & p.gmask;
  return p;
}

// one 256-word segment of a row: nonzero bits of this lane's four words and
// the group's ballots
template <int G>
__device__ __forceinline__ void seg_bits(const PkLane<G> &p, bool ok, const uint4 &v, bool (&nz)[4],
                                         uint64_t (&b)[4]) {
  nz[0] = ok && v.x != 0u;
  nz[1] = ok && v.y != 0u;
  nz[2] = ok && v.z != 0u;
  nz[3] = ok && v.w != 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = (__ballot(nz[j]) & p.gmask) >> (p.grp * G);
}

template <int G>
__global__ __launch_bounds__(64 * kPkWaves) void pack_count_kernel(int64_t n, int F,
                                                                   const float *__restrict__ X,
                                                                   int64_t ldx,
                                                                   uint32_t *__restrict__ hdr,
                                                                   int32_t *__restrict__ counts) {
  const PkLane<G> p = pk_lane<G>();
  constexpr int RPW = 64 / G;  // rows per wave
  const int64_t stride = (int64_t)gridDim.x * kPkWaves * RPW;
  const int words = F >> 5;
  for (int64_t r = ((int64_t)blockIdx.x * kPkWaves + (threadIdx.x >> 6)) * RPW + p.grp; r < n + p.grp;
       r += stride) {
    // (r < n) is not group-uniform across the wave: every lane runs the loop
    // the same number of times and masks its loads
    const bool rok = r < n;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(X + (rok ? r : 0) * ldx);
    int cnt = 0;
    for (int f0 = 0; f0 < F; f0 += 4 * G) {
      const int f = f0 + 4 * p.gl;
      const bool ok = rok && f < F;
      const uint4 v = ok ? *reinterpret_cast<const uint4 *>(x + f) : make_uint4(0u, 0u, 0u, 0u);
      bool nz[4];
      uint64_t b[4];
      seg_bits<G>(p, ok, v, nz, b);
      cnt += __popcll(b[0]) + __popcll(b[1]) + __popcll(b[2]) + __popcll(b[3]);
      const int w0 = f0 >> 5;
      if (rok && p.gl < G / 8 && w0 + p.gl < words) hdr[2 * (r * words + w0 + p.gl)] = seg_word(b, p.gl);
    }
    if (rok && p.gl == 0) counts[r] = cnt;
  }
}

template <int G>
__global__ __launch_bounds__(64 * kPkWaves) void pack_values_kernel(
    int64_t n, int F, const float *__restrict__ X, int64_t ldx, const int32_t *__restrict__ offs,
    uint32_t *__restrict__ hdr, uint32_t *__restrict__ vals) {
  const PkLane<G> p = pk_lane<G>();
  constexpr int RPW = 64 / G;
  const int64_t stride = (int64_t)gridDim.x * kPkWaves * RPW;
  const int words = F >> 5;
  for (int64_t r = ((int64_t)blockIdx.x * kPkWaves + (threadIdx.x >> 6)) * RPW + p.grp; r < n + p.grp;
       r += stride) {
    const bool rok = r < n;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(X + (rok ? r : 0) * ldx);
    int64_t pos = rok ? offs[r] : 0;
    for (int f0 = 0; f0 < F; f0 += 4 * G) {
      const int f = f0 + 4 * p.gl;
      const bool ok = rok && f < F;
      const uint4 v = ok ? *reinterpret_cast<const uint4 *>(x + f) : make_uint4(0u, 0u, 0u, 0u);
      bool nz[4];
      uint64_t b[4];
      seg_bits<G>(p, ok, v, nz, b);
      const uint64_t lo = p.below >> (p.grp * G);
      int64_t q = pos + __popcll(b[0] & lo) + __popcll(b[1] & lo) + __popcll(b[2] & lo) +
                  __popcll(b[3] & lo);
      // the first lane of each mask word's 8 writes the word's value position
      if (ok && (p.gl & 7) == 0) hdr[2 * (r * words + (f >> 5)) + 1] = (uint32_t)q;
      if (nz[0]) vals[q++] = v.x;
      if (nz[1]) vals[q++] = v.y;
      if (nz[2]) vals[q++] = v.z;
      if (nz[3]) vals[q++] = v.w;
      pos += __popcll(b[0]) + __popcll(b[1]) + __popcll(b[2]) + __popcll(b[3]);
    }
  }
}

// Unpack, software-pipelined one row ahead (round 5): a row costs two
// dependent round trips (its offset and mask word, then its values); the next
// row's offset and first mask word are loaded while this row's values are in
// flight, so a wave's rows cost about one round trip each (4.0 TB/s before).
template <int G>
__global__ __launch_bounds__(64 * kPkWaves) void unpack_kernel(int64_t n_seg, int64_t n, int F,
                                                               const uint32_t *__restrict__ buf,
                                                               int64_t seg_words,
                                                               float *__restrict__ T,
                                                               int64_t ldt) {
  const PkLane<G> p = pk_lane<G>();
  constexpr int RPW = 64 / G;
  const int64_t total = n_seg * n;
  const int64_t stride = (int64_t)gridDim.x * kPkWaves * RPW;
  const int words = F >> 5;
  const uint64_t lo = p.below >> (p.grp * G);
  // header of row kk: its value offset and this lane's nibble of segment 0
  auto header = [&](int64_t kk, int64_t &pos, uint32_t &nib) {
    const bool rok = kk < total;
    const int64_t sg = rok ? kk / n : 0, i = rok ? kk - sg * n : 0;
    const uint32_t *seg = buf + sg * seg_words;
    const int f = 4 * p.gl;
    pos = rok ? (int64_t)seg[2 * i * words + 1] : 0;  // pos_0: the row's offset
    nib = (rok && f < F) ? (seg[2 * (i * words + (f >> 5))] >> (f & 31)) & 0xfu : 0u;
  };
  int64_t k = ((int64_t)blockIdx.x * kPkWaves + (threadIdx.x >> 6)) * RPW + p.grp;
  int64_t pos_n;
  uint32_t nib_n;
  header(k, pos_n, nib_n);
  for (; k < total + p.grp; k += stride) {
    const bool rok = k < total;
    int64_t pos = pos_n;
    uint32_t nib0 = nib_n;
    header(k + stride, pos_n, nib_n);  // the next row's header, under this row's values
    const int64_t sg = rok ? k / n : 0, i = rok ? k - sg * n : 0;
    const uint32_t *seg = buf + sg * seg_words;
    const uint32_t *hd = seg + 2 * i * words;
    const uint32_t *vals = seg + 2 * n * words;
    uint32_t *t = reinterpret_cast<uint32_t *>(T + (rok ? k : 0) * ldt);
    for (int f0 = 0; f0 < F; f0 += 4 * G) {
      const int f = f0 + 4 * p.gl;
      const bool ok = rok && f < F;
      // this lane's nibble of its mask word: word f >> 5, bits (f & 31) .. + 3
      const uint32_t nib = f0 == 0 ? nib0 : ok ? (hd[2 * (f >> 5)] >> (f & 31)) & 0xfu : 0u;
      bool nz[4] = {(nib & 1u) != 0, (nib & 2u) != 0, (nib & 4u) != 0, (nib & 8u) != 0};
      uint64_t b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (__ballot(nz[j]) & p.gmask) >> (p.grp * G);
      const int64_t q = pos + __popcll(b[0] & lo) + __popcll(b[1] & lo) + __popcll(b[2] & lo) +
                        __popcll(b[3] & lo);
      // the four value loads issued together (a lane's values are consecutive)
      const int64_t q1 = q + (nz[0] ? 1 : 0);
      const int64_t q2 = q1 + (nz[1] ? 1 : 0);
      const int64_t q3 = q2 + (nz[2] ? 1 : 0);
      // (a zero word reads the segment's first header word: always in bounds)
      const uint32_t x0 = *(nz[0] ? vals + q : seg), x1 = *(nz[1] ? vals + q1 : seg);
      const uint32_t x2 = *(nz[2] ? vals + q2 : seg), x3 = *(nz[3] ? vals + q3 : seg);
      const uint4 v = make_uint4(nz[0] ? x0 : 0u, nz[1] ? x1 : 0u, nz[2] ? x2 : 0u, nz[3] ? x3 : 0u);
      if (ok) *reinterpret_cast<uint4 *>(t + f) = v;
      pos += __popcll(b[0]) + __popcll(b[1]) + __popcll(b[2]) + __popcll(b[3]);
    }
  }
}

// Single-pass pack (round 6): counts, offsets and values in ONE read of the
// chunk.  A workgroup takes a tile of rows -- a ticket (atomicAdd) orders the
// tiles by start, so every tile's predecessors are resident or done -- and
// holds them in registers (kPrIters 16-B loads per lane); it publishes its
// nonzero count, looks back over its predecessors' published counts for its
// offset (decoupled look-back: a predecessor's aggregate, or its inclusive
// prefix, which ends the walk), publishes its own inclusive prefix and writes
// the header pairs and values from the registers.  The two-pass form reads
// every row twice (count, then values) and scans the counts between them.
// Values leave through a 1-KB LDS row per wave: an iteration's values are one
// contiguous run, stored by consecutive lanes (0.69 vs 0.81 ms for a config-5
// chunk with each lane storing its own words; 8 / 24 / 32 iterations per
// lane: 0.77 (with staging) / 0.73 / 0.70 -- scripts/bench_pack.py,
// profiles/r06/pack_one_pass.json).  The rows are read with the nt policy
// (read once: 0.669 vs 0.691 ms).  Against the two passes: 0.67 vs 1.07 ms.
// Rows of one 256-word segment only (F = 4 G: 32, 64, 128, 256).
// Status word of a tile: (flag << 62) | value, flag 1 = aggregate, 2 =
// inclusive prefix; 0 = not yet published.  Relaxed agent-scope atomics: the
// word carries its own data.  A walk that waits past the spin bound stores
// kDevErrPack and takes 0 for the missing part (every wave still finishes;
// the offsets then only come out too SMALL, so every store stays inside the
// chunk's buffers).
#ifndef MGCN_PR_NTLOAD
#define MGCN_PR_NTLOAD 1
#endif
#ifndef MGCN_PR_LDS
#define MGCN_PR_LDS 1
#endif
#ifndef MGCN_PR_ITERS
#define MGCN_PR_ITERS 16
#endif
constexpr int kPrIters = MGCN_PR_ITERS;
constexpr uint64_t kPrAgg = 1ull << 62, kPrInc = 2ull << 62, kPrVal = (1ull << 62) - 1;

template <int G>
constexpr int pr_tile_rows() { return kPrIters * (64 / G) * kPkWaves; }

template <int G>
__global__ __launch_bounds__(64 * kPkWaves) void pack_rows_kernel(
    int64_t n, const float *__restrict__ X, int64_t ldx, uint32_t *__restrict__ hdr,
    uint32_t *__restrict__ vals, int64_t *__restrict__ total, uint64_t *__restrict__ status,
    unsigned *__restrict__ ticket, int64_t n_tiles, uint32_t spin_limit, unsigned *err) {
  const PkLane<G> p = pk_lane<G>();
  constexpr int RPW = 64 / G;
  constexpr int RW = kPrIters * RPW;  // rows per wave
  constexpr int RT = RW * kPkWaves;   // rows per tile
  constexpr int WORDS = G / 8;        // mask words per row (F = 4 G)
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  __shared__ int64_t s_tile, s_prefix;
  __shared__ int64_t s_wsum[kPkWaves];
#if MGCN_PR_LDS
  __shared__ uint32_t s_stage[kPkWaves][256];
#endif
  if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t r0 = tile * RT + (int64_t)wave * RW + p.grp;

  // the tile's rows into registers; per row, this lane's row offset in the wave
  uint4 v[kPrIters];
#pragma unroll
  for (int i = 0; i < kPrIters; ++i) {
    const int64_t r = r0 + (int64_t)i * RPW;
#if MGCN_PR_NTLOAD
    if (r < n) {
      const wl_u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const wl_u32x4 *>(X + r * ldx + 4 * p.gl));
      v[i] = make_uint4(t.x, t.y, t.z, t.w);
    } else {
      v[i] = make_uint4(0u, 0u, 0u, 0u);
    }
#else
    v[i] = r < n ? *reinterpret_cast<const uint4 *>(X + r * ldx + 4 * p.gl)
                 : make_uint4(0u, 0u, 0u, 0u);
#endif
  }
  const uint64_t groups_below = (1ull << (p.grp * G)) - 1ull;  // lanes of the lower groups
  int64_t wsum = 0;  // wave-uniform: values of the wave's rows so far
  int32_t roff[kPrIters];
#pragma unroll
  for (int i = 0; i < kPrIters; ++i) {
    const uint64_t b0 = __ballot(v[i].x != 0u), b1 = __ballot(v[i].y != 0u);
    const uint64_t b2 = __ballot(v[i].z != 0u), b3 = __ballot(v[i].w != 0u);
    roff[i] = (int32_t)(wsum + __popcll(b0 & groups_below) + __popcll(b1 & groups_below) +
                        __popcll(b2 & groups_below) + __popcll(b3 & groups_below));
    wsum += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
  }
  if (lane == 0) s_wsum[wave] = wsum;
  __syncthreads();
  int64_t agg = 0, woff = 0;
#pragma unroll
  for (int w = 0; w < kPkWaves; ++w) {
    woff += w < wave ? s_wsum[w] : 0;
    agg += s_wsum[w];
  }

  if (wave == 0) {
    int64_t excl = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(status, kPrInc | (uint64_t)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(status + tile, kPrAgg | (uint64_t)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t look = tile - 1;
      uint32_t spins = 0;
      for (;;) {
        // lane l reads tile look - l (before tile 0: an inclusive 0)
        const int64_t q = look - lane;
        const uint64_t st = q >= 0 ? __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : kPrInc;
        const uint64_t inc = __ballot((st >> 62) == 2u);
        const uint64_t none = __ballot((st >> 62) == 0u);
        const int first = inc != 0 ? __builtin_ctzll(inc) : 64;  // nearest inclusive prefix
        const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
        if (none & need) {  // a tile on the way has not published yet
          if (++spins > spin_limit) {
            report_device_error(err, kDevErrPack);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        int64_t part = lane <= first ? (int64_t)(st & kPrVal) : 0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off, 64);
        excl += part;
        if (first < 64) break;
        look -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(status + tile, kPrInc | (uint64_t)(excl + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_prefix = excl;
      if (tile == n_tiles - 1) *total = excl + agg;
    }
  }
  __syncthreads();

  // header pairs and values from the registers
  const int64_t base = s_prefix + woff;
  const uint64_t lo = p.below >> (p.grp * G);
#pragma unroll
  for (int i = 0; i < kPrIters; ++i) {
    const int64_t r = r0 + (int64_t)i * RPW;
    const bool ok = r < n;
    bool nz[4];
    uint64_t b[4];
    seg_bits<G>(p, ok, v[i], nz, b);
    const int64_t rowpos = base + roff[i];
    if (ok && p.gl < WORDS) {
      const uint64_t under = (1ull << (8 * p.gl)) - 1ull;  // the lanes of words below gl
      const int64_t pw = rowpos + __popcll(b[0] & under) + __popcll(b[1] & under) +
                         __popcll(b[2] & under) + __popcll(b[3] & under);
      *reinterpret_cast<uint2 *>(hdr + 2 * (r * WORDS + p.gl)) = make_uint2(seg_word(b, p.gl), (uint32_t)pw);
    }
    int64_t q = rowpos + __popcll(b[0] & lo) + __popcll(b[1] & lo) + __popcll(b[2] & lo) + __popcll(b[3] & lo);
#if MGCN_PR_LDS
    // the iteration's values are one contiguous run [ib, ib + ic): staged in
    // the wave's LDS row, then stored by consecutive lanes (a wave's LDS
    // operations execute in order: no barrier between the writes and reads)
    const int64_t ib = base + __builtin_amdgcn_readfirstlane(roff[i]);
    const int ic = __popcll(__ballot(nz[0])) + __popcll(__ballot(nz[1])) + __popcll(__ballot(nz[2])) +
                   __popcll(__ballot(nz[3]));
    uint32_t *st = s_stage[wave];
    int l = (int)(q - ib);
    if (nz[0]) st[l++] = v[i].x;
    if (nz[1]) st[l++] = v[i].y;
    if (nz[2]) st[l++] = v[i].z;
    if (nz[3]) st[l++] = v[i].w;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lane + 64 * k < ic) vals[ib + lane + 64 * k] = st[lane + 64 * k];
    __builtin_amdgcn_wave_barrier();
#else
    if (nz[0]) vals[q++] = v[i].x;
    if (nz[1]) vals[q++] = v[i].y;
    if (nz[2]) vals[q++] = v[i].z;
    if (nz[3]) vals[q++] = v[i].w;
#endif
  }
}

int pk_group(int F) { return F >= 256 ? 64 : F >= 128 ? 32 : F >= 64 ? 16 : 8; }

unsigned pk_grid(int64_t rows, int G) {
  return grid_for((rows * G / 64 + kPkWaves - 1) / kPkWaves, 1);
}

bool pk_aligned(const void *p, int64_t ld) { return (uintptr_t)p % 16 == 0 && ld % 4 == 0; }

}  // namespace
}  // namespace mgcn

using namespace mgcn;

#define PK_DISPATCH(G, KERNEL, ...)                                                          \
  switch (G) {                                                                               \
    case 64: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                             \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                             \
    case 16: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break;                             \
    default: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                              \
  }

extern "C" int mgcn_pack_rows_count(int64_t n, int32_t F, const float *X, int64_t ldx,
                                    uint32_t *hdr, int32_t *counts, void *stream) {
  clear_error();
  MGCN_REQUIRE(n >= 0 && F > 0 && F % 32 == 0 && ldx >= F,
               "mgcn_pack_rows_count: need n >= 0, F a multiple of 32, ldx >= F");
  if (n == 0) return MGCN_OK;
  MGCN_REQUIRE(X && hdr && counts, "mgcn_pack_rows_count: null array");
  MGCN_REQUIRE(pk_aligned(X, ldx), "mgcn_pack_rows_count: rows must be 16-byte aligned");
  const int G = pk_group(F);
  PK_DISPATCH(G, pack_count_kernel, dim3(pk_grid(n, G)), dim3(64 * kPkWaves), 0,
              as_stream(stream), n, (int)F, X, ldx, hdr, counts);
  return check_launch("pack_count_kernel");
}

extern "C" int mgcn_pack_rows_values(int64_t n, int32_t F, const float *X, int64_t ldx,
                                     const int32_t *offs, uint32_t *hdr, uint32_t *vals,
                                     void *stream) {
  clear_error();
  MGCN_REQUIRE(n >= 0 && F > 0 && F % 32 == 0 && ldx >= F,
               "mgcn_pack_rows_values: need n >= 0, F a multiple of 32, ldx >= F");
  if (n == 0) return MGCN_OK;
  MGCN_REQUIRE(X && hdr && offs && vals, "mgcn_pack_rows_values: null array");
  MGCN_REQUIRE(n <= (int64_t)(UINT32_MAX / (uint32_t)F),
               "mgcn_pack_rows_values: n F must fit the header's 32-bit value positions");
  MGCN_REQUIRE(pk_aligned(X, ldx), "mgcn_pack_rows_values: rows must be 16-byte aligned");
  // the masks are recomputed from the rows (the same bits pack_count wrote)
  const int G = pk_group(F);
  PK_DISPATCH(G, pack_values_kernel, dim3(pk_grid(n, G)), dim3(64 * kPkWaves), 0,
              as_stream(stream), n, (int)F, X, ldx, offs, hdr, vals);
  return check_launch("pack_values_kernel");
}

extern "C" size_t mgcn_pack_rows_workspace_bytes(int64_t n, int32_t F) {
  if (n <= 0 || (F != 32 && F != 64 && F != 128 && F != 256)) return 0;
  const int G = pk_group(F);
  const int64_t rt = G == 64 ? pr_tile_rows<64>() : G == 32 ? pr_tile_rows<32>()
                     : G == 16 ? pr_tile_rows<16>() : pr_tile_rows<8>();
  return (size_t)(16 + 8 * ((n + rt - 1) / rt));
}

extern "C" int mgcn_pack_rows(int64_t n, int32_t F, const float *X, int64_t ldx, uint32_t *hdr,
                              uint32_t *vals, int64_t *total, void *workspace,
                              size_t workspace_bytes, void *stream) {
  clear_error();
  if (int rc = take_device_error()) return rc;  // a previous launch failed on the device
  MGCN_REQUIRE(n >= 0 && (F == 32 || F == 64 || F == 128 || F == 256) && ldx >= F,
               "mgcn_pack_rows: need n >= 0, F in {32, 64, 128, 256}, ldx >= F");
  MGCN_REQUIRE(total != nullptr, "mgcn_pack_rows: null total");
  MGCN_REQUIRE(n <= (int64_t)(UINT32_MAX / (uint32_t)F),
               "mgcn_pack_rows: n F must fit the header's 32-bit value positions");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    MGCN_HIP_TRY(hipMemsetAsync(total, 0, sizeof(int64_t), s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(X && hdr && vals && workspace, "mgcn_pack_rows: null array");
  MGCN_REQUIRE(pk_aligned(X, ldx), "mgcn_pack_rows: rows must be 16-byte aligned");
  MGCN_REQUIRE((uintptr_t)hdr % 8 == 0 && (uintptr_t)workspace % 16 == 0,
               "mgcn_pack_rows: hdr must be 8-byte and workspace 16-byte aligned");
  const size_t need = mgcn_pack_rows_workspace_bytes(n, F);
  MGCN_REQUIRE(workspace_bytes >= need, "mgcn_pack_rows: workspace of %zu bytes < %zu",
               workspace_bytes, need);
  unsigned *err = device_error_word();
  if (err == nullptr) return MGCN_EHIP;
  const int64_t n_tiles = (int64_t)(need - 16) / 8;
  MGCN_REQUIRE(n_tiles < (1ll << 31), "mgcn_pack_rows: too many rows");
  // the ticket and the tiles' status words start at 0 every launch
  MGCN_HIP_TRY(hipMemsetAsync(workspace, 0, need, s));
  unsigned *ticket = static_cast<unsigned *>(workspace);
  uint64_t *status = reinterpret_cast<uint64_t *>(static_cast<char *>(workspace) + 16);
  PK_DISPATCH(pk_group(F), pack_rows_kernel, dim3((unsigned)n_tiles), dim3(64 * kPkWaves), 0, s,
              n, X, ldx, hdr, vals, total, status, ticket, n_tiles, g_spin_limit, err);
  return check_launch("pack_rows_kernel");
}

extern "C" int mgcn_unpack_rows(int64_t n_seg, int64_t n, int32_t F, const uint32_t *buf,
                                int64_t seg_words, float *T, int64_t ldt, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_seg >= 0 && n >= 0 && F > 0 && F % 32 == 0 && ldt >= F,
               "mgcn_unpack_rows: need n_seg, n >= 0, F a multiple of 32, ldt >= F");
  if (n_seg == 0 || n == 0) return MGCN_OK;
  MGCN_REQUIRE(buf && T, "mgcn_unpack_rows: null array");
  MGCN_REQUIRE(pk_aligned(T, ldt), "mgcn_unpack_rows: T rows must be 16-byte aligned");
  MGCN_REQUIRE(seg_words >= n * 2 * (F / 32), "mgcn_unpack_rows: segment of %lld words < header",
               (long long)seg_words);
  const int G = pk_group(F);
  PK_DISPATCH(G, unpack_kernel, dim3(pk_grid(n_seg * n, G)), dim3(64 * kPkWaves), 0,
              as_stream(stream), n_seg, n, (int)F, buf, seg_words, T, ldt);
  return check_launch("unpack_kernel");
}

#if MGCN_EXPERIMENT
// Experiment build only (libmgcn_exp.so; not in mgcn.h): a stand-in for the
// HBM writes of a rank's RCCL receive, for scripts/config5_rank.py
// --recv-load-wgs.  `workgroups` 256-thread workgroups (a collective's
// footprint: RCCL runs its all-gather in a few dozen workgroups) write
// `total_bytes` of zeros with 16-B nt stores, wrapping over [buf, buf +
// buf_bytes): the received words landing in HBM while the rank computes.
// A bounded grid-stride loop (no flag, no spin).
namespace {
__global__ __launch_bounds__(256) void hbm_write_load_kernel(wl_u32x4 *__restrict__ buf, int64_t n16,
                                                             int64_t total16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const wl_u32x4 z = {0u, 0u, 0u, 0u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total16; i += stride)
    __builtin_nontemporal_store(z, buf + (i % n16));
}
}  // namespace

// the same with reads: copy [buf, buf + buf_bytes / 2) to the other half,
// wrapping -- `total_bytes` written AND read (a rank's all-gather both reads
// its own segment for every peer and receives theirs)
namespace {
__global__ __launch_bounds__(256) void hbm_copy_load_kernel(wl_u32x4 *__restrict__ buf, int64_t half16,
                                                            int64_t total16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total16; i += stride) {
    const int64_t j = i % half16;
    __builtin_nontemporal_store(__builtin_nontemporal_load(buf + j), buf + half16 + j);
  }
}
}  // namespace

extern "C" int mgcn_exp_hbm_copy_load(void *buf, int64_t buf_bytes, int64_t total_bytes,
                                      int32_t workgroups, void *stream) {
  clear_error();
  MGCN_REQUIRE(buf != nullptr && buf_bytes >= 32 && total_bytes >= 0 && workgroups > 0 &&
                   reinterpret_cast<uintptr_t>(buf) % 16 == 0,
               "mgcn_exp_hbm_copy_load: bad arguments");
  if (total_bytes == 0) return MGCN_OK;
  hipLaunchKernelGGL(hbm_copy_load_kernel, dim3((unsigned)workgroups), dim3(256), 0,
                     as_stream(stream), static_cast<wl_u32x4 *>(buf), buf_bytes / 32,
                     total_bytes / 16);
  return check_launch("hbm_copy_load_kernel");
}

extern "C" int mgcn_exp_hbm_write_load(void *buf, int64_t buf_bytes, int64_t total_bytes,
                                       int32_t workgroups, void *stream) {
  clear_error();
  MGCN_REQUIRE(buf != nullptr && buf_bytes >= 16 && total_bytes >= 0 && workgroups > 0 &&
                   reinterpret_cast<uintptr_t>(buf) % 16 == 0,
               "mgcn_exp_hbm_write_load: bad arguments");
  if (total_bytes == 0) return MGCN_OK;
  hipLaunchKernelGGL(hbm_write_load_kernel, dim3((unsigned)workgroups), dim3(256), 0,
                     as_stream(stream), static_cast<wl_u32x4 *>(buf), buf_bytes / 16,
                     total_bytes / 16);
  return check_launch("hbm_write_load_kernel");
}
#endif
