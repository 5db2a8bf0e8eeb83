// CSR row-block SpMM for GCN message passing on gfx950 (MI355X).
//
// Forward (rows = destination nodes, CSR grouped by dst, COO order kept):
//     y_i = epi( reduce_{k in row i} H[col_k, :] * w_k )
// Adjoint (rows = source nodes, CSR grouped by src):
//     dH_s = sum_{k in row s} g(dY[col_k, :]) * w_k   [* row_scale_s]
//
// What the reference does instead (jzhou316/meta-gcn):
//     x_j = index_select(x, 0, src) * norm          gcn_base_models.py:223-224
//     x   = torch_scatter.scatter_add(x_j, dst)      common.py:59
// i.e. it materialises an [E, F] tensor (5.6 GB at 11M edges, F=128) and
// scatters it with atomics (GPU) or a serial loop (CPU).  Here nothing of size
// [E, F] exists: each destination row is owned by one lane group, which
// gathers its source rows straight from HBM into registers (G lanes x VEC
// floats = one coalesced row read per edge), multiplies, and accumulates in
// registers -- no atomics, deterministic, and in COO edge order, so the
// result is bit-identical to the reference's sequential CPU scatter_add given
// the same H.  Products and sums are rounded separately (no FMA contraction:
// __fmul_rn/__fadd_rn, and -ffp-contract=off for the whole library).
//
// Roofline: HBM-bound.  Algorithmic bytes per launch
//     8 (n_rows + 1) + nnz * (4 col + 4 w + 4 F) + 4 n_rows F
// (SURVEY.md §8(d) B_spmm); the gathered feature rows dominate.
//
// Layout of a wave: 64 lanes = RPW row groups of G lanes; a group covers
// G*VEC consecutive features of one row per chunk (F = 128, VEC = 4: G = 32,
// two rows per wave).  Edge metadata (col, w, eid) is loaded lane-parallel,
// G edges per instruction, and broadcast inside the group by ds_bpermute
// (__shfl) -- or by v_readlane when a group is the whole wave.  U gathers are
// issued back to back before any of them is consumed (U rows in flight per
// group), then folded into the accumulator strictly in edge order.

#include <hipcub/hipcub.hpp>

#include "heavy.h"
#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kWaves = 4;  // waves per 256-thread block
constexpr int kBlock = 64 * kWaves;

// Broadcast lane `k` of this lane's group (groups of G lanes).  G == 64: the
// group is the wave and k is wave-uniform -> v_readlane into an SGPR.
template <int G>
__device__ __forceinline__ int bcast_i(int v, int group_base, int k) {
  if constexpr (G == 64) {
    return __builtin_amdgcn_readlane(v, k);
  } else {
    return __shfl(v, group_base + k, 64);
  }
}
template <int G>
__device__ __forceinline__ float bcast_f(float v, int group_base, int k) {
  return __int_as_float(bcast_i<G>(__float_as_int(v), group_base, k));
}

// max over the wave of a per-group value (groups of G lanes; all lanes active)
template <int G>
__device__ __forceinline__ int64_t wave_max_over_groups(int64_t v) {
#pragma unroll
  for (int off = G; off < 64; off <<= 1) {
    const int64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

template <int VEC, int G, int U, int MODE>
__global__ __launch_bounds__(kBlock) void spmm_kernel(const SpmmArgs a) {
  constexpr int RPW = 64 / G;  // rows per wave
  constexpr bool kFwd = (MODE == FWD_SUM || MODE == FWD_MAX);
  // the forward max tracks its winner as the edge's position in the row (the
  // winner bits are per slot; argmax rows are mapped to edge ids at the end)
  constexpr bool kNeedEid = (MODE == BWD_MAX);
  // forward max, F a multiple of 128 at 4 x 32 lanes: winner bits assembled
  // in LDS (one 16-B record per edge and 128-feature chunk, 32 edges a window)
  constexpr bool kWinLds = (MODE == FWD_MAX && VEC == 4 && G == 32);
  __shared__ __attribute__((aligned(16))) uint32_t win_rec[kWinLds ? kWaves * 2 * 32 * 4 : 1];
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);
  const int grp = lane / G;
  const int gbase = grp * G;
  const int wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_work = a.order != nullptr ? a.n_rows - a.n_heavy : a.n_rows;
  const int32_t *__restrict__ light = a.order != nullptr ? a.order + a.n_heavy : nullptr;
  const int64_t n_row_groups = (n_work + RPW - 1) / RPW;
  const int64_t wave_stride = (int64_t)gridDim.x * kWaves;
  const float *__restrict__ X = a.X;
  const bool has_w = a.w != nullptr;

  // Row metadata runs ahead of the rows: the row pointers of the next task
  // and the row id of the one after are loaded while the current row is
  // gathered, so a task costs col -> rows instead of order -> rowptr -> col
  // -> rows round trips (short rows, config 3's F = 32 light rows, are
  // bound by that chain).
  auto row_of = [&](int64_t wv, bool &ok) -> int64_t {
    const int64_t item = wv * RPW + grp;
    ok = wv < n_row_groups && item < n_work;
    return !ok ? 0 : light != nullptr ? (int64_t)light[item] : item;
  };
  const int64_t wv0 = (int64_t)blockIdx.x * kWaves + wave_in_block;
  bool ok_n, ok_nn;
  int64_t row_n = row_of(wv0, ok_n);
  int64_t beg_n = ok_n ? a.rowptr[row_n] : 0, end_n = ok_n ? a.rowptr[row_n + 1] : 0;
  int64_t row_nn = row_of(wv0 + wave_stride, ok_nn);
  for (int64_t wv = wv0; wv < n_row_groups; wv += wave_stride) {
    const bool row_ok = ok_n;
    const int64_t row = row_n;
    const int64_t beg = beg_n;
    const int64_t deg = end_n - beg_n;
    row_n = row_nn;
    ok_n = ok_nn;
    beg_n = ok_n ? a.rowptr[row_n] : 0;
    end_n = ok_n ? a.rowptr[row_n + 1] : 0;
    row_nn = row_of(wv + 2 * wave_stride, ok_nn);
    const int64_t maxdeg = (RPW > 1) ? wave_max_over_groups<G>(deg) : deg;

    for (int c = 0; c < a.n_chunks; ++c) {
      const int f0 = (c * G + gl) * VEC;
      const bool f_ok = f0 < a.F;
      F32v<VEC> acc;
      I32v<VEC> arg;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        acc.v[j] = (MODE == FWD_MAX) ? MGCN_MAX_FILL : 0.0f;
        arg.v[j] = -1;
      }

      for (int64_t e0 = 0; e0 < maxdeg; e0 += G) {
        // lane-parallel metadata for the next (up to) G edges of this row
        const int64_t my = e0 + gl;
        int mc = 0, me = 0;
        float mw = 1.0f, mcnt = 1.0f;
        if (my < deg) {
          mc = a.col[beg + my];
          if (has_w) mw = a.w[beg + my];
          if constexpr (kNeedEid) me = a.eid[beg + my];
          if constexpr (MODE == BWD_MAXM) me = a.slot_map[beg + my];  // fwd slot of this edge
          if constexpr (MODE == BWD_MEAN) mcnt = a.cnt[mc];
        }
        const int64_t rem = deg - e0;
        const int nb = rem <= 0 ? 0 : (rem < G ? (int)rem : G);  // this group
        const int64_t remw = maxdeg - e0;
        const int nbmax = remw < G ? (int)remw : G;              // wave-uniform

        for (int k0 = 0; k0 < nbmax; k0 += U) {
          F32v<VEC> xv[U];
          float wk[U];
          int ek[U];
          bool ok[U];
          uint32_t wbits[U];  // BWD_MAXM: the edge's winner word
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = k0 + u;
            const int kk = k & (G - 1);
            const int ck = bcast_i<G>(mc, gbase, kk);
            wk[u] = bcast_f<G>(mw, gbase, kk);
            ek[u] = (MODE == FWD_MAX) ? (int)(e0 + k)
                    : (kNeedEid || MODE == BWD_MAXM) ? bcast_i<G>(me, gbase, kk) : 0;
            float cntk = 1.0f;
            if constexpr (MODE == BWD_MEAN) cntk = bcast_f<G>(mcnt, gbase, kk);
            ok[u] = (k < nb) && f_ok;
            const float *src = X + (int64_t)ck * a.ldx + f0;
            if constexpr (MODE == BWD_MAXM) {
              // dY row and the edge's winner bits (at its fwd slot) are loaded
              // unconditionally (masked edges read row 0 / word 0, never
              // used) and selected in the fold: a select here, between the
              // loads, would make every load wait for the previous one
              const int64_t W = (a.F + 31) >> 5;
              wbits[u] = a.win_mask[ok[u] ? (int64_t)ek[u] * W + (f0 >> 5) : 0];
              xv[u] = load_f<VEC>(ok[u] ? src : X);
            } else if constexpr (MODE == BWD_MAX) {
              // route dY only through the (d, f) entries whose argmax is this edge
#pragma unroll
              for (int j = 0; j < VEC; ++j) xv[u].v[j] = 0.0f;
              if (ok[u]) {
                const I32v<VEC> am = load_i<VEC>(a.argmax_in + (int64_t)ck * a.F + f0);
                bool any = false;
#pragma unroll
                for (int j = 0; j < VEC; ++j) any |= (am.v[j] == ek[u]);
                if (any) {
                  const F32v<VEC> g = load_f<VEC>(src);
#pragma unroll
                  for (int j = 0; j < VEC; ++j) xv[u].v[j] = (am.v[j] == ek[u]) ? g.v[j] : 0.0f;
                }
              }
            } else {
              if (ok[u]) {
                xv[u] = load_f<VEC>(src);
              } else {
#pragma unroll
                for (int j = 0; j < VEC; ++j) xv[u].v[j] = 0.0f;
              }
              if constexpr (MODE == BWD_MEAN) {
#pragma unroll
                for (int j = 0; j < VEC; ++j) xv[u].v[j] = __fdiv_rn(xv[u].v[j], cntk);
              }
            }
          }
          // fold in strictly ascending edge order
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (ok[u]) {
              if constexpr (MODE == BWD_MAXM) {
                const uint32_t bits = wbits[u] >> (f0 & 31);
#pragma unroll
                for (int j = 0; j < VEC; ++j) xv[u].v[j] = ((bits >> j) & 1u) ? xv[u].v[j] : 0.0f;
              }
#pragma unroll
              for (int j = 0; j < VEC; ++j) {
                const float p = __fmul_rn(xv[u].v[j], wk[u]);
                if constexpr (MODE == FWD_MAX) {
                  if (p >= acc.v[j]) {  // torch_scatter 1.x CPU: `>=`, later edge wins ties
                    acc.v[j] = p;
                    arg.v[j] = ek[u];
                  }
                } else {
                  acc.v[j] = __fadd_rn(acc.v[j], p);
                }
              }
            }
          }
        }
      }

      if constexpr (MODE == FWD_MAX) {
        if (a.win_mask_out != nullptr) {
          // winner bits of every edge of this row, at its own (fwd) slot
          int32_t winner[VEC];  // position of the winning edge in the row, -1: none
#pragma unroll
          for (int j = 0; j < VEC; ++j) winner[j] = (acc.v[j] == MGCN_MAX_FILL) ? -1 : arg.v[j];
          const int64_t W = (a.F + 31) >> 5;
          if (kWinLds && (a.F & 127) == 0) {
            // each lane ORs its four winner bits into the window's records
            // (word gl / 8 of an edge's record, bit 4 (gl % 8) + j), then
            // lane gl writes record gl out: 512 contiguous bytes per group.
            // One wave's LDS operations execute in order, so the zeroing,
            // the ORs and the read-back of a window need no barrier.
            // the lane constants below are derived from an opaque copy of the
            // lane id: hoisted out of the edge loop they would stay live
            // through it (+21 VGPRs: 4 instead of 5 waves per SIMD)
            int tl = (int)threadIdx.x;
            asm volatile("" : "+v"(tl));
            const int gl2 = tl & (G - 1);
            uint32_t *rec = win_rec + ((tl >> 6) * 2 + ((tl & 63) / G)) * 32 * 4;
            const int sh = (gl2 & 7) << 2;
            for (int64_t w0 = 0; w0 < maxdeg; w0 += 32) {
              *reinterpret_cast<uint4 *>(rec + 4 * gl2) = make_uint4(0u, 0u, 0u, 0u);
              __builtin_amdgcn_wave_barrier();
#pragma unroll
              for (int j = 0; j < VEC; ++j) {
                const int64_t p = winner[j] - w0;
                if (winner[j] >= 0 && p >= 0 && p < 32)
                  atomicOr(rec + 4 * p + (gl2 >> 3), 1u << (sh + j));
              }
              __builtin_amdgcn_wave_barrier();
              const uint4 r = *reinterpret_cast<const uint4 *>(rec + 4 * gl2);
              if (w0 + gl2 < deg)
                *reinterpret_cast<uint4 *>(a.win_mask_out + (beg + w0 + gl2) * W + 4 * c) = r;
              __builtin_amdgcn_wave_barrier();
            }
          } else {
            // a pass over the row's edge positions; each 32-bit word is OR-ed
            // over its lanes (all lanes of the group take part)
            constexpr int LW = (32 / VEC) < G ? (32 / VEC) : G;  // lanes per word in a group
            for (int64_t e0 = 0; e0 < maxdeg; e0 += G) {
              const int64_t rem = deg - e0;
              const int nb = rem <= 0 ? 0 : (rem < G ? (int)rem : G);
              const int64_t remw = maxdeg - e0;
              const int nbmax = remw < G ? (int)remw : G;  // wave-uniform
              for (int k = 0; k < nbmax; ++k) {
                const int32_t ek = (int32_t)(e0 + k);
                uint32_t v = 0;
#pragma unroll
                for (int j = 0; j < VEC; ++j) v |= (winner[j] == ek ? 1u : 0u) << j;
                v <<= (f0 & 31);
#pragma unroll
                for (int off = 1; off < LW; off <<= 1) v |= __shfl_xor(v, off, 64);
                if (k < nb && f_ok && (f0 & 31) == 0)
                  a.win_mask_out[(beg + e0 + k) * W + (f0 >> 5)] = v;
              }
            }
          }
        }
      }
      if (!(row_ok && f_ok)) continue;
      float *dst = a.Y + row * a.ldy + f0;
      if constexpr (kFwd) {
        const float inv_cnt = (float)(deg > 1 ? deg : 1);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float y = acc.v[j];
          if constexpr (MODE == FWD_MAX) {
            if (y == MGCN_MAX_FILL) {  // common.py:63-64 (and no gradient there)
              y = 0.0f;
              arg.v[j] = -1;
            }
          } else {
            if (a.mean) y = __fdiv_rn(y, inv_cnt);
          }
          if (a.bias != nullptr) y = __fadd_rn(y, a.bias[f0 + j]);
          if (a.relu) y = (y < 0.0f) ? 0.0f : y;
          acc.v[j] = y;
        }
        if constexpr (MGCN_NT_EXTRA != 0 && G >= 32) store_f_nt<VEC>(dst, acc);
        else store_f<VEC>(dst, acc);
        if constexpr (VEC == 4 && G == 32) {
          // ReLU mask for the dX GEMM epilogue: lane gl holds features 4 gl + j,
          // so word j of the row is the group's 32 bits of one ballot
          if (a.relu_mask != nullptr) {
            uint32_t mw[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) mw[j] = (uint32_t)(__ballot(acc.v[j] > 0.0f) >> gbase);
            if (gl == 0)
              *reinterpret_cast<uint4 *>(a.relu_mask + row * 4) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
          }
        }
        if constexpr (MODE == FWD_MAX) {
          if (a.argmax_out != nullptr) {
            // winner positions -> edge ids (torch_scatter's argmax)
#pragma unroll
            for (int j = 0; j < VEC; ++j) arg.v[j] = arg.v[j] >= 0 ? a.eid[beg + arg.v[j]] : -1;
            store_i<VEC>(a.argmax_out + row * a.F + f0, arg);
          }
        }
      } else {
        if (a.row_scale != nullptr) {
          const float s = a.row_scale[row];
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc.v[j] = __fmul_rn(acc.v[j], s);
        }
        if (a.accumulate) {
          const F32v<VEC> old = load_f<VEC>(dst);
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc.v[j] = __fadd_rn(old.v[j], acc.v[j]);
        }
        if constexpr (MGCN_NT_EXTRA != 0 && G >= 32) store_f_nt<VEC>(dst, acc);
        else store_f<VEC>(dst, acc);
      }
    }
  }
}

template <int VEC, int MODE, int HB, int Q>
__global__ __launch_bounds__(HB) void spmm_heavy_kernel(const SpmmArgs a, int FC, int BE) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  heavy_row_block<VEC, MODE, HB, Q>(a, FC, BE, blockIdx.x, smem);
}

__global__ __launch_bounds__(kBlock) void row_degree_kernel(int64_t n_rows,
                                                            const int64_t *__restrict__ rowptr,
                                                            int64_t thr, int64_t giant_thr,
                                                            int32_t *__restrict__ deg,
                                                            int32_t *__restrict__ iota,
                                                            unsigned long long *__restrict__ count) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = rowptr[r + 1] - rowptr[r];
    deg[r] = d < INT32_MAX ? (int32_t)d : INT32_MAX;
    iota[r] = (int32_t)r;
    if (d > thr) {
      atomicAdd(&count[0], 1ull);
      if (d > giant_thr) atomicAdd(&count[1], 1ull);
    }
  }
}

// mgcn_slot_map: inverse permutation of the fwd view's edge ids, then the
// fwd slot of every bwd slot.
__global__ __launch_bounds__(kBlock) void invert_eid_kernel(int64_t nnz,
                                                             const int32_t *__restrict__ eid_t,
                                                             int32_t *__restrict__ inv) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nnz;
       j += (int64_t)gridDim.x * blockDim.x)
    inv[eid_t[j]] = (int32_t)j;
}

__global__ __launch_bounds__(kBlock) void slot_map_kernel(int64_t nnz,
                                                           const int32_t *__restrict__ eid,
                                                           const int32_t *__restrict__ inv,
                                                           int32_t *__restrict__ slot_map) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz;
       k += (int64_t)gridDim.x * blockDim.x)
    slot_map[k] = inv[eid[k]];
}

// mgcn_max_mask: for every fwd row d and edge k of it, the features f whose
// argmax[d, f] is that edge, as bits at win_mask[k][f / 32].  A 32-lane group per (row, 128-feature chunk), 4
// features per lane: argmax of row d is read once (coalesced), the row's
// (eid, slot) pairs lane-parallel and broadcast; each 32-bit word is OR-ed
// over its 8 lanes by shuffles, and the 4 word lanes store an edge's 16 B.
__global__ __launch_bounds__(kBlock) void max_mask_kernel(int64_t n_rows, int32_t F,
                                                          const int64_t *__restrict__ rowptr,
                                                          const int32_t *__restrict__ eid,
                                                          const int32_t *__restrict__ argmax,
                                                          uint32_t *__restrict__ win_mask) {
  const int gl = threadIdx.x & 31;
  const int nchunk = (F + 127) >> 7;
  const int W = (F + 31) >> 5;
  const int64_t groups = n_rows * nchunk;
  const int64_t gstride = (int64_t)gridDim.x * (kBlock / 32);
  for (int64_t gid = (int64_t)blockIdx.x * (kBlock / 32) + (threadIdx.x >> 5); gid < groups;
       gid += gstride) {
    const int64_t d = gid / nchunk;
    const int c = (int)(gid - d * nchunk);
    const int f0 = c * 128 + 4 * gl;
    int32_t am[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) am[j] = (f0 + j < F) ? argmax[d * F + f0 + j] : -1;
    const int64_t beg = rowptr[d], end = rowptr[d + 1];
    for (int64_t e0 = beg; e0 < end; e0 += 32) {
      const int64_t my = e0 + gl;
      const int32_t me = my < end ? eid[my] : -1;
      const int nb = (end - e0) < 32 ? (int)(end - e0) : 32;
      for (int k = 0; k < nb; ++k) {
        const int32_t ek = __shfl(me, k, 32);
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) v |= (am[j] == ek ? 1u : 0u) << j;
        v <<= 4 * (gl & 7);
        v |= __shfl_xor(v, 1, 32);
        v |= __shfl_xor(v, 2, 32);
        v |= __shfl_xor(v, 4, 32);
        if ((gl & 7) == 0 && f0 < F) win_mask[(e0 + k) * W + (f0 >> 5)] = v;
      }
    }
  }
}

int pick_vec(int32_t F, const void *p0, int64_t ld0, const void *p1, int64_t ld1) {
  auto ok = [&](int v) {
    if (F % v) return false;
    if (ld0 % v || ld1 % v) return false;
    if (reinterpret_cast<uintptr_t>(p0) % (4 * v)) return false;
    if (reinterpret_cast<uintptr_t>(p1) % (4 * v)) return false;
    return true;
  };
  if (ok(4)) return 4;
  if (ok(2)) return 2;
  return 1;
}

// ReLU mask of rows of Y (F <= 128; layout as SpmmArgs::relu_mask): two
// rows per wave, lane gl of a row's 32 holds features 4 gl .. 4 gl + 3.
// rows == NULL: rows 0 .. n - 1, else rows[0 .. n).
__global__ __launch_bounds__(256) void relu_mask_kernel(int64_t n, int F, const float *__restrict__ Y,
                                                        int64_t ldy, const int32_t *__restrict__ rows,
                                                        uint32_t *__restrict__ mask) {
  const int lane = threadIdx.x & 63;
  const int gl = lane & 31, gbase = lane & 32;
  const int64_t item = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool ok = item < n;
  const int64_t row = !ok ? 0 : rows != nullptr ? (int64_t)rows[item] : item;
  uint32_t mw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = 4 * gl + j;
    const bool pos = ok && f < F && Y[row * ldy + f] > 0.0f;
    mw[j] = (uint32_t)(__ballot(pos) >> gbase);
  }
  if (ok && gl == 0) *reinterpret_cast<uint4 *>(mask + row * 4) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
}

int launch_relu_mask(int64_t n, int F, const float *Y, int64_t ldy, const int32_t *rows,
                     uint32_t *mask, hipStream_t stream) {
  if (n <= 0) return MGCN_OK;
  const int64_t blocks = (n + 7) / 8;
  hipLaunchKernelGGL(relu_mask_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, n, F, Y, ldy,
                     rows, mask);
  return check_launch("relu_mask_kernel");
}

int g_force_vec = 0;  // tuning knobs (mgcn_set_option)
int g_unroll = 8;
bool g_unroll_set = false;  // spmm_unroll given explicitly: every mode takes it
int g_heavy_side = 1;  // heavy-row launch on a side stream (concurrent)

template <int VEC, int G, int U, int MODE>
int launch_one(const SpmmArgs &a, hipStream_t stream) {
  constexpr int RPW = 64 / G;
  const int64_t waves = (a.n_rows + RPW - 1) / RPW;
  int64_t blocks = (waves + kWaves - 1) / kWaves;
  if (blocks > (int64_t(1) << 20)) blocks = int64_t(1) << 20;  // grid-stride beyond
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((spmm_kernel<VEC, G, U, MODE>), dim3((unsigned)blocks), dim3(kBlock), 0,
                     stream, a);
  return check_launch("spmm_kernel");
}

template <int VEC, int MODE>
int launch_g(const SpmmArgs &a, hipStream_t stream) {
  const int lanes = (a.F + VEC - 1) / VEC;
  if (lanes > 32) {
    if (g_unroll == 16) return launch_one<VEC, 64, 16, MODE>(a, stream);
    if (g_unroll == 4) return launch_one<VEC, 64, 4, MODE>(a, stream);
    return launch_one<VEC, 64, 8, MODE>(a, stream);
  }
  if (lanes > 16) {
    if (g_unroll == 16) return launch_one<VEC, 32, 16, MODE>(a, stream);
    // the forward max at U = 8 holds 104 VGPRs (4 waves per SIMD); at U = 6
    // it fits 93 (5 waves, the sum kernel's occupancy, 30 rows in flight per
    // SIMD lane slot against U = 4's 20)
    if (g_unroll == 6 || (MODE == FWD_MAX && !g_unroll_set)) return launch_one<VEC, 32, 6, MODE>(a, stream);
    if (g_unroll == 4) return launch_one<VEC, 32, 4, MODE>(a, stream);
    return launch_one<VEC, 32, 8, MODE>(a, stream);
  }
  if (lanes > 8) return launch_one<VEC, 16, 8, MODE>(a, stream);
  if (lanes > 4) return launch_one<VEC, 8, 8, MODE>(a, stream);
  return launch_one<VEC, 4, 4, MODE>(a, stream);
}

// LDS per heavy workgroup (two product buffers + the metadata ring).  The
// per-batch cost is about one gather round trip, so long rows want big
// batches: a giant row's workgroup takes the whole 160 KB of a CU; the other
// heavy rows (a few hundred edges) take little, so several share a CU.
int g_heavy_lds = 160 * 1024;     // giant rows
int g_heavy_mid_lds = 40 * 1024;  // other heavy rows
int g_heavy_mid_q1 = 1;           // narrow rows: one edge quad in flight (heavy_mid_q1)
int g_heavy_block = 1024;         // threads per giant-row workgroup
int64_t g_giant_thr = 512;        // degree above which a heavy row is giant

template <int VEC, int MODE, int HB, int Q>
int launch_heavy_q(const SpmmArgs &a, int64_t n, int FC, int BE, size_t lds, hipStream_t stream) {
  // the 160 KB dynamic-LDS attribute is per device: one bit per device id,
  // per instantiation (VEC, MODE, HB, Q); racing threads at worst both set it
  static std::atomic<uint64_t> attr_set{0};
  int dev = 0;
  MGCN_HIP_TRY(hipGetDevice(&dev));
  const uint64_t bit = uint64_t(1) << (dev & 63);
  if (!(attr_set.load(std::memory_order_acquire) & bit)) {
    MGCN_HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(&spmm_heavy_kernel<VEC, MODE, HB, Q>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set.fetch_or(bit, std::memory_order_release);
  }
  hipLaunchKernelGGL((spmm_heavy_kernel<VEC, MODE, HB, Q>), dim3((unsigned)n), dim3(HB), lds, stream,
                     a, FC, BE);
  return check_launch("spmm_heavy_kernel");
}

template <int VEC, int MODE, int HB>
int launch_heavy_hb(SpmmArgs a, const int32_t *rows, int64_t n, int lds_budget,
                    hipStream_t stream) {
  if (n <= 0) return MGCN_OK;
  a.heavy_rows = rows;
  int FC = a.F < 128 ? a.F : 128;
  FC = (FC + VEC - 1) / VEC * VEC;
  const int producers = HB - 64 * ((FC + 63) / 64);
  // 2 product buffers of FC x (BE + 4) floats + a 3-slot ring of 4 x BE words
  int BE = (lds_budget / 4 - 8 * FC) / (2 * FC + 12);
  if (BE > 4 * producers) BE = 4 * producers;  // kEpt metadata entries per producer
  BE &= ~15;
  if (BE < 16) BE = 16;  // a small budget still gets one 16-edge batch (<= 21 KB)
  const size_t lds = sizeof(float) * ((size_t)2 * FC * (BE + 4) + (size_t)12 * BE);
  // narrow rows (FC <= 32, config 3's F = 32) in the 256-thread workgroups:
  // one edge quad in flight per producer (84 VGPRs instead of 172-188, so
  // LDS, not registers, sets the workgroups per CU): 2.77 -> 2.67 ms/step
  if constexpr (HB == 256)
    if (FC <= 32 && g_heavy_mid_q1) return launch_heavy_q<VEC, MODE, HB, 1>(a, n, FC, BE, lds, stream);
  return launch_heavy_q<VEC, MODE, HB, 0>(a, n, FC, BE, lds, stream);
}

template <int VEC, int MODE>
int launch_heavy(const SpmmArgs &a, bool giant, hipStream_t stream) {
  if (!giant)
    return launch_heavy_hb<VEC, MODE, 256>(a, a.order + a.n_giant, a.n_heavy - a.n_giant,
                                           g_heavy_mid_lds, stream);
  if (g_heavy_block == 256)
    return launch_heavy_hb<VEC, MODE, 256>(a, a.order, a.n_giant, g_heavy_lds, stream);
  if (g_heavy_block == 512)
    return launch_heavy_hb<VEC, MODE, 512>(a, a.order, a.n_giant, g_heavy_lds, stream);
  return launch_heavy_hb<VEC, MODE, 1024>(a, a.order, a.n_giant, g_heavy_lds, stream);
}

template <int MODE>
int launch_heavy_v(const SpmmArgs &a, int vec, bool giant, hipStream_t stream) {
  if (vec == 4) return launch_heavy<4, MODE>(a, giant, stream);
  if (vec == 2) return launch_heavy<2, MODE>(a, giant, stream);
  return launch_heavy<1, MODE>(a, giant, stream);
}

// Side stream per device for the heavy-row launch: fork from the caller's
// stream with an event, join back with another (caller-visible ordering is
// unchanged: everything after the call on `stream` waits for both launches).
struct SideStream {
  hipStream_t stream = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;   // device-scope release (same-GPU streams)
  hipEvent_t fork_sys = nullptr, join_sys = nullptr;  // with the system-scope fence
};
int g_side_fence = 0;  // mgcn_set_option("heavy_side_fence"): 1 = system-scope events

int side_stream(SideStream **out) {
  static thread_local SideStream per_dev[64];  // per host thread: events never shared
  int dev = 0;
  MGCN_HIP_TRY(hipGetDevice(&dev));
  MGCN_REQUIRE(dev >= 0 && dev < 64, "side_stream: device id %d", dev);
  SideStream &s = per_dev[dev];
  if (s.stream == nullptr) {
    MGCN_HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    // the fork / join only order two streams of one GPU: no system-scope
    // fence (an L2 writeback for host / peer visibility) at each record
    const unsigned fl = hipEventDisableTiming | hipEventDisableSystemFence;
    MGCN_HIP_TRY(hipEventCreateWithFlags(&s.fork, fl));
    MGCN_HIP_TRY(hipEventCreateWithFlags(&s.join, fl));
    MGCN_HIP_TRY(hipEventCreateWithFlags(&s.fork_sys, hipEventDisableTiming));
    MGCN_HIP_TRY(hipEventCreateWithFlags(&s.join_sys, hipEventDisableTiming));
  }
  static thread_local SideStream view[64];
  view[dev] = s;
  if (g_side_fence) view[dev].fork = s.fork_sys, view[dev].join = s.join_sys;
  *out = &view[dev];
  return MGCN_OK;
}

// Launch order: giant rows on the side stream (forked from `stream`, joined
// back), then the other heavy rows and the lane-group kernel on `stream`; the
// giant rows -- the critical path -- overlap everything else.
template <int MODE>
int launch_mode(SpmmArgs a, int vec, hipStream_t stream) {
  const int G_lanes_max = 64;
  const int per_chunk = G_lanes_max * vec;
  a.n_chunks = (a.F + per_chunk - 1) / per_chunk;
  if (a.n_chunks < 1) a.n_chunks = 1;
  if (a.order == nullptr) {
    a.n_heavy = 0;
    a.n_giant = 0;
  }
  SideStream *side = nullptr;
  if (a.n_giant > 0) {
    if (g_heavy_side) {
      if (int rc = side_stream(&side)) return rc;
      MGCN_HIP_TRY(hipEventRecord(side->fork, stream));
      MGCN_HIP_TRY(hipStreamWaitEvent(side->stream, side->fork, 0));
      if (int rc = launch_heavy_v<MODE>(a, vec, true, side->stream)) return rc;
      MGCN_HIP_TRY(hipEventRecord(side->join, side->stream));
    } else if (int rc = launch_heavy_v<MODE>(a, vec, true, stream)) {
      return rc;
    }
  }
  int rc = a.n_heavy > a.n_giant ? launch_heavy_v<MODE>(a, vec, false, stream) : MGCN_OK;
  if (rc == MGCN_OK) {
    rc = vec == 4   ? launch_g<4, MODE>(a, stream)
         : vec == 2 ? launch_g<2, MODE>(a, stream)
                    : launch_g<1, MODE>(a, stream);
  }
  if (side != nullptr) MGCN_HIP_TRY(hipStreamWaitEvent(stream, side->join, 0));
  if (rc == MGCN_OK && a.relu_mask != nullptr) {
    // the lane-group kernel fuses the mask when a row is 32 lanes x 4
    // floats; heavy rows and other layouts get it from Y afterwards
    const int lanes = (a.F + vec - 1) / vec;
    const bool fused = vec == 4 && lanes > 16 && lanes <= 32;
    if (!fused)
      rc = launch_relu_mask(a.n_rows, a.F, a.Y, a.ldy, nullptr, a.relu_mask, stream);
    else if (a.n_heavy > 0)
      rc = launch_relu_mask(a.n_heavy, a.F, a.Y, a.ldy, a.order, a.relu_mask, stream);
  }
  return rc;
}

}  // namespace

// Heavy rows only (residual.hip's fused layer kernels aggregate the light
// rows themselves): the giant rows on the side stream, the other heavy rows
// on `stream`.  Forward (bwd = 0): Y[row] = sum / mean of the row's gathered
// X rows; backward (bwd = 1): Y[row] = the adjoint sum (* row_scale).
// *side_used: the caller must heavy_rows_join(stream) before reading the
// giant rows' results.
int heavy_rows(int bwd, int64_t n_rows, int32_t F, const int64_t *rowptr, const int32_t *col,
               const int32_t *eid, const float *w, const float *X, int64_t ldx, float *Y,
               int64_t ldy, const float *row_scale, int mean, const int32_t *order,
               int64_t n_heavy, int64_t n_giant, hipStream_t stream, bool *side_used,
               const ResEpi *rs) {
  *side_used = false;
  if (order == nullptr || n_heavy <= 0) return MGCN_OK;
  SpmmArgs a{};
  a.n_rows = n_rows;
  a.F = F;
  a.n_chunks = 1;
  a.rowptr = rowptr;
  a.col = col;
  a.eid = eid;
  a.w = w;
  a.X = X;
  a.ldx = ldx;
  a.Y = Y;
  a.ldy = ldy;
  a.row_scale = row_scale;
  a.mean = mean;
  a.order = order;
  a.n_heavy = n_heavy;
  a.n_giant = n_giant;
  if (rs != nullptr) a.rs = *rs;
  const int vec = pick_vec(F, X, ldx, Y, ldy);
  if (n_giant > 0) {
    SideStream *side = nullptr;
    if (g_heavy_side) {
      if (int rc = side_stream(&side)) return rc;
      MGCN_HIP_TRY(hipEventRecord(side->fork, stream));
      MGCN_HIP_TRY(hipStreamWaitEvent(side->stream, side->fork, 0));
      const int rc = bwd ? launch_heavy_v<BWD_SUM>(a, vec, true, side->stream)
                         : launch_heavy_v<FWD_SUM>(a, vec, true, side->stream);
      if (rc) return rc;
      MGCN_HIP_TRY(hipEventRecord(side->join, side->stream));
      *side_used = true;
    } else {
      const int rc = bwd ? launch_heavy_v<BWD_SUM>(a, vec, true, stream)
                         : launch_heavy_v<FWD_SUM>(a, vec, true, stream);
      if (rc) return rc;
    }
  }
  if (n_heavy > n_giant)
    return bwd ? launch_heavy_v<BWD_SUM>(a, vec, false, stream)
               : launch_heavy_v<FWD_SUM>(a, vec, false, stream);
  return MGCN_OK;
}

int heavy_rows_join(hipStream_t stream) {
  SideStream *side = nullptr;
  if (int rc = side_stream(&side)) return rc;
  MGCN_HIP_TRY(hipStreamWaitEvent(stream, side->join, 0));
  return MGCN_OK;
}

}  // namespace mgcn

using namespace mgcn;

#ifdef MGCN_HEAVY_PROFILE
extern "C" int mgcn_debug_heavy_prof(unsigned long long *host) {
  MGCN_HIP_TRY(hipDeviceSynchronize());
  MGCN_HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hprof), sizeof(g_hprof)));
  return MGCN_OK;
}
#endif

extern "C" int mgcn_set_option(const char *name, int value) {
  clear_error();
  MGCN_REQUIRE(name != nullptr, "mgcn_set_option: null name");
  const std::string n(name);
  if (n == "spmm_vec") {
    MGCN_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4, "spmm_vec must be 0,1,2,4");
    g_force_vec = value;
    return MGCN_OK;
  }
  if (n == "spmm_unroll") {
    MGCN_REQUIRE(value == 4 || value == 6 || value == 8 || value == 16,
                 "spmm_unroll must be 4, 6, 8 or 16");
    g_unroll = value;
    g_unroll_set = true;
    return MGCN_OK;
  }
  if (n == "heavy_lds_kb") {
    MGCN_REQUIRE(value >= 16 && value <= 160, "heavy_lds_kb must be in [16, 160]");
    g_heavy_lds = value * 1024;
    return MGCN_OK;
  }
  if (n == "heavy_block") {
    MGCN_REQUIRE(value == 256 || value == 512 || value == 1024, "heavy_block must be 256, 512 or 1024");
    g_heavy_block = value;
    return MGCN_OK;
  }
  if (n == "heavy_mid_q1") {
    MGCN_REQUIRE(value == 0 || value == 1, "heavy_mid_q1 must be 0 or 1");
    g_heavy_mid_q1 = value;
    return MGCN_OK;
  }
  if (n == "heavy_mid_lds_kb") {
    MGCN_REQUIRE(value >= 16 && value <= 160, "heavy_mid_lds_kb must be in [16, 160]");
    g_heavy_mid_lds = value * 1024;
    return MGCN_OK;
  }
  if (n == "heavy_giant_thr") {
    MGCN_REQUIRE(value >= 0, "heavy_giant_thr must be >= 0");
    g_giant_thr = value;
    return MGCN_OK;
  }
  if (n == "gemm_tn_variant") {
    MGCN_REQUIRE(value >= 0 && value <= 2, "gemm_tn_variant must be 0, 1 or 2");
    return gemm_set_tn_variant(value);
  }
  if (n == "gemm_tn_staged") {
    MGCN_REQUIRE(value == 0 || value == 1, "gemm_tn_staged must be 0 or 1");
    return gemm_set_tn_staged(value);
  }
  if (n == "gemm_precision") {
    MGCN_REQUIRE(value == 0 || value == 1, "gemm_precision must be 0 (f32) or 1 (bf16x6)");
    return gemm_set_precision(value);
  }
  if (n == "spmm_xw_unroll") return xw_set_unroll(value);
  if (n == "xw_ws_dbg" || n == "xw_ws_full" || n == "xw_ws_max" || n == "xw_ws_full_unroll" ||
      n == "xw_pk_unroll" || n == "xw_pk_bwd_unroll")
    return xw_set_ws(name, value);
  if (n == "wide_pair" || n == "wide_ws" || n == "wide_dbg" || n == "wide_mfma") return wide_set_option(name, value);
  if (n == "residual_blocks") {
    MGCN_REQUIRE(value >= 64 && value <= 65536, "residual_blocks must be in [64, 65536]");
    g_rl_cap = value;
    return MGCN_OK;
  }
  if (n == "residual_fused_mask") {
    MGCN_REQUIRE(value == 0 || value == 1, "residual_fused_mask must be 0 or 1");
    g_fused_mask = value;
    return MGCN_OK;
  }
  if (n == "heavy_side_fence") {
    MGCN_REQUIRE(value == 0 || value == 1, "heavy_side_fence must be 0 or 1");
    g_side_fence = value;
    return MGCN_OK;
  }
  if (n == "ws_spin_limit") {  // the warp-specialised kernels' hand-off bound (abort-path tests)
    if (!MGCN_EXPERIMENT) {
      set_error("ws_spin_limit: experiment builds only (make exp -> libmgcn_exp.so)");
      return MGCN_EINVAL;
    }
    MGCN_REQUIRE(value >= 1, "ws_spin_limit must be >= 1");
    g_spin_limit = (uint32_t)value;
    return MGCN_OK;
  }
  if (n == "heavy_side_stream") {
    MGCN_REQUIRE(value == 0 || value == 1, "heavy_side_stream must be 0 or 1");
    g_heavy_side = value;
    return MGCN_OK;
  }
  set_error("mgcn_set_option: unknown option '%s'", name);
  return MGCN_EINVAL;
}

static int choose_vec(int32_t F, const void *p0, int64_t ld0, const void *p1, int64_t ld1) {
  int v = pick_vec(F, p0, ld0, p1, ld1);
  if (g_force_vec != 0 && g_force_vec < v) v = g_force_vec;
  return v;
}

extern "C" int mgcn_spmm_fwd(int64_t n_rows, int32_t F, const int64_t *rowptr, const int32_t *col,
                             const int32_t *eid, const float *w, const float *H, int64_t ldh,
                             float *Y, int64_t ldy, int reduce, const float *bias, int relu,
                             int32_t *argmax, uint32_t *win_mask, uint32_t *relu_mask,
                             const int32_t *order, int64_t n_heavy, int64_t n_giant,
                             void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_spmm_fwd: negative size");
  MGCN_REQUIRE(relu_mask == nullptr || (relu && F <= 128),
               "mgcn_spmm_fwd: relu_mask needs relu and F <= 128");
  MGCN_REQUIRE(reduce == MGCN_REDUCE_SUM || reduce == MGCN_REDUCE_MEAN || reduce == MGCN_REDUCE_MAX,
               "mgcn_spmm_fwd: bad reduce %d", reduce);
  if (n_rows == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && H && Y, "mgcn_spmm_fwd: null array");  // col may be NULL when nnz == 0
  MGCN_REQUIRE(ldh >= F && ldy >= F, "mgcn_spmm_fwd: leading dimension < F");
  MGCN_REQUIRE(reduce != MGCN_REDUCE_MAX || argmax != nullptr || win_mask != nullptr,
               "mgcn_spmm_fwd: MAX needs argmax and/or win_mask (+ eid)");
  SpmmArgs a{};
  a.n_rows = n_rows;
  a.F = F;
  a.rowptr = rowptr;
  a.col = col;
  a.eid = eid;
  a.w = w;
  a.X = H;
  a.ldx = ldh;
  a.Y = Y;
  a.ldy = ldy;
  a.bias = bias;
  a.argmax_out = argmax;
  a.win_mask_out = reduce == MGCN_REDUCE_MAX ? win_mask : nullptr;
  a.relu_mask = relu_mask;
  MGCN_REQUIRE(order == nullptr || (0 <= n_giant && n_giant <= n_heavy && n_heavy <= n_rows),
               "spmm: need 0 <= n_giant <= n_heavy <= n_rows");
  a.order = order;
  a.n_heavy = n_heavy;
  a.n_giant = n_giant;
  a.mean = reduce == MGCN_REDUCE_MEAN;
  a.relu = relu != 0;
  int vec = choose_vec(F, H, ldh, Y, ldy);
  if (reduce == MGCN_REDUCE_MAX && argmax != nullptr &&
      reinterpret_cast<uintptr_t>(argmax) % (4 * vec))
    vec = 1;
  MGCN_REQUIRE(bias == nullptr || reinterpret_cast<uintptr_t>(bias) % 4 == 0,
               "mgcn_spmm_fwd: bias not 4-byte aligned");
  hipStream_t s = as_stream(stream);
  if (reduce == MGCN_REDUCE_MAX) return launch_mode<FWD_MAX>(a, vec, s);
  return launch_mode<FWD_SUM>(a, vec, s);
}

extern "C" int mgcn_relu_mask(int64_t n_rows, int32_t F, const float *Z, int64_t ldz,
                              uint32_t *relu_mask, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0 && F <= 128, "mgcn_relu_mask: need 0 <= F <= 128");
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(Z && relu_mask && ldz >= F, "mgcn_relu_mask: bad arguments");
  return launch_relu_mask(n_rows, F, Z, ldz, nullptr, relu_mask, as_stream(stream));
}

extern "C" int mgcn_spmm_bwd(int64_t n_rows, int32_t F, const int64_t *rowptr_t,
                             const int32_t *col_t, const int32_t *eid_t, const float *w_t,
                             const float *row_scale, const float *dY, int64_t lddy, float *dH,
                             int64_t lddh, int reduce, const float *cnt, const int32_t *argmax,
                             const uint32_t *win_mask, const int32_t *slot_map, int accumulate,
                             const int32_t *order, int64_t n_heavy, int64_t n_giant,
                             void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_spmm_bwd: negative size");
  MGCN_REQUIRE(reduce == MGCN_REDUCE_SUM || reduce == MGCN_REDUCE_MEAN || reduce == MGCN_REDUCE_MAX,
               "mgcn_spmm_bwd: bad reduce %d", reduce);
  if (n_rows == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr_t && dY && dH, "mgcn_spmm_bwd: null array");  // col may be NULL when nnz == 0
  MGCN_REQUIRE(lddy >= F && lddh >= F, "mgcn_spmm_bwd: leading dimension < F");
  MGCN_REQUIRE(reduce != MGCN_REDUCE_MEAN || cnt != nullptr, "mgcn_spmm_bwd: MEAN needs cnt");
  MGCN_REQUIRE(reduce != MGCN_REDUCE_MAX || argmax != nullptr || win_mask != nullptr,
               "mgcn_spmm_bwd: MAX needs argmax (+ eid) or win_mask (+ slot_map)");
  MGCN_REQUIRE(win_mask == nullptr || slot_map != nullptr || reduce != MGCN_REDUCE_MAX,
               "mgcn_spmm_bwd: win_mask needs slot_map");
  SpmmArgs a{};
  a.n_rows = n_rows;
  a.F = F;
  a.rowptr = rowptr_t;
  a.col = col_t;
  a.eid = eid_t;
  a.w = w_t;
  a.X = dY;
  a.ldx = lddy;
  a.Y = dH;
  a.ldy = lddh;
  a.row_scale = row_scale;
  a.cnt = cnt;
  a.argmax_in = argmax;
  a.win_mask = reduce == MGCN_REDUCE_MAX ? win_mask : nullptr;
  a.slot_map = slot_map;
  a.accumulate = accumulate != 0;
  MGCN_REQUIRE(order == nullptr || (0 <= n_giant && n_giant <= n_heavy && n_heavy <= n_rows),
               "spmm: need 0 <= n_giant <= n_heavy <= n_rows");
  a.order = order;
  a.n_heavy = n_heavy;
  a.n_giant = n_giant;
  int vec = choose_vec(F, dY, lddy, dH, lddh);
  if (reduce == MGCN_REDUCE_MAX && a.win_mask == nullptr &&
      reinterpret_cast<uintptr_t>(argmax) % (4 * vec))
    vec = 1;
  hipStream_t s = as_stream(stream);
  if (reduce == MGCN_REDUCE_MAX)
    return a.win_mask != nullptr ? launch_mode<BWD_MAXM>(a, vec, s) : launch_mode<BWD_MAX>(a, vec, s);
  if (reduce == MGCN_REDUCE_MEAN) return launch_mode<BWD_MEAN>(a, vec, s);
  return launch_mode<BWD_SUM>(a, vec, s);
}

namespace {
struct ScheduleScratch {
  size_t deg, deg_sorted, iota, count, cub, total;
};

ScheduleScratch schedule_scratch(int64_t n_rows) {
  ScheduleScratch s{};
  const size_t b4 = align_up(static_cast<size_t>(n_rows > 0 ? n_rows : 1) * 4, 256);
  size_t cub_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(
      nullptr, cub_bytes, (const int32_t *)nullptr, (int32_t *)nullptr, (const int32_t *)nullptr,
      (int32_t *)nullptr, static_cast<int>(n_rows > 0 ? n_rows : 1), 0, 31, (hipStream_t)0);
  s.deg = 0;
  s.deg_sorted = b4;
  s.iota = 2 * b4;
  s.count = 3 * b4;
  s.cub = s.count + 256;
  s.total = s.cub + align_up(cub_bytes, 256);
  return s;
}
}  // namespace

extern "C" size_t mgcn_row_schedule_workspace_bytes(int64_t n_rows) {
  return schedule_scratch(n_rows).total;
}

extern "C" int mgcn_row_schedule(int64_t n_rows, const int64_t *rowptr, int64_t heavy_thr,
                                 int32_t *order, int64_t *n_heavy_out, int64_t *n_giant_out,
                                 void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && n_rows < (int64_t(1) << 31) && heavy_thr >= 0 &&
                   n_heavy_out != nullptr && n_giant_out != nullptr,
               "mgcn_row_schedule: bad arguments");
  *n_heavy_out = 0;
  *n_giant_out = 0;
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && order, "mgcn_row_schedule: null array");
  const ScheduleScratch s = schedule_scratch(n_rows);
  if (workspace == nullptr || workspace_bytes < s.total) {
    set_error("mgcn_row_schedule: workspace %zu bytes < required %zu", workspace_bytes, s.total);
    return MGCN_EWORKSPACE;
  }
  char *ws = static_cast<char *>(workspace);
  int32_t *deg = reinterpret_cast<int32_t *>(ws + s.deg);
  int32_t *deg_sorted = reinterpret_cast<int32_t *>(ws + s.deg_sorted);
  int32_t *iota = reinterpret_cast<int32_t *>(ws + s.iota);
  auto *count = reinterpret_cast<unsigned long long *>(ws + s.count);
  size_t cub_bytes = s.total - s.cub;
  hipStream_t st = as_stream(stream);
  MGCN_HIP_TRY(hipMemsetAsync(count, 0, 2 * sizeof(unsigned long long), st));
  hipLaunchKernelGGL(row_degree_kernel, dim3(grid_for(n_rows, kBlock)), dim3(kBlock), 0, st,
                     n_rows, rowptr, heavy_thr, g_giant_thr, deg, iota, count);
  if (int rc = check_launch("row_degree_kernel")) return rc;
  // stable: equal degrees keep ascending row ids
  MGCN_HIP_TRY(hipcub::DeviceRadixSort::SortPairsDescending(
      ws + s.cub, cub_bytes, deg, deg_sorted, iota, order, static_cast<int>(n_rows), 0, 31, st));
  unsigned long long c[2] = {0, 0};
  MGCN_HIP_TRY(hipMemcpyAsync(c, count, sizeof(c), hipMemcpyDeviceToHost, st));
  MGCN_HIP_TRY(hipStreamSynchronize(st));
  *n_heavy_out = (int64_t)c[0];
  *n_giant_out = (int64_t)c[1];
  return MGCN_OK;
}

extern "C" size_t mgcn_slot_map_workspace_bytes(int64_t nnz) {
  return align_up((size_t)(nnz > 0 ? nnz : 1) * sizeof(int32_t), 256);
}

extern "C" int mgcn_slot_map(int64_t nnz, const int32_t *eid, const int32_t *eid_t,
                             int32_t *slot_map, void *workspace, size_t workspace_bytes,
                             void *stream) {  // slot_map[j] = fwd slot of bwd slot j
  clear_error();
  MGCN_REQUIRE(nnz >= 0, "mgcn_slot_map: negative nnz");
  if (nnz == 0) return MGCN_OK;
  MGCN_REQUIRE(eid && eid_t && slot_map, "mgcn_slot_map: null array");
  if (workspace == nullptr || workspace_bytes < mgcn_slot_map_workspace_bytes(nnz)) {
    set_error("mgcn_slot_map: workspace %zu < %zu", workspace_bytes,
              mgcn_slot_map_workspace_bytes(nnz));
    return MGCN_EWORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  int32_t *inv = static_cast<int32_t *>(workspace);
  hipLaunchKernelGGL(invert_eid_kernel, dim3(grid_for(nnz, kBlock)), dim3(kBlock), 0, s, nnz,
                     eid, inv);
  if (int rc = check_launch("invert_eid_kernel")) return rc;
  hipLaunchKernelGGL(slot_map_kernel, dim3(grid_for(nnz, kBlock)), dim3(kBlock), 0, s, nnz, eid_t,
                     inv, slot_map);
  return check_launch("slot_map_kernel");
}

extern "C" int mgcn_max_mask(int64_t n_rows, int32_t F, const int64_t *rowptr,
                             const int32_t *eid, const int32_t *argmax, uint32_t *win_mask,
                             void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_max_mask: negative size");
  if (n_rows == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && argmax, "mgcn_max_mask: null array");  // eid/slot_map/mask: nnz > 0
  hipStream_t s = as_stream(stream);
  const int64_t threads = n_rows * ((F + 127) / 128) * 32;
  hipLaunchKernelGGL(max_mask_kernel, dim3(grid_for(threads, kBlock)), dim3(kBlock), 0, s, n_rows,
                     F, rowptr, eid, argmax, win_mask);
  return check_launch("max_mask_kernel");
}
