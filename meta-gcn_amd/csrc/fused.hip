// Fused GCN layer kernels on gfx950: the aggregation and the layer's dense
// product in one pass, forward and backward (F_in = F_out = 128, sum / mean).
//
// Forward:   Y = epi( (A_norm X) W + b ),   epi = optional ReLU (+ row mask)
// Backward:  dH = A_norm^T dY [* row_scale];  dW = X^T dH;
//            dX = relu'(lower) (dH W^T) [/ row_div],  colsum = sum_rows dX
//
// The reference computes a layer as  x @ W  then  gather -> * norm ->
// scatter_add  (src/gcn_meta/models/gcn_base_models.py:201, 223-237; PyG
// GCNConv: x @ W then propagate), and autograd runs the adjoints in reverse.
// Unfused here that is two launches per direction: mgcn_gemm_nn (reads X,
// writes H = X W) + mgcn_spmm_fwd (gathers H), and mgcn_spmm_bwd (writes dH)
// + mgcn_gemm_bwd (reads X and dH, writes dX).  For a linear aggregator
// A (X W) = (A X) W, so the forward gathers X itself and multiplies the
// aggregated rows of a 32-row chunk by W on MFMA in the same workgroup, and
// the backward multiplies the chunk's dH rows by W^T and X^T before they
// ever leave the workgroup.  H and dH never exist: per layer at config 2 this
// removes 1 GB of HBM traffic in each direction and a launch.  Max does not
// commute with W and keeps the two-launch path.
//
// Numerics: aggregated rows are summed exactly as the SpMM sums (edge order,
// separately rounded products and adds: mgcn_spmm_fwd / _bwd bit for bit);
// the dense products are the bf16x6 MFMA arithmetic of gemm.hip.  The
// forward's association differs from the reference's (A (X W) vs (A X) W),
// so the layer output matches within fp32 tolerance, not bitwise -- except
// for W = I, where every bf16x6 product is exact.  The backward's dX is
// mgcn_gemm_bwd's bit for bit (same dH, same products and order); dW and
// the column sums fold the same products over a different split-K grid.
//
// Chunk layout (both directions): persistent 512-thread workgroups (8
// waves), two per CU; chunk c (rows 32 c .. 32 c + 31) goes to workgroup
// c % grid.
//   Phase A (gather): row 16 p + 2 wave + grp of the chunk is owned by the
//     32-lane group grp of wave `wave` in pass p; lane gl holds features
//     4 gl .. 4 gl + 3 of every gathered 512-B row, U gathers in flight per
//     group, folded in edge order; the finished row is split into the
//     chunk's bf16 hi / mid / lo images (x6.h layout).
//   Phase B (MFMA): wave w owns output columns 16 w .. 16 w + 15 of the
//     chunk (v_mfma_f32_16x16x32_bf16); the backward's dW tiles are
//     gemm_bwd's (32x32x16 on transposed image reads).  Results go to an
//     fp32 staging tile in LDS.
//   The staged tile is written out as whole 512-B rows (16 B per lane) at
//   the start of the next chunk, beside its gathers: 4-byte column stores
//   straight from the MFMA layout cost 0.19 ms per 512 MB (store issue).
//
// Roofline: HBM-bound like the SpMM, with the GEMMs' bytes removed:
//   forward  8 (N + 1) + nnz (4 col + 4 w + 4 F) + 4 N F (+ 16 N mask)
//   backward the same + 4 N F (X) (+ 16 N mask)
// and 2 N F^2 (forward) / 4 N F^2 (backward) x 6 bf16 MFMA flops under it.

#include <string>

#include "mgcn_internal.h"
#include "x6.h"

// cache policy of the streamed (read-once / written-once) rows -- Z written
// by the forward, the own X rows of the backward: 2 = nt (config 2: 5.16 ->
// 5.11-5.12 ms/step, A/B on one box: the fwd-with-Z launch 0.933 -> 0.917 ms,
// the full backward 1.14 -> 1.13 ms)
#ifndef MGCN_NT_AUX
#define MGCN_NT_AUX 2
#endif
// and for the layer outputs (Y forward, dX backward), although they are the
// next kernel's gathered table: the config-2 tables are twice the 256-MB
// Infinity Cache, and allocating the written lines there costs more than it
// saves the next gather (5.14 -> 5.07-5.08 ms/step, three A/B pairs on one
// box: forward 0.864 -> 0.852 ms, dX-only 0.883 -> 0.868, full 1.134 -> 1.119)
#ifndef MGCN_NT_OUT
#define MGCN_NT_OUT 2
#endif

namespace mgcn {
namespace {

using namespace x6;

constexpr int kXwF = 128;
constexpr int kXwRows = 32;
constexpr int kXwWaves = 8;
constexpr int kXwThreads = 64 * kXwWaves;
constexpr int kXwImg = kXwRows * 256;          // one bf16 term image of a chunk
constexpr int kXwStageLd = kXwF + 8;           // backward staging row: 128 values, the row's
                                               // 4 ReLU mask words, its divisor, padding
constexpr int kXwStage = kXwRows * kXwStageLd * 4;
constexpr int kXfStage = kXwRows * kXwF * 4;   // forward staging tile (unpadded: 2 fit)
constexpr int kXwPerCU = 2;  // resident workgroups per CU the grid is sized for

constexpr int EPI_STORE = 0, EPI_RELU = 1, EPI_RELU_DIV = 2;

typedef __attribute__((address_space(3))) void lds_void_t;

// Aggregate one row in the 32-lane group `grp` of the wave (both groups of a
// wave call this together): acc = sum_k X[col_k] * w_k in edge order,
// products and sums rounded separately -- the SpMM's arithmetic, bit for bit.
// Lane gl holds features 4 gl .. 4 gl + 3; edge metadata is loaded 32 edges
// at a time lane-parallel and broadcast by ds_bpermute; U gathers of whole
// 512-B rows are in flight per group before any is folded.
// MAXM (the max adjoint): each edge's dY row counts only at the features
// whose forward winner it was -- the edge's winner word (found through
// slot_map, the fwd slot of each bwd slot; word gl / 8 of its 16-B record,
// bits 4 (gl % 8) + j) is loaded beside the row and selects in the fold.
template <int U, bool MAXM = false>
__device__ __forceinline__ void gather_row(const __amdgpu_buffer_rsrc_t rx, uint32_t ldx_b,
                                           const int64_t *__restrict__ rowptr,
                                           const int32_t *__restrict__ col,
                                           const float *__restrict__ w, int64_t row, bool row_ok,
                                           int gl, int grp, float (&acc)[4], int &deg_out,
                                           const uint32_t *__restrict__ win = nullptr,
                                           const int32_t *__restrict__ slot_map = nullptr) {
  const bool has_w = w != nullptr;
  const int64_t beg = row_ok ? rowptr[row] : 0;
  // a row's degree fits 32 bits; the edge slots are addressed from beg
  const int deg = row_ok ? (int)(rowptr[row + 1] - beg) : 0;
  const int odeg = __shfl_xor(deg, 32, 64);
  const int maxdeg = deg > odeg ? deg : odeg;
  const int32_t *__restrict__ colr = col + beg;
  const float *__restrict__ wr = has_w ? w + beg : nullptr;
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0f;
  for (int e0 = 0; e0 < maxdeg; e0 += 32) {
    const int my = e0 + gl;
    int mc = 0, ms = 0;
    float mw = 1.0f;
    if (my < deg) {
      mc = colr[my];
      if (has_w) mw = wr[my];
      if constexpr (MAXM) ms = slot_map[beg + my];
    }
    const int rem = deg - e0;
    const int nb = rem <= 0 ? 0 : (rem < 32 ? rem : 32);
    const int remw = maxdeg - e0;
    const int nbmax = remw < 32 ? remw : 32;  // wave-uniform
    for (int k0 = 0; k0 < nbmax; k0 += U) {
      float4 xv[U];
      float wk[U];
      bool ok[U];
      uint32_t wbits[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u;
        const int ck = __shfl(mc, 32 * grp + (k & 31), 64);
        wk[u] = __shfl(mw, 32 * grp + (k & 31), 64);
        ok[u] = k < nb;
        // past-the-row edges get an offset beyond the buffer: no access, zeros
        const uint32_t off = ok[u] ? (uint32_t)ck * ldx_b + 16u * gl : 0xfffffff0u;
        xv[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
        if constexpr (MAXM) {
          // loaded unconditionally (masked edges read word 0, never used)
          const int sk = __shfl(ms, 32 * grp + (k & 31), 64);
          wbits[u] = win[ok[u] ? (int64_t)sk * 4 + (gl >> 3) : 0];
        }
      }
      // fold in strictly ascending edge order (as the SpMM, bit for bit)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ok[u]) {
          if constexpr (MAXM) {
            const uint32_t bits = wbits[u] >> (4 * (gl & 7));
            xv[u].x = (bits & 1u) ? xv[u].x : 0.0f;
            xv[u].y = (bits & 2u) ? xv[u].y : 0.0f;
            xv[u].z = (bits & 4u) ? xv[u].z : 0.0f;
            xv[u].w = (bits & 8u) ? xv[u].w : 0.0f;
          }
          acc[0] = __fadd_rn(acc[0], __fmul_rn(xv[u].x, wk[u]));
          acc[1] = __fadd_rn(acc[1], __fmul_rn(xv[u].y, wk[u]));
          acc[2] = __fadd_rn(acc[2], __fmul_rn(xv[u].z, wk[u]));
          acc[3] = __fadd_rn(acc[3], __fmul_rn(xv[u].w, wk[u]));
        }
      }
    }
  }
  deg_out = deg;
}

// Broadcast of lane 32 grp + k (k wave-uniform) to its 32-lane group
// (ds_bpermute; the two-v_readlane form measured slower, exp/ in git history)
__device__ __forceinline__ int bcast_g(int v, int grp, int k) {
  return __shfl(v, 32 * grp + k, 64);
}
__device__ __forceinline__ float bcast_g(float v, int grp, int k) {
  return __int_as_float(bcast_g(__float_as_int(v), grp, k));
}

// Pipelined form for a wave that walks a known sequence of rows: the row
// pointer pair of row k + 2 and the first 32 edge slots (col, w) of row k + 1
// are loaded while row k's feature rows are gathered, so a row costs one
// gather round trip instead of three dependent ones (rowptr -> col -> row).
struct RowMeta {
  int64_t beg;
  int32_t deg;  // a row's degree fits 32 bits (the slots are addressed from beg)
  int mc;
  float mw;
  int ms;  // max adjoint (meta_first_m): fwd slot of the lane's edge
  int mv;  // packed table (meta_first_pk): word offset of the lane's edge's segment values
};

__device__ __forceinline__ void meta_rowptr(const int64_t *__restrict__ rowptr, int64_t row,
                                            bool ok, RowMeta &m) {
  m.beg = ok ? rowptr[row] : 0;
  m.deg = ok ? (int32_t)(rowptr[row + 1] - m.beg) : 0;
}

__device__ __forceinline__ void meta_first(const int32_t *__restrict__ col,
                                           const float *__restrict__ w, int gl, RowMeta &m) {
  m.mc = 0;
  m.mw = 1.0f;
  if (gl < m.deg) {
    m.mc = col[m.beg + gl];
    if (w != nullptr) m.mw = w[m.beg + gl];
  }
}

// meta_first plus the lane's edge's fwd slot (the max adjoint's slot_map)
__device__ __forceinline__ void meta_first_m(const int32_t *__restrict__ col,
                                             const float *__restrict__ w,
                                             const int32_t *__restrict__ slot_map, int gl,
                                             RowMeta &m) {
  meta_first(col, w, gl, m);
  m.ms = gl < m.deg ? slot_map[m.beg + gl] : 0;
}

template <int U>
__device__ __forceinline__ void gather_row_meta(const __amdgpu_buffer_rsrc_t rx, uint32_t ldx_b,
                                                const int32_t *__restrict__ col,
                                                const float *__restrict__ w, const RowMeta &m,
                                                int gl, int grp, float (&acc)[4]) {
  const int64_t beg = m.beg, deg = m.deg;
  const int64_t odeg = __shfl_xor(deg, 32, 64);
  const int64_t maxdeg = deg > odeg ? deg : odeg;
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0f;
  int mc = m.mc;
  float mw = m.mw;
  for (int64_t e0 = 0; e0 < maxdeg; e0 += 32) {
    if (e0 > 0) {  // rows longer than one metadata batch load the rest in place
      const int64_t my = e0 + gl;
      mc = 0;
      mw = 1.0f;
      if (my < deg) {
        mc = col[beg + my];
        if (w != nullptr) mw = w[beg + my];
      }
    }
    const int64_t rem = deg - e0;
    const int nb = rem <= 0 ? 0 : (rem < 32 ? (int)rem : 32);
    const int64_t remw = maxdeg - e0;
    const int nbmax = remw < 32 ? (int)remw : 32;  // wave-uniform
    for (int k0 = 0; k0 < nbmax; k0 += U) {
      float4 xv[U];
      float wk[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u;
        const int ck = bcast_g(mc, grp, k & 31);
        wk[u] = bcast_g(mw, grp, k & 31);
        ok[u] = k < nb;
        const uint32_t off = ok[u] ? (uint32_t)ck * ldx_b + 16u * gl : 0xfffffff0u;
        xv[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ok[u]) {
          acc[0] = __fadd_rn(acc[0], __fmul_rn(xv[u].x, wk[u]));
          acc[1] = __fadd_rn(acc[1], __fmul_rn(xv[u].y, wk[u]));
          acc[2] = __fadd_rn(acc[2], __fmul_rn(xv[u].z, wk[u]));
          acc[3] = __fadd_rn(acc[3], __fmul_rn(xv[u].w, wk[u]));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// In-place gather from a PACKED table at F = 128 (round 6; pack.hip's layout;
// fused_wide.hip's wide_gather2_pk is the 256-wide form).  The two lane groups
// of a wave walk different rows, so a row's address is per lane: the table is
// read through ONE buffer resource (every segment at a word offset below
// 2^29, the mgcn_spmm_xw_*_packed check), and the metadata loads turn a
// slot's packed col (s << rbits) | i into the word offsets of its row header
// (base[s] + 8 i) and of its segment's values (base[s] + head) -- base[]
// lane-resident, one ds_bpermute per 32 slots, not per slot.  Lane gl reads
// the header pair w = gl / 8 (8 B), then 16 B of values at pos_w +
// popc(mask_w below bit 4 (gl % 8)), expanded by pk_expand: the dense row's
// bits, so the fold is gather_row_meta's, bit for bit.  The headers of batch
// k + 1 (after a row's last batch: the next row's first) load under batch k's
// values, so a row costs the dense gather's round trips.
struct Pk128 {
  __amdgpu_buffer_rsrc_t r;  // the whole table
  uint32_t rbits, head;      // col = (s << rbits) | i; head = seg_rows * 8 words
  uint32_t base;             // lane-resident: base[lane], word offset of segment `lane`
};

// packed col -> (header word offset, value-area word offset); all lanes
// active (ds_bpermute), masked slots carry col 0
__device__ __forceinline__ void pk128_meta(const Pk128 &pk, int c, int &mh, int &mv) {
  const uint32_t s = (uint32_t)c >> pk.rbits;
  const uint32_t i = (uint32_t)c & ((1u << pk.rbits) - 1u);
  const uint32_t b = (uint32_t)__shfl((int)pk.base, (int)(s & 63u), 64);
  mh = (int)(b + 8u * i);
  mv = (int)(b + pk.head);
}

__device__ __forceinline__ void meta_first_pk(const Pk128 &pk, const int32_t *__restrict__ col,
                                              const float *__restrict__ w, int gl, RowMeta &m) {
  meta_first(col, w, gl, m);
  pk128_meta(pk, m.mc, m.mc, m.mv);
}

// the header pairs of slots k0 .. k0 + U - 1 of the group's row (slots past
// n: the "no load" offset, the pair reads 0 and its values are never read)
template <int U>
__device__ __forceinline__ void pk128_headers(const Pk128 &pk, int mh, int grp, int k0, int n,
                                              uint32_t hoff, u32x2 (&h)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = k0 + u;
    const uint32_t hk = (uint32_t)bcast_g(mh, grp, k & 31);
    h[u] = __builtin_amdgcn_raw_buffer_load_b64(pk.r, k < n ? 4u * hk + hoff : 0xfffffff0u, 0, 0);
  }
}

// gather_row_meta from a packed table: hh holds, on entry, the header pairs
// of the row's first U slots and, on return, those of row nx's
template <int U>
__device__ __forceinline__ void gather_row_meta_pk(const Pk128 &pk, const int32_t *__restrict__ col,
                                                   const float *__restrict__ w, const RowMeta &m,
                                                   const RowMeta &nx, int gl, int grp,
                                                   float (&acc)[4], u32x2 (&hh)[U]) {
  const int64_t beg = m.beg, deg = m.deg;
  const int64_t odeg = __shfl_xor(deg, 32, 64);
  const int64_t maxdeg = deg > odeg ? deg : odeg;
  // (two empty rows still run one all-masked batch: the next rows' headers
  // are issued from the one call site below)
  const int64_t maxdeg1 = maxdeg > 0 ? maxdeg : 1;
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0f;
  int mh = m.mc, mv = m.mv;
  float mw = m.mw;
  const uint32_t hoff = 8u * (uint32_t)(gl >> 3);
  const uint32_t sh = 4u * (uint32_t)(gl & 7);  // the lane's nibble in mask_w
  const uint32_t below = (1u << sh) - 1u;
  const int nn = nx.deg < 32 ? nx.deg : 32;
  for (int64_t e0 = 0; e0 < maxdeg1; e0 += 32) {
    const int64_t rem = deg - e0;
    const int nb = rem <= 0 ? 0 : (rem < 32 ? (int)rem : 32);
    const int64_t remw = maxdeg1 - e0;
    const int nbmax = remw < 32 ? (int)remw : 32;  // wave-uniform
    if (e0 > 0) {  // rows longer than one metadata batch load the rest in place
      const int64_t my = e0 + gl;
      int c = 0;
      mw = 1.0f;
      if (my < deg) {
        c = col[beg + my];
        if (w != nullptr) mw = w[beg + my];
      }
      pk128_meta(pk, c, mh, mv);
      pk128_headers<U>(pk, mh, grp, 0, nb, hoff, hh);
    }
    const bool last_window = e0 + 32 >= maxdeg1;
    for (int k0 = 0; k0 < nbmax; k0 += U) {
      u32x4 v[U];
      uint32_t nib[U];
      float wk[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u;
        wk[u] = bcast_g(mw, grp, k & 31);
        const uint32_t vk = (uint32_t)bcast_g(mv, grp, k & 31);
        nib[u] = (hh[u][0] >> sh) & 0xfu;
        const uint32_t q = hh[u][1] + (uint32_t)__builtin_popcount(hh[u][0] & below);
        // a lane with no nonzero word moves no bytes (offset past the range)
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(pk.r, nib[u] ? 4u * (vk + q) : 0xfffffff0u, 0, 0);
      }
      // the next headers, under these values: this window's next batch, or
      // (the last batch of the last window) row nx's first -- one call site
      const bool more = k0 + U < nbmax;
      if (more || last_window)
        pk128_headers<U>(pk, more ? mh : nx.mc, grp, more ? k0 + U : 0, more ? nb : nn, hoff, hh);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u < nb) {  // strictly ascending edge order (gather_row_meta)
          const float4 x = pk_expand(nib[u], v[u]);
          acc[0] = __fadd_rn(acc[0], __fmul_rn(x.x, wk[u]));
          acc[1] = __fadd_rn(acc[1], __fmul_rn(x.y, wk[u]));
          acc[2] = __fadd_rn(acc[2], __fmul_rn(x.z, wk[u]));
          acc[3] = __fadd_rn(acc[3], __fmul_rn(x.w, wk[u]));
        }
      }
    }
  }
}

// Two rows per lane group at once (the warp-specialised adjoint's gather
// waves): U slots of EACH row in flight per round, so a wave keeps four rows'
// gathers in flight; each row folded in its own edge order, products and
// sums rounded separately (gather_row_meta bit for bit).
template <int U, bool MAXM = false>
__device__ __forceinline__ void gather_row2_meta(const __amdgpu_buffer_rsrc_t rx, uint32_t ldx_b,
                                                 const int32_t *__restrict__ col,
                                                 const float *__restrict__ w, const RowMeta &ma,
                                                 const RowMeta &mb, int gl, int grp,
                                                 float (&aa)[4], float (&ab)[4],
                                                 const uint32_t *__restrict__ win = nullptr,
                                                 const int32_t *__restrict__ slot_map = nullptr) {
#pragma unroll
  for (int j = 0; j < 4; ++j) aa[j] = ab[j] = 0.0f;
  const int64_t da = ma.deg, db = mb.deg;
  int64_t dm = da > db ? da : db;
  const int64_t odm = __shfl_xor(dm, 32, 64);
  dm = dm > odm ? dm : odm;  // wave-uniform loop bound
  int mca = ma.mc, mcb = mb.mc;
  float mwa = ma.mw, mwb = mb.mw;
  int msa = 0, msb = 0;
  if constexpr (MAXM) {
    msa = ma.ms;
    msb = mb.ms;
  }
  for (int64_t e0 = 0; e0 < dm; e0 += 32) {
    if (e0 > 0) {  // rows longer than one metadata batch load the rest in place
      const int64_t my = e0 + gl;
      mca = mcb = 0;
      mwa = mwb = 1.0f;
      if (my < da) {
        mca = col[ma.beg + my];
        if (w != nullptr) mwa = w[ma.beg + my];
        if constexpr (MAXM) msa = slot_map[ma.beg + my];
      }
      if (my < db) {
        mcb = col[mb.beg + my];
        if (w != nullptr) mwb = w[mb.beg + my];
        if constexpr (MAXM) msb = slot_map[mb.beg + my];
      }
    }
    const int64_t ra = da - e0, rb = db - e0;
    const int na = ra <= 0 ? 0 : (ra < 32 ? (int)ra : 32);
    const int nb = rb <= 0 ? 0 : (rb < 32 ? (int)rb : 32);
    const int64_t remw = dm - e0;
    const int nbmax = remw < 32 ? (int)remw : 32;  // wave-uniform
    for (int k0 = 0; k0 < nbmax; k0 += U) {
      float4 xa[U], xb[U];
      float wa[U], wb[U];
      uint32_t ba[U], bb[U];  // MAXM: the edges' winner words (word gl / 8 of the record)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u;
        const int ca = bcast_g(mca, grp, k & 31);
        const int cb = bcast_g(mcb, grp, k & 31);
        wa[u] = bcast_g(mwa, grp, k & 31);
        wb[u] = bcast_g(mwb, grp, k & 31);
        const uint32_t oa = k < na ? (uint32_t)ca * ldx_b + 16u * gl : 0xfffffff0u;
        const uint32_t ob = k < nb ? (uint32_t)cb * ldx_b + 16u * gl : 0xfffffff0u;
        xa[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, oa, 0, 0));
        xb[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, ob, 0, 0));
        if constexpr (MAXM) {
          // loaded unconditionally (masked edges read word 0, never used)
          const int sa = bcast_g(msa, grp, k & 31);
          const int sb = bcast_g(msb, grp, k & 31);
          ba[u] = win[k < na ? (int64_t)sa * 4 + (gl >> 3) : 0];
          bb[u] = win[k < nb ? (int64_t)sb * 4 + (gl >> 3) : 0];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (MAXM) {  // each edge's dY counts only where it won (gather_row's select)
          const uint32_t qa = ba[u] >> (4 * (gl & 7)), qb = bb[u] >> (4 * (gl & 7));
          xa[u].x = (qa & 1u) ? xa[u].x : 0.0f;
          xa[u].y = (qa & 2u) ? xa[u].y : 0.0f;
          xa[u].z = (qa & 4u) ? xa[u].z : 0.0f;
          xa[u].w = (qa & 8u) ? xa[u].w : 0.0f;
          xb[u].x = (qb & 1u) ? xb[u].x : 0.0f;
          xb[u].y = (qb & 2u) ? xb[u].y : 0.0f;
          xb[u].z = (qb & 4u) ? xb[u].z : 0.0f;
          xb[u].w = (qb & 8u) ? xb[u].w : 0.0f;
        }
        if (k0 + u < na) {
          aa[0] = __fadd_rn(aa[0], __fmul_rn(xa[u].x, wa[u]));
          aa[1] = __fadd_rn(aa[1], __fmul_rn(xa[u].y, wa[u]));
          aa[2] = __fadd_rn(aa[2], __fmul_rn(xa[u].z, wa[u]));
          aa[3] = __fadd_rn(aa[3], __fmul_rn(xa[u].w, wa[u]));
        }
        if (k0 + u < nb) {
          ab[0] = __fadd_rn(ab[0], __fmul_rn(xb[u].x, wb[u]));
          ab[1] = __fadd_rn(ab[1], __fmul_rn(xb[u].y, wb[u]));
          ab[2] = __fadd_rn(ab[2], __fmul_rn(xb[u].z, wb[u]));
          ab[3] = __fadd_rn(ab[3], __fmul_rn(xb[u].w, wb[u]));
        }
      }
    }
  }
}

// The row sequence of one lane group in the chunk loop: row k is slot
// 16 (k & 1) + 2 wave + grp of the workgroup's chunk k >> 1 (chunks
// blockIdx.x + i gridDim.x).  Used by the forward (-2.5 %) and the dX-only
// backward (-0.5 %); the dW + dX backward has no registers to spare for the
// extra state (its spills cost more).
struct RowSeq {
  int64_t base;  // blockIdx.x * 32 + 2 wave + grp
  int64_t step;  // gridDim.x * 32
  int64_t n_rows;
  __device__ __forceinline__ int64_t row(int64_t k) const { return base + (k >> 1) * step + 16 * (k & 1); }
};

// chunks of this workgroup in a grid-stride chunk loop
__device__ __forceinline__ int64_t my_chunks(int64_t n_chunks) {
  return blockIdx.x < n_chunks ? (n_chunks - 1 - blockIdx.x) / gridDim.x + 1 : 0;
}

// One row's four features -> its three bf16 term images (lane gl of the group)
__device__ __forceinline__ void store_row_terms(char *img_base, int lr, int gl, const float (&v)[4]) {
  uint32_t hi[2], mid[2], lo[2];
  split3_pair(f32x2{v[0], v[1]}, hi[0], mid[0], lo[0]);
  split3_pair(f32x2{v[2], v[3]}, hi[1], mid[1], lo[1]);
  char *img = img_base + img_off(lr, gl >> 1) + 8 * (gl & 1);
  *reinterpret_cast<uint2 *>(img) = make_uint2(hi[0], hi[1]);
  *reinterpret_cast<uint2 *>(img + kXwImg) = make_uint2(mid[0], mid[1]);
  *reinterpret_cast<uint2 *>(img + 2 * kXwImg) = make_uint2(lo[0], lo[1]);
}

// 16x16x32 products of the chunk's 32 rows (A image at `img`) with this
// wave's 16 columns of B (fragments in registers): acc[t] = rows 16 t + 4 g4 + r
__device__ __forceinline__ void mfma_rows(const char *img, const bf16x8 (&b)[3], int ks, int l16,
                                          int g4, f32x4_t (&acc)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int off = img_off(16 * t + l16, 4 * ks + g4);
    const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(img + off);
    const bf16x8 am = *reinterpret_cast<const bf16x8 *>(img + kXwImg + off);
    const bf16x8 al = *reinterpret_cast<const bf16x8 *>(img + 2 * kXwImg + off);
    acc[t] = mfma16_x6(ah, am, al, b[0], b[1], b[2], acc[t]);
  }
}

// ---------------------------------------------------------------------------
// Forward.  LDS: two image sets and two fp32 staging tiles, double-buffered
// so that one barrier per chunk orders everything: chunk c's images are
// written before barrier c and read after it; its output rows are staged
// after barrier c and written out after barrier c + 1.  80 KB: two per CU.
constexpr int kXfBuf = 3 * kXwImg;
constexpr int kXfStageOff = 2 * kXfBuf;
constexpr int kXfLds = kXfStageOff + 2 * kXfStage;
static_assert(2 * kXfLds <= 160 * 1024, "two forward workgroups per CU");

struct XwArgs {
  int64_t n_rows;
  const int64_t *rowptr;
  const int32_t *col;
  const float *w;     // per-slot weights, nullable
  const float *X;     // gathered rows [n_cols][128]
  int64_t ldx;
  int64_t n_cols;
  const float *W;     // [128][128], Y = Z W
  int64_t ldw;
  const float *bias;  // nullable
  float *Y;
  int64_t ldy;
  uint32_t *relu_mask;  // nullable; [n_rows][4], bit b of word v <=> Y[row][4 b + v] > 0
  float *Z;             // nullable; the aggregated rows before W (and before mean's division)
  int64_t ldz;
  int mean;
  int relu;
  // packed table (PK kernels; mgcn_spmm_xw_fwd_packed): X unused
  const uint32_t *pk;
  uint32_t pk_bytes, pk_rbits, pk_head;
  uint32_t pk_base[64];
};

template <int U, bool PK = false>
__global__ __launch_bounds__(kXwThreads, 2 * kXwPerCU) void spmm_xw_fwd_kernel(const XwArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[kXfLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gl = lane & 31, grp = lane >> 5;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int64_t n_chunks = (a.n_rows + kXwRows - 1) / kXwRows;
  const bool has_b = a.bias != nullptr;
  // gathers through one buffer resource over X: 32-bit offsets, 1 VGPR each
  const auto rx = buf_rsrc(PK ? nullptr : a.X, PK ? 0u : (uint32_t)(a.n_cols * a.ldx * 4));
  const uint32_t ldx_b = (uint32_t)a.ldx * 4u;
  Pk128 pk{};
  u32x2 hh[PK ? U : 1];
  if constexpr (PK) {
    pk.r = buf_rsrc(a.pk, a.pk_bytes);
    pk.rbits = a.pk_rbits;
    pk.head = a.pk_head;
    pk.base = a.pk_base[lane];
  }

  // W fragments of this wave's 16 output columns: B[k][n] = W[k][n], lane
  // (g4, l16) holds k = 32 ks + 8 g4 + j of column n = 16 wave + l16
  const int ncol = 16 * wave + l16;
  bf16x8 wb[4][3];
  {
    const float *wp = a.W + (int64_t)(8 * g4) * a.ldw + ncol;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = wp[(int64_t)(32 * ks + j) * a.ldw];
      split3_bf16(v, wb[ks][0], wb[ks][1], wb[ks][2]);
    }
  }
  const float bcol = has_b ? a.bias[ncol] : 0.0f;

  // staged rows of chunk `c` -> Y (thread: rows tid >> 5 and 16 + (tid >> 5),
  // float4 gl), and the ReLU mask words of each row from four ballots
  auto flush = [&](int64_t c, const float *stage) {
    const int64_t r0 = c * kXwRows;
    const int64_t left = a.n_rows - r0;
    const uint32_t rows_in = (uint32_t)(left >= kXwRows ? kXwRows : left);
    const auto ry = buf_rsrc(a.Y + r0 * a.ldy, rows_in * (uint32_t)a.ldy * 4u);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int lr = 16 * m + (tid >> 5);
      const float4 v = *reinterpret_cast<const float4 *>(stage + lr * kXwF + 4 * gl);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ry,
                                             4 * (int)(lr * a.ldy + 4 * gl), 0, MGCN_NT_OUT);
      if (a.relu_mask != nullptr) {
        // word j of the row: bit gl <=> feature 4 gl + j > 0 (the SpMM's layout)
        const uint32_t m0 = (uint32_t)(__ballot(v.x > 0.0f) >> (32 * grp));
        const uint32_t m1 = (uint32_t)(__ballot(v.y > 0.0f) >> (32 * grp));
        const uint32_t m2 = (uint32_t)(__ballot(v.z > 0.0f) >> (32 * grp));
        const uint32_t m3 = (uint32_t)(__ballot(v.w > 0.0f) >> (32 * grp));
        if (gl == 0 && (uint32_t)lr < rows_in)
          *reinterpret_cast<uint4 *>(a.relu_mask + (r0 + lr) * 4) = make_uint4(m0, m1, m2, m3);
      }
    }
  };

  const int64_t n_my = my_chunks(n_chunks);
  const RowSeq seq{(int64_t)blockIdx.x * kXwRows + 2 * wave + grp, (int64_t)gridDim.x * kXwRows,
                   a.n_rows};
  RowMeta cur, nxt;
  meta_rowptr(a.rowptr, seq.row(0), seq.row(0) < a.n_rows, cur);
  if constexpr (PK) {
    meta_first_pk(pk, a.col, a.w, gl, cur);
    pk128_headers<U>(pk, cur.mc, grp, 0, cur.deg < 32 ? cur.deg : 32, 8u * (uint32_t)(gl >> 3), hh);
  } else {
    meta_first(a.col, a.w, gl, cur);
  }
  meta_rowptr(a.rowptr, seq.row(1), seq.row(1) < a.n_rows, nxt);
  int it = 0;
  for (int64_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x, ++it) {
    char *buf = lds + (it & 1) * kXfBuf;
    float *stage = reinterpret_cast<float *>(lds + kXfStageOff + (it & 1) * kXfStage);

    // ---- Phase A: aggregate the chunk's rows into the bf16 images --------
#pragma unroll 1
    for (int p = 0; p < 2; ++p) {
      const int lr = 16 * p + 2 * wave + grp;
      const int64_t k = 2 * it + p;
      if constexpr (PK)
        meta_first_pk(pk, a.col, a.w, gl, nxt);
      else
        meta_first(a.col, a.w, gl, nxt);
      RowMeta nn;
      const int64_t r2 = seq.row(k + 2);
      meta_rowptr(a.rowptr, r2, r2 < a.n_rows && k + 2 < 2 * n_my, nn);
      float acc[4];
      if constexpr (PK)
        gather_row_meta_pk<U>(pk, a.col, a.w, cur, nxt, gl, grp, acc, hh);
      else
        gather_row_meta<U>(rx, ldx_b, a.col, a.w, cur, gl, grp, acc);
      if (a.Z != nullptr) {
        // the aggregate the backward's dW = Z^T dY reads (whole 512-B rows;
        // rows past the end fall outside the chunk's buffer range)
        const int64_t r0 = chunk * kXwRows;
        const int64_t left = a.n_rows - r0;
        const uint32_t rows_in = (uint32_t)(left >= kXwRows ? kXwRows : left);
        const auto rz = buf_rsrc(a.Z + r0 * a.ldz, rows_in * (uint32_t)a.ldz * 4u);
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, make_float4(acc[0], acc[1], acc[2], acc[3])), rz,
            4 * (int)(lr * a.ldz + 4 * gl), 0, MGCN_NT_AUX);
      }
      if (a.mean) {
        const float c = (float)(cur.deg > 1 ? cur.deg : 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __fdiv_rn(acc[j], c);
      }
      store_row_terms(buf, lr, gl, acc);
      cur = nxt;
      nxt = nn;
    }
    __syncthreads();
    // the previous chunk's output rows (staged before this barrier) go out
    if (it > 0)
      flush(chunk - gridDim.x, reinterpret_cast<const float *>(lds + kXfStageOff +
                                                                ((it + 1) & 1) * kXfStage));

    // ---- Phase B: Y = Z W (+ b), ReLU -> staging tile ----------------------
    f32x4_t acc2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc2[t][r] = 0.0f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) mfma_rows(buf, wb[ks], ks, l16, g4, acc2);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc2[t][r];
        if (has_b) v = __fadd_rn(v, bcol);
        if (a.relu) v = (v < 0.0f) ? 0.0f : v;
        stage[(16 * t + 4 * g4 + r) * kXwF + ncol] = v;
      }
  }
  if (it > 0) {
    __syncthreads();
    flush(blockIdx.x + (int64_t)(it - 1) * gridDim.x,
          reinterpret_cast<const float *>(lds + kXfStageOff + ((it + 1) & 1) * kXfStage));
  }
}

// ---------------------------------------------------------------------------
// Backward.  LDS: X images, dH images (single-buffered: two barriers per
// chunk), the chunk's mask / divisor words, the dX staging tile.  dX: wave w
// owns columns 16 w .. +15; its W^T fragments are re-read from L2 (W is
// 64 KB) and split per chunk -- held for the whole kernel they would take 48
// VGPRs beside the gather's and dW's (the dX-only form, DW = false, holds
// them: it has no dW accumulators).
constexpr int kXbHOff = 3 * kXwImg;
constexpr int kXbMaskOff = 6 * kXwImg;                 // [32][4] mask words
constexpr int kXbDivOff = kXbMaskOff + kXwRows * 16;   // [32] row divisors
constexpr int kXbStageOff = kXbDivOff + kXwRows * 4;
constexpr int kXbColsumOff = kXbStageOff + kXwStage;     // [512 threads][4] column sums
constexpr int kXbLds = kXbColsumOff + kXwThreads * 16;
static_assert(2 * kXbLds <= 160 * 1024, "two backward workgroups per CU");

struct XbArgs {
  int64_t n_rows;  // source nodes: rows of the bwd view, of X and of dX
  const int64_t *rowptr;
  const int32_t *col;
  const float *w;
  const float *row_scale;  // nullable ('rw')
  const float *dY;         // gathered rows [n_cols][128]
  int64_t lddy;
  int64_t n_cols;
  const float *X;  // layer input [n_rows][128]
  int64_t ldx;
  const float *W;  // [128][128], H = X W
  int64_t ldw;
  float *dX;  // nullable
  int64_t lddx;
  const uint32_t *relu_mask;  // lower layer's output > 0 (mgcn_spmm_fwd layout)
  const float *row_div;
  float *dw_partial;      // [grid][128][128]
  float *colsum_partial;  // [grid][128]
  const uint32_t *win_mask;  // max adjoint: winner bits per fwd slot ([nnz][4])
  const int32_t *slot_map;   // max adjoint: fwd slot of every bwd slot
  // packed dY (dX-only PK kernel; mgcn_spmm_xw_bwd_packed): dY unused
  const uint32_t *pk;
  uint32_t pk_bytes, pk_rbits, pk_head;
  uint32_t pk_base[64];
};

#ifdef MGCN_XW_PROFILE
// phase timestamps of workgroup 0, waves 0 and 7 (scripts/prof_fused.py):
// [wave][chunk iteration][stamp]
__device__ unsigned long long g_xprof[2][64][6];
#define XPROF(it, k)                                                                      \
  if (blockIdx.x == 0 && (wave == 0 || wave == 7) && (it) < 64 && lane == 0)              \
    g_xprof[wave == 7][it][k] = __builtin_readcyclecounter();
#else
#define XPROF(it, k)
#endif

// DW = false: dX only (X == NULL) -- the caller forms dW = Z^T dY from the
// forward's aggregate (mgcn_gemm_bwd, dW-only), so the chunk's X rows, their
// images and the dW MFMAs drop out.
template <int U, bool DX, int EPI, bool MAXM, bool DW = true, bool PK = false>
__global__ __launch_bounds__(kXwThreads, 2 * kXwPerCU) void spmm_xw_bwd_kernel(const XbArgs a) {
  static_assert(!PK || (!DW && !MAXM), "the packed gather serves the dX-only adjoint");
  __shared__ __attribute__((aligned(16))) char lds[kXbLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gl = lane & 31, grp = lane >> 5;
  const int h = lane >> 5, lc = lane & 31;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int64_t n_chunks = (a.n_rows + kXwRows - 1) / kXwRows;
  const auto rdy = buf_rsrc(PK ? nullptr : a.dY, PK ? 0u : (uint32_t)(a.n_cols * a.lddy * 4));
  const uint32_t ldy_b = (uint32_t)a.lddy * 4u;
  Pk128 pk{};
  u32x2 hh[PK ? U : 1];
  if constexpr (PK) {
    pk.r = buf_rsrc(a.pk, a.pk_bytes);
    pk.rbits = a.pk_rbits;
    pk.head = a.pk_head;
    pk.base = a.pk_base[lane];
  }
  float *stage = reinterpret_cast<float *>(lds + kXbStageOff);
  const float *wp = a.W + (int64_t)(16 * wave + l16) * a.ldw + 8 * g4;  // B[k][n] = W[n][k]

  // dW fragment offsets (gemm_bwd mapping): lane = 16 g + 4 q + p reads
  // row 8 h + q (+ 4) of chunk (col0 >> 3) + 2 (g & 1) + (p >> 1), half p & 1
  const int q = (lane >> 2) & 3, p4 = lane & 3;
  auto frag_off = [&](int col0, int second) {
    return img_off(8 * h + q + 4 * second, (col0 >> 3) + 2 * (g4 & 1) + (p4 >> 1)) + 8 * (p4 & 1);
  };
  const int ti = wave >> 1, tj0 = 2 * (wave & 1);
  int offa[2], offb[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    offa[r] = frag_off(32 * ti, r);
    offb[0][r] = kXbHOff + frag_off(32 * tj0, r);
    offb[1][r] = kXbHOff + frag_off(32 * (tj0 + 1), r);
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
  const int ncol = 16 * wave + l16;  // dX column of this lane
  const int xoff = 4 * (int)((tid >> 5) * a.ldx + 4 * (tid & 31));
  // dX only: no dW accumulators, so this wave's W^T fragments are split once
  // and held (48 VGPRs) instead of re-read from L2 every chunk
  bf16x8 wt[DW ? 1 : 4][3];
  if constexpr (!DW) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float4 w0 = *reinterpret_cast<const float4 *>(wp + 32 * ks);
      const float4 w1 = *reinterpret_cast<const float4 *>(wp + 32 * ks + 4);
      const float v[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      split3_bf16(v, wt[ks][0], wt[ks][1], wt[ks][2]);
    }
  }

  // staged dX rows of chunk `c` -> dX (16 B per lane, whole rows)
  // The ReLU mask, the bias column sums and mean's division are applied here,
  // on whole staged rows, rather than in the MFMA epilogue (whose registers
  // are the kernel's peak): thread (q, lc) owns features 4 lc .. 4 lc + 3 of
  // rows q and 16 + q; feature 4 lc + j is bit lc of the row's mask word j.
  // column sums of this thread's features, kept in LDS (registers are the
  // kernel's limit)
  float *cs = reinterpret_cast<float *>(lds + kXbColsumOff) + 4 * tid;
  if constexpr (DX && EPI != EPI_STORE)
    *reinterpret_cast<float4 *>(cs) = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  auto flush = [&](int64_t c) {
    const int64_t r0 = c * kXwRows;
    const int64_t left = a.n_rows - r0;
    const uint32_t rows_in = (uint32_t)(left >= kXwRows ? kXwRows : left);
    const auto rx = buf_rsrc(a.dX + r0 * a.lddx, rows_in * (uint32_t)a.lddx * 4u);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int lr = 16 * m + (tid >> 5);
      const float *srow = stage + lr * kXwStageLd;
      float v[4];
      *reinterpret_cast<float4 *>(v) = *reinterpret_cast<const float4 *>(srow + 4 * lc);
      if constexpr (EPI != EPI_STORE) {
        const u32x4 mw = *reinterpret_cast<const u32x4 *>(srow + kXwF);
        // rows past the end were staged from zero dH rows with zero mask words
        float c[4];
        *reinterpret_cast<float4 *>(c) = *reinterpret_cast<const float4 *>(cs);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = ((mw[j] >> lc) & 1u) ? v[j] : 0.0f;
          c[j] = __fadd_rn(c[j], v[j]);
        }
        *reinterpret_cast<float4 *>(cs) = *reinterpret_cast<const float4 *>(c);
        if constexpr (EPI == EPI_RELU_DIV) {
          const float d = srow[kXwF + 4];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = __fdiv_rn(v[j], d);
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, *reinterpret_cast<float4 *>(v)),
                                             rx, 4 * (int)(lr * a.lddx + 4 * lc), 0, MGCN_NT_OUT);
    }
  };

  // dX only: the row metadata runs one row ahead as in the forward
  // (gather_row_meta: row k + 1's first edge slots and row k + 2's pointers
  // load under row k's gathers)
  const int64_t n_my = my_chunks(n_chunks);
  const RowSeq seq{(int64_t)blockIdx.x * kXwRows + 2 * wave + grp, (int64_t)gridDim.x * kXwRows,
                   a.n_rows};
  RowMeta cur{}, nxt{};
  if constexpr (!DW && !MAXM) {
    meta_rowptr(a.rowptr, seq.row(0), seq.row(0) < a.n_rows, cur);
    if constexpr (PK) {
      meta_first_pk(pk, a.col, a.w, gl, cur);
      pk128_headers<U>(pk, cur.mc, grp, 0, cur.deg < 32 ? cur.deg : 32, 8u * (uint32_t)(gl >> 3), hh);
    } else {
      meta_first(a.col, a.w, gl, cur);
    }
    meta_rowptr(a.rowptr, seq.row(1), seq.row(1) < a.n_rows, nxt);
  }
  int it = 0;
  for (int64_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x, ++it) {
    const int64_t r0 = chunk * kXwRows;
    const int64_t left = a.n_rows - r0;
    const uint32_t rows_in = (uint32_t)(left >= kXwRows ? kXwRows : left);
    XPROF(it, 0);
    if constexpr (DX) {
      if (it > 0) flush(chunk - gridDim.x);
    }
    // the chunk's X rows (q and 16 + q, float4 tid & 31), issued first so
    // they land under the gathers
    u32x4 xa{}, xb{};
    if constexpr (DW) {
      const auto rxx = buf_rsrc(a.X + r0 * a.ldx, rows_in * (uint32_t)a.ldx * 4u);
      xa = __builtin_amdgcn_raw_buffer_load_b128(rxx, xoff, 0, MGCN_NT_AUX);
      xb = __builtin_amdgcn_raw_buffer_load_b128(rxx, xoff + 64 * (int)a.ldx, 0, MGCN_NT_AUX);
    }
    // the chunk's mask / divisor words straight into LDS (LDS-DMA: no registers
    // held across the gathers); rows past the end read row r0 and are never used
    if constexpr (DX && EPI != EPI_STORE) {
      if (wave == 0 && h == 0) {
        const int64_t mr = r0 + ((uint32_t)lc < rows_in ? lc : 0);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a.relu_mask + mr * 4),
                                         (lds_void_t *)(lds + kXbMaskOff), 16, 0, 0);
        if constexpr (EPI == EPI_RELU_DIV)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a.row_div + mr),
                                           (lds_void_t *)(lds + kXbDivOff), 4, 0, 0);
      }
    }

    // ---- Phase A: dH rows of the chunk -> bf16 images; X rows -> images --
#pragma unroll 1
    for (int p = 0; p < 2; ++p) {
      const int lr = 16 * p + 2 * wave + grp;
      const int64_t row = r0 + lr;
      const bool row_ok = row < a.n_rows;
      int deg;
      float acc[4];
      if constexpr (!DW && !MAXM) {
        const int64_t k = 2 * it + p;
        if constexpr (PK)
          meta_first_pk(pk, a.col, a.w, gl, nxt);
        else
          meta_first(a.col, a.w, gl, nxt);
        RowMeta nn;
        const int64_t rk2 = seq.row(k + 2);
        meta_rowptr(a.rowptr, rk2, rk2 < a.n_rows && k + 2 < 2 * n_my, nn);
        if constexpr (PK)
          gather_row_meta_pk<U>(pk, a.col, a.w, cur, nxt, gl, grp, acc, hh);
        else
          gather_row_meta<U>(rdy, ldy_b, a.col, a.w, cur, gl, grp, acc);
        cur = nxt;
        nxt = nn;
      } else {
        gather_row<U, MAXM>(rdy, ldy_b, a.rowptr, a.col, a.w, row, row_ok, gl, grp, acc, deg,
                            a.win_mask, a.slot_map);
      }
      if (a.row_scale != nullptr && row_ok) {
        const float sc = a.row_scale[row];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __fmul_rn(acc[j], sc);
      }
      store_row_terms(lds + kXbHOff, lr, gl, acc);
    }
    XPROF(it, 1);
    if constexpr (DW) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const float4 v = __builtin_bit_cast(float4, m == 0 ? xa : xb);
        const float f[4] = {v.x, v.y, v.z, v.w};
        store_row_terms(lds, 16 * m + (tid >> 5), lc, f);
      }
    }
    // the mask / divisor LDS-DMA (older than this wave's gathers) has landed
    if constexpr (DX && EPI != EPI_STORE)
      if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // this wave's W^T fragments (B[k][n] = W[n][k], 32 floats per lane): issued
    // before the barrier, so the L2 round trip (thousands of cycles while the
    // other workgroup's gathers load the memory system) is hidden by the
    // barrier wait and the dW MFMAs
    float4 wr[4][2];
    if constexpr (DX && DW) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) wr[ks][j] = *reinterpret_cast<const float4 *>(wp + 32 * ks + 4 * j);
    }
    __syncthreads();
    XPROF(it, 2);

    // ---- Phase B1: dW += X^T dH (two 16-row k-steps) ---------------------
#pragma unroll
    for (int ks = 0; ks < (DW ? 2 : 0); ++ks) {
      const char *kb = lds + ks * 16 * 256;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[3], fb[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          fa[t] = read8(kb + t * kXwImg, offa);
          fb[t] = read8(kb + t * kXwImg, offb[s]);
        }
        accw[s] = mfma_x6(fa[0], fa[1], fa[2], fb[0], fb[1], fb[2], accw[s]);
      }
    }
    XPROF(it, 3);
    // ---- Phase B2: dX = relu'(lower) (dH W^T) [/ row_div] -> staging ------
    if constexpr (DX) {
      f32x4_t acc2[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc2[t][r] = 0.0f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if constexpr (DW) {
          bf16x8 wb[3];
          const float v[8] = {wr[ks][0].x, wr[ks][0].y, wr[ks][0].z, wr[ks][0].w,
                              wr[ks][1].x, wr[ks][1].y, wr[ks][1].z, wr[ks][1].w};
          split3_bf16(v, wb[0], wb[1], wb[2]);
          mfma_rows(lds + kXbHOff, wb, ks, l16, g4, acc2);
        } else {
          mfma_rows(lds + kXbHOff, wt[ks], ks, l16, g4, acc2);
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) stage[(16 * t + 4 * g4 + r) * kXwStageLd + ncol] = acc2[t][r];
      if constexpr (EPI != EPI_STORE) {
        // the chunk's mask words (and divisors) travel with the staged rows
        if (wave == 0 && h == 0) {
          *reinterpret_cast<u32x4 *>(stage + lc * kXwStageLd + kXwF) =
              *reinterpret_cast<const u32x4 *>(lds + kXbMaskOff + 16 * lc);
          if constexpr (EPI == EPI_RELU_DIV)
            stage[lc * kXwStageLd + kXwF + 4] = *reinterpret_cast<const float *>(lds + kXbDivOff + 4 * lc);
        }
      }
    }
    XPROF(it, 4);
    __syncthreads();
    XPROF(it, 5);
  }
  if constexpr (DX) {
    if (it > 0) flush(blockIdx.x + (int64_t)(it - 1) * gridDim.x);  // staged before the last barrier
  }

  // dW partial slab of this workgroup; C map: col = lc, row = (r & 3) + 8 (r >> 2) + 4 h
  float *slab = a.dw_partial + (int64_t)blockIdx.x * kXwF * kXwF;
#pragma unroll
  for (int s = 0; s < (DW ? 2 : 0); ++s)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * ti + (r & 3) + 8 * (r >> 2) + 4 * h;
      slab[row * kXwF + 32 * (tj0 + s) + lc] = accw[s][r];
    }
  if constexpr (DX && EPI != EPI_STORE) {
    // fold the 16 row slots of each column in fixed order: thread (q, lc)
    // holds features 4 lc .. 4 lc + 3 at cs slot 32 q + lc
    __syncthreads();
    const float *red = reinterpret_cast<const float *>(lds + kXbColsumOff);
    if (tid < kXwF) {
      float c = 0.0f;
#pragma unroll
      for (int q = 0; q < 16; ++q) c = __fadd_rn(c, red[4 * (32 * q + (tid >> 2)) + (tid & 3)]);
      a.colsum_partial[(int64_t)blockIdx.x * kXwF + tid] = c;
    }
  }
}

int g_xw_unroll = 5;  // forward gathers in flight per row (5: config 2 5.06 -> 5.005 ms/step; 6 spills)
// packed-table forms: slots in flight per row (experiment builds sweep them;
// config 2's shape, profiles/r06/packed_unroll_sweep.json: forward 1.20 / 1.27
// / 1.39 / 1.41 ms at U = 3 / 4 / 5 / 6 -- the extra registers spill more as U
// grows --, adjoint 1.07 / 1.05 / 1.08 ms at 2 / 3 / 4)
int g_xw_pk_unroll = 3;
int g_xw_pk_bwd_unroll = 3;

int xw_grid() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return kXwPerCU * cus;
}

template <int U, bool PK = false>
int launch_xw(const XwArgs &a, hipStream_t s) {
  const int64_t n_chunks = (a.n_rows + kXwRows - 1) / kXwRows;
  int64_t grid = xw_grid();
  if (grid > n_chunks) grid = n_chunks;
  hipLaunchKernelGGL((spmm_xw_fwd_kernel<U, PK>), dim3((unsigned)grid), dim3(kXwThreads), 0, s, a);
  return check_launch("spmm_xw_fwd_kernel");
}

template <int U, bool DX, int EPI, bool MAXM, bool DW = true, bool PK = false>
int launch_xb(const XbArgs &a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((spmm_xw_bwd_kernel<U, DX, EPI, MAXM, DW, PK>), dim3((unsigned)grid),
                     dim3(kXwThreads), 0, s, a);
  return check_launch("spmm_xw_bwd_kernel");
}

// dX only (no X, no dW), sum adjoint
template <int U, bool PK = false>
int launch_xb_dx(const XbArgs &a, int epi, int grid, hipStream_t s) {
  if (epi == EPI_RELU_DIV) return launch_xb<U, true, EPI_RELU_DIV, false, false, PK>(a, grid, s);
  if (epi == EPI_RELU) return launch_xb<U, true, EPI_RELU, false, false, PK>(a, grid, s);
  return launch_xb<U, true, EPI_STORE, false, false, PK>(a, grid, s);
}

template <int U, bool MAXM>
int launch_xb_m(const XbArgs &a, int epi, int grid, hipStream_t s) {
  if (a.dX == nullptr) return launch_xb<U, false, EPI_STORE, MAXM>(a, grid, s);
  if (epi == EPI_RELU_DIV) return launch_xb<U, true, EPI_RELU_DIV, MAXM>(a, grid, s);
  if (epi == EPI_RELU) return launch_xb<U, true, EPI_RELU, MAXM>(a, grid, s);
  return launch_xb<U, true, EPI_STORE, MAXM>(a, grid, s);
}

template <int U>
int launch_xb_u(const XbArgs &a, int epi, int grid, hipStream_t s) {
  return a.win_mask != nullptr ? launch_xb_m<U, true>(a, epi, grid, s)
                               : launch_xb_m<U, false>(a, epi, grid, s);
}

// ===================== warp-specialised adjoint (round 5) =====================
//
// DWS: the layer's whole adjoint re-cut by role as fused_wide.hip's F = 256
// kernels (dW = X^T dH and dX = relu'(lower) (dH W^T) [/ row_div], dH =
// A^T dY [* rs] never leaving the chip):
//
// One 1024-thread workgroup per CU: 8 GATHER waves aggregate dH rows (two
// 32-lane groups per wave, gather_row_meta's edge order: bit for bit the
// SpMM's adjoint), write them as bf16 term images into a ring of two chunk
// buffers and load the chunk's own X rows (fp32) beside them under the
// gathers; 8 MFMA waves form the chunk's dX (W^T as the A operand from an LDS
// copy of W: a lane's fragment is 4 consecutive columns of one row, one 16-B
// store; the same six products in the same order as the two-phase kernel, so
// dX is bit for bit its result), apply the epilogue, and fold their two 32x32
// tiles of X^T dH straight from the ring -- one 128 x 128 partial per
// workgroup over a one-workgroup-per-CU split-K grid, folded in workgroup
// order.  Hand-offs: LDS counters as in fused_wide.hip (bounded spins, abort
// word, reported through the device error word).  (The dX-only form of this
// kernel and DWL -- the lower layer's dW fused into the dX-only adjoint --
// measured slower than the two-phase kernel / the separate dW pass, round 5,
// and are removed.)
constexpr int kBsDws = 2, kBsDwsH = 3, kBsDwsM = 4;  // spmm_xw_bwd_ws_kernel MODE
#ifndef MGCN_DS_MASK_RING
#define MGCN_DS_MASK_RING 1  // DWS: ReLU mask words / divisors through the ring (0: MFMA waves load them)
#endif
constexpr int kBsImgSet = 3 * kXwImg;          // dH's three term images: 24 KB
// Layout: a ring of two (dH term images + X fp32 rows) chunk buffers and
// W in fp32 (rows padded to 528 B: the 16 rows of a W^T fragment read and the
// two row halves of an X^T fragment read fall on distinct banks); the MFMA
// waves split W^T and X^T fragments as they read them
constexpr int kDsXLd = kXwF + 4;                    // floats per padded row
constexpr int kDsXOff = kBsImgSet;                  // X rows within a ring buffer
constexpr int kDsMaskOff = kDsXOff + kXwRows * kDsXLd * 4;  // [32][4] mask words
constexpr int kDsDivOff = kDsMaskOff + kXwRows * 16;         // [32] row divisors
constexpr int kDsRingBuf = kDsDivOff + kXwRows * 4;
constexpr int kDsWOff = 2 * kDsRingBuf;
constexpr int kDsCtrOff = kDsWOff + kXwF * kDsXLd * 4;
constexpr int kDsLds = kDsCtrOff + 64;
static_assert(kDsLds <= 160 * 1024, "one DWS workgroup per CU");
static_assert(16 * kXwF * 4 <= kDsWOff, "column-sum fold fits in the ring");
constexpr int kBsNG = 8, kBsNM = 8;
constexpr int kBsThreads = 64 * (kBsNG + kBsNM);

__device__ __forceinline__ int bs_lds_load(const int *p) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

__device__ __forceinline__ bool bs_wait_ge(const int *p, int target, int *abort_word,
                                           uint32_t limit) {
  for (uint32_t n = 0;; ++n) {
    if (bs_lds_load(p) >= target) break;
    if (bs_lds_load(abort_word) != 0) return false;
    if (n >= limit) {
      __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
  return true;
}

__device__ __forceinline__ int bs_signal(int *p, int v, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(old);
}

// the two-phase kernel's six products (dH_l W_h, dH_h W_l, dH_m W_m, dH_m W_h,
// dH_h W_m, dH_h W_h) with W^T as the A operand
__device__ __forceinline__ f32x4_t mfma16_x6_at(const bf16x8 (&w)[3], const bf16x8 &xh,
                                               const bf16x8 &xm, const bf16x8 &xl, f32x4_t c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], xh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], xm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], xh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xh, c, 0, 0, 0);
}

struct XbsArgs {
  XbArgs b;             // rowptr .. colsum_partial; X, dw_partial: [grid][128][128]
  float *hcs_partial;   // DWS (nullable): [grid][128] column sums of dY's own rows
  int dbg;              // xw_ws_dbg (experiment builds only; masked by kDbgMask)
  uint32_t spin;        // hand-off spin bound (g_spin_limit)
  unsigned *err;        // device error word: kDevErrDws when a hand-off gave up
};

template <int U, int EPI, int MODE>
__global__ __launch_bounds__(kBsThreads) void spmm_xw_bwd_ws_kernel(const XbsArgs A) {
  constexpr bool HCS = MODE == kBsDwsH;  // DWS + dY's column sums (hcs_partial)
  constexpr bool MAXM = MODE == kBsDwsM;  // DWS on the max adjoint (win_mask + slot_map)
  constexpr bool MRING = MGCN_DS_MASK_RING;
  constexpr int kRing = kDsRingBuf;
  // The max adjoint keeps the timing switches' runtime branches in the
  // product too (A.dbg is 0 there: the product rejects xw_ws_dbg, bs_prepare
  // passes g_bs_dbg = 0): compiled out, their block boundaries went with them
  // and this kernel ran 1.55 vs 1.34 ms at config 4 (round 6, A/B on one box;
  // sched_barrier fences at the same places did not restore it).  The sum
  // adjoint measured the same either way and compiles them out.
  constexpr int kDbgMask = MAXM ? ~0 : mgcn::kDbgMask;
  const XbArgs &a = A.b;
  __shared__ __attribute__((aligned(16))) char lds[kDsLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gl = lane & 31, grp = lane >> 5;
  const int l16 = lane & 15, g4 = lane >> 4;
  int *ctr = reinterpret_cast<int *>(lds + kDsCtrOff);
  int *filled = ctr, *mdone = ctr + 2, *freed = ctr + 4, *abort_word = ctr + 8;
  if (tid < 16) ctr[tid] = 0;
  // W (64 KB) into LDS once: four float4 per thread
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = tid + kBsThreads * j;  // float4 e: row e >> 5, columns 4 (e & 31) ..
    const float4 v = *reinterpret_cast<const float4 *>(a.W + (int64_t)(e >> 5) * a.ldw + 4 * (e & 31));
    *reinterpret_cast<float4 *>(lds + kDsWOff + 4 * ((e >> 5) * kDsXLd + 4 * (e & 31))) = v;
  }
  __syncthreads();

  const int64_t n_chunks = (a.n_rows + kXwRows - 1) / kXwRows;
  const int64_t n_my = my_chunks(n_chunks);
  auto chunk_of = [&](int64_t i) { return (int64_t)blockIdx.x + i * gridDim.x; };
  auto rows_in = [&](int64_t c) -> uint32_t {
    const int64_t r = a.n_rows - c * kXwRows;
    return (uint32_t)(r <= 0 ? 0 : r >= kXwRows ? kXwRows : r);
  };

  float cs[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // MFMA waves: column sums of their 4 columns
  float hc[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // gather waves (hcs_partial): dY column sums
  f32x16 accw[2];                          // MFMA waves: two 32 x 32 dW tiles
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int r = 0; r < 16; ++r) accw[s][r] = 0.0f;

  if (wave < kBsNG) {
    // ------------------------------- gather waves ---------------------------
    // the wave's k-th quad is q = wave + 8 k: chunk q >> 3, rows
    // 4 (q & 7) + grp and 4 (q & 7) + 2 + grp for lane group grp
    const int64_t n_quads = 8 * n_my;
    auto row_of = [&](int64_t k, int second) -> int64_t {
      const int64_t q = wave + kBsNG * k;
      return chunk_of(q >> 3) * kXwRows + 4 * (q & 7) + 2 * second + grp;
    };
    const auto rdy = buf_rsrc(a.dY, (uint32_t)(a.n_cols * a.lddy * 4));
    const uint32_t ldy_b = (uint32_t)a.lddy * 4u;
    RowMeta cur[2] = {}, nxt[2] = {};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      meta_rowptr(a.rowptr, row_of(0, j), row_of(0, j) < a.n_rows && wave < n_quads, cur[j]);
      if constexpr (MAXM)
        meta_first_m(a.col, a.w, a.slot_map, gl, cur[j]);
      else
        meta_first(a.col, a.w, gl, cur[j]);
      meta_rowptr(a.rowptr, row_of(1, j), row_of(1, j) < a.n_rows && wave + kBsNG < n_quads,
                  nxt[j]);
    }
    int64_t k = 0;
    for (int64_t q = wave; q < n_quads; q += kBsNG, ++k) {
      RowMeta nn[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (MAXM)
          meta_first_m(a.col, a.w, a.slot_map, gl, nxt[j]);
        else
          meta_first(a.col, a.w, gl, nxt[j]);
        const int64_t r2 = row_of(k + 2, j);
        meta_rowptr(a.rowptr, r2, r2 < a.n_rows && q + 2 * kBsNG < n_quads, nn[j]);
      }
      const int64_t i = q >> 3;
      const int64_t c = chunk_of(i);
      const int64_t r0 = c * kXwRows;
      const int lr0 = 4 * (int)(q & 7) + grp;
      u32x4 zv[2] = {};
      if (!(A.dbg & kDbgMask & 4)) {  // the rows' X, under the gathers (streamed once)
        const auto rz = buf_rsrc(a.X + r0 * a.ldx, rows_in(c) * (uint32_t)a.ldx * 4u);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          zv[j] = __builtin_amdgcn_raw_buffer_load_b128(
              rz, 4 * (int)((lr0 + 2 * j) * a.ldx + 4 * gl), 0, MGCN_NT_AUX);
      }
      // DWS + hcs_partial (n_cols == n_rows): the rows' own dY rows, whose
      // column sums are the layer's bias gradient -- every dY row once, rows
      // q then q + 2 of every quad: a fixed order
      // DWS: the rows' ReLU mask words (lanes 0-3) and divisor (lane 4) ride
      // through the ring to the MFMA waves' epilogue (no registers held there)
      uint32_t mv[2] = {0u, 0u};
      if constexpr (MRING && EPI != EPI_STORE) {
        const auto rm = buf_rsrc(a.relu_mask + r0 * 4, rows_in(c) * 16u);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (gl < 4) mv[j] = __builtin_amdgcn_raw_buffer_load_b32(rm, 4 * ((lr0 + 2 * j) * 4 + gl), 0, 0);
        if constexpr (EPI == EPI_RELU_DIV) {
          const auto rd = buf_rsrc(a.row_div + r0, rows_in(c) * 4u);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            if (gl == 4) mv[j] = __builtin_amdgcn_raw_buffer_load_b32(rd, 4 * (lr0 + 2 * j), 0, 0);
        }
      }
      u32x4 yv[2] = {};
      if constexpr (HCS) {
        const auto ry = buf_rsrc(a.dY + r0 * a.lddy, rows_in(c) * (uint32_t)a.lddy * 4u);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          yv[j] = __builtin_amdgcn_raw_buffer_load_b128(
              ry, 4 * (int)((lr0 + 2 * j) * a.lddy + 4 * gl), 0, 0);
      }
      float acc[2][4];
      gather_row2_meta<U, MAXM>(rdy, ldy_b, a.col, a.w, cur[0], cur[1], gl, grp, acc[0], acc[1],
                                a.win_mask, a.slot_map);
      if constexpr (HCS) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4 y = __builtin_bit_cast(float4, yv[j]);
          hc[0] = __fadd_rn(hc[0], y.x);
          hc[1] = __fadd_rn(hc[1], y.y);
          hc[2] = __fadd_rn(hc[2], y.z);
          hc[3] = __fadd_rn(hc[3], y.w);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t row = r0 + lr0 + 2 * j;
        if (a.row_scale != nullptr && row < a.n_rows) {
          const float sc = a.row_scale[row];
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[j][t] = __fmul_rn(acc[j][t], sc);
        }
      }
      const int b = (int)(i & 1);
      const int gen = (int)(i >> 1);
      if (!bs_wait_ge(freed + b, gen, abort_word, A.spin)) break;
      char *buf = lds + b * kRing;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        store_row_terms(buf, lr0 + 2 * j, gl, acc[j]);
        // the X rows as they are (split by the MFMA waves)
        *reinterpret_cast<u32x4 *>(buf + kDsXOff + 4 * ((lr0 + 2 * j) * kDsXLd + 4 * gl)) = zv[j];
        if constexpr (MRING && EPI != EPI_STORE) {
          if (gl < 4)
            *reinterpret_cast<uint32_t *>(buf + kDsMaskOff + 4 * ((lr0 + 2 * j) * 4 + gl)) = mv[j];
          if (EPI == EPI_RELU_DIV && gl == 4)
            *reinterpret_cast<uint32_t *>(buf + kDsDivOff + 4 * (lr0 + 2 * j)) = mv[j];
        }
      }
      bs_signal(filled + b, 4, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        cur[j] = nxt[j];
        nxt[j] = nn[j];
      }
    }
  } else {
    // -------------------------------- MFMA waves ----------------------------
    const int m = wave - kBsNG;  // dX columns 16 m .. 16 m + 15
    // dW tiles (gemm_bwd's mapping): rows 32 ti, columns 32 (tj0 + s)
    const int ti = m >> 1, tj0 = 2 * (m & 1);
    auto read8 = [&](const char *base, const int (&o)[2]) {
      const v4i16 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t *)(base + o[0]));
      const v4i16 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t *)(base + o[1]));
      const short y[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      return __builtin_bit_cast(bf16x8, y);
    };
    const int bit = 4 * m + g4;  // mask bit of this lane's columns (word r: column 16 m + 4 g4 + r)
    for (int64_t i = 0; i < n_my; ++i) {
      // the lane-derived LDS offsets, recomputed per chunk from an opaque copy
      // of the lane id: hoisted out of the loop they were spilled, and every
      // scratch reload waited behind s_waitcnt vmcnt(0) -- i.e. for the
      // previous chunk's dX stores too
      int lane_o = lane;
      asm volatile("" : "+v"(lane_o));
      const int l16 = lane_o & 15, g4 = lane_o >> 4, h = lane_o >> 5;
      int offb[2][2];
      {
        const int q = (lane_o >> 2) & 3, p4 = lane_o & 3;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int r = 0; r < 2; ++r)
            offb[s2][r] = img_off(8 * h + q + 4 * r, 4 * (tj0 + s2) + 2 * (g4 & 1) + (p4 >> 1)) +
                          8 * (p4 & 1);
      }
      const int b = (int)(i & 1);
      const int gen = (int)(i >> 1);
      const int64_t c = chunk_of(i);
      const int64_t r0 = c * kXwRows;
      const uint32_t rv = rows_in(c);
      u32x4 mk[2] = {};
      float dv[2] = {1.0f, 1.0f};
      if constexpr (EPI != EPI_STORE && !MRING) {
        const auto rm = buf_rsrc(a.relu_mask + r0 * 4, rv * 16u);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          mk[rt] = __builtin_amdgcn_raw_buffer_load_b128(rm, 16 * (16 * rt + l16), 0, 0);
        if constexpr (EPI == EPI_RELU_DIV) {
          const auto rd = buf_rsrc(a.row_div + r0, rv * 4u);
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
            dv[rt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rd, 4 * (16 * rt + l16), 0, 0));
        }
      }
      if (!bs_wait_ge(filled + b, kXwRows * (gen + 1), abort_word, A.spin)) break;
      uint32_t mbits[2] = {0u, 0u};  // MRING: this lane's 4 mask bits per row tile
      if constexpr (EPI != EPI_STORE && MRING) {  // from the ring (the gather waves loaded them)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const u32x4 w4 = *reinterpret_cast<const u32x4 *>(lds + b * kRing + kDsMaskOff + 16 * (16 * rt + l16));
#pragma unroll
          for (int r = 0; r < 4; ++r) mbits[rt] |= ((w4[r] >> bit) & 1u) << r;
          if constexpr (EPI == EPI_RELU_DIV)
            dv[rt] = *reinterpret_cast<const float *>(lds + b * kRing + kDsDivOff + 4 * (16 * rt + l16));
        }
      }
      if constexpr (EPI == EPI_RELU_DIV) {
        // rows past the end read divisor 0: make it 1, so their zero rows stay
        // 0 (not 0 / 0) in the dX images dWl reads
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          if ((uint32_t)(16 * rt + l16) >= rv) dv[rt] = 1.0f;
      }
      const char *buf = lds + b * kRing;
      {
        // (first: nothing but the dW accumulators is live across it)
        // dW += X^T dH: X^T fragments (lane: column 32 ti + lc of rows
        // 16 ks + 8 h + j) read from the fp32 rows and split here, dH^T
        // fragments from the term images
          if (!(A.dbg & kDbgMask & 1)) {
          const float *xr = reinterpret_cast<const float *>(buf + kDsXOff) + 32 * ti + (lane_o & 31);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            float xv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] = xr[(16 * ks + 8 * h + j) * kDsXLd];
            bf16x8 fa[3];
            split3_bf16(xv, fa[0], fa[1], fa[2]);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              bf16x8 fb[3];
#pragma unroll
              for (int t = 0; t < 3; ++t) fb[t] = read8(buf + ks * 16 * 256 + t * kXwImg, offb[s2]);
              accw[s2] = mfma_x6(fa[0], fa[1], fa[2], fb[0], fb[1], fb[2], accw[s2]);
            }
          }
        }
        }
      const auto rx = buf_rsrc(a.dX + r0 * a.lddx, rv * (uint32_t)a.lddx * 4u);
      f32x4_t acc2[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc2[rt][r] = 0.0f;
      // W^T fragment rows from the LDS copy
      const float *wq = reinterpret_cast<const float *>(lds + kDsWOff) + (16 * m + l16) * kDsXLd + 8 * g4;
      float4 wn0{}, wn1{};
      if (!(A.dbg & kDbgMask & 8)) {  // dbg 8: no W^T loads (timing only: dX wrong)
        wn0 = *reinterpret_cast<const float4 *>(wq);
        wn1 = *reinterpret_cast<const float4 *>(wq + 4);
      }
      // dX == NULL: dW alone (the same partials as with dX)
      if (a.dX != nullptr) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 wk[3];
        {
          const float v8[8] = {wn0.x, wn0.y, wn0.z, wn0.w, wn1.x, wn1.y, wn1.z, wn1.w};
              if (ks + 1 < 4 && !(A.dbg & kDbgMask & 8)) {
            wn0 = *reinterpret_cast<const float4 *>(wq + 32 * (ks + 1));
            wn1 = *reinterpret_cast<const float4 *>(wq + 32 * (ks + 1) + 4);
          }
              split3_bf16(v8, wk[0], wk[1], wk[2]);
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const int off = img_off(16 * rt + l16, 4 * ks + g4);
          const bf16x8 xh = *reinterpret_cast<const bf16x8 *>(buf + off);
          const bf16x8 xm = *reinterpret_cast<const bf16x8 *>(buf + kXwImg + off);
          const bf16x8 xl = *reinterpret_cast<const bf16x8 *>(buf + 2 * kXwImg + off);
          acc2[rt] = mfma16_x6_at(wk, xh, xm, xl, acc2[rt]);
        }
      }
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int row = 16 * rt + l16;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc2[rt][r];
          if constexpr (EPI != EPI_STORE) {
            const uint32_t on = MRING ? (mbits[rt] >> r) & 1u : (mk[rt][r] >> bit) & 1u;
            v[r] = on ? v[r] : 0.0f;
            cs[r] = __fadd_rn(cs[r], v[r]);  // rows past the end: zero mask words
            if constexpr (EPI == EPI_RELU_DIV) v[r] = __fdiv_rn(v[r], dv[rt]);
          }
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, make_float4(v[0], v[1], v[2], v[3])), rx,
            4 * (int)(row * a.lddx + 16 * m + 4 * g4), 0, MGCN_NT_OUT);
      }
      }
      const int old = bs_signal(mdone + b, 1, lane);
      if (old == kBsNM * gen + kBsNM - 1) bs_signal(freed + b, 1, lane);
    }
  }
  __syncthreads();
  // a hand-off gave up: this launch's dX / dW are incomplete -- say so (the
  // host turns the word into MGCN_EDEVICE) instead of returning them silently
  if (wave == 0 && bs_lds_load(abort_word) != 0) report_device_error(A.err, kDevErrDws);
  if (wave >= kBsNG) {
    const int m = wave - kBsNG;
    {
      const int h = lane >> 5, lc = lane & 31;
      const int ti = m >> 1, tj0 = 2 * (m & 1);
      float *slab = a.dw_partial + (int64_t)blockIdx.x * kXwF * kXwF;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * ti + (r & 3) + 8 * (r >> 2) + 4 * h;
          slab[row * kXwF + 32 * (tj0 + s2) + lc] = accw[s2][r];
        }
    }
    if constexpr (EPI != EPI_STORE) {
      float *red = reinterpret_cast<float *>(lds);  // [16 row lanes][128]
      *reinterpret_cast<float4 *>(red + l16 * kXwF + 16 * m + 4 * g4) =
          make_float4(cs[0], cs[1], cs[2], cs[3]);
    }
  }
  if constexpr (HCS) {  // (past the dX column sums' [16][128] in LDS)
    float *red2 = reinterpret_cast<float *>(lds) + 16 * kXwF;
    if (wave < kBsNG)
      *reinterpret_cast<float4 *>(red2 + (2 * wave + grp) * kXwF + 4 * gl) =
          make_float4(hc[0], hc[1], hc[2], hc[3]);
  }
  if (EPI != EPI_STORE || HCS) {
    __syncthreads();
    if constexpr (EPI != EPI_STORE) {
      if (tid < kXwF) {
        const float *red = reinterpret_cast<const float *>(lds);
        float s = 0.0f;
#pragma unroll
        for (int l = 0; l < 16; ++l) s = __fadd_rn(s, red[l * kXwF + tid]);
        a.colsum_partial[(int64_t)blockIdx.x * kXwF + tid] = s;
      }
    }
    if (HCS && tid >= kXwF && tid < 2 * kXwF) {
      const int f = tid - kXwF;
      const float *red2 = reinterpret_cast<const float *>(lds) + 16 * kXwF;
      float s = 0.0f;
#pragma unroll
      for (int l = 0; l < 16; ++l) s = __fadd_rn(s, red2[l * kXwF + f]);
      A.hcs_partial[(int64_t)blockIdx.x * kXwF + f] = s;
    }
  }
}

int g_xw_ws_full = 1;  // mgcn_set_option("xw_ws_full"): the warp-specialised dW + dX adjoint (DWS)
int g_xw_ws_max = 1;   // mgcn_set_option("xw_ws_max"): ... and its max adjoint (DWS + win_mask)

int bs_grid() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return cus;  // one workgroup per CU
}

template <int U, int MODE>
int launch_bs_u(const XbsArgs &a, int epi, int grid, hipStream_t s) {
  if (epi == EPI_RELU_DIV)
    hipLaunchKernelGGL((spmm_xw_bwd_ws_kernel<U, EPI_RELU_DIV, MODE>), dim3(grid), dim3(kBsThreads),
                       0, s, a);
  else if (epi == EPI_RELU)
    hipLaunchKernelGGL((spmm_xw_bwd_ws_kernel<U, EPI_RELU, MODE>), dim3(grid), dim3(kBsThreads), 0,
                       s, a);
  else
    hipLaunchKernelGGL((spmm_xw_bwd_ws_kernel<U, EPI_STORE, MODE>), dim3(grid), dim3(kBsThreads), 0,
                       s, a);
  return check_launch("spmm_xw_bwd_ws_kernel");
}

// mgcn_set_option("xw_ws_dbg") (experiment builds): timing experiments (dW / dX
// WRONG when set): bit 0 skip the dW products, bit 2 skip the X loads, bit 3
// skip the W^T reads
int g_bs_dbg = 0;

int g_bs_full_unroll = 5;  // mgcn_set_option("xw_ws_full_unroll"): DWS gathers in flight per row (5: 0.984-0.991 vs 1.000-1.012 ms at 4)

template <int MODE>
int launch_bs(const XbsArgs &a, int epi, int grid, hipStream_t s) {
  if constexpr (MODE == kBsDwsM) {  // the winner words take registers: 3 slots per row
    return launch_bs_u<3, MODE>(a, epi, grid, s);
  } else {
    return g_bs_full_unroll == 4 ? launch_bs_u<4, MODE>(a, epi, grid, s)
         : g_bs_full_unroll == 5 ? launch_bs_u<5, MODE>(a, epi, grid, s)
                                 : launch_bs_u<6, MODE>(a, epi, grid, s);
  }
}

// the warp-specialised launch's failure plumbing: spin bound, error word
int bs_prepare(XbsArgs &sa) {
  sa.dbg = MGCN_EXPERIMENT ? g_bs_dbg : 0;  // (always 0 in the product)
  sa.spin = g_spin_limit;
  sa.err = device_error_word();
  return sa.err == nullptr ? MGCN_EHIP : MGCN_OK;
}

}  // namespace

int xw_set_ws(const char *name, int value) {
  const std::string n(name);
  auto flag = [&](int &g) {
    if (value < 0 || value > 1) {
      set_error("%s must be 0 or 1", name);
      return (int)MGCN_EINVAL;
    }
    g = value;
    return (int)MGCN_OK;
  };
  auto unroll = [&](int &g, std::initializer_list<int> ok) {
    for (int v : ok)
      if (v == value) {
        g = value;
        return (int)MGCN_OK;
      }
    set_error("%s: unsupported value %d", name, value);
    return (int)MGCN_EINVAL;
  };
  if (n == "xw_pk_unroll" || n == "xw_pk_bwd_unroll") {  // (experiment builds: the sweep)
    if (!MGCN_EXPERIMENT) {
      set_error("%s: experiment builds only (make exp -> libmgcn_exp.so)", name);
      return MGCN_EINVAL;
    }
    return n == "xw_pk_unroll" ? unroll(g_xw_pk_unroll, {3, 4, 5, 6})
                               : unroll(g_xw_pk_bwd_unroll, {2, 3, 4});
  }
  if (n == "xw_ws_max") return flag(g_xw_ws_max);
  if (n == "xw_ws_full") return flag(g_xw_ws_full);
  if (n == "xw_ws_dbg") {  // (timing experiments: results WRONG when set)
    if (!MGCN_EXPERIMENT) {
      set_error("xw_ws_dbg: experiment builds only (make exp -> libmgcn_exp.so)");
      return MGCN_EINVAL;
    }
    g_bs_dbg = value;
    return MGCN_OK;
  }
  return unroll(g_bs_full_unroll, {4, 5, 6});  // "xw_ws_full_unroll"
}

int xw_set_unroll(int value) {
  if (value != 4 && value != 5 && value != 6 && value != 8) {
    set_error("spmm_xw_unroll must be 4, 5, 6 or 8 (5 / 6: the forward only)");
    return MGCN_EINVAL;
  }
  g_xw_unroll = value;
  return MGCN_OK;
}

}  // namespace mgcn

using namespace mgcn;

extern "C" int mgcn_spmm_xw_supported(int32_t F_in, int32_t F_out, int reduce) {
  return F_in == F_out && (F_in == kXwF || F_in == 256) && gemm_precision_is_x6() &&
         (reduce == MGCN_REDUCE_SUM || reduce == MGCN_REDUCE_MEAN);
}

extern "C" int mgcn_spmm_xw_bwd_full_supported(int32_t F_in, int32_t F_out) {
  // the dW-accumulating backward and the max adjoint: 128 x 128 only (at
  // 256 the dW accumulators do not fit beside the gather: Z^T dY instead)
  return F_in == kXwF && F_out == kXwF && gemm_precision_is_x6();
}

extern "C" size_t mgcn_spmm_xw_fwd_workspace_bytes(int32_t F_in, int32_t F_out) {
  return F_in == 256 && F_out == 256 ? xw_wide_workspace_bytes(false) : 0;
}

extern "C" int mgcn_spmm_xw_fwd(int64_t n_rows, int64_t n_cols, int32_t F_in, int32_t F_out,
                                const int64_t *rowptr, const int32_t *col, const float *w,
                                const float *X, int64_t ldx, const float *W, int64_t ldw,
                                const float *bias, float *Y, int64_t ldy, int reduce, int relu,
                                uint32_t *relu_mask, float *Z, int64_t ldz, void *workspace,
                                size_t workspace_bytes, void *stream) {
  clear_error();
  if (int rc = take_device_error()) return rc;  // a previous launch failed on the device
  MGCN_REQUIRE(n_rows >= 0, "mgcn_spmm_xw_fwd: negative size");
  MGCN_REQUIRE(mgcn_spmm_xw_supported(F_in, F_out, reduce),
               "mgcn_spmm_xw_fwd: unsupported F_in=%d F_out=%d reduce=%d (needs 128 x 128 or "
               "256 x 256, sum/mean, bf16x6)",
               F_in, F_out, reduce);
  MGCN_REQUIRE(relu_mask == nullptr || relu, "mgcn_spmm_xw_fwd: relu_mask needs relu");
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && X && W && Y, "mgcn_spmm_xw_fwd: null array");
  MGCN_REQUIRE(ldx >= F_in && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0,
               "mgcn_spmm_xw_fwd: X must have 16-byte aligned rows");
  MGCN_REQUIRE(ldw >= F_out && ldy >= F_out, "mgcn_spmm_xw_fwd: leading dimension too small");
  if (F_in == 256) {
    // the wide kernels address every gathered row through a 64-bit base:
    // no table-size limit; 32-bit offsets only within a 16-row chunk
    MGCN_REQUIRE(n_cols > 0 && (uint64_t)16 * (uint64_t)(ldy > ldz ? ldy : ldz) * 4u < (1ull << 31),
                 "mgcn_spmm_xw_fwd: leading dimension too large");
    MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
                 "mgcn_spmm_xw_fwd: relu_mask not 16-byte aligned");
    MGCN_REQUIRE(Z == nullptr || (ldz >= F_in && ldz % 4 == 0 && reinterpret_cast<uintptr_t>(Z) % 16 == 0),
                 "mgcn_spmm_xw_fwd: Z must have 16-byte aligned rows (ldz >= F_in)");
    MGCN_REQUIRE(ldy % 4 == 0 && reinterpret_cast<uintptr_t>(Y) % 16 == 0,
                 "mgcn_spmm_xw_fwd: Y must have 16-byte aligned rows at F = 256");
    const size_t need = mgcn_spmm_xw_fwd_workspace_bytes(F_in, F_out);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_spmm_xw_fwd: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    return xw_wide_fwd(n_rows, rowptr, col, w, X, ldx, W, ldw, bias, Y, ldy,
                       reduce == MGCN_REDUCE_MEAN, relu != 0, relu_mask, Z, ldz, workspace,
                       as_stream(stream));
  }
  MGCN_REQUIRE(n_cols > 0 && (uint64_t)n_cols * (uint64_t)ldx * 4u <= 0xfffffff0ull,
               "mgcn_spmm_xw_fwd: X must hold 1 .. 4 GiB - 1 bytes (32-bit gather offsets)");
  MGCN_REQUIRE((uint64_t)kXwRows * (uint64_t)ldy * 4u < (1ull << 31),
               "mgcn_spmm_xw_fwd: ldy too large");
  MGCN_REQUIRE(bias == nullptr || reinterpret_cast<uintptr_t>(bias) % 4 == 0,
               "mgcn_spmm_xw_fwd: bias not 4-byte aligned");
  MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
               "mgcn_spmm_xw_fwd: relu_mask not 16-byte aligned");
  MGCN_REQUIRE(Z == nullptr || (ldz >= F_in && ldz % 4 == 0 && reinterpret_cast<uintptr_t>(Z) % 16 == 0 &&
                                (uint64_t)kXwRows * (uint64_t)ldz * 4u < (1ull << 31)),
               "mgcn_spmm_xw_fwd: Z must have 16-byte aligned rows (ldz >= F_in)");
  XwArgs a{};
  a.n_rows = n_rows;
  a.rowptr = rowptr;
  a.col = col;
  a.w = w;
  a.X = X;
  a.ldx = ldx;
  a.n_cols = n_cols;
  a.W = W;
  a.ldw = ldw;
  a.bias = bias;
  a.Y = Y;
  a.ldy = ldy;
  a.relu_mask = relu_mask;
  a.Z = Z;
  a.ldz = ldz;
  a.mean = reduce == MGCN_REDUCE_MEAN;
  a.relu = relu != 0;
  hipStream_t s = as_stream(stream);
  return g_xw_unroll == 4 ? launch_xw<4>(a, s)
       : g_xw_unroll == 5 ? launch_xw<5>(a, s)
       : g_xw_unroll == 6 ? launch_xw<6>(a, s)
                          : launch_xw<8>(a, s);
}

extern "C" size_t mgcn_spmm_xw_bwd_workspace_bytes(int64_t n_rows, int32_t F_in, int32_t F_out) {
  (void)n_rows;
  if (F_in == 256 && F_out == 256) return xw_wide_workspace_bytes(true);
  const size_t g = (size_t)xw_grid();
  return align_up(g * kXwF * kXwF * 4, 256) + align_up(g * kXwF * 4, 256);
}

namespace {
// mgcn_spmm_xw_bwd and (dy_colsum != NULL) mgcn_spmm_xw_bwd_hcs
int xw_bwd_impl(int64_t n_rows, int64_t n_cols, int32_t F_in, int32_t F_out,
                const int64_t *rowptr_t, const int32_t *col_t, const float *w_t,
                const float *row_scale, const float *dY, int64_t lddy, const float *X,
                int64_t ldx, const float *W, int64_t ldw, float *dW, int64_t lddw, int accumulate,
                float *dX, int64_t lddx, const uint32_t *relu_mask, const float *row_div,
                float *colsum, const uint32_t *win_mask, const int32_t *slot_map,
                float *dy_colsum, void *workspace, size_t workspace_bytes, void *stream) {
  if (int rc = take_device_error()) return rc;  // a previous launch failed on the device
  MGCN_REQUIRE(n_rows >= 0, "mgcn_spmm_xw_bwd: negative size");
  MGCN_REQUIRE((win_mask == nullptr) == (slot_map == nullptr),
               "mgcn_spmm_xw_bwd: win_mask and slot_map go together (max adjoint)");
  MGCN_REQUIRE(mgcn_spmm_xw_supported(F_in, F_out, MGCN_REDUCE_SUM),
               "mgcn_spmm_xw_bwd: unsupported F_in=%d F_out=%d (needs 128 x 128 or 256 x 256, "
               "bf16x6)", F_in, F_out);
  // X == NULL and dW == NULL: dX only (dW formed by the caller from Z^T dY)
  const bool dx_only = X == nullptr && dW == nullptr;
  MGCN_REQUIRE(dx_only || mgcn_spmm_xw_bwd_full_supported(F_in, F_out),
               "mgcn_spmm_xw_bwd: at F=%d only the dX-only form (X = dW = NULL)", F_in);
  MGCN_REQUIRE(dx_only || (X != nullptr && dW != nullptr && lddw >= F_out),
               "mgcn_spmm_xw_bwd: bad dW (X and dW are given together, or both NULL for dX only)");
  MGCN_REQUIRE(row_div == nullptr || relu_mask != nullptr,
               "mgcn_spmm_xw_bwd: row_div needs relu_mask");
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) {  // an empty row range (a sharded chunk): no dX rows to write
    if (dy_colsum) MGCN_HIP_TRY(hipMemsetAsync(dy_colsum, 0, sizeof(float) * F_out, s));
    if (!accumulate && dW != nullptr)
      for (int32_t r = 0; r < F_in; ++r)
        MGCN_HIP_TRY(hipMemsetAsync(dW + r * lddw, 0, sizeof(float) * F_out, s));
    if (colsum && !(dx_only && accumulate))
      MGCN_HIP_TRY(hipMemsetAsync(colsum, 0, sizeof(float) * F_in, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(!dx_only || (dX != nullptr && win_mask == nullptr),
               "mgcn_spmm_xw_bwd: the dX-only form needs dX and takes no win_mask");
  const int epi = relu_mask == nullptr ? EPI_STORE : row_div != nullptr ? EPI_RELU_DIV : EPI_RELU;
  MGCN_REQUIRE(epi == EPI_STORE || (dX != nullptr && colsum != nullptr),
               "mgcn_spmm_xw_bwd: relu_mask needs dX and colsum");
  MGCN_REQUIRE(rowptr_t && dY, "mgcn_spmm_xw_bwd: null array");
  MGCN_REQUIRE(lddy >= F_out && lddy % 4 == 0 && reinterpret_cast<uintptr_t>(dY) % 16 == 0,
               "mgcn_spmm_xw_bwd: dY must have 16-byte aligned rows");
  if (F_in == 256) {
    MGCN_REQUIRE(dX != nullptr && win_mask == nullptr, "mgcn_spmm_xw_bwd: the dX-only form needs dX");
    MGCN_REQUIRE(W != nullptr && ldw >= F_out && lddx >= F_in && lddx % 4 == 0 &&
                     reinterpret_cast<uintptr_t>(dX) % 16 == 0 &&
                     (uint64_t)16 * (uint64_t)lddx * 4u < (1ull << 31),
                 "mgcn_spmm_xw_bwd: bad W/dX (16-byte aligned dX rows)");
    MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
                 "mgcn_spmm_xw_bwd: relu_mask not 16-byte aligned");
    const size_t need = mgcn_spmm_xw_bwd_workspace_bytes(n_rows, F_in, F_out);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_spmm_xw_bwd: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    return xw_wide_bwd_dx(n_rows, rowptr_t, col_t, w_t, row_scale, dY, lddy, W, ldw, dX, lddx,
                          relu_mask, row_div, colsum, accumulate, workspace, s);
  }
  MGCN_REQUIRE(dx_only || (ldx >= F_in && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0),
               "mgcn_spmm_xw_bwd: X must have 16-byte aligned rows");
  if (dx_only) ldx = 0;
  MGCN_REQUIRE(n_cols > 0 && (uint64_t)n_cols * (uint64_t)lddy * 4u <= 0xfffffff0ull,
               "mgcn_spmm_xw_bwd: dY must hold 1 .. 4 GiB - 1 bytes (32-bit gather offsets)");
  MGCN_REQUIRE((uint64_t)kXwRows * (uint64_t)(ldx > lddx ? ldx : lddx) * 4u < (1ull << 31),
               "mgcn_spmm_xw_bwd: leading dimension too large");
  MGCN_REQUIRE(dX == nullptr || (W != nullptr && ldw >= F_out && lddx >= F_in),
               "mgcn_spmm_xw_bwd: bad W/dX");
  // the warp-specialised adjoint copies W into LDS with 16-byte loads
  MGCN_REQUIRE(W == nullptr || (ldw % 4 == 0 && reinterpret_cast<uintptr_t>(W) % 16 == 0),
               "mgcn_spmm_xw_bwd: W must have 16-byte aligned rows");
  MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
               "mgcn_spmm_xw_bwd: relu_mask not 16-byte aligned");
  const size_t need = mgcn_spmm_xw_bwd_workspace_bytes(n_rows, F_in, F_out);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_spmm_xw_bwd: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  const int64_t n_chunks = (n_rows + kXwRows - 1) / kXwRows;
  int grid = xw_grid();
  if (grid > n_chunks) grid = (int)n_chunks;
  XbArgs a{};
  a.n_rows = n_rows;
  a.rowptr = rowptr_t;
  a.col = col_t;
  a.w = w_t;
  a.row_scale = row_scale;
  a.dY = dY;
  a.lddy = lddy;
  a.n_cols = n_cols;
  a.X = X;
  a.ldx = ldx;
  a.W = W;
  a.ldw = ldw;
  a.dX = dX;
  a.lddx = lddx;
  a.relu_mask = relu_mask;
  a.row_div = row_div;
  a.win_mask = win_mask;
  a.slot_map = slot_map;
  a.dw_partial = static_cast<float *>(workspace);
  a.colsum_partial = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                               align_up((size_t)xw_grid() * kXwF * kXwF * 4, 256));
  int rc;
  if (dx_only) {
    rc = g_xw_unroll == 8 ? launch_xb_dx<8>(a, epi, grid, s) : launch_xb_dx<4>(a, epi, grid, s);
    if (rc || epi == EPI_STORE) return rc;
    // dX only: accumulate != 0 adds the column sums into colsum (row chunks
    // of one adjoint fold their bias gradient on the device)
    return launch_fold(a.colsum_partial, grid, kXwF, kXwF, colsum, kXwF, accumulate, s);
  }
  float *hcs_partial = nullptr;
  // (the max adjoint's dW-only form stays two-phase: 1.10 vs 1.22 ms at config 4)
  if ((g_xw_ws_full || dy_colsum) && (win_mask == nullptr || (g_xw_ws_max && dX != nullptr))) {
    // the warp-specialised dW + dX (or dW-only) form (one workgroup per CU; DWS)
    XbsArgs sa{};
    sa.b = a;
    if (int rc2 = bs_prepare(sa)) return rc2;
    grid = bs_grid() < n_chunks ? bs_grid() : (int)n_chunks;
    // dY's column sums: [grid][128] partials past the grid's dW slabs (the
    // dW partial area holds xw_grid() = 2 x CUs slabs, this grid <= CUs)
    if (dy_colsum) hcs_partial = a.dw_partial + (size_t)grid * kXwF * kXwF;
    sa.hcs_partial = hcs_partial;
    rc = hcs_partial ? launch_bs<kBsDwsH>(sa, epi, grid, s)
         : win_mask  ? launch_bs<kBsDwsM>(sa, epi, grid, s)
                     : launch_bs<kBsDws>(sa, epi, grid, s);
  } else {
    rc = g_xw_unroll == 8 ? launch_xb_u<8>(a, epi, grid, s) : launch_xb_u<4>(a, epi, grid, s);
  }
  if (rc) return rc;
  rc = launch_split_reduce(a.dw_partial, grid, (int64_t)kXwF * kXwF, kXwF, dW, lddw, accumulate, s);
  if (rc == MGCN_OK && hcs_partial) rc = launch_colsum_fold(hcs_partial, grid, kXwF, dy_colsum, s);
  if (rc || epi == EPI_STORE) return rc;
  return launch_colsum_fold(a.colsum_partial, grid, kXwF, colsum, s);
}
}  // namespace

extern "C" int mgcn_spmm_xw_bwd(int64_t n_rows, int64_t n_cols, int32_t F_in, int32_t F_out,
                                const int64_t *rowptr_t, const int32_t *col_t, const float *w_t,
                                const float *row_scale, const float *dY, int64_t lddy,
                                const float *X, int64_t ldx, const float *W, int64_t ldw,
                                float *dW, int64_t lddw, int accumulate, float *dX, int64_t lddx,
                                const uint32_t *relu_mask, const float *row_div, float *colsum,
                                const uint32_t *win_mask, const int32_t *slot_map,
                                void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  return xw_bwd_impl(n_rows, n_cols, F_in, F_out, rowptr_t, col_t, w_t, row_scale, dY, lddy, X,
                     ldx, W, ldw, dW, lddw, accumulate, dX, lddx, relu_mask, row_div, colsum,
                     win_mask, slot_map, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int mgcn_spmm_xw_bwd_hcs(int64_t n_rows, int64_t n_cols, const int64_t *rowptr_t,
                                    const int32_t *col_t, const float *w_t,
                                    const float *row_scale, const float *dY, int64_t lddy,
                                    const float *X, int64_t ldx, const float *W, int64_t ldw,
                                    float *dW, int64_t lddw, int accumulate, float *dX,
                                    int64_t lddx, const uint32_t *relu_mask,
                                    const float *row_div, float *colsum, float *dy_colsum,
                                    void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows == n_cols, "mgcn_spmm_xw_bwd_hcs: needs n_rows == n_cols (%lld, %lld): "
               "every dY row a row of the view", (long long)n_rows, (long long)n_cols);
  MGCN_REQUIRE(X != nullptr && dW != nullptr && dX != nullptr && dy_colsum != nullptr,
               "mgcn_spmm_xw_bwd_hcs: X, dW, dX and dy_colsum are required");
  return xw_bwd_impl(n_rows, n_cols, kXwF, kXwF, rowptr_t, col_t, w_t, row_scale, dY, lddy, X,
                     ldx, W, ldw, dW, lddw, accumulate, dX, lddx, relu_mask, row_div, colsum,
                     nullptr, nullptr, dy_colsum, workspace, workspace_bytes, stream);
}

#ifdef MGCN_XW_PROFILE
extern "C" int mgcn_debug_xw_prof(unsigned long long *host) {
  MGCN_HIP_TRY(hipDeviceSynchronize());
  MGCN_HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xprof), sizeof(g_xprof)));
  return MGCN_OK;
}
#endif

// ---------------------------------------------------------------- packed tables
namespace {
int check_packed(const mgcn_packed_table *t, int32_t F, const char *who) {
  MGCN_REQUIRE(t != nullptr && t->words != nullptr, "%s: null packed table", who);
  MGCN_REQUIRE(t->F == F, "%s: packed table of F = %d for a layer of F = %d", who, t->F, F);
  MGCN_REQUIRE(t->n_seg >= 1 && t->n_seg <= 64, "%s: n_seg %d outside 1 .. 64", who, t->n_seg);
  MGCN_REQUIRE(t->row_bits >= 0 && t->row_bits + 6 <= 31 && t->seg_rows >= 1 &&
                   (int64_t)t->seg_rows <= ((int64_t)1 << t->row_bits),
               "%s: seg_rows %d does not fit row_bits %d", who, t->seg_rows, t->row_bits);
  // in-segment byte offsets stay below 2 GiB (the header plus a dense-size
  // value area): the kernels' buffer ranges are capped there
  MGCN_REQUIRE((uint64_t)t->seg_rows * (2 * (F / 32) + F) * 4u + 16u < (1ull << 31),
               "%s: seg_rows %d too large for the 2-GiB in-segment offsets", who, t->seg_rows);
  MGCN_REQUIRE(t->n_words >= 0, "%s: negative n_words", who);
  if (F == kXwF) {
    // F = 128: one buffer resource over the whole table (32-bit offsets)
    MGCN_REQUIRE((uint64_t)t->n_words * 4u <= 0x7ffffff0ull,
                 "%s: an F = 128 packed table spans at most 2 GiB - 16 B (got %lld words)", who,
                 (long long)t->n_words);
    for (int s = 0; s < t->n_seg; ++s)
      MGCN_REQUIRE(t->seg_base[s] >= 0 && t->seg_base[s] <= t->n_words,
                   "%s: segment %d at word %lld outside the table's %lld words", who, s,
                   (long long)t->seg_base[s], (long long)t->n_words);
  }
  return MGCN_OK;
}

// the F = 128 kernels' view of a checked packed table
template <class Args>
void fill_pk128(Args &a, const mgcn_packed_table *t) {
  a.pk = t->words;
  a.pk_bytes = (uint32_t)(t->n_words * 4);
  a.pk_rbits = (uint32_t)t->row_bits;
  a.pk_head = (uint32_t)t->seg_rows * 8u;
  for (int s = 0; s < 64; ++s) a.pk_base[s] = s < t->n_seg ? (uint32_t)t->seg_base[s] : 0u;
}
}  // namespace

extern "C" int mgcn_spmm_xw_fwd_packed(int64_t n_rows, int32_t F_in, int32_t F_out,
                                       const int64_t *rowptr, const int32_t *col, const float *w,
                                       const mgcn_packed_table *X, const float *W, int64_t ldw,
                                       const float *bias, float *Y, int64_t ldy, int reduce,
                                       int relu, uint32_t *relu_mask, float *Z, int64_t ldz,
                                       void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  if (int rc = take_device_error()) return rc;  // a previous launch failed on the device
  MGCN_REQUIRE(n_rows >= 0, "mgcn_spmm_xw_fwd_packed: negative size");
  MGCN_REQUIRE(mgcn_spmm_xw_supported(F_in, F_out, reduce),
               "mgcn_spmm_xw_fwd_packed: 128 x 128 or 256 x 256, sum / mean, bf16x6 only");
  MGCN_REQUIRE(relu_mask == nullptr || relu, "mgcn_spmm_xw_fwd_packed: relu_mask needs relu");
  if (n_rows == 0) return MGCN_OK;
  if (int rc = check_packed(X, F_in, "mgcn_spmm_xw_fwd_packed")) return rc;
  MGCN_REQUIRE(rowptr && W && Y, "mgcn_spmm_xw_fwd_packed: null array");
  if (F_in == kXwF) {
    MGCN_REQUIRE(ldw >= F_out && ldy >= F_out && (uint64_t)kXwRows * (uint64_t)ldy * 4u < (1ull << 31),
                 "mgcn_spmm_xw_fwd_packed: bad ldw / ldy");
    MGCN_REQUIRE(bias == nullptr || reinterpret_cast<uintptr_t>(bias) % 4 == 0,
                 "mgcn_spmm_xw_fwd_packed: bias not 4-byte aligned");
    MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
                 "mgcn_spmm_xw_fwd_packed: relu_mask not 16-byte aligned");
    MGCN_REQUIRE(Z == nullptr || (ldz >= F_in && ldz % 4 == 0 && reinterpret_cast<uintptr_t>(Z) % 16 == 0 &&
                                  (uint64_t)kXwRows * (uint64_t)ldz * 4u < (1ull << 31)),
                 "mgcn_spmm_xw_fwd_packed: Z must have 16-byte aligned rows (ldz >= F_in)");
    XwArgs a{};
    a.n_rows = n_rows;
    a.rowptr = rowptr;
    a.col = col;
    a.w = w;
    a.W = W;
    a.ldw = ldw;
    a.bias = bias;
    a.Y = Y;
    a.ldy = ldy;
    a.relu_mask = relu_mask;
    a.Z = Z;
    a.ldz = ldz;
    a.mean = reduce == MGCN_REDUCE_MEAN;
    a.relu = relu != 0;
    fill_pk128(a, X);
    hipStream_t s = as_stream(stream);
    // (the product build instantiates U = 3 only)
    constexpr bool X = MGCN_EXPERIMENT;
    if (X && g_xw_pk_unroll == 4) return launch_xw<X ? 4 : 3, true>(a, s);
    if (X && g_xw_pk_unroll == 5) return launch_xw<X ? 5 : 3, true>(a, s);
    if (X && g_xw_pk_unroll == 6) return launch_xw<X ? 6 : 3, true>(a, s);
    return launch_xw<3, true>(a, s);
  }
  MGCN_REQUIRE(ldw >= F_out && ldy >= F_out && ldy % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(Y) % 16 == 0 &&
                   (uint64_t)16 * (uint64_t)(ldy > ldz ? ldy : ldz) * 4u < (1ull << 31),
               "mgcn_spmm_xw_fwd_packed: Y must have 16-byte aligned rows");
  MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
               "mgcn_spmm_xw_fwd_packed: relu_mask not 16-byte aligned");
  MGCN_REQUIRE(Z == nullptr || (ldz >= F_in && ldz % 4 == 0 && reinterpret_cast<uintptr_t>(Z) % 16 == 0),
               "mgcn_spmm_xw_fwd_packed: Z must have 16-byte aligned rows (ldz >= F_in)");
  const size_t need = mgcn_spmm_xw_fwd_workspace_bytes(F_in, F_out);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_spmm_xw_fwd_packed: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  return xw_wide_fwd(n_rows, rowptr, col, w, nullptr, 0, W, ldw, bias, Y, ldy,
                     reduce == MGCN_REDUCE_MEAN, relu != 0, relu_mask, Z, ldz, workspace,
                     as_stream(stream), X);
}

extern "C" int mgcn_spmm_xw_bwd_packed(int64_t n_rows, int32_t F_in, int32_t F_out,
                                       const int64_t *rowptr_t, const int32_t *col_t,
                                       const float *w_t, const float *row_scale,
                                       const mgcn_packed_table *dY, const float *W, int64_t ldw,
                                       float *dX, int64_t lddx, const uint32_t *relu_mask,
                                       const float *row_div, float *colsum, int accumulate,
                                       void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  if (int rc = take_device_error()) return rc;  // a previous launch failed on the device
  MGCN_REQUIRE(n_rows >= 0, "mgcn_spmm_xw_bwd_packed: negative size");
  MGCN_REQUIRE(mgcn_spmm_xw_supported(F_in, F_out, MGCN_REDUCE_SUM),
               "mgcn_spmm_xw_bwd_packed: 128 x 128 or 256 x 256, bf16x6 only");
  MGCN_REQUIRE(row_div == nullptr || relu_mask != nullptr,
               "mgcn_spmm_xw_bwd_packed: row_div needs relu_mask");
  MGCN_REQUIRE(relu_mask == nullptr || colsum != nullptr,
               "mgcn_spmm_xw_bwd_packed: relu_mask needs colsum");
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) {  // an empty row range: no dX rows to write
    if (colsum && !accumulate) MGCN_HIP_TRY(hipMemsetAsync(colsum, 0, sizeof(float) * F_in, s));
    return MGCN_OK;
  }
  if (int rc = check_packed(dY, F_out, "mgcn_spmm_xw_bwd_packed")) return rc;
  MGCN_REQUIRE(rowptr_t && W && dX, "mgcn_spmm_xw_bwd_packed: null array");
  if (F_in == kXwF) {
    MGCN_REQUIRE(ldw >= F_out && lddx >= F_in && (uint64_t)kXwRows * (uint64_t)lddx * 4u < (1ull << 31),
                 "mgcn_spmm_xw_bwd_packed: bad W/dX");
    MGCN_REQUIRE(ldw % 4 == 0 && reinterpret_cast<uintptr_t>(W) % 16 == 0,
                 "mgcn_spmm_xw_bwd_packed: W must have 16-byte aligned rows");
    MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
                 "mgcn_spmm_xw_bwd_packed: relu_mask not 16-byte aligned");
    const size_t need = mgcn_spmm_xw_bwd_workspace_bytes(n_rows, F_in, F_out);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_spmm_xw_bwd_packed: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    const int epi = relu_mask == nullptr ? EPI_STORE : row_div != nullptr ? EPI_RELU_DIV : EPI_RELU;
    const int64_t n_chunks = (n_rows + kXwRows - 1) / kXwRows;
    int grid = xw_grid();
    if (grid > n_chunks) grid = (int)n_chunks;
    XbArgs a{};
    a.n_rows = n_rows;
    a.rowptr = rowptr_t;
    a.col = col_t;
    a.w = w_t;
    a.row_scale = row_scale;
    a.W = W;
    a.ldw = ldw;
    a.dX = dX;
    a.lddx = lddx;
    a.relu_mask = relu_mask;
    a.row_div = row_div;
    a.dw_partial = static_cast<float *>(workspace);
    a.colsum_partial = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                                 align_up((size_t)xw_grid() * kXwF * kXwF * 4, 256));
    fill_pk128(a, dY);
    constexpr bool X = MGCN_EXPERIMENT;  // (the product build instantiates U = 3 only)
    int rc;
    if (X && g_xw_pk_bwd_unroll == 2)
      rc = launch_xb_dx<X ? 2 : 3, true>(a, epi, grid, s);
    else if (X && g_xw_pk_bwd_unroll == 4)
      rc = launch_xb_dx<X ? 4 : 3, true>(a, epi, grid, s);
    else
      rc = launch_xb_dx<3, true>(a, epi, grid, s);
    if (rc || epi == EPI_STORE) return rc;
    return launch_fold(a.colsum_partial, grid, kXwF, kXwF, colsum, kXwF, accumulate, s);
  }
  MGCN_REQUIRE(ldw >= F_out && lddx >= F_in && lddx % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(dX) % 16 == 0 &&
                   (uint64_t)16 * (uint64_t)lddx * 4u < (1ull << 31),
               "mgcn_spmm_xw_bwd_packed: bad W/dX (16-byte aligned dX rows)");
  MGCN_REQUIRE(relu_mask == nullptr || reinterpret_cast<uintptr_t>(relu_mask) % 16 == 0,
               "mgcn_spmm_xw_bwd_packed: relu_mask not 16-byte aligned");
  const size_t need = mgcn_spmm_xw_bwd_workspace_bytes(n_rows, F_in, F_out);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_spmm_xw_bwd_packed: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  return xw_wide_bwd_dx(n_rows, rowptr_t, col_t, w_t, row_scale, nullptr, 0, W, ldw, dX, lddx,
                        relu_mask, row_div, colsum, accumulate, workspace, s, dY);
}
