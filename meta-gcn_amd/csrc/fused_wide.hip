// Fused GCN layer kernels at F_in = F_out = 256 (config 5, BASELINE.json
// configs[4]: 50M nodes, 500M edges, F = 256) on gfx950:
//
//   forward   Y = epi((A X) W + b)   (+ Z = A X, + ReLU mask words)
//   backward  dX = relu'(lower) ((A^T dY) W^T) [/ row_div], colsum = sum_rows dX
//             (the dX-only form: dW = Z^T dY is the caller's dense pass)
//
// The reference computes a layer as x @ W then gather -> * norm ->
// scatter_add (src/gcn_meta/models/gcn_base_models.py:201, 223-237); the
// association and the numerics follow fused.hip's F = 128 kernels (the
// aggregation bit for bit the SpMM's, the dense product bf16x6), but the
// shapes of a 256-wide layer change three things:
//
// * one WAVE per row: a gathered row is 1 KB = 64 lanes x 16 B, so the
//   row's edges are wave-uniform.  Edge metadata is loaded 64 slots at a time
//   lane-parallel and broadcast with v_readlane into SGPRs, and every gathered
//   row gets its own buffer resource whose base is X + col * ldx computed in
//   64-bit scalar arithmetic: no 32-bit offset limit on the table (config 5's
//   [50M, 256] table is 51 GB), and a slot past the row's end gets a
//   zero-byte resource (the load returns 0 without touching memory).
// * W does not fit on chip: its three bf16 terms are 384 KB, the LDS holds
//   160 KB and a wave's share of the fragments (32 columns x 256 k) would be
//   192 VGPRs.  A prep launch splits W (W^T for the adjoint) once into a
//   fragment-ordered image (ks, n-tile, term, lane; 16 B per lane), and each
//   wave streams its two n-tiles' fragments from L2 every chunk (48 KB per
//   wave per 16-row chunk), one k-step ahead of the MFMAs, the first k-step
//   issued under the tail of the gathers.
// * 16-row chunks: the three term images of a chunk are 24 KB (rows of
//   512 B, 16-B chunk ch of row r at ch ^ (r & 15): conflict-free for the
//   16x16x32 A-operand reads and the row writes), double-buffered, plus two
//   fp32 staging tiles of 16 KB (column c of row r at c ^ (((r >> 2) & 3) << 4):
//   conflict-free MFMA-layout writes and whole-row reads): 80 KB, two
//   workgroups per CU, one barrier per chunk as in the F = 128 forward.
//
// Chunk loop (persistent 512-thread workgroups, chunk c to workgroup
// c % grid): Phase A -- wave w aggregates rows 2w, 2w + 1 of the chunk (U
// gathered rows in flight, folded in edge order with separately rounded
// products and adds: mgcn_spmm_fwd / _bwd bit for bit) into the images;
// barrier; the previous chunk's staged rows leave as whole 1-KB rows (the
// ReLU mask words from four ballots; backward: the lower layer's mask,
// column sums and divisor applied on the staged row); Phase B -- wave w
// multiplies the chunk by its 32 output columns on v_mfma_f32_16x16x32_bf16
// (bf16x6) and stages the result.
//
// ReLU mask words at F = 256: [rows][8] u32, feature f at word
// 4 (f >> 7) + (f & 3), bit (f & 127) >> 2 (the F <= 128 layout, twice).
//
// Roofline: HBM-bound like the SpMM (B_spmm = 8 (N + 1) + nnz (8 + 4F) +
// 4 N F; + 4 N F for Z, + 32 N for the masks); 2 N F^2 x 6 bf16 MFMA flops
// and 24 KB of L2-resident W fragments per row ride under the gathers.

#include "mgcn_internal.h"
#include "x6.h"

namespace mgcn {

// mgcn_set_option("wide_pair"): both rows of a wave's pair gathered together
// or one after the other -- bit 0 the forward, bit 1 the adjoint (default 3:
// both paired).  Gathered rows in flight per row and round: 4 (5 / 6 / 8
// measured slower, round 5, and removed)
int g_wide_pair = 3;
constexpr int kWideU = 4;
// mgcn_set_option("wide_ws"): the warp-specialised kernels (below) -- bit 0
// the forward, bit 1 the adjoint
int g_wide_ws = 3;
// mgcn_set_option("wide_dbg"): timing experiments on the warp-specialised
// kernels (results are WRONG when set): bit 0 the MFMA waves skip their W
// loads, bit 1 they skip the products, bit 2 the gather waves skip the gathers;
// bits 3 / 4: s_setprio 2 on the gather / MFMA waves (results stay exact)
int g_wide_dbg = 0;
// mgcn_set_option("wide_mfma"): MFMA waves of the warp-specialised kernels (4 or 8)
int g_wide_mfma = 8;

int wide_set_option(const char *name, int value) {
  if (name[5] == 'm') {
    if (value != 4 && value != 8) {
      set_error("wide_mfma must be 4 or 8");
      return MGCN_EINVAL;
    }
    g_wide_mfma = value;
    return MGCN_OK;
  }
  if (name[5] == 'd') {  // (timing experiments: results WRONG when set)
    if (!MGCN_EXPERIMENT) {
      set_error("wide_dbg: experiment builds only (make exp -> libmgcn_exp.so)");
      return MGCN_EINVAL;
    }
    g_wide_dbg = value;
    return MGCN_OK;
  }
  if (name[5] == 'w') {
    if (value < 0 || value > 3) {
      set_error("wide_ws must be 0 .. 3");
      return MGCN_EINVAL;
    }
    g_wide_ws = value;
    return MGCN_OK;
  }
  if (value < 0 || value > 3) {  // "wide_pair"
    set_error("wide_pair must be 0 .. 3");
    return MGCN_EINVAL;
  }
  g_wide_pair = value;
  return MGCN_OK;
}

namespace {

using namespace x6;

constexpr int kWF = 256;
constexpr int kWRows = 16;
constexpr int kWWaves = 8;
constexpr int kWThreads = 64 * kWWaves;
constexpr int kWImg = kWRows * kWF * 2;           // one bf16 term image: 8 KB
constexpr int kWBuf = 3 * kWImg;                  // a chunk's three images: 24 KB
constexpr int kWStage = kWRows * kWF * 4;         // fp32 staging tile: 16 KB
constexpr int kWStageOff = 2 * kWBuf;
constexpr int kWLds = kWStageOff + 2 * kWStage;   // 80 KB
static_assert(2 * kWLds <= 160 * 1024, "two wide workgroups per CU");
constexpr int kWKs = kWF / 32;                    // k-steps of 16x16x32
constexpr int kWNt = kWF / 16;                    // 16-column n-tiles
constexpr int kWImgFrags = kWKs * kWNt * 3 * 64;  // 16-B fragments of the W image
constexpr int kWMaskWords = 8;                    // mask words per row

constexpr int WEPI_STORE = 0, WEPI_RELU = 1, WEPI_RELU_DIV = 2;
// Y / Z rows leave with the nt cache policy, as in fused.hip (a 51-GB table
// never stays in the Infinity Cache anyway)
constexpr int kWideNt = 2;

__device__ __forceinline__ int wimg_off(int row, int ch) {
  return 512 * row + 16 * (ch ^ (row & 15));
}
__device__ __forceinline__ int wstage(int row, int col) {
  return row * kWF + (col ^ (((row >> 2) & 3) << 4));
}

// W (B[k][n] = W[k][n], the forward) or W^T (B[k][n] = W[n][k], the
// adjoint's dX = dH W^T) split into bf16 terms in MFMA fragment order:
// fragment ((ks * 16 + nt) * 3 + term) * 64 + lane holds, for lane
// (g4 = lane >> 4, l16 = lane & 15), B[32 ks + 8 g4 + j][16 nt + l16], j < 8.
__global__ __launch_bounds__(256) void wide_wimg_kernel(const float *__restrict__ W, int64_t ldw,
                                                        int trans, u32x4 *__restrict__ img) {
  const int idx = (int)(blockIdx.x * 256 + threadIdx.x);
  if (idx >= kWKs * kWNt * 64) return;
  const int lane = idx & 63, nt = (idx >> 6) & (kWNt - 1), ks = idx >> 10;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int n = 16 * nt + l16;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 32 * ks + 8 * g4 + j;
    v[j] = trans ? W[(int64_t)n * ldw + k] : W[(int64_t)k * ldw + n];
  }
  bf16x8 h, m, l;
  split3_bf16(v, h, m, l);
  u32x4 *o = img + ((ks * kWNt + nt) * 3) * 64 + lane;
  o[0] = __builtin_bit_cast(u32x4, h);
  o[64] = __builtin_bit_cast(u32x4, m);
  o[128] = __builtin_bit_cast(u32x4, l);
}

struct WideArgs {
  int64_t n_rows;
  const int64_t *rowptr;
  const int32_t *col;
  const float *w;         // per-slot weights, nullable
  const float *X;         // gathered table (X forward, dY backward), rows of ldx floats
  int64_t ldx;
  const u32x4 *wimg;      // wide_wimg_kernel's image (W forward, W^T backward)
  const float *bias;      // forward, nullable
  float *Y;               // forward Y / backward dX
  int64_t ldy;
  uint32_t *mask_out;     // forward: [n_rows][8] ReLU mask words, nullable
  float *Z;               // forward: the aggregate, nullable
  int64_t ldz;
  const float *row_scale;      // backward 'rw' post-scale, nullable
  const uint32_t *mask_in;     // backward: the lower layer's [n_rows][8] mask words
  const float *row_div;        // backward mean divisor
  float *colsum_partial;       // backward: [grid][256]
  int mean, relu;
  int dbg;                     // wide_dbg (experiment builds only; masked by kDbgMask)
  uint32_t spin;               // warp-specialised hand-off spin bound (g_spin_limit)
  unsigned *err;               // device error word: kDevErrWide when a hand-off gave up
  // packed table (mgcn_packed_table; the warp-specialised kernels, PK): X is
  // then unused and col holds (segment << pk_rbits) | row
  const uint32_t *pk;
  int64_t pk_words;
  int pk_nseg;
  uint32_t pk_rbits, pk_head;
  int64_t pk_base[64];         // segment word offsets (mgcn_packed_table.seg_base)
};

// a row's edge slots: [beg, beg + deg) (wave-uniform), and lane l's slot
// beg + l (col, weight) of the first 64
struct WRow {
  int64_t beg;
  int64_t deg;
  int mc;
  float mw;
};

__device__ __forceinline__ void wrow_ptr(const int64_t *__restrict__ rowptr, int64_t row, bool ok,
                                         WRow &m) {
  m.beg = ok ? rowptr[row] : 0;
  m.deg = ok ? rowptr[row + 1] - m.beg : 0;
}

__device__ __forceinline__ void wrow_first(const int32_t *__restrict__ col,
                                           const float *__restrict__ w, int lane, WRow &m) {
  m.mc = 0;
  m.mw = 1.0f;
  if (lane < m.deg) {
    m.mc = col[m.beg + lane];
    if (w != nullptr) m.mw = w[m.beg + lane];
  }
}

// acc = sum_k X[col_k] * w_k over the row's slots in order (products and
// sums rounded separately): lane l holds features 4 l .. 4 l + 3
template <int U>
__device__ __forceinline__ void wide_gather(const float *__restrict__ X, int64_t ldx,
                                            const int32_t *__restrict__ col,
                                            const float *__restrict__ w, const WRow &m, int lane,
                                            float (&acc)[4]) {
  acc[0] = acc[1] = acc[2] = acc[3] = 0.0f;
  int mc = m.mc;
  float mw = m.mw;
  const int64_t deg = m.deg;
  for (int64_t e0 = 0; e0 < deg; e0 += 64) {
    if (e0 > 0) {  // rows longer than one metadata batch load the rest in place
      mc = 0;
      mw = 1.0f;
      if (e0 + lane < deg) {
        mc = col[m.beg + e0 + lane];
        if (w != nullptr) mw = w[m.beg + e0 + lane];
      }
    }
    const int nb = (int)(deg - e0 < 64 ? deg - e0 : 64);  // wave-uniform
    for (int k0 = 0; k0 < nb; k0 += U) {
      float4 xv[U];
      float wk[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = (k0 + u) & 63;
        const int ck = __builtin_amdgcn_readlane(mc, k);
        wk[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mw), k));
        // the row's own resource (64-bit base in SGPRs); slots past the row
        // end get a zero-byte one: the load returns 0 and moves no bytes
        const auto rs = buf_rsrc(X + (int64_t)ck * ldx, k0 + u < nb ? kWF * 4 : 0);
        xv[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u < nb) {  // wave-uniform: strictly ascending edge order
          acc[0] = __fadd_rn(acc[0], __fmul_rn(xv[u].x, wk[u]));
          acc[1] = __fadd_rn(acc[1], __fmul_rn(xv[u].y, wk[u]));
          acc[2] = __fadd_rn(acc[2], __fmul_rn(xv[u].z, wk[u]));
          acc[3] = __fadd_rn(acc[3], __fmul_rn(xv[u].w, wk[u]));
        }
      }
    }
  }
}

// Both rows of a wave's pair gathered together (PAIR kernels): U slots of
// EACH row in flight per round, so a wave keeps 2 U gathered 1-KB rows in
// flight instead of U -- one wave's rows are the chunk's rows 2 w and 2 w + 1,
// and alone each pays its dependent round trips (deg 11 at U = 4: three)
// while the other waits.  Each row is still folded in its own edge order
// with separately rounded products and adds (bit for bit wide_gather).
template <int U>
__device__ __forceinline__ void wide_gather2(const float *__restrict__ X, int64_t ldx,
                                             const int32_t *__restrict__ col,
                                             const float *__restrict__ w, const WRow &ma,
                                             const WRow &mb, int lane, float (&aa)[4],
                                             float (&ab)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) aa[j] = ab[j] = 0.0f;
  int mca = ma.mc, mcb = mb.mc;
  float mwa = ma.mw, mwb = mb.mw;
  const int64_t da = ma.deg, db = mb.deg;
  const int64_t dm = da > db ? da : db;
  for (int64_t e0 = 0; e0 < dm; e0 += 64) {
    if (e0 > 0) {  // rows longer than one metadata batch load the rest in place
      mca = mcb = 0;
      mwa = mwb = 1.0f;
      if (e0 + lane < da) {
        mca = col[ma.beg + e0 + lane];
        if (w != nullptr) mwa = w[ma.beg + e0 + lane];
      }
      if (e0 + lane < db) {
        mcb = col[mb.beg + e0 + lane];
        if (w != nullptr) mwb = w[mb.beg + e0 + lane];
      }
    }
    const int na = (int)(da - e0 <= 0 ? 0 : da - e0 < 64 ? da - e0 : 64);  // wave-uniform
    const int nb = (int)(db - e0 <= 0 ? 0 : db - e0 < 64 ? db - e0 : 64);
    const int nm = na > nb ? na : nb;
    for (int k0 = 0; k0 < nm; k0 += U) {
      float4 xa[U], xb[U];
      float wa[U], wb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = (k0 + u) & 63;
        const int ca = __builtin_amdgcn_readlane(mca, k);
        const int cb = __builtin_amdgcn_readlane(mcb, k);
        wa[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mwa), k));
        wb[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mwb), k));
        // a 64-bit scalar row base + the lane's 16-B offset (global_load
        // saddr form: 2 SGPRs per load, no buffer resource); a slot past a
        // row's end reads row col = 0 of its batch (loaded, never folded)
        const float4 *pa = reinterpret_cast<const float4 *>(X + (int64_t)ca * ldx) + lane;
        const float4 *pb = reinterpret_cast<const float4 *>(X + (int64_t)cb * ldx) + lane;
        xa[u] = *pa;
        xb[u] = *pb;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u < na) {  // wave-uniform: strictly ascending edge order per row
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

// ---------------------------------------------------------------------------
// In-place gather from a PACKED table (round 6; mgcn_packed_table, pack.hip's
// layout).  Gathered row col = (s << rbits) | i is row i of packed segment s,
// which starts at word base[s] of the buffer; the wave holds base[0 .. 63]
// lane-resident (lane s: base[s], loaded once) and takes a row's base with
// two v_readlane -- the row's whole address stays in SGPRs, as the dense
// gather's does.  Lane l (words 4 l .. 4 l + 3 of the row) reads the pair
// (mask_w, pos_w), w = l / 8, of the row's header (8 B), then 16 B of values
// at pos_w + popc(mask_w below bit 4 (l % 8)) -- its own nonzero words first,
// any excess belongs to the lanes above and is dropped -- and puts each word
// back where its mask bit says, +0.0 elsewhere: exactly the dense row, so the
// fold below is wide_gather2's, bit for bit.  Per row pair and U-slot batch:
// the headers of batch k + 1 are issued under batch k's value loads.
struct PkView {
  const uint32_t *words;
  uint32_t rbits;   // col = (s << rbits) | i
  uint32_t head;    // header words of a segment (seg_rows x 16)
  uint32_t base_lo, base_hi;  // lane-resident: base[lane] (word offset of segment `lane`)
  uint32_t bytes;             // lane-resident: readable bytes from that segment's start
};

// segment `lane`'s base and readable bytes (once per wave).  The range is
// capped at 2 GiB: every in-segment offset is below that (the
// mgcn_spmm_xw_*_packed check), so the 0xfffffff0 "no load" offset below
// always falls outside it (a cap at 4 GiB would let it read the last bytes
// before the cap -- unmapped memory when the buffers lie far apart)
__device__ __forceinline__ void pk_view_init(PkView &pv, const uint32_t *words, int64_t n_words,
                                             int n_seg, uint32_t rbits, uint32_t head,
                                             int64_t base, int lane) {
  pv.words = words;
  pv.rbits = rbits;
  pv.head = head;
  pv.base_lo = (uint32_t)base;
  pv.base_hi = (uint32_t)((uint64_t)base >> 32);
  const int64_t avail = n_words - base;
  pv.bytes = lane >= n_seg || avail <= 0 ? 0u
             : avail >= (int64_t)0x1ffffffc ? 0x7ffffff0u : (uint32_t)avail * 4u;
}

// the range of packed row `col` (its segment) and the row's index in it; a
// zero-byte range when !ok.  Everything here is wave-uniform (SGPRs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pk_rsrc(const PkView &pv, int col, bool ok,
                                                          uint32_t &row) {
  const uint32_t c = (uint32_t)col;
  const int s = (int)(c >> pv.rbits);
  row = c & ((1u << pv.rbits) - 1u);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)pv.base_lo, s);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)pv.base_hi, s);
  const uint32_t bytes = (uint32_t)__builtin_amdgcn_readlane((int)pv.bytes, s);
  const uint32_t *p = pv.words + (int64_t)(((uint64_t)hi << 32) | lo);
  // (through readfirstlane, as buf_rsrc: provably uniform even where the
  // compiler parks the parts in VGPRs -- else it wraps the load in a waterfall
  // loop that waits for every load in flight)
  return buf_rsrc(p, ok ? bytes : 0u);
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// the byte offset of the lane's header pair within a row header (w = lane / 8)
__device__ __forceinline__ uint32_t pk_hoff(int lane) { return 8u * (uint32_t)(lane >> 3); }

// the header pairs of U slots k0 .. of a row pair (slots past na / nb: a
// zero-byte range, the pair reads 0)
template <int U>
__device__ __forceinline__ void pk_headers(const PkView &pv, int mca, int mcb, int k0, int na,
                                           int nb, uint32_t hoff, u32x2 (&ha)[U],
                                           u32x2 (&hb)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = (k0 + u) & 63;
    uint32_t ia, ib;
    const auto ra = pk_rsrc(pv, __builtin_amdgcn_readlane(mca, k), k0 + u < na, ia);
    const auto rb = pk_rsrc(pv, __builtin_amdgcn_readlane(mcb, k), k0 + u < nb, ib);
    ha[u] = __builtin_amdgcn_raw_buffer_load_b64(ra, 64u * ia + hoff, 0, 0);
    hb[u] = __builtin_amdgcn_raw_buffer_load_b64(rb, 64u * ib + hoff, 0, 0);
  }
}

// ha / hb hold, on entry, the header pairs of the first U slots of (ma, mb)
// -- issued by the caller for the first pair, by the previous call for the
// others -- and, on return, those of the next pair (na, nb), issued under this
// pair's last value loads: a row pair then costs the dense gather's round
// trips (one per batch), not one more for its first headers
template <int U>
__device__ __forceinline__ void wide_gather2_pk(const PkView &pv, const int32_t *__restrict__ col,
                                                const float *__restrict__ w, const WRow &ma,
                                                const WRow &mb, const WRow &na_, const WRow &nb_,
                                                int lane, float (&aa)[4], float (&ab)[4],
                                                u32x2 (&ha)[U], u32x2 (&hb)[U]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) aa[j] = ab[j] = 0.0f;
  int mca = ma.mc, mcb = mb.mc;
  float mwa = ma.mw, mwb = mb.mw;
  // (row degrees are wave-uniform: in SGPRs, the batch branches are scalar)
  const int64_t da = uniform64(ma.deg), db = uniform64(mb.deg);
  const int64_t dm = da > db ? da : db;
  const uint32_t hoff = pk_hoff(lane);
  const uint32_t sh = 4u * (uint32_t)(lane & 7);  // the lane's nibble in mask_w
  const uint32_t below = (1u << sh) - 1u;
  const int64_t dna = uniform64(na_.deg), dnb = uniform64(nb_.deg);
  const int nxa = (int)(dna < 64 ? dna : 64), nxb = (int)(dnb < 64 ? dnb : 64);
  // (an empty pair still runs one all-masked batch: the next pair's headers
  // are then issued from the one call site below -- two call sites let the
  // compiler merge their operands into VGPR phis and wrap the loads in
  // waterfall loops)
  const int64_t dm1 = dm > 0 ? dm : 1;
  for (int64_t e0 = 0; e0 < dm1; e0 += 64) {
    const int na = (int)(da - e0 <= 0 ? 0 : da - e0 < 64 ? da - e0 : 64);  // wave-uniform
    const int nb = (int)(db - e0 <= 0 ? 0 : db - e0 < 64 ? db - e0 : 64);
    const int nm = na > nb ? na : nb;
    const int nm1 = nm > 0 ? nm : 1;
    if (e0 > 0) {  // rows longer than one metadata batch load the rest in place
      mca = mcb = 0;
      mwa = mwb = 1.0f;
      if (e0 + lane < da) {
        mca = col[ma.beg + e0 + lane];
        if (w != nullptr) mwa = w[ma.beg + e0 + lane];
      }
      if (e0 + lane < db) {
        mcb = col[mb.beg + e0 + lane];
        if (w != nullptr) mwb = w[mb.beg + e0 + lane];
      }
      pk_headers<U>(pv, mca, mcb, 0, na, nb, hoff, ha, hb);
    }
    const bool last_window = e0 + 64 >= dm1;
    for (int k0 = 0; k0 < nm1; k0 += U) {
      u32x4 va[U], vb[U];
      uint32_t nia[U], nib_b[U];
      float wa[U], wb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = (k0 + u) & 63;
        wa[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mwa), k));
        wb[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mwb), k));
        uint32_t ia, ib;
        const auto ra = pk_rsrc(pv, __builtin_amdgcn_readlane(mca, k), k0 + u < na, ia);
        const auto rb = pk_rsrc(pv, __builtin_amdgcn_readlane(mcb, k), k0 + u < nb, ib);
        nia[u] = (ha[u][0] >> sh) & 0xfu;
        nib_b[u] = (hb[u][0] >> sh) & 0xfu;
        const uint32_t qa = ha[u][1] + (uint32_t)__builtin_popcount(ha[u][0] & below);
        const uint32_t qb = hb[u][1] + (uint32_t)__builtin_popcount(hb[u][0] & below);
        // a lane with no nonzero word moves no bytes (offset past the range)
        va[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, nia[u] ? 4u * (pv.head + qa) : 0xfffffff0u, 0, 0);
        vb[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, nib_b[u] ? 4u * (pv.head + qb) : 0xfffffff0u, 0, 0);
      }
      // the next headers, under these values: this window's next batch, or
      // (the last batch of the last window) the next pair's first -- one call
      // site, its inputs selected
      const bool more = k0 + U < nm;
      if (more || last_window) {
        const int sa = more ? mca : na_.mc, sb = more ? mcb : nb_.mc;
        pk_headers<U>(pv, sa, sb, more ? k0 + U : 0, more ? na : nxa, more ? nb : nxb, hoff, ha,
                      hb);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u < na) {  // wave-uniform: strictly ascending edge order per row
          const float4 x = pk_expand(nia[u], va[u]);
          aa[0] = __fadd_rn(aa[0], __fmul_rn(x.x, wa[u]));
          aa[1] = __fadd_rn(aa[1], __fmul_rn(x.y, wa[u]));
          aa[2] = __fadd_rn(aa[2], __fmul_rn(x.z, wa[u]));
          aa[3] = __fadd_rn(aa[3], __fmul_rn(x.w, wa[u]));
        }
        if (k0 + u < nb) {
          const float4 x = pk_expand(nib_b[u], vb[u]);
          ab[0] = __fadd_rn(ab[0], __fmul_rn(x.x, wb[u]));
          ab[1] = __fadd_rn(ab[1], __fmul_rn(x.y, wb[u]));
          ab[2] = __fadd_rn(ab[2], __fmul_rn(x.z, wb[u]));
          ab[3] = __fadd_rn(ab[3], __fmul_rn(x.w, wb[u]));
        }
      }
    }
  }
}

// one 16-row chunk's W fragments of k-step ks for this wave's two n-tiles
struct WFrag {
  u32x4 t[2][3];
};

__device__ __forceinline__ void load_wfrag(const __amdgpu_buffer_rsrc_t rw, int wave, int ks,
                                           int lane, WFrag &f) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int term = 0; term < 3; ++term)
      f.t[t][term] = __builtin_amdgcn_raw_buffer_load_b128(
          rw, 16 * ((((ks * kWNt + 2 * wave + t) * 3) + term) * 64 + lane), 0, 0);
}

template <int U, bool BWD, int EPI, bool PAIR>
__global__ __launch_bounds__(kWThreads, 4) void spmm_xw_wide_kernel(const WideArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[kWLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g4 = lane >> 4;
  const int64_t n_chunks = (a.n_rows + kWRows - 1) / kWRows;
  const auto rw = buf_rsrc(a.wimg, (uint32_t)(kWImgFrags * 16));
  const bool has_b = !BWD && a.bias != nullptr;
  float bcol[2] = {0.0f, 0.0f};
  if (has_b) {
    bcol[0] = a.bias[32 * wave + l16];
    bcol[1] = a.bias[32 * wave + 16 + l16];
  }
  auto rows_in = [&](int64_t c) -> uint32_t {
    const int64_t r = a.n_rows - c * kWRows;
    return (uint32_t)(r <= 0 ? 0 : r >= kWRows ? kWRows : r);
  };

  // backward epilogue state: the flushed rows' mask words / divisors are
  // loaded at the start of the iteration (under the gathers), the column
  // sums of this thread's four features (rows w and w + 8 of its chunks)
  float cs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  u32x4 mk[2] = {};
  float dv[2] = {1.0f, 1.0f};
  auto prefetch_epi = [&](int64_t c) {
    if constexpr (BWD && EPI != WEPI_STORE) {
      const int64_t r0 = c * kWRows;
      const uint32_t rv = rows_in(c);
      const auto rm = buf_rsrc(a.mask_in + r0 * kWMaskWords, rv * kWMaskWords * 4u);
#pragma unroll
      for (int m = 0; m < 2; ++m)
        mk[m] = __builtin_amdgcn_raw_buffer_load_b128(
            rm, 4 * ((wave + 8 * m) * kWMaskWords + 4 * (lane >> 5)), 0, 0);
      if constexpr (EPI == WEPI_RELU_DIV) {
        const auto rd = buf_rsrc(a.row_div + r0, rv * 4u);
#pragma unroll
        for (int m = 0; m < 2; ++m)
          dv[m] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rd, 4 * (wave + 8 * m), 0, 0));
      }
    }
  };

  // staged rows of chunk c leave as whole 1-KB rows: wave w takes rows w, w + 8
  auto flush = [&](int64_t c, const float *stage) {
    const int64_t r0 = c * kWRows;
    const uint32_t rv = rows_in(c);
    const auto ry = buf_rsrc(a.Y + r0 * a.ldy, rv * (uint32_t)a.ldy * 4u);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int lr = wave + 8 * m;
      float v[4];
      *reinterpret_cast<float4 *>(v) = *reinterpret_cast<const float4 *>(stage + wstage(lr, 4 * lane));
      if constexpr (BWD && EPI != WEPI_STORE) {
        // feature 4 lane + j: word 4 (lane >> 5) + j, bit lane & 31
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = ((mk[m][j] >> (lane & 31)) & 1u) ? v[j] : 0.0f;
          cs[j] = __fadd_rn(cs[j], v[j]);  // rows past the end staged zeros
        }
        if constexpr (EPI == WEPI_RELU_DIV) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = __fdiv_rn(v[j], dv[m]);
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, *reinterpret_cast<float4 *>(v)),
                                             ry, 4 * (int)(lr * a.ldy + 4 * lane), 0, kWideNt);
      if constexpr (!BWD) {
        if (a.mask_out != nullptr) {
          const uint64_t b0 = __ballot(v[0] > 0.0f), b1 = __ballot(v[1] > 0.0f);
          const uint64_t b2 = __ballot(v[2] > 0.0f), b3 = __ballot(v[3] > 0.0f);
          if (lane == 0 && (uint32_t)lr < rv) {
            uint4 *mo = reinterpret_cast<uint4 *>(a.mask_out + (r0 + lr) * kWMaskWords);
            mo[0] = make_uint4((uint32_t)b0, (uint32_t)b1, (uint32_t)b2, (uint32_t)b3);
            mo[1] = make_uint4((uint32_t)(b0 >> 32), (uint32_t)(b1 >> 32), (uint32_t)(b2 >> 32),
                               (uint32_t)(b3 >> 32));
          }
        }
      }
    }
  };

  const int64_t n_my = blockIdx.x < n_chunks ? (n_chunks - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  // the rows of this wave in order: row k = chunk (k >> 1) of this workgroup, row 2 wave + (k & 1)
  auto row_of = [&](int64_t k) -> int64_t {
    return ((int64_t)blockIdx.x + (k >> 1) * gridDim.x) * kWRows + 2 * wave + (k & 1);
  };
  // row pipeline: one row (PAIR = false) or the wave's pair (PAIR) ahead --
  // the next rows' first edge slots and the pointers of the rows after them
  // load under the current gathers
  WRow cur, nxt, cur2, nxt2;
  if constexpr (PAIR) {
    wrow_ptr(a.rowptr, row_of(0), row_of(0) < a.n_rows, cur);
    wrow_ptr(a.rowptr, row_of(1), row_of(1) < a.n_rows, cur2);
    wrow_first(a.col, a.w, lane, cur);
    wrow_first(a.col, a.w, lane, cur2);
    wrow_ptr(a.rowptr, row_of(2), row_of(2) < a.n_rows && 1 < n_my, nxt);
    wrow_ptr(a.rowptr, row_of(3), row_of(3) < a.n_rows && 1 < n_my, nxt2);
  } else {
    wrow_ptr(a.rowptr, row_of(0), row_of(0) < a.n_rows, cur);
    wrow_first(a.col, a.w, lane, cur);
    wrow_ptr(a.rowptr, row_of(1), row_of(1) < a.n_rows && 1 < 2 * n_my, nxt);
  }
  int it = 0;
  for (int64_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x, ++it) {
    char *buf = lds + (it & 1) * kWBuf;
    const int64_t r0 = chunk * kWRows;
    if (it > 0) prefetch_epi(chunk - gridDim.x);
    // a finished row (lane: features 4 lane .. + 3) -> Z / scaling -> images
    auto finish_row = [&](int lr, float (&acc)[4], int64_t deg) {
      const bool row_ok = r0 + lr < a.n_rows;
      if constexpr (!BWD) {
        if (a.Z != nullptr) {
          const auto rz = buf_rsrc(a.Z + r0 * a.ldz, rows_in(chunk) * (uint32_t)a.ldz * 4u);
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4, make_float4(acc[0], acc[1], acc[2], acc[3])), rz,
              4 * (int)(lr * a.ldz + 4 * lane), 0, kWideNt);
        }
        if (a.mean) {
          const float c = (float)(deg > 1 ? deg : 1);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = __fdiv_rn(acc[j], c);
        }
      } else {
        if (a.row_scale != nullptr && row_ok) {
          const float sc = a.row_scale[r0 + lr];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = __fmul_rn(acc[j], sc);
        }
      }
      uint32_t hi[2], mid[2], lo[2];
      split3_pair(f32x2{acc[0], acc[1]}, hi[0], mid[0], lo[0]);
      split3_pair(f32x2{acc[2], acc[3]}, hi[1], mid[1], lo[1]);
      char *img = buf + wimg_off(lr, lane >> 1) + 8 * (lane & 1);
      *reinterpret_cast<uint2 *>(img) = make_uint2(hi[0], hi[1]);
      *reinterpret_cast<uint2 *>(img + kWImg) = make_uint2(mid[0], mid[1]);
      *reinterpret_cast<uint2 *>(img + 2 * kWImg) = make_uint2(lo[0], lo[1]);
    };
    // ---- Phase A: the chunk's rows -> bf16 term images ------------------
    if constexpr (PAIR) {
      wrow_first(a.col, a.w, lane, nxt);
      wrow_first(a.col, a.w, lane, nxt2);
      WRow nn, nn2;
      const int64_t ra = row_of(2 * (int64_t)it + 4), rb = row_of(2 * (int64_t)it + 5);
      wrow_ptr(a.rowptr, ra, ra < a.n_rows && it + 2 < n_my, nn);
      wrow_ptr(a.rowptr, rb, rb < a.n_rows && it + 2 < n_my, nn2);
      float acc[4], acc2r[4];
      wide_gather2<U>(a.X, a.ldx, a.col, a.w, cur, cur2, lane, acc, acc2r);
      finish_row(2 * wave, acc, cur.deg);
      finish_row(2 * wave + 1, acc2r, cur2.deg);
      cur = nxt;
      cur2 = nxt2;
      nxt = nn;
      nxt2 = nn2;
    } else {
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const int lr = 2 * wave + p;
        const int64_t k = 2 * it + p;
        wrow_first(a.col, a.w, lane, nxt);
        WRow nn;
        const int64_t rk2 = row_of(k + 2);
        wrow_ptr(a.rowptr, rk2, rk2 < a.n_rows && k + 2 < 2 * n_my, nn);
        float acc[4];
        wide_gather<U>(a.X, a.ldx, a.col, a.w, cur, lane, acc);
        finish_row(lr, acc, cur.deg);
        cur = nxt;
        nxt = nn;
      }
    }
    // the first k-step's W fragments, in flight across the barrier
    WFrag fc, fn;
    load_wfrag(rw, wave, 0, lane, fc);
    __syncthreads();
    // the previous chunk's staged rows go out
    if (it > 0)
      flush(chunk - gridDim.x,
            reinterpret_cast<const float *>(lds + kWStageOff + ((it + 1) & 1) * kWStage));

    // ---- Phase B: the chunk (16 x 256) times this wave's 32 columns ------
    f32x4_t acc2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc2[t][r] = 0.0f;
#pragma unroll
    for (int ks = 0; ks < kWKs; ++ks) {
      if (ks + 1 < kWKs) load_wfrag(rw, wave, ks + 1, lane, fn);
      const int off = wimg_off(l16, 4 * ks + g4);
      const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(buf + off);
      const bf16x8 am = *reinterpret_cast<const bf16x8 *>(buf + kWImg + off);
      const bf16x8 al = *reinterpret_cast<const bf16x8 *>(buf + 2 * kWImg + off);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc2[t] = mfma16_x6(ah, am, al, __builtin_bit_cast(bf16x8, fc.t[t][0]),
                            __builtin_bit_cast(bf16x8, fc.t[t][1]),
                            __builtin_bit_cast(bf16x8, fc.t[t][2]), acc2[t]);
      if (ks + 1 < kWKs) fc = fn;
    }
    float *stage = reinterpret_cast<float *>(lds + kWStageOff + (it & 1) * kWStage);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc2[t][r];
        if constexpr (!BWD) {
          if (has_b) v = __fadd_rn(v, bcol[t]);
          if (a.relu) v = (v < 0.0f) ? 0.0f : v;
        }
        stage[wstage(4 * g4 + r, 32 * wave + 16 * t + l16)] = v;
      }
  }
  if (it > 0) {
    prefetch_epi(blockIdx.x + (int64_t)(it - 1) * gridDim.x);
    __syncthreads();
    flush(blockIdx.x + (int64_t)(it - 1) * gridDim.x,
          reinterpret_cast<const float *>(lds + kWStageOff + ((it + 1) & 1) * kWStage));
  }
  if constexpr (BWD && EPI != WEPI_STORE) {
    // column sums: fold the eight waves of each feature in wave order
    __syncthreads();
    float *red = reinterpret_cast<float *>(lds);  // [8 waves][256]
    *reinterpret_cast<float4 *>(red + wave * kWF + 4 * lane) = make_float4(cs[0], cs[1], cs[2], cs[3]);
    __syncthreads();
    if (tid < kWF) {
      float c = 0.0f;
#pragma unroll
      for (int w = 0; w < kWWaves; ++w) c = __fadd_rn(c, red[w * kWF + tid]);
      a.colsum_partial[(int64_t)blockIdx.x * kWF + tid] = c;
    }
  }
}

// ===================== warp-specialised form (round 5) =====================
//
// The kernel above pays for its 16-row chunks twice: every chunk streams the
// whole W image from L2 (384 KB per 16 rows = 24 KB per row, twice the
// gathered bytes), and every wave stops gathering for the chunk's barrier and
// Phase B.  Here one 1024-thread workgroup per CU splits the work by role:
//
// * 12 GATHER waves take the workgroup's row pairs in turn (pair p = rows
//   2 (p & 15), + 1 of its chunk p >> 4; wave g: p = g, g + 12, ...), each
//   pair's U slots per row in flight (wide_gather2, bit for bit the SpMM's
//   fold), write Z and the rows' bf16 term images into a ring of three
//   32-row chunk buffers (48 KB each), and count the rows in (filled[b]).
//   They never wait for the MFMAs except when the ring is full.
// * 4 MFMA waves (one per SIMD) take the chunks in order: wave m computes the
//   32 rows x its 64 output columns as D = W^T-image x rows (the rows are the
//   B operand, so a lane's D fragment is 4 CONSECUTIVE columns of one row and
//   leaves as one 16-B store -- no staging tile), each W fragment serving both
//   16-row tiles: 384 KB of W per 32 rows, half the L2 stream.  The epilogue
//   (bias, ReLU, mask ballots -- combined across the two waves of a 128-column
//   half by ds_or in LDS; backward: the lower layer's mask, column sums,
//   divisor) runs on the fragments; the last wave out of a chunk writes its
//   mask words and frees the buffer (freed[b]).
//
// Hand-offs are LDS counters inside the workgroup (monotonic per buffer; a
// wave's LDS operations complete in order, so its image writes land before
// its counter add), polled with s_sleep and bounded: a spin that exceeds
// the bound (g_spin_limit) sets the abort word and every wave leaves its loop.  The MFMA
// term order is the 16-row kernel's with the operands swapped (the same six
// products per k-step in the same order), so Y / dX equal its results.
constexpr int kSRows = 32;
constexpr int kSBufs = 3;
constexpr int kSImg = kSRows * kWF * 2;     // one term image of a chunk: 16 KB
constexpr int kSBuf = 3 * kSImg;            // 48 KB
constexpr int kSThreads = 1024;  // 16 waves: 16 - NM gather, NM MFMA
constexpr int kSMaskOff = kSBufs * kSBuf;                                 // [3][32][8] u32
constexpr int kSCtrOff = kSMaskOff + kSBufs * kSRows * kWMaskWords * 4;  // counters
constexpr int kSLds = kSCtrOff + 64;
static_assert(kSLds <= 160 * 1024, "one warp-specialised workgroup per CU");
static_assert(16 * kWF * 4 <= kSMaskOff, "column-sum fold fits in the image ring");

// the 16-row kernel's six products (rows_l W_h, rows_h W_l, rows_m W_m,
// rows_m W_h, rows_h W_m, rows_h W_h) with W as the A operand
__device__ __forceinline__ f32x4_t mfma16_x6_wt(const u32x4 (&w)[3], const bf16x8 &xh,
                                               const bf16x8 &xm, const bf16x8 &xl, f32x4_t c) {
  const bf16x8 wh = __builtin_bit_cast(bf16x8, w[0]);
  const bf16x8 wm = __builtin_bit_cast(bf16x8, w[1]);
  const bf16x8 wl = __builtin_bit_cast(bf16x8, w[2]);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, xm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, xh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh, c, 0, 0, 0);
}

__device__ __forceinline__ int lds_load(const int *p) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

// wait until *p >= target (false: the abort word is set, leave)
__device__ __forceinline__ bool lds_wait_ge(const int *p, int target, int *abort_word,
                                            uint32_t limit) {
  for (uint32_t n = 0;; ++n) {
    if (lds_load(p) >= target) break;
    if (lds_load(abort_word) != 0) return false;
    if (n >= limit) {
      __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
  return true;
}

// this wave's LDS writes complete, then lane 0 adds v to *p; returns the old value
__device__ __forceinline__ int lds_signal(int *p, int v, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(old);
}

template <int U, bool BWD, int EPI, int NM, bool PK>
__global__ __launch_bounds__(kSThreads) void spmm_xw_wide_ws_kernel(const WideArgs a) {
  // NM MFMA waves (4 or 8), 16 - NM gather waves; MFMA wave m owns the NT
  // n-tiles NT m .. NT m + NT - 1 (16 NT output columns)
  constexpr int NG = 16 - NM;
  constexpr int NT = kWNt / NM;
  constexpr int KSI = 4 / NT;  // k-steps per ring turn (4 W steps)
  __shared__ __attribute__((aligned(16))) char lds[kSLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g4 = lane >> 4;
  int *ctr = reinterpret_cast<int *>(lds + kSCtrOff);
  int *filled = ctr, *mdone = ctr + 3, *freed = ctr + 6, *abort_word = ctr + 9;
  uint32_t *maskbuf = reinterpret_cast<uint32_t *>(lds + kSMaskOff);
  if (tid < 16) ctr[tid] = 0;
  __syncthreads();

  const int64_t n_chunks = (a.n_rows + kSRows - 1) / kSRows;
  const int64_t n_my = blockIdx.x < n_chunks ? (n_chunks - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  auto chunk_of = [&](int64_t i) { return (int64_t)blockIdx.x + i * gridDim.x; };
  auto rows_in = [&](int64_t c) -> uint32_t {
    const int64_t r = a.n_rows - c * kSRows;
    return (uint32_t)(r <= 0 ? 0 : r >= kSRows ? kSRows : r);
  };

  float cs[NT][4];  // backward column sums (MFMA waves)
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[t][r] = 0.0f;

  if (wave < NG) {
    // ------------------------------- gather waves ---------------------------
    if (a.dbg & kDbgMask & 8) __builtin_amdgcn_s_setprio(2);
    PkView pv{};
    if constexpr (PK)
      pk_view_init(pv, a.pk, a.pk_words, a.pk_nseg, a.pk_rbits, a.pk_head, a.pk_base[lane], lane);
    const int64_t n_pairs = 16 * n_my;
    auto pair_row = [&](int64_t p) { return chunk_of(p >> 4) * kSRows + 2 * (p & 15); };
    WRow cur, cur2, nxt, nxt2;
    {
      const int64_t p = wave, ra = pair_row(p);
      const bool ok = p < n_pairs;
      wrow_ptr(a.rowptr, ra, ok && ra < a.n_rows, cur);
      wrow_ptr(a.rowptr, ra + 1, ok && ra + 1 < a.n_rows, cur2);
      wrow_first(a.col, a.w, lane, cur);
      wrow_first(a.col, a.w, lane, cur2);
      const int64_t q = p + NG, rq = pair_row(q);
      wrow_ptr(a.rowptr, rq, q < n_pairs && rq < a.n_rows, nxt);
      wrow_ptr(a.rowptr, rq + 1, q < n_pairs && rq + 1 < a.n_rows, nxt2);
    }
    // PK: the header pairs of the current pair's first U slots (carried from
    // pair to pair by wide_gather2_pk)
    u32x2 pha[PK ? U : 1], phb[PK ? U : 1];
    if constexpr (PK) {
      const int64_t d0 = uniform64(cur.deg), d1 = uniform64(cur2.deg);
      pk_headers<U>(pv, cur.mc, cur2.mc, 0, (int)(d0 < 64 ? d0 : 64), (int)(d1 < 64 ? d1 : 64),
                    pk_hoff(lane), pha, phb);
    }
    for (int64_t p = wave; p < n_pairs; p += NG) {
      wrow_first(a.col, a.w, lane, nxt);
      wrow_first(a.col, a.w, lane, nxt2);
      WRow nn, nn2;
      const int64_t q = p + 2 * NG, rq = pair_row(q);
      wrow_ptr(a.rowptr, rq, q < n_pairs && rq < a.n_rows, nn);
      wrow_ptr(a.rowptr, rq + 1, q < n_pairs && rq + 1 < a.n_rows, nn2);
      float acc[2][4];
      if (a.dbg & kDbgMask & 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[0][j] = acc[1][j] = 0.0f;
      } else {
        if constexpr (PK)
          wide_gather2_pk<U>(pv, a.col, a.w, cur, cur2, nxt, nxt2, lane, acc[0], acc[1], pha, phb);
        else
          wide_gather2<U>(a.X, a.ldx, a.col, a.w, cur, cur2, lane, acc[0], acc[1]);
      }
      const int64_t i = p >> 4;
      const int b = (int)(i % kSBufs);
      const int gen = (int)(i / kSBufs);
      const int64_t c = chunk_of(i);
      const int64_t r0 = c * kSRows;
      const int lr0 = 2 * (int)(p & 15);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int lr = lr0 + k;
        const int64_t deg = k == 0 ? cur.deg : cur2.deg;
        if constexpr (!BWD) {
          if (a.Z != nullptr) {
            const auto rz = buf_rsrc(a.Z + r0 * a.ldz, rows_in(c) * (uint32_t)a.ldz * 4u);
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(u32x4, make_float4(acc[k][0], acc[k][1], acc[k][2], acc[k][3])),
                rz, 4 * (int)(lr * a.ldz + 4 * lane), 0, kWideNt);
          }
          if (a.mean) {
            const float dc = (float)(deg > 1 ? deg : 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[k][j] = __fdiv_rn(acc[k][j], dc);
          }
        } else {
          if (a.row_scale != nullptr && r0 + lr < a.n_rows) {
            const float sc = a.row_scale[r0 + lr];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[k][j] = __fmul_rn(acc[k][j], sc);
          }
        }
      }
      uint32_t hi[2][2], mid[2][2], lo[2][2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        split3_pair(f32x2{acc[k][0], acc[k][1]}, hi[k][0], mid[k][0], lo[k][0]);
        split3_pair(f32x2{acc[k][2], acc[k][3]}, hi[k][1], mid[k][1], lo[k][1]);
      }
      // the buffer's previous chunk has left the MFMA waves
      if (!lds_wait_ge(freed + b, gen, abort_word, a.spin)) break;
      char *buf = lds + b * kSBuf;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        char *img = buf + wimg_off(lr0 + k, lane >> 1) + 8 * (lane & 1);
        *reinterpret_cast<uint2 *>(img) = make_uint2(hi[k][0], hi[k][1]);
        *reinterpret_cast<uint2 *>(img + kSImg) = make_uint2(mid[k][0], mid[k][1]);
        *reinterpret_cast<uint2 *>(img + 2 * kSImg) = make_uint2(lo[k][0], lo[k][1]);
      }
      if constexpr (!BWD) {  // the rows' mask words start empty (the MFMA waves OR into them)
        if (lane < 2 * kWMaskWords) maskbuf[(b * kSRows + lr0) * kWMaskWords + lane] = 0u;
      }
      lds_signal(filled + b, 2, lane);
      cur = nxt;
      cur2 = nxt2;
      nxt = nn;
      nxt2 = nn2;
    }
  } else {
    // -------------------------------- MFMA waves ----------------------------
    if (a.dbg & kDbgMask & 16) __builtin_amdgcn_s_setprio(2);
    const int m = wave - NG;
    const int nt0 = NT * m;
    const int h = nt0 >> 3;  // 128-column half: mask words 4 h .. 4 h + 3
    const auto rw = buf_rsrc(a.wimg, (uint32_t)(kWImgFrags * 16));
    // W step s = NT ks + t (t < NT), 8 NT steps per chunk; a four-deep ring
    // two steps ahead (the step after a chunk's last is the next chunk's first)
    constexpr int kSteps = kWKs * NT;
    auto load_step = [&](int s, u32x4 (&f)[3]) {
      const int ks = s / NT, nt = nt0 + s % NT;
#pragma unroll
      for (int term = 0; term < 3; ++term)
        f[term] = __builtin_amdgcn_raw_buffer_load_b128(
            rw, 16 * (((ks * kWNt + nt) * 3 + term) * 64 + lane), 0, 0);
    };
    u32x4 wf[4][3];
    load_step(0, wf[0]);
    load_step(1, wf[1]);
    for (int64_t i = 0; i < n_my; ++i) {
      const int b = (int)(i % kSBufs);
      const int gen = (int)(i / kSBufs);
      const int64_t c = chunk_of(i);
      const int64_t r0 = c * kSRows;
      const uint32_t rv = rows_in(c);
      u32x4 mk[2] = {};
      float dv[2] = {1.0f, 1.0f};
      if constexpr (BWD && EPI != WEPI_STORE) {
        const auto rm = buf_rsrc(a.mask_in + r0 * kWMaskWords, rv * kWMaskWords * 4u);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          mk[rt] = __builtin_amdgcn_raw_buffer_load_b128(
              rm, 4 * ((16 * rt + l16) * kWMaskWords + 4 * h), 0, 0);
        if constexpr (EPI == WEPI_RELU_DIV) {
          const auto rd = buf_rsrc(a.row_div + r0, rv * 4u);
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
            dv[rt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rd, 4 * (16 * rt + l16), 0, 0));
        }
      }
      if (!lds_wait_ge(filled + b, kSRows * (gen + 1), abort_word, a.spin)) break;
      if (a.dbg & kDbgMask & 2) {
        const int old = lds_signal(mdone + b, 1, lane);
        if (old == NM * gen + NM - 1) lds_signal(freed + b, 1, lane);
        continue;
      }
      const char *buf = lds + b * kSBuf;
      f32x4_t acc[NT][2];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][rt][r] = 0.0f;
#pragma unroll 1
      for (int k0 = 0; k0 < kWKs; k0 += KSI) {
#pragma unroll
        for (int kk = 0; kk < KSI; ++kk) {
          const int ks = k0 + kk;
          bf16x8 xf[2][3];
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            const int off = wimg_off(16 * rt + l16, 4 * ks + g4);
#pragma unroll
            for (int term = 0; term < 3; ++term)
              xf[rt][term] = *reinterpret_cast<const bf16x8 *>(buf + term * kSImg + off);
          }
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int q = kk * NT + t;  // step within the ring turn: ring slot q
            if (!(a.dbg & kDbgMask & 1)) load_step((NT * ks + t + 2) % kSteps, wf[(q + 2) & 3]);
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
              acc[t][rt] = mfma16_x6_wt(wf[q], xf[rt][0], xf[rt][1], xf[rt][2], acc[t][rt]);
          }
        }
      }
      const auto ry = buf_rsrc(a.Y + r0 * a.ldy, rv * (uint32_t)a.ldy * 4u);
      uint32_t mw[2][4] = {};
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int nt = nt0 + t;
          const int bit = 4 * (nt & 7) + g4;
          float v[4];
          float bb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
          if (!BWD && a.bias != nullptr)
            *reinterpret_cast<float4 *>(bb) =
                *reinterpret_cast<const float4 *>(a.bias + 16 * nt + 4 * g4);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[t][rt][r];
            if constexpr (!BWD) {
              if (a.bias != nullptr) v[r] = __fadd_rn(v[r], bb[r]);
              if (a.relu) v[r] = (v[r] < 0.0f) ? 0.0f : v[r];
              mw[rt][r] |= (v[r] > 0.0f ? 1u : 0u) << bit;
            } else if constexpr (EPI != WEPI_STORE) {
              v[r] = ((mk[rt][r] >> bit) & 1u) ? v[r] : 0.0f;
              cs[t][r] = __fadd_rn(cs[t][r], v[r]);  // rows past the end: zero mask words
              if constexpr (EPI == WEPI_RELU_DIV) v[r] = __fdiv_rn(v[r], dv[rt]);
            }
          }
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4, make_float4(v[0], v[1], v[2], v[3])), ry,
              4 * (int)((16 * rt + l16) * a.ldy + 16 * nt + 4 * g4), 0, kWideNt);
        }
      if constexpr (!BWD) {
        if (a.mask_out != nullptr) {
          // the four lanes of a row (g4) hold its bits of this wave's n-tiles;
          // lane g4 ORs word 4 h + g4 into the chunk's mask row
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            uint32_t mine = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              uint32_t x = mw[rt][r];
              x |= (uint32_t)__shfl_xor((int)x, 16);
              x |= (uint32_t)__shfl_xor((int)x, 32);
              mine = (r == g4) ? x : mine;
            }
            __hip_atomic_fetch_or(maskbuf + (b * kSRows + 16 * rt + l16) * kWMaskWords + 4 * h + g4,
                                  mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
      const int old = lds_signal(mdone + b, 1, lane);
      if (old == NM * gen + NM - 1) {
        // the last MFMA wave out: the chunk's mask words leave, the buffer is free
        if constexpr (!BWD) {
          if (a.mask_out != nullptr) {
            const int row = lane >> 1;
            const u32x4 wv = *reinterpret_cast<const u32x4 *>(
                maskbuf + (b * kSRows + row) * kWMaskWords + 4 * (lane & 1));
            const auto rmo = buf_rsrc(a.mask_out + r0 * kWMaskWords, rv * kWMaskWords * 4u);
            __builtin_amdgcn_raw_buffer_store_b128(wv, rmo, 4 * (row * kWMaskWords + 4 * (lane & 1)),
                                                   0, 0);
          }
        }
        lds_signal(freed + b, 1, lane);
      }
    }
  }
  __syncthreads();
  // a hand-off gave up: this launch's rows are incomplete -- say so (the host
  // turns the word into MGCN_EDEVICE) instead of returning them silently
  if (wave == 0 && lds_load(abort_word) != 0) report_device_error(a.err, kDevErrWide);
  if constexpr (BWD && EPI != WEPI_STORE) {
    // column sums: each column's 16 row lanes (one MFMA wave) folded in lane order
    float *red = reinterpret_cast<float *>(lds);  // [16 row lanes][256]
    if (wave >= NG) {
      const int m = wave - NG;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        *reinterpret_cast<float4 *>(red + l16 * kWF + 16 * (NT * m + t) + 4 * g4) =
            make_float4(cs[t][0], cs[t][1], cs[t][2], cs[t][3]);
    }
    __syncthreads();
    if (tid < kWF) {
      float s = 0.0f;
#pragma unroll
      for (int l = 0; l < 16; ++l) s = __fadd_rn(s, red[l * kWF + tid]);
      a.colsum_partial[(int64_t)blockIdx.x * kWF + tid] = s;
    }
  }
}

template <int U, int NM, bool PK>
int launch_wide_ws_unp(const WideArgs &a, bool bwd, int epi, int grid, hipStream_t s) {
  if (!bwd)
    hipLaunchKernelGGL((spmm_xw_wide_ws_kernel<U, false, WEPI_STORE, NM, PK>), dim3(grid),
                       dim3(kSThreads), 0, s, a);
  else if (epi == WEPI_RELU_DIV)
    hipLaunchKernelGGL((spmm_xw_wide_ws_kernel<U, true, WEPI_RELU_DIV, NM, PK>), dim3(grid),
                       dim3(kSThreads), 0, s, a);
  else if (epi == WEPI_RELU)
    hipLaunchKernelGGL((spmm_xw_wide_ws_kernel<U, true, WEPI_RELU, NM, PK>), dim3(grid),
                       dim3(kSThreads), 0, s, a);
  else
    hipLaunchKernelGGL((spmm_xw_wide_ws_kernel<U, true, WEPI_STORE, NM, PK>), dim3(grid),
                       dim3(kSThreads), 0, s, a);
  return check_launch("spmm_xw_wide_ws_kernel");
}

template <int U, int NM>
int launch_wide_ws_un(const WideArgs &a, bool bwd, int epi, int grid, hipStream_t s) {
  return a.pk != nullptr ? launch_wide_ws_unp<U, NM, true>(a, bwd, epi, grid, s)
                         : launch_wide_ws_unp<U, NM, false>(a, bwd, epi, grid, s);
}

template <int U>
int launch_wide_ws_u(const WideArgs &a, bool bwd, int epi, int grid, hipStream_t s) {
  return g_wide_mfma == 8 ? launch_wide_ws_un<U, 8>(a, bwd, epi, grid, s)
                          : launch_wide_ws_un<U, 4>(a, bwd, epi, grid, s);
}

int wide_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return cus;
}
int wide_grid() { return 2 * wide_cus(); }  // the two-phase kernels: two workgroups per CU
// The warp-specialised kernels hold one workgroup per CU at a time (their LDS),
// over a grid of kWideWsGridMult x CUs: the hardware hands the next workgroup
// to whichever CU frees first, so a CU slowed by work beside it -- a rank's
// RCCL workgroups during the exchange -- takes fewer chunks instead of
// holding the whole launch back (round 6, config-5 rank beside a 64-workgroup
// stand-in for the receive writes: 183.8 -> 154.9 ms/step, 4 / 16 / 32 x:
// 162.5 / 155.7 / 156.7; alone 119.4 vs 120.1 ms, profiles/r06/recv_load_ab.json)
constexpr int kWideWsGridMult = 8;
int wide_ws_grid() { return kWideWsGridMult * wide_cus(); }

template <int U, bool PAIR>
int launch_wide_p(const WideArgs &a, bool bwd, int epi, int grid, hipStream_t s) {
  if (!bwd)
    hipLaunchKernelGGL((spmm_xw_wide_kernel<U, false, WEPI_STORE, PAIR>), dim3(grid),
                       dim3(kWThreads), 0, s, a);
  else if (epi == WEPI_RELU_DIV)
    hipLaunchKernelGGL((spmm_xw_wide_kernel<U, true, WEPI_RELU_DIV, PAIR>), dim3(grid),
                       dim3(kWThreads), 0, s, a);
  else if (epi == WEPI_RELU)
    hipLaunchKernelGGL((spmm_xw_wide_kernel<U, true, WEPI_RELU, PAIR>), dim3(grid),
                       dim3(kWThreads), 0, s, a);
  else
    hipLaunchKernelGGL((spmm_xw_wide_kernel<U, true, WEPI_STORE, PAIR>), dim3(grid),
                       dim3(kWThreads), 0, s, a);
  return check_launch("spmm_xw_wide_kernel");
}

int launch_wide_legacy(const WideArgs &a, bool bwd, int epi, int grid, hipStream_t s);

// *grid: the workgroups launched (= the column-sum partials written)
int launch_wide(const WideArgs &a, bool bwd, int epi, int *grid, hipStream_t s) {
  if (a.pk != nullptr || (g_wide_ws & (bwd ? 2 : 1))) {  // (packed tables: this form only)
    const int64_t n_chunks = (a.n_rows + kSRows - 1) / kSRows;
    const int64_t g = wide_ws_grid();  // one workgroup per CU resident at a time
    *grid = (int)(g < n_chunks ? g : n_chunks);
    return launch_wide_ws_u<kWideU>(a, bwd, epi, *grid, s);
  }
  const int64_t n_chunks = (a.n_rows + kWRows - 1) / kWRows;
  const int64_t g = wide_grid();
  *grid = (int)(g < n_chunks ? g : n_chunks);
  return launch_wide_legacy(a, bwd, epi, *grid, s);
}

int launch_wide_legacy(const WideArgs &a, bool bwd, int epi, int grid, hipStream_t s) {
  if (g_wide_pair & (bwd ? 2 : 1)) return launch_wide_p<kWideU, true>(a, bwd, epi, grid, s);
  return launch_wide_p<kWideU, false>(a, bwd, epi, grid, s);
}

int launch_wimg(const float *W, int64_t ldw, bool trans, u32x4 *img, hipStream_t s) {
  hipLaunchKernelGGL(wide_wimg_kernel, dim3(kWKs * kWNt * 64 / 256), dim3(256), 0, s, W, ldw,
                     trans ? 1 : 0, img);
  return check_launch("wide_wimg_kernel");
}

}  // namespace

namespace {
void set_packed(WideArgs &a, const mgcn_packed_table *pk) {
  if (pk == nullptr) return;
  a.X = nullptr;
  a.ldx = 0;
  a.pk = pk->words;
  a.pk_words = pk->n_words;
  for (int i = 0; i < 64; ++i) a.pk_base[i] = i < pk->n_seg ? pk->seg_base[i] : 0;
  a.pk_nseg = pk->n_seg;
  a.pk_rbits = (uint32_t)pk->row_bits;
  a.pk_head = (uint32_t)pk->seg_rows * 2u * (kWF / 32);
}
}  // namespace

size_t xw_wide_workspace_bytes(bool bwd) {
  return align_up((size_t)kWImgFrags * 16, 256) +
         (bwd ? align_up((size_t)(wide_ws_grid() > wide_grid() ? wide_ws_grid() : wide_grid()) *
                             kWF * 4, 256)
              : 0);
}

int xw_wide_fwd(int64_t n_rows, const int64_t *rowptr, const int32_t *col, const float *w,
                const float *X, int64_t ldx, const float *W, int64_t ldw, const float *bias,
                float *Y, int64_t ldy, int mean, int relu, uint32_t *relu_mask, float *Z,
                int64_t ldz, void *workspace, hipStream_t s, const mgcn_packed_table *pk) {
  u32x4 *img = static_cast<u32x4 *>(workspace);
  if (int rc = launch_wimg(W, ldw, false, img, s)) return rc;
  WideArgs a{};
  a.n_rows = n_rows;
  a.rowptr = rowptr;
  a.col = col;
  a.w = w;
  a.X = X;
  a.ldx = ldx;
  a.wimg = img;
  a.bias = bias;
  a.Y = Y;
  a.ldy = ldy;
  a.mask_out = relu_mask;
  a.Z = Z;
  a.ldz = ldz;
  a.mean = mean;
  a.relu = relu;
  a.dbg = g_wide_dbg;
  a.spin = g_spin_limit;
  a.err = device_error_word();
  if (a.err == nullptr) return MGCN_EHIP;
  set_packed(a, pk);
  int grid = 0;
  return launch_wide(a, false, WEPI_STORE, &grid, s);
}

int xw_wide_bwd_dx(int64_t n_rows, const int64_t *rowptr_t, const int32_t *col_t,
                   const float *w_t, const float *row_scale, const float *dY, int64_t lddy,
                   const float *W, int64_t ldw, float *dX, int64_t lddx,
                   const uint32_t *relu_mask, const float *row_div, float *colsum,
                   int accumulate, void *workspace, hipStream_t s, const mgcn_packed_table *pk) {
  u32x4 *img = static_cast<u32x4 *>(workspace);
  float *partial = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                             align_up((size_t)kWImgFrags * 16, 256));
  if (int rc = take_device_error()) return rc;  // a previous launch failed on the device
  if (int rc = launch_wimg(W, ldw, true, img, s)) return rc;
  const int epi = relu_mask == nullptr ? WEPI_STORE : row_div != nullptr ? WEPI_RELU_DIV : WEPI_RELU;
  WideArgs a{};
  a.n_rows = n_rows;
  a.rowptr = rowptr_t;
  a.col = col_t;
  a.w = w_t;
  a.X = dY;
  a.ldx = lddy;
  a.wimg = img;
  a.Y = dX;
  a.ldy = lddx;
  a.row_scale = row_scale;
  a.mask_in = relu_mask;
  a.row_div = row_div;
  a.colsum_partial = partial;
  a.dbg = g_wide_dbg;
  a.spin = g_spin_limit;
  a.err = device_error_word();
  if (a.err == nullptr) return MGCN_EHIP;
  set_packed(a, pk);
  int grid = 0;
  int rc = launch_wide(a, true, epi, &grid, s);
  if (rc || epi == WEPI_STORE) return rc;
  return launch_fold(partial, grid, kWF, kWF, colsum, kWF, accumulate, s);
}

}  // namespace mgcn
