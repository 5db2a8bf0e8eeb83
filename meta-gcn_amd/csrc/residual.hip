// Fused GCNModel residual layer on gfx950, F = 32 (the botnet stack of
// config 3: run_botnet.sh:14, 12 layers of GCNModel(enc=[32]*12,
// residual_hop=1), src/gcn_meta/models/gcn_model.py:86-105):
//
//   Z1 = relu1( A (X W) + b )        GCNLayer: NodeModelAdditive + activation
//   R  = X Wr^T + br                 the residual Linear of the same input
//   Z  = relu2( Z1 + R )             the join (no relu2 after the last layer)
//
// Round 2 ran a layer as four passes over [N, 32] tensors (one [W | Wr^T]
// GEMM writing [H | R], the SpMM of H, the join; backward the join's
// adjoint, the adjoint SpMM, a dX GEMM and the weight GEMM) -- 10+ launches
// per layer at 15-40 us each.  Here the aggregation and both 32 x 32
// products happen in one pass over the rows:
//
// forward   an 8-lane group gathers the rows of X over the in-edges of two
//           destination rows at once (tile rows g and 8 + g; each row in its
//           edge order, separately rounded products and sums: the SpMM's
//           arithmetic), so (A X) is on chip; the group stages them and their
//           own rows of X in a 16-row LDS tile of the wave, whose
//           (A X) W and X Wr^T run on v_mfma_f32_16x16x4_f32 (exact f32
//           products; W / Wr^T operands staged once per workgroup), then the
//           bias, ReLU, join and ReLU; writes Z as whole rows and two 32-bit
//           ReLU masks per row (bit c: Z1[c] > 0, Z[c] > 0) -- the
//           backward's only record of the activations.
//           (A X) W instead of the reference's A (X W): the same layer to
//           fp32 rounding (the fused F = 128 kernels make the same choice).
// backward  a mask pass forms dS = relu2'(dZ) (the residual branch), dA =
//           relu1'(dS) [/ in-degree for mean] and both bias gradients'
//           column sums; the fused kernel then gathers dA over each source
//           row's out-edges (= dH, the adjoint SpMM bit for bit), writes dH
//           beside dS (the weight GEMM's [dH | dS]) and forms
//           dX = dH W^T + dS Wr in the same group.  [dW | dWr^T] = X^T [dH | dS]
//           stays one split-K GEMM (mgcn_gemm_tn_split).
// heavy rows (degree > the schedule's threshold: the botnet graphs have
//           ~1k rows holding a third of the edges) are aggregated by the
//           SpMM's workgroup-per-row kernels (giant rows on the side stream,
//           overlapping the light rows); forward, those kernels apply the
//           layer's transform in their epilogue (spmm.hip, ResEpi); backward,
//           a second launch of the fused kernel without the gather finishes
//           them, with the layer's weight GEMM riding beside.
//
// Roofline: HBM-bound like the SpMM; bytes per forward launch
//   8 (N + 1) + nnz (4 col + 4 w + 4 F) + 4 N F (own X rows) + 4 N F (Z) + 8 N
// and the 2 x 2 N F^2 FMA flops ride under the gathers.

#include "mgcn_internal.h"
#include "tn_staged.h"

namespace mgcn {
namespace {

// light-row tiles: U slots of each of a lane group's two rows per round
// (round 6: both 8-row steps of a tile aggregated together at U = 4, config 3
// 2.48 -> 2.41 ms/step, against one step after the other at U = 8)
constexpr int kRlU = 4;


constexpr int kRF = 32;             // features (in = out)
constexpr int kRG = 8;              // lanes per row: 4 floats each
constexpr int kRWaves = 4;
constexpr int kRBlock = 64 * kRWaves;

struct RlArgs {
  int64_t n_items;        // rows of this launch
  const int32_t *items;   // their ids (a slice of the view's schedule), NULL: rows 0 .. n_items-1
  const int64_t *rowptr;
  const int32_t *col;
  const float *w;          // per-slot weights, nullable
  const float *row_scale;  // backward 'rw' post-scale, nullable
  const float *T;          // gathered rows: X (forward), dA (backward)
  int64_t ldt;
  const float *own;        // the row's own operand: X (forward residual), dS (backward)
  int64_t ldo;
  float *agg;              // forward: Z (heavy rows: their aggregate, in place); backward: dH
  int64_t ldagg;
  float *out;              // forward: Z; backward: dX
  int64_t ldout;
  uint32_t *masks;         // forward: [row][2] = bits of Z1 > 0, Z > 0
  const float *W;
  int64_t ldw;
  const float *Wr;  // residual Linear weight [out][in]
  int64_t ldwr;
  const float *b, *br;
  int mean, relu1, relu2;
  int gather;  // 0: the aggregate is already in agg (heavy rows)
  // backward inside a stack: the mask pass of the layer below fused into the
  // store of dX (= that layer's dZ): instead of dX the kernel writes its dS
  // (mds) and dA (mda, / mrow_div for mean) and per-block column sums of both
  // ([gridDim.x][2F]: dA | dS) -- residual_mask_bwd_kernel's outputs
  const uint32_t *mmask;  // the lower layer's [row][2] masks; NULL: write dX
  int mrelu1, mrelu2;
  const float *mrow_div;
  float *mds;
  int64_t ldmds;
  float *mda;
  int64_t ldmda;
  float *mpart;
  // independent work riding in this launch, in extra workgroups after the
  // rows' ones: the weight GEMM of the stack's layer (tn_staged.h, on the
  // heavy-row transform launch) and up to two folds of the layer above (its
  // GEMM's split-K partials, the lower layer's bias-gradient column sums)
  TnJob gemm;
  SideFold side[2];
};

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

typedef float rf4 __attribute__((ext_vector_type(4)));

// Tile of one wave: 16 rows x (32 aggregated | 32 own) floats, row stride
// kTileLd (68: the 16 rows of an MFMA operand read land on distinct banks).
constexpr int kTileRows = 16;
constexpr int kTileLd = 2 * kRF + 4;
// one LDS block per workgroup: the waves' tiles, the two B operands, the
// tiles' row ids; an extra workgroup takes it whole
constexpr int kTileFloats = kRWaves * kTileRows * kTileLd;
constexpr int kBFloats = 2 * 64 * 8;
constexpr int kLdsFloats = kTileFloats + 2 * kBFloats + 2 * kRWaves * kTileRows;

// occupancy: the forward light rows fit 96 VGPRs (5 waves per SIMD), the
// backward ones 107 (4 waves; held to 96 they spill 10 VGPRs)
template <int U, bool BWD>
__global__ __launch_bounds__(kRBlock) __attribute__((amdgpu_waves_per_eu(BWD ? 4 : 5)))
void residual_layer_kernel(const RlArgs a) {
  __shared__ __attribute__((aligned(16))) float lds_all[kLdsFloats];
  float(*tile)[kTileRows][kTileLd] = reinterpret_cast<float(*)[kTileRows][kTileLd]>(lds_all);
  // grid: [the rows' workgroups][GEMM, folds]; the rows' grid stride
  // excludes the others
  const unsigned n_extra = (unsigned)(a.gemm.blocks + a.side[0].blocks + a.side[1].blocks);
  const unsigned row_blocks = gridDim.x - n_extra;
  const unsigned rblk = blockIdx.x;  // this workgroup's index among the rows'
  {
    if (rblk >= row_blocks) {
      int b = (int)(rblk - row_blocks);
      float *lds = lds_all;  // >= the GEMM's 4096 floats / the fold's 256
      if (b < a.gemm.blocks) {
        tn_staged_block<2, 32>(a.gemm.A, a.gemm.lda, a.gemm.B, a.gemm.ldb, a.gemm.K, a.gemm.kps,
                               a.gemm.partial, b, lds);
        return;
      }
      b -= a.gemm.blocks;
      if (b < a.side[0].blocks) {
        side_fold_block(a.side[0], b, lds);
        return;
      }
      side_fold_block(a.side[1], b - a.side[0].blocks, lds);
      return;
    }
  }
  // B operands of v_mfma_f32_16x16x4_f32 (lane l: B[k][16 cb + (l & 15)]);
  // the k-steps are permuted so that step s of lane group kk = l >> 4 is
  // k = 8 kk + s: a lane's A operands are then 8 contiguous floats of its
  // tile row, and its 8 B values per column block are contiguous here.
  //   forward : B1[k][n] = W[k][n],  B2[k][n] = Wr[n][k]   (h = agg W, r = x Wr^T)
  //   backward: B1[k][n] = W[n][k],  B2[k][n] = Wr[k][n]   (dX = dH W^T + dS Wr)
  float(*B1)[64][8] = reinterpret_cast<float(*)[64][8]>(lds_all + kTileFloats);
  float(*B2)[64][8] = reinterpret_cast<float(*)[64][8]>(lds_all + kTileFloats + kBFloats);
  int64_t(*tile_row)[kTileRows] =
      reinterpret_cast<int64_t(*)[kTileRows]>(lds_all + kTileFloats + 2 * kBFloats);
  const int tid = threadIdx.x;
  for (int e = tid; e < 2 * 64 * 8; e += kRBlock) {
    const int cb = e >> 9, l = (e >> 3) & 63, st = e & 7;
    const int k = 8 * (l >> 4) + st, n = 16 * cb + (l & 15);
    if constexpr (!BWD) {
      B1[cb][l][st] = a.W[k * a.ldw + n];
      B2[cb][l][st] = a.Wr[n * a.ldwr + k];
    } else {
      B1[cb][l][st] = a.W[n * a.ldw + k];
      B2[cb][l][st] = a.Wr[k * a.ldwr + n];
    }
  }
  __syncthreads();
  const int lane = tid & 63;
  const int gl = lane & (kRG - 1), grp = lane / kRG, gbase = grp * kRG;
  const int wib = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int f0 = 4 * gl;
  const int r16 = lane & 15, kk = lane >> 4;  // MFMA roles
  float(*T)[kTileLd] = tile[wib];
  const bool has_w = a.w != nullptr;
  const bool fmask = BWD && a.mmask != nullptr;
  float msa[4] = {0.f, 0.f, 0.f, 0.f}, mss[4] = {0.f, 0.f, 0.f, 0.f};  // fmask column sums
  const int64_t n_tiles = (a.n_items + kTileRows - 1) / kTileRows;
  // a tile's row ids (tile rows grp, 8 + grp; -1 past the launch's rows)
  auto tile_ids = [&](int64_t wv, int (&r)[2]) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int64_t item = wv * kTileRows + 8 * st + grp;
      r[st] = item >= a.n_items ? -1 : a.items != nullptr ? a.items[item] : (int)item;
    }
  };
  auto tile_meta = [&](const int (&r)[2], int64_t (&b)[2], int (&d)[2]) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      b[st] = r[st] >= 0 ? a.rowptr[r[st]] : 0;
      d[st] = r[st] >= 0 ? (int)(a.rowptr[r[st] + 1] - b[st]) : 0;
    }
  };
  for (int64_t wv = (int64_t)rblk * kRWaves + wib; wv < n_tiles;
       wv += (int64_t)row_blocks * kRWaves) {
    // ---- the tile's 16 rows, two per lane group (tile rows grp, 8 + grp),
    // aggregated together: one dependent chain (schedule id -> row pointers
    // -> slots -> gathered rows) per tile instead of one per 8-row step, and
    // U slots of EACH row in flight per round; each row folds in its own
    // edge order (the SpMM's sums, bit for bit) ----
    {
      int rid[2], deg[2];
      int64_t beg[2];
      tile_ids(wv, rid);
      tile_meta(rid, beg, deg);
      int64_t row[2];
      bool ok[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        ok[st] = rid[st] >= 0;
        row[st] = ok[st] ? rid[st] : 0;
      }
      float acc[2][4] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
      if (a.gather) {
        int maxdeg = deg[0] > deg[1] ? deg[0] : deg[1];
#pragma unroll
        for (int off = kRG; off < 64; off <<= 1) {
          const int o = __shfl_xor(maxdeg, off, 64);
          maxdeg = o > maxdeg ? o : maxdeg;
        }
        for (int e0 = 0; e0 < maxdeg; e0 += kRG) {
          const int my = e0 + gl;
          int mc[2] = {0, 0};
          float mw[2] = {1.0f, 1.0f};
          int nb[2];
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            if (my < deg[st]) {
              mc[st] = a.col[beg[st] + my];
              if (has_w) mw[st] = a.w[beg[st] + my];
            }
            const int rem = deg[st] - e0;
            nb[st] = rem <= 0 ? 0 : (rem < kRG ? rem : kRG);
          }
          const int remw = maxdeg - e0;
          const int nbmax = remw < kRG ? remw : kRG;  // wave-uniform
          for (int k0 = 0; k0 < nbmax; k0 += U) {
            float4 xv[2][U];
            float wk[2][U];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
              for (int st = 0; st < 2; ++st) {
                const int k = (k0 + u) & (kRG - 1);
                const int ck = __shfl(mc[st], gbase + k, 64);
                wk[st][u] = __shfl(mw[st], gbase + k, 64);
                xv[st][u] = k0 + u < nb[st] ? ld4(a.T + (int64_t)ck * a.ldt + f0)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
              }
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
              for (int u = 0; u < U; ++u) {
                if (k0 + u < nb[st]) {
                  acc[st][0] = __fadd_rn(acc[st][0], __fmul_rn(xv[st][u].x, wk[st][u]));
                  acc[st][1] = __fadd_rn(acc[st][1], __fmul_rn(xv[st][u].y, wk[st][u]));
                  acc[st][2] = __fadd_rn(acc[st][2], __fmul_rn(xv[st][u].z, wk[st][u]));
                  acc[st][3] = __fadd_rn(acc[st][3], __fmul_rn(xv[st][u].w, wk[st][u]));
                }
              }
          }
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          if (!BWD && a.mean) {
            const float c = (float)(deg[st] > 1 ? deg[st] : 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[st][j] = __fdiv_rn(acc[st][j], c);
          }
          if (BWD && a.row_scale != nullptr && ok[st]) {
            const float sc = a.row_scale[row[st]];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[st][j] = __fmul_rn(acc[st][j], sc);
          }
          // backward: dH goes out for the weight GEMM
          if (BWD && ok[st])
            st4(a.agg + row[st] * a.ldagg + f0,
                make_float4(acc[st][0], acc[st][1], acc[st][2], acc[st][3]));
        }
      } else {
#pragma unroll
        for (int st = 0; st < 2; ++st)
          if (ok[st]) {
            const float4 v = ld4(a.agg + row[st] * a.ldagg + f0);
            acc[st][0] = v.x, acc[st][1] = v.y, acc[st][2] = v.z, acc[st][3] = v.w;
          }
      }
      // the own operands are loaded here, not held across the gathers
      // (registers set the occupancy)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int tr = 8 * st + grp;
        const float4 ov = ok[st] ? ld4(a.own + row[st] * a.ldo + f0) : make_float4(0.f, 0.f, 0.f, 0.f);
        st4(&T[tr][f0], make_float4(acc[st][0], acc[st][1], acc[st][2], acc[st][3]));
        st4(&T[tr][kRF + f0], ov);
        if (gl == 0) tile_row[wib][tr] = ok[st] ? row[st] : -1;
      }
    }
    __builtin_amdgcn_wave_barrier();

    // ---- both 32 x 32 products of the 16 rows on v_mfma_f32_16x16x4_f32 ----
    // (exact f32 products, f32 accumulation in a fixed k order)
    float av[8], xv8[8];
    {
      const float4 a0 = ld4(&T[r16][8 * kk]), a1 = ld4(&T[r16][8 * kk + 4]);
      const float4 x0 = ld4(&T[r16][kRF + 8 * kk]), x1 = ld4(&T[r16][kRF + 8 * kk + 4]);
      av[0] = a0.x, av[1] = a0.y, av[2] = a0.z, av[3] = a0.w;
      av[4] = a1.x, av[5] = a1.y, av[6] = a1.z, av[7] = a1.w;
      xv8[0] = x0.x, xv8[1] = x0.y, xv8[2] = x0.z, xv8[3] = x0.w;
      xv8[4] = x1.x, xv8[5] = x1.y, xv8[6] = x1.z, xv8[7] = x1.w;
    }
    int bl = lane;  // opaque: the B reads stay here, not hoisted into registers
    asm volatile("" : "+v"(bl));
    rf4 ch[2], cr[2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      ch[cb] = rf4{0.0f, 0.0f, 0.0f, 0.0f};
      cr[cb] = rf4{0.0f, 0.0f, 0.0f, 0.0f};
    }
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const float4 b10 = ld4(&B1[cb][bl][0]), b11 = ld4(&B1[cb][bl][4]);
      const float4 b20 = ld4(&B2[cb][bl][0]), b21 = ld4(&B2[cb][bl][4]);
      const float b1[8] = {b10.x, b10.y, b10.z, b10.w, b11.x, b11.y, b11.z, b11.w};
      const float b2[8] = {b20.x, b20.y, b20.z, b20.w, b21.x, b21.y, b21.z, b21.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        ch[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], b1[s], ch[cb], 0, 0, 0);
        cr[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv8[s], b2[s], cr[cb], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the tile's operand reads precede the result writes

    // ---- epilogue: lane holds rows 4 kk + j, columns 16 cb + r16 ----------
    if constexpr (!BWD) {
      float bc[2], brc[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        bc[cb] = a.b != nullptr ? a.b[16 * cb + r16] : 0.0f;
        brc[cb] = a.br != nullptr ? a.br[16 * cb + r16] : 0.0f;
      }
      // per register j: both column blocks, their ballots (the ReLU masks,
      // bit c of a row's word <=> feature c; lane bit l is row 4 (l >> 4) + j,
      // column 16 cb + (l & 15)) and the staged result -- short live ranges
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint64_t p[2], q[2];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          float v = __fadd_rn(ch[cb][j], bc[cb]);
          if (a.relu1 && v < 0.0f) v = 0.0f;
          float w = __fadd_rn(v, __fadd_rn(cr[cb][j], brc[cb]));
          if (a.relu2 && w < 0.0f) w = 0.0f;
          p[cb] = __ballot(v > 0.0f);
          q[cb] = __ballot(w > 0.0f);
          T[4 * kk + j][16 * cb + r16] = w;
        }
        const int sh = 16 * kk;
        const uint32_t m1 = (uint32_t)((p[0] >> sh) & 0xffffu) | ((uint32_t)((p[1] >> sh) & 0xffffu) << 16);
        const uint32_t m2 = (uint32_t)((q[0] >> sh) & 0xffffu) | ((uint32_t)((q[1] >> sh) & 0xffffu) << 16);
        const int64_t row = tile_row[wib][4 * kk + j];
        if (r16 == 0 && row >= 0) *reinterpret_cast<uint2 *>(a.masks + 2 * row) = make_uint2(m1, m2);
      }
    } else {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int j = 0; j < 4; ++j) T[4 * kk + j][16 * cb + r16] = __fadd_rn(ch[cb][j], cr[cb][j]);
    }
    __builtin_amdgcn_wave_barrier();
    // whole 128-B rows out: group grp writes tile rows grp and 8 + grp
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int tr = 8 * st + grp;
      const int64_t row = tile_row[wib][tr];
      if (row < 0) continue;
      if (!fmask) {
        st4(a.out + row * a.ldout + f0, ld4(&T[tr][f0]));
        continue;
      }
      // the lower layer's mask pass on this dZ row (residual_mask_bwd_kernel's
      // arithmetic): dS = relu2'(dZ), dA = relu1'(dS) [/ in-degree]
      const float4 g4 = ld4(&T[tr][f0]);
      const uint2 mk = *reinterpret_cast<const uint2 *>(a.mmask + 2 * row);
      const float dv = a.mrow_div != nullptr ? a.mrow_div[row] : 1.0f;
      float g[4] = {g4.x, g4.y, g4.z, g4.w}, av[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int bit = f0 + j;
        if (a.mrelu2 && !((mk.y >> bit) & 1u)) g[j] = 0.0f;
        av[j] = (a.mrelu1 && !((mk.x >> bit) & 1u)) ? 0.0f : g[j];
        mss[j] = __fadd_rn(mss[j], g[j]);
        msa[j] = __fadd_rn(msa[j], av[j]);
        if (a.mrow_div != nullptr) av[j] = __fdiv_rn(av[j], dv);
      }
      st4(a.mds + row * a.ldmds + f0, make_float4(g[0], g[1], g[2], g[3]));
      st4(a.mda + row * a.ldmda + f0, make_float4(av[0], av[1], av[2], av[3]));
    }
    __builtin_amdgcn_wave_barrier();  // the tile is restaged by the next 16 rows
  }
  if (fmask) {
    // block partial of the column sums: the 32 lane groups of the block in a
    // fixed order (every block writes one, zeros where it had no rows)
    __syncthreads();
    float *red = &tile[0][0][0];  // 4 x 16 x 68 floats >= 256 threads x 8
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[tid * 8 + j] = msa[j];
      red[tid * 8 + 4 + j] = mss[j];
    }
    __syncthreads();
    if (tid < 2 * kRF) {
      const int which = tid / kRF, f = tid % kRF;
      const int q = f >> 2, j = f & 3;
      float x = 0.0f;
      for (int g = 0; g < kRBlock / kRG; ++g) x = __fadd_rn(x, red[(g * kRG + q) * 8 + 4 * which + j]);
      a.mpart[(int64_t)rblk * 2 * kRF + tid] = x;
    }
  }
}

// Backward mask pass: dS = relu2 ? dZ . [Z > 0] : dZ,  dA = relu1 ? dS . [Z1 > 0] : dS
// (/ row_div for mean), dS written beside dH (DH[:, F:]), dA to its own
// buffer, and the column sums of dA (bias b) and dS (rbias) into block
// partials [block][2F] in a fixed row order (launch_colsum_fold folds them).
// Thread (t_row, q): features 4 q .. 4 q + 3 of rows t_row, t_row + R, ...
constexpr int kMaxParts = 1024;
// fused mask pass: partials per residual_layer_kernel launch, i.e. its
// workgroup cap (grid-stride beyond): 2048 -> 4096 took config 3 2.67 -> 2.63
// ms/step (the backward light pass had fewer workgroups than row tiles);
// 8192 no better
constexpr int kMaxRlParts = 4096;

__global__ __launch_bounds__(256) void residual_mask_bwd_kernel(
    int64_t n, const float *__restrict__ dZ, int64_t lddz, const uint32_t *__restrict__ masks,
    int relu1, int relu2, const float *__restrict__ row_div, float *__restrict__ dA, int64_t ldda,
    float *__restrict__ dS, int64_t ldds, float *__restrict__ partial) {
  __shared__ float red[2][256 * 4];
  constexpr int T = kRF / 4, R = 256 / T;
  const int q = threadIdx.x % T, t_row = threadIdx.x / T;
  const int f0 = 4 * q;
  float sa[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = (int64_t)gridDim.x * R;
  for (int64_t r = (int64_t)blockIdx.x * R + t_row; r < n; r += stride) {
    const float4 g4 = ld4(dZ + r * lddz + f0);
    const uint2 mk = *reinterpret_cast<const uint2 *>(masks + 2 * r);
    const float dv = row_div != nullptr ? row_div[r] : 1.0f;
    float g[4] = {g4.x, g4.y, g4.z, g4.w}, av[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int bit = f0 + j;
      if (relu2 && !((mk.y >> bit) & 1u)) g[j] = 0.0f;
      av[j] = (relu1 && !((mk.x >> bit) & 1u)) ? 0.0f : g[j];
      ss[j] = __fadd_rn(ss[j], g[j]);
      sa[j] = __fadd_rn(sa[j], av[j]);
      if (row_div != nullptr) av[j] = __fdiv_rn(av[j], dv);
    }
    st4(dS + r * ldds + f0, make_float4(g[0], g[1], g[2], g[3]));
    st4(dA + r * ldda + f0, make_float4(av[0], av[1], av[2], av[3]));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[0][threadIdx.x * 4 + j] = sa[j];
    red[1][threadIdx.x * 4 + j] = ss[j];
  }
  __syncthreads();
  if (t_row == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x = red[0][q * 4 + j], y = red[1][q * 4 + j];
      for (int rr = 1; rr < R; ++rr) {
        x = __fadd_rn(x, red[0][(rr * T + q) * 4 + j]);
        y = __fadd_rn(y, red[1][(rr * T + q) * 4 + j]);
      }
      partial[(int64_t)blockIdx.x * 2 * kRF + f0 + j] = x;
      partial[(int64_t)blockIdx.x * 2 * kRF + kRF + f0 + j] = y;
    }
  }
}

int mask_parts(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > kMaxParts) b = kMaxParts;
  if (b < 1) b = 1;
  return (int)b;
}

// blocks of one launch: grid-stride beyond (W / Wr^T staged once per block);
// with the fused mask pass, each block also writes one partial of the sums
}  // namespace
int g_rl_cap = 8192;  // mgcn_set_option("residual_blocks"): workgroups per light-row launch
namespace {
int64_t rl_blocks(int64_t n_items, bool fused_mask) {
  if (n_items <= 0) return 0;
  const int64_t waves = (n_items + kTileRows - 1) / kTileRows;
  int64_t blocks = (waves + kRWaves - 1) / kRWaves;
  int64_t cap = g_rl_cap;
  if (fused_mask && cap > kMaxRlParts) cap = kMaxRlParts;
  return blocks > cap ? cap : blocks;
}

template <bool BWD>
int launch_rl(const RlArgs &a, hipStream_t s) {
  if (a.n_items <= 0) {  // nothing to ride in (callers attach the GEMM only to a launch with rows)
    if (int rc = launch_side_fold(a.side[0], s)) return rc;
    return launch_side_fold(a.side[1], s);
  }
  const int64_t blocks = rl_blocks(a.n_items, BWD && a.mmask != nullptr) + a.gemm.blocks +
                         a.side[0].blocks + a.side[1].blocks;
  hipLaunchKernelGGL((residual_layer_kernel<kRlU, BWD>), dim3((unsigned)blocks), dim3(kRBlock), 0, s, a);
  return check_launch("residual_layer_kernel");
}

bool al16(const void *p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % 4 == 0); }


}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" int mgcn_residual_layer_supported(int32_t F_in, int32_t F_out, int reduce) {
  return F_in == kRF && F_out == kRF && (reduce == MGCN_REDUCE_SUM || reduce == MGCN_REDUCE_MEAN);
}

extern "C" int mgcn_residual_layer_fwd(int64_t n_rows, int32_t F, const int64_t *rowptr,
                                       const int32_t *col, const int32_t *eid, const float *w,
                                       const float *X, int64_t ldx, const float *W, int64_t ldw,
                                       const float *bias, const float *Wr, int64_t ldwr,
                                       const float *rbias, int reduce, int relu1, int relu2,
                                       float *Z, int64_t ldz, uint32_t *masks,
                                       const int32_t *order, int64_t n_heavy, int64_t n_giant,
                                       void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0, "mgcn_residual_layer_fwd: negative size");
  MGCN_REQUIRE(mgcn_residual_layer_supported(F, F, reduce),
               "mgcn_residual_layer_fwd: unsupported F=%d reduce=%d (needs F = 32, sum/mean)", F,
               reduce);
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && X && W && Wr && Z && masks, "mgcn_residual_layer_fwd: null array");
  MGCN_REQUIRE(al16(X, ldx) && al16(Z, ldz) && ldx >= F && ldz >= F && ldw >= F && ldwr >= F,
               "mgcn_residual_layer_fwd: X / Z need 16-byte aligned rows");
  MGCN_REQUIRE((uintptr_t)masks % 8 == 0, "mgcn_residual_layer_fwd: masks not 8-byte aligned");
  MGCN_REQUIRE(Z != X, "mgcn_residual_layer_fwd: Z must not alias X (X is gathered)");
  MGCN_REQUIRE(order == nullptr || (0 <= n_giant && n_giant <= n_heavy && n_heavy <= n_rows),
               "mgcn_residual_layer_fwd: need 0 <= n_giant <= n_heavy <= n_rows");
  hipStream_t s = as_stream(stream);
  const bool mean = reduce == MGCN_REDUCE_MEAN;
  if (order == nullptr) n_heavy = n_giant = 0;
  // heavy rows: the workgroup-per-row kernels aggregate them and apply the
  // layer's transform in their epilogue (giant ones on the side stream)
  bool side = false;
  if (n_heavy > 0) {
    ResEpi rs{W, Wr, bias, rbias, ldw, ldwr, X, ldx, masks, relu1 != 0, relu2 != 0};
    if (int rc = heavy_rows(0, n_rows, F, rowptr, col, eid, w, X, ldx, Z, ldz, nullptr, mean, order,
                            n_heavy, n_giant, s, &side, &rs))
      return rc;
  }
  RlArgs a{};
  a.rowptr = rowptr;
  a.col = col;
  a.w = w;
  a.T = X;
  a.ldt = ldx;
  a.own = X;
  a.ldo = ldx;
  a.agg = Z;
  a.ldagg = ldz;
  a.out = Z;
  a.ldout = ldz;
  a.masks = masks;
  a.W = W;
  a.ldw = ldw;
  a.Wr = Wr;
  a.ldwr = ldwr;
  a.b = bias;
  a.br = rbias;
  a.mean = mean;
  a.relu1 = relu1 != 0;
  a.relu2 = relu2 != 0;
  // light rows: the whole layer in one pass
  a.gather = 1;
  a.items = order != nullptr ? order + n_heavy : nullptr;
  a.n_items = n_rows - n_heavy;
  if (int rc = launch_rl<false>(a, s)) return rc;
  // the next reader of Z needs the giant rows too
  if (side)
    if (int rc = heavy_rows_join(s)) return rc;
  return MGCN_OK;
}

namespace mgcn {
int g_fused_mask = 1;  // mgcn_set_option("residual_fused_mask")
namespace {
// The mask pass of the layer below, fused into this layer's dX store (stack
// backward): its masks / flags / mean divisor, where dS and dA go, the block
// partials of the column sums ([2 kMaxRlParts][2F]) and their fold.
struct LowerMask {
  const uint32_t *masks;
  int relu1, relu2;
  const float *row_div;
  float *dS;
  int64_t ldds;
  float *dA;
  int64_t ldda;
  float *partial;
  float *colsums;
};

// Heavy rows (workgroup kernels into DH), the light rows' fused pass, the
// heavy rows' transform: dA gathered into dH = DH[:, :F], dS = DH[:, F:]
// read as the own operand, dX = dH W^T + dS Wr (or, with lm, the lower
// layer's dS / dA and column sums).
int residual_bwd_core(int64_t n_rows, const int64_t *rowptr_t, const int32_t *col_t,
                      const int32_t *eid_t, const float *w_t, const float *row_scale,
                      const float *dA, const float *W, int64_t ldw, const float *Wr, int64_t ldwr,
                      float *dX, int64_t lddx, float *DH, int64_t lddh, const int32_t *order,
                      int64_t n_heavy, int64_t n_giant, const LowerMask *lm, hipStream_t s,
                      int64_t *defer_parts = nullptr, const SideFold *ride = nullptr,
                      const TnJob *gemm = nullptr, bool *gemm_done = nullptr) {
  const int F = kRF;
  if (order == nullptr) n_heavy = n_giant = 0;
  bool side = false;
  if (n_heavy > 0)
    if (int rc = heavy_rows(1, n_rows, F, rowptr_t, col_t, eid_t, w_t, dA, F, DH, lddh, row_scale,
                            0, order, n_heavy, n_giant, s, &side))
      return rc;
  RlArgs a{};
  a.rowptr = rowptr_t;
  a.col = col_t;
  a.w = w_t;
  a.row_scale = row_scale;
  a.T = dA;
  a.ldt = F;
  a.own = DH + F;
  a.ldo = lddh;
  a.agg = DH;
  a.ldagg = lddh;
  a.out = dX;
  a.ldout = lddx;
  a.W = W;
  a.ldw = ldw;
  a.Wr = Wr;
  a.ldwr = ldwr;
  if (lm != nullptr) {
    a.mmask = lm->masks;
    a.mrelu1 = lm->relu1;
    a.mrelu2 = lm->relu2;
    a.mrow_div = lm->row_div;
    a.mds = lm->dS;
    a.ldmds = lm->ldds;
    a.mda = lm->dA;
    a.ldmda = lm->ldda;
    a.mpart = lm->partial;
  }
  a.gather = 1;
  a.items = order != nullptr ? order + n_heavy : nullptr;
  a.n_items = n_rows - n_heavy;
  if (ride != nullptr) a.side[0] = ride[0], a.side[1] = ride[1];
  if (int rc = launch_rl<true>(a, s)) return rc;
  a.side[0] = a.side[1] = SideFold{};
  int64_t parts = rl_blocks(a.n_items, lm != nullptr);
  if (n_heavy > 0) {
    if (side)
      if (int rc = heavy_rows_join(s)) return rc;
    a.gather = 0;
    a.items = order;
    a.n_items = n_heavy;
    if (gemm != nullptr) {  // the layer's weight GEMM beside the heavy rows' transform
      a.gemm = *gemm;
      *gemm_done = true;
    }
    if (lm != nullptr) a.mpart = lm->partial + parts * 2 * F;
    if (int rc = launch_rl<true>(a, s)) return rc;
    parts += rl_blocks(n_heavy, lm != nullptr);
  }
  if (lm == nullptr) return MGCN_OK;
  if (defer_parts != nullptr) {  // the caller folds them (in its weight-GEMM launch)
    *defer_parts = parts;
    return MGCN_OK;
  }
  return launch_colsum_fold(lm->partial, parts, 2 * F, lm->colsums, s);
}
}  // namespace
}  // namespace mgcn

extern "C" size_t mgcn_residual_layer_bwd_workspace_bytes(int64_t n_rows, int32_t F) {
  const int64_t n = n_rows > 0 ? n_rows : 1;
  const int32_t f = F > 0 ? F : 1;
  return align_up((size_t)n * f * sizeof(float), 256) +
         align_up((size_t)mask_parts(n) * 2 * f * sizeof(float), 256);
}

extern "C" int mgcn_residual_layer_bwd(int64_t n_rows, int32_t F, const int64_t *rowptr_t,
                                       const int32_t *col_t, const int32_t *eid_t,
                                       const float *w_t, const float *row_scale,
                                       const float *row_div, const float *dZ, int64_t lddz,
                                       const uint32_t *masks, int relu1, int relu2,
                                       const float *W, int64_t ldw, const float *Wr, int64_t ldwr,
                                       float *dX, int64_t lddx, float *DH, int64_t lddh,
                                       float *colsums, const int32_t *order, int64_t n_heavy,
                                       int64_t n_giant, void *workspace, size_t workspace_bytes,
                                       void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0, "mgcn_residual_layer_bwd: negative size");
  MGCN_REQUIRE(F == kRF, "mgcn_residual_layer_bwd: unsupported F=%d (needs 32)", F);
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) {
    if (colsums) MGCN_HIP_TRY(hipMemsetAsync(colsums, 0, sizeof(float) * 2 * F, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(rowptr_t && dZ && masks && W && Wr && dX && DH && colsums,
               "mgcn_residual_layer_bwd: null array");
  MGCN_REQUIRE(al16(dZ, lddz) && al16(dX, lddx) && al16(DH, lddh) && lddz >= F && lddx >= F &&
                   lddh >= 2 * F && ldw >= F && ldwr >= F,
               "mgcn_residual_layer_bwd: dZ / dX / DH need 16-byte aligned rows (DH: 2F wide)");
  MGCN_REQUIRE(order == nullptr || (0 <= n_giant && n_giant <= n_heavy && n_heavy <= n_rows),
               "mgcn_residual_layer_bwd: need 0 <= n_giant <= n_heavy <= n_rows");
  const size_t need = mgcn_residual_layer_bwd_workspace_bytes(n_rows, F);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_residual_layer_bwd: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  float *dA = static_cast<float *>(workspace);
  float *partial = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                             align_up((size_t)n_rows * F * sizeof(float), 256));
  const int nparts = mask_parts(n_rows);
  hipLaunchKernelGGL(residual_mask_bwd_kernel, dim3(nparts), dim3(256), 0, s, n_rows, dZ, lddz,
                     masks, relu1, relu2, row_div, dA, (int64_t)F, DH + F, lddh, partial);
  if (int rc = check_launch("residual_mask_bwd_kernel")) return rc;
  if (int rc = launch_colsum_fold(partial, nparts, 2 * F, colsums, s)) return rc;
  return residual_bwd_core(n_rows, rowptr_t, col_t, eid_t, w_t, row_scale, dA, W, ldw, Wr, ldwr,
                           dX, lddx, DH, lddh, order, n_heavy, n_giant, nullptr, s);
}

// ---------------------------------------------------------------------------
// A whole stack of such layers per call (GCNModel's 32 -> 32 layers, config 3):
// one host call per direction instead of one (forward) / two (backward) per
// layer -- the host's issue time, not the GPU, bounded the 12-layer step.

extern "C" int mgcn_residual_stack_fwd(int64_t n_rows, int32_t F, int32_t n_layers,
                                       const int64_t *rowptr, const int32_t *col,
                                       const int32_t *eid, const float *w, const float *X0,
                                       int64_t ldx, const float *const *W,
                                       const float *const *bias, const float *const *Wr,
                                       const float *const *rbias, int reduce,
                                       const int32_t *relu1, const int32_t *relu2, float *Z,
                                       uint32_t *masks, const int32_t *order, int64_t n_heavy,
                                       int64_t n_giant, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && n_layers >= 0, "mgcn_residual_stack_fwd: negative size");
  MGCN_REQUIRE(n_layers == 0 || (W && Wr && relu1 && relu2 && Z && masks),
               "mgcn_residual_stack_fwd: null array");
  for (int32_t l = 0; l < n_layers; ++l) {
    const float *xin = l == 0 ? X0 : Z + (int64_t)(l - 1) * n_rows * F;
    const int64_t ldin = l == 0 ? ldx : F;
    if (int rc = mgcn_residual_layer_fwd(n_rows, F, rowptr, col, eid, w, xin, ldin, W[l], F,
                                         bias ? bias[l] : nullptr, Wr[l], F,
                                         rbias ? rbias[l] : nullptr, reduce, relu1[l], relu2[l],
                                         Z + (int64_t)l * n_rows * F, F,
                                         masks + (int64_t)l * n_rows * 2, order, n_heavy, n_giant,
                                         stream))
      return rc;
  }
  return MGCN_OK;
}

namespace {
// [mask partials of the top layer's pass] [dA x 2] [DH x 2] [dX of layer 0]
// [fused-mask partials x 2] [gemm_tn_split workspace]
struct StackScratch {
  size_t mpart, da, dh, dx, fpart, fpart_half, gemm, total;
  size_t nf, n2f;  // bytes of one [n, F] / [n, 2F] buffer
};
StackScratch stack_scratch(int64_t n_rows, int32_t F) {
  StackScratch s{};
  const int64_t n = n_rows > 0 ? n_rows : 1;
  s.nf = align_up((size_t)n * F * sizeof(float), 256);
  s.n2f = align_up((size_t)n * 2 * F * sizeof(float), 256);
  s.mpart = 0;
  s.da = align_up((size_t)mask_parts(n) * 2 * F * sizeof(float), 256);
  s.dh = s.da + 2 * s.nf;
  s.dx = s.dh + 2 * s.n2f;
  s.fpart = s.dx + s.nf;
  s.fpart_half = align_up((size_t)2 * kMaxRlParts * 2 * F * sizeof(float), 256);
  s.gemm = s.fpart + 2 * s.fpart_half;  // two buffers: a layer's partials are folded
                                        // while the next layer writes its own
  s.total = s.gemm + align_up(mgcn_gemm_tn_workspace_bytes(n_rows, F, 2 * F), 256);
  return s;
}
}  // namespace

extern "C" size_t mgcn_residual_stack_bwd_workspace_bytes(int64_t n_rows, int32_t F) {
  return stack_scratch(n_rows, F).total;
}

extern "C" int mgcn_residual_stack_bwd(int64_t n_rows, int32_t F, int32_t n_layers,
                                       const int64_t *rowptr_t, const int32_t *col_t,
                                       const int32_t *eid_t, const float *w_t,
                                       const float *row_scale, const float *row_div,
                                       const float *dZ, int64_t lddz, const float *X0,
                                       int64_t ldx, const float *Z, const uint32_t *masks,
                                       const int32_t *relu1, const int32_t *relu2,
                                       const float *const *W, const float *const *Wr, float *dX0,
                                       float *const *dW, float *const *dWr, float *sums,
                                       const int32_t *order, int64_t n_heavy, int64_t n_giant,
                                       void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && n_layers >= 0, "mgcn_residual_stack_bwd: negative size");
  if (n_layers == 0) return MGCN_OK;
  MGCN_REQUIRE(W && Wr && dW && dWr && sums && relu1 && relu2 && masks && Z && dZ && X0,
               "mgcn_residual_stack_bwd: null array");
  const StackScratch sc = stack_scratch(n_rows, F);
  if (workspace == nullptr || workspace_bytes < sc.total) {
    set_error("mgcn_residual_stack_bwd: workspace %zu < %zu", workspace_bytes, sc.total);
    return MGCN_EWORKSPACE;
  }
  char *ws = static_cast<char *>(workspace);
  float *dAb[2] = {reinterpret_cast<float *>(ws + sc.da), reinterpret_cast<float *>(ws + sc.da + sc.nf)};
  float *DHb[2] = {reinterpret_cast<float *>(ws + sc.dh), reinterpret_cast<float *>(ws + sc.dh + sc.n2f)};
  float *mpart = reinterpret_cast<float *>(ws + sc.mpart);
  float *fpart = reinterpret_cast<float *>(ws + sc.fpart);
  const size_t gemm_bytes = sc.total - sc.gemm;
  hipStream_t s = as_stream(stream);
  const int64_t nl = n_rows;
  if (n_rows == 0) {
    // no rows: every weight and bias gradient is zero
    for (int32_t l = 0; l < n_layers; ++l) {
      MGCN_HIP_TRY(hipMemsetAsync(dW[l], 0, sizeof(float) * F * F, s));
      MGCN_HIP_TRY(hipMemsetAsync(dWr[l], 0, sizeof(float) * F * F, s));
    }
    MGCN_HIP_TRY(hipMemsetAsync(sums, 0, sizeof(float) * 2 * F * n_layers, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(F == kRF && al16(dZ, lddz) && lddz >= F && al16(X0, ldx) && ldx >= F,
               "mgcn_residual_stack_bwd: F must be 32, dZ / X0 16-byte aligned rows");
  // the top layer's mask pass reads dZ; every lower layer's runs fused in the
  // store of the layer above's dX (its dS / dA / column sums straight from there)
  const int32_t top = n_layers - 1;
  const int nparts = mask_parts(n_rows);
  hipLaunchKernelGGL(residual_mask_bwd_kernel, dim3(nparts), dim3(256), 0, s, n_rows, dZ, lddz,
                     masks + (int64_t)top * nl * 2, relu1[top], relu2[top], row_div, dAb[top & 1],
                     (int64_t)F, DHb[top & 1] + F, (int64_t)2 * F, mpart);
  if (int rc = check_launch("residual_mask_bwd_kernel")) return rc;
  if (int rc = launch_colsum_fold(mpart, nparts, 2 * F, sums + (int64_t)top * 2 * F, s)) return rc;
  // folds of the layer above riding in the next layer's light-row launch:
  // [0] its weight GEMM's split-K partials, [1] the column sums of the bias
  // gradients its passes produced (partials double-buffered by layer parity)
  SideFold pend[2] = {};
  for (int32_t l = top; l >= 0; --l) {
    const int c = l & 1, o = c ^ 1;
    float *dx = (l == 0 && dX0 != nullptr) ? dX0 : reinterpret_cast<float *>(ws + sc.dx);
    LowerMask lm{};
    if (l > 0) {
      lm.masks = masks + (int64_t)(l - 1) * nl * 2;
      lm.relu1 = relu1[l - 1];
      lm.relu2 = relu2[l - 1];
      lm.row_div = row_div;
      lm.dS = DHb[o] + F;
      lm.ldds = 2 * F;
      lm.dA = dAb[o];
      lm.ldda = F;
      lm.partial = fpart + (size_t)c * sc.fpart_half / sizeof(float);
      lm.colsums = sums + (int64_t)(l - 1) * 2 * F;
    }
    const bool fuse = l > 0 && g_fused_mask;
    // [dW | dWr^T] = X_l^T [dH | dS]: on the staged GEMM's workgroups of the
    // heavy-row transform launch where there is one, else its own launch
    const float *xin = l == 0 ? X0 : Z + (int64_t)(l - 1) * n_rows * F;
    const int64_t ldxin = l == 0 ? ldx : F;
    TnJob job{};
    const bool staged = tn_staged_plan(n_rows, F, 2 * F, xin, ldxin, DHb[c], 2 * F, ws + sc.gemm,
                                       gemm_bytes, &job);
    bool gemm_done = false;
    int64_t parts = 0;
    if (int rc = residual_bwd_core(n_rows, rowptr_t, col_t, eid_t, w_t, row_scale, dAb[c], W[l], F,
                                   Wr[l], F, dx, F, DHb[c], 2 * F, order, n_heavy, n_giant,
                                   fuse ? &lm : nullptr, s, fuse ? &parts : nullptr, pend,
                                   staged ? &job : nullptr, &gemm_done))
      return rc;
    pend[0] = pend[1] = SideFold{};
    if (l > 0 && !fuse) {  // the lower layer's mask pass as its own kernel
      hipLaunchKernelGGL(residual_mask_bwd_kernel, dim3(nparts), dim3(256), 0, s, n_rows, dx,
                         (int64_t)F, lm.masks, lm.relu1, lm.relu2, row_div, dAb[o], (int64_t)F,
                         DHb[o] + F, (int64_t)2 * F, mpart);
      if (int rc = check_launch("residual_mask_bwd_kernel")) return rc;
      if (int rc = launch_colsum_fold(mpart, nparts, 2 * F, lm.colsums, s)) return rc;
    }
    if (gemm_done) {
      pend[0] = make_side_fold(job.partial, job.blocks, (int64_t)F * 2 * F, 2 * F, dW[l], F, F,
                               dWr[l], F);
    } else if (int rc = gemm_tn_split_fold(n_rows, F, 2 * F, F, xin, ldxin, DHb[c], 2 * F, dW[l],
                                           F, dWr[l], F, ws + sc.gemm, gemm_bytes, SideFold{}, s,
                                           &pend[0])) {
      return rc;
    }
    if (fuse)
      pend[1] = make_side_fold(lm.partial, parts, 2 * F, 2 * F, lm.colsums, 2 * F, 2 * F,
                               nullptr, 0);
  }
  // the bottom layer's folds: nothing left to ride in
  if (int rc = launch_side_fold(pend[0], s)) return rc;
  return launch_side_fold(pend[1], s);
}
