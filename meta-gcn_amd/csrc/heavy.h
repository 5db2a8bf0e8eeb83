// The SpMM argument block, its vector helpers and the heavy-row body
// (spmm.hip's spmm_heavy_kernel) as a device function that other launches can
// run per workgroup.  Internal header.
#pragma once

#include "mgcn_internal.h"

namespace mgcn {

enum Mode : int {
  FWD_SUM = 0,  // sum or mean (mean divides in the epilogue)
  FWD_MAX = 1,
  BWD_SUM = 2,
  BWD_MEAN = 3,
  BWD_MAX = 4,   // routed through argmax rows
  BWD_MAXM = 5,  // routed through per-slot winner bits (win_mask)
};

struct SpmmArgs {
  int64_t n_rows;
  int32_t F;
  int32_t n_chunks;
  const int64_t *rowptr;
  const int32_t *col;
  const int32_t *eid;
  const float *w;          // nullable: unweighted
  const float *X;          // gathered operand (H forward, dY adjoint)
  int64_t ldx;
  float *Y;                // output rows
  int64_t ldy;
  const float *bias;       // fwd, nullable
  const float *row_scale;  // bwd RW post-scale, nullable
  const float *cnt;        // bwd MEAN: max(in-degree,1) per gathered row
  int32_t *argmax_out;     // fwd MAX
  const int32_t *argmax_in;  // bwd MAX (argmax routing), or:
  const uint32_t *win_mask;  // bwd MAXM: winner bits per fwd slot ([nnz][ceil(F/32)])
  const int32_t *slot_map;   // bwd MAXM: the fwd slot of every bwd slot
  uint32_t *win_mask_out;    // fwd MAX (optional): winner bits of every fwd slot
  uint32_t *relu_mask;       // fwd (optional, F <= 128): Y > 0 bits per row, 4 words,
                             // bit b of word v <=> Y[row][4 b + v] > 0
  int mean;                // fwd: divide by max(deg,1)
  int relu;                // fwd
  int accumulate;          // bwd: Y += result
  // row schedule (mgcn_row_schedule): rows by degree, heaviest first;
  // order[0, n_heavy) go to spmm_heavy_kernel (the first n_giant of them as
  // giant rows), order[n_heavy, n_rows) to the lane-group kernel in that
  // order.  order == NULL: natural row order, no heavy path.
  const int32_t *order;
  int64_t n_heavy;
  int64_t n_giant;
  const int32_t *heavy_rows;  // per heavy launch: its slice of order
  // FWD_SUM at F = 32 with rs.W set: the heavy row's aggregate goes through
  // the residual layer's transform in the epilogue (residual.hip) instead of
  // a second launch
  ResEpi rs;
};

template <int V>
struct F32v {
  float v[V];
};
template <int V>
struct I32v {
  int32_t v[V];
};

template <int V>
__device__ __forceinline__ F32v<V> load_f(const float *p) {
  F32v<V> r;
  if constexpr (V == 4) {
    const float4 t = *reinterpret_cast<const float4 *>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (V == 2) {
    const float2 t = *reinterpret_cast<const float2 *>(p);
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = *p;
  }
  return r;
}

template <int V>
__device__ __forceinline__ I32v<V> load_i(const int32_t *p) {
  I32v<V> r;
  if constexpr (V == 4) {
    const int4 t = *reinterpret_cast<const int4 *>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (V == 2) {
    const int2 t = *reinterpret_cast<const int2 *>(p);
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = *p;
  }
  return r;
}

// rows of a wide SpMM output (G >= 32 lanes: F >= 128) leave with the nt
// cache policy: at config 4 (tables twice the Infinity Cache) max forward
// 0.997 -> 0.970 ms, max adjoint 1.055 -> 1.027, 7.67 -> 7.54 ms/step (two
// A/B pairs); MGCN_NT_EXTRA=0 builds the default-policy form
#ifndef MGCN_NT_EXTRA
#define MGCN_NT_EXTRA 1
#endif
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef float nt_f2 __attribute__((ext_vector_type(2)));
template <int V>
__device__ __forceinline__ void store_f_nt(float *p, const F32v<V> &r) {
  if constexpr (V == 4) {
    __builtin_nontemporal_store(nt_f4{r.v[0], r.v[1], r.v[2], r.v[3]}, reinterpret_cast<nt_f4 *>(p));
  } else if constexpr (V == 2) {
    __builtin_nontemporal_store(nt_f2{r.v[0], r.v[1]}, reinterpret_cast<nt_f2 *>(p));
  } else {
    __builtin_nontemporal_store(r.v[0], p);
  }
}

template <int V>
__device__ __forceinline__ void store_f(float *p, const F32v<V> &r) {
  if constexpr (V == 4) {
    *reinterpret_cast<float4 *>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
  } else if constexpr (V == 2) {
    *reinterpret_cast<float2 *>(p) = make_float2(r.v[0], r.v[1]);
  } else {
    *p = r.v[0];
  }
}

template <int V>
__device__ __forceinline__ void store_i(int32_t *p, const I32v<V> &r) {
  if constexpr (V == 4) {
    *reinterpret_cast<int4 *>(p) = make_int4(r.v[0], r.v[1], r.v[2], r.v[3]);
  } else if constexpr (V == 2) {
    *reinterpret_cast<int2 *>(p) = make_int2(r.v[0], r.v[1]);
  } else {
    *p = r.v[0];
  }
}

#ifdef MGCN_HEAVY_PROFILE
// phase timestamps of workgroup 0 (scripts/prof_heavy.py): [role][batch][begin, end]
// role 0: fold wave, 1: first producer wave, 2: last producer wave
// (spmm.hip's profiling build only: the variable is per translation unit)
__device__ unsigned long long g_hprof[3][256][2];
#define HPROF(role, b, which)                                              \
  if (blockIdx.x == 0 && (b) < 256) g_hprof[role][b][which] = clock64();
#else
#define HPROF(role, b, which)
#endif

// ---------------------------------------------------------------------------
// Heavy rows (degree > heavy_thr; the botnet graphs reach ~6k, config 3):
// one workgroup of HB threads per row, software-pipelined over batches of BE
// edges with two LDS product buffers.  While the first ceil(FC/64) waves FOLD
// batch b -- one sequential chain per feature, in edge order: the reference's
// scatter_add order, bit for bit -- the remaining PRODUCER waves gather batch
// b + 1 and form every product p[f][k] = g(X[col_k, f]) * w_k into the other
// buffer (independent multiplies: exactly the reference's index_select *
// norm).  One barrier per batch.
//
// Producers: thread (c, g) owns vector column c (VEC features) of the edge
// quads g, g + dk, ...: the nv threads of one quad read consecutive 16-byte
// pieces of each source row (coalesced), transpose the 4 x VEC block in
// registers and store one ds_write_b128 per feature.  Products are
// feature-major: feature f = c*VEC + q lives in row q*nv + c of stride BEp
// (BEp/4 odd: the nv stores of one instruction hit distinct banks), so a
// folding lane reads four consecutive edges per ds_read_b128 from an 8-deep
// register ring.  Edge metadata travels one batch ahead through a 3-slot LDS
// ring (fold: slot b, producers: slot b + 1, loads behind the gathers: slot
// b + 2).  The launch runs on a side stream, concurrently with the lane-group
// kernel (launch_mode).
// One heavy row (schedule slot `hidx` of a.heavy_rows) by the calling
// workgroup of HB threads, with `smem` >= 2 FC (BE + 4) + 12 BE floats of LDS:
// the body of spmm_heavy_kernel.  Taking the LDS block as a restrict pointer
// made the heavy kernels 3-4 us faster per launch than the same code over the
// kernel's extern array (config 3).
// (Q: edge quads in flight per producer thread, 0 = the kernel's choice; a
// caller with fewer registers to spare passes a smaller one)
template <int VEC, int MODE, int HB, int Q = 0>
__device__ __forceinline__ void heavy_row_block(const SpmmArgs &a, int FC, int BE, int64_t hidx,
                                                float *__restrict__ smem) {
  constexpr bool kFwd = (MODE == FWD_SUM || MODE == FWD_MAX);
  constexpr bool kNeedEid = (MODE == FWD_MAX || MODE == BWD_MAX);
  constexpr bool kMaxBwd = (MODE == BWD_MAX || MODE == BWD_MAXM);
  constexpr int kQ = Q > 0 ? Q : HB >= 1024 ? (kMaxBwd ? 1 : 2) : 4;  // edge quads in flight / thread
  constexpr int kEpt = 4;  // metadata entries per producer thread (BE <= kEpt * producers)
  const int BEp = BE + 4;  // product row stride (BE % 16 == 0, so BEp / 4 is odd)
  int32_t *ring = reinterpret_cast<int32_t *>(smem + 2 * FC * BEp);  // [3][4][BE]
  auto ColR = [&](int b) { return ring + (b % 3) * 4 * BE; };
  auto EidR = [&](int b) { return ColR(b) + BE; };
  auto WtR = [&](int b) { return reinterpret_cast<float *>(ColR(b) + 2 * BE); };
  auto CntR = [&](int b) { return reinterpret_cast<float *>(ColR(b) + 3 * BE); };
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t row = a.heavy_rows[hidx];
  const int64_t beg = a.rowptr[row];
  const int64_t deg = a.rowptr[row + 1] - beg;
  const bool has_w = a.w != nullptr;
  const int nbatch = (int)((deg + BE - 1) / BE);
  auto batch_len = [&](int b) {
    const int64_t left = deg - (int64_t)b * BE;
    return left < BE ? (int)left : BE;
  };

  for (int f0 = 0; f0 < a.F; f0 += FC) {
    const int fc = (a.F - f0) < FC ? (a.F - f0) : FC;
    const int nv = fc / VEC;                   // vectors per row segment
    const int fold_waves = (fc + 63) / 64;     // 1 or 2
    const int np = HB - 64 * fold_waves;       // producer threads
    const int pt = t - 64 * fold_waves;        // producer index (< 0: folder)
    const int dk = np / nv, npe = dk * nv;     // quad producers: npe threads
    const int g_first = pt / nv, c_first = pt - (pt / nv) * nv;

    int mcol[kEpt], meid[kEpt];
    float mw[kEpt];
    auto load_meta = [&](int b) {  // registers <- edges pt + np*i of batch b
      if (b >= nbatch) return;
      const int nb = batch_len(b);
#pragma unroll
      for (int i = 0; i < kEpt; ++i) {
        const int k = pt + np * i;
        if (k < nb) {
          const int64_t slot = beg + (int64_t)b * BE + k;
          mcol[i] = a.col[slot];
          mw[i] = has_w ? a.w[slot] : 1.0f;
          if constexpr (kNeedEid) meid[i] = a.eid[slot];
          if constexpr (MODE == BWD_MAXM) meid[i] = a.slot_map[slot];  // fwd slot
        }
      }
    };
    auto store_meta = [&](int b) {  // ring slot of batch b <- registers
      if (b >= nbatch) return;
      const int nb = batch_len(b);
      int32_t *Col = ColR(b), *Eid = EidR(b);
      float *Wt = WtR(b), *Cnt = CntR(b);
#pragma unroll
      for (int i = 0; i < kEpt; ++i) {
        const int k = pt + np * i;
        if (k < nb) {
          Col[k] = mcol[i];
          Wt[k] = mw[i];
          if constexpr (kNeedEid || MODE == BWD_MAXM) Eid[k] = meid[i];
          if constexpr (MODE == BWD_MEAN) Cnt[k] = a.cnt[mcol[i]];
        }
      }
    };
    // products of batch b (metadata already in its ring slot); batch b + 1's
    // metadata is loaded behind the first round of gathers
    auto produce = [&](int b) {
      float *P = smem + (b & 1) * FC * BEp + c_first * BEp;  // row q*nv + c: + q*nv*BEp
      const int32_t *Col = ColR(b), *Eid = EidR(b);
      const float *Wt = WtR(b), *Cnt = CntR(b);
      const int nb = batch_len(b);
      const int nq = (nb + 3) >> 2;
      const float *xs = a.X + f0 + c_first * VEC;
      bool first = true;
      if (pt < npe) {
        for (int g0 = g_first; g0 < nq; g0 += kQ * dk) {
          F32v<VEC> x[kQ][4];
          I32v<VEC> am[kQ][4];
#pragma unroll
          for (int u = 0; u < kQ; ++u) {
            const int g = g0 + u * dk;
            if (g < nq) {
              const I32v<4> cols = load_i<4>(Col + 4 * g);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                if (4 * g + e < nb) {
                  x[u][e] = load_f<VEC>(xs + (int64_t)cols.v[e] * a.ldx);
                  if constexpr (kMaxBwd) {
                    if constexpr (MODE == BWD_MAXM) {  // winner flags of this edge (1 / 0)
                      const int64_t W = (a.F + 31) >> 5;
                      const int f = f0 + c_first * VEC;
                      const int32_t fslot = Eid[4 * g + e];  // ring holds the fwd slot
                      const uint32_t bits = a.win_mask[(int64_t)fslot * W + (f >> 5)] >> (f & 31);
#pragma unroll
                      for (int q = 0; q < VEC; ++q) am[u][e].v[q] = (bits >> q) & 1u;
                    } else {
                      am[u][e] = load_i<VEC>(a.argmax_in + (int64_t)cols.v[e] * a.F + f0 +
                                             c_first * VEC);
                    }
                  }
                }
              }
            }
          }
          if (first) load_meta(b + 1);
          first = false;
#pragma unroll
          for (int u = 0; u < kQ; ++u) {
            const int g = g0 + u * dk;
            if (g < nq) {
              const F32v<4> w = load_f<4>(Wt + 4 * g);
              I32v<4> eid;
              F32v<4> cnt;
              if constexpr (MODE == BWD_MAXM) {
                eid.v[0] = eid.v[1] = eid.v[2] = eid.v[3] = 1;  // flags: 1 = winner
              } else if constexpr (MODE == BWD_MAX) {
                eid = load_i<4>(Eid + 4 * g);
              }
              if constexpr (MODE == BWD_MEAN) cnt = load_f<4>(Cnt + 4 * g);
              int off = 4 * g;
              asm volatile("" : "+v"(off));  // keep per-quad store offsets out of registers
#pragma unroll
              for (int q = 0; q < VEC; ++q) {
                F32v<4> o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  float v = x[u][e].v[q];
                  if constexpr (kMaxBwd) v = (am[u][e].v[q] == eid.v[e]) ? v : 0.0f;
                  if constexpr (MODE == BWD_MEAN) v = __fdiv_rn(v, cnt.v[e]);
                  o.v[e] = __fmul_rn(v, w.v[e]);
                }
                store_f<4>(P + q * nv * BEp + off, o);
              }
            }
          }
        }
      }
      if (first) load_meta(b + 1);
      store_meta(b + 1);
    };

    float acc = (MODE == FWD_MAX) ? MGCN_MAX_FILL : 0.0f;
    int32_t arg = -1;
    if (pt >= 0) {
      load_meta(0);
      store_meta(0);
    }
    __syncthreads();
    if (pt >= 0 && nbatch > 0) produce(0);
    __syncthreads();
#ifdef MGCN_HEAVY_PROFILE
    const int prole = t == 0 ? 0 : t == 64 * fold_waves ? 1 : t == HB - 64 ? 2 : -1;
#endif
    const int frow = (t % VEC) * nv + t / VEC;  // this folding lane's product row
    for (int bi = 0; bi < nbatch; ++bi) {
#ifdef MGCN_HEAVY_PROFILE
      if (prole >= 0) HPROF(prole, bi, 0);
#endif
      if (wave < fold_waves) {
        if (t < fc) {  // fold batch bi: one sequential chain per feature, edge order
          const float *pr = smem + (bi & 1) * FC * BEp + frow * BEp;
          const int nb = batch_len(bi);
          const int n4 = nb >> 2;
          if constexpr (MODE == FWD_MAX) {
            const int32_t *Eid = EidR(bi);
            for (int c4 = 0; c4 < n4; ++c4) {
              const F32v<4> p = load_f<4>(pr + 4 * c4);
              const I32v<4> e = load_i<4>(Eid + 4 * c4);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                if (p.v[q] >= acc) {
                  acc = p.v[q];
                  arg = e.v[q];
                }
              }
            }
            for (int k = 4 * n4; k < nb; ++k) {
              if (pr[k] >= acc) {
                acc = pr[k];
                arg = Eid[k];
              }
            }
          } else {
            // 8-deep ring of 4-edge reads; reads past nb (at most 32 floats)
            // stay inside the LDS allocation and are never added
            constexpr int kR = 8;
            F32v<4> R[kR];
#pragma unroll
            for (int j = 0; j < kR; ++j) R[j] = load_f<4>(pr + 4 * j);
            int c4 = 0;
            for (; c4 + kR <= n4; c4 += kR) {
#pragma unroll
              for (int j = 0; j < kR; ++j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) acc = __fadd_rn(acc, R[j].v[q]);
                R[j] = load_f<4>(pr + 4 * (c4 + kR + j));
                __builtin_amdgcn_sched_barrier(0);  // keep each refill behind its adds
              }
            }
#pragma unroll
            for (int j = 0; j < kR; ++j) {
              if (c4 + j < n4) {
#pragma unroll
                for (int q = 0; q < 4; ++q) acc = __fadd_rn(acc, R[j].v[q]);
              }
            }
            for (int k = 4 * n4; k < nb; ++k) acc = __fadd_rn(acc, pr[k]);
          }
        }
      } else if (bi + 1 < nbatch) {
        produce(bi + 1);
      }
#ifdef MGCN_HEAVY_PROFILE
      if (prole >= 0) HPROF(prole, bi, 1);
#endif
      __syncthreads();
    }
    if constexpr (MODE == FWD_SUM) {
      if (a.rs.W != nullptr) {
        // the residual layer's transform of this row (F = 32: one chunk, one
        // fold lane per feature): Z = relu2(relu1(agg W + b) + x Wr^T + br)
        // and its two mask words, the light rows' epilogue with the two
        // 32-term products summed in k order
        float *ep = smem;  // the product buffers are free after the last barrier
        if (t < 32) {
          ep[t] = a.mean ? __fdiv_rn(acc, (float)(deg > 1 ? deg : 1)) : acc;
          ep[32 + t] = a.rs.X[row * a.rs.ldx + t];
        }
        __syncthreads();
        if (t < 32) {
          float hv = 0.0f, rv = 0.0f;
#pragma unroll 8
          for (int k = 0; k < 32; ++k) {
            hv = __fadd_rn(hv, __fmul_rn(ep[k], a.rs.W[k * a.rs.ldw + t]));
            rv = __fadd_rn(rv, __fmul_rn(ep[32 + k], a.rs.Wr[t * a.rs.ldwr + k]));
          }
          float v = __fadd_rn(hv, a.rs.b != nullptr ? a.rs.b[t] : 0.0f);
          if (a.rs.relu1 && v < 0.0f) v = 0.0f;
          float z = __fadd_rn(v, __fadd_rn(rv, a.rs.br != nullptr ? a.rs.br[t] : 0.0f));
          if (a.rs.relu2 && z < 0.0f) z = 0.0f;
          const uint32_t m1 = (uint32_t)__ballot(v > 0.0f), m2 = (uint32_t)__ballot(z > 0.0f);
          a.Y[row * a.ldy + t] = z;
          if (t == 0) *reinterpret_cast<uint2 *>(a.rs.masks + 2 * row) = make_uint2(m1, m2);
        }
        continue;  // F = 32: the only feature chunk
      }
    }
    if (t < fc) {
      const int f = f0 + t;
      float *dst = a.Y + row * a.ldy + f;
      if constexpr (kFwd) {
        float y = acc;
        if constexpr (MODE == FWD_MAX) {
          if (y == MGCN_MAX_FILL) {
            y = 0.0f;
            arg = -1;
          }
          if (a.argmax_out != nullptr) a.argmax_out[row * a.F + f] = arg;
        } else {
          if (a.mean) y = __fdiv_rn(y, (float)(deg > 1 ? deg : 1));
        }
        if (a.bias != nullptr) y = __fadd_rn(y, a.bias[f]);
        if (a.relu) y = (y < 0.0f) ? 0.0f : y;
        *dst = y;
      } else {
        float v = acc;
        if (a.row_scale != nullptr) v = __fmul_rn(v, a.row_scale[row]);
        if (a.accumulate) v = __fadd_rn(*dst, v);
        *dst = v;
      }
    }
    if constexpr (MODE == FWD_MAX) {
      if (a.win_mask_out != nullptr) {
        // winner bits of every edge of the row: the chunk's winners go to
        // LDS, then every wave takes edges k = wave, wave + HB/64, ... and
        // forms each 64-feature slice with one ballot
        int32_t *win_lds = reinterpret_cast<int32_t *>(smem);  // buffers are free here
        if (t < fc) win_lds[t] = (acc == MGCN_MAX_FILL) ? -1 : arg;
        __syncthreads();
        const int64_t W = (a.F + 31) >> 5;
        const int lane = t & 63;
        int32_t wv[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) wv[r] = (64 * r + lane < fc) ? win_lds[64 * r + lane] : -1;
        for (int64_t k = wave; k < deg; k += HB / 64) {
          const int32_t ek = a.eid[beg + k];
          const int64_t sk = beg + k;  // own fwd slot
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            if (64 * r >= fc) break;
            const uint64_t bal = __ballot(wv[r] == ek);
            const int fb = f0 + 64 * r;  // 32-aligned (FC is 128 or F)
            if (lane == 0) a.win_mask_out[sk * W + (fb >> 5)] = (uint32_t)bal;
            if (lane == 32 && fb + 32 < a.F) a.win_mask_out[sk * W + (fb >> 5) + 1] = (uint32_t)(bal >> 32);
          }
        }
      }
    }
    __syncthreads();  // buffers are reused by the next feature chunk
  }
}

}  // namespace mgcn
