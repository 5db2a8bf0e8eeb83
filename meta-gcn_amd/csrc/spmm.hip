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

#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kWaves = 4;  // waves per 256-thread block
constexpr int kBlock = 64 * kWaves;

enum Mode : int {
  FWD_SUM = 0,  // sum or mean (mean divides in the epilogue)
  FWD_MAX = 1,
  BWD_SUM = 2,
  BWD_MEAN = 3,
  BWD_MAX = 4,
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
  const int32_t *argmax_in;  // bwd MAX
  int mean;                // fwd: divide by max(deg,1)
  int relu;                // fwd
  int accumulate;          // bwd: Y += result
  const int32_t *heavy_rows;  // rows with deg > heavy_thr, done by spmm_heavy_kernel
  int64_t n_heavy;
  int64_t heavy_thr;          // INT64_MAX: no heavy path
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
  constexpr bool kNeedEid = (MODE == FWD_MAX || MODE == BWD_MAX);
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);
  const int grp = lane / G;
  const int gbase = grp * G;
  const int wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_row_groups = (a.n_rows + RPW - 1) / RPW;
  const int64_t wave_stride = (int64_t)gridDim.x * kWaves;
  const float *__restrict__ X = a.X;
  const bool has_w = a.w != nullptr;

  for (int64_t wv = (int64_t)blockIdx.x * kWaves + wave_in_block; wv < n_row_groups;
       wv += wave_stride) {
    const int64_t row = wv * RPW + grp;
    const bool row_ok = row < a.n_rows;
    const int64_t beg = row_ok ? a.rowptr[row] : 0;
    int64_t deg = row_ok ? a.rowptr[row + 1] - beg : 0;
    const bool heavy = deg > a.heavy_thr;  // owned by spmm_heavy_kernel
    if (heavy) deg = 0;
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
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = k0 + u;
            const int kk = k & (G - 1);
            const int ck = bcast_i<G>(mc, gbase, kk);
            wk[u] = bcast_f<G>(mw, gbase, kk);
            ek[u] = kNeedEid ? bcast_i<G>(me, gbase, kk) : 0;
            float cntk = 1.0f;
            if constexpr (MODE == BWD_MEAN) cntk = bcast_f<G>(mcnt, gbase, kk);
            ok[u] = (k < nb) && f_ok;
            const float *src = X + (int64_t)ck * a.ldx + f0;
            if constexpr (MODE == BWD_MAX) {
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

      if (!(row_ok && f_ok) || heavy) continue;
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
        store_f<VEC>(dst, acc);
        if constexpr (MODE == FWD_MAX) store_i<VEC>(a.argmax_out + row * a.F + f0, arg);
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
        store_f<VEC>(dst, acc);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Heavy rows (degree > heavy_thr; the botnet graphs reach ~6k, config 3):
// one 256-thread workgroup per row.  The row's edges are taken in batches of
// BE: phase A gathers BE source rows (a feature chunk of FC floats each) and
// forms every product p[k][f] = g(X[col_k, f]) * w_k in parallel into LDS
// (the multiplies are independent, so this is exactly the reference's
// index_select * norm); phase B folds p[.][f] for each feature f sequentially
// in edge order (FC threads, one chain per feature) -- the reference's
// scatter_add order, bit for bit.  BE rows in flight per CU instead of U per
// lane group: the row no longer serialises on HBM latency.
template <int VEC, int MODE>
__global__ __launch_bounds__(kBlock) void spmm_heavy_kernel(const SpmmArgs a, int FC, int BE) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *P = smem;                                            // [BE][FC] products
  int32_t *Eid = reinterpret_cast<int32_t *>(smem + BE * FC);  // [BE] per-edge metadata
  int32_t *Col = Eid + BE;
  float *Wt = reinterpret_cast<float *>(Col + BE);
  float *Cnt = Wt + BE;
  constexpr bool kFwd = (MODE == FWD_SUM || MODE == FWD_MAX);
  constexpr bool kNeedEid = (MODE == FWD_MAX || MODE == BWD_MAX);
  constexpr int kInFlight = 8;  // independent gathers per thread
  const int t = threadIdx.x;
  const int64_t row = a.heavy_rows[blockIdx.x];
  const int64_t beg = a.rowptr[row];
  const int64_t deg = a.rowptr[row + 1] - beg;
  const bool has_w = a.w != nullptr;

  for (int f0 = 0; f0 < a.F; f0 += FC) {
    const int fc = (a.F - f0) < FC ? (a.F - f0) : FC;
    const int nv = fc / VEC;  // vectors per row segment
    float acc = (MODE == FWD_MAX) ? MGCN_MAX_FILL : 0.0f;
    int32_t arg = -1;
    for (int64_t e0 = 0; e0 < deg; e0 += BE) {
      const int nb = (deg - e0) < BE ? (int)(deg - e0) : BE;
      // phase A0: the batch's edge metadata -> LDS (coalesced)
      for (int k = t; k < nb; k += kBlock) {
        const int64_t slot = beg + e0 + k;
        const int col = a.col[slot];
        Col[k] = col;
        Wt[k] = has_w ? a.w[slot] : 1.0f;
        if constexpr (kNeedEid) Eid[k] = a.eid[slot];
        if constexpr (MODE == BWD_MEAN) Cnt[k] = a.cnt[col];
      }
      __syncthreads();
      // phase A1: kInFlight independent row-segment gathers per thread, then
      // the products (one rounding each, as x_j * norm) -> LDS
      const int total = nb * nv;
      for (int base = t; base < total; base += kBlock * kInFlight) {
        F32v<VEC> x[kInFlight];
        I32v<VEC> am[kInFlight];
#pragma unroll
        for (int j = 0; j < kInFlight; ++j) {
          const int idx = base + j * kBlock;
          if (idx < total) {
            const int k = idx / nv, c = idx - (idx / nv) * nv;
            const int64_t off = (int64_t)Col[k] * a.ldx + f0 + c * VEC;
            x[j] = load_f<VEC>(a.X + off);
            if constexpr (MODE == BWD_MAX)
              am[j] = load_i<VEC>(a.argmax_in + (int64_t)Col[k] * a.F + f0 + c * VEC);
          }
        }
#pragma unroll
        for (int j = 0; j < kInFlight; ++j) {
          const int idx = base + j * kBlock;
          if (idx < total) {
            const int k = idx / nv, c = idx - (idx / nv) * nv;
            const float w = Wt[k];
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
              float v = x[j].v[q];
              if constexpr (MODE == BWD_MAX) v = (am[j].v[q] == Eid[k]) ? v : 0.0f;
              if constexpr (MODE == BWD_MEAN) v = __fdiv_rn(v, Cnt[k]);
              P[k * FC + c * VEC + q] = __fmul_rn(v, w);
            }
          }
        }
      }
      __syncthreads();
      if (t < fc) {  // phase B: one sequential chain per feature
        const float *pc = P + t;
        if constexpr (MODE == FWD_MAX) {
          for (int k = 0; k < nb; ++k) {
            const float p = pc[k * FC];
            if (p >= acc) {
              acc = p;
              arg = Eid[k];
            }
          }
        } else {
#pragma unroll 8
          for (int k = 0; k < nb; ++k) acc = __fadd_rn(acc, pc[k * FC]);
        }
      }
      __syncthreads();
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
          a.argmax_out[row * a.F + f] = arg;
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
  }
}

__global__ __launch_bounds__(kBlock) void heavy_rows_kernel(int64_t n_rows,
                                                            const int64_t *__restrict__ rowptr,
                                                            int64_t thr, int32_t *__restrict__ out,
                                                            unsigned long long *__restrict__ count) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rows;
       r += (int64_t)gridDim.x * blockDim.x)
    if (rowptr[r + 1] - rowptr[r] > thr) out[atomicAdd(count, 1ull)] = (int32_t)r;
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

int g_force_vec = 0;  // tuning knobs (mgcn_set_option)
int g_unroll = 8;

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
    if (g_unroll == 4) return launch_one<VEC, 32, 4, MODE>(a, stream);
    return launch_one<VEC, 32, 8, MODE>(a, stream);
  }
  if (lanes > 8) return launch_one<VEC, 16, 8, MODE>(a, stream);
  if (lanes > 4) return launch_one<VEC, 8, 8, MODE>(a, stream);
  return launch_one<VEC, 4, 4, MODE>(a, stream);
}

constexpr int kHeavyLdsBytes = 65536;  // products + edge ids per batch (default LDS limit)

template <int VEC, int MODE>
int launch_heavy(const SpmmArgs &a, hipStream_t stream) {
  int FC = a.F < 128 ? a.F : 128;
  FC = (FC + VEC - 1) / VEC * VEC;
  const int BE = kHeavyLdsBytes / (4 * (FC + 4));  // products + 4 metadata words per edge
  const size_t lds = sizeof(float) * (size_t)BE * (FC + 4);
  hipLaunchKernelGGL((spmm_heavy_kernel<VEC, MODE>), dim3((unsigned)a.n_heavy), dim3(kBlock), lds,
                     stream, a, FC, BE);
  return check_launch("spmm_heavy_kernel");
}

template <int MODE>
int launch_mode(SpmmArgs a, int vec, hipStream_t stream) {
  const int G_lanes_max = 64;
  const int per_chunk = G_lanes_max * vec;
  a.n_chunks = (a.F + per_chunk - 1) / per_chunk;
  if (a.n_chunks < 1) a.n_chunks = 1;
  if (a.heavy_rows == nullptr || a.n_heavy <= 0) {
    a.heavy_rows = nullptr;
    a.n_heavy = 0;
    a.heavy_thr = INT64_MAX;
  } else {
    int rc = vec == 4   ? launch_heavy<4, MODE>(a, stream)
             : vec == 2 ? launch_heavy<2, MODE>(a, stream)
                        : launch_heavy<1, MODE>(a, stream);
    if (rc) return rc;
  }
  if (vec == 4) return launch_g<4, MODE>(a, stream);
  if (vec == 2) return launch_g<2, MODE>(a, stream);
  return launch_g<1, MODE>(a, stream);
}

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" int mgcn_set_option(const char *name, int value) {
  clear_error();
  if (name == nullptr) return MGCN_EINVAL;
  const std::string n(name);
  if (n == "spmm_vec") {
    MGCN_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4, "spmm_vec must be 0,1,2,4");
    g_force_vec = value;
    return MGCN_OK;
  }
  if (n == "spmm_unroll") {
    MGCN_REQUIRE(value == 4 || value == 8 || value == 16, "spmm_unroll must be 4, 8 or 16");
    g_unroll = value;
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
                             int32_t *argmax, const int32_t *heavy_rows, int64_t n_heavy,
                             int64_t heavy_thr, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_spmm_fwd: negative size");
  MGCN_REQUIRE(reduce == MGCN_REDUCE_SUM || reduce == MGCN_REDUCE_MEAN || reduce == MGCN_REDUCE_MAX,
               "mgcn_spmm_fwd: bad reduce %d", reduce);
  if (n_rows == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && H && Y, "mgcn_spmm_fwd: null array");  // col may be NULL when nnz == 0
  MGCN_REQUIRE(ldh >= F && ldy >= F, "mgcn_spmm_fwd: leading dimension < F");
  MGCN_REQUIRE(reduce != MGCN_REDUCE_MAX || argmax != nullptr,  // eid NULL only if nnz == 0
               "mgcn_spmm_fwd: MAX needs argmax and eid");
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
  a.heavy_rows = heavy_rows;
  a.n_heavy = n_heavy;
  a.heavy_thr = heavy_thr;
  a.mean = reduce == MGCN_REDUCE_MEAN;
  a.relu = relu != 0;
  int vec = choose_vec(F, H, ldh, Y, ldy);
  if (reduce == MGCN_REDUCE_MAX && reinterpret_cast<uintptr_t>(argmax) % (4 * vec)) vec = 1;
  if (bias != nullptr && reinterpret_cast<uintptr_t>(bias) % 4) return MGCN_EINVAL;
  hipStream_t s = as_stream(stream);
  if (reduce == MGCN_REDUCE_MAX) return launch_mode<FWD_MAX>(a, vec, s);
  return launch_mode<FWD_SUM>(a, vec, s);
}

extern "C" int mgcn_spmm_bwd(int64_t n_rows, int32_t F, const int64_t *rowptr_t,
                             const int32_t *col_t, const int32_t *eid_t, const float *w_t,
                             const float *row_scale, const float *dY, int64_t lddy, float *dH,
                             int64_t lddh, int reduce, const float *cnt, const int32_t *argmax,
                             int accumulate, const int32_t *heavy_rows, int64_t n_heavy,
                             int64_t heavy_thr, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_spmm_bwd: negative size");
  MGCN_REQUIRE(reduce == MGCN_REDUCE_SUM || reduce == MGCN_REDUCE_MEAN || reduce == MGCN_REDUCE_MAX,
               "mgcn_spmm_bwd: bad reduce %d", reduce);
  if (n_rows == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr_t && dY && dH, "mgcn_spmm_bwd: null array");  // col may be NULL when nnz == 0
  MGCN_REQUIRE(lddy >= F && lddh >= F, "mgcn_spmm_bwd: leading dimension < F");
  MGCN_REQUIRE(reduce != MGCN_REDUCE_MEAN || cnt != nullptr, "mgcn_spmm_bwd: MEAN needs cnt");
  MGCN_REQUIRE(reduce != MGCN_REDUCE_MAX || argmax != nullptr,  // eid NULL only if nnz == 0
               "mgcn_spmm_bwd: MAX needs argmax and eid");
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
  a.accumulate = accumulate != 0;
  a.heavy_rows = heavy_rows;
  a.n_heavy = n_heavy;
  a.heavy_thr = heavy_thr;
  int vec = choose_vec(F, dY, lddy, dH, lddh);
  if (reduce == MGCN_REDUCE_MAX && reinterpret_cast<uintptr_t>(argmax) % (4 * vec)) vec = 1;
  hipStream_t s = as_stream(stream);
  if (reduce == MGCN_REDUCE_MAX) return launch_mode<BWD_MAX>(a, vec, s);
  if (reduce == MGCN_REDUCE_MEAN) return launch_mode<BWD_MEAN>(a, vec, s);
  return launch_mode<BWD_SUM>(a, vec, s);
}

extern "C" int mgcn_heavy_rows(int64_t n_rows, const int64_t *rowptr, int64_t thr, int32_t *rows_out,
                               int64_t *n_out, void *workspace, size_t workspace_bytes,
                               void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && thr >= 0 && n_out != nullptr, "mgcn_heavy_rows: bad arguments");
  *n_out = 0;
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && rows_out, "mgcn_heavy_rows: null array");
  if (workspace == nullptr || workspace_bytes < sizeof(unsigned long long)) {
    set_error("mgcn_heavy_rows: workspace needs %zu bytes", sizeof(unsigned long long));
    return MGCN_EWORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  auto *count = static_cast<unsigned long long *>(workspace);
  MGCN_HIP_TRY(hipMemsetAsync(count, 0, sizeof(*count), s));
  hipLaunchKernelGGL(heavy_rows_kernel, dim3(grid_for(n_rows, kBlock)), dim3(kBlock), 0, s, n_rows,
                     rowptr, thr, rows_out, count);
  if (int rc = check_launch("heavy_rows_kernel")) return rc;
  unsigned long long c = 0;
  MGCN_HIP_TRY(hipMemcpyAsync(&c, count, sizeof(c), hipMemcpyDeviceToHost, s));
  MGCN_HIP_TRY(hipStreamSynchronize(s));
  *n_out = (int64_t)c;
  return MGCN_OK;
}
