// Dense epilogue passes around the aggregation (gfx950, HBM-bound).
//
//  * mgcn_relu_bwd_colsum: dY = Z > 0 ? dZ : 0 and db = column sums of dY in
//    one read of dZ/Z (autograd's threshold_backward + the bias-gradient sum of
//    `x + self.bias`, gcn_base_models.py:240-241 / gcn_model.py:196).
//    Algorithmic bytes: 8 n F read + 4 n F written (relu) or 4 n F read.
//    The column sum is two-stage and deterministic: block partials in a fixed
//    row order, then one block folds the partials in block order.
//  * mgcn_segment_mean: PyG global_mean_pool over a collated batch whose nodes
//    are contiguous per graph (kernel/gcn.py:29), summed in node order.

#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxPartialBlocks = 1024;

template <int VEC>
__device__ __forceinline__ void load_vec(const float *p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    const float4 a = *reinterpret_cast<const float4 *>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
    v[0] = p[0];
  }
}
template <int VEC>
__device__ __forceinline__ void store_vec(float *p, const float (&v)[VEC]) {
  if constexpr (VEC == 4)
    *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else
    p[0] = v[0];
}

// Block b owns rows b, b + gridDim.x, ... ; thread t owns columns
// [c*T*4 + t_col*4, +4) for column chunk c, where T threads cover a row.
template <int VEC>
__global__ __launch_bounds__(kBlock) void relu_bwd_colsum_kernel(
    int64_t n, int F, const float *__restrict__ dZ, const float *__restrict__ Z, int relu,
    const float *__restrict__ row_div, float *__restrict__ dY,
    float *__restrict__ partial /*[gridDim.x][F]*/, int T) {
  __shared__ float red[kBlock * VEC];
  const int R = kBlock / T;  // row slots per block iteration
  const int t_col = threadIdx.x % T;
  const int t_row = threadIdx.x / T;
  for (int c0 = 0; c0 < F; c0 += T * VEC) {
    const int f0 = c0 + t_col * VEC;
    const bool f_ok = (t_row < R) && (f0 < F);
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.0f;
    if (f_ok) {
      // kUR rows per step, their loads issued before any is used: with the
      // dY store in the loop a row at a time waited a full memory round
      // trip per row (mean's top layer: 0.41 ms at config 2).  Rows are
      // still summed in ascending order: the same column sums bit for bit.
      constexpr int kUR = 4;
      const int64_t stride = (int64_t)gridDim.x * R;
      for (int64_t r0 = (int64_t)blockIdx.x * R + t_row; r0 < n; r0 += kUR * stride) {
        float g[kUR][VEC], z[kUR][VEC], dv[kUR];
#pragma unroll
        for (int u = 0; u < kUR; ++u) {
          const int64_t r = r0 + u * stride;
          const bool ok = r < n;
          const int64_t off = (ok ? r : 0) * F + f0;
          load_vec<VEC>(dZ + off, g[u]);
          if (relu) load_vec<VEC>(Z + off, z[u]);
          dv[u] = row_div != nullptr ? row_div[ok ? r : 0] : 1.0f;
        }
#pragma unroll
        for (int u = 0; u < kUR; ++u) {
          const int64_t r = r0 + u * stride;
          if (r >= n) break;
          if (relu) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) g[u][j] = (z[u][j] > 0.0f) ? g[u][j] : 0.0f;
          }
          if ((relu || row_div != nullptr) && dY != nullptr) {
            float o[VEC];  // mean aggregation: rows pre-divided by their count
#pragma unroll
            for (int j = 0; j < VEC; ++j) o[j] = row_div != nullptr ? __fdiv_rn(g[u][j], dv[u]) : g[u][j];
            store_vec<VEC>(dY + r * F + f0, o);
          }
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], g[u][j]);
        }
      }
    }
    if (partial == nullptr) continue;
    // fold the R row slots of this block (fixed order)
#pragma unroll
    for (int j = 0; j < VEC; ++j) red[threadIdx.x * VEC + j] = acc[j];
    __syncthreads();
    if (t_row == 0 && f0 < F) {
      float s[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) s[j] = red[t_col * VEC + j];
      for (int rr = 1; rr < R; ++rr)
#pragma unroll
        for (int j = 0; j < VEC; ++j) s[j] = __fadd_rn(s[j], red[(rr * T + t_col) * VEC + j]);
#pragma unroll
      for (int j = 0; j < VEC; ++j) partial[(int64_t)blockIdx.x * F + f0 + j] = s[j];
    }
    __syncthreads();
  }
}


// GCNModel residual join (gcn_model.py:99-105): Z = act(Z1 + (R + rb)),
// the residual Linear's bias added to its product first (as F.linear does).
template <int VEC>
__global__ __launch_bounds__(kBlock) void residual_act_kernel(
    int64_t n, int F, const float *__restrict__ Z1, int64_t ldz1, const float *__restrict__ R,
    int64_t ldr, const float *__restrict__ rb, int relu, float *__restrict__ Z, int64_t ldz) {
  const int fv = F / VEC;
  const int64_t total = n * fv;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / fv;
    const int f0 = (int)(i % fv) * VEC;
    float z1[VEC], v[VEC], b[VEC];
    load_vec<VEC>(Z1 + r * ldz1 + f0, z1);
    load_vec<VEC>(R + r * ldr + f0, v);
    if (rb != nullptr) load_vec<VEC>(rb + f0, b);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      if (rb != nullptr) v[j] = __fadd_rn(v[j], b[j]);
      v[j] = __fadd_rn(z1[j], v[j]);
      if (relu && v[j] < 0.0f) v[j] = 0.0f;
    }
    store_vec<VEC>(Z + r * ldz + f0, v);
  }
}

// Its adjoint with the layer's own ReLU (Z1 = relu(A Z W + b)):
//   dS = relu ? (Z > 0 ? dZ : 0) : dZ       (grad of the residual branch R)
//   dA = relu1 ? (Z1 > 0 ? dS : 0) : dS     (grad of the aggregation, / row_div)
// and the column sums of dA (bias b) and dS (residual bias rb) into block
// partials [block][2F] in a fixed row order (launch_colsum_fold folds them).
template <int VEC>
__global__ __launch_bounds__(kBlock) void residual_act_bwd_kernel(
    int64_t n, int F, const float *__restrict__ dZ, int64_t lddz, const float *__restrict__ Z,
    int64_t ldz, int relu, const float *__restrict__ Z1, int64_t ldz1, int relu1,
    const float *__restrict__ row_div, float *__restrict__ dA, int64_t ldda,
    float *__restrict__ dS, int64_t ldds, float *__restrict__ partial, int T) {
  __shared__ float red[2][kBlock * VEC];
  const int R = kBlock / T;
  const int t_col = threadIdx.x % T, t_row = threadIdx.x / T;
  for (int c0 = 0; c0 < F; c0 += T * VEC) {
    const int f0 = c0 + t_col * VEC;
    const bool ok = t_row < R && f0 < F;
    float sa[VEC], ss[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) sa[j] = ss[j] = 0.0f;
    if (ok) {
      // kUR rows per step with their loads issued first (see
      // relu_bwd_colsum_kernel); rows summed in ascending order as before
      constexpr int kUR = 4;
      const int64_t stride = (int64_t)gridDim.x * R;
      for (int64_t r0 = (int64_t)blockIdx.x * R + t_row; r0 < n; r0 += kUR * stride) {
        float g[kUR][VEC], z[kUR][VEC], z1[kUR][VEC], dv[kUR];
#pragma unroll
        for (int u = 0; u < kUR; ++u) {
          const int64_t r0u = r0 + u * stride;
          const int64_t r = r0u < n ? r0u : 0;
          load_vec<VEC>(dZ + r * lddz + f0, g[u]);
          if (relu) load_vec<VEC>(Z + r * ldz + f0, z[u]);
          if (relu1) load_vec<VEC>(Z1 + r * ldz1 + f0, z1[u]);
          dv[u] = row_div != nullptr ? row_div[r] : 1.0f;
        }
#pragma unroll
        for (int u = 0; u < kUR; ++u) {
          const int64_t r = r0 + u * stride;
          if (r >= n) break;
          float a[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            if (relu && !(z[u][j] > 0.0f)) g[u][j] = 0.0f;
            a[j] = (relu1 && !(z1[u][j] > 0.0f)) ? 0.0f : g[u][j];
            ss[j] = __fadd_rn(ss[j], g[u][j]);
            sa[j] = __fadd_rn(sa[j], a[j]);
            if (row_div != nullptr) a[j] = __fdiv_rn(a[j], dv[u]);
          }
          if (dS != nullptr) store_vec<VEC>(dS + r * ldds + f0, g[u]);
          store_vec<VEC>(dA + r * ldda + f0, a);
        }
      }
    }
    if (partial == nullptr) continue;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      red[0][threadIdx.x * VEC + j] = sa[j];
      red[1][threadIdx.x * VEC + j] = ss[j];
    }
    __syncthreads();
    if (t_row == 0 && f0 < F) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float a = red[0][t_col * VEC + j], b = red[1][t_col * VEC + j];
        for (int rr = 1; rr < R; ++rr) {
          a = __fadd_rn(a, red[0][(rr * T + t_col) * VEC + j]);
          b = __fadd_rn(b, red[1][(rr * T + t_col) * VEC + j]);
        }
        partial[(int64_t)blockIdx.x * 2 * F + f0 + j] = a;
        partial[(int64_t)blockIdx.x * 2 * F + F + f0 + j] = b;
      }
    }
    __syncthreads();
  }
}


// GCNModel's input layer (in_channels = 1, the botnet node feature; gcn_model.py
// :89-105 with residual_hop = 1) associated as (A x) W: with a = A x (the
// 1-wide aggregation, mgcn_spmm_fwd) every output is elementwise,
//   Z[i, j] = relu2( relu1(a_i W_j + b_j) + (x_i Wr_j + br_j) )
// -- the reference's A (x W) to fp32 rounding, without the 32-wide gather.
// Thread t of a row group owns columns 4 t .. 4 t + 3.
__global__ __launch_bounds__(kBlock) void input_layer_fwd_kernel(
    int64_t n, int F, const float *__restrict__ a, const float *__restrict__ x,
    const float *__restrict__ W, const float *__restrict__ b, const float *__restrict__ Wr,
    const float *__restrict__ br, int relu1, int relu2, float *__restrict__ Z, int64_t ldz) {
  const int fv = F / 4;
  const int64_t total = n * fv;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / fv;
    const int f0 = (int)(i % fv) * 4;
    const float ar = a[r], xr = x[r];
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float z1 = __fmul_rn(ar, W[f0 + j]);
      if (b != nullptr) z1 = __fadd_rn(z1, b[f0 + j]);
      if (relu1 && z1 < 0.0f) z1 = 0.0f;
      float rv = __fmul_rn(xr, Wr[f0 + j]);
      if (br != nullptr) rv = __fadd_rn(rv, br[f0 + j]);
      v[j] = __fadd_rn(z1, rv);
      if (relu2 && v[j] < 0.0f) v[j] = 0.0f;
    }
    *reinterpret_cast<float4 *>(Z + r * ldz + f0) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Its adjoint: dS = relu2' dZ, dA = relu1' dS (relu1's decision recomputed
// with the forward's arithmetic, bit for bit), and the four parameter
// gradients as column sums in a fixed row order (block partials [block][4F]:
// dW_j = sum a_i dA_ij | db_j = sum dA_ij | dWr_j = sum x_i dS_ij | dbr_j =
// sum dS_ij); with da (nullable): da_i = sum_j dA_ij W_j [/ row_div_i] (the
// 1-wide adjoint SpMM's input) and dxr_i = sum_j dS_ij Wr_j, the row sums in
// a fixed xor-butterfly over the row's T threads.
__global__ __launch_bounds__(kBlock) void input_layer_bwd_kernel(
    int64_t n, int F, const float *__restrict__ dZ, int64_t lddz, const float *__restrict__ Z,
    int64_t ldz, const float *__restrict__ a, const float *__restrict__ x,
    const float *__restrict__ W, const float *__restrict__ b, const float *__restrict__ Wr,
    int relu1, int relu2, const float *__restrict__ row_div, float *__restrict__ da,
    float *__restrict__ dxr, float *__restrict__ partial, int T) {
  __shared__ float red[kBlock * 16];
  const int R = kBlock / T;
  const int t_col = threadIdx.x % T, t_row = threadIdx.x / T;
  const int f0 = t_col * 4;
  float sw[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0}, swr[4] = {0, 0, 0, 0}, sbr[4] = {0, 0, 0, 0};
  float w[4], bb[4], wr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w[j] = W[f0 + j];
    bb[j] = b != nullptr ? b[f0 + j] : 0.0f;
    wr[j] = Wr[f0 + j];
  }
  const int64_t stride = (int64_t)gridDim.x * R;
  // every thread of a row group runs the same rows (the butterfly below)
  for (int64_t r = (int64_t)blockIdx.x * R + t_row; r - t_row < n; r += stride) {
    const bool ok = r < n;
    const int64_t rr = ok ? r : 0;
    const float4 g4 = *reinterpret_cast<const float4 *>(dZ + rr * lddz + f0);
    float4 z4 = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    if (relu2) z4 = *reinterpret_cast<const float4 *>(Z + rr * ldz + f0);
    const float ar = a[rr], xr = x[rr];
    const float g[4] = {g4.x, g4.y, g4.z, g4.w}, zz[4] = {z4.x, z4.y, z4.z, z4.w};
    float pa = 0.0f, ps = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float ds = (!ok || (relu2 && !(zz[j] > 0.0f))) ? 0.0f : g[j];
      float z1 = __fmul_rn(ar, w[j]);
      if (b != nullptr) z1 = __fadd_rn(z1, bb[j]);
      const float dA = (relu1 && !(z1 > 0.0f)) ? 0.0f : ds;
      sw[j] = __fadd_rn(sw[j], __fmul_rn(ar, dA));
      sb[j] = __fadd_rn(sb[j], dA);
      swr[j] = __fadd_rn(swr[j], __fmul_rn(xr, ds));
      sbr[j] = __fadd_rn(sbr[j], ds);
      if (da != nullptr) {
        pa = __fadd_rn(pa, __fmul_rn(dA, w[j]));
        ps = __fadd_rn(ps, __fmul_rn(ds, wr[j]));
      }
    }
    if (da != nullptr) {
      for (int m = 1; m < T; m <<= 1) {
        pa = __fadd_rn(pa, __shfl_xor(pa, m, 64));
        ps = __fadd_rn(ps, __shfl_xor(ps, m, 64));
      }
      if (ok && t_col == 0) {
        da[r] = row_div != nullptr ? __fdiv_rn(pa, row_div[r]) : pa;
        dxr[r] = ps;
      }
    }
  }
  if (partial == nullptr) return;
  float *my = red + threadIdx.x * 16;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    my[j] = sw[j];
    my[4 + j] = sb[j];
    my[8 + j] = swr[j];
    my[12 + j] = sbr[j];
  }
  __syncthreads();
  if (t_row == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float acc = red[t_col * 16 + q];
      for (int k = 1; k < R; ++k) acc = __fadd_rn(acc, red[(k * T + t_col) * 16 + q]);
      // [dW | db | dWr | dbr], 4 columns per quantity
      partial[(int64_t)blockIdx.x * 4 * F + (q >> 2) * F + f0 + (q & 3)] = acc;
    }
  }
}

// one wave per segment; lanes stride the features
__global__ __launch_bounds__(kBlock) void segment_mean_kernel(int64_t n_seg, int F,
                                                              const int64_t *__restrict__ ptr,
                                                              const float *__restrict__ x,
                                                              int64_t ldx, float *__restrict__ out,
                                                              int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (seg >= n_seg) return;
  const int64_t b = ptr[seg], e = ptr[seg + 1];
  const float cnt = (float)((e - b) > 1 ? (e - b) : 1);
  for (int f = lane; f < F; f += 64) {
    float s = 0.0f;
    for (int64_t i = b; i < e; ++i) s = __fadd_rn(s, x[i * ldx + f]);
    out[seg * ldo + f] = __fdiv_rn(s, cnt);
  }
}

int colsum_blocks(int64_t n) {
  int64_t b = (n + 63) / 64;
  if (b > kMaxPartialBlocks) b = kMaxPartialBlocks;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" size_t mgcn_colsum_workspace_bytes(int64_t n_rows, int32_t F) {
  return align_up((size_t)colsum_blocks(n_rows) * (size_t)(F > 0 ? F : 1) * sizeof(float), 256);
}

extern "C" int mgcn_relu_bwd_colsum(int64_t n_rows, int32_t F, const float *dZ, const float *Z,
                                    int relu, const float *row_div, float *dY, float *db,
                                    void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_relu_bwd_colsum: negative size");
  hipStream_t s = as_stream(stream);
  if (F == 0) return MGCN_OK;
  if (n_rows == 0) {
    if (db) MGCN_HIP_TRY(hipMemsetAsync(db, 0, sizeof(float) * F, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(dZ != nullptr, "mgcn_relu_bwd_colsum: dZ is null");
  MGCN_REQUIRE(!relu || Z != nullptr, "mgcn_relu_bwd_colsum: relu needs Z");
  const int nblk = colsum_blocks(n_rows);
  float *partial = nullptr;
  if (db != nullptr) {
    const size_t need = mgcn_colsum_workspace_bytes(n_rows, F);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_relu_bwd_colsum: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    partial = static_cast<float *>(workspace);
  }
  const bool v4 = (F % 4 == 0) && ((uintptr_t)dZ % 16 == 0) && (!relu || (uintptr_t)Z % 16 == 0) &&
                  (dY == nullptr || (uintptr_t)dY % 16 == 0);
  if (v4) {
    int T = 1;
    while (T < F / 4 && T < kBlock) T <<= 1;
    hipLaunchKernelGGL(relu_bwd_colsum_kernel<4>, dim3(nblk), dim3(kBlock), 0, s, n_rows, F, dZ, Z,
                       relu, row_div, dY, partial, T);
  } else {
    int T = 1;
    while (T < F && T < kBlock) T <<= 1;
    hipLaunchKernelGGL(relu_bwd_colsum_kernel<1>, dim3(nblk), dim3(kBlock), 0, s, n_rows, F, dZ, Z,
                       relu, row_div, dY, partial, T);
  }
  if (int rc = check_launch("relu_bwd_colsum_kernel")) return rc;
  if (db != nullptr) {
    return launch_colsum_fold(partial, nblk, F, db, s);
  }
  return MGCN_OK;
}

namespace mgcn {
namespace {
// C = A . B for a handful of K (the 1 -> 32 input layer x @ [W | Wr^T] and
// the 32 -> 2 projection's dX = dY W of config 3): one thread per 4 outputs
// of a row, the K products accumulated in k order on fma (a BLAS's order for
// K <= 8); HBM-bound: 4 M (K + N) bytes.  hipBLASLt spends 35-38 us on
// these shapes at config 3, this ~8.
constexpr int kSmallK = 8;
constexpr int kSmallN = 128;
__global__ __launch_bounds__(256) void gemm_small_k_kernel(int64_t M, int K, int N,
                                                           const float *__restrict__ A,
                                                           int64_t lda,
                                                           const float *__restrict__ B,
                                                           int64_t sbk, int64_t sbn,
                                                           float *__restrict__ C, int64_t ldc) {
  // B staged once per workgroup as [k][n] (zeros past K / N)
  __shared__ __attribute__((aligned(16))) float Bs[kSmallK][kSmallN];
  for (int e = threadIdx.x; e < kSmallK * kSmallN; e += 256) {
    const int k = e / kSmallN, n = e % kSmallN;
    Bs[k][n] = (k < K && n < N) ? B[k * sbk + n * sbn] : 0.0f;
  }
  __syncthreads();
  const int nq = (N + 3) / 4;
  const int64_t total = M * nq;
  const bool vec = (ldc & 3) == 0 && ((uintptr_t)C & 15) == 0 && (N & 3) == 0;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / nq;
    const int j0 = 4 * (int)(t - i * nq);
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < kSmallK; ++k) {
      if (k < K) {
        const float a = A[i * lda + k];
        const float4 b = *reinterpret_cast<const float4 *>(&Bs[k][j0]);
        if (k == 0) {
          c = make_float4(__fmul_rn(a, b.x), __fmul_rn(a, b.y), __fmul_rn(a, b.z),
                          __fmul_rn(a, b.w));
        } else {
          c.x = __fmaf_rn(a, b.x, c.x);
          c.y = __fmaf_rn(a, b.y, c.y);
          c.z = __fmaf_rn(a, b.z, c.z);
          c.w = __fmaf_rn(a, b.w, c.w);
        }
      }
    }
    float *dst = C + i * ldc + j0;
    if (vec) {
      *reinterpret_cast<float4 *>(dst) = c;
    } else {
      const float cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q < N) dst[q] = cv[q];
    }
  }
}
}  // namespace
}  // namespace mgcn

extern "C" int mgcn_gemm_small_k(int64_t M, int32_t K, int32_t N, const float *A, int64_t lda,
                                 const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                                 void *stream) {
  clear_error();
  MGCN_REQUIRE(M >= 0 && N >= 0 && K >= 1 && K <= kSmallK && N <= kSmallN,
               "mgcn_gemm_small_k: need 1 <= K <= %d, N <= %d (K=%d, N=%d)", kSmallK, kSmallN, K,
               N);
  if (M == 0 || N == 0) return MGCN_OK;
  MGCN_REQUIRE(A && B && C && lda >= K && ldc >= N, "mgcn_gemm_small_k: bad arguments");
  const int64_t work = M * ((N + 3) / 4);
  hipLaunchKernelGGL(gemm_small_k_kernel, dim3(grid_for(work, 256)), dim3(256), 0,
                     as_stream(stream), M, K, N, A, lda, B, sbk, sbn, C, ldc);
  return check_launch("gemm_small_k_kernel");
}

extern "C" int mgcn_segment_mean(int64_t n_seg, int32_t F, const int64_t *ptr, const float *x,
                                 int64_t ldx, float *out, int64_t ldo, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_seg >= 0 && F >= 0, "mgcn_segment_mean: negative size");
  if (n_seg == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(ptr && x && out && ldx >= F && ldo >= F, "mgcn_segment_mean: bad arguments");
  const int64_t blocks = (n_seg + (kBlock / 64) - 1) / (kBlock / 64);
  hipLaunchKernelGGL(segment_mean_kernel, dim3((unsigned)blocks), dim3(kBlock), 0,
                     as_stream(stream), n_seg, F, ptr, x, ldx, out, ldo);
  return check_launch("segment_mean_kernel");
}

extern "C" int mgcn_residual_act(int64_t n_rows, int32_t F, const float *Z1, int64_t ldz1,
                                 const float *R, int64_t ldr, const float *rbias, int relu,
                                 float *Z, int64_t ldz, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_residual_act: negative size");
  if (n_rows == 0 || F == 0) return MGCN_OK;
  MGCN_REQUIRE(Z1 && R && Z && ldz1 >= F && ldr >= F && ldz >= F,
               "mgcn_residual_act: bad arguments");
  const bool v4 = F % 4 == 0 && ldz1 % 4 == 0 && ldr % 4 == 0 && ldz % 4 == 0 &&
                  (uintptr_t)Z1 % 16 == 0 && (uintptr_t)R % 16 == 0 && (uintptr_t)Z % 16 == 0 &&
                  (rbias == nullptr || (uintptr_t)rbias % 16 == 0);
  const int vec = v4 ? 4 : 1;
  const unsigned g = grid_for(n_rows * (F / vec), kBlock);
  if (vec == 4)
    hipLaunchKernelGGL(residual_act_kernel<4>, dim3(g), dim3(kBlock), 0, as_stream(stream), n_rows,
                       F, Z1, ldz1, R, ldr, rbias, relu, Z, ldz);
  else
    hipLaunchKernelGGL(residual_act_kernel<1>, dim3(g), dim3(kBlock), 0, as_stream(stream), n_rows,
                       F, Z1, ldz1, R, ldr, rbias, relu, Z, ldz);
  return check_launch("residual_act_kernel");
}

extern "C" size_t mgcn_residual_act_bwd_workspace_bytes(int64_t n_rows, int32_t F) {
  return mgcn_colsum_workspace_bytes(n_rows, 2 * (F > 0 ? F : 1));
}

extern "C" int mgcn_residual_act_bwd(int64_t n_rows, int32_t F, const float *dZ, int64_t lddz,
                                     const float *Z, int64_t ldz, int relu, const float *Z1,
                                     int64_t ldz1, int relu1, const float *row_div, float *dA,
                                     int64_t ldda, float *dS, int64_t ldds, float *colsums,
                                     void *workspace, size_t workspace_bytes, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 0, "mgcn_residual_act_bwd: negative size");
  hipStream_t s = as_stream(stream);
  if (F == 0) return MGCN_OK;
  if (n_rows == 0) {
    if (colsums) MGCN_HIP_TRY(hipMemsetAsync(colsums, 0, sizeof(float) * 2 * F, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(dZ && dA && lddz >= F && ldda >= F, "mgcn_residual_act_bwd: bad dZ/dA");
  MGCN_REQUIRE(!relu || (Z && ldz >= F), "mgcn_residual_act_bwd: relu needs Z");
  MGCN_REQUIRE(!relu1 || (Z1 && ldz1 >= F), "mgcn_residual_act_bwd: relu1 needs Z1");
  MGCN_REQUIRE(dS == nullptr || ldds >= F, "mgcn_residual_act_bwd: bad dS");
  const int nblk = colsum_blocks(n_rows);
  float *partial = nullptr;
  if (colsums != nullptr) {
    const size_t need = mgcn_residual_act_bwd_workspace_bytes(n_rows, F);
    if (workspace == nullptr || workspace_bytes < need) {
      set_error("mgcn_residual_act_bwd: workspace %zu < %zu", workspace_bytes, need);
      return MGCN_EWORKSPACE;
    }
    partial = static_cast<float *>(workspace);
  }
  auto al = [](const void *p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % 4 == 0); };
  const bool v4 = F % 4 == 0 && al(dZ, lddz) && (!relu || al(Z, ldz)) &&
                  (!relu1 || al(Z1, ldz1)) && al(dA, ldda) && al(dS, ldds);
  int T = 1;
  if (v4) {
    while (T < F / 4 && T < kBlock) T <<= 1;
    hipLaunchKernelGGL(residual_act_bwd_kernel<4>, dim3(nblk), dim3(kBlock), 0, s, n_rows, F, dZ,
                       lddz, Z, ldz, relu, Z1, ldz1, relu1, row_div, dA, ldda, dS, ldds, partial, T);
  } else {
    while (T < F && T < kBlock) T <<= 1;
    hipLaunchKernelGGL(residual_act_bwd_kernel<1>, dim3(nblk), dim3(kBlock), 0, s, n_rows, F, dZ,
                       lddz, Z, ldz, relu, Z1, ldz1, relu1, row_div, dA, ldda, dS, ldds, partial, T);
  }
  if (int rc = check_launch("residual_act_bwd_kernel")) return rc;
  if (colsums == nullptr) return MGCN_OK;
  return launch_colsum_fold(partial, nblk, 2 * F, colsums, s);
}

extern "C" int mgcn_input_layer_supported(int32_t F_in, int32_t F) {
  return F_in == 1 && F >= 4 && F <= 256 && F % 4 == 0 && ((F / 4) & (F / 4 - 1)) == 0;
}

extern "C" int mgcn_input_layer_fwd(int64_t n_rows, int32_t F, const float *a, const float *x,
                                    const float *W, const float *b, const float *Wr,
                                    const float *br, int relu1, int relu2, float *Z, int64_t ldz,
                                    void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && mgcn_input_layer_supported(1, F),
               "mgcn_input_layer_fwd: F = %d (needs F / 4 a power of two, 4 <= F <= 256)", F);
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(a && x && W && Wr && Z && ldz >= F && ldz % 4 == 0 && (uintptr_t)Z % 16 == 0,
               "mgcn_input_layer_fwd: bad arguments (Z needs 16-byte aligned rows)");
  const unsigned g = grid_for(n_rows * (F / 4), kBlock);
  hipLaunchKernelGGL(input_layer_fwd_kernel, dim3(g), dim3(kBlock), 0, as_stream(stream), n_rows,
                     (int)F, a, x, W, b, Wr, br, relu1, relu2, Z, ldz);
  return check_launch("input_layer_fwd_kernel");
}

extern "C" size_t mgcn_input_layer_bwd_workspace_bytes(int64_t n_rows, int32_t F) {
  return mgcn_colsum_workspace_bytes(n_rows, 4 * (F > 0 ? F : 1));
}

extern "C" int mgcn_input_layer_bwd(int64_t n_rows, int32_t F, const float *dZ, int64_t lddz,
                                    const float *Z, int64_t ldz, const float *a, const float *x,
                                    const float *W, const float *b, const float *Wr, int relu1,
                                    int relu2, const float *row_div, float *da, float *dxr,
                                    float *grads, void *workspace, size_t workspace_bytes,
                                    void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && mgcn_input_layer_supported(1, F),
               "mgcn_input_layer_bwd: F = %d (needs F / 4 a power of two, 4 <= F <= 256)", F);
  MGCN_REQUIRE(grads != nullptr && (da == nullptr) == (dxr == nullptr),
               "mgcn_input_layer_bwd: grads required; da and dxr go together");
  hipStream_t s = as_stream(stream);
  if (n_rows == 0) {
    MGCN_HIP_TRY(hipMemsetAsync(grads, 0, sizeof(float) * 4 * F, s));
    return MGCN_OK;
  }
  MGCN_REQUIRE(dZ && a && x && W && Wr && lddz >= F && lddz % 4 == 0 && (uintptr_t)dZ % 16 == 0 &&
                   (!relu2 || (Z && ldz >= F && ldz % 4 == 0 && (uintptr_t)Z % 16 == 0)),
               "mgcn_input_layer_bwd: bad arguments (dZ / Z need 16-byte aligned rows)");
  const size_t need = mgcn_input_layer_bwd_workspace_bytes(n_rows, F);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_input_layer_bwd: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  const int nblk = colsum_blocks(n_rows);
  float *partial = static_cast<float *>(workspace);
  hipLaunchKernelGGL(input_layer_bwd_kernel, dim3(nblk), dim3(kBlock), 0, s, n_rows, (int)F, dZ,
                     lddz, Z, ldz, a, x, W, b, Wr, relu1, relu2, row_div, da, dxr, partial,
                     (int)(F / 4));
  if (int rc = check_launch("input_layer_bwd_kernel")) return rc;
  return launch_colsum_fold(partial, nblk, 4 * F, grads, s);
}
