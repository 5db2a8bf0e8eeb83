// Adjoint of the per-edge normalisation weights (gfx950): the gradient that
// flows from the aggregation back into edge_weight / deg through
// NodeModelBase.degnorm_const (src/gcn_meta/models/gcn_base_models.py:65-146).
//
// The reference scales every gathered message by its edge's weight,
//   x_j = index_select(H, 0, src) * norm.view(-1, 1)     (:217-224)
// and autograd's mul backward reduces the message gradient against the
// gathered row:  dnorm_e = sum_f dX_j[e, f] * H[src_e, f],  dX_j[e] = dY[dst_e]
// (scatter_add's backward is a gather, :237; scatter_max's routes through the
// winner only, common.py:59-64).  That is a sampled dense-dense product
// (SDDMM) over the edges: one dot product of two F-wide rows per edge.
//
// Here: one wave per destination row of the fwd CSR view (row = dst, col =
// src), grid-stride over rows; the row's dY (already divided by the in-degree
// for mean, as the SpMM adjoint receives it) is held in registers, FPL floats
// per lane (feature lane + 64 i), and each edge gathers its H row (coalesced,
// U rows in flight), forms its products lane-locally in feature order and
// reduces them across the wave by a fixed xor-butterfly: deterministic, but
// not the reference's summation order (a CPU sum over [E, F]), so the result
// matches it to fp32 rounding, not bit for bit.  Max: a feature counts only
// where the edge won it (win_mask, mgcn_spmm_fwd's layout).  The output is in
// fwd slot order (the slot's edge id is view.eid[slot]).
//
// Roofline: HBM-bound like the SpMM -- 8 (N + 1) + nnz (4 col + 4F row + 4
// out) + 4 N F (dY) bytes; 2 nnz F flops.  The chain from dnorm to
// edge_weight / deg (degree sums, x^-1/2 derivative) is E- and N-length
// elementwise work done by the host layer (meta-gcn_amd/mgcn/graph.py).

#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kSdWaves = 4;
constexpr int kSdThreads = 64 * kSdWaves;
constexpr int kSdU = 4;

template <int FPL>
__global__ __launch_bounds__(kSdThreads) void sddmm_kernel(
    int64_t n_rows, int32_t F, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const float *__restrict__ H, int64_t ldh, const float *__restrict__ dY, int64_t lddy,
    const uint32_t *__restrict__ win, int nw, float *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = blockIdx.x * (int64_t)kSdWaves + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * kSdWaves;
  for (int64_t row = wave0; row < n_rows; row += nwaves) {
    float dy[FPL];
#pragma unroll
    for (int i = 0; i < FPL; ++i) {
      const int f = lane + 64 * i;
      dy[i] = f < F ? dY[row * lddy + f] : 0.0f;
    }
    const int64_t beg = rowptr[row], end = rowptr[row + 1];
    for (int64_t k0 = beg; k0 < end; k0 += kSdU) {
      float h[kSdU][FPL];
      int32_t ck[kSdU];
#pragma unroll
      for (int u = 0; u < kSdU; ++u) {
        const int64_t k = k0 + u;
        ck[u] = k < end ? col[k] : 0;
#pragma unroll
        for (int i = 0; i < FPL; ++i) {
          const int f = lane + 64 * i;
          h[u][i] = (k < end && f < F) ? H[(int64_t)ck[u] * ldh + f] : 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < kSdU; ++u) {
        const int64_t k = k0 + u;
        float p = 0.0f;
#pragma unroll
        for (int i = 0; i < FPL; ++i) {
          float t = __fmul_rn(dy[i], h[u][i]);
          if (win != nullptr) {
            const int f = lane + 64 * i;
            const uint32_t bits = (k < end && f < F) ? win[k * nw + (f >> 5)] : 0u;
            t = ((bits >> (f & 31)) & 1u) ? t : 0.0f;
          }
          p = __fadd_rn(p, t);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) p = __fadd_rn(p, __shfl_xor(p, off, 64));
        if (lane == 0 && k < end) out[k] = p;
      }
    }
  }
}

template <int FPL>
int launch_sddmm(int64_t n_rows, int32_t F, const int64_t *rowptr, const int32_t *col,
                 const float *H, int64_t ldh, const float *dY, int64_t lddy, const uint32_t *win,
                 float *out, hipStream_t s) {
  int64_t blocks = (n_rows + kSdWaves - 1) / kSdWaves;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((sddmm_kernel<FPL>), dim3((unsigned)blocks), dim3(kSdThreads), 0, s, n_rows,
                     F, rowptr, col, H, ldh, dY, lddy, win, (F + 31) / 32, out);
  return check_launch("sddmm_kernel");
}

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" int mgcn_edge_weight_grad(int64_t n_rows, int32_t F, const int64_t *rowptr,
                                     const int32_t *col, const float *H, int64_t ldh,
                                     const float *dY, int64_t lddy, const uint32_t *win_mask,
                                     float *dw, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && F >= 1 && F <= 1024,
               "mgcn_edge_weight_grad: need n_rows >= 0 and 1 <= F <= 1024 (F = %d)", F);
  if (n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(rowptr && H && dY && dw, "mgcn_edge_weight_grad: null array");
  MGCN_REQUIRE(ldh >= F && lddy >= F, "mgcn_edge_weight_grad: leading dimension too small");
  hipStream_t s = as_stream(stream);
  const int fpl = (F + 63) / 64;
  if (fpl <= 1) return launch_sddmm<1>(n_rows, F, rowptr, col, H, ldh, dY, lddy, win_mask, dw, s);
  if (fpl <= 2) return launch_sddmm<2>(n_rows, F, rowptr, col, H, ldh, dY, lddy, win_mask, dw, s);
  if (fpl <= 4) return launch_sddmm<4>(n_rows, F, rowptr, col, H, ldh, dY, lddy, win_mask, dw, s);
  if (fpl <= 8) return launch_sddmm<8>(n_rows, F, rowptr, col, H, ldh, dY, lddy, win_mask, dw, s);
  return launch_sddmm<16>(n_rows, F, rowptr, col, H, ldh, dY, lddy, win_mask, dw, s);
}
