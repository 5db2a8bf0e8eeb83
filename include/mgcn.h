/*
 * mgcn.h -- C ABI of libmgcn.so, the MI355X (gfx950) engine behind the GCN
 * neighbourhood aggregation  Y = reduce_{e: dst_e = i} w_e * H[src_e]  and its
 * adjoint  dH = A^T dY.
 *
 * Plain C: pointers, sizes and a `void *stream` (a hipStream_t; NULL = the
 * default stream).  No torch types.  Every buffer is BORROWED: the library
 * never allocates or frees device memory; scratch space is passed in by the
 * caller (see the *_workspace_bytes queries).  Every call returns 0 on
 * success or an MGCN_E* code; mgcn_last_error() (thread-local) says why.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to jzhou316/meta-gcn @ 2025-08-24):
 *
 *  - torch_scatter.scatter_{add,mean,max}(src, index, 0, out, dim_size, fill)
 *      called at src/gcn_meta/models/common.py:56-59 on the gathered-and-scaled
 *      edge tensor built at src/gcn_meta/models/gcn_base_models.py:209-224.
 *      The reference materialises x_j = x[src] * norm  ([E, F]) and then
 *      scatters it; mgcn_spmm_fwd fuses gather, scale, reduce, the
 *      `out[out == fill] = 0` fix-up (common.py:63-64), the bias add
 *      (gcn_base_models.py:240-241) and the layer ReLU
 *      (gcn_model.py:196, kernel/gcn.py:26-28) and never materialises [E, F].
 *  - the autograd adjoints of those ops (index_select -> index_add_,
 *      mul -> mul, scatter -> gather / argmax routing): mgcn_spmm_bwd.
 *  - NodeModelBase.degnorm_const (src/gcn_meta/models/gcn_base_models.py:65-146):
 *      mgcn_degree_norm + mgcn_edge_norm.
 *  - the per-forward graph bookkeeping of PyG (edge_index kept as COO and
 *      re-scattered every call): mgcn_csr_build, run once per static graph.
 */
#ifndef MGCN_H
#define MGCN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGCN_ABI_VERSION 22

/* return codes */
#define MGCN_OK 0
#define MGCN_EINVAL 1   /* bad argument (shape, alignment, null pointer)      */
#define MGCN_EINDEX 2   /* an edge index is outside [0, n)                    */
#define MGCN_EHIP 3     /* a HIP runtime call or kernel launch failed          */
#define MGCN_EWORKSPACE 4 /* caller-provided workspace is too small            */
#define MGCN_EDEVICE 5  /* a kernel reported a failure from the device: the
                           outputs of that launch are invalid (see
                           mgcn_check_device)                                 */

/* reductions (common.py:54 `name in ['add', 'mean', 'max']`) */
#define MGCN_REDUCE_SUM 0
#define MGCN_REDUCE_MEAN 1
#define MGCN_REDUCE_MAX 2

/* degree normalisation methods (gcn_base_models.py:45 deg_norm) */
#define MGCN_NORM_NONE 0
#define MGCN_NORM_SM 1 /* symmetric:  deg^-1/2[src] * w * deg^-1/2[dst]  */
#define MGCN_NORM_RW 2 /* random walk: deg^-1[src] * w                    */

/* fill value of the 'max' reduction (common.py:57) */
#define MGCN_MAX_FILL (-1e38f)

int mgcn_abi_version(void);
const char *mgcn_last_error(void);

/* Device-side failures (ABI 21).  The warp-specialised kernels (the 128-wide
 * adjoint behind mgcn_spmm_xw_bwd, the 256-wide layer kernels behind
 * mgcn_spmm_xw_fwd / _bwd) hand chunks between their waves through LDS
 * counters with bounded spins; a spin that runs past its bound makes every
 * wave leave, and the kernel then stores a code into a host-mapped error
 * word instead of finishing silently.  That word is reported as MGCN_EDEVICE
 * (+ mgcn_last_error naming the kernel) by the next mgcn_spmm_xw_* call, or
 * here: sync != 0 synchronises `stream` first, so every launch issued on it
 * before this call is covered.  Reading the word clears it.  No reference
 * counterpart (torch_scatter reports nothing from the device either). */
int mgcn_check_device(void *stream, int sync);

/* Tuning knobs (ABI 21: only knobs that keep every result within its tested
 * bound -- bit for bit, except gemm_precision).  Process-wide settings meant
 * to be set once at start-up (MGCN_OPTIONS="name=value,..." does that from
 * the environment), not per call; the defaults are the measured-fastest
 * forms.  Switches that change results (timing experiments: wide_dbg,
 * xw_ws_dbg) and the warp-specialised spin bound (ws_spin_limit) exist only
 * in the experiment build libmgcn_exp.so (make -C meta-gcn_amd/csrc exp);
 * this library rejects them (MGCN_EINVAL).
 *   "spmm_vec"    : cap the floats per lane of the SpMM gathers (1, 2, 4)
 *   "spmm_unroll" : gathers in flight per lane group (4, 8 or 16)
 *   "heavy_side_stream": 1 (default) runs the heavy-row launch on a side
 *                   stream concurrently with the lane-group launch; 0 serial
 *   "heavy_side_fence": 1 = system-scope events on that side stream
 *   "heavy_lds_kb": LDS per giant-row workgroup, 16..160 (default 160)
 *   "heavy_block" : threads per giant-row workgroup, 256/512/1024 (1024)
 *   "heavy_mid_lds_kb": LDS per (non-giant) heavy-row workgroup (default 40)
 *   "heavy_mid_q1": 1 (default) = one edge quad in flight per producer in the
 *                   non-giant heavy-row workgroups when a row is <= 32 floats
 *                   wide (fewer registers, more workgroups per CU); 0 = four
 *   "heavy_giant_thr" : degree above which a heavy row is giant, read by
 *                   mgcn_row_schedule (default 512)
 *   "residual_blocks": workgroup cap of the fused residual layer's launches
 *                   (default 8192; the backward's is also capped at 4096)
 *   "residual_fused_mask": 1 (default) the residual stack's lower-layer mask
 *                   pass fused into its launches
 *   "gemm_tn_variant": LDS-staged dW kernel chunk depth (M, N multiples of
 *                   128): 0 = 64 rows (default), 1 = 32, 2 = 16
 *   "gemm_tn_staged": 1 (default) the staged small-C kernel at M = 32
 *   "gemm_precision": product arithmetic of mgcn_gemm_nn / mgcn_gemm_tn:
 *                   1 = bf16x6 (default; fp32 operands split exactly into
 *                   three bf16 terms, six products on bf16 MFMA, fp32
 *                   accumulate -- fp32-level error), 0 = f32
 *                   MFMA (v_mfma_f32_32x32x2_f32)
 *   "spmm_xw_unroll": gathers in flight per row of the fused 128-wide layer
 *                   forward, 4 / 5 (default) / 6 / 8 (the two-phase adjoints:
 *                   8, else 4); every value folds in edge order (same bits)
 *   "xw_ws_full"  : 1 (default) = mgcn_spmm_xw_bwd's dW (+ dX) form on the
 *                   warp-specialised kernel (DWS), 0 = the two-phase kernel
 *   "xw_ws_max"   : 1 (default) = the max adjoint with dX on DWS as well
 *   "xw_ws_full_unroll": DWS gathers in flight per row, 4 / 5 (default) / 6
 *   "wide_ws"     : the 256-wide layer kernels: bit 0 the forward, bit 1 the
 *                   adjoint on the warp-specialised form (default 3), else
 *                   the 16-row two-phase form
 *   "wide_pair"   : the two-phase 256-wide form gathers a wave's two rows
 *                   together (bit 0 forward, bit 1 adjoint; default 3)
 *   "wide_mfma"   : MFMA waves of the warp-specialised 256-wide kernels, 4 / 8
 *                   (default)
 * (Measured-slower forms removed in round 6 live as patches under exp/.) */
int mgcn_set_option(const char *name, int value);

/* ------------------------------------------------------------------ graph */

/* Bytes of scratch mgcn_csr_build needs for `nnz` edges over `n` rows. */
size_t mgcn_csr_workspace_bytes(int64_t nnz, int64_t n);

/*
 * Build a CSR view of a COO edge list, grouping edges by `key` (pass
 * edge_index[1] = dst for the forward view, edge_index[0] = src for the
 * transposed view used by the backward pass).  Within a row the edges keep
 * their original (COO) order -- the order in which the reference's CPU
 * scatter_add / index_add_ accumulate -- so sums are reproduced bit for bit.
 *
 *   key[nnz], other[nnz] : int64 device arrays (rows of edge_index)
 *   rowptr[n + 1]        : int64 out
 *   col[nnz]             : int32 out, other[e] of each edge, row-grouped
 *   eid[nnz]             : int32 out, original edge id e of each CSR slot
 * Indices are validated: any key or other outside [0, n_key) / [0, n_other)
 * returns MGCN_EINDEX (this call synchronises `stream` once to check).
 * Replaces: COO edge_index consumed by index_select/scatter at
 * gcn_base_models.py:211-237 on every forward.
 */
int mgcn_csr_build(const int64_t *key, const int64_t *other, int64_t nnz,
                   int64_t n_key, int64_t n_other, int64_t *rowptr,
                   int32_t *col, int32_t *eid, void *workspace,
                   size_t workspace_bytes, void *stream);

/*
 * Node degrees and their inverse powers (gcn_base_models.py:117-135).
 *   deg_in      : optional precomputed degrees [n] (the `deg` argument);
 *                 when NULL the degree is the sum of edge weights (or the
 *                 edge count) over the rows of the given CSR, which must be
 *                 grouped by SOURCE node (gcn_base_models.py:124-126 sums
 *                 over edge_index[0]); the sum runs in edge order.
 *   edge_weight : optional [nnz] weights in COO order (indexed through eid).
 *   method      : MGCN_NORM_SM -> dinv = 1/sqrt(deg), MGCN_NORM_RW -> 1/deg;
 *                 +inf results become 0 (gcn_base_models.py:135).
 *   deg_out     : [n] degree actually used (may alias deg_in)
 *   dinv_out    : [n]
 */
int mgcn_degree_norm(int64_t n, const int64_t *rowptr_src, const int32_t *eid_src,
                     const float *deg_in, const float *edge_weight, int method,
                     float *deg_out, float *dinv_out, void *stream);

/*
 * Per-slot edge weights of a CSR view (gcn_base_models.py:137-142), stored in
 * the CSR's own slot order so the SpMM streams them:
 *   SM, no edge_weight : dinv[src] * dinv[dst]
 *   SM, edge_weight    : (dinv[src] * ew) * dinv[dst]
 *   RW, no edge_weight : dinv[src]   (the reference scales x rows before the
 *                                     gather, :217-220; same products)
 *   RW, edge_weight    : dinv[src] * ew
 *   NONE, edge_weight  : ew          (PyG GraphConv/SAGEConv message weights)
 * rows_are_dst = 1 for the forward (dst-grouped) view, 0 for the transposed.
 */
int mgcn_edge_norm(int64_t n_rows, int64_t nnz, const int64_t *rowptr, const int32_t *col,
                   const int32_t *eid, int rows_are_dst, const float *dinv,
                   const float *edge_weight, int method, float *w_out,
                   void *stream);

/* ------------------------------------------------------------ aggregation */

/*
 * Forward aggregation over a dst-grouped CSR (rows = destinations):
 *   acc_i = reduce_{k in row i, in edge order} ( H[col_k, :] * w_k )
 *   SUM : acc_i                   MEAN : acc_i / max(deg_i, 1)
 *   MAX : max with fill -1e38, ties -> later edge; fill entries -> 0;
 *         argmax[i, f] = eid of the winning edge, -1 where the output was fill
 *   then  y = acc (+ bias[f]) ; if relu: y = y < 0 ? 0 : y
 * w may be NULL (unweighted).  H rows have stride ldh floats, Y rows ldy.
 * argmax: int32 [n_rows, F] (stride F) for MAX, ignored otherwise; and/or
 * win_mask (see mgcn_max_mask): MAX also writes every edge's winner bits at
 * its slot (argmax may then be NULL).
 * relu_mask (nullable; needs relu and F <= 128): uint32 [n_rows][4], bit b
 * of word v set iff y[i, 4 b + v] > 0 -- the ReLU mask mgcn_gemm_nn's dX
 * epilogue reads (16 B per row instead of the 4F-byte Z row).
 * No floating-point contraction: products and sums are rounded separately,
 * in edge order, exactly as the reference's mul + scatter_add sequence.
 */
int mgcn_spmm_fwd(int64_t n_rows, int32_t F, const int64_t *rowptr,
                  const int32_t *col, const int32_t *eid, const float *w,
                  const float *H, int64_t ldh, float *Y, int64_t ldy,
                  int reduce, const float *bias, int relu, int32_t *argmax,
                  uint32_t *win_mask, uint32_t *relu_mask, const int32_t *order,
                  int64_t n_heavy, int64_t n_giant, void *stream);

/* The ReLU mask of rows Z (layout as mgcn_spmm_fwd's relu_mask; F <= 128),
 * for callers whose Z was not produced by mgcn_spmm_fwd. */
int mgcn_relu_mask(int64_t n_rows, int32_t F, const float *Z, int64_t ldz,
                   uint32_t *relu_mask, void *stream);

/*
 * Adjoint aggregation over the transposed (src-grouped) CSR:
 *   dH_s = sum_{k in row s, in edge order} ( g_k * w_k ) [* row_scale_s]
 *   g_k  = dY[col_k, :]                         (SUM)
 *        = dY[col_k, :] / cnt[col_k]            (MEAN; cnt = max(in-deg, 1))
 *        = argmax[col_k, f] == eid_k ? dY : 0   (MAX; or bit f of the edge's
 *                       win_mask word, found through slot_map = mgcn_slot_map)
 * row_scale (nullable) is the RW post-scale dinv[src] (gcn_base_models.py:218).
 * If accumulate != 0 the result is added to dH (dH += ...), else stored.
 */
int mgcn_spmm_bwd(int64_t n_rows, int32_t F, const int64_t *rowptr_t,
                  const int32_t *col_t, const int32_t *eid_t, const float *w_t,
                  const float *row_scale, const float *dY, int64_t lddy,
                  float *dH, int64_t lddh, int reduce, const float *cnt,
                  const int32_t *argmax, const uint32_t *win_mask,
                  const int32_t *slot_map, int accumulate,
                  const int32_t *order, int64_t n_heavy, int64_t n_giant, void *stream);

/*
 * Row schedule (degree skew: the botnet graphs reach degree ~6k, config 3).
 * mgcn_row_schedule writes every row id into order[n_rows], by degree,
 * heaviest first (stable: equal degrees keep ascending ids), and returns
 * n_heavy = #rows with degree > heavy_thr and n_giant = #those with degree >
 * the "heavy_giant_thr" option; it synchronises `stream`.  Passed to
 * mgcn_spmm_fwd/bwd as (order, n_heavy, n_giant): each heavy row gets a whole
 * workgroup that gathers a batch of its edges in parallel and folds them per
 * feature in edge order (same bits) -- giant rows a 1024-thread workgroup with
 * the whole LDS of a CU on a side stream, the others a 256-thread one -- and
 * the lane-group kernel takes order[n_heavy, n_rows) longest first, so the
 * rows of one wave have similar degrees.  order = NULL: natural row order,
 * no heavy path (n_heavy, n_giant ignored).
 */
size_t mgcn_row_schedule_workspace_bytes(int64_t n_rows);
int mgcn_row_schedule(int64_t n_rows, const int64_t *rowptr, int64_t heavy_thr, int32_t *order,
                      int64_t *n_heavy_out, int64_t *n_giant_out, void *workspace,
                      size_t workspace_bytes, void *stream);

/*
 * Max aggregation adjoint without the per-edge argmax gather (config 4 max).
 * mgcn_max_mask: from the forward's argmax [n_rows, F], for every fwd row d
 * and edge slot k of it, bit f of win_mask[k * ceil(F/32) + f/32] =
 * (argmax[d, f] == eid[k]) -- the edges each output feature came from (16 B
 * per edge at F = 128); mgcn_spmm_fwd writes the same bits itself when given
 * win_mask.  mgcn_slot_map: slot_map[j] = the fwd slot of the edge in bwd
 * slot j (eid / eid_t of the two views; workspace
 * mgcn_slot_map_workspace_bytes).  mgcn_spmm_bwd(MAX, win_mask, slot_map)
 * then reads one word per edge, issued with the dY gather instead of after a
 * 4F-byte argmax row.  Same routing as argmax (torch_scatter 1.x scatter_max
 * backward), same bits.
 */
size_t mgcn_slot_map_workspace_bytes(int64_t nnz);
int mgcn_slot_map(int64_t nnz, const int32_t *eid, const int32_t *eid_t, int32_t *slot_map,
                  void *workspace, size_t workspace_bytes, void *stream);
int mgcn_max_mask(int64_t n_rows, int32_t F, const int64_t *rowptr, const int32_t *eid,
                  const int32_t *argmax, uint32_t *win_mask, void *stream);

/* ------------------------------------------------------------------ dense */

/* Bytes of scratch mgcn_gemm_tn needs. */
size_t mgcn_gemm_tn_workspace_bytes(int64_t K, int32_t M, int32_t N);

/*
 * C[M, N] = A^T B (accumulate != 0: C += A^T B) for row-major A [K, M] (row
 * stride lda) and B [K, N] (ldb), fp32 on MFMA (gemm_precision), K split over
 * the chip with a deterministic fixed-order reduction of the partials.
 * Replaces autograd's weight gradient of `torch.matmul(x, self.weight_node)`
 * (gcn_base_models.py:201): dW = x^T dH with K = number of nodes.
 */
int mgcn_gemm_tn(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda,
                 const float *B, int64_t ldb, float *C, int64_t ldc, int accumulate,
                 void *workspace, size_t workspace_bytes, void *stream);

/*
 * mgcn_gemm_tn with the product's columns split over two outputs: columns
 * [0, N1) of A^T B go to C1 [M, N1] (row stride ldc1), columns [N1, N) go
 * TRANSPOSED to C2t [N - N1, M] (row stride ldc2t).  Workspace as
 * mgcn_gemm_tn(K, M, N).  Replaces the two weight gradients of a GCNModel
 * layer and its residual Linear (gcn_model.py:94-105: weight_node [F_in,
 * F_out] and the Linear's weight [F_out, F_in]) from ONE pass over x and
 * [dH | dS], each written in its parameter's own layout.
 */
int mgcn_gemm_tn_split(int64_t K, int32_t M, int32_t N, int32_t N1, const float *A, int64_t lda,
                       const float *B, int64_t ldb, float *C1, int64_t ldc1, float *C2t,
                       int64_t ldc2t, int accumulate, void *workspace, size_t workspace_bytes,
                       void *stream);

/*
 * C[M, N] = A[M, K] . B[K, N] for 1 <= K <= 8, N <= 128, B addressed as B[k * sbk +
 * n * sbn] (W or W^T): the products accumulated in k order on fma.  Replaces
 * `torch.matmul` where the contraction is a handful of features (a 1 -> F
 * input layer, gcn_model.py:64-66; the F -> 2 projection's input gradient).
 */
int mgcn_gemm_small_k(int64_t M, int32_t K, int32_t N, const float *A, int64_t lda,
                      const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                      void *stream);

/* 1 if mgcn_gemm_nn handles this (K, N): every K, N >= 1 (ABI v15). */
int mgcn_gemm_nn_supported(int32_t K, int32_t N);
/* 1 if (K, N) takes the tuned tall-skinny kernel (K in {32, 64, 128, 256},
 * any N; A rows must also be 16-byte aligned): else the generic tiled one. */
int mgcn_gemm_nn_fast(int32_t K, int32_t N);
/* 1 if the fused ReLU-mask epilogue (relu_mask != NULL) is available for
 * (K, N): the tuned kernel with N <= 128. */
int mgcn_gemm_nn_epi_supported(int32_t K, int32_t N);
/* Bytes of scratch mgcn_gemm_nn needs for its fused column sums. */
size_t mgcn_gemm_nn_workspace_bytes(int64_t M, int32_t N);

/*
 * C[M, N] = A[M, K] . B[K, N] on MFMA (gemm_precision: bf16x6 or f32); A
 * row-major (lda), B addressed as B[k * sbk + n * sbn] (so W or W^T).
 * K in {32, 64, 128, 256} with 16-byte aligned A rows: the tuned
 * tall-skinny kernel (B^T split once per workgroup into LDS, A streamed;
 * N wider than 128 (64 at K = 256) as XCD-local column groups); any other
 * shape: a generic 64 x 64-tiled kernel.  Replaces `torch.matmul(x,
 * self.weight_node)` (gcn_base_models.py:201), its input gradient
 * dX = dH W^T, and the Linear layers of the module surface.  If relu_mask
 * != NULL (mgcn_spmm_fwd / mgcn_relu_mask layout, the previous layer's
 * output Z > 0) the ReLU backward and bias gradient are fused into the
 * epilogue:
 *   C = Z > 0 ? A.B : 0,  colsum[n] = sum_m C[m, n]  (deterministic)
 * (gcn_model.py:196 + gcn_base_models.py:240-241 adjoints); with row_div
 * (mean aggregation, = max(in-degree, 1)) C is stored divided by it, the
 * column sums stay undivided (mgcn_gemm_nn_epi_supported shapes only).
 */
int mgcn_gemm_nn(int64_t M, int32_t K, int32_t N, const float *A, int64_t lda,
                 const float *B, int64_t sbk, int64_t sbn, float *C, int64_t ldc,
                 const uint32_t *relu_mask, const float *row_div, float *colsum,
                 void *workspace, size_t workspace_bytes, void *stream);

/* 1 if mgcn_gemm_bwd handles (F_in, F_out): 128 x 128 under bf16x6 precision. */
int mgcn_gemm_bwd_supported(int32_t F_in, int32_t F_out);
/* Bytes of scratch mgcn_gemm_bwd needs (split-K partials + column sums). */
size_t mgcn_gemm_bwd_workspace_bytes(int64_t M, int32_t F_in, int32_t F_out);

/*
 * Both dense adjoints of H = X W (gcn_base_models.py:201) from one pass over
 * X [M, F_in] (ldx) and dH [M, F_out] (lddh), W [F_in, F_out] row-major (ldw):
 *   dW  = X^T dH          (accumulate != 0: dW += X^T dH; deterministic split-K)
 *   dX  = dH W^T          (skipped when dX == NULL)
 * With relu_mask (mgcn_spmm_fwd layout; the lower layer's output > 0) the
 * ReLU backward and that layer's bias gradient are fused as in mgcn_gemm_nn:
 *   dX = mask ? dH W^T : 0 (stored / row_div[m] when row_div != NULL),
 *   colsum[n] = sum_m dX[m, n] (undivided).
 * With dX == NULL and colsum != NULL: colsum[n] = sum_m dH[m, n] (F_out
 * entries; the bias gradient when dH is a layer output's gradient).
 * Replaces autograd's two matmul adjoints of `torch.matmul(x, self.weight_node)`
 * plus the threshold_backward/sum of gcn_model.py:196 and
 * gcn_base_models.py:240-241 (mgcn_gemm_tn + mgcn_gemm_nn in one launch).
 */
int mgcn_gemm_bwd(int64_t M, int32_t F_in, int32_t F_out, const float *X, int64_t ldx,
                  const float *dH, int64_t lddh, const float *W, int64_t ldw,
                  float *dW, int64_t lddw, int accumulate, float *dX, int64_t lddx,
                  const uint32_t *relu_mask, const float *row_div, float *colsum,
                  void *workspace, size_t workspace_bytes, void *stream);

/* Bytes of scratch mgcn_gemm_bwd_dw_cs needs (ABI v20). */
size_t mgcn_gemm_bwd_dw_cs_workspace_bytes(int64_t M);

/*
 * mgcn_gemm_bwd's dW-only form at 128 x 128 (ABI v20) that also returns
 *   s_colsum[128] = sum over the M rows of S   (S [M, 128], lds, 16-byte rows)
 * streamed in the same pass: dW (+)= X^T dH, colsum (nullable) = dH's column
 * sums as mgcn_gemm_bwd.  A GCN stack folds its TOP layer's bias gradient
 * (the column sums of the upstream gradient, gcn_base_models.py:240) into the
 * BOTTOM layer's dW = Z^T dY pass this way, instead of a separate pass over
 * the upstream gradient.  Deterministic (fixed-order folds).
 */
int mgcn_gemm_bwd_dw_cs(int64_t M, const float *X, int64_t ldx, const float *dH, int64_t lddh,
                        float *dW, int64_t lddw, int accumulate, float *colsum, const float *S,
                        int64_t lds, float *s_colsum, void *workspace, size_t workspace_bytes,
                        void *stream);

/* ------------------------------------------------- fused layer forward */

/* 1 if mgcn_spmm_xw_fwd / _bwd handle (F_in, F_out, reduce): 128 x 128 or
 * 256 x 256 (ABI v15), sum or mean, under bf16x6 precision.  At 256 the
 * backward is the dX-only form. */
int mgcn_spmm_xw_supported(int32_t F_in, int32_t F_out, int reduce);
/* 1 if mgcn_spmm_xw_bwd's dW-accumulating form and its max adjoint apply
 * (128 x 128 only). */
int mgcn_spmm_xw_bwd_full_supported(int32_t F_in, int32_t F_out);
/* Bytes of scratch mgcn_spmm_xw_fwd needs: 0 at 128, the split W image at 256. */
size_t mgcn_spmm_xw_fwd_workspace_bytes(int32_t F_in, int32_t F_out);

/*
 * One GCN layer forward in one launch, aggregating before transforming:
 *   Y[i] = epi( (reduce_{k in row i} X[col_k] * w_k) . W + bias )
 * over the fwd CSR view (rowptr/col as mgcn_spmm_fwd; w nullable), X
 * [n_cols, F_in] (ldx, 16-byte aligned rows; under 4 GiB at F = 128, any
 * size at F = 256, whose kernel gives every gathered row a 64-bit base), W
 * [F_in, F_out] row-major (ldw),
 * reduce SUM or MEAN (divides the aggregated row by max(in-degree, 1)), epi =
 * optional ReLU, relu_mask (nullable, needs relu) in mgcn_spmm_fwd's layout.
 * Equals mgcn_gemm_nn (X W) followed by mgcn_spmm_fwd up to the association
 * of the sums (A (X W) = (A X) W for a linear aggregator): the reference's
 * `x @ weight_node` then gather / scale / scatter_add
 * (gcn_base_models.py:201, 223-241; PyG GCNConv x @ W then propagate) without
 * materialising X W.  Rows with heavy degree are handled, but slowly (one
 * lane group per row): callers route skewed graphs to the two-launch path.
 * Z (nullable, [n_rows, F_in], ldz, 16-byte aligned rows) receives the
 * aggregated rows before W -- for MEAN before the division -- so the
 * backward can form dW = Z^T dY' (dY' = dY pre-divided by the counts for
 * MEAN) with mgcn_gemm_bwd instead of a second gather over the graph
 * (the adjoint of `x @ weight_node`, gcn_base_models.py:201, reassociated).
 * At F = 256 (fused_wide.hip) W is split once per call into a fragment
 * image in `workspace` (mgcn_spmm_xw_fwd_workspace_bytes; NULL at 128), Y
 * needs 16-byte aligned rows, and relu_mask holds 8 words per row (feature f
 * at word 4 (f >> 7) + (f & 3), bit (f & 127) >> 2).
 */
int mgcn_spmm_xw_fwd(int64_t n_rows, int64_t n_cols, int32_t F_in, int32_t F_out, const int64_t *rowptr,
                     const int32_t *col, const float *w, const float *X, int64_t ldx,
                     const float *W, int64_t ldw, const float *bias, float *Y, int64_t ldy,
                     int reduce, int relu, uint32_t *relu_mask, float *Z, int64_t ldz,
                     void *workspace, size_t workspace_bytes, void *stream);

/* Bytes of scratch mgcn_spmm_xw_bwd needs (split-K partials + column sums;
 * at 256: the split W^T image + column-sum partials). */
size_t mgcn_spmm_xw_bwd_workspace_bytes(int64_t n_rows, int32_t F_in, int32_t F_out);

/*
 * One GCN layer backward in one launch (F_in = F_out = 128; sum / mean
 * aggregation, whose adjoint is a plain sum once dY is pre-divided):
 *   dH  = reduce_{k in row s} dY[col_k] * w_k  [* row_scale[s]]   (bwd view:
 *         rows = source nodes; = mgcn_spmm_bwd's dH, bit for bit)
 *   dW  = X^T dH   (accumulate != 0: dW += ...; deterministic split-K)
 *   dX  = dH W^T   with relu_mask / row_div / colsum as mgcn_gemm_bwd
 *         (skipped when dX == NULL)
 * dH is never written: it goes from the gather into LDS and through both
 * MFMA products.  Replaces mgcn_spmm_bwd + mgcn_gemm_bwd (the adjoints of
 * gcn_base_models.py:201-241: autograd's index_add of the gathered dY and
 * the two matmul adjoints, plus the ReLU / bias gradient of the layer below,
 * gcn_model.py:196).  dY rows [n_cols, 128] (lddy, 16-byte aligned, under
 * 4 GiB), X [n_rows, 128] (ldx, 16-byte aligned), W [128, 128] row-major.
 * Max (win_mask + slot_map, both or neither): the adjoint of
 * mgcn_spmm_fwd(MAX) -- each edge's dY row counts only at the features whose
 * winner it was (its bits in win_mask at its fwd slot slot_map[k], as
 * mgcn_spmm_bwd(MAX, win_mask, slot_map)); dH bit for bit that function's.
 * dX only: X == NULL and dW == NULL (dX required, no win_mask) -- the
 * gather, dX = dH W^T and its epilogue, nothing else; dX bit for bit the
 * full form's.  Pair with mgcn_spmm_xw_fwd's Z and mgcn_gemm_bwd (dW-only).
 * In the dX-only form `accumulate` != 0 ADDS the column sums into colsum
 * (colsum += ...; ABI v17), so the row chunks of one adjoint fold their bias
 * gradient on the device, in chunk order.
 * F = 256: the dX-only form only (dY any size: 64-bit row bases; relu_mask
 * in the 8-word layout of mgcn_spmm_xw_fwd at 256; dX 16-byte aligned rows).
 */
int mgcn_spmm_xw_bwd(int64_t n_rows, int64_t n_cols, int32_t F_in, int32_t F_out,
                     const int64_t *rowptr_t, const int32_t *col_t, const float *w_t,
                     const float *row_scale, const float *dY, int64_t lddy, const float *X,
                     int64_t ldx, const float *W, int64_t ldw, float *dW, int64_t lddw,
                     int accumulate, float *dX, int64_t lddx, const uint32_t *relu_mask,
                     const float *row_div, float *colsum, const uint32_t *win_mask,
                     const int32_t *slot_map, void *workspace, size_t workspace_bytes,
                     void *stream);

/*
 * The top layer's adjoint (ABI v19; F = 128, bf16x6): mgcn_spmm_xw_bwd's
 * dW + dX form (X, dW and dX required; no max) that also returns
 *   dy_colsum[128] = sum over the rows of dY   (the layer's own bias gradient,
 *                    autograd of `+ self.bias`, gcn_base_models.py:240)
 * from the launch that already streams dY -- each workgroup sums the dY rows
 * of its own row chunks beside the gathers -- so the top layer of a stack
 * needs neither a separate pass over dY nor the forward's Z and the dense
 * Z^T dY pass.  Needs n_rows == n_cols (every dY row is a row of the view:
 * a whole, square graph).  Runs the warp-specialised kernel (one workgroup
 * per CU); dX bit for bit mgcn_spmm_xw_bwd's; dW and the column sums folded
 * in a fixed order (deterministic).  Scratch: mgcn_spmm_xw_bwd_workspace_bytes.
 */
int mgcn_spmm_xw_bwd_hcs(int64_t n_rows, int64_t n_cols, const int64_t *rowptr_t,
                         const int32_t *col_t, const float *w_t, const float *row_scale,
                         const float *dY, int64_t lddy, const float *X, int64_t ldx,
                         const float *W, int64_t ldw, float *dW, int64_t lddw, int accumulate,
                         float *dX, int64_t lddx, const uint32_t *relu_mask, const float *row_div,
                         float *colsum, float *dy_colsum, void *workspace, size_t workspace_bytes,
                         void *stream);

/* ---------------------------------------------------- edge weight adjoint */

/*
 * Gradient of the per-edge message weights (the SDDMM of the aggregation's
 * adjoint): over the fwd view (rowptr / col: rows = destinations, col =
 * sources), for every slot k of row d
 *   dw[k] = sum_f dY[d, f] * H[col[k], f]   (MAX: only the features f whose
 *           winner slot k is, bit f of win_mask[k * ceil(F/32) + f/32])
 * in fwd slot order; dY as the SpMM adjoint receives it (mean: divided by the
 * in-degree).  This is what autograd of the reference's
 * `index_select(x, 0, src) * norm.view(-1, 1)` gives the norm
 * (gcn_base_models.py:217-224), from which degnorm_const's edge_weight / deg
 * gradients follow (gcn_base_models.py:102-140; chained by the host).
 * Deterministic; fp32 products, a fixed butterfly sum over features (the
 * reference's CPU sum order differs: equal to fp32 rounding, not bitwise).
 * 1 <= F <= 1024; H rows stride ldh, dY rows lddy.
 */
int mgcn_edge_weight_grad(int64_t n_rows, int32_t F, const int64_t *rowptr, const int32_t *col,
                          const float *H, int64_t ldh, const float *dY, int64_t lddy,
                          const uint32_t *win_mask, float *dw, void *stream);

/* ------------------------------------------------------- pooling support */

/*
 * Batched dense product (ABI v18), DiffPool's dense operators (PyG 1.3
 * DenseSAGEConv adj @ x @ weight and dense_diff_pool's S^T X, S^T A S, S S^T,
 * reference kernel/diff_pool.py:13-14, 68, 76):
 *   C[b][m][n] (+)= sum_k A[b][m][k] B[b][k][n]      (accumulate != 0: +=)
 * every operand addressed through (batch, row, column) element strides, so
 * transposed views need no copies; fp32 products and accumulation on MFMA.
 * batch <= 65535.
 */
int mgcn_gemm_batched(int64_t batch, int32_t M, int32_t N, int32_t K, const float *A, int64_t sab,
                      int64_t sam, int64_t sak, const float *B, int64_t sbb, int64_t sbk,
                      int64_t sbn, float *C, int64_t scb, int64_t scm, int64_t scn,
                      int accumulate, void *stream);

/* Bytes of scratch mgcn_edge_merge_greedy needs. */
size_t mgcn_edge_merge_workspace_bytes(int64_t n_nodes, int64_t n_edges);

/*
 * EdgePooling's edge contraction (PyG 1.3 EdgePooling.__merge_edges__, the
 * pool of reference kernel/edge_pool.py:19,42): walking the edges in `order`
 * (edge ids by descending score), an edge whose endpoints are both unmatched
 * is taken; taken edges become clusters 0..n_chosen-1 in walk order, the
 * unmatched nodes the clusters after them in ascending node order.  Built on
 * the device as the equivalent locally-dominant matching (same result bit for
 * bit).  src / dst: the two rows of edge_index (int64, E each); order: a
 * permutation of 0..E-1.  Outputs (device): cluster[N], chosen[0..n_chosen)
 * (edge ids, walk order; E entries of room), counts = {n_chosen, n_clusters}.
 * N, E < 2^31 - 1.
 */
int mgcn_edge_merge_greedy(int64_t n_nodes, int64_t n_edges, const int64_t *src, const int64_t *dst,
                           const int64_t *order, void *workspace, size_t workspace_bytes,
                           int64_t *cluster, int64_t *chosen, int64_t *counts, void *stream);

/* ----------------------------------------------------------- elementwise */

/* Bytes of scratch mgcn_relu_bwd_colsum needs. */
size_t mgcn_colsum_workspace_bytes(int64_t n_rows, int32_t F);

/*
 * ReLU backward + bias gradient in one pass over [n_rows, F]:
 *   dY = Z > 0 ? dZ : 0   (written only when relu != 0 or row_div != NULL,
 *                          and dY != NULL; divided by row_div[i] when given:
 *                          the mean aggregation's 1/count, applied once per
 *                          row instead of once per edge in the adjoint)
 *   db[f] = sum_i dY[i, f] (undivided; when db != NULL; deterministic)
 * Replaces autograd's threshold_backward + sum for `x + bias` then ReLU
 * (gcn_base_models.py:240-241, gcn_model.py:196).
 */
int mgcn_relu_bwd_colsum(int64_t n_rows, int32_t F, const float *dZ,
                         const float *Z, int relu, const float *row_div, float *dY,
                         float *db, void *workspace, size_t workspace_bytes,
                         void *stream);

/*
 * GCNModel's residual join (gcn_model.py:99-105, residual_hop = 1):
 *   Z = act(Z1 + (R + rbias))      act = ReLU if relu != 0 (layers before the
 * last, :103) else identity (:105); R = the residual Linear's x Wr^T (its
 * bias rbias may be NULL).  Replaces `xo + xr` and `self.non_linear(...)`.
 */
int mgcn_residual_act(int64_t n_rows, int32_t F, const float *Z1, int64_t ldz1,
                      const float *R, int64_t ldr, const float *rbias, int relu,
                      float *Z, int64_t ldz, void *stream);

/* Bytes of scratch mgcn_residual_act_bwd needs for its column sums. */
size_t mgcn_residual_act_bwd_workspace_bytes(int64_t n_rows, int32_t F);

/*
 * Adjoint of the residual join and of the layer's own ReLU in one pass:
 *   dS = relu ? (Z > 0 ? dZ : 0) : dZ          (written when dS != NULL)
 *   dA = relu1 ? (Z1 > 0 ? dS : 0) : dS        (stored / row_div[i] if given)
 *   colsums[0:F] = sum_i dA (undivided), colsums[F:2F] = sum_i dS
 * (deterministic; colsums may be NULL).  dA feeds the adjoint SpMM, dS the
 * residual Linear's gradients, the sums the two bias gradients.
 */
int mgcn_residual_act_bwd(int64_t n_rows, int32_t F, const float *dZ, int64_t lddz,
                          const float *Z, int64_t ldz, int relu, const float *Z1,
                          int64_t ldz1, int relu1, const float *row_div, float *dA,
                          int64_t ldda, float *dS, int64_t ldds, float *colsums,
                          void *workspace, size_t workspace_bytes, void *stream);

/*
 * GCNModel's INPUT layer with its residual Linear when in_channels = 1 (the
 * botnet node feature; GCNLayer(1, F) + residuals[0] + the join,
 * gcn_model.py:89-105 with residual_hop = 1) associated as (A x) W (ABI
 * v17): with a = A x (mgcn_spmm_fwd at F = 1; for MEAN already divided)
 *   Z[i][j] = relu2( relu1(a[i] W[j] + b[j]) + (x[i] Wr[j] + br[j]) )
 * W = weight_node [1][F], Wr = the Linear weight [F][1] (contiguous: F
 * floats each), b / br nullable; Z [n_rows][F] (ldz, 16-byte aligned rows).
 * The reference's A (x W) to fp32 rounding, without an F-wide gather.
 * Supported: F_in = 1, F / 4 a power of two, 4 <= F <= 256.
 */
int mgcn_input_layer_supported(int32_t F_in, int32_t F);
int mgcn_input_layer_fwd(int64_t n_rows, int32_t F, const float *a, const float *x,
                         const float *W, const float *b, const float *Wr, const float *br,
                         int relu1, int relu2, float *Z, int64_t ldz, void *stream);
/* Bytes of scratch mgcn_input_layer_bwd needs (block partials of 4 F sums). */
size_t mgcn_input_layer_bwd_workspace_bytes(int64_t n_rows, int32_t F);
/*
 * Its adjoint in one pass over dZ (and Z when relu2): dS = relu2' dZ, dA =
 * relu1' dS (relu1's decision recomputed bit for bit), and
 *   grads[0:F] = dW = sum_i a[i] dA[i]    grads[F:2F]  = db  = sum_i dA[i]
 *   grads[2F:3F] = dWr = sum_i x[i] dS[i] grads[3F:4F] = dbr = sum_i dS[i]
 * (deterministic fixed-order sums).  da / dxr (nullable, together): da[i] =
 * sum_j dA[i][j] W[j] [/ row_div[i]] -- the input of the 1-wide adjoint
 * SpMM (dx = A^T da + dxr) -- and dxr[i] = sum_j dS[i][j] Wr[j].
 */
int mgcn_input_layer_bwd(int64_t n_rows, int32_t F, const float *dZ, int64_t lddz,
                         const float *Z, int64_t ldz, const float *a, const float *x,
                         const float *W, const float *b, const float *Wr, int relu1, int relu2,
                         const float *row_div, float *da, float *dxr, float *grads,
                         void *workspace, size_t workspace_bytes, void *stream);

/*
 * One GCNModel layer with its residual Linear, F = 32 (the botnet stack of
 * config 3: GCNLayer + residuals[n] + the join, gcn_model.py:89-105 with
 * residual_hop = 1; NodeModelAdditive.forward gcn_base_models.py:199-243):
 *   Z1 = relu1((A X) W + bias),  Z = relu2(Z1 + (X Wr^T + rbias))
 * in one pass over the rows (fwd view: rows = destinations; order / n_heavy /
 * n_giant its row schedule, as mgcn_spmm_fwd).  W is [F][F] (H = X W), Wr
 * the Linear weight [out][in]; bias / rbias may be NULL; reduce SUM or MEAN.
 * masks[2 i] / masks[2 i + 1]: bit c <=> Z1[i][c] > 0 / Z[i][c] > 0
 * (the activations the backward needs).  Z must not alias X.  Replaces the
 * reference's x @ W, gather / scale / scatter_add, + b, ReLU, the residual
 * Linear, `xo + xr` and the join's ReLU.
 */
int mgcn_residual_layer_supported(int32_t F_in, int32_t F_out, int reduce);
int mgcn_residual_layer_fwd(int64_t n_rows, int32_t F, const int64_t *rowptr,
                            const int32_t *col, const int32_t *eid, const float *w,
                            const float *X, int64_t ldx, const float *W, int64_t ldw,
                            const float *bias, const float *Wr, int64_t ldwr,
                            const float *rbias, int reduce, int relu1, int relu2,
                            float *Z, int64_t ldz, uint32_t *masks, const int32_t *order,
                            int64_t n_heavy, int64_t n_giant, void *stream);

/* Bytes of scratch mgcn_residual_layer_bwd needs (dA rows + column sums). */
size_t mgcn_residual_layer_bwd_workspace_bytes(int64_t n_rows, int32_t F);

/*
 * Its adjoint (bwd view: rows = sources; row_scale the 'rw' post-scale,
 * row_div the in-degree divisor for MEAN, both nullable):
 *   dS = relu2' dZ,  dA = relu1' dS [/ row_div]        (from masks)
 *   DH[:, 0:F] = dH = A^T dA,  DH[:, F:2F] = dS         (lddh >= 2F)
 *   dX = dH W^T + dS Wr
 *   colsums[0:F] = sum_i dA (undivided: the bias gradient), [F:2F] = sum_i dS
 * [dW | dWr^T] = X^T DH is then one mgcn_gemm_tn_split.  dH is bit for bit
 * mgcn_spmm_bwd's of dA.
 */
int mgcn_residual_layer_bwd(int64_t n_rows, int32_t F, const int64_t *rowptr_t,
                            const int32_t *col_t, const int32_t *eid_t, const float *w_t,
                            const float *row_scale, const float *row_div, const float *dZ,
                            int64_t lddz, const uint32_t *masks, int relu1, int relu2,
                            const float *W, int64_t ldw, const float *Wr, int64_t ldwr,
                            float *dX, int64_t lddx, float *DH, int64_t lddh, float *colsums,
                            const int32_t *order, int64_t n_heavy, int64_t n_giant,
                            void *workspace, size_t workspace_bytes, void *stream);

/*
 * A stack of n_layers such layers in one call (GCNModel's 32 -> 32 layers):
 * layer l reads X0 (l = 0) or Z[l - 1] and writes Z[l] = Z + l n_rows F and
 * masks + 2 l n_rows; W / bias / Wr / rbias / relu1 / relu2 are host arrays
 * with one entry per layer (device pointers; bias / rbias arrays or entries
 * may be NULL).  The backward runs the layers top-down: dZ the top layer's
 * upstream gradient, dW[l] ([F][F]) and dWr[l] ([F][F], the Linear layout)
 * written per layer, sums + 2 F l = (bias | rbias gradient) of layer l, dX0
 * (nullable) the gradient of X0.  Bitwise the layer-by-layer calls.
 */
int mgcn_residual_stack_fwd(int64_t n_rows, int32_t F, int32_t n_layers, const int64_t *rowptr,
                            const int32_t *col, const int32_t *eid, const float *w,
                            const float *X0, int64_t ldx, const float *const *W,
                            const float *const *bias, const float *const *Wr,
                            const float *const *rbias, int reduce, const int32_t *relu1,
                            const int32_t *relu2, float *Z, uint32_t *masks,
                            const int32_t *order, int64_t n_heavy, int64_t n_giant, void *stream);
size_t mgcn_residual_stack_bwd_workspace_bytes(int64_t n_rows, int32_t F);
int mgcn_residual_stack_bwd(int64_t n_rows, int32_t F, int32_t n_layers, const int64_t *rowptr_t,
                            const int32_t *col_t, const int32_t *eid_t, const float *w_t,
                            const float *row_scale, const float *row_div, const float *dZ,
                            int64_t lddz, const float *X0, int64_t ldx, const float *Z,
                            const uint32_t *masks, const int32_t *relu1, const int32_t *relu2,
                            const float *const *W, const float *const *Wr, float *dX0,
                            float *const *dW, float *const *dWr, float *sums,
                            const int32_t *order, int64_t n_heavy, int64_t n_giant,
                            void *workspace, size_t workspace_bytes, void *stream);

/*
 * Segment mean over contiguous node ranges (PyG global_mean_pool on a
 * collated Batch, kernel/gcn.py:29; GCNModel pred_on='graph',
 * gcn_model.py:112-123):  out[g, :] = sum_{i in [ptr[g], ptr[g+1])} x[i, :]
 *                                     / max(ptr[g+1] - ptr[g], 1)
 * summed in node order.
 */
int mgcn_segment_mean(int64_t n_seg, int32_t F, const int64_t *ptr,
                      const float *x, int64_t ldx, float *out, int64_t ldo,
                      void *stream);

/*
 * Zero-skipping row packing for the sharded path's table exchange
 * (mgcn.dist: the all-gathered tables between layers are ReLU outputs or
 * ReLU-masked gradients, about half +0.0 words; the reference is
 * single-device, so this replaces nothing of it -- it shrinks the exchange of
 * SURVEY.md §8(e)'s destination-range sharding).  A chunk of n rows of F
 * floats (F % 32 == 0, W = F / 32) travels as one int32 buffer (ABI 21)
 *   [hdr: n x W pairs (mask_w, pos_w)][vals: the rows' words that are not +0.0]
 * bit b of mask_w of a row <=> word 32 w + b is not +0.0 (bit-pattern test:
 * -0.0 / NaN travel as values); pos_w = index in vals of the row's first
 * value at or after word 32 w (offs[i] + the popcounts of mask_0 .. w-1).
 * mgcn_pack_rows_count writes the masks (hdr[2 (i W + w)]) and per-row
 * counts; the caller forms offs (exclusive prefix sum of counts);
 * mgcn_pack_rows_values writes vals and the positions (hdr[2 (i W + w) + 1]).
 * mgcn_unpack_rows expands n_seg such segments (segment p at buf + p
 * seg_words) into rows p n + i of T, bit for bit the packed rows; the fused
 * 256-wide layer kernels also gather straight from them
 * (mgcn_spmm_xw_fwd_packed / _bwd_packed).
 */
int mgcn_pack_rows_count(int64_t n, int32_t F, const float *X, int64_t ldx, uint32_t *hdr,
                         int32_t *counts, void *stream);
int mgcn_pack_rows_values(int64_t n, int32_t F, const float *X, int64_t ldx,
                          const int32_t *offs, uint32_t *hdr, uint32_t *vals, void *stream);
int mgcn_unpack_rows(int64_t n_seg, int64_t n, int32_t F, const uint32_t *buf, int64_t seg_words,
                     float *T, int64_t ldt, void *stream);

/*
 * The same packed chunk in ONE pass (ABI 22; F in {32, 64, 128, 256}): hdr
 * (masks and positions), vals and *total (device int64: the number of
 * values) from a single read of the rows -- a workgroup holds its tile of
 * rows in registers and takes its offset from its predecessors' published
 * counts (decoupled look-back), so neither the count pass's read nor the
 * host-side scan of the counts is needed.  Bit for bit the two-pass output.
 * workspace: mgcn_pack_rows_workspace_bytes(n, F) bytes, 16-byte aligned
 * (cleared by the call on `stream`).  A look-back that waits past the spin
 * bound reports MGCN_EDEVICE (see mgcn_check_device).
 */
size_t mgcn_pack_rows_workspace_bytes(int64_t n, int32_t F);
int mgcn_pack_rows(int64_t n, int32_t F, const float *X, int64_t ldx, uint32_t *hdr,
                   uint32_t *vals, int64_t *total, void *workspace, size_t workspace_bytes,
                   void *stream);

/*
 * A packed exchange table gathered in place (ABI 21; the fused 128- and
 * 256-wide layer kernels).  The zero-skipping exchange delivers a table of C row
 * chunks x P ranks as C * P packed segments of `seg_rows` rows each (the
 * layout above, segment s = c P + k at words + seg_base[s]); instead of
 * expanding them into a dense [C P seg_rows, F] table (mgcn_unpack_rows: a
 * write of the whole table and its re-read by the next layer), the gather
 * reads each needed row from its segment: one 8-B header pair per lane, then
 * the lane's nonzero words -- the bytes of the packed row only.  The view's
 * column indices address packed rows as col = (s << row_bits) | i (row i of
 * segment s; mgcn.dist builds these once per shard).  Results are bit for bit
 * those of the dense table (every +0.0 the packing skipped is folded as 0.0).
 * F = 128: the kernels read the whole table through ONE 32-bit range (the two
 * rows a wave gathers at once are addressed per lane), so every seg_base lies
 * in 0 .. n_words and n_words * 4 <= 2 GiB - 16 B (one receive buffer;
 * MGCN_EINVAL otherwise).  F = 256 (a wave per row, its address in SGPRs):
 * segments anywhere in one device's address space.
 */
typedef struct mgcn_packed_table {
  const uint32_t *words;   /* device: base the segment offsets count from */
  int64_t n_words;         /* words readable at `words` (loads past it read 0) */
  int32_t n_seg;           /* C * P segments, 1 .. 64 */
  int32_t seg_rows;        /* rows per segment (the chunk rows) */
  int32_t row_bits;        /* col = (s << row_bits) | i; seg_rows <= 2^row_bits */
  int32_t F;               /* row width (128 or 256) */
  int64_t seg_base[64];    /* word offset of segment s from `words` (host values,
                              passed to the kernels by value; the segments may
                              live in separate allocations of one device) */
} mgcn_packed_table;

/* mgcn_spmm_xw_fwd (F_in = F_out = 128 or 256, sum / mean) gathering X from a
 * packed table: Y = epi((A X) W + b) (+ Z = A X, + ReLU mask words) -- bit for
 * bit mgcn_spmm_xw_fwd on the unpacked table.  Scratch:
 * mgcn_spmm_xw_fwd_workspace_bytes(F, F). */
int mgcn_spmm_xw_fwd_packed(int64_t n_rows, int32_t F_in, int32_t F_out, const int64_t *rowptr,
                            const int32_t *col, const float *w, const mgcn_packed_table *X,
                            const float *W, int64_t ldw, const float *bias, float *Y,
                            int64_t ldy, int reduce, int relu, uint32_t *relu_mask, float *Z,
                            int64_t ldz, void *workspace, size_t workspace_bytes, void *stream);

/* mgcn_spmm_xw_bwd's dX-only form (F = 128 or 256) gathering dY from a packed
 * table: dX = relu'(lower) ((A^T dY [* row_scale]) W^T) [/ row_div], colsum
 * (+)= sum_rows dX -- bit for bit the dense-table call.  Scratch:
 * mgcn_spmm_xw_bwd_workspace_bytes(n_rows, F, F). */
int mgcn_spmm_xw_bwd_packed(int64_t n_rows, int32_t F_in, int32_t F_out, const int64_t *rowptr_t,
                            const int32_t *col_t, const float *w_t, const float *row_scale,
                            const mgcn_packed_table *dY, const float *W, int64_t ldw, float *dX,
                            int64_t lddx, const uint32_t *relu_mask, const float *row_div,
                            float *colsum, int accumulate, void *workspace,
                            size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MGCN_H */
