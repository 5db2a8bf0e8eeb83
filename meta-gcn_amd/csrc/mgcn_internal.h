// Internal helpers shared by the libmgcn translation units (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "mgcn.h"

namespace mgcn {

void set_error(const char *fmt, ...);
void clear_error();

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Experiment builds (make exp -> libmgcn_exp.so, -DMGCN_EXPERIMENT=1) accept
// the timing-only switches that change results (wide_dbg, xw_ws_dbg) and a
// settable hand-off spin bound (ws_spin_limit); the product library compiles
// those switches out and rejects their names.
#ifndef MGCN_EXPERIMENT
#define MGCN_EXPERIMENT 0
#endif
constexpr int kDbgMask = MGCN_EXPERIMENT ? ~0 : 0;  // (a.dbg & kDbgMask): constant 0 in the product
constexpr uint32_t kSpinLimitDefault = 1u << 25;    // ~1 s of s_sleep(1) polls per hand-off
extern uint32_t g_spin_limit;                       // kSpinLimitDefault unless an experiment build sets it

// Device-side failure reporting (round 6): the host-mapped error word
// (graph.hip).  A kernel that cannot finish its work correctly stores a code
// there; take_device_error() turns a stored code into MGCN_EDEVICE + the
// message (and clears it).  The launchers of such kernels call it first, so a
// failed launch fails the next call at the latest; mgcn_check_device() reads
// it after a stream sync.
constexpr unsigned kDevErrDws = 1;   // spmm_xw_bwd_ws_kernel: hand-off spin bound exceeded
constexpr unsigned kDevErrWide = 2;  // spmm_xw_wide_ws_kernel: hand-off spin bound exceeded
constexpr unsigned kDevErrPack = 3;  // pack_rows_kernel: look-back spin bound exceeded
unsigned *device_error_word();       // device pointer (nullptr + set_error on failure)
int take_device_error();

// lane 0 of the calling wave stores `code` into the error word (a vector
// store to host-coherent memory at system scope)
__device__ inline void report_device_error(unsigned *err, unsigned code) {
  if (err != nullptr && (threadIdx.x & 63) == 0)
    __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Check the last launch on this thread; record the HIP error string on failure.
inline int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return MGCN_EHIP;
  }
  return MGCN_OK;
}

#define MGCN_HIP_TRY(call)                                                    \
  do {                                                                        \
    hipError_t _e = (call);                                                   \
    if (_e != hipSuccess) {                                                   \
      ::mgcn::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), \
                        __FILE__, __LINE__);                                  \
      return MGCN_EHIP;                                                       \
    }                                                                         \
  } while (0)

#define MGCN_REQUIRE(cond, ...)       \
  do {                                \
    if (!(cond)) {                    \
      ::mgcn::set_error(__VA_ARGS__); \
      return MGCN_EINVAL;             \
    }                                 \
  } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Grid sizing for grid-stride loops over memory-bound work: enough blocks to
// fill 256 CUs several times over, capped (cdna_hip_programming.md G11).
inline unsigned grid_for(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 8192) g = 8192;
  return static_cast<unsigned>(g);
}

// mgcn_set_option("gemm_tn_variant") -> gemm.hip
int gemm_set_tn_variant(int value);
int gemm_set_tn_staged(int value);  // mgcn_set_option("gemm_tn_staged")
int gemm_set_precision(int value);
int gemm_precision_is_x6();  // 1 under bf16x6 (the fused kernels need it)
int xw_set_unroll(int value);  // fused.hip
int xw_set_ws(const char *name, int value);  // fused.hip: "xw_ws" / "xw_ws_unroll"
extern int g_fused_mask;       // residual.hip: the stack's fused lower-layer mask pass
extern int g_rl_cap;           // residual.hip: workgroups per light-row launch (grid-stride beyond)
// deterministic folds of per-workgroup partials (gemm.hip)
// deterministic fold of split partials: C[e] (+)= sum_sp partial[sp * MN + e]
int launch_fold(const float *partial, int64_t splits, int64_t MN, int N, float *C, int64_t ldc,
                int accumulate, hipStream_t s);
int launch_fold_split(const float *partial, int64_t splits, int64_t MN, int N, float *C,
                      int64_t ldc, int N1, float *C2, int64_t ldc2, int accumulate, hipStream_t s);
int launch_split_reduce(const float *partial, int splits, int64_t MN, int N, float *C,
                        int64_t ldc, int accumulate, hipStream_t s);
int launch_colsum_fold(const float *partial, int64_t nparts, int N, float *out, hipStream_t s);
// A fold of split partials (launch_fold_split's job: C[e] = sum_sp
// partial[sp * MN + e], columns [N1, N) of the [MN / N, N] result to C2
// transposed) run by `blocks` extra 256-thread workgroups of a launch that
// has other work; a workgroup b < blocks calls side_fold_block(f, b, red).
struct SideFold {
  const float *partial;
  int64_t parts, MN;
  int N, N1, log_eb, blocks;
  float *C, *C2;
  int64_t ldc, ldc2;
};
SideFold make_side_fold(const float *partial, int64_t parts, int64_t MN, int N, float *C,
                        int64_t ldc, int N1, float *C2, int64_t ldc2);
int launch_side_fold(const SideFold &f, hipStream_t s);  // on its own (nothing to ride in)

// the same fixed order as fold_partials_kernel (strided partial sums of EB
// elements per workgroup, then a tree over the 256 / EB groups); red: 256
// floats of LDS; every thread of the workgroup calls it
__device__ inline void side_fold_block(const SideFold &f, int b, float *red) {
  const int EB = 1 << f.log_eb, T = 256 >> f.log_eb;
  const int el = threadIdx.x & (EB - 1), g = threadIdx.x >> f.log_eb;
  const int64_t e = (int64_t)b * EB + el;
  float acc = 0.0f;
  if (e < f.MN) {
#pragma unroll 4
    for (int64_t sp = g; sp < f.parts; sp += T) acc = __fadd_rn(acc, f.partial[sp * f.MN + e]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = T >> 1; h >= 1; h >>= 1) {
    if (g < h) red[threadIdx.x] = __fadd_rn(red[threadIdx.x], red[threadIdx.x + h * EB]);
    __syncthreads();
  }
  if (g == 0 && e < f.MN) {
    const int64_t row = e / f.N, col = e % f.N;
    float *dst = col < f.N1 ? f.C + row * f.ldc + col : f.C2 + (col - f.N1) * f.ldc2 + row;
    *dst = red[el];
  }
}

// The staged small-C GEMM C = A^T B as a job for other launches (tn_staged.h:
// tn_staged_block over `blocks` workgroups into the split partials at
// `partial`, folded afterwards with make_side_fold(partial, blocks, M N, ...)).
struct TnJob {
  const float *A;
  int64_t lda;
  const float *B;
  int64_t ldb;
  int64_t K, kps;
  float *partial;
  int blocks;
};
bool tn_staged_plan(int64_t K, int32_t M, int32_t N, const float *A, int64_t lda, const float *B,
                    int64_t ldb, void *workspace, size_t workspace_bytes, TnJob *job);

// mgcn_gemm_tn_split (accumulate = 0) with `side` folded by extra workgroups
// of the same launch; where the staged kernel takes the shape and `defer` is
// given, its own split-K fold is left to the caller (*defer, to ride in a
// later launch: launch_side_fold if none does), else folded here
int gemm_tn_split_fold(int64_t K, int32_t M, int32_t N, int32_t N1, const float *A, int64_t lda,
                       const float *B, int64_t ldb, float *C1, int64_t ldc1, float *C2t,
                       int64_t ldc2t, void *workspace, size_t workspace_bytes,
                       const SideFold &side, hipStream_t s, SideFold *defer = nullptr);
// The residual layer's forward transform (residual.hip, F = 32) applied by
// the heavy-row kernels to their rows' aggregates: Z = relu2(relu1(agg W + b)
// + x Wr^T + br) and the rows' two mask words.  W == NULL: plain aggregate.
struct ResEpi {
  const float *W, *Wr, *b, *br;
  int64_t ldw, ldwr;
  const float *X;  // the rows' own inputs
  int64_t ldx;
  uint32_t *masks;
  int relu1, relu2;
};
// heavy rows of a view alone (spmm.hip), for the fused layer kernels of residual.hip
int heavy_rows(int bwd, int64_t n_rows, int32_t F, const int64_t *rowptr, const int32_t *col,
               const int32_t *eid, const float *w, const float *X, int64_t ldx, float *Y,
               int64_t ldy, const float *row_scale, int mean, const int32_t *order,
               int64_t n_heavy, int64_t n_giant, hipStream_t stream, bool *side_used,
               const ResEpi *rs = nullptr);
int heavy_rows_join(hipStream_t stream);
// fused layer kernels at F = 256 (fused_wide.hip)
size_t xw_wide_workspace_bytes(bool bwd);
int xw_wide_fwd(int64_t n_rows, const int64_t *rowptr, const int32_t *col, const float *w,
                const float *X, int64_t ldx, const float *W, int64_t ldw, const float *bias,
                float *Y, int64_t ldy, int mean, int relu, uint32_t *relu_mask, float *Z,
                int64_t ldz, void *workspace, hipStream_t s,
                const mgcn_packed_table *pk = nullptr);
int xw_wide_bwd_dx(int64_t n_rows, const int64_t *rowptr_t, const int32_t *col_t,
                   const float *w_t, const float *row_scale, const float *dY, int64_t lddy,
                   const float *W, int64_t ldw, float *dX, int64_t lddx,
                   const uint32_t *relu_mask, const float *row_div, float *colsum,
                   int accumulate, void *workspace, hipStream_t s,
                   const mgcn_packed_table *pk = nullptr);
int wide_set_option(const char *name, int value);  // "wide_pair" / "wide_unroll" / "wide_ws"

}  // namespace mgcn
