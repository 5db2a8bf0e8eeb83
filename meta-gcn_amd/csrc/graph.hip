// Graph preparation for the GCN aggregation engine (gfx950).
//
// One-time, per static graph: COO edge_index -> two CSR views (grouped by
// destination for the forward SpMM, by source for its adjoint), degrees,
// inverse-degree factors and per-slot normalised edge weights.  The reference
// recomputes the equivalent every forward (gcn_base_models.py:65-146 and the
// index_select/scatter of :211-237); here it is built once and cached by the
// host layer (meta-gcn_amd/mgcn/graph.py).
//
// Integer work (sort, bounds, counts) is HBM-bound; nothing here is shaped
// into a GEMM.  Ordering: hipcub's LSD radix sort is stable, so each CSR row
// keeps its edges in COO order -- the order in which the reference's CPU
// scatter_add/index_add_ accumulate (common.py:59).

#include <hipcub/hipcub.hpp>

#include <cstring>
#include <mutex>
#include <string>

#include "mgcn_internal.h"

namespace mgcn {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

void clear_error() { g_last_error.clear(); }

// warp-specialised hand-off spin bound (mgcn_internal.h; settable in experiment builds)
uint32_t g_spin_limit = kSpinLimitDefault;

// Device-side failure word (round 6).  One 64-B line of pinned, coherent,
// portable host memory mapped into every device's address space: a kernel
// that fails after launch (a warp-specialised kernel whose LDS hand-off spin
// ran past its bound) stores its code there with one vector store, and the
// host reads it with a plain load -- no copy, no synchronisation.

namespace {
std::once_flag g_dev_err_once;
volatile unsigned *g_dev_err_host = nullptr;
unsigned *g_dev_err_dev = nullptr;
hipError_t g_dev_err_status = hipSuccess;
}  // namespace

unsigned *device_error_word() {
  std::call_once(g_dev_err_once, [] {
    void *p = nullptr;
    g_dev_err_status = hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent |
                                                 hipHostMallocPortable);
    if (g_dev_err_status != hipSuccess) return;
    std::memset(p, 0, 64);
    void *d = nullptr;
    g_dev_err_status = hipHostGetDevicePointer(&d, p, 0);
    if (g_dev_err_status != hipSuccess) return;
    g_dev_err_host = static_cast<volatile unsigned *>(p);
    g_dev_err_dev = static_cast<unsigned *>(d);
  });
  if (g_dev_err_dev == nullptr)
    set_error("device error word: %s", hipGetErrorString(g_dev_err_status));
  return g_dev_err_dev;
}

const char *device_error_what(unsigned code) {
  switch (code) {
    case kDevErrDws: return "spmm_xw_bwd_ws_kernel (128-wide adjoint)";
    case kDevErrWide: return "spmm_xw_wide_ws_kernel (256-wide layer)";
    case kDevErrPack: return "pack_rows_kernel (single-pass pack)";
    default: return "unknown kernel";
  }
}

int take_device_error() {
  if (g_dev_err_host == nullptr) return MGCN_OK;
  const unsigned code = *g_dev_err_host;
  if (code == 0) return MGCN_OK;
  *g_dev_err_host = 0u;
  set_error("device: %s stopped at a hand-off that exceeded its spin bound; "
            "the outputs of that launch are invalid (code %u)",
            device_error_what(code), code);
  return MGCN_EDEVICE;
}

namespace {

constexpr int kBlock = 256;

// key (int64) -> int32 sort key + iota values; flag out-of-range indices.
__global__ __launch_bounds__(kBlock) void prep_keys_kernel(
    const int64_t *__restrict__ key, const int64_t *__restrict__ other,
    int64_t nnz, int64_t n_key, int64_t n_other, int32_t *__restrict__ key32,
    int32_t *__restrict__ iota, int *__restrict__ bad) {
  int local_bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = key[i];
    const int64_t o = other[i];
    local_bad |= (k < 0 || k >= n_key) ? 1 : 0;
    local_bad |= (o < 0 || o >= n_other) ? 2 : 0;
    key32[i] = static_cast<int32_t>(k);
    iota[i] = static_cast<int32_t>(i);
  }
  // one atomic per wave that saw a bad index
  if (__any(local_bad != 0)) {
    if ((threadIdx.x & 63) == 0) atomicOr(bad, 3);
  }
}

// rowptr[r] = first slot whose sorted key >= r (lower bound), r in [0, n].
__global__ __launch_bounds__(kBlock) void rowptr_kernel(
    const int32_t *__restrict__ sorted_key, int64_t nnz, int64_t n,
    int64_t *__restrict__ rowptr) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= n;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)sorted_key[mid] < r)
        lo = mid + 1;
      else
        hi = mid;
    }
    rowptr[r] = lo;
  }
}

__global__ __launch_bounds__(kBlock) void gather_col_kernel(
    const int64_t *__restrict__ other, const int32_t *__restrict__ eid,
    int64_t nnz, int32_t *__restrict__ col) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz;
       i += (int64_t)gridDim.x * blockDim.x)
    col[i] = static_cast<int32_t>(other[eid[i]]);
}

// deg / dinv.  One thread per node; weighted degrees sum the row's weights
// sequentially in edge order, as the reference's CPU scatter_add does
// (gcn_base_models.py:126).  pow(-0.5) is evaluated as 1/sqrt(x) with both
// operations correctly rounded (ATen's CPU rsqrt path for pow(x, -0.5)):
// sqrtf (__builtin_sqrtf), NOT __fsqrt_rn, which hipcc lowers to the
// approximate __ocml_native_sqrt_f32;
// pow(-1) as 1/x (ATen reciprocal).  Only +inf is replaced by 0 (:135).
__global__ __launch_bounds__(kBlock) void degree_norm_kernel(
    int64_t n, const int64_t *__restrict__ rowptr,
    const int32_t *__restrict__ eid, const float *__restrict__ deg_in,
    const float *__restrict__ ew, int method, float *__restrict__ deg_out,
    float *__restrict__ dinv_out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float d;
    if (deg_in != nullptr) {
      d = deg_in[i];
    } else if (ew != nullptr) {
      d = 0.0f;
      for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) d = __fadd_rn(d, ew[eid[k]]);
    } else {
      d = static_cast<float>(rowptr[i + 1] - rowptr[i]);
    }
    deg_out[i] = d;
    float v;
    if (method == MGCN_NORM_SM)
      v = __fdiv_rn(1.0f, sqrtf(d));
    else if (method == MGCN_NORM_RW)
      v = __fdiv_rn(1.0f, d);
    else
      v = 1.0f;
    if (v == __builtin_inff()) v = 0.0f;
    dinv_out[i] = v;
  }
}

// One thread per CSR slot; the row of a slot is found by binary search on
// rowptr (slot-parallel keeps heavy rows from serialising a thread).
__global__ __launch_bounds__(kBlock) void edge_norm_kernel(
    int64_t n_rows, int64_t nnz, const int64_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ eid,
    int rows_are_dst, const float *__restrict__ dinv,
    const float *__restrict__ ew, int method, float *__restrict__ w_out) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz;
       k += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = n_rows;  // find r with rowptr[r] <= k < rowptr[r+1]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (rowptr[mid] <= k)
        lo = mid;
      else
        hi = mid;
    }
    const int64_t r = lo;
    const int64_t c = col[k];
    const int64_t s = rows_are_dst ? c : r;
    const int64_t d = rows_are_dst ? r : c;
    float w;
    if (method == MGCN_NORM_SM) {
      w = (ew != nullptr) ? __fmul_rn(__fmul_rn(dinv[s], ew[eid[k]]), dinv[d])
                          : __fmul_rn(dinv[s], dinv[d]);
    } else if (method == MGCN_NORM_RW) {
      w = (ew != nullptr) ? __fmul_rn(dinv[s], ew[eid[k]]) : dinv[s];
    } else {
      w = (ew != nullptr) ? ew[eid[k]] : 1.0f;
    }
    w_out[k] = w;
  }
}

struct SortScratch {
  size_t key32, key32_sorted, iota, cub, total;
};

SortScratch sort_scratch(int64_t nnz, int64_t n) {
  SortScratch s{};
  const size_t b4 = align_up(static_cast<size_t>(nnz > 0 ? nnz : 1) * 4, 256);
  size_t cub_bytes = 0;
  int end_bit = 1;
  while ((int64_t(1) << end_bit) < n && end_bit < 31) ++end_bit;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (const int32_t *)nullptr,
                                     (int32_t *)nullptr, (const int32_t *)nullptr,
                                     (int32_t *)nullptr, static_cast<int>(nnz > 0 ? nnz : 1), 0,
                                     end_bit, (hipStream_t)0);
  s.key32 = 0;
  s.key32_sorted = b4;
  s.iota = 2 * b4;
  s.cub = 3 * b4;
  s.total = 3 * b4 + align_up(cub_bytes, 256);
  return s;
}

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" int mgcn_abi_version(void) { return MGCN_ABI_VERSION; }

extern "C" const char *mgcn_last_error(void) { return g_last_error.c_str(); }

extern "C" int mgcn_check_device(void *stream, int sync) {
  clear_error();
  if (sync) MGCN_HIP_TRY(hipStreamSynchronize(as_stream(stream)));
  return take_device_error();
}

extern "C" size_t mgcn_csr_workspace_bytes(int64_t nnz, int64_t n) {
  return sort_scratch(nnz, n).total;
}

extern "C" int mgcn_csr_build(const int64_t *key, const int64_t *other, int64_t nnz,
                              int64_t n_key, int64_t n_other, int64_t *rowptr,
                              int32_t *col, int32_t *eid, void *workspace,
                              size_t workspace_bytes, void *stream_) {
  clear_error();
  hipStream_t stream = as_stream(stream_);
  MGCN_REQUIRE(nnz >= 0 && n_key >= 0 && n_other >= 0, "mgcn_csr_build: negative size");
  MGCN_REQUIRE(nnz < (int64_t(1) << 31) && n_key < (int64_t(1) << 31) && n_other < (int64_t(1) << 31),
               "mgcn_csr_build: nnz and n must be < 2^31 (int32 col/eid)");
  MGCN_REQUIRE(rowptr != nullptr, "mgcn_csr_build: rowptr is null");
  if (nnz == 0) {
    MGCN_HIP_TRY(hipMemsetAsync(rowptr, 0, sizeof(int64_t) * (n_key + 1), stream));
    return MGCN_OK;
  }
  MGCN_REQUIRE(key && other && col && eid, "mgcn_csr_build: null array");
  const SortScratch s = sort_scratch(nnz, n_key);
  if (workspace == nullptr || workspace_bytes < s.total) {
    set_error("mgcn_csr_build: workspace %zu bytes < required %zu", workspace_bytes, s.total);
    return MGCN_EWORKSPACE;
  }
  char *ws = static_cast<char *>(workspace);
  int32_t *key32 = reinterpret_cast<int32_t *>(ws + s.key32);
  int32_t *key32_sorted = reinterpret_cast<int32_t *>(ws + s.key32_sorted);
  int32_t *iota = reinterpret_cast<int32_t *>(ws + s.iota);
  void *cub_tmp = ws + s.cub;
  size_t cub_bytes = s.total - s.cub;

  // the bad-index flag lives in the first word of the (not yet used) cub region
  int *bad = reinterpret_cast<int *>(cub_tmp);
  MGCN_HIP_TRY(hipMemsetAsync(bad, 0, sizeof(int), stream));
  hipLaunchKernelGGL(prep_keys_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0, stream, key, other,
                     nnz, n_key, n_other, key32, iota, bad);
  if (int rc = check_launch("prep_keys_kernel")) return rc;
  int bad_host = 0;
  MGCN_HIP_TRY(hipMemcpyAsync(&bad_host, bad, sizeof(int), hipMemcpyDeviceToHost, stream));
  MGCN_HIP_TRY(hipStreamSynchronize(stream));
  if (bad_host != 0) {
    set_error("mgcn_csr_build: edge index out of range (expected 0 <= index < %lld / %lld)",
              (long long)n_key, (long long)n_other);
    return MGCN_EINDEX;
  }

  int end_bit = 1;
  while ((int64_t(1) << end_bit) < n_key && end_bit < 31) ++end_bit;
  MGCN_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, key32, key32_sorted, iota,
                                                  eid, static_cast<int>(nnz), 0, end_bit,
                                                  stream));
  hipLaunchKernelGGL(rowptr_kernel, dim3(grid_for(n_key + 1, 256)), dim3(256), 0, stream,
                     key32_sorted, nnz, n_key, rowptr);
  if (int rc = check_launch("rowptr_kernel")) return rc;
  hipLaunchKernelGGL(gather_col_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0, stream, other,
                     eid, nnz, col);
  return check_launch("gather_col_kernel");
}

extern "C" int mgcn_degree_norm(int64_t n, const int64_t *rowptr_src, const int32_t *eid_src,
                                const float *deg_in, const float *edge_weight, int method,
                                float *deg_out, float *dinv_out, void *stream) {
  clear_error();
  MGCN_REQUIRE(n >= 0, "mgcn_degree_norm: negative n");
  MGCN_REQUIRE(method == MGCN_NORM_NONE || method == MGCN_NORM_SM || method == MGCN_NORM_RW,
               "mgcn_degree_norm: bad method %d", method);
  MGCN_REQUIRE(deg_out && dinv_out, "mgcn_degree_norm: null output");
  MGCN_REQUIRE(deg_in != nullptr || rowptr_src != nullptr,
               "mgcn_degree_norm: need deg_in or the source-grouped CSR");
  MGCN_REQUIRE(edge_weight == nullptr || deg_in != nullptr || eid_src != nullptr,
               "mgcn_degree_norm: weighted degree needs eid_src");
  if (n == 0) return MGCN_OK;
  hipLaunchKernelGGL(degree_norm_kernel, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream),
                     n, rowptr_src, eid_src, deg_in, edge_weight, method, deg_out, dinv_out);
  return check_launch("degree_norm_kernel");
}

extern "C" int mgcn_edge_norm(int64_t n_rows, int64_t nnz, const int64_t *rowptr,
                              const int32_t *col, const int32_t *eid, int rows_are_dst,
                              const float *dinv, const float *edge_weight, int method,
                              float *w_out, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_rows >= 0 && nnz >= 0 && rowptr, "mgcn_edge_norm: bad arguments");
  if (nnz == 0 || n_rows == 0) return MGCN_OK;
  MGCN_REQUIRE(col && w_out, "mgcn_edge_norm: null array");
  MGCN_REQUIRE(method == MGCN_NORM_NONE || dinv != nullptr, "mgcn_edge_norm: dinv is null");
  MGCN_REQUIRE(edge_weight == nullptr || eid != nullptr, "mgcn_edge_norm: eid is null");
  hipLaunchKernelGGL(edge_norm_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0, as_stream(stream),
                     n_rows, nnz, rowptr, col, eid, rows_are_dst, dinv, edge_weight, method,
                     w_out);
  return check_launch("edge_norm_kernel");
}
