// EdgePooling's edge contraction on the device (gfx950).
//
// reference kernel/edge_pool.py:4,19,42 pools with PyG 1.3's EdgePooling,
// whose __merge_edges__ walks the edges by descending score and contracts an
// edge when both endpoints are still unmatched (a sequential greedy
// matching), numbering the clusters in the order the edges are taken and the
// nodes left over after them in ascending node order.
//
// With distinct priorities (an edge's position p in the score order) the
// greedy matching is the unique locally-dominant matching: an edge is in it
// iff, once the edges matched before it are removed, no available edge at
// either endpoint comes earlier.  So it is built in rounds, every available
// edge at once: each free node takes the earliest available edge incident to
// it (atomicMin over positions), and an edge that both its endpoints took is
// matched (a self loop needs its one endpoint).  The earliest available edge
// of the whole graph always matches, so every round matches at least one edge
// and the loop ends; a round leaves the same matched set the sequential walk
// reaches, so the result is the sequential one bit for bit.
//
// Then the cluster ids: chosen edges numbered in position order (an exclusive
// scan of the per-position flags), the free nodes after them in node order
// (a scan of the free flags).
//
// One 1024-thread workgroup (rounds are separated by workgroup barriers; the
// pooled graphs are mini-batches of small graphs).  Integer work over E and N,
// latency-bound per round: ~(2E + 2N) x 4 B of workspace traffic per round.
// Rounds: every round matches at least the globally earliest available edge,
// so at most min(E, N) rounds; the worst case is a long monotone priority
// chain (a path whose scores rise along it matches two edges from its ends
// per round: ~N / 4 rounds), the typical TU mini-batch takes a handful.
// Inputs are validated on the device (endpoints in [0, N), order a
// permutation) before any indexed write.

#include "mgcn_internal.h"

namespace mgcn {
namespace {

constexpr int kMgThreads = 1024;
constexpr int kMgWaves = kMgThreads / 64;

// Workspace words shared between the workgroup's waves go through the L2
// (agent-scope relaxed atomics: the atomicMin results are read back without
// trusting a line the CU's L1 may hold from an earlier access); the barriers
// order the phases.
__device__ __forceinline__ int ld(const int32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st(int32_t *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive scan of v over the workgroup; returns the prefix, *total = sum
__device__ int block_exclusive_scan(int v, int *lds_wave, int *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) lds_wave[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int w = lane < kMgWaves ? lds_wave[lane] : 0;
#pragma unroll
    for (int off = 1; off < kMgWaves; off <<= 1) {
      const int y = __shfl_up(w, off, 64);
      if (lane >= off) w += y;
    }
    if (lane < kMgWaves) lds_wave[kMgWaves + lane] = w;  // inclusive wave totals
  }
  __syncthreads();
  const int before = wave == 0 ? 0 : lds_wave[kMgWaves + wave - 1];
  *total = lds_wave[2 * kMgWaves - 1];
  __syncthreads();  // lds_wave is reused by the next call
  return before + x - v;
}

__global__ __launch_bounds__(kMgThreads) void edge_merge_kernel(
    int32_t N, int32_t E, const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
    const int64_t *__restrict__ order, int32_t *__restrict__ rank, int32_t *__restrict__ flag,
    int32_t *__restrict__ best, int32_t *__restrict__ freen, int64_t *__restrict__ cluster,
    int64_t *__restrict__ chosen, int64_t *__restrict__ counts) {
  __shared__ int lds_wave[2 * kMgWaves];
  __shared__ int matched[3];  // round r writes slot r % 3, resets slot (r + 1) % 3
  const int tid = threadIdx.x;
  // malformed input (an endpoint outside [0, N), an order that is not a
  // permutation of [0, E)) ends the kernel before any indexed write:
  // counts = {-1, -1}, the host raises
  int bad = 0;
  for (int e = tid; e < E; e += kMgThreads) {
    const int64_t s = src[e], t = dst[e], o = order[e];
    bad |= (s < 0) | (s >= N) | (t < 0) | (t >= N) | (o < 0) | (o >= E);
    st(&rank[e], -1);
  }
  if (__syncthreads_or(bad)) {
    if (tid == 0) counts[0] = counts[1] = -1;
    return;
  }
  for (int p = tid; p < E; p += kMgThreads) {
    st(&rank[(int32_t)order[p]], p);
    st(&flag[p], 0);
  }
  for (int u = tid; u < N; u += kMgThreads) st(&freen[u], 1);
  if (tid < 3) matched[tid] = 0;
  __syncthreads();
  for (int e = tid; e < E; e += kMgThreads) bad |= ld(&rank[e]) < 0;  // a repeated position
  if (__syncthreads_or(bad)) {
    if (tid == 0) counts[0] = counts[1] = -1;
    return;
  }

  for (int round = 0;; ++round) {
    for (int u = tid; u < N; u += kMgThreads)
      if (ld(&freen[u])) st(&best[u], INT32_MAX);
    if (tid == 0) matched[(round + 1) % 3] = 0;  // last read in round - 2
    __syncthreads();
    for (int e = tid; e < E; e += kMgThreads) {
      const int32_t s = (int32_t)src[e], t = (int32_t)dst[e];
      if (ld(&freen[s]) && ld(&freen[t])) {
        const int r = ld(&rank[e]);
        atomicMin(&best[s], r);
        if (t != s) atomicMin(&best[t], r);
      }
    }
    __syncthreads();
    // best[] is final for this round: an edge matches where both its
    // endpoints chose it; its endpoints leave the free set after a barrier
    int any = 0;
    for (int e = tid; e < E; e += kMgThreads) {
      const int32_t s = (int32_t)src[e], t = (int32_t)dst[e];
      const int r = ld(&rank[e]);
      if (ld(&freen[s]) && ld(&freen[t]) && ld(&best[s]) == r && ld(&best[t]) == r) {
        st(&flag[r], 1);
        any = 1;
      }
    }
    __syncthreads();
    for (int e = tid; e < E; e += kMgThreads)
      if (ld(&flag[ld(&rank[e])])) {
        st(&freen[(int32_t)src[e]], 0);
        st(&freen[(int32_t)dst[e]], 0);
      }
    if (any) matched[round % 3] = 1;  // plain LDS store: every writer writes 1
    __syncthreads();
    if (!matched[round % 3]) break;
  }

  // cluster ids: chosen edges in position order, then free nodes in node order
  int base = 0;
  for (int p0 = 0; p0 < E; p0 += kMgThreads) {
    const int p = p0 + tid;
    const int f = p < E ? ld(&flag[p]) : 0;
    int tot;
    const int id = base + block_exclusive_scan(f, lds_wave, &tot);
    if (f) {
      const int64_t e = order[p];
      chosen[id] = e;
      cluster[src[e]] = id;
      cluster[dst[e]] = id;
    }
    base += tot;
  }
  const int n_chosen = base;
  for (int u0 = 0; u0 < N; u0 += kMgThreads) {
    const int u = u0 + tid;
    const int f = u < N ? ld(&freen[u]) : 0;
    int tot;
    const int id = base + block_exclusive_scan(f, lds_wave, &tot);
    if (f) cluster[u] = id;
    base += tot;
  }
  if (tid == 0) {
    counts[0] = n_chosen;
    counts[1] = base;
  }
}

// ---------------------------------------------------------------------------
// Batched dense product of DiffPool's dense operators (round 5): PyG 1.3's
// DenseSAGEConv (adj @ x, @ weight) and dense_diff_pool (S^T X, S^T A S,
// S S^T) as used by reference kernel/diff_pool.py:13-14, 68, 76 -- small
// per-graph matrices (a padded mini-batch: B x N x N with N the largest
// graph), so one wave per 16 x 16 output tile on v_mfma_f32_16x16x4_f32
// (exact fp32 products, fp32 accumulation), operands read straight from
// global memory through arbitrary (batch, row, column) strides, so
// transposed operands -- the adjoints' A^T dC and dC B^T -- need no copies.
//   C[b][m][n] (+)= sum_k A[b][m][k] B[b][k][n]
__global__ __launch_bounds__(64) void gemm_batched_kernel(
    int32_t M, int32_t N, int32_t K, const float *__restrict__ A, int64_t sab, int64_t sam,
    int64_t sak, const float *__restrict__ B, int64_t sbb, int64_t sbk, int64_t sbn,
    float *__restrict__ C, int64_t scb, int64_t scm, int64_t scn, int accumulate) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.z;
  const int m0 = 16 * (int)blockIdx.y, n0 = 16 * (int)blockIdx.x;
  const int l16 = lane & 15, g4 = lane >> 4;
  const float *a = A + b * sab + (int64_t)(m0 + l16) * sam;
  const float *bb = B + b * sbb + (int64_t)(n0 + l16) * sbn;
  const bool mok = m0 + l16 < M, nok = n0 + l16 < N;
  f32x4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + g4;
    const float av = (mok && k < K) ? a[(int64_t)k * sak] : 0.0f;
    const float bv = (nok && k < K) ? bb[(int64_t)k * sbk] : 0.0f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
  }
  // lane (l16, g4) holds C[m0 + 4 g4 + r][n0 + l16]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + 4 * g4 + r;
    if (m < M && nok) {
      float *c = C + b * scb + (int64_t)m * scm + (int64_t)(n0 + l16) * scn;
      *c = accumulate ? __fadd_rn(*c, acc[r]) : acc[r];
    }
  }
}

}  // namespace
}  // namespace mgcn

using namespace mgcn;

extern "C" size_t mgcn_edge_merge_workspace_bytes(int64_t n_nodes, int64_t n_edges) {
  const int64_t n = n_nodes > 0 ? n_nodes : 0, e = n_edges > 0 ? n_edges : 0;
  return align_up((size_t)(2 * e + 2 * n) * 4 + 4, 256);
}

extern "C" int mgcn_edge_merge_greedy(int64_t n_nodes, int64_t n_edges, const int64_t *src,
                                      const int64_t *dst, const int64_t *order, void *workspace,
                                      size_t workspace_bytes, int64_t *cluster, int64_t *chosen,
                                      int64_t *counts, void *stream) {
  clear_error();
  MGCN_REQUIRE(n_nodes >= 0 && n_edges >= 0 && n_nodes < INT32_MAX && n_edges < INT32_MAX,
               "mgcn_edge_merge_greedy: need 0 <= n_nodes, n_edges < 2^31 - 1");
  MGCN_REQUIRE(counts != nullptr, "mgcn_edge_merge_greedy: null counts");
  MGCN_REQUIRE(n_edges == 0 || (src && dst && order && chosen), "mgcn_edge_merge_greedy: null edges");
  MGCN_REQUIRE(n_nodes == 0 || cluster != nullptr, "mgcn_edge_merge_greedy: null cluster");
  MGCN_REQUIRE(n_edges == 0 || n_nodes > 0, "mgcn_edge_merge_greedy: edges without nodes");
  const size_t need = mgcn_edge_merge_workspace_bytes(n_nodes, n_edges);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("mgcn_edge_merge_greedy: workspace %zu < %zu", workspace_bytes, need);
    return MGCN_EWORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  int32_t *rank = static_cast<int32_t *>(workspace);
  int32_t *flag = rank + n_edges;
  int32_t *best = flag + n_edges;
  int32_t *freen = best + n_nodes;
  hipLaunchKernelGGL(edge_merge_kernel, dim3(1), dim3(kMgThreads), 0, s, (int32_t)n_nodes,
                     (int32_t)n_edges, src, dst, order, rank, flag, best, freen, cluster, chosen,
                     counts);
  return check_launch("edge_merge_kernel");
}

extern "C" int mgcn_gemm_batched(int64_t batch, int32_t M, int32_t N, int32_t K, const float *A,
                                 int64_t sab, int64_t sam, int64_t sak, const float *B,
                                 int64_t sbb, int64_t sbk, int64_t sbn, float *C, int64_t scb,
                                 int64_t scm, int64_t scn, int accumulate, void *stream) {
  clear_error();
  MGCN_REQUIRE(batch >= 0 && M >= 0 && N >= 0 && K >= 0, "mgcn_gemm_batched: negative size");
  MGCN_REQUIRE(batch <= 65535, "mgcn_gemm_batched: batch %lld > 65535", (long long)batch);
  if (batch == 0 || M == 0 || N == 0) return MGCN_OK;
  MGCN_REQUIRE(C != nullptr && (K == 0 || (A != nullptr && B != nullptr)),
               "mgcn_gemm_batched: null array");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)((N + 15) / 16), (unsigned)((M + 15) / 16), (unsigned)batch);
  hipLaunchKernelGGL(gemm_batched_kernel, grid, dim3(64), 0, s, M, N, K, A, sab, sam, sak, B, sbb,
                     sbk, sbn, C, scb, scm, scn, accumulate);
  return check_launch("gemm_batched_kernel");
}
