// f2 — source-major transpose of a dst-major CSR block, for the aggregation backward.
//
// The forward gather (a1) walks in-edges per destination row.  Its gradient w.r.t. the
// source rows is the same sum with the roles swapped: grad_X[u] = Σ_{e: src_e = u}
// w_e · g[dst_e].  Scattering that with float atomics is capped by the L2 atomic units
// (≈0.32 T float atomics/s measured, tools/bench_spmm_bwd.py), well below what a gather
// moves; transposing the block once (the library's stable LSD radix sort of the int32
// source ids, csrsort.hip) turns it into the same bandwidth-bound gather as the forward, and the
// stable order (ascending edge id inside each source row) makes the gradient bitwise
// repeatable.  Reference: DGL's backward of update_all(copy_u, mean/sum) used by
// ConvLayer training (src/model.py:161-167, src/train/run.py:136-138).
#include "common.hpp"
#include "csrsort.hpp"

namespace gnnrec {
namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// one wave per dst row: edge id, dst id and the per-edge weight (ew · 1/deg for mean)
__global__ __launch_bounds__(256) void edge_rows_kernel(const int64_t* __restrict__ indptr,
                                                        const float* __restrict__ ew,
                                                        int64_t n_dst, int mean,
                                                        int32_t* __restrict__ eid,
                                                        int32_t* __restrict__ dst_of,
                                                        float* __restrict__ w_e) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); v < n_dst; v += wstride) {
    const int64_t beg = indptr[v], end = indptr[v + 1];
    const float inv = mean && end > beg ? 1.f / (float)(end - beg) : 1.f;
    for (int64_t e = beg + lane; e < end; e += kWave) {
      eid[e] = (int32_t)e;
      dst_of[e] = (int32_t)v;
      if (w_e) w_e[e] = ew ? ew[e] * inv : inv;
    }
  }
}

// unweighted blocks: dst row of every edge, and 1 / deg(dst) per dst row for mean (the
// sort then carries the dst rows themselves, no edge-id permutation)
__global__ __launch_bounds__(256) void edge_dst_kernel(const int64_t* __restrict__ indptr,
                                                       int64_t n_dst, int mean,
                                                       int32_t* __restrict__ dst_of,
                                                       float* __restrict__ inv_deg) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); v < n_dst; v += wstride) {
    const int64_t beg = indptr[v], end = indptr[v + 1];
    if (mean && lane == 0) inv_deg[v] = end > beg ? 1.f / (float)(end - beg) : 1.f;
    for (int64_t e = beg + lane; e < end; e += kWave) dst_of[e] = (int32_t)v;
  }
}

// ew_t[k] = 1 / deg(indices_t[k]) (the table is n_dst floats: L2-resident)
__global__ __launch_bounds__(256) void row_weight_kernel(const int32_t* __restrict__ rows,
                                                         const float* __restrict__ inv_deg,
                                                         int64_t E, float* __restrict__ w) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < E; k += stride)
    w[k] = inv_deg[rows[k]];
}

// indptr_t[u] = first k with keys[k] >= u (lower bound in the sorted keys; one thread per
// source row, so long runs of unused source ids cost nothing extra)
__global__ __launch_bounds__(256) void bounds_kernel(const int32_t* __restrict__ keys,
                                                     int64_t E, int64_t n_src,
                                                     int64_t* __restrict__ indptr_t) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= n_src; u += stride) {
    int64_t lo = 0, hi = E;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)keys[mid] < u) lo = mid + 1;
      else hi = mid;
    }
    indptr_t[u] = lo;
  }
}

__global__ __launch_bounds__(256) void permute_kernel(const int32_t* __restrict__ perm,
                                                      const int32_t* __restrict__ dst_of,
                                                      const float* __restrict__ w_e, int64_t E,
                                                      int32_t* __restrict__ indices_t,
                                                      float* __restrict__ ew_t) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < E; k += stride) {
    const int32_t e = perm[k];
    indices_t[k] = dst_of[e];
    if (ew_t) ew_t[k] = w_e[e];
  }
}

inline unsigned flat_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 256 * 16) b = 256 * 16;
  return (unsigned)(b < 1 ? 1 : b);
}

// stable sort of row keys: perm = edge ids ordered by (key, edge id) — eid_ready's values
// when given, else the identity — and indptr[n_rows+1].  Scratch: [free slot | sorted keys |
// radix scratch].
int sort_rows(const int32_t* keys_in, int64_t E, int64_t n_rows, char* p, size_t bytes,
              int64_t* indptr, int32_t* perm, int32_t* eid_ready, hipStream_t s) {
  const size_t slot = align_up((size_t)E * 4);
  uint32_t* keys = reinterpret_cast<uint32_t*>(p + slot);
  return radix_sort_rows(keys_in, false, eid_ready, E, n_rows, keys, perm, nullptr, indptr,
                         p + 2 * slot, bytes - 2 * slot, s);
}

size_t sort_rows_bytes(int64_t E, int64_t n_rows) {
  return 2 * align_up((size_t)E * 4) + radix_ws_bytes(E, n_rows);
}

}  // namespace
}  // namespace gnnrec

extern "C" size_t gnnrec_csr_transpose_workspace_bytes(int64_t n_edges, int64_t n_src) {
  using namespace gnnrec;
  if (n_edges <= 0) return 0;
  // weighted: eid | dst_of | w_e | sort_rows scratch; unweighted: dst_of | keys | inv_deg
  // | radix temp (taken only when inv_deg fits in three edge slots)
  return 3 * align_up((size_t)n_edges * 4) + sort_rows_bytes(n_edges, n_src);
}

extern "C" int gnnrec_csr_transpose(const int64_t* indptr, const int32_t* indices,
                                    const float* ew, int64_t n_dst, int64_t n_src,
                                    int64_t n_edges, int mean, void* workspace,
                                    size_t workspace_bytes, int64_t* indptr_t,
                                    int32_t* indices_t, float* ew_t, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_dst >= 0 && n_src >= 0 && n_edges >= 0, "gnnrec_csr_transpose: negative size");
  GNNREC_REQUIRE(n_edges < (int64_t(1) << 31) && n_src < (int64_t(1) << 31),
                 "gnnrec_csr_transpose: int32 edge / node ids");
  GNNREC_REQUIRE(indptr && indptr_t, "gnnrec_csr_transpose: null pointer");
  hipStream_t s = as_stream(stream);
  if (n_edges == 0) {
    hipLaunchKernelGGL(bounds_kernel, dim3(flat_grid(n_src + 1)), dim3(256), 0, s,
                       (const int32_t*)nullptr, (int64_t)0, n_src, indptr_t);
    return check_launch("gnnrec_csr_transpose");
  }
  GNNREC_REQUIRE(indices && indices_t && workspace, "gnnrec_csr_transpose: null pointer");
  GNNREC_REQUIRE(!(ew || mean) || ew_t, "gnnrec_csr_transpose: weights need ew_t");
  const size_t need = gnnrec_csr_transpose_workspace_bytes(n_edges, n_src);
  GNNREC_REQUIRE(workspace_bytes >= need, "gnnrec_csr_transpose: workspace %zu < %zu bytes",
                 workspace_bytes, need);
  char* p = static_cast<char*>(workspace);
  const size_t slot = align_up((size_t)n_edges * 4);
  if (!ew && (!mean || align_up((size_t)(n_dst + 1) * 4) <= 3 * slot)) {
    // unweighted: sort (source id, dst row) pairs straight into indices_t; mean weights
    // from a per-dst-row table.  Scratch: dst_of | sorted keys | inv_deg | radix temp
    int32_t* dst_of = reinterpret_cast<int32_t*>(p);
    int32_t* keys = reinterpret_cast<int32_t*>(p + slot);
    float* inv_deg = reinterpret_cast<float*>(p + 2 * slot);
    const size_t deg_bytes = align_up((size_t)(n_dst + 1) * 4);
    void* temp = p + 2 * slot + deg_bytes;
    size_t temp_bytes = need - 2 * slot - deg_bytes;
    hipLaunchKernelGGL(edge_dst_kernel, dim3(flat_grid(n_dst * 16)), dim3(256), 0, s, indptr,
                       n_dst, mean, dst_of, inv_deg);
    const int rc = radix_sort_rows(indices, false, dst_of, n_edges, n_src,
                                   reinterpret_cast<uint32_t*>(keys), indices_t, nullptr,
                                   indptr_t, temp, temp_bytes, s);
    if (rc != GNNREC_OK) return rc;
    if (mean)
      hipLaunchKernelGGL(row_weight_kernel, dim3(flat_grid(n_edges)), dim3(256), 0, s, indices_t,
                         inv_deg, n_edges, ew_t);
    return check_launch("gnnrec_csr_transpose");
  }
  int32_t* eid = reinterpret_cast<int32_t*>(p);
  int32_t* dst_of = reinterpret_cast<int32_t*>(p + slot);
  float* w_e = (ew || mean) ? reinterpret_cast<float*>(p + 2 * slot) : nullptr;
  hipLaunchKernelGGL(edge_rows_kernel, dim3(flat_grid(n_dst * 16)), dim3(256), 0, s, indptr, ew,
                     n_dst, mean, eid, dst_of, w_e);
  // sort_rows' scratch follows the three edge arrays; with eid supplied as the sort's
  // values its first slot is free and holds the permutation
  char* q = p + 3 * slot;
  int32_t* perm = reinterpret_cast<int32_t*>(q);
  const int rc = sort_rows(indices, n_edges, n_src, q, need - 3 * slot, indptr_t, perm, eid, s);
  if (rc != GNNREC_OK) return rc;
  hipLaunchKernelGGL(permute_kernel, dim3(flat_grid(n_edges)), dim3(256), 0, s, perm, dst_of,
                     w_e, n_edges, indices_t, (ew || mean) ? ew_t : nullptr);
  return check_launch("gnnrec_csr_transpose");
}

extern "C" size_t gnnrec_csr_from_keys_workspace_bytes(int64_t n_edges, int64_t n_rows) {
  return n_edges <= 0 ? 0 : gnnrec::sort_rows_bytes(n_edges, n_rows);
}

extern "C" int gnnrec_csr_from_keys(const int32_t* keys, int64_t n_edges, int64_t n_rows,
                                    void* workspace, size_t workspace_bytes, int64_t* indptr,
                                    int32_t* perm, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_edges >= 0 && n_rows >= 0, "gnnrec_csr_from_keys: negative size");
  GNNREC_REQUIRE(n_edges < (int64_t(1) << 31) && n_rows < (int64_t(1) << 31),
                 "gnnrec_csr_from_keys: int32 edge / row ids");
  GNNREC_REQUIRE(indptr, "gnnrec_csr_from_keys: null pointer");
  hipStream_t s = as_stream(stream);
  if (n_edges == 0) {
    hipLaunchKernelGGL(bounds_kernel, dim3(flat_grid(n_rows + 1)), dim3(256), 0, s,
                       (const int32_t*)nullptr, (int64_t)0, n_rows, indptr);
    return check_launch("gnnrec_csr_from_keys");
  }
  GNNREC_REQUIRE(keys && perm && workspace, "gnnrec_csr_from_keys: null pointer");
  const size_t need = gnnrec_csr_from_keys_workspace_bytes(n_edges, n_rows);
  GNNREC_REQUIRE(workspace_bytes >= need, "gnnrec_csr_from_keys: workspace %zu < %zu bytes",
                 workspace_bytes, need);
  int rc = sort_rows(keys, n_edges, n_rows, static_cast<char*>(workspace), need, indptr, perm,
                     nullptr, s);
  if (rc != GNNREC_OK) return rc;
  return check_launch("gnnrec_csr_from_keys");
}
