// f1 — recommendation top-k over a block of score rows.
//
// Replaces the per-user Python loop of reference src/metrics.py:52-77
// (`get_recs`: score every item, np.argsort(-ratings), drop already-bought
// items, keep the first k).  Scores come from gnnrec_gemm_f32 (a
// [users x d] . [d x items] fp32 MFMA product of L2-normalised embeddings) or
// the edge-MLP head; this kernel selects, per row, the k best columns that are
// not in the row's exclusion list, ordered by (score desc, column asc).
//
// One 256-thread block per row: every thread keeps a sorted top-K of its
// strided columns in registers (insertions are rare after the first few
// hundred columns), then k rounds of a block-wide argmax over the 256 list
// heads emit the result.  k > 64 (the reference's --k has no bound,
// main_inference.py:198) runs in passes of up to 64 columns: pass p keeps only
// candidates ordered after the last result of pass p-1 (the row's "floor").  The exclusion list (already-bought items, a CSR over
// rows) is staged in LDS, sorted, and binary-searched only for candidates that
// would enter a thread's list.
#include "common.hpp"
#include <cmath>

namespace gnnrec {
namespace {

constexpr int kTopkThreads = 256;
constexpr int kMaxExcl = 2048;  // excluded ids staged in LDS per row (larger lists: global search)

__device__ __forceinline__ bool better(float a, int64_t ia, float b, int64_t ib) {
  return a > b || (a == b && ia < ib);
}

template <int KMAX>
__global__ __launch_bounds__(kTopkThreads) void topk_rows_kernel(
    const float* __restrict__ S, int64_t ld, int64_t n_rows, int64_t n_cols, int k,
    const int64_t* __restrict__ ex_ptr, const int64_t* __restrict__ ex_idx,
    float* __restrict__ out_v, int64_t* __restrict__ out_i, int64_t ldo, int col0, bool vec) {
  __shared__ int64_t excl[kMaxExcl];
  __shared__ float red_v[kTopkThreads / 64];
  __shared__ int64_t red_i[kTopkThreads / 64];
  __shared__ int red_t[kTopkThreads / 64];
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  if (row >= n_rows) return;
  const float* srow = S + row * ld;
  out_v += row * ldo + col0;
  out_i += row * ldo + col0;
  // floor: the previous pass's last result; candidates must come after it
  float fl_v = INFINITY;
  int64_t fl_i = -1;
  if (col0 > 0) {
    fl_v = out_v[-1];
    fl_i = out_i[-1];
    if (fl_i < 0) {  // the previous pass ran out of columns: so does this one
      for (int r = tid; r < k; r += kTopkThreads) { out_v[r] = -INFINITY; out_i[r] = -1; }
      return;
    }
  }

  // stage and sort (odd-even transposition over LDS) the exclusion list
  int64_t n_ex = 0, ex0 = 0;
  if (ex_ptr) {
    ex0 = ex_ptr[row];
    n_ex = ex_ptr[row + 1] - ex0;
  }
  const int n_lds = (int)(n_ex < kMaxExcl ? n_ex : kMaxExcl);
  for (int i = tid; i < n_lds; i += kTopkThreads) excl[i] = ex_idx[ex0 + i];
  __syncthreads();
  for (int phase = 0; phase < n_lds; ++phase) {
    for (int i = 2 * tid + (phase & 1); i + 1 < n_lds; i += 2 * kTopkThreads) {
      const int64_t a = excl[i], b = excl[i + 1];
      if (a > b) { excl[i] = b; excl[i + 1] = a; }
    }
    __syncthreads();
  }
  auto excluded = [&](int64_t c) -> bool {
    int lo = 0, hi = n_lds;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (excl[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    if (lo < n_lds && excl[lo] == c) return true;
    for (int64_t j = kMaxExcl; j < n_ex; ++j)  // overflow (rare): linear scan in global
      if (ex_idx[ex0 + j] == c) return true;
    return false;
  };

  // per-thread sorted top-K (descending)
  float tv[KMAX];
  int64_t ti[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) { tv[j] = -INFINITY; ti[j] = INT64_MAX; }
  float thr_v = -INFINITY;  // current k-th best of this thread (kept out of the
  int64_t thr_i = INT64_MAX;  // register array: a runtime index would spill it to scratch)
  auto offer = [&](float v, int64_t c) {
    if (!better(v, c, thr_v, thr_i)) return;
    if (col0 > 0 && !better(fl_v, fl_i, v, c)) return;
    if (n_ex && excluded(c)) return;
    // insert (unrolled bubble from the tail)
    float cv = v;
    int64_t ci = c;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      if (j < k && better(cv, ci, tv[j], ti[j])) {
        const float t1 = tv[j]; const int64_t t2 = ti[j];
        tv[j] = cv; ti[j] = ci;
        cv = t1; ci = t2;
      }
    }
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
      if (j == k - 1) { thr_v = tv[j]; thr_i = ti[j]; }
  };
  // streaming scan: 16-B loads, kUnroll of them in flight per thread before the
  // (almost always rejecting) threshold tests; scalar loop for the tail / unaligned rows
  int64_t c_tail = 0;
  if (vec) {
    constexpr int kUnroll = 4;
    constexpr int64_t kStep = (int64_t)kTopkThreads * 4;
    const int64_t n4 = n_cols & ~int64_t(3);
    int64_t c0 = (int64_t)tid * 4;
    for (; c0 + (kUnroll - 1) * kStep < n4; c0 += kUnroll * kStep) {
      float4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        v[u] = *reinterpret_cast<const float4*>(srow + c0 + u * kStep);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t c = c0 + u * kStep;
        offer(v[u].x, c);
        offer(v[u].y, c + 1);
        offer(v[u].z, c + 2);
        offer(v[u].w, c + 3);
      }
    }
    for (; c0 < n4; c0 += kStep) {
      const float4 v = *reinterpret_cast<const float4*>(srow + c0);
      offer(v.x, c0);
      offer(v.y, c0 + 1);
      offer(v.z, c0 + 2);
      offer(v.w, c0 + 3);
    }
    c_tail = n4;
  }
  for (int64_t c = c_tail + tid; c < n_cols; c += kTopkThreads) offer(srow[c], c);

  // k rounds of block argmax over the list heads
  int head = 0;
  const int lane = tid & 63, wave = tid >> 6;
  for (int r = 0; r < k; ++r) {
    float hv = -INFINITY;
    int64_t hi = INT64_MAX;
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
      if (j == head) { hv = tv[j]; hi = ti[j]; }
    float bv = hv;
    int64_t bi = hi;
    int bt = tid;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(bv, off);
      const int64_t oi = __shfl_xor(bi, off);
      const int ot = __shfl_xor(bt, off);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; bt = ot; }
    }
    if (lane == 0) { red_v[wave] = bv; red_i[wave] = bi; red_t[wave] = bt; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < kTopkThreads / 64; ++w)
        if (better(red_v[w], red_i[w], bv, bi)) { bv = red_v[w]; bi = red_i[w]; bt = red_t[w]; }
      out_v[r] = bv;
      out_i[r] = (bi == INT64_MAX) ? -1 : bi;
      red_t[0] = bt;
    }
    __syncthreads();
    if (tid == red_t[0]) ++head;
    __syncthreads();
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_topk_rows_f32(const float* scores, int64_t ld, int64_t n_rows, int64_t n_cols,
                                    int64_t k, const int64_t* exclude_indptr,
                                    const int64_t* exclude_indices, float* out_vals,
                                    int64_t* out_idx, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_rows >= 0 && n_cols >= 0, "gnnrec_topk_rows_f32: negative size");
  GNNREC_REQUIRE(k >= 1 && k <= (int64_t)1 << 20,
                 "gnnrec_topk_rows_f32: k must be in [1, 2^20] (got %lld)", (long long)k);
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(scores && out_vals && out_idx && ld >= n_cols,
                 "gnnrec_topk_rows_f32: bad pointers / ld");
  GNNREC_REQUIRE(!exclude_indptr || exclude_indices,
                 "gnnrec_topk_rows_f32: exclusion indptr without indices");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)n_rows);
  const bool vec = aligned16(scores) && ld % 4 == 0;
  for (int64_t c0 = 0; c0 < k; c0 += 64) {  // passes of <= 64 columns, each after the last
    const int kk = (int)(k - c0 < 64 ? k - c0 : 64);
    if (kk <= 16)
      hipLaunchKernelGGL((topk_rows_kernel<16>), grid, dim3(kTopkThreads), 0, s, scores, ld,
                         n_rows, n_cols, kk, exclude_indptr, exclude_indices, out_vals, out_idx,
                         k, (int)c0, vec);
    else if (kk <= 32)
      hipLaunchKernelGGL((topk_rows_kernel<32>), grid, dim3(kTopkThreads), 0, s, scores, ld,
                         n_rows, n_cols, kk, exclude_indptr, exclude_indices, out_vals, out_idx,
                         k, (int)c0, vec);
    else
      hipLaunchKernelGGL((topk_rows_kernel<64>), grid, dim3(kTopkThreads), 0, s, scores, ld,
                         n_rows, n_cols, kk, exclude_indptr, exclude_indices, out_vals, out_idx,
                         k, (int)c0, vec);
  }
  return check_launch("gnnrec_topk_rows_f32");
}
