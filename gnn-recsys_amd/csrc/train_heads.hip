// f2 — the edge-score side of the training step, fused.
//
// max_margin_loss (reference src/model.py:473-533): per etype
//   s[e,k] = relu(((neg[e,k] + delta) - pos[e]) - mask[e,k]) (/ recency[e]),
//   loss   = mean over the concatenation of every etype's s.
// The reference builds it from ~10 torch ops per etype and autograd adds as many for the
// backward; here one launch per etype writes per-block partial sums (fixed grid, fixed
// order: deterministic) and the unscaled gradient of every score in the same pass, and one
// single-block launch folds the partials.
//
// CosinePrediction backward (reference src/model.py:317-327 under loss.backward()): for
// cos_e = <u_s, v_t> / (max(|u_s|,eps) max(|v_t|,eps)),
//   dL/du_s = inv_s (G_s - û_s (û_s · G_s))   (|u_s| > eps;  G_s · inv_s otherwise)
//   G_s     = Σ_{e: src_e = s} g_e inv_t v_t,  û_s = u_s inv_s,  inv = 1 / max(|row|, eps)
// and symmetrically for v.  G is a weighted gSpMM over the pair graph grouped by src (by
// dst for v) — DGL's rule that an SDDMM's backward is an SpMM.  One C call runs both sides:
// inverse norms, a stable key sort (gnnrec_csr_from_keys), a permute that folds the other
// endpoint's inverse norm into the edge weight, the planned (heavy-row split) gather, and a
// row epilogue — so the host issues one call instead of ~60 small tensor ops.
#include "common.hpp"
#include <cmath>

namespace gnnrec {
namespace {

constexpr int kLossBlocksMax = 1024;

inline unsigned flat_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 256 * 16) b = 256 * 16;
  return (unsigned)(b < 1 ? 1 : b);
}

__device__ inline float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// one wave per positive edge e (grid-stride over e with a grid fixed by n_pos), lanes over k
__global__ __launch_bounds__(256) void margin_loss_kernel(
    const float* __restrict__ pos, const float* __restrict__ neg, int64_t n_pos, int64_t K,
    float delta, const float* __restrict__ mask, const void* __restrict__ rec, int rec_i64,
    float* __restrict__ g_pos, float* __restrict__ g_neg, float* __restrict__ partial) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * 4 + w; e < n_pos; e += (int64_t)gridDim.x * 4) {
    const float p = pos[e];
    float r = 1.f;
    if (rec) r = rec_i64 ? (float)reinterpret_cast<const int64_t*>(rec)[e]
                         : reinterpret_cast<const float*>(rec)[e];
    const float inv_r = 1.f / r;
    float gsum = 0.f, row = 0.f;
    for (int64_t k = lane; k < K; k += kWave) {
      const int64_t i = e * K + k;
      float x = neg[i] + delta - p;  // (neg + delta) - pos, the reference's order
      if (mask) x = x - mask[i];
      const bool on = x > 0.f;
      // the reference divides the ReLU output by the recency (not a multiply by 1/r)
      row += on ? (rec ? x / r : x) : 0.f;
      const float gi = on ? inv_r : 0.f;
      g_neg[i] = gi;
      gsum += gi;
    }
    gsum = wave_sum(gsum);
    if (lane == 0) g_pos[e] = -gsum;
    acc += row;
  }
  acc = wave_sum(acc);
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[0] = scale · Σ x[i] in a fixed order (one block)
__global__ __launch_bounds__(256) void sum_scaled_kernel(const float* __restrict__ x, int64_t n,
                                                         float scale, float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
}

// inv[r] = 1 / max(|T[r]|, 1e-12): one wave per row
__global__ __launch_bounds__(256) void row_inv_norm_kernel(const float* __restrict__ T, int64_t ld,
                                                           int64_t n, int64_t d,
                                                           float* __restrict__ inv) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n;
       r += (int64_t)gridDim.x * 4) {
    const float* p = T + r * ld;
    float s = 0.f;
    for (int64_t c = lane; c < d; c += kWave) s += p[c] * p[c];
    s = wave_sum(s);
    if (lane == 0) inv[r] = 1.f / fmaxf(sqrtf(s), 1e-12f);
  }
}

__global__ __launch_bounds__(256) void keys_to_i32_kernel(const int64_t* __restrict__ k64,
                                                          int64_t n, int32_t* __restrict__ k32) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    k32[i] = (int32_t)k64[i];
}

// edges in row-grouped order: other endpoint (int32) and weight g_e · inv_other
__global__ __launch_bounds__(256) void cos_permute_kernel(const int32_t* __restrict__ perm,
                                                          const int64_t* __restrict__ other,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ inv_other,
                                                          int64_t E, int32_t* __restrict__ ix,
                                                          float* __restrict__ w) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < E; k += stride) {
    const int32_t e = perm[k];
    const int64_t o = other[e];
    ix[k] = (int32_t)o;
    w[k] = g[e] * inv_other[o];
  }
}

// gT[r] = inv_r (G[r] - û (û·G[r])) with û = T[r] inv_r when |T[r]| > eps, else G[r] inv_r
__global__ __launch_bounds__(256) void cos_epilogue_kernel(const float* __restrict__ T,
                                                           int64_t ldt, const float* __restrict__ G,
                                                           int64_t n, int64_t d,
                                                           float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n;
       r += (int64_t)gridDim.x * 4) {
    const float* t = T + r * ldt;
    const float* gr = G + r * d;
    float ss = 0.f, dot = 0.f;
    for (int64_t c = lane; c < d; c += kWave) {
      ss += t[c] * t[c];
      dot += t[c] * gr[c];
    }
    ss = wave_sum(ss);
    dot = wave_sum(dot);
    const float nrm = sqrtf(ss);
    const float inv = 1.f / fmaxf(nrm, 1e-12f);
    const bool big = nrm > 1e-12f;
    const float proj = big ? dot * inv * inv : 0.f;  // û·G with û = t·inv, times inv again
    float* o = out + r * d;
    for (int64_t c = lane; c < d; c += kWave) o[c] = inv * (gr[c] - (big ? t[c] * proj : 0.f));
  }
}

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }
constexpr int64_t kCosSplit = 2048;  // edges per chunk of a heavy row (ops.DEFAULT_SPLIT)

struct CosSide {
  int64_t cap_h, cap_c;
};
inline CosSide side_caps(int64_t E, int64_t n_rows) {
  CosSide c;
  c.cap_h = n_rows < E / (kCosSplit + 1) ? n_rows : E / (kCosSplit + 1);
  c.cap_c = E / kCosSplit + c.cap_h;
  return c;
}

// scratch of one side (reused by the other): keys32 | indptr | perm | ix | w | sort | plan | ws | G
size_t side_bytes(int64_t E, int64_t n_rows, int64_t d) {
  const CosSide c = side_caps(E, n_rows);
  size_t b = 0;
  b += align_up((size_t)E * 4);                // keys32
  b += align_up((size_t)(n_rows + 1) * 8);     // indptr
  b += align_up((size_t)E * 4) * 3;            // perm, ix, w
  b += align_up(gnnrec_csr_from_keys_workspace_bytes(E, n_rows));
  if (c.cap_h > 0) {
    b += align_up((size_t)(2 + c.cap_h + c.cap_h + 1 + c.cap_c) * 8);  // plan
    b += align_up((size_t)c.cap_c * d * 4);                            // chunk partials
  }
  b += align_up((size_t)n_rows * d * 4);  // G
  return b;
}

int run_side(const int64_t* keys, const int64_t* other, const float* g, int64_t E,
             const float* T, int64_t ldt, int64_t n_rows, const float* O, int64_t ldo,
             const float* inv_other, int64_t d, float* gT, char* p, hipStream_t s) {
  const CosSide c = side_caps(E, n_rows);
  int32_t* k32 = reinterpret_cast<int32_t*>(p);
  p += align_up((size_t)E * 4);
  int64_t* indptr = reinterpret_cast<int64_t*>(p);
  p += align_up((size_t)(n_rows + 1) * 8);
  int32_t* perm = reinterpret_cast<int32_t*>(p);
  p += align_up((size_t)E * 4);
  int32_t* ix = reinterpret_cast<int32_t*>(p);
  p += align_up((size_t)E * 4);
  float* w = reinterpret_cast<float*>(p);
  p += align_up((size_t)E * 4);
  const size_t sort_bytes = gnnrec_csr_from_keys_workspace_bytes(E, n_rows);
  void* sort_ws = p;
  p += align_up(sort_bytes);
  int64_t* plan = nullptr;
  float* chunk_ws = nullptr;
  if (c.cap_h > 0) {
    plan = reinterpret_cast<int64_t*>(p);
    p += align_up((size_t)(2 + c.cap_h + c.cap_h + 1 + c.cap_c) * 8);
    chunk_ws = reinterpret_cast<float*>(p);
    p += align_up((size_t)c.cap_c * d * 4);
  }
  float* G = reinterpret_cast<float*>(p);

  hipLaunchKernelGGL(keys_to_i32_kernel, dim3(flat_grid(E)), dim3(256), 0, s, keys, E, k32);
  int rc = gnnrec_csr_from_keys(k32, E, n_rows, sort_ws, sort_bytes, indptr, perm, s);
  if (rc != GNNREC_OK) return rc;
  hipLaunchKernelGGL(cos_permute_kernel, dim3(flat_grid(E)), dim3(256), 0, s, perm, other, g,
                     inv_other, E, ix, w);
  if (c.cap_h > 0) {
    rc = gnnrec_spmm_plan_build(indptr, n_rows, kCosSplit, c.cap_h, c.cap_c, plan, s);
    if (rc != GNNREC_OK) return rc;
    rc = gnnrec_spmm_csr_planned_f32(indptr, ix, w, O, ldo, n_rows, d, GNNREC_REDUCE_SUM, 0, G,
                                     d, kCosSplit, plan, c.cap_h, c.cap_c, chunk_ws, s);
  } else {
    rc = gnnrec_spmm_csr_f32(indptr, ix, w, O, ldo, n_rows, d, GNNREC_REDUCE_SUM, 0, G, d, s);
  }
  if (rc != GNNREC_OK) return rc;
  int64_t blocks = (n_rows + 3) / 4;
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (blocks > 0)
    hipLaunchKernelGGL(cos_epilogue_kernel, dim3((unsigned)blocks), dim3(256), 0, s, T, ldt, G,
                       n_rows, d, gT);
  return GNNREC_OK;
}

}  // namespace
}  // namespace gnnrec

extern "C" int64_t gnnrec_margin_loss_blocks(int64_t n_pos) {
  int64_t b = (n_pos + 3) / 4;
  if (b > gnnrec::kLossBlocksMax) b = gnnrec::kLossBlocksMax;
  return b < 1 ? 1 : b;
}

extern "C" int gnnrec_margin_loss_f32(const float* pos, const float* neg, int64_t n_pos,
                                      int64_t K, float delta, const float* mask,
                                      const void* recency, int recency_i64, float* g_pos,
                                      float* g_neg, float* partial, int64_t n_partial,
                                      void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_pos >= 0 && K >= 0, "gnnrec_margin_loss_f32: negative size");
  const int64_t blocks = gnnrec_margin_loss_blocks(n_pos);
  GNNREC_REQUIRE(partial && n_partial >= blocks,
                 "gnnrec_margin_loss_f32: partial needs %lld entries", (long long)blocks);
  GNNREC_REQUIRE(n_pos == 0 || (pos && g_pos && (K == 0 || (neg && g_neg))),
                 "gnnrec_margin_loss_f32: null pointer");
  hipLaunchKernelGGL(margin_loss_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     pos, neg, n_pos, K, delta, mask, recency, recency_i64, g_pos, g_neg, partial);
  return check_launch("gnnrec_margin_loss_f32");
}

extern "C" int gnnrec_sum_scaled_f32(const float* x, int64_t n, float scale, float* out,
                                     void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n >= 0 && out && (n == 0 || x), "gnnrec_sum_scaled_f32: bad arguments");
  hipLaunchKernelGGL(sum_scaled_kernel, dim3(1), dim3(256), 0, as_stream(stream), x, n, scale,
                     out);
  return check_launch("gnnrec_sum_scaled_f32");
}

extern "C" size_t gnnrec_sddmm_cos_backward_workspace_bytes(int64_t n_edges, int64_t n_src,
                                                            int64_t n_dst, int64_t d) {
  using namespace gnnrec;
  if (n_edges <= 0) return 0;
  const size_t a = side_bytes(n_edges, n_src, d), b = side_bytes(n_edges, n_dst, d);
  return align_up((size_t)n_src * 4) + align_up((size_t)n_dst * 4) + (a > b ? a : b);
}

extern "C" int gnnrec_sddmm_cos_backward_f32(const int64_t* src, const int64_t* dst,
                                             int64_t n_edges, const float* Hs, int64_t lds,
                                             int64_t n_src, const float* Hd, int64_t ldd,
                                             int64_t n_dst, int64_t d, const float* grad,
                                             float* gHs, float* gHd, void* workspace,
                                             size_t workspace_bytes, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_edges >= 0 && n_src >= 0 && n_dst >= 0 && d > 0,
                 "gnnrec_sddmm_cos_backward_f32: bad sizes");
  GNNREC_REQUIRE(n_edges < (int64_t(1) << 31) && n_src < (int64_t(1) << 31) &&
                     n_dst < (int64_t(1) << 31),
                 "gnnrec_sddmm_cos_backward_f32: int32 edge / node ids");
  GNNREC_REQUIRE(lds >= d && ldd >= d, "gnnrec_sddmm_cos_backward_f32: leading dimension < d");
  hipStream_t s = as_stream(stream);
  if (n_edges == 0) {
    if (gHs && n_src) (void)hipMemsetAsync(gHs, 0, (size_t)n_src * d * 4, s);
    if (gHd && n_dst) (void)hipMemsetAsync(gHd, 0, (size_t)n_dst * d * 4, s);
    return check_launch("gnnrec_sddmm_cos_backward_f32");
  }
  GNNREC_REQUIRE(src && dst && Hs && Hd && grad && workspace,
                 "gnnrec_sddmm_cos_backward_f32: null pointer");
  const size_t need = gnnrec_sddmm_cos_backward_workspace_bytes(n_edges, n_src, n_dst, d);
  GNNREC_REQUIRE(workspace_bytes >= need,
                 "gnnrec_sddmm_cos_backward_f32: workspace %zu < %zu bytes", workspace_bytes,
                 need);
  char* p = static_cast<char*>(workspace);
  float* inv_s = reinterpret_cast<float*>(p);
  p += align_up((size_t)n_src * 4);
  float* inv_d = reinterpret_cast<float*>(p);
  p += align_up((size_t)n_dst * 4);
  auto norm_grid = [](int64_t n) {
    int64_t b = (n + 3) / 4;
    return (unsigned)(b < 1 ? 1 : (b > 256 * 16 ? 256 * 16 : b));
  };
  // the src side weighs by the dst norms and vice versa
  if (gHs && n_dst)
    hipLaunchKernelGGL(row_inv_norm_kernel, dim3(norm_grid(n_dst)), dim3(256), 0, s, Hd, ldd,
                       n_dst, d, inv_d);
  if (gHd && n_src)
    hipLaunchKernelGGL(row_inv_norm_kernel, dim3(norm_grid(n_src)), dim3(256), 0, s, Hs, lds,
                       n_src, d, inv_s);
  int rc;
  if (gHs) {
    rc = run_side(src, dst, grad, n_edges, Hs, lds, n_src, Hd, ldd, inv_d, d, gHs, p, s);
    if (rc != GNNREC_OK) return rc;
  }
  if (gHd) {
    rc = run_side(dst, src, grad, n_edges, Hd, ldd, n_dst, Hs, lds, inv_s, d, gHd, p, s);
    if (rc != GNNREC_OK) return rc;
  }
  return check_launch("gnnrec_sddmm_cos_backward_f32");
}
