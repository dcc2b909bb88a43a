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
    // a lane's negatives in its own order (k = lane, lane + 64, ...), their loads requested
    // kMlU at a time: one wave per positive leaves few waves per CU, so a load per
    // iteration left the launch latency-bound (18 µs for C2's 1024 x 2500)
    constexpr int kMlU = 8;
    for (int64_t k0 = lane; k0 < K; k0 += kMlU * kWave) {
      float nv[kMlU], mv[kMlU];
#pragma unroll
      for (int u = 0; u < kMlU; ++u) {
        const int64_t k = k0 + (int64_t)u * kWave;
        nv[u] = k < K ? neg[e * K + k] : 0.f;
        mv[u] = mask && k < K ? mask[e * K + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kMlU; ++u) {
        const int64_t k = k0 + (int64_t)u * kWave;
        if (k >= K) break;
        const int64_t i = e * K + k;
        float x = nv[u] + delta - p;  // (neg + delta) - pos, the reference's order
        if (mask) x = x - mv[u];
        const bool on = x > 0.f;
        // the reference divides the ReLU output by the recency (not a multiply by 1/r)
        row += on ? (rec ? x / r : x) : 0.f;
        const float gi = on ? inv_r : 0.f;
        g_neg[i] = gi;
        gsum += gi;
      }
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

// edges in row-grouped order: other endpoint (int32) and weight g_e · inv_other.
// gK > 0: the grouped layout [G positives | G x gK negatives] (run_grouped_src_side), where
// edge e's other endpoint is its group's positive's, other[e < G ? e : (e - G) / gK] — a
// read from the G-entry head of the array (cache-resident) instead of a random one over E
__global__ __launch_bounds__(256) void cos_permute_kernel(const int32_t* __restrict__ perm,
                                                          const int64_t* __restrict__ other,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ inv_other,
                                                          int64_t E, uint32_t gG, uint32_t gK,
                                                          int32_t* __restrict__ ix,
                                                          float* __restrict__ w) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < E; k += stride) {
    const int32_t e = perm[k];
    const uint32_t ue = (uint32_t)e;
    const int64_t o = gK == 0 ? other[e] : other[ue < gG ? ue : (ue - gG) / gK];
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

// gG, gK: the grouped layout's group count and negatives per group (cos_permute_kernel), or 0
int run_side(const int64_t* keys, const int64_t* other, const float* g, int64_t E,
             const float* T, int64_t ldt, int64_t n_rows, const float* O, int64_t ldo,
             const float* inv_other, int64_t d, float* gT, char* p, hipStream_t s,
             int64_t gG = 0, int64_t gK = 0) {
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
                     inv_other, E, (uint32_t)gG, (uint32_t)gK, ix, w);
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

// ---- grouped source side (negative_sampler.Uniform's pair graphs) ----------------------
// Edges [G positives | G x K negatives] with src[G + g K + j] = src[g] (the reference's
// src.repeat_interleave(K), src/sampling.py:163-165): a group's K + 1 edges share their source
// row, so the source side needs no sort of the E edges — only of the G group keys.  A wave
// gathers one 64-edge chunk of one group (weights g_e inv_t, rows Hd[t]) into a partial
// row; a source row then sums its groups' chunks in key-sorted group order and applies the
// normalisation epilogue of cos_epilogue_kernel.  Every sum runs in a fixed order.
constexpr int kCosBwdChunk = 64;

template <int LPR>
__global__ __launch_bounds__(256) void cos_bwd_chunk_kernel(
    const int64_t* __restrict__ dst, const float* __restrict__ grad,
    const float* __restrict__ inv_d, const float* __restrict__ Hd, int64_t ldd, int d,
    int64_t G, int64_t K, int64_t chunks, float* __restrict__ part) {
  constexpr int NPW = kWave / LPR;  // edges per wave-instruction
  constexpr int U = 16;             // edges in flight per lane group
  static_assert(kCosBwdChunk <= kWave, "a chunk's edges fit one wave load");
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR, gl = lane % LPR;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= G * chunks) return;  // wave-uniform
  const int64_t g = task / chunks, c = task - g * chunks;
  const int col = gl * 4;
  const bool cok = col < d;
  const int64_t q0 = c * kCosBwdChunk;
  const int64_t q1 = q0 + kCosBwdChunk < K + 1 ? q0 + kCosBwdChunk : K + 1;
  auto edge_of = [&](int64_t q) { return q == 0 ? g : G + g * K + (q - 1); };
  // the chunk's ids and weights g_e inv_t in one load per lane (lane l: edge q0 + l), so the
  // gathers below wait on one id load, not one per step of U edges
  int my_t = 0;  // (row ids < 2^31)
  float my_w = 0.f;
  if (q0 + lane < q1) {
    const int64_t e = edge_of(q0 + lane);
    my_t = (int)dst[e];
    my_w = grad[e] * inv_d[my_t];
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // lane group grp sums edges q0 + grp, q0 + grp + NPW, ... in increasing order
  for (int qb = 0; qb < kCosBwdChunk && q0 + qb < q1; qb += NPW * U) {
    const int qo = qb + grp;
    float4 v[U];
    float w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int slot = qo + u * NPW;  // this group's edge q0 + slot (uniform per group)
      const int64_t t = bcast_groups<NPW>(my_t, qb + u * NPW, grp);
      w[u] = bcast_groups<NPW>(my_w, qb + u * NPW, grp);
      const bool ok = slot < kCosBwdChunk && q0 + slot < q1;
      v[u] = cok && ok ? *reinterpret_cast<const float4*>(Hd + t * ldd + col)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int slot = qo + u * NPW;
      if (slot < kCosBwdChunk && q0 + slot < q1) {
        acc.x += w[u] * v[u].x;
        acc.y += w[u] * v[u].y;
        acc.z += w[u] * v[u].z;
        acc.w += w[u] * v[u].w;
      }
    }
  }
  // the NPW lane groups' partials, combined by a fixed xor tree
#pragma unroll
  for (int off = LPR; off < kWave; off <<= 1) {
    acc.x += __shfl_xor(acc.x, off);
    acc.y += __shfl_xor(acc.y, off);
    acc.z += __shfl_xor(acc.z, off);
    acc.w += __shfl_xor(acc.w, off);
  }
  if (grp == 0 && cok) *reinterpret_cast<float4*>(part + task * d + col) = acc;
}

// one wave per source row: G_s = its groups' chunk partials in order, then
// gHs[s] = inv (G_s - û (û . G_s)) as cos_epilogue_kernel
__global__ __launch_bounds__(256) void cos_bwd_combine_kernel(
    const int64_t* __restrict__ indptr_g, const int32_t* __restrict__ perm_g,
    const float* __restrict__ part, int64_t chunks, const float* __restrict__ T, int64_t ldt,
    int64_t n, int d, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int col = lane * 4;
  const bool cok = col < d;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n;
       r += (int64_t)gridDim.x * 4) {
    float4 Gv = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = indptr_g[r]; i < indptr_g[r + 1]; ++i) {
      const float* pg = part + (int64_t)perm_g[i] * chunks * d;
      // the group's chunk partials in chunk order, their loads requested 8 at a time (one
      // per step left ~40 dependent loads per group: 65 µs for C2's K = 2500 head)
      constexpr int CU = 8;
      for (int64_t c0 = 0; c0 < chunks; c0 += CU) {
        float4 x[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u)
          x[u] = cok && c0 + u < chunks
                     ? *reinterpret_cast<const float4*>(pg + (c0 + u) * d + col)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          if (cok && c0 + u < chunks) {
            Gv.x += x[u].x;
            Gv.y += x[u].y;
            Gv.z += x[u].z;
            Gv.w += x[u].w;
          }
        }
      }
    }
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cok) t = *reinterpret_cast<const float4*>(T + r * ldt + col);
    float ss = t.x * t.x + t.y * t.y + t.z * t.z + t.w * t.w;
    float dot = t.x * Gv.x + t.y * Gv.y + t.z * Gv.z + t.w * Gv.w;
    ss = wave_sum(ss);
    dot = wave_sum(dot);
    const float nrm = sqrtf(ss);
    const float inv = 1.f / fmaxf(nrm, 1e-12f);
    const bool big = nrm > 1e-12f;
    const float proj = big ? dot * inv * inv : 0.f;
    if (cok) {
      float4 o;
      o.x = inv * (Gv.x - (big ? t.x * proj : 0.f));
      o.y = inv * (Gv.y - (big ? t.y * proj : 0.f));
      o.z = inv * (Gv.z - (big ? t.z * proj : 0.f));
      o.w = inv * (Gv.w - (big ? t.w * proj : 0.f));
      *reinterpret_cast<float4*>(out + r * d + col) = o;
    }
  }
}

inline int64_t cos_bwd_chunks(int64_t K) { return (K + 1 + kCosBwdChunk - 1) / kCosBwdChunk; }

// scratch of the grouped source side: keys32 | indptr_g | perm_g | sort | partials
size_t grouped_side_bytes(int64_t G, int64_t K, int64_t n_src, int64_t d) {
  size_t b = 0;
  b += align_up((size_t)G * 4);
  b += align_up((size_t)(n_src + 1) * 8);
  b += align_up((size_t)G * 4);
  b += align_up(gnnrec_csr_from_keys_workspace_bytes(G, n_src));
  b += align_up((size_t)G * cos_bwd_chunks(K) * d * 4);
  return b;
}

int run_grouped_src_side(const int64_t* src, const int64_t* dst, const float* grad, int64_t G,
                         int64_t K, const float* Hs, int64_t lds, int64_t n_src, const float* Hd,
                         int64_t ldd, const float* inv_d, int64_t d, float* gHs, char* p,
                         hipStream_t s) {
  int32_t* k32 = reinterpret_cast<int32_t*>(p);
  p += align_up((size_t)G * 4);
  int64_t* indptr_g = reinterpret_cast<int64_t*>(p);
  p += align_up((size_t)(n_src + 1) * 8);
  int32_t* perm_g = reinterpret_cast<int32_t*>(p);
  p += align_up((size_t)G * 4);
  const size_t sort_bytes = gnnrec_csr_from_keys_workspace_bytes(G, n_src);
  void* sort_ws = p;
  p += align_up(sort_bytes);
  float* part = reinterpret_cast<float*>(p);
  hipLaunchKernelGGL(keys_to_i32_kernel, dim3(flat_grid(G)), dim3(256), 0, s, src, G, k32);
  int rc = gnnrec_csr_from_keys(k32, G, n_src, sort_ws, sort_bytes, indptr_g, perm_g, s);
  if (rc != GNNREC_OK) return rc;
  const int64_t chunks = cos_bwd_chunks(K), tasks = G * chunks;
  const dim3 grid((unsigned)((tasks + 3) / 4));
  const int lanes = (int)(d / 4);
  if (lanes <= 16)
    hipLaunchKernelGGL(cos_bwd_chunk_kernel<16>, grid, dim3(256), 0, s, dst, grad, inv_d, Hd,
                       ldd, (int)d, G, K, chunks, part);
  else if (lanes <= 32)
    hipLaunchKernelGGL(cos_bwd_chunk_kernel<32>, grid, dim3(256), 0, s, dst, grad, inv_d, Hd,
                       ldd, (int)d, G, K, chunks, part);
  else
    hipLaunchKernelGGL(cos_bwd_chunk_kernel<64>, grid, dim3(256), 0, s, dst, grad, inv_d, Hd,
                       ldd, (int)d, G, K, chunks, part);
  int64_t blocks = (n_src + 3) / 4;
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (blocks > 0)
    hipLaunchKernelGGL(cos_bwd_combine_kernel, dim3((unsigned)blocks), dim3(256), 0, s, indptr_g,
                       perm_g, part, chunks, Hs, lds, n_src, (int)d, gHs);
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

// the grouped layout (include/gnnrec.h): the source side from the group keys alone
extern "C" size_t gnnrec_sddmm_cos_backward_grouped_workspace_bytes(int64_t n_groups, int64_t K,
                                                                    int64_t n_src, int64_t n_dst,
                                                                    int64_t d) {
  using namespace gnnrec;
  const int64_t E = n_groups * (K + 1);
  if (E <= 0) return 0;
  const size_t a = grouped_side_bytes(n_groups, K, n_src, d), b = side_bytes(E, n_dst, d);
  return align_up((size_t)n_src * 4) + align_up((size_t)n_dst * 4) + (a > b ? a : b);
}

extern "C" int gnnrec_sddmm_cos_backward_grouped_f32(const int64_t* src, const int64_t* dst,
                                                     int64_t n_groups, int64_t K, const float* Hs,
                                                     int64_t lds, int64_t n_src, const float* Hd,
                                                     int64_t ldd, int64_t n_dst, int64_t d,
                                                     const float* grad, float* gHs, float* gHd,
                                                     void* workspace, size_t workspace_bytes,
                                                     void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_groups >= 0 && K >= 0 && n_src >= 0 && n_dst >= 0 && d > 0,
                 "gnnrec_sddmm_cos_backward_grouped_f32: bad sizes");
  const int64_t E = n_groups * (K + 1);
  GNNREC_REQUIRE(E < (int64_t(1) << 31) && n_src < (int64_t(1) << 31) &&
                     n_dst < (int64_t(1) << 31),
                 "gnnrec_sddmm_cos_backward_grouped_f32: int32 edge / node ids");
  GNNREC_REQUIRE(lds >= d && ldd >= d,
                 "gnnrec_sddmm_cos_backward_grouped_f32: leading dimension < d");
  GNNREC_REQUIRE(d % 4 == 0 && d <= 256 && lds % 4 == 0 && ldd % 4 == 0 && aligned16(Hs) &&
                     aligned16(Hd) && (!gHs || aligned16(gHs)),
                 "gnnrec_sddmm_cos_backward_grouped_f32: d %% 4 == 0, d <= 256, 16-B rows");
  hipStream_t s = as_stream(stream);
  if (E == 0) {
    if (gHs && n_src) (void)hipMemsetAsync(gHs, 0, (size_t)n_src * d * 4, s);
    if (gHd && n_dst) (void)hipMemsetAsync(gHd, 0, (size_t)n_dst * d * 4, s);
    return check_launch("gnnrec_sddmm_cos_backward_grouped_f32");
  }
  GNNREC_REQUIRE(src && dst && Hs && Hd && grad && workspace,
                 "gnnrec_sddmm_cos_backward_grouped_f32: null pointer");
  const size_t need = gnnrec_sddmm_cos_backward_grouped_workspace_bytes(n_groups, K, n_src,
                                                                        n_dst, d);
  GNNREC_REQUIRE(workspace_bytes >= need,
                 "gnnrec_sddmm_cos_backward_grouped_f32: workspace %zu < %zu bytes",
                 workspace_bytes, need);
  char* p = static_cast<char*>(workspace);
  float* inv_s = reinterpret_cast<float*>(p);
  p += align_up((size_t)n_src * 4);
  float* inv_d = reinterpret_cast<float*>(p);
  p += align_up((size_t)n_dst * 4);
  auto norm_grid = [](int64_t n) {
    int64_t b = (n + 3) / 4;
    return (unsigned)(b < 1 ? 1 : (b > 256 * 16 ? 256 * 16 : b));
  };
  if (gHs && n_dst)
    hipLaunchKernelGGL(row_inv_norm_kernel, dim3(norm_grid(n_dst)), dim3(256), 0, s, Hd, ldd,
                       n_dst, d, inv_d);
  if (gHd && n_src)
    hipLaunchKernelGGL(row_inv_norm_kernel, dim3(norm_grid(n_src)), dim3(256), 0, s, Hs, lds,
                       n_src, d, inv_s);
  int rc;
  if (gHs) {
    rc = run_grouped_src_side(src, dst, grad, n_groups, K, Hs, lds, n_src, Hd, ldd, inv_d, d,
                              gHs, p, s);
    if (rc != GNNREC_OK) return rc;
  }
  if (gHd) {
    // (K == 0: every edge a positive, the per-edge read)
    rc = run_side(dst, src, grad, E, Hd, ldd, n_dst, Hs, lds, inv_s, d, gHd, p, s, n_groups,
                  K);
    if (rc != GNNREC_OK) return rc;
  }
  return check_launch("gnnrec_sddmm_cos_backward_grouped_f32");
}
