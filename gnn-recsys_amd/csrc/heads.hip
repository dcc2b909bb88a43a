// a7/a8 — edge-score heads.
//
// a7 CosinePrediction (reference src/model.py:317-327): per canonical etype
//    F.normalize(h, p=2, dim=-1, eps=1e-12) on both endpoint tables, then
//    DGL apply_edges(fn.u_dot_v).  Fused here into one pass over the edges:
//    each edge reads its two rows once, and the dot product and both squared
//    norms are reduced together (no normalised copy of either table is
//    materialised).  out = dot / (max(|u|,eps) · max(|v|,eps)).
//
// a8 PredictingModule/PredictingLayer (reference src/model.py:290-305,
//    256-271): σ(w3·relu(W2·relu(W1[h_u‖h_v]+b1)+b2)+b3).  W1[h_u‖h_v] is
//    re-associated into P[u] + Q[v] with P = H_src·W1aᵀ + b1, Q = H_dst·W1bᵀ
//    computed once per node by gnnrec_gemm_f32, so the per-edge work is a
//    128-wide gather-add + ReLU feeding a [E×128]·[128×32] MFMA product, then
//    a 32-wide dot and the sigmoid — the [E, 2d] concatenation of the
//    reference is never built.
#include "common.hpp"
#include <cmath>

namespace gnnrec {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- cosine ----
// one lane's 4-column partial of <a, b>, the fma chain written out: the per-edge and the
// grouped kernel must round every score the same way (left to the compiler's contraction,
// the same source expression fused differently in the two kernels: 1-ulp differences)
__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}

template <int LPR, int VEC>
__global__ __launch_bounds__(256) void sddmm_cos_kernel(const int64_t* __restrict__ src,
                                                        const int64_t* __restrict__ dst,
                                                        int64_t n_edges,
                                                        const float* __restrict__ Hs, int64_t lds,
                                                        const float* __restrict__ Hd, int64_t ldd,
                                                        int d, float* __restrict__ out) {
  constexpr int NPW = kWave / LPR;  // edges per wave per step
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR;
  const int gl = lane % LPR;
  const int64_t wstride = (int64_t)gridDim.x * 4 * NPW;
  for (int64_t e0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * NPW; e0 < n_edges;
       e0 += wstride) {
    const int64_t e = e0 + grp;
    const bool eok = e < n_edges;
    float dot = 0.f, su = 0.f, sv = 0.f;
    if (eok) {
      const float* pu = Hs + src[e] * lds;
      const float* pv = Hd + dst[e] * ldd;
      for (int c = gl * VEC; c < d; c += LPR * VEC) {
        if constexpr (VEC == 4) {
          const float4 a = *reinterpret_cast<const float4*>(pu + c);
          const float4 b = *reinterpret_cast<const float4*>(pv + c);
          dot += dot4(a, b);
          su += dot4(a, a);
          sv += dot4(b, b);
        } else {
          const float a = pu[c], b = pv[c];
          dot += a * b;
          su += a * a;
          sv += b * b;
        }
      }
    }
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) {
      dot += __shfl_xor(dot, off);
      su += __shfl_xor(su, off);
      sv += __shfl_xor(sv, off);
    }
    if (eok && gl == 0) {
      const float nu = fmaxf(sqrtf(su), 1e-12f);
      const float nv = fmaxf(sqrtf(sv), 1e-12f);
      out[e] = dot / (nu * nv);
    }
  }
}

template <int LPR, int VEC>
int launch_cos(const int64_t* src, const int64_t* dst, int64_t n, const float* Hs, int64_t lds,
               const float* Hd, int64_t ldd, int d, float* out, hipStream_t s) {
  constexpr int NPW = kWave / LPR;
  int64_t blocks = (n + 4 * NPW - 1) / (4 * NPW);
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((sddmm_cos_kernel<LPR, VEC>), dim3((unsigned)blocks), dim3(256), 0, s, src,
                     dst, n, Hs, lds, Hd, ldd, d, out);
  return check_launch("gnnrec_sddmm_cos_f32");
}

// ------------------------------------------------------- grouped cosine ----
// The training pair graphs of EdgeDataLoader + negative_sampler.Uniform(K) (reference
// src/sampling.py:163-165: neg src = pos src repeated K times, dst uniform): group g is one
// positive edge (u_g, first[g]) and its K negatives (u_g, dst[g K + j]).  A wave takes a
// chunk of one group's negatives and keeps h_u — its fragment in registers, its norm
// reduced once — so every edge reads one gathered row (4d B) and its dst id, not two rows and
// two ids, and the u norm is not recomputed K times.  Each value is formed exactly as
// sddmm_cos_kernel forms it (same lane fragments, same xor tree, same final expression):
// the scores are bitwise those of the per-edge kernel.
constexpr int kCosU = 16;      // edges in flight per lane group
constexpr int kCosChunk = 64;  // negatives per wave (40 waves per group at K = 2500: the
                               // grid ends in a short tail; 256 per wave left a 25 % round)

template <int LPR>
__global__ __launch_bounds__(256) void sddmm_cos_grouped_kernel(
    const int64_t* __restrict__ src_g, int64_t n_groups, const int64_t* __restrict__ first,
    float* __restrict__ out_first, int64_t K, int64_t chunks, const int64_t* __restrict__ dst,
    float* __restrict__ out, const float* __restrict__ Hs, int64_t lds,
    const float* __restrict__ Hd, int64_t ldd, int d) {
  constexpr int NPW = kWave / LPR;   // edges per wave-instruction
  constexpr int STEP = NPW * kCosU;  // edges per step (<= 64: one id per lane)
  static_assert(kCosChunk <= 64 && kCosChunk % STEP == 0, "a chunk's ids fit one wave load");
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR;
  const int gl = lane % LPR;
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= n_groups * chunks) return;  // wave-uniform
  const int64_t g = task / chunks, c = task - g * chunks;
  const int col = gl * 4;
  const bool cok = col < d;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  float su = 0.f;
  if (cok) {
    a = *reinterpret_cast<const float4*>(Hs + src_g[g] * lds + col);
    su += dot4(a, a);
  }
#pragma unroll
  for (int off = 1; off < LPR; off <<= 1) su += __shfl_xor(su, off);
  const float nu = fmaxf(sqrtf(su), 1e-12f);
  auto score = [&](const float4& b, bool ok) {  // -> the cosine on lane gl == 0 of the group
    float dot = 0.f, sv = 0.f;
    if (ok) {
      dot += dot4(a, b);
      sv += dot4(b, b);
    }
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) {
      dot += __shfl_xor(dot, off);
      sv += __shfl_xor(sv, off);
    }
    const float nv = fmaxf(sqrtf(sv), 1e-12f);
    return dot / (nu * nv);
  };
  if (c == 0 && first != nullptr) {  // the group's positive edge
    const int64_t v = first[g];
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cok) b = *reinterpret_cast<const float4*>(Hd + v * ldd + col);
    const float r = score(b, cok);
    if (lane == 0) out_first[g] = r;
  }
  const int64_t e_beg = g * K + c * kCosChunk;
  const int64_t e_end = g * K + min<int64_t>(K, (c + 1) * kCosChunk);
  // the chunk's ids in one coalesced load (lane l: the chunk's l-th edge)
  const int64_t all_ids = e_beg + lane < e_end ? dst[e_beg + lane] : 0;
  for (int64_t e0 = e_beg; e0 < e_end; e0 += STEP) {
    const int64_t id = STEP == kCosChunk ? all_ids : __shfl(all_ids, (int)(e0 - e_beg) + lane);
    float4 b[kCosU];
#pragma unroll
    for (int k = 0; k < kCosU; ++k) {
      const int slot = k * NPW + grp;
      const int64_t v = __shfl(id, slot);
      b[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cok && e0 + slot < e_end) b[k] = *reinterpret_cast<const float4*>(Hd + v * ldd + col);
    }
#pragma unroll
    for (int k = 0; k < kCosU; ++k) {
      const int64_t e = e0 + k * NPW + grp;
      const float r = score(b[k], cok && e < e_end);
      if (gl == 0 && e < e_end) out[e] = r;
    }
  }
}

template <int LPR>
int launch_cos_grouped(const int64_t* src_g, int64_t G, const int64_t* first, float* out_first,
                       int64_t K, const int64_t* dst, float* out, const float* Hs, int64_t lds,
                       const float* Hd, int64_t ldd, int d, hipStream_t s) {
  const int64_t chunks = K > 0 ? (K + kCosChunk - 1) / kCosChunk : 1;
  const int64_t waves = G * chunks;
  hipLaunchKernelGGL(sddmm_cos_grouped_kernel<LPR>, dim3((unsigned)((waves + 3) / 4)), dim3(256),
                     0, s, src_g, G, first, out_first, K, chunks, dst, out, Hs, lds, Hd, ldd, d);
  return check_launch("gnnrec_sddmm_cos_grouped_f32");
}

// ------------------------------------------------------------- edge MLP ----
// One wave scores 32 edges: A[i][k] = relu(P[src_i][k] + Q[dst_i][k]) (k < 128),
// B[k][j] = W2[j][k]; lane half h consumes k in [64h, 64h+64).  Output
// C[i][j] (col j = lane&31) -> relu(+b2) -> dot with w3 across the 32 lanes.
constexpr int kHid1 = 128;

__global__ __launch_bounds__(256) void edge_mlp_kernel(const int64_t* __restrict__ src,
                                                       const int64_t* __restrict__ dst,
                                                       int64_t n_edges,
                                                       const float* __restrict__ P,
                                                       const float* __restrict__ Q,
                                                       const float* __restrict__ W2,
                                                       const float* __restrict__ b2,
                                                       const float* __restrict__ w3,
                                                       const float* __restrict__ b3,
                                                       float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  const float b2r = b2[r];
  const float w3r = w3[r];
  const float b3v = b3[0];
  const int64_t gstride = (int64_t)gridDim.x * 4 * 32;
  for (int64_t e0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32; e0 < n_edges;
       e0 += gstride) {
    const int64_t e = e0 + r;
    const bool eok = e < n_edges;
    const float* pp = P + (eok ? src[e] : 0) * kHid1 + h * 64;
    const float* pq = Q + (eok ? dst[e] : 0) * kHid1 + h * 64;
    const float* pw = W2 + r * kHid1 + h * 64;
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      f32x4 a = *reinterpret_cast<const f32x4*>(pp + c * 4) +
                *reinterpret_cast<const f32x4*>(pq + c * 4);
      const f32x4 b = *reinterpret_cast<const f32x4*>(pw + c * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float av = eok ? fmaxf(a[s], 0.f) : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b[s], acc, 0, 0, 0);
      }
    }
    // acc[v] = hidden2 pre-activation of edge row (v&3)+8(v>>2)+4h, unit r
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      float y = fmaxf(acc[v] + b2r, 0.f) * w3r;
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) y += __shfl_xor(y, off);
      const int64_t er = e0 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (r == 0 && er < n_edges) out[er] = 1.f / (1.f + expf(-(y + b3v)));
    }
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_sddmm_cos_f32(const int64_t* src, const int64_t* dst, int64_t n_edges,
                                    const float* Hs, int64_t lds, const float* Hd, int64_t ldd,
                                    int64_t d, float* out, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_edges >= 0 && d >= 0, "gnnrec_sddmm_cos_f32: negative size");
  if (n_edges == 0) return GNNREC_OK;
  GNNREC_REQUIRE(src && dst && out && Hs && Hd, "gnnrec_sddmm_cos_f32: null pointer");
  GNNREC_REQUIRE(lds >= d && ldd >= d, "gnnrec_sddmm_cos_f32: leading dimension < d");
  hipStream_t s = as_stream(stream);
  const bool vec4 = d % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0 && aligned16(Hs) && aligned16(Hd);
  if (!vec4) return launch_cos<64, 1>(src, dst, n_edges, Hs, lds, Hd, ldd, (int)d, out, s);
  if (d <= 64) return launch_cos<16, 4>(src, dst, n_edges, Hs, lds, Hd, ldd, (int)d, out, s);
  if (d <= 128) return launch_cos<32, 4>(src, dst, n_edges, Hs, lds, Hd, ldd, (int)d, out, s);
  return launch_cos<64, 4>(src, dst, n_edges, Hs, lds, Hd, ldd, (int)d, out, s);
}

extern "C" int gnnrec_sddmm_cos_grouped_f32(const int64_t* src_g, int64_t n_groups,
                                            const int64_t* first, float* out_first, int64_t K,
                                            const int64_t* dst, float* out, const float* Hs,
                                            int64_t lds, const float* Hd, int64_t ldd, int64_t d,
                                            void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_groups >= 0 && K >= 0 && d >= 0, "gnnrec_sddmm_cos_grouped_f32: negative size");
  if (n_groups == 0 || (K == 0 && first == nullptr)) return GNNREC_OK;
  GNNREC_REQUIRE(src_g && Hs && Hd && (K == 0 || (dst && out)) && (!first || out_first),
                 "gnnrec_sddmm_cos_grouped_f32: null pointer");
  GNNREC_REQUIRE(lds >= d && ldd >= d, "gnnrec_sddmm_cos_grouped_f32: leading dimension < d");
  GNNREC_REQUIRE(d % 4 == 0 && d <= 256 && lds % 4 == 0 && ldd % 4 == 0 && aligned16(Hs) &&
                     aligned16(Hd),
                 "gnnrec_sddmm_cos_grouped_f32: needs d %% 4 == 0, d <= 256 and 16-B aligned "
                 "rows (gnnrec_sddmm_cos_f32 takes the rest)");
  // one wave per (group, kCosChunk negatives): the launch's work-items (4 waves per
  // 256-thread block) must stay below 2^32
  GNNREC_REQUIRE((n_groups * (K > 0 ? (K + kCosChunk - 1) / kCosChunk : 1) + 3) / 4 * 256 <
                     (int64_t(1) << 32),
                 "gnnrec_sddmm_cos_grouped_f32: too many groups x negatives for one launch");
  hipStream_t s = as_stream(stream);
  if (d <= 64)
    return launch_cos_grouped<16>(src_g, n_groups, first, out_first, K, dst, out, Hs, lds, Hd, ldd,
                                  (int)d, s);
  if (d <= 128)
    return launch_cos_grouped<32>(src_g, n_groups, first, out_first, K, dst, out, Hs, lds, Hd, ldd,
                                  (int)d, s);
  return launch_cos_grouped<64>(src_g, n_groups, first, out_first, K, dst, out, Hs, lds, Hd, ldd,
                                (int)d, s);
}

extern "C" int gnnrec_edge_mlp_f32(const int64_t* src, const int64_t* dst, int64_t n_edges,
                                   const float* P, const float* Q, const float* W2,
                                   const float* b2, const float* w3, const float* b3, float* out,
                                   void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_edges >= 0, "gnnrec_edge_mlp_f32: negative size");
  if (n_edges == 0) return GNNREC_OK;
  GNNREC_REQUIRE(src && dst && P && Q && W2 && b2 && w3 && b3 && out,
                 "gnnrec_edge_mlp_f32: null pointer");
  GNNREC_REQUIRE(aligned16(P) && aligned16(Q) && aligned16(W2),
                 "gnnrec_edge_mlp_f32: P/Q/W2 must be 16-byte aligned");
  int64_t blocks = (n_edges + 127) / 128;
  if (blocks > 256 * 32) blocks = 256 * 32;
  hipLaunchKernelGGL(edge_mlp_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     src, dst, n_edges, P, Q, W2, b2, w3, b3, out);
  return check_launch("gnnrec_edge_mlp_f32");
}
