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

// Sum over a lane group of LPR (16, 32 or 64) lanes by DPP adds — VALU only, where a
// __shfl_xor tree is one ds_bpermute per level — valid in the group's LAST lane.  Each level
// adds the same two partial sums the xor tree adds (quad_perm [1,0,3,2] / [2,3,0,1] pair the
// xor-1 / xor-2 partners; after them a quad's lanes agree, so row_half_mirror and row_mirror
// add the xor-4 / xor-8 partner's value; row_bcast15 / 31 add the lower row's / half's sum
// to the upper one): the bits of the xor tree, which the u-norm reductions still use.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_add(float x) {
  const int y = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, ROWS, 0xF, false);
  return x + __builtin_bit_cast(float, y);
}

template <int LPR>
__device__ __forceinline__ float group_sum_last(float x) {
  static_assert(LPR == 16 || LPR == 32 || LPR == 64, "lane groups of 16, 32 or 64");
  x = dpp_add<0xB1, 0xF>(x);   // quad_perm [1,0,3,2]
  x = dpp_add<0x4E, 0xF>(x);   // quad_perm [2,3,0,1]
  x = dpp_add<0x141, 0xF>(x);  // row_half_mirror
  x = dpp_add<0x140, 0xF>(x);  // row_mirror
  if constexpr (LPR >= 32) x = dpp_add<0x142, 0xA>(x);  // row_bcast15 into rows 1 and 3
  if constexpr (LPR >= 64) x = dpp_add<0x143, 0xC>(x);  // row_bcast31 into rows 2 and 3
  return x;
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
    dot = group_sum_last<LPR>(dot);
    su = group_sum_last<LPR>(su);
    sv = group_sum_last<LPR>(sv);
    if (eok && gl == LPR - 1) {
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
// sddmm_cos_kernel forms it (same lane fragments, same reduction tree, same final expression):
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
    dot = group_sum_last<LPR>(dot);
    sv = group_sum_last<LPR>(sv);
    const float nv = fmaxf(sqrtf(sv), 1e-12f);
    return dot / (nu * nv);  // (valid in the group's last lane)
  };
  if (c == 0 && first != nullptr) {  // the group's positive edge
    const int64_t v = first[g];
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cok) b = *reinterpret_cast<const float4*>(Hd + v * ldd + col);
    const float r = score(b, cok);
    if (lane == LPR - 1) out_first[g] = r;
  }
  const int64_t e_beg = g * K + c * kCosChunk;
  const int64_t e_end = g * K + min<int64_t>(K, (c + 1) * kCosChunk);
  // the chunk's ids in one coalesced load (lane l: the chunk's l-th edge; row ids < 2^31)
  const int all_ids = e_beg + lane < e_end ? (int)dst[e_beg + lane] : 0;
  for (int64_t e0 = e_beg; e0 < e_end; e0 += STEP) {
    const int id = STEP == kCosChunk ? all_ids : __shfl(all_ids, (int)(e0 - e_beg) + lane);
    float4 b[kCosU];
#pragma unroll
    for (int k = 0; k < kCosU; ++k) {
      const int slot = k * NPW + grp;
      const int64_t v = bcast_groups<NPW>(id, k * NPW, grp);
      b[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cok && e0 + slot < e_end) b[k] = *reinterpret_cast<const float4*>(Hd + v * ldd + col);
    }
#pragma unroll
    for (int k = 0; k < kCosU; ++k) {
      const int64_t e = e0 + k * NPW + grp;
      const float r = score(b[k], cok && e < e_end);
      if (gl == LPR - 1 && e < e_end) out[e] = r;
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
// A[i][k] = relu(P[src_i][k] + Q[dst_i][k]) (k < 128) feeds the 128x32 layer on the MFMA,
// then relu(+b2) . w3 and the sigmoid; hidden sizes 128 and 32 (src/model.py:258-260).

// One wave scores tiles of 32 edges: the tile's hidden-1 activations
// A[i][k] = relu(P[u_i][k] + Q[v_i][k]) are built from coalesced row loads (two 512-B rows
// of P and of Q per wave-instruction, each row's 32 16-B chunks in one lane half) and
// stored to the wave's LDS image with row i's chunk j at position j ^ (i & 15), so that the
// MFMA-layout reads (lane r reads row r) meet 16 distinct 4-bank groups per lane group.
// (Per-lane row loads in the MFMA layout — lane r reading its own edge's rows — touch 32
// rows per wave-instruction and each row's 128-B lines again from eight instructions:
// 0.37 ms against 0.27 ms at 2.56M edges, tools/micro/edge_mlp_ab.py.)  The 128x32 layer runs transposed, C^T = W2 A^T: W2 as the A operand
// (lane r holds hidden-2 unit r's row, in registers for the wave's life) and the staged A
// as the B operand (lane r = edge r), so lane (r, h) ends with 16 of edge r's 32 hidden-2
// units: the output dot is an in-register sum and one add across the lane halves.
// GROUPED: the edges are n_groups runs of one source (negative_sampler.Uniform's negatives:
// group g = optionally its positive (g, first[g]) then its K negatives (g, dst[g K + j])).
constexpr int kMlpTile = 32;        // edges per MFMA tile
constexpr int kMlpChunkTiles = 8;   // tiles per work item, at most
constexpr int kMlpWaves = 4;        // waves per 256-thread block, each with its own image
constexpr int kMlpResidentWaves = 2 * 256 * kMlpWaves;  // two blocks per CU (registers)

struct EdgeMlpArgs {
  const int64_t* src;    // per edge; GROUPED: per group
  const int64_t* dst;    // per edge; GROUPED: [n_groups x K] negatives
  const int64_t* first;  // GROUPED: per-group positive destination, or null
  float* out_first;
  float* out;
  const float* P;
  const float* Q;
  const float* W2;
  const float* b2;
  const float* w3;
  const float* b3;
  int64_t n_edges;       // ungrouped edge count
  int64_t K;             // GROUPED: negatives per group
  int64_t per_group;     // GROUPED: K + (first != null)
  int64_t chunks;        // GROUPED: work items per group
  int64_t n_items;
  int64_t chunk_tiles;   // tiles per work item
};

// A tile's 32 edges: lane r's destination row (and source row, per-edge form); -1 past the
// end.  Both lane halves hold the same ids.
template <bool GROUPED>
__device__ __forceinline__ void mlp_tile_ids(const EdgeMlpArgs& a, int64_t g, int64_t e,
                                             int64_t e_end, int64_t lead, int& v, int& u) {
  v = -1;
  if (e >= e_end) return;
  if constexpr (GROUPED) {
    v = (int)(e < lead ? a.first[g] : a.dst[g * a.K + e - lead]);
  } else {
    v = (int)a.dst[e];
    u = (int)a.src[e];
  }
}

// Row loads of a tile, wave-instruction i = rows 2 i + h (lane half h), chunk r ^ (row & 15):
// GROUPED the Q chunks of rows i in [i0, i0 + N); per edge the (Q, P) chunk pairs.
template <bool GROUPED, int N>
__device__ __forceinline__ void mlp_load(const float4* __restrict__ Q4,
                                         const float4* __restrict__ P4, int v, int u, int r,
                                         int h, int i0, float4 (&q)[N], float4 (&p)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int row = 2 * (i0 + i) + h;
    const int vr = bcast_groups<2>(v, 2 * (i0 + i), h);
    const int ur = GROUPED ? 0 : bcast_groups<2>(u, 2 * (i0 + i), h);
    const int j = r ^ (row & 15);
    q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (!GROUPED) p[i] = q[i];
    if (vr >= 0) {
      q[i] = Q4[(int64_t)vr * 32 + j];
      if constexpr (!GROUPED) p[i] = P4[(int64_t)ur * 32 + j];
    }
  }
}

__device__ __forceinline__ float4 relu_add4(const float4& p, const float4& q) {
  return make_float4(fmaxf(p.x + q.x, 0.f), fmaxf(p.y + q.y, 0.f), fmaxf(p.z + q.z, 0.f),
                     fmaxf(p.w + q.w, 0.f));
}

// The 128x32 layer of one staged tile (C^T = W2 A^T) and the output: sigmoid(w3 . relu(. + b2)
// + b3) of edge r, stored by lane r of the first half.  RELU_P: the image holds Q rows only,
// A = relu(P + Q) formed here with the source's P chunks pc (16 h + c).
template <bool RELU_P>
__device__ __forceinline__ float mlp_tile_score(const EdgeMlpArgs& a, const float4* S,
                                                const float4 (&w)[16], const float4* pc, int r,
                                                int h, float b3v) {
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    float4 x = S[r * 32 + ((16 * h + c) ^ (r & 15))];
    if constexpr (RELU_P) x = relu_add4(pc[c], x);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[c].x, x.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[c].y, x.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[c].z, x.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[c].w, x.w, acc, 0, 0, 0);
  }
  // acc[q]: hidden-2 unit 8 (q >> 2) + 4 h + (q & 3) of edge r
  float y = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int jj = 8 * (q >> 2) + 4 * h + (q & 3);
    y = fmaf(fmaxf(acc[q] + a.b2[jj], 0.f), a.w3[jj], y);
  }
  y += __shfl_xor(y, 32);
  return 1.f / (1.f + expf(-(y + b3v)));
}

__device__ __forceinline__ void mlp_store(const EdgeMlpArgs& a, bool grouped, int64_t g,
                                          int64_t e, int64_t lead, float sc) {
  if (!grouped) a.out[e] = sc;
  else if (e < lead) a.out_first[g] = sc;
  else a.out[g * a.K + e - lead] = sc;
}

__device__ __forceinline__ void mlp_load_w2(const EdgeMlpArgs& a, int r, int h, float4 (&w)[16]) {
  const float4* W4 = reinterpret_cast<const float4*>(a.W2) + r * 32 + 16 * h;
#pragma unroll
  for (int c = 0; c < 16; ++c) w[c] = W4[c];  // W2 row r, chunks 16 h + c: k = 64 h + 4 c + s
}

// work item -> (group, tiles [t0, t1), edge end)
template <bool GROUPED>
__device__ __forceinline__ void mlp_item(const EdgeMlpArgs& a, int64_t item, int64_t tiles_pg,
                                         int64_t& g, int64_t& t0, int64_t& t1, int64_t& e_end) {
  if constexpr (GROUPED) {
    g = item / a.chunks;
    t0 = (item - g * a.chunks) * a.chunk_tiles;
    t1 = t0 + a.chunk_tiles < tiles_pg ? t0 + a.chunk_tiles : tiles_pg;
    e_end = a.per_group;
  } else {
    g = 0;
    t0 = item * a.chunk_tiles;
    t1 = t0 + a.chunk_tiles;
    e_end = a.n_edges;
  }
}

template <bool GROUPED>
__global__ __launch_bounds__(256, 2) void edge_mlp_lds_kernel(EdgeMlpArgs a) {
  __shared__ float4 image[kMlpWaves][kMlpTile * 32];  // 16 KB per wave
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  float4* S = image[wv];
  const float4* P4 = reinterpret_cast<const float4*>(a.P);
  const float4* Q4 = reinterpret_cast<const float4*>(a.Q);
  float4 w[16];
  mlp_load_w2(a, r, h, w);
  const float b3v = a.b3[0];
  const int64_t tiles_pg = GROUPED ? (a.per_group + kMlpTile - 1) / kMlpTile : 0;
  const int64_t lead = (GROUPED && a.first) ? 1 : 0;
  for (int64_t item = (int64_t)blockIdx.x * kMlpWaves + wv; item < a.n_items;
       item += (int64_t)gridDim.x * kMlpWaves) {
    int64_t g, t0, t1, e_end;
    mlp_item<GROUPED>(a, item, tiles_pg, g, t0, t1, e_end);
    const int u_g = GROUPED ? (int)a.src[g] : 0;
    // GROUPED: the source's P chunks this lane adds, r ^ (row & 15) for the 16 row
    // residues of one lane half (rows 2 i + h, i < 8, then the same residues again)
    float4 pg[8];
    if constexpr (GROUPED) {
#pragma unroll
      for (int i = 0; i < 8; ++i) pg[i] = P4[(int64_t)u_g * 32 + (r ^ ((2 * i + h) & 15))];
    }
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t e = t * kMlpTile + r;  // this lane's edge (both halves)
      int v, u = u_g;
      mlp_tile_ids<GROUPED>(a, g, e, e_end, lead, v, u);
      // stage, eight row pairs at a time
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float4 q[8], p[8];
        mlp_load<GROUPED, 8>(Q4, P4, v, u, r, h, 8 * half, q, p);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          S[(2 * (8 * half + i) + h) * 32 + r] = relu_add4(GROUPED ? pg[i] : p[i], q[i]);
      }
      // (the wave's own LDS writes precede its reads in issue order)
      const float sc = mlp_tile_score<false>(a, S, w, nullptr, r, h, b3v);
      if (h == 0 && e < e_end) mlp_store(a, GROUPED, g, e, lead, sc);
    }
  }
}

// tiles per work item: up to kMlpChunkTiles (the wave's W2 / P registers reused), fewer when
// the launch would otherwise leave resident waves idle
int64_t mlp_chunk_tiles(int64_t tiles) {
  int64_t c = (tiles + kMlpResidentWaves - 1) / kMlpResidentWaves;
  return c < 1 ? 1 : (c > kMlpChunkTiles ? kMlpChunkTiles : c);
}

int launch_edge_mlp_lds(bool grouped, EdgeMlpArgs& a, hipStream_t s) {
  if (a.n_items <= 0) return GNNREC_OK;
  int64_t blocks = (a.n_items + kMlpWaves - 1) / kMlpWaves;
  if (blocks > kMlpResidentWaves / kMlpWaves) blocks = kMlpResidentWaves / kMlpWaves;
  if (grouped)
    hipLaunchKernelGGL(edge_mlp_lds_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(edge_mlp_lds_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return check_launch(grouped ? "gnnrec_edge_mlp_grouped_f32" : "gnnrec_edge_mlp_f32");
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
  const int64_t tiles = (n_edges + kMlpTile - 1) / kMlpTile;
  const int64_t ct = mlp_chunk_tiles(tiles);
  EdgeMlpArgs a{src, dst, nullptr, nullptr, out, P, Q, W2, b2, w3, b3, n_edges, 0, 0, 0,
                (tiles + ct - 1) / ct, ct};
  return launch_edge_mlp_lds(false, a, as_stream(stream));
}

extern "C" int gnnrec_edge_mlp_grouped_f32(const int64_t* src_g, int64_t n_groups,
                                           const int64_t* first, float* out_first, int64_t K,
                                           const int64_t* dst, float* out, const float* P,
                                           const float* Q, const float* W2, const float* b2,
                                           const float* w3, const float* b3, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_groups >= 0 && K >= 0, "gnnrec_edge_mlp_grouped_f32: negative size");
  if (n_groups == 0 || (K == 0 && first == nullptr)) return GNNREC_OK;
  GNNREC_REQUIRE(src_g && P && Q && W2 && b2 && w3 && b3 && (K == 0 || (dst && out)) &&
                     (!first || out_first),
                 "gnnrec_edge_mlp_grouped_f32: null pointer");
  GNNREC_REQUIRE(aligned16(P) && aligned16(Q) && aligned16(W2),
                 "gnnrec_edge_mlp_grouped_f32: P/Q/W2 must be 16-byte aligned");
  const int64_t per_group = K + (first ? 1 : 0);
  const int64_t tiles = (per_group + kMlpTile - 1) / kMlpTile;
  const int64_t ct = mlp_chunk_tiles(n_groups * tiles);
  const int64_t chunks = (tiles + ct - 1) / ct;
  EdgeMlpArgs a{src_g, dst, first, out_first, out, P, Q, W2, b2, w3, b3, 0, K, per_group, chunks,
                n_groups * chunks, ct};
  return launch_edge_mlp_lds(true, a, as_stream(stream));
}
