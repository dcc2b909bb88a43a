// Shared device helpers of the neighbour gather (a1): used by the plain
// aggregation kernels (spmm.hip) and the fused aggregate+project kernel
// (spmm_project.hip), so both reduce every row in the same fixed order.
#pragma once
#include "common.hpp"
#include <cmath>

namespace gnnrec {
namespace {

template <int VEC>
struct Frag {
  float v[VEC];
};

// Streams read or written once per launch (CSR indices / indptr, self rows, outputs and
// partials) vs the gathered source table, which should keep the caches: the streams use
// non-temporal loads / stores (C4 pass 143.0 -> 142.3 ms against plain ones in an alternating
// A/B, tools/micro/bench_ab.sh; tiles 4.45 -> 4.42 ms, fused 34.58 -> 34.45).
typedef float f32x4s __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  return __builtin_nontemporal_load(p);
}
__device__ __forceinline__ float4 ld_stream4(const float* p) {
  const f32x4s t = __builtin_nontemporal_load(reinterpret_cast<const f32x4s*>(p));
  return make_float4(t[0], t[1], t[2], t[3]);
}
__device__ __forceinline__ void st_stream4(float* p, float a, float b, float c, float d) {
  const f32x4s t = {a, b, c, d};
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4s*>(p));
}

template <int VEC>
__device__ __forceinline__ void load_frag(Frag<VEC>& f, const float* p) {
  if constexpr (VEC == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    f.v[0] = t.x; f.v[1] = t.y; f.v[2] = t.z; f.v[3] = t.w;
  } else {
    f.v[0] = *p;
  }
}

template <int VEC>
__device__ __forceinline__ void store_frag(float* p, const Frag<VEC>& f) {
  if constexpr (VEC == 4) {
    st_stream4(p, f.v[0], f.v[1], f.v[2], f.v[3]);
  } else {
    *p = f.v[0];
  }
}

// A gather step's per-edge source index (and weight) to each lane group: lane group grp
// takes the range's edge base + grp, held by that lane of the index load.
// (readlane + select: at C4 the same pass time as __shfl's ds_bpermute, 142.56 ms both,
// with the LDS pipe left free; profiles/r06ad_c4_gather_readlane_ab.txt)
template <int NPI, typename T>
__device__ __forceinline__ T edge_bcast(T x, int base, int grp) {
  return bcast_groups<NPI>(x, base, grp);
}

template <int REDUCE>
__device__ __forceinline__ float combine(float a, float b) {
  return REDUCE == GNNREC_REDUCE_MAX ? fmaxf(a, b) : a + b;
}

// Per-lane partial reduction of edges [beg, end) (lane group grp takes k % NPI == grp).
// PRE: the first 64 indices of the range were loaded by the caller (lane k holds
// indices[beg + k]) — a row kernel prefetches them for row i+1 while row i gathers.
template <int LPR, int VEC, int REDUCE, bool WEIGHTED, int UNROLL, bool PRE = false>
__device__ __forceinline__ void gather_range(int64_t beg, int64_t end,
                                             const int32_t* __restrict__ indices,
                                             const float* __restrict__ ew,
                                             const float* __restrict__ X, int64_t ldx, int col,
                                             bool colok, int lane, int grp, Frag<VEC>& acc,
                                             int pre_idx = 0) {
  constexpr int NPI = kWave / LPR;
  for (int64_t base = beg; base < end; base += 64) {
    const int cnt = (int)((end - base) < 64 ? (end - base) : 64);
    int myidx;
    if (PRE && base == beg) myidx = pre_idx;
    else myidx = lane < cnt ? ld_stream(indices + base + lane) : 0;
    float myw = 0.f;
    if constexpr (WEIGHTED) myw = lane < cnt ? ld_stream(ew + base + lane) : 0.f;
    for (int j = 0; j < cnt; j += NPI * UNROLL) {
      Frag<VEC> val[UNROLL];
      bool ok[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int k = j + u * NPI + grp;
        ok[u] = (k < cnt) && colok;
        const int src = edge_bcast<NPI>(myidx, j + u * NPI, grp);
        if (ok[u]) {
          load_frag<VEC>(val[u], X + (int64_t)src * ldx + col);
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) val[u].v[v] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        float w = 1.f;
        if constexpr (WEIGHTED) w = edge_bcast<NPI>(myw, j + u * NPI, grp);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float m = WEIGHTED ? val[u].v[v] * w : val[u].v[v];
          if constexpr (REDUCE == GNNREC_REDUCE_MAX) {
            if (ok[u]) acc.v[v] = fmaxf(acc.v[v], m);
          } else {
            acc.v[v] += m;
          }
        }
      }
    }
  }
}

template <int LPR, int VEC, int REDUCE>
__device__ __forceinline__ void combine_groups(Frag<VEC>& acc) {
#pragma unroll
  for (int off = LPR; off < kWave; off <<= 1) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc.v[v] = combine<REDUCE>(acc.v[v], __shfl_xor(acc.v[v], off));
  }
}

// acc = out[row] (+ | max) acc: a source-range tile added to the partial of earlier tiles
template <int VEC, int REDUCE>
__device__ __forceinline__ void accumulate_into(Frag<VEC>& acc, const float* p) {
  Frag<VEC> o;
  if constexpr (VEC == 4) {
    const float4 t = ld_stream4(p);
    o.v[0] = t.x; o.v[1] = t.y; o.v[2] = t.z; o.v[3] = t.w;
  } else {
    load_frag<VEC>(o, p);
  }
#pragma unroll
  for (int v = 0; v < VEC; ++v) acc.v[v] = combine<REDUCE>(o.v[v], acc.v[v]);
}

template <int VEC, int REDUCE>
__device__ __forceinline__ void finalize(Frag<VEC>& acc, int64_t deg, int empty_neginf) {
  if constexpr (REDUCE == GNNREC_REDUCE_MEAN) {
    const float dd = (float)(deg > 0 ? deg : 1);
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc.v[v] = acc.v[v] / dd;
  } else if constexpr (REDUCE == GNNREC_REDUCE_MAX) {
    if (deg == 0 && !empty_neginf) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = 0.f;
    }
  }
}

}  // namespace
}  // namespace gnnrec
