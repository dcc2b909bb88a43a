// a1 — neighbour gather + segmented mean / max / sum over a dst-major CSR.
//
// Replaces DGL 0.5.2's gSpMM behind graph.update_all(fn.copy_src|fn.u_mul_e,
// fn.mean|fn.max) as called from ConvLayer.forward (reference
// src/model.py:143-208).  Semantics restated from DGL: mean = sum / max(deg,1),
// max of an empty neighbourhood = 0, u_mul_e multiplies the source row by the
// scalar edge weight before reducing.
//
// Layout / mapping (gfx950, wave64):
//   * one wavefront per destination row (grid-stride over rows);
//   * a source row of d fp32 is read by LPR lanes with 16-B (float4) loads, so
//     one wave-instruction fetches NPI = 64/LPR neighbour rows (d=128: two
//     512-B rows = 1 KiB per instruction, the widest CDNA load);
//   * 64 neighbour indices are fetched with one coalesced 256-B load and
//     broadcast with ds_bpermute (__shfl); UNROLL wave-instructions are issued
//     back to back so every lane keeps UNROLL x 16 B in flight;
//   * neighbour k of a row always lands in lane group k % NPI and groups are
//     combined by a fixed xor-tree, so the per-row reduction order depends only
//     on the CSR row: results are bitwise reproducible and identical for any
//     row partition across ranks.
#include "common.hpp"
#include <cmath>

namespace gnnrec {
namespace {

template <int VEC>
struct Frag {
  float v[VEC];
};

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
    *reinterpret_cast<float4*>(p) = make_float4(f.v[0], f.v[1], f.v[2], f.v[3]);
  } else {
    *p = f.v[0];
  }
}

template <int LPR, int VEC, int REDUCE, bool WEIGHTED, int UNROLL>
__global__ __launch_bounds__(256) void spmm_csr_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx, int64_t n_dst, int d,
    float* __restrict__ out, int64_t ldo, int empty_neginf) {
  constexpr int NPI = kWave / LPR;  // neighbour rows per wave-instruction
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR;
  const int col = blockIdx.y * (LPR * VEC) + (lane % LPR) * VEC;
  const bool colok = col < d;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const int64_t wstride = (int64_t)gridDim.x * 4;

  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_dst; row += wstride) {
    const int64_t beg = indptr[row];
    const int64_t end = indptr[row + 1];
    Frag<VEC> acc;
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc.v[v] = init;

    for (int64_t base = beg; base < end; base += 64) {
      const int cnt = (int)((end - base) < 64 ? (end - base) : 64);
      const int myidx = lane < cnt ? indices[base + lane] : 0;
      float myw = 0.f;
      if constexpr (WEIGHTED) myw = lane < cnt ? ew[base + lane] : 0.f;
      for (int j = 0; j < cnt; j += NPI * UNROLL) {
        Frag<VEC> val[UNROLL];
        bool ok[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          const int k = j + u * NPI + grp;
          ok[u] = (k < cnt) && colok;
          const int src = __shfl(myidx, k & 63);
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
          if constexpr (WEIGHTED) w = __shfl(myw, (j + u * NPI + grp) & 63);
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
    // combine the NPI lane groups with a fixed xor tree
#pragma unroll
    for (int off = LPR; off < kWave; off <<= 1) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float o = __shfl_xor(acc.v[v], off);
        acc.v[v] = (REDUCE == GNNREC_REDUCE_MAX) ? fmaxf(acc.v[v], o) : acc.v[v] + o;
      }
    }
    const int64_t deg = end - beg;
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
    if (grp == 0 && colok) store_frag<VEC>(out + row * ldo + col, acc);
  }
}

template <int LPR, int VEC, int REDUCE, bool WEIGHTED>
int launch4(const int64_t* indptr, const int32_t* indices, const float* ew, const float* X,
            int64_t ldx, int64_t n_dst, int d, float* out, int64_t ldo, int flags, hipStream_t s) {
  constexpr int UNROLL = (VEC == 4) ? 4 : 2;
  const int64_t waves_needed = n_dst;
  int64_t blocks = (waves_needed + 3) / 4;
  const int64_t max_blocks = 256 * 32;  // 256 CUs x 32 blocks: grid-stride beyond that
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  const int cols_per_slice = LPR * VEC;
  dim3 grid((unsigned)blocks, (unsigned)((d + cols_per_slice - 1) / cols_per_slice));
  hipLaunchKernelGGL((spmm_csr_kernel<LPR, VEC, REDUCE, WEIGHTED, UNROLL>), grid, dim3(256), 0, s,
                     indptr, indices, ew, X, ldx, n_dst, d, out, ldo,
                     (flags & GNNREC_SPMM_EMPTY_NEGINF) ? 1 : 0);
  return check_launch("gnnrec_spmm_csr_f32");
}

template <int VEC, int REDUCE, bool WEIGHTED>
int dispatch_lpr(int lpr, const int64_t* indptr, const int32_t* indices, const float* ew,
                 const float* X, int64_t ldx, int64_t n_dst, int d, float* out, int64_t ldo,
                 int flags, hipStream_t s) {
  if constexpr (VEC == 1) {
    return launch4<64, 1, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
  } else {
    switch (lpr) {
      case 4: return launch4<4, 4, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
      case 8: return launch4<8, 4, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
      case 16: return launch4<16, 4, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
      case 32: return launch4<32, 4, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
      default: return launch4<64, 4, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
    }
  }
}

template <int VEC>
int dispatch_reduce(int reduce, bool weighted, int lpr, const int64_t* indptr,
                    const int32_t* indices, const float* ew, const float* X, int64_t ldx,
                    int64_t n_dst, int d, float* out, int64_t ldo, int flags, hipStream_t s) {
#define GNNREC_SPMM_CASE(R)                                                                          \
  if (weighted)                                                                                      \
    return dispatch_lpr<VEC, R, true>(lpr, indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s); \
  return dispatch_lpr<VEC, R, false>(lpr, indptr, indices, ew, X, ldx, n_dst, d, out, ldo, flags, s);
  switch (reduce) {
    case GNNREC_REDUCE_SUM: { GNNREC_SPMM_CASE(GNNREC_REDUCE_SUM) }
    case GNNREC_REDUCE_MEAN: { GNNREC_SPMM_CASE(GNNREC_REDUCE_MEAN) }
    default: { GNNREC_SPMM_CASE(GNNREC_REDUCE_MAX) }
  }
#undef GNNREC_SPMM_CASE
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_spmm_csr_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                                   const float* X, int64_t ldx, int64_t n_dst, int64_t d,
                                   int reduce, int flags, float* out, int64_t ldo, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_dst >= 0 && d >= 0, "gnnrec_spmm_csr_f32: negative size");
  GNNREC_REQUIRE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN ||
                     reduce == GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_csr_f32: unknown reduce %d", reduce);
  GNNREC_REQUIRE(d <= (1 << 20), "gnnrec_spmm_csr_f32: d=%lld too large", (long long)d);
  if (n_dst == 0 || d == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr && out, "gnnrec_spmm_csr_f32: null indptr/out");
  GNNREC_REQUIRE(ldx >= d && ldo >= d, "gnnrec_spmm_csr_f32: leading dimension < d");
  const bool vec4 = (d % 4 == 0) && (ldx % 4 == 0) && (ldo % 4 == 0) && aligned16(X) &&
                    aligned16(out);
  int lpr = 64;
  if (vec4) {
    const int64_t lanes = d / 4;
    lpr = 4;
    while (lpr < lanes && lpr < 64) lpr <<= 1;
  }
  hipStream_t s = as_stream(stream);
  if (vec4)
    return dispatch_reduce<4>(reduce, ew != nullptr, lpr, indptr, indices, ew, X, ldx, n_dst,
                              (int)d, out, ldo, flags, s);
  return dispatch_reduce<1>(reduce, ew != nullptr, lpr, indptr, indices, ew, X, ldx, n_dst, (int)d,
                            out, ldo, flags, s);
}
