// a1+a3+a4 fused for TWO relations that gather from ONE source table (C5's clicked-by and
// bought-by, both item -> user), the projections on the fp32 MFMA:
//   out[v] = combine( epi(h[v]·W_self,aᵀ + agg_a(v)·W_neigh,aᵀ + b_a [+ bne_a]),
//                     epi(h[v]·W_self,bᵀ + agg_b(v)·W_neigh,bᵀ + b_b [+ bne_b]) ) / out_div
// agg_r = sum / mean over relation r's in-edges of X[src] (· w_e), X the SHARED source table.
// Reference: ConvLayer.forward (src/model.py:143-148 aggregation, :226-235 projection, ReLU,
// norm) for each relation, HeteroGraphConv's cross-relation combine (:384-406).
//
// Why a second pair kernel: gnnrec_spmm_project2_f32 gathers two PRE-projected tables
// (X·W_neigh,aᵀ and X·W_neigh,bᵀ, 512 MB each at C5): a 1 GB working set against the
// 256 MB Infinity Cache, so the lower-degree relation's gathers go to HBM proper (the
// launch ran at 0.906 of 8 TB/s against 0.955 for C4's one-table launch), and the two
// pre-projection GEMMs sit on the layer's critical path.  Here both relations gather the
// one raw 512 MB table, and all four 128×128 projections run in the epilogue.  Four fp32
// weight matrices (256 KiB) do not fit in LDS, so the VALU matvec of the one-relation kernel
// is out; instead a block owns 32-row tiles:
//   gather   each of the 8 waves gathers 4 rows of relation a, then of relation b, in
//            lockstep (the 4 rows' bounds and first 64 indices requested together, then
//            steps of 2·LU neighbours of all 4 rows; per row the summation order of
//            spmm_csr_kernel's gather_range, so each aggregate has its bits), into the
//            LDS tile A = [h_self | agg_a | agg_b] (32 × 384 fp32, row stride 388 floats:
//            conflict-free ds_read_b128);
//   project  wave w owns output columns 32·(w & 3) of relation (w >> 2): C = [h | agg_r] ·
//            [W_self,r | W_neigh,r]ᵀ, K = 256, as 128 v_mfma_f32_32x32x2_f32 — lane half 0
//            consumes the self half of K, lane half 1 the neighbour half (a fixed
//            permutation of the reference's summation order); the B operands stream from L2
//            by buffer loads out of ONE packed [4][128][128] k-major weight array (a
//            wave-uniform base), in chunks of 16 double-buffered under the MFMAs — 256 KiB
//            per 32 rows instead of per row pair;
//   epilogue C of both relations lands in LDS over the A tile; each wave finishes 4 rows:
//            bias (+ the non-empty bias), ReLU, zero-guarded L2 norm and the combine (sum,
//            max, or the attention softmax over the two relations) in registers, one
//            non-temporal 512-B store per row.
// Two blocks per CU (≈50 KiB of LDS each), so one block's MFMA phase runs under the other's
// gather.  Rows come from the row queue in whole tiles, or an XCD-contiguous static walk.
//
// Measured (C5 user side, 10M rows × (40 + 10) edges, 268 GB, tools/gpu/r04c_pairvar.sh and
// r04e_pairh.sh): the gather phase alone (a round-4 timing build) 34.6 ms = 0.969 of
// 8 TB/s — one 512 MB table is the cache-friendly working set the pre-projected launch lacks —
// the MFMA phase alone 14.8 ms, the launch 38.4–38.6 ms (0.87): while one block sits in its
// MFMA phase only the other block's 8 waves gather.  The pre-projected launch takes 36.6–37.8
// ms plus its two 1M-row GEMMs, so the C5 passes come out within 0.5 ms of each other
// (153.3–154.0 vs 154.0–154.4 ms); the sharded pass keeps the pre-projected form by default
// (GNNREC_PAIR_RAW=1 selects this one).  Not kept: a software-pipelined form (the previous
// tile's MFMAs interleaved into this tile's gather steps, operands loaded one chunk ahead,
// aggregates double-buffered, self rows straight from H by buffer loads) — 43.9 ms, its MFMA
// state and gather share 128 VGPRs and spill 124–152 B/lane; LU = 1 / 3 lockstep unrolls 39.9
// / 39.1 ms; the self rows requested ahead of the gathers: unchanged.
//
// Not kept either (tools/EXPERIMENTS.md): the projections as six bf16 MFMA products of
// three-way split operands (fp32-accurate, 2.7x fewer MFMA issue cycles but 1.5x the weight
// bytes per tile: launch 47.3 vs 38.7 ms, profiles/r04j_pair_bf16x3_ab.md).  What bounds the
// projection phase (14.2 ms against 8.3 ms of MFMA issue at 2.4 GHz) is not the weight
// stream's latency — streaming the weights 8, 16 or 32 k-steps ahead changed nothing
// (profiles/r04r_pair_weight_stream.md) — but the clock under MFMA load (≈2.0-2.2 GHz) and
// each tile's epilogue and barriers beside the MFMAs; both phases need all 16 resident waves
// (profiles/r04s_pair_waves_per_cu.md).  48-row tiles / a third block per CU were not
// attempted: the pre-projected launch stays the default.
#include "common.hpp"
#include "gather.hpp"
#include "rowq.hpp"

namespace gnnrec {
namespace {

constexpr int kQD = 128;                 // d (source, self and output width)
constexpr int kQT = 32;                  // rows per tile
constexpr int kQWaves = 8;               // waves per block
constexpr int kQRows = kQT / kQWaves;    // rows gathered per wave per tile
constexpr int kQALd = 3 * kQD + 4;       // A tile row stride (floats)
constexpr int kQCLd = kQD + 8;           // C tile row stride
constexpr int kQLU = 2;   // lockstep gather: steps of 2·LU neighbours of 4 rows at once
constexpr int kQU = 4;    // gather_range unroll for rows above 64 edges
constexpr int kQWC = 16;  // B operands per chunk
static_assert(2 * kQT * kQCLd <= kQT * kQALd, "C tiles must fit over the A tile");

typedef float f32x16q __attribute__((ext_vector_type(16)));
typedef float f32x4q __attribute__((ext_vector_type(4)));

// Four consecutive A-tile elements of row `row`, columns [c, c + 4)
__device__ __forceinline__ void put4(float* tile, int row, int c, float4 v) {
  *reinterpret_cast<float4*>(tile + row * kQALd + c) = v;
}

struct RawRel {
  const int64_t* indptr;
  const int32_t* indices;
  const float* ew;
  const float* bias;     // b_r (NULL: none)
  const float* bias_ne;  // added to rows with >= 1 in-edge (NULL: none)
  int mean;
};

__device__ __forceinline__ void activate_q(bool relu, bool l2, float& y0, float& y1) {
  if (relu) {
    y0 = fmaxf(y0, 0.f);
    y1 = fmaxf(y1, 0.f);
  }
  if (l2) {
    float ss = y0 * y0 + y1 * y1;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) ss += __shfl_xor(ss, off);
    float nrm = sqrtf(ss);
    if (nrm == 0.f) nrm = 1.f;
    y0 = y0 / nrm;
    y1 = y1 / nrm;
  }
}

// The 4 rows [rbase, rbase + nv) of one relation, gathered in lockstep into A tile columns
// [cofs, cofs + 128) of tile rows [r0, r0 + 4); their non-empty flags into ne[].
template <bool W>
__device__ __forceinline__ void gather4(const RawRel& r, const float* __restrict__ X,
                                        int64_t ldx, int64_t rbase, int nv, float* As,
                                        int r0, int cofs, int* ne, int lane) {
  constexpr int LPR = 32, VEC = 4, NPI = kWave / LPR, U = kQLU, kLR = 4;
  const int grp = lane / LPR, col = (lane % LPR) * VEC;
  const int64_t ipl = nv > 0 && lane <= nv ? ld_stream(r.indptr + rbase + lane) : 0;
  int64_t b[kLR + 1];
#pragma unroll
  for (int i = 0; i <= kLR; ++i) b[i] = __shfl(ipl, i <= nv ? i : nv);
  int ridx[kLR], dg[kLR];
  float rwt[kLR];
  int dmax = 0;
#pragma unroll
  for (int i = 0; i < kLR; ++i) {
    dg[i] = i < nv ? (int)(b[i + 1] - b[i]) : 0;
    ridx[i] = lane < dg[i] ? ld_stream(r.indices + b[i] + lane) : 0;
    rwt[i] = 0.f;
    if constexpr (W) rwt[i] = lane < dg[i] ? ld_stream(r.ew + b[i] + lane) : 0.f;
    dmax = dg[i] > dmax ? dg[i] : dmax;
  }
  Frag<VEC> acc[kLR];
#pragma unroll
  for (int i = 0; i < kLR; ++i)
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[i].v[v] = 0.f;
  if (dmax <= 64) {
    for (int j = 0; j < dmax; j += NPI * U) {
      Frag<VEC> val[kLR][U];
#pragma unroll
      for (int i = 0; i < kLR; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = j + u * NPI + grp;
          const int src = __shfl(ridx[i], k & 63);
          if (k < dg[i]) {
            load_frag<VEC>(val[i][u], X + (int64_t)src * ldx + col);
          } else {
#pragma unroll
            for (int v = 0; v < VEC; ++v) val[i][u].v[v] = 0.f;
          }
        }
#pragma unroll
      for (int i = 0; i < kLR; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float w = 1.f;
          if constexpr (W) w = __shfl(rwt[i], (j + u * NPI + grp) & 63);
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[i].v[v] += W ? val[i][u].v[v] * w : val[i][u].v[v];
        }
    }
  } else {
#pragma unroll
    for (int i = 0; i < kLR; ++i)
      if (i < nv)
        gather_range<LPR, VEC, GNNREC_REDUCE_SUM, W, kQU, true>(
            b[i], b[i + 1], r.indices, r.ew, X, ldx, col, true, lane, grp, acc[i], ridx[i]);
  }
#pragma unroll
  for (int i = 0; i < kLR; ++i) {
    combine_groups<LPR, VEC, GNNREC_REDUCE_SUM>(acc[i]);
    if (r.mean) finalize<VEC, GNNREC_REDUCE_MEAN>(acc[i], dg[i], 0);
    if (grp == 0)
      put4(As, r0 + i, cofs + col,
                make_float4(acc[i].v[0], acc[i].v[1], acc[i].v[2], acc[i].v[3]));
    if (lane == 0) ne[r0 + i] = dg[i] > 0;
  }
}

template <bool WA, bool WB>
__global__ __launch_bounds__(kQWaves * 64, 4) void spmm_pair_mfma_kernel(
    RawRel ra, RawRel rb, const float* __restrict__ X, int64_t ldx, const float* __restrict__ H,
    int64_t ldh, const float* __restrict__ WT4, int64_t n_dst, int epilogue, int combine,
    const float* __restrict__ attn_vec, float out_div, float* __restrict__ out, int64_t ldo,
    unsigned* rq, int rq_ch) {
  __shared__ __attribute__((aligned(16))) float As[kQT * kQALd];
  __shared__ int nes[2][kQT];
  __shared__ int64_t blk_r[2];
  float* const Ca = reinterpret_cast<float*>(As);  // over the A tile once the MFMAs read it
  float* const Cb = Ca + kQT * kQCLd;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, bh = lane >> 5;
  const int col = li * 4;
  const int j0 = 2 * lane;
  const int cb = wave & 3, rr = wave >> 2;
  const bool relu = epilogue & GNNREC_EPI_RELU, l2 = epilogue & GNNREC_EPI_L2NORM;

  // B operands: lane half bh of a relation-rr wave reads matrix 2·rr + bh of the packed
  // [W_self,aᵀ, W_neigh,aᵀ, W_self,bᵀ, W_neigh,bᵀ] (each k-major 128×128): element
  // [i][32·cb + li]; one 32-bit per-lane offset + an immediate row offset per load
  const void* const wsrc = WT4;
  const uint64_t wbase = ((uint64_t)__builtin_amdgcn_readfirstlane(
                              (unsigned)((uintptr_t)wsrc >> 32)) << 32) |
                         (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)wsrc);
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(wbase), 0, 4 * kQD * kQD * 4, 0x00020000);
  const int wvoff = ((2 * rr + bh) * kQD * kQD + 32 * cb + li) * 4;
  // A operands: row li of the tile, K columns [0, 128) (self) for lane half 0 and the
  // relation's aggregate [128 + 128·rr, +128) for lane half 1
  const int acol = bh ? kQD + kQD * rr : 0;
  const float* const ap = As + li * kQALd + acol;

  auto tile = [&](int64_t t0, int64_t lim) __attribute__((always_inline)) {
    const int64_t rbase = t0 + wave * kQRows;
    const int64_t left = lim - rbase;
    const int nv = (int)(left <= 0 ? 0 : left < kQRows ? left : kQRows);
    const int r0 = wave * kQRows;
    // self rows, two per instruction, requested before the gathers (their latency hides
    // under the gathers instead of ahead of the MFMA phase's barrier)
    float4 hs[kQRows / 2];
#pragma unroll
    for (int q = 0; q < kQRows / 2; ++q) {
      const int rl = 2 * q + bh;
      hs[q] = rl < nv ? ld_stream4(H + (rbase + rl) * ldh + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    gather4<WA>(ra, X, ldx, rbase, nv, As, r0, kQD, nes[0], lane);
    gather4<WB>(rb, X, ldx, rbase, nv, As, r0, 2 * kQD, nes[1], lane);
#pragma unroll
    for (int q = 0; q < kQRows / 2; ++q) put4(As, r0 + 2 * q + bh, col, hs[q]);
    __syncthreads();

    constexpr int kWC = kQWC;
    float bw[2][kWC];
    auto load_w = [&](float* dst, int i0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < kWC; ++i)
        dst[i] = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(wrsrc, wvoff, (i0 + i) * kQD * 4, 0));
    };
    f32x16q c;
#pragma unroll
    for (int v = 0; v < 16; ++v) c[v] = 0.f;
    load_w(bw[0], 0);
#pragma unroll
    for (int ch = 0; ch < kQD / kWC; ++ch) {
      if (ch + 1 < kQD / kWC) load_w(bw[(ch + 1) & 1], (ch + 1) * kWC);
      __builtin_amdgcn_sched_barrier(0);
      const float* w = bw[ch & 1];
#pragma unroll
      for (int i = 0; i < kWC; i += 4) {
        const f32x4q a = *reinterpret_cast<const f32x4q*>(ap + ch * kWC + i);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0], w[i], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1], w[i + 1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2], w[i + 2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[3], w[i + 3], c, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // every wave's MFMAs have read the A tile: C goes over it
    // D map of the 32x32 MFMA: col = lane & 31, row = (v & 3) + 8 (v >> 2) + 4 bh
    float* cp = (rr ? Cb : Ca) + 32 * cb + li;
#pragma unroll
    for (int v = 0; v < 16; ++v) cp[((v & 3) + 8 * (v >> 2) + 4 * bh) * kQCLd] = c[v];
    __syncthreads();

    const float ba0 = ra.bias ? ra.bias[j0] : 0.f, ba1 = ra.bias ? ra.bias[j0 + 1] : 0.f;
    const float bb0 = rb.bias ? rb.bias[j0] : 0.f, bb1 = rb.bias ? rb.bias[j0 + 1] : 0.f;
#pragma unroll
    for (int r = 0; r < kQRows; ++r) {
      const int rl = r0 + r;
      const float2 za = *reinterpret_cast<const float2*>(&Ca[rl * kQCLd + j0]);
      const float2 zb = *reinterpret_cast<const float2*>(&Cb[rl * kQCLd + j0]);
      float ya0 = za.x + ba0, ya1 = za.y + ba1;
      float yb0 = zb.x + bb0, yb1 = zb.y + bb1;
      if (ra.bias_ne && nes[0][rl]) {
        ya0 += ra.bias_ne[j0];
        ya1 += ra.bias_ne[j0 + 1];
      }
      if (rb.bias_ne && nes[1][rl]) {
        yb0 += rb.bias_ne[j0];
        yb1 += rb.bias_ne[j0 + 1];
      }
      activate_q(relu, l2, ya0, ya1);
      activate_q(relu, l2, yb0, yb1);
      float y0, y1;
      if (combine == GNNREC_ACC_MAX) {
        y0 = fmaxf(ya0, yb0);
        y1 = fmaxf(ya1, yb1);
      } else if (combine == GNNREC_ACC_ATTN_LAST) {
        // softmax over the two relations of s_r = a·y_r, as the single-relation launches'
        // online form: a first (max s_a, sum 1), then b rescales and normalises
        const float at0 = attn_vec[j0], at1 = attn_vec[j0 + 1];
        float sa = ya0 * at0 + ya1 * at1, sb = yb0 * at0 + yb1 * at1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          sa += __shfl_xor(sa, off);
          sb += __shfl_xor(sb, off);
        }
        const float mnew = fmaxf(sa, sb);
        const float keep = expf(sa - mnew), cnew = expf(sb - mnew);
        const float nrm = 1.f / (1.f * keep + cnew);
        y0 = (ya0 * keep + yb0 * cnew) * nrm;
        y1 = (ya1 * keep + yb1 * cnew) * nrm;
      } else {
        y0 = ya0 + yb0;
        y1 = ya1 + yb1;
      }
      if (out_div > 0.f) {
        y0 = y0 / out_div;
        y1 = y1 / out_div;
      }
      if (r < nv) {
        typedef float f32x2s __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(f32x2s{y0, y1},
                                    reinterpret_cast<f32x2s*>(out + (rbase + r) * ldo + j0));
      }
    }
    __syncthreads();  // the tile's LDS is free for the next one
  };

  // whole tiles from the row queue, or statically from this block's XCD's contiguous
  // eighth of the tiles (block-strided below 8 blocks); wave 0 draws, the block follows
  RqCursor cur;
  if (rq != nullptr && wave == 0) rq_begin(cur, rq);
  const int64_t tiles = (n_dst + kQT - 1) / kQT;
  const bool by_xcd = gridDim.x >= (unsigned)kRqHeads;
  const int xcd = by_xcd ? blockIdx.x % kRqHeads : 0;
  const int64_t per = by_xcd ? (int64_t)(gridDim.x - xcd + kRqHeads - 1) / kRqHeads
                             : (int64_t)gridDim.x;
  int64_t st = by_xcd ? tiles * xcd / kRqHeads + blockIdx.x / kRqHeads : (int64_t)blockIdx.x;
  const int64_t st_hi = by_xcd ? tiles * (xcd + 1) / kRqHeads : tiles;
  while (true) {
    if (wave == 0) {
      int64_t r0 = -1, r1 = 0;
      if (rq != nullptr) {
        if (!rq_next(cur, rq, n_dst, rq_ch, r0, r1)) r0 = -1;
      } else if (st < st_hi) {
        r0 = st * kQT;
        r1 = r0 + kQT < n_dst ? r0 + kQT : n_dst;
        st += per;
      }
      if (lane == 0) {
        blk_r[0] = r0;
        blk_r[1] = r1;
      }
    }
    __syncthreads();
    const int64_t r0 = blk_r[0], r1 = blk_r[1];
    __syncthreads();  // blk_r read by every wave before wave 0 may overwrite it
    if (r0 < 0) break;
    for (int64_t t0 = r0; t0 < r1; t0 += kQT) tile(t0, r1);
  }
  if (rq != nullptr) rq_finish(rq);
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_spmm_pair_f32(
    const int64_t* indptr_a, const int32_t* indices_a, const float* ew_a, int reduce_a,
    const float* bias_a, const float* bias_nonempty_a, const int64_t* indptr_b,
    const int32_t* indices_b, const float* ew_b, int reduce_b, const float* bias_b,
    const float* bias_nonempty_b, const float* X, int64_t n_src, int64_t ldx, const float* H,
    int64_t ldh, const float* WT4, int64_t n_dst, int64_t d, int epilogue,
    int combine, const float* attn_vec, float out_div, float* out, int64_t ldo, void* stream) {
  GNNREC_REQUIRE(d == kQD, "gnnrec_spmm_pair_f32: only d = %d (got %lld)", kQD, (long long)d);
  GNNREC_REQUIRE((reduce_a == GNNREC_REDUCE_SUM || reduce_a == GNNREC_REDUCE_MEAN) &&
                     (reduce_b == GNNREC_REDUCE_SUM || reduce_b == GNNREC_REDUCE_MEAN),
                 "gnnrec_spmm_pair_f32: both relations reduce by sum or mean");
  GNNREC_REQUIRE((epilogue & ~(GNNREC_EPI_RELU | GNNREC_EPI_L2NORM)) == 0,
                 "gnnrec_spmm_pair_f32: epilogue must be RELU|L2NORM");
  GNNREC_REQUIRE(combine == GNNREC_ACC_ADD || combine == GNNREC_ACC_MAX ||
                     combine == GNNREC_ACC_ATTN_LAST,
                 "gnnrec_spmm_pair_f32: combine must be GNNREC_ACC_ADD, _MAX or _ATTN_LAST");
  GNNREC_REQUIRE((combine == GNNREC_ACC_ATTN_LAST) == (attn_vec != nullptr),
                 "gnnrec_spmm_pair_f32: attn_vec goes with combine GNNREC_ACC_ATTN_LAST");
  GNNREC_REQUIRE(n_dst >= 0, "gnnrec_spmm_pair_f32: negative n_dst");
  if (n_dst == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr_a && indptr_b && X && H && out, "gnnrec_spmm_pair_f32: null pointer");
  GNNREC_REQUIRE(WT4 != nullptr, "gnnrec_spmm_pair_f32: null WT4");
  GNNREC_REQUIRE(aligned16(X) && aligned16(H) && aligned16(WT4) && ldx % 4 == 0 &&
                     ldh % 4 == 0 && ldo % 2 == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                 "gnnrec_spmm_pair_f32: X/H/W need 16-B aligned rows, out 8-B");
  const int64_t tiles = (n_dst + kQT - 1) / kQT;
  const int64_t cus = device_cus() - cu_reserve();
  int64_t blocks = 2 * (cus > 8 ? cus : 8);
  if (blocks > tiles) blocks = tiles;
  constexpr int rq_ch = 2 * kQT;  // rows per queue ticket (whole tiles)
  hipStream_t s = as_stream(stream);
  int ticket = -1;
  unsigned* rq = n_dst >= blocks * rq_ch * 4 ? rowq_slot(s, &ticket) : nullptr;
  const RawRel a{indptr_a, indices_a, ew_a, bias_a, bias_nonempty_a,
                 reduce_a == GNNREC_REDUCE_MEAN};
  const RawRel b{indptr_b, indices_b, ew_b, bias_b, bias_nonempty_b,
                 reduce_b == GNNREC_REDUCE_MEAN};
  const dim3 grid((unsigned)blocks), block(kQWaves * 64);
  GNNREC_REQUIRE(n_src >= 0, "gnnrec_spmm_pair_f32: negative n_src");
#define GNNREC_SPQ(WA_, WB_)                                                                 \
  hipLaunchKernelGGL((spmm_pair_mfma_kernel<WA_, WB_>), grid, block, 0, s, a, b, X, ldx, H, ldh, \
                     WT4, n_dst, epilogue, combine, attn_vec, out_div, out, ldo, rq, rq_ch)
  if (ew_a) {
    if (ew_b) GNNREC_SPQ(true, true);
    else GNNREC_SPQ(true, false);
  } else {
    if (ew_b) GNNREC_SPQ(false, true);
    else GNNREC_SPQ(false, false);
  }
#undef GNNREC_SPQ
  rowq_launched(ticket, s);
  return check_launch("gnnrec_spmm_pair_f32");
}
