// a1+a3 fused — neighbour aggregation with the SAGE projection in its epilogue:
//   out[v] (accum)= epi( h_self[v] · W_selfᵀ + agg(v) · W_neighᵀ ),
//   agg(v) = mean / sum / max over v's in-edges of X[src] (· w_e)
// for ConvLayer.forward's aggregation + projection (reference src/model.py:143-208,
// 226-235) and HeteroGraphConv's cross-relation sum/mean/max (:384-406).
//
// Why: the gather is HBM-bound (≈6.5 TB/s) and leaves the CU's VALU and LDS mostly
// idle, while the separate projection GEMM re-reads h_self and the aggregate from HBM,
// writes the output again and, run beside the next gather, competes with it for HBM.
// Here each wave owns ROWS destination rows at a time end to end: gather (the same
// gather_range / fixed xor-tree combine as spmm_csr_kernel, so the aggregate is
// bit-identical to the plain kernel's), then a 128×128 matvec per row on the VALU with
// both weight matrices resident in LDS (loaded once per persistent block), ReLU,
// zero-guarded row L2 norm, hetero accumulate, one 512-B store.  HBM per row: the
// gathered rows + h_self row + output row; no aggregate round trip, no GEMM launch.
//
// Shapes: d_neigh = d_self = N = 128 (the C4/C5 shapes); the wrapper falls back to
// spmm + gemm otherwise, and when the CSR has rows above the heavy-row split.
// LDS: W_selfᵀ, W_neighᵀ (2 × 64 KiB, k-major so a lane's two output columns are one
// ds_read_b64) + per wave ROWS × (agg, self) row slots read back as broadcasts.
#include "common.hpp"
#include "gather.hpp"
#include "rowq.hpp"
#include <cstdlib>
#include <type_traits>

namespace gnnrec {
namespace {

constexpr int kPD = 128;       // d_neigh = d_self = N
constexpr int kPWaves = 16;    // waves per block (one persistent block per CU)
constexpr int kPRows = 2;      // rows per wave per iteration (halves the LDS weight reads)
// rows per queue ticket (rowq.hpp): four iterations, ≈120 µs at C4 (a multiple of kPRows)
constexpr int kFusedChunk = 8;

// The per-row epilogue both fused kernels share: lane = output columns j0, j0+1 of `row`
// (y = the projected pre-activation incl. bias): ReLU, zero-guarded L2 norm over the 64
// lanes, the cross-relation accumulate (store / add / max / online-softmax attention),
// out_div, one float2 store per lane.  `valid` (wave-uniform) is false for padding rows
// past the range end: they take part in the shuffles, store nothing.
struct EpiArgs {
  bool relu, l2, attn;
  int accum;
  float out_div, a0, a1;
  float* attn_state;
  float* out;
  int64_t ldo;
  int j0;
};

// ReLU and the zero-guarded row L2 norm over the wave's 64 lanes (2 columns per lane)
__device__ __forceinline__ void activate(bool relu, bool l2, float& y0, float& y1) {
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

__device__ __forceinline__ void epilogue_row(const EpiArgs& e, int64_t row, bool valid,
                                             float y0, float y1) {
  activate(e.relu, e.l2, y0, y1);
  float keep = 0.f, nrm_attn = 1.f;
  if (e.attn) {  // online softmax over relations, score s = a . y (row-uniform)
    float sc = y0 * e.a0 + y1 * e.a1;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) sc += __shfl_xor(sc, off);
    float mnew = sc, snew = 1.f, cnew = 1.f;
    if (valid && e.accum != GNNREC_ACC_ATTN_FIRST) {
      const float2 st = reinterpret_cast<const float2*>(e.attn_state)[row];
      mnew = fmaxf(st.x, sc);
      keep = expf(st.x - mnew);
      cnew = expf(sc - mnew);
      snew = st.y * keep + cnew;
    }
    if (e.accum == GNNREC_ACC_ATTN_LAST) nrm_attn = 1.f / snew;
    if (valid && (threadIdx.x & 63) == 0)
      reinterpret_cast<float2*>(e.attn_state)[row] = make_float2(mnew, snew);
    y0 *= cnew;
    y1 *= cnew;
  }
  if (!valid) return;
  float2* p = reinterpret_cast<float2*>(e.out + row * e.ldo + e.j0);
  if (e.attn) {
    if (e.accum != GNNREC_ACC_ATTN_FIRST) {
      const float2 o = *p;
      y0 = o.x * keep + y0;
      y1 = o.y * keep + y1;
    }
    y0 *= nrm_attn;
    y1 *= nrm_attn;
  } else if (e.accum != GNNREC_ACC_STORE) {
    const float2 o = *p;
    if (e.accum == GNNREC_ACC_ADD) {
      y0 = o.x + y0;
      y1 = o.y + y1;
    } else {
      y0 = fmaxf(o.x, y0);
      y1 = fmaxf(o.y, y1);
    }
  }
  if (e.out_div > 0.f) {
    y0 = y0 / e.out_div;
    y1 = y1 / e.out_div;
  }
  typedef float f32x2s __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(f32x2s{y0, y1}, reinterpret_cast<f32x2s*>(p));  // (gather.hpp)
}

template <int REDUCE, bool WEIGHTED, int UNROLL>
__global__ __launch_bounds__(kPWaves * 64) void spmm_project_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx,
    const float* __restrict__ H, int64_t ldh, const float* __restrict__ WsT,
    const float* __restrict__ WnT, const float* __restrict__ bias,
    const float* __restrict__ bias_ne, int64_t n_dst, int epilogue, int accum, float out_div,
    const float* __restrict__ attn_vec, float* __restrict__ attn_state,
    float* __restrict__ out, int64_t ldo, unsigned* rq, int rq_ch) {
  __shared__ float Ws[kPD * kPD];
  __shared__ float Wn[kPD * kPD];
  __shared__ float slots[kPWaves][kPRows][2][kPD];
  for (int i = threadIdx.x; i < kPD * kPD / 4; i += kPWaves * 64) {
    reinterpret_cast<float4*>(Ws)[i] = reinterpret_cast<const float4*>(WsT)[i];
    reinterpret_cast<float4*>(Wn)[i] = reinterpret_cast<const float4*>(WnT)[i];
  }
  __syncthreads();

  constexpr int LPR = 32, VEC = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPR;
  const int col = (lane % LPR) * VEC;
  const int j0 = 2 * lane;  // this lane's two output columns
  const bool relu = epilogue & GNNREC_EPI_RELU;
  const bool l2 = epilogue & GNNREC_EPI_L2NORM;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const int64_t stride = (int64_t)gridDim.x * kPWaves * kPRows;
  const float b0 = bias ? bias[j0] : 0.f, b1 = bias ? bias[j0 + 1] : 0.f;
  const float c0 = bias_ne ? bias_ne[j0] : 0.f, c1 = bias_ne ? bias_ne[j0 + 1] : 0.f;
  const bool attn = accum >= GNNREC_ACC_ATTN_FIRST;
  const float a0 = attn ? attn_vec[j0] : 0.f, a1 = attn ? attn_vec[j0 + 1] : 0.f;
  const EpiArgs ep{relu, l2, attn, accum, out_div, a0, a1, attn_state, out, ldo, j0};

  // rows [row0, row0 + kPRows) of this wave, those at or past `lim` skipped
  auto step = [&](int64_t row0, int64_t lim) {
    bool nonempty[kPRows];
    // both rows' bounds (one load), first 64 indices and self rows are requested before
    // either row gathers: the second row's indptr -> indices chain hides under the first
    // row's gather (it is the fixed per-row cost that low-degree relations feel)
    const int nv = (int)(lim - row0 < kPRows ? lim - row0 : kPRows);  // valid rows, >= 1
    const int64_t ipl = lane <= nv ? ld_stream(indptr + row0 + lane) : 0;
    int64_t rb[kPRows + 1];
#pragma unroll
    for (int r = 0; r <= kPRows; ++r) rb[r] = __shfl(ipl, r <= nv ? r : nv);
    int pidx[kPRows];
    float4 hsr[kPRows];
#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      const bool valid = r < nv;  // uniform per wave
      pidx[r] = valid && lane < rb[r + 1] - rb[r] ? ld_stream(indices + rb[r] + lane) : 0;
      hsr[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid && grp == 1) hsr[r] = ld_stream4(H + (row0 + r) * ldh + col);
    }
#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      const bool valid = r < nv;  // uniform per wave
      const float4 hs = hsr[r];
      Frag<VEC> acc;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = init;
      int64_t deg = 0;
      if (valid) {
        const int64_t beg = rb[r], end = rb[r + 1];
        deg = end - beg;
        gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL, true>(beg, end, indices, ew, X, ldx,
                                                               col, true, lane, grp, acc, pidx[r]);
      }
      combine_groups<LPR, VEC, REDUCE>(acc);
      finalize<VEC, REDUCE>(acc, deg, 0);
      nonempty[r] = deg > 0;
      if (grp == 0)
        *reinterpret_cast<float4*>(&slots[wave][r][0][col]) =
            make_float4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
      else
        *reinterpret_cast<float4*>(&slots[wave][r][1][col]) = hs;
    }
    // the slots are written and read by this wave only: LDS is in order per wave, the
    // clobber keeps the compiler from hoisting the reads above the writes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    // bias: a folded NodeEmbedding's W_self·b; bias_ne: its W_neigh·b, which only
    // rows with at least one neighbour receive (the mean of an empty set is 0)
    float z[kPRows][2];
#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      z[r][0] = b0 + (nonempty[r] ? c0 : 0.f);
      z[r][1] = b1 + (nonempty[r] ? c1 : 0.f);
    }
#pragma unroll 2
    for (int k = 0; k < kPD; k += 4) {
      float4 a4[kPRows], s4[kPRows];
#pragma unroll
      for (int r = 0; r < kPRows; ++r) {
        a4[r] = *reinterpret_cast<const float4*>(&slots[wave][r][0][k]);
        s4[r] = *reinterpret_cast<const float4*>(&slots[wave][r][1][k]);
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const float2 ws = *reinterpret_cast<const float2*>(&Ws[(k + kk) * kPD + j0]);
        const float2 wn = *reinterpret_cast<const float2*>(&Wn[(k + kk) * kPD + j0]);
#pragma unroll
        for (int r = 0; r < kPRows; ++r) {
          const float s = kk == 0 ? s4[r].x : kk == 1 ? s4[r].y : kk == 2 ? s4[r].z : s4[r].w;
          const float a = kk == 0 ? a4[r].x : kk == 1 ? a4[r].y : kk == 2 ? a4[r].z : a4[r].w;
          z[r][0] = fmaf(s, ws.x, z[r][0]);
          z[r][0] = fmaf(a, wn.x, z[r][0]);
          z[r][1] = fmaf(s, ws.y, z[r][1]);
          z[r][1] = fmaf(a, wn.y, z[r][1]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slots free for the next rows

#pragma unroll
    for (int r = 0; r < kPRows; ++r) epilogue_row(ep, row0 + r, row0 + r < lim, z[r][0], z[r][1]);
  };

  if (rq != nullptr) {  // rows from the queue: blocks that start late take fewer
    rq_for_each(rq, n_dst, rq_ch, [&](int64_t r0, int64_t r1) {
      for (int64_t row0 = r0; row0 < r1; row0 += kPRows) step(row0, r1);
    });
    rq_finish(rq);
    return;
  }
  for (int64_t row0 = ((int64_t)blockIdx.x * kPWaves + wave) * kPRows; row0 < n_dst;
       row0 += stride)
    step(row0, n_dst);
}


// ---------------------------------------------------------------------------------------
// The same fused operation for LOW-DEGREE relations, projection on the MFMA.
//
// Why: the VALU kernel above re-reads both 64 KiB weight matrices from LDS for every 2
// rows, a fixed per-row cost that the gather hides at C4's 50 edges/row but that bounds
// a 10-edges/row relation (C5 bought-by: 18.0 ms fused vs 7.6 ms gather + 7.1 ms GEMM).
// Here a block of 8 waves owns 32-row tiles: the waves gather 4 rows each (the same
// gather_range / xor tree as spmm_csr_kernel, so the aggregate is bit-identical) into an
// LDS tile A = [h_self | agg] (32 × 256 fp32), then 32×128 = A · [W_self | W_neigh]ᵀ
// runs as v_mfma_f32_32x32x2_f32: wave w owns output columns 32·(w&3) and K half (w>>2)
// (W_self or W_neigh), i.e. 64 B operands per lane, re-read from L2 per tile by buffer
// loads (held across the gather they would spill: 128 VGPRs is the budget at two 8-wave
// blocks per CU) — the weights cross the CU once per 32 rows instead of once per 2.  Each
// lane half h of an MFMA consumes k ∈ [64h, 64h+64) of its K half (a fixed permutation of
// the summation order; vectorised ds_read_b128 of A).  The two K halves meet in LDS, then
// each wave finishes 4 rows with the shared epilogue.  Two blocks per CU (≈ 67 KiB LDS
// each; HIP's second launch-bounds argument is waves per SIMD), so one block's MFMA phase
// runs under the other's gather.
//
// The gather runs the wave's 4 rows in lockstep (all 4 rows' index loads, then steps of
// 2·LU neighbours of every row), so a 10-edge row does not pay its own index -> row round
// trips; the W operands stream from L2 in chunks of 16 under the MFMAs.
//
// PRE (W_neighT = NULL): the source rows arrive already projected (Y = X·W_neighᵀ, linear
// reductions only), the neighbour term is their aggregate, read from the A tile in the
// epilogue, and the 8 waves split the self half's K = 128 (two 32-row·32-col partials).
//
// Measured (C5 bought-by, 10M rows × 10 edges, tools/probe_c5.py, one box): 12.8–13.1 ms
// (13.1 with the rows gathered one after another), PRE 10.6 ms + 0.38 ms for the 1M-row
// source projection; 18.0 ms for the VALU kernel; 7.6 + 7.1 ms for gather + GEMM launched
// back to back.  Timing builds (round 2, tools/EXPERIMENTS.md): the GEMM phase alone (no neighbour
// loads) takes 7.3–7.8 ms — the fp32 MFMA at ≈0.6 of its peak, as in the plain GEMM
// (profiles/r02_gemm_experiments.md) — so the two phases overlap by ≈2 ms only.  Not kept
// (same session A/B): 64-row tiles (C in the A tile's LDS, 12.6–12.7 ms, within noise of
// 32), all 64 W operands up front (14.7 vs 13.1 ms once the lockstep gather holds its
// registers), three blocks per CU at 80 VGPRs (16.4 ms: spills), LU = 4 (spills).  A
// variant splitting the block into 8 gather waves and 8 MFMA waves (weights resident in
// the MFMA waves' registers, one barrier per pipelined step) took 17–22 ms: 8 gathering
// waves per CU cannot keep HBM busy at 10 edges per row.  The sharded pass fuses such a
// relation only in the PRE form (else gather + GEMM on the side stream).
constexpr int kSppU = 4;   // the VALU kernel's gather wave-instructions in flight per lane
constexpr int kSpmU = 4;   // the MFMA kernel's, rows > 64 edges
constexpr int kSpmLU = 2;  // lockstep gather: steps of 2·LU neighbours of 4 rows at once
constexpr int kSpmWC = 16; // W operands per chunk (64 — all loaded up front — measured slower)
constexpr int kSpmEU = 4;  // epilogue rows unrolled
constexpr int kMT = 32;                  // rows per tile
constexpr int kMB = kMT / 32;            // 32-row MFMA blocks per tile
constexpr int kMWaves = 8;               // waves per block
constexpr int kMRows = kMT / kMWaves;    // rows gathered per wave per tile
constexpr int kALd = 2 * kPD + 4;        // A tile row stride (floats): conflict-free b128 reads
constexpr int kCLd = kPD + 8;            // C tile row stride: the two lane halves' stores
                                         // land on disjoint banks
constexpr int kALds = kMT * kALd;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int REDUCE, bool WEIGHTED, int UNROLL, bool PRE>
__global__ __launch_bounds__(kMWaves * 64, 4) void spmm_project_mfma_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx,
    const float* __restrict__ H, int64_t ldh, const float* __restrict__ WsT,
    const float* __restrict__ WnT, const float* __restrict__ bias,
    const float* __restrict__ bias_ne, int64_t n_dst, int epilogue, int accum, float out_div,
    const float* __restrict__ attn_vec, float* __restrict__ attn_state,
    float* __restrict__ out, int64_t ldo, unsigned* rq, int rq_ch) {
  __shared__ float lds[kALds + 2 * kMT * kCLd];
  __shared__ int nes[kMT];
  __shared__ int64_t blk_r[2];
  float* const As = lds;
  float* const Cs0 = lds + kALds;
  float* const Cs1 = Cs0 + kMT * kCLd;

  constexpr int LPR = 32, VEC = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPR;
  const int li = lane & 31, bh = lane >> 5;
  const int col = li * VEC;
  const int j0 = 2 * lane;
  const int cb = wave & 3, kh = wave >> 2;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const bool attn = accum >= GNNREC_ACC_ATTN_FIRST;
  const float a0 = attn ? attn_vec[j0] : 0.f, a1 = attn ? attn_vec[j0 + 1] : 0.f;
  const EpiArgs ep{(epilogue & GNNREC_EPI_RELU) != 0, (epilogue & GNNREC_EPI_L2NORM) != 0,
                   attn, accum, out_div, a0, a1, attn_state, out, ldo, j0};

  // B operands: lane supplies Wᵀ[k][n], k = 64·bh + i of this wave's K half, n = 32·cb + li
  // (PRE: the self half alone, split over the two wave halves: k = 64·kh + 32·bh + i).
  // Buffer loads: one 32-bit per-lane offset plus an immediate row offset, instead of 64
  // hoisted 64-bit addresses (which the compiler spills)
  constexpr int kKL = PRE ? 32 : 64;  // K per lane half
  const float* WTb = (kh && !PRE) ? WnT : WsT;
  const uint64_t wbase = ((uint64_t)__builtin_amdgcn_readfirstlane(
                              (unsigned)((uintptr_t)WTb >> 32)) << 32) |
                         (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)WTb);
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(wbase), 0,
                                                       kPD * kPD * 4, 0x00020000);
  const int wvoff = ((PRE ? 64 * kh + 32 * bh : 64 * bh) * kPD + 32 * cb + li) * 4;

  // one tile: rows [t0, min(t0 + kMT, lim)); every wave of the block takes part
  auto tile = [&](int64_t t0, int64_t lim) __attribute__((always_inline)) {
    const int64_t rbase = t0 + wave * kMRows;
    const int64_t left = lim - rbase;
    const int nv = (int)(left <= 0 ? 0 : left < kMRows ? left : kMRows);
    // the rows' bounds in one load (nv == 0: rows past the range end — nothing is read,
    // the tile rows stay zero); self rows two per instruction, after the gather
    const int64_t ipl = nv > 0 && lane <= nv ? indptr[rbase + lane] : 0;
    auto bound = [&](int r) { return __shfl(ipl, r <= nv ? r : nv); };
    auto self_rows = [&](int q) {  // lanes of half bh: self row 2q + bh
      const int rl = 2 * q + bh;
      return rl < nv ? *reinterpret_cast<const float4*>(H + (rbase + rl) * ldh + col)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    // Lockstep gather, 4 rows at a time: their bounds and first 64 indices are requested up
    // front, then every step issues the loads of all 4 rows (4·LU·2 source rows in flight
    // per wave), so a 10-edge row does not pay its own index -> row round trips.  Each
    // row's neighbours are still summed by group in gather_range's order
    // (k = j + u·NPI + grp, ascending — the same sequence for any LU): the same aggregate
    // bits.  Rows with more than 64 edges take gather_range row by row.
    constexpr int NPI = kWave / LPR, U = kSpmLU, kLR = 4;
#pragma unroll
    for (int g = 0; g < kMRows; g += kLR) {
      int ridx[kLR];
      float rwt[kLR];
      int dg[kLR];
      int dmax = 0;
#pragma unroll
      for (int r = 0; r < kLR; ++r) {
        const int64_t b = bound(g + r);
        dg[r] = g + r < nv ? (int)(bound(g + r + 1) - b) : 0;
        ridx[r] = lane < dg[r] ? ld_stream(indices + b + lane) : 0;
        rwt[r] = 0.f;
        if constexpr (WEIGHTED) rwt[r] = lane < dg[r] ? ld_stream(ew + b + lane) : 0.f;
        dmax = dg[r] > dmax ? dg[r] : dmax;
      }
      Frag<VEC> acc[kLR];
#pragma unroll
      for (int r = 0; r < kLR; ++r)
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[r].v[v] = init;
      if (dmax <= 64) {
        for (int j = 0; j < dmax; j += NPI * U) {
          Frag<VEC> val[kLR][U];
          bool ok[kLR][U];
#pragma unroll
          for (int r = 0; r < kLR; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int k = j + u * NPI + grp;
              ok[r][u] = k < dg[r];
              const int src = edge_bcast<NPI>(ridx[r], j + u * NPI, grp);
              if (ok[r][u]) {
                load_frag<VEC>(val[r][u], X + (int64_t)src * ldx + col);
              } else {
#pragma unroll
                for (int v = 0; v < VEC; ++v) val[r][u].v[v] = 0.f;
              }
            }
#pragma unroll
          for (int r = 0; r < kLR; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
              float w = 1.f;
              if constexpr (WEIGHTED) w = edge_bcast<NPI>(rwt[r], j + u * NPI, grp);
#pragma unroll
              for (int v = 0; v < VEC; ++v) {
                const float m = WEIGHTED ? val[r][u].v[v] * w : val[r][u].v[v];
                if constexpr (REDUCE == GNNREC_REDUCE_MAX) {
                  if (ok[r][u]) acc[r].v[v] = fmaxf(acc[r].v[v], m);
                } else {
                  acc[r].v[v] += m;
                }
              }
            }
        }
      } else {
#pragma unroll
        for (int r = 0; r < kLR; ++r)
          if (g + r < nv)
            gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL, true>(
                bound(g + r), bound(g + r + 1), indices, ew, X, ldx, col, true, lane, grp,
                acc[r], ridx[r]);
      }
#pragma unroll
      for (int r = 0; r < kLR; ++r) {
        combine_groups<LPR, VEC, REDUCE>(acc[r]);
        finalize<VEC, REDUCE>(acc[r], dg[r], 0);
        const int rl = wave * kMRows + g + r;
        if (grp == 0)
          *reinterpret_cast<float4*>(&As[rl * kALd + kPD + col]) =
              make_float4(acc[r].v[0], acc[r].v[1], acc[r].v[2], acc[r].v[3]);
        if (lane == 0) nes[rl] = dg[r] > 0;
      }
    }
#pragma unroll
    for (int q = 0; q < kMRows / 2; ++q)
      *reinterpret_cast<float4*>(&As[(wave * kMRows + 2 * q + bh) * kALd + col]) = self_rows(q);
    __syncthreads();

    // C_kh[rows 32·b.., 32 × 32 block cb] = A[:, K half kh] · Wᵀ[K half kh, block cb], the
    // W operands loaded once for the tile's kMB row blocks
    // W operands stream in 4 chunks of 16 (double-buffered, the next chunk's loads in
    // flight under this chunk's MFMAs) instead of 64 live registers
    constexpr int kWC = kSpmWC;
    float bw[2][kWC];
    auto load_w = [&](float* dst, int i0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < kWC; ++i)
        dst[i] = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(wrsrc, wvoff, (i0 + i) * kPD * 4, 0));
    };
    f32x16 c[kMB];
#pragma unroll
    for (int b = 0; b < kMB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) c[b][v] = 0.f;
    const float* ap = As + li * kALd + (PRE ? 64 * kh + 32 * bh : kh * kPD + 64 * bh);
    {
      load_w(bw[0], 0);
#pragma unroll
      for (int ch = 0; ch < kKL / kWC; ++ch) {
        if (ch + 1 < kKL / kWC) load_w(bw[(ch + 1) & 1], (ch + 1) * kWC);
        __builtin_amdgcn_sched_barrier(0);
        const float* w = bw[ch & 1];
#pragma unroll
        for (int i = 0; i < kWC; i += 4) {
#pragma unroll
          for (int b = 0; b < kMB; ++b) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(ap + 32 * b * kALd + ch * kWC + i);
            c[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0], w[i], c[b], 0, 0, 0);
            c[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1], w[i + 1], c[b], 0, 0, 0);
            c[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2], w[i + 2], c[b], 0, 0, 0);
            c[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[3], w[i + 3], c[b], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // D map of the 32x32 MFMA: col = lane & 31, row = (v & 3) + 8 (v >> 2) + 4 h
    float* cp = (kh ? Cs1 : Cs0) + 32 * cb + li;
#pragma unroll
    for (int b = 0; b < kMB; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        cp[(32 * b + (v & 3) + 8 * (v >> 2) + 4 * bh) * kCLd] = c[b][v];
    __syncthreads();

#pragma unroll kSpmEU
    for (int r = 0; r < kMRows; ++r) {
      const int rl = wave * kMRows + r;
      const float2 s2 = *reinterpret_cast<const float2*>(&Cs0[rl * kCLd + j0]);
      const float2 n2 = *reinterpret_cast<const float2*>(&Cs1[rl * kCLd + j0]);
      float z0 = s2.x + n2.x, z1 = s2.y + n2.y;
      if constexpr (PRE) {  // + the aggregate of the pre-projected rows
        const float2 g2 = *reinterpret_cast<const float2*>(&As[rl * kALd + kPD + j0]);
        z0 += g2.x;
        z1 += g2.y;
      }
      if (bias) {
        z0 = bias[j0] + z0;
        z1 = bias[j0 + 1] + z1;
      }
      if (bias_ne && nes[rl]) {
        z0 = bias_ne[j0] + z0;
        z1 = bias_ne[j0 + 1] + z1;
      }
      epilogue_row(ep, rbase + r, r < nv, z0, z1);
    }
    __syncthreads();  // As / Cs / nes free for the next tile
  };

  // chunks of rows come from the queue (blocks that start late, behind another kernel,
  // take fewer) or, statically, one tile at a time from this block's XCD's contiguous
  // eighth of the tiles (blocks are dispatched round-robin over the 8, so each XCD's L2
  // sees contiguous indptr / H / out rows); wave 0 draws and publishes each chunk, and
  // the whole block processes it — one call site of the tile body
  RqCursor cur;
  if (rq != nullptr && wave == 0) rq_begin(cur, rq);
  const int64_t tiles = (n_dst + kMT - 1) / kMT;
  // a grid of fewer than 8 blocks (small relations) leaves some XCDs without a block: then
  // a plain block-strided walk, so no eighth of the tiles is left without an owner
  const bool by_xcd = gridDim.x >= (unsigned)kRqHeads;
  const int xcd = by_xcd ? blockIdx.x % kRqHeads : 0;
  const int64_t per = by_xcd ? (int64_t)(gridDim.x - xcd + kRqHeads - 1) / kRqHeads  // blocks on xcd
                             : (int64_t)gridDim.x;
  int64_t st = by_xcd ? tiles * xcd / kRqHeads + blockIdx.x / kRqHeads : (int64_t)blockIdx.x;
  const int64_t st_hi = by_xcd ? tiles * (xcd + 1) / kRqHeads : tiles;
  while (true) {
    if (wave == 0) {
      int64_t r0 = -1, r1 = 0;
      if (rq != nullptr) {
        if (!rq_next(cur, rq, n_dst, rq_ch, r0, r1)) r0 = -1;
      } else if (st < st_hi) {
        r0 = st * kMT;
        r1 = r0 + kMT < n_dst ? r0 + kMT : n_dst;
        st += per;
      }
      if (lane == 0) {
        blk_r[0] = r0;
        blk_r[1] = r1;
      }
    }
    __syncthreads();
    const int64_t r0 = blk_r[0], r1 = blk_r[1];
    if (r0 < 0) break;
    for (int64_t t0 = r0; t0 < r1; t0 += kMT) tile(t0, r1);  // ends with a barrier
  }
  if (rq != nullptr) rq_finish(rq);
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_spmm_project_f32(const int64_t* indptr, const int32_t* indices,
                                       const float* ew, const float* X, int64_t ldx,
                                       const float* H, int64_t ldh, const float* W_selfT,
                                       const float* W_neighT, const float* bias,
                                       const float* bias_nonempty, int64_t n_dst, int64_t d,
                                       int reduce, int epilogue, int accum, float out_div,
                                       const float* attn_vec, float* attn_state, float* out,
                                       int64_t ldo, void* stream) {
  GNNREC_REQUIRE(d == kPD, "gnnrec_spmm_project_f32: only d = %d (got %lld)", kPD,
                 (long long)d);
  GNNREC_REQUIRE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN ||
                     reduce == GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_project_f32: unknown reduce %d", reduce);
  GNNREC_REQUIRE((epilogue & ~(GNNREC_EPI_RELU | GNNREC_EPI_L2NORM)) == 0,
                 "gnnrec_spmm_project_f32: epilogue must be RELU|L2NORM");
  GNNREC_REQUIRE(accum >= GNNREC_ACC_STORE && accum <= GNNREC_ACC_ATTN_LAST,
                 "gnnrec_spmm_project_f32: unknown accumulate mode %d", accum);
  GNNREC_REQUIRE(accum < GNNREC_ACC_ATTN_FIRST || (attn_vec && attn_state),
                 "gnnrec_spmm_project_f32: attention accumulation needs attn_vec, attn_state");
  GNNREC_REQUIRE(n_dst >= 0, "gnnrec_spmm_project_f32: negative n_dst");
  if (n_dst == 0) return GNNREC_OK;
  GNNREC_REQUIRE(W_neighT, "gnnrec_spmm_project_f32: W_neighT = NULL (pre-projected source "
                           "rows) is gnnrec_spmm_project_mfma_f32's form");
  GNNREC_REQUIRE(indptr && X && H && W_selfT && out, "gnnrec_spmm_project_f32: null pointer");
  GNNREC_REQUIRE(aligned16(X) && aligned16(H) && aligned16(W_selfT) && aligned16(W_neighT) &&
                     ldx % 4 == 0 && ldh % 4 == 0 && ldo % 2 == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                 "gnnrec_spmm_project_f32: X/H/W need 16-B aligned rows, out 8-B");
  // one persistent block per CU, minus the CUs reserved for concurrent kernels
  const int64_t per_block = (int64_t)kPWaves * kPRows;
  int64_t blocks = (n_dst + per_block - 1) / per_block;
  const int64_t cus = device_cus() - cu_reserve();
  if (blocks > (cus > 8 ? cus : 8)) blocks = cus > 8 ? cus : 8;
  // queued rows when every wave has several tickets of work
  const int rq_ch = kFusedChunk;
  hipStream_t s = as_stream(stream);
  int ticket = -1;
  unsigned* rq = n_dst >= blocks * kPWaves * rq_ch * 4 ? rowq_slot(s, &ticket) : nullptr;
  const dim3 grid((unsigned)blocks), block(kPWaves * 64);
#define GNNREC_SPP(R, W)                                                                      \
  hipLaunchKernelGGL((spmm_project_kernel<R, W, kSppU>), grid, block, 0, s, indptr, indices, ew, \
                     X, ldx, H, ldh, W_selfT, W_neighT, bias, bias_nonempty, n_dst, epilogue,    \
                     accum, out_div, attn_vec, attn_state, out, ldo, rq, rq_ch)
  if (ew) {
    if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPP(GNNREC_REDUCE_SUM, true);
    else if (reduce == GNNREC_REDUCE_MEAN) GNNREC_SPP(GNNREC_REDUCE_MEAN, true);
    else GNNREC_SPP(GNNREC_REDUCE_MAX, true);
  } else {
    if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPP(GNNREC_REDUCE_SUM, false);
    else if (reduce == GNNREC_REDUCE_MEAN) GNNREC_SPP(GNNREC_REDUCE_MEAN, false);
    else GNNREC_SPP(GNNREC_REDUCE_MAX, false);
  }
#undef GNNREC_SPP
  rowq_launched(ticket, s);
  return check_launch("gnnrec_spmm_project_f32");
}

extern "C" int gnnrec_spmm_project_mfma_f32(const int64_t* indptr, const int32_t* indices,
                                            const float* ew, const float* X, int64_t ldx,
                                            const float* H, int64_t ldh, const float* W_selfT,
                                            const float* W_neighT, const float* bias,
                                            const float* bias_nonempty, int64_t n_dst,
                                            int64_t d, int reduce, int epilogue, int accum,
                                            float out_div, const float* attn_vec,
                                            float* attn_state, float* out, int64_t ldo,
                                            void* stream) {
  GNNREC_REQUIRE(d == kPD, "gnnrec_spmm_project_mfma_f32: only d = %d (got %lld)", kPD,
                 (long long)d);
  GNNREC_REQUIRE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN ||
                     reduce == GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_project_mfma_f32: unknown reduce %d", reduce);
  GNNREC_REQUIRE((epilogue & ~(GNNREC_EPI_RELU | GNNREC_EPI_L2NORM)) == 0,
                 "gnnrec_spmm_project_mfma_f32: epilogue must be RELU|L2NORM");
  GNNREC_REQUIRE(accum >= GNNREC_ACC_STORE && accum <= GNNREC_ACC_ATTN_LAST,
                 "gnnrec_spmm_project_mfma_f32: unknown accumulate mode %d", accum);
  GNNREC_REQUIRE(accum < GNNREC_ACC_ATTN_FIRST || (attn_vec && attn_state),
                 "gnnrec_spmm_project_mfma_f32: attention accumulation needs attn_vec, "
                 "attn_state");
  GNNREC_REQUIRE(n_dst >= 0, "gnnrec_spmm_project_mfma_f32: negative n_dst");
  if (n_dst == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr && X && H && W_selfT && out,
                 "gnnrec_spmm_project_mfma_f32: null pointer");
  // W_neighT == NULL: X holds pre-projected source rows (X·W_neighᵀ), the neighbour half
  // is their aggregate itself — linear reductions only
  const bool pre = W_neighT == nullptr;
  GNNREC_REQUIRE(!pre || reduce != GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_project_mfma_f32: pre-projected rows (W_neighT = NULL) need a "
                 "sum or mean reduce");
  GNNREC_REQUIRE(aligned16(X) && aligned16(H) && aligned16(W_selfT) &&
                     (pre || aligned16(W_neighT)) && ldx % 4 == 0 && ldh % 4 == 0 &&
                     ldo % 2 == 0 && (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                 "gnnrec_spmm_project_mfma_f32: X/H/W need 16-B aligned rows, out 8-B");
  // two persistent 8-wave blocks per CU, minus the CUs reserved for concurrent kernels
  const int64_t tiles = (n_dst + kMT - 1) / kMT;
  const int64_t cus = device_cus() - cu_reserve();
  int64_t blocks = 2 * (cus > 8 ? cus : 8);
  if (blocks > tiles) blocks = tiles;
  constexpr int rq_ch = 2 * kMT;  // rows per queue ticket (whole tiles)
  hipStream_t s = as_stream(stream);
  int ticket = -1;
  unsigned* rq = n_dst >= blocks * rq_ch * 4 ? rowq_slot(s, &ticket) : nullptr;
  const dim3 grid((unsigned)blocks), block(kMWaves * 64);
#define GNNREC_SPM(R, W, P)                                                                     \
  hipLaunchKernelGGL((spmm_project_mfma_kernel<R, W, kSpmU, P>), grid, block, 0, s,      \
                     indptr, indices, ew, X, ldx, H, ldh, W_selfT, W_neighT, bias,              \
                     bias_nonempty, n_dst, epilogue, accum, out_div, attn_vec, attn_state, out, \
                     ldo, rq, rq_ch)
  if (pre) {
    if (ew) {
      if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPM(GNNREC_REDUCE_SUM, true, true);
      else GNNREC_SPM(GNNREC_REDUCE_MEAN, true, true);
    } else {
      if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPM(GNNREC_REDUCE_SUM, false, true);
      else GNNREC_SPM(GNNREC_REDUCE_MEAN, false, true);
    }
  } else if (ew) {
    if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPM(GNNREC_REDUCE_SUM, true, false);
    else if (reduce == GNNREC_REDUCE_MEAN) GNNREC_SPM(GNNREC_REDUCE_MEAN, true, false);
    else GNNREC_SPM(GNNREC_REDUCE_MAX, true, false);
  } else {
    if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPM(GNNREC_REDUCE_SUM, false, false);
    else if (reduce == GNNREC_REDUCE_MEAN) GNNREC_SPM(GNNREC_REDUCE_MEAN, false, false);
    else GNNREC_SPM(GNNREC_REDUCE_MAX, false, false);
  }
#undef GNNREC_SPM
  rowq_launched(ticket, s);
  return check_launch("gnnrec_spmm_project_mfma_f32");
}

// ---------------------------------------------------------------------------------------
// Two pre-projected relations into one destination type in one launch:
//   out[v] = combine( epi(h[v]·W_aᵀ + agg_a(v) + b_a [+ bne_a]),
//                     epi(h[v]·W_bᵀ + agg_b(v) + b_b [+ bne_b]) ) / out_div
// agg_r = sum / mean over relation r's in-edges of Y_r = X_r·W_neigh,rᵀ (pre-projected
// source rows), combine = + (HeteroGraphConv sum / mean), max, or the per-relation
// attention softmax of s_r = a·y_r (the build-defined C5 aggregate).  For C5's user side
// (clicked-by, 40 edges/row, and bought-by, 10 edges/row, both from the 1M-row item
// table): the h_self row is read once instead of twice, the output written once instead
// of stored and read-modified-written, and the two gathers share the waves — the
// launch streams 50 source rows per destination row and stays HBM-bound.  The self
// halves of both relations are the 2 × 128×128 matvec per row (the same VALU work per
// row as the single-relation kernel's W_self + W_neigh), both W_selfᵀ resident in LDS.
// The aggregates never touch LDS: the wave's float4-per-lane fragment is turned into
// this lane's two output columns by four shuffles.
namespace gnnrec {
namespace {

// waves per (one-per-CU) block: 12 waves at U = 8-10 took 59.5 ms, 8 waves at U = 12-16
// 75 ms (vs 38.2): the wave count, not the loads in flight per wave, sets this kernel's rate
constexpr int kP2Waves = 16;
// gather wave-instructions in flight per lane (C5: 5 beats 4 by ≈0.6 ms; 6 and 8 slow down)
constexpr int kP2U = 5;

struct PreRel {
  const int64_t* indptr;
  const int32_t* indices;
  const float* ew;
  const float* Y;
  int64_t ldy;
  const float* bias_ne;
  int mean;
};

// ---- each step's row heads prefetched one step ahead ------------------------------------
// A wave that takes 2 rows at a time and gathers both relations of each (the round-2 form,
// tools/EXPERIMENTS.md) spent 64 % of its wave cycles parked on s_waitcnt (DESIGN.md §9 item
// 8): every step of 2 rows opens with two dependent round trips — indptr, then the first
// indices of both relations — before the first source row can be requested.  Here a wave
// knows its NEXT row pair while it works on the current one (the static walk, or the row
// queue's chunk / next ticket), so during step i it
//   * loads step i+1's bounds (indptr of both relations) into registers right at the start
//     (they arrive under step i's gathers) and parks them in its LDS area, and
//   * DMAs step i+1's first 48 indices of every (row, relation) straight into LDS with
//     global_load_lds (no registers live across the matvec: the earlier register-carried
//     form spilled to scratch and ran at 73 ms),
// so step i+1 starts gathering immediately from LDS-resident heads.  A row's later index
// windows (past 48 edges) load as before.  Summation order per row is gather_range's: the
// aggregate bits equal spmm_csr_kernel's.
// LDS: 2 x 64 KiB weights + 16 KiB self-row slots + 16 waves x (4 x 192 B index windows +
// 48 B bounds) = 156.75 KiB of the CU's 160.
constexpr int kP2Win = 48;  // prefetched indices per (row, relation)

__device__ __forceinline__ void dma4(const int32_t* src, int32_t* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
#endif
}

// the row pairs of one wave, in order: the static grid-stride walk, or the row queue's chunks
struct PairWalk {
  RqCursor c;
  int64_t pos, c1;
  bool queued;
};

__device__ __forceinline__ bool walk_next(PairWalk& w, unsigned* rq, int64_t n_dst, int rq_ch,
                                          int64_t stride, int64_t& row0, int64_t& lim) {
  if (!w.queued) {
    if (w.pos >= n_dst) return false;
    row0 = w.pos;
    lim = n_dst;
    w.pos += stride;
    return true;
  }
  if (w.pos >= w.c1) {
    int64_t r0, r1;
    if (!rq_next(w.c, rq, n_dst, rq_ch, r0, r1)) return false;
    w.pos = r0;
    w.c1 = r1;
  }
  row0 = w.pos;
  lim = w.c1;
  w.pos += kPRows;
  return true;
}

// NT: the source rows of relation a (1) or b (2) loaded non-temporally, so the other
// relation's pre-projected table keeps the caches (0: both temporal)
template <bool WA, bool WB, int NT = 0>
__global__ __launch_bounds__(kP2Waves * 64) void spmm_project2_pipe_kernel(
    PreRel ra, PreRel rb, const float* __restrict__ H, int64_t ldh,
    const float* __restrict__ WaT, const float* __restrict__ WbT,
    const float* __restrict__ bias_a, const float* __restrict__ bias_b, int64_t n_dst,
    int epilogue, int combine, const float* __restrict__ attn_vec, float out_div,
    float* __restrict__ out, int64_t ldo, unsigned* rq, int rq_ch) {
  __shared__ float Wa[kPD * kPD];
  __shared__ float Wb[kPD * kPD];
  __shared__ float slots[kP2Waves][kPRows][kPD];
  __shared__ int32_t win[kP2Waves][2][kPRows][kP2Win];  // [wave][relation][row] first indices
  __shared__ int64_t bnd[kP2Waves][2][kPRows + 1];      // [wave][relation] row bounds
  for (int i = threadIdx.x; i < kPD * kPD / 4; i += kP2Waves * 64) {
    reinterpret_cast<float4*>(Wa)[i] = reinterpret_cast<const float4*>(WaT)[i];
    reinterpret_cast<float4*>(Wb)[i] = reinterpret_cast<const float4*>(WbT)[i];
  }
  __syncthreads();

  constexpr int LPR = 32, VEC = 4, U = kP2U, NPI = kWave / LPR;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPR;
  const int col = (lane % LPR) * VEC;
  const int j0 = 2 * lane;
  const bool relu = epilogue & GNNREC_EPI_RELU;
  const bool l2 = epilogue & GNNREC_EPI_L2NORM;
  const int64_t stride = (int64_t)gridDim.x * kP2Waves * kPRows;
  const float ba0 = bias_a ? bias_a[j0] : 0.f, ba1 = bias_a ? bias_a[j0 + 1] : 0.f;
  const float bb0 = bias_b ? bias_b[j0] : 0.f, bb1 = bias_b ? bias_b[j0 + 1] : 0.f;
  const float ca0 = ra.bias_ne ? ra.bias_ne[j0] : 0.f, ca1 = ra.bias_ne ? ra.bias_ne[j0 + 1] : 0.f;
  const float cb0 = rb.bias_ne ? rb.bias_ne[j0] : 0.f, cb1 = rb.bias_ne ? rb.bias_ne[j0 + 1] : 0.f;
  const float at0 = attn_vec ? attn_vec[j0] : 0.f, at1 = attn_vec ? attn_vec[j0 + 1] : 0.f;

  // bounds of rows [row0, row0 + nv) of both relations: lanes 0..nv hold relation a's,
  // lanes 32..32+nv relation b's (one load instruction each, no wait)
  auto load_bounds = [&](int64_t row0, int nv) __attribute__((always_inline)) {
    const int l = lane & 31;
    const int64_t* ip = lane < 32 ? ra.indptr : rb.indptr;
    return l <= nv ? ld_stream(ip + row0 + l) : (int64_t)0;
  };
  // park them in LDS and DMA the first kP2Win indices of every (row, relation)
  auto stage_heads = [&](int64_t bv, int nv) __attribute__((always_inline)) {
    int64_t ba[kPRows + 1], bb[kPRows + 1];
#pragma unroll
    for (int i = 0; i <= kPRows; ++i) {
      ba[i] = __shfl(bv, i <= nv ? i : nv);
      bb[i] = __shfl(bv, 32 + (i <= nv ? i : nv));
    }
    if (lane <= kPRows) {
      bnd[wave][0][lane] = ba[lane <= nv ? lane : nv];
      bnd[wave][1][lane] = bb[lane <= nv ? lane : nv];
    }
#pragma unroll
    for (int i = 0; i < kPRows; ++i) {
      if (i < nv) {
        if (lane < ba[i + 1] - ba[i] && lane < kP2Win)
          dma4(ra.indices + ba[i] + lane, &win[wave][0][i][0]);
        if (lane < bb[i + 1] - bb[i] && lane < kP2Win)
          dma4(rb.indices + bb[i] + lane, &win[wave][1][i][0]);
      }
    }
  };
  // relation r's aggregate of row i (bounds beg, end; its first kP2Win indices in LDS)
  auto gather_row = [&](const PreRel& r, auto weighted, auto nt, int64_t beg, int64_t end,
                        int pre_idx, Frag<VEC>& acc) __attribute__((always_inline)) {
    constexpr bool W = decltype(weighted)::value;
    constexpr bool NTR = decltype(nt)::value;
    int64_t base = beg;
    int wlen = kP2Win;
    while (base < end) {
      const int cnt = (int)((end - base) < wlen ? (end - base) : wlen);
      const int myidx = base == beg ? pre_idx : (lane < cnt ? ld_stream(r.indices + base + lane) : 0);
      float myw = 0.f;
      if constexpr (W) myw = lane < cnt ? ld_stream(r.ew + base + lane) : 0.f;
      for (int j = 0; j < cnt; j += NPI * U) {
        Frag<VEC> val[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = j + u * NPI + grp;
          ok[u] = k < cnt;
          const int src = edge_bcast<NPI>(myidx, j + u * NPI, grp);
          if (ok[u]) {
            if constexpr (NTR) {
              const float4 t = ld_stream4(r.Y + (int64_t)src * r.ldy + col);
              val[u].v[0] = t.x; val[u].v[1] = t.y; val[u].v[2] = t.z; val[u].v[3] = t.w;
            } else {
              load_frag<VEC>(val[u], r.Y + (int64_t)src * r.ldy + col);
            }
          } else {
#pragma unroll
            for (int v = 0; v < VEC; ++v) val[u].v[v] = 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float w = 1.f;
          if constexpr (W) w = edge_bcast<NPI>(myw, j + u * NPI, grp);
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc.v[v] += W ? val[u].v[v] * w : val[u].v[v];
        }
      }
      base += wlen;
      wlen = 64;
    }
  };
  // the reduced fragment of a relation's row -> this lane's two output columns
  auto finish_rel = [&](const PreRel& r, Frag<VEC>& acc, int64_t deg, float (&g)[2])
      __attribute__((always_inline)) {
    combine_groups<LPR, VEC, GNNREC_REDUCE_SUM>(acc);
    if (r.mean) finalize<VEC, GNNREC_REDUCE_MEAN>(acc, deg, 0);
    const int sl = lane >> 1;
    const float x0 = __shfl(acc.v[0], sl), x1 = __shfl(acc.v[1], sl);
    const float x2 = __shfl(acc.v[2], sl), x3 = __shfl(acc.v[3], sl);
    g[0] = (lane & 1) ? x2 : x0;
    g[1] = (lane & 1) ? x3 : x1;
  };

  PairWalk walk;
  walk.queued = rq != nullptr;
  walk.pos = ((int64_t)blockIdx.x * kP2Waves + wave) * kPRows;
  walk.c1 = 0;
  if (walk.queued) rq_begin(walk.c, rq);
  int64_t row0, lim;
  bool have = walk_next(walk, rq, n_dst, rq_ch, stride, row0, lim);
  if (have) {  // prologue: the first step's heads, synchronously
    const int nv = (int)(lim - row0 < kPRows ? lim - row0 : kPRows);
    stage_heads(load_bounds(row0, nv), nv);
  }
  while (have) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // heads DMA'd and parked
    const int nv = (int)(lim - row0 < kPRows ? lim - row0 : kPRows);  // valid rows, >= 1
    int64_t rba[kPRows + 1], rbb[kPRows + 1];
    int pa[kPRows], pb[kPRows];
#pragma unroll
    for (int i = 0; i <= kPRows; ++i) {
      rba[i] = bnd[wave][0][i];
      rbb[i] = bnd[wave][1][i];
    }
#pragma unroll
    for (int i = 0; i < kPRows; ++i) {
      pa[i] = lane < kP2Win ? win[wave][0][i][lane] : 0;
      pb[i] = lane < kP2Win ? win[wave][1][i][lane] : 0;
    }
    // the next step's bounds, in flight under this step's gathers
    int64_t nrow0 = 0, nlim = 0;
    const bool next = walk_next(walk, rq, n_dst, rq_ch, stride, nrow0, nlim);
    const int nnv = next ? (int)(nlim - nrow0 < kPRows ? nlim - nrow0 : kPRows) : 0;
    const int64_t nbv = next ? load_bounds(nrow0, nnv) : 0;
#pragma unroll
    for (int i = 0; i < kPRows; ++i) {  // self rows into this wave's slots
      const float4 hs = i < nv && grp == 0 ? ld_stream4(H + (row0 + i) * ldh + col)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      if (grp == 0) *reinterpret_cast<float4*>(&slots[wave][i][col]) = hs;
    }
    float ga[kPRows][2], gb[kPRows][2];
    bool nea[kPRows], neb[kPRows];
#pragma unroll
    for (int i = 0; i < kPRows; ++i) {
      Frag<VEC> acc;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = 0.f;
      const int64_t deg = i < nv ? rba[i + 1] - rba[i] : 0;
      if (i < nv)
        gather_row(ra, std::integral_constant<bool, WA>{}, std::integral_constant<bool, NT == 1>{},
                   rba[i], rba[i + 1], pa[i], acc);
      finish_rel(ra, acc, deg, ga[i]);
      nea[i] = deg > 0;
    }
    // this step's index windows are in registers (pa / pb; their LDS reads retired): the
    // next step's land in LDS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (next) stage_heads(nbv, nnv);
#pragma unroll
    for (int i = 0; i < kPRows; ++i) {
      Frag<VEC> acc;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = 0.f;
      const int64_t deg = i < nv ? rbb[i + 1] - rbb[i] : 0;
      if (i < nv)
        gather_row(rb, std::integral_constant<bool, WB>{}, std::integral_constant<bool, NT == 2>{},
                   rbb[i], rbb[i + 1], pb[i], acc);
      finish_rel(rb, acc, deg, gb[i]);
      neb[i] = deg > 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    float za[kPRows][2], zb[kPRows][2];
#pragma unroll
    for (int i = 0; i < kPRows; ++i) {
      za[i][0] = ba0 + (nea[i] ? ca0 : 0.f);
      za[i][1] = ba1 + (nea[i] ? ca1 : 0.f);
      zb[i][0] = bb0 + (neb[i] ? cb0 : 0.f);
      zb[i][1] = bb1 + (neb[i] ? cb1 : 0.f);
    }
#pragma unroll 2
    for (int k = 0; k < kPD; k += 4) {
      float4 s4[kPRows];
#pragma unroll
      for (int i = 0; i < kPRows; ++i) s4[i] = *reinterpret_cast<const float4*>(&slots[wave][i][k]);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const float2 wa = *reinterpret_cast<const float2*>(&Wa[(k + kk) * kPD + j0]);
        const float2 wb = *reinterpret_cast<const float2*>(&Wb[(k + kk) * kPD + j0]);
#pragma unroll
        for (int i = 0; i < kPRows; ++i) {
          const float sv = kk == 0 ? s4[i].x : kk == 1 ? s4[i].y : kk == 2 ? s4[i].z : s4[i].w;
          za[i][0] = fmaf(sv, wa.x, za[i][0]);
          za[i][1] = fmaf(sv, wa.y, za[i][1]);
          zb[i][0] = fmaf(sv, wb.x, zb[i][0]);
          zb[i][1] = fmaf(sv, wb.y, zb[i][1]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slots free for the next rows

#pragma unroll
    for (int i = 0; i < kPRows; ++i) {
      float ya0 = za[i][0] + ga[i][0], ya1 = za[i][1] + ga[i][1];
      float yb0 = zb[i][0] + gb[i][0], yb1 = zb[i][1] + gb[i][1];
      activate(relu, l2, ya0, ya1);
      activate(relu, l2, yb0, yb1);
      float y0, y1;
      if (combine == GNNREC_ACC_MAX) {
        y0 = fmaxf(ya0, yb0);
        y1 = fmaxf(ya1, yb1);
      } else if (combine == GNNREC_ACC_ATTN_LAST) {
        float sa = ya0 * at0 + ya1 * at1, sb = yb0 * at0 + yb1 * at1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          sa += __shfl_xor(sa, off);
          sb += __shfl_xor(sb, off);
        }
        const float mnew = fmaxf(sa, sb);
        const float keep = expf(sa - mnew), cnew = expf(sb - mnew);
        const float nrm = 1.f / (1.f * keep + cnew);
        y0 = ya0 * keep + yb0 * cnew;
        y1 = ya1 * keep + yb1 * cnew;
        y0 *= nrm;
        y1 *= nrm;
      } else {
        y0 = ya0 + yb0;
        y1 = ya1 + yb1;
      }
      if (out_div > 0.f) {
        y0 = y0 / out_div;
        y1 = y1 / out_div;
      }
      if (i < nv) {
        typedef float f32x2s __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(f32x2s{y0, y1},
                                    reinterpret_cast<f32x2s*>(out + (row0 + i) * ldo + j0));
      }
    }
    row0 = nrow0;
    lim = nlim;
    have = next;
  }
  if (rq != nullptr) rq_finish(rq);
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_spmm_project2_f32(
    const int64_t* indptr_a, const int32_t* indices_a, const float* ew_a, const float* Ya,
    int64_t ldya, int reduce_a, const float* bias_nonempty_a, const int64_t* indptr_b,
    const int32_t* indices_b, const float* ew_b, const float* Yb, int64_t ldyb, int reduce_b,
    const float* bias_nonempty_b, const float* H, int64_t ldh, const float* W_self_aT,
    const float* W_self_bT, const float* bias_a, const float* bias_b, int64_t n_dst, int64_t d,
    int epilogue, int combine, const float* attn_vec, float out_div, float* out, int64_t ldo,
    void* stream) {
  GNNREC_REQUIRE(d == kPD, "gnnrec_spmm_project2_f32: only d = %d (got %lld)", kPD,
                 (long long)d);
  // GNNREC_SRC_STREAM on one relation: its source rows non-temporal (NT = 1: a, 2: b)
  int nt = ((reduce_a & GNNREC_SRC_STREAM) ? 1 : 0) | ((reduce_b & GNNREC_SRC_STREAM) ? 2 : 0);
  if (nt == 3) nt = 0;  // both: nothing to keep in the caches for
  reduce_a &= ~GNNREC_SRC_STREAM;
  reduce_b &= ~GNNREC_SRC_STREAM;
  GNNREC_REQUIRE((reduce_a == GNNREC_REDUCE_SUM || reduce_a == GNNREC_REDUCE_MEAN) &&
                     (reduce_b == GNNREC_REDUCE_SUM || reduce_b == GNNREC_REDUCE_MEAN),
                 "gnnrec_spmm_project2_f32: pre-projected relations reduce by sum or mean");
  GNNREC_REQUIRE((epilogue & ~(GNNREC_EPI_RELU | GNNREC_EPI_L2NORM)) == 0,
                 "gnnrec_spmm_project2_f32: epilogue must be RELU|L2NORM");
  GNNREC_REQUIRE(combine == GNNREC_ACC_ADD || combine == GNNREC_ACC_MAX ||
                     combine == GNNREC_ACC_ATTN_LAST,
                 "gnnrec_spmm_project2_f32: combine must be GNNREC_ACC_ADD, _MAX or _ATTN_LAST");
  GNNREC_REQUIRE((combine == GNNREC_ACC_ATTN_LAST) == (attn_vec != nullptr),
                 "gnnrec_spmm_project2_f32: attn_vec goes with combine GNNREC_ACC_ATTN_LAST");
  GNNREC_REQUIRE(n_dst >= 0, "gnnrec_spmm_project2_f32: negative n_dst");
  if (n_dst == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr_a && Ya && indptr_b && Yb && H && W_self_aT && W_self_bT && out,
                 "gnnrec_spmm_project2_f32: null pointer");
  GNNREC_REQUIRE(aligned16(Ya) && aligned16(Yb) && aligned16(H) && aligned16(W_self_aT) &&
                     aligned16(W_self_bT) && ldya % 4 == 0 && ldyb % 4 == 0 && ldh % 4 == 0 &&
                     ldo % 2 == 0 && (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                 "gnnrec_spmm_project2_f32: Y/H/W need 16-B aligned rows, out 8-B");
  const int64_t per_block = (int64_t)kP2Waves * kPRows;
  int64_t blocks = (n_dst + per_block - 1) / per_block;
  const int64_t cus = device_cus() - cu_reserve();
  if (blocks > (cus > 8 ? cus : 8)) blocks = cus > 8 ? cus : 8;
  // rows per queue ticket: 16 (C5 user side, one session: 38.4–38.8 ms at 8, 37.4 at 16,
  // 37.5 at 32 — within the kernel's ±1 ms run-to-run spread)
  constexpr int rq_ch = 16;
  hipStream_t s = as_stream(stream);
  int ticket = -1;
  unsigned* rq = n_dst >= blocks * kP2Waves * rq_ch * 4 ? rowq_slot(s, &ticket) : nullptr;
  const dim3 grid((unsigned)blocks), block(kP2Waves * 64);
  const PreRel a{indptr_a, indices_a, ew_a, Ya, ldya, bias_nonempty_a,
                 reduce_a == GNNREC_REDUCE_MEAN};
  const PreRel b{indptr_b, indices_b, ew_b, Yb, ldyb, bias_nonempty_b,
                 reduce_b == GNNREC_REDUCE_MEAN};
#define GNNREC_SPP2(WA_, WB_)                                                                \
  hipLaunchKernelGGL((spmm_project2_pipe_kernel<WA_, WB_>), grid, block, 0, s, a, b, H, ldh,    \
                     W_self_aT, W_self_bT, bias_a, bias_b, n_dst, epilogue, combine, attn_vec, \
                     out_div, out, ldo, rq, rq_ch)
  if (nt && !ew_a && !ew_b) {
    if (nt == 1)
      hipLaunchKernelGGL((spmm_project2_pipe_kernel<false, false, 1>), grid, block, 0, s, a, b,
                         H, ldh, W_self_aT, W_self_bT, bias_a, bias_b, n_dst, epilogue, combine,
                         attn_vec, out_div, out, ldo, rq, rq_ch);
    else
      hipLaunchKernelGGL((spmm_project2_pipe_kernel<false, false, 2>), grid, block, 0, s, a, b,
                         H, ldh, W_self_aT, W_self_bT, bias_a, bias_b, n_dst, epilogue, combine,
                         attn_vec, out_div, out, ldo, rq, rq_ch);
  } else if (ew_a) {
    if (ew_b) GNNREC_SPP2(true, true);
    else GNNREC_SPP2(true, false);
  } else {
    if (ew_b) GNNREC_SPP2(false, true);
    else GNNREC_SPP2(false, false);
  }
#undef GNNREC_SPP2
  rowq_launched(ticket, s);
  return check_launch("gnnrec_spmm_project2_f32");
}
