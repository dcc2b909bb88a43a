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
//   * neighbour k of a range always lands in lane group k % NPI and groups are
//     combined by a fixed xor-tree, so the reduction order depends only on the
//     CSR row: results are bitwise reproducible run to run.
// Heavy rows (deg > split, e.g. Zipf-popular items) are skipped by the row
// kernel and reduced instead by one wave per `split`-edge chunk into a
// workspace, then combined per row in chunk order (deterministic two-phase).
#include "common.hpp"
#include "gather.hpp"
#include "rowq.hpp"
#include <cmath>
#include <cstdlib>

namespace gnnrec {
namespace {

// rows per queue ticket of the row kernel (rowq.hpp): about kRqTicketEdges edges per ticket
// from the CSR's mean degree (C4 tiles: 8 rows ≈ 280 µs of one wave, 0.5 % faster than 4;
// minibatch blocks at 7-10 edges/row: 51-64 rows, so the ticket round trip stays amortised);
// the kernels' `chunk` argument > 0 would fix it (0: this rule)
constexpr int64_t kRqTicketEdges = 512;
// Below 32 rows per wave the static grid-stride wins: the queue's dequeues are bound by
// the heads' atomic rate (≈88 per µs each), so a short launch either takes few long tickets
// (a fraction of the waves walk 51-row chains) or many short ones (atomic-bound).  A C2
// block relation (100k rows x 10 edges, d = 64): 52 µs static vs 127-165 µs queued; 1M rows:
// 444 µs queued vs 472 static (tools/micro/spmm_one.py, profiles/r03_spmm_rowq.txt).
constexpr int64_t kRqMinRowsPerWave = 32;
constexpr int kRowChunk = 0;

// rows per ticket: about kRqTicketEdges edges, but at least 4 tickets per wave of the grid.
// A minibatch block (100k rows at 10 edges) at 51 rows per ticket fed 1960 of the grid's
// 8192 waves, each walking its 51 rows one latency chain after another (C2: 130-180 µs per
// launch); the cap keeps every wave busy.  The reduction of a row does not depend on it.
__device__ __forceinline__ int ticket_rows(int64_t avg_deg, int64_t n_dst, int64_t waves) {
  int64_t c = kRqTicketEdges / (avg_deg > 0 ? avg_deg : 1);
  const int64_t cap = n_dst / (waves * 4);
  if (c > cap) c = cap;
  return (int)(c < 1 ? 1 : c > 64 ? 64 : c);
}

// Low-degree rows, d <= LPR * VEC: one group of LPR lanes per row, NPI = 64 / LPR rows per
// wave.  A wave-per-row launch over a 1M-row CSR at 2-3 edges per row (a K = 2500
// minibatch's transposed blocks) is a chain of indptr -> indices -> source-row loads per row
// with 2-3 of its 4-16 neighbour slots busy; here every group walks its own row, so a wave
// keeps NPI rows' chains in flight.  The reduction order is the wave kernel's: neighbour k of
// a row goes to partial (k - beg) % NPI in increasing k, and the partials are combined by
// the same pairwise tree as combine_groups -- bitwise the same rows (tests/test_gpu_parity).
// No cross-lane traffic: each lane loads the (group-uniform) index and weight itself.
template <int LPR, int VEC, int REDUCE, bool WEIGHTED>
__device__ __forceinline__ void group_rows(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx, int64_t n_dst, int d,
    float* __restrict__ out, int64_t ldo, int flags, int64_t max_deg) {
  constexpr int NPI = kWave / LPR;
  constexpr int U = NPI >= 8 ? NPI : 8;  // neighbours in flight per group; a multiple of NPI
  const int empty_neginf = flags & GNNREC_SPMM_EMPTY_NEGINF;
  const int lane = threadIdx.x & 63;
  const int col = (lane % LPR) * VEC;
  const bool colok = col < d;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const int64_t stride = (int64_t)gridDim.x * 4 * NPI;
  int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * NPI + lane / LPR;
  int64_t beg = 0, end = 0;
  if (row < n_dst) {
    beg = ld_stream(indptr + row);
    end = ld_stream(indptr + row + 1);
  }
  for (; row < n_dst; row += stride) {
    // the next row's bounds are requested before this row gathers
    const int64_t nrow = row + stride;
    int64_t nbeg = 0, nend = 0;
    if (nrow < n_dst) {
      nbeg = ld_stream(indptr + nrow);
      nend = ld_stream(indptr + nrow + 1);
    }
    if (end - beg <= max_deg) {  // heavy rows: reduced by the chunk kernels
      Frag<VEC> p[NPI];
#pragma unroll
      for (int i = 0; i < NPI; ++i)
#pragma unroll
        for (int v = 0; v < VEC; ++v) p[i].v[v] = init;
      for (int64_t k = beg; k < end; k += U) {
        const int cnt = (int)(end - k < U ? end - k : U);
        int src[U];
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          src[u] = u < cnt ? ld_stream(indices + k + u) : 0;
          if constexpr (WEIGHTED) w[u] = u < cnt ? ld_stream(ew + k + u) : 0.f;
        }
        Frag<VEC> val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < cnt && colok) {
            load_frag<VEC>(val[u], X + (int64_t)src[u] * ldx + col);
          } else {
#pragma unroll
            for (int v = 0; v < VEC; ++v) val[u].v[v] = 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < cnt) {
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
              const float m = WEIGHTED ? val[u].v[v] * w[u] : val[u].v[v];
              if constexpr (REDUCE == GNNREC_REDUCE_MAX) p[u % NPI].v[v] = fmaxf(p[u % NPI].v[v], m);
              else p[u % NPI].v[v] += m;
            }
          }
        }
      }
#pragma unroll
      for (int s = 1; s < NPI; s <<= 1)
#pragma unroll
        for (int i = 0; i < NPI; i += 2 * s)
#pragma unroll
          for (int v = 0; v < VEC; ++v) p[i].v[v] = combine<REDUCE>(p[i].v[v], p[i + s].v[v]);
      finalize<VEC, REDUCE>(p[0], end - beg, empty_neginf);
      if (colok) {
        if (flags & GNNREC_SPMM_ACCUM) accumulate_into<VEC, REDUCE>(p[0], out + row * ldo + col);
        store_frag<VEC>(out + row * ldo + col, p[0]);
      }
    }
    beg = nbeg;
    end = nend;
  }
}

// Mean degree up to which the group kernel takes a d <= 64 CSR.
constexpr int64_t kGroupMaxAvgDeg = 16;

template <int LPR, int VEC, int REDUCE, bool WEIGHTED, int UNROLL>
__global__ __launch_bounds__(256) void spmm_csr_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx, int64_t n_dst, int d,
    float* __restrict__ out, int64_t ldo, int flags, int64_t max_deg, unsigned* rq,
    int rq_ch, int64_t group_deg, const int64_t* __restrict__ live,
    const int64_t* __restrict__ plan_counts) {
  // a device-built plan that overflowed its capacities (plan_chunks_kernel: n_heavy < 0)
  // covers no row: every row, heavy or not, is reduced here instead
  if (plan_counts != nullptr && plan_counts[0] < 0) max_deg = INT64_MAX;
  if (live != nullptr) {
    // rows from the device count on (a static block's padding and dump rows): the empty
    // row's value (0: sum / mean), no gathers; left as they are under ACCUM (+= 0)
    const int64_t l = *live;
    const int64_t n_rows = l < 0 ? 0 : (l < n_dst ? l : n_dst);
    if (!(flags & GNNREC_SPMM_ACCUM) && blockIdx.y == 0) {
      const int64_t nw = (int64_t)gridDim.x * 4;
      for (int64_t r = n_rows + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_dst; r += nw)
        for (int c = threadIdx.x & 63; c < d; c += 64) out[r * ldo + c] = 0.f;
    }
    n_dst = n_rows;
    if (n_dst == 0) {
      if (rq != nullptr) rq_finish(rq);
      return;
    }
  }
  if constexpr (VEC == 4 && (LPR == 8 || LPR == 16)) {  // d in (16, 64]; at LPR 4 the 16
                                                        // partials cost occupancy
    // low mean degree: one lane group per row (the choice needs the CSR's edge count,
    // which only the device holds)
    if (group_deg > 0 && indptr[n_dst] - indptr[0] <= group_deg * n_dst) {
      group_rows<LPR, VEC, REDUCE, WEIGHTED>(indptr, indices, ew, X, ldx, n_dst, d, out, ldo,
                                             flags, max_deg);
      if (rq != nullptr) rq_finish(rq);
      return;
    }
  }
  const int empty_neginf = flags & GNNREC_SPMM_EMPTY_NEGINF;
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR;
  const int col = blockIdx.y * (LPR * VEC) + (lane % LPR) * VEC;
  const bool colok = col < d;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  auto one_row = [&](int64_t row) {
    const int64_t beg = indptr[row];
    const int64_t end = indptr[row + 1];
    if (end - beg > max_deg) return;  // heavy row: reduced by the chunk kernels
    Frag<VEC> acc;
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc.v[v] = init;
    gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL>(beg, end, indices, ew, X, ldx, col, colok,
                                                     lane, grp, acc);
    combine_groups<LPR, VEC, REDUCE>(acc);
    finalize<VEC, REDUCE>(acc, end - beg, empty_neginf);
    if (grp == 0 && colok) {
      if (flags & GNNREC_SPMM_ACCUM) accumulate_into<VEC, REDUCE>(acc, out + row * ldo + col);
      store_frag<VEC>(out + row * ldo + col, acc);
    }
  };
  if (rq != nullptr) {  // queued rows (one column slice: the launcher checks gridDim.y == 1)
    if (rq_ch <= 0) {
      const int64_t avg = (indptr[n_dst] - indptr[0]) / n_dst;
      rq_ch = ticket_rows(avg, n_dst, gridDim.x * 4);
    }
    // a ticket's row bounds come from one coalesced indptr load, and the next row's first
    // 64 indices are requested before the current row gathers: of the indptr -> indices ->
    // source-row chain only the last link stays exposed at a row boundary
    rq_for_each(rq, n_dst, rq_ch, [&](int64_t r0, int64_t r1) {
      const int nr = (int)(r1 - r0);  // <= 64
      const int64_t ipl = lane < nr ? ld_stream(indptr + r0 + lane) : 0;
      const int64_t ip_end = indptr[r1];
      auto bound = [&](int k) { return k < nr ? __shfl(ipl, k) : ip_end; };
      int64_t beg = bound(0), end = bound(1);
      int nidx = lane < end - beg ? ld_stream(indices + beg + lane) : 0;
      for (int k = 0; k < nr; ++k) {
        const int idx = nidx;
        const int64_t nbeg = end, nend = k + 1 < nr ? bound(k + 2) : end;
        if (k + 1 < nr) nidx = lane < nend - nbeg ? ld_stream(indices + nbeg + lane) : 0;
        if (end - beg <= max_deg) {  // heavy rows: reduced by the chunk kernels
          Frag<VEC> acc;
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc.v[v] = init;
          gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL, true>(
              beg, end, indices, ew, X, ldx, col, colok, lane, grp, acc, idx);
          combine_groups<LPR, VEC, REDUCE>(acc);
          finalize<VEC, REDUCE>(acc, end - beg, empty_neginf);
          const int64_t row = r0 + k;
          if (grp == 0 && colok) {
            if (flags & GNNREC_SPMM_ACCUM) accumulate_into<VEC, REDUCE>(acc, out + row * ldo + col);
            store_frag<VEC>(out + row * ldo + col, acc);
          }
        }
        beg = nbeg;
        end = nend;
      }
    });
    rq_finish(rq);
    return;
  }
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_dst; row += wstride)
    one_row(row);
}

// phase 1 of heavy rows: one wave per chunk of `split` edges -> raw partial in ws[chunk]
template <int LPR, int VEC, int REDUCE, bool WEIGHTED, int UNROLL>
__global__ __launch_bounds__(256) void spmm_chunk_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx, int d,
    int64_t split, const int64_t* __restrict__ heavy_rows, const int64_t* __restrict__ chunk_ptr,
    const int64_t* __restrict__ chunk_row, int64_t n_chunks, const int64_t* __restrict__ counts,
    float* __restrict__ ws) {
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR;
  const int col = blockIdx.y * (LPR * VEC) + (lane % LPR) * VEC;
  const bool colok = col < d;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  if (counts) n_chunks = counts[1];  // device-built plan: the grid covers its capacity
                                     // (0 when it overflowed)
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < n_chunks; c += wstride) {
    const int64_t h = chunk_row[c];
    const int64_t row = heavy_rows[h];
    const int64_t rbeg = indptr[row], rend = indptr[row + 1];
    const int64_t beg = rbeg + (c - chunk_ptr[h]) * split;
    const int64_t end = (beg + split < rend) ? beg + split : rend;
    Frag<VEC> acc;
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc.v[v] = init;
    gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL>(beg, end, indices, ew, X, ldx, col, colok,
                                                     lane, grp, acc);
    combine_groups<LPR, VEC, REDUCE>(acc);
    if (grp == 0 && colok) store_frag<VEC>(ws + c * (int64_t)d + col, acc);
  }
}

// phase 2 of heavy rows: one wave per heavy row, partials combined in chunk order
template <int VEC, int REDUCE>
__global__ __launch_bounds__(256) void spmm_combine_kernel(
    const int64_t* __restrict__ indptr, int d, const int64_t* __restrict__ heavy_rows,
    int64_t n_heavy, const int64_t* __restrict__ chunk_ptr, const float* __restrict__ ws,
    float* __restrict__ out, int64_t ldo, int flags, const int64_t* __restrict__ counts) {
  const int empty_neginf = flags & GNNREC_SPMM_EMPTY_NEGINF;
  const int lane = threadIdx.x & 63;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  if (counts) n_heavy = counts[0];  // < 0: an overflowed plan (the row kernel took them)
  for (int64_t h = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); h < n_heavy; h += wstride) {
    const int64_t row = heavy_rows[h];
    const int64_t deg = indptr[row + 1] - indptr[row];
    for (int col = blockIdx.y * 64 * VEC + lane * VEC; col < d; col += gridDim.y * 64 * VEC) {
      Frag<VEC> acc;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = init;
      // chunk partials in chunk order; 16 loads in flight ahead of the (ordered) adds: a
      // Zipf head row has thousands of chunks per tile, and one load per add made its
      // combine a 0.87 ms latency chain (C4 --zipf 1.0, 16 launches per pass)
      const int64_t c_end = chunk_ptr[h + 1];
      int64_t c = chunk_ptr[h];
      for (; c + 16 <= c_end; c += 16) {
        Frag<VEC> p[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) load_frag<VEC>(p[u], ws + (c + u) * (int64_t)d + col);
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc.v[v] = combine<REDUCE>(acc.v[v], p[u].v[v]);
      }
      for (; c < c_end; ++c) {
        Frag<VEC> p;
        load_frag<VEC>(p, ws + c * (int64_t)d + col);
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc.v[v] = combine<REDUCE>(acc.v[v], p.v[v]);
      }
      finalize<VEC, REDUCE>(acc, deg, empty_neginf);
      if (flags & GNNREC_SPMM_ACCUM) accumulate_into<VEC, REDUCE>(acc, out + row * ldo + col);
      store_frag<VEC>(out + row * ldo + col, acc);
    }
  }
}

struct SpmmArgs {
  const int64_t* indptr; const int32_t* indices; const float* ew; const float* X; int64_t ldx;
  int64_t n_dst; int d; float* out; int64_t ldo; int flags;
  int64_t split; const int64_t* heavy_rows; int64_t n_heavy; const int64_t* chunk_ptr;
  const int64_t* chunk_row; int64_t n_chunks; float* ws;
  const int64_t* counts;  // device-built plan: {n_heavy, n_chunks}; n_heavy/n_chunks above
                          // are then the plan's capacities (grid sizes)
  const int64_t* live;    // device row count (nullable): rows from it on are empty rows
};

// Resident 256-thread blocks per CU the row kernels occupy (grid-stride beyond): every wave
// slot of a CU (CUs kept for concurrent kernels come off through gnnrec_set_concurrency).
constexpr int64_t kBlocksPerCu = 8;

inline unsigned grid_waves(int64_t units) {
  int64_t blocks = (units + 3) / 4;
  // CUs reserved for concurrent kernels (gnnrec_set_concurrency) come off the grid
  const int cus = device_cus() - cu_reserve();
  const int64_t max_blocks = (int64_t)(cus > 8 ? cus : 8) * kBlocksPerCu;
  if (blocks > max_blocks) blocks = max_blocks;
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

constexpr int kSpmmUnroll = 4;  // wave-instructions in flight per lane (6, 8: the same)
template <int LPR, int VEC, int REDUCE, bool WEIGHTED>
int launch_all(const SpmmArgs& a, hipStream_t s) {
  constexpr int UNROLL = (VEC == 4) ? kSpmmUnroll : 2;
  const int cols_per_slice = LPR * VEC;
  const unsigned slices = (unsigned)((a.d + cols_per_slice - 1) / cols_per_slice);
  const int eni = a.flags & (GNNREC_SPMM_EMPTY_NEGINF | GNNREC_SPMM_ACCUM);
  const int64_t max_deg = a.n_heavy > 0 ? a.split : INT64_MAX;
  const unsigned grid = grid_waves(a.n_dst);
  // the queue pays off on long launches only (≥ kRqMinRowsPerWave rows per wave of the grid)
  int ticket = -1;
  unsigned* rq = slices == 1 && a.n_dst >= (int64_t)grid * 4 * kRqMinRowsPerWave
                     ? rowq_slot(s, &ticket)
                     : nullptr;
  hipLaunchKernelGGL((spmm_csr_kernel<LPR, VEC, REDUCE, WEIGHTED, UNROLL>),
                     dim3(grid, slices), dim3(256), 0, s, a.indptr, a.indices, a.ew,
                     a.X, a.ldx, a.n_dst, a.d, a.out, a.ldo, eni, max_deg, rq, kRowChunk,
                     kGroupMaxAvgDeg, a.live, a.counts);
  rowq_launched(ticket, s);
  if (a.n_heavy > 0) {
    hipLaunchKernelGGL((spmm_chunk_kernel<LPR, VEC, REDUCE, WEIGHTED, UNROLL>),
                       dim3(grid_waves(a.n_chunks), slices), dim3(256), 0, s, a.indptr, a.indices,
                       a.ew, a.X, a.ldx, a.d, a.split, a.heavy_rows, a.chunk_ptr, a.chunk_row,
                       a.n_chunks, a.counts, a.ws);
    const unsigned cslices = (unsigned)((a.d + 64 * VEC - 1) / (64 * VEC));
    hipLaunchKernelGGL((spmm_combine_kernel<VEC, REDUCE>), dim3(grid_waves(a.n_heavy), cslices),
                       dim3(256), 0, s, a.indptr, a.d, a.heavy_rows, a.n_heavy, a.chunk_ptr, a.ws,
                       a.out, a.ldo, eni, a.counts);
  }
  return check_launch("gnnrec_spmm_csr_f32");
}

// ---- two relations into one destination type, one launch ----------------------------
// C5's user->item relations (clicks: 50 edges per item row and source tile, buys: 12.5)
// gather from the same user slice into separate partial tables.  Launched apart, the
// low-degree relation's tiles are bound by their per-row latency chain (1.2-1.36 ms for
// 12.5M edges); here every queue ticket takes rows [r0, r1) of relation A and then the
// same rows of relation B, so the short rows run beside long ones on every wave.  Each
// relation's rows are reduced exactly as by spmm_csr_kernel (bitwise the same partials).
// No heavy-row split (callers check both CSRs are plan-free), one column slice (d <= 256).
struct Csr2 {
  const int64_t* indptr[2];
  const int32_t* indices[2];
  const float* ew[2];
  float* out[2];
};

template <int LPR, int VEC, int REDUCE, bool WEIGHTED, int UNROLL>
__global__ __launch_bounds__(256) void spmm_csr2_kernel(Csr2 c, const float* __restrict__ X,
                                                        int64_t ldx, int64_t n_dst, int d,
                                                        int64_t ldo, int flags, unsigned* rq,
                                                        int rq_ch) {
  const int empty_neginf = flags & GNNREC_SPMM_EMPTY_NEGINF;
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPR;
  const int col = (lane % LPR) * VEC;
  const bool colok = col < d;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  // rows [r0, r1) of relation rel: the queued row loop of spmm_csr_kernel
  auto rows = [&](const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                  const float* __restrict__ ew, float* __restrict__ out, int64_t r0,
                  int64_t r1) __attribute__((always_inline)) {
    const int nr = (int)(r1 - r0);  // <= 64
    const int64_t ipl = lane < nr ? ld_stream(indptr + r0 + lane) : 0;
    const int64_t ip_end = indptr[r1];
    auto bound = [&](int k) { return k < nr ? __shfl(ipl, k) : ip_end; };
    int64_t beg = bound(0), end = bound(1);
    int nidx = lane < end - beg ? ld_stream(indices + beg + lane) : 0;
    for (int k = 0; k < nr; ++k) {
      const int idx = nidx;
      const int64_t nbeg = end, nend = k + 1 < nr ? bound(k + 2) : end;
      if (k + 1 < nr) nidx = lane < nend - nbeg ? ld_stream(indices + nbeg + lane) : 0;
      Frag<VEC> acc;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = init;
      gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL, true>(beg, end, indices, ew, X, ldx, col,
                                                             colok, lane, grp, acc, idx);
      combine_groups<LPR, VEC, REDUCE>(acc);
      finalize<VEC, REDUCE>(acc, end - beg, empty_neginf);
      const int64_t row = r0 + k;
      if (grp == 0 && colok) {
        if (flags & GNNREC_SPMM_ACCUM) accumulate_into<VEC, REDUCE>(acc, out + row * ldo + col);
        store_frag<VEC>(out + row * ldo + col, acc);
      }
      beg = nbeg;
      end = nend;
    }
  };
  auto both = [&](int64_t r0, int64_t r1) __attribute__((always_inline)) {
    rows(c.indptr[0], c.indices[0], c.ew[0], c.out[0], r0, r1);
    rows(c.indptr[1], c.indices[1], c.ew[1], c.out[1], r0, r1);
  };
  if (rq != nullptr) {
    if (rq_ch <= 0) {  // ≈ kRqTicketEdges edges of both relations per ticket
      const int64_t e = c.indptr[0][n_dst] - c.indptr[0][0] + c.indptr[1][n_dst] - c.indptr[1][0];
      rq_ch = ticket_rows(e / n_dst, n_dst, gridDim.x * 4);
    }
    rq_for_each(rq, n_dst, rq_ch, both);
    rq_finish(rq);
    return;
  }
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_dst; row += wstride)
    both(row, row + 1);
}

template <int LPR, int REDUCE, bool WEIGHTED>
int launch_csr2(const Csr2& c, const float* X, int64_t ldx, int64_t n_dst, int d, int64_t ldo,
                int flags, hipStream_t s) {
  const unsigned grid = grid_waves(n_dst);
  int ticket = -1;
  unsigned* rq = n_dst >= (int64_t)grid * 4 * 8 ? rowq_slot(s, &ticket) : nullptr;
  hipLaunchKernelGGL((spmm_csr2_kernel<LPR, 4, REDUCE, WEIGHTED, kSpmmUnroll>),
                     dim3(grid), dim3(256), 0, s, c, X, ldx, n_dst, d, ldo, flags, rq,
                     kRowChunk);
  rowq_launched(ticket, s);
  return check_launch("gnnrec_spmm_csr2_f32");
}

template <int VEC, int REDUCE, bool WEIGHTED>
int dispatch_lpr(int lpr, const SpmmArgs& a, hipStream_t s) {
  if constexpr (VEC == 1) {
    return launch_all<64, 1, REDUCE, WEIGHTED>(a, s);
  } else {
    switch (lpr) {
      case 4: return launch_all<4, 4, REDUCE, WEIGHTED>(a, s);
      case 8: return launch_all<8, 4, REDUCE, WEIGHTED>(a, s);
      case 16: return launch_all<16, 4, REDUCE, WEIGHTED>(a, s);
      case 32: return launch_all<32, 4, REDUCE, WEIGHTED>(a, s);
      default: return launch_all<64, 4, REDUCE, WEIGHTED>(a, s);
    }
  }
}

template <int VEC>
int dispatch_reduce(int reduce, int lpr, const SpmmArgs& a, hipStream_t s) {
  const bool w = a.ew != nullptr;
  switch (reduce) {
    case GNNREC_REDUCE_SUM:
      return w ? dispatch_lpr<VEC, GNNREC_REDUCE_SUM, true>(lpr, a, s)
               : dispatch_lpr<VEC, GNNREC_REDUCE_SUM, false>(lpr, a, s);
    case GNNREC_REDUCE_MEAN:
      return w ? dispatch_lpr<VEC, GNNREC_REDUCE_MEAN, true>(lpr, a, s)
               : dispatch_lpr<VEC, GNNREC_REDUCE_MEAN, false>(lpr, a, s);
    default:
      return w ? dispatch_lpr<VEC, GNNREC_REDUCE_MAX, true>(lpr, a, s)
               : dispatch_lpr<VEC, GNNREC_REDUCE_MAX, false>(lpr, a, s);
  }
}

int spmm_entry(SpmmArgs a, int64_t d, int reduce, void* stream) {
  GNNREC_REQUIRE(a.n_dst >= 0 && d >= 0, "gnnrec_spmm_csr_f32: negative size");
  GNNREC_REQUIRE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN ||
                     reduce == GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_csr_f32: unknown reduce %d", reduce);
  GNNREC_REQUIRE(d <= (1 << 20), "gnnrec_spmm_csr_f32: d=%lld too large", (long long)d);
  if (a.n_dst == 0 || d == 0) return GNNREC_OK;
  GNNREC_REQUIRE(a.indptr && a.out, "gnnrec_spmm_csr_f32: null indptr/out");
  GNNREC_REQUIRE(a.ldx >= d && a.ldo >= d, "gnnrec_spmm_csr_f32: leading dimension < d");
  GNNREC_REQUIRE(a.n_heavy == 0 || (a.split > 0 && a.heavy_rows && a.chunk_ptr && a.chunk_row &&
                                    a.ws && a.n_chunks > 0),
                 "gnnrec_spmm_csr_split_f32: incomplete heavy-row plan");
  GNNREC_REQUIRE(a.live == nullptr || reduce != GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_csr_live_f32: a device row count needs sum or mean");
  a.d = (int)d;
  const bool vec4 = (d % 4 == 0) && (a.ldx % 4 == 0) && (a.ldo % 4 == 0) && aligned16(a.X) &&
                    aligned16(a.out) && (a.n_heavy == 0 || aligned16(a.ws));
  int lpr = 64;
  if (vec4) {
    const int64_t lanes = d / 4;
    lpr = 4;
    while (lpr < lanes && lpr < 64) lpr <<= 1;
  }
  hipStream_t s = as_stream(stream);
  return vec4 ? dispatch_reduce<4>(reduce, lpr, a, s) : dispatch_reduce<1>(reduce, lpr, a, s);
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_spmm_csr_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                                   const float* X, int64_t ldx, int64_t n_dst, int64_t d,
                                   int reduce, int flags, float* out, int64_t ldo, void* stream) {
  gnnrec::SpmmArgs a{indptr, indices, ew, X, ldx, n_dst, 0, out, ldo, flags,
                     0, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr};
  return gnnrec::spmm_entry(a, d, reduce, stream);
}

extern "C" int gnnrec_spmm_csr_live_f32(const int64_t* indptr, const int32_t* indices,
                                        const float* ew, const float* X, int64_t ldx,
                                        int64_t n_dst, int64_t d, int reduce, int flags,
                                        float* out, int64_t ldo, const int64_t* live,
                                        void* stream) {
  gnnrec::SpmmArgs a{indptr, indices, ew, X, ldx, n_dst, 0, out, ldo, flags,
                     0, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, live};
  return gnnrec::spmm_entry(a, d, reduce, stream);
}

extern "C" int gnnrec_spmm_csr_split_f32(const int64_t* indptr, const int32_t* indices,
                                         const float* ew, const float* X, int64_t ldx,
                                         int64_t n_dst, int64_t d, int reduce, int flags,
                                         float* out, int64_t ldo, int64_t split,
                                         const int64_t* heavy_rows, int64_t n_heavy,
                                         const int64_t* chunk_ptr, const int64_t* chunk_row,
                                         int64_t n_chunks, float* workspace, void* stream) {
  gnnrec::SpmmArgs a{indptr, indices, ew, X, ldx, n_dst, 0, out, ldo, flags,
                     split, heavy_rows, n_heavy, chunk_ptr, chunk_row, n_chunks, workspace,
                     nullptr, nullptr};
  return gnnrec::spmm_entry(a, d, reduce, stream);
}

// ---- device-built heavy-row plan (no host readback) ----------------------------------
// Rows of degree > split number at most n_edges / (split + 1) and give at most
// n_edges / split + n_heavy chunks, so the plan is sized on the host from n_edges alone and
// filled on the device; the chunk / combine grids cover those capacities and read the real
// counts from plan[0..1].  Heavy rows land in atomic order, which only changes which wave
// reduces which chunk: each row still sums its own chunks in edge order (deterministic).
namespace gnnrec {
namespace {

__global__ __launch_bounds__(256) void plan_mark_kernel(const int64_t* __restrict__ indptr,
                                                        int64_t n_dst, int64_t split,
                                                        int64_t cap_h,
                                                        unsigned long long* __restrict__ counts,
                                                        int64_t* __restrict__ heavy_rows,
                                                        const int64_t* __restrict__ live) {
  if (live != nullptr) {  // rows past the device count are empty rows, never heavy
    const int64_t l = *live;
    n_dst = l < 0 ? 0 : (l < n_dst ? l : n_dst);
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n_dst; v += stride) {
    if (indptr[v + 1] - indptr[v] > split) {
      const unsigned long long h = atomicAdd(counts, 1ull);
      if ((int64_t)h < cap_h) heavy_rows[h] = v;
    }
  }
}

// the plan's two counts zeroed by a kernel, not hipMemsetAsync: the plan is rebuilt inside
// captured training steps (gnnrec.capture), and a kernel node re-runs on every replay
__global__ void plan_zero_kernel(int64_t* __restrict__ plan) {
  if (threadIdx.x < 2) plan[threadIdx.x] = 0;
}

// Plans whose heavy rows or chunks exceed their capacities (a CSR breaking the host's bound
// from its edge count): counted here, read by gnnrec_spmm_plan_overflows.  Atomic adds are
// vector-memory atomics; nothing else writes it.
__device__ unsigned long long g_plan_overflows = 0;

// one block: chunk_ptr = exclusive scan of ceil(deg/split) over the heavy rows, then
// chunk_row[c] = owning heavy row (at most cap_c chunks: the host's bound from the edge
// count, enforced here too so a CSR that breaks it cannot write past the plan).  A plan
// past either capacity is marked overflowed — plan[0] = -(heavy rows found), plan[1] = 0 —
// and counted: its chunk and combine kernels then do nothing and the row kernel reduces
// every row itself (exact, one wave per row), so no aggregate is ever clipped.
__global__ __launch_bounds__(1024) void plan_chunks_kernel(const int64_t* __restrict__ indptr,
                                                           int64_t split, int64_t* __restrict__ plan,
                                                           int64_t cap_h, int64_t cap_c) {
  __shared__ int64_t buf[1024];
  int64_t* heavy_rows = plan + 2;
  int64_t* chunk_ptr = heavy_rows + cap_h;
  int64_t* chunk_row = chunk_ptr + cap_h + 1;
  const int64_t n = plan[0] < cap_h ? plan[0] : cap_h;
  const int t = threadIdx.x;
  int64_t carry = 0;
  for (int64_t base = 0; base < n; base += 1024) {
    int64_t x = 0;
    if (base + t < n) {
      const int64_t r = heavy_rows[base + t];
      x = (indptr[r + 1] - indptr[r] + split - 1) / split;
    }
    buf[t] = x;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t y = t >= off ? buf[t - off] : 0;
      __syncthreads();
      buf[t] += y;
      __syncthreads();
    }
    if (base + t < n) chunk_ptr[base + t] = carry + buf[t] - x;
    carry += buf[1023];
    __syncthreads();
  }
  if (t == 0) {
    chunk_ptr[n] = carry;
    plan[1] = carry;
  }
  __syncthreads();
  for (int64_t h = t; h < n; h += 1024) {
    const int64_t c1 = chunk_ptr[h + 1] < cap_c ? chunk_ptr[h + 1] : cap_c;
    for (int64_t c = chunk_ptr[h]; c < c1; ++c) chunk_row[c] = h;
  }
  if (t == 0 && (carry > cap_c || plan[0] > cap_h)) {
    plan[0] = -(plan[0] > 0 ? plan[0] : 1);
    plan[1] = 0;
    atomicAdd(&g_plan_overflows, 1ull);
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_spmm_plan_build_live(const int64_t* indptr, int64_t n_dst, int64_t split,
                                           int64_t cap_h, int64_t cap_c, int64_t* plan,
                                           const int64_t* live, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_dst >= 0 && split > 0 && cap_h >= 0 && cap_c >= 0,
                 "gnnrec_spmm_plan_build: bad sizes");
  GNNREC_REQUIRE(indptr && plan, "gnnrec_spmm_plan_build: null pointer");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(plan_zero_kernel, dim3(1), dim3(64), 0, s, plan);
  if (n_dst > 0 && cap_h > 0) {
    int64_t blocks = (n_dst + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(plan_mark_kernel, dim3((unsigned)blocks), dim3(256), 0, s, indptr, n_dst,
                       split, cap_h, reinterpret_cast<unsigned long long*>(plan), plan + 2, live);
    hipLaunchKernelGGL(plan_chunks_kernel, dim3(1), dim3(1024), 0, s, indptr, split, plan, cap_h,
                       cap_c);
  }
  return check_launch("gnnrec_spmm_plan_build");
}

extern "C" int gnnrec_spmm_plan_overflows(int64_t* count) {
  GNNREC_REQUIRE(count, "gnnrec_spmm_plan_overflows: null pointer");
  unsigned long long v = 0;
  hipError_t e = hipDeviceSynchronize();  // every plan build issued so far has run
  if (e == hipSuccess)
    e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(gnnrec::g_plan_overflows), sizeof(v), 0,
                                     hipMemcpyDeviceToHost);
  GNNREC_REQUIRE(e == hipSuccess, "gnnrec_spmm_plan_overflows: %s", hipGetErrorString(e));
  *count = (int64_t)v;
  return GNNREC_OK;
}

extern "C" int gnnrec_spmm_plan_build(const int64_t* indptr, int64_t n_dst, int64_t split,
                                      int64_t cap_h, int64_t cap_c, int64_t* plan, void* stream) {
  return gnnrec_spmm_plan_build_live(indptr, n_dst, split, cap_h, cap_c, plan, nullptr, stream);
}

extern "C" int gnnrec_spmm_csr_planned_live_f32(const int64_t* indptr, const int32_t* indices,
                                                const float* ew, const float* X, int64_t ldx,
                                                int64_t n_dst, int64_t d, int reduce, int flags,
                                                float* out, int64_t ldo, int64_t split,
                                                const int64_t* plan, int64_t cap_h,
                                                int64_t cap_c, float* workspace,
                                                const int64_t* live, void* stream) {
  GNNREC_REQUIRE(plan && cap_h > 0 && cap_c > 0, "gnnrec_spmm_csr_planned_f32: empty plan");
  gnnrec::SpmmArgs a{indptr, indices, ew, X, ldx, n_dst, 0, out, ldo, flags,
                     split, plan + 2, cap_h, plan + 2 + cap_h, plan + 3 + 2 * cap_h, cap_c,
                     workspace, plan, live};
  return gnnrec::spmm_entry(a, d, reduce, stream);
}

extern "C" int gnnrec_spmm_csr_planned_f32(const int64_t* indptr, const int32_t* indices,
                                           const float* ew, const float* X, int64_t ldx,
                                           int64_t n_dst, int64_t d, int reduce, int flags,
                                           float* out, int64_t ldo, int64_t split,
                                           const int64_t* plan, int64_t cap_h, int64_t cap_c,
                                           float* workspace, void* stream) {
  return gnnrec_spmm_csr_planned_live_f32(indptr, indices, ew, X, ldx, n_dst, d, reduce, flags,
                                          out, ldo, split, plan, cap_h, cap_c, workspace,
                                          nullptr, stream);
}

// ---------------------------------------------------------------- backward --
// f2 — gradient of a1 w.r.t. the source rows (training through ConvLayer,
// reference src/train/run.py:136-138).  sum/mean: grad_X[src_e] += w_e/deg·g[v];
// max: the gradient of column c goes to the FIRST edge (CSR order) whose message
// equals the forward maximum (DGL's arg-max convention).  Float atomics into
// grad_X (no reproducibility requirement on training gradients).
namespace gnnrec {
namespace {

// One wave per dst row.  The row's gradient slice (NC columns per lane) stays in registers
// while the wave walks its edges 64 at a time: one coalesced load of 64 indices (and
// weights), then per edge a broadcast source id and NC no-return global_atomic_add_f32 on
// a contiguous 256-B column run, so many atomics are in flight per wave instead of one
// dependent index load per edge.
template <int REDUCE, bool WEIGHTED, int NC>
__global__ __launch_bounds__(256) void spmm_backward_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ G, int64_t ldg,
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ Y, int64_t ldy,
    int64_t n_dst, int d, float* __restrict__ gX, int64_t ldgx) {
  const int lane = threadIdx.x & 63;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); v < n_dst; v += wstride) {
    const int64_t beg = indptr[v], end = indptr[v + 1];
    if (beg == end) continue;
    const float scale = REDUCE == GNNREC_REDUCE_MEAN ? 1.f / (float)(end - beg) : 1.f;
    for (int c0 = 0; c0 < d; c0 += kWave * NC) {
      float g[NC], y[NC];
      bool live[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int c = c0 + lane + kWave * j;
        g[j] = c < d ? G[v * ldg + c] * scale : 0.f;
        live[j] = g[j] != 0.f;
        if constexpr (REDUCE == GNNREC_REDUCE_MAX) y[j] = live[j] ? Y[v * ldy + c] : 0.f;
      }
      for (int64_t eb = beg; eb < end; eb += kWave) {
        const int n = (int)(end - eb < kWave ? end - eb : kWave);
        const int my_u = lane < n ? indices[eb + lane] : 0;
        const float my_w = WEIGHTED && lane < n ? ew[eb + lane] : 1.f;
        if constexpr (REDUCE == GNNREC_REDUCE_MAX) {
          // first edge (CSR order) whose message equals the forward maximum, per column;
          // 8 edges' values are loaded before any compare so 8·NC loads are in flight
          constexpr int kB = 8;
          for (int k0 = 0; k0 < n; k0 += kB) {
            float m[kB][NC], wv[kB];
            int64_t uv[kB];
#pragma unroll
            for (int q = 0; q < kB; ++q) {
              const bool ok = k0 + q < n;
              uv[q] = __shfl(my_u, ok ? k0 + q : 0);
              wv[q] = WEIGHTED ? __shfl(my_w, ok ? k0 + q : 0) : 1.f;
              const float* xr = X + uv[q] * ldx + c0 + lane;
#pragma unroll
              for (int j = 0; j < NC; ++j) m[q][j] = (ok && live[j]) ? xr[kWave * j] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < kB; ++q) {
              if (k0 + q >= n) break;
              float* gr = gX + uv[q] * ldgx + c0 + lane;
#pragma unroll
              for (int j = 0; j < NC; ++j) {
                if (!live[j]) continue;
                const float mv = WEIGHTED ? m[q][j] * wv[q] : m[q][j];
                if (mv == y[j]) {
                  unsafeAtomicAdd(gr + kWave * j, WEIGHTED ? g[j] * wv[q] : g[j]);
                  live[j] = false;
                }
              }
            }
          }
          bool any = false;
#pragma unroll
          for (int j = 0; j < NC; ++j) any |= live[j];
          if (__ballot(any) == 0) break;
        } else {
          for (int k = 0; k < n; ++k) {
            const int64_t u = __shfl(my_u, k);
            const float w = WEIGHTED ? __shfl(my_w, k) : 1.f;
            float* gr = gX + u * ldgx + c0 + lane;
#pragma unroll
            for (int j = 0; j < NC; ++j)
              if (live[j]) unsafeAtomicAdd(gr + kWave * j, WEIGHTED ? g[j] * w : g[j]);
          }
        }
      }
    }
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_spmm_backward_f32(const int64_t* indptr, const int32_t* indices,
                                        const float* ew, const float* grad_out, int64_t ldg,
                                        const float* X, int64_t ldx, const float* out,
                                        int64_t ldo, int64_t n_dst, int64_t d, int reduce,
                                        float* grad_X, int64_t ldgx, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_dst >= 0 && d >= 0, "gnnrec_spmm_backward_f32: negative size");
  if (n_dst == 0 || d == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr && grad_out && grad_X, "gnnrec_spmm_backward_f32: null pointer");
  GNNREC_REQUIRE(reduce != GNNREC_REDUCE_MAX || (X && out),
                 "gnnrec_spmm_backward_f32: max needs the forward input and output");
  hipStream_t s = as_stream(stream);
  const unsigned grid = grid_waves(n_dst);
#define GNNREC_BWD_NC(R, W, NC)                                                               \
  hipLaunchKernelGGL((spmm_backward_kernel<R, W, NC>), dim3(grid), dim3(256), 0, s, indptr,      \
                     indices, ew, grad_out, ldg, X, ldx, out, ldo, n_dst, (int)d, grad_X, ldgx)
#define GNNREC_BWD_W(R, W)                                                                    \
  if (d <= 64) GNNREC_BWD_NC(R, W, 1);                                                        \
  else if (d <= 128) GNNREC_BWD_NC(R, W, 2);                                                  \
  else GNNREC_BWD_NC(R, W, 4);
#define GNNREC_BWD(R)                                                                         \
  if (ew) { GNNREC_BWD_W(R, true) } else { GNNREC_BWD_W(R, false) }
  switch (reduce) {
    case GNNREC_REDUCE_SUM: GNNREC_BWD(GNNREC_REDUCE_SUM) break;
    case GNNREC_REDUCE_MEAN: GNNREC_BWD(GNNREC_REDUCE_MEAN) break;
    case GNNREC_REDUCE_MAX: GNNREC_BWD(GNNREC_REDUCE_MAX) break;
    default: GNNREC_REQUIRE(false, "gnnrec_spmm_backward_f32: unknown reduce %d", reduce);
  }
#undef GNNREC_BWD
#undef GNNREC_BWD_W
#undef GNNREC_BWD_NC
  return check_launch("gnnrec_spmm_backward_f32");
}

extern "C" int gnnrec_spmm_csr2_f32(const int64_t* indptr_a, const int32_t* indices_a,
                                    const float* ew_a, const int64_t* indptr_b,
                                    const int32_t* indices_b, const float* ew_b, const float* X,
                                    int64_t ldx, int64_t n_dst, int64_t d, int reduce, int flags,
                                    float* out_a, float* out_b, int64_t ldo, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_dst >= 0 && d >= 0, "gnnrec_spmm_csr2_f32: negative size");
  GNNREC_REQUIRE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN ||
                     reduce == GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_csr2_f32: unknown reduce %d", reduce);
  GNNREC_REQUIRE((ew_a == nullptr) == (ew_b == nullptr),
                 "gnnrec_spmm_csr2_f32: edge weights on both relations or on neither");
  if (n_dst == 0 || d == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr_a && indptr_b && X && out_a && out_b, "gnnrec_spmm_csr2_f32: null pointer");
  GNNREC_REQUIRE(d % 4 == 0 && d <= 256 && ldx % 4 == 0 && ldo % 4 == 0 && ldx >= d && ldo >= d &&
                     aligned16(X) && aligned16(out_a) && aligned16(out_b),
                 "gnnrec_spmm_csr2_f32: needs d %% 4 == 0, d <= 256 and 16-B aligned rows");
  Csr2 c{{indptr_a, indptr_b}, {indices_a, indices_b}, {ew_a, ew_b}, {out_a, out_b}};
  hipStream_t s = as_stream(stream);
  const int eni = flags & (GNNREC_SPMM_EMPTY_NEGINF | GNNREC_SPMM_ACCUM);
  int lpr = 4;
  while (lpr < d / 4 && lpr < 64) lpr <<= 1;
#define GNNREC_CSR2(L)                                                                        \
  do {                                                                                        \
    const bool w = ew_a != nullptr;                                                           \
    if (reduce == GNNREC_REDUCE_SUM)                                                          \
      return w ? launch_csr2<L, GNNREC_REDUCE_SUM, true>(c, X, ldx, n_dst, (int)d, ldo, eni, s)  \
               : launch_csr2<L, GNNREC_REDUCE_SUM, false>(c, X, ldx, n_dst, (int)d, ldo, eni, s); \
    if (reduce == GNNREC_REDUCE_MEAN)                                                         \
      return w ? launch_csr2<L, GNNREC_REDUCE_MEAN, true>(c, X, ldx, n_dst, (int)d, ldo, eni, s) \
               : launch_csr2<L, GNNREC_REDUCE_MEAN, false>(c, X, ldx, n_dst, (int)d, ldo, eni, s); \
    return w ? launch_csr2<L, GNNREC_REDUCE_MAX, true>(c, X, ldx, n_dst, (int)d, ldo, eni, s)    \
             : launch_csr2<L, GNNREC_REDUCE_MAX, false>(c, X, ldx, n_dst, (int)d, ldo, eni, s);  \
  } while (0)
  switch (lpr) {
    case 4: GNNREC_CSR2(4);
    case 8: GNNREC_CSR2(8);
    case 16: GNNREC_CSR2(16);
    case 32: GNNREC_CSR2(32);
    default: GNNREC_CSR2(64);
  }
#undef GNNREC_CSR2
}
