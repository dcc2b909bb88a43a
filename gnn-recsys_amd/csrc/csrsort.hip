// f3 — COO -> CSR construction on the device: a stable LSD radix sort of the row keys.
//
// Reference: create_graph / dgl.heterograph (src/builder.py:377-383) and the reverse
// relations of src/utils_data.py:204-238, whose in-CSR DGL builds when update_all first
// runs; the CSR keeps the edges of a row in edge-id order.  Here: per pass of DB key bits
// (radix_plan: the fewest passes of at most 10 bits, then the narrowest digit that many
// passes need — 17-bit keys in 2 passes of 9, 20-bit in 2 of 10, 24-bit in 3 of 8),
//   radix_hist    one 256-thread block per tile (4096 edges, 2048 below 512 such tiles) counts
//                 the tile's digits,
//                 stored digit-major [2^DB][tiles];
//   scan          exclusive scan of that table (gnnrec_exclusive_scan_i32): the first
//                 output position of every (digit, tile);
//   radix_scatter each wave ranks its quarter of the tile, 64 edges at a time, by digit: DB
//                 ballots give the lanes holding the same digit, mbcnt the rank among them,
//                 and an LDS counter per (wave, digit) the edges of earlier rounds — so
//                 equal digits keep their input order (stable); the tile is placed in LDS
//                 in output order and written out by consecutive threads (runs of a digit).
// The final pass writes the CSR directly (indices = src[e], eids = e), and the row
// pointers come from the sorted keys' run boundaries.  Bytes per edge per pass: 4 (hist)
// + 8 read + 8 written (scatter) + 12 · 2^DB / 2048 for the digit table and its scan;
// C4's 500M-edge relation sorts in 3 passes.  The sorted order is unique (a stable sort by
// key), so the digit width changes launches and bytes, never the result.
#include "common.hpp"
#include "csrsort.hpp"

namespace gnnrec {
namespace {

constexpr int kRT = 256;                 // threads per tile block
// 64-edge rounds per wave: 16 (4096-edge tiles: the scatter writes longer runs) when that
// still gives at least 512 tiles, else 8 (2048-edge tiles: enough blocks for the chip)
inline int radix_rounds(int64_t E) { return (E + kRT * 16 - 1) / (kRT * 16) >= 512 ? 16 : 8; }
inline int64_t radix_tiles(int64_t E) {
  const int64_t tile = (int64_t)kRT * radix_rounds(E);
  return (E + tile - 1) / tile;
}
constexpr int kMaxDigitBits = 10;

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct RadixPlan {
  int passes, bits;  // passes of `bits` key bits each
};
inline RadixPlan radix_plan(int64_t n_rows) {
  int b = 1;
  while (b < 32 && (int64_t(1) << b) < n_rows) ++b;
  RadixPlan r;
  r.passes = (b + kMaxDigitBits - 1) / kMaxDigitBits;
  r.bits = (b + r.passes - 1) / r.passes;
  if (r.bits < 8) r.bits = 8;
  return r;
}

inline unsigned tile_grid(int64_t n_tiles) {
  int64_t g = n_tiles < 256 * 16 ? n_tiles : 256 * 16;
  return (unsigned)(g < 1 ? 1 : g);
}

template <class K, int DB, int RR>
__global__ __launch_bounds__(kRT) void radix_hist_kernel(const K* __restrict__ keys, int64_t E,
                                                         int shift, int64_t n_tiles,
                                                         int32_t* __restrict__ hist) {
  constexpr int ND = 1 << DB;
  __shared__ int cnt[ND];
  const int tid = threadIdx.x;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
#pragma unroll
    for (int d = tid; d < ND; d += kRT) cnt[d] = 0;
    __syncthreads();
    const int64_t base = t * (kRT * RR);
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      const int64_t i = base + j * kRT + tid;
      if (i < E) atomicAdd(&cnt[((uint32_t)keys[i] >> shift) & (ND - 1)], 1);
    }
    __syncthreads();
#pragma unroll
    for (int d = tid; d < ND; d += kRT) hist[(int64_t)d * n_tiles + t] = cnt[d];
    __syncthreads();
  }
}

// MODE 0: keys_out / vals_out; MODE 1: keys_out + the CSR gather (idx_out, eid_out)
// (positions fit int32: E < 2^31, radix_sort_rows).  The tile's edges are first placed in
// LDS in their output order (digit-major, stable), then written out by consecutive threads:
// a digit's edges of the tile land in consecutive lanes, so a wave-instruction writes runs
// of the output instead of one 4-B store per digit region per lane.
template <class K, bool VIN, int MODE, int DB, int RR>
__global__ __launch_bounds__(kRT) void radix_scatter_kernel(
    const K* __restrict__ keys, const int32_t* __restrict__ vals, int64_t E, int shift,
    int64_t n_tiles, const int64_t* __restrict__ offs, uint32_t* __restrict__ keys_out,
    int32_t* __restrict__ vals_out, const int64_t* __restrict__ src,
    int32_t* __restrict__ idx_out, int64_t* __restrict__ eid_out) {
  constexpr int ND = 1 << DB;
  constexpr int NW = kRT / kWave;
  constexpr int PER = ND / kRT;  // digits per thread in the tile's digit scan (DB >= 8)
  static_assert(PER >= 1 && ND % kRT == 0, "at least one digit per thread");
  // per (wave, digit): the wave's running count, then (in place) its first tile position
  __shared__ int cnt[NW][ND];
  __shared__ int gbase[ND];        // a digit's first output position minus its first tile position
  constexpr int kRTile = kRT * RR;  // edges per tile
  __shared__ uint32_t skey[kRTile];
  __shared__ int32_t sval[kRTile];
  __shared__ int wtot[NW];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid >> 6;
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    for (int i = tid; i < NW * ND; i += kRT) cnt[i / ND][i % ND] = 0;
    __syncthreads();
    const int64_t base = t * kRTile + (int64_t)w * (RR * kWave);
    uint32_t kk[RR];
    int32_t vv[RR];
    uint32_t dr[RR];  // digit << 16 | rank among the wave's edges of that digit
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      const int64_t i = base + j * kWave + lane;
      const bool act = i < E;
      const uint32_t k = act ? (uint32_t)keys[i] : 0u;
      kk[j] = k;
      vv[j] = act ? (VIN ? vals[i] : (int32_t)i) : 0;
      const uint32_t d = (k >> shift) & (ND - 1);
      uint64_t peers = __ballot(act);
#pragma unroll
      for (int b = 0; b < DB; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bb : ~bb;
      }
      const unsigned r = __builtin_amdgcn_mbcnt_hi(
          (unsigned)(peers >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)peers, 0u));
      // every lane of a digit reads the wave's running count, then the lowest one adds the
      // round's count (one wave: the LDS sees the read before the write)
      const int old = act ? cnt[w][d] : 0;
      if (act && r == 0) cnt[w][d] = old + __popcll(peers);
      dr[j] = (d << 16) | (uint32_t)(old + (int)r);
    }
    __syncthreads();
    // the tile's digit starts: thread tid owns digits [tid PER, tid PER + PER); an exclusive
    // scan of the owners' totals over the block gives each its first tile position
    int own = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k)
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) own += cnt[ww][tid * PER + k];
    int inc = own;  // inclusive scan within the wave
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    if (lane == kWave - 1) wtot[w] = inc;
    __syncthreads();
    int run = inc - own;
    for (int ww = 0; ww < w; ++ww) run += wtot[ww];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int d = tid * PER + k;
      gbase[d] = (int)offs[(int64_t)d * n_tiles + t] - run;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        const int c = cnt[ww][d];
        cnt[ww][d] = run;
        run += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      const int64_t i = base + j * kWave + lane;
      if (i >= E) continue;
      const int q = cnt[w][dr[j] >> 16] + (int)(dr[j] & 0xffff);
      skey[q] = kk[j];
      sval[q] = vv[j];
    }
    __syncthreads();
    const int64_t rem = E - t * kRTile;
    const int n_here = rem < kRTile ? (int)rem : kRTile;
    for (int q = tid; q < n_here; q += kRT) {
      const uint32_t k = skey[q];
      const int32_t v = sval[q];
      const int64_t p = (int64_t)gbase[(k >> shift) & (ND - 1)] + q;
      if (keys_out) keys_out[p] = k;
      if (MODE == 0) {
        vals_out[p] = v;
      } else {
        idx_out[p] = (int32_t)src[v];
        eid_out[p] = v;
      }
    }
    __syncthreads();
  }
}

// first position in keys[lo, hi) with key >= r
__device__ __forceinline__ int64_t lower_bound_u32(const uint32_t* __restrict__ keys, int64_t lo,
                                                   int64_t hi, int64_t r) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)keys[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// row_ptr[r] = first sorted position with key >= r, one thread per row: the block finds its
// 256 rows' key span with two searches, each row searches inside that span.  (Run boundaries
// written by the edge after each run cost a serial loop over every empty row of a gap — a
// static-shape block's unused padding slots: 1.3 ms for one 130k-row gap.)
__global__ __launch_bounds__(256) void row_bounds_kernel(const uint32_t* __restrict__ keys,
                                                         int64_t E, int64_t n_rows,
                                                         int64_t* __restrict__ row_ptr) {
  __shared__ int64_t span[2];
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int64_t r1 = min(r0 + 256, n_rows + 1);
  if (threadIdx.x < 2) span[threadIdx.x] = lower_bound_u32(keys, 0, E, threadIdx.x ? r1 : r0);
  __syncthreads();
  const int64_t r = r0 + threadIdx.x;
  if (r < r1) row_ptr[r] = r == n_rows ? E : lower_bound_u32(keys, span[0], span[1], r);
}

__global__ __launch_bounds__(256) void zero_rows_kernel(int64_t* __restrict__ p, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0;
}

inline unsigned flat_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 256 * 16) b = 256 * 16;
  return (unsigned)(b < 1 ? 1 : b);
}

template <class K, int DB, int RR>
void launch_pass(const K* keys, const int32_t* vals, int64_t E, int shift, int64_t n_tiles,
                 int32_t* hist, int64_t* offs, void* scan_ws, uint32_t* k_out, int32_t* v_out,
                 const CsrGather* g, hipStream_t s) {
  const unsigned grid = tile_grid(n_tiles);
  hipLaunchKernelGGL((radix_hist_kernel<K, DB, RR>), dim3(grid), dim3(kRT), 0, s, keys, E, shift,
                     n_tiles, hist);
  (void)gnnrec_exclusive_scan_i32(hist, ((int64_t)1 << DB) * n_tiles, offs, scan_ws, s);
  const int64_t* src = g ? g->src : nullptr;
  int32_t* idx = g ? g->idx_out : nullptr;
  int64_t* eid = g ? g->eid_out : nullptr;
#define GNNREC_SCATTER(VIN, MODE)                                                        \
  hipLaunchKernelGGL((radix_scatter_kernel<K, VIN, MODE, DB, RR>), dim3(grid), dim3(kRT), 0, s, \
                     keys, vals, E, shift, n_tiles, offs, k_out, v_out, src, idx, eid)
  if (g) {
    if (vals) GNNREC_SCATTER(true, 1);
    else GNNREC_SCATTER(false, 1);
  } else {
    if (vals) GNNREC_SCATTER(true, 0);
    else GNNREC_SCATTER(false, 0);
  }
#undef GNNREC_SCATTER
}

template <class K, int RR>
void launch_pass_bits(int bits, const K* keys, const int32_t* vals, int64_t E, int shift,
                      int64_t n_tiles, int32_t* hist, int64_t* offs, void* scan_ws,
                      uint32_t* k_out, int32_t* v_out, const CsrGather* g, hipStream_t s) {
  if (bits == 8)
    launch_pass<K, 8, RR>(keys, vals, E, shift, n_tiles, hist, offs, scan_ws, k_out, v_out, g, s);
  else if (bits == 9)
    launch_pass<K, 9, RR>(keys, vals, E, shift, n_tiles, hist, offs, scan_ws, k_out, v_out, g, s);
  else
    launch_pass<K, 10, RR>(keys, vals, E, shift, n_tiles, hist, offs, scan_ws, k_out, v_out, g, s);
}

template <class K>
void launch_pass_tiles(int bits, const K* keys, const int32_t* vals, int64_t E, int shift,
                       int64_t n_tiles, int32_t* hist, int64_t* offs, void* scan_ws,
                       uint32_t* k_out, int32_t* v_out, const CsrGather* g, hipStream_t s) {
  if (radix_rounds(E) == 16)
    launch_pass_bits<K, 16>(bits, keys, vals, E, shift, n_tiles, hist, offs, scan_ws, k_out,
                            v_out, g, s);
  else
    launch_pass_bits<K, 8>(bits, keys, vals, E, shift, n_tiles, hist, offs, scan_ws, k_out,
                           v_out, g, s);
}

}  // namespace

size_t radix_ws_bytes(int64_t E, int64_t n_rows) {
  if (E <= 0) return 0;
  const int64_t n_tiles = radix_tiles(E);
  const int64_t n_hist = ((int64_t)1 << radix_plan(n_rows).bits) * n_tiles;
  return 4 * align_up((size_t)E * 4)                            // two (key, value) buffers
         + align_up((size_t)n_hist * 4)                         // per-tile digit counts
         + align_up((size_t)(n_hist + 1) * 8)                   // their scan
         + align_up((size_t)gnnrec_scan_workspace_bytes(n_hist));
}

int radix_sort_rows(const void* keys_in, bool keys64, const int32_t* vals_in, int64_t E,
                    int64_t n_rows, uint32_t* keys_out, int32_t* vals_out, const CsrGather* g,
                    int64_t* row_ptr, void* ws, size_t ws_bytes, hipStream_t s) {
  GNNREC_REQUIRE(E >= 0 && E < (int64_t(1) << 31) && n_rows >= 0 && n_rows < (int64_t(1) << 31),
                 "radix sort: %lld keys / %lld rows exceed the int32 range", (long long)E,
                 (long long)n_rows);
  if (E == 0) {
    if (row_ptr)
      hipLaunchKernelGGL(zero_rows_kernel, dim3(flat_grid(n_rows + 1)), dim3(256), 0, s, row_ptr,
                         n_rows + 1);
    return check_launch("radix sort");
  }
  GNNREC_REQUIRE(keys_in && ws && (g || vals_out) && (!row_ptr || keys_out),
                 "radix sort: null pointer");
  GNNREC_REQUIRE(ws_bytes >= radix_ws_bytes(E, n_rows), "radix sort: workspace %zu < %zu bytes",
                 ws_bytes, radix_ws_bytes(E, n_rows));
  const RadixPlan plan = radix_plan(n_rows);
  const int64_t n_tiles = radix_tiles(E);
  const int64_t n_hist = ((int64_t)1 << plan.bits) * n_tiles;
  char* p = static_cast<char*>(ws);
  const size_t slot = align_up((size_t)E * 4);
  uint32_t* kb[2] = {reinterpret_cast<uint32_t*>(p), reinterpret_cast<uint32_t*>(p + slot)};
  int32_t* vb[2] = {reinterpret_cast<int32_t*>(p + 2 * slot),
                    reinterpret_cast<int32_t*>(p + 3 * slot)};
  int32_t* hist = reinterpret_cast<int32_t*>(p + 4 * slot);
  int64_t* offs = reinterpret_cast<int64_t*>(p + 4 * slot + align_up((size_t)n_hist * 4));
  void* scan_ws = p + 4 * slot + align_up((size_t)n_hist * 4) + align_up((size_t)(n_hist + 1) * 8);
  const int bits = plan.bits;
  for (int ps = 0; ps < plan.passes; ++ps) {
    const bool last = ps == plan.passes - 1;
    uint32_t* k_out = last ? keys_out : kb[ps & 1];
    int32_t* v_out = last ? vals_out : vb[ps & 1];
    const CsrGather* gg = last ? g : nullptr;
    if (ps == 0) {
      if (keys64)
        launch_pass_tiles(bits, static_cast<const int64_t*>(keys_in), vals_in, E, 0, n_tiles,
                          hist, offs, scan_ws, k_out, v_out, gg, s);
      else
        launch_pass_tiles(bits, static_cast<const int32_t*>(keys_in), vals_in, E, 0, n_tiles,
                          hist, offs, scan_ws, k_out, v_out, gg, s);
    } else {
      launch_pass_tiles(bits, (const uint32_t*)kb[(ps - 1) & 1], vb[(ps - 1) & 1], E, bits * ps,
                        n_tiles, hist, offs, scan_ws, k_out, v_out, gg, s);
    }
  }
  if (row_ptr)
    hipLaunchKernelGGL(row_bounds_kernel, dim3((unsigned)((n_rows + 1 + 255) / 256)), dim3(256), 0,
                       s, keys_out, E, n_rows, row_ptr);
  return check_launch("radix sort");
}

}  // namespace gnnrec

extern "C" size_t gnnrec_csr_build_workspace_bytes(int64_t n_edges, int64_t n_dst) {
  using namespace gnnrec;
  if (n_edges <= 0) return 0;
  return align_up((size_t)n_edges * 4) + radix_ws_bytes(n_edges, n_dst);
}

extern "C" int gnnrec_csr_build(const int64_t* src, const int64_t* dst, int64_t n_edges,
                                int64_t n_dst, void* workspace, size_t workspace_bytes,
                                int64_t* indptr, int32_t* indices, int64_t* eids,
                                void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n_edges >= 0 && n_dst >= 0, "gnnrec_csr_build: negative size");
  GNNREC_REQUIRE(indptr, "gnnrec_csr_build: null indptr");
  hipStream_t s = as_stream(stream);
  if (n_edges == 0)
    return radix_sort_rows(nullptr, true, nullptr, 0, n_dst, nullptr, nullptr, nullptr, indptr,
                           nullptr, 0, s);
  GNNREC_REQUIRE(n_dst > 0, "gnnrec_csr_build: %lld edges into 0 rows", (long long)n_edges);
  GNNREC_REQUIRE(src && dst && indices && eids && workspace, "gnnrec_csr_build: null pointer");
  const size_t need = gnnrec_csr_build_workspace_bytes(n_edges, n_dst);
  GNNREC_REQUIRE(workspace_bytes >= need, "gnnrec_csr_build: workspace %zu < %zu bytes",
                 workspace_bytes, need);
  char* p = static_cast<char*>(workspace);
  uint32_t* keys = reinterpret_cast<uint32_t*>(p);  // sorted dst ids (for the row pointers)
  const size_t slot = align_up((size_t)n_edges * 4);
  CsrGather g;
  g.src = src;
  g.idx_out = indices;
  g.eid_out = eids;
  return radix_sort_rows(dst, true, nullptr, n_edges, n_dst, keys, nullptr, &g, indptr, p + slot,
                         workspace_bytes - slot, s);
}

// K10 — has_edges_between (reference src/train/run.py:95-101,160-166: the false-negative
// mask of the training loss, 1024 x K negative pairs per batch against the validation
// graph).  The membership CSR is the relation's in-CSR with each row's source ids in
// ascending order (gnnrec_csr_build over the edges taken in source order: the stable sort
// keeps that order inside a row), so a query (u, v) is one lower-bound search of row v:
// ceil(log2(deg + 1)) dependent 4-B loads, one thread per query, ids outside the node
// ranges answer false.
namespace gnnrec {
namespace {
__global__ __launch_bounds__(256) void has_edges_kernel(const int64_t* __restrict__ indptr,
                                                        const int32_t* __restrict__ idx,
                                                        int64_t n_dst, int64_t n_src,
                                                        const int64_t* __restrict__ u,
                                                        const int64_t* __restrict__ v, int64_t n,
                                                        uint8_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t a = __builtin_nontemporal_load(u + i), b = __builtin_nontemporal_load(v + i);
    uint8_t hit = 0;
    if (a >= 0 && a < n_src && b >= 0 && b < n_dst) {
      int64_t lo = indptr[b];
      const int64_t end = indptr[b + 1];
      int64_t hi = end;
      const int32_t key = (int32_t)a;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (idx[mid] < key) lo = mid + 1;
        else hi = mid;
      }
      hit = lo < end && idx[lo] == key;
    }
    __builtin_nontemporal_store(hit, out + i);
  }
}
}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_csr_has_edges(const int64_t* indptr, const int32_t* sorted_indices,
                                    int64_t n_dst, int64_t n_src, const int64_t* u,
                                    const int64_t* v, int64_t n, uint8_t* out, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n >= 0 && n_dst >= 0 && n_src >= 0 && n_src < (int64_t(1) << 31),
                 "gnnrec_csr_has_edges: bad sizes");
  if (n == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr && u && v && out,  // sorted_indices: null for an edgeless relation
                 "gnnrec_csr_has_edges: null pointer");
  hipLaunchKernelGGL(has_edges_kernel, dim3(flat_grid(n)), dim3(256), 0, as_stream(stream),
                     indptr, sorted_indices, n_dst, n_src, u, v, n, out);
  return check_launch("gnnrec_csr_has_edges");
}
