// a9 — block sampler building blocks (DGL MultiLayerFullNeighborSampler /
// MultiLayerNeighborSampler + to_block), reference src/sampling.py:153-161,
// main_inference.py:129-138; DGL 0.5.2 semantics restated:
//   * frontier = in-edges of the seeds (all of them, or `fanout` of them drawn
//     without replacement), THEN edges whose eid is excluded are removed
//     (BlockSampler.sample_blocks removes exclude_eids after sampling);
//   * to_block: per node type, dst nodes form the prefix of the src nodes, new
//     src nodes follow.  DGL orders them by first appearance (hash map); this
//     build orders them ascending by global id (a set-equal, deterministic
//     choice — see DESIGN.md §parity).
// Pipeline per relation: count -> exclusive scan -> fill; per node type:
// mark -> scan -> compact (new src ids) -> relabel (local src ids).
#include "common.hpp"
#include "rowq.hpp"
#include "sampler.hpp"

namespace gnnrec {
namespace {

constexpr int kBlock = 256;

template <int G>
__global__ __launch_bounds__(kBlock) void sample_count_kernel(
    const int64_t* __restrict__ indptr, const int64_t* __restrict__ eids,
    const uint8_t* __restrict__ excluded_all, const uint8_t* __restrict__ xrows,
    const int64_t* __restrict__ seeds, int64_t n_seeds, int64_t fanout, uint64_t key,
    int64_t* __restrict__ counts) {
  const Group<G> grp;
  const int64_t i = (int64_t)blockIdx.x * (kBlock / G) + (threadIdx.x / G);
  if (i >= n_seeds) return;  // uniform per group; groups never share a ballot result
  const int64_t v = seeds[i];
  const int64_t beg = indptr[v], end = indptr[v + 1], deg = end - beg;
  // xrows[v] == 0: none of v's in-edges is excluded (the exclusions are one batch's edges),
  // so v's count needs neither its picks nor their eids
  const uint8_t* const excluded = excluded_all && (!xrows || xrows[v]) ? excluded_all : nullptr;
  int64_t c;
  if (fanout < 0 || deg <= fanout) {
    if (!excluded) {
      c = deg;
    } else {
      c = 0;
      for (int64_t e0 = beg; e0 < end; e0 += G) {
        const int64_t e = e0 + grp.lane;
        c += __popcll(grp.ballot(e < end && !excluded[eids[e]]));
      }
    }
  } else if (!excluded) {
    c = fanout;
  } else {
    const int64_t p = floyd_pick(grp, key, v, deg, (int)fanout);
    c = __popcll(grp.ballot(p >= 0 && !excluded[eids[beg + p]]));
  }
  if (grp.lane == 0) counts[i] = c;
}

template <int G>
__global__ __launch_bounds__(kBlock) void sample_fill_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const int64_t* __restrict__ eids, const uint8_t* __restrict__ excluded_all,
    const uint8_t* __restrict__ xrows, const int64_t* __restrict__ seeds, int64_t n_seeds,
    int64_t fanout, uint64_t key, const int64_t* __restrict__ out_indptr,
    int64_t* __restrict__ out_src, int64_t* __restrict__ out_eid) {
  const Group<G> grp;
  const int64_t i = (int64_t)blockIdx.x * (kBlock / G) + (threadIdx.x / G);
  if (i >= n_seeds) return;
  const int64_t v = seeds[i];
  const int64_t beg = indptr[v], end = indptr[v + 1], deg = end - beg;
  const uint8_t* const excluded = excluded_all && (!xrows || xrows[v]) ? excluded_all : nullptr;
  int64_t o = out_indptr[i];
  if (fanout < 0 || deg <= fanout) {
    // whole row in edge order; two chunks in flight per iteration
    for (int64_t e0 = beg; e0 < end; e0 += 2 * G) {
      const int64_t ea = e0 + grp.lane, eb = ea + G;
      const bool va = ea < end, vb = eb < end;
      const int64_t ida = va ? eids[ea] : 0, idb = vb ? eids[eb] : 0;
      const int32_t sa = va ? indices[ea] : 0, sb = vb ? indices[eb] : 0;
      const bool ka = va && !(excluded && excluded[ida]);
      const bool kb = vb && !(excluded && excluded[idb]);
      const uint64_t ma = grp.ballot(ka), mb = grp.ballot(kb);
      if (ka) {
        const int64_t q = o + grp.below(ma);
        out_src[q] = sa;
        out_eid[q] = ida;
      }
      o += __popcll(ma);
      if (kb) {
        const int64_t q = o + grp.below(mb);
        out_src[q] = sb;
        out_eid[q] = idb;
      }
      o += __popcll(mb);
    }
  } else {
    const int k = (int)fanout;
    const int64_t p = floyd_pick(grp, key, v, deg, k);
    const bool valid = p >= 0;
    const int64_t e = beg + (valid ? p : 0);
    const int64_t id = valid ? eids[e] : 0;
    const bool keep = valid && !(excluded && excluded[id]);
    int slot = 0;
    for (int r = 0; r < k; ++r) {
      const int64_t pr = __shfl(p, grp.base + r);
      const int kr = __shfl((int)keep, grp.base + r);
      slot += (kr && pr < p) ? 1 : 0;
    }
    if (keep) {
      out_src[o + slot] = indices[e];
      out_eid[o + slot] = id;
    }
  }
}

// ---------------------------------------------------------------- scan -----
constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;  // per thread
constexpr int kScanTile = kScanBlock * kScanItems;

template <typename T>
__device__ int64_t block_exclusive_scan(int64_t x, int64_t* sh) {
  // x: per-thread value; returns exclusive prefix within block; sh[kScanBlock] scratch
  const int t = threadIdx.x;
  sh[t] = x;
  __syncthreads();
  for (int off = 1; off < kScanBlock; off <<= 1) {
    const int64_t y = t >= off ? sh[t - off] : 0;
    __syncthreads();
    sh[t] += y;
    __syncthreads();
  }
  const int64_t incl = sh[t];
  return incl - x;
}

template <typename T>
__global__ __launch_bounds__(kScanBlock) void scan_tile_sums(const T* __restrict__ in, int64_t n,
                                                             int64_t* __restrict__ sums) {
  __shared__ int64_t sh[kScanBlock];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j)
    if (base + j < n) s += (int64_t)in[base + j];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int off = kScanBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = sh[0];
}

// single block: exclusive scan of the tile sums in place, total at sums[n]
__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(int64_t* __restrict__ sums,
                                                               int64_t n) {
  __shared__ int64_t sh[kScanBlock];
  int64_t carry = 0;
  for (int64_t b = 0; b < n; b += kScanBlock) {
    const int64_t i = b + threadIdx.x;
    const int64_t x = i < n ? sums[i] : 0;
    const int64_t ex = block_exclusive_scan<int64_t>(x, sh);
    const int64_t tot = sh[kScanBlock - 1];
    __syncthreads();
    if (i < n) sums[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[n] = carry;
}

template <typename T>
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const T* in, int64_t n,
                                                                const int64_t* __restrict__ sums,
                                                                int64_t* out) {
  __shared__ int64_t sh[kScanBlock];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t vals[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    vals[j] = base + j < n ? (int64_t)in[base + j] : 0;
    s += vals[j];
  }
  __syncthreads();  // in may alias out: all reads of this tile precede writes
  int64_t run = block_exclusive_scan<int64_t>(s, sh) + sums[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j < n) out[base + j] = run;
    run += vals[j];
  }
  const int64_t n_tiles = (n + kScanTile - 1) / kScanTile;
  if (blockIdx.x == n_tiles - 1 && threadIdx.x == kScanBlock - 1) out[n] = sums[n_tiles];
}

// arrays of up to kScan1Tile entries (the sampler's per-seed counts, the radix sort's digit
// tables of a block CSR): one launch of one 1024-thread block instead of three
constexpr int kScan1Block = 1024;
constexpr int kScan1Items = 16;
constexpr int64_t kScan1Tile = (int64_t)kScan1Block * kScan1Items;

template <typename T>
__global__ __launch_bounds__(kScan1Block) void scan_one_block_kernel(const T* in, int64_t n,
                                                                    int64_t* out) {
  __shared__ int64_t sh[kScan1Block];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)t * kScan1Items;
  int64_t vals[kScan1Items];
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kScan1Items; ++j) {
    vals[j] = base + j < n ? (int64_t)in[base + j] : 0;
    s += vals[j];
  }
  sh[t] = s;
  __syncthreads();  // (in may alias out: every read above precedes the writes below)
  for (int off = 1; off < kScan1Block; off <<= 1) {
    const int64_t y = t >= off ? sh[t - off] : 0;
    __syncthreads();
    sh[t] += y;
    __syncthreads();
  }
  int64_t run = sh[t] - s;
#pragma unroll
  for (int j = 0; j < kScan1Items; ++j) {
    if (base + j < n) out[base + j] = run;
    run += vals[j];
  }
  if (t == kScan1Block - 1) out[n] = run;  // the total
}

// ---- single pass: chained tiles with decoupled look-back ------------------------------
// One launch instead of three (tile sums, their scan, apply) and one read of the input:
// a block takes the next tile in dispatch order (atomic tile counter), publishes its
// aggregate, and its first wave walks back over the predecessors' flags — 64 at a time —
// until one that holds an inclusive prefix; then it publishes its own inclusive prefix.
// A tile waits only on tiles taken before it, by blocks already running, so every wave
// finishes.  Flags are 64-bit words: status in the top 2 bits (0 none, 1 aggregate,
// 2 inclusive), a signed 62-bit value below.  The slot (rowq.hpp: scan_slot) is zero
// between users: the last block out resets the counters and the flags it used.
// The minibatch step scans its relabel marks (1M users, 100k items) and per-seed counts
// about 14 times per step: ~290 µs over 40-odd launches in three-kernel form (C2 trace).
constexpr int kCsThreads = 256;
constexpr int kCsItems = 16;
constexpr int64_t kCsTile = (int64_t)kCsThreads * kCsItems;
constexpr unsigned long long kCsAgg = 1ull << 62, kCsIncl = 2ull << 62;

__device__ __forceinline__ unsigned long long cs_pack(unsigned long long status, int64_t v) {
  return status | ((unsigned long long)v & ((1ull << 62) - 1));
}
__device__ __forceinline__ int64_t cs_value(unsigned long long f) {
  return (int64_t)(f << 2) >> 2;  // sign-extend the 62-bit value
}

// exclusive scan of one value per thread over the block (wave shuffles, 2 barriers);
// *total = the block's sum
__device__ __forceinline__ int64_t cs_block_scan(int64_t x, int64_t* wsum, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t v = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(v, off);
    if (lane >= off) v += y;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  constexpr int NW = kCsThreads / 64;
  int64_t before = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int64_t s = wsum[i];
    if (i < w) before += s;
    tot += s;
  }
  *total = tot;
  return before + v - x;
}

template <typename T>
__global__ __launch_bounds__(kCsThreads) void scan_chained_kernel(const T* in, int64_t n,
                                                                  int64_t* out,
                                                                  unsigned long long* slot,
                                                                  int64_t n_tiles) {
  __shared__ int64_t wsum[kCsThreads / 64];
  __shared__ int64_t sh_tile, sh_prefix;
  __shared__ int sh_last;
  // the tile staged through LDS: loaded and stored coalesced (lane i of a wave on element
  // i), scanned blocked (16 consecutive elements per thread); one pad word per 16 keeps the
  // blocked reads off a single bank group
  __shared__ int64_t stage[kCsTile + kCsTile / kCsItems];
  // slot == nullptr: a one-tile scan (no predecessors, no counters)
  unsigned long long* flags = slot ? slot + kScanFlags0 : nullptr;
  if (threadIdx.x == 0)
    sh_tile = slot ? (int64_t)__hip_atomic_fetch_add(slot, 1ull, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)
                   : 0;
  __syncthreads();
  const int64_t tile = sh_tile;
  const int64_t t0 = tile * kCsTile;
  auto pad = [](int i) { return i + i / kCsItems; };
#pragma unroll
  for (int j = 0; j < kCsItems; ++j) {
    const int i = j * kCsThreads + threadIdx.x;
    stage[pad(i)] = t0 + i < n ? (int64_t)in[t0 + i] : 0;
  }
  __syncthreads();
  int64_t vals[kCsItems];
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kCsItems; ++j) {
    vals[j] = stage[pad(threadIdx.x * kCsItems + j)];
    s += vals[j];
  }
  int64_t agg;
  const int64_t ex = cs_block_scan(s, wsum, &agg);  // (its barrier: every read of in is done)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (slot == nullptr) {
      if (lane == 0) sh_prefix = 0;
    } else if (tile == 0) {
      if (lane == 0) {
        __hip_atomic_store(flags, cs_pack(kCsIncl, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        sh_prefix = 0;
      }
    } else {
      if (lane == 0)
        __hip_atomic_store(flags + tile, cs_pack(kCsAgg, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      int64_t prefix = 0;
      for (int64_t j = tile - 1;; j -= 64) {  // window [j - 63, j], nearest first
        const int64_t idx = j - lane;
        unsigned long long f = kCsIncl;  // before tile 0: an inclusive prefix of 0
        if (idx >= 0) {
          f = __hip_atomic_load(flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          while ((f >> 62) == 0) {
            __builtin_amdgcn_s_sleep(1);
            f = __hip_atomic_load(flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        const uint64_t incl = __ballot((f >> 62) == 2);
        const int stop = incl ? __builtin_ctzll(incl) : 64;
        int64_t v = lane <= stop ? cs_value(f) : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        prefix += v;
        if (incl) break;
      }
      if (lane == 0) {
        __hip_atomic_store(flags + tile, cs_pack(kCsIncl, prefix + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        sh_prefix = prefix;
      }
    }
  }
  __syncthreads();
  int64_t run = sh_prefix + ex;
#pragma unroll
  for (int j = 0; j < kCsItems; ++j) {
    stage[pad(threadIdx.x * kCsItems + j)] = run;
    run += vals[j];
  }
  if (tile == n_tiles - 1 && threadIdx.x == kCsThreads - 1) out[n] = run;  // the total
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kCsItems; ++j) {
    const int i = j * kCsThreads + threadIdx.x;
    if (t0 + i < n) out[t0 + i] = stage[pad(i)];
  }
  if (slot == nullptr) return;
  // count the block out; the last one resets the slot for its next user
  if (threadIdx.x == 0)
    sh_last = __hip_atomic_fetch_add(slot + 1, 1ull, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) == (unsigned long long)n_tiles - 1;
  __syncthreads();
  if (sh_last) {
    for (int64_t t = threadIdx.x; t < n_tiles; t += kCsThreads)
      __hip_atomic_store(flags + t, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) {
      __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(slot + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <typename T>
int exclusive_scan(const T* in, int64_t n, int64_t* out, void* workspace, hipStream_t s) {
  GNNREC_REQUIRE(n >= 0, "scan: negative n");
  if (n == 0) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(int64_t), s);
    if (e != hipSuccess) {
      set_error("scan: %s", hipGetErrorString(e));
      return GNNREC_EHIP;
    }
    return GNNREC_OK;
  }
  const int64_t cs_tiles = (n + kCsTile - 1) / kCsTile;
  if (cs_tiles == 1) {
    hipLaunchKernelGGL(scan_chained_kernel<T>, dim3(1), dim3(kCsThreads), 0, s, in, n, out,
                       nullptr, (int64_t)1);
    return check_launch("gnnrec_exclusive_scan");
  }
  if (cs_tiles <= kScanMaxTiles) {
    int ticket = -1;
    if (unsigned long long* slot = scan_slot(s, &ticket)) {
      hipLaunchKernelGGL(scan_chained_kernel<T>, dim3((unsigned)cs_tiles), dim3(kCsThreads), 0, s,
                         in, n, out, slot, cs_tiles);
      scan_launched(ticket, s);
      return check_launch("gnnrec_exclusive_scan");
    }
  }
  if (n <= kScan1Tile) {
    hipLaunchKernelGGL(scan_one_block_kernel<T>, dim3(1), dim3(kScan1Block), 0, s, in, n, out);
    return check_launch("gnnrec_exclusive_scan");
  }
  GNNREC_REQUIRE(workspace != nullptr, "scan: null workspace");
  const int64_t n_tiles = (n + kScanTile - 1) / kScanTile;
  int64_t* sums = reinterpret_cast<int64_t*>(workspace);
  hipLaunchKernelGGL(scan_tile_sums<T>, dim3((unsigned)n_tiles), dim3(kScanBlock), 0, s, in, n,
                     sums);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanBlock), 0, s, sums, n_tiles);
  hipLaunchKernelGGL(scan_apply_kernel<T>, dim3((unsigned)n_tiles), dim3(kScanBlock), 0, s, in, n,
                     sums, out);
  return check_launch("gnnrec_exclusive_scan");
}

// -------------------------------------------------------------- relabel ----
__global__ void mark_ids_kernel(const int64_t* __restrict__ ids, int64_t n,
                                const int64_t* __restrict__ prefix_pos, int32_t* __restrict__ mark) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  if (id < 0) return;  // unused capacity of a bounded sample buffer
  if (prefix_pos[id] < 0) mark[id] = 1;  // benign race: all writers store 1
}

__global__ void relabel_kernel(const int64_t* __restrict__ ids, int64_t n,
                               const int64_t* __restrict__ prefix_pos,
                               const int64_t* __restrict__ rank, int64_t n_prefix,
                               int64_t* __restrict__ local) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t id = ids[i];
  if (id < 0) {  // unused capacity of a bounded sample buffer
    local[i] = -1;
    return;
  }
  const int64_t p = prefix_pos[id];
  local[i] = p >= 0 ? p : n_prefix + rank[id];
}

__global__ void compact_kernel(const int32_t* __restrict__ mark, const int64_t* __restrict__ rank,
                               int64_t n_nodes, int64_t* __restrict__ out_ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_nodes) return;
  if (mark[i]) out_ids[rank[i]] = i;
}

__global__ void set_prefix_kernel(const int64_t* __restrict__ prefix, int64_t n,
                                  int64_t* __restrict__ prefix_pos, int clear) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  prefix_pos[prefix[i]] = clear ? -1 : i;
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_sample_count(const int64_t* indptr, const int64_t* eids,
                                   const uint8_t* excluded, const uint8_t* excluded_rows,
                                   const int64_t* seeds, int64_t n_seeds, int64_t fanout,
                                   uint64_t seed_key, int64_t* counts, void* stream) {
  GNNREC_REQUIRE(n_seeds >= 0, "gnnrec_sample_count: negative n_seeds");
  GNNREC_REQUIRE(fanout < 0 || fanout <= kMaxFanout, "gnnrec_sample_count: fanout > %d",
                 kMaxFanout);
  GNNREC_REQUIRE(!excluded || eids, "gnnrec_sample_count: exclusion needs eids");
  if (n_seeds == 0) return GNNREC_OK;
  const int G = group_size(fanout);
  const dim3 grid((unsigned)((n_seeds + kBlock / G - 1) / (kBlock / G)));
#define GNNREC_COUNT(g)                                                                     \
  hipLaunchKernelGGL(sample_count_kernel<g>, grid, dim3(kBlock), 0, as_stream(stream), indptr, \
                     eids, excluded, excluded_rows, seeds, n_seeds, fanout, seed_key, counts)
  switch (G) {
    case 8: GNNREC_COUNT(8); break;
    case 16: GNNREC_COUNT(16); break;
    case 32: GNNREC_COUNT(32); break;
    default: GNNREC_COUNT(64); break;
  }
#undef GNNREC_COUNT
  return check_launch("gnnrec_sample_count");
}

extern "C" int gnnrec_sample_fill(const int64_t* indptr, const int32_t* indices,
                                  const int64_t* eids, const uint8_t* excluded,
                                  const uint8_t* excluded_rows,
                                  const int64_t* seeds, int64_t n_seeds, int64_t fanout,
                                  uint64_t seed_key, const int64_t* out_indptr, int64_t* out_src,
                                  int64_t* out_eid, void* stream) {
  GNNREC_REQUIRE(n_seeds >= 0, "gnnrec_sample_fill: negative n_seeds");
  GNNREC_REQUIRE(fanout < 0 || fanout <= kMaxFanout, "gnnrec_sample_fill: fanout > %d",
                 kMaxFanout);
  if (n_seeds == 0) return GNNREC_OK;
  const int G = group_size(fanout);
  const dim3 grid((unsigned)((n_seeds + kBlock / G - 1) / (kBlock / G)));
#define GNNREC_FILL(g)                                                                      \
  hipLaunchKernelGGL(sample_fill_kernel<g>, grid, dim3(kBlock), 0, as_stream(stream), indptr,  \
                     indices, eids, excluded, excluded_rows, seeds, n_seeds, fanout, seed_key, \
                     out_indptr, out_src, out_eid)
  switch (G) {
    case 8: GNNREC_FILL(8); break;
    case 16: GNNREC_FILL(16); break;
    case 32: GNNREC_FILL(32); break;
    default: GNNREC_FILL(64); break;
  }
#undef GNNREC_FILL
  return check_launch("gnnrec_sample_fill");
}

extern "C" int64_t gnnrec_scan_workspace_bytes(int64_t n) {
  const int64_t n_tiles = (n + kScanTile - 1) / kScanTile;
  return (n_tiles + 1) * (int64_t)sizeof(int64_t);
}

extern "C" int gnnrec_exclusive_scan_i64(const int64_t* in, int64_t n, int64_t* out,
                                         void* workspace, void* stream) {
  return exclusive_scan<int64_t>(in, n, out, workspace, as_stream(stream));
}

extern "C" int gnnrec_exclusive_scan_i32(const int32_t* in, int64_t n, int64_t* out,
                                         void* workspace, void* stream) {
  return exclusive_scan<int32_t>(in, n, out, workspace, as_stream(stream));
}

extern "C" int gnnrec_mark_ids(const int64_t* ids, int64_t n, const int64_t* prefix_pos,
                               int32_t* mark, void* stream) {
  if (n <= 0) return GNNREC_OK;
  hipLaunchKernelGGL(mark_ids_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), ids, n,
                     prefix_pos, mark);
  return check_launch("gnnrec_mark_ids");
}

extern "C" int gnnrec_relabel_ids(const int64_t* ids, int64_t n, const int64_t* prefix_pos,
                                  const int64_t* rank, int64_t n_prefix, int64_t* local,
                                  void* stream) {
  if (n <= 0) return GNNREC_OK;
  hipLaunchKernelGGL(relabel_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), ids, n,
                     prefix_pos, rank, n_prefix, local);
  return check_launch("gnnrec_relabel_ids");
}

extern "C" int gnnrec_compact_marked(const int32_t* mark, const int64_t* rank, int64_t n_nodes,
                                     int64_t* out_ids, void* stream) {
  if (n_nodes <= 0) return GNNREC_OK;
  hipLaunchKernelGGL(compact_kernel, dim3(nblk(n_nodes)), dim3(256), 0, as_stream(stream), mark,
                     rank, n_nodes, out_ids);
  return check_launch("gnnrec_compact_marked");
}

extern "C" int gnnrec_set_prefix_pos(const int64_t* prefix, int64_t n, int64_t* prefix_pos,
                                     void* stream) {
  if (n <= 0) return GNNREC_OK;
  hipLaunchKernelGGL(set_prefix_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), prefix, n,
                     prefix_pos, 0);
  return check_launch("gnnrec_set_prefix_pos");
}

extern "C" int gnnrec_clear_prefix_pos(const int64_t* prefix, int64_t n, int64_t* prefix_pos,
                                       void* stream) {
  if (n <= 0) return GNNREC_OK;
  hipLaunchKernelGGL(set_prefix_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), prefix, n,
                     prefix_pos, 1);
  return check_launch("gnnrec_clear_prefix_pos");
}
