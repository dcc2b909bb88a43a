// a9 — every block of one bounded-fanout BlockSampler.sample_blocks call in 1 + 3L launches
// (reference src/sampling.py:153-161: MultiLayerNeighborSampler + to_block + exclude_eids,
// DGL 0.5.2's _CAPI_DGLSampleNeighbors / _CAPI_DGLToBlock per layer).  The blocks are
// bitwise those of the per-layer path (sampler.hip: count -> scan -> fill, mark -> scan ->
// compact -> relabel): the same Floyd picks in the same slots, the same local ids (a seed
// keeps its position, a new source follows the seeds in ascending global id).
//
// What changes is where the relabel state lives and how many launches it takes:
//   * seed positions: `pos[id]` = (stamp << 32) | ~position, int64 per node, two arrays per
//     type used alternately: step s reads the one its seeds were written to (by begin or by
//     step s-1's finalize) and its finalize writes step s+1's seeds (its source nodes) into
//     the other, so no kernel reads an array it writes.  A step's seeds are the entries
//     holding its stamp: nothing is ever cleared, and a call starts at a stamp no earlier
//     call used.  The position is stored complemented and written by atomicMax, so a seed
//     listed twice keeps its FIRST position, whatever the order the writes land in (DGL's
//     to_block hash map keeps the first insertion too).
//   * new sources: one BIT per node (a 1M-node type: 128 KB, not a 4 MB mark array and an
//     8 MB scan), ranked by a scan of the words' popcounts; two bitmaps per type, the pick
//     kernel of step s zeroing the one step s+1 uses (the other was read by step s-1).
//   * sizes stay on the device (`sizes`): step s+1's grids are sized by capacities
//     (seeds x fanout) and read the actual counts there, so one host read after the call
//     sizes every block (the per-layer path read back twice per layer).
//   * static shapes (plan.static_shapes): every block at its capacity, nothing to read back,
//     so a training step over it can be captured into a hipGraph.  Seed slots holding -1
//     (a suffix) are padding rows; after the seed rows each block gets D "dump" rows per
//     destination type, D = 1 + ceil(edge_cap / kDumpEdges) over the relations into it: a
//     padding row holds `fanout` padding edges, the dump rows the rest of the edge capacity
//     in runs of at most kDumpEdges (so no row is heavier than a heavy-row split: no plan,
//     no serial row anywhere), every padding edge from one of the source list's padding
//     slots (past the real sources, spread evenly; node_cap - 1 always is one) with eid -1.
//     The source list is the exact one — the real seeds, the new sources after them, at
//     the same positions — then -1 up to node_cap + D' entries, D' the next block's dump
//     rows (their index there starts at its seed_cap = this node_cap), so a layer's output
//     rows are the next block's source rows.  A padding row may sit over a real source's
//     slot: its output is garbage no real row reads, and its gradient is 0.
#include "common.hpp"
#include "sampler.hpp"

namespace gnnrec {
namespace {

constexpr int kSbBlock = 256;
constexpr int64_t kDumpEdges = 2048;  // a static block's dump row: at most ops.DEFAULT_SPLIT
constexpr int kScanThreads = 1024;
constexpr int kStrideBlocks = 2048;  // grid-stride sections (static padding): 8 per CU
constexpr int kMaxSec = 4 * GNNREC_SB_MAX_TYPES + 2 * GNNREC_SB_MAX_RELS;

struct RelArgs {
  const int64_t* indptr;
  const int32_t* indices;
  const int64_t* eids;
  const uint64_t* rec;  // packed {eid << 32 | src} per CSR edge (NULL: indices / eids); the
                        // picks then go to pick_eid packed the same way (pick_src unused)
  const uint8_t* excl_mask;  // NULL: nothing excluded in this call
  const uint8_t* excl_rows;
  int src_t, dst_t;
  int64_t fanout;
  uint64_t key;
  int64_t* counts;
  int32_t* pick_src;
  int64_t* pick_eid;
  int64_t* out_indptr;
  int32_t* out_src;
  int64_t* out_eid;
  int64_t* edge_total;  // sizes entry
  int64_t edge_cap;     // static shapes: the block's edge count (the dump rows end there)
  int64_t dump_rows;    // static shapes: the destination type's dump rows
  // exclusion flags set by begin, cleared by the last finalize
  const int64_t* excl_eids;
  int64_t n_excl;
  const int64_t* coo_dst;
  uint8_t* mask_w;
  uint8_t* rows_w;
};

struct TypeArgs {
  const int64_t* seeds;    // this step's destination nodes
  const int64_t* n_seeds;  // device count of the real seeds (sizes row s - 1)
  int64_t seed_cap;
  unsigned long long* pos_cur;   // this step's seed positions (read)
  unsigned long long* pos_next;  // the next step's (written by finalize)
  unsigned long long* bits_cur;
  unsigned long long* bits_next;
  // this step's seeds as one byte per node (set by begin / the previous finalize, by plain
  // byte stores like the new-source marks), the next step's written by finalize: the pick's
  // "is this source a seed" test reads a byte of a 1 MB array (a 1M-node type), not the
  // 8-byte stamped position of a random node (an 8 MB array)
  uint8_t* smark_cur;
  uint8_t* smark_next;
  uint8_t* mark_cur;       // new-source marks, one byte per node (64 * words), alternating
  uint8_t* mark_next;
  int64_t* word_rank;
  int64_t words;
  int64_t* nodes;          // this step's source node list (the next step's seeds)
  int64_t* n_nodes_out;    // sizes entry
  int64_t n_seeds_host;    // begin only: the batch's seed count
  int64_t node_cap;        // static shapes: the source list's length
  int64_t node_len;        // static shapes: node_cap + the next block's dump rows (all -1)
};

// sections of one launch: block ranges [begin[k], begin[k+1]) run job kind[k] on index idx[k]
struct Sections {
  int n;
  int kind[kMaxSec];
  int idx[kMaxSec];
  int begin[kMaxSec + 1];
  __device__ int find(int b) const {
    int k = 0;
    while (k + 1 < n && b >= begin[k + 1]) ++k;
    return k;
  }
};

struct StepArgs {
  int n_rels, n_types, last, stat;
  int64_t* overflow;  // static shapes with capacity hints: set when a batch does not fit
  uint32_t stamp;
  RelArgs rel[GNNREC_SB_MAX_RELS];
  TypeArgs type[GNNREC_SB_MAX_TYPES];
  Sections sec;
  int64_t* sizes_seed_row;  // begin: sizes row -1
  // the scan's chained tiles: per segment (relations, then types) a ticket word and one
  // flag word per tile, scan_stride words apart (zeroed by the step's pick kernel); the
  // scan's grid covers each segment's capacity in tiles from seg_block0
  unsigned long long* scan_ws;
  int64_t scan_stride, scan_words;
  int seg_block0[GNNREC_SB_MAX_RELS + GNNREC_SB_MAX_TYPES + 1];
};

enum { kSecSeedPos, kSecZeroBits, kSecExclSet, kSecPick, kSecZeroNext, kSecCompact,
       kSecNewNodes, kSecPrefix, kSecExclClear, kSecDumpEdges, kSecPadNodes, kSecZeroScan,
       kSecSeedClear };

// (stamp << 32) | ~position: the atomicMax of two writes of one stamp keeps the smaller
// position, and any write of a newer stamp beats every older entry
__device__ __forceinline__ unsigned long long pack_pos(uint32_t stamp, int64_t p) {
  return ((unsigned long long)stamp << 32) | (unsigned long long)(~(uint32_t)p);
}
__device__ __forceinline__ int64_t pos_of(unsigned long long v) {
  return (int64_t)(~(uint32_t)v);
}
__device__ __forceinline__ void set_pos(unsigned long long* pos, int64_t id, uint32_t stamp,
                                        int64_t p) {
  __hip_atomic_fetch_max(pos + id, pack_pos(stamp, p), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}

// 64 mark bytes (each 0 / 1) -> their word of the bitmap.  New sources are MARKED by plain
// byte stores, not OR-ed into the bitmap: at C2 the 1.1M picks of a step land on 100k items,
// ~700 atomic ORs per 64-item word, serialised at the L2 (the pick kernel's largest cost);
// the scan builds each word from its 64 bytes instead.
__device__ __forceinline__ unsigned long long word_of_marks(const uint8_t* __restrict__ m) {
  unsigned long long w = 0ull;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 x = reinterpret_cast<const uint4*>(m)[q];
    const uint32_t part[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        w |= (unsigned long long)((part[k] >> (8 * b)) & 1u) << (q * 16 + k * 4 + b);
  }
  return w;
}

// the destination rows of a step: the seeds, or (static shapes) the seed capacity
__device__ __forceinline__ int64_t seed_rows(const StepArgs& A, const TypeArgs& T) {
  return A.stat ? T.seed_cap : *T.n_seeds;
}

// ---------------------------------------------------------------- begin
__global__ __launch_bounds__(kSbBlock) void sb_begin_kernel(StepArgs A) {
  const int k = A.sec.find((int)blockIdx.x);
  const int64_t t = (int64_t)((int)blockIdx.x - A.sec.begin[k]) * kSbBlock + threadIdx.x;
  const int i = A.sec.idx[k];
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)A.n_types &&
      (!A.stat || A.type[threadIdx.x].n_seeds_host == 0))
    A.sizes_seed_row[threadIdx.x] = A.type[threadIdx.x].n_seeds_host;
  switch (A.sec.kind[k]) {
    case kSecSeedPos: {
      const TypeArgs& T = A.type[i];
      if (t >= T.n_seeds_host) break;
      const int64_t v = T.seeds[t];
      if (v >= 0) {
        set_pos(T.pos_cur, v, A.stamp, t);
        T.smark_cur[v] = 1;  // (zero: the previous call's last finalize cleared it)
      }
      // static shapes: the real seeds' count = the end of the non-negative prefix (one
      // writer: the last real seed, or slot 0 when there is none)
      if (A.stat && ((v >= 0 && (t + 1 == T.n_seeds_host || T.seeds[t + 1] < 0)) ||
                     (t == 0 && v < 0)))
        A.sizes_seed_row[i] = v >= 0 ? t + 1 : 0;
      break;
    }
    case kSecZeroBits: {  // the first step's marks (64 B per word, 16 B per thread)
      const TypeArgs& T = A.type[i];
      if (t < T.words * 4) reinterpret_cast<uint4*>(T.mark_cur)[t] = make_uint4(0, 0, 0, 0);
      break;
    }
    case kSecExclSet: {
      const RelArgs& R = A.rel[i];
      if (t < R.n_excl) {
        const int64_t e = R.excl_eids[t];
        R.mask_w[e] = 1;
        R.rows_w[R.coo_dst[e]] = 1;
      }
      break;
    }
    default: break;
  }
}

// ---------------------------------------------------------------- pick (step s)
// A group of G lanes per seed, SPG seeds per group: each of the seed -> indptr -> record
// chain's loads is issued for all SPG seeds before any is consumed, so a wave keeps
// SPG x (64 / G) seeds' round trips in flight (the kernel is bound by those dependent round
// trips: the K = 2500 first block's 0.8M seeds at one seed per group ran at 3 TB/s).  Each
// seed's picks, slots and counts are exactly the one-seed form's.
constexpr int kPickSpg = 2;

// Floyd's fanout of one seed's row (sampler.hpp floyd_pick: the same candidates, the same
// duplicate resolution, the same picks) with the group's candidates exchanged through LDS:
// each lane stores its step's candidate, every lane reads the group's G candidates back with
// G/4 broadcast ds_read_b128, and the k sequential duplicate checks run on registers and
// ballots — where floyd_pick spent two ds_bpermute per step (64-bit __shfl), the LDS pipe
// that bounded the pick kernel.  Positions fit 31 bits (a row holds < 2^31 edges).
template <int G>
__device__ __forceinline__ int floyd_pick_lds(const Group<G>& grp, uint64_t key, int64_t v,
                                              int64_t deg, int k, int* __restrict__ sh) {
  const int64_t jl = deg - k + grp.lane;  // this lane's step (valid for lane < k)
  const int tl = grp.lane < k ? (int)(hash3(key, (uint64_t)v, (uint64_t)jl) % (uint64_t)(jl + 1))
                              : -1;
  sh[grp.lane] = tl;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  int t[G];
#pragma unroll
  for (int q = 0; q < G / 4; ++q) {
    const int4 x = reinterpret_cast<const int4*>(sh)[q];
    t[4 * q] = x.x;
    t[4 * q + 1] = x.y;
    t[4 * q + 2] = x.z;
    t[4 * q + 3] = x.w;
  }
  int mine = -1;
#pragma unroll
  for (int s = 0; s < G; ++s) {
    if (s < k) {
      const bool dup = grp.ballot(grp.lane < s && mine == t[s]) != 0ull;
      if (grp.lane == s) mine = dup ? (int)jl : t[s];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // sh is rewritten next
  return mine;  // lanes >= k: -1
}

// a kept pick's slot in its row: the kept picks at smaller positions (picks are distinct),
// from the group's positions exchanged through LDS (not kept: INT_MAX, counted by no lane)
template <int G>
__device__ __forceinline__ int kept_rank_lds(const Group<G>& grp, bool keep, int pos,
                                             int* __restrict__ sh) {
  sh[grp.lane] = keep ? pos : 0x7fffffff;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  int slot = 0;
#pragma unroll
  for (int q = 0; q < G / 4; ++q) {
    const int4 x = reinterpret_cast<const int4*>(sh)[q];
    slot += (x.x < pos) + (x.y < pos) + (x.z < pos) + (x.w < pos);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return slot;
}

template <int G, int SPG>
__global__ __launch_bounds__(kSbBlock) void sb_pick_kernel(StepArgs A) {
  const int k = A.sec.find((int)blockIdx.x);
  const int b = (int)blockIdx.x - A.sec.begin[k];
  if (A.sec.kind[k] == kSecZeroNext) {  // the next step's new-source and seed marks
    const TypeArgs& T = A.type[A.sec.idx[k]];
    const int64_t w = (int64_t)b * kSbBlock + threadIdx.x;
    if (w < T.words * 4) {
      reinterpret_cast<uint4*>(T.mark_next)[w] = make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(T.smark_next)[w] = make_uint4(0, 0, 0, 0);
    }
    return;
  }
  if (A.sec.kind[k] == kSecZeroScan) {  // the scan's tickets and tile flags, for this step
    const int64_t w = (int64_t)b * kSbBlock + threadIdx.x;
    if (w < A.scan_words) A.scan_ws[w] = 0ull;
    return;
  }
  const RelArgs& R = A.rel[A.sec.idx[k]];
  const TypeArgs& D = A.type[R.dst_t];
  const TypeArgs& S = A.type[R.src_t];
  const Group<G> grp;
  __shared__ int4 sh_all[kSbBlock / 4];  // G ints per group: candidates, then positions
  int* const sh = reinterpret_cast<int*>(sh_all) + (threadIdx.x & ~(G - 1));
  const int64_t rows = seed_rows(A, D);
  const int64_t i0 = ((int64_t)b * (kSbBlock / G) + (threadIdx.x / G)) * SPG;
  if (i0 >= rows) return;  // group-uniform
  const int64_t f = R.fanout;
  const int kf = (int)f;
  int64_t v[SPG], beg[SPG], end[SPG];
  const uint8_t* excluded[SPG];
#pragma unroll
  for (int u = 0; u < SPG; ++u) v[u] = i0 + u < rows ? D.seeds[i0 + u] : -2;  // -2: no row
#pragma unroll
  for (int u = 0; u < SPG; ++u) {
    beg[u] = end[u] = 0;
    excluded[u] = nullptr;
    if (v[u] >= 0) {
      beg[u] = R.indptr[v[u]];
      end[u] = R.indptr[v[u] + 1];
      excluded[u] = R.excl_mask && (!R.excl_rows || R.excl_rows[v[u]]) ? R.excl_mask : nullptr;
    }
  }
  // each seed's pick position: the whole row (deg <= fanout <= G: one chunk, in edge order)
  // or Floyd's fanout of deg (lanes >= fanout: -1)
  int64_t pos[SPG];
  bool whole[SPG];
#pragma unroll
  for (int u = 0; u < SPG; ++u) {
    const int64_t deg = end[u] - beg[u];
    whole[u] = deg <= f;
    if (v[u] < 0) pos[u] = -1;
    else if (whole[u]) pos[u] = grp.lane < deg ? grp.lane : -1;
    else pos[u] = floyd_pick_lds(grp, R.key, v[u], deg, kf, sh);
  }
  // the picked edges: one packed record, or the index and the eid
  int32_t src[SPG];
  int64_t id[SPG];
#pragma unroll
  for (int u = 0; u < SPG; ++u) {
    src[u] = 0;
    id[u] = 0;
    if (pos[u] >= 0) {
      const int64_t e = beg[u] + pos[u];
      if (R.rec != nullptr) {
        const uint64_t r = R.rec[e];
        src[u] = (int32_t)(uint32_t)r;
        id[u] = (int64_t)(r >> 32);
      } else {
        id[u] = R.eids[e];
        src[u] = R.indices[e];
      }
    }
  }
  bool keep[SPG];
  uint8_t is_seed[SPG];
#pragma unroll
  for (int u = 0; u < SPG; ++u) {
    keep[u] = pos[u] >= 0 && !(excluded[u] && excluded[u][id[u]]);
    is_seed[u] = keep[u] ? S.smark_cur[src[u]] : 1;  // (issued for every seed first)
  }
#pragma unroll
  for (int u = 0; u < SPG; ++u) {
    const int64_t i = i0 + u;
    if (v[u] == -2) continue;  // group-uniform
    if (v[u] < 0) {  // a padding seed (static shapes): its row holds `fanout` padding edges
      if (grp.lane == 0) R.counts[i] = f;
      continue;
    }
    int slot;
    const uint64_t m = grp.ballot(keep[u]);
    if (whole[u]) slot = grp.below(m);
    else slot = kept_rank_lds(grp, keep[u], (int)pos[u], sh);  // kept picks in position order
    if (keep[u]) {
      const int64_t q = i * f + slot;
      if (R.rec != nullptr) {
        R.pick_eid[q] = (int64_t)(((uint64_t)id[u] << 32) | (uint32_t)src[u]);
      } else {
        R.pick_src[q] = src[u];
        R.pick_eid[q] = id[u];
      }
      // a source that is not one of its type's seeds at this step is a new node
      if (!is_seed[u]) S.mark_cur[src[u]] = 1;
    }
    if (grp.lane == 0) R.counts[i] = __popcll(m);
  }
}

// ---------------------------------------------------------------- scan (step s)
// one block per relation (counts -> out_indptr, total) and per type (popcounts of the
// new-source bitmap -> word ranks, total new nodes)
__device__ __forceinline__ int64_t block_excl_scan(int64_t x, int64_t* wsum, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t v = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(v, off);
    if (lane >= off) v += y;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  constexpr int NW = kScanThreads / 64;
  int64_t before = 0, tot = 0;
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int64_t s = wsum[j];
    if (j < w) before += s;
    tot += s;
  }
  __syncthreads();  // wsum is reused by the next chunk
  *total = tot;
  return before + v - x;
}

// Chained tiles with decoupled look-back (the library's exclusive scan, sampler.hip): every
// segment is cut into tiles of kScanTile items, a block takes its segment's next tile by
// ticket (so a tile only ever waits on tiles taken before it), publishes the tile's
// aggregate, its first wave walks back over the predecessors' flags 64 at a time until an
// inclusive prefix, and publishes its own.  The grid covers each segment's capacity; tiles
// past the device count exit.  (One block per segment took 0.3-0.46 ms on the 1M-row
// segments of a K = 2500 batch.)
constexpr int kScanItems = 4;
constexpr int64_t kScanTile = (int64_t)kScanThreads * kScanItems;
constexpr unsigned long long kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62;
__device__ __forceinline__ unsigned long long flag_pack(unsigned long long st, int64_t v) {
  return st | ((unsigned long long)v & ((1ull << 62) - 1));
}
__device__ __forceinline__ int64_t flag_value(unsigned long long f) {
  return (int64_t)(f << 2) >> 2;
}

// The first wave of a tile's block (threadIdx.x < 64): publish the tile's aggregate, walk back
// over the predecessors' flags 64 at a time until an inclusive prefix, publish the tile's own
// inclusive value -> the tile's exclusive prefix (every lane).  Tile 0 publishes at once.
__device__ __forceinline__ int64_t look_back(unsigned long long* flags, int64_t tile,
                                             int64_t agg) {
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0)
      __hip_atomic_store(flags, flag_pack(kFlagIncl, agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(flags + tile, flag_pack(kFlagAgg, agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  int64_t prefix = 0;
  for (int64_t j = tile - 1;; j -= 64) {  // window [j - 63, j], nearest first
    const int64_t idx = j - lane;
    unsigned long long f = kFlagIncl;  // before tile 0: an inclusive prefix of 0
    if (idx >= 0) {
      f = __hip_atomic_load(flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while ((f >> 62) == 0) {
        __builtin_amdgcn_s_sleep(1);
        f = __hip_atomic_load(flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const uint64_t incl = __ballot((f >> 62) == 2);
    const int stop = incl ? __builtin_ctzll(incl) : 64;
    int64_t x = lane <= stop ? flag_value(f) : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    prefix += x;
    if (incl) break;
  }
  if (lane == 0)
    __hip_atomic_store(flags + tile, flag_pack(kFlagIncl, prefix + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return prefix;
}

__global__ __launch_bounds__(kScanThreads) void sb_scan_kernel(StepArgs A) {
  __shared__ int64_t wsum[kScanThreads / 64];
  __shared__ int64_t sh_tile, sh_prefix;
  int seg = 0;
  while (seg + 1 < A.n_rels + A.n_types && (int)blockIdx.x >= A.seg_block0[seg + 1]) ++seg;
  const bool is_rel = seg < A.n_rels;
  int64_t n;
  const int64_t* cnt = nullptr;
  unsigned long long* bits = nullptr;
  const uint8_t* marks = nullptr;
  int64_t* out;
  if (is_rel) {
    const RelArgs& R = A.rel[seg];
    n = seed_rows(A, A.type[R.dst_t]);
    cnt = R.counts;
    out = R.out_indptr;
  } else {
    const TypeArgs& T = A.type[seg - A.n_rels];
    n = T.words;
    bits = T.bits_cur;
    marks = T.mark_cur;
    out = T.word_rank;
  }
  unsigned long long* ticket = A.scan_ws + seg * A.scan_stride;
  unsigned long long* flags = ticket + 1;
  if (threadIdx.x == 0)
    sh_tile = (int64_t)__hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int64_t tile = sh_tile;
  const int64_t n_tiles = n > 0 ? (n + kScanTile - 1) / kScanTile : 1;
  if (tile >= n_tiles) return;  // block-uniform: past the device count
  const int64_t i0 = tile * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems], s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    const int64_t i = i0 + j;
    if (i >= n) {
      v[j] = 0;
    } else if (is_rel) {
      v[j] = cnt[i];
    } else {  // the bitmap word from its marks (finalize ranks new sources in it)
      const unsigned long long w = word_of_marks(marks + i * 64);
      bits[i] = w;
      v[j] = __popcll(w);
    }
    s += v[j];
  }
  int64_t agg;
  const int64_t ex = block_excl_scan(s, wsum, &agg);
  if (threadIdx.x < 64) {
    const int64_t pr = look_back(flags, tile, agg);
    if (threadIdx.x == 0) sh_prefix = pr;
  }
  __syncthreads();
  int64_t run = sh_prefix + ex;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (i0 + j < n) out[i0 + j] = run;
    run += v[j];
  }
  if (tile != n_tiles - 1) return;  // the last tile closes the segment
  const int64_t carry = sh_prefix + agg;
  if (is_rel && A.stat) {  // the dump rows' bounds: runs of kDumpEdges up to the capacity
    const RelArgs& R = A.rel[seg];
    for (int64_t j = 1 + threadIdx.x; j < R.dump_rows; j += kScanThreads)
      out[n + 1 + j] = min(carry + (j + 1) * kDumpEdges, R.edge_cap);
  }
  if (threadIdx.x == 0) {
    out[n] = carry;
    if (is_rel) {
      *A.rel[seg].edge_total = carry;
      if (A.stat) out[n + 1] = min(carry + kDumpEdges, A.rel[seg].edge_cap);
    } else {
      const TypeArgs& T = A.type[seg - A.n_rels];
      // static shapes: at most node_cap - 1 real sources (a hinted capacity may cut them)
      *T.n_nodes_out = A.stat ? min(*T.n_seeds + carry, T.node_cap - 1) : *T.n_seeds + carry;
    }
  }
}

// ---------------------------------------------------------------- finalize (step s)
// n_p: where the new sources start (the real seeds' count)
__device__ __forceinline__ int64_t local_id(const TypeArgs& T, int64_t n_p, uint32_t stamp,
                                            int32_t s) {
  // the position and the rank words requested together: one round trip, not two
  const int64_t w = s >> 6;
  const unsigned long long v = T.pos_cur[s];
  const int64_t rank = T.word_rank[w];
  const unsigned long long bw = T.bits_cur[w];
  if ((uint32_t)(v >> 32) == stamp) return pos_of(v);  // one of this step's seeds
  return n_p + rank + __popcll(bw & ((1ull << (s & 63)) - 1ull));  // a new source: its rank
}

// static shapes: the source slot of padding edge k — spread over the list's padding slots
// [real sources, node_cap + 1), all -1, so the backward's transposed block has no single
// source row holding every padding edge (a radix sort's worst case, and a heavy row)
__device__ __forceinline__ int32_t pad_src(const TypeArgs& S, int64_t k) {
  const int64_t real = min(*S.n_seeds + S.word_rank[S.words], S.node_cap - 1);
  return (int32_t)(real + k % (S.node_len - real));
}

__global__ __launch_bounds__(kSbBlock) void sb_finalize_kernel(StepArgs A) {
  const int k = A.sec.find((int)blockIdx.x);
  const int64_t t = (int64_t)((int)blockIdx.x - A.sec.begin[k]) * kSbBlock + threadIdx.x;
  const int x = A.sec.idx[k];
  switch (A.sec.kind[k]) {
    case kSecCompact: {  // capacity slot t = (seed i, pick j) -> the block CSR
      const RelArgs& R = A.rel[x];
      const TypeArgs& D = A.type[R.dst_t];
      const TypeArgs& S = A.type[R.src_t];
      const int64_t i = t / R.fanout, j = t - i * R.fanout;
      if (i >= seed_rows(A, D)) return;
      // the slot's loads requested together before any of them is tested (the pick slot
      // may be unwritten past the row's count: read, not used)
      const int64_t cnt = R.counts[i];
      const int64_t row0 = R.out_indptr[i];
      const int64_t seed = D.seeds[i];
      int32_t ps;
      int64_t pe;
      if (R.rec != nullptr) {
        const uint64_t pk = (uint64_t)R.pick_eid[t];
        ps = (int32_t)(uint32_t)pk;
        pe = (int64_t)(pk >> 32);
      } else {
        ps = R.pick_src[t];
        pe = R.pick_eid[t];
      }
      if (j >= cnt) return;
      const int64_t o = row0 + j;
      if (seed < 0) {  // a padding row's padding edge
        R.out_src[o] = pad_src(S, o);
        R.out_eid[o] = -1;
        break;
      }
      int64_t loc = local_id(S, *S.n_seeds, A.stamp, ps);
      if (A.stat && loc >= S.node_cap - 1) {  // past a hinted capacity: a padding slot
        if (A.overflow) *A.overflow = 1;
        loc = S.node_cap - 1;
      }
      R.out_src[o] = (int32_t)loc;
      R.out_eid[o] = pe;
      break;
    }
    case kSecDumpEdges: {  // static shapes: the edge capacity's rest -> the dump rows
      // (a grid-stride section of at most kStrideBlocks blocks: the rest is known only
      // here, and a grid covering the whole capacity was mostly idle threads)
      const RelArgs& R = A.rel[x];
      const TypeArgs& S = A.type[R.src_t];
      const int64_t nth = (int64_t)(A.sec.begin[k + 1] - A.sec.begin[k]) * kSbBlock;
      const int64_t real = min(*S.n_seeds + S.word_rank[S.words], S.node_cap - 1);
      const int64_t span = S.node_len - real;  // pad_src's slots, read once
      for (int64_t e = R.out_indptr[A.type[R.dst_t].seed_cap] + t; e < R.edge_cap; e += nth) {
        R.out_src[e] = (int32_t)(real + e % span);
        R.out_eid[e] = -1;
      }
      break;
    }
    case kSecPadNodes: {  // static shapes: the list past the real seeds and new sources
      const TypeArgs& T = A.type[x];
      const int64_t nth = (int64_t)(A.sec.begin[k + 1] - A.sec.begin[k]) * kSbBlock;
      for (int64_t p = min(*T.n_seeds + T.word_rank[T.words], T.node_cap - 1) + t;
           p < T.node_len; p += nth)
        T.nodes[p] = -1;
      break;
    }
    case kSecNewNodes: {  // bitmap word t -> its new nodes, ascending, after the seeds
      const TypeArgs& T = A.type[x];
      if (t >= T.words) return;
      unsigned long long word = T.bits_cur[t];
      if (!word) return;
      int64_t p = *T.n_seeds + T.word_rank[t];
      while (word) {
        const int64_t id = t * 64 + __builtin_ctzll(word);
        if (A.stat && p >= T.node_cap - 1) {  // past a hinted capacity: left out
          if (A.overflow) *A.overflow = 1;
          break;
        }
        T.nodes[p] = id;
        T.pos_next[id] = pack_pos(A.stamp + 1u, p);  // (new ids are distinct)
        if (!A.last) T.smark_next[id] = 1;
        word &= word - 1ull;
        ++p;
      }
      break;
    }
    case kSecPrefix: {  // the seeds open the source node list, at their positions
      const TypeArgs& T = A.type[x];
      if (t >= *T.n_seeds) return;
      const int64_t id = T.seeds[t];
      T.nodes[t] = id;
      if (id >= 0) {
        set_pos(T.pos_next, id, A.stamp + 1u, t);
        if (!A.last) T.smark_next[id] = 1;
      }
      break;
    }
    case kSecSeedClear: {  // the last step: its seed marks are the next call's step-0 marks
      const TypeArgs& T = A.type[x];
      if (t < T.words * 4) reinterpret_cast<uint4*>(T.smark_cur)[t] = make_uint4(0, 0, 0, 0);
      break;
    }
    case kSecExclClear: {
      const RelArgs& R = A.rel[x];
      if (t < R.n_excl) {
        const int64_t e = R.excl_eids[t];
        R.mask_w[e] = 0;
        R.rows_w[R.coo_dst[e]] = 0;
      }
      break;
    }
    default: break;
  }
}

// ---------------------------------------------------------------- compact_ids
struct CompactArgs {
  int n_lists, n_types;
  const int64_t* ids[GNNREC_COMPACT_MAX_LISTS];
  int64_t n[GNNREC_COMPACT_MAX_LISTS];
  int type[GNNREC_COMPACT_MAX_LISTS];
  int64_t* local[GNNREC_COMPACT_MAX_LISTS];
  unsigned long long* bits_cur[GNNREC_SB_MAX_TYPES];
  unsigned long long* bits_next[GNNREC_SB_MAX_TYPES];
  uint8_t* mark_cur[GNNREC_SB_MAX_TYPES];
  uint8_t* mark_next[GNNREC_SB_MAX_TYPES];
  int64_t* word_rank[GNNREC_SB_MAX_TYPES];
  int64_t words[GNNREC_SB_MAX_TYPES];
  int64_t* nodes[GNNREC_SB_MAX_TYPES];
  int64_t cap[GNNREC_SB_MAX_TYPES];
  int64_t* count;
  unsigned long long* scan_ws[GNNREC_SB_MAX_TYPES];  // ticket + tile flags per type
  int tile0[GNNREC_SB_MAX_TYPES + 1];                // first scan block of each type
  Sections sec;
};
enum { kCxMark, kCxZero, kCxZeroScan, kCxLocal, kCxNodes, kCxPad };
constexpr int64_t kCxTile = kScanThreads;  // bitmap words per scan tile (64 KiB of marks)
__host__ __device__ inline int64_t cx_tiles(int64_t words) {
  return words > 0 ? (words + kCxTile - 1) / kCxTile : 1;
}

__global__ __launch_bounds__(kSbBlock) void cx_mark_kernel(CompactArgs A) {
  const int k = A.sec.find((int)blockIdx.x);
  const int64_t t = (int64_t)((int)blockIdx.x - A.sec.begin[k]) * kSbBlock + threadIdx.x;
  const int x = A.sec.idx[k];
  if (A.sec.kind[k] == kCxZero) {  // the other parity's marks, for the next call
    if (t < A.words[x] * 4)
      reinterpret_cast<uint4*>(A.mark_next[x])[t] = make_uint4(0, 0, 0, 0);
    return;
  }
  if (A.sec.kind[k] == kCxZeroScan) {  // this call's scan ticket and tile flags
    if (t < 1 + cx_tiles(A.words[x])) A.scan_ws[x][t] = 0ull;
    return;
  }
  if (t >= A.n[x]) return;
  A.mark_cur[A.type[x]][A.ids[x][t]] = 1;  // plain byte stores (see word_of_marks)
}

// Per type the bitmap words from the marks and their exclusive popcount ranks: chained tiles
// of kCxTile words with decoupled look-back, as sb_scan_kernel (one block per type walked a
// 1M-node type's 1 MB of marks alone: 56 us of a K = 10 batch's 445)
__global__ __launch_bounds__(kScanThreads) void cx_scan_kernel(CompactArgs A) {
  __shared__ int64_t wsum[kScanThreads / 64];
  __shared__ int64_t sh_tile, sh_prefix;
  int t = 0;
  while (t + 1 < A.n_types && (int)blockIdx.x >= A.tile0[t + 1]) ++t;
  const int64_t n = A.words[t];
  unsigned long long* ticket = A.scan_ws[t];
  if (threadIdx.x == 0)
    sh_tile = (int64_t)__hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int64_t tile = sh_tile;
  const int64_t n_tiles = cx_tiles(n);
  if (tile >= n_tiles) return;  // block-uniform
  const int64_t i = tile * kCxTile + threadIdx.x;
  int64_t v = 0;
  if (i < n) {
    const unsigned long long w = word_of_marks(A.mark_cur[t] + i * 64);
    A.bits_cur[t][i] = w;
    v = __popcll(w);
  }
  int64_t agg;
  const int64_t ex = block_excl_scan(v, wsum, &agg);
  if (threadIdx.x < 64) {
    const int64_t pr = look_back(ticket + 1, tile, agg);
    if (threadIdx.x == 0) sh_prefix = pr;
  }
  __syncthreads();
  if (i < n) A.word_rank[t][i] = sh_prefix + ex;
  if (tile == n_tiles - 1 && threadIdx.x == 0) {
    A.word_rank[t][n] = sh_prefix + agg;
    A.count[t] = sh_prefix + agg;
  }
}

__global__ __launch_bounds__(kSbBlock) void cx_finalize_kernel(CompactArgs A) {
  const int k = A.sec.find((int)blockIdx.x);
  const int64_t t = (int64_t)((int)blockIdx.x - A.sec.begin[k]) * kSbBlock + threadIdx.x;
  const int x = A.sec.idx[k];
  switch (A.sec.kind[k]) {
    case kCxLocal: {
      if (t >= A.n[x]) return;
      const int ty = A.type[x];
      const int64_t id = A.ids[x][t], w = id >> 6;
      A.local[x][t] = A.word_rank[ty][w] + __popcll(A.bits_cur[ty][w] & ((1ull << (id & 63)) - 1ull));
      break;
    }
    case kCxNodes: {
      if (t >= A.words[x]) return;
      unsigned long long word = A.bits_cur[x][t];
      int64_t p = A.word_rank[x][t];
      while (word && p < A.cap[x]) {
        A.nodes[x][p++] = t * 64 + __builtin_ctzll(word);
        word &= word - 1ull;
      }
      break;
    }
    case kCxPad: {
      const int64_t p = A.word_rank[x][A.words[x]] + t;
      if (p < A.cap[x]) A.nodes[x][p] = -1;
      break;
    }
    default: break;
  }
}

inline int64_t words_of(int64_t n) { return (n + 63) / 64; }
inline int64_t up256(int64_t b) { return (b + 255) & ~(int64_t)255; }
inline int nblocks(int64_t threads) { return (int)((threads + kSbBlock - 1) / kSbBlock); }

struct Caps {
  int64_t seed[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_TYPES];
  int64_t edge[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  int64_t node[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_TYPES];
  int64_t dump[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_TYPES];  // static: dump rows per dst type
  int64_t len[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_TYPES];   // static: node list lengths
  int64_t scan_stride;  // words per scan segment: a ticket + the most tiles of any step
  int64_t ws_bytes;
};

int plan_caps(const gnnrec_sample_plan* P, Caps* C) {
  GNNREC_REQUIRE(P, "gnnrec_sample_blocks: null plan");
  GNNREC_REQUIRE(P->n_rels >= 0 && P->n_rels <= GNNREC_SB_MAX_RELS && P->n_types >= 1 &&
                     P->n_types <= GNNREC_SB_MAX_TYPES && P->n_steps >= 1 &&
                     P->n_steps <= GNNREC_SB_MAX_STEPS,
                 "gnnrec_sample_blocks: %d relations (<= %d), %d types (1..%d), %d steps (1..%d)",
                 P->n_rels, GNNREC_SB_MAX_RELS, P->n_types, GNNREC_SB_MAX_TYPES, P->n_steps,
                 GNNREC_SB_MAX_STEPS);
  for (int r = 0; r < P->n_rels; ++r) {
    const gnnrec_sample_rel& R = P->rel[r];
    GNNREC_REQUIRE(R.src_type >= 0 && R.src_type < P->n_types && R.dst_type >= 0 &&
                       R.dst_type < P->n_types,
                   "gnnrec_sample_blocks: relation %d: node-type index out of range", r);
    for (int s = 0; s < P->n_steps; ++s)
      GNNREC_REQUIRE(P->fanout[s][r] >= 0 && P->fanout[s][r] <= kMaxFanout,
                     "gnnrec_sample_blocks: fanout %lld at step %d (bounded: 0..%d)",
                     (long long)P->fanout[s][r], s, kMaxFanout);
    GNNREC_REQUIRE(R.n_excl >= 0, "gnnrec_sample_blocks: negative exclusion count");
  }
  for (int t = 0; t < P->n_types; ++t) {
    GNNREC_REQUIRE(P->type[t].n_seeds >= 0 && P->type[t].n_nodes >= 0 &&
                       P->type[t].n_nodes < (int64_t(1) << 31),
                   "gnnrec_sample_blocks: type %d: sizes", t);
    C->seed[0][t] = P->type[t].n_seeds;
  }
  int64_t ws = 0;
  for (int s = 0; s < P->n_steps; ++s) {
    for (int r = 0; r < P->n_rels; ++r) {
      C->edge[s][r] = C->seed[s][P->rel[r].dst_type] * P->fanout[s][r];
      ws += up256(8 * C->seed[s][P->rel[r].dst_type]) + up256(4 * C->edge[s][r]) +
            up256(8 * C->edge[s][r]);
    }
    for (int t = 0; t < P->n_types; ++t) {  // static: dump rows per destination type
      int64_t dmax = 0;
      for (int r = 0; r < P->n_rels; ++r)
        if (P->rel[r].dst_type == t)
          dmax = std::max<int64_t>(dmax, (C->edge[s][r] + kDumpEdges - 1) / kDumpEdges);
      C->dump[s][t] = P->static_shapes ? 1 + dmax : 0;
    }
    for (int t = 0; t < P->n_types; ++t) {
      int64_t e = 0;
      for (int r = 0; r < P->n_rels; ++r)
        if (P->rel[r].src_type == t) e += C->edge[s][r];
      // static shapes: the real sources (at most n_nodes) and one padding slot, and never
      // fewer rows than the destinations with their dump rows (a block's dst rows are a
      // prefix of its sources)
      int64_t real_cap = std::min<int64_t>(C->seed[s][t] + e, P->type[t].n_nodes) + 1;
      if (P->static_shapes && P->node_cap_hint[s][t] > 0)  // a caller's tighter bound
        real_cap = std::min<int64_t>(real_cap, P->node_cap_hint[s][t]);
      C->node[s][t] = P->static_shapes
                          ? std::max<int64_t>(C->seed[s][t] + C->dump[s][t], real_cap)
                          : C->seed[s][t] + std::min<int64_t>(e, P->type[t].n_nodes);
      if (s + 1 < P->n_steps) C->seed[s + 1][t] = C->node[s][t];
    }
  }
  for (int s = 0; s < P->n_steps; ++s)
    for (int t = 0; t < P->n_types; ++t)
      C->len[s][t] = C->node[s][t] +
                     (P->static_shapes ? (s + 1 < P->n_steps ? C->dump[s + 1][t] : 1) : 0);
  int64_t tiles = 1;
  for (int s = 0; s < P->n_steps; ++s) {
    for (int r = 0; r < P->n_rels; ++r)
      tiles = std::max<int64_t>(tiles, (C->seed[s][P->rel[r].dst_type] + kScanTile - 1) / kScanTile);
  }
  for (int t = 0; t < P->n_types; ++t)
    tiles = std::max<int64_t>(tiles, (words_of(P->type[t].n_nodes) + kScanTile - 1) / kScanTile);
  C->scan_stride = 1 + tiles;
  ws += up256(8 * (int64_t)(P->n_rels + P->n_types) * C->scan_stride);
  C->ws_bytes = ws;
  return GNNREC_OK;
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_sample_blocks_caps(const gnnrec_sample_plan* plan, int64_t* seed_cap,
                                         int64_t* edge_cap, int64_t* node_cap,
                                         int64_t* dump_rows, int64_t* workspace_bytes) {
  Caps C{};
  if (int st = plan_caps(plan, &C)) return st;
  for (int s = 0; s < GNNREC_SB_MAX_STEPS; ++s) {
    for (int t = 0; t < GNNREC_SB_MAX_TYPES; ++t) {
      if (seed_cap) seed_cap[s * GNNREC_SB_MAX_TYPES + t] = C.seed[s][t];
      if (node_cap) node_cap[s * GNNREC_SB_MAX_TYPES + t] = C.node[s][t];
      if (dump_rows) dump_rows[s * GNNREC_SB_MAX_TYPES + t] = C.dump[s][t];
    }
    for (int r = 0; r < GNNREC_SB_MAX_RELS; ++r)
      if (edge_cap) edge_cap[s * GNNREC_SB_MAX_RELS + r] = C.edge[s][r];
  }
  if (workspace_bytes) *workspace_bytes = C.ws_bytes;
  return GNNREC_OK;
}

extern "C" int gnnrec_sample_blocks(const gnnrec_sample_plan* P, void* stream) {
  Caps C{};
  if (int st = plan_caps(P, &C)) return st;
  GNNREC_REQUIRE(P->stamp >= 1u && P->stamp <= 0xFFFFFFFFu - (uint32_t)P->n_steps - 2u,
                 "gnnrec_sample_blocks: stamp %u out of range (restart at 1 with zeroed pos)",
                 P->stamp);
  GNNREC_REQUIRE(P->sizes && (C.ws_bytes == 0 || P->workspace),
                 "gnnrec_sample_blocks: null sizes / workspace");
  const int R = P->n_rels, T = P->n_types, L = P->n_steps;
  for (int t = 0; t < T; ++t) {
    const gnnrec_sample_type& ty = P->type[t];
    GNNREC_REQUIRE(ty.pos && ty.bits && ty.marks && ty.word_rank && (ty.n_seeds == 0 || ty.seeds),
                   "gnnrec_sample_blocks: type %d: null scratch or seeds", t);
    GNNREC_REQUIRE((reinterpret_cast<uintptr_t>(ty.marks) & 15u) == 0,
                   "gnnrec_sample_blocks: type %d: marks must be 16-byte aligned", t);
    for (int s = 0; s < L; ++s)
      GNNREC_REQUIRE(P->nodes[s][t] || C.node[s][t] == 0,
                     "gnnrec_sample_blocks: null nodes output (step %d, type %d)", s, t);
  }
  for (int r = 0; r < R; ++r) {
    const gnnrec_sample_rel& re = P->rel[r];
    GNNREC_REQUIRE(re.indptr && ((re.indices && re.eids) || re.edge_rec),
                   "gnnrec_sample_blocks: relation %d: null CSR", r);
    GNNREC_REQUIRE(re.n_excl == 0 || (re.excl_eids && re.coo_dst && re.excl_mask && re.excl_rows),
                   "gnnrec_sample_blocks: relation %d: exclusion needs eids, coo_dst and flags", r);
    for (int s = 0; s < L; ++s)
      GNNREC_REQUIRE(P->out_indptr[s][r] && (C.edge[s][r] == 0 ||
                                             (P->out_src[s][r] && P->out_eid[s][r])),
                     "gnnrec_sample_blocks: null output (step %d, relation %d)", s, r);
  }
  hipStream_t hs = as_stream(stream);
  // workspace: per (step, relation) counts, pick sources, pick eids
  char* ws = static_cast<char*>(P->workspace);
  int64_t* cnt[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  int32_t* psrc[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  int64_t* peid[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  for (int s = 0; s < L; ++s)
    for (int r = 0; r < R; ++r) {
      cnt[s][r] = reinterpret_cast<int64_t*>(ws);
      ws += up256(8 * C.seed[s][P->rel[r].dst_type]);
      psrc[s][r] = reinterpret_cast<int32_t*>(ws);
      ws += up256(4 * C.edge[s][r]);
      peid[s][r] = reinterpret_cast<int64_t*>(ws);
      ws += up256(8 * C.edge[s][r]);
    }
  unsigned long long* scan_ws = reinterpret_cast<unsigned long long*>(ws);
  int64_t* node_count = P->sizes;                   // [(L + 1) x T], row -1 first
  int64_t* edge_count = P->sizes + (int64_t)(L + 1) * T;  // [L x R]

  auto step_args = [&](int s, StepArgs& A) {
    A = StepArgs{};
    A.n_rels = R;
    A.n_types = T;
    A.last = s == L - 1;
    A.stat = P->static_shapes ? 1 : 0;
    A.overflow = P->overflow;
    A.stamp = P->stamp + (uint32_t)s;
    A.sizes_seed_row = node_count;
    A.scan_ws = scan_ws;
    A.scan_stride = C.scan_stride;
    A.scan_words = (int64_t)(R + T) * C.scan_stride;
    A.seg_block0[0] = 0;
    for (int r = 0; r < R; ++r)  // the scan's grid: each segment's capacity in tiles
      A.seg_block0[r + 1] = A.seg_block0[r] +
          (int)std::max<int64_t>(1, (C.seed[s][P->rel[r].dst_type] + kScanTile - 1) / kScanTile);
    for (int t = 0; t < T; ++t)
      A.seg_block0[R + t + 1] = A.seg_block0[R + t] +
          (int)std::max<int64_t>(1, (words_of(P->type[t].n_nodes) + kScanTile - 1) / kScanTile);
    for (int t = 0; t < T; ++t) {
      const gnnrec_sample_type& ty = P->type[t];
      TypeArgs& a = A.type[t];
      const int64_t W = words_of(ty.n_nodes);
      a.seeds = s == 0 ? ty.seeds : P->nodes[s - 1][t];
      a.n_seeds = node_count + (int64_t)s * T + t;
      a.seed_cap = C.seed[s][t];
      a.n_seeds_host = ty.n_seeds;
      a.pos_cur = reinterpret_cast<unsigned long long*>(ty.pos) + (A.stamp & 1u) * ty.n_nodes;
      a.pos_next =
          reinterpret_cast<unsigned long long*>(ty.pos) + ((A.stamp + 1u) & 1u) * ty.n_nodes;
      a.bits_cur = reinterpret_cast<unsigned long long*>(ty.bits) + (A.stamp & 1u) * W;
      a.bits_next = reinterpret_cast<unsigned long long*>(ty.bits) + ((A.stamp + 1u) & 1u) * W;
      a.mark_cur = ty.marks + (A.stamp & 1u) * 64 * W;
      a.mark_next = ty.marks + ((A.stamp + 1u) & 1u) * 64 * W;
      a.smark_cur = ty.marks + (2 + (A.stamp & 1u)) * 64 * W;
      a.smark_next = ty.marks + (2 + ((A.stamp + 1u) & 1u)) * 64 * W;
      a.word_rank = ty.word_rank;
      a.words = W;
      a.nodes = P->nodes[s][t];
      a.n_nodes_out = node_count + (int64_t)(s + 1) * T + t;
      a.node_cap = C.node[s][t];
      a.node_len = C.len[s][t];
    }
    for (int r = 0; r < R; ++r) {
      const gnnrec_sample_rel& re = P->rel[r];
      RelArgs& a = A.rel[r];
      a.indptr = re.indptr;
      a.indices = re.indices;
      a.eids = re.eids;
      a.rec = re.edge_rec;
      a.excl_mask = re.n_excl ? re.excl_mask : nullptr;
      a.excl_rows = re.n_excl ? re.excl_rows : nullptr;
      a.src_t = re.src_type;
      a.dst_t = re.dst_type;
      a.fanout = P->fanout[s][r];
      a.key = P->key[s][r];
      a.counts = cnt[s][r];
      a.pick_src = psrc[s][r];
      a.pick_eid = peid[s][r];
      a.out_indptr = P->out_indptr[s][r];
      a.out_src = P->out_src[s][r];
      a.out_eid = P->out_eid[s][r];
      a.edge_total = edge_count + (int64_t)s * R + r;
      a.edge_cap = C.edge[s][r];
      a.dump_rows = C.dump[s][re.dst_type];
      a.excl_eids = re.excl_eids;
      a.n_excl = re.n_excl;
      a.coo_dst = re.coo_dst;
      a.mask_w = re.excl_mask;
      a.rows_w = re.excl_rows;
    }
  };
  auto add_sec = [](Sections& S, int kind, int idx, int blocks) {
    if (blocks <= 0) return;
    S.kind[S.n] = kind;
    S.idx[S.n] = idx;
    S.begin[S.n + 1] = S.begin[S.n] + blocks;
    ++S.n;
  };

  StepArgs A;
  // begin: seed positions, the first step's bitmaps, the exclusion flags
  step_args(0, A);
  A.sec.n = 0;
  A.sec.begin[0] = 0;
  for (int t = 0; t < T; ++t) add_sec(A.sec, kSecSeedPos, t, nblocks(P->type[t].n_seeds));
  for (int t = 0; t < T; ++t) add_sec(A.sec, kSecZeroBits, t, nblocks(4 * A.type[t].words));
  for (int r = 0; r < R; ++r) add_sec(A.sec, kSecExclSet, r, nblocks(P->rel[r].n_excl));
  if (A.sec.n == 0) add_sec(A.sec, kSecSeedPos, 0, 1);  // the seed-count row still lands
  hipLaunchKernelGGL(sb_begin_kernel, dim3((unsigned)A.sec.begin[A.sec.n]), dim3(kSbBlock), 0, hs,
                     A);
  if (int st = check_launch("gnnrec_sample_blocks(begin)")) return st;

  for (int s = 0; s < L; ++s) {
    step_args(s, A);
    int64_t fmax = 1;
    for (int r = 0; r < R; ++r) fmax = std::max<int64_t>(fmax, P->fanout[s][r]);
    const int G = group_size(fmax);
    // pick
    A.sec.n = 0;
    A.sec.begin[0] = 0;
    for (int r = 0; r < R; ++r)  // kPickSpg seeds per group of G lanes
      add_sec(A.sec, kSecPick, r,
              (int)((C.seed[s][P->rel[r].dst_type] + kPickSpg * (kSbBlock / G) - 1) /
                    (kPickSpg * (kSbBlock / G))));
    for (int t = 0; t < T; ++t) add_sec(A.sec, kSecZeroNext, t, nblocks(4 * A.type[t].words));
    add_sec(A.sec, kSecZeroScan, 0, nblocks(A.scan_words));
    if (A.sec.n) {
      const dim3 grid((unsigned)A.sec.begin[A.sec.n]);
      switch (G) {
        case 8: hipLaunchKernelGGL((sb_pick_kernel<8, kPickSpg>), grid, dim3(kSbBlock), 0, hs, A); break;
        case 16: hipLaunchKernelGGL((sb_pick_kernel<16, kPickSpg>), grid, dim3(kSbBlock), 0, hs, A); break;
        case 32: hipLaunchKernelGGL((sb_pick_kernel<32, kPickSpg>), grid, dim3(kSbBlock), 0, hs, A); break;
        default: hipLaunchKernelGGL((sb_pick_kernel<64, kPickSpg>), grid, dim3(kSbBlock), 0, hs, A); break;
      }
      if (int st = check_launch("gnnrec_sample_blocks(pick)")) return st;
    }
    // scan: chained tiles over every relation's counts and every type's bitmap words
    hipLaunchKernelGGL(sb_scan_kernel, dim3((unsigned)A.seg_block0[R + T]), dim3(kScanThreads),
                       0, hs, A);
    if (int st = check_launch("gnnrec_sample_blocks(scan)")) return st;
    // finalize
    A.sec.n = 0;
    A.sec.begin[0] = 0;
    for (int r = 0; r < R; ++r) add_sec(A.sec, kSecCompact, r, nblocks(C.edge[s][r]));
    for (int t = 0; t < T; ++t) add_sec(A.sec, kSecNewNodes, t, nblocks(A.type[t].words));
    for (int t = 0; t < T; ++t) add_sec(A.sec, kSecPrefix, t, nblocks(C.seed[s][t]));
    if (s == L - 1)
      for (int t = 0; t < T; ++t) add_sec(A.sec, kSecSeedClear, t, nblocks(4 * A.type[t].words));
    if (s == L - 1)
      for (int r = 0; r < R; ++r) add_sec(A.sec, kSecExclClear, r, nblocks(P->rel[r].n_excl));
    if (P->static_shapes) {
      for (int r = 0; r < R; ++r)
        add_sec(A.sec, kSecDumpEdges, r, std::min(nblocks(C.edge[s][r]), kStrideBlocks));
      for (int t = 0; t < T; ++t)
        add_sec(A.sec, kSecPadNodes, t, std::min(nblocks(C.len[s][t]), kStrideBlocks));
    }
    if (A.sec.n) {
      hipLaunchKernelGGL(sb_finalize_kernel, dim3((unsigned)A.sec.begin[A.sec.n]), dim3(kSbBlock),
                         0, hs, A);
      if (int st = check_launch("gnnrec_sample_blocks(finalize)")) return st;
    }
  }
  return GNNREC_OK;
}

extern "C" int gnnrec_compact_ids(const gnnrec_compact_list* lists, int n_lists,
                                  const gnnrec_compact_type* types, int n_types, int parity,
                                  int64_t* count, void* stream) {
  GNNREC_REQUIRE(n_lists >= 0 && n_lists <= GNNREC_COMPACT_MAX_LISTS && n_types >= 1 &&
                     n_types <= GNNREC_SB_MAX_TYPES,
                 "gnnrec_compact_ids: %d lists (<= %d), %d types (1..%d)", n_lists,
                 GNNREC_COMPACT_MAX_LISTS, n_types, GNNREC_SB_MAX_TYPES);
  GNNREC_REQUIRE((parity == 0 || parity == 1) && count, "gnnrec_compact_ids: parity / count");
  CompactArgs A{};
  A.n_lists = n_lists;
  A.n_types = n_types;
  A.count = count;
  for (int t = 0; t < n_types; ++t) {
    const gnnrec_compact_type& ty = types[t];
    GNNREC_REQUIRE(ty.n_nodes >= 0 && ty.cap >= 0 && ty.bits && ty.marks && ty.word_rank &&
                       (ty.cap == 0 || ty.nodes) && (reinterpret_cast<uintptr_t>(ty.marks) & 15u) == 0,
                   "gnnrec_compact_ids: type %d: sizes / null or unaligned scratch", t);
    const int64_t W = words_of(ty.n_nodes);
    A.bits_cur[t] = reinterpret_cast<unsigned long long*>(ty.bits) + parity * W;
    A.bits_next[t] = reinterpret_cast<unsigned long long*>(ty.bits) + (1 - parity) * W;
    A.mark_cur[t] = ty.marks + parity * 64 * W;
    A.mark_next[t] = ty.marks + (1 - parity) * 64 * W;
    A.word_rank[t] = ty.word_rank;
    A.words[t] = W;
    A.nodes[t] = ty.nodes;
    A.cap[t] = ty.cap;
    GNNREC_REQUIRE(ty.scan_ws, "gnnrec_compact_ids: type %d: null scan_ws", t);
    A.scan_ws[t] = reinterpret_cast<unsigned long long*>(ty.scan_ws);
  }
  A.tile0[0] = 0;
  for (int t = 0; t < n_types; ++t) A.tile0[t + 1] = A.tile0[t] + (int)cx_tiles(A.words[t]);
  for (int l = 0; l < n_lists; ++l) {
    const gnnrec_compact_list& li = lists[l];
    GNNREC_REQUIRE(li.n >= 0 && li.type >= 0 && li.type < n_types && (li.n == 0 || (li.ids && li.local)),
                   "gnnrec_compact_ids: list %d: size / type / null pointer", l);
    A.ids[l] = li.ids;
    A.n[l] = li.n;
    A.type[l] = li.type;
    A.local[l] = li.local;
  }
  auto add_sec = [](Sections& S, int kind, int idx, int blocks) {
    if (blocks <= 0) return;
    S.kind[S.n] = kind;
    S.idx[S.n] = idx;
    S.begin[S.n + 1] = S.begin[S.n] + blocks;
    ++S.n;
  };
  hipStream_t hs = as_stream(stream);
  A.sec.n = 0;
  A.sec.begin[0] = 0;
  for (int l = 0; l < n_lists; ++l) add_sec(A.sec, kCxMark, l, nblocks(A.n[l]));
  for (int t = 0; t < n_types; ++t) add_sec(A.sec, kCxZero, t, nblocks(4 * A.words[t]));
  for (int t = 0; t < n_types; ++t) add_sec(A.sec, kCxZeroScan, t, nblocks(1 + cx_tiles(A.words[t])));
  {
    hipLaunchKernelGGL(cx_mark_kernel, dim3((unsigned)A.sec.begin[A.sec.n]), dim3(kSbBlock), 0, hs, A);
    if (int st = check_launch("gnnrec_compact_ids(mark)")) return st;
  }
  hipLaunchKernelGGL(cx_scan_kernel, dim3((unsigned)A.tile0[n_types]), dim3(kScanThreads), 0, hs,
                     A);
  if (int st = check_launch("gnnrec_compact_ids(scan)")) return st;
  A.sec.n = 0;
  A.sec.begin[0] = 0;
  for (int l = 0; l < n_lists; ++l) add_sec(A.sec, kCxLocal, l, nblocks(A.n[l]));
  for (int t = 0; t < n_types; ++t) add_sec(A.sec, kCxNodes, t, nblocks(A.words[t]));
  for (int t = 0; t < n_types; ++t) add_sec(A.sec, kCxPad, t, nblocks(A.cap[t]));
  if (A.sec.n) {
    hipLaunchKernelGGL(cx_finalize_kernel, dim3((unsigned)A.sec.begin[A.sec.n]), dim3(kSbBlock), 0,
                       hs, A);
    if (int st = check_launch("gnnrec_compact_ids(finalize)")) return st;
  }
  return GNNREC_OK;
}
