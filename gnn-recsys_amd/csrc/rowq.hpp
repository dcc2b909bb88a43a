// Dynamic row distribution for the long-running row kernels (spmm_csr_kernel, the fused
// spmm_project_kernel) when they share the chip with another kernel — in a multi-rank
// pass, RCCL's collective kernels launched on their own stream beside the aggregation.
//
// Why: those kernels hand out rows statically (grid-stride), and the fused one keeps one
// block per CU with all 160 KiB of its LDS.  A collective kernel dispatched first holds
// some CUs; the fused blocks bound to those CUs start only when it ends and then still
// owe their whole static share, so the launch ends one collective later (the exchange is
// serialised, not overlapped).  With a queue, a late block simply takes fewer rows.
//
// Shape: the rows are cut into 8 contiguous ranges, one per XCD; a wave dequeues chunks of
// `ch` rows from its own XCD's head (agent-scope atomic, ≈1 µs; ≈30 dequeues/µs per head
// at C4 shapes, under the ≈88/µs a single word sustains) and, once that range is drained,
// from the other heads (all 8 read at once), so every wave sees every head drained and
// exits.  The next ticket is requested before the current chunk runs.  Which wave reduces a row does
// not change how it is reduced: outputs stay bitwise identical to the static schedule.
//
// Slots: every launch takes the next slot of a per-device ring (host side, rowq.hip); the
// last block to finish resets the slot's heads, so the next user finds zeros without a
// memset.  An event per slot records its launch's completion: a slot whose last launch
// (on any stream) is still running is not reused — that launch runs the static schedule.  A slot holds 8 heads + 1 exit counter, each on its own 128-B line.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gnnrec {

constexpr int kRqHeads = 8;
constexpr int kRqStride = 32;  // uint32 words per head: 128-B lines
constexpr int kRqSlotWords = (kRqHeads + 1) * kRqStride;

// host (rowq.hip)
// next slot of the current device's ring, or nullptr (static mode, or the slot's previous
// launch still running); after launching with a slot, rowq_launched(ticket, stream)
unsigned* rowq_slot(hipStream_t stream, int* ticket);
void rowq_launched(int ticket, hipStream_t stream);
// the single-pass scan's slots (sampler.hip): [0] tile counter, [1] done counter, tile
// flags from word kScanFlags0; zero between users (the last block resets what it used)
constexpr int kScanMaxTiles = 4096;
constexpr int kScanFlags0 = 16;
constexpr int kScanSlotWords = kScanFlags0 + kScanMaxTiles;
constexpr unsigned kScanSlots = 128;
unsigned long long* scan_slot(hipStream_t stream, int* ticket);  // nullptr: no slot free
void scan_launched(int ticket, hipStream_t stream);
int device_cus();       // CUs of the current device
int cu_reserve();       // CUs the row kernels leave free for concurrent kernels

__device__ inline int xcc_id() {
  // s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): size-1 in [15:11], offset [10:6], id 20
  return __builtin_amdgcn_s_getreg((3 << 11) | 20) & (kRqHeads - 1);
}

// lane 0 draws a ticket; the value is read (broadcast) only when the chunk is claimed
__device__ inline unsigned rq_take(unsigned* head) {
  unsigned t = 0;
  if ((threadIdx.x & 63) == 0)
    t = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return t;
}

// tickets of head h until its range is drained: f(r0, r1) per chunk (wave-uniform)
template <class F>
__device__ inline void rq_drain(unsigned* q, int64_t n, int ch, int h, F& f) {
  const int64_t lo = n * h / kRqHeads, hi = n * (h + 1) / kRqHeads;
  if (lo >= hi) return;
  unsigned* head = q + h * kRqStride;
  unsigned t = rq_take(head);
  while (true) {
    const int64_t r0 = lo + (int64_t)__shfl(t, 0) * ch;
    if (r0 >= hi) return;
    t = rq_take(head);  // the next ticket is in flight while this chunk runs
    f(r0, r0 + ch < hi ? r0 + ch : hi);
  }
}

// f(r0, r1) for chunks [r0, r1) of [0, n) until every head is drained (wave-uniform):
// the wave's own XCD's head first, then, with lanes 0..7 reading all heads in one
// instruction, the next head (after its own) that still has rows — one round trip per
// steal instead of one per head, which short launches feel
template <class F>
__device__ inline void rq_for_each(unsigned* q, int64_t n, int ch, F&& f) {
  const int home = xcc_id();
  rq_drain(q, n, ch, home, f);
  const int lane = threadIdx.x & 63;
  while (true) {
    bool open = false;
    if (lane < kRqHeads) {
      const int64_t lo = n * lane / kRqHeads, hi = n * (lane + 1) / kRqHeads;
      const unsigned v =
          __hip_atomic_load(q + lane * kRqStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      open = lo + (int64_t)v * ch < hi;
    }
    uint64_t m = __ballot(open) & ((1ull << kRqHeads) - 1);
    if (m == 0) return;
    m = ((m >> (home + 1)) | (m << (kRqHeads - 1 - home))) & ((1ull << kRqHeads) - 1);
    rq_drain(q, n, ch, (home + 1 + __builtin_ctzll(m)) & (kRqHeads - 1), f);
  }
}

// The same walk as rq_for_each as a cursor, for kernels whose whole block consumes one
// chunk at a time (one wave draws, the block processes): rq_next returns the next chunk
// [r0, r1) of [0, n) or false once every head is drained.  Wave-uniform; call rq_begin
// once, then rq_next until it returns false.
struct RqCursor {
  int home, h;
  unsigned t;
};

__device__ inline void rq_begin(RqCursor& c, unsigned* q) {
  c.home = xcc_id();
  c.h = c.home;
  c.t = rq_take(q + c.h * kRqStride);
}

__device__ inline bool rq_next(RqCursor& c, unsigned* q, int64_t n, int ch, int64_t& r0,
                               int64_t& r1) {
  const int lane = threadIdx.x & 63;
  while (true) {
    const int64_t lo = n * c.h / kRqHeads, hi = n * (c.h + 1) / kRqHeads;
    const int64_t s = lo + (int64_t)__shfl(c.t, 0) * ch;
    if (s < hi) {
      c.t = rq_take(q + c.h * kRqStride);  // in flight while this chunk runs
      r0 = s;
      r1 = s + ch < hi ? s + ch : hi;
      return true;
    }
    bool open = false;  // head c.h drained: the next head after home that has rows
    if (lane < kRqHeads) {
      const int64_t l2 = n * lane / kRqHeads, h2 = n * (lane + 1) / kRqHeads;
      const unsigned v =
          __hip_atomic_load(q + lane * kRqStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      open = l2 + (int64_t)v * ch < h2;
    }
    uint64_t m = __ballot(open) & ((1ull << kRqHeads) - 1);
    if (m == 0) return false;
    m = ((m >> (c.home + 1)) | (m << (kRqHeads - 1 - c.home))) & ((1ull << kRqHeads) - 1);
    c.h = (c.home + 1 + __builtin_ctzll(m)) & (kRqHeads - 1);
    c.t = rq_take(q + c.h * kRqStride);
  }
}

// end of a queued launch: after every wave of the block has left rq_for_each, one lane
// counts the block out; the last block of the grid zeroes the slot for its next user
__device__ inline void rq_finish(unsigned* q) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nblk = gridDim.x * gridDim.y * gridDim.z;
    unsigned* done = q + kRqHeads * kRqStride;
    if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        nblk - 1) {
      for (int h = 0; h < kRqHeads; ++h)
        __hip_atomic_store(q + h * kRqStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace gnnrec
