// a9 — the fanout pick shared by the per-layer sampler (sampler.hip) and the fused
// multi-layer sampler (sample_blocks.hip): a group of G lanes per seed, Floyd's algorithm
// keyed on a counter hash (restated in oracle/oracle.c: oracle_sample_*).
#pragma once
#include "common.hpp"

namespace gnnrec {

// A group of G lanes (G = 8..64, a power of two >= fanout) per seed.  Fanout
// choice for a row of degree deg > k: Robert Floyd's algorithm keyed on a
// counter hash (restated in oracle.c).  The hash of every step is independent
// of the others, so lane s computes step s's candidate; only the duplicate
// resolution is sequential (a ballot over the group's lanes < s per step).
// Picks are emitted in ascending position order: a lane's output slot = number
// of kept picks with a smaller position (picks are distinct), so no sort and
// no scratch array is needed.
constexpr int kMaxFanout = 64;

template <int G>
struct Group {
  int lane;        // lane within the group
  int base;        // first wave lane of the group
  uint64_t bits;   // the group's bits in a wave ballot
  __device__ Group() {
    const int wl = (int)(threadIdx.x & (kWave - 1));
    lane = wl & (G - 1);
    base = wl - lane;
    bits = (G == 64 ? ~0ull : ((1ull << G) - 1)) << base;
  }
  __device__ uint64_t ballot(bool p) const { return __ballot(p) & bits; }
  // set lanes of the group below this one
  __device__ int below(uint64_t mask) const {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
  }
};

template <int G>
__device__ inline int64_t floyd_pick(const Group<G>& grp, uint64_t key, int64_t v, int64_t deg,
                                     int k) {
  const int64_t jl = deg - k + grp.lane;  // this lane's step (valid for lane < k)
  const int64_t tl = grp.lane < k
      ? (int64_t)(hash3(key, (uint64_t)v, (uint64_t)jl) % (uint64_t)(jl + 1)) : -1;
  int64_t mine = -1;
  for (int s = 0; s < k; ++s) {
    const int64_t t = __shfl(tl, grp.base + s);
    const bool dup = grp.ballot(grp.lane < s && mine == t) != 0ull;
    if (grp.lane == s) mine = dup ? jl : t;
  }
  return mine;  // lanes >= k: -1
}

// lanes per seed: full rows 64 (long rows stream), else the smallest power of two >= fanout
inline int group_size(int64_t fanout) {
  if (fanout < 0 || fanout > 32) return 64;
  if (fanout > 16) return 32;
  if (fanout > 8) return 16;
  return 8;
}

}  // namespace gnnrec
