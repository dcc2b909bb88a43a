// Shared helpers for the gnnrec HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>

#include "gnnrec.h"

namespace gnnrec {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return GNNREC_EHIP;
  }
  return GNNREC_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// CDNA4 wavefront is 64 lanes.
constexpr int kWave = 64;

// Lane group g (of NPW groups of kWave / NPW consecutive lanes) receives lane (base + g)'s x,
// base wave-uniform: NPW v_readlane (VALU -> SGPR) and selects, where __shfl is one
// ds_bpermute through the LDS pipe per call.  Lane indices wrap at 64 (a group whose lane
// is past the data ignores the value).
template <int NPW>
__device__ __forceinline__ int bcast_groups(int x, int base, int grp) {
  int r = __builtin_amdgcn_readlane(x, base & 63);
#pragma unroll
  for (int g = 1; g < NPW; ++g) {
    const int y = __builtin_amdgcn_readlane(x, (base + g) & 63);
    r = grp == g ? y : r;
  }
  return r;
}
template <int NPW>
__device__ __forceinline__ float bcast_groups(float x, int base, int grp) {
  return __builtin_bit_cast(float, bcast_groups<NPW>(__builtin_bit_cast(int, x), base, grp));
}

// 64-bit counter hash (splitmix64 finaliser): the synthetic generator and the
// Philox-free fanout sampler both key on it; oracle/oracle.c restates it.
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t hash3(uint64_t seed, uint64_t a, uint64_t b) {
  return mix64(mix64(seed ^ mix64(a)) ^ (b * 0xD1B54A32D192ED03ull));
}

}  // namespace gnnrec

#define GNNREC_REQUIRE(cond, ...)        \
  do {                                   \
    if (!(cond)) {                       \
      ::gnnrec::set_error(__VA_ARGS__);  \
      return GNNREC_EINVAL;              \
    }                                    \
  } while (0)
