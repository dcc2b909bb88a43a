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
