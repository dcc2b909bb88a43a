// Synthetic bipartite edge generator for the benchmark graph shapes
// (BASELINE.json configs; no reference counterpart — the reference reads
// real data through src/builder.py).  Counter-based: edge e's endpoints are
// a pure function of (seed, e), so every rank of a sharded run regenerates
// exactly the edges it needs without any exchange, and oracle/oracle.c
// reproduces the same graph bit for bit.
//   user(e) = hash3(seed, e, 0) mod n_u
//   item(e) = hash3(seed, e, 1) mod n_i                      (uniform)
//           = first j with cdf[j] > U53(hash3(seed, e, 1))   (Zipf, cdf given)
// U53(x) = (x >> 11) * 2^-53.
#include "common.hpp"

namespace gnnrec {
namespace {

__global__ void synth_edges_kernel(uint64_t seed, int64_t e0, int64_t n, int64_t n_u, int64_t n_i,
                                   const double* __restrict__ cdf, int32_t* __restrict__ u,
                                   int32_t* __restrict__ it) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint64_t e = (uint64_t)(e0 + k);
  u[k] = (int32_t)(hash3(seed, e, 0) % (uint64_t)n_u);
  const uint64_t hi = hash3(seed, e, 1);
  if (!cdf) {
    it[k] = (int32_t)(hi % (uint64_t)n_i);
  } else {
    const double x = (double)(hi >> 11) * (1.0 / 9007199254740992.0);
    int64_t lo = 0, hi_ = n_i - 1;  // first j with cdf[j] > x
    while (lo < hi_) {
      const int64_t mid = (lo + hi_) >> 1;
      if (cdf[mid] > x) hi_ = mid;
      else lo = mid + 1;
    }
    it[k] = (int32_t)lo;
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_synth_edges(uint64_t seed, int64_t e0, int64_t n, int64_t n_u, int64_t n_i,
                                  const double* zipf_cdf, int32_t* u, int32_t* i, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(n >= 0 && e0 >= 0, "gnnrec_synth_edges: negative range");
  GNNREC_REQUIRE(n_u > 0 && n_i > 0 && n_u < (1ll << 31) && n_i < (1ll << 31),
                 "gnnrec_synth_edges: node counts must be in [1, 2^31)");
  if (n == 0) return GNNREC_OK;
  GNNREC_REQUIRE(u && i, "gnnrec_synth_edges: null output");
  hipLaunchKernelGGL(synth_edges_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), seed, e0, n, n_u, n_i, zipf_cdf, u, i);
  return check_launch("gnnrec_synth_edges");
}
