// a10 — block feature / edge-data gather: dst[i] = src[idx[i]] for rows of any
// fixed byte width (reference: DGL copies node features into blocks[0].srcdata
// and edge data into every block at block creation, read by src/train/run.py:112,340).
// Rows are moved in the widest unit their alignment allows (16, 8, 4 or 1 B), one
// unit per thread, consecutive threads on consecutive units of a row — so a 512-B
// feature row is one coalesced 16-B-per-lane sweep and 8-B edge ids pack 8 rows per
// 64 B.
#include "common.hpp"

namespace gnnrec {
namespace {

template <typename U>
__global__ __launch_bounds__(256) void gather_rows_kernel(const char* __restrict__ src,
                                                          int64_t src_ld,
                                                          const int64_t* __restrict__ idx,
                                                          int64_t n, int64_t units_per_row,
                                                          char* __restrict__ dst, int64_t dst_ld) {
  const int64_t total = n * units_per_row;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / units_per_row, u = t - row * units_per_row;
    const int64_t r = idx[row];
    U* d = reinterpret_cast<U*>(dst + row * dst_ld) + u;
    if (r < 0) {  // a padding slot of a static-shape block: a zero row
      *d = U{};
      continue;
    }
    *d = *(reinterpret_cast<const U*>(src + r * src_ld) + u);
  }
}

template <typename U>
int launch(const void* src, int64_t src_ld, const int64_t* idx, int64_t n, int64_t row_bytes,
           void* dst, int64_t dst_ld, hipStream_t s) {
  const int64_t upr = row_bytes / (int64_t)sizeof(U);
  const int64_t total = n * upr;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(gather_rows_kernel<U>, dim3((unsigned)blocks), dim3(256), 0, s,
                     static_cast<const char*>(src), src_ld, idx, n, upr, static_cast<char*>(dst),
                     dst_ld);
  return check_launch("gnnrec_gather_rows");
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_gather_rows(const void* src, int64_t src_ld_bytes, const int64_t* idx,
                                  int64_t n, int64_t row_bytes, void* dst, int64_t dst_ld_bytes,
                                  void* stream) {
  GNNREC_REQUIRE(n >= 0 && row_bytes >= 0, "gnnrec_gather_rows: negative size");
  if (n == 0 || row_bytes == 0) return GNNREC_OK;
  GNNREC_REQUIRE(src && idx && dst, "gnnrec_gather_rows: null pointer");
  GNNREC_REQUIRE(src_ld_bytes >= row_bytes && dst_ld_bytes >= row_bytes,
                 "gnnrec_gather_rows: row stride below the row width");
  const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                       (uintptr_t)src_ld_bytes | (uintptr_t)dst_ld_bytes | (uintptr_t)row_bytes;
  hipStream_t s = as_stream(stream);
  if ((al & 15u) == 0) return launch<uint4>(src, src_ld_bytes, idx, n, row_bytes, dst, dst_ld_bytes, s);
  if ((al & 7u) == 0) return launch<uint64_t>(src, src_ld_bytes, idx, n, row_bytes, dst, dst_ld_bytes, s);
  if ((al & 3u) == 0) return launch<uint32_t>(src, src_ld_bytes, idx, n, row_bytes, dst, dst_ld_bytes, s);
  return launch<uint8_t>(src, src_ld_bytes, idx, n, row_bytes, dst, dst_ld_bytes, s);
}

// ---- many gathers in one launch (a sampled batch's edge data + input features) ----
namespace gnnrec {
namespace {

struct GatherJobs {
  const char* src[GNNREC_GATHER_MAX_JOBS];
  char* dst[GNNREC_GATHER_MAX_JOBS];
  const int64_t* idx[GNNREC_GATHER_MAX_JOBS];
  int64_t src_ld[GNNREC_GATHER_MAX_JOBS], dst_ld[GNNREC_GATHER_MAX_JOBS];
  int64_t n[GNNREC_GATHER_MAX_JOBS], upr[GNNREC_GATHER_MAX_JOBS];
  const int64_t* n_dev[GNNREC_GATHER_MAX_JOBS];
  int unit[GNNREC_GATHER_MAX_JOBS];  // log2 of the unit bytes: 4, 3, 2 or 0
  int block0[GNNREC_GATHER_MAX_JOBS + 1];
  int n_jobs;
};

template <typename U>
__device__ __forceinline__ void gather_job(const GatherJobs& J, int j, int64_t t0, int64_t step) {
  const int64_t rows = J.n_dev[j] ? min(*J.n_dev[j], J.n[j]) : J.n[j];
  const int64_t upr = J.upr[j], total = rows * upr;
  for (int64_t t = t0; t < total; t += step) {
    const int64_t row = t / upr, u = t - row * upr;
    const int64_t r = J.idx[j][row];
    U* d = reinterpret_cast<U*>(J.dst[j] + row * J.dst_ld[j]) + u;
    if (r < 0) {  // a padding slot of a static-shape block: a zero row
      *d = U{};
      continue;
    }
    *d = *(reinterpret_cast<const U*>(J.src[j] + r * J.src_ld[j]) + u);
  }
}

__global__ __launch_bounds__(256) void gather_rows_batch_kernel(GatherJobs J) {
  int j = 0;
  while (j + 1 < J.n_jobs && (int)blockIdx.x >= J.block0[j + 1]) ++j;  // block-uniform
  const int nb = J.block0[j + 1] - J.block0[j];
  const int64_t t0 = (int64_t)((int)blockIdx.x - J.block0[j]) * 256 + threadIdx.x;
  const int64_t step = (int64_t)nb * 256;
  switch (J.unit[j]) {
    case 4: gather_job<uint4>(J, j, t0, step); break;
    case 3: gather_job<uint64_t>(J, j, t0, step); break;
    case 2: gather_job<uint32_t>(J, j, t0, step); break;
    default: gather_job<uint8_t>(J, j, t0, step); break;
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_gather_rows_batch(const gnnrec_gather_job* jobs, int n_jobs, void* stream) {
  GNNREC_REQUIRE(n_jobs >= 0 && n_jobs <= GNNREC_GATHER_MAX_JOBS,
                 "gnnrec_gather_rows_batch: n_jobs=%d (0..%d)", n_jobs, GNNREC_GATHER_MAX_JOBS);
  GNNREC_REQUIRE(n_jobs == 0 || jobs, "gnnrec_gather_rows_batch: null jobs");
  gnnrec::GatherJobs J{};
  int blocks = 0;
  for (int i = 0; i < n_jobs; ++i) {
    const gnnrec_gather_job& g = jobs[i];
    GNNREC_REQUIRE(g.n >= 0 && g.row_bytes >= 0, "gnnrec_gather_rows_batch: job %d: negative size", i);
    if (g.n == 0 || g.row_bytes == 0) continue;
    GNNREC_REQUIRE(g.src && g.idx && g.dst, "gnnrec_gather_rows_batch: job %d: null pointer", i);
    GNNREC_REQUIRE(g.src_ld_bytes >= g.row_bytes && g.dst_ld_bytes >= g.row_bytes,
                   "gnnrec_gather_rows_batch: job %d: row stride below the row width", i);
    const uintptr_t al = reinterpret_cast<uintptr_t>(g.src) | reinterpret_cast<uintptr_t>(g.dst) |
                         (uintptr_t)g.src_ld_bytes | (uintptr_t)g.dst_ld_bytes | (uintptr_t)g.row_bytes;
    const int unit = (al & 15u) == 0 ? 4 : (al & 7u) == 0 ? 3 : (al & 3u) == 0 ? 2 : 0;
    const int k = J.n_jobs++;
    J.src[k] = static_cast<const char*>(g.src);
    J.dst[k] = static_cast<char*>(g.dst);
    J.idx[k] = g.idx;
    J.src_ld[k] = g.src_ld_bytes;
    J.dst_ld[k] = g.dst_ld_bytes;
    J.n[k] = g.n;
    J.n_dev[k] = g.n_dev;
    J.unit[k] = unit;
    J.upr[k] = g.row_bytes >> unit;
    int64_t nb = (g.n * J.upr[k] + 255) / 256;
    if (nb > 8192) nb = 8192;  // grid-stride beyond: 2M units in flight per job
    J.block0[k] = blocks;
    blocks += (int)nb;
  }
  if (J.n_jobs == 0) return GNNREC_OK;
  J.block0[J.n_jobs] = blocks;
  hipLaunchKernelGGL(gnnrec::gather_rows_batch_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     gnnrec::as_stream(stream), J);
  return gnnrec::check_launch("gnnrec_gather_rows_batch");
}

// ---- many contiguous copies in one launch (a captured step's input hand-over) ----
namespace gnnrec {
namespace {

struct CopyJobs {
  const char* src[GNNREC_COPY_MAX_JOBS];
  char* dst[GNNREC_COPY_MAX_JOBS];
  int64_t units[GNNREC_COPY_MAX_JOBS];
  int unit[GNNREC_COPY_MAX_JOBS];  // log2 of the unit bytes: 4 or 0
  int block0[GNNREC_COPY_MAX_JOBS + 1];
  int n;
};

template <typename U>
__device__ __forceinline__ void copy_job(const CopyJobs& J, int j, int64_t t0, int64_t step) {
  const U* s = reinterpret_cast<const U*>(J.src[j]);
  U* d = reinterpret_cast<U*>(J.dst[j]);
  for (int64_t t = t0; t < J.units[j]; t += step) d[t] = s[t];
}

__global__ __launch_bounds__(256) void copy_batch_kernel(CopyJobs J) {
  int j = 0;
  while (j + 1 < J.n && (int)blockIdx.x >= J.block0[j + 1]) ++j;  // block-uniform
  const int64_t t0 = (int64_t)((int)blockIdx.x - J.block0[j]) * 256 + threadIdx.x;
  const int64_t step = (int64_t)(J.block0[j + 1] - J.block0[j]) * 256;
  if (J.unit[j] == 4) copy_job<uint4>(J, j, t0, step);
  else copy_job<uint8_t>(J, j, t0, step);
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_copy_batch(const void* const* src, void* const* dst, const int64_t* bytes,
                                 int n, void* stream) {
  GNNREC_REQUIRE(n >= 0 && n <= GNNREC_COPY_MAX_JOBS, "gnnrec_copy_batch: n=%d (0..%d)", n,
                 GNNREC_COPY_MAX_JOBS);
  GNNREC_REQUIRE(n == 0 || (src && dst && bytes), "gnnrec_copy_batch: null arrays");
  gnnrec::CopyJobs J{};
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    GNNREC_REQUIRE(bytes[i] >= 0, "gnnrec_copy_batch: job %d: negative size", i);
    if (bytes[i] == 0) continue;
    GNNREC_REQUIRE(src[i] && dst[i], "gnnrec_copy_batch: job %d: null pointer", i);
    const uintptr_t al = reinterpret_cast<uintptr_t>(src[i]) | reinterpret_cast<uintptr_t>(dst[i]) |
                         (uintptr_t)bytes[i];
    const int k = J.n++;
    J.src[k] = static_cast<const char*>(src[i]);
    J.dst[k] = static_cast<char*>(dst[i]);
    J.unit[k] = (al & 15u) == 0 ? 4 : 0;
    J.units[k] = bytes[i] >> J.unit[k];
    int64_t nb = (J.units[k] + 255) / 256;
    if (nb > 4096) nb = 4096;  // grid-stride beyond: 1M units in flight per job
    J.block0[k] = blocks;
    blocks += (int)nb;
  }
  if (J.n == 0) return GNNREC_OK;
  J.block0[J.n] = blocks;
  hipLaunchKernelGGL(gnnrec::copy_batch_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     gnnrec::as_stream(stream), J);
  return gnnrec::check_launch("gnnrec_copy_batch");
}

// ---- partial-table add (the deterministic pass's fixed tree over source-range tiles) ----
namespace gnnrec {
namespace {

// 4 float4 per thread, all loads issued before the adds (8 x 16 B in flight per lane)
constexpr int kAddU = 4;
__global__ __launch_bounds__(256) void add_f32x4_kernel(const float4* __restrict__ a,
                                                        const float4* __restrict__ b,
                                                        float4* __restrict__ out, int64_t n4) {
  const int64_t base = (int64_t)blockIdx.x * (256 * kAddU) + threadIdx.x;
  float4 x[kAddU], y[kAddU];
#pragma unroll
  for (int k = 0; k < kAddU; ++k) {
    const int64_t i = base + k * 256;
    if (i < n4) {
      x[k] = a[i];
      y[k] = b[i];
    }
  }
#pragma unroll
  for (int k = 0; k < kAddU; ++k) {
    const int64_t i = base + k * 256;
    if (i < n4) out[i] = make_float4(x[k].x + y[k].x, x[k].y + y[k].y, x[k].z + y[k].z,
                                     x[k].w + y[k].w);
  }
}

__global__ __launch_bounds__(256) void add_f32_kernel(const float* __restrict__ a,
                                                      const float* __restrict__ b,
                                                      float* __restrict__ out, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = a[i] + b[i];
}

// Whole fixed pairwise tree ((p0+p1)+(p2+p3))+... over NP = 2/4/8 tables in one pass:
// every input read once and one write, instead of NP-1 add launches that re-read and
// re-write the intermediate sums (the same additions in the same order: bitwise equal)
struct TreeParts {
  const float4* p[8];
};
template <int NP>
__global__ __launch_bounds__(256) void tree_sum_f32x4_kernel(TreeParts parts,
                                                             float4* __restrict__ out,
                                                             int64_t n4) {
  constexpr int U = NP >= 8 ? 2 : 4;  // 16 x 16 B in flight per lane
  const int64_t base = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  float4 x[U][NP];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int64_t i = base + k * 256;
    if (i < n4) {
#pragma unroll
      for (int j = 0; j < NP; ++j) x[k][j] = parts.p[j][i];
    }
  }
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int64_t i = base + k * 256;
    if (i < n4) {
#pragma unroll
      for (int w = 1; w < NP; w <<= 1) {
#pragma unroll
        for (int j = 0; j < NP; j += 2 * w)
          x[k][j] = make_float4(x[k][j].x + x[k][j + w].x, x[k][j].y + x[k][j + w].y,
                                x[k][j].z + x[k][j + w].z, x[k][j].w + x[k][j + w].w);
      }
      out[i] = x[k][0];
    }
  }
}

template <int NP>
void launch_tree(const float* const* parts, int64_t n4, float* out, hipStream_t s) {
  constexpr int U = NP >= 8 ? 2 : 4;
  TreeParts tp{};
  for (int j = 0; j < NP; ++j) tp.p[j] = reinterpret_cast<const float4*>(parts[j]);
  const int64_t blocks = (n4 + 256 * U - 1) / (256 * U);
  hipLaunchKernelGGL(tree_sum_f32x4_kernel<NP>, dim3((unsigned)blocks), dim3(256), 0, s, tp,
                     reinterpret_cast<float4*>(out), n4);
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_add_f32(const float* a, const float* b, float* out, int64_t n,
                              void* stream) {
  GNNREC_REQUIRE(n >= 0, "gnnrec_add_f32: negative size");
  if (n == 0) return GNNREC_OK;
  GNNREC_REQUIRE(a && b && out, "gnnrec_add_f32: null pointer");
  hipStream_t s = as_stream(stream);
  const bool v4 = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                    reinterpret_cast<uintptr_t>(out)) & 15u) == 0 && n % 4 == 0;
  if (v4) {
    const int64_t n4 = n / 4;
    const int64_t blocks = (n4 + 256 * kAddU - 1) / (256 * kAddU);
    GNNREC_REQUIRE(blocks < (int64_t(1) << 31), "gnnrec_add_f32: n too large");
    hipLaunchKernelGGL(add_f32x4_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
                       reinterpret_cast<float4*>(out), n4);
  } else {
    int64_t blocks = (n + 255) / 256;
    if (blocks > 256 * 32) blocks = 256 * 32;
    hipLaunchKernelGGL(add_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, out, n);
  }
  return check_launch("gnnrec_add_f32");
}

extern "C" int gnnrec_tree_sum_f32(const float* const* parts, int n_parts, int64_t n, float* out,
                                   void* stream) {
  GNNREC_REQUIRE(n >= 0, "gnnrec_tree_sum_f32: negative size");
  GNNREC_REQUIRE(n_parts == 2 || n_parts == 4 || n_parts == 8,
                 "gnnrec_tree_sum_f32: n_parts=%d (2, 4 or 8)", n_parts);
  if (n == 0) return GNNREC_OK;
  GNNREC_REQUIRE(parts && out, "gnnrec_tree_sum_f32: null pointer");
  uintptr_t al = reinterpret_cast<uintptr_t>(out);
  for (int j = 0; j < n_parts; ++j) {
    GNNREC_REQUIRE(parts[j], "gnnrec_tree_sum_f32: null part %d", j);
    al |= reinterpret_cast<uintptr_t>(parts[j]);
  }
  hipStream_t s = as_stream(stream);
  GNNREC_REQUIRE((al & 15u) == 0 && n % 4 == 0,
                 "gnnrec_tree_sum_f32: tables must be 16-B aligned with n %% 4 == 0");
  const int64_t n4 = n / 4;
  GNNREC_REQUIRE(n4 / 512 < (int64_t(1) << 31), "gnnrec_tree_sum_f32: n too large");
  switch (n_parts) {
    case 2: launch_tree<2>(parts, n4, out, s); break;
    case 4: launch_tree<4>(parts, n4, out, s); break;
    default: launch_tree<8>(parts, n4, out, s); break;
  }
  return check_launch("gnnrec_tree_sum_f32");
}
