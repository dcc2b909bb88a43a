// f2 — training-step companions of the projection GEMMs (reference model.py:98-102,
// 226-235, 256-271 under torch autograd):
//   * weight gradient  C[M,N] (+)= A[K,M]^T · B[K,N]   (dW = dYᵀ·X, K = rows ≫ M,N)
//     as a deterministic split-K fp32 MFMA: one launch writes per-split partials,
//     a second sums them in split order;
//   * the row-wise backward of the fused ReLU / zero-guarded L2-norm epilogue
//     (z = u / (‖u‖ or 1)), so the projection's input gradients are two plain GEMMs.
#include "common.hpp"

namespace gnnrec {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 128;       // output super-tile per block (M and N)
constexpr int kKStep = 16;       // rows per unrolled step (8 MFMA k-pairs)
constexpr int kTargetBlocks = 1024;

// Block: 4 waves; wave w owns output rows [32w, 32w+32) of the super-tile and all
// four 32-column blocks.  MFMA 32x32x2 f32 operands: lane l supplies
// A^T[i=l&31][k=l>>5] = A[k][i] and B[k=l>>5][j=l&31]; both are 32 consecutive
// floats of one input row per half-wave (coalesced 128-B segments).
__global__ __launch_bounds__(256) void gemm_tn_partial_kernel(
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
    int64_t K, int64_t M, int64_t N, int64_t kchunk, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, lk = lane >> 5;
  const int64_t split = blockIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * kTile + 32 * w;
  const int64_t j0 = (int64_t)blockIdx.z * kTile;
  const int64_t kb = split * kchunk, ke = kb + kchunk < K ? kb + kchunk : K;

  f32x16 acc[4];
  for (int q = 0; q < 4; ++q)
    for (int v = 0; v < 16; ++v) acc[q][v] = 0.f;

  // clamped (always in-bounds) addresses, zeroed by select: branch-free loads
  const bool ia_ok = i0 + li < M;
  const int64_t ia = ia_ok ? i0 + li : 0;
  bool jb_ok[4];
  int64_t jb[4];
  for (int q = 0; q < 4; ++q) {
    jb_ok[q] = j0 + 32 * q + li < N;
    jb[q] = jb_ok[q] ? j0 + 32 * q + li : 0;
  }
  if (kb < ke) {
    for (int64_t k0 = kb; k0 < ke; k0 += kKStep) {
      float a[kKStep / 2], b[kKStep / 2][4];
#pragma unroll
      for (int s = 0; s < kKStep / 2; ++s) {
        const int64_t k = k0 + 2 * s + lk;
        const bool k_ok = k < ke;
        const int64_t kc = k_ok ? k : ke - 1;
        const float av = A[kc * lda + ia];
        a[s] = (k_ok && ia_ok) ? av : 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float bv = B[kc * ldb + jb[q]];
          b[s][q] = (k_ok && jb_ok[q]) ? bv : 0.f;
        }
      }
#pragma unroll
      for (int s = 0; s < kKStep / 2; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s][q], acc[q], 0, 0, 0);
    }
  }
  float* P = part + split * M * N;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t j = j0 + 32 * q + li;
    if (j >= N) continue;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int64_t i = i0 + (v & 3) + 8 * (v >> 2) + 4 * lk;
      if (i < M) P[i * N + j] = acc[q][v];
    }
  }
}

__global__ void gemm_tn_reduce_kernel(const float* __restrict__ part, int64_t splits, int64_t M,
                                      int64_t N, float* __restrict__ C, int64_t ldc,
                                      int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * N) return;
  float s = 0.f;
  for (int64_t p = 0; p < splits; ++p) s += part[p * M * N + t];
  const int64_t i = t / N, j = t - i * N;
  float* c = C + i * ldc + j;
  *c = accumulate ? *c + s : s;
}

inline int64_t tn_splits(int64_t K, int64_t M, int64_t N) {
  const int64_t tiles = ((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  int64_t s = kTargetBlocks / (tiles > 0 ? tiles : 1);
  const int64_t by_rows = (K + 255) / 256;  // >= 256 rows per split
  if (s > by_rows) s = by_rows;
  return s < 1 ? 1 : s;
}

inline int64_t tn_chunk(int64_t K, int64_t splits) {
  const int64_t c = (K + splits - 1) / splits;
  return (c + kKStep - 1) / kKStep * kKStep;
}

// z = u / (‖u‖ or 1) [L2NORM] after relu [RELU]; gu from gz (u = pre-activation when RELU,
// recomputed by the caller).  One wave per row.
__global__ __launch_bounds__(256) void act_backward_kernel(
    const float* __restrict__ u, int64_t ldu, const float* __restrict__ gz, int64_t ldg,
    int64_t n_rows, int64_t d, int flags, float* __restrict__ gu, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const float* ur = u + r * ldu;
  const float* gr = gz + r * ldg;
  float* orow = gu + r * ldo;
  const bool relu = flags & GNNREC_EPI_RELU, l2 = flags & GNNREC_EPI_L2NORM;
  float ss = 0.f, dot = 0.f;
  if (l2) {
    for (int64_t c = lane; c < d; c += 64) {
      const float a = relu ? fmaxf(ur[c], 0.f) : ur[c];
      ss += a * a;
      dot += a * gr[c];
    }
    for (int off = 32; off > 0; off >>= 1) {
      ss += __shfl_xor(ss, off);
      dot += __shfl_xor(dot, off);
    }
  }
  const float n = sqrtf(ss);
  const bool scale = l2 && n != 0.f;
  const float inv = scale ? 1.f / n : 1.f;
  // gu = (gz - a·(a·gz)/n²) / n  for n > 0, else gz; then the relu mask
  const float coef = scale ? dot * inv * inv : 0.f;
  for (int64_t c = lane; c < d; c += 64) {
    const float x = ur[c];
    const float a = relu ? fmaxf(x, 0.f) : x;
    float g = (gr[c] - a * coef) * inv;
    if (relu && !(x > 0.f)) g = 0.f;
    orow[c] = g;
  }
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int64_t gnnrec_gemm_tn_workspace_bytes(int64_t K, int64_t M, int64_t N) {
  if (K <= 0 || M <= 0 || N <= 0) return 0;
  return tn_splits(K, M, N) * M * N * (int64_t)sizeof(float);
}

extern "C" int gnnrec_gemm_tn_f32(const float* A, int64_t lda, const float* B, int64_t ldb,
                                  int64_t K, int64_t M, int64_t N, float* C, int64_t ldc,
                                  int accumulate, float* workspace, void* stream) {
  GNNREC_REQUIRE(K >= 0 && M >= 0 && N >= 0, "gnnrec_gemm_tn_f32: negative size");
  GNNREC_REQUIRE(lda >= M && ldb >= N && ldc >= N, "gnnrec_gemm_tn_f32: bad leading dims");
  if (M == 0 || N == 0) return GNNREC_OK;
  hipStream_t s = as_stream(stream);
  if (K == 0) {
    if (accumulate) return GNNREC_OK;
    if (hipMemset2DAsync(C, ldc * sizeof(float), 0, N * sizeof(float), M, s) != hipSuccess) {
      set_error("gnnrec_gemm_tn_f32: hipMemset2DAsync failed");
      return GNNREC_EHIP;
    }
    return GNNREC_OK;
  }
  GNNREC_REQUIRE(A && B && C && workspace, "gnnrec_gemm_tn_f32: null pointer");
  const int64_t splits = tn_splits(K, M, N), chunk = tn_chunk(K, splits);
  const dim3 grid((unsigned)splits, (unsigned)((M + kTile - 1) / kTile),
                  (unsigned)((N + kTile - 1) / kTile));
  hipLaunchKernelGGL(gemm_tn_partial_kernel, grid, dim3(256), 0, s, A, lda, B, ldb, K, M, N,
                     chunk, workspace);
  const int64_t mn = M * N;
  hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, s,
                     workspace, splits, M, N, C, ldc, accumulate);
  return check_launch("gnnrec_gemm_tn_f32");
}

extern "C" int gnnrec_act_backward_f32(const float* u, int64_t ldu, const float* gz, int64_t ldg,
                                       int64_t n_rows, int64_t d, int flags, float* gu,
                                       int64_t ldo, void* stream) {
  GNNREC_REQUIRE(n_rows >= 0 && d >= 0, "gnnrec_act_backward_f32: negative size");
  GNNREC_REQUIRE(ldu >= d && ldg >= d && ldo >= d, "gnnrec_act_backward_f32: bad leading dims");
  GNNREC_REQUIRE((flags & ~(GNNREC_EPI_RELU | GNNREC_EPI_L2NORM)) == 0,
                 "gnnrec_act_backward_f32: flags must be RELU|L2NORM");
  if (n_rows == 0 || d == 0) return GNNREC_OK;
  hipLaunchKernelGGL(act_backward_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0,
                     as_stream(stream), u, ldu, gz, ldg, n_rows, d, flags, gu, ldo);
  return check_launch("gnnrec_act_backward_f32");
}
