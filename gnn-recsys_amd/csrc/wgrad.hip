// f2 — training-step companions of the projection GEMMs (reference model.py:98-102,
// 226-235, 256-271 under torch autograd):
//   * weight gradient  C[M,N] (+)= A[K,M]^T · B[K,N]   (dW = dYᵀ·X, K = rows ≫ M,N)
//     as a deterministic split-K fp32 MFMA: one launch writes per-split partials,
//     a second sums them in split order;
//   * the row-wise backward of the fused ReLU / zero-guarded L2-norm epilogue
//     (z = u / (‖u‖ or 1)), so the projection's input gradients are two plain GEMMs.
#include "common.hpp"
#include <cstdlib>

namespace gnnrec {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 128;       // output super-tile per block (M and N)
constexpr int kKStep = 16;       // input rows per pipeline step (8 MFMA k-pairs)
constexpr int kTargetBlocks = 512;

// One KS-row step of a [K, ld] operand restricted to columns [c0, c0+T):
// KS·T/4 float4 slots, KS·T/1024 per thread (row = slot / (T/4), cols 4*(slot % (T/4)) .. +3).
// VEC: 16-B loads (ld % 4 == 0, 16-B aligned base, full columns checked per slot);
// otherwise per-element loads.  Rows >= ke and columns >= ncol read as zero.
template <bool VEC, int T, int KS>
__device__ inline void load_step(const float* __restrict__ X, int64_t ld, int64_t ncol,
                                 int64_t c0, int64_t k0, int64_t ke, float4 (&r)[KS * T / 1024]) {
#pragma unroll
  for (int h = 0; h < KS * T / 1024; ++h) {
    const int slot = threadIdx.x + 256 * h;
    const int64_t k = k0 + slot / (T / 4);
    const int64_t c = c0 + 4 * (slot % (T / 4));
    const bool k_ok = k < ke;
    const int64_t kc = k_ok ? k : ke - 1;
    const float* row = X + kc * ld;
    if (VEC) {
      const bool c_ok = c < ncol;  // ncol % 4 == 0 on this path
      const float4 v = *reinterpret_cast<const float4*>(row + (c_ok ? c : 0));
      const bool ok = k_ok && c_ok;
      r[h] = make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
    } else {
      float e[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = k_ok && c + q < ncol;
        const float v = row[ok ? c + q : 0];
        e[q] = ok ? v : 0.f;
      }
      r[h] = make_float4(e[0], e[1], e[2], e[3]);
    }
  }
}

template <int T, int KS>
__device__ inline void store_step(float* lds, const float4 (&r)[KS * T / 1024]) {
#pragma unroll
  for (int h = 0; h < KS * T / 1024; ++h) {
    const int slot = threadIdx.x + 256 * h;
    *reinterpret_cast<float4*>(lds + (slot / (T / 4)) * (T + 4) + 4 * (slot % (T / 4))) = r[h];
  }
}

// Block: 4 waves as 2x2 wave tiles of T/2 x T/2 (NT x NT MFMA 32x32 tiles each, NT = T/64)
// over a T x T output super-tile; K slice [kb, ke) streamed through double-buffered LDS
// with a register prefetch of the next KS-row step (one barrier per step).
// MFMA 32x32x2 f32 operands: lane l supplies A^T[i=l&31][k=l>>5] = A[k][i] and
// B[k=l>>5][j=l&31]; both are consecutive LDS words across the half-wave.
// T = 64 serves M, N <= 64 (the d = 64 layers of the minibatch step): the 128 tile spent
// 3/4 of its MFMAs on zero padding and was MFMA-bound at 4x the useful work.  Its steps
// are KS = 64 rows (8 KB of each operand per block in flight, not 2): at 16 rows the
// 512 blocks kept 4 MB in flight and a 200k-row gradient ran latency-bound at 2 TB/s.
// Rows past the split read as zero and add exact zeros, so the partials do not depend on
// KS: every output element sees the same MFMA sequence over the same split.
template <bool VEC, int T, int KS>
__global__ __launch_bounds__(256) void gemm_tn_partial_kernel(
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
    int64_t K, int64_t M, int64_t N, int64_t kchunk, float* __restrict__ part,
    float* __restrict__ part_b, const int64_t* __restrict__ row_ptr) {
  constexpr int NT = T / 64, S = T + 4, LI = KS * T / 1024;
  __shared__ float As[2][KS * S];
  __shared__ float Bs[2][KS * S];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 31, lk = lane >> 5;
  const int wi = (w & 1) * (T / 2), wj = (w >> 1) * (T / 2);
  const int64_t split = blockIdx.x;
  const int64_t i_base = (int64_t)blockIdx.y * T, j_base = (int64_t)blockIdx.z * T;
  const int64_t kb = split * kchunk, ke = kb + kchunk < K ? kb + kchunk : K;

  // part_b: column sums of A over this split (the bias gradient Σ_k dY[k, i]); the blocks
  // of the first N tile add up the A tiles they already hold in LDS.  row_ptr (nullable):
  // only rows k with row_ptr[k+1] > row_ptr[k] count (a folded NodeEmbedding's bias on the
  // rows with an in-edge): lane r of a summing wave loads step row r's test with the step's
  // operand prefetch, and a ballot hands the wave the step's row mask
  const bool colsum = part_b != nullptr && blockIdx.z == 0 && threadIdx.x < T;
  const bool masked = colsum && row_ptr != nullptr;
  const int mlane = threadIdx.x & 63;
  auto row_ne = [&](int64_t k0, int64_t ke) {
    const int64_t k = k0 + mlane;
    return mlane < KS && k < ke && row_ptr[k + 1] > row_ptr[k];
  };
  bool ne_cur = false, ne_next = false;
  float csum = 0.f;
  f32x16 acc[NT][NT];
#pragma unroll
  for (int x = 0; x < NT; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[x][y][v] = 0.f;

  if (kb < ke) {  // uniform per block
    float4 ra[LI], rb[LI];
    load_step<VEC, T, KS>(A, lda, M, i_base, kb, ke, ra);
    load_step<VEC, T, KS>(B, ldb, N, j_base, kb, ke, rb);
    if (masked) ne_cur = row_ne(kb, ke);
    store_step<T, KS>(As[0], ra);
    store_step<T, KS>(Bs[0], rb);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += KS) {
      const bool more = k0 + KS < ke;
      if (more) {
        load_step<VEC, T, KS>(A, lda, M, i_base, k0 + KS, ke, ra);
        load_step<VEC, T, KS>(B, ldb, N, j_base, k0 + KS, ke, rb);
        if (masked) ne_next = row_ne(k0 + KS, ke);
      }
      const float* as = As[buf];
      const float* bs = Bs[buf];
#pragma unroll 8
      for (int s = 0; s < KS / 2; ++s) {
        const int kr = (2 * s + lk) * S;
        float a[NT], b[NT];
#pragma unroll
        for (int x = 0; x < NT; ++x) {
          a[x] = as[kr + wi + 32 * x + li];
          b[x] = bs[kr + wj + 32 * x + li];
        }
#pragma unroll
        for (int x = 0; x < NT; ++x)
#pragma unroll
          for (int y = 0; y < NT; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[x], b[y], acc[x][y], 0, 0, 0);
      }
      if (colsum) {
        if (row_ptr == nullptr) {
#pragma unroll 16
          for (int r = 0; r < KS; ++r) csum += as[r * S + threadIdx.x];
        } else {  // (rows past the split test false)
          const unsigned long long mask = __ballot(ne_cur);
#pragma unroll 16
          for (int r = 0; r < KS; ++r)
            if ((mask >> r) & 1ull) csum += as[r * S + threadIdx.x];
        }
      }
      ne_cur = ne_next;
      if (more) {
        store_step<T, KS>(As[buf ^ 1], ra);
        store_step<T, KS>(Bs[buf ^ 1], rb);
      }
      __syncthreads();
      buf ^= 1;
    }
  }
  if (colsum && i_base + threadIdx.x < M) part_b[split * M + i_base + threadIdx.x] = csum;
  float* P = part + split * M * N;
#pragma unroll
  for (int x = 0; x < NT; ++x)
#pragma unroll
    for (int y = 0; y < NT; ++y) {
      const int64_t j = j_base + wj + 32 * y + li;
      if (j >= N) continue;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t i = i_base + wi + 32 * x + (v & 3) + 8 * (v >> 2) + 4 * lk;
        if (i < M) P[i * N + j] = acc[x][y][v];
      }
    }
}

// C = (accumulate ? C : 0) + sum_p part[p]; 64 outputs per block, the 4 waves sum
// interleaved quarters of the splits, combined in a fixed order (deterministic).
__global__ __launch_bounds__(256) void gemm_tn_reduce_kernel(
    const float* __restrict__ part, const float* __restrict__ part_b, int64_t splits, int64_t M,
    int64_t N, float* __restrict__ C, int64_t ldc, float* __restrict__ Cb, int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t mn = M * N;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  // outputs [0, mn) are C, [mn, mn + M) the column sums (when Cb)
  const int64_t nout = mn + (Cb ? M : 0);
  const float* src = t < mn ? part + t : part_b + (t - mn);
  const int64_t pstride = t < mn ? mn : M;
  float s = 0.f;
  if (t < nout) {
    // this wave's splits w, w+4, w+8, ... summed in order; 16 loads in flight ahead of the
    // adds (4 made a 512-split sum a chain of 32 round trips)
    int64_t p = w;
    for (; p + 60 < splits; p += 64) {
      float x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = src[(p + 4 * u) * pstride];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += x[u];
    }
    for (; p < splits; p += 4) s += src[p * pstride];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && t < nout) {
    const float tot = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    float* c;
    if (t < mn) {
      const int64_t i = t / N, j = t - i * N;
      c = C + i * ldc + j;
    } else {
      c = Cb + (t - mn);
    }
    *c = accumulate ? *c + tot : tot;
  }
}

// blocks the split-K grid aims for: kTargetBlocks (1024 / 2048: slower at 200k rows, equal
// at 1M, profiles/r03e_tn_blocks_ab.txt)

inline int64_t tn_splits(int64_t K, int64_t M, int64_t N) {
  const int64_t tiles = ((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  int64_t s = (int64_t)kTargetBlocks / (tiles > 0 ? tiles : 1);
  // >= 256 rows per split (128 on the 64 x 64 tile: a short gradient — a 1k-row block
  // layer — then spreads over 8 blocks instead of 4 serial 16-step chains)
  const int64_t min_rows = M <= 64 && N <= 64 ? 128 : 256;
  const int64_t by_rows = (K + min_rows - 1) / min_rows;
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

// z = a / |a| (a = relu(u)) kept with the row norms: gu = [z > 0] (gz - z (z.gz)) / |a|,
// or gz masked when |a| == 0 — the same Jacobian as act_backward_kernel without u
__global__ __launch_bounds__(256) void act_backward_normed_kernel(
    const float* __restrict__ z, int64_t ldz, const float* __restrict__ nrm,
    const float* __restrict__ gz, int64_t ldg, int64_t n_rows, int64_t d, int relu,
    float* __restrict__ gu, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const float* zr = z + r * ldz;
  const float* gr = gz + r * ldg;
  float* orow = gu + r * ldo;
  float dot = 0.f;
  for (int64_t c = lane; c < d; c += 64) dot += zr[c] * gr[c];
  for (int off = 32; off > 0; off >>= 1) dot += __shfl_xor(dot, off);
  const float n = nrm[r];
  const bool scale = n != 0.f;
  const float inv = scale ? 1.f / n : 1.f;
  const float coef = scale ? dot : 0.f;
  for (int64_t c = lane; c < d; c += 64) {
    const float x = zr[c];
    float g = (gr[c] - x * coef) * inv;
    if (relu && !(x > 0.f)) g = 0.f;
    orow[c] = g;
  }
}

// The same for d <= 64 (d % 4 == 0, 16-B aligned rows): 16 lanes per row with one float4
// each, four rows per wave, so a wave keeps 4 rows (2 KB) of z and gz in flight instead of
// one — the one-row-per-wave form read a 1M-row layer at 2.8 TB/s (C2 at K = 2500).  The
// dot is summed per lane over its 4 columns, then over the 16 lanes by an xor tree.
__global__ __launch_bounds__(256) void act_backward_normed_v4_kernel(
    const float* __restrict__ z, int64_t ldz, const float* __restrict__ nrm,
    const float* __restrict__ gz, int64_t ldg, int64_t n_rows, int64_t d, int relu,
    float* __restrict__ gu, int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
  const int64_t c = (int64_t)(lane & 15) * 4;
  const bool ok = r < n_rows && c < d;
  float4 zz = make_float4(0.f, 0.f, 0.f, 0.f), gg = zz;
  if (ok) {
    zz = *reinterpret_cast<const float4*>(z + r * ldz + c);
    gg = *reinterpret_cast<const float4*>(gz + r * ldg + c);
  }
  float dot = zz.x * gg.x + zz.y * gg.y + zz.z * gg.z + zz.w * gg.w;
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) dot += __shfl_xor(dot, off);
  if (!ok) return;
  const float n = nrm[r];
  const bool scale = n != 0.f;
  const float inv = scale ? 1.f / n : 1.f;
  const float coef = scale ? dot : 0.f;
  float4 o;
  o.x = (gg.x - zz.x * coef) * inv;
  o.y = (gg.y - zz.y * coef) * inv;
  o.z = (gg.z - zz.z * coef) * inv;
  o.w = (gg.w - zz.w * coef) * inv;
  if (relu) {
    if (!(zz.x > 0.f)) o.x = 0.f;
    if (!(zz.y > 0.f)) o.y = 0.f;
    if (!(zz.z > 0.f)) o.z = 0.f;
    if (!(zz.w > 0.f)) o.w = 0.f;
  }
  *reinterpret_cast<float4*>(gu + r * ldo + c) = o;
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int64_t gnnrec_gemm_tn_workspace_bytes(int64_t K, int64_t M, int64_t N) {
  if (K <= 0 || M <= 0 || N <= 0) return 0;
  return tn_splits(K, M, N) * (M * N + M) * (int64_t)sizeof(float);
}

extern "C" int gnnrec_gemm_tn_bias_rows_f32(const float* A, int64_t lda, const float* B,
                                            int64_t ldb, int64_t K, int64_t M, int64_t N,
                                            float* C, int64_t ldc, float* colsum,
                                            const int64_t* row_ptr, int accumulate,
                                            float* workspace, void* stream) {
  GNNREC_REQUIRE(K >= 0 && M >= 0 && N >= 0, "gnnrec_gemm_tn_f32: negative size");
  GNNREC_REQUIRE(lda >= M && ldb >= N && ldc >= N, "gnnrec_gemm_tn_f32: bad leading dims");
  if (M == 0 || N == 0) return GNNREC_OK;
  hipStream_t s = as_stream(stream);
  if (K == 0) {
    if (accumulate) return GNNREC_OK;
    if (hipMemset2DAsync(C, ldc * sizeof(float), 0, N * sizeof(float), M, s) != hipSuccess ||
        (colsum && hipMemsetAsync(colsum, 0, M * sizeof(float), s) != hipSuccess)) {
      set_error("gnnrec_gemm_tn_f32: hipMemset2DAsync failed");
      return GNNREC_EHIP;
    }
    return GNNREC_OK;
  }
  GNNREC_REQUIRE(A && B && C && workspace, "gnnrec_gemm_tn_f32: null pointer");
  const int64_t splits = tn_splits(K, M, N), chunk = tn_chunk(K, splits);
  const dim3 grid((unsigned)splits, (unsigned)((M + kTile - 1) / kTile),
                  (unsigned)((N + kTile - 1) / kTile));
  const bool vec = aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0 &&
                   M % 4 == 0 && N % 4 == 0;
  float* part_b = colsum ? workspace + splits * M * N : nullptr;
  if (M <= 64 && N <= 64) {  // one 64 x 64 tile, 64-row steps
    if (vec)
      hipLaunchKernelGGL((gemm_tn_partial_kernel<true, 64, 64>), grid, dim3(256), 0, s, A, lda,
                         B, ldb, K, M, N, chunk, workspace, part_b, row_ptr);
    else
      hipLaunchKernelGGL((gemm_tn_partial_kernel<false, 64, 64>), grid, dim3(256), 0, s, A, lda,
                         B, ldb, K, M, N, chunk, workspace, part_b, row_ptr);
  } else if (vec) {
    hipLaunchKernelGGL((gemm_tn_partial_kernel<true, kTile, kKStep>), grid, dim3(256), 0, s, A,
                       lda, B, ldb, K, M, N, chunk, workspace, part_b, row_ptr);
  } else {
    hipLaunchKernelGGL((gemm_tn_partial_kernel<false, kTile, kKStep>), grid, dim3(256), 0, s, A,
                       lda, B, ldb, K, M, N, chunk, workspace, part_b, row_ptr);
  }
  const int64_t nout = M * N + (colsum ? M : 0);
  hipLaunchKernelGGL(gemm_tn_reduce_kernel, dim3((unsigned)((nout + 63) / 64)), dim3(256), 0, s,
                     workspace, part_b, splits, M, N, C, ldc, colsum, accumulate);
  return check_launch("gnnrec_gemm_tn_f32");
}

extern "C" int gnnrec_gemm_tn_bias_f32(const float* A, int64_t lda, const float* B, int64_t ldb,
                                       int64_t K, int64_t M, int64_t N, float* C, int64_t ldc,
                                       float* colsum, int accumulate, float* workspace,
                                       void* stream) {
  return gnnrec_gemm_tn_bias_rows_f32(A, lda, B, ldb, K, M, N, C, ldc, colsum, nullptr,
                                      accumulate, workspace, stream);
}

extern "C" int gnnrec_gemm_tn_f32(const float* A, int64_t lda, const float* B, int64_t ldb,
                                  int64_t K, int64_t M, int64_t N, float* C, int64_t ldc,
                                  int accumulate, float* workspace, void* stream) {
  return gnnrec_gemm_tn_bias_f32(A, lda, B, ldb, K, M, N, C, ldc, nullptr, accumulate, workspace,
                                 stream);
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

// ---- row epilogue for outputs wider than one GEMM block ------------------------------
// gnnrec_gemm_f32 applies the zero-guarded row L2 norm and the attention accumulation
// inside a block that holds the whole output row (N <= 256).  The reference's widest
// layers (hidden 384 / 512, main.py:87) go GEMM -> this kernel: one wave per row, the row
// read once into registers-as-needed, norm, then store / add / max / attention update.
namespace gnnrec {
namespace {

__global__ __launch_bounds__(256) void row_epilogue_kernel(
    const float* __restrict__ z, int64_t ldz, int64_t M, int64_t N, int l2, int accum,
    float out_div, const float* __restrict__ attn_vec, float* __restrict__ attn_state,
    float* __restrict__ out, int64_t ldo) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int lane = threadIdx.x & 63;
  const float* zr = z + row * ldz;
  float* orow = out + row * ldo;
  float ss = 0.f, e = 0.f;
  for (int64_t c = lane; c < N; c += 64) {
    const float x = zr[c];
    ss += x * x;
    if (attn_vec) e += x * attn_vec[c];
  }
  for (int off = 32; off > 0; off >>= 1) {
    ss += __shfl_xor(ss, off);
    e += __shfl_xor(e, off);
  }
  float nrm = 1.f;
  if (l2) {
    nrm = sqrtf(ss);
    if (nrm == 0.f) nrm = 1.f;
    e = e / nrm;
  }
  const bool attn = accum >= GNNREC_ACC_ATTN_FIRST;
  float keep = 0.f, cnew = 1.f, fin = 1.f;
  if (attn) {
    float mnew = e, snew = 1.f;
    if (accum != GNNREC_ACC_ATTN_FIRST) {
      const float2 st = reinterpret_cast<const float2*>(attn_state)[row];
      mnew = fmaxf(st.x, e);
      keep = expf(st.x - mnew);
      cnew = expf(e - mnew);
      snew = st.y * keep + cnew;
    }
    if (accum == GNNREC_ACC_ATTN_LAST) fin = 1.f / snew;
    if (lane == 0) reinterpret_cast<float2*>(attn_state)[row] = make_float2(mnew, snew);
  }
  for (int64_t c = lane; c < N; c += 64) {
    float y = zr[c] / nrm;
    if (attn) {
      y *= cnew;
      if (accum != GNNREC_ACC_ATTN_FIRST) y = orow[c] * keep + y;
      y *= fin;
    } else if (accum == GNNREC_ACC_ADD) {
      y = orow[c] + y;
    } else if (accum == GNNREC_ACC_MAX) {
      y = fmaxf(orow[c], y);
    }
    if (out_div > 0.f) y = y / out_div;
    orow[c] = y;
  }
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_row_epilogue_f32(const float* z, int64_t ldz, int64_t M, int64_t N, int l2norm,
                                       int accum, float out_div, const float* attn_vec,
                                       float* attn_state, float* out, int64_t ldo, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(M >= 0 && N >= 0 && ldz >= N && ldo >= N,
                 "gnnrec_row_epilogue_f32: bad sizes / leading dims");
  GNNREC_REQUIRE(accum >= GNNREC_ACC_STORE && accum <= GNNREC_ACC_ATTN_LAST,
                 "gnnrec_row_epilogue_f32: unknown accumulate mode %d", accum);
  GNNREC_REQUIRE(accum < GNNREC_ACC_ATTN_FIRST || (attn_vec && attn_state),
                 "gnnrec_row_epilogue_f32: attention needs attn_vec and attn_state");
  if (M == 0 || N == 0) return GNNREC_OK;
  hipLaunchKernelGGL(row_epilogue_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0,
                     as_stream(stream), z, ldz, M, N, l2norm, accum, out_div,
                     accum >= GNNREC_ACC_ATTN_FIRST ? attn_vec : nullptr, attn_state, out, ldo);
  return check_launch("gnnrec_row_epilogue_f32");
}

extern "C" int gnnrec_act_backward_normed_f32(const float* z, int64_t ldz, const float* row_norm,
                                              const float* gz, int64_t ldg, int64_t n_rows,
                                              int64_t d, int relu, float* gu, int64_t ldo,
                                              void* stream) {
  GNNREC_REQUIRE(n_rows >= 0 && d >= 0 && ldz >= d && ldg >= d && ldo >= d,
                 "gnnrec_act_backward_normed_f32: bad sizes");
  if (n_rows == 0 || d == 0) return GNNREC_OK;
  GNNREC_REQUIRE(z && row_norm && gz && gu, "gnnrec_act_backward_normed_f32: null pointer");
  if (d <= 64 && d % 4 == 0 && ldz % 4 == 0 && ldg % 4 == 0 && ldo % 4 == 0 && aligned16(z) &&
      aligned16(gz) && aligned16(gu)) {
    hipLaunchKernelGGL(act_backward_normed_v4_kernel, dim3((unsigned)((n_rows + 15) / 16)),
                       dim3(256), 0, as_stream(stream), z, ldz, row_norm, gz, ldg, n_rows, d,
                       relu, gu, ldo);
    return check_launch("gnnrec_act_backward_normed_f32");
  }
  hipLaunchKernelGGL(act_backward_normed_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0,
                     as_stream(stream), z, ldz, row_norm, gz, ldg, n_rows, d, relu, gu, ldo);
  return check_launch("gnnrec_act_backward_normed_f32");
}
