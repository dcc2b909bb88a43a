// f4 — LSTM neighbourhood reducer (reference ConvLayer._lstm_reducer,
// src/model.py:106-121, driven by update_all at :164-169 under DGL 0.5.2
// degree bucketing): per destination, torch nn.LSTM (1 layer, h0 = c0 = 0,
// gates i, f, g, o) over its in-neighbour messages in edge order; output =
// final hidden state, 0 for zero in-degree.
//
// Schedule: destinations sorted by in-degree, descending (`order`), so the rows
// still running at step t are the prefix [0, n_t).  The input projection of
// every source row, P = X W_ihᵀ + b_ih + b_hh, is one gnnrec_gemm_f32 launch;
// one launch of this kernel per step t does, for the n_t running rows,
//   gates = P[src(row, t)] + h W_hhᵀ   (fp32 MFMA, h tile staged in LDS)
//   c = σ(f)·c + σ(i)·tanh(g);  h' = σ(o)·tanh(c)
// and writes h' straight to out[dst] at the row's last step.
#include "common.hpp"

namespace gnnrec {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kRows = 32;    // destinations per block
constexpr int kUnits = 128;  // hidden units per block (4 waves x 32)
constexpr int kMaxD = 512;

__device__ inline float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// MFMA 32x32x2 f32: lane l supplies A[i=l&31][k=l>>5] (h row i, unit k) and
// B[k=l>>5][j=l&31] = W_hhᵀ[k][gate*d + unit j]; C/D lane l, v: column j = l&31,
// row i = (v&3) + 8(v>>2) + 4(l>>5).
__global__ __launch_bounds__(256) void lstm_step_kernel(
    const float* __restrict__ P, int64_t ldp, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ order, int64_t t,
    int64_t n_act, const float* __restrict__ h_in, float* __restrict__ h_out,
    float* __restrict__ c, int64_t d, const float* __restrict__ WT, float* __restrict__ out,
    int64_t ldo) {
  extern __shared__ float hs[];  // [kRows][d + 1]
  __shared__ int64_t src_row[kRows], dst_row[kRows];
  __shared__ int last_step[kRows];
  const int tid = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kRows;
  const int64_t hd = d + 1;
  if (tid < kRows) {
    const int64_t p = p0 + tid;
    int64_t s = 0, v = 0;
    int last = 0;
    if (p < n_act) {
      v = order[p];
      const int64_t beg = indptr[v];
      s = indices[beg + t];
      last = (t == indptr[v + 1] - beg - 1);
    }
    src_row[tid] = s;
    dst_row[tid] = v;
    last_step[tid] = last;
  }
  for (int64_t idx = tid; idx < kRows * d; idx += 256) {
    const int64_t r = idx / d, k = idx - r * d;
    hs[r * hd + k] = (p0 + r < n_act) ? h_in[(p0 + r) * d + k] : 0.f;
  }
  __syncthreads();

  const int lane = tid & 63, w = tid >> 6;
  const int li = lane & 31, lk = lane >> 5;
  const int64_t u = (int64_t)blockIdx.y * kUnits + 32 * w + li;  // this lane's unit
  if ((int64_t)blockIdx.y * kUnits + 32 * w >= d) return;          // whole wave idle
  const bool u_ok = u < d;
  const int64_t uc = u_ok ? u : 0;

  f32x16 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[q][v] = 0.f;
  const int64_t ldw = 4 * d;
  for (int64_t k0 = 0; k0 < d; k0 += 2) {
    const int64_t k = k0 + lk;
    const bool k_ok = k < d;
    const int64_t kc = k_ok ? k : 0;
    const float av = hs[li * hd + kc];
    const float a = k_ok ? av : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float bv = WT[kc * ldw + q * d + uc];
      const float b = (k_ok && u_ok) ? bv : 0.f;
      acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[q], 0, 0, 0);
    }
  }
  if (!u_ok) return;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int r = (v & 3) + 8 * (v >> 2) + 4 * lk;
    const int64_t p = p0 + r;
    if (p >= n_act) continue;
    const float* pr = P + src_row[r] * ldp;
    const float gi = acc[0][v] + pr[u];
    const float gf = acc[1][v] + pr[d + u];
    const float gg = acc[2][v] + pr[2 * d + u];
    const float go = acc[3][v] + pr[3 * d + u];
    const float cn = sigm(gf) * c[p * d + u] + sigm(gi) * tanhf(gg);
    const float hn = sigm(go) * tanhf(cn);
    c[p * d + u] = cn;
    h_out[p * d + u] = hn;
    if (last_step[r]) out[dst_row[r] * ldo + u] = hn;
  }
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_lstm_step_f32(const float* P, int64_t ldp, const int64_t* indptr,
                                    const int32_t* indices, const int64_t* order, int64_t t,
                                    int64_t n_act, const float* h_in, float* h_out, float* c,
                                    int64_t d, const float* W_hhT, float* out, int64_t ldo,
                                    void* stream) {
  GNNREC_REQUIRE(d > 0 && d <= kMaxD, "gnnrec_lstm_step_f32: hidden size %lld not in [1, %d]",
                 (long long)d, kMaxD);
  GNNREC_REQUIRE(ldp >= 4 * d && ldo >= d, "gnnrec_lstm_step_f32: bad leading dims");
  GNNREC_REQUIRE(t >= 0 && n_act >= 0, "gnnrec_lstm_step_f32: negative step / row count");
  if (n_act == 0) return GNNREC_OK;
  const dim3 grid((unsigned)((n_act + kRows - 1) / kRows), (unsigned)((d + kUnits - 1) / kUnits));
  const size_t lds = (size_t)kRows * (d + 1) * sizeof(float);
  hipLaunchKernelGGL(lstm_step_kernel, grid, dim3(256), lds, as_stream(stream), P, ldp, indptr,
                     indices, order, t, n_act, h_in, h_out, c, d, W_hhT, out, ldo);
  return check_launch("gnnrec_lstm_step_f32");
}
