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
// c_in == c_out: the state updated in place (inference); c_in == nullptr: zero state (step 0
// of the training recompute); z_out (nullable): the pre-activation gates [n_act, 4d], which
// the backward (lstm_backward_step_kernel) differentiates
__global__ __launch_bounds__(256) void lstm_step_kernel(
    const float* __restrict__ P, int64_t ldp, const int64_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const int64_t* __restrict__ order, int64_t t,
    int64_t n_act, const float* __restrict__ h_in, float* __restrict__ h_out,
    const float* c_in, float* c_out, float* __restrict__ z_out, int64_t d,
    const float* __restrict__ WT, float* __restrict__ out, int64_t ldo) {
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
    const float cp = c_in ? c_in[p * d + u] : 0.f;
    const float cn = sigm(gf) * cp + sigm(gi) * tanhf(gg);
    const float hn = sigm(go) * tanhf(cn);
    c_out[p * d + u] = cn;
    h_out[p * d + u] = hn;
    if (z_out) {
      float* zr = z_out + p * 4 * d;
      zr[u] = gi;
      zr[d + u] = gf;
      zr[2 * d + u] = gg;
      zr[3 * d + u] = go;
    }
    if (last_step[r]) out[dst_row[r] * ldo + u] = hn;
  }
}

// ---- backward through time: one step, t descending ------------------------------------
// For the n_act rows of step t (row p = order[p]), from the saved pre-activation gates z,
// the cell states c_t and c_{t-1} (0 at t = 0) and the gradients arriving at h_t and c_t —
// from step t+1 for the rows still running there (p < n_next), from the output for the
// rows whose last step is t (p >= n_next: dh = g_out[order[p]], dc = 0):
//   dc  = dc_in + dh·o·(1 − tanh²c_t)
//   dz  = [dc·g·i(1−i), dc·c_{t−1}·f(1−f), dc·i·(1−g²), dh·tanh(c_t)·o(1−o)]
//   dc_{t−1} = dc·f
// dz feeds dh_{t−1} = dz·W_hh (a GEMM), dW_hh, and dP[src] (the input projection).
__global__ __launch_bounds__(256) void lstm_backward_step_kernel(
    const float* __restrict__ z, const float* __restrict__ c_t, const float* __restrict__ c_prev,
    const float* __restrict__ dh_next, const float* __restrict__ dc_next, int64_t n_next,
    const float* __restrict__ g_out, int64_t ldg, const int64_t* __restrict__ order,
    int64_t n_act, int64_t d, float* __restrict__ dz, float* __restrict__ dc_prev) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_act * d) return;
  const int64_t p = i / d, u = i - p * d;
  const float* zr = z + p * 4 * d;
  const float si = sigm(zr[u]), sf = sigm(zr[d + u]), tg = tanhf(zr[2 * d + u]);
  const float so = sigm(zr[3 * d + u]);
  const float ct = c_t[i];
  const float cp = c_prev ? c_prev[i] : 0.f;
  const bool carried = p < n_next;
  const float dh = carried ? dh_next[i] : g_out[order[p] * ldg + u];
  const float tc = tanhf(ct);
  const float dc = (carried ? dc_next[i] : 0.f) + dh * so * (1.f - tc * tc);
  float* dr = dz + p * 4 * d;
  dr[u] = dc * tg * si * (1.f - si);
  dr[d + u] = dc * cp * sf * (1.f - sf);
  dr[2 * d + u] = dc * si * (1.f - tg * tg);
  dr[3 * d + u] = dh * tc * so * (1.f - so);
  dc_prev[i] = dc * sf;
}

// slot s of the step-major packing (step t holds rows [0, n_t) at slots [off[t], off[t+1])):
// its source row indices[indptr[order[p]] + t] and the slot of the same row one step
// earlier (-1 at t = 0) — the scatter of dz into dP and the h_{t-1} rows of dW_hh
__global__ void lstm_slots_kernel(const int64_t* __restrict__ indptr,
                                  const int32_t* __restrict__ indices,
                                  const int64_t* __restrict__ order,
                                  const int64_t* __restrict__ off, int64_t n_steps,
                                  int64_t n_slots, int64_t* __restrict__ src,
                                  int64_t* __restrict__ prev) {
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= n_slots) return;
  int64_t lo = 0, hi = n_steps;  // the step t with off[t] <= s < off[t+1]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (off[mid] <= s) lo = mid;
    else hi = mid;
  }
  const int64_t t = lo, p = s - off[t];
  src[s] = indices[indptr[order[p]] + t];
  prev[s] = t > 0 ? off[t - 1] + p : -1;
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
                     indices, order, t, n_act, h_in, h_out, c, c, nullptr, d, W_hhT, out, ldo);
  return check_launch("gnnrec_lstm_step_f32");
}

extern "C" int gnnrec_lstm_step_save_f32(const float* P, int64_t ldp, const int64_t* indptr,
                                         const int32_t* indices, const int64_t* order, int64_t t,
                                         int64_t n_act, const float* h_in, float* h_out,
                                         const float* c_in, float* c_out, float* z_out,
                                         int64_t d, const float* W_hhT, float* out, int64_t ldo,
                                         void* stream) {
  GNNREC_REQUIRE(d > 0 && d <= kMaxD,
                 "gnnrec_lstm_step_save_f32: hidden size %lld not in [1, %d]", (long long)d,
                 kMaxD);
  GNNREC_REQUIRE(ldp >= 4 * d && ldo >= d, "gnnrec_lstm_step_save_f32: bad leading dims");
  GNNREC_REQUIRE(t >= 0 && n_act >= 0, "gnnrec_lstm_step_save_f32: negative step / row count");
  if (n_act == 0) return GNNREC_OK;
  GNNREC_REQUIRE(P && indptr && indices && order && h_in && h_out && c_out && z_out && W_hhT &&
                     out,
                 "gnnrec_lstm_step_save_f32: null pointer");
  const dim3 grid((unsigned)((n_act + kRows - 1) / kRows), (unsigned)((d + kUnits - 1) / kUnits));
  const size_t lds = (size_t)kRows * (d + 1) * sizeof(float);
  hipLaunchKernelGGL(lstm_step_kernel, grid, dim3(256), lds, as_stream(stream), P, ldp, indptr,
                     indices, order, t, n_act, h_in, h_out, c_in, c_out, z_out, d, W_hhT, out,
                     ldo);
  return check_launch("gnnrec_lstm_step_save_f32");
}

extern "C" int gnnrec_lstm_backward_step_f32(const float* z, const float* c_t,
                                             const float* c_prev, const float* dh_next,
                                             const float* dc_next, int64_t n_next,
                                             const float* g_out, int64_t ldg,
                                             const int64_t* order, int64_t n_act, int64_t d,
                                             float* dz, float* dc_prev, void* stream) {
  GNNREC_REQUIRE(d > 0 && n_act >= 0 && n_next >= 0 && n_next <= n_act && ldg >= d,
                 "gnnrec_lstm_backward_step_f32: bad sizes");
  if (n_act == 0) return GNNREC_OK;
  GNNREC_REQUIRE(z && c_t && g_out && order && dz && dc_prev && (n_next == 0 || (dh_next && dc_next)),
                 "gnnrec_lstm_backward_step_f32: null pointer");
  const int64_t n = n_act * d;
  hipLaunchKernelGGL(lstm_backward_step_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), z, c_t, c_prev, dh_next, dc_next, n_next, g_out, ldg,
                     order, n_act, d, dz, dc_prev);
  return check_launch("gnnrec_lstm_backward_step_f32");
}

extern "C" int gnnrec_lstm_slots(const int64_t* indptr, const int32_t* indices,
                                 const int64_t* order, const int64_t* step_off, int64_t n_steps,
                                 int64_t n_slots, int64_t* src, int64_t* prev, void* stream) {
  GNNREC_REQUIRE(n_steps >= 0 && n_slots >= 0, "gnnrec_lstm_slots: negative size");
  if (n_slots == 0) return GNNREC_OK;
  GNNREC_REQUIRE(n_steps > 0 && indptr && indices && order && step_off && src && prev,
                 "gnnrec_lstm_slots: null pointer");
  hipLaunchKernelGGL(lstm_slots_kernel, dim3((unsigned)((n_slots + 255) / 256)), dim3(256), 0,
                     as_stream(stream), indptr, indices, order, step_off, n_steps, n_slots, src,
                     prev);
  return check_launch("gnnrec_lstm_slots");
}
