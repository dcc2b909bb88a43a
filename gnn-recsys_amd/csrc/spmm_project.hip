// a1+a3 fused — neighbour aggregation with the SAGE projection in its epilogue:
//   out[v] (accum)= epi( h_self[v] · W_selfᵀ + agg(v) · W_neighᵀ ),
//   agg(v) = mean / sum / max over v's in-edges of X[src] (· w_e)
// for ConvLayer.forward's aggregation + projection (reference src/model.py:143-208,
// 226-235) and HeteroGraphConv's cross-relation sum/mean/max (:384-406).
//
// Why: the gather is HBM-bound (≈6.5 TB/s) and leaves the CU's VALU and LDS mostly
// idle, while the separate projection GEMM re-reads h_self and the aggregate from HBM,
// writes the output again and, run beside the next gather, competes with it for HBM.
// Here each wave owns ROWS destination rows at a time end to end: gather (the same
// gather_range / fixed xor-tree combine as spmm_csr_kernel, so the aggregate is
// bit-identical to the plain kernel's), then a 128×128 matvec per row on the VALU with
// both weight matrices resident in LDS (loaded once per persistent block), ReLU,
// zero-guarded row L2 norm, hetero accumulate, one 512-B store.  HBM per row: the
// gathered rows + h_self row + output row; no aggregate round trip, no GEMM launch.
//
// Shapes: d_neigh = d_self = N = 128 (the C4/C5 shapes); the wrapper falls back to
// spmm + gemm otherwise, and when the CSR has rows above the heavy-row split.
// LDS: W_selfᵀ, W_neighᵀ (2 × 64 KiB, k-major so a lane's two output columns are one
// ds_read_b64) + per wave ROWS × (agg, self) row slots read back as broadcasts.
#include "common.hpp"
#include "gather.hpp"
#include "rowq.hpp"
#include <cstdlib>

namespace gnnrec {
namespace {

constexpr int kPD = 128;       // d_neigh = d_self = N
constexpr int kPWaves = 16;    // waves per block (one persistent block per CU)
constexpr int kPRows = 2;      // rows per wave per iteration (halves the LDS weight reads)
// rows per queue ticket (rowq.hpp): four iterations, ≈120 µs at C4; GNNREC_RQ_CHUNK_FUSED
// overrides (tuning; rounded up to a multiple of kPRows)
inline int fused_chunk() {
  static const int v = [] {
    const char* e = getenv("GNNREC_RQ_CHUNK_FUSED");
    const int x = e ? atoi(e) : 0;
    return x > 0 && x <= 64 ? (x + kPRows - 1) / kPRows * kPRows : 8;
  }();
  return v;
}

template <int REDUCE, bool WEIGHTED, int UNROLL>
__global__ __launch_bounds__(kPWaves * 64) void spmm_project_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ ew, const float* __restrict__ X, int64_t ldx,
    const float* __restrict__ H, int64_t ldh, const float* __restrict__ WsT,
    const float* __restrict__ WnT, const float* __restrict__ bias,
    const float* __restrict__ bias_ne, int64_t n_dst, int epilogue, int accum, float out_div,
    const float* __restrict__ attn_vec, float* __restrict__ attn_state,
    float* __restrict__ out, int64_t ldo, unsigned* rq, int rq_ch) {
  __shared__ float Ws[kPD * kPD];
  __shared__ float Wn[kPD * kPD];
  __shared__ float slots[kPWaves][kPRows][2][kPD];
  for (int i = threadIdx.x; i < kPD * kPD / 4; i += kPWaves * 64) {
    reinterpret_cast<float4*>(Ws)[i] = reinterpret_cast<const float4*>(WsT)[i];
    reinterpret_cast<float4*>(Wn)[i] = reinterpret_cast<const float4*>(WnT)[i];
  }
  __syncthreads();

  constexpr int LPR = 32, VEC = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPR;
  const int col = (lane % LPR) * VEC;
  const int j0 = 2 * lane;  // this lane's two output columns
  const bool relu = epilogue & GNNREC_EPI_RELU;
  const bool l2 = epilogue & GNNREC_EPI_L2NORM;
  const float init = (REDUCE == GNNREC_REDUCE_MAX) ? -INFINITY : 0.f;
  const int64_t stride = (int64_t)gridDim.x * kPWaves * kPRows;
  const float b0 = bias ? bias[j0] : 0.f, b1 = bias ? bias[j0 + 1] : 0.f;
  const float c0 = bias_ne ? bias_ne[j0] : 0.f, c1 = bias_ne ? bias_ne[j0 + 1] : 0.f;
  const bool attn = accum >= GNNREC_ACC_ATTN_FIRST;
  const float a0 = attn ? attn_vec[j0] : 0.f, a1 = attn ? attn_vec[j0 + 1] : 0.f;

  // rows [row0, row0 + kPRows) of this wave, those at or past `lim` skipped
  auto step = [&](int64_t row0, int64_t lim) {
    bool nonempty[kPRows];
    // both rows' bounds (one load), first 64 indices and self rows are requested before
    // either row gathers: the second row's indptr -> indices chain hides under the first
    // row's gather (it is the fixed per-row cost that low-degree relations feel)
    const int nv = (int)(lim - row0 < kPRows ? lim - row0 : kPRows);  // valid rows, >= 1
    const int64_t ipl = lane <= nv ? indptr[row0 + lane] : 0;
    int64_t rb[kPRows + 1];
#pragma unroll
    for (int r = 0; r <= kPRows; ++r) rb[r] = __shfl(ipl, r <= nv ? r : nv);
    int pidx[kPRows];
    float4 hsr[kPRows];
#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      const bool valid = r < nv;  // uniform per wave
      pidx[r] = valid && lane < rb[r + 1] - rb[r] ? indices[rb[r] + lane] : 0;
      hsr[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid && grp == 1) hsr[r] = *reinterpret_cast<const float4*>(H + (row0 + r) * ldh + col);
    }
#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      const bool valid = r < nv;  // uniform per wave
      const float4 hs = hsr[r];
      Frag<VEC> acc;
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc.v[v] = init;
      int64_t deg = 0;
      if (valid) {
        const int64_t beg = rb[r], end = rb[r + 1];
        deg = end - beg;
        gather_range<LPR, VEC, REDUCE, WEIGHTED, UNROLL, true>(beg, end, indices, ew, X, ldx,
                                                               col, true, lane, grp, acc, pidx[r]);
      }
      combine_groups<LPR, VEC, REDUCE>(acc);
      finalize<VEC, REDUCE>(acc, deg, 0);
      nonempty[r] = deg > 0;
      if (grp == 0)
        *reinterpret_cast<float4*>(&slots[wave][r][0][col]) =
            make_float4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
      else
        *reinterpret_cast<float4*>(&slots[wave][r][1][col]) = hs;
    }
    // the slots are written and read by this wave only: LDS is in order per wave, the
    // clobber keeps the compiler from hoisting the reads above the writes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    // bias: a folded NodeEmbedding's W_self·b; bias_ne: its W_neigh·b, which only
    // rows with at least one neighbour receive (the mean of an empty set is 0)
    float z[kPRows][2];
#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      z[r][0] = b0 + (nonempty[r] ? c0 : 0.f);
      z[r][1] = b1 + (nonempty[r] ? c1 : 0.f);
    }
#pragma unroll 2
    for (int k = 0; k < kPD; k += 4) {
      float4 a4[kPRows], s4[kPRows];
#pragma unroll
      for (int r = 0; r < kPRows; ++r) {
        a4[r] = *reinterpret_cast<const float4*>(&slots[wave][r][0][k]);
        s4[r] = *reinterpret_cast<const float4*>(&slots[wave][r][1][k]);
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const float2 ws = *reinterpret_cast<const float2*>(&Ws[(k + kk) * kPD + j0]);
        const float2 wn = *reinterpret_cast<const float2*>(&Wn[(k + kk) * kPD + j0]);
#pragma unroll
        for (int r = 0; r < kPRows; ++r) {
          const float s = kk == 0 ? s4[r].x : kk == 1 ? s4[r].y : kk == 2 ? s4[r].z : s4[r].w;
          const float a = kk == 0 ? a4[r].x : kk == 1 ? a4[r].y : kk == 2 ? a4[r].z : a4[r].w;
          z[r][0] = fmaf(s, ws.x, z[r][0]);
          z[r][0] = fmaf(a, wn.x, z[r][0]);
          z[r][1] = fmaf(s, ws.y, z[r][1]);
          z[r][1] = fmaf(a, wn.y, z[r][1]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slots free for the next rows

#pragma unroll
    for (int r = 0; r < kPRows; ++r) {
      const int64_t row = row0 + r;
      float y0 = z[r][0], y1 = z[r][1];
      if (relu) {
        y0 = fmaxf(y0, 0.f);
        y1 = fmaxf(y1, 0.f);
      }
      if (l2) {
        float ss = y0 * y0 + y1 * y1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) ss += __shfl_xor(ss, off);
        float nrm = sqrtf(ss);
        if (nrm == 0.f) nrm = 1.f;
        y0 = y0 / nrm;
        y1 = y1 / nrm;
      }
      float keep = 0.f, nrm_attn = 1.f;
      if (attn) {  // online softmax over relations, score e = a . y (row-uniform)
        float e = y0 * a0 + y1 * a1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) e += __shfl_xor(e, off);
        float mnew = e, snew = 1.f, cnew = 1.f;
        if (row < lim && accum != GNNREC_ACC_ATTN_FIRST) {
          const float2 st = reinterpret_cast<const float2*>(attn_state)[row];
          mnew = fmaxf(st.x, e);
          keep = expf(st.x - mnew);
          cnew = expf(e - mnew);
          snew = st.y * keep + cnew;
        }
        if (accum == GNNREC_ACC_ATTN_LAST) nrm_attn = 1.f / snew;
        if (row < lim && lane == 0)
          reinterpret_cast<float2*>(attn_state)[row] = make_float2(mnew, snew);
        y0 *= cnew;
        y1 *= cnew;
      }
      if (row >= lim) continue;
      float2* p = reinterpret_cast<float2*>(out + row * ldo + j0);
      if (attn) {
        if (accum != GNNREC_ACC_ATTN_FIRST) {
          const float2 o = *p;
          y0 = o.x * keep + y0;
          y1 = o.y * keep + y1;
        }
        y0 *= nrm_attn;
        y1 *= nrm_attn;
      } else if (accum != GNNREC_ACC_STORE) {
        const float2 o = *p;
        if (accum == GNNREC_ACC_ADD) {
          y0 = o.x + y0;
          y1 = o.y + y1;
        } else {
          y0 = fmaxf(o.x, y0);
          y1 = fmaxf(o.y, y1);
        }
      }
      if (out_div > 0.f) {
        y0 = y0 / out_div;
        y1 = y1 / out_div;
      }
      *p = make_float2(y0, y1);
    }
  };

  if (rq != nullptr) {  // rows from the queue: blocks that start late take fewer
    rq_for_each(rq, n_dst, rq_ch, [&](int64_t r0, int64_t r1) {
      for (int64_t row0 = r0; row0 < r1; row0 += kPRows) step(row0, r1);
    });
    rq_finish(rq);
    return;
  }
  for (int64_t row0 = ((int64_t)blockIdx.x * kPWaves + wave) * kPRows; row0 < n_dst;
       row0 += stride)
    step(row0, n_dst);
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_spmm_project_f32(const int64_t* indptr, const int32_t* indices,
                                       const float* ew, const float* X, int64_t ldx,
                                       const float* H, int64_t ldh, const float* W_selfT,
                                       const float* W_neighT, const float* bias,
                                       const float* bias_nonempty, int64_t n_dst, int64_t d,
                                       int reduce, int epilogue, int accum, float out_div,
                                       const float* attn_vec, float* attn_state, float* out,
                                       int64_t ldo, void* stream) {
  GNNREC_REQUIRE(d == kPD, "gnnrec_spmm_project_f32: only d = %d (got %lld)", kPD,
                 (long long)d);
  GNNREC_REQUIRE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN ||
                     reduce == GNNREC_REDUCE_MAX,
                 "gnnrec_spmm_project_f32: unknown reduce %d", reduce);
  GNNREC_REQUIRE((epilogue & ~(GNNREC_EPI_RELU | GNNREC_EPI_L2NORM)) == 0,
                 "gnnrec_spmm_project_f32: epilogue must be RELU|L2NORM");
  GNNREC_REQUIRE(accum >= GNNREC_ACC_STORE && accum <= GNNREC_ACC_ATTN_LAST,
                 "gnnrec_spmm_project_f32: unknown accumulate mode %d", accum);
  GNNREC_REQUIRE(accum < GNNREC_ACC_ATTN_FIRST || (attn_vec && attn_state),
                 "gnnrec_spmm_project_f32: attention accumulation needs attn_vec, attn_state");
  GNNREC_REQUIRE(n_dst >= 0, "gnnrec_spmm_project_f32: negative n_dst");
  if (n_dst == 0) return GNNREC_OK;
  GNNREC_REQUIRE(indptr && X && H && W_selfT && W_neighT && out,
                 "gnnrec_spmm_project_f32: null pointer");
  GNNREC_REQUIRE(aligned16(X) && aligned16(H) && aligned16(W_selfT) && aligned16(W_neighT) &&
                     ldx % 4 == 0 && ldh % 4 == 0 && ldo % 2 == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 7u) == 0,
                 "gnnrec_spmm_project_f32: X/H/W need 16-B aligned rows, out 8-B");
  // one persistent block per CU, minus the CUs reserved for concurrent kernels
  const int64_t per_block = (int64_t)kPWaves * kPRows;
  int64_t blocks = (n_dst + per_block - 1) / per_block;
  const int64_t cus = device_cus() - cu_reserve();
  if (blocks > (cus > 8 ? cus : 8)) blocks = cus > 8 ? cus : 8;
  // queued rows when every wave has several tickets of work
  const int rq_ch = fused_chunk();
  hipStream_t s = as_stream(stream);
  int ticket = -1;
  unsigned* rq = n_dst >= blocks * kPWaves * rq_ch * 4 ? rowq_slot(s, &ticket) : nullptr;
  const dim3 grid((unsigned)blocks), block(kPWaves * 64);
  static const int unroll = [] {  // gather wave-instructions in flight per lane (tuning knob)
    const char* e = getenv("GNNREC_SPP_UNROLL");
    return e ? atoi(e) : 4;
  }();
#define GNNREC_SPP_ONE(R, W, U)                                                              \
  hipLaunchKernelGGL((spmm_project_kernel<R, W, U>), grid, block, 0, s, indptr, indices, ew, X, \
                     ldx, H, ldh, W_selfT, W_neighT, bias, bias_nonempty, n_dst, epilogue, accum, \
                     out_div, attn_vec, attn_state, out, ldo, rq, rq_ch)
#define GNNREC_SPP(R, W)                                  \
  do {                                                    \
    if (unroll == 8) GNNREC_SPP_ONE(R, W, 8);             \
    else if (unroll == 2) GNNREC_SPP_ONE(R, W, 2);        \
    else GNNREC_SPP_ONE(R, W, 4);                         \
  } while (0)
  if (ew) {
    if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPP(GNNREC_REDUCE_SUM, true);
    else if (reduce == GNNREC_REDUCE_MEAN) GNNREC_SPP(GNNREC_REDUCE_MEAN, true);
    else GNNREC_SPP(GNNREC_REDUCE_MAX, true);
  } else {
    if (reduce == GNNREC_REDUCE_SUM) GNNREC_SPP(GNNREC_REDUCE_SUM, false);
    else if (reduce == GNNREC_REDUCE_MEAN) GNNREC_SPP(GNNREC_REDUCE_MEAN, false);
    else GNNREC_SPP(GNNREC_REDUCE_MAX, false);
  }
#undef GNNREC_SPP
#undef GNNREC_SPP_ONE
  rowq_launched(ticket, s);
  return check_launch("gnnrec_spmm_project_f32");
}
