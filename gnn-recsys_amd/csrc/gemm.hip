// a2/a3/a4 — fp32 MFMA GEMM with the SAGE epilogue fused in.
//
// Replaces (reference src/model.py):
//   fc_self(h_self) + fc_neigh(h_neigh), relu, zero-guarded row L2 norm   :98-99,226-235
//   relu(fc_preagg(h_neigh))                                              :102,151,158,185,198
//   NodeEmbedding (Linear + bias)                                         :19-24
//   PredictingLayer hidden_1 (bias)                                       :258
//   HeteroGraphConv(aggregate='sum'|'mean'|'max') across relations [DGL]  :384-406
//
// One launch computes, for a block of BM=128 rows and the full (padded) output
// width BN, acc = A1·W1ᵀ + T(A2)·W2ᵀ with v_mfma_f32_32x32x2_f32 (exact fp32,
// one rounding per product — no reduced-precision path exists for f32 on
// gfx950), then bias, activation, the row L2 norm (the whole row is in the
// block, reduced across the 32 lanes that hold it) and the cross-relation
// accumulate into `out`.
//
// Tiling: 4 waves, each owning 32 rows × BN columns (BN/32 accumulators of
// 16 regs).  K is staged through LDS 32 deep; the A and W tiles are stored
// [row][k] with a 36-float row stride so the per-lane ds_read_b128 of 4
// consecutive k is bank-conflict free (r·36 mod 64 covers 16 distinct 4-bank
// slots).  Lane half h of the MFMA consumes k ∈ [16h, 16h+16) of the tile — a
// permutation of the summation order inside the tile that keeps both operand
// reads vectorised (fp32 sums stay within the 1e-4 parity tolerance).
#include "common.hpp"
#include <cmath>
#include <cstdlib>

namespace gnnrec {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int LDSK = 36;  // padded k stride (floats)
constexpr int GEMM_WAVES_PER_SIMD = 2;

struct GemmArgs {
  const float* A1; int64_t lda1; int64_t K1; const float* W1;
  const float* A2; int64_t lda2; int64_t K2; const float* W2;
  const int32_t* a2_deg; int a2_mode;
  const int64_t* a2_ip;  // GNNREC_A2_DEG_INDPTR: the degrees as indptr differences instead
  const float* bias;
  const float* bias_ne;  // added on rows with a2_deg > 0 (a folded NodeEmbedding's W_n b_e)
  int64_t M; int64_t N;
  int epilogue; int accum; float out_div;
  const float* attn_vec; float* attn_state;
  float* out; int64_t ldo;
  float* row_norm;  // nullable: |row| before the L2 norm (training keeps it for the backward)
  int vecA1, vecA2, vecW1, vecW2, vecO;
};

__device__ __forceinline__ int32_t a2_degree(const GemmArgs& g, int64_t row) {
  return g.a2_ip ? (int32_t)(g.a2_ip[row + 1] - g.a2_ip[row]) : g.a2_deg[row];
}

__device__ __forceinline__ f32x4 load4(const float* base, int64_t row, int64_t ld, int64_t k,
                                        int64_t K, bool rowok, bool vec) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (!rowok || k >= K) return v;
  const float* p = base + row * ld + k;
  if (vec) {
    v = *reinterpret_cast<const f32x4*>(p);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k + j < K) v[j] = p[j];
  }
  return v;
}

// the epilogue stages the output tile in LDS in column halves, so the block's LDS
// is just the K-loop tiles (36.9 KB at BN=128) and LDS never limits occupancy
template <int BN>
constexpr int stage_cols() { return BN >= 64 ? BN / 2 : BN; }

template <int BN>
constexpr int smem_floats() {
  // K-loop tiles, or the epilogue's output staging + 2 attention factors per row
  return (BM + BN) * LDSK > BM * (stage_cols<BN>() + 4) + 2 * BM
             ? (BM + BN) * LDSK
             : BM * (stage_cols<BN>() + 4) + 2 * BM;
}

// Shared epilogue: bias, activation, zero-guarded row L2 norm, then the cross-relation
// accumulate into `out`, staged through LDS (column halves) into whole-row 16-B stores.
template <int BN>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, f32x16 (&acc)[BN / 32],
                                              float* smem, int64_t m0, int64_t n0, int wave,
                                              int lane) {
  constexpr int NT = BN / 32;
  const int r = lane & 31;
  const int h = lane >> 5;
  // ---- epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (v&3) + 8(v>>2) + 4h
  const bool relu = g.epilogue & GNNREC_EPI_RELU;
  const bool sigm = g.epilogue & GNNREC_EPI_SIGMOID;
  const bool l2 = g.epilogue & GNNREC_EPI_L2NORM;
  float bias_t[NT], bne_t[NT];
  bool colok[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int64_t col = n0 + t * 32 + r;
    colok[t] = col < g.N;
    bias_t[t] = (g.bias && colok[t]) ? g.bias[col] : 0.f;
    bne_t[t] = (g.bias_ne && colok[t]) ? g.bias_ne[col] : 0.f;
  }
  // staged store: the wave's 32 x BN tile goes through LDS (in column halves) and leaves
  // as whole rows of 16-B stores (4x fewer, fully coalesced store instructions)
  constexpr int SC = stage_cols<BN>();
  constexpr int OSTR = SC + 4;
  constexpr int TPR = SC / 32;  // accumulator tiles per staging round
  const bool attn = g.accum >= GNNREC_ACC_ATTN_FIRST;
  const bool staged = g.vecO;
  float* Ot = smem + wave * 32 * OSTR;
  float* Fa = smem + BM * OSTR + wave * 64;  // attention: (keep, norm) per staged row
  float z[16][NT];
  float a_t[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) a_t[t] = (attn && colok[t]) ? g.attn_vec[n0 + t * 32 + r] : 0.f;
  float keep[16], norm[16];  // attention: weight of the running out, 1 / running sum
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    float ss = 0.f;
    bool ne = false;
    if (g.bias_ne) {
      const int64_t row = m0 + wave * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      ne = row < g.M && a2_degree(g, row) > 0;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float x = acc[t][v] + bias_t[t];
      if (ne) x += bne_t[t];
      if (relu) x = fmaxf(x, 0.f);
      if (sigm) x = 1.f / (1.f + expf(-x));
      if (!colok[t]) x = 0.f;
      z[v][t] = x;
      ss += x * x;
    }
    if (l2) {
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) ss += __shfl_xor(ss, off);
      float nrm = sqrtf(ss);
      if (g.row_norm && r == 0) {
        const int64_t row = m0 + wave * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row < g.M) g.row_norm[row] = nrm;
      }
      if (nrm == 0.f) nrm = 1.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) z[v][t] = z[v][t] / nrm;
    }
    keep[v] = 0.f;
    norm[v] = 1.f;
    if (attn) {  // online softmax over relations: score e = a . z(row)
      float e = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) e += z[v][t] * a_t[t];
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) e += __shfl_xor(e, off);
      const int64_t row = m0 + wave * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      float mnew = e, snew = 1.f, cnew = 1.f;
      if (row < g.M && g.accum != GNNREC_ACC_ATTN_FIRST) {
        const float2 st = reinterpret_cast<const float2*>(g.attn_state)[row];
        mnew = fmaxf(st.x, e);
        keep[v] = expf(st.x - mnew);
        cnew = expf(e - mnew);
        snew = st.y * keep[v] + cnew;
      }
      if (g.accum == GNNREC_ACC_ATTN_LAST) norm[v] = 1.f / snew;
      if (row < g.M && r == 0)
        reinterpret_cast<float2*>(g.attn_state)[row] = make_float2(mnew, snew);

#pragma unroll
      for (int t = 0; t < NT; ++t) z[v][t] *= cnew;
    }
  }
  if (!staged) {
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int64_t row = m0 + wave * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (row >= g.M) continue;
      float* orow = g.out + row * g.ldo + n0;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (!colok[t]) continue;
        float* p = orow + t * 32 + r;
        float y = z[v][t];
        if (g.accum == GNNREC_ACC_ADD) y = *p + y;
        else if (g.accum == GNNREC_ACC_MAX) y = fmaxf(*p, y);
        else if (attn) {
          if (g.accum != GNNREC_ACC_ATTN_FIRST) y = *p * keep[v] + y;
          y = y * norm[v];
        }
        if (g.out_div > 0.f) y = y / g.out_div;
        *p = y;
      }
    }
    return;
  }
#pragma unroll
  for (int round = 0; round < NT / TPR; ++round) {
    __syncthreads();  // K-loop tiles (or the previous round) fully read
    if (attn && round == 0 && r == 0) {  // per-row factors for the store loop (Fa may
#pragma unroll                              // overlap the K-loop tiles: written after the barrier)
      for (int v = 0; v < 16; ++v) {
        const int rl = (v & 3) + 8 * (v >> 2) + 4 * h;
        Fa[2 * rl] = keep[v];
        Fa[2 * rl + 1] = norm[v];
      }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int rl = (v & 3) + 8 * (v >> 2) + 4 * h;
#pragma unroll
      for (int tt = 0; tt < TPR; ++tt) Ot[rl * OSTR + tt * 32 + r] = z[v][round * TPR + tt];
    }
    __syncthreads();
    constexpr int C4 = SC / 4;               // float4 per staged row
    constexpr int ITER = 32 * C4 / kWave;    // float4 per lane
#pragma unroll 4
    for (int q = 0; q < ITER; ++q) {
      const int flat = q * kWave + lane;
      const int rl = flat / C4;
      const int c = (flat % C4) * 4;
      const int64_t row = m0 + wave * 32 + rl;
      const int64_t col = n0 + round * SC + c;
      if (row >= g.M || col >= g.N) continue;
      f32x4 y = *reinterpret_cast<const f32x4*>(Ot + rl * OSTR + c);
      f32x4* p = reinterpret_cast<f32x4*>(g.out + row * g.ldo + col);
      if (g.accum == GNNREC_ACC_ADD) {
        y = *p + y;
      } else if (g.accum == GNNREC_ACC_MAX) {
        const f32x4 o = *p;
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = fmaxf(o[j], y[j]);
      } else if (attn) {
        if (g.accum != GNNREC_ACC_ATTN_FIRST) y = *p * Fa[2 * rl] + y;
        y = y * Fa[2 * rl + 1];
      }
      if (g.out_div > 0.f) y = y / g.out_div;
      *p = y;
    }
  }
}

// The common epilogues with their flags known at compile time — FE = bias | relu << 1 |
// l2norm << 2 (the SAGE projection: ReLU + row norm; fc_preagg: ReLU; NodeEmbedding: bias),
// store-only, full 128-column tiles, 16-B aligned output — instead of runtime flags in the
// unrolled value loops (selects per value: the 1M x 256 x 128 GEMM issued 4.8 non-MFMA VALU
// instructions per MFMA, profiles/r03_gemm_pmc.md).  The row norm divides once per row and
// scales by the reciprocal.
template <int BN, int FE>
__device__ __forceinline__ void gemm_epilogue_fast(const GemmArgs& g, f32x16 (&acc)[BN / 32],
                                                   float* smem, int64_t m0, int wave, int lane) {
  constexpr int NT = BN / 32;
  constexpr bool BIAS = FE & 1, RELU = FE & 2, L2 = FE & 4;
  const int r = lane & 31;
  const int h = lane >> 5;
  float bias_t[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bias_t[t] = BIAS ? g.bias[t * 32 + r] : 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    float ss = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float x = acc[t][v];
      if constexpr (BIAS) x += bias_t[t];
      if constexpr (RELU) x = fmaxf(x, 0.f);
      acc[t][v] = x;
      if constexpr (L2) ss = fmaf(x, x, ss);
    }
    if constexpr (L2) {
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) ss += __shfl_xor(ss, off);
      const float nrm = sqrtf(ss);
      if (g.row_norm && r == 0) {
        const int64_t row = m0 + wave * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row < g.M) g.row_norm[row] = nrm;
      }
      const float inv = 1.f / (nrm == 0.f ? 1.f : nrm);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t][v] *= inv;
    }
  }
  constexpr int SC = stage_cols<BN>();
  constexpr int OSTR = SC + 4;
  constexpr int TPR = SC / 32;
  float* Ot = smem + wave * 32 * OSTR;
#pragma unroll
  for (int round = 0; round < NT / TPR; ++round) {
    __syncthreads();
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int rl = (v & 3) + 8 * (v >> 2) + 4 * h;
#pragma unroll
      for (int tt = 0; tt < TPR; ++tt) Ot[rl * OSTR + tt * 32 + r] = acc[round * TPR + tt][v];
    }
    __syncthreads();
    constexpr int C4 = SC / 4;
    constexpr int ITER = 32 * C4 / kWave;
#pragma unroll
    for (int q = 0; q < ITER; ++q) {
      const int flat = q * kWave + lane;
      const int rl = flat / C4;
      const int c = (flat % C4) * 4;
      const int64_t row = m0 + wave * 32 + rl;
      if (row < g.M) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(Ot + rl * OSTR + c);
        f32x4* o = reinterpret_cast<f32x4*>(g.out + row * g.ldo + round * SC + c);
        *o = v;  // (non-temporal stores: +1 %, no store at all: the K loop still holds it —
                 // profiles/r04i_gemm_store_ab.md)
      }
    }
  }
}

// the general form (any alignment, any K): bounds-checked loads staged through registers;
// aligned operands with K a multiple of BK take gemm_f32_glds_kernel / gemm_f32_glds16_kernel
template <int BN>
__global__ __launch_bounds__(256, GEMM_WAVES_PER_SIMD) void gemm_f32_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float smem[smem_floats<BN>()];
  float* As = smem;
  float* Ws = smem + BM * LDSK;
  constexpr int NT = BN / 32;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

  // rows / columns this thread stages (fixed for the whole kernel)
  bool arow_ok[4];
  int64_t arow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t gm = m0 + ((tid + i * 256) >> 3);
    arow_ok[i] = gm < g.M;
    arow[i] = arow_ok[i] ? gm : g.M - 1;
  }
  bool wrow_ok[NT];
  int64_t wrow[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int64_t gn = n0 + ((tid + i * 256) >> 3);
    wrow_ok[i] = gn < g.N;
    wrow[i] = wrow_ok[i] ? gn : g.N - 1;
  }
  const int kc = (tid & 7) * 4;  // k offset of this thread's float4 inside a tile

#pragma unroll 1
  for (int seg = 0; seg < 2; ++seg) {
    const float* A = seg ? g.A2 : g.A1;
    const float* W = seg ? g.W2 : g.W1;
    const int64_t K = seg ? g.K2 : g.K1;
    const int64_t lda = seg ? g.lda2 : g.lda1;
    const bool vecA = seg ? g.vecA2 : g.vecA1;
    const bool vecW = seg ? g.vecW2 : g.vecW1;
    if (K == 0) continue;
    const int mode = seg ? g.a2_mode : GNNREC_A2_NONE;
    // per-row transform of the A rows this thread stages (uniform branch on `mode`)
    float rowdiv[4];
    bool rowzero[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rowdiv[i] = 1.f;
      rowzero[i] = !arow_ok[i];
    }
    if (mode != GNNREC_A2_NONE) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t dg = a2_degree(g, arow[i]);
        if (mode == GNNREC_A2_DIV_DEG) rowdiv[i] = (float)(dg > 0 ? dg : 1);
        else rowzero[i] = rowzero[i] || dg == 0;
      }
    }
    f32x4 ra[4], rw[NT];
    auto load_tile = [&](int64_t k0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) ra[i] = load4(A, arow[i], lda, k0 + kc, K, true, vecA);
#pragma unroll
      for (int i = 0; i < NT; ++i) rw[i] = load4(W, wrow[i], K, k0 + kc, K, true, vecW);
    };
    load_tile(0);
#pragma unroll 1
    for (int64_t k0 = 0; k0 < K; k0 += BK) {
      __syncthreads();  // previous tile fully consumed
      const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
      if (mode == GNNREC_A2_DIV_DEG) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[i] = ra[i] / rowdiv[i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + i * 256;
        *reinterpret_cast<f32x4*>(As + (idx >> 3) * LDSK + kc) = rowzero[i] ? zero : ra[i];
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int idx = tid + i * 256;
        *reinterpret_cast<f32x4*>(Ws + (idx >> 3) * LDSK + kc) = wrow_ok[i] ? rw[i] : zero;
      }
      __syncthreads();
      if (k0 + BK < K) load_tile(k0 + BK);
      const float* Ar = As + (wave * 32 + r) * LDSK + h * 16;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(Ar + s4 * 4);
        f32x4 b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          b[t] = *reinterpret_cast<const f32x4*>(Ws + (t * 32 + r) * LDSK + h * 16 + s4 * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[t][s], acc[t], 0, 0, 0);
      }
    }
  }

  gemm_epilogue<BN>(g, acc, smem, m0, n0, wave, lane);
}

// ---- LDS-DMA variant (aligned operands, K1/K2 multiples of 32) -------------------
// Tiles move global -> LDS with global_load_lds_dwordx4 (no staging registers), double
// buffered: tile k+1 is in flight while the MFMAs consume tile k; a counted
// `s_waitcnt vmcnt` + raw s_barrier publishes it (a __syncthreads() would drain the DMA).
// The LDS image is lane-linear per wave-instruction (1 KiB = 8 rows x 128 B, unpadded), so
// bank conflicts are removed on the SOURCE side: 16-B chunk j of tile row R is stored at
// chunk j ^ ((R >> 1) & 7) of that row, which makes every 16-lane ds_read_b128 group of the
// fragment reads hit 16 distinct 4-bank slots.
// one 16-B-per-lane LDS-DMA (global_load_lds_dwordx4): lane L's bytes land at lds + 16 L.
// (Kept out of lambdas and host-invisible: a device builtin inside a kernel-template
// lambda makes hipcc drop the kernel's host launch stub.)
__device__ __forceinline__ void dma16(const float* src, float* lds) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
#endif
}

template <int N>
__device__ __forceinline__ void wait_vmcnt_barrier() {
  static_assert(N >= 0 && N <= 15, "vmcnt immediate");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
  else static_assert(N == 0, "add the vmcnt immediate");
}

template <int BN>
constexpr int glds_smem_floats() {
  return 2 * (BM + BN) * BK > smem_floats<BN>() ? 2 * (BM + BN) * BK : smem_floats<BN>();
}

template <int BN>
__global__ __launch_bounds__(256, (BN > 128 ? 1 : GEMM_WAVES_PER_SIMD)) void gemm_f32_glds_kernel(GemmArgs g) {
  constexpr int NT = BN / 32;
  constexpr int AI = BM * BK * 4 / 1024 / 4;   // A-tile DMA instructions per wave (4)
  constexpr int WI = BN * BK * 4 / 1024 / 4;   // W-tile DMA instructions per wave (BN/32)
  constexpr int TILE = (BM + BN) * BK;         // floats per buffer
  __shared__ __attribute__((aligned(16))) float smem[glds_smem_floats<BN>()];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  const int sw = (r >> 1) & 7;                 // read-side swizzle of this lane's rows

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

  // DMA source rows of this lane (tile row R = instr*8 + lane/8, physical chunk lane%8)
  int64_t a_row[AI], w_row[WI];
  int a_chk[AI], w_chk[WI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    const int R = (wave * AI + q) * 8 + (lane >> 3);
    const int64_t gm = m0 + R;
    a_row[q] = gm < g.M ? gm : g.M - 1;
    a_chk[q] = ((lane & 7) ^ ((R >> 1) & 7)) * 4;
  }
#pragma unroll
  for (int q = 0; q < WI; ++q) {
    const int R = (wave * WI + q) * 8 + (lane >> 3);
    const int64_t gn = n0 + R;
    w_row[q] = gn < g.N ? gn : g.N - 1;
    w_chk[q] = ((lane & 7) ^ ((R >> 1) & 7)) * 4;
  }
  const int64_t my_row = m0 + wave * 32 + r;  // the A row this lane's fragments come from

  // both operand pairs (A1,W1) then (A2,W2) as ONE stream of K tiles, so the DMA of the
  // first A2 tile overlaps the last A1 tile's MFMAs (no pipeline restart between segments)
  const int nk1 = (int)(g.K1 / BK), nk = nk1 + (int)(g.K2 / BK);
  float rowdiv2 = 1.f;
  bool rowzero2 = false;
  if (g.K2 > 0 && g.a2_mode != GNNREC_A2_NONE) {
    const int32_t dg = a2_degree(g, my_row < g.M ? my_row : g.M - 1);
    if (g.a2_mode == GNNREC_A2_DIV_DEG) rowdiv2 = (float)(dg > 0 ? dg : 1);
    else rowzero2 = dg == 0;
  }
  auto issue = [&](int kt, int buf) {
    const bool s2 = kt >= nk1;
    const float* A = s2 ? g.A2 : g.A1;
    const float* W = s2 ? g.W2 : g.W1;
    const int64_t K = s2 ? g.K2 : g.K1;
    const int64_t lda = s2 ? g.lda2 : g.lda1;
    const int64_t k0 = (int64_t)(s2 ? kt - nk1 : kt) * BK;
    float* base = smem + buf * TILE;
#pragma unroll
    for (int q = 0; q < AI; ++q)
      dma16(A + a_row[q] * lda + k0 + a_chk[q], base + (wave * AI + q) * 256);
#pragma unroll
    for (int q = 0; q < WI; ++q)
      dma16(W + w_row[q] * K + k0 + w_chk[q], base + BM * BK + (wave * WI + q) * 256);
  };
  if (nk > 0) issue(0, 0);
#pragma unroll 1
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      issue(kt + 1, buf ^ 1);
      wait_vmcnt_barrier<AI + WI>();  // this wave's tile-kt DMA landed; all waves past it
    } else {
      wait_vmcnt_barrier<0>();
    }
    const bool s2 = kt >= nk1;
    const bool divide = s2 && g.a2_mode == GNNREC_A2_DIV_DEG;
    const bool zero = s2 && rowzero2;
    const float* As = smem + buf * TILE + (wave * 32 + r) * BK;
    const float* Ws = smem + buf * TILE + BM * BK + r * BK;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int pc = ((h * 4 + s4) ^ sw) * 4;
      f32x4 a = *reinterpret_cast<const f32x4*>(As + pc);
      if (divide) a = a / rowdiv2;
      else if (zero) a = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 b[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        b[t] = *reinterpret_cast<const f32x4*>(Ws + t * 32 * BK + pc);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[t][s], acc[t], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // buffer free for reuse
  }
  gemm_epilogue<BN>(g, acc, smem, m0, n0, wave, lane);
}

// ---- the same with 16-deep K tiles (short-K shapes) --------------------------------
// Half the LDS of the 32-deep kernel (2 x 16 KB at BN=128), so three blocks share a CU
// (three waves per SIMD): one block's DMA prologue and store epilogue overlap the others'
// MFMAs, which is where a K=128..256 GEMM loses its time.  LDS image per wave-instruction:
// 16 rows x 64 B; 16-B chunk j of tile row R sits at chunk j ^ ((R >> 2) & 3), so the 16
// rows a 16-lane ds_read_b128 group touches map to 16 distinct 4-bank slots.
constexpr int BK16 = 16;

//
// S stages (S−1 tiles in flight while one is consumed): a 16-deep tile is only 2048 MFMA
// cycles per wave, shorter than an HBM round trip, so with two stages each block waited
// on its DMA about as long as it computed (MFMA busy ≈56 % at M=1M, K=256, N=128).
template <int BN, int S>
constexpr int glds16_smem_floats() {
  return S * (BM + BN) * BK16 > smem_floats<BN>() ? S * (BM + BN) * BK16 : smem_floats<BN>();
}

// waves per SIMD the S-stage kernel is built for: LDS allows 3 blocks per CU up to 3 stages
template <int S>
constexpr int glds16_waves() {
  return S <= 3 ? 3 : 2;
}

template <int BN, int S, int FE = -1>
__global__ __launch_bounds__(256, glds16_waves<S>()) void gemm_f32_glds16_kernel(GemmArgs g) {
  constexpr int NT = BN / 32;
  constexpr int AI = BM * BK16 * 4 / 1024 / 4;   // A-tile DMA instructions per wave (2)
  constexpr int WI = BN * BK16 * 4 / 1024 / 4;   // W-tile DMA instructions per wave (BN/64)
  constexpr int TILE = (BM + BN) * BK16;
  static_assert(WI >= 1, "BN >= 64");
  static_assert(S >= 2 && S <= 4, "stages");
  __shared__ __attribute__((aligned(16))) float smem[glds16_smem_floats<BN, S>()];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  const int sw = (r >> 2) & 3;

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

  // DMA source rows of this lane (tile row R = instr*16 + lane/4, physical chunk lane%4)
  int64_t a_row[AI], w_row[WI];
  int a_chk[AI], w_chk[WI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    const int R = (wave * AI + q) * 16 + (lane >> 2);
    const int64_t gm = m0 + R;
    a_row[q] = gm < g.M ? gm : g.M - 1;
    a_chk[q] = ((lane & 3) ^ ((R >> 2) & 3)) * 4;
  }
#pragma unroll
  for (int q = 0; q < WI; ++q) {
    const int R = (wave * WI + q) * 16 + (lane >> 2);
    const int64_t gn = n0 + R;
    w_row[q] = gn < g.N ? gn : g.N - 1;
    w_chk[q] = ((lane & 3) ^ ((R >> 2) & 3)) * 4;
  }
  const int64_t my_row = m0 + wave * 32 + r;
  // this lane's DMA source pointers of both operand pairs, formed once (a tile adds k0):
  // the 64-bit row-offset products are not redone per tile
  const float* pa[2][AI];
  const float* pw[2][WI];
#pragma unroll
  for (int q = 0; q < AI; ++q) {
    pa[0][q] = g.A1 + a_row[q] * g.lda1 + a_chk[q];
    pa[1][q] = g.K2 > 0 ? g.A2 + a_row[q] * g.lda2 + a_chk[q] : pa[0][q];
  }
#pragma unroll
  for (int q = 0; q < WI; ++q) {
    pw[0][q] = g.W1 + w_row[q] * g.K1 + w_chk[q];
    pw[1][q] = g.K2 > 0 ? g.W2 + w_row[q] * g.K2 + w_chk[q] : pw[0][q];
  }

  // both operand pairs (A1,W1) then (A2,W2) as ONE stream of K tiles, so the DMA of the
  // first A2 tile overlaps the last A1 tile's MFMAs (no pipeline restart between segments)
  const int nk1 = (int)(g.K1 / BK16), nk = nk1 + (int)(g.K2 / BK16);
  // the mean's 1/deg (GNNREC_A2_DIV_DEG): one division per row, then a multiply per operand
  // (64 IEEE divisions per lane per launch otherwise: half the VALU of the owned-row GEMM)
  float rowinv2 = 1.f;
  bool rowzero2 = false;
  if (g.K2 > 0 && g.a2_mode != GNNREC_A2_NONE) {
    const int32_t dg = a2_degree(g, my_row < g.M ? my_row : g.M - 1);
    if (g.a2_mode == GNNREC_A2_DIV_DEG) rowinv2 = 1.f / (float)(dg > 0 ? dg : 1);
    else rowzero2 = dg == 0;
  }
  auto issue = [&](int kt, int buf) {
    const int s2 = kt >= nk1;
    const int k0 = (s2 ? kt - nk1 : kt) * BK16;
    float* base = smem + buf * TILE;
#pragma unroll
    for (int q = 0; q < AI; ++q) dma16(pa[s2][q] + k0, base + (wave * AI + q) * 256);
#pragma unroll
    for (int q = 0; q < WI; ++q) dma16(pw[s2][q] + k0, base + BM * BK16 + (wave * WI + q) * 256);
  };
#pragma unroll
  for (int j = 0; j < S - 1; ++j)
    if (j < nk) issue(j, j);
#pragma unroll 1
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt % S;
    if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
    // this wave's tile-kt DMA landed (the younger tiles may still fly); all waves past it
    const int ahead = nk - 1 - kt < S - 1 ? nk - 1 - kt : S - 1;
    if (ahead >= 3) wait_vmcnt_barrier<3 * (AI + WI)>();
    else if (ahead == 2) wait_vmcnt_barrier<2 * (AI + WI)>();
    else if (ahead == 1) wait_vmcnt_barrier<AI + WI>();
    else wait_vmcnt_barrier<0>();
    const bool s2 = kt >= nk1;
    const bool divide = s2 && g.a2_mode == GNNREC_A2_DIV_DEG;
    const bool zero = s2 && rowzero2;
    const float* As = smem + buf * TILE + (wave * 32 + r) * BK16;
    const float* Ws = smem + buf * TILE + BM * BK16 + r * BK16;
    // both halves' fragments are requested before the first MFMA: the second half's LDS
    // latency hides under the first half's 16 MFMAs (one lgkmcnt wait per half, not a
    // full drain before each)
    f32x4 a[2], b[2][NT];
#pragma unroll
    for (int s4 = 0; s4 < 2; ++s4) {
      const int pc = ((h * 2 + s4) ^ sw) * 4;
      a[s4] = *reinterpret_cast<const f32x4*>(As + pc);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        b[s4][t] = *reinterpret_cast<const f32x4*>(Ws + t * 32 * BK16 + pc);
    }
#pragma unroll
    for (int s4 = 0; s4 < 2; ++s4) {
      if (divide) a[s4] = a[s4] * rowinv2;
      else if (zero) a[s4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s4][s], b[s4][t][s], acc[t], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // buffer free for reuse
  }
  if constexpr (FE >= 0) gemm_epilogue_fast<BN, FE>(g, acc, smem, m0, wave, lane);
  else gemm_epilogue<BN>(g, acc, smem, m0, n0, wave, lane);
}

template <int BN>
int launch_gemm(const GemmArgs& g, hipStream_t s) {
  dim3 grid((unsigned)((g.M + BM - 1) / BM), (unsigned)((g.N + BN - 1) / BN));
  const bool fast = g.vecA1 && g.vecW1 && g.K1 % BK == 0 &&
                    (g.K2 == 0 || (g.vecA2 && g.vecW2 && g.K2 % BK == 0));
  // 16-deep K tiles, three stages (three blocks per CU) for 128- and 64-column outputs:
  // +5-10 % at K = 128..256 (tools/bench_gemm_k.py; the d = 64 minibatch layers overlap one
  // block's DMA prologue and epilogue with the other blocks' MFMAs), and the compile-time
  // epilogue (gemm_epilogue_fast) for the common flag sets (profiles/r03_gemm_experiments.md)
  if constexpr (BN == 128 || BN == 64) {
    const bool fast16 = g.vecA1 && g.vecW1 && g.K1 % BK16 == 0 &&
                        (g.K2 == 0 || (g.vecA2 && g.vecW2 && g.K2 % BK16 == 0));
    if (fast16) {
      const bool sig = g.epilogue & GNNREC_EPI_SIGMOID;
      const int fe = (g.bias ? 1 : 0) | ((g.epilogue & GNNREC_EPI_RELU) ? 2 : 0) |
                     ((g.epilogue & GNNREC_EPI_L2NORM) ? 4 : 0);
      if (!sig && g.accum == GNNREC_ACC_STORE && !g.bias_ne && g.N == BN && g.vecO &&
          (g.row_norm == nullptr || (fe & 4))) {
        switch (fe) {
          case 0: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3, 0>), grid, dim3(256), 0, s, g); break;
          case 1: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3, 1>), grid, dim3(256), 0, s, g); break;
          case 2: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3, 2>), grid, dim3(256), 0, s, g); break;
          case 3: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3, 3>), grid, dim3(256), 0, s, g); break;
          case 6: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3, 6>), grid, dim3(256), 0, s, g); break;
          case 7: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3, 7>), grid, dim3(256), 0, s, g); break;
          default: hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3>), grid, dim3(256), 0, s, g);
        }
        return check_launch("gnnrec_gemm_f32");
      }
      hipLaunchKernelGGL((gemm_f32_glds16_kernel<BN, 3>), grid, dim3(256), 0, s, g);
      return check_launch("gnnrec_gemm_f32");
    }
  }
  if (fast) hipLaunchKernelGGL((gemm_f32_glds_kernel<BN>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_f32_kernel<BN>), grid, dim3(256), 0, s, g);
  return check_launch("gnnrec_gemm_f32");
}

}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_gemm_f32(const float* A1, int64_t lda1, int64_t K1, const float* W1,
                               const float* A2, int64_t lda2, int64_t K2, const float* W2,
                               const int32_t* a2_deg, int a2_mode, const float* bias,
                               const float* bias_nonempty, int64_t M,
                               int64_t N, int epilogue, int accum, float out_div,
                               const float* attn_vec, float* attn_state, float* out,
                               int64_t ldo, void* stream) {
  return gnnrec_gemm_rownorm_f32(A1, lda1, K1, W1, A2, lda2, K2, W2, a2_deg, a2_mode, bias,
                                 bias_nonempty, M, N, epilogue, accum, out_div, attn_vec,
                                 attn_state, out, ldo, nullptr, stream);
}

extern "C" int gnnrec_gemm_rownorm_f32(const float* A1, int64_t lda1, int64_t K1,
                                       const float* W1, const float* A2, int64_t lda2,
                                       int64_t K2, const float* W2, const int32_t* a2_deg,
                                       int a2_mode, const float* bias,
                                       const float* bias_nonempty, int64_t M, int64_t N,
                                       int epilogue, int accum, float out_div,
                                       const float* attn_vec, float* attn_state, float* out,
                                       int64_t ldo, float* row_norm, void* stream) {
  using namespace gnnrec;
  GNNREC_REQUIRE(row_norm == nullptr || (epilogue & GNNREC_EPI_L2NORM),
                 "gnnrec_gemm_rownorm_f32: row_norm needs the L2NORM epilogue");
  GNNREC_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "gnnrec_gemm_f32: negative size");
  if (M == 0 || N == 0) return GNNREC_OK;
  GNNREC_REQUIRE(out != nullptr && ldo >= N, "gnnrec_gemm_f32: bad output");
  GNNREC_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1), "gnnrec_gemm_f32: bad A1/W1");
  GNNREC_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2), "gnnrec_gemm_f32: bad A2/W2");
  // GNNREC_A2_DEG_INDPTR: a2_deg is an int64 indptr [M + 1] (a block CSR's: no degree array
  // to build first)
  const bool deg_ip = (a2_mode & GNNREC_A2_DEG_INDPTR) != 0;
  a2_mode &= ~GNNREC_A2_DEG_INDPTR;
  GNNREC_REQUIRE(a2_mode == GNNREC_A2_NONE || a2_deg != nullptr,
                 "gnnrec_gemm_f32: a2_mode needs a2_deg");
  GNNREC_REQUIRE(bias_nonempty == nullptr || a2_deg != nullptr,
                 "gnnrec_gemm_f32: bias_nonempty needs a2_deg");
  GNNREC_REQUIRE(accum >= GNNREC_ACC_STORE && accum <= GNNREC_ACC_ATTN_LAST,
                 "gnnrec_gemm_f32: unknown accumulate mode %d", accum);
  const bool attn = accum >= GNNREC_ACC_ATTN_FIRST;
  GNNREC_REQUIRE(!attn || (attn_vec && attn_state && N <= 256),
                 "gnnrec_gemm_f32: attention accumulation needs attn_vec, attn_state, N <= 256");
  GNNREC_REQUIRE(!(epilogue & GNNREC_EPI_L2NORM) || N <= 256,
                 "gnnrec_gemm_f32: L2NORM needs N <= 256 (got %lld)", (long long)N);
  GemmArgs g;
  g.A1 = A1; g.lda1 = lda1; g.K1 = K1; g.W1 = W1;
  g.A2 = A2; g.lda2 = lda2; g.K2 = K2; g.W2 = W2;
  g.a2_deg = deg_ip ? nullptr : a2_deg;
  g.a2_ip = deg_ip ? reinterpret_cast<const int64_t*>(a2_deg) : nullptr;
  g.a2_mode = a2_mode; g.bias = bias; g.bias_ne = bias_nonempty;
  g.M = M; g.N = N; g.epilogue = epilogue; g.accum = accum; g.out_div = out_div;
  g.attn_vec = attn_vec; g.attn_state = attn_state;
  g.out = out; g.ldo = ldo;
  g.row_norm = row_norm;
  g.vecA1 = (K1 % 4 == 0) && (lda1 % 4 == 0) && aligned16(A1);
  g.vecA2 = (K2 % 4 == 0) && (lda2 % 4 == 0) && aligned16(A2);
  g.vecW1 = (K1 % 4 == 0) && aligned16(W1);
  g.vecW2 = (K2 % 4 == 0) && aligned16(W2);
  g.vecO = (N % 4 == 0) && (ldo % 4 == 0) && aligned16(out);
  hipStream_t s = as_stream(stream);
  if (N <= 32) return launch_gemm<32>(g, s);
  if (N <= 64) return launch_gemm<64>(g, s);
  if (N <= 128) return launch_gemm<128>(g, s);
  // wider outputs: 128-column blocks (two waves per SIMD) unless the row norm needs the
  // whole row in one block (the 256-column tile runs at one wave per SIMD)
  if (!(epilogue & GNNREC_EPI_L2NORM) && !attn) return launch_gemm<128>(g, s);
  return launch_gemm<256>(g, s);
}
