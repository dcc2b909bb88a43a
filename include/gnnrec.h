/*
 * gnnrec.h — C ABI of the MI355X-native message-passing path for the
 * hieucnm/GNN-RecSys user–item GNN.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and
 * returns an int status (GNNREC_OK == 0).  On failure gnnrec_last_error()
 * returns a thread-local message.  All data pointers are DEVICE pointers,
 * owned by the caller; outputs are preallocated by the caller (the same
 * contract as DGL's `_CAPI_DGLKernelSpMM`, whose outputs are allocated in
 * Python before the call).  `stream` is a hipStream_t passed as void*
 * (NULL = legacy default stream).  No entry point allocates, synchronises
 * or blocks the host unless its comment says so, so every call can be
 * captured into a hipGraph.
 *
 * Reference interfaces replaced (DGL 0.5.2 is the reference's pinned
 * third-party dependency, requirements.txt:2; it is not vendored):
 *   - gnnrec_spmm_csr_f32      <- graph.update_all(fn.copy_src|fn.u_mul_e,
 *                                 fn.mean|fn.max)  src/model.py:143-208
 *                                 (DGL gspmm -> _CAPI_DGLKernelSpMM)
 *   - gnnrec_spmm_project_f32  <- the two above fused for d = 128 (update_all +
 *                                 fc_self/fc_neigh + relu + norm in one launch)
 *   - gnnrec_spmm_project_mfma_f32 / gnnrec_spmm_project2_f32 <- the same for
 *                                 low-degree CSRs, pre-projected source rows, and
 *                                 two relations + the HeteroGraphConv aggregate
 *                                 (src/model.py:384-406) in one launch
 *   - gnnrec_gemm_f32          <- nn.Linear fc_self/fc_neigh/fc_preagg +
 *                                 relu + zero-guarded L2 norm + HeteroGraphConv
 *                                 aggregate, src/model.py:98-102,151,226-235,
 *                                 384-406; NodeEmbedding src/model.py:19-24;
 *                                 PredictingLayer src/model.py:258-271
 *   - gnnrec_sddmm_cos_f32     <- CosinePrediction.forward, F.normalize +
 *                                 apply_edges(fn.u_dot_v) src/model.py:317-327
 *                                 (DGL gsddmm -> _CAPI_DGLKernelSDDMM)
 *   - gnnrec_edge_mlp_f32      <- PredictingModule.forward src/model.py:290-305
 *   - gnnrec_edge_mlp_grouped_f32 <- the same over negative_sampler.Uniform's pair graphs
 *   - gnnrec_sample_*          <- dgl.dataloading.MultiLayer{Full,}Neighbor-
 *                                 Sampler / to_block, src/sampling.py:153-161
 *                                 (_CAPI_DGLSampleNeighbors, _CAPI_DGLToBlock)
 *   - gnnrec_gemm_tn_f32,      <- torch autograd of those layers in the
 *     gnnrec_act_backward_f32     training step, src/train/run.py:124-138
 *   - gnnrec_lstm_step_f32     <- ConvLayer._lstm_reducer src/model.py:106-121
 *   - gnnrec_lstm_step_save_f32, gnnrec_lstm_backward_step_f32, gnnrec_lstm_slots
 *                              <- autograd of _lstm_reducer (src/train/run.py:124-138)
 *   - gnnrec_gather_rows       <- blocks[0].srcdata / block edata copies
 *                                 (src/train/run.py:112,340)
 *   - gnnrec_synth_edges       <- (no reference counterpart: synthetic graph
 *                                 generator for the benchmark shapes)
 */
#ifndef GNNREC_H_
#define GNNREC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNNREC_OK 0
#define GNNREC_EINVAL 1 /* bad argument (shape, null pointer, unsupported mode) */
#define GNNREC_EHIP 2   /* HIP runtime error (launch failure, ...) */

/* reduce op for gnnrec_spmm_csr_f32 (DGL fn.sum / fn.mean / fn.max) */
#define GNNREC_REDUCE_SUM 0
#define GNNREC_REDUCE_MEAN 1
#define GNNREC_REDUCE_MAX 2
/* gnnrec_spmm_project2_f32 only: OR'ed into a relation's reduce, its source rows are read
 * non-temporally (the launch's other relation keeps the caches for its table) */
#define GNNREC_SRC_STREAM 0x100

/* gnnrec_spmm_csr_f32 flags */
#define GNNREC_SPMM_EMPTY_NEGINF 1 /* MAX: leave rows with no edge at -inf (partial
                                      maxima that are max-reduced across ranks) */
#define GNNREC_SPMM_ACCUM 2        /* out = out (+ | max) result: accumulate source-range
                                      tiles of one relation into one partial table */

/* gnnrec_gemm_f32 epilogue bits */
#define GNNREC_EPI_RELU 1
#define GNNREC_EPI_L2NORM 2 /* z /= ||z||_2, rows with ||z|| == 0 left unchanged */
#define GNNREC_EPI_SIGMOID 4

/* gnnrec_gemm_f32 accumulate modes (HeteroGraphConv aggregate across relations) */
#define GNNREC_ACC_STORE 0
#define GNNREC_ACC_ADD 1
#define GNNREC_ACC_MAX 2
/* per-relation attention across relations (build-defined, for C5; not in the reference):
 * out(v) = sum_r softmax_r(a . z_r(v)) z_r(v), accumulated online over the relation
 * launches with a per-row (running max, running sum) state [M, 2] floats:
 * FIRST initialises out/state, ATTN folds in one more relation, ATTN_LAST folds in the
 * last one and divides by the sum.  Needs attn_vec [N] and attn_state; the row must fit
 * one block (N <= 256 for gnnrec_gemm_f32). */
#define GNNREC_ACC_ATTN_FIRST 3
#define GNNREC_ACC_ATTN 4
#define GNNREC_ACC_ATTN_LAST 5

/* gnnrec_gemm_f32 row transform applied to A2 rows before the product */
#define GNNREC_A2_NONE 0
#define GNNREC_A2_DIV_DEG 1  /* row / max(deg,1)   (mean of a summed neighbourhood) */
#define GNNREC_A2_ZERO_DEG 2 /* row := 0 where deg == 0 (max of an empty neighbourhood) */
#define GNNREC_A2_DEG_INDPTR 16 /* or-ed in: a2_deg points at an int64 indptr [M + 1] and the
                                 * degrees are its differences (no degree array to build) */

/* ---- library ---------------------------------------------------------- */
int gnnrec_version(void);
const char* gnnrec_last_error(void);

/* Concurrency mode of the long-running row kernels (gnnrec_spmm_csr_f32 and its
 * _split / _planned forms, gnnrec_spmm_project_f32) when they share the chip with
 * kernels on other streams — RCCL's collectives in a multi-rank pass:
 *   reserve_cus  CUs the launches leave free (grids sized for CUs - reserve_cus);
 *   dynamic      1: rows are handed out by a device work queue (one head per XCD,
 *                then the other heads in turn) instead of a static grid-stride, so
 *                blocks that start late, behind a collective, take fewer rows.
 * The queue also keeps each XCD on a contiguous eighth of the rows (one range per
 * XCD), which is faster alone (C4 fused launch 36.7 -> 34.7 ms).  Outputs are bitwise
 * identical in every mode.  Process-wide, read at launch time; default (0, 1).  The
 * first queued launch on a device allocates its queue ring (1.2 MB, hipMalloc +
 * memset, synchronous, once). */
int gnnrec_set_concurrency(int reserve_cus, int dynamic);
int gnnrec_get_concurrency(int* reserve_cus, int* dynamic);

/* Diagnostic counters of the row queue since the library loaded: launches that ran
 * queued, and launches that fell back to the static schedule because their ring slot's
 * previous launch (on any stream) had not completed yet. */
int gnnrec_rowq_stats(int64_t* queued, int64_t* busy);

/* Diagnostic (no reference counterpart): `blocks` workgroups of `threads` threads,
 * each holding `lds_bytes` of LDS, stay resident for `usec` microseconds on
 * `stream` — a stand-in for a collective kernel's residency when measuring how the
 * row kernels share the chip with one (tools/probe_comm_overlap.py).  sink:
 * >= threads floats, never written in practice. */
int gnnrec_hold_cus(int blocks, int threads, int lds_bytes, int64_t usec, float* sink,
                    void* stream);

/* ---- a1: gather + aggregate over a dst-major CSR (K1-K3) ----------------
 * out[v, :] = reduce_{e in [indptr[v], indptr[v+1])} X[indices[e], :] * (ew ? ew[e] : 1)
 * MEAN divides the sum by max(deg,1); MAX of an empty row is 0 (or -inf with
 * GNNREC_SPMM_EMPTY_NEGINF).  Per-row reduction order is fixed, so results are
 * bitwise reproducible run to run.  indices are LOCAL row ids of X.
 * Replaces graph.update_all(...) at src/model.py:143-208. */
int gnnrec_spmm_csr_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                        const float* X, int64_t ldx, int64_t n_dst, int64_t d, int reduce,
                        int flags, float* out, int64_t ldo, void* stream);

/* Same, with heavy rows split for load balance (Zipf-skewed degrees): rows
 * with deg > split are skipped by the row kernel and reduced instead by one
 * wave per `split`-edge chunk into workspace[n_chunks, d], then combined per
 * row in chunk order (deterministic).  heavy_rows[n_heavy] = the rows with
 * deg > split; chunk_ptr[n_heavy+1] = prefix sum of ceil(deg/split);
 * chunk_row[n_chunks] = index into heavy_rows of each chunk. */
int gnnrec_spmm_csr_split_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                              const float* X, int64_t ldx, int64_t n_dst, int64_t d, int reduce,
                              int flags, float* out, int64_t ldo, int64_t split,
                              const int64_t* heavy_rows, int64_t n_heavy, const int64_t* chunk_ptr,
                              const int64_t* chunk_row, int64_t n_chunks, float* workspace,
                              void* stream);

/* The same split with the plan built on the device (no host readback of the heavy-row
 * count): plan = int64[2 + cap_h + (cap_h + 1) + cap_c] laid out {n_heavy, n_chunks,
 * heavy_rows[cap_h], chunk_ptr[cap_h+1], chunk_row[cap_c]}, with cap_h = min(n_dst,
 * n_edges / (split + 1)) and cap_c = n_edges / split + cap_h (bounds that hold for any
 * degree distribution; the build never writes past cap_h rows or cap_c chunks).
 * gnnrec_spmm_plan_build fills it (no host call in it but kernels: replayable inside a
 * captured graph); gnnrec_spmm_csr_planned_f32
 * reduces with workspace[cap_c, d].  Used for blocks whose edge count is known on the
 * host but whose degrees are not (sampled blocks, the backward's transposed blocks).
 * Overflow: a CSR that breaks those bounds (its edge count understated) gets a plan marked
 * overflowed — n_heavy = -(heavy rows found) < 0, n_chunks = 0 — and counted in a device
 * counter; the planned gather then reduces EVERY row in the row kernel (exact, unsplit), so
 * no aggregate is clipped.  gnnrec_spmm_plan_overflows synchronises the device and returns
 * how many plans have overflowed since the library loaded (0 on every well-formed CSR). */
int gnnrec_spmm_plan_overflows(int64_t* count);
int gnnrec_spmm_plan_build(const int64_t* indptr, int64_t n_dst, int64_t split, int64_t cap_h,
                           int64_t cap_c, int64_t* plan, void* stream);
int gnnrec_spmm_csr_planned_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                                const float* X, int64_t ldx, int64_t n_dst, int64_t d,
                                int reduce, int flags, float* out, int64_t ldo, int64_t split,
                                const int64_t* plan, int64_t cap_h, int64_t cap_c,
                                float* workspace, void* stream);

/* The row gathers above driven by a device row count: rows >= *live (read on the device;
 * a static-shape block's padding and dump rows, whose real count only the sampler's sizes
 * hold) are empty rows — written as 0 (sum / mean only), left alone under
 * GNNREC_SPMM_ACCUM — with no gathers, and the plan never marks them heavy.  Rows below it
 * are bitwise the plain calls'.  A captured training step over static blocks (gnnrec.capture)
 * so gathers only the batch's real edges. */
int gnnrec_spmm_csr_live_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                             const float* X, int64_t ldx, int64_t n_dst, int64_t d, int reduce,
                             int flags, float* out, int64_t ldo, const int64_t* live,
                             void* stream);
int gnnrec_spmm_plan_build_live(const int64_t* indptr, int64_t n_dst, int64_t split,
                                int64_t cap_h, int64_t cap_c, int64_t* plan,
                                const int64_t* live, void* stream);
int gnnrec_spmm_csr_planned_live_f32(const int64_t* indptr, const int32_t* indices,
                                     const float* ew, const float* X, int64_t ldx, int64_t n_dst,
                                     int64_t d, int reduce, int flags, float* out, int64_t ldo,
                                     int64_t split, const int64_t* plan, int64_t cap_h,
                                     int64_t cap_c, float* workspace, const int64_t* live,
                                     void* stream);

/* Two relations into one destination type in one launch: out_a[v] = reduce over relation
 * A's in-edges of v, out_b[v] likewise over relation B, both gathering from the same source
 * table X (C5's clicks and buys source tiles: the 12.5-edges-per-row relation runs beside
 * the 50-edges-per-row one on every wave instead of as its own latency-bound launch).  Each
 * output row is bitwise what gnnrec_spmm_csr_f32 computes for that relation; reduce / flags
 * apply to both.  No heavy-row split (callers route CSRs with rows above their split
 * threshold to gnnrec_spmm_csr_split_f32); d % 4 == 0, d <= 256, 16-B aligned rows; ew_a and
 * ew_b both given or both NULL.  Replaces two update_all calls of one HeteroGraphConv
 * layer, src/model.py:143-208,384-406. */
int gnnrec_spmm_csr2_f32(const int64_t* indptr_a, const int32_t* indices_a, const float* ew_a,
                         const int64_t* indptr_b, const int32_t* indices_b, const float* ew_b,
                         const float* X, int64_t ldx, int64_t n_dst, int64_t d, int reduce,
                         int flags, float* out_a, float* out_b, int64_t ldo, void* stream);

/* Gradient of gnnrec_spmm_csr_f32 w.r.t. X (training):
 * grad_X[indices[e]] += (ew ? ew[e] : 1) * grad_out[v] (/ deg for MEAN); for MAX the
 * gradient of each column goes to the first edge whose message equals out[v]
 * (X and out are required then).  grad_X is ACCUMULATED with float atomics. */
int gnnrec_spmm_backward_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                             const float* grad_out, int64_t ldg, const float* X, int64_t ldx,
                             const float* out, int64_t ldo, int64_t n_dst, int64_t d, int reduce,
                             float* grad_X, int64_t ldgx, void* stream);

/* ---- a2/a3/a4: fp32 MFMA GEMM with fused SAGE epilogue (K4, K7) ---------
 * acc[m,n] = sum_k A1[m,k] W1[n,k] + sum_k T(A2)[m,k] W2[n,k]   (W row-major [N,K] = nn.Linear.weight)
 * z = epi(acc + bias)      epi: relu / sigmoid, then optional row L2 norm
 * out = accumulate(out, z) (store | add | max), then out /= out_div if out_div > 0.
 * A2/W2 may be NULL with K2 == 0.  bias may be NULL.  N <= 256 when L2NORM.
 * bias_nonempty (nullable, needs a2_deg) is added before epi only on rows with
 * a2_deg > 0: a NodeEmbedding (W_e, b_e) folded into the neighbour side contributes
 * W_neigh b_e exactly on rows that have neighbours (the empty mean is 0, not b_e).
 * Replaces fc_self(h_self)+fc_neigh(h_neigh), relu, norm (src/model.py:226-235) and
 * HeteroGraphConv's cross-relation sum/mean/max (src/model.py:384-406). */
int gnnrec_gemm_f32(const float* A1, int64_t lda1, int64_t K1, const float* W1,
                    const float* A2, int64_t lda2, int64_t K2, const float* W2,
                    const int32_t* a2_deg, int a2_mode, const float* bias,
                    const float* bias_nonempty, int64_t M, int64_t N, int epilogue, int accum,
                    float out_div,
                    const float* attn_vec, float* attn_state,
                    float* out, int64_t ldo, void* stream);
/* Same; with the L2NORM epilogue, row_norm[M] (nullable) receives each row's norm before
 * the normalisation (0 for a zero row) — what the training backward needs besides z. */
int gnnrec_gemm_rownorm_f32(const float* A1, int64_t lda1, int64_t K1, const float* W1,
                            const float* A2, int64_t lda2, int64_t K2, const float* W2,
                            const int32_t* a2_deg, int a2_mode, const float* bias,
                            const float* bias_nonempty, int64_t M, int64_t N, int epilogue,
                            int accum, float out_div, const float* attn_vec, float* attn_state,
                            float* out, int64_t ldo, float* row_norm, void* stream);

/* ---- a1+a3 fused: aggregation with the projection in its epilogue -----------
 * out[v] (accum)= epi( H[v] W_self^T + agg(v) W_neigh^T ),  agg(v) = reduce over v's
 * in-edges of X[indices[e]] (* ew[e]) exactly as gnnrec_spmm_csr_f32 computes it
 * (bit-identical aggregate), epi = RELU / L2NORM bits, accum / out_div as gnnrec_gemm_f32.
 * W_selfT / W_neighT: the TRANSPOSED nn.Linear weights, [d, d] row-major (k-major).
 * bias [d] (nullable) is added to every row before epi; bias_nonempty [d] (nullable) only
 * to rows with in-degree > 0 — together they carry a NodeEmbedding folded into the layer
 * (H = raw features, W_self <- W_self W_emb, bias = W_self b_emb; X = raw features,
 * W_neigh <- W_neigh W_emb, bias_nonempty = W_neigh b_emb; mean/sum reducers only).
 * d = 128 only (d_neigh = d_self = out); X, H, W 16-B aligned with ld % 4 == 0.
 * Rows of any degree are reduced by one wavefront (callers route CSRs with heavy
 * rows to spmm_csr_split + gemm).  Replaces update_all + fc_self/fc_neigh + relu +
 * norm, src/model.py:143-208,226-235, and HeteroGraphConv's aggregate (:384-406). */
int gnnrec_spmm_project_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                            const float* X, int64_t ldx, const float* H, int64_t ldh,
                            const float* W_selfT, const float* W_neighT, const float* bias,
                            const float* bias_nonempty, int64_t n_dst, int64_t d, int reduce,
                            int epilogue, int accum, float out_div, const float* attn_vec,
                            float* attn_state, float* out, int64_t ldo, void* stream);

/* The same operation with the projection on the MFMA, for low-degree CSRs (callers
 * pick it below ~24 edges per row): 32-row tiles, [h_self | agg] staged in LDS and
 * multiplied by the register-resident weights with v_mfma_f32_32x32x2_f32, so the
 * weights are read once per 32 rows.  Same arguments, contract and aggregate bits as
 * gnnrec_spmm_project_f32; the projection's summation order differs (fp32 rounding).
 * W_neighT == NULL (reduce SUM / MEAN only): X holds pre-projected source rows
 * (X W_neigh^T, e.g. from gnnrec_gemm_f32) and the neighbour term is agg(v) itself —
 * the projection moved ahead of the linear reduction (equal up to fp32 rounding), worth
 * it where the source type has fewer rows than the destination.  gnnrec_spmm_project_f32
 * rejects a NULL W_neighT (GNNREC_EINVAL). */
int gnnrec_spmm_project_mfma_f32(const int64_t* indptr, const int32_t* indices,
                                 const float* ew, const float* X, int64_t ldx, const float* H,
                                 int64_t ldh, const float* W_selfT, const float* W_neighT,
                                 const float* bias, const float* bias_nonempty, int64_t n_dst,
                                 int64_t d, int reduce, int epilogue, int accum, float out_div,
                                 const float* attn_vec, float* attn_state, float* out,
                                 int64_t ldo, void* stream);

/* Two pre-projected relations into one destination type in one launch (HeteroGraphConv
 * with exactly two relations into the type, both reduced by sum / mean — C5's clicked-by
 * and bought-by into users):
 *   out[v] = combine( epi(H[v] W_self_a^T + agg_a(v) + bias_a [+ bias_nonempty_a]),
 *                     epi(H[v] W_self_b^T + agg_b(v) + bias_b [+ bias_nonempty_b]) ) / out_div
 * agg_r = reduce_r over relation r's in-edges of Y_r[indices_r[e]] (* ew_r[e]), Y_r the
 * source rows already multiplied by W_neigh,r^T; combine GNNREC_ACC_ADD (sum; mean with
 * out_div = 2), GNNREC_ACC_MAX, or GNNREC_ACC_ATTN_LAST with attn_vec [d] (out = the
 * softmax over r of attn_vec . y_r weighting the y_r; attn_vec NULL otherwise); out_div <= 0:
 * none.  reduce_r may carry GNNREC_SRC_STREAM: relation r's gathered rows are loaded
 * non-temporally (give it to the relation with fewer edges: C5's bought-by next to
 * clicked-by, 39.5 -> 37.8 ms — the two 512 MB tables no longer share the Infinity Cache);
 * the values are the same either way.  Both CSRs have n_dst rows.  The
 * self row is read once and the output written once.  d = 128; alignment as
 * gnnrec_spmm_project_f32.  Equal to the two single-relation launches up to fp32 rounding
 * (the projection's summation order).  Replaces two ConvLayer.forward calls + the
 * HeteroGraphConv aggregate, src/model.py:143-235,384-406. */
int gnnrec_spmm_project2_f32(const int64_t* indptr_a, const int32_t* indices_a,
                             const float* ew_a, const float* Ya, int64_t ldya, int reduce_a,
                             const float* bias_nonempty_a, const int64_t* indptr_b,
                             const int32_t* indices_b, const float* ew_b, const float* Yb,
                             int64_t ldyb, int reduce_b, const float* bias_nonempty_b,
                             const float* H, int64_t ldh, const float* W_self_aT,
                             const float* W_self_bT, const float* bias_a, const float* bias_b,
                             int64_t n_dst, int64_t d, int epilogue, int combine,
                             const float* attn_vec, float out_div, float* out, int64_t ldo,
                             void* stream);

/* Two relations into one destination type that gather from ONE source table (C5's
 * clicked-by and bought-by, both from the item table), all four projections in the launch:
 *   out[v] = combine( epi(H[v] W_self_a^T + agg_a(v) W_neigh_a^T + bias_a [+ bias_nonempty_a]),
 *                     epi(H[v] W_self_b^T + agg_b(v) W_neigh_b^T + bias_b [+ bias_nonempty_b]) )
 *            / out_div
 * agg_r = sum / mean over relation r's in-edges of X[indices_r[e]] (* ew_r[e]), X [n_src, d]
 * with row stride ldx (indices_r < n_src).  WT4 is the
 * packed k-major weight array [W_self_a^T | W_neigh_a^T | W_self_b^T | W_neigh_b^T], four
 * contiguous d x d blocks (block[k][n] = W[n][k]); the projections run on the fp32 MFMA.
 * 32-row tiles; the gathered working set is the one table (gnnrec_spmm_project2_f32 gathers
 * two pre-projected ones).
 * combine / attn_vec / out_div / epilogue / d /
 * alignment as gnnrec_spmm_project2_f32; bias_r NULL: none.  Each aggregate has the bits
 * of gnnrec_spmm_csr_f32's; the projection sums k in a fixed order of its own.  Replaces two
 * ConvLayer.forward calls + the HeteroGraphConv aggregate, src/model.py:143-235,384-406. */
int gnnrec_spmm_pair_f32(const int64_t* indptr_a, const int32_t* indices_a, const float* ew_a,
                         int reduce_a, const float* bias_a, const float* bias_nonempty_a,
                         const int64_t* indptr_b, const int32_t* indices_b, const float* ew_b,
                         int reduce_b, const float* bias_b, const float* bias_nonempty_b,
                         const float* X, int64_t n_src, int64_t ldx, const float* H,
                         int64_t ldh, const float* WT4, int64_t n_dst,
                         int64_t d, int epilogue, int combine, const float* attn_vec,
                         float out_div, float* out, int64_t ldo, void* stream);

/* ---- a7: cosine edge score (K5) ------------------------------------------
 * out[e] = < Hs[src[e]] / max(||Hs[src[e]]||,1e-12) , Hd[dst[e]] / max(||Hd[dst[e]]||,1e-12) >
 * Replaces CosinePrediction.forward, src/model.py:317-327. */
int gnnrec_sddmm_cos_f32(const int64_t* src, const int64_t* dst, int64_t n_edges,
                         const float* Hs, int64_t lds, const float* Hd, int64_t ldd, int64_t d,
                         float* out, void* stream);
/* The same scores for the training pair graphs of negative_sampler.Uniform(K)
 * (src/sampling.py:163-165: every positive edge's source repeated K times): group g = source
 * src_g[g], its positive edge to first[g] (may be NULL) -> out_first[g], and its K negatives
 * to dst[g K + j] -> out[g K + j].  One gathered row per edge; bitwise the scores of
 * gnnrec_sddmm_cos_f32 on the expanded edge lists.  d % 4 == 0, d <= 256, 16-B aligned. */
int gnnrec_sddmm_cos_grouped_f32(const int64_t* src_g, int64_t n_groups, const int64_t* first,
                                 float* out_first, int64_t K, const int64_t* dst, float* out,
                                 const float* Hs, int64_t lds, const float* Hd, int64_t ldd,
                                 int64_t d, void* stream);

/* ---- a8: PredictingLayer over gathered edge endpoints (K6) ---------------
 * P = Hs W1a^T + b1 and Q = Hd W1b^T are precomputed per node by gnnrec_gemm_f32
 * (W1 = [W1a | W1b], hidden_1 of PredictingLayer).  Per edge:
 * out[e] = sigmoid( w3 . relu( W2 relu(P[src[e]] + Q[dst[e]]) + b2 ) + b3 )
 * with hidden sizes fixed by the reference at 128 and 32 (src/model.py:258-260). */
int gnnrec_edge_mlp_f32(const int64_t* src, const int64_t* dst, int64_t n_edges,
                        const float* P, const float* Q, const float* W2, const float* b2,
                        const float* w3, const float* b3, float* out, void* stream);
/* The same scores for negative_sampler.Uniform(K)'s pair graphs (src/sampling.py:163-165),
 * grouped as gnnrec_sddmm_cos_grouped_f32: group g = source src_g[g], its positive edge to
 * first[g] (may be NULL) -> out_first[g], and its K negatives to dst[g K + j] -> out[g K + j];
 * the source's P row is read once per 256 edges.  The scores equal gnnrec_edge_mlp_f32's on
 * the expanded edge lists (the same kernel body). */
int gnnrec_edge_mlp_grouped_f32(const int64_t* src_g, int64_t n_groups, const int64_t* first,
                                float* out_first, int64_t K, const int64_t* dst, float* out,
                                const float* P, const float* Q, const float* W2, const float* b2,
                                const float* w3, const float* b3, void* stream);

/* ---- a9: block sampler (K8) ----------------------------------------------
 * Per relation, for each seed (dst) v: collect its in-edges from the global
 * in-CSR (indptr/indices/eids), skipping edges whose eid is marked in
 * `excluded` (byte per eid, may be NULL), keeping all of them (fanout < 0)
 * or min(fanout, deg) chosen without replacement by a counter-based RNG
 * keyed on (seed_key, v).  Two phases: count, then fill at caller offsets.
 * excluded_rows (byte per dst node, may be NULL): when given, only seeds v with
 * excluded_rows[v] != 0 have excluded in-edges (the caller marks the dst of every
 * excluded eid) — the others skip the eid checks; the result is the same. */
int gnnrec_sample_count(const int64_t* indptr, const int64_t* eids, const uint8_t* excluded,
                        const uint8_t* excluded_rows, const int64_t* seeds, int64_t n_seeds,
                        int64_t fanout, uint64_t seed_key, int64_t* counts, void* stream);
int gnnrec_sample_fill(const int64_t* indptr, const int32_t* indices, const int64_t* eids,
                       const uint8_t* excluded, const uint8_t* excluded_rows,
                       const int64_t* seeds, int64_t n_seeds, int64_t fanout,
                       uint64_t seed_key, const int64_t* out_indptr, int64_t* out_src,
                       int64_t* out_eid, void* stream);
/* exclusive prefix sum of n int64 values (in-place allowed); workspace of
 * gnnrec_scan_workspace_bytes(n) bytes; out[n] receives the total. */
int64_t gnnrec_scan_workspace_bytes(int64_t n);
int gnnrec_exclusive_scan_i64(const int64_t* in, int64_t n, int64_t* out, void* workspace,
                              void* stream);
int gnnrec_exclusive_scan_i32(const int32_t* in, int64_t n, int64_t* out, void* workspace,
                              void* stream);
/* relabel (DGL to_block): mark[id] = 1 for every id in ids (global), then
 * after a scan of mark, local[i] = n_prefix + rank(ids[i]) unless ids[i] is
 * one of the dst-prefix nodes (prefix_pos[id] >= 0), which keep their slot.  Negative ids
 * (the unused tail of a capacity-sized sample buffer) are skipped: no mark, local = -1. */
int gnnrec_mark_ids(const int64_t* ids, int64_t n, const int64_t* prefix_pos, int32_t* mark,
                    void* stream);
int gnnrec_relabel_ids(const int64_t* ids, int64_t n, const int64_t* prefix_pos,
                       const int64_t* rank, int64_t n_prefix, int64_t* local, void* stream);
int gnnrec_compact_marked(const int32_t* mark, const int64_t* rank, int64_t n_nodes,
                          int64_t* out_ids, void* stream);
int gnnrec_set_prefix_pos(const int64_t* prefix, int64_t n, int64_t* prefix_pos, void* stream);
int gnnrec_clear_prefix_pos(const int64_t* prefix, int64_t n, int64_t* prefix_pos, void* stream);

/* ---- a9: every block of one bounded-fanout sample_blocks call, fused ------
 * BlockSampler.sample_blocks (src/sampling.py:153-161: MultiLayerNeighborSampler, the
 * per-layer to_block, exclude_eids) for L steps — step 0 is the OUTPUT block, sampled from
 * the batch seeds; step s+1 samples from step s's source nodes — in 1 + 3L launches with no
 * host synchronisation (DGL: _CAPI_DGLSampleNeighbors + _CAPI_DGLToBlock per layer):
 *   begin       every type's seed positions, the first step's new-source bitmaps zeroed,
 *               the exclusion flags set (excl_mask[eid], excl_rows[dst(eid)]);
 *   pick(s)     per (relation, seed) the in-edges (all when deg <= fanout, else `fanout`
 *               by Floyd's algorithm on the counter hash — the picks of gnnrec_sample_fill),
 *               excluded eids dropped, written at seed x fanout capacity slots with the
 *               per-seed count; every picked source that is not a seed of its type sets its
 *               bit in the type's bitmap; the next step's bitmaps are zeroed;
 *   scan(s)     per relation the counts -> out_indptr, per type the bitmap popcounts ->
 *               word ranks (one block per relation / type);
 *   finalize(s) the picks compacted into the block CSR with LOCAL source ids (a seed keeps
 *               its position, a new source = n_seeds + its rank among the new ids, i.e.
 *               ascending global id: the relabel of gnnrec_mark_ids/relabel_ids), the
 *               source node list (seeds, then new ids ascending) = the next step's seeds,
 *               and the last step clears the exclusion flags.
 * The blocks are bitwise those of gnnrec_sample_count/fill + the mark/scan/relabel path
 * with the same keys.  Capacities bound every output (gnnrec_sample_blocks_caps), and the
 * actual sizes land in `sizes` on the device: [-1..L-1][types] source node counts
 * (row -1: the seed counts) at sizes[0 .. (L+1)*T), then [0..L-1][rels] edge counts.
 * Per type the caller keeps `pos` (int64 [2 * n_nodes], all zero before the first call) and
 * `bits` (uint64 [2 * ceil(n_nodes/64)]) / `word_rank` (int64 [ceil(n_nodes/64) + 1])
 * scratch across calls; `stamp` >= 1 grows by L + 1 per call on the same `pos` arrays (the
 * caller zeroes `pos` and restarts at 1 before it would pass 2^32 - 2).  A seed listed twice
 * keeps its first position (its later copies get local ids but no edges point at them).
 * Static shapes (static_shapes = 1): every output at its capacity and nothing to read back,
 * so the call (and a training step over its blocks) can be captured into a hipGraph.  Seed
 * slots holding -1 are padding rows and form a suffix (step 0's seeds: the batch padded to
 * a fixed count).  After its seed_cap seed rows every destination type gets D dump rows,
 * D = dump_rows[s][t] = 1 + max over the relations into it of ceil(edge_cap / 2048):
 * out_indptr holds seed_cap + 1 + D entries.  A padding row holds `fanout` padding edges;
 * the dump rows hold the rest of the edge capacity in runs of at most 2048 edges (no row
 * heavier than a heavy-row split, so nothing downstream needs a plan); every padding edge
 * comes from a padding slot of the source list (past its real sources, spread evenly;
 * node_cap - 1 always is one) with eid -1.  The source list holds the exact call's list
 * (real seeds, then the new sources, at the same positions and local ids), then -1 up to
 * node_cap + D' entries, D' = the next step's dump rows (1 at the last step): their index
 * there starts at seed_cap, this step's node_cap, so one layer's output rows are exactly
 * the source rows of the block it feeds.  A padding row may sit over a real source's slot:
 * no real row reads its output and its gradient is zero.  node_cap = max(seed_cap + D,
 * min(n_nodes, seed_cap + edges sourced from the type) + 1); `sizes` then holds the real
 * seed / node counts per step and the edge counts of the seed rows (the dump rows' aside). */
#define GNNREC_SB_MAX_RELS 8
#define GNNREC_SB_MAX_TYPES 4
#define GNNREC_SB_MAX_STEPS 4

typedef struct gnnrec_sample_rel {
  const int64_t* indptr;  /* in-CSR over global ids: [n_dst + 1] */
  const int32_t* indices; /* global source ids [E] */
  const int64_t* eids;    /* [E] */
  int32_t src_type, dst_type;
  const int64_t* excl_eids; /* excluded eids of this relation (NULL / 0: none) */
  int64_t n_excl;
  const int64_t* coo_dst; /* [E] dst of every eid (for the excluded eids' dst rows) */
  uint8_t* excl_mask;     /* [E] flags, zero between calls */
  uint8_t* excl_rows;     /* [n_dst] flags, zero between calls */
  /* optional (NULL: read indices / eids): the CSR's edges as one 8-byte record each,
   * rec[e] = (uint64)eids[e] << 32 | (uint32)indices[e] (every eid < 2^31) — a pick then
   * reads ONE record, one cache line, where the two arrays cost two (a fanout pick from a
   * long row touches a line of each per edge); the same picks and outputs either way */
  const uint64_t* edge_rec;
} gnnrec_sample_rel;

typedef struct gnnrec_sample_type {
  int64_t n_nodes;
  const int64_t* seeds; /* step 0's destination nodes (the batch) */
  int64_t n_seeds;
  int64_t* pos;         /* scratch, see above: [2 * n_nodes] */
  uint64_t* bits;
  int64_t* word_rank;
  uint8_t* marks;       /* scratch: [4 * 64 * ceil(n_nodes/64)] bytes, zero before the first
                         * call, 16-byte aligned: two new-source mark arrays (new sources are
                         * marked by byte stores, the scan packs them into `bits`), then two
                         * seed mark arrays (a step's seeds, one byte per node; each call
                         * leaves them zero) */
} gnnrec_sample_type;

typedef struct gnnrec_sample_plan {
  int n_rels, n_types, n_steps;
  gnnrec_sample_rel rel[GNNREC_SB_MAX_RELS];
  gnnrec_sample_type type[GNNREC_SB_MAX_TYPES];
  int64_t fanout[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS]; /* 0..64 */
  uint64_t key[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  uint32_t stamp;
  int static_shapes;    /* 0: exact sizes (read `sizes`), 1: capacities, -1-padded (above) */
  /* static shapes: a tighter node capacity per step and type than the provable one (0: none;
   * never below seed_cap + D).  A batch whose real sources do not fit sets *overflow to 1
   * (device, nullable) and stays memory-safe — sources past the capacity are left out and
   * their edges point at a padding slot — so the caller discards or redoes that batch. */
  int64_t node_cap_hint[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_TYPES];
  int64_t* overflow;
  /* outputs, sized by gnnrec_sample_blocks_caps: per step s and relation r the block CSR
   * (out_indptr [seed_cap + 1 (+ D static)], out_src int32 local ids [edge_cap], out_eid
   * [edge_cap]), per step and type the source node ids [node_cap (+ D' static)] (seeds first) */
  int64_t* out_indptr[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  int32_t* out_src[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  int64_t* out_eid[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_RELS];
  int64_t* nodes[GNNREC_SB_MAX_STEPS][GNNREC_SB_MAX_TYPES];
  int64_t* sizes;       /* device, (L + 1) * T + L * R int64 */
  void* workspace;      /* device, gnnrec_sample_blocks_caps' workspace_bytes */
} gnnrec_sample_plan;

/* Host only: per step the capacities of the outputs (seed_cap [s][t]: destination nodes,
 * edge_cap [s][r] = seed_cap[s][dst] x fanout, node_cap [s][t] = seed_cap[s][t] +
 * min(n_nodes_t, sum of edge_cap[s][r] over relations sourced from t), static shapes: see
 * above; seed_cap[s+1] = node_cap[s]) and the static dump rows (0 otherwise; nullable), each
 * flattened [step][GNNREC_SB_MAX_*], and the workspace bytes. */
int gnnrec_sample_blocks_caps(const gnnrec_sample_plan* plan, int64_t* seed_cap,
                              int64_t* edge_cap, int64_t* node_cap, int64_t* dump_rows,
                              int64_t* workspace_bytes);
int gnnrec_sample_blocks(const gnnrec_sample_plan* plan, void* stream);

/* compact_graphs over id lists (EdgeDataLoader's pair graphs, src/sampling.py:167-207 ->
 * DGL compact_graphs([pos, neg])) at static shapes, for a captured training step: per node
 * type the ids of its lists form one ascending node list, padded with -1 to `cap` (the
 * caller's bound on the distinct ids: past it ids are left out of the list and their local ids
 * point past cap, so the caller must rule that out), and every list
 * element gets its position in that list.  3 launches (mark bits, a chained scan of the
 * popcounts, relabel + list), no host synchronisation; `bits` (uint64 [2 * ceil(n_nodes/64)], zero before the
 * first call) and `word_rank` (int64 [ceil(n_nodes/64) + 1]) are the caller's scratch, and
 * `parity` alternates 0 / 1 between calls on the same scratch.  count [n_types] (device)
 * receives each type's number of distinct ids.  The lists' order does not matter: the node
 * lists are those of the per-type mark / scan / compact path (gnnrec_mark_ids & co.). */
#define GNNREC_COMPACT_MAX_LISTS 8
typedef struct gnnrec_compact_list {
  const int64_t* ids; /* global ids (>= 0) of node type `type` */
  int64_t n;
  int32_t type;
  int64_t* local;     /* [n] out: position in the type's node list */
} gnnrec_compact_list;
typedef struct gnnrec_compact_type {
  int64_t n_nodes;
  uint64_t* bits;
  int64_t* word_rank;
  int64_t* nodes;     /* [cap] out */
  int64_t cap;
  uint8_t* marks;     /* [2 * 64 * ceil(n_nodes/64)] bytes, zero before the first call,
                       * 16-byte aligned, parity halves like `bits` */
  uint64_t* scan_ws;  /* [GNNREC_COMPACT_SCAN_WS(n_nodes)] words, any contents (the call
                       * zeroes them): the scan's ticket and tile flags */
} gnnrec_compact_type;
#define GNNREC_COMPACT_SCAN_WS(n_nodes) (2 + ((n_nodes) + 63) / 64 / 1024)
int gnnrec_compact_ids(const gnnrec_compact_list* lists, int n_lists,
                       const gnnrec_compact_type* types, int n_types, int parity, int64_t* count,
                       void* stream);

/* ---- f1: recommendation top-k --------------------------------------------
 * For each row r of scores[n_rows, n_cols] (leading dimension ld): the k
 * (1..2^20) best columns ordered by (score desc, column asc), skipping the
 * columns listed in exclude_indices[exclude_indptr[r] .. exclude_indptr[r+1])
 * (already-bought items; both pointers may be NULL).  Rows with fewer than k
 * eligible columns are padded with (-inf, -1).  out_vals/out_idx: [n_rows, k].
 * k > 64 streams the rows once per 64 results (reference --k is unbounded,
 * main_inference.py:198). 
 * Replaces the per-user argsort / filter loop of src/metrics.py:52-77. */
int gnnrec_topk_rows_f32(const float* scores, int64_t ld, int64_t n_rows, int64_t n_cols,
                         int64_t k, const int64_t* exclude_indptr, const int64_t* exclude_indices,
                         float* out_vals, int64_t* out_idx, void* stream);

/* ---- f2: projection backward (training step) -----------------------------
 * Replace torch autograd of the reference's nn.Linear layers and the
 * relu/normalise epilogue when train_model calls loss.backward()
 * (src/train/run.py:124-138; layers src/model.py:98-102,226-235,258-271).
 *
 * Weight gradient, C[M,N] (+)= A[K,M]^T B[K,N] (A = dY, B = X, K = rows):
 * deterministic split-K fp32 MFMA.  workspace: gnnrec_gemm_tn_workspace_bytes(K,M,N)
 * bytes of device memory (may be NULL when that is 0). */
int64_t gnnrec_gemm_tn_workspace_bytes(int64_t K, int64_t M, int64_t N);
int gnnrec_gemm_tn_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K,
                       int64_t M, int64_t N, float* C, int64_t ldc, int accumulate,
                       float* workspace, void* stream);
/* Same, plus colsum[M] (+)= sum_k A[k, :] (the bias gradient db = column sums of dY),
 * accumulated from the A tiles the GEMM already stages (no separate reduction pass). */
int gnnrec_gemm_tn_bias_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t K,
                            int64_t M, int64_t N, float* C, int64_t ldc, float* colsum,
                            int accumulate, float* workspace, void* stream);
/* Same, the column sum over only the rows k with row_ptr[k+1] > row_ptr[k] (row_ptr: the
 * int64 indptr of a CSR over A's K rows; NULL = every row): a NodeEmbedding folded into the
 * neighbour side adds its bias on rows with an in-edge only, so that bias's gradient sums
 * those rows (torch_ops sage_rel_backward; replaces (dY * (deg > 0)).sum(0)). */
int gnnrec_gemm_tn_bias_rows_f32(const float* A, int64_t lda, const float* B, int64_t ldb,
                                 int64_t K, int64_t M, int64_t N, float* C, int64_t ldc,
                                 float* colsum, const int64_t* row_ptr, int accumulate,
                                 float* workspace, void* stream);
/* gu = d/du of z = norm?(relu?(u)) applied to gz, flags = GNNREC_EPI_RELU|GNNREC_EPI_L2NORM
 * (norm: z = a / ||a||, rows with ||a|| == 0 unchanged — the zero-guarded norm of
 * src/model.py:231-235).  u: the pre-activation rows [n_rows, d]. */
int gnnrec_act_backward_f32(const float* u, int64_t ldu, const float* gz, int64_t ldg,
                            int64_t n_rows, int64_t d, int flags, float* gu, int64_t ldo,
                            void* stream);
/* The same Jacobian from the NORMALISED output z = a / |a| (a = relu?(u)) and the row
 * norms |a| that gnnrec_gemm_rownorm_f32 wrote: gu = mask (gz - z (z.gz)) / |a| (gz for
 * |a| == 0), mask = [z > 0] when relu — the training forward keeps z, not u. */
int gnnrec_act_backward_normed_f32(const float* z, int64_t ldz, const float* row_norm,
                                   const float* gz, int64_t ldg, int64_t n_rows, int64_t d,
                                   int relu, float* gu, int64_t ldo, void* stream);

/* f2: source-major transpose of a dst-major CSR block (training backward of a1; the
 * reference's DGL update_all backward, src/model.py:161-167).  indptr_t[n_src+1] (int64),
 * indices_t[n_edges] = dst row of each edge, grouped by source row, ascending edge id
 * inside a row (stable).  ew_t[k] = ew[e] (· 1/deg(dst_e) when mean != 0); ew_t may be
 * NULL when ew is NULL and mean == 0.  int32 ids (n_edges, n_src < 2^31).  Workspace
 * from gnnrec_csr_transpose_workspace_bytes (radix-sort scratch + 5 edge arrays). */
size_t gnnrec_csr_transpose_workspace_bytes(int64_t n_edges, int64_t n_src);
int gnnrec_csr_transpose(const int64_t* indptr, const int32_t* indices, const float* ew,
                         int64_t n_dst, int64_t n_src, int64_t n_edges, int mean,
                         void* workspace, size_t workspace_bytes, int64_t* indptr_t,
                         int32_t* indices_t, float* ew_t, void* stream);

/* Rows of a COO edge list: stable sort of int32 row keys.  indptr[n_rows+1] (int64),
 * perm[n_edges] = edge ids grouped by row, ascending inside a row.  Replaces the
 * argsort/bincount/cumsum CSR build on the training path (no host readback). */
size_t gnnrec_csr_from_keys_workspace_bytes(int64_t n_edges, int64_t n_rows);
int gnnrec_csr_from_keys(const int32_t* keys, int64_t n_edges, int64_t n_rows, void* workspace,
                         size_t workspace_bytes, int64_t* indptr, int32_t* perm, void* stream);

/* ---- f3: graph construction ----------------------------------------------
 * dst-major CSR of a COO relation (src[e], dst[e]) e = 0..n_edges-1, in-row order =
 * edge id (DGL's in-CSR of a heterograph built by dgl.heterograph, reference
 * src/builder.py:377-383, reverse relations src/utils_data.py:204-238; the reverse
 * relation's CSR is the same call with src and dst swapped).  indptr[n_dst+1] (int64),
 * indices[n_edges] = src[e] narrowed to int32, eids[n_edges] (int64).  Every dst id must
 * lie in [0, n_dst); n_edges, n_dst < 2^31.  A stable LSD radix sort of the dst ids
 * (8 bits per pass, own kernels, no vendor sort): 3 passes for up to 16M rows.  Workspace
 * from gnnrec_csr_build_workspace_bytes (≈ 20 B per edge). */
size_t gnnrec_csr_build_workspace_bytes(int64_t n_edges, int64_t n_dst);
int gnnrec_csr_build(const int64_t* src, const int64_t* dst, int64_t n_edges, int64_t n_dst,
                     void* workspace, size_t workspace_bytes, int64_t* indptr, int32_t* indices,
                     int64_t* eids, void* stream);

/* K10 — DGLGraph.has_edges_between(u, v, etype) (reference src/train/run.py:95-101,160-166,
 * the false-negative mask; DGL 0.5.2 [ext]: `_CAPI_DGLHeteroHasEdgesBetween`): out[i] = 1
 * when some edge u[i] -> v[i] exists, else 0; ids outside [0, n_src) / [0, n_dst) give 0.
 * (indptr, sorted_indices) is the relation's dst-major CSR with every row's source ids in
 * ASCENDING order — gnnrec_csr_build over the edges listed in source order (the stable
 * sort keeps it inside a row) — and each query is one binary search of its row. */
int gnnrec_csr_has_edges(const int64_t* indptr, const int32_t* sorted_indices, int64_t n_dst,
                         int64_t n_src, const int64_t* u, const int64_t* v, int64_t n,
                         uint8_t* out, void* stream);

/* out[i] = a[i] + b[i] over n floats (out may alias a or b): the upper levels of the
 * deterministic pass's fixed pairwise tree over source-range partial tables. */
int gnnrec_add_f32(const float* a, const float* b, float* out, int64_t n, void* stream);

/* out[i] = ((p0[i]+p1[i])+(p2[i]+p3[i]))+... over n_parts = 2, 4 or 8 tables of n floats in
 * one pass (out may alias any part; 16-B aligned, n % 4 == 0): a whole level-by-level fold of
 * the fixed pairwise tree, bitwise equal to n_parts-1 gnnrec_add_f32 launches.  `parts` is a
 * host array of device pointers. */
int gnnrec_tree_sum_f32(const float* const* parts, int n_parts, int64_t n, float* out,
                        void* stream);

/* Row epilogue for projections wider than one GEMM block (N > 256): out (accum)=
 * l2norm?(z) row by row, accum / out_div / attention as gnnrec_gemm_f32.  z holds the
 * GEMM result with bias and ReLU already applied (the reference's hidden 384 / 512 with
 * norm=True, main.py:87, src/model.py:226-235). */
int gnnrec_row_epilogue_f32(const float* z, int64_t ldz, int64_t M, int64_t N, int l2norm,
                            int accum, float out_div, const float* attn_vec, float* attn_state,
                            float* out, int64_t ldo, void* stream);

/* ---- f4: LSTM neighbourhood reducer (one recurrence step) ------------------
 * Replaces ConvLayer._lstm_reducer (src/model.py:106-121, update_all at :164-169;
 * DGL 0.5.2 degree bucketing, messages in edge order).  Destinations are visited in
 * `order` (sorted by in-degree, descending); at step t the n_act rows order[0..n_act)
 * all have in-degree > t.  For those rows:
 *   gates = P[indices[indptr[v] + t]] + h_in W_hh^T     (P = X W_ih^T + b_ih + b_hh,
 *                                                         [N_src, 4d], gate order i,f,g,o)
 *   c = sig(f) c + sig(i) tanh(g);  h_out = sig(o) tanh(c);  out[v] = h_out at v's last step.
 * h_in/h_out/c: [n_rows, d] dense, row p = order[p]; W_hhT: [d, 4d]; d <= 512. */
int gnnrec_lstm_step_f32(const float* P, int64_t ldp, const int64_t* indptr,
                         const int32_t* indices, const int64_t* order, int64_t t, int64_t n_act,
                         const float* h_in, float* h_out, float* c, int64_t d,
                         const float* W_hhT, float* out, int64_t ldo, void* stream);

/* ---- f4/f2: the LSTM reducer's backward through time ----------------------
 * Replaces torch autograd of ConvLayer._lstm_reducer (src/model.py:106-121) under
 * loss.backward() (src/train/run.py:124-138).  Training keeps every step's state in a
 * step-major packing: step t holds rows order[0..n_t) at slots [off[t], off[t] + n_t).
 *
 * gnnrec_lstm_step_save_f32: gnnrec_lstm_step_f32 with the state split into c_in (NULL:
 *   zero, step 0) and c_out, and the pre-activation gates written to z_out [n_act, 4d].
 * gnnrec_lstm_backward_step_f32: one step t of BPTT for its n_act rows: from z, c_t and
 *   c_prev (NULL at t = 0) and the gradient arriving at h_t / c_t — dh_next / dc_next
 *   [n_next, d] for the rows still running at t+1 (p < n_next), g_out[order[p]] (row
 *   stride ldg) and 0 for the rows whose last step is t — writes dz [n_act, 4d] (gate
 *   order i, f, g, o) and dc_prev [n_act, d]; dh_{t-1} = dz W_hh is a gnnrec_gemm_f32.
 * gnnrec_lstm_slots: for every slot s < n_slots, src[s] = the source row the slot's step
 *   read (indices[indptr[order[p]] + t]) and prev[s] = the same row's slot at t - 1 (-1 at
 *   t = 0); step_off [n_steps] holds off[t] on the device. */
int gnnrec_lstm_step_save_f32(const float* P, int64_t ldp, const int64_t* indptr,
                              const int32_t* indices, const int64_t* order, int64_t t,
                              int64_t n_act, const float* h_in, float* h_out, const float* c_in,
                              float* c_out, float* z_out, int64_t d, const float* W_hhT,
                              float* out, int64_t ldo, void* stream);
int gnnrec_lstm_backward_step_f32(const float* z, const float* c_t, const float* c_prev,
                                  const float* dh_next, const float* dc_next, int64_t n_next,
                                  const float* g_out, int64_t ldg, const int64_t* order,
                                  int64_t n_act, int64_t d, float* dz, float* dc_prev,
                                  void* stream);
int gnnrec_lstm_slots(const int64_t* indptr, const int32_t* indices, const int64_t* order,
                      const int64_t* step_off, int64_t n_steps, int64_t n_slots, int64_t* src,
                      int64_t* prev, void* stream);

/* ---- a10: row gather (block features / edge data) -------------------------
 * dst row i (dst_ld_bytes apart) = src row idx[i] (src_ld_bytes apart), row_bytes each,
 * any dtype; a negative idx[i] writes a zero row.  Replaces DGL's copy of node features into
 * blocks[0].srcdata and of edge data into the blocks (read at src/train/run.py:112,340). */
/* Up to GNNREC_GATHER_MAX_JOBS independent row gathers of gnnrec_gather_rows in ONE launch
 * (a sampled batch's edge data for every block and relation plus the input block's node
 * features: one launch instead of one per table).  A negative index (a padding slot of a
 * static-shape block, gnnrec_sample_blocks) writes a zero row. */
#define GNNREC_GATHER_MAX_JOBS 16
typedef struct gnnrec_gather_job {
  const void* src;
  int64_t src_ld_bytes;
  const int64_t* idx;
  int64_t n;
  int64_t row_bytes;
  void* dst;
  int64_t dst_ld_bytes;
  const int64_t* n_dev; /* device row count (NULL: n); rows min(*n_dev, n) are gathered, so a
                         * gather can be queued before the producer's sizes reach the host */
} gnnrec_gather_job;
int gnnrec_gather_rows_batch(const gnnrec_gather_job* jobs, int n_jobs, void* stream);
int gnnrec_gather_rows(const void* src, int64_t src_ld_bytes, const int64_t* idx, int64_t n,
                       int64_t row_bytes, void* dst, int64_t dst_ld_bytes, void* stream);

/* Up to GNNREC_COPY_MAX_JOBS contiguous device copies dst[j] <- src[j] (bytes[j]) in one
 * launch: a static-shape batch handed into the buffers a captured training step replays
 * over (gnnrec/capture.py), instead of one copy engine / blit launch per tensor. */
#define GNNREC_COPY_MAX_JOBS 64
int gnnrec_copy_batch(const void* const* src, void* const* dst, const int64_t* bytes, int n,
                      void* stream);

/* ---- f2: edge-score side of the training step ----------------------------
 * max_margin_loss (src/model.py:473-533) for one etype, forward and gradient in one pass:
 *   s[e,k] = relu(((neg[e,k] + delta) - pos[e]) - mask[e,k]) / recency[e]
 * partial[b] (b < gnnrec_margin_loss_blocks(n_pos)) = sum of s over block b's rows (fixed
 * grid, fixed order); g_neg[e,k] = [pre > 0] / recency[e], g_pos[e] = -sum_k g_neg[e,k]
 * (unscaled: the caller multiplies by dL/dloss / N_total).  mask, recency nullable (0 / 1);
 * recency float32, or int64 when recency_i64 != 0.  neg is [n_pos, K] row-major. */
int64_t gnnrec_margin_loss_blocks(int64_t n_pos);
int gnnrec_margin_loss_f32(const float* pos, const float* neg, int64_t n_pos, int64_t K,
                           float delta, const float* mask, const void* recency, int recency_i64,
                           float* g_pos, float* g_neg, float* partial, int64_t n_partial,
                           void* stream);
/* out[0] = scale * sum(x[0..n)) in a fixed order (one block): the loss mean. */
int gnnrec_sum_scaled_f32(const float* x, int64_t n, float scale, float* out, void* stream);

/* Backward of gnnrec_sddmm_cos_f32 (CosinePrediction under loss.backward(), DGL's
 * SDDMM backward = SpMM): for cos_e = <u_s, v_t> / (max(|u_s|,eps) max(|v_t|,eps)),
 *   gHs[s] = inv_s (G_s - û_s (û_s . G_s)),  G_s = sum_{e: src_e = s} grad_e v_t / max(|v_t|,eps)
 * (G_s inv_s for rows with |u_s| <= eps), and symmetrically gHd.  Either output may be NULL.
 * Rows grouped by a stable key sort, heavy rows split (deterministic).  gHs / gHd are
 * dense [n, d].  Workspace: gnnrec_sddmm_cos_backward_workspace_bytes. */
size_t gnnrec_sddmm_cos_backward_workspace_bytes(int64_t n_edges, int64_t n_src, int64_t n_dst,
                                                 int64_t d);
int gnnrec_sddmm_cos_backward_f32(const int64_t* src, const int64_t* dst, int64_t n_edges,
                                  const float* Hs, int64_t lds, int64_t n_src, const float* Hd,
                                  int64_t ldd, int64_t n_dst, int64_t d, const float* grad,
                                  float* gHs, float* gHd, void* workspace,
                                  size_t workspace_bytes, void* stream);
/* The same for negative_sampler.Uniform(K)'s pair graphs (src/sampling.py:163-165): the
 * n_edges = n_groups (K + 1) edges are laid out [n_groups positives | n_groups x K
 * negatives] with src[n_groups + g K + j] = src[g], so the source side sorts only the group
 * keys: one wave per 64-edge chunk of a group gathers its weighted rows into a partial, and
 * each source row sums its groups' chunks in key order before the normalisation epilogue
 * (no sort of the n_edges).  The destination side is the call above's, each edge's source
 * taken from its group's positive.  Only src[0, n_groups) is read: the negatives' entries
 * may be absent (src = the positives' sources alone).  Sums in a fixed order; d % 4 == 0,
 * d <= 256, 16-byte aligned rows. */
size_t gnnrec_sddmm_cos_backward_grouped_workspace_bytes(int64_t n_groups, int64_t K,
                                                         int64_t n_src, int64_t n_dst, int64_t d);
int gnnrec_sddmm_cos_backward_grouped_f32(const int64_t* src, const int64_t* dst,
                                          int64_t n_groups, int64_t K, const float* Hs,
                                          int64_t lds, int64_t n_src, const float* Hd,
                                          int64_t ldd, int64_t n_dst, int64_t d,
                                          const float* grad, float* gHs, float* gHd,
                                          void* workspace, size_t workspace_bytes,
                                          void* stream);

/* ---- synthetic graph generator (benchmark shapes; no reference analogue) --
 * For e in [e0, e0+n): u[e-e0] = h(seed, e, 0) mod n_u, i[e-e0] = item(h(seed, e, 1)),
 * item() uniform (zipf_s == 0) or inverse-CDF Zipf over the table `zipf_cdf`
 * (n_i doubles, NULL for uniform).  h = splitmix64-based counter hash.
 * Reproduced bit-exactly by oracle/oracle.c. */
int gnnrec_synth_edges(uint64_t seed, int64_t e0, int64_t n, int64_t n_u, int64_t n_i,
                       const double* zipf_cdf, int32_t* u, int32_t* i, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GNNREC_H_ */
