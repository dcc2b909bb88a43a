// torch_ops.cpp — TORCH_LIBRARY(gnnrec) over the C ABI of libgnnrec.so (include/gnnrec.h).
//
// Every op is a thin, validated wrapper of one C-ABI entry point: device pointers and the
// current HIP stream of the operand's device in, the library's status out (GNNREC_EINVAL
// -> ValueError, anything else -> RuntimeError with gnnrec_last_error()).  Outputs are
// preallocated by the caller and declared mutable in the schema (Tensor(a!)), the same
// contract as the C ABI, so torch.compile functionalises them (auto_functionalize).  The
// Meta kernel of each op is the same function: on meta /
// fake tensors it runs the shape checks and returns before the launch, which is all that
// shape inference of an op with mutated outputs needs.
//
// Reference call sites these ops serve (the nn.Module drop-ins in gnnrec/nn.py):
//   spmm_csr*, spmm_project, gemm   <- ConvLayer.forward src/model.py:143-208,226-235
//   sddmm_cos                       <- CosinePrediction.forward src/model.py:317-327
//   edge_mlp                        <- PredictingModule.forward src/model.py:290-305
//   edge_mlp_grouped                <- the same over negative_sampler.Uniform's pair graphs
//   sample_*, scan, relabel ops     <- dgl samplers / to_block, src/sampling.py:153-161
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <utility>
#include <map>
#include <vector>

#include "gnnrec.h"

namespace {

using at::Tensor;
using c10::optional;

void ck(int rc, const char* what) {
  if (rc == GNNREC_OK) return;
  const char* msg = gnnrec_last_error();
  TORCH_CHECK_VALUE(rc != GNNREC_EINVAL, what, ": ", msg);
  TORCH_CHECK(false, what, ": ", msg, " (status ", rc, ")");
}

void* stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// Every device operand of one op must sit on ONE device: the guard and the stream come from
// one of them, and a pointer into another GPU's memory would fault in the kernel instead of
// raising.  Each op opens a OneDevice scope; dev()/same_dev() compare every operand with
// the first one seen in it.
thread_local bool g_op_dev_set = false;
thread_local c10::Device g_op_device{c10::DeviceType::CPU};
struct OneDevice {
  OneDevice() { g_op_dev_set = false; }
  ~OneDevice() { g_op_dev_set = false; }
};
void same_dev(const Tensor& t, const char* name) {
  if (!t.defined() || !t.is_cuda()) return;
  if (!g_op_dev_set) {
    g_op_device = t.device();
    g_op_dev_set = true;
    return;
  }
  TORCH_CHECK_VALUE(t.device() == g_op_device, name, " is on ", t.device(),
                    " but the op's other operands are on ", g_op_device);
}

// device operand (or meta/fake during tracing) of the given dtype
void dev(const Tensor& t, const char* name, c10::ScalarType dt) {
  TORCH_CHECK_VALUE(t.is_cuda() || t.is_meta(), name,
                    " must be a HIP device tensor (gnnrec has no CPU path), got ", t.device());
  TORCH_CHECK_VALUE(t.scalar_type() == dt, name, " must be ", dt, ", got ", t.scalar_type());
  same_dev(t, name);
}
void dev(const optional<Tensor>& t, const char* name, c10::ScalarType dt) {
  if (t.has_value() && t->defined()) dev(*t, name, dt);
}

bool has(const optional<Tensor>& t) { return t.has_value() && t->defined(); }

template <typename T>
T* p(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
T* p(const optional<Tensor>& t) { return has(t) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr; }

// leading dimension of a 2-D row-major operand (unit column stride)
int64_t ld(const Tensor& t, const char* name) {
  TORCH_CHECK_VALUE(t.dim() == 2, name, " must be 2-D, got ", t.sizes());
  TORCH_CHECK_VALUE(t.stride(1) == 1 || t.size(1) <= 1, name, " must have unit column stride");
  return std::max<int64_t>({t.stride(0), t.size(1), 1});
}

bool meta(const Tensor& t) { return t.is_meta(); }

// ---------------------------------------------------------------- a1 aggregation
// live (nullable, one device int64): rows from it on are empty rows (gnnrec_spmm_csr_live_f32)
const int64_t* live_ptr(const optional<Tensor>& live) {
  if (!has(live)) return nullptr;
  dev(live, "live", at::kLong);
  TORCH_CHECK_VALUE(live->numel() == 1, "live must hold one row count");
  return p<int64_t>(live);
}

void spmm_csr(const Tensor& indptr, const Tensor& indices, const optional<Tensor>& ew,
              const Tensor& X, int64_t reduce, int64_t flags, Tensor& out,
              const optional<Tensor>& live) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(X, "X", at::kFloat);
  dev(ew, "edge_weight", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t n_dst = indptr.numel() - 1, d = X.size(1);
  TORCH_CHECK_VALUE(out.size(0) == n_dst && out.size(1) == d, "out must be [", n_dst, ", ", d,
                    "], got ", out.sizes());
  const int64_t ldx = ld(X, "X"), ldo = ld(out, "out");
  if (meta(X)) return;
  const c10::DeviceGuard g(X.device());
  ck(gnnrec_spmm_csr_live_f32(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ew), p<float>(X),
                              ldx, n_dst, d, (int)reduce, (int)flags, p<float>(out), ldo,
                              live_ptr(live), stream_of(X)),
     "gnnrec_spmm_csr_f32");
}

void spmm_csr_split(const Tensor& indptr, const Tensor& indices, const optional<Tensor>& ew,
                    const Tensor& X, int64_t reduce, int64_t flags, int64_t split,
                    const Tensor& heavy, const Tensor& chunk_ptr, const Tensor& chunk_row,
                    int64_t n_chunks, Tensor& out, Tensor& ws) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(X, "X", at::kFloat);
  dev(ew, "edge_weight", at::kFloat);
  dev(heavy, "heavy_rows", at::kLong);
  dev(chunk_ptr, "chunk_ptr", at::kLong);
  dev(chunk_row, "chunk_row", at::kLong);
  dev(out, "out", at::kFloat);
  dev(ws, "workspace", at::kFloat);
  const int64_t n_dst = indptr.numel() - 1, d = X.size(1);
  TORCH_CHECK_VALUE(out.size(0) == n_dst && out.size(1) == d, "out must be [", n_dst, ", ", d, "]");
  TORCH_CHECK_VALUE(ws.numel() >= n_chunks * d, "workspace must hold n_chunks x d floats");
  const int64_t ldx = ld(X, "X"), ldo = ld(out, "out");
  if (meta(X)) return;
  const c10::DeviceGuard g(X.device());
  ck(gnnrec_spmm_csr_split_f32(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ew), p<float>(X),
                               ldx, n_dst, d, (int)reduce, (int)flags, p<float>(out), ldo, split,
                               p<int64_t>(heavy), heavy.numel(), p<int64_t>(chunk_ptr),
                               p<int64_t>(chunk_row), n_chunks, p<float>(ws), stream_of(X)),
     "gnnrec_spmm_csr_split_f32");
}

void spmm_csr2(const Tensor& indptr_a, const Tensor& indices_a, const optional<Tensor>& ew_a,
               const Tensor& indptr_b, const Tensor& indices_b, const optional<Tensor>& ew_b,
               const Tensor& X, int64_t reduce, int64_t flags, Tensor& out_a, Tensor& out_b) {
  const OneDevice one_device_;
  dev(indptr_a, "indptr_a", at::kLong);
  dev(indices_a, "indices_a", at::kInt);
  dev(ew_a, "ew_a", at::kFloat);
  dev(indptr_b, "indptr_b", at::kLong);
  dev(indices_b, "indices_b", at::kInt);
  dev(ew_b, "ew_b", at::kFloat);
  dev(X, "X", at::kFloat);
  dev(out_a, "out_a", at::kFloat);
  dev(out_b, "out_b", at::kFloat);
  const int64_t n_dst = indptr_a.numel() - 1, d = X.size(1);
  TORCH_CHECK_VALUE(indptr_b.numel() == n_dst + 1, "spmm_csr2: the relations' row counts differ");
  TORCH_CHECK_VALUE(out_a.size(0) == n_dst && out_a.size(1) == d && out_b.sizes() == out_a.sizes(),
                    "out_a / out_b must be [", n_dst, ", ", d, "]");
  const int64_t ldx = ld(X, "X"), ldo = ld(out_a, "out_a");
  TORCH_CHECK_VALUE(ld(out_b, "out_b") == ldo, "out_a and out_b must share a row stride");
  if (meta(X)) return;
  const c10::DeviceGuard g(X.device());
  ck(gnnrec_spmm_csr2_f32(p<int64_t>(indptr_a), p<int32_t>(indices_a), p<float>(ew_a),
                          p<int64_t>(indptr_b), p<int32_t>(indices_b), p<float>(ew_b), p<float>(X),
                          ldx, n_dst, d, (int)reduce, (int)flags, p<float>(out_a), p<float>(out_b),
                          ldo, stream_of(X)),
     "gnnrec_spmm_csr2_f32");
}

void spmm_plan_build(const Tensor& indptr, int64_t split, int64_t cap_h, Tensor& plan,
                     const optional<Tensor>& live) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(plan, "plan", at::kLong);
  const int64_t cap_c = plan.numel() - (3 + 2 * cap_h);  // plan = {2 | cap_h | cap_h+1 | cap_c}
  TORCH_CHECK_VALUE(cap_h >= 0 && cap_c >= 0, "spmm_plan_build: plan shorter than 3 + 2 cap_h");
  if (meta(indptr)) return;
  const c10::DeviceGuard g(indptr.device());
  ck(gnnrec_spmm_plan_build_live(p<int64_t>(indptr), indptr.numel() - 1, split, cap_h, cap_c,
                                 p<int64_t>(plan), live_ptr(live), stream_of(indptr)),
     "gnnrec_spmm_plan_build");
}

void spmm_csr_planned(const Tensor& indptr, const Tensor& indices, const optional<Tensor>& ew,
                      const Tensor& X, int64_t reduce, int64_t flags, int64_t split,
                      const Tensor& plan, int64_t cap_h, int64_t cap_c, Tensor& out, Tensor& ws,
                      const optional<Tensor>& live) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(X, "X", at::kFloat);
  dev(ew, "edge_weight", at::kFloat);
  dev(plan, "plan", at::kLong);
  dev(out, "out", at::kFloat);
  dev(ws, "workspace", at::kFloat);
  const int64_t n_dst = indptr.numel() - 1, d = X.size(1);
  TORCH_CHECK_VALUE(out.size(0) == n_dst && out.size(1) == d, "out must be [", n_dst, ", ", d, "]");
  TORCH_CHECK_VALUE(ws.numel() >= cap_c * d, "workspace must hold cap_c x d floats");
  const int64_t ldx = ld(X, "X"), ldo = ld(out, "out");
  if (meta(X)) return;
  const c10::DeviceGuard g(X.device());
  ck(gnnrec_spmm_csr_planned_live_f32(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ew),
                                      p<float>(X), ldx, n_dst, d, (int)reduce, (int)flags,
                                      p<float>(out), ldo, split, p<int64_t>(plan), cap_h, cap_c,
                                      p<float>(ws), live_ptr(live), stream_of(X)),
     "gnnrec_spmm_csr_planned_f32");
}

void spmm_backward(const Tensor& indptr, const Tensor& indices, const optional<Tensor>& ew,
                   const Tensor& grad_out, const optional<Tensor>& X,
                   const optional<Tensor>& out, int64_t reduce, Tensor& grad_X) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(ew, "edge_weight", at::kFloat);
  dev(grad_out, "grad_out", at::kFloat);
  dev(X, "X", at::kFloat);
  dev(out, "out", at::kFloat);
  dev(grad_X, "grad_X", at::kFloat);
  const int64_t n_dst = grad_out.size(0), d = grad_out.size(1);
  const int64_t ldg = ld(grad_out, "grad_out"), ldgx = ld(grad_X, "grad_X");
  const int64_t ldx = has(X) ? ld(*X, "X") : 0, ldo = has(out) ? ld(*out, "out") : 0;
  if (meta(grad_out)) return;
  const c10::DeviceGuard g(grad_out.device());
  ck(gnnrec_spmm_backward_f32(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ew),
                              p<float>(grad_out), ldg, p<float>(X), ldx, p<float>(out), ldo,
                              n_dst, d, (int)reduce, p<float>(grad_X), ldgx, stream_of(grad_out)),
     "gnnrec_spmm_backward_f32");
}

// ---------------------------------------------------------------- a2-a4 projections
void gemm(const Tensor& A1, const Tensor& W1, const optional<Tensor>& A2,
          const optional<Tensor>& W2, const optional<Tensor>& a2_deg, int64_t a2_mode,
          const optional<Tensor>& bias, const optional<Tensor>& bias_nonempty, int64_t epilogue,
          int64_t accum, double out_div, const optional<Tensor>& attn_vec,
          const optional<Tensor>& attn_state, Tensor& out, const optional<Tensor>& row_norm) {
  const OneDevice one_device_;
  dev(A1, "A1", at::kFloat);
  dev(W1, "W1", at::kFloat);
  dev(A2, "A2", at::kFloat);
  dev(W2, "W2", at::kFloat);
  dev(a2_deg, "a2_deg", at::kInt);
  dev(bias, "bias", at::kFloat);
  dev(bias_nonempty, "bias_nonempty", at::kFloat);
  dev(attn_vec, "attn_vec", at::kFloat);
  dev(attn_state, "attn_state", at::kFloat);
  dev(out, "out", at::kFloat);
  dev(row_norm, "row_norm", at::kFloat);
  const int64_t M = A1.size(0), K1 = A1.size(1), N = W1.size(0);
  TORCH_CHECK_VALUE(W1.size(1) == K1 && W1.is_contiguous(), "W1 must be a contiguous [N, ", K1, "]");
  const int64_t lda1 = ld(A1, "A1");
  int64_t K2 = 0, lda2 = 1;
  if (has(A2)) {
    TORCH_CHECK_VALUE(has(W2) && A2->size(0) == M && W2->size(0) == N &&
                          W2->size(1) == A2->size(1) && W2->is_contiguous(),
                      "A2/W2 shape mismatch");
    K2 = A2->size(1);
    lda2 = ld(*A2, "A2");
  }
  TORCH_CHECK_VALUE(out.size(0) == M && out.size(1) == N, "out must be [", M, ", ", N, "]");
  const int64_t ldo = ld(out, "out");
  if (meta(A1)) return;
  const c10::DeviceGuard g(A1.device());
  ck(gnnrec_gemm_rownorm_f32(p<float>(A1), lda1, K1, p<float>(W1), p<float>(A2), lda2, K2,
                             p<float>(W2), p<int32_t>(a2_deg), (int)a2_mode, p<float>(bias),
                             p<float>(bias_nonempty), M, N, (int)epilogue, (int)accum,
                             (float)out_div, p<float>(attn_vec), p<float>(attn_state),
                             p<float>(out), ldo, p<float>(row_norm), stream_of(A1)),
     "gnnrec_gemm_f32");
}

void row_epilogue(const Tensor& z, int64_t l2norm, int64_t accum, double out_div,
                  const optional<Tensor>& attn_vec, const optional<Tensor>& attn_state,
                  Tensor& out) {
  const OneDevice one_device_;
  dev(z, "z", at::kFloat);
  dev(attn_vec, "attn_vec", at::kFloat);
  dev(attn_state, "attn_state", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t M = z.size(0), N = z.size(1);
  TORCH_CHECK_VALUE(out.size(0) == M && out.size(1) == N, "out must be [", M, ", ", N, "]");
  const int64_t ldz = ld(z, "z"), ldo = ld(out, "out");
  if (meta(z)) return;
  const c10::DeviceGuard g(z.device());
  ck(gnnrec_row_epilogue_f32(p<float>(z), ldz, M, N, (int)l2norm, (int)accum, (float)out_div,
                             p<float>(attn_vec), p<float>(attn_state), p<float>(out), ldo,
                             stream_of(z)),
     "gnnrec_row_epilogue_f32");
}

void spmm_project(const Tensor& indptr, const Tensor& indices, const optional<Tensor>& ew,
                  const Tensor& X, const Tensor& H, const Tensor& W_selfT,
                  const optional<Tensor>& W_neighT, const optional<Tensor>& bias,
                  const optional<Tensor>& bias_nonempty, int64_t reduce, int64_t epilogue,
                  int64_t accum, double out_div, const optional<Tensor>& attn_vec,
                  const optional<Tensor>& attn_state, bool mfma, Tensor& out) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(ew, "edge_weight", at::kFloat);
  dev(X, "X", at::kFloat);
  dev(H, "H", at::kFloat);
  dev(W_selfT, "W_selfT", at::kFloat);
  dev(W_neighT, "W_neighT", at::kFloat);
  dev(bias, "bias", at::kFloat);
  dev(bias_nonempty, "bias_nonempty", at::kFloat);
  dev(attn_vec, "attn_vec", at::kFloat);
  dev(attn_state, "attn_state", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t n_dst = indptr.numel() - 1, d = X.size(1);
  TORCH_CHECK_VALUE(H.size(0) >= n_dst, "H has ", H.size(0), " rows, the CSR ", n_dst,
                    " destinations");
  TORCH_CHECK_VALUE(out.size(0) == n_dst && out.size(1) == d, "out must be [", n_dst, ", ", d, "]");
  TORCH_CHECK_VALUE(W_selfT.is_contiguous() && (!has(W_neighT) || W_neighT->is_contiguous()),
                    "transposed weights must be contiguous");
  TORCH_CHECK_VALUE(has(W_neighT) || mfma, "pre-projected source rows (W_neighT None) need the "
                    "mfma variant");
  const int64_t ldx = ld(X, "X"), ldh = ld(H, "H"), ldo = ld(out, "out");
  if (meta(X)) return;
  const c10::DeviceGuard g(X.device());
  auto fn = mfma ? gnnrec_spmm_project_mfma_f32 : gnnrec_spmm_project_f32;
  ck(fn(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ew), p<float>(X), ldx, p<float>(H), ldh,
        p<float>(W_selfT), p<float>(W_neighT), p<float>(bias), p<float>(bias_nonempty), n_dst, d,
        (int)reduce, (int)epilogue, (int)accum, (float)out_div, p<float>(attn_vec),
        p<float>(attn_state), p<float>(out), ldo, stream_of(X)),
     mfma ? "gnnrec_spmm_project_mfma_f32" : "gnnrec_spmm_project_f32");
}

void spmm_project2(const Tensor& indptr_a, const Tensor& indices_a, const optional<Tensor>& ew_a,
                   const Tensor& Ya, int64_t reduce_a, const optional<Tensor>& bias_nonempty_a,
                   const Tensor& indptr_b, const Tensor& indices_b, const optional<Tensor>& ew_b,
                   const Tensor& Yb, int64_t reduce_b, const optional<Tensor>& bias_nonempty_b,
                   const Tensor& H, const Tensor& W_self_aT, const Tensor& W_self_bT,
                   const optional<Tensor>& bias_a, const optional<Tensor>& bias_b,
                   int64_t epilogue, int64_t combine, const optional<Tensor>& attn_vec,
                   double out_div, Tensor& out) {
  const OneDevice one_device_;
  dev(indptr_a, "indptr_a", at::kLong);
  dev(indices_a, "indices_a", at::kInt);
  dev(ew_a, "ew_a", at::kFloat);
  dev(Ya, "Ya", at::kFloat);
  dev(bias_nonempty_a, "bias_nonempty_a", at::kFloat);
  dev(indptr_b, "indptr_b", at::kLong);
  dev(indices_b, "indices_b", at::kInt);
  dev(ew_b, "ew_b", at::kFloat);
  dev(Yb, "Yb", at::kFloat);
  dev(bias_nonempty_b, "bias_nonempty_b", at::kFloat);
  dev(H, "H", at::kFloat);
  dev(W_self_aT, "W_self_aT", at::kFloat);
  dev(W_self_bT, "W_self_bT", at::kFloat);
  dev(bias_a, "bias_a", at::kFloat);
  dev(bias_b, "bias_b", at::kFloat);
  dev(attn_vec, "attn_vec", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t n_dst = indptr_a.numel() - 1, d = Ya.size(1);
  TORCH_CHECK_VALUE(indptr_b.numel() == n_dst + 1,
                    "spmm_project2: the relations' row counts differ");
  TORCH_CHECK_VALUE(Yb.size(1) == d && H.size(0) >= n_dst, "spmm_project2: Yb / H shapes");
  TORCH_CHECK_VALUE(out.size(0) == n_dst && out.size(1) == d, "out must be [", n_dst, ", ", d,
                    "]");
  TORCH_CHECK_VALUE(W_self_aT.is_contiguous() && W_self_bT.is_contiguous(),
                    "transposed weights must be contiguous");
  const int64_t ldya = ld(Ya, "Ya"), ldyb = ld(Yb, "Yb"), ldh = ld(H, "H"), ldo = ld(out, "out");
  if (meta(Ya)) return;
  const c10::DeviceGuard g(Ya.device());
  ck(gnnrec_spmm_project2_f32(p<int64_t>(indptr_a), p<int32_t>(indices_a), p<float>(ew_a),
                              p<float>(Ya), ldya, (int)reduce_a, p<float>(bias_nonempty_a),
                              p<int64_t>(indptr_b), p<int32_t>(indices_b), p<float>(ew_b),
                              p<float>(Yb), ldyb, (int)reduce_b, p<float>(bias_nonempty_b),
                              p<float>(H), ldh, p<float>(W_self_aT), p<float>(W_self_bT),
                              p<float>(bias_a), p<float>(bias_b), n_dst, d, (int)epilogue,
                              (int)combine, p<float>(attn_vec), (float)out_div, p<float>(out),
                              ldo, stream_of(Ya)),
     "gnnrec_spmm_project2_f32");
}

void spmm_pair(const Tensor& indptr_a, const Tensor& indices_a, const optional<Tensor>& ew_a,
               int64_t reduce_a, const optional<Tensor>& bias_a,
               const optional<Tensor>& bias_nonempty_a, const Tensor& indptr_b,
               const Tensor& indices_b, const optional<Tensor>& ew_b, int64_t reduce_b,
               const optional<Tensor>& bias_b, const optional<Tensor>& bias_nonempty_b,
               const Tensor& X, const Tensor& H, const Tensor& WT4, int64_t epilogue,
               int64_t combine,
               const optional<Tensor>& attn_vec, double out_div, Tensor& out) {
  const OneDevice one_device_;
  dev(indptr_a, "indptr_a", at::kLong);
  dev(indices_a, "indices_a", at::kInt);
  dev(ew_a, "ew_a", at::kFloat);
  dev(bias_a, "bias_a", at::kFloat);
  dev(bias_nonempty_a, "bias_nonempty_a", at::kFloat);
  dev(indptr_b, "indptr_b", at::kLong);
  dev(indices_b, "indices_b", at::kInt);
  dev(ew_b, "ew_b", at::kFloat);
  dev(bias_b, "bias_b", at::kFloat);
  dev(bias_nonempty_b, "bias_nonempty_b", at::kFloat);
  dev(X, "X", at::kFloat);
  dev(H, "H", at::kFloat);
  dev(WT4, "WT4", at::kFloat);
  dev(attn_vec, "attn_vec", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t n_dst = indptr_a.numel() - 1, d = X.size(1);
  TORCH_CHECK_VALUE(indptr_b.numel() == n_dst + 1, "spmm_pair: the relations' row counts differ");
  TORCH_CHECK_VALUE(H.size(1) == d && H.size(0) >= n_dst, "spmm_pair: H shape");
  TORCH_CHECK_VALUE(WT4.is_contiguous() && WT4.numel() == 4 * d * d,
                    "spmm_pair: WT4 must be a contiguous [4, d, d] weight array");
  TORCH_CHECK_VALUE(out.size(0) == n_dst && out.size(1) == d, "out must be [", n_dst, ", ", d,
                    "]");
  // the kernel reads d entries of every bias and of the attention vector
  for (const auto& v : {std::make_pair(&bias_a, "bias_a"), std::make_pair(&bias_b, "bias_b"),
                        std::make_pair(&bias_nonempty_a, "bias_nonempty_a"),
                        std::make_pair(&bias_nonempty_b, "bias_nonempty_b"),
                        std::make_pair(&attn_vec, "attn_vec")})
    TORCH_CHECK_VALUE(!has(*v.first) || ((*v.first)->numel() == d && (*v.first)->is_contiguous()),
                      "spmm_pair: ", v.second, " must be a contiguous vector of ", d, " floats");
  const int64_t ldx = ld(X, "X"), ldh = ld(H, "H"), ldo = ld(out, "out");
  if (meta(X)) return;
  const c10::DeviceGuard g(X.device());
  ck(gnnrec_spmm_pair_f32(p<int64_t>(indptr_a), p<int32_t>(indices_a), p<float>(ew_a),
                          (int)reduce_a, p<float>(bias_a), p<float>(bias_nonempty_a),
                          p<int64_t>(indptr_b), p<int32_t>(indices_b), p<float>(ew_b),
                          (int)reduce_b, p<float>(bias_b), p<float>(bias_nonempty_b),
                          p<float>(X), X.size(0), ldx, p<float>(H), ldh, p<float>(WT4), n_dst, d,
                          (int)epilogue, (int)combine, p<float>(attn_vec), (float)out_div,
                          p<float>(out), ldo, stream_of(X)),
     "gnnrec_spmm_pair_f32");
}

// ---------------------------------------------------------------- a7 / a8 heads
void sddmm_cos(const Tensor& src, const Tensor& dst, const Tensor& Hs, const Tensor& Hd,
               Tensor& out) {
  const OneDevice one_device_;
  dev(src, "src", at::kLong);
  dev(dst, "dst", at::kLong);
  dev(Hs, "Hs", at::kFloat);
  dev(Hd, "Hd", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t E = src.numel();
  TORCH_CHECK_VALUE(dst.numel() == E && out.numel() == E, "src/dst/out length mismatch");
  TORCH_CHECK_VALUE(Hs.size(1) == Hd.size(1), "endpoint feature sizes differ");
  TORCH_CHECK_VALUE(src.is_contiguous() && dst.is_contiguous(), "src/dst must be contiguous");
  const int64_t lds = ld(Hs, "Hs"), ldd = ld(Hd, "Hd");
  if (meta(Hs)) return;
  const c10::DeviceGuard g(Hs.device());
  ck(gnnrec_sddmm_cos_f32(p<int64_t>(src), p<int64_t>(dst), E, p<float>(Hs), lds, p<float>(Hd),
                          ldd, Hs.size(1), p<float>(out), stream_of(Hs)),
     "gnnrec_sddmm_cos_f32");
}

void sddmm_cos_grouped(const Tensor& src_g, const optional<Tensor>& first, int64_t K,
                       const Tensor& dst, const Tensor& Hs, const Tensor& Hd,
                       Tensor& out_first, Tensor& out) {
  const OneDevice one_device_;
  dev(src_g, "src_g", at::kLong);
  dev(first, "first", at::kLong);
  dev(dst, "dst", at::kLong);
  dev(Hs, "Hs", at::kFloat);
  dev(Hd, "Hd", at::kFloat);
  dev(out_first, "out_first", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t G = src_g.numel();
  TORCH_CHECK_VALUE(K >= 0 && dst.numel() == G * K && out.numel() == G * K,
                    "sddmm_cos_grouped: dst and out must hold n_groups x K entries");
  TORCH_CHECK_VALUE(!has(first) || (first->numel() == G && out_first.numel() == G),
                    "sddmm_cos_grouped: first and out_first must hold n_groups entries");
  TORCH_CHECK_VALUE(Hs.size(1) == Hd.size(1), "endpoint feature sizes differ");
  TORCH_CHECK_VALUE(src_g.is_contiguous() && dst.is_contiguous() &&
                        (!has(first) || first->is_contiguous()) && out.is_contiguous() &&
                        out_first.is_contiguous(),
                    "sddmm_cos_grouped: contiguous ids and outputs");
  const int64_t lds = ld(Hs, "Hs"), ldd = ld(Hd, "Hd");
  if (meta(Hs)) return;
  const c10::DeviceGuard g(Hs.device());
  ck(gnnrec_sddmm_cos_grouped_f32(p<int64_t>(src_g), G, p<int64_t>(first), p<float>(out_first),
                                  K, p<int64_t>(dst), p<float>(out), p<float>(Hs), lds,
                                  p<float>(Hd), ldd, Hs.size(1), stream_of(Hs)),
     "gnnrec_sddmm_cos_grouped_f32");
}

// groups > 0: the grouped layout of gnnrec_sddmm_cos_backward_grouped_f32 (K negatives per
// positive, E = groups (K + 1))
void sddmm_cos_backward(const Tensor& src, const Tensor& dst, const Tensor& Hs, const Tensor& Hd,
                        const Tensor& grad, const optional<Tensor>& gHs,
                        const optional<Tensor>& gHd, Tensor& ws, int64_t groups, int64_t K) {
  const OneDevice one_device_;
  dev(src, "src", at::kLong);
  dev(dst, "dst", at::kLong);
  dev(Hs, "Hs", at::kFloat);
  dev(Hd, "Hd", at::kFloat);
  dev(grad, "grad", at::kFloat);
  dev(gHs, "gHs", at::kFloat);
  dev(gHd, "gHd", at::kFloat);
  // grouped (groups > 0): src may hold only the positives' sources (the only entries read)
  const int64_t E = dst.numel(), d = Hs.size(1);
  TORCH_CHECK_VALUE((src.numel() == E || (groups > 0 && src.numel() == groups)) &&
                        grad.numel() == E,
                    "src/dst/grad length mismatch");
  TORCH_CHECK_VALUE(Hd.size(1) == d, "endpoint feature sizes differ");
  TORCH_CHECK_VALUE(groups <= 0 || (K >= 0 && groups * (K + 1) == E),
                    "sddmm_cos_backward: groups x (K + 1) must equal the edge count");
  const int64_t lds = ld(Hs, "Hs"), ldd = ld(Hd, "Hd");
  if (meta(Hs)) return;
  const c10::DeviceGuard g(Hs.device());
  if (groups > 0) {
    ck(gnnrec_sddmm_cos_backward_grouped_f32(
           p<int64_t>(src), p<int64_t>(dst), groups, K, p<float>(Hs), lds, Hs.size(0),
           p<float>(Hd), ldd, Hd.size(0), d, p<float>(grad), p<float>(gHs), p<float>(gHd),
           ws.data_ptr(), ws.nbytes(), stream_of(Hs)),
       "gnnrec_sddmm_cos_backward_grouped_f32");
    return;
  }
  ck(gnnrec_sddmm_cos_backward_f32(p<int64_t>(src), p<int64_t>(dst), E, p<float>(Hs), lds,
                                   Hs.size(0), p<float>(Hd), ldd, Hd.size(0), d, p<float>(grad),
                                   p<float>(gHs), p<float>(gHd), ws.data_ptr(), ws.nbytes(),
                                   stream_of(Hs)),
     "gnnrec_sddmm_cos_backward_f32");
}

void edge_mlp(const Tensor& src, const Tensor& dst, const Tensor& P, const Tensor& Q,
              const Tensor& W2, const Tensor& b2, const Tensor& w3, const Tensor& b3,
              Tensor& out) {
  const OneDevice one_device_;
  dev(src, "src", at::kLong);
  dev(dst, "dst", at::kLong);
  for (auto* t : {&P, &Q, &W2, &b2, &w3, &b3}) dev(*t, "edge_mlp operand", at::kFloat);
  dev(out, "out", at::kFloat);
  TORCH_CHECK_VALUE(P.size(1) == 128 && Q.size(1) == 128 && W2.size(0) == 32 && W2.size(1) == 128,
                    "edge_mlp expects the reference's 128/32 hidden sizes");
  TORCH_CHECK_VALUE(P.is_contiguous() && Q.is_contiguous() && W2.is_contiguous(),
                    "edge_mlp operands must be contiguous");
  const int64_t E = src.numel();
  TORCH_CHECK_VALUE(dst.numel() == E && out.numel() == E, "src/dst/out length mismatch");
  if (meta(P)) return;
  const c10::DeviceGuard g(P.device());
  ck(gnnrec_edge_mlp_f32(p<int64_t>(src), p<int64_t>(dst), E, p<float>(P), p<float>(Q),
                         p<float>(W2), p<float>(b2), p<float>(w3), p<float>(b3), p<float>(out),
                         stream_of(P)),
     "gnnrec_edge_mlp_f32");
}

void edge_mlp_grouped(const Tensor& src_g, const optional<Tensor>& first, int64_t K,
                      const Tensor& dst, const Tensor& P, const Tensor& Q, const Tensor& W2,
                      const Tensor& b2, const Tensor& w3, const Tensor& b3, Tensor& out_first,
                      Tensor& out) {
  const OneDevice one_device_;
  dev(src_g, "src_g", at::kLong);
  dev(first, "first", at::kLong);
  dev(dst, "dst", at::kLong);
  for (auto* t : {&P, &Q, &W2, &b2, &w3, &b3}) dev(*t, "edge_mlp operand", at::kFloat);
  dev(out_first, "out_first", at::kFloat);
  dev(out, "out", at::kFloat);
  TORCH_CHECK_VALUE(P.size(1) == 128 && Q.size(1) == 128 && W2.size(0) == 32 && W2.size(1) == 128,
                    "edge_mlp expects the reference's 128/32 hidden sizes");
  TORCH_CHECK_VALUE(P.is_contiguous() && Q.is_contiguous() && W2.is_contiguous(),
                    "edge_mlp operands must be contiguous");
  const int64_t G = src_g.numel();
  TORCH_CHECK_VALUE(K >= 0 && dst.numel() == G * K && out.numel() == G * K,
                    "edge_mlp_grouped: dst and out must hold n_groups x K entries");
  TORCH_CHECK_VALUE(!has(first) || (first->numel() == G && out_first.numel() == G),
                    "edge_mlp_grouped: first and out_first must hold n_groups entries");
  TORCH_CHECK_VALUE(src_g.is_contiguous() && dst.is_contiguous() &&
                        (!has(first) || first->is_contiguous()) && out.is_contiguous() &&
                        out_first.is_contiguous(),
                    "edge_mlp_grouped: contiguous ids and outputs");
  if (meta(P)) return;
  const c10::DeviceGuard g(P.device());
  ck(gnnrec_edge_mlp_grouped_f32(p<int64_t>(src_g), G, p<int64_t>(first), p<float>(out_first), K,
                                 p<int64_t>(dst), p<float>(out), p<float>(P), p<float>(Q),
                                 p<float>(W2), p<float>(b2), p<float>(w3), p<float>(b3),
                                 stream_of(P)),
     "gnnrec_edge_mlp_grouped_f32");
}

// ---------------------------------------------------------------- a9 sampler / relabel
// excluded_rows flags one byte per destination row (the kernels index it by the seed's global
// id) and only narrows the exclusion: it means nothing without the eid mask
void check_excluded_rows(const Tensor& indptr, const optional<Tensor>& excluded,
                         const optional<Tensor>& excluded_rows) {
  if (!has(excluded_rows)) return;
  TORCH_CHECK_VALUE(has(excluded), "excluded_rows given without the excluded eid mask");
  TORCH_CHECK_VALUE(excluded_rows->numel() >= indptr.numel() - 1,
                    "excluded_rows must hold one flag per destination row (",
                    indptr.numel() - 1, "), got ", excluded_rows->numel());
}

void sample_count(const Tensor& indptr, const Tensor& eids, const optional<Tensor>& excluded,
                  const Tensor& seeds, int64_t fanout, int64_t seed_key, Tensor& counts,
                  const optional<Tensor>& excluded_rows) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(eids, "eids", at::kLong);
  dev(excluded, "excluded", at::kByte);
  dev(excluded_rows, "excluded_rows", at::kByte);
  dev(seeds, "seeds", at::kLong);
  dev(counts, "counts", at::kLong);
  TORCH_CHECK_VALUE(counts.numel() >= seeds.numel(), "counts shorter than seeds");
  check_excluded_rows(indptr, excluded, excluded_rows);
  if (meta(seeds)) return;
  const c10::DeviceGuard g(seeds.device());
  ck(gnnrec_sample_count(p<int64_t>(indptr), p<int64_t>(eids), p<uint8_t>(excluded),
                         p<uint8_t>(excluded_rows), p<int64_t>(seeds), seeds.numel(), fanout,
                         (uint64_t)seed_key,
                         p<int64_t>(counts), stream_of(seeds)),
     "gnnrec_sample_count");
}

void sample_fill(const Tensor& indptr, const Tensor& indices, const Tensor& eids,
                 const optional<Tensor>& excluded, const Tensor& seeds, int64_t fanout,
                 int64_t seed_key, const Tensor& out_indptr, Tensor& out_src, Tensor& out_eid,
                 const optional<Tensor>& excluded_rows) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(eids, "eids", at::kLong);
  dev(excluded, "excluded", at::kByte);
  dev(excluded_rows, "excluded_rows", at::kByte);
  dev(seeds, "seeds", at::kLong);
  dev(out_indptr, "out_indptr", at::kLong);
  dev(out_src, "out_src", at::kLong);
  dev(out_eid, "out_eid", at::kLong);
  TORCH_CHECK_VALUE(out_indptr.numel() >= seeds.numel() + 1, "out_indptr shorter than seeds + 1");
  check_excluded_rows(indptr, excluded, excluded_rows);
  if (meta(seeds)) return;
  const c10::DeviceGuard g(seeds.device());
  ck(gnnrec_sample_fill(p<int64_t>(indptr), p<int32_t>(indices), p<int64_t>(eids),
                        p<uint8_t>(excluded), p<uint8_t>(excluded_rows), p<int64_t>(seeds),
                        seeds.numel(), fanout,
                        (uint64_t)seed_key, p<int64_t>(out_indptr), p<int64_t>(out_src),
                        p<int64_t>(out_eid), stream_of(seeds)),
     "gnnrec_sample_fill");
}

void exclusive_scan(const Tensor& x, Tensor& out, Tensor& ws) {
  const OneDevice one_device_;
  dev(out, "out", at::kLong);
  TORCH_CHECK_VALUE(x.is_cuda() || x.is_meta(), "x must be a HIP device tensor");
  TORCH_CHECK_VALUE(x.scalar_type() == at::kLong || x.scalar_type() == at::kInt,
                    "exclusive_scan supports int32/int64");
  TORCH_CHECK_VALUE(x.is_contiguous() && out.numel() == x.numel() + 1,
                    "exclusive_scan: contiguous x [n] and out [n+1]");
  if (meta(x)) return;
  const c10::DeviceGuard g(x.device());
  if (x.scalar_type() == at::kLong)
    ck(gnnrec_exclusive_scan_i64(p<int64_t>(x), x.numel(), p<int64_t>(out), ws.data_ptr(),
                                 stream_of(x)),
       "gnnrec_exclusive_scan_i64");
  else
    ck(gnnrec_exclusive_scan_i32(p<int32_t>(x), x.numel(), p<int64_t>(out), ws.data_ptr(),
                                 stream_of(x)),
       "gnnrec_exclusive_scan_i32");
}

void mark_ids(const Tensor& ids, const Tensor& prefix_pos, Tensor& mark) {
  const OneDevice one_device_;
  dev(ids, "ids", at::kLong);
  dev(prefix_pos, "prefix_pos", at::kLong);
  dev(mark, "mark", at::kInt);
  if (meta(ids)) return;
  const c10::DeviceGuard g(ids.device());
  ck(gnnrec_mark_ids(p<int64_t>(ids), ids.numel(), p<int64_t>(prefix_pos), p<int32_t>(mark),
                     stream_of(ids)),
     "gnnrec_mark_ids");
}

void relabel_ids(const Tensor& ids, const Tensor& prefix_pos, const Tensor& rank, int64_t n_prefix,
                 Tensor& local) {
  const OneDevice one_device_;
  dev(ids, "ids", at::kLong);
  dev(prefix_pos, "prefix_pos", at::kLong);
  dev(rank, "rank", at::kLong);
  dev(local, "local", at::kLong);
  TORCH_CHECK_VALUE(local.numel() >= ids.numel(), "local shorter than ids");
  if (meta(ids)) return;
  const c10::DeviceGuard g(ids.device());
  ck(gnnrec_relabel_ids(p<int64_t>(ids), ids.numel(), p<int64_t>(prefix_pos), p<int64_t>(rank),
                        n_prefix, p<int64_t>(local), stream_of(ids)),
     "gnnrec_relabel_ids");
}

void compact_marked(const Tensor& mark, const Tensor& rank, Tensor& out_ids) {
  const OneDevice one_device_;
  dev(mark, "mark", at::kInt);
  dev(rank, "rank", at::kLong);
  dev(out_ids, "out_ids", at::kLong);
  if (meta(mark)) return;
  const c10::DeviceGuard g(mark.device());
  ck(gnnrec_compact_marked(p<int32_t>(mark), p<int64_t>(rank), mark.numel(), p<int64_t>(out_ids),
                           stream_of(mark)),
     "gnnrec_compact_marked");
}

void set_prefix_pos(const Tensor& prefix, Tensor& prefix_pos) {
  const OneDevice one_device_;
  dev(prefix, "prefix", at::kLong);
  dev(prefix_pos, "prefix_pos", at::kLong);
  if (meta(prefix)) return;
  const c10::DeviceGuard g(prefix.device());
  ck(gnnrec_set_prefix_pos(p<int64_t>(prefix), prefix.numel(), p<int64_t>(prefix_pos),
                           stream_of(prefix)),
     "gnnrec_set_prefix_pos");
}

void clear_prefix_pos(const Tensor& prefix, Tensor& prefix_pos) {
  const OneDevice one_device_;
  dev(prefix, "prefix", at::kLong);
  dev(prefix_pos, "prefix_pos", at::kLong);
  if (meta(prefix)) return;
  const c10::DeviceGuard g(prefix.device());
  ck(gnnrec_clear_prefix_pos(p<int64_t>(prefix), prefix.numel(), p<int64_t>(prefix_pos),
                             stream_of(prefix)),
     "gnnrec_clear_prefix_pos");
}

// ---------------------------------------------------------------- f1 top-k
void topk_rows(const Tensor& scores, int64_t k, const optional<Tensor>& exclude_indptr,
               const optional<Tensor>& exclude_indices, Tensor& out_vals, Tensor& out_idx) {
  const OneDevice one_device_;
  dev(scores, "scores", at::kFloat);
  dev(exclude_indptr, "exclude_indptr", at::kLong);
  dev(exclude_indices, "exclude_indices", at::kLong);
  dev(out_vals, "out_vals", at::kFloat);
  dev(out_idx, "out_idx", at::kLong);
  const int64_t n_rows = scores.size(0), n_cols = scores.size(1);
  TORCH_CHECK_VALUE(out_vals.numel() == n_rows * k && out_idx.numel() == n_rows * k,
                    "out_vals / out_idx must be [n_rows, k]");
  const int64_t lds = ld(scores, "scores");
  if (meta(scores)) return;
  const c10::DeviceGuard g(scores.device());
  ck(gnnrec_topk_rows_f32(p<float>(scores), lds, n_rows, n_cols, k, p<int64_t>(exclude_indptr),
                          p<int64_t>(exclude_indices), p<float>(out_vals), p<int64_t>(out_idx),
                          stream_of(scores)),
     "gnnrec_topk_rows_f32");
}

// ---------------------------------------------------------------- f2 training
void gemm_tn(const Tensor& A, const Tensor& B, const optional<Tensor>& colsum, bool accumulate,
             Tensor& out, Tensor& ws, const optional<Tensor>& row_ptr) {
  const OneDevice one_device_;
  dev(A, "A", at::kFloat);
  dev(B, "B", at::kFloat);
  dev(colsum, "colsum", at::kFloat);
  dev(out, "out", at::kFloat);
  dev(row_ptr, "row_ptr", at::kLong);
  const int64_t K = A.size(0), M = A.size(1), N = B.size(1);
  TORCH_CHECK_VALUE(B.size(0) == K, "gemm_tn: A and B differ in K");
  TORCH_CHECK_VALUE(out.size(0) == M && out.size(1) == N, "out must be [", M, ", ", N, "]");
  TORCH_CHECK_VALUE(!has(row_ptr) || (has(colsum) && row_ptr->numel() == K + 1 &&
                                      row_ptr->is_contiguous()),
                    "gemm_tn: row_ptr must be a contiguous [", K + 1, "] indptr beside colsum");
  const int64_t lda = ld(A, "A"), ldb = ld(B, "B"), ldc = ld(out, "out");
  if (meta(A)) return;
  const c10::DeviceGuard g(A.device());
  ck(gnnrec_gemm_tn_bias_rows_f32(p<float>(A), lda, p<float>(B), ldb, K, M, N, p<float>(out),
                                  ldc, p<float>(colsum), p<int64_t>(row_ptr), (int)accumulate,
                                  p<float>(ws), stream_of(A)),
     "gnnrec_gemm_tn_bias_rows_f32");
}

void act_backward(const Tensor& u, const Tensor& gz, int64_t flags, Tensor& out) {
  const OneDevice one_device_;
  dev(u, "u", at::kFloat);
  dev(gz, "gz", at::kFloat);
  dev(out, "out", at::kFloat);
  TORCH_CHECK_VALUE(u.sizes() == gz.sizes() && u.sizes() == out.sizes(),
                    "act_backward: u / gz / out shapes differ");
  const int64_t ldu = ld(u, "u"), ldg = ld(gz, "gz"), ldo = ld(out, "out");
  if (meta(u)) return;
  const c10::DeviceGuard g(u.device());
  ck(gnnrec_act_backward_f32(p<float>(u), ldu, p<float>(gz), ldg, u.size(0), u.size(1),
                             (int)flags, p<float>(out), ldo, stream_of(u)),
     "gnnrec_act_backward_f32");
}

void act_backward_normed(const Tensor& z, const Tensor& row_norm, const Tensor& gz, bool relu,
                         Tensor& out) {
  const OneDevice one_device_;
  dev(z, "z", at::kFloat);
  dev(row_norm, "row_norm", at::kFloat);
  dev(gz, "gz", at::kFloat);
  dev(out, "out", at::kFloat);
  TORCH_CHECK_VALUE(z.sizes() == gz.sizes() && z.sizes() == out.sizes() &&
                        row_norm.numel() == z.size(0) && row_norm.is_contiguous(),
                    "act_backward_normed: shape mismatch");
  const int64_t ldz = ld(z, "z"), ldg = ld(gz, "gz"), ldo = ld(out, "out");
  if (meta(z)) return;
  const c10::DeviceGuard g(z.device());
  ck(gnnrec_act_backward_normed_f32(p<float>(z), ldz, p<float>(row_norm), p<float>(gz), ldg,
                                    z.size(0), z.size(1), (int)relu, p<float>(out), ldo,
                                    stream_of(z)),
     "gnnrec_act_backward_normed_f32");
}

void csr_transpose(const Tensor& indptr, const Tensor& indices, const optional<Tensor>& ew,
                   int64_t n_src, int64_t n_edges, bool mean, Tensor& ws, Tensor& indptr_t,
                   Tensor& indices_t, const optional<Tensor>& ew_t) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(ew, "edge_weight", at::kFloat);
  dev(indptr_t, "indptr_t", at::kLong);
  dev(indices_t, "indices_t", at::kInt);
  dev(ew_t, "ew_t", at::kFloat);
  TORCH_CHECK_VALUE(indices.numel() >= n_edges, "csr_transpose: indices shorter than the edge count");
  TORCH_CHECK_VALUE(indptr_t.numel() == n_src + 1 && indices_t.numel() >= n_edges,
                    "csr_transpose: output sizes");
  if (meta(indptr)) return;
  const c10::DeviceGuard g(indptr.device());
  ck(gnnrec_csr_transpose(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ew),
                          indptr.numel() - 1, n_src, n_edges, (int)mean, ws.data_ptr(), ws.nbytes(),
                          p<int64_t>(indptr_t), p<int32_t>(indices_t), p<float>(ew_t),
                          stream_of(indptr)),
     "gnnrec_csr_transpose");
}

void csr_from_keys(const Tensor& keys, int64_t n_rows, Tensor& ws, Tensor& indptr, Tensor& perm) {
  const OneDevice one_device_;
  dev(keys, "keys", at::kInt);
  dev(indptr, "indptr", at::kLong);
  dev(perm, "perm", at::kInt);
  TORCH_CHECK_VALUE(keys.is_contiguous() && indptr.numel() == n_rows + 1 &&
                        perm.numel() == keys.numel(),
                    "csr_from_keys: output sizes");
  if (meta(keys)) return;
  const c10::DeviceGuard g(keys.device());
  ck(gnnrec_csr_from_keys(p<int32_t>(keys), keys.numel(), n_rows, ws.data_ptr(), ws.nbytes(),
                          p<int64_t>(indptr), p<int32_t>(perm), stream_of(keys)),
     "gnnrec_csr_from_keys");
}

// ---------------------------------------------------------------- f3 graph construction
void csr_build(const Tensor& src, const Tensor& dst, int64_t n_dst, Tensor& ws, Tensor& indptr,
               Tensor& indices, Tensor& eids) {
  const OneDevice one_device_;
  dev(src, "src", at::kLong);
  dev(dst, "dst", at::kLong);
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(eids, "eids", at::kLong);
  const int64_t E = dst.numel();
  TORCH_CHECK_VALUE(src.numel() == E && src.is_contiguous() && dst.is_contiguous(),
                    "csr_build: src and dst must be contiguous 1-D tensors of one length");
  TORCH_CHECK_VALUE(indptr.numel() == n_dst + 1 && indices.numel() == E && eids.numel() == E,
                    "csr_build: output sizes");
  if (meta(dst)) return;
  const c10::DeviceGuard g(dst.device());
  ck(gnnrec_csr_build(p<int64_t>(src), p<int64_t>(dst), E, n_dst, ws.data_ptr(), ws.nbytes(),
                      p<int64_t>(indptr), p<int32_t>(indices), p<int64_t>(eids), stream_of(dst)),
     "gnnrec_csr_build");
}

// ---------------------------------------------------------------- f2 fused relation
// One ConvLayer relation of a TRAINING step (sum / mean aggregation), forward and backward
// each as ONE dispatcher call that issues every launch from C++ (gnnrec/autograd.py
// SageRelFn): the per-launch Python wrappers and the second autograd node per relation were
// most of the C2 step's host time (profiles/r03_c2_step_probe.txt).  Same kernels, same
// order, same values as SpmmFn + SageProjectFn.
//   forward:  agg = spmm(indptr, indices, m, reduce, ew); z = norm?(relu(h_self[:M] Wsᵀ +
//             agg Wnᵀ)) with the row norms kept (norm, N <= 256) -> (z, agg, row_norm)
//   backward: gu = the ReLU / norm Jacobian applied to gz; g_self = gu Ws (whole table,
//             zero past M); g_m = transposed gather of gu Wn over the source-major CSR (the
//             mean's 1/deg folded into the edge weights); g_Ws = guᵀ h_self; g_Wn = guᵀ agg
namespace {
constexpr int64_t kSplit = 2048;  // ops.DEFAULT_SPLIT: heavy rows of the transposed gather

float* pw(const Tensor& t) { return t.defined() ? p<float>(t) : nullptr; }

Tensor gemm_nt(const Tensor& A, const Tensor& W, const Tensor* A2, const Tensor* W2, int epi,
               Tensor out, Tensor* row_norm, int accum = GNNREC_ACC_STORE,
               const float* bias = nullptr, const float* bias_ne = nullptr,
               const int32_t* a2_deg = nullptr, int a2_mode = GNNREC_A2_NONE) {
  const int64_t M = A.size(0), K1 = A.size(1), N = W.size(0);
  const int64_t K2 = A2 ? A2->size(1) : 0;
  ck(gnnrec_gemm_rownorm_f32(p<float>(A), ld(A, "A"), K1, p<float>(W), A2 ? p<float>(*A2) : nullptr,
                             A2 ? ld(*A2, "A2") : 1, K2, W2 ? p<float>(*W2) : nullptr, a2_deg,
                             a2_mode, bias, bias_ne, M, N, epi, accum, 0.f,
                             nullptr, nullptr, p<float>(out), ld(out, "out"),
                             row_norm ? p<float>(*row_norm) : nullptr, stream_of(A)),
     "gnnrec_gemm_f32");
  return out;
}

// guᵀ X, split-K MFMA; colsum (nullable, [M]) receives Σ_k gu[k] from the same pass — over
// the rows with row_ptr[k+1] > row_ptr[k] only, when row_ptr is given
Tensor weight_grad(const Tensor& gu, const Tensor& X, Tensor* colsum = nullptr,
                   const Tensor* row_ptr = nullptr) {
  const int64_t K = gu.size(0), M = gu.size(1), N = X.size(1);
  Tensor out = at::empty({M, N}, gu.options());
  const int64_t wsb = gnnrec_gemm_tn_workspace_bytes(K, M, N);
  Tensor ws = at::empty({std::max<int64_t>(wsb / 4, 1)}, gu.options());
  ck(gnnrec_gemm_tn_bias_rows_f32(p<float>(gu), ld(gu, "gu"), p<float>(X), ld(X, "X"), K, M, N,
                                  p<float>(out), ld(out, "out"),
                                  colsum ? p<float>(*colsum) : nullptr,
                                  row_ptr ? p<int64_t>(*row_ptr) : nullptr, 0, p<float>(ws),
                                  stream_of(gu)),
     "gnnrec_gemm_tn_bias_rows_f32");
  return out;
}

// int32 in-degrees of a CSR's rows (the GEMM epilogue's non-empty test for bias_nonempty)
Tensor row_degrees(const Tensor& indptr) {
  const int64_t M = indptr.numel() - 1;
  return (indptr.narrow(0, 1, M) - indptr.narrow(0, 0, M)).to(at::kInt).contiguous();
}

// gather of X over a CSR whose edge count is known on the host but whose degrees are
// not (the transposed block, a static-shape block's dump row): heavy rows planned on the
// device, as ops.spmm does
void gather_planned(const Tensor& ip, const Tensor& ix, const Tensor& w, const Tensor& X,
                    int64_t nnz, Tensor& out, bool accumulate = false,
                    int reduce = GNNREC_REDUCE_SUM, const int64_t* live = nullptr) {
  const int64_t n = ip.numel() - 1, d = X.size(1);
  const int64_t cap_h = std::min<int64_t>(n, nnz / (kSplit + 1));
  void* s = stream_of(X);
  const int flags = accumulate ? GNNREC_SPMM_ACCUM : 0;
  if (cap_h <= 0) {
    ck(gnnrec_spmm_csr_live_f32(p<int64_t>(ip), p<int32_t>(ix), pw(w), p<float>(X), ld(X, "X"), n,
                                d, reduce, flags, p<float>(out), ld(out, "out"), live, s),
       "gnnrec_spmm_csr_f32");
    return;
  }
  const int64_t cap_c = nnz / kSplit + cap_h;
  Tensor plan = at::empty({2 + cap_h + cap_h + 1 + cap_c}, ip.options());
  ck(gnnrec_spmm_plan_build_live(p<int64_t>(ip), n, kSplit, cap_h, cap_c, p<int64_t>(plan), live,
                                 s),
     "gnnrec_spmm_plan_build");
  Tensor wsp = at::empty({cap_c, d}, X.options());
  ck(gnnrec_spmm_csr_planned_live_f32(p<int64_t>(ip), p<int32_t>(ix), pw(w), p<float>(X),
                                      ld(X, "X"), n, d, reduce, flags, p<float>(out),
                                      ld(out, "out"), kSplit, p<int64_t>(plan), cap_h, cap_c,
                                      p<float>(wsp), live, s),
     "gnnrec_spmm_csr_planned_f32");
}
}  // namespace

std::tuple<Tensor, Tensor, Tensor> sage_rel_forward(const Tensor& m, const Tensor& h_self,
                                                    int64_t n_self, const Tensor& Ws,
                                                    const Tensor& Wn, const Tensor& indptr,
                                                    const Tensor& indices,
                                                    const optional<Tensor>& ew, int64_t reduce,
                                                    bool norm, const optional<Tensor>& bias,
                                                    const optional<Tensor>& bias_ne,
                                                    const optional<Tensor>& live) {
  const OneDevice one_device_;
  dev(m, "m", at::kFloat);
  dev(h_self, "h_self", at::kFloat);
  dev(Ws, "W_self", at::kFloat);
  dev(Wn, "W_neigh", at::kFloat);
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(ew, "edge_weight", at::kFloat);
  TORCH_CHECK_VALUE(reduce == GNNREC_REDUCE_SUM || reduce == GNNREC_REDUCE_MEAN,
                    "sage_rel_forward: sum or mean");
  const int64_t M = indptr.numel() - 1, N = Ws.size(0);
  TORCH_CHECK_VALUE(N <= 256 || !norm, "sage_rel_forward: the row norm needs N <= 256");
  TORCH_CHECK_VALUE(h_self.size(0) >= M && (n_self == 0 || n_self == M),
                    "sage_rel_forward: h_self must hold the ", M, " destination rows first");
  TORCH_CHECK_VALUE(Wn.size(0) == N && Ws.size(1) == h_self.size(1) && Wn.size(1) == m.size(1),
                    "sage_rel_forward: weight shapes");
  // bias (every row) and bias_ne (rows with an in-edge): a NodeEmbedding folded into the
  // layer (autograd.HeteroSageFn's first-layer fold): W_self b_e and W_neigh b_e
  dev(bias, "bias", at::kFloat);
  dev(bias_ne, "bias_nonempty", at::kFloat);
  TORCH_CHECK_VALUE((!has(bias) || bias->numel() == N) && (!has(bias_ne) || bias_ne->numel() == N),
                    "sage_rel_forward: biases must have ", N, " entries");
  const Tensor X = m.contiguous(), H = h_self.narrow(0, 0, M).contiguous();
  const Tensor bc = has(bias) ? bias->contiguous() : Tensor();
  const Tensor bnc = has(bias_ne) ? bias_ne->contiguous() : Tensor();
  const optional<Tensor> ewc = has(ew) ? optional<Tensor>(ew->contiguous()) : ew;
  const Tensor Wsc = Ws.contiguous(), Wnc = Wn.contiguous();
  Tensor agg = at::empty({M, m.size(1)}, m.options());
  Tensor z = at::empty({M, N}, m.options());
  Tensor nrm = norm ? at::empty({M}, m.options()) : at::empty({0}, m.options());
  if (meta(m)) return {z, agg, nrm};
  const c10::DeviceGuard g(m.device());
  // live: the static block's real destination count on the device (its padding and dump
  // rows aggregate nothing: their outputs feed no real row and get no gradient)
  // The forward blocks' rows are bounded (fanout rows; a static block's dump rows hold at
  // most kDumpEdges = the heavy-row split), so the gather needs no heavy-row plan; a
  // full-neighbour block's long rows run unsplit (one wave each, the same values)
  const int64_t* lv = live_ptr(live);
  ck(gnnrec_spmm_csr_live_f32(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ewc),
                              p<float>(X), ld(X, "m"), M, X.size(1), (int)reduce, 0,
                              p<float>(agg), ld(agg, "agg"), lv, stream_of(m)),
     "gnnrec_spmm_csr_f32");
  // bias_ne's non-empty test reads the block CSR's indptr directly (GNNREC_A2_DEG_INDPTR)
  const Tensor ipc = bnc.defined() ? indptr.contiguous() : Tensor();
  gemm_nt(H, Wsc, &agg, &Wnc, GNNREC_EPI_RELU | (norm ? GNNREC_EPI_L2NORM : 0), z,
          norm ? &nrm : nullptr, GNNREC_ACC_STORE, bc.defined() ? p<float>(bc) : nullptr,
          bnc.defined() ? p<float>(bnc) : nullptr,
          ipc.defined() ? reinterpret_cast<const int32_t*>(p<int64_t>(ipc)) : nullptr,
          ipc.defined() ? GNNREC_A2_DEG_INDPTR : GNNREC_A2_NONE);
  return {z, agg, nrm};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> sage_rel_backward(
    const Tensor& gz_in, const Tensor& z, const Tensor& row_norm, const Tensor& h_self,
    const Tensor& agg, const Tensor& Ws, const Tensor& Wn, const Tensor& indptr,
    const Tensor& indices, const optional<Tensor>& ew, int64_t reduce, int64_t n_src,
    int64_t nnz, bool norm, int64_t need, const optional<Tensor>& indptr_t_in,
    const optional<Tensor>& indices_t_in, const optional<Tensor>& w_mean_in,
    const optional<Tensor>& g_self_out, bool g_self_acc, const optional<Tensor>& g_m_out,
    bool g_m_acc, const optional<Tensor>& live_src) {
  // need bits: 1 g_self, 2 g_m, 4 g_Ws, 8 g_Wn, 16 g_bias (Σ rows of the pre-activation
  // gradient), 32 g_bias_nonempty (the same over rows with an in-edge)
  const OneDevice one_device_;
  dev(gz_in, "gz", at::kFloat);
  dev(z, "z", at::kFloat);
  dev(h_self, "h_self", at::kFloat);
  dev(agg, "agg", at::kFloat);
  dev(Ws, "W_self", at::kFloat);
  dev(Wn, "W_neigh", at::kFloat);
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(ew, "edge_weight", at::kFloat);
  const int64_t M = z.size(0), N = z.size(1);
  TORCH_CHECK_VALUE(gz_in.sizes() == z.sizes() && agg.size(0) == M && h_self.size(0) >= M &&
                        indptr.numel() == M + 1 && (!norm || row_norm.numel() == M),
                    "sage_rel_backward: shapes");
  const Tensor gz = gz_in.contiguous();
  // g_self_out / g_m_out: a layer's gradient tables (autograd.HeteroSageFn) written in place
  // — stored, or accumulated when *_acc — instead of fresh tensors that autograd then adds
  dev(g_self_out, "g_self_out", at::kFloat);
  dev(g_m_out, "g_m_out", at::kFloat);
  TORCH_CHECK_VALUE(!has(g_self_out) || (g_self_out->is_contiguous() &&
                                         g_self_out->size(0) == h_self.size(0) &&
                                         g_self_out->size(1) == Ws.size(1)),
                    "sage_rel_backward: g_self_out must be a contiguous [h_self rows, d_self]");
  TORCH_CHECK_VALUE(!has(g_m_out) || (g_m_out->is_contiguous() && g_m_out->size(0) == n_src &&
                                      g_m_out->size(1) == Wn.size(1)),
                    "sage_rel_backward: g_m_out must be a contiguous [n_src, d_neigh]");
  Tensor none = at::empty({0}, z.options());  // outputs not asked for (`need` bits)
  Tensor g_self = none, g_m = none, g_Ws = none, g_Wn = none, g_b = none, g_bne = none;
  if (meta(z)) {
    if ((need & 1) && !has(g_self_out)) g_self = at::empty({h_self.size(0), Ws.size(1)}, z.options());
    if ((need & 2) && !has(g_m_out)) g_m = at::empty({n_src, Wn.size(1)}, z.options());
    if (need & 4) g_Ws = at::empty_like(Ws);
    if (need & 8) g_Wn = at::empty_like(Wn);
    if (need & 16) g_b = at::empty({N}, z.options());
    if (need & 32) g_bne = at::empty({N}, z.options());
    return {g_self, g_m, g_Ws, g_Wn, g_b, g_bne};
  }
  const c10::DeviceGuard g(z.device());
  void* s = stream_of(z);
  Tensor gu = at::empty({M, N}, z.options());
  if (norm) {
    dev(row_norm, "row_norm", at::kFloat);
    ck(gnnrec_act_backward_normed_f32(p<float>(z), ld(z, "z"), p<float>(row_norm), p<float>(gz),
                                      ld(gz, "gz"), M, N, 1, p<float>(gu), N, s),
       "gnnrec_act_backward_normed_f32");
  } else {  // z = relu(u): the same mask
    ck(gnnrec_act_backward_f32(p<float>(z), ld(z, "z"), p<float>(gz), ld(gz, "gz"), M, N,
                               GNNREC_EPI_RELU, p<float>(gu), N, s),
       "gnnrec_act_backward_f32");
  }
  if (need & 1) {  // gu Ws over the whole source table of the dst type (zero past M)
    const bool acc = has(g_self_out) && g_self_acc;
    g_self = has(g_self_out) ? *g_self_out : at::empty({h_self.size(0), Ws.size(1)}, z.options());
    Tensor head = g_self.narrow(0, 0, M);
    gemm_nt(gu, Ws.t().contiguous(), nullptr, nullptr, 0, head, nullptr,
            acc ? GNNREC_ACC_ADD : GNNREC_ACC_STORE);
    if (!acc && h_self.size(0) > M) g_self.narrow(0, M, h_self.size(0) - M).zero_();
  }
  if (need & 2) {  // transposed gather of g_agg = gu Wn (DGL: the backward of a gSpMM)
    Tensor g_agg = at::empty({M, Wn.size(1)}, z.options());
    gemm_nt(gu, Wn.t().contiguous(), nullptr, nullptr, 0, g_agg, nullptr);
    const bool mean = reduce == GNNREC_REDUCE_MEAN;
    Tensor ip_t, ix_t, w_t;
    if (has(indptr_t_in) && !has(ew)) {
      // the block's source-major CSR, built by the sampler (block_transposes) beside the
      // block itself: no sort on the training thread
      TORCH_CHECK_VALUE(indptr_t_in->numel() == n_src + 1 && has(indices_t_in) &&
                            (!mean || has(w_mean_in)),
                        "sage_rel_backward: precomputed transpose does not fit the block");
      ip_t = *indptr_t_in;
      ix_t = *indices_t_in;
      if (mean) w_t = *w_mean_in;
    } else {
      ip_t = at::empty({n_src + 1}, indptr.options());
      ix_t = at::empty({std::max<int64_t>(nnz, 1)}, indices.options());
      if (has(ew) || mean) w_t = at::empty({std::max<int64_t>(nnz, 1)}, z.options());
      const size_t wsb = gnnrec_csr_transpose_workspace_bytes(nnz, n_src);
      Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 1)},
                            indptr.options().dtype(at::kByte));
      const optional<Tensor> ewc = has(ew) ? optional<Tensor>(ew->contiguous()) : ew;
      ck(gnnrec_csr_transpose(p<int64_t>(indptr), p<int32_t>(indices), p<float>(ewc), M, n_src,
                              nnz, (int)mean, ws.data_ptr(), ws.nbytes(), p<int64_t>(ip_t),
                              p<int32_t>(ix_t), pw(w_t), s),
         "gnnrec_csr_transpose");
    }
    g_m = has(g_m_out) ? *g_m_out : at::empty({n_src, Wn.size(1)}, z.options());
    // live_src: the static block's real source count (its padding sources' gradient rows
    // are zero: only padding rows, whose gradient is zero, point at them)
    gather_planned(ip_t, ix_t, w_t, g_agg, nnz, g_m, has(g_m_out) && g_m_acc, GNNREC_REDUCE_SUM,
                   live_ptr(live_src));
  }
  if (need & 16) g_b = at::empty({N}, z.options());
  if (need & 4) {
    g_Ws = weight_grad(gu, h_self.narrow(0, 0, M).contiguous(), (need & 16) ? &g_b : nullptr);
  } else if (need & 16) {
    g_b = gu.sum(0);
  }
  // g_bne: Σ over the rows with an in-edge (the mean of an empty set carries no bias), from
  // the W_neigh gradient's own pass over gu
  if (need & 32) g_bne = at::empty({N}, z.options());
  if (need & 8) {
    const Tensor ip = indptr.contiguous();
    g_Wn = weight_grad(gu, agg.contiguous(), (need & 32) ? &g_bne : nullptr,
                       (need & 32) ? &ip : nullptr);
  } else if (need & 32) {
    const Tensor ne = (row_degrees(indptr) > 0).to(gu.scalar_type()).unsqueeze(1);
    g_bne = (gu * ne).sum(0);
  }
  // gradients written in place come back as empty tensors (the caller holds the tables)
  return {has(g_self_out) ? none : g_self, has(g_m_out) ? none : g_m, g_Ws, g_Wn, g_b, g_bne};
}

// Every relation's source-major CSR of one sampled block, in one call (the sampler's
// training side, gnnrec/sampling.py): (indptr_t, dst rows, 1/deg(dst) per edge) per relation,
// the transposes the aggregation backward gathers over (sage_rel_backward).
std::tuple<std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>> block_transposes(
    at::TensorList indptrs, at::TensorList indices, at::IntArrayRef n_src,
    at::IntArrayRef nnz) {
  const OneDevice one_device_;
  const size_t R = indptrs.size();
  TORCH_CHECK_VALUE(indices.size() == R && n_src.size() == R && nnz.size() == R,
                    "block_transposes: one entry per relation");
  std::vector<Tensor> ips(R), ixs(R), ws_(R);
  for (size_t r = 0; r < R; ++r) {
    dev(indptrs[r], "indptr", at::kLong);
    dev(indices[r], "indices", at::kInt);
    const int64_t E = nnz[r], ns = n_src[r];
    TORCH_CHECK_VALUE(indices[r].numel() >= E && ns >= 0, "block_transposes: sizes");
    ips[r] = at::empty({ns + 1}, indptrs[r].options());
    ixs[r] = at::empty({std::max<int64_t>(E, 1)}, indices[r].options());
    ws_[r] = at::empty({std::max<int64_t>(E, 1)}, indptrs[r].options().dtype(at::kFloat));
    if (meta(indptrs[r])) continue;
    const c10::DeviceGuard g(indptrs[r].device());
    const size_t wsb = gnnrec_csr_transpose_workspace_bytes(E, ns);
    Tensor ws = at::empty({(int64_t)std::max<size_t>(wsb, 1)},
                          indptrs[r].options().dtype(at::kByte));
    ck(gnnrec_csr_transpose(p<int64_t>(indptrs[r]), p<int32_t>(indices[r]), nullptr,
                            indptrs[r].numel() - 1, ns, E, 1, ws.data_ptr(), ws.nbytes(),
                            p<int64_t>(ips[r]), p<int32_t>(ixs[r]), p<float>(ws_[r]),
                            stream_of(indptrs[r])),
       "gnnrec_csr_transpose");
  }
  return {ips, ixs, ws_};
}

// K10 membership: has_edges_between over a source-sorted in-CSR
void csr_has_edges(const Tensor& indptr, const Tensor& sorted_indices, int64_t n_src, const Tensor& u,
               const Tensor& v, Tensor& out) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(sorted_indices, "sorted_indices", at::kInt);
  dev(u, "u", at::kLong);
  dev(v, "v", at::kLong);
  dev(out, "out", at::kBool);
  const int64_t n = u.numel();
  TORCH_CHECK_VALUE(v.numel() == n && out.numel() == n && u.is_contiguous() && v.is_contiguous() &&
                        out.is_contiguous() && indptr.numel() >= 1,
                    "has_edges: contiguous u, v, out of one length and a non-empty indptr");
  if (meta(u)) return;
  const c10::DeviceGuard g(u.device());
  ck(gnnrec_csr_has_edges(p<int64_t>(indptr), p<int32_t>(sorted_indices), indptr.numel() - 1,
                          n_src, p<int64_t>(u), p<int64_t>(v), n,
                          reinterpret_cast<uint8_t*>(out.data_ptr()), stream_of(u)),
     "gnnrec_csr_has_edges");
}

// ---------------------------------------------------------------- sharded-pass helpers
void add_(Tensor& a, const Tensor& b) {
  const OneDevice one_device_;
  dev(a, "a", at::kFloat);
  dev(b, "b", at::kFloat);
  TORCH_CHECK_VALUE(a.sizes() == b.sizes() && a.is_contiguous() && b.is_contiguous(),
                    "add_: operands must be contiguous and of one shape");
  if (meta(a)) return;
  const c10::DeviceGuard g(a.device());
  ck(gnnrec_add_f32(p<float>(a), p<float>(b), p<float>(a), a.numel(), stream_of(a)),
     "gnnrec_add_f32");
}

void tree_sum_(Tensor& a, at::TensorList rest) {
  const OneDevice one_device_;
  dev(a, "part", at::kFloat);
  const int n = (int)rest.size() + 1;
  TORCH_CHECK_VALUE(n == 2 || n == 4 || n == 8, "tree_sum_: 2, 4 or 8 tables");
  TORCH_CHECK_VALUE(a.is_contiguous(), "tree_sum_: operands must be contiguous");
  for (const Tensor& t : rest) {
    dev(t, "part", at::kFloat);
    TORCH_CHECK_VALUE(t.sizes() == a.sizes() && t.is_contiguous(),
                      "tree_sum_: operands must be contiguous and of one shape");
  }
  if (meta(a)) return;
  std::vector<const float*> parts{p<float>(a)};
  for (const Tensor& t : rest) parts.push_back(p<float>(t));
  const c10::DeviceGuard g(a.device());
  ck(gnnrec_tree_sum_f32(parts.data(), n, a.numel(), p<float>(a), stream_of(a)),
     "gnnrec_tree_sum_f32");
}

// ---------------------------------------------------------------- f4 LSTM reducer
void lstm_step(const Tensor& P, const Tensor& indptr, const Tensor& indices, const Tensor& order,
               int64_t t, int64_t n_act, const Tensor& h_in, Tensor& h_out, Tensor& c,
               const Tensor& W_hhT, Tensor& out) {
  const OneDevice one_device_;
  dev(P, "P", at::kFloat);
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(order, "order", at::kLong);
  dev(h_in, "h_in", at::kFloat);
  dev(h_out, "h_out", at::kFloat);
  dev(c, "c", at::kFloat);
  dev(W_hhT, "W_hhT", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t d = h_in.size(1);
  TORCH_CHECK_VALUE(W_hhT.size(0) == d && W_hhT.size(1) == 4 * d && W_hhT.is_contiguous(),
                    "W_hhT must be a contiguous [d, 4d]");
  const int64_t ldp = ld(P, "P"), ldo = ld(out, "out");
  if (meta(P)) return;
  const c10::DeviceGuard g(P.device());
  ck(gnnrec_lstm_step_f32(p<float>(P), ldp, p<int64_t>(indptr), p<int32_t>(indices),
                          p<int64_t>(order), t, n_act, p<float>(h_in), p<float>(h_out),
                          p<float>(c), d, p<float>(W_hhT), p<float>(out), ldo, stream_of(P)),
     "gnnrec_lstm_step_f32");
}

// training: the step with its state kept (step-major packing), one step of BPTT, and the
// slots' source rows / previous-step slots (gnnrec_lstm_step_save_f32 & co., lstm.hip)
void lstm_step_save(const Tensor& P, const Tensor& indptr, const Tensor& indices,
                    const Tensor& order, int64_t t, int64_t n_act, const Tensor& h_in,
                    Tensor& h_out, const optional<Tensor>& c_in, Tensor& c_out, Tensor& z_out,
                    const Tensor& W_hhT, Tensor& out) {
  const OneDevice one_device_;
  dev(P, "P", at::kFloat);
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(order, "order", at::kLong);
  dev(h_in, "h_in", at::kFloat);
  dev(h_out, "h_out", at::kFloat);
  dev(c_in, "c_in", at::kFloat);
  dev(c_out, "c_out", at::kFloat);
  dev(z_out, "z_out", at::kFloat);
  dev(W_hhT, "W_hhT", at::kFloat);
  dev(out, "out", at::kFloat);
  const int64_t d = h_out.size(1);
  TORCH_CHECK_VALUE(W_hhT.size(0) == d && W_hhT.size(1) == 4 * d && W_hhT.is_contiguous(),
                    "W_hhT must be a contiguous [d, 4d]");
  for (const Tensor* x : std::initializer_list<const Tensor*>{&h_in, &h_out, &c_out})
    TORCH_CHECK_VALUE(x->is_contiguous() && x->dim() == 2 && x->size(0) >= n_act &&
                          x->size(1) == d,
                      "h_in / h_out / c_out must be contiguous [>= n_act, d]");
  TORCH_CHECK_VALUE(!has(c_in) || (c_in->is_contiguous() && c_in->size(0) >= n_act &&
                                   c_in->size(1) == d),
                    "c_in must be a contiguous [>= n_act, d]");
  TORCH_CHECK_VALUE(z_out.is_contiguous() && z_out.size(0) >= n_act && z_out.size(1) == 4 * d,
                    "z_out must be a contiguous [>= n_act, 4d]");
  TORCH_CHECK_VALUE(order.numel() >= n_act, "order shorter than n_act");
  const int64_t ldp = ld(P, "P"), ldo = ld(out, "out");
  if (meta(P)) return;
  const c10::DeviceGuard g(P.device());
  ck(gnnrec_lstm_step_save_f32(p<float>(P), ldp, p<int64_t>(indptr), p<int32_t>(indices),
                               p<int64_t>(order), t, n_act, p<float>(h_in), p<float>(h_out),
                               p<float>(c_in), p<float>(c_out), p<float>(z_out), d,
                               p<float>(W_hhT), p<float>(out), ldo, stream_of(P)),
     "gnnrec_lstm_step_save_f32");
}

void lstm_backward_step(const Tensor& z, const Tensor& c_t, const optional<Tensor>& c_prev,
                        const optional<Tensor>& dh_next, const optional<Tensor>& dc_next,
                        int64_t n_next, const Tensor& g_out, const Tensor& order, int64_t n_act,
                        Tensor& dz, Tensor& dc_prev) {
  const OneDevice one_device_;
  dev(z, "z", at::kFloat);
  dev(c_t, "c_t", at::kFloat);
  dev(c_prev, "c_prev", at::kFloat);
  dev(dh_next, "dh_next", at::kFloat);
  dev(dc_next, "dc_next", at::kFloat);
  dev(g_out, "g_out", at::kFloat);
  dev(order, "order", at::kLong);
  dev(dz, "dz", at::kFloat);
  dev(dc_prev, "dc_prev", at::kFloat);
  const int64_t d = c_t.size(1);
  TORCH_CHECK_VALUE(n_next >= 0 && n_next <= n_act && order.numel() >= n_act,
                    "lstm_backward_step: need 0 <= n_next <= n_act <= order.numel()");
  auto rows = [&](const Tensor& x, int64_t n, int64_t w, const char* name) {
    TORCH_CHECK_VALUE(x.is_contiguous() && x.dim() == 2 && x.size(0) >= n && x.size(1) == w,
                      name, ": expected a contiguous [>= ", n, ", ", w, "] tensor");
  };
  rows(z, n_act, 4 * d, "z");
  rows(c_t, n_act, d, "c_t");
  if (has(c_prev)) rows(*c_prev, n_act, d, "c_prev");
  TORCH_CHECK_VALUE(n_next == 0 || (has(dh_next) && has(dc_next)),
                    "lstm_backward_step: rows carried from step t+1 need dh_next and dc_next");
  if (n_next > 0) {
    rows(*dh_next, n_next, d, "dh_next");
    rows(*dc_next, n_next, d, "dc_next");
  }
  rows(dz, n_act, 4 * d, "dz");
  rows(dc_prev, n_act, d, "dc_prev");
  TORCH_CHECK_VALUE(g_out.dim() == 2 && g_out.size(1) == d && g_out.stride(1) == 1,
                    "g_out must be [n_dst, d] with unit column stride");
  if (meta(z)) return;
  const c10::DeviceGuard g(z.device());
  ck(gnnrec_lstm_backward_step_f32(p<float>(z), p<float>(c_t), p<float>(c_prev),
                                   p<float>(dh_next), p<float>(dc_next), n_next, p<float>(g_out),
                                   g_out.stride(0), p<int64_t>(order), n_act, d, p<float>(dz),
                                   p<float>(dc_prev), stream_of(z)),
     "gnnrec_lstm_backward_step_f32");
}

void lstm_slots(const Tensor& indptr, const Tensor& indices, const Tensor& order,
                const Tensor& step_off, int64_t n_slots, Tensor& src, Tensor& prev) {
  const OneDevice one_device_;
  dev(indptr, "indptr", at::kLong);
  dev(indices, "indices", at::kInt);
  dev(order, "order", at::kLong);
  dev(step_off, "step_off", at::kLong);
  dev(src, "src", at::kLong);
  dev(prev, "prev", at::kLong);
  TORCH_CHECK_VALUE(src.numel() >= n_slots && prev.numel() >= n_slots && step_off.dim() == 1,
                    "lstm_slots: src / prev shorter than n_slots");
  if (meta(indptr)) return;
  const c10::DeviceGuard g(indptr.device());
  ck(gnnrec_lstm_slots(p<int64_t>(indptr), p<int32_t>(indices), p<int64_t>(order),
                       p<int64_t>(step_off), step_off.numel(), n_slots, p<int64_t>(src),
                       p<int64_t>(prev), stream_of(indptr)),
     "gnnrec_lstm_slots");
}

// ---------------------------------------------------------------- a10 row gather
void gather_rows(const Tensor& src, const Tensor& idx, Tensor& out) {
  const OneDevice one_device_;
  dev(idx, "idx", at::kLong);
  TORCH_CHECK_VALUE(src.is_cuda() || src.is_meta(), "src: expected a device tensor (there is no CPU path)");
  same_dev(src, "src");
  same_dev(out, "out");
  TORCH_CHECK_VALUE(src.dim() >= 1 && out.dim() == src.dim() && out.scalar_type() == src.scalar_type(),
                    "gather_rows: out must match src's dtype and rank");
  TORCH_CHECK_VALUE(idx.is_contiguous() && out.size(0) == idx.numel() && out.is_contiguous(),
                    "gather_rows: contiguous idx [n] and out [n, ...]");
  const int64_t es = src.element_size();
  int64_t row_elems = 1;
  for (int64_t k = 1; k < src.dim(); ++k) {
    TORCH_CHECK_VALUE(out.size(k) == src.size(k), "gather_rows: row shapes differ");
    row_elems *= src.size(k);
  }
  // rows are copied as flat byte runs: within a row the elements must be contiguous
  int64_t inner = 1;
  for (int64_t k = src.dim() - 1; k >= 1; --k) {
    TORCH_CHECK_VALUE(src.size(k) <= 1 || src.stride(k) == inner,
                      "gather_rows: src rows must be contiguous (stride ", src.stride(k),
                      " in dim ", k, ")");
    inner *= src.size(k);
  }
  const int64_t row_bytes = es * row_elems;
  if (meta(src)) return;
  const c10::DeviceGuard g(src.device());
  ck(gnnrec_gather_rows(src.data_ptr(), src.stride(0) * es, p<int64_t>(idx), idx.numel(),
                        row_bytes, out.data_ptr(), row_bytes, stream_of(src)),
     "gnnrec_gather_rows");
}

// ---------------------------------------------------------------- f2 loss
void margin_loss(const Tensor& pos, const Tensor& neg, int64_t K, double delta,
                 const optional<Tensor>& mask, const optional<Tensor>& recency, Tensor& g_pos,
                 Tensor& g_neg, Tensor& partial) {
  const OneDevice one_device_;
  dev(pos, "pos_score", at::kFloat);
  dev(neg, "neg_score", at::kFloat);
  dev(mask, "negative_mask", at::kFloat);
  dev(g_pos, "g_pos", at::kFloat);
  dev(g_neg, "g_neg", at::kFloat);
  dev(partial, "partial", at::kFloat);
  const int64_t n_pos = pos.numel();
  TORCH_CHECK_VALUE(neg.numel() == n_pos * K, "neg must hold n_pos x K scores");
  TORCH_CHECK_VALUE(pos.is_contiguous() && neg.is_contiguous(), "scores must be contiguous");
  int rec_i64 = 0;
  if (has(recency)) {
    TORCH_CHECK_VALUE(recency->scalar_type() == at::kLong || recency->scalar_type() == at::kFloat,
                      "recency must be float32 or int64");
    rec_i64 = recency->scalar_type() == at::kLong;
  }
  if (meta(pos)) return;
  const c10::DeviceGuard g(pos.device());
  ck(gnnrec_margin_loss_f32(p<float>(pos), p<float>(neg), n_pos, K, (float)delta, p<float>(mask),
                            has(recency) ? recency->data_ptr() : nullptr, rec_i64, p<float>(g_pos),
                            p<float>(g_neg), p<float>(partial), partial.numel(), stream_of(pos)),
     "gnnrec_margin_loss_f32");
}

void sum_scaled(const Tensor& x, double scale, Tensor& out) {
  const OneDevice one_device_;
  dev(x, "x", at::kFloat);
  dev(out, "out", at::kFloat);
  if (meta(x)) return;
  const c10::DeviceGuard g(x.device());
  ck(gnnrec_sum_scaled_f32(p<float>(x), x.numel(), (float)scale, p<float>(out), stream_of(x)),
     "gnnrec_sum_scaled_f32");
}

// ---------------------------------------------------------------- synthetic generator
void synth_edges(int64_t seed, int64_t e0, int64_t n_u, int64_t n_i,
                 const optional<Tensor>& zipf_cdf, Tensor& u, Tensor& i) {
  const OneDevice one_device_;
  dev(zipf_cdf, "zipf_cdf", at::kDouble);
  dev(u, "u", at::kInt);
  dev(i, "i", at::kInt);
  TORCH_CHECK_VALUE(u.numel() == i.numel(), "u and i must have one length");
  if (meta(u)) return;
  const c10::DeviceGuard g(u.device());
  ck(gnnrec_synth_edges((uint64_t)seed, e0, u.numel(), n_u, n_i, p<double>(zipf_cdf),
                        p<int32_t>(u), p<int32_t>(i), stream_of(u)),
     "gnnrec_synth_edges");
}

void hold_cus(int64_t blocks, int64_t threads, int64_t lds_bytes, int64_t usec, Tensor& sink) {
  const OneDevice one_device_;
  dev(sink, "sink", at::kFloat);
  TORCH_CHECK_VALUE(sink.numel() >= threads, "sink must hold >= threads floats");
  if (meta(sink)) return;
  const c10::DeviceGuard g(sink.device());
  ck(gnnrec_hold_cus((int)blocks, (int)threads, (int)lds_bytes, usec, p<float>(sink),
                     stream_of(sink)),
     "gnnrec_hold_cus");
}

// ---------------------------------------------------------------- a9 one sampled layer
// The whole of one block layer of BlockSampler.sample_blocks (gnnrec/sampling.py) issued
// from C++: per relation count -> scan; ONE host read of the sampled edge counts; fills;
// per node type the to_block relabel (prefix map, marks of the new sources, scan); ONE
// host read of the new-source counts; compaction, relabel of every relation's sources,
// scratch reset.  The same kernels in the same order with the same keys as the Python
// form it replaces (bitwise the same blocks), minus ≈ 40 Python-level launches per layer
// (the C2 step's sampler spent 1.5 ms of host time per batch on them).
//   relations r: CSR (indptr, indices int32, eids), optional exclusion mask, source / dst
//   node-type index, fanout (-1 = all), RNG key; node types t: the seeds (dst prefix) and
//   the Relabeler scratch (prefix_pos int64 [n_t] = -1, mark int32 [n_t] = 0, restored on
//   exit).  Returns per relation (out indptr, local src int32, eids), per type the src
//   node ids (prefix first), and the edge counts.
Tensor exclusive_scan_new(const Tensor& x) {
  const OneDevice one_device_;
  const int64_t n = x.numel();
  Tensor out = at::empty({n + 1}, x.options().dtype(at::kLong));
  Tensor ws = at::empty({std::max<int64_t>(1, (gnnrec_scan_workspace_bytes(n) + 7) / 8)},
                        x.options().dtype(at::kLong));
  exclusive_scan(x, out, ws);
  return out;
}

std::tuple<std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>,
           std::vector<int64_t>>
sample_layer(at::TensorList indptrs, at::TensorList indices, at::TensorList eids,
             const c10::List<optional<Tensor>>& masks,
             const c10::List<optional<Tensor>>& mask_rows, at::IntArrayRef src_type,
             at::IntArrayRef dst_type, at::IntArrayRef fanouts, at::IntArrayRef keys,
             at::TensorList seeds, at::TensorList prefix_pos, at::TensorList marks) {
  const OneDevice one_device_;
  const size_t R = indptrs.size(), NT = seeds.size();
  TORCH_CHECK_VALUE(indices.size() == R && eids.size() == R && masks.size() == R &&
                        mask_rows.size() == R &&
                        src_type.size() == R && dst_type.size() == R && fanouts.size() == R &&
                        keys.size() == R,
                    "sample_layer: one entry per relation in every relation list");
  TORCH_CHECK_VALUE(prefix_pos.size() == NT && marks.size() == NT,
                    "sample_layer: one seed list and one scratch pair per node type");
  for (size_t r = 0; r < R; ++r)
    TORCH_CHECK_VALUE(src_type[r] >= 0 && (size_t)src_type[r] < NT && dst_type[r] >= 0 &&
                          (size_t)dst_type[r] < NT,
                      "sample_layer: node-type index out of range");
  TORCH_CHECK_VALUE(NT > 0, "sample_layer: no node types");
  const c10::DeviceGuard g(seeds[0].device());
  // Bounded fanouts (every relation samples at most fanout >= 0 in-edges per seed): the
  // fills write into capacity-sized buffers (seeds x fanout, unused tail = -1, which the
  // mark / relabel kernels skip) and the new-source scan runs before any size is known,
  // so the layer's edge counts and new-node counts come back in ONE readback.  Unbounded
  // (full-neighbour) layers read the edge counts first to size the fills (two readbacks).
  bool bounded = true;
  for (size_t r = 0; r < R; ++r) bounded = bounded && fanouts[r] >= 0;
  // counts -> out indptr per relation
  std::vector<Tensor> o_ip(R), o_src(R), o_eid(R), src_loc(R), src_nid(NT);
  for (size_t r = 0; r < R; ++r) {
    const Tensor& sd = seeds[dst_type[r]];
    Tensor counts = at::empty({sd.numel()}, sd.options().dtype(at::kLong));
    const optional<Tensor> m = masks.get(r);
    sample_count(indptrs[r], eids[r], m, sd, fanouts[r], keys[r], counts, mask_rows.get(r));
    o_ip[r] = exclusive_scan_new(counts);
  }
  std::vector<int64_t> totals(R, 0);
  auto read_totals = [&](std::vector<Tensor> extra) {  // one device -> host copy
    std::vector<Tensor> last;
    for (size_t r = 0; r < R; ++r) last.push_back(o_ip[r].narrow(0, o_ip[r].numel() - 1, 1));
    for (auto& t : extra) last.push_back(t);
    const Tensor t = at::cat(last).to(at::kCPU);
    for (size_t r = 0; r < R; ++r) totals[r] = t.data_ptr<int64_t>()[r];
    std::vector<int64_t> rest;
    for (size_t i = R; i < last.size(); ++i) rest.push_back(t.data_ptr<int64_t>()[i]);
    return rest;
  };
  if (R && !bounded) read_totals({});  // the unbounded layer's first readback
  for (size_t r = 0; r < R; ++r) {
    const Tensor& sd = seeds[dst_type[r]];
    const int64_t cap = bounded ? sd.numel() * fanouts[r] : totals[r];
    o_src[r] = bounded ? at::full({cap}, -1, sd.options().dtype(at::kLong))
                       : at::empty({cap}, sd.options().dtype(at::kLong));
    o_eid[r] = at::empty({cap}, sd.options().dtype(at::kLong));
    const optional<Tensor> m = masks.get(r);
    sample_fill(indptrs[r], indices[r], eids[r], m, sd, fanouts[r], keys[r], o_ip[r], o_src[r],
                o_eid[r], mask_rows.get(r));
  }
  // relabel: per node type, mark the new sources and scan
  std::vector<Tensor> rank(NT);
  for (size_t t = 0; t < NT; ++t) {
    Tensor pp = prefix_pos[t], mk = marks[t];
    set_prefix_pos(seeds[t], pp);
    for (size_t r = 0; r < R; ++r)
      if ((size_t)src_type[r] == t) mark_ids(o_src[r], pp, mk);
    rank[t] = exclusive_scan_new(mk);
  }
  // local source ids and (bounded) the fresh nodes, before any count is on the host
  std::vector<Tensor> nodes(NT);
  auto relabel_all = [&](size_t t) {
    Tensor pp = prefix_pos[t];
    const int64_t n_p = seeds[t].numel();
    for (size_t r = 0; r < R; ++r) {
      if ((size_t)src_type[r] != t) continue;
      Tensor loc = at::empty({o_src[r].numel()}, seeds[t].options().dtype(at::kLong));
      relabel_ids(o_src[r], pp, rank[t], n_p, loc);
      src_loc[r] = loc;
    }
  };
  std::vector<int64_t> n_new(NT, 0);
  if (bounded) {
    for (size_t t = 0; t < NT; ++t) {
      const Tensor& pre = seeds[t];
      const int64_t n_p = pre.numel();
      int64_t cap = 0;  // new sources of type t: at most the sampled edges from it
      for (size_t r = 0; r < R; ++r)
        if ((size_t)src_type[r] == t) cap += o_src[r].numel();
      cap = std::min(cap, marks[t].numel());
      nodes[t] = at::empty({n_p + cap}, pre.options().dtype(at::kLong));
      nodes[t].narrow(0, 0, n_p).copy_(pre);
      if (cap) {
        Tensor tail = nodes[t].narrow(0, n_p, cap);
        compact_marked(marks[t], rank[t], tail);
      }
      relabel_all(t);
    }
    std::vector<Tensor> last;
    for (size_t t = 0; t < NT; ++t) last.push_back(rank[t].narrow(0, rank[t].numel() - 1, 1));
    const std::vector<int64_t> nn = read_totals(last);  // the layer's one size readback
    for (size_t t = 0; t < NT; ++t) n_new[t] = nn[t];
    for (size_t r = 0; r < R; ++r) {
      o_src[r] = o_src[r].narrow(0, 0, totals[r]);
      o_eid[r] = o_eid[r].narrow(0, 0, totals[r]);
    }
  } else {
    std::vector<Tensor> last;
    for (size_t t = 0; t < NT; ++t) last.push_back(rank[t].narrow(0, rank[t].numel() - 1, 1));
    const Tensor c = at::cat(last).to(at::kCPU);  // the layer's second size readback
    for (size_t t = 0; t < NT; ++t) n_new[t] = c.data_ptr<int64_t>()[t];
    for (size_t t = 0; t < NT; ++t) {
      const Tensor& pre = seeds[t];
      const int64_t n_p = pre.numel();
      nodes[t] = at::empty({n_p + n_new[t]}, pre.options().dtype(at::kLong));
      nodes[t].narrow(0, 0, n_p).copy_(pre);
      if (n_new[t]) {
        Tensor fresh = nodes[t].narrow(0, n_p, n_new[t]);
        compact_marked(marks[t], rank[t], fresh);
      }
      relabel_all(t);
    }
  }
  for (size_t t = 0; t < NT; ++t) {
    const Tensor& pre = seeds[t];
    const int64_t n_p = pre.numel();
    Tensor fresh = nodes[t].narrow(0, n_p, n_new[t]);
    Tensor pp = prefix_pos[t], mk = marks[t];
    clear_prefix_pos(pre, pp);
    if (n_new[t]) mk.index_fill_(0, fresh, 0);
    src_nid[t] = bounded ? nodes[t].narrow(0, 0, n_p + n_new[t]) : nodes[t];
  }
  for (size_t r = 0; r < R; ++r)
    src_loc[r] = src_loc[r].narrow(0, 0, totals[r]).to(at::kInt);
  return {o_ip, src_loc, o_eid, src_nid, totals};
}

// ---------------------------------------------------------------- a9 fused sample_blocks
// Every block of one bounded-fanout BlockSampler.sample_blocks call (gnnrec_sample_blocks:
// 1 + 3L launches, include/gnnrec.h) with ONE host read of the sizes at the end: outputs are
// allocated at their capacities and returned narrowed to the actual sizes.
//   relations r: global in-CSR, src / dst type index, exclusion (eids, COO dst, flag arrays:
//   all four or none); types t: node count, step-0 seeds, scratch (pos int64 [2n], bits int64
//   [2 ceil(n/64)], word_rank int64 [ceil(n/64) + 1]); fanouts / keys flattened [step][r].
//   -> per step s and relation r (flattened [s][r]): out_indptr [n_dst + 1], local src int32,
//   eids; per step and type ([s][t]): the source node ids (seeds first); the sizes (node
//   counts rows -1..L-1 x T, then edge counts L x R).
std::tuple<std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>,
           std::vector<int64_t>, std::vector<Tensor>>
sample_blocks(at::TensorList indptrs, at::TensorList indices, at::TensorList eids,
              at::IntArrayRef src_type, at::IntArrayRef dst_type,
              const c10::List<optional<Tensor>>& excl_eids,
              const c10::List<optional<Tensor>>& coo_dst,
              const c10::List<optional<Tensor>>& excl_masks,
              const c10::List<optional<Tensor>>& excl_rows, at::IntArrayRef n_nodes,
              at::TensorList seeds, at::TensorList pos, at::TensorList bits,
              at::TensorList word_rank, at::TensorList marks, at::IntArrayRef fanouts,
              at::IntArrayRef keys, int64_t steps, int64_t stamp, bool static_shapes,
              const optional<Tensor>& sizes_out,
              at::IntArrayRef node_cap_hint, const optional<Tensor>& overflow,
              at::TensorList edge_tables, at::IntArrayRef edge_table_rel,
              at::TensorList node_tables, at::IntArrayRef node_table_type,
              at::TensorList edge_recs) {
  const OneDevice one_device_;
  const size_t R = indptrs.size(), NT = n_nodes.size();
  TORCH_CHECK_VALUE(edge_recs.empty() || edge_recs.size() == R,
                    "sample_blocks: edge_recs holds one packed record array per relation or none");
  TORCH_CHECK_VALUE(indices.size() == R && eids.size() == R && src_type.size() == R &&
                        dst_type.size() == R && excl_eids.size() == R && coo_dst.size() == R &&
                        excl_masks.size() == R && excl_rows.size() == R,
                    "sample_blocks: one entry per relation in every relation list");
  TORCH_CHECK_VALUE(seeds.size() == NT && pos.size() == NT && bits.size() == NT &&
                        word_rank.size() == NT && marks.size() == NT,
                    "sample_blocks: one seed list and one scratch set per node type");
  TORCH_CHECK_VALUE(steps >= 1 && steps <= GNNREC_SB_MAX_STEPS && R <= GNNREC_SB_MAX_RELS &&
                        NT >= 1 && NT <= GNNREC_SB_MAX_TYPES,
                    "sample_blocks: ", steps, " steps, ", R, " relations, ", NT,
                    " types exceed the fused sampler's limits");
  TORCH_CHECK_VALUE((int64_t)fanouts.size() == steps * (int64_t)R &&
                        (int64_t)keys.size() == steps * (int64_t)R,
                    "sample_blocks: fanouts / keys must hold steps x relations entries");
  gnnrec_sample_plan P{};
  P.n_rels = (int)R;
  P.n_types = (int)NT;
  P.n_steps = (int)steps;
  P.stamp = (uint32_t)stamp;
  P.static_shapes = static_shapes ? 1 : 0;
  // static capacity hints [step][type] (empty: none) and the overflow flag they may raise
  TORCH_CHECK_VALUE(node_cap_hint.empty() || (int64_t)node_cap_hint.size() == steps * (int64_t)NT,
                    "sample_blocks: node_cap_hint must hold steps x types entries");
  for (int64_t s = 0; s < steps && !node_cap_hint.empty(); ++s)
    for (size_t t = 0; t < NT; ++t) P.node_cap_hint[s][t] = node_cap_hint[s * NT + t];
  if (has(overflow)) {
    dev(overflow, "overflow", at::kLong);
    TORCH_CHECK_VALUE(overflow->numel() >= 1, "sample_blocks: overflow holds one flag");
    P.overflow = p<int64_t>(overflow);
  }
  for (size_t r = 0; r < R; ++r) {
    dev(indptrs[r], "indptr", at::kLong);
    dev(indices[r], "indices", at::kInt);
    dev(eids[r], "eids", at::kLong);
    TORCH_CHECK_VALUE(src_type[r] >= 0 && (size_t)src_type[r] < NT && dst_type[r] >= 0 &&
                          (size_t)dst_type[r] < NT,
                      "sample_blocks: node-type index out of range");
    TORCH_CHECK_VALUE(indptrs[r].numel() == n_nodes[dst_type[r]] + 1 &&
                          eids[r].numel() == indices[r].numel(),
                      "sample_blocks: relation ", r, ": indptr must hold n_dst + 1 entries and "
                      "eids one per index");
    gnnrec_sample_rel& re = P.rel[r];
    re.indptr = p<int64_t>(indptrs[r]);
    re.indices = p<int32_t>(indices[r]);
    re.eids = p<int64_t>(eids[r]);
    if (!edge_recs.empty()) {  // {eid << 32 | src} per CSR edge (HeteroGraph.edge_records)
      dev(edge_recs[r], "edge_recs", at::kLong);
      TORCH_CHECK_VALUE(edge_recs[r].is_contiguous() && edge_recs[r].numel() == eids[r].numel(),
                        "sample_blocks: relation ", r, ": edge_recs must hold one record per edge");
      re.edge_rec = p<uint64_t>(edge_recs[r]);
    }
    re.src_type = (int32_t)src_type[r];
    re.dst_type = (int32_t)dst_type[r];
    const optional<Tensor> xe = excl_eids.get(r), cd = coo_dst.get(r), xm = excl_masks.get(r),
                           xr = excl_rows.get(r);
    TORCH_CHECK_VALUE(has(xe) == has(cd) && has(xe) == has(xm) && has(xe) == has(xr),
                      "sample_blocks: relation ", r,
                      ": exclusion needs the eids, the COO dst and both flag arrays");
    if (has(xe)) {
      dev(xe, "excl_eids", at::kLong);
      dev(cd, "coo_dst", at::kLong);
      dev(xm, "excl_mask", at::kByte);
      dev(xr, "excl_rows", at::kByte);
      TORCH_CHECK_VALUE(xe->is_contiguous() && cd->numel() == eids[r].numel() &&
                            xm->numel() == eids[r].numel() &&
                            xr->numel() == n_nodes[dst_type[r]],
                        "sample_blocks: relation ", r, ": exclusion arrays sized E, E, n_dst");
      re.excl_eids = p<int64_t>(xe);
      re.n_excl = xe->numel();
      re.coo_dst = p<int64_t>(cd);
      re.excl_mask = p<uint8_t>(xm);
      re.excl_rows = p<uint8_t>(xr);
    }
    for (int64_t s = 0; s < steps; ++s) {
      P.fanout[s][r] = fanouts[s * R + r];
      P.key[s][r] = (uint64_t)keys[s * R + r];
    }
  }
  for (size_t t = 0; t < NT; ++t) {
    dev(seeds[t], "seeds", at::kLong);
    dev(pos[t], "pos", at::kLong);
    dev(bits[t], "bits", at::kLong);
    dev(word_rank[t], "word_rank", at::kLong);
    dev(marks[t], "marks", at::kByte);
    const int64_t W = (n_nodes[t] + 63) / 64;
    TORCH_CHECK_VALUE(seeds[t].is_contiguous() && pos[t].numel() == 2 * n_nodes[t] &&
                          bits[t].numel() == 2 * W && word_rank[t].numel() == W + 1 &&
                          marks[t].numel() == 4 * 64 * W,
                      "sample_blocks: type ", t,
                      ": scratch sized 2n, 2 ceil(n/64), ceil(n/64)+1, 256 ceil(n/64) bytes");
    gnnrec_sample_type& ty = P.type[t];
    ty.n_nodes = n_nodes[t];
    ty.seeds = p<int64_t>(seeds[t]);
    ty.n_seeds = seeds[t].numel();
    ty.pos = p<int64_t>(pos[t]);
    ty.bits = p<uint64_t>(bits[t]);
    ty.word_rank = p<int64_t>(word_rank[t]);
    ty.marks = p<uint8_t>(marks[t]);
  }
  int64_t seed_cap[GNNREC_SB_MAX_STEPS * GNNREC_SB_MAX_TYPES];
  int64_t edge_cap[GNNREC_SB_MAX_STEPS * GNNREC_SB_MAX_RELS];
  int64_t node_cap[GNNREC_SB_MAX_STEPS * GNNREC_SB_MAX_TYPES];
  int64_t dump_rows[GNNREC_SB_MAX_STEPS * GNNREC_SB_MAX_TYPES];
  int64_t ws_bytes = 0;
  ck(gnnrec_sample_blocks_caps(&P, seed_cap, edge_cap, node_cap, dump_rows, &ws_bytes),
     "gnnrec_sample_blocks_caps");
  // static shapes: a node list also holds the next step's dump rows (the last step: one)
  auto node_len = [&](int64_t s, size_t t) {
    if (!static_shapes) return node_cap[s * GNNREC_SB_MAX_TYPES + t];
    return node_cap[s * GNNREC_SB_MAX_TYPES + t] +
           (s + 1 < steps ? dump_rows[(s + 1) * GNNREC_SB_MAX_TYPES + t] : 1);
  };
  const c10::DeviceGuard g(pos[0].device());
  const auto i64 = pos[0].options();
  std::vector<Tensor> o_ip(steps * R), o_src(steps * R), o_eid(steps * R), nodes(steps * NT);
  for (int64_t s = 0; s < steps; ++s) {
    for (size_t r = 0; r < R; ++r) {
      const int64_t sc = seed_cap[s * GNNREC_SB_MAX_TYPES + dst_type[r]];
      const int64_t ec = edge_cap[s * GNNREC_SB_MAX_RELS + r];
      o_ip[s * R + r] = at::empty(
          {sc + 1 + (static_shapes ? dump_rows[s * GNNREC_SB_MAX_TYPES + dst_type[r]] : 0)}, i64);
      o_src[s * R + r] = at::empty({ec}, i64.dtype(at::kInt));
      o_eid[s * R + r] = at::empty({ec}, i64);
      P.out_indptr[s][r] = p<int64_t>(o_ip[s * R + r]);
      P.out_src[s][r] = p<int32_t>(o_src[s * R + r]);
      P.out_eid[s][r] = p<int64_t>(o_eid[s * R + r]);
    }
    for (size_t t = 0; t < NT; ++t) {
      nodes[s * NT + t] = at::empty({node_len(s, t)}, i64);
      P.nodes[s][t] = p<int64_t>(nodes[s * NT + t]);
    }
  }
  const int64_t n_sizes = (steps + 1) * (int64_t)NT + steps * (int64_t)R;
  // sizes_out: the device sizes land there and nothing is read back — the caller queues
  // work sized by them (gathers with device row counts) before its own one read
  if (has(sizes_out)) {
    dev(sizes_out, "sizes_out", at::kLong);
    TORCH_CHECK_VALUE(sizes_out->numel() == n_sizes && sizes_out->is_contiguous(),
                      "sample_blocks: sizes_out must hold ", n_sizes, " entries");
  }
  Tensor sizes = has(sizes_out) ? *sizes_out : at::empty({n_sizes}, i64);
  Tensor ws = at::empty({std::max<int64_t>(ws_bytes, 1)}, i64.dtype(at::kByte));
  P.sizes = p<int64_t>(sizes);
  P.workspace = ws.data_ptr();
  ck(gnnrec_sample_blocks(&P, stream_of(pos[0])), "gnnrec_sample_blocks");
  // the block data (a10): every step's edge data tables at its edge ids, the input block's
  // node tables at its source ids — queued behind the sampler, row counts read on the device
  // (static shapes: every slot; -1 ids give zero rows), ahead of the one size read below
  TORCH_CHECK_VALUE(edge_table_rel.size() == edge_tables.size() &&
                        node_table_type.size() == node_tables.size(),
                    "sample_blocks: one relation / node type per data table");
  std::vector<Tensor> gathered;
  std::vector<gnnrec_gather_job> jobs;
  auto add_job = [&](const Tensor& src, const Tensor& idx, int64_t n, const int64_t* n_dev) {
    TORCH_CHECK_VALUE(src.is_cuda() && src.dim() >= 1, "sample_blocks: data tables on the device");
    same_dev(src, "data table");
    std::vector<int64_t> shape(src.sizes().begin(), src.sizes().end());
    shape[0] = n;
    int64_t inner = 1;
    for (int64_t k = src.dim() - 1; k >= 1; --k) {
      TORCH_CHECK_VALUE(src.size(k) <= 1 || src.stride(k) == inner,
                        "sample_blocks: data table rows must be contiguous");
      inner *= src.size(k);
    }
    Tensor out = at::empty(shape, src.options());
    const int64_t es = src.element_size();
    jobs.push_back(gnnrec_gather_job{src.data_ptr(), src.stride(0) * es, p<int64_t>(idx), n,
                                     inner * es, out.data_ptr(), inner * es, n_dev});
    gathered.push_back(out);
  };
  const bool exact = !static_shapes;
  for (int64_t s = 0; s < steps; ++s)
    for (size_t j = 0; j < edge_tables.size(); ++j) {
      const int64_t r = edge_table_rel[j];
      TORCH_CHECK_VALUE(r >= 0 && (size_t)r < R, "sample_blocks: edge table relation");
      add_job(edge_tables[j], o_eid[s * R + r], edge_cap[s * GNNREC_SB_MAX_RELS + r],
              exact ? p<int64_t>(sizes) + (steps + 1) * NT + s * R + r : nullptr);
    }
  for (size_t j = 0; j < node_tables.size(); ++j) {
    const int64_t t = node_table_type[j];
    TORCH_CHECK_VALUE(t >= 0 && (size_t)t < NT, "sample_blocks: node table type");
    add_job(node_tables[j], nodes[(steps - 1) * NT + t], node_len(steps - 1, t),
            exact ? p<int64_t>(sizes) + steps * NT + t : nullptr);
  }
  for (size_t i = 0; i < jobs.size(); i += GNNREC_GATHER_MAX_JOBS)
    ck(gnnrec_gather_rows_batch(jobs.data() + i,
                                (int)std::min<size_t>(GNNREC_GATHER_MAX_JOBS, jobs.size() - i),
                                stream_of(pos[0])),
       "gnnrec_gather_rows_batch");
  if (static_shapes || has(sizes_out)) {  // every output at its capacity: return those
    std::vector<int64_t> caps;  // seed caps [T], node caps [L x T], edge caps [L x R], and
    for (size_t t = 0; t < NT; ++t) caps.push_back(seed_cap[t]);  // dump rows [L x T]
    for (int64_t s = 0; s < steps; ++s)
      for (size_t t = 0; t < NT; ++t) caps.push_back(node_cap[s * GNNREC_SB_MAX_TYPES + t]);
    for (int64_t s = 0; s < steps; ++s)
      for (size_t r = 0; r < R; ++r) caps.push_back(edge_cap[s * GNNREC_SB_MAX_RELS + r]);
    for (int64_t s = 0; s < steps; ++s)
      for (size_t t = 0; t < NT; ++t) caps.push_back(dump_rows[s * GNNREC_SB_MAX_TYPES + t]);
    return {o_ip, o_src, o_eid, nodes, caps, gathered};
  }
  const Tensor hs = sizes.to(at::kCPU);  // the call's one size readback
  const int64_t* h = hs.data_ptr<int64_t>();
  std::vector<int64_t> out_sizes(h, h + n_sizes);
  for (int64_t s = 0; s < steps; ++s) {
    for (size_t r = 0; r < R; ++r) {
      const int64_t n_dst = h[s * NT + dst_type[r]];
      const int64_t ne = h[(steps + 1) * NT + s * R + r];
      o_ip[s * R + r] = o_ip[s * R + r].narrow(0, 0, n_dst + 1);
      o_src[s * R + r] = o_src[s * R + r].narrow(0, 0, ne);
      o_eid[s * R + r] = o_eid[s * R + r].narrow(0, 0, ne);
    }
    for (size_t t = 0; t < NT; ++t)
      nodes[s * NT + t] = nodes[s * NT + t].narrow(0, 0, h[(s + 1) * NT + t]);
  }
  size_t gi = 0;
  for (int64_t s = 0; s < steps; ++s)
    for (size_t j = 0; j < edge_tables.size(); ++j, ++gi)
      gathered[gi] = gathered[gi].narrow(0, 0, h[(steps + 1) * NT + s * R + edge_table_rel[j]]);
  for (size_t j = 0; j < node_tables.size(); ++j, ++gi)
    gathered[gi] = gathered[gi].narrow(0, 0, h[steps * NT + node_table_type[j]]);
  return {o_ip, o_src, o_eid, nodes, out_sizes, gathered};
}

// a10: several row gathers in one launch (gnnrec_gather_rows_batch): out[j] = src[j][idx[j]]
void gather_rows_batch(at::TensorList src, at::TensorList idx, at::TensorList out,
                       at::TensorList n_dev) {
  const OneDevice one_device_;
  const size_t n = src.size();
  TORCH_CHECK_VALUE(idx.size() == n && out.size() == n && n <= GNNREC_GATHER_MAX_JOBS &&
                        (n_dev.empty() || n_dev.size() == n),
                    "gather_rows_batch: one idx and out (and n_dev, if any) per src, at most ",
                    GNNREC_GATHER_MAX_JOBS, " jobs");
  std::vector<gnnrec_gather_job> jobs(n);
  for (size_t j = 0; j < n; ++j) {
    dev(idx[j], "idx", at::kLong);
    TORCH_CHECK_VALUE(src[j].is_cuda() || src[j].is_meta(),
                      "src: expected a device tensor (there is no CPU path)");
    same_dev(src[j], "src");
    same_dev(out[j], "out");
    TORCH_CHECK_VALUE(src[j].dim() >= 1 && out[j].dim() == src[j].dim() &&
                          out[j].scalar_type() == src[j].scalar_type() && idx[j].is_contiguous() &&
                          out[j].size(0) == idx[j].numel() && out[j].is_contiguous(),
                      "gather_rows_batch: job ", j, ": out [n, ...] of src's dtype and rank, "
                      "contiguous idx [n]");
    int64_t inner = 1;
    for (int64_t k = src[j].dim() - 1; k >= 1; --k) {
      TORCH_CHECK_VALUE(out[j].size(k) == src[j].size(k), "gather_rows_batch: row shapes differ");
      TORCH_CHECK_VALUE(src[j].size(k) <= 1 || src[j].stride(k) == inner,
                        "gather_rows_batch: src rows must be contiguous");
      inner *= src[j].size(k);
    }
    const int64_t es = src[j].element_size();
    // n_dev[j] (one device int64, or empty): rows min(*n_dev, n) — a producer's count
    const int64_t* cnt = nullptr;
    if (!n_dev.empty() && n_dev[j].numel() > 0) {
      dev(n_dev[j], "n_dev", at::kLong);
      TORCH_CHECK_VALUE(n_dev[j].numel() == 1, "gather_rows_batch: n_dev entries hold one count");
      cnt = p<int64_t>(n_dev[j]);
    }
    jobs[j] = gnnrec_gather_job{src[j].data_ptr(), src[j].stride(0) * es, p<int64_t>(idx[j]),
                                idx[j].numel(), inner * es, out[j].data_ptr(), inner * es, cnt};
  }
  if (n == 0 || meta(src[0])) return;
  const c10::DeviceGuard g(src[0].device());
  ck(gnnrec_gather_rows_batch(jobs.data(), (int)n, stream_of(src[0])), "gnnrec_gather_rows_batch");
}

// a11: compact_graphs over id lists at static shapes (gnnrec_compact_ids): per node type the
// sorted distinct ids of its lists in nodes[t] [caps[t]] (-1 past the count), each list
// relabelled to local ids, the per-type counts left on the device — no host read, so a
// loader feeding a captured step keeps every shape fixed.  bits [2 ceil(n/64) +
// GNNREC_COMPACT_SCAN_WS(n)] and word_rank [ceil(n/64) + 1] per type; the bitmaps zero before
// the first call, parity alternating.
std::tuple<std::vector<Tensor>, std::vector<Tensor>, Tensor>
compact_ids(at::TensorList ids, at::IntArrayRef type, at::IntArrayRef n_nodes,
            at::IntArrayRef caps, at::TensorList bits, at::TensorList word_rank,
            at::TensorList marks, int64_t parity) {
  const OneDevice one_device_;
  const size_t L = ids.size(), NT = n_nodes.size();
  TORCH_CHECK_VALUE(type.size() == L && L <= GNNREC_COMPACT_MAX_LISTS && NT >= 1 &&
                        NT <= GNNREC_SB_MAX_TYPES && caps.size() == NT && bits.size() == NT &&
                        word_rank.size() == NT && marks.size() == NT,
                    "compact_ids: at most ", GNNREC_COMPACT_MAX_LISTS, " lists (one type each) "
                    "and 1..", GNNREC_SB_MAX_TYPES, " types (a cap and a scratch pair each)");
  TORCH_CHECK_VALUE(parity == 0 || parity == 1, "compact_ids: parity is 0 or 1");
  gnnrec_compact_type T[GNNREC_SB_MAX_TYPES] = {};
  gnnrec_compact_list Ls[GNNREC_COMPACT_MAX_LISTS] = {};
  const c10::DeviceGuard g(bits[0].device());
  const auto i64 = bits[0].options();
  std::vector<Tensor> nodes(NT), local(L);
  for (size_t t = 0; t < NT; ++t) {
    dev(bits[t], "bits", at::kLong);
    dev(word_rank[t], "word_rank", at::kLong);
    const int64_t W = (n_nodes[t] + 63) / 64;
    dev(marks[t], "marks", at::kByte);
    // bits: the two parity bitmaps, then the scan's workspace
    const int64_t ws = GNNREC_COMPACT_SCAN_WS(n_nodes[t]);
    TORCH_CHECK_VALUE(n_nodes[t] >= 0 && caps[t] >= 0 && bits[t].numel() == 2 * W + ws &&
                          word_rank[t].numel() == W + 1 && marks[t].numel() == 2 * 64 * W,
                      "compact_ids: type ", t, ": scratch sized 2 ceil(n/64) + ", ws,
                      ", ceil(n/64)+1, 128 ceil(n/64) bytes");
    nodes[t] = at::empty({caps[t]}, i64);
    T[t] = gnnrec_compact_type{n_nodes[t], p<uint64_t>(bits[t]), p<int64_t>(word_rank[t]),
                               p<int64_t>(nodes[t]), caps[t], p<uint8_t>(marks[t]),
                               p<uint64_t>(bits[t]) + 2 * W};
  }
  // the lists' local ids are consecutive views of one buffer (lists given one after the
  // other, e.g. an etype's positive then negative sources, come back joined)
  int64_t n_all = 0;
  for (size_t l = 0; l < L; ++l) n_all += ids[l].numel();
  const Tensor local_all = at::empty({n_all}, i64);
  int64_t off = 0;
  for (size_t l = 0; l < L; ++l) {
    dev(ids[l], "ids", at::kLong);
    TORCH_CHECK_VALUE(type[l] >= 0 && (size_t)type[l] < NT && ids[l].is_contiguous(),
                      "compact_ids: list ", l, ": type out of range or ids not contiguous");
    local[l] = local_all.narrow(0, off, ids[l].numel());
    off += ids[l].numel();
    Ls[l] = gnnrec_compact_list{p<int64_t>(ids[l]), ids[l].numel(), (int32_t)type[l],
                                p<int64_t>(local[l])};
  }
  Tensor count = at::empty({(int64_t)NT}, i64);
  ck(gnnrec_compact_ids(Ls, (int)L, T, (int)NT, (int)parity, p<int64_t>(count),
                        stream_of(bits[0])),
     "gnnrec_compact_ids");
  return {nodes, local, count};
}

// a12: many contiguous same-size copies dst[j] <- src[j] in one launch per 64
// (gnnrec_copy_batch: a static batch into a captured step's buffers, gnnrec/capture.py)
void copy_batch(at::TensorList src, at::TensorList dst) {
  const OneDevice one_device_;
  TORCH_CHECK_VALUE(src.size() == dst.size(), "copy_batch: one dst per src");
  std::vector<const void*> sp;
  std::vector<void*> dp;
  std::vector<int64_t> nb;
  for (size_t j = 0; j < src.size(); ++j) {
    TORCH_CHECK_VALUE(src[j].is_cuda() && dst[j].is_cuda(),
                      "copy_batch: device tensors (there is no CPU path)");
    same_dev(src[j], "src");
    same_dev(dst[j], "dst");
    TORCH_CHECK_VALUE(src[j].scalar_type() == dst[j].scalar_type() &&
                          src[j].sizes() == dst[j].sizes() && src[j].is_contiguous() &&
                          dst[j].is_contiguous(),
                      "copy_batch: job ", j, ": contiguous tensors of one dtype and shape");
    sp.push_back(src[j].data_ptr());
    dp.push_back(dst[j].data_ptr());
    nb.push_back(src[j].nbytes());
  }
  if (src.empty()) return;
  const c10::DeviceGuard g(src[0].device());
  for (size_t i = 0; i < sp.size(); i += GNNREC_COPY_MAX_JOBS) {
    const int n = (int)std::min<size_t>(GNNREC_COPY_MAX_JOBS, sp.size() - i);
    ck(gnnrec_copy_batch(sp.data() + i, dp.data() + i, nb.data() + i, n, stream_of(src[0])),
       "gnnrec_copy_batch");
  }
}

// EdgeDataLoader's batch head in one call (gnnrec/sampling.py _iter_batches): the batch's
// positive pairs (find_edges), the uniform negatives (src repeated K times, dst =
// randint(N_dst) from the default generator — the same draws as negative_sampler.Uniform),
// and DGL's compact_graphs([pos, neg]) over both (relabel per node type, ONE size
// readback), returning every pair list in local ids.  The same kernels, generator calls and
// order as the Python form it replaces (bitwise the same pair graphs), issued from C++ with
// the GIL released, so a prefetching loader thread leaves the training thread alone.
//   batch[r]: edge ids of relation r in the batch (empty: not in it); neg_order: the
//   relations in the order their negatives are drawn (the batch's type order)
std::tuple<std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>, std::vector<Tensor>,
           std::vector<Tensor>>
edge_batch_pairs(at::TensorList rel_src, at::TensorList rel_dst, at::IntArrayRef src_type,
                 at::IntArrayRef dst_type, at::TensorList batch, at::IntArrayRef neg_order,
                 int64_t K, at::IntArrayRef n_nodes, at::TensorList prefix_pos,
                 at::TensorList marks) {
  const OneDevice one_device_;
  const size_t R = rel_src.size(), NT = n_nodes.size();
  TORCH_CHECK_VALUE(rel_dst.size() == R && src_type.size() == R && dst_type.size() == R &&
                        batch.size() == R && prefix_pos.size() == NT && marks.size() == NT &&
                        NT > 0,
                    "edge_batch_pairs: list lengths");
  for (size_t r = 0; r < R; ++r)
    TORCH_CHECK_VALUE(src_type[r] >= 0 && (size_t)src_type[r] < NT && dst_type[r] >= 0 &&
                          (size_t)dst_type[r] < NT,
                      "edge_batch_pairs: node-type index out of range");
  const c10::DeviceGuard g(prefix_pos[0].device());
  const auto opt = prefix_pos[0].options();  // int64 on the device
  const Tensor empty = at::empty({0}, opt);
  std::vector<Tensor> ps(R, empty), pd(R, empty), ns(R, empty), nd(R, empty);
  for (size_t r = 0; r < R; ++r) {
    if (batch[r].numel() == 0) continue;
    ps[r] = rel_src[r].index_select(0, batch[r]);
    pd[r] = rel_dst[r].index_select(0, batch[r]);
  }
  if (K > 0) {
    for (int64_t r : neg_order) {
      TORCH_CHECK_VALUE(r >= 0 && (size_t)r < R, "edge_batch_pairs: neg_order out of range");
      if (batch[r].numel() == 0) continue;
      ns[r] = ps[r].repeat_interleave(K);
      nd[r] = at::randint(0, n_nodes[dst_type[r]], {ns[r].numel()}, opt);
    }
  }
  // compact_graphs([pos, neg]): per node type the lists in (pos, neg) x relation order
  std::vector<std::vector<Tensor*>> lists(NT);
  for (auto* side : {&ps, &ns})
    for (size_t r = 0; r < R; ++r) {
      lists[src_type[r]].push_back(&(*side)[r]);
      auto& dlist = side == &ps ? pd : nd;
      lists[dst_type[r]].push_back(&dlist[r]);
    }
  // a relation's positive and negative local ids of one side are written into one buffer
  // [positives | negatives]: the cosine backward then joins them as a view, not a cat
  std::map<const Tensor*, Tensor> joined_out;
  for (size_t r = 0; r < R; ++r)
    for (auto side : {std::make_pair(&ps[r], &ns[r]), std::make_pair(&pd[r], &nd[r])}) {
      const int64_t a = side.first->numel(), b = side.second->numel();
      if (a == 0 || b == 0) continue;
      const Tensor buf = at::empty({a + b}, opt);
      joined_out[side.first] = buf.narrow(0, 0, a);
      joined_out[side.second] = buf.narrow(0, a, b);
    }
  std::vector<Tensor> rank(NT);
  for (size_t t = 0; t < NT; ++t) {
    Tensor pp = prefix_pos[t], mk = marks[t];
    set_prefix_pos(empty, pp);
    for (Tensor* ids : lists[t]) mark_ids(*ids, pp, mk);
    rank[t] = exclusive_scan_new(mk);
  }
  std::vector<Tensor> last;
  for (size_t t = 0; t < NT; ++t) last.push_back(rank[t].narrow(0, rank[t].numel() - 1, 1));
  const Tensor n_new = at::cat(last).to(at::kCPU);  // the one size readback
  std::vector<Tensor> nodes(NT);
  for (size_t t = 0; t < NT; ++t) {
    const int64_t nn = n_new.data_ptr<int64_t>()[t];
    Tensor pp = prefix_pos[t], mk = marks[t];
    nodes[t] = at::empty({nn}, opt);
    if (nn) compact_marked(mk, rank[t], nodes[t]);
    for (Tensor* ids : lists[t]) {
      const auto j = joined_out.find(ids);
      Tensor loc = j != joined_out.end() ? j->second : at::empty({ids->numel()}, opt);
      relabel_ids(*ids, pp, rank[t], 0, loc);
      *ids = loc;  // the list entry becomes its local ids
    }
    clear_prefix_pos(empty, pp);
    if (nn) mk.index_fill_(0, nodes[t], 0);
  }
  return {nodes, ps, pd, ns, nd};
}

// ---------------------------------------------------------------- host-only queries
int64_t version() { return gnnrec_version(); }
void set_concurrency(int64_t reserve_cus, bool dynamic) {
  const OneDevice one_device_;
  ck(gnnrec_set_concurrency((int)reserve_cus, (int)dynamic), "gnnrec_set_concurrency");
}
std::tuple<int64_t, int64_t> get_concurrency() {
  const OneDevice one_device_;
  int r = 0, d = 0;
  ck(gnnrec_get_concurrency(&r, &d), "gnnrec_get_concurrency");
  return {r, d};
}
int64_t spmm_plan_overflows() {
  int64_t n = 0;
  ck(gnnrec_spmm_plan_overflows(&n), "gnnrec_spmm_plan_overflows");
  return n;
}

std::tuple<int64_t, int64_t> rowq_stats() {
  const OneDevice one_device_;
  int64_t q = 0, b = 0;
  ck(gnnrec_rowq_stats(&q, &b), "gnnrec_rowq_stats");
  return {q, b};
}
int64_t scan_workspace_bytes(int64_t n) { return gnnrec_scan_workspace_bytes(n); }
int64_t gemm_tn_workspace_bytes(int64_t K, int64_t M, int64_t N) {
  const OneDevice one_device_;
  return gnnrec_gemm_tn_workspace_bytes(K, M, N);
}
int64_t csr_transpose_workspace_bytes(int64_t E, int64_t n_src) {
  const OneDevice one_device_;
  return (int64_t)gnnrec_csr_transpose_workspace_bytes(E, n_src);
}
int64_t csr_from_keys_workspace_bytes(int64_t E, int64_t n_rows) {
  const OneDevice one_device_;
  return (int64_t)gnnrec_csr_from_keys_workspace_bytes(E, n_rows);
}
int64_t csr_build_workspace_bytes(int64_t E, int64_t n_dst) {
  const OneDevice one_device_;
  return (int64_t)gnnrec_csr_build_workspace_bytes(E, n_dst);
}
int64_t sddmm_cos_backward_workspace_bytes(int64_t E, int64_t n_src, int64_t n_dst, int64_t d,
                                           int64_t groups, int64_t K) {
  if (groups > 0)
    return (int64_t)gnnrec_sddmm_cos_backward_grouped_workspace_bytes(groups, K, n_src, n_dst, d);
  const OneDevice one_device_;
  return (int64_t)gnnrec_sddmm_cos_backward_workspace_bytes(E, n_src, n_dst, d);
}
int64_t margin_loss_blocks(int64_t n_pos) { return gnnrec_margin_loss_blocks(n_pos); }

}  // namespace

// Schemas: mutated outputs are annotated (a!) so functionalisation knows what each op
// writes; every launch op returns ().
TORCH_LIBRARY(gnnrec, m) {
  m.def("spmm_csr(Tensor indptr, Tensor indices, Tensor? edge_weight, Tensor X, int reduce, "
        "int flags, Tensor(a!) out, Tensor? live=None) -> ()");
  m.def("spmm_csr_split(Tensor indptr, Tensor indices, Tensor? edge_weight, Tensor X, "
        "int reduce, int flags, int split, Tensor heavy_rows, Tensor chunk_ptr, "
        "Tensor chunk_row, int n_chunks, Tensor(a!) out, Tensor(b!) workspace) -> ()");
  m.def("spmm_plan_build(Tensor indptr, int split, int cap_h, Tensor(a!) plan, "
        "Tensor? live=None) -> ()");
  m.def("spmm_csr2(Tensor indptr_a, Tensor indices_a, Tensor? ew_a, Tensor indptr_b, "
        "Tensor indices_b, Tensor? ew_b, Tensor X, int reduce, int flags, Tensor(a!) out_a, "
        "Tensor(b!) out_b) -> ()");
  m.def("spmm_csr_planned(Tensor indptr, Tensor indices, Tensor? edge_weight, Tensor X, "
        "int reduce, int flags, int split, Tensor plan, int cap_h, int cap_c, Tensor(a!) out, "
        "Tensor(b!) workspace, Tensor? live=None) -> ()");
  m.def("spmm_backward(Tensor indptr, Tensor indices, Tensor? edge_weight, Tensor grad_out, "
        "Tensor? X, Tensor? out, int reduce, Tensor(a!) grad_X) -> ()");
  m.def("gemm(Tensor A1, Tensor W1, Tensor? A2, Tensor? W2, Tensor? a2_deg, int a2_mode, "
        "Tensor? bias, Tensor? bias_nonempty, int epilogue, int accum, float out_div, "
        "Tensor? attn_vec, Tensor(b!)? attn_state, Tensor(a!) out, Tensor(c!)? row_norm) -> ()");
  m.def("row_epilogue(Tensor z, int l2norm, int accum, float out_div, Tensor? attn_vec, "
        "Tensor(b!)? attn_state, Tensor(a!) out) -> ()");
  m.def("spmm_project(Tensor indptr, Tensor indices, Tensor? edge_weight, Tensor X, Tensor H, "
        "Tensor W_selfT, Tensor? W_neighT, Tensor? bias, Tensor? bias_nonempty, int reduce, "
        "int epilogue, int accum, float out_div, Tensor? attn_vec, Tensor(b!)? attn_state, "
        "bool mfma, Tensor(a!) out) -> ()");
  m.def("spmm_project2(Tensor indptr_a, Tensor indices_a, Tensor? ew_a, Tensor Ya, int reduce_a, "
        "Tensor? bias_nonempty_a, Tensor indptr_b, Tensor indices_b, Tensor? ew_b, Tensor Yb, "
        "int reduce_b, Tensor? bias_nonempty_b, Tensor H, Tensor W_self_aT, Tensor W_self_bT, "
        "Tensor? bias_a, Tensor? bias_b, int epilogue, int combine, Tensor? attn_vec, "
        "float out_div, Tensor(a!) out) -> ()");
  m.def("spmm_pair(Tensor indptr_a, Tensor indices_a, Tensor? ew_a, int reduce_a, "
        "Tensor? bias_a, Tensor? bias_nonempty_a, Tensor indptr_b, Tensor indices_b, "
        "Tensor? ew_b, int reduce_b, Tensor? bias_b, Tensor? bias_nonempty_b, Tensor X, "
        "Tensor H, Tensor WT4, int epilogue, int combine, Tensor? attn_vec, "
        "float out_div, "
        "Tensor(a!) out) -> ()");
  m.def("sddmm_cos(Tensor src, Tensor dst, Tensor Hs, Tensor Hd, Tensor(a!) out) -> ()");
  m.def("sddmm_cos_grouped(Tensor src_g, Tensor? first, int K, Tensor dst, Tensor Hs, Tensor Hd, "
        "Tensor(a!) out_first, Tensor(b!) out) -> ()");
  m.def("sddmm_cos_backward(Tensor src, Tensor dst, Tensor Hs, Tensor Hd, Tensor grad, "
        "Tensor(a!)? gHs, Tensor(b!)? gHd, Tensor(c!) workspace, int groups=0, int K=0) -> ()");
  m.def("edge_mlp(Tensor src, Tensor dst, Tensor P, Tensor Q, Tensor W2, Tensor b2, Tensor w3, "
        "Tensor b3, Tensor(a!) out) -> ()");
  m.def("edge_mlp_grouped(Tensor src_g, Tensor? first, int K, Tensor dst, Tensor P, Tensor Q, "
        "Tensor W2, Tensor b2, Tensor w3, Tensor b3, Tensor(a!) out_first, Tensor(b!) out) -> ()");
  m.def("sample_count(Tensor indptr, Tensor eids, Tensor? excluded, Tensor seeds, int fanout, "
        "int seed_key, Tensor(a!) counts, Tensor? excluded_rows=None) -> ()");
  m.def("sample_fill(Tensor indptr, Tensor indices, Tensor eids, Tensor? excluded, Tensor seeds, "
        "int fanout, int seed_key, Tensor out_indptr, Tensor(a!) out_src, Tensor(b!) out_eid, "
        "Tensor? excluded_rows=None) -> ()");
  m.def("exclusive_scan(Tensor x, Tensor(a!) out, Tensor(b!) workspace) -> ()");
  m.def("mark_ids(Tensor ids, Tensor prefix_pos, Tensor(a!) mark) -> ()");
  m.def("relabel_ids(Tensor ids, Tensor prefix_pos, Tensor rank, int n_prefix, "
        "Tensor(a!) local) -> ()");
  m.def("compact_marked(Tensor mark, Tensor rank, Tensor(a!) out_ids) -> ()");
  m.def("set_prefix_pos(Tensor prefix, Tensor(a!) prefix_pos) -> ()");
  m.def("clear_prefix_pos(Tensor prefix, Tensor(a!) prefix_pos) -> ()");
  m.def("topk_rows(Tensor scores, int k, Tensor? exclude_indptr, Tensor? exclude_indices, "
        "Tensor(a!) out_vals, Tensor(b!) out_idx) -> ()");
  m.def("gemm_tn(Tensor A, Tensor B, Tensor(b!)? colsum, bool accumulate, Tensor(a!) out, "
        "Tensor(c!) workspace, Tensor? row_ptr=None) -> ()");
  m.def("act_backward(Tensor u, Tensor gz, int flags, Tensor(a!) out) -> ()");
  m.def("act_backward_normed(Tensor z, Tensor row_norm, Tensor gz, bool relu, "
        "Tensor(a!) out) -> ()");
  m.def("csr_transpose(Tensor indptr, Tensor indices, Tensor? edge_weight, int n_src, "
        "int n_edges, bool mean, Tensor(a!) workspace, Tensor(b!) indptr_t, "
        "Tensor(c!) indices_t, Tensor(d!)? ew_t) -> ()");
  m.def("csr_from_keys(Tensor keys, int n_rows, Tensor(a!) workspace, Tensor(b!) indptr, "
        "Tensor(c!) perm) -> ()");
  m.def("csr_build(Tensor src, Tensor dst, int n_dst, Tensor(a!) workspace, Tensor(b!) indptr, "
        "Tensor(c!) indices, Tensor(d!) eids) -> ()");
  m.def("add_(Tensor(a!) a, Tensor b) -> ()");
  m.def("tree_sum_(Tensor(a!) a, Tensor[] rest) -> ()");
  m.def("lstm_step(Tensor P, Tensor indptr, Tensor indices, Tensor order, int t, int n_act, "
        "Tensor h_in, Tensor(a!) h_out, Tensor(b!) c, Tensor W_hhT, Tensor(c!) out) -> ()");
  m.def("lstm_step_save(Tensor P, Tensor indptr, Tensor indices, Tensor order, int t, "
        "int n_act, Tensor h_in, Tensor(a!) h_out, Tensor? c_in, Tensor(b!) c_out, "
        "Tensor(c!) z_out, Tensor W_hhT, Tensor(d!) out) -> ()");
  m.def("lstm_backward_step(Tensor z, Tensor c_t, Tensor? c_prev, Tensor? dh_next, "
        "Tensor? dc_next, int n_next, Tensor g_out, Tensor order, int n_act, Tensor(a!) dz, "
        "Tensor(b!) dc_prev) -> ()");
  m.def("lstm_slots(Tensor indptr, Tensor indices, Tensor order, Tensor step_off, int n_slots, "
        "Tensor(a!) src, Tensor(b!) prev) -> ()");
  m.def("gather_rows(Tensor src, Tensor idx, Tensor(a!) out) -> ()");
  m.def("csr_has_edges(Tensor indptr, Tensor sorted_indices, int n_src, Tensor u, Tensor v, "
        "Tensor(a!) out) -> ()");
  m.def("sage_rel_forward(Tensor m, Tensor h_self, int n_self, Tensor W_self, Tensor W_neigh, "
        "Tensor indptr, Tensor indices, Tensor? edge_weight, int reduce, bool norm, "
        "Tensor? bias=None, Tensor? bias_nonempty=None, Tensor? live=None) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("sage_rel_backward(Tensor gz, Tensor z, Tensor row_norm, Tensor h_self, Tensor agg, "
        "Tensor W_self, Tensor W_neigh, Tensor indptr, Tensor indices, Tensor? edge_weight, "
        "int reduce, int n_src, int nnz, bool norm, int need, Tensor? indptr_t=None, "
        "Tensor? indices_t=None, Tensor? w_mean=None, Tensor(a!)? g_self_out=None, "
        "bool g_self_acc=False, Tensor(b!)? g_m_out=None, bool g_m_acc=False, "
        "Tensor? live_src=None) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("block_transposes(Tensor[] indptrs, Tensor[] indices, int[] n_src, int[] nnz) "
        "-> (Tensor[], Tensor[], Tensor[])");
  m.def("edge_batch_pairs(Tensor[] rel_src, Tensor[] rel_dst, int[] src_type, int[] dst_type, "
        "Tensor[] batch, int[] neg_order, int K, int[] n_nodes, Tensor[] prefix_pos, "
        "Tensor[] marks) -> (Tensor[], Tensor[], Tensor[], Tensor[], Tensor[])");
  m.def("margin_loss(Tensor pos, Tensor neg, int K, float delta, Tensor? mask, Tensor? recency, "
        "Tensor(a!) g_pos, Tensor(b!) g_neg, Tensor(c!) partial) -> ()");
  m.def("sum_scaled(Tensor x, float scale, Tensor(a!) out) -> ()");
  m.def("synth_edges(int seed, int e0, int n_u, int n_i, Tensor? zipf_cdf, Tensor(a!) u, "
        "Tensor(b!) i) -> ()");
  m.def("hold_cus(int blocks, int threads, int lds_bytes, int usec, Tensor(a!) sink) -> ()");
  m.def("sample_layer(Tensor[] indptrs, Tensor[] indices, Tensor[] eids, Tensor?[] masks, "
        "Tensor?[] mask_rows, int[] src_type, int[] dst_type, int[] fanouts, int[] keys, Tensor[] seeds, "
        "Tensor(a!)[] prefix_pos, Tensor(b!)[] marks) -> "
        "(Tensor[] out_indptr, Tensor[] src_local, Tensor[] eids, Tensor[] src_nid, int[] n_edges)");
  m.def("sample_blocks(Tensor[] indptrs, Tensor[] indices, Tensor[] eids, int[] src_type, "
        "int[] dst_type, Tensor?[] excl_eids, Tensor?[] coo_dst, Tensor?[] excl_masks, "
        "Tensor?[] excl_rows, int[] n_nodes, Tensor[] seeds, Tensor(a!)[] pos, "
        "Tensor(b!)[] bits, Tensor(c!)[] word_rank, Tensor(f!)[] marks, int[] fanouts, "
        "int[] keys, int steps, "
        "int stamp, bool static_shapes, Tensor(d!)? sizes_out, int[] node_cap_hint, "
        "Tensor(e!)? overflow, Tensor[] edge_tables, int[] edge_table_rel, Tensor[] node_tables, "
        "int[] node_table_type, Tensor[] edge_recs) -> (Tensor[] out_indptr, Tensor[] src_local, Tensor[] eids, "
        "Tensor[] src_nid, int[] sizes, Tensor[] data)");
  m.def("gather_rows_batch(Tensor[] src, Tensor[] idx, Tensor(a!)[] out, Tensor[] n_dev) -> ()");
  m.def("copy_batch(Tensor[] src, Tensor(a!)[] dst) -> ()");
  m.def("compact_ids(Tensor[] ids, int[] type, int[] n_nodes, int[] caps, Tensor(a!)[] bits, "
        "Tensor(b!)[] word_rank, Tensor(c!)[] marks, int parity) -> (Tensor[] nodes, "
        "Tensor[] local, Tensor count)");
  // host-only entry points (no tensors: one catch-all kernel each)
  m.def("version() -> int", &version);
  m.def("set_concurrency(int reserve_cus, bool dynamic) -> ()", &set_concurrency);
  m.def("get_concurrency() -> (int, int)", &get_concurrency);
  m.def("rowq_stats() -> (int, int)", &rowq_stats);
  m.def("spmm_plan_overflows() -> int", &spmm_plan_overflows);
  m.def("scan_workspace_bytes(int n) -> int", &scan_workspace_bytes);
  m.def("gemm_tn_workspace_bytes(int K, int M, int N) -> int", &gemm_tn_workspace_bytes);
  m.def("csr_transpose_workspace_bytes(int n_edges, int n_src) -> int",
        &csr_transpose_workspace_bytes);
  m.def("csr_from_keys_workspace_bytes(int n_edges, int n_rows) -> int",
        &csr_from_keys_workspace_bytes);
  m.def("csr_build_workspace_bytes(int n_edges, int n_dst) -> int", &csr_build_workspace_bytes);
  m.def("sddmm_cos_backward_workspace_bytes(int n_edges, int n_src, int n_dst, int d, "
        "int groups=0, int K=0) -> int", &sddmm_cos_backward_workspace_bytes);
  m.def("margin_loss_blocks(int n_pos) -> int", &margin_loss_blocks);
}

#define GNNREC_IMPLS(m)                                  \
  m.impl("spmm_csr", &spmm_csr);                         \
  m.impl("spmm_csr_split", &spmm_csr_split);             \
  m.impl("spmm_plan_build", &spmm_plan_build);           \
  m.impl("spmm_csr2", &spmm_csr2);                       \
  m.impl("spmm_csr_planned", &spmm_csr_planned);         \
  m.impl("spmm_backward", &spmm_backward);               \
  m.impl("gemm", &gemm);                                 \
  m.impl("row_epilogue", &row_epilogue);                 \
  m.impl("spmm_project", &spmm_project);                 \
  m.impl("spmm_project2", &spmm_project2);               \
  m.impl("spmm_pair", &spmm_pair);                       \
  m.impl("sddmm_cos", &sddmm_cos);                       \
  m.impl("sddmm_cos_grouped", &sddmm_cos_grouped);       \
  m.impl("sddmm_cos_backward", &sddmm_cos_backward);     \
  m.impl("edge_mlp", &edge_mlp);                         \
  m.impl("edge_mlp_grouped", &edge_mlp_grouped);         \
  m.impl("sample_count", &sample_count);                 \
  m.impl("sample_fill", &sample_fill);                   \
  m.impl("exclusive_scan", &exclusive_scan);             \
  m.impl("mark_ids", &mark_ids);                         \
  m.impl("relabel_ids", &relabel_ids);                   \
  m.impl("compact_marked", &compact_marked);             \
  m.impl("set_prefix_pos", &set_prefix_pos);             \
  m.impl("clear_prefix_pos", &clear_prefix_pos);         \
  m.impl("topk_rows", &topk_rows);                       \
  m.impl("gemm_tn", &gemm_tn);                           \
  m.impl("act_backward", &act_backward);                 \
  m.impl("act_backward_normed", &act_backward_normed);   \
  m.impl("csr_transpose", &csr_transpose);               \
  m.impl("csr_from_keys", &csr_from_keys);               \
  m.impl("csr_build", &csr_build);                       \
  m.impl("add_", &add_);                                 \
  m.impl("tree_sum_", &tree_sum_);                       \
  m.impl("lstm_step", &lstm_step);                       \
  m.impl("lstm_step_save", &lstm_step_save);             \
  m.impl("lstm_backward_step", &lstm_backward_step);     \
  m.impl("lstm_slots", &lstm_slots);                     \
  m.impl("gather_rows", &gather_rows);                   \
  m.impl("gather_rows_batch", &gather_rows_batch);       \
  m.impl("csr_has_edges", &csr_has_edges);               \
  m.impl("sage_rel_forward", &sage_rel_forward);         \
  m.impl("sage_rel_backward", &sage_rel_backward);       \
  m.impl("block_transposes", &block_transposes);         \
  m.impl("margin_loss", &margin_loss);                   \
  m.impl("sum_scaled", &sum_scaled);                     \
  m.impl("synth_edges", &synth_edges);                   \
  m.impl("hold_cus", &hold_cus)

// HIP tensors dispatch under the CUDA key in ROCm PyTorch.
TORCH_LIBRARY_IMPL(gnnrec, CUDA, m) {
  GNNREC_IMPLS(m);
  m.impl("sample_layer", &sample_layer);  // data-dependent sizes: device only, no meta form
  m.impl("edge_batch_pairs", &edge_batch_pairs);
  m.impl("sample_blocks", &sample_blocks);
  m.impl("compact_ids", &compact_ids);
  m.impl("copy_batch", &copy_batch);
}
// Meta / fake tensors (torch.compile tracing): the same functions stop after their checks.
TORCH_LIBRARY_IMPL(gnnrec, Meta, m) { GNNREC_IMPLS(m); }
// CPU tensors: the same functions refuse them in their first operand check (ValueError:
// "must be a HIP device tensor") — there is no CPU path, and the error says so.
TORCH_LIBRARY_IMPL(gnnrec, CPU, m) { GNNREC_IMPLS(m); }
