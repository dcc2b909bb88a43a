// Stable LSD radix sort of row keys for CSR construction (row f3) and the backward
// transposes (f2) — the library's own, so no vendor sort runs on the graph-build path.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace gnnrec {

// Optional fused final pass of a CSR build: for the edge e landing at sorted position p,
// idx_out[p] = src[e] (narrowed to int32) and eid_out[p] = e.
struct CsrGather {
  const int64_t* src = nullptr;
  int32_t* idx_out = nullptr;
  int64_t* eid_out = nullptr;
};

// scratch bytes of radix_sort_rows for E keys in [0, n_rows)
size_t radix_ws_bytes(int64_t E, int64_t n_rows);

// Stable sort of E keys in [0, n_rows) (int64 when keys64, else int32), carrying values
// (vals_in, or the identity 0..E-1 when null).  Outputs: keys_out (sorted keys, may be null
// unless row_ptr is wanted) and vals_out, or the CsrGather outputs instead of vals_out.
// row_ptr (optional, [n_rows+1]): first sorted position of every key.  E < 2^31.
int radix_sort_rows(const void* keys_in, bool keys64, const int32_t* vals_in, int64_t E,
                    int64_t n_rows, uint32_t* keys_out, int32_t* vals_out, const CsrGather* g,
                    int64_t* row_ptr, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace gnnrec
