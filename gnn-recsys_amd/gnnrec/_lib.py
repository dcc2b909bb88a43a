"""Loader for libgnnrec.so — the C ABI declared in include/gnnrec.h.

The library is the product: there is no CPU or eager-PyTorch fallback.  If it
is missing or cannot be loaded every op raises ``GnnrecLibraryError``.

torch is imported first on purpose: torch ROCm ships its own libamdhip64
(soname libamdhip64.so.7) and libgnnrec.so's NEEDED entry resolves to that
already-loaded copy, so both share one HIP runtime, one device context and
torch's streams.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GNNREC_LIB", os.path.join(_HERE, "libgnnrec.so"))

# status codes / enums (mirror include/gnnrec.h)
OK = 0
REDUCE_SUM, REDUCE_MEAN, REDUCE_MAX = 0, 1, 2
SRC_STREAM = 0x100  # spmm_project2: a relation's source rows read non-temporally
SPMM_EMPTY_NEGINF = 1
SPMM_ACCUM = 2
EPI_RELU, EPI_L2NORM, EPI_SIGMOID = 1, 2, 4
ACC_STORE, ACC_ADD, ACC_MAX = 0, 1, 2
ACC_ATTN_FIRST, ACC_ATTN, ACC_ATTN_LAST = 3, 4, 5
A2_NONE, A2_DIV_DEG, A2_ZERO_DEG = 0, 1, 2


class GnnrecLibraryError(RuntimeError):
    pass


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_INT = ctypes.c_int
_F32 = ctypes.c_float

# name -> (restype, argtypes); every symbol declared in include/gnnrec.h
SIGNATURES = {
    "gnnrec_version": (_INT, []),
    "gnnrec_last_error": (ctypes.c_char_p, []),
    "gnnrec_set_concurrency": (_INT, [_INT, _INT]),
    "gnnrec_get_concurrency": (_INT, [_P, _P]),
    "gnnrec_rowq_stats": (_INT, [_P, _P]),
    "gnnrec_hold_cus": (_INT, [_INT, _INT, _INT, _I64, _P, _P]),
    "gnnrec_spmm_csr_f32": (_INT, [_P, _P, _P, _P, _I64, _I64, _I64, _INT, _INT, _P, _I64, _P]),
    "gnnrec_spmm_csr_split_f32": (_INT, [_P, _P, _P, _P, _I64, _I64, _I64, _INT, _INT, _P, _I64,
                                         _I64, _P, _I64, _P, _P, _I64, _P, _P]),
    "gnnrec_spmm_plan_overflows": (_INT, [_P]),
    "gnnrec_spmm_plan_build": (_INT, [_P, _I64, _I64, _I64, _I64, _P, _P]),
    "gnnrec_spmm_plan_build_live": (_INT, [_P, _I64, _I64, _I64, _I64, _P, _P, _P]),
    "gnnrec_spmm_csr_live_f32": (_INT, [_P, _P, _P, _P, _I64, _I64, _I64, _INT, _INT, _P, _I64,
                                        _P, _P]),
    "gnnrec_spmm_csr_planned_live_f32": (_INT, [_P, _P, _P, _P, _I64, _I64, _I64, _INT, _INT, _P,
                                                _I64, _I64, _P, _I64, _I64, _P, _P, _P]),
    "gnnrec_spmm_csr2_f32": (_INT, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _INT, _INT, _P,
                                    _P, _I64, _P]),
    "gnnrec_spmm_csr_planned_f32": (_INT, [_P, _P, _P, _P, _I64, _I64, _I64, _INT, _INT, _P, _I64,
                                           _I64, _P, _I64, _I64, _P, _P]),
    "gnnrec_spmm_backward_f32": (_INT, [_P, _P, _P, _P, _I64, _P, _I64, _P, _I64, _I64, _I64,
                                        _INT, _P, _I64, _P]),
    "gnnrec_gemm_f32": (_INT, [_P, _I64, _I64, _P, _P, _I64, _I64, _P, _P, _INT, _P, _P,
                               _I64, _I64, _INT, _INT, _F32, _P, _P, _P, _I64, _P]),
    "gnnrec_gemm_rownorm_f32": (_INT, [_P, _I64, _I64, _P, _P, _I64, _I64, _P, _P, _INT, _P, _P,
                                       _I64, _I64, _INT, _INT, _F32, _P, _P, _P, _I64, _P, _P]),
    "gnnrec_act_backward_normed_f32": (_INT, [_P, _I64, _P, _P, _I64, _I64, _I64, _INT, _P, _I64,
                                              _P]),
    "gnnrec_sddmm_cos_f32": (_INT, [_P, _P, _I64, _P, _I64, _P, _I64, _I64, _P, _P]),
    "gnnrec_sddmm_cos_grouped_f32": (_INT, [_P, _I64, _P, _P, _I64, _P, _P, _P, _I64, _P, _I64,
                                            _I64, _P]),
    "gnnrec_edge_mlp_f32": (_INT, [_P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gnnrec_edge_mlp_grouped_f32": (_INT, [_P, _I64, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P,
                                            _P, _P]),
    "gnnrec_sample_count": (_INT, [_P, _P, _P, _P, _P, _I64, _I64, _U64, _P, _P]),
    "gnnrec_sample_fill": (_INT, [_P, _P, _P, _P, _P, _P, _I64, _I64, _U64, _P, _P, _P, _P]),
    "gnnrec_scan_workspace_bytes": (_I64, [_I64]),
    "gnnrec_gemm_tn_workspace_bytes": (_I64, [_I64, _I64, _I64]),
    "gnnrec_gemm_tn_f32": (_INT, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _INT, _P, _P]),
    "gnnrec_gemm_tn_bias_f32": (_INT, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _INT,
                                       _P, _P]),
    "gnnrec_gemm_tn_bias_rows_f32": (_INT, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P,
                                            _P, _INT, _P, _P]),
    "gnnrec_lstm_step_f32": (_INT, [_P, _I64, _P, _P, _P, _I64, _I64, _P, _P, _P, _I64, _P, _P,
                                    _I64, _P]),
    "gnnrec_lstm_step_save_f32": (_INT, [_P, _I64, _P, _P, _P, _I64, _I64, _P, _P, _P, _P, _P,
                                         _I64, _P, _P, _I64, _P]),
    "gnnrec_lstm_backward_step_f32": (_INT, [_P, _P, _P, _P, _P, _I64, _P, _I64, _P, _I64, _I64,
                                             _P, _P, _P]),
    "gnnrec_lstm_slots": (_INT, [_P, _P, _P, _P, _I64, _I64, _P, _P, _P]),
    "gnnrec_spmm_project_f32": (_INT, [_P, _P, _P, _P, _I64, _P, _I64, _P, _P, _P, _P, _I64, _I64,
                                       _INT, _INT, _INT, _F32, _P, _P, _P, _I64, _P]),
    "gnnrec_spmm_project_mfma_f32": (_INT, [_P, _P, _P, _P, _I64, _P, _I64, _P, _P, _P, _P, _I64, _I64,
                                       _INT, _INT, _INT, _F32, _P, _P, _P, _I64, _P]),
    "gnnrec_spmm_project2_f32": (_INT, [_P, _P, _P, _P, _I64, _INT, _P, _P, _P, _P, _P, _I64, _INT,
                                        _P, _P, _I64, _P, _P, _P, _P, _I64, _I64, _INT, _INT,
                                        _P, _F32, _P, _I64, _P]),
    "gnnrec_spmm_pair_f32": (_INT, [_P, _P, _P, _INT, _P, _P, _P, _P, _P, _INT, _P, _P, _P, _I64,
                                    _I64, _P, _I64, _P, _I64, _I64, _INT, _INT, _P, _F32,
                                    _P, _I64, _P]),
    "gnnrec_gather_rows": (_INT, [_P, _I64, _P, _I64, _I64, _P, _I64, _P]),
    "gnnrec_gather_rows_batch": (_INT, [_P, _INT, _P]),
    "gnnrec_copy_batch": (_INT, [_P, _P, _P, _INT, _P]),
    # (plan*, seed_cap*, edge_cap*, node_cap*, workspace_bytes*) / (plan*, stream)
    "gnnrec_sample_blocks_caps": (_INT, [_P, _P, _P, _P, _P, _P]),
    "gnnrec_sample_blocks": (_INT, [_P, _P]),
    # (lists*, n_lists, types*, n_types, parity, count*, stream)
    "gnnrec_compact_ids": (_INT, [_P, _INT, _P, _INT, _INT, _P, _P]),
    "gnnrec_csr_transpose_workspace_bytes": (_U64, [_I64, _I64]),
    "gnnrec_csr_transpose": (_INT, [_P, _P, _P, _I64, _I64, _I64, _INT, _P, _U64, _P, _P, _P, _P]),
    "gnnrec_csr_from_keys_workspace_bytes": (_U64, [_I64, _I64]),
    "gnnrec_csr_from_keys": (_INT, [_P, _I64, _I64, _P, _U64, _P, _P, _P]),
    "gnnrec_csr_build_workspace_bytes": (_U64, [_I64, _I64]),
    "gnnrec_csr_build": (_INT, [_P, _P, _I64, _I64, _P, _U64, _P, _P, _P, _P]),
    "gnnrec_csr_has_edges": (_INT, [_P, _P, _I64, _I64, _P, _P, _I64, _P, _P]),
    "gnnrec_add_f32": (_INT, [_P, _P, _P, _I64, _P]),
    "gnnrec_tree_sum_f32": (_INT, [_P, _INT, _I64, _P, _P]),
    "gnnrec_row_epilogue_f32": (_INT, [_P, _I64, _I64, _I64, _INT, _INT, _F32, _P, _P, _P, _I64,
                                       _P]),
    "gnnrec_act_backward_f32": (_INT, [_P, _I64, _P, _I64, _I64, _I64, _INT, _P, _I64, _P]),
    "gnnrec_exclusive_scan_i64": (_INT, [_P, _I64, _P, _P, _P]),
    "gnnrec_exclusive_scan_i32": (_INT, [_P, _I64, _P, _P, _P]),
    "gnnrec_mark_ids": (_INT, [_P, _I64, _P, _P, _P]),
    "gnnrec_relabel_ids": (_INT, [_P, _I64, _P, _P, _I64, _P, _P]),
    "gnnrec_compact_marked": (_INT, [_P, _P, _I64, _P, _P]),
    "gnnrec_set_prefix_pos": (_INT, [_P, _I64, _P, _P]),
    "gnnrec_clear_prefix_pos": (_INT, [_P, _I64, _P, _P]),
    "gnnrec_topk_rows_f32": (_INT, [_P, _I64, _I64, _I64, _I64, _P, _P, _P, _P, _P]),
    "gnnrec_synth_edges": (_INT, [_U64, _I64, _I64, _I64, _I64, _P, _P, _P, _P]),
    "gnnrec_margin_loss_blocks": (_I64, [_I64]),
    "gnnrec_margin_loss_f32": (_INT, [_P, _P, _I64, _I64, _F32, _P, _P, _INT, _P, _P, _P, _I64,
                                      _P]),
    "gnnrec_sum_scaled_f32": (_INT, [_P, _I64, _F32, _P, _P]),
    "gnnrec_sddmm_cos_backward_workspace_bytes": (_U64, [_I64, _I64, _I64, _I64]),
    "gnnrec_sddmm_cos_backward_grouped_workspace_bytes": (_U64, [_I64, _I64, _I64, _I64, _I64]),
    "gnnrec_sddmm_cos_backward_grouped_f32": (_INT, [_P, _P, _I64, _I64, _P, _I64, _I64, _P,
                                                     _I64, _I64, _I64, _P, _P, _P, _P, _U64,
                                                     _P]),
    "gnnrec_sddmm_cos_backward_f32": (_INT, [_P, _P, _I64, _P, _I64, _I64, _P, _I64, _I64, _I64,
                                             _P, _P, _P, _P, _U64, _P]),
}

_lib = None
_load_error = None


def load() -> ctypes.CDLL:
    """Return the loaded library, raising GnnrecLibraryError if unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise GnnrecLibraryError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"libgnnrec.so not found at {LIB_PATH}; build it with "
                       f"`make -C gnn-recsys_amd/csrc` (or __graft_entry__.build()). "
                       f"There is no fallback path.")
        raise GnnrecLibraryError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as exc:  # pragma: no cover - depends on the box
        _load_error = f"failed to load {LIB_PATH}: {exc}"
        raise GnnrecLibraryError(_load_error) from exc
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


TORCH_LIB_PATH = os.environ.get("GNNREC_TORCH_LIB", os.path.join(_HERE, "libgnnrec_torch.so"))
_ops = None


def torch_ops():
    """torch.ops.gnnrec: the TORCH_LIBRARY(gnnrec) registration (csrc/torch_ops.cpp) over
    the C ABI, loaded after libgnnrec.so itself.  The product path launches every kernel
    through it; ctypes (load()) stays the C-ABI test path.  GnnrecLibraryError if absent."""
    global _ops
    if _ops is not None:
        return _ops
    load()
    if not os.path.exists(TORCH_LIB_PATH):
        raise GnnrecLibraryError(f"libgnnrec_torch.so not found at {TORCH_LIB_PATH}; build it "
                                 f"with `make -C gnn-recsys_amd/csrc`. There is no fallback path.")
    try:
        torch.ops.load_library(TORCH_LIB_PATH)
    except OSError as exc:  # pragma: no cover - depends on the box
        raise GnnrecLibraryError(f"failed to load {TORCH_LIB_PATH}: {exc}") from exc
    _ops = torch.ops.gnnrec
    return _ops


def i64(v: int) -> int:
    """A 64-bit unsigned key (RNG seeds) as the signed int a torch schema `int` carries."""
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= (1 << 63) else v


def available() -> bool:
    try:
        torch_ops()
        return True
    except GnnrecLibraryError:
        return False


def check(rc: int, what: str) -> None:
    if rc != OK:
        msg = load().gnnrec_last_error().decode(errors="replace")
        if rc == 1:
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg} (status {rc})")


def ptr(t) -> int:
    """Device pointer of a tensor (0 for None)."""
    if t is None:
        return 0
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
