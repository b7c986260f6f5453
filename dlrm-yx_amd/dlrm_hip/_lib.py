"""ctypes binding of libdlrm_hip.so (the C-ABI declared in include/dlrm_hip.h).

The product path has no fallback: if the shared library is missing the import of
any op fails loudly (``DLRMHipUnavailable``).  Only plain pointers, sizes and the
HIP stream handle cross the boundary — torch is plumbing here.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int32, c_int64, c_size_t, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# DLRM_ABI_VERSION of include/dlrm_hip.h that these signatures mirror; load() refuses a
# library built from any other header (tests/test_cpu_host.py checks header == this).
ABI_VERSION = 10
LIB_PATH = os.environ.get("DLRM_HIP_LIB", os.path.join(_HERE, "libdlrm_hip.so"))


class DLRMHipUnavailable(RuntimeError):
    pass


class DLRMHipError(RuntimeError):
    """A non-zero dlrm_status from the C-ABI (message from dlrm_last_error())."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed (status {code}): {msg}")
        self.code = code


class GemmProblem(ctypes.Structure):
    """struct dlrm_gemm_problem (include/dlrm_hip.h)."""
    _fields_ = [("trans_a", c_int32), ("trans_b", c_int32), ("M", c_int64), ("N", c_int64),
                ("K", c_int64), ("alpha", c_float), ("A", c_void_p), ("lda", c_int64),
                ("B", c_void_p), ("ldb", c_int64), ("C", c_void_p), ("ldc", c_int64),
                ("epilogue", c_int32), ("bias", c_void_p), ("aux", c_void_p),
                ("ld_aux", c_int64), ("ones_col", c_int64), ("mode", c_int32),
                ("splits", c_int32), ("partial", c_void_p)]


MLP_MAX_LAYERS = 4


class MlpChain(ctypes.Structure):
    """struct dlrm_mlp_chain (include/dlrm_hip.h)."""
    _fields_ = [("layers", c_int32), ("rows", c_int64), ("X", c_void_p), ("ldx", c_int64),
                ("in_width", c_int64 * MLP_MAX_LAYERS), ("out_width", c_int64 * MLP_MAX_LAYERS),
                ("W", c_void_p * MLP_MAX_LAYERS), ("ldw", c_int64 * MLP_MAX_LAYERS),
                ("Y", c_void_p * MLP_MAX_LAYERS), ("ldy", c_int64 * MLP_MAX_LAYERS),
                ("parts", c_int32), ("split_layer", c_int32), ("tickets", c_void_p)]


# name -> (restype, argtypes); mirrors include/dlrm_hip.h exactly.
class LaunchRole(ctypes.Structure):
    """struct dlrm_launch_role (include/dlrm_hip.h): a deferred embedding update."""
    _fields_ = [("opaque", ctypes.c_uint64 * 32)]


P = c_void_p
SIGNATURES = {
    "dlrm_abi_version": (c_int32, []),
    "dlrm_last_error": (ctypes.c_char_p, []),
    "dlrm_set_tuning": (c_int32, [c_int32, c_int64]),
    "dlrm_get_tuning": (c_int64, [c_int32]),
    "dlrm_tbe_forward": (c_int32, [P, c_int64, P, c_int32, c_int32, P, c_int32, P, c_int32, P, P,
                                   c_int64, P, P]),
    "dlrm_tbe_backward_workspace_size": (c_size_t, [c_int64, c_int64, c_int64]),
    "dlrm_tbe_backward_sort": (c_int32, [c_int64, P, c_int32, c_int32, P, c_int32, P, c_int32,
                                         c_int64, c_int64, P, c_int64, P, c_size_t, P, P]),
    "dlrm_tbe_backward_sgd": (c_int32, [P, c_int64, P, c_int32, c_int32, P, c_int32, P, c_int32,
                                        c_int64, c_int64, P, P, c_int64, c_float, c_int64, P,
                                        c_size_t, P, c_int32, P]),
    "dlrm_tbe_backward_sgd_f16": (c_int32, [P, c_int64, P, c_int32, c_int32, P, c_int32, P,
                                            c_int32, c_int64, c_int64, P, P, c_int64, c_float,
                                            c_int64, P, c_size_t, P, c_int32, P]),
    "dlrm_tbe_backward_rowwise_adagrad": (c_int32, [P, P, c_int64, P, c_int32, c_int32, P,
                                                    c_int32, P, c_int32, c_int64, c_int64, P, P,
                                                    c_int64, c_float, c_float, c_int64, P,
                                                    c_size_t, P, c_int32, P]),
    "dlrm_tbe_backward_dense": (c_int32, [P, c_int64, P, c_int32, c_int32, P, c_int32, P,
                                          c_int32, c_int64, c_int64, P, P, c_int64, c_int64, P,
                                          c_size_t, P, c_int32, P]),
    "dlrm_tbe_forward_presort": (c_int32, [P, c_int64, P, c_int32, c_int32, P, c_int32, P,
                                           c_int32, P, P, c_int64, c_int64, c_int64, c_int64, P,
                                           c_size_t, P, P, P]),
    "dlrm_mlp_chain_supported": (c_int32, [P]),
    "dlrm_tbe_row_bytes": (c_int64, [c_int32, c_int64]),
    "dlrm_tbe_psw_grad": (c_int32, [P, c_int64, P, c_int32, c_int32, P, c_int32, P, c_int32,
                                    c_int64, P, c_int64, P, P]),
    "dlrm_tbe_forward_rows": (c_int32, [P, c_int32, c_int64, c_int64, P, c_int32, c_int32, P,
                                        c_int32, P, c_int32, P, P, c_int64, P, P]),
    "dlrm_mlp_chain_forward": (c_int32, [P, P]),
    "dlrm_tbe_expand_grad": (c_int32, [c_int64, c_int32, c_int32, P, c_int32, c_int64, P, P,
                                       c_int64, P, P]),
    "dlrm_qr_split_indices": (c_int32, [P, c_int32, c_int64, c_int64, P, P, P]),
    "dlrm_qr_combine_forward": (c_int32, [c_int32, c_int64, c_int64, P, P, P, P]),
    "dlrm_qr_combine_backward": (c_int32, [c_int32, c_int64, c_int64, P, P, P, P, P, P]),
    "dlrm_qr_expand_csr": (c_int32, [c_int32, c_int32, P, c_int32, P, c_int32, P, P, P, c_int64,
                                     P, P, c_int64, P, P]),
    "dlrm_qr_pool_combine_forward": (c_int32, [c_int32, c_int32, c_int64, c_int64, P, P, P,
                                               c_int64, P, c_int64, P]),
    "dlrm_qr_pool_combine_backward": (c_int32, [c_int32, c_int32, c_int64, c_int64, P, P, P,
                                                c_int64, P, c_int64, P, c_int64, P]),
    "dlrm_interact_dot_forward": (c_int32, [c_int32, c_int32, c_int32, P, P, c_int32, P, c_int64,
                                            P]),
    "dlrm_interact_dot_backward": (c_int32, [c_int32, c_int32, c_int32, P, P, c_int32, P,
                                             c_int64, P, P, c_int32, P]),
    "dlrm_interact_dot_forward_gather": (c_int32, [c_int32, c_int32, c_int32, P, c_int64, P, P,
                                                   P, c_int32, P, c_int64, P, P]),
    "dlrm_interact_dot_backward_gather": (c_int32, [c_int32, c_int32, c_int32, P, c_int64, P, P,
                                                    P, c_int32, P, c_int64, P, P, c_int32, P]),
    "dlrm_interact_cat_forward": (c_int32, [c_int32, c_int32, c_int32, P, P, P, c_int64, P]),
    "dlrm_interact_cat_backward": (c_int32, [c_int32, c_int32, c_int32, P, c_int64, P, P, P]),
    "dlrm_gemm_f32_workspace_size": (c_size_t, [c_int32, c_int32, c_int64, c_int64, c_int64]),
    "dlrm_gemm_f32": (c_int32, [c_int32, c_int32, c_int64, c_int64, c_int64, c_float, P, c_int64,
                                P, c_int64, P, c_int64, c_int32, P, P, c_int64, P, c_size_t, P]),
    "dlrm_gemm_f32_group_workspace_size": (c_size_t, [c_int32, P]),
    "dlrm_gemm_f32_group": (c_int32, [c_int32, P, P, c_size_t, P]),
    "dlrm_gemm_f32_group_role": (c_int32, [c_int32, P, P, c_size_t, P, c_int32, P]),
    "dlrm_tbe_backward_defer": (c_int32, [c_int32, P, P, c_int64, P, c_int32, c_int32, P,
                                          c_int32, P, c_int32, c_int64, c_int64, P, P,
                                          c_int64, c_float, c_float, c_int64, P, c_size_t, P,
                                          c_int32, P, P]),
    "dlrm_role_blocks": (c_int32, [P]),
    "dlrm_head_step_defer": (c_int32, [c_int64, c_int64, P, c_int64, P, P, c_int32, c_float,
                                       c_float, P, P, P, P, c_int64, c_int32, P, c_int32,
                                       c_float, P, c_size_t, P, P]),
    "dlrm_gemm_f32_splits": (c_int32, [P]),
    "dlrm_gemm_f32_partial_bytes": (c_size_t, [c_int64, c_int64, c_int32]),
    "dlrm_colsum_workspace_size": (c_size_t, [c_int64, c_int64]),
    "dlrm_colsum_f32": (c_int32, [c_int64, c_int64, P, c_int64, P, c_float, P, c_int32, P,
                                  c_float, P, c_size_t, P]),
    "dlrm_head_workspace_size": (c_size_t, [c_int64]),
    "dlrm_head_forward_backward": (c_int32, [c_int64, c_int64, P, c_int64, P, P, P, c_int32,
                                             c_float, c_float, P, P, P, P, c_size_t, P]),
    "dlrm_head_step_workspace_size": (c_size_t, [c_int64, c_int64]),
    "dlrm_head_step": (c_int32, [c_int64, c_int64, P, c_int64, P, P, c_int32, c_float, c_float,
                                 P, P, P, P, c_int64, c_int32, P, c_int32, c_float, P, c_size_t,
                                 P]),
    "dlrm_outer_drelu": (c_int32, [c_int64, c_int64, P, P, P, c_int64, c_int32, P, c_int64, P]),
    "dlrm_sgd_update": (c_int32, [P, P, c_int64, c_float, P]),
    "dlrm_adagrad_update": (c_int32, [P, P, P, c_int64, c_float, c_float, P]),
    "dlrm_adagrad_update_scaled": (c_int32, [P, P, P, c_int64, c_float, c_float, c_float, P]),
    "dlrm_scale_f32": (c_int32, [P, c_int64, c_float, P]),
    "dlrm_sigmoid_forward": (c_int32, [c_int64, P, P, P]),
    "dlrm_sigmoid_backward": (c_int32, [c_int64, P, P, P, P]),
    "dlrm_relu_backward": (c_int32, [c_int64, c_int64, P, c_int64, P, c_int64, P, c_int64, P]),
    "dlrm_uniform_fill": (c_int32, [P, c_int64, c_float, c_float, c_uint64, P]),
    "dlrm_uniform_int_fill": (c_int32, [P, c_int32, c_int64, c_int64, c_uint64, P]),
    "dlrm_csr_from_tables": (c_int32, [c_int32, c_int32, P, P, P, c_int32, P]),
    "dlrm_criteo_decode": (c_int32, [P, c_int64, c_int32, c_int32, c_int64, P, c_int64, P, P,
                                     c_int32, P, c_int32, P]),
}

STATUS_NAMES = {0: "OK", 1: "INVALID_ARG", 2: "SHAPE", 3: "UNSUPPORTED", 4: "WORKSPACE", 5: "HIP"}

_lib = None


def load() -> ctypes.CDLL:
    """Load libdlrm_hip.so once and attach every signature; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DLRMHipUnavailable(
            f"libdlrm_hip.so not found at {LIB_PATH}; build it with "
            f"`make -C dlrm-yx_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    lib.dlrm_abi_version.restype = c_int32
    got = int(lib.dlrm_abi_version())
    if got != ABI_VERSION:
        raise DLRMHipUnavailable(
            f"{LIB_PATH} has ABI version {got}, the bindings expect {ABI_VERSION}; rebuild it "
            f"with `make -C dlrm-yx_amd/csrc`")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    """Invoke a status-returning entry point; raise DLRMHipError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.dlrm_last_error().decode(errors="replace")
        raise DLRMHipError(name, rc, f"{STATUS_NAMES.get(rc, rc)}: {msg}")


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
