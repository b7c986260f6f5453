"""Tensor-level launchers over the C-ABI (one function per dlrm_* entry point).

Every launcher enqueues on ``torch.cuda.current_stream()`` and returns without
synchronising; all device buffers (outputs, workspaces) are allocated here by the
torch caching allocator and handed to the C-ABI as raw pointers.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _lib

EPI_STORE, EPI_BIAS, EPI_BIAS_RELU, EPI_DRELU, EPI_SGD, EPI_ACCUM, EPI_RELU = range(7)
TBE_ERR_INDEX, TBE_ERR_TABLE_CAP = 1, 2  # dlrm_tbe_error bits


class TBEIndexError(IndexError):
    """Raised by check_tbe_errors: the reference's EmbeddingBag raises IndexError for an
    index outside its table; the device kernels skip such lookups and flag them."""


def check_tbe_errors(flag: torch.Tensor, reset: bool = True) -> None:
    """Read a TBE error flag (synchronises with its stream) and raise on any bit."""
    v = int(flag.item())
    if reset:
        flag.zero_()
    if v & TBE_ERR_INDEX:
        raise TBEIndexError("embedding index out of range for its table (lookup skipped)")
    if v & TBE_ERR_TABLE_CAP:
        raise ValueError("a table had more lookups than max_lookups_per_table "
                         "(its backward update was skipped)")


def _raise_bits(v: int) -> None:
    if v & TBE_ERR_INDEX:
        raise TBEIndexError("embedding index out of range for its table (lookup skipped)")
    if v & TBE_ERR_TABLE_CAP:
        raise ValueError("a table had more lookups than max_lookups_per_table "
                         "(its backward update was skipped)")


class DeferredErrorCheck:
    """Reads a TBE error flag without a host sync on the calling step: ``post()`` enqueues
    an async copy of the flag into pinned host memory (then clears it) and records an event;
    ``poll()`` - at the next call, by then long complete - raises on what the previous call
    flagged.  ``flush()`` waits for the last copy and raises (end of training / tests).
    Skipped while the stream is being captured into a graph."""

    def __init__(self):
        self._host = None
        self._event = None

    def poll(self) -> None:
        if self._event is None:
            return
        self._event.synchronize()  # recorded a call ago: normally already complete
        self._event = None
        v = int(self._host[0])
        self._host[0] = 0
        _raise_bits(v)

    def post(self, flag: torch.Tensor) -> None:
        if torch.cuda.is_current_stream_capturing():
            return
        if self._host is None:
            self._host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._event = None
        self._host.copy_(flag, non_blocking=True)
        flag.zero_()
        self._event = torch.cuda.Event()
        self._event.record()

    def flush(self) -> None:
        self.poll()


# dlrm_tune_key (include/dlrm_hip.h): plan overrides for sweeps and coverage tests
TUNE_KEYS = {"gemm_tile": 1, "gemm_split": 2, "tbe_block": 3, "tbe_sort": 4, "tbe_lean": 5,
             "interact_bwd": 6, "interact_fwd": 7}


class tuning:
    """Context manager over dlrm_set_tuning (thread-local plan overrides; results stay
    exact, only the plan changes), e.g. ``with ops.tuning(gemm_tile=64064, gemm_split=4):``
    or ``tuning(tbe_block=64)``; the previous values are restored on exit."""

    def __init__(self, **kw):
        for k in kw:
            if k not in TUNE_KEYS:
                raise KeyError(f"unknown tuning key {k!r} (one of {sorted(TUNE_KEYS)})")
        self.kw = kw
        self.prev = {}

    def __enter__(self):
        lib = _lib.load()
        for k, v in self.kw.items():
            self.prev[k] = int(lib.dlrm_get_tuning(TUNE_KEYS[k]))
            _lib.call("dlrm_set_tuning", TUNE_KEYS[k], int(v))
        return self

    def __exit__(self, *a):
        for k, v in self.prev.items():
            _lib.call("dlrm_set_tuning", TUNE_KEYS[k], int(v))
        return False


LOSS_MSE, LOSS_BCE = 0, 1
QR_OPS = {"mult": 0, "add": 1, "concat": 2}


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device: Optional[torch.device] = None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("dlrm_hip ops take device tensors (got a CPU tensor)")


def _bits(t: torch.Tensor) -> int:
    if t.dtype == torch.int32:
        return 32
    if t.dtype == torch.int64:
        return 64
    raise TypeError(f"index/offset tensors must be int32 or int64, got {t.dtype}")


class Workspace:
    """Grow-only device scratch buffer (one per owner, reused across calls).  Zeroed when
    allocated: the GEMM split-K tickets at its start must begin at 0 (the kernels leave
    them at 0 after every launch)."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None

    def get(self, nbytes: int, device) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != torch.device(device):
            self.buf = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        return self.buf


_default_ws = {}


def _ws(tag: str, nbytes: int, device) -> torch.Tensor:
    key = (tag, str(device))
    w = _default_ws.get(key)
    if w is None:
        w = _default_ws[key] = Workspace()
    return w.get(nbytes, device)


# ------------------------------------------------------------------ TBE ----
def tbe_forward(weights: torch.Tensor, row_base: torch.Tensor, T: int, B: int,
                indices: torch.Tensor, offsets: torch.Tensor,
                per_sample_weights: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, out_batch_stride: Optional[int] = None,
                error_flag: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Pooled-sum lookup -> [B, T, D] (or into ``out`` with a custom batch stride)."""
    _check_cuda(weights, row_base, indices, offsets, per_sample_weights)
    D = weights.shape[1]
    if out is None:
        out = torch.empty((B, T, D), dtype=torch.float32, device=weights.device)
        out_batch_stride = T * D
    elif out_batch_stride is None:
        out_batch_stride = T * D
    _lib.call("dlrm_tbe_forward", _p(weights), D, _p(row_base), T, B, _p(indices),
              _bits(indices), _p(offsets), _bits(offsets), _p(per_sample_weights), _p(out),
              out_batch_stride, _p(error_flag), _stream(weights.device))
    return out


def mlp_chain(X: torch.Tensor, layers, parts: int = 1, split_layer: int = -1,
              tickets: Optional[torch.Tensor] = None) -> "_lib.MlpChain":
    """dlrm_mlp_chain for a bias-folded Linear+ReLU stack: ``X`` [rows, >= in_width[0]]
    carries its own bias column; ``layers`` = [(W [n, >= kin], Y [rows, >= n], kin)].
    ``parts`` 2 / 4: that many workgroups per 16-row block, splitting layer ``split_layer``
    (default: the largest in_width * out_width) by output columns; ``tickets``: zeroed int32
    [ceil(rows / 16)] device buffer owned by this chain (allocated when None)."""
    c = _lib.MlpChain()
    if parts > 1:
        if split_layer < 0:
            split_layer = max(range(len(layers)), key=lambda i: layers[i][2] * layers[i][0].shape[0])
        if tickets is None:
            tickets = torch.zeros((X.shape[0] + 15) // 16, dtype=torch.int32, device=X.device)
        c.parts, c.split_layer, c.tickets = int(parts), int(split_layer), tickets.data_ptr()
        c._keep = tickets  # the chain struct refers to it
    c.layers = len(layers)
    c.rows = X.shape[0]
    c.X = X.data_ptr()
    c.ldx = X.stride(0)
    for i, (W, Y, kin) in enumerate(layers):
        c.in_width[i] = int(kin)
        c.out_width[i] = W.shape[0]
        c.W[i] = W.data_ptr()
        c.ldw[i] = W.stride(0)
        c.Y[i] = Y.data_ptr()
        c.ldy[i] = Y.stride(0)
    return c


def mlp_chain_supported(chain) -> bool:
    return bool(_lib.load().dlrm_mlp_chain_supported(ctypes.byref(chain)))


def mlp_chain_forward(chain, device=None) -> None:
    """Every layer of the chain in one launch (dlrm_mlp_chain_forward)."""
    dev = device if device is not None else torch.cuda.current_device()
    _lib.call("dlrm_mlp_chain_forward", ctypes.cast(ctypes.byref(chain), ctypes.c_void_p),
              _stream(dev))


# the TBE backward's sort keys are 32-bit global rows (ABI v4): a table set that one
# backward call serves must hold fewer rows (checked where tables are built, so a forward
# is never accepted for a configuration the backward would refuse)
TBE_MAX_ROWS = 0xFFFFFFFF - 1


def check_tbe_rows(total_rows: int, what: str) -> None:
    if int(total_rows) > TBE_MAX_ROWS:
        raise ValueError(f"{what}: {int(total_rows)} rows in one table-batched buffer; the "
                         f"embedding backward supports < 2^32 - 1 rows per call (shard the "
                         f"tables over more ranks or modules)")


# lookups per table the in-launch per-table sort handles (tbe_bwd.hip kSegCap)
TBE_PRESORT_SEG_CAP = 4096


def tbe_forward_presort(weights: torch.Tensor, row_base: torch.Tensor, T: int, B: int,
                        indices: torch.Tensor, offsets: torch.Tensor, workspace: torch.Tensor,
                        max_lookups_per_table: int, out: Optional[torch.Tensor] = None,
                        out_batch_stride: Optional[int] = None,
                        per_sample_weights: Optional[torch.Tensor] = None,
                        error_flag: Optional[torch.Tensor] = None, bottom=None,
                        lookup: bool = True) -> Optional[torch.Tensor]:
    """tbe_forward + this batch's backward sort in one launch (dlrm_tbe_forward_presort);
    follow with tbe_backward(..., workspace, presorted=True).  ``bottom``: an mlp_chain
    (the bottom MLP forward) run as a third role of the same launch.

    ``lookup=False``: the sort-only launch (the C-ABI's ``out = NULL``): no pooled output
    is allocated or written, the lookup is done by its consumer (the gather-fused dot
    interaction); returns None.  Only valid where the per-table sort applies (the library
    returns DLRM_ERR_UNSUPPORTED otherwise)."""
    _check_cuda(weights, row_base, indices, offsets, workspace, per_sample_weights)
    D = weights.shape[1]
    if not lookup:
        if out is not None:
            raise ValueError("tbe_forward_presort: lookup=False takes no out tensor")
        out_batch_stride = T * D
    elif out is None:
        out = torch.empty((B, T, D), dtype=torch.float32, device=weights.device)
        out_batch_stride = T * D
    elif out_batch_stride is None:
        out_batch_stride = T * D
    _lib.call("dlrm_tbe_forward_presort", _p(weights), D, _p(row_base), T, B, _p(indices),
              _bits(indices), _p(offsets), _bits(offsets), _p(per_sample_weights), _p(out),
              out_batch_stride, indices.numel(), weights.shape[0], int(max_lookups_per_table),
              _p(workspace), workspace.numel(), _p(error_flag),
              ctypes.cast(ctypes.byref(bottom), ctypes.c_void_p) if bottom is not None else None,
              _stream(weights.device))
    return out


def tbe_psw_grad(weights: torch.Tensor, row_base: torch.Tensor, T: int, B: int,
                 indices: torch.Tensor, offsets: torch.Tensor, grad_out: torch.Tensor,
                 grad_batch_stride: Optional[int] = None) -> torch.Tensor:
    """d loss / d per_sample_weights of a weighted lookup (dlrm_tbe_psw_grad)."""
    _check_cuda(weights, row_base, indices, offsets, grad_out)
    D = weights.shape[1]
    if grad_batch_stride is None:
        grad_batch_stride = T * D
    g = torch.empty(indices.numel(), dtype=torch.float32, device=weights.device)
    _lib.call("dlrm_tbe_psw_grad", _p(weights), D, _p(row_base), T, B, _p(indices),
              _bits(indices), _p(offsets), _bits(offsets), indices.numel(), _p(grad_out),
              grad_batch_stride, _p(g), _stream(weights.device))
    return g


ROWS_F32, ROWS_F16, ROWS_Q8, ROWS_Q4 = 0, 1, 2, 3


def tbe_row_bytes(fmt: int, D: int) -> int:
    return int(_lib.load().dlrm_tbe_row_bytes(fmt, D))


def tbe_forward_rows(weights: torch.Tensor, fmt: int, D: int, row_base: torch.Tensor, T: int,
                     B: int, indices: torch.Tensor, offsets: torch.Tensor,
                     per_sample_weights: Optional[torch.Tensor] = None,
                     out: Optional[torch.Tensor] = None, out_batch_stride: Optional[int] = None,
                     error_flag: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dlrm_tbe_forward_rows: table-batched pooled lookup over F16 rows ([rows, D] half) or
    row-wise quantized rows ([rows, row_bytes] uint8, torch.ops.quantized prepack layout)."""
    _check_cuda(weights, row_base, indices, offsets, per_sample_weights)
    if fmt == ROWS_F16:
        assert weights.dtype == torch.float16 and weights.shape[1] == D
        row_bytes = 2 * weights.stride(0)
    else:
        assert weights.dtype == torch.uint8 and weights.dim() == 2
        row_bytes = weights.stride(0)
    if out is None:
        out = torch.empty((B, T, D), dtype=torch.float32, device=weights.device)
        out_batch_stride = T * D
    elif out_batch_stride is None:
        out_batch_stride = T * D
    _lib.call("dlrm_tbe_forward_rows", _p(weights), fmt, row_bytes, D, _p(row_base), T, B,
              _p(indices), _bits(indices), _p(offsets), _bits(offsets), _p(per_sample_weights),
              _p(out), out_batch_stride, _p(error_flag), _stream(weights.device))
    return out


def tbe_backward_workspace_size(num_lookups: int, total_rows: int, D: int) -> int:
    return _lib.query("dlrm_tbe_backward_workspace_size", num_lookups, total_rows, D)


PRESORTED_ANY = 2  # DLRM_PRESORTED_ANY


def tbe_backward_sort(weights: torch.Tensor, row_base: torch.Tensor, T: int, B: int,
                      indices: torch.Tensor, offsets: torch.Tensor, workspace: torch.Tensor,
                      max_lookups_per_table: int = 0,
                      per_sample_weights: Optional[torch.Tensor] = None,
                      error_flag: Optional[torch.Tensor] = None) -> None:
    """The backward's sort alone (dlrm_tbe_backward_sort): it depends only on the indices,
    so it can run early (e.g. on a side stream beside the forward); follow with
    tbe_backward(..., workspace, presorted=PRESORTED_ANY) of the same batch (same bound and
    per_sample_weights nullness)."""
    _check_cuda(weights, row_base, indices, offsets, workspace, per_sample_weights)
    _lib.call("dlrm_tbe_backward_sort", weights.shape[1], _p(row_base), T, B, _p(indices),
              _bits(indices), _p(offsets), _bits(offsets), indices.numel(), weights.shape[0],
              _p(per_sample_weights), int(max_lookups_per_table), _p(workspace),
              workspace.numel(), _p(error_flag), _stream(weights.device))


def tbe_backward(mode: str, weights: torch.Tensor, row_base: torch.Tensor, T: int, B: int,
                 indices: torch.Tensor, offsets: torch.Tensor, grad_out: torch.Tensor,
                 lr: float = 0.0, eps: float = 0.0, momentum: Optional[torch.Tensor] = None,
                 per_sample_weights: Optional[torch.Tensor] = None,
                 grad_batch_stride: Optional[int] = None,
                 workspace: Optional[torch.Tensor] = None,
                 max_lookups_per_table: int = 0,
                 error_flag: Optional[torch.Tensor] = None, presorted: int = False) -> None:
    """mode: 'sgd' (fused exact SGD; fp32 or fp16 weights), 'rowwise_adagrad' (fused
    RWSAdagrad) or 'dense' (weights is a gradient buffer to accumulate into).  max_lookups_per_table:
    upper bound on any table's lookups (0 = unknown); <= 4096 selects the per-table LDS
    sort (bitwise the same result as the device-wide radix sort).  ``error_flag``: device
    int32 that receives TBE_ERR_INDEX / TBE_ERR_TABLE_CAP bits (see check_tbe_errors).
    ``presorted``: True - the per-table sort ran in tbe_forward_presort; PRESORTED_ANY -
    tbe_backward_sort ran for this batch."""
    _check_cuda(weights, row_base, indices, offsets, grad_out, momentum, per_sample_weights)
    D = weights.shape[1]
    N = indices.numel()
    total_rows = weights.shape[0]
    if grad_batch_stride is None:
        grad_batch_stride = T * D
    need = tbe_backward_workspace_size(N, total_rows, D)
    if workspace is None:
        workspace = _ws("tbe_bwd", need, weights.device)
    args_common = (D, _p(row_base), T, B, _p(indices), _bits(indices), _p(offsets),
                   _bits(offsets), N, total_rows, _p(per_sample_weights), _p(grad_out),
                   grad_batch_stride)
    st = _stream(weights.device)
    mx = int(max_lookups_per_table)
    if mode == "sgd" and weights.dtype == torch.float16:
        _lib.call("dlrm_tbe_backward_sgd_f16", _p(weights), *args_common, lr, mx,
                  _p(workspace), workspace.numel(), _p(error_flag), int(presorted), st)
    elif mode == "sgd":
        _lib.call("dlrm_tbe_backward_sgd", _p(weights), *args_common, lr, mx, _p(workspace),
                  workspace.numel(), _p(error_flag), int(presorted), st)
    elif mode == "rowwise_adagrad":
        _lib.call("dlrm_tbe_backward_rowwise_adagrad", _p(weights), _p(momentum), *args_common,
                  lr, eps, mx, _p(workspace), workspace.numel(), _p(error_flag), int(presorted),
                  st)
    elif mode == "dense":
        _lib.call("dlrm_tbe_backward_dense", _p(weights), *args_common, mx, _p(workspace),
                  workspace.numel(), _p(error_flag), int(presorted), st)
    else:
        raise ValueError(mode)


def tbe_backward_defer(mode: str, weights: torch.Tensor, row_base: torch.Tensor, T: int, B: int,
                       indices: torch.Tensor, offsets: torch.Tensor, grad_out: torch.Tensor,
                       lr: float = 0.0, eps: float = 0.0,
                       momentum: Optional[torch.Tensor] = None,
                       per_sample_weights: Optional[torch.Tensor] = None,
                       grad_batch_stride: Optional[int] = None,
                       workspace: Optional[torch.Tensor] = None,
                       max_lookups_per_table: int = 0,
                       error_flag: Optional[torch.Tensor] = None, presorted: bool = False):
    """tbe_backward ('sgd' on fp32 weights or 'rowwise_adagrad') with its two update passes
    deferred (dlrm_tbe_backward_defer): returns the role to hand to gemm_group(...,
    role=, phase=1) and then phase=2 - or None when the update already ran in full (shape
    the fused passes do not cover).  The workspace, weights, momentum and grad_out must stay
    untouched until phase 2 has run."""
    _check_cuda(weights, row_base, indices, offsets, grad_out, momentum, per_sample_weights)
    if weights.dtype != torch.float32 or mode not in ("sgd", "rowwise_adagrad"):
        raise ValueError("tbe_backward_defer: fp32 'sgd' or 'rowwise_adagrad' only")
    D = weights.shape[1]
    N = indices.numel()
    total_rows = weights.shape[0]
    if grad_batch_stride is None:
        grad_batch_stride = T * D
    need = tbe_backward_workspace_size(N, total_rows, D)
    if workspace is None:
        workspace = _ws("tbe_bwd", need, weights.device)
    role = _lib.LaunchRole()
    _lib.call("dlrm_tbe_backward_defer", 0 if mode == "sgd" else 1, _p(weights), _p(momentum),
              D, _p(row_base), T, B, _p(indices), _bits(indices), _p(offsets), _bits(offsets), N,
              total_rows, _p(per_sample_weights), _p(grad_out), grad_batch_stride, lr, eps,
              int(max_lookups_per_table), _p(workspace), workspace.numel(), _p(error_flag),
              int(presorted), ctypes.byref(role), _stream(weights.device))
    return role if role_blocks(role) > 0 else None


def role_blocks(role) -> int:
    """Workgroups a deferred update pass adds to the launch carrying it (0: none)."""
    return 0 if role is None else _lib.query("dlrm_role_blocks", ctypes.byref(role))


def tbe_expand_grad(D: int, T: int, B: int, offsets: torch.Tensor, num_lookups: int,
                    grad_out: torch.Tensor, per_sample_weights: Optional[torch.Tensor] = None,
                    grad_batch_stride: Optional[int] = None) -> torch.Tensor:
    _check_cuda(offsets, grad_out, per_sample_weights)
    values = torch.empty((num_lookups, D), dtype=torch.float32, device=grad_out.device)
    if grad_batch_stride is None:
        grad_batch_stride = T * D
    _lib.call("dlrm_tbe_expand_grad", D, T, B, _p(offsets), _bits(offsets), num_lookups,
              _p(per_sample_weights), _p(grad_out), grad_batch_stride, _p(values),
              _stream(grad_out.device))
    return values


# ------------------------------------------------------------------- QR ----
def qr_split_indices(indices: torch.Tensor, collisions: int):
    _check_cuda(indices)
    n = indices.numel()
    q = torch.empty(n, dtype=torch.int64, device=indices.device)
    r = torch.empty(n, dtype=torch.int64, device=indices.device)
    _lib.call("dlrm_qr_split_indices", _p(indices), _bits(indices), n, collisions, _p(q), _p(r),
              _stream(indices.device))
    return q, r


def qr_combine_forward(op: str, eq: torch.Tensor, er: torch.Tensor) -> torch.Tensor:
    n, D = eq.shape
    out = torch.empty((n, 2 * D if op == "concat" else D), dtype=torch.float32, device=eq.device)
    _lib.call("dlrm_qr_combine_forward", QR_OPS[op], n, D, _p(eq), _p(er), _p(out),
              _stream(eq.device))
    return out


def qr_combine_backward(op: str, eq: torch.Tensor, er: torch.Tensor, grad_out: torch.Tensor):
    n, D = eq.shape
    geq = torch.empty_like(eq)
    ger = torch.empty_like(er)
    _lib.call("dlrm_qr_combine_backward", QR_OPS[op], n, D, _p(eq), _p(er),
              _p(grad_out.contiguous()), _p(geq), _p(ger), _stream(eq.device))
    return geq, ger


def qr_expand_csr(T_phys: int, B: int, indices: torch.Tensor, offsets: torch.Tensor,
                  src: torch.Tensor, kind: torch.Tensor, coll: torch.Tensor,
                  max_lookups_per_table: int, phys_indices: torch.Tensor,
                  phys_offsets: torch.Tensor, error_flag: Optional[torch.Tensor] = None) -> None:
    """Logical table-batched CSR -> the physical CSR of the QR engine (dlrm_qr_expand_csr):
    physical table p = logical table src[p]'s bags with its indices (kind 0), quotients
    (kind 1) or remainders (kind 2) by coll[p]; int32 outputs.  Lookups past
    phys_indices.numel() are dropped and raise TBE_ERR_TABLE_CAP in ``error_flag``."""
    _check_cuda(indices, offsets, src, kind, coll, phys_indices, phys_offsets)
    _lib.call("dlrm_qr_expand_csr", T_phys, B, _p(indices), _bits(indices), _p(offsets),
              _bits(offsets), _p(src), _p(kind), _p(coll), int(max_lookups_per_table),
              _p(phys_indices), _p(phys_offsets), phys_indices.numel(), _p(error_flag),
              _stream(indices.device))


def qr_pool_combine_forward(op: str, T: int, B: int, D: int, pq: torch.Tensor, pr: torch.Tensor,
                            P: torch.Tensor, E: torch.Tensor) -> None:
    """E[b, t] = op(P[b, pq[t]], P[b, pr[t]]) (or P[b, pq[t]] where pr[t] < 0)."""
    _lib.call("dlrm_qr_pool_combine_forward", QR_OPS[op], T, B, D, _p(pq), _p(pr), _p(P),
              P.stride(0), _p(E), E.stride(0), _stream(P.device))


def qr_pool_combine_backward(op: str, T: int, B: int, D: int, pq: torch.Tensor,
                             pr: torch.Tensor, P: torch.Tensor, dE: torch.Tensor,
                             dP: torch.Tensor) -> None:
    _lib.call("dlrm_qr_pool_combine_backward", QR_OPS[op], T, B, D, _p(pq), _p(pr), _p(P),
              P.stride(0), _p(dE), dE.stride(0), _p(dP), dP.stride(0), _stream(P.device))


# ---------------------------------------------------------- interaction ----
def _feature_arrays(feats: Sequence[torch.Tensor], strides: Sequence[int]):
    F = len(feats)
    ptrs = (ctypes.c_void_p * F)(*[t.data_ptr() for t in feats])
    bs = (ctypes.c_int64 * F)(*[int(s) for s in strides])
    return ptrs, bs


def feature_views(x: torch.Tensor, ly) -> tuple:
    """(tensors, batch strides, D) for feature 0 = x and ly = [B,T,D] tensor or list of [B,D]."""
    feats = [x]
    strides = [x.stride(0)]
    if isinstance(ly, torch.Tensor):
        ly = [ly]
    for y in ly:
        if y.dim() == 3:  # [B, T, D], rows contiguous in D
            if y.stride(2) != 1:
                raise ValueError("interaction features must be contiguous in D")
            for t in range(y.shape[1]):
                feats.append(y[:, t, :])
                strides.append(y.stride(0))
        else:
            if y.stride(1) != 1:
                raise ValueError("interaction features must be contiguous in D")
            feats.append(y)
            strides.append(y.stride(0))
    return feats, strides


def interact_forward(op: str, x: torch.Tensor, ly, self_interaction: bool = False,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    feats, strides = feature_views(x, ly)
    _check_cuda(*feats)
    B, D = x.shape
    F = len(feats)
    ptrs, bs = _feature_arrays(feats, strides)
    if op == "dot":
        npairs = F * (F + 1) // 2 if self_interaction else F * (F - 1) // 2
        if out is None:
            out = torch.empty((B, D + npairs), dtype=torch.float32, device=x.device)
        _lib.call("dlrm_interact_dot_forward", B, F, D, ptrs, bs, int(self_interaction), _p(out),
                  out.stride(0), _stream(x.device))
    elif op == "cat":
        if out is None:
            out = torch.empty((B, F * D), dtype=torch.float32, device=x.device)
        _lib.call("dlrm_interact_cat_forward", B, F, D, ptrs, bs, _p(out), out.stride(0),
                  _stream(x.device))
    else:
        raise ValueError(op)
    return out


def interact_backward(op: str, x: torch.Tensor, ly, grad_out: torch.Tensor,
                      self_interaction: bool = False, grad_x: Optional[torch.Tensor] = None,
                      grad_ly=None, relu_x: bool = False):
    """Returns (grad_x, grad_ly) with grad_ly shaped like ly ([B,T,D] or list of [B,D]).
    relu_x: grad_x also gets ReLU'(x) applied (x = output of a ReLU layer; dot only)."""
    feats, strides = feature_views(x, ly)
    B, D = x.shape
    F = len(feats)
    if grad_x is None:
        grad_x = torch.empty_like(x, memory_format=torch.contiguous_format)
    if grad_ly is None:
        if isinstance(ly, torch.Tensor):
            grad_ly = torch.empty(ly.shape, dtype=torch.float32, device=x.device)
        else:
            grad_ly = [torch.empty(y.shape, dtype=torch.float32, device=x.device) for y in ly]
    gfeats, gstrides = feature_views(grad_x, grad_ly)
    ptrs, bs = _feature_arrays(feats, strides)
    gptrs, gbs = _feature_arrays(gfeats, gstrides)
    g = grad_out if grad_out.stride(1) == 1 else grad_out.contiguous()  # row stride is passed
    if op == "dot":
        _lib.call("dlrm_interact_dot_backward", B, F, D, ptrs, bs, int(self_interaction), _p(g),
                  g.stride(0), gptrs, gbs, int(relu_x), _stream(x.device))
    else:
        _lib.call("dlrm_interact_cat_backward", B, F, D, _p(g), g.stride(0), gptrs, gbs,
                  _stream(x.device))
        if relu_x:
            relu_backward(grad_x, x, out=grad_x)
    return grad_x, grad_ly


def interact_forward_gather(x: torch.Tensor, weights: torch.Tensor, row_base: torch.Tensor,
                            indices: torch.Tensor, self_interaction: bool = False,
                            out: Optional[torch.Tensor] = None,
                            error_flag: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Dot interaction of x and the one-hot lookups (L = 1) of T = len(row_base) - 1 tables
    gathered straight from ``weights`` (dlrm_interact_dot_forward_gather): the same R as
    interact_forward(x, tbe_forward(...)) without the pooled [B, T, D] buffer."""
    _check_cuda(x, weights, row_base, indices)
    B, D = x.shape
    F = row_base.numel()
    npairs = F * (F + 1) // 2 if self_interaction else F * (F - 1) // 2
    if indices.dtype != torch.int32 or indices.numel() != (F - 1) * B:
        raise ValueError("gather interaction: int32 indices [(F-1) * B] (one per bag)")
    if out is None:
        out = torch.empty(B, D + npairs, dtype=torch.float32, device=x.device)
    _lib.call("dlrm_interact_dot_forward_gather", B, F, D, _p(x), x.stride(0), _p(weights),
              _p(row_base), _p(indices), int(self_interaction), _p(out), out.stride(0),
              _p(error_flag), _stream(x.device))
    return out


def interact_backward_gather(x: torch.Tensor, weights: torch.Tensor, row_base: torch.Tensor,
                             indices: torch.Tensor, grad_out: torch.Tensor,
                             self_interaction: bool = False,
                             grad_x: Optional[torch.Tensor] = None,
                             grad_ly: Optional[torch.Tensor] = None, relu_x: bool = False):
    """Backward of interact_forward_gather (rows re-gathered; call before the embedding
    update): grad_x [B, D] and grad_ly [B, T, D]."""
    B, D = x.shape
    T = row_base.numel() - 1
    if grad_x is None:
        grad_x = torch.empty_like(x, memory_format=torch.contiguous_format)
    if grad_ly is None:
        grad_ly = torch.empty(B, T, D, dtype=torch.float32, device=x.device)
    gfeats, gstrides = feature_views(grad_x, grad_ly)
    gptrs, gbs = _feature_arrays(gfeats, gstrides)
    g = grad_out if grad_out.stride(1) == 1 else grad_out.contiguous()
    _lib.call("dlrm_interact_dot_backward_gather", B, T + 1, D, _p(x), x.stride(0), _p(weights),
              _p(row_base), _p(indices), int(self_interaction), _p(g), g.stride(0), gptrs, gbs,
              int(relu_x), _stream(x.device))
    return grad_x, grad_ly


# ------------------------------------------------------------------ MLP ----
def gemm_workspace_size(M: int, N: int, K: int, trans_a: bool = False,
                        trans_b: bool = False) -> int:
    return _lib.query("dlrm_gemm_f32_workspace_size", int(trans_a), int(trans_b), M, N, K)


GEMM_FULL, GEMM_PARTIAL, GEMM_REDUCE = 0, 1, 2  # dlrm_gemm_mode


def gemm_problem(A: torch.Tensor, B: torch.Tensor, trans_a: bool = False,
                 trans_b: bool = False, C: Optional[torch.Tensor] = None, alpha: float = 1.0,
                 epilogue: int = EPI_STORE, bias: Optional[torch.Tensor] = None,
                 aux: Optional[torch.Tensor] = None, ones_col: int = -1,
                 partial: Optional[torch.Tensor] = None, splits: int = 0):
    """One dlrm_gemm_problem: C = epilogue(alpha * op(A) @ op(B)) with row-major 2-D
    operands (unit inner stride); ones_col >= 0 also writes C[:, ones_col] =
    epilogue(alpha * op(A).sum(1)) (a Linear bias gradient).  With ``partial`` the problem
    is a PARTIAL one: K split ``splits`` ways, raw partials into ``partial``, C untouched
    until reduce_problem(...) runs in a later launch.  Returns (struct, C)."""
    _check_cuda(A, B, C, bias, aux)
    if A.stride(1) != 1 or B.stride(1) != 1:
        raise ValueError("gemm operands need unit inner stride")
    M = A.shape[1] if trans_a else A.shape[0]
    K = A.shape[0] if trans_a else A.shape[1]
    N = B.shape[0] if trans_b else B.shape[1]
    Kb = B.shape[1] if trans_b else B.shape[0]
    if K != Kb:
        raise ValueError(f"gemm inner dims differ: {K} vs {Kb}")
    if C is None:
        C = torch.empty((M, N if ones_col < 0 else max(N, ones_col + 1)), dtype=torch.float32,
                        device=A.device)
    if C.stride(1) != 1 or C.shape[0] != M or C.shape[1] < N:
        raise ValueError("gemm output must be [M, >= N] with unit inner stride")
    if ones_col >= 0 and not (N <= ones_col < C.shape[1]):
        raise ValueError("ones_col must be a column of C outside [0, N)")
    pr = _lib.GemmProblem(int(trans_a), int(trans_b), M, N, K, float(alpha), A.data_ptr(),
                          A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                          int(epilogue), bias.data_ptr() if bias is not None else None,
                          aux.data_ptr() if aux is not None else None,
                          aux.stride(0) if aux is not None else 0, int(ones_col),
                          GEMM_PARTIAL if partial is not None else GEMM_FULL, int(splits),
                          partial.data_ptr() if partial is not None else None)
    return pr, C


def gemm_splits(pr, partial: bool = False, requested: int = 0) -> int:
    """The planner's K split for a problem launched alone (dlrm_gemm_f32_splits); with
    partial=True, as a PARTIAL problem (deferred reduction).  ``requested`` > 0 (PARTIAL):
    that count normalized to K - the count a PARTIAL launch accepts and its REDUCE repeats."""
    q = _lib.GemmProblem.from_buffer_copy(pr)
    if partial:
        q.mode = GEMM_PARTIAL
    q.splits = int(requested) if partial else 0
    return int(_lib.load().dlrm_gemm_f32_splits(ctypes.byref(q)))


def gemm_partial_bytes(M: int, N: int, splits: int) -> int:
    return _lib.query("dlrm_gemm_f32_partial_bytes", M, N, splits)


def sgd_job(param: torch.Tensor, grad: torch.Tensor, lr: float):
    """param -= lr * grad (flat fp32, numel % 4 == 0, 16-B aligned) as a one-split REDUCE job:
    an elementwise GEMM-group problem, so the update rides on a launch that exists anyway
    (C = SGD(alpha * sum_s part[s]) with one split: param - lr * grad, the SGD epilogue's
    rounding)."""
    _check_cuda(param, grad)
    n = param.numel()
    if grad.numel() != n or n % 4 or param.data_ptr() % 16 or grad.data_ptr() % 16:
        raise ValueError("sgd_job: flat fp32 tensors of equal size, numel % 4 == 0, 16-B aligned")
    return _lib.GemmProblem(0, 0, 1, n, 0, float(lr), None, 0, None, 0, param.data_ptr(), n,
                            EPI_SGD, None, None, 0, -1, GEMM_REDUCE, 1, grad.data_ptr())


def reduce_problem(pr_partial):
    """The REDUCE problem finishing a PARTIAL one (same C, alpha, epilogue, ones_col)."""
    q = _lib.GemmProblem.from_buffer_copy(pr_partial)
    q.mode = GEMM_REDUCE
    return q


def _problems(prs):
    arr = (_lib.GemmProblem * len(prs))(*prs)
    return arr


def gemm_group_workspace_size(problems) -> int:
    return _lib.query("dlrm_gemm_f32_group_workspace_size", len(problems),
                      ctypes.cast(_problems(problems), ctypes.c_void_p))


def gemm_group(problems, workspace: Optional[torch.Tensor] = None, device=None, role=None,
               phase: int = 0) -> None:
    """Launch up to 6 independent GEMM problems (gemm_problem structs) in ONE kernel.
    ``workspace``: zero-initialised uint8 buffer (split-K tickets + partials); a cached one
    is used when None.  ``role`` (tbe_backward_defer) + ``phase`` (1, then 2): that pass of
    the deferred embedding update runs as extra workgroups of the same launch (problems
    may then be empty)."""
    arr = _problems(problems)
    need = _lib.query("dlrm_gemm_f32_group_workspace_size", len(problems),
                      ctypes.cast(arr, ctypes.c_void_p)) if problems else 0
    dev = device if device is not None else torch.cuda.current_device()
    if need and workspace is None:
        workspace = _ws("gemm", need, dev)
    elif need and workspace.numel() < need:
        # never fall back to a shared buffer behind the caller's back: two streams could
        # then write split-K partials into the same scratch
        raise ValueError(f"gemm workspace too small: {workspace.numel()} < {need} bytes")
    if role is not None:
        _lib.call("dlrm_gemm_f32_group_role", len(problems), ctypes.cast(arr, ctypes.c_void_p),
                  _p(workspace) if need else None, workspace.numel() if need else 0,
                  ctypes.byref(role), int(phase), _stream(dev))
        return
    _lib.call("dlrm_gemm_f32_group", len(problems), ctypes.cast(arr, ctypes.c_void_p),
              _p(workspace) if need else None, workspace.numel() if need else 0,
              _stream(dev))


def gemm(A: torch.Tensor, B: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
         C: Optional[torch.Tensor] = None, alpha: float = 1.0, epilogue: int = EPI_STORE,
         bias: Optional[torch.Tensor] = None, aux: Optional[torch.Tensor] = None,
         workspace: Optional[torch.Tensor] = None, ones_col: int = -1) -> torch.Tensor:
    """C = epilogue(alpha * op(A) @ op(B)) with row-major 2-D operands (unit inner stride).
    Split-K uses ``workspace`` (or a cached one) when the planner asks for it."""
    pr, C = gemm_problem(A, B, trans_a, trans_b, C, alpha, epilogue, bias, aux, ones_col)
    gemm_group([pr], workspace, A.device)
    return C


def colsum(Y: torch.Tensor, scale: Optional[torch.Tensor] = None, alpha: float = 1.0,
           out: Optional[torch.Tensor] = None, accumulate: bool = False,
           sgd_param: Optional[torch.Tensor] = None, lr: float = 0.0,
           workspace: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    M, N = Y.shape
    need = _lib.query("dlrm_colsum_workspace_size", M, N)
    if workspace is None or workspace.numel() < need:
        workspace = _ws("colsum", need, Y.device)
    _lib.call("dlrm_colsum_f32", M, N, _p(Y), Y.stride(0), _p(scale), float(alpha), _p(out),
              int(accumulate), _p(sgd_param), float(lr), _p(workspace), workspace.numel(),
              _stream(Y.device))
    return out


def head_forward_backward(X: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
                          target: Optional[torch.Tensor], loss: str = "mse",
                          clamp_lo: float = 0.0, grad_scale: float = 1.0,
                          prob: Optional[torch.Tensor] = None, dz: Optional[torch.Tensor] = None,
                          loss_out: Optional[torch.Tensor] = None,
                          workspace: Optional[torch.Tensor] = None):
    M, K = X.shape
    need = _lib.query("dlrm_head_workspace_size", M)
    if workspace is None or workspace.numel() < need:
        workspace = _ws("head", need, X.device)
    _lib.call("dlrm_head_forward_backward", M, K, _p(X), X.stride(0), _p(w), _p(b), _p(target),
              LOSS_BCE if loss == "bce" else LOSS_MSE, float(clamp_lo), float(grad_scale),
              _p(prob), _p(dz), _p(loss_out), _p(workspace), workspace.numel(), _stream(X.device))
    return prob, dz, loss_out


def head_step(X: torch.Tensor, w: torch.Tensor, target: torch.Tensor, loss: str = "mse",
              clamp_lo: float = 0.0, grad_scale: float = 1.0,
              prob: Optional[torch.Tensor] = None, dz: Optional[torch.Tensor] = None,
              loss_out: Optional[torch.Tensor] = None, dX: Optional[torch.Tensor] = None,
              relu_mask: bool = True, dw: Optional[torch.Tensor] = None, accumulate: bool = False,
              lr: float = 0.0, workspace: Optional[torch.Tensor] = None, defer: bool = False):
    """Fused head (dlrm_head_step): X [M, K] with the folded bias column, w [K] (updated in
    place by SGD when lr != 0 and dw is None).  ``defer``: the second launch (column sums,
    update, mean loss) becomes the returned role, pass 4 of a later gemm_group
    (dlrm_head_step_defer); w / dw / loss_out / workspace untouched until then."""
    M, K = X.shape
    need = _lib.query("dlrm_head_step_workspace_size", M, K)
    if workspace is None or workspace.numel() < need:
        workspace = _ws("head_step", need, X.device)
    _check_cuda(X, w, target)
    args = (M, K, _p(X), X.stride(0), _p(w), _p(target),
            LOSS_BCE if loss == "bce" else LOSS_MSE, float(clamp_lo), float(grad_scale),
            _p(prob), _p(dz), _p(loss_out), _p(dX), dX.stride(0) if dX is not None else 0,
            int(relu_mask), _p(dw), int(accumulate), float(lr), _p(workspace), workspace.numel())
    if defer:
        role = _lib.LaunchRole()
        _lib.call("dlrm_head_step_defer", *args, ctypes.byref(role), _stream(X.device))
        return role
    _lib.call("dlrm_head_step", *args, _stream(X.device))
    return prob, dz, loss_out


def outer_drelu(dz: torch.Tensor, w: torch.Tensor, X: Optional[torch.Tensor], relu_mask: bool,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    M = dz.shape[0]
    K = w.numel()
    if out is None:
        out = torch.empty((M, K), dtype=torch.float32, device=dz.device)
    _lib.call("dlrm_outer_drelu", M, K, _p(dz), _p(w), _p(X), X.stride(0) if X is not None else 0,
              int(relu_mask), _p(out), out.stride(0), _stream(dz.device))
    return out


def sigmoid_forward(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    x = x.contiguous()
    out = torch.empty_like(x) if out is None else out
    _lib.call("dlrm_sigmoid_forward", x.numel(), _p(x), _p(out), _stream(x.device))
    return out


def sigmoid_backward(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    dy = dy.contiguous()
    dx = torch.empty_like(dy)
    _lib.call("dlrm_sigmoid_backward", dy.numel(), _p(dy), _p(y), _p(dx), _stream(dy.device))
    return dx


def relu_backward(dy: torch.Tensor, y: torch.Tensor,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = dy * (y > 0) for 2-D row-strided operands (unit inner stride)."""
    if dy.dim() == 1:
        dy, y = dy.view(1, -1), y.reshape(1, -1)
        out = None if out is None else out.view(1, -1)
    if dy.stride(1) != 1 or y.stride(1) != 1:
        raise ValueError("relu_backward needs unit inner strides")
    M, K = dy.shape
    dx = torch.empty((M, K), dtype=torch.float32, device=dy.device) if out is None else out
    _lib.call("dlrm_relu_backward", M, K, _p(dy), dy.stride(0), _p(y), y.stride(0), _p(dx),
              dx.stride(0), _stream(dy.device))
    return dx


# ----------------------------------------------------------- optimizers ----
def sgd_update(param: torch.Tensor, grad: torch.Tensor, lr: float) -> None:
    _lib.call("dlrm_sgd_update", _p(param), _p(grad), param.numel(), float(lr),
              _stream(param.device))


def adagrad_update(param: torch.Tensor, grad: torch.Tensor, state_sum: torch.Tensor, clr: float,
                   eps: float, grad_scale: float = 1.0) -> None:
    """state_sum += g'^2; param -= clr * g' / (sqrt(state_sum) + eps) with g' = grad_scale * g
    (grad itself is not modified)."""
    if grad_scale != 1.0:
        _lib.call("dlrm_adagrad_update_scaled", _p(param), _p(grad), _p(state_sum),
                  param.numel(), float(grad_scale), float(clr), float(eps),
                  _stream(param.device))
        return
    _lib.call("dlrm_adagrad_update", _p(param), _p(grad), _p(state_sum), param.numel(),
              float(clr), float(eps), _stream(param.device))


def scale_(x: torch.Tensor, alpha: float) -> None:
    _lib.call("dlrm_scale_f32", _p(x), x.numel(), float(alpha), _stream(x.device))


# -------------------------------------------------------------- utility ----
def uniform_fill_(out: torch.Tensor, lo: float, hi: float, seed: int) -> torch.Tensor:
    _lib.call("dlrm_uniform_fill", _p(out), out.numel(), float(lo), float(hi),
              int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(out.device))
    return out


def uniform_int_fill_(out: torch.Tensor, hi: int, seed: int) -> torch.Tensor:
    _lib.call("dlrm_uniform_int_fill", _p(out), _bits(out), out.numel(), int(hi),
              int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(out.device))
    return out


def csr_from_tables(table_offsets: Sequence[torch.Tensor], table_nnz: Sequence[int], B: int,
                    out_dtype=torch.int32) -> torch.Tensor:
    """Device CSR builder: per-table int64 offsets [B] -> batched offsets [T*B+1]."""
    T = len(table_offsets)
    offs = [o if o.dtype == torch.int64 else o.long() for o in table_offsets]
    _check_cuda(*offs)
    out = torch.empty(T * B + 1, dtype=out_dtype, device=offs[0].device)
    ptrs = (ctypes.c_void_p * T)(*[o.data_ptr() for o in offs])
    nnz = (ctypes.c_int64 * T)(*[int(n) for n in table_nnz])
    _lib.call("dlrm_csr_from_tables", T, B, ptrs, nnz, _p(out),
              32 if out_dtype == torch.int32 else 64, _stream(offs[0].device))
    return out


def criteo_decode(records: torch.Tensor, n_dense: int = 13, n_sparse: int = 26,
                  max_ind_range: int = -1, batched: bool = False,
                  dense: Optional[torch.Tensor] = None, label: Optional[torch.Tensor] = None,
                  indices: Optional[torch.Tensor] = None,
                  offsets: Optional[torch.Tensor] = None):
    """Device decode of raw Criteo binary records int32 [n, 1+n_dense+n_sparse]
    (dlrm_criteo_decode; data_loader_terabyte.py:83-114).  Returns (dense [n, n_dense]
    log(x+1), lS_o, lS_i, label [n, 1]) in the reference's layouts: batched -> int32
    offsets [T*n+1] and int32 indices [T*n]; else int64 lS_o [T, n] = arange and int64
    lS_i [T, n].  ``dense`` may be a caller buffer (row stride >= n_dense); so may
    ``label`` (n fp32), ``indices`` and (batched) ``offsets``, e.g. the fixed buffers a
    captured step graph reads."""
    _check_cuda(records, dense, label, indices, offsets)
    nf = 1 + n_dense + n_sparse
    if records.dtype != torch.int32 or not records.is_contiguous() or records.numel() % nf:
        raise ValueError(f"criteo_decode: need contiguous int32 records of {nf} fields")
    n = records.numel() // nf
    dev = records.device
    if dense is None:
        dense = torch.empty((n, n_dense), dtype=torch.float32, device=dev)
    elif dense.shape[0] != n or dense.shape[1] < n_dense or dense.stride(1) != 1:
        raise ValueError("criteo_decode: dense buffer must be [n, >= n_dense] row-major")
    idt = torch.int32 if batched else torch.int64
    if label is None:
        label = torch.empty((n, 1), dtype=torch.float32, device=dev)
    if indices is None:
        indices = torch.empty(n_sparse * n, dtype=idt, device=dev)
    if offsets is None and batched:
        offsets = torch.empty(n_sparse * n + 1, dtype=torch.int32, device=dev)
    if (label.numel() != n or label.dtype != torch.float32 or not label.is_contiguous()
            or indices.numel() != n_sparse * n or indices.dtype != idt
            or not indices.is_contiguous()
            or (batched and (offsets.numel() != n_sparse * n + 1 or offsets.dtype != torch.int32
                             or not offsets.is_contiguous()))):
        raise ValueError("criteo_decode: label / indices / offsets buffers of the wrong shape")
    _lib.call("dlrm_criteo_decode", _p(records), n, n_dense, n_sparse, int(max_ind_range),
              _p(dense), dense.stride(0) if n else n_dense, _p(label), _p(indices),
              32 if batched else 64, _p(offsets), 32, _stream(dev))
    if batched:
        return dense, offsets, indices, label
    lS_o = torch.arange(n, device=dev).reshape(1, -1).repeat(n_sparse, 1)
    return dense, lS_o, indices.view(n_sparse, n), label
