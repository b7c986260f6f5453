"""nn.Module mirrors of the reference's embedding / MLP building blocks, on HIP kernels.

* ``HipEmbeddingBag``        — nn.EmbeddingBag(n, m, mode="sum", sparse=...) equivalent
                               (dlrm_s_pytorch.py:300-308); a member of a
* ``HipEmbeddingBagList``    — the DLRM_Net.emb_l ModuleList whose plain tables share ONE
                               flat [sum rows, D] device buffer, so apply_emb is a single
                               table-batched kernel launch instead of T launches;
* ``TableBatchedEmbeddingBags`` — the external TBE API used by --batched-emb
                               (dlrm_s_pytorch.py:321-334): forward(indices, offsets[T*B+1])
                               -> [B, T, D], optimizer fused into the backward;
* ``HipQREmbeddingBag``      — tricks/qr_embedding_bag.py QREmbeddingBag;
* ``HipMLP``                 — the nn.Sequential of create_mlp, run as one fused Function.
"""
from __future__ import annotations

import enum
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import ops
from .functional import EmbeddingBagsFunction, MLPFunction


class Optimizer(enum.Enum):
    """table_batched_embeddings_ops.Optimizer (the members DLRM uses)."""
    SGD = 1
    APPROX_SGD = 2
    EXACT_ROWWISE_ADAGRAD = 3


# ------------------------------------------------------------ embeddings ----
class HipEmbeddingBag(nn.Module):
    """One table of a HipEmbeddingBagList; ``weight`` is a view of the list's flat buffer."""

    def __init__(self, num_embeddings: int, embedding_dim: int, weight: torch.Tensor,
                 sparse: bool = True):
        super().__init__()
        self.num_embeddings = int(num_embeddings)
        self.embedding_dim = int(embedding_dim)
        self.mode = "sum"
        self.sparse = sparse
        self.weight = Parameter(weight)

    def extra_repr(self):
        return f"{self.num_embeddings}, {self.embedding_dim}, mode='sum'"


class HipEmbeddingBagList(nn.ModuleList):
    """ModuleList of tables; plain HipEmbeddingBag members share one flat buffer."""

    def __init__(self, modules: Sequence[nn.Module], weight_flat: Optional[torch.Tensor],
                 row_ranges: Sequence[tuple], plain_index: Sequence[int], D: int):
        super().__init__(modules)
        ops.check_tbe_rows(row_ranges[-1][1] if row_ranges else 0, "HipEmbeddingBagList")
        self.weight_flat = weight_flat
        self.row_ranges = list(row_ranges)      # per plain table: (start, end) rows
        self.plain_index = list(plain_index)    # table ids of the plain tables
        self.D = D
        self.T = len(self.plain_index)
        self.grad_mode = "sparse"
        self._row_base = None

    @property
    def row_base(self) -> torch.Tensor:
        dev = self.weight_flat.device
        if self._row_base is None or self._row_base.device != dev:
            self._row_base = torch.tensor([0] + [b for _, b in self.row_ranges],
                                          dtype=torch.int64, device=dev)
        return self._row_base

    def _apply(self, fn, recurse=True):
        # Move the shared buffer once and re-point every table's Parameter at its view
        # (the default per-parameter move would break the sharing).
        plain = set(self.plain_index)
        for i, m in enumerate(self):
            if i not in plain:
                m._apply(fn)
        if self.weight_flat is not None:
            self.weight_flat = fn(self.weight_flat)
            for t, (a, b) in zip(self.plain_index, self.row_ranges):
                self[t].weight.data = self.weight_flat[a:b]
        self._row_base = None
        return self

    def plain_params(self) -> List[Parameter]:
        return [self[t].weight for t in self.plain_index]


def make_embedding_list(ln_emb, D, tables: Sequence[Optional[np.ndarray]],
                        extra: Optional[dict] = None, sparse: bool = True) -> HipEmbeddingBagList:
    """Build emb_l with the given initial weights (numpy fp32 per table); ``extra`` maps
    table id -> a module used instead of a plain table (QR tables)."""
    extra = extra or {}
    plain = [t for t in range(len(ln_emb)) if t not in extra]
    rows = [int(ln_emb[t]) for t in plain]
    total = int(sum(rows))
    flat = torch.empty((max(total, 1), D), dtype=torch.float32)
    ranges, o = [], 0
    for t, n in zip(plain, rows):
        if tables[t] is not None:
            flat[o:o + n] = torch.as_tensor(tables[t])
        ranges.append((o, o + n))
        o += n
    mods: List[nn.Module] = []
    pi = 0
    for t in range(len(ln_emb)):
        if t in extra:
            mods.append(extra[t])
        else:
            a, b = ranges[pi]
            mods.append(HipEmbeddingBag(b - a, D, flat[a:b], sparse))
            pi += 1
    lst = HipEmbeddingBagList(mods, flat, ranges, plain, D)
    lst.grad_mode = "sparse" if sparse else "dense"
    return lst


class TableBatchedEmbeddingBags(nn.Module):
    """Drop-in for table_batched_embeddings_ops.TableBatchedEmbeddingBags as the reference
    constructs it (dlrm_s_pytorch.py:321-334) and calls it (:589-591):
    module(indices int32 [N], offsets int32 [T*B+1]) -> [B, T, D], with the optimizer
    (exact SGD, or exact row-wise Adagrad) applied inside the backward."""

    def __init__(self, num_tables: int, num_embeddings: Sequence[int], embedding_dim: int,
                 optimizer: Optimizer = Optimizer.SGD, learning_rate: float = 0.01,
                 eps: float = 1.0e-8, stochastic_rounding: bool = False, tables=None,
                 seed: int = 0):
        super().__init__()
        Es = [int(e) for e in num_embeddings]
        assert num_tables == len(Es), "num_tables must match num_embeddings"
        ops.check_tbe_rows(sum(Es), "TableBatchedEmbeddingBags")
        if stochastic_rounding:
            raise ValueError("stochastic rounding applies to fp16 tables only (fp32 here)")
        self.T = num_tables
        self.D = int(embedding_dim)
        self.optimizer = optimizer
        self.learning_rate = float(learning_rate)
        self.eps = float(eps)
        total = int(sum(Es))
        self.weights = Parameter(torch.empty(total, self.D), requires_grad=True)
        self.row_ranges = []
        o = 0
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for t, n in enumerate(Es):
                if tables is not None:
                    self.weights[o:o + n] = torch.as_tensor(tables[t])
                else:
                    a = float(np.sqrt(1.0 / n))
                    self.weights[o:o + n].uniform_(-a, a, generator=g)
                self.row_ranges.append((o, o + n))
                o += n
        self.register_buffer("table_offsets", torch.tensor([0] + [b for _, b in self.row_ranges],
                                                           dtype=torch.int64))
        self.register_buffer("momentum", torch.zeros(total) if optimizer ==
                             Optimizer.EXACT_ROWWISE_ADAGRAD else torch.zeros(0))
        self.grad_mode = "fused"

    # EmbeddingBagsFunction protocol
    @property
    def weight_flat(self):
        return self.weights.data

    @property
    def row_base(self):
        return self.table_offsets

    def fused_update(self, indices, offsets, grad, psw, B):
        if self.optimizer == Optimizer.EXACT_ROWWISE_ADAGRAD:
            ops.tbe_backward("rowwise_adagrad", self.weights.data, self.table_offsets, self.T, B,
                             indices, offsets, grad, lr=self.learning_rate, eps=self.eps,
                             momentum=self.momentum, per_sample_weights=psw)
        else:
            ops.tbe_backward("sgd", self.weights.data, self.table_offsets, self.T, B, indices,
                             offsets, grad, lr=self.learning_rate, per_sample_weights=psw)

    def split_embedding_weights(self) -> List[torch.Tensor]:
        return [self.weights.data[a:b] for a, b in self.row_ranges]

    def forward(self, indices, offsets, per_sample_weights=None):
        return EmbeddingBagsFunction.apply(self, None, indices, offsets, per_sample_weights,
                                           self.weights)


class SplitTableBatchedEmbeddingBags(nn.Module):
    """FP16-weight table-batched EmbeddingBag with exact SGD fused into the backward: the
    module DLRM_Net.create_emb_fbgemm builds (fbgemm_gpu's
    SplitTableBatchedEmbeddingBagsCodegen with weights_precision=FP16, OptimType.EXACT_SGD,
    dlrm_s_pytorch.py:337-366) and apply_emb_fbgemm calls (:593-598):
    module(indices, offsets[T*B+1], per_sample_weights=None) -> [B, T*D] fp32.

    Forward: dlrm_tbe_forward_rows (F16 rows, fp32 accumulation).  Backward:
    dlrm_tbe_backward_sgd_f16 (deterministic per-row fp32 gradient sum, round-to-nearest
    fp16 store).  fbgemm_gpu itself is not in the reference tree, so its init bound, its
    LFU cache and its stochastic rounding are not reproduced (parity unpinned against it);
    tables are drawn U(+-sqrt(1/n)) like the other DLRM paths."""

    def __init__(self, embedding_specs, learning_rate: float = 0.01, eps: float = 1.0e-8,
                 tables=None, seed: int = 0, device=None, **unused):
        super().__init__()
        Es = [int(e) for e, *_ in embedding_specs]
        Ds = {int(d) for _, d, *_ in embedding_specs}
        if len(Ds) != 1:
            raise NotImplementedError("mixed embedding dims in one fp16 TBE")
        self.T = len(Es)
        self.D = Ds.pop()
        self.learning_rate = float(learning_rate)
        self.eps = float(eps)
        self.row_format = ops.ROWS_F16
        total = int(sum(Es))
        ops.check_tbe_rows(total, "SplitTableBatchedEmbeddingBags")
        w = torch.empty(total, self.D)
        self.row_ranges = []
        o = 0
        g = torch.Generator().manual_seed(seed)
        for t, n in enumerate(Es):
            if tables is not None:
                w[o:o + n] = torch.as_tensor(tables[t])
            else:
                a = float(np.sqrt(1.0 / n))
                w[o:o + n].uniform_(-a, a, generator=g)
            self.row_ranges.append((o, o + n))
            o += n
        self.weights = Parameter(w.half(), requires_grad=True)
        self.register_buffer("table_offsets", torch.tensor([0] + [b for _, b in self.row_ranges],
                                                           dtype=torch.int64))
        self.grad_mode = "fused"
        if device is not None:
            self.to(device)

    @property
    def weight_flat(self):
        return self.weights.data

    @property
    def row_base(self):
        return self.table_offsets

    def fused_update(self, indices, offsets, grad, psw, B):
        ops.tbe_backward("sgd", self.weights.data, self.table_offsets, self.T, B, indices,
                         offsets, grad, lr=self.learning_rate, per_sample_weights=psw)

    def split_embedding_weights(self) -> List[torch.Tensor]:
        return [self.weights.data[a:b] for a, b in self.row_ranges]

    def forward(self, indices, offsets, per_sample_weights=None):
        B = (offsets.numel() - 1) // self.T
        out = EmbeddingBagsFunction.apply(self, None, indices, offsets, per_sample_weights,
                                          self.weights)
        return out.reshape(B, self.T * self.D)


class _SingleTable:
    """EmbeddingBagsFunction adapter for one standalone weight matrix."""

    def __init__(self, weight: torch.Tensor, grad_mode: str = "sparse"):
        self.weight_flat = weight.data
        self.T = 1
        self.D = weight.shape[1]
        self.row_ranges = [(0, weight.shape[0])]
        self.row_base = torch.tensor([0, weight.shape[0]], dtype=torch.int64,
                                     device=weight.device)
        self.grad_mode = grad_mode


def single_table_lookup(weight: Parameter, indices: torch.Tensor, bag_offsets: torch.Tensor,
                        per_sample_weights=None, sparse: bool = True) -> torch.Tensor:
    """nn.functional.embedding_bag(sum) on one table: bag_offsets are the B starts of the
    reference layout (the last bag ends at len(indices)) -> [B, D]."""
    B = bag_offsets.numel()
    off = ops.csr_from_tables([bag_offsets], [indices.numel()], B)
    m = _SingleTable(weight, "sparse" if sparse else "dense")
    out = EmbeddingBagsFunction.apply(m, [indices.numel()], indices, off, per_sample_weights,
                                      weight)
    return out.view(B, -1)


class HipStandaloneEmbeddingBag(nn.Module):
    """One plain table kept outside the list's shared buffer (a --load-processed table
    whose dim differs from the shared buffer's): nn.EmbeddingBag(n, m, mode="sum",
    sparse=True) semantics on the TBE kernel; ``weight`` as the reference's."""

    def __init__(self, num_embeddings: int, embedding_dim: int, weight, sparse: bool = True):
        super().__init__()
        self.num_embeddings = int(num_embeddings)
        self.embedding_dim = int(embedding_dim)
        self.mode = "sum"
        self.sparse = sparse
        self.weight = Parameter(torch.as_tensor(weight))

    def forward(self, input, offsets=None, per_sample_weights=None):
        return single_table_lookup(self.weight, input, offsets, per_sample_weights, self.sparse)

    def extra_repr(self):
        return f"{self.num_embeddings}, {self.embedding_dim}, mode='sum'"


class QRCombine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, op, eq, er):
        ctx.op = op
        ctx.save_for_backward(eq, er)
        return ops.qr_combine_forward(op, eq.contiguous(), er.contiguous())

    @staticmethod
    def backward(ctx, g):
        eq, er = ctx.saved_tensors
        geq, ger = ops.qr_combine_backward(ctx.op, eq.contiguous(), er.contiguous(), g)
        return None, geq, ger


class HipQREmbeddingBag(nn.Module):
    """QREmbeddingBag (tricks/qr_embedding_bag.py:113-174), sum mode: the quotient/remainder
    split (float division, truncated) runs on device, each half is a table-batched
    lookup and the combine (mult | add | concat) an elementwise kernel."""

    def __init__(self, num_categories, embedding_dim, num_collisions, operation="mult",
                 mode="sum", sparse=True, _weight=None):
        super().__init__()
        assert operation in ("concat", "mult", "add"), "Not valid operation!"
        assert mode == "sum", "only sum pooling is on the DLRM path"
        self.num_categories = int(num_categories)
        self.embedding_dim = [int(embedding_dim)] * 2
        self.num_collisions = int(num_collisions)
        self.operation = operation
        self.mode = mode
        self.sparse = sparse
        nq = int(np.ceil(num_categories / num_collisions))
        self.num_embeddings = [nq, self.num_collisions]
        if _weight is None:
            self.weight_q = Parameter(torch.empty(nq, embedding_dim))
            self.weight_r = Parameter(torch.empty(num_collisions, embedding_dim))
            # :152-154 nn.init.uniform_(w, sqrt(1/n)) -> U[sqrt(1/n), 1)
            nn.init.uniform_(self.weight_q, np.sqrt(1 / self.num_categories))
            nn.init.uniform_(self.weight_r, np.sqrt(1 / self.num_categories))
        else:
            self.weight_q = Parameter(torch.as_tensor(_weight[0]))
            self.weight_r = Parameter(torch.as_tensor(_weight[1]))

    def forward(self, input, offsets=None, per_sample_weights=None):
        q, r = ops.qr_split_indices(input, self.num_collisions)
        eq = single_table_lookup(self.weight_q, q, offsets, per_sample_weights, self.sparse)
        er = single_table_lookup(self.weight_r, r, offsets, per_sample_weights, self.sparse)
        return QRCombine.apply(self.operation, eq, er)


class HipPrEmbeddingBag(nn.Module):
    """PrEmbeddingBag (tricks/md_embedding_bag.py:61-85): a table of dim embedding_dim
    pooled by the TBE kernel, then projected to base_dim by a bias-free Linear on the GEMM
    kernel (identity when the dims are equal).  The constructor builds the same torch
    modules in the same order as the reference (nn.EmbeddingBag, xavier_uniform_,
    nn.Linear, xavier_uniform_), so the torch RNG stream and the projection init match
    it under a seed; state_dict keys are the reference's (embs.weight, proj.weight)."""

    def __init__(self, num_embeddings, embedding_dim, base_dim):
        super().__init__()
        ref = nn.EmbeddingBag(num_embeddings, embedding_dim, mode="sum", sparse=True)
        nn.init.xavier_uniform_(ref.weight)
        self.embs = HipEmbeddingBag(num_embeddings, embedding_dim, ref.weight.data.clone(),
                                    sparse=True)
        self.base_dim = int(base_dim)
        if embedding_dim < base_dim:
            self.proj = nn.Linear(embedding_dim, base_dim, bias=False)
            nn.init.xavier_uniform_(self.proj.weight)
        elif embedding_dim == base_dim:
            self.proj = nn.Identity()
        else:
            raise ValueError("Embedding dim " + str(embedding_dim) + " > base dim " +
                             str(base_dim))

    def forward(self, input, offsets=None, per_sample_weights=None):
        y = single_table_lookup(self.embs.weight, input, offsets, per_sample_weights,
                                self.embs.sparse)
        if isinstance(self.proj, nn.Identity):
            return y
        zero_bias = torch.zeros(self.base_dim, dtype=y.dtype, device=y.device)
        return MLPFunction.apply(y, ("none",), self.proj.weight, zero_bias)


# ------------------------------------------------------------------- MLP ----
class HipMLP(nn.Sequential):
    """The nn.Sequential[Linear, ReLU|Sigmoid]* built by create_mlp; forward runs all layers
    through one MLPFunction (state_dict keys unchanged: '0.weight', '0.bias', ...)."""

    def forward(self, x):
        acts, params = [], []
        mods = list(self)
        for i, m in enumerate(mods):
            if isinstance(m, nn.Linear):
                nxt = mods[i + 1] if i + 1 < len(mods) else None
                acts.append("relu" if isinstance(nxt, nn.ReLU) else
                            "sigmoid" if isinstance(nxt, nn.Sigmoid) else "none")
                params += [m.weight, m.bias]
        return MLPFunction.apply(x, tuple(acts), *params)
