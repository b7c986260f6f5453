"""CPU restatement of the reference DLRM hot path (ORACLE — test infrastructure only).

Each function cites the reference file:line it restates (YuxinxinChen/dlrm-yx).  The
floating-point path uses torch CPU fp32 ops exactly as the reference calls them
(nn.EmbeddingBag(mode="sum", sparse=True), nn.Linear, torch.bmm + tril gather,
MSELoss/BCELoss, torch.optim.SGD), the integer path (sharders, splits, CSR) is plain
Python/numpy.  Pinned by tests/test_oracle_golden.py against tests/golden/.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "get_splits", "shard", "get_my_slice", "get_split_lengths",
    "generate_uniform_input_batch", "generate_random_output_batch", "batched_csr",
    "distribute_batched", "init_emb_tables", "init_mlp", "embedding_bag_sum", "interact",
    "OracleDLRM", "QREmbeddingBagOracle", "RWSAdagradOracle", "distributed_step",
    "criteo_transform", "KAGGLE_ROWS", "TERABYTE_ROWS", "dequantize_rows",
    "embedding_bag_rows", "md_solver", "pr_embedding_bag",
]

# tools/visualize.py:949 (Kaggle) and :964 (Terabyte) row counts; Terabyte capped at 1e7
# the way the MLPerf config hashes it (--max-ind-range=10000000, bench/run_and_time.sh:17).
KAGGLE_ROWS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
               27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]
TERABYTE_ROWS = [10000000, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 10000000, 2953546,
                 403346, 10, 2208, 11938, 155, 4, 976, 14, 10000000, 10000000, 10000000, 585935,
                 12972, 108, 36]


# ------------------------------------------------------------- sharders ----
def get_splits(T: int, ndevices: int) -> List[int]:
    """sharders.py:3-9."""
    k, m = divmod(T, ndevices)
    return [k] * ndevices if m == 0 else [(k + 1) if i < m else k for i in range(ndevices)]


def shard(Es: Sequence[int], ndevices: int, alg: str = "naive") -> List[int]:
    """sharders.py:23-60: table -> device index."""
    T = len(Es)
    if alg == "naive":  # :30-32
        return [x % ndevices for x in range(T)]
    if alg == "naive_chunk":  # :35-42
        out: List[int] = []
        for d, s in enumerate(get_splits(T, ndevices)):
            out.extend([d] * s)
        return out
    if alg == "greedy":  # :45-54 (row-balanced, ties -> lowest rank)
        buckets = [0] * ndevices
        out = [0] * T
        for k, E in enumerate(Es):
            d = buckets.index(min(buckets))
            buckets[d] += int(E)
            out[k] = d
        return out
    if alg == "hardcode":  # :57-60
        return [0] + [1] * (T - 1)
    raise ValueError(f"sharder {alg!r} not found")


# -------------------------------------------------------- batch splits ----
def get_my_slice(n: int, rank: int, size: int) -> slice:
    """extend_distributed.py:47-51."""
    k, m = divmod(n, size)
    return slice(rank * k + min(rank, m), (rank + 1) * k + min(rank + 1, m), 1)


def get_split_lengths(n: int, rank: int, size: int):
    """extend_distributed.py:58-66 -> (my_len, splits or None)."""
    k, m = divmod(n, size)
    if m == 0:
        return k, None
    splits = [(k + 1) if i < m else k for i in range(size)]
    return splits[rank], splits


# ------------------------------------------------------------ synthetic ----
def generate_uniform_input_batch(m_den, ln_emb, n, num_indices_per_lookup, fixed,
                                 rng=np.random):
    """dlrm_data_pytorch.py:1109-1161 (numpy global RNG consumption order preserved)."""
    Xt = torch.tensor(rng.rand(n, m_den).astype(np.float32))
    lS_o, lS_i = [], []
    for size in ln_emb:
        offs, idxs = [], []
        offset = 0
        for _ in range(n):
            if fixed:
                group = np.int64(num_indices_per_lookup)
                if size < num_indices_per_lookup:
                    raise ValueError("fixed L with rows < L never terminates in the reference")
                while True:  # :1134-1138 redraw until exactly L unique
                    r = rng.random(group)
                    sg = np.unique(np.round(r * (size - 1)).astype(np.int64))
                    if sg.size == num_indices_per_lookup:
                        break
            else:
                r = rng.random(1)
                group = np.int64(np.round(max([1.0], r * min(size, num_indices_per_lookup))))
                r = rng.random(group)
                sg = np.unique(np.round(r * (size - 1)).astype(np.int64))
                group = np.int32(sg.size)
            offs.append(offset)
            idxs += sg.tolist()
            offset += group
        lS_o.append(torch.tensor(offs))
        lS_i.append(torch.tensor(idxs))
    return Xt, lS_o, lS_i


def generate_random_output_batch(n, num_targets, round_targets=False, rng=np.random):
    """dlrm_data_pytorch.py:1098-1105."""
    if round_targets:
        P = np.round(rng.rand(n, num_targets).astype(np.float32)).astype(np.float32)
    else:
        P = rng.rand(n, num_targets).astype(np.float32)
    return torch.tensor(P)


def batched_csr(lS_o: Sequence[torch.Tensor], lS_i: Sequence[torch.Tensor]):
    """Table-batched flatten, dlrm_data_pytorch.py:748-753 / 834-843:
    indices = cat(lS_i) (int32); offsets = cat(lS_o[t] + E_off[t]) ++ [E_off[T]] (int32)."""
    indices = torch.cat([x.view(-1) for x in lS_i], dim=0).int()
    E_off = [0] + np.cumsum([x.view(-1).shape[0] for x in lS_i]).tolist()
    offsets = torch.cat([x + y for x, y in zip(lS_o, E_off[:-1])] +
                        [torch.tensor([E_off[-1]])], dim=0).int()
    return offsets, indices


def distribute_batched(offsets: torch.Tensor, indices: torch.Tensor, B: int, T: int,
                       local_tables: Sequence[int]):
    """DLRM_Net.distribute_batched_emb_data, distributed branch (dlrm_s_pytorch.py:772-800):
    keep the local tables' bags, rebase each table's offsets onto the previous one's end."""
    L = int(indices.shape[0] / B / T)
    tmp = []
    for k in range(T):
        o = offsets[k * B:(k + 1) * B + 1]
        tmp.append((o - o[0], indices[k * B * L:(k + 1) * B * L]))
    tmp_o, tmp_i = [], []
    for k in local_tables:
        o, i = tmp[k]
        tmp_o.append(o if not tmp_o else o[1:] + tmp_o[-1][-1])
        tmp_i.append(i)
    return torch.cat(tmp_o, dim=0), torch.cat(tmp_i, dim=0)


# ----------------------------------------------------------------- init ----
def init_emb_tables(ln_emb, m, rng=np.random) -> List[np.ndarray]:
    """DLRM_Net.create_emb plain-EmbeddingBag init (dlrm_s_pytorch.py:300-308)."""
    return [rng.uniform(low=-np.sqrt(1 / n), high=np.sqrt(1 / n), size=(n, m)).astype(np.float32)
            for n in ln_emb]


def init_mlp(ln, rng=np.random):
    """DLRM_Net.create_mlp init (dlrm_s_pytorch.py:235-247): W ~ N(0, sqrt(2/(m+n))),
    b ~ N(0, sqrt(1/m)), drawn W then b per layer."""
    out = []
    for i in range(len(ln) - 1):
        n, m = int(ln[i]), int(ln[i + 1])
        W = rng.normal(0.0, np.sqrt(2 / (m + n)), size=(m, n)).astype(np.float32)
        b = rng.normal(0.0, np.sqrt(1 / m), size=m).astype(np.float32)
        out.append((W, b))
    return out


# ------------------------------------------------------------------ ops ----
def embedding_bag_sum(W: torch.Tensor, idx: torch.Tensor, off: torch.Tensor,
                      psw: Optional[torch.Tensor] = None) -> torch.Tensor:
    """nn.EmbeddingBag(mode='sum') as DLRM_Net.apply_emb calls it (dlrm_s_pytorch.py:571-576):
    off = B bag starts, the last bag ends at len(idx)."""
    return F.embedding_bag(idx, W, off, mode="sum", per_sample_weights=psw)


def dequantize_rows(packed: np.ndarray, bits: int, D: int) -> np.ndarray:
    """Row-wise quantized rows -> fp32 [rows, D] (the layout of
    torch.ops.quantized.embedding_bag_{byte,4bit}_prepack that DLRM_Net.quantize_embedding
    uses, dlrm_s_pytorch.py:609-625): 8-bit = D uint8 | fp32 scale | fp32 bias; 4-bit =
    ceil(D/2) bytes (element 2i = low nibble of byte i) | fp16 scale | fp16 bias.
    Returns (q, scale, bias) with q as float levels."""
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    if bits == 8:
        q = packed[:, :D].astype(np.float32)
        sb = packed[:, D:D + 8].copy().view(np.float32)
    else:
        nb = (D + 1) // 2
        by = packed[:, :nb]
        q = np.empty((packed.shape[0], 2 * nb), dtype=np.float32)
        q[:, 0::2] = by & 0xF
        q[:, 1::2] = by >> 4
        q = q[:, :D]
        sb = packed[:, nb:nb + 4].copy().view(np.float16).astype(np.float32)
    return q, sb[:, 0].copy(), sb[:, 1].copy()


def embedding_bag_rows(packed: np.ndarray, bits: int, D: int, idx: np.ndarray,
                       off: np.ndarray, psw: Optional[np.ndarray] = None) -> np.ndarray:
    """embedding_bag_{byte,4bit}_rowwise_offsets (dlrm_s_pytorch.py:554-567) restated in
    float32: per lookup, acc = fma(w*scale, q, acc + w*bias), in lookup order (off = B bag
    starts; the last bag ends at len(idx)).  Within fp32 rounding of the torch op."""
    q, sc, bi = dequantize_rows(packed, bits, D)
    B = len(off)
    out = np.zeros((B, D), dtype=np.float32)
    ends = list(off[1:]) + [len(idx)]
    for b in range(B):
        acc = np.zeros(D, dtype=np.float32)
        for l in range(int(off[b]), int(ends[b])):
            r = int(idx[l])
            w = np.float32(1.0 if psw is None else psw[l])
            acc = (np.float32(w * sc[r]) * q[r] + (acc + np.float32(w * bi[r]))).astype(np.float32)
        out[b] = acc
    return out


def md_solver(n: Sequence[int], alpha: float, d0: Optional[float] = None,
              B: Optional[float] = None, round_dim: bool = True, k=None) -> List[int]:
    """tricks/md_embedding_bag.py:20-60 (md_solver + alpha_power_rule + pow_2_round):
    per-table dims d_i = lambda * (n_i / k_i)^(-alpha), the smallest table (after a stable
    ascending sort) pinned to d0, others clamped at 1, rounded, optionally to a power of 2."""
    n_t = torch.tensor(list(n))
    ns, idx = torch.sort(n_t)
    kk = torch.as_tensor(k)[idx] if k is not None else torch.ones(len(ns))
    x = ns.type(torch.float) / kk
    if d0 is not None:
        lamb = d0 * (x[0].type(torch.float) ** alpha)
    elif B is not None:
        lamb = B / torch.sum(x.type(torch.float) ** (1 - alpha))
    else:
        raise ValueError("Must specify either d0 or B")
    d = torch.ones(len(x)) * lamb * (x.type(torch.float) ** (-alpha))
    for i in range(len(d)):
        if i == 0 and d0 is not None:
            d[i] = d0
        else:
            d[i] = 1 if d[i] < 1 else d[i]
    d = torch.round(d).type(torch.long)
    if round_dim:
        d = 2 ** torch.round(torch.log2(d.type(torch.float)))
    undo = [0] * len(idx)
    for i, v in enumerate(idx):
        undo[v] = i
    return [int(v) for v in d[undo].tolist()]


def pr_embedding_bag(W: torch.Tensor, P: Optional[torch.Tensor], idx: torch.Tensor,
                     off: torch.Tensor, psw: Optional[torch.Tensor] = None) -> torch.Tensor:
    """PrEmbeddingBag.forward (tricks/md_embedding_bag.py:81-85): sum pooling of the
    dim-m_i table, then the bias-free projection to the base dim (P [base, m_i], or None
    for the identity)."""
    y = F.embedding_bag(idx, W, off, mode="sum", per_sample_weights=psw)
    return y if P is None else y @ P.t()


def interact(x: torch.Tensor, ly: Sequence[torch.Tensor], op: str = "dot",
             itself: bool = False) -> torch.Tensor:
    """DLRM_Net.interact_features, non-batched branch (dlrm_s_pytorch.py:627-665)."""
    B, d = x.shape
    if op == "dot":
        T = torch.cat([x] + list(ly), dim=1).view((B, -1, d))
        Z = torch.bmm(T, torch.transpose(T, 1, 2))
        _, ni, nj = Z.shape
        li, lj = torch.tril_indices(ni, nj, offset=0 if itself else -1)
        return torch.cat([x, Z[:, li, lj]], dim=1)
    if op == "cat":
        return torch.cat([x] + list(ly), dim=1)
    raise ValueError(op)


# -------------------------------------------------------------- model ----
class OracleDLRM(nn.Module):
    """DLRM_Net restated for the single-process (sequential_forward, :732-770) path.

    Construction draws numpy's global RNG in the reference order: all embedding
    tables (create_emb, :469-474) and then the bottom and top MLPs (:495-496).
    """

    def __init__(self, m_spa, ln_emb, ln_bot, ln_top, arch_interaction_op="dot",
                 arch_interaction_itself=False, sigmoid_bot=-1, sigmoid_top=None,
                 loss_function="mse", loss_threshold=0.0, rng=np.random, tables=None):
        super().__init__()
        self.m_spa = m_spa
        self.ln_emb = list(ln_emb)
        self.ln_bot = list(ln_bot)
        self.ln_top = list(ln_top)
        self.op = arch_interaction_op
        self.itself = arch_interaction_itself
        self.loss_threshold = loss_threshold
        self.loss_function = loss_function
        sigmoid_top = len(ln_top) - 2 if sigmoid_top is None else sigmoid_top
        Ws = tables if tables is not None else init_emb_tables(ln_emb, m_spa, rng)
        self.emb_l = nn.ModuleList()
        for n, W in zip(ln_emb, Ws):
            e = nn.EmbeddingBag(int(n), m_spa, mode="sum", sparse=True)
            e.weight.data = torch.tensor(W)
            self.emb_l.append(e)
        self.bot_l = self._mlp(ln_bot, sigmoid_bot, rng)
        self.top_l = self._mlp(ln_top, sigmoid_top, rng)
        if loss_function == "mse":
            self.loss_fn = nn.MSELoss(reduction="mean")
        elif loss_function == "bce":
            self.loss_fn = nn.BCELoss(reduction="mean")
        else:
            raise ValueError(loss_function)

    @staticmethod
    def _mlp(ln, sigmoid_layer, rng):
        layers = []
        for i, (W, b) in enumerate(init_mlp(ln, rng)):
            L = nn.Linear(W.shape[1], W.shape[0], bias=True)
            L.weight.data = torch.tensor(W)
            L.bias.data = torch.tensor(b)
            layers.append(L)
            layers.append(nn.Sigmoid() if i == sigmoid_layer else nn.ReLU())
        return nn.Sequential(*layers)

    def apply_emb(self, lS_o, lS_i):
        """:526-587 (sum pooling, D split into ln_bot[-1] chunks)."""
        ly = [self.emb_l[k](lS_i[k], lS_o[k]) for k in range(len(self.emb_l))]
        d = self.ln_bot[-1]
        out = []
        for y in ly:
            out.extend([y] if y.shape[1] == d else list(y.split(d, dim=1)))
        return out

    def forward(self, X, lS_o, lS_i):
        x = self.bot_l(X)
        ly = self.apply_emb(lS_o, lS_i)
        z = interact(x, ly, self.op, self.itself)
        p = self.top_l(z)
        if 0.0 < self.loss_threshold < 1.0:
            p = torch.clamp(p, min=self.loss_threshold, max=1.0 - self.loss_threshold)
        return p

    def train_step(self, X, lS_o, lS_i, T, lr):
        """One reference training iteration (dlrm_s_pytorch.py:1886-1934) with SGD."""
        Z = self(X, lS_o, lS_i)
        E = self.loss_fn(Z, T)
        for p in self.parameters():
            p.grad = None
        E.backward()
        with torch.no_grad():
            for p in self.parameters():
                if p.grad is not None:
                    p.add_(p.grad, alpha=-lr)
        return Z.detach(), E.detach()


def distributed_step(model: OracleDLRM, W: int, device_indices: Sequence[int], X, lS_o, lS_i,
                     T, lr: float, optimizer=None):
    """distributed_forward semantics (dlrm_s_pytorch.py:686-730, extend_distributed.py:
    405-508, DDP :1626-1633) simulated in one process for W ranks:
      * the all-to-all delivers features in RANK-MAJOR table order;
      * rank s's loss is the mean over its batch slice; embedding gradients are the SUM of
        the per-rank gradients (a2a backward, no averaging -> W x the global-mean grad);
      * dense (MLP) gradients are averaged over ranks (DDP).
    Returns the list of per-rank Z and losses; updates the model in place: SGD at ``lr``, or
    ``optimizer`` (e.g. RWSAdagradOracle over model.parameters(), the driver's C4 run
    :1636-1666) stepped on those gradients (its own lr; ``lr`` unused)."""
    B = X.shape[0]
    order = [t for r in range(W) for t in range(len(model.emb_l)) if device_indices[t] == r]
    ly = [model.emb_l[t](lS_i[t], lS_o[t]) for t in range(len(model.emb_l))]
    Zs, Es = [], []
    total = 0.0
    for s in range(W):
        sl = get_my_slice(B, s, W)
        x = model.bot_l(X[sl])
        z = interact(x, [ly[t][sl] for t in order], model.op, model.itself)
        p = model.top_l(z)
        E = model.loss_fn(p, T[sl])
        total = total + E
        Zs.append(p.detach())
        Es.append(E.detach())
    for p in model.parameters():
        p.grad = None
    total.backward()
    with torch.no_grad():
        for name, p in model.named_parameters():
            if p.grad is None:
                continue
            g = p.grad if name.startswith("emb_l") else p.grad / W
            if optimizer is None:
                p.add_(g, alpha=-lr)
            else:
                p.grad = g
        if optimizer is not None:
            optimizer.step()
    return Zs, Es


# ------------------------------------------------------------------- QR ----
class QREmbeddingBagOracle(nn.Module):
    """QREmbeddingBag (tricks/qr_embedding_bag.py:113-174), sum mode, sparse grads."""

    def __init__(self, num_categories, embedding_dim, num_collisions, operation="mult",
                 weight_q=None, weight_r=None):
        super().__init__()
        self.c = num_collisions
        self.operation = operation
        nq = int(np.ceil(num_categories / num_collisions))
        self.weight_q = nn.Parameter(torch.tensor(weight_q) if weight_q is not None
                                     else torch.empty(nq, embedding_dim))
        self.weight_r = nn.Parameter(torch.tensor(weight_r) if weight_r is not None
                                     else torch.empty(num_collisions, embedding_dim))
        if weight_q is None:  # :152-154 uniform_(w, a=sqrt(1/n)) -> U[sqrt(1/n), 1)
            nn.init.uniform_(self.weight_q, np.sqrt(1 / num_categories))
            nn.init.uniform_(self.weight_r, np.sqrt(1 / num_categories))

    @staticmethod
    def split(idx, c):
        """:157-158 — true division in fp32, truncated; remainder with the divisor's sign."""
        return (idx / c).long(), torch.remainder(idx, c).long()

    def forward(self, idx, off):
        q, r = self.split(idx, self.c)
        eq = F.embedding_bag(q, self.weight_q, off, mode="sum", sparse=True)
        er = F.embedding_bag(r, self.weight_r, off, mode="sum", sparse=True)
        if self.operation == "concat":
            return torch.cat((eq, er), dim=1)
        if self.operation == "add":
            return eq + er
        return eq * er


class RWSAdagradOracle:
    """RWSAdagrad (optim/rwsadagrad.py:56-122): sparse rows get row-wise momentum
    (mean of squared coalesced grad), dense params plain Adagrad."""

    def __init__(self, params, lr=1e-2, lr_decay=0.0, eps=1e-10, initial_accumulator_value=0.0):
        self.params = list(params)
        self.lr, self.lr_decay, self.eps = lr, lr_decay, eps
        self.init = initial_accumulator_value
        self.state = {id(p): {"step": 0} for p in self.params}

    def step(self):
        for p in self.params:
            if p.grad is None:
                continue
            st = self.state[id(p)]
            if "momentum" not in st and "sum" not in st:
                if p.grad.is_sparse:
                    st["momentum"] = torch.full([p.shape[0]], self.init, dtype=p.dtype)
                else:
                    st["sum"] = torch.full_like(p.data, self.init)
            st["step"] += 1
            clr = self.lr / (1.0 + (st["step"] - 1.0) * self.lr_decay)
            g = p.grad
            if g.is_sparse:
                g = g.coalesce()
                gi, gv = g._indices(), g._values()
                if gv.numel() == 0:
                    continue
                rows = gi[0]
                st["momentum"].index_add_(0, rows, gv.pow(2).mean(dim=1))
                std = st["momentum"][rows].sqrt().add_(self.eps)
                p.data.index_add_(0, rows, gv / std.view(-1, 1), alpha=-clr)
            else:
                st["sum"].addcmul_(g, g, value=1.0)
                std = st["sum"].sqrt().add_(self.eps)
                p.data.addcdiv_(g, std, value=-clr)

    def zero_grad(self):
        for p in self.params:
            p.grad = None


def criteo_transform(records: np.ndarray, max_ind_range: int = -1, batched: bool = False,
                     n_dense: int = 13):
    """CriteoBinDataset.__getitem__ -> _transform_features(flag_input_torch_tensor=True)
    (data_loader_terabyte.py:237-252, 83-114) on an int32 record block [n, 1+13+26]:
    X = log(float(x_int) + 1); x_cat % max_ind_range (torch floor mod) when > 0;
    lS_o = arange(n) per table, lS_i = x_cat.t(); batched: int32 cat(lS_i) and
    offsets cat(lS_o[t] + t*n) ++ [T*n]."""
    t = torch.from_numpy(np.ascontiguousarray(records, dtype=np.int32)).view(-1, 1 + n_dense + 26)
    x_int, x_cat, y = t[:, 1:1 + n_dense], t[:, 1 + n_dense:], t[:, 0]
    if max_ind_range > 0:
        x_cat = x_cat % max_ind_range
    X = torch.log(x_int.clone().detach().type(torch.float) + 1)
    x_cat = x_cat.clone().detach().type(torch.long)
    y = y.clone().detach().type(torch.float32).view(-1, 1)
    n, T = x_cat.shape
    lS_o = torch.arange(n).reshape(1, -1).repeat(T, 1)
    lS_i = x_cat.t()
    if batched:
        indices = torch.cat([x.reshape(-1) for x in lS_i]).int()
        starts = [0] + np.cumsum([x.numel() for x in lS_i]).tolist()
        offsets = torch.cat([o + s for o, s in zip(lS_o, starts[:-1])]
                            + [torch.tensor([starts[-1]])]).int()
        lS_i, lS_o = indices, offsets
    return X, lS_o, lS_i, y
