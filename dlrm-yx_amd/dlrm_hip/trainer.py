"""Fused DLRM training step on MI355X: every FLOP and byte of the step goes through the
HIP kernels of libdlrm_hip.so; torch provides device memory, streams and RCCL.

One step = the reference iteration (dlrm_s_pytorch.py:1886-1934): forward
(sequential_forward :732-770 or distributed_forward :686-730), loss, backward and the
optimizer update.  Layout decisions (MI355X-first):

* All local embedding tables live row-concatenated in ONE [sum rows, D] fp32 buffer with
  64-bit row bases (C3 = 54 M rows x 128 = 27.7 GB, resident in HBM); the batch is the
  reference's table-batched CSR (int32 offsets [T*B+1], int32 indices).
* All MLP parameters live in ONE flat fp32 bucket (bottom then top, W then b per layer)
  so the data-parallel gradient is one RCCL all-reduce and the dense update one kernel.
  Every layer's input width is padded to a multiple of 4 floats (zero columns in both
  the activation and the weight) so every GEMM operand row is 16-B aligned.
* Single GPU: the optimizer is fused into the backward — wgrad GEMMs run with the SGD
  epilogue (W -= lr * dY^T X after dX = dY W has consumed the old W), bias columns sums
  apply their update, the embedding backward applies exact SGD per unique row.
* Multi GPU (one process per GPU, RCCL over xGMI): tables are sharded table-wise with the
  reference sharders; pooled embeddings go through one all_to_all_single per direction
  (rank-major feature order, the W x embedding gradient of the reference is reproduced);
  the bottom MLP overlaps the forward exchange, the backward exchange overlaps the bottom
  MLP backward, and the dense all-reduce overlaps the embedding update.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch
from torch.autograd.profiler import record_function

from . import ops
from .sharders import shard


def _pad4(n: int) -> int:
    return (int(n) + 3) // 4 * 4


@dataclass
class TrainerConfig:
    m_spa: int
    ln_emb: Sequence[int]
    ln_bot: Sequence[int]
    ln_top: Sequence[int]          # full top widths (first = number of interactions)
    arch_interaction_op: str = "dot"
    arch_interaction_itself: bool = False
    loss_function: str = "mse"     # mse | bce
    loss_threshold: float = 0.0
    learning_rate: float = 0.01
    emb_learning_rate: Optional[float] = None  # default: learning_rate
    optimizer: str = "sgd"         # sgd | rwsadagrad
    adagrad_eps: float = 1e-10
    sharder: str = "greedy"
    allocation: Optional[Sequence[int]] = None
    # QR compositional embeddings (--qr-flag, dlrm_s_pytorch.py:282-290): tables with more
    # than qr_threshold rows become a quotient table (ceil(n/c) rows) and a remainder table
    # (c rows) combined by qr_operation (mult | add)
    qr_flag: bool = False
    qr_collisions: int = 4
    qr_operation: str = "mult"
    qr_threshold: int = 200


@dataclass
class Batch:
    X: torch.Tensor        # [B_local, Kp0] dense input (padded, zero pad columns)
    offsets: torch.Tensor  # [T_local*B + 1] int32 CSR of the local tables, full batch
    indices: torch.Tensor  # int32 table-local rows
    target: torch.Tensor   # [B_local] fp32
    max_per_table: int = 0  # upper bound on one table's lookups (0 = unknown)
    one_hot: bool = False   # every bag holds exactly one index (offsets = arange)


@dataclass
class _Layer:
    N: int
    K: int
    Kp: int
    Np: int
    W: torch.Tensor
    b: torch.Tensor
    gW: Optional[torch.Tensor] = None
    gb: Optional[torch.Tensor] = None
    sumW: Optional[torch.Tensor] = None  # Adagrad state views
    sumb: Optional[torch.Tensor] = None


class DLRMTrainer:
    def __init__(self, cfg: TrainerConfig, device="cuda:0", rank: int = 0, world_size: int = 1,
                 process_group=None, seed: int = 0, init: bool = True, comm=None,
                 force_dist: bool = False):
        """``comm``: the step's collectives (default: TorchComm over ``process_group``, the
        dense all-reduce on a second group of the same ranks); EmulatedComm runs rank
        ``rank`` of ``world_size`` alone on one GPU (bench --emulate-world).
        ``force_dist``: the multi-GPU schedule (all-to-all, gradient bucket, all-reduce)
        even at world_size 1, on a 1-rank group (its tests run RCCL on one GPU)."""
        self.cfg = cfg
        self.dev = torch.device(device)
        self.rank, self.world = rank, world_size
        self.pg = process_group
        self.distributed = world_size > 1 or bool(force_dist)
        if self.distributed and comm is None:
            if process_group is None:
                raise ValueError("the multi-GPU schedule needs a process group (or a comm)")
            comm = TorchComm(process_group)
        self.comm = comm
        D = int(cfg.m_spa)
        if int(cfg.ln_bot[-1]) != D:
            raise ValueError("trainer needs ln_bot[-1] == m_spa (the reference splits wider "
                             "tables into D-sized features; not on this path)")
        if D % 4:
            raise ValueError("trainer needs the embedding dim to be a multiple of 4")
        self.D = D
        T = len(cfg.ln_emb)
        self.T = T
        if world_size > 1:
            if T < world_size:
                raise ValueError(f"only {T} tables for {world_size} ranks")
            di = list(cfg.allocation) if cfg.allocation is not None else \
                shard(list(cfg.ln_emb), world_size, cfg.sharder)
        else:
            di = [0] * T
        self.device_indices = di
        self.local_tables = [t for t in range(T) if di[t] == rank]
        self.tables_per_rank = [sum(1 for t in range(T) if di[t] == r) for r in range(world_size)]
        # rank-major global feature order after the all-to-all (extend_distributed.py:475-487)
        self.feature_order = [t for r in range(world_size) for t in range(T) if di[t] == r]
        self.T_local = len(self.local_tables)
        rows = [int(cfg.ln_emb[t]) for t in self.local_tables]
        self.rows_local = rows
        # physical tables: the local tables, with every QR table split into its quotient and
        # remainder tables (the lookup runs on the physical CSR, a combine kernel forms the
        # logical features; the a2a / interaction see logical tables only)
        self.qr = bool(cfg.qr_flag)
        if self.qr and cfg.qr_operation not in ("mult", "add"):
            raise NotImplementedError("trainer QR: qr_operation mult or add (concat widens "
                                      "the feature; the module path DLRM_Net has it)")
        prow, psrc, pkind, pcoll, pq, pr = [], [], [], [], [], []
        for j, n in enumerate(rows):
            if self.qr and n > cfg.qr_threshold:
                c = int(cfg.qr_collisions)
                pq.append(len(prow))
                prow.append(int(math.ceil(n / c)))
                psrc.append(j), pkind.append(1), pcoll.append(c)
                pr.append(len(prow))
                prow.append(c)
                psrc.append(j), pkind.append(2), pcoll.append(c)
            else:
                pq.append(len(prow))
                pr.append(-1)
                prow.append(n)
                psrc.append(j), pkind.append(0), pcoll.append(1)
        self.phys_rows, self.phys_src, self.phys_kind = prow, psrc, pkind
        self.T_phys = len(prow)
        self.qr_active = self.T_phys != self.T_local
        i32 = dict(dtype=torch.int32, device=self.dev)
        self._qr_src = torch.tensor(psrc, **i32)
        self._qr_kind = torch.tensor(pkind, **i32)
        self._qr_coll = torch.tensor(pcoll, **i32)
        self._qr_pq = torch.tensor(pq, **i32)
        self._qr_pr = torch.tensor(pr, **i32)
        self._qr_csr = {}
        rows = prow
        self.row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64,
                                     device=self.dev)
        self.total_rows = int(sum(rows))
        ops.check_tbe_rows(self.total_rows, "DLRMTrainer (this rank's tables)")
        self.weights = torch.empty((max(self.total_rows, 1), D), dtype=torch.float32,
                                   device=self.dev)
        self.momentum = None
        if cfg.optimizer == "rwsadagrad":
            self.momentum = torch.zeros(max(self.total_rows, 1), dtype=torch.float32,
                                        device=self.dev)
        elif cfg.optimizer != "sgd":
            raise ValueError(f"optimizer {cfg.optimizer!r} not supported")
        # ---- dense parameters: one flat bucket
        ln_bot, ln_top = [int(v) for v in cfg.ln_bot], [int(v) for v in cfg.ln_top]
        if ln_top[-1] != 1:
            raise ValueError("the fused head needs a single output (ln_top[-1] == 1)")
        F = T + 1
        if cfg.arch_interaction_op == "dot":
            npairs = F * (F + 1) // 2 if cfg.arch_interaction_itself else F * (F - 1) // 2
            self.num_int = D + npairs
        else:
            self.num_int = F * D
        if ln_top[0] != self.num_int:
            raise ValueError(f"ln_top[0]={ln_top[0]} != number of interactions {self.num_int}")
        specs = [(ln_bot[i + 1], ln_bot[i]) for i in range(len(ln_bot) - 1)] + \
                [(ln_top[i + 1], ln_top[i]) for i in range(len(ln_top) - 1)]
        # Bias folding: layer l stores [W | b | 0-pad] as one [N, Kp] block with
        # Kp = pad4(K + 1); every layer input carries a constant-1 column at index K, so
        # the forward GEMM adds the bias as its last k-term and the wgrad GEMM yields db.
        sizes = [n * _pad4(k + 1) for n, k in specs]
        self.n_params = int(sum(sizes))
        self.params = torch.zeros(self.n_params, dtype=torch.float32, device=self.dev)
        self.grads = torch.zeros_like(self.params) if (self.distributed or
                                                      cfg.optimizer == "rwsadagrad") else None
        self.adagrad_sum = torch.zeros_like(self.params) if cfg.optimizer == "rwsadagrad" else None
        self.layers: List[_Layer] = []
        o = 0
        for n, k in specs:
            kp = _pad4(k + 1)
            W = self.params[o:o + n * kp].view(n, kp)
            L = _Layer(N=n, K=k, Kp=kp, Np=_pad4(n + 1), W=W, b=W[:, k])
            if self.grads is not None:
                L.gW = self.grads[o:o + n * kp].view(n, kp)
                L.gb = L.gW[:, k]
            o += n * kp
            self.layers.append(L)
        self.n_bot = len(ln_bot) - 1
        # DDP buckets of the flat gradient (bottom layers first): the top MLP's gradients
        # are complete after the top backward, the bottom's after the bottom backward
        self.n_bot_params = int(sum(sizes[:self.n_bot]))
        self.bot = self.layers[:self.n_bot]
        self.top = self.layers[self.n_bot:]
        self._bufs = {}
        # independent kernels of a step run on a side stream (see step())
        self.concurrent = True
        # which overlaps to use (attribute, A/B only): "fwd" (bottom MLP || lookup),
        # "bot" (bottom-MLP backward || embedding backward).  Off by default: measured on
        # MI355X, each cross-queue dependency in a replayed hipGraph costs ~10 us, more than
        # the overlap recovers at C3 (profiles/r01_overlap_ab.txt).
        self.overlaps = set()
        self._side = torch.cuda.Stream(device=self.dev)
        self._tbe_ws: Optional[torch.Tensor] = None
        # run the embedding backward's per-table sort inside the lookup launch
        # (dlrm_tbe_forward_presort); False: the backward sorts itself
        self.tbe_presort = True
        # MLP backward: a layer's split wgrad (partials only) in the same launch as its dgrad
        self.group_wgrad = True
        self.full_last_wgrad = False
        # bottom-MLP backward schedule: "partial" (split wgrads reduced in the next launch),
        # "full" (in-launch split-K, n_bot launches; bottom_bwd_full) or "auto": full at
        # <= 128 rows per GPU, else partial (measured, one MI355X: full 0.976 vs partial
        # 0.857 M samples/s at the Kaggle shape, B = 128; partial ahead at C3 B = 2048, 4.67
        # vs 4.54 M, and at B = 256, 1.21 vs 1.19 M; profiles/r04_bot_sched_ab.txt.  A third
        # schedule - the data gradients as one row-block launch - lost at every shape and
        # was removed in ABI v8)
        self.bot_sched = "auto"
        # one GPU: the bottom MLP forward as a role of the lookup launch (mlp_rows.hpp)
        self.fuse_bottom = True
        # several GPUs: the bottom MLP forward as a role of the lookup launch too (True), or
        # as its own chain launch beside the in-flight all-to-all (False).  The emulated
        # W = 8 rank 2 step: 16.3 us of chain launch -> a few us inside the lookup launch;
        # the cost is the all-to-all starting after the (longer) fused launch
        self.dist_bottom_in_lookup = True
        # one GPU, tables past the per-table LDS sort (C1's L = 100): the backward's tiled
        # sort (dlrm_tbe_backward_sort) on the side stream at the start of the step, beside
        # the forward, joined before the embedding backward.  The one cross-queue join of
        # the graph costs ~11 us of idle GPU; the 6 sort launches (~69 us) hide behind the
        # forward: C1 step 0.588 -> 0.572 ms (profiles/r06_early_sort_ab.txt).  2 = forked
        # after the lookup launch instead: ~5 % slower (profiles/r06_early_sort_fork_ab.txt)
        self.early_sort = True
        # one GPU: the pooled embeddings E and their gradient dE with a batch stride of an odd
        # number of 256-byte chunks.  The embedding update reads dE[b, t] in sorted-row order
        # (random b) and each XCD works through one table's lookups: at a stride of 8 chunks
        # (C1: 8 x 64 floats) every such read lands in the same two of an XCD's L2 channels.
        # Measured: C1's update pass 105.7 -> 99.1 us, the step -0.3..-0.8 %, C3 / C2 within
        # noise (profiles/r06_feature_pad_ab.txt) - an option, off by default
        self.feature_pad = False
        # one GPU, one-hot batches: the dot interaction gathers the embedding rows itself
        # (dlrm_interact_dot_forward_gather); the lookup launch keeps only its sort role
        self.fuse_gather = True
        # one GPU: the embedding update's passes as extra workgroups of the bottom-MLP
        # backward's GEMM launches (dlrm_gemm_f32_group_role); False: launches of their own
        self.tbe_role = True
        # one GPU: the head's finalize pass as a role of the top-MLP backward's first launch
        self.head_role = True
        # bottom-MLP forward workgroups per 16-row block in the lookup launch (0 = auto)
        self.bottom_parts = 0
        self._cus = torch.cuda.get_device_properties(self.dev).multi_processor_count \
            if torch.cuda.is_available() else 256
        self.tbe_role_at = (0, 1)  # bottom-backward launches carrying pass 1 and pass 2
        self._roles = []  # pending (role, phase) passes for the next _gemm launches
        self.gather_fused = False  # set by the last step
        self.bottom_fused = False  # set by the last step
        # device TBE error bits (ops.TBE_ERR_*): out-of-range indices are skipped by the
        # kernels and flagged here; check_errors() reads it (the step never syncs)
        self.tbe_error_flag = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._colsum_ws: Optional[torch.Tensor] = None
        self._head_ws: Optional[torch.Tensor] = None
        self.step_count = 0
        self.capture_mode = None  # "whole" | "segments": how the last capture() was built
        self.graphs_per_step = 0  # hipGraphs one replay of the last capture() launches
        if init:
            self.init_random(seed)

    # ---------------------------------------------------------------- init --
    def init_random(self, seed: int = 0):
        """Reference-distribution random init on device: tables U(+-sqrt(1/n))
        (dlrm_s_pytorch.py:304-308), W ~ N(0, sqrt(2/(m+n))), b ~ N(0, sqrt(1/m)) (:240-247)."""
        for p, j in enumerate(self.phys_src):
            t = self.local_tables[j]
            n = int(self.cfg.ln_emb[t])
            a = math.sqrt(1.0 / n)
            view = self.weights[int(self.row_base[p].item()):int(self.row_base[p + 1].item())]
            if self.phys_kind[p] == 0:
                ops.uniform_fill_(view, -a, a, seed * 1000003 + t)
            else:  # QR tables: uniform [sqrt(1/n), 1] (tricks/qr_embedding_bag.py:153-154)
                ops.uniform_fill_(view, a, 1.0, seed * 1000003 + t + 7919 * self.phys_kind[p])
        g = torch.Generator(device=self.dev)
        g.manual_seed(seed + 12345)
        with torch.no_grad():
            for L in self.layers:
                L.W.zero_()
                L.W[:, :L.K].normal_(0.0, math.sqrt(2.0 / (L.N + L.K)), generator=g)
                L.b.normal_(0.0, math.sqrt(1.0 / L.N), generator=g)

    def load_dense(self, mlp_params: Sequence[tuple], tables: Optional[Sequence] = None):
        """Copy (W [N,K], b [N]) per layer (bottom then top) and optionally GLOBAL tables."""
        with torch.no_grad():
            for L, (W, b) in zip(self.layers, mlp_params):
                L.W.zero_()
                L.W[:, :L.K].copy_(torch.as_tensor(W))
                L.b.copy_(torch.as_tensor(b))
            if tables is not None:  # QR tables: (weight_q, weight_r) pairs
                for p, j in enumerate(self.phys_src):
                    t = self.local_tables[j]
                    s, e = int(self.row_base[p].item()), int(self.row_base[p + 1].item())
                    src = tables[t]
                    if self.phys_kind[p] != 0:
                        src = src[self.phys_kind[p] - 1]
                    self.weights[s:e].copy_(torch.as_tensor(src))

    @classmethod
    def from_oracle(cls, cfg: TrainerConfig, ref, device="cuda:0", **kw):
        """Build with the exact weights of an oracle.OracleDLRM (test/smoke helper)."""
        tr = cls(cfg, device=device, init=False, **kw)
        mlp = []
        for seq in (ref.bot_l, ref.top_l):
            for m in seq:
                if isinstance(m, torch.nn.Linear):
                    mlp.append((m.weight.detach(), m.bias.detach()))
        tabs = [(e.weight_q.detach(), e.weight_r.detach()) if hasattr(e, "weight_q")
                else e.weight.detach() for e in ref.emb_l]
        tr.load_dense(mlp, tabs)
        return tr

    def dense_state(self):
        return [(L.W[:, :L.K].detach().clone(), L.b.detach().clone()) for L in self.layers]

    def table(self, t: int):
        """Local table t's weights (a (quotient, remainder) pair for a QR table)."""
        j = self.local_tables.index(t)
        views = [self.weights[int(self.row_base[p].item()):int(self.row_base[p + 1].item())]
                 for p, jj in enumerate(self.phys_src) if jj == j]
        return views[0] if len(views) == 1 else tuple(views)

    def table_momentum(self, t: int):
        """RWSAdagrad row-wise momentum of local table t (a (quotient, remainder) pair for a
        QR table), the reference's optimizer state['momentum'] (optim/rwsadagrad.py:80-84)."""
        if self.momentum is None:
            raise ValueError("no row-wise momentum: optimizer is not rwsadagrad")
        j = self.local_tables.index(t)
        views = [self.momentum[int(self.row_base[p].item()):int(self.row_base[p + 1].item())]
                 for p, jj in enumerate(self.phys_src) if jj == j]
        return views[0] if len(views) == 1 else tuple(views)

    def dense_adagrad_state(self):
        """Per layer (sum of squared W gradients [N, K], of b [N]): the dense branch's
        state['sum'] of RWSAdagrad (optim/rwsadagrad.py:116-119)."""
        if self.adagrad_sum is None:
            raise ValueError("no Adagrad state: optimizer is not rwsadagrad")
        out, o = [], 0
        for L in self.layers:
            S = self.adagrad_sum[o:o + L.N * L.Kp].view(L.N, L.Kp)
            out.append((S[:, :L.K].detach().clone(), S[:, L.K].detach().clone()))
            o += L.N * L.Kp
        return out

    # ------------------------------------------------------------- batches --
    @property
    def lr(self) -> float:
        return float(self.cfg.learning_rate)

    @property
    def emb_lr(self) -> float:
        return float(self.cfg.emb_learning_rate if self.cfg.emb_learning_rate is not None
                     else self.cfg.learning_rate)

    def local_batch_size(self, B: int) -> int:
        if B % self.world:
            raise ValueError(f"batch {B} not divisible by {self.world} ranks "
                             "(dlrm_s_pytorch.py:139-143)")
        return B // self.world

    def make_batch(self, X, lS_o, lS_i, target) -> Batch:
        """From the reference's non-batched layout (X [B,m_den] GLOBAL batch, lS_o [T,B],
        lS_i list of T index tensors) -> this rank's device Batch."""
        B = X.shape[0]
        Bl = self.local_batch_size(B)
        sl = slice(self.rank * Bl, (self.rank + 1) * Bl)
        L0 = self.bot[0]
        Xp = torch.zeros((Bl, L0.Kp), dtype=torch.float32, device=self.dev)
        Xp[:, :L0.K] = torch.as_tensor(X)[sl].to(self.dev)
        Xp[:, L0.K] = 1.0  # bias column
        offs, idxs, start = [], [], 0
        for t in self.local_tables:
            o = torch.as_tensor(lS_o[t]).to(torch.int64)
            ii = torch.as_tensor(lS_i[t]).to(torch.int64)
            offs.append(o + start)
            idxs.append(ii)
            start += ii.numel()
        offsets = torch.cat(offs + [torch.tensor([start])]).to(torch.int32).to(self.dev)
        indices = (torch.cat(idxs) if idxs else torch.zeros(0, dtype=torch.int64)).to(
            torch.int32).to(self.dev)  # a rank may own no table
        tg = torch.as_tensor(target).reshape(-1)[sl].to(torch.float32).to(self.dev)
        mx = max([int(i.numel()) for i in idxs], default=0)
        one_hot = all(torch.equal(torch.as_tensor(lS_o[t]).to(torch.int64),
                                  torch.arange(Bl * self.world)) and
                      int(torch.as_tensor(lS_i[t]).numel()) == Bl * self.world
                      for t in self.local_tables)
        return Batch(Xp, offsets, indices, tg, mx, one_hot and bool(self.local_tables))

    def batch_from_records(self, records: torch.Tensor, max_ind_range: int = -1) -> Batch:
        """A Batch straight from raw Criteo binary records on the device (int32
        [B_global, 1+13+26], the CriteoBinDataset block, data_loader_terabyte.py:237-252):
        one dlrm_criteo_decode launch writes log(x+1) into the padded X (bias column kept),
        the table-major indices (% max_ind_range) and the L = 1 CSR.  Same batch as
        make_batch on the reference's transformed tensors."""
        L0 = self.bot[0]
        nf = 1 + L0.K + self.T
        if records.dim() != 2 or records.shape[1] != nf:
            raise ValueError(f"batch_from_records: records must be [B, {nf}] (1 + m_den + T)")
        B = records.shape[0]
        Bl = self.local_batch_size(B)
        rec = records.reshape(-1).to(device=self.dev, dtype=torch.int32).contiguous()
        dense = torch.empty((B, L0.Kp), dtype=torch.float32, device=self.dev)
        dense[:, L0.K:] = 0.0
        dense[:, L0.K] = 1.0  # bias column
        X, offsets, indices, label = ops.criteo_decode(rec, L0.K, self.T, max_ind_range,
                                                       batched=True, dense=dense)
        sl = slice(self.rank * Bl, (self.rank + 1) * Bl)
        if self.T_local != self.T:
            indices = indices.view(self.T, B)[self.local_tables].reshape(-1).contiguous()
            offsets = offsets[:self.T_local * B + 1].contiguous()
        return Batch(dense[sl].contiguous() if Bl != B else dense, offsets, indices,
                     label.reshape(-1)[sl].contiguous(), B, True)

    def record_batch(self, B: int) -> Batch:
        """Fixed device buffers for global batches of B Criteo records (L = 1), filled by
        ``decode_into`` (data.RecordPipeline): the tensors keep their addresses, so a step
        graph captured on this Batch replays on every decoded batch."""
        Bl = self.local_batch_size(B)
        L0 = self.bot[0]
        X = torch.zeros((Bl, L0.Kp), dtype=torch.float32, device=self.dev)
        X[:, L0.K] = 1.0  # bias column
        offsets = torch.arange(0, self.T_local * B + 1, dtype=torch.int32, device=self.dev)
        indices = torch.zeros(self.T_local * B, dtype=torch.int32, device=self.dev)
        target = torch.zeros(Bl, dtype=torch.float32, device=self.dev)
        if self.world > 1 or self.T_local != self.T:  # full-batch decode scratch
            full = torch.zeros((B, L0.Kp), dtype=torch.float32, device=self.dev)
            self._rec_scratch = dict(
                X=full, label=torch.empty(B, dtype=torch.float32, device=self.dev),
                indices=torch.empty(self.T * B, dtype=torch.int32, device=self.dev),
                offsets=torch.empty(self.T * B + 1, dtype=torch.int32, device=self.dev),
                tables=torch.tensor(self.local_tables, dtype=torch.int64, device=self.dev))
        return Batch(X, offsets, indices, target, B, True)

    def decode_into(self, records: torch.Tensor, batch: Batch, max_ind_range: int = -1) -> Batch:
        """Decode device records int32 [B * (1 + m_den + T)] into ``batch`` (from
        ``record_batch``) on the current stream: one dlrm_criteo_decode launch (plus, on
        several ranks, the copies of this rank's batch slice and local tables).  Enqueues
        only; capturable."""
        L0 = self.bot[0]
        B = batch.max_per_table
        Bl = batch.X.shape[0]
        if self.world == 1 and self.T_local == self.T:
            ops.criteo_decode(records, L0.K, self.T, max_ind_range, batched=True,
                              dense=batch.X, label=batch.target, indices=batch.indices,
                              offsets=self._rec_offsets(B))
            return batch
        sc = self._rec_scratch
        ops.criteo_decode(records, L0.K, self.T, max_ind_range, batched=True, dense=sc["X"],
                          label=sc["label"], indices=sc["indices"], offsets=sc["offsets"])
        sl = slice(self.rank * Bl, (self.rank + 1) * Bl)
        batch.X[:, :L0.K].copy_(sc["X"][sl, :L0.K])
        batch.target.copy_(sc["label"][sl])
        torch.index_select(sc["indices"].view(self.T, B), 0, sc["tables"],
                           out=batch.indices.view(self.T_local, B))
        return batch

    def _rec_offsets(self, B: int) -> torch.Tensor:
        # the decode rewrites the L = 1 CSR offsets (arange); a private buffer keeps the
        # batch's own copy untouched while a graph may be reading it
        t = self._rec_off.get(B) if hasattr(self, "_rec_off") else None
        if t is None:
            self._rec_off = getattr(self, "_rec_off", {})
            t = self._rec_off[B] = torch.empty(self.T * B + 1, dtype=torch.int32, device=self.dev)
        return t

    def synthetic_batch(self, B: int, L: int, seed: int, dist: str = "uniform",
                        zipf_a: float = 1.05) -> Batch:
        """Device-generated synthetic batch of the reference's shape: X ~ log(1+U[0,1))
        (dlrm_data_pytorch.py:727), L uniform indices per bag per table, targets U[0,1)
        (rounded for bce).  dist="zipf": the skew-sensitivity run of SURVEY.md §8d - each
        table's indices are Zipf(zipf_a) ranks - 1 folded onto its rows (row 0 hottest),
        drawn on the host (numpy) and uploaded."""
        if dist not in ("uniform", "zipf"):
            raise ValueError(f"dist {dist!r}: uniform or zipf")
        Bl = self.local_batch_size(B)
        L0 = self.bot[0]
        g = torch.Generator(device=self.dev)
        g.manual_seed(seed * 7919 + self.rank)
        Xp = torch.zeros((Bl, L0.Kp), dtype=torch.float32, device=self.dev)
        Xp[:, :L0.K] = torch.log1p(torch.rand((Bl, L0.K), generator=g, device=self.dev))
        Xp[:, L0.K] = 1.0  # bias column
        Tl = self.T_local
        indices = torch.empty(Tl * B * L, dtype=torch.int32, device=self.dev)
        rng = np.random.RandomState(seed) if dist == "zipf" else None
        for j, t in enumerate(self.local_tables):
            n = int(self.cfg.ln_emb[t])
            if rng is not None:
                z = (rng.zipf(zipf_a, B * L) - 1) % n
                indices[j * B * L:(j + 1) * B * L] = torch.from_numpy(z.astype(np.int32))
            else:
                ops.uniform_int_fill_(indices[j * B * L:(j + 1) * B * L], n,
                                      seed * 1000003 + t * 7 + 1)
        offsets = torch.arange(0, Tl * B * L + 1, L, dtype=torch.int32, device=self.dev)
        tg = torch.rand(Bl, generator=g, device=self.dev)
        if self.cfg.loss_function == "bce":
            tg = tg.round()
        return Batch(Xp, offsets, indices, tg, B * L, L == 1)

    # ------------------------------------------------------------- buffers --
    def _buffers(self, Bl: int, B: int):
        key = (Bl, B)
        if key in self._bufs:
            return self._bufs[key]
        dev, D = self.dev, self.D
        f32 = dict(dtype=torch.float32, device=dev)
        bufs = {}
        # activations carry the constant-1 bias column right after their N real columns
        bufs["bot_act"] = [torch.zeros((Bl, L.Np), **f32) for L in self.bot]
        self.ldR = _pad4(self.num_int + 1)
        bufs["R"] = torch.zeros((Bl, self.ldR), **f32)
        bufs["top_act"] = [torch.zeros((Bl, L.Np), **f32) for L in self.top[:-1]]
        for L, a in zip(self.bot + self.top[:-1], bufs["bot_act"] + bufs["top_act"]):
            a[:, L.N] = 1.0
        bufs["R"][:, self.num_int] = 1.0
        wmax = max([L.Kp for L in self.layers] + [self.ldR])
        # split-K workspaces: sized on the first step for this batch size (self._gemm grows
        # them before any capture), zeroed because the split-K tile tickets must start at 0
        # (the kernels leave them at 0).  They belong to this batch size: a hipGraph
        # captured for it keeps their addresses, and the main and side streams never share.
        bufs["gemm_ws"] = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        bufs["gemm_ws_side"] = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        # three gradient buffers: a weight-gradient GEMM on the side stream may still read
        # g_l while the main stream's next two data-gradient GEMMs produce g_{l-1}, g_{l-2}
        bufs["g"] = [torch.zeros((Bl, wmax), **f32) for _ in range(3)]
        wbot = max(L.Kp for L in self.bot)
        bufs["gb"] = [torch.zeros((Bl, wbot), **f32) for _ in range(3)]
        bufs["dx"] = torch.zeros((Bl, D), **f32)
        bufs["gx"] = torch.zeros((Bl, D), **f32)
        Tl = max(self.T_local, 1)
        pad = 0
        if self.feature_pad and not self.distributed and not self.qr_active:
            pad = ((256 - (Tl * D * 4) % 512) % 512) // 4  # stride = 256 B mod 512 B
        for name in ("E", "dE"):
            store = torch.zeros((B, Tl * D + pad), **f32)
            bufs[name] = store[:, :Tl * D].view(B, Tl, D)
        if self.qr_active:  # pooled physical tables (quotient / remainder halves)
            bufs["P"] = torch.zeros((B, self.T_phys, D), **f32)
            bufs["dP"] = torch.zeros_like(bufs["P"])
        if self.distributed:
            bufs["recv"] = torch.zeros(self.T * Bl * D, **f32)
            bufs["drecv"] = torch.zeros_like(bufs["recv"])
        bufs["prob"] = torch.zeros(Bl, **f32)
        bufs["dz"] = torch.zeros(Bl, **f32)
        bufs["loss"] = torch.zeros(1, **f32)
        self._bufs[key] = bufs
        return bufs

    def _features(self, bufs, Bl: int, grad: bool = False):
        """(x, per-feature tensors) for the interaction: feature 0 = bottom-MLP output,
        then the embedding features in rank-major order (single GPU: table order)."""
        D = self.D
        x = bufs["dx"] if grad else bufs["bot_act"][-1][:, :D]
        if not self.distributed:
            return x, bufs["dE" if grad else "E"]
        flat = bufs["drecv" if grad else "recv"]
        feats, o = [], 0
        for r in range(self.world):
            Tr = self.tables_per_rank[r]
            chunk = flat[o:o + Bl * Tr * D].view(Bl, Tr, D)
            feats.extend(chunk[:, j, :] for j in range(Tr))
            o += Bl * Tr * D
        return x, feats

    # ---------------------------------------------------------------- step --
    def step(self, batch: Batch, profile=None):
        """One fwd + loss + bwd + update.  Returns (prob [B_local], loss [1]) device tensors.
        ``profile``: optional callable(name) -> context manager around kernel groups (the
        step then runs on one stream so each group's events bracket only its kernels)."""
        for _kind, fn in self.segments(batch, profile):
            fn()
        return self._cur["prob"], self._cur["loss"]

    def segments(self, batch: Batch, profile=None):
        """The step as an ordered list of ("gpu", fn) / ("a2a", fn) / ("ar", fn) /
        ("host", fn) items.  "gpu" items only enqueue HIP kernels on the current stream (no
        host sync, no allocation after the first step of a batch size): each one can be
        captured in a hipGraph.  "a2a" / "ar" items issue or wait for the all-to-alls / the
        dense all-reduces between them (multi GPU only): RCCL's all-reduces are captured
        with the kernels, its all-to-alls run eagerly between the graphs (capture); on
        gloo every collective runs eagerly.  "host" items are host bookkeeping, run on
        every replay.

        MLP backward: each layer's weight gradient is split-K into a per-layer partial
        buffer and its reduction (+ fused SGD on one GPU) is a REDUCE job inside the NEXT
        GEMM launch (the kernel boundary publishes the partials: no reduce launch, no
        in-launch hand-off); the dgrad in that launch reads W_l, never the W_{l+1} the job
        writes.  Optional side-stream overlaps (self.overlaps): "fwd" = bottom MLP || lookup,
        "bot" = bottom-MLP backward || embedding backward (joined inside the segment)."""
        cfg = self.cfg
        D = self.D
        Bl = batch.X.shape[0]
        B = Bl * self.world
        # the all-to-all splits assume every rank holds B / W samples of a B-sample batch
        # (dlrm_s_pytorch.py:139-143); a batch built for another world size or table set
        # would send wrong-sized chunks
        n_off = self.T_local * B + 1
        if self.T_local > 0 and batch.offsets.numel() != n_off:
            raise ValueError(f"batch offsets hold {batch.offsets.numel()} entries, expected "
                             f"T_local*B+1 = {n_off} (B = {Bl} x {self.world} ranks)")
        bufs = self._buffers(Bl, B)
        self._cur = bufs
        prof = profile or (lambda name: _NullCtx())
        self._prof = prof
        fused_opt = self.grads is None  # single GPU SGD: updates fused into backward
        lr, elr = self.lr, self.emb_lr
        conc = self.concurrent and profile is None
        dist = self.distributed
        c_fwd = conc and "fwd" in self.overlaps and not dist
        c_bot = conc and "bot" in self.overlaps and not dist
        st = {}  # state shared by the segments (collective handles, pending reductions)
        presort = self.tbe_presort
        gather = presort and not dist and self._gather_applies(batch)
        self.gather_fused = gather

        def streams():
            s0 = torch.cuda.current_stream(self.dev)
            return s0, self._side if conc else s0

        def side_if(flag, s1):
            return torch.cuda.stream(s1) if flag else _NullCtx()

        # the reference's profiler phase names (dlrm_s_pytorch.py:692-721, 171, 1923), so a
        # torch.profiler trace of this step lines up with one of the reference's
        emb_sizes = "-".join(str(int(cfg.ln_emb[t])) for t in self.local_tables)

        def lookup():  # embeddings (full batch, local tables)
            if dist:
                self._roles = []  # first segment: no pass of an aborted step carries over
            with record_function("module::forward_pass::embedding_lookup", emb_sizes), \
                    prof("tbe_fwd"):
                if self.T_local > 0:
                    if "csr" not in st:
                        st["csr"] = self._phys_csr(batch, B)
                    idx, off = st["csr"]
                    out = bufs["P"] if self.qr_active else bufs["E"]
                if self.T_local > 0 and presort:
                    # the backward's per-table sort runs inside the lookup launch (alone,
                    # when the interaction gathers the rows itself); several GPUs: with the
                    # bottom MLP forward as a third role (dist_bottom_in_lookup)
                    chain = self._bottom_chain(batch, bufs) if dist and profile is None and \
                        self.dist_bottom_in_lookup else None
                    st["bottom_done"] = chain is not None
                    ops.tbe_forward_presort(self.weights, self.row_base, self.T_phys, B, idx,
                                            off, self._ws_tbe(idx.numel()),
                                            batch.max_per_table, out=None if gather else out,
                                            out_batch_stride=out.stride(0),
                                            error_flag=self.tbe_error_flag, bottom=chain,
                                            lookup=not gather)
                elif self.T_local > 0:
                    ops.tbe_forward(self.weights, self.row_base, self.T_phys, B, idx, off,
                                    out=out, out_batch_stride=out.stride(0),
                                    error_flag=self.tbe_error_flag)
                if self.T_local > 0 and self.qr_active:
                    self._qr_combine(bufs, B)

        def bottom_fwd():
            h = batch.X
            if st.pop("bottom_done", False):  # ran inside the lookup launch
                return _EMPTY
            with record_function("module::forward_pass::bottom_mlp"):
                if dist and profile is None:
                    # several GPUs: the bottom MLP as one row-block chain launch (activations
                    # in LDS between layers, mlp_rows.hpp) while the all-to-all is in flight
                    chain = self._bottom_chain(batch, bufs, sort_wgs=0, standalone=True)
                    if chain is not None:
                        ops.mlp_chain_forward(chain, self.dev)
                        return
                for L, out in zip(self.bot, bufs["bot_act"]):
                    self._gemm([self._fwd(L, h, out)], side=c_fwd)
                    h = out

        def early_sort():  # the backward's sort on the side stream, beside the forward
            s0, s1 = streams()
            idx, off = st["csr"] = self._phys_csr(batch, B)
            s1.wait_stream(s0)
            with torch.cuda.stream(s1), prof("tbe_sort"):
                ops.tbe_backward_sort(self.weights, self.row_base, self.T_phys, B, idx, off,
                                      self._ws_tbe(idx.numel()), batch.max_per_table,
                                      error_flag=self.tbe_error_flag)
            st["sorted"] = s1

        def fwd_single():  # one GPU: bottom MLP || lookup
            # first segment of the step: a launch role deferred by an aborted step (raw
            # pointers of that step) must never ride on this step's launches
            self._roles = []
            es = (self.early_sort and conc and self.T_local > 0 and presort
                  and not 0 < batch.max_per_table <= ops.TBE_PRESORT_SEG_CAP)
            if es and self.early_sort != 2:  # 2: forked after the lookup launch instead
                early_sort()
            chain = self._bottom_chain(batch, bufs) if presort and not c_fwd else None
            self.bottom_fused = chain is not None
            if chain is not None:
                # the bottom MLP forward runs as a role of the lookup launch
                with record_function("module::forward_pass::embedding_lookup", emb_sizes), \
                        record_function("module::forward_pass::bottom_mlp"), prof("tbe_fwd"):
                    if "csr" not in st:
                        st["csr"] = self._phys_csr(batch, B)
                    idx, off = st["csr"]
                    out = None if gather else bufs["P"] if self.qr_active else bufs["E"]
                    ops.tbe_forward_presort(self.weights, self.row_base, self.T_phys, B, idx,
                                            off, self._ws_tbe(idx.numel()),
                                            batch.max_per_table, out=out,
                                            out_batch_stride=None if out is None else
                                            out.stride(0),
                                            error_flag=self.tbe_error_flag, bottom=chain,
                                            lookup=not gather)
                    if self.qr_active:
                        self._qr_combine(bufs, B)
                if es and self.early_sort == 2:
                    early_sort()
                return
            s0, s1 = streams()
            if es and self.early_sort == 2:
                lookup()
                early_sort()
                s0, s1 = streams()
            if c_fwd:
                s1.wait_stream(s0)
            if not (es and self.early_sort == 2):
                lookup()
            with side_if(c_fwd, s1):
                bottom_fwd()
            if c_fwd:
                s0.wait_stream(s1)

        def top():  # interaction, top MLP, head, top backward
            x, feats = self._features(bufs, Bl)
            with record_function("module::forward_pass::interaction"), prof("interaction_fwd"):
                if gather:  # one-hot lookup fused: rows read straight from the tables
                    ops.interact_forward_gather(x, self.weights, self.row_base, batch.indices,
                                                cfg.arch_interaction_itself, out=bufs["R"],
                                                error_flag=self.tbe_error_flag)
                else:
                    ops.interact_forward(cfg.arch_interaction_op, x, feats,
                                         cfg.arch_interaction_itself, out=bufs["R"])
            h = bufs["R"]
            with record_function("module::forward_pass::top_mlp"):
                for L, out in zip(self.top[:-1], bufs["top_act"]):
                    self._gemm([self._fwd(L, h, out)])
                    h = out
            last = self.top[-1]
            # head: last layer + sigmoid + loss + dz + input grad + [dw | db] (bias folded:
            # [h | 1] . [w | b]) in two launches; the update follows every read of w
            G = bufs["g"]
            gi = 0
            gview = G[gi][:, :last.Kp]
            # the head's second launch (column sums + update or gradient + mean loss) rides
            # on the top-MLP backward's first GEMM launch (dlrm_head_step_defer)
            head_role = self.head_role and profile is None and len(self.top) > 1
            with record_function("## Loss Compute ##"), prof("head"):
                r = ops.head_step(h[:, :last.Kp], last.W[0, :last.Kp], batch.target,
                                  cfg.loss_function, cfg.loss_threshold, 1.0, prob=bufs["prob"],
                                  dz=bufs["dz"], loss_out=bufs["loss"], dX=gview,
                                  relu_mask=len(self.top) > 1,
                                  dw=None if fused_opt else last.gW[0, :last.Kp],
                                  lr=lr if fused_opt else 0.0,
                                  workspace=self._ws_head_step(Bl, last.Kp), defer=head_role)
                if head_role:
                    self._roles = [x for x in self._roles if x is not None] + [(r, 4)]
            g = gview
            rq = []  # reduce jobs riding on the next launch; G rotates over three buffers
            bwd = record_function("## Backward ##")
            bwd.__enter__()
            for li in range(len(self.top) - 2, -1, -1):
                L = self.top[li]
                inp = bufs["top_act"][li - 1] if li > 0 else bufs["R"]
                gn = (gi + 1) % 3
                dg = self._dgrad(L, g, inp if li > 0 else None, G[gn])
                # several GPUs: the top bucket is all-reduced right after this loop, so its
                # last wgrad reduces its K split inside its own launch
                w, r = self._wg(L, g, inp, fused_opt, lr, ("top", li), full=dist and li == 0)
                if r is not None and self.group_wgrad:
                    # the split wgrad only writes partials (its update rides on the next
                    # launch's reduce job), so it may run beside the dgrad reading W
                    self._gemm([dg, w] + rq)
                    rq = [r]
                elif r is None and not fused_opt:
                    # the wgrad writes the gradient bucket, not W: beside the dgrad
                    self._gemm([dg, w] + rq)
                    rq = []
                elif r is not None:
                    # a split wgrad kept out of the dgrad's launch (group_wgrad off): its
                    # partials in a launch of their own, its reduce job on the next one
                    self._gemm([dg] + rq)
                    self._gemm([w])
                    rq = [r]
                else:
                    # an unsplit wgrad updates W_l in its epilogue: it rides on the NEXT
                    # launch (dgrad of layer l-1 reads W_{l-1}, not W_l; its g_l buffer
                    # is not overwritten there: G rotates over three)
                    self._gemm([dg] + rq)
                    rq = [w]
                g, gi = G[gn], gn
            bwd.__exit__(None, None, None)
            st.update(rq=rq, x=x, feats=feats, g=g)

        def interaction_bwd():
            x, feats, g = st.pop("x"), st.pop("feats"), st.pop("g")
            bwd = record_function("## Backward ##")
            bwd.__enter__()
            _, gfeats = self._features(bufs, Bl, grad=True)
            with prof("interaction_bwd"):  # + the backward of the bottom MLP's last ReLU
                if gather:  # rows re-gathered (the embedding update comes later)
                    ops.interact_backward_gather(x, self.weights, self.row_base, batch.indices,
                                                 g[:, :self.num_int], cfg.arch_interaction_itself,
                                                 grad_x=bufs["gx"], grad_ly=gfeats, relu_x=True)
                else:
                    ops.interact_backward(cfg.arch_interaction_op, x, feats, g[:, :self.num_int],
                                          cfg.arch_interaction_itself, grad_x=bufs["gx"],
                                          grad_ly=gfeats, relu_x=True)
            bwd.__exit__(None, None, None)

        def middle():  # interaction, top MLP, head, top backward, interaction backward
            top()
            interaction_bwd()

        def bottom_bwd_full():
            """Bottom-MLP backward with in-launch split-K wgrads (FULL, SGD fused): the
            wgrad of layer l rides in the launch of dgrad(l-1), which does not read W_l,
            and the last launch holds the two lowest wgrads - n_bot launches, no trailing
            REDUCE.  dgrad(l) writes g_{l-1} into buffer l % 3: the wgrad it shares a launch
            with reads g_{l+1} from buffer (l+2) % 3."""
            rq = st.pop("rq")
            g = bufs["gx"]
            pending = []
            for li in range(self.n_bot - 1, -1, -1):
                L = self.bot[li]
                inp = bufs["bot_act"][li - 1] if li > 0 else batch.X
                w = self._wgrad(L, g, inp, fused_opt, lr)
                if li > 0:
                    out = bufs["gb"][li % 3]
                    self._gemm([self._dgrad(L, g, inp, out)] + pending + rq)
                    rq, pending, g = [], [w], out
                else:
                    self._gemm(pending + [w] + rq)

        def bottom_bwd(s1=None, hold_last=False):
            """hold_last: the last launch's problems go to st["bot_last"] instead of being
            launched (several GPUs: it then carries the embedding update's first pass once
            the reverse all-to-all has landed)."""
            sched = self.bot_sched
            if sched == "auto":
                sched = "full" if Bl <= 128 else "partial"
            if sched == "full" and not c_bot and fused_opt:
                return bottom_bwd_full()
            rq = st.pop("rq")
            g = bufs["gx"]  # dLoss/d(pre-ReLU bottom output), from the interaction backward
            bg = [bufs["gb"][0], bufs["gb"][1]]
            launches = []
            for li in range(self.n_bot - 1, -1, -1):
                L = self.bot[li]
                inp = bufs["bot_act"][li - 1] if li > 0 else batch.X
                w, r = self._wg(L, g, inp, fused_opt, lr, ("bot", li), last=li == 0)
                if li > 0 and r is not None and self.group_wgrad:
                    launches.append([self._dgrad(L, g, inp, bg[li % 2]), w] + rq)
                elif li > 0 and r is None and not fused_opt:
                    # the wgrad writes the gradient bucket, not W: beside the dgrad
                    launches.append([self._dgrad(L, g, inp, bg[li % 2]), w] + rq)
                else:
                    if li > 0:
                        launches.append([self._dgrad(L, g, inp, bg[li % 2])] + rq)
                        rq = []
                    launches.append([w] + rq)
                rq = [r] if r is not None else []
                if li > 0:
                    g = bg[li % 2]
            if rq:
                launches.append(rq)
            if hold_last:
                st["bot_last"] = launches.pop()
            for probs in launches:
                self._gemm(probs, side=c_bot)

        def emb_bwd(defer=False):  # embedding backward + fused update
            """defer=True: the update's two passes are returned as a role for the next two
            GEMM launches (None: it ran in full here)."""
            with prof("tbe_bwd"):
                if self.T_local > 0:
                    mode = "rowwise_adagrad" if cfg.optimizer == "rwsadagrad" else "sgd"
                    idx, off = st["csr"]
                    grad = bufs["dE"]
                    if self.qr_active:
                        ops.qr_pool_combine_backward(cfg.qr_operation, self.T_local, B, D,
                                                     self._qr_pq, self._qr_pr, bufs["P"],
                                                     bufs["dE"], bufs["dP"])
                        grad = bufs["dP"]
                    fn = ops.tbe_backward_defer if defer else ops.tbe_backward
                    s1 = st.pop("sorted", None)
                    if s1 is not None:  # join the early sort
                        torch.cuda.current_stream(self.dev).wait_stream(s1)
                    return fn(mode, self.weights, self.row_base, self.T_phys, B, idx, off,
                              grad, lr=elr, eps=cfg.adagrad_eps, momentum=self.momentum,
                              grad_batch_stride=grad.stride(0),
                              workspace=self._ws_tbe(idx.numel()),
                              max_lookups_per_table=batch.max_per_table,
                              error_flag=self.tbe_error_flag,
                              presorted=ops.PRESORTED_ANY if s1 is not None else presort)

        @record_function("## Backward ##")
        def backward_single():  # one GPU: bottom backward || embedding backward
            s0, s1 = streams()
            if c_bot:
                rq = st["rq"]
                if rq:
                    self._gemm(rq)
                st["rq"] = []
                s1.wait_stream(s0)
            # the embedding update's two HBM-bound passes ride as extra workgroups on the
            # first two (MFMA-bound) bottom-backward launches: overlap with no cross-queue
            # dependency (dlrm_tbe_backward_defer / dlrm_gemm_f32_group_role)
            deferred = (self.tbe_role and not c_bot and self.T_local > 0 and profile is None
                        and self.weights.dtype == torch.float32)
            if deferred:
                a, b = self._check_role_at(self.tbe_role_at)
                role = emb_bwd(defer=True)
                if role is not None:  # pass p rides on bottom-backward launch tbe_role_at[p-1]
                    self._roles = [None] * (b + 1)
                    self._roles[a], self._roles[b] = (role, 1), (role, 2)
            with side_if(c_bot, s1):
                bottom_bwd()
            while self._roles:  # a pass the bottom backward had no launch left for
                if self._roles[0] is None:
                    self._roles.pop(0)
                else:
                    self._gemm([])
            if not deferred:
                emb_bwd()
            if c_bot:
                s0.wait_stream(s1)

        def dense_update():
            with record_function("## Backward ##"), prof("dense_update"):
                scale = 1.0 / self.world
                if cfg.optimizer == "sgd" and st.pop("top_updated", False):
                    # the top bucket's update rode on the embedding update's second pass
                    nb = self.n_bot_params
                    ops.sgd_update(self.params[:nb], self.grads[:nb], lr * scale)
                elif cfg.optimizer == "sgd":
                    ops.sgd_update(self.params, self.grads, lr * scale)
                else:  # the 1/W folded into the update (one pass over the bucket)
                    ops.adagrad_update(self.params, self.grads, self.adagrad_sum, lr,
                                       cfg.adagrad_eps, grad_scale=scale)

        def done():
            self.step_count += 1

        if not dist:
            segs = [("gpu", fwd_single), ("gpu", middle), ("gpu", backward_single)]
            if not fused_opt:
                segs.append(("gpu", dense_update))
            return segs + [("host", done)]
        # multi GPU (distributed_forward, dlrm_s_pytorch.py:686-730; DDP :1626-1633):
        #  * the pooled-embedding all-to-all overlaps the bottom MLP (one chain launch);
        #  * the top MLP's gradient bucket is all-reduced as soon as the top backward is
        #    done (DDP's per-module buckets), overlapping the interaction backward, the
        #    bottom backward and the embedding update; the bottom bucket follows the bottom
        #    backward.  The all-reduces run on a communicator of their own, so they never
        #    queue the reverse all-to-all that the embedding update waits for;
        #  * the reverse all-to-all overlaps the bottom backward.
        def ar(bucket):
            def start():
                g = self.grads[self.n_bot_params:] if bucket == "top" else \
                    self.grads[:self.n_bot_params]
                st["ar_" + bucket] = self.comm.allreduce(g)
            return start

        def wait(key):
            return lambda: st.pop(key).wait()

        a2a_fwd = lambda: st.__setitem__("a2a", self._alltoall_fwd(bufs, Bl))  # noqa: E731
        a2a_bwd = lambda: st.__setitem__("a2a", self._alltoall_bwd(bufs, Bl))  # noqa: E731
        # the embedding update's two passes as launch roles (as on one GPU): the first on
        # the bottom backward's last launch, held back until the reverse all-to-all has
        # landed; the second on a launch that also applies the top bucket's SGD update.
        # The choice must not depend on the rank (T_local): every rank issues the same
        # collectives in the same order (a rank without tables just carries no role)
        roles_dist = self.tbe_role and profile is None and self.weights.dtype == torch.float32

        def bottom_head():
            bottom_bwd(hold_last=roles_dist)

        def bottom_tail():  # after All2All_Wait: the update's passes ride on GEMM launches
            role = emb_bwd(defer=True)
            if role is not None:
                self._roles = [(role, 1)]
                st["emb_role"] = role
            self._gemm(st.pop("bot_last"))
            self._roles = []

        def emb_pass2():
            role = st.pop("emb_role", None)
            if role is None:
                return
            jobs = []
            if cfg.optimizer == "sgd":  # the top bucket was all-reduced (waited) already
                nb = self.n_bot_params
                jobs = [ops.sgd_job(self.params[nb:], self.grads[nb:], lr * (1.0 / self.world))]
                st["top_updated"] = True
            self._roles = [(role, 2)]
            self._gemm(jobs)
            self._roles = []

        # RCCL: the all-reduces capture into hipGraphs, the all-to-alls do not (DESIGN.md §8:
        # a captured all_to_all_single or send/recv crashes hipStreamEndCapture on this
        # stack).  Each all-reduce is waited in the graph that issues it, so the step is FOUR
        # graphs around the two eager all-to-alls: the top bucket overlaps the bottom
        # backward and the reverse all-to-all, the bottom bucket the embedding update's
        # second pass.  gloo (host-staged, synchronous) runs the same order eagerly.
        if roles_dist:
            return [
                ("gpu", lookup),
                ("a2a", a2a_fwd),
                ("gpu", bottom_fwd),
                ("a2a", wait("a2a")),  # All2All_Wait (extend_distributed.py:489)
                ("gpu", top),
                ("gpu", interaction_bwd),
                ("a2a", a2a_bwd),
                ("ar", ar("top")),
                ("gpu", record_function("## Backward ##")(bottom_head)),
                ("ar", wait("ar_top")),
                ("a2a", wait("a2a")),
                ("gpu", record_function("## Backward ##")(bottom_tail)),
                ("ar", ar("bot")),
                ("gpu", record_function("## Backward ##")(emb_pass2)),
                ("ar", wait("ar_bot")),
                ("gpu", dense_update),
                ("host", done),
            ]
        if getattr(self.comm, "capture_ar", False):
            return [
                ("gpu", lookup),
                ("a2a", a2a_fwd),
                ("gpu", bottom_fwd),
                ("a2a", wait("a2a")),  # All2All_Wait (extend_distributed.py:489)
                ("gpu", top),
                ("gpu", interaction_bwd),
                ("a2a", a2a_bwd),
                ("ar", ar("top")),
                ("gpu", record_function("## Backward ##")(bottom_bwd)),
                ("ar", wait("ar_top")),
                ("a2a", wait("a2a")),
                ("ar", ar("bot")),
                ("gpu", record_function("## Backward ##")(emb_bwd)),
                ("ar", wait("ar_bot")),
                ("gpu", dense_update),
                ("host", done),
            ]
        return [
            ("gpu", lookup),
            ("a2a", a2a_fwd),
            ("gpu", bottom_fwd),
            ("a2a", wait("a2a")),  # All2All_Wait (extend_distributed.py:489)
            ("gpu", top),
            ("ar", ar("top")),
            ("gpu", interaction_bwd),
            ("a2a", a2a_bwd),
            ("gpu", record_function("## Backward ##")(bottom_bwd)),
            ("ar", ar("bot")),
            ("a2a", wait("a2a")),
            ("gpu", record_function("## Backward ##")(emb_bwd)),
            ("ar", wait("ar_top")),
            ("ar", wait("ar_bot")),
            ("gpu", dense_update),
            ("host", done),
        ]


    @staticmethod
    def _check_role_at(at):
        """tbe_role_at = (a, b): the bottom-backward launches carrying the update's block
        pass and its combine pass.  The combine pass reads what the block pass wrote, so it
        must ride on a LATER launch: 0 <= a < b."""
        a, b = (int(v) for v in at)
        if not 0 <= a < b:
            raise ValueError(f"tbe_role_at={tuple(at)}: need 0 <= a < b (the combine pass "
                             "rides on a later launch than the block pass)")
        return a, b

    def _gather_applies(self, batch: Batch) -> bool:
        """One-hot lookups gathered inside the dot interaction: one GPU, plain tables, every
        bag one index, and the lookup launch able to run its sort role alone (the per-table
        sort of dlrm_tbe_forward_presort: <= 4096 lookups per table, 32-bit row keys)."""
        return (self.fuse_gather and batch.one_hot and not self.distributed and not self.qr_active
                and self.cfg.arch_interaction_op == "dot" and self.D in (16, 32, 64, 128)
                and 1 <= self.T_local == self.T and self.T + 1 <= 32
                and 0 < batch.max_per_table <= ops.TBE_PRESORT_SEG_CAP
                and self.weights.shape[0] < 0xFFFFFFFF
                and batch.indices.numel() == self.T * batch.X.shape[0])

    def _phys_csr(self, batch: Batch, B: int):
        """(indices, offsets) of the physical tables for this batch: the batch's own CSR, or
        (QR) the expanded CSR written by one dlrm_qr_expand_csr launch into buffers owned by
        this (batch size, lookup count) so captured graphs keep their addresses."""
        if not self.qr_active:
            return batch.indices, batch.offsets
        n_log = batch.indices.numel()
        mx = int(batch.max_per_table)
        if mx > 0 and mx * self.T_local == n_log:  # every table has mx lookups
            n = mx * self.T_phys
        else:  # bound: the tail past the last bag is skipped by the kernels
            n = n_log + (self.T_phys - self.T_local) * (mx if mx > 0 else n_log)
        key = (B, n)
        if key not in self._qr_csr:
            self._qr_csr[key] = (
                torch.zeros(max(n, 1), dtype=torch.int32, device=self.dev),
                torch.zeros(self.T_phys * B + 1, dtype=torch.int32, device=self.dev))
        pidx, poff = self._qr_csr[key]
        ops.qr_expand_csr(self.T_phys, B, batch.indices, batch.offsets, self._qr_src,
                          self._qr_kind, self._qr_coll, mx if mx > 0 else n_log, pidx, poff,
                          error_flag=self.tbe_error_flag)
        return pidx, poff

    def _qr_combine(self, bufs, B: int) -> None:
        ops.qr_pool_combine_forward(self.cfg.qr_operation, self.T_local, B, self.D, self._qr_pq,
                                    self._qr_pr, bufs["P"], bufs["E"])

    def capture(self, batch: Batch, pool=None, whole: Optional[bool] = None):
        """A replayable step for ``batch``.  whole (default: one GPU, or a comm whose
        collectives all capture): the step's kernels AND its collectives in ONE hipGraph (a
        graph-to-graph boundary costs ~9 us of idle GPU, profiles/r05_step_timeline_emul8_
        r2.txt); else the "gpu" segments - with the collectives the comm can capture
        (``capture_ar``: RCCL's all-reduces) - as graphs, and the rest ("a2a": RCCL's
        all-to-alls, everything on gloo) run eagerly between them.  Run one eager step of
        this batch size first (allocations).  Returns a callable; each call is one full
        training step on the captured buffers."""
        auto = whole is None
        if auto:
            whole = not self.distributed or bool(getattr(self.comm, "capturable", False))
        if whole:
            segs = self.segments(batch)
            host = [fn for kind, fn in segs if kind == "host"]
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, pool=pool):
                    for kind, fn in segs:
                        if kind != "host":
                            fn()
            except Exception as e:  # noqa: BLE001
                if not (auto and self.distributed):
                    raise
                import warnings
                warnings.warn(f"whole-step capture with the collectives failed ({e!r}); "
                              "capturing the kernel segments between eager collectives")
                torch.cuda.synchronize()
                return self.capture(batch, pool=pool, whole=False)
            self.capture_mode = "whole"
            self.graphs_per_step = 1

            def run_whole():
                g.replay()
                for fn in host:
                    fn()
            return run_whole
        self.capture_mode = "segments"
        in_graph = {"gpu"}
        if getattr(self.comm, "capture_ar", False):
            in_graph.add("ar")
        items = []
        pending = []
        segs = self.segments(batch)
        self.graphs_per_step = 0

        def flush():
            if not pending:
                return
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                launched = [fn() is not _EMPTY for fn in pending]
            if any(launched):  # a segment that enqueued nothing is not replayed
                items.append(g.replay)
                self.graphs_per_step += 1
            pending.clear()

        for kind, fn in segs:
            if kind in in_graph:
                pending.append(fn)
            elif kind == "host":
                items.append(fn)
            else:
                flush()
                items.append(fn)
        flush()

        def run():
            for f in items:
                f()
        return run

    def check_errors(self) -> None:
        """Raise (ops.TBEIndexError / ValueError) if any step since the last check hit an
        index outside its table or exceeded max_per_table; synchronises the device.  The
        reference's EmbeddingBag raises IndexError at the bad lookup itself."""
        ops.check_tbe_errors(self.tbe_error_flag)

    # -------------------------------------------------------------- pieces --
    @staticmethod
    def _fwd(L: _Layer, h, out):
        """[h | 1] . [W | b]^T with ReLU (bias folded into the last k-term)."""
        return ops.gemm_problem(h[:, :L.Kp], L.W, trans_b=True, C=out, epilogue=ops.EPI_RELU)[0]

    @staticmethod
    def _dgrad(L: _Layer, g, inp, out):
        """dX = g W (x ReLU'(inp) when inp is given).  Widths that are not a multiple of 4
        run over Kp (the bias column's gradient lands in a column nobody reads)."""
        n = L.K if L.K % 4 == 0 else L.Kp
        if inp is not None:
            return ops.gemm_problem(g[:, :L.N], L.W[:, :n], C=out[:, :n], epilogue=ops.EPI_DRELU,
                                    aux=inp)[0]
        return ops.gemm_problem(g[:, :L.N], L.W[:, :n], C=out[:, :n])[0]

    @staticmethod
    def _wgrad(L: _Layer, g, inp, fused_opt, lr, **part):
        """[dW | db] = g^T [inp | 1]; fused SGD on one GPU.  With K % 4 == 0 the bias
        gradient is the row sum of g^T (ones_col) and the GEMM covers only the K weight
        columns; otherwise the constant-1 column of inp is multiplied like a weight column."""
        C = L.W if fused_opt else L.gW
        kw = dict(alpha=lr, epilogue=ops.EPI_SGD) if fused_opt else {}
        if L.K % 4 == 0:
            return ops.gemm_problem(g[:, :L.N], inp[:, :L.K], trans_a=True, C=C, ones_col=L.K,
                                    **kw, **part)[0]
        return ops.gemm_problem(g[:, :L.N], inp[:, :L.Kp], trans_a=True, C=C, **kw, **part)[0]

    def _wg(self, L: _Layer, g, inp, fused_opt, lr, key, last=False, full=False):
        """The wgrad of L as (problem, reduce job or None): split-K wgrads write partials
        into a per-layer buffer and their reduction (+ SGD) runs in the NEXT launch.  The
        last GEMM of the step (last=True) has no next launch to carry a reduce job: its
        K split, if any, is reduced inside its own launch (FULL mode), and so is a wgrad
        whose result is needed right after its launch (full=True)."""
        if full or (last and self.full_last_wgrad):
            return self._wgrad(L, g, inp, fused_opt, lr), None
        bufs = self._cur
        sp = bufs.setdefault("splits", {})
        if key not in sp:
            sp[key] = ops.gemm_splits(self._wgrad(L, g, inp, fused_opt, lr), partial=True)
        s = sp[key]
        if s <= 1:
            return self._wgrad(L, g, inp, fused_opt, lr), None
        parts = bufs.setdefault("partials", {})
        M, N = L.N, (L.K if L.K % 4 == 0 else L.Kp)
        need = ops.gemm_partial_bytes(M, N, s)
        if key not in parts or parts[key].numel() * 4 < need:
            parts[key] = torch.empty((need + 3) // 4, dtype=torch.float32, device=self.dev)
        pr = self._wgrad(L, g, inp, fused_opt, lr, partial=parts[key], splits=s)
        return pr, ops.reduce_problem(pr)

    def _gemm(self, problems, side=False):
        """One grouped launch; it also carries the next pending pass of a deferred
        embedding update (self._roles, set by the single-GPU backward)."""
        with self._prof("gemm"):
            ws = self._cur["gemm_ws_side" if side else "gemm_ws"]
            need = ops.gemm_group_workspace_size(problems) if problems else 0
            if need > ws.numel():  # first use of a new group shape: grow (not in capture)
                ws = torch.zeros(need, dtype=torch.uint8, device=self.dev)
                self._cur["gemm_ws_side" if side else "gemm_ws"] = ws
            nxt = self._roles.pop(0) if self._roles and not side else None
            role, phase = nxt if nxt is not None else (None, 0)
            ops.gemm_group(problems, ws, self.dev, role=role, phase=phase)

    def _colsum(self, *args, **kw):
        with self._prof("colsum"):
            ops.colsum(*args, **kw)

    def _bias_and_w_head(self, last: _Layer, hin, dz, fused_opt, lr):
        """Head layer (K -> 1): [dw | db] = sum_m dz[m] [hin[m] | 1] as one column sum."""
        Bl = hin.shape[0]
        if fused_opt:
            self._colsum(hin[:, :last.Kp], scale=dz, sgd_param=last.W[0], lr=lr,
                         workspace=self._ws_colsum(Bl, last.Kp))
        else:
            self._colsum(hin[:, :last.Kp], scale=dz, out=last.gW[0],
                         workspace=self._ws_colsum(Bl, last.Kp))

    def _bottom_chain(self, batch: Batch, bufs, sort_wgs: Optional[int] = None,
                      standalone: bool = False):
        """The bottom MLP forward as a dlrm_mlp_chain (None when unsupported or disabled or,
        unless it runs as its own launch (standalone), when there are no local tables to
        share the lookup launch with)."""
        if not self.fuse_bottom or (self.T_local == 0 and not standalone):
            return None
        layers = [(L.W, out, L.Kp) for L, out in zip(self.bot, bufs["bot_act"])]
        # several workgroups per 16-row block while the lookup launch still fits the
        # chip in one wave (its T_local + 1 sort workgroups beside them): small batches
        # then run the bottom MLP on 2-4x the CUs (mlp_rows.hpp, split chains)
        nrb = (batch.X.shape[0] + 15) // 16
        parts = self.bottom_parts
        others = self.T_local + 1 if sort_wgs is None else sort_wgs
        if parts <= 0:
            parts = next((p for p in (4, 2) if nrb * p + others <= self._cus), 1)
        widest = max(range(len(layers)), key=lambda i: layers[i][2] * layers[i][0].shape[0])
        if (layers[widest][0].shape[0] + 15) // 16 < parts:
            parts = 1
        if parts > 1:
            tk = bufs.get("mlp_tickets")
            if tk is None or tk.numel() < nrb:
                tk = bufs["mlp_tickets"] = torch.zeros(nrb, dtype=torch.int32,
                                                       device=self.dev)
            chain = ops.mlp_chain(batch.X, layers, parts=parts, split_layer=widest,
                                  tickets=tk)
            if ops.mlp_chain_supported(chain):
                return chain
        chain = ops.mlp_chain(batch.X, layers)
        return chain if ops.mlp_chain_supported(chain) else None

    def _ws_tbe(self, n: int) -> torch.Tensor:
        need = ops.tbe_backward_workspace_size(n, self.total_rows, self.D)
        if self._tbe_ws is None or self._tbe_ws.numel() < need:
            self._tbe_ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
        return self._tbe_ws

    def _ws_colsum(self, M: int, N: int) -> torch.Tensor:
        need = int(ops._lib.query("dlrm_colsum_workspace_size", M, max(N, 1024)))
        if self._colsum_ws is None or self._colsum_ws.numel() < need:
            self._colsum_ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
        return self._colsum_ws

    def _ws_head_step(self, M: int, K: int) -> torch.Tensor:
        need = int(ops._lib.query("dlrm_head_step_workspace_size", M, K))
        if getattr(self, "_head_step_ws", None) is None or self._head_step_ws.numel() < need:
            self._head_step_ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
        return self._head_step_ws

    def _ws_head(self, M: int) -> torch.Tensor:
        need = int(ops._lib.query("dlrm_head_workspace_size", M))
        if self._head_ws is None or self._head_ws.numel() < need:
            self._head_ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
        return self._head_ws

    # ------------------------------------------------------ communication --
    def _split_sizes(self, Bl: int):
        D = self.D
        send = [Bl * self.T_local * D] * self.world
        recv = [Bl * self.tables_per_rank[r] * D for r in range(self.world)]
        return send, recv

    def _alltoall_fwd(self, bufs, Bl):
        """All2All_Req.forward (extend_distributed.py:405-444): [B, T_r*D] -> W chunks of
        [B/W, T_s*D] in rank order.  A rank that owns no table sends nothing (its E
        buffer is a 1-table placeholder: only the first sum(send) floats take part)."""
        send, recv = self._split_sizes(Bl)
        return self.comm.a2a(bufs["recv"], bufs["E"].view(-1)[:sum(send)], recv, send)

    def _alltoall_bwd(self, bufs, Bl):
        """All2All_Wait.backward (extend_distributed.py:489-508): reverse exchange."""
        send, recv = self._split_sizes(Bl)
        return self.comm.a2a(bufs["dE"].view(-1)[:sum(send)], bufs["drecv"], send, recv)

    def lookup_balance(self, B: int, L: int = 1):
        """Per-rank load of the table-wise sharding: tables, rows and lookups per step
        (greedy balances rows, not lookups: SURVEY.md §7 hard part 6)."""
        rows = [0] * self.world
        tabs = [0] * self.world
        for t, r in enumerate(self.device_indices):
            rows[r] += int(self.cfg.ln_emb[t])
            tabs[r] += 1
        look = [n * B * L for n in tabs]
        mean = sum(look) / max(self.world, 1)
        return {"tables": tabs, "rows": rows, "lookups": look,
                "lookup_max_over_mean": round(max(look) / mean, 3) if mean else None}

_EMPTY = object()  # returned by a "gpu" segment that enqueued nothing this step


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _Done:
    def wait(self):
        return None


class TorchComm:
    """The step's collectives on torch.distributed (backend nccl = RCCL over xGMI).  The
    all-to-all runs on the trainer's process group; the dense all-reduce on a SECOND
    group of the same ranks (its own communicator, so its own stream): a 9.5 MB gradient
    all-reduce in flight never queues the reverse all-to-all the embedding update waits
    for.  gloo groups with CUDA tensors (tests: several ranks on one GPU) stage through
    the host, synchronously."""

    def __init__(self, pg, dense_pg=None, separate_dense: bool = True):
        """``separate_dense`` False: the all-reduces share the all-to-all's communicator
        (one stream; the fallback if two concurrent communicators misbehave at W > 1 -
        that overlap has run on 1-rank RCCL and multi-rank gloo only)."""
        import torch.distributed as dist
        self.pg = pg
        if dense_pg is None:
            if separate_dense:
                # the SAME ranks as pg (global rank ids: pg need not be WORLD)
                dense_pg = dist.new_group(ranks=dist.get_process_group_ranks(pg),
                                          backend=dist.get_backend(pg))
            else:
                dense_pg = pg
        self.dense_pg = dense_pg
        # What captures into a hipGraph on this stack (tools/rccl_capture_probe.py,
        # profiles/r06_rccl_capture_probe.txt): RCCL all-reduces (sync or async + wait, on
        # either communicator) and all-gathers capture and replay correctly; an
        # all_to_all_single - warmed eagerly first or not - crashes hipStreamEndCapture
        # (unbounded recursion inside libamdhip64).  So the all-reduces ride inside the
        # step's graphs and only the two all-to-alls run eagerly between them (the
        # round-5 "hang" was this crash in a spawned test worker, its parent waiting on a
        # queue that never filled).  gloo: nothing captures.
        nccl = dist.get_backend(pg) == "nccl" and dist.get_backend(dense_pg) == "nccl"
        self.capturable = False
        self.capture_ar = nccl

    def a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        import torch.distributed as dist
        if out.is_cuda and dist.get_backend(self.pg) == "gloo":
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.pg)
            out.copy_(o)
            return _Done()
        return dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.pg,
                                      async_op=True)

    def allreduce(self, t: torch.Tensor):
        import torch.distributed as dist
        if t.is_cuda and dist.get_backend(self.dense_pg) == "gloo":
            h = t.cpu()
            dist.all_reduce(h, group=self.dense_pg)
            t.copy_(h)
            return _Done()
        return dist.all_reduce(t, group=self.dense_pg, async_op=True)


class EmulatedComm:
    """Rank r of a W-rank job on ONE GPU with no peers (bench --emulate-world): every
    kernel of the step runs at rank r's W-rank shapes (its tables over the global batch,
    the B/W local batch, the rank-major features).  The all-to-all becomes one device copy
    of min(send, recv) bytes on the current stream (the rest of the receive buffer keeps
    whatever it holds); the all-reduce does nothing.  Times the rank's own work, not the
    fabric.  By default it captures like RCCL does (``capture_ar``: the all-reduces inside
    the step's graphs, the all-to-alls eager between four graphs), so the projection pays
    the same graph boundaries as the real path; ``whole=True``: one graph (what the step
    would cost if RCCL's all-to-all captured)."""

    def __init__(self, whole: bool = False):
        self.capturable = bool(whole)
        self.capture_ar = True

    def a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        n = min(int(sum(out_splits)), int(sum(in_splits)))
        if n:
            out.view(-1)[:n].copy_(inp.reshape(-1)[:n])
        return _Done()

    def allreduce(self, t: torch.Tensor):
        return _Done()
