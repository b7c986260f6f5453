"""DLRM_Net mirror on the MI355X HIP kernels — the drop-in module surface.

Same class name, constructor signature, methods and attributes as the reference's
DLRM_Net (dlrm_s_pytorch.py:226-989) so that its driver run() (:1165-2244) can use it
unchanged (assign it to the driver's global ``dlrm``, trap 8 of SURVEY.md App. A):

  create_mlp / create_emb / create_emb_batched / apply_mlp / apply_emb /
  apply_emb_batched / interact_features / forward / distributed_forward /
  sequential_forward / distribute_batched_emb_data, attributes emb_l, bot_l, top_l,
  loss_fn, v_W_l, ndevices, local_emb_indices, n_emb_per_rank, batched_emb, ...

Initialisation consumes numpy's global RNG in the reference order (all tables, then the
bottom and top MLPs), so a seeded construction reproduces the reference weights
bit-exactly.  Compute runs on the HIP kernels: the plain tables of emb_l share one flat
device buffer and apply_emb is ONE table-batched launch; the MLPs are HipMLP
(one fused Function per MLP); the interaction is the MFMA kernel.

Not on this path (documented in DESIGN.md): parallel_forward (single-process multi-GPU;
the MI355X path is one process per GPU) and --load-processed per-table dims.
Mixed-dimension tables (md_flag) are HipPrEmbeddingBag (lookup + bias-free projection
GEMM); learned weighted pooling trains v_W_l through dlrm_tbe_psw_grad.  4/8-bit quantized inference (quantize_embedding) and the fp16 fbgemm TBE
(fbgemm_emb=True) run on dlrm_tbe_forward_rows / dlrm_tbe_backward_sgd_f16.
"""
from __future__ import annotations

import sys
from typing import List

import numpy as np
import torch
import torch.nn as nn
from torch.autograd.profiler import record_function
from torch.nn.parameter import Parameter

from . import extend_distributed as ext_dist
from . import functional as HF
from . import ops, sharders
from .modules import (HipEmbeddingBagList, HipMLP, HipPrEmbeddingBag, HipQREmbeddingBag,
                      HipStandaloneEmbeddingBag,
                      Optimizer, SplitTableBatchedEmbeddingBags, TableBatchedEmbeddingBags,
                      make_embedding_list)


class DLRM_Net(nn.Module):
    def create_mlp(self, ln, sigmoid_layer):
        """dlrm_s_pytorch.py:227-265 (same init draws: W ~ N(0, sqrt(2/(m+n))) then
        b ~ N(0, sqrt(1/m)) per layer)."""
        layers = []
        for i in range(0, ln.size - 1):
            n, m = int(ln[i]), int(ln[i + 1])
            LL = nn.Linear(n, m, bias=True)
            W = np.random.normal(0.0, np.sqrt(2 / (m + n)), size=(m, n)).astype(np.float32)
            bt = np.random.normal(0.0, np.sqrt(1 / m), size=m).astype(np.float32)
            LL.weight.data = torch.tensor(W, requires_grad=True)
            LL.bias.data = torch.tensor(bt, requires_grad=True)
            layers.append(LL)
            layers.append(nn.Sigmoid() if i == sigmoid_layer else nn.ReLU())
        return HipMLP(*layers)

    def create_emb(self, lm, ln, weighted_pooling=None):
        """dlrm_s_pytorch.py:267-318: plain tables U(+-sqrt(1/n)) (numpy draws in table
        order), QR tables (n > qr_threshold with --qr-flag) as HipQREmbeddingBag."""
        tables: List = []
        extra = {}
        local = []
        for i in range(0, ln.size):
            if ext_dist.my_size > 1 and i not in self.local_emb_indices:
                continue
            local.append(i)
        ln_local = [int(ln[i]) for i in local]
        # with --md-flag, lm is md_solver's per-table dim list (dlrm_s_pytorch.py:1510-1516)
        md_dims = list(lm) if (np.ndim(lm) > 0 and not self.load_processed) else None
        base = int(max(md_dims)) if md_dims is not None else None
        # --load-processed: lm is the per-table dim list of table_configs.json (:1434-1435,
        # create_emb :276-279); the most common dim shares the flat buffer, the other
        # tables are standalone modules (apply_emb splits every output into ln_bot[-1]
        # features, :579-585)
        pdims = [int(lm[i]) for i in local] if self.load_processed else None
        if pdims is not None:
            base = max(sorted(set(pdims)), key=pdims.count) if pdims else int(self.ln_bot[-1])
        elif base is None:
            base = int(lm)
        for j, n in enumerate(ln_local):
            m = pdims[j] if pdims is not None else base
            if self.qr_flag and n > self.qr_threshold:
                extra[j] = HipQREmbeddingBag(n, m, self.qr_collisions,
                                             operation=self.qr_operation, mode="sum",
                                             sparse=True)
                tables.append(None)
            elif self.md_flag and n > self.md_threshold:
                # :291-299: PrEmbeddingBag(n, m[i], max(m)), rows re-drawn from numpy
                _m = int(md_dims[local[j]])
                EE = HipPrEmbeddingBag(n, _m, base)
                W = np.random.uniform(low=-np.sqrt(1 / n), high=np.sqrt(1 / n),
                                      size=(n, _m)).astype(np.float32)
                EE.embs.weight.data = torch.tensor(W)
                extra[j] = EE
                tables.append(None)
            else:
                # (under --md-flag the reference builds nn.EmbeddingBag(n, <dim list>) here
                # and fails; small tables get the base dim instead)
                if self.md_flag:
                    # nn.EmbeddingBag's own init draws from the torch RNG before the numpy
                    # overwrite; keep that stream aligned for the projections drawn later
                    torch.empty(n, m).normal_()
                W = np.random.uniform(low=-np.sqrt(1 / n), high=np.sqrt(1 / n),
                                      size=(n, m)).astype(np.float32)
                if m != base:
                    extra[j] = HipStandaloneEmbeddingBag(n, m, W)
                    tables.append(None)
                else:
                    tables.append(W)
        emb_l = make_embedding_list(ln_local, base, tables, extra, sparse=True)
        if weighted_pooling is None:
            v_W_l = [None] * len(ln_local)
        else:
            v_W_l = [torch.ones(n, dtype=torch.float32) for n in ln_local]
        return emb_l, v_W_l

    def create_emb_batched(self, D, Es, weighted_pooling=None, learning_rate=0.1):
        """dlrm_s_pytorch.py:321-334 (exact SGD fused, lr 0.1 hard-coded like the reference).

        The reference hands table init to the external TableBatchedEmbeddingBags, which is
        not in the reference tree (parity unpinned).  The tables are drawn from a private
        numpy RandomState seeded from torch.initial_seed(), so the global numpy stream the
        MLP init draws from afterwards is the same as the reference's."""
        assert weighted_pooling is None, "Weighted pooling not supported yet!"
        self.Es = Es[self.local_emb_indices] if ext_dist.my_size > 1 else Es
        T = len(self.Es)
        rng = np.random.RandomState(torch.initial_seed() % (2 ** 32))
        tables = [rng.uniform(low=-np.sqrt(1 / n), high=np.sqrt(1 / n),
                              size=(int(n), D)).astype(np.float32) for n in self.Es]
        return TableBatchedEmbeddingBags(T, self.Es, D, optimizer=Optimizer.SGD,
                                         learning_rate=learning_rate, eps=0.1,
                                         stochastic_rounding=False, tables=tables), [None] * T

    def create_emb_fbgemm(self, Ds, Es, weighted_pooling=None):
        """dlrm_s_pytorch.py:337-366: one FP16-weight TBE over the local tables with exact
        SGD fused (modules.SplitTableBatchedEmbeddingBags; fbgemm's default learning rate
        0.01, eps 0.01 as the reference passes it)."""
        T = len(Es)
        emb_indices = ([i for i in range(T) if i in self.local_emb_indices]
                       if ext_dist.my_size > 1 else list(range(T)))
        if not self.load_processed:
            Ds = [Ds] * T
        rng = np.random.RandomState(torch.initial_seed() % (2 ** 32))
        tables = [rng.uniform(low=-np.sqrt(1 / Es[i]), high=np.sqrt(1 / Es[i]),
                              size=(int(Es[i]), int(Ds[i]))).astype(np.float32)
                  for i in emb_indices]
        return SplitTableBatchedEmbeddingBags([(int(Es[i]), int(Ds[i])) for i in emb_indices],
                                              learning_rate=0.01, eps=0.01,
                                              tables=tables), [None] * T

    def __init__(self, m_spa=None, ln_emb=None, ln_bot=None, ln_top=None,
                 arch_interaction_op=None, arch_interaction_itself=False, sigmoid_bot=-1,
                 sigmoid_top=-1, sync_dense_params=True, loss_threshold=0.0, ndevices=-1,
                 qr_flag=False, qr_operation="mult", qr_collisions=0, qr_threshold=200,
                 md_flag=False, md_threshold=200, weighted_pooling=None, loss_function="bce",
                 batched_emb=False, fbgemm_emb=False, load_processed=False, sharder="naive",
                 allocation=None):
        super().__init__()
        if (m_spa is None or ln_emb is None or ln_bot is None or ln_top is None or
                arch_interaction_op is None):
            return
        self.m_spa = m_spa
        self.ln_emb = np.asarray(ln_emb)
        self.ln_bot = np.asarray(ln_bot)
        self.ln_top = np.asarray(ln_top)
        self.ndevices = ndevices
        self.output_d = 0
        self.device_indices = [0]
        self.parallel_model_batch_size = -1
        self.parallel_model_is_not_prepared = True
        self.arch_interaction_op = arch_interaction_op
        self.arch_interaction_itself = arch_interaction_itself
        self.sync_dense_params = sync_dense_params
        self.loss_threshold = loss_threshold
        self.loss_function = loss_function
        if weighted_pooling is not None and weighted_pooling != "fixed":
            self.weighted_pooling = "learned"
        else:
            self.weighted_pooling = weighted_pooling
        self.qr_flag = qr_flag
        if self.qr_flag:
            self.qr_collisions = qr_collisions
            self.qr_operation = qr_operation
            self.qr_threshold = qr_threshold
        self.md_flag = md_flag
        if self.md_flag:
            self.md_threshold = md_threshold
        self.batched_emb = batched_emb
        self.fbgemm_emb = fbgemm_emb
        self.load_processed = load_processed
        self.sharder = sharder
        self.local_emb_indices = list(range(len(self.ln_emb)))
        if ndevices <= 1:
            if ext_dist.my_size > 1:
                n_emb = len(self.ln_emb)
                if n_emb < ext_dist.my_size:
                    sys.exit("only (%d) sparse features for (%d) devices, table partitions will "
                             "fail" % (n_emb, ext_dist.my_size))
                self.n_global_emb = n_emb
                if sharder == "input":
                    self.device_indices = list(map(int, allocation.split(",")))
                else:
                    self.device_indices = sharders.shard(self.ln_emb, ext_dist.my_size, sharder)
                if load_processed:  # per-table dims (:457-460)
                    num_splits = [int(m) // int(self.ln_bot[-1]) for m in m_spa]
                else:
                    num_splits = [m_spa // int(self.ln_bot[-1])] * n_emb
                self.n_emb_per_rank = [0] * ext_dist.my_size
                for i, s in enumerate(num_splits):
                    self.n_emb_per_rank[self.device_indices[i]] += s
                self.local_emb_indices = [i for i, j in enumerate(self.device_indices)
                                          if j == ext_dist.my_local_rank]
            if batched_emb:
                self.emb_l, w_list = self.create_emb_batched(m_spa, self.ln_emb, weighted_pooling)
            elif fbgemm_emb:
                self.emb_l, w_list = self.create_emb_fbgemm(m_spa, self.ln_emb, weighted_pooling)
            else:
                self.emb_l, w_list = self.create_emb(m_spa, self.ln_emb, weighted_pooling)
            if self.weighted_pooling == "learned":
                # :475-478: one trainable weight per row; its gradient comes from the lookup
                # backward (dlrm_tbe_psw_grad) through the per-sample-weight gather
                self.v_W_l = nn.ParameterList()
                for w in w_list:
                    self.v_W_l.append(Parameter(w))
            else:
                self.v_W_l = w_list
        else:
            raise NotImplementedError("single-process multi-GPU (parallel_forward) is replaced "
                                      "by one process per GPU (distributed_forward)")
        self.bot_l = self.create_mlp(self.ln_bot, sigmoid_bot)
        self.top_l = self.create_mlp(self.ln_top, sigmoid_top)
        self.quantize_emb = False
        self.emb_l_q = []
        self.quantize_bits = 32
        if self.loss_function == "mse":
            self.loss_fn = torch.nn.MSELoss(reduction="mean")
        elif self.loss_function == "bce":
            self.loss_fn = torch.nn.BCELoss(reduction="mean")
        else:
            sys.exit("ERROR: --loss-function=" + self.loss_function + " is not supported")

    # ------------------------------------------------------------- apply --
    def apply_mlp(self, x, layers):
        return layers(x)

    def quantize_embedding(self, bits):
        """dlrm_s_pytorch.py:609-625: 4- or 8-bit row-wise quantization of every table with
        the reference's own packers (torch.ops.quantized.embedding_bag_{4bit,byte}_prepack,
        CPU, once); the packed rows are then kept on the device as ONE [sum rows, row_bytes]
        buffer that apply_emb reads with one dlrm_tbe_forward_rows launch."""
        n = len(self.emb_l)
        self.emb_l_q = [None] * n
        if bits not in (4, 8):
            return
        pack = (torch.ops.quantized.embedding_bag_4bit_prepack if bits == 4
                else torch.ops.quantized.embedding_bag_byte_prepack)
        dev = None
        for k in range(n):
            w = self.emb_l[k].weight
            dev = w.device
            self.emb_l_q[k] = pack(w.detach().float().cpu().contiguous())
        rows = [int(q.shape[0]) for q in self.emb_l_q]
        self._q_rows = torch.cat(self.emb_l_q, 0).to(dev)
        self._q_row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64,
                                        device=dev)
        self._q_fmt = ops.ROWS_Q4 if bits == 4 else ops.ROWS_Q8
        self.emb_l = None
        self.quantize_emb = True
        self.quantize_bits = bits

    def _apply_emb_quantized(self, lS_o, lS_i):
        """apply_emb's quantized branch (dlrm_s_pytorch.py:554-567) for all tables in one
        launch: embedding_bag_{4bit,byte}_rowwise_offsets semantics, per-sample weights
        from v_W_l as in the reference."""
        T = len(self.emb_l_q)
        dev = self._q_rows.device
        offs = [lS_o[k].to(dev) for k in range(T)]
        idxs = [lS_i[k].reshape(-1).to(dev) for k in range(T)]
        B = int(offs[0].numel())
        counts = [int(i.numel()) for i in idxs]
        offsets = ops.csr_from_tables(offs, counts, B, out_dtype=torch.int64)
        indices = torch.cat(idxs) if T > 1 else idxs[0]
        psw = None
        if any(w is not None for w in self.v_W_l):
            psw = torch.cat([(self.v_W_l[k].to(dev).gather(0, idxs[k]) if self.v_W_l[k] is not None
                              else torch.ones(counts[k], device=dev)) for k in range(T)])
        D = int(self.m_spa)
        out = ops.tbe_forward_rows(self._q_rows, self._q_fmt, D, self._q_row_base, T, B, indices,
                                   offsets, per_sample_weights=psw)
        return [out[:, k, :] for k in range(T)]

    def apply_emb(self, lS_o, lS_i):
        """dlrm_s_pytorch.py:526-587.  lS_o: [T, B] tensor or T tensors of B bag starts;
        lS_i: [T, N] tensor or T index tensors (table-local rows).  Plain tables run as ONE
        table-batched kernel (device CSR build + pooled sum); QR tables per table."""
        if self.quantize_emb:
            return self._apply_emb_quantized(lS_o, lS_i)
        emb_l = self.emb_l
        T = len(emb_l)
        offs = [lS_o[k] for k in range(T)]
        idxs = [lS_i[k] for k in range(T)]
        ly: List = [None] * T
        if isinstance(emb_l, HipEmbeddingBagList) and emb_l.T > 0:
            plain = emb_l.plain_index
            dev = emb_l.weight_flat.device
            B = int(offs[plain[0]].numel())
            o_list = [offs[t].to(dev) for t in plain]
            i_list = [idxs[t].reshape(-1).to(dev) for t in plain]
            counts = [int(i.numel()) for i in i_list]
            offsets = ops.csr_from_tables(o_list, counts, B, out_dtype=torch.int64)
            indices = torch.cat(i_list) if len(i_list) > 1 else i_list[0]
            psw = None
            if any(self.v_W_l[t] is not None for t in plain):
                psw = torch.cat([self.v_W_l[t].to(dev).gather(0, idxs[t].reshape(-1).to(dev))
                                 for t in plain])
            out = HF.EmbeddingBagsFunction.apply(emb_l, counts, indices, offsets, psw,
                                                 *emb_l.plain_params())
            for j, t in enumerate(plain):
                ly[t] = out[:, j, :]
        for k in range(T):
            if ly[k] is None:  # QR / mixed-dim tables: their own module, on its device
                dk = next(emb_l[k].parameters()).device
                ik, ok_ = idxs[k].to(dk), offs[k].to(dk)
                psw = None if self.v_W_l[k] is None else self.v_W_l[k].to(dk).gather(0, ik)
                ly[k] = emb_l[k](ik, ok_, per_sample_weights=psw)
        d = int(self.ln_bot[-1])
        out_l = []
        for y in ly:
            if y.shape[1] == d:
                out_l.append(y)
            else:
                out_l.extend(y.split(d, dim=1))
        return out_l

    def apply_emb_batched(self, lS_o, lS_i, device_ids=None):
        """dlrm_s_pytorch.py:589-591 (one TBE per device; here one per process)."""
        emb = self.emb_l[0] if isinstance(self.emb_l, nn.ModuleList) else self.emb_l
        return [emb(lS_i[0], lS_o[0])]

    def apply_emb_fbgemm(self, lS_o, lS_i, device_ids=None):
        """dlrm_s_pytorch.py:593-598: [B, T*D] from the fp16 TBE, viewed as [B, T, D]."""
        emb = self.emb_l[0] if isinstance(self.emb_l, nn.ModuleList) else self.emb_l
        y = emb(lS_i[0], lS_o[0])
        B = y.shape[0]
        return [y.reshape(B, -1, int(self.ln_bot[-1]))]

    def interact_features(self, x, ly):
        """dlrm_s_pytorch.py:627-665 on the MFMA interaction kernel."""
        (batch_size, d) = x.shape
        # every tensor wider than d holds several d-wide features (batched [B, T*D] lookups,
        # or the [B/W, T_r*D] per-rank chunks after the all-to-all): view them as [B, k, d]
        ly = [l if (l.dim() == 2 and l.shape[1] == d) else l.reshape(batch_size, -1, d)
              for l in ly]
        if self.arch_interaction_op not in ("dot", "cat"):
            sys.exit("ERROR: --arch-interaction-op=" + self.arch_interaction_op +
                     " is not supported")
        # cat returns [B, F*d] (the shape the top MLP consumes)
        return HF.interact(self.arch_interaction_op, x, ly, self.arch_interaction_itself)

    def flush_index_errors(self) -> None:
        """Raise ops.TBEIndexError if the LAST lookup of any embedding module hit an index
        outside its table.  With the default strict_indices="deferred" a module raises at
        its next forward (one call late, no host sync per lookup); call this after the
        final training / evaluation step so the last call is checked too."""
        if not isinstance(self.emb_l, nn.Module):
            return
        for m in self.emb_l.modules():  # (includes emb_l itself)
            chk = getattr(m, "tbe_errors", None)
            if chk is not None:
                chk.flush()

    # ----------------------------------------------------------- forward --
    def forward(self, dense_x, lS_o, lS_i):
        if ext_dist.my_size > 1:
            return self.distributed_forward(dense_x, lS_o, lS_i)
        if self.ndevices <= 1:
            return self.sequential_forward(dense_x, lS_o, lS_i)
        return self.parallel_forward(dense_x, lS_o, lS_i)

    def _clamp(self, p):
        if 0.0 < self.loss_threshold and self.loss_threshold < 1.0:
            return torch.clamp(p, min=self.loss_threshold, max=(1.0 - self.loss_threshold))
        return p

    def distributed_forward(self, dense_x, lS_o, lS_i):
        """dlrm_s_pytorch.py:686-730: local lookups -> RCCL all-to-all (async) -> bottom MLP
        overlapped -> wait -> interaction -> top MLP."""
        table_sizes = self.ln_emb[self.local_emb_indices].tolist()
        with record_function("module::forward_pass::embedding_lookup",
                             "-".join(str(s) for s in table_sizes)):
            if self.batched_emb:
                ly = self.apply_emb_batched(lS_o, lS_i)
            elif self.fbgemm_emb:
                ly = self.apply_emb_fbgemm(lS_o, lS_i)
            else:
                ly = self.apply_emb(lS_o, lS_i)
            a2a_req = ext_dist.alltoall(ly, self.n_emb_per_rank,
                                        self.batched_emb or self.fbgemm_emb)
        with record_function("module::forward_pass::bottom_mlp"):
            x = self.apply_mlp(dense_x, self.bot_l)
            ly = list(a2a_req.wait())
        with record_function("module::forward_pass::interaction"):
            z = self.interact_features(x, ly)
        with record_function("module::forward_pass::top_mlp"):
            p = self.apply_mlp(z, self.top_l)
        return self._clamp(p)

    def sequential_forward(self, dense_x, lS_o, lS_i):
        """dlrm_s_pytorch.py:732-770."""
        with record_function("module::forward_pass::bottom_mlp"):
            x = self.apply_mlp(dense_x, self.bot_l)
        with record_function("module::forward_pass::embedding_lookup"):
            if self.batched_emb:
                ly = self.apply_emb_batched([lS_o], [lS_i])
            elif self.fbgemm_emb:
                ly = self.apply_emb_fbgemm([lS_o], [lS_i])
            else:
                ly = self.apply_emb(lS_o, lS_i)
        with record_function("module::forward_pass::interaction"):
            z = self.interact_features(x, ly)
        with record_function("module::forward_pass::top_mlp"):
            p = self.apply_mlp(z, self.top_l)
        return self._clamp(p)

    def parallel_forward(self, dense_x, lS_o, lS_i):
        raise NotImplementedError("single-process multi-GPU is replaced by one process per GPU "
                                  "(launch with torch.distributed.run; distributed_forward)")

    def distribute_batched_emb_data(self, batch_size, lS_o, lS_i):
        """dlrm_s_pytorch.py:772-800 (distributed branch): keep the local tables' bags of the
        table-batched CSR and rebase each table's offsets onto the previous one's end."""
        B = batch_size
        T = len(self.ln_emb)
        L = int(lS_i.shape[0] / B / T)
        tmp = []
        for k in range(T):
            o = lS_o[(k * B):((k + 1) * B + 1)]
            tmp.append((o - o[0], lS_i[(k * B * L):((k + 1) * B * L)]))
        tmp_o, tmp_i = [], []
        for k in self.local_emb_indices:
            o, i = tmp[k]
            tmp_o.append(o if not tmp_o else o[1:] + tmp_o[-1][-1])
            tmp_i.append(i)
        return [torch.cat(tmp_o, dim=0)], [torch.cat(tmp_i, dim=0)]
