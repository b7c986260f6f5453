"""Synthetic DLRM inputs in the reference's layouts (dlrm_data_pytorch.py:596-1228).

Host generators mirror the reference's numpy draws (same global-RNG consumption order,
so a seeded run reproduces its batches); the table-batched CSR flatten has a device
variant (ops.csr_from_tables).  Device-side random batches for benchmarking live in
DLRMTrainer.synthetic_batch.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from . import ops


def generate_uniform_input_batch(m_den, ln_emb, n, num_indices_per_lookup,
                                 num_indices_per_lookup_fixed, rng=np.random):
    """dlrm_data_pytorch.py:1109-1161: X ~ U[0,1) [n, m_den]; per table n bags of sorted
    unique indices (fixed L: redrawn until exactly L unique — needs rows >= L)."""
    Xt = torch.tensor(rng.rand(n, m_den).astype(np.float32))
    lS_o: List[torch.Tensor] = []
    lS_i: List[torch.Tensor] = []
    for size in ln_emb:
        offs, idxs, offset = [], [], 0
        for _ in range(n):
            if num_indices_per_lookup_fixed:
                if size < num_indices_per_lookup:
                    raise ValueError("fixed L larger than the table never terminates "
                                     "(dlrm_data_pytorch.py:1134-1138)")
                group = np.int64(num_indices_per_lookup)
                while True:
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
    P = rng.rand(n, num_targets).astype(np.float32)
    if round_targets:
        P = np.round(P).astype(np.float32)
    return torch.tensor(P)


def batched_csr(lS_o: Sequence[torch.Tensor], lS_i: Sequence[torch.Tensor]):
    """Table-batched flatten (dlrm_data_pytorch.py:834-843): int32 indices = cat(lS_i),
    int32 offsets [T*B+1] = cat(lS_o[t] + start[t]) ++ [total].  Runs the device kernel
    when the inputs are on the GPU, numpy otherwise."""
    if lS_o[0].is_cuda:
        counts = [int(i.numel()) for i in lS_i]
        off = ops.csr_from_tables(list(lS_o), counts, int(lS_o[0].numel()))
        return off, torch.cat([i.reshape(-1) for i in lS_i]).int()
    counts = [int(i.numel()) for i in lS_i]
    starts = np.concatenate([[0], np.cumsum(counts)])
    off = np.concatenate([np.asarray(o, dtype=np.int64) + s for o, s in zip(lS_o, starts[:-1])]
                         + [starts[-1:]])
    idx = np.concatenate([np.asarray(i, dtype=np.int64).reshape(-1) for i in lS_i])
    return torch.tensor(off.astype(np.int32)), torch.tensor(idx.astype(np.int32))


def log1p_dense(X: torch.Tensor) -> torch.Tensor:
    """The cached random path feeds log(X + 1) (dlrm_data_pytorch.py:727)."""
    return torch.log(X.to(torch.float32) + 1)
