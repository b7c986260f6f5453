"""Device optimizers on the HIP kernels.

``RWSAdagrad`` mirrors optim/rwsadagrad.py:11-122 (same constructor, same state names)
but keeps its state on the GPU — the reference allocates it on the CPU and the driver
therefore refuses rwsadagrad on GPU (dlrm_s_pytorch.py:1636-1637).  Sparse gradients
(COO, possibly uncoalesced, as nn.EmbeddingBag(sparse=True) produces them) are coalesced
and applied by the deterministic sorted TBE backward kernel in row-wise Adagrad mode;
dense gradients use the elementwise Adagrad kernel.
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from . import ops


class RWSAdagrad(Optimizer):
    def __init__(self, params, lr=1e-2, lr_decay=0.0, weight_decay=0.0,
                 initial_accumulator_value=0.0, eps=1e-10):
        if not 0.0 <= lr:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if not 0.0 <= lr_decay:
            raise ValueError("Invalid lr_decay value: {}".format(lr_decay))
        if not 0.0 <= weight_decay:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        if not 0.0 <= initial_accumulator_value:
            raise ValueError("Invalid initial_accumulator_value value: {}".format(
                initial_accumulator_value))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {}".format(eps))
        self.defaults = dict(lr=lr, lr_decay=lr_decay, eps=eps, weight_decay=weight_decay,
                             initial_accumulator_value=initial_accumulator_value)
        super().__init__(params, self.defaults)
        for group in self.param_groups:
            for p in group["params"]:
                self.state[p]["step"] = 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                grad = p.grad
                if "momentum" not in st and "sum" not in st:
                    init = self.defaults["initial_accumulator_value"]
                    if grad.is_sparse:
                        st["momentum"] = torch.full([p.shape[0]], init, dtype=torch.float32,
                                                    device=p.device)
                    else:
                        st["sum"] = torch.full_like(p.data, init, dtype=torch.float32)
                st["step"] += 1
                if group["weight_decay"] != 0:
                    if grad.is_sparse:
                        raise RuntimeError("weight_decay option is not compatible with sparse "
                                           "gradients")
                    grad = grad.add(p.data, alpha=group["weight_decay"])
                clr = group["lr"] / (1.0 + (st["step"] - 1.0) * group["lr_decay"])
                if grad.is_sparse:
                    idx = grad._indices()[0]
                    vals = grad._values().contiguous()
                    n = idx.numel()
                    if n == 0:
                        continue
                    # each lookup its own bag: T=1, B=nnz, offsets = 0..nnz
                    off = torch.arange(n + 1, dtype=torch.int64, device=p.device)
                    rb = torch.tensor([0, p.shape[0]], dtype=torch.int64, device=p.device)
                    ops.tbe_backward("rowwise_adagrad", p.data, rb, 1, n, idx, off, vals,
                                     lr=clr, eps=group["eps"], momentum=st["momentum"])
                else:
                    ops.adagrad_update(p.data, grad.contiguous(), st["sum"], clr, group["eps"])
        return loss


class SparseSGD(Optimizer):
    """torch.optim.SGD (lr only, the DLRM usage) with sparse embedding gradients applied by
    the deterministic sorted TBE backward kernel instead of torch's sparse add_."""

    def __init__(self, params, lr=0.01):
        super().__init__(params, dict(lr=lr))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            lr = group["lr"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    idx = g._indices()[0]
                    vals = g._values().contiguous()
                    n = idx.numel()
                    if n == 0:
                        continue
                    off = torch.arange(n + 1, dtype=torch.int64, device=p.device)
                    rb = torch.tensor([0, p.shape[0]], dtype=torch.int64, device=p.device)
                    ops.tbe_backward("sgd", p.data, rb, 1, n, idx, off, vals, lr=lr)
                else:
                    ops.sgd_update(p.data, g.contiguous(), lr)
        return loss
