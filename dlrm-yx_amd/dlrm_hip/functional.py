"""torch.autograd Functions over the HIP kernels — the drop-in module path.

These back the DLRM_Net mirror (dlrm_net.py) so that the reference driver's
``E.backward(); optimizer.step()`` (dlrm_s_pytorch.py:1923-1934) runs the gfx950
kernels; the perf path (trainer.py) calls the same kernels without autograd.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import ops


# ------------------------------------------------------------------- MLP ----
class MLPFunction(torch.autograd.Function):
    """A whole nn.Sequential[Linear, ReLU|Sigmoid]* as one Function
    (DLRM_Net.create_mlp / apply_mlp, dlrm_s_pytorch.py:227-265, 518-524).

    Forward: one GEMM per layer with bias(+ReLU) fused in the epilogue (sigmoid as a
    separate elementwise kernel).  Backward: the ReLU mask of a hidden activation is
    fused into the dgrad GEMM that produces its gradient (DRELU epilogue), weight
    gradients are g^T x GEMMs, bias gradients deterministic column sums.
    """

    @staticmethod
    def forward(ctx, x, acts: Sequence[str], *params):
        x = x.contiguous()
        outs = []
        h = x
        n = len(acts)
        for i in range(n):
            W, b = params[2 * i], params[2 * i + 1]
            act = acts[i]
            y = ops.gemm(h, W, trans_b=True,
                         epilogue=ops.EPI_BIAS_RELU if act == "relu" else ops.EPI_BIAS, bias=b)
            if act == "sigmoid":
                y = ops.sigmoid_forward(y)
            outs.append(y)
            h = y
        ctx.acts = list(acts)
        ctx.save_for_backward(x, *params, *outs)
        return h

    @staticmethod
    def backward(ctx, gout):
        acts = ctx.acts
        n = len(acts)
        saved = ctx.saved_tensors
        x = saved[0]
        params = saved[1:1 + 2 * n]
        outs = saved[1 + 2 * n:]
        g = gout.contiguous()
        if acts[-1] == "sigmoid":
            g = ops.sigmoid_backward(g, outs[-1])
        elif acts[-1] == "relu":
            g = ops.relu_backward(g, outs[-1])
        grads: List[Optional[torch.Tensor]] = [None] * (2 * n)
        gx = None
        for i in range(n - 1, -1, -1):
            W = params[2 * i]
            inp = outs[i - 1] if i > 0 else x
            grads[2 * i] = ops.gemm(g, inp, trans_a=True)
            db = torch.empty(W.shape[0], dtype=torch.float32, device=g.device)
            ops.colsum(g, out=db)
            grads[2 * i + 1] = db
            if i > 0:
                prev = acts[i - 1]
                if prev == "relu":
                    g = ops.gemm(g, W, epilogue=ops.EPI_DRELU, aux=inp)
                else:
                    g = ops.gemm(g, W)
                    if prev == "sigmoid":
                        g = ops.sigmoid_backward(g, inp)
            elif ctx.needs_input_grad[0]:
                gx = ops.gemm(g, W)
        return (gx, None, *grads)


# ----------------------------------------------------------- interaction ----
class InteractionFunction(torch.autograd.Function):
    """DLRM_Net.interact_features (dlrm_s_pytorch.py:627-665) on the HIP kernels.
    ly: [B, T, D] tensor (table-batched) or T tensors [B, D]."""

    @staticmethod
    def forward(ctx, op: str, itself: bool, x, *ly):
        ly_arg = ly[0] if (len(ly) == 1 and ly[0].dim() == 3) else list(ly)
        R = ops.interact_forward(op, x, ly_arg, itself)
        ctx.op, ctx.itself = op, itself
        ctx.save_for_backward(x, *ly)
        return R

    @staticmethod
    def backward(ctx, gR):
        x, *ly = ctx.saved_tensors
        ly_arg = ly[0] if (len(ly) == 1 and ly[0].dim() == 3) else list(ly)
        gx, gly = ops.interact_backward(ctx.op, x, ly_arg, gR, ctx.itself)
        if isinstance(gly, torch.Tensor):
            gly = [gly]
        return (None, None, gx, *gly)


def interact(op: str, x: torch.Tensor, ly, itself: bool = False) -> torch.Tensor:
    if isinstance(ly, torch.Tensor):
        ly = [ly]
    ly = [y if y.stride(-1) == 1 else y.contiguous() for y in ly]
    return InteractionFunction.apply(op, itself, x if x.stride(1) == 1 else x.contiguous(), *ly)


# ------------------------------------------------------------ embeddings ----
def _error_flag(module, device) -> torch.Tensor:
    """The module's device TBE error flag (int32, created on first use)."""
    f = getattr(module, "tbe_error_flag", None)
    if f is None or f.device != device:
        f = torch.zeros(1, dtype=torch.int32, device=device)
        try:
            module.tbe_error_flag = f
        except AttributeError:
            pass
    return f


class EmbeddingBagsFunction(torch.autograd.Function):
    """Pooled-sum lookup over T tables that live in one flat [sum rows, D] buffer.

    Forward: one dlrm_tbe_forward launch for all tables -> [B, T, D].
    Backward, by mode:
      'sparse' — per-table sparse COO gradients (indices = table-local rows, values =
                 per-lookup gradient rows), exactly what nn.EmbeddingBag(sparse=True)
                 hands torch.optim (dlrm_s_pytorch.py:304-318, 1929-1934);
      'dense'  — dense per-table gradients (deterministic sorted scatter);
      'fused'  — the optimizer runs inside the backward (exact SGD or row-wise Adagrad)
                 and no gradient is returned (TableBatchedEmbeddingBags semantics).
    """

    @staticmethod
    def forward(ctx, module, counts, indices, offsets, per_sample_weights, *table_params):
        B = (offsets.numel() - 1) // module.T
        flag = _error_flag(module, indices.device)
        fmt = getattr(module, "row_format", ops.ROWS_F32)
        if fmt == ops.ROWS_F32:
            out = ops.tbe_forward(module.weight_flat, module.row_base, module.T, B, indices,
                                  offsets, per_sample_weights=per_sample_weights, error_flag=flag)
        else:  # fp16 / quantized rows
            out = ops.tbe_forward_rows(module.weight_flat, fmt, module.D, module.row_base,
                                       module.T, B, indices, offsets,
                                       per_sample_weights=per_sample_weights, error_flag=flag)
        # nn.EmbeddingBag raises IndexError on an out-of-range index; the kernel skips and
        # flags it.  module.strict_indices picks when the flag is read:
        #   "deferred" (default): no host sync - the flag is copied to pinned memory
        #       asynchronously and the NEXT forward of this module raises (or
        #       module.tbe_errors.flush() after the last step);
        #   "sync" / True: read now (one host sync per forward, e.g. for debugging);
        #   False: never (the caller checks the flag itself).
        mode = getattr(module, "strict_indices", "deferred")
        if mode == "sync" or mode is True:
            ops.check_tbe_errors(flag)
        elif mode:
            chk = getattr(module, "tbe_errors", None)
            if chk is None:
                chk = ops.DeferredErrorCheck()
                try:
                    module.tbe_errors = chk
                except AttributeError:
                    chk = None
            if chk is not None:
                chk.poll()
                chk.post(flag)
        ctx.module, ctx.B, ctx.counts = module, B, counts
        ctx.save_for_backward(indices, offsets, per_sample_weights)
        ctx.n_params = len(table_params)
        return out

    @staticmethod
    def backward(ctx, gout):
        m = ctx.module
        indices, offsets, psw = ctx.saved_tensors
        B = ctx.B
        g = gout.contiguous()
        nones = [None] * ctx.n_params
        # learned weighted pooling: the per-sample weights' own gradient, from the weights
        # as they were in the forward (before a fused update below changes them)
        gpsw = None
        if psw is not None and ctx.needs_input_grad[4]:
            gpsw = ops.tbe_psw_grad(m.weight_flat, m.row_base, m.T, B, indices, offsets, g)
        if m.grad_mode == "fused":
            m.fused_update(indices, offsets, g, psw, B)
            return (None, None, None, None, gpsw, *nones)
        mx = max(ctx.counts) if ctx.counts else 0
        if m.grad_mode == "dense":
            gw = torch.zeros_like(m.weight_flat)
            ops.tbe_backward("dense", gw, m.row_base, m.T, B, indices, offsets, g,
                             per_sample_weights=psw, max_lookups_per_table=mx)
            grads = [gw[a:b] for a, b in m.row_ranges]
            return (None, None, None, None, gpsw, *grads)
        # sparse COO per table
        vals = ops.tbe_expand_grad(m.D, m.T, B, offsets, indices.numel(), g,
                                   per_sample_weights=psw)
        counts = ctx.counts
        if counts is None:  # not known on the host: read the table boundaries once
            tb = offsets[::B].to("cpu", torch.int64)
            counts = (tb[1:] - tb[:-1]).tolist()
        grads = []
        o = 0
        for t, (a, b) in enumerate(m.row_ranges):
            c = counts[t]
            idx_t = indices[o:o + c].to(torch.int64).view(1, -1)
            grads.append(torch.sparse_coo_tensor(idx_t, vals[o:o + c], (b - a, m.D)))
            o += c
        return (None, None, None, None, gpsw, *grads)
