"""Explained ReLU flips (test infrastructure, used with the oracle).

Two correct fp32 implementations of the same Linear may round a pre-activation that is
within a few ulp of 0 to opposite signs.  The ReLU then passes (or blocks) that sample's
gradient through that unit in one and not the other, and every weight it touches moves by a
full gradient step: a real, legitimate difference far above 1e-5.  Instead of allowing a
COUNT of out-of-bound weights, these tests EXPLAIN every one of them:

* after each engine step the test reads the engine's post-ReLU activations (the trainer's
  bot_act / top_act buffers: its ReLU mask is act > 0, the same mask its DRELU epilogues
  and the interaction backward use);
* the oracle runs the same step with every nn.ReLU replaced by ``AlignedReLU``, which takes
  that mask.  Where the oracle's own sign disagrees with it, the disagreement must be
  EXPLAINED: the oracle's pre-activation z must satisfy |z| <= tau, tau = 4e-5 *
  (|x| . |W|^T + |b|) for that sample and unit (the spread a 1e-5-close input and weight
  set can give a dot product; a few ulp of its magnitude for the rounding alone).  An
  unexplained disagreement is recorded and fails the test;
* the oracle then follows the engine's mask (forward value z or 0, derivative = mask), so
  every later value - Z, loss, tables, dense weights, optimizer state - must match at the
  plain 1e-5 bound, with no element exempt.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn

TAU_REL = 4e-5


class AlignedReLU(nn.Module):
    def __init__(self, linear: nn.Linear):
        super().__init__()
        self.linear = [linear]  # not a submodule (no duplicate parameters)
        self.queue: List[torch.Tensor] = []
        self.flips = 0
        self.unexplained: List[str] = []
        self._x = None
        linear.register_forward_hook(self._keep_input)

    def _keep_input(self, mod, inp, out):
        self._x = inp[0].detach()

    def forward(self, z):
        if not self.queue:
            raise RuntimeError("AlignedReLU: no engine mask queued for this call")
        mask = torch.as_tensor(self.queue.pop(0)).to(torch.bool)
        if mask.shape != z.shape:
            raise RuntimeError(f"AlignedReLU: mask {tuple(mask.shape)} vs z {tuple(z.shape)}")
        mine = z.detach() > 0
        diff = mine != mask
        if bool(diff.any()):
            lin = self.linear[0]
            tau = TAU_REL * (self._x.abs() @ lin.weight.detach().abs().t()
                             + lin.bias.detach().abs())
            bad = diff & (z.detach().abs() > tau)
            self.flips += int(diff.sum())
            for i, j in bad.nonzero().tolist()[:4]:
                self.unexplained.append(f"sample {i} unit {j}: z={float(z[i, j])!r} "
                                        f"tau={float(tau[i, j])!r} engine={bool(mask[i, j])}")
        return torch.where(mask, z, torch.zeros_like(z))


def align(model) -> List[AlignedReLU]:
    """Replace every nn.ReLU of model.bot_l / model.top_l (after its Linear) by an
    AlignedReLU; returns them bottom then top, in layer order."""
    out = []
    for seq in (model.bot_l, model.top_l):
        mods = list(seq)
        for i, m in enumerate(mods):
            if isinstance(m, nn.ReLU):
                a = AlignedReLU(mods[i - 1])
                seq[i] = a
                out.append(a)
    return out


def engine_masks(tr, Bl: int, B: int) -> List[torch.Tensor]:
    """The engine's ReLU masks of its last step, bottom then top (act > 0, [B_local, N])."""
    bufs = tr._bufs[(Bl, B)]
    out = []
    for L, a in zip(tr.bot, bufs["bot_act"]):
        out.append((a[:, :L.N] > 0).cpu())
    for L, a in zip(tr.top[:-1], bufs["top_act"]):
        out.append((a[:, :L.N] > 0).cpu())
    return out


def queue(relus: List[AlignedReLU], masks: List[torch.Tensor]) -> None:
    """Queue one forward's masks (one per AlignedReLU, same order as align())."""
    if len(relus) != len(masks):
        raise ValueError(f"{len(relus)} ReLUs, {len(masks)} masks")
    for r, m in zip(relus, masks):
        r.queue.append(m)


def report(relus: List[AlignedReLU]):
    """(ok, message, flips): ok when every disagreement was explained and every queued mask
    was consumed."""
    bad = [u for r in relus for u in r.unexplained]
    left = sum(len(r.queue) for r in relus)
    flips = sum(r.flips for r in relus)
    if bad or left:
        return False, f"{len(bad)} unexplained ReLU flips ({bad[:4]}), {left} masks unused", flips
    return True, "", flips
