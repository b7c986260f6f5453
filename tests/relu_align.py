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
                self.unexplained.append(f"sample {i} unit {j}: z={float(z.detach()[i, j])!r} "
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


# Conditioning of the result itself.  Some elements of a multi-step trajectory are
# ill-conditioned at fp32: Adagrad's step lr * g / (sqrt(S) + eps) turns a gradient that has
# cancelled down to its rounding noise into a full-size step of either sign, and a
# saturated sigmoid turns a 1-ulp change of p into a different BCE gradient.  Two correct
# fp32 implementations then legitimately differ there by more than 1e-5.  PermutedTwin
# measures that per element: a second fp32 oracle runs the SAME steps with the samples of
# each rank's batch in a different order (every sum over the batch - the loss mean, the
# weight and embedding gradients - then rounds differently; mathematically nothing
# changes), following the engine's ReLU / head decisions permuted alike.  The comparison
# becomes
#     |engine - oracle| <= 1e-5 max(1, |oracle|) + SPREAD * |oracle - twin|:
# an element beyond 1e-5 is EXPLAINED only where the reference arithmetic itself moves that
# much under a mere change of summation order; everywhere else the plain 1e-5 bound holds.
SPREAD = 4.0


class PermutedTwin:
    def __init__(self, model, B: int, world: int = 1, seed: int = 1234):
        """Build right after align(model) (deepcopy maps each AlignedReLU's Linear and the
        forward hook bound to it onto the copies).  The permutation keeps every sample in
        its rank's slice of the B-sample batch (W equal slices)."""
        import copy
        import numpy as np
        self.model = copy.deepcopy(model)
        self.relus = [m for seq in (self.model.bot_l, self.model.top_l) for m in seq
                      if isinstance(m, AlignedReLU)]
        self.head = None
        rng = np.random.RandomState(seed)
        bl = B // world
        self.local = [torch.as_tensor(rng.permutation(bl)) for _ in range(world)]
        self.perm = torch.cat([p + r * bl for r, p in enumerate(self.local)])

    def with_head(self):
        self.head = AlignedHead(self.model)
        return self

    def batch(self, X, lS_o, lS_i, T):
        """The batch with its samples permuted (one lookup per bag: offsets unchanged)."""
        p = self.perm
        for o in lS_o:
            if not torch.equal(torch.as_tensor(o).long(), torch.arange(len(p))):
                raise ValueError("PermutedTwin: one-hot bags (offsets = arange) only")
        return (torch.as_tensor(X)[p], lS_o, [torch.as_tensor(i)[p] for i in lS_i],
                torch.as_tensor(T)[p])

    def queue(self, masks, rank: int = 0):
        """Queue one rank's engine ReLU masks, permuted like its samples."""
        pl = self.local[rank]
        queue(self.relus, [torch.as_tensor(m)[pl] for m in masks])

    def push_head(self, dz, target, n: int, rank: int = 0):
        pl = self.local[rank]
        self.head.push(torch.as_tensor(dz).reshape(-1)[pl], torch.as_tensor(target).reshape(-1)[pl],
                       n)

    def close(self, got, ref, twin, what="", stats=None):
        """(ok, message, n_explained) for the engine's value of an oracle quantity ``ref``
        whose twin value is ``twin``.  ``stats``: an ExplainStats that counts the compared
        and explained elements (the tests cap them)."""
        return close_explained(got, ref, twin, None, what, stats)


# Adagrad's step lr * g / (sqrt(S) + eps) is ill-conditioned where g is small against the
# error it can carry: its derivative in g is up to lr / (sqrt(S) + eps).  AdagradBound
# bounds the error of every dense weight gradient g = dY^T X of every step by running
# error analysis (u = ROUND_REL, the relative error allowed per dot product, which also
# covers the <= 1e-5 weight and state differences carried from earlier steps):
#  * forward, per MLP: dX_0 = 0 (bottom: the exact dense input) or u |R| (top: the
#    interaction output); dY_k = u (|X_k| |W_k|^T + |b_k|) + dX_k |W_k|^T, masked by the
#    ReLU to give dX_{k+1}: a pre-activation that cancels to almost nothing is relatively
#    inaccurate, and so is everything computed from it;
#  * backward magnitudes E_k of the terms dY_k is summed from: |dLoss/dz| at the head, then
#    E_k = E_{k+1} |W_{k+1}| masked (top MLP; bottom MLP: E = |dY|);
#  * |error of g_k| <= u E_k^T |X_k| + |dY_k|^T dX_k.
# It accumulates lr * scale * that / (sqrt(S_t) + eps) per element over the steps; close()
# then explains an element by EITHER the permuted twin's spread or this bound.
ROUND_REL = 64 * 2.0 ** -24


class AdagradBound:
    def __init__(self, model, lr: float, eps: float = 1e-10, scale: float = 1.0):
        self.lr, self.eps, self.scale = lr, eps, scale
        self.mlps = {"bot": [m for m in model.bot_l if isinstance(m, nn.Linear)],
                     "top": [m for m in model.top_l if isinstance(m, nn.Linear)]}
        self.bound = {id(p): torch.zeros_like(p, dtype=torch.float64)
                      for Ls in self.mlps.values() for L in Ls for p in (L.weight, L.bias)}
        self.grad = {id(p): torch.zeros_like(p, dtype=torch.float64)
                     for Ls in self.mlps.values() for L in Ls for p in (L.weight, L.bias)}
        self.calls = []  # per forward of an MLP: (which, {k: |X_k|}, {k: |dY_k|})
        for which, Ls in self.mlps.items():
            for k, L in enumerate(Ls):
                L.register_forward_hook(lambda m, i, o, w=which, k=k: self._hook(w, k, i, o))

    def _hook(self, which, k, inp, out):
        if k == 0:
            self.calls.append((which, {}, {}))
        _, xs, dys = self.calls[-1]
        xs[k] = inp[0].detach().abs().double()
        if out.requires_grad:
            out.register_hook(lambda g: dys.__setitem__(k, g.detach().abs().double()))

    def after_step(self, opt) -> None:
        """Call after the oracle optimizer's step (its state holds the new sums)."""
        u = ROUND_REL
        for which, xs, dys in self.calls:
            Ls = self.mlps[which]
            n = len(Ls)
            Wa = [L.weight.detach().abs().double() for L in Ls]
            ba = [L.bias.detach().abs().double() for L in Ls]
            dX = torch.zeros_like(xs[0]) if which == "bot" else u * xs[0]
            dXs = []
            for k in range(n):  # forward error bounds
                dXs.append(dX)
                dY = u * (xs[k] @ Wa[k].t() + ba[k]) + dX @ Wa[k].t()
                dX = dY * (xs[k + 1] > 0) if k + 1 < n else None
            E = dys[n - 1]
            for k in range(n - 1, -1, -1):  # backward magnitudes + the gradient bound
                if which == "bot":
                    E = dys[k]
                gw = u * (E.t() @ xs[k]) + dys[k].t() @ dXs[k]
                gb = u * E.sum(0)
                self.grad[id(Ls[k].weight)].add_(gw)
                self.grad[id(Ls[k].bias)].add_(gb)
                if which == "top" and k > 0:
                    E = (E @ Wa[k]) * (xs[k] > 0)
        self.calls = []
        for Ls in self.mlps.values():
            for L in Ls:
                for p in (L.weight, L.bias):
                    S = opt.state[id(p)]["sum"].double()
                    g = self.grad[id(p)]
                    self.bound[id(p)].add_(self.lr * self.scale * g / (S.sqrt() + self.eps))
                    g.zero_()


class ExplainStats:
    """What the explained comparisons used, for the tests' caps: elements compared, those
    beyond 1e-5 explained by the permuted twin's spread (``n_twin``), those explained ONLY
    by the Adagrad conditioning allowance (``n_bound``), and the largest error among the
    latter (``max_bound_err``, to compare with lr: one Adagrad step moves an element by
    at most ~lr)."""

    def __init__(self):
        self.compared = 0
        self.n_twin = 0
        self.n_bound = 0
        self.max_bound_err = 0.0

    @property
    def n_explained(self):
        return self.n_twin + self.n_bound

    def __repr__(self):
        return (f"ExplainStats(compared={self.compared}, twin={self.n_twin}, "
                f"bound={self.n_bound}, max_bound_err={self.max_bound_err:.3g})")


def close_explained(got, ref, twin, bound=None, what="", stats=None):
    """(ok, message, n_explained): |got - ref| <= 1e-5 max(1, |ref|) + max(SPREAD |ref -
    twin|, bound) element-wise (bound: an AdagradBound allowance, or None).  An element
    with a small allowance (a well-conditioned gradient: large |g| against its error, a
    large Adagrad sum S) gets the plain 1e-5 bound (tests/test_relu_align_cpu.py injects
    such errors and checks they are rejected)."""
    import numpy as np
    a = np.asarray(got, dtype=np.float64)
    b = torch.as_tensor(ref).detach().double().numpy()
    c = torch.as_tensor(twin).detach().double().numpy()
    base = 1e-5 * np.maximum(1.0, np.abs(b))
    twin_lim = base + SPREAD * np.abs(b - c)
    extra = SPREAD * np.abs(b - c)
    if bound is not None:
        extra = np.maximum(extra, torch.as_tensor(bound).double().numpy())
    err = np.abs(a - b)
    lim = base + extra
    beyond = err > base
    by_twin = beyond & (err <= twin_lim)
    by_bound = beyond & ~by_twin & (err <= lim)
    n_expl = int(by_twin.sum() + by_bound.sum())
    if stats is not None:
        stats.compared += int(a.size)
        stats.n_twin += int(by_twin.sum())
        stats.n_bound += int(by_bound.sum())
        if by_bound.any():
            stats.max_bound_err = max(stats.max_bound_err, float(err[by_bound].max()))
    if (err > lim).any():
        i = np.unravel_index(np.argmax(err - lim), a.shape)
        bd = float(torch.as_tensor(bound).numpy()[i]) if bound is not None else 0.0
        return False, (f"{what} got {a[i]!r} oracle {b[i]!r} twin {c[i]!r} at {i}: beyond 1e-5, "
                       f"{SPREAD} x the permuted twin's spread and the Adagrad conditioning "
                       f"allowance {bd!r}"), n_expl
    return True, "", n_expl


# The sigmoid + BCE head has its own ill-conditioned points: the reference's BCE backward
# divides by max(p (1 - p), 1e-12), and p rounds to exactly 1.0 for z > ~16.6, so a
# sample's dLoss/dz jumps (to 0 at p == 1, by orders of magnitude inside the clamp) when
# the last bit of its z moves.  AlignedHead treats those samples like ReLU flips: a hook on
# the last Linear's output takes the engine's dz (trainer bufs["dz"]) for the samples whose
# oracle dz is not stable under a +-tau change of z (tau as for the ReLUs), and requires
# every OTHER sample's engine dz to match the oracle's within the fp32 bound.
def _bce_dz(z, t, inv_m):
    p = torch.sigmoid(z)
    dp = (p - t) / torch.clamp((1 - p) * p, min=1e-12) * inv_m
    return dp * (1 - p) * p


class AlignedHead:
    def __init__(self, model):
        lins = [m for m in model.top_l if isinstance(m, nn.Linear)]
        self.last = lins[-1]
        self.queue = []  # (engine dz [n], target [n], 1 / n) per forward of the head
        self.aligned = 0
        self.unexplained: List[str] = []
        self.seen = []  # (oracle z, tau, target) of every forward, for loss_interval()
        self.last.register_forward_hook(self._hook)

    def push(self, dz, target, n: int) -> None:
        dt = self.last.weight.dtype
        self.queue.append((torch.as_tensor(dz).reshape(-1, 1).to(dt),
                           torch.as_tensor(target).reshape(-1, 1).to(dt), 1.0 / n))

    def _hook(self, mod, inp, out):
        if not self.queue:
            raise RuntimeError("AlignedHead: no engine dz queued for this call")
        dz_e, t, inv_m = self.queue.pop(0)
        z = out.detach()
        tau = TAU_REL * (inp[0].detach().abs() @ mod.weight.detach().abs().t()
                         + mod.bias.detach().abs())
        self.seen.append((z.clone(), tau.clone(), t.clone()))
        d0 = _bce_dz(z, t, inv_m)
        dlo, dhi = _bce_dz(z - tau, t, inv_m), _bce_dz(z + tau, t, inv_m)
        scale = torch.clamp(d0.abs(), min=inv_m)
        unstable = ((dlo - d0).abs() > 1e-5 * scale) | ((dhi - d0).abs() > 1e-5 * scale)
        agree = (dz_e - d0).abs() <= 1e-5 * scale
        bad = ~unstable & ~agree
        for i in bad.nonzero()[:, 0].tolist()[:4]:
            self.unexplained.append(f"sample {i}: z={float(z[i, 0])!r} engine dz="
                                    f"{float(dz_e[i, 0])!r} oracle dz={float(d0[i, 0])!r}")
        take = unstable & ~agree
        self.aligned += int(take.sum())
        if out.requires_grad and bool(take.any()):
            out.register_hook(lambda g: torch.where(take, dz_e, g))

    def report(self):
        left = len(self.queue)
        if self.unexplained or left:
            return False, (f"{len(self.unexplained)} unexplained head gradients "
                           f"({self.unexplained[:4]}), {left} queued unused")
        return True, ""


def _bce_terms(p, t):
    """nn.BCELoss's per-sample terms (log clamped at -100, dlrm_s_pytorch.py:170-178) of
    fp32 probabilities p, evaluated in fp64."""
    p, t = p.double(), t.double()
    return -(t * torch.log(p).clamp(min=-100) + (1 - t) * torch.log1p(-p).clamp(min=-100))


def loss_interval(z, tau, t):
    """The BCE loss a correct fp32 engine may report for a batch whose oracle logits are z,
    from the ORACLE's state only.  A sample's clamped BCE term is ILL-CONDITIONED at fp32
    where one ulp of its fp32 probability p moves the term by more than 1e-5 max(1, term)
    (p within a few thousand ulp of 1 for t = 0, or of 0 for t = 1: the clamped log of a
    difference that has cancelled); there the term may be anywhere between its values at
    the fp32 sigmoid of z - tau and z + tau, widened by one ulp of p (the term is monotone
    in p for t in {0, 1}).  Every other sample contributes the oracle's own term.  Returns
    (lo, hi, n_ill): the interval of the batch mean and the number of ill-conditioned
    samples.  The engine's own Z plays no part: a saturated step's loss is checked against
    the oracle's logits."""
    z32 = z.float().reshape(-1)
    tau32 = tau.float().reshape(-1)
    t32 = t.float().reshape(-1)
    p = torch.sigmoid(z32)
    mid = _bce_terms(p, t32)
    up = _bce_terms(torch.nextafter(p, torch.ones_like(p)), t32)
    dn = _bce_terms(torch.nextafter(p, torch.zeros_like(p)), t32)
    ill = torch.maximum((up - mid).abs(), (dn - mid).abs()) > 1e-5 * torch.clamp(mid.abs(), min=1.0)
    p_lo = torch.nextafter(torch.sigmoid(z32 - tau32), torch.zeros_like(p))
    p_hi = torch.nextafter(torch.sigmoid(z32 + tau32), torch.ones_like(p))
    a, b = _bce_terms(p_lo, t32), _bce_terms(p_hi, t32)
    lo = torch.where(ill, torch.minimum(torch.minimum(a, b), mid), mid)
    hi = torch.where(ill, torch.maximum(torch.maximum(a, b), mid), mid)
    return float(lo.mean()), float(hi.mean()), int(ill.sum())
