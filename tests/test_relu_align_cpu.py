"""CPU checks of the explained-ReLU-flip helper the GPU parity tests use (relu_align.py)."""
import torch

import oracle as O
import relu_align as RA


def _model():
    import numpy as np
    np.random.seed(3)
    return O.OracleDLRM(4, [50, 60], [13, 16, 4], [7, 8, 1], loss_function="bce")


def _batch():
    import numpy as np
    rng = np.random.RandomState(4)
    X = torch.tensor(rng.rand(6, 13).astype("float32"))
    lS_o = torch.arange(6).repeat(2, 1)
    lS_i = [torch.tensor(rng.randint(0, 50, 6)), torch.tensor(rng.randint(0, 60, 6))]
    return X, lS_o, lS_i


def test_own_masks_reproduce_plain_relu_exactly():
    X, lS_o, lS_i = _batch()
    plain = _model()
    ref = plain(X, lS_o, lS_i)
    al = _model()
    relus = RA.align(al)
    assert len(relus) == 3  # two bottom ReLUs, one top ReLU (the last top layer is Sigmoid)
    # masks = the oracle's own decisions: identical output, no flips
    acts, h = [], X
    for seq in (plain.bot_l,):
        for m in seq:
            h = m(h)
            if isinstance(m, torch.nn.ReLU):
                acts.append(h > 0)
    x = h
    ly = plain.apply_emb(lS_o, lS_i)
    h = O.interact(x, ly)
    for m in list(plain.top_l)[:-2]:
        h = m(h)
        if isinstance(m, torch.nn.ReLU):
            acts.append(h > 0)
    RA.queue(relus, acts)
    out = al(X, lS_o, lS_i)
    assert torch.equal(out, ref)
    ok, msg, flips = RA.report(relus)
    assert ok and flips == 0, msg


def test_unexplained_flip_is_reported_and_explained_one_is_not():
    lin = torch.nn.Linear(3, 2)
    with torch.no_grad():
        lin.weight.copy_(torch.tensor([[1.0, -1.0, 0.0], [1.0, 1.0, 1.0]]))
        lin.bias.zero_()
    r = RA.AlignedReLU(lin)
    x = torch.tensor([[1.0, 1.0 + 1e-7, 0.0]])  # unit 0: z ~ -1e-7 (rounding), unit 1: z = 2
    z = lin(x)
    r.queue.append(torch.tensor([[True, True]]))  # unit 0 flipped: explained (|z| <= tau)
    out = r(z)
    assert r.flips == 1 and not r.unexplained
    assert float(out[0, 0]) == float(z[0, 0])  # follows the engine's decision
    z = lin(x)
    r.queue.append(torch.tensor([[True, False]]))  # unit 1 (z = 2) flipped: unexplained
    r(z)
    ok, msg, _ = RA.report([r])
    assert not ok and "unit 1" in msg
