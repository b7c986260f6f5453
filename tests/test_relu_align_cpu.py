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


def test_permuted_twin_explains_only_the_oracles_own_spread():
    X, lS_o, lS_i = _batch()
    T = torch.tensor([[0.0], [1.0], [1.0], [0.0], [1.0], [0.0]])
    m = _model()
    tw = RA.PermutedTwin(m, 6, world=2)  # no AlignedReLU in m: plain ReLUs
    assert sorted(tw.perm[:3].tolist()) == [0, 1, 2] and sorted(tw.perm[3:].tolist()) == [3, 4, 5]
    X2, o2, i2, T2 = tw.batch(X, lS_o, lS_i, T)
    assert torch.equal(X2, X[tw.perm]) and torch.equal(i2[1], lS_i[1][tw.perm])
    for mod, batch in ((m, (X, lS_o, lS_i, T)), (tw.model, (X2, o2, i2, T2))):
        opt = O.RWSAdagradOracle(mod.parameters(), lr=1e-3)
        E = mod.loss_fn(mod(*batch[:3]), batch[3])
        opt.zero_grad()
        E.backward()
        opt.step()
    W, W2 = m.top_l[0].weight, tw.model.top_l[0].weight
    ok, _, n = tw.close(W.detach().numpy(), W, W2)
    assert ok and n == 0
    d = (W.detach() - W2.detach()).abs().double()
    got = W.detach().clone().double()
    got[0, 0] += 1e-5 * max(1.0, abs(float(W[0, 0]))) + RA.SPREAD * float(d[0, 0]) + 1e-7
    ok, msg, _ = tw.close(got.numpy(), W, W2)
    assert not ok and "permuted" in msg


def test_aligned_head_takes_engine_dz_only_for_saturated_samples():
    X, lS_o, lS_i = _batch()
    T = torch.tensor([[0.0], [1.0], [1.0], [0.0], [1.0], [0.0]])

    def saturated(m):
        with torch.no_grad():  # z near the sigmoid's rounding-to-1 point for every sample
            m.top_l[2].bias.fill_(16.6)
        return m
    plain = saturated(_model())
    acts, zs = [], []
    for seq in (plain.bot_l, plain.top_l):
        for mod in seq:
            if isinstance(mod, torch.nn.ReLU):
                mod.register_forward_hook(lambda mm, i, o: acts.append(o > 0))
    plain.top_l[2].register_forward_hook(lambda mm, i, o: zs.append(o.detach()))
    plain(X, lS_o, lS_i)
    dz = RA._bce_dz(zs[0], T, 1.0 / 6)
    for flip, expect_ok in ((False, True), (True, False)):
        m = saturated(_model())
        relus = RA.align(m)
        head = RA.AlignedHead(m)
        RA.queue(relus, acts)
        d = dz.clone()
        if flip:  # a wrong engine dz on a sample whose dz is well-conditioned
            stable = (zs[0].abs() < 10).nonzero()
            i = int(stable[0, 0]) if stable.numel() else 0
            d[i] += 1.0
        head.push(d.numpy(), T.numpy(), 6)
        m.loss_fn(m(X, lS_o, lS_i), T).backward()
        ok, _ = head.report()
        assert ok == expect_ok or (flip and zs[0].abs().min() >= 10)


def test_two_fp32_summation_orders_of_c4_w8_are_explained_by_the_twin():
    """Rehearsal of the C4 W=8 parity check on CPU: the 'engine' is the fp32 oracle itself
    with every rank's samples in another order.  Two correct fp32 implementations of the
    same three steps (QR + RWSAdagrad at lr 1e-3) may differ beyond 1e-5 on a few dense
    elements (Adagrad amplifies cancelled gradients); the ReLU alignment and the permuted
    twin must explain every such element, and nothing else may exceed 1e-5."""
    import test_gpu_dist as TD
    W, B, lr = 8, 64, 1e-3
    _, alloc = TD._c3_spec(W)
    eng = TD._c3_model(True)
    eopt = O.RWSAdagradOracle(eng.parameters(), lr=lr)
    ref = TD._c3_model(True)
    relus = RA.align(ref)
    tw = RA.PermutedTwin(ref, B, W)
    ab = RA.AdagradBound(ref, lr, scale=1.0 / W)
    opt = O.RWSAdagradOracle(ref.parameters(), lr=lr)
    opt2 = O.RWSAdagradOracle(tw.model.parameters(), lr=lr)
    eperm = RA.PermutedTwin(eng, B, W, seed=99)
    inv = [torch.argsort(p) for p in eperm.local]
    for X, lS_o, lS_i, T in TD._c3_batches(B, 3):
        acts = []
        hs = [m.register_forward_hook(lambda mm, i, o: acts.append(o > 0))
              for seq in (eng.bot_l, eng.top_l) for m in seq if isinstance(m, torch.nn.ReLU)]
        O.distributed_step(eng, W, alloc, *eperm.batch(X, lS_o, lS_i, T), lr, optimizer=eopt)
        for h in hs:
            h.remove()
        for r in range(W):
            ms = [a[inv[r]] for a in acts[r * len(relus):(r + 1) * len(relus)]]
            RA.queue(relus, ms)
            tw.queue(ms, rank=r)
        O.distributed_step(ref, W, alloc, X, lS_o, lS_i, T, lr, optimizer=opt)
        ab.after_step(opt)
        O.distributed_step(tw.model, W, alloc, *tw.batch(X, lS_o, lS_i, T), lr, optimizer=opt2)
    assert RA.report(relus)[0] and RA.report(tw.relus)[0]
    lin = lambda m: [x for seq in (m.bot_l, m.top_l) for x in seq  # noqa: E731
                     if isinstance(x, torch.nn.Linear)]
    n_expl = 0
    for L, L2, Le in zip(lin(ref), lin(tw.model), lin(eng)):
        for p, p2, pe in ((L.weight, L2.weight, Le.weight), (L.bias, L2.bias, Le.bias)):
            ok, msg, n = RA.close_explained(pe.detach().numpy(), p, p2, ab.bound[id(p)])
            assert ok, msg
            n_expl += n
            # the conditioning allowance alone explains it too
            ok, msg, _ = RA.close_explained(pe.detach().numpy(), p, p, ab.bound[id(p)])
            assert ok, ("Adagrad bound alone", msg)
    print(f"elements beyond 1e-5 between two fp32 orders, all explained: {n_expl}")
