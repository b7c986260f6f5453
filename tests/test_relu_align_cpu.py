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


def _c4_like_run(steps=3, lr=1e-3):
    """The small model (BCE) with RWSAdagrad over a few steps, with the permuted twin and
    AdagradBound the GPU tests use; returns (ref, twin, bound, opt)."""
    import numpy as np
    ref = _model()
    tw = RA.PermutedTwin(ref, 6, world=2)
    ab = RA.AdagradBound(ref, lr)
    opt = O.RWSAdagradOracle(ref.parameters(), lr=lr)
    opt2 = O.RWSAdagradOracle(tw.model.parameters(), lr=lr)
    rng = np.random.RandomState(5)
    for _ in range(steps):
        X, lS_o, lS_i = _batch()
        X = X + torch.tensor(rng.rand(*X.shape).astype("float32"))
        T = torch.tensor(rng.randint(0, 2, (6, 1)).astype("float32"))
        E = ref.loss_fn(ref(X, lS_o, lS_i), T)
        opt.zero_grad()
        E.backward()
        opt.step()
        ab.after_step(opt)
        E2 = tw.model.loss_fn(tw.model(*tw.batch(X, lS_o, lS_i, T)[:3]), tw.batch(X, lS_o, lS_i, T)[3])
        opt2.zero_grad()
        E2.backward()
        opt2.step()
    return ref, tw, ab, opt


def test_adagrad_bound_rejects_an_error_in_a_well_conditioned_dense_weight():
    """the conditioning allowance must not hide a real error.  The
    element with the smallest AdagradBound allowance (a large |g| against its error bound,
    a large Adagrad sum S) gets a 1e-4 error: close_explained must reject it, with the
    permuted twin and the bound in place; the untouched weights must pass."""
    ref, tw, ab, opt = _c4_like_run()
    L, L2 = ref.top_l[0], tw.model.top_l[0]
    bound = ab.bound[id(L.weight)]
    S = opt.state[id(L.weight)]["sum"]
    spread = (L.weight.detach() - L2.weight.detach()).abs().double()
    # well conditioned: S >> 0 (a unit that saw gradients), a small allowance and a small
    # twin spread
    score = bound + RA.SPREAD * spread + (S.double() < 1e-8) * 1e9
    i = divmod(int(torch.argmin(score)), score.shape[1])
    assert float(S[i]) >= 1e-8
    assert float(bound[i]) < 1e-6 and float(spread[i]) < 1e-6, (float(bound[i]), float(spread[i]))
    got = L.weight.detach().clone().double()
    st = RA.ExplainStats()
    ok, msg, n = RA.close_explained(got.numpy(), L.weight, L2.weight, bound, "dense", st)
    assert ok and n == 0 and st.compared == got.numel(), msg
    got[i] += 1e-4
    ok, msg, _ = RA.close_explained(got.numpy(), L.weight, L2.weight, bound, "dense", st)
    assert not ok and "Adagrad conditioning allowance" in msg, msg
    # and the caps see what an allowance was used for
    got[i] -= 1e-4
    j = divmod(int(torch.argmax(bound)), bound.shape[1])
    got[j] += 0.5 * float(bound[j]) + 1e-5 * max(1.0, abs(float(L.weight[j])))
    st2 = RA.ExplainStats()
    ok, _, _ = RA.close_explained(got.numpy(), L.weight, L2.weight, bound, "dense", st2)
    if float(bound[j]) > RA.SPREAD * float(spread[j]) * 2:  # explained by the bound only
        assert ok and st2.n_bound == 1 and st2.max_bound_err > 0, st2


def test_permuted_twin_rejects_an_error_in_a_table_row():
    """A 1e-4 error in an updated embedding row and in a row no lookup touched: tw.close
    must reject both (a table has no conditioning allowance, only the twin's spread)."""
    ref, tw, _, opt = _c4_like_run()
    e, e2 = ref.emb_l[0], tw.model.emb_l[0]
    X, lS_o, lS_i = _batch()
    touched = int(lS_i[0][0])
    untouched = next(r for r in range(50) if r not in set(lS_i[0].tolist()))
    for row in (touched, untouched):
        got = e.weight.detach().clone().double()
        ok, msg, n = tw.close(got.numpy(), e.weight, e2.weight, "table 0")
        assert ok and n == 0, msg
        got[row, 1] += 1e-4
        ok, msg, _ = tw.close(got.numpy(), e.weight, e2.weight, "table 0")
        assert not ok and "permuted" in msg, (row, msg)
    m, m2 = opt.state[id(e.weight)]["momentum"], None
    assert m.shape[0] == 50 and float(m[touched]) > 0


def test_loss_interval_is_the_oracles_and_rejects_a_wrong_loss():
    """The saturated-step loss check: the interval comes from the
    oracle's logits only, contains the oracle's own loss, is wide only on saturated
    samples, and rejects a loss off by more than the ill-conditioned terms allow."""
    z = torch.tensor([[0.3], [-1.2], [20.0], [-30.0], [16.7]])
    t = torch.tensor([[1.0], [0.0], [0.0], [1.0], [0.0]])
    tau = torch.full_like(z, 1e-3)
    lo, hi, n_ill = RA.loss_interval(z, tau, t)
    own = float(RA._bce_terms(torch.sigmoid(z.float()), t).mean())
    assert lo <= own <= hi
    assert n_ill == 2  # z = 20 and 16.7 with t = 0: log(1 - p) of a p within an ulp of 1
    # (z = -30 with t = 1 is well conditioned: log(p) of a tiny but exact p)
    lo2, hi2, n2 = RA.loss_interval(z[:2], tau[:2], t[:2])
    assert n2 == 0 and hi2 == lo2  # unsaturated: the oracle's own terms
    assert not (lo2 - 1e-5 <= own + 1e-3 <= hi2 + 1e-5)
