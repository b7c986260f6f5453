"""Diagnostics for the C4 trajectory parity test (lr 1e-3): per step, for the dense
elements where the engine and the oracle end furthest apart, the engine / oracle / permuted
twin values, the oracle's gradient, its |dY|^T|X| magnitude and Adagrad sum.

    python tools/c4_explain_probe.py [--lr 1e-3] [--steps 10]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "dlrm-yx_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import bench
    import oracle as O
    import relu_align as RA
    from test_gpu_trainer import _num_int, _rand_batch
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    lr = args.lr
    c = bench.CONFIGS["terabyte_qr_rwsadagrad"]
    rows = [min(r, 20000) for r in c["rows"]]
    D, bot = c["D"], c["bot"]
    ln_top = [_num_int(len(rows), D)] + c["top"]
    B, thr = 256, c["qr"]["threshold"]
    np.random.seed(0)
    torch.manual_seed(0)
    ref = O.OracleDLRM(D, rows, bot, ln_top, loss_function="bce")
    for k, n in enumerate(rows):
        if n > thr:
            ref.emb_l[k] = O.QREmbeddingBagOracle(n, D, 4, "mult")
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=bot, ln_top=ln_top, loss_function="bce",
                        learning_rate=lr, optimizer="rwsadagrad", qr_flag=True, qr_collisions=4,
                        qr_operation="mult", qr_threshold=thr)
    tr = DLRMTrainer.from_oracle(cfg, ref, device="cuda:0")
    relus = RA.align(ref)
    tw = RA.PermutedTwin(ref, B).with_head()
    head = RA.AlignedHead(ref)
    opt = O.RWSAdagradOracle(ref.parameters(), lr=lr)
    opt2 = O.RWSAdagradOracle(tw.model.parameters(), lr=lr)
    lin = [m for seq in (ref.bot_l, ref.top_l) for m in seq if isinstance(m, torch.nn.Linear)]
    lin2 = [m for seq in (tw.model.bot_l, tw.model.top_l) for m in seq
            if isinstance(m, torch.nn.Linear)]
    absdot = {}

    def hook(mod, inp, out):
        xa = inp[0].detach().abs().double()

        def g(gr):
            absdot[id(mod)] = gr.detach().abs().double().t() @ xa
        out.register_hook(g)
    for L in lin:
        L.register_forward_hook(hook)
    hist = []
    rng = np.random.RandomState(1)
    for s in range(args.steps):
        X, lS_o, lS_i, T = _rand_batch(rng, rows, B, 1, bot[0], "bce")
        tr.step(tr.make_batch(X, lS_o, lS_i, T))
        masks = RA.engine_masks(tr, B, B)
        dz = tr._bufs[(B, B)]["dz"].cpu()
        RA.queue(relus, masks)
        tw.queue(masks)
        head.push(dz, T, B)
        tw.push_head(dz, T, B)
        Xt, ot, it, Tt = (torch.tensor(X), torch.tensor(lS_o), [torch.tensor(i) for i in lS_i],
                          torch.tensor(T))
        E = ref.loss_fn(ref(Xt, ot, it), Tt)
        opt.zero_grad()
        E.backward()
        grads = [L.weight.grad.detach().clone() for L in lin]
        opt.step()
        X2, o2, i2, T2 = tw.batch(Xt, ot, it, Tt)
        E2 = tw.model.loss_fn(tw.model(X2, o2, i2), T2)
        opt2.zero_grad()
        E2.backward()
        opt2.step()
        eng = [W.cpu() for W, _ in tr.dense_state()]
        hist.append(dict(eng=eng, ref=[L.weight.detach().clone() for L in lin],
                         twin=[L.weight.detach().clone() for L in lin2], g=grads,
                         S=[opt.state[id(L.weight)]["sum"].clone() for L in lin],
                         A=[absdot[id(L)].clone() for L in lin]))
    print("flips", RA.report(relus)[2], "head aligned", head.aligned, tw.head.aligned)
    last = hist[-1]
    for li in range(len(lin)):
        err = (last["eng"][li].double() - last["ref"][li].double()).abs()
        spread = (last["twin"][li].double() - last["ref"][li].double()).abs()
        ex = err - 1e-5 - 4 * spread
        k = int(torch.argmax(ex))
        i, j = divmod(k, err.shape[1])
        print(f"layer {li} {tuple(err.shape)}: max err {float(err.max()):.3g}, worst excess "
              f"{float(ex.max()):.3g} at ({i},{j}); n(err>1e-5)={int((err > 1e-5).sum())}")
        if float(ex.max()) > 0:
            for s, h in enumerate(hist):
                print(f"   s{s}: eng {float(h['eng'][li][i, j]):+.8f} ref {float(h['ref'][li][i, j]):+.8f}"
                      f" twin {float(h['twin'][li][i, j]):+.8f} g {float(h['g'][li][i, j]):+.4e}"
                      f" A {float(h['A'][li][i, j]):.4e} S {float(h['S'][li][i, j]):.4e}")


if __name__ == "__main__":
    main()
