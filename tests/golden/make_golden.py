"""Generate the golden fixtures in tests/golden/ by running the REFERENCE implementation.

Runs only in the build container (it imports /root/reference, which never exists on the
GPU box).  Outputs are small .npz/.json data files: inputs, initial weights and the
reference's outputs / gradients / updated weights.  The GPU box only reads these files.

Import shims (the reference imports packages absent from this image; see SURVEY.md
Appendix B): torchviz and h5py are stubbed, torch.utils.tensorboard.SummaryWriter is a
no-op class and torch.profiler.ExecutionGraphObserver aliases ExecutionTraceObserver.
None of these stubs is on the code path exercised below.

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def import_reference(ref_dir: str):
    shim = tempfile.mkdtemp(prefix="dlrm_ref_shim_")
    os.makedirs(os.path.join(shim, "torchviz"))
    with open(os.path.join(shim, "torchviz", "__init__.py"), "w") as f:
        f.write("def make_dot(*a, **k):\n    raise RuntimeError('torchviz stub')\n")
    os.makedirs(os.path.join(shim, "h5py"))
    with open(os.path.join(shim, "h5py", "__init__.py"), "w") as f:
        f.write("class File:\n    def __init__(self, *a, **k):\n"
                "        raise RuntimeError('h5py stub')\n")
    sys.path.insert(0, shim)
    import torch.profiler
    if not hasattr(torch.profiler, "ExecutionGraphObserver"):
        torch.profiler.ExecutionGraphObserver = torch.profiler.ExecutionTraceObserver
    tb = types.ModuleType("torch.utils.tensorboard")

    class _SW:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

    tb.SummaryWriter = _SW
    sys.modules["torch.utils.tensorboard"] = tb
    sys.path.insert(0, ref_dir)
    import dlrm_s_pytorch as ref  # noqa: E402
    import extend_distributed as ext_dist  # noqa: E402
    import sharders  # noqa: E402
    import dlrm_data_pytorch as dp  # noqa: E402
    from tricks.qr_embedding_bag import QREmbeddingBag  # noqa: E402
    from optim.rwsadagrad import RWSAdagrad  # noqa: E402
    return types.SimpleNamespace(ref=ref, ext_dist=ext_dist, sharders=sharders, dp=dp,
                                 QREmbeddingBag=QREmbeddingBag, RWSAdagrad=RWSAdagrad)


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def make_net(R, m_spa, ln_emb, ln_bot, ln_top, **kw):
    kw.setdefault("arch_interaction_op", "dot")
    kw.setdefault("sigmoid_top", len(ln_top) - 2)
    kw.setdefault("loss_function", "mse")
    return R.ref.DLRM_Net(m_spa, np.array(ln_emb), np.array(ln_bot), np.array(ln_top), **kw)


def fixed_l_batch(rng, ln_emb, B, L, m_den):
    """Inputs in the reference's non-batched layout: X [B,m_den], lS_o [T,B], lS_i list."""
    X = rng.rand(B, m_den).astype(np.float32)
    offs, idxs = [], []
    for n in ln_emb:
        o, ii = [], []
        for b in range(B):
            o.append(b * L)
            ii.extend(sorted(rng.choice(n, size=L, replace=False).tolist()))
        offs.append(o)
        idxs.append(np.array(ii, dtype=np.int64))
    T = rng.rand(B, 1).astype(np.float32)
    return X, np.array(offs, dtype=np.int64), idxs, T


def gen_c0_training(R, out):
    """C0: 3 tables x 1000 rows, D=4, bot 13-512-4, top 10-4-2-1, B=2, L=10, mse, SGD 0.01."""
    import torch
    ln_emb, ln_bot, ln_top = [1000, 1000, 1000], [13, 512, 4], [10, 4, 2, 1]
    np.random.seed(123)
    torch.manual_seed(123)
    net = make_net(R, 4, ln_emb, ln_bot, ln_top)
    data = {}
    for k, e in enumerate(net.emb_l):
        data[f"init_emb{k}"] = np32(e.weight)
    for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
        for name, p in seq.named_parameters():
            data[f"init_{pre}.{name}"] = np32(p)
    opt = torch.optim.SGD(net.parameters(), lr=0.01)
    rng = np.random.RandomState(7)
    for step in range(3):
        X, lS_o, lS_i, T = fixed_l_batch(rng, ln_emb, 2, 10, 13)
        Xt = torch.log(torch.tensor(X) + 1)
        Z = net(Xt, torch.tensor(lS_o), [torch.tensor(i) for i in lS_i])
        E = net.loss_fn(Z, torch.tensor(T))
        opt.zero_grad()
        E.backward()
        opt.step()
        data[f"s{step}_X"] = np32(Xt)
        data[f"s{step}_lS_o"] = lS_o
        for t, ii in enumerate(lS_i):
            data[f"s{step}_lS_i{t}"] = ii
        data[f"s{step}_T"] = T
        data[f"s{step}_Z"] = np32(Z)
        data[f"s{step}_loss"] = np.array([E.item()], dtype=np.float32)
    for k, e in enumerate(net.emb_l):
        data[f"final_emb{k}"] = np32(e.weight)
    for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
        for name, p in seq.named_parameters():
            data[f"final_{pre}.{name}"] = np32(p)
    np.savez_compressed(os.path.join(out, "c0_train.npz"), **data)


def gen_tbe(R, out):
    """apply_emb (nn.EmbeddingBag sum) fwd + sparse bwd + SGD, variable L with empty bags."""
    import torch
    rng = np.random.RandomState(11)
    for D in (4, 16, 64, 128):
        ln_emb = [1000, 37, 500, 3]
        np.random.seed(5 + D)
        net = make_net(R, D, ln_emb, [4, D], [4, 1])
        B = 16
        lS_o, lS_i = [], []
        for n in ln_emb:
            lens = rng.randint(0, 12, size=B)
            lens[3] = 0  # an empty bag
            o = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            ii = rng.randint(0, n, size=int(lens.sum())).astype(np.int64)  # duplicates allowed
            lS_o.append(o)
            lS_i.append(ii)
        w0 = [np32(e.weight) for e in net.emb_l]
        ly = net.apply_emb(torch.tensor(np.stack(lS_o)), [torch.tensor(i) for i in lS_i])
        g = [rng.randn(B, D).astype(np.float32) for _ in ln_emb]
        loss = sum((y * torch.tensor(gg)).sum() for y, gg in zip(ly, g))
        opt = torch.optim.SGD([e.weight for e in net.emb_l], lr=0.1)
        opt.zero_grad()
        loss.backward()
        opt.step()
        data = {"D": np.array([D]), "rows": np.array(ln_emb), "B": np.array([B])}
        for t in range(len(ln_emb)):
            data[f"w0_{t}"] = w0[t]
            data[f"lS_o{t}"] = lS_o[t]
            data[f"lS_i{t}"] = lS_i[t]
            data[f"out{t}"] = np32(ly[t])
            data[f"g{t}"] = g[t]
            data[f"w1_{t}"] = np32(net.emb_l[t].weight)
        np.savez_compressed(os.path.join(out, f"tbe_D{D}.npz"), **data)


def gen_interaction(R, out):
    import torch
    rng = np.random.RandomState(13)
    for F, D, itself in ((4, 4, False), (9, 64, False), (27, 128, False), (27, 16, False),
                         (9, 64, True), (27, 128, True)):
        T = F - 1
        np.random.seed(3)
        net = make_net(R, D, [10] * T, [4, D], [D + 4, 1], arch_interaction_itself=itself)
        B = 8
        x = torch.tensor(rng.randn(B, D).astype(np.float32), requires_grad=True)
        ly = [torch.tensor(rng.randn(B, D).astype(np.float32), requires_grad=True)
              for _ in range(T)]
        Rz = net.interact_features(x, ly)
        g = rng.randn(*Rz.shape).astype(np.float32)
        (Rz * torch.tensor(g)).sum().backward()
        data = {"F": np.array([F]), "D": np.array([D]), "itself": np.array([int(itself)]),
                "x": np32(x), "ly": np.stack([np32(y) for y in ly], axis=1), "R": np32(Rz),
                "g": g, "gx": np32(x.grad), "gly": np.stack([np32(y.grad) for y in ly], axis=1)}
        np.savez_compressed(os.path.join(out, f"interact_F{F}_D{D}_s{int(itself)}.npz"), **data)
    # cat interaction
    F, D = 5, 16
    np.random.seed(3)
    net = make_net(R, D, [10] * (F - 1), [4, D], [F * D, 1], arch_interaction_op="cat")
    x = torch.tensor(rng.randn(8, D).astype(np.float32), requires_grad=True)
    ly = [torch.tensor(rng.randn(8, D).astype(np.float32), requires_grad=True) for _ in range(F - 1)]
    Rz = net.interact_features(x, ly)
    np.savez_compressed(os.path.join(out, "interact_cat.npz"), x=np32(x),
                        ly=np.stack([np32(y) for y in ly], axis=1), R=np32(Rz).reshape(8, -1))


def gen_mlp(R, out):
    """create_mlp init (numpy RNG order) + fwd/bwd of the C3-width bottom and a top MLP."""
    import torch
    rng = np.random.RandomState(17)
    for tag, ln, sig in (("bot_c3", [13, 512, 256, 128], -1), ("top_small", [479, 64, 32, 1], 2)):
        np.random.seed(99)
        net = make_net(R, 4, [10, 10], [4, 4], [4, 1])
        seq = net.create_mlp(np.array(ln), sig)
        B = 16
        x = torch.tensor(rng.randn(B, ln[0]).astype(np.float32), requires_grad=True)
        y = seq(x)
        g = rng.randn(*y.shape).astype(np.float32)
        (y * torch.tensor(g)).sum().backward()
        data = {"ln": np.array(ln), "sigmoid_layer": np.array([sig]), "x": np32(x), "y": np32(y),
                "g": g, "gx": np32(x.grad)}
        for name, p in seq.named_parameters():
            data[f"p.{name}"] = np32(p)
            data[f"grad.{name}"] = np32(p.grad)
        np.savez_compressed(os.path.join(out, f"mlp_{tag}.npz"), **data)
    # loss functions (dlrm_s_pytorch.py:504-516)
    Z = torch.tensor(rng.rand(32, 1).astype(np.float32), requires_grad=True)
    Tt = torch.tensor(np.round(rng.rand(32, 1)).astype(np.float32))
    data = {"Z": np32(Z), "T": np32(Tt)}
    for lf in ("mse", "bce"):
        net = make_net(R, 4, [10, 10], [4, 4], [4, 1], loss_function=lf)
        Zc = Z.detach().clone().requires_grad_(True)
        L = net.loss_fn(Zc, Tt)
        L.backward()
        data[f"{lf}_loss"] = np.array([L.item()], dtype=np.float32)
        data[f"{lf}_gZ"] = np32(Zc.grad)
    np.savez_compressed(os.path.join(out, "loss.npz"), **data)


def gen_qr(R, out):
    import torch
    rng = np.random.RandomState(19)
    data = {}
    for op in ("mult", "add", "concat"):
        torch.manual_seed(23)
        n, D, c = 1000, 8, 4
        qr = R.QREmbeddingBag(n, D, c, operation=op, mode="sum", sparse=True)
        data[f"{op}_wq0"] = np32(qr.weight_q)
        data[f"{op}_wr0"] = np32(qr.weight_r)
        B = 12
        lens = rng.randint(0, 6, size=B)
        off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        idx = rng.randint(0, n, size=int(lens.sum())).astype(np.int64)
        data[f"{op}_off"] = off
        data[f"{op}_idx"] = idx
        opt = R.RWSAdagrad(qr.parameters(), lr=0.05)
        for step in range(3):
            y = qr(torch.tensor(idx), torch.tensor(off))
            g = rng.randn(*y.shape).astype(np.float32)
            opt.zero_grad()
            (y * torch.tensor(g)).sum().backward()
            opt.step()
            data[f"{op}_y{step}"] = np32(y)
            data[f"{op}_g{step}"] = g
            data[f"{op}_wq{step + 1}"] = np32(qr.weight_q)
            data[f"{op}_wr{step + 1}"] = np32(qr.weight_r)
            data[f"{op}_momq{step + 1}"] = np32(opt.state[qr.weight_q]["momentum"])
            data[f"{op}_momr{step + 1}"] = np32(opt.state[qr.weight_r]["momentum"])
    # float-division quotient semantics at large indices (c = 3 rounds in fp32)
    big = np.array([0, 1, 2, 3, 16777215, 16777216, 16777217, 25165823, 33554431, 9999999,
                    8388609, 12582911], dtype=np.int64)
    big = np.concatenate([big, rng.randint(0, 40_000_000, size=200)])
    qq = (torch.tensor(big) / 3).long().numpy()
    rr = torch.remainder(torch.tensor(big), 3).long().numpy()
    data["split_idx"] = big
    data["split_q3"] = qq
    data["split_r3"] = rr
    np.savez_compressed(os.path.join(out, "qr.npz"), **data)


def gen_sharders(R, out):
    import sys as _s
    kaggle = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
              27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]
    tb = [10000000, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 10000000, 2953546, 403346, 10,
          2208, 11938, 155, 4, 976, 14, 10000000, 10000000, 10000000, 585935, 12972, 108, 36]
    res = {"kaggle": kaggle, "terabyte": tb, "cases": []}
    for name, Es in (("kaggle", kaggle), ("terabyte", tb)):
        for W in (1, 2, 4, 8):
            for alg in ("naive", "naive_chunk", "greedy", "hardcode"):
                if alg == "hardcode" and W < 2:
                    continue
                res["cases"].append({"tables": name, "W": W, "alg": alg,
                                     "device_indices": [int(v) for v in R.sharders.shard(Es, W, alg)]})
    # split helpers (extend_distributed.py:47-66)
    splits = []
    for n, size in ((4, 2), (5, 3), (13, 4), (2048, 8), (2048, 3), (7, 7)):
        for rank in range(size):
            R.ext_dist.my_size, R.ext_dist.my_rank = size, rank
            sl = R.ext_dist.get_my_slice(n)
            ml, sp = R.ext_dist.get_split_lengths(n)
            splits.append({"n": n, "size": size, "rank": rank, "slice": [sl.start, sl.stop],
                           "my_len": ml, "splits": sp})
    R.ext_dist.my_size, R.ext_dist.my_rank = -1, -1
    res["splits"] = splits
    with open(os.path.join(out, "sharders.json"), "w") as f:
        json.dump(res, f)


def gen_data(R, out):
    """Synthetic generator (fixed L) and the table-batched CSR flatten."""
    import torch
    data = {}
    np.random.seed(31)
    X, lS_o, lS_i = R.dp.generate_uniform_input_batch(13, np.array([50, 200, 1000]), 6, 5, True,
                                                       False)
    data["u_X"] = np32(X)
    for t in range(3):
        data[f"u_o{t}"] = lS_o[t].numpy()
        data[f"u_i{t}"] = lS_i[t].numpy()
    np.random.seed(32)
    P = R.dp.generate_random_output_batch(6, 1, False)
    data["u_T"] = np32(P)
    # batched-emb flatten through RandomDataset.__getitem__ (dlrm_data_pytorch.py:834-843)
    ds = R.dp.RandomDataset(13, np.array([50, 200, 1000]), 24, 0, 4, 3, True, True,
                            reset_seed_on_access=True, rand_seed=41, rand_data_dist="uniform",
                            rand_data_min=0, rand_data_max=1, from_dataset=False)
    X, o, i, T = ds[0]
    data["b_X"] = np32(X)
    data["b_offsets"] = o.numpy()
    data["b_indices"] = i.numpy()
    ds2 = R.dp.RandomDataset(13, np.array([50, 200, 1000]), 24, 0, 4, 3, True, False,
                             reset_seed_on_access=True, rand_seed=41, rand_data_dist="uniform",
                             rand_data_min=0, rand_data_max=1, from_dataset=False)
    X2, o2, i2, T2 = ds2[0]
    for t in range(3):
        data[f"p_o{t}"] = o2[t].numpy()
        data[f"p_i{t}"] = i2[t].numpy()
    np.savez_compressed(os.path.join(out, "data.npz"), **data)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    R = import_reference(args.ref)
    import torch
    torch.set_num_threads(4)
    for fn in (gen_c0_training, gen_tbe, gen_interaction, gen_mlp, gen_qr, gen_sharders, gen_data):
        fn(R, args.out)
        print("wrote", fn.__name__)


if __name__ == "__main__":
    main()
