"""Distributed golden fixtures (SURVEY.md §8c fixture viii) from the REFERENCE itself.

Runs the reference's own multi-process path on CPU with the gloo backend, W = 2 and 4
ranks: ext_dist.init_distributed (extend_distributed.py:81-207), DLRM_Net built in
distributed mode (sharders.shard + local tables, dlrm_s_pytorch.py:443-474), the MLPs
wrapped in ext_dist.DDP (:1626-1633), inputs sliced exactly as dlrm_wrap does (:130-153),
DLRM_Net.distributed_forward (:686-730: local lookups on the full batch -> All2All_Req /
All2All_Wait, extend_distributed.py:405-508 -> interaction -> top MLP), the loss on the
rank's slice of the targets (:1903-1907), backward and torch.optim.SGD.

Every rank loads the same global initial weights (drawn once by a single-process
DLRM_Net under a seed), so the ranks' results are comparable with one single-process
model (the reference's per-rank init differs under seeding: SURVEY.md §8e item 4).

Written: tests/golden/dist.npz with, per (W, sharder) case and rank r:
  Z and loss of 3 SGD steps, the step-0 embedding gradients of the rank's local tables
  (dense form of the sparse COO grads) and DDP-averaged dense gradients, the final local
  tables and dense parameters.  Inputs and initial weights are stored once.

With --qr (BASELINE configs[4]'s model, C4, across ranks): the same W-rank gloo run with
--qr-flag (QREmbeddingBag for tables above QR_THRESHOLD rows, dlrm_s_pytorch.py:282-290,
tricks/qr_embedding_bag.py:113-174) and the reference's RWSAdagrad (optim/rwsadagrad.py:
56-122) over the driver's three parameter groups (dlrm_s_pytorch.py:1636-1666).  Written:
tests/golden/dist_qr.npz with, per (W, sharder, operation) case and rank r: Z and loss of
3 steps, the final local tables (quotient / remainder for QR tables), their row-wise
momentum, the final dense parameters and their Adagrad sums.

Runs only in the build container (imports /root/reference); the GPU box reads the .npz.
Usage:  python tests/golden/make_golden_dist.py [--ref /root/reference] [--qr]
"""
from __future__ import annotations

import argparse
import os
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

M_SPA = 8
LN_EMB = [300, 40, 1000, 7, 120]
LN_BOT = [13, 32, 8]
LN_TOP = [23, 16, 1]
B = 12
STEPS = 3
LR = 0.05
CASES = [(2, "naive_chunk"), (2, "naive"), (2, "greedy"), (4, "naive_chunk"), (4, "greedy")]
# --qr: tables 0 (300 rows), 2 (1000) and 4 (120) become QR tables, 1 and 3 stay plain
QR_THRESHOLD = 100
QR_COLLISIONS = 4
QR_LR = 0.05
QR_SCALE = 0.2
QR_CASES = [(2, "greedy", "mult"), (2, "naive", "add"), (4, "greedy", "mult")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_state(R):
    """Initial weights (single-process DLRM_Net, numpy seed 77) and 3 input batches drawn
    by the reference's own generate_uniform_input_batch (variable L <= 5)."""
    import torch
    R.ext_dist.my_size = -1
    np.random.seed(77)
    net = R.ref.DLRM_Net(M_SPA, np.array(LN_EMB), np.array(LN_BOT), np.array(LN_TOP),
                         arch_interaction_op="dot", sigmoid_top=len(LN_TOP) - 2,
                         loss_function="bce")
    st = {f"init_emb{k}": e.weight.detach().numpy().copy() for k, e in enumerate(net.emb_l)}
    for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
        for name, p in seq.named_parameters():
            st[f"init_{pre}.{name}"] = p.detach().numpy().copy()
    np.random.seed(99)
    rng = np.random.RandomState(8)
    for s in range(STEPS):
        X, lS_o, lS_i = R.dp.generate_uniform_input_batch(13, np.array(LN_EMB), B, 5, False,
                                                          False)
        st[f"s{s}_X"] = torch.log(X + 1).numpy()
        st[f"s{s}_lS_o"] = torch.stack(lS_o).numpy()
        for t, ii in enumerate(lS_i):
            st[f"s{s}_lS_i{t}"] = ii.numpy()
        st[f"s{s}_T"] = rng.randint(0, 2, size=(B, 1)).astype(np.float32)
    return st


def _qr_kw(op):
    return dict(qr_flag=True, qr_collisions=QR_COLLISIONS, qr_operation=op,
                qr_threshold=QR_THRESHOLD)


def _global_state_qr(R):
    """Initial weights of the QR model (single-process DLRM_Net, numpy seed 77 for the plain
    tables and the MLPs, torch seed 77 for QREmbeddingBag.reset_parameters) and the same 3
    input batches as the SGD fixture."""
    import torch
    st = _global_state(R)
    R.ext_dist.my_size = -1
    np.random.seed(77)
    torch.manual_seed(77)
    net = R.ref.DLRM_Net(M_SPA, np.array(LN_EMB), np.array(LN_BOT), np.array(LN_TOP),
                         arch_interaction_op="dot", sigmoid_top=len(LN_TOP) - 2,
                         loss_function="bce", **_qr_kw("mult"))
    for k in list(st):
        if k.startswith("init_"):
            del st[k]
    for k, e in enumerate(net.emb_l):
        if hasattr(e, "weight_q"):
            # QR_SCALE: at the reference's QR init (U[sqrt(1/n), 1] per factor) every case's
            # sigmoid is saturated before the first step (BCE 33.3 = clamped logs): scaled
            # rows keep the gradients alive, so the fixture pins the update arithmetic
            st[f"init_emb{k}_q"] = e.weight_q.detach().numpy() * np.float32(QR_SCALE)
            st[f"init_emb{k}_r"] = e.weight_r.detach().numpy() * np.float32(QR_SCALE)
        else:
            st[f"init_emb{k}"] = e.weight.detach().numpy().copy()
    for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
        for name, p in seq.named_parameters():
            st[f"init_{pre}.{name}"] = p.detach().numpy().copy()
    return st


def _worker_qr(rank, W, port, sharder, op, ref_dir, st, q):
    """One rank of the reference's C4 run: QR tables + RWSAdagrad, distributed_forward, DDP."""
    try:
        sys.path.insert(0, HERE)
        from make_golden import import_reference
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(W), LOCAL_RANK=str(rank))
        R = import_reference(ref_dir)
        import torch
        torch.set_num_threads(1)
        ed = R.ext_dist
        ed.init_distributed(rank=rank, local_rank=rank, size=W, use_gpu=False, backend="gloo")
        net = R.ref.DLRM_Net(M_SPA, np.array(LN_EMB), np.array(LN_BOT), np.array(LN_TOP),
                             arch_interaction_op="dot", sigmoid_top=len(LN_TOP) - 2,
                             loss_function="bce", sharder=sharder, **_qr_kw(op))
        local = list(net.local_emb_indices)
        with torch.no_grad():  # the same global weights on every rank
            for k, t in enumerate(local):
                e = net.emb_l[k]
                if hasattr(e, "weight_q"):
                    e.weight_q.copy_(torch.tensor(st[f"init_emb{t}_q"]))
                    e.weight_r.copy_(torch.tensor(st[f"init_emb{t}_r"]))
                else:
                    e.weight.copy_(torch.tensor(st[f"init_emb{t}"]))
            for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
                for name, p in seq.named_parameters():
                    p.copy_(torch.tensor(st[f"init_{pre}.{name}"]))
        net.bot_l = ed.DDP(net.bot_l)
        net.top_l = ed.DDP(net.top_l)
        groups = [{"params": [p for emb in net.emb_l for p in emb.parameters()], "lr": QR_LR},
                  {"params": net.bot_l.parameters(), "lr": QR_LR},
                  {"params": net.top_l.parameters(), "lr": QR_LR}]
        opt = R.RWSAdagrad(groups, lr=QR_LR)
        out = {"local": np.array(local), "device_indices": np.array(net.device_indices)}
        sl = ed.get_my_slice(B)
        for s in range(STEPS):
            X = torch.tensor(st[f"s{s}_X"])[sl]
            lS_o = [torch.tensor(st[f"s{s}_lS_o"][t]) for t in local]
            lS_i = [torch.tensor(st[f"s{s}_lS_i{t}"]) for t in local]
            T = torch.tensor(st[f"s{s}_T"])[sl]
            Z = net(X, lS_o, lS_i)
            E = net.loss_fn(Z, T)
            opt.zero_grad()
            E.backward()
            opt.step()
            out[f"s{s}_Z"] = Z.detach().numpy().copy()
            out[f"s{s}_loss"] = np.array([E.item()], dtype=np.float32)
        for k, t in enumerate(local):
            e = net.emb_l[k]
            if hasattr(e, "weight_q"):
                for part in ("q", "r"):
                    w = getattr(e, f"weight_{part}")
                    out[f"final_emb{t}_{part}"] = w.detach().numpy().copy()
                    out[f"final_mom{t}_{part}"] = opt.state[w]["momentum"].numpy().copy()
            else:
                out[f"final_emb{t}"] = e.weight.detach().numpy().copy()
                out[f"final_mom{t}"] = opt.state[e.weight]["momentum"].numpy().copy()
        for pre, seq in (("bot", net.bot_l.module), ("top", net.top_l.module)):
            for name, p in seq.named_parameters():
                out[f"final_{pre}.{name}"] = p.detach().numpy().copy()
                out[f"final_sum_{pre}.{name}"] = opt.state[p]["sum"].numpy().copy()
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
        q.put((rank, out))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


def _worker(rank, W, port, sharder, ref_dir, st, q):
    try:
        sys.path.insert(0, HERE)
        from make_golden import import_reference
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(W), LOCAL_RANK=str(rank))
        R = import_reference(ref_dir)
        import torch
        torch.set_num_threads(1)
        ed = R.ext_dist
        ed.init_distributed(rank=rank, local_rank=rank, size=W, use_gpu=False, backend="gloo")
        net = R.ref.DLRM_Net(M_SPA, np.array(LN_EMB), np.array(LN_BOT), np.array(LN_TOP),
                             arch_interaction_op="dot", sigmoid_top=len(LN_TOP) - 2,
                             loss_function="bce", sharder=sharder)
        local = list(net.local_emb_indices)
        with torch.no_grad():  # the same global weights on every rank
            for k, t in enumerate(local):
                net.emb_l[k].weight.copy_(torch.tensor(st[f"init_emb{t}"]))
            for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
                for name, p in seq.named_parameters():
                    p.copy_(torch.tensor(st[f"init_{pre}.{name}"]))
        net.bot_l = ed.DDP(net.bot_l)
        net.top_l = ed.DDP(net.top_l)
        opt = torch.optim.SGD(net.parameters(), lr=LR)
        out = {"local": np.array(local), "device_indices": np.array(net.device_indices),
               "n_emb_per_rank": np.array(net.n_emb_per_rank)}
        sl = ed.get_my_slice(B)
        for s in range(STEPS):
            X = torch.tensor(st[f"s{s}_X"])[sl]                      # dlrm_wrap :130-153
            lS_o = [torch.tensor(st[f"s{s}_lS_o"][t]) for t in local]
            lS_i = [torch.tensor(st[f"s{s}_lS_i{t}"]) for t in local]
            T = torch.tensor(st[f"s{s}_T"])[sl]                      # :1903
            Z = net(X, lS_o, lS_i)                                    # distributed_forward
            E = net.loss_fn(Z, T)
            opt.zero_grad()
            E.backward()
            if s == 0:
                for k, t in enumerate(local):
                    out[f"g0_emb{t}"] = net.emb_l[k].weight.grad.to_dense().numpy().copy()
                for pre, seq in (("bot", net.bot_l.module), ("top", net.top_l.module)):
                    for name, p in seq.named_parameters():
                        out[f"g0_{pre}.{name}"] = p.grad.numpy().copy()
            opt.step()
            out[f"s{s}_Z"] = Z.detach().numpy().copy()
            out[f"s{s}_loss"] = np.array([E.item()], dtype=np.float32)
        for k, t in enumerate(local):
            out[f"final_emb{t}"] = net.emb_l[k].weight.detach().numpy().copy()
        for pre, seq in (("bot", net.bot_l.module), ("top", net.top_l.module)):
            for name, p in seq.named_parameters():
                out[f"final_{pre}.{name}"] = p.detach().numpy().copy()
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
        q.put((rank, out))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--qr", action="store_true", help="write dist_qr.npz (QR + RWSAdagrad)")
    args = ap.parse_args()
    sys.path.insert(0, HERE)
    from make_golden import import_reference
    R = import_reference(args.ref)
    import torch.multiprocessing as mp
    if args.qr:
        return main_qr(R, args, mp)
    st = _global_state(R)
    data = dict(st)
    data.update(m_spa=np.array([M_SPA]), ln_emb=np.array(LN_EMB), ln_bot=np.array(LN_BOT),
                ln_top=np.array(LN_TOP), B=np.array([B]), lr=np.array([LR], np.float32),
                steps=np.array([STEPS]))
    ctx = mp.get_context("spawn")
    for W, sharder in CASES:
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_worker, args=(r, W, port, sharder, args.ref, st, q))
              for r in range(W)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(W))
        for p in ps:
            p.join(timeout=60)
        for r in range(W):
            if not isinstance(res[r], dict):
                raise RuntimeError(f"W={W} {sharder} rank {r}:\n{res[r]}")
            for k, v in res[r].items():
                data[f"W{W}_{sharder}_r{r}_{k}"] = v
        print("wrote case", W, sharder, "device_indices", res[0]["device_indices"].tolist())
    np.savez_compressed(os.path.join(args.out, "dist.npz"), **data)
    print("wrote dist.npz")


def main_qr(R, args, mp):
    st = _global_state_qr(R)
    data = dict(st)
    data.update(m_spa=np.array([M_SPA]), ln_emb=np.array(LN_EMB), ln_bot=np.array(LN_BOT),
                ln_top=np.array(LN_TOP), B=np.array([B]), lr=np.array([QR_LR], np.float32),
                steps=np.array([STEPS]), qr_threshold=np.array([QR_THRESHOLD]),
                qr_collisions=np.array([QR_COLLISIONS]), qr_scale=np.array([QR_SCALE], np.float32))
    ctx = mp.get_context("spawn")
    for W, sharder, op in QR_CASES:
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_worker_qr, args=(r, W, port, sharder, op, args.ref, st, q))
              for r in range(W)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(W))
        for p in ps:
            p.join(timeout=60)
        for r in range(W):
            if not isinstance(res[r], dict):
                raise RuntimeError(f"W={W} {sharder} {op} rank {r}:\n{res[r]}")
            for k, v in res[r].items():
                data[f"W{W}_{sharder}_{op}_r{r}_{k}"] = v
        print("wrote case", W, sharder, op, "device_indices", res[0]["device_indices"].tolist(),
              "losses r0", [float(res[0][f"s{s}_loss"][0]) for s in range(STEPS)])
    np.savez_compressed(os.path.join(args.out, "dist_qr.npz"), **data)
    print("wrote dist_qr.npz")


if __name__ == "__main__":
    main()
