"""Shared access to tests/golden/dist.npz: the reference's own gloo W = 2 / 4 runs of
distributed_forward + DDP + SGD (tests/golden/make_golden_dist.py, SURVEY.md §8c
fixture viii)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = [(2, "naive_chunk"), (2, "naive"), (2, "greedy"), (4, "naive_chunk"), (4, "greedy")]


def load():
    return np.load(os.path.join(GOLDEN, "dist.npz"), allow_pickle=False)


def config(g):
    return dict(m_spa=int(g["m_spa"][0]), ln_emb=[int(v) for v in g["ln_emb"]],
                ln_bot=[int(v) for v in g["ln_bot"]], ln_top=[int(v) for v in g["ln_top"]])


def batches(g):
    """The 3 global batches: (X [B,13] already log(x+1), lS_o [T,B], lS_i list, T [B,1])."""
    T = len(g["ln_emb"])
    out = []
    for s in range(int(g["steps"][0])):
        out.append((torch.tensor(g[f"s{s}_X"]), torch.tensor(g[f"s{s}_lS_o"]),
                    [torch.tensor(g[f"s{s}_lS_i{t}"]) for t in range(T)],
                    torch.tensor(g[f"s{s}_T"])))
    return out


def init_tables(g):
    return [g[f"init_emb{t}"] for t in range(len(g["ln_emb"]))]


def init_mlp(g):
    """[(W, b)] of the bottom then top Linear layers."""
    out = []
    for pre, n in (("bot", len(g["ln_bot"]) - 1), ("top", len(g["ln_top"]) - 1)):
        for i in range(n):
            out.append((g[f"init_{pre}.{2 * i}.weight"], g[f"init_{pre}.{2 * i}.bias"]))
    return out


def rank_key(W, sharder, r, name):
    return f"W{W}_{sharder}_r{r}_{name}"


# tests/golden/dist_qr.npz: the reference's gloo runs of the C4 model (QR tables above
# qr_threshold rows + RWSAdagrad over the driver's parameter groups); keys
# W{W}_{sharder}_{op}_r{r}_*, QR tables as init_emb{t}_q / _r
QR_CASES = [(2, "greedy", "mult"), (2, "naive", "add"), (4, "greedy", "mult")]


def load_qr():
    return np.load(os.path.join(GOLDEN, "dist_qr.npz"), allow_pickle=False)


def qr_rank_key(W, sharder, op, r, name):
    return f"W{W}_{sharder}_{op}_r{r}_{name}"


def init_tables_qr(g):
    """Per table: [rows, D] (plain) or (weight_q, weight_r) (QR)."""
    out = []
    for t in range(len(g["ln_emb"])):
        if f"init_emb{t}_q" in g:
            out.append((g[f"init_emb{t}_q"], g[f"init_emb{t}_r"]))
        else:
            out.append(g[f"init_emb{t}"])
    return out
