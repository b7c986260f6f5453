"""C4 (Terabyte widths + QR mult + RWSAdagrad) loss trajectory vs learning rate on the
oracle (the reference semantics): tables capped at 20k rows, B = 256, 20 steps over 10
batches.  Shows which lr keeps the loss finite and falling for the C4 bench line.

    python tools/c4_lr_probe.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dlrm-yx_amd")]
import bench  # noqa: E402
import oracle as O  # noqa: E402


def main():
    c = dict(bench.CONFIGS["terabyte_qr_rwsadagrad"])
    rows = [min(r, 20000) for r in c["rows"]]
    D = c["D"]
    ln_top = [bench.num_int(len(rows), D)] + c["top"]
    B = 256
    rng = np.random.RandomState(1)
    batches = []
    for _ in range(10):
        X = torch.log1p(torch.tensor(rng.rand(B, c["bot"][0]).astype(np.float32)))
        lS_o = torch.arange(B).repeat(len(rows), 1)
        lS_i = [torch.tensor(rng.randint(0, n, size=B)) for n in rows]
        T = torch.tensor(np.round(rng.rand(B, 1)).astype(np.float32))
        batches.append((X, lS_o, lS_i, T))
    for lr in (1.0, 0.1, 0.01, 0.001):
        np.random.seed(0)
        torch.manual_seed(0)
        m = O.OracleDLRM(D, rows, c["bot"], ln_top, loss_function="bce")
        for k, n in enumerate(rows):
            if n > c["qr"]["threshold"]:
                m.emb_l[k] = O.QREmbeddingBagOracle(n, D, c["qr"]["collisions"],
                                                    c["qr"]["operation"])
        opt = O.RWSAdagradOracle(m.parameters(), lr=lr)
        losses = []
        for s in range(20):
            X, lS_o, lS_i, T = batches[s % 10]
            E = m.loss_fn(m.forward(X, lS_o, lS_i), T)
            opt.zero_grad()
            E.backward()
            opt.step()
            losses.append(round(float(E), 3))
        print("lr", lr, losses, flush=True)


if __name__ == "__main__":
    main()
