"""Golden vectors for the mixed-dimension trick, produced by the
REFERENCE's own md_solver and PrEmbeddingBag (tricks/md_embedding_bag.py, pure torch).

Runs only in the build container (imports /root/reference).  Writes tests/golden/md.npz:
md_solver dims for several (rows, alpha, d0 / B, round) cases (C2/C3 row counts
included), and one seeded PrEmbeddingBag per (rows, dim, base) case: its init (torch RNG),
a bag batch and its forward output.

Usage:  python tests/golden/make_golden_md.py [--ref /root/reference]
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from tricks.md_embedding_bag import PrEmbeddingBag, md_solver
    import oracle as O
    out = {}
    rows_sets = {"small": [10, 300, 4000, 50, 7], "terabyte": O.TERABYTE_ROWS,
                 "kaggle": O.KAGGLE_ROWS}
    cases = []
    for name, rows in rows_sets.items():
        for alpha in (0.0, 0.25, 0.5):
            for rd in (True, False):
                cases.append((name, rows, alpha, 128.0, None, rd))
        cases.append((name, rows, 0.3, None, 1e6, True))
    for c, (name, rows, alpha, d0, Bud, rd) in enumerate(cases):
        d = md_solver(torch.tensor(rows), alpha, d0=d0, B=Bud, round_dim=rd)
        out[f"solver{c}_rows"] = np.array(rows, dtype=np.int64)
        out[f"solver{c}_args"] = np.array([alpha, -1 if d0 is None else d0,
                                           -1 if Bud is None else Bud, float(rd)])
        out[f"solver{c}_dims"] = np.array([int(v) for v in d.tolist()], dtype=np.int64)
    out["n_solver"] = np.array([len(cases)])
    pr_cases = [(300, 4, 16), (50, 16, 16), (1000, 8, 64)]
    for c, (n, m, base) in enumerate(pr_cases):
        torch.manual_seed(100 + c)
        E = PrEmbeddingBag(n, m, base)
        rng = np.random.RandomState(c)
        lens = rng.randint(0, 4, 12)
        idx = torch.tensor(rng.randint(0, n, int(lens.sum())))
        off = torch.tensor(np.concatenate([[0], np.cumsum(lens)[:-1]]))
        y = E(idx, off).detach().numpy()
        out[f"pr{c}_shape"] = np.array([n, m, base])
        out[f"pr{c}_W"] = E.embs.weight.detach().numpy()
        out[f"pr{c}_P"] = (E.proj.weight.detach().numpy() if m < base
                           else np.zeros((0, 0), np.float32))
        out[f"pr{c}_idx"] = idx.numpy()
        out[f"pr{c}_off"] = off.numpy()
        out[f"pr{c}_y"] = y
    out["n_pr"] = np.array([len(pr_cases)])
    np.savez_compressed(os.path.join(HERE, "md.npz"), **out)
    print("wrote", os.path.join(HERE, "md.npz"))


if __name__ == "__main__":
    main()
