"""Mixed-dimension embeddings on CPU: the oracle's md_solver and
PrEmbeddingBag restatements vs golden vectors from the reference's own
tricks/md_embedding_bag.py (tests/golden/make_golden_md.py), and the mirror module's
seeded init vs the reference's."""
import numpy as np
import torch

import oracle as O
from conftest import fp32_close


def test_md_solver_matches_reference(golden):
    g = golden("md.npz")
    for c in range(int(g["n_solver"][0])):
        alpha, d0, Bud, rd = g[f"solver{c}_args"]
        d = O.md_solver(g[f"solver{c}_rows"].tolist(), float(alpha),
                        d0=None if d0 < 0 else float(d0), B=None if Bud < 0 else float(Bud),
                        round_dim=bool(rd))
        assert d == g[f"solver{c}_dims"].tolist(), c


def test_pr_embedding_bag_oracle_and_mirror_init(golden):
    from dlrm_hip.modules import HipPrEmbeddingBag
    g = golden("md.npz")
    for c in range(int(g["n_pr"][0])):
        n, m, base = (int(v) for v in g[f"pr{c}_shape"])
        W = torch.from_numpy(g[f"pr{c}_W"])
        P = torch.from_numpy(g[f"pr{c}_P"]) if m < base else None
        y = O.pr_embedding_bag(W, P, torch.from_numpy(g[f"pr{c}_idx"]),
                               torch.from_numpy(g[f"pr{c}_off"]))
        ok, msg = fp32_close(y.numpy(), g[f"pr{c}_y"])
        assert ok, (c, msg)
        torch.manual_seed(100 + c)  # same seed as the generator: same torch RNG stream
        E = HipPrEmbeddingBag(n, m, base)
        assert torch.equal(E.embs.weight.data, W)
        if P is not None:
            assert torch.equal(E.proj.weight.data, P)
        assert set(E.state_dict().keys()) == ({"embs.weight", "proj.weight"} if P is not None
                                              else {"embs.weight"})
