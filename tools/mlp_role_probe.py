"""Time the lookup launch's roles apart (MI355X): the bottom-MLP row-block chain alone
(dlrm_mlp_chain_forward) with 1..L layers, the sort-only presort launch alone, and both
roles in one launch - C3 (13-512-256-128, B 2048 / 256) and C2 (13-512-256-64-16, B 128).
Prints microseconds per launch (mean over reps, events on the current stream)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402

dev = "cuda:0"


def setup(rows, dims, seed=5):
    g = torch.Generator(device=dev).manual_seed(seed)
    pad4 = lambda n: (n + 3) // 4 * 4  # noqa: E731
    X = torch.zeros(rows, pad4(dims[0] + 1), device=dev)
    X[:, :dims[0]] = torch.rand(rows, dims[0], generator=g, device=dev)
    X[:, dims[0]] = 1.0
    layers = []
    for k, n in zip(dims[:-1], dims[1:]):
        W = torch.randn(n, pad4(k + 1), generator=g, device=dev) / (k ** 0.5)
        W[:, k + 1:] = 0.0
        Y = torch.zeros(rows, pad4(n + 1), device=dev)
        layers.append((W, Y, pad4(k + 1)))
    return X, layers


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / reps


def sort_case(T, rows_per_table, B, D):
    torch.manual_seed(1)
    idx = torch.randint(0, rows_per_table, (T * B,), dtype=torch.int32, device=dev)
    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev)
    row_base = torch.arange(T + 1, dtype=torch.int64, device=dev) * rows_per_table
    W = torch.zeros(T * rows_per_table, D, device=dev)
    ws = torch.zeros(ops.tbe_backward_workspace_size(T * B, T * rows_per_table, D),
                     dtype=torch.uint8, device=dev)
    return W, row_base, idx, off, ws


def sort_sweep():
    """Sort-only presort launch vs table count, key bits (rows per table) and keys per table."""
    for T in (1, 26):
        for rows in (200, 60000, 10000000):
            for B in (128, 2048):
                W, row_base, idx, off, ws = sort_case(T, rows, B, 4)
                us = timeit(lambda: ops.tbe_forward_presort(W, row_base, T, B, idx, off, ws, B,
                                                            lookup=False))
                print(f"sort T={T:2d} rows={rows:8d} ({int(rows).bit_length():2d} bits) "
                      f"B={B:4d}: {us:7.2f} us", flush=True)


def main():
    if "--sort" in sys.argv:
        sort_sweep()
    for name, dims, B, D in (("C3", [13, 512, 256, 128], 2048, 128),
                             ("C3@256", [13, 512, 256, 128], 256, 128),
                             ("C2", [13, 512, 256, 64, 16], 128, 16)):
        X, layers = setup(B, dims)
        for L in range(1, len(layers) + 1):
            chain = ops.mlp_chain(X, layers[:L])
            us = timeit(lambda: ops.mlp_chain_forward(chain))
            print(f"{name} B={B} chain layers 1..{L}: {us:7.2f} us", flush=True)
        W, row_base, idx, off, ws = sort_case(26, 100000, B, D)
        us = timeit(lambda: ops.tbe_forward_presort(W, row_base, 26, B, idx, off, ws, B,
                                                    lookup=False))
        print(f"{name} B={B} sort-only presort: {us:7.2f} us", flush=True)
        for parts in (1, 2, 4):
            chain = ops.mlp_chain(X, layers, parts=parts)
            us = timeit(lambda: ops.mlp_chain_forward(chain))
            print(f"{name} B={B} chain parts={parts}: {us:7.2f} us", flush=True)
            us = timeit(lambda: ops.tbe_forward_presort(W, row_base, 26, B, idx, off, ws, B,
                                                        bottom=chain, lookup=False))
            print(f"{name} B={B} sort + bottom roles, parts={parts}: {us:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
