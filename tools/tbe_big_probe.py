"""Embedding backward + SGD on 8 x 1 M-row tables (D 64, L 100, B 2048: the bench's
fresh-batch HBM shape, one batch re-used); run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

T, R, D, L, B = 8, 1_000_000, 64, 100, 2048
g = torch.Generator(device="cuda").manual_seed(7)
W = torch.empty(T * R, D, device="cuda").uniform_(-0.003, 0.003, generator=g)
rb = torch.arange(T + 1, dtype=torch.int64, device="cuda") * R
idx = torch.randint(0, R, (T * B * L,), dtype=torch.int32, device="cuda", generator=g)
off = torch.arange(T * B + 1, dtype=torch.int32, device="cuda") * L
G = torch.empty(B, T, D, device="cuda").uniform_(-1e-3, 1e-3, generator=g)
ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), T * R, D), dtype=torch.uint8,
                 device="cuda")
t = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-9, workspace=ws,
                                    max_lookups_per_table=B * L), n=10)
print(f"8 x 1M rows, D 64, L 100, B 2048: bwd+sgd {t * 1e6:.1f} us", flush=True)
# the C1 shape with no per-table bound: the device-wide sort (one segment of global keys)
R = 100_000
W = torch.empty(T * R, D, device="cuda").uniform_(-0.003, 0.003, generator=g)
rb = torch.arange(T + 1, dtype=torch.int64, device="cuda") * R
idx = torch.randint(0, R, (T * B * L,), dtype=torch.int32, device="cuda", generator=g)
ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), T * R, D), dtype=torch.uint8,
                 device="cuda")
for mx, what in ((B * L, "tiled per-table sort"), (0, "device-wide sort (no bound)")):
    t = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-9, workspace=ws,
                                        max_lookups_per_table=mx), n=10)
    print(f"C1 shape, {what}: bwd+sgd {t * 1e6:.1f} us", flush=True)
