"""TBE forward / backward (+ fused SGD) at the C1 table shape (8 x 1e5 rows, D=64, L=100,
B=2048: 1.64 M lookups per batch), graph-timed; run under rocprofv3 --kernel-trace --stats
for the per-kernel split."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

dev = "cuda"
T, R, D, L, B = 8, 100000, 64, 100, 2048
if len(sys.argv) > 1:
    T, R, D, L, B = (int(v) for v in sys.argv[1].split(","))
g = torch.Generator(device=dev).manual_seed(7)
W = torch.empty(T * R, D, device=dev).uniform_(-0.003, 0.003, generator=g)
rb = torch.arange(T + 1, dtype=torch.int64, device=dev) * R
idx = torch.randint(0, R, (T * B * L,), dtype=torch.int32, device=dev, generator=g)
off = torch.arange(T * B + 1, dtype=torch.int32, device=dev) * L
G = torch.empty(B, T, D, device=dev).uniform_(-1e-3, 1e-3, generator=g)
ws = torch.empty(ops.tbe_backward_workspace_size(idx.numel(), T * R, D), dtype=torch.uint8,
                 device=dev)
n = T * B * L
tf = timeit(lambda: ops.tbe_forward(W, rb, T, B, idx, off), n=10)
tb = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-9, workspace=ws,
                                     max_lookups_per_table=B * L), n=10)
fb = n * (4 * D + 4) + 4 * (T * B + 1) + 4 * T * B * D
print(f"T={T} R={R} D={D} L={L} B={B}: fwd {tf * 1e6:.1f} us ({fb / tf / 1e9:.0f} GB/s)  "
      f"bwd+sgd {tb * 1e6:.1f} us", flush=True)
