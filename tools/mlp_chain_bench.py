"""Time the bottom MLP forward at C3 (B=2048, 13-512-256-128): the row-block chain kernel
(dlrm_mlp_chain_forward) vs the three GEMM launches the trainer otherwise issues."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

dev = "cuda"
pad4 = lambda n: (n + 3) // 4 * 4  # noqa: E731
B, dims = 2048, [13, 512, 256, 128]
X = torch.zeros(B, pad4(dims[0] + 1), device=dev)
X[:, :dims[0]] = torch.rand(B, dims[0], device=dev)
X[:, dims[0]] = 1
layers = []
for k, n in zip(dims[:-1], dims[1:]):
    W = torch.randn(n, pad4(k + 1), device=dev) / k ** 0.5
    Y = torch.zeros(B, pad4(n + 1), device=dev)
    Y[:, n] = 1
    layers.append((W, Y, pad4(k + 1)))
chain = ops.mlp_chain(X, layers)
ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)


def gemms():
    h = X
    for W, Y, kin in layers:
        ops.gemm_group([ops.gemm_problem(h[:, :kin], W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0]], ws)
        h = Y


t_chain = timeit(lambda: ops.mlp_chain_forward(chain))
t_gemm = timeit(gemms)
print(f"chain kernel {t_chain * 1e6:.1f} us, three GEMM launches {t_gemm * 1e6:.1f} us")
