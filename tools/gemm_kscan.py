"""Time vs K for one (M, N): separates per-K-tile cost (slope) from fixed cost."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

M, N = (int(v) for v in sys.argv[1].split(","))
cfgs = sys.argv[2].split(",")
dev = "cuda"
for K in (32, 128, 512, 1024, 2048):
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    row = [f"K={K:5d} blas {timeit(lambda: torch.matmul(A, B.t(), out=C)) * 1e6:6.1f}"]
    for cfg in cfgs:
        os.environ["DLRM_GEMM_CFG"] = cfg
        os.environ["DLRM_GEMM_SPLIT"] = "1"
        row.append(f"{cfg} {timeit(lambda: ops.gemm(A, B, trans_b=True, C=C)) * 1e6:6.1f}")
    print("  ".join(row), flush=True)
