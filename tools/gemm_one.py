"""Run one GEMM shape/config N times (for rocprofv3 counter passes).
    DLRM_GEMM_CFG=64x64x32 python tools/gemm_one.py M,N,K,ta,tb [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402

M, N, K, ta, tb = (int(v) for v in sys.argv[1].split(","))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = "cuda"
A = torch.randn((K, M) if ta else (M, K), device=dev)
B = torch.randn((N, K) if tb else (K, N), device=dev)
C = torch.empty(M, N, device=dev)
ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)  # split-K tickets start at 0
blas = os.environ.get("GEMM_ONE_BLAS") == "1"
At = A.t() if ta else A
Bt = B.t() if tb else B
for _ in range(reps):
    if blas:
        torch.matmul(At, Bt, out=C)
    else:
        ops.gemm(A, B, trans_a=bool(ta), trans_b=bool(tb), C=C, workspace=ws)
torch.cuda.synchronize()
print("done")
