"""Time a few GEMM configs on one shape (used with DLRM_HIP_LIB experiment builds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

M, N, K, ta, tb = (int(v) for v in sys.argv[1].split(","))
cfgs = sys.argv[2].split(",")
dev = "cuda"
A = torch.randn((K, M) if ta else (M, K), device=dev)
B = torch.randn((N, K) if tb else (K, N), device=dev)
C = torch.empty(M, N, device=dev)
out = []
for cfg in cfgs:
    os.environ["DLRM_GEMM_CFG"] = cfg
    os.environ["DLRM_GEMM_SPLIT"] = "1"
    t = timeit(lambda: ops.gemm(A, B, trans_a=bool(ta), trans_b=bool(tb), C=C))
    out.append(f"{cfg}:{t * 1e6:.1f}us")
print(os.environ.get("DLRM_HIP_LIB", "default").split("/")[-1], " ".join(out), flush=True)
