"""One C3 GEMM shape repeated (for rocprofv3 --pmc passes): L4 forward 2048x1024x1028 on the
x6d body from planes (arg "x6d") or on the exact-f32 body (arg "f32")."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402

dev = "cuda"
which = sys.argv[1] if len(sys.argv) > 1 else "x6d"
torch.manual_seed(0)
B, N, K = 2048, 1024, 1028
X = torch.relu(torch.randn(B, K, device=dev))
W = torch.randn(N, K, device=dev) * 0.03
Y = torch.empty(B, N, device=dev)
ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
kw = dict(a_planes=ops.split_planes(X), b_planes=ops.split_planes(W)) if which == "x6d" else {}
pr = ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU, **kw)[0]
for _ in range(50):
    ops.gemm_group([pr], ws)
torch.cuda.synchronize()
print(which, "done")
