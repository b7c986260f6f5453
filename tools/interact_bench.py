"""Time the dot-interaction forward/backward at the C3 shape (B=2048, F=27, D=128)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

B, F, D = 2048, 27, 128
dev = "cuda"
x = torch.randn(B, D, device=dev)
E = torch.randn(B, F - 1, D, device=dev)
npairs = F * (F - 1) // 2
R = torch.empty(B, D + npairs, device=dev)
gR = torch.randn(B, D + npairs, device=dev)
gx = torch.empty(B, D, device=dev)
gE = torch.empty(B, F - 1, D, device=dev)
for tag in ("default", "v1"):
    if tag == "v1":
        os.environ["DLRM_INTERACT_V1"] = "1"
    tf = timeit(lambda: ops.interact_forward("dot", x, E, False, out=R))
    tb = timeit(lambda: ops.interact_backward("dot", x, E, gR, False, grad_x=gx, grad_ly=gE))
    byt_f = 4 * (B * F * D + B * (D + npairs))
    byt_b = 4 * (B * F * D + B * (D + npairs) + B * F * D)
    print(f"{tag}: fwd {tf * 1e6:.1f} us ({byt_f / tf / 1e9:.0f} GB/s)  "
          f"bwd {tb * 1e6:.1f} us ({byt_b / tb / 1e9:.0f} GB/s)", flush=True)
