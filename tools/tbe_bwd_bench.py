"""Time the TBE backward (fused SGD) at C3-like sizes: device radix sort vs per-table sort vs
sorted inside the forward (presort); and the forward with / without the presort."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

TB = [10000000, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 10000000, 2953546, 403346, 10,
      2208, 11938, 155, 4, 976, 14, 10000000, 10000000, 10000000, 585935, 12972, 108, 36]
dev = "cuda"
D, B = 128, 2048
for rows in (TB, TB[:1], [3]):
    T = len(rows)
    W = torch.zeros(sum(rows), D, device=dev)
    rb = torch.tensor([0] + torch.tensor(rows).cumsum(0).tolist(), dtype=torch.int64, device=dev)
    idx = torch.cat([torch.randint(0, n, (B,), device=dev) for n in rows]).int()
    off = torch.arange(0, T * B + 1, dtype=torch.int32, device=dev)
    G = torch.randn(B, T, D, device=dev)
    ws = torch.empty(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D), dtype=torch.uint8,
                     device=dev)
    res = []
    for mx in (0, B):
        t = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-6,
                                            workspace=ws, max_lookups_per_table=mx))
        res.append(f"hint={mx}: {t * 1e6:.1f} us")
    ops.tbe_forward_presort(W, rb, T, B, idx, off, ws, B)
    t = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-6, workspace=ws,
                                        max_lookups_per_table=B, presorted=True))
    res.append(f"presorted: {t * 1e6:.1f} us")
    t = timeit(lambda: ops.tbe_forward(W, rb, T, B, idx, off))
    res.append(f"fwd: {t * 1e6:.1f} us")
    t = timeit(lambda: ops.tbe_forward_presort(W, rb, T, B, idx, off, ws, B))
    res.append(f"fwd+presort: {t * 1e6:.1f} us")
    print(f"T={T}", "  ".join(res), flush=True)
