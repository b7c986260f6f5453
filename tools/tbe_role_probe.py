"""The embedding backward's update passes: the standalone block / combine kernels (16 rows
in flight per lane group) vs the same passes as launch roles run alone (4 rows in flight,
lean registers: dlrm_tbe_backward_defer + dlrm_gemm_f32_group_role with no GEMM problems),
at the C1 shape (8 x 1e5 rows, D 64, L 100, B 2048) and the C3 shape (26 tables, D 128,
L 1).  Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

dev = "cuda"


def case(T, R, D, L, B):
    g = torch.Generator(device=dev).manual_seed(7)
    W = torch.empty(T * R, D, device=dev).uniform_(-0.003, 0.003, generator=g)
    rb = torch.arange(T + 1, dtype=torch.int64, device=dev) * R
    idx = torch.randint(0, R, (T * B * L,), dtype=torch.int32, device=dev, generator=g)
    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev) * L
    G = torch.empty(B, T, D, device=dev).uniform_(-1e-3, 1e-3, generator=g)
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), T * R, D), dtype=torch.uint8,
                     device=dev)
    mx = B * L
    ts = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-9, workspace=ws,
                                         max_lookups_per_table=mx), n=10)
    with ops.tuning(tbe_lean=1):
        t16 = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-9,
                                              workspace=ws, max_lookups_per_table=mx), n=10)

    def roles():
        r = ops.tbe_backward_defer("sgd", W, rb, T, B, idx, off, G, lr=1e-9, workspace=ws,
                                   max_lookups_per_table=mx)
        ops.gemm_group([], None, dev, role=r, phase=1)
        ops.gemm_group([], None, dev, role=r, phase=2)

    tr = timeit(roles, n=10)
    with ops.tuning(tbe_sort=2):
        t3 = timeit(lambda: ops.tbe_backward("sgd", W, rb, T, B, idx, off, G, lr=1e-9,
                                             workspace=ws, max_lookups_per_table=mx), n=10)
    print(f"T={T} R={R} D={D} L={L} B={B}: bwd+sgd {ts * 1e6:.1f} us (16-in-flight passes "
          f"{t16 * 1e6:.1f} us), as roles (alone) {tr * 1e6:.1f} us, "
          f"chunked digit scan {t3 * 1e6:.1f} us", flush=True)


if __name__ == "__main__":
    case(8, 100000, 64, 100, 2048)
    case(8, 100000, 64, 100, 2048)
    case(26, 400000, 128, 1, 2048)
    case(26, 5000, 16, 1, 128)
