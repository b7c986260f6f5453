"""A/B of the production pre-split GEMM body (x6d) on the C3 step shapes: exact-f32 body vs
x6d without output planes vs x6d with the step's epilogue and c_planes; graph-timed us.

    python tools/x6d_probe.py
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "dlrm-yx_amd")]
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

dev = "cuda"


def main():
    torch.manual_seed(0)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    B = 2048
    # (name, N_out, K_in incl. bias column / padding)
    fwd = [("L3", 1024, 480), ("L4", 1024, 1028), ("L5", 512, 1028), ("L6", 256, 516)]
    for name, N, K in fwd:
        X = torch.relu(torch.randn(B, K, device=dev))
        W = torch.randn(N, K, device=dev) * 0.03
        XP, WP = ops.split_planes(X), ops.split_planes(W)
        Y = torch.empty(B, N + 4, device=dev)
        YP = ops.planes_empty(B, N + 4, dev)
        f32 = ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0]
        x6 = ops.gemm_problem(X, W, trans_b=True, C=Y, a_planes=XP, b_planes=WP)[0]
        x6e = ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU, a_planes=XP,
                               b_planes=WP, c_planes=YP)[0]
        t = [timeit(lambda pr=pr: ops.gemm_group([pr], ws)) * 1e6 for pr in (f32, x6, x6e)]
        print(f"{name} fwd   {B}x{N}x{K}: f32 {t[0]:6.1f}  x6d {t[1]:6.1f}  x6d+relu+planes "
              f"{t[2]:6.1f} us", flush=True)
    bwd = [("L4", 1024, 1024), ("L5", 512, 1024), ("L3", 1024, 480), ("L6", 256, 512)]
    for name, N, K in bwd:
        G = torch.randn(B, N, device=dev)
        X = torch.relu(torch.randn(B, K + 4, device=dev))
        W = torch.randn(N, K + 4, device=dev) * 0.03
        GP, XP, WP = ops.split_planes(G), ops.split_planes(X), ops.split_planes(W)
        dX = torch.empty(B, K, device=dev)
        dXP = ops.planes_empty(B, K, dev)
        d32 = ops.gemm_problem(G, W[:, :K], C=dX, epilogue=ops.EPI_DRELU, aux=X)[0]
        d6 = ops.gemm_problem(G, W[:, :K], C=dX, epilogue=ops.EPI_DRELU, aux=X, a_planes=GP,
                              b_planes=WP, c_planes=dXP)[0]
        Wc = W.clone()
        w32 = ops.gemm_problem(G, X[:, :K], trans_a=True, C=Wc, alpha=1e-6, epilogue=ops.EPI_SGD,
                               ones_col=K)[0]
        w6 = ops.gemm_problem(G, X[:, :K], trans_a=True, C=Wc, alpha=1e-6, epilogue=ops.EPI_SGD,
                              ones_col=K, a_planes=GP, b_planes=XP, c_planes=WP)[0]
        t = [timeit(lambda pr=pr: ops.gemm_group([pr], ws)) * 1e6 for pr in (d32, d6, w32, w6)]
        s6 = ops.gemm_splits(w6)
        print(f"{name} dgrad {B}x{K}x{N}: f32 {t[0]:6.1f}  x6d+drelu+planes {t[1]:6.1f} | wgrad "
              f"{N}x{K}x{B}: f32 {t[2]:6.1f}  x6d+sgd+planes {t[3]:6.1f} (x6d split {s6})",
              flush=True)


if __name__ == "__main__":
    main()
