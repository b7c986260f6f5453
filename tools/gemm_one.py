"""Run one trainer-shaped GEMM back to back (for rocprofv3 PMC / kernel-trace passes).

    python tools/gemm_one.py --kind fwd --B 2048 --K 1024 --N 1024 [--iters 200] [--cfg 64x32]

kind: fwd (X[B,Kp] . W[N,Kp]^T -> Y, ReLU), dgrad (G[B,N] . W[N,K] -> dX, ReLU'),
wgrad (G^T[N,B] . X[B,K] -> W, fused SGD, PARTIAL + REDUCE as in the trainer).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402


def pad4(n):
    return (n + 3) // 4 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="fwd")
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--cfg", default="")
    ap.add_argument("--split", default="")
    args = ap.parse_args()
    if args.cfg:  # plan override (dlrm_set_tuning, this thread)
        bm, bn = (int(v) for v in args.cfg.split("x")[:2])
        ops.tuning(gemm_tile=bm * 1000 + bn, gemm_split=int(args.split or 0)).__enter__()
    dev = "cuda"
    B, K, N = args.B, args.K, args.N
    Kp = pad4(K + 1)
    torch.manual_seed(0)
    X = torch.randn(B, Kp, device=dev)
    W = torch.randn(N, Kp, device=dev) * 0.01
    Y = torch.empty(B, pad4(N + 1), device=dev)
    G = torch.randn(B, N, device=dev)
    dX = torch.empty(B, Kp, device=dev)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    if args.kind == "fwd":
        probs = [[ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0]]]
    elif args.kind == "dgrad":
        nd = K if K % 4 == 0 else Kp
        probs = [[ops.gemm_problem(G, W[:, :nd], C=dX[:, :nd], epilogue=ops.EPI_DRELU, aux=X)[0]]]
    else:
        part = torch.empty(ops.gemm_partial_bytes(N, Kp, 32) // 4 + 64, device=dev)
        pr = ops.gemm_problem(G, X[:, :K], trans_a=True, C=W, alpha=1e-9, epilogue=ops.EPI_SGD,
                              ones_col=K, partial=part, splits=0)[0]
        s = ops.gemm_splits(pr, partial=True)
        pr = ops.gemm_problem(G, X[:, :K], trans_a=True, C=W, alpha=1e-9, epilogue=ops.EPI_SGD,
                              ones_col=K, partial=part, splits=s)[0]
        probs = [[pr]]
        if s > 1:
            probs.append([ops.reduce_problem(pr)])
    for _ in range(args.iters):
        for p in probs:
            ops.gemm_group(p, ws)
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    for _ in range(args.iters):
        for p in probs:
            ops.gemm_group(p, ws)
    e_.record()
    torch.cuda.synchronize()
    t = s_.elapsed_time(e_) / args.iters * 1e-3
    print(f"{args.kind} B{B} K{K} N{N}: {t * 1e6:.1f} us/iter (eager), "
          f"{2 * B * N * K / t / 1e12:.1f} TF")


if __name__ == "__main__":
    main()
