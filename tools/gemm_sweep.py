"""Sweep GEMM tile shape x split-K for every GEMM of the C3 step (tuning aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402


def pad4(n):
    return (n + 3) // 4 * 4


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e-3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    layers = [(13, 512), (512, 256), (256, 128), (479, 1024), (1024, 1024), (1024, 512),
              (512, 256)]
    tiles = ["64x64", "64x128", "128x64", "128x128"]
    splits = [1, 2, 3, 4, 6, 8, 16]
    dev = "cuda"
    best_total, default_total = 0.0, 0.0
    for li, (K, N) in enumerate(layers):
        Kp = pad4(K + 1)
        X = torch.randn(B, Kp, device=dev)
        W = torch.randn(N, Kp, device=dev)
        Y = torch.empty(B, pad4(N + 1), device=dev)
        G = torch.randn(B, N, device=dev)
        dX = torch.empty(B, Kp, device=dev)
        cases = [("fwd", lambda: ops.gemm(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU))]
        if li != 0:
            cases.append(("dgrad", lambda: ops.gemm(G, W[:, :K], C=dX[:, :K],
                                                     epilogue=ops.EPI_DRELU, aux=X)))
        cases.append(("wgrad", lambda: ops.gemm(G, X, trans_a=True, C=W, alpha=1e-9,
                                                 epilogue=ops.EPI_SGD)))
        fl = 2 * B * N * K
        for name, fn in cases:
            os.environ.pop("DLRM_GEMM_TILE", None)
            os.environ.pop("DLRM_GEMM_SPLIT", None)
            t0 = timeit(fn)
            res = []
            for tile in tiles:
                for s in splits:
                    os.environ["DLRM_GEMM_TILE"] = tile
                    os.environ["DLRM_GEMM_SPLIT"] = str(s)
                    res.append((timeit(fn), tile, s))
            res.sort()
            best_total += res[0][0]
            default_total += t0
            top = " ".join(f"{t}/{s}:{tt*1e6:.1f}" for tt, t, s in res[:4])
            print(f"L{li} {K:5d}->{N:5d} {name:6s} default {t0*1e6:7.1f}us ({fl/t0/1e12:5.1f}TF) "
                  f"best {res[0][0]*1e6:7.1f}us ({fl/res[0][0]/1e12:5.1f}TF) | {top}", flush=True)
    os.environ.pop("DLRM_GEMM_TILE", None)
    os.environ.pop("DLRM_GEMM_SPLIT", None)
    print(f"TOTAL default {default_total*1e6:.1f}us best {best_total*1e6:.1f}us")


if __name__ == "__main__":
    main()
