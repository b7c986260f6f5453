"""Time GEMM variants (split-K hand-off protocol, tiles, splits) on the C3 step shapes.
    python tools/gemm_probe2.py   (env knobs are set per case; each case is graph-timed)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


def main():
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    B = 2048
    X = torch.randn(B, 1028, device=dev)
    W = torch.randn(1024, 1028, device=dev)
    Y = torch.empty(B, 1028, device=dev)
    G = torch.randn(B, 1024, device=dev)
    cases = {
        "fwd 2048x1024x1028": lambda: ops.gemm(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU,
                                               workspace=ws),
        "fwd 2048x512x1028": lambda: ops.gemm(X, W[:512], trans_b=True, C=Y[:, :512],
                                              epilogue=ops.EPI_RELU, workspace=ws),
        "dgrad 2048x1024x1024": lambda: ops.gemm(G, W[:, :1024], C=Y[:, :1024],
                                                 epilogue=ops.EPI_DRELU, aux=X, workspace=ws),
        "wgrad 1024x1024x2048+b": lambda: ops.gemm(G, X[:, :1024], trans_a=True, C=W,
                                                   alpha=1e-9, epilogue=ops.EPI_SGD,
                                                   ones_col=1024, workspace=ws),
        "wgrad 512x1024x2048+b": lambda: ops.gemm(G[:, :512], X[:, :1024], trans_a=True,
                                                  C=W[:512], alpha=1e-9, epilogue=ops.EPI_SGD,
                                                  ones_col=1024, workspace=ws),
        "wgrad 256x512x2048+b": lambda: ops.gemm(G[:, :256], X[:, :512], trans_a=True,
                                                 C=W[:256, :516], alpha=1e-9,
                                                 epilogue=ops.EPI_SGD, ones_col=512,
                                                 workspace=ws),
    }
    for name, fn in cases.items():
        res = []
        for cfg in ("64x64", "128x64", "64x128"):
            os.environ["DLRM_GEMM_CFG"] = cfg
            for split in (1, 2, 4, 8):
                os.environ["DLRM_GEMM_SPLIT"] = str(split)
                for pub in ((0, 1) if split > 1 else (1,)):
                    os.environ["DLRM_GEMM_PUB"] = str(pub)
                    t = timeit(fn)
                    res.append((t, f"{cfg} s{split} pub{pub}"))
        res.sort()
        print(f"{name:24s} best {res[0][0]:7.1f} us ({res[0][1]}); "
              + "  ".join(f"{r}:{t:.1f}" for t, r in res), flush=True)
    for k in ("DLRM_GEMM_CFG", "DLRM_GEMM_SPLIT", "DLRM_GEMM_PUB"):
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
