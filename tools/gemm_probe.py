"""Print every (config, split) time for a few GEMM shapes, next to hipBLASLt.

    python tools/gemm_probe.py  M,N,K,ta,tb  [...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import CFGS, timeit  # noqa: E402


def main():
    shapes = sys.argv[1:] or ["4096,4096,4096,0,1", "2048,1024,1028,0,1", "2048,1024,1024,0,0",
                              "1024,1028,2048,1,0"]
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)  # split-K tickets start at 0
    for sh in shapes:
        M, N, K, ta, tb = (int(v) for v in sh.split(","))
        A = torch.randn((K, M) if ta else (M, K), device=dev)
        B = torch.randn((N, K) if tb else (K, N), device=dev)
        C = torch.empty(M, N, device=dev)
        fl = 2 * M * N * K
        At = A.t() if ta else A
        Bt = B.t() if tb else B
        tbl = timeit(lambda: torch.matmul(At, Bt, out=C))
        print(f"{M}x{N}x{K} ta={ta} tb={tb}: hipBLASLt {tbl * 1e6:.1f}us {fl / tbl / 1e12:.1f}TF",
              flush=True)
        res = []
        for cfg in CFGS:
            for s in (1, 2, 3, 4, 6, 8):
                if s > 1 and K // s < 128:
                    continue
                os.environ["DLRM_GEMM_CFG"] = cfg
                os.environ["DLRM_GEMM_SPLIT"] = str(s)
                t = timeit(lambda: ops.gemm(A, B, trans_a=bool(ta), trans_b=bool(tb), C=C,
                                            workspace=ws))
                res.append((t, cfg, s))
        os.environ.pop("DLRM_GEMM_CFG", None)
        os.environ.pop("DLRM_GEMM_SPLIT", None)
        res.sort()
        print("   " + "  ".join(f"{c}/{s}:{t * 1e6:.1f}({fl / t / 1e12:.0f})" for t, c, s in res),
              flush=True)


if __name__ == "__main__":
    main()
