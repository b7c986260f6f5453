"""wgrad with the bias as a row sum (ones_col) vs the folded bias column, per shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402
from gemm_group_ab import timeit  # noqa: E402


def main():
    dev = "cuda"
    B = 2048
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    for (K, N) in [(512, 256), (256, 128), (479, 1024), (1024, 1024)]:
        Kp = (K + 4) // 4 * 4
        for dist in ("randn", "rand"):
            mk = torch.randn if dist == "randn" else torch.rand
            g = torch.randn(B, N, device=dev)
            x = mk(B, Kp, device=dev)
            W = torch.randn(N, Kp, device=dev)
            res = []
            for split in ("", "2", "4", "8"):
                if split:
                    os.environ["DLRM_GEMM_SPLIT"] = split
                    os.environ["DLRM_GEMM_CFG"] = "64x64"
                else:
                    os.environ.pop("DLRM_GEMM_SPLIT", None)
                    os.environ.pop("DLRM_GEMM_CFG", None)
                t_fold = timeit(lambda: ops.gemm(g, x[:, :Kp], trans_a=True, C=W, alpha=1e-9,
                                                 epilogue=ops.EPI_SGD, workspace=ws))
                t_rs = -1.0
                if K % 4 == 0:
                    t_rs = timeit(lambda: ops.gemm(g, x[:, :K], trans_a=True, C=W, alpha=1e-9,
                                                   epilogue=ops.EPI_SGD, ones_col=K, workspace=ws))
                res.append(f"s{split or 'auto'}: fold {t_fold:.1f} rs {t_rs:.1f}")
            print(f"wgrad {N}x{K} {dist:5s} " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
