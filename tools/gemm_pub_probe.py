"""Cost breakdown of the in-launch split-K hand-off (DLRM_GEMM_PUB 0/1 real, 2 = no records,
3 = records but no hand-off; 2 and 3 compute wrong sums - timing only)."""
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
    os.environ["DLRM_GEMM_CFG"] = "64x64"
    for (K, N) in [(512, 256), (256, 128), (1024, 1024), (1024, 512)]:
        Kp = (K + 4) // 4 * 4
        g = torch.randn(B, N, device=dev)
        x = torch.randn(B, Kp, device=dev)
        W = torch.randn(N, Kp, device=dev)
        line = []
        for split in ("1", "2", "4", "8"):
            os.environ["DLRM_GEMM_SPLIT"] = split
            ts = []
            for pub in ("2", "3", "1", "0"):
                os.environ["DLRM_GEMM_PUB"] = pub
                ts.append(timeit(lambda: ops.gemm(g, x[:, :Kp], trans_a=True, C=W, alpha=1e-9,
                                                  epilogue=ops.EPI_SGD, workspace=ws)))
            line.append(f"s{split}: " + "/".join(f"{t:.1f}" for t in ts))
        print(f"wgrad {N}x{Kp} [nopub/store/wt/fence] " + " | ".join(line), flush=True)
    os.environ["DLRM_GEMM_PUB"] = "1"
    for k in ("DLRM_GEMM_SPLIT", "DLRM_GEMM_CFG"):
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
