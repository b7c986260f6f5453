"""Mainloop A/B for the C3 wgrad shapes: round-1 pipe kernel (tools/_old/libdlrm_old.so,
forced 64x64x32x32 + split s, its own workspace) vs the current pipelined body in PARTIAL
mode (no reduction).  Run under rocprofv3 --kernel-trace --stats to read per-kernel times."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402
from gemm_ab import load  # noqa: E402


def main():
    old = load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_old", "libdlrm_old.so"))
    dev = "cuda"
    B = 2048
    ws_old = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    for (K, N, s) in [(1024, 1024, 6), (1024, 1024, 4), (1024, 512, 4), (512, 256, 8), (256, 128, 8)]:
        Kp = (K + 4) // 4 * 4
        G = torch.randn(B, N, device=dev)
        X = torch.randn(B, Kp, device=dev)
        W = torch.randn(N, Kp, device=dev)
        os.environ["DLRM_GEMM_CFG"] = "64x64x32x32"
        os.environ["DLRM_GEMM_SPLIT"] = str(s)
        for _ in range(30):
            rc = old.dlrm_gemm_f32(1, 0, N, Kp, B, 1e-9, G.data_ptr(), N, X.data_ptr(), Kp,
                                   W.data_ptr(), Kp, 4, None, None, 0, ws_old.data_ptr(),
                                   ws_old.numel(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0
        torch.cuda.synchronize()
        os.environ["DLRM_GEMM_CFG"] = "64x64"
        part = torch.empty(ops.gemm_partial_bytes(N, Kp, s) // 4, device=dev)
        for ones in (False, True):
            xin = X[:, :K] if ones else X
            pr, _ = ops.gemm_problem(G, xin, trans_a=True, C=W, alpha=1e-9, epilogue=ops.EPI_SGD,
                                     ones_col=K if ones else -1, partial=part, splits=s)
            for _ in range(30):
                ops.gemm_group([pr])
            torch.cuda.synchronize()
            red = ops.reduce_problem(pr)
            for _ in range(30):
                ops.gemm_group([red])
            torch.cuda.synchronize()
        print(f"done {N}x{Kp} s{s}", flush=True)
    for k in ("DLRM_GEMM_SPLIT", "DLRM_GEMM_CFG"):
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
