"""A/B: the exact-f32 GEMM body with LDS-DMA staging through an S-stage ring
(tools/proto/gemm_dma.hip) vs the production body (ops.gemm), same operands, C3 shapes.

    make -C tools/proto && python tools/dma_probe.py
"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "dlrm-yx_amd")]
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

P = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "proto", "libdlrm_dma.so"))
lib.dlrm_last_error.restype = ctypes.c_char_p
lib.dlrm_dma_gemm.restype = ctypes.c_int32
lib.dlrm_dma_gemm.argtypes = [ctypes.c_int32] * 3 + [ctypes.c_int64] * 3 + [
    ctypes.c_float, P, ctypes.c_int64, P, ctypes.c_int64, P, ctypes.c_int64, P]


def main():
    dev = "cuda"
    torch.manual_seed(0)
    cases = [("L4 fwd", 0, 2048, 1024, 1024), ("L4 dgrad", 1, 2048, 1024, 1024),
             ("L4 wgrad", 2, 1024, 1024, 2048), ("L3 fwd", 0, 2048, 1024, 480),
             ("L5 fwd", 0, 2048, 512, 1024), ("L5 dgrad", 1, 2048, 1024, 512),
             ("L6 fwd", 0, 2048, 256, 512), ("L6 dgrad", 1, 2048, 512, 256)]
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    for name, lay, M, N, K in cases:
        A = torch.randn((K, M) if lay == 2 else (M, K), device=dev)
        B = torch.randn((N, K) if lay == 0 else (K, N), device=dev)
        opA = A.double().t() if lay == 2 else A.double()
        opB = B.double().t() if lay == 0 else B.double()
        ref = opA @ opB
        bound = opA.abs() @ opB.abs()
        Cf = torch.empty(M, N, device=dev)

        def f32():
            ops.gemm(A, B, trans_a=lay == 2, trans_b=lay == 0, C=Cf, workspace=ws)
        f32()
        tf = timeit(f32) * 1e6
        fl = 2 * M * N * K
        line = f"{name:9s} {M}x{N}x{K} prod {tf:6.1f} us ({fl / tf / 1e6:5.1f} TF)"
        for tile in (0, 1):
            for S in (3, 4, 13, 14):
                C = torch.full((M, N), float("nan"), device=dev)

                def go():
                    rc = lib.dlrm_dma_gemm(lay, tile, S, M, N, K, 1.0, P(A.data_ptr()),
                                           A.stride(0), P(B.data_ptr()), B.stride(0),
                                           P(C.data_ptr()), N, P(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0, lib.dlrm_last_error()
                go()
                torch.cuda.synchronize()
                err = float(((C.double() - ref).abs() / bound).max())
                t = timeit(go) * 1e6
                line += f" | {'64x64' if tile == 0 else '64x32'}{'P' if S > 9 else ''}S{S % 10} {t:6.1f} ({fl / t / 1e6:5.1f} TF, err {err:.0e})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
