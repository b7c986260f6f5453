"""A/B of the pre-split x6 prototype (csrc/gemm6p.hip): fp32 GEMMs of the C3 step on the
bf16 matrix core from bf16 (h, m, l) planes, vs the exact-f32 MFMA body (ops.gemm) on the
same operands.  Accuracy against fp64; graph-timed us per GEMM; split cost separately.

    python tools/x6p_probe.py
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
# the prototype library (make -C tools/proto): its own copy of the error plumbing
lib = ctypes.CDLL(os.path.join(HERE, "proto", "libdlrm_x6p.so"))
lib.dlrm_last_error.restype = ctypes.c_char_p
lib.dlrm_x6_split_planes.restype = ctypes.c_int32
lib.dlrm_x6_split_planes.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P,
                                     ctypes.c_int64, ctypes.c_int64, P]
lib.dlrm_x6p_gemm.restype = ctypes.c_int32
lib.dlrm_x6p_gemm.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_float, P, ctypes.c_int64, ctypes.c_int64,
                              P, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int64, P]


def stream():
    return P(torch.cuda.current_stream().cuda_stream)


def planes_of(X):
    r, c = X.shape
    ldp = (c + 7) // 8 * 8
    Pl = torch.empty(3 * r * ldp, dtype=torch.bfloat16, device=X.device)
    rc = lib.dlrm_x6_split_planes(P(X.data_ptr()), r, c, X.stride(0), P(Pl.data_ptr()), ldp,
                                  r * ldp, stream())
    assert rc == 0, lib.dlrm_last_error()
    return Pl, ldp, r * ldp


TILES = (0, 2, 3, 4, 5)
TNAME = {0: "x6p64x64", 2: "x6p128x64", 3: "dma128x64s4", 4: "dma64x64s4", 5: "dma64x64s3"}


def main():
    dev = "cuda"
    torch.manual_seed(0)
    # (name, layout, M, N, K): layout 0 fwd (A [M][K], B [N][K]); 1 dgrad (A [M][K],
    # B stored [K][N]); 2 wgrad (A stored [K][M], B stored [K][N])
    cases = [("L4 fwd", 0, 2048, 1024, 1024), ("L4 dgrad", 1, 2048, 1024, 1024),
             ("L4 wgrad", 2, 1024, 1024, 2048), ("L3 fwd", 0, 2048, 1024, 480),
             ("L5 fwd", 0, 2048, 512, 1024), ("L5 dgrad", 1, 2048, 1024, 512),
             ("L5 wgrad", 2, 512, 1024, 2048), ("L6 fwd", 0, 2048, 256, 512)]
    for name, lay, M, N, K in cases:
        A = torch.randn((K, M) if lay == 2 else (M, K), device=dev)
        B = torch.randn((N, K) if lay == 0 else (K, N), device=dev)
        opA = A.double().t() if lay == 2 else A.double()
        opB = B.double().t() if lay == 0 else B.double()
        ref = opA @ opB
        bound = opA.abs() @ opB.abs()
        Ap, lda, psa = planes_of(A)
        Bp, ldb, psb = planes_of(B)
        split_us = timeit(lambda: (planes_of(A), planes_of(B)), n=10) * 1e6
        res = {}
        for tile in TILES:
            C = torch.empty(M, N, device=dev)

            def go():
                rc = lib.dlrm_x6p_gemm(lay, tile, M, N, K, 1.0, P(Ap.data_ptr()), lda, psa,
                                       P(Bp.data_ptr()), ldb, psb, P(C.data_ptr()), N, stream())
                assert rc == 0, lib.dlrm_last_error()
            go()
            torch.cuda.synchronize()
            err = float(((C.double() - ref).abs() / bound).max())
            res[TNAME[tile]] = (timeit(go) * 1e6, err)
        Cf = torch.empty(M, N, device=dev)
        ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)

        def f32():
            ops.gemm(A, B, trans_a=lay == 2, trans_b=lay == 0, C=Cf, workspace=ws)
        f32()
        torch.cuda.synchronize()
        errf = float(((Cf.double() - ref).abs() / bound).max())
        tf = timeit(f32) * 1e6
        fl = 2 * M * N * K
        line = f"{name:9s} {M}x{N}x{K} f32 {tf:6.1f} us ({fl / tf / 1e6:5.1f} TF, err {errf:.1e})"
        for k, (t, e) in res.items():
            line += f" | {k} {t:6.1f} us ({fl / t / 1e6:5.1f} TF-eq, err {e:.1e})"
        line += f" | split A+B {split_us:5.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
