"""Production x6d body vs the r03 prototype DMA kernel (tools/proto, tile 3) on identical planes:
separates kernel differences from operand pitch effects (K = 1024 vs 1028 -> plane pitch
1024 vs 1032)."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "dlrm-yx_amd")]
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import timeit  # noqa: E402

P = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "proto", "libdlrm_x6p.so"))
lib.dlrm_x6p_gemm.restype = ctypes.c_int32
lib.dlrm_x6p_gemm.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_float, P, ctypes.c_int64, ctypes.c_int64,
                              P, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int64, P]
dev = "cuda"
ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
for (M, N, K, ldk) in [(2048, 1024, 1024, 1024), (2048, 1024, 1024, 1032), (2048, 1024, 1032, 1032),
                       (2048, 1024, 480, 480), (2048, 256, 512, 512), (2048, 256, 512, 520)]:
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    AP = torch.zeros(3, M, ldk, dtype=torch.bfloat16, device=dev)
    BP = torch.zeros(3, N, ldk, dtype=torch.bfloat16, device=dev)
    ops.split_planes(A, out=AP)
    ops.split_planes(B, out=BP)
    C = torch.empty(M, N, device=dev)
    st = lambda: P(torch.cuda.current_stream().cuda_stream)

    def proto():
        lib.dlrm_x6p_gemm(0, 3, M, N, K, 1.0, P(AP.data_ptr()), ldk, M * ldk, P(BP.data_ptr()), ldk,
                          N * ldk, P(C.data_ptr()), N, st())
    pr = ops.gemm_problem(A, B, trans_b=True, C=C, a_planes=AP, b_planes=BP)[0]
    tp = timeit(proto) * 1e6
    tx = timeit(lambda: ops.gemm_group([pr], ws)) * 1e6
    print(f"{M}x{N}x{K} ld {ldk}: proto dma128x64 {tp:6.1f} us  production x6d {tx:6.1f} us",
          flush=True)
