"""One C3 GEMM shape three ways for a rocprofv3 --pmc pass (tools/pmc_sq_summary.py reads
the csv): the library's planned launch, lab configs (tools/gemm_lab.hip) and torch.mm
(hipBLASLt), 20 launches each, so their wait / MFMA-busy counters can be compared.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/gemm_pmc_probe.py [shape] [cfgs]
    shape: fwd1 (2048x1024x1028, default) | wgrad1 (1024x1024x2048)
"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "dlrm-yx_amd"))
from dlrm_hip import ops, _lib  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
shape = sys.argv[1] if len(sys.argv) > 1 else "fwd1"
cfgs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "100,101").split(",")]
dev = "cuda"
ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
B, K, N = 2048, 1024, 1024
X = torch.randn(B, K + 4, device=dev)
W = torch.randn(N, K + 4, device=dev)
G = torch.randn(B, N, device=dev)
Y = torch.zeros(B, N + 4, device=dev)
Wg = torch.zeros(N, K + 4, device=dev)
if shape == "fwd1":
    pr = ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0]
    blas = lambda: torch.mm(X, W.t())  # noqa: E731
else:
    pr = ops.gemm_problem(G, X[:, :K], trans_a=True, C=Wg, ones_col=K)[0]
    blas = lambda: torch.mm(G.t(), X[:, :K])  # noqa: E731
arr = (_lib.GemmProblem * 1)(pr)
lab = ctypes.CDLL(os.path.join(HERE, "_lab", "libgemm_lab.so"))
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(20):
    ops.gemm_group([pr], ws)
for c in cfgs:
    for _ in range(20):
        assert lab.lab_gemm(c, 1, 1, arr, ctypes.c_void_p(ws.data_ptr()),
                            ctypes.c_size_t(ws.numel()), st) == 0
for _ in range(20):
    blas()
torch.cuda.synchronize()
print("done", shape, cfgs)
