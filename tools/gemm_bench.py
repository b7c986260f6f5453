"""Time every GEMM shape of the C3 training step (fwd, dgrad, wgrad) with HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402


def pad4(n):
    return (n + 3) // 4 * 4


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    layers = [(13, 512), (512, 256), (256, 128), (479, 1024), (1024, 1024), (1024, 512),
              (512, 256)]
    dev = "cuda"
    total_f, total_t = 0, 0.0
    rows = []
    for li, (K, N) in enumerate(layers):
        Kp = pad4(K + 1)
        X = torch.randn(B, Kp, device=dev)
        W = torch.randn(N, Kp, device=dev)
        Y = torch.empty(B, pad4(N + 1), device=dev)
        G = torch.randn(B, N, device=dev)
        dX = torch.empty(B, Kp, device=dev)
        cases = [("fwd", lambda: ops.gemm(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU),
                  2 * B * N * K)]
        if li not in (0,):
            cases.append(("dgrad", lambda: ops.gemm(G, W, C=dX, epilogue=ops.EPI_DRELU, aux=X),
                          2 * B * N * K))
        cases.append(("wgrad", lambda: ops.gemm(G, X, trans_a=True, C=W, alpha=1e-9,
                                                 epilogue=ops.EPI_SGD), 2 * B * N * K))
        for name, fn, fl in cases:
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            s.record()
            for _ in range(n):
                fn()
            e.record()
            torch.cuda.synchronize()
            t = s.elapsed_time(e) / n * 1e-3
            total_f += fl
            total_t += t
            rows.append(f"L{li} {K:5d}->{N:5d} {name:6s} {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF")
    for r in rows:
        print(r)
    print(f"TOTAL {total_t*1e6:.1f} us  {total_f/total_t/1e12:.1f} TF  ({total_f/1e9:.2f} GF)")


if __name__ == "__main__":
    main()
