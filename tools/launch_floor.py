"""Per-kernel cost floor on the device: N back-to-back tiny launches (eager and in a
hipGraph), and launches that dirty a few MB each (kernel-boundary cache writeback).

    python tools/launch_floor.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dlrm-yx_amd"))

import torch  # noqa: E402

from dlrm_hip import ops  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    N = 100
    for nel in (256, 1 << 18, 1 << 21):
        x = torch.ones(nel, device=dev)

        def burst():
            for _ in range(N):
                ops.scale_(x, 1.0)

        t_eager = timed(burst) * 1000 / N
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            burst()
        t_graph = timed(g.replay) * 1000 / N
        print(f"scale_ {nel * 4 / 1e6:8.3f} MB  eager {t_eager:6.2f} us/launch  "
              f"graph {t_graph:6.2f} us/launch", flush=True)
    # a GEMM of the step in isolation vs back-to-back
    A = torch.randn(2048, 1028, device=dev)
    W = torch.randn(1024, 1028, device=dev)
    C = torch.empty(2048, 1024, device=dev)
    ws = torch.zeros(ops.gemm_workspace_size(2048, 1024, 1028, False, True) + 256,
                     dtype=torch.uint8, device=dev)

    def gemms():
        for _ in range(10):
            ops.gemm(A, W, trans_b=True, C=C, workspace=ws)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gemms()
    t = timed(g.replay) * 1000 / 10
    print(f"gemm 2048x1024x1028 fwd: {t:.2f} us  ({2 * 2048 * 1024 * 1028 / t / 1e6:.1f} TF)")
    C2 = torch.empty(2048, 1024, device=dev)
    t0 = time.perf_counter()
    r = torch.matmul(A, W.t(), out=C2)
    torch.cuda.synchronize()

    def blas():
        for _ in range(10):
            torch.matmul(A, W.t(), out=C2)

    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        blas()
    t = timed(g2.replay) * 1000 / 10
    print(f"hipBLASLt 2048x1024x1028 fwd: {t:.2f} us ({2 * 2048 * 1024 * 1028 / t / 1e6:.1f} TF)")
    del r, t0


if __name__ == "__main__":
    main()
