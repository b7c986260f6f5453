"""Grouped vs separate launches for the C3 MLP-backward pairs [dgrad(l), wgrad(l+1)]
(new library, default plans).  Each variant is timed as 20 launches in a hipGraph."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


def pad4(n):
    return (n + 3) // 4 * 4


def main():
    dev = "cuda"
    B = int(os.environ.get("AB_BATCH", "2048"))
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    # (K, N) of top layers 0..3 and bottom 0..2
    top = [(479, 1024), (1024, 1024), (1024, 512), (512, 256)]
    bot = [(13, 512), (512, 256), (256, 128)]

    def mk(K, N):
        Kp = pad4(K + 1)
        return dict(K=K, N=N, Kp=Kp, W=torch.randn(N, Kp, device=dev),
                    act_in=torch.rand(B, Kp, device=dev), g=torch.randn(B, N, device=dev),
                    dx=torch.empty(B, Kp, device=dev))

    def dgrad(L):
        n = L["K"] if L["K"] % 4 == 0 else L["Kp"]
        return ops.gemm_problem(L["g"], L["W"][:, :n], C=L["dx"][:, :n], epilogue=ops.EPI_DRELU,
                                aux=L["act_in"])[0]

    def wgrad(L):
        if L["K"] % 4 == 0:
            return ops.gemm_problem(L["g"], L["act_in"][:, :L["K"]], trans_a=True, C=L["W"],
                                    alpha=1e-9, epilogue=ops.EPI_SGD, ones_col=L["K"])[0]
        return ops.gemm_problem(L["g"], L["act_in"][:, :L["Kp"]], trans_a=True, C=L["W"],
                                alpha=1e-9, epilogue=ops.EPI_SGD)[0]

    T = [mk(*s) for s in top]
    Bo = [mk(*s) for s in bot]
    pairs = [("top d2+w3", [dgrad(T[2]), wgrad(T[3])]), ("top d1+w2", [dgrad(T[1]), wgrad(T[2])]),
             ("top d0+w1", [dgrad(T[0]), wgrad(T[1])]), ("bot d2+topw0", [dgrad(Bo[2]), wgrad(T[0])]),
             ("bot d1+w2", [dgrad(Bo[1]), wgrad(Bo[2])]), ("bot w1+w0", [wgrad(Bo[1]), wgrad(Bo[0])]),
             ("top d3", [dgrad(T[3])])]
    for name, probs in pairs:
        tsep = [timeit(lambda p=p: ops.gemm_group([p], ws)) for p in probs]
        tgrp = timeit(lambda: ops.gemm_group(probs, ws))
        print(f"{name:14s} separate {' + '.join(f'{t:.1f}' for t in tsep)} = {sum(tsep):7.1f} us"
              f"   grouped {tgrp:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
