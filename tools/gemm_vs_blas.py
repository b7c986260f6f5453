"""Per-shape GEMM table: this library's fp32 MFMA GEMM vs torch.matmul (hipBLASLt / rocBLAS,
fp32, no TF32) on the same box in the same process, for every GEMM of the DLRM step at a
batch size (C3: B = 2048; the W = 8 per-rank and B = 256 shapes: B = 256).

Each case is captured 50 times back to back into one hipGraph and replayed (5 replays, HIP
events), so neither side pays host launch overhead.  Ours runs as a single-problem launch
with the planner's tile / split for that shape (the step groups some of them); torch's
matmul has no fused epilogue (ours does: ReLU / ReLU' / SGD), so it does slightly less.

    python tools/gemm_vs_blas.py [B ...]      (default: 2048 256)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
PEAK = 157.3  # fp32 MFMA TFLOP/s (MI355X_MICROARCH.md)
LAYERS = [("bot", 13, 512), ("bot", 512, 256), ("bot", 256, 128), ("top", 479, 1024),
          ("top", 1024, 1024), ("top", 1024, 512), ("top", 512, 256)]


def pad4(n):
    return (n + 3) // 4 * 4


def graph_time(fn, reps=50, replays=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(replays):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e3  # us
        best = t if best is None else min(best, t)
    return best


def cases(B):
    dev = "cuda"
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    for li, (side, K, N) in enumerate(LAYERS):
        Kp = pad4(K + 1)
        X = torch.randn(B, Kp, device=dev).relu()
        W = torch.randn(N, Kp, device=dev) * 0.05
        Y = torch.empty(B, pad4(N + 1), device=dev)
        G = torch.randn(B, N, device=dev)
        dX = torch.empty(B, Kp, device=dev)
        Wt = W.clone()
        fl = 2 * B * N * K
        yield (f"L{li} {side} {K}->{N} fwd  [{B}x{N}x{Kp}]", fl,
               lambda X=X, W=W, Y=Y: ops.gemm(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU,
                                               workspace=ws),
               lambda X=X, W=W: torch.mm(X, W.t()))
        # the trainer's problems (trainer._dgrad / _wgrad): widths that are not a multiple
        # of 4 run over Kp; a wgrad with K % 4 == 0 takes the bias gradient as a row sum
        n = K if K % 4 == 0 else Kp
        if li != 0:  # the first bottom layer has no data gradient
            yield (f"L{li} {side} {K}->{N} dgrad [{B}x{n}x{N}]", fl,
                   lambda G=G, W=W, dX=dX, X=X, n=n: ops.gemm(G, W[:, :n], C=dX[:, :n],
                                                              epilogue=ops.EPI_DRELU,
                                                              aux=X[:, :n], workspace=ws),
                   lambda G=G, W=W, n=n: torch.mm(G, W[:, :n]))
        oc = K if K % 4 == 0 else -1
        # the step's wgrad (trainer._wg): split-K as PARTIAL slabs + the REDUCE job (with the
        # SGD epilogue) that rides on the next launch, timed here as two launches
        kw = dict(trans_a=True, C=Wt, alpha=1e-9, epilogue=ops.EPI_SGD, ones_col=oc)
        pr = ops.gemm_problem(G, X[:, :n], **kw)[0]
        s = ops.gemm_splits(pr, partial=True)
        if s > 1:
            part = torch.empty(ops.gemm_partial_bytes(N, n, s) // 4 + 1, device=dev)
            pp = ops.gemm_problem(G, X[:, :n], partial=part, splits=s, **kw)[0]
            rq = ops.reduce_problem(pp)

            def ours(pp=pp, rq=rq):
                ops.gemm_group([pp], ws)
                ops.gemm_group([rq], ws)
            tag = f"PARTIAL s{s} + REDUCE"
        else:
            def ours(pr=pr):
                ops.gemm_group([pr], ws)
            tag = "FULL"
        yield (f"L{li} {side} {K}->{N} wgrad [{N}x{n}x{B}] {tag}", fl, ours,
               lambda G=G, X=X, n=n: torch.mm(G.t(), X[:, :n]))


def main():
    blas_only = "--blas-only" in sys.argv  # (under rocprofv3: hipBLASLt's kernel names)
    Bs = [int(v) for v in sys.argv[1:] if not v.startswith("--")] or [2048, 256]
    out = {"peak_tflops": PEAK, "device": torch.cuda.get_device_name(), "batches": {}}
    for B in Bs:
        rows = []
        tot_o = tot_t = tot_f = 0.0
        for name, fl, ours, blas in cases(B):
            to = 1.0 if blas_only else graph_time(ours)
            tt = graph_time(blas)
            tot_o += to
            tot_t += tt
            tot_f += fl
            r = {"shape": name, "flop": fl, "ours_us": round(to, 2), "blas_us": round(tt, 2),
                 "ours_frac": round(fl / to / 1e6 / PEAK, 3),
                 "blas_frac": round(fl / tt / 1e6 / PEAK, 3),
                 "ours_over_blas_speed": round(tt / to, 3)}
            rows.append(r)
            print(f"B={B:5d} {name:58s} ours {to:7.1f} us ({r['ours_frac']:.3f})  "
                  f"hipBLASLt {tt:7.1f} us ({r['blas_frac']:.3f})  speed ratio "
                  f"{r['ours_over_blas_speed']:.2f}", flush=True)
        print(f"B={B:5d} TOTAL ours {tot_o:.1f} us ({tot_f / tot_o / 1e6 / PEAK:.3f})  "
              f"hipBLASLt {tot_t:.1f} us ({tot_f / tot_t / 1e6 / PEAK:.3f})", flush=True)
        out["batches"][str(B)] = {"rows": rows, "ours_us": round(tot_o, 1),
                                  "blas_us": round(tot_t, 1), "flop": tot_f}
    path = os.environ.get("GEMM_VS_BLAS_OUT")
    if path:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
