"""Sweep tile (BMxBN) x K-split for every GEMM of the DLRM training step (the trainer's
problems: fwd FULL, dgrad FULL, wgrad PARTIAL with the bias as a row sum when K % 4 == 0)
at the given local batch sizes; prints per-shape results and writes the best plan per
shape as JSON (input for dlrm-yx_amd/csrc/gemm_plans.inc via tools/gen_gemm_plans.py).

    python tools/gemm_sweep.py [--batches 2048,256] [--out gpurun_out/gemm_plans.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402

CFGS = ["64x64", "32x64", "64x32", "128x64", "64x128", "32x32"]
LAYERS = {  # (K, N) of the C3 (terabyte) layers
    "terabyte": [(13, 512), (512, 256), (256, 128), (479, 1024), (1024, 1024), (1024, 512),
                 (512, 256)],
    # C2 (Criteo Kaggle): bot 13-512-256-64-16, top 367-512-256 (the 256 -> 1 head is not a GEMM)
    "kaggle": [(13, 512), (512, 256), (256, 64), (64, 16), (367, 512), (512, 256)],
}


def pad4(n):
    return (n + 3) // 4 * 4


def timeit(fn, n=20, reps=5):
    """Device time per call: n calls captured in one hipGraph (no host launch gaps)."""
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
    return s.elapsed_time(e) / (n * reps) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="2048")
    ap.add_argument("--layers", default="terabyte")
    ap.add_argument("--out", default="")
    ap.add_argument("--fwd-splits", action="store_true", help="also sweep K splits of fwd/dgrad")
    args = ap.parse_args()
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    plans = []
    tot_def, tot_best = 0.0, 0.0
    for B in [int(b) for b in args.batches.split(",")]:
        for li, (K, N) in enumerate(LAYERS[args.layers]):
            Kp = pad4(K + 1)
            X = torch.randn(B, Kp, device=dev)
            W = torch.randn(N, Kp, device=dev)
            Y = torch.empty(B, pad4(N + 1), device=dev)
            G = torch.randn(B, N, device=dev)
            dX = torch.empty(B, Kp, device=dev)
            nd = K if K % 4 == 0 else Kp
            part = torch.empty(ops.gemm_partial_bytes(N, Kp, 32) // 4 + 64, device=dev)
            cases = [("fwd", 0, B, N, Kp, [1, 2],
                      lambda s: ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0])]
            if li != 0:
                cases.append(("dgrad", 1, B, nd, N, [1, 2],
                              lambda s: ops.gemm_problem(G, W[:, :nd], C=dX[:, :nd],
                                                         epilogue=ops.EPI_DRELU, aux=X)[0]))
            if K % 4 == 0:
                wg = lambda s: ops.gemm_problem(G, X[:, :K], trans_a=True, C=W, alpha=1e-9,
                                                epilogue=ops.EPI_SGD, ones_col=K, partial=part,
                                                splits=s)[0]
                nw = K
            else:
                wg = lambda s: ops.gemm_problem(G, X, trans_a=True, C=W, alpha=1e-9,
                                                epilogue=ops.EPI_SGD, partial=part, splits=s)[0]
                nw = Kp
            cases.append(("wgrad", 2, N, nw, B, [1, 2, 3, 4, 6, 8, 12, 16], wg))
            if args.fwd_splits:  # latency-bound small batches: split the K of fwd / dgrad too
                cases = [(n_, l_, m_, nn_, kk_, sp_ if n_ == "wgrad" else [1, 2, 4, 8, 16], f_)
                         for n_, l_, m_, nn_, kk_, sp_, f_ in cases]
            for name, layout, M, Nn, KK, splits, mk in cases:
                t_def = timeit(lambda: ops.gemm_group([mk(0)], ws))
                res = []
                for cfg in CFGS:
                    bm_, bn_ = (int(v) for v in cfg.split("x"))
                    for s in splits:
                        pr = mk(s) if name == "wgrad" else mk(0)
                        try:
                            with ops.tuning(gemm_tile=bm_ * 1000 + bn_, gemm_split=s):
                                t = timeit(lambda: ops.gemm_group([pr], ws))
                        except Exception as e:  # noqa: BLE001
                            print("skip", name, cfg, s, e, flush=True)
                            continue
                        res.append((t, cfg, s))
                res.sort()
                t, cfg, s = res[0]
                bm, bn = (int(v) for v in cfg.split("x"))
                tot_def += t_def
                tot_best += t
                fl = 2 * B * N * K
                print(f"B{B} L{li} {name:5s} {M}x{Nn}x{KK}: default {t_def * 1e6:7.1f} us, best "
                      f"{t * 1e6:7.1f} us ({cfg} s{s}, {fl / t / 1e12:.1f} TF); "
                      + " ".join(f"{c}s{sp}:{tt * 1e6:.1f}" for tt, c, sp in res[:6]), flush=True)
                plans.append(dict(M=M, N=Nn, K=KK, layout=layout, bm=bm, bn=bn, split=s,
                                  us=round(t * 1e6, 1)))
    print(f"TOTAL default {tot_def * 1e6:.1f} us, best {tot_best * 1e6:.1f} us")
    if args.out:
        json.dump(plans, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
