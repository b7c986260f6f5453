"""Sweep tile (BMxBNxBK) x split-K for every GEMM of the DLRM step at the given local
batch sizes; prints per-shape results and writes the best plan per shape as JSON
(input for dlrm-yx_amd/csrc/gemm_plans.inc via tools/gen_gemm_plans.py).

    python tools/gemm_sweep.py [--batches 2048,1024,512,256] [--out gpurun_out/gemm_plans.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402

CFGS = ["64x64x32", "128x64x32", "64x128x32", "128x128x32", "64x64x64", "128x64x64",
        "64x128x64", "128x128x64", "64x64x32x2", "128x64x32x2", "64x128x32x2", "128x128x32x2",
        "64x64x64x2", "64x64x32x16", "128x64x32x16", "64x128x32x16", "128x128x32x16", "64x64x32x32", "128x64x32x32", "64x128x32x32"]
SPLITS = [1, 2, 3, 4, 6, 8, 12, 16]
# (K, N) of the C3 (terabyte) layers and the C1/C2 widths
LAYER_SETS = {
    "terabyte": [(13, 512), (512, 256), (256, 128), (479, 1024), (1024, 1024), (1024, 512),
                 (512, 256)],
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
    args = ap.parse_args()
    dev = "cuda"
    plans = []
    grand_default, grand_best = 0.0, 0.0
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    for B in [int(b) for b in args.batches.split(",")]:
        tot_default, tot_best = 0.0, 0.0
        for li, (K, N) in enumerate(LAYER_SETS[args.layers]):
            Kp = pad4(K + 1)
            X = torch.randn(B, Kp, device=dev)
            W = torch.randn(N, Kp, device=dev)
            Y = torch.empty(B, pad4(N + 1), device=dev)
            G = torch.randn(B, N, device=dev)
            dX = torch.empty(B, Kp, device=dev)
            # (name, fn, M, N, K, ta, tb) with the trainer's exact operand shapes
            cases = [("fwd", lambda: ops.gemm(X, W, trans_b=True, C=Y[:, :N],
                                              epilogue=ops.EPI_RELU, workspace=ws),
                      B, N, Kp, 0, 1)]
            blas = {"fwd": lambda: torch.matmul(X, W.t(), out=Yb),
                    "dgrad": lambda: torch.matmul(G, W[:, :K], out=dXb),
                    "wgrad": lambda: torch.matmul(G.t(), X, out=Wb)}
            Yb = torch.empty(B, N, device=dev)
            dXb = torch.empty(B, K, device=dev)
            Wb = torch.empty(N, Kp, device=dev)
            if li != 0:
                cases.append(("dgrad", lambda: ops.gemm(G, W[:, :K], C=dX[:, :K],
                                                        epilogue=ops.EPI_DRELU, aux=X,
                                                        workspace=ws),
                              B, K, N, 0, 0))
            cases.append(("wgrad", lambda: ops.gemm(G, X, trans_a=True, C=W, alpha=1e-9,
                                                    epilogue=ops.EPI_SGD, workspace=ws),
                          N, Kp, B, 1, 0))
            fl = 2 * B * N * K
            for name, fn, M_, N_, K_, ta, tb in cases:
                os.environ.pop("DLRM_GEMM_CFG", None)
                os.environ.pop("DLRM_GEMM_SPLIT", None)
                t0 = timeit(fn)
                tb_ = timeit(blas[name])
                res = []
                for cfg in CFGS:
                    for s in SPLITS:
                        if s > 1 and K_ // s < 128:
                            continue
                        os.environ["DLRM_GEMM_CFG"] = cfg
                        os.environ["DLRM_GEMM_SPLIT"] = str(s)
                        res.append((timeit(fn), cfg, s))
                res.sort()
                os.environ.pop("DLRM_GEMM_CFG", None)
                os.environ.pop("DLRM_GEMM_SPLIT", None)
                tot_best += res[0][0]
                tot_default += t0
                parts = [int(v) for v in res[0][1].split("x")]
                bm, bn, bk = parts[:3]
                ks = parts[3] if len(parts) > 3 else 1
                plans.append({"M": M_, "N": N_, "K": K_, "trans_a": ta, "trans_b": tb,
                              "bm": bm, "bn": bn, "bk": bk, "ks": ks, "split": res[0][2],
                              "us": round(res[0][0] * 1e6, 2)})
                top = " ".join(f"{c}/{s}:{tt * 1e6:.1f}" for tt, c, s in res[:4])
                print(f"B{B} L{li} {K:5d}->{N:5d} {name:6s} blas {tb_ * 1e6:6.1f}us "
                      f"default {t0 * 1e6:7.1f}us "
                      f"({fl / t0 / 1e12:5.1f}TF) best {res[0][0] * 1e6:7.1f}us "
                      f"({fl / res[0][0] / 1e12:5.1f}TF) | {top}", flush=True)
        print(f"B{B} TOTAL default {tot_default * 1e6:.1f}us best {tot_best * 1e6:.1f}us",
              flush=True)
        grand_default += tot_default
        grand_best += tot_best
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(plans, f, indent=0)


if __name__ == "__main__":
    main()
