"""A/B of the GEMM math: exact-f32 MFMA vs the split-bf16 body (DLRM_GEMM_MATH=x6).

1. Accuracy on every operand layout (fwd / dgrad / wgrad with row sums / trans-trans) and
   split-K: max |C - C_fp64| / (sum_k |a||b|) and the max error against 1e-5 * max(1, |ref|).
2. Time of every GEMM of the C3 training step (the trainer's problems, graph-timed), f32 vs
   x6 under the plan table, and x6 under a few tile / split overrides.

    python tools/gemm_x6_ab.py [--batch 2048] [--cfgs 64x64,64x32,32x64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import LAYERS, pad4, timeit  # noqa: E402


def set_math(m):
    os.environ["DLRM_GEMM_MATH"] = m


def accuracy(dev):
    torch.manual_seed(0)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    shapes = [(2048, 1024, 1024), (2048, 512, 480), (1024, 1024, 2048), (200, 72, 36),
              (64, 32, 4096)]
    print("accuracy (err / sum|a||b|, max err / max(1,|ref|)):")
    for (M, N, K) in shapes:
        for ta, tb in [(0, 1), (0, 0), (1, 0), (1, 1)]:
            A = torch.randn((K, M) if ta else (M, K), device=dev)
            B = torch.randn((N, K) if tb else (K, N), device=dev)
            A64, B64 = A.double(), B.double()
            opA = A64.t() if ta else A64
            opB = B64.t() if tb else B64
            ref = opA @ opB
            bound = opA.abs() @ opB.abs()
            line = f"  {M}x{N}x{K} ta{ta} tb{tb}:"
            for m in ("f32", "x6"):
                set_math(m)
                C = ops.gemm(A, B, trans_a=bool(ta), trans_b=bool(tb), workspace=ws)
                torch.cuda.synchronize()
                e = (C.double() - ref).abs()
                line += (f"  {m}: {float((e / bound).max()):.2e} "
                         f"{float((e / ref.abs().clamp(min=1)).max()):.2e}")
            print(line, flush=True)
    # wgrad with the row sum (ones_col) through the split path
    M, K, N = 1024, 2048, 480
    G = torch.randn(K, M, device=dev)
    X = torch.randn(K, N + 4, device=dev)
    ref = G.double().t() @ X[:, :N].double()
    rs = G.double().sum(0)
    line = f"  wgrad+rowsum {M}x{N}x{K}:"
    for m in ("f32", "x6"):
        set_math(m)
        C = torch.zeros(M, N + 4, device=dev)
        pr, _ =ops.gemm_problem(G, X[:, :N], trans_a=True, C=C, ones_col=N)
        ops.gemm_group([pr], ws)
        torch.cuda.synchronize()
        e = float((C[:, :N].double() - ref).abs().max())
        er = float((C[:, N].double() - rs).abs().max())
        line += f"  {m}: max|dC| {e:.2e} max|drowsum| {er:.2e}"
    print(line, flush=True)


def timing(dev, B, cfgs, maths=("x6",)):
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    tot = {}
    for li, (K, N) in enumerate(LAYERS["terabyte"]):
        Kp = pad4(K + 1)
        X = torch.randn(B, Kp, device=dev)
        W = torch.randn(N, Kp, device=dev) * 0.01
        Y = torch.empty(B, pad4(N + 1), device=dev)
        G = torch.randn(B, N, device=dev)
        dX = torch.empty(B, Kp, device=dev)
        nd = K if K % 4 == 0 else Kp
        part = torch.empty(ops.gemm_partial_bytes(N, Kp, 32) // 4 + 64, device=dev)
        cases = [("fwd", lambda s: ops.gemm_problem(X, W, trans_b=True, C=Y,
                                                    epilogue=ops.EPI_RELU)[0])]
        if li != 0:
            cases.append(("dgrad", lambda s: ops.gemm_problem(G, W[:, :nd], C=dX[:, :nd],
                                                              epilogue=ops.EPI_DRELU, aux=X)[0]))
        if K % 4 == 0:
            cases.append(("wgrad", lambda s: ops.gemm_problem(
                G, X[:, :K], trans_a=True, C=W, alpha=1e-9, epilogue=ops.EPI_SGD, ones_col=K,
                partial=part, splits=s)[0]))
        for name, mk in cases:
            fl = 2 * B * N * K
            res = {}
            for m in ("f32", "x6"):
                set_math(m)
                os.environ.pop("DLRM_GEMM_CFG", None)
                pr = mk(0)
                s = ops.gemm_splits(pr, partial=name == "wgrad") if name == "wgrad" else 0
                pr = mk(s)
                res[m] = timeit(lambda: ops.gemm_group([pr], ws))
            for math in maths:
                set_math(math)
                for c in cfgs:
                    os.environ["DLRM_GEMM_CFG"] = c
                    for s in ([1, 2, 4, 8] if name == "wgrad" else [1, 2]):
                        os.environ["DLRM_GEMM_SPLIT"] = str(s)
                        pr = mk(s)
                        try:
                            res[f"{math}:{c}s{s}"] = timeit(lambda: ops.gemm_group([pr], ws))
                        except Exception as e:  # noqa: BLE001
                            print("skip", c, s, e)
                    os.environ.pop("DLRM_GEMM_SPLIT", None)
            os.environ.pop("DLRM_GEMM_CFG", None)
            best = min((v, k) for k, v in res.items() if k.startswith("x6") or ":" in k)
            for k, v in res.items():
                tot[k] = tot.get(k, 0.0) + v
            tot["x6best"] = tot.get("x6best", 0.0) + best[0]
            print(f"L{li} {name:5s} {fl / 1e9:5.2f} GF  f32 {res['f32'] * 1e6:6.1f} us "
                  f"({fl / res['f32'] / 1e12:5.1f} TF)  x6 {res['x6'] * 1e6:6.1f} us "
                  f"({fl / res['x6'] / 1e12:5.1f} TF)  best x6 {best[1]} {best[0] * 1e6:6.1f} us  | "
                  + " ".join(f"{k}:{v * 1e6:.1f}" for k, v in res.items()
                             if ":" in k), flush=True)
    print("TOTAL " + " ".join(f"{k}:{v * 1e6:.1f}" for k, v in tot.items()
                              if ":" not in k))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--cfgs", default="64x64,64x32,32x64")
    ap.add_argument("--skip-acc", action="store_true")
    ap.add_argument("--maths", default="x6")
    args = ap.parse_args()
    dev = "cuda"
    if not args.skip_acc:
        accuracy(dev)
    timing(dev, args.batch, args.cfgs.split(","), args.maths.split(","))
    os.environ.pop("DLRM_GEMM_MATH", None)


if __name__ == "__main__":
    main()
