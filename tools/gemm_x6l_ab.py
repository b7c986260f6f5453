"""A/B of the 128x128 split-bf16 GEMM body (DLRM_GEMM_MATH=x6l, gemm.hip pipe_body6L)
against the exact-f32 plan on the C3 step GEMMs.

1. Accuracy vs fp64 on every operand layout, ragged M/N/K, in-launch split-K, PARTIAL +
   REDUCE and the wgrad row sums: max |C - C64| / (sum_k |a||b|) for f32 and x6l.
2. Graph-timed us of every C3 GEMM (trainer problems): f32 plan vs x6l at split 1/2/4/8.

    python tools/gemm_x6l_ab.py [--batch 2048] [--skip-acc]
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
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    shapes = [(2048, 1024, 1024), (2048, 512, 480), (1024, 1024, 2048), (1000, 520, 200),
              (300, 900, 36)]
    print("accuracy (max err / sum|a||b|):", flush=True)
    worst = {"f32": 0.0, "x6l": 0.0}
    for (M, N, K) in shapes:
        for ta, tb in [(0, 1), (0, 0), (1, 0), (1, 1)]:
            A = torch.randn((K, M) if ta else (M, K), device=dev)
            B = torch.randn((N, K) if tb else (K, N), device=dev)
            opA = A.double().t() if ta else A.double()
            opB = B.double().t() if tb else B.double()
            ref = opA @ opB
            bound = opA.abs() @ opB.abs()
            line = f"  {M}x{N}x{K} ta{ta} tb{tb}:"
            for m in ("f32", "x6l"):
                set_math(m)
                C = ops.gemm(A, B, trans_a=bool(ta), trans_b=bool(tb), workspace=ws)
                torch.cuda.synchronize()
                e = float(((C.double() - ref).abs() / bound).max())
                worst[m] = max(worst[m], e)
                line += f"  {m}: {e:.2e}"
            print(line, flush=True)
    for mode in ("full", "partial"):
        M, K, N = 1024, 2048, 480
        G = torch.randn(K, M, device=dev)
        X = torch.randn(K, N + 4, device=dev)
        ref = G.double().t() @ X[:, :N].double()
        rs = G.double().sum(0)
        bound = G.double().abs().t() @ X[:, :N].double().abs()
        line = f"  wgrad+rowsum {mode} {M}x{N}x{K}:"
        for m in ("f32", "x6l"):
            set_math(m)
            C = torch.zeros(M, N + 4, device=dev)
            if mode == "full":
                pr, _ = ops.gemm_problem(G, X[:, :N], trans_a=True, C=C, ones_col=N)
                ops.gemm_group([pr], ws)
            else:
                pr0, _ = ops.gemm_problem(G, X[:, :N], trans_a=True, C=C, ones_col=N)
                s = ops.gemm_splits(pr0, partial=True)
                part = torch.empty(ops.gemm_partial_bytes(M, N, s) // 4, device=dev)
                pr, _ = ops.gemm_problem(G, X[:, :N], trans_a=True, C=C, ones_col=N,
                                         partial=part, splits=s)
                ops.gemm_group([pr], ws)
                ops.gemm_group([ops.reduce_problem(pr)], ws)
            torch.cuda.synchronize()
            e = float(((C[:, :N].double() - ref).abs() / bound).max())
            er = float((C[:, N].double() - rs).abs().max())
            worst[m] = max(worst[m], e)
            line += f"  {m}: {e:.2e} rowsum {er:.2e}"
        print(line, flush=True)
    print("worst", worst, flush=True)
    return worst


def timing(dev, B):
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
                partial=part if s > 0 else None, splits=s)[0]))
        for name, mk in cases:
            fl = 2 * B * N * K
            res = {}
            set_math("f32")
            pr = mk(0)
            res["f32"] = timeit(lambda: ops.gemm_group([pr], ws))
            set_math("x6l")
            for s in (0, 1, 2, 4, 8):
                if s:
                    os.environ["DLRM_GEMM_SPLIT"] = str(s)
                pr = mk(0)
                try:
                    res[f"x6l s{s or 'auto'}"] = timeit(lambda: ops.gemm_group([pr], ws))
                except Exception as e:  # noqa: BLE001
                    print("skip", s, e)
                os.environ.pop("DLRM_GEMM_SPLIT", None)
            best = min((v, k) for k, v in res.items() if k != "f32")
            tot["f32"] = tot.get("f32", 0.0) + res["f32"]
            tot["x6l_best"] = tot.get("x6l_best", 0.0) + min(best[0], res["f32"])
            print(f"L{li} {name:5s} {B}x{N}x{K} {fl / 1e9:5.2f} GF  f32 {res['f32'] * 1e6:6.1f} us "
                  f"({fl / res['f32'] / 1e12:5.1f} TF) | best {best[1]} {best[0] * 1e6:6.1f} us "
                  f"({fl / best[0] / 1e12:5.1f} TF-eq) | "
                  + " ".join(f"{k}:{v * 1e6:.1f}" for k, v in res.items() if k != "f32"),
                  flush=True)
    print("TOTAL " + " ".join(f"{k}:{v * 1e6:.1f}" for k, v in tot.items()), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--skip-acc", action="store_true")
    args = ap.parse_args()
    if not args.skip_acc:
        accuracy("cuda")
    timing("cuda", args.batch)
    os.environ.pop("DLRM_GEMM_MATH", None)


if __name__ == "__main__":
    main()
