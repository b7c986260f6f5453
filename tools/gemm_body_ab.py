"""Per-GEMM A/B of the fp32 bodies on the C3 step's problems (the trainer's layouts,
epilogues and PARTIAL split wgrads): register-staged pipe_body (DLRM_GEMM_BODY=reg) vs the
LDS-DMA pipe_body_dma (default), under the plan table and under tile / split overrides.

    python tools/gemm_body_ab.py [--cfgs 64x32,64x64,32x64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dlrm-yx_amd"))
from dlrm_hip import ops  # noqa: E402
from gemm_sweep import LAYERS, pad4, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--cfgs", default="64x32,64x64,32x64")
    args = ap.parse_args()
    dev, B = "cuda", args.batch
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
            res = {}
            for body in ("reg", "dma"):
                os.environ["DLRM_GEMM_BODY"] = body
                os.environ.pop("DLRM_GEMM_CFG", None)
                pr = mk(0)
                s = ops.gemm_splits(pr, partial=True) if name == "wgrad" else 0
                pr = mk(s)
                res[f"{body}:plan"] = timeit(lambda: ops.gemm_group([pr], ws))
                for c in args.cfgs.split(","):
                    os.environ["DLRM_GEMM_CFG"] = c
                    for sp in ([1, 2, 4, 8] if name == "wgrad" else [1]):
                        os.environ["DLRM_GEMM_SPLIT"] = str(sp)
                        pr = mk(sp if name == "wgrad" else 0)
                        try:
                            res[f"{body}:{c}s{sp}"] = timeit(lambda: ops.gemm_group([pr], ws))
                        except Exception as e:  # noqa: BLE001
                            print("skip", body, c, sp, e)
                    os.environ.pop("DLRM_GEMM_SPLIT", None)
                os.environ.pop("DLRM_GEMM_CFG", None)
            for k, v in res.items():
                tot[k] = tot.get(k, 0.0) + v
            best = {b: min((v, k) for k, v in res.items() if k.startswith(b)) for b in ("reg", "dma")}
            for b in ("reg", "dma"):
                tot[f"{b}:best"] = tot.get(f"{b}:best", 0.0) + best[b][0]
            print(f"L{li} {name:5s} {2 * B * N * K / 1e9:5.2f} GF | reg plan {res['reg:plan'] * 1e6:6.1f} "
                  f"best {best['reg'][1]} {best['reg'][0] * 1e6:6.1f} | dma plan "
                  f"{res['dma:plan'] * 1e6:6.1f} best {best['dma'][1]} {best['dma'][0] * 1e6:6.1f} | "
                  + " ".join(f"{k}:{v * 1e6:.1f}" for k, v in res.items()), flush=True)
    os.environ.pop("DLRM_GEMM_BODY", None)
    print("TOTAL " + " ".join(f"{k}:{v * 1e6:.1f}" for k, v in tot.items()
                              if k.endswith("plan") or k.endswith("best")))


if __name__ == "__main__":
    main()
