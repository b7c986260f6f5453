"""Time each trainer GEMM shape (tools/gemm_sweep.py's problems) under a list of tile
configs (ops.tuning gemm_tile overrides, with the plan table's split), graph-timed.

    python tools/gemm_cfg_ab.py [--batches 2048] [--cfgs 64x32,64x32x2x1,...]
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
    ap.add_argument("--batches", default="2048")
    ap.add_argument("--cfgs", default="64x32,64x32x2x1,32x64x1x2,128x32x4x1,64x64")
    args = ap.parse_args()
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    cfgs = args.cfgs.split(",")
    tot = {c: 0.0 for c in ["plan"] + cfgs}
    for B in [int(b) for b in args.batches.split(",")]:
        for li, (K, N) in enumerate(LAYERS["terabyte"]):
            Kp = pad4(K + 1)
            X = torch.randn(B, Kp, device=dev)
            W = torch.randn(N, Kp, device=dev)
            Y = torch.empty(B, pad4(N + 1), device=dev)
            G = torch.randn(B, N, device=dev)
            dX = torch.empty(B, Kp, device=dev)
            nd = K if K % 4 == 0 else Kp
            part = torch.empty(ops.gemm_partial_bytes(N, Kp, 32) // 4 + 64, device=dev)
            cases = [("fwd", lambda: ops.gemm_problem(X, W, trans_b=True, C=Y,
                                                      epilogue=ops.EPI_RELU)[0])]
            if li != 0:
                cases.append(("dgrad", lambda: ops.gemm_problem(G, W[:, :nd], C=dX[:, :nd],
                                                                epilogue=ops.EPI_DRELU,
                                                                aux=X)[0]))
            for name, mk in cases:
                res = []
                for c in ["plan"] + cfgs:
                    pr0 = mk()
                    s = ops.gemm_splits(pr0)
                    tile = 0 if c == "plan" else int(c.split("x")[0]) * 1000 + int(c.split("x")[1])
                    pr = mk()
                    with ops.tuning(gemm_tile=tile, gemm_split=s if tile else 0):
                        t = timeit(lambda: ops.gemm_group([pr], ws))
                    tot[c] += t
                    res.append(f"{c}:{t * 1e6:.1f}")
                fl = 2 * B * N * K
                print(f"B{B} L{li} {name:5s} {fl / 1e9:.2f} GF  " + "  ".join(res), flush=True)
    print("TOTAL " + "  ".join(f"{c}:{t * 1e6:.1f}" for c, t in tot.items()))


if __name__ == "__main__":
    main()
