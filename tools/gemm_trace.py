"""Where a GEMM launch spends its time, per workgroup: the timeline build of the GEMM lab
(tools/_lab/libgemm_trace.so, `python tools/gemm_lab.py --build-trace`) stamps the shader
clock at the pipelined body's prologue, after every 32-deep K-tile and around the epilogue.
One launch per (shape, cfg) after a warm-up; prints the prologue, the steady K-tile, the
epilogue and the start / end spread over the workgroups (s_memrealtime, 100 MHz).

    python tools/gemm_trace.py [--cfgs 101,100,102] [--shapes fwd1,dgrad1,fwd0]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "dlrm-yx_amd"))
from dlrm_hip import ops, _lib  # noqa: E402


def pct(a, q):
    return float(np.percentile(a, q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="101,100,102")
    ap.add_argument("--shapes", default="fwd1,dgrad1,fwd0")
    args = ap.parse_args()
    lab = ctypes.CDLL(os.path.join(HERE, "_lab", "libgemm_trace.so"))
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    B = 2048
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    for shape in args.shapes.split(","):
        K = {"fwd1": 1028, "dgrad1": 1024, "fwd0": 480}[shape]
        X = torch.randn(B, K, device=dev)
        W = torch.randn(1024, K, device=dev)
        G = torch.randn(B, 1024, device=dev)
        Y = torch.zeros(B, 1028, device=dev)
        dX = torch.zeros(B, 1024, device=dev)
        if shape.startswith("fwd"):
            pr = ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0]
            flop = 2 * B * 1024 * K
        else:
            pr = ops.gemm_problem(G, W[:, :1024], C=dX, epilogue=ops.EPI_DRELU, aux=X)[0]
            flop = 2 * B * 1024 * 1024
        arr = (_lib.GemmProblem * 1)(pr)
        for cfg in [int(c) for c in args.cfgs.split(",")]:
            buf = torch.zeros(8192 * 72, dtype=torch.int64, device=dev)

            def run():
                assert lab.lab_gemm(cfg, 1, 1, arr, ctypes.c_void_p(ws.data_ptr()),
                                    ctypes.c_size_t(ws.numel()), st()) == 0
            lab.lab_set_stamps(ctypes.c_void_p(0))
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            lab.lab_set_stamps(ctypes.c_void_p(buf.data_ptr()))
            run()
            torch.cuda.synchronize()
            lab.lab_set_stamps(ctypes.c_void_p(0))
            s = buf.view(-1, 72).cpu().numpy()
            s = s[s[:, 0] != 0]
            nk = max(i for i in range(2, 68) if (s[:, i] != 0).all()) - 1
            pro = s[:, 1] - s[:, 0]
            tiles = np.diff(s[:, 1:2 + nk], axis=1)
            epi = s[:, 69] - s[:, 68]
            tot = s[:, 69] - s[:, 0]
            mid = tiles[:, 2:-2] if nk > 6 else tiles
            t0 = s[:, 70] - s[:, 70].min()
            t1 = s[:, 71] - s[:, 70].min()
            # s_memtime ticks per us from this launch: median total ticks / median realtime
            rt = (s[:, 71] - s[:, 70]) / 100.0  # us at 100 MHz
            tpu = float(np.median(tot / np.maximum(rt, 1e-3)))
            print(f"{shape} cfg {cfg}: {us:6.1f} us ({flop / us / 1e6:5.1f} TF), {len(s)} workgroups, "
                  f"{nk} K-tiles, clock {tpu:.0f} ticks/us", flush=True)
            print(f"   per workgroup (us, p10/p50/p90): prologue {pct(pro, 10) / tpu:5.2f} "
                  f"{pct(pro, 50) / tpu:5.2f} {pct(pro, 90) / tpu:5.2f} | K-tile (steady) "
                  f"{pct(mid, 10) / tpu:5.3f} {pct(mid, 50) / tpu:5.3f} {pct(mid, 90) / tpu:5.3f} | "
                  f"first K-tile {pct(tiles[:, 0], 50) / tpu:5.3f} | epilogue {pct(epi, 10) / tpu:5.2f} "
                  f"{pct(epi, 50) / tpu:5.2f} {pct(epi, 90) / tpu:5.2f} | total {pct(tot, 50) / tpu:5.1f}",
                  flush=True)
            print(f"   start spread (us): p50 {pct(t0, 50) / 100:5.2f} p90 {pct(t0, 90) / 100:5.2f} "
                  f"max {t0.max() / 100:5.2f} | end: p10 {pct(t1, 10) / 100:5.2f} p50 "
                  f"{pct(t1, 50) / 100:5.2f} max {t1.max() / 100:5.2f}", flush=True)


if __name__ == "__main__":
    main()
