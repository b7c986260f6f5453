"""Step time vs position in a long run (is the short driver run slower because the chip
ramps its clocks?): the bench's C3 step graphs replayed N times with an event per step,
mean per window of 50 steps; optionally after a pre-heat of PRE ms of a 4096^3 GEMM.

    python tools/ramp_probe.py [--steps 1500] [--preheat-ms 0]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dlrm-yx_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--preheat-ms", type=float, default=0.0)
    ap.add_argument("--win", type=int, default=50)
    args = ap.parse_args()
    from dlrm_hip import ops
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    dev = torch.device("cuda", 0)
    c = bench.CONFIGS["terabyte"]
    ln_top = [bench.num_int(26, c["D"])] + c["top"]
    cfg = TrainerConfig(m_spa=c["D"], ln_emb=c["rows"], ln_bot=c["bot"], ln_top=ln_top,
                        loss_function=c["loss"], learning_rate=c["lr"], sharder="greedy")
    tr = DLRMTrainer(cfg, device=dev, seed=1)
    batches = [tr.synthetic_batch(2048, 1, seed=100 + i) for i in range(10)]
    for b in batches[:3]:
        tr.step(b)
    torch.cuda.synchronize()
    pool = torch.cuda.graph_pool_handle()
    graphs = [tr.capture(b, pool=pool) for b in batches]
    for g in graphs:
        g()
    torch.cuda.synchronize()
    time.sleep(1.0)  # let the chip idle down first
    if args.preheat_ms > 0:
        n = 4096
        A = torch.randn(n, n, device=dev)
        C = torch.empty(n, n, device=dev)
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < args.preheat_ms:
            ops.gemm(A, A, C=C)
            torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    evs[0].record()
    for k in range(args.steps):
        graphs[k % 10]()
        evs[k + 1].record()
    torch.cuda.synchronize()
    ts = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
    out = []
    for w in range(0, args.steps, args.win):
        seg = ts[w:w + args.win]
        out.append(f"{w}:{sum(seg) / len(seg) * 1e3:.1f}")
    print(f"preheat {args.preheat_ms} ms; us/step per {args.win}-step window:", " ".join(out),
          flush=True)


if __name__ == "__main__":
    main()
