"""C4 bench config on the engine (full Terabyte tables, B = 2048, QR + RWSAdagrad): loss of
the first N steps at a few learning rates, from the bench's own init and synthetic batches.

    python tools/c4_trajectory.py [--steps 60]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dlrm-yx_amd")]
import bench  # noqa: E402
from dlrm_hip.trainer import DLRMTrainer, TrainerConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--lrs", default="0.001,0.0001")
    ap.add_argument("--seeds", default="1", help="trainer init seeds (bench: 1)")
    args = ap.parse_args()
    c = bench.CONFIGS["terabyte_qr_rwsadagrad"]
    ln_top = [bench.num_int(len(c["rows"]), c["D"])] + c["top"]
    runs = [(float(lr), int(sd)) for lr in args.lrs.split(",") for sd in args.seeds.split(",")]
    for lr, seed in runs:
        qr = c["qr"]
        cfg = TrainerConfig(m_spa=c["D"], ln_emb=c["rows"], ln_bot=c["bot"], ln_top=ln_top,
                            loss_function="bce", learning_rate=lr, optimizer="rwsadagrad",
                            qr_flag=True, qr_collisions=qr["collisions"],
                            qr_operation=qr["operation"], qr_threshold=qr["threshold"])
        tr = DLRMTrainer(cfg, device="cuda", seed=seed)
        batches = [tr.synthetic_batch(c["B"], 1, seed=100 + s) for s in range(10)]  # as bench
        out = []
        for s in range(args.steps):
            _, E = tr.step(batches[s % 10])
            out.append(round(E.item(), 3))
        print("lr", lr, "seed", seed, out, flush=True)
        del tr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
