"""Calibrate the CPU baseline: time the REFERENCE's own DLRM_Net training
step (dlrm_s_pytorch.py: forward, loss_fn, zero_grad, backward, torch.optim.SGD.step) and
the oracle restatement bench.py times on the GPU box (oracle.OracleDLRM.train_step), on
the same cores, shapes and batches.  The two must agree within +-10 %.

Build container only (imports /root/reference through tests/golden/make_golden.py's
shims).  Writes profiles/<tag>_cpu_calibration.json.

    python tools/cpu_calibrate.py [--tag r03] [--seconds 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]


def batches(c, rows, n=4):
    import torch
    rng = np.random.RandomState(1)
    B, L = c["B"], c["L"]
    out = []
    for _ in range(n):
        X = torch.log1p(torch.tensor(rng.rand(B, c["bot"][0]).astype(np.float32)))
        lS_o = torch.arange(B).mul(L).repeat(len(rows), 1)
        lS_i = [torch.tensor(rng.randint(0, r, size=B * L)) for r in rows]
        T = torch.tensor(np.round(rng.rand(B, 1)).astype(np.float32))
        out.append((X, lS_o, lS_i, T))
    return out


def timed(step, bs, seconds):
    for i in range(2):
        step(*bs[i % len(bs)])
    ts = []
    t0 = time.perf_counter()
    while True:
        a = time.perf_counter()
        step(*bs[len(ts) % len(bs)])
        ts.append(time.perf_counter() - a)
        if time.perf_counter() - t0 >= seconds and len(ts) >= 5:
            break
    ts = np.array(ts) * 1e3
    return {"mean_ms": round(float(ts.mean()), 2), "median_ms": round(float(np.median(ts)), 2),
            "best_ms": round(float(ts.min()), 2), "steps": len(ts)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r03")
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--configs", default="terabyte,small,kaggle")
    args = ap.parse_args()
    from make_golden import import_reference
    R = import_reference("/root/reference")
    import torch
    import bench
    import oracle as O
    cores = sorted(os.sched_getaffinity(0))
    torch.set_num_threads(len(cores))
    res = {"cores": len(cores), "cpu_model": bench.cpu_model(), "torch_threads": len(cores),
           "what": "reference DLRM_Net step (torch.optim.SGD) vs oracle.OracleDLRM.train_step, "
                   "same shapes / batches / cores; tables capped at 1e6 rows", "configs": {}}
    for name in args.configs.split(","):
        c = dict(bench.CONFIGS[name])
        rows = [min(r, 1_000_000) for r in c["rows"]]
        D = c["D"]
        ln_top = [bench.num_int(len(rows), D)] + c["top"]
        bs = batches(c, rows)
        lr = c["lr"] * 0.01
        R.ext_dist.my_size = -1
        np.random.seed(0)
        net = R.ref.DLRM_Net(D, np.array(rows), np.array(c["bot"]), np.array(ln_top),
                             arch_interaction_op="dot", sigmoid_top=len(ln_top) - 2,
                             loss_function=c["loss"])
        opt = torch.optim.SGD(net.parameters(), lr=lr)

        def ref_step(X, lS_o, lS_i, T):
            Z = net(X, lS_o, lS_i)
            E = net.loss_fn(Z, T)
            opt.zero_grad()
            E.backward()
            opt.step()

        m = O.OracleDLRM(D, rows, c["bot"], ln_top, loss_function=c["loss"],
                         tables=[e.weight.detach().numpy() for e in net.emb_l])
        r_ref = timed(ref_step, bs, args.seconds)
        r_orc = timed(lambda X, o, i, T: m.train_step(X, o, i, T, lr), bs, args.seconds)
        ratio = r_orc["median_ms"] / r_ref["median_ms"]
        res["configs"][name] = {"reference": r_ref, "oracle": r_orc,
                                "oracle_over_reference_median": round(ratio, 3),
                                "within_10pct": abs(ratio - 1.0) <= 0.10}
        print(name, json.dumps(res["configs"][name]), flush=True)
        del net, m, opt
    out = os.path.join(ROOT, "profiles", f"{args.tag}_cpu_calibration.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
