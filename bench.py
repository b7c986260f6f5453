#!/usr/bin/env python3
"""DLRM training-step throughput on MI355X (samples/s, fwd + loss + bwd + update).

Workload (BASELINE.json configs[3], the metric's headline config): MLPerf Terabyte-shaped
synthetic DLRM — 26 tables with the terabyte row counts hashed to 1e7 (54,063,992 rows,
27.7 GB fp32 resident in HBM), D=128, bottom 13-512-256-128, top 479-1024-1024-512-256-1,
dot interaction, BCE, SGD lr 1.0, global batch 2048 (strong scaling over ranks, the
reference methodology of bench/dlrm_s_benchmark.sh), one lookup per bag (Criteo one-hot).

    python bench.py [--gpus N --steps K --warmup W]      # N>1 via torch.distributed.run

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dlrm-yx_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "DLRM samples/sec fwd+bwd at 1/2/4/8 MI355X; embedding HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: fp32 matrix peak (= vector peak)

TERABYTE_ROWS = [10000000, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 10000000, 2953546,
                 403346, 10, 2208, 11938, 155, 4, 976, 14, 10000000, 10000000, 10000000, 585935,
                 12972, 108, 36]
KAGGLE_ROWS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194,
               27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]

CONFIGS = {
    "terabyte": dict(workload="mlperf_terabyte_synthetic", rows=TERABYTE_ROWS, D=128,
                     bot=[13, 512, 256, 128], top=[1024, 1024, 512, 256, 1], B=2048, L=1,
                     loss="bce", lr=1.0, optimizer="sgd"),
    # C4: --qr-flag --qr-collisions=4 --qr-operation=mult --qr-threshold=200
    # --optimizer=rwsadagrad
    "terabyte_qr_rwsadagrad": dict(workload="mlperf_terabyte_synthetic+qr+rwsadagrad",
                                   rows=TERABYTE_ROWS, D=128, bot=[13, 512, 256, 128],
                                   top=[1024, 1024, 512, 256, 1], B=2048, L=1, loss="bce",
                                   lr=1.0, optimizer="rwsadagrad",
                                   qr=dict(collisions=4, operation="mult", threshold=200)),
    "small": dict(workload="synthetic_small", rows=[100000] * 8, D=64, bot=[512, 512, 64],
                  top=[1024, 1024, 1024, 1], B=2048, L=100, loss="mse", lr=0.1, optimizer="sgd"),
    "kaggle": dict(workload="criteo_kaggle_synthetic", rows=KAGGLE_ROWS, D=16,
                   bot=[13, 512, 256, 64, 16], top=[512, 256, 1], B=128, L=1, loss="bce", lr=0.1,
                   optimizer="sgd"),
}


def num_int(T, D):
    F = T + 1
    return D + F * (F - 1) // 2


def algorithmic_work(c, B_local, B_global, T_local, world, bottom_fused=False):
    """Per-step algorithmic FLOPs of the GEMM launches and bytes of the TBE kernels
    (SURVEY.md §8d formulas).  bottom_fused: the bottom MLP forward
    ran inside the lookup launch, so its FLOPs are not GEMM-launch work."""
    D, L, T = c["D"], c["L"], len(c["rows"])
    bot = c["bot"]
    top = [num_int(T, D)] + c["top"]
    layers = [(bot[i], bot[i + 1]) for i in range(len(bot) - 1)] + \
             [(top[i], top[i + 1]) for i in range(len(top) - 2)]  # head (K->1) is not a GEMM
    fl = 0
    for li, (k, n) in enumerate(layers):
        if not (bottom_fused and li < len(bot) - 1):
            fl += 2 * B_local * n * k      # forward
        fl += 2 * B_local * n * k          # wgrad
        if li != 0:
            fl += 2 * B_local * n * k      # dgrad (no dgrad for the bottom input layer)
    # top first layer dgrad (into the interaction) is included (li != 0 for it)
    s_idx = 4
    lookups = T_local * B_global * L
    fwd_bytes = lookups * (4 * D + s_idx) + 4 * (T_local * B_global + 1) + 4 * T_local * B_global * D
    bwd_bytes = 4 * T_local * B_global * D + lookups * (s_idx + 8 * D)
    return fl, fwd_bytes, bwd_bytes


class GroupGraphTimer:
    """Per-kernel-group device time of one step.  Passed as the trainer's ``profile`` hook:
    every launch inside a named scope ("gemm", "tbe_fwd", ...) goes to that name's own
    stream, which is capturing a hipGraph; after the steps each name's graph holds exactly
    that group's launches of the steps, in order, and is timed on its own with HIP events
    (on the stream it replays on) over repeated replays: the launches run back-to-back as
    in the step's graph, without per-launch event markers in between."""

    def __init__(self, dev):
        self.dev = dev
        self.caps = {}  # name -> (stream, graph, launches)

    def __call__(self, name):
        timer = self
        if name not in self.caps:
            st = torch.cuda.Stream(device=self.dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(st):
                g.capture_begin(capture_error_mode="relaxed")
            self.caps[name] = [st, g, 0]

        class _Ctx:
            def __enter__(self_inner):
                cap = timer.caps[name]
                cap[2] += 1
                self_inner.ctx = torch.cuda.stream(cap[0])
                self_inner.ctx.__enter__()
                return self_inner

            def __exit__(self_inner, *a):
                self_inner.ctx.__exit__(*a)
                return False
        return _Ctx()

    def finish(self):
        for st, g, _ in self.caps.values():
            with torch.cuda.stream(st):
                g.capture_end()

    def time(self, reps: int, sleep_cycles: int):
        """us per step of each group, and its launch count."""
        out, cnt = {}, {}
        for name, (st, g, n) in self.caps.items():
            with torch.cuda.stream(st):
                g.replay()  # upload / first-run costs
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(sleep_cycles)  # queue every replay before any runs
                s.record()
                for _ in range(reps):
                    g.replay()
                e.record()
                torch.cuda.synchronize()
            out[name] = s.elapsed_time(e) / reps * 1000.0
            cnt[name] = n
        return out, cnt


def _sleep_cycles_for(ms: float) -> int:
    """Cycles of torch.cuda._sleep that park the stream for about ``ms`` milliseconds."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 1_000_000
    s.record()
    torch.cuda._sleep(n)
    e.record()
    torch.cuda.synchronize()
    per_ms = n / max(s.elapsed_time(e), 1e-3)
    return int(per_ms * ms)


def pmc_traffic():
    """HBM bytes per step of the GEMM group from the newest committed PMC summary
    (profiles/rNN_pmc_traffic.json, made by tools/pmc_summary.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench); None when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    g = d.get("gemm")
    if not g:
        return None, None
    return (int(g["hbm_bytes_per_launch"] * g["launches_per_step_approx"]),
            os.path.relpath(files[-1], ROOT))


def _graph_time_us(fn, n=20, reps=5):
    """Device time per call of ``fn``: n calls captured in one hipGraph, replayed ``reps``
    times between HIP events on the capturing stream."""
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
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
    return s.elapsed_time(e) / (n * reps) * 1000.0


def gather_rooflines(tr, batch, B, c, dev):
    """TBE kernels timed on their own (SURVEY.md §8d bytes):
    * the C3 step's gather (dlrm_tbe_forward on the bench batch, without the sort and the
      bottom MLP that share the step's lookup launch);
    * the bandwidth regime the embedding metric is about: the C1 table shape (8 x 1e5 rows,
      D=64, L=100, B=2048: 0.43 GB gathered per batch), forward and backward + exact SGD."""
    from dlrm_hip import ops
    D, L = c["D"], c["L"]
    T = tr.T_local
    out = {}
    if T > 0 and not tr.qr_active:  # (QR: the lookup runs on the expanded physical CSR)
        pooled = torch.empty(B, T, D, device=dev)
        us = _graph_time_us(lambda: ops.tbe_forward(tr.weights, tr.row_base, T, B, batch.indices,
                                                    batch.offsets, out=pooled))
        n = T * B * L
        by = n * (4 * D + 4) + 4 * (T * B + 1) + 4 * T * B * D
        out["c3_gather_only"] = {"us": round(us, 2), "bytes": by,
                                 "achieved": round(by / us / 1e3, 1),
                                 "frac": round(by / us / 1e3 / HBM_PEAK_GBS, 4)}
    T1, R1, D1, L1, B1 = 8, 100000, 64, 100, 2048
    g = torch.Generator(device=dev).manual_seed(7)
    W1 = torch.empty(T1 * R1, D1, device=dev).uniform_(-0.003, 0.003, generator=g)
    rb1 = torch.arange(T1 + 1, dtype=torch.int64, device=dev) * R1
    idx1 = torch.randint(0, R1, (T1 * B1 * L1,), dtype=torch.int32, device=dev, generator=g)
    off1 = torch.arange(T1 * B1 + 1, dtype=torch.int32, device=dev) * L1
    pooled1 = torch.empty(B1, T1, D1, device=dev)
    grad1 = torch.empty(B1, T1, D1, device=dev).uniform_(-1e-3, 1e-3, generator=g)
    ws1 = torch.empty(ops.tbe_backward_workspace_size(idx1.numel(), T1 * R1, D1),
                      dtype=torch.uint8, device=dev)
    n1 = T1 * B1 * L1
    fwd_by = n1 * (4 * D1 + 4) + 4 * (T1 * B1 + 1) + 4 * T1 * B1 * D1
    bwd_by = 4 * T1 * B1 * D1 + n1 * (4 + 8 * D1)
    fus = _graph_time_us(lambda: ops.tbe_forward(W1, rb1, T1, B1, idx1, off1, out=pooled1), n=10)
    bus = _graph_time_us(lambda: ops.tbe_backward("sgd", W1, rb1, T1, B1, idx1, off1, grad1,
                                                  lr=1e-9, workspace=ws1,
                                                  max_lookups_per_table=B1 * L1), n=10)
    uniq = int(torch.unique((idx1.view(T1, -1).long()
                             + torch.arange(T1, device=dev).view(-1, 1) * R1)).numel())
    out["c1_shape"] = {"tables": T1, "rows": R1, "emb_dim": D1, "lookups_per_bag": L1,
                       "batch": B1,
                       "fwd_us": round(fus, 2), "fwd_bytes": fwd_by,
                       "fwd_achieved": round(fwd_by / fus / 1e3, 1),
                       "fwd_frac": round(fwd_by / fus / 1e3 / HBM_PEAK_GBS, 4),
                       "bwd_sgd_us": round(bus, 2), "bwd_bytes_upper": bwd_by,
                       "unique_rows": uniq,
                       "bwd_bytes_dedup": 4 * T1 * B1 * D1 + n1 * 4 + uniq * 8 * D1,
                       "bwd_achieved_upper": round(bwd_by / bus / 1e3, 1),
                       "bwd_achieved_dedup": round((4 * T1 * B1 * D1 + n1 * 4 + uniq * 8 * D1)
                                                   / bus / 1e3, 1)}
    return out


def input_pipeline_rate(tr, c, B, dev, steps=60, warmup=5, nb=16):
    """The step fed from Criteo binary records on the host: a
    synthetic record file of the workload's shape (label, 13 dense counts, 26 indices within
    each table's rows; ~5 MB), read by dlrm_hip.data.RecordPipeline (reader thread ->
    pinned slots -> H2D on a copy stream -> one decode launch into the fixed Batch), the
    step replayed from a hipGraph captured on that Batch.  PCIe- and file-inclusive rate:
    reported beside ``value``, never as it."""
    import tempfile
    from dlrm_hip.data import RecordPipeline
    rows = c["rows"]
    rng = np.random.RandomState(5)
    rec = np.empty((nb * B, 1 + 13 + len(rows)), dtype=np.int32)
    rec[:, 0] = rng.randint(0, 2, nb * B)
    rec[:, 1:14] = rng.randint(0, 1000, (nb * B, 13))
    for t, n in enumerate(rows):
        rec[:, 14 + t] = rng.randint(0, n, nb * B)
    fd, path = tempfile.mkstemp(suffix=".bin")
    os.close(fd)
    pipe = None
    try:
        rec.tofile(path)
        pipe = RecordPipeline(path, B, tr, max_ind_range=10_000_000, depth=3)
        batch = pipe.next()
        tr.step(batch)
        torch.cuda.synchronize()
        run = tr.capture(batch)
        for _ in range(warmup):
            pipe.next()
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            pipe.next()
            run()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return {"value": round(B * steps / el, 1), "unit": "samples/s",
                "ms_per_step": round(el / steps * 1000.0, 4), "steps": steps,
                "what": "records on the host (file, page cache) -> pinned -> H2D (copy stream) "
                        "-> device decode -> step graph; PCIe-inclusive, not `value`"}
    except Exception as e:  # noqa: BLE001 - reported, the headline line must still print
        return {"error": repr(e)}
    finally:
        if pipe is not None:
            pipe.close()
        os.unlink(path)


def cpu_baseline(c, seconds: float):
    """The CPU oracle (a restatement of the reference step, pinned to its golden vectors)
    timed on this host's cores: bounded sample of the same workload."""
    sys.path.insert(0, ROOT)
    import oracle as O
    threads = torch.get_num_threads()
    cap = 1_000_000
    rows = [min(r, cap) for r in c["rows"]]
    D = c["D"]
    ln_top = [num_int(len(rows), D)] + c["top"]
    B, L = c["B"], c["L"]
    tables = []
    g = torch.Generator().manual_seed(0)
    for n in rows:
        a = float(np.sqrt(1.0 / n))
        tables.append(torch.empty(n, D).uniform_(-a, a, generator=g).numpy())
    np.random.seed(0)
    m = O.OracleDLRM(D, rows, c["bot"], ln_top, loss_function=c["loss"], tables=tables)
    qr = c.get("qr")
    if qr:  # QR tables with the capped row counts
        torch.manual_seed(0)
        for k, n in enumerate(rows):
            if n > qr["threshold"]:
                m.emb_l[k] = O.QREmbeddingBagOracle(n, D, qr["collisions"], qr["operation"])
    rng = np.random.RandomState(1)
    batches = []
    for _ in range(4):
        X = torch.log1p(torch.tensor(rng.rand(B, c["bot"][0]).astype(np.float32)))
        lS_o = torch.arange(B).mul(L).repeat(len(rows), 1)
        lS_i = [torch.tensor(rng.randint(0, n, size=B * L)) for n in rows]
        T = torch.tensor(np.round(rng.rand(B, 1)).astype(np.float32))
        batches.append((X, lS_o, lS_i, T))
    for i in range(2):
        m.train_step(*batches[i % 4], c["lr"] * 0.01)
    n, t0 = 0, time.perf_counter()
    while True:
        m.train_step(*batches[n % 4], c["lr"] * 0.01)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 3) or n >= 2000:
            break
    return {"value": B * n / el, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"oracle (torch-CPU restatement of the reference step) on the "
                      f"{c['workload']} shape with tables capped at {cap} rows, B={B}, "
                      f"{n} timed steps ({el:.1f} s), {threads} threads",
            "ms_per_step": 1000.0 * el / n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="terabyte", choices=list(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="global batch (default: config's)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraphs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-kernel-timing", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("error: --gpus N>1 must be launched with torch.distributed.run", file=sys.stderr)
            sys.exit(2)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        pg = dist.group.WORLD

    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig

    c = dict(CONFIGS[args.config])
    B = args.batch or c["B"]
    T = len(c["rows"])
    ln_top = [num_int(T, c["D"])] + c["top"]
    qr = c.get("qr")
    cfg = TrainerConfig(m_spa=c["D"], ln_emb=c["rows"], ln_bot=c["bot"], ln_top=ln_top,
                        loss_function=c["loss"], learning_rate=c["lr"], optimizer=c["optimizer"],
                        sharder="greedy", qr_flag=qr is not None,
                        qr_collisions=qr["collisions"] if qr else 4,
                        qr_operation=qr["operation"] if qr else "mult",
                        qr_threshold=qr["threshold"] if qr else 200)
    tr = DLRMTrainer(cfg, device=dev, rank=rank, world_size=world, process_group=pg, seed=1)
    nb = 10  # the reference cycles 10 pre-generated batches (dlrm_data_pytorch.py:631)
    batches = [tr.synthetic_batch(B, c["L"], seed=100 + i) for i in range(nb)]
    torch.cuda.synchronize()

    # hipGraphs: one per batch on one GPU; on several GPUs the step's kernel segments are
    # graphs replayed around the eager RCCL collectives (trainer.capture)
    use_graph = not args.no_graph
    graphs = None
    if use_graph:
        try:
            for i in range(3):
                tr.step(batches[i % nb])
            torch.cuda.synchronize()
            pool = torch.cuda.graph_pool_handle()
            graphs = [tr.capture(batches[i], pool=pool) for i in range(nb)]
            torch.cuda.synchronize()
        except Exception as e:  # capture unsupported -> eager
            print(f"[bench] hipGraph capture failed ({e!r}); eager launches", file=sys.stderr)
            graphs = None
            use_graph = False

    def run_step(k):
        if graphs is not None:
            graphs[k % nb]()
        else:
            tr.step(batches[k % nb])

    for k in range(args.warmup):
        run_step(k)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for k in range(args.steps):
        run_step(k)
        evs[k + 1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per_step = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps))
    pct = {q: round(per_step[min(len(per_step) - 1, int(q / 100 * len(per_step)))], 4)
           for q in (10, 50, 90)}
    barrier()
    el_t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el_t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el_t.item())
    value = B * args.steps / elapsed
    loss = float(tr._bufs[(B // world, B)]["loss"].item())

    # ---- per-kernel HIP-event timing pass (same step, eager launches) for the roofline
    roofline, emb_roof, groups = None, None, None
    Bl = B // world
    # lookups run on the physical tables (a QR table is a quotient + a remainder table)
    flops, fwd_bytes, bwd_bytes = algorithmic_work(c, Bl, B, tr.T_phys, world,
                                                   bottom_fused=tr.bottom_fused)
    if not args.no_kernel_timing:
        # capture one eager step's launches per kernel group (after the timed region: the
        # captured groups run on stale data, which does not change their timing)
        timer = GroupGraphTimer(dev)
        cap_steps, reps = 10, 5
        for _ in range(cap_steps):  # each group graph holds cap_steps steps' launches
            tr.step(batches[0], profile=timer)
        timer.finish()
        torch.cuda.synchronize()
        tot_us, cnt = timer.time(reps, _sleep_cycles_for(2.0))
        tot_us = {k: v / cap_steps for k, v in tot_us.items()}
        cnt = {k: v // cap_steps for k, v in cnt.items()}
        tot = {k: v / 1000.0 for k, v in tot_us.items()}  # ms per step
        groups = {k: round(v, 2) for k, v in tot_us.items()}  # us per step
        gemm_ms = tot.get("gemm", 0.0)
        if gemm_ms > 0:
            ach = flops / (gemm_ms * 1e-3) / 1e12
            traffic, tsrc = pmc_traffic() if world == 1 else (None, None)
            roofline = {"bound": "mfma", "kernel": "gemm_f32_mfma (all MLP GEMM launches)",
                        "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFS,
                        "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFS, 4),
                        "traffic": traffic,
                        "traffic_unit": "HBM bytes per step, GEMM group (FETCH_SIZE x2 + "
                                        "WRITE_SIZE)" if traffic else None,
                        "traffic_source": tsrc,
                        "launches_per_step": cnt.get("gemm", 0),
                        "us_per_step": round(gemm_ms * 1000.0, 2),
                        "timing": f"per-group hipGraph of {cap_steps} steps' launches, HIP "
                                  f"events over {reps} replays",
                        "algorithmic_flop_per_step": flops}
        f_ms = tot.get("tbe_fwd", 0.0)
        b_ms = tot.get("tbe_bwd", 0.0)
        if f_ms > 0 and b_ms > 0:
            emb_roof = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                        "fwd_achieved": round(fwd_bytes / (f_ms * 1e-3) / 1e9, 1),
                        "fwd_frac": round(fwd_bytes / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "fwd_bytes": fwd_bytes, "fwd_us": round(f_ms * 1000.0, 2),
                        "bwd_achieved_upper": round(bwd_bytes / (b_ms * 1e-3) / 1e9, 1),
                        "bwd_bytes_upper": bwd_bytes, "bwd_us": round(b_ms * 1000.0, 2),
                        "fwd_note": "fwd_us is the step's lookup launch, which also runs the "
                                    "backward's index sort and the bottom MLP forward"}
        if rank == 0 and world == 1 and emb_roof is not None:
            emb_roof.update(gather_rooflines(tr, batches[0], B, c, dev))

    pipe_rate = None
    if world == 1 and not args.no_kernel_timing:
        pipe_rate = input_pipeline_rate(tr, c, B, dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(c, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000.0, 4),
            "ms_per_step_p10_p50_p90": [pct[10], pct[50], pct[90]],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (device-generated, reference distributions; random init)",
            "config": {"workload": c["workload"], "global_batch": B, "local_batch": Bl,
                       "tables": T, "rows_total": int(sum(c["rows"])), "emb_dim": c["D"],
                       "lookups_per_bag": c["L"], "bot": c["bot"], "top": ln_top,
                       "optimizer": c["optimizer"], "qr": c.get("qr"),
                       "parallelism": f"table-sharded emb x{world} + dp{world}",
                       "hip_graph": use_graph},
            "loss_last": loss,
            "roofline": roofline,
            "embedding_roofline": emb_roof,
            "kernel_us_per_step": groups,
            "input_pipeline": pipe_rate,
            "cpu_baseline": cpu,
        }
        if cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
