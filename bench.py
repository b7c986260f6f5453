#!/usr/bin/env python3
"""DLRM training-step throughput on MI355X (samples/s, fwd + loss + bwd + update).

Workload (BASELINE.json configs[3], the metric's headline config): MLPerf Terabyte-shaped
synthetic DLRM — 26 tables with the terabyte row counts hashed to 1e7 (54,063,992 rows,
27.7 GB fp32 resident in HBM), D=128, bottom 13-512-256-128, top 479-1024-1024-512-256-1,
dot interaction, BCE, SGD lr 1.0, global batch 2048 (strong scaling over ranks, the
reference methodology of bench/dlrm_s_benchmark.sh), one lookup per bag (Criteo one-hot).

    python bench.py [--gpus N --steps K --warmup W]
        N > 1: one process per GPU.  Launched by torch.distributed.run (the driver's form)
        or, when WORLD_SIZE is unset, bench.py starts torch.distributed.run itself (a child
        process, before any GPU call) and returns its exit status.
    python bench.py --emulate-world 8 --emulate-rank 2     # one rank of the W=8 job, 1 GPU

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
    # --optimizer=rwsadagrad.  lr 1e-4: with the QR init U[sqrt(1/n), 1]
    # the reference's model saturates its sigmoid after one RWSAdagrad step at lr >= 0.01
    # (BCE ~50: every output exactly 0 or 1, zero gradient, no recovery; tools/c4_lr_probe.py
    # on the oracle), and at 1e-3 it recovers or not depending on the init seed; at 1e-4 the
    # loss stays near 0.69 and falls for every seed tried (tools/c4_trajectory.py on the
    # engine at full size, profiles/r03_c4_trajectory.txt).  The step's work does not
    # depend on lr.
    "terabyte_qr_rwsadagrad": dict(workload="mlperf_terabyte_synthetic+qr+rwsadagrad",
                                   rows=TERABYTE_ROWS, D=128, bot=[13, 512, 256, 128],
                                   top=[1024, 1024, 512, 256, 1], B=2048, L=1, loss="bce",
                                   lr=0.0001, optimizer="rwsadagrad",
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


def pmc_traffic(config: str):
    """HBM bytes per step of the GEMM group from the newest committed PMC summary of this
    bench config (profiles/rNN_pmc_traffic.json, made by tools/pmc_summary.py from
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench); None when absent."""
    import glob
    files = [f for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
             if json.load(open(f)).get("_config", "terabyte") == config]
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


def preheat_device(dev, ms: float) -> float:
    """Setup, not measurement: a 4096^3 GEMM loop on scratch buffers (no model state read or
    written) for ~ms milliseconds.  From idle the chip needs ~50 steps (~25 ms) of load to
    reach its steady clocks (tools/ramp_probe.py, profiles/r03_ramp_probe.txt: the first 50
    steps average 487 us against 451 us after), which a 5-step warm-up does not give.  It runs
    on torch.matmul (hipBLASLt), so a kernel trace of the bench keeps the library's GEMM
    kernels to the step's own launches."""
    n = 4096
    A = torch.randn(n, n, device=dev)
    C = torch.empty(n, n, device=dev)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(4):
            torch.matmul(A, A, out=C)
        torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3
    del A, C
    return round(el, 1)


def box_calibration(dev):
    """Fixed-work probes that separate box-to-box variance from code regressions: a 4096^3
    f32 GEMM on hipBLASLt (torch.matmul, TFLOP/s; a kernel the step never runs, so the
    bench's kernel trace keeps the library's GEMM kernels to the step), a 1 GiB
    device-to-device copy (GB/s, read + write), and the clocks the SMI reports (rocm-smi;
    may be absent)."""
    out = {}
    try:
        g = torch.Generator(device=dev).manual_seed(3)
        n = 4096
        A = torch.randn(n, n, device=dev, generator=g)
        Bm = torch.randn(n, n, device=dev, generator=g)
        C = torch.empty(n, n, device=dev)
        us = _graph_time_us(lambda: torch.matmul(A, Bm, out=C), n=5, reps=4)
        out["gemm_f32_4096_tflops_hipblaslt"] = round(2 * n ** 3 / us / 1e6, 2)
        src = torch.empty(1 << 28, device=dev)  # 1 GiB
        dst = torch.empty_like(src)
        us = _graph_time_us(lambda: dst.copy_(src), n=5, reps=4)
        out["copy_1gib_gbs"] = round(2 * src.numel() * 4 / us / 1e3, 1)
        del A, Bm, C, src, dst
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)
    try:
        import subprocess
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True,
                           text=True, timeout=30)
        d = json.loads(r.stdout) if r.returncode == 0 else {}
        card = d.get(sorted(d)[0], {}) if d else {}
        out["smi_clocks"] = {k: v for k, v in card.items()
                             if k.lower().startswith(("sclk", "mclk", "fclk"))}
    except Exception as e:  # noqa: BLE001
        out["smi_clocks"] = repr(e)
    return out


def hbm_gather_roofline(dev, nb=10):
    """The lookup's HBM rate with the caches out of the picture: a C1-like lookup (8 tables,
    D = 64, L = 100, B = 2048: 1.64 M random rows per call) over 8 x 1e6 rows (2 GB, 8x the
    256 MB Infinity Cache), a FRESH batch per call (10 distinct index sets replayed in
    turn), forward and backward + exact SGD.  The C1-shape figures above reuse one batch
    over a 205 MB table set that the Infinity Cache holds."""
    from dlrm_hip import ops
    T, R, D, L, B = 8, 1_000_000, 64, 100, 2048
    g = torch.Generator(device=dev).manual_seed(11)
    W = torch.empty(T * R, D, device=dev).uniform_(-0.003, 0.003, generator=g)
    rb = torch.arange(T + 1, dtype=torch.int64, device=dev) * R
    idxs = [torch.randint(0, R, (T * B * L,), dtype=torch.int32, device=dev, generator=g)
            for _ in range(nb)]
    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev) * L
    pooled = torch.empty(B, T, D, device=dev)
    grad = torch.empty(B, T, D, device=dev).uniform_(-1e-3, 1e-3, generator=g)
    ws = torch.empty(ops.tbe_backward_workspace_size(T * B * L, T * R, D), dtype=torch.uint8,
                     device=dev)
    k = [0]

    def fwd():
        ops.tbe_forward(W, rb, T, B, idxs[k[0] % nb], off, out=pooled)
        k[0] += 1

    def bwd():
        ops.tbe_backward("sgd", W, rb, T, B, idxs[k[0] % nb], off, grad, lr=1e-9, workspace=ws,
                         max_lookups_per_table=B * L)
        k[0] += 1
    n = T * B * L
    fus = _graph_time_us(fwd, n=nb, reps=3)
    bus = _graph_time_us(bwd, n=nb, reps=3)
    fby = n * (4 * D + 4) + 4 * (T * B + 1) + 4 * T * B * D
    uniq = int(torch.unique(idxs[0].view(T, -1).long()
                            + torch.arange(T, device=dev).view(-1, 1) * R).numel())
    bby = 4 * T * B * D + n * 4 + uniq * 8 * D
    del W, idxs, ws
    return {"tables": T, "rows": R, "emb_dim": D, "lookups_per_bag": L, "batch": B,
            "table_bytes": T * R * D * 4, "fresh_batches": nb,
            "fwd_us": round(fus, 2), "fwd_bytes": fby, "fwd_achieved": round(fby / fus / 1e3, 1),
            "fwd_frac": round(fby / fus / 1e3 / HBM_PEAK_GBS, 4),
            "bwd_sgd_us": round(bus, 2), "unique_rows": uniq, "bwd_bytes_dedup": bby,
            "bwd_achieved_dedup": round(bby / bus / 1e3, 1),
            "bwd_frac_dedup": round(bby / bus / 1e3 / HBM_PEAK_GBS, 4)}


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


def skew_rate(tr, c, B, uniform_ms, steps=200, warmup=20, nb=10, a=1.05):
    """SURVEY.md §8d's skew-sensitivity run: the same step on batches whose indices are
    Zipf(1.05) ranks folded onto each table's rows (hot rows: long runs of equal rows in the
    sorted backward), graph-replayed like the headline loop; reported beside ``value``."""
    try:
        batches = [tr.synthetic_batch(B, c["L"], seed=500 + i, dist="zipf", zipf_a=a)
                   for i in range(nb)]
        idx = batches[0].indices.cpu().numpy()
        hot = float((idx == 0).mean())
        tr.step(batches[0])
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        graphs = [tr.capture(b, pool=pool) for b in batches]
        for k in range(warmup):
            graphs[k % nb]()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            graphs[k % nb]()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ms = el / steps * 1000.0
        return {"value": round(B * steps / el, 1), "unit": "samples/s",
                "ms_per_step": round(ms, 4), "vs_uniform": round(uniform_ms / ms, 4),
                "steps": steps, "dist": f"zipf({a}) ranks mod rows, per table",
                "row0_share_of_lookups": round(hot, 4)}
    except Exception as e:  # noqa: BLE001 - reported, the headline line must still print
        return {"error": repr(e)}


def comm_timing(tr, Bl: int, B: int, reps: int = 20):
    """Multi-GPU only: the step's three collectives timed on their own, on the step's own
    buffers and splits (after the timed loop; the all-reduce then scrambles the gradient
    bucket, which nothing reads any more): the pooled-embedding all-to-all forward
    ([B, T_r*D] -> rank-major [B/W, T*D], All2All_Req extend_distributed.py:405-444), its
    reverse (All2All_Wait.backward :489-508) and the dense all-reduce (DDP :1626-1633).
    HIP events on the current stream around `reps` blocking collectives; per-rank values
    are gathered so rank 0 reports every rank (the slowest rank bounds the step)."""
    import torch.distributed as dist
    bufs = tr._bufs[(Bl, B)]
    send, recv = tr._split_sizes(Bl)
    pg = tr.pg

    def t(fn):
        fn()
        torch.cuda.synchronize()
        dist.barrier(group=pg)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1000.0

    a2a_f = t(lambda: dist.all_to_all_single(bufs["recv"], bufs["E"].view(-1)[:sum(send)],
                                             recv, send, group=pg))
    a2a_b = t(lambda: dist.all_to_all_single(bufs["dE"].view(-1)[:sum(send)], bufs["drecv"],
                                             send, recv, group=pg))
    ar = t(lambda: dist.all_reduce(tr.grads, group=pg))
    mine = torch.tensor([a2a_f, a2a_b, ar, 4.0 * sum(send), 4.0 * sum(recv)], dtype=torch.float64,
                        device=tr.dev)
    allv = [torch.zeros_like(mine) for _ in range(tr.world)]
    dist.all_gather(allv, mine, group=pg)
    rows = [v.tolist() for v in allv]
    ar_bytes = 4 * tr.grads.numel()
    return {"reps": reps, "a2a_fwd_us": [round(r[0], 2) for r in rows],
            "a2a_bwd_us": [round(r[1], 2) for r in rows],
            "allreduce_us": [round(r[2], 2) for r in rows],
            "a2a_send_bytes": [int(r[3]) for r in rows], "a2a_recv_bytes": [int(r[4]) for r in rows],
            "allreduce_bytes": ar_bytes,
            "allreduce_busbw_gbs": round(2 * (tr.world - 1) / tr.world * ar_bytes
                                         / (max(r[2] for r in rows) * 1e-6) / 1e9, 1),
            "note": "each collective alone, blocking, on the step's buffers; in the step the "
                    "forward all-to-all overlaps the bottom MLP, the reverse the bottom-MLP "
                    "backward and the all-reduce the embedding backward"}


def launch_ranks(n: int) -> int:
    """bench.py --gpus N without torch.distributed.run's environment: start
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <same args>` as a child
    process (the driver's own launch form, rendezvous on 127.0.0.1), wait for it and return
    its exit status.  Rank 0 of the child job prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def physical_cores():
    """{package: [one hardware thread per physical core]} within this process's allowed
    CPUs."""
    seen, out = set(), {}
    for cpu in sorted(os.sched_getaffinity(0)):
        base = f"/sys/devices/system/cpu/cpu{cpu}/topology"
        try:
            pkg = int(open(f"{base}/physical_package_id").read())
            core = int(open(f"{base}/core_id").read())
        except OSError:
            pkg, core = 0, cpu
        if (pkg, core) in seen:
            continue
        seen.add((pkg, core))
        out.setdefault(pkg, []).append(cpu)
    return out


def socket0_physical_cores(limit: int):
    """One hardware thread per physical core of CPU package 0, within this process's allowed
    CPUs (bench/dlrm_s_benchmark.sh:20-25 binds `numactl --physcpubind=<socket 0 physical
    cores> -m 0`), at most ``limit`` of them (the GPU box's CPU share per GPU is 16)."""
    pc = physical_cores()
    cores = pc.get(0) or next(iter(pc.values()), [])
    return cores[:limit] if cores else sorted(os.sched_getaffinity(0))[:limit]


def all_socket_cores(limit: int):
    """The all-sockets secondary figure's cores: physical cores dealt round-robin over every
    package, at most ``limit`` (the lease's CPU share)."""
    pc = physical_cores()
    lists = [pc[k] for k in sorted(pc)]
    out = []
    for i in range(max((len(v) for v in lists), default=0)):
        for v in lists:
            if i < len(v):
                out.append(v[i])
    return out[:limit]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# The GPU box's CPU share per GPU (its OMP_NUM_THREADS / MAX_JOBS are set to it; nproc
# shows the whole machine): the CPU baseline never runs more threads than this.
LEASE_CPU_SHARE = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)


def _cpu_child_run(config_name: str, seconds: float, cores):
    import subprocess
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               ROCR_VISIBLE_DEVICES="", OMP_NUM_THREADS=str(len(cores)))
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child", "--config", config_name,
           "--cpu-seconds", str(seconds), "--cpu-cores", ",".join(map(str, cores))]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=seconds * 4 + 240)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        return {"error": f"cpu child rc={r.returncode}: {r.stderr[-400:]}"}
    return json.loads(line[-1])


def cpu_baseline(c, seconds: float, config_name: str, max_cores: int = 0):
    """The CPU oracle (a restatement of the reference step, pinned to its golden vectors and
    calibrated against the reference's own DLRM_Net step: profiles/r03_cpu_calibration.json)
    timed on this host: a CHILD process (no GPU runtime in it: HIP/CUDA devices hidden) pinned
    to socket 0's physical cores, one torch thread per core; memory is first-touch on the
    pinned cores' node (numactl is not in the image).  Bounded sample of the same workload.
    The methodology of bench/dlrm_s_benchmark.sh:20-25 binds ALL of socket 0's physical
    cores; the lease gives this job LEASE_CPU_SHARE of them, which caps the thread count
    (recorded with the affinity mask).  Secondary figure: the same number
    of cores dealt over every socket."""
    max_cores = max_cores or LEASE_CPU_SHARE
    try:
        cores = socket0_physical_cores(max_cores)
        out = _cpu_child_run(config_name, seconds, cores)
        if "error" in out:
            return out
        pc = physical_cores()
        out.update({
            "affinity_cpus": len(os.sched_getaffinity(0)),
            "physical_cores_per_socket": {str(k): len(v) for k, v in sorted(pc.items())},
            "lease_cpu_share": LEASE_CPU_SHARE,
            "binding_note": f"socket 0 has {len(pc.get(0, []))} physical cores in this "
                            f"process's affinity mask; the lease's CPU share caps the run at "
                            f"{max_cores} threads (one per physical core)"})
        alls = all_socket_cores(max_cores)
        if len(pc) > 1 and alls:
            sec = _cpu_child_run(config_name, max(seconds / 2, 4.0), alls)
            out["all_sockets"] = {k: sec.get(k) for k in
                                  ("value", "cores", "cpu_list", "ms_per_step",
                                   "ms_per_step_p10_p50_p90", "error") if k in sec}
        return out
    except Exception as e:  # noqa: BLE001 - reported; the headline line must still print
        return {"error": repr(e)}


def cpu_child(c, seconds: float, cores):
    """Runs in the pinned child: times the oracle's training step (SGD at the workload's lr
    scaled by 0.01 so the capped tables stay finite; the step's work does not depend on lr)."""
    os.sched_setaffinity(0, cores)
    torch.set_num_threads(len(cores))
    sys.path.insert(0, ROOT)
    import oracle as O
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
    times = []
    while True:
        t1 = time.perf_counter()
        m.train_step(*batches[n % 4], c["lr"] * 0.01)
        times.append(time.perf_counter() - t1)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 3) or n >= 2000:
            break
    capped = sum(1 for r in c["rows"] if r > cap)
    times.sort()
    q = lambda f: 1000.0 * times[min(len(times) - 1, int(f * len(times)))]  # noqa: E731
    print(json.dumps({
        "value": B * n / el, "unit": "samples/s", "cores": len(cores), "kind": "port",
        "median_value": B / (q(0.5) / 1000.0),
        "ms_per_step_p10_p50_p90": [round(q(0.1), 3), round(q(0.5), 3), round(q(0.9), 3)],
        "cpu_model": cpu_model(), "cpu_list": cores,
        "binding": "socket 0, one thread per physical core (os.sched_setaffinity; first-touch "
                   "memory on that node), torch threads = cores",
        "sample": f"oracle (torch-CPU restatement of the reference step) on the "
                  f"{c['workload']} shape, B={B}, {n} timed steps ({el:.1f} s)"
                  + (f", {capped} tables capped at {cap} rows" if capped else ""),
        "ms_per_step": 1000.0 * el / n}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="terabyte", choices=list(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="global batch (default: config's)")
    ap.add_argument("--lr", type=float, default=0.0, help="learning rate (default: config's)")
    ap.add_argument("--preheat-ms", type=float, default=300.0,
                    help="setup: ms of a model-independent 4096^3 GEMM loop before the warm-up "
                         "steps, so the clocks have left their idle state (tools/ramp_probe.py)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraphs")
    ap.add_argument("--bot-sched", default="", help="A/B: bottom-MLP backward schedule "
                    "(partial | full | auto; default: the trainer's)")
    ap.add_argument("--tbe-role", type=int, default=-1, help="A/B: 1 = the embedding update's "
                    "passes ride on the bottom-backward GEMM launches, 0 = own launches "
                    "(default: the trainer's)")
    ap.add_argument("--full-last-wgrad", type=int, default=-1, help="A/B: 1 = the step's last "
                    "wgrad reduces its K split inside its own launch (no trailing REDUCE launch)")
    ap.add_argument("--head-role", type=int, default=-1, help="A/B: 1 = the head's finalize "
                    "pass rides on the top-MLP backward's first launch, 0 = own launch")
    ap.add_argument("--early-sort", type=int, default=-1, help="A/B: 1 = the backward's "
                    "sort on the side stream beside the forward (tables past the LDS sort)")
    ap.add_argument("--feature-pad", type=int, default=-1, help="A/B: 1 = E / dE rows at a "
                    "batch stride of an odd number of 256-byte chunks (one GPU)")
    ap.add_argument("--bottom-parts", type=int, default=-1, help="A/B: workgroups per 16-row "
                    "block of the fused bottom MLP (1, 2, 4; 0 = auto)")
    ap.add_argument("--tbe-role-at", default="", help="A/B: bottom-backward launches "
                    "carrying the update's two passes, e.g. 0,2")
    ap.add_argument("--tune", default="", help="A/B: library plan overrides, e.g. "
                    "gemm_tile=64032 (dlrm_set_tuning keys, ops.TUNE_KEYS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--emulate-world", type=int, default=0, help="one GPU runs rank "
                    "--emulate-rank of a W-rank job: its tables over the global batch, the "
                    "B/W dense batch, collectives replaced by same-size device copies "
                    "(trainer.EmulatedComm); a builder's projection, not a multi-GPU figure")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--emulate-capture", choices=["segments", "whole"], default="segments",
                    help="segments (default): captured as RCCL captures - four graphs around "
                    "the eager all-to-alls; whole: one graph (no RCCL path can do that today)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-cores", default="", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_child:  # the pinned CPU-baseline process (no GPU runtime)
        cpu_child(dict(CONFIGS[args.config]), args.cpu_seconds,
                  [int(v) for v in args.cpu_cores.split(",") if v])
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not started by torch.distributed.run: start it as a CHILD process (nothing here
        # has touched the GPU; never exec) and return its exit status
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.launch_probe:  # launcher test: report the rank environment, touch no GPU
        print(json.dumps({"probe": True, "rank": rank, "world": world,
                          "local_rank": local_rank,
                          "master": os.environ.get("MASTER_ADDR")}), flush=True)
        return
    emulated = args.emulate_world > 1
    if emulated and (world > 1 or not 0 <= args.emulate_rank < args.emulate_world):
        print("error: --emulate-world runs alone, with 0 <= --emulate-rank < W", file=sys.stderr)
        sys.exit(2)
    procs = world  # processes of this job; the trainer's rank count may be emulated
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        pg = dist.group.WORLD

    from dlrm_hip.trainer import DLRMTrainer, EmulatedComm, TrainerConfig
    tune = None
    if args.tune:
        from dlrm_hip import ops
        tune = ops.tuning(**{k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(","))})
        tune.__enter__()  # this (launching) thread, for the whole run

    c = dict(CONFIGS[args.config])
    if args.lr > 0:
        c["lr"] = args.lr
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
    if emulated:
        world, rank = args.emulate_world, args.emulate_rank
        tr = DLRMTrainer(cfg, device=dev, rank=rank, world_size=world,
                         comm=EmulatedComm(whole=args.emulate_capture == "whole"), seed=1)
    else:
        tr = DLRMTrainer(cfg, device=dev, rank=rank, world_size=world, process_group=pg,
                         seed=1)
    if args.bot_sched:
        tr.bot_sched = args.bot_sched
    if args.tbe_role >= 0:
        tr.tbe_role = bool(args.tbe_role)
    if args.full_last_wgrad >= 0:
        tr.full_last_wgrad = bool(args.full_last_wgrad)
    if args.head_role >= 0:
        tr.head_role = bool(args.head_role)
    if args.early_sort >= 0:
        tr.early_sort = args.early_sort  # 1: at the start of the step, 2: after the lookup
    if args.feature_pad >= 0:
        tr.feature_pad = bool(args.feature_pad)
    if args.bottom_parts >= 0:
        tr.bottom_parts = args.bottom_parts
    if args.tbe_role_at:
        tr.tbe_role_at = tr._check_role_at(int(v) for v in args.tbe_role_at.split(","))
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
            # setup, not warm-up: replay every captured graph twice so the first (upload)
            # replay of each of the nb graphs happens here, whatever --warmup is
            for _ in range(2):
                for gr in graphs:
                    gr()
            torch.cuda.synchronize()
        except Exception as e:  # capture unsupported -> eager
            print(f"[bench] hipGraph capture failed ({e!r}); eager launches", file=sys.stderr)
            graphs = None
            use_graph = False

    preheat = preheat_device(dev, args.preheat_ms) if args.preheat_ms > 0 else 0.0

    def run_step(k):
        if graphs is not None:
            graphs[k % nb]()
        else:
            tr.step(batches[k % nb])

    for k in range(args.warmup):
        run_step(k)

    def barrier():
        if procs > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    loss_first = float(tr._bufs[(B // world, B)]["loss"].item())  # after setup + warm-up
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for k in range(args.steps):
        run_step(k)
        evs[k + 1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per_step = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps))
    gpu_event_ms = evs[0].elapsed_time(evs[-1])  # the timed region on the GPU's own clock
    pct = {q: round(per_step[min(len(per_step) - 1, int(q / 100 * len(per_step)))], 4)
           for q in (10, 50, 90)}
    barrier()
    el_t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if procs > 1:
        torch.distributed.all_reduce(el_t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el_t.item())
    value = B * args.steps / elapsed
    loss = float(tr._bufs[(B // world, B)]["loss"].item())

    # ---- per-kernel HIP-event timing pass (same step, eager launches) for the roofline
    roofline, emb_roof, groups, interaction_roof = None, None, None, None
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
            traffic, tsrc = pmc_traffic(args.config) if world == 1 else (None, None)
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
        i_us = tot_us.get("interaction_fwd", 0.0) + tot_us.get("interaction_bwd", 0.0)
        if i_us > 0 and c.get("interaction", "dot") == "dot":
            F = len(c["rows"]) + 1
            alg = 3 * F * (F - 1) * c["D"] * Bl          # fwd F(F-1)D + bwd 2F(F-1)D per sample
            Fp = (F + 31) // 32 * 32                       # the kernels' 32-padded Gram tiles
            issued = 3 * 2 * Fp * Fp * c["D"] * Bl
            interaction_roof = {
                "bound": "mfma (fp32 v_mfma_f32_32x32x2f32)", "us_per_step": round(i_us, 2),
                "algorithmic_flop_per_step": alg, "mfma_flop_per_step": issued,
                "achieved_tflops": round(alg / i_us / 1e6, 3),
                "frac_of_fp32_peak": round(alg / i_us / 1e6 / FP32_MFMA_PEAK_TFS, 4),
                "issued_mfma_frac": round(issued / i_us / 1e6 / FP32_MFMA_PEAK_TFS, 4),
                "hbm_bytes_per_step": (F * c["D"] + F * (F - 1) // 2 + c["D"]) * 4 * Bl * 2,
                "hbm_achieved_gbs": round((F * c["D"] + F * (F - 1) // 2 + c["D"]) * 8 * Bl
                                          / i_us / 1e3, 1)}
        f_ms = tot.get("tbe_fwd", 0.0)
        b_ms = tot.get("tbe_bwd", 0.0)
        if f_ms > 0 and b_ms > 0:
            emb_roof = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                        "bwd_achieved_upper": round(bwd_bytes / (b_ms * 1e-3) / 1e9, 1),
                        "bwd_bytes_upper": bwd_bytes, "bwd_us": round(b_ms * 1000.0, 2),
                        "gather_fused": bool(tr.gather_fused)}
            if tr.gather_fused:
                # one-hot batches: the lookup launch only sorts (and runs the bottom MLP);
                # the rows are gathered by the interaction forward, which also reads x and
                # writes R: the gather's bytes are attributed to that kernel's time
                i_ms = tot.get("interaction_fwd", 0.0)
                D_ = c["D"]
                F_ = tr.T_phys + 1
                n_look = tr.T_phys * B * c["L"]
                i_bytes = n_look * (4 * D_ + 4) + Bl * 4 * (D_ + D_ + F_ * (F_ - 1) // 2)
                emb_roof.update({
                    "lookup_launch_us": round(f_ms * 1000.0, 2),
                    "lookup_launch_note": "sort-only lookup launch (dlrm_tbe_forward_presort "
                                          "out=NULL) + the bottom MLP forward role",
                    "fwd_bytes": fwd_bytes,
                    "fwd_in_interaction_us": round(i_ms * 1000.0, 2),
                    "fwd_in_interaction_bytes": i_bytes,
                    "fwd_achieved": round(i_bytes / (i_ms * 1e-3) / 1e9, 1) if i_ms else None,
                    "fwd_frac": round(i_bytes / (i_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                    if i_ms else None,
                    "fwd_note": "the gather runs inside interaction_fwd (dlrm_interact_dot_"
                                "forward_gather): bytes = gathered rows + indices + x + R"})
            else:
                emb_roof.update({
                    "fwd_achieved": round(fwd_bytes / (f_ms * 1e-3) / 1e9, 1),
                    "fwd_frac": round(fwd_bytes / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "fwd_bytes": fwd_bytes, "fwd_us": round(f_ms * 1000.0, 2),
                    "fwd_note": "fwd_us is the step's lookup launch, which also runs the "
                                "backward's index sort (and the bottom MLP forward)"})
        if rank == 0 and world == 1 and emb_roof is not None:
            emb_roof.update(gather_rooflines(tr, batches[0], B, c, dev))
            try:
                emb_roof["hbm_fresh_batches"] = hbm_gather_roofline(dev)
            except Exception as e:  # noqa: BLE001 - reported; the line must still print
                emb_roof["hbm_fresh_batches"] = {"error": repr(e)}

    calib = None
    if not args.no_kernel_timing:
        calib = box_calibration(dev)
    pipe_rate = None
    if world == 1 and not args.no_kernel_timing:
        pipe_rate = input_pipeline_rate(tr, c, B, dev)
    skew = None
    if world == 1 and not args.no_kernel_timing and not args.no_graph:
        skew = skew_rate(tr, c, B, uniform_ms=elapsed / args.steps * 1000.0)

    comm = None
    if procs > 1:
        try:
            comm = comm_timing(tr, B // world, B)
        except Exception as e:  # noqa: BLE001 - reported; the headline line must still print
            comm = {"error": repr(e)}

    cpu = None
    if rank == 0 and world == 1 and not emulated and not args.no_cpu_baseline:
        cpu = cpu_baseline(c, args.cpu_seconds, args.config)

    if (rank == 0 and not emulated) or (emulated and local_rank == 0):
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": procs,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000.0, 4),
            "ms_per_step_p10_p50_p90": [pct[10], pct[50], pct[90]],
            "gpu_event_ms_timed_region": round(gpu_event_ms, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (device-generated, reference distributions; random init)",
            "config": {"workload": c["workload"], "global_batch": B, "local_batch": Bl,
                       "tables": T, "rows_total": int(sum(c["rows"])), "emb_dim": c["D"],
                       "lookups_per_bag": c["L"], "bot": c["bot"], "top": ln_top,
                       "optimizer": c["optimizer"], "qr": c.get("qr"),
                       "parallelism": f"table-sharded emb x{world} + dp{world}",
                       "hip_graph": use_graph, "capture": tr.capture_mode,
                       "graphs_per_step": tr.graphs_per_step if use_graph else None,
                       "bot_sched": tr.bot_sched, "tbe_role": tr.tbe_role,
                       "tbe_role_at": list(tr.tbe_role_at), "bottom_parts": tr.bottom_parts,
                       "head_role": tr.head_role, "early_sort": tr.early_sort,
                       "feature_pad": tr.feature_pad,
                       "full_last_wgrad": tr.full_last_wgrad,
                       "tune": args.tune or None},
            "shard_balance": tr.lookup_balance(B, c["L"]) if world > 1 else None,
            "comm": comm,
            "loss_before_timed": loss_first, "loss_last": loss, "lr": c["lr"],
            "roofline": roofline,
            "embedding_roofline": emb_roof,
            "interaction_roofline": interaction_roof,
            "kernel_us_per_step": groups,
            "box_calibration": calib,
            "setup_preheat_ms": preheat,
            "input_pipeline": pipe_rate,
            "skew_zipf": skew,
            "cpu_baseline": cpu,
        }
        if cpu and "value" in cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 1)
        if emulated:
            # a projection, never the headline metric: its own metric name,
            # value null, the projected rate inside the emulated block
            line["metric"] = "EMULATED one-rank projection (not a multi-GPU measurement)"
            line["value"] = None
            line["emulated"] = {
                "projected_samples_per_s": round(value, 1),
                "world": world, "rank": rank, "local_batch": Bl,
                "tables_this_rank": tr.T_local, "tables_per_rank": tr.tables_per_rank,
                "what": "one GPU runs this rank's kernels at the W-rank shapes; the "
                        "all-to-all is a same-size device copy and the all-reduce a no-op "
                        "(trainer.EmulatedComm): the rank's compute schedule, not the "
                        "fabric; projected_samples_per_s = global batch / this rank's step "
                        "time",
                "note": "builder-run projection; never a multi-GPU measurement"}
        print(json.dumps(line), flush=True)
    if procs > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
