"""The fused HIP training step vs the reference (golden) and the CPU oracle."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import fp32_close

pytestmark = pytest.mark.gpu
dev = "cuda:0"


def _trainer(**kw):
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    return DLRMTrainer, TrainerConfig


def _num_int(T, D, itself=False):
    F = T + 1
    return D + (F * (F + 1) // 2 if itself else F * (F - 1) // 2)


def _compare_state(tr, ref, tol_scale=1.0):
    for k, e in enumerate(ref.emb_l):
        ok, msg = fp32_close(tr.table(k).cpu().numpy(), e.weight.detach().numpy(),
                             atol=1e-5 * tol_scale)
        assert ok, ("emb", k, msg)
    i = 0
    for seq in (ref.bot_l, ref.top_l):
        for m in seq:
            if isinstance(m, torch.nn.Linear):
                W, b = tr.dense_state()[i]
                ok, msg = fp32_close(W.cpu().numpy(), m.weight.detach().numpy(),
                                     atol=1e-5 * tol_scale)
                assert ok, ("W", i, msg)
                ok, msg = fp32_close(b.cpu().numpy(), m.bias.detach().numpy(),
                                     atol=1e-5 * tol_scale)
                assert ok, ("b", i, msg)
                i += 1


def test_c0_three_steps_vs_reference_golden(golden):
    DLRMTrainer, TrainerConfig = _trainer()
    g = golden("c0_train.npz")
    np.random.seed(123)
    ref = O.OracleDLRM(4, [1000] * 3, [13, 512, 4], [10, 4, 2, 1], loss_function="mse")
    cfg = TrainerConfig(m_spa=4, ln_emb=[1000] * 3, ln_bot=[13, 512, 4], ln_top=[10, 4, 2, 1],
                        loss_function="mse", learning_rate=0.01)
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    for s in range(3):
        lS_i = [g[f"s{s}_lS_i{t}"] for t in range(3)]
        b = tr.make_batch(g[f"s{s}_X"], g[f"s{s}_lS_o"], lS_i, g[f"s{s}_T"])
        Z, E = tr.step(b)
        ok, msg = fp32_close(Z.cpu().numpy(), g[f"s{s}_Z"].ravel())
        assert ok, (s, msg)
        ok, msg = fp32_close(E.cpu().numpy(), g[f"s{s}_loss"])
        assert ok, (s, msg)
    for k in range(3):
        ok, msg = fp32_close(tr.table(k).cpu().numpy(), g[f"final_emb{k}"])
        assert ok, msg
    names = [f"bot.{i}" for i in (0, 2)] + [f"top.{i}" for i in (0, 2, 4)]
    for (W, b), nm in zip(tr.dense_state(), names):
        pre, idx = nm.split(".")
        ok, msg = fp32_close(W.cpu().numpy(), g[f"final_{pre}.{idx}.weight"])
        assert ok, (nm, msg)
        ok, msg = fp32_close(b.cpu().numpy(), g[f"final_{pre}.{idx}.bias"])
        assert ok, (nm, msg)


CASES = {
    # C3 shape with rows capped (bench/run_and_time.sh:17 widths), bce
    "c3_small": dict(D=128, rows=[min(r, 2000) for r in O.TERABYTE_ROWS], bot=[13, 512, 256, 128],
                     top=[1024, 1024, 512, 256, 1], B=256, L=1, loss="bce", lr=0.1),
    # C1 shape (bench/dlrm_s_benchmark.sh:38-41) with fewer rows, L=100
    "c1_small": dict(D=64, rows=[20000] * 8, bot=[512, 512, 64], top=[1024, 1024, 1024, 1],
                     B=128, L=100, loss="mse", lr=0.1),
    # C2 Kaggle shape (bench/dlrm_s_criteo_kaggle.sh:24), rows capped
    "c2_small": dict(D=16, rows=[min(r, 5000) for r in O.KAGGLE_ROWS],
                     bot=[13, 512, 256, 64, 16], top=[512, 256, 1], B=128, L=1, loss="bce",
                     lr=0.1),
}


def _rand_batch(rng, rows, B, L, m_den, loss, dist="uniform"):
    X = np.log1p(rng.rand(B, m_den).astype(np.float32))
    lS_o = np.array([np.arange(B) * L for _ in rows], dtype=np.int64)
    if dist == "zipf":  # SURVEY.md §8d skew run: Zipf(1.05) ranks folded onto the rows
        lS_i = [((rng.zipf(1.05, size=B * L) - 1) % n).astype(np.int64) for n in rows]
    else:
        lS_i = [rng.randint(0, n, size=B * L).astype(np.int64) for n in rows]
    T = rng.rand(B, 1).astype(np.float32)
    if loss == "bce":
        T = np.round(T)
    return X, lS_o, lS_i, T


@pytest.mark.parametrize("name", list(CASES))
def test_step_vs_oracle(name):
    """Two steps vs the oracle."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    ln_top = [_num_int(len(rows), D)] + c["top"]
    np.random.seed(7)
    ref = O.OracleDLRM(D, rows, c["bot"], ln_top, loss_function=c["loss"])
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"], ln_top=ln_top,
                        loss_function=c["loss"], learning_rate=c["lr"])
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    rng = np.random.RandomState(3)
    for s in range(2):
        X, lS_o, lS_i, T = _rand_batch(rng, rows, c["B"], c["L"], c["bot"][0], c["loss"])
        Zr, Er = ref.train_step(torch.tensor(X), torch.tensor(lS_o),
                                [torch.tensor(i) for i in lS_i], torch.tensor(T), c["lr"])
        Z, E = tr.step(tr.make_batch(X, lS_o, lS_i, T))
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.numpy().ravel())
        assert ok, (s, msg)
        ok, msg = fp32_close(E.cpu().numpy(), [Er.item()])
        assert ok, (s, msg)
    _compare_state(tr, ref)


def test_synthetic_batch_and_determinism():
    DLRMTrainer, TrainerConfig = _trainer()
    rows, D = [5000] * 4, 32
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=[13, 64, 32], ln_top=[_num_int(4, D), 64, 1],
                        loss_function="bce", learning_rate=0.1)
    outs = []
    for _ in range(2):
        tr = DLRMTrainer(cfg, device=dev, seed=5)
        b = tr.synthetic_batch(512, 3, seed=1)
        assert b.indices.numel() == 4 * 512 * 3 and int(b.offsets[-1]) == 4 * 512 * 3
        assert int(b.indices.max()) < 5000 and int(b.indices.min()) >= 0
        for _ in range(3):
            Z, E = tr.step(b)
        outs.append((Z.cpu().clone(), tr.weights.cpu().clone(), tr.params.cpu().clone()))
    # the whole step is bitwise reproducible (sorted embedding backward, no float atomics)
    for a, b2 in zip(outs[0], outs[1]):
        assert torch.equal(a, b2)


@pytest.mark.parametrize("graph", [False, True])
def test_side_stream_schedule_matches_serial(graph):
    """The two-stream schedule (bottom MLP || lookup, wgrad || next dgrad, bottom backward ||
    embedding backward), eager and captured in a hipGraph, gives bitwise the serial result."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES["c3_small"]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function="bce",
                        learning_rate=0.1)
    res = []
    for conc in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.concurrent = conc
        tr.overlaps = {"fwd", "top", "bot"}
        tr.fuse_bottom = False  # the "fwd" overlap runs the bottom MLP as GEMMs: compare alike
        batches = [tr.synthetic_batch(512, 1, seed=s) for s in range(3)]
        if graph and conc:
            tr.step(batches[0])  # allocate buffers outside capture
            torch.cuda.synchronize()
            gs = []
            for b in batches[1:]:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    tr.step(b)
                gs.append(g)
            for g in gs:
                g.replay()
            for g in gs:
                g.replay()
        else:
            tr.step(batches[0])
            for _ in range(2):
                for b in batches[1:]:
                    tr.step(b)
        torch.cuda.synchronize()
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(),
                    tr._bufs[(512, 512)]["prob"].cpu().clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_batch_size_changes_with_overlaps_match_serial():
    """B, a smaller B', then B again (a short last Criteo block does this) with every side-
    stream overlap on: each batch size keeps its own split-K workspaces, so the result is
    bitwise the serial schedule's (a shared workspace raced between streams)."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES["c3_small"]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function="bce",
                        learning_rate=0.1)
    res = []
    for conc in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=13)
        tr.concurrent = conc
        tr.overlaps = {"fwd", "top", "bot"}
        tr.fuse_bottom = False
        seq = [tr.synthetic_batch(B, 1, seed=s) for s, B in enumerate((2048, 1000, 2048, 1000))]
        for b in seq:
            tr.step(b)
        torch.cuda.synchronize()
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(),
                    tr._bufs[(2048, 2048)]["prob"].cpu().clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_out_of_range_index_is_flagged():
    """The reference's EmbeddingBag raises IndexError on a bad index; the fused step skips
    the lookup, flags it on the device, and check_errors() raises."""
    from dlrm_hip import ops
    DLRMTrainer, TrainerConfig = _trainer()
    rows, D = [100, 50], 8
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=[13, 16, 8], ln_top=[_num_int(2, D), 8, 1],
                        loss_function="bce", learning_rate=0.1)
    tr = DLRMTrainer(cfg, device=dev, seed=1)
    rng = np.random.RandomState(0)
    X, lS_o, lS_i, T = _rand_batch(rng, rows, 16, 1, 13, "bce")
    tr.step(tr.make_batch(X, lS_o, lS_i, T))
    tr.check_errors()  # clean batch: no error
    lS_i[1][3] = 50    # == rows of table 1
    tr.step(tr.make_batch(X, lS_o, lS_i, T))
    with pytest.raises(ops.TBEIndexError):
        tr.check_errors()
    tr.check_errors()  # the flag was reset


def test_fused_bottom_mlp_step_matches_gemm_path():
    """The bottom MLP forward inside the lookup launch (mlp_rows.hpp) vs the same step with
    the bottom MLP as GEMM launches: the two sum in different orders, so the trained state
    agrees within fp32 tolerance, not bitwise."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES["c3_small"]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function="bce",
                        learning_rate=0.1)
    res = []
    for fuse in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.fuse_bottom = fuse
        batches = [tr.synthetic_batch(512, 1, seed=s) for s in range(3)]
        for b in batches:
            tr.step(b)
        assert tr.bottom_fused == fuse
        torch.cuda.synchronize()
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(),
                    tr._bufs[(512, 512)]["prob"].cpu().clone()))
    for a, b in zip(*res):
        ok, msg = fp32_close(b.numpy(), a.numpy(), atol=1e-4)  # 3 steps of drift
        assert ok, msg


@pytest.mark.parametrize("op", ["mult", "add"])
@pytest.mark.parametrize("optimizer", ["sgd", "rwsadagrad"])
@pytest.mark.parametrize("graph", [False, True])
def test_qr_step_vs_oracle(op, optimizer, graph):
    """C4 on the fused engine: tables with more than qr_threshold rows become QR tables
    (quotient ceil(n/c) + remainder c rows, tricks/qr_embedding_bag.py) looked up on the
    expanded physical CSR, combined by the pooled combine kernel; SGD or RWSAdagrad fused
    into the backward.  Against the oracle's QREmbeddingBag + SGD / RWSAdagrad, 3 steps,
    eager or replayed from a captured graph."""
    DLRMTrainer, TrainerConfig = _trainer()
    D, B, c, thr = 32, 256, 4, 200
    rows = [3, 5000, 150, 201, 2000, 64, 1000, 7]
    bot, top = [13, 64, 32], [64, 1]
    ln_top = [_num_int(len(rows), D)] + top
    lr = 0.05
    np.random.seed(11)
    ref = O.OracleDLRM(D, rows, bot, ln_top, loss_function="bce")
    torch.manual_seed(5)
    for k, n in enumerate(rows):
        if n > thr:
            ref.emb_l[k] = O.QREmbeddingBagOracle(n, D, c, op)
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=bot, ln_top=ln_top, loss_function="bce",
                        learning_rate=lr, optimizer=optimizer, qr_flag=True, qr_collisions=c,
                        qr_operation=op, qr_threshold=thr)
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    assert tr.T_phys == len(rows) + sum(1 for n in rows if n > thr)
    opt = O.RWSAdagradOracle(ref.parameters(), lr=lr) if optimizer == "rwsadagrad" else None
    rng = np.random.RandomState(3)
    batches = [_rand_batch(rng, rows, B, 1, bot[0], "bce") for _ in range(3)]
    run = None
    for s, (X, lS_o, lS_i, T) in enumerate(batches):
        Xt, ot, it, Tt = (torch.tensor(X), torch.tensor(lS_o), [torch.tensor(i) for i in lS_i],
                          torch.tensor(T))
        if opt is None:
            Zr, Er = ref.train_step(Xt, ot, it, Tt, lr)
        else:
            Zr = ref(Xt, ot, it)
            Er = ref.loss_fn(Zr, Tt)
            opt.zero_grad()
            Er.backward()
            opt.step()
            Zr, Er = Zr.detach(), Er.detach()
        b = tr.make_batch(X, lS_o, lS_i, T)
        if graph and s == 1:
            static = b
            run = tr.capture(static)
        if run is not None:
            for dst, src in zip((static.X, static.offsets, static.indices, static.target),
                                (b.X, b.offsets, b.indices, b.target)):
                dst.copy_(src)
            run()
            Z, E = tr._cur["prob"], tr._cur["loss"]
        else:
            Z, E = tr.step(b)
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.numpy().ravel())
        assert ok, (s, msg)
        ok, msg = fp32_close(E.cpu().numpy(), [Er.item()])
        assert ok, (s, msg)
    for k, e in enumerate(ref.emb_l):
        got = tr.table(k)
        want = (e.weight_q, e.weight_r) if hasattr(e, "weight_q") else (e.weight,)
        got = got if isinstance(got, tuple) else (got,)
        for g_, w_ in zip(got, want):
            ok, msg = fp32_close(g_.cpu().numpy(), w_.detach().numpy())
            assert ok, ("emb", k, msg)


def test_c1_full_shape_step_vs_oracle():
    """C1 (bench/dlrm_s_benchmark.sh:36-43) at its FULL shape: 8 x 1e5 rows, D = 64,
    B = 2048, L = 100 (1.64 M lookups per step: the long-block TBE backward and the tiled
    per-table sort, the paths bench --config small times), 2 SGD steps vs the oracle."""
    DLRMTrainer, TrainerConfig = _trainer()
    D, rows, B, L = 64, [100000] * 8, 2048, 100
    bot, top = [512, 512, 64], [1024, 1024, 1024, 1]
    ln_top = [_num_int(len(rows), D)] + top
    np.random.seed(21)
    ref = O.OracleDLRM(D, rows, bot, ln_top, loss_function="mse")
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=bot, ln_top=ln_top, loss_function="mse",
                        learning_rate=0.1)
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    rng = np.random.RandomState(4)
    for s in range(2):
        X, lS_o, lS_i, T = _rand_batch(rng, rows, B, L, bot[0], "mse")
        Zr, Er = ref.train_step(torch.tensor(X), torch.tensor(lS_o),
                                [torch.tensor(i) for i in lS_i], torch.tensor(T), 0.1)
        Z, E = tr.step(tr.make_batch(X, lS_o, lS_i, T))
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.numpy().ravel())
        assert ok, (s, msg)
        ok, msg = fp32_close(E.cpu().numpy(), [Er.item()])
        assert ok, (s, msg)
    tr.check_errors()
    _compare_state(tr, ref)


def _checksums(W: torch.Tensor, row_base):
    """Per-table (sum, row-weighted sum) of the device tables in fp64, in 1 M-row pieces."""
    out = []
    for t in range(len(row_base) - 1):
        s0 = s1 = 0.0
        a, b = int(row_base[t]), int(row_base[t + 1])
        for c in range(a, b, 1 << 20):
            e = min(b, c + (1 << 20))
            blk = W[c:e].double()
            w = (torch.arange(c, e, device=W.device, dtype=torch.float64) % 1021 + 1)
            s0 += float(blk.sum())
            s1 += float((blk.sum(1) * w).sum())
        out.append((s0, s1))
    return out


def test_c3_true_terabyte_rows_vs_touched_row_oracle():
    """C3 at the TRUE Terabyte row counts (54,063,992 rows, 27.7 GB on the device; 24-bit
    keys in the per-table LDS sort of the lookup launch, 64-bit row bases), B = 2048, the
    bench's synthetic batches and fused step, 2 steps.  The CPU oracle materialises only the
    rows the batches touch: each table's indices are remapped to its sorted unique-row list
    and those rows copied from the device.  Compared: Z and loss per step, every touched
    row after the updates, and per-table checksums of the whole tables (untouched rows
    unchanged: the checksum moves by exactly the touched rows' change)."""
    DLRMTrainer, TrainerConfig = _trainer()
    rows, D, B = list(O.TERABYTE_ROWS), 128, 2048
    bot, top = [13, 512, 256, 128], [1024, 1024, 512, 256, 1]
    ln_top = [_num_int(len(rows), D)] + top
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=bot, ln_top=ln_top, loss_function="bce",
                        learning_rate=0.1)
    tr = DLRMTrainer(cfg, device=dev, seed=3)
    assert tr.total_rows == 54063992
    batches = [tr.synthetic_batch(B, 1, seed=40 + s) for s in range(2)]
    T = len(rows)
    idx = [b.indices.view(T, B).long().cpu() for b in batches]
    uniq = [torch.unique(torch.cat([i[t] for i in idx])) for t in range(T)]
    assert max(int(u.max()) for u in uniq) >= (1 << 23)  # 24-bit keys really occur
    rb = tr.row_base.cpu()
    gidx = [(u + int(rb[t])).to(dev) for t, u in enumerate(uniq)]
    tabs0 = [tr.weights.index_select(0, g).cpu().numpy() for g in gidx]
    sums0 = _checksums(tr.weights, rb)
    ref = O.OracleDLRM(D, [len(u) for u in uniq], bot, ln_top, loss_function="bce",
                       tables=tabs0)
    lin = [m for seq in (ref.bot_l, ref.top_l) for m in seq if isinstance(m, torch.nn.Linear)]
    with torch.no_grad():
        for m, (W, b) in zip(lin, tr.dense_state()):
            m.weight.copy_(W.cpu())
            m.bias.copy_(b.cpu())
    for s, b in enumerate(batches):
        X = b.X[:, :13].cpu()
        lS_o = torch.arange(B).repeat(T, 1)
        lS_i = [torch.searchsorted(uniq[t], idx[s][t]) for t in range(T)]  # compact rows
        Tg = b.target.cpu().view(-1, 1)
        Zr, Er = ref.train_step(X, lS_o, lS_i, Tg, 0.1)
        Z, E = tr.step(b)
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.numpy().ravel())
        assert ok, (s, msg)
        ok, msg = fp32_close(E.cpu().numpy(), [Er.item()])
        assert ok, (s, msg)
    torch.cuda.synchronize()
    tr.check_errors()
    sums1 = _checksums(tr.weights, rb)
    for t in range(T):
        got = tr.weights.index_select(0, gidx[t]).cpu().double()
        want = ref.emb_l[t].weight.detach()
        ok, msg = fp32_close(got.numpy(), want.double().numpy())
        assert ok, ("table", t, msg)
        w = (gidx[t].cpu().double() % 1021 + 1)
        d0 = float((got - torch.tensor(tabs0[t]).double()).sum())
        d1 = float(((got - torch.tensor(tabs0[t]).double()).sum(1) * w).sum())
        tol = 1e-6 * (1 + abs(sums0[t][0])) + 1e-4
        assert abs((sums1[t][0] - sums0[t][0]) - d0) <= tol, ("checksum", t)
        assert abs((sums1[t][1] - sums0[t][1]) - d1) <= 1100 * tol, ("weighted checksum", t)
    for m, (W, b_) in zip(lin, tr.dense_state()):
        ok, msg = fp32_close(W.cpu().numpy(), m.weight.detach().numpy())
        assert ok, msg


@pytest.mark.parametrize("name", ["c3_small", "c2_small"])
def test_bottom_backward_full_schedule_vs_oracle(name):
    """bot_sched="full": the bottom-MLP wgrads split K inside their own launch (SGD fused)
    and ride in the next dgrad's launch (n_bot launches, no trailing REDUCE); C3 (3 bottom
    layers) and C2 (4: the third g buffer) widths, 2 steps vs the oracle."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    ln_top = [_num_int(len(rows), D)] + c["top"]
    np.random.seed(7)
    ref = O.OracleDLRM(D, rows, c["bot"], ln_top, loss_function=c["loss"])
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"], ln_top=ln_top,
                        loss_function=c["loss"], learning_rate=c["lr"])
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    tr.bot_sched = "full"
    rng = np.random.RandomState(3)
    for s in range(2):
        X, lS_o, lS_i, T = _rand_batch(rng, rows, c["B"], c["L"], c["bot"][0], c["loss"])
        Zr, Er = ref.train_step(torch.tensor(X), torch.tensor(lS_o),
                                [torch.tensor(i) for i in lS_i], torch.tensor(T), c["lr"])
        Z, E = tr.step(tr.make_batch(X, lS_o, lS_i, T))
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.numpy().ravel())
        assert ok, (s, msg)
    _compare_state(tr, ref)


@pytest.mark.parametrize("graph", [False, True])
def test_gather_fused_step_matches_pooled_path(graph):
    """One-hot batches with the lookup gathered inside the dot interaction (the lookup
    launch keeping only its sort role) vs the pooled path (lookup -> [B, T, D] -> interaction):
    the interaction sees identical rows, so 3 SGD steps leave identical state.  Eager and
    replayed from a captured graph; a batch with L = 2 keeps the pooled path."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES["c3_small"]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function="bce",
                        learning_rate=0.1)
    res = []
    for fuse in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.fuse_gather = fuse
        batches = [tr.synthetic_batch(512, 1, seed=s) for s in range(3)]
        poison = None
        if graph:
            tr.step(batches[0])  # eager warm-up step (allocations), then capture
            if fuse:  # the gather-fused step must never write the pooled E
                poison = tr._bufs[(512, 512)]["E"]
                poison.fill_(float("nan"))
            run = tr.capture(batches[0])
            for b in batches:
                for src, dst in zip((b.X, b.offsets, b.indices, b.target),
                                    (batches[0].X, batches[0].offsets, batches[0].indices,
                                     batches[0].target)):
                    if src is not dst:
                        dst.copy_(src)
                run()
        else:
            for i, b in enumerate(batches):
                tr.step(b)
                if fuse and i == 0:
                    poison = tr._bufs[(512, 512)]["E"]
                    poison.fill_(float("nan"))
        assert tr.gather_fused == fuse
        if fuse:  # sort-only lookup launch: E untouched, no other [B, T, D] buffer made
            torch.cuda.synchronize()
            assert bool(torch.isnan(poison).all())
        torch.cuda.synchronize()
        tr.check_errors()
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(),
                    tr._bufs[(512, 512)]["prob"].cpu().clone()))
        tr.step(tr.synthetic_batch(256, 2, seed=9))
        assert not tr.gather_fused
    for a, b in zip(*res):
        assert torch.equal(a, b)


C4_TRAJ_CAPS = {"flips": 2, "aligned": 2, "ill_loss": 8, "bound": 4}


@pytest.mark.parametrize("lr", [1e-4, 1e-3])
def test_c4_terabyte_widths_trajectory_vs_oracle(lr):
    """C4 (QR mult, 4 collisions, threshold 200 + RWSAdagrad) at the Terabyte widths (D = 128,
    bot 13-512-256-128, top 479-1024-1024-512-256-1) with the 26 tables capped at 20k rows,
    B = 256: 10 steps on 10 batches against the oracle's QREmbeddingBag + RWSAdagrad.
    Every step: Z and the loss within the 1e-5 bound (the loss only on steps whose sigmoid
    is not saturated: a clamped log(0) turns a 1-ulp difference of p into O(10) of loss).
    After the last step: every quotient / remainder / plain table and its row-wise momentum
    within 1e-5, and so are the dense weights and their Adagrad sums: every ReLU decision
    on which the engine and the oracle disagree must be explained by an oracle
    pre-activation within rounding of 0 (tests/relu_align.py), and the oracle then follows
    the engine's decision.  lr 1e-4 is the bench's C4 lr (no saturation); at 1e-3 the
    reference's own trajectory swings through saturation (tools/c4_lr_probe.py) and the
    engine must follow it.  On saturated steps the engine's loss must lie in the interval
    the ORACLE's logits allow (relu_align.loss_interval: every sample's clamped BCE term at
    z -+ tau, widened by one ulp of p); the engine's own Z plays no part there.

    Caps (VERDICT r05 "What's weak" #1), from the logged runs (r05 logs; r06
    gpurun_out/r06/pytest_caps.log, profiles/r06_parity_caps.txt):
      * explained ReLU flips <= 2 (logged: r05 0 at lr 1e-4 / 1 at 1e-3; r06 1 / 0);
      * saturated-head samples aligned <= 2 (logged: 0 / 0 in every run);
      * samples with an ill-conditioned loss term <= 8 over the 10 steps (logged: 0 / 0);
      * elements explained beyond 1e-5 <= 1e-5 of the elements compared (13.2 M; logged: r06
        0 at lr 1e-4, 4 at 1e-3 - 1 by the permuted twin, 3 by AdagradBound), those
        explained ONLY by AdagradBound <= 4, each with an error <= 0.1 lr (one Adagrad step
        moves an element by ~lr at most; logged: 2.8e-5 = 0.028 lr, r05 3.3e-5,
        profiles/r05_c4_explain_probe.txt)."""
    import bench
    import relu_align as RA
    DLRMTrainer, TrainerConfig = _trainer()
    c = bench.CONFIGS["terabyte_qr_rwsadagrad"]
    rows = [min(r, 20000) for r in c["rows"]]
    D, bot = c["D"], c["bot"]
    ln_top = [_num_int(len(rows), D)] + c["top"]
    B, thr = 256, c["qr"]["threshold"]
    np.random.seed(0)
    torch.manual_seed(0)
    ref = O.OracleDLRM(D, rows, bot, ln_top, loss_function="bce")
    for k, n in enumerate(rows):
        if n > thr:
            ref.emb_l[k] = O.QREmbeddingBagOracle(n, D, 4, "mult")
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=bot, ln_top=ln_top, loss_function="bce",
                        learning_rate=lr, optimizer="rwsadagrad", qr_flag=True, qr_collisions=4,
                        qr_operation="mult", qr_threshold=thr)
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    relus = RA.align(ref)
    tw = RA.PermutedTwin(ref, B).with_head()  # the oracle's own summation-order spread
    head = RA.AlignedHead(ref)
    ab = RA.AdagradBound(ref, lr)  # after the head: its hooks see the aligned dz
    opt = O.RWSAdagradOracle(ref.parameters(), lr=lr)
    opt2 = O.RWSAdagradOracle(tw.model.parameters(), lr=lr)
    rng = np.random.RandomState(1)
    losses = []
    n_loss_checked = 0
    n_ill_loss = 0
    for s in range(10):
        X, lS_o, lS_i, T = _rand_batch(rng, rows, B, 1, bot[0], "bce")
        Z, E = tr.step(tr.make_batch(X, lS_o, lS_i, T))
        masks = RA.engine_masks(tr, B, B)
        dz = tr._bufs[(B, B)]["dz"].cpu()
        RA.queue(relus, masks)
        tw.queue(masks)
        head.push(dz, T, B)
        tw.push_head(dz, T, B)
        Xt, ot, it, Tt = (torch.tensor(X), torch.tensor(lS_o), [torch.tensor(i) for i in lS_i],
                          torch.tensor(T))
        Zr = ref(Xt, ot, it)
        Er = ref.loss_fn(Zr, Tt)
        opt.zero_grad()
        Er.backward()
        opt.step()
        ab.after_step(opt)
        X2, o2, i2, T2 = tw.batch(Xt, ot, it, Tt)
        E2 = tw.model.loss_fn(tw.model(X2, o2, i2), T2)
        opt2.zero_grad()
        E2.backward()
        opt2.step()
        losses.append((round(E.item(), 5), round(Er.item(), 5)))
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.detach().numpy().ravel())
        assert ok, (s, "Z", losses, msg)
        zr = Zr.detach().double()
        if bool(((zr > 1e-6) & (zr < 1 - 1e-6)).all()):  # no sample saturated
            n_loss_checked += 1
            ok, msg = fp32_close(E.cpu().numpy(), [Er.item()])
            assert ok, (s, "loss", losses, msg)
        else:  # saturated: the interval the oracle's own logits allow (loss_interval)
            lo, hi, n_ill = RA.loss_interval(*head.seen[s])
            n_ill_loss += n_ill
            tol = 1e-5 * max(1.0, abs(Er.item()))
            assert lo - tol <= E.item() <= hi + tol, (s, "saturated loss", E.item(), lo, hi,
                                                      Er.item(), n_ill)
    print("C4 losses (engine, oracle):", losses)
    assert n_loss_checked == 10 if lr <= 1e-4 else n_loss_checked >= 1, n_loss_checked
    ok, msg, flips = RA.report(relus)
    assert ok, msg
    for r in (head, tw.head):
        ok, msg = r.report()
        assert ok, msg
    ok, msg, _ = RA.report(tw.relus)
    assert ok, ("permuted twin", msg)
    torch.cuda.synchronize()
    tr.check_errors()
    st = RA.ExplainStats()
    for t, (e, e2) in enumerate(zip(ref.emb_l, tw.model.emb_l)):
        got_w, got_m = tr.table(t), tr.table_momentum(t)
        parts = [(e.weight_q, e2.weight_q, got_w[0], got_m[0]),
                 (e.weight_r, e2.weight_r, got_w[1], got_m[1])] \
            if hasattr(e, "weight_q") else [(e.weight, e2.weight, got_w, got_m)]
        for p, p2, gw, gm in parts:
            ok, msg, _ = tw.close(gw.cpu().numpy(), p, p2, f"table {t}", st)
            assert ok, msg
            ok, msg, _ = tw.close(gm.cpu().numpy(), opt.state[id(p)]["momentum"],
                                  opt2.state[id(p2)]["momentum"], f"momentum {t}", st)
            assert ok, msg
    lin = [m for seq in (ref.bot_l, ref.top_l) for m in seq if isinstance(m, torch.nn.Linear)]
    lin2 = [m for seq in (tw.model.bot_l, tw.model.top_l) for m in seq
            if isinstance(m, torch.nn.Linear)]
    for L, L2, (W, b), (sW, sb) in zip(lin, lin2, tr.dense_state(), tr.dense_adagrad_state()):
        for got, p, p2 in ((W, L.weight, L2.weight), (b, L.bias, L2.bias)):
            # beyond 1e-5 only where the oracle itself moves that much under a permuted
            # summation order, or where Adagrad's conditioning allows it
            # (relu_align.PermutedTwin, AdagradBound)
            ok, msg, _ = RA.close_explained(got.cpu().numpy(), p, p2, ab.bound[id(p)], "dense",
                                            st)
            assert ok, msg
        for got, p, p2 in ((sW, L.weight, L2.weight), (sb, L.bias, L2.bias)):
            ok, msg, _ = tw.close(got.cpu().numpy(), opt.state[id(p)]["sum"],
                                  opt2.state[id(p2)]["sum"], "adagrad sum", st)
            assert ok, msg
    print(f"lr {lr}: explained ReLU flips {flips}; saturated-head samples aligned "
          f"{head.aligned}; ill-conditioned loss terms {n_ill_loss}; {st}")
    caps = C4_TRAJ_CAPS
    assert flips <= caps["flips"], flips
    assert head.aligned <= caps["aligned"], head.aligned
    assert n_ill_loss <= caps["ill_loss"], n_ill_loss
    assert st.n_explained <= 1e-5 * st.compared, st
    assert st.n_bound <= caps["bound"], st
    assert st.max_bound_err <= 0.1 * lr, st


@pytest.mark.parametrize("graph", [False, True])
def test_c3_zipf_hot_rows_vs_oracle(graph):
    """C3 widths with Zipf(1.05) indices (hot rows: row 0 takes ~5 % of every table's
    lookups, runs of equal rows across many backward blocks) on the bench's path (presort
    launch, gather-fused interaction, sorted block + combine backward), eager and
    graph-replayed, three steps vs the oracle."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES["c3_small"]
    D, rows = c["D"], c["rows"]
    ln_top = [_num_int(len(rows), D)] + c["top"]
    np.random.seed(11)
    ref = O.OracleDLRM(D, rows, c["bot"], ln_top, loss_function=c["loss"])
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"], ln_top=ln_top,
                        loss_function=c["loss"], learning_rate=c["lr"])
    tr = DLRMTrainer.from_oracle(cfg, ref, device=dev)
    rng = np.random.RandomState(13)
    B = 1024
    for s in range(3):
        X, lS_o, lS_i, T = _rand_batch(rng, rows, B, 1, c["bot"][0], c["loss"], dist="zipf")
        assert max(float((i == 0).mean()) for i in lS_i) > 0.03
        Zr, Er = ref.train_step(torch.tensor(X), torch.tensor(lS_o),
                                [torch.tensor(i) for i in lS_i], torch.tensor(T), c["lr"])
        b = tr.make_batch(X, lS_o, lS_i, T)
        if graph and s > 0:  # (the first step of a batch size runs eagerly: allocations)
            tr.capture(b)()
            Z, E = tr._cur["prob"], tr._cur["loss"]
        else:
            Z, E = tr.step(b)
        assert tr.gather_fused
        ok, msg = fp32_close(Z.cpu().numpy(), Zr.numpy().ravel())
        assert ok, (s, msg)
        ok, msg = fp32_close(E.cpu().numpy(), [Er.item()])
        assert ok, (s, msg)
    _compare_state(tr, ref)


@pytest.mark.parametrize("name,sched,optimizer,at", [
    ("c3_small", "partial", "sgd", (0, 1)), ("c3_small", "full", "sgd", (0, 1)),
    ("c2_small", "full", "sgd", (0, 1)),
    ("c2_small", "partial", "rwsadagrad", (0, 1)), ("c3_small", "partial", "rwsadagrad", (0, 1)),
    ("c3_small", "partial", "sgd", (0, 3)), ("c3_small", "partial", "sgd", (1, 2)),
    ("c2_small", "full", "sgd", (2, 9))])
@pytest.mark.parametrize("graph", [False, True])
def test_tbe_update_roles_match_own_launches(name, sched, optimizer, at, graph):
    """The embedding update's block and combine passes as extra workgroups of the first two
    bottom-backward GEMM launches (tbe_role, dlrm_gemm_f32_group_role) vs their own
    launches: 3 steps leave bitwise the same tables, momentum, dense parameters and
    predictions, under each bottom-backward schedule (chain: one GEMM launch, so the
    combine pass runs as a launch of its own), SGD and row-wise Adagrad, eager and
    replayed from a captured graph; passes placed on later launches (tbe_role_at), the
    second past the last launch (run as a launch of its own)."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function=c["loss"],
                        learning_rate=c["lr"] if optimizer == "sgd" else 1e-3,
                        optimizer=optimizer)
    B = 256
    res = []
    for role in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.tbe_role = role
        tr.tbe_role_at = at
        tr.bot_sched = sched
        batches = [tr.synthetic_batch(B, 1, seed=s) for s in range(3)]
        if graph:
            tr.step(batches[0])
            run = tr.capture(batches[0])
            for b in batches[1:]:
                for src, dst in zip((b.X, b.offsets, b.indices, b.target),
                                    (batches[0].X, batches[0].offsets, batches[0].indices,
                                     batches[0].target)):
                    dst.copy_(src)
                run()
        else:
            for b in batches:
                tr.step(b)
        torch.cuda.synchronize()
        tr.check_errors()
        assert not tr._roles  # every deferred pass ran
        mom = tr.momentum.cpu().clone() if tr.momentum is not None else None
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(), mom,
                    tr._bufs[(B, B)]["prob"].cpu().clone()))
    for a, b in zip(*res):
        assert (a is None and b is None) or torch.equal(a, b)


@pytest.mark.parametrize("name,optimizer,L", [("c3_small", "sgd", 20),
                                              ("c2_small", "rwsadagrad", 40)])
@pytest.mark.parametrize("graph", [False, True])
def test_early_sort_matches_in_backward_sort(name, optimizer, L, graph):
    """Tables past the per-table LDS sort (B * L > 4096 lookups, C1's shape): the backward's
    tiled sort on the side stream at the start of the step (early_sort, joined before the
    embedding backward) vs inside the backward - 3 steps leave bitwise the same tables,
    momentum, dense parameters and predictions, eager and replayed from a captured graph
    (the fork and join inside one graph)."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function=c["loss"],
                        learning_rate=c["lr"] if optimizer == "sgd" else 1e-3,
                        optimizer=optimizer)
    B = 256
    res = []
    for early in (False, 1, 2):  # 1: forked at the start of the step, 2: after the lookup
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.early_sort = early
        batches = [tr.synthetic_batch(B, L, seed=s) for s in range(3)]
        assert batches[0].max_per_table > 4096
        if graph:
            tr.step(batches[0])
            run = tr.capture(batches[0])
            for b in batches[1:]:
                for src, dst in zip((b.X, b.offsets, b.indices, b.target),
                                    (batches[0].X, batches[0].offsets, batches[0].indices,
                                     batches[0].target)):
                    dst.copy_(src)
                run()
        else:
            for b in batches:
                tr.step(b)
        torch.cuda.synchronize()
        tr.check_errors()
        mom = tr.momentum.cpu().clone() if tr.momentum is not None else None
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(), mom,
                    tr._bufs[(B, B)]["prob"].cpu().clone()))
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert (a is None and b is None) or torch.equal(a, b)


@pytest.mark.parametrize("name,optimizer,L", [("c3_small", "sgd", 20), ("c3_small", "sgd", 1),
                                              ("c2_small", "rwsadagrad", 1)])
@pytest.mark.parametrize("graph", [False, True])
def test_feature_pad_matches_dense_rows(name, optimizer, L, graph):
    """E / dE at a padded batch stride (feature_pad: an odd number of 256-byte chunks per
    sample) vs dense rows: 3 steps leave bitwise the same state - the lookup, the interaction
    (pooled and gather-fused), the embedding update and the early sort read and write the
    same values through the stride."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function=c["loss"],
                        learning_rate=c["lr"] if optimizer == "sgd" else 1e-3,
                        optimizer=optimizer)
    B = 256
    res = []
    for pad in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.feature_pad = pad
        batches = [tr.synthetic_batch(B, L, seed=s) for s in range(3)]
        if graph:
            tr.step(batches[0])
            run = tr.capture(batches[0])
            for b in batches[1:]:
                for src, dst in zip((b.X, b.offsets, b.indices, b.target),
                                    (batches[0].X, batches[0].offsets, batches[0].indices,
                                     batches[0].target)):
                    dst.copy_(src)
                run()
        else:
            for b in batches:
                tr.step(b)
        torch.cuda.synchronize()
        tr.check_errors()
        E = tr._bufs[(B, B)]["E"]
        assert (E.stride(0) * 4 // 256) % 2 == (1 if pad else (E.stride(0) * 4 // 256) % 2)
        mom = tr.momentum.cpu().clone() if tr.momentum is not None else None
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(), mom,
                    tr._bufs[(B, B)]["prob"].cpu().clone()))
    for a, b in zip(*res):
        assert (a is None and b is None) or torch.equal(a, b)


@pytest.mark.parametrize("name,B", [("c2_small", 128), ("c3_small", 256)])
def test_bottom_parts_split_chain_matches_single(name, B):
    """The fused bottom MLP with 2 / 4 workgroups per 16-row block (auto at these batch
    sizes) vs one: 3 steps leave bitwise the same state (same dot products, same order)."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function=c["loss"],
                        learning_rate=c["lr"])
    res = []
    for parts in (1, 2, 4):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.bottom_parts = parts
        for s in range(3):
            tr.step(tr.synthetic_batch(B, 1, seed=s))
        torch.cuda.synchronize()
        assert tr.bottom_fused
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(),
                    tr._bufs[(B, B)]["prob"].cpu().clone()))
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("name,B", [("c3_small", 512), ("c2_small", 128)])
@pytest.mark.parametrize("graph", [False, True])
def test_head_role_matches_two_launch_head(name, B, graph):
    """The head's finalize pass as a role of the top-MLP backward's first launch
    (head_role) vs its own launch: 3 steps leave bitwise the same state and loss."""
    DLRMTrainer, TrainerConfig = _trainer()
    c = CASES[name]
    D, rows = c["D"], c["rows"]
    cfg = TrainerConfig(m_spa=D, ln_emb=rows, ln_bot=c["bot"],
                        ln_top=[_num_int(len(rows), D)] + c["top"], loss_function=c["loss"],
                        learning_rate=c["lr"])
    res = []
    for role in (False, True):
        tr = DLRMTrainer(cfg, device=dev, seed=11)
        tr.head_role = role
        batches = [tr.synthetic_batch(B, 1, seed=s) for s in range(3)]
        if graph:
            tr.step(batches[0])
            run = tr.capture(batches[0])
            for b in batches[1:]:
                for src, dst in zip((b.X, b.offsets, b.indices, b.target),
                                    (batches[0].X, batches[0].offsets, batches[0].indices,
                                     batches[0].target)):
                    dst.copy_(src)
                run()
        else:
            for b in batches:
                tr.step(b)
        torch.cuda.synchronize()
        assert not tr._roles
        bufs = tr._bufs[(B, B)]
        res.append((tr.weights.cpu().clone(), tr.params.cpu().clone(),
                    bufs["prob"].cpu().clone(), bufs["loss"].cpu().clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)
