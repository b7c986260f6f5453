"""Criteo binary record path: numpy_to_binary, CriteoBinDataset and
the device decode (dlrm_criteo_decode) vs golden vectors from the reference's own
CriteoBinDataset / numpy_to_binary (tests/golden/make_golden_criteo.py,
data_loader_terabyte.py:83-114, 195-293)."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from conftest import GOLDEN, fp32_close

CASES = [(-1, False), (-1, True), (1000, False), (1000, True), (10000000, True)]
BATCH = 64


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(GOLDEN, "criteo_bin.npz"), allow_pickle=False))


def _items(g, mir, batched):
    rec = g["records"].reshape(-1, 40)
    n = int(g[f"len_{mir}_{int(batched)}"])
    for i in range(n):
        yield i, rec[i * BATCH:(i + 1) * BATCH], f"{mir}_{int(batched)}_{i}"


@pytest.mark.parametrize("mir,batched", CASES)
def test_oracle_transform_matches_reference(gold, mir, batched):
    for i, rec, key in _items(gold, mir, batched):
        X, o, idx, y = O.criteo_transform(rec, mir, batched)
        # log(x+1): torch's CPU log may differ by an ulp between host CPUs (vectorised libm),
        # so the dense part is held to the fp32 tolerance; the integer parts are exact
        ok, msg = fp32_close(X.numpy(), gold[f"X_{key}"])
        assert ok, (key, msg)
        assert np.array_equal(o.numpy(), gold[f"o_{key}"]) and o.dtype == torch.from_numpy(
            gold[f"o_{key}"]).dtype, key
        assert np.array_equal(idx.numpy(), gold[f"i_{key}"]), key
        assert idx.dtype == torch.from_numpy(gold[f"i_{key}"]).dtype, key
        assert np.array_equal(y.numpy(), gold[f"y_{key}"]), key


def test_numpy_to_binary_matches_reference(gold, tmp_path):
    from dlrm_hip.data import numpy_to_binary
    rec = gold["records"].reshape(-1, 40)
    day = tmp_path / "day_0_reordered.npz"
    np.savez(day, y=rec[:, 0].astype(np.int64), X_int=rec[:, 1:14].astype(np.int64),
             X_cat=rec[:, 14:].astype(np.int64))
    for split in ("train", "test", "val"):
        out = tmp_path / f"{split}.bin"
        numpy_to_binary([str(day)], str(out), split=split)
        assert np.array_equal(np.fromfile(out, dtype=np.int32), gold[f"bin_{split}"]), split
    with pytest.raises(ValueError):
        numpy_to_binary([str(day)], str(tmp_path / "x.bin"), split="bogus")


def test_dataset_length_and_blocks(gold, tmp_path):
    from dlrm_hip.data import CriteoBinDataset
    path = tmp_path / "train.bin"
    gold["records"].tofile(path)
    counts = tmp_path / "counts.npz"
    np.savez(counts, counts=np.full(26, 7))
    ds = CriteoBinDataset(str(path), str(counts), batch_size=BATCH, device="cpu")
    assert len(ds) == int(gold["len_-1_0"]) == 3
    assert list(ds.counts) == [7] * 26
    last = ds.read_raw(2).numpy()
    assert np.array_equal(last, gold["records"][2 * BATCH * 40:])
    with pytest.raises(NotImplementedError):
        CriteoBinDataset(str(path), str(counts), batch_size=BATCH, bytes_per_feature=2)


@pytest.mark.gpu
@pytest.mark.parametrize("mir,batched", CASES)
def test_device_decode_matches_reference(gold, tmp_path, mir, batched):
    from dlrm_hip.data import CriteoBinDataset
    path = tmp_path / "train.bin"
    gold["records"].tofile(path)
    counts = tmp_path / "counts.npz"
    np.savez(counts, counts=np.full(26, 10000000))
    ds = CriteoBinDataset(str(path), str(counts), batch_size=BATCH, max_ind_range=mir,
                          batched_or_fbgemm_emb=batched, device="cuda:0")
    assert len(ds) == int(gold[f"len_{mir}_{int(batched)}"])
    for i, _, key in _items(gold, mir, batched):
        X, o, idx, y = ds[i]
        assert X.is_cuda and idx.is_cuda
        ok, msg = fp32_close(X.cpu().numpy(), gold[f"X_{key}"])
        assert ok, (key, msg)
        for got, ref in ((o, gold[f"o_{key}"]), (idx, gold[f"i_{key}"]), (y, gold[f"y_{key}"])):
            assert got.dtype == torch.from_numpy(ref).dtype, key
            assert tuple(got.shape) == ref.shape, key
            assert np.array_equal(got.cpu().numpy(), ref), key


@pytest.mark.gpu
def test_device_decode_strided_dense_and_empty():
    """Decode into a caller buffer with the trainer's padded row stride (bias column kept),
    plus an empty block."""
    from dlrm_hip import ops
    rng = np.random.RandomState(5)
    rec = rng.randint(0, 1 << 24, (300, 40)).astype(np.int32)
    dense = torch.full((300, 16), 7.0, device="cuda:0")
    X, o, idx, y = ops.criteo_decode(torch.from_numpy(rec).cuda().view(-1), max_ind_range=977,
                                     batched=True, dense=dense)
    Xr, orf, ir, yr = O.criteo_transform(rec, 977, True)
    assert X.data_ptr() == dense.data_ptr()
    ok, msg = fp32_close(dense[:, :13].cpu().numpy(), Xr.numpy())
    assert ok, msg
    assert torch.equal(dense[:, 13:].cpu(), torch.full((300, 3), 7.0))
    assert torch.equal(o.cpu(), orf) and torch.equal(idx.cpu(), ir) and torch.equal(y.cpu(), yr)
    X, o, idx, y = ops.criteo_decode(torch.empty(0, dtype=torch.int32, device="cuda:0"),
                                     batched=True)
    assert X.shape == (0, 13) and o.tolist() == [0] and idx.numel() == 0


@pytest.mark.gpu
def test_trainer_batch_from_records_matches_make_batch():
    """A trainer step fed by the device decode equals one fed by make_batch on the
    reference transform of the same records (fp32 tolerance: device logf vs torch log)."""
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    rng = np.random.RandomState(17)
    B, mir = 256, 1000
    rec = rng.randint(0, 1 << 20, (B, 40)).astype(np.int32)
    rec[:, 0] = rng.randint(0, 2, B)
    cfg = TrainerConfig(m_spa=4, ln_emb=[mir] * 26, ln_bot=[13, 16, 4],
                        ln_top=[4 + 27 * 26 // 2, 8, 1], loss_function="bce",
                        learning_rate=0.1)
    out = []
    for use_records in (True, False):
        tr = DLRMTrainer(cfg, device="cuda:0", seed=3)
        if use_records:
            batch = tr.batch_from_records(torch.from_numpy(rec).cuda(), max_ind_range=mir)
        else:
            X, lS_o, lS_i, y = O.criteo_transform(rec, mir, batched=False)
            batch = tr.make_batch(X, lS_o, list(lS_i), y)
        Z, E = tr.step(batch)
        torch.cuda.synchronize()
        out.append((Z.cpu().numpy().ravel(), float(E.item()), tr.weights.cpu().numpy()))
    for a, b in zip(out[0], out[1]):
        ok, msg = fp32_close(a, b)
        assert ok, msg


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_record_pipeline_matches_batch_from_records(tmp_path, graph):
    """RecordPipeline (file -> pinned slot -> copy stream -> decode into a fixed Batch) feeds
    the same training as batch_from_records on the same blocks, bitwise: eager steps, or a
    step graph captured once on the pipeline's Batch and replayed per decoded batch.  The
    file wraps around (5 full batches + a partial one that is skipped) for 8 steps."""
    from dlrm_hip.data import RecordPipeline
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    rng = np.random.RandomState(23)
    B, mir, nb = 128, 1000, 5
    rec = rng.randint(0, 1 << 20, (B * nb + 17, 40)).astype(np.int32)
    rec[:, 0] = rng.randint(0, 2, rec.shape[0])
    path = tmp_path / "train.bin"
    rec.tofile(path)
    cfg = TrainerConfig(m_spa=4, ln_emb=[mir] * 26, ln_bot=[13, 16, 4],
                        ln_top=[4 + 27 * 26 // 2, 8, 1], loss_function="bce",
                        learning_rate=0.1)
    steps = 8
    ref = DLRMTrainer(cfg, device="cuda:0", seed=3)
    losses_ref = []
    for k in range(steps):
        blk = torch.from_numpy(rec[(k % nb) * B:(k % nb + 1) * B]).cuda()
        _, E = ref.step(ref.batch_from_records(blk, max_ind_range=mir))
        losses_ref.append(float(E.item()))
    tr = DLRMTrainer(cfg, device="cuda:0", seed=3)
    pipe = RecordPipeline(str(path), B, tr, max_ind_range=mir, depth=3)
    assert pipe.n_batches == nb
    losses = []
    try:
        if graph:
            batch = pipe.next()
            _, E = tr.step(batch)  # eager step of this batch size (allocations)
            losses.append(float(E.item()))
            run = tr.capture(batch)
            for _ in range(steps - 1):
                pipe.next()
                run()
                losses.append(float(tr._cur["loss"].item()))
        else:
            for _ in range(steps):
                _, E = tr.step(pipe.next())
                losses.append(float(E.item()))
    finally:
        pipe.close()
    torch.cuda.synchronize()
    assert losses == losses_ref
    assert torch.equal(tr.weights, ref.weights)


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [1, 3])
def test_record_pipeline_no_loop_ends_with_stop_iteration(tmp_path, nb):
    """loop=False reads the file once: every batch in order, then StopIteration on this and
    every later call - never a blocked queue (the prefetch consumed the reader's
    end marker one batch early).  Batches equal batch_from_records on the same blocks."""
    from dlrm_hip.data import RecordPipeline
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    rng = np.random.RandomState(29)
    B, mir = 64, 1000
    rec = rng.randint(0, 1 << 20, (B * nb + 5, 40)).astype(np.int32)
    rec[:, 0] = rng.randint(0, 2, rec.shape[0])
    path = tmp_path / "once.bin"
    rec.tofile(path)
    cfg = TrainerConfig(m_spa=4, ln_emb=[mir] * 26, ln_bot=[13, 16, 4],
                        ln_top=[4 + 27 * 26 // 2, 8, 1], loss_function="bce")
    tr = DLRMTrainer(cfg, device="cuda:0", seed=3)
    pipe = RecordPipeline(str(path), B, tr, max_ind_range=mir, depth=2, loop=False)
    try:
        for k in range(nb):
            got = pipe.next()
            want = tr.batch_from_records(torch.from_numpy(rec[k * B:(k + 1) * B]).cuda(),
                                         max_ind_range=mir)
            assert torch.equal(got.indices, want.indices) and torch.equal(got.X, want.X)
            assert torch.equal(got.target, want.target)
        for _ in range(3):
            with pytest.raises(StopIteration):
                pipe.next()
    finally:
        pipe.close()
