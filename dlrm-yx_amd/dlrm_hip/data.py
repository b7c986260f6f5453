"""Synthetic DLRM inputs in the reference's layouts (dlrm_data_pytorch.py:596-1228).

Host generators mirror the reference's numpy draws (same global-RNG consumption order,
so a seeded run reproduces its batches); the table-batched CSR flatten has a device
variant (ops.csr_from_tables).  Device-side random batches for benchmarking live in
DLRMTrainer.synthetic_batch.
"""
from __future__ import annotations

import os
from typing import List, Sequence

import numpy as np
import torch

from . import ops


def generate_uniform_input_batch(m_den, ln_emb, n, num_indices_per_lookup,
                                 num_indices_per_lookup_fixed, rng=np.random):
    """dlrm_data_pytorch.py:1109-1161: X ~ U[0,1) [n, m_den]; per table n bags of sorted
    unique indices (fixed L: redrawn until exactly L unique — needs rows >= L)."""
    Xt = torch.tensor(rng.rand(n, m_den).astype(np.float32))
    lS_o: List[torch.Tensor] = []
    lS_i: List[torch.Tensor] = []
    for size in ln_emb:
        offs, idxs, offset = [], [], 0
        for _ in range(n):
            if num_indices_per_lookup_fixed:
                if size < num_indices_per_lookup:
                    raise ValueError("fixed L larger than the table never terminates "
                                     "(dlrm_data_pytorch.py:1134-1138)")
                group = np.int64(num_indices_per_lookup)
                while True:
                    r = rng.random(group)
                    sg = np.unique(np.round(r * (size - 1)).astype(np.int64))
                    if sg.size == num_indices_per_lookup:
                        break
            else:
                r = rng.random(1)
                group = np.int64(np.round(max([1.0], r * min(size, num_indices_per_lookup))))
                r = rng.random(group)
                sg = np.unique(np.round(r * (size - 1)).astype(np.int64))
                group = np.int32(sg.size)
            offs.append(offset)
            idxs += sg.tolist()
            offset += group
        lS_o.append(torch.tensor(offs))
        lS_i.append(torch.tensor(idxs))
    return Xt, lS_o, lS_i


def generate_random_output_batch(n, num_targets, round_targets=False, rng=np.random):
    """dlrm_data_pytorch.py:1098-1105."""
    P = rng.rand(n, num_targets).astype(np.float32)
    if round_targets:
        P = np.round(P).astype(np.float32)
    return torch.tensor(P)


def batched_csr(lS_o: Sequence[torch.Tensor], lS_i: Sequence[torch.Tensor]):
    """Table-batched flatten (dlrm_data_pytorch.py:834-843): int32 indices = cat(lS_i),
    int32 offsets [T*B+1] = cat(lS_o[t] + start[t]) ++ [total].  Runs the device kernel
    when the inputs are on the GPU, numpy otherwise."""
    if lS_o[0].is_cuda:
        counts = [int(i.numel()) for i in lS_i]
        off = ops.csr_from_tables(list(lS_o), counts, int(lS_o[0].numel()))
        return off, torch.cat([i.reshape(-1) for i in lS_i]).int()
    counts = [int(i.numel()) for i in lS_i]
    starts = np.concatenate([[0], np.cumsum(counts)])
    off = np.concatenate([np.asarray(o, dtype=np.int64) + s for o, s in zip(lS_o, starts[:-1])]
                         + [starts[-1:]])
    idx = np.concatenate([np.asarray(i, dtype=np.int64).reshape(-1) for i in lS_i])
    return torch.tensor(off.astype(np.int32)), torch.tensor(idx.astype(np.int32))


def log1p_dense(X: torch.Tensor) -> torch.Tensor:
    """The cached random path feeds log(X + 1) (dlrm_data_pytorch.py:727)."""
    return torch.log(X.to(torch.float32) + 1)


class CriteoBinDataset(torch.utils.data.Dataset):
    """Binary Criteo records, decoded on the GPU (data_loader_terabyte.py:195-252).

    Same constructor, length and item layout as the reference: item ``idx`` is the
    ``idx``-th block of ``batch_size`` int32 records [label | 13 dense | 26 sparse]
    (the last block may be short), returned as (X, lS_o, lS_i, y) exactly as
    ``_transform_features(..., flag_input_torch_tensor=True)`` returns them.  The raw block
    goes to the device once (pinned, 160 B/sample) and one ``dlrm_criteo_decode`` launch
    does the split, log(x+1), ``% max_ind_range`` and the (table-batched) CSR there.
    """

    def __init__(self, data_file, counts_file, batch_size=1, max_ind_range=-1,
                 bytes_per_feature=4, batched_or_fbgemm_emb=False, device="cuda"):
        if bytes_per_feature != 4:
            raise NotImplementedError("CriteoBinDataset: only int32 records (bytes_per_feature=4)")
        self.tar_fea, self.den_fea, self.spa_fea = 1, 13, 26
        self.tad_fea = self.tar_fea + self.den_fea
        self.tot_fea = self.tad_fea + self.spa_fea
        self.batch_size = batch_size
        self.max_ind_range = max_ind_range
        self.bytes_per_entry = bytes_per_feature * self.tot_fea * batch_size
        self.num_entries = -(-os.path.getsize(data_file) // self.bytes_per_entry)
        self.data_file = data_file
        with np.load(counts_file) as data:
            self.counts = data["counts"]
        self.m_den = 13
        self.batched_or_fbgemm_emb = batched_or_fbgemm_emb
        self.device = torch.device(device)

    def __len__(self):
        return self.num_entries

    def read_raw(self, idx: int) -> torch.Tensor:
        """The idx-th raw int32 block, host-side (the file read; no transform)."""
        with open(self.data_file, "rb") as f:
            f.seek(idx * self.bytes_per_entry, 0)
            raw = f.read(self.bytes_per_entry)
        return torch.from_numpy(np.frombuffer(raw, dtype=np.int32).copy())

    def __getitem__(self, idx):
        if idx < 0 or idx >= self.num_entries:
            raise IndexError(idx)
        rec = self.read_raw(idx)
        if self.device.type == "cuda":
            rec = rec.pin_memory().to(self.device, non_blocking=True)
        return ops.criteo_decode(rec, self.den_fea, self.spa_fea, self.max_ind_range,
                                 batched=self.batched_or_fbgemm_emb)


class RecordPipeline:
    """Overlapped input pipeline for Criteo binary records (replaces
    the reference's per-step host transform and ``.cpu()`` sync: dlrm_s_pytorch.py:1910,
    data_loader_terabyte.py:237-252).

    Three stages, each on its own resource, with ``depth`` slots in flight:
      * a reader thread fills pinned host slots straight from the file (``readinto``: one
        read per global batch, 160 B per sample, the GIL released during the read);
      * a copy stream moves a filled slot to a device slot (async H2D over PCIe) one batch
        ahead of the step that needs it;
      * ``next()`` makes the current stream wait for that copy and enqueues one
        ``dlrm_criteo_decode`` launch into the trainer's fixed record Batch (so a captured
        step graph replays on it).  Nothing on the host waits for the GPU.
    The file is read in order and, with ``loop``, wraps around (a trailing partial batch is
    skipped, as the reference's drop-last loaders do for training).
    """

    def __init__(self, data_file, batch_size, trainer, max_ind_range=-1, depth=3, loop=True,
                 n_dense=13, n_sparse=26):
        import threading
        import queue
        self.trainer = trainer
        self.B = batch_size
        self.max_ind_range = max_ind_range
        self.depth = max(2, depth)
        self.loop = loop
        self.nf = 1 + n_dense + n_sparse
        self.rec_bytes = 4 * self.nf * batch_size
        self.n_batches = os.path.getsize(data_file) // self.rec_bytes
        if self.n_batches < 1:
            raise ValueError("RecordPipeline: file holds less than one batch")
        self.data_file = data_file
        dev = trainer.dev
        n = self.nf * batch_size
        self.host = [torch.empty(n, dtype=torch.int32, pin_memory=True) for _ in range(self.depth)]
        self.devs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(self.depth)]
        self.copied = [torch.cuda.Event() for _ in range(self.depth)]
        self.consumed = [torch.cuda.Event() for _ in range(self.depth)]
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.batch = trainer.record_batch(batch_size)
        self._free = [threading.Semaphore(1) for _ in range(self.depth)]  # host slot refillable
        self._filled = queue.Queue()
        self._stop = False
        self._k = 0            # next batch next() returns
        self._issued = 0       # batches whose H2D copy has been enqueued
        self._eof = False      # the reader reached the end (loop=False): never block again
        self._err = None       # the reader's failure, re-raised by every later next()
        self._thread = threading.Thread(target=self._reader, daemon=True)
        self._thread.start()

    def _reader(self):
        try:
            self._read_loop()
        except BaseException as e:  # noqa: BLE001 - handed to next(), which raises it
            self._filled.put(e)

    def _read_loop(self):
        j = 0
        with open(self.data_file, "rb", buffering=0) as f:
            while not self._stop:
                b = j % self.n_batches
                if b == 0 and j > 0 and not self.loop:
                    self._filled.put(None)
                    return
                i = j % self.depth
                self._free[i].acquire()
                if self._stop:
                    return
                self.copied[i].synchronize()  # the slot's previous H2D copy has finished
                f.seek(b * self.rec_bytes)
                mv = memoryview(self.host[i].numpy()).cast("B")
                got = f.readinto(mv)
                if got != self.rec_bytes:
                    raise IOError(f"RecordPipeline: short read ({got} of {self.rec_bytes} B)")
                self._filled.put(i)
                j += 1

    def _issue_copy(self):
        if self._err is not None:
            raise RuntimeError("RecordPipeline: the reader thread failed") from self._err
        if self._eof:  # the reader has exited: the queue gets nothing more
            return False
        i = self._filled.get()
        if i is None:
            self._eof = True
            return False
        if isinstance(i, BaseException):
            self._err = i
            raise RuntimeError("RecordPipeline: the reader thread failed") from i
        cs = self.copy_stream
        cs.wait_event(self.consumed[i])  # the device slot's previous decode is done
        with torch.cuda.stream(cs):
            self.devs[i].copy_(self.host[i], non_blocking=True)
            self.copied[i].record(cs)
        self._free[i].release()  # the reader refills after copied[i] completes
        self._issued += 1
        return True

    def next(self):
        """The next global batch, decoded into the trainer's fixed record Batch on the current
        stream (the H2D copy of the batch after it is already in flight)."""
        while self._issued <= self._k + 1:
            if not self._issue_copy():
                if self._issued <= self._k:
                    raise StopIteration
                break
        i = self._k % self.depth
        st = torch.cuda.current_stream(self.trainer.dev)
        st.wait_event(self.copied[i])
        self.trainer.decode_into(self.devs[i], self.batch, self.max_ind_range)
        self.consumed[i].record(st)
        self._k += 1
        return self.batch

    def close(self):
        self._stop = True
        for s in self._free:
            s.release()
        self._thread.join(timeout=5)


def numpy_to_binary(input_files, output_file_path, split="train"):
    """Write day_*_reordered.npz files as int32 records [y | X_int | X_cat]
    (data_loader_terabyte.py:255-293): train concatenates every file; test / val take the
    first / second half (ceil split) of the single input file."""
    def rows(path):
        with np.load(path) as d:
            return np.concatenate([d["y"].reshape(-1, 1), d["X_int"], d["X_cat"]],
                                  axis=1).astype(np.int32)

    with open(output_file_path, "wb") as out:
        if split == "train":
            for path in input_files:
                out.write(rows(path).tobytes())
            return
        if len(input_files) != 1:
            raise ValueError("numpy_to_binary: test/val split takes exactly one input file")
        data = rows(input_files[0])
        mid = -(-data.shape[0] // 2)
        if split == "test":
            out.write(data[:mid].tobytes())
        elif split == "val":
            out.write(data[mid:].tobytes())
        else:
            raise ValueError(f"Unknown split value: {split}")
