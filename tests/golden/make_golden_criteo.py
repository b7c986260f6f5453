"""Golden vectors for the Criteo binary record path, produced by the REFERENCE's own
CriteoBinDataset (data_loader_terabyte.py:195-252) and numpy_to_binary (:255-293).

Runs only in the build container (imports /root/reference; that module needs only numpy,
torch and tqdm, so no shims).  Writes tests/golden/criteo_bin.npz: the raw int32 records
(2.5 batches of 64, so the last item is ragged) and, for every (max_ind_range, batched)
case and item, the reference's (X, lS_o, lS_i, y).

Usage:  python tests/golden/make_golden_criteo.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BATCH = 64
N = 160
CASES = [(-1, False), (-1, True), (1000, False), (1000, True), (10000000, True)]


def make_npz_day(path: str, rng) -> None:
    """A synthetic day_*_reordered.npz: y, X_int (>= 0, incl. 0 and large), X_cat (incl.
    negatives and values >= max_ind_range so the floor mod is exercised)."""
    y = rng.randint(0, 2, N)
    x_int = rng.randint(0, 1 << 20, (N, 13))
    x_int[::7, 3] = 0
    x_int[::11, 5] = (1 << 31) - 1
    x_cat = rng.randint(-(1 << 31), (1 << 31) - 1, (N, 26), dtype=np.int64)
    x_cat[::3] = rng.randint(0, 5000, (len(x_cat[::3]), 26))
    np.savez(path, y=y, X_int=x_int, X_cat=x_cat)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    import data_loader_terabyte as dlt  # the reference module

    rng = np.random.RandomState(4242)
    tmp = tempfile.mkdtemp(prefix="criteo_golden_")
    day = os.path.join(tmp, "day_0_reordered.npz")
    make_npz_day(day, rng)
    out = {}
    for split in ("train", "test", "val"):
        path = os.path.join(tmp, f"bin_{split}.bin")
        dlt.numpy_to_binary([day], path, split=split)
        out[f"bin_{split}"] = np.fromfile(path, dtype=np.int32)
    counts = os.path.join(tmp, "counts.npz")
    np.savez(counts, counts=np.full(26, 10000000))
    out["records"] = out["bin_train"]
    for mir, batched in CASES:
        ds = dlt.CriteoBinDataset(os.path.join(tmp, "bin_train.bin"), counts, batch_size=BATCH,
                                  max_ind_range=mir, batched_or_fbgemm_emb=batched)
        out[f"len_{mir}_{int(batched)}"] = np.array(len(ds))
        for i in range(len(ds)):
            X, lS_o, lS_i, y = ds[i]
            key = f"{mir}_{int(batched)}_{i}"
            out[f"X_{key}"] = X.numpy()
            out[f"o_{key}"] = lS_o.numpy()
            out[f"i_{key}"] = lS_i.numpy()
            out[f"y_{key}"] = y.numpy()
    np.savez_compressed(os.path.join(HERE, "criteo_bin.npz"), **out)
    print("wrote", os.path.join(HERE, "criteo_bin.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
