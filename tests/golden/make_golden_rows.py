"""Golden vectors for the reduced-precision embedding rows, produced
by the ops the reference itself calls for quantized inference (dlrm_s_pytorch.py:554-567,
609-625): torch.ops.quantized.embedding_bag_{byte,4bit}_prepack and
embedding_bag_{byte,4bit}_rowwise_offsets (PyTorch CPU, fbgemm kernels).

Writes tests/golden/rows.npz: per (bits, D) case, T=3 tables of fp32 weights, their packed
rows, per-table indices / bag starts (empty bags, repeated rows), per-sample weights, and
the reference op's pooled output with and without the weights.

Usage:  python tests/golden/make_golden_rows.py
"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [(8, 16), (8, 64), (8, 128), (4, 16), (4, 64), (4, 128)]
ROWS = [37, 5, 120]
B = 24


def main():
    rng = np.random.RandomState(1234)
    out = {}
    for bits, D in CASES:
        key = f"b{bits}_D{D}"
        pack = (torch.ops.quantized.embedding_bag_4bit_prepack if bits == 4
                else torch.ops.quantized.embedding_bag_byte_prepack)
        look = (torch.ops.quantized.embedding_bag_4bit_rowwise_offsets if bits == 4
                else torch.ops.quantized.embedding_bag_byte_rowwise_offsets)
        for t, n in enumerate(ROWS):
            w = rng.uniform(-1, 1, (n, D)).astype(np.float32)
            w[0] = 0.25  # a constant row (zero range)
            q = pack(torch.from_numpy(w))
            lens = rng.randint(0, 6, B)
            lens[3] = 0
            idx = rng.randint(0, n, int(lens.sum())).astype(np.int64)
            if len(idx) > 2:
                idx[1] = idx[0]  # a repeated row inside a bag
            off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            psw = rng.uniform(0.5, 2.0, len(idx)).astype(np.float32)
            y = look(q, torch.from_numpy(idx), torch.from_numpy(off)).numpy()
            yw = look(q, torch.from_numpy(idx), torch.from_numpy(off),
                      per_sample_weights=torch.from_numpy(psw)).numpy()
            out[f"{key}_w{t}"] = w
            out[f"{key}_q{t}"] = q.numpy()
            out[f"{key}_idx{t}"] = idx
            out[f"{key}_off{t}"] = off
            out[f"{key}_psw{t}"] = psw
            out[f"{key}_y{t}"] = y
            out[f"{key}_yw{t}"] = yw
    np.savez_compressed(os.path.join(HERE, "rows.npz"), rows=np.array(ROWS), B=np.array([B]),
                        **out)
    print("wrote", os.path.join(HERE, "rows.npz"))


if __name__ == "__main__":
    main()
