"""Reduced-precision rows on CPU: the oracle's restatement of the
quantized lookup vs golden vectors from the reference's own quantized ops
(tests/golden/make_golden_rows.py), and the row-size query of the C-ABI."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import fp32_close

CASES = [(8, 16), (8, 64), (8, 128), (4, 16), (4, 64), (4, 128)]


@pytest.mark.parametrize("bits,D", CASES)
def test_oracle_quantized_lookup_matches_reference_ops(golden, bits, D):
    g = golden("rows.npz")
    key = f"b{bits}_D{D}"
    for t in range(len(g["rows"])):
        q, idx, off, psw = (g[f"{key}_q{t}"], g[f"{key}_idx{t}"], g[f"{key}_off{t}"],
                            g[f"{key}_psw{t}"])
        ok, msg = fp32_close(O.embedding_bag_rows(q, bits, D, idx, off), g[f"{key}_y{t}"])
        assert ok, (t, msg)
        ok, msg = fp32_close(O.embedding_bag_rows(q, bits, D, idx, off, psw), g[f"{key}_yw{t}"])
        assert ok, (t, msg)


@pytest.mark.parametrize("bits,D", CASES)
def test_prepack_layout_is_the_oracles(golden, bits, D):
    """The packed rows are the reference packer's (re-run here bit-exactly), and the
    oracle's dequantisation of them is within one quantisation step of the fp32 weights."""
    g = golden("rows.npz")
    key = f"b{bits}_D{D}"
    pack = (torch.ops.quantized.embedding_bag_4bit_prepack if bits == 4
            else torch.ops.quantized.embedding_bag_byte_prepack)
    for t in range(len(g["rows"])):
        w, q = g[f"{key}_w{t}"], g[f"{key}_q{t}"]
        assert np.array_equal(pack(torch.from_numpy(w)).numpy(), q)
        lv, sc, bi = O.dequantize_rows(q, bits, D)
        deq = lv * sc[:, None] + bi[:, None]
        step = np.maximum(sc, 1e-6)[:, None]
        assert np.all(np.abs(deq - w) <= 0.51 * step + 2e-3 * np.abs(w) + 1e-3)


def test_row_bytes_query():
    from dlrm_hip import ops
    assert ops.tbe_row_bytes(ops.ROWS_F16, 128) == 256
    assert ops.tbe_row_bytes(ops.ROWS_Q8, 128) == 136
    assert ops.tbe_row_bytes(ops.ROWS_Q4, 128) == 68
    assert ops.tbe_row_bytes(99, 128) == -1
