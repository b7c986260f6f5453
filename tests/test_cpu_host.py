"""Host-side logic of the product package (no GPU): C-ABI exports, sharders, batch
splits, synthetic data + CSR, DLRM_Net construction / init parity with the reference."""
import json
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "dlrm_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dlrm_[a-z0-9_]+)\s*\(", txt)))


def test_abi_library_exports_every_header_symbol():
    from dlrm_hip import _lib
    lib = _lib.load()  # loads without a GPU (HIP runtime initialises lazily)
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/dlrm_hip.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(names)
    assert lib.dlrm_abi_version() == 4


def test_abi_rejects_bad_arguments_without_gpu():
    from dlrm_hip import _lib
    with pytest.raises(_lib.DLRMHipError) as e:
        _lib.call("dlrm_gemm_f32", 0, 0, 4, 4, 4, 1.0, None, 4, None, 4, None, 4, 0, None, None,
                  0, None, 0, None)
    assert e.value.code == 1 and "null" in str(e.value)
    with pytest.raises(_lib.DLRMHipError) as e:
        _lib.call("dlrm_tbe_forward", None, 4, None, 1, 1, None, 16, None, 32, None, None, 4,
                  None, None)
    assert e.value.code == 1
    # split-bf16 planes: the pitch must hold whole 16-B chunks (checked before any launch)
    with pytest.raises(_lib.DLRMHipError) as e:
        _lib.call("dlrm_split_planes", None, 4, 7, 7, None, 7, 28, None)
    assert e.value.code == 1
    # workspace queries are pure host arithmetic
    assert _lib.query("dlrm_tbe_backward_workspace_size", 53248, 54063992, 128) > 53248 * 20
    assert _lib.query("dlrm_gemm_f32_workspace_size", 1, 0, 1024, 1024, 2048) > 0
    assert _lib.query("dlrm_gemm_f32_workspace_size", 0, 1, 2048, 1024, 1024) == 0


def test_product_sharders_match_reference():
    from dlrm_hip import sharders
    g = json.load(open(os.path.join(GOLDEN, "sharders.json")))
    for c in g["cases"]:
        assert sharders.shard(g[c["tables"]], c["W"], c["alg"]) == c["device_indices"], c


def test_product_split_helpers_match_reference():
    from dlrm_hip import extend_distributed as ed
    g = json.load(open(os.path.join(GOLDEN, "sharders.json")))
    try:
        for s in g["splits"]:
            ed.my_size, ed.my_rank = s["size"], s["rank"]
            sl = ed.get_my_slice(s["n"])
            assert [sl.start, sl.stop] == s["slice"]
            assert list(ed.get_split_lengths(s["n"])) == [s["my_len"], s["splits"]]
    finally:
        ed.my_size, ed.my_rank = -1, -1


def test_product_data_generator_and_csr(golden):
    from dlrm_hip import data
    g = golden("data.npz")
    np.random.seed(31)
    X, lS_o, lS_i = data.generate_uniform_input_batch(13, [50, 200, 1000], 6, 5, True)
    assert np.array_equal(X.numpy(), g["u_X"])
    for t in range(3):
        assert np.array_equal(lS_o[t].numpy(), g[f"u_o{t}"])
        assert np.array_equal(lS_i[t].numpy(), g[f"u_i{t}"])
    np.random.seed(32)
    assert np.array_equal(data.generate_random_output_batch(6, 1).numpy(), g["u_T"])
    off, idx = data.batched_csr([torch.tensor(g[f"p_o{t}"]) for t in range(3)],
                                [torch.tensor(g[f"p_i{t}"]) for t in range(3)])
    assert off.dtype == torch.int32 and np.array_equal(off.numpy(), g["b_offsets"])
    assert np.array_equal(idx.numpy(), g["b_indices"])


def test_dlrm_net_mirror_init_matches_reference_bit_exactly(golden):
    """The mirror draws numpy's RNG in the reference order (tables, bottom, top)."""
    from dlrm_hip.dlrm_net import DLRM_Net
    g = golden("c0_train.npz")
    np.random.seed(123)
    net = DLRM_Net(4, np.array([1000, 1000, 1000]), np.array([13, 512, 4]),
                   np.array([10, 4, 2, 1]), arch_interaction_op="dot", sigmoid_top=2,
                   loss_function="mse")
    for k in range(3):
        assert np.array_equal(net.emb_l[k].weight.detach().numpy(), g[f"init_emb{k}"])
    for pre, seq in (("bot", net.bot_l), ("top", net.top_l)):
        for name, p in seq.named_parameters():
            assert np.array_equal(p.detach().numpy(), g[f"init_{pre}.{name}"]), (pre, name)
    # state_dict keys are the reference's
    keys = set(net.state_dict().keys())
    assert {"emb_l.0.weight", "bot_l.0.weight", "bot_l.2.bias", "top_l.4.weight"} <= keys
    # tables share one flat buffer (one kernel launch for all tables)
    flat = net.emb_l.weight_flat
    assert net.emb_l[1].weight.data_ptr() == flat[1000:].data_ptr()


def test_trainer_layout_bias_folding():
    """Flat-bucket layout of the fused engine: [W | b | 0] per layer, 16-B aligned rows."""
    from dlrm_hip.trainer import _pad4
    for k in (13, 479, 512, 1024):
        kp = _pad4(k + 1)
        assert kp % 4 == 0 and kp >= k + 1


def _fake_problem(M, N, K, mode, splits):
    """A dlrm_gemm_problem with aligned placeholder pointers (host-side checks only)."""
    from dlrm_hip import _lib
    return _lib.GemmProblem(1, 0, M, N, K, 1.0, 256, M, 256, N, 256, N + 4, 0, None, None, 0,
                            N, mode, splits, 256)


def test_gemm_partial_split_counts_are_normalized_or_rejected():
    """a PARTIAL count the planner would lower (K too short for it, or over 32)
    must not reach the kernel, because its REDUCE repeats the caller's count.
    dlrm_gemm_f32_splits returns the normalized count; the launch rejects the raw one."""
    import ctypes
    from dlrm_hip import _lib, ops
    lib = _lib.load()
    for K, req, want in ((2048, 12, 11), (2048, 24, 22), (2048, 8, 8), (2048, 64, 32),
                         (96, 8, 3), (1024, 1, 1)):
        q = _fake_problem(1024, 1024, K, ops.GEMM_PARTIAL, req)
        assert lib.dlrm_gemm_f32_splits(ctypes.byref(q)) == want, (K, req)
        q.splits = want  # a normalized count maps to itself
        assert lib.dlrm_gemm_f32_splits(ctypes.byref(q)) == want
    arr = (_lib.GemmProblem * 1)(_fake_problem(1024, 1024, 2048, ops.GEMM_PARTIAL, 12))
    with pytest.raises(_lib.DLRMHipError) as e:  # rejected on the host, before any launch
        _lib.call("dlrm_gemm_f32_group", 1, ctypes.cast(arr, ctypes.c_void_p), None, 0, None)
    assert e.value.code == 1 and "normalized" in str(e.value)


def test_planes_host_api_checks_without_gpu():
    """ops.split_planes / gemm_problem plane arguments are validated on the host: device
    tensors only, bf16 [3, rows, ld] planes with unit inner stride."""
    import torch
    from dlrm_hip import ops
    with pytest.raises(ValueError, match="device tensors"):
        ops.split_planes(torch.zeros(4, 8))
    P = torch.zeros(3, 4, 8, dtype=torch.bfloat16)
    assert ops._plane_args(None) == (None, 0, 0)
    assert ops._plane_args(P) == (P.data_ptr(), 8, 32)
    with pytest.raises(ValueError, match="bf16"):
        ops._plane_args(torch.zeros(3, 4, 8))
    with pytest.raises(ValueError, match="bf16"):
        ops._plane_args(P[:2])
