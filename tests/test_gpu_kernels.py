"""HIP kernels (through the C-ABI) vs the oracle / golden fixtures, on the GPU."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import fp32_close

pytestmark = pytest.mark.gpu

dev = "cuda:0"


@pytest.fixture(scope="module")
def ops():
    from dlrm_hip import ops as _ops
    return _ops


def _csr_from_golden(g, idx_dtype=torch.int32):
    T = len(g["rows"])
    lo = [torch.tensor(g[f"lS_o{t}"]) for t in range(T)]
    li = [torch.tensor(g[f"lS_i{t}"]) for t in range(T)]
    off, idx = O.batched_csr(lo, li)
    rows = [int(r) for r in g["rows"]]
    row_base = torch.tensor(np.concatenate([[0], np.cumsum(rows)]), dtype=torch.int64)
    W = torch.cat([torch.tensor(g[f"w0_{t}"]) for t in range(T)], 0)
    return off, idx.to(idx_dtype), row_base, W, rows


@pytest.mark.parametrize("D", [4, 16, 64, 128])
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
def test_tbe_forward_golden(ops, golden, D, idx_dtype):
    g = golden(f"tbe_D{D}.npz")
    off, idx, row_base, W, rows = _csr_from_golden(g, idx_dtype)
    T, B = len(rows), int(g["B"][0])
    out = ops.tbe_forward(W.to(dev), row_base.to(dev), T, B, idx.to(dev),
                          off.to(dev, idx_dtype)).cpu()
    for t in range(T):  # sequential fp32 sum in lookup order == CPU EmbeddingBag
        ok, msg = fp32_close(out[:, t].numpy(), g[f"out{t}"])
        assert ok, (t, msg)


@pytest.mark.parametrize("D", [4, 16, 64, 128])
@pytest.mark.parametrize("per_table_sort", [False, True])
def test_tbe_backward_sgd_golden(ops, golden, D, per_table_sort):
    g = golden(f"tbe_D{D}.npz")
    off, idx, row_base, W, rows = _csr_from_golden(g)
    T, B = len(rows), int(g["B"][0])
    grad = torch.stack([torch.tensor(g[f"g{t}"]) for t in range(T)], 1)  # [B, T, D]
    Wd = W.to(dev)
    seg = off[::B].long()
    mx = int((seg[1:] - seg[:-1]).max()) if per_table_sort else 0
    ops.tbe_backward("sgd", Wd, row_base.to(dev), T, B, idx.to(dev), off.to(dev), grad.to(dev),
                     lr=0.1, max_lookups_per_table=mx)
    W1 = Wd.cpu().split(rows, 0)
    for t in range(T):
        ok, msg = fp32_close(W1[t].numpy(), g[f"w1_{t}"])
        assert ok, (t, msg)


def test_tbe_weighted_and_dense_grad(ops):
    torch.manual_seed(0)
    rows, D, B = [300, 7, 50], 32, 24
    T = len(rows)
    W = torch.randn(sum(rows), D)
    lo, li = [], []
    for n in rows:
        lens = torch.randint(0, 9, (B,))
        lo.append(torch.cat([torch.zeros(1, dtype=torch.int64), lens.cumsum(0)[:-1]]))
        li.append(torch.randint(0, n, (int(lens.sum()),)))
    off, idx = O.batched_csr(lo, li)
    psw = torch.rand(idx.numel())
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64)
    out = ops.tbe_forward(W.to(dev), row_base.to(dev), T, B, idx.to(dev), off.to(dev),
                          per_sample_weights=psw.to(dev)).cpu()
    Ws = W.split(rows, 0)
    pw = psw.split([x.numel() for x in li])
    for t in range(T):
        ref = torch.nn.functional.embedding_bag(li[t], Ws[t], lo[t], mode="sum",
                                                per_sample_weights=pw[t])
        ok, msg = fp32_close(out[:, t].numpy(), ref.numpy())
        assert ok, msg
    # dense gradient accumulation == index_add of the expanded per-lookup grads
    G = torch.randn(B, T, D)
    gw = torch.zeros_like(W).to(dev)
    ops.tbe_backward("dense", gw, row_base.to(dev), T, B, idx.to(dev), off.to(dev), G.to(dev),
                     per_sample_weights=psw.to(dev))
    ref = torch.zeros_like(W)
    for t in range(T):
        Wt = Ws[t].clone().requires_grad_(True)
        y = torch.nn.functional.embedding_bag(li[t], Wt, lo[t], mode="sum",
                                              per_sample_weights=pw[t])
        (y * G[:, t]).sum().backward()
        ref[row_base[t]:row_base[t + 1]] = Wt.grad
    ok, msg = fp32_close(gw.cpu().numpy(), ref.numpy())
    assert ok, msg
    vals = ops.tbe_expand_grad(D, T, B, off.to(dev), idx.numel(), G.to(dev),
                               per_sample_weights=psw.to(dev)).cpu()
    bag = torch.repeat_interleave(torch.arange(T * B), off[1:] - off[:-1])
    ref_vals = G.permute(1, 0, 2).reshape(T * B, D)[bag] * psw[:, None]
    ok, msg = fp32_close(vals.numpy(), ref_vals.numpy())
    assert ok, msg


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad", "dense"])
@pytest.mark.parametrize("invalid", [False, True])
@pytest.mark.parametrize("B,L", [(512, 2), (100, 1), (256, 2)])
def test_tbe_backward_per_table_sort_vs_global_sort(ops, mode, invalid, B, L):
    """The per-table LDS sort and the device-wide radix sort order lookups by (row, position)
    alike: with all indices valid the updates are bitwise identical.  Out-of-range indices
    (skipped) sit at a different place in the two sorted arrays, which shifts the fixed
    16-lookup reduction blocks; both then still match the reference within fp32 tolerance.
    Skewed tables (3 rows, ~340 lookups per row) exercise runs spanning many blocks.  100
    and 512 lookups per table take the per-table rank sort (<= 512), 1024 the radix passes."""
    torch.manual_seed(7)
    rows, D = [3, 5000, 4, 700, 1], 64
    T = len(rows)
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    if invalid:
        li[1][5] = 999999  # out of range
    off, idx = O.batched_csr(lo, li)
    if invalid:
        idx = torch.cat([idx, torch.tensor([1, 2], dtype=torch.int32)])  # outside every bag
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    G = torch.randn(B, T, D, device=dev)
    W0 = torch.randn(sum(rows), D, device=dev)
    mom0 = torch.rand(sum(rows), device=dev)
    res = []
    for mx in (0, B * L):
        W = W0.clone() if mode != "dense" else torch.zeros_like(W0)
        mom = mom0.clone()
        ops.tbe_backward(mode, W, row_base, T, B, idx.to(dev), off.to(dev), G, lr=0.3, eps=1e-8,
                         momentum=mom, max_lookups_per_table=mx)
        res.append((W.cpu(), mom.cpu()))
    if not invalid:
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    # reference coalesced gradient
    gsum = torch.zeros(sum(rows), D, dtype=torch.float64)
    gt = G.cpu().double()
    for t in range(T):
        r = li[t]
        ok_ = r < rows[t]
        bag = torch.arange(B * L) // L
        gsum.index_add_(0, (int(row_base[t]) + r[ok_]), gt[bag[ok_], t])
    if mode == "dense":
        ref = gsum
    elif mode == "sgd":
        ref = W0.cpu().double() - 0.3 * gsum
    else:
        touched = gsum.abs().sum(1) > 0
        m = mom0.cpu().double() + torch.where(touched, (gsum ** 2).mean(1), torch.zeros(1, dtype=torch.float64))
        ref = W0.cpu().double() - 0.3 * gsum / (m.sqrt()[:, None] + 1e-8)
    for W, _ in res:
        ok, msg = fp32_close(W.numpy(), ref.numpy())
        assert ok, msg


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad", "dense"])
@pytest.mark.parametrize("invalid", [False, True])
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("mx_kind", ["cap", "none"])
def test_tbe_forward_presort_matches_separate_sort(ops, mode, invalid, idx_dtype, mx_kind):
    """dlrm_tbe_forward_presort (gather + the backward's per-table sort in one launch)
    followed by the backward with presorted=1 is bitwise identical to tbe_forward + the
    self-sorting backward; with no per-table bound (mx 0) presort degrades to the plain
    forward and the backward sorts itself."""
    torch.manual_seed(11)
    rows, D, B, L = [3, 5000, 4, 700, 1, 90000], 64, 512, 3
    T = len(rows)
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    if invalid:
        li[1][5] = 999999
    off, idx = O.batched_csr(lo, li)
    idx, off = idx.to(idx_dtype).to(dev), off.to(dev)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    G = torch.randn(B, T, D, device=dev)
    W0 = torch.randn(sum(rows), D, device=dev)
    mom0 = torch.rand(sum(rows), device=dev)
    psw = torch.rand(idx.numel(), device=dev) if mode == "dense" else None
    mx = B * L if mx_kind == "cap" else 0
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D),
                     dtype=torch.uint8, device=dev)
    res = []
    for pre in (False, True):
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        ws.zero_()
        if pre:
            out = ops.tbe_forward_presort(W0, row_base, T, B, idx, off, ws, mx,
                                          per_sample_weights=psw, error_flag=flag)
        else:
            out = ops.tbe_forward(W0, row_base, T, B, idx, off, per_sample_weights=psw,
                                  error_flag=flag)
        W = W0.clone() if mode != "dense" else torch.zeros_like(W0)
        mom = mom0.clone()
        ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8, momentum=mom,
                         per_sample_weights=psw, workspace=ws, max_lookups_per_table=mx,
                         error_flag=flag, presorted=pre)
        res.append((out.cpu(), W.cpu(), mom.cpu(), flag.item()))
    (o0, w0, m0, f0), (o1, w1, m1, f1) = res
    assert torch.equal(o0, o1)
    assert torch.equal(w0, w1) and torch.equal(m0, m1)
    assert f0 == f1 == (ops.TBE_ERR_INDEX if invalid else 0)


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
@pytest.mark.parametrize("invalid", [False, True])
@pytest.mark.parametrize("with_bottom", [False, True])
def test_tbe_presort_sort_only_matches_separate_sort(ops, mode, invalid, with_bottom):
    """The sort-only presort launch (C-ABI out = NULL, ops lookup=False: the lookup is left
    to the gather-fused interaction) followed by tbe_backward(presorted=True) applies the
    same update, bit for bit, as the self-sorting backward; it writes no pooled output
    and (with a bottom chain) the chain's output equals dlrm_mlp_chain_forward's."""
    torch.manual_seed(12)
    rows, D, B = [3, 5000, 4, 700, 1, 90000, 17], 128, 1024
    T = len(rows)
    lo = [torch.arange(B) for _ in rows]
    li = [torch.randint(0, n, (B,)) for n in rows]
    if invalid:
        li[2][9] = 77
    off, idx = O.batched_csr(lo, li)
    idx, off = idx.to(torch.int32).to(dev), off.to(torch.int32).to(dev)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    G = torch.randn(B, T, D, device=dev)
    W0 = torch.randn(sum(rows), D, device=dev)
    mom0 = torch.rand(sum(rows), device=dev)
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D),
                     dtype=torch.uint8, device=dev)
    chain = layers = layers2 = None
    if with_bottom:
        X, layers = _mlp_setup(B, [13, 512, 256, 128])
        layers2 = [(w, y.clone(), k) for w, y, k in layers]
        chain = ops.mlp_chain(X, layers)
        ops.mlp_chain_forward(ops.mlp_chain(X.clone(), layers2))
    res = []
    for pre in (False, True):
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        ws.zero_()
        if pre:
            r = ops.tbe_forward_presort(W0, row_base, T, B, idx, off, ws, B, error_flag=flag,
                                        bottom=chain, lookup=False)
            assert r is None
        W = W0.clone()
        mom = mom0.clone()
        ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8, momentum=mom,
                         workspace=ws, max_lookups_per_table=B, error_flag=flag, presorted=pre)
        res.append((W.cpu(), mom.cpu(), flag.item()))
    (w0, m0, f0), (w1, m1, f1) = res
    assert torch.equal(w0, w1) and torch.equal(m0, m1)
    assert f0 == f1 == (ops.TBE_ERR_INDEX if invalid else 0)
    if with_bottom:
        torch.cuda.synchronize()
        for (_, y1, _), (_, y2, _) in zip(layers, layers2):
            assert torch.equal(y1, y2)


def test_tbe_presort_sort_only_rejected_without_per_table_bound(ops):
    """out = NULL needs the per-table sort: with no lookup bound the library refuses
    (DLRM_ERR_UNSUPPORTED) instead of silently running a lookup into nothing."""
    rows, D, B = [10, 20], 16, 8
    off = torch.arange(0, 2 * B + 1, dtype=torch.int32, device=dev)
    idx = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    row_base = torch.tensor([0, 10, 30], dtype=torch.int64, device=dev)
    W = torch.randn(30, D, device=dev)
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), 30, D), dtype=torch.uint8,
                     device=dev)
    with pytest.raises(Exception, match="needs the per-table sort"):
        ops.tbe_forward_presort(W, row_base, 2, B, idx, off, ws, 0, lookup=False)


def test_tbe_out_of_range_flag(ops):
    W = torch.randn(10, 8, device=dev)
    row_base = torch.tensor([0, 10], dtype=torch.int64, device=dev)
    off = torch.tensor([0, 2, 3], dtype=torch.int32, device=dev)
    idx = torch.tensor([1, 12, 3], dtype=torch.int32, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = ops.tbe_forward(W, row_base, 1, 2, idx, off, error_flag=flag)
    assert flag.item() == 1
    assert torch.allclose(out[0, 0], W[1]) and torch.allclose(out[1, 0], W[3])


def test_tbe_rowwise_adagrad_matches_oracle(ops):
    torch.manual_seed(1)
    rows, D, B = [40, 3], 16, 10
    T = len(rows)
    W = torch.randn(sum(rows), D)
    lo, li = [], []
    for n in rows:
        lens = torch.randint(0, 6, (B,))
        lo.append(torch.cat([torch.zeros(1, dtype=torch.int64), lens.cumsum(0)[:-1]]))
        li.append(torch.randint(0, n, (int(lens.sum()),)))
    off, idx = O.batched_csr(lo, li)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64)
    mom = torch.zeros(sum(rows))
    Wd, md = W.to(dev), mom.to(dev)
    ref_params = [torch.nn.Parameter(w.clone()) for w in W.split(rows, 0)]
    opt = O.RWSAdagradOracle(ref_params, lr=0.05)
    for step in range(3):
        G = torch.randn(B, T, D)
        ops.tbe_backward("rowwise_adagrad", Wd, row_base.to(dev), T, B, idx.to(dev), off.to(dev),
                         G.to(dev), lr=0.05, eps=1e-10, momentum=md)
        opt.zero_grad()
        for t in range(T):
            y = torch.nn.functional.embedding_bag(li[t], ref_params[t], lo[t], mode="sum",
                                                  sparse=True)
            (y * G[:, t]).sum().backward()
        opt.step()
        ok, msg = fp32_close(Wd.cpu().numpy(), torch.cat([p.data for p in ref_params]).numpy())
        assert ok, (step, msg)


@pytest.mark.parametrize("case", ["F4_D4_s0", "F9_D64_s0", "F27_D128_s0", "F27_D16_s0",
                                  "F9_D64_s1", "F27_D128_s1"])
def test_interaction_golden(ops, golden, case):
    g = golden(f"interact_{case}.npz")
    itself = bool(g["itself"][0])
    x = torch.tensor(g["x"]).to(dev)
    ly = torch.tensor(g["ly"]).to(dev)  # [B, T, D]
    R = ops.interact_forward("dot", x, ly, itself).cpu()
    ok, msg = fp32_close(R.numpy(), g["R"])
    assert ok, msg
    gx, gly = ops.interact_backward("dot", x, ly, torch.tensor(g["g"]).to(dev), itself)
    ok, msg = fp32_close(gx.cpu().numpy(), g["gx"])
    assert ok, msg
    ok, msg = fp32_close(gly.cpu().numpy(), g["gly"])
    assert ok, msg
    # list-of-[B, D] layout (the reference's apply_emb output) through the same kernel
    lyl = [ly[:, t].contiguous() for t in range(ly.shape[1])]
    R2 = ops.interact_forward("dot", x, lyl, itself).cpu()
    assert torch.equal(R2, R)


def test_interaction_large_F_generic_path(ops):
    torch.manual_seed(2)
    B, T, D = 5, 40, 8  # F = 41 > 32 -> VALU path
    x, ly = torch.randn(B, D), torch.randn(B, T, D)
    ref_x, ref_ly = x.clone().requires_grad_(True), ly.clone().requires_grad_(True)
    R_ref = O.interact(ref_x, list(ref_ly.unbind(1)), "dot", False)
    R = ops.interact_forward("dot", x.to(dev), ly.to(dev)).cpu()
    ok, msg = fp32_close(R.numpy(), R_ref.detach().numpy())
    assert ok, msg
    gR = torch.randn_like(R)
    (R_ref * gR).sum().backward()
    gx, gly = ops.interact_backward("dot", x.to(dev), ly.to(dev), gR.to(dev))
    ok, msg = fp32_close(gly.cpu().numpy(), ref_ly.grad.numpy())
    assert ok, msg
    ok, msg = fp32_close(gx.cpu().numpy(), ref_x.grad.numpy())
    assert ok, msg


def test_interaction_cat(ops, golden):
    g = golden("interact_cat.npz")
    R = ops.interact_forward("cat", torch.tensor(g["x"]).to(dev), torch.tensor(g["ly"]).to(dev))
    assert np.array_equal(R.cpu().numpy(), g["R"])


def gemm_close(C, ref, absprod, K):
    """fp32 GEMM error bound vs an fp64 reference: |C - ref| <= 1e-5*max(1,|ref|) +
    2*K*u*(|A||B|), u = 2^-24 (the deterministic dot-product bound gamma_K)."""
    C, ref, absprod = (np.asarray(x, dtype=np.float64) for x in (C, ref, absprod))
    tol = 1e-5 * np.maximum(1.0, np.abs(ref)) + 2.0 * K * 2.0 ** -24 * absprod
    bad = np.abs(C - ref) > tol
    if bad.any():
        i = np.unravel_index(np.argmax(np.abs(C - ref) - tol), C.shape)
        return False, f"at {i}: got {C[i]!r} ref {ref[i]!r} tol {tol[i]!r} ({bad.sum()} bad)"
    return True, ""


GEMM_SHAPES = [(2048, 1024, 479), (64, 64, 64), (100, 37, 13), (2, 4, 10), (1000, 1, 256),
               (256, 512, 2048), (33, 129, 67)]


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_vs_fp64(ops, M, N, K, ta, tb):
    """The exact-f32 MFMA GEMM within the fp32 dot-product bound of an fp64 product."""
    torch.manual_seed(M + N + K)
    A = torch.randn(K, M) if ta else torch.randn(M, K)
    Bm = torch.randn(N, K) if tb else torch.randn(K, N)
    opA = A.double().t() if ta else A.double()
    opB = Bm.double().t() if tb else Bm.double()
    ref = opA @ opB
    C = ops.gemm(A.to(dev), Bm.to(dev), bool(ta), bool(tb)).cpu()
    ok, msg = gemm_close(C.numpy(), ref.numpy(), (opA.abs() @ opB.abs()).numpy(), K)
    assert ok, msg


# workgroup tiles the planner can pick (dlrm_set_tuning DLRM_TUNE_GEMM_TILE = BM*1000 + BN)
GEMM_CFGS = [64064, 128064, 64128, 64032, 32064, 32032]


@pytest.mark.parametrize("cfg", GEMM_CFGS)
def test_gemm_every_kernel_config(ops, cfg):
    """Every tile instantiation the planner can pick, forced via the tuning override
    (ops.tuning / dlrm_set_tuning), on ragged shapes in all four operand layouts, with and
    without split-K."""
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)  # split-K tickets start at 0
    for (M, N, K) in [(130, 70, 300), (64, 128, 256), (3, 5, 1030)]:
        for ta, tb in [(0, 1), (0, 0), (1, 0), (1, 1)]:
            for split in (1, 3, 7):
                torch.manual_seed(M * 7 + N + K + ta * 3 + tb)
                A = torch.randn(K, M) if ta else torch.randn(M, K)
                Bm = torch.randn(N, K) if tb else torch.randn(K, N)
                opA = A.double().t() if ta else A.double()
                opB = Bm.double().t() if tb else Bm.double()
                with ops.tuning(gemm_tile=cfg, gemm_split=split):
                    C = ops.gemm(A.to(dev), Bm.to(dev), bool(ta), bool(tb), workspace=ws).cpu()
                ok, msg = gemm_close(C.numpy(), (opA @ opB).numpy(),
                                     (opA.abs() @ opB.abs()).numpy(), K)
                assert ok, (cfg, M, N, K, ta, tb, split, msg)


def test_gemm_epilogues(ops):
    torch.manual_seed(3)
    M, N, K = 300, 200, 130
    X, W, b = torch.randn(M, K), torch.randn(N, K), torch.randn(N)
    ref = X.double() @ W.double().t() + b.double()
    Y = ops.gemm(X.to(dev), W.to(dev), False, True, epilogue=ops.EPI_BIAS_RELU, bias=b.to(dev))
    ap = X.double().abs() @ W.double().abs().t() + b.double().abs()
    ok, msg = gemm_close(Y.cpu().numpy(), ref.clamp_min(0).numpy(), ap.numpy(), K)
    assert ok, msg
    aux = torch.randn(M, N)
    dY = torch.randn(M, K)
    ref = (dY.double() @ W.double().t()) * (aux > 0)
    Z = ops.gemm(dY.to(dev), W.to(dev), False, True, epilogue=ops.EPI_DRELU, aux=aux.to(dev))
    ap = dY.double().abs() @ W.double().abs().t()
    ok, msg = gemm_close(Z.cpu().numpy(), ref.numpy(), ap.numpy(), K)
    assert ok, msg
    P = torch.randn(N, K)
    Pd = P.to(dev)
    G = torch.randn(M, N)
    ops.gemm(G.to(dev), X.to(dev), True, False, C=Pd, alpha=0.1, epilogue=ops.EPI_SGD)
    ap = P.double().abs() + 0.1 * (G.double().abs().t() @ X.double().abs())
    ok, msg = gemm_close(Pd.cpu().numpy(), (P.double() - 0.1 * (G.double().t() @ X.double())).numpy(),
                         ap.numpy(), M)
    assert ok, msg


def test_colsum_head_outer(ops):
    torch.manual_seed(4)
    M, N = 2048, 300
    Y, s = torch.randn(M, N), torch.randn(M)
    out = torch.empty(N, device=dev)
    ops.colsum(Y.to(dev), out=out)
    ok, msg = gemm_close(out.cpu().numpy(), Y.double().sum(0).numpy(),
                         Y.double().abs().sum(0).numpy(), M)
    assert ok, msg
    ops.colsum(Y.to(dev), scale=s.to(dev), out=out)
    sy = s.double()[:, None] * Y.double()
    ok, msg = gemm_close(out.cpu().numpy(), sy.sum(0).numpy(), sy.abs().sum(0).numpy(), M)
    assert ok, msg
    K = 256
    X, w, b = torch.randn(M, K).relu(), torch.randn(K) * 0.1, torch.randn(1)
    t = torch.rand(M)
    for loss in ("mse", "bce"):
        prob = torch.empty(M, device=dev)
        dz = torch.empty(M, device=dev)
        L = torch.empty(1, device=dev)
        ops.head_forward_backward(X.to(dev), w.to(dev), b.to(dev), t.to(dev), loss, prob=prob,
                                  dz=dz, loss_out=L)
        Xr = X.clone()
        wr = w.clone().requires_grad_(True)
        z = Xr @ wr + b
        z.retain_grad()
        p = torch.sigmoid(z)
        fn = torch.nn.MSELoss() if loss == "mse" else torch.nn.BCELoss()
        E = fn(p, t)
        E.backward()
        ok, msg = fp32_close(prob.cpu().numpy(), p.detach().numpy())
        assert ok, msg
        ok, msg = fp32_close(L.cpu().numpy(), [E.item()])
        assert ok, msg
        ok, msg = fp32_close(dz.cpu().numpy(), z.grad.numpy())
        assert ok, msg
    dX = ops.outer_drelu(dz, w.to(dev), X.to(dev), True).cpu()
    ref = dz.cpu()[:, None] * w[None, :] * (X > 0)
    ok, msg = fp32_close(dX.numpy(), ref.numpy())
    assert ok, msg


@pytest.mark.parametrize("loss,clamp", [("mse", 0.0), ("bce", 0.0), ("bce", 0.2)])
@pytest.mark.parametrize("M,K", [(2048, 260), (37, 13), (100, 700)])
def test_head_step_fused(ops, loss, clamp, M, K):
    """dlrm_head_step (bias folded into X's last column) vs torch autograd: prob, loss, dz,
    the ReLU-masked input gradient, and the weight gradient (stored and as fused SGD)."""
    torch.manual_seed(M + K)
    X = torch.randn(M, K).relu()
    X[:, K - 1] = 1.0  # folded bias column
    w = torch.randn(K) * 0.1
    t = torch.rand(M).round() if loss == "bce" else torch.rand(M)
    Xr = X.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    z = Xr @ wr
    z.retain_grad()
    p = torch.sigmoid(z)
    pc = p.clamp(clamp, 1 - clamp) if clamp > 0 else p
    fn = torch.nn.MSELoss() if loss == "mse" else torch.nn.BCELoss()
    E = fn(pc, t)
    E.backward()
    Xd, wd, td = X.to(dev), w.to(dev), t.to(dev)
    prob, dz, L = (torch.empty(M, device=dev), torch.empty(M, device=dev),
                   torch.empty(1, device=dev))
    dX = torch.full((M, K + 3), 7.0, device=dev)
    dw = torch.empty(K, device=dev)
    ops.head_step(Xd, wd, td, loss, clamp, 1.0, prob=prob, dz=dz, loss_out=L, dX=dX[:, :K],
                  relu_mask=True, dw=dw)
    for got, ref in ((prob, pc.detach()), (L, E.detach().reshape(1)), (dz, z.grad),
                     (dw, wr.grad)):
        ok, msg = fp32_close(got.cpu().numpy(), ref.numpy())
        assert ok, msg
    ref_dx = dz.cpu()[:, None] * w[None, :] * (X > 0)
    ok, msg = fp32_close(dX[:, :K].cpu().numpy(), ref_dx.numpy())
    assert ok, msg
    assert torch.all(dX[:, K:] == 7.0)
    w2 = w.to(dev)
    ops.head_step(Xd, w2, td, loss, clamp, 1.0, dX=None, lr=0.5)
    ok, msg = fp32_close(w2.cpu().numpy(), (w - 0.5 * wr.grad).numpy())
    assert ok, msg


@pytest.mark.parametrize("M,K", [(2048, 260), (37, 13), (128, 260)])
@pytest.mark.parametrize("sgd", [True, False])
def test_head_step_deferred_into_gemm_launch(ops, M, K, sgd):
    """dlrm_head_step_defer + its finalize pass as pass 4 of a grouped GEMM launch (or of an
    otherwise empty one): prob, dz, dX, the loss and the weight update / gradient bitwise
    the two-launch dlrm_head_step's; the GEMM result bitwise the plain launch's."""
    torch.manual_seed(M + K)
    X = torch.randn(M, K, device=dev).relu()
    X[:, K - 1] = 1.0
    w0 = torch.randn(K, device=dev) * 0.1
    t = torch.rand(M, device=dev).round()
    A1, B1 = torch.randn(300, 260, device=dev), torch.randn(260, 512, device=dev)
    res = []
    for defer in (False, True):
        w = w0.clone()
        prob, dz, L = (torch.empty(M, device=dev), torch.empty(M, device=dev),
                       torch.empty(1, device=dev))
        dX = torch.empty(M, K, device=dev)
        dw = None if sgd else torch.full((K,), 0.25, device=dev)
        kw = dict(prob=prob, dz=dz, loss_out=L, dX=dX, relu_mask=True, dw=dw,
                  accumulate=not sgd, lr=0.5 if sgd else 0.0)
        p1, c1 = ops.gemm_problem(A1, B1)
        if defer:
            role = ops.head_step(X, w, t, "bce", 0.0, 1.0, defer=True, **kw)
            assert ops.role_blocks(role) % 8 == 0 and ops.role_blocks(role) * 4 >= K
            ops.gemm_group([p1] if M != 37 else [], None, dev, role=role, phase=4)
            if M == 37:
                ops.gemm_group([p1], None, dev)
        else:
            ops.head_step(X, w, t, "bce", 0.0, 1.0, **kw)
            ops.gemm_group([p1], None, dev)
        torch.cuda.synchronize()
        res.append([v.cpu() for v in (w, prob, dz, L, dX, c1)] + ([dw.cpu()] if dw is not None else []))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_gemm_group_role_phase_must_match_the_role(ops):
    """A role used with another kind's phase (an update role as pass 3 / 4, a head role
    as pass 1) is refused (INVALID_ARG) before anything is launched."""
    from dlrm_hip import _lib
    X = torch.rand(64, 20, device=dev)
    role = ops.head_step(X, torch.rand(20, device=dev), torch.rand(64, device=dev), "mse",
                         defer=True, lr=0.1)
    for ph in (1, 2, 3):
        with pytest.raises(_lib.DLRMHipError):
            ops.gemm_group([], None, dev, role=role, phase=ph)
    ops.gemm_group([], None, dev, role=role, phase=4)
    torch.cuda.synchronize()


def test_dense_optimizers(ops):
    torch.manual_seed(5)
    p, g = torch.randn(1000), torch.randn(1000)
    pd = p.to(dev)
    ops.sgd_update(pd, g.to(dev), 0.1)
    ok, msg = fp32_close(pd.cpu().numpy(), (p - 0.1 * g).numpy())
    assert ok, msg
    s = torch.rand(1000)
    pd, sd = p.to(dev), s.to(dev)
    ops.adagrad_update(pd, g.to(dev), sd, 0.05, 1e-10)
    s_ref = s + g * g
    ok, msg = fp32_close(pd.cpu().numpy(), (p - 0.05 * g / (s_ref.sqrt() + 1e-10)).numpy())
    assert ok, msg


@pytest.mark.parametrize("scale", [0.125, 1.0 / 3.0])
def test_adagrad_update_scaled_is_scale_then_update_bitwise(ops, scale):
    """dlrm_adagrad_update_scaled (ABI v9, the W-rank dense step with 1/W folded in) gives
    bitwise the two-pass form dlrm_scale_f32 + dlrm_adagrad_update, and leaves grad alone."""
    torch.manual_seed(6)
    p, g, s = torch.randn(4099), torch.randn(4099), torch.rand(4099)
    pa, ga, sa = p.to(dev), g.to(dev), s.to(dev)
    ops.scale_(ga, scale)
    ops.adagrad_update(pa, ga, sa, 0.05, 1e-8)
    pb, gb, sb = p.to(dev), g.to(dev), s.to(dev)
    ops.adagrad_update(pb, gb, sb, 0.05, 1e-8, grad_scale=scale)
    torch.cuda.synchronize()
    assert torch.equal(pa, pb) and torch.equal(sa, sb)
    assert torch.equal(gb.cpu(), g)


def test_qr_split_and_combine(ops, golden):
    g = golden("qr.npz")
    q, r = ops.qr_split_indices(torch.tensor(g["split_idx"]).to(dev), 3)
    assert np.array_equal(q.cpu().numpy(), g["split_q3"])
    assert np.array_equal(r.cpu().numpy(), g["split_r3"])
    eq, er = torch.randn(6, 4, device=dev), torch.randn(6, 4, device=dev)
    for op in ("mult", "add", "concat"):
        y = ops.qr_combine_forward(op, eq, er)
        ref = {"mult": eq * er, "add": eq + er, "concat": torch.cat([eq, er], 1)}[op]
        assert torch.allclose(y, ref)


def test_qr_expand_csr_vs_oracle_and_capacity(ops):
    """dlrm_qr_expand_csr: logical CSR -> physical (plain | quotient | remainder) CSR, bit-
    exact vs the oracle's split (float division, truncation; torch remainder), and with an
    undersized phys_indices buffer: no write past it, offsets clamped to it,
    TBE_ERR_TABLE_CAP raised."""
    rng = np.random.RandomState(3)
    B, rows = 5, [30, 700, 9]
    lo = [torch.tensor(np.concatenate([[0], np.sort(rng.randint(0, 9, B - 1))]))
          for _ in rows]
    li = [torch.tensor(rng.randint(0, n, int(o[-1]) + 3)) for n, o in zip(rows, lo)]
    off, idx = O.batched_csr(lo, li)
    # physical tables: t0 plain, t1 -> quotient (c=4) + remainder, t2 plain
    src, kind, coll = [0, 1, 1, 2], [0, 1, 2, 0], [1, 4, 4, 1]
    per = [int(li[t].numel()) for t in range(3)]
    n = sum(per[s_] for s_ in src)
    want_idx, want_off, base = [], [], 0
    for p_, s_ in enumerate(src):
        v = li[s_].long()
        q, r = O.QREmbeddingBagOracle.split(v, coll[p_]) if kind[p_] else (v, v)
        want_idx.append([v, q, r][kind[p_]])
        want_off.append(lo[s_] + base)
        base += per[s_]
    want_off = torch.cat(want_off + [torch.tensor([base])]).to(torch.int32)
    want_idx = torch.cat(want_idx).to(torch.int32)
    i32 = dict(dtype=torch.int32, device=dev)
    args = (torch.tensor(src, **i32), torch.tensor(kind, **i32), torch.tensor(coll, **i32))
    for cap in (n, n - 7):
        pidx = torch.full((cap + 16,), -5, **i32)  # 16 guard entries past the capacity
        poff = torch.empty(4 * B + 1, **i32)
        flag = torch.zeros(1, **i32)
        ops.qr_expand_csr(4, B, idx.to(dev), off.to(dev), *args, max(per), pidx[:cap], poff,
                          error_flag=flag)
        torch.cuda.synchronize()
        assert torch.equal(pidx[:cap].cpu(), want_idx[:cap])
        assert (pidx[cap:] == -5).all()
        assert torch.equal(poff.cpu(), want_off.clamp(max=cap))
        assert int(flag.item()) == (0 if cap == n else ops.TBE_ERR_TABLE_CAP)


def test_csr_builder_device(ops):
    lo = [torch.tensor([0, 3, 5]), torch.tensor([0, 0, 2]), torch.tensor([0, 1, 4])]
    li = [torch.arange(7), torch.arange(4), torch.arange(6)]
    ref, _ = O.batched_csr(lo, li)
    out = ops.csr_from_tables([o.to(dev) for o in lo], [7, 4, 6], 3)
    assert torch.equal(out.cpu(), ref)


def test_uniform_fill(ops):
    x = torch.empty(1 << 20, device=dev)
    ops.uniform_fill_(x, -0.5, 0.25, 7)
    assert x.min().item() >= -0.5 and x.max().item() < 0.25
    assert abs(x.mean().item() + 0.125) < 2e-3
    i = torch.empty(1 << 20, dtype=torch.int32, device=dev)
    ops.uniform_int_fill_(i, 1000, 9)
    assert i.min().item() >= 0 and i.max().item() == 999


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
def test_tbe_backward_table_cap_violation_is_skipped_and_flagged(ops, mode):
    """A caller bound below a table's real lookup count (contract violation):
    the per-table sort must not leave stale keys behind.  That table is skipped and flagged
    (TBE_ERR_TABLE_CAP); the other tables are updated exactly as without the bound."""
    torch.manual_seed(3)
    rows, D, B = [1000, 300, 50], 32, 2048
    T = len(rows)
    L = [1, 3, 1]  # table 1 has 6144 > 4096 lookups
    lo = [torch.arange(B) * L[t] for t in range(T)]
    li = [torch.randint(0, rows[t], (B * L[t],)) for t in range(T)]
    off, idx = O.batched_csr(lo, li)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    G = torch.randn(B, T, D, device=dev)
    W0 = torch.randn(sum(rows), D, device=dev)
    mom0 = torch.rand(sum(rows), device=dev)
    out = []
    for mx in (0, 2048):  # exact (device sort) vs underestimated bound
        W, mom = W0.clone(), mom0.clone()
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.tbe_backward(mode, W, row_base, T, B, idx.to(dev), off.to(dev), G, lr=0.3,
                         eps=1e-8, momentum=mom, max_lookups_per_table=mx, error_flag=flag)
        out.append((W.cpu(), mom.cpu(), int(flag.item())))
    (Wa, ma, fa), (Wb, mb, fb) = out
    assert fa == 0 and fb == ops.TBE_ERR_TABLE_CAP
    a1, b1 = int(row_base[1]), int(row_base[2])
    assert torch.equal(Wb[a1:b1], W0.cpu()[a1:b1])  # skipped table untouched
    assert torch.equal(mb[a1:b1], mom0.cpu()[a1:b1])
    for s, e in ((0, a1), (b1, sum(rows))):  # the others: same values as the exact run
        ok, msg = fp32_close(Wb[s:e].numpy(), Wa[s:e].numpy())
        assert ok, msg


def test_module_lookup_raises_index_error(ops):
    """The drop-in EmbeddingBag path raises IndexError like nn.EmbeddingBag: at once with
    strict_indices="sync", at the module's next call by default (no host sync per call;
    test_gpu_module.py::test_module_index_errors_are_deferred_not_synced)."""
    from dlrm_hip.modules import TableBatchedEmbeddingBags
    m = TableBatchedEmbeddingBags(2, [10, 20], 8).to(dev)
    off = torch.tensor([0, 1, 2, 3, 4], dtype=torch.int32, device=dev)
    idx = torch.tensor([1, 2, 3, 4], dtype=torch.int32, device=dev)
    assert m(idx, off).shape == (2, 2, 8)
    bad = torch.tensor([1, 10, 3, 4], dtype=torch.int32, device=dev)  # 10 >= rows of table 0
    m(bad, off)
    with pytest.raises(IndexError):
        m(idx, off)
    m.strict_indices = "sync"
    with pytest.raises(IndexError):
        m(bad, off)


def test_gemm_splitk_in_launch_fixup_is_deterministic_and_resets(ops):
    """In-launch split-K: the last workgroup of a tile sums the partials in split order.
    Repeated calls on one workspace (tickets reset by the kernel) are bitwise identical,
    equal the unsplit sum within fp32 tolerance, and the tickets end at zero."""
    torch.manual_seed(0)
    M, N, K = 1024, 1028, 2048  # a wgrad shape of C3
    A = torch.randn(K, M, device=dev)
    Bm = torch.randn(K, N, device=dev)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    outs = [ops.gemm(A, Bm, True, False, workspace=ws).cpu() for _ in range(3)]
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    ref = (A.double().t() @ Bm.double()).cpu()
    ok, msg = gemm_close(outs[0].numpy(), ref.numpy(),
                         (A.double().abs().t() @ Bm.double().abs()).cpu().numpy(), K)
    assert ok, msg
    tiles = 16384  # the fixed ticket region
    assert int(ws[:4 * tiles].view(torch.int32).abs().sum()) == 0
    for tile, split in ((64064, 2), (64064, 5), (64064, 9), (32032, 2), (32032, 7)):
        # forced tiles and splits, fused SGD epilogue (32x32: the small-batch plans' tile)
        C0 = torch.randn(M, N, device=dev)
        C = C0.clone()
        with ops.tuning(gemm_tile=tile, gemm_split=split):
            ops.gemm(A, Bm, True, False, C=C, alpha=0.5, epilogue=ops.EPI_SGD, workspace=ws)
        ok, msg = gemm_close((C0 - C).cpu().numpy() / 0.5, ref.numpy(),
                             (A.double().abs().t() @ Bm.double().abs()).cpu().numpy(), K + 4)
        assert ok, (tile, split, msg)
        assert int(ws[:4 * tiles].view(torch.int32).abs().sum()) == 0


@pytest.mark.parametrize("cfg", GEMM_CFGS)
@pytest.mark.parametrize("split", [1, 4])
def test_gemm_ones_col_bias_gradient(ops, cfg, split):
    """ones_col: C[:, ones_col] = epi(alpha * rowsum(op(A))) beside the GEMM - the bias
    gradient of a Linear layer whose bias is the weight column ones_col (fused SGD)."""
    with ops.tuning(gemm_tile=cfg, gemm_split=split):
        _ones_col_cases(ops)


def _ones_col_cases(ops):
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    for (Bt, Nout, K) in [(2048, 256, 512), (300, 130, 64), (64, 16, 8)]:
        torch.manual_seed(Bt + Nout + K)
        g = torch.randn(Bt, Nout, device=dev)
        X = torch.randn(Bt, K, device=dev)
        W0 = torch.randn(Nout, K + 4, device=dev)
        W = W0.clone()
        ops.gemm(g, X, trans_a=True, C=W, alpha=0.25, epilogue=ops.EPI_SGD, ones_col=K,
                 workspace=ws)
        gd, Xd = g.double().cpu(), X.double().cpu()
        dW = gd.t() @ Xd
        db = gd.sum(0)
        got = ((W0 - W).double().cpu() / 0.25)
        ok, msg = gemm_close(got[:, :K].numpy(), dW.numpy(), (gd.abs().t() @ Xd.abs()).numpy(),
                             Bt + 8)
        assert ok, (Bt, Nout, K, msg)
        ok, msg = gemm_close(got[:, K].numpy(), db.numpy(), gd.abs().sum(0).numpy(), Bt + 8)
        assert ok, (Bt, Nout, K, "bias", msg)
        assert torch.equal(W[:, K + 1:], W0[:, K + 1:])  # untouched pad columns


def test_gemm_group_matches_separate_launches(ops):
    """A grouped launch (dgrad of layer l || wgrad+SGD of layer l+1, plus two more problems
    of other layouts) gives bitwise the results of the same problems launched one by one."""
    torch.manual_seed(5)
    Bt = 1024
    g1 = torch.randn(Bt, 512, device=dev)
    W1 = torch.randn(512, 260, device=dev)
    a1 = torch.rand(Bt, 260, device=dev)
    g2 = torch.randn(Bt, 256, device=dev)
    x2 = torch.randn(Bt, 516, device=dev)
    W2 = torch.randn(256, 516, device=dev)
    X3 = torch.randn(Bt, 132, device=dev)
    W3 = torch.randn(64, 132, device=dev)
    A4 = torch.randn(96, 200, device=dev)
    B4 = torch.randn(48, 96, device=dev)

    def problems(outs):
        dX, W2c, Y3, C4 = outs
        return [ops.gemm_problem(g1, W1[:, :256], C=dX, epilogue=ops.EPI_DRELU, aux=a1)[0],
                ops.gemm_problem(g2, x2[:, :512], trans_a=True, C=W2c, alpha=0.1,
                                 epilogue=ops.EPI_SGD, ones_col=512)[0],
                ops.gemm_problem(X3, W3, trans_b=True, C=Y3, epilogue=ops.EPI_RELU)[0],
                ops.gemm_problem(A4, B4, trans_a=True, trans_b=True, C=C4)[0]]

    def fresh():
        return [torch.zeros(Bt, 256, device=dev), W2.clone(), torch.zeros(Bt, 64, device=dev),
                torch.zeros(200, 48, device=dev)]

    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    sep = fresh()
    for pr in problems(sep):
        ops.gemm_group([pr], ws)
    grp = fresh()
    ops.gemm_group(problems(grp), ws)
    torch.cuda.synchronize()
    for a, b in zip(sep, grp):  # splits are planned per problem: bitwise equal
        assert torch.equal(a, b)
    ref = (g1.double() @ W1[:, :256].double()) * (a1[:, :256] > 0)
    assert torch.allclose(grp[0].double(), ref, rtol=1e-5, atol=1e-3)
    ref4 = A4.double().t() @ B4.double().t()
    assert torch.allclose(grp[3].double(), ref4, rtol=1e-5, atol=1e-3)
    grp2 = fresh()
    ops.gemm_group(problems(grp2), ws)  # the same group again: bitwise reproducible
    for a, b in zip(grp, grp2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("ones", [False, True])
def test_gemm_partial_then_reduce_equals_full(ops, ones):
    """A PARTIAL problem (split-K partials to a buffer) finished by a REDUCE job in a later
    launch gives bitwise the in-launch split-K result (same splits, same sum order), with
    the fused SGD epilogue and the ones_col bias row sums."""
    torch.manual_seed(11)
    Bt, Nout, K = 2048, 256, 512
    g = torch.randn(Bt, Nout, device=dev)
    X = torch.randn(Bt, K + 4, device=dev)
    W0 = torch.randn(Nout, K + 4, device=dev)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    kw = dict(trans_a=True, alpha=0.5, epilogue=ops.EPI_SGD, ones_col=K if ones else -1)
    xin = X[:, :K] if ones else X
    W1 = W0.clone()
    pr, _ = ops.gemm_problem(g, xin, C=W1, **kw)
    s = ops.gemm_splits(pr)
    assert s > 1
    ops.gemm_group([pr], ws)  # FULL, in-launch split-K
    W2 = W0.clone()
    part = torch.empty(ops.gemm_partial_bytes(Nout, xin.shape[1], s) // 4, device=dev)
    pp, _ = ops.gemm_problem(g, xin, C=W2, partial=part, splits=s, **kw)
    ops.gemm_group([pp], ws)
    assert torch.equal(W2, W0)  # PARTIAL does not touch C
    ops.gemm_group([ops.reduce_problem(pp)], ws)
    torch.cuda.synchronize()
    assert torch.equal(W1, W2)


@pytest.mark.parametrize("path", ["staged", "runtime_d"])
@pytest.mark.parametrize("D", [16, 128])
def test_interact_backward_relu_x_and_paths(ops, path, D):
    """relu_x fuses ReLU'(x) into feature 0's gradient, on the LDS-staged kernel and on the
    fallback path (features not 16-B aligned: the runtime-D MFMA kernel + a separate mask
    pass); both agree with autograd on a torch fp32 reference (bmm + tril gather), within
    the fp32 tolerance."""
    torch.manual_seed(D)
    B, F = 70, 27
    x = torch.randn(B, D)          # mixed signs: the mask matters
    ly = torch.randn(B, F - 1, D)
    gR = torch.randn(B, D + F * (F - 1) // 2)
    xr = x.clone().requires_grad_(True)
    lr_ = ly.clone().requires_grad_(True)
    T = torch.cat([xr[:, None, :], lr_], 1)
    Z = torch.bmm(T, T.transpose(1, 2))
    li, lj = torch.tril_indices(F, F, -1)
    R = torch.cat([xr, Z[:, li, lj]], 1)
    (R * gR).sum().backward()
    def dev_(t):  # runtime_d: a 1-float offset breaks the 16-B alignment of every row
        if path == "staged":
            return t.to(dev)
        buf = torch.empty(t.numel() + 1, device=dev)
        v = buf[1:].view(t.shape)
        v.copy_(t)
        return v
    gx, gly = ops.interact_backward("dot", dev_(x), dev_(ly), gR.to(dev), relu_x=True)
    ok, msg = fp32_close(gx.cpu().numpy(), (xr.grad * (x > 0)).numpy())
    assert ok, msg
    ok, msg = fp32_close(gly.cpu().numpy(), lr_.grad.numpy())
    assert ok, msg
    # forward on both paths vs the same reference
    out = ops.interact_forward("dot", dev_(x), dev_(ly))
    ok, msg = fp32_close(out.cpu().numpy(), R.detach().numpy())
    assert ok, msg


@pytest.mark.parametrize("D", [16, 32, 64, 128])
@pytest.mark.parametrize("F,self_int", [(2, False), (9, True), (27, False), (32, False)])
@pytest.mark.parametrize("gather", [False, True])
def test_interact_backward_v4_matches_v3(ops, D, F, self_int, gather):
    """The interaction backward as one wave per sample x 32-column block (v4, forced by
    DLRM_TUNE_INTERACT_BWD = 4; the default for D <= 32), one wave per sample (v3, forced
    by 3), one workgroup per sample with a wave per column block (v5, forced by 5; the
    default for D >= 64) and the default pick: bitwise the same gradients -
    every element is the same 32-deep MFMA sum - pooled and gather-fused, ReLU' of x fused,
    a ragged batch (B = 203) and strided x."""
    torch.manual_seed(D * 10 + F)
    T, B = F - 1, 203
    rows = [int(r) for r in torch.randint(1, 500, (T,))]
    row_base = torch.tensor([0] + list(np.cumsum(rows)), dtype=torch.int64, device=dev)
    W = torch.randn(int(row_base[-1]), D, device=dev)
    idx = torch.cat([torch.randint(0, n, (B,)) for n in rows]).to(torch.int32).to(dev)
    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev)
    x = torch.randn(B, D + 4, device=dev)[:, :D]
    E = ops.tbe_forward(W, row_base, T, B, idx, off)
    npairs = F * (F + 1) // 2 if self_int else F * (F - 1) // 2
    gR = torch.randn(B, D + npairs, device=dev)
    res = []
    for v in (4, 3, 5, 0):
        with ops.tuning(interact_bwd=v):
            if gather:
                g = ops.interact_backward_gather(x, W, row_base, idx, gR, self_int, relu_x=True)
            else:
                g = ops.interact_backward("dot", x, E, gR, self_int, relu_x=True)
        torch.cuda.synchronize()
        res.append([t.cpu().clone() for t in g])
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("F,self_int", [(2, False), (9, True), (27, False), (32, False)])
@pytest.mark.parametrize("gather", [False, True])
def test_interact_forward_v5_matches_v4_and_reference(ops, D, F, self_int, gather):
    """The interaction forward as one workgroup per sample (v5: a wave per 32-column block,
    the partial Gram matrices added in LDS; the default for D >= 64) vs one wave per sample
    (v4, forced by DLRM_TUNE_INTERACT_FWD = 4) and a torch fp64 bmm + tril reference:
    within 1e-5 plus the D-term accumulation bound (the k sum is split into blocks), pooled
    and gather-fused, a ragged batch (B = 203) and strided x."""
    torch.manual_seed(D * 7 + F)
    T, B = F - 1, 203
    rows = [int(r) for r in torch.randint(1, 500, (T,))]
    row_base = torch.tensor([0] + list(np.cumsum(rows)), dtype=torch.int64, device=dev)
    W = torch.randn(int(row_base[-1]), D, device=dev)
    idx = torch.cat([torch.randint(0, n, (B,)) for n in rows]).to(torch.int32).to(dev)
    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev)
    x = torch.randn(B, D + 4, device=dev)[:, :D]
    E = ops.tbe_forward(W, row_base, T, B, idx, off)
    Tm = torch.cat([x[:, None, :], E], 1).double()
    Z = torch.bmm(Tm, Tm.transpose(1, 2))
    Za = torch.bmm(Tm.abs(), Tm.abs().transpose(1, 2))
    li, lj = torch.tril_indices(F, F, 0 if self_int else -1)
    ref = torch.cat([x.double(), Z[:, li, lj]], 1).cpu().numpy()
    # fp32 vs fp64: 1e-5 plus the standard D-term accumulation bound 2 D u |T| |T|^T
    acc = torch.cat([torch.zeros_like(x.double()), Za[:, li, lj]], 1).cpu().numpy()
    lim = 1e-5 * np.maximum(1.0, np.abs(ref)) + 2 * D * 2.0 ** -24 * acc
    outs = []
    for v in (4, 5, 0):
        with ops.tuning(interact_fwd=v):
            R = ops.interact_forward_gather(x, W, row_base, idx, self_int) if gather else \
                ops.interact_forward("dot", x, E, self_int)
        torch.cuda.synchronize()
        outs.append(R.cpu())
        err = np.abs(R.cpu().numpy() - ref)
        assert (err <= lim).all(), (v, float((err - lim).max()))
    assert torch.equal(outs[1], outs[2])  # v5 is the default


def _mlp_ref(X, layers):
    """fp64 reference of the bias-folded ReLU chain (trainer layout)."""
    h = X.double()
    outs = []
    for W, Y, kin in layers:
        n = W.shape[0]
        y = torch.relu(h[:, :kin] @ W[:, :kin].double().t())
        outs.append(y)
        h = torch.zeros(X.shape[0], (n + 1 + 3) // 4 * 4, dtype=torch.float64, device=X.device)
        h[:, :n] = y
        h[:, n] = 1.0
    return outs


def _mlp_setup(rows, dims, seed=5):
    g = torch.Generator(device=dev).manual_seed(seed)
    pad4 = lambda n: (n + 3) // 4 * 4  # noqa: E731
    k0 = dims[0]
    X = torch.zeros(rows, pad4(k0 + 1), device=dev)
    X[:, :k0] = torch.rand(rows, k0, generator=g, device=dev)
    X[:, k0] = 1.0
    layers = []
    for k, n in zip(dims[:-1], dims[1:]):
        W = torch.randn(n, pad4(k + 1), generator=g, device=dev) / (k ** 0.5)
        W[:, k + 1:] = 0.0
        Y = torch.full((rows, pad4(n + 1)), -7.0, device=dev)
        layers.append((W, Y, pad4(k + 1)))
    return X, layers


@pytest.mark.parametrize("rows,dims", [(2048, [13, 512, 256, 128]), (37, [13, 512, 256, 128]),
                                       (100, [3, 64, 16]), (48, [200, 120, 500, 33, 7])])
def test_mlp_chain_forward_matches_reference(ops, rows, dims):
    """The row-block bottom-MLP kernel (every layer in one launch, activations in LDS) vs an
    fp64 chain; ragged batch (37 rows), widths that are not multiples of 16 or 64, 4 layers.
    Only columns < out_width of each output are written."""
    X, layers = _mlp_setup(rows, dims)
    chain = ops.mlp_chain(X, layers)
    assert ops.mlp_chain_supported(chain)
    ops.mlp_chain_forward(chain)
    torch.cuda.synchronize()
    ref = _mlp_ref(X, layers)
    for (W, Y, kin), r in zip(layers, ref):
        n = W.shape[0]
        got = Y[:, :n].double()
        err = (got - r).abs().max().item()
        scale = max(1.0, r.abs().max().item())
        assert err <= 1e-5 * scale, err
        assert torch.all(Y[:, n:] == -7.0)  # padding / bias column untouched


def test_mlp_chain_unsupported_is_refused(ops):
    X, layers = _mlp_setup(16, [13, 1024, 8])  # out_width 1024 > 512
    chain = ops.mlp_chain(X, layers)
    assert not ops.mlp_chain_supported(chain)
    with pytest.raises(Exception):
        ops.mlp_chain_forward(chain)


@pytest.mark.parametrize("rows,dims", [(2048, [13, 512, 256, 128]), (37, [13, 512, 256, 128]),
                                       (128, [13, 512, 256, 64, 16]), (100, [3, 64, 48])])
@pytest.mark.parametrize("parts", [2, 4])
def test_mlp_chain_split_parts_bitwise(ops, rows, dims, parts):
    """Split chains (parts workgroups per 16-row block, every split layer in turn - the
    last one needs no hand-off): bitwise the one-workgroup chain's outputs, also as the
    lookup launch's bottom role; the tickets are left zero for the next call."""
    X, layers = _mlp_setup(rows, dims)
    ops.mlp_chain_forward(ops.mlp_chain(X, layers))
    ref = [Y.clone() for _, Y, _ in layers]
    for split in range(len(layers)):
        if (layers[split][0].shape[0] + 15) // 16 < parts:
            continue
        for fused in (False, True):
            for _, Y, _ in layers:
                Y.fill_(-7.0)
            tk = torch.zeros((rows + 15) // 16, dtype=torch.int32, device=dev)
            chain = ops.mlp_chain(X, layers, parts=parts, split_layer=split, tickets=tk)
            assert ops.mlp_chain_supported(chain)
            for _ in range(2):  # twice: the tickets must be reusable
                if fused:
                    T, B = 3, rows
                    idx = torch.randint(0, 50, (T * B,), dtype=torch.int32, device=dev)
                    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev)
                    row_base = torch.arange(T + 1, dtype=torch.int64, device=dev) * 50
                    W = torch.zeros(T * 50, 16, device=dev)
                    ws = torch.zeros(ops.tbe_backward_workspace_size(T * B, T * 50, 16),
                                     dtype=torch.uint8, device=dev)
                    ops.tbe_forward_presort(W, row_base, T, B, idx, off, ws, B, bottom=chain,
                                            lookup=False)
                else:
                    ops.mlp_chain_forward(chain)
            torch.cuda.synchronize()
            assert int(tk.abs().sum()) == 0
            for (W_, Y, kin), r in zip(layers, ref):
                n = W_.shape[0]
                assert torch.equal(Y[:, :n], r[:, :n]), (split, fused)


def test_tbe_forward_presort_with_bottom_chain(ops):
    """The fused launch (sort + gather + bottom MLP) gives the plain forward's E bitwise and
    the standalone chain's activations bitwise; the presorted backward still matches."""
    torch.manual_seed(3)
    rows, D, B, L = [3, 5000, 700, 90000], 128, 2048, 1
    T = len(rows)
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    off, idx = O.batched_csr(lo, li)
    idx, off = idx.to(dev), off.to(dev)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    W = torch.randn(sum(rows), D, device=dev)
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D),
                     dtype=torch.uint8, device=dev)
    X, layers = _mlp_setup(B, [13, 512, 256, 128])
    X2, layers2 = X.clone(), [(w, y.clone(), k) for w, y, k in layers]
    E0 = ops.tbe_forward(W, row_base, T, B, idx, off)
    E1 = ops.tbe_forward_presort(W, row_base, T, B, idx, off, ws, B,
                                 bottom=ops.mlp_chain(X, layers))
    ops.mlp_chain_forward(ops.mlp_chain(X2, layers2))
    torch.cuda.synchronize()
    assert torch.equal(E0, E1)
    for (_, y1, _), (_, y2, _) in zip(layers, layers2):
        assert torch.equal(y1, y2)
    G = torch.randn(B, T, D, device=dev)
    Wa, Wb = W.clone(), W.clone()
    ops.tbe_backward("sgd", Wa, row_base, T, B, idx, off, G, lr=0.1, workspace=ws,
                     max_lookups_per_table=B, presorted=True)
    ops.tbe_backward("sgd", Wb, row_base, T, B, idx, off, G, lr=0.1, max_lookups_per_table=B)
    assert torch.equal(Wa, Wb)


@pytest.mark.parametrize("D,L,bound,idx_dtype,weighted", [
    (64, 3, False, torch.int32, False),   # no bound: no sort, lookup + MLP in one launch
    (64, 3, True, torch.int64, True),     # bound B * L above the LDS sort's 4096 per table
    (40, 5, False, torch.int32, False),   # D % 4 != 0: the scalar gather lanes
    (600, 9, True, torch.int32, False),   # D > 512: lookup, then the chain's own launch
])
def test_tbe_forward_presort_unsorted_with_bottom_chain(ops, D, L, bound, idx_dtype, weighted):
    """Tables too large for the per-table sort (C1's L = 100 shape): the lookup and the
    bottom MLP still share one launch (no sort role).  E and the error flag equal the plain
    forward's bitwise (an out-of-range index included), the chain's activations the
    standalone chain's bitwise, and the backward (which then sorts itself) is unchanged."""
    torch.manual_seed(5)
    rows, B = [3, 5000, 700, 90000], 2048 if D <= 64 else 512
    T = len(rows)
    mx = B * L if bound else 0
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    li[1][11] = 10 ** 6
    off, idx = O.batched_csr(lo, li)
    idx, off = idx.to(idx_dtype).to(dev), off.to(dev)
    psw = torch.rand(idx.numel(), device=dev) if weighted else None
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    W = torch.randn(sum(rows), D, device=dev)
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D),
                     dtype=torch.uint8, device=dev)
    X, layers = _mlp_setup(B, [13, 512, 256, 64])
    X2, layers2 = X.clone(), [(w, y.clone(), k) for w, y, k in layers]
    f0 = torch.zeros(1, dtype=torch.int32, device=dev)
    f1 = torch.zeros(1, dtype=torch.int32, device=dev)
    E0 = ops.tbe_forward(W, row_base, T, B, idx, off, per_sample_weights=psw, error_flag=f0)
    for _ in range(2):  # twice: the split chain's tickets are reusable
        E1 = ops.tbe_forward_presort(W, row_base, T, B, idx, off, ws, mx,
                                     per_sample_weights=psw, error_flag=f1,
                                     bottom=ops.mlp_chain(X, layers))
    ops.mlp_chain_forward(ops.mlp_chain(X2, layers2))
    torch.cuda.synchronize()
    assert torch.equal(E0, E1)
    assert int(f0.item()) == int(f1.item()) != 0
    for (_, y1, _), (_, y2, _) in zip(layers, layers2):
        assert torch.equal(y1, y2)
    if weighted:
        return
    G = torch.randn(B, T, D, device=dev)
    Wa, Wb = W.clone(), W.clone()
    ops.tbe_backward("sgd", Wa, row_base, T, B, idx, off, G, lr=0.1, workspace=ws,
                     max_lookups_per_table=mx, presorted=True)
    ops.tbe_backward("sgd", Wb, row_base, T, B, idx, off, G, lr=0.1, max_lookups_per_table=mx)
    assert torch.equal(Wa, Wb)


@pytest.mark.parametrize("L,bound,idx_dtype,weighted,mode", [
    (1, True, torch.int32, False, "sgd"),       # per-table LDS sort
    (3, True, torch.int32, False, "sgd"),       # tiled per-table sort
    (3, True, torch.int64, True, "rowwise_adagrad"),
    (3, False, torch.int32, False, "sgd"),      # device-wide sort (its pass parity)
    (2, False, torch.int64, True, "dense"),
])
def test_tbe_backward_sort_then_presorted_any(ops, L, bound, idx_dtype, weighted, mode):
    """dlrm_tbe_backward_sort (the backward's sort alone, run early) followed by the backward
    with presorted = PRESORTED_ANY: bitwise the backward that sorts itself, for every sort
    variant (per-table, tiled, device-wide), an out-of-range index flagged the same."""
    torch.manual_seed(9)
    rows, B, D = [3, 5000, 700, 90000], 2048, 64
    T = len(rows)
    mx = B * L if bound else 0
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    li[2][5] = 10 ** 6
    off, idx = O.batched_csr(lo, li)
    idx, off = idx.to(idx_dtype).to(dev), off.to(dev)
    psw = torch.rand(idx.numel(), device=dev) if weighted else None
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    W = torch.randn(sum(rows), D, device=dev)
    G = torch.randn(B, T, D, device=dev)
    mom = torch.rand(sum(rows), device=dev) if mode == "rowwise_adagrad" else None
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D),
                     dtype=torch.uint8, device=dev)
    out = []
    for early in (False, True):
        Wx = torch.zeros_like(W) if mode == "dense" else W.clone()
        mx_ = mom.clone() if mom is not None else None
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        ws.fill_(0xA5)
        if early:
            ops.tbe_backward_sort(Wx, row_base, T, B, idx, off, ws, mx,
                                  per_sample_weights=psw, error_flag=flag)
        ops.tbe_backward(mode, Wx, row_base, T, B, idx, off, G, lr=0.05, eps=1e-6,
                         momentum=mx_, per_sample_weights=psw, workspace=ws,
                         max_lookups_per_table=mx, error_flag=flag,
                         presorted=ops.PRESORTED_ANY if early else False)
        torch.cuda.synchronize()
        out.append((Wx.cpu(), None if mx_ is None else mx_.cpu(), int(flag.item())))
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] is None or torch.equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2] != 0


def _tbe_bwd_case(rows, B, L, D, seed, invalid=False, idx_dtype=torch.int32):
    torch.manual_seed(seed)
    T = len(rows)
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    if invalid:
        li[0][7] = 10 ** 9
        li[-1][B * L - 1] = -1
    off, idx = O.batched_csr(lo, li)
    if invalid:  # lookups after the last bag
        idx = torch.cat([idx, torch.tensor([1, 2, 3], dtype=idx.dtype)])
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    G = torch.randn(B, T, D, device=dev)
    return T, lo, li, off.to(idx_dtype).to(dev), idx.to(idx_dtype).to(dev), row_base, G


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad", "dense"])
@pytest.mark.parametrize("invalid", [False, True])
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
def test_tbe_backward_tiled_sort(ops, mode, invalid, idx_dtype):
    """Tables with more than 4096 lookups (L = 100 pooling): the tiled per-table radix sort
    gives bitwise the updates of the device-wide sort when every index is valid (same
    (row, position) order), and matches the fp64 coalesced reference either way; skewed
    (3-row) and large tables, 10-bit digits (2^17 rows)."""
    rows, B, L, D = [64, 130000, 700, 9000], 256, 40, 64
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 5, invalid, idx_dtype)
    W0 = torch.randn(sum(rows), D, device=dev) * 0.1
    mom0 = torch.rand(sum(rows), device=dev)
    res = []
    for tiled in (True, False):  # False: the device-wide sort forced (DLRM_TUNE_TBE_SORT)
        W = W0.clone() if mode != "dense" else torch.zeros_like(W0)
        mom = mom0.clone()
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        with ops.tuning(tbe_sort=0 if tiled else 1):
            ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8,
                             momentum=mom, max_lookups_per_table=B * L, error_flag=flag)
        torch.cuda.synchronize()
        assert (int(flag.item()) != 0) == invalid
        res.append((W.cpu(), mom.cpu()))
    if not invalid:
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    gsum = torch.zeros(sum(rows), D, dtype=torch.float64)
    gt = G.cpu().double()
    bag = torch.arange(B * L) // L
    for t in range(T):
        r = li[t]
        ok_ = (r >= 0) & (r < rows[t])
        gsum.index_add_(0, int(row_base[t]) + r[ok_], gt[bag[ok_], t])
    if mode == "dense":
        ref = gsum
    elif mode == "sgd":
        ref = W0.cpu().double() - 0.3 * gsum
    else:
        touched = gsum.abs().sum(1) > 0
        m = mom0.cpu().double() + torch.where(touched, (gsum ** 2).mean(1),
                                              torch.zeros(1, dtype=torch.float64))
        ref = W0.cpu().double() - 0.3 * gsum / (m.sqrt()[:, None] + 1e-8)
    for W, _ in res:
        ok, msg = fp32_close(W.numpy(), ref.numpy())
        assert ok, msg


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
@pytest.mark.parametrize("D", [16, 32, 64, 128, 6, 256])
@pytest.mark.parametrize("sort", ["presorted", "per_table", "tiled", "global"])
def test_tbe_backward_deferred_into_gemm_launches(ops, mode, D, sort):
    """dlrm_tbe_backward_defer + the two passes as extra workgroups of grouped GEMM launches
    (phase 1 beside a dgrad + wgrad pair, phase 2 alone or beside a FULL split-K problem):
    the embedding update is bitwise the standalone dlrm_tbe_backward's and the GEMM results
    bitwise the plain group launch's.  D = 6 (no float4 rows) and 256 (two chunks per lane)
    are outside the fused variants: the role comes back None, the update already done."""
    L = 40 if sort in ("tiled", "global") else 1
    rows, B = [3, 5000, 700, 90000], 256
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 21, invalid=True)
    W0 = torch.randn(sum(rows), D, device=dev) * 0.1
    mom0 = torch.rand(sum(rows), device=dev)
    mx = B * L
    ws = torch.zeros(ops.tbe_backward_workspace_size(idx.numel(), sum(rows), D),
                     dtype=torch.uint8, device=dev)
    torch.manual_seed(3)
    A1, B1 = torch.randn(300, 260, device=dev), torch.randn(260, 512, device=dev)
    A2, B2 = torch.randn(512, 300, device=dev), torch.randn(512, 260, device=dev)
    A3, B3 = torch.randn(64, 4096, device=dev), torch.randn(4096, 96, device=dev)

    def probs():
        p1, c1 = ops.gemm_problem(A1, B1)
        p2, c2 = ops.gemm_problem(A2, B2, trans_a=True)
        p3, c3 = ops.gemm_problem(A3, B3)  # FULL, split in-launch (K = 4096, 2 tiles)
        return [p1, p2], [p3], (c1, c2, c3)

    res = []
    for defer in (False, True):
        W, mom = W0.clone(), mom0.clone()
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        ws.zero_()
        gws = torch.zeros(1 << 22, dtype=torch.uint8, device=dev)
        tune = dict(tbe_sort=1) if sort == "global" else {}
        with ops.tuning(**tune):
            if sort == "presorted":
                assert ops.tbe_forward_presort(W0, row_base, T, B, idx, off, ws, mx,
                                               error_flag=flag, lookup=False) is None
            kw = dict(lr=0.3, eps=1e-8, momentum=mom, workspace=ws,
                      max_lookups_per_table=0 if sort == "global" else mx, error_flag=flag,
                      presorted=sort == "presorted")
            first, second, outs = probs()
            if defer:
                role = ops.tbe_backward_defer(mode, W, row_base, T, B, idx, off, G, **kw)
                fusable = D in (16, 32, 64, 128)
                assert (role is not None) == fusable
                assert ops.role_blocks(role) % 8 == 0
                ops.gemm_group(first, gws, dev, role=role, phase=1)
                ops.gemm_group([] if D == 16 else second, gws, dev, role=role, phase=2)
                if D != 16:
                    second = []
            else:
                ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, **kw)
                ops.gemm_group(first, gws, dev)
            if second:
                ops.gemm_group(second, gws, dev)
        torch.cuda.synchronize()
        res.append((W.cpu(), mom.cpu(), flag.item(), [c.cpu() for c in outs]))
    (w0, m0, f0, c0), (w1, m1, f1, c1) = res
    assert torch.equal(w0, w1) and torch.equal(m0, m1)
    assert f0 == f1 and f0 & ops.TBE_ERR_INDEX
    for a, b in zip(c0, c1):
        assert torch.equal(a, b)


def test_gemm_group_role_rejects_a_foreign_role(ops):
    """A role struct not filled by dlrm_tbe_backward_defer is refused (INVALID_ARG)."""
    import ctypes
    from dlrm_hip import _lib
    role = _lib.LaunchRole()
    ctypes.memset(ctypes.byref(role), 0x5a, ctypes.sizeof(role))
    with pytest.raises(_lib.DLRMHipError):
        ops.gemm_group([], None, dev, role=role, phase=1)


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
@pytest.mark.parametrize("sort,D", [("per_table", 128), ("tiled", 64), ("global", 16),
                                    ("tiled", 32)])
def test_tbe_backward_lean_passes_match_16_in_flight(ops, mode, sort, D):
    """The lean update passes (4 gradient rows in flight per lane group, the default where
    they apply) vs the 16-in-flight kernels (DLRM_TUNE_TBE_LEAN = 1): bitwise the same
    tables and momentum - the rows in flight change the load schedule, not the add order."""
    L = 1 if sort == "per_table" else 40
    rows, B = [3, 5000, 700, 90000], 256
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 23, invalid=True)
    W0 = torch.randn(sum(rows), D, device=dev) * 0.1
    mom0 = torch.rand(sum(rows), device=dev)
    res = []
    for lean in (0, 1):
        W, mom = W0.clone(), mom0.clone()
        with ops.tuning(tbe_lean=lean, tbe_sort=1 if sort == "global" else 0):
            ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8,
                             momentum=mom,
                             max_lookups_per_table=0 if sort == "global" else B * L)
        torch.cuda.synchronize()
        res.append((W.cpu(), mom.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
def test_tbe_backward_tiled_sort_per_table_pass_counts(ops, mode):
    """Tables needing 1, 3, 1 and 2 passes of 10-bit digits in one call (2, 21, 10 and 16
    key bits; the call's 21 global bits ask for 3): each table runs only its own passes,
    its last one landing in the output buffers - with the wide digit scan (default), the
    chunked scan (DLRM_TUNE_TBE_SORT = 2) and the device-wide sort (1): bitwise the same
    update."""
    rows, B, L, D = [3, 2_000_000, 700, 40000], 256, 40, 16
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 29)
    W0 = torch.randn(sum(rows), D, device=dev) * 0.1
    mom0 = torch.rand(sum(rows), device=dev)
    res = []
    for sort in (0, 2, 1):
        W, mom = W0.clone(), mom0.clone()
        with ops.tuning(tbe_sort=sort):
            ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8,
                             momentum=mom, max_lookups_per_table=B * L)
        torch.cuda.synchronize()
        res.append((W.cpu(), mom.cpu()))
    for other in res[1:]:
        assert torch.equal(res[0][0], other[0]) and torch.equal(res[0][1], other[1])
    assert not torch.equal(res[0][0], W0.cpu())


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
@pytest.mark.parametrize("case", ["c1", "invalid", "hot", "two_tiles", "global"])
def test_tbe_backward_wide_scan_matches_chunked_scan(ops, mode, case):
    """The tiled sort's digit scan as one wide launch (a workgroup per 64 digits, the
    scatter adding each digit's start) vs the chunked csum / scan launches
    (DLRM_TUNE_TBE_SORT = 2): bitwise the same update at the C1 shape (8 x 1e5 rows, L 100:
    50 tiles per table), invalid and outside-bag lookups with a 3-pass (2^20-row) table,
    hot rows (long runs of one digit across tiles), tables of two tiles, and the device-
    wide sort's one segment (no per-table bound: 400 tiles)."""
    if case in ("c1", "global"):
        rows, B, L, D, inv = [100000] * 8, 2048, 100, 64, False
    elif case == "invalid":
        rows, B, L, D, inv = [3, 70000, 1 << 20, 900], 512, 37, 16, True
    elif case == "hot":
        rows, B, L, D, inv = [50000, 3000], 1024, 60, 32, False
    else:
        rows, B, L, D, inv = [4000, 9000], 64, 70, 16, False
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 41, invalid=inv)
    if case == "hot":  # most lookups on a few rows: the same digit in every tile
        hot = (torch.rand(idx.shape, device=dev) < 0.8)
        idx = torch.where(hot, idx % 7, idx)
    W0 = torch.randn(sum(rows), D, device=dev) * 0.1
    mom0 = torch.rand(sum(rows), device=dev)
    mx = 0 if case == "global" else B * L
    res = []
    for sort in (0, 2):
        W, mom = W0.clone(), mom0.clone()
        with ops.tuning(tbe_sort=sort):
            ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8,
                             momentum=mom, max_lookups_per_table=mx)
        torch.cuda.synchronize()
        res.append((W.cpu(), mom.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert not torch.equal(res[0][0], W0.cpu())


@pytest.mark.parametrize("mode", ["sgd", "rowwise_adagrad"])
def test_tbe_backward_device_wide_sort_chunked_scan(ops, mode):
    """The device-wide sort at the C1 lookup count (1.64 M lookups: 400 tiles, the scan in
    25 chunks of 16 over two launches) vs the tiled per-table sort (50 tiles per table, one
    chunk): bitwise the same update."""
    rows, B, L, D = [100000] * 8, 2048, 100, 16
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 37)
    W0 = torch.randn(sum(rows), D, device=dev) * 0.1
    mom0 = torch.rand(sum(rows), device=dev)
    res = []
    for mx in (B * L, 0):
        W, mom = W0.clone(), mom0.clone()
        ops.tbe_backward(mode, W, row_base, T, B, idx, off, G, lr=0.3, eps=1e-8, momentum=mom,
                         max_lookups_per_table=mx)
        torch.cuda.synchronize()
        res.append((W.cpu(), mom.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_tbe_backward_tiled_sort_cap_violation(ops):
    """max_lookups_per_table underestimated (tiles cover 8192 of a table's 12800 lookups):
    that table is skipped (no update) and flagged; the others are updated."""
    rows, B, L, D = [5000, 6000], 128, 100, 16
    T, lo, li, off, idx, row_base, G = _tbe_bwd_case(rows, B, L, D, 9)
    W0 = torch.randn(sum(rows), D, device=dev)
    for sort in (0, 2):  # wide / chunked digit scan
        W = W0.clone()
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        with ops.tuning(tbe_sort=sort):
            ops.tbe_backward("sgd", W, row_base, T, B, idx, off, G, lr=0.5,
                             max_lookups_per_table=8000, error_flag=flag)
        torch.cuda.synchronize()
        assert int(flag.item()) & 2  # TBE_ERR_TABLE_CAP
        assert torch.equal(W, W0)  # both tables overflow their 2 tiles: nothing updated


def _c1_case(dist: str, seed: int):
    """C1 table shape: 8 x 1e5 rows, D = 64, B = 2048, L = 100 (1.64 M lookups, >= 2^18:
    the long-block path).  uniform: the reference generator's distribution (sorted within
    a bag); zipf: Zipf(1.05) ranks folded onto the rows (SURVEY.md §8d's skew run: row 0
    takes ~5 % of a table's lookups, so its run crosses ~160 blocks of 64)."""
    T, R, D, B, L = 8, 100000, 64, 2048, 100
    rng = np.random.RandomState(seed)
    if dist == "uniform":
        li = np.sort(rng.randint(0, R, (T, B, L)), axis=2)
    else:
        li = (rng.zipf(1.05, (T, B, L)) - 1) % R
    idx = torch.tensor(li.reshape(-1), dtype=torch.int32)
    off = torch.arange(T * B + 1, dtype=torch.int32) * L
    g = torch.Generator().manual_seed(seed)
    W0 = torch.empty(T * R, D).uniform_(-0.05, 0.05, generator=g)
    G = torch.empty(B, T, D).uniform_(-1.0, 1.0, generator=g)
    row_base = torch.arange(T + 1, dtype=torch.int64) * R
    return T, R, D, B, L, idx, off, W0, G, row_base


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_tbe_c1_full_shape_forward_and_backward_vs_oracle(ops, dist):
    """The C1-shape lookup and its backward + exact SGD at FULL size against the oracle:
    forward vs nn.EmbeddingBag (fp32, lookup order), backward vs the fp64 coalesced update
    W0 - lr * sum(g), with the block length forced to 16 and to 64 and left
    to the planner (64 at this size; the planner's choice is bitwise the forced 64).  The
    forced lengths go through ops.tuning (dlrm_set_tuning DLRM_TUNE_TBE_BLOCK)."""
    T, R, D, B, L, idx, off, W0, G, row_base = _c1_case(dist, 17 if dist == "uniform" else 18)
    lr = 0.25
    out = ops.tbe_forward(W0.to(dev), row_base.to(dev), T, B, idx.to(dev), off.to(dev)).cpu()
    for t in range(T):
        e = torch.nn.functional.embedding_bag(idx[t * B * L:(t + 1) * B * L].long(),
                                              W0[t * R:(t + 1) * R],
                                              torch.arange(B) * L, mode="sum")
        ok, msg = fp32_close(out[:, t].numpy(), e.numpy())
        assert ok, (t, msg)
    gsum = torch.zeros(T * R, D, dtype=torch.float64)
    bag = torch.arange(B * L) // L
    for t in range(T):
        gsum.index_add_(0, t * R + idx[t * B * L:(t + 1) * B * L].long(), G[bag, t].double())
    ref = (W0.double() - lr * gsum).numpy()
    res = {}
    for ch in ("16", "64", ""):
        W = W0.to(dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        with ops.tuning(tbe_block=int(ch or 0)):
            ops.tbe_backward("sgd", W, row_base.to(dev), T, B, idx.to(dev), off.to(dev),
                             G.to(dev), lr=lr, max_lookups_per_table=B * L, error_flag=flag)
        torch.cuda.synchronize()
        assert int(flag.item()) == 0
        res[ch] = W.cpu()
        ok, msg = fp32_close(res[ch].numpy(), ref)
        assert ok, (ch, msg)
    assert torch.equal(res["64"], res[""])


@pytest.mark.parametrize("D", [16, 32, 64, 128])
@pytest.mark.parametrize("F,self_int", [(2, False), (9, True), (27, False), (32, False)])
def test_interact_gather_matches_lookup_then_interact(ops, D, F, self_int):
    """The one-hot lookup fused into the dot interaction (dlrm_interact_dot_*_gather) vs
    tbe_forward (L = 1) followed by interact_forward / interact_backward on the pooled
    buffer: the same rows feed the same MFMA sequence, so results are bit-identical.  An
    out-of-range index reads as a zero row and raises the TBE index bit, as the lookup does."""
    torch.manual_seed(D * 100 + F)
    T, B = F - 1, 203  # B not a multiple of the 4 samples per block
    rows = [int(r) for r in torch.randint(1, 500, (T,))]
    row_base = torch.tensor([0] + list(np.cumsum(rows)), dtype=torch.int64, device=dev)
    W = torch.randn(int(row_base[-1]), D, device=dev)
    idx = torch.cat([torch.randint(0, n, (B,)) for n in rows]).to(torch.int32).to(dev)
    off = torch.arange(T * B + 1, dtype=torch.int32, device=dev)
    x = torch.randn(B, D + 4, device=dev)[:, :D]  # strided x, as the trainer passes it
    E = ops.tbe_forward(W, row_base, T, B, idx, off)
    R0 = ops.interact_forward("dot", x, E, self_int)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    R1 = ops.interact_forward_gather(x, W, row_base, idx, self_int, error_flag=err)
    torch.cuda.synchronize()
    assert torch.equal(R0, R1)
    assert int(err.item()) == 0
    gR = torch.randn_like(R0)
    gx0, gly0 = ops.interact_backward("dot", x, E, gR, self_int, relu_x=True)
    gx1, gly1 = ops.interact_backward_gather(x, W, row_base, idx, gR, self_int, relu_x=True)
    torch.cuda.synchronize()
    assert torch.equal(gx0, gx1)
    assert torch.equal(gly0, gly1)
    # an out-of-range index of the last table: a zero row, flagged
    bad = idx.clone()
    bad[(T - 1) * B + 5] = rows[-1]
    E2 = E.clone()
    E2[5, T - 1] = 0.0
    R2 = ops.interact_forward_gather(x, W, row_base, bad, self_int, error_flag=err)
    torch.cuda.synchronize()
    assert int(err.item()) & ops.TBE_ERR_INDEX
    assert torch.equal(R2, ops.interact_forward("dot", x, E2, self_int))
