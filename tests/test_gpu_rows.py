"""Reduced-precision rows on the GPU: dlrm_tbe_forward_rows (F16 / 8-bit / 4-bit row-wise)
vs the reference's quantized ops' golden outputs, table-batched; the quantized inference
path of DLRM_Net (quantize_embedding -> apply_emb)."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import fp32_close

pytestmark = pytest.mark.gpu
dev = "cuda:0"
CASES = [(8, 16), (8, 64), (8, 128), (4, 16), (4, 64), (4, 128)]


@pytest.fixture(scope="module")
def ops():
    from dlrm_hip import ops as _ops
    return _ops


def _batched(g, key, T, idx_dtype):
    lo = [torch.from_numpy(g[f"{key}_off{t}"]) for t in range(T)]
    li = [torch.from_numpy(g[f"{key}_idx{t}"]) for t in range(T)]
    off, idx = O.batched_csr(lo, li)
    return off.to(dev), idx.to(idx_dtype).to(dev)


@pytest.mark.parametrize("bits,D", CASES)
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("weighted", [False, True])
def test_quantized_forward_matches_reference_ops(ops, golden, bits, D, idx_dtype, weighted):
    g = golden("rows.npz")
    key = f"b{bits}_D{D}"
    rows = [int(r) for r in g["rows"]]
    T, B = len(rows), int(g["B"][0])
    packed = torch.from_numpy(np.concatenate([g[f"{key}_q{t}"] for t in range(T)])).to(dev)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    off, idx = _batched(g, key, T, idx_dtype)
    psw = None
    if weighted:
        psw = torch.from_numpy(np.concatenate([g[f"{key}_psw{t}"] for t in range(T)])).to(dev)
    fmt = ops.ROWS_Q4 if bits == 4 else ops.ROWS_Q8
    out = ops.tbe_forward_rows(packed, fmt, D, row_base, T, B, idx, off,
                               per_sample_weights=psw).cpu()
    for t in range(T):
        ok, msg = fp32_close(out[:, t].numpy(), g[f"{key}_{'yw' if weighted else 'y'}{t}"])
        assert ok, (t, msg)


@pytest.mark.parametrize("D", [16, 64, 128, 512])
def test_f16_forward_matches_fp32_of_half_weights(ops, D):
    torch.manual_seed(2)
    rows, B = [50, 3, 700], 40
    T = len(rows)
    W = torch.randn(sum(rows), D).half()
    lo, li = [], []
    for n in rows:
        lens = torch.randint(0, 7, (B,))
        lo.append(torch.cat([torch.zeros(1, dtype=torch.int64), lens.cumsum(0)[:-1]]))
        li.append(torch.randint(0, n, (int(lens.sum()),)))
    off, idx = O.batched_csr(lo, li)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64)
    psw = torch.rand(idx.numel())
    out = ops.tbe_forward_rows(W.to(dev), ops.ROWS_F16, D, row_base.to(dev), T, B, idx.to(dev),
                               off.to(dev), per_sample_weights=psw.to(dev)).cpu()
    Wf = W.float().split(rows, 0)
    pw = psw.split([x.numel() for x in li])
    for t in range(T):
        ref = torch.nn.functional.embedding_bag(li[t], Wf[t], lo[t], mode="sum",
                                                per_sample_weights=pw[t])
        ok, msg = fp32_close(out[:, t].numpy(), ref.numpy())
        assert ok, msg


def test_rows_out_of_range_index_is_flagged(ops):
    w = torch.randn(10, 16)
    q = torch.ops.quantized.embedding_bag_byte_prepack(w).to(dev)
    row_base = torch.tensor([0, 10], dtype=torch.int64, device=dev)
    off = torch.tensor([0, 2, 3], dtype=torch.int32, device=dev)
    idx = torch.tensor([1, 12, 3], dtype=torch.int32, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = ops.tbe_forward_rows(q, ops.ROWS_Q8, 16, row_base, 1, 2, idx, off, error_flag=flag)
    assert flag.item() == ops.TBE_ERR_INDEX
    ref = torch.ops.quantized.embedding_bag_byte_rowwise_offsets(
        q.cpu(), torch.tensor([1, 3]), torch.tensor([0, 1]))
    ok, msg = fp32_close(out[:, 0].cpu().numpy(), ref.numpy())
    assert ok, msg


@pytest.mark.parametrize("bits", [4, 8])
def test_dlrm_net_quantize_embedding(ops, bits):
    """DLRM_Net.quantize_embedding + apply_emb (one launch for all tables) vs the
    reference's per-table quantized ops on the same packed rows."""
    from dlrm_hip.dlrm_net import DLRM_Net
    np.random.seed(3)
    ln_emb = np.array([40, 7, 300])
    net = DLRM_Net(m_spa=16, ln_emb=ln_emb, ln_bot=np.array([5, 16]),
                   ln_top=np.array([22, 8, 1]), arch_interaction_op="dot").to(dev)
    net.quantize_embedding(bits)
    assert net.quantize_emb and net.emb_l is None
    B = 12
    lS_o, lS_i = [], []
    for n in ln_emb:
        lens = np.random.randint(1, 4, B)
        lS_o.append(torch.tensor(np.concatenate([[0], np.cumsum(lens)[:-1]])))
        lS_i.append(torch.tensor(np.random.randint(0, n, int(lens.sum()))))
    ly = net.apply_emb(lS_o, lS_i)
    look = (torch.ops.quantized.embedding_bag_4bit_rowwise_offsets if bits == 4
            else torch.ops.quantized.embedding_bag_byte_rowwise_offsets)
    for k in range(len(ln_emb)):
        ref = look(net.emb_l_q[k], lS_i[k], lS_o[k])
        ok, msg = fp32_close(ly[k].cpu().numpy(), ref.numpy())
        assert ok, (k, msg)
    x = torch.rand(B, 5)
    p = net(x.to(dev), lS_o, lS_i)
    assert p.shape == (B, 1) and torch.isfinite(p).all()


@pytest.mark.parametrize("mx_kind", ["cap", "none"])
def test_tbe_backward_sgd_f16(ops, mx_kind):
    """Exact SGD on fp16 rows: per-row gradient summed in fp32 (sorted, deterministic),
    w = float(w16) - lr * g rounded to nearest fp16.  Reference: the same update in fp64
    from the same half weights, rounded to fp16 -> equal within one fp16 ulp; skewed tables
    exercise runs crossing blocks; bitwise reproducible run to run."""
    torch.manual_seed(9)
    rows, D, B, L = [3, 5000, 4, 700], 128, 512, 2
    T = len(rows)
    lo = [torch.arange(B) * L for _ in rows]
    li = [torch.randint(0, n, (B * L,)) for n in rows]
    off, idx = O.batched_csr(lo, li)
    row_base = torch.tensor([0] + np.cumsum(rows).tolist(), dtype=torch.int64, device=dev)
    G = torch.randn(B, T, D, device=dev)
    W0 = (torch.randn(sum(rows), D) * 0.5).half().to(dev)
    mx = B * L if mx_kind == "cap" else 0
    outs = []
    for _ in range(2):
        W = W0.clone()
        ops.tbe_backward("sgd", W, row_base, T, B, idx.to(dev), off.to(dev), G, lr=0.05,
                         max_lookups_per_table=mx)
        outs.append(W.cpu())
    assert torch.equal(outs[0], outs[1])
    gsum = torch.zeros(sum(rows), D, dtype=torch.float64)
    gt = G.cpu().double()
    bag = torch.arange(B * L) // L
    for t in range(T):
        gsum.index_add_(0, int(row_base[t]) + li[t], gt[bag, t])
    ref = (W0.cpu().double() - 0.05 * gsum).half()
    got = outs[0]
    ulp = torch.clamp(ref.float().abs(), min=2.0 ** -14) * 2.0 ** -10
    assert torch.all((got.float() - ref.float()).abs() <= ulp * 1.01)
    assert (got != W0.cpu()).any()


def test_dlrm_net_fbgemm_fp16_path(ops):
    """DLRM_Net(fbgemm_emb=True): the fp16 TBE module's lookup equals fp32 math on its half
    weights, and a backward step applies exact SGD (lr 0.01) to the fp16 rows."""
    from dlrm_hip.dlrm_net import DLRM_Net
    np.random.seed(4)
    torch.manual_seed(4)
    ln_emb = np.array([60, 9, 400])
    T, D, B = len(ln_emb), 16, 10
    net = DLRM_Net(m_spa=D, ln_emb=ln_emb, ln_bot=np.array([5, D]),
                   ln_top=np.array([D + T * (T + 1) // 2, 8, 1]), arch_interaction_op="dot",
                   fbgemm_emb=True).to(dev)
    emb = net.emb_l
    assert emb.weights.dtype == torch.float16
    lS_o = torch.arange(0, T * B * 2 + 1, 2, dtype=torch.int32)
    lS_i = torch.cat([torch.randint(0, int(n), (B * 2,)) for n in ln_emb]).int()
    W0 = emb.weights.detach().clone()
    y = net.apply_emb_fbgemm([lS_o.to(dev)], [lS_i.to(dev)])[0]
    Wf = W0.float().cpu()
    rb = [0] + np.cumsum(ln_emb).tolist()
    for t in range(T):
        idx = lS_i[t * B * 2:(t + 1) * B * 2].long() + rb[t]
        ref = Wf[idx].view(B, 2, D).sum(1)
        ok, msg = fp32_close(y[:, t].detach().cpu().numpy(), ref.numpy())
        assert ok, msg
    g = torch.randn_like(y)
    (y * g).sum().backward()
    torch.cuda.synchronize()
    W1 = emb.weights.detach().cpu()
    gsum = torch.zeros(Wf.shape, dtype=torch.float64)
    for t in range(T):
        idx = lS_i[t * B * 2:(t + 1) * B * 2].long() + rb[t]
        gsum.index_add_(0, idx, g[:, t].cpu().double().repeat_interleave(2, 0))
    ref = (Wf.double() - 0.01 * gsum).half()
    ulp = torch.clamp(ref.float().abs(), min=2.0 ** -14) * 2.0 ** -10
    assert torch.all((W1.float() - ref.float()).abs() <= ulp * 1.01)
