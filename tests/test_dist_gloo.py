"""World-size-2 gloo tests (CPU) of the distributed exchange of the drop-in path:
extend_distributed.alltoall forward (rank-major receive layout) and backward (gradients
routed back to the owning rank), non-batched and batched; the batched input split
(distribute_batched_emb_data) against the oracle restatement."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, W, port):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "dlrm-yx_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(W), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(W))
    from dlrm_hip import extend_distributed as ed
    ed.init_distributed(rank=rank, local_rank=rank, size=W, use_gpu=False, backend="gloo")
    return ed


def _global_features(B, D, T):
    g = torch.Generator().manual_seed(5)
    return [torch.randn(B, D, generator=g) for _ in range(T)]


def _a2a_worker(rank, W, port, batched, B, D, device_indices, q):
    try:
        ed = _setup(rank, W, port)
        T = len(device_indices)
        feats = _global_features(B, D, T)
        local = [t for t in range(T) if device_indices[t] == rank]
        n_per_rank = [sum(1 for t in range(T) if device_indices[t] == r) for r in range(W)]
        if batched:
            inp = [torch.stack([feats[t] for t in local], dim=1).requires_grad_()]
        else:
            inp = [feats[t].clone().requires_grad_() for t in local]
        outs = list(ed.alltoall(inp, n_per_rank, batched).wait())
        sl = ed.get_my_slice(B)
        order = [t for r in range(W) for t in range(T) if device_indices[t] == r]
        got = torch.cat([o.reshape(o.shape[0], -1) for o in outs], dim=1)
        want = torch.cat([feats[t][sl] for t in order], dim=1)
        assert torch.equal(got, want), "rank-major receive layout"
        # loss = sum(out * c) with c depending on (global row, global table): the input
        # gradient of table t at row b must be c[b, t] regardless of who computed it
        rows = torch.arange(B, dtype=torch.float32)[sl].view(-1, 1)
        coef = torch.cat([(rows + 100 * t).expand(-1, D) for t in order], dim=1)
        (got * coef).sum().backward()
        ed.myreq.req.wait() if ed.myreq.req is not None else None
        for j, t in enumerate(local):
            g = inp[0].grad[:, j] if batched else inp[j].grad
            exp = (torch.arange(B, dtype=torch.float32) + 100 * t).view(-1, 1).expand(-1, D)
            assert torch.equal(g, exp), f"grad of table {t}"
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


def _run(fn, W, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=fn, args=(r, W, port, *args, q)) for r in range(W)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(W))
    for p in ps:
        p.join(timeout=60)
    for r in range(W):
        assert res[r] == "ok", res[r]


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("B", [8, 7])
def test_alltoall_roundtrip_world2(batched, B):
    # uneven table split: rank 0 owns 3 tables, rank 1 owns 2; B=7 -> uneven batch split
    _run(_a2a_worker, 2, batched, B, 4, [0, 1, 0, 1, 0])


def _split_worker(rank, W, port, q):
    try:
        _setup(rank, W, port)
        from oracle import dlrm_oracle as O
        from dlrm_hip.dlrm_net import DLRM_Net
        import numpy as np
        B, T, L = 6, 4, 3
        g = torch.Generator().manual_seed(3)
        offsets = torch.arange(0, T * B * L + 1, L, dtype=torch.int32)
        indices = torch.randint(0, 50, (T * B * L,), generator=g, dtype=torch.int32)
        net = DLRM_Net.__new__(DLRM_Net)
        torch.nn.Module.__init__(net)
        net.ln_emb = np.array([50] * T)
        net.local_emb_indices = [t for t in range(T) if t % W == rank]
        o, i = net.distribute_batched_emb_data(B, offsets, indices)
        eo, ei = O.distribute_batched(offsets, indices, B, T, net.local_emb_indices)
        assert torch.equal(o[0], eo) and torch.equal(i[0], ei)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_distribute_batched_emb_data_world2():
    _run(_split_worker, 2)
