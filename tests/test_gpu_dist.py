"""Two ranks of the fused trainer sharing one GPU (gloo, host-staged exchange) against the
oracle's W-rank restatement of distributed_forward + DDP (oracle.distributed_step):
rank-major features after the all-to-all, W x embedding gradients, averaged dense grads.
The N>1 bench runs the same code over RCCL (nccl) with one GPU per rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CFG = dict(m_spa=8, ln_emb=[300, 40, 1000, 7, 120], ln_bot=[13, 32, 8], ln_top=[23, 16, 1])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ref_model():
    import oracle as O
    np.random.seed(77)
    return O.OracleDLRM(CFG["m_spa"], CFG["ln_emb"], CFG["ln_bot"], CFG["ln_top"],
                        loss_function="bce")


def _batches(n, B):
    import oracle as O
    rng = np.random.RandomState(8)
    np.random.seed(99)
    out = []
    for _ in range(n):
        X, lS_o, lS_i = O.generate_uniform_input_batch(13, CFG["ln_emb"], B, 5, False)
        T = torch.tensor(rng.randint(0, 2, size=(B, 1)).astype(np.float32))
        out.append((torch.log(X + 1), torch.stack(lS_o), lS_i, T))
    return out


def _worker(rank, W, port, sharder, q, graph=False):
    try:
        sys.path[:0] = [ROOT, os.path.join(ROOT, "dlrm-yx_amd")]
        import torch.distributed as dist
        from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=W)
        cfg = TrainerConfig(**CFG, loss_function="bce", learning_rate=0.05, sharder=sharder)
        ref = _ref_model()
        tr = DLRMTrainer.from_oracle(cfg, ref, device="cuda:0", rank=rank, world_size=W,
                                     process_group=dist.group.WORLD)
        res = {"Z": [], "E": [], "local": tr.local_tables}
        batches = [tr.make_batch(X, lS_o, lS_i, T) for X, lS_o, lS_i, T in _batches(3, 12)]
        runs = [lambda b=b: tr.step(b) for b in batches]
        if graph:  # step 0 eager (allocations), steps 1-2 replayed from captured segments
            tr.step(batches[0])
            torch.cuda.synchronize()
            runs = [None] + [tr.capture(b) for b in batches[1:]]
        for i, b in enumerate(batches):
            if runs[i] is not None:
                runs[i]()
            bufs = tr._bufs[(b.X.shape[0], b.X.shape[0] * W)]
            Z, E = bufs["prob"], bufs["loss"]
            res["Z"].append(Z.cpu().numpy())
            res["E"].append(float(E.cpu()))
        torch.cuda.synchronize()
        res["tables"] = {t: tr.table(t).cpu().numpy() for t in tr.local_tables}
        res["dense"] = [(w.cpu().numpy(), b.cpu().numpy()) for w, b in tr.dense_state()]
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("sharder,graph", [("naive", False), ("greedy", False),
                                           ("greedy", True)])
def test_two_ranks_match_oracle_distributed_step(sharder, graph):
    """graph=True: steps replayed from trainer.capture (kernel segments as hipGraphs, the
    exchanges eager between them), the bench's multi-GPU path."""
    import oracle as O
    from conftest import fp32_close
    from dlrm_hip.sharders import shard
    W = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, W, port, sharder, q, graph)) for r in range(W)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(W))
    for p in ps:
        p.join(timeout=60)
    for r in range(W):
        assert isinstance(res[r], dict), res[r]
    ref = _ref_model()
    di = shard(CFG["ln_emb"], W, sharder)
    for s, (X, lS_o, lS_i, T) in enumerate(_batches(3, 12)):
        Zs, Es = O.distributed_step(ref, W, di, X, lS_o, lS_i, T, 0.05)
        for r in range(W):
            ok, msg = fp32_close(res[r]["Z"][s], Zs[r].numpy().ravel())
            assert ok, (s, r, msg)
            ok, msg = fp32_close(np.array([res[r]["E"][s]]), Es[r].numpy().reshape(1))
            assert ok, (s, r, msg)
    for r in range(W):
        for t, w in res[r]["tables"].items():
            assert di[t] == r
            ok, msg = fp32_close(w, ref.emb_l[t].weight.detach().numpy())
            assert ok, (r, t, msg)
        lin = [m for seq in (ref.bot_l, ref.top_l) for m in seq
               if isinstance(m, torch.nn.Linear)]
        for i, (w, b) in enumerate(res[r]["dense"]):
            ok, msg = fp32_close(w, lin[i].weight.detach().numpy())
            assert ok, (r, "W", i, msg)
            ok, msg = fp32_close(b, lin[i].bias.detach().numpy())
            assert ok, (r, "b", i, msg)
