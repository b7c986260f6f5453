"""Which RCCL collectives issued through torch.distributed capture into a hipGraph (and
replay correctly) on this stack?  One variant per process, 1-rank nccl group on cuda:0:

  python tools/rccl_capture_probe.py <variant> [thread_local]

Variants (each: eager warm-up where stated, capture, 3 replays, check the result):
  ar_sync        dist.all_reduce(t) (blocking form) on WORLD, warmed eagerly
  ar_async       all_reduce(async_op=True) + work.wait() under capture, warmed
  a2a_cold       all_to_all_single(async_op=True) + wait; WORLD warmed by an all_reduce only
                 (the all-to-all's own first use is inside the capture)
  a2a_async      all_to_all_single(async_op=True) + wait, warmed by one eager all-to-all
  a2a_splits     the same with explicit split lists (the trainer's uneven form)
  a2a_sync       all_to_all_single, blocking form, warmed
  allgather      all_gather_into_tensor, warmed
  p2p            batch_isend_irecv to self (the grouped send/recv an all-to-all is made of)
  g2_cold        a second group (dist.new_group), FIRST collective inside the capture
  g2_warm        the second group warmed by one eager all_reduce before the capture
  two_groups     a2a on WORLD || all_reduce on the second group, both async, both warmed by
                 one eager run of the body
  trainer        DLRMTrainer force_dist (C3 widths, B = 128): eager step, capture(whole=True)

faulthandler dumps every thread's stack if a variant does not finish in 60 s, so a hang
names the call it sits in.  Used for DESIGN.md §8 (the round-5 capture hang)."""
import faulthandler
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dlrm-yx_amd")]


def say(*a):
    print(f"[{time.time() - T0:7.2f}s]", *a, flush=True)


def graph_of(fn, mode):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, capture_error_mode=mode):
        fn()
    return g


def main():
    variant = sys.argv[1]
    mode = sys.argv[2] if len(sys.argv) > 2 else "global"
    faulthandler.dump_traceback_later(60, exit=True)
    bt = os.path.join(ROOT, "tools", "segv", "libsegv_bt.so")
    if os.path.exists(bt):  # native backtrace on SIGSEGV, then faulthandler's Python one
        import ctypes
        ctypes.CDLL(bt).segv_bt_install()
    faulthandler.enable()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1,
                            device_id=dev)
    say("init", variant, mode, "torch", torch.__version__)
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    y = torch.zeros_like(x)
    if variant.startswith("trainer"):
        return trainer(variant, mode, dev)
    g2 = dist.new_group(ranks=[0], backend="nccl") if variant.startswith(("g2", "two")) else None
    n = x.numel()
    if variant != "g2_cold":
        dist.all_reduce(x)  # warm WORLD's communicator
        if g2 is not None:
            dist.all_reduce(x, group=g2)
        torch.cuda.synchronize()
        say("warmed")

    def body():
        if variant == "ar_sync":
            dist.all_reduce(x)
        elif variant == "ar_async":
            dist.all_reduce(x, async_op=True).wait()
        elif variant in ("a2a_async", "a2a_cold"):
            dist.all_to_all_single(y, x, async_op=True).wait()
        elif variant == "a2a_sync":
            dist.all_to_all_single(y, x)
        elif variant == "allgather":
            dist.all_gather_into_tensor(y, x)
        elif variant == "p2p":
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0),
                                             dist.P2POp(dist.irecv, y, 0)]):
                w.wait()
        elif variant == "a2a_splits":
            dist.all_to_all_single(y, x, [n], [n], async_op=True).wait()
        elif variant in ("g2_cold", "g2_warm"):
            dist.all_reduce(x, group=g2, async_op=True).wait()
        elif variant == "two_groups":
            a = dist.all_to_all_single(y, x, async_op=True)
            b = dist.all_reduce(x, group=g2, async_op=True)
            a.wait()
            b.wait()
        else:
            raise SystemExit(f"unknown variant {variant}")
    if variant in ("a2a_async", "a2a_splits", "a2a_sync", "allgather", "p2p", "two_groups"):
        body()  # one eager run: the all-to-all's peer connections are set up here
        torch.cuda.synchronize()
        say("body warmed")
    say("capture begin")
    g = graph_of(body, mode)
    say("capture end")
    for i in range(3):
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        say("replay", i)
    ok = bool(torch.equal(x, torch.arange(1 << 20, dtype=torch.float32, device=dev)))
    if variant in ("a2a_async", "a2a_cold", "a2a_splits", "a2a_sync", "allgather", "p2p",
                   "two_groups"):
        ok = ok and bool(torch.equal(y, x))
    say("RESULT", variant, mode, "ok" if ok else "WRONG")
    dist.destroy_process_group()


def trainer(variant, mode, dev):
    from dlrm_hip.trainer import DLRMTrainer, TrainerConfig
    import oracle as O
    rows = [min(r, 2000) for r in O.TERABYTE_ROWS]
    cfg = TrainerConfig(m_spa=128, ln_emb=rows, ln_bot=[13, 512, 256, 128],
                        ln_top=[128 + 27 * 26 // 2, 1024, 1024, 512, 256, 1],
                        loss_function="bce", learning_rate=0.1)
    tr_ref = DLRMTrainer(cfg, device=dev, seed=3)
    tr = DLRMTrainer(cfg, device=dev, seed=3, force_dist=True, process_group=dist.group.WORLD)
    bs = [tr.synthetic_batch(128, 1, seed=i) for i in range(3)]
    tr.step(bs[0])
    tr_ref.step(bs[0])
    torch.cuda.synchronize()
    say("eager step done")
    run = tr.capture(bs[1], whole=True)
    say("captured", tr.capture_mode)
    run()
    torch.cuda.synchronize()
    say("replayed once")
    tr_ref.step(bs[1])
    torch.cuda.synchronize()
    d = (tr.params - tr_ref.params).abs().max().item()
    dt = (tr.weights - tr_ref.weights).abs().max().item()
    say("RESULT", variant, mode, f"max|dense diff| {d:.3g} max|table diff| {dt:.3g}")
    dist.destroy_process_group()


if __name__ == "__main__":
    T0 = time.time()
    main()
