"""Distributed plumbing with the reference's API (extend_distributed.py:1-666), on
torch.distributed — "nccl" is RCCL on ROCm, over xGMI between the MI355X of one node.

Kept API: module globals my_rank / my_size / my_local_rank / my_local_size,
init_distributed(), get_my_slice(), get_split_lengths(), alltoall() -> Request with
.wait(), all_gather(), barrier(), print_all().  The pooled-embedding exchange is one
all_to_all_single per direction with the reference's splits (batch-major send chunks,
rank-major receive chunks, extend_distributed.py:405-508); the scatter/gather fallbacks
of DLRM_ALLTOALL_IMPL are not on the MI355X path (RCCL implements all_to_all natively).
"""
from __future__ import annotations

import builtins
import os
import sys

import torch
import torch.distributed as dist
from torch.autograd import Function
from torch.autograd.profiler import record_function
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: F401 (re-exported)

my_rank = -1
my_size = -1
my_local_rank = -1
my_local_size = -1
alltoall_supported = False
myreq = None


def env2int(env_list, default=-1):
    for e in env_list:
        val = int(os.environ.get(e, -1))
        if val >= 0:
            return val
    return default


def get_my_slice(n):
    """This rank's contiguous batch slice; the first n % size ranks get one extra."""
    k, m = divmod(n, my_size)
    return slice(my_rank * k + min(my_rank, m), (my_rank + 1) * k + min(my_rank + 1, m), 1)


def get_split_lengths(n):
    """(my_len, splits) with splits None when n divides evenly."""
    k, m = divmod(n, my_size)
    if m == 0:
        return k, None
    splits = [(k + 1) if i < m else k for i in range(my_size)]
    return splits[my_rank], splits


def init_distributed(rank=-1, local_rank=-1, size=-1, use_gpu=False, backend=""):
    """Backend resolution as the reference (extend_distributed.py:81-207): with a GPU the
    backend is "nccl" (= RCCL); otherwise gloo.  Rank/size come from the launcher env."""
    global my_rank, my_size, my_local_rank, my_local_size, alltoall_supported, myreq
    n = env2int(["PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "MV2_COMM_WORLD_SIZE", "WORLD_SIZE"])
    if backend == "" and n > 1:
        backend = "nccl" if (use_gpu and dist.is_nccl_available()) else "gloo"
    if backend != "":
        if rank == -1:
            rank = env2int(["PMI_RANK", "OMPI_COMM_WORLD_RANK", "MV2_COMM_WORLD_RANK", "RANK"], 0)
        if size == -1:
            size = env2int(["PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "MV2_COMM_WORLD_SIZE",
                            "WORLD_SIZE"], 1)
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(size))
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if size > 1:
        my_local_rank = local_rank if local_rank != -1 else env2int(
            ["MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "MV2_COMM_WORLD_LOCAL_RANK",
             "LOCAL_RANK"], 0)
        my_local_size = env2int(["MPI_LOCALNRANKS", "OMPI_COMM_WORLD_LOCAL_SIZE",
                                 "MV2_COMM_WORLD_LOCAL_SIZE", "LOCAL_WORLD_SIZE"], 1)
        if use_gpu:
            if my_local_size > torch.cuda.device_count():
                print("Not sufficient GPUs available... local_size = %d, ngpus = %d"
                      % (my_local_size, torch.cuda.device_count()))
                sys.exit(1)
            torch.cuda.set_device(my_local_rank)
        if not dist.is_initialized():
            dist.init_process_group(backend, rank=rank, world_size=size)
        my_rank = dist.get_rank()
        my_size = dist.get_world_size()
        if my_rank == 0:
            print("Running on %d ranks using %s backend" % (my_size, backend))
        alltoall_supported = hasattr(dist, "all_to_all_single")
    else:
        my_rank, my_size, my_local_rank, my_local_size = 0, 1, 0, 1
    print_all("world size: %d, current rank: %d, local rank: %d"
              % (my_size, my_rank, my_local_rank))
    myreq = Request()


class All2AllInfo(object):
    pass


class _Done(object):
    """A completed request (the host-staged gloo exchange below is synchronous)."""

    def wait(self):
        return None


def _all_to_all_single(out, inp, out_splits, in_splits):
    """all_to_all_single, async.  Device tensors under gloo (several ranks sharing one GPU
    in the tests, or a CPU rendezvous) go through host memory synchronously; under nccl
    (RCCL over xGMI, the MI355X path) the exchange stays on the device and async."""
    if out.is_cuda and dist.get_backend() == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
        out.copy_(o)
        return _Done()
    return dist.all_to_all_single(out, inp, out_splits, in_splits, async_op=True)


class Request(object):
    def __init__(self):
        self.req = None
        self.tensor = None
        self.a2a_info = None
        self.WaitFunction = All2All_Wait

    def wait(self):
        ret = self.WaitFunction.apply(*self.tensor)
        self.req = None
        self.tensor = None
        return ret


class All2All_Req(Function):
    """[B, T_local*D] (or [B, T_local, D]) local lookups -> async all_to_all_single whose
    receive buffer holds, per source rank, its [B/W, T_src*D] chunk (rank-major)."""

    @staticmethod
    def forward(ctx, a2a_info, *inputs):
        global myreq
        with record_function("DLRM alltoall_req_fwd_single"):
            bsl = a2a_info.global_batch_partition_slices
            if bsl:
                bsl = [m * a2a_info.emb_dim * a2a_info.local_table_num for m in bsl]
            tsl = a2a_info.global_table_wise_partition_slices
            if tsl:
                tsl = [a2a_info.local_batch_num * e * a2a_info.emb_dim for e in tsl]
            inp = torch.cat([x.reshape(x.shape[0], -1) for x in inputs], dim=1).view(-1)
            out = inp.new_empty([a2a_info.global_table_num * a2a_info.local_batch_num *
                                 a2a_info.emb_dim])
            req = _all_to_all_single(out, inp, tsl, bsl)
            a2a_info.batch_split_lengths = bsl
            a2a_info.table_split_lengths = tsl
            myreq.req = req
            myreq.tensor = (out,)
            myreq.a2a_info = a2a_info
            ctx.a2a_info = a2a_info
            return myreq.tensor

    @staticmethod
    def backward(ctx, *grad_output):
        global myreq
        with record_function("DLRM alltoall_req_bwd_single"):
            a2a_info = ctx.a2a_info
            myreq.req.wait()
            myreq.req = None
            grad_input = myreq.tensor
            if a2a_info.batched_emb:
                gi = [grad_input.view([a2a_info.batch_size, -1, a2a_info.emb_dim])]
            else:
                gi = grad_input.view([a2a_info.batch_size, -1]).split(a2a_info.emb_dim, dim=1)
            myreq.tensor = None
            return (None, *[g.contiguous() for g in gi])


class All2All_Wait(Function):
    @staticmethod
    def forward(ctx, *output):
        global myreq
        with record_function("DLRM alltoall_wait_fwd_single"):
            a2a_info = myreq.a2a_info
            ctx.a2a_info = a2a_info
            myreq.req.wait()
            myreq.req = None
            myreq.tensor = None
            tsl = a2a_info.table_split_lengths or (a2a_info.local_table_num *
                                                   a2a_info.local_batch_num * a2a_info.emb_dim)
            outs = output[0].split(tsl)
            if a2a_info.batched_emb:
                return tuple(o.view([a2a_info.local_batch_num, -1, a2a_info.emb_dim])
                             for o in outs)
            return tuple(o.view([a2a_info.local_batch_num, -1]) for o in outs)

    @staticmethod
    def backward(ctx, *grad_outputs):
        global myreq
        with record_function("DLRM alltoall_wait_bwd_single"):
            a2a_info = ctx.a2a_info
            go = torch.cat([g.contiguous().view(-1) for g in grad_outputs])
            gi = go.new_empty([a2a_info.batch_size * a2a_info.local_table_num *
                               a2a_info.emb_dim])
            req = _all_to_all_single(gi, go, a2a_info.batch_split_lengths,
                                     a2a_info.table_split_lengths)
            myreq.req = req
            myreq.tensor = gi
            return (go,)


def alltoall(inputs, per_rank_table_splits, batched_emb=False):
    """extend_distributed.py:601-639 (the all_to_all_single implementation)."""
    global myreq
    if myreq is None:
        myreq = Request()
    info = All2AllInfo()
    if batched_emb:
        info.batch_size, info.local_table_num, info.emb_dim = inputs[0].size()
    else:
        info.batch_size, info.emb_dim = inputs[0].size()
        info.local_table_num = len(inputs)
    info.global_table_wise_partition_slices = per_rank_table_splits
    info.local_batch_num, info.global_batch_partition_slices = get_split_lengths(info.batch_size)
    info.global_table_num = (sum(per_rank_table_splits) if per_rank_table_splits
                             else info.local_table_num * my_size)
    info.batched_emb = batched_emb
    All2All_Req.apply(info, *inputs)
    myreq.WaitFunction = All2All_Wait
    return myreq


class AllGather(Function):
    @staticmethod
    def forward(ctx, input, global_lengths, dim=0):
        if not isinstance(global_lengths, (list, tuple)):
            global_lengths = [global_lengths] * my_size
        ctx.dim = dim
        ctx.local_start = sum(global_lengths[:my_rank])
        ctx.local_length = global_lengths[my_rank]
        input = input.contiguous()
        staged = input.is_cuda and dist.get_backend() == "gloo"
        src = input.cpu() if staged else input
        parts = []
        for length in global_lengths:
            shp = list(input.size())
            shp[dim] = length
            parts.append(src.new_empty(shp))
        dist.all_gather(parts, src)
        out = torch.cat(parts, dim=dim)
        return out.to(input.device) if staged else out

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output.narrow(ctx.dim, ctx.local_start, ctx.local_length), None, None


def all_gather(input, lengths, dim=0):
    if not lengths:
        lengths = [input.size(0)] * my_size
    return AllGather.apply(input, lengths, dim)


def barrier():
    if my_size > 1:
        dist.barrier()


orig_print = builtins.print


def rank0_print(*args, **kwargs):
    if my_rank <= 0 or kwargs.pop("print_all", False):
        orig_print(*args, **kwargs)


def print_all(*args, **kwargs):
    orig_print(*args, **kwargs)
